// fqz_codec.cpp — fqz_compress / fqz_decompress on the GPU
// (htscodecs fqzcomp_qual.c:1008-1646, fork ABI).
//
// Encode: the block's bytes go to HBM once; the statistics of
// fqz_qual_stats are gathered by kernels (fqz_kernels.hip); the host makes
// the reference's decisions from them (entropy comparisons in double, the
// same expressions in the same order), serialises the parameters and the
// serial model + range-coder kernel writes the stream.  Decode parses the
// parameters on the host and runs the serial decode kernel.
#include <algorithm>
#include <atomic>
#include <chrono>
#include <climits>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <stdexcept>
#include <map>
#include <mutex>
#include <vector>

#include "../../include/fqz5_mi355x.h"
#include "fqz_format.hpp"
#include "fqz_kernels.h"
#include "gpu_ctx.hpp"
#include "rans_format.hpp"
#include "fqz_codec.hpp"

namespace fqz5 {
using namespace fqz;

namespace {

struct Records {
    std::vector<uint32_t> len, flags;
    std::vector<uint64_t> off;
    uint32_t walked = 0;      // records the statistics loop visits
};

// Records as fqz_qual_stats walks them (fqzcomp_qual.c:464-501): every
// record starting before the end of the data; with no records the whole
// buffer is one.
Records walk_records(int nrec, const uint32_t *lens, const uint32_t *flags, size_t n) {
    Records R;
    if (nrec <= 0) {
        R.len.assign(1, uint32_t(n));
        R.flags.assign(1, 0);
        R.off.assign(1, 0);
        R.walked = n ? 1 : 0;
        return R;
    }
    R.len.assign(lens, lens + nrec);
    R.flags.assign(flags, flags + nrec);
    R.off.resize(size_t(nrec));
    uint64_t o = 0;
    for (int r = 0; r < nrec; r++) {
        R.off[size_t(r)] = o;
        if (o < n) R.walked = uint32_t(r + 1);
        o += R.len[size_t(r)];
    }
    return R;
}

// The statistics and auto-tuning of fqz_qual_stats (fqzcomp_qual.c:424-704)
// with the histograms from the GPU.  Updates pm and the caller's flags.
// Staged so that the requests of a batch share their round trips: launch()
// for each, one sync, mid() for each (it launches the per-class histograms
// when the average-quality split is searched), one sync, finish() for each.
struct Tune {
    Param *pm = nullptr;
    int nrec = 0;
    uint32_t *flags = nullptr;
    const Records *R = nullptr;
    uint32_t *qhist = nullptr;
    int max_sel = 0, has_r2 = 0;
    FqzStatJob J{};
    std::vector<uint2> chunks;
    std::vector<uint32_t> h1, h2, ahist, ravg, amap, b4;
    uint32_t dups = 0;
    bool classes = false;

    void launch(GpuCtx &g, Param &p, int nr, uint32_t *fl, const Records &rec,
                const uint8_t *d_q, uint32_t *qh) {
        pm = &p, nrec = nr, flags = fl, R = &rec, qhist = qh;
        for (int r = 0; r < nrec; r++) {
            max_sel = std::max(max_sel, int(flags[r] >> 16));
            if (flags[r] & F_READ2) has_r2 = 1;
        }
        const uint32_t W = R->walked;
        // ---- GPU: per-record averages / dups, (len & 127, q) histograms ----
        for (uint32_t r = 0; r < W;) {
            uint32_t e = r, bytes = 0;
            while (e < W && (e == r || bytes + R->len[e] <= 65535u)) bytes += R->len[e++];
            chunks.push_back(make_uint2(r, e));
            r = e;
        }
        J.q = d_q;
        J.off = g.upload(R->off);
        J.len = g.upload(R->len);
        J.flags = g.upload(R->flags);
        J.nrec = W;
        J.rec_avg = g.arena.alloc_n<uint32_t>(W + 1);
        J.avg_hist = g.arena.alloc_n<uint32_t>(NAVG);
        J.dups = g.arena.alloc_n<uint32_t>(1);
        J.chunks = g.upload(chunks);
        J.h1 = g.arena.alloc_n<uint32_t>(NPOS * 256);
        J.h2 = g.arena.alloc_n<uint32_t>(NPOS * 256);
        J.b4 = g.arena.alloc_n<uint32_t>(4 * NPOS * 256);
        g.memset0(J.rec_avg, (W + 1) * 4);
        g.memset0(J.avg_hist, NAVG * 4);
        g.memset0(J.dups, 4);
        g.memset0(J.h1, NPOS * 256 * 4);
        g.memset0(J.h2, NPOS * 256 * 4);
        g.memset0(J.b4, 4 * NPOS * 256 * 4);
        FQZ5_HIP(launch_fqz_records(J, g.stream));
        FQZ5_HIP(launch_fqz_hist(J, int(chunks.size()), 0, g.stream));
        h1.resize(NPOS * 256), h2.resize(NPOS * 256), ahist.resize(NAVG), ravg.resize(W + 1);
        g.download(h1.data(), J.h1, h1.size());
        g.download(h2.data(), J.h2, h2.size());
        g.download(ahist.data(), J.avg_hist, ahist.size());
        g.download(ravg.data(), J.rec_avg, ravg.size());
        g.download(&dups, J.dups, 1);
    }

    void mid(GpuCtx &g) {
        const uint32_t W = R->walked;
        for (int j = 0; j < NPOS; j++)
            for (int s = 0; s < 256; s++) qhist[s] += h1[size_t(j) * 256 + s] + h2[size_t(j) * 256 + s];
        pm->dedup = ((W + 1) / (dups + 1) < 500);
        pm->max_sym = pm->nsym = 0;
        for (int s = 0; s < 256; s++)
            if (qhist[s]) pm->max_sym = s, pm->nsym++;
        if (pm->qa == 0) return;
        // rank the averages into four classes (fqzcomp_qual.c:522-557)
        const double f0 = pm->nsym > 8 ? 0.2 : 0.05;
        const double f1 = pm->nsym > 8 ? 0.5 : 0.22;
        const double f2 = pm->nsym > 8 ? 0.8 : 0.60;
        amap = ahist;
        const double cut[3] = {f0, f1, f2};
        int total = 0, k = 0;
        for (int cls = 0; cls < 3; cls++) {
            while (k < NAVG) {
                total += int(amap[size_t(k)]);
                if (total > cut[cls] * nrec) break;
                amap[size_t(k++)] = uint32_t(cls);
            }
        }
        while (k < NAVG) amap[size_t(k++)] = 3;
        // ---- GPU: histograms per class ----
        J.amap = g.upload(amap);
        FQZ5_HIP(launch_fqz_hist(J, int(chunks.size()), 1, g.stream));
        FQZ5_HIP(launch_fqz_hist(J, int(chunks.size()), 2, g.stream));
        b4.resize(4 * NPOS * 256);
        g.download(b4.data(), J.b4, b4.size());
        classes = true;
    }

    void finish() {
        Param &p = *pm;
        const uint32_t W = R->walked;
        // per-record average of every record (unwalked ones: 0, as calloc)
        auto rec_avg = [&](int r) -> uint32_t {
            if (nrec <= 0) return ravg[0];
            return uint32_t(r) < W ? ravg[size_t(r)] : 0u;
        };
        if (classes) {
            auto B4 = [&](int c, int j, int s) { return double(b4[(size_t(c) * NPOS + j) * 256 + s]); };
            // counts per (class, position) and the merged 2-class / 1-class bins
            std::vector<double> n4(4 * NPOS, 0);
            for (int c = 0; c < 4; c++)
                for (int j = 0; j < NPOS; j++)
                    for (int s = 0; s < 256; s++) n4[size_t(c) * NPOS + j] += B4(c, j, s);
            double e1 = 0, e2 = 0, e4 = 0;
            for (int j = 0; j < NPOS; j++) {
                const double c20 = n4[size_t(0) * NPOS + j] + n4[size_t(1) * NPOS + j];
                const double c21 = n4[size_t(2) * NPOS + j] + n4[size_t(3) * NPOS + j];
                const double c1 = c20 + c21;
                for (int s = 0; s < 256; s++) {
                    const double a0 = B4(0, j, s), a1 = B4(1, j, s), a2 = B4(2, j, s), a3 = B4(3, j, s);
                    const double q20 = a0 + a1, q21 = a2 + a3, q1 = q20 + q21;
                    if (q1) e1 += q1 * std::log(q1 / c1);
                    if (q20) e2 += q20 * std::log(q20 / c20);
                    if (q21) e2 += q21 * std::log(q21 / c21);
                    if (a0) e4 += a0 * std::log(a0 / n4[size_t(0) * NPOS + j]);
                    if (a1) e4 += a1 * std::log(a1 / n4[size_t(1) * NPOS + j]);
                    if (a2) e4 += a2 * std::log(a2 / n4[size_t(2) * NPOS + j]);
                    if (a3) e4 += a3 * std::log(a3 / n4[size_t(3) * NPOS + j]);
                }
            }
            e1 /= -std::log(2) / 8;
            e2 /= -std::log(2) / 8;
            e4 /= -std::log(2) / 8;
            const double m = p.qa > 0 ? 1 : 0.98;
            if ((p.qa == -1 || p.qa >= 4) && e4 + nrec / 4 < e2 * m + nrec / 8 && e4 + nrec / 4 < e1 * m) {
                for (int r = 0; r < nrec; r++) flags[r] |= amap[std::min(2559u, rec_avg(r))] << 16;
                p.sel = true;
                max_sel = 3;
            } else if ((p.qa == -1 || p.qa >= 2) && e2 + nrec / 8 < e1 * m) {
                for (int r = 0; r < nrec; r++) flags[r] |= (amap[std::min(2559u, rec_avg(r))] >> 1) << 16;
                p.sel = true;
                max_sel = 1;
            }
            if (p.qa == -1) {
                if (p.pbits > 0 && p.dbits > 0) {
                    p.sloc = p.dloc - 1;
                    p.pbits--;
                    p.dbits--;
                    p.dloc++;
                } else if (p.dbits >= 2) {
                    p.sloc = p.dloc;
                    p.dbits -= 2;
                    p.dloc += 2;
                } else if (p.qbits >= 2) {
                    p.qbits -= 2;
                    p.ploc -= 2;
                    p.sloc = unsigned(16 - 2 - p.r2);
                    if (p.qbits == 6 && p.qshift == 5) p.qbits--;
                }
                p.qa = 4;
            }
        }

        if (has_r2 || p.r2) {   // READ1 / READ2 split (fqzcomp_qual.c:658-695)
            std::vector<uint64_t> t1(NPOS, 0), t2(NPOS, 0);
            for (int j = 0; j < NPOS; j++)
                for (int s = 0; s < 256; s++) {
                    t1[size_t(j)] += h1[size_t(j) * 256 + s];
                    t2[size_t(j)] += h2[size_t(j) * 256 + s];
                }
            double e1 = 0, e2 = 0;
            for (int j = 0; j < NPOS; j++) {
                if (!t1[size_t(j)] || !t2[size_t(j)]) continue;
                for (int s = 0; s < 256; s++) {
                    const double a = h1[size_t(j) * 256 + s], b = h2[size_t(j) * 256 + s];
                    const double ab = a + b;
                    if (!ab) continue;
                    e1 -= ab * std::log(ab / double(t1[size_t(j)] + t2[size_t(j)]));
                    if (a) e2 -= a * std::log(a / double(t1[size_t(j)]));
                    if (b) e2 -= b * std::log(b / double(t2[size_t(j)]));
                }
            }
            e1 /= std::log(2) * 8;
            e2 /= std::log(2) * 8;
            const double m = p.r2 > 0 ? 1 : 0.95;
            if (e2 + (8 + nrec / 8) < e1 * m) {
                for (int r = 0; r < nrec; r++) {
                    const uint32_t sel = flags[r] >> 16;
                    flags[r] = (flags[r] & 0xffff) | ((sel * 2 + ((flags[r] & F_READ2) ? 1 : 0)) << 16);
                    max_sel = std::max(max_sel, int(flags[r] >> 16));
                }
            }
        }
        if (max_sel > 0) {
            p.sel = true;
            p.max_sel = max_sel;
        }
    }
};

// The rest of fqz_pick_parameters (fqzcomp_qual.c:842-1000).
void pick_finish(Global &g, Param &pm, int strat, int nrec, const uint32_t *lens,
                 const uint32_t *flags, size_t n, const uint32_t qhist[256]) {
    if (strat >= NSTRATS) strat = NSTRATS - 1;
    int dsq[64] = {0, 1, 1, 1, 2, 2, 2, 2, 2, 3, 3, 3, 3, 3, 3, 3,
                   4, 4, 4, 4, 4, 4, 4, 4, 4, 5, 5, 5, 5, 5, 5, 5,
                   5, 5, 5, 5, 6, 6, 6, 6, 6, 6, 6, 6, 6, 6, 6, 6,
                   6, 7, 7, 7, 7, 7, 7, 7, 7, 7, 7, 7, 7, 7, 7, 7};
    pm.qmap_stored = (pm.nsym <= 8 && pm.nsym * 2 < pm.max_sym);
    int r = 1;
    while (r < nrec && lens[r] == lens[0]) r++;
    pm.fixed = (r == nrec);
    pm.qtab_on = false;
    if (strat < NSTRATS - 1) {
        if (pm.pshift < 0) {
            const double v = std::log(double(lens[0]) / (1 << pm.pbits)) / std::log(2) + .5;
            pm.pshift = v > 0 ? int(v) : 0;
        }
        if (pm.nsym <= 4) {
            pm.qshift = 2;
            if (n < 5000000) pm.pbits = 2, pm.pshift = 5;
        } else if (pm.nsym <= 8) {
            pm.qbits = std::min(pm.qbits, 9u);
            pm.qshift = 3;
            if (n < 5000000) pm.qbits = 6;
        }
        if (n < 300000) {
            pm.qbits = unsigned(pm.qshift);
            pm.dbits = 2;
        }
    }
    for (int k = 0; k < 64; k++) dsq[k] = std::min(dsq[k], (1 << pm.dbits) - 1);
    if (pm.qmap_stored) {
        int j = 0;
        for (int s = 0; s < 256; s++) pm.qmap[s] = qhist[s] ? unsigned(j++) : unsigned(INT_MAX);
        pm.max_sym = pm.nsym;
    } else {
        pm.nsym = 255;
        for (int s = 0; s < 256; s++) pm.qmap[s] = unsigned(s);
    }
    g.max_sym = std::max(g.max_sym, pm.max_sym);
    if (pm.qbits)
        for (int s = 0; s < 256; s++) pm.qtab[s] = unsigned(s);
    if (size_t(qhist['~' - '!']) * 2 > n && strat == 3) {     // HiFi qtab
        pm.qtab_on = true;
        unsigned v = 0;
        for (int s = 0; s < 256; s++) {
            if (s == '~' - '!' || s == '~' - '!' + 1 || s % 16 == 0) v++;
            pm.qtab[s] = v;
        }
        pm.qbits = 9, pm.qshift = 3;
        pm.bbits = 6, pm.bloc = 9, pm.boff = 2;
    }
    if (pm.pbits)
        for (int k = 0; k < 1024; k++)
            pm.ptab[k] = std::min((1u << pm.pbits) - 1, unsigned(k >> pm.pshift));
    if (pm.dbits)
        for (int k = 0; k < 256; k++) pm.dtab[k] = unsigned(dsq[std::min(63, k >> pm.dshift)]);
    pm.ptab_on = pm.pbits > 0;
    pm.dtab_on = pm.dbits > 0;
    pm.pflags = (pm.qtab_on ? PF_QTAB : 0) | (pm.dtab_on ? PF_DTAB : 0) |
                (pm.ptab_on ? PF_PTAB : 0) | (pm.sel ? PF_SEL : 0) | (pm.fixed ? PF_LEN : 0) |
                (pm.dedup ? PF_DEDUP : 0) | (pm.qmap_stored ? PF_QMAP : 0);
    g.max_sel = 0;
    if (pm.sel) {
        g.gflags |= GF_STAB;
        int mx = 0;
        for (int k = 0; k < nrec; k++) mx = std::max(mx, int(flags[k] >> 16));
        g.max_sel = mx;
    }
}

// Parameters as the kernels read them; position / delta tables shifted to
// their context location (fqzcomp_qual.c:1067-1076).
FqzDevGlobal dev_params(const Global &g) {
    if (g.nparam > FQZ_MAX_PARAMS) throw std::runtime_error("fqz: too many parameter blocks");
    FqzDevGlobal d;
    std::memset(&d, 0, sizeof d);
    d.gflags = g.gflags;
    d.nparam = uint32_t(g.nparam);
    d.max_sel = uint32_t(g.max_sel);
    d.max_sym = uint32_t(g.max_sym);
    for (int i = 0; i < 256; i++) d.stab[i] = uint8_t(g.stab[i]);
    for (int k = 0; k < g.nparam; k++) {
        const Param &pm = g.p[size_t(k)];
        FqzDevParam &o = d.p[k];
        o.ctx0 = pm.ctx0;
        o.qshift = unsigned(pm.qshift);
        o.qloc = pm.qloc;
        o.sloc = pm.sloc;
        o.bbits = pm.bbits;
        o.bloc = pm.bloc;
        o.boff = pm.boff;
        o.qmask = pm.qmask();
        o.sel = pm.sel;
        o.dedup = pm.dedup;
        o.fixed = pm.fixed;
        for (int i = 0; i < 256; i++) {
            o.qtab[i] = pm.qtab[i];
            o.dtab[i] = pm.dtab[i] << pm.dloc;
            o.qmap[i] = uint8_t(pm.qmap[i]);
        }
        for (int i = 0; i < 1024; i++) o.ptab[i] = pm.ptab[i] << pm.ploc;
    }
    return d;
}

// Sequence bytes per record as the coder reads them: the reference reads
// seq[r][0 .. max(len, boff)) (fqzcomp_qual.c:1163-1173).  Records without
// a sequence get offset ~0.
void gather_seq(GpuCtx &g, unsigned char **seq, int nrec, const uint32_t *lens,
                unsigned boff, const uint8_t **d_seq, const uint64_t **d_off) {
    std::vector<uint64_t> off(size_t(std::max(nrec, 1)), ~0ull);
    uint64_t tot = 0;
    for (int r = 0; r < nrec; r++)
        if (seq[r]) {
            off[size_t(r)] = tot;
            tot += std::max<uint64_t>(lens[r], boff);
        }
    std::vector<uint8_t> buf(size_t(tot) + 1, 0);
    for (int r = 0; r < nrec; r++)
        if (seq[r]) std::memcpy(&buf[off[size_t(r)]], seq[r], std::max<size_t>(lens[r], boff));
    *d_seq = g.upload(buf);
    *d_off = g.upload(off);
}

// Device sequence bytes laid out back to back: record r at the sum of the
// earlier lengths (fqzcomp5 passes pointers into its contiguous seq_buf).
const uint64_t *seq_offsets(GpuCtx &g, int nrec, const uint32_t *lens) {
    std::vector<uint64_t> off(size_t(std::max(nrec, 1)), ~0ull);
    uint64_t o = 0;
    for (int r = 0; r < nrec; r++) off[size_t(r)] = o, o += lens[r];
    return g.upload(off);
}

void copy_gparams(Global &G, const fqz_gparams *gp) {
    // caller-supplied parameters (fqzcomp_qual.c:1040-1045)
    G.vers = gp->vers;
    G.gflags = gp->gflags;
    G.nparam = gp->nparam;
    G.max_sel = gp->max_sel;
    G.max_sym = gp->max_sym;
    for (int i = 0; i < 256; i++) G.stab[i] = gp->stab[i];
    G.p.assign(size_t(gp->nparam), Param());
    for (int k = 0; k < gp->nparam; k++) {
        const fqz_param &a = gp->p[k];
        Param &b = G.p[size_t(k)];
        b.ctx0 = a.context;
        b.pflags = a.pflags;
        b.sel = a.do_sel, b.dedup = a.do_dedup, b.qmap_stored = a.store_qmap,
        b.fixed = a.fixed_len;
        b.qtab_on = a.use_qtab, b.dtab_on = a.use_dtab, b.ptab_on = a.use_ptab;
        b.qbits = a.qbits, b.qloc = a.qloc, b.pbits = a.pbits, b.ploc = a.ploc;
        b.dbits = a.dbits, b.dloc = a.dloc, b.sloc = a.sloc;
        b.bbits = a.bbits, b.bloc = a.bloc, b.boff = a.boff;
        b.max_sym = a.max_sym, b.nsym = a.nsym, b.max_sel = a.max_sel;
        b.qshift = a.qshift, b.pshift = a.pshift, b.dshift = a.dshift;
        std::memcpy(b.qmap, a.qmap, sizeof b.qmap);
        std::memcpy(b.qtab, a.qtab, sizeof b.qtab);
        std::memcpy(b.ptab, a.ptab, sizeof b.ptab);
        std::memcpy(b.dtab, a.dtab, sizeof b.dtab);
    }
}

}  // namespace

// Coder output bytes P (before the 5 flush bytes) from the events' entropy
// sum H = sum log2(total / freq) and slack S = sum -log2(1 - total 2^-24):
// 8 P >= H - 8 (the final range over the initial one is at least 2^-8) and
// 8 P <= H + S (the final range is at most the initial 2^32 - 1); margins
// cover the rounding of the double sums.
uint64_t rc_bytes_lower(double bits) {
    bits = bits * (1.0 - 1e-9) - 8.0 - 64.0;
    return bits > 0 ? uint64_t(bits / 8.0) : 0;
}
uint64_t rc_bytes_upper(double bits, double slack) {
    return uint64_t(((bits + slack) * (1.0 + 1e-9) + 64.0) / 8.0);
}

struct FqzEncReq::Work {
    Global G;
    std::vector<uint8_t> hdr;
    FqzEncJob E{};
    FqzEvJob J{};
    bool parallel = false;
    size_t room = 0;
    uint32_t last[2] = {0, 0};          // last record's event offset and count
    uint32_t P = 0, clen = 0;
    uint64_t lb = 0;                    // lower bound of the output size (0: unknown)
    uint64_t ub = 0;                    // upper bound (valid when lb is)
};

// Every block of the batch goes through each stage before the next one:
// parameters (statistics kernels, host decisions), events, sort, the
// per-model pass (one launch for all blocks), the range chain (one launch,
// one wave per block), the big-number bytes (carry: one launch).
// The hot-model threshold (fqz5_set_hot_min; $FQZ5_HOT_MIN overrides the
// default; 1 sends every eligible quality model through k_fqz_model_hot,
// 0 none).
static std::atomic<uint32_t> &hot_min_var() {
    static std::atomic<uint32_t> v([] {
        const char *e = std::getenv("FQZ5_HOT_MIN");
        return e ? uint32_t(std::strtoul(e, nullptr, 10)) : FQZ_HOT_MIN;
    }());
    return v;
}
uint32_t fqz_hot_min() { return hot_min_var().load(); }
uint32_t fqz_set_hot_min(uint32_t v) { return hot_min_var().exchange(v); }

void fqz_encode_prepare(GpuCtx &g, std::vector<FqzEncReq> &reqs) {
    // $FQZ5_STEP_TRACE: the stages' times (a sync after each: the trace
    // perturbs the overlap it measures)
    static const bool trace = std::getenv("FQZ5_STEP_TRACE") != nullptr;
    using clk = std::chrono::steady_clock;
    std::vector<std::pair<const char *, double>> st;
    auto t_prev = clk::now();
    auto mark = [&](const char *what) {
        if (!trace) return;
        g.sync();
        const auto t = clk::now();
        st.emplace_back(what, std::chrono::duration<double, std::milli>(t - t_prev).count());
        t_prev = t;
    };
    // fqz_pick_parameters of every request without caller parameters, their
    // statistics round trips shared (Tune)
    struct Pick {
        Records rec;
        Tune t;
        uint32_t qhist[256] = {0};
    };
    std::vector<Pick> picks(reqs.size());
    std::vector<size_t> tuned;
    for (size_t i = 0; i < reqs.size(); i++) {
        FqzEncReq &R = reqs[i];
        R.ok = false;
        R.out.clear();
        R.w = std::make_shared<FqzEncReq::Work>();
        if (R.gp) continue;
        Global &G = R.w->G;
        pick_begin(G, R.vers, R.strat, R.nrec, R.lens, R.n);
        picks[i].rec = walk_records(R.nrec, R.lens, R.flags, R.n);
        picks[i].t.launch(g, G.p[0], R.nrec, R.flags, picks[i].rec, R.d_in, picks[i].qhist);
        tuned.push_back(i);
    }
    if (!tuned.empty()) {
        g.sync();
        for (size_t i : tuned) picks[i].t.mid(g);
        g.sync();
        for (size_t i : tuned) {
            FqzEncReq &R = reqs[i];
            picks[i].t.finish();
            pick_finish(R.w->G, R.w->G.p[0], R.strat, R.nrec, R.lens, R.flags, R.n, picks[i].qhist);
        }
    }
    std::vector<FqzEncReq *> par;
    for (FqzEncReq &R : reqs) {
        FqzEncReq::Work &W = *R.w;
        Global &G = W.G;
        const int nrec = R.nrec;
        const size_t n = R.n;
        const uint64_t *d_soff =
            (R.d_seq && nrec > 0) ? seq_offsets(g, nrec, R.lens) : nullptr;
        if (R.gp) copy_gparams(G, R.gp);
        const bool have_seq = nrec > 0 && (R.d_seq || (R.h_seq && R.h_seq[0]));
        if (!have_seq) {
            for (Param &pm : G.p) pm.bbits = pm.bloc = 0;
            G.gflags &= ~unsigned(GF_SEQ);
        } else {
            for (Param &pm : G.p)
                if (pm.bbits) G.gflags |= GF_SEQ;
        }
        if (R.gp) {   // the reference edits the caller's block in place
            R.gp->gflags = G.gflags;
            for (int k = 0; k < R.gp->nparam; k++) {
                R.gp->p[k].bbits = G.p[size_t(k)].bbits;
                R.gp->p[k].bloc = G.p[size_t(k)].bloc;
                for (int i = 0; i < 1024; i++) R.gp->p[k].ptab[i] <<= R.gp->p[k].ploc;
                for (int i = 0; i < 256; i++) R.gp->p[k].dtab[i] <<= R.gp->p[k].dloc;
            }
        }
        W.hdr.assign(16 + 8192 * size_t(std::max(G.nparam, 1)), 0);
        size_t hdr = size_t(varint_put(W.hdr.data(), W.hdr.data() + W.hdr.size(), uint32_t(n)));
        hdr += size_t(put_params(G, W.hdr.data() + hdr));
        W.hdr.resize(hdr);

        const FqzDevGlobal dg = dev_params(G);
        FqzEncJob &E = W.E;
        E.g = g.upload(&dg, 1);
        E.q = R.d_in;
        E.n = n;
        std::vector<uint32_t> lens(R.lens, R.lens + std::max(nrec, 0));
        std::vector<uint32_t> sels(size_t(std::max(nrec, 0))), fl(size_t(std::max(nrec, 0)));
        for (int r = 0; r < nrec; r++) {
            sels[size_t(r)] = R.flags[r] >> 16;
            fl[size_t(r)] = R.flags[r];
        }
        lens.push_back(0);
        sels.push_back(0);
        fl.push_back(0);
        E.len = g.upload(lens);
        E.sel = g.upload(sels);
        E.flags = g.upload(fl);
        E.nrec = uint32_t(std::max(nrec, 0));
        if (have_seq && R.d_seq) {
            E.seq = R.d_seq;
            E.seq_off = d_soff;
        } else if (have_seq) {
            unsigned boff = 0;
            for (const Param &pm : G.p) boff = std::max(boff, pm.boff);
            gather_seq(g, R.h_seq, nrec, R.lens, boff, &E.seq, &E.seq_off);
        }
        W.room = size_t(double(n) * 1.1 + 100000);
        E.out = g.arena.alloc_n<uint8_t>(W.room);
        E.out_len = g.arena.alloc_n<uint32_t>(1);
        // The parallel encoder covers one parameter block and non-empty
        // records (the reference's loop codes the next record's first byte
        // inside an empty record, which only its literal serial form
        // reproduces).
        W.parallel = G.nparam == 1 && !(G.gflags & GF_MULTI) && nrec > 0;
        for (int r = 0; W.parallel && r < nrec; r++) W.parallel = R.lens[r] > 0;
        if (!W.parallel) {
            E.models = g.fqz_tmp.alloc_n<uint8_t>(size_t(FQZ_CTX) * FQZ_QMODEL_BYTES);
            FQZ5_HIP(launch_fqz_model_init(E.models, G.max_sym + 1, g.stream));
            FQZ5_HIP(launch_fqz_encode(E, g.stream));
            continue;
        }
        par.push_back(&R);
        FqzEvJob &J = W.J;
        J.g = E.g;
        J.q = E.q;
        J.len = E.len;
        J.sel = E.sel;
        J.flags = E.flags;
        J.nrec = uint32_t(nrec);
        J.seq = E.seq;
        J.seq_off = E.seq_off;
        std::vector<uint64_t> off(static_cast<size_t>(nrec));
        uint64_t o = 0;
        for (int r = 0; r < nrec; r++) off[size_t(r)] = o, o += R.lens[r];
        J.off = g.upload(off);
        J.nev_rec = g.fqz_tmp.alloc_n<uint32_t>(size_t(nrec));
        uint32_t *ev_off = g.fqz_tmp.alloc_n<uint32_t>(size_t(nrec));
        J.ev_off = ev_off;
        J.dup = g.fqz_tmp.alloc_n<uint8_t>(size_t(nrec));
        FQZ5_HIP(launch_fqz_events(J, 0, g.stream));
        size_t tb = 0;
        FQZ5_HIP(fqz_exclusive_scan(J.nev_rec, ev_off, nrec, nullptr, tb, g.stream));
        void *tmp = g.fqz_tmp.alloc_n<uint8_t>(tb);
        FQZ5_HIP(fqz_exclusive_scan(J.nev_rec, ev_off, nrec, tmp, tb, g.stream));
        g.download(&W.last[0], ev_off + nrec - 1, 1);
        g.download(&W.last[1], J.nev_rec + nrec - 1, 1);
    }
    g.sync();
    mark("pick + counts");

    // events of every block, sorted by model; then one model pass for all
    std::vector<FqzEvJob> jobs;
    for (FqzEncReq *R : par) {
        FqzEvJob &J = R->w->J;
        const uint64_t nev = uint64_t(R->w->last[0]) + R->w->last[1];
        if (nev >= (1ull << 31)) throw std::runtime_error("fqz: block too large");
        J.nev = uint32_t(nev);
        J.key = g.sort_tmp.alloc_n<uint32_t>(nev);
        J.val = g.sort_tmp.alloc_n<uint64_t>(nev);
        uint32_t *skey = g.ev_tmp.alloc_n<uint32_t>(nev);
        uint64_t *sval = g.ev_tmp.alloc_n<uint64_t>(nev + 2);   // + room: model_run reads pairs
        J.skey = skey;
        J.sval = sval;
        J.code = g.ev_tmp.alloc_n<uint64_t>(nev);
        {
            ProfSpan sp(PK_FQZ_EV_FILL, g.stream);
            FQZ5_HIP(launch_fqz_events(J, 1, g.stream));
            sp.end(double(R->n));
        }
        size_t tb = 0;
        FQZ5_HIP(fqz_sort_by_model(J.key, skey, J.val, sval, int(nev), int(FQZ_MODEL_BITS),
                                   nullptr, tb, g.stream));
        void *tmp = g.sort_tmp.alloc_n<uint8_t>(tb);
        FQZ5_HIP(fqz_sort_by_model(J.key, skey, J.val, sval, int(nev), int(FQZ_MODEL_BITS), tmp,
                                   tb, g.stream));
        // the unsorted events and the sort's buffers back to the pool, so
        // the next block's reuse them (the peak holds one block's, not all)
        g.tmp_done(g.sort_tmp);
        J.seg_lo = g.fqz_tmp.alloc_n<uint32_t>(FQZ_NMODELS);
        J.seg_hi = g.fqz_tmp.alloc_n<uint32_t>(FQZ_NMODELS);
        g.memset0(J.seg_lo, FQZ_NMODELS * 4);
        g.memset0(J.seg_hi, FQZ_NMODELS * 4);
        FQZ5_HIP(launch_fqz_events(J, 2, g.stream));
        J.scratch = g.fqz_tmp.alloc_n<uint8_t>(8192);
        jobs.push_back(J);
    }
    mark("events + sort");
    const int np = int(par.size());
    if (np && std::getenv("FQZ5_FQZ_SEGSTATS")) {   // diagnostics: events per model
        for (int k = 0; k < np; k++) {
            std::vector<uint32_t> lo(FQZ_NMODELS), hi(FQZ_NMODELS);
            g.download(lo.data(), jobs[size_t(k)].seg_lo, FQZ_NMODELS);
            g.download(hi.data(), jobs[size_t(k)].seg_hi, FQZ_NMODELS);
            g.sync();
            std::vector<uint32_t> c;
            for (uint32_t m = 0; m < FQZ_NMODELS; m++) if (hi[m] > lo[m]) c.push_back(hi[m] - lo[m]);
            std::sort(c.rbegin(), c.rend());
            std::fprintf(stderr, "fqz job %d: %u events, %zu models, top:", k, jobs[size_t(k)].nev, c.size());
            for (size_t i = 0; i < c.size() && i < 12; i++) std::fprintf(stderr, " %u", c[i]);
            std::fprintf(stderr, "\n");
        }
    }
    if (np) {
        const uint32_t hot_min = fqz_hot_min();
        uint32_t stride = 1;
        for (const FqzEvJob &J : jobs)
            stride = std::max(stride, 1u + std::min(FQZ_M_SEL, J.nev / std::max(hot_min, 1u) + 1));
        uint32_t *hot = g.fqz_tmp.alloc_n<uint32_t>(size_t(stride) * size_t(np));
        g.memset0(hot, size_t(stride) * size_t(np) * 4);
        const FqzEvJob *d_jobs = g.upload(jobs);
        double qb = 0;
        for (FqzEncReq *R : par) qb += double(R->n);
        if (hot_min) {
            ProfSpan sp(PK_FQZ_MODEL_HOT, g.stream);
            FQZ5_HIP(launch_fqz_model_hot(d_jobs, np, hot, stride, hot_min, g.stream));
            sp.end(qb);
        }
        FQZ5_HIP(launch_fqz_model_pass(d_jobs, np, hot_min, g.stream));
        mark("model passes");
        // the entropy of each block's events and the coder's slack: lower
        // and upper bounds of its size
        constexpr uint32_t EB = 1024;
        double *part = g.fqz_tmp.alloc_n<double>(2 * size_t(EB) * size_t(np));
        for (int k = 0; k < np; k++)
            FQZ5_HIP(launch_fqz_entropy(jobs[size_t(k)], part + 2 * size_t(k) * EB, EB, g.stream));
        std::vector<double> hp(2 * size_t(EB) * size_t(np));
        g.download(hp.data(), part, hp.size());
        g.sync();
        for (int k = 0; k < np; k++) {
            double bits = 0, slack = 0;
            for (uint32_t b = 0; b < EB; b++) {
                bits += hp[2 * size_t(k) * EB + b];
                slack += hp[(2 * size_t(k) + 1) * EB + b];
            }
            FqzEncReq::Work &W = *par[size_t(k)]->w;
            W.lb = uint64_t(W.hdr.size()) + rc_bytes_lower(bits) + 5;
            W.ub = uint64_t(W.hdr.size()) + rc_bytes_upper(bits, slack) + 5;
        }
        mark("entropy");
    }
    g.tmp_done(g.sort_tmp);                // the unsorted events back to the pool
    if (trace && !st.empty()) {
        std::string line = "fqz prepare:";
        for (auto &x : st) line += " " + std::string(x.first) + " " + std::to_string(int(x.second * 10) / 10.0).substr(0, 6) + " ms,";
        std::fprintf(stderr, "%s\n", line.c_str());
    }
}

// The range coder back end for event jobs whose rec[] holds every event in
// stream order: the range chain of every job (one wave each, hedged), the
// scan of the byte shifts, and the big-number bytes into J.out / *J.out_len.
void rc_backend(GpuCtx &g, std::vector<FqzEvJob *> &js) {
    const int np = int(js.size());
    if (!np) return;
    std::vector<FqzEvJob> rj;
    // per job: the hedge claim word, zeroed
    uint32_t *d_words = g.fqz_tmp.alloc_n<uint32_t>(size_t(np));
    g.memset0(d_words, size_t(np) * 4);
    uint32_t max_nev = 0;
    for (int k = 0; k < np; k++) {
        FqzEvJob *J = js[size_t(k)];
        J->addend = g.fqz_tmp.alloc_n<uint32_t>(J->nev);
        J->shifts = g.fqz_tmp.alloc_n<uint32_t>(J->nev + 1);
        J->ck = g.fqz_tmp.alloc_n<uint32_t>(J->nev / 64 + 1);
        J->done = nullptr;
        max_nev = std::max(max_nev, J->nev);
        rj.push_back(*J);
    }
    // hedge: each range chain on 2-4 CUs
    HedgeShare share(size_t(g.cus));
    const size_t copies = hedge_copies(rj.size(), share.cus);
    if (copies > 1) {
        for (size_t k = 0; k < rj.size(); k++) rj[k].done = d_words + k;
        for (size_t c = 1; c < copies; c++) rj.insert(rj.end(), rj.begin(), rj.begin() + long(np));
    }
    const FqzEvJob *d_rj = g.upload(rj);
    FQZ5_HIP(launch_fqz_rc(d_rj, int(rj.size()), np, max_nev, 0, g.stream));
    EventPair ev(prof_on(), g.stream);
    FQZ5_HIP(launch_fqz_rc(d_rj, int(rj.size()), np, max_nev, 1, g.stream));
    ev.stop(g.stream);
    FQZ5_HIP(launch_fqz_rc(d_rj, int(rj.size()), np, max_nev, 2, g.stream));
    std::vector<uint32_t> P(size_t(np), 0);
    for (int k = 0; k < np; k++) {
        FqzEvJob &J = *js[size_t(k)];
        uint32_t *pos = g.fqz_tmp.alloc_n<uint32_t>(J.nev + 1);
        g.memset0(J.shifts + J.nev, 4);
        size_t tb = 0;
        FQZ5_HIP(fqz_exclusive_scan(J.shifts, pos, int(J.nev + 1), nullptr, tb, g.stream));
        void *tmp = g.fqz_tmp.alloc_n<uint8_t>(tb);
        FQZ5_HIP(fqz_exclusive_scan(J.shifts, pos, int(J.nev + 1), tmp, tb, g.stream));
        J.pos = pos;
        J.nshift = pos + J.nev;
        g.download(&P[size_t(k)], pos + J.nev, 1);
    }
    g.sync();
    if (ev.on) {   // the chain reads 16 B of event record per event
        double ev_n = 0;
        for (FqzEvJob *J : js) ev_n += J->nev;
        prof_add(PK_FQZ_RC, ev.ms(), ev_n * 16.0);
    }
    for (int k = 0; k < np; k++) {
        FqzEvJob &J = *js[size_t(k)];
        J.nwords = (P[size_t(k)] + 5 + 3) / 4 + 2;
        J.acc = reinterpret_cast<unsigned long long *>(g.fqz_tmp.alloc_n<uint64_t>(J.nwords));
        g.memset0(J.acc, size_t(J.nwords) * 8);
        FQZ5_HIP(launch_fqz_bytes(J, 0, g.stream));
        // carries through the columns: codes, their scan, digits
        uint32_t *sw = g.fqz_tmp.alloc_n<uint32_t>(J.nwords);
        uint8_t *code = g.fqz_tmp.alloc_n<uint8_t>(J.nwords);
        uint8_t *pref = g.fqz_tmp.alloc_n<uint8_t>(J.nwords);
        FQZ5_HIP(launch_fqz_norm(J, 1, sw, code, g.stream));
        size_t tb = 0;
        FQZ5_HIP(fqz_carry_scan(code, pref, int(J.nwords), nullptr, tb, g.stream));
        void *tmp = g.fqz_tmp.alloc_n<uint8_t>(tb);
        FQZ5_HIP(fqz_carry_scan(code, pref, int(J.nwords), tmp, tb, g.stream));
        FQZ5_HIP(launch_fqz_norm(J, 2, sw, pref, g.stream));
        FQZ5_HIP(launch_fqz_bytes(J, 2, g.stream));
    }
}

// The range chain and the output bytes of every parallel request not in
// `skip` (skip[i] != 0: request i is left without output), and the sizes.
void fqz_encode_finish(GpuCtx &g, std::vector<FqzEncReq> &reqs, const std::vector<char> *skip) {
    std::vector<FqzEncReq *> par;
    for (size_t i = 0; i < reqs.size(); i++)
        if (reqs[i].w->parallel && !(skip && (*skip)[i])) par.push_back(&reqs[i]);
    const int np = int(par.size());
    std::vector<FqzEvJob *> js;
    for (int k = 0; k < np; k++) {
        FqzEncReq::Work &W = *par[size_t(k)]->w;
        FqzEvJob &J = W.J;
        J.rec = g.fqz_tmp.alloc_n<uint4>(J.nev + RC_PAD);
        FQZ5_HIP(launch_fqz_expand(J, g.stream));
        J.out = W.E.out;
        J.out_len = W.E.out_len;
        js.push_back(&J);
    }
    g.tmp_done(g.ev_tmp);                  // the sorted events, now records, back to the pool
    rc_backend(g, js);

    for (size_t i = 0; i < reqs.size(); i++)
        if (!(skip && (*skip)[i])) g.download(&reqs[i].w->clen, reqs[i].w->E.out_len, 1);
    // the outputs and sizes are all that is left to need: the event tables
    // and the coder's buffers go back to the pool
    g.tmp_done(g.fqz_tmp);
    for (size_t i = 0; i < reqs.size(); i++) {
        FqzEncReq &R = reqs[i];
        FqzEncReq::Work &W = *R.w;
        for (int r = 0; r < R.nrec; r++) R.flags[r] &= 0xffff;
        if (skip && (*skip)[i]) continue;
        if (W.clen > W.room) continue;   // (cannot happen: the bound covers the coder)
        if (W.lb > uint64_t(W.hdr.size()) + W.clen)   // the entropy bound is a theorem
            throw std::runtime_error("fqz: size below its entropy bound");
        if (W.ub && W.ub < uint64_t(W.hdr.size()) + W.clen)   // and so is the slack bound (0: none, serial path)
            throw std::runtime_error("fqz: size above its upper bound");
        Piece h;
        h.host = W.hdr;
        Piece d;
        d.dev = W.E.out;
        d.len = W.clen;
        R.out.push_back(std::move(h));
        R.out.push_back(d);
        R.ok = true;
    }
}

uint64_t fqz_size_lower_bound(const FqzEncReq &r) { return r.w ? r.w->lb : 0; }
uint64_t fqz_size_upper_bound(const FqzEncReq &r) { return r.w && r.w->lb ? r.w->ub : 0; }

void fqz_encode_batch(GpuCtx &g, std::vector<FqzEncReq> &reqs) {
    static const bool trace = std::getenv("FQZ5_STEP_TRACE") != nullptr;
    const auto t0 = std::chrono::steady_clock::now();
    fqz_encode_prepare(g, reqs);
    const auto t1 = std::chrono::steady_clock::now();
    fqz_encode_finish(g, reqs, nullptr);
    if (trace) {
        size_t n = 0;
        for (const FqzEncReq &R : reqs) n = std::max(n, R.n);
        std::fprintf(stderr, "fqz encode: %zu requests (largest %zu symbols): prepare %.1f ms, "
                     "range chains + bytes %.1f ms\n", reqs.size(), n,
                     std::chrono::duration<double, std::milli>(t1 - t0).count(),
                     std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t1).count());
    }
}

uint8_t *fqz_encode_gpu(int vers, fqz_slice *s, const uint8_t *in, size_t n, size_t *out_size,
                        int strat, fqz_gparams *gp) {
    GpuCtx &g = gpu();
    g.reset();
    std::vector<FqzEncReq> reqs(1);
    FqzEncReq &R = reqs[0];
    R.d_in = g.upload(in, n);
    R.n = n;
    R.nrec = s ? s->num_records : 0;
    R.lens = s ? s->len : nullptr;
    R.flags = s ? s->flags : nullptr;
    R.h_seq = s ? s->seq : nullptr;
    R.vers = vers;
    R.strat = strat;
    R.gp = gp;
    fqz_encode_batch(g, reqs);
    if (!R.ok) throw std::runtime_error("fqz: output overflow");
    const uint32_t sz = layout_size(R.out);
    uint8_t *out = static_cast<uint8_t *>(std::malloc(sz ? sz : 1));
    if (!out) throw std::runtime_error("fqz: out of host memory");
    write_layout_host(g, R.out, out);
    *out_size = sz;
    return out;
}

static std::atomic<uint64_t> g_dec_blocks[2];
uint64_t fqz_dec_blocks(bool small) { return g_dec_blocks[small ? 1 : 0].load(); }
int small_copies() {   // read per launch (experiments change it in-process)
    const char *e = std::getenv("FQZ5_SMALL_COPIES");
    return e ? std::max(1, std::atoi(e)) : 2;
}

struct FqzDecReq::Work {
    Global G;
    FqzDecJob D{};
    int ne = 1, map_mode = 0;
    bool seq_ctx = false, qid = true, dedup = false, rev = false;
    bool small = false, dt = false;   // the small-alphabet decoder; delta terms
    uint32_t total = 0, cap = 0;
    int32_t st = 0;
};

namespace {

// every set of the small decoder's 4-way cache starts with the fresh models
// of 4 distinct contexts that map to it (fqz_decode_small.hip, same hash)
bool small_sets_ok(uint32_t ns) {
    static std::mutex mu;
    static std::map<uint32_t, bool> seen;
    std::lock_guard<std::mutex> lk(mu);
    auto it = seen.find(ns);
    if (it != seen.end()) return it->second;
    std::vector<uint8_t> cnt(ns, 0);
    const uint64_t ns8 = uint64_t(ns << 8) & 0xffffffu;
    for (uint32_t c = 0; c < uint32_t(FQZ_CTX); c++) {
        const uint64_t h = (c * 0x9E3779u) & 0xffffffu;
        uint8_t &k = cnt[size_t((h * ns8) >> 32)];
        if (k < FQZ_SMALL_WAYS) k++;
    }
    bool ok = ns > 0 && (ns << 8) <= 0xffffffu;
    for (uint8_t k : cnt) ok = ok && k == FQZ_SMALL_WAYS;
    return seen[ns] = ok;
}

void dec_lists(GpuCtx &g, FqzDecReq::Work &W) {
    FqzDecJob &D = W.D;
    D.cap_list = (W.dedup || W.rev || W.map_mode == 2) ? std::min<uint32_t>(W.cap, W.total + 1) : 0;
    const size_t c = std::max<uint32_t>(D.cap_list, 1);
    D.recs = g.arena.alloc_n<uint4>(W.map_mode == 2 ? c : 1);
    D.dups = g.arena.alloc_n<uint2>(W.dedup ? c : 1);
    D.revs = g.arena.alloc_n<uint2>(W.rev ? c : 1);
}

}  // namespace

// All blocks of the batch decode in one launch per decoder variant (one
// workgroup each), then the qmap / duplicate / reversal fix-ups.
void fqz_decode_batch(GpuCtx &g, std::vector<FqzDecReq> &reqs) {
    std::vector<FqzDecReq *> live;
    for (FqzDecReq &R : reqs) {
        R.ok = false;
        R.out_size = 0;
        R.w = std::make_shared<FqzDecReq::Work>();
        FqzDecReq::Work &W = *R.w;
        uint32_t total = 0;
        const int vk = varint_get(R.h_in, R.h_in + R.in_size, &total);
        if (vk <= 0) continue;
        size_t k = size_t(vk);
        const int u = get_params(W.G, R.h_in + k, R.in_size - k);
        if (u < 0) continue;
        k += size_t(u);
        const Global &G = W.G;
        const uint32_t nlive = uint32_t(G.max_sym) + 1;
        if (nlive > FQZ_DEC_MAX_LIVE) continue;
        if (R.d_out && R.out_cap < total) continue;
        W.total = total;
        R.out_size = total;
        const FqzDevGlobal dg = dev_params(G);
        FqzDecJob &D = W.D;
        D.g = g.upload(&dg, 1);
        D.in = R.d_in + k;
        D.in_len = R.in_size - k;
        D.n = total;
        const int nrec = R.nrec;
        if (nrec > 0 && R.d_seq) {
            D.seq = R.d_seq;
            D.seq_off = seq_offsets(g, nrec, R.lens);
            D.nseq = uint32_t(nrec);
        } else if (nrec > 0 && R.h_seq && R.lens) {
            unsigned boff = 0;
            for (const Param &pm : G.p) boff = std::max(boff, pm.boff);
            gather_seq(g, R.h_seq, nrec, R.lens, boff, &D.seq, &D.seq_off);
            D.nseq = uint32_t(nrec);
        }
        D.nlengths = R.lengths && R.nlengths > 0 ? uint32_t(R.nlengths) : 0;
        D.lengths = g.arena.alloc_n<uint32_t>(std::max<uint32_t>(D.nlengths, 1));
        D.out = R.d_out ? R.d_out : g.arena.alloc_n<uint8_t>(std::max<uint32_t>(total, 1));
        R.d_out = D.out;
        D.status = g.arena.alloc_n<int32_t>(1);
        D.nrec_out = g.arena.alloc_n<uint32_t>(1);
        D.counts = g.arena.alloc_n<uint32_t>(32);
        g.memset0(D.counts, 32 * sizeof(uint32_t));
        D.ment = fqz_dec_model_bytes(nlive);
        D.nsets = FQZ_DEC_CACHE_BYTES / D.ment;
        D.back = nullptr;
        if (nlive > 62) {
            D.back_hi = g.arena.alloc_n<uint32_t>(size_t(FQZ_CTX) * 64);
            D.hi_bits = g.arena.alloc_n<uint32_t>(FQZ_CTX / 32);
            g.memset0(D.hi_bits, FQZ_CTX / 8);
        }
        for (const Param &pm : G.p) {
            W.seq_ctx = W.seq_ctx || pm.bbits > 0;
            W.dedup = W.dedup || pm.dedup;
            for (int i = 0; i < 256; i++) {
                W.qid = W.qid && (pm.qtab[i] & 0xffffu) == (G.p[0].qtab[i] & 0xffffu);   // one shared qtab
                W.map_mode = W.map_mode || pm.qmap[i] != unsigned(i);
            }
        }
        W.seq_ctx = W.seq_ctx && D.seq;
        W.rev = (G.gflags & GF_REV) != 0;
        if (W.map_mode) W.map_mode = G.nparam > 1 ? 2 : 1;
        W.ne = nlive + 2 <= 64 ? 1 : 2;
        // the small-alphabet decoder: <= 9 live symbols, qtab the identity on
        // them, no sequence bases in the context (fqz_decode_small.hip)
        bool ident = true;
        for (const Param &pm : G.p) {
            for (uint32_t i = 0; i < nlive; i++) ident = ident && (pm.qtab[i] & 0xffffu) == i;
            for (int i = 0; i < 256; i++) W.dt = W.dt || pm.dtab[i] != 0;
        }
        uint32_t small_ns = fqz_small_sets(uint32_t(G.nparam));
        if (const char *e = std::getenv("FQZ5_DEC_SETS"))   // tests: force misses
            small_ns = std::max<uint32_t>(1, std::min<uint32_t>(small_ns, uint32_t(std::atoi(e))));
        W.small = small_decoder_on() && nlive <= FQZ_SMALL_MAX_LIVE && nlive >= 2 && ident &&
                  !W.seq_ctx && small_sets_ok(small_ns);
        if (W.small) {
            D.ment = FQZ_SMALL_MODEL_BYTES;
            D.nsets = small_ns;
            D.back = g.arena.alloc_n<uint8_t>(size_t(FQZ_CTX) * D.ment);
            D.back_hi = nullptr;
            D.hi_bits = nullptr;
        } else {
            D.back = g.arena.alloc_n<uint8_t>(size_t(FQZ_CTX) * D.ment);
        }
        // record lists: sized for the records the caller announced, grown to
        // the byte count (every record holds at least one byte) on overflow
        W.cap = std::max<uint32_t>({D.nlengths, D.nseq, 1u}) + 1024;
        dec_lists(g, W);
        live.push_back(&R);
    }
    auto launch_group = [&](const std::vector<FqzDecReq *> &rs) {
        // variants: the general decoder by (ne, seq, qid), then the small one
        // by dt (variant 8 + dt)
        for (int var = 0; var < 10; var++) {
            const bool smallv = var >= 8;
            const int ne = 1 + (var >> 2), sq = (var >> 1) & 1, qi = var & 1, dtv = var & 1;
            std::vector<FqzDecJob> js;
            std::vector<uint64_t> steps;
            std::vector<uint32_t> live_syms;
            for (FqzDecReq *R : rs) {
                const FqzDecReq::Work &W = *R->w;
                const bool mine = smallv ? (W.small && int(W.dt) == dtv)
                                         : (!W.small && W.ne == ne && int(W.seq_ctx) == sq && int(W.qid) == qi);
                if (mine) {
                    js.push_back(W.D);
                    steps.push_back(W.D.n);
                    live_syms.push_back(uint32_t(W.G.max_sym) + 1);
                }
            }
            // hedge: copies of the long blocks on spare CUs (one
            // workgroup per CU: its LDS), as the rANS decode chains
            // (DESIGN.md section 4); a copy needs its own backing store
            HedgeShare share(size_t(g.cus));
            const bool long_block =
                !steps.empty() && *std::max_element(steps.begin(), steps.end()) >= (1u << 20);
            std::vector<int> cp = long_block ? hedge_plan(steps, share.cus)
                                             : std::vector<int>(js.size(), 1);
            // the small decoder's copies each keep a 1.5 MB backing store
            // that should stay in its XCD's L2 ($FQZ5_SMALL_COPIES, default 2)
            if (smallv)
                for (int &c : cp) c = std::min(c, small_copies());
            const size_t nj = js.size();
            for (size_t k = 0; k < nj; k++) {
                if (cp[k] <= 1) continue;
                uint32_t *done = g.arena.alloc_n<uint32_t>(1);
                g.memset0(done, 4);
                js[k].done = done;
                for (int c = 1; c < cp[k]; c++) {
                    FqzDecJob J = js[k];
                    J.back = g.arena.alloc_n<uint8_t>(size_t(FQZ_CTX) * J.ment);
                    if (!smallv && ne == 2) {
                        J.back_hi = g.arena.alloc_n<uint32_t>(size_t(FQZ_CTX) * 64);
                        J.hi_bits = g.arena.alloc_n<uint32_t>(FQZ_CTX / 32);
                        g.memset0(J.hi_bits, FQZ_CTX / 8);
                    }
                    js.push_back(J);
                    live_syms.push_back(live_syms[k]);
                }
            }
            // the small decoder's backing stores start as every context's
            // fresh model (again on a second launch of the same block)
            if (smallv)
                for (size_t k = 0; k < js.size(); k++)
                    FQZ5_HIP(launch_fqz_small_back(js[k].back, live_syms[k], g.stream));
            if (!js.empty()) {
                g_dec_blocks[smallv ? 1 : 0] += nj;
                EventPair ev(prof_on(), g.stream);
                if (smallv)
                    FQZ5_HIP(launch_fqz_dec_small(g.upload(js), int(js.size()), dtv != 0, g.stream));
                else
                    FQZ5_HIP(launch_fqz_dec(g.upload(js), int(js.size()), ne, sq != 0,
                                            qi != 0, g.stream));
                ev.stop(g.stream);
                if (ev.on) {   // compressed bytes in, quality bytes out
                    g.sync();
                    double b = 0;
                    for (size_t k = 0; k < nj; k++) b += double(js[k].in_len) + double(js[k].n);
                    prof_add(PK_FQZ_DEC, ev.ms(), b);
                }
            }
        }
        for (FqzDecReq *R : rs) {
            FqzDecReq::Work &W = *R->w;
            FQZ5_HIP(launch_fqz_dec_fix(W.D, W.map_mode, W.dedup, W.rev, g.stream));
            g.download(&W.st, W.D.status, 1);
        }
        g.sync();
    };
    launch_group(live);
    std::vector<FqzDecReq *> again;
    for (FqzDecReq *R : live)
        if (R->w->st == -2) {
            R->w->cap = R->w->total + 1;
            dec_lists(g, *R->w);
            again.push_back(R);
        }
    if (!again.empty()) launch_group(again);
    if (std::getenv("FQZ5_DEBUG"))
        for (FqzDecReq *R : live) {
            const FqzDecReq::Work &W = *R->w;
            uint32_t c[5];
            uint64_t pr[6];
            g.download(c, W.D.counts, 5);
            g.download(pr, reinterpret_cast<const uint64_t *>(W.D.counts + 8), 6);
            g.sync();
            std::fprintf(stderr, "[fqz dec] n=%u ment=%u sets=%u recs=%u dups=%u revs=%u misses=%u slow=%u\n",
                         W.total, W.D.ment, W.D.nsets, c[0], c[1], c[2], c[3], c[4]);
            if (pr[0] | pr[1])
                std::fprintf(stderr, "[fqz dec] probe: %.1f cycles/symbol inside the run asm over %llu symbols "
                             "(%.1f%% of %u), %llu asm calls; %.0f cycles per miss() call, %.0f cycles "
                             "between runs (%llu)\n",
                             double(pr[0]) / double(pr[1] ? pr[1] : 1), (unsigned long long)pr[1],
                             100.0 * double(pr[1]) / W.total, W.total, (unsigned long long)pr[2],
                             double(pr[3]) / double(c[3] ? c[3] : 1), double(pr[4]) / double(pr[5] ? pr[5] : 1),
                             (unsigned long long)pr[5]);
        }
    std::vector<std::vector<uint32_t>> lens(live.size());
    for (size_t i = 0; i < live.size(); i++) {
        FqzDecReq &R = *live[i];
        if (R.w->st) continue;
        lens[i].resize(R.w->D.nlengths);
        g.download(lens[i].data(), R.w->D.lengths, lens[i].size());
    }
    g.sync();
    for (size_t i = 0; i < live.size(); i++) {
        FqzDecReq &R = *live[i];
        if (R.w->st) continue;
        for (size_t r = 0; r < lens[i].size(); r++) R.lengths[r] = int(lens[i][r]);
        R.ok = true;
    }
}

uint8_t *fqz_decode_gpu(const uint8_t *in, size_t in_size, size_t *out_size, int *lengths,
                        int nlengths, fqz_slice *s) {
    GpuCtx &g = gpu();
    g.reset();
    std::vector<FqzDecReq> reqs(1);
    FqzDecReq &R = reqs[0];
    R.h_in = in;
    R.d_in = g.upload(in, in_size);
    R.in_size = in_size;
    R.lengths = lengths;
    R.nlengths = nlengths;
    if (s && s->seq && s->num_records > 0 && s->len) {
        R.nrec = s->num_records;
        R.lens = s->len;
        R.h_seq = s->seq;
    }
    fqz_decode_batch(g, reqs);
    *out_size = R.out_size;
    if (!R.ok) return nullptr;
    uint8_t *out = static_cast<uint8_t *>(std::malloc(R.out_size ? R.out_size : 1));
    if (!out) throw std::runtime_error("fqz: out of host memory");
    g.download(out, R.d_out, R.out_size);
    g.sync();
    return out;
}

}  // namespace fqz5
