// host_dec.cpp — the adaptive-model decode chains on host cores: the
// fqzcomp_qual decoder (uncompress_block_fqz2f, htscodecs
// fqzcomp_qual.c:1410-1634) and the sequence context model (decode_seq,
// fqzcomp5.c:1272-1406).
//
// Both are one dependent chain per block: every symbol needs the coder state
// and the model its predecessor selected.  A GPU wave issues one instruction
// per ~4.5 cycles, so one chain runs 5-15x slower there than on a host core;
// the GPU wins only with many blocks at once.  fqz5_decode_sections runs
// these chains here, on a pool of host threads beside the GPU's rANS and name
// work, when the host mode asks for it (fqz5_set_host_decode).  Same inputs,
// same bytes as the GPU decoders (tests/test_host_dec.py checks both against
// the reference's vectors).
//
// Models (own layout, reference arithmetic): an adaptive list per context
// (c_simple_model.h: freq +16, halved past 65519, one bubble step per
// update) stored as parallel u16 frequency / u8 symbol arrays; the 4- and
// 2-symbol sequence models (c_small_model.h: +1, halved at a total of 255)
// as four u8 counts.
#include <sched.h>
#include <algorithm>
#include <cstdint>
#include <cstdlib>
#include <atomic>
#include <cstring>
#include <vector>

#include "../../include/fqz5_mi355x.h"
#include "fqz_format.hpp"
#include "host_dec.hpp"
#include "rans_format.hpp"

namespace fqz5 {
namespace host {

namespace {

constexpr uint32_t MAXF = 65519u, STEP = 16u, TOP = 1u << 24;

// c_range_coder.h decoder: RC_StartDecode, RC_GetFreq, RC_Decode (the
// renormalisation stops at the end of the input)
struct Coder {
    uint32_t range = 0xFFFFFFFFu, code = 0;
    const uint8_t *p, *end;
    Coder(const uint8_t *in, size_t n) : p(in), end(in + n) {
        if (n < 5) { p = end; return; }
        for (int i = 0; i < 5; i++) code = (code << 8) | *p++;
    }
    // the target of a total; the range keeps its division either way
    uint32_t target(uint32_t tot) {
        if (!tot || range < tot) return 0;
        range /= tot;
        return code / range;
    }
    void take(uint32_t cum, uint32_t f) {
        code -= cum * range;
        range *= f;
        while (range < TOP) {
            if (p >= end) return;
            code = (code << 8) | *p++;
            range <<= 8;
        }
    }
};

// An adaptive list of up to `cap` symbols (cap <= 256) in one run of words:
// word 0 the total, then per slot {u16 freq, u16 symbol}, then a zero
// frequency after the live slots (the halving loop's end).  (The quality
// lists are cut to the live symbols: the reference's dead slots are never
// decoded.)
struct List {
    uint32_t *w;
    uint32_t &total() { return w[0]; }
    uint16_t &f(int k) { return reinterpret_cast<uint16_t *>(w + 1)[2 * k]; }
    uint16_t &s(int k) { return reinterpret_cast<uint16_t *>(w + 1)[2 * k + 1]; }
};

inline void list_init(List m, int cap, int live) {
    for (int i = 0; i < cap; i++) {
        m.s(i) = uint16_t(i);
        m.f(i) = i < live ? 1 : 0;
    }
    m.f(cap) = 0;
    m.s(cap) = 0;
    m.total() = uint32_t(live);
}

// SIMPLE_MODEL decodeSymbol: 0 without any update when the target is out of
// range (a damaged stream)
inline uint32_t list_decode(List m, Coder &c) {
    uint32_t total = m.total();
    const uint32_t t = c.target(total);
    if (t >= total) return 0;
    uint16_t *e = reinterpret_cast<uint16_t *>(m.w + 1);
    uint32_t acc = 0;
    int k = 0;
    while (acc + e[2 * k] <= t) acc += e[2 * k++];
    c.take(acc, e[2 * k]);
    const uint32_t sym = e[2 * k + 1];
    e[2 * k] = uint16_t(e[2 * k] + STEP);
    total += STEP;
    if (total > MAXF) {
        total = 0;
        for (int i = 0; e[2 * i]; i++) {
            e[2 * i] = uint16_t(e[2 * i] - (e[2 * i] >> 1));
            total += e[2 * i];
        }
    }
    m.total() = total;
    if (k > 0 && e[2 * k] > e[2 * k - 2]) {
        uint32_t *p = m.w + 1;
        std::swap(p[k], p[k - 1]);
    }
    return sym;
}

// storage for lists of capacity cap
struct ListStore {
    int cap = 0;
    size_t words = 0;
    std::vector<uint32_t> mem;
    void reset(int c, size_t n) {
        cap = c;
        words = size_t(cap) + 2;
        if (mem.size() < n * words) mem.resize(n * words);
    }
    List at(size_t i) { return List{mem.data() + i * words}; }
};

inline uint32_t base2(uint8_t b) {
    switch (b) {
    case 'C': case 'c': return 1;
    case 'G': case 'g': return 2;
    case 'T': case 't': case 'U': case 'u': return 3;
    default: return 0;
    }
}

// the per-thread model memory, kept between blocks
struct FqzScratch {
    ListStore q;                         // FQZ_CTX quality lists
    ListStore sm;                        // sel, len[4], rev, dup
};
thread_local FqzScratch t_fqz;

struct SeqScratch {
    std::vector<uint8_t> ctx;            // 4 u8 counts per k-mer context
};
thread_local SeqScratch t_seq;

}  // namespace

int fqz_decode(const uint8_t *in, size_t in_size, uint8_t *out, size_t out_cap, size_t *out_size,
               int *lengths, int nlengths, const uint8_t *const *seq, int nrec) {
    using namespace fqz;
    uint32_t total = 0;
    int k = varint_get(in, in + in_size, &total);
    if (k <= 0) return -1;
    Global G;
    const int u = get_params(G, in + k, in_size - size_t(k));
    if (u < 0) return -1;
    k += u;
    if (total > out_cap) return -1;
    *out_size = total;
    const int live = G.max_sym + 1;
    FqzScratch &S = t_fqz;
    // every context's list starts fresh: one built, copied to all
    S.q.reset(live, CTX_SIZE);
    list_init(S.q.at(0), live, live);
    for (size_t c = 1; c < size_t(CTX_SIZE); c++)
        std::memcpy(S.q.mem.data() + c * S.q.words, S.q.mem.data(), S.q.words * 4);
    S.sm.reset(256, 7);
    List len_m[4], sel_m = S.sm.at(4), rev_m = S.sm.at(5), dup_m = S.sm.at(6);
    for (int b = 0; b < 4; b++) {
        len_m[b] = S.sm.at(size_t(b));
        list_init(len_m[b], 256, 256);
    }
    list_init(sel_m, 256, G.max_sel + 1);
    list_init(rev_m, 2, 2);
    list_init(dup_m, 2, 2);
    // the parameter tables with their context shifts applied
    // (uncompress_block_fqz2f: ptab <<= ploc, dtab <<= dloc)
    for (Param &pm : G.p) {
        for (int i = 0; i < 1024; i++) pm.ptab[i] <<= pm.ploc;
        for (int i = 0; i < 256; i++) pm.dtab[i] <<= pm.dloc;
    }

    Coder rc(in + k, in_size - size_t(k));
    std::vector<std::pair<uint32_t, uint32_t>> revs;   // reversed records {start, len}
    uint32_t delta = 0, prevq = 0, qctx = 0, p = 0, sel = 0, seqc = 0;
    uint32_t last_len = 0;
    bool first_len = true;
    const Param *pm = &G.p[0];
    uint32_t ctx = 0;
    const uint8_t *sp = nullptr, *se = nullptr;
    uint32_t rec = 0;
    for (uint32_t i = 0; i < total; i++) {
        if (p == 0) {
            // ---- record header (fqzcomp_qual.c:1484-1553) --------------------
            sel = (pm->sel || (G.gflags & GF_MULTI)) ? list_decode(sel_m, rc) : 0u;
            const uint32_t x = (G.gflags & GF_STAB) ? G.stab[std::min(255u, sel)] : sel;
            if (x >= uint32_t(G.nparam)) return -1;
            pm = &G.p[x];
            uint32_t len = last_len;
            if (!pm->fixed || first_len) {
                len = 0;
                for (int b = 0; b < 4; b++) len |= list_decode(len_m[b], rc) << (8 * b);
                first_len = false;
                last_len = len;
            }
            if (len > total - i || len == 0) return -1;
            if (lengths && int(rec) < nlengths) lengths[rec] = int(len);
            if (G.gflags & GF_REV) {
                if (list_decode(rev_m, rc)) revs.emplace_back(i, len);
            }
            if (pm->dedup && list_decode(dup_m, rc)) {   // a copy of the previous record
                if (len > i) return -1;
                std::memmove(out + i, out + i - len, len);
                i += len - 1;
                p = 0;
                rec++;
                continue;
            }
            p = len;
            delta = prevq = qctx = 0;
            seqc = 0;
            sp = se = nullptr;
            if (seq && rec < uint32_t(nrec) && seq[rec]) {   // s->seq[rec] (:1529-1537)
                const uint8_t *r0 = seq[rec];
                sp = r0 + pm->boff;
                se = r0 + len;
                for (uint32_t b = 0; b < pm->boff; b++) seqc = (seqc << 2) | base2(r0[b]);
            }
            rec++;
            ctx = pm->ctx0;
        }
        // ---- one quality symbol in its context's list ------------------------
        const uint32_t q = list_decode(S.q.at(ctx), rc);
        out[i] = uint8_t(pm->qmap[q]);
        // fqz_update_ctx (fqzcomp_qual.c:361-418)
        const uint32_t b = (sp && sp < se) ? base2(*sp++) : 0u;
        qctx = (qctx << pm->qshift) + pm->qtab[q];
        uint32_t c = (qctx & pm->qmask()) << pm->qloc;
        c += pm->ptab[std::min(1023u, p)];
        c += pm->dtab[std::min(255u, delta)];
        seqc = ((seqc << 2) | b) & ((1u << pm->bbits) - 1u);
        c += seqc << pm->bloc;
        c += sel << pm->sloc;
        ctx = c & uint32_t(CTX_SIZE - 1);
        delta += prevq != q;
        prevq = q;
        p--;
    }
    // GFLAG_DO_REV: reversed records back to their order (:1597-1611)
    for (const auto &r : revs) std::reverse(out + r.first, out + r.first + r.second);
    return 0;
}

// decode_seq (fqzcomp5.c:1272-1406): k-mer context model for ACGT runs,
// run lengths per class, literals for the rest, class switches
int seq_decode(const uint8_t *in, uint32_t in_size, const uint32_t *lens, int nrec, int both, int ksz,
               uint8_t *out, uint32_t n) {
    if (ksz < 1 || ksz > 16 || nrec <= 0) return -1;
    const uint32_t msize = 1u << (2 * ksz), mask = msize - 1;
    SeqScratch &S = t_seq;
    if (S.ctx.size() < size_t(msize) * 4) S.ctx.resize(size_t(msize) * 4);
    uint8_t *cm = S.ctx.data();
    std::memset(cm, 1, size_t(msize) * 4);
    // c_small_model.h (STEP 1, halved when the total before the update is
    // at least 255); decode without a bounds check as the reference
    auto small_update = [](uint8_t *F, int nsym, uint32_t tot, int sym) {
        F[sym] = uint8_t(F[sym] + 1);
        if (tot >= 255)
            for (int i = 0; i < nsym; i++) F[i] = uint8_t(F[i] - (F[i] >> 1));
    };
    uint8_t state_m[3][2] = {{1, 1}, {1, 1}, {1, 1}};
    ListStore ls;
    ls.reset(256, 4);
    List run_m[3], lit = ls.at(3);
    for (int s = 0; s < 3; s++) {
        run_m[s] = ls.at(size_t(s));
        list_init(run_m[s], 256, 256);
    }
    list_init(lit, 256, 256);
    Coder rc(in, in_size);
    const uint32_t start1 = 0x007616c7u & mask, start2 = (0x2c6b62ffu >> (32 - 2 * ksz)) & mask;
    uint32_t last = start1, last2 = start2;
    int state = 0;   // 0 upper ACGT, 1 lower acgt, 2 other
    // the reference counts a record down in an int: a length of 0 or past
    // 2^31 never reaches 0 again (no later record start)
    int nseq = 0;
    int64_t left = int32_t(lens[nseq++]);
    auto next_record = [&](uint32_t at) -> bool {   // after out[at]
        if (--left == 0 && at + 1 < n) {
            if (nseq >= nrec) return false;
            left = int32_t(lens[nseq++]);
            last = start1;
            last2 = start2;
        }
        return true;
    };
    // a valid stream has at most one empty run in a row (the first, or one
    // before a class switch): more means a damaged stream that would
    // otherwise switch classes forever without output
    int empty_runs = 0;
    for (uint32_t i = 0; i < n;) {
        uint32_t run = 0, r2;
        do {
            r2 = list_decode(run_m[state], rc);
            run += r2;
        } while (r2 == 255 && run <= n - i);
        if (run > n - i) run = n - i;
        if (run == 0 && ++empty_runs > 2) return -1;
        if (run) empty_runs = 0;
        if (state != 2) {
            const char *bases = state == 1 ? "acgt" : "ACGT";
            for (uint32_t j = 0; j < run; j++) {
                uint8_t *F = cm + size_t(last) * 4;
                const uint32_t tot = uint32_t(F[0]) + F[1] + F[2] + F[3];
                const uint32_t t = rc.target(tot);
                if (t >= tot) return -1;                 // a damaged stream
                uint32_t acc = 0;
                int b = 0;
                while (acc + F[b] <= t) acc += F[b++];   // b < 4: t < tot
                rc.take(acc, F[b]);
                small_update(F, 4, tot, b);
                last = ((last << 2) + uint32_t(b)) & mask;
                out[i + j] = uint8_t(bases[b]);
                if (both) {
                    const int b2 = int(last2 & 3);
                    last2 = last2 / 4 + (uint32_t(3 - b) << (2 * ksz - 2));
                    uint8_t *R = cm + size_t(last2) * 4;
                    small_update(R, 4, uint32_t(R[0]) + R[1] + R[2] + R[3], b2);
                }
                if (!next_record(i + j)) return -1;
            }
        } else {
            for (uint32_t j = 0; j < run; j++) {
                out[i + j] = uint8_t(list_decode(lit, rc));
                if (!next_record(i + j)) return -1;
            }
        }
        i += run;
        if (i >= n) break;
        uint8_t *F = state_m[state];
        const uint32_t tot = uint32_t(F[0]) + F[1];
        const uint32_t t = rc.target(tot);
        const int ns = t >= F[0] ? 1 : 0;
        if (ns && t >= tot) return -1;
        rc.take(ns ? F[0] : 0u, F[ns]);
        small_update(F, 2, tot, ns);
        if (state == 0) state = ns ? 2 : 1;
        else if (state == 1) state = ns ? 2 : 0;
        else state = ns ? 1 : 0;
    }
    return 0;
}

namespace {
// ns per symbol [kind][gpu]: priors from r04 on MI355X boxes (host: this
// file's decoders on one core of the box, the -5 Illumina hybrid step; GPU:
// k_fqz_dec_small 170-190, the general decoder with sequence contexts
// 350-470, k_seq_dec 290-380)
std::atomic<double> g_ns[CK_N][2] = {{{30.0}, {330.0}}, {{16.0}, {180.0}}, {{24.0}, {400.0}}};
}  // namespace

double chain_ns(int kind, bool gpu) { return g_ns[kind][gpu ? 1 : 0].load(std::memory_order_relaxed); }

void chain_measured(int kind, bool gpu, double ns) {
    if (!(ns > 0.0) || kind < 0 || kind >= CK_N) return;
    std::atomic<double> &a = g_ns[kind][gpu ? 1 : 0];
    double cur = a.load(std::memory_order_relaxed);
    // an exponential average: a chain's cost moves with its data
    while (!a.compare_exchange_weak(cur, 0.5 * cur + 0.5 * ns, std::memory_order_relaxed)) {}
}

std::vector<char> plan(const std::vector<uint64_t> &n, const std::vector<int> &kind, int threads) {
    std::vector<char> host(n.size(), 0);
    std::vector<size_t> ord(n.size());
    for (size_t i = 0; i < ord.size(); i++) ord[i] = i;
    std::stable_sort(ord.begin(), ord.end(), [&](size_t a, size_t b) {
        return double(n[a]) * chain_ns(kind[a], false) > double(n[b]) * chain_ns(kind[b], false);
    });
    std::vector<double> core(size_t(std::max(threads, 1)), 0.0);   // each core's finish time
    double gpu_t = 0.0;
    for (size_t i : ord) {
        auto lo = std::min_element(core.begin(), core.end());
        const double th = *lo + double(n[i]) * chain_ns(kind[i], false);
        const double tg = double(n[i]) * chain_ns(kind[i], true);
        double cmax = 0.0;
        for (double c : core) cmax = std::max(cmax, c);
        const double on_host = std::max({cmax, th, gpu_t});
        const double on_gpu = std::max({cmax, gpu_t, tg});
        if (on_host <= on_gpu) {
            *lo = th;
            host[i] = 1;
        } else {
            gpu_t = std::max(gpu_t, tg);
        }
    }
    return host;
}

int cores_of_rank() {
    // the cores this process may run on (its affinity mask, which
    // hardware_concurrency() ignores: a cgroup or taskset share), split
    // evenly among the ranks of this node that share it
    // ($LOCAL_WORLD_SIZE, set by torch.distributed.run), and no more than
    // the per-GPU CPU share the box states ($OMP_NUM_THREADS)
    int n = 0;
    cpu_set_t set;
    CPU_ZERO(&set);
    if (sched_getaffinity(0, sizeof set, &set) == 0) n = CPU_COUNT(&set);
    if (n <= 0) n = int(std::max(1u, std::thread::hardware_concurrency()));
    if (const char *e = std::getenv("LOCAL_WORLD_SIZE")) {
        const int w = std::atoi(e);
        if (w > 1) n /= w;
    }
    if (const char *e = std::getenv("OMP_NUM_THREADS")) {
        const int o = std::atoi(e);
        if (o > 0) n = std::min(n, o);
    }
    return std::max(1, n);
}

int threads() {
    static const int n = [] {
        if (const char *e = std::getenv("FQZ5_HOST_THREADS")) return std::max(1, std::atoi(e));
        return std::min(16, cores_of_rank());
    }();
    return n;
}

}  // namespace host
}  // namespace fqz5

using namespace fqz5;

extern "C" {

char *fqz5_fqz_decompress_host(char *in, size_t in_size, size_t *out_size, int *lengths,
                               int nlengths, fqz_slice *s) {
    if (!in || !out_size) return nullptr;
    uint32_t total = 0;
    if (varint_get(reinterpret_cast<const uint8_t *>(in), reinterpret_cast<const uint8_t *>(in) + in_size,
                   &total) <= 0)
        return nullptr;
    uint8_t *out = static_cast<uint8_t *>(std::malloc(total ? total : 1));
    if (!out) return nullptr;
    const bool sq = s && s->seq && s->num_records > 0;
    if (host::fqz_decode(reinterpret_cast<const uint8_t *>(in), in_size, out, total, out_size, lengths,
                         nlengths, sq ? const_cast<const uint8_t *const *>(s->seq) : nullptr,
                         sq ? s->num_records : 0)) {
        std::free(out);
        return nullptr;
    }
    return reinterpret_cast<char *>(out);
}

char *fqz5_seq_decode_host(unsigned char *in, unsigned int in_size, unsigned int *len, int nrecords,
                           int both_strands, int ctx_size, unsigned int out_size) {
    if ((!in && in_size) || !len || nrecords < 1) return nullptr;
    uint8_t *out = static_cast<uint8_t *>(std::malloc(out_size ? out_size : 1));
    if (!out) return nullptr;
    if (host::seq_decode(in, in_size, len, nrecords, both_strands, ctx_size, out, out_size)) {
        std::free(out);
        return nullptr;
    }
    return reinterpret_cast<char *>(out);
}

}  // extern "C"
