// fqz_format.hpp — fqzcomp_qual parameters (host side): the strategy table,
// the auto-tuning decisions made from GPU-gathered statistics, and the
// parameter block serialisation.  Byte-exact with htscodecs fqzcomp_qual.c
// (fork ABI, fqzcomp_qual.h:59-139); each function cites what it restates.
#pragma once
#include <climits>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <vector>

namespace fqz5 {

namespace fqz {

enum : unsigned { GF_MULTI = 1, GF_STAB = 2, GF_REV = 4, GF_SEQ = 8 };
enum : unsigned { PF_DEDUP = 2, PF_LEN = 4, PF_SEL = 8, PF_QMAP = 16, PF_PTAB = 32,
                  PF_DTAB = 64, PF_QTAB = 128 };
constexpr uint32_t F_READ2 = 128, F_REVERSE = 16;   // fqzcomp_qual.h:37-38
constexpr int NPOS = 128;                            // fqzcomp_qual.c:429
constexpr int NAVG = 2560;
constexpr int CTX_SIZE = 65536;
constexpr int QSYMS = 96;                            // QMAX, fqzcomp_qual.c:84

struct Param {
    unsigned ctx0 = 0, pflags = 0;
    bool sel = false, dedup = false, qmap_stored = false, fixed = false;
    bool qtab_on = false, dtab_on = false, ptab_on = false;
    unsigned qbits = 0, qloc = 0, pbits = 0, ploc = 0, dbits = 0, dloc = 0, sloc = 0;
    unsigned bbits = 0, bloc = 0, boff = 0;
    int max_sym = 0, nsym = 0, max_sel = 0;
    int qshift = 0, pshift = 0, dshift = 0;
    int r2 = 0, qa = 0;
    unsigned qmap[256] = {0}, qtab[256] = {0}, ptab[1024] = {0}, dtab[256] = {0};
    unsigned qmask() const { return (1u << qbits) - 1; }
};

struct Global {
    int vers = 5;
    unsigned gflags = 0;
    int nparam = 1, max_sel = 0, max_sym = 0;
    unsigned stab[256] = {0};
    std::vector<Param> p;
};

// Statistics of one block gathered on the GPU (fqz_qual_stats,
// fqzcomp_qual.c:424-512): histograms by (remaining length & 127) for
// READ1 / READ2 records, per-record average quality in tenths, and the
// duplicate-record count.
struct Stats {
    std::vector<uint32_t> h1, h2;       // [NPOS][256]
    std::vector<uint32_t> avg_hist;     // [NAVG]
    std::vector<uint32_t> rec_avg;      // per record (nrec + 1)
    uint32_t dups = 0;
    uint32_t nrec_seen = 0;             // records walked (incl. a tail)
};

// strat_opts (fqzcomp_qual.c:204-218): qbits qshift pbits pshift dbits
// dshift qloc sloc ploc dloc r2 qa bbits bloc boff
inline const int (&strat_row(int s))[15] {
    static const int T[6][15] = {
        {10, 5, 4, -1, 2, 1, 0, 14, 10, 14, 0, -1, 0, 0, 0},
        {8, 5, 7, 0, 0, 0, 0, 14, 8, 14, 1, -1, 0, 0, 0},
        {12, 6, 0, 0, 0, 0, 0, 12, 0, 0, 0, 0, 0, 0, 0},
        {6, 6, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 10, 6, 3},
        {8, 5, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 8, 8, 2},
        {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0},
    };
    return T[s];
}
constexpr int NSTRATS = 6;

// store_array (fqzcomp_qual.c:111-153): run lengths of the values 0,1,..
// (255-continued), then a second RLE over repeated run-length bytes.
inline int put_table(uint8_t *out, const unsigned *t, int n) {
    std::vector<uint8_t> runs;
    int i = 0;
    for (unsigned v = 0; i < n; v++) {
        int b = i;
        while (i < n && t[i] == v) i++;
        int r = i - b;
        do {
            const int part = r < 255 ? r : 255;
            runs.push_back(uint8_t(part));
            r -= part;
            if (part < 255) break;
        } while (true);
    }
    int o = 0, prev = -1;
    for (size_t k = 0; k < runs.size();) {
        const uint8_t b = runs[k++];
        out[o++] = b;
        if (b == prev) {
            const size_t k0 = k;
            while (k < runs.size() && runs[k] == b) k++;
            out[o++] = uint8_t(k - k0);
        } else {
            prev = b;
        }
    }
    return o;
}

// read_array (fqzcomp_qual.c:155-199); -1 on malformed input
inline int get_table(const uint8_t *in, size_t avail, unsigned *t, int n) {
    uint8_t runs[1024];
    int nr = 0, covered = 0, prev = -1;
    size_t k = 0;
    if (n > 1024) n = 1024;
    for (; covered < n && k < avail; k++) {
        const int b = in[k];
        runs[nr++] = uint8_t(b);
        covered += b;
        if (b == prev) {
            if (k + 1 >= avail) return -1;
            int more = in[++k];
            covered += b * more;
            while (more-- && covered <= n && nr < 1024) runs[nr++] = uint8_t(b);
        }
        if (nr >= 1024) return -1;
        prev = b;
    }
    const int used = int(k);
    int r = 0, o = 0;
    for (unsigned v = 0; o < n; v++) {
        int len = 0, part;
        if (r >= nr) return -1;
        do {
            part = runs[r++];
            len += part;
        } while (part == 255 && r < nr);
        if (part == 255) return -1;
        while (len && o < n) len--, t[o++] = v;
    }
    return used;
}

// fqz_store_parameters1 / fqz_store_parameters (fqzcomp_qual.c:707-769)
inline int put_params(const Global &g, uint8_t *o) {
    int k = 0;
    o[k++] = uint8_t(g.vers);
    o[k++] = uint8_t(g.gflags);
    if (g.gflags & GF_MULTI) o[k++] = uint8_t(g.nparam);
    if (g.gflags & GF_STAB) {
        o[k++] = uint8_t(g.max_sel);
        k += put_table(o + k, g.stab, 256);
    }
    for (const Param &pm : g.p) {
        o[k++] = uint8_t(pm.ctx0);
        o[k++] = uint8_t(pm.ctx0 >> 8);
        o[k++] = uint8_t(pm.pflags);
        o[k++] = uint8_t(pm.max_sym);
        o[k++] = uint8_t((pm.qbits << 4) | unsigned(pm.qshift));
        o[k++] = uint8_t((pm.qloc << 4) | pm.sloc);
        o[k++] = uint8_t((pm.ploc << 4) | pm.dloc);
        if (g.gflags & GF_SEQ) {
            o[k++] = uint8_t((pm.bbits << 4) | pm.bloc);
            o[k++] = uint8_t(pm.boff << 4);
        }
        if (pm.qmap_stored)
            for (int s = 0; s < 256; s++)
                if (pm.qmap[s] != unsigned(INT_MAX)) o[k++] = uint8_t(s);
        if (pm.qbits && pm.qtab_on) k += put_table(o + k, pm.qtab, 256);
        if (pm.pbits && pm.ptab_on) k += put_table(o + k, pm.ptab, 1024);
        if (pm.dbits && pm.dtab_on) k += put_table(o + k, pm.dtab, 256);
    }
    return k;
}

// fqz_read_parameters1 / fqz_read_parameters (fqzcomp_qual.c:1256-1407)
inline int get_params(Global &g, const uint8_t *in, size_t avail) {
    size_t k = 0;
    if (avail < 10) return -1;
    g.vers = in[k++];
    if (g.vers != 5) return -1;
    g.gflags = in[k++];
    g.nparam = (g.gflags & GF_MULTI) ? in[k++] : 1;
    if (g.nparam <= 0) return -1;
    g.max_sel = g.nparam > 1 ? g.nparam : 0;
    if (g.gflags & GF_STAB) {
        g.max_sel = in[k++];
        const int u = get_table(in + k, avail - k, g.stab, 256);
        if (u < 0) return -1;
        k += size_t(u);
    } else {
        for (int i = 0; i < 256; i++) g.stab[i] = unsigned(i < g.nparam ? i : g.nparam - 1);
    }
    g.p.assign(size_t(g.nparam), Param());
    g.max_sym = 0;
    for (Param &pm : g.p) {
        const size_t a = avail - k;
        const uint8_t *q = in + k;
        size_t j = 0;
        if (a < 7) return -1;
        pm.ctx0 = q[0] | (q[1] << 8);
        j = 2;
        pm.pflags = q[j++];
        pm.qtab_on = pm.pflags & PF_QTAB;
        pm.dtab_on = pm.pflags & PF_DTAB;
        pm.ptab_on = pm.pflags & PF_PTAB;
        pm.sel = pm.pflags & PF_SEL;
        pm.fixed = pm.pflags & PF_LEN;
        pm.dedup = pm.pflags & PF_DEDUP;
        pm.qmap_stored = pm.pflags & PF_QMAP;
        pm.max_sym = q[j++];
        pm.qbits = q[j] >> 4;
        pm.qshift = q[j++] & 15;
        pm.qloc = q[j] >> 4;
        pm.sloc = q[j++] & 15;
        pm.ploc = q[j] >> 4;
        pm.dloc = q[j++] & 15;
        if (g.gflags & GF_SEQ) {
            pm.bbits = q[j] >> 4;
            pm.bloc = q[j++] & 15;
            pm.boff = q[j++] >> 4;
        }
        if (pm.qmap_stored) {
            for (int s = 0; s < 256; s++) pm.qmap[s] = unsigned(INT_MAX);
            if (j + size_t(pm.max_sym) > a) return -1;
            for (int s = 0; s < pm.max_sym; s++) pm.qmap[s] = q[j++];
        } else {
            for (int s = 0; s < 256; s++) pm.qmap[s] = unsigned(s);
        }
        if (pm.qbits) {
            if (pm.qtab_on) {
                const int u = get_table(q + j, a - j, pm.qtab, 256);
                if (u < 0) return -1;
                j += size_t(u);
            } else {
                for (int s = 0; s < 256; s++) pm.qtab[s] = unsigned(s);
            }
        }
        if (pm.ptab_on) {
            const int u = get_table(q + j, a - j, pm.ptab, 1024);
            if (u < 0) return -1;
            j += size_t(u);
        }
        if (pm.dtab_on) {
            const int u = get_table(q + j, a - j, pm.dtab, 256);
            if (u < 0) return -1;
            j += size_t(u);
        }
        if (pm.sel && g.max_sel == 0) return -1;
        k += j;
        if (g.max_sym < pm.max_sym) g.max_sym = pm.max_sym;
    }
    return int(k);
}

// Everything of fqz_pick_parameters (fqzcomp_qual.c:774-1001) that precedes
// fqz_qual_stats: the strategy row and the length fix-up of the slice.
inline void pick_begin(Global &g, int vers, int strat, int nrec, uint32_t *lens, size_t n) {
    if (strat >= NSTRATS) strat = NSTRATS - 1;
    g = Global();
    g.p.assign(1, Param());
    Param &pm = g.p[0];
    const int *so = strat_row(strat);
    pm.qbits = unsigned(so[0]);
    pm.qshift = so[1];
    pm.pbits = unsigned(so[2]);
    pm.pshift = so[3];
    pm.dbits = unsigned(so[4]);
    pm.dshift = so[5];
    pm.qloc = unsigned(so[6]);
    pm.sloc = unsigned(so[7]);
    pm.ploc = unsigned(so[8]);
    pm.dloc = unsigned(so[9]);
    pm.r2 = so[10];
    pm.qa = so[11];
    pm.bbits = unsigned(so[12]);
    pm.bloc = unsigned(so[13]);
    pm.boff = unsigned(so[14]);
    if (vers == 3 && pm.bbits == 0) g.gflags |= GF_REV;
    size_t tl = 0;
    for (int r = 0; r < nrec; r++) {
        if (tl + lens[r] > n) lens[r] = uint32_t(n - tl);
        tl += lens[r];
    }
    if (nrec > 0 && tl < n) lens[nrec - 1] += uint32_t(n - tl);
}

}  // namespace fqz
}  // namespace fqz5
