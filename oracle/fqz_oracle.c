/* fqz_oracle.c — TEST ORACLE ONLY (never linked into the product).
 *
 * Plain-C restatement of htscodecs' fqzcomp_qual codec as vendored by the
 * reference (fork ABI, fqzcomp_qual.h:59-64,155-170):
 *   adaptive frequency lists   c_simple_model.h:63-171
 *   carry-less range coder     c_range_coder.h:20-164
 *   array RLE store/read       fqzcomp_qual.c:111-199
 *   strategy table             fqzcomp_qual.c:204-218
 *   context update             fqzcomp_qual.c:361-418
 *   statistics + auto-tune     fqzcomp_qual.c:424-704
 *   parameter store/read       fqzcomp_qual.c:707-769, :1256-1407
 *   parameter pick             fqzcomp_qual.c:774-1001
 *   encoder / decoder          fqzcomp_qual.c:1008-1247, :1410-1634
 * Used by tests/ as the bit-exact checker of the GPU path and pinned by
 * vectors from the compiled reference (tests/golden/make_golden_fqz.py).
 */
#include <limits.h>
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "oracle.h"

#include "cm_common.h"

/* ------------------------------------------------------------------ */
/* parameters                                                          */
/* ------------------------------------------------------------------ */
enum { GF_MULTI = 1, GF_STAB = 2, GF_REV = 4, GF_SEQ = 8 };
enum { PF_DEDUP = 2, PF_LEN = 4, PF_SEL = 8, PF_QMAP = 16, PF_PTAB = 32,
       PF_DTAB = 64, PF_QTAB = 128 };
#define F_READ2 128u
#define F_REVERSE 16u
#define NCTX 65536
#define QSYMS 96

typedef struct {
    unsigned ctx0, pflags;
    int sel, dedup, qmap_stored, fixed;
    int qtab_on, dtab_on, ptab_on;
    unsigned qbits, qloc, pbits, ploc, dbits, dloc, sloc;
    unsigned bbits, bloc, boff;
    int max_sym, nsym, max_sel;
    unsigned qmap[256], qtab[256], ptab[1024], dtab[256];
    int qshift, pshift, dshift;
    unsigned qmask;
    int r2, qa;
} fparam;

typedef struct {
    int vers;
    unsigned gflags;
    int nparam, max_sel, max_sym;
    unsigned stab[256];
    fparam *p;
} fglobal;

/* strategy rows: qbits qshift pbits pshift dbits dshift qloc sloc ploc dloc
 * r2 qa bbits bloc boff (fqzcomp_qual.c:204-218) */
static const int STRATS[6][15] = {
    {10, 5, 4, -1, 2, 1, 0, 14, 10, 14, 0, -1, 0, 0, 0},
    {8, 5, 7, 0, 0, 0, 0, 14, 8, 14, 1, -1, 0, 0, 0},
    {12, 6, 0, 0, 0, 0, 0, 12, 0, 0, 0, 0, 0, 0, 0},
    {6, 6, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 10, 6, 3},
    {8, 5, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 8, 8, 2},
    {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0},
};
#define NSTRATS 6

/* Two-level RLE of a monotone table: first the run length of each value
 * 0,1,2,... (255-continued), then byte runs of equal run lengths (a
 * repeated byte is followed by its extra repeat count). */
static int tab_store(uint8_t *out, const unsigned *t, int n) {
    uint8_t runs[2048];
    int nr = 0, i = 0;
    for (unsigned v = 0; i < n; v++) {
        int start = i;
        while (i < n && t[i] == v) i++;
        int r = i - start;
        for (;;) {
            int part = r < 255 ? r : 255;
            runs[nr++] = (uint8_t)part;
            r -= part;
            if (part != 255) break;
        }
    }
    int o = 0, prev = -1;
    for (int k = 0; k < nr;) {
        uint8_t b = runs[k++];
        out[o++] = b;
        if (b == prev) {
            int k0 = k;
            while (k < nr && runs[k] == prev) k++;
            out[o++] = (uint8_t)(k - k0);
        } else {
            prev = b;
        }
    }
    return o;
}

static int tab_read(const uint8_t *in, size_t avail, unsigned *t, int n) {
    uint8_t runs[1024];
    int nr = 0, covered = 0, prev = -1;
    size_t k = 0;
    if (n > 1024) n = 1024;
    for (; covered < n && k < avail; k++) {
        int b = in[k];
        runs[nr++] = (uint8_t)b;
        covered += b;
        if (b == prev) {
            if (k + 1 >= avail) return -1;
            int more = in[++k];
            covered += b * more;
            while (more-- && covered <= n && nr < 1024) runs[nr++] = (uint8_t)b;
        }
        if (nr >= 1024) return -1;
        prev = b;
    }
    int used = (int)k;
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

/* ------------------------------------------------------------------ */
/* statistics and auto-tuning (fqzcomp_qual.c:424-704)                  */
/* ------------------------------------------------------------------ */
#define NPOS 128

static void qual_stats(int nrec, uint32_t *lens, uint32_t *flags, const uint8_t *q,
                       size_t n, fparam *pm, uint32_t qhist[256]) {
    static uint32_t hb[NPOS][256], h1[NPOS][256], h2[NPOS][256];
    uint64_t c1[NPOS] = {0}, c2[NPOS] = {0};
    static uint32_t amap[2560];
    memset(hb, 0, sizeof hb);
    memset(h1, 0, sizeof h1);
    memset(h2, 0, sizeof h2);
    memset(amap, 0, sizeof amap);

    int max_sel = 0, has_r2 = 0;
    for (int r = 0; r < nrec; r++) {
        if (max_sel < (int)(flags[r] >> 16)) max_sel = (int)(flags[r] >> 16);
        if (flags[r] & F_READ2) has_r2 = 1;
    }
    int *ravg = calloc((size_t)nrec + 1, sizeof(int));
    if (!ravg) return;

    size_t i = 0;
    int r = 0, dups = 0;
    size_t prev_len = 0;
    while (i < n) {
        size_t len;
        int second;
        if (r < nrec) {
            len = lens[r];
            second = (flags[r] & F_READ2) != 0;
            if (i > 0 && len == prev_len && !memcmp(q + i - prev_len, q + i, len)) dups++;
        } else {
            len = n - i;
            second = 0;
        }
        prev_len = len;
        uint32_t(*hh)[256] = second ? h2 : h1;
        uint64_t *cc = second ? c2 : c1;
        uint32_t sum = 0;
        for (size_t j = len; i < n && j > 0; i++, j--) {
            sum += q[i];
            qhist[q[i]]++;
            hb[j & (NPOS - 1)][q[i]]++;
            hh[j & (NPOS - 1)][q[i]]++;
            cc[j & (NPOS - 1)]++;
        }
        /* average in tenths, rounded (fqzcomp_qual.c:495) */
        sum = prev_len ? (uint32_t)((sum * 10.0) / prev_len + .5) : 0;
        ravg[r] = (int)sum;
        amap[sum < 2559 ? sum : 2559]++;
        r++;
    }
    pm->dedup = ((r + 1) / (dups + 1) < 500);

    pm->max_sym = pm->nsym = 0;
    for (int s = 0; s < 256; s++)
        if (qhist[s]) pm->max_sym = s, pm->nsym++;

    if (pm->qa != 0) {
        /* rank the per-record averages into 4 classes */
        double f0 = pm->nsym > 8 ? 0.2 : 0.05;
        double f1 = pm->nsym > 8 ? 0.5 : 0.22;
        double f2 = pm->nsym > 8 ? 0.8 : 0.60;
        int cum = 0, k = 0;
        const double cut[3] = {f0, f1, f2};
        for (int cls = 0; cls < 3; cls++) {
            while (k < 2560) {
                cum += (int)amap[k];
                if (cum > cut[cls] * nrec) break;
                amap[k++] = (uint32_t)cls;
            }
        }
        while (k < 2560) amap[k++] = 3;

        static int b4[4][NPOS][256], b2[2][NPOS][256], b1[NPOS][256];
        int n4[4][NPOS] = {{0}}, n2[4][NPOS] = {{0}}, n1[NPOS] = {0};
        memset(b4, 0, sizeof b4);
        memset(b2, 0, sizeof b2);
        memset(b1, 0, sizeof b1);
        i = 0;
        r = 0;
        while (i < n) {
            size_t len = r < nrec ? lens[r] : n - i;
            int c4 = (int)amap[ravg[r] < 2559 ? ravg[r] : 2559], c2x = c4 / 2;
            for (size_t j = len; i < n && j > 0; i++, j--) {
                int x = (int)(j & (NPOS - 1));
                b4[c4][x][q[i]]++, n4[c4][x]++;
                b2[c2x][x][q[i]]++, n2[c2x][x]++;
                b1[x][q[i]]++, n1[x]++;
            }
            r++;
        }
        double e1 = 0, e2 = 0, e4 = 0;
        for (int x = 0; x < NPOS; x++) {
            for (int s = 0; s < 256; s++) {
                if (b1[x][s]) e1 += b1[x][s] * log(b1[x][s] / (double)n1[x]);
                if (b2[0][x][s]) e2 += b2[0][x][s] * log(b2[0][x][s] / (double)n2[0][x]);
                if (b2[1][x][s]) e2 += b2[1][x][s] * log(b2[1][x][s] / (double)n2[1][x]);
                if (b4[0][x][s]) e4 += b4[0][x][s] * log(b4[0][x][s] / (double)n4[0][x]);
                if (b4[1][x][s]) e4 += b4[1][x][s] * log(b4[1][x][s] / (double)n4[1][x]);
                if (b4[2][x][s]) e4 += b4[2][x][s] * log(b4[2][x][s] / (double)n4[2][x]);
                if (b4[3][x][s]) e4 += b4[3][x][s] * log(b4[3][x][s] / (double)n4[3][x]);
            }
        }
        e1 /= -log(2) / 8;
        e2 /= -log(2) / 8;
        e4 /= -log(2) / 8;
        double m = pm->qa > 0 ? 1 : 0.98;
        if ((pm->qa == -1 || pm->qa >= 4) && e4 + nrec / 4 < e2 * m + nrec / 8 &&
            e4 + nrec / 4 < e1 * m) {
            for (int k2 = 0; k2 < nrec; k2++)
                flags[k2] |= amap[ravg[k2] < 2559 ? ravg[k2] : 2559] << 16;
            pm->sel = 1;
            max_sel = 3;
        } else if ((pm->qa == -1 || pm->qa >= 2) && e2 + nrec / 8 < e1 * m) {
            for (int k2 = 0; k2 < nrec; k2++)
                flags[k2] |= (amap[ravg[k2] < 2559 ? ravg[k2] : 2559] >> 1) << 16;
            pm->sel = 1;
            max_sel = 1;
        }
        if (pm->qa == -1) {
            /* make room for the selector bits in the context */
            if (pm->pbits > 0 && pm->dbits > 0) {
                pm->sloc = pm->dloc - 1;
                pm->pbits--;
                pm->dbits--;
                pm->dloc++;
            } else if (pm->dbits >= 2) {
                pm->sloc = pm->dloc;
                pm->dbits -= 2;
                pm->dloc += 2;
            } else if (pm->qbits >= 2) {
                pm->qbits -= 2;
                pm->ploc -= 2;
                pm->sloc = 16 - 2 - pm->r2;
                if (pm->qbits == 6 && pm->qshift == 5) pm->qbits--;
            }
            pm->qa = 4;
        }
    }

    if (has_r2 || pm->r2) {
        double e1 = 0, e2 = 0;
        for (int x = 0; x < NPOS; x++) {
            if (!c1[x] || !c2[x]) continue;
            for (int s = 0; s < 256; s++) {
                if (!hb[x][s]) continue;
                e1 -= hb[x][s] * log(hb[x][s] / (double)(c1[x] + c2[x]));
                if (h1[x][s]) e2 -= h1[x][s] * log(h1[x][s] / (double)c1[x]);
                if (h2[x][s]) e2 -= h2[x][s] * log(h2[x][s] / (double)c2[x]);
            }
        }
        e1 /= log(2) * 8;
        e2 /= log(2) * 8;
        double m = pm->r2 > 0 ? 1 : 0.95;
        if (e2 + (8 + nrec / 8) < e1 * m) {
            for (int k2 = 0; k2 < nrec; k2++) {
                unsigned sel = flags[k2] >> 16;
                flags[k2] = (flags[k2] & 0xffff) |
                            ((sel * 2 + ((flags[k2] & F_READ2) ? 1 : 0)) << 16);
                if (max_sel < (int)(flags[k2] >> 16)) max_sel = (int)(flags[k2] >> 16);
            }
        }
    }
    if (max_sel > 0) {
        pm->sel = 1;
        pm->max_sel = max_sel;
    }
    free(ravg);
}

static int put_param(const fglobal *g, const fparam *pm, uint8_t *o) {
    int k = 0;
    o[k++] = (uint8_t)pm->ctx0;
    o[k++] = (uint8_t)(pm->ctx0 >> 8);
    o[k++] = (uint8_t)pm->pflags;
    o[k++] = (uint8_t)pm->max_sym;
    o[k++] = (uint8_t)((pm->qbits << 4) | pm->qshift);
    o[k++] = (uint8_t)((pm->qloc << 4) | pm->sloc);
    o[k++] = (uint8_t)((pm->ploc << 4) | pm->dloc);
    if (g->gflags & GF_SEQ) {
        o[k++] = (uint8_t)((pm->bbits << 4) | pm->bloc);
        o[k++] = (uint8_t)(pm->boff << 4);
    }
    if (pm->qmap_stored)
        for (int s = 0; s < 256; s++)
            if (pm->qmap[s] != INT_MAX) o[k++] = (uint8_t)s;
    if (pm->qbits && pm->qtab_on) k += tab_store(o + k, pm->qtab, 256);
    if (pm->pbits && pm->ptab_on) k += tab_store(o + k, pm->ptab, 1024);
    if (pm->dbits && pm->dtab_on) k += tab_store(o + k, pm->dtab, 256);
    return k;
}

static int put_params(const fglobal *g, uint8_t *o) {
    int k = 0;
    o[k++] = (uint8_t)g->vers;
    o[k++] = (uint8_t)g->gflags;
    if (g->gflags & GF_MULTI) o[k++] = (uint8_t)g->nparam;
    if (g->gflags & GF_STAB) {
        o[k++] = (uint8_t)g->max_sel;
        k += tab_store(o + k, g->stab, 256);
    }
    for (int i = 0; i < g->nparam; i++) k += put_param(g, &g->p[i], o + k);
    return k;
}

static int pick_params(fglobal *g, int vers, int strat, int nrec, uint32_t *lens,
                       uint32_t *flags, const uint8_t *q, size_t n) {
    int dsq[64] = {0, 1, 1, 1, 2, 2, 2, 2, 2, 3, 3, 3, 3, 3, 3, 3,
                   4, 4, 4, 4, 4, 4, 4, 4, 4, 5, 5, 5, 5, 5, 5, 5,
                   5, 5, 5, 5, 6, 6, 6, 6, 6, 6, 6, 6, 6, 6, 6, 6,
                   6, 7, 7, 7, 7, 7, 7, 7, 7, 7, 7, 7, 7, 7, 7, 7};
    uint32_t qhist[256] = {0};
    if (strat >= NSTRATS) strat = NSTRATS - 1;
    memset(g, 0, sizeof *g);
    g->vers = 5;
    if (!(g->p = calloc(1, sizeof(fparam)))) return -1;
    g->nparam = 1;
    fparam *pm = g->p;
    const int *so = STRATS[strat];
    pm->qbits = (unsigned)so[0];
    pm->qshift = so[1];
    pm->pbits = (unsigned)so[2];
    pm->pshift = so[3];
    pm->dbits = (unsigned)so[4];
    pm->dshift = so[5];
    pm->qloc = (unsigned)so[6];
    pm->sloc = (unsigned)so[7];
    pm->ploc = (unsigned)so[8];
    pm->dloc = (unsigned)so[9];
    pm->bbits = (unsigned)so[12];
    pm->bloc = (unsigned)so[13];
    pm->boff = (unsigned)so[14];
    if (vers == 3 && pm->bbits == 0) g->gflags |= GF_REV;
    pm->r2 = so[10];
    pm->qa = so[11];

    /* fit the record lengths to the buffer (fqzcomp_qual.c:827-837) */
    size_t tl = 0;
    for (int r = 0; r < nrec; r++) {
        if (tl + lens[r] > n) lens[r] = (uint32_t)(n - tl);
        tl += lens[r];
    }
    if (nrec > 0 && tl < n) lens[nrec - 1] += (uint32_t)(n - tl);

    qual_stats(nrec, lens, flags, q, n, pm, qhist);
    pm->qmap_stored = (pm->nsym <= 8 && pm->nsym * 2 < pm->max_sym);
    int r = 1;
    while (r < nrec && lens[r] == lens[0]) r++;
    pm->fixed = (r == nrec);
    pm->qtab_on = 0;

    if (strat < NSTRATS - 1) {
        if (pm->pshift < 0) {
            double v = log((double)lens[0] / (1 << pm->pbits)) / log(2) + .5;
            pm->pshift = v > 0 ? (int)v : 0;
        }
        if (pm->nsym <= 4) {
            pm->qshift = 2;
            if (n < 5000000) pm->pbits = 2, pm->pshift = 5;
        } else if (pm->nsym <= 8) {
            pm->qbits = pm->qbits < 9 ? pm->qbits : 9;
            pm->qshift = 3;
            if (n < 5000000) pm->qbits = 6;
        }
        if (n < 300000) {
            pm->qbits = (unsigned)pm->qshift;
            pm->dbits = 2;
        }
    }
    for (int k = 0; k < 64; k++)
        if (dsq[k] > (1 << pm->dbits) - 1) dsq[k] = (1 << pm->dbits) - 1;
    if (pm->qmap_stored) {
        int j = 0;
        for (int s = 0; s < 256; s++) pm->qmap[s] = qhist[s] ? (unsigned)j++ : INT_MAX;
        pm->max_sym = pm->nsym;
    } else {
        pm->nsym = 255;
        for (int s = 0; s < 256; s++) pm->qmap[s] = (unsigned)s;
    }
    if (g->max_sym < pm->max_sym) g->max_sym = pm->max_sym;
    if (pm->qbits)
        for (int s = 0; s < 256; s++) pm->qtab[s] = (unsigned)s;
    if (qhist['~' - '!'] * 2 > n && strat == 3) {     /* HiFi */
        pm->qtab_on = 1;
        int v = 0;
        for (int s = 0; s < 256; s++) {
            if (s == '~' - '!' || s == '~' - '!' + 1 || s % 16 == 0) v++;
            pm->qtab[s] = (unsigned)v;
        }
        pm->qbits = 9, pm->qshift = 3;
        pm->bbits = 6, pm->bloc = 9, pm->boff = 2;
    }
    pm->qmask = (1u << pm->qbits) - 1;
    if (pm->pbits)
        for (int k = 0; k < 1024; k++) {
            unsigned v = (unsigned)(k >> pm->pshift), cap = (1u << pm->pbits) - 1;
            pm->ptab[k] = v < cap ? v : cap;
        }
    if (pm->dbits)
        for (int k = 0; k < 256; k++) {
            int idx = k >> pm->dshift;
            pm->dtab[k] = (unsigned)dsq[idx < 63 ? idx : 63];
        }
    pm->ptab_on = pm->pbits > 0;
    pm->dtab_on = pm->dbits > 0;
    pm->pflags = (pm->qtab_on ? PF_QTAB : 0) | (pm->dtab_on ? PF_DTAB : 0) |
                 (pm->ptab_on ? PF_PTAB : 0) | (pm->sel ? PF_SEL : 0) |
                 (pm->fixed ? PF_LEN : 0) | (pm->dedup ? PF_DEDUP : 0) |
                 (pm->qmap_stored ? PF_QMAP : 0);
    g->max_sel = 0;
    if (pm->sel) {
        g->gflags |= GF_STAB;
        int mx = 0;
        for (int k = 0; k < nrec; k++)
            if (mx < (int)(flags[k] >> 16)) mx = (int)(flags[k] >> 16);
        g->max_sel = mx;
    }
    return 0;
}

/* ------------------------------------------------------------------ */
/* per-record context (fqzcomp_qual.c:361-418)                          */
/* ------------------------------------------------------------------ */
typedef struct {
    unsigned qctx, left, delta, prevq, sel, seq;
} fctx;

static unsigned next_ctx(const fparam *pm, fctx *st, unsigned q, unsigned base) {
    st->qctx = (st->qctx << pm->qshift) + pm->qtab[q];
    unsigned c = (st->qctx & pm->qmask) << pm->qloc;
    c += pm->ptab[st->left < 1023 ? st->left : 1023];
    c += pm->dtab[st->delta < 255 ? st->delta : 255];
    st->seq = ((st->seq << 2) | base) & ((1u << pm->bbits) - 1);
    c += st->seq << pm->bloc;
    c += st->sel << pm->sloc;
    st->delta += (st->prevq != q);
    st->prevq = q;
    st->left--;
    return c & (NCTX - 1);
}

static unsigned base2(uint8_t c) {
    switch (c) {
    case 'C': case 'c': return 1;
    case 'G': case 'g': return 2;
    case 'T': case 't': case 'U': case 'u': return 3;
    default: return 0;
    }
}

typedef struct {
    flist *qual;
    flist len[4], rev, sel, dup;
} fmodels;

static int models_new(fmodels *m, const fglobal *g) {
    if (!(m->qual = malloc(sizeof(flist) * NCTX))) return -1;
    for (int c = 0; c < NCTX; c++) fl_init(&m->qual[c], QSYMS, g->max_sym + 1);
    for (int k = 0; k < 4; k++) fl_init(&m->len[k], 256, 256);
    fl_init(&m->rev, 2, 2);
    fl_init(&m->dup, 2, 2);
    if (g->max_sel > 0) fl_init(&m->sel, 256, g->max_sel + 1);
    else memset(&m->sel, 0, sizeof m->sel);
    return 0;
}

static void flip_records(uint8_t *q, size_t n, int nrec, const uint32_t *lens,
                         const uint32_t *flags) {
    size_t i = 0;
    for (int r = 0; i < n; r++) {
        size_t len = r < nrec - 1 ? lens[r] : n - i;
        if (flags[r] & F_REVERSE)
            for (size_t a = 0, b = len - 1; len && a < b; a++, b--) {
                uint8_t t = q[i + a];
                q[i + a] = q[i + b];
                q[i + b] = t;
            }
        i += len;
    }
}

uint8_t *ora_fqz_compress(int vers, ora_fqz_slice *s, uint8_t *q, size_t n,
                          size_t *out_size, int strat, void *gp_unused) {
    (void)gp_unused;
    size_t cap = (size_t)(n * 1.1 + 100000);
    uint8_t *out = malloc(cap);
    if (!out) return NULL;
    fglobal g;
    if (pick_params(&g, vers, strat, s->num_records, s->len, s->flags, q, n) < 0) {
        free(out);
        return NULL;
    }
    if (!s->seq || !s->seq[0]) {
        for (int k = 0; k < g.nparam; k++) g.p[k].bbits = g.p[k].bloc = 0;
        g.gflags &= ~(unsigned)GF_SEQ;
    } else {
        for (int k = 0; k < g.nparam; k++)
            if (g.p[k].bbits) g.gflags |= GF_SEQ;
    }
    int hdr = ora_var_put_u32(out, out + cap, (uint32_t)n);
    hdr += put_params(&g, out + hdr);
    for (int k = 0; k < g.nparam; k++) {
        for (int i = 0; i < 1024; i++) g.p[k].ptab[i] <<= g.p[k].ploc;
        for (int i = 0; i < 256; i++) g.p[k].dtab[i] <<= g.p[k].dloc;
    }
    fmodels m;
    if (models_new(&m, &g) < 0) {
        free(g.p);
        free(out);
        return NULL;
    }
    rcoder rc;
    rc_enc_start(&rc, out + hdr);
    if (g.gflags & GF_REV) flip_records(q, n, s->num_records, s->len, s->flags);

    fparam *pm = &g.p[0];
    fctx st;
    memset(&st, 0, sizeof st);
    int first_len = 1, rec = 0;
    size_t prev_len = 0;
    unsigned ctx = 0;
    const uint8_t *sp = NULL, *se = NULL;
    for (size_t i = 0; i < n; i++) {
        if (st.left == 0) {
            if (pm->sel || (g.gflags & GF_MULTI)) {
                st.sel = rec < s->num_records ? s->flags[rec] >> 16 : 0;
                fl_encode(&m.sel, &rc, st.sel);
            } else {
                st.sel = 0;
            }
            pm = &g.p[(g.gflags & GF_STAB) ? g.stab[st.sel] : st.sel];
            unsigned len = s->len[rec];
            if (!pm->fixed || first_len) {
                for (int b = 0; b < 4; b++) fl_encode(&m.len[b], &rc, (len >> (8 * b)) & 0xff);
                first_len = 0;
            }
            if (g.gflags & GF_REV)
                fl_encode(&m.rev, &rc, (s->flags[rec] & F_REVERSE) ? 1 : 0);
            st.left = len;
            st.delta = st.qctx = st.prevq = 0;
            if (s->seq && s->seq[rec]) {
                sp = s->seq[rec] + pm->boff;
                se = s->seq[rec] + len;
                st.seq = 0;
                for (unsigned b = 0; b < pm->boff; b++)
                    st.seq = (st.seq << 2) | base2(s->seq[rec][b]);
            } else {
                sp = se = NULL;
                st.seq = 0;
            }
            rec++;
            ctx = pm->ctx0;
            if (pm->dedup) {
                if (i && len == prev_len && !memcmp(q + i - prev_len, q + i, len)) {
                    fl_encode(&m.dup, &rc, 1);
                    i += len - 1;
                    st.left = 0;
                    continue;
                }
                fl_encode(&m.dup, &rc, 0);
                prev_len = len;
            }
        }
        unsigned sym = pm->qmap[q[i]];
        unsigned base = sp && sp < se ? base2(*sp++) : 0;
        fl_encode(&m.qual[ctx], &rc, sym);
        ctx = next_ctx(pm, &st, sym, base);
    }
    rc_enc_finish(&rc);
    if (g.gflags & GF_REV) flip_records(q, n, s->num_records, s->len, s->flags);
    for (int r = 0; r < s->num_records; r++) s->flags[r] &= 0xffff;
    *out_size = (size_t)hdr + (size_t)(rc.p - rc.start);
    free(m.qual);
    free(g.p);
    return out;
}

static int get_param(const fglobal *g, fparam *pm, const uint8_t *in, size_t avail) {
    size_t k = 0;
    memset(pm, 0, sizeof *pm);
    if (avail < 7) return -1;
    pm->ctx0 = in[0] | (in[1] << 8);
    k = 2;
    pm->pflags = in[k++];
    pm->qtab_on = pm->pflags & PF_QTAB;
    pm->dtab_on = pm->pflags & PF_DTAB;
    pm->ptab_on = pm->pflags & PF_PTAB;
    pm->sel = pm->pflags & PF_SEL;
    pm->fixed = pm->pflags & PF_LEN;
    pm->dedup = pm->pflags & PF_DEDUP;
    pm->qmap_stored = pm->pflags & PF_QMAP;
    pm->max_sym = in[k++];
    pm->qbits = in[k] >> 4;
    pm->qmask = (1u << pm->qbits) - 1;
    pm->qshift = in[k++] & 15;
    pm->qloc = in[k] >> 4;
    pm->sloc = in[k++] & 15;
    pm->ploc = in[k] >> 4;
    pm->dloc = in[k++] & 15;
    if (g->gflags & GF_SEQ) {
        pm->bbits = in[k] >> 4;
        pm->bloc = in[k++] & 15;
        pm->boff = in[k++] >> 4;
    }
    if (pm->qmap_stored) {
        for (int s = 0; s < 256; s++) pm->qmap[s] = INT_MAX;
        if (k + (size_t)pm->max_sym > avail) return -1;
        for (int s = 0; s < pm->max_sym; s++) pm->qmap[s] = in[k++];
    } else {
        for (int s = 0; s < 256; s++) pm->qmap[s] = (unsigned)s;
    }
    if (pm->qbits) {
        if (pm->qtab_on) {
            int u = tab_read(in + k, avail - k, pm->qtab, 256);
            if (u < 0) return -1;
            k += (size_t)u;
        } else {
            for (int s = 0; s < 256; s++) pm->qtab[s] = (unsigned)s;
        }
    }
    if (pm->ptab_on) {
        int u = tab_read(in + k, avail - k, pm->ptab, 1024);
        if (u < 0) return -1;
        k += (size_t)u;
    }
    if (pm->dtab_on) {
        int u = tab_read(in + k, avail - k, pm->dtab, 256);
        if (u < 0) return -1;
        k += (size_t)u;
    }
    return (int)k;
}

static int get_params(fglobal *g, const uint8_t *in, size_t avail) {
    size_t k = 0;
    if (avail < 10) return -1;
    g->vers = in[k++];
    if (g->vers != 5) return -1;
    g->gflags = in[k++];
    g->nparam = (g->gflags & GF_MULTI) ? in[k++] : 1;
    if (g->nparam <= 0) return -1;
    g->max_sel = g->nparam > 1 ? g->nparam : 0;
    if (g->gflags & GF_STAB) {
        g->max_sel = in[k++];
        int u = tab_read(in + k, avail - k, g->stab, 256);
        if (u < 0) return -1;
        k += (size_t)u;
    } else {
        for (int i = 0; i < 256; i++) g->stab[i] = (unsigned)(i < g->nparam ? i : g->nparam - 1);
    }
    if (!(g->p = malloc(sizeof(fparam) * (size_t)g->nparam))) return -1;
    g->max_sym = 0;
    for (int i = 0; i < g->nparam; i++) {
        int u = get_param(g, &g->p[i], in + k, avail - k);
        if (u < 0 || (g->p[i].sel && g->max_sel == 0)) {
            free(g->p);
            g->p = NULL;
            return -1;
        }
        k += (size_t)u;
        if (g->max_sym < g->p[i].max_sym) g->max_sym = g->p[i].max_sym;
    }
    return (int)k;
}

uint8_t *ora_fqz_decompress(uint8_t *in, size_t in_size, size_t *out_size, int *lengths,
                            int nlengths, ora_fqz_slice *s) {
    uint32_t total;
    size_t k = (size_t)ora_var_get_u32(in, in + in_size, &total);
    *out_size = total;
    fglobal g;
    memset(&g, 0, sizeof g);
    int u = get_params(&g, in + k, in_size - k);
    if (u < 0) return NULL;
    k += (size_t)u;
    for (int p = 0; p < g.nparam; p++) {
        for (int i = 0; i < 1024; i++) g.p[p].ptab[i] <<= g.p[p].ploc;
        for (int i = 0; i < 256; i++) g.p[p].dtab[i] <<= g.p[p].dloc;
    }
    fmodels m;
    if (models_new(&m, &g) < 0) {
        free(g.p);
        return NULL;
    }
    rcoder rc;
    rc_dec_start(&rc, in + k, in + in_size);
    uint8_t *out = malloc(total ? total : 1);
    int cap_rec = 1000;
    uint8_t *revs = malloc((size_t)cap_rec);
    unsigned *lens = malloc(sizeof(unsigned) * (size_t)cap_rec);
    if (!out || !revs || !lens) goto fail;

    fctx st;
    memset(&st, 0, sizeof st);
    int first_len = 1, rec = 0, rev = 0;
    unsigned prev_len = 0, ctx = 0;
    fparam *pm = &g.p[0];
    const uint8_t *sp = NULL, *se = NULL;
    for (size_t i = 0; i < total; i++) {
        if (rec >= cap_rec) {
            cap_rec *= 2;
            uint8_t *r2 = realloc(revs, (size_t)cap_rec);
            unsigned *l2 = realloc(lens, sizeof(unsigned) * (size_t)cap_rec);
            if (!r2 || !l2) { free(r2 ? r2 : revs); free(l2 ? l2 : lens); revs = NULL; lens = NULL; goto fail; }
            revs = r2;
            lens = l2;
        }
        if (st.left == 0) {
            if (pm->sel || (g.gflags & GF_MULTI))
                st.sel = fl_decode(&m.sel, &rc, 256);
            else
                st.sel = 0;
            unsigned x = (g.gflags & GF_STAB) ? g.stab[st.sel < 255 ? st.sel : 255] : st.sel;
            if ((int)x >= g.nparam) goto fail;
            pm = &g.p[x];
            unsigned len = prev_len;
            if (!pm->fixed || first_len) {
                len = 0;
                for (int b = 0; b < 4; b++) len |= fl_decode(&m.len[b], &rc, 256) << (8 * b);
                first_len = 0;
                prev_len = len;
            }
            if (len > total - i || len == 0) goto fail;
            if (lengths && rec < nlengths) lengths[rec] = (int)len;
            if (g.gflags & GF_REV) {
                rev = (int)fl_decode(&m.rev, &rc, 2);
                revs[rec] = (uint8_t)rev;
                lens[rec] = len;
            }
            if (pm->dedup && fl_decode(&m.dup, &rc, 2)) {
                if (len > i) goto fail;
                memcpy(out + i, out + i - len, len);
                i += len - 1;
                st.left = 0;
                rec++;
                continue;
            }
            st.left = len;
            st.delta = st.prevq = st.qctx = 0;
            if (s && s->seq && s->seq[rec]) {
                sp = s->seq[rec] + pm->boff;
                se = s->seq[rec] + len;
                st.seq = 0;
                for (unsigned b = 0; b < pm->boff; b++)
                    st.seq = (st.seq << 2) | base2(s->seq[rec][b]);
            } else {
                sp = se = NULL;
                st.seq = 0;
            }
            rec++;
            ctx = pm->ctx0;
        }
        unsigned sym = fl_decode(&m.qual[ctx], &rc, QSYMS);
        out[i] = (uint8_t)pm->qmap[sym];
        unsigned base = sp && sp < se ? base2(*sp++) : 0;
        ctx = next_ctx(pm, &st, sym, base);
    }
    if (g.gflags & GF_REV) {
        /* records recorded by the decoder; the last covers the remainder */
        size_t i = 0;
        for (int r = 0; i < total && r < rec; i += lens[r++]) {
            if (!revs[r]) continue;
            for (size_t a = 0, b = lens[r] - 1; a < b; a++, b--) {
                uint8_t t = out[i + a];
                out[i + a] = out[i + b];
                out[i + b] = t;
            }
        }
    }
    free(revs);
    free(lens);
    free(m.qual);
    free(g.p);
    return out;
fail:
    free(revs);
    free(lens);
    free(out);
    free(m.qual);
    free(g.p);
    return NULL;
}
