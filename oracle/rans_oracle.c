/*
 * rans_oracle.c — CPU restatement of the htscodecs rANS 4x16 / 32x16
 * "pr" family, written from the reference's behaviour for use as a
 * TEST ORACLE ONLY.  Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg load it (via oracle/binding.py); the product library
 * never links or calls it.
 *
 * Pinned against byte-level golden vectors produced by the compiled
 * reference (tests/golden/rans.json, generator tests/golden/make_golden.py)
 * and, where oracle/_ref exists, against the reference directly.
 *
 * Everything is plain scalar C with one generic code path per concept:
 * the number of interleaved states NX (4 or 32) is a parameter, not an
 * unrolling.  Citations are to /root/reference/htscodecs/.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <limits.h>
#include <math.h>

#include "oracle.h"

/* ---- order-byte flags: rANS_static16_int.h:48-59, rANS_static4x16.h ---- */
#define F_PACK    0x80
#define F_RLE     0x40
#define F_CAT     0x20
#define F_NOSZ    0x10
#define F_STRIPE  0x08
#define F_X32     0x04
#define F_NO0     (1<<16)  /* STRIPE_NO0 */
#define F_AUTO32  (1<<17)  /* SIMD_AUTO, encoder-only hint */

#define RANS_L    (1u<<15) /* rANS_word.h:64 */

/* ---------------------------------------------------------------------- */
/* varint.h:206 / :267 (BIG_END variant): 7-bit groups, most significant   */
/* first, continuation bit 0x80 on all but the last byte.                  */

int ora_var_put_u32(uint8_t *cp, const uint8_t *endp, uint32_t v) {
    int n = 1;
    for (uint32_t t = v >> 7; t; t >>= 7) n++;
    if (endp && (endp - cp) < 5 && (endp - cp) * 7 < n * 7)
        return 0;                       /* varint.h:173 "safe" refusal */
    for (int k = n - 1; k >= 0; k--)
        *cp++ = (uint8_t)(((v >> (7 * k)) & 0x7f) | (k ? 0x80 : 0));
    return n;
}

int ora_var_get_u32(const uint8_t *cp, const uint8_t *endp, uint32_t *v) {
    const uint8_t *op = cp;
    uint32_t j = 0;
    int n = 0;
    if (endp && cp >= endp) { *v = 0; return 0; }
    uint8_t c;
    do {
        c = *cp++;
        j = (j << 7) | (c & 0x7f);
        n++;
    } while ((c & 0x80) && n < 6 && (!endp || cp < endp));
    *v = j;
    return (int)(cp - op);
}

/* ---------------------------------------------------------------------- */
/* Frequency normalisation: rANS_static16_int.h:86-162                    */

static uint32_t round2(uint32_t v) {
    uint32_t r = 1;
    if (v == 0) return 0;
    while (r < v) r <<= 1;
    return r;
}

/* normalise_freq (rANS_static16_int.h:97): scale F (summing to `size`) to
 * sum exactly `tot` using a 31-bit fixed-point ratio; zeros stay zero,
 * non-zeros floor at 1, the residual lands on the largest symbol with one
 * retry and a spread-out fallback. */
static int normalise_freq(uint32_t *F, int size, uint32_t tot) {
    if (!size) return 0;
    for (int pass = 0; ; pass++) {
        uint64_t tr = ((uint64_t)tot << 31) / size + (1 << 30) / size;
        int biggest = 0, bigsym = 0, sum = 0;
        for (int j = 0; j < 256; j++) {
            if (!F[j]) continue;
            if (biggest < (int)F[j]) { biggest = F[j]; bigsym = j; }
            F[j] = (uint32_t)(((uint64_t)F[j] * tr) >> 31);
            if (!F[j]) F[j] = 1;
            sum += F[j];
        }
        int adjust = (int)tot - sum;
        if (adjust > 0) {
            F[bigsym] += adjust;
        } else if (adjust < 0) {
            if ((int)F[bigsym] > -adjust &&
                (pass == 1 || (int)F[bigsym] / 2 >= -adjust)) {
                F[bigsym] += adjust;
            } else if (pass < 1) {
                size = sum;             /* retry from the scaled values */
                continue;
            } else {
                adjust += F[bigsym] - 1;
                F[bigsym] = 1;
                for (int j = 0; adjust && j < 256; j++) {
                    if (F[j] < 2) continue;
                    int d = (int)F[j] > -adjust ? adjust : 1 - (int)F[j];
                    F[j] += d;
                    adjust -= d;
                }
            }
        }
        return F[bigsym] > 0 ? 0 : -1;
    }
}

static void normalise_freq_shift(uint32_t *F, uint32_t size, uint32_t max_tot) {
    if (size == 0 || size == max_tot) return;
    int sh = 0;
    while (size < max_tot) { size *= 2; sh++; }
    for (int i = 0; i < 256; i++) F[i] <<= sh;
}

/* ---------------------------------------------------------------------- */
/* Table serialisation: rANS_static16_int.h:165-306, 425-456              */

/* Symbol list: present symbols ascending; a symbol whose predecessor is
 * present is followed by a count of further consecutive present symbols
 * that are implied; 0 terminates. */
static int encode_alphabet(uint8_t *cp, const uint32_t *F) {
    uint8_t *op = cp;
    int skip = 0;
    for (int j = 0; j < 256; j++) {
        if (!F[j]) continue;
        if (skip) { skip--; continue; }
        *cp++ = (uint8_t)j;
        if (j && F[j - 1]) {
            int k = j + 1;
            while (k < 256 && F[k]) k++;
            skip = k - (j + 1);
            *cp++ = (uint8_t)skip;
        }
    }
    *cp++ = 0;
    return (int)(cp - op);
}

static int decode_alphabet(const uint8_t *cp, const uint8_t *end, uint32_t *F) {
    const uint8_t *op = cp;
    if (cp >= end) return 0;
    int j = *cp++, run = 0;
    do {
        F[j] = 1;
        if (!run && cp < end && j + 1 == *cp) {
            if (cp + 1 >= end) return 0;
            j = *cp++;
            run = *cp++;
        } else if (run) {
            run--;
            if (++j > 255) return 0;
        } else {
            if (cp >= end) return 0;
            j = *cp++;
        }
    } while (j);
    return (int)(cp - op);
}

static int encode_freq0(uint8_t *cp, const uint32_t *F) {
    uint8_t *op = cp;
    cp += encode_alphabet(cp, F);
    for (int j = 0; j < 256; j++)
        if (F[j]) cp += ora_var_put_u32(cp, NULL, F[j]);
    return (int)(cp - op);
}

static int decode_freq0(const uint8_t *cp, const uint8_t *end, uint32_t *F,
                        uint32_t *tot) {
    const uint8_t *op = cp;
    int n = decode_alphabet(cp, end, F);
    if (!n) return 0;
    cp += n;
    uint32_t t = 0;
    for (int j = 0; j < 256; j++) {
        if (!F[j]) continue;
        if (cp >= end) return 0;
        cp += ora_var_get_u32(cp, end, &F[j]);
        t += F[j];
    }
    *tot = t;
    return (int)(cp - op);
}

/* O1 row against the O0 alphabet A: zero entries are run-length coded as a
 * 0 followed by (run-1). */
static int encode_freq_row(uint8_t *cp, const uint32_t *A, const uint32_t *F) {
    uint8_t *op = cp;
    int zeros = 0;
    for (int j = 0; j < 256; j++) {
        if (!A[j]) continue;
        if (F[j]) {
            if (zeros) { *cp++ = 0; *cp++ = (uint8_t)(zeros - 1); zeros = 0; }
            cp += ora_var_put_u32(cp, NULL, F[j]);
        } else {
            zeros++;
        }
    }
    if (zeros) { *cp++ = 0; *cp++ = (uint8_t)(zeros - 1); }
    return (int)(cp - op);
}

static int decode_freq_row(const uint8_t *cp, const uint8_t *end,
                           const uint32_t *A, uint32_t *F, uint32_t *tot) {
    const uint8_t *op = cp;
    int zeros = 0;
    uint32_t t = 0;
    for (int j = 0; j < 256; j++) {
        if (!A[j]) continue;
        uint32_t f;
        if (zeros) {
            f = 0; zeros--;
        } else {
            if (cp >= end) return 0;
            cp += ora_var_get_u32(cp, end, &f);
            if (f == 0) {
                if (cp >= end) return 0;
                zeros = *cp++;
            }
        }
        F[j] = f;
        t += f;
    }
    *tot = t;
    return (int)(cp - op);
}

/* ---------------------------------------------------------------------- */
/* Encoder symbol (rANS_word.h:201-272) and state update (:287-336)       */

typedef struct { uint32_t x_max, rcp, bias, cmpl, shift; } esym_t;

static void esym_init(esym_t *s, uint32_t start, uint32_t freq, int bits) {
    s->x_max = ((RANS_L >> bits) << 16) * freq - 1;
    s->cmpl = (1u << bits) - freq;
    if (freq < 2) {
        s->rcp = ~0u;
        s->shift = 32;
        s->bias = start + (1u << bits) - 1;
    } else {
        uint32_t sh = 0;
        while (freq > (1u << sh)) sh++;
        s->rcp = (uint32_t)(((1ull << (sh + 31)) + freq - 1) / freq);
        s->shift = sh - 1 + 32;
        s->bias = start;
    }
}

/* Encoder output grows downwards from the end of a scratch buffer. */
typedef struct { uint8_t *end, *ptr; } wbuf_t;

static uint32_t esym_put(uint32_t x, wbuf_t *w, const esym_t *s) {
    if (x > s->x_max) {
        w->ptr -= 2;
        w->ptr[0] = (uint8_t)x;
        w->ptr[1] = (uint8_t)(x >> 8);
        x >>= 16;
    }
    uint32_t q = (uint32_t)(((uint64_t)x * s->rcp) >> s->shift);
    return x + s->bias + q * s->cmpl;
}

static void flush_states(const uint32_t *R, int NX, wbuf_t *w) {
    for (int z = NX - 1; z >= 0; z--) {
        w->ptr -= 4;
        for (int b = 0; b < 4; b++) w->ptr[b] = (uint8_t)(R[z] >> (8 * b));
    }
}

/* ---------------------------------------------------------------------- */
/* compress bound: rANS_static4x16pr.c:93-106                             */

unsigned int ora_rans_compress_bound_4x16(unsigned int size, int order) {
    int N = (order >> 8) & 0xff;
    if (!N) N = 4;
    int o = order & 0xff;
    double base = o == 0 ? 1.05 * size + 257 * 3 + 4
                         : 1.05 * size + 257 * 257 * 3 + 4 + 257 * 3 + 4;
    unsigned int sz = (unsigned int)(base
        + ((o & F_PACK) ? 1 : 0)
        + ((o & F_RLE) ? 1 + 257 * 3 + 4 : 0) + 20
        + ((o & F_X32) ? (32 - 4) * 4 : 0)
        + ((o & F_STRIPE) ? 7 + 5 * N : 0));
    return sz + (sz & 1) + 2;
}

/* ---------------------------------------------------------------------- */
/* Order-0 with NX interleaved states                                     */
/* rANS_static4x16pr.c:112-232 (NX=4), rANS_static32x16pr.c:67-254 (NX=32)*/
/* Symbol i belongs to state i % NX; symbols are pushed from i = n-1 down. */

static int enc_o0(const uint8_t *in, uint32_t n, uint8_t *out,
                  uint32_t *out_size, int NX) {
    uint32_t bound = ora_rans_compress_bound_4x16(n, 0) - 20;
    if (bound > *out_size) return -1;
    if (n == 0) { *out_size = 0; return 0; }

    uint32_t F[256] = {0};
    for (uint32_t i = 0; i < n; i++) F[in[i]]++;
    uint32_t max_val = round2(n);
    if (max_val > 4096) max_val = 4096;
    if (normalise_freq(F, n, max_val) < 0) return -1;
    int tab = encode_freq0(out, F);
    if (normalise_freq(F, max_val, 4096) < 0) return -1;

    esym_t S[256];
    memset(S, 0, sizeof(S));
    for (uint32_t j = 0, x = 0; j < 256; j++)
        if (F[j]) { esym_init(&S[j], x, F[j], 12); x += F[j]; }

    uint8_t *scratch = malloc(bound);
    if (!scratch) return -1;
    wbuf_t w = { scratch + bound, scratch + bound };
    uint32_t R[32];
    for (int z = 0; z < NX; z++) R[z] = RANS_L;
    for (uint32_t i = n; i-- > 0; )
        R[i % NX] = esym_put(R[i % NX], &w, &S[in[i]]);
    flush_states(R, NX, &w);
    uint32_t body = (uint32_t)(w.end - w.ptr);
    memcpy(out + tab, w.ptr, body);
    free(scratch);
    *out_size = tab + body;
    return 0;
}

/* O0 decode table: slot -> (sym, freq, slot-start) */
typedef struct { uint8_t sym[4096]; uint16_t f[256], b[256]; } o0tab_t;

static int build_o0tab(const uint32_t *F, int bits, o0tab_t *t) {
    uint32_t x = 0;
    for (int j = 0; j < 256; j++) {
        if (!F[j]) continue;
        if (F[j] > (1u << bits) - x) return -1;
        t->f[j] = (uint16_t)F[j];
        t->b[j] = (uint16_t)x;
        memset(&t->sym[x], j, F[j]);
        x += F[j];
    }
    return x == (1u << bits) ? 0 : -1;
}

/* Word reader used by all decoders: renormalise one state if below L. */
typedef struct { const uint8_t *p, *end; } rbuf_t;

static uint32_t renorm(uint32_t x, rbuf_t *r) {
    if (x < RANS_L && r->p + 1 < r->end) {
        x = (x << 16) | r->p[0] | ((uint32_t)r->p[1] << 8);
        r->p += 2;
    }
    return x;
}

static int read_states(uint32_t *R, int NX, rbuf_t *r) {
    if (r->end - r->p < 4 * NX) return -1;
    for (int z = 0; z < NX; z++) {
        R[z] = r->p[0] | (r->p[1] << 8) | (r->p[2] << 16) |
               ((uint32_t)r->p[3] << 24);
        r->p += 4;
        if (R[z] < RANS_L) return -1;
    }
    return 0;
}

static int dec_o0(const uint8_t *in, uint32_t in_size, uint8_t *out,
                  uint32_t n, int NX) {
    if (in_size < 16) return -1;
    uint32_t F[256] = {0}, tot = 0;
    int hs = decode_freq0(in, in + in_size, F, &tot);
    if (!hs) return -1;
    normalise_freq_shift(F, tot, 4096);
    o0tab_t *t = malloc(sizeof(*t));
    if (!t || build_o0tab(F, 12, t)) { free(t); return -1; }
    rbuf_t r = { in + hs, in + in_size };
    uint32_t R[32];
    if (read_states(R, NX, &r)) { free(t); return -1; }
    for (uint32_t i = 0; i < n; i++) {
        uint32_t *x = &R[i % NX];
        uint32_t m = *x & 4095;
        uint8_t s = t->sym[m];
        out[i] = s;
        *x = t->f[s] * (*x >> 12) + m - t->b[s];
        *x = renorm(*x, &r);
    }
    free(t);
    return 0;
}

/* ---------------------------------------------------------------------- */
/* Order-1: rANS_static4x16pr.c:357-821, rANS_static32x16pr.c:414-758,    */
/* table codec rANS_static16_int.h:312-421.                               */

static double fast_log2ish(double a) {           /* utils.h:69 */
    union { double d; long long x; } u = { a };
    return (u.x - 4606921278410026770LL) * 1.539095918623324e-16;
}

/* rans_compute_shift: 10- vs 12-bit decision plus per-row maxima S[]. */
static int compute_shift(const uint32_t *T, uint32_t (*F)[256], uint32_t *S) {
    double e10 = 0, e12 = 0;
    uint32_t max_tot = 0;
    for (int i = 0; i < 256; i++) {
        if (!T[i]) continue;
        uint32_t mv = round2(T[i]);
        int ns = 0, sm10 = 0, sm12 = 0;
        for (int j = 0; j < 256; j++) {
            if (F[i][j] && mv / F[i][j] > 1024) sm10++;
            if (F[i][j] && mv / F[i][j] > 4096) sm12++;
        }
        double l10 = log(1024 + sm10), l12 = log(4096 + sm12);
        double ts = 4096.0 / T[i], tf = 1024.0 / T[i];
        for (int j = 0; j < 256; j++) {
            if (!F[i][j]) continue;
            ns++;
            double a = F[i][j] * tf, b = F[i][j] * ts;
            e10 -= F[i][j] * (fast_log2ish(a > 1 ? a : 1) - l10);
            e12 -= F[i][j] * (fast_log2ish(b > 1 ? b : 1) - l12);
            e10 += 1.3;
            e12 += 4.7;
        }
        if (ns < 64 && mv > 128) mv /= 2;
        if (mv > 1024) mv /= 2;
        if (mv > 4096) mv = 4096;
        S[i] = mv;
        if (max_tot < mv) max_tot = mv;
    }
    return (e10 / e12 < 1.01 || max_tot <= 1024) ? 10 : 12;
}

/* Builds the O1 tables and serialised header.  hdr must hold ~200 KB.
 * Returns shift (10/12) or -1; *hdr_len set. */
static int o1_tables(const uint8_t *in, uint32_t n, int NX, esym_t (*S)[256],
                     uint8_t *hdr, uint32_t *hdr_len) {
    uint32_t (*F)[256] = calloc(256, sizeof(*F));
    uint32_t T[256] = {0}, Smax[256] = {0};
    if (!F) return -1;
    /* hist1_4 (utils.h:280): context of in[0] is 0; T[last]++ */
    uint8_t prev = 0;
    for (uint32_t i = 0; i < n; i++) { F[prev][in[i]]++; prev = in[i]; }
    T[prev]++;
    for (int i = 0; i < 256; i++)
        for (int j = 0; j < 256; j++) T[i] += F[i][j];
    /* encode_freq1 (rANS_static16_int.h:322-327) */
    uint32_t isz = n / NX;
    for (int z = 1; z < NX; z++) F[0][in[z * isz]]++;
    T[0] += NX - 1;

    uint8_t *cp = hdr;
    *cp++ = 0;
    uint32_t t0 = T[0];
    T[0] = 1;
    cp += encode_alphabet(cp, T);
    T[0] = t0;

    int shift = compute_shift(T, F, Smax);
    for (int i = 0; i < 256; i++) {
        if (!T[i]) continue;
        uint32_t mv = Smax[i];
        if (shift == 10 && mv > 1024) mv = 1024;
        if (normalise_freq(F[i], T[i], mv) < 0) { free(F); return -1; }
        cp += encode_freq_row(cp, T, F[i]);
        normalise_freq_shift(F[i], mv, 1u << shift);
        for (uint32_t j = 0, x = 0; j < 256; j++) {
            esym_init(&S[i][j], x, F[i][j], shift);
            x += F[i][j];
        }
    }
    free(F);
    hdr[0] = (uint8_t)(shift << 4);
    uint32_t raw = (uint32_t)(cp - hdr);
    if (raw > 1000) {
        /* O0-4x16 compress the table (rANS_static16_int.h:397-412) */
        uint32_t u = raw - 1;
        uint32_t cap = ora_rans_compress_bound_4x16(u, 0);
        uint8_t *c = malloc(cap);
        uint32_t clen = cap;
        if (c && enc_o0(hdr + 1, u, c, &clen, 4) == 0 && clen + 6 < raw) {
            uint8_t *op = hdr;
            *op++ |= 1;
            op += ora_var_put_u32(op, NULL, u);
            op += ora_var_put_u32(op, NULL, clen);
            memcpy(op, c, clen);
            cp = op + clen;
        }
        free(c);
    }
    *hdr_len = (uint32_t)(cp - hdr);
    return shift;
}

/* Segment layout shared by encoder and decoder: state z owns
 * [z*isz, (z+1)*isz), the last state also owns the remainder. */
static int enc_o1(const uint8_t *in, uint32_t n, uint8_t *out,
                  uint32_t *out_size, int NX) {
    uint32_t bound = ora_rans_compress_bound_4x16(n, 1) - 20;
    if (NX == 32 && n < 32) return -1;
    if (bound > *out_size) return -1;
    esym_t (*S)[256] = malloc(256 * sizeof(*S));
    uint8_t *hdr = malloc(257 * 257 * 3 + 1024);
    uint8_t *scratch = malloc(bound);
    if (!S || !hdr || !scratch) { free(S); free(hdr); free(scratch); return -1; }
    uint32_t hlen;
    if (o1_tables(in, n, NX, S, hdr, &hlen) < 0) {
        free(S); free(hdr); free(scratch); return -1;
    }
    wbuf_t w = { scratch + bound, scratch + bound };
    uint32_t R[32];
    for (int z = 0; z < NX; z++) R[z] = RANS_L;
    uint32_t isz = n / NX;
    /* remainder of the last state first */
    for (uint32_t p = n; p-- > NX * isz; )
        R[NX - 1] = esym_put(R[NX - 1], &w, &S[in[p - 1]][in[p]]);
    /* then all states in lock-step, highest state first */
    for (uint32_t k = isz; k-- > 0; )
        for (int z = NX - 1; z >= 0; z--) {
            uint32_t p = z * isz + k;
            uint8_t ctx = k ? in[p - 1] : 0;
            R[z] = esym_put(R[z], &w, &S[ctx][in[p]]);
        }
    flush_states(R, NX, &w);
    uint32_t body = (uint32_t)(w.end - w.ptr);
    memcpy(out, hdr, hlen);
    memcpy(out + hlen, w.ptr, body);
    *out_size = hlen + body;
    free(S); free(hdr); free(scratch);
    return 0;
}

static int dec_o1(const uint8_t *in, uint32_t in_size, uint8_t *out,
                  uint32_t n, int NX) {
    if (in_size < (uint32_t)(NX == 4 ? 16 : 4 * NX)) return -1;
    const uint8_t *cp = in, *end = in + in_size, *tab_end = NULL;
    uint8_t *ubuf = NULL;
    int shift = *cp >> 4;
    const uint8_t *hend = end;
    if (*cp++ & 1) {
        uint32_t u, c;
        cp += ora_var_get_u32(cp, end, &u);
        cp += ora_var_get_u32(cp, end, &c);
        if (c > (uint32_t)(end - cp)) return -1;
        tab_end = cp + c;
        ubuf = malloc(u ? u : 1);
        if (!ubuf || dec_o0(cp, c, ubuf, u, 4)) { free(ubuf); return -1; }
        cp = ubuf;
        hend = ubuf + u;
    }
    uint32_t A[256] = {0};
    int k = decode_alphabet(cp, hend, A);
    if (!k) { free(ubuf); return -1; }
    cp += k;
    o0tab_t *tab = calloc(256, sizeof(o0tab_t));
    if (!tab) { free(ubuf); return -1; }
    for (int i = 0; i < 256; i++) {
        if (!A[i]) continue;
        uint32_t F[256] = {0}, T = 0;
        k = decode_freq_row(cp, hend, A, F, &T);
        if (!k) { free(ubuf); free(tab); return -1; }
        cp += k;
        if (!T) continue;
        normalise_freq_shift(F, T, 1u << shift);
        if (build_o0tab(F, shift, &tab[i])) { free(ubuf); free(tab); return -1; }
    }
    if (tab_end) cp = tab_end;
    free(ubuf);

    rbuf_t r = { cp, end };
    uint32_t R[32];
    if (read_states(R, NX, &r)) { free(tab); return -1; }
    uint32_t isz = n / NX, mask = (1u << shift) - 1;
    uint8_t L[32] = {0};
    for (uint32_t kk = 0; kk < isz; kk++)
        for (int z = 0; z < NX; z++) {
            const o0tab_t *t = &tab[L[z]];
            uint32_t m = R[z] & mask;
            uint8_t s = t->sym[m];
            out[z * isz + kk] = s;
            R[z] = t->f[s] * (R[z] >> shift) + m - t->b[s];
            R[z] = renorm(R[z], &r);
            L[z] = s;
        }
    for (uint32_t p = NX * isz; p < n; p++) {
        const o0tab_t *t = &tab[L[NX - 1]];
        uint32_t m = R[NX - 1] & mask;
        uint8_t s = t->sym[m];
        out[p] = s;
        R[NX - 1] = t->f[s] * (R[NX - 1] >> shift) + m - t->b[s];
        R[NX - 1] = renorm(R[NX - 1], &r);
        L[NX - 1] = s;
    }
    free(tab);
    return 0;
}

static int enc_entropy(const uint8_t *in, uint32_t n, uint8_t *out,
                       uint32_t *out_size, int x32, int o1) {
    int NX = x32 ? 32 : 4;
    return o1 ? enc_o1(in, n, out, out_size, NX)
              : enc_o0(in, n, out, out_size, NX);
}

static int dec_entropy(const uint8_t *in, uint32_t in_size, uint8_t *out,
                       uint32_t n, int x32, int o1) {
    int NX = x32 ? 32 : 4;
    return o1 ? dec_o1(in, in_size, out, n, NX)
              : dec_o0(in, in_size, out, n, NX);
}

/* ---------------------------------------------------------------------- */
/* PACK: pack.c:56-147, unpack pack.c:161-344                             */

static uint8_t *pack(const uint8_t *d, uint32_t n, uint8_t *meta,
                     int *meta_len, uint32_t *out_len) {
    int code[256] = {0}, ns = 0;
    for (uint32_t i = 0; i < n; i++) code[d[i]] = 1;
    for (int i = 0; i < 256; i++)
        if (code[i]) { code[i] = ns++; meta[ns] = (uint8_t)i; }
    meta[0] = (uint8_t)ns;
    if (ns > 16) return NULL;
    *meta_len = ns + 1;
    int per = ns > 4 ? 2 : ns > 2 ? 4 : ns > 1 ? 8 : 0;
    uint8_t *o = malloc(n + 1);
    if (!o) return NULL;
    if (per == 0) { *out_len = 0; return o; }
    int bits = 8 / per;
    uint32_t j = 0;
    for (uint32_t i = 0; i < n; i += per) {
        uint8_t b = 0;
        for (int k = 0; k < per && i + k < n; k++)
            b |= (uint8_t)(code[d[i + k]] << (k * bits));
        o[j++] = b;
    }
    *out_len = j;
    return o;
}

static int unpack_meta(const uint8_t *d, uint32_t len, uint8_t *map, int *per) {
    if (!len) return 0;
    unsigned ns = d[0] ? d[0] : 256;
    *per = ns <= 1 ? 0 : ns <= 2 ? 8 : ns <= 4 ? 4 : ns <= 16 ? 2 : 1;
    if (*per == 1) return 1;
    if (len < 1 + ns) return 0;
    memcpy(map, d + 1, ns);
    return 1 + ns;
}

static int unpack(const uint8_t *d, uint32_t len, uint8_t *out, uint32_t n,
                  int per, const uint8_t *map) {
    if (per == 1) { memcpy(out, d, len); return 0; }
    if (per == 0) { memset(out, map[0], n); return 0; }
    int bits = 8 / per;
    if ((n + per - 1) / per > len) return -1;
    for (uint32_t i = 0; i < n; i++)
        out[i] = map[(d[i / per] >> ((i % per) * bits)) & ((1 << bits) - 1)];
    return 0;
}

/* shared with arith_oracle.c */
uint8_t *ora_pack(const uint8_t *d, uint32_t n, uint8_t *meta, int *meta_len, uint32_t *out_len) {
    return pack(d, n, meta, meta_len, out_len);
}
int ora_unpack_meta(const uint8_t *d, uint32_t len, uint8_t *map, int *per) {
    return unpack_meta(d, len, map, per);
}
int ora_unpack(const uint8_t *d, uint32_t len, uint8_t *out, uint32_t n, int per,
               const uint8_t *map) {
    return unpack(d, len, out, n, per, map);
}

/* ---------------------------------------------------------------------- */
/* RLE: rle.c:48-189                                                      */

static uint8_t *rle_encode(const uint8_t *d, uint32_t n, uint8_t *runs,
                           uint64_t *runs_len, uint8_t *syms, int *nsyms,
                           uint64_t *lit_len) {
    int64_t score[256] = {0};
    for (uint32_t i = 0; i < n; i++)
        score[d[i]] += (i && d[i] == d[i - 1]) ? 1 : -1;
    int ns = 0;
    for (int i = 0; i < 256; i++) if (score[i] > 0) syms[ns++] = (uint8_t)i;
    *nsyms = ns;
    uint8_t *lit = malloc(2 * (size_t)n + 1);
    if (!lit) return NULL;
    uint64_t k = 0, j = 0;
    for (uint32_t i = 0; i < n; i++) {
        lit[k++] = d[i];
        if (score[d[i]] > 0) {
            uint32_t s = i;
            while (i + 1 < n && d[i + 1] == d[s]) i++;
            j += ora_var_put_u32(runs + j, NULL, i - s);
        }
    }
    *runs_len = j;
    *lit_len = k;
    return lit;
}

static int rle_decode(const uint8_t *lit, uint64_t lit_len, const uint8_t *run,
                      uint64_t run_len, const uint8_t *syms, int nsyms,
                      uint8_t *out, uint64_t *out_len) {
    int is[256] = {0};
    for (int j = 0; j < nsyms; j++) is[syms[j]] = 1;
    const uint8_t *rend = run + run_len;
    uint64_t o = 0, cap = *out_len;
    for (uint64_t i = 0; i < lit_len; i++) {
        if (o >= cap) return -1;
        uint8_t b = lit[i];
        uint32_t r = 0;
        if (is[b]) run += ora_var_get_u32(run, rend, &r);
        if (o + r >= cap && r) return -1;
        memset(out + o, b, r + 1);
        o += r + 1;
    }
    *out_len = o;
    return 0;
}

/* ---------------------------------------------------------------------- */
/* Dispatcher: rans_compress_to_4x16 (rANS_static4x16pr.c:1224-1600)      */

uint8_t *ora_rans_compress_to_4x16(uint8_t *in, unsigned int in_size,
                                   uint8_t *out, unsigned int *out_size,
                                   int order) {
    if (in_size > INT_MAX || (out && *out_size == 0)) { *out_size = 0; return NULL; }
    uint8_t *owned = NULL;
    if (!out) {
        *out_size = ora_rans_compress_bound_4x16(in_size, order);
        if (!*out_size || !(owned = out = malloc(*out_size))) { *out_size = 0; return NULL; }
    }
    uint8_t *out_end = out + *out_size;

    if ((order & F_AUTO32) && in_size >= 50000 && !(order & F_STRIPE))
        order |= F_X32;
    if (in_size <= 20) order &= ~F_STRIPE;
    if (in_size <= 1000) order &= ~F_X32;

    if (order & F_STRIPE) {
        unsigned N = (order >> 8) & 0xff;
        if (!N) N = 4;
        if (N > in_size) N = in_size;
        uint32_t plen[256], pidx[256];
        for (unsigned i = 0; i < N; i++) {
            plen[i] = in_size / N + ((in_size % N) > i);
            pidx[i] = i ? pidx[i - 1] + plen[i - 1] : 0;
        }
        uint8_t *tr = malloc(in_size);
        if (!tr) { free(owned); *out_size = 0; return NULL; }
        for (uint32_t i = 0; i < in_size; i++)
            tr[pidx[i % N] + i / N] = in[i];        /* byte i -> stripe i%N */
        uint32_t hl = 1;
        out[0] = (uint8_t)(order & ~F_NOSZ);
        hl += ora_var_put_u32(out + hl, out_end, in_size);
        if (hl >= *out_size) { free(tr); free(owned); *out_size = 0; return NULL; }
        out[hl++] = (uint8_t)N;
        uint8_t *dst0 = out + 7 + 5 * N, *dst = dst0;
        uint8_t *best = NULL;
        uint32_t best_cap = 0;
        const int cand[4] = {1, 64, 128, 0};
        for (unsigned s = 0; s < N; s++) {
            uint32_t best_sz = UINT_MAX;
            for (int c = 0; c < 4; c++) {
                int m = cand[c];
                if ((order & m) != m) continue;
                if ((order & F_NO0) && !(m & 1)) continue;
                if (dst - out > (long)*out_size) continue;
                uint32_t olen = *out_size - (uint32_t)(dst - out);
                uint8_t *r = ora_rans_compress_to_4x16(tr + pidx[s], plen[s], dst,
                                                       &olen, m | F_NOSZ | (order & F_X32));
                if (r && olen && best_sz > olen) {
                    best_sz = olen;
                    if (olen > best_cap) {
                        uint8_t *nb = realloc(best, olen);
                        if (!nb) { free(best); free(tr); free(owned); *out_size = 0; return NULL; }
                        best = nb; best_cap = olen;
                    }
                    memcpy(best, dst, olen);
                }
            }
            if (best_sz == UINT_MAX) { free(best); free(tr); free(owned); *out_size = 0; return NULL; }
            memcpy(dst, best, best_sz);
            dst += best_sz;
            hl += ora_var_put_u32(out + hl, out_end, best_sz);
        }
        free(best);
        memmove(out + hl, dst0, dst - dst0);
        free(tr);
        *out_size = hl + (uint32_t)(dst - dst0);
        return out;
    }

    if (order & F_CAT) {
        out[0] = F_CAT;
        uint32_t hl = 1 + ora_var_put_u32(out + 1, out_end, in_size);
        if (hl + in_size > *out_size) { free(owned); *out_size = 0; return NULL; }
        if (in_size) memcpy(out + hl, in, in_size);
        *out_size = hl + in_size;
        return out;
    }

    int do_pack = order & F_PACK, do_rle = order & F_RLE;
    int no_size = order & F_NOSZ, x32 = order & F_X32;
    uint8_t *packed = NULL, *lits = NULL;
    out[0] = (uint8_t)order;
    uint32_t hl = 1;
    if (!no_size) hl += ora_var_put_u32(out + 1, out_end, in_size);
    int o1 = order & 1;  /* order &= 3 in the reference; only bit 0 is used */

    if (do_pack && in_size) {
        int ml;
        uint32_t plen;
        if (hl + 256 > *out_size) { free(owned); *out_size = 0; return NULL; }
        packed = pack(in, in_size, out + hl, &ml, &plen);
        if (!packed) {
            out[0] &= ~F_PACK;
            do_pack = 0;
        } else {
            in = packed;
            in_size = plen;
            hl += ml;
            int vs = ora_var_put_u32(out + hl, out_end, in_size);
            hl += vs;
            *out_size -= vs;   /* reference quirk (rANS_static4x16pr.c:1453) */
            if (x32 && in_size < 32) { x32 = 0; out[0] &= ~F_X32; }
        }
    } else if (do_pack) {
        out[0] &= ~F_PACK;
    }

    if (do_rle && in_size) {
        uint8_t *meta = malloc((size_t)in_size + 257);
        uint8_t syms[256];
        int nsyms = 0;
        uint64_t rmeta64, llen;
        if (!meta) { free(packed); free(owned); *out_size = 0; return NULL; }
        lits = rle_encode(in, in_size, meta + 257, &rmeta64, syms, &nsyms, &llen);
        /* meta = [nsyms][syms...][run varints] */
        memmove(meta + 1 + nsyms, meta + 257, rmeta64);
        meta[0] = (uint8_t)nsyms;
        memcpy(meta + 1, syms, nsyms);
        uint32_t rmeta = (uint32_t)(rmeta64 + nsyms + 1);
        if (!lits || llen + rmeta >= .99 * in_size) {
            out[0] &= ~F_RLE;
            do_rle = 0;
            free(lits);
            lits = NULL;
        } else {
            int sz = ora_var_put_u32(out + hl, out_end, rmeta * 2);
            sz += ora_var_put_u32(out + hl + sz, out_end, (uint32_t)llen);
            if (hl + sz + 5 > *out_size) {
                free(meta); free(lits); free(packed); free(owned); *out_size = 0; return NULL;
            }
            uint32_t cm = *out_size - (hl + sz + 5);
            if (x32 && (rmeta < 32 || llen < 32)) { x32 = 0; out[0] &= ~F_X32; }
            if (enc_entropy(meta, rmeta, out + hl + sz + 5, &cm, x32, 0)) {
                free(meta); free(lits); free(packed); free(owned); *out_size = 0; return NULL;
            }
            int sz2;
            if (cm < rmeta) {
                sz2 = ora_var_put_u32(out + hl + sz, out_end, cm);
                memmove(out + hl + sz + sz2, out + hl + sz + 5, cm);
            } else {
                sz = ora_var_put_u32(out + hl, out_end, rmeta * 2 + 1);
                sz2 = ora_var_put_u32(out + hl + sz, out_end, (uint32_t)llen);
                memcpy(out + hl + sz + sz2, meta, rmeta);
                cm = rmeta;
            }
            hl += sz + sz2 + cm;
            in = lits;
            in_size = (uint32_t)llen;
        }
        free(meta);
    } else if (do_rle) {
        out[0] &= ~F_RLE;
    }

    if (hl > *out_size) { free(lits); free(packed); free(owned); *out_size = 0; return NULL; }
    *out_size -= hl;
    if (o1 && in_size < 8) { out[0] &= ~1; o1 = 0; }
    if (enc_entropy(in, in_size, out + hl, out_size, x32, o1)) {
        free(lits); free(packed); free(owned); *out_size = 0; return NULL;
    }
    if (*out_size >= in_size) {
        out[0] &= ~3;
        out[0] |= F_CAT | no_size;
        if (out + hl + in_size > out_end) {
            free(lits); free(packed); free(owned); *out_size = 0; return NULL;
        }
        if (in_size) memcpy(out + hl, in, in_size);
        *out_size = in_size;
    }
    free(lits);
    free(packed);
    *out_size += hl;
    return out;
}

uint8_t *ora_rans_compress_4x16(uint8_t *in, unsigned int in_size,
                                unsigned int *out_size, int order) {
    return ora_rans_compress_to_4x16(in, in_size, NULL, out_size, order);
}

/* rans_uncompress_to_4x16 (rANS_static4x16pr.c:1607-1894) for valid and
 * moderately malformed streams. */
uint8_t *ora_rans_uncompress_to_4x16(uint8_t *in, unsigned int in_size,
                                     uint8_t *out, unsigned int *out_size) {
    const uint8_t *end = in + in_size;
    if (!in_size) return NULL;
    uint8_t *owned = NULL;

    if (*in & F_STRIPE) {
        uint32_t ulen, hl = 1;
        hl += ora_var_get_u32(in + hl, end, &ulen);
        if (hl >= in_size) return NULL;
        unsigned N = in[hl++];
        if (N < 1) return NULL;
        if (!out) {
            if (ulen >= INT_MAX || !(owned = out = malloc(ulen ? ulen : 1))) return NULL;
            *out_size = ulen;
        }
        if (ulen != *out_size) { free(owned); return NULL; }
        uint32_t clen[256], plen[256], pidx[256];
        uint64_t ctot = 0;
        for (unsigned i = 0; i < N; i++) {
            plen[i] = ulen / N + ((ulen % N) > i);
            pidx[i] = i ? pidx[i - 1] + plen[i - 1] : 0;
            hl += ora_var_get_u32(in + hl, end, &clen[i]);
            ctot += clen[i];
            if (hl > in_size || clen[i] > in_size || clen[i] < 1) { free(owned); return NULL; }
        }
        if (hl + ctot > in_size) { free(owned); return NULL; }
        uint8_t *tmp = malloc(ulen ? ulen : 1);
        if (!tmp) { free(owned); return NULL; }
        for (unsigned i = 0; i < N; i++) {
            uint32_t ol = plen[i];
            if (!ora_rans_uncompress_to_4x16(in + hl, (uint32_t)(hl + ctot) - hl,
                                             tmp + pidx[i], &ol) || ol != plen[i]) {
                free(tmp); free(owned); return NULL;
            }
            hl += clen[i];
            ctot -= clen[i];
        }
        for (uint32_t i = 0; i < ulen; i++)
            out[i] = tmp[pidx[i % N] + i / N];
        free(tmp);
        *out_size = ulen;
        return out;
    }

    int order = *in++;
    in_size--;
    int do_pack = order & F_PACK, do_rle = order & F_RLE, do_cat = order & F_CAT;
    int no_size = order & F_NOSZ, x32 = order & F_X32, o1 = order & 1;
    uint32_t osz;
    if (!no_size) {
        int k = ora_var_get_u32(in, end, &osz);
        in += k; in_size -= k;
    } else {
        if (!out) return NULL;
        osz = *out_size;
    }
    if (!out) {
        *out_size = osz;
        if (!(owned = out = malloc(osz ? osz : 1))) return NULL;
    } else {
        if (*out_size < osz) return NULL;
        *out_size = osz;
    }

    uint8_t map[256];
    int per = 1;
    uint32_t ent_len = osz;          /* size the entropy stage decodes to */
    if (do_pack) {
        int k = unpack_meta(in, in_size, map, &per);
        if (!k) goto err;
        in += k; in_size -= k;
        uint32_t pl;
        k = ora_var_get_u32(in, end, &pl);
        in += k; in_size -= k;
        if (pl > osz) goto err;
        ent_len = pl;
    }
    uint8_t *meta = NULL, *meta_owned = NULL;
    uint32_t meta_len = 0;
    if (do_rle) {
        uint32_t um, lit_len, cm;
        int k = ora_var_get_u32(in, end, &um);
        k += ora_var_get_u32(in + k, end, &lit_len);
        if (lit_len > ent_len) goto err;
        if (um & 1) {
            meta = in + k;
            meta_len = um / 2;
            if (meta_len > (uint32_t)(end - meta)) meta_len = (uint32_t)(end - meta);
            cm = meta_len;
        } else {
            k += ora_var_get_u32(in + k, end, &cm);
            meta_len = um / 2;
            meta_owned = meta = malloc(meta_len ? meta_len : 1);
            if (!meta || dec_entropy(in + k, in_size - k, meta, meta_len, x32, 0)) {
                free(meta_owned); goto err;
            }
        }
        if (cm + k > in_size) { free(meta_owned); goto err; }
        in += cm + k;
        in_size -= cm + k;
        ent_len = lit_len;
    }

    uint8_t *ent = malloc(ent_len ? ent_len : 1);
    if (!ent) { free(meta_owned); goto err; }
    if (in_size) {
        if (do_cat) {
            if (ent_len > in_size) { free(ent); free(meta_owned); goto err; }
            memcpy(ent, in, ent_len);
        } else if (dec_entropy(in, in_size, ent, ent_len, x32, o1)) {
            free(ent); free(meta_owned); goto err;
        }
    } else {
        ent_len = 0;
    }

    uint8_t *stage = ent;
    uint32_t stage_len = ent_len;
    if (do_rle) {
        if (!meta_len) { free(ent); free(meta_owned); goto err; }
        int nsyms = meta[0] ? meta[0] : 256;
        if (meta_len < (uint32_t)(1 + nsyms)) { free(ent); free(meta_owned); goto err; }
        uint64_t ul = osz;
        uint8_t *un = malloc(osz ? osz : 1);
        if (!un || rle_decode(ent, ent_len, meta + 1 + nsyms, meta_len - 1 - nsyms,
                              meta + 1, nsyms, un, &ul)) {
            free(un); free(ent); free(meta_owned); goto err;
        }
        free(ent);
        stage = un;
        stage_len = (uint32_t)ul;
    }
    free(meta_owned);
    if (do_pack) {
        /* unpacked size is the stored size, except for the raw 'pack' of
         * >16 symbols (rANS_static4x16pr.c:1874) */
        uint32_t ul = per == 1 ? stage_len : osz;
        if (unpack(stage, stage_len, out, ul, per, map)) { free(stage); goto err; }
        stage_len = ul;
        free(stage);
    } else {
        memcpy(out, stage, stage_len);
        free(stage);
    }
    *out_size = stage_len;
    return out;

err:
    free(owned);
    return NULL;
}

uint8_t *ora_rans_uncompress_4x16(uint8_t *in, unsigned int in_size,
                                  unsigned int *out_size) {
    return ora_rans_uncompress_to_4x16(in, in_size, NULL, out_size);
}
