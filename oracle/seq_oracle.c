/* seq_oracle.c — TEST ORACLE ONLY (never linked into the product).
 *
 * Plain-C restatement of fqzcomp5's sequence context model (the SEQ10 ..
 * SEQ14B methods, strat byte (k << 4) | (both << 3) | 1):
 *   encoder                 fqzcomp5.c:1073-1270 (encode_seq)
 *   decoder                 fqzcomp5.c:1272-1406 (decode_seq)
 *   4- and 2-symbol models  htscodecs/c_small_model.h:86-153 (STEP 1,
 *                           halving when the total before the update is
 *                           >= 255), instantiated at fqzcomp5.c:1065-1070
 *   run-length / literal    htscodecs/c_simple_model.h (256 symbols; the
 *                           header's own STEP 16 replaces the caller's
 *                           STEP 8 at fqzcomp5.c:1059-1061)
 *   range coder             htscodecs/c_range_coder.h
 * Pinned against the reference's own encode_seq / decode_seq, compiled from
 * /root/reference into oracle/_ref/libfqz5ref.so (oracle/Makefile), by
 * tests/test_seq_oracle.py and the vectors of tests/golden/make_golden_seq.py.
 */
#include <stdlib.h>

#include "cm_common.h"
#include "oracle.h"

enum { CL_UC = 0, CL_LC = 1, CL_OTHER = 2 };

/* fqzcomp5.c:1107-1118: ACGT -> uppercase run, acgt -> lowercase run,
 * anything else (N, IUPAC codes, ...) -> literal run */
static int base_class(uint8_t c) {
    switch (c) {
    case 'A': case 'C': case 'G': case 'T': return CL_UC;
    case 'a': case 'c': case 'g': case 't': return CL_LC;
    default: return CL_OTHER;
    }
}

static unsigned base_code(uint8_t c) {
    switch (c | 0x20) {
    case 'a': return 0;
    case 'c': return 1;
    case 'g': return 2;
    default: return 3;
    }
}

/* ---- small direct-lookup models (u8 counts) ---------------------------- */
static unsigned sm_total(const uint8_t *f, int ns) {
    unsigned t = 0;
    for (int i = 0; i < ns; i++) t += f[i];
    return t;
}

static void sm_bump(uint8_t *f, int ns, unsigned sym, unsigned tot) {
    f[sym]++;
    if (tot >= 255)
        for (int i = 0; i < ns; i++) f[i] = (uint8_t)(f[i] - (f[i] >> 1));
}

static void sm_put(uint8_t *f, int ns, rcoder *c, unsigned sym) {
    unsigned tot = 0, cum = 0;
    for (int i = 0; i < ns; i++) {
        if ((unsigned)i == sym) cum = tot;
        tot += f[i];
    }
    rc_put(c, cum, f[sym], tot);
    sm_bump(f, ns, sym, tot);
}

static unsigned sm_get(uint8_t *f, int ns, rcoder *c) {
    const unsigned tot = sm_total(f, ns);
    const uint32_t t = rc_target(c, tot);
    unsigned cum = 0, s = 0;
    while (s + 1 < (unsigned)ns && cum + f[s] <= t) cum += f[s++];
    rc_take(c, cum, f[s]);
    sm_bump(f, ns, s, tot);
    return s;
}

/* ---- k-mer contexts ----------------------------------------------------- */
typedef struct {
    int k, both;
    uint32_t mask;
    uint32_t fw, rv;    /* forward k-mer, reverse-complement k-mer */
    uint8_t *m;         /* 4 counts per context */
} kmers;

/* the seeds of fqzcomp5.c:1103-1105: a 12-mer absent from the human genome */
static void kmers_reset(kmers *x) {
    x->fw = 0x007616c7u & x->mask;
    x->rv = (0x2c6b62ffu >> (32 - 2 * x->k)) & x->mask;
}

/* after base b: the forward context shifts it in; in both-strand mode the
 * reverse strand's context takes its complement at the top and its model
 * counts the base that fell out at the bottom, without coding it */
static void kmers_push(kmers *x, unsigned b) {
    x->fw = ((x->fw << 2) + b) & x->mask;
    if (x->both) {
        const unsigned out = x->rv & 3;
        x->rv = (x->rv >> 2) + ((3 - b) << (2 * x->k - 2));
        uint8_t *f = x->m + 4 * (size_t)x->rv;
        sm_bump(f, 4, out, sm_total(f, 4));
    }
}

/* record boundaries: after each symbol the current record's count goes down;
 * reaching zero before the last symbol starts the next record (and resets the
 * contexts).  A record of length 0 makes the count negative, so no later
 * boundary is ever seen — the reference's int countdown, kept as is. */
typedef struct {
    const uint32_t *len;
    int nrec, next;
    long long left;
} recs;

static int recs_after_symbol(recs *r, kmers *x, size_t pos, size_t n) {
    if (--r->left == 0 && pos + 1 < n) {
        if (r->next >= r->nrec) return -1;
        r->left = (int)r->len[r->next++];
        kmers_reset(x);
    }
    return 0;
}

typedef struct {
    flist run[3], lit;
    uint8_t state[3][2];
} side_models;

static void side_init(side_models *s) {
    for (int i = 0; i < 3; i++) {
        fl_init(&s->run[i], 256, 256);
        s->state[i][0] = s->state[i][1] = 1;
    }
    fl_init(&s->lit, 256, 256);
}

/* the stored bit of a state change (fqzcomp5.c:1120-1124, :1243-1261) */
static unsigned switch_bit(int from, int to) {
    if (to == CL_UC) return 0;
    if (to == CL_LC) return from == CL_OTHER;
    return 1;
}

static int switch_to(int from, unsigned bit) {
    if (from == CL_UC) return bit ? CL_OTHER : CL_LC;
    if (from == CL_LC) return bit ? CL_OTHER : CL_UC;
    return bit ? CL_LC : CL_UC;
}

uint8_t *ora_seq_encode(const uint8_t *in, uint32_t n, const uint32_t *len, int nrec,
                        int both, int k, uint32_t *out_size) {
    if (k < 1 || k > 16 || nrec < 1) return NULL;
    uint8_t *out = malloc((size_t)n + (size_t)n / 8 + 1024);
    kmers x = {k, both, (uint32_t)((1ull << (2 * k)) - 1), 0, 0, NULL};
    x.m = malloc(4 * ((size_t)x.mask + 1));
    side_models *sm = malloc(sizeof *sm);
    if (!out || !x.m || !sm) {
        free(out); free(x.m); free(sm);
        return NULL;
    }
    memset(x.m, 1, 4 * ((size_t)x.mask + 1));
    side_init(sm);
    kmers_reset(&x);
    recs r = {len, nrec, 1, (int)len[0]};
    rcoder c;
    rc_enc_start(&c, out);

    int state = CL_UC;
    size_t i = 0;
    int bad = 0;
    while (i < n && !bad) {
        size_t j = i;
        while (j < n && base_class(in[j]) == state) j++;
        /* the run length as 255-digits, last digit < 255 */
        size_t rl = j - i;
        for (;;) {
            fl_encode(&sm->run[state], &c, rl < 255 ? (unsigned)rl : 255u);
            if (rl < 255) break;
            rl -= 255;
        }
        for (size_t p = i; p < j && !bad; p++) {
            if (state == CL_OTHER) {
                fl_encode(&sm->lit, &c, in[p]);
            } else {
                const unsigned b = base_code(in[p]);
                sm_put(x.m + 4 * (size_t)x.fw, 4, &c, b);
                kmers_push(&x, b);
            }
            bad = recs_after_symbol(&r, &x, p, n) < 0;
        }
        i = j;
        if (i >= n || bad) break;
        const int to = base_class(in[i]);
        sm_put(sm->state[state], 2, &c, switch_bit(state, to));
        state = to;
    }
    free(x.m);
    free(sm);
    if (bad) {
        free(out);
        return NULL;
    }
    rc_enc_finish(&c);
    *out_size = (uint32_t)(c.p - out);
    return out;
}

uint8_t *ora_seq_decode(const uint8_t *in, uint32_t in_size, const uint32_t *len, int nrec,
                        int both, int k, uint32_t out_size) {
    if (k < 1 || k > 16 || nrec < 1) return NULL;
    uint8_t *out = malloc(out_size ? out_size : 1);
    kmers x = {k, both, (uint32_t)((1ull << (2 * k)) - 1), 0, 0, NULL};
    x.m = malloc(4 * ((size_t)x.mask + 1));
    side_models *sm = malloc(sizeof *sm);
    if (!out || !x.m || !sm) {
        free(out); free(x.m); free(sm);
        return NULL;
    }
    memset(x.m, 1, 4 * ((size_t)x.mask + 1));
    side_init(sm);
    kmers_reset(&x);
    recs r = {len, nrec, 1, (int)len[0]};
    rcoder c;
    rc_dec_start(&c, (uint8_t *)in, (uint8_t *)in + in_size);

    int state = CL_UC;
    size_t i = 0;
    int bad = 0, idle = 0;
    while (i < out_size && !bad) {
        size_t run = 0;
        unsigned d;
        do {
            d = fl_decode(&sm->run[state], &c, 256);
            run += d;
        } while (d == 255);
        if (i + run > out_size) run = out_size - i;
        /* only the first run can be empty in a valid stream; stop a damaged
         * one instead of switching states forever */
        if (run == 0 && ++idle > 2) {
            bad = 1;
            break;
        }
        const char *abc = state == CL_LC ? "acgt" : "ACGT";
        for (size_t p = i; p < i + run && !bad; p++) {
            if (state == CL_OTHER) {
                out[p] = (uint8_t)fl_decode(&sm->lit, &c, 256);
            } else {
                const unsigned b = sm_get(x.m + 4 * (size_t)x.fw, 4, &c);
                out[p] = (uint8_t)abc[b];
                kmers_push(&x, b);
            }
            bad = recs_after_symbol(&r, &x, p, out_size) < 0;
        }
        i += run;
        if (i >= out_size || bad) break;
        state = switch_to(state, sm_get(sm->state[state], 2, &c));
    }
    free(x.m);
    free(sm);
    if (bad) {
        free(out);
        return NULL;
    }
    return out;
}
