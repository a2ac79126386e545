/* arith_oracle.c — TEST ORACLE ONLY.  Plain-C restatement of htscodecs
 * arith_dynamic.c (the CRAM 3.1 adaptive arithmetic codec) for checking the
 * GPU build; never linked into the product.
 *
 *   models   c_simple_model.h:63-171 (STEP 16, MAX_FREQ 65519, one bubble
 *            step, halve until the first zero, sentinel before slot 0)
 *   coder    c_range_coder.h:51-164 (carry-less, output-end check, decode
 *            end-of-input error)
 *   O0 / O1  arith_dynamic.c:97-270; RLE variants :436-728 (258 run models,
 *            MAX_RUN 4)
 *   to/from  arith_compress_to :730-1025, arith_uncompress_to :1032-1277,
 *            arith_compress_bound :77-87.  EXT (bzip2) is compiled out in the
 *            reference build (HAVE_LIBBZ2 undefined): NULL.
 */
#include <limits.h>
#include <stdlib.h>
#include <string.h>

#include "oracle.h"

#define AX_PACK 0x80
#define AX_RLE 0x40
#define AX_CAT 0x20
#define AX_NOSZ 0x10
#define AX_STRIPE 0x08
#define AX_EXT 0x04

#define AMAX 65519u
#define ASTEP 16u
#define MAX_RUN 4

/* list: slot 0 sentinel (MAX), 1..cap symbols, cap+1 zero, cap+2 MAX */
typedef struct {
    uint32_t total;
    int cap;
    uint16_t fr[262];
    uint16_t sy[262];
} alist;

static void al_init(alist *m, int cap, int live) {
    m->cap = cap;
    m->fr[0] = AMAX;
    m->sy[0] = 0;
    for (int k = 0; k < cap; k++) {
        m->sy[k + 1] = (uint16_t)k;
        m->fr[k + 1] = k < live ? 1 : 0;
    }
    m->fr[cap + 1] = 0;
    m->sy[cap + 1] = 0;
    m->fr[cap + 2] = AMAX;
    m->sy[cap + 2] = 0;
    m->total = (uint32_t)live;
}

static void al_bump(alist *m, int k) {
    m->fr[k] += ASTEP;
    m->total += ASTEP;
    if (m->total > AMAX) {
        uint32_t t = 0;
        for (int i = 1; m->fr[i]; i++) {
            m->fr[i] = (uint16_t)(m->fr[i] - (m->fr[i] >> 1));
            t += m->fr[i];
        }
        m->total = t;
    }
    if (m->fr[k] > m->fr[k - 1]) {
        uint16_t f = m->fr[k], s = m->sy[k];
        m->fr[k] = m->fr[k - 1];
        m->sy[k] = m->sy[k - 1];
        m->fr[k - 1] = f;
        m->sy[k - 1] = s;
    }
}

typedef struct {
    uint32_t low, rng, code, ffnum, cache, carry;
    uint8_t *p, *start, *end;
    const uint8_t *ip, *iend;
    int err;
} arc;

static void enc_start(arc *c, uint8_t *out, uint8_t *end) {
    memset(c, 0, sizeof *c);
    c->rng = 0xFFFFFFFFu;
    c->p = c->start = out;
    c->end = end;
}

static void shift_low(arc *c) {
    if (c->low < 0xFF000000u || c->carry) {
        if (c->end && c->ffnum >= (uint32_t)(c->end - c->p)) {
            c->err = -1;
            return;
        }
        *c->p++ = (uint8_t)(c->cache + c->carry);
        for (; c->ffnum; c->ffnum--) *c->p++ = (uint8_t)(c->carry - 1);
        c->cache = c->low >> 24;
        c->carry = 0;
    } else {
        c->ffnum++;
    }
    c->low <<= 8;
}

static void enc_put(arc *c, uint32_t cum, uint32_t f, uint32_t tot) {
    uint32_t before = c->low;
    c->low += cum * (c->rng /= tot);
    c->rng *= f;
    c->carry += c->low < before;
    while (c->rng < (1u << 24)) {
        c->rng <<= 8;
        shift_low(c);
    }
}

static int enc_finish(arc *c) {
    for (int k = 0; k < 5; k++) shift_low(c);
    return c->err;
}

static void dec_start(arc *c, const uint8_t *in, const uint8_t *end) {
    memset(c, 0, sizeof *c);
    c->rng = 0xFFFFFFFFu;
    c->ip = in;
    c->iend = end;
    if (in + 5 > end) {
        c->ip = end;
        return;
    }
    for (int k = 0; k < 5; k++) c->code = (c->code << 8) | *c->ip++;
}

static void al_encode(alist *m, arc *c, unsigned sym) {
    uint32_t acc = 0;
    int k = 1;
    while (m->sy[k] != sym) acc += m->fr[k++];
    enc_put(c, acc, m->fr[k], m->total);
    al_bump(m, k);
}

static unsigned al_decode(alist *m, arc *c) {
    uint32_t t = 0;
    if (m->total && c->rng >= m->total) t = c->code / (c->rng /= m->total);
    if (t > AMAX) return 0;
    uint32_t acc = 0;
    int k = 1;
    while ((acc += m->fr[k]) <= t) k++;
    if (k - 1 > m->cap) return 0;
    acc -= m->fr[k];
    c->code -= acc * c->rng;
    c->rng *= m->fr[k];
    while (c->rng < (1u << 24)) {
        if (c->ip >= c->iend) {
            c->err = -1;
            break;
        }
        c->code = (c->code << 8) + *c->ip++;
        c->rng <<= 8;
    }
    unsigned s = m->sy[k];
    al_bump(m, k);
    return s;
}

unsigned int ora_arith_compress_bound(unsigned int size, int order) {
    int N = (order >> 8) & 0xff;
    if (!N) N = 4;
    return (unsigned int)((order == 0 ? 1.05 * size + 257 * 3 + 4
                                      : 1.05 * size + 257 * 257 * 3 + 4 + 257 * 3 + 4) +
                          5 + ((order & AX_PACK) ? 1 : 0) +
                          ((order & AX_RLE) ? 1 + 257 * 3 + 4 : 0) +
                          ((order & AX_STRIPE) ? 7 + 5 * N : 0));
}

/* the four entropy coders: out[0] = max symbol + 1, then the coder bytes
 * (arith_dynamic.c:97-135, :172-223, :441-514, :575-656) */
static int ent_compress(const uint8_t *in, uint32_t n, uint8_t *out, uint32_t *out_size,
                        int o1, int rle) {
    int bound = (int)ora_arith_compress_bound(n, 0) - 5;
    if (bound > (int)*out_size) return -1;
    unsigned m = 0;
    for (uint32_t i = 0; i < n; i++)
        if (m < in[i]) m = in[i];
    m++;
    out[0] = (uint8_t)m;
    alist *bm = malloc(sizeof(alist) * 256);
    alist *rm = rle ? malloc(sizeof(alist) * 258) : NULL;
    if (!bm || (rle && !rm)) {
        free(bm);
        free(rm);
        return -1;
    }
    for (int i = 0; i < 256; i++) al_init(&bm[i], 256, (int)m);
    for (int i = 0; rle && i < 258; i++) al_init(&rm[i], 258, MAX_RUN);
    arc c;
    enc_start(&c, out + 1, out + *out_size);
    unsigned last = 0;
    if (!rle) {
        for (uint32_t i = 0; i < n; i++) {
            al_encode(&bm[o1 ? last : 0], &c, in[i]);
            last = in[i];
        }
    } else {
        for (uint32_t i = 0; i < n;) {
            al_encode(&bm[o1 ? last : 0], &c, in[i]);
            int run = 0;
            last = in[i++];
            while (i < n && in[i] == last) run++, i++;
            int rctx = (int)last;
            do {
                int cc = run < MAX_RUN ? run : MAX_RUN - 1;
                al_encode(&rm[rctx], &c, (unsigned)cc);
                run -= cc;
                if (rctx == (int)last)
                    rctx = 256;
                else
                    rctx += (rctx < 258 - 1);
                if (cc == MAX_RUN - 1 && run == 0) al_encode(&rm[rctx], &c, 0);
            } while (run);
        }
    }
    int e = enc_finish(&c);
    free(bm);
    free(rm);
    if (e < 0) return -1;
    *out_size = (uint32_t)(c.p - c.start) + 1;
    return 0;
}

static int ent_uncompress(const uint8_t *in, uint32_t in_size, uint8_t *out, uint32_t n,
                          int o1, int rle) {
    unsigned m = in[0] ? in[0] : 256;
    alist *bm = malloc(sizeof(alist) * 256);
    alist *rm = rle ? malloc(sizeof(alist) * 258) : NULL;
    if (!bm || (rle && !rm)) {
        free(bm);
        free(rm);
        return -1;
    }
    for (int i = 0; i < 256; i++) al_init(&bm[i], 256, (int)m);
    for (int i = 0; rle && i < 258; i++) al_init(&rm[i], 258, MAX_RUN);
    arc c;
    dec_start(&c, in + 1, in + in_size);
    unsigned last = 0;
    if (!rle) {
        for (uint32_t i = 0; i < n; i++) {
            out[i] = (uint8_t)al_decode(&bm[o1 ? last : 0], &c);
            last = out[i];
        }
    } else {
        for (uint32_t i = 0; i < n; i++) {
            out[i] = (uint8_t)al_decode(&bm[o1 ? last : 0], &c);
            last = out[i];
            uint32_t run = 0, r;
            int rctx = (int)last;
            do {
                r = al_decode(&rm[rctx], &c);
                if (rctx == (int)last)
                    rctx = 256;
                else
                    rctx += (rctx < 258 - 1);
                run += r;
            } while (r == MAX_RUN - 1 && run < n);
            while (run-- && i + 1 < n) out[++i] = (uint8_t)last;
        }
    }
    free(bm);
    free(rm);
    return c.err;
}

uint8_t *ora_arith_compress_to(uint8_t *in, unsigned int in_size, uint8_t *out,
                               unsigned int *out_size, int order) {
    if (in_size > INT_MAX || (out && *out_size == 0)) {
        *out_size = 0;
        return NULL;
    }
    uint8_t *own = NULL;
    if (!out) {
        *out_size = ora_arith_compress_bound(in_size, order);
        if (!(own = out = malloc(*out_size))) {
            *out_size = 0;
            return NULL;
        }
    }
    uint8_t *out_end = out + *out_size;
    unsigned c_meta_len;
    if (in_size <= 20) order &= ~AX_STRIPE;
    if (order & AX_CAT) {                 /* (:743-752, then falls through) */
        out[0] = AX_CAT;
        c_meta_len = 1 + (unsigned)ora_var_put_u32(&out[1], out_end, in_size);
        if (c_meta_len + in_size > *out_size) {
            free(own);
            *out_size = 0;
            return NULL;
        }
        memcpy(out + c_meta_len, in, in_size);
        *out_size = in_size + c_meta_len;
    }
    if (order & AX_STRIPE) {              /* (:754-869) */
        int N = (order >> 8) & 0xff;
        if (N == 0) N = 4;
        if ((unsigned)N > in_size) N = (int)in_size;
        uint8_t *tr = malloc(in_size);
        unsigned part[256], idx[256];
        if (!tr) {
            free(own);
            *out_size = 0;
            return NULL;
        }
        for (int i = 0; i < N; i++) {
            part[i] = in_size / (unsigned)N + ((in_size % (unsigned)N) > (unsigned)i);
            idx[i] = i ? idx[i - 1] + part[i - 1] : 0;
        }
        unsigned i, x;
        for (i = x = 0; i < in_size - (unsigned)N; i += (unsigned)N, x++)
            for (int j = 0; j < N; j++) tr[idx[j] + x] = in[i + (unsigned)j];
        for (; i < in_size; i += (unsigned)N, x++)
            for (int j = 0; i + (unsigned)j < in_size; j++) tr[idx[j] + x] = in[i + (unsigned)j];
        c_meta_len = 1;
        *out = (uint8_t)(order & ~AX_NOSZ);
        c_meta_len += (unsigned)ora_var_put_u32(out + c_meta_len, out_end, in_size);
        if (c_meta_len >= *out_size) {
            free(tr);
            free(own);
            *out_size = 0;
            return NULL;
        }
        out[c_meta_len++] = (uint8_t)N;
        uint8_t *out2 = out + 7 + 5 * N, *out2_start = out2;
        static const int M[4][4] = {{3, 1, 64, 0}, {2, 1, 0}, {2, 1, 128}, {2, 1, 128}};
        for (int s = 0; s < N; s++) {
            const int *m = M[s < 3 ? s : 3];
            int j, best_j = 0;
            unsigned best_sz = INT_MAX, olen2;
            for (j = 1; j <= m[0]; j++) {
                if (out2 - out > (long)*out_size) continue;
                olen2 = *out_size - (unsigned)(out2 - out);
                if ((order & 3) == 0 && (m[j] & 1)) continue;
                uint8_t *r = ora_arith_compress_to(tr + idx[s], part[s], out2, &olen2,
                                                   m[j] | AX_NOSZ);
                if (r && olen2 && best_sz > olen2) {
                    best_sz = olen2;
                    best_j = j;
                }
            }
            if (best_sz == INT_MAX) {
                free(tr);
                free(own);
                *out_size = 0;
                return NULL;
            }
            if (best_j != j - 1) {
                olen2 = *out_size - (unsigned)(out2 - out);
                if (!ora_arith_compress_to(tr + idx[s], part[s], out2, &olen2,
                                           m[best_j] | AX_NOSZ)) {
                    free(tr);
                    free(own);
                    *out_size = 0;
                    return NULL;
                }
            }
            out2 += olen2;
            c_meta_len += (unsigned)ora_var_put_u32(out + c_meta_len, out_end, olen2);
        }
        memmove(out + c_meta_len, out2_start, (size_t)(out2 - out2_start));
        free(tr);
        *out_size = c_meta_len + (unsigned)(out2 - out2_start);
        return out;
    }

    int do_pack = order & AX_PACK, do_rle = order & AX_RLE, no_size = order & AX_NOSZ;
    int do_ext = order & AX_EXT;
    out[0] = (uint8_t)order;
    c_meta_len = 1;
    if (!no_size) c_meta_len += (unsigned)ora_var_put_u32(&out[1], out_end, in_size);
    order &= 3;
    uint8_t *packed = NULL;
    if (do_pack && in_size) {             /* (:886-913) */
        if (c_meta_len + 256 > *out_size) {
            free(own);
            *out_size = 0;
            return NULL;
        }
        int pmeta_len;
        uint32_t plen;
        packed = ora_pack(in, in_size, out + c_meta_len, &pmeta_len, &plen);
        if (!packed) {
            out[0] &= (uint8_t)~AX_PACK;
            do_pack = 0;
        } else {
            in = packed;
            in_size = plen;
            c_meta_len += (unsigned)pmeta_len;
            int sz = ora_var_put_u32(out + c_meta_len, out_end, in_size);
            c_meta_len += (unsigned)sz;
            *out_size -= (unsigned)sz;
        }
    } else if (do_pack) {
        out[0] &= (uint8_t)~AX_PACK;
    }
    if (do_rle && !in_size) out[0] &= (uint8_t)~AX_RLE;
    *out_size -= c_meta_len;
    if (order && in_size < 8) {
        out[0] &= (uint8_t)~3;
        order &= ~3;
    }
    if (do_ext) {                         /* no libbz2 in the reference build */
        free(packed);
        free(own);
        *out_size = 0;
        return NULL;
    }
    if (ent_compress(in, in_size, out + c_meta_len, out_size, order == 1, do_rle != 0) < 0) {
        free(packed);
        free(own);
        *out_size = 0;
        return NULL;
    }
    if (*out_size >= in_size) {           /* (:980-993) */
        out[0] &= (uint8_t)~(3 | AX_EXT);
        out[0] |= (uint8_t)(AX_CAT | no_size);
        if (out + c_meta_len + in_size > out_end) {
            free(packed);
            free(own);
            *out_size = 0;
            return NULL;
        }
        memcpy(out + c_meta_len, in, in_size);
        *out_size = in_size;
    }
    free(packed);
    *out_size += c_meta_len;
    return out;
}

uint8_t *ora_arith_uncompress_to(uint8_t *in, unsigned int in_size, uint8_t *out,
                                 unsigned int *out_size) {
    const uint8_t *in_end = in + in_size;
    uint8_t *own = NULL;
    if (in_size == 0) return NULL;
    if (*in & AX_STRIPE) {                /* (:1040-1122) */
        unsigned ulen, c_meta_len = 1;
        uint64_t clen_tot = 0;
        c_meta_len += (unsigned)ora_var_get_u32(in + c_meta_len, in_end, &ulen);
        if (c_meta_len >= in_size) return NULL;
        unsigned N = in[c_meta_len++];
        if (N < 1) return NULL;
        unsigned clenN[256], ulenN[256], idxN[256];
        if (!out) {
            if (ulen >= INT_MAX) return NULL;
            if (!(own = out = malloc(ulen ? ulen : 1))) return NULL;
            *out_size = ulen;
        }
        if (ulen != *out_size) {
            free(own);
            return NULL;
        }
        for (unsigned i = 0; i < N; i++) {
            ulenN[i] = ulen / N + ((ulen % N) > i);
            idxN[i] = i ? idxN[i - 1] + ulenN[i - 1] : 0;
            c_meta_len += (unsigned)ora_var_get_u32(in + c_meta_len, in_end, &clenN[i]);
            clen_tot += clenN[i];
            if (c_meta_len > in_size || clenN[i] > in_size || clenN[i] < 1) {
                free(own);
                return NULL;
            }
        }
        if (c_meta_len + clen_tot > in_size) {
            free(own);
            return NULL;
        }
        in_size = c_meta_len + (unsigned)clen_tot;
        uint8_t *outN = malloc(ulen ? ulen : 1);
        if (!outN) {
            free(own);
            return NULL;
        }
        for (unsigned i = 0; i < N; i++) {
            unsigned olen = ulenN[i];
            if (in_size < c_meta_len ||
                !ora_arith_uncompress_to(in + c_meta_len, in_size - c_meta_len, outN + idxN[i],
                                         &olen) ||
                olen != ulenN[i]) {
                free(own);
                free(outN);
                return NULL;
            }
            c_meta_len += clenN[i];
        }
        /* unstripe (utils.h:79-138): byte k of stripe j -> out[k*N + j] */
        for (unsigned j = 0; j < N; j++)
            for (unsigned k = 0; k < ulenN[j]; k++) out[k * N + j] = outN[idxN[j] + k];
        free(outN);
        *out_size = ulen;
        return out;
    }
    int order = *in++;
    in_size--;
    int do_pack = order & AX_PACK, do_rle = order & AX_RLE, do_cat = order & AX_CAT;
    int no_size = order & AX_NOSZ, do_ext = order & AX_EXT;
    order &= 3;
    int sz = 0;
    unsigned osz;
    if (!no_size)
        sz = ora_var_get_u32(in, in_end, &osz);
    else
        osz = *out_size;
    in += sz;
    in_size -= (unsigned)sz;
    if (osz >= INT_MAX) return NULL;
    if (no_size && !out) return NULL;
    if (!out) {
        *out_size = osz;
        if (!(own = out = malloc(osz ? osz : 1))) return NULL;
    } else {
        if (*out_size < osz) return NULL;
        *out_size = osz;
    }
    unsigned tmp1_size = *out_size;
    uint8_t *tmp = NULL, *tmp1 = out;
    uint8_t map[256] = {0};
    int per = 0;
    uint64_t unpacked_sz = 0;
    if (do_pack) {                        /* (:1199-1218) */
        if (!(tmp = malloc(*out_size ? *out_size : 1))) goto err;
        tmp1 = tmp;
        int c_meta = ora_unpack_meta(in, in_size, map, &per) & 0xff;
        if (c_meta == 0) goto err;
        unpacked_sz = osz;
        in += c_meta;
        in_size -= (unsigned)c_meta;
        unsigned o2;
        sz = ora_var_get_u32(in, in_end, &o2);
        in += sz;
        in_size -= (unsigned)sz;
        if (o2 > tmp1_size) goto err;
        tmp1_size = o2;
    }
    if (in_size) {
        if (do_cat) {
            if (tmp1_size > in_size || tmp1_size > *out_size) goto err;
            memcpy(tmp1, in, tmp1_size);
        } else if (do_ext) {
            goto err;
        } else if (ent_uncompress(in, in_size, tmp1, tmp1_size, order == 1, do_rle != 0) < 0) {
            goto err;
        }
    } else {
        tmp1_size = 0;
    }
    unsigned tmp2_size = tmp1_size;
    if (do_pack) {
        if (per == 1) unpacked_sz = tmp1_size;   /* npacked_sym == 1 (no packing) */
        if (ora_unpack(tmp1, tmp1_size, out, (uint32_t)unpacked_sz, per, map)) goto err;
        tmp2_size = (unsigned)unpacked_sz;
    }
    free(tmp);
    *out_size = tmp2_size;
    return out;
err:
    free(tmp);
    free(own);
    return NULL;
}
