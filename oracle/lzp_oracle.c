/* lzp_oracle.c — TEST ORACLE ONLY (never linked into the product).
 *
 * Plain-C restatement of fqzcomp5's LZP pre-pass and its LZP3 sequence
 * method:
 *   lzp / unlzp        lzp16e.c:113-164 / :166-214 (HASH_LEN 16, MIN_LEN 3,
 *                      MATCH_CHAR 233; FAST_MODE is not defined)
 *   match length       lzp16e.c:58-95
 *   hash update        lzp16e.c:102, evaluated in unsigned 32-bit arithmetic
 *                      (the reference multiplies a signed int and relies on
 *                      two's-complement wrap-around; only the low 16 bits
 *                      are kept, which wrap-around does not change)
 *   LZP3               fqzcomp5.c:2013-2021 (lzp, then rANS 4x16 order 5 =
 *                      X32 order 1) and :2431-2445 (rANS, then unlzp)
 * Every table position is the position of a byte: ht[h] = i for every input
 * position i, whether it starts a token or lies inside a match, and a token
 * at i looks up ht[h_i] before position i is stored.  ht[h] == 0 (never set,
 * or set by position 0) means "no prediction".
 * Pinned against the reference's lzp / unlzp compiled from /root/reference
 * into oracle/_ref/libhtsref.so by tests/test_lzp_oracle.py and the vectors
 * of tests/golden/make_golden_lzp.py.
 */
#include <stdlib.h>
#include <string.h>

#include "oracle.h"

#define LZP_HBITS 16
#define LZP_MIN 3
#define LZP_MARK 233

static uint32_t lzp_hash(uint32_t h, uint8_t c) {
    return ((((h * 0x8ca6b53u) << 4) + (h << 5) * 17u) ^ c) & ((1u << LZP_HBITS) - 1);
}

/* lzp16e.c:58-95: 0 unless at least MIN_LEN bytes remain and match */
static uint32_t lzp_match(const uint8_t *in, uint32_t i, uint32_t n, uint32_t p) {
    const uint32_t left = n - i;
    if (left < LZP_MIN) return 0;
    uint32_t k = 0;
    while (k < left && in[i + k] == in[p + k]) k++;
    return k < LZP_MIN ? 0 : k;
}

/* lzp(): returns the output length; `out` needs room for 3 bytes per input
 * byte in the worst case (escaped literals). */
int ora_lzp(const uint8_t *in, int in_len, uint8_t *out) {
    uint32_t *ht = calloc(1u << LZP_HBITS, sizeof *ht);
    if (!ht) return -1;
    const uint32_t n = in_len > 0 ? (uint32_t)in_len : 0;
    uint32_t h = 0, o = 0, i = 0;
    while (i < n) {
        const uint32_t p = ht[h];
        uint32_t ml = p ? lzp_match(in, i, n, p) : 0;
        if (ml > 65535) ml = 65535;
        if (ml >= LZP_MIN) {
            if (ml <= 255) {
                out[o++] = LZP_MARK;
                out[o++] = (uint8_t)ml;
            } else {
                out[o++] = LZP_MARK + 1;
                out[o++] = (uint8_t)(ml >> 8);
                out[o++] = (uint8_t)ml;
            }
            for (uint32_t k = 0; k < ml; k++, i++) {   /* every matched byte enters */
                ht[h] = i;
                h = lzp_hash(h, in[i]);
            }
            continue;
        }
        /* a literal; with a prediction, a literal that looks like a marker
         * is escaped as a zero-length match */
        if (p && (in[i] == LZP_MARK || in[i] == LZP_MARK + 1)) {
            out[o++] = LZP_MARK;
            out[o++] = 0;
        }
        out[o++] = in[i];
        ht[h] = i;
        h = lzp_hash(h, in[i]);
        i++;
    }
    free(ht);
    return (int)o;
}

/* unlzp(): returns the output length, or -1 when the stream would write
 * more than out_cap bytes or ends inside a token (the reference has no such
 * checks; on valid input the result is the same). */
int ora_unlzp(const uint8_t *in, int in_len, uint8_t *out, int out_cap) {
    uint32_t *ht = calloc(1u << LZP_HBITS, sizeof *ht);
    if (!ht) return -1;
    const uint32_t n = in_len > 0 ? (uint32_t)in_len : 0, cap = out_cap > 0 ? (uint32_t)out_cap : 0;
    uint32_t h = 0, i = 0, j = 0;
    int rc = 0;
    while (i < n) {
        const uint32_t p = ht[h];
        uint32_t ml = 0;
        uint8_t lit = in[i];
        uint32_t adv = 1;                         /* input bytes of this token */
        if (p && (in[i] == LZP_MARK || in[i] == LZP_MARK + 1)) {
            if (in[i] == LZP_MARK) {
                if (i + 1 >= n) { rc = -1; break; }
                ml = in[i + 1];
                adv = 2;
            } else {
                if (i + 2 >= n) { rc = -1; break; }
                ml = (uint32_t)in[i + 1] << 8 | in[i + 2];
                adv = 3;
            }
            if (!ml) {                            /* escaped literal follows */
                if (i + adv >= n) { rc = -1; break; }
                lit = in[i + adv];
                adv++;
            }
        }
        if (ml) {
            if (j + ml > cap) { rc = -1; break; }
            for (uint32_t k = 0; k < ml; k++) out[j + k] = out[p + k];   /* forward: overlaps repeat */
            for (uint32_t k = 0; k < ml; k++, j++) {
                ht[h] = j;
                h = lzp_hash(h, out[j]);
            }
        } else {
            if (j >= cap) { rc = -1; break; }
            out[j] = lit;
            ht[h] = j++;
            h = lzp_hash(h, lit);
        }
        i += adv;
    }
    free(ht);
    return rc ? -1 : (int)j;
}

/* LZP3 (fqzcomp5.c:2013-2021): rANS 4x16 order 5 of the lzp output. */
uint8_t *ora_lzp3_compress(uint8_t *in, unsigned int in_size, unsigned int *out_size) {
    uint8_t *tmp = malloc((size_t)in_size * 3 + 16);
    if (!tmp) return NULL;
    const int t = ora_lzp(in, (int)in_size, tmp);
    uint8_t *out = t < 0 ? NULL : ora_rans_compress_4x16(tmp, (unsigned)t, out_size, 5);
    free(tmp);
    return out;
}

/* fqzcomp5.c:2431-2445; u_len is the section's stored size. */
uint8_t *ora_lzp3_uncompress(uint8_t *in, unsigned int in_size, unsigned int u_len,
                             unsigned int *out_size) {
    unsigned int rl = 0;
    uint8_t *r = ora_rans_uncompress_4x16(in, in_size, &rl);
    if (!r) return NULL;
    uint8_t *out = malloc(u_len ? u_len : 1);
    const int j = out ? ora_unlzp(r, (int)rl, out, (int)u_len) : -1;
    free(r);
    if (j < 0) {
        free(out);
        return NULL;
    }
    *out_size = (unsigned)j;
    return out;
}
