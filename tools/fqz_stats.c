/* fqz_stats.c — decoder design statistics (tool, not product): runs the
 * oracle's fqz decoder (oracle/fqz_oracle.c) over a stream and counts, per
 * quality symbol, the decoded slot, one-step bubble swaps, halvings, repeats
 * of the previous context, and the misses of direct-mapped caches of a few
 * sizes.  Build: gcc -O2 -I oracle tools/fqz_stats.c oracle/rans_oracle.c -lm -o /tmp/fqz_stats
 * (see tools/fqz_stats.py for the driver).
 */
#include <stdio.h>
#include <stdlib.h>
#include "cm_common.h"

static struct {
    void *base;
    size_t stride;
    unsigned long long n, ksum, kge[8], swaps, halves, same, uniq;
    int prev;
    FILE *dump;                       /* $FQZ_CTX_DUMP: the context of every symbol, u16 */
    unsigned char seen[65536];
    int tags[8][65536];
    int wtags[6][65536];              /* set-associative: ways consecutive, MRU first */
    unsigned char evicted[6][65536];
} S;
static const unsigned NSETS[8] = {256, 512, 760, 1024, 2048, 2456, 3548, 65536};
static unsigned long long MISS[8];
/* models in the cache x ways (LRU within a set): the 8-byte-slot decoder's
 * capacity for 42 live symbols (362 models) and a 5-byte layout's (580) */
static const unsigned WMODELS[6] = {362, 362, 362, 580, 580, 580};
static const unsigned WWAYS[6] = {1, 2, 4, 1, 2, 4};
static unsigned long long WMISS[6], WREFETCH[6];

static unsigned fl_decode_stats(flist *m, rcoder *c, int cap) {
    if (cap != 96 || !S.base) return fl_decode(m, c, cap);
    const int ctx = (int)(((char *)m - (char *)S.base) / (long)S.stride);
    const uint32_t tot0 = m->total;
    uint32_t t = 0;
    {
        rcoder cc = *c;
        t = rc_target(&cc, m->total);
    }
    int k = 1;
    uint32_t acc = 0;
    while ((acc += m->fr[k]) <= t && k < 258) k++;
    S.n++;
    S.ksum += (unsigned long long)k;
    for (int b = 0; b < 8; b++) S.kge[b] += k > (1 << b);
    const uint16_t before = m->fr[k];
    (void)before;
    unsigned s = fl_decode(m, c, cap);
    if (tot0 + FL_STEP > FL_CAP_MAX) S.halves++;
    if (m->sy[k] != s) S.swaps++;
    S.same += ctx == S.prev;
    S.prev = ctx;
    if (!S.seen[ctx]) { S.seen[ctx] = 1; S.uniq++; }
    if (S.dump) { const uint16_t c16 = (uint16_t)ctx; fwrite(&c16, 2, 1, S.dump); }
    const uint32_t h = ((uint32_t)ctx * 0x9E3779u) & 0xffffffu;   /* the decoder's set_addr */
    for (int i = 0; i < 6; i++) {
        const unsigned ways = WWAYS[i], nset = WMODELS[i] / ways;
        const unsigned set = (unsigned)(((uint64_t)h * nset) >> 24);
        int *t = &S.wtags[i][set * ways];
        unsigned w = 0;
        while (w < ways && t[w] != ctx + 1) w++;
        if (w == ways) {   /* miss: evict the LRU way */
            WMISS[i]++;
            if (S.evicted[i][ctx]) WREFETCH[i]++;
            w = ways - 1;
            if (t[w]) S.evicted[i][t[w] - 1] = 1;
        }
        for (; w > 0; w--) t[w] = t[w - 1];
        t[0] = ctx + 1;
    }
    for (int i = 0; i < 8; i++) {
        const unsigned set = NSETS[i] == 65536 ? (unsigned)ctx : (unsigned)(((uint64_t)h * NSETS[i]) >> 24);
        if (S.tags[i][set] != ctx + 1) { MISS[i]++; S.tags[i][set] = ctx + 1; }
    }
    return s;
}
static void *cap_malloc(size_t n) {
    void *p = malloc(n);
    if (n == sizeof(flist) * 65536) {   /* the quality models (models_new) */
        S.base = p;
        S.stride = sizeof(flist);
    }
    return p;
}
#define fl_decode fl_decode_stats
#define malloc cap_malloc
#include "fqz_oracle.c"
#undef malloc

int main(int argc, char **argv) {
    if (argc < 2) return 2;
    FILE *f = fopen(argv[1], "rb");
    if (!f) return 2;
    fseek(f, 0, SEEK_END);
    long n = ftell(f);
    fseek(f, 0, SEEK_SET);
    uint8_t *in = malloc((size_t)n);
    if (fread(in, 1, (size_t)n, f) != (size_t)n) return 2;
    fclose(f);
    S.prev = -1;
    if (getenv("FQZ_CTX_DUMP")) S.dump = fopen(getenv("FQZ_CTX_DUMP"), "wb");
    size_t out = 0;
    uint8_t *o = ora_fqz_decompress(in, (size_t)n, &out, NULL, 0, NULL);
    if (!o) { fprintf(stderr, "decode failed\n"); return 1; }
    if (S.dump) fclose(S.dump);
    printf("{\"n\": %llu, \"k_mean\": %.3f, \"k_gt\": [", S.n, (double)S.ksum / (double)S.n);
    for (int b = 0; b < 8; b++) printf("%s%.4f", b ? ", " : "", (double)S.kge[b] / (double)S.n);
    printf("], \"swap\": %.4f, \"halve\": %.5f, \"same_ctx\": %.4f, \"contexts\": %llu, \"miss\": {",
           (double)S.swaps / (double)S.n, (double)S.halves / (double)S.n, (double)S.same / (double)S.n, S.uniq);
    for (int i = 0; i < 8; i++) printf("%s\"%u\": %.4f", i ? ", " : "", NSETS[i], (double)MISS[i] / (double)S.n);
    printf("}, \"assoc\": {");
    for (int i = 0; i < 6; i++)
        printf("%s\"%ux%u\": [%.4f, %.4f]", i ? ", " : "", WMODELS[i], WWAYS[i], (double)WMISS[i] / (double)S.n,
               (double)WREFETCH[i] / (double)S.n);
    printf("}}\n");
    return 0;
}
