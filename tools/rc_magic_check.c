/* The range chain's division (k_rc_magic / k_fqz_rc, fqz_kernels.hip):
 * floor(R / t) = (mulhi(R, m) + R) >> l with l = ceil(log2 t),
 * m = floor(2^32 (2^l - t) / t) + 1, for every total t of an adaptive model
 * (1 <= t < 2^16) and R < 2^32.  Every t against edge and random ranges, then
 * five divisors over all 2^32 ranges (~1 min).
 *   gcc -O3 -march=native -o /tmp/rc_magic_check tools/rc_magic_check.c */
#include <stdint.h>
#include <stdio.h>

static uint32_t magic_l(uint32_t t) { return t > 1 ? 32u - (uint32_t)__builtin_clz(t - 1) : 0u; }
static uint32_t magic_m(uint32_t t, uint32_t l) {
    return (uint32_t)((((1ull << l) - t) << 32) / t + 1);
}
static uint32_t div_magic(uint32_t R, uint32_t m, uint32_t l) {
    const uint32_t hi = (uint32_t)(((uint64_t)R * m) >> 32);
    return (uint32_t)(((uint64_t)hi + R) >> l);
}

int main(void) {
    unsigned long bad = 0, n = 0;
    uint64_t s = 88172645463325252ull;
    for (uint32_t t = 1; t < 65536; t++) {
        const uint32_t l = magic_l(t), m = magic_m(t, l);
        uint32_t R[64];
        int k = 0;
        R[k++] = 0xffffffffu;
        R[k++] = 1u << 24;
        R[k++] = (1u << 24) - 1 + t;
        R[k++] = 0xffffffffu - 0xffffffffu % t;
        R[k++] = 0xffffffffu - 0xffffffffu % t - 1;
        for (; k < 64; k++) {
            s ^= s << 13; s ^= s >> 7; s ^= s << 17;
            R[k] = (uint32_t)s;
            if (k & 1) R[k] = R[k] - R[k] % t + ((k & 2) ? t - 1 : 0);
        }
        for (int i = 0; i < 64; i++, n++)
            if (div_magic(R[i], m, l) != R[i] / t) {
                if (bad < 5) printf("t %u R %u\n", t, R[i]);
                bad++;
            }
    }
    printf("all totals: %lu ranges checked, %lu wrong\n", n, bad);
    const uint32_t ts[] = {3, 7, 641, 40961, 65519};
    for (int j = 0; j < 5; j++) {
        const uint32_t t = ts[j], l = magic_l(t), m = magic_m(t, l);
        unsigned long b = 0;
        uint32_t R = 0;
        do { b += div_magic(R, m, l) != R / t; } while (++R != 0);
        printf("t %u: all 2^32 ranges, %lu wrong\n", t, b);
        bad += b;
    }
    return bad != 0;
}
