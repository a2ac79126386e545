// rans_format.hpp — host-side pieces of the rANS 4x16/32x16 stream format
// that are decisions or small tables rather than data-parallel work:
// varints, frequency normalisation, table (de)serialisation and the
// 10/12-bit shift decision.  The byte-parallel and chain work lives in
// rans_kernels.hip.
//
// Every function states the reference behaviour it reproduces
// (/root/reference/htscodecs/...).  Output bytes must be identical.
#pragma once
#include <cstdint>
#include <cstring>
#include <cmath>
#include <vector>

namespace fqz5 {

// order-byte flags (rANS_static4x16.h:75-103, rANS_static16_int.h:48-53)
enum : int {
    ORD_PACK = 0x80, ORD_RLE = 0x40, ORD_CAT = 0x20, ORD_NOSZ = 0x10,
    ORD_STRIPE = 0x08, ORD_X32 = 0x04,
    ORD_STRIPE_NO0 = 1 << 16, ORD_SIMD_AUTO = 1 << 17,
};

constexpr uint32_t RANS_LOW = 1u << 15;  // rANS_word.h:64

// ---- varint.h:206/:267 (BIG_END): 7-bit groups, most significant first --
inline int varint_len(uint32_t v) {
    int n = 1;
    while (v >>= 7) n++;
    return n;
}

// With an end pointer and fewer than 5 bytes of room, the reference's
// var_put_u32_safe (varint.h:173) refuses to write and returns 0.
inline int varint_put(uint8_t *cp, const uint8_t *endp, uint32_t v) {
    int n = varint_len(v);
    if (endp && endp - cp < 5 && endp - cp < n) return 0;
    for (int k = n - 1; k >= 0; k--)
        *cp++ = uint8_t(((v >> (7 * k)) & 0x7f) | (k ? 0x80 : 0));
    return n;
}

inline int varint_get(const uint8_t *cp, const uint8_t *endp, uint32_t *v) {
    if (cp >= endp) { *v = 0; return 0; }
    uint32_t r = 0;
    int n = 0;
    uint8_t c;
    do {
        c = cp[n++];
        r = (r << 7) | (c & 0x7f);
    } while ((c & 0x80) && n < 6 && cp + n < endp);
    *v = r;
    return n;
}

// ---- rANS_static4x16pr.c:93 --------------------------------------------
inline unsigned compress_bound(unsigned size, int order) {
    int N = (order >> 8) & 0xff;
    if (!N) N = 4;
    int o = order & 0xff;
    double d = (o == 0 ? 1.05 * size + 775.0 : 1.05 * size + 198926.0)
             + ((o & ORD_PACK) ? 1 : 0) + ((o & ORD_RLE) ? 776 : 0) + 20
             + ((o & ORD_X32) ? 112 : 0) + ((o & ORD_STRIPE) ? 7 + 5 * N : 0);
    unsigned sz = unsigned(d);
    return sz + (sz & 1) + 2;
}

inline uint32_t pow2_ceil(uint32_t v) {          // round2, rANS_static16_int.h:86
    if (!v) return 0;
    uint32_t r = 1;
    while (r < v) r <<= 1;
    return r;
}

// normalise_freq (rANS_static16_int.h:97-146): 31-bit fixed-point rescale of
// F (summing to `size`) to sum to `tot`; non-zero entries stay >= 1; the
// residual goes to the most frequent symbol, with one re-scale pass and a
// final spread when that symbol cannot absorb it.
inline int normalise_freq(uint32_t *F, int size, uint32_t tot) {
    if (!size) return 0;
    bool retried = false;
    for (;;) {
        uint64_t scale = (uint64_t(tot) << 31) / size + (1 << 30) / size;
        int top = 0, topsym = 0, sum = 0;
        for (int s = 0; s < 256; s++) {
            if (!F[s]) continue;
            if (top < int(F[s])) { top = int(F[s]); topsym = s; }
            uint32_t v = uint32_t((uint64_t(F[s]) * scale) >> 31);
            F[s] = v ? v : 1;
            sum += int(F[s]);
        }
        int excess = int(tot) - sum;
        if (excess < 0) {
            int need = -excess, have = int(F[topsym]);
            if (have > need && (retried || have / 2 >= need)) {
                F[topsym] -= need;
            } else if (!retried) {
                retried = true;
                size = sum;
                continue;
            } else {
                excess += have - 1;
                F[topsym] = 1;
                for (int s = 0; excess && s < 256; s++) {
                    if (F[s] < 2) continue;
                    int d = int(F[s]) > -excess ? excess : 1 - int(F[s]);
                    F[s] += d;
                    excess -= d;
                }
            }
        } else if (excess > 0) {
            F[topsym] += excess;
        }
        return F[topsym] > 0 ? 0 : -1;
    }
}

// normalise_freq_shift (rANS_static16_int.h:151): power-of-two up-scale.
inline void scale_pow2(uint32_t *F, uint32_t size, uint32_t target) {
    if (!size || size == target) return;
    int sh = 0;
    while (size < target) { size <<= 1; sh++; }
    for (int s = 0; s < 256; s++) F[s] <<= sh;
}

// ---- symbol lists (rANS_static16_int.h:165-238) -------------------------
// Ascending present symbols; a symbol whose predecessor is also present is
// followed by the count of further consecutive present symbols it implies;
// a 0 byte terminates the list.
inline int put_alphabet(uint8_t *cp, const uint32_t *F) {
    uint8_t *p = cp;
    for (int s = 0; s < 256; s++) {
        if (!F[s]) continue;
        *p++ = uint8_t(s);
        if (s && F[s - 1]) {
            int e = s + 1;
            while (e < 256 && F[e]) e++;
            *p++ = uint8_t(e - s - 1);
            s = e - 1;
        }
    }
    *p++ = 0;
    return int(p - cp);
}

inline int get_alphabet(const uint8_t *cp, const uint8_t *end, uint32_t *F) {
    const uint8_t *p = cp;
    if (p >= end) return 0;
    int s = *p++, run = 0;
    for (;;) {
        F[s] = 1;
        if (run) {
            run--;
            if (++s > 255) return 0;
        } else if (p < end && *p == s + 1) {
            if (p + 1 >= end) return 0;
            s = *p++;
            run = *p++;
        } else {
            if (p >= end) return 0;
            s = *p++;
        }
        if (!s) break;
    }
    return int(p - cp);
}

// O0 table: alphabet then one varint per present symbol (:240-272)
inline int put_freq0(uint8_t *cp, const uint32_t *F) {
    int n = put_alphabet(cp, F);
    for (int s = 0; s < 256; s++)
        if (F[s]) n += varint_put(cp + n, nullptr, F[s]);
    return n;
}

inline int get_freq0(const uint8_t *cp, const uint8_t *end, uint32_t *F,
                     uint32_t *tot) {
    int n = get_alphabet(cp, end, F);
    if (!n) return 0;
    uint32_t t = 0;
    for (int s = 0; s < 256; s++) {
        if (!F[s]) continue;
        if (cp + n >= end) return 0;
        n += varint_get(cp + n, end, &F[s]);
        t += F[s];
    }
    *tot = t;
    return n;
}

// O1 row against the context alphabet A; zero runs as {0, run-1} (:278-306)
inline int put_freq_row(uint8_t *cp, const uint32_t *A, const uint32_t *F) {
    uint8_t *p = cp;
    int zrun = 0;
    for (int s = 0; s < 256; s++) {
        if (!A[s]) continue;
        if (!F[s]) { zrun++; continue; }
        if (zrun) { *p++ = 0; *p++ = uint8_t(zrun - 1); zrun = 0; }
        p += varint_put(p, nullptr, F[s]);
    }
    if (zrun) { *p++ = 0; *p++ = uint8_t(zrun - 1); }
    return int(p - cp);
}

inline int get_freq_row(const uint8_t *cp, const uint8_t *end,
                        const uint32_t *A, uint32_t *F, uint32_t *tot) {
    const uint8_t *p = cp;
    int zrun = 0;
    uint32_t t = 0;
    for (int s = 0; s < 256; s++) {
        if (!A[s]) continue;
        uint32_t f = 0;
        if (zrun) {
            zrun--;
        } else {
            if (p >= end) return 0;
            p += varint_get(p, end, &f);
            if (!f) {
                if (p >= end) return 0;
                zrun = *p++;
            }
        }
        F[s] = f;
        t += f;
    }
    *tot = t;
    return int(p - cp);
}

// fast_log (utils.h:69): linear-in-exponent log2 approximation.
inline double approx_log2(double a) {
    int64_t bits;
    std::memcpy(&bits, &a, sizeof bits);
    return double(bits - 4606921278410026770LL) * 1.539095918623324e-16;
}

// rans_compute_shift (rANS_static4x16pr.c:357-420): estimate the cost of a
// 10-bit vs 12-bit O1 table and each row's power-of-two storage scale.
inline int o1_pick_shift(const uint32_t *T, const uint32_t (*F)[256],
                         uint32_t *rowmax) {
    double c10 = 0, c12 = 0;
    uint32_t maxall = 0;
    for (int i = 0; i < 256; i++) {
        if (!T[i]) continue;
        uint32_t mv = pow2_ceil(T[i]);
        int used = 0, tiny10 = 0, tiny12 = 0;
        for (int j = 0; j < 256; j++) {
            if (!F[i][j]) continue;
            if (mv / F[i][j] > 1024) tiny10++;
            if (mv / F[i][j] > 4096) tiny12++;
        }
        double lg10 = std::log(double(1024 + tiny10));
        double lg12 = std::log(double(4096 + tiny12));
        double r12 = 4096.0 / T[i], r10 = 1024.0 / T[i];
        for (int j = 0; j < 256; j++) {
            if (!F[i][j]) continue;
            used++;
            double a = F[i][j] * r10, b = F[i][j] * r12;
            c10 -= F[i][j] * (approx_log2(a > 1 ? a : 1) - lg10);
            c12 -= F[i][j] * (approx_log2(b > 1 ? b : 1) - lg12);
            c10 += 1.3;
            c12 += 4.7;
        }
        if (used < 64 && mv > 128) mv >>= 1;
        if (mv > 1024) mv >>= 1;
        if (mv > 4096) mv = 4096;
        rowmax[i] = mv;
        if (maxall < mv) maxall = mv;
    }
    return (c10 / c12 < 1.01 || maxall <= 1024) ? 10 : 12;
}

// Encoder symbol of the GPU encode kernel (16 bytes), from
// RansEncSymbolInit (rANS_word.h:201-272):
//   x_max = ((L >> bits) << 16) * f - 1
//   rcp   = ceil(2^(s+31)/f) with s = ceil(log2 f), or ~0 when f < 2
//   bias  = start (f >= 2) or start + 2^bits - 1 (f < 2)
//   cmpl_sh = (2^bits - f) | (rcp_shift - 32) << 16
struct EncSym { uint32_t rcp, xmax, bias, cmpl_sh; };

inline EncSym make_encsym(uint32_t start, uint32_t f, int bits) {
    EncSym e;
    uint32_t sh;
    e.xmax = ((RANS_LOW >> bits) << 16) * f - 1;
    if (f < 2) {
        e.rcp = ~0u;
        sh = 0;
        e.bias = start + (1u << bits) - 1;
    } else {
        uint32_t s = 0;
        while (f > (1u << s)) s++;
        e.rcp = uint32_t(((1ull << (s + 31)) + f - 1) / f);
        sh = s - 1;
        e.bias = start;
    }
    e.cmpl_sh = (((1u << bits) - f) & 0xffff) | (sh << 16);
    return e;
}

}  // namespace fqz5
