// ubench.hip — single-wave dependent-chain latencies on gfx950, to size the
// rANS chain kernels.  Each test runs a chain of N dependent
// operations in one wave and reports shader cycles (s_memtime) per op and
// the shader clock (s_memtime vs the 100 MHz s_memrealtime).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define N 4096

__device__ __forceinline__ uint64_t now() { return __builtin_amdgcn_s_memtime(); }
__device__ __forceinline__ uint64_t rnow() { return __builtin_amdgcn_s_memrealtime(); }

template <int T>
__global__ void k(uint32_t *out, uint64_t *cyc, uint32_t a, uint32_t b) {
    __shared__ uint32_t lds[4096];
    const int l = threadIdx.x;
    for (int i = l; i < 4096; i += 64) lds[i] = (i * 2654435761u) & 4095;
    __syncthreads();
    uint32_t x = a + l, y = b;
    uint32_t nw = 0, flags = 0;
    __builtin_amdgcn_s_waitcnt(0);
    uint64_t t0 = now(), r0 = rnow();
#pragma unroll 16
    for (int i = 0; i < N; i++) {
        if (T == 0) x = x + y;                                   // v_add dep chain
        if (T == 1) x = __umulhi(x, y) + 1;                      // mul_hi + add
        if (T == 2) x = __umul24(x, y) + 1;                      // mul24 + add
        if (T == 3) x = lds[x & 4095];                           // LDS dep chain
        if (T == 4) {                                            // ballot chain
            const bool c = x > y;
            nw += __popcll(__ballot(c));
            x = x + nw;
        }
        if (T == 5) {                                            // encoder step
            const uint32_t xo = x;
            const bool c = xo > y;
            const uint32_t xr = c ? (xo >> 16) : xo;
            const uint32_t q = __umulhi(xr, b) >> (a & 7);
            x = __umul24(q, 3u) + (xr + 12345u);
        }
        if (T == 6) {                                            // enc step + word write
            const uint32_t xo = x;
            const bool c = xo > y;
            const uint32_t xr = c ? (xo >> 16) : xo;
            const uint32_t q = __umulhi(xr, b) >> (a & 7);
            x = __umul24(q, 3u) + (xr + 12345u);
            const uint64_t m = __ballot(c) & 15;
            const uint32_t g = nw + __popcll(m & (~0ull << (l + 1)));
            lds[(c && l < 4) ? (g & 2047) : (2048 + l)] = xo;
            nw += __popcll(m);
        }
        if (T == 7) {                                            // dec step (O0, LDS table)
            const uint32_t e = lds[x & 4095];
            const uint32_t xh = x >> 12;
            const uint32_t xd = __umul24(e >> 20, xh) + xh + ((e >> 8) & 4095);
            const bool c = xd < (1u << 15);
            const uint64_t m = __ballot(c) & 15;
            const uint32_t rank = __builtin_amdgcn_mbcnt_lo(uint32_t(m), 0u);
            const uint32_t w = uint32_t((uint64_t(y) << 16 | nw) >> (rank * 16));
            x = c ? __builtin_amdgcn_perm(xd, w, 0x05040100u) : xd;
            nw += __popcll(m);
        }
        if (T == 8) {                                            // enc step, private stack
            const uint32_t xo = x;
            const bool c = xo > y;
            const uint32_t xr = c ? (xo >> 16) : xo;
            const uint32_t q = __umulhi(xr, b) >> (a & 7);
            x = __umul24(q, 3u) + (xr + 12345u);
            lds[c ? ((l << 6) + (nw & 63)) : (3072 + l)] = xo;
            nw += c;
            flags = (flags << 1) | c;
        }
        if (T == 9) {                                            // dec step, DPP quad rank
            const uint32_t e = lds[x & 4095];
            const uint32_t xh = x >> 12;
            const uint32_t xd = __umul24(e >> 20, xh) + xh + ((e >> 8) & 4095);
            const uint32_t c = xd < (1u << 15);
            // inclusive prefix over the quad: row_shr:1 then row_shr:2 (bound_ctrl 0)
            uint32_t s1 = c + __builtin_amdgcn_update_dpp(0u, c, 0x111, 0xf, 0xf, true);
            uint32_t s2 = s1 + __builtin_amdgcn_update_dpp(0u, s1, 0x112, 0xf, 0xf, true);
            const uint32_t tot = __builtin_amdgcn_update_dpp(0u, s2, 0xff, 0xf, 0xf, false);
            const uint32_t rank = s2 - c;
            const uint32_t w = uint32_t((uint64_t(y) << 16 | nw) >> (rank * 16));
            x = c ? __builtin_amdgcn_perm(xd, w, 0x05040100u) : xd;
            nw += tot;
        }
        if (T == 10) {                                           // dec step, ballot + v_bcnt ptr
            const uint32_t e = lds[x & 4095];
            const uint32_t xh = x >> 12;
            const uint32_t xd = __umul24(e >> 20, xh) + xh + ((e >> 8) & 4095);
            const bool c = xd < (1u << 15);
            const uint64_t m = __ballot(c);
            const uint32_t rank = __builtin_amdgcn_mbcnt_lo(uint32_t(m) & 15u, 0u);
            const uint32_t w = uint32_t((uint64_t(y) << 16 | nw) >> (rank * 16));
            x = c ? __builtin_amdgcn_perm(xd, w, 0x05040100u) : xd;
            nw = __builtin_amdgcn_mbcnt_lo(uint32_t(m) & 15u, nw + 0u * l) + 0;
        }
        if (T == 12) {                                           // f64 fma dep chain
            double d = double(x);
            d = __fma_rn(d, 1.0000001, 0.5);
            x = uint32_t(__double_as_longlong(d));
        }
        if (T == 13) {                                           // u32 -> f64 -> fma -> u32
            x = uint32_t(__fma_rn(double(x), 0.999999, 1.0 / 524288.0));
        }
        if (T == 14) {                                           // mul_lo u32 dep
            x = x * y + 1;
        }
        if (T == 15) {                                           // fqz range step
            const uint32_t q = uint32_t(__fma_rn(double(x | 0x1000000u), 1.0 / 3000.0, 1.0 / 524288.0));
            uint32_t r = q * (y & 0xfff);
            const uint32_t k = r < (1u << 24) ? (__clz(r) >> 3) : 0u;
            x = r << (8 * k);
        }
        if (T == 16) {                                           // f32 rcp-based u32 div + fix
            const float fq = float(x) * __builtin_amdgcn_rcpf(float(y | 1));
            uint32_t q = uint32_t(fq);
            q += (x - q * (y | 1)) >= (y | 1);
            x = q + 12345;
        }
        if (T == 17) {                                           // ballot -> popc -> readlane -> SALU
            const uint64_t m = __ballot(x > y);
            const uint32_t k = uint32_t(__popcll(m)) & 63u;
            y = __builtin_amdgcn_readlane(x, k) + 1u;
        }
        if (T == 18) {                                           // LDS read -> readlane -> address
            const uint32_t v = lds[(y + l) & 4095];
            y = __builtin_amdgcn_readlane(v, 0) & 4095u;
        }
        if (T == 19) {                                           // LDS write then dependent read
            lds[(y + l) & 4095] = x;
            x = lds[(y + l + 1) & 4095] + 1u;
            y = __builtin_amdgcn_readfirstlane(x) & 4095u;
        }
        if (T == 20) {                                           // recip: cvt, rcp, 2 fma, use
            const double d = double(x | 1u);
            const double r0 = __builtin_amdgcn_rcp(d);
            const double e = __fma_rn(-d, r0, 1.0);
            x = uint32_t(__fma_rn(r0, e, r0) * 1e9);
        }
        if (T == 21) {                                           // model step skeleton, no LDS
            const uint64_t m = __ballot(x * 3u <= y) & 0x3eull;
            const uint32_t k = uint32_t(__popcll(m));
            const uint32_t pk = __builtin_amdgcn_readlane(x, k), pk1 = __builtin_amdgcn_readlane(x, k + 1);
            y = (y - pk) + (pk1 - pk);
            x += l > k ? 0x100000u : (l == k ? 16u : 0u);
        }
        if (T == 11) {                                           // dec: table lookup + arith only
            const uint32_t e = lds[x & 4095];
            const uint32_t xh = x >> 12;
            x = __umul24(e >> 20, xh) + xh + ((e >> 8) & 4095);
        }
    }
    uint64_t t1 = now(), r1 = rnow();
    out[l] = x + nw + flags;
    if (l == 0) { cyc[0] = t1 - t0; cyc[1] = r1 - r0; }
}

template <int T> void run(const char *name) {
    uint32_t *d;
    uint64_t *c, h[2];
    (void)hipMalloc(&d, 64 * 4);
    (void)hipMalloc(&c, 16);
    for (int rep = 0; rep < 2; rep++) {
        hipLaunchKernelGGL(k<T>, dim3(1), dim3(64), 0, 0, d, c, 0x12345u, 0x9e3779b9u);
        (void)hipDeviceSynchronize();
    }
    (void)hipMemcpy(h, c, 16, hipMemcpyDeviceToHost);
    double cyc = double(h[0]) / N, ghz = double(h[0]) / (double(h[1]) * 10.0);
    printf("%-28s %7.1f cycles/iter  %6.2f ns/iter  clock %.2f GHz\n", name, cyc,
           cyc / ghz, ghz);
    (void)hipFree(d);
    (void)hipFree(c);
}

int main() {
    run<0>("v_add dep");
    run<1>("mul_hi + add dep");
    run<2>("mul24 + add dep");
    run<3>("LDS read dep");
    run<4>("ballot/popc dep");
    run<5>("enc step (chain only)");
    run<6>("enc step + word write");
    run<7>("dec step O0 (LDS table)");
    run<8>("enc step, private stack");
    run<9>("dec step, DPP quad rank");
    run<10>("dec step, mbcnt ptr");
    run<11>("dec lookup+arith only");
    run<12>("f64 fma dep (+bitcast)");
    run<13>("u32->f64 fma->u32 dep");
    run<14>("mul_lo u32 + add dep");
    run<15>("fqz range step");
    run<16>("f32 rcp div + 1 fix");
    run<17>("ballot->popc->readlane->s");
    run<18>("LDS rd->readlane->addr");
    run<19>("LDS wr + dep rd + rfl");
    run<20>("f64 recip (rcp+2fma)+use");
    run<21>("ballot/readlane step");
    return 0;
}
