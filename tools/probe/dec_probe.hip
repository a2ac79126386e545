// dec_probe.hip — variants of the NX=4 order-0 decode step, timed on one
// real stream (encoded by the library's own GPU path) to decide the step
// design of dec4_body.  Variant V:
//   0  production-like: LDS table, window ds_read_b64 after the table read
//   1  as 0 without the window LDS read (register window; output invalid)
//   2  as 0 without packing the symbols (output invalid)
//   3  as 0 with exec limited to the 4 state lanes around the loop
//   5  as 3 without the window LDS read (output invalid)
//   6  as 3 with the window from scalar loads of the payload
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstring>
#include <vector>
#include <random>
#include "../../fqzcomp5_amd/csrc/rans_format.hpp"
#include "../../include/fqz5_mi355x.h"

using namespace fqz5;
#define DEV __device__ __forceinline__

constexpr uint32_t RING = 4096;

template <int V>
__global__ __launch_bounds__(64) void kdec(const uint8_t *in, uint32_t in_len, const uint32_t *gtab,
                                           uint8_t *out, uint32_t n, uint64_t *cyc) {
    __shared__ uint32_t tab[4096];
    __shared__ uint16_t ring[RING + 8];
    __shared__ uint8_t obuf[1024 + 2048];
    const int l = threadIdx.x;
    for (int i = l; i < 4096; i += 64) tab[i] = gtab[i];
    uint32_t x = 1u << 16;
    if (l < 4) x = in[4 * l] | (in[4 * l + 1] << 8) | (in[4 * l + 2] << 16) | (uint32_t(in[4 * l + 3]) << 24);
    const uint16_t *w16 = reinterpret_cast<const uint16_t *>(in + 16);   // in is 2-aligned here
    const uint32_t nwords = (in_len - 16) / 2;
    uint32_t ptr = 0, filled = 0;
    const uint32_t T = n / 4;
    uint8_t *myob = obuf + (l < 4 ? l * 256 : 1024 + 64);
    uint64_t t_loop = 0;
    for (uint32_t t0 = 0; t0 + 256 <= T; t0 += 256) {
        while (filled < ptr + 2560 && filled < nwords + 512) {
            for (int i = l; i < 512; i += 64) {
                const uint32_t wi = filled + i;
                const uint16_t v = wi < nwords ? w16[wi] : 0;
                ring[wi & (RING - 1)] = v;
                if ((wi & (RING - 1)) < 8) ring[RING + (wi & (RING - 1))] = v;
            }
            filled += 512;
        }
        __syncthreads();
        const uint64_t c0 = __builtin_amdgcn_s_memtime();
        if (V < 3 || l < 4) {
        for (uint32_t tt = 0; tt < 256; tt += 16) {
            uint32_t acc[4] = {0, 0, 0, 0};
#pragma unroll
            for (int u = 0; u < 16; u++) {
                const uint32_t e = tab[x & 4095];
                __builtin_amdgcn_sched_barrier(0);
                uint64_t win;
                if (V == 1 || V == 5) win = (uint64_t(ptr) << 32) | (ptr * 7u);
                else if (V == 6) {
                    // scalar-cache window: 8 words at the dword below 2*ptr
                    typedef const uint32_t __attribute__((address_space(4))) cu32;
                    cu32 *q = (cu32 *)(uintptr_t)(w16) + (ptr >> 1);
                    const uint64_t lo = (uint64_t(q[1]) << 32) | q[0];
                    const uint64_t hi = q[2];
                    win = (ptr & 1) ? ((lo >> 16) | (hi << 48)) : lo;
                }
                else {
                    const uint2 v = *reinterpret_cast<const uint2 *>(
                        __builtin_assume_aligned(ring + (ptr & (RING - 1)), 8));
                    win = (uint64_t(v.y) << 32) | v.x;
                }
                __builtin_amdgcn_sched_barrier(0);
                const uint32_t xh = x >> 12;
                const uint32_t xd = __umul24(e >> 20, xh) + (xh + ((e >> 8) & 4095));
                const bool c = xd < 32768u;
                const uint64_t m = __ballot(c);
                const uint32_t r16 = __builtin_amdgcn_mbcnt_lo(uint32_t(m), 0u) << 4;
                const uint32_t w = uint32_t(win >> r16);
                x = c ? __builtin_amdgcn_perm(xd, w, 0x05040100u) : xd;
                ptr += uint32_t(__popcll(m & 15u));
                if (V != 2) {
                    constexpr uint32_t SEL[4] = {0x07060500u, 0x07060004u, 0x07000504u, 0x00060504u};
                    acc[u >> 2] = __builtin_amdgcn_perm(acc[u >> 2], e, SEL[u & 3]);
                }
            }
            *reinterpret_cast<uint4 *>(myob + tt) = make_uint4(acc[0], acc[1], acc[2], acc[3]);
        }
        }
        ptr = __builtin_amdgcn_readfirstlane(ptr);
        t_loop += __builtin_amdgcn_s_memtime() - c0;
        __syncthreads();
        for (uint32_t i = l; i < 1024; i += 64) out[4 * t0 + i] = obuf[(i & 3) * 256 + (i >> 2)];
        __syncthreads();
    }
    if (l == 0) { cyc[0] = t_loop; cyc[1] = ptr; }
}

// Variants 7-9 (exec = 4 state lanes):
//   7  window for step t+1 read right after step t's pointer update
//   8  next table address / next state selected from precomputed candidates
//   9  7 + 8
template <int V>
__global__ __launch_bounds__(64) void kdec2(const uint8_t *in, uint32_t in_len, const uint32_t *gtab,
                                            uint8_t *out, uint32_t n, uint64_t *cyc) {
    __shared__ uint32_t tab[4096];
    __shared__ uint16_t ring[RING + 8];
    __shared__ uint8_t obuf[1024 + 2048];
    const int l = threadIdx.x;
    for (int i = l; i < 4096; i += 64) tab[i] = gtab[i];
    uint32_t x = 1u << 16;
    if (l < 4) x = in[4 * l] | (in[4 * l + 1] << 8) | (in[4 * l + 2] << 16) | (uint32_t(in[4 * l + 3]) << 24);
    const uint16_t *w16 = reinterpret_cast<const uint16_t *>(in + 16);
    const uint32_t nwords = (in_len - 16) / 2;
    uint32_t ptr = 0, filled = 0;
    const uint32_t T = n / 4;
    uint8_t *myob = obuf + (l < 4 ? l * 256 : 1024 + 64);
    uint64_t t_loop = 0;
    const uint8_t *tb = reinterpret_cast<const uint8_t *>(tab);
    for (uint32_t t0 = 0; t0 + 256 <= T; t0 += 256) {
        while (filled < ptr + 2560 && filled < nwords + 512) {
            for (int i = l; i < 512; i += 64) {
                const uint32_t wi = filled + i;
                const uint16_t v = wi < nwords ? w16[wi] : 0;
                ring[wi & (RING - 1)] = v;
                if ((wi & (RING - 1)) < 8) ring[RING + (wi & (RING - 1))] = v;
            }
            filled += 512;
        }
        __syncthreads();
        const uint64_t c0 = __builtin_amdgcn_s_memtime();
        if (l < 4) {
            auto rw = [&](uint32_t p) {
                const uint2 v = *reinterpret_cast<const uint2 *>(
                    __builtin_assume_aligned(ring + (p & (RING - 1)), 8));
                return (uint64_t(v.y) << 32) | v.x;
            };
            uint64_t win = rw(ptr);
            uint32_t a4 = (x & 4095) << 2;           // byte address of the next entry
            for (uint32_t tt = 0; tt < 256; tt += 16) {
                uint32_t acc[4] = {0, 0, 0, 0};
#pragma unroll
                for (int u = 0; u < 16; u++) {
                    const uint32_t e = *reinterpret_cast<const uint32_t *>(tb + a4);
                    __builtin_amdgcn_sched_barrier(0);
                    if (V == 8) win = rw(ptr);
                    __builtin_amdgcn_sched_barrier(0);
                    const uint32_t xh = x >> 12;
                    const uint32_t xd = __umul24(e >> 20, xh) + (xh + ((e >> 8) & 4095));
                    const bool c = xd < 32768u;
                    const uint64_t m = __ballot(c);
                    const uint32_t r16 = __builtin_amdgcn_mbcnt_lo(uint32_t(m), 0u) << 4;
                    if (V == 7) {
                        const uint32_t w = uint32_t(win >> r16);
                        x = c ? __builtin_amdgcn_perm(xd, w, 0x05040100u) : xd;
                        a4 = (x & 4095) << 2;
                    } else {
                        // candidates: no renorm -> xd; renorm -> xd<<16 | w
                        const uint32_t sel = c ? 0x05040100u : 0x07060504u;
                        const uint32_t ad = (xd & 4095) << 2;
                        const uint64_t win4 = win << 2;
                        const uint32_t aw = uint32_t(win4 >> r16) & 0x3ffcu;
                        const uint32_t w = uint32_t(win >> r16);
                        x = __builtin_amdgcn_perm(xd, w, sel);
                        a4 = c ? aw : ad;
                    }
                    ptr += uint32_t(__popcll(m & 15u));
                    if (V != 8) win = rw(ptr);
                    constexpr uint32_t SEL[4] = {0x07060500u, 0x07060004u, 0x07000504u, 0x00060504u};
                    acc[u >> 2] = __builtin_amdgcn_perm(acc[u >> 2], e, SEL[u & 3]);
                }
                *reinterpret_cast<uint4 *>(myob + tt) = make_uint4(acc[0], acc[1], acc[2], acc[3]);
            }
        }
        ptr = __builtin_amdgcn_readfirstlane(ptr);
        t_loop += __builtin_amdgcn_s_memtime() - c0;
        __syncthreads();
        for (uint32_t i = l; i < 1024; i += 64) out[4 * t0 + i] = obuf[(i & 3) * 256 + (i >> 2)];
        __syncthreads();
    }
    if (l == 0) { cyc[0] = t_loop; cyc[1] = ptr; }
}

template <int V>
void run(const char *name, const uint8_t *d_in, uint32_t len, const uint32_t *d_tab, uint8_t *d_out,
         uint32_t n, const std::vector<uint8_t> &ref, uint64_t *d_cyc, int grid = 1,
         uint32_t dyn = 0) {
    auto kern = V >= 7 ? kdec2<V> : kdec<V>;
    (void)hipFuncSetAttribute(reinterpret_cast<const void *>(kern),
                              hipFuncAttributeMaxDynamicSharedMemorySize, 128 * 1024);
    hipEvent_t a, b;
    (void)hipEventCreate(&a); (void)hipEventCreate(&b);
    (void)hipMemset(d_out, 0, n);
    (void)hipEventRecord(a);
    hipLaunchKernelGGL(kern, dim3(grid), dim3(64), dyn, 0, d_in, len, d_tab, d_out, n, d_cyc);
    (void)hipEventRecord(b); (void)hipEventSynchronize(b);
    float ms; (void)hipEventElapsedTime(&ms, a, b);
    uint64_t cyc[2]; (void)hipMemcpy(cyc, d_cyc, 16, hipMemcpyDeviceToHost);
    std::vector<uint8_t> o(n);
    (void)hipMemcpy(o.data(), d_out, n, hipMemcpyDeviceToHost);
    const uint32_t full = (n / 4 / 256) * 256 * 4;
    const bool ok = memcmp(o.data(), ref.data(), full) == 0;
    printf("V%d g%-3d %-30s %8.2f ms  %6.2f ns/step  loop %6.1f cyc/step  ok=%d\n", V, grid, name, ms,
           ms * 1e6 / (n / 4), double(cyc[0]) / (full / 4), ok);
    (void)grid;
}

int main() {
    const uint32_t n = 43500000;
    std::vector<uint8_t> in(n);
    std::mt19937 rng(1);
    const char al[5] = {'A', 'C', 'G', 'T', 'N'};
    for (auto &c : in) { uint32_t r = rng() % 1000; c = al[r < 5 ? 4 : r % 4]; }
    std::vector<uint8_t> comp(rans_compress_bound_4x16(n, 0));
    unsigned clen = unsigned(comp.size());
    if (!rans_compress_to_4x16(in.data(), n, comp.data(), &clen, 0)) { printf("encode failed\n"); return 1; }
    // order byte, varint size, O0 frequency table, then the payload
    uint32_t usz; int p = 1 + varint_get(comp.data() + 1, comp.data() + clen, &usz);
    uint32_t F[256] = {0}, tot = 0;
    p += get_freq0(comp.data() + p, comp.data() + clen, F, &tot);
    scale_pow2(F, tot, 4096);
    std::vector<uint32_t> tab(4096);
    uint32_t x = 0;
    for (int s = 0; s < 256; s++) {
        for (uint32_t y = 0; y < F[s]; y++) tab[x + y] = ((F[s] - 1) << 20) | (y << 8) | s;
        x += F[s];
    }
    const uint32_t len = clen - p;
    uint8_t *d_in; uint32_t *d_tab; uint8_t *d_out; uint64_t *d_cyc;
    (void)hipMalloc(&d_in, len + 64); (void)hipMalloc(&d_tab, 16384);
    (void)hipMalloc(&d_out, n); (void)hipMalloc(&d_cyc, 16);
    (void)hipMemcpy(d_in, comp.data() + p, len, hipMemcpyHostToDevice);
    (void)hipMemcpy(d_tab, tab.data(), 16384, hipMemcpyHostToDevice);
    printf("n=%u comp=%u payload=%u\n", n, clen, len);
    for (int rep = 0; rep < 3; rep++) {
        run<3>("exec4: window after table read", d_in, len, d_tab, d_out, n, in, d_cyc);
        run<5>("exec4: no window read", d_in, len, d_tab, d_out, n, in, d_cyc);
        run<7>("exec4: window a step ahead", d_in, len, d_tab, d_out, n, in, d_cyc);
        run<8>("exec4: candidates, window after", d_in, len, d_tab, d_out, n, in, d_cyc);
        run<9>("exec4: candidates + step ahead", d_in, len, d_tab, d_out, n, in, d_cyc);
    }
    return 0;
}
