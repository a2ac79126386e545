// ub2.hip — cycles per dependent step of the pieces of the O0 decode step,
// one wave, exec limited to the 4 state lanes (as in dec4_o0_body).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define N 4096
typedef __attribute__((address_space(3))) uint64_t lds64_t;

template <int T, int L = 4>
__global__ void k(uint32_t *out, uint64_t *cyc, uint32_t a, uint32_t b) {
    __shared__ uint64_t lds[4096];
    uint32_t *lds32 = reinterpret_cast<uint32_t *>(lds);
    uint4 *lds128 = reinterpret_cast<uint4 *>(lds);
    const int l = threadIdx.x;
    for (int i = l; i < 4096; i += 64) lds[i] = (uint64_t((i * 40503u) & 4095) << 32) | ((i * 2654435761u) & 4095);
    __syncthreads();
    uint32_t x = a + l, y = b, p = 0;
    uint64_t win = (uint64_t(b) << 32) | a;
    uint64_t t0 = 0, t1 = 0;
    if (l < L) {
        __builtin_amdgcn_s_waitcnt(0);
        t0 = __builtin_amdgcn_s_memtime();
#pragma unroll 16
        for (int i = 0; i < N; i++) {
            if (T == 0) x = uint32_t(lds[x & 4095]);                       // LDS b64 chain
            if (T == 1) x = x + y;                                          // v_add chain
            if (T == 2) x = __umul24(x, y) + p;                            // mad chain
            if (T == 3) x = uint32_t(win >> (x & 48)) + x;                  // 64-bit shift + add
            if (T == 4) x = __builtin_amdgcn_perm(x, y, 0x05040100u) + 1;  // perm + add
            if (T == 5) x = __builtin_amdgcn_mbcnt_lo(uint32_t(__ballot(x < y)), x);   // cmp + mbcnt
            if (T == 6) x = (x < y) ? (x >> 1) : (x + 3);                   // cmp + cndmask
            if (T == 7) {                                                   // fast path no branch
                const uint64_t e = lds[x & 4095];
                x = __umul24(uint32_t(e), x >> 12) + uint32_t(e >> 32);
            }
            if (T == 8) {                                                   // fast path + never-taken branch
                const uint64_t e = lds[x & 4095];
                x = __umul24(uint32_t(e), x >> 12) + uint32_t(e >> 32);
                if (__ballot(x == 0xdeadbeefu)) { p += x; y ^= p; }
            }
            if (T == 9) {                                                   // fast path + ~50% taken branch
                const uint64_t e = lds[x & 4095];
                x = __umul24(uint32_t(e), x >> 12) + uint32_t(e >> 32);
                if (__ballot((x & 3) == 0)) { p += x; y ^= p; }
            }
            if (T == 11) {                                                  // encoder step, cmp + cndmask
                const uint32_t xr = (x > y) ? (x >> 16) : x;
                const uint32_t q = __umulhi(xr, 0x9e3779b1u) >> (a & 7);
                x = __umul24(q, 3u) + (xr + 12345u);
            }
            if (T == 12) {                                                  // encoder step, shift from the sign of y - x
                const uint32_t s = ((y - x) >> 27) & 16u;
                const uint32_t xr = x >> s;
                const uint32_t q = __umulhi(xr, 0x9e3779b1u) >> (a & 7);
                x = __umul24(q, 3u) + (xr + 12345u);
            }
            if (T == 13) {                                                  // encoder step, v_sub_co borrow
                uint32_t d;
                const bool c = __builtin_sub_overflow(y, x, &d);
                const uint32_t xr = c ? (x >> 16) : x;
                const uint32_t q = __umulhi(xr, 0x9e3779b1u) >> (a & 7);
                x = __umul24(q, 3u) + (xr + 12345u);
            }
            if (T == 14) {                                                  // fqz range step, f64 reciprocal
                const double rd = __longlong_as_double((long long)(uint64_t(b) << 32 | a));
                const uint32_t q = uint32_t(__fma_rn(double(x), rd, 1.0 / 524288.0));
                x = q * (y | 1u);
                x <<= __builtin_clz(x | 1u) & 24u;
            }
            if (T == 15) {                                                  // fqz range step, 48-bit magic
                const uint32_t hi = __umulhi(x, a);
                const uint64_t P = uint64_t(x) * (b & 0xffffu) + hi;
                const uint32_t q = uint32_t(P >> 16);
                x = q * (y | 1u);
                x <<= __builtin_clz(x | 1u) & 24u;
            }
            if (T == 16) {                                                  // O0 step, LDS table (16 B entry)
                const uint64_t e = lds[x & 4095];
                const uint32_t xh = x >> 12;
                x = __umul24(uint32_t(e) & 4095, xh) + uint32_t(e >> 32) + 0x8000;
            }
            if (T == 17) {                                                  // O0 step, register lookup (<= 4 boundaries)
                const uint32_t sl = x & 4095;
                const uint32_t s2 = sl | (sl << 16);
                const uint32_t d1 = __builtin_amdgcn_perm(0, 0, 0) + (s2 - (a & 0x0fff0fffu)); // stand-in pk_sub
                const uint32_t d2 = s2 - (b & 0x0fff0fffu);
                const uint32_t n = __builtin_popcount(d1 & 0x80008000u) + __builtin_popcount(d2 & 0x80008000u);
                const uint32_t sel = n * 0x0202u + 0x0100u;
                const uint32_t f = __builtin_amdgcn_perm(a, b, sel) & 0xffffu;
                const uint32_t st = __builtin_amdgcn_perm(b, a, sel) & 0xffffu;
                const uint32_t xh = x >> 12;
                x = __umul24(f | 1u, xh) + (sl - st) + 0x8000;
            }
            if (T == 18) x = lds32[x & 4095];                                   // LDS b32 chain
            if (T == 19) { const uint4 v = lds128[x & 1023]; x = v.x ^ v.z; }  // LDS b128 chain
            if (T == 20) {                                                  // renorm select via perm selector
                const uint64_t m = __ballot(x < y);
                const uint32_t sel = __builtin_amdgcn_mbcnt_lo(uint32_t(m), 0x0c0c0100u >> 0) * 0x0202u;
                const uint32_t w = __builtin_amdgcn_perm(uint32_t(win >> 32), uint32_t(win), 0x0c0c0100u + sel);
                x = (x < y) ? ((x << 16) | w) : x + 7;
            }
            if (T == 21) x = __umulhi(x, y);                                 // mul_hi chain
            if (T == 22) {                                                  // enc q via f64
                const double rd = __longlong_as_double((long long)(uint64_t(b) << 32 | a));
                x = uint32_t(__fma_rn(double(x), rd, 1.0 / 1048576.0)) + y;
            }
            if (T == 23) {                                                  // cmp via VGPR sign, cndmask-free
                const uint32_t s = ((y - x) >> 27) & 16u;
                x = (x >> s) + 3;
            }
            if (T == 24) {                                                  // enc step asm, cndmask sdwa
                uint32_t q;
                asm volatile(
                    "v_cmp_gt_u32_e32 vcc, %0, %3\n\t"
                    "s_nop 1\n\t"
                    "v_cndmask_b32_sdwa %0, %0, %0, vcc dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_1\n\t"
                    "v_mul_hi_u32 %1, %0, %2\n\t"
                    "v_lshrrev_b32_sdwa %1, %5, %1 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:WORD_1 src1_sel:DWORD\n\t"
                    "v_mul_u32_u24_sdwa %1, %1, %5 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_0\n\t"
                    "v_add3_u32 %0, %0, %4, %1"
                    : "+v"(x), "=&v"(q) : "v"(0x9e3779b1u), "v"(y), "v"(12345u), "v"(0x00030003u | (a & 7) << 16) : "vcc");
            }
            if (T == 25) {                                                  // enc step C (cmp+cndmask), ref for T24
                const uint32_t w = 0x00030003u | (a & 7) << 16;
                const uint32_t xr = (x > y) ? (x >> 16) : x;
                const uint32_t q = __umulhi(xr, 0x9e3779b1u) >> (w >> 16);
                x = __umul24(q, w & 0xffffu) + (xr + 12345u);
            }
            if (T == 10) {                                                  // full renorm select chain
                const uint64_t m = __ballot(x < y);
                const uint32_t r16 = __builtin_amdgcn_mbcnt_lo(uint32_t(m), 0u) << 4;
                const uint32_t w = uint32_t(win >> r16);
                x = (x < y) ? __builtin_amdgcn_perm(x, w, 0x05040100u) : x + 7;
            }
        }
        t1 = __builtin_amdgcn_s_memtime();
    }
    out[l] = x + p + y;
    if (l == 0) cyc[L == 4 ? T : 32 + T] = t1 - t0;
}

int main() {
    uint32_t *out; uint64_t *cyc;
    hipMalloc(&out, 64 * 4); hipMalloc(&cyc, 64 * 8);
    const char *names[] = {"ds_read_b64 chain", "v_add", "mad24", "lshr_b64+add", "perm+add",
                           "cmp+mbcnt", "cmp+cndmask", "and,lshl_add,ds_read,mad", "same + never-taken branch",
                           "same + ~68%-taken branch", "renorm select (cmp,mbcnt,lshl,lshr64,perm,cndmask)",
                           "enc step cmp+cndmask", "enc step sign shift", "enc step sub borrow",
                           "fqz range step f64", "fqz range step int magic",
                           "O0 step LDS lookup + mad", "O0 step register lookup + mad",
                           "ds_read_b32 chain", "ds_read_b128 chain", "renorm select via perm selector",
                           "mul_hi chain", "enc q via f64 (cvt,fma,cvt,add)", "sign-shift (sub,lshr,and,lshr,add)",
                           "enc step asm cndmask_sdwa", "enc step C, packed cmpl|shift"};
#define RUN(T) hipLaunchKernelGGL(k<T>, dim3(1), dim3(64), 0, 0, out, cyc, 12345u, 99999u);
#define RUN64(T) hipLaunchKernelGGL((k<T, 64>), dim3(1), dim3(64), 0, 0, out, cyc, 12345u, 99999u);
    for (int rep = 0; rep < 2; rep++) {
        RUN(0) RUN(1) RUN(2) RUN(3) RUN(4) RUN(5) RUN(6) RUN(7) RUN(8) RUN(9) RUN(10) RUN(11) RUN(12) RUN(13) RUN(14) RUN(15) RUN(16) RUN(17) RUN(18) RUN(19) RUN(20) RUN(21) RUN(22) RUN(23) RUN(24) RUN(25) RUN64(11) RUN64(21) RUN64(24) RUN64(25) RUN64(16)
    }
    hipDeviceSynchronize();
    uint64_t h[64];
    hipMemcpy(h, cyc, sizeof(h), hipMemcpyDeviceToHost);
    for (int t = 0; t <= 25; t++) printf("T%-2d %-55s %7.1f cyc/step\n", t, names[t], double(h[t]) / N);
    for (int t : {11, 21, 24, 25, 16}) printf("T%-2d %-55s %7.1f cyc/step (64 lanes)\n", t, names[t], double(h[32 + t]) / N);
    return 0;
}
