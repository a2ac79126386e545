// Dependent-chain latencies on one wave (tool), in shader cycles per link
// (s_memtime ticks at the 2.4 GHz shader clock, calibrated by lds_lat).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstdlib>

#define N 4096
__global__ void k(uint64_t *out, int mode) {
    __shared__ uint32_t lds[16384];
    const uint32_t l = threadIdx.x;
    for (uint32_t i = l; i < 16384; i += 64) lds[i] = (i * 7 + 64) & 0x3fffu;
    __syncthreads();
    uint32_t v = l, sv = 1;
    double d = 3.0;
    const uint64_t t0 = __builtin_amdgcn_s_memtime();
    switch (mode) {
    case 0:   // LDS pointer chase in a lane: v_and, ds_read_b32, wait
        for (int i = 0; i < N; i++)
            asm volatile("v_and_b32 %0, 0xfffc, %0\n ds_read_b32 %0, %0\n s_waitcnt lgkmcnt(0)" : "+v"(v));
        break;
    case 1:   // VALU -> SGPR -> VALU: v_readfirstlane, s_add, v_add
        for (int i = 0; i < N; i++)
            asm volatile("v_readfirstlane_b32 %1, %0\n s_add_u32 %1, %1, 1\n v_add_u32 %0, %1, %0" : "+v"(v), "+s"(sv) : : "scc");
        break;
    case 2:   // v_cmp -> SGPR pair -> s_ff1 -> v_readlane -> v_add
        for (int i = 0; i < N; i++) {
            uint64_t m;
            asm volatile("v_cmp_gt_u32 %2, %0, 31\n s_ff1_i32_b64 %1, %2\n v_readlane_b32 %1, %0, %1\n v_add_u32 %0, %1, %0"
                         : "+v"(v), "+s"(sv), "=&s"(m));
        }
        break;
    case 3:   // the reciprocal and quotient: cvt, rcp, fma, fma, fma, cvt (f64)
        for (int i = 0; i < N; i++) {
            double a, b;
            asm volatile("v_cvt_f64_u32 %1, %0\n v_rcp_f64 %2, %1\n v_fma_f64 %1, -%1, %2, 1.0\n"
                         " v_fma_f64 %2, %2, %1, %2\n v_fma_f64 %2, %2, %2, %2\n v_cvt_u32_f64 %0, %2"
                         : "+v"(v), "=&v"(a), "=&v"(b));
        }
        break;
    case 4:   // v_mul_lo_u32 chain
        for (int i = 0; i < N; i++) asm volatile("v_mul_lo_u32 %0, %0, %0" : "+v"(v));
        break;
    case 5:   // SALU chain
        for (int i = 0; i < N; i++) asm volatile("s_add_u32 %0, %0, 1\n s_add_u32 %0, %0, 1\n s_add_u32 %0, %0, 1\n s_add_u32 %0, %0, 1" : "+s"(sv) : : "scc");
        break;
    case 6:   // VALU v_add chain (4 per link)
        for (int i = 0; i < N; i++) asm volatile("v_add_u32 %0, 1, %0\n v_add_u32 %0, 1, %0\n v_add_u32 %0, 1, %0\n v_add_u32 %0, 1, %0" : "+v"(v));
        break;
    case 7:   // independent VALU issue (4 per link)
        for (int i = 0; i < N; i++) {
            uint32_t a = 1, b = 2, c = 3, e = 4;
            asm volatile("v_add_u32 %0, 1, %0\n v_add_u32 %1, 1, %1\n v_add_u32 %2, 1, %2\n v_add_u32 %3, 1, %3" : "+v"(a), "+v"(b), "+v"(c), "+v"(e));
        }
        break;
    case 8:   // independent SALU issue (4 per link)
        for (int i = 0; i < N; i++) {
            uint32_t a = 1, b = 2, c = 3, e = 4;
            asm volatile("s_add_u32 %0, %0, 1\n s_add_u32 %1, %1, 1\n s_add_u32 %2, %2, 1\n s_add_u32 %3, %3, 1" : "+s"(a), "+s"(b), "+s"(c), "+s"(e) : : "scc");
        }
        break;
    case 9:   // SGPR written by SALU -> ds_read address via v_add -> wait -> readfirstlane
        for (int i = 0; i < N; i++)
            asm volatile("v_add_u32 %0, %1, %0\n ds_read_b32 %0, %0\n s_waitcnt lgkmcnt(0)\n v_readfirstlane_b32 %1, %0\n s_and_b32 %1, %1, 0xfffc\n v_mov_b32 %0, 0"
                         : "+v"(v), "+s"(sv) : : "scc");
        break;
    case 10:  // ds_read issued, 16 independent SALU, then the wait (latency hidden?)
        for (int i = 0; i < N; i++) {
            uint32_t a = 1;
            asm volatile("v_and_b32 %0, 0xfffc, %0\n ds_read_b32 %0, %0\n"
                         " s_add_u32 %1, %1, 1\n s_add_u32 %1, %1, 1\n s_add_u32 %1, %1, 1\n s_add_u32 %1, %1, 1\n"
                         " s_add_u32 %1, %1, 1\n s_add_u32 %1, %1, 1\n s_add_u32 %1, %1, 1\n s_add_u32 %1, %1, 1\n"
                         " s_add_u32 %1, %1, 1\n s_add_u32 %1, %1, 1\n s_add_u32 %1, %1, 1\n s_add_u32 %1, %1, 1\n"
                         " s_add_u32 %1, %1, 1\n s_add_u32 %1, %1, 1\n s_add_u32 %1, %1, 1\n s_add_u32 %1, %1, 1\n"
                         " s_waitcnt lgkmcnt(0)" : "+v"(v), "+s"(a) : : "scc");
        }
        break;
    }
    const uint64_t t1 = __builtin_amdgcn_s_memtime();
    if (l == 0) { out[0] = t1 - t0; out[1] = v + sv + uint32_t(d); }
}

int main(int argc, char **argv) {
    setvbuf(stdout, nullptr, _IONBF, 0);
    const int only = argc > 1 ? atoi(argv[1]) : -1;
    uint64_t *d, h[2];
    (void)hipMalloc(&d, 16);
    const char *names[] = {"lds chase (and+read)", "readfirstlane+sadd+vadd", "cmp+ff1+readlane+vadd",
                           "f64 rcp+3fma+2cvt", "v_mul_lo_u32", "4 dep SALU", "4 dep VALU add",
                           "4 indep VALU", "4 indep SALU", "sgpr->lds->readfirstlane", "lds + 16 SALU"};
    for (int m = 0; m < 11; m++) {
        if (only >= 0 && m != only) continue;
        hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d, m);
        hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d, m);
        (void)hipMemcpy(h, d, 16, hipMemcpyDeviceToHost);
        printf("%-26s %7.1f cycles per link\n", names[m], double(h[0]) / N);
    }
    return 0;
}
