// dpp_probe.hip — what the small fqz decoder's DPP sequence computes on the
// hardware (tool, not product): v_sub_u32_dpp row_shr:1 of U (bound_ctrl),
// then of that (no bound_ctrl), SW = 16 > d (signed); measured: x[i-1] - x[i].
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

__global__ void k(const uint32_t *U, uint32_t *out) {
    const uint32_t l = threadIdx.x;
    uint32_t vU = U[l], t4 = 0, vsw = l == 0 ? 0x7fffffffu : 0u, t5 = 0;
    uint64_t SW;
    asm volatile(
        "v_sub_u32_dpp %[t4], %[vU], %[vU] row_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:0\n"
        "s_nop 4\n"
        "v_sub_u32_dpp %[vsw], %[t4], %[t4] row_shr:1 row_mask:0xf bank_mask:0xf\n"
        "s_nop 4\n"
        "v_cmp_gt_i32_e64 %[SW], 16, %[vsw]\n"
        "v_mov_b32_dpp %[t5], %[vU] row_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:0\n"
        "s_nop 4\n"
        : [t4] "+v"(t4), [vsw] "+v"(vsw), [SW] "=s"(SW), [t5] "+v"(t5)
        : [vU] "v"(vU));
    out[l] = t4;
    out[64 + l] = vsw;
    out[128 + l] = t5;
    if (l == 0) {
        out[192] = uint32_t(SW);
        out[193] = uint32_t(SW >> 32);
    }
}

int main() {
    uint32_t h[64];
    const uint32_t U1[8] = {1, 2, 3, 4, 21, 22, 23, 24};   // f = 1 1 1 1 17 1 1 1
    for (int i = 0; i < 64; i++) h[i] = i < 8 ? U1[i] : 24;
    uint32_t *dU, *dO, o[200];
    hipMalloc(&dU, 256);
    hipMalloc(&dO, 800);
    hipMemcpy(dU, h, 256, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, dU, dO);
    hipMemcpy(o, dO, 800, hipMemcpyDeviceToHost);
    printf("f  :");
    for (int i = 0; i < 10; i++) printf(" %d", int(o[i]));
    printf("\nd  :");
    for (int i = 0; i < 10; i++) printf(" %d", int(o[64 + i]));
    printf("\nprv:");
    for (int i = 0; i < 10; i++) printf(" %d", int(o[128 + i]));
    printf("\nSW : %08x %08x\n", o[193], o[192]);
    return 0;
}
