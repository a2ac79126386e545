#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
__global__ void k(const uint8_t *in, uint32_t n, uint32_t *out) {
    __shared__ uint16_t ring[1024];
    const int l = threadIdx.x;
    for (int i = l; i < 1024; i += 64) ring[i] = uint16_t(i * 7 + 1);
    __syncthreads();
    // unaligned 8-byte LDS read at a 2-byte aligned address
    const uint2 v = *reinterpret_cast<const uint2 *>(__builtin_assume_aligned(ring + 1 + 2 * l, 8));
    __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void *)in, 0, n, 0x00020000);
    const uint32_t b = __builtin_amdgcn_raw_buffer_load_b8(r, l * 100, 0, 0);
    out[3 * l] = v.x; out[3 * l + 1] = v.y; out[3 * l + 2] = b;
}
int main() {
    uint8_t h[4096]; for (int i = 0; i < 4096; i++) h[i] = uint8_t(i * 13 + 5);
    uint8_t *d; uint32_t *o; (void)hipMalloc(&d, 4096); (void)hipMalloc(&o, 64 * 12);
    (void)hipMemcpy(d, h, 4096, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d, 3000u, o);
    uint32_t r[192]; (void)hipMemcpy(r, o, sizeof r, hipMemcpyDeviceToHost);
    int bad = 0;
    for (int l = 0; l < 64; l++) {
        uint32_t i = 1 + 2 * l;
        uint32_t ex = uint16_t(i * 7 + 1) | (uint32_t(uint16_t((i + 1) * 7 + 1)) << 16);
        uint32_t ey = uint16_t((i + 2) * 7 + 1) | (uint32_t(uint16_t((i + 3) * 7 + 1)) << 16);
        uint32_t eb = l * 100 < 3000 ? h[l * 100] : 0;
        if (r[3 * l] != ex || r[3 * l + 1] != ey || r[3 * l + 2] != eb) bad++;
    }
    printf("unaligned-lds+buffer-oob bad=%d (lane1: %08x %08x %u)\n", bad, r[3], r[4], r[5]);
    return 0;
}
