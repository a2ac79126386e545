// LDS latency on one wave (tool): dependent ds_read chains of different
// shapes, timed with s_memtime around 4096 links.
//   0: ds_read_b32, every lane its own dword (contiguous, no conflicts)
//   1: ds_read_b32, a 64-lane gather of random dwords (bank conflicts)
//   2: ds_read_u8, contiguous bytes
//   3: ds_read_b32 contiguous + a ds_write_b32 of the same lanes before it
//   4: the fqz pattern: gather read, wait, then contiguous read + u8 read
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

__global__ void k(uint64_t *out, int mode, uint32_t seed) {
    __shared__ uint32_t lds[16384];
    const uint32_t l = threadIdx.x;
    for (uint32_t i = l; i < 16384; i += 64) lds[i] = (i * 2654435761u + seed) & 0x3fffu;
    __syncthreads();
    uint32_t a = l, acc = 0;
    const uint64_t t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < (1 << 18); it++) {
        if (mode == 0) {
            uint32_t x = lds[(a & 255) * 64 + l];
            acc += x;
            a = __builtin_amdgcn_readfirstlane(x) + it;
        } else if (mode == 1) {
            uint32_t x = lds[a & 16383];
            acc += x;
            a = x + l * 977 + it;
        } else if (mode == 2) {
            uint32_t x = reinterpret_cast<volatile uint8_t *>(lds)[((a & 255) * 64 + l) * 4];
            acc += x;
            a = __builtin_amdgcn_readfirstlane(x) + it;
        } else if (mode == 3) {
            lds[((a + 7) & 255) * 64 + l] = acc;
            uint32_t x = lds[(a & 255) * 64 + l];
            acc += x;
            a = __builtin_amdgcn_readfirstlane(x) + it;
        } else {
            uint32_t g = lds[(a + l * 977) & 16383];
            uint32_t b = __builtin_amdgcn_readfirstlane(g);
            uint32_t x = lds[(b & 255) * 64 + l];
            uint32_t y = reinterpret_cast<volatile uint8_t *>(lds)[((b & 255) * 64 + l) * 4 + 1];
            acc += x + y;
            a = __builtin_amdgcn_readfirstlane(x + y) + it;
        }
    }
    const uint64_t t1 = __builtin_amdgcn_s_memtime();
    if (l == 0) { out[0] = t1 - t0; out[1] = acc; }
}

int main() {
    uint64_t *d, h[2];
    hipMalloc(&d, 16);
    const char *names[] = {"b32 contiguous", "b32 gather", "u8 contiguous", "write+read", "fqz gather+model"};
    for (int m = 0; m < 5; m++) {
        hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d, m, 1u);
        hipEvent_t e0, e1;
        hipEventCreate(&e0);
        hipEventCreate(&e1);
        hipEventRecord(e0, 0);
        hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d, m, 2u);
        hipEventRecord(e1, 0);
        hipEventSynchronize(e1);
        float ms = 0;
        hipEventElapsedTime(&ms, e0, e1);
        hipMemcpy(h, d, 16, hipMemcpyDeviceToHost);
        printf("%-20s %.1f memtime units per link, %.1f ns per link (events)\n", names[m],
               double(h[0]) / (1 << 18), ms * 1e6 / (1 << 18));
    }
    return 0;
}
