// v_rcp_f64 accuracy over the decoder's totals (1 .. 65536): is the raw
// hardware reciprocal close enough for q = floor(RN(rng * r + 2^-19)) to
// equal floor(rng / T) for every 32-bit rng, without a Newton step?
// Condition (fqz_decode.hip): 2^32 |r - 1/T| + 2^-21 < 2^-19.
// Also checks the bound exhaustively on a sample of rng per T.
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstdint>

__global__ void k_rcp(double *out, int n) {
    int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= n) return;
    double x = double(t + 1), r;
    asm volatile("v_rcp_f64 %0, %1" : "=v"(r) : "v"(x));
    out[t] = r;
}

int main() {
    const int n = 65536;
    double *d, *h = new double[n];
    if (hipMalloc(&d, n * sizeof(double)) != hipSuccess) return 1;
    hipLaunchKernelGGL(k_rcp, dim3(n / 256), dim3(256), 0, 0, d, n);
    if (hipMemcpy(h, d, n * sizeof(double), hipMemcpyDeviceToHost) != hipSuccess) return 1;
    long double worst = 0;
    int wt = 0, bad = 0, exact = 0;
    for (int t = 1; t <= n; t++) {
        const long double e = fabsl((long double)h[t - 1] - 1.0L / t);
        if (h[t - 1] == 1.0 / t) exact++;
        if (e > worst) { worst = e; wt = t; }
        if (ldexpl(e, 32) + ldexpl(1.0L, -21) >= ldexpl(1.0L, -19)) bad++;
    }
    // direct check: every T, rng from a stride over [2^24, 2^32) plus the
    // multiples of T and their neighbours near the top
    long long fails = 0;
    for (int t = 1; t <= n; t++) {
        const double r = h[t - 1];
        for (uint64_t k = 0; k < 4096; k++) {
            uint64_t rng = (1ull << 24) + k * ((0xFFFFFFFFull - (1ull << 24)) / 4096);
            for (int dlt = -1; dlt <= 1; dlt++) {
                uint64_t x = (rng / t) * t + dlt;
                if (x < (1ull << 24) || x > 0xFFFFFFFFull) continue;
                uint32_t q = uint32_t(fma(double(x), r, 0x1p-19));
                if (q != uint32_t(x / t)) fails++;
            }
        }
    }
    printf("rcp_f64: exact %d of %d, worst |r-1/T| = %.3Le at T=%d (%.3Lf ulp of 2^-52), bound failures %d, direct failures %lld\n",
           exact, n, worst, wt, ldexpl(worst, 52), bad, fails);
    return 0;
}
