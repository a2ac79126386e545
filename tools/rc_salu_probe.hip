// Probe: the fqz range chain (k_fqz_rc's serial part) as a scalar-unit
// recurrence against the lane-0 double-reciprocal one.  Standalone:
//   hipcc --offload-arch=gfx950 -O3 -o tools/vbuild/rc_salu_probe tools/rc_salu_probe.hip
// Prints ns/event of each form and checks both against a host loop.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstdint>
#include <vector>
#include <random>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
    std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); std::exit(1); } } while (0)

// form A: the current chain (lane 0 of a wave; records staged in LDS)
constexpr uint32_t BLK = 1024, PER = BLK / 64;
__global__ __launch_bounds__(64) void k_chain_f64(const uint4 *rec, uint32_t nev, uint32_t *qout) {
    __shared__ double s_rd[BLK];
    __shared__ uint32_t s_f[BLK];
    __shared__ uint32_t s_q[BLK];
    const int l = int(threadIdx.x);
    uint32_t rng = 0xFFFFFFFFu;
    const double bias = 1.0 / 524288.0;
    uint4 pf[PER];
    auto fetch = [&](uint32_t base) {
        for (uint32_t r = 0; r < PER; r++) {
            const uint32_t i = base + uint32_t(l) + 64u * r;
            pf[r] = i < nev ? rec[i] : make_uint4(0, 0, 0, 0);
        }
    };
    auto stage = [&]() {
        for (uint32_t r = 0; r < PER; r++) {
            const uint32_t i = uint32_t(l) + 64u * r;
            s_rd[i] = __longlong_as_double((long long)(uint64_t(pf[r].y) << 32 | pf[r].x));
            s_f[i] = pf[r].z;
        }
    };
    fetch(0);
    stage();
    __syncthreads();
    for (uint32_t base = 0; base < nev; base += BLK) {
        const uint32_t cnt = min(BLK, nev - base);
        if (base + BLK < nev) fetch(base + BLK);
        if (l == 0) {
            for (uint32_t i = 0; i < cnt; i++) {
                const uint32_t q = uint32_t(__fma_rn(double(rng), s_rd[i], bias));
                rng = q * s_f[i];
                rng <<= uint32_t(__builtin_clz(rng)) & 24u;
                s_q[i] = q;
            }
        }
        __syncthreads();
        for (uint32_t r = 0; r < PER; r++) {
            const uint32_t i = uint32_t(l) + 64u * r;
            if (base + i < nev) qout[base + i] = s_q[i];
        }
        if (base + BLK < nev) stage();
        __syncthreads();
    }
    if (l == 0) qout[nev] = rng;
}

// form B: the range in a scalar register.  Records {M lo, M hi, f, 0} with
// M = ceil(2^64 / total): q = (R * M) >> 64.  The chain stores nothing per
// event; every 64th event's range goes into a lane of a vector register
// (v_writelane) and out with a vector store, for a parallel replay.
template <int U>
__device__ __forceinline__ void put_lane(uint32_t &v, uint32_t s) {
    asm volatile("v_writelane_b32 %0, %1, %2" : "+v"(v) : "s"(s), "i"(U));
}

typedef const __attribute__((address_space(4))) uint32_t *cptr;
__device__ __forceinline__ uint32_t rc_step(uint32_t R, uint32_t ml, uint32_t mh, uint32_t f) {
    uint32_t q, t1, t2, t3;
    asm("s_mul_hi_u32 %1, %4, %5\n\t"
        "s_mul_i32 %2, %4, %6\n\t"
        "s_mul_hi_u32 %3, %4, %6\n\t"
        "s_add_u32 %1, %2, %1\n\t"
        "s_addc_u32 %0, %3, 0"
        : "=s"(q), "=&s"(t1), "=&s"(t2), "=&s"(t3) : "s"(R), "s"(ml), "s"(mh) : "scc");
    R = q * f;
    return R << (uint32_t(__builtin_clz(R)) & 24u);
}

constexpr int CH = 8;   // events per scalar-load chunk
typedef uint32_t u32x16 __attribute__((ext_vector_type(16)));
typedef const __attribute__((address_space(4))) u32x16 *cptr16;
struct Chunk { u32x16 a, b; };
__device__ __forceinline__ Chunk load_chunk(cptr p) {
    Chunk c;
    c.a = ((cptr16)p)[0];
    c.b = ((cptr16)p)[1];
    return c;
}

__global__ __launch_bounds__(64) void k_chain_salu(const uint4 *__restrict__ rec, uint32_t nev,
                                                   uint32_t *__restrict__ ck) {
    const int l = int(threadIdx.x);
    uint32_t R = 0xFFFFFFFFu;
    cptr base_p = (cptr)rec;
    const auto rrec = __builtin_amdgcn_make_buffer_rsrc((void *)rec, 0, nev * 16u, 0x00020000);
    uint32_t warm[8], sink = 0;
#pragma unroll
    for (uint32_t r = 0; r < 8; r++) warm[r] = __builtin_amdgcn_raw_buffer_load_b32(rrec, (r * 64u + l) * 128u, 0, 0);
    // nev a multiple of 4096 here
    Chunk A = load_chunk(base_p), B;
    for (uint32_t base = 0; base < nev; base += 4096) {
        uint32_t v = 0;
        // warm L2 with the next 4096 records: one dword per 128-byte line
        // (bounds-checked buffer loads; the values are folded in a block later)
#pragma unroll
        for (uint32_t r = 0; r < 8; r++) {
            sink ^= warm[r];
            warm[r] = __builtin_amdgcn_raw_buffer_load_b32(rrec, (base + 4096) * 16u + (r * 64u + l) * 128u, 0, 0);
        }
#define HALF(X, Y, U, OFF) { \
            R = rc_step(R, X.a[0], X.a[1], X.a[2]); \
            __builtin_amdgcn_sched_barrier(0); \
            Y = load_chunk(base_p + 4ull * (base + (U) * 64 + (OFF) + CH)); \
            __builtin_amdgcn_sched_barrier(0); \
            _Pragma("unroll") for (int i = 1; i < CH; i++) R = i < 4 ? rc_step(R, X.a[4 * i], X.a[4 * i + 1], X.a[4 * i + 2]) : rc_step(R, X.b[4 * i - 16], X.b[4 * i - 15], X.b[4 * i - 14]); \
            asm volatile("" :: "s"(X.a), "s"(X.b)); \
            __builtin_amdgcn_sched_barrier(0); }
        _Pragma("unroll 1") for (uint32_t g = 0; g < 64; g++) {
            v = uint32_t(l) == g ? R : v;
            _Pragma("unroll 1") for (int o = 0; o < 64; o += 2 * CH) { HALF(A, B, g, o) HALF(B, A, g, o + CH) }
        }
#undef HALF
        ck[base / 64 + l] = v;
    }
    if (l == 0) ck[nev / 64] = R;
    if (sink == 0x9e3779b9u && nev == 0u) ck[0] = sink;
}

int main(int argc, char **argv) {
    const uint32_t nev = (argc > 1 ? uint32_t(std::atoi(argv[1])) : 8u << 20) & ~4095u;
    std::mt19937_64 rg(7);
    std::vector<uint4> ra(nev), rb(nev);
    std::vector<uint32_t> t(nev), f(nev);
    for (uint32_t i = 0; i < nev; i++) {
        // totals of an adaptive model: mostly large, some small
        uint32_t tt = (rg() & 7) ? 20000 + uint32_t(rg() % 45519) : 2 + uint32_t(rg() % 300);
        uint32_t ff = 1 + uint32_t(rg() % tt);
        if (rg() & 1) ff = 1 + ff / 64;
        t[i] = tt;
        f[i] = ff;
        const double rd = 1.0 / double(tt);
        const uint64_t bits = uint64_t(__builtin_bit_cast(uint64_t, rd));
        ra[i] = make_uint4(uint32_t(bits), uint32_t(bits >> 32), ff, 0);
        const unsigned __int128 two64 = (unsigned __int128)1 << 64;
        const uint64_t M = uint64_t((two64 + tt - 1) / tt);
        rb[i] = make_uint4(uint32_t(M), uint32_t(M >> 32), ff, 0);
    }
    // host chain
    std::vector<uint32_t> hq(nev), hR(nev / 64 + 1);
    uint32_t R = 0xFFFFFFFFu;
    for (uint32_t i = 0; i < nev; i++) {
        if (i % 64 == 0) hR[i / 64] = R;
        const uint32_t q = R / t[i];
        hq[i] = q;
        R = q * f[i];
        while (R < (1u << 24)) R <<= 8;
    }
    hR[nev / 64] = R;
    uint4 *da, *db;
    uint32_t *dq, *dck;
    CK(hipMalloc(&da, nev * 16ull));
    CK(hipMalloc(&db, nev * 16ull + 4096));
    CK(hipMalloc(&dq, (nev + 1) * 4ull));
    CK(hipMalloc(&dck, (nev / 64 + 1) * 4ull));
    CK(hipMemcpy(da, ra.data(), nev * 16ull, hipMemcpyHostToDevice));
    CK(hipMemcpy(db, rb.data(), nev * 16ull, hipMemcpyHostToDevice));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (int rep = 0; rep < 3; rep++) {
        float ta, tb;
        CK(hipEventRecord(e0));
        hipLaunchKernelGGL(k_chain_f64, dim3(1), dim3(64), 0, 0, da, nev, dq);
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        CK(hipEventElapsedTime(&ta, e0, e1));
        CK(hipEventRecord(e0));
        hipLaunchKernelGGL(k_chain_salu, dim3(1), dim3(64), 0, 0, db, nev, dck);
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        CK(hipEventElapsedTime(&tb, e0, e1));
        std::vector<uint32_t> gq(nev + 1), gck(nev / 64 + 1);
        CK(hipMemcpy(gq.data(), dq, (nev + 1) * 4ull, hipMemcpyDeviceToHost));
        CK(hipMemcpy(gck.data(), dck, (nev / 64 + 1) * 4ull, hipMemcpyDeviceToHost));
        size_t bada = 0, badb = 0;
        for (uint32_t i = 0; i < nev; i++) bada += gq[i] != hq[i];
        bada += gq[nev] != hR[nev / 64];
        for (uint32_t i = 0; i <= nev / 64; i++) badb += gck[i] != hR[i];
        std::printf("nev %u  f64 chain %.3f ms (%.2f ns/ev, bad %zu)  salu chain %.3f ms (%.2f ns/ev, bad %zu)\n",
                    nev, ta, ta * 1e6 / nev, bada, tb, tb * 1e6 / nev, badb);
    }
    return 0;
}
