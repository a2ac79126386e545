// crc32.hip — zlib's crc32() on the GPU (reflected CRC-32, polynomial
// 0xEDB88320), for fqzcomp5's block and index checksums (fqzcomp5.c:2268-2269,
// :2310-2311, :4443-4444, :4670-4671).
//
// The CRC register after a byte string is linear in (initial register,
// bytes) over GF(2):  raw(c, A||B) = shift(raw(c, A), |B|) ^ raw(0, B),
// where shift(v, L) runs v through L zero bytes.  So
//   k_crc_tiles   every thread takes 256 contiguous bytes (raw(0, .) with
//                 slice-by-4 tables in LDS), then the workgroup combines its
//                 256 segments in a tree: one 64 KiB tile per workgroup;
//   k_crc_tree    pairs (crc, length) are combined 256 at a time, in passes,
//                 until one is left.
// shift(v, 2^m bytes) is a 32x32 GF(2) matrix, applied as 4 lookups in its
// byte tables (4 x 256 words, built on the host for m < 40); a length is
// the product of the matrices of its set bits.
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstring>
#include <mutex>
#include <stdexcept>
#include <vector>

#include "../../include/fqz5_mi355x.h"
#include "gpu_ctx.hpp"

namespace fqz5 {

GpuCtx &gpu();
void fqz5_set_error(const char *msg);

constexpr uint32_t CRC_SEG = 256;                 // bytes per thread
constexpr uint32_t CRC_TPB = 256;                 // threads per tile
constexpr uint32_t CRC_TILE = CRC_SEG * CRC_TPB;  // 64 KiB
constexpr int CRC_SHIFTS = 40;                    // shift tables for 2^0 .. 2^39 bytes

#define DEV __device__ __forceinline__

// v run through `len` zero bytes
DEV uint32_t crc_shift(const uint32_t *__restrict__ sh, uint32_t v, uint64_t len) {
    for (int m = 0; len; m++, len >>= 1) {
        if (!(len & 1)) continue;
        const uint32_t *t = sh + size_t(m) * 1024;
        v = t[v & 255u] ^ t[256 + ((v >> 8) & 255u)] ^ t[512 + ((v >> 16) & 255u)] ^
            t[768 + (v >> 24)];
    }
    return v;
}

struct CrcJob {
    const uint8_t *in;
    uint64_t n;
    const uint32_t *tab;        // slice-by-4 byte tables, 4 x 256
    const uint32_t *sh;         // shift tables, CRC_SHIFTS x 1024
    uint32_t *tile_crc;         // per tile raw(0, tile)
    uint64_t *tile_len;
};

__global__ __launch_bounds__(CRC_TPB) void k_crc_tiles(CrcJob J) {
    __shared__ uint32_t t4[4][256];
    __shared__ uint32_t v[CRC_TPB];
    const uint32_t l = threadIdx.x;
    for (uint32_t i = l; i < 1024; i += CRC_TPB) t4[i >> 8][i & 255] = J.tab[i];
    __syncthreads();
    const uint64_t t0 = uint64_t(blockIdx.x) * CRC_TILE;
    const uint64_t s0 = t0 + uint64_t(l) * CRC_SEG;
    const uint64_t end = J.n;
    uint32_t c = 0;
    // each thread reads its own 256 bytes (16-byte loads; staging the tile
    // through LDS for coalesced loads measured slower: 68 KiB per
    // workgroup halves the waves per CU)
    if (s0 + CRC_SEG <= end && (reinterpret_cast<uintptr_t>(J.in) & 15) == 0) {
        const uint4 *p = reinterpret_cast<const uint4 *>(J.in + s0);
#pragma unroll 4
        for (int i = 0; i < int(CRC_SEG / 16); i++) {
            const uint4 w = p[i];
            const uint32_t ws[4] = {w.x, w.y, w.z, w.w};
#pragma unroll
            for (int k = 0; k < 4; k++) {   // slice-by-4 (little-endian words)
                const uint32_t x = c ^ ws[k];
                c = t4[3][x & 255u] ^ t4[2][(x >> 8) & 255u] ^ t4[1][(x >> 16) & 255u] ^
                    t4[0][x >> 24];
            }
        }
    } else {
        for (uint64_t i = s0; i < end && i < s0 + CRC_SEG; i++)
            c = t4[0][(c ^ J.in[i]) & 255u] ^ (c >> 8);
    }
    v[l] = c;
    __syncthreads();
    // tree: v[l] covers segments [l, l + 2s) after the pass with step s
    for (uint32_t s = 1; s < CRC_TPB; s <<= 1) {
        if ((l & (2 * s - 1)) == 0) {
            const uint64_t a = t0 + uint64_t(l + s) * CRC_SEG, b = t0 + uint64_t(l + 2 * s) * CRC_SEG;
            const uint64_t rlen = (b < end ? b : end) - (a < end ? a : end);
            if (rlen) v[l] = crc_shift(J.sh, v[l], rlen) ^ v[l + s];
        }
        __syncthreads();
    }
    if (l == 0) {
        J.tile_crc[blockIdx.x] = v[0];
        const uint64_t e = t0 + CRC_TILE;
        J.tile_len[blockIdx.x] = (e < end ? e : end) - t0;
    }
}

// one pass: groups of 256 (crc, len) pairs -> one pair each
__global__ __launch_bounds__(CRC_TPB) void k_crc_tree(const uint32_t *sh, const uint32_t *ci,
                                                     const uint64_t *li, uint32_t n,
                                                     uint32_t *co, uint64_t *lo) {
    __shared__ uint32_t v[CRC_TPB];
    __shared__ uint64_t L[CRC_TPB];
    const uint32_t l = threadIdx.x, i = blockIdx.x * CRC_TPB + l;
    v[l] = i < n ? ci[i] : 0u;
    L[l] = i < n ? li[i] : 0u;
    __syncthreads();
    for (uint32_t s = 1; s < CRC_TPB; s <<= 1) {
        if ((l & (2 * s - 1)) == 0 && L[l + s]) {
            v[l] = crc_shift(sh, v[l], L[l + s]) ^ v[l + s];
            L[l] += L[l + s];
        }
        __syncthreads();
    }
    if (l == 0) {
        co[blockIdx.x] = v[0];
        lo[blockIdx.x] = L[0];
    }
}

__global__ void k_crc_final(const uint32_t *sh, const uint32_t *c, const uint64_t *n, uint32_t crc,
                            uint32_t *out) {
    // crc32(crc, buf) = ~(shift(~crc, |buf|) ^ raw(0, buf))
    *out = ~(crc_shift(sh, ~crc, *n) ^ *c);
}

// ---------------------------------------------------------------------------
// host tables
namespace {

struct CrcTables {
    std::vector<uint32_t> tab, sh;
};

uint32_t gf2_apply(const uint32_t *M, uint32_t v) {   // M: images of the 32 bits
    uint32_t r = 0;
    for (int b = 0; v; b++, v >>= 1)
        if (v & 1) r ^= M[b];
    return r;
}

const CrcTables &crc_tables() {
    static CrcTables T;
    static std::once_flag once;
    std::call_once(once, [] {
        uint32_t t0[256];
        for (uint32_t i = 0; i < 256; i++) {
            uint32_t c = i;
            for (int k = 0; k < 8; k++) c = (c & 1) ? 0xEDB88320u ^ (c >> 1) : c >> 1;
            t0[i] = c;
        }
        T.tab.resize(1024);
        for (uint32_t i = 0; i < 256; i++) {
            uint32_t c = t0[i];
            T.tab[i] = c;
            for (int k = 1; k < 4; k++) {
                c = t0[c & 255u] ^ (c >> 8);
                T.tab[size_t(k) * 256 + i] = c;
            }
        }
        // one zero byte: v -> t0[v & 255] ^ (v >> 8); then squarings
        uint32_t M[32], S[32];
        for (int b = 0; b < 32; b++) {
            const uint32_t v = 1u << b;
            M[b] = t0[v & 255u] ^ (v >> 8);
        }
        T.sh.resize(size_t(CRC_SHIFTS) * 1024);
        for (int m = 0; m < CRC_SHIFTS; m++) {
            uint32_t *t = T.sh.data() + size_t(m) * 1024;
            for (int k = 0; k < 4; k++)
                for (uint32_t x = 0; x < 256; x++) t[k * 256 + x] = gf2_apply(M, x << (8 * k));
            for (int b = 0; b < 32; b++) S[b] = gf2_apply(M, M[b]);   // M <- M o M
            std::memcpy(M, S, sizeof M);
        }
    });
    return T;
}

}  // namespace

// crc32(crc, d_in[0..n)) of device bytes; the result lands in *d_out
// (device) — callers sync.  tab / sh are uploaded per call (5 KB + 160 KB).
void crc32_dev(GpuCtx &g, uint32_t crc, const uint8_t *d_in, uint64_t n, uint32_t *d_out) {
    const CrcTables &T = crc_tables();
    CrcJob J{};
    J.in = d_in;
    J.n = n;
    J.tab = g.upload(T.tab);
    J.sh = g.upload(T.sh);
    const uint64_t tiles = n ? (n + CRC_TILE - 1) / CRC_TILE : 1;
    if (tiles >= (1ull << 31)) throw GpuError("fqz5_crc32: input too large");
    J.tile_crc = g.arena.alloc_n<uint32_t>(tiles);
    J.tile_len = g.arena.alloc_n<uint64_t>(tiles);
    if (n) {
        hipLaunchKernelGGL(k_crc_tiles, dim3(uint32_t(tiles)), dim3(CRC_TPB), 0, g.stream, J);
    } else {
        g.memset0(J.tile_crc, 4);
        g.memset0(J.tile_len, 8);
    }
    FQZ5_HIP(hipGetLastError());
    uint32_t cnt = uint32_t(tiles);
    uint32_t *c = J.tile_crc;
    uint64_t *L = J.tile_len;
    while (cnt > 1) {
        const uint32_t groups = (cnt + CRC_TPB - 1) / CRC_TPB;
        uint32_t *c2 = g.arena.alloc_n<uint32_t>(groups);
        uint64_t *L2 = g.arena.alloc_n<uint64_t>(groups);
        hipLaunchKernelGGL(k_crc_tree, dim3(groups), dim3(CRC_TPB), 0, g.stream, J.sh, c, L, cnt,
                           c2, L2);
        FQZ5_HIP(hipGetLastError());
        c = c2;
        L = L2;
        cnt = groups;
    }
    hipLaunchKernelGGL(k_crc_final, dim3(1), dim3(1), 0, g.stream, J.sh, c, L, crc, d_out);
    FQZ5_HIP(hipGetLastError());
}

}  // namespace fqz5

using namespace fqz5;

extern "C" {

unsigned long fqz5_crc32(unsigned long crc, const unsigned char *buf, unsigned int len) {
    if (!buf) return 0ul;   // zlib: crc32(x, Z_NULL, len) is the initial value 0
    GpuCtx *gp = nullptr;
    try {
        GpuCtx &g = gpu();
        gp = &g;
        const uint8_t *d = g.upload(buf, len);
        uint32_t *d_out = g.arena.alloc_n<uint32_t>(1);
        crc32_dev(g, uint32_t(crc), d, len, d_out);
        uint32_t r = 0;
        g.download(&r, d_out, 1);
        g.reset();
        return r;
    } catch (const std::exception &e) {
        fqz5_set_error(e.what());
        try { if (gp) gp->reset(); } catch (...) {}
        return 0ul;
    }
}

int fqz5_crc32_dev(uint32_t crc, const uint8_t *d_buf, uint64_t len, uint32_t *out) {
    GpuCtx *gp = nullptr;
    try {
        GpuCtx &g = gpu();
        gp = &g;
        uint32_t *d_out = g.arena.alloc_n<uint32_t>(1);
        crc32_dev(g, crc, d_buf, len, d_out);
        g.download(out, d_out, 1);
        g.reset();
        return 0;
    } catch (const std::exception &e) {
        fqz5_set_error(e.what());
        try { if (gp) gp->reset(); } catch (...) {}
        return -1;
    }
}

}  // extern "C"
