// rans_chain.hip — the dependent rANS chains (gfx950).
//
// A stream in the 4x16 / 32x16 formats is NX dependent chains (states) whose
// 16-bit renormalisation words are interleaved into one byte stream; that
// parallelism is fixed by the format (SURVEY.md §7 hard part (i)).  One
// 64-lane wave owns one stream and lane z owns state z; throughput comes
// from running every stream of a batch at once, so the per-step cost of a
// single chain is what these kernels minimise:
//   * symbol tables live in LDS (template TLDS) and are read with ds_read;
//   * everything that does not depend on the state (symbol bytes, table
//     entries, output bytes) is staged by all 64 lanes outside the chain;
//   * word emission / consumption order across states comes from a ballot
//     and an in-register rank, with no branches on the chain.
//
// Step geometry (rANS_static4x16pr.c:112-232, :423-821 and
// rANS_static32x16pr.c:67-758):
//   O0: step k, lane z handles byte p = NX*k + z        (valid if p < n)
//   O1: step k, lane z handles byte p = z*isz + k        (valid if k < len_z)
//       isz = n/NX, len_z = isz except the last lane, which owns the tail.
// The encoder walks k from T-1 down to 0 and emits words in descending lane
// order per step; the decoder walks k upward and consumes words in
// ascending lane order (the reference's RansDecRenorm order).
#include <hip/hip_runtime.h>
#include <cstdint>

#include "kernels.h"
#include "rans_format.hpp"

namespace fqz5 {

#define DEV __device__ __forceinline__

extern __shared__ uint4 chain_lds[];

// ===========================================================================
// Encoder
// ===========================================================================
// Per step and lane (RansEncPutSymbol, rANS_word.h:287-336), with the
// encoder symbol {rcp, x_max, bias, cmpl | shift << 16}:
//   renorm  x > x_max      => emit the low 16 bits, x >>= 16
//   encode  q = mulhi(x, rcp) >> shift;  x += bias + q * cmpl
// q < 2^21 (x <= x_max < f << 21) so q * cmpl is a 24-bit multiply.
// Steps outside the input carry the identity symbol {0, ~0, 0, 0}.
constexpr int ENC_W = 16;                  // steps staged per lane per chunk
constexpr uint32_t WRING = 2048;           // renorm-word ring (words)
constexpr uint32_t ENC_ENT_BYTES = 16384;  // S * NX * 16 (S*NX = 1024)
constexpr uint32_t ENC_RING_BYTES = 2 * (WRING + 64);
constexpr uint32_t ENC_LDS_BASE = ENC_ENT_BYTES + ENC_RING_BYTES + 256;
constexpr uint32_t ENC_TAB_LDS_MAX = 65536;

template <bool O1, int NX, bool TLDS>
static DEV void enc_body(const EncJob &J) {
    constexpr uint32_t S = uint32_t(64 / NX) * ENC_W;   // steps per chunk
    constexpr uint64_t LANES = (1ull << NX) - 1;
    uint8_t *lds = reinterpret_cast<uint8_t *>(chain_lds);
    uint4 *ent = reinterpret_cast<uint4 *>(lds);
    uint16_t *wring = reinterpret_cast<uint16_t *>(lds + ENC_ENT_BYTES);
    uint8_t *rm = lds + ENC_ENT_BYTES + ENC_RING_BYTES;
    uint4 *ltab = reinterpret_cast<uint4 *>(lds + ENC_LDS_BASE);

    const int l = int(threadIdx.x);
    const uint32_t n = J.n;
    const uint32_t A = uint32_t(J.A);
    const uint4 *gtab = reinterpret_cast<const uint4 *>(J.tab);
    if (TLDS) {
        const uint32_t ntab = O1 ? A * A : 256u;
        for (uint32_t i = l; i < ntab; i += 64) ltab[i] = gtab[i];
    }
    if (O1)
        for (int i = l; i < 256; i += 64) rm[i] = J.remap[i];
    const uint4 *tab = TLDS ? ltab : gtab;

    const uint32_t isz = n / NX;
    const uint32_t T = O1 ? n - uint32_t(NX - 1) * isz : (n + NX - 1) / NX;
    // staging: lane l stages chain zs for steps kh - sub*W - w, w < W
    const int zs = l % NX, sub = l / NX;
    const uint32_t lens = O1 ? ((zs == NX - 1) ? T : isz) : 0;
    const uint8_t *__restrict__ in = J.in;

    // b[w] = symbol of step k_w;  b[W] = context byte of step k_{W-1} (O1)
    auto load_bytes = [&](int64_t kh, uint32_t *b) {
#pragma unroll
        for (int w = 0; w <= ENC_W; w++) {
            const int64_t k = kh - int64_t(sub) * ENC_W - w;
            uint32_t v = 0;
            if (O1) {
                if (k >= 0 && k < int64_t(lens)) v = in[zs * isz + uint32_t(k)];
            } else if (w < ENC_W && k >= 0) {
                const uint64_t p = uint64_t(NX) * uint64_t(k) + zs;
                if (p < n) v = in[p];
            }
            b[w] = v;
        }
    };

    uint32_t cb[ENC_W + 1], nb[ENC_W + 1];
    int64_t kh = int64_t(T) - 1;
    load_bytes(kh, cb);
    __syncthreads();

    const int zl = l & (NX - 1);
    const bool chain = l < NX;
    const uint64_t above = (l >= 63) ? 0ull : (LANES & (~0ull << (l + 1)));
    uint32_t x = RANS_LOW_D;
    uint32_t nw = 0, flushed = 0;       // words emitted / written out
    uint16_t *out16 = reinterpret_cast<uint16_t *>(J.out_end);
    const uint4 ID = make_uint4(0, 0xffffffffu, 0, 0);

    auto step = [&](const uint4 e) {
        const uint32_t xo = x;
        const bool c = xo > e.y;
        const uint32_t xr = c ? (xo >> 16) : xo;
        const uint32_t q = __umulhi(xr, e.x) >> (e.w >> 16);
        x = __umul24(q, e.w & 0xffffu) + (xr + e.z);
        const uint64_t m = __ballot(c) & LANES;
        const uint32_t g = nw + __popcll(m & above);
        wring[(c && chain) ? (g & (WRING - 1)) : (WRING + l)] = uint16_t(xo);
        nw += __popcll(m);
    };

    for (; kh >= 0; kh -= int64_t(S)) {
        load_bytes(kh - int64_t(S), nb);              // next chunk, in flight
        // ---- stage the encoder symbols of this chunk ----
#pragma unroll
        for (int w = 0; w < ENC_W; w++) {
            const int64_t k = kh - int64_t(sub) * ENC_W - w;
            bool ok;
            if (O1) ok = k >= 0 && k < int64_t(lens);
            else ok = k >= 0 && uint64_t(NX) * uint64_t(k) + zs < n;
            uint4 e = ID;
            if (ok) {
                uint32_t idx;
                if (O1) {
                    const uint32_t ctx = k ? cb[w + 1] : 0u;
                    idx = uint32_t(rm[ctx]) * A + rm[cb[w]];
                } else {
                    idx = cb[w];
                }
                e = tab[idx];
            }
            ent[(uint32_t(sub) * ENC_W + w) * NX + zs] = e;
        }
        __syncthreads();
        // ---- the chain: entries are read 8 steps ahead ----
        uint4 E0[8], E1[8];
#pragma unroll
        for (int j = 0; j < 8; j++) E0[j] = ent[j * NX + zl];
        for (uint32_t t = 0; t < S; t += 16) {
#pragma unroll
            for (int j = 0; j < 8; j++) E1[j] = ent[(t + 8 + j) * NX + zl];
#pragma unroll
            for (int j = 0; j < 8; j++) step(E0[j]);
            if (t + 16 < S) {
#pragma unroll
                for (int j = 0; j < 8; j++) E0[j] = ent[(t + 16 + j) * NX + zl];
            }
#pragma unroll
            for (int j = 0; j < 8; j++) step(E1[j]);
        }
        __syncthreads();
        // ---- complete 512-word groups: 16-byte stores, words reversed ----
        while (nw - flushed >= 512) {
            // words f .. f+511 live at ring[f & mask ...]; memory order is
            // descending word index: lane l covers words f+504-8l .. f+511-8l
            const uint32_t base = (flushed + 504 - 8 * l) & (WRING - 1);
            const uint4 v = *reinterpret_cast<const uint4 *>(wring + base);
            uint4 r;
            r.x = __builtin_amdgcn_alignbit(v.w, v.w, 16);
            r.y = __builtin_amdgcn_alignbit(v.z, v.z, 16);
            r.z = __builtin_amdgcn_alignbit(v.y, v.y, 16);
            r.w = __builtin_amdgcn_alignbit(v.x, v.x, 16);
            reinterpret_cast<uint4 *>(out16 - int64_t(flushed) - 512)[l] = r;
            flushed += 512;
        }
#pragma unroll
        for (int w = 0; w <= ENC_W; w++) cb[w] = nb[w];
    }
    __syncthreads();
    for (uint32_t g = flushed + l; g < nw; g += 64)
        out16[-int64_t(g) - 1] = wring[g & (WRING - 1)];
    // states: state z at bytes [-(2*nw + 4*(NX-z)), +4) (RansEncFlush order)
    if (chain) {
        uint16_t *s = out16 - int64_t(nw) - 2 * int64_t(NX - l);
        s[0] = uint16_t(x);
        s[1] = uint16_t(x >> 16);
    }
    if (l == 0) *J.out_len = 2 * nw + 4 * uint32_t(NX);
}

__global__ __launch_bounds__(64) void k_rans_enc(const EncJob *jobs) {
    const EncJob J = jobs[blockIdx.x];
    const bool o1 = J.remap != nullptr;
    const uint32_t ntab = o1 ? uint32_t(J.A) * uint32_t(J.A) : 256u;
    const bool tl = ntab * 16u <= ENC_TAB_LDS_MAX;
    if (o1) {
        if (J.nx == 32) { if (tl) enc_body<true, 32, true>(J); else enc_body<true, 32, false>(J); }
        else            { if (tl) enc_body<true, 4, true>(J);  else enc_body<true, 4, false>(J); }
    } else {
        if (J.nx == 32) enc_body<false, 32, true>(J);
        else            enc_body<false, 4, true>(J);
    }
}

uint32_t enc_lds_bytes(int o1, uint32_t A) {
    const uint32_t ntab = o1 ? A * A : 256u;
    return ENC_LDS_BASE + (ntab * 16u <= ENC_TAB_LDS_MAX ? ntab * 16u : 0u);
}

// ===========================================================================
// Decoder
// ===========================================================================
// Table entries (32 bit): (f-1) << (bits+8) | (slot-start) << 8 | s, rows of
// 2^bits slots.  O0: one row, s = symbol.  O1: one row per context in
// alphabet order, s = alphabet index of the symbol, which is also the next
// step's row; alpha[s] is the output byte.  Per step (RansDecAdvance +
// RansDecRenorm, rANS_word.h:145-161, :439-448):
//   e = row[x & (2^bits-1)];  x = f*(x>>bits) + (slot-start)
//   if x < 2^15: x = x << 16 | next word
constexpr uint32_t RING_WORDS = 4096;      // words per ring copy
constexpr uint32_t SLAB_WORDS = 512;       // 64 lanes x 8 words
constexpr uint32_t DEC_OBUF = 1024;        // staged output bytes per group
constexpr uint32_t DEC_TAB_LDS_MAX = 114688;
// LDS: 4 ring copies (NX=4 window) | obuf (+64 dummy bytes) | alpha | table
constexpr uint32_t DEC_LDS_BASE = 4 * 2 * RING_WORDS + DEC_OBUF + 64 + 256;

struct DecShared {
    uint16_t *ring;     // NX=4: 4 copies, copy k holds word (i + k) at i
    uint8_t *obuf;
    uint8_t *alpha;
    uint32_t *ltab;
};

static DEV DecShared dec_shared() {
    uint8_t *lds = reinterpret_cast<uint8_t *>(chain_lds);
    DecShared d;
    d.ring = reinterpret_cast<uint16_t *>(lds);
    d.obuf = lds + 8 * RING_WORDS;
    d.alpha = d.obuf + DEC_OBUF + 64;
    d.ltab = reinterpret_cast<uint32_t *>(lds + DEC_LDS_BASE);
    return d;
}

// Lane z fetches words [s*512 + 8z, +8) of the payload (beyond the end: 0).
static DEV uint4 load_slab(const uint8_t *wbase, uint32_t nwords, uint32_t s, int z) {
    uint32_t t[4] = {0, 0, 0, 0};
    const uint32_t w0 = s * SLAB_WORDS + uint32_t(z) * 8;
#pragma unroll
    for (int b = 0; b < 8; b++) {
        const uint32_t w = w0 + b;
        uint32_t v = 0;
        if (w < nwords) v = wbase[2 * w] | (uint32_t(wbase[2 * w + 1]) << 8);
        t[b >> 1] |= v << ((b & 1) * 16);
    }
    return make_uint4(t[0], t[1], t[2], t[3]);
}

// Write one slab into the ring; COPIES = 4 keeps the shifted copies of the
// NX=4 window (copy k, position i = word i+k).
template <int COPIES>
static DEV void store_slab(uint16_t *ring, uint32_t s, int z, uint4 v) {
    const uint32_t w0 = s * SLAB_WORDS + uint32_t(z) * 8;
    *reinterpret_cast<uint4 *>(ring + (w0 & (RING_WORDS - 1))) = v;
    if (COPIES > 1) {
        const uint32_t wd[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int k = 1; k < COPIES; k++)
#pragma unroll
            for (int b = 0; b < 8; b++)
                ring[k * RING_WORDS + ((w0 + b - k) & (RING_WORDS - 1))] =
                    uint16_t(wd[b >> 1] >> ((b & 1) * 16));
    }
}

template <bool O1, int NX, bool TLDS>
static DEV void dec_body(const DecJob &J) {
    constexpr uint32_t G = DEC_OBUF / NX;     // steps per output group
    constexpr int COPIES = NX == 4 ? 4 : 1;
    constexpr uint64_t LANES = (1ull << NX) - 1;
    const DecShared sh = dec_shared();
    const int z = int(threadIdx.x);
    const uint32_t n = J.n;
    const int bits = J.bits;
    const uint32_t mask = (1u << bits) - 1;
    if (TLDS) {
        const uint32_t ntab = J.rows << bits;
        for (uint32_t i = z; i < ntab; i += 64) sh.ltab[i] = J.tab[i];
    }
    if (O1)
        for (int i = z; i < 256; i += 64) sh.alpha[i] = i < int(J.rows) ? J.alpha[i] : 0;
    const uint32_t *tab = TLDS ? sh.ltab : J.tab;

    uint32_t x = 0;
    if (z < NX) {
        const uint8_t *p = J.in + 4 * z;
        x = p[0] | (uint32_t(p[1]) << 8) | (uint32_t(p[2]) << 16) | (uint32_t(p[3]) << 24);
    }
    const uint8_t *wbase = J.in + 4 * NX;
    const uint32_t nwords = (J.in_len - 4 * uint32_t(NX)) / 2;
    uint32_t slabs = 0;
    uint4 pf = load_slab(wbase, nwords, 0, z);
    store_slab<COPIES>(sh.ring, 0, z, pf);
    pf = load_slab(wbase, nwords, 1, z);
    store_slab<COPIES>(sh.ring, 1, z, pf);
    slabs = 2;
    pf = load_slab(wbase, nwords, 2, z);

    const uint32_t isz = n / NX;
    const uint32_t lenz = O1 ? ((z == NX - 1) ? n - uint32_t(NX - 1) * isz : isz) : 0;
    const uint32_t T = O1 ? n - uint32_t(NX - 1) * isz : (n + NX - 1) / NX;
    // steps where every lane is active (then a short tail, <= NX-1 steps)
    const uint32_t Tfull = O1 ? isz : n / NX;
    uint32_t rowbase = 0;
    uint32_t ptr = 0;                        // words consumed (uniform)
    const bool lane_ok = z < NX;
    __syncthreads();

    for (uint32_t t0 = 0; t0 < T; t0 += G) {
        while (slabs * SLAB_WORDS < ptr + G * uint32_t(NX) + SLAB_WORDS &&
               slabs * SLAB_WORDS < nwords + SLAB_WORDS) {
            store_slab<COPIES>(sh.ring, slabs, z, pf);
            slabs++;
            pf = load_slab(wbase, nwords, slabs, z);
        }
        __syncthreads();
        const uint32_t t1 = (T - t0 < G) ? T : t0 + G;
        const uint32_t tf = t1 < Tfull ? t1 : (t0 > Tfull ? t0 : Tfull);
        uint32_t t = t0;
        // ---- all lanes active ----
        if (NX == 4) {
            // 4-word window at ptr, read from copy (ptr & 3) before each step
            for (; t < tf; t++) {
                const uint32_t k = ptr & 3;
                const uint2 wv = *reinterpret_cast<const uint2 *>(
                    sh.ring + k * RING_WORDS + ((ptr - k) & (RING_WORDS - 1)));
                const uint64_t win = (uint64_t(wv.y) << 32) | wv.x;
                const uint32_t e = tab[rowbase + (x & mask)];
                const uint32_t xh = x >> bits;
                const uint32_t xd = __umul24(e >> (bits + 8), xh) + xh + ((e >> 8) & mask);
                const bool c = xd < RANS_LOW_D;
                const uint64_t m = __ballot(c) & LANES;
                const uint32_t rank = __builtin_amdgcn_mbcnt_lo(uint32_t(m), 0u);
                const uint32_t w = uint32_t(win >> (rank * 16));
                x = c ? __builtin_amdgcn_perm(xd, w, 0x05040100u) : xd;
                ptr += __popcll(m);
                // lanes >= NX write to a dummy byte
                sh.obuf[lane_ok ? (t - t0) * NX + z : DEC_OBUF + z] = uint8_t(e);
                if (O1) rowbase = (e & 0xffu) << bits;
            }
        } else {
            for (; t < tf; t++) {
                const uint32_t e = tab[rowbase + (x & mask)];
                const uint32_t xh = x >> bits;
                const uint32_t xd = __umul24(e >> (bits + 8), xh) + xh + ((e >> 8) & mask);
                const bool c = lane_ok && xd < RANS_LOW_D;
                const uint64_t m = __ballot(c) & LANES;
                const uint32_t rank = __builtin_amdgcn_mbcnt_lo(uint32_t(m), 0u);
                const uint32_t w = sh.ring[(ptr + rank) & (RING_WORDS - 1)];
                x = c ? __builtin_amdgcn_perm(xd, w, 0x05040100u) : xd;
                ptr += __popcll(m);
                if (lane_ok) sh.obuf[(t - t0) * NX + z] = uint8_t(e);
                if (O1) rowbase = (e & 0xffu) << bits;
            }
        }
        // ---- tail: only some lanes active ----
        for (; t < t1; t++) {
            const bool act = lane_ok && (O1 ? t < lenz : uint32_t(NX) * t + z < n);
            uint32_t w = 0;
            const uint32_t e = tab[rowbase + (x & mask)];
            const uint32_t xh = x >> bits;
            const uint32_t xd = __umul24(e >> (bits + 8), xh) + xh + ((e >> 8) & mask);
            const bool c = act && xd < RANS_LOW_D;
            const uint64_t m = __ballot(c) & LANES;
            if (c) {
                const uint32_t rank = __builtin_amdgcn_mbcnt_lo(uint32_t(m), 0u);
                w = sh.ring[(ptr + rank) & (RING_WORDS - 1)];
            }
            ptr += __popcll(m);
            if (act) {
                x = c ? __builtin_amdgcn_perm(xd, w, 0x05040100u) : xd;
                sh.obuf[(t - t0) * NX + z] = uint8_t(e);
                if (O1) rowbase = (e & 0xffu) << bits;
            }
        }
        __syncthreads();
        // ---- write the group out, chain-major for O1 ----
        const uint32_t steps = t1 - t0, cnt = steps * uint32_t(NX);
        for (uint32_t i = z; i < cnt; i += 64) {
            uint32_t zc, tt;
            if (O1) { zc = i / steps; tt = i % steps; }
            else    { tt = i / NX; zc = i % NX; }
            const uint32_t tg = t0 + tt;
            const uint8_t v = sh.obuf[tt * NX + zc];
            if (O1) {
                const uint32_t lz = (int(zc) == NX - 1) ? n - uint32_t(NX - 1) * isz : isz;
                if (tg < lz) J.out[zc * isz + tg] = sh.alpha[v];
            } else {
                const uint32_t p = uint32_t(NX) * tg + zc;
                if (p < n) J.out[p] = v;
            }
        }
        __syncthreads();
    }
    if (z == 0) *J.status = (ptr <= nwords) ? 0 : -1;
}

__global__ __launch_bounds__(64) void k_rans_dec(const DecJob *jobs) {
    const DecJob J = jobs[blockIdx.x];
    const bool o1 = J.alpha != nullptr;
    const bool tl = (J.rows << J.bits) * 4u <= DEC_TAB_LDS_MAX;
    if (o1) {
        if (J.nx == 32) { if (tl) dec_body<true, 32, true>(J); else dec_body<true, 32, false>(J); }
        else            { if (tl) dec_body<true, 4, true>(J);  else dec_body<true, 4, false>(J); }
    } else {
        if (J.nx == 32) dec_body<false, 32, true>(J);
        else            dec_body<false, 4, true>(J);
    }
}

uint32_t dec_lds_bytes(uint32_t rows, int bits) {
    const uint32_t ntab = rows << bits;
    return DEC_LDS_BASE + (ntab * 4u <= DEC_TAB_LDS_MAX ? ntab * 4u : 0u);
}

hipError_t launch_enc(const EncJob *d_jobs, int njobs, uint32_t lds, hipStream_t s) {
    if (!njobs) return hipSuccess;
    static bool attr = false;
    if (!attr) {
        (void)hipFuncSetAttribute(reinterpret_cast<const void *>(k_rans_enc),
                                  hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
        attr = true;
    }
    hipLaunchKernelGGL(k_rans_enc, dim3(njobs), dim3(64), lds, s, d_jobs);
    return hipGetLastError();
}

hipError_t launch_dec(const DecJob *d_jobs, int njobs, uint32_t lds, hipStream_t s) {
    if (!njobs) return hipSuccess;
    static bool attr = false;
    if (!attr) {
        (void)hipFuncSetAttribute(reinterpret_cast<const void *>(k_rans_dec),
                                  hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
        attr = true;
    }
    hipLaunchKernelGGL(k_rans_dec, dim3(njobs), dim3(64), lds, s, d_jobs);
    return hipGetLastError();
}

}  // namespace fqz5
