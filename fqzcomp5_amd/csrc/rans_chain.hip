// rans_chain.hip — the dependent rANS chains (gfx950).
//
// A stream in the 4x16 / 32x16 formats is NX dependent chains (states) whose
// 16-bit renormalisation words are interleaved into one byte stream; that
// parallelism is fixed by the format (SURVEY.md §7 hard part (i)).  One
// 64-lane wave owns one stream and lane z owns state z; throughput comes
// from running every stream of a batch at once, so the per-step latency of
// a single chain is what these kernels minimise.  A wave64 VALU instruction
// costs at least 4 cycles whatever its exec mask, so the rule is: the fewest
// instructions per step on the chain, everything else amortised over
// chunks of steps and done by all 64 lanes (measured with tools/ubench.hip
// and tools/chain_probe.hip):
//   * symbol tables live in LDS and are read with ds_read;
//   * symbol bytes are fetched with bounds-checked buffer loads (reads past
//     the end return 0), one chunk ahead, by all lanes;
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
#ifdef FQZ5_CHAIN_PROBE
__device__ uint64_t g_probe[8];
__device__ uint64_t g_jobt[512][8];   // per decode job: start, end (100 MHz), cycles, info, loop cycles, loop steps, rows|nx<<16|mode<<24, in_len
#endif

// Raw buffer over [p, p+n): loads past n return 0, stores past n are dropped.
static DEV __amdgpu_buffer_rsrc_t buf(const void *p, uint32_t n) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void *>(p), 0, n, 0x00020000);
}
static DEV uint32_t ld8(__amdgpu_buffer_rsrc_t r, uint32_t off) {
    return __builtin_amdgcn_raw_buffer_load_b8(r, off, 0, 0);
}
static DEV void st8(__amdgpu_buffer_rsrc_t r, uint32_t off, uint32_t v) {
    __builtin_amdgcn_raw_buffer_store_b8(uint8_t(v), r, off, 0, 0);
}

// ===========================================================================
// Encoder
// ===========================================================================
// Per step and lane (RansEncPutSymbol, rANS_word.h:287-336), with the
// encoder symbol {rcp, x_max, bias, cmpl | shift << 16}:
//   renorm  x > x_max      => emit the low 16 bits, x >>= 16
//   encode  q = mulhi(x, rcp) >> shift;  x += bias + q * cmpl
// q < 2^21 (x <= x_max < f << 21) so q * cmpl is a 24-bit multiply.
// Steps outside the input carry the identity symbol {0, ~0, 0, 0}.
//
// Encoding is split so that the only sequential work is the bare chain:
//   1. k_enc_chain   one wave per stream runs the NX chains (7 VALU ops and
//                    one LDS read per step) and checkpoints the states at
//                    every chunk of S = 1024/NX steps;
//   2. k_enc_replay  every chunk of every stream is re-run from its
//                    checkpoint in parallel (64/NX chunks per wave), counting
//                    the renormalisation words each chunk emits;
//   3. k_enc_scan    per stream, exclusive scan of the chunk word counts;
//   4. k_enc_replay  again, writing every word straight to its final place
//                    (and the final states after the last chunk).
// Chunks are aligned to S from step 0: chunk j holds steps [jS, jS+S) and is
// processed in descending j; checkpoint c (= jtop - j) is the state before
// chunk j.  The word order is the reference's: steps from the top of the
// input down, within a step the lanes in descending order, the stream
// growing downward from out_end.
constexpr uint32_t ENC_ENT = 1024;                        // entries per chunk
constexpr uint32_t ENC_ENT_BYTES = (ENC_ENT + 512) * 16;  // + chain over-read
constexpr uint32_t ENC_LDS_BASE = ENC_ENT_BYTES + 256;    // + remap
constexpr int REPLAY_THREADS = 1024;
constexpr int ENC_W = 16;                    // replay: steps per byte batch

template <int NX> constexpr uint32_t enc_chunk() { return ENC_ENT / NX; }

// The reciprocal of every frequency (RansEncSymbolInit, rANS_word.h:201-272:
// ceil(2^(s+31) / f), s = ceil(log2 f); ~0 below 2) into LDS, by `nthr`
// threads; the caller synchronises.
static DEV void enc_rcp_lds(uint32_t *rc, int tid, int nthr) {
    for (int f = tid; f < int(ENC_RCP_N); f += nthr) {
        if (f < 2) { rc[f] = ~0u; continue; }
        const uint32_t s = 32u - uint32_t(__builtin_clz(uint32_t(f) - 1u));
        rc[f] = uint32_t(((1ull << (s + 31)) + uint64_t(f) - 1) / uint64_t(f));
    }
}
// a compact entry (freq | start << 13) as the 16-B encoder symbol
// (make_encsym, rans_format.hpp)
static DEV uint4 enc_expand(uint32_t c, int bits, const uint32_t *rc) {
    const uint32_t f = c & 0x1fffu, start = c >> 13;
    uint4 e;
    e.y = ((RANS_LOW_D >> bits) << 16) * f - 1u;
    uint32_t sh = 0;
    e.x = rc[f];
    if (f < 2) {
        e.z = start + (1u << bits) - 1u;
    } else {
        sh = 31u - uint32_t(__builtin_clz(f - 1u));
        e.z = start;
    }
    e.w = (((1u << bits) - f) & 0xffffu) | (sh << 16);
    return e;
}

template <bool O1, int NX>
static DEV uint32_t enc_steps(uint32_t n) {
    return O1 ? n - uint32_t(NX - 1) * (n / NX) : (n + NX - 1) / NX;
}

template <bool O1, int NX, bool TLDS>
static DEV void chain_body(const EncJob &J) {
    constexpr uint32_t S = enc_chunk<NX>();
    constexpr int R = int(ENC_ENT / 64);           // entries staged per lane
    uint8_t *lds = reinterpret_cast<uint8_t *>(chain_lds);
    uint4 *ent = reinterpret_cast<uint4 *>(lds);
    uint8_t *rm = lds + ENC_ENT_BYTES;
    uint4 *ltab = reinterpret_cast<uint4 *>(lds + ENC_LDS_BASE);
    uint32_t *rc = reinterpret_cast<uint32_t *>(lds + ENC_LDS_BASE);   // (!TLDS: compact table)

    const int l = int(threadIdx.x);
    const uint32_t n = J.n;
    const uint32_t A = uint32_t(J.A);
    const uint4 *gtab = reinterpret_cast<const uint4 *>(J.tab);
    const uint32_t *ctab = reinterpret_cast<const uint32_t *>(J.tab);
    if (TLDS) {
        const uint32_t ntab = O1 ? A * A : 256u;
        for (uint32_t i = l; i < ntab; i += 64) ltab[i] = gtab[i];
    } else {
        enc_rcp_lds(rc, l, 64);
    }
    if (O1)
        for (int i = l; i < 256; i += 64) rm[i] = J.remap[i];
    const uint4 *tab = ltab;

    const uint32_t isz = n / NX;
    const uint32_t T = enc_steps<O1, NX>(n);
    const uint32_t jtop = (T - 1) / S;
    const auto in = buf(J.in, n);

    // Staged entry r of lane l is i = l + 64r: O0 (step kk, lane z) with
    // i = kk*NX + z; O1 chain-major, i = z*S + kk.  It lands at
    // ent[(S-1-kk)*NX + z] so that the chain reads ascending addresses.
    uint32_t sb[R], cb[R];
    auto issue = [&](uint32_t j) {
#pragma unroll
        for (int r = 0; r < R; r++) {
            const uint32_t i = uint32_t(l) + 64u * r;
            if (O1) {
                const uint32_t z = i / S, k = j * S + i % S;
                sb[r] = ld8(in, z * isz + k);
                cb[r] = ld8(in, z * isz + k - 1u);
            } else {
                sb[r] = ld8(in, NX * S * j + i);
            }
        }
    };
    const uint4 ID = make_uint4(0, 0xffffffffu, 0, 0);
    auto stage = [&](uint32_t j) {
#pragma unroll
        for (int r = 0; r < R; r++) {
            const uint32_t i = uint32_t(l) + 64u * r;
            uint32_t z, kk, idx;
            bool ok;
            if (O1) {
                z = i / S;
                kk = i % S;
                const uint32_t k = j * S + kk;
                ok = k < ((z == NX - 1) ? T : isz);
                const uint32_t ctx = k ? cb[r] : 0u;
                idx = uint32_t(rm[ctx]) * A + rm[sb[r]];
            } else {
                z = i % NX;
                kk = i / NX;
                ok = NX * S * j + i < n;
                idx = sb[r];
            }
            uint4 e = TLDS ? tab[ok ? idx : 0u] : enc_expand(ctab[ok ? idx : 0u], J.bits, rc);
            if (!ok) e = ID;
            ent[(S - 1 - kk) * NX + z] = e;
        }
    };

    issue(jtop);
    __syncthreads();
    stage(jtop);

    const int zl = l & (NX - 1);
    const bool writer = l < NX;
    uint32_t x = RANS_LOW_D;
    uint32_t *ck = J.ck + zl;
    const uint4 *ep = ent + zl;

    auto step = [&](const uint4 e) {
        const bool c = x > e.y;
        const uint32_t xr = c ? (x >> 16) : x;
        const uint32_t q = __umulhi(xr, e.x) >> (e.w >> 16);
        x = __umul24(q, e.w & 0xffffu) + (xr + e.z);
    };

#ifdef FQZ5_CHAIN_PROBE
    uint64_t t_stage = 0, t_chain = 0;
#endif
    for (int32_t j = int32_t(jtop); j >= 0; j--) {
        __syncthreads();
#ifdef FQZ5_CHAIN_PROBE
        const uint64_t tp0 = __builtin_amdgcn_s_memtime();
#endif
        if (writer) *ck = x;
        ck += NX;
        if (j > 0) issue(uint32_t(j - 1));
        // ---- the chain: entries of block b+1 are read while block b runs
        // (at most 16 reads in flight, within what lgkmcnt can track);
        // sched_barrier keeps the compiler from batching all reads up front
        // The reads of block b+1 are issued after the first step of block b:
        // the compiler's (conservative) lgkmcnt(0) before that step then
        // only waits for block b's own reads, issued a block earlier.  (All
        // 64 lanes run it: limiting exec to the NX state lanes measured
        // slower here, unlike the decoder.)
        constexpr int CB = 8;
        uint4 E[2][CB];
#pragma unroll
        for (int i = 0; i < CB; i++) E[0][i] = ep[i * NX];
#pragma unroll
        for (uint32_t b = 0; b < S / CB; b++) {
            step(E[b & 1][0]);
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int i = 0; i < CB; i++) E[(b + 1) & 1][i] = ep[(CB * (b + 1) + i) * NX];
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int i = 1; i < CB; i++) step(E[b & 1][i]);
            __builtin_amdgcn_sched_barrier(0);
        }
        __syncthreads();
#ifdef FQZ5_CHAIN_PROBE
        const uint64_t tp1 = __builtin_amdgcn_s_memtime();
        t_chain += tp1 - tp0;
#endif
        if (j > 0) stage(uint32_t(j - 1));
#ifdef FQZ5_CHAIN_PROBE
        t_stage += __builtin_amdgcn_s_memtime() - tp1;
#endif
    }
    if (writer) *ck = x;                              // checkpoint nchunks
#ifdef FQZ5_CHAIN_PROBE
    if (l == 0) { g_probe[0] += t_stage; g_probe[1] += t_chain; }
#endif
}

// NX = 4 with the table in LDS (the long chains): a workgroup of two waves.
// Wave 0 runs the chain over one entry buffer while wave 1 loads the next
// chunk's symbols and stages its entries into the other; they meet at one
// barrier per chunk.  The staging (~7 cycles per step when the chain wave
// did it between chunks) then costs the chain nothing: the waves sit on
// different SIMDs and the staging finishes well within the chain's time.
constexpr uint32_t ENC_BUF_ENT = ENC_ENT + 512;                // entries per buffer, + chain over-read
constexpr uint32_t ENC_2W_BASE = 2 * ENC_BUF_ENT * 16 + 256;   // 2 buffers + remap

template <bool O1>
static DEV void chain_body_2w(const EncJob &J) {
    constexpr int NX = 4;
    constexpr uint32_t S = enc_chunk<NX>();               // 256 steps per chunk
    constexpr int R = int(ENC_ENT / 64);                  // 16 entries staged per lane
    constexpr int CB = 8;
    uint8_t *lds = reinterpret_cast<uint8_t *>(chain_lds);
    uint4 *entb = reinterpret_cast<uint4 *>(lds);
    uint8_t *rm = lds + 2 * ENC_BUF_ENT * 16;
    uint4 *ltab = reinterpret_cast<uint4 *>(lds + ENC_2W_BASE);

    const int tid = int(threadIdx.x);
    const int wave = tid >> 6, l = tid & 63;
    const uint32_t n = J.n;
    const uint32_t A = uint32_t(J.A);
    {
        const uint4 *gtab = reinterpret_cast<const uint4 *>(J.tab);
        const uint32_t ntab = O1 ? A * A : 256u;
        for (uint32_t i = tid; i < ntab; i += 128) ltab[i] = gtab[i];
    }
    if (O1)
        for (int i = tid; i < 256; i += 128) rm[i] = J.remap[i];
    __syncthreads();

    const uint32_t isz = n / NX;
    const uint32_t T = enc_steps<O1, NX>(n);
    const uint32_t jtop = (T - 1) / S;
    const auto in = buf(J.in, n);

    // wave 1: chunk j's entries into dst (as chain_body's issue + stage)
    auto stage = [&](uint32_t j, uint4 *dst) {
        uint32_t sb[R], cb[R];
#pragma unroll
        for (int r = 0; r < R; r++) {
            const uint32_t i = uint32_t(l) + 64u * r;
            if (O1) {
                const uint32_t z = i / S, k = j * S + i % S;
                sb[r] = ld8(in, z * isz + k);
                cb[r] = ld8(in, z * isz + k - 1u);
            } else {
                sb[r] = ld8(in, NX * S * j + i);
            }
        }
        const uint4 ID = make_uint4(0, 0xffffffffu, 0, 0);
#pragma unroll
        for (int r = 0; r < R; r++) {
            const uint32_t i = uint32_t(l) + 64u * r;
            uint32_t z, kk, idx;
            bool ok;
            if (O1) {
                z = i / S;
                kk = i % S;
                const uint32_t k = j * S + kk;
                ok = k < ((z == NX - 1) ? T : isz);
                idx = uint32_t(rm[k ? cb[r] : 0u]) * A + rm[sb[r]];
            } else {
                z = i % NX;
                kk = i / NX;
                ok = NX * S * j + i < n;
                idx = sb[r];
            }
            uint4 e = ltab[ok ? idx : 0u];
            if (!ok) e = ID;
            dst[(S - 1 - kk) * NX + z] = e;
        }
    };

    if (wave == 1) stage(jtop, entb);
    __syncthreads();

    const int zl = l & (NX - 1);
    const bool writer = wave == 0 && l < NX;
    uint32_t x = RANS_LOW_D;
    uint32_t *ck = J.ck + zl;
    auto step = [&](const uint4 e) {
        const bool c = x > e.y;
        const uint32_t xr = c ? (x >> 16) : x;
        const uint32_t q = __umulhi(xr, e.x) >> (e.w >> 16);
        x = __umul24(q, e.w & 0xffffu) + (xr + e.z);
    };
#ifdef FQZ5_CHAIN_PROBE
    uint64_t t_chain = 0;
#endif
    for (int32_t j = int32_t(jtop); j >= 0; j--) {
        const uint32_t cur = (jtop - uint32_t(j)) & 1u;
        if (wave == 0) {
#ifdef FQZ5_CHAIN_PROBE
            const uint64_t tp0 = __builtin_amdgcn_s_memtime();
#endif
            if (writer) *ck = x;
            ck += NX;
            const uint4 *ep = entb + cur * ENC_BUF_ENT + zl;
            uint4 E[2][CB];
#pragma unroll
            for (int i = 0; i < CB; i++) E[0][i] = ep[i * NX];
#pragma unroll
            for (uint32_t b = 0; b < S / CB; b++) {
                step(E[b & 1][0]);
                __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                for (int i = 0; i < CB; i++) E[(b + 1) & 1][i] = ep[(CB * (b + 1) + i) * NX];
                __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                for (int i = 1; i < CB; i++) step(E[b & 1][i]);
                __builtin_amdgcn_sched_barrier(0);
            }
#ifdef FQZ5_CHAIN_PROBE
            t_chain += __builtin_amdgcn_s_memtime() - tp0;
#endif
        } else if (j > 0) {
            stage(uint32_t(j) - 1u, entb + (cur ^ 1u) * ENC_BUF_ENT);
        }
        __syncthreads();
    }
    if (writer) *ck = x;                              // checkpoint nchunks
#ifdef FQZ5_CHAIN_PROBE
    if (tid == 0) g_probe[1] += t_chain;
#endif
}

__global__ __launch_bounds__(128) void k_enc_chain2w(const EncJob *jobs) {
    const EncJob J = jobs[blockIdx.x];
    if (J.remap != nullptr) chain_body_2w<true>(J);
    else                    chain_body_2w<false>(J);
}

__global__ __launch_bounds__(64) void k_enc_chain(const EncJob *jobs) {
    const EncJob J = jobs[blockIdx.x];
    const bool o1 = J.remap != nullptr;
    const uint32_t ntab = o1 ? uint32_t(J.A) * uint32_t(J.A) : 256u;
    const bool tl = ntab * 16u <= ENC_TAB_LDS_MAX;
    if (o1) {
        if (J.nx == 32) { if (tl) chain_body<true, 32, true>(J); else chain_body<true, 32, false>(J); }
        else            { if (tl) chain_body<true, 4, true>(J);  else chain_body<true, 4, false>(J); }
    } else {
        if (J.nx == 32) chain_body<false, 32, true>(J);
        else            chain_body<false, 4, true>(J);
    }
}

// Replay of chunks c0 .. c0 + 16*(64/NX) - 1 of one stream; wave w, lane l
// re-runs state z = l % NX of chunk c0 + w*(64/NX) + l/NX from its
// checkpoint.  Without EMIT it stores the chunk's word count; with EMIT the
// counts have become exclusive offsets and the words are written.
template <bool O1, int NX, bool TLDS, bool EMIT>
static DEV void replay_body(const EncJob &J, uint32_t c0) {
    constexpr uint32_t S = enc_chunk<NX>();
    constexpr uint32_t G = 64 / NX;
    constexpr uint64_t LANES = (NX == 32) ? 0xffffffffull : ((1ull << NX) - 1);
    uint8_t *lds = reinterpret_cast<uint8_t *>(chain_lds);
    uint8_t *rm = lds;
    uint4 *ltab = reinterpret_cast<uint4 *>(lds + 256);
    uint32_t *rc = reinterpret_cast<uint32_t *>(lds + 256);   // (!TLDS: compact table)
    const int tid = int(threadIdx.x);
    const uint32_t n = J.n;
    const uint32_t A = uint32_t(J.A);
    const uint4 *gtab = reinterpret_cast<const uint4 *>(J.tab);
    const uint32_t *ctab = reinterpret_cast<const uint32_t *>(J.tab);
    if (TLDS) {
        const uint32_t ntab = O1 ? A * A : 256u;
        for (uint32_t i = tid; i < ntab; i += REPLAY_THREADS) ltab[i] = gtab[i];
    } else {
        enc_rcp_lds(rc, tid, REPLAY_THREADS);
    }
    if (O1)
        for (int i = tid; i < 256; i += REPLAY_THREADS) rm[i] = J.remap[i];
    __syncthreads();
    const uint4 *tab = ltab;

    const int l = tid & 63;
    const uint32_t c = c0 + uint32_t(tid >> 6) * G + uint32_t(l / NX);
    if (c0 + uint32_t(tid >> 6) * G >= J.nchunks) return;   // whole wave idle
    const int z = l % NX;
    const int gsh = (l / NX) * NX;
    const bool act = c < J.nchunks;
    const uint32_t isz = n / NX;
    const uint32_t T = enc_steps<O1, NX>(n);
    const uint32_t lens = O1 ? ((z == NX - 1) ? T : isz) : 0;
    const uint8_t *__restrict__ in = J.in;
    uint32_t x = act ? J.ck[uint64_t(c) * NX + z] : RANS_LOW_D;
    // chunk c covers steps [j*S, j*S + S) with j = nchunks - 1 - c
    const int64_t khi = (int64_t(J.nchunks) - int64_t(c)) * S - 1;
    const uint32_t base = (EMIT && act) ? J.cnt[c] : 0u;
    uint32_t cnt = 0;
    uint16_t *out16 = reinterpret_cast<uint16_t *>(J.out_end);

    for (uint32_t t0 = 0; t0 < S; t0 += ENC_W) {
        uint32_t b[ENC_W + 1];
        bool ok[ENC_W];
#pragma unroll
        for (int w = 0; w <= ENC_W; w++) {
            const int64_t k = khi - int64_t(t0) - w;
            uint32_t v = 0;
            bool o;
            if (O1) {
                o = act && k >= 0 && k < int64_t(lens);
                if (o) v = in[z * isz + uint32_t(k)];
            } else {
                o = act && w < ENC_W && k >= 0 && uint64_t(NX) * uint64_t(k) + z < n;
                if (o) v = in[uint64_t(NX) * uint64_t(k) + z];
            }
            b[w] = v;
            if (w < ENC_W) ok[w] = o;
        }
#pragma unroll
        for (int w = 0; w < ENC_W; w++) {
            uint4 e = make_uint4(0, 0xffffffffu, 0, 0);
            if (ok[w]) {
                const int64_t k = khi - int64_t(t0) - w;
                const uint32_t idx = O1 ? uint32_t(rm[k ? b[w + 1] : 0u]) * A + rm[b[w]] : b[w];
                e = TLDS ? tab[idx] : enc_expand(ctab[idx], J.bits, rc);
            }
            const uint32_t xo = x;
            const bool cf = xo > e.y;
            const uint32_t xr = cf ? (xo >> 16) : xo;
            const uint32_t q = __umulhi(xr, e.x) >> (e.w >> 16);
            x = __umul24(q, e.w & 0xffffu) + (xr + e.z);
            const uint64_t gm = (__ballot(cf) >> gsh) & LANES;
            if (EMIT && cf)
                out16[-int64_t(base + cnt + uint32_t(__popcll(gm >> (z + 1)))) - 1] = uint16_t(xo);
            cnt += uint32_t(__popcll(gm));
        }
    }
    if (!EMIT) {
        if (act && z == 0) J.cnt[c] = cnt;
    } else if (act && c == J.nchunks - 1) {
        // states: state z at bytes [-(2*nw + 4*(NX-z)), +4) (RansEncFlush order)
        const uint32_t tot = base + cnt;
        uint16_t *s = out16 - int64_t(tot) - 2 * int64_t(NX - z);
        s[0] = uint16_t(x);
        s[1] = uint16_t(x >> 16);
        if (z == 0) *J.out_len = 2 * tot + 4 * uint32_t(NX);
    }
}

template <bool EMIT>
__global__ __launch_bounds__(REPLAY_THREADS) void k_enc_replay(const EncJob *jobs,
                                                              const uint2 *items) {
    const uint2 it = items[blockIdx.x];
    const EncJob J = jobs[it.x];
    const bool o1 = J.remap != nullptr;
    const uint32_t ntab = o1 ? uint32_t(J.A) * uint32_t(J.A) : 256u;
    const bool tl = ntab * 16u <= ENC_TAB_LDS_MAX;
    if (o1) {
        if (J.nx == 32) { if (tl) replay_body<true, 32, true, EMIT>(J, it.y); else replay_body<true, 32, false, EMIT>(J, it.y); }
        else            { if (tl) replay_body<true, 4, true, EMIT>(J, it.y);  else replay_body<true, 4, false, EMIT>(J, it.y); }
    } else {
        if (J.nx == 32) replay_body<false, 32, true, EMIT>(J, it.y);
        else            replay_body<false, 4, true, EMIT>(J, it.y);
    }
}

// Exclusive scan of one stream's chunk word counts, in place.
__global__ __launch_bounds__(1024) void k_enc_scan(const EncJob *jobs) {
    __shared__ uint32_t part[1024];
    const EncJob J = jobs[blockIdx.x];
    const uint32_t nc = J.nchunks, t = threadIdx.x;
    const uint32_t per = (nc + 1023) / 1024;
    const uint32_t b = min(nc, t * per), e = min(nc, b + per);
    uint32_t s = 0;
    for (uint32_t i = b; i < e; i++) s += J.cnt[i];
    part[t] = s;
    __syncthreads();
    for (uint32_t d = 1; d < 1024; d <<= 1) {
        const uint32_t v = t >= d ? part[t - d] : 0u;
        __syncthreads();
        part[t] += v;
        __syncthreads();
    }
    uint32_t run = part[t] - s;
    for (uint32_t i = b; i < e; i++) {
        const uint32_t v = J.cnt[i];
        J.cnt[i] = run;
        run += v;
    }
}

uint32_t enc_lds_bytes(int o1, uint32_t A) {
    const uint32_t ntab = o1 ? A * A : 256u;
    return ENC_LDS_BASE + (ntab * 16u <= ENC_TAB_LDS_MAX ? ntab * 16u : ENC_RCP_N * 4u);
}

// Jobs that run k_enc_chain2w (NX=4, table in LDS) and their LDS.
bool enc_chain_2w(int o1, int nx, uint32_t A) {
    const uint32_t ntab = o1 ? A * A : 256u;
    return nx == 4 && ntab * 16u <= ENC_TAB_LDS_MAX;
}
uint32_t enc_2w_lds_bytes(int o1, uint32_t A) {
    return ENC_2W_BASE + (o1 ? A * A : 256u) * 16u;
}

uint32_t enc_replay_lds_bytes(int o1, uint32_t A) {
    const uint32_t ntab = o1 ? A * A : 256u;
    return 256u + (ntab * 16u <= ENC_TAB_LDS_MAX ? ntab * 16u : ENC_RCP_N * 4u);
}

// ===========================================================================
// Decoder
// ===========================================================================
// Per step (RansDecAdvance + RansDecRenorm, rANS_word.h:145-161, :439-448):
//   slot = x & (2^bits-1);  x = f*(x>>bits) + slot - start
//   if x < 2^15: x = x << 16 | next word
// Tables (kernels.h dec_table_mode): LDS/GLOBAL hold per slot the u32
// (f-1) << 16 | (slot-start) and the u8 symbol; SPLIT (O1 tables too big
// for that in LDS) holds the u8 symbol per slot and (f-1) << 16 | start per
// (context, symbol), two dependent LDS reads.  For O1 the symbol is the
// alphabet index, which is also the next step's row; alpha[] maps it back.
//
// Words are staged from global memory into an LDS ring in slabs of 512.
// NX=4: each step reads the 4-word window at the (uniform) read pointer
// with one unaligned ds_read_b64 issued a step ahead, and lane z takes the
// word at its rank among the renormalising lanes, from a 64-bit shift.
// NX=32: the renormalising lanes read ring[ptr + rank] directly.
constexpr uint32_t RING_WORDS = 4096;
constexpr uint32_t SLAB_WORDS = 512;                      // 64 lanes x 8 words
constexpr uint32_t DEC_OBUF = 1024;                       // output bytes / group
constexpr uint32_t DEC_RING_BYTES = RING_WORDS * 2 + 16;  // + wrap copy
constexpr uint32_t DEC_OBUF_BYTES = DEC_OBUF + 2048 + 128;  // + idle-lane sink
constexpr uint32_t DEC_LDS_BASE = DEC_RING_BYTES + DEC_OBUF_BYTES + 256;
static_assert(DEC_LDS_BASE % 16 == 0, "table alignment");

// A 32-bit LDS byte address as a pointer (an unaligned 8-byte window is read
// with one ds_read_b64: gfx950 LDS runs in unaligned mode).
template <typename T>
static DEV const __attribute__((address_space(3))) T *lds_ptr(uint32_t a) {
    return reinterpret_cast<const __attribute__((address_space(3))) T *>(size_t(a));
}

// acc + popcount(m) in one VALU op.  `after` ties it behind the mbcnt of
// the same ballot, which already waited out the VALU-writes-SGPR hazard
// that the hazard recognizer does not see through inline asm.

static DEV uint32_t vbcnt(uint32_t m, uint32_t acc, uint32_t after) {
    uint32_t r;
    asm volatile("v_bcnt_u32_b32 %0, %1, %2" : "=v"(r) : "s"(m), "v"(acc), "v"(after));
    return r;
}

// Hedged chains (DecJob::done != nullptr): the host launches every stream
// 2-4 times, on different CUs, because the same chain runs up to ~20 %
// slower on some CUs than on others.  All copies
// compute identical bytes.  *done is a claim word: a copy starting group g
// raises it to g+1 (atomic max) and writes group g only if it was the first
// to start it, so every group is written once; the first copy to finish sets
// it to ~0 and the others leave after their current group.  The claim is
// issued at a group's start and its old value looked at the group's end, so
// the chain never waits for it.  Unhedged (done == nullptr): always write.
static DEV uint32_t hedge_claim(const DecJob &J, uint32_t g) {
    uint32_t v = 0u;
    if (J.done && threadIdx.x == 0)
        v = __hip_atomic_fetch_max(J.done, g + 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return v;
}
static DEV bool hedge_first(uint32_t v, uint32_t g) { return __builtin_amdgcn_readlane(v, 0) <= g; }
static DEV bool hedge_lost(uint32_t v) { return __builtin_amdgcn_readlane(v, 0) == ~0u; }
static DEV void hedge_won(const DecJob &J) {
    if (J.done && threadIdx.x == 0)
        __hip_atomic_store(J.done, ~0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

struct DecShared {
    uint16_t *ring;
    uint8_t *obuf;
    uint8_t *alpha;
    uint32_t *ltab;
};

static DEV DecShared dec_shared() {
    uint8_t *lds = reinterpret_cast<uint8_t *>(chain_lds);
    DecShared d;
    d.ring = reinterpret_cast<uint16_t *>(lds);
    d.obuf = lds + DEC_RING_BYTES;
    d.alpha = d.obuf + DEC_OBUF_BYTES;
    d.ltab = reinterpret_cast<uint32_t *>(lds + DEC_LDS_BASE);
    return d;
}

// Lane z fetches words [s*512 + 8z, +8) of the payload (past the end: 0).
static DEV uint4 load_slab(__amdgpu_buffer_rsrc_t w, uint32_t s, int z) {
    uint32_t t[4];
    const uint32_t b0 = (s * SLAB_WORDS + uint32_t(z) * 8) * 2;
#pragma unroll
    for (int b = 0; b < 4; b++)
        t[b] = ld8(w, b0 + 4 * b) | (ld8(w, b0 + 4 * b + 1) << 8) |
               (ld8(w, b0 + 4 * b + 2) << 16) | (ld8(w, b0 + 4 * b + 3) << 24);
    return make_uint4(t[0], t[1], t[2], t[3]);
}

// Ring slot = word index mod RING_WORDS; words 0..7 are mirrored past the
// end so that a 4-word window never wraps.
static DEV void store_slab(uint16_t *ring, uint32_t s, int z, uint4 v) {
    const uint32_t w0 = (s * SLAB_WORDS + uint32_t(z) * 8) & (RING_WORDS - 1);
    *reinterpret_cast<uint4 *>(ring + w0) = v;
    if (w0 == 0) *reinterpret_cast<uint4 *>(ring + RING_WORDS) = v;
}

static DEV uint64_t ring_win(const uint16_t *ring, uint32_t ptr) {
    const uint2 v = *reinterpret_cast<const uint2 *>(
        __builtin_assume_aligned(ring + (ptr & (RING_WORDS - 1)), 8));
    return (uint64_t(v.y) << 32) | v.x;
}

struct DecTabs {
    const uint32_t *ta;     // LDS/GLOBAL: u32 per slot
    const uint8_t *ts;      // SPLIT: u8 symbol per slot
    const uint32_t *fb;     // SPLIT: (f-1) << 16 | start
};

template <int TM>
static DEV DecTabs dec_tables(const DecJob &J, const DecShared &sh, int l) {
    const uint32_t rows = J.rows, slots = rows << J.bits;
    if (TM != DEC_TAB_GLOBAL) {
        const uint32_t nw = dec_tab_words(TM, rows, J.bits);
        for (uint32_t i = l; i < nw; i += 64) sh.ltab[i] = J.tab[i];
    }
    const uint32_t *base = TM == DEC_TAB_GLOBAL ? J.tab : sh.ltab;
    DecTabs t;
    t.ta = base;
    t.ts = reinterpret_cast<const uint8_t *>(base);
    t.fb = base + slots / 4;
    return t;
}

// One decode step's table work, split so the caller can order the LDS
// reads: dec_read issues the (first) table read, dec_finish completes the
// symbol and the pre-renorm state xd.
// rowoff: byte offset of the row (row << bits, times 4 for u32 slots).
template <int TM>
static DEV uint32_t dec_read(const DecTabs &t, uint32_t rowoff, uint32_t x, uint32_t mask) {
    if (TM == DEC_TAB_SPLIT) return t.ts[rowoff + (x & mask)];
    return *reinterpret_cast<const uint32_t *>(reinterpret_cast<const uint8_t *>(t.ta) + rowoff +
                                               ((x & mask) << 2));
}
template <int TM>
static DEV uint32_t dec_rowoff(uint32_t sy, int bits) {
    return (sy & 0xffu) << (TM == DEC_TAB_SPLIT ? bits : bits + 2);
}
template <int TM>
static DEV uint32_t dec_finish(const DecTabs &t, uint32_t rd, uint32_t rowfb, uint32_t x,
                               int bits, uint32_t mask, uint32_t &xd) {
    const uint32_t xh = x >> bits;
    if (TM == DEC_TAB_SPLIT) {      // rowfb: byte offset of the fb row
        const uint32_t e = *reinterpret_cast<const uint32_t *>(
            reinterpret_cast<const uint8_t *>(t.fb) + rowfb + (rd << 2));
        xd = __umul24(e >> 16, xh) + xh + (x & mask) - (e & 0xffffu);
        return rd;
    } else {
        xd = __umul24(rd >> (bits + 8), xh) + (xh + ((rd >> 8) & mask));
        return rd;                       // symbol in the low byte
    }
}

// Output of one group [t0, t0+steps).  LM (NX=4): obuf is lane-major,
// byte (tt, z) at z*G + tt; otherwise step-major at tt*NX + z.
template <bool O1, int NX, bool LM>
static DEV void dec_flush(const DecJob &J, const DecShared &sh, uint32_t t0, uint32_t steps,
                          int l) {
    constexpr uint32_t G = DEC_OBUF / NX;
    const uint32_t n = J.n, isz = n / NX;
    const auto out = buf(J.out, n);
    if (O1) {
        for (uint32_t zc = 0; zc < uint32_t(NX); zc++) {
            const uint32_t lz = (zc == NX - 1) ? n - uint32_t(NX - 1) * isz : isz;
            for (uint32_t tt = l; tt < steps; tt += 64) {
                const uint32_t v = LM ? sh.obuf[zc * G + tt] : sh.obuf[tt * NX + zc];
                if (t0 + tt < lz) st8(out, zc * isz + t0 + tt, sh.alpha[v]);
            }
        }
    } else {
        const uint32_t cnt = steps * NX;
        for (uint32_t i = l; i < cnt; i += 64) {
            const uint32_t v = LM ? sh.obuf[(i % NX) * G + i / NX] : sh.obuf[i];
            st8(out, NX * t0 + i, v);          // past n: dropped
        }
    }
}

template <bool O1, int TM>
static DEV void dec4_body(const DecJob &J) {
    constexpr int NX = 4;
    constexpr uint32_t G = DEC_OBUF / NX;     // steps per output group
    const DecShared sh = dec_shared();
    const int l = int(threadIdx.x);
    const int z = l & 3;
    const uint32_t n = J.n;
    const int bits = J.bits;
    const uint32_t mask = (1u << bits) - 1;
    const uint32_t rpl = dec_rp_log(J.rows);
    const DecTabs tb = dec_tables<TM>(J, sh, l);
    if (O1)
        for (int i = l; i < 256; i += 64) sh.alpha[i] = i < int(J.rows) ? J.alpha[i] : 0;

    uint32_t x = 1u << 16;                    // idle lanes: any in-range state
    if (l < NX) {
        const uint8_t *p = J.in + 4 * l;
        x = p[0] | (uint32_t(p[1]) << 8) | (uint32_t(p[2]) << 16) | (uint32_t(p[3]) << 24);
    }
    const uint32_t nwords = (J.in_len - 4 * uint32_t(NX)) / 2;
    const auto wsrc = buf(J.in + 4 * NX, nwords * 2);
    uint32_t slabs = 0;
    uint4 pf = load_slab(wsrc, 0, l);

    const uint32_t isz = n / NX;
    const uint32_t lenz = O1 ? ((z == NX - 1) ? n - uint32_t(NX - 1) * isz : isz) : 0;
    const uint32_t T = O1 ? n - uint32_t(NX - 1) * isz : (n + NX - 1) / NX;
    const uint32_t Tfull = O1 ? isz : n / NX;   // steps with all lanes active
    uint32_t rowbase = 0, rowfb = 0;
    uint32_t ptr = 0;                        // words consumed (uniform)
    // lane z < NX owns obuf[z*G, +G); idle lanes store into a sink
    uint8_t *myob = sh.obuf + (l < NX ? uint32_t(l) * G : DEC_OBUF + 64);

    // One step on all lanes.  Order of the LDS traffic: the table read (on
    // the chain) first, then the window of the next words; the symbol is
    // packed into acc (byte u&3) and 16 symbols go out in one store.
    auto fstep = [&](uint32_t &acc, int u) {
        uint32_t xd, sy;
        uint64_t win;
        if (TM == DEC_TAB_SPLIT) {
            // both table reads, then the window (rowfb is a byte offset)
            sy = tb.ts[rowbase + (x & mask)];
            const uint32_t e = *reinterpret_cast<const uint32_t *>(
                reinterpret_cast<const uint8_t *>(tb.fb) + rowfb + (sy << 2));
            __builtin_amdgcn_sched_barrier(0);
            win = ring_win(sh.ring, ptr);
            __builtin_amdgcn_sched_barrier(0);
            const uint32_t xh = x >> bits;
            xd = __umul24(e >> 16, xh) + xh + (x & mask) - (e & 0xffffu);
        } else {
            const uint32_t rd = dec_read<TM>(tb, rowbase, x, mask);
            __builtin_amdgcn_sched_barrier(0);
            win = ring_win(sh.ring, ptr);
            __builtin_amdgcn_sched_barrier(0);
            sy = dec_finish<TM>(tb, rd, rowfb, x, bits, mask, xd);
        }
        const bool c = xd < RANS_LOW_D;
        const uint64_t m = __ballot(c);
        const uint32_t r16 = __builtin_amdgcn_mbcnt_lo(uint32_t(m), 0u) << 4;
        const uint32_t w = uint32_t(win >> r16);
        x = c ? __builtin_amdgcn_perm(xd, w, 0x05040100u) : xd;
        ptr = vbcnt(uint32_t(m), ptr, r16);      // exec = the 4 state lanes
        // acc byte (u&3) <- sy byte 0, other bytes kept
        constexpr uint32_t SEL[4] = {0x07060500u, 0x07060004u, 0x07000504u, 0x00060504u};
        acc = __builtin_amdgcn_perm(acc, sy, SEL[u & 3]);
        if (O1) {
            rowbase = dec_rowoff<TM>(sy, bits);
            rowfb = (sy & 0xffu) << (TM == DEC_TAB_SPLIT ? rpl + 2 : rpl);
        }
    };

    for (uint32_t t0 = 0; t0 < T; t0 += G) {
        // keep the ring 2.5 groups of words ahead, never overwriting unread words
        while (slabs * SLAB_WORDS < ptr + 2560 && slabs * SLAB_WORDS < nwords + SLAB_WORDS) {
            store_slab(sh.ring, slabs, l, pf);
            slabs++;
            pf = load_slab(wsrc, slabs, l);
        }
        __syncthreads();
        const uint32_t hedge = hedge_claim(J, t0 / G);
        const uint32_t t1 = (T - t0 < G) ? T : t0 + G;
        const uint32_t tf = t1 < Tfull ? t1 : (t0 > Tfull ? t0 : Tfull);
        uint32_t t = t0;
        // Full steps on the 4 state lanes only (LDS traffic scales with the
        // active lanes); ptr stays uniform among them and is re-broadcast.
        if (l < NX) {
            for (; t + 16 <= tf; t += 16) {
                uint32_t a0 = 0, a1 = 0, a2 = 0, a3 = 0;
#pragma unroll
                for (int u = 0; u < 4; u++) fstep(a0, u);
#pragma unroll
                for (int u = 4; u < 8; u++) fstep(a1, u);
#pragma unroll
                for (int u = 8; u < 12; u++) fstep(a2, u);
#pragma unroll
                for (int u = 12; u < 16; u++) fstep(a3, u);
                *reinterpret_cast<uint4 *>(myob + (t - t0)) = make_uint4(a0, a1, a2, a3);
            }
        }
        ptr = __builtin_amdgcn_readfirstlane(ptr);
        t = __builtin_amdgcn_readfirstlane(t);
        // rest: byte stores; the last <= NX-1 steps have idle lanes
        for (; t < t1; t++) {
            const bool act = l < NX && (O1 ? t < lenz : uint32_t(NX) * t + z < n);
            const uint32_t rd = dec_read<TM>(tb, rowbase, x, mask);
            uint32_t xd;
            const uint32_t sy = dec_finish<TM>(tb, rd, rowfb, x, bits, mask, xd);
            const uint64_t win = ring_win(sh.ring, ptr);
            const bool c = act && xd < RANS_LOW_D;
            const uint64_t m = __ballot(c);
            const uint32_t r16 = __builtin_amdgcn_mbcnt_lo(uint32_t(m), 0u) << 4;
            const uint32_t w = uint32_t(win >> r16);
            if (act) {
                x = c ? __builtin_amdgcn_perm(xd, w, 0x05040100u) : xd;
                myob[t - t0] = uint8_t(sy);
                if (O1) {
                    rowbase = dec_rowoff<TM>(sy, bits);
                    rowfb = (sy & 0xffu) << (TM == DEC_TAB_SPLIT ? rpl + 2 : rpl);
                }
            }
            ptr += uint32_t(__popcll(m & 15u));
        }
        __syncthreads();
        if (hedge_first(hedge, t0 / G)) dec_flush<O1, NX, true>(J, sh, t0, t1 - t0, l);
        __syncthreads();
        if (hedge_lost(hedge)) return;
    }
    if (l == 0) *J.status = (ptr <= nwords) ? 0 : -1;
    hedge_won(J);
}

// NX = 32: lanes 0..31 are the states; each renormalising lane reads its
// word from the ring at ptr + rank.
template <bool O1, int TM>
static DEV void dec32_body(const DecJob &J) {
    constexpr int NX = 32;
    constexpr uint32_t G = DEC_OBUF / NX;
    const DecShared sh = dec_shared();
    const int l = int(threadIdx.x);
    const int z = l & 31;
    const uint32_t n = J.n;
    const int bits = J.bits;
    const uint32_t mask = (1u << bits) - 1;
    const uint32_t rpl = dec_rp_log(J.rows);
    const DecTabs tb = dec_tables<TM>(J, sh, l);
    if (O1)
        for (int i = l; i < 256; i += 64) sh.alpha[i] = i < int(J.rows) ? J.alpha[i] : 0;
    uint32_t x = 1u << 16;
    if (l < NX) {
        const uint8_t *p = J.in + 4 * l;
        x = p[0] | (uint32_t(p[1]) << 8) | (uint32_t(p[2]) << 16) | (uint32_t(p[3]) << 24);
    }
    const uint32_t nwords = (J.in_len - 4 * uint32_t(NX)) / 2;
    const auto wsrc = buf(J.in + 4 * NX, nwords * 2);
    uint32_t slabs = 0;
    uint4 pf = load_slab(wsrc, 0, l);
    const uint32_t isz = n / NX;
    const uint32_t lenz = O1 ? ((z == NX - 1) ? n - uint32_t(NX - 1) * isz : isz) : 0;
    const uint32_t T = O1 ? n - uint32_t(NX - 1) * isz : (n + NX - 1) / NX;
    uint32_t rowbase = 0, rowfb = 0, ptr = 0;
    for (uint32_t t0 = 0; t0 < T; t0 += G) {
        while (slabs * SLAB_WORDS < ptr + 2560 && slabs * SLAB_WORDS < nwords + SLAB_WORDS) {
            store_slab(sh.ring, slabs, l, pf);
            slabs++;
            pf = load_slab(wsrc, slabs, l);
        }
        __syncthreads();
        const uint32_t hedge = hedge_claim(J, t0 / G);
        const uint32_t t1 = (T - t0 < G) ? T : t0 + G;
        for (uint32_t t = t0; t < t1; t++) {
            const bool act = l < NX && (O1 ? t < lenz : uint32_t(NX) * t + z < n);
            uint32_t xd;
            const uint32_t rd = dec_read<TM>(tb, rowbase, x, mask);
            const uint32_t sy = dec_finish<TM>(tb, rd, rowfb, x, bits, mask, xd) & 0xffu;
            const bool c = act && xd < RANS_LOW_D;
            const uint64_t m = __ballot(c);
            const uint32_t rank = __builtin_amdgcn_mbcnt_lo(uint32_t(m), 0u);
            const uint32_t w = sh.ring[(ptr + rank) & (RING_WORDS - 1)];
            if (act) {
                x = c ? __builtin_amdgcn_perm(xd, w, 0x05040100u) : xd;
                sh.obuf[(t - t0) * NX + z] = uint8_t(sy);
                if (O1) { rowbase = dec_rowoff<TM>(sy, bits); rowfb = sy << (rpl + 2); }
            }
            ptr += uint32_t(__popcll(m & 0xffffffffull));
        }
        __syncthreads();
        if (hedge_first(hedge, t0 / G)) dec_flush<O1, NX, false>(J, sh, t0, t1 - t0, l);
        __syncthreads();
        if (hedge_lost(hedge)) return;
    }
    if (l == 0) *J.status = (ptr <= nwords) ? 0 : -1;
    hedge_won(J);
}

// ---------------------------------------------------------------------------
// NX = 4, O0 and small-table O1: the lean chain.  The step carries only what
// the next state needs and a table index is emitted in place of the symbol
// (mapped to the symbol at the group flush):
//   LDS entry per (row, slot)   {f, slot - start, T, next} (16 B), with
//                        T = ceil((2^15 - (slot - start)) / f) and next the
//                        LDS address of the row the decoded symbol selects
//                        (O1: the next step's context; O0: the one row)
//   entry address = row + slot * 16      (one shift-add; row = last entry's next)
//   xd   = f * (x >> bits) + (slot - start)             (one mad24)
//   renormalise  <=>  xd < 2^15  <=>  (x >> bits) < T, so the ballot does
//        not wait for the mad24
//   ptr  lives in a VGPR and advances with one v_bcnt of the renorm ballot;
//        the ring is linear over a group (a mirrored head), so the window
//        address is one shift-add of ptr.
// O1 thus costs what O0 does: the context is a field of the entry read on
// the chain anyway.  It applies while the table's rows x 2^bits entries
// fit (dec_lean: at most 8192, i.e. up to 8 contexts at TF_SHIFT 10 — the
// quality and sequence alphabets of the bench's data).
// Per step: 2 VALU for the table address, the table and window reads, 2 for
// xd, the ballot, 6 for the renorm select and ptr (slots stay in VGPRs): no
// SALU on the chain (a wave issues one instruction per ~4 cycles whatever the
// unit, so SALU round trips cost as much as VALU ones).
constexpr uint32_t O0_G = 512;                         // steps per group (per-group work: ~2 %)
constexpr uint32_t O0_MIRROR = 2056;                   // >= 4*G + 4, slab-unit multiple of 8
constexpr uint32_t O0_RING_BYTES = (RING_WORDS + O0_MIRROR) * 2;
constexpr uint32_t O0_OBUF_BYTES = 4 * O0_G * 2;       // u16 table indices, lane-major
constexpr uint32_t O0_SYM_OFF = O0_RING_BYTES + O0_OBUF_BYTES;
constexpr uint32_t O0_TAB_OFF = O0_SYM_OFF + DEC_LEAN_ENTRIES;   // 16-B entries, 16-B aligned
static_assert(O0_TAB_OFF % 16 == 0, "lean table alignment");
constexpr uint32_t O0_LDS_BYTES = O0_TAB_OFF + DEC_LEAN_ENTRIES * 16;
static_assert(O0_LDS_BYTES <= 160 * 1024, "lean decoder LDS");
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

static DEV void store_slab_o0(uint16_t *ring, uint32_t s, int z, uint4 v) {
    const uint32_t w0 = (s * SLAB_WORDS + uint32_t(z) * 8) & (RING_WORDS - 1);
    *reinterpret_cast<uint4 *>(ring + w0) = v;
    if (w0 < O0_MIRROR) *reinterpret_cast<uint4 *>(ring + RING_WORDS + w0) = v;
}

// Register decoder (K > 0, O0 only): the stream's K <= 8 symbols cover the
// 2^bits slots, and per symbol i a key = (start_i << (32 - bits)) - f_i
// lives in a register (uniform).  With T = x << (32 - bits) (the slot in the
// top bits, one shift), the symbol holding the slot is the one whose start
// is the largest <= slot, i.e. the smallest T - key_i (larger starts wrap
// past 2^32 - 2^(32-bits)), and that difference is (slot - start) <<
// (32 - bits) | f: K subtractions and a v_min3 tree, no table read (~64
// cycles on the chain) and no compare whose SGPR result a select would wait
// for (~20 cycles each).  The slot is still what the group keeps.  (Round 5:
// keys with the slot at bit 16, T = (x & mask) << 16 | 0xffff, cost one more
// dependent op: 139-152 -> 129-147 cycles a step, tools/dec_probe_run.py.)
template <bool O1, int K = 0>
static DEV void dec4_lean_body(const DecJob &J) {
    constexpr int NX = 4;
    constexpr uint32_t G = O0_G;
    uint8_t *lds = reinterpret_cast<uint8_t *>(chain_lds);
    uint16_t *ring = reinterpret_cast<uint16_t *>(lds);
    uint16_t *obuf = reinterpret_cast<uint16_t *>(lds + O0_RING_BYTES);
    uint8_t *s2sym = lds + O0_SYM_OFF;
    uint4 *tab = reinterpret_cast<uint4 *>(lds + O0_TAB_OFF);
    const int l = int(threadIdx.x);
    const uint32_t n = J.n;
    const int bits = J.bits;
    const uint32_t mask = (1u << bits) - 1;
    const uint32_t tab_lds = uint32_t(reinterpret_cast<uintptr_t>(
        (__attribute__((address_space(3))) uint4 *)(tab)));
    const uint32_t rows = O1 ? J.rows : 1u;
    const uint32_t idx0 = tab_lds >> 4;                // emitted index = entry address / 16
    // (f-1) << (bits+8) | (slot-start) << 8 | sym  ->  {f, slot-start, T, row of sym}
    for (uint32_t i = l; i < (rows << bits); i += 64) {
        const uint32_t e = J.tab[i];
        const uint32_t f = (e >> (bits + 8)) + 1, b = (e >> 8) & mask, sy = e & 0xffu;
        tab[i] = make_uint4(f, b, (RANS_LOW_D - b + f - 1) / f,
                            O1 ? tab_lds + ((sy << bits) << 4) : tab_lds);
        s2sym[i] = O1 ? J.alpha[sy] : uint8_t(sy);
    }
    uint32_t x = 1u << 16;
    if (l < NX) {
        const uint8_t *p = J.in + 4 * l;
        x = p[0] | (uint32_t(p[1]) << 8) | (uint32_t(p[2]) << 16) | (uint32_t(p[3]) << 24);
    }
    const uint32_t nwords = (J.in_len - 4 * uint32_t(NX)) / 2;
    const auto wsrc = buf(J.in + 4 * NX, nwords * 2);
    uint32_t slabs = 0;
    uint4 pf = load_slab(wsrc, 0, l);
    // O0: step t, lane z -> byte 4t + z.  O1: lane z owns the bytes
    // [z*isz, z*isz + lenz), the last lane the tail (rANS_static4x16pr.c:464-481)
    const uint32_t isz = n / NX;
    const uint32_t lenz = O1 ? ((l & 3) == NX - 1 ? n - uint32_t(NX - 1) * isz : isz) : 0;
    const uint32_t T = O1 ? n - uint32_t(NX - 1) * isz : (n + NX - 1) / NX;
    const uint32_t Tfull = O1 ? isz : n / NX;          // steps with all lanes active
    uint32_t ptr = 0;                                  // words consumed (uniform)
    uint32_t row = tab_lds;                            // O1: context 0 at a segment start
    const uint32_t ring_lds = uint32_t(reinterpret_cast<uintptr_t>(
        (__attribute__((address_space(3))) uint16_t *)(ring)));
    uint16_t *myob = obuf + (l & 3) * G;
    uint32_t KEY[K > 0 ? K : 1], NKEY[K > 0 ? K : 1], KSH[K > 0 ? K : 1];
    // keys start << (32 - bits) - f: T = x << (32 - bits) is one shift, and
    // T - key = (slot - start) << (32 - bits) | f (f <= 2^bits < 2^(32 - bits));
    // NKEY = -key, so that T - key is one v_lshl_add_u32 of x.  KSH holds one
    // opaque copy of the shift per key: with a shared x << ksh the compiler
    // computes T once and subtracts (one more op on the chain)
    const uint32_t ksh = 32u - uint32_t(bits);
#pragma unroll
    for (int i = 0; i < (K > 0 ? K : 1); i++) {
        KEY[i] = K > 0 ? ((J.reg[i] & 0xffffu) << ksh) - (J.reg[i] >> 16) : 0u;
        NKEY[i] = 0u - KEY[i];
        uint32_t k = ksh;
        asm volatile("; opaque shift %0" : "+v"(k));
        KSH[i] = k;
    }
    (void)KEY;
#ifdef FQZ5_CHAIN_PROBE
    const uint64_t pr0 = __builtin_amdgcn_s_memtime(), rr0 = __builtin_amdgcn_s_memrealtime();
    uint64_t t_steps = 0, n_steps = 0;
#endif

    for (uint32_t t0 = 0; t0 < T; t0 += G) {
        while (slabs * SLAB_WORDS < ptr + 2560 && slabs * SLAB_WORDS < nwords + SLAB_WORDS) {
            store_slab_o0(ring, slabs, l, pf);
            slabs++;
            pf = load_slab(wsrc, slabs, l);
        }
        __syncthreads();
        const uint32_t hedge = hedge_claim(J, t0 / G);
        // word p of this group sits at byte wbase + 2p of the LDS (p - gp < 1028)
        const uint32_t gp = ptr;
        const uint32_t wbase = ring_lds + 2 * ((gp & (RING_WORDS - 1)) - gp);
        const uint32_t t1 = (T - t0 < G) ? T : t0 + G;
        const uint32_t tf = t1 < Tfull ? t1 : (t0 > Tfull ? t0 : Tfull);
        uint32_t t = t0;
#ifdef FQZ5_CHAIN_PROBE
        const uint64_t ps0 = __builtin_amdgcn_s_memtime();
#endif
        if (l < NX) {
            for (; t + 16 <= tf; t += 16) {
                uint32_t a[16];
#pragma unroll
                for (int u = 0; u < 16; u++) {
                    if (K > 0) {
#ifdef FQZ5_REGDEC_OLD
                        // (round 5's step, for A/B builds)
                        const uint64_t win = *lds_ptr<uint64_t>(wbase + (ptr << 1));
                        __builtin_amdgcn_sched_barrier(0);
                        const uint32_t T = x << ksh;
                        a[u] = x & mask;
                        const uint32_t xh = x >> bits;
                        uint32_t d = T - KEY[0];
#pragma unroll
                        for (int i = 1; i < K; i++) d = min(d, T - KEY[i]);
                        const uint32_t xd = __umul24(d & ((1u << ksh) - 1u), xh) + (d >> ksh);
                        const bool c = xd < RANS_LOW_D;
                        const uint64_t m = __ballot(c);
                        const uint32_t r16 = __builtin_amdgcn_mbcnt_lo(uint32_t(m), 0u) << 4;
                        const uint32_t w = uint32_t(win >> r16);
                        x = c ? __builtin_amdgcn_perm(xd, w, 0x05040100u) : xd;
                        ptr = vbcnt(uint32_t(m), ptr, r16);
                        continue;
#else
                        // the window read first (its address is known since
                        // the last step), so its latency hides behind the
                        // selection.  Round 6, three issue slots fewer a
                        // step: each key's difference is one shift-add of x
                        // (no separate T); the group keeps x itself (its low
                        // 16 bits, the slot masked at the flush) instead of
                        // x & mask; the word is a byte permute of the window
                        // by a selector from the lane's rank (one mad24) in
                        // place of the 64-bit shift.
                        const uint64_t win = *lds_ptr<uint64_t>(wbase + (ptr << 1));
                        __builtin_amdgcn_sched_barrier(0);
                        a[u] = x;
                        const uint32_t xh = x >> bits;
                        uint32_t d = (x << KSH[0]) + NKEY[0];
#pragma unroll
                        for (int i = 1; i < K; i++) d = min(d, (x << KSH[i]) + NKEY[i]);
                        const uint32_t xd = __umul24(d & ((1u << ksh) - 1u), xh) + (d >> ksh);
                        const bool c = xd < RANS_LOW_D;
                        const uint64_t m = __ballot(c);
                        const uint32_t sel = __umul24(__builtin_amdgcn_mbcnt_lo(uint32_t(m), 0u),
                                                      0x0202u) + 0x0c0c0100u;
                        const uint32_t w = __builtin_amdgcn_perm(uint32_t(win >> 32), uint32_t(win), sel);
                        x = c ? __builtin_amdgcn_perm(xd, w, 0x05040100u) : xd;
                        ptr = vbcnt(uint32_t(m), ptr, sel);
                        continue;
#endif
                    }
                    const uint32_t ea = O1 ? row + ((x & mask) << 4) : tab_lds + ((x & mask) << 4);
                    a[u] = O1 ? (ea >> 4) - idx0 : x & mask;
                    const uint32_t xh = x >> bits;          // ready before the reads return
                    // the window read (address known since the last step)
                    // goes first so neither read waits for the other
                    const uint64_t win = *lds_ptr<uint64_t>(wbase + (ptr << 1));
                    __builtin_amdgcn_sched_barrier(0);
                    const u32x4 e = *lds_ptr<u32x4>(ea);
                    __builtin_amdgcn_sched_barrier(0);
                    const bool c = xh < e.z;
                    const uint32_t xd = __umul24(e.x, xh) + e.y;
                    const uint64_t m = __ballot(c);
                    const uint32_t r16 = __builtin_amdgcn_mbcnt_lo(uint32_t(m), 0u) << 4;
                    const uint32_t w = uint32_t(win >> r16);
                    x = c ? __builtin_amdgcn_perm(xd, w, 0x05040100u) : xd;
                    ptr = vbcnt(uint32_t(m), ptr, r16);
                    if (O1) row = e.w;
                }
                // pairs of low halves (a register decoder's a[] hold whole x)
                auto pk = [](uint32_t lo, uint32_t hi) { return __builtin_amdgcn_perm(hi, lo, 0x05040100u); };
                uint4 *o = reinterpret_cast<uint4 *>(myob + (t - t0));
                o[0] = make_uint4(pk(a[0], a[1]), pk(a[2], a[3]), pk(a[4], a[5]), pk(a[6], a[7]));
                o[1] = make_uint4(pk(a[8], a[9]), pk(a[10], a[11]), pk(a[12], a[13]), pk(a[14], a[15]));
            }
#ifdef FQZ5_CHAIN_PROBE
            t_steps += __builtin_amdgcn_s_memtime() - ps0;
            n_steps += t - t0;
#endif
            // rest of the group: single steps; where lanes run out of
            // bytes (O0: the last step's lanes z >= n % 4, O1: all but the
            // last lane's tail) they are inactive
            for (; t < t1; t++) {
                const bool act = O1 ? t < lenz : uint32_t(NX) * t + uint32_t(l) < n;
                const uint32_t ea = (O1 ? row : tab_lds) + ((x & mask) << 4);
                const uint4 e = *reinterpret_cast<const uint4 *>(
                    lds + O0_TAB_OFF + (ea - tab_lds));
                const uint64_t win = *lds_ptr<uint64_t>(wbase + (ptr << 1));
                const uint32_t xd = __umul24(e.x, x >> bits) + e.y;
                const bool c = act && xd < RANS_LOW_D;
                const uint64_t m = __ballot(c);
                const uint32_t r16 = __builtin_amdgcn_mbcnt_lo(uint32_t(m), 0u) << 4;
                const uint32_t w = uint32_t(win >> r16);
                if (act) {
                    x = c ? __builtin_amdgcn_perm(xd, w, 0x05040100u) : xd;
                    myob[t - t0] = uint16_t((ea >> 4) - idx0);
                    if (O1) row = e.w;
                }
                ptr += uint32_t(__popcll(m));
            }
        }
        ptr = __builtin_amdgcn_readfirstlane(ptr);
        __syncthreads();
        const uint32_t cnt = (t1 - t0) * NX;
        if (!hedge_first(hedge, t0 / G)) {
            // another copy started this group first and writes it
        } else if (O1) {
            // lane-major: byte (t, z) at z*isz + t; lanes past their length
            // (the tail of the last) hold nothing
            const auto out = buf(J.out, n);
            for (uint32_t i = l; i < cnt; i += 64) {
                const uint32_t zc = i / (t1 - t0), tt = i % (t1 - t0);
                const uint32_t lz = (zc == NX - 1) ? n - uint32_t(NX - 1) * isz : isz;
                if (t0 + tt < lz) st8(out, zc * isz + t0 + tt, s2sym[obuf[zc * G + tt]]);
            }
        } else if (cnt == NX * G && NX * t0 + NX * G <= n &&
                   (reinterpret_cast<uintptr_t>(J.out) & 15) == 0) {
            // a whole group: lane l writes output bytes [16l, 16l+16) of each
            // 1 KB, i.e. steps 4l..4l+3 of the 4 states, as one 16-byte store
#pragma unroll
            for (uint32_t h = 0; h < G / 256; h++) {
                uint32_t v[4] = {0, 0, 0, 0};
#pragma unroll
                for (int z = 0; z < NX; z++) {
                    const uint2 q = *reinterpret_cast<const uint2 *>(obuf + z * G + 256 * h + 4 * l);
#pragma unroll
                    for (int k = 0; k < 4; k++) {
                        const uint32_t sl = (k & 2 ? q.y : q.x) >> (16 * (k & 1)) & mask;
                        v[k] |= uint32_t(s2sym[sl]) << (8 * z);
                    }
                }
                *reinterpret_cast<uint4 *>(J.out + NX * t0 + 1024 * h + 16 * l) =
                    make_uint4(v[0], v[1], v[2], v[3]);
            }
        } else {
            const auto out = buf(J.out, n);
            for (uint32_t i = l; i < cnt; i += 64)
                st8(out, NX * t0 + i, s2sym[obuf[(i & 3) * G + (i >> 2)] & mask]);   // past n: dropped
        }
        __syncthreads();
        if (hedge_lost(hedge)) return;
    }
    if (l == 0) *J.status = (ptr <= nwords) ? 0 : -1;
    hedge_won(J);
#ifdef FQZ5_CHAIN_PROBE
    if (l == 0 && blockIdx.x < 512) { g_jobt[blockIdx.x][4] = t_steps; g_jobt[blockIdx.x][5] = n_steps; }
    if (l == 0 && blockIdx.x == 0) {
        g_probe[2] = __builtin_amdgcn_s_memtime() - pr0;
        g_probe[3] = __builtin_amdgcn_s_memrealtime() - rr0;
        g_probe[4] = t_steps;
        g_probe[5] = n_steps;
        g_probe[6] = T;
    }
#endif
}

// ---------------------------------------------------------------------------
// NX = 4, O1 with few (context, symbol) pairs: the replicated-state register
// decoder.  State z lives in all 16 lanes of row z (lanes 16z..16z+15), each
// lane holding up to 4 of the stream's keys
//   K = ctx << rowsh | start << 16 | (0xffff - ((f-1) << 4 | sym))
// (rowsh 29 for 12-bit slots and <= 8 contexts, 28 for <= 10 bits and <= 16).
// With T = ctx << rowsh | slot << 16 | 0xffff, T - K is
//   (slot - start) << 16 | (f-1) << 4 | sym   for the key of this context
//                                              whose start is the largest <= slot,
// below 2^(rowsh-1), and at least that for every other key (other contexts
// differ in the top bits, a guard bit apart; larger starts wrap).  So one
// subtraction per key held and a 16-lane minimum (4 DPP row rotations, every
// lane of the row ending with it) give f, slot - start and the symbol, which
// is the next context: no table read on the chain (the LDS table of the
// general O1 path, ~220 cycles a step at -5, dec4_body).  rANS_static4x16pr.c
// :525-821 (O1 decode), rANS_static16_int.h:468 (decode_freq1).
// ---------------------------------------------------------------------------
static DEV uint32_t row_min16(uint32_t d) {
    // (DPP reads a VGPR two wait states after its VALU write)
    asm volatile(
        "s_nop 1\n"
        "v_min_u32_dpp %0, %0, %0 row_ror:8 row_mask:0xf bank_mask:0xf\n"
        "s_nop 1\n"
        "v_min_u32_dpp %0, %0, %0 row_ror:4 row_mask:0xf bank_mask:0xf\n"
        "s_nop 1\n"
        "v_min_u32_dpp %0, %0, %0 row_ror:2 row_mask:0xf bank_mask:0xf\n"
        "s_nop 1\n"
        "v_min_u32_dpp %0, %0, %0 row_ror:1 row_mask:0xf bank_mask:0xf\n"
        : "+v"(d));
    return d;
}

template <int NK>
static DEV void dec4_o1reg_body(const DecJob &J) {
    constexpr int NX = 4;
    constexpr uint32_t G = O0_G;
    static_assert(O0_RING_BYTES + 4 * G + 256 <= DEC_O1REG_LDS_BYTES, "o1reg LDS");
    uint8_t *lds = reinterpret_cast<uint8_t *>(chain_lds);
    uint16_t *ring = reinterpret_cast<uint16_t *>(lds);
    uint8_t *obuf = lds + O0_RING_BYTES;                 // symbols, lane-major z*G + tt
    uint8_t *a2b = obuf + 4 * G;                         // symbol index -> byte
    const int l = int(threadIdx.x);
    const uint32_t z = uint32_t(l) >> 4, jl = uint32_t(l) & 15u;
    const uint32_t n = J.n;
    const int bits = J.bits;
    const uint32_t mask = (1u << bits) - 1;
    const uint32_t rowsh = J.rowsh;
    for (uint32_t i = l; i < J.rows; i += 64) a2b[i] = J.alpha[i];
    uint32_t KEY[NK];
#pragma unroll
    for (int k = 0; k < NK; k++) KEY[k] = J.okey[16 * k + jl];
    uint32_t x;
    {
        const uint8_t *p = J.in + 4 * z;
        x = p[0] | (uint32_t(p[1]) << 8) | (uint32_t(p[2]) << 16) | (uint32_t(p[3]) << 24);
    }
    const uint32_t nwords = (J.in_len - 4 * uint32_t(NX)) / 2;
    const auto wsrc = buf(J.in + 4 * NX, nwords * 2);
    uint32_t slabs = 0;
    uint4 pf = load_slab(wsrc, 0, l);
    // lane z owns the bytes [z*isz, z*isz + lenz), the last the tail
    // (rANS_static4x16pr.c:464-481)
    const uint32_t isz = n / NX;
    const uint32_t lenz = z == NX - 1 ? n - uint32_t(NX - 1) * isz : isz;
    const uint32_t T = n - uint32_t(NX - 1) * isz;
    const uint32_t Tfull = isz;
    uint32_t ptr = 0;                                  // words consumed (same in every lane)
    uint32_t rowb = 0xffffu;                           // context 0 at a segment start
    const uint32_t ring_lds = uint32_t(reinterpret_cast<uintptr_t>(
        (__attribute__((address_space(3))) uint16_t *)(ring)));
    uint8_t *myob = obuf + z * G;
    constexpr uint64_t LAST = 0x8000800080008000ull;   // lane 16z+15 of every row

    for (uint32_t t0 = 0; t0 < T; t0 += G) {
        while (slabs * SLAB_WORDS < ptr + 2560 && slabs * SLAB_WORDS < nwords + SLAB_WORDS) {
            store_slab_o0(ring, slabs, l, pf);
            slabs++;
            pf = load_slab(wsrc, slabs, l);
        }
        __syncthreads();
        const uint32_t hedge = hedge_claim(J, t0 / G);
        const uint32_t gp = ptr;
        const uint32_t wbase = ring_lds + 2 * ((gp & (RING_WORDS - 1)) - gp);
        const uint32_t t1 = (T - t0 < G) ? T : t0 + G;
        const uint32_t tf = t1 < Tfull ? t1 : (t0 > Tfull ? t0 : Tfull);
        uint32_t t = t0;
        for (; t + 16 <= tf; t += 16) {               // every state active
            uint32_t a[16];
#pragma unroll
            for (int u = 0; u < 16; u++) {
                const uint64_t win = *lds_ptr<uint64_t>(wbase + (ptr << 1));
                __builtin_amdgcn_sched_barrier(0);
                const uint32_t Tk = ((x & mask) << 16) | rowb;
                uint32_t d = Tk - KEY[0];
#pragma unroll
                for (int k = 1; k < NK; k++) d = min(d, Tk - KEY[k]);
                const uint32_t xh = x >> bits;
                d = row_min16(d);
                const uint32_t xd = __umul24((d >> 4) & 0xfffu, xh) + (xh + (d >> 16));
                rowb = (d << rowsh) | 0xffffu;
                a[u] = d;
                const bool c = xd < RANS_LOW_D;
                const uint64_t m = __ballot(c) & LAST;
                const uint32_t r16 = __builtin_amdgcn_mbcnt_hi(
                    uint32_t(m >> 32), __builtin_amdgcn_mbcnt_lo(uint32_t(m), 0u)) << 4;
                const uint32_t w = uint32_t(win >> r16);
                x = c ? __builtin_amdgcn_perm(xd, w, 0x05040100u) : xd;
                ptr += uint32_t(__popcll(m));
            }
            if (jl == 0) {
                uint32_t v[4];
#pragma unroll
                for (int q = 0; q < 4; q++)
                    v[q] = (a[4 * q] & 15u) | (a[4 * q + 1] & 15u) << 8 |
                           (a[4 * q + 2] & 15u) << 16 | (a[4 * q + 3] & 15u) << 24;
                *reinterpret_cast<uint4 *>(myob + (t - t0)) = make_uint4(v[0], v[1], v[2], v[3]);
            }
        }
        // the rest of the group one step at a time; states past their bytes
        // (all but the last one's tail) stand still
        for (; t < t1; t++) {
            const bool act = t < lenz;
            const uint64_t win = *lds_ptr<uint64_t>(wbase + (ptr << 1));
            const uint32_t Tk = ((x & mask) << 16) | rowb;
            uint32_t d = Tk - KEY[0];
#pragma unroll
            for (int k = 1; k < NK; k++) d = min(d, Tk - KEY[k]);
            const uint32_t xh = x >> bits;
            d = row_min16(d);
            const uint32_t xd = __umul24((d >> 4) & 0xfffu, xh) + (xh + (d >> 16));
            const bool c = act && xd < RANS_LOW_D;
            const uint64_t m = __ballot(c) & LAST;
            const uint32_t r16 = __builtin_amdgcn_mbcnt_hi(
                uint32_t(m >> 32), __builtin_amdgcn_mbcnt_lo(uint32_t(m), 0u)) << 4;
            const uint32_t w = uint32_t(win >> r16);
            if (act) {
                x = c ? __builtin_amdgcn_perm(xd, w, 0x05040100u) : xd;
                rowb = (d << rowsh) | 0xffffu;
                if (jl == 0) myob[t - t0] = uint8_t(d & 15u);
            }
            ptr += uint32_t(__popcll(m));
        }
        ptr = __builtin_amdgcn_readfirstlane(ptr);
        __syncthreads();
        if (hedge_first(hedge, t0 / G)) {
            const auto out = buf(J.out, n);
            const uint32_t steps = t1 - t0, cnt = steps * NX;
            for (uint32_t i = l; i < cnt; i += 64) {
                const uint32_t zc = i / steps, tt = i % steps;
                const uint32_t lz = (zc == NX - 1) ? n - uint32_t(NX - 1) * isz : isz;
                if (t0 + tt < lz) st8(out, zc * isz + t0 + tt, a2b[obuf[zc * G + tt]]);
            }
        }
        __syncthreads();
        if (hedge_lost(hedge)) return;
    }
    if (l == 0) *J.status = (ptr <= nwords) ? 0 : -1;
    hedge_won(J);
}

template <bool O1, int TM>
static DEV void dec_any(const DecJob &J) {
    if (J.nx == 32) dec32_body<O1, TM>(J);
    else if (!O1) {
#ifdef FQZ5_NO_REG_VARIANTS                  // experiments: code size of the kernel
        dec4_lean_body<false>(J);
        return;
#endif
        switch (J.nreg) {
        case 1: dec4_lean_body<false, 1>(J); break;
        case 2: dec4_lean_body<false, 2>(J); break;
        case 3: dec4_lean_body<false, 3>(J); break;
        case 4: dec4_lean_body<false, 4>(J); break;
        case 5: dec4_lean_body<false, 5>(J); break;
        case 6: dec4_lean_body<false, 6>(J); break;
        case 7: dec4_lean_body<false, 7>(J); break;
        case 8: dec4_lean_body<false, 8>(J); break;
        default: dec4_lean_body<false>(J);
        }
    }
    else if (TM == DEC_TAB_LDS && dec_lean(J.rows, J.bits)) dec4_lean_body<true>(J);
    else            dec4_body<O1, TM>(J);
}

__global__ __launch_bounds__(64) void k_rans_dec(const DecJob *jobs) {
    const DecJob J = jobs[blockIdx.x];
    if (J.nx == 0) return;                   // padding of an XCD-grouped launch
#ifdef FQZ5_CHAIN_PROBE
    const uint64_t jt0 = __builtin_amdgcn_s_memrealtime(), jc0 = __builtin_amdgcn_s_memtime();
    struct End {
        uint64_t t0, c0; const DecJob &J;
        __device__ ~End() {
            if (threadIdx.x == 0 && blockIdx.x < 512) {
                uint32_t hw, xcc;
                asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
                asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
                g_jobt[blockIdx.x][0] = t0;
                g_jobt[blockIdx.x][1] = __builtin_amdgcn_s_memrealtime();
                g_jobt[blockIdx.x][2] = __builtin_amdgcn_s_memtime() - c0;
                g_jobt[blockIdx.x][3] = uint64_t(J.n) << 32 | (xcc & 0xf) << 24 | ((hw >> 8) & 0x1f) << 16 | ((hw >> 13) & 0x7) << 8 | ((hw >> 4) & 3);
                g_jobt[blockIdx.x][6] = uint64_t(J.alpha ? J.rows : 0u) | uint64_t(J.nx) << 16 | uint64_t(J.mode) << 24;
                g_jobt[blockIdx.x][7] = J.in_len;
            }
        }
    } end_{jt0, jc0, J};
#endif
    const int tm = int(J.mode);
    if (J.alpha != nullptr && J.okeys) {
        switch (J.okeys >> 4) {
        case 1: dec4_o1reg_body<1>(J); break;
        case 2: dec4_o1reg_body<2>(J); break;
        case 3: dec4_o1reg_body<3>(J); break;
        default: dec4_o1reg_body<4>(J);
        }
    } else if (J.alpha != nullptr) {
        if (tm == DEC_TAB_LDS) dec_any<true, DEC_TAB_LDS>(J);
        else if (tm == DEC_TAB_SPLIT) dec_any<true, DEC_TAB_SPLIT>(J);
        else dec_any<true, DEC_TAB_GLOBAL>(J);
    } else {
        dec_any<false, DEC_TAB_LDS>(J);
    }
}

uint32_t dec_lds_bytes(uint32_t rows, int bits, int mode) {
    if (mode == DEC_TAB_GLOBAL) return DEC_LDS_BASE;
    const uint32_t b = DEC_LDS_BASE + dec_tab_words(uint32_t(mode), rows, bits) * 4u;
    return dec_lean(rows, bits) && b < O0_LDS_BYTES ? O0_LDS_BYTES : b;   // dec4_lean_body
}

static void lds_attr(const void *f) {
    (void)hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
}

hipError_t launch_enc_chain(const EncJob *d_jobs, int njobs, uint32_t lds, hipStream_t s) {
    if (!njobs) return hipSuccess;
    static bool attr = false;
    if (!attr) { lds_attr(reinterpret_cast<const void *>(k_enc_chain)); attr = true; }
    hipLaunchKernelGGL(k_enc_chain, dim3(njobs), dim3(64), lds, s, d_jobs);
    return hipGetLastError();
}

hipError_t launch_enc_chain2w(const EncJob *d_jobs, int njobs, uint32_t lds, hipStream_t s) {
    if (!njobs) return hipSuccess;
    static bool attr = false;
    if (!attr) { lds_attr(reinterpret_cast<const void *>(k_enc_chain2w)); attr = true; }
    hipLaunchKernelGGL(k_enc_chain2w, dim3(njobs), dim3(128), lds, s, d_jobs);
    return hipGetLastError();
}

hipError_t launch_enc_replay(const EncJob *d_jobs, const uint32_t *d_items, int nitems,
                             bool emit, uint32_t lds, hipStream_t s) {
    if (!nitems) return hipSuccess;
    static bool attr = false;
    if (!attr) {
        lds_attr(reinterpret_cast<const void *>(k_enc_replay<false>));
        lds_attr(reinterpret_cast<const void *>(k_enc_replay<true>));
        attr = true;
    }
    const uint2 *it = reinterpret_cast<const uint2 *>(d_items);
    if (emit) hipLaunchKernelGGL(k_enc_replay<true>, dim3(nitems), dim3(REPLAY_THREADS), lds, s, d_jobs, it);
    else      hipLaunchKernelGGL(k_enc_replay<false>, dim3(nitems), dim3(REPLAY_THREADS), lds, s, d_jobs, it);
    return hipGetLastError();
}

hipError_t launch_enc_scan(const EncJob *d_jobs, int njobs, hipStream_t s) {
    if (!njobs) return hipSuccess;
    hipLaunchKernelGGL(k_enc_scan, dim3(njobs), dim3(1024), 0, s, d_jobs);
    return hipGetLastError();
}

hipError_t launch_dec(const DecJob *d_jobs, int njobs, uint32_t lds, hipStream_t s) {
    if (!njobs) return hipSuccess;
    static bool attr = false;
    if (!attr) { lds_attr(reinterpret_cast<const void *>(k_rans_dec)); attr = true; }
    hipLaunchKernelGGL(k_rans_dec, dim3(njobs), dim3(64), lds, s, d_jobs);
    return hipGetLastError();
}

#ifdef FQZ5_CHAIN_PROBE
extern "C" int fqz5_chain_probe_read(uint64_t *out) {
    return int(hipMemcpyFromSymbol(out, HIP_SYMBOL(g_probe), sizeof(g_probe)));
}
extern "C" int fqz5_chain_jobs_read(uint64_t *out) {
    return int(hipMemcpyFromSymbol(out, HIP_SYMBOL(g_jobt), sizeof(g_jobt)));
}
#endif

}  // namespace fqz5
