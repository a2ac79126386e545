// rans_kernels.hip — CDNA4 (gfx950) kernels for the rANS 4x16/32x16 "pr"
// codecs of htscodecs, as used by fqzcomp5's block encoder.
//
// Data-parallel byte work (histograms, bit-packing, stripe transposes,
// copies) runs one thread per byte/word over many workgroups.  The entropy
// coder is a set of NX (4 or 32) dependent rANS chains per stream: the
// format fixes that parallelism (SURVEY.md §7 hard part (i)), so one
// 64-lane wave owns one stream, lane z owns state z, and all chains of a
// stream step in lock-step.  Where the reference serialises the 16-bit
// renormalisation words of the NX states into one stream, the wave uses a
// ballot + popcount to give each emitting lane its slot:
//   encode: states emit in descending lane order   (rANS_static4x16pr.c:187-197,
//                                                    rANS_static32x16pr.c:187-239)
//   decode: states consume in ascending lane order (rANS_static4x16pr.c:320-327)
//
// Step geometry (shared by encoder and decoder, derived from
// rANS_static4x16pr.c:112-232/:423-518 and rANS_static32x16pr.c:67-525):
//   O0: step k, lane z handles byte p = NX*k + z        (valid if p < n)
//   O1: step k, lane z handles byte p = z*isz + k        (valid if k < len_z)
//       isz = n/NX, len_z = isz except the last lane, which owns the tail.
// The encoder walks k from T-1 down to 0, the decoder from 0 up to T-1.
#include <hip/hip_runtime.h>
#include <cstdint>

#include "kernels.h"
#include "rans_format.hpp"

namespace fqz5 {

#define DEV __device__ __forceinline__

static DEV uint32_t lane_id() { return threadIdx.x & 63; }

// ---------------------------------------------------------------------------
// Histograms (utils.h:146 hist8 and the repeat counts used by rle.c:48
// rle_find_syms: eq[s] = #{i : d[i] == d[i-1] == s}).
// One workgroup per work item (segment slice); LDS counters; global atomics.
// ---------------------------------------------------------------------------
// Counting is privatised: thread t adds into copy t % C of the bins (rows
// padded by one word so that the copies of a bin fall in different LDS
// banks), so a wave's atomics on one bin (the common case on skewed quality
// or base data) conflict at most 64 / C ways instead of 64.
constexpr uint32_t HIST0_C = 16;
constexpr uint32_t HIST0_ROW = 513;                  // h[256], e[256], pad

__global__ __launch_bounds__(256) void k_hist0(const HistItem *items,
                                               uint32_t *counts) {
    __shared__ uint32_t h[HIST0_C * HIST0_ROW];
    const HistItem it = items[blockIdx.x];
    for (uint32_t i = threadIdx.x; i < HIST0_C * HIST0_ROW; i += blockDim.x) h[i] = 0;
    __syncthreads();
    const uint8_t *d = it.data;
    uint32_t *mine = h + (threadIdx.x % HIST0_C) * HIST0_ROW;
    // e[c]: bytes equal to their predecessor (hist8e's run count).  Each
    // thread reads 16-byte aligned chunks (one load; the chunk's first byte
    // takes its predecessor from one more byte load); bytes outside
    // [begin, end) are skipped.  A chunk never leaves the 16-byte blocks
    // that hold the slice's own bytes.
    const uint32_t mis = uint32_t(reinterpret_cast<uintptr_t>(d) & 15u);
    const uint4 *al = reinterpret_cast<const uint4 *>(d - mis);
    for (uint32_t c = (it.begin + mis) / 16 + threadIdx.x; 16 * c < it.end + mis; c += blockDim.x) {
        const uint4 v = al[c];
        const uint32_t w[4] = {v.x, v.y, v.z, v.w};
        const int64_t p0 = int64_t(16 * c) - int64_t(mis);
        int prev = p0 >= 1 ? int(d[p0 - 1]) : -1;
#pragma unroll
        for (int k = 0; k < 16; k++) {
            const int b = int((w[k >> 2] >> (8 * (k & 3))) & 0xffu);
            const int64_t p = p0 + k;
            if (p >= int64_t(it.begin) && p < int64_t(it.end)) {
                atomicAdd(&mine[b], 1u);
                if (b == prev && p > 0) atomicAdd(&mine[256 + b], 1u);   // byte 0: none
            }
            prev = b;
        }
    }
    __syncthreads();
    uint32_t *out = counts + size_t(it.seg) * 512;
    for (uint32_t b = threadIdx.x; b < 512; b += blockDim.x) {
        uint32_t v = 0;
#pragma unroll
        for (uint32_t c = 0; c < HIST0_C; c++) v += h[c * HIST0_ROW + b];
        if (v) atomicAdd(&out[b], v);
    }
}

// Order-1 pair counts F[ctx][sym] over the compacted alphabet
// (utils.h:280 hist1_4; context of byte 0 is 0).  `remap` maps a byte to
// its alphabet index (alphabet always contains 0).
//   A*A < 16384: the bins live in LDS in C privatised copies (C = 32 down
//                to 1 as A*A grows, within 64 KB);
//   larger (packed bytes, A up to 256): 16-bit counters, two per LDS word,
//                128 KB for all 65536 bins.  A counter that reaches 0x8000
//                spills: the add that saw 0x7fff takes 0x8000 back out of LDS
//                and adds it to the global count (the other adds that can
//                land in between are a few hundred, far from the 16-bit
//                limit), so a workgroup takes a multi-MB slice and flushes its
//                65536 bins once per slice.  (With 64 KB slices a -5 NovaSeq
//                step's packed candidates were ~24 000 workgroups that each
//                flushed every bin by global atomics: ~110 ms, with the
//                128 KB-LDS workgroups holding every CU meanwhile.)
template <bool BIG>
__global__ __launch_bounds__(256) void k_hist1(const Hist1Item *items,
                                               uint32_t *counts) {
    extern __shared__ uint32_t bins[];
    const Hist1Item it = items[blockIdx.x];
    const uint32_t A = it.A, nb = A * A;
    uint32_t C = 1;
    if (!BIG)
        while (C < 32 && 2 * C * (nb + 1) <= 16384) C *= 2;
    const uint32_t row = nb + 1;
    const uint32_t words = BIG ? (nb + 1) / 2 : C * row;
    __shared__ uint8_t rm[256];
    for (int i = threadIdx.x; i < 256; i += blockDim.x) rm[i] = it.remap[i];
    for (uint32_t i = threadIdx.x; i < words; i += blockDim.x) bins[i] = 0;
    __syncthreads();
    uint32_t *gout = counts + it.out_off;
    uint32_t *mine = bins + (threadIdx.x & (C - 1)) * row;
    const uint8_t *d = it.data;
    // 16-byte aligned chunks per thread, as in k_hist0
    const uint32_t mis = uint32_t(reinterpret_cast<uintptr_t>(d) & 15u);
    const uint4 *al = reinterpret_cast<const uint4 *>(d - mis);
    for (uint32_t ch = (it.begin + mis) / 16 + threadIdx.x; 16 * ch < it.end + mis; ch += blockDim.x) {
        const uint4 v = al[ch];
        const uint32_t w[4] = {v.x, v.y, v.z, v.w};
        const int64_t p0 = int64_t(16 * ch) - int64_t(mis);
        uint32_t p = p0 >= 1 ? rm[d[p0 - 1]] : rm[0];
#pragma unroll
        for (int k = 0; k < 16; k++) {
            const uint32_t c = rm[(w[k >> 2] >> (8 * (k & 3))) & 0xffu];
            const int64_t q = p0 + k;
            if (q >= int64_t(it.begin) && q < int64_t(it.end)) {
                const uint32_t b = (q == 0 ? uint32_t(rm[0]) : p) * A + c;   // byte 0: context 0
                if (BIG) {
                    const uint32_t sh = 16u * (b & 1u);
                    const uint32_t old = atomicAdd(&bins[b >> 1], 1u << sh);
                    if (((old >> sh) & 0xffffu) == 0x7fffu) {
                        atomicSub(&bins[b >> 1], 0x8000u << sh);
                        atomicAdd(&gout[b], 0x8000u);
                    }
                } else {
                    atomicAdd(&mine[b], 1u);
                }
            }
            p = c;
        }
    }
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < nb; i += blockDim.x) {
        uint32_t v = 0;
        if (BIG) {
            v = (bins[i >> 1] >> (16 * (i & 1))) & 0xffffu;
        } else {
            for (uint32_t c = 0; c < C; c++) v += bins[c * row + i];
        }
        if (v) atomicAdd(&gout[i], v);
    }
}

// ---------------------------------------------------------------------------
// PACK (pack.c:56-147): 2/4/8 symbols per byte, low bits first.
// One thread per output byte.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_pack(const PackItem *items) {
    const PackItem it = items[blockIdx.y];
    uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
    uint32_t nout = (it.n + it.per - 1) / it.per;
    if (j >= nout) return;
    const int bits = 8 / it.per;
    uint32_t i0 = j * it.per;
    uint32_t v = 0;
    for (int k = 0; k < it.per; k++) {
        uint32_t i = i0 + k;
        if (i < it.n) v |= uint32_t(it.code[it.in[i]]) << (k * bits);
    }
    it.out[j] = uint8_t(v);
}

// Inverse (pack.c:207-344).  One thread per output symbol.
__global__ __launch_bounds__(256) void k_unpack(const PackItem *items) {
    const PackItem it = items[blockIdx.y];
    uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= it.n) return;
    if (it.per == 0) { it.out[i] = it.code[0]; return; }
    const int bits = 8 / it.per;
    uint32_t v = (it.in[i / it.per] >> ((i % it.per) * bits)) & ((1u << bits) - 1);
    it.out[i] = it.code[v];
}

// STRIPE (rANS_static4x16pr.c:1283-1309): byte i goes to stripe i%N at
// offset i/N.  `dir` 0 = transpose (encode), 1 = untranspose (decode,
// utils.h:79 unstripe).  A workgroup takes a tile of N*C interleaved bytes
// (C = STRIPE_TILE / N of each stripe): the interleaved side moves through
// LDS with consecutive threads on consecutive bytes, and so does each
// stripe's run of C bytes.  (Up to round 6 one thread per byte scattered
// to N stripes: -5 NovaSeq up to 16.5 GB of HBM traffic in a dispatch,
// profiles/r06_pmc_l5.json.)
constexpr uint32_t STRIPE_TILE = 32768;
__global__ __launch_bounds__(256) void k_stripe(const StripeItem *items) {
    __shared__ uint8_t t[STRIPE_TILE];
    const StripeItem it = items[blockIdx.y];
    const uint32_t N = it.N, C = STRIPE_TILE / N, T = N * C;
    const uint64_t i0 = uint64_t(blockIdx.x) * T;
    if (i0 >= it.n) return;
    const uint32_t q = it.n / N, r = it.n % N;
    const uint32_t o0 = blockIdx.x * C;
    const uint32_t tn = uint32_t(min(uint64_t(T), uint64_t(it.n) - i0));
    if (it.dir == 0) {
        for (uint32_t k = threadIdx.x; k < tn; k += 256) t[k] = it.in[i0 + k];
        __syncthreads();
        for (uint32_t k = threadIdx.x; k < T; k += 256) {
            const uint32_t s = k / C, o = o0 + (k - s * C);
            if (o < q + (s < r ? 1u : 0u)) it.out[s * q + min(s, r) + o] = t[(o - o0) * N + s];
        }
    } else {
        for (uint32_t k = threadIdx.x; k < T; k += 256) {
            const uint32_t s = k / C, o = o0 + (k - s * C);
            if (o < q + (s < r ? 1u : 0u)) t[(o - o0) * N + s] = it.in[s * q + min(s, r) + o];
        }
        __syncthreads();
        for (uint32_t k = threadIdx.x; k < tn; k += 256) it.out[i0 + k] = t[k];
    }
}

__global__ __launch_bounds__(256) void k_gather(const GatherItem *items, int n,
                                                uint8_t *out) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) out[i] = *items[i].src;
}

// Gather copies for final stream assembly.  One workgroup per segment
// chunk of up to 64 KiB.
__global__ __launch_bounds__(256) void k_copy(const CopyItem *items) {
    const CopyItem it = items[blockIdx.x];
    for (uint32_t i = threadIdx.x; i < it.len; i += blockDim.x)
        it.dst[i] = it.src[i];
}

// ---------------------------------------------------------------------------
// RLE (rle.c:100-189).  Byte i starts a literal unless it repeats the
// previous byte and that byte is an RLE symbol; the run length stored for
// an RLE-symbol literal is the number of repeats that follow it, i.e. the
// distance to the next literal minus one, as a big-endian varint.
// Work is cut into chunks of RLE_CH bytes (one 256-thread workgroup each,
// RLE_PT consecutive bytes per thread).  Pass 1 counts literals and varint
// bytes per chunk; the host scans the per-chunk totals; pass 2 writes.
// ---------------------------------------------------------------------------
constexpr uint32_t RLE_PT = 256;
constexpr uint32_t RLE_CH = 256 * RLE_PT;
constexpr uint32_t NONE = 0xffffffffu;

static DEV uint32_t vlen32(uint32_t r) {
    return 1u + (r >= (1u << 7)) + (r >= (1u << 14)) + (r >= (1u << 21)) + (r >= (1u << 28));
}

static DEV bool rle_is_lit(const uint8_t *d, uint32_t i, const uint8_t *saved) {
    return i == 0 || d[i] != d[i - 1] || !saved[d[i]];
}

// Inclusive block-wide suffix minimum over 256 threads (Hillis-Steele).
static DEV uint32_t block_suffix_min(uint32_t v, uint32_t *tmp) {
    const int t = threadIdx.x;
    tmp[t] = v;
    __syncthreads();
    for (int o = 1; o < 256; o <<= 1) {
        uint32_t w = (t + o < 256) ? tmp[t + o] : NONE;
        __syncthreads();
        v = v < w ? v : w;
        tmp[t] = v;
        __syncthreads();
    }
    return v;
}

// Exclusive block-wide prefix sum over 256 threads.
static DEV uint32_t block_excl_sum(uint32_t v, uint32_t *tmp, uint32_t *total) {
    const int t = threadIdx.x;
    tmp[t] = v;
    __syncthreads();
    uint32_t acc = v;
    for (int o = 1; o < 256; o <<= 1) {
        uint32_t w = (t >= o) ? tmp[t - o] : 0;
        __syncthreads();
        acc += w;
        tmp[t] = acc;
        __syncthreads();
    }
    if (total) *total = tmp[255];
    __syncthreads();
    return acc - v;
}

// Per-thread scan of [a, b): literal count, first/last literal and the
// varint bytes of every RLE literal whose successor lies inside [a, b).
struct RleThr { uint32_t cnt, first, last, vsum; };

static DEV RleThr rle_thread_scan(const uint8_t *d, uint32_t a, uint32_t b,
                                  const uint8_t *saved) {
    RleThr r{0, NONE, NONE, 0};
    for (uint32_t i = a; i < b; i++) {
        if (!rle_is_lit(d, i, saved)) continue;
        if (r.last != NONE && saved[d[r.last]]) r.vsum += vlen32(i - r.last - 1);
        if (r.first == NONE) r.first = i;
        r.last = i;
        r.cnt++;
    }
    return r;
}

// The chunk's bytes [c0, c1) and the one before it, staged through LDS with
// coalesced 16-byte loads (the scan then reads LDS): returns a pointer that
// indexes like the input (dv[i] for i in [c0 - 1, c1)).
static DEV const uint8_t *rle_stage(const uint8_t *in, uint32_t c0, uint32_t c1, uint8_t *stage) {
    const uint8_t *src = in + c0;
    const uint32_t mis = uint32_t(reinterpret_cast<uintptr_t>(src) & 15u);
    const uint4 *al = reinterpret_cast<const uint4 *>(src - mis);
    const uint32_t len = c1 - c0, nblk = (len + mis + 15) / 16;
    for (uint32_t j = threadIdx.x; j < nblk; j += blockDim.x) {
        const uint4 v = al[j];
        const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int k = 0; k < 16; k++) {
            const int64_t o = int64_t(16 * j + k) - int64_t(mis);   // offset from c0
            if (o >= 0 && o < int64_t(len)) stage[1 + o] = uint8_t(w[k >> 2] >> (8 * (k & 3)));
        }
    }
    if (threadIdx.x == 0) stage[0] = c0 ? in[c0 - 1] : 0;
    __syncthreads();
    return stage + 1 - int64_t(c0);
}

// Pass 1: per chunk {lit count, first lit, last lit, varint bytes excluding
// the chunk's last literal, whether that literal is an RLE symbol}.
__global__ __launch_bounds__(256) void k_rle_count(const RleItem *items,
                                                   const uint32_t *chunk_item,
                                                   uint32_t *cstat) {
    __shared__ uint32_t tmp[256];
    __shared__ uint8_t saved[256];
    const uint32_t c = blockIdx.x;
    const RleItem it = items[chunk_item[2 * c]];
    const uint32_t lc = chunk_item[2 * c + 1];
    __shared__ uint8_t stage[RLE_CH + 1];
    saved[threadIdx.x] = it.saved[threadIdx.x];
    const uint32_t c0 = lc * RLE_CH, c1 = min(it.n, c0 + RLE_CH);
    const uint8_t *dv = rle_stage(it.in, c0, c1, stage);
    const uint32_t a = min(c1, c0 + threadIdx.x * RLE_PT), b = min(c1, a + RLE_PT);
    RleThr r = rle_thread_scan(dv, a, b, saved);
    // successor of my last literal inside the chunk = first literal of a later thread
    // suffix minimum of first-literal positions over the threads after me
    block_suffix_min(r.first, tmp);
    uint32_t later = (threadIdx.x < 255) ? tmp[threadIdx.x + 1] : NONE;
    __syncthreads();
    uint32_t vs = r.vsum;
    if (r.last != NONE && later != NONE && saved[dv[r.last]])
        vs += vlen32(later - r.last - 1);
    uint32_t tot_cnt, tot_vs;
    block_excl_sum(r.cnt, tmp, &tot_cnt);
    block_excl_sum(vs, tmp, &tot_vs);
    // chunk first / last literal
    __shared__ uint32_t cf, cl1;           // first literal, last literal + 1
    if (threadIdx.x == 0) { cf = NONE; cl1 = 0; }
    __syncthreads();
    if (r.first != NONE) atomicMin(&cf, r.first);
    if (r.last != NONE) atomicMax(&cl1, r.last + 1);
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t *o = cstat + 5 * c;
        o[0] = tot_cnt; o[1] = cf; o[2] = cl1 ? cl1 - 1 : NONE; o[3] = tot_vs;
        o[4] = cl1 ? saved[dv[cl1 - 1]] : 0;
    }
}

// Pass 2: write literals and varints.  cmeta per chunk: {lit_off,
// run_off, next literal after the chunk (or n)}.
__global__ __launch_bounds__(256) void k_rle_emit(const RleItem *items,
                                                  const uint32_t *chunk_item,
                                                  const uint32_t *cmeta) {
    __shared__ uint32_t tmp[256];
    __shared__ uint8_t saved[256];
    const uint32_t c = blockIdx.x;
    const RleItem it = items[chunk_item[2 * c]];
    const uint32_t lc = chunk_item[2 * c + 1];
    __shared__ uint8_t stage[RLE_CH + 1];
    saved[threadIdx.x] = it.saved[threadIdx.x];
    const uint32_t c0 = lc * RLE_CH, c1 = min(it.n, c0 + RLE_CH);
    const uint8_t *dv = rle_stage(it.in, c0, c1, stage);
    const uint32_t a = min(c1, c0 + threadIdx.x * RLE_PT), b = min(c1, a + RLE_PT);
    const uint32_t lit_off = cmeta[3 * c], run_off = cmeta[3 * c + 1],
                   chunk_next = cmeta[3 * c + 2];
    RleThr r = rle_thread_scan(dv, a, b, saved);
    // successor of this thread's last literal
    block_suffix_min(r.first, tmp);
    uint32_t later = (threadIdx.x < 255) ? tmp[threadIdx.x + 1] : NONE;
    __syncthreads();
    if (later == NONE) later = chunk_next;
    uint32_t vs = r.vsum;
    if (r.last != NONE && saved[dv[r.last]]) vs += vlen32(later - r.last - 1);
    uint32_t lo = block_excl_sum(r.cnt, tmp, nullptr) + lit_off;
    uint32_t ro = block_excl_sum(vs, tmp, nullptr) + run_off;
    // sequential write of this thread's literals and run varints
    uint32_t prev = NONE;
    auto put_run = [&](uint32_t rl) {
        int nb = int(vlen32(rl));
        for (int k = nb - 1; k >= 0; k--)
            it.runs[ro++] = uint8_t(((rl >> (7 * k)) & 0x7f) | (k ? 0x80 : 0));
    };
    for (uint32_t i = a; i < b; i++) {
        if (!rle_is_lit(dv, i, saved)) continue;
        if (prev != NONE && saved[dv[prev]]) put_run(i - prev - 1);
        it.lits[lo++] = dv[i];
        prev = i;
    }
    if (prev != NONE && saved[dv[prev]]) put_run(later - prev - 1);
}

// ---------------------------------------------------------------------------
// RLE decode (rle.c:142-189), three passes over chunks of literals:
//   1. per chunk: number of RLE-symbol literals                (host scans)
//   2. per chunk of run bytes: positions of varint terminators  (host scans)
//      -> vend[k] = byte index of the last byte of varint k
//   3. per chunk of literals: run lengths -> output sizes       (host scans)
//   4. per chunk of literals: write the expanded bytes
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_unrle_count(const UnRleItem *items,
                                                     const uint32_t *chunk_item,
                                                     uint32_t *cstat, int what) {
    __shared__ uint32_t tmp[256];
    __shared__ uint8_t saved[256];
    const uint32_t c = blockIdx.x;
    const UnRleItem it = items[chunk_item[2 * c]];
    const uint32_t lc = chunk_item[2 * c + 1];
    saved[threadIdx.x] = it.saved[threadIdx.x];
    __syncthreads();
    uint32_t cnt = 0;
    if (what == 0) {            // RLE literals per chunk of literals
        const uint32_t c0 = lc * RLE_CH, c1 = min(it.nlit, c0 + RLE_CH);
        const uint32_t a = min(c1, c0 + threadIdx.x * RLE_PT), b = min(c1, a + RLE_PT);
        for (uint32_t i = a; i < b; i++) cnt += saved[it.lits[i]];
    } else {                    // varint terminators per chunk of run bytes
        const uint32_t c0 = lc * RLE_CH, c1 = min(it.nrun, c0 + RLE_CH);
        const uint32_t a = min(c1, c0 + threadIdx.x * RLE_PT), b = min(c1, a + RLE_PT);
        for (uint32_t i = a; i < b; i++) cnt += !(it.runs[i] & 0x80);
    }
    uint32_t tot;
    block_excl_sum(cnt, tmp, &tot);
    if (threadIdx.x == 0) cstat[c] = tot;
}

__global__ __launch_bounds__(256) void k_unrle_vend(const UnRleItem *items,
                                                    const uint32_t *chunk_item,
                                                    const uint32_t *coff) {
    __shared__ uint32_t tmp[256];
    const uint32_t c = blockIdx.x;
    const UnRleItem it = items[chunk_item[2 * c]];
    const uint32_t lc = chunk_item[2 * c + 1];
    const uint32_t c0 = lc * RLE_CH, c1 = min(it.nrun, c0 + RLE_CH);
    const uint32_t a = min(c1, c0 + threadIdx.x * RLE_PT), b = min(c1, a + RLE_PT);
    uint32_t cnt = 0;
    for (uint32_t i = a; i < b; i++) cnt += !(it.runs[i] & 0x80);
    uint32_t k = block_excl_sum(cnt, tmp, nullptr) + coff[c];
    for (uint32_t i = a; i < b; i++)
        if (!(it.runs[i] & 0x80)) it.vend[k++] = i;
}

static DEV uint32_t unrle_run(const UnRleItem &it, uint32_t k) {
    // varint k spans (vend[k-1], vend[k]]
    uint32_t s = k ? it.vend[k - 1] + 1 : 0, e = it.vend[k];
    uint32_t v = 0;
    for (uint32_t i = s; i <= e; i++) v = (v << 7) | (it.runs[i] & 0x7f);
    return v;
}

// what 0: per chunk output length; what 1: write.  coff: {rle-literal
// offset, output offset} per chunk.
__global__ __launch_bounds__(256) void k_unrle_expand(const UnRleItem *items,
                                                      const uint32_t *chunk_item,
                                                      const uint32_t *coff,
                                                      uint32_t *cstat, int what) {
    __shared__ uint32_t tmp[256];
    __shared__ uint8_t saved[256];
    const uint32_t c = blockIdx.x;
    const UnRleItem it = items[chunk_item[2 * c]];
    const uint32_t lc = chunk_item[2 * c + 1];
    saved[threadIdx.x] = it.saved[threadIdx.x];
    __syncthreads();
    const uint32_t c0 = lc * RLE_CH, c1 = min(it.nlit, c0 + RLE_CH);
    const uint32_t a = min(c1, c0 + threadIdx.x * RLE_PT), b = min(c1, a + RLE_PT);
    uint32_t ns = 0;
    for (uint32_t i = a; i < b; i++) ns += saved[it.lits[i]];
    uint32_t k = block_excl_sum(ns, tmp, nullptr) + coff[2 * c];
    uint32_t olen = 0, k0 = k;
    for (uint32_t i = a; i < b; i++) {
        uint32_t r = 0;
        if (saved[it.lits[i]]) { r = k < it.nvarint ? unrle_run(it, k) : 0; k++; }
        olen += r + 1;
    }
    uint32_t tot;
    uint32_t o = block_excl_sum(olen, tmp, &tot) + coff[2 * c + 1];
    if (what == 0) {
        if (threadIdx.x == 0) cstat[c] = tot;
        return;
    }
    k = k0;
    for (uint32_t i = a; i < b; i++) {
        uint32_t r = 0;
        uint8_t ch = it.lits[i];
        if (saved[ch]) { r = k < it.nvarint ? unrle_run(it, k) : 0; k++; }
        for (uint32_t j = 0; j <= r; j++)
            if (o + j < it.nout) it.out[o + j] = ch;
        o += r + 1;
    }
}

// ---------------------------------------------------------------------------
// Host-side launchers
// ---------------------------------------------------------------------------
hipError_t launch_gather(const GatherItem *items, int n, uint8_t *out, hipStream_t s) {
    if (!n) return hipSuccess;
    hipLaunchKernelGGL(k_gather, dim3((n + 255) / 256), dim3(256), 0, s, items, n, out);
    return hipGetLastError();
}

hipError_t launch_hist0(const HistItem *d_items, int nitems, uint32_t *d_counts,
                        hipStream_t s) {
    if (!nitems) return hipSuccess;
    hipLaunchKernelGGL(k_hist0, dim3(nitems), dim3(256), 0, s, d_items, d_counts);
    return hipGetLastError();
}

hipError_t launch_hist1(const Hist1Item *d_items, int nitems, uint32_t *d_counts, bool big,
                        hipStream_t s) {
    if (!nitems) return hipSuccess;
    static bool attr = false;
    if (!attr) {
        (void)hipFuncSetAttribute(reinterpret_cast<const void *>(k_hist1<true>),
                                  hipFuncAttributeMaxDynamicSharedMemorySize, 131072);
        attr = true;
    }
    if (big) hipLaunchKernelGGL(k_hist1<true>, dim3(nitems), dim3(256), 131072, s, d_items, d_counts);
    else hipLaunchKernelGGL(k_hist1<false>, dim3(nitems), dim3(256), 16384 * 4, s, d_items, d_counts);
    return hipGetLastError();
}

hipError_t launch_pack(const PackItem *d_items, int nitems, uint32_t max_out,
                       bool unpack, hipStream_t s) {
    if (!nitems || !max_out) return hipSuccess;
    dim3 g((max_out + 255) / 256, nitems);
    if (unpack) hipLaunchKernelGGL(k_unpack, g, dim3(256), 0, s, d_items);
    else hipLaunchKernelGGL(k_pack, g, dim3(256), 0, s, d_items);
    return hipGetLastError();
}

hipError_t launch_stripe(const StripeItem *d_items, int nitems, uint32_t max_n,
                         hipStream_t s) {
    if (!nitems || !max_n) return hipSuccess;
    // tiles of at least STRIPE_TILE - 254 interleaved bytes (N <= 255)
    dim3 g((max_n + STRIPE_TILE - 255) / (STRIPE_TILE - 254), nitems);
    hipLaunchKernelGGL(k_stripe, g, dim3(256), 0, s, d_items);
    return hipGetLastError();
}

hipError_t launch_copy(const CopyItem *d_items, int nitems, hipStream_t s) {
    if (!nitems) return hipSuccess;
    hipLaunchKernelGGL(k_copy, dim3(nitems), dim3(256), 0, s, d_items);
    return hipGetLastError();
}

hipError_t launch_rle_count(const RleItem *items, const uint32_t *chunk_item,
                            int nchunks, uint32_t *cstat, hipStream_t s) {
    if (!nchunks) return hipSuccess;
    hipLaunchKernelGGL(k_rle_count, dim3(nchunks), dim3(256), 0, s, items, chunk_item, cstat);
    return hipGetLastError();
}

hipError_t launch_rle_emit(const RleItem *items, const uint32_t *chunk_item,
                           int nchunks, const uint32_t *cmeta, hipStream_t s) {
    if (!nchunks) return hipSuccess;
    hipLaunchKernelGGL(k_rle_emit, dim3(nchunks), dim3(256), 0, s, items, chunk_item, cmeta);
    return hipGetLastError();
}

hipError_t launch_unrle_count(const UnRleItem *items, const uint32_t *chunk_item,
                              int nchunks, uint32_t *cstat, int what, hipStream_t s) {
    if (!nchunks) return hipSuccess;
    hipLaunchKernelGGL(k_unrle_count, dim3(nchunks), dim3(256), 0, s, items, chunk_item,
                       cstat, what);
    return hipGetLastError();
}

hipError_t launch_unrle_vend(const UnRleItem *items, const uint32_t *chunk_item,
                             int nchunks, const uint32_t *coff, hipStream_t s) {
    if (!nchunks) return hipSuccess;
    hipLaunchKernelGGL(k_unrle_vend, dim3(nchunks), dim3(256), 0, s, items, chunk_item, coff);
    return hipGetLastError();
}

hipError_t launch_unrle_expand(const UnRleItem *items, const uint32_t *chunk_item,
                               int nchunks, const uint32_t *coff, uint32_t *cstat,
                               int what, hipStream_t s) {
    if (!nchunks) return hipSuccess;
    hipLaunchKernelGGL(k_unrle_expand, dim3(nchunks), dim3(256), 0, s, items, chunk_item,
                       coff, cstat, what);
    return hipGetLastError();
}


// ---------------------------------------------------------------------------
// Order-1 encoder tables (build_o1's last loop, rANS_static4x16pr.c:423-518
// with RansEncSymbolInit, rANS_word.h:201-272): workgroup (row, job) scans
// the row's frequencies into starts and writes one EncSym per symbol — the
// host sends 2 bytes per (context, symbol) instead of 16 (a -5 trial batch
// has ~150 jobs of 256 x 256 entries).
__global__ __launch_bounds__(256) void k_enc_tab(const EncTabItem *items) {
    const EncTabItem it = items[blockIdx.y];
    const uint32_t r = blockIdx.x, t = threadIdx.x, A = it.A;
    if (r >= A) return;
    __shared__ uint32_t sc[256];
    const uint32_t f = t < A ? it.f[r * A + t] : 0u;
    sc[t] = f;
    __syncthreads();
    for (uint32_t d = 1; d < 256; d <<= 1) {          // inclusive scan
        const uint32_t v = t >= d ? sc[t - d] : 0u;
        __syncthreads();
        sc[t] += v;
        __syncthreads();
    }
    if (t >= A) return;
    const uint32_t start = sc[t] - f;
    const int bits = int(it.bits);
    EncSym e{0, 0, 0, 0};
    if (f) {                                          // = make_encsym(start, f, bits)
        uint32_t sh;
        e.xmax = ((RANS_LOW >> bits) << 16) * f - 1;
        if (f < 2) {
            e.rcp = ~0u;
            sh = 0;
            e.bias = start + (1u << bits) - 1;
        } else {
            uint32_t sbits = 0;
            while (f > (1u << sbits)) sbits++;
            e.rcp = uint32_t(((1ull << (sbits + 31)) + f - 1) / f);
            sh = sbits - 1;
            e.bias = start;
        }
        e.cmpl_sh = (((1u << bits) - f) & 0xffff) | (sh << 16);
    }
    if (enc_tab_compact(true, A))                     // (kernels.h: 4 B per entry)
        reinterpret_cast<uint32_t *>(it.out)[r * A + t] = f | (start << 13);
    else
        it.out[r * A + t] = e;
}

hipError_t launch_enc_tab(const EncTabItem *d_items, int nitems, hipStream_t s) {
    if (!nitems) return hipSuccess;
    hipLaunchKernelGGL(k_enc_tab, dim3(256, nitems), dim3(256), 0, s, d_items);
    return hipGetLastError();
}

}  // namespace fqz5
