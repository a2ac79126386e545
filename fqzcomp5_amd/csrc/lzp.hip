// lzp.hip — fqzcomp5's LZP pre-pass on the GPU (lzp16e.c:113-214), the
// first stage of the LZP3 sequence method (fqzcomp5.c:2013-2021).
//
// Encoder.  The reference walks the block once, keeping a 2^16-entry table
// ht[h] of the last position seen with hash h.  Every position enters the
// table (ht[h_i] = i, literal or inside a match, lzp16e.c:140-159), and the
// hash update keeps 16 bits of ((h*K)<<4) + 544h, XORed with the byte, so
// bits 0..k of h_{i+1} depend only on bits 0..k-4 of h_i: h_i is a function
// of the 4 bytes before i alone.  Hence, with no serial pass:
//   h_i      from in[i-4..i-1] (positions 0..3 from the start value 0)
//   pred_i   the last j < i with h_j == h_i: a stable sort of positions by
//            hash, then the neighbour in the sorted order (ht[h] == 0 for
//            "none" also covers j == 0, as in the reference)
//   L_i      the common prefix of in[i..] and in[pred_i..] (capped 65535):
//            L_i = 1 + L_{i+1} when in[i] == in[pred_i] and pred_{i+1} ==
//            pred_i + 1, so L is a backward segmented scan whose segment
//            ends are computed directly.  An end i has distance d = i -
//            pred_i; its common prefix is the run of in[k] == in[k - d] from
//            i.  Ends sorted by (d, i): each compares bytes only up to the
//            next end of the same distance, and when it gets there its run
//            continues that end's (a second segmented scan).  Periodic input
//            (the comments of a name block) thus costs a few bytes per end
//            instead of up to 65535.
//   tokens   a match of L_i >= 3 at i jumps to i + L_i, else i + 1.  Each
//            64 KiB chunk parses from its own start speculatively; one walk
//            joins them (the true path runs serially only until it meets a
//            chunk's speculative path, after which the two coincide)
//   bytes    marker + length (2 or 3 B), an escaped literal (233 0 c) where a
//            prediction exists and the byte is 233/234, or the byte; written
//            at the exclusive scan of the token sizes.
//
// Decoder: one wave per block (below).
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include "lzp.h"

namespace fqz5 {

#define DEV __device__ __forceinline__

// lzp16e.c:102, in u32 arithmetic (the low 16 bits do not depend on how the
// reference's signed multiply wraps)
DEV uint32_t lzp_upd(uint32_t h, uint32_t c) {
    return ((((h * 0x8ca6b53u) << 4) + (h << 5) * 17u) ^ c) & 0xffffu;
}

__global__ void k_lzp_hash(LzpEncJob J) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= J.n) return;
    uint32_t h = 0;
    for (uint32_t k = i >= 4 ? i - 4 : 0; k < i; k++) h = lzp_upd(h, J.in[k]);
    J.key[i] = h;
    J.val[i] = i;
}

__global__ void k_lzp_pred(LzpEncJob J) {
    const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= J.n) return;
    const uint32_t i = J.sval[k];
    J.pred[i] = (k > 0 && J.skey[k - 1] == J.skey[k]) ? J.sval[k - 1] : 0u;
}

// Segment ends of the backward length scan: position i links to i+1 when
// in[i] == in[p] and pred[i+1] == p+1 (p = pred[i] > 0).  rev[n-1-i] = i at
// an end, UINT32_MAX where linked.  An end with in[i] != in[p] has length 0
// (base[i]); the others get key = their distance i - p for the sort by
// (distance, position), every other position the key n (last).
__global__ void k_lzp_stops(LzpEncJob J) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t n = J.n;
    if (i >= n) return;
    const uint32_t p = J.pred[i];
    const bool eq = p > 0 && J.in[i] == J.in[p];
    const bool link = eq && i + 1 < n && J.pred[i + 1] == p + 1;
    J.val[i] = i;
    J.key[i] = (!link && eq) ? i - p : n;
    if (link) {
        J.rev[n - 1 - i] = 0xffffffffu;
        return;
    }
    J.rev[n - 1 - i] = i;
    if (!eq) J.base[i] = 0;
}

// Ends in (distance, position) order, k-th: compare from i = sval[k] at
// distance d up to the next end of the same distance (or the cap / the
// block end).  Reaching it links k to k+1 (rev2[n-1-k] = UINT32_MAX);
// otherwise the run length is direct (dl[k]).  dl aliases key, rev2 val.
__global__ void k_lzp_endscan(LzpEncJob J) {
    const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t n = J.n;
    if (k >= n) return;
    const uint32_t d = J.skey[k];
    uint32_t *dl = J.key, *rev2 = J.val;
    if (d >= n) {                                  // not an end to measure
        rev2[n - 1 - k] = k;
        dl[k] = 0;
        return;
    }
    const uint32_t i = J.sval[k];
    const bool has_next = k + 1 < n && J.skey[k + 1] == d;
    const uint32_t left = n - i;
    const uint32_t lim = left < LZP_MAX_LEN ? left : LZP_MAX_LEN;
    const uint32_t gap = has_next ? J.sval[k + 1] - i : 0xffffffffu;
    const uint32_t stop = gap < lim ? gap : lim;
    const uint8_t *a = J.in + i, *b = J.in + (i - d);
    uint32_t L = 0;
    while (L < stop && a[L] == b[L]) L++;
    const bool linked = has_next && gap < lim && L == gap;
    rev2[n - 1 - k] = linked ? 0xffffffffu : k;
    dl[k] = L;
}

// After the min-scan of rev2 (into off): the first unlinked end k2 >= k of
// the same distance; the run from i is (i2 - i) + dl[k2], capped.
__global__ void k_lzp_resolve(LzpEncJob J) {
    const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t n = J.n;
    if (k >= n || J.skey[k] >= n) return;
    const uint32_t i = J.sval[k];
    const uint32_t k2 = J.off[n - 1 - k];
    const uint64_t L = uint64_t(J.sval[k2] - i) + J.key[k2];
    J.base[i] = L > LZP_MAX_LEN ? LZP_MAX_LEN : uint32_t(L);
}

// match length per position: the next segment end e >= i gives
// L_i = (e - i) + base[e]; a match needs a prediction and L >= 3
__global__ void k_lzp_lengths(LzpEncJob J) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t n = J.n;
    if (i >= n) return;
    uint32_t ml = 0;
    if (J.pred[i] > 0) {
        const uint32_t e = J.nxt[n - 1 - i];
        const uint64_t L = uint64_t(e - i) + J.base[e];
        const uint32_t Lc = L > LZP_MAX_LEN ? LZP_MAX_LEN : uint32_t(L);
        ml = Lc >= LZP_MIN_LEN ? Lc : 0u;
    }
    J.ml[i] = uint16_t(ml);
}

// speculative parse of each chunk from its first position
__global__ void k_lzp_chunks(LzpEncJob J) {
    const uint32_t c = blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= J.nchunk) return;
    uint64_t pos = uint64_t(c) * LZP_CHUNK;
    const uint64_t end = pos + LZP_CHUNK < J.n ? pos + LZP_CHUNK : J.n;
    while (pos < end) {
        J.spec[pos] = 1;
        const uint32_t m = J.ml[pos];
        pos += m ? m : 1u;
    }
    J.exitp[c] = uint32_t(pos);
}

// the true path: walk until it meets the speculative path of its chunk, then
// jump to that chunk's exit (one thread; O(chunks) when the parses agree)
__global__ void k_lzp_walk(LzpEncJob J) {
    if (threadIdx.x || blockIdx.x) return;
    uint32_t pos = 0;
    const uint32_t n = J.n;
    while (pos < n) {
        const uint32_t c = pos / LZP_CHUNK;
        if (J.spec[pos]) {
            J.conv[c] = pos;
            pos = J.exitp[c];
            continue;
        }
        J.walk[pos] = 1;
        const uint32_t m = J.ml[pos];
        pos += m ? m : 1u;
    }
}

DEV bool lzp_start(const LzpEncJob &J, uint32_t i) {
    return J.walk[i] || (J.spec[i] && i >= J.conv[i / LZP_CHUNK]);
}

__global__ void k_lzp_sizes(LzpEncJob J) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= J.n) return;
    uint32_t sz = 0;
    if (lzp_start(J, i)) {
        const uint32_t m = J.ml[i];
        const uint32_t c = J.in[i];
        sz = m ? (m <= 255 ? 2u : 3u)
               : (J.pred[i] > 0 && (c == LZP_MARK || c == LZP_MARK + 1) ? 3u : 1u);
    }
    J.size[i] = sz;
}

__global__ void k_lzp_emit(LzpEncJob J) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t n = J.n;
    if (i >= n) return;
    const uint32_t sz = J.size[i];
    if (i == n - 1) *J.out_len = J.off[i] + sz;
    if (!sz) return;
    uint8_t *o = J.out + J.off[i];
    const uint32_t m = J.ml[i];
    const uint8_t c = J.in[i];
    if (m) {
        if (m <= 255) {
            o[0] = LZP_MARK;
            o[1] = uint8_t(m);
        } else {
            o[0] = LZP_MARK + 1;
            o[1] = uint8_t(m >> 8);
            o[2] = uint8_t(m);
        }
    } else if (sz == 3) {
        o[0] = LZP_MARK;
        o[1] = 0;
        o[2] = c;
    } else {
        o[0] = c;
    }
}

static dim3 grid_of(uint32_t n, uint32_t b = 256) { return dim3((n + b - 1) / b ? (n + b - 1) / b : 1); }

hipError_t launch_lzp_hash(const LzpEncJob &j, hipStream_t s) {
    if (j.n) hipLaunchKernelGGL(k_lzp_hash, grid_of(j.n), dim3(256), 0, s, j);
    return hipGetLastError();
}
hipError_t launch_lzp_pred(const LzpEncJob &j, hipStream_t s) {
    if (j.n) hipLaunchKernelGGL(k_lzp_pred, grid_of(j.n), dim3(256), 0, s, j);
    return hipGetLastError();
}
hipError_t launch_lzp_stops(const LzpEncJob &j, hipStream_t s) {
    if (j.n) hipLaunchKernelGGL(k_lzp_stops, grid_of(j.n), dim3(256), 0, s, j);
    return hipGetLastError();
}
hipError_t launch_lzp_endscan(const LzpEncJob &j, hipStream_t s) {
    if (j.n) hipLaunchKernelGGL(k_lzp_endscan, grid_of(j.n), dim3(256), 0, s, j);
    return hipGetLastError();
}
hipError_t launch_lzp_resolve(const LzpEncJob &j, hipStream_t s) {
    if (j.n) hipLaunchKernelGGL(k_lzp_resolve, grid_of(j.n), dim3(256), 0, s, j);
    return hipGetLastError();
}
hipError_t launch_lzp_lengths(const LzpEncJob &j, hipStream_t s) {
    if (j.n) hipLaunchKernelGGL(k_lzp_lengths, grid_of(j.n), dim3(256), 0, s, j);
    return hipGetLastError();
}
hipError_t launch_lzp_parse(const LzpEncJob &j, hipStream_t s) {
    if (!j.n) return hipSuccess;
    hipLaunchKernelGGL(k_lzp_chunks, grid_of(j.nchunk, 64), dim3(64), 0, s, j);
    hipLaunchKernelGGL(k_lzp_walk, dim3(1), dim3(64), 0, s, j);
    return hipGetLastError();
}
hipError_t launch_lzp_sizes(const LzpEncJob &j, hipStream_t s) {
    if (j.n) hipLaunchKernelGGL(k_lzp_sizes, grid_of(j.n), dim3(256), 0, s, j);
    return hipGetLastError();
}
hipError_t launch_lzp_emit(const LzpEncJob &j, hipStream_t s) {
    if (j.n) hipLaunchKernelGGL(k_lzp_emit, grid_of(j.n), dim3(256), 0, s, j);
    return hipGetLastError();
}

hipError_t lzp_sort(const LzpEncJob &j, void *tmp, size_t &bytes, hipStream_t s) {
    return hipcub::DeviceRadixSort::SortPairs(tmp, bytes, j.key, j.skey, j.val, j.sval, int(j.n),
                                              0, int(LZP_HASH_BITS), s);
}
hipError_t lzp_min_scan(const LzpEncJob &j, void *tmp, size_t &bytes, hipStream_t s) {
    return hipcub::DeviceScan::InclusiveScan(tmp, bytes, j.rev, j.nxt, hipcub::Min(), int(j.n), s);
}
static int bits_of(uint32_t n) { return n ? 32 - __builtin_clz(n) : 1; }
hipError_t lzp_sort_ends(const LzpEncJob &j, void *tmp, size_t &bytes, hipStream_t s) {
    return hipcub::DeviceRadixSort::SortPairs(tmp, bytes, j.key, j.skey, j.val, j.sval, int(j.n),
                                              0, bits_of(j.n), s);
}
hipError_t lzp_end_scan(const LzpEncJob &j, void *tmp, size_t &bytes, hipStream_t s) {
    return hipcub::DeviceScan::InclusiveScan(tmp, bytes, j.val, j.off, hipcub::Min(), int(j.n), s);
}
hipError_t lzp_size_scan(const LzpEncJob &j, void *tmp, size_t &bytes, hipStream_t s) {
    return hipcub::DeviceScan::ExclusiveSum(tmp, bytes, j.size, j.off, int(j.n), s);
}

// ---------------------------------------------------------------------------
// Decoder (unlzp, lzp16e.c:166-214), one wave per block.
//
// A token starting with a byte other than 233/234 is a literal whatever the
// table holds (with a prediction the reference reads it as a zero-length
// "match" and steps back, :201).  So a window of 64 input bytes up to its
// first marker byte is a run of literals: the lanes write them and enter
// their positions in the table (atomic max: positions only grow, so the
// largest is the last), each hash from the 4 bytes before it.  A marker byte
// needs the table entry of its position: with none it is a literal itself;
// otherwise it carries a length (0: an escaped literal follows) and a match
// copies from out[pred..] forward (an overlapping copy repeats with period
// op - pred), 64 bytes per step.  Table and output reads are coherent
// (agent-scope loads after the wave's stores and atomics have completed).

DEV uint32_t lzp_hash4(uint32_t b4, uint32_t b3, uint32_t b2, uint32_t b1) {
    return lzp_upd(lzp_upd(lzp_upd(lzp_upd(0, b4), b3), b2), b1);
}

DEV uint32_t ld_coherent_u8(const uint8_t *p) {
    const uintptr_t a = reinterpret_cast<uintptr_t>(p);
    uint32_t *w = reinterpret_cast<uint32_t *>(a & ~uintptr_t(3));
    const uint32_t v = __hip_atomic_load(w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return (v >> (8 * (a & 3))) & 0xffu;
}

// the wave's earlier stores and table atomics are performed before what follows
DEV void wait_mem() { __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "agent"); }

// Hash of position P (the state before byte P is added), with `byte(q)`
// giving output byte q for q in [P-4, P).  Positions 0..3 from the start
// value 0 (lzp16e.c:117).
template <class B>
DEV uint32_t lzp_hash_at(uint32_t P, B byte) {
    if (P >= 4) return lzp_hash4(byte(P - 4), byte(P - 3), byte(P - 2), byte(P - 1));
    uint32_t h = 0;
    for (uint32_t q = 0; q < P; q++) h = lzp_upd(h, byte(q));
    return h;
}

__global__ __launch_bounds__(64) void k_lzp_dec(const LzpDecJob *jobs) {
    const LzpDecJob J = jobs[blockIdx.x];
    const uint32_t l = threadIdx.x;
    uint32_t ip = 0, op = 0;
    uint32_t last4 = 0;          // byte k = out[op-1-k]
    int32_t st = 0;
    auto hist = [&](uint32_t q) -> uint32_t { return (last4 >> (8 * (op - 1 - q))) & 0xffu; };
    while (ip < J.in_len) {
        const uint32_t q = ip + l;
        const uint32_t b = q < J.in_len ? J.in[q] : 0x100u;
        const uint64_t mk = __ballot(b == LZP_MARK || b == LZP_MARK + 1 || b == 0x100u);
        const uint32_t R = mk ? uint32_t(__builtin_ctzll(mk)) : 64u;
        if (R) {                                       // a run of literals
            if (op + R > J.cap) { st = -1; break; }
            // byte of position P (P < op: history; else lane P - op)
            const uint32_t bsh1 = __shfl_up(b, 1), bsh2 = __shfl_up(b, 2), bsh3 = __shfl_up(b, 3),
                           bsh4 = __shfl_up(b, 4);
            const uint32_t P = op + l;
            auto byte = [&](uint32_t x) -> uint32_t {
                if (x < op) return hist(x);
                const uint32_t d = P - x;             // 1..4
                return d == 1 ? bsh1 : d == 2 ? bsh2 : d == 3 ? bsh3 : bsh4;
            };
            if (l < R) {
                const uint32_t h = lzp_hash_at(P, byte);
                J.out[P] = uint8_t(b);
                if (P) __hip_atomic_fetch_max(J.ht + h, P, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
            // the 4 bytes before op + R
            uint32_t nl = 0;
            for (uint32_t k = 0; k < 4; k++) {
                const uint32_t x = op + R - 1 - k;    // position
                uint32_t v = 0;
                if (x < op + R && op + R >= k + 1) {
                    v = x < op ? hist(x) : __shfl(b, int(x - op));
                }
                nl |= (v & 0xffu) << (8 * k);
            }
            last4 = nl;
            ip += R;
            op += R;
            continue;
        }
        // a marker byte at ip: the table entry of position op decides
        auto byte0 = [&](uint32_t x) -> uint32_t { return hist(x); };
        const uint32_t h = lzp_hash_at(op, byte0);
        wait_mem();
        const uint32_t p = __hip_atomic_load(J.ht + h, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const uint32_t b0 = __shfl(b, 0);
        uint32_t ml = 0, adv = 1, lit = b0;
        if (p) {
            if (b0 == LZP_MARK) {
                if (ip + 1 >= J.in_len) { st = -1; break; }
                ml = __shfl(b, 1);
                adv = 2;
            } else {
                if (ip + 2 >= J.in_len) { st = -1; break; }
                ml = (__shfl(b, 1) << 8) | __shfl(b, 2);
                adv = 3;
            }
            if (!ml) {
                if (ip + adv >= J.in_len) { st = -1; break; }
                lit = __shfl(b, int(adv));
                adv++;
            }
        }
        if (!ml) {                                     // one literal
            if (op + 1 > J.cap) { st = -1; break; }
            if (l == 0) {
                J.out[op] = uint8_t(lit);
                if (op) __hip_atomic_fetch_max(J.ht + h, op, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
            last4 = (last4 << 8) | lit;
            op++;
            ip += adv;
            continue;
        }
        if (op + ml > J.cap) { st = -1; break; }
        // the match: out[op + k] = out[p + k % d], d = op - p, 64 bytes a step
        const uint32_t d = op - p;
        wait_mem();
        for (uint32_t k0 = 0; k0 < ml; k0 += 64) {
            const uint32_t k = k0 + l;
            const bool act = k < ml;
            const uint32_t v = act ? ld_coherent_u8(J.out + p + (k % d)) : 0u;
            const uint32_t vsh1 = __shfl_up(v, 1), vsh2 = __shfl_up(v, 2), vsh3 = __shfl_up(v, 3),
                           vsh4 = __shfl_up(v, 4);
            const uint32_t base = op + k0;            // first position of this step
            const uint32_t P = base + l;
            auto byte = [&](uint32_t x) -> uint32_t {
                if (x < base) return (last4 >> (8 * (base - 1 - x))) & 0xffu;
                const uint32_t dd = P - x;
                return dd == 1 ? vsh1 : dd == 2 ? vsh2 : dd == 3 ? vsh3 : vsh4;
            };
            if (act) {
                const uint32_t hh = lzp_hash_at(P, byte);
                J.out[P] = uint8_t(v);
                if (P) __hip_atomic_fetch_max(J.ht + hh, P, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
            const uint32_t cnt = ml - k0 < 64 ? ml - k0 : 64;
            uint32_t nl = 0;
            for (uint32_t t = 0; t < 4; t++) {
                const uint32_t x = base + cnt - 1 - t;
                uint32_t w = 0;
                if (base + cnt >= t + 1) w = x < base ? (last4 >> (8 * (base - 1 - x))) & 0xffu
                                                      : __shfl(v, int(x - base));
                nl |= (w & 0xffu) << (8 * t);
            }
            last4 = nl;
        }
        op += ml;
        ip += adv;
    }
    wait_mem();
    if (l == 0) {
        *J.out_len = op;
        *J.status = st;
    }
}

hipError_t launch_lzp_dec(const LzpDecJob *d_jobs, int njobs, hipStream_t s) {
    if (njobs) hipLaunchKernelGGL(k_lzp_dec, dim3(njobs), dim3(64), 0, s, d_jobs);
    return hipGetLastError();
}

}  // namespace fqz5
