// seq_cm.hip — fqzcomp5's sequence context model (SEQ10 .. SEQ14B,
// fqzcomp5.c:1073-1406) on the GPU.
//
// Encoder.  A k-mer context model (4 u8 counts per context,
// c_small_model.h) plus run-length, literal and state models feed one range
// coder.  A model's counts depend only on the events of that model, so, as
// for fqzcomp_qual (fqz_kernels.hip), every context runs over its own events
// in parallel after a stable sort by context, the side models run in one
// pass over the runs, and the range coder back end (rc_backend,
// fqz_codec.cpp) codes the events in stream order.
//   heads / runs  the block's runs of one class (uppercase ACGT / lowercase
//                 acgt / other bytes), their starts and event counts
//   ctx           per record, the forward k-mer of every base and, in
//                 both-strand mode, the reverse-complement k-mer whose model
//                 counts the base that leaves it (fqzcomp5.c:1176-1199)
//   model         per context, its events in stream order -> {1/total,
//                 freq, cum} of the coded ones
//   side          run-length digits, literal bytes and class switches
// Decoder.  Each symbol selects the next context, so a block is one chain
// (k_seq_dec).
#include <algorithm>
#include <cstdlib>

#include "fqz_model.hpp"
#include "seq_cm.h"

namespace fqz5 {

// fqzcomp5.c:1107-1118
DEV uint32_t seq_class(uint32_t c) {
    switch (c) {
    case 'A': case 'C': case 'G': case 'T': return 0u;
    case 'a': case 'c': case 'g': case 't': return 1u;
    default: return 2u;
    }
}

DEV uint32_t seq_code(uint32_t c) {
    switch (c | 0x20u) {
    case 'a': return 0u;
    case 'c': return 1u;
    case 'g': return 2u;
    default: return 3u;
    }
}

// the stored bit of a class switch (fqzcomp5.c:1120-1124, :1243-1261)
DEV uint32_t switch_bit(uint32_t from, uint32_t to) {
    return to == 0u ? 0u : to == 1u ? uint32_t(from == 2u) : 1u;
}

DEV uint32_t switch_to(uint32_t from, uint32_t bit) {
    if (from == 0u) return bit ? 2u : 1u;
    if (from == 1u) return bit ? 2u : 0u;
    return bit ? 1u : 0u;
}

// the context seeds of fqzcomp5.c:1103-1105
DEV uint32_t seed_fw(uint32_t mask) { return 0x007616c7u & mask; }
DEV uint32_t seed_rv(uint32_t k, uint32_t mask) { return (0x2c6b62ffu >> (32u - 2u * k)) & mask; }

// 4 u8 counts in one word: total, cumulative count below `sym`, update
DEV uint32_t sm4_total(uint32_t F) { return __builtin_amdgcn_sad_u8(F, 0u, 0u); }
DEV uint32_t sm4_cum(uint32_t F, uint32_t sym) {
    return sym ? __builtin_amdgcn_sad_u8(F & ((1u << (8u * sym)) - 1u), 0u, 0u) : 0u;
}
// c_small_model.h:104-131: +1, then halve every count if the total before
// the update was >= 255 (counts stay <= 253, so bytes never carry)
DEV uint32_t sm4_bump(uint32_t F, uint32_t sym, uint32_t tot) {
    F += 1u << (8u * sym);
    if (tot >= 255u) F -= (F >> 1) & 0x7F7F7F7Fu;
    return F;
}

DEV uint4 rc_rec(uint32_t f, uint32_t cum, uint32_t tot) {
    const uint64_t bits = uint64_t(__double_as_longlong(1.0 / double(tot)));
    return make_uint4(uint32_t(bits), uint32_t(bits >> 32), f, cum);
}

// ---------------------------------------------------------------------------
__global__ void k_seq_heads(SeqJob J) {
    const uint32_t p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= J.n) return;
    J.flag[p] = p == 0 || seq_class(J.in[p]) != seq_class(J.in[p - 1]);
}

__global__ void k_seq_run_starts(SeqJob J) {
    const uint32_t p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p < J.n && J.flag[p]) J.run_start[J.ex[p]] = p;
}

// per run: its digit count D = L/255 + 1 plus the switch after it
__global__ void k_seq_run_cnt(SeqJob J) {
    const uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r > J.nrun) return;
    if (r == J.nrun) {
        J.cnt[r] = 0;
        return;
    }
    const uint32_t end = r + 1 < J.nrun ? J.run_start[r + 1] : J.n;
    J.cnt[r] = (end - J.run_start[r]) / 255u + 2u;
}

// event index of the symbol at byte p (seq_cm.h)
DEV uint32_t sym_event(const SeqJob &J, uint32_t p) {
    const uint32_t r = J.ex[p] + J.flag[p] - 1u;
    return p + J.lead + J.run_off[r] + J.cnt[r] - 1u;
}

// The context events, a wave per 64 record segments (contexts restart at a
// segment's start; the 64 segments are one contiguous range of bytes and of
// events).  Per window of SEQ_CTX_W bytes: the wave stages the bytes and
// each forward symbol's event index (sym_event) into LDS with coalesced
// loads, each lane walks its own segment's bytes of the window (the k-mers
// are a serial recurrence) into LDS, and the wave writes the window's keys
// and values out as whole lines.  The value carries the event index of the
// forward symbol, so the model pass writes its record without a gather.
// (Up to round 6 one thread per segment wrote its events itself and a
// separate pass, k_seq_ev, kept a byte -> event table for the model pass to
// gather from: ~8.5 GB of HBM traffic per k_seq_ctx dispatch and one random
// read per event in k_seq_model_runs, profiles/r06_pmc_l5.json.)
constexpr uint32_t SEQ_CTX_W = 2048;
__global__ __launch_bounds__(64) void k_seq_ctx(SeqJob J) {
    __shared__ uint8_t cin[SEQ_CTX_W];
    __shared__ uint32_t cev[SEQ_CTX_W];
    __shared__ uint32_t okey[2 * SEQ_CTX_W];
    __shared__ uint8_t osym[2 * SEQ_CTX_W];
    const uint32_t lane = threadIdx.x;
    const uint32_t s0 = blockIdx.x * 64u;
    const uint32_t s = s0 + lane;
    const bool act = s < J.nseg;
    const uint32_t send = min(s0 + 64u, J.nseg);
    const uint32_t P0 = J.seg[s0], P1 = J.seg[send];
    uint32_t p = act ? J.seg[s] : P1;
    const uint32_t pend = act ? J.seg[s + 1] : P1;
    const uint32_t mask = J.mask, inval = mask + 1u, top = 2u * J.k - 2u;
    const uint32_t both = J.both, sh = both ? 1u : 0u;
    uint32_t fw = seed_fw(mask), rv = seed_rv(J.k, mask);
    for (uint32_t w0 = P0; w0 < P1; w0 += SEQ_CTX_W) {
        const uint32_t wn = min(SEQ_CTX_W, P1 - w0);
        for (uint32_t i = lane; i < wn; i += 64u) {
            const uint32_t c = J.in[w0 + i];
            cin[i] = uint8_t(c);
            cev[i] = seq_class(c) < 2u ? sym_event(J, w0 + i) : 0u;
        }
        __syncthreads();
        const uint32_t stop = min(pend, w0 + wn);
        for (; p < stop; p++) {
            const uint32_t o = (p - w0) << sh;
            const uint32_t c = cin[p - w0];
            if (seq_class(c) < 2u) {
                const uint32_t b = seq_code(c);
                okey[o] = fw;
                osym[o] = uint8_t(b);
                fw = ((fw << 2) + b) & mask;
                if (both) {
                    const uint32_t b2 = rv & 3u;
                    rv = (rv >> 2) + ((3u - b) << top);
                    okey[o + 1] = rv;
                    osym[o + 1] = uint8_t(b2);
                }
            } else {
                okey[o] = inval;
                if (both) okey[o + 1] = inval;
            }
        }
        __syncthreads();
        const uint64_t e0 = uint64_t(w0) << sh;
        for (uint32_t i = lane; i < (wn << sh); i += 64u) {
            const uint32_t k = okey[i];
            J.key[e0 + i] = k;
            J.val[e0 + i] = k == inval ? 0ull
                                       : (uint64_t(2u * cev[i >> sh] + (i & sh)) << 8) | osym[i];
        }
        __syncthreads();
    }
}

// The model pass: per context, the head of its run in the sorted order walks
// it (its counts are a serial recurrence over its events).  The walks are
// latency-bound (a dependent load of the next event per step), so their
// length, not the event count, sets the kernel's time: the contexts that
// every record starts from are the longest (fqzcomp5.c:1176-1199: each
// record restarts at the seed context, so it alone holds one event per
// record, ~300k in a 100 MB block; the next ones a quarter of that, ...).
// Walked one step per ~0.8 us that one run took the whole ~250 ms launch.
//   short runs  one lane each (the lane walks its run)
//   long runs   one wave each, 64 events per round: a coalesced load of the
//               round's events, the count recurrence over them in scalar
//               registers (each lane takes its event's counts with
//               v_writelane), then every lane's record write in parallel
// A workgroup takes a tile of `span` sorted events (about 256 runs), lists
// the heads in it in LDS, walks its long runs a wave each and then its short
// runs a lane each; a run that starts in the tile may end past it (the last
// one counts as long).
constexpr uint32_t SEQ_SPAN_MAX = 4096;
constexpr uint32_t SEQ_LONG = 48;             // events: a wave rather than a lane

DEV void seq_walk(const SeqJob &J, uint32_t i) {
    const uint32_t key = J.skey[i];
    uint32_t F = 0x01010101u;
    for (uint32_t j = i; j < J.nkeys && J.skey[j] == key; j++) {
        const uint64_t v = J.sval[j];
        const uint32_t sym = uint32_t(v) & 3u;
        const uint32_t ord = uint32_t(v >> 8);
        const uint32_t tot = sm4_total(F);
        if (!(ord & 1u)) {
            J.rec[ord >> 1] = rc_rec((F >> (8u * sym)) & 255u, sm4_cum(F, sym), tot);
        }
        F = sm4_bump(F, sym, tot);
    }
}

// Events U.. of a round: lane U takes the counts before its event, then
// they count it (scalar registers; the lane index is an immediate, as gfx9's
// constant bus allows one SGPR per VALU op).
template <int U>
DEV void seq_wave_steps(uint32_t cnt, uint32_t sym, uint32_t &F, uint32_t &myF) {
    if constexpr (U < 64) {
        if (U >= cnt) return;
        const uint32_t su = uint32_t(__builtin_amdgcn_readlane(int(sym), U));
        asm volatile("v_writelane_b32 %0, %1, %2" : "+v"(myF) : "s"(F), "i"(U));
        const uint32_t tot = (F & 255u) + ((F >> 8) & 255u) + ((F >> 16) & 255u) + (F >> 24);
        F += 1u << (8u * su);
        if (tot >= 255u) F -= (F >> 1) & 0x7F7F7F7Fu;
        seq_wave_steps<U + 1>(cnt, sym, F, myF);
    }
}

// the run at i by all 64 lanes of the calling wave (i uniform)
DEV void seq_walk_wave(const SeqJob &J, uint32_t i) {
    const uint32_t l = threadIdx.x & 63u;
    const uint32_t key = __builtin_amdgcn_readfirstlane(J.skey[i]);
    uint32_t F = 0x01010101u;
    uint32_t j = i + l;
    bool in = j < J.nkeys && J.skey[j] == key;
    uint64_t v = in ? J.sval[j] : 0ull;
    for (;;) {
        const uint64_t m = __ballot(in);
        const uint32_t cnt = uint32_t(__popcll(m));   // a prefix of the lanes (sorted keys)
        if (!cnt) break;
        // the next round's events load while this round's recurrence runs
        const uint32_t jn = j + 64u;
        const bool in_n = cnt == 64u && jn < J.nkeys && J.skey[jn] == key;
        const uint64_t vn = in_n ? J.sval[jn] : 0ull;
        const uint32_t sym = uint32_t(v) & 3u;
        uint32_t myF = 0;
        seq_wave_steps<0>(cnt, sym, F, myF);
        if (in) {
            const uint32_t ord = uint32_t(v >> 8);
            if (!(ord & 1u))
                J.rec[ord >> 1] = rc_rec((myF >> (8u * sym)) & 255u, sm4_cum(myF, sym), sm4_total(myF));
        }
        if (cnt < 64u) break;
        j = jn;
        in = in_n;
        v = vn;
    }
}

// (the one-lane-per-event form, $FQZ5_SEQ_MODEL_EVENTS: experiments)
__global__ void k_seq_model(SeqJob J) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= J.nkeys) return;
    const uint32_t key = J.skey[i];
    if (key > J.mask || (i > 0 && J.skey[i - 1] == key)) return;
    seq_walk(J, i);
}

__global__ __launch_bounds__(256) void k_seq_model_runs(SeqJob J, uint32_t span) {
    __shared__ uint32_t heads[SEQ_SPAN_MAX];
    __shared__ uint8_t lng[SEQ_SPAN_MAX];
    __shared__ uint32_t wcnt[4], nh_s;
    const uint32_t t = threadIdx.x, w = t >> 6, l = t & 63u;
    const uint64_t base = uint64_t(blockIdx.x) * span;
    if (t == 0) nh_s = 0;
    __syncthreads();
    for (uint32_t c = 0; c < span; c += 256) {
        const uint64_t i = base + c + t;
        bool h = false;
        if (i < J.nkeys) {
            const uint32_t key = J.skey[i];
            h = key <= J.mask && (i == 0 || J.skey[i - 1] != key);
        }
        const uint64_t m = __ballot(h);
        if (l == 0) wcnt[w] = uint32_t(__popcll(m));
        __syncthreads();
        uint32_t off = nh_s;
        for (uint32_t q = 0; q < w; q++) off += wcnt[q];
        const uint32_t r = __builtin_amdgcn_mbcnt_hi(uint32_t(m >> 32), __builtin_amdgcn_mbcnt_lo(uint32_t(m), 0u));
        if (h) heads[off + r] = uint32_t(i);
        __syncthreads();
        if (t == 0) nh_s += wcnt[0] + wcnt[1] + wcnt[2] + wcnt[3];
        __syncthreads();
    }
    const uint32_t nh = nh_s;
    for (uint32_t h = t; h < nh; h += 256)
        lng[h] = (h + 1 == nh || heads[h + 1] - heads[h] >= SEQ_LONG) ? 1 : 0;
    __syncthreads();
    // long runs: wave w takes those at list positions = w mod 4
    for (uint32_t c = 0; c < nh; c += 64) {
        uint64_t m = __ballot(c + l < nh && lng[c + l] && ((c + l) & 3u) == w);
        while (m) {
            const uint32_t b = uint32_t(__builtin_ctzll(m));
            m &= m - 1;
            seq_walk_wave(J, heads[c + b]);
        }
    }
    for (uint32_t h = t; h < nh; h += 256)
        if (!lng[h]) seq_walk(J, heads[h]);
}

// the run-length, literal and state models over the runs in stream order
__global__ __launch_bounds__(64) void k_seq_side(SeqJob J) {
    __shared__ FList<256> run[3], lit;
    if (threadIdx.x != 0 || J.n == 0) return;
    for (int c = 0; c < 3; c++) fl_init(&run[c], 256);
    fl_init(&lit, 256);
    uint32_t st[3] = {0x0101u, 0x0101u, 0x0101u};   // 2 u8 counts each
    auto put_fl = [&](FList<256> *m, uint32_t sym, uint32_t e) {
        uint32_t acc = 0;
        int k = 1;
        while (m->sy[k] != sym) acc += m->fr[k++];
        J.rec[e] = rc_rec(m->fr[k], acc, m->total);
        fl_bump(m, k);
    };
    auto put_st = [&](uint32_t c, uint32_t bit, uint32_t e) {
        const uint32_t F = st[c], tot = (F & 255u) + (F >> 8);
        J.rec[e] = rc_rec(bit ? F >> 8 : F & 255u, bit ? F & 255u : 0u, tot);
        st[c] = sm4_bump(F, bit, tot);
    };
    const uint32_t n = J.n;
    if (J.lead) {
        put_fl(&run[0], 0u, 0u);
        put_st(0u, switch_bit(0u, seq_class(J.in[0])), 1u);
    }
    for (uint32_t r = 0; r < J.nrun; r++) {
        const uint32_t s = J.run_start[r];
        const uint32_t L = (r + 1 < J.nrun ? J.run_start[r + 1] : n) - s;
        const uint32_t c = seq_class(J.in[s]);
        const uint32_t D = J.cnt[r] - 1u;
        const uint32_t base = s + J.lead + J.run_off[r];   // first digit
        for (uint32_t d = 0; d < D; d++) put_fl(&run[c], d + 1 < D ? 255u : L - 255u * (D - 1u), base + d);
        if (c == 2u)
            for (uint32_t p = s; p < s + L; p++) put_fl(&lit, J.in[p], p + J.lead + J.run_off[r] + D);
        if (r + 1 < J.nrun)
            put_st(c, switch_bit(c, seq_class(J.in[s + L])), base + D + L);
    }
}

// ---------------------------------------------------------------------------
// Decoder: one lane per block runs the chain; models of the k-mer contexts
// in HBM, the side models in LDS.
__global__ void k_seq_models_init(uint32_t *m, size_t n) {
    for (size_t i = size_t(blockIdx.x) * blockDim.x + threadIdx.x; i < n; i += size_t(gridDim.x) * blockDim.x)
        m[i] = 0x01010101u;
}

#ifdef FQZ5_SEQ_PROBE
// shader cycles of the decoder's base steps (block 0): load + symbol,
// renorm + stores, next counts + reverse update, from one step's end to the
// next one's start, steps
__device__ uint64_t g_seqprobe[8];
extern "C" int fqz5_seq_probe_read(uint64_t *out) {
    return int(hipMemcpyFromSymbol(out, HIP_SYMBOL(g_seqprobe), sizeof(g_seqprobe)));
}
#endif

__global__ __launch_bounds__(64) void k_seq_dec(const SeqDecJob *Js) {
    __shared__ FList<256> run[3], lit;
    if (threadIdx.x != 0) return;
    const SeqDecJob J = Js[blockIdx.x];   // one block per workgroup
    for (int c = 0; c < 3; c++) fl_init(&run[c], 256);
    fl_init(&lit, 256);
    uint32_t st[3] = {0x0101u, 0x0101u, 0x0101u};
    const uint8_t *in = J.in;
    const uint32_t len = J.in_len, n = J.n, mask = J.mask, top = 2u * J.k - 2u;
    // input bytes through two 16-byte registers, the next one loaded a
    // register ahead (buffer loads: zero past the end)
    const uint32_t ia = uint32_t(reinterpret_cast<uintptr_t>(in) & 15u);
    const auto rin = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t *>(in - ia), 0,
                                                       int(len + ia), 0x00020000);
    const uint32_t iend = len + ia;
    auto ld16 = [&](uint32_t off) {
        if (off + 16u <= iend) {
            const auto v = __builtin_amdgcn_raw_buffer_load_b128(rin, off, 0, 0);
            return make_uint4(v[0], v[1], v[2], v[3]);
        }
        // the chunk with the end in it: byte loads (a load that straddles
        // the end of the range reads as zero)
        uint32_t w[4] = {0, 0, 0, 0};
        for (uint32_t i = 0; i < 16u; i++)
            w[i >> 2] |= uint32_t(__builtin_amdgcn_raw_buffer_load_b8(rin, off + i, 0, 0)) << (8u * (i & 3u));
        return make_uint4(w[0], w[1], w[2], w[3]);
    };
    uint32_t cb = 0;                                    // cur = buffer bytes [cb, cb + 16)
    uint4 cur = ld16(0), nxt = ld16(16);
    uint32_t ip = 0;
    auto next_byte = [&]() -> uint32_t {
        const uint32_t o = ip++ + ia;
        if (o - cb >= 16u) {                            // bytes are read in order
            cb += 16u;
            cur = nxt;
            nxt = ld16(cb + 16u);
        }
        const uint32_t r = o - cb;
        const uint32_t w = r < 8u ? (r < 4u ? cur.x : cur.y) : (r < 12u ? cur.z : cur.w);
        return (w >> (8u * (r & 3u))) & 255u;
    };
    // range decoder (c_range_coder.h); input past the end stops the chain
    uint32_t code = 0, rng = 0xFFFFFFFFu;
    bool bad = false;
    if (len >= 5) {
        for (int i = 0; i < 5; i++) code = (code << 8) | next_byte();
    } else {
        bad = n > 0;
    }
    auto target = [&](uint32_t tot) -> uint32_t {
        if (!tot || rng < tot) return 0u;
        rng /= tot;
        return code / rng;
    };
    // the next input bytes, MSB first: bb holds bn bits (whole bytes)
    uint64_t bb = 0;
    uint32_t bn = 0;
    auto fill = [&]() {
        while (bn <= 56u) {
            bb |= uint64_t(next_byte()) << (56u - bn);
            bn += 8u;
        }
    };
    auto used = [&]() { return ip - (bn >> 3); };       // bytes the coder has taken
    auto take = [&](uint32_t cum, uint32_t f) {
        code -= cum * rng;
        rng *= f;
        while (rng < (1u << 24)) {
            if (used() >= len) {
                bad = true;
                return;
            }
            if (!bn) fill();
            code = (code << 8) | uint32_t(bb >> 56);
            bb <<= 8;
            bn -= 8u;
            rng <<= 8;
        }
    };
    auto get_fl = [&](FList<256> *m) -> uint32_t {
        const uint32_t t = target(m->total);
        if (t > FL_MAX) {
            bad = true;
            return 0u;
        }
        uint32_t acc = 0;
        int k = 1;
        while (acc + m->fr[k] <= t) acc += m->fr[k++];
        if (k > 256) {
            bad = true;
            return 0u;
        }
        take(acc, m->fr[k]);
        const uint32_t s = m->sy[k];
        fl_bump(m, k);
        return s;
    };
    auto get_st = [&](uint32_t c) -> uint32_t {
        const uint32_t F = st[c], f0 = F & 255u, tot = f0 + (F >> 8);
        const uint32_t bit = target(tot) >= f0;
        take(bit ? f0 : 0u, bit ? F >> 8 : f0);
        st[c] = sm4_bump(F, bit, tot);
        return bit;
    };

    uint32_t fw = seed_fw(mask), rv = seed_rv(J.k, mask);
    uint32_t si = 0, state = 0, p = 0, idle = 0;
    uint32_t F = 0;          // counts of context fw, when have
    bool have = false;
    // the next record start, kept in a register (a reload per symbol would
    // wait for memory: the output stores may alias seg as far as the
    // compiler knows)
    uint32_t next_seg = J.nseg > 1 ? J.seg[1] : 0xFFFFFFFFu;
    uint32_t *M = J.models;
#ifdef FQZ5_SEQ_PROBE
    uint64_t pr_ab = 0, pr_bc = 0, pr_cd = 0, pr_loop = 0, pr_last = 0, pr_n = 0;
#endif
    while (p < n && !bad) {
        uint32_t runlen = 0, d;
        do {
            d = get_fl(&run[state]);
            runlen += d;
        } while (d == 255u && !bad && runlen <= n);
        if (bad) break;
        if (runlen > n - p) runlen = n - p;
        if (runlen == 0 && ++idle > 2) {   // only the first run can be empty
            bad = true;
            break;
        }
        const uint32_t end = p + runlen;
        have = false;
        while (p < end && !bad) {
            if (p == next_seg) {                           // a record starts
                si++;
                next_seg = si + 1 < J.nseg ? J.seg[si + 1] : 0xFFFFFFFFu;
                fw = seed_fw(mask);
                rv = seed_rv(J.k, mask);
                have = false;
            }
            // up to the run's end or the next record start, without
            // per-base checks
            const uint32_t stop = end < next_seg ? end : next_seg;
            if (state == 2u) {
                for (; p < stop && !bad; p++) J.out[p] = uint8_t(get_fl(&lit));
                continue;
            }
            for (; p < stop; p++) {
                // The counts of the 4 contexts that can follow fw (16 aligned
                // bytes) and, both strands, of the 4 reverse contexts the base
                // can lead to are loaded before this step's arithmetic; this
                // step's own stores are patched in below.
#ifdef FQZ5_SEQ_PROBE
                const uint64_t pa = __builtin_amdgcn_s_memtime();
#endif
                if (bn < 8u) fill();                           // one byte is all a step takes
                if (!have) F = M[fw];
                // (u32 loads, the type of the stores, so that the compiler keeps
                // them behind the previous step's stores)
                const uint32_t *wp = M + ((fw << 2) & mask);
                const uint4 win = make_uint4(wp[0], wp[1], wp[2], wp[3]);
                uint32_t rc4[4] = {0, 0, 0, 0};
                if (J.both)
                    for (uint32_t j = 0; j < 4; j++) rc4[j] = M[(rv >> 2) + (j << top)];
                const uint32_t tot = sm4_total(F);
                // symbol: the number of cumulative counts c with c * q <= code
                // (q = range / total; c * q <= range, no overflow)
                const uint32_t q = quot(rng, recip(tot));
                const uint32_t c0 = F & 255u, c1 = c0 + ((F >> 8) & 255u), c2 = c1 + ((F >> 16) & 255u);
                const uint32_t b = uint32_t(c0 * q <= code) + uint32_t(c1 * q <= code) +
                                   uint32_t(c2 * q <= code);
#ifdef FQZ5_SEQ_PROBE
                asm volatile("" :: "v"(b));
                const uint64_t pb = __builtin_amdgcn_s_memtime();
#endif
                // q >= 2^24 / 255, so q * freq >= 2^16: at most one byte in
                code -= sm4_cum(F, b) * q;
                rng = q * ((F >> (8u * b)) & 255u);
                const bool sh = rng < (1u << 24);
                code = sh ? (code << 8) | uint32_t(bb >> 56) : code;
                rng = sh ? rng << 8 : rng;
                bb = sh ? bb << 8 : bb;
                bn -= sh ? 8u : 0u;
                const uint32_t Fu = sm4_bump(F, b, tot);
                M[fw] = Fu;
                J.out[p] = uint8_t(((0x54474341u >> (8u * b)) & 255u) | (state << 5));   // ACGT / acgt
#ifdef FQZ5_SEQ_PROBE
                asm volatile("" :: "v"(code), "v"(rng));
                const uint64_t pc = __builtin_amdgcn_s_memtime();
#endif
                const uint32_t fn = ((fw << 2) + b) & mask;
                uint32_t Fn = b == 0 ? win.x : b == 1 ? win.y : b == 2 ? win.z : win.w;
                if (fn == fw) Fn = Fu;
                if (J.both) {
                    const uint32_t b2 = rv & 3u;
                    const uint32_t j = 3u - b;
                    rv = (rv >> 2) + (j << top);
                    uint32_t G = j == 0 ? rc4[0] : j == 1 ? rc4[1] : j == 2 ? rc4[2] : rc4[3];
                    if (rv == fw) G = Fu;
                    const uint32_t Gu = sm4_bump(G, b2, sm4_total(G));
                    M[rv] = Gu;
                    if (fn == rv) Fn = Gu;
                }
                fw = fn;
                F = Fn;
                have = true;
#ifdef FQZ5_SEQ_PROBE
                asm volatile("" :: "v"(F), "v"(rv));
                const uint64_t pd = __builtin_amdgcn_s_memtime();
                pr_ab += pb - pa;
                pr_bc += pc - pb;
                pr_cd += pd - pc;
                if (pr_last) pr_loop += pa - pr_last;
                pr_last = pd;
                pr_n++;
#endif
            }
        }
        if (p >= n || bad) break;
        state = switch_to(state, get_st(state));
    }
    if (used() > len) bad = true;                      // took bytes past the end
    *J.status = bad ? -1 : 0;
#ifdef FQZ5_SEQ_PROBE
    if (blockIdx.x == 0) {
        g_seqprobe[0] = pr_ab;
        g_seqprobe[1] = pr_bc;
        g_seqprobe[2] = pr_cd;
        g_seqprobe[3] = pr_loop;
        g_seqprobe[4] = pr_n;
    }
#endif
}

// ---------------------------------------------------------------------------
// The decoder with a lookahead of SD bases (k >= SD).  The counts a base
// reads are loaded SD steps before it by the whole wave:
//  - forward: the contexts SD bases after fw are the 4^SD consecutive models
//    ((fw << 2 SD) & mask) + x, one dword per lane (SD = 3: 64 lanes);
//  - reverse (both strands): after SD bases rv becomes (rv >> 2 SD) +
//    (J << (2k - 2 SD)), J < 4^SD: a gather, one model per lane.
// A window is issued at the end of the step 1 + SD before the one it serves
// (after that step's stores), so the last SD steps' stores are not in it:
// those (context, counts) pairs are kept and applied in time order over the
// value read from the window.  At a record or run start the SD windows are
// primed from the first context (window d: 4^d live lanes).  The scalar
// state (coder, contexts, run models) is uniform; every lane runs it.
// ---------------------------------------------------------------------------
constexpr int SD = 3;
__global__ __launch_bounds__(64) void k_seq_dec_la(const SeqDecJob *Js) {
    __shared__ FList<256> run[3], lit;
    const uint32_t l = threadIdx.x;
    const SeqDecJob J = Js[blockIdx.x];   // one block per workgroup
    for (int c = 0; c < 3; c++) fl_init(&run[c], 256);
    fl_init(&lit, 256);
    __builtin_amdgcn_wave_barrier();
    uint32_t st[3] = {0x0101u, 0x0101u, 0x0101u};
    const uint8_t *in = J.in;
    const uint32_t len = J.in_len, n = J.n, mask = J.mask, top = 2u * J.k - 2u;
    const uint32_t ia = uint32_t(reinterpret_cast<uintptr_t>(in) & 15u);
    const auto rin = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t *>(in - ia), 0,
                                                       int(len + ia), 0x00020000);
    const uint32_t iend = len + ia;
    // whole 16-byte chunks through the scalar cache (s_load: lgkmcnt, so the
    // model windows' vmcnt waits do not see them); the chunk with the end in
    // it by bounded byte loads
    const __attribute__((address_space(4))) uint32_t *cin =
        (const __attribute__((address_space(4))) uint32_t *)(uintptr_t(in - ia));
    auto ld16 = [&](uint32_t off) {
        if (off + 16u <= iend) {
            const uint32_t w = off >> 2;
            return make_uint4(cin[w], cin[w + 1], cin[w + 2], cin[w + 3]);
        }
        uint32_t w[4] = {0, 0, 0, 0};
        for (uint32_t i = 0; i < 16u; i++)
            w[i >> 2] |= uint32_t(__builtin_amdgcn_raw_buffer_load_b8(rin, off + i, 0, 0)) << (8u * (i & 3u));
        return make_uint4(__builtin_amdgcn_readfirstlane(w[0]), __builtin_amdgcn_readfirstlane(w[1]),
                          __builtin_amdgcn_readfirstlane(w[2]), __builtin_amdgcn_readfirstlane(w[3]));
    };
    uint32_t cb = 0;
    uint4 cur = ld16(0), nxt = ld16(16);
    uint32_t ip = 0;
    auto next_byte = [&]() -> uint32_t {
        const uint32_t o = ip++ + ia;
        if (o - cb >= 16u) {
            cb += 16u;
            cur = nxt;
            nxt = ld16(cb + 16u);
        }
        const uint32_t r = o - cb;
        const uint32_t w = r < 8u ? (r < 4u ? cur.x : cur.y) : (r < 12u ? cur.z : cur.w);
        return (w >> (8u * (r & 3u))) & 255u;
    };
    uint32_t code = 0, rng = 0xFFFFFFFFu;
    bool bad = false;
    if (len >= 5) {
        for (int i = 0; i < 5; i++) code = (code << 8) | next_byte();
    } else {
        bad = n > 0;
    }
    auto target = [&](uint32_t tot) -> uint32_t {
        if (!tot || rng < tot) return 0u;
        rng /= tot;
        return code / rng;
    };
    uint64_t bb = 0;
    uint32_t bn = 0;
    auto fill = [&]() {
        while (bn <= 56u) {
            bb |= uint64_t(next_byte()) << (56u - bn);
            bn += 8u;
        }
    };
    auto used = [&]() { return ip - (bn >> 3); };
    auto take = [&](uint32_t cum, uint32_t f) {
        code -= cum * rng;
        rng *= f;
        while (rng < (1u << 24)) {
            if (used() >= len) {
                bad = true;
                return;
            }
            if (!bn) fill();
            code = (code << 8) | uint32_t(bb >> 56);
            bb <<= 8;
            bn -= 8u;
            rng <<= 8;
        }
    };
    auto get_fl = [&](FList<256> *m) -> uint32_t {
        const uint32_t t = target(m->total);
        if (t > FL_MAX) {
            bad = true;
            return 0u;
        }
        uint32_t acc = 0;
        int k = 1;
        while (acc + m->fr[k] <= t) acc += m->fr[k++];
        if (k > 256) {
            bad = true;
            return 0u;
        }
        take(acc, m->fr[k]);
        const uint32_t s = m->sy[k];
        __builtin_amdgcn_wave_barrier();
        fl_bump(m, k);
        __builtin_amdgcn_wave_barrier();
        return s;
    };
    auto get_st = [&](uint32_t c) -> uint32_t {
        const uint32_t F = st[c], f0 = F & 255u, tot = f0 + (F >> 8);
        const uint32_t bit = target(tot) >= f0;
        take(bit ? f0 : 0u, bit ? F >> 8 : f0);
        st[c] = sm4_bump(F, bit, tot);
        return bit;
    };

    uint32_t *M = J.models;
    // models and output through buffer ops (vmcnt only, no flat counters)
    const auto rM = __builtin_amdgcn_make_buffer_rsrc(M, 0, int((mask + 1u) * 4u), 0x00020000);
    const auto rO = __builtin_amdgcn_make_buffer_rsrc(J.out, 0, int(n), 0x00020000);
    auto ldM = [&](uint32_t ctx) { return __builtin_amdgcn_raw_buffer_load_b32(rM, ctx * 4u, 0, 0); };
    auto stM = [&](uint32_t ctx, uint32_t v) { __builtin_amdgcn_raw_buffer_store_b32(v, rM, ctx * 4u, 0, 0); };
    const bool both = J.both != 0;
    const uint32_t rsh = 2u * J.k - 2u * SD;   // the reverse window's lane shift, steady state
    // the window ring (lane values) and, per slot, its base context and the
    // reverse window's base and shift
    uint32_t W[SD], R[SD], wb[SD], rb[SD], rs[SD];
    // the stores the windows may miss: per step slot, forward and reverse
    uint32_t hf[SD], hfv[SD], hr[SD], hrv[SD];
    uint32_t fw = seed_fw(mask), rv = seed_rv(J.k, mask);
    uint32_t si = 0, state = 0, p = 0, idle = 0;
    uint32_t F = 0;
    uint32_t next_seg = J.nseg > 1 ? J.seg[1] : 0xFFFFFFFFu;
    // prime the windows from fw / rv for the next SD steps; F = counts of fw
    auto prime = [&]() {
        F = __builtin_amdgcn_readfirstlane(ldM(fw));
#pragma unroll
        for (int d = 1; d <= SD; d++) {
            const int slot = d % SD;
            const uint32_t b0 = (fw << (2 * d)) & mask;
            W[slot] = ldM((b0 + l) & mask);
            wb[slot] = b0;
            if (both) {
                const uint32_t r0 = rv >> (2 * d), sh = 2u * J.k - 2u * uint32_t(d);
                R[slot] = ldM((r0 + (l << sh)) & mask);
                rb[slot] = r0;
                rs[slot] = sh;
            }
        }
#pragma unroll
        for (int i = 0; i < SD; i++) hf[i] = hr[i] = 0xFFFFFFFFu;
    };
    // one base of a record's run, ring position U (= step % SD)
#define SEQ_LA_STEP(U)                                                                          \
    {                                                                                           \
        constexpr int u = (U), n1 = ((U) + 1) % SD;                                             \
        if (bn < 8u) fill();                                                                    \
        const uint32_t tot = sm4_total(F);                                                      \
        const uint32_t q = quot(rng, recip(tot));                                               \
        const uint32_t c0 = F & 255u, c1 = c0 + ((F >> 8) & 255u), c2 = c1 + ((F >> 16) & 255u); \
        const uint32_t b = uint32_t(c0 * q <= code) + uint32_t(c1 * q <= code) +                \
                           uint32_t(c2 * q <= code);                                            \
        code -= sm4_cum(F, b) * q;                                                              \
        rng = q * ((F >> (8u * b)) & 255u);                                                     \
        const bool sh = rng < (1u << 24);                                                       \
        code = sh ? (code << 8) | uint32_t(bb >> 56) : code;                                    \
        rng = sh ? rng << 8 : rng;                                                              \
        bb = sh ? bb << 8 : bb;                                                                 \
        bn -= sh ? 8u : 0u;                                                                     \
        const uint32_t Fu = sm4_bump(F, b, tot);                                                \
        stM(fw, Fu);                                                                            \
        __builtin_amdgcn_raw_buffer_store_b8(uint8_t(((0x54474341u >> (8u * b)) & 255u) | (state << 5)), rO, p, 0, 0); \
        hf[u] = fw;                                                                             \
        hfv[u] = Fu;                                                                            \
        const uint32_t fn = ((fw << 2) + b) & mask;                                             \
        uint32_t Fn = __builtin_amdgcn_readlane(W[n1], (fn - wb[n1]) & 63u);                    \
        uint32_t G = 0, rn = 0;                                                                 \
        if (both) {                                                                             \
            const uint32_t b2 = rv & 3u;                                                        \
            rn = (rv >> 2) + ((3u - b) << top);                                                 \
            G = __builtin_amdgcn_readlane(R[n1], ((rn - rb[n1]) >> rs[n1]) & 63u);              \
            /* the stores since the window, oldest first */                                    \
            _Pragma("unroll") for (int i = 1; i <= SD; i++) {                                   \
                const int h = (u + i) % SD;                                                     \
                if (rn == hf[h]) G = hfv[h];                                                    \
                if (i < SD && rn == hr[h]) G = hrv[h];                                          \
            }                                                                                   \
            const uint32_t Gu = sm4_bump(G, b2, sm4_total(G));                                  \
            stM(rn, Gu);                                                                        \
            hr[u] = rn;                                                                         \
            hrv[u] = Gu;                                                                        \
        }                                                                                       \
        _Pragma("unroll") for (int i = 1; i <= SD; i++) {                                       \
            const int h = (u + i) % SD;                                                         \
            if (fn == hf[h]) Fn = hfv[h];                                                       \
            if (both && fn == hr[h]) Fn = hrv[h];                                               \
        }                                                                                       \
        /* the window SD steps after the next base */                                          \
        const uint32_t nb0 = (fn << (2 * SD)) & mask;                                           \
        W[n1] = ldM((nb0 + l) & mask);                                                          \
        wb[n1] = nb0;                                                                           \
        if (both) {                                                                             \
            const uint32_t r0 = rn >> (2 * SD);                                                 \
            R[n1] = ldM((r0 + (l << rsh)) & mask);                                              \
            rb[n1] = r0;                                                                        \
            rs[n1] = rsh;                                                                       \
            rv = rn;                                                                            \
        }                                                                                       \
        fw = fn;                                                                                \
        F = Fn;                                                                                 \
        p++;                                                                                    \
    }
    while (p < n && !bad) {
        uint32_t runlen = 0, d;
        do {
            d = get_fl(&run[state]);
            runlen += d;
        } while (d == 255u && !bad && runlen <= n);
        if (bad) break;
        if (runlen > n - p) runlen = n - p;
        if (runlen == 0 && ++idle > 2) {
            bad = true;
            break;
        }
        const uint32_t end = p + runlen;
        bool primed = false;
        while (p < end && !bad) {
            if (p == next_seg) {                           // a record starts
                si++;
                next_seg = si + 1 < J.nseg ? J.seg[si + 1] : 0xFFFFFFFFu;
                fw = seed_fw(mask);
                rv = seed_rv(J.k, mask);
                primed = false;
            }
            const uint32_t stop = end < next_seg ? end : next_seg;
            if (state == 2u) {
                for (; p < stop && !bad; p++) __builtin_amdgcn_raw_buffer_store_b8(uint8_t(get_fl(&lit)), rO, p, 0, 0);
                continue;
            }
            if (!primed) {
                prime();
                primed = true;
            }
            // the ring position of p: steps since the priming, mod SD
            while (p + SD <= stop) {
                SEQ_LA_STEP(0)
                SEQ_LA_STEP(1)
                SEQ_LA_STEP(2)
            }
            if (p < stop) SEQ_LA_STEP(0)
            if (p < stop) SEQ_LA_STEP(1)
            // a segment end inside the ring: the next piece starts primed anew
            primed = false;
        }
        if (p >= n || bad) break;
        state = switch_to(state, get_st(state));
    }
#undef SEQ_LA_STEP
    if (used() > len) bad = true;
    if (l == 0) *J.status = bad ? -1 : 0;
}

// ---------------------------------------------------------------------------
static dim3 grid_of(uint64_t n) { return dim3(unsigned((n + 255) / 256)); }

hipError_t launch_seq_heads(const SeqJob &j, hipStream_t s) {
    if (j.n) hipLaunchKernelGGL(k_seq_heads, grid_of(j.n), dim3(256), 0, s, j);
    return hipGetLastError();
}

hipError_t launch_seq_runs(const SeqJob &j, hipStream_t s) {
    if (j.n) hipLaunchKernelGGL(k_seq_run_starts, grid_of(j.n), dim3(256), 0, s, j);
    hipLaunchKernelGGL(k_seq_run_cnt, grid_of(uint64_t(j.nrun) + 1), dim3(256), 0, s, j);
    return hipGetLastError();
}

hipError_t launch_seq_ctx(const SeqJob &j, hipStream_t s) {
    if (j.nseg && j.n) hipLaunchKernelGGL(k_seq_ctx, dim3((j.nseg + 63) / 64), dim3(64), 0, s, j);
    return hipGetLastError();
}

hipError_t launch_seq_model(const SeqJob &j, hipStream_t s) {
    if (!j.nkeys) return hipGetLastError();
    static const bool per_event = std::getenv("FQZ5_SEQ_MODEL_EVENTS") != nullptr;
    if (per_event) {
        hipLaunchKernelGGL(k_seq_model, grid_of(j.nkeys), dim3(256), 0, s, j);
        return hipGetLastError();
    }
    // ~256 runs per tile: the mean run is the events over the contexts
    const uint64_t nctx = std::min<uint64_t>(uint64_t(j.mask) + 1, j.nkeys);
    const uint64_t run = std::min<uint64_t>((j.nkeys + nctx - 1) / nctx, SEQ_SPAN_MAX / 256);
    const uint32_t span = uint32_t(256 * std::max<uint64_t>(run, 1));
    hipLaunchKernelGGL(k_seq_model_runs, dim3(unsigned((j.nkeys + span - 1) / span)), dim3(256), 0, s,
                       j, span);
    return hipGetLastError();
}

hipError_t launch_seq_side(const SeqJob &j, hipStream_t s) {
    if (j.n) hipLaunchKernelGGL(k_seq_side, dim3(1), dim3(64), 0, s, j);
    return hipGetLastError();
}

hipError_t launch_seq_models_init(uint32_t *models, size_t nctx, hipStream_t s) {
    hipLaunchKernelGGL(k_seq_models_init, dim3(1024), dim3(256), 0, s, models, nctx);
    return hipGetLastError();
}

hipError_t launch_seq_dec(const SeqDecJob *d_jobs, int njobs, hipStream_t s, bool lookahead) {
    if (njobs) {
        if (lookahead) hipLaunchKernelGGL(k_seq_dec_la, dim3(njobs), dim3(64), 0, s, d_jobs);
        else hipLaunchKernelGGL(k_seq_dec, dim3(njobs), dim3(64), 0, s, d_jobs);
    }
    return hipGetLastError();
}

}  // namespace fqz5
