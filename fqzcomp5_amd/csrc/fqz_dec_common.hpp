// fqz_dec_common.hpp — pieces shared by the fqzcomp_qual decoders
// (fqz_decode.hip: any alphabet; fqz_decode_small.hip: up to 9 symbols in
// compact models): the staged input window, the range coder's byte reads,
// the small per-record models and the per-record parameter scalars.
// Everything here follows uncompress_block_fqz2f (fqzcomp_qual.c:1410-1634)
// and the range coder of c_range_coder.h.
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>

#include "fqz_kernels.h"
#include "fqz_model.hpp"

namespace fqz5 {
namespace dec {

constexpr uint32_t RING = 4096, HALF = 2048;   // staged input bytes (an LDS ring)

DEV __amdgpu_buffer_rsrc_t rsrc(const void *p, uint32_t n) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void *>(p), 0, n, 0x00020000);
}
DEV uint32_t ld8(__amdgpu_buffer_rsrc_t r, uint32_t off) {
    return __builtin_amdgcn_raw_buffer_load_b8(r, off, 0, 0);
}
DEV void st8(__amdgpu_buffer_rsrc_t r, uint32_t off, uint32_t v) {
    __builtin_amdgcn_raw_buffer_store_b8(uint8_t(v), r, off, 0, 0);
}
DEV uint32_t U(uint32_t v) { return __builtin_amdgcn_readfirstlane(v); }
DEV uint32_t RL(uint32_t v, uint32_t lane) { return __builtin_amdgcn_readlane(v, lane); }

// ---------------------------------------------------------------------------
// input: a 4 KB LDS ring at byte RO of the workgroup's LDS, refilled 2 KB at
// a time, read through a 64-bit big-endian window W: `vb` bytes from stream
// position `rb` were valid at the last refill, `ub` bits have been shifted
// out since.
// ---------------------------------------------------------------------------
struct In {
    __amdgpu_buffer_rsrc_t r;
    uint32_t len, rb, ub, vb, lp;
    uint64_t W;
    DEV uint32_t rp() const { return rb + (ub >> 3); }
    DEV uint32_t avail() const { return vb - (ub >> 3); }
};

template <uint32_t RO> DEV void stage(uint8_t *lds, const In &in) {
    const uint32_t l = threadIdx.x;
    const uint32_t src = in.lp + 32 * l;
    uint32_t w[8];
#pragma unroll
    for (int i = 0; i < 8; i++)
        w[i] = ld8(in.r, src + 4 * i) | ld8(in.r, src + 4 * i + 1) << 8 |
               ld8(in.r, src + 4 * i + 2) << 16 | ld8(in.r, src + 4 * i + 3) << 24;
    const uint32_t at = RO + (in.lp & (RING - 1)) + 32 * l;
    *reinterpret_cast<uint4 *>(lds + at) = make_uint4(w[0], w[1], w[2], w[3]);
    *reinterpret_cast<uint4 *>(lds + at + 16) = make_uint4(w[4], w[5], w[6], w[7]);
    if ((in.lp & (RING - 1)) == 0 && l == 0)   // mirror for reads across the end
        *reinterpret_cast<uint4 *>(lds + RO + RING) = make_uint4(w[0], w[1], w[2], w[3]);
}

template <uint32_t RO> DEV void refill(uint8_t *lds, In &in) {
    const uint32_t rp = in.rp();
    if (in.lp - rp < HALF) {
        stage<RO>(lds, in);
        in.lp += HALF;
    }
    const uint32_t i = rp & (RING - 1), a = i & ~7u, sh = (i & 7u) * 8u;
    const uint64_t lo = *reinterpret_cast<const uint64_t *>(lds + RO + a);
    const uint64_t hi = *reinterpret_cast<const uint64_t *>(lds + RO + a + 8);
    const uint64_t v = sh ? (lo >> sh) | (hi << (64u - sh)) : lo;
    const uint64_t be = __builtin_bswap64(v);
    in.W = (uint64_t(U(uint32_t(be >> 32))) << 32) | U(uint32_t(be));
    const uint32_t rem = in.len - rp;
    in.vb = rem < 8u ? rem : 8u;
    in.rb = rp;
    in.ub = 0;
}

// the coder's start (RC_StartDecode: 5 bytes into code)
template <uint32_t RO> DEV void in_start(uint8_t *lds, In &in, const uint8_t *p, uint32_t n, uint32_t &code) {
    in.r = rsrc(p, n);
    in.len = n;
    in.lp = 0;
    stage<RO>(lds, in);
    in.lp = HALF;
    stage<RO>(lds, in);
    in.lp = RING;
    in.rb = in.ub = in.vb = 0;
    in.W = 0;
    __builtin_amdgcn_wave_barrier();
    code = 0;
    if (in.len >= 5) {
        refill<RO>(lds, in);
        for (int k = 0; k < 5; k++) {
            code = (code << 8) | uint32_t(in.W >> 56);
            in.W <<= 8;
        }
        in.ub = 40;
        refill<RO>(lds, in);
    } else {
        in.rb = in.len;
    }
}

// one byte into the coder (the reference's renormalisation reads, with its
// end-of-input stop, c_range_coder.h RC_GetFreq / RC_Decode)
template <uint32_t RO> DEV bool take_byte(uint8_t *lds, In &in, uint32_t &code) {
    if (in.rp() >= in.len) return false;
    code = (code << 8) | uint32_t(in.W >> 56);
    in.W <<= 8;
    in.ub += 8;
    if (in.avail() < 4u) refill<RO>(lds, in);
    return true;
}

template <uint32_t RO> DEV void renorm_slow(uint8_t *lds, In &in, uint32_t &rng, uint32_t &code) {
    while (rng < (1u << 24)) {
        if (!take_byte<RO>(lds, in, code)) break;
        rng <<= 8;
    }
}

// a small model (selector / length bytes / reverse / duplicate) in LDS,
// decoded serially with the reference's arithmetic
template <uint32_t RO, int CAP> DEV uint32_t small_decode(FList<CAP> *m, uint8_t *lds, In &in, uint32_t &rng,
                                                          uint32_t &code) {
    const uint32_t tot = U(m->total);
    uint32_t t = 0;
    if (tot && rng >= tot) {
        rng /= tot;
        t = code / rng;
    }
    if (t > FL_MAX) return 0;
    uint32_t acc = 0;
    int k = 1;
    while ((acc += U(m->fr[k])) <= t) k++;
    if (k - 1 > CAP) return 0;
    const uint32_t f = U(m->fr[k]);
    acc -= f;
    code -= acc * rng;
    rng *= f;
    renorm_slow<RO>(lds, in, rng, code);
    const uint32_t s = U(m->sy[k]);
    if (threadIdx.x == 0) fl_bump(m, k);
    __builtin_amdgcn_wave_barrier();
    return s;
}

template <int CAP> DEV void small_init(FList<CAP> *m, int live) {
    const int l = threadIdx.x;
    if (l == 0) {
        m->fr[0] = uint16_t(FL_MAX);
        m->sy[0] = 0;
        m->fr[CAP + 1] = 0;
        m->sy[CAP + 1] = 0;
        m->fr[CAP + 2] = uint16_t(FL_MAX);
        m->sy[CAP + 2] = 0;
        m->total = uint32_t(live);
    }
    for (int k = l; k < CAP; k += 64) {
        m->sy[k + 1] = uint8_t(k);
        m->fr[k + 1] = k < live ? 1 : 0;
    }
}

DEV void small_models_init(SmallModels &sm, const FqzDevGlobal &g) {
    for (int b = 0; b < 4; b++) small_init(&sm.len[b], 256);
    small_init(&sm.rev, 2);
    small_init(&sm.dup, 2);
    if (U(g.max_sel) > 0) small_init(&sm.sel, int(U(g.max_sel)) + 1);
}

// per-record parameter scalars (fqzcomp_qual.c:1067-1076)
struct PS {
    uint32_t x, ctx0, qshift, qloc, qmask, sloc, bbits, bloc, boff, sel, dedup, fixed;
};

DEV PS load_ps(const FqzDevGlobal &g, uint32_t x) {
    const FqzDevParam &p = g.p[x];
    return PS{x, U(p.ctx0), U(p.qshift), U(p.qloc), U(p.qmask), U(p.sloc), U(p.bbits), U(p.bloc),
              U(p.boff), U(p.sel), U(p.dedup), U(p.fixed)};
}

}  // namespace dec
}  // namespace fqz5
