// fqz_model.hpp — the adaptive frequency list of fqzcomp_qual
// (c_simple_model.h) and the small per-record models, shared by the
// encoder (fqz_kernels.hip) and the decoder (fqz_decode.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>

#include "fqz_kernels.h"

namespace fqz5 {

#define DEV __device__ __forceinline__

// A job struct from device memory (one per block of a batched launch), read
// word by word through readfirstlane: every field is then a scalar register
// and the compiler keeps the code that depends on it uniform, as with a
// by-value kernel argument.
template <class T> DEV T load_job(const T *p) {
    static_assert(sizeof(T) % 4 == 0, "job size");
    T v;
    const uint32_t *src = reinterpret_cast<const uint32_t *>(p);
    uint32_t *dst = reinterpret_cast<uint32_t *>(&v);
#pragma unroll
    for (unsigned i = 0; i < sizeof(T) / 4; i++) dst[i] = __builtin_amdgcn_readfirstlane(src[i]);
    return v;
}

// --------------------------------------------------------------------------
// adaptive frequency lists (c_simple_model.h:63-171)
// --------------------------------------------------------------------------
// Slot 0: permanent head (never loses the bubble comparison); slots 1..CAP:
// symbols in approximate descending frequency; CAP+1: zero terminator of
// the halving loop; CAP+2: maximal terminator of a decode scan.
constexpr uint32_t FL_MAX = 65519u;   // (1<<16)-17
constexpr uint32_t FL_STEP = 16u;

template <int CAP> struct FList {
    uint32_t total;
    uint16_t fr[CAP + 3];
    uint8_t sy[CAP + 3];
};
static_assert(sizeof(FList<FQZ_QSYMS>) == FQZ_QMODEL_BYTES, "qual model size");

template <int CAP> DEV void fl_init(FList<CAP> *m, int live) {
    m->fr[0] = uint16_t(FL_MAX);
    m->sy[0] = 0;
    for (int k = 0; k < CAP; k++) {
        m->sy[k + 1] = uint8_t(k);
        m->fr[k + 1] = k < live ? 1 : 0;
    }
    m->fr[CAP + 1] = 0;
    m->sy[CAP + 1] = 0;
    m->fr[CAP + 2] = uint16_t(FL_MAX);
    m->sy[CAP + 2] = 0;
    m->total = uint32_t(live);
}

template <int CAP> DEV void fl_bump(FList<CAP> *m, int k) {
    m->fr[k] += FL_STEP;
    m->total += FL_STEP;
    if (m->total > FL_MAX) {
        uint32_t t = 0;
        for (int i = 1; m->fr[i]; i++) {
            m->fr[i] = uint16_t(m->fr[i] - (m->fr[i] >> 1));
            t += m->fr[i];
        }
        m->total = t;
    }
    if (m->fr[k] > m->fr[k - 1]) {
        const uint16_t f = m->fr[k];
        const uint8_t s = m->sy[k];
        m->fr[k] = m->fr[k - 1];
        m->sy[k] = m->sy[k - 1];
        m->fr[k - 1] = f;
        m->sy[k - 1] = s;
    }
}

// floor(range / t) without a division (decoders): RN(1/t) to within one
// ulp from the hardware reciprocal plus one Newton step, then
// q = (u32)fma(range, RN(1/t), 2^-19), exact for range < 2^32 and t < 2^16
// (fqz_div_selftest checks every t).
// RN(1/t) to within one ulp: hardware reciprocal plus one Newton step.
DEV double recip(uint32_t t) {
    const double d = double(t);
    const double r = __builtin_amdgcn_rcp(d);
    const double e = __fma_rn(-d, r, 1.0);
    return __fma_rn(r, e, r);
}
DEV uint32_t quot(uint32_t rng, double rd) { return uint32_t(__fma_rn(double(rng), rd, 0x1p-19)); }

DEV uint32_t base2(uint8_t b) {
    switch (b) {
    case 'C': case 'c': return 1;
    case 'G': case 'g': return 2;
    case 'T': case 't': case 'U': case 'u': return 3;
    default: return 0;
    }
}

struct SmallModels {
    FList<256> len[4], sel;
    FList<2> rev, dup;
};


}  // namespace fqz5
