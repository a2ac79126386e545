// arith_kernels.hip — the entropy coders of htscodecs arith_dynamic.c
// (O0 :97-135, O1 :172-223, O0+RLE :441-514, O1+RLE :575-656 and their
// decoders) on gfx950: one wavefront per stream, the coder a single
// dependent chain.  The dispatcher (PACK / STRIPE / CAT framing) is host
// code over GPU transforms (arith_codec.cpp).
//
// Models are c_simple_model.h lists (STEP 16, MAX_FREQ 65519, one bubble
// step) stored compactly: a list of NSYM symbols of which `live` start with
// frequency 1 keeps only its live slots plus the two terminators.  Zero
// slots never move, never halve and never stop a scan short of the
// terminator, so every decision (including the decoder's out-of-range
// "symbol 0" exit) is the reference's.  Byte models hold the `m` symbols
// below the stream's maximum + 1, run models the MAX_RUN = 4 run symbols.
// They live in LDS when they fit, in HBM otherwise.
//
// Input bytes come through a 4 KB LDS ring refilled by the whole wave, output
// bytes go through a 4 KB LDS page flushed by the whole wave; the serial
// loop runs on all lanes with uniform values (readfirstlane), model stores
// from lane 0.
#include <hip/hip_runtime.h>
#include <cstdint>

#include "arith_kernels.h"
#include "fqz_model.hpp"

namespace fqz5 {
namespace {

constexpr uint32_t RING = 4096, HALF = 2048, PAGE = 4096;
constexpr uint32_t A_RING = 0, A_PAGE = RING + 16, A_MODELS = A_PAGE + PAGE;
constexpr uint32_t MAX_RUN = 4, RUN_MODELS = 258;

DEV uint32_t U(uint32_t v) { return __builtin_amdgcn_readfirstlane(v); }

// compact list: u32 total | u16 fr[C+3] | u8 sy[C+3]; slot 0 the sentinel,
// 1..C the symbols, C+1 a zero terminator, C+2 a maximal one
template <class P> struct CL {
    P b;
    uint32_t C;
    DEV uint32_t total() const { return U(*reinterpret_cast<const uint32_t *>(b)); }
    DEV uint32_t fr(uint32_t k) const { return U(reinterpret_cast<const uint16_t *>(b + 4)[k]); }
    DEV uint32_t sy(uint32_t k) const { return U(b[4 + 2 * (C + 3) + k]); }
    DEV void set_total(uint32_t v) const { *reinterpret_cast<uint32_t *>(b) = v; }
    DEV void set_fr(uint32_t k, uint32_t v) const { reinterpret_cast<uint16_t *>(b + 4)[k] = uint16_t(v); }
    DEV void set_sy(uint32_t k, uint32_t v) const { b[4 + 2 * (C + 3) + k] = uint8_t(v); }
};

__host__ __device__ constexpr uint32_t cl_bytes(uint32_t C) { return (4u + 3u * (C + 3u) + 3u) & ~3u; }

template <class P> DEV void cl_init(CL<P> m, uint32_t live) {
    const uint32_t l = threadIdx.x;
    for (uint32_t k = l; k < m.C + 3; k += 64) {
        uint32_t f = 0, s = 0;
        if (k == 0 || k == m.C + 2) f = FL_MAX;
        else if (k <= m.C) f = (k - 1) < live ? 1u : 0u, s = k - 1;
        m.set_fr(k, f);
        m.set_sy(k, s);
    }
    if (l == 0) m.set_total(live);
}

// bump, halve past MAX_FREQ, one bubble step (c_simple_model.h:125-137);
// lane 0 stores
template <class P> DEV void cl_bump(CL<P> m, uint32_t k) {
    if (threadIdx.x == 0) {
        uint32_t tot = m.total() + FL_STEP;
        m.set_fr(k, m.fr(k) + FL_STEP);
        if (tot > FL_MAX) {
            tot = 0;
            for (uint32_t i = 1; m.fr(i); i++) {
                const uint32_t f = m.fr(i) - (m.fr(i) >> 1);
                m.set_fr(i, f);
                tot += f;
            }
        }
        m.set_total(tot);
        const uint32_t fk = m.fr(k), fp = m.fr(k - 1);
        if (fk > fp) {
            const uint32_t sk = m.sy(k), sp = m.sy(k - 1);
            m.set_fr(k, fp);
            m.set_sy(k, sp);
            m.set_fr(k - 1, fk);
            m.set_sy(k - 1, sk);
        }
    }
    __builtin_amdgcn_wave_barrier();
}

DEV __amdgpu_buffer_rsrc_t rsrc(const void *p, uint32_t n) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void *>(p), 0, n, 0x00020000);
}

// the whole wave copies [pos, pos + HALF) of the input into the ring
DEV void ring_fill(uint8_t *lds, __amdgpu_buffer_rsrc_t r, uint32_t pos) {
    const uint32_t l = threadIdx.x;
    for (uint32_t o = l * 4; o < HALF; o += 256) {
        uint32_t w = 0;
#pragma unroll
        for (uint32_t b = 0; b < 4; b++)
            w |= uint32_t(__builtin_amdgcn_raw_buffer_load_b8(r, pos + o + b, 0, 0)) << (8 * b);
        *reinterpret_cast<uint32_t *>(lds + A_RING + ((pos + o) & (RING - 1))) = w;
    }
    __syncthreads();
}

struct Reader {
    __amdgpu_buffer_rsrc_t r;
    uint32_t rp, lp;                    // next byte, bytes staged
    DEV void start(uint8_t *lds, const uint8_t *p, uint32_t n) {
        r = rsrc(p, n);
        rp = 0;
        ring_fill(lds, r, 0);
        ring_fill(lds, r, HALF);
        lp = RING;
    }
    DEV uint32_t peek(uint8_t *lds) const { return U(lds[A_RING + (rp & (RING - 1))]); }
    DEV uint32_t get(uint8_t *lds) {
        const uint32_t v = peek(lds);
        rp++;
        if (lp - rp < HALF) {
            ring_fill(lds, r, lp);
            lp += HALF;
        }
        return v;
    }
};

struct Writer {
    uint8_t *out;
    uint32_t base, fill, cap;           // page covers [base, base + fill)
    DEV void put(uint8_t *lds, uint32_t v) {
        if (threadIdx.x == 0) lds[A_PAGE + fill] = uint8_t(v);
        fill++;
        if (fill == PAGE) flush(lds);
    }
    DEV void flush(uint8_t *lds) {
        __syncthreads();
        for (uint32_t o = threadIdx.x; o < fill; o += 64)
            if (base + o < cap) out[base + o] = lds[A_PAGE + o];
        base += fill;
        fill = 0;
        __syncthreads();
    }
};

// ---------------------------------------------------------------------------
// encoder (c_range_coder.h RC_Encode / RC_ShiftLowCheck / RC_FinishEncode)
// ---------------------------------------------------------------------------
struct Enc {
    uint32_t low, rng, ffnum, cache, carry;
    uint32_t written, cap;              // coder bytes written, room
    int err;
    Writer w;
    DEV void shift(uint8_t *lds) {
        if (low < 0xFF000000u || carry) {
            if (ffnum >= cap - written) {
                err = -1;
                return;
            }
            w.put(lds, cache + carry);
            written++;
            for (; ffnum; ffnum--) {
                w.put(lds, carry - 1);
                written++;
            }
            cache = low >> 24;
            carry = 0;
        } else {
            ffnum++;
        }
        low <<= 8;
    }
    DEV void put_sym(uint8_t *lds, uint32_t cum, uint32_t f, uint32_t tot) {
        const uint32_t before = low;
        rng /= tot;
        low += cum * rng;
        rng *= f;
        carry += low < before;
        while (rng < (1u << 24)) {
            rng <<= 8;
            shift(lds);
        }
    }
};

template <class P> DEV void cl_encode(CL<P> m, Enc &e, uint8_t *lds, uint32_t sym) {
    uint32_t acc = 0, k = 1;
    while (m.sy(k) != sym) acc += m.fr(k++);
    e.put_sym(lds, acc, m.fr(k), m.total());
    cl_bump(m, k);
}

template <bool G> __global__ __launch_bounds__(64) void k_arith_enc(const ArithJob *Js) {
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    const ArithJob J = load_job(Js + blockIdx.x);
    using P = uint8_t *;
    P mb = G ? J.models : lds + A_MODELS;
    const uint32_t nb = J.o1 ? 256u : 1u, bb = cl_bytes(J.m), rb = cl_bytes(MAX_RUN);
    for (uint32_t i = 0; i < nb; i++) cl_init(CL<P>{mb + i * bb, J.m}, J.m);
    P rbase = mb + nb * bb;
    if (J.rle)
        for (uint32_t i = 0; i < RUN_MODELS; i++) cl_init(CL<P>{rbase + i * rb, MAX_RUN}, MAX_RUN);
    __syncthreads();
    Reader in;
    in.start(lds, J.in, J.n);
    Enc e{};
    e.rng = 0xFFFFFFFFu;
    e.cap = J.cap;
    e.w = Writer{J.out, 0, 0, J.cap};
    uint32_t last = 0;
    if (!J.rle) {
        for (uint32_t i = 0; i < J.n && !e.err; i++) {
            const uint32_t c = in.get(lds);
            cl_encode(CL<P>{mb + (J.o1 ? last : 0u) * bb, J.m}, e, lds, c);
            last = c;
        }
    } else {
        uint32_t i = 0;
        while (i < J.n && !e.err) {
            const uint32_t c = in.get(lds);
            cl_encode(CL<P>{mb + (J.o1 ? last : 0u) * bb, J.m}, e, lds, c);
            uint32_t run = 0;
            last = c;
            i++;
            while (i < J.n && in.peek(lds) == last) {
                in.get(lds);
                run++;
                i++;
            }
            uint32_t rctx = last;
            do {
                const uint32_t cc = run < MAX_RUN ? run : MAX_RUN - 1;
                cl_encode(CL<P>{rbase + rctx * rb, MAX_RUN}, e, lds, cc);
                run -= cc;
                if (rctx == last) rctx = 256;
                else rctx += rctx < RUN_MODELS - 1;
                if (cc == MAX_RUN - 1 && run == 0)
                    cl_encode(CL<P>{rbase + rctx * rb, MAX_RUN}, e, lds, 0u);
            } while (run && !e.err);
        }
    }
    for (int k = 0; k < 5 && !e.err; k++) e.shift(lds);
    e.w.flush(lds);
    if (threadIdx.x == 0) {
        *J.out_len = e.written;
        *J.status = e.err;
    }
}

// ---------------------------------------------------------------------------
// decoder (RC_GetFreq / RC_Decode with the end-of-input error)
// ---------------------------------------------------------------------------
struct Dec {
    uint32_t rng, code, left;           // left: coder bytes still unread
    int err;
    Reader in;
};

template <class P> DEV uint32_t cl_decode(CL<P> m, Dec &d, uint8_t *lds) {
    const uint32_t tot = m.total();
    uint32_t t = 0;
    if (tot && d.rng >= tot) {
        d.rng /= tot;
        t = d.code / d.rng;
    }
    if (t > FL_MAX) return 0;
    uint32_t acc = 0, k = 1;
    while ((acc += m.fr(k)) <= t) k++;
    if (k - 1 > m.C) return 0;
    const uint32_t f = m.fr(k);
    acc -= f;
    d.code -= acc * d.rng;
    d.rng *= f;
    while (d.rng < (1u << 24)) {
        if (!d.left) {
            d.err = -1;
            break;
        }
        d.code = (d.code << 8) + d.in.get(lds);
        d.left--;
        d.rng <<= 8;
    }
    const uint32_t s = m.sy(k);
    cl_bump(m, k);
    return s;
}

template <bool G> __global__ __launch_bounds__(64) void k_arith_dec(const ArithJob *Js) {
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    const ArithJob J = load_job(Js + blockIdx.x);
    using P = uint8_t *;
    P mb = G ? J.models : lds + A_MODELS;
    const uint32_t nb = J.o1 ? 256u : 1u, bb = cl_bytes(J.m), rb = cl_bytes(MAX_RUN);
    for (uint32_t i = 0; i < nb; i++) cl_init(CL<P>{mb + i * bb, J.m}, J.m);
    P rbase = mb + nb * bb;
    if (J.rle)
        for (uint32_t i = 0; i < RUN_MODELS; i++) cl_init(CL<P>{rbase + i * rb, MAX_RUN}, MAX_RUN);
    __syncthreads();
    Dec d{};
    d.rng = 0xFFFFFFFFu;
    d.in.start(lds, J.in, J.in_len);
    d.left = J.in_len;
    if (J.in_len >= 5) {
        for (int k = 0; k < 5; k++) d.code = (d.code << 8) | d.in.get(lds);
        d.left -= 5;
    } else {
        d.left = 0;
    }
    Writer w{J.out, 0, 0, J.n};
    uint32_t last = 0;
    const uint32_t n = J.n;
    for (uint32_t i = 0; i < n; i++) {
        const uint32_t c = cl_decode(CL<P>{mb + (J.o1 ? last : 0u) * bb, J.m}, d, lds) & 0xffu;
        w.put(lds, c);
        last = c;
        if (J.rle) {
            uint32_t run = 0, r, rctx = last;
            do {
                r = cl_decode(CL<P>{rbase + rctx * rb, MAX_RUN}, d, lds);
                if (rctx == last) rctx = 256;
                else rctx += rctx < RUN_MODELS - 1;
                run += r;
            } while (r == MAX_RUN - 1 && run < n);
            while (run-- && i + 1 < n) {
                w.put(lds, last);
                i++;
            }
        }
    }
    w.flush(lds);
    if (threadIdx.x == 0) *J.status = d.err;
}

}  // namespace

uint32_t arith_model_bytes(uint32_t m, bool o1, bool rle) {
    return (o1 ? 256u : 1u) * cl_bytes(m) + (rle ? RUN_MODELS * cl_bytes(MAX_RUN) : 0u);
}

bool arith_models_in_lds(uint32_t m, bool o1, bool rle) {
    return A_MODELS + arith_model_bytes(m, o1, rle) <= 163840u;
}

hipError_t launch_arith(const ArithJob *d_jobs, int njobs, bool decode, bool global_models,
                        uint32_t lds_bytes, hipStream_t s) {
    if (!njobs) return hipSuccess;
    const uint32_t lds = A_MODELS + (global_models ? 0u : lds_bytes);
    const void *f = decode ? (global_models ? reinterpret_cast<const void *>(k_arith_dec<true>)
                                            : reinterpret_cast<const void *>(k_arith_dec<false>))
                           : (global_models ? reinterpret_cast<const void *>(k_arith_enc<true>)
                                            : reinterpret_cast<const void *>(k_arith_enc<false>));
    hipError_t e = hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, int(lds));
    if (e != hipSuccess) return e;
    if (decode) {
        if (global_models)
            hipLaunchKernelGGL(k_arith_dec<true>, dim3(njobs), dim3(64), lds, s, d_jobs);
        else
            hipLaunchKernelGGL(k_arith_dec<false>, dim3(njobs), dim3(64), lds, s, d_jobs);
    } else {
        if (global_models)
            hipLaunchKernelGGL(k_arith_enc<true>, dim3(njobs), dim3(64), lds, s, d_jobs);
        else
            hipLaunchKernelGGL(k_arith_enc<false>, dim3(njobs), dim3(64), lds, s, d_jobs);
    }
    return hipGetLastError();
}

}  // namespace fqz5
