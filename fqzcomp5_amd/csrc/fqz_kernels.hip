// fqz_kernels.hip — fqzcomp_qual on gfx950 (htscodecs fqzcomp_qual.c).
//
// Data-parallel part: the statistics fqz_pick_parameters
// decides from — per-record quality sums / rounded averages / duplicate
// flags, and quality histograms binned by (remaining length & 127) for
// READ1/READ2 records and for the four average-quality classes.  Bins are
// privatised in LDS per workgroup (128 x 256 packed u16 pairs = 128 KiB)
// and flushed with global atomics.
//
// Serial part (a13/a16/a18): the adaptive frequency lists and the range
// coder are one dependent chain per block (every symbol updates the model of
// its context and the coder state).  One lane runs the block; the 65536
// quality-context models live in HBM (304 B each), the length / selector /
// duplicate models in LDS.
#include <hip/hip_runtime.h>
#include <cstdint>

#include "fqz_kernels.h"

namespace fqz5 {

#define DEV __device__ __forceinline__

// --------------------------------------------------------------------------
// statistics
// --------------------------------------------------------------------------
// fqz_qual_stats per-record loop (fqzcomp_qual.c:464-502): the sum, the
// average in tenths rounded as (tot*10.0)/len+.5 in double, the duplicate
// test against the previous record and the average histogram.
__global__ void k_fqz_records(FqzStatJob J) {
    const uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= J.nrec) return;
    const uint64_t off = J.off[r];
    const uint32_t len = J.len[r];
    const uint8_t *q = J.q + off;
    uint32_t sum = 0;
    for (uint32_t t = 0; t < len; t++) sum += q[t];
    const uint32_t avg = len ? uint32_t((double(sum) * 10.0) / double(len) + .5) : 0u;
    J.rec_avg[r] = avg;
    atomicAdd(&J.avg_hist[avg < 2559u ? avg : 2559u], 1u);
    if (r > 0 && off > 0 && J.len[r - 1] == len) {
        const uint8_t *p = q - len;
        uint32_t t = 0;
        while (t < len && p[t] == q[t]) t++;
        if (t == len) atomicAdd(J.dups, 1u);
    }
}

// Histogram of one chunk of records into LDS, packed pairs: lo half for the
// first class, hi half for the second.  mode 0: class = READ2 flag;
// mode 1/2: class = quality class (0/1 or 2/3) from amap[rec_avg].
extern __shared__ uint32_t fqz_lds[];

__global__ __launch_bounds__(256) void k_fqz_hist(FqzStatJob J, int mode) {
    uint32_t *h = fqz_lds;
    const uint2 ch = J.chunks[blockIdx.x];           // records [x, y)
    for (int i = threadIdx.x; i < 128 * 256; i += 256) h[i] = 0;
    __syncthreads();
    for (uint32_t r = ch.x; r < ch.y; r++) {
        const uint32_t len = J.len[r];
        const uint8_t *q = J.q + J.off[r];
        uint32_t inc;
        bool use = true;
        if (mode == 0) {
            inc = (J.flags[r] & 128u) ? 65536u : 1u;
        } else {
            const uint32_t a = J.rec_avg[r];
            const uint32_t cls = J.amap[a < 2559u ? a : 2559u];
            const uint32_t lo = mode == 1 ? 0u : 2u;
            use = cls == lo || cls == lo + 1;
            inc = cls == lo ? 1u : 65536u;
        }
        if (!use) continue;
        for (uint32_t t = threadIdx.x; t < len; t += 256)
            atomicAdd(&h[(((len - t) & 127u) << 8) | q[t]], inc);
    }
    __syncthreads();
    uint32_t *g0 = mode == 0 ? J.h1 : J.b4 + (mode == 1 ? 0 : 2) * 32768;
    uint32_t *g1 = mode == 0 ? J.h2 : J.b4 + (mode == 1 ? 1 : 3) * 32768;
    for (int i = threadIdx.x; i < 128 * 256; i += 256) {
        const uint32_t v = h[i];
        if (v & 0xffffu) atomicAdd(&g0[i], v & 0xffffu);
        if (v >> 16) atomicAdd(&g1[i], v >> 16);
    }
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

// --------------------------------------------------------------------------
// range coder (c_range_coder.h:20-164)
// --------------------------------------------------------------------------
struct RC {
    uint32_t lo, rng, code, ffrun, pend, carry;
    uint8_t *p;
    const uint8_t *in, *end;
    int err;
};

DEV void rc_shift(RC &c) {
    if (c.lo < 0xFF000000u || c.carry) {
        *c.p++ = uint8_t(c.pend + c.carry);
        for (; c.ffrun; c.ffrun--) *c.p++ = uint8_t(c.carry - 1);
        c.pend = c.lo >> 24;
        c.carry = 0;
    } else {
        c.ffrun++;
    }
    c.lo <<= 8;
}

DEV void rc_put(RC &c, uint32_t cum, uint32_t f, uint32_t tot) {
    const uint32_t before = c.lo;
    c.rng /= tot;
    c.lo += cum * c.rng;
    c.rng *= f;
    c.carry += c.lo < before;
    while (c.rng < (1u << 24)) {
        c.rng <<= 8;
        rc_shift(c);
    }
}

template <int CAP> DEV void fl_encode(FList<CAP> *m, RC &c, uint32_t sym) {
    uint32_t acc = 0;
    int k = 1;
    while (m->sy[k] != sym) acc += m->fr[k++];
    rc_put(c, acc, m->fr[k], m->total);
    fl_bump(m, k);
}

template <int CAP> DEV uint32_t fl_decode(FList<CAP> *m, RC &c) {
    uint32_t t = 0;
    if (m->total && c.rng >= m->total) {
        c.rng /= m->total;
        t = c.code / c.rng;
    }
    if (t > FL_MAX) return 0;
    uint32_t acc = 0;
    int k = 1;
    while ((acc += m->fr[k]) <= t) k++;
    if (k - 1 > CAP) return 0;
    acc -= m->fr[k];
    c.code -= acc * c.rng;
    c.rng *= m->fr[k];
    while (c.rng < (1u << 24)) {
        if (c.in >= c.end) { c.err = -1; break; }
        c.code = (c.code << 8) + *c.in++;
        c.rng <<= 8;
    }
    const uint32_t s = m->sy[k];
    fl_bump(m, k);
    return s;
}

__global__ void k_fqz_model_init(uint8_t *models, int live) {
    const uint32_t c = blockIdx.x * blockDim.x + threadIdx.x;
    if (c < uint32_t(FQZ_CTX)) fl_init(reinterpret_cast<FList<FQZ_QSYMS> *>(models) + c, live);
}

// --------------------------------------------------------------------------
// per-record context (fqz_update_ctx, fqzcomp_qual.c:361-418)
// --------------------------------------------------------------------------
struct Ctx {
    uint32_t qctx, left, delta, prevq, sel, seq;
};

DEV uint32_t next_ctx(const FqzDevParam &pm, Ctx &st, uint32_t q, uint32_t base) {
    st.qctx = (st.qctx << pm.qshift) + pm.qtab[q];
    uint32_t c = (st.qctx & pm.qmask) << pm.qloc;
    c += pm.ptab[st.left < 1023u ? st.left : 1023u];
    c += pm.dtab[st.delta < 255u ? st.delta : 255u];
    st.seq = ((st.seq << 2) | base) & ((1u << pm.bbits) - 1);
    c += st.seq << pm.bloc;
    c += st.sel << pm.sloc;
    st.delta += (st.prevq != q);
    st.prevq = q;
    st.left--;
    return c & uint32_t(FQZ_CTX - 1);
}

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

// --------------------------------------------------------------------------
// encoder (compress_block_fqz2f, fqzcomp_qual.c:1112-1208)
// --------------------------------------------------------------------------
__global__ __launch_bounds__(64) void k_fqz_encode(FqzEncJob J) {
    __shared__ SmallModels sm;
    if (threadIdx.x) return;
    const FqzDevGlobal &g = *J.g;
    for (int b = 0; b < 4; b++) fl_init(&sm.len[b], 256);
    fl_init(&sm.rev, 2);
    fl_init(&sm.dup, 2);
    if (g.max_sel > 0) fl_init(&sm.sel, int(g.max_sel) + 1);
    FList<FQZ_QSYMS> *qm = reinterpret_cast<FList<FQZ_QSYMS> *>(J.models);

    RC rc{};
    rc.rng = 0xFFFFFFFFu;
    rc.p = J.out;
    const FqzDevParam *pm = &g.p[0];
    Ctx st{};
    bool first_len = true;
    uint32_t rec = 0, prev_len = 0, ctx = 0;
    const uint8_t *sp = nullptr, *se = nullptr;
    const uint8_t *q = J.q;
    for (uint64_t i = 0; i < J.n; i++) {
        if (st.left == 0) {
            if (pm->sel || (g.gflags & 1u)) {
                st.sel = rec < J.nrec ? J.sel[rec] : 0u;
                fl_encode(&sm.sel, rc, st.sel);
            } else {
                st.sel = 0;
            }
            pm = &g.p[(g.gflags & 2u) ? g.stab[st.sel] : st.sel];
            const uint32_t len = J.len[rec];
            if (!pm->fixed || first_len) {
                for (int b = 0; b < 4; b++) fl_encode(&sm.len[b], rc, (len >> (8 * b)) & 0xffu);
                first_len = false;
            }
            if (g.gflags & 4u) fl_encode(&sm.rev, rc, (J.flags[rec] & 16u) ? 1u : 0u);
            st.left = len;
            st.delta = st.qctx = st.prevq = 0;
            if (J.seq && J.seq_off[rec] != ~0ull) {
                const uint8_t *s0 = J.seq + J.seq_off[rec];
                sp = s0 + pm->boff;
                se = s0 + len;
                st.seq = 0;
                for (uint32_t b = 0; b < pm->boff; b++) st.seq = (st.seq << 2) | base2(s0[b]);
            } else {
                sp = se = nullptr;
                st.seq = 0;
            }
            rec++;
            ctx = pm->ctx0;
            if (pm->dedup) {
                bool dup = i && len == prev_len;
                for (uint32_t t = 0; dup && t < len; t++) dup = q[i - prev_len + t] == q[i + t];
                if (dup) {
                    fl_encode(&sm.dup, rc, 1u);
                    i += len - 1;
                    st.left = 0;
                    continue;
                }
                fl_encode(&sm.dup, rc, 0u);
                prev_len = len;
            }
        }
        const uint32_t sym = pm->qmap[q[i]];
        const uint32_t base = sp && sp < se ? base2(*sp++) : 0u;
        fl_encode(&qm[ctx], rc, sym);
        ctx = next_ctx(*pm, st, sym, base);
    }
    for (int k = 0; k < 5; k++) rc_shift(rc);
    *J.out_len = uint32_t(rc.p - J.out);
}

// --------------------------------------------------------------------------
// decoder (uncompress_block_fqz2f, fqzcomp_qual.c:1480-1585)
// --------------------------------------------------------------------------
__global__ __launch_bounds__(64) void k_fqz_decode(FqzDecJob J) {
    __shared__ SmallModels sm;
    if (threadIdx.x) return;
    const FqzDevGlobal &g = *J.g;
    for (int b = 0; b < 4; b++) fl_init(&sm.len[b], 256);
    fl_init(&sm.rev, 2);
    fl_init(&sm.dup, 2);
    if (g.max_sel > 0) fl_init(&sm.sel, int(g.max_sel) + 1);
    FList<FQZ_QSYMS> *qm = reinterpret_cast<FList<FQZ_QSYMS> *>(J.models);

    RC rc{};
    rc.rng = 0xFFFFFFFFu;
    rc.in = J.in;
    rc.end = J.in + J.in_len;
    if (J.in_len < 5) {
        rc.in = rc.end;
    } else {
        for (int k = 0; k < 5; k++) rc.code = (rc.code << 8) | *rc.in++;
    }
    const FqzDevParam *pm = &g.p[0];
    Ctx st{};
    bool first_len = true;
    uint32_t rec = 0, prev_len = 0, ctx = 0;
    const uint8_t *sp = nullptr, *se = nullptr;
    uint8_t *out = J.out;
    int status = 0;
    for (uint64_t i = 0; i < J.n; i++) {
        if (st.left == 0) {
            st.sel = (pm->sel || (g.gflags & 1u)) ? fl_decode(&sm.sel, rc) : 0u;
            const uint32_t x = (g.gflags & 2u) ? g.stab[st.sel < 255u ? st.sel : 255u] : st.sel;
            if (x >= g.nparam) { status = -1; break; }
            pm = &g.p[x];
            uint32_t len = prev_len;
            if (!pm->fixed || first_len) {
                len = 0;
                for (int b = 0; b < 4; b++) len |= fl_decode(&sm.len[b], rc) << (8 * b);
                first_len = false;
                prev_len = len;
            }
            if (uint64_t(len) > J.n - i || len == 0) { status = -1; break; }
            if (rec < J.nlengths) J.lengths[rec] = len;
            if (g.gflags & 4u) {
                const uint32_t rv = fl_decode(&sm.rev, rc);
                if (rec < J.max_rec) { J.rev[rec] = uint8_t(rv); J.rlen[rec] = len; }
            }
            if (pm->dedup && fl_decode(&sm.dup, rc)) {
                if (len > i) { status = -1; break; }
                for (uint32_t t = 0; t < len; t++) out[i + t] = out[i - len + t];
                i += len - 1;
                st.left = 0;
                rec++;
                continue;
            }
            st.left = len;
            st.delta = st.prevq = st.qctx = 0;
            if (J.seq && rec < J.nseq && J.seq_off[rec] != ~0ull) {
                const uint8_t *s0 = J.seq + J.seq_off[rec];
                sp = s0 + pm->boff;
                se = s0 + len;
                st.seq = 0;
                for (uint32_t b = 0; b < pm->boff; b++) st.seq = (st.seq << 2) | base2(s0[b]);
            } else {
                sp = se = nullptr;
                st.seq = 0;
            }
            rec++;
            ctx = pm->ctx0;
        }
        const uint32_t sym = fl_decode(&qm[ctx], rc) & 0xffu;
        out[i] = pm->qmap[sym];
        const uint32_t base = sp && sp < se ? base2(*sp++) : 0u;
        ctx = next_ctx(*pm, st, sym, base);
    }
    // GFLAG_DO_REV: reverse the flagged records back (fqzcomp_qual.c:1597-1611)
    if (status == 0 && (g.gflags & 4u)) {
        uint64_t i = 0;
        for (uint32_t r = 0; i < J.n && r < rec && r < J.max_rec; i += J.rlen[r++]) {
            if (!J.rev[r]) continue;
            for (uint32_t a = 0, b = J.rlen[r] - 1; a < b; a++, b--) {
                const uint8_t t = out[i + a];
                out[i + a] = out[i + b];
                out[i + b] = t;
            }
        }
    }
    *J.status = status;
    *J.nrec_out = rec;
}

// --------------------------------------------------------------------------
hipError_t launch_fqz_records(const FqzStatJob &j, hipStream_t s) {
    if (!j.nrec) return hipSuccess;
    hipLaunchKernelGGL(k_fqz_records, dim3((j.nrec + 255) / 256), dim3(256), 0, s, j);
    return hipGetLastError();
}

hipError_t launch_fqz_hist(const FqzStatJob &j, int nchunks, int mode, hipStream_t s) {
    if (!nchunks) return hipSuccess;
    static bool attr = false;
    if (!attr) {
        (void)hipFuncSetAttribute(reinterpret_cast<const void *>(k_fqz_hist),
                                  hipFuncAttributeMaxDynamicSharedMemorySize, 128 * 1024);
        attr = true;
    }
    hipLaunchKernelGGL(k_fqz_hist, dim3(nchunks), dim3(256), 128 * 1024, s, j, mode);
    return hipGetLastError();
}

hipError_t launch_fqz_model_init(uint8_t *models, int live, hipStream_t s) {
    hipLaunchKernelGGL(k_fqz_model_init, dim3(FQZ_CTX / 256), dim3(256), 0, s, models, live);
    return hipGetLastError();
}

hipError_t launch_fqz_encode(const FqzEncJob &j, hipStream_t s) {
    hipLaunchKernelGGL(k_fqz_encode, dim3(1), dim3(64), 0, s, j);
    return hipGetLastError();
}

hipError_t launch_fqz_decode(const FqzDecJob &j, hipStream_t s) {
    hipLaunchKernelGGL(k_fqz_decode, dim3(1), dim3(64), 0, s, j);
    return hipGetLastError();
}

}  // namespace fqz5
