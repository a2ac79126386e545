// fqz_kernels.hip — fqzcomp_qual on gfx950 (htscodecs fqzcomp_qual.c).
//
// Data-parallel part: the statistics fqz_pick_parameters
// decides from — per-record quality sums / rounded averages / duplicate
// flags, and quality histograms binned by (remaining length & 127) for
// READ1/READ2 records and for the four average-quality classes.  Bins are
// privatised in LDS per workgroup (128 x 256 packed u16 pairs = 128 KiB)
// and flushed with global atomics.
//
// Encoder (a13/a16): the parallel path (events sorted by model, per-model
// frequency pass, range-only serial chain, big-number byte assembly) and
// the serial literal encoder for multi-parameter blocks.  The decoder
// (a18) is fqz_decode.hip.
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdint>

#include "fqz_kernels.h"
#include "fqz_model.hpp"

namespace fqz5 {


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
// parallel encoder
// --------------------------------------------------------------------------
// Records of a block are independent except through the models and the
// coder: the duplicate test compares a record with its predecessor only,
// and the context of every quality symbol depends only on its own record
// (the context state resets at each record, fqzcomp_qual.c:1154-1173).

// Phase 0: per-record duplicate flag and event count.
__global__ void k_fqz_ev_count(FqzEvJob J) {
    const uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= J.nrec) return;
    const FqzDevGlobal &g = *J.g;
    const FqzDevParam &pm = g.p[0];
    const uint32_t len = J.len[r];
    const uint64_t off = J.off[r];
    bool dup = false;
    if (pm.dedup && off > 0 && J.len[r - 1] == len) {
        const uint8_t *a = J.q + off - len, *b = J.q + off;
        uint32_t t = 0;
        while (t < len && a[t] == b[t]) t++;
        dup = t == len;
    }
    J.dup[r] = dup;
    uint32_t n = 0;
    if (pm.sel || (g.gflags & 1u)) n++;
    if (!pm.fixed || r == 0) n += 4;
    if (g.gflags & 4u) n++;
    if (pm.dedup) n++;
    if (!dup) n += len;
    J.nev_rec[r] = n;
}

// Phase 1: the events of each record in stream order (compress_block_fqz2f
// record header, fqzcomp_qual.c:1119-1192, then one event per quality).
// A wave takes 64 records, whose events are one contiguous range of the
// list and whose quality bytes one contiguous range of q.  Per window of
// EVW events: the wave stages the window's quality bytes into LDS with
// coalesced loads, each lane generates its own record's events of the
// window in order (the context chain is serial within a record) into LDS,
// packed as model << 8 | symbol, and the wave writes the window out with
// consecutive lanes on consecutive events.  The parameter tables are read
// from an LDS copy.  (Up to round 6 one thread per record read its bytes and
// wrote its events itself: every load and store touched 64 lines, ~300 B of
// HBM traffic per event at -5 Illumina, profiles/r06_pmc_l5i.json.)
constexpr uint32_t EVW = 4096;          // events per window
constexpr uint32_t EVQ = 8192;          // quality bytes staged per window
__global__ __launch_bounds__(64) void k_fqz_ev_fill(FqzEvJob J) {
    __shared__ uint32_t win[EVW];
    __shared__ uint32_t qst[EVQ / 4];
    __shared__ FqzDevParam pm;
    const uint32_t lane = threadIdx.x;
    const FqzDevGlobal &g = *J.g;
    {
        const uint32_t *src = reinterpret_cast<const uint32_t *>(&g.p[0]);
        uint32_t *dst = reinterpret_cast<uint32_t *>(&pm);
        static_assert(sizeof(FqzDevParam) % 4 == 0, "parameter copy by words");
        for (uint32_t i = lane; i < sizeof(FqzDevParam) / 4; i += 64u) dst[i] = src[i];
    }
    __syncthreads();
    const uint32_t r0 = blockIdx.x * 64u;
    const uint32_t r = r0 + lane;
    const bool act = r < J.nrec;
    const uint32_t rend = min(r0 + 64u, J.nrec);
    const uint32_t E0 = J.ev_off[r0];
    const uint32_t E1 = rend < J.nrec ? J.ev_off[rend] : J.nev;
    const uint64_t qtot = J.off[J.nrec - 1] + J.len[J.nrec - 1];
    uint32_t e = act ? J.ev_off[r] : E1;
    const uint32_t e_end = act ? (r + 1 < J.nrec ? J.ev_off[r + 1] : J.nev) : E1;
    const uint32_t len = act ? J.len[r] : 0u;
    const bool dup = act && J.dup[r];
    const bool has_sel = pm.sel || (g.gflags & 1u);
    const bool has_len = !pm.fixed || r == 0;
    const bool has_rev = (g.gflags & 4u) != 0u;
    const uint32_t nh = (has_sel ? 1u : 0u) + (has_len ? 4u : 0u) + (has_rev ? 1u : 0u) +
                        (pm.dedup ? 1u : 0u);
    Ctx st{};
    if (act && has_sel) st.sel = J.sel[r];
    const uint32_t rev = act && has_rev && (J.flags[r] & 16u) ? 1u : 0u;
    st.left = len;
    const uint8_t *sp = nullptr, *se = nullptr;
    if (act && !dup && J.seq && J.seq_off[r] != ~0ull) {
        const uint8_t *s0 = J.seq + J.seq_off[r];
        sp = s0 + pm.boff;
        se = s0 + len;
        for (uint32_t b = 0; b < pm.boff; b++) st.seq = (st.seq << 2) | base2(s0[b]);
    }
    const uint64_t qoff = act ? J.off[r] : 0ull;
    uint32_t ctx = pm.ctx0, h = 0, t = 0;
    // header event i of the record: selector, four length bytes, reverse
    // flag, duplicate flag (each only where the parameters code it)
    auto header = [&](uint32_t i) -> uint32_t {
        if (has_sel) { if (i == 0) return FQZ_M_SEL << 8 | st.sel; i--; }
        if (has_len) { if (i < 4) return (FQZ_M_LEN + i) << 8 | ((len >> (8 * i)) & 0xffu); i -= 4; }
        if (has_rev) { if (i == 0) return FQZ_M_REV << 8 | rev; i--; }
        return FQZ_M_DUP << 8 | (dup ? 1u : 0u);
    };
    const uint8_t *qsb = reinterpret_cast<const uint8_t *>(qst);
    for (uint32_t w0 = E0; w0 < E1; w0 += EVW) {
        const uint32_t wend = min(w0 + EVW, E1);
        const uint32_t stop = min(wend, e_end);
        // the window's quality bytes start at the first lane (records are
        // in lane order) that codes a quality symbol in it; a byte past the
        // staged range (duplicate records in between) is read from q
        const bool inq = e < stop && (h >= nh || nh - h < stop - e);
        const uint64_t qm = __ballot(inq);
        uint64_t qb = 0;
        if (qm) {
            const int fl = __builtin_ctzll(qm);
            const uint64_t qpos = qoff + t;
            qb = (uint64_t(__shfl(uint32_t(qpos >> 32), fl)) << 32 | __shfl(uint32_t(qpos), fl)) & ~3ull;
            for (uint32_t i = lane; i < EVQ / 4; i += 64u) {
                const uint64_t a = qb + 4ull * i;
                uint32_t v = 0;
                if (a + 4 <= qtot) {
                    v = *reinterpret_cast<const uint32_t *>(J.q + a);
                } else {
                    for (uint32_t k = 0; k < 4; k++)
                        if (a + k < qtot) v |= uint32_t(J.q[a + k]) << (8 * k);
                }
                qst[i] = v;
            }
        }
        __syncthreads();
        for (; e < stop; e++) {
            uint32_t v;
            if (h < nh) {
                v = header(h++);
            } else {
                const uint64_t p = qoff + t - qb;
                const uint32_t raw = p < EVQ ? qsb[p] : J.q[qoff + t];
                t++;
                const uint32_t sym = pm.qmap[raw];
                const uint32_t base = sp && sp < se ? base2(*sp++) : 0u;
                v = ctx << 8 | sym;
                ctx = next_ctx(pm, st, sym, base);
            }
            win[e - w0] = v;
        }
        __syncthreads();
        for (uint32_t i = lane; i < wend - w0; i += 64u) {
            const uint32_t v = win[i];
            J.key[w0 + i] = v >> 8;
            J.val[w0 + i] = (uint64_t(w0 + i) << 8) | (v & 0xffu);
        }
        __syncthreads();
    }
}

// Phase 2 (after the sort): each model's range in the sorted events.
__global__ void k_fqz_segments(FqzEvJob J) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= J.nev) return;
    const uint32_t k = J.skey[i];
    if (i == 0 || J.skey[i - 1] != k) J.seg_lo[k] = i;
    if (i == J.nev - 1 || J.skey[i + 1] != k) J.seg_hi[k] = i + 1;
}

// Phase 3: every model over its own events, in stream order, writing the
// codes in sorted order.  Quality models live in LDS (one per lane); the
// header models in global scratch.  Events go in batches of 32: the loads
// of a batch are issued together and its stores after it, so a lane waits
// for memory once per batch.
template <int CAP> DEV void model_run(FList<CAP> *m, const FqzEvJob &J, uint32_t lo, uint32_t hi) {
    constexpr uint32_t B = 32;
    // Slot 1 (the head) and the total are kept in registers while the
    // symbols hit the head; LDS is synchronised before any other update.
    // The head never bubbles (slot 0 always wins the comparison).
    // The next batch's symbols are loaded (bounds-checked buffer loads over
    // all events: a lane may read past its model, never past the array)
    // while this batch is coded, so a lane waits for memory only when a
    // batch codes faster than a load returns.
    uint32_t s1 = m->sy[1], f1 = m->fr[1], tot = m->total;
    // (sval has 2 events of room past nev, so a pair's load never straddles
    // the end of the range)
    const auto rsv = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint64_t *>(J.sval), 0,
                                                       J.nev * 8u + 16u, 0x00020000);
    // two events per load and per store: 32 of each per batch kept a
    // lane's memory operations at the 63 the counter allows, so every batch
    // waited out a full HBM round trip (the length models' ~297K events per
    // block ran at ~640 cycles each)
    const auto rcd = __builtin_amdgcn_make_buffer_rsrc(J.code, 0, J.nev * 8u, 0x00020000);
    typedef uint32_t u32x4_t __attribute__((ext_vector_type(4)));
    typedef uint32_t u32x2_t __attribute__((ext_vector_type(2)));
    u32x4_t pn[B / 2];
    auto fetch = [&](uint32_t k) {
#pragma unroll
        for (uint32_t v = 0; v < B / 2; v++)
            pn[v] = __builtin_amdgcn_raw_buffer_load_b128(rsv, (k + 2 * v) * 8u, 0, 0);
    };
    fetch(lo);
    for (uint32_t k0 = lo; k0 < hi; k0 += B) {
        const uint32_t nb = min(B, hi - k0);
        uint32_t sv[B];
#pragma unroll
        for (uint32_t u = 0; u < B; u++) sv[u] = (u & 1 ? pn[u / 2][2] : pn[u / 2][0]) & 0xffu;
        if (k0 + B < hi) fetch(k0 + B);
        uint64_t cd[B];
#pragma unroll
        for (uint32_t u = 0; u < B; u++) {
            cd[u] = 0;
            if (u < nb) {
                const uint32_t sym = sv[u];
                if (sym == s1 && tot + FL_STEP <= FL_MAX) {
                    cd[u] = (uint64_t(f1) << 16) | (uint64_t(tot) << 32);
                    f1 += FL_STEP;
                    tot += FL_STEP;
                } else {
                    m->fr[1] = uint16_t(f1);
                    m->total = tot;
                    uint32_t acc = 0;
                    int s = 1;
                    while (m->sy[s] != sym) acc += m->fr[s++];
                    cd[u] = uint64_t(acc) | (uint64_t(m->fr[s]) << 16) | (uint64_t(tot) << 32);
                    fl_bump(m, s);
                    s1 = m->sy[1];
                    f1 = m->fr[1];
                    tot = m->total;
                }
            }
        }
#pragma unroll
        for (uint32_t v = 0; v < B / 2; v++) {
            const uint32_t u = 2 * v;
            if (u + 1 < nb) {
                u32x4_t w = {uint32_t(cd[u]), uint32_t(cd[u] >> 32), uint32_t(cd[u + 1]),
                             uint32_t(cd[u + 1] >> 32)};
                __builtin_amdgcn_raw_buffer_store_b128(w, rcd, (k0 + u) * 8u, 0, 0);
            } else if (u < nb) {   // (the next model's events are another lane's)
                u32x2_t w = {uint32_t(cd[u]), uint32_t(cd[u] >> 32)};
                __builtin_amdgcn_raw_buffer_store_b64(w, rcd, (k0 + u) * 8u, 0, 0);
            }
        }
    }
    m->fr[1] = uint16_t(f1);
    m->total = tot;
}

// one launch for a batch of blocks: workgroup b handles models
// [256 (b % nblk), +256) of block b / nblk
// Hot quality models (at least hot_min events, at most FQZ_HOT_LIVE live
// symbols) go to k_fqz_model_hot instead; hot_min = 0 disables that path.
constexpr uint32_t FQZ_HOT_LIVE = 126;           // slots 0..live+1 in two lane registers
DEV bool fqz_is_hot(uint32_t m, uint32_t cnt, uint32_t live, uint32_t hot_min) {
    return hot_min && m < FQZ_M_SEL && live <= FQZ_HOT_LIVE && cnt >= hot_min;
}

#ifdef FQZ5_MP_PROBE
// the slowest lane of the model pass: {cycles << 24 | model, its events}
__device__ unsigned long long g_mpprobe[2];
extern "C" int fqz5_mp_probe_read(uint64_t *out) {
    hipError_t e = hipMemcpyFromSymbol(out, HIP_SYMBOL(g_mpprobe), sizeof(g_mpprobe));
    const unsigned long long z[2] = {0, 0};
    if (e == hipSuccess) e = hipMemcpyToSymbol(HIP_SYMBOL(g_mpprobe), z, sizeof(z));
    return int(e);
}
#endif

__global__ __launch_bounds__(256) void k_fqz_model_pass(const FqzEvJob *Js, uint32_t nblk,
                                                        uint32_t hot_min) {
    FList<FQZ_QSYMS> *lm = reinterpret_cast<FList<FQZ_QSYMS> *>(fqz_lds);   // 256 models
    const FqzEvJob J = load_job(Js + blockIdx.x / nblk);
    const uint32_t m = (blockIdx.x % nblk) * blockDim.x + threadIdx.x;
    static_assert(5 * sizeof(FList<256>) + 2 * sizeof(FList<2>) <= 256 * sizeof(FList<FQZ_QSYMS>),
                  "header models in the pass's LDS");
    static_assert(FQZ_M_SEL % 256 == 0 && FQZ_NMODELS - FQZ_M_SEL <= 256,
                  "the header models share one workgroup");
    if (m >= FQZ_NMODELS) return;
    const uint32_t lo = J.seg_lo[m], hi = J.seg_hi[m];
    if (lo >= hi) return;
    const FqzDevGlobal &g = *J.g;
    if (fqz_is_hot(m, hi - lo, g.max_sym + 1, hot_min)) return;
#ifdef FQZ5_MP_PROBE
    const uint64_t c0 = __builtin_amdgcn_s_memtime();
#endif
    if (m < FQZ_M_SEL) {
        FList<FQZ_QSYMS> *ml = &lm[threadIdx.x];
        fl_init(ml, int(g.max_sym) + 1);
        model_run(ml, J, lo, hi);
    } else if (m < FQZ_M_REV) {
        // the header models (selector, 4 length bytes; then REV and DUP) in
        // the LDS of the last workgroup, whose other lanes hold no model: in
        // global scratch their searches and halvings (a length model codes
        // one event per record) made this lane the pass's longest, 145 ms
        // on a -5 Illumina block
        FList<256> *mg = reinterpret_cast<FList<256> *>(fqz_lds) + (m - FQZ_M_SEL);
        fl_init(mg, m == FQZ_M_SEL ? int(g.max_sel) + 1 : 256);
        model_run(mg, J, lo, hi);
    } else {
        FList<2> *mg = reinterpret_cast<FList<2> *>(reinterpret_cast<uint8_t *>(fqz_lds) +
                                                    5 * sizeof(FList<256>)) +
                       (m - FQZ_M_REV);
        fl_init(mg, 2);
        model_run(mg, J, lo, hi);
    }
#ifdef FQZ5_MP_PROBE
    const uint64_t dc = __builtin_amdgcn_s_memtime() - c0;
    const unsigned long long key = ((unsigned long long)(dc >> 4) << 24) | m;
    const unsigned long long old = atomicMax(&g_mpprobe[0], key);
    if (key > old) atomicExch(&g_mpprobe[1], (unsigned long long)(hi - lo));
#endif
}

// The hot models of each block: list[0] = count, list[1..] = model ids.
__global__ void k_fqz_hot_list(const FqzEvJob *Js, uint32_t *hot, uint32_t stride,
                               uint32_t hot_min) {
    const FqzEvJob &J = Js[blockIdx.y];
    const uint32_t m = blockIdx.x * blockDim.x + threadIdx.x;
    if (m >= FQZ_M_SEL) return;
    const uint32_t lo = J.seg_lo[m], hi = J.seg_hi[m];
    if (hi <= lo || !fqz_is_hot(m, hi - lo, J.g->max_sym + 1, hot_min)) return;
    uint32_t *list = hot + size_t(blockIdx.y) * stride;
    const uint32_t k = atomicAdd(list, 1u);
    if (k + 1 < stride) list[1 + k] = m;
}

// Phase 3, hot models: one wave per model with the list in lanes (lane dw =
// l + 64 r of register r = slot dw: fr, cum = the sum of fr over slots
// 1..dw-1, sy; NE = 2 for alphabets past 62 symbols, as HiFi's Q0-Q93) and
// the model's events in chunks of 64, one per lane.  Runs of events that hit
// the head symbol are coded in parallel in closed form (event n of a run:
// cum 0, freq f1 + 16n, total tot + 16n, while no halving is due), every
// other event takes the list update (fl_bump: +16, halve past FL_MAX, one
// bubble step) with ballots and readlanes.  Codes are identical to
// model_run's.
template <int NE>
DEV void hot_models(const FqzEvJob &J, const uint32_t *list, uint32_t nh, uint32_t L) {
    const uint32_t l = threadIdx.x;
    const auto rsv = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint64_t *>(J.sval), 0,
                                                       J.nev * 8u, 0x00020000);
    auto rlane = [&](const uint32_t (&x)[NE], uint32_t dw) -> uint32_t {
        if (NE == 1) return __builtin_amdgcn_readlane(x[0], dw);
        const uint32_t a = __builtin_amdgcn_readlane(x[0], dw & 63u);
        const uint32_t b = __builtin_amdgcn_readlane(x[NE - 1], dw & 63u);
        return dw < 64 ? a : b;
    };
    uint64_t slots[NE];   // lanes of slots 1..L
#pragma unroll
    for (int r = 0; r < NE; r++) {
        const uint32_t b0 = 64u * r;
        const uint32_t lo = b0 < 1u ? 1u : b0, hi = L + 1u < b0 + 64u ? L + 1u : b0 + 64u;   // [lo, hi)
        slots[r] = hi > lo ? (((hi - lo) == 64 ? ~0ull : ((1ull << (hi - lo)) - 1)) << (lo - b0)) : 0ull;
    }
    for (uint32_t h = blockIdx.x; h < nh; h += gridDim.x) {
        const uint32_t m = __builtin_amdgcn_readfirstlane(list[1 + h]);
        const uint32_t lo = __builtin_amdgcn_readfirstlane(J.seg_lo[m]);
        const uint32_t hi = __builtin_amdgcn_readfirstlane(J.seg_hi[m]);
        // fl_init(live = L)
        uint32_t fr[NE], cum[NE], sy[NE];
#pragma unroll
        for (int r = 0; r < NE; r++) {
            const uint32_t dw = l + 64u * r;
            fr[r] = dw == 0 ? FL_MAX : (dw <= L ? 1u : 0u);
            cum[r] = dw == 0 ? 0u : (dw <= L + 1 ? dw - 1 : L);
            sy[r] = dw ? dw - 1 : 0u;
        }
        uint32_t tot = L;
        uint32_t sn = __builtin_amdgcn_raw_buffer_load_b32(rsv, (lo + l) * 8u, 0, 0);
        for (uint32_t k0 = lo; k0 < hi; k0 += 64) {
            const uint32_t sym = sn & 0xffu;
            if (k0 + 64 < hi) sn = __builtin_amdgcn_raw_buffer_load_b32(rsv, (k0 + 64 + l) * 8u, 0, 0);
            const uint32_t nv = min(64u, hi - k0);
            uint64_t P = nv == 64 ? ~0ull : ((1ull << nv) - 1);
            uint32_t s1 = __builtin_amdgcn_readlane(sy[0], 1), f1 = __builtin_amdgcn_readlane(fr[0], 1);
            uint64_t *code = J.code + k0;
            while (P) {
                // ---- a run of head hits, coded in parallel ----------------
                const uint32_t start = uint32_t(__builtin_ctzll(P));
                const uint64_t miss = P & ~uint64_t(__ballot(sym == s1));
                uint32_t run = (miss ? uint32_t(__builtin_ctzll(miss)) : nv) - start;
                const uint32_t cap = tot < FL_MAX ? (FL_MAX - tot) / FL_STEP : 0u;
                run = min(run, cap);
                if (run) {
                    if (l >= start && l < start + run) {
                        const uint32_t n = l - start;
                        code[l] = (uint64_t(f1 + FL_STEP * n) << 16) |
                                  (uint64_t(tot + FL_STEP * n) << 32);
                    }
                    fr[0] += l == 1 ? FL_STEP * run : 0u;
#pragma unroll
                    for (int r = 0; r < NE; r++) cum[r] += l + 64u * r >= 2 ? FL_STEP * run : 0u;
                    f1 += FL_STEP * run;
                    tot += FL_STEP * run;
                    P &= ~(((run == 64) ? ~0ull : ((1ull << run) - 1)) << start);
                    if (!P) break;
                }
                // ---- one event through fl_bump ----------------------------
                const uint32_t j0 = uint32_t(__builtin_ctzll(P));
                const uint32_t sj = __builtin_amdgcn_readlane(sym, j0);
                uint32_t sl = L + 1;   // always found
#pragma unroll
                for (int r = NE - 1; r >= 0; r--) {
                    const uint64_t sm = uint64_t(__ballot(sy[r] == sj)) & slots[r];
                    if (sm) sl = 64u * r + uint32_t(__builtin_ctzll(sm));
                }
                const uint32_t fs = rlane(fr, sl);
                const uint32_t cs = rlane(cum, sl);
                if (l == j0) code[l] = uint64_t(cs) | (uint64_t(fs) << 16) | (uint64_t(tot) << 32);
#pragma unroll
                for (int r = 0; r < NE; r++) {
                    const uint32_t dw = l + 64u * r;
                    fr[r] += dw == sl ? FL_STEP : 0u;
                    cum[r] += dw > sl ? FL_STEP : 0u;
                }
                tot += FL_STEP;
                if (tot > FL_MAX) {                 // halve slots 1..L, rebuild cum
                    uint32_t carry = 0;
#pragma unroll
                    for (int r = 0; r < NE; r++) {
                        const uint32_t dw = l + 64u * r;
                        const bool live = dw >= 1 && dw <= L;
                        if (live) fr[r] -= fr[r] >> 1;
                        const uint32_t x = live ? fr[r] : 0u;
                        uint32_t inc = x;
#pragma unroll
                        for (int d = 1; d < 64; d <<= 1) {
                            const uint32_t o = __shfl_up(inc, d, 64);
                            if (int(l) >= d) inc += o;
                        }
                        if (dw >= 1) cum[r] = carry + inc - x;
                        carry += __builtin_amdgcn_readlane(inc, 63);
                    }
                    tot = carry;
                }
                if (sl >= 2) {                      // one bubble step
                    const uint32_t fa = rlane(fr, sl - 1);
                    const uint32_t fb = rlane(fr, sl);
                    if (fb > fa) {
                        const uint32_t sa = rlane(sy, sl - 1);
                        const uint32_t sb = rlane(sy, sl);
                        const uint32_t ca = rlane(cum, sl - 1);
#pragma unroll
                        for (int r = 0; r < NE; r++) {
                            const uint32_t dw = l + 64u * r;
                            if (dw == sl - 1) { fr[r] = fb; sy[r] = sb; }
                            if (dw == sl) { fr[r] = fa; sy[r] = sa; cum[r] = ca + fb; }
                        }
                    }
                }
                s1 = __builtin_amdgcn_readlane(sy[0], 1);
                f1 = __builtin_amdgcn_readlane(fr[0], 1);
                P &= ~(1ull << j0);
            }
        }
    }
}

__global__ __launch_bounds__(64) void k_fqz_model_hot(const FqzEvJob *Js, const uint32_t *hot,
                                                      uint32_t stride) {
    const FqzEvJob J = load_job(Js + blockIdx.y);
    const uint32_t *list = hot + size_t(blockIdx.y) * stride;
    const uint32_t nh = min(__builtin_amdgcn_readfirstlane(list[0]), stride - 1);
    const uint32_t L = __builtin_amdgcn_readfirstlane(J.g->max_sym) + 1;   // live symbols
    if (L + 2 <= 64) hot_models<1>(J, list, nh, L);
    else hot_models<2>(J, list, nh, L);
}

// Entropy of a block's events under the adaptive models: sum of
// log2(total / freq) over the codes the model pass wrote, one partial sum
// per workgroup (the host adds them).  The coder's byte count P satisfies
// 8 P >= this - 8, so it bounds the output size from
// below before the range chain runs.
// The upper bound: floor(range / total) >= range/total
// - 1 and range >= 2^24 before every event, so an event narrows the range by
// at most (total / freq) / (1 - total / 2^24): 8 P <= sum log2(total / freq)
// + sum -log2(1 - total 2^-24).  partial[gridDim.x + b] gets the second sum.
DEV double rc_slack(double t) { return -log1p(-t * 0x1p-24) * 1.4426950408889634; }

DEV void entropy_reduce(double acc, double slack, double *partial) {
    __shared__ double red[256], rs[256];
    red[threadIdx.x] = acc;
    rs[threadIdx.x] = slack;
    __syncthreads();
    for (uint32_t o = 128; o; o >>= 1) {
        if (threadIdx.x < o) {
            red[threadIdx.x] += red[threadIdx.x + o];
            rs[threadIdx.x] += rs[threadIdx.x + o];
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        partial[blockIdx.x] = red[0];
        partial[gridDim.x + blockIdx.x] = rs[0];
    }
}

__global__ __launch_bounds__(256) void k_fqz_entropy(FqzEvJob J, double *partial) {
    double acc = 0.0, slack = 0.0;
    for (uint32_t k = blockIdx.x * blockDim.x + threadIdx.x; k < J.nev; k += gridDim.x * blockDim.x) {
        const uint64_t c = J.code[k];
        const uint32_t f = uint32_t(c >> 16) & 0xffffu, t = uint32_t(c >> 32);
        acc += log2(double(t)) - log2(double(f));
        slack += rc_slack(double(t));
    }
    entropy_reduce(acc, slack, partial);
}

// The same bound from coder records {RN(1/total) (2 words), freq, cum} in
// stream order (the sequence model's events): log2(total) = -log2(RN(1/total))
// to within 2^-52 relative, far inside the host's margin.
__global__ __launch_bounds__(256) void k_rec_entropy(const uint4 *rec, uint32_t nev, double *partial) {
    double acc = 0.0, slack = 0.0;
    for (uint32_t k = blockIdx.x * blockDim.x + threadIdx.x; k < nev; k += gridDim.x * blockDim.x) {
        const uint4 r = rec[k];
        const double rn = __longlong_as_double((long long)((uint64_t(r.y) << 32) | r.x));
        acc += -log2(rn) - log2(double(r.z));
        slack += rc_slack(rint(1.0 / rn));
    }
    entropy_reduce(acc, slack, partial);
}

hipError_t launch_rec_entropy(const uint4 *rec, uint32_t nev, double *partial, uint32_t nblk,
                              hipStream_t s) {
    if (nblk) hipLaunchKernelGGL(k_rec_entropy, dim3(nblk), dim3(256), 0, s, rec, nev, partial);
    return hipGetLastError();
}

hipError_t launch_fqz_entropy(const FqzEvJob &j, double *partial, uint32_t nblk, hipStream_t s) {
    if (nblk) hipLaunchKernelGGL(k_fqz_entropy, dim3(nblk), dim3(256), 0, s, j, partial);
    return hipGetLastError();
}

// Phase 3b: per event (in stream order) the record the range chain reads:
// {RN(1/total) as two words, freq, cum}.
__global__ void k_fqz_expand(FqzEvJob J) {
    const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= J.nev) return;
    const uint32_t e = uint32_t(J.sval[k] >> 8);
    const uint64_t c = J.code[k];
    const double rd = 1.0 / double(uint32_t(c >> 32));
    const uint64_t bits = uint64_t(__double_as_longlong(rd));
    J.rec[e] = make_uint4(uint32_t(bits), uint32_t(bits >> 32), uint32_t(c >> 16) & 0xffffu,
                          uint32_t(c) & 0xffffu);
}

// Phase 4: the range coder over the events in stream order (RC_Encode,
// c_range_coder.h:133-145).  The only serial dependence is the range:
//   q = range / total;  range = renorm(q * freq)
// k_rc_magic first turns each record's RN(1/total) into the divisor's
// round-up magic number (Granlund & Montgomery 1994, thm 4.2, N = 32):
// total t = rint(1 / RN(1/t)) exactly, l = ceil(log2 t), m = floor(2^32
// (2^l - t) / t) + 1 < 2^32; then for every range R < 2^32
//   q = floor(R / t) = (mulhi(R, m) + R) >> l    (a 33-bit sum)
// (t = 1: m = 1, l = 0; a power of two: m = 1).  k_fqz_rc runs the chain on
// the scalar unit: the range lives in an SGPR, the records come in 8 at a
// time by two s_load_dwordx16 (double buffered: a chunk's loads go out right
// after the wait for the previous one), and an event costs 8 scalar
// instructions (multiply-high, add, add-with-carry, 64-bit shift, multiply,
// find-first-bit, and, shift), no vector work and no LDS.  One wave issues
// about one instruction per 4 cycles, so the count is the cost.  The chain
// keeps only each group of 64 events' starting range (a lane of a vector
// register, stored per RC_BLK events); k_fqz_rc_replay then recomputes every
// event's q and byte-shift count, one lane per group, all in parallel.  The
// scalar loads run ahead of nothing: every RC_BLK events the wave warms L2
// with the next RC_BLK events' records by vector loads.
constexpr uint32_t RC_GRP = 64;                  // events per kept range
constexpr uint32_t RC_BLK = RC_GRP * 64;         // events per store of kept ranges
constexpr uint32_t RC_CH = 8;                    // events per scalar-load chunk

typedef uint32_t rc_u32x16 __attribute__((ext_vector_type(16)));
typedef const __attribute__((address_space(4))) rc_u32x16 *rc_cp16;
struct RcChunk { rc_u32x16 a, b; };
DEV RcChunk rc_chunk(const uint4 *p) {
    RcChunk c;
    c.a = ((rc_cp16)p)[0];
    c.b = ((rc_cp16)p)[1];
    return c;
}

// one event, record {m, l, f, cum}: q = (mulhi(R, m) + R) >> l, R = renorm(q * f)
DEV uint32_t rc_sstep(uint32_t R, uint32_t m, uint32_t l, uint32_t f) {
    const uint32_t q = uint32_t((uint64_t(__umulhi(R, m)) + R) >> l);
    R = q * f;
    return R << (uint32_t(__builtin_clz(R)) & 24u);
}

DEV void rc_chunk_steps(uint32_t &R, const RcChunk &X, RcChunk &Y, const uint4 *next) {
    R = rc_sstep(R, X.a[0], X.a[1], X.a[2]);   // (waits for X's loads)
    __builtin_amdgcn_sched_barrier(0);
    Y = rc_chunk(next);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (uint32_t i = 1; i < RC_CH; i++)
        R = i < 4 ? rc_sstep(R, X.a[4 * i], X.a[4 * i + 1], X.a[4 * i + 2])
                  : rc_sstep(R, X.b[4 * i - 16], X.b[4 * i - 15], X.b[4 * i - 14]);
    // all of X stays live to here: no temporary may take a register that
    // a load still in flight will write
    asm volatile("" ::"s"(X.a), "s"(X.b));
    __builtin_amdgcn_sched_barrier(0);
}

#ifdef FQZ5_RC_PROBE
__device__ uint64_t g_rcprobe[4];
extern "C" int fqz5_rc_probe_read(uint64_t *out) {
    return int(hipMemcpyFromSymbol(out, HIP_SYMBOL(g_rcprobe), sizeof(g_rcprobe)));
}
#endif

// J.rec has RC_PAD records of room past nev: the last group's chunks read
// into it (and the range past nev is never used).
__global__ __launch_bounds__(64) void k_fqz_rc(const FqzEvJob *Js) {
    const FqzEvJob J = load_job(Js + blockIdx.x);   // one wave per block of a batch
    const uint32_t l = threadIdx.x;
    const uint32_t nev = J.nev, ngrp = (nev + RC_GRP - 1) / RC_GRP;
    const auto rck = __builtin_amdgcn_make_buffer_rsrc(J.ck, 0, ngrp * 4u, 0x00020000);
    const auto rrec = __builtin_amdgcn_make_buffer_rsrc(J.rec, 0, nev * 16u, 0x00020000);
    uint32_t R = 0xFFFFFFFFu;
    // L2 warming: 8 dwords per lane, one per 128-byte line of the next RC_BLK
    // records; their values are folded in one block later (so the wait for
    // them never stalls the chain) and stored nowhere
    uint32_t warm[8], sink = 0;
#pragma unroll
    for (uint32_t r = 0; r < 8; r++)
        warm[r] = __builtin_amdgcn_raw_buffer_load_b32(rrec, (r * 64u + l) * 128u, 0, 0);
#ifdef FQZ5_RC_PROBE
    const uint64_t p0 = __builtin_amdgcn_s_memtime();
#endif
    RcChunk A = rc_chunk(J.rec), B;
    for (uint32_t base = 0; base < nev; base += RC_BLK) {
        const uint32_t blk = base / RC_BLK;
        // hedged launch (done != nullptr): 2-4 copies of the chain on
        // different CUs compute identical outputs.  *done is a claim word
        // (as in rans_chain.hip): the copy that starts this block first
        // writes it; ~0 means a copy has finished, and the others leave
        // after their current block.  The old value is looked at after it.
        uint32_t hedge = 0u;
        if (J.done && l == 0)
            hedge = __hip_atomic_fetch_max(J.done, blk + 1u, __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_AGENT);
#pragma unroll
        for (uint32_t r = 0; r < 8; r++) {
            sink ^= warm[r];
            warm[r] = __builtin_amdgcn_raw_buffer_load_b32(
                rrec, (base + RC_BLK) * 16u + (r * 64u + l) * 128u, 0, 0);
        }
        const uint32_t groups = min(64u, (nev - base + RC_GRP - 1) / RC_GRP);
        uint32_t v = 0;
        for (uint32_t g = 0; g < groups; g++) {
            v = l == g ? R : v;
            const uint4 *gp = J.rec + base + g * RC_GRP;
#pragma unroll
            for (uint32_t o = 0; o < RC_GRP; o += 2 * RC_CH) {
                rc_chunk_steps(R, A, B, gp + o + RC_CH);
                rc_chunk_steps(R, B, A, gp + o + 2 * RC_CH);
            }
        }
        hedge = __builtin_amdgcn_readlane(hedge, 0);
        if (hedge <= blk) __builtin_amdgcn_raw_buffer_store_b32(v, rck, (blk * 64u + l) * 4u, 0, 0);
        if (hedge == ~0u) return;
    }
    if (J.done && l == 0)
        __hip_atomic_store(J.done, ~0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    // (never true: keeps the warming loads)
    if (sink == 0x9e3779b9u && nev == 0u) J.ck[0] = sink;
#ifdef FQZ5_RC_PROBE
    if (l == 0 && blockIdx.x == 0) {
        g_rcprobe[0] = __builtin_amdgcn_s_memtime() - p0;
        g_rcprobe[1] = 0;
        g_rcprobe[2] = nev;
    }
#endif
}

// each event's q and byte-shift count from its group's starting range: a
// wave per 64 groups, lane t replays group t.  The records come in and the
// outputs go out through LDS, RP_CH events of every group at a time, so
// that a load or store instruction covers whole runs of consecutive events
// (a lane reading its own group straight from HBM strides 1 KB per lane).
constexpr uint32_t RP_CH = 16;
__global__ __launch_bounds__(64) void k_fqz_rc_replay(const FqzEvJob *Js) {
    const FqzEvJob J = load_job(Js + blockIdx.y);
    const uint32_t nev = J.nev, ngrp = (nev + RC_GRP - 1) / RC_GRP;
    const uint32_t g0 = blockIdx.x * 64u;
    if (g0 >= ngrp) return;
    __shared__ uint4 s_rec[64][RP_CH + 1];
    __shared__ uint32_t s_q[64][RP_CH + 1], s_k[64][RP_CH + 1];
    const uint32_t t = threadIdx.x;
    uint32_t R = g0 + t < ngrp ? J.ck[g0 + t] : 0u;
    for (uint32_t c = 0; c < RC_GRP; c += RP_CH) {
#pragma unroll 4
        for (uint32_t r = 0; r < RP_CH; r++) {
            const uint32_t j = r * 64u + t, gg = j / RP_CH, ee = j % RP_CH;
            const uint32_t e = (g0 + gg) * RC_GRP + c + ee;
            s_rec[gg][ee] = e < nev ? J.rec[e] : make_uint4(0, 0, 0, 0);
        }
        __syncthreads();
#pragma unroll 4
        for (uint32_t ee = 0; ee < RP_CH; ee++) {   // (past nev: never stored)
            const uint4 rr = s_rec[t][ee];
            const uint32_t q = uint32_t((uint64_t(__umulhi(R, rr.x)) + R) >> rr.y);
            const uint32_t nr = q * rr.z;
            const uint32_t sh = uint32_t(__builtin_clz(nr | 1u)) & 24u;
            s_q[t][ee] = q;          // cum * q in k_fqz_accum
            s_k[t][ee] = sh >> 3;
            R = nr << sh;
        }
        __syncthreads();
#pragma unroll 4
        for (uint32_t r = 0; r < RP_CH; r++) {
            const uint32_t j = r * 64u + t, gg = j / RP_CH, ee = j % RP_CH;
            const uint32_t e = (g0 + gg) * RC_GRP + c + ee;
            if (e < nev) {
                J.addend[e] = s_q[gg][ee];
                J.shifts[e] = s_k[gg][ee];
            }
        }
        __syncthreads();
    }
}

// each record's RN(1/total) into {m, l} (k_fqz_rc)
__global__ __launch_bounds__(256) void k_rc_magic(const FqzEvJob *Js) {
    const FqzEvJob J = load_job(Js + blockIdx.y);
    const uint32_t e = blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= J.nev) return;
    uint2 *p = reinterpret_cast<uint2 *>(J.rec + e);
    const uint2 w = *p;
    const double rd = __longlong_as_double((long long)(uint64_t(w.y) << 32 | w.x));
    const uint32_t t = uint32_t(rint(1.0 / rd));
    const uint32_t l = t > 1 ? 32u - uint32_t(__clz(int(t - 1))) : 0u;
    const uint32_t m = uint32_t((((uint64_t(1) << l) - t) << 32) / t + 1);
    *p = make_uint2(m, l);
}

// The coder's output is the base-256 number S = sum_i addend_i *
// 256^(P - P_i) written as P + 5 bytes, most significant first (P_i: shifts
// before event i, P: all shifts): low is a 4-byte window that moves one byte
// per shift, and the pending-byte / FF-run / carry logic of RC_ShiftLow
// (c_range_coder.h:78-101) is exactly the carry propagation of that sum.
// Phase A: add every addend into little-endian 32-bit columns (u64 each).
__global__ void k_fqz_accum(FqzEvJob J) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= J.nev) return;
    const uint32_t e = *J.nshift - J.pos[i];          // byte index of the LSB
    const uint32_t cum = J.rec[i].w;
    const uint64_t v = uint64_t(cum * J.addend[i]) << (8 * (e & 3));
    atomicAdd(&J.acc[e >> 2], (unsigned long long)(v & 0xffffffffull));
    if (v >> 32) atomicAdd(&J.acc[(e >> 2) + 1], (unsigned long long)(v >> 32));
}

// Phase B: carry propagation through the columns, in parallel.  The
// serial form is t = acc[w] + carry; digit_w = t mod 2^32; carry = t >> 32.
// hi(acc[w]) < 2^31 (a column takes one low part per event and nev < 2^31),
// so the carry out of word w is hi(acc[w]) + b_{w+1} with a bit
//   b_{w+1} = [s_w + b_w >= 2^32],   s_w = lo(acc[w]) + hi(acc[w-1]),
// and digit_w = (s_w + b_w) mod 2^32.  Word w thus kills (s_w < 2^32 - 1),
// propagates (s_w = 2^32 - 1) or generates (s_w >= 2^32) the bit: B1 writes
// s_w mod 2^32 and that code, an inclusive scan composes the codes
// (fqz_carry_scan: the later one wins unless it propagates), and B2 adds
// b_w = [prefix w-1 generates] to every digit.
__global__ void k_fqz_norm1(FqzEvJob J, uint32_t *sw, uint8_t *code) {
    const uint32_t w = blockIdx.x * blockDim.x + threadIdx.x;
    if (w >= J.nwords) return;
    const unsigned long long a0 = J.acc[w], a1 = w ? J.acc[w - 1] : 0ull;
    const unsigned long long sv = (a0 & 0xffffffffull) + (a1 >> 32);
    sw[w] = uint32_t(sv);
    code[w] = sv >> 32 ? FQZ_CARRY_GEN : (uint32_t(sv) == 0xffffffffu ? FQZ_CARRY_PROP : FQZ_CARRY_KILL);
}

__global__ void k_fqz_norm2(FqzEvJob J, const uint32_t *sw, const uint8_t *pref) {
    const uint32_t w = blockIdx.x * blockDim.x + threadIdx.x;
    if (w >= J.nwords) return;
    const uint32_t b = (w && pref[w - 1] == FQZ_CARRY_GEN) ? 1u : 0u;
    J.acc[w] = uint32_t(sw[w] + b);
}

// Phase C: bytes, most significant first.
__global__ void k_fqz_emit(FqzEvJob J) {
    const uint32_t nb = *J.nshift + 5;
    const uint32_t d = blockIdx.x * blockDim.x + threadIdx.x;
    if (d == 0) *J.out_len = nb;
    if (d >= nb) return;
    const uint32_t e = nb - 1 - d;
    J.out[d] = uint8_t(J.acc[e >> 2] >> (8 * (e & 3)));
}

hipError_t launch_fqz_events(const FqzEvJob &j, int phase, hipStream_t s) {
    if (phase == 0 && j.nrec)
        hipLaunchKernelGGL(k_fqz_ev_count, dim3((j.nrec + 255) / 256), dim3(256), 0, s, j);
    else if (phase == 1 && j.nrec)
        hipLaunchKernelGGL(k_fqz_ev_fill, dim3((j.nrec + 63) / 64), dim3(64), 0, s, j);
    else if (phase == 2 && j.nev)
        hipLaunchKernelGGL(k_fqz_segments, dim3((j.nev + 255) / 256), dim3(256), 0, s, j);
    return hipGetLastError();
}

hipError_t launch_fqz_expand(const FqzEvJob &j, hipStream_t s) {
    if (j.nev) hipLaunchKernelGGL(k_fqz_expand, dim3((j.nev + 255) / 256), dim3(256), 0, s, j);
    return hipGetLastError();
}

hipError_t launch_fqz_model_hot(const FqzEvJob *d_jobs, int njobs, uint32_t *hot,
                                uint32_t stride, uint32_t hot_min, hipStream_t s) {
    if (!njobs || !hot_min) return hipSuccess;
    hipLaunchKernelGGL(k_fqz_hot_list, dim3((FQZ_M_SEL + 255) / 256, njobs), dim3(256), 0, s,
                       d_jobs, hot, stride, hot_min);
    // a wave per hot model (up to stride - 1 of them per block), at
    // least FQZ_HOT_GRID: the launch then lasts as long as the longest
    // model's chain, not a wave's share of a thousand models (-7 ONT:
    // ~1 000 hot models per FQZ0 candidate)
    const uint32_t grid = std::min(std::max(stride - 1, FQZ_HOT_GRID), FQZ_HOT_GRID_MAX);
    hipLaunchKernelGGL(k_fqz_model_hot, dim3(grid, njobs), dim3(64), 0, s, d_jobs,
                       hot, stride);
    return hipGetLastError();
}

hipError_t launch_fqz_model_pass(const FqzEvJob *d_jobs, int njobs, uint32_t hot_min,
                                 hipStream_t s) {
    constexpr uint32_t lds = 256 * sizeof(FList<FQZ_QSYMS>);
    constexpr uint32_t nblk = (FQZ_NMODELS + 255) / 256;
    static bool attr = false;
    if (!attr) {
        (void)hipFuncSetAttribute(reinterpret_cast<const void *>(k_fqz_model_pass),
                                  hipFuncAttributeMaxDynamicSharedMemorySize, lds);
        attr = true;
    }
    if (!njobs) return hipSuccess;
    hipLaunchKernelGGL(k_fqz_model_pass, dim3(nblk * uint32_t(njobs)), dim3(256), lds, s,
                       d_jobs, nblk, hot_min);
    return hipGetLastError();
}

hipError_t launch_fqz_rc(const FqzEvJob *d_jobs, int njobs, int nbase, uint32_t max_nev,
                         int phase, hipStream_t s) {
    if (!njobs || !nbase) return hipSuccess;
    if (phase != 1 && !max_nev) return hipSuccess;
    if (phase == 0)
        hipLaunchKernelGGL(k_rc_magic, dim3((max_nev + 255) / 256, uint32_t(nbase)), dim3(256), 0, s,
                           d_jobs);
    else if (phase == 1)
        hipLaunchKernelGGL(k_fqz_rc, dim3(uint32_t(njobs)), dim3(64), 0, s, d_jobs);
    else {
        const uint32_t ngrp = (max_nev + RC_GRP - 1) / RC_GRP;
        hipLaunchKernelGGL(k_fqz_rc_replay, dim3((ngrp + 63) / 64, uint32_t(nbase)), dim3(64), 0,
                           s, d_jobs);
    }
    return hipGetLastError();
}

hipError_t launch_fqz_norm(const FqzEvJob &j, int phase, uint32_t *sw, uint8_t *code,
                           hipStream_t s) {
    if (!j.nwords) return hipSuccess;
    const dim3 grid((j.nwords + 255) / 256);
    if (phase == 1) hipLaunchKernelGGL(k_fqz_norm1, grid, dim3(256), 0, s, j, sw, code);
    else hipLaunchKernelGGL(k_fqz_norm2, grid, dim3(256), 0, s, j, sw, code);
    return hipGetLastError();
}

// phase 0: columns; 2: bytes (grid from the host's bound); carries: launch_fqz_carry
hipError_t launch_fqz_bytes(const FqzEvJob &j, int phase, hipStream_t s) {
    if (phase == 0 && j.nev)
        hipLaunchKernelGGL(k_fqz_accum, dim3((j.nev + 255) / 256), dim3(256), 0, s, j);
    else if (phase == 2)
        hipLaunchKernelGGL(k_fqz_emit, dim3((4 * j.nwords + 255) / 256), dim3(256), 0, s, j);
    return hipGetLastError();
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


}  // namespace fqz5
