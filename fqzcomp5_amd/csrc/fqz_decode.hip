// fqz_decode.hip — fqzcomp_qual decoder (uncompress_block_fqz2f,
// fqzcomp_qual.c:1410-1634) on one wavefront per block.
//
// Decoding is one dependent chain per block: every symbol needs the coder
// state and the model of its context, both left by the previous symbol.  A
// single wave issues roughly one instruction every four cycles, so the loop
// is built to minimise instructions per symbol rather than latency alone:
//
//  * the coder (range, code, input window) is uniform scalar state;
//  * the quality model of the current context sits in lanes: lane j holds
//    list slot j as freq | cum << 16 and its symbol, with a sentinel slot
//    `live` whose cum is the list total.  The reference's linear scan
//    (c_simple_model.h:136-171) becomes one ballot: with q = range / total,
//    the decoded slot k is the last j with cum_j * q <= code, since
//    t = code / q >= cum_j  <=>  code >= cum_j * q.  k == live means
//    t >= total (only in corrupt streams: symbol 0, no update).  The new
//    range is p_{k+1} - p_k = freq_k * q without another multiply;
//  * q = floor(range / total) is (u32)fma(range, RN(1/total), 2^-19), exact
//    for range < 2^32 and total < 2^16 whenever the stored reciprocal is
//    within one ulp (see fqz_div_selftest);
//  * while the ballot runs, every lane computes the context its own symbol
//    would lead to (fqz_update_ctx, fqzcomp_qual.c:361-418) and that
//    context's cache address, so the next model read waits only for a
//    readlane;
//  * models live in a direct-mapped LDS cache (~125 KB) backed by HBM;
//    blocks touch a few thousand of the 65536 contexts;
//  * output symbols go through LDS in 4 KB pages; qmap, duplicate records
//    and GFLAG_DO_REV reversal are applied by parallel fix-up kernels.
#include <hip/hip_runtime.h>
#include <cstdint>

#include "fqz_kernels.h"
#include "fqz_model.hpp"
#include "fqz_dec_common.hpp"

// v_writelane_b32 (the LLVM intrinsic; this clang has no builtin for it)
__device__ int amdgcn_writelane(int value, int lane, int old) __asm("llvm.amdgcn.writelane");

namespace fqz5 {
namespace {

using dec::RING;
using dec::HALF;
constexpr uint32_t OBUF = 4096;                // output page
constexpr uint32_t SEQB = 2048;                // staged sequence bases
constexpr uint32_t PBYTES = 3072;              // qtab u16[256], ptab u16[1024], dtab u16[256]
constexpr uint32_t P_QTAB = 0, P_PTAB = 512, P_DTAB = 2560;

constexpr uint32_t L_SMALL = 0;
constexpr uint32_t L_PAR = 4096;
constexpr uint32_t L_RING = L_PAR + FQZ_MAX_PARAMS * PBYTES;   // 16384
constexpr uint32_t L_OBUF = L_RING + RING + 16;
constexpr uint32_t L_DUMMY = L_OBUF + OBUF;                     // lanes != 0 write here
constexpr uint32_t L_SEQ = L_DUMMY + 256;
constexpr uint32_t L_BITS = L_SEQ + SEQB;                       // evicted-model bitmap
constexpr uint32_t L_CACHE = L_BITS + FQZ_CTX / 8;
constexpr uint32_t LDS_BYTES = 163840;
static_assert(L_CACHE == 35088, "keep FQZ_DEC_CACHE_BYTES in step");
static_assert(sizeof(SmallModels) <= L_PAR, "small models");
static_assert(L_CACHE + FQZ_DEC_CACHE_BYTES + 1024 == LDS_BYTES, "cache bytes");

using dec::rsrc;
using dec::ld8;
using dec::st8;
using dec::U;
using dec::RL;
using dec::In;
using dec::PS;
using dec::load_ps;
using dec::small_init;

#ifdef FQZ5_DEC_PROBE   // cycle stamps per stage of the fast loop (tools/)
#define PROBE_DECL uint64_t pr_t = 0, pr_x = 0, pr[6] = {0, 0, 0, 0, 0, 0};
#define PROBE_START pr_t = __builtin_amdgcn_s_memtime();
#define PROBE(i)                                        \
    {                                                   \
        const uint64_t t_ = __builtin_amdgcn_s_memtime(); \
        pr[i] += t_ - pr_t;                             \
        pr_t = t_;                                      \
    }
#define PROBE_OUT                                                            \
    if (l == 0)                                                              \
        for (int i = 0; i < 6; i++) reinterpret_cast<uint64_t *>(J.counts + 8)[i] = pr[i];
#else
#define PROBE_DECL
#define PROBE_START
#define PROBE(i)
#define PROBE_OUT
#endif



// the shared input / small-model helpers (fqz_dec_common.hpp) at this
// kernel's ring offset
DEV void stage(uint8_t *lds, const In &in) { dec::stage<L_RING>(lds, in); }
DEV void refill(uint8_t *lds, In &in) { dec::refill<L_RING>(lds, in); }
DEV void renorm_slow(uint8_t *lds, In &in, uint32_t &rng, uint32_t &code) {
    dec::renorm_slow<L_RING>(lds, in, rng, code);
}
template <int CAP> DEV uint32_t small_decode(FList<CAP> *m, uint8_t *lds, In &in, uint32_t &rng, uint32_t &code) {
    return dec::small_decode<L_RING>(m, lds, in, rng, code);
}

// cache set of a context: multiplicative hash with 24-bit multiplies
// (full rate), then a 24-bit fraction scaled to the set count
DEV uint32_t set_addr(uint32_t ctx, uint32_t ns8, uint32_t me) {
    const uint32_t h = ctx * 0x9E3779u;                             // low 24 bits used
    const uint32_t set = uint32_t((uint64_t(h & 0xffffffu) * (ns8 & 0xffffffu)) >> 32);
    return L_CACHE + (set & 0xffffu) * (me & 0xffffu);   // both < 2^16: v_mad_u32_u24
}


// ---------------------------------------------------------------------------
// The fast run of k_fqz_dec<NE = 1> as one hand-scheduled loop, a symbol per
// iteration.  The model of the current context sits in a VGPR pair, lane j
// holding slot j (e = freq | cum << 16 in the low register, w = qtab value |
// symbol << 24 in the high one), with the sentinel (e = context | total <<
// 16) broadcast to every lane in tv.  Per symbol:
//   miss    the sentinel names another context (the set holds another
//           context's model): the miss path (below) brings this one in and
//           the symbol starts over, before any work that needs the model
//   u       the context terms of this position and delta (pvv / dvv lanes)
//   q       floor(range / total) from RN(1/total) (rcp + one Newton step)
//   p_j     cum_j * q;  G = lanes with p_j > code;  kl = first of G - 1
//   every lane j: the context its symbol leads to (fqz_update_ctx), that
//           context's cache set, qctx << qshift, whether it is this context
//           again (SM), and whether the bump would bubble slot j over j-1
//   the next model's read is issued from lane kl's set as soon as kl is
//   known, into the other register pair; the checks (a total that the +16
//   would take past FL_MAX, t >= total) leave with flags 2 before any
//   state changes
//   bump    +16 to lane kl's frequency and every later cum; one bubble step
//           by DPP lane shifts when it swaps; the model is written back
//   coder   c_range_coder.h RC_Decode: code -= cum q, range = freq q,
//           renormalise by whole bytes from the 64-bit window
// Two register pairs (A: v[2:3], B: v[4:5]) and two copies of the scalar
// state that a context change replaces (context, qctx << qshift, previous
// symbol, model address, sequence context): iteration X moves into Y when
// the context changes and loops on itself when it repeats.  code is s41 with
// s40 its scratch ({s40, s41} << z brings the window's top bits in), the
// window is s[42:43].  m0 counts the run's symbols (lane selects).
// It leaves after `lim` symbols or when the input window needs a refill,
// writing the current model back (unless its sentinel names another
// context: the read of a context that shares the set).
// gfx950 wait states: DPP reads of a VGPR written by the VALU get two, an
// SGPR written by the SALU and read as a VALU mask two (s_nop 1).
// ---------------------------------------------------------------------------
#define FQZ_QT1_W(WX) ""
#define FQZ_QT2_W(X, WX) "v_add_u32 %[t0], %[qs" X "], " WX "\n"
#define FQZ_QT1_TAB(WX)                                                     \
    "v_lshrrev_b32 %[t0], 24, " WX "\n"                                     \
    "v_lshl_add_u32 %[t0], %[t0], 1, %[qtab]\n"                             \
    "ds_read_u16 %[t0], %[t0]\n"
#define FQZ_QT2_TAB(X, WX)                                                  \
    "s_waitcnt lgkmcnt(0)\n"                                                \
    "v_add_u32 %[t0], %[qs" X "], %[t0]\n"
#define FQZ_SEQ_NONE(X, Y) ""
#define FQZ_SEQ_CTX(X, Y)                                                   \
    "v_readlane_b32 %[x], %[sqv], m0\n"                                     \
    "s_lshl_b32 %[sq" Y "], %[sq" X "], 2\n"                                \
    "s_or_b32 %[sq" Y "], %[sq" Y "], %[x]\n"                               \
    "s_and_b32 %[sq" Y "], %[sq" Y "], %[bmask]\n"                          \
    "s_lshl_b32 %[x], %[sq" Y "], %[bloc]\n"                                \
    "s_add_u32 %[u], %[u], %[x]\n"
#define FQZ_SEQ_SAME(X, Y) "s_mov_b32 %[sq" X "], %[sq" Y "]\n"
// the symbol's decode and the next context's hypotheses; leaves for SAMEL
// when the context repeats.  The wait is for the model read (the write-back
// issued after it may still be in flight); an iteration of the same context
// enters at SKIPL, past it.  WCNT: the writes issued after the read.
#define FQZ_TOP(X, Y, EX, WX, QT1, QT2, SEQCTX, WCNT, SKIPL, SAMEL, MISSL)  \
    "s_waitcnt lgkmcnt(" WCNT ")\n"                                         \
    SKIPL ":\n"                                                             \
    "v_cmp_ne_u16_e32 vcc, %[c" X "], %[tv" X "]\n"                         \
    "v_readlane_b32 %[u], %[pvv], m0\n"                                     \
    "v_lshrrev_b32 %[t6], 16, %[tv" X "]\n"                                 \
    "v_readlane_b32 %[x], %[dvv], %[dd]\n"                                  \
    "v_cvt_f64_u32 %[d1], %[t6]\n"                                          \
    QT1(WX)                                                                 \
    "v_cvt_f64_u32 %[d0], %[rng]\n"                                         \
    "v_rcp_f64 %[d2], %[d1]\n"                                              \
    "s_add_u32 %[u], %[u], %[x]\n"                                          \
    SEQCTX(X, Y)                                                            \
    "s_cbranch_vccnz " MISSL "\n"                                           \
    "v_lshrrev_b32 %[t4], 16, " EX "\n"                                     \
    "v_fma_f64 %[d1], -%[d1], %[d2], 1.0\n"                                 \
    QT2(X, WX)                                                              \
    "v_cmp_lt_u32_e64 %[HV], %[c65503], %[t6]\n"                            \
    "v_fma_f64 %[d2], %[d2], %[d1], %[d2]\n"                                \
    "v_and_b32 %[t1], %[qmask], %[t0]\n"                                    \
    "v_add_u16 %[t5], 16, " EX "\n"                                         \
    "v_fma_f64 %[d0], %[d0], %[d2], %[c19]\n"                               \
    "v_lshl_add_u32 %[t1], %[t1], %[qlocv], %[u]\n"                         \
    "v_mov_b32_dpp %[t6], " EX " wave_shr:1 row_mask:0xf bank_mask:0xf\n"   \
    "v_cvt_u32_f64 %[t3], %[d0]\n"                                          \
    "v_and_b32 %[t1], 0xffff, %[t1]\n"                                      \
    "v_mul_lo_u32 %[t3], %[t4], %[t3]\n"                                    \
    "v_mul_u32_u24 %[t2], 0x9e3779, %[t1]\n"                                \
    "v_cmp_eq_u32_e64 %[SM], %[c" X "], %[t1]\n"                            \
    "v_mul_hi_u32_u24 %[t2], %[ns8], %[t2]\n"                               \
    "v_cmp_gt_u32_e64 %[G], %[t3], s41\n"                                   \
    "v_mad_u32_u24 %[t2], %[t2], %[vme], %[base]\n"                         \
    "v_cmp_lt_u16_e64 %[SW], %[t6], %[t5]\n"                                \
    "s_ff1_i32_b64 %[k1], %[G]\n"                                           \
    "s_lshr_b64 %[E], %[G], 1\n"                                            \
    "s_sub_u32 %[kl], %[k1], 1\n"                                           \
    "s_andn2_b64 %[E], %[E], %[G]\n"                                        \
    "v_readlane_b32 %[ma" Y "], %[t2], %[kl]\n"                             \
    "s_and_b64 %[SM], %[SM], %[E]\n"                                        \
    "s_cbranch_scc1 " SAMEL "\n"
// the checks; SLOWL leaves with the state unchanged
#define FQZ_CHECK(SLOWL)                                                    \
    "s_andn2_b64 %[E], %[E], %[HV]\n"                                       \
    "s_cbranch_scc0 " SLOWL "\n"
// the coded slot's update (fl_bump): +16 to lane kl's frequency (E) and to
// every later cum (G); a bubble step (SW & E) goes out of line to SWL and
// comes back to RETL
#define FQZ_BUMP(EX, SWL, RETL)                                             \
    "v_cndmask_b32 %[t4], 0, 16, %[E]\n"                                    \
    "v_cndmask_b32 %[t4], %[t4], %[cbig], %[G]\n"                           \
    "s_and_b64 %[SW], %[SW], %[E]\n"                                        \
    "v_add_u32 " EX ", " EX ", %[t4]\n"                                     \
    "s_cbranch_scc1 " SWL "f\n"                                             \
    RETL ":\n"
// one bubble step by DPP lane shifts: slot kl over slot kl-1
#define FQZ_SWAP(EX, WX, SWL, RETL)                                         \
    SWL ":\n"                                                               \
    "s_nop 1\n"                                                             \
    "v_mov_b32_dpp %[t4], " EX " wave_shr:1 row_mask:0xf bank_mask:0xf\n"   \
    "v_mov_b32_dpp %[t5], " EX " wave_shl:1 row_mask:0xf bank_mask:0xf\n"   \
    "v_mov_b32_dpp %[t6], " WX " wave_shr:1 row_mask:0xf bank_mask:0xf\n"   \
    "v_mov_b32_dpp %[t1], " WX " wave_shl:1 row_mask:0xf bank_mask:0xf\n"   \
    "v_and_b32 %[t3], 0xffff, " EX "\n"                                     \
    "v_lshrrev_b32 %[t2], 16, %[t4]\n"                                      \
    "v_add_u32 %[t3], %[t3], %[t2]\n"                                       \
    "v_and_b32 %[t2], 0xffff, %[t4]\n"                                      \
    "v_lshl_or_b32 %[t3], %[t3], 16, %[t2]\n"                               \
    "v_and_b32 %[t2], 0xffff0000, " EX "\n"                                 \
    "v_and_b32 %[t5], 0xffff, %[t5]\n"                                      \
    "v_or_b32 %[t5], %[t5], %[t2]\n"                                        \
    "s_lshr_b64 %[SW], %[E], 1\n"                                           \
    "v_cndmask_b32 " EX ", " EX ", %[t3], %[E]\n"                           \
    "v_cndmask_b32 " WX ", " WX ", %[t6], %[E]\n"                           \
    "s_nop 1\n"                                                             \
    "v_cndmask_b32 " EX ", " EX ", %[t5], %[SW]\n"                          \
    "v_cndmask_b32 " WX ", " WX ", %[t1], %[SW]\n"                          \
    "s_branch " RETL "b\n"
// the slot's values: range coder terms, qctx, symbol (into pv Y)
#define FQZ_TAKE(Y, WX)                                                     \
    "v_readlane_b32 %[pk], %[t3], %[kl]\n"                                  \
    "v_readlane_b32 %[pk1], %[t3], %[k1]\n"                                 \
    "v_readlane_b32 %[qsk], %[t0], %[kl]\n"                                 \
    "v_readlane_b32 %[pv" Y "], " WX ", %[kl]\n"
// renormalise by whole bytes (z = 0, 8, 16 or 24 bits) out of line at RNL,
// back at RETL; then the run's symbol limit
#define FQZ_RENORM(RNL, RETL)                                               \
    "s_and_b32 %[z], %[z], 24\n"                                            \
    "s_cbranch_scc1 " RNL "f\n"                                             \
    RETL ":\n"                                                              \
    "s_cmp_lt_u32 m0, %[lim]\n"
// When the window runs low (ub > ulim) its next 4 bytes come from the LDS
// input ring (stream bytes rb + 8 .. rb + 11, big-endian into the window
// below its valid bits); EXITL when the ring does not hold them yet (the
// run's caller stages the next half) or the input ends.
#define FQZ_RENORM_OUT(RNL, RETL, EXITL)                                    \
    RNL ":\n"                                                               \
    "s_mov_b32 s40, s43\n"                                                  \
    "s_lshl_b64 s[40:41], s[40:41], %[z]\n"                                 \
    "s_lshl_b64 s[42:43], s[42:43], %[z]\n"                                 \
    "s_lshl_b32 %[rng], %[rng], %[z]\n"                                     \
    "s_add_u32 %[ub], %[ub], %[z]\n"                                        \
    "s_cmp_gt_u32 %[ub], %[ulim]\n"                                         \
    "s_cbranch_scc0 " RETL "b\n"                                            \
    "s_cmp_ge_u32 %[rb], %[rbend]\n"                                        \
    "s_cbranch_scc1 " EXITL "\n"                                            \
    "s_add_u32 %[x], %[rb], 8\n"                                            \
    "s_and_b32 %[k1], %[x], 0xffc\n"                                        \
    "s_and_b32 %[kl], %[x], 3\n"                                            \
    "s_add_u32 %[k1], %[k1], %[lring]\n"                                    \
    "v_mov_b32 %[t4], %[k1]\n"                                              \
    "ds_read_b32 %[t5], %[t4]\n"                                            \
    "ds_read_b32 %[t6], %[t4] offset:4\n"                                   \
    "s_lshl_b32 %[kl], %[kl], 3\n"                                          \
    "s_sub_u32 %[ub], %[ub], 32\n"                                          \
    "s_add_u32 %[rb], %[rb], 4\n"                                           \
    "s_waitcnt lgkmcnt(0)\n"                                                \
    "v_alignbit_b32 %[t5], %[t6], %[t5], %[kl]\n"                           \
    "v_perm_b32 %[t5], %[t5], %[t5], %[bswp]\n"                             \
    "s_mov_b32 s45, 0\n"                                                    \
    "v_readfirstlane_b32 s44, %[t5]\n"                                      \
    "s_lshl_b64 s[44:45], s[44:45], %[ub]\n"                                \
    "s_or_b64 s[42:43], s[42:43], s[44:45]\n"                               \
    "s_branch " RETL "b\n"
// A miss (the set holds another context, ev): ev's model, read again from
// the set (the read that found it may predate the last write-back of the
// same set), goes back to HBM (J.back, plain stores and loads: the store is
// private to this wave, so its lines may stay in the caches; device scope,
// sc1, sent every fetch past the XCD's L2) and into the LDS bitmap of evicted
// contexts; the current context's comes from HBM when the bitmap has it,
// else fresh (fe / fw; the sentinel lanes get context | L << 16); then the
// set is rewritten and the symbol starts over at SKIPL.
#define FQZ_MSENT_NONE(X, Y) ""
#define FQZ_MSENT_NONE1(X) ""
#define FQZ_MSENT_ST(X, Y)                                                  \
    "v_mad_u32_u24 %[t5], %[x], %[vme], %[vsent]\n"                         \
    "global_store_dword %[t5], %[tv" X "], %[back]\n"
// a context's model from HBM into v[6:7] (and tvp: PFT)
#define FQZ_FETCH(C, PFT)                                                   \
    "v_mad_u32_u24 %[t4], %[c" C "], %[vme], %[voff]\n"                     \
    "global_load_dwordx2 v[6:7], %[t4], %[back]\n"                          \
    PFT(C)
#define FQZ_IF_0(a, b) b
#define FQZ_IF_1(a, b) a
#define FQZ_IF(P, a, b) FQZ_IF_##P(a, b)
#define FQZ_PF_NONE(Y) ""
#define FQZ_PF_SENT(Y)                                                      \
    "v_mad_u32_u24 %[t5], %[c" Y "], %[vme], %[vsent]\n"                    \
    "global_load_dword %[tvp], %[t5], %[back]\n"
#define FQZ_MSENT_MOV(X, Y, EX) "v_mov_b32 %[tv" X "], %[tvp]\n"
#define FQZ_MSENT_LANE(X, Y, EX)                                            \
    "v_readlane_b32 %[x], " EX ", %[sidx]\n"                                \
    "v_mov_b32 %[tv" X "], %[x]\n"
#define FQZ_MSENT_WR(X)                                                     \
    "v_add_u32 %[t5], %[ma" X "], %[vsent]\n"                               \
    "ds_write_b32 %[t5], %[tv" X "]\n"
// With PF = 1 (a run that misses often) the model of every context the run
// switches to (and of the one it starts in, which the caller may not have
// brought in) is fetched from HBM at the switch, speculatively, so that a
// miss finds it on its way; with PF = 0 the miss fetches it first thing.
// The miss reads the set and the bitmap word together and writes the
// resident model back; the wait is for the fetch only (MVW: the write-back
// stores issued after it).
#define FQZ_MISS(X, Y, MX, EX, WX, MY, EY, WY, MISSL, SKIPL, MST, PF, PFT, MMOV, MWB, MVW) \
    MISSL ":\n"                                                             \
    "s_waitcnt lgkmcnt(0)\n"                                                \
    FQZ_IF(PF, "", FQZ_FETCH(X, PFT))                                       \
    "s_lshr_b32 %[k1], %[c" X "], 3\n"                                      \
    "s_and_b32 %[k1], %[k1], 0x1ffc\n"                                      \
    "s_add_u32 %[k1], %[k1], %[lbits]\n"                                    \
    "v_add_u32 %[t4], %[ma" X "], %[voff]\n"                                \
    "v_add_u32 %[t5], %[ma" X "], %[vsent]\n"                               \
    "v_mov_b32 %[t6], %[k1]\n"                                              \
    "ds_read_b64 " MX ", %[t4]\n"                                           \
    "ds_read_b32 %[tv" X "], %[t5]\n"                                       \
    "ds_read_b32 %[t6], %[t6]\n"                                            \
    "s_add_u32 %[nm], %[nm], 1\n"                                           \
    "s_waitcnt lgkmcnt(0)\n"                                                \
    "v_readfirstlane_b32 %[x], %[tv" X "]\n"                                \
    "v_readfirstlane_b32 %[kl], %[t6]\n"                                    \
    "s_and_b32 %[x], %[x], 0xffff\n"                                        \
    "v_mad_u32_u24 %[t4], %[x], %[vme], %[voff]\n"                          \
    "global_store_dwordx2 %[t4], " MX ", %[back]\n"                     \
    MST(X, Y)                                                               \
    "s_lshr_b32 %[k1], %[x], 3\n"                                           \
    "s_and_b32 %[k1], %[k1], 0x1ffc\n"                                      \
    "s_add_u32 %[k1], %[k1], %[lbits]\n"                                    \
    "s_lshl_b32 %[z], 1, %[x]\n"                                            \
    "v_mov_b32 %[t5], %[k1]\n"                                              \
    "v_mov_b32 %[t6], %[z]\n"                                               \
    "ds_or_b32 %[t5], %[t6]\n"                                              \
    "s_bitcmp1_b32 %[kl], %[c" X "]\n"                                      \
    "s_waitcnt vmcnt(" MVW ")\n"                                            \
    "s_cbranch_scc0 6f\n"                                                   \
    "v_mov_b32 " EX ", v6\n"                                                \
    "v_mov_b32 " WX ", v7\n"                                                \
    MMOV(X, Y, EX)                                                          \
    "s_branch 7f\n"                                                         \
    "6:\n"                                                                  \
    "s_or_b32 %[k1], %[c" X "], %[lsh]\n"                                   \
    "v_mov_b32 %[tv" X "], %[k1]\n"                                         \
    "v_cmp_eq_u32_e64 %[G], %[voff], %[vsent]\n"                            \
    "v_mov_b32 " WX ", %[fw]\n"                                             \
    "s_nop 1\n"                                                             \
    "v_cndmask_b32 " EX ", %[fe], %[tv" X "], %[G]\n"                       \
    "7:\n"                                                                  \
    "v_add_u32 %[t4], %[ma" X "], %[voff]\n"                                \
    "ds_write_b64 %[t4], " MX "\n"                                          \
    MWB(X)                                                                  \
    "s_branch " SKIPL "b\n"
// the coder and the context state; the symbol to output lane m0
#define FQZ_CODER(X, Y, QSD)                                                \
    "s_sub_u32 s41, s41, %[pk]\n"                                           \
    "s_sub_u32 %[rng], %[pk1], %[pk]\n"                                     \
    "s_lshr_b32 %[pv" Y "], %[pv" Y "], 24\n"                               \
    "s_flbit_i32_b32 %[z], %[rng]\n"                                        \
    "s_lshl_b32 %[qs" QSD "], %[qsk], %[qshift]\n"                          \
    "v_writelane_b32 %[vout], %[pv" Y "], m0\n"                             \
    "s_cmp_lg_u32 %[pv" X "], %[pv" Y "]\n"                                 \
    "s_addc_u32 %[dd], %[dd], 0\n"                                          \
    "s_add_u32 m0, m0, 1\n"
// the sentinel (total + 16), when no lane carries it (NE = 2)
#define FQZ_SENT_NONE(X) ""
#define FQZ_SENT_WB(X)                                                      \
    "v_add_u32 %[tv" X "], %[cbig], %[tv" X "]\n"                           \
    "v_add_u32 %[t5], %[ma" X "], %[vsent]\n"                               \
    "ds_write_b32 %[t5], %[tv" X "]\n"
#define FQZ_SENT_EXIT(X)                                                    \
    "v_add_u32 %[t5], %[ma" X "], %[vsent]\n"                               \
    "ds_write_b32 %[t5], %[tv" X "]\n"
// context change: the next model into (MY, tv Y), this one written back
#define FQZ_SWITCH(X, Y, MX, EX, WX, MY, SENTWB, PF, PFT, SLOWL, SWL, RNL, R1, R2) \
    "v_add_u32 %[t4], %[ma" Y "], %[voff]\n"                                \
    "v_add_u32 %[t5], %[ma" Y "], %[vsent]\n"                               \
    "ds_read_b64 " MY ", %[t4]\n"                                           \
    "ds_read_b32 %[tv" Y "], %[t5]\n"                                       \
    FQZ_CHECK(SLOWL)                                                        \
    "v_readlane_b32 %[c" Y "], %[t1], %[kl]\n"                              \
    FQZ_TAKE(Y, WX)                                                         \
    FQZ_IF(PF, FQZ_FETCH(Y, PFT), "")                                       \
    FQZ_BUMP(EX, SWL, R1)                                                   \
    "v_add_u32 %[t2], %[ma" X "], %[voff]\n"                                \
    "ds_write_b64 %[t2], " MX "\n"                                          \
    SENTWB(X)                                                               \
    FQZ_CODER(X, Y, Y)                                                      \
    FQZ_RENORM(RNL, R2)
// the same context again: the model stays in (MX, tv X)
#define FQZ_SAME(X, Y, EX, WX, SEQSAME, SLOWL, SWL, RNL, R1, R2)            \
    FQZ_CHECK(SLOWL)                                                        \
    FQZ_TAKE(Y, WX)                                                         \
    FQZ_BUMP(EX, SWL, R1)                                                   \
    "v_add_u32 %[tv" X "], %[cbig], %[tv" X "]\n"                           \
    FQZ_CODER(X, Y, X)                                                      \
    "s_mov_b32 %[pv" X "], %[pv" Y "]\n"                                    \
    SEQSAME(X, Y)                                                           \
    FQZ_RENORM(RNL, R2)
// labels: 10/20 the A/B iteration (13/23 past its wait), 11/21 their
// same-context paths, 12/22 the slow exits; 30 exits in the A state, 31 in
// the B state; 41-48 out-of-line bubble steps and renormalisations, 51-58
// their way back
#define FQZ_RUN_ASM(QT1, QT2, SEQCTX, SEQSAME, SENTWB, SENTEX, WCNT, MST, PF, PFT, MMOV, MWB, MVW) \
    "s_mov_b32 %[m0s], m0\n"                                                \
    "s_mov_b32 m0, %[done]\n"                                               \
    "s_mov_b32 %[flags], 0\n"                                               \
    FQZ_IF(PF, FQZ_FETCH("A", PFT), "")                                     \
    "10:\n"                                                                 \
    FQZ_TOP("A", "B", "v2", "v3", QT1, QT2, SEQCTX, WCNT, "13", "11f", "60f") \
    FQZ_SWITCH("A", "B", "v[2:3]", "v2", "v3", "v[4:5]", SENTWB, PF, PFT, "12f", "41", "42", "51", "52") \
    "s_cbranch_scc0 31f\n"                                                  \
    "20:\n"                                                                 \
    FQZ_TOP("B", "A", "v4", "v5", QT1, QT2, SEQCTX, WCNT, "23", "21f", "61f") \
    FQZ_SWITCH("B", "A", "v[4:5]", "v4", "v5", "v[2:3]", SENTWB, PF, PFT, "22f", "43", "44", "53", "54") \
    "s_cbranch_scc1 10b\n"                                                  \
    "s_branch 30f\n"                                                        \
    "11:\n"                                                                 \
    FQZ_SAME("A", "B", "v2", "v3", SEQSAME, "12f", "45", "46", "55", "56")  \
    "s_cbranch_scc1 13b\n"                                                  \
    "s_branch 30f\n"                                                        \
    "21:\n"                                                                 \
    FQZ_SAME("B", "A", "v4", "v5", SEQSAME, "22f", "47", "48", "57", "58")  \
    "s_cbranch_scc1 23b\n"                                                  \
    "s_branch 31f\n"                                                        \
    FQZ_SWAP("v2", "v3", "41", "51")                                        \
    FQZ_RENORM_OUT("42", "52", "31f")                                       \
    FQZ_SWAP("v4", "v5", "43", "53")                                        \
    FQZ_RENORM_OUT("44", "54", "30f")                                       \
    FQZ_SWAP("v2", "v3", "45", "55")                                        \
    FQZ_RENORM_OUT("46", "56", "30f")                                       \
    FQZ_SWAP("v4", "v5", "47", "57")                                        \
    FQZ_RENORM_OUT("48", "58", "31f")                                       \
    FQZ_MISS("A", "B", "v[2:3]", "v2", "v3", "v[4:5]", "v4", "v5", "60", "13", MST, PF, PFT, MMOV, MWB, MVW) \
    FQZ_MISS("B", "A", "v[4:5]", "v4", "v5", "v[2:3]", "v2", "v3", "61", "23", MST, PF, PFT, MMOV, MWB, MVW) \
    "12:\n"                                                                 \
    "s_mov_b32 %[flags], 2\n"                                               \
    "s_branch 30f\n"                                                        \
    "22:\n"                                                                 \
    "s_mov_b32 %[flags], 2\n"                                               \
    "31:\n"                                                                 \
    "s_waitcnt lgkmcnt(0)\n"                                                \
    "v_mov_b32 v2, v4\n"                                                    \
    "v_mov_b32 v3, v5\n"                                                    \
    "v_mov_b32 %[tvA], %[tvB]\n"                                            \
    "s_mov_b32 %[cA], %[cB]\n"                                              \
    "s_mov_b32 %[qsA], %[qsB]\n"                                            \
    "s_mov_b32 %[pvA], %[pvB]\n"                                            \
    "s_mov_b32 %[maA], %[maB]\n"                                            \
    "s_mov_b32 %[sqA], %[sqB]\n"                                            \
    "30:\n"                                                                 \
    "s_waitcnt lgkmcnt(0)\n"                                                \
    "v_cmp_ne_u16_e64 %[TG], %[cA], %[tvA]\n"                               \
    "s_cmp_lg_u64 %[TG], 0\n"                                               \
    "s_cbranch_scc1 5f\n"                                                   \
    "v_add_u32 %[t2], %[maA], %[voff]\n"                                    \
    "ds_write_b64 %[t2], v[2:3]\n"                                          \
    SENTEX("A")                                                             \
    "s_waitcnt lgkmcnt(0)\n"                                                \
    "5:\n"                                                                  \
    "s_waitcnt vmcnt(0)\n"                                                  \
    "s_mov_b32 %[done], m0\n"                                               \
    "s_mov_b32 m0, %[m0s]\n"

// ---------------------------------------------------------------------------
// the decoder.  Model in lanes: lane j holds slot j of the cached model
// (fqz_dec_model_bytes): a guard slot, the L list slots, the sentinel whose
// cum is the total and whose low half names the context the model belongs
// to.  QW: every parameter set shares one qtab, whose value for the slot's
// symbol sits in w (else the run reads the record's table).
// ---------------------------------------------------------------------------
template <int NE, bool SEQ, bool QW>
__global__ __launch_bounds__(64) void k_fqz_dec(const FqzDecJob *Js) {
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    const FqzDecJob J = load_job(Js + blockIdx.x);   // one block of a batch per workgroup
    const uint32_t l = threadIdx.x;
    const FqzDevGlobal &g = *J.g;
    SmallModels &sm = *reinterpret_cast<SmallModels *>(lds + L_SMALL);
    const uint32_t gfl = U(g.gflags), nparam = U(g.nparam);
    const uint32_t L = U(g.max_sym) + 1;              // live symbols per quality model
    const uint32_t ME = J.ment, NS = J.nsets, NS8 = NS << 8;
    // the hand-scheduled run addresses LDS by these offsets: the dynamic
    // block must start at LDS address 0 (no static __shared__ here)
    if (uint32_t(size_t((__attribute__((address_space(3))) uint8_t *)lds)) != 0) __builtin_trap();
    // the cached model: slots 0 .. LL and the sentinel S (NE = 2: the list
    // slots past lane 63 stay in HBM, J.back_hi)
    const uint32_t LL = L < 63u ? L : 63u, S = LL + 1u;
    const uint32_t sent = 8u * S;                     // the sentinel slot within a model
    const uint32_t n = uint32_t(J.n);

    // ---- set-up: small models, parameter tables, cache tags, bitmap ------
    for (int b = 0; b < 4; b++) small_init(&sm.len[b], 256);
    small_init(&sm.rev, 2);
    small_init(&sm.dup, 2);
    if (U(g.max_sel) > 0) small_init(&sm.sel, int(U(g.max_sel)) + 1);
    for (uint32_t x = 0; x < nparam; x++) {
        uint16_t *pt = reinterpret_cast<uint16_t *>(lds + L_PAR + x * PBYTES);
        for (uint32_t i = l; i < 256; i += 64) pt[(P_QTAB >> 1) + i] = uint16_t(g.p[x].qtab[i]);
        for (uint32_t i = l; i < 1024; i += 64) pt[(P_PTAB >> 1) + i] = uint16_t(g.p[x].ptab[i]);
        for (uint32_t i = l; i < 256; i += 64) pt[(P_DTAB >> 1) + i] = uint16_t(g.p[x].dtab[i]);
    }
    for (uint32_t i = l; i < FQZ_CTX / 32; i += 64) reinterpret_cast<uint32_t *>(lds + L_BITS)[i] = 0;
    const uint16_t *qt0 = reinterpret_cast<const uint16_t *>(lds + L_PAR + P_QTAB);
    __builtin_amdgcn_wave_barrier();
    // a fresh model (every live symbol frequency 1) in slots 0 .. LL; the
    // sentinel is written apart
    auto fresh_slots = [&](uint32_t a) {
        for (uint32_t j = l; j <= LL; j += 64) {
            const uint32_t e = j ? 1u | ((j - 1u) << 16) : 0xffffu;
            const uint32_t w = j ? uint32_t(qt0[j - 1u]) | ((j - 1u) << 24) : 0u;
            *reinterpret_cast<uint2 *>(lds + a + 8u * j) = make_uint2(e, w);
        }
    };
    // every cache set starts as the fresh model of a context that maps to
    // it, so that a set always holds some context's true state (sets no
    // context maps to are never read)
    for (uint32_t c = l; c < FQZ_CTX; c += 64)
        *reinterpret_cast<uint2 *>(lds + set_addr(c, NS8, ME) + sent) = make_uint2(c | (L << 16), 0u);
    for (uint32_t s = 0; s < NS; s++) fresh_slots(L_CACHE + s * ME);
    __builtin_amdgcn_wave_barrier();

    In in;
    in.r = rsrc(J.in, uint32_t(J.in_len));
    in.len = uint32_t(J.in_len);
    in.lp = 0;
    stage(lds, in);
    in.lp = HALF;
    stage(lds, in);
    in.lp = RING;
    in.rb = in.ub = in.vb = 0;
    in.W = 0;
    __builtin_amdgcn_wave_barrier();
    uint32_t rng = 0xFFFFFFFFu, code = 0;
    if (in.len >= 5) {
        refill(lds, in);
        for (int k = 0; k < 5; k++) {
            code = (code << 8) | uint32_t(in.W >> 56);
            in.W <<= 8;
        }
        in.ub = 40;
        refill(lds, in);
    } else {
        in.rb = in.len;
    }

    const __amdgpu_buffer_rsrc_t orsrc = rsrc(J.out, n);
    uint32_t obase = 0, fill = 0;             // output page covers [obase, obase + fill)
    uint32_t rec = 0, prev_len = 0, left = 0;
    uint32_t nrecs = 0, ndups = 0, nrevs = 0, nmiss = 0, nslow = 0;
    // the run's prefetch mode, from the miss rate of the last >= 256 symbols
    uint32_t pf_syms = 0, pf_miss = 0, pfon = 0;
    PROBE_DECL
    bool first_len = true;
    int status = 0;
    PS ps = load_ps(g, 0);
    uint32_t qctx = 0, delta = 0, prevq = 0, sel = 0, seq = 0, selterm = 0;
    uint32_t ctx = 0, maddr = L_CACHE;
    const uint8_t *sbase = nullptr;           // record's sequence (SEQ)
    uint32_t rlen = 0, sb0 = 0;               // record length, first staged base index
    uint32_t tpos = 0;                        // symbol index within the record
    const uint32_t dlane = L_DUMMY + 4 * l;

    auto flush = [&]() {
        for (uint32_t o = l * 4; o < fill; o += 256) {
            const uint32_t w = *reinterpret_cast<const uint32_t *>(lds + L_OBUF + o);
#pragma unroll
            for (uint32_t b = 0; b < 4; b++)
                if (o + b < fill) st8(orsrc, obase + o + b, w >> (8 * b));
        }
        obase += fill;
        fill = 0;
    };
    auto stage_seq = [&]() {   // bases of symbols [sb0, sb0 + SEQB) of the record
        for (uint32_t j = l; j < SEQB; j += 64) {
            const uint32_t pos = ps.boff + sb0 + j;
            lds[L_SEQ + j] = uint8_t(sbase && pos < rlen ? base2(sbase[pos]) : 0u);
        }
        __builtin_amdgcn_wave_barrier();
    };
    const uint8_t *ptab = nullptr;            // this record's tables (LDS)
    const uint16_t *pt16 = nullptr;
    auto seq_next = [&]() -> uint32_t {       // context bits of the sequence, next symbol
        if (!SEQ) return 0u;
        const uint32_t b = U(lds[L_SEQ + (tpos - sb0)]);
        return ((seq << 2) | b) & ((1u << ps.bbits) - 1u);
    };
    // the context after symbol `sym`, uniform (slow paths)
    auto next_uniform = [&](uint32_t sym) {
        const uint32_t seqn = seq_next();
        uint32_t u = U(pt16[(P_PTAB >> 1) + (left < 1023u ? left : 1023u)]);
        u += U(pt16[(P_DTAB >> 1) + (delta < 255u ? delta : 255u)]);
        u += selterm + (seqn << ps.bloc);
        qctx = (qctx << ps.qshift) + U(pt16[(P_QTAB >> 1) + sym]);
        ctx = (((qctx & ps.qmask) << ps.qloc) + u) & uint32_t(FQZ_CTX - 1);
        maddr = set_addr(ctx, NS8, ME);
        seq = seqn;
        delta += prevq != sym;
        prevq = sym;
        left--;
        tpos++;
    };

    // the fast path's model registers: lane j holds slot j of the cached
    // model, e in v0 and w in s0.  NE = 1: lanes past the sentinel read (and
    // write back) the sentinel's own slot, so every lane is the guard, a list
    // slot or a copy of the sentinel (cum = total) and the decoder's ballot
    // needs no lane mask.  NE = 2: the 64 lanes are the guard and slots
    // 0 .. 62; the sentinel is read apart (a code past slot 62's range takes
    // the slow path).
    uint32_t v0 = 0, s0 = 0;
    const uint32_t voff0 = 8u * (l < S ? l : S);
    auto issue_model = [&]() {
        const uint2 ew = *reinterpret_cast<const uint2 *>(lds + maddr + voff0);
        v0 = ew.x;
        s0 = ew.y;
    };
    auto write_model = [&](uint32_t a) { *reinterpret_cast<uint2 *>(lds + a + voff0) = make_uint2(v0, s0); };
    // the sentinel: context | total << 16
    auto model_sentinel = [&]() { return U(*reinterpret_cast<const uint32_t *>(lds + maddr + sent)); };
    // miss: write the resident model (context `tag`) back to HBM, fetch or
    // create ctx's
    auto miss = [&](uint32_t tag) {
        nmiss++;
#ifdef FQZ5_DEC_PROBE
        const uint64_t tm = __builtin_amdgcn_s_memtime();
#endif
        uint32_t *m32 = reinterpret_cast<uint32_t *>(lds + maddr);
        uint32_t *bits = reinterpret_cast<uint32_t *>(lds + L_BITS);
        uint32_t *dst = reinterpret_cast<uint32_t *>(J.back + size_t(tag) * ME);
        for (uint32_t o = l; o < ME / 4; o += 64)
            __hip_atomic_store(dst + o, m32[o], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
        if (l == 0) bits[tag >> 5] |= 1u << (tag & 31);
        __builtin_amdgcn_wave_barrier();
        if ((U(bits[ctx >> 5]) >> (ctx & 31)) & 1u) {
            const uint32_t *src = reinterpret_cast<const uint32_t *>(J.back + size_t(ctx) * ME);
            for (uint32_t o = l; o < ME / 4; o += 64)
                m32[o] = __hip_atomic_load(src + o, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
        } else {
            fresh_slots(maddr);
            if (l == 0) *reinterpret_cast<uint2 *>(lds + maddr + sent) = make_uint2(ctx | (L << 16), 0u);
        }
        __builtin_amdgcn_wave_barrier();
#ifdef FQZ5_DEC_PROBE
        (void)U(m32[0]);
        pr[3] += __builtin_amdgcn_s_memtime() - tm;   // cycles in miss()
#endif
    };
    auto load_model = [&]() {
        for (;;) {
            const uint32_t tag = model_sentinel() & 0xffffu;
            if (tag == ctx) break;
            miss(tag);
        }
        issue_model();
    };

    // ---- the slow path: the whole model in registers, lane dw of register
    // r (dw = l + 64 r) holding slot dw, the sentinel and its copies past L.
    // NE = 2: the slots past lane 63 as freq | sym << 16 per context in
    // J.back_hi (fresh until J.hi_bits marks them written).
    uint32_t fv[NE], fs[NE];
    auto rlane = [&](const uint32_t (&x)[NE], uint32_t dw) -> uint32_t {
        if (NE == 1) return RL(x[0], dw);
        const uint32_t a = RL(x[0], dw & 63u), b = RL(x[NE - 1], dw & 63u);
        return dw < 64 ? a : b;
    };
    auto full_model = [&]() {
        load_model();
        fv[0] = v0;
        fs[0] = s0;
        if constexpr (NE == 2) {
            const uint32_t sv = model_sentinel(), dw = 64u + l;
            const bool hi = (__hip_atomic_load(J.hi_bits + (ctx >> 5), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT) >>
                             (ctx & 31)) & 1u;
            uint32_t f = 0, sy = 0;
            if (dw <= L) {
                if (hi) {
                    const uint32_t x = __hip_atomic_load(J.back_hi + size_t(ctx) * 64u + l, __ATOMIC_RELAXED,
                                                         __HIP_MEMORY_SCOPE_WAVEFRONT);
                    f = x & 0xffffu;
                    sy = x >> 16;
                } else {
                    f = 1;
                    sy = dw - 1u;
                }
            }
            uint32_t inc = f;
#pragma unroll
            for (int d = 1; d < 64; d <<= 1) {
                const uint32_t o = __shfl_up(inc, d, 64);
                if (int(l) >= d) inc += o;
            }
            const uint32_t e63 = RL(v0, 63), cb = (e63 >> 16) + (e63 & 0xffffu);
            fv[1] = dw <= L ? f | ((cb + inc - f) << 16) : sv;
            fs[1] = dw <= L ? uint32_t(qt0[sy]) | (sy << 24) : 0u;
        }
    };
    auto write_full = [&]() {
        v0 = fv[0];
        s0 = fs[0];
        write_model(maddr);
        if constexpr (NE == 2) {
            const uint32_t sv = rlane(fv, L + 1), dw = 64u + l;
            if (l == 0) *reinterpret_cast<uint2 *>(lds + maddr + sent) = make_uint2(sv, 0u);
            if (dw <= L)
                __hip_atomic_store(J.back_hi + size_t(ctx) * 64u + l, (fv[1] & 0xffffu) | ((fs[1] >> 24) << 16),
                                   __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
            if (l == 0) {
                uint32_t *hb = J.hi_bits + (ctx >> 5);
                __hip_atomic_store(hb, __hip_atomic_load(hb, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT) |
                                       (1u << (ctx & 31)), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
            }
        }
        __builtin_amdgcn_wave_barrier();
    };
    // halve every live slot (c_simple_model.h:106-115): prefix sums of the
    // halved frequencies give the new cumulative counts
    auto halve = [&]() {
        uint32_t carry = 0;
#pragma unroll
        for (int r = 0; r < NE; r++) {
            const uint32_t dw = l + 64 * r;
            uint32_t f = dw >= 1 && dw <= L ? (fv[r] & 0xffffu) : 0u;
            f -= f >> 1;
            uint32_t inc = f;
#pragma unroll
            for (int d = 1; d < 64; d <<= 1) {
                const uint32_t o = __shfl_up(inc, d, 64);
                if (int(l) >= d) inc += o;
            }
            // (the sentinel and its copies keep their context in the low half)
            if (dw >= 1) fv[r] = (dw <= L ? f : (fv[r] & 0xffffu)) | ((carry + inc - f) << 16);
            carry += RL(inc, 63);
        }
    };
    // one bubble step at lane kl >= 2
    auto bubble = [&](uint32_t kl) {
        const uint32_t ek = rlane(fv, kl), ep = rlane(fv, kl - 1);
        const uint32_t fk = ek & 0xffffu, fp = ep & 0xffffu;
        if (fk > fp) {
            const uint32_t cp = ep >> 16;
            const uint32_t sk = rlane(fs, kl), sp = rlane(fs, kl - 1);
#pragma unroll
            for (int r = 0; r < NE; r++) {
                const uint32_t dw = l + 64 * r;
                if (dw == kl - 1) { fv[r] = fk | (cp << 16); fs[r] = sk; }
                if (dw == kl) { fv[r] = fp | ((cp + fk) << 16); fs[r] = sp; }
            }
        }
    };
    // the list update after coding the slot in lane kl (fl_bump): +16,
    // halve past FL_MAX, one bubble step
    auto update = [&](uint32_t kl, uint32_t total) {
#pragma unroll
        for (int r = 0; r < NE; r++) {
            const uint32_t dw = l + 64 * r;
            fv[r] += dw > kl ? 0x100000u : (dw == kl ? FL_STEP : 0u);
        }
        if (total + FL_STEP > FL_MAX) halve();
        if (kl >= 2) bubble(kl);
    };
    // one symbol with the reference's arithmetic, any state (corrupt or
    // truncated streams, the last bytes of the input, NE = 2 slots past 62)
    auto slow_symbol = [&]() {
        nslow++;
        full_model();
        const uint32_t total = rlane(fv, L + 1) >> 16;
        uint32_t t = 0;
        if (total && rng >= total) {   // the division stays even when no symbol follows
            rng /= total;
            t = code / rng;
        }
        uint32_t sym = 0;
        if (t < total) {   // (t > FL_MAX implies t >= total)
            uint32_t kl = 1;
            while (kl < L && (rlane(fv, kl + 1) >> 16) <= t) kl++;
            const uint32_t ek = rlane(fv, kl);
            code -= (ek >> 16) * rng;
            rng *= ek & 0xffffu;
            renorm_slow(lds, in, rng, code);
            sym = rlane(fs, kl) >> 24;
            update(kl, total);
            write_full();
        }
        lds[l ? dlane : L_OBUF + fill] = uint8_t(sym);
        fill++;
        next_uniform(sym);
    };

    // hedged copies: every 64 loop turns (~4 K symbols) lane 0 reads *done
    // by an atomic (at L2, coherent), and the copy leaves once another has
    // finished the block
    uint32_t turns = 0;
    bool lost = false;
    for (;;) {
        if (J.done && (++turns & 63u) == 0u) {
            uint32_t d = 0;
            if (l == 0) d = __hip_atomic_fetch_add(J.done, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (RL(d, 0)) { lost = true; break; }
        }
        if (left == 0) {
            // ---- record header (fqzcomp_qual.c:1484-1540) --------------------
            if (obase + fill >= n) break;
            if (fill == OBUF) flush();
            const uint32_t i = obase + fill;
            sel = (ps.sel || (gfl & 1u)) ? small_decode(&sm.sel, lds, in, rng, code) : 0u;
            const uint32_t x = (gfl & 2u) ? U(g.stab[sel < 255u ? sel : 255u]) : sel;
            if (x >= nparam) { status = -1; break; }
            ps = load_ps(g, x);
            uint32_t len = prev_len;
            if (!ps.fixed || first_len) {
                len = 0;
                for (int b = 0; b < 4; b++) len |= small_decode(&sm.len[b], lds, in, rng, code) << (8 * b);
                first_len = false;
                prev_len = len;
            }
            if (len > n - i || len == 0) { status = -1; break; }
            if (rec < J.nlengths && l == 0) J.lengths[rec] = len;
            if (gfl & 4u) {
                if (small_decode(&sm.rev, lds, in, rng, code)) {
                    if (nrevs >= J.cap_list) { status = -2; break; }
                    if (l == 0) J.revs[nrevs] = make_uint2(i, len);
                    nrevs++;
                }
            }
            rec++;
            if (ps.dedup && small_decode(&sm.dup, lds, in, rng, code)) {
                if (len > i) { status = -1; break; }
                if (ndups >= J.cap_list) { status = -2; break; }
                if (l == 0) J.dups[ndups] = make_uint2(i, len);
                ndups++;
                flush();
                obase += len;
                continue;
            }
            if (nparam > 1) {
                if (nrecs >= J.cap_list) { status = -2; break; }
                if (l == 0) J.recs[nrecs] = make_uint4(i, len, x, 0u);
                nrecs++;
            }
            left = len;
            rlen = len;
            tpos = 0;
            delta = prevq = qctx = 0;
            seq = 0;
            selterm = sel << ps.sloc;
            ptab = lds + L_PAR + ps.x * PBYTES;
            pt16 = reinterpret_cast<const uint16_t *>(ptab);
            if (SEQ) {
                sbase = nullptr;
                if (J.seq && rec - 1 < J.nseq && J.seq_off[rec - 1] != ~0ull) {
                    sbase = J.seq + J.seq_off[rec - 1];
                    for (uint32_t b = 0; b < ps.boff; b++) seq = (seq << 2) | base2(uint8_t(U(sbase[b])));
                }
                sb0 = 0;
                stage_seq();
            }
            ctx = ps.ctx0;
            maddr = set_addr(ctx, NS8, ME);
        }
        if (in.avail() < 4u) {   // the last bytes of the input: reference arithmetic
            slow_symbol();
            if (fill == OBUF) flush();
            if (SEQ && tpos - sb0 == SEQB) { sb0 = tpos; stage_seq(); }
            continue;
        }
        // ---- fast run: up to 64 symbols of this record within the output
        // page (and the staged bases); the model of the current context
        // stays in registers while the context repeats --------------------
        uint32_t lim = left < OBUF - fill ? left : OBUF - fill;
        if (lim > 64u) lim = 64u;
        if (SEQ && lim > SEQB - (tpos - sb0)) lim = SEQB - (tpos - sb0);
        uint32_t ulim = (in.vb - 4u) * 8u;
        // per-step uniform context terms of the run (fqz_update_ctx uses the
        // position and delta before this symbol's update): lane i the
        // position term of step i, lane j the delta term of delta0 + j
        const uint32_t delta0 = U(delta);
        const uint32_t pvv = uint32_t(pt16[(P_PTAB >> 1) + (left - l < 1023u ? left - l : 1023u)]) + selterm;
        const uint32_t dvv = pt16[(P_DTAB >> 1) + (delta + l < 255u ? delta + l : 255u)];
        const uint32_t sqv = SEQ ? uint32_t(lds[L_SEQ + ((tpos - sb0 + l) & (SEQB - 1))]) : 0u;
        uint32_t qs = qctx << ps.qshift;
        const uint32_t qmask = U(ps.qmask), qshift = U(ps.qshift);
        uint32_t vout = 0;
        uint32_t done = 0;
        bool to_slow = false;
        PROBE_START
        load_model();
        {
            // the run's scalar state, as uniform values (the asm keeps it in
            // SGPRs: A the current copy, B the other)
            uint64_t cw = uint64_t(U(code)) << 32;   // {scratch, code}
            uint64_t win = (uint64_t(U(uint32_t(in.W >> 32))) << 32) | U(uint32_t(in.W));
            uint64_t mA = (uint64_t(s0) << 32) | v0, mB = 0;
            uint32_t tvA = model_sentinel(), tvB = 0;
            uint32_t cA = U(ctx), qsA = U(qs), pvA = U(prevq), maA = U(maddr), sqA = U(seq);
            uint32_t cB, qsB, pvB, maB, sqB;
            uint32_t dd = 0, nm = 0, tvp;
            uint64_t scr, pf;
            // the miss path: the backing store, fresh slots (guard, list; the
            // sentinel lanes are set from the context)
            const uint64_t back = reinterpret_cast<uint64_t>(J.back);
            const uint32_t lsh = U(L << 16), sidx = U(S);
            const uint32_t fe = l == 0 ? 0xffffu : (l <= LL ? 1u | ((l - 1u) << 16) : 0u);
            const uint32_t fw = l == 0 || l > LL ? 0u : uint32_t(qt0[l - 1u]) | ((l - 1u) << 24);
            rng = U(rng);
            in.rb = U(in.rb);
            const uint32_t bswp = 0x00010203u;   // v_perm byte reversal
            // the window refills in the run while the ring holds rb + 8 .. rb + 11
            auto rb_end = [&]() {
                const uint32_t e = in.len < in.lp ? in.len : in.lp;
                return U(e >= 12u ? e - 11u : 0u);
            };
            uint32_t rbend = rb_end();
            in.ub = U(in.ub);
            lim = U(lim);
            ulim = U(ulim);
            uint32_t flags = 0;
            const uint32_t base = L_CACHE, vme = ME, cbig = 0x100000u, c65503 = 65503u;
            const uint32_t ns8 = U(NS8), qlocv = ps.qloc, bmask = U((1u << ps.bbits) - 1u), bloc = U(ps.bloc);
            const uint32_t qtab = U(L_PAR + ps.x * PBYTES + P_QTAB);   // LDS address (the dynamic base is 0)
            const uint32_t vsent = sent;
            const double c19 = 0x1p-19;
            uint32_t u, x, k1, kl, pk, pk1, qsk, z, m0s;
            uint64_t G, E, SW, SM, TG, HV;
            uint32_t t0, t1, t2, t3, t4, t5, t6;
            double d0, d1, d2;
            for (;;) {
#define FQZ_RUN_OPERANDS                                                                      \
                : [mA] "+{v[2:3]}"(mA), [mB] "+{v[4:5]}"(mB), [cw] "+{s[40:41]}"(cw),          \
                  [win] "+{s[42:43]}"(win), [scr] "=&{s[44:45]}"(scr), [rb] "+s"(in.rb),        \
                  [nm] "+s"(nm), [pf] "=&{v[6:7]}"(pf), [tvp] "=&v"(tvp),                       \
                  [vout] "+v"(vout), [tvA] "+v"(tvA), [tvB] "=&v"(tvB),                           \
                  [rng] "+s"(rng), [ub] "+s"(in.ub), [dd] "+s"(dd), [done] "+s"(done),        \
                  [cA] "+s"(cA), [qsA] "+s"(qsA), [pvA] "+s"(pvA), [maA] "+s"(maA), [sqA] "+s"(sqA), \
                  [cB] "=&s"(cB), [qsB] "=&s"(qsB), [pvB] "=&s"(pvB), [maB] "=&s"(maB), [sqB] "=&s"(sqB), \
                  [flags] "=&s"(flags), [u] "=&s"(u), [x] "=&s"(x), [k1] "=&s"(k1), [kl] "=&s"(kl), \
                  [pk] "=&s"(pk), [pk1] "=&s"(pk1), [qsk] "=&s"(qsk), [z] "=&s"(z), [m0s] "=&s"(m0s), \
                  [G] "=&s"(G), [E] "=&s"(E), [SW] "=&s"(SW), [SM] "=&s"(SM), [TG] "=&s"(TG),  \
                  [HV] "=&s"(HV),                                                              \
                  [t0] "=&v"(t0), [t1] "=&v"(t1), [t2] "=&v"(t2), [t3] "=&v"(t3),             \
                  [t4] "=&v"(t4), [t5] "=&v"(t5), [t6] "=&v"(t6),                              \
                  [d0] "=&v"(d0), [d1] "=&v"(d1), [d2] "=&v"(d2)                               \
                : [lim] "s"(lim), [ulim] "s"(ulim), [qmask] "s"(qmask), [qshift] "s"(qshift), \
                  [ns8] "s"(ns8), [base] "s"(base), [qtab] "s"(qtab), [bmask] "s"(bmask),     \
                  [bloc] "s"(bloc), [c65503] "s"(c65503), [rbend] "s"(rbend), [bswp] "s"(bswp), \
                  [lring] "i"(L_RING), [lbits] "i"(L_BITS), [back] "s"(back), [lsh] "s"(lsh),   \
                  [fe] "v"(fe), [fw] "v"(fw), [sidx] "s"(sidx),                                 \
                  [voff] "v"(voff0), [vsent] "v"(vsent), [qlocv] "v"(qlocv),                   \
                  [cbig] "v"(cbig), [c19] "v"(c19), [vme] "v"(vme), [pvv] "v"(pvv),          \
                  [dvv] "v"(dvv), [sqv] "v"(sqv)                                              \
                : "memory", "scc", "vcc"
#ifdef FQZ5_DEC_PROBE
                const uint32_t done_in = done;
                const uint64_t ta = __builtin_amdgcn_s_memtime();
                if (pr_x) {
                    pr[4] += ta - pr_x;   // cycles between runs
                    pr[5] += 1;
                }
#endif
#define FQZ_RUN_NE(SENTWB, SENTEX, WCNT, MST, PF, PFT, MMOV, MWB, MVW)                                                                           \
                if constexpr (QW && SEQ)                                                                     \
                    asm volatile(FQZ_RUN_ASM(FQZ_QT1_W, FQZ_QT2_W, FQZ_SEQ_CTX, FQZ_SEQ_SAME, SENTWB, SENTEX, WCNT, MST, PF, PFT, MMOV, MWB, MVW) FQZ_RUN_OPERANDS); \
                else if constexpr (QW)                                                                       \
                    asm volatile(FQZ_RUN_ASM(FQZ_QT1_W, FQZ_QT2_W, FQZ_SEQ_NONE, FQZ_SEQ_NONE, SENTWB, SENTEX, WCNT, MST, PF, PFT, MMOV, MWB, MVW) FQZ_RUN_OPERANDS); \
                else if constexpr (SEQ)                                                                      \
                    asm volatile(FQZ_RUN_ASM(FQZ_QT1_TAB, FQZ_QT2_TAB, FQZ_SEQ_CTX, FQZ_SEQ_SAME, SENTWB, SENTEX, WCNT, MST, PF, PFT, MMOV, MWB, MVW) FQZ_RUN_OPERANDS); \
                else                                                                                         \
                    asm volatile(FQZ_RUN_ASM(FQZ_QT1_TAB, FQZ_QT2_TAB, FQZ_SEQ_NONE, FQZ_SEQ_NONE, SENTWB, SENTEX, WCNT, MST, PF, PFT, MMOV, MWB, MVW) FQZ_RUN_OPERANDS);
                const uint32_t nm_in = nm, done_at = done;
                if constexpr (NE == 1) {
                    if (pfon) { FQZ_RUN_NE(FQZ_SENT_NONE, FQZ_SENT_NONE, "1", FQZ_MSENT_NONE, 1, FQZ_PF_NONE, FQZ_MSENT_LANE, FQZ_MSENT_NONE1, "1") }
                    else { FQZ_RUN_NE(FQZ_SENT_NONE, FQZ_SENT_NONE, "1", FQZ_MSENT_NONE, 0, FQZ_PF_NONE, FQZ_MSENT_LANE, FQZ_MSENT_NONE1, "1") }
                } else {
                    if (pfon) { FQZ_RUN_NE(FQZ_SENT_WB, FQZ_SENT_EXIT, "2", FQZ_MSENT_ST, 1, FQZ_PF_SENT, FQZ_MSENT_MOV, FQZ_MSENT_WR, "2") }
                    else { FQZ_RUN_NE(FQZ_SENT_WB, FQZ_SENT_EXIT, "2", FQZ_MSENT_ST, 0, FQZ_PF_SENT, FQZ_MSENT_MOV, FQZ_MSENT_WR, "2") }
                }
#undef FQZ_RUN_NE
#undef FQZ_RUN_OPERANDS
#ifdef FQZ5_DEC_PROBE
                pr_x = __builtin_amdgcn_s_memtime();
                pr[0] += pr_x - ta;                           // cycles inside the run asm
                pr[1] += U(done) - done_in;                   // symbols it decoded
                pr[2] += 1;                                   // calls
#endif
                // (the compiler takes every output of an asm with VGPR outputs
                // for divergent: the scalar ones are re-read as uniform)
                rng = U(rng);
                in.ub = U(in.ub);
                in.rb = U(in.rb);
                dd = U(dd);
                done = U(done);
                nm = U(nm);
                pf_syms += done - done_at;
                pf_miss += nm - nm_in;
                if (pf_syms >= 256u) {   // prefetch when more than one symbol in 8 misses
                    pfon = U(pf_miss * 8u > pf_syms ? 1u : 0u);
                    pf_syms = 0;
                    pf_miss = 0;
                }
                cA = U(cA);
                qsA = U(qsA);
                pvA = U(pvA);
                maA = U(maA);
                sqA = U(sqA);
                flags = U(flags);
                cw = (uint64_t(U(uint32_t(cw >> 32))) << 32);
                win = (uint64_t(U(uint32_t(win >> 32))) << 32) | U(uint32_t(win));
                if (flags == 2) {   // a context not in its set (the next run fetches it) or the slow path
                    to_slow = (U(*reinterpret_cast<const uint32_t *>(lds + maA + sent)) & 0xffffu) == cA;
                    break;
                }
                if (done == lim) break;
                in.W = win;   // the input window needs a refill
                refill(lds, in);
                win = in.W;
                if (in.vb < 4u) break;
                ulim = (in.vb - 4u) * 8u;
                rbend = rb_end();
            }
            in.W = win;
            code = uint32_t(cw >> 32);
            ctx = cA;
            qs = qsA;
            prevq = pvA;
            maddr = maA;
            seq = sqA;
            delta = delta0 + dd;
            nmiss += nm;
            left -= done;
            if (SEQ) tpos += done;
        }
        qctx = qs >> qshift;
        if (l < done) lds[L_OBUF + fill + l] = uint8_t(vout);
        fill += done;
        if (to_slow) slow_symbol();
        if (fill == OBUF) flush();
        if (SEQ && left && tpos - sb0 == SEQB) { sb0 = tpos; stage_seq(); }
    }
    if (lost) return;   // another copy decodes (decoded) this block
    if (status == 0) flush();
    if (J.done && l == 0) __hip_atomic_store(J.done, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (l == 0) {
        *J.status = status;
        *J.nrec_out = rec;
        J.counts[0] = nrecs;
        J.counts[1] = ndups;
        J.counts[2] = nrevs;
        J.counts[3] = nmiss;
        J.counts[4] = nslow;
    }
    PROBE_OUT
}

// ---------------------------------------------------------------------------
// fix-ups, in the reference's order: symbols -> qmap (during decode in the
// reference), duplicate copies (during decode), reversal (after decode,
// fqzcomp_qual.c:1597-1611)
// ---------------------------------------------------------------------------
__global__ void k_fqz_map_all(FqzDecJob J) {
    const uint8_t *qm = J.g->p[0].qmap;
    for (uint64_t i = blockIdx.x * uint64_t(blockDim.x) + threadIdx.x; i < J.n;
         i += uint64_t(gridDim.x) * blockDim.x)
        J.out[i] = qm[J.out[i]];
}

__global__ void k_fqz_map_recs(FqzDecJob J) {
    const uint32_t nr = J.counts[0];
    for (uint32_t r = blockIdx.x; r < nr; r += gridDim.x) {
        const uint4 R = J.recs[r];
        const uint8_t *qm = J.g->p[R.z].qmap;
        for (uint32_t t = threadIdx.x; t < R.y; t += blockDim.x) J.out[R.x + t] = qm[J.out[R.x + t]];
    }
}

// duplicates copy the `len` bytes before them, in record order
__global__ __launch_bounds__(256) void k_fqz_dups(FqzDecJob J) {
    const uint32_t nd = J.counts[1];
    for (uint32_t d = 0; d < nd; d++) {
        const uint2 D = J.dups[d];
        for (uint32_t t = threadIdx.x; t < D.y; t += blockDim.x)
            J.out[D.x + t] = __hip_atomic_load(J.out + D.x - D.y + t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __threadfence();
        __syncthreads();
    }
}

__global__ void k_fqz_revs(FqzDecJob J) {
    const uint32_t nr = J.counts[2];
    for (uint32_t r = blockIdx.x; r < nr; r += gridDim.x) {
        const uint2 R = J.revs[r];
        uint8_t *o = J.out + R.x;
        for (uint32_t a = threadIdx.x; a < R.y / 2; a += blockDim.x) {
            const uint32_t b = R.y - 1 - a;
            const uint8_t t = o[a];
            o[a] = o[b];
            o[b] = t;
        }
    }
}

// q = (u32)fma(n, recip(t), 2^-19) against n / t for every total t and a
// spread of numerators (including multiples of t and their neighbours)
__global__ void k_fqz_div_selftest(uint32_t *bad) {
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x + 1;
    if (t > 65535u) return;
    const double rd = recip(t);
    uint32_t nb = 0;
    uint32_t x = t * 2654435761u;
    for (int i = 0; i < 512; i++) {
        x = x * 1664525u + 1013904223u;
        const uint32_t m = x / t;
        const uint32_t cands[4] = {x, m * t, m * t - 1u, m * t + t - 1u};
        for (int c = 0; c < 4; c++) nb += quot(cands[c], rd) != cands[c] / t;
    }
    nb += quot(0xFFFFFFFFu, rd) != 0xFFFFFFFFu / t;
    if (nb) atomicAdd(bad, nb);
}

}  // namespace

template <int NE, bool SEQ, bool QW>
static hipError_t launch_dec(const FqzDecJob *j, int n, hipStream_t s) {
    auto *f = k_fqz_dec<NE, SEQ, QW>;
    hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void *>(f),
                                       hipFuncAttributeMaxDynamicSharedMemorySize, LDS_BYTES);
    if (e != hipSuccess) return e;
    if (n) hipLaunchKernelGGL(f, dim3(n), dim3(64), LDS_BYTES, s, j);
    return hipGetLastError();
}

hipError_t launch_fqz_dec(const FqzDecJob *j, int n, int ne, bool seq, bool qid, hipStream_t s) {
    if (ne == 1) {
        if (seq) return qid ? launch_dec<1, true, true>(j, n, s) : launch_dec<1, true, false>(j, n, s);
        return qid ? launch_dec<1, false, true>(j, n, s) : launch_dec<1, false, false>(j, n, s);
    }
    if (seq) return qid ? launch_dec<2, true, true>(j, n, s) : launch_dec<2, true, false>(j, n, s);
    return qid ? launch_dec<2, false, true>(j, n, s) : launch_dec<2, false, false>(j, n, s);
}

hipError_t launch_fqz_dec_fix(const FqzDecJob &j, int map_mode, bool dups, bool revs, hipStream_t s) {
    if (map_mode == 1) hipLaunchKernelGGL(k_fqz_map_all, dim3(1024), dim3(256), 0, s, j);
    if (map_mode == 2) hipLaunchKernelGGL(k_fqz_map_recs, dim3(4096), dim3(64), 0, s, j);
    if (dups) hipLaunchKernelGGL(k_fqz_dups, dim3(1), dim3(256), 0, s, j);
    if (revs) hipLaunchKernelGGL(k_fqz_revs, dim3(4096), dim3(64), 0, s, j);
    return hipGetLastError();
}

hipError_t fqz_div_selftest(uint32_t *d_bad, hipStream_t s) {
    hipLaunchKernelGGL(k_fqz_div_selftest, dim3(256), dim3(256), 0, s, d_bad);
    return hipGetLastError();
}

}  // namespace fqz5
