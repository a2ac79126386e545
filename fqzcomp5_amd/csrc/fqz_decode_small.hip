// fqz_decode_small.hip — fqzcomp_qual decoder (uncompress_block_fqz2f,
// fqzcomp_qual.c:1410-1634) for small alphabets: at most 9 live symbols per
// quality model (Illumina 8-level and NovaSeq 4-level data, whose qmap makes
// max_sym = nsym, fqzcomp_qual.c:842,891-898), one qtab that is the
// identity on the live symbols, no sequence bases in the context.
//
// Why a second decoder.  The general decoder (fqz_decode.hip) keeps a model
// as 8 bytes per list slot, so an LDS cache of ~125 KB holds ~1 500 models
// of 9 symbols.  FQZ1 (fqzcomp_qual.c:207, position in the context) on
// Illumina data cycles through ~6 100 contexts; half of its symbols missed
// and each miss went to HBM.  Here a model is 24 bytes:
//
//    bytes  0..15  U[1..8]  u16: cumulative frequency through list slot j
//                           (U_j = total for j >= live)
//    bytes 16..17  tag      u16: the context the model belongs to
//    bytes 18..19  total    u16
//    bytes 20..23  S        u32: nibble i = symbol of list slot i + 1 (slots
//                           1..8; with 9 live symbols slot 9's symbol is the
//                           one missing from the eight)
//
// so ~6 280 models fit one LDS cache, and the backing store (65 536 x 24 B =
// 1.5 MB, pre-filled with fresh models so a miss never asks whether a
// context was seen) stays in the XCD's L2.
//
// The cache is 4-way set associative (1 570 sets of 96 bytes): the run's
// 64 lanes are 4 rows of 16, row w reads way w of the set, the tag test is
// one v_cmp per lane and the decode ballot is masked to the hit row.  A miss
// replaces a round-robin victim way.  Measured on the FQZ1 Illumina contexts
// (tools/fqz_stats.c dump, ~6 270 contexts in a cycle): direct-mapped 8.4 %
// misses, 4-way LRU 0.43 %, 4-way round robin 0.68 % (GPU counters: 0.7 %).
//
// (Measured and not kept: reading the set of the context that slot 1 leads
// to a symbol early, slot 1 being decoded for ~87 % of the symbols, into a
// second register set with a twin loop body: 177 -> 213 ns per symbol; the
// set addresses on the scalar unit instead of three VALU hashes: 226.)
//
// The decode of a symbol (lane i holds U_{i+1}, the model of the current
// context in registers):
//   q      = floor(range / total) (RN(1/total) by rcp + one Newton step)
//   p_i    = U_{i+1} * q;  k = first lane with p_i > code  (the reference's
//            linear scan of c_simple_model.h:140-171 as one ballot)
//   code  -= p_{k-1};  range = p_k - p_{k-1}
//   update = +16 to U_j for j >= k (fl_bump's freq and total); a bubble
//            step, a halving, the 9th slot or a bad code go to the slow path
//   every lane meanwhile computes the context its own symbol would lead to
//   (fqz_update_ctx, fqzcomp_qual.c:361-418) and that context's cache set,
//   so the next model read waits for one readlane.
#include <hip/hip_runtime.h>
#include <cstdint>

#include "fqz_kernels.h"
#include "fqz_model.hpp"
#include "fqz_dec_common.hpp"

namespace fqz5 {
namespace {

using namespace dec;

constexpr uint32_t S_SMALL = 0;                          // SmallModels
constexpr uint32_t S_RING = 4096;                        // RING + 16 (mirror)
constexpr uint32_t S_OBUF = S_RING + RING + 16;          // output page
constexpr uint32_t SOBUF = 2048;
constexpr uint32_t S_DUMMY = S_OBUF + SOBUF;             // lanes != 0 write here
constexpr uint32_t S_PAR = S_DUMMY + 256;                // per parameter block: ptab u16[1024], dtab u16[256]
constexpr uint32_t SPB = 2560, S_DTAB = 2048;
constexpr uint32_t LDS_BYTES = 163840;
static_assert(S_PAR == FQZ_SMALL_LDS_FIXED, "keep fqz_kernels.h in step");
static_assert(SPB == FQZ_SMALL_PARAM_BYTES, "keep fqz_kernels.h in step");
static_assert(sizeof(SmallModels) <= S_RING, "small models");
constexpr uint32_t ME = FQZ_SMALL_MODEL_BYTES;           // 24
constexpr uint32_t WAYS = FQZ_SMALL_WAYS, SETB = WAYS * ME;   // a set: 4 models
static_assert(WAYS == 4 && SETB == 96, "the run's lane rows are the ways");

DEV void stage_s(uint8_t *lds, const In &in) { stage<S_RING>(lds, in); }
DEV void refill_s(uint8_t *lds, In &in) { refill<S_RING>(lds, in); }

// the cache set of a context (the asm computes the same with 24-bit
// multiplies: v_mul_u32_u24, v_mul_hi_u32_u24, v_mad_u32_u24)
DEV uint32_t sset(uint32_t ctx, uint32_t ns8, uint32_t cb) {
    const uint32_t h = ctx * 0x9E3779u;
    const uint32_t set = uint32_t((uint64_t(h & 0xffffffu) * (ns8 & 0xffffffu)) >> 32);
    return cb + set * SETB;
}

// the fresh model's words (every live symbol frequency 1, in symbol order)
DEV uint32_t fresh_word(uint32_t w, uint32_t L, uint32_t ctx) {
    auto u = [&](uint32_t j) { return j < L ? j : L; };
    if (w < 4) return u(2 * w + 1) | (u(2 * w + 2) << 16);
    if (w == 4) return (ctx & 0xffffu) | (L << 16);
    return 0x76543210u;
}

// ---------------------------------------------------------------------------
// The fast run: up to `lim` symbols of one record, one symbol per loop turn.
// Operands: code is s41 (s40 its scratch), the window s[42:43], the model's
// broadcast words v2 (tag | total << 16) and v3 (S); vU lane i = U_{i+1}
// (lanes 8.. the total), vaddr its per-lane LDS address (set + voff), vb the
// set address in every lane.  Labels: 10/11 the top (11 past the wait),
// 12 the slow exit, 20 the same-context tail, 40/41 renormalisation out of
// line (back at 30/31), 60 a miss, 90 the exit.
// The bubble test (tools/probe/dpp_probe.hip measured it on gfx950): with
// row_shr:1, v_sub_u32_dpp d, x, x gives x[i-1] - x[i]; bound_ctrl:0 reads
// 0 for lane 0 of a row, without it lane 0 keeps d.  So t4 = U_i - U_{i+1}
// = -f(i) (f(i) the frequency of lane i's slot) and vsw = f(i) - f(i-1); a
// decode in lane k >= 1 bubbles when f(k) + 16 > f(k-1), i.e. vsw > -16;
// vsw's lane 0 stays INT_MIN (never).
// gfx950 wait states kept by the order: a DPP read of a VGPR two VALU
// instructions after its write; an SGPR written by the SALU and read as a
// VALU mask two instructions later; a VGPR written by the VALU and read by
// v_readlane / v_readfirstlane one instruction later; v_rcp_f64's result
// one instruction later.
// ---------------------------------------------------------------------------
#define FQS_DT_U                                                            \
    "v_readlane_b32 %[x], %[dvv], %[dd]\n"
#define FQS_DT_ADD "s_add_u32 %[u], %[u], %[x]\n"
#define FQS_DT_UPD                                                          \
    "s_cmp_lg_u32 %[pv], %[sym]\n"                                          \
    "s_addc_u32 %[dd], %[dd], 0\n"                                          \
    "s_mov_b32 %[pv], %[sym]\n"
#define FQS_NONE ""
#define FQS_RENORM_OUT(RNL, RETL)                                           \
    RNL ":\n"                                                               \
    "s_mov_b32 s40, s43\n"                                                  \
    "s_lshl_b64 s[40:41], s[40:41], %[z]\n"                                 \
    "s_lshl_b64 s[42:43], s[42:43], %[z]\n"                                 \
    "s_lshl_b32 %[rng], %[rng], %[z]\n"                                     \
    "s_add_u32 %[ub], %[ub], %[z]\n"                                        \
    "s_cmp_gt_u32 %[ub], %[ulim]\n"                                         \
    "s_cbranch_scc0 " RETL "b\n"                                            \
    "s_cmp_ge_u32 %[rb], %[rbend]\n"                                        \
    "s_cbranch_scc1 90f\n"                                                  \
    "s_add_u32 %[x], %[rb], 8\n"                                            \
    "s_and_b32 %[k1], %[x], 0xffc\n"                                        \
    "s_and_b32 %[x], %[x], 3\n"                                             \
    "s_add_u32 %[k1], %[k1], %[lring]\n"                                    \
    "v_mov_b32 %[t4], %[k1]\n"                                              \
    "ds_read_b32 %[t5], %[t4]\n"                                            \
    "ds_read_b32 %[t6], %[t4] offset:4\n"                                   \
    "s_lshl_b32 %[x], %[x], 3\n"                                            \
    "s_sub_u32 %[ub], %[ub], 32\n"                                          \
    "s_add_u32 %[rb], %[rb], 4\n"                                           \
    "s_waitcnt lgkmcnt(0)\n"                                                \
    "v_alignbit_b32 %[t5], %[t6], %[t5], %[x]\n"                            \
    "v_perm_b32 %[t5], %[t5], %[t5], %[bswp]\n"                             \
    "s_mov_b32 s45, 0\n"                                                    \
    "v_readfirstlane_b32 s44, %[t5]\n"                                      \
    "s_lshl_b64 s[44:45], s[44:45], %[ub]\n"                                \
    "s_or_b64 s[42:43], s[42:43], s[44:45]\n"                               \
    "s_branch " RETL "b\n"

// Probe build (-DFQZ5_SMALL_PROBE, tools/dec_small_probe.sh): s_memtime
// stamps at the symbol's top (A, past the model-read wait), after q
// (B: the rcp/Newton division, with the context terms interleaved), after
// the ballot's branch (C: p_i, the next set's hash, the ballot), after the
// model write-back (D: readlanes, coder, +16 update) and at the loop end (E:
// the next model read issued); E to the next A is the wait for that read.
// Each stamp is an SMEM read and the loop end waits for them, so the probe
// build runs slower than the plain one (both are reported).
#ifdef FQZ5_SMALL_PROBE
#define FQS_PA "s_memtime s[46:47]\n"
#define FQS_PB "s_memtime s[48:49]\n"
#define FQS_PC "s_memtime s[50:51]\n"
#define FQS_PD "s_memtime s[52:53]\n"
#define FQS_PE                                                              \
    "s_memtime s[54:55]\n"                                                  \
    "s_waitcnt lgkmcnt(0)\n"                                                \
    "s_sub_u32 %[x], s48, s46\n"                                            \
    "s_add_u32 %[pr1], %[pr1], %[x]\n"                                      \
    "s_sub_u32 %[x], s50, s48\n"                                            \
    "s_add_u32 %[pr2], %[pr2], %[x]\n"                                      \
    "s_sub_u32 %[x], s52, s50\n"                                            \
    "s_add_u32 %[pr3], %[pr3], %[x]\n"                                      \
    "s_sub_u32 %[x], s54, s52\n"                                            \
    "s_add_u32 %[pr4], %[pr4], %[x]\n"                                      \
    "s_sub_u32 %[x], s46, s56\n"                                            \
    "s_add_u32 %[pr5], %[pr5], %[x]\n"                                      \
    "s_mov_b64 s[56:57], s[54:55]\n"
#define FQS_P0 "s_memtime s[56:57]\n"
#else
#define FQS_PA ""
#define FQS_PB ""
#define FQS_PC ""
#define FQS_PD ""
#define FQS_PE ""
#define FQS_P0 ""
#endif

#define FQS_RUN_ASM(DTU, DTADD, DTUPD)                                      \
    "s_mov_b32 %[m0s], m0\n"                                                \
    "s_mov_b32 m0, %[done]\n"                                               \
    "s_mov_b32 %[flags], 0\n"                                               \
    "v_add_u32 %[vaddr], %[ma], %[voff]\n"                                  \
    "v_add_u32 %[vb], %[ma], %[vwoff]\n"                                    \
    "ds_read_u16 %[vU], %[vaddr]\n"                                         \
    "ds_read_b64 v[2:3], %[vb] offset:16\n"                                 \
    FQS_P0                                                                  \
    "10:\n"                                                                 \
    "s_waitcnt lgkmcnt(0)\n"                                                \
    "11:\n"                                                                 \
    FQS_PA                                                                  \
    "v_cmp_eq_u16_e32 vcc, %[c], v2\n"                                      \
    "v_sub_u32_dpp %[t4], %[vU], %[vU] row_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:0\n"\
    "v_readlane_b32 %[u], %[pvv], m0\n"                                     \
    "v_lshrrev_b32 %[t6], 16, v2\n"                                         \
    DTU                                                                     \
    "v_cvt_f64_u32 %[d0], %[rng]\n"                                         \
    "v_sub_u32_dpp %[vsw], %[t4], %[t4] row_shr:1 row_mask:0xf bank_mask:0xf\n"\
    "v_cvt_f64_u32 %[d1], %[t6]\n"                                          \
    DTADD                                                                   \
    "v_rcp_f64 %[d2], %[d1]\n"                                              \
    "s_cbranch_vccz 60f\n"                                                  \
    "v_bfe_u32 %[t0], v3, %[vsh4], 4\n"                                     \
    "v_fma_f64 %[d1], -%[d1], %[d2], 1.0\n"                                 \
    "v_cmp_lt_i32_e64 %[SW], -16, %[vsw]\n"                                 \
    "v_cmp_lt_u32_e64 %[HV], %[c65503], %[t6]\n"                            \
    "v_fma_f64 %[d2], %[d2], %[d1], %[d2]\n"                                \
    "v_add_u32 %[t0], %[qs], %[t0]\n"                                       \
    "v_and_b32 %[t1], %[qmask], %[t0]\n"                                    \
    "v_fma_f64 %[d0], %[d0], %[d2], %[c19]\n"                               \
    "v_lshl_add_u32 %[t1], %[t1], %[qlocv], %[u]\n"                         \
    "v_and_b32 %[t1], 0xffff, %[t1]\n"                                      \
    "v_cvt_u32_f64 %[t3], %[d0]\n"                                          \
    FQS_PB                                                                  \
    "v_mul_u32_u24 %[t2], 0x9e3779, %[t1]\n"                                \
    "v_mul_lo_u32 %[t3], %[vU], %[t3]\n"                                    \
    "v_mul_hi_u32_u24 %[t2], %[ns8], %[t2]\n"                               \
    "v_mad_u32_u24 %[t2], %[t2], %[v96], %[base]\n"                         \
    "v_cmp_gt_u32_e64 %[G], %[t3], s41\n"                                   \
    "v_and_b32 %[t5], %[vm63], %[t3]\n"                                     \
    "s_nop 1\n"                                                             \
    "s_andn2_b64 %[G], %[G], %[HV]\n"                                       \
    "s_and_b64 %[G], %[G], vcc\n"                                           \
    "s_ff1_i32_b64 %[k1], %[G]\n"                                           \
    "s_or_b64 %[SW], %[SW], %[lslow]\n"                                     \
    "s_bitcmp1_b64 %[SW], %[k1]\n"                                          \
    "s_cbranch_scc1 12f\n"                                                  \
    FQS_PC                                                                  \
    "v_readlane_b32 %[pk1], %[t3], %[k1]\n"                                 \
    "s_sub_u32 %[pk], %[k1], 1\n"                                           \
    "v_readlane_b32 %[pk], %[t5], %[pk]\n"                                  \
    "v_readlane_b32 %[cn], %[t1], %[k1]\n"                                  \
    "v_readlane_b32 %[man], %[t2], %[k1]\n"                                 \
    "v_readlane_b32 %[qsk], %[t0], %[k1]\n"                                 \
    "v_cndmask_b32 %[t4], 0, 16, %[G]\n"                                    \
    "v_add_u32 %[vU], %[vU], %[t4]\n"                                       \
    "s_sub_u32 s41, s41, %[pk]\n"                                           \
    "s_sub_u32 %[rng], %[pk1], %[pk]\n"                                     \
    "s_sub_u32 %[sym], %[qsk], %[qs]\n"                                     \
    "s_flbit_i32_b32 %[z], %[rng]\n"                                        \
    "v_writelane_b32 %[vout], %[sym], m0\n"                                 \
    DTUPD                                                                   \
    "s_lshl_b32 %[qs], %[qsk], %[qshift]\n"                                 \
    "s_add_u32 m0, m0, 1\n"                                                 \
    "ds_write_b16 %[vaddr], %[vU]\n"                                        \
    FQS_PD                                                                  \
    "s_cmp_eq_u32 %[cn], %[c]\n"                                            \
    "s_cbranch_scc1 20f\n"                                                  \
    "s_mov_b32 %[c], %[cn]\n"                                               \
    "s_mov_b32 %[ma], %[man]\n"                                             \
    "v_add_u32 %[vaddr], %[man], %[voff]\n"                                 \
    "v_add_u32 %[vb], %[man], %[vwoff]\n"                                   \
    "ds_read_u16 %[vU], %[vaddr]\n"                                         \
    "ds_read_b64 v[2:3], %[vb] offset:16\n"                                 \
    "s_and_b32 %[z], %[z], 24\n"                                            \
    "s_cbranch_scc1 40f\n"                                                  \
    "30:\n"                                                                 \
    FQS_PE                                                                  \
    "s_cmp_lt_u32 m0, %[lim]\n"                                             \
    "s_cbranch_scc1 10b\n"                                                  \
    "s_branch 90f\n"                                                        \
    "20:\n"                                                                 \
    "v_add_u32 v2, %[cbig], v2\n"                                           \
    "s_and_b32 %[z], %[z], 24\n"                                            \
    "s_cbranch_scc1 41f\n"                                                  \
    "31:\n"                                                                 \
    FQS_PE                                                                  \
    "s_cmp_lt_u32 m0, %[lim]\n"                                             \
    "s_cbranch_scc1 11b\n"                                                  \
    "s_branch 90f\n"                                                        \
    FQS_RENORM_OUT("40", "30")                                              \
    FQS_RENORM_OUT("41", "31")                                              \
    "60:\n"                                                                 \
    "s_add_u32 %[vic], %[vic], 1\n"                                         \
    "s_and_b32 %[x], %[vic], 3\n"                                           \
    "s_lshl_b32 %[x], %[x], 4\n"                                            \
    "s_lshl_b64 %[HV], 0xffff, %[x]\n"                                      \
    "v_readlane_b32 %[k1], v2, %[x]\n"                                      \
    "s_mov_b64 exec, %[HV]\n"                                               \
    "s_and_b32 %[k1], %[k1], 0xffff\n"                                      \
    "v_mad_u32_u24 %[t4], %[k1], 24, %[vjoff]\n"                            \
    "v_mad_u32_u24 %[t5], %[k1], 24, 20\n"                                  \
    "global_store_short %[t4], %[vU], %[back]\n"                            \
    "global_store_dword %[t5], v3, %[back]\n"                               \
    "v_mad_u32_u24 %[t4], %[c], 24, %[vjoff]\n"                             \
    "v_mad_u32_u24 %[t5], %[c], 24, 16\n"                                   \
    "global_load_ushort %[vU], %[t4], %[back]\n"                            \
    "global_load_dwordx2 v[2:3], %[t5], %[back]\n"                          \
    "s_add_u32 %[nm], %[nm], 1\n"                                           \
    "s_waitcnt vmcnt(0)\n"                                                  \
    "v_and_b32 v2, 0xffff0000, v2\n"                                        \
    "v_or_b32 v2, %[c], v2\n"                                               \
    "ds_write_b16 %[vaddr], %[vU]\n"                                        \
    "ds_write_b64 %[vb], v[2:3] offset:16\n"                                \
    "s_mov_b64 exec, -1\n"                                                  \
    "s_nop 4\n"                                                             \
    "s_branch 11b\n"                                                        \
    "12:\n"                                                                 \
    "s_mov_b32 %[flags], 2\n"                                               \
    "90:\n"                                                                 \
    "s_waitcnt vmcnt(0) lgkmcnt(0)\n"                                       \
    "s_mov_b32 %[done], m0\n"                                               \
    "s_mov_b32 m0, %[m0s]\n"

// ---------------------------------------------------------------------------
// (The miss path sets the fetched model's tag to the context it asked for,
// so a damaged store can give wrong bytes but never an endless miss loop.)
// the decoder: one workgroup (one wave) per block of the batch.  DT: some
// parameter block has delta terms (dtab not all zero).
// ---------------------------------------------------------------------------
#ifdef FQZ5_SMALL_PROBE
// cycles per segment (A-B, B-C, C-D, D-E, E-A) summed over every fast
// symbol of every launch since the last read, and the symbols
__device__ unsigned long long g_fqsprobe[6];
extern "C" int fqz5_small_probe_read(uint64_t *out) {
    hipError_t e = hipMemcpyFromSymbol(out, HIP_SYMBOL(g_fqsprobe), sizeof(g_fqsprobe));
    const unsigned long long z[6] = {0, 0, 0, 0, 0, 0};
    if (e == hipSuccess) e = hipMemcpyToSymbol(HIP_SYMBOL(g_fqsprobe), z, sizeof(z));
    return int(e);
}
#endif

template <bool DT>
__global__ __launch_bounds__(64) void k_fqz_dec_small(const FqzDecJob *Js) {
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    const FqzDecJob J = load_job(Js + blockIdx.x);
    const uint32_t l = threadIdx.x;
    const FqzDevGlobal &g = *J.g;
    SmallModels &sm = *reinterpret_cast<SmallModels *>(lds + S_SMALL);
    const uint32_t gfl = U(g.gflags), nparam = U(g.nparam);
    const uint32_t L = U(g.max_sym) + 1;             // live symbols, 2..9 (host)
    const uint32_t NS = J.nsets, NS8 = NS << 8;
    const uint32_t CB = S_PAR + nparam * SPB;        // the model cache
    // the run addresses LDS by these offsets: the dynamic block must start
    // at LDS address 0 (no static __shared__ here)
    if (uint32_t(size_t((__attribute__((address_space(3))) uint8_t *)lds)) != 0) __builtin_trap();
    const uint32_t n = uint32_t(J.n);

    small_models_init(sm, g);
    for (uint32_t x = 0; x < nparam; x++) {
        uint16_t *pt = reinterpret_cast<uint16_t *>(lds + S_PAR + x * SPB);
        for (uint32_t i = l; i < 1024; i += 64) pt[i] = uint16_t(g.p[x].ptab[i]);
        for (uint32_t i = l; i < 256; i += 64) pt[(S_DTAB >> 1) + i] = uint16_t(g.p[x].dtab[i]);
    }
    // every way of a set holds the fresh model of a distinct context that
    // maps to the set (the backing store holds every context's fresh model),
    // so a way always holds some context's true state: way r takes the r-th
    // context to claim the set (an LDS counter in way 0's symbol word; the
    // host checks that every set has at least 4 contexts)
    for (uint32_t s = l; s < NS; s += 64) *reinterpret_cast<uint32_t *>(lds + CB + s * SETB + 20) = 0u;
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_s_waitcnt(0xc07f);
    for (uint32_t c = l; c < FQZ_CTX; c += 64) {
        const uint32_t a = sset(c, NS8, CB);
        uint32_t *cnt = static_cast<uint32_t *>(__builtin_assume_aligned(lds + a + 20, 4));
        const uint32_t r = atomicAdd(cnt, 1u);
        if (r < WAYS) *reinterpret_cast<uint16_t *>(lds + a + r * ME + 16) = uint16_t(c);
    }
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_s_waitcnt(0xc07f);
    for (uint32_t m = l; m < NS * WAYS; m += 64) {
        uint8_t *mm = lds + CB + m * ME;
        for (uint32_t w = 0; w < 4; w++) reinterpret_cast<uint32_t *>(mm)[w] = fresh_word(w, L, 0);
        *reinterpret_cast<uint16_t *>(mm + 18) = uint16_t(L);
        reinterpret_cast<uint32_t *>(mm)[5] = fresh_word(5, L, 0);
    }
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_s_waitcnt(0xc07f);

    In in;
    uint32_t code = 0;
    in_start<S_RING>(lds, in, J.in, uint32_t(J.in_len), code);
    uint32_t rng = 0xFFFFFFFFu;

    const __amdgpu_buffer_rsrc_t orsrc = rsrc(J.out, n);
    uint32_t obase = 0, fill = 0;             // output page covers [obase, obase + fill)
    uint32_t rec = 0, prev_len = 0, left = 0;
    uint32_t nrecs = 0, ndups = 0, nrevs = 0, nmiss = 0, nslow = 0;
    bool first_len = true;
    int status = 0;
    PS ps = load_ps(g, 0);
    uint32_t qctx = 0, delta = 0, prevq = 0, sel = 0, selterm = 0;
    uint32_t ctx = 0, maddr = CB;
    const uint32_t dlane = S_DUMMY + 4 * l;
    const uint16_t *pt16 = reinterpret_cast<const uint16_t *>(lds + S_PAR);
    // the run's lanes are 4 rows of 16, row w = way w of the set: lane 16w + i
    // holds U_{i+1} of that way's model, lanes 16w + 8.. its total
    const uint32_t vjoff = (l & 15u) < 8u ? 2u * (l & 15u) : 18u;
    const uint32_t vwoff = ME * (l >> 4), voff = vwoff + vjoff;
    uint32_t vic = 0;                                  // the miss victim: way vic & 3

    auto flush = [&]() {
        for (uint32_t o = l * 4; o < fill; o += 256) {
            const uint32_t w = *reinterpret_cast<const uint32_t *>(lds + S_OBUF + o);
#pragma unroll
            for (uint32_t b = 0; b < 4; b++)
                if (o + b < fill) st8(orsrc, obase + o + b, w >> (8 * b));
        }
        obase += fill;
        fill = 0;
    };
    // the context after symbol `sym`, uniform (fqz_update_ctx with qtab the
    // identity; the slow paths)
    auto next_uniform = [&](uint32_t sym) {
        uint32_t u = U(pt16[left < 1023u ? left : 1023u]);
        if (DT) u += U(pt16[(S_DTAB >> 1) + (delta < 255u ? delta : 255u)]);
        u += selterm;
        qctx = (qctx << ps.qshift) + sym;
        ctx = (((qctx & ps.qmask) << ps.qloc) + u) & uint32_t(FQZ_CTX - 1);
        maddr = sset(ctx, NS8, CB);
        delta += prevq != sym;
        prevq = sym;
        left--;
    };
    // the way of ctx's set that holds its model; on a miss the victim way's
    // model goes back to the store and ctx's comes in (the run's rule)
    auto ensure = [&]() -> uint32_t {
        for (uint32_t w = 0; w < WAYS; w++)
            if (U(*reinterpret_cast<const uint16_t *>(lds + maddr + w * ME + 16)) == ctx)
                return maddr + w * ME;
        nmiss++;
        vic = U(vic + 1u);
        const uint32_t wa = maddr + (vic & 3u) * ME;
        const uint32_t tag = U(*reinterpret_cast<const uint16_t *>(lds + wa + 16));
        uint32_t *m32 = reinterpret_cast<uint32_t *>(lds + wa);
        const uint32_t mine = l < 6 ? m32[l] : 0u;
        uint32_t *dst = reinterpret_cast<uint32_t *>(J.back + size_t(tag) * ME);
        const uint32_t *src = reinterpret_cast<const uint32_t *>(J.back + size_t(ctx) * ME);
        if (l < 6) __hip_atomic_store(dst + l, mine, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
        const uint32_t v = l < 6 ? __hip_atomic_load(src + l, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT) : 0u;
        __builtin_amdgcn_wave_barrier();
        if (l < 6) m32[l] = l == 4 ? (v & 0xffff0000u) | ctx : v;
        __builtin_amdgcn_wave_barrier();
        return wa;
    };
    // one symbol with the reference's arithmetic (c_simple_model.h:140-171,
    // fl_bump): halving, bubble steps, the 9th slot, corrupt or truncated
    // streams, the last bytes of the input
    auto slow_symbol = [&]() {
        nslow++;
        const uint32_t wa = ensure();
        const uint32_t uw = *reinterpret_cast<const uint16_t *>(lds + wa + vjoff);
        const uint32_t S = U(*reinterpret_cast<const uint32_t *>(lds + wa + 20));
        uint32_t total = U(*reinterpret_cast<const uint16_t *>(lds + wa + 18));
        uint32_t t = 0;
        if (total && rng >= total) {   // the division stays even when no symbol follows
            rng /= total;
            t = code / rng;
        }
        uint32_t sym = 0;
        if (t < total) {
            const bool live = l < L;
            const uint32_t up = live ? uw : 0u;                       // U_{l+1}
            const uint32_t lo_l = __shfl_up(up, 1, 64);
            const uint32_t lo = l ? lo_l : 0u;                        // U_l
            uint32_t f = live ? up - lo : 0u;                         // freq of slot l+1
            // the symbols: nibbles for slots 1..8, slot 9 the missing one
            uint32_t sy = (S >> (4 * (l & 7))) & 15u;
            if (L == 9 && l == 8) {
                uint32_t sum = 0;
                for (uint32_t i = 0; i < 8; i++) sum += (S >> (4 * i)) & 15u;
                sy = 36u - sum;
            }
            const uint64_t gt = __ballot(live && up > t);
            const uint32_t k = uint32_t(__builtin_ctzll(gt));        // slot k + 1
            const uint32_t lk = RL(lo, k), fk = RL(f, k);
            code -= lk * rng;
            rng *= fk;
            renorm_slow<S_RING>(lds, in, rng, code);
            sym = RL(sy, k);
            if (l == k) f += FL_STEP;
            total += FL_STEP;
            if (total > FL_MAX) f -= f >> 1;                          // halve every live slot
            // bubble: slot k + 1 over slot k when its frequency passes it
            if (k >= 1) {
                const uint32_t fa = RL(f, k - 1), fb = RL(f, k);
                if (fb > fa) {
                    const uint32_t sa = RL(sy, k - 1), sb = RL(sy, k);
                    if (l == k - 1) { f = fb; sy = sb; }
                    if (l == k) { f = fa; sy = sa; }
                }
            }
            // cumulative counts again
            uint32_t inc = f;
#pragma unroll
            for (int d = 1; d < 64; d <<= 1) {
                const uint32_t o = __shfl_up(inc, d, 64);
                if (int(l) >= d) inc += o;
            }
            total = RL(inc, L - 1);
            uint32_t nS = 0;
            for (uint32_t i = 0; i < 8; i++) nS |= (RL(sy, i) & 15u) << (4 * i);
            if (l < 8) *reinterpret_cast<uint16_t *>(lds + wa + 2 * l) = uint16_t(live ? inc : total);
            if (l == 0) {
                *reinterpret_cast<uint16_t *>(lds + wa + 18) = uint16_t(total);
                *reinterpret_cast<uint32_t *>(lds + wa + 20) = nS;
            }
            __builtin_amdgcn_wave_barrier();
        }
        lds[l ? dlane : S_OBUF + fill] = uint8_t(sym);
        fill++;
        next_uniform(sym);
    };

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
            if (fill == SOBUF) flush();
            const uint32_t i = obase + fill;
            sel = (ps.sel || (gfl & 1u)) ? small_decode<S_RING>(&sm.sel, lds, in, rng, code) : 0u;
            const uint32_t x = (gfl & 2u) ? U(g.stab[sel < 255u ? sel : 255u]) : sel;
            if (x >= nparam) { status = -1; break; }
            ps = load_ps(g, x);
            uint32_t len = prev_len;
            if (!ps.fixed || first_len) {
                len = 0;
                for (int b = 0; b < 4; b++) len |= small_decode<S_RING>(&sm.len[b], lds, in, rng, code) << (8 * b);
                first_len = false;
                prev_len = len;
            }
            if (len > n - i || len == 0) { status = -1; break; }
            if (rec < J.nlengths && l == 0) J.lengths[rec] = len;
            if (gfl & 4u) {
                if (small_decode<S_RING>(&sm.rev, lds, in, rng, code)) {
                    if (nrevs >= J.cap_list) { status = -2; break; }
                    if (l == 0) J.revs[nrevs] = make_uint2(i, len);
                    nrevs++;
                }
            }
            rec++;
            if (ps.dedup && small_decode<S_RING>(&sm.dup, lds, in, rng, code)) {
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
            delta = prevq = qctx = 0;
            selterm = sel << ps.sloc;
            pt16 = reinterpret_cast<const uint16_t *>(lds + S_PAR + ps.x * SPB);
            ctx = ps.ctx0;
            maddr = sset(ctx, NS8, CB);
        }
        if (in.avail() < 4u) {   // the last bytes of the input: reference arithmetic
            slow_symbol();
            if (fill == SOBUF) flush();
            continue;
        }
        // ---- fast run: up to 64 symbols of this record within the output
        // page ----------------------------------------------------------------
        uint32_t lim = left < SOBUF - fill ? left : SOBUF - fill;
        if (lim > 64u) lim = 64u;
        uint32_t ulim = (in.vb - 4u) * 8u;
        // per-step context terms of the run (fqz_update_ctx uses the position
        // and delta before this symbol's update): lane i the position term of
        // step i, lane j the delta term of delta0 + j
        const uint32_t delta0 = U(delta);
        const uint32_t pvv = uint32_t(pt16[left - l < 1023u ? left - l : 1023u]) + selterm;
        const uint32_t dvv = DT ? uint32_t(pt16[(S_DTAB >> 1) + (delta + l < 255u ? delta + l : 255u)]) : 0u;
        const uint32_t qshift = U(ps.qshift);
        uint32_t qs = U(qctx << qshift);
        uint32_t vout = 0, done = 0, flags = 0;
        {
            uint64_t cw = uint64_t(U(code)) << 32;   // {scratch, code}
            uint64_t win = (uint64_t(U(uint32_t(in.W >> 32))) << 32) | U(uint32_t(in.W));
            uint64_t mAS = 0;
            uint32_t cc = U(ctx), pv = U(prevq), ma = U(maddr);
            uint32_t dd = 0, nm = 0;
            uint32_t vU = 0, vaddr = 0, vsw = (l & 15u) == 0 ? 0x80000000u : 0u;
            uint64_t scr;
            const uint64_t back = reinterpret_cast<uint64_t>(J.back);
            rng = U(rng);
            in.rb = U(in.rb);
            const uint32_t bswp = 0x00010203u;   // v_perm byte reversal
            auto rb_end = [&]() {   // the window refills in the run while the ring holds rb + 8 .. rb + 11
                const uint32_t e = in.len < in.lp ? in.len : in.lp;
                return U(e >= 12u ? e - 11u : 0u);
            };
            uint32_t rbend = rb_end();
            in.ub = U(in.ub);
            lim = U(lim);
            ulim = U(ulim);
            const uint32_t base = U(CB), cbig = 0x100000u, c65503 = 65503u;
            const uint32_t ns8 = U(NS8), qlocv = ps.qloc, qmask = U(ps.qmask);
            // slots past min(L, 8) of every row go to the slow path with
            // the bubbles (one mask); p_{k-1} of slot 1 (a row's lane 0) is
            // read from the lane before the row: 0
            const uint32_t lfast = U(L < 8u ? L : 8u), vsh4 = 4u * (l & 7u);
            const uint64_t lslow = 0x0001000100010001ull * uint64_t(0xffffu & ~((1u << lfast) - 1u));
            const uint32_t vm63 = (l & 15u) == 15u ? 0u : ~0u;
            const double c19 = 0x1p-19;
            uint32_t u, x, k1, pk, pk1, cn, man, qsk, sym, z, m0s;
            uint64_t G, SW, HV;
            uint32_t t0, t1, t2, t3, t4, t5, t6, vb;
            double d0, d1, d2;
#ifdef FQZ5_SMALL_PROBE
            uint32_t pr1 = 0, pr2 = 0, pr3 = 0, pr4 = 0, pr5 = 0;
            uint64_t ps0, ps1, ps2, ps3, ps4, ps5;
#define FQS_PROBE_OPS , [pr1] "+s"(pr1), [pr2] "+s"(pr2), [pr3] "+s"(pr3), [pr4] "+s"(pr4), \
    [pr5] "+s"(pr5), [ps0] "=&{s[46:47]}"(ps0), [ps1] "=&{s[48:49]}"(ps1),                      \
    [ps2] "=&{s[50:51]}"(ps2), [ps3] "=&{s[52:53]}"(ps3), [ps4] "=&{s[54:55]}"(ps4),          \
    [ps5] "=&{s[56:57]}"(ps5)
#else
#define FQS_PROBE_OPS
#endif
            for (;;) {
#define FQS_OPERANDS                                                                           \
                : [mAS] "+{v[2:3]}"(mAS), [cw] "+{s[40:41]}"(cw), [win] "+{s[42:43]}"(win),   \
                  [scr] "=&{s[44:45]}"(scr), [rb] "+s"(in.rb), [ub] "+s"(in.ub),               \
                  [rng] "+s"(rng), [dd] "+s"(dd), [done] "+s"(done), [nm] "+s"(nm),            \
                  [c] "+s"(cc), [qs] "+s"(qs), [pv] "+s"(pv), [ma] "+s"(ma), [vic] "+s"(vic),  \
                  [flags] "=&s"(flags), [vU] "+v"(vU), [vaddr] "+v"(vaddr), [vout] "+v"(vout),  \
                  [vsw] "+v"(vsw), [vb] "=&v"(vb),                                             \
                  [u] "=&s"(u), [x] "=&s"(x), [k1] "=&s"(k1), [pk] "=&s"(pk), [pk1] "=&s"(pk1), \
                  [cn] "=&s"(cn), [man] "=&s"(man), [qsk] "=&s"(qsk), [sym] "=&s"(sym),        \
                  [z] "=&s"(z), [m0s] "=&s"(m0s), [G] "=&s"(G), [SW] "=&s"(SW), [HV] "=&s"(HV), \
                  [t0] "=&v"(t0), [t1] "=&v"(t1), [t2] "=&v"(t2), [t3] "=&v"(t3),             \
                  [t4] "=&v"(t4), [t5] "=&v"(t5), [t6] "=&v"(t6),                              \
                  [d0] "=&v"(d0), [d1] "=&v"(d1), [d2] "=&v"(d2) FQS_PROBE_OPS                  \
                : [lim] "s"(lim), [ulim] "s"(ulim), [qmask] "s"(qmask), [qshift] "s"(qshift), \
                  [ns8] "s"(ns8), [base] "s"(base), [lslow] "s"(lslow), [c65503] "s"(c65503), \
                  [rbend] "s"(rbend), [bswp] "s"(bswp), [lring] "i"(S_RING), [back] "s"(back),  \
                  [voff] "v"(voff), [vsh4] "v"(vsh4), [qlocv] "v"(qlocv), [cbig] "v"(cbig),   \
                  [c19] "v"(c19), [pvv] "v"(pvv), [dvv] "v"(dvv),                              \
                  [vm63] "v"(vm63), [vwoff] "v"(vwoff), [vjoff] "v"(vjoff), [v96] "v"(SETB)    \
                : "memory", "scc", "vcc"
                if constexpr (DT)
                    asm volatile(FQS_RUN_ASM(FQS_DT_U, FQS_DT_ADD, FQS_DT_UPD) FQS_OPERANDS);
                else
                    asm volatile(FQS_RUN_ASM(FQS_NONE, FQS_NONE, FQS_NONE) FQS_OPERANDS);
#undef FQS_OPERANDS
#undef FQS_PROBE_OPS
                // (the compiler takes every output of an asm with VGPR outputs
                // for divergent: the scalar ones are re-read as uniform)
                rng = U(rng);
                in.ub = U(in.ub);
                in.rb = U(in.rb);
                dd = U(dd);
                done = U(done);
                nm = U(nm);
                cc = U(cc);
                qs = U(qs);
                pv = U(pv);
                ma = U(ma);
                vic = U(vic);
                flags = U(flags);
                cw = (uint64_t(U(uint32_t(cw >> 32))) << 32);
                win = (uint64_t(U(uint32_t(win >> 32))) << 32) | U(uint32_t(win));
#ifdef FQZ5_SMALL_PROBE
                if (l == 0 && blockIdx.x == 0) {
                    atomicAdd(&g_fqsprobe[0], (unsigned long long)U(pr1));
                    atomicAdd(&g_fqsprobe[1], (unsigned long long)U(pr2));
                    atomicAdd(&g_fqsprobe[2], (unsigned long long)U(pr3));
                    atomicAdd(&g_fqsprobe[3], (unsigned long long)U(pr4));
                    atomicAdd(&g_fqsprobe[4], (unsigned long long)U(pr5));
                    atomicAdd(&g_fqsprobe[5], (unsigned long long)U(done));
                }
                pr1 = pr2 = pr3 = pr4 = pr5 = 0;
#endif
                if (flags == 2 || done == lim) break;
                in.W = win;   // the input window needs a refill
                refill_s(lds, in);
                win = in.W;
                if (in.vb < 4u) break;
                ulim = (in.vb - 4u) * 8u;
                rbend = rb_end();
            }
            in.W = win;
            code = uint32_t(cw >> 32);
            ctx = cc;
            prevq = pv;
            maddr = ma;
            delta = delta0 + dd;
            nmiss += nm;
            left -= done;
        }
        qctx = qs >> qshift;
        if (l < done) lds[S_OBUF + fill + l] = uint8_t(vout);
        fill += done;
        if (flags == 2) slow_symbol();
        if (fill == SOBUF) flush();
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
}

// the backing store: every context's fresh model (its tag the context)
__global__ void k_fqz_small_back(uint32_t *back, uint32_t L) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;   // word of the store
    if (i >= uint32_t(FQZ_CTX) * 6u) return;
    back[i] = fresh_word(i % 6u, L, i / 6u);
}

}  // namespace

hipError_t launch_fqz_dec_small(const FqzDecJob *j, int n, bool dt, hipStream_t s) {
    auto *f = dt ? k_fqz_dec_small<true> : k_fqz_dec_small<false>;
    hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void *>(f),
                                       hipFuncAttributeMaxDynamicSharedMemorySize, LDS_BYTES);
    if (e != hipSuccess) return e;
    if (n) hipLaunchKernelGGL(f, dim3(n), dim3(64), LDS_BYTES, s, j);
    return hipGetLastError();
}

hipError_t launch_fqz_small_back(uint8_t *back, uint32_t live, hipStream_t s) {
    const uint32_t words = uint32_t(FQZ_CTX) * 6u;
    hipLaunchKernelGGL(k_fqz_small_back, dim3((words + 255) / 256), dim3(256), 0, s,
                       reinterpret_cast<uint32_t *>(back), live);
    return hipGetLastError();
}

}  // namespace fqz5
