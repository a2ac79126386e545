// fastq.hip — FASTQ text in HBM to fqzcomp5 blocks and back:
// the record parse of load_seqs_kseq (fqzcomp5.c:423-623, kseq.h:178-218)
// for 4-line FASTQ, its block split rule (fqzcomp5.c:471-477), the gather of
// a block's name / sequence / quality sections with the records' lengths and
// READ2 flags, and output_fastq / output_fasta (fqzcomp5.c:3441-3480,
// :3503-3517) on decoded blocks.
//
// Lines: every '\n' of the text is found by 64 KiB tiles (counts, a scan,
// then ordered writes), so FASTQ record r is lines 4r..4r+3.  FASTA (text
// whose first byte is '>'): a record per header line, its sequence lines
// joined as kseq joins them; the block then has no quality section
// (fqzcomp5.c:575-578, :2258-2264).  Records are parsed one per thread (FASTA:
// one wave); the section bytes are gathered one wave per record at the
// scanned offsets.  FASTQ that is not 4-line (multi-line records) is refused
// with an error, never parsed on the host.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <cstring>
#include <vector>

#include "../../include/fqz5_fastq.h"
#include "gpu_ctx.hpp"

namespace fqz5 {
GpuCtx &gpu();
void fqz5_set_error(const char *msg);

namespace {

constexpr int FQ_TPB = 256;
constexpr uint32_t FQ_STEP = FQ_TPB * 16;          // bytes per workgroup iteration
constexpr uint32_t FQ_ITERS = 16;
constexpr uint64_t FQ_TILE = uint64_t(FQ_STEP) * FQ_ITERS;   // 64 KiB

__device__ __forceinline__ uint32_t count_in16(const uint8_t *t, uint64_t at, uint64_t len,
                                               uint8_t ch) {
    uint32_t c = 0;
    if (at + 16 <= len && !(reinterpret_cast<uintptr_t>(t + at) & 15)) {
        const uint4 v = *reinterpret_cast<const uint4 *>(t + at);
        const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int k = 0; k < 4; k++)
#pragma unroll
            for (int b = 0; b < 4; b++) c += ((w[k] >> (8 * b)) & 0xffu) == ch;
    } else {
        const uint64_t e = at + 16 < len ? at + 16 : len;
        for (uint64_t p = at; p < e; p++) c += t[p] == ch;
    }
    return c;
}

// per 64 KiB tile: the number of `ch` bytes
__global__ void k_delim_count(const uint8_t *t, uint64_t len, uint8_t ch, uint32_t *tile_cnt) {
    using BR = hipcub::BlockReduce<uint32_t, FQ_TPB>;
    __shared__ typename BR::TempStorage tmp;
    const uint64_t base = uint64_t(blockIdx.x) * FQ_TILE;
    uint32_t c = 0;
    for (uint32_t it = 0; it < FQ_ITERS; it++) {
        const uint64_t at = base + uint64_t(it) * FQ_STEP + uint64_t(threadIdx.x) * 16;
        if (at < len) c += count_in16(t, at, len, ch);
    }
    const uint32_t s = BR(tmp).Sum(c);
    if (threadIdx.x == 0) tile_cnt[blockIdx.x] = s;
}

// positions of every `ch` byte, in text order, from the tiles' scanned counts
__global__ void k_delim_write(const uint8_t *t, uint64_t len, uint8_t ch, const uint32_t *tile_off,
                              uint64_t *pos) {
    using BS = hipcub::BlockScan<uint32_t, FQ_TPB>;
    __shared__ typename BS::TempStorage tmp;
    const uint64_t base = uint64_t(blockIdx.x) * FQ_TILE;
    uint64_t o = tile_off[blockIdx.x];
    for (uint32_t it = 0; it < FQ_ITERS; it++) {
        const uint64_t at = base + uint64_t(it) * FQ_STEP + uint64_t(threadIdx.x) * 16;
        const uint32_t c = at < len ? count_in16(t, at, len, ch) : 0u;
        uint32_t ex, tot;
        BS(tmp).ExclusiveSum(c, ex, tot);
        __syncthreads();
        if (c) {
            uint64_t w = o + ex;
            const uint64_t e = at + 16 < len ? at + 16 : len;   // (count_in16's bytes)
            for (uint64_t p = at; p < e; p++)
                if (t[p] == ch) pos[w++] = p;
        }
        o += tot;
    }
}

__device__ __forceinline__ bool ks_space(uint8_t c) { return c == ' ' || (c >= 9 && c <= 13); }

// kseq's line read: drop a trailing '\r' when the line has more than one
// byte (kseq.h:141)
__device__ __forceinline__ uint64_t strip_cr(const uint8_t *t, uint64_t s, uint64_t e) {
    return (e - s > 1 && t[e - 1] == '\r') ? e - 1 : e;
}

// the header line [s0, e0): name up to the first isspace(), the comment
// after it to the line end (kseq.h:188-189)
__device__ __forceinline__ void header(const uint8_t *t, uint64_t s0, uint64_t e0, fqz5_fastq_rec &R) {
    uint64_t p = s0 + 1;
    while (p < e0 && !ks_space(t[p])) p++;
    R.name = s0 + 1;
    R.name_len = uint32_t(p - (s0 + 1));
    R.comment = p < e0 ? p + 1 : e0;
    R.comment_len = p < e0 ? uint32_t(strip_cr(t, p + 1, e0) - (p + 1)) : 0u;
}

// record r = lines 4r..4r+3 (kseq_read, kseq.h:178-218)
__global__ void k_fq_records(const uint8_t *t, const uint64_t *nl, uint64_t nrec,
                             fqz5_fastq_rec *recs, uint32_t *rec_size, int32_t *status) {
    const uint64_t r = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x;
    if (r >= nrec) return;
    const uint64_t s0 = r ? nl[4 * r - 1] + 1 : 0, e0 = nl[4 * r];
    const uint64_t s1 = e0 + 1, e1 = nl[4 * r + 1];
    const uint64_t s2 = e1 + 1, e2 = nl[4 * r + 2];
    const uint64_t s3 = e2 + 1, e3 = nl[4 * r + 3];
    int bad = 0;
    if (e0 <= s0 || t[s0] != '@') bad = 1;            // header
    if (e2 <= s2 || t[s2] != '+') bad = 1;            // '+' line
    if (e1 > s1 && (t[s1] == '@' || t[s1] == '>' || t[s1] == '+')) bad = 1;
    fqz5_fastq_rec R;
    header(t, s0, e0, R);
    R.seq = s1;
    R.seq_len = uint32_t(strip_cr(t, s1, e1) - s1);
    R.qual = s3;
    R.fasta = 0;
    R.end = e3 + 1;
    const uint32_t ql = uint32_t(strip_cr(t, s3, e3) - s3);
    if (ql != R.seq_len) bad = 1;                     // kseq -2 (:213-216)
    recs[r] = R;
    rec_size[r] = R.name_len + 1 + 2 * R.seq_len;     // load_seqs_kseq's record_size (:472)
    if (bad) atomicMin(status, int32_t(-1 - int32_t(r < 0x7ffffffeull ? r : 0x7ffffffeull)));
}

// FASTA lines: a header starts with '>'; a line starting with '@' or '+'
// would make kseq read a FASTQ record (kseq.h:194, :206) and is refused, as
// is text whose first line is not a header
__global__ void k_fa_lines(const uint8_t *t, const uint64_t *nl, uint64_t nlines, uint32_t *hdr,
                           int32_t *status) {
    const uint64_t i = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x;
    if (i >= nlines) return;
    const uint64_t s = i ? nl[i - 1] + 1 : 0, e = nl[i];
    const uint8_t c = e > s ? t[s] : uint8_t('\n');
    hdr[i] = c == '>';
    if (c == '@' || c == '+' || (i == 0 && c != '>'))
        atomicMin(status, int32_t(-1 - int32_t(i < 0x7ffffffeull ? i : 0x7ffffffeull)));
}

__global__ void k_fa_scatter(const uint32_t *hdr, const uint32_t *pos, uint64_t nlines, uint64_t *hl) {
    const uint64_t i = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x;
    if (i < nlines && hdr[i]) hl[pos[i]] = i;
}

// kseq's FASTA sequence over text [sb, se) (kseq.h:194-198): every line's
// bytes joined, empty lines skipped, a '\r' before a line end dropped unless
// it would be the sequence's only byte (the KS_SEP_LINE strip, :141, tests
// the whole sequence's length).  One wave: returns the byte count and, with
// `out`, writes the bytes.
__device__ uint32_t fa_seq(const uint8_t *t, uint64_t sb, uint64_t se, uint8_t *out) {
    const uint32_t lane = threadIdx.x & 63;
    uint32_t n = 0;
    bool any = false;                                 // a non-'\n' byte before
    for (uint64_t base = sb; base < se; base += 64) {
        const uint64_t p = base + lane;
        const uint8_t c = p < se ? t[p] : uint8_t('\n');
        const uint64_t nonl = __builtin_amdgcn_ballot_w64(c != '\n');
        const uint64_t below = (lane ? (~0ull >> (64 - lane)) : 0ull);
        const bool before = any || (nonl & below) != 0;
        bool keep = c != '\n';
        if (c == '\r' && (p + 1 == se || t[p + 1] == '\n') && before) keep = false;
        const uint64_t km = __builtin_amdgcn_ballot_w64(keep);
        if (keep && out) out[n + __builtin_popcountll(km & below)] = c;
        n += uint32_t(__builtin_popcountll(km));
        any = any || nonl != 0;
    }
    return n;
}

// one wave per FASTA record: header line hl[r], its sequence up to the next
// header (or the text end); R.qual holds that end offset
__global__ void k_fa_records(const uint8_t *t, uint64_t len, const uint64_t *nl, const uint64_t *hl,
                             uint64_t nrec, fqz5_fastq_rec *recs, uint32_t *rec_size) {
    const uint64_t r = (uint64_t(blockIdx.x) * blockDim.x + threadIdx.x) / 64;
    if (r >= nrec) return;
    const uint64_t h = hl[r];
    const uint64_t s0 = h ? nl[h - 1] + 1 : 0, e0 = nl[h];
    const uint64_t sb = e0 + 1 < len ? e0 + 1 : len;
    const uint64_t se = r + 1 < nrec ? nl[hl[r + 1] - 1] + 1 : len;
    const uint32_t n = fa_seq(t, sb, se, nullptr);
    if ((threadIdx.x & 63) == 0) {
        fqz5_fastq_rec R;
        header(t, s0, e0, R);
        R.seq = sb;
        R.qual = se;
        R.seq_len = n;
        R.fasta = 1;
        R.end = se;
        recs[r] = R;
        rec_size[r] = R.name_len + 1 + n;             // qual.l = 0 (:472)
    }
}

// ---------------------------------------------------------------------------
// Wrapped (multi-line) FASTQ, as kseq_read reads it (kseq.h:194-216): after
// the header, sequence lines up to a line starting with '+' (empty lines
// skipped; a line starting with '@' or '>' would end the record without
// qualities), then quality lines until their bytes reach the sequence's
// length.  The record that starts at a '@' line is fixed by the lines after
// it alone, so every '@' line is tried as a header in parallel (its '+' line,
// sequence length and last quality line by binary searches over the line
// tables) and yields the '@' line the next record would start at; the true
// records are the chain of those links from line 0, walked on the host over
// one int per '@' line.  Lines: `cls` the first byte (0 empty, 1 a lone
// '\r'), `ls` the bytes kseq keeps (a trailing '\r' dropped, KS_SEP_LINE
// :141), P their prefix sums.  kseq's two odd layouts are followed (round
// 6): a lone-'\r' line before the first kept byte of a sequence or quality
// block is kept as a '\r' byte (the strip needs two bytes in the string,
// kseq.h:141; the record's fasta field carries FQ_KEEP_CR_SEQ / _QUAL), and
// bytes between records (or before the first) are skipped to the next
// header as kseq_read's scan for '@' / '>' skips them (:180-186), when those
// lines hold neither byte (`ga`, a line holding '@' or '>' anywhere, and its
// prefix sums GA).  Refused (never guessed): a record without a '+' line,
// qualities longer than the bases, skipped bytes holding '@' or '>' away
// from a line start (kseq would start a record mid-line there).
// ---------------------------------------------------------------------------
constexpr int32_t ML_END = -1, ML_MORE = -2, ML_BAD = -3;
constexpr uint32_t FQ_KEEP_CR_SEQ = 1u << 8, FQ_KEEP_CR_QUAL = 1u << 9;   // fasta field bits

__global__ void k_ml_lines(const uint8_t *t, const uint64_t *nl, uint64_t nlines, uint8_t *cls,
                           uint32_t *ls, uint32_t *f_at, uint32_t *f_stop, uint32_t *f_cr,
                           uint32_t *f_ga) {
    const uint64_t i = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x;
    if (i >= nlines) return;
    const uint64_t s = i ? nl[i - 1] + 1 : 0, e = nl[i];
    const uint64_t L = e - s;
    uint8_t c = L ? t[s] : uint8_t(0);
    const bool cr = L && t[e - 1] == '\r';
    if (L == 1 && cr) c = 1;
    cls[i] = c;
    ls[i] = uint32_t(L - (cr ? 1 : 0));
    f_at[i] = c == '@';
    f_stop[i] = c == '@' || c == '+' || c == '>';
    f_cr[i] = c == 1;
    // '@' or '>' anywhere in the line: where kseq's skip to the next header
    // would stop (a line start already stops at a header line)
    uint32_t ga = 0;
    for (uint64_t p = s; p < e && !ga; p++) ga = t[p] == '@' || t[p] == '>';
    f_ga[i] = ga;
}

__global__ void k_ends4(const uint64_t *nl, uint64_t n4, uint64_t len, uint64_t *ends) {
    const uint64_t r = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x;
    if (r < n4) ends[r] = nl[4 * r + 3] + 1 < len ? nl[4 * r + 3] + 1 : len;
}

__global__ void k_widen(const uint32_t *in, uint64_t *out, uint64_t n) {
    const uint64_t i = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x;
    if (i < n) out[i] = in[i];
}

__global__ void k_ml_scatter(const uint32_t *flag, const uint32_t *pos, uint64_t n, uint32_t *list) {
    const uint64_t i = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x;
    if (i < n && flag[i]) list[pos[i]] = uint32_t(i);
}

// first index of sorted a[0..n) with a[i] >= x (n if none)
__device__ __forceinline__ uint32_t lower_u32(const uint32_t *a, uint32_t n, uint32_t x) {
    uint32_t lo = 0, hi = n;
    while (lo < hi) {
        const uint32_t m = (lo + hi) >> 1;
        if (a[m] < x) lo = m + 1; else hi = m;
    }
    return lo;
}

// '@' line ats[a] taken as a header: next[a] = the '@' index of the next
// record (ML_END: none, the rest empty; ML_MORE: the text ends inside the
// record and more is coming; ML_BAD: not a record kseq reads the same way)
// a lone-'\r' line in the block of lines [a, b) before any kept byte: kseq
// would keep that '\r' (its strip needs two bytes, kseq.h:141)
__device__ __forceinline__ bool lone_cr_first(const uint64_t *P, const uint32_t *crs, uint32_t ncr,
                                              uint32_t a, uint32_t b) {
    const uint32_t i = lower_u32(crs, ncr, a);
    return i < ncr && crs[i] < b && P[crs[i]] == P[a];
}

__global__ void k_ml_cand(const uint8_t *cls, const uint64_t *P, const uint32_t *crs, uint32_t ncr,
                          const uint32_t *GA, uint32_t nlines, const uint32_t *ats, uint32_t nat,
                          const uint32_t *stops, uint32_t nst, int eof, int32_t *next, uint32_t *jq,
                          uint32_t *kq, uint32_t *slen, uint32_t *kcr) {
    const uint32_t a = blockIdx.x * blockDim.x + threadIdx.x;
    if (a >= nat) return;
    const uint32_t h = ats[a];
    const int32_t short_ = eof ? ML_BAD : ML_MORE;
    int32_t r = ML_BAD;
    uint32_t j = 0, k = 0, sl = 0, crf = 0;
    do {
        const uint32_t js = lower_u32(stops, nst, h + 1);
        if (js >= nst) { r = short_; break; }            // no '+' line yet
        j = stops[js];
        if (cls[j] != '+') break;                         // a record without qualities
        // a lone '\r' line before the first kept base: kseq keeps it (one byte)
        const uint32_t cs = lone_cr_first(P, crs, ncr, h + 1, j) ? 1u : 0u;
        const uint64_t seq_len = P[j] - P[h + 1] + cs;
        if (seq_len > 0xffffffffull) break;
        sl = uint32_t(seq_len);
        if (j + 1 >= nlines) { r = short_; break; }       // no quality line yet
        const uint64_t base = P[j + 1];
        // the same for the qualities: a lone-'\r' line cq before any kept
        // quality byte counts one byte from its line on
        const uint32_t ic = lower_u32(crs, ncr, j + 1);
        const bool hc = ic < ncr && P[crs[ic]] == base;
        const uint32_t cq = hc ? crs[ic] : 0u;
        // the smallest k >= j + 1 whose quality bytes through line k reach
        // seq_len (kseq reads at least one quality line)
        uint32_t lo = j + 1, hi = nlines;
        if (hc && seq_len <= 1 && seq_len) {
            lo = cq;                                      // the '\r' alone is the qualities
        } else {
            const uint64_t need = hc && seq_len ? seq_len - 1 : seq_len;
            while (lo < hi) {
                const uint32_t m = lo + ((hi - lo) >> 1);
                if (P[m + 1] - base >= need) hi = m; else lo = m + 1;
            }
        }
        if (lo >= nlines) { r = short_; break; }
        k = lo;
        const uint64_t got = P[k + 1] - base + ((hc && cq <= k) ? 1u : 0u);
        if (got != seq_len) break;                        // kseq -2
        crf = (cs ? FQ_KEEP_CR_SEQ : 0u) | ((hc && cq <= k) ? FQ_KEEP_CR_QUAL : 0u);
        const uint32_t an = lower_u32(ats, nat, k + 1);
        const uint32_t stop = an < nat ? ats[an] : nlines;
        // lines between the record and the next header: kseq skips them to
        // the next '@' or '>' byte; followed when they hold neither
        if (GA[stop] != GA[k + 1]) break;                 // a header would start mid-line
        r = an < nat ? int32_t(an) : (eof ? ML_END : ML_MORE);
    } while (false);
    next[a] = r;
    jq[a] = j;
    kq[a] = k;
    slen[a] = sl;
    kcr[a] = crf;
}

// record r of the chain: header line, first sequence line, first quality line
__global__ void k_ml_records(const uint8_t *t, uint64_t len, const uint64_t *nl, uint32_t nlines,
                             const uint32_t *chain, uint64_t nrec, const uint32_t *ats, const uint32_t *jq,
                             const uint32_t *kq, const uint32_t *slen, const uint32_t *kcr,
                             fqz5_fastq_rec *recs, uint32_t *rec_size, uint64_t *ends) {
    const uint64_t r = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x;
    if (r >= nrec) return;
    const uint32_t a = chain[r], h = ats[a], j = jq[a], k = kq[a];
    const uint64_t s0 = h ? nl[h - 1] + 1 : 0, e0 = nl[h];
    fqz5_fastq_rec R;
    header(t, s0, e0, R);
    R.seq = e0 + 1 < len ? e0 + 1 : len;
    R.qual = nl[j] + 1 < len ? nl[j] + 1 : len;
    R.seq_len = slen[a];
    R.fasta = 2u | kcr[a];
    R.end = nl[k] + 1 < len ? nl[k] + 1 : len;
    if (recs) recs[r] = R;
    if (rec_size) rec_size[r] = R.name_len + 1 + 2 * R.seq_len;   // (:472)
    if (ends) ends[r] = R.end;
    (void)nlines;
}

// kseq's joined lines (kseq.h:194-198, :213): n kept bytes from text offset
// s on, every '\n' and a '\r' before a '\n' skipped.  One wave; sub: 33 for
// qualities.
__device__ void ml_copy(const uint8_t *t, uint64_t tlen, uint64_t s, uint32_t n, uint8_t *out,
                        uint8_t sub, bool keep_cr) {
    const uint32_t lane = threadIdx.x & 63;
    const uint64_t below = lane ? (~0ull >> (64 - lane)) : 0ull;
    uint32_t w = 0;
    if (keep_cr && n) {
        // the block's first kept byte is a lone-'\r' line's '\r' (kseq.h:141):
        // skip the empty lines before it, keep it, go on after its '\n'
        while (s < tlen && t[s] == '\n') s++;
        if (lane == 0) out[0] = uint8_t(uint8_t('\r') - sub);
        s += 2;
        w = 1;
    }
    for (uint64_t base = s; w < n && base < tlen; base += 64) {
        const uint64_t p = base + lane;
        const bool in = p < tlen;
        const uint8_t c = in ? t[p] : uint8_t('\n');
        const uint8_t c1 = p + 1 < tlen ? t[p + 1] : uint8_t(0);
        const bool keep = in && c != '\n' && !(c == '\r' && c1 == '\n');
        const uint64_t km = __builtin_amdgcn_ballot_w64(keep);
        const uint32_t at = w + uint32_t(__builtin_popcountll(km & below));
        if (keep && at < n) out[at] = uint8_t(c - sub);
        w += uint32_t(__builtin_popcountll(km));
    }
}

// per record of [a, b): name bytes (name [' ' comment] '\0') and bases
__global__ void k_fq_counts(const fqz5_fastq_rec *recs, uint64_t a, uint64_t n, uint32_t *nb,
                            uint32_t *sb) {
    const uint64_t k = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x;
    if (k >= n) return;
    const fqz5_fastq_rec R = recs[a + k];
    nb[k] = R.name_len + (R.comment_len ? 1 + R.comment_len : 0) + 1;
    sb[k] = R.seq_len;
}

// one wave per record: the names (name ' ' comment '\0'), the bases and the
// qualities - 33 (load_seqs_kseq, fqzcomp5.c:491-565)
__global__ void k_fq_gather(const uint8_t *t, const fqz5_fastq_rec *recs, uint64_t a, uint64_t n,
                            const uint32_t *noff, const uint32_t *soff, uint8_t *names,
                            uint8_t *seq, uint8_t *qual) {
    const uint64_t k = (uint64_t(blockIdx.x) * blockDim.x + threadIdx.x) / 64;
    const uint32_t lane = threadIdx.x & 63;
    if (k >= n) return;
    const fqz5_fastq_rec R = recs[a + k];
    uint8_t *o = names + noff[k];
    for (uint32_t i = lane; i < R.name_len; i += 64) o[i] = t[R.name + i];
    uint32_t w = R.name_len;
    if (R.comment_len) {
        if (lane == 0) o[w] = ' ';
        for (uint32_t i = lane; i < R.comment_len; i += 64) o[w + 1 + i] = t[R.comment + i];
        w += 1 + R.comment_len;
    }
    if (lane == 0) o[w] = 0;
    uint8_t *so = seq + soff[k];
    if (R.fasta == 1) {                               // lines joined (fa_seq)
        fa_seq(t, R.seq, R.qual, so);
        return;
    }
    uint8_t *qo = qual + soff[k];
    if ((R.fasta & 0xffu) == 2) {                     // wrapped FASTQ: lines joined
        ml_copy(t, R.end, R.seq, R.seq_len, so, 0, (R.fasta & FQ_KEEP_CR_SEQ) != 0);
        ml_copy(t, R.end, R.qual, R.seq_len, qo, 33, (R.fasta & FQ_KEEP_CR_QUAL) != 0);
        return;
    }
    for (uint32_t i = lane; i < R.seq_len; i += 64) {
        so[i] = t[R.seq + i];
        qo[i] = uint8_t(t[R.qual + i] - 33);
    }
}

// READ2 flags (fqzcomp5.c:518-527): the name (with its comment) ends in
// "/2", or equals the previous name of the block
__global__ void k_fq_flags(const fqz5_fastq_rec *recs, uint64_t a, uint64_t n, const uint8_t *names,
                           const uint32_t *noff, const uint32_t *nb, uint32_t *flags) {
    const uint64_t k = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x;
    if (k >= n) return;
    const uint8_t *s = names + noff[k];
    const uint32_t l = nb[k] - 1;                     // without the '\0'
    uint32_t f = 0;
    if (recs[a + k].name_len > 1 && l >= 2 && s[l - 1] == '2' && s[l - 2] == '/') f = 128;
    if (k > 0 && nb[k - 1] == nb[k]) {
        const uint8_t *q = names + noff[k - 1];
        uint32_t i = 0;
        while (i < l && s[i] == q[i]) i++;
        if (i == l) f = 128;
    }
    flags[k] = f;
}

// output_fastq (fqzcomp5.c:3441-3480): '@' name '\n' seq '\n' '+' [name] '\n'
// qual+33 '\n'; without qualities output_fasta (:3503-3517): '>' name '\n'
// seq '\n'.  One wave per record.
__global__ void k_fq_format(const uint8_t *names, const uint64_t *zpos, const uint8_t *seq,
                            const uint8_t *qual, const uint64_t *soff, const uint32_t *lens,
                            const uint64_t *ooff, uint64_t n, int plus_name, uint8_t *out) {
    const uint64_t k = (uint64_t(blockIdx.x) * blockDim.x + threadIdx.x) / 64;
    const uint32_t lane = threadIdx.x & 63;
    if (k >= n) return;
    const uint64_t ns = k ? zpos[k - 1] + 1 : 0;
    const uint32_t nl = uint32_t(zpos[k] - ns), L = lens[k];
    uint8_t *o = out + ooff[k];
    if (lane == 0) o[0] = qual ? '@' : '>';
    for (uint32_t i = lane; i < nl; i += 64) o[1 + i] = names[ns + i];
    uint64_t w = 1 + nl;
    if (lane == 0) o[w] = '\n';
    w++;
    const uint8_t *sp = seq + soff[k], *qp = qual + soff[k];
    for (uint32_t i = lane; i < L; i += 64) o[w + i] = sp[i];
    w += L;
    if (!qual) {
        if (lane == 0) o[w] = '\n';
        return;
    }
    if (lane == 0) {
        o[w] = '\n';
        o[w + 1] = '+';
    }
    w += 2;
    if (plus_name) {
        for (uint32_t i = lane; i < nl; i += 64) o[w + i] = names[ns + i];
        w += nl;
    }
    if (lane == 0) o[w] = '\n';
    w++;
    for (uint32_t i = lane; i < L; i += 64) o[w + i] = uint8_t(qp[i] + 33);
    w += L;
    if (lane == 0) o[w] = '\n';
}

dim3 grid_for(uint64_t n, uint32_t per) { return dim3(uint32_t((n + per - 1) / per ? (n + per - 1) / per : 1)); }

// every `ch` position of d_text[0..len) into a device array (arena); returns it
uint64_t *find_delims(GpuCtx &g, const uint8_t *d_text, uint64_t len, uint8_t ch, uint64_t *count) {
    const uint64_t tiles = (len + FQ_TILE - 1) / FQ_TILE;
    if (tiles == 0) { *count = 0; return nullptr; }
    if (tiles >= (1ull << 31)) throw GpuError("fastq: text too large");
    uint32_t *cnt = g.arena.alloc_n<uint32_t>(tiles + 1);
    uint32_t *off = g.arena.alloc_n<uint32_t>(tiles + 1);
    hipLaunchKernelGGL(k_delim_count, dim3(uint32_t(tiles)), dim3(FQ_TPB), 0, g.stream, d_text, len,
                       ch, cnt);
    FQZ5_HIP(hipGetLastError());
    g.memset0(cnt + tiles, 4);
    size_t tb = 0;
    FQZ5_HIP(hipcub::DeviceScan::ExclusiveSum(nullptr, tb, cnt, off, int(tiles + 1), g.stream));
    void *tmp = g.arena.alloc_n<uint8_t>(tb);
    FQZ5_HIP(hipcub::DeviceScan::ExclusiveSum(tmp, tb, cnt, off, int(tiles + 1), g.stream));
    uint32_t total = 0;
    g.download(&total, off + tiles, 1);
    g.sync();
    *count = total;
    uint64_t *pos = g.arena.alloc_n<uint64_t>(size_t(total) + 1);
    hipLaunchKernelGGL(k_delim_write, dim3(uint32_t(tiles)), dim3(FQ_TPB), 0, g.stream, d_text, len,
                       ch, off, pos);
    FQZ5_HIP(hipGetLastError());
    return pos;
}

template <class T> void excl_sum(GpuCtx &g, const T *in, T *out, uint64_t n) {
    size_t tb = 0;
    FQZ5_HIP(hipcub::DeviceScan::ExclusiveSum(nullptr, tb, in, out, int(n), g.stream));
    void *tmp = g.arena.alloc_n<uint8_t>(tb ? tb : 1);
    FQZ5_HIP(hipcub::DeviceScan::ExclusiveSum(tmp, tb, in, out, int(n), g.stream));
}

// Wrapped-FASTQ records of the text whose lines end at lines[0..nlines)
// (see k_ml_cand): the records into d_recs (device, may be NULL) with their
// sizes (h_rec_size, host, may be NULL) and text ends (h_ends, may be NULL);
// returns their number.  eof: the text ends the input (else a record it cuts
// off is left out).  Throws on text kseq would not read as these records.
uint64_t ml_index(GpuCtx &g, const uint8_t *d_text, uint64_t len, const uint64_t *lines, uint64_t nlines,
                  int eof, fqz5_fastq_rec *d_recs, uint64_t max_rec, uint32_t *h_rec_size,
                  std::vector<uint64_t> *h_ends) {
    if (nlines >= (1ull << 31)) throw GpuError("fastq: too many lines");
    const uint32_t n = uint32_t(nlines);
    if (!n) return 0;
    uint8_t *cls = g.arena.alloc_n<uint8_t>(size_t(n) + 1);
    uint32_t *ls = g.arena.alloc_n<uint32_t>(size_t(n) + 1);
    uint32_t *fa = g.arena.alloc_n<uint32_t>(size_t(n) + 1), *fs = g.arena.alloc_n<uint32_t>(size_t(n) + 1);
    uint32_t *fc = g.arena.alloc_n<uint32_t>(size_t(n) + 1);
    uint32_t *fg = g.arena.alloc_n<uint32_t>(size_t(n) + 1);
    hipLaunchKernelGGL(k_ml_lines, grid_for(n, 256), dim3(256), 0, g.stream, d_text, lines, nlines, cls, ls,
                       fa, fs, fc, fg);
    FQZ5_HIP(hipGetLastError());
    g.memset0(ls + n, 4);
    g.memset0(fa + n, 4);
    g.memset0(fs + n, 4);
    g.memset0(fc + n, 4);
    g.memset0(fg + n, 4);
    // P: kept bytes before each line (u64: widened first)
    uint64_t *ls64 = g.arena.alloc_n<uint64_t>(size_t(n) + 1);
    uint64_t *P = g.arena.alloc_n<uint64_t>(size_t(n) + 2);
    hipLaunchKernelGGL(k_widen, grid_for(uint64_t(n) + 1, 256), dim3(256), 0, g.stream, ls, ls64, uint64_t(n) + 1);
    FQZ5_HIP(hipGetLastError());
    excl_sum(g, ls64, P, uint64_t(n) + 1);
    uint32_t *pa = g.arena.alloc_n<uint32_t>(size_t(n) + 1), *ps = g.arena.alloc_n<uint32_t>(size_t(n) + 1);
    uint32_t *pc = g.arena.alloc_n<uint32_t>(size_t(n) + 1);
    excl_sum(g, fa, pa, uint64_t(n) + 1);
    excl_sum(g, fs, ps, uint64_t(n) + 1);
    excl_sum(g, fc, pc, uint64_t(n) + 1);
    uint32_t *GA = g.arena.alloc_n<uint32_t>(size_t(n) + 1);
    excl_sum(g, fg, GA, uint64_t(n) + 1);
    uint32_t cnt[3] = {0, 0, 0};
    g.download(&cnt[0], pa + n, 1);
    g.download(&cnt[1], ps + n, 1);
    g.download(&cnt[2], pc + n, 1);
    g.sync();
    const uint32_t nat = cnt[0], nst = cnt[1], ncr = cnt[2];
    uint32_t *ats = g.arena.alloc_n<uint32_t>(size_t(nat) + 1), *stops = g.arena.alloc_n<uint32_t>(size_t(nst) + 1);
    uint32_t *crs = g.arena.alloc_n<uint32_t>(size_t(ncr) + 1);
    hipLaunchKernelGGL(k_ml_scatter, grid_for(n, 256), dim3(256), 0, g.stream, fa, pa, uint64_t(n), ats);
    hipLaunchKernelGGL(k_ml_scatter, grid_for(n, 256), dim3(256), 0, g.stream, fs, ps, uint64_t(n), stops);
    hipLaunchKernelGGL(k_ml_scatter, grid_for(n, 256), dim3(256), 0, g.stream, fc, pc, uint64_t(n), crs);
    FQZ5_HIP(hipGetLastError());
    if (!nat) {                            // no header: only empty lines are no records
        uint64_t tot = 0;
        g.download(&tot, P + n, 1);
        g.sync();
        if (tot) throw GpuError("fastq: text without a FASTQ header line");
        return 0;
    }
    int32_t *nx = g.arena.alloc_n<int32_t>(nat);
    uint32_t *jq = g.arena.alloc_n<uint32_t>(nat), *kq = g.arena.alloc_n<uint32_t>(nat);
    uint32_t *sl = g.arena.alloc_n<uint32_t>(nat), *kc = g.arena.alloc_n<uint32_t>(nat);
    hipLaunchKernelGGL(k_ml_cand, grid_for(nat, 256), dim3(256), 0, g.stream, cls, P, crs, ncr, GA, n, ats,
                       nat, stops, nst, eof, nx, jq, kq, sl, kc);
    FQZ5_HIP(hipGetLastError());
    std::vector<int32_t> hn(nat);
    uint32_t a0 = 0, before = 0;
    g.download(hn.data(), nx, nat);
    g.download(&a0, ats, 1);
    g.sync();
    g.download(&before, GA + a0, 1);
    g.sync();
    // lines before the first header: kseq skips them to the first '@' or
    // '>' byte (kseq.h:180-186); followed when they hold neither
    if (before) throw GpuError("fastq: text before the first FASTQ header line holds '@' or '>'");
    // the records: the chain of next-header links from the first '@' line
    std::vector<uint32_t> chain;
    for (uint32_t a = 0;;) {
        chain.push_back(a);
        const int32_t r = hn[a];
        if (r >= 0) {
            if (uint32_t(r) <= a) throw GpuError("fastq: record chain does not advance");
            a = uint32_t(r);
            continue;
        }
        if (r == ML_END) break;
        if (r == ML_MORE && !eof) {
            chain.pop_back();
            break;
        }
        char msg[160];
        std::snprintf(msg, sizeof msg, "fastq: record %zu is not a FASTQ record kseq reads (a record without "
                      "a '+' line, qualities longer than the bases, or '@' / '>' inside the bytes after it)",
                      chain.size() - 1);
        throw GpuError(msg);
    }
    const uint64_t nrec = chain.size();
    if (d_recs && nrec > max_rec) throw GpuError("fastq: more records than max_rec");
    if (!nrec) return 0;
    const uint32_t *d_chain = g.upload(chain);
    uint32_t *rs = h_rec_size ? g.arena.alloc_n<uint32_t>(nrec) : nullptr;
    uint64_t *ends = h_ends ? g.arena.alloc_n<uint64_t>(nrec) : nullptr;
    hipLaunchKernelGGL(k_ml_records, grid_for(nrec, 256), dim3(256), 0, g.stream, d_text, len, lines, n, d_chain,
                       nrec, ats, jq, kq, sl, kc, d_recs, rs, ends);
    FQZ5_HIP(hipGetLastError());
    if (rs) g.download(h_rec_size, rs, nrec);
    if (ends) {
        h_ends->resize(size_t(nrec));
        g.download(h_ends->data(), ends, nrec);
    }
    g.sync();
    return nrec;
}

// lines of d_text (newline positions, plus the text end when the text does
// not end in '\n' and `eof`); *nlines receives their count
uint64_t *text_lines(GpuCtx &g, const uint8_t *d_text, uint64_t len, bool eof, uint64_t *nlines) {
    uint64_t nn = 0;
    uint64_t *nl = find_delims(g, d_text, len, '\n', &nn);
    uint8_t last = '\n';
    if (len) {
        g.download(&last, d_text + len - 1, 1);
        g.sync();
    }
    *nlines = nn;
    if (!(eof && len && last != '\n')) return nl;
    uint64_t *lines = g.arena.alloc_n<uint64_t>(size_t(nn) + 1);
    if (nn) FQZ5_HIP(hipMemcpyAsync(lines, nl, nn * 8, hipMemcpyDeviceToDevice, g.stream));
    uint64_t *st = reinterpret_cast<uint64_t *>(g.staging.alloc(8));
    *st = len;
    FQZ5_HIP(hipMemcpyAsync(lines + nn, st, 8, hipMemcpyHostToDevice, g.stream));
    *nlines = nn + 1;
    return lines;
}

// 4-line FASTQ check of the complete groups of lines: records into d_recs
// (scratch when NULL); true when every group is a 4-line record and (eof)
// the lines after them are empty
bool four_line(GpuCtx &g, const uint8_t *d_text, const uint64_t *lines, uint64_t nlines, bool eof,
               fqz5_fastq_rec *d_recs, uint32_t *rs, uint64_t *n4out) {
    const uint64_t n4 = nlines / 4;
    *n4out = n4;
    if (eof && nlines % 4) {
        std::vector<uint64_t> tail(size_t(nlines % 4) + 1);
        const uint64_t first = n4 * 4;
        g.download(tail.data() + 1, lines + first, nlines - first);
        if (first) g.download(tail.data(), lines + first - 1, 1);
        g.sync();
        uint64_t prev = first ? tail[0] : uint64_t(-1);
        for (uint64_t k = 1; k <= nlines - first; k++) {
            if (tail[k] != prev + 1) return false;
            prev = tail[k];
        }
    }
    if (!n4) return true;
    if (!d_recs) d_recs = g.arena.alloc_n<fqz5_fastq_rec>(size_t(n4));
    if (!rs) rs = g.arena.alloc_n<uint32_t>(size_t(n4));
    int32_t *st = g.arena.alloc_n<int32_t>(1);
    g.memset0(st, 4);
    hipLaunchKernelGGL(k_fq_records, grid_for(n4, 256), dim3(256), 0, g.stream, d_text, lines, n4, d_recs, rs, st);
    FQZ5_HIP(hipGetLastError());
    int32_t status = 0;
    g.download(&status, st, 1);
    g.sync();
    return status >= 0;
}

}  // namespace
}  // namespace fqz5

using namespace fqz5;

extern "C" {

int fqz5_fastq_index(const uint8_t *d_text, uint64_t len, fqz5_fastq_rec *d_recs,
                     uint64_t max_rec, uint64_t *nrec, uint32_t *h_rec_size) {
    GpuCtx *gp = nullptr;
    try {
        GpuCtx &g = gpu();
        gp = &g;
        *nrec = 0;
        uint64_t nn = 0;
        uint64_t *nl = find_delims(g, d_text, len, '\n', &nn);
        // a last line without '\n' ends at the text end (kseq reads to EOF)
        uint8_t last = '\n';
        if (len) {
            g.download(&last, d_text + len - 1, 1);
            g.sync();
        }
        // FASTA when the text starts with '>' (a record without a quality
        // line; the reference decides on the block's first record, :575-578)
        uint8_t first_byte = 0;
        if (len) g.download(&first_byte, d_text, 1);
        g.sync();
        const bool fasta = first_byte == '>';
        uint64_t *lines = nl;
        uint64_t nlines = nn;
        if (len && last != '\n') {
            lines = g.arena.alloc_n<uint64_t>(size_t(nn) + 1);
            if (nn) FQZ5_HIP(hipMemcpyAsync(lines, nl, nn * 8, hipMemcpyDeviceToDevice, g.stream));
            const uint64_t e = len;
            uint64_t *st = reinterpret_cast<uint64_t *>(g.staging.alloc(8));
            *st = e;
            FQZ5_HIP(hipMemcpyAsync(lines + nn, st, 8, hipMemcpyHostToDevice, g.stream));
            nlines = nn + 1;
        }
        int32_t *st = g.arena.alloc_n<int32_t>(1);
        const int32_t ok = 0;
        FQZ5_HIP(hipMemcpyAsync(st, &ok, 4, hipMemcpyHostToDevice, g.stream));
        uint64_t n4 = 0;
        uint32_t *rs = nullptr;
        if (fasta) {
            // records = header lines (any number of sequence lines each)
            uint32_t *hdr = g.arena.alloc_n<uint32_t>(size_t(nlines) + 1);
            uint32_t *pos = g.arena.alloc_n<uint32_t>(size_t(nlines) + 1);
            if (nlines >= (1ull << 31)) throw GpuError("fasta: too many lines");
            if (nlines)
                hipLaunchKernelGGL(k_fa_lines, grid_for(nlines, 256), dim3(256), 0, g.stream, d_text, lines,
                                   nlines, hdr, st);
            g.memset0(hdr + nlines, 4);
            excl_sum(g, hdr, pos, nlines + 1);
            uint32_t nh = 0;
            g.download(&nh, pos + nlines, 1);
            g.sync();
            n4 = nh;
            if (n4 > max_rec) throw GpuError("fastq: more records than max_rec");
            uint64_t *hl = g.arena.alloc_n<uint64_t>(size_t(n4) + 1);
            rs = g.arena.alloc_n<uint32_t>(size_t(n4) + 1);
            if (nlines)
                hipLaunchKernelGGL(k_fa_scatter, grid_for(nlines, 256), dim3(256), 0, g.stream, hdr, pos,
                                   nlines, hl);
            if (n4)
                hipLaunchKernelGGL(k_fa_records, grid_for(n4 * 64, 256), dim3(256), 0, g.stream, d_text,
                                   len, lines, hl, n4, d_recs, rs);
        } else {
            // trailing empty lines (kseq skips to the next header) are ignored
            n4 = nlines / 4;
            if (nlines % 4) {
                std::vector<uint64_t> tail(size_t(nlines % 4) + 1);
                const uint64_t first = n4 * 4;
                g.download(tail.data() + 1, lines + first, nlines - first);
                if (first) g.download(tail.data(), lines + first - 1, 1);
                g.sync();
                uint64_t prev = first ? tail[0] : uint64_t(-1);
                for (uint64_t k = 1; k <= nlines - first; k++) {
                    if (tail[k] != prev + 1) throw GpuError("fastq: not 4-line FASTQ (stray lines at the end)");
                    prev = tail[k];
                }
            }
            if (n4 > max_rec) throw GpuError("fastq: more records than max_rec");
            rs = g.arena.alloc_n<uint32_t>(size_t(n4) + 1);
            if (n4)
                hipLaunchKernelGGL(k_fq_records, grid_for(n4, 256), dim3(256), 0, g.stream, d_text, lines,
                                   n4, d_recs, rs, st);
        }
        FQZ5_HIP(hipGetLastError());
        int32_t status = 0;
        g.download(&status, st, 1);
        if (h_rec_size && n4) g.download(h_rec_size, rs, n4);
        g.sync();
        if (status < 0) {
            char msg[128];
            std::snprintf(msg, sizeof msg, fasta ? "fasta: line %lld starts a FASTQ record or precedes the first header"
                                                 : "fastq: record %lld is not a 4-line FASTQ record",
                          static_cast<long long>(-1 - int64_t(status)));
            throw GpuError(msg);
        }
        *nrec = n4;
        g.reset();
        return fasta ? 1 : 0;
    } catch (const std::exception &e) {
        fqz5_set_error(e.what());
        try { if (gp) gp->reset(); } catch (...) {}
        return -1;
    }
}

int fqz5_fastq_index_any(const uint8_t *d_text, uint64_t len, fqz5_fastq_rec *d_recs,
                         uint64_t max_rec, uint64_t *nrec, uint32_t *h_rec_size) {
    const int r = fqz5_fastq_index(d_text, len, d_recs, max_rec, nrec, h_rec_size);
    if (r >= 0) return r;
    // not FASTA, not 4-line FASTQ: kseq's wrapped records
    GpuCtx *gp = nullptr;
    try {
        GpuCtx &g = gpu();
        gp = &g;
        uint8_t first_byte = 0;
        if (len) {
            g.download(&first_byte, d_text, 1);
            g.sync();
        }
        if (first_byte == '>') return -1;       // (FASTA's own error stands)
        uint64_t nlines = 0;
        const uint64_t *lines = text_lines(g, d_text, len, true, &nlines);
        *nrec = ml_index(g, d_text, len, lines, nlines, 1, d_recs, max_rec, h_rec_size, nullptr);
        g.reset();
        return 0;
    } catch (const std::exception &e) {
        fqz5_set_error(e.what());
        try { if (gp) gp->reset(); } catch (...) {}
        return -1;
    }
}

int fqz5_fastq_record_ends(const uint8_t *d_text, uint64_t len, int eof, uint64_t *h_ends,
                           uint64_t max_ends, uint64_t *n_ends) {
    GpuCtx *gp = nullptr;
    try {
        GpuCtx &g = gpu();
        gp = &g;
        *n_ends = 0;
        uint64_t nlines = 0;
        const uint64_t *lines = text_lines(g, d_text, len, eof != 0, &nlines);
        std::vector<uint64_t> ends;
        uint64_t n4 = 0;
        if (four_line(g, d_text, lines, nlines, eof != 0, nullptr, nullptr, &n4)) {
            // record r ends after line 4r + 3 (load_seqs_kseq's 4-line records)
            ends.resize(size_t(n4));
            if (n4) {
                uint64_t *e = g.arena.alloc_n<uint64_t>(size_t(n4));
                hipLaunchKernelGGL(k_ends4, grid_for(n4, 256), dim3(256), 0, g.stream, lines, n4, len, e);
                FQZ5_HIP(hipGetLastError());
                g.download(ends.data(), e, n4);
                g.sync();
            }
        } else {
            ml_index(g, d_text, len, lines, nlines, eof, nullptr, 0, nullptr, &ends);
        }
        if (eof && len && (ends.empty() || ends.back() != len)) ends.push_back(len);
        if (ends.size() > max_ends) throw GpuError("fastq: more records than max_ends");
        std::memcpy(h_ends, ends.data(), ends.size() * 8);
        *n_ends = ends.size();
        g.reset();
        return 0;
    } catch (const std::exception &e) {
        fqz5_set_error(e.what());
        try { if (gp) gp->reset(); } catch (...) {}
        return -1;
    }
}

int fqz5_fastq_blocks(const uint32_t *rec_size, uint64_t nrec, uint32_t blk_size, uint64_t *first,
                      int max_blocks) {
    // load_seqs_kseq (fqzcomp5.c:471-479): a record that would take a
    // non-empty block past blk_size starts the next one
    int nb = 0;
    uint64_t total = 0;
    for (uint64_t r = 0; r < nrec; r++) {
        if (r == 0 || (total > 0 && total + rec_size[r] > blk_size)) {
            if (nb >= max_blocks) return -1;
            first[nb++] = r;
            total = 0;
        }
        total += rec_size[r];
    }
    if (nb > max_blocks) return -1;
    first[nb] = nrec;
    return nb;
}

int fqz5_fastq_gather(const uint8_t *d_text, const fqz5_fastq_rec *d_recs, uint64_t a, uint64_t b,
                      uint8_t *d_names, uint8_t *d_seq, uint8_t *d_qual, uint32_t *h_len,
                      uint32_t *h_flag, uint64_t *sizes) {
    GpuCtx *gp = nullptr;
    try {
        GpuCtx &g = gpu();
        gp = &g;
        const uint64_t n = b > a ? b - a : 0;
        if (n >= (1ull << 31)) throw GpuError("fastq: block too large");
        uint32_t *nb = g.arena.alloc_n<uint32_t>(size_t(n) + 1);
        uint32_t *sb = g.arena.alloc_n<uint32_t>(size_t(n) + 1);
        uint32_t *noff = g.arena.alloc_n<uint32_t>(size_t(n) + 1);
        uint32_t *soff = g.arena.alloc_n<uint32_t>(size_t(n) + 1);
        if (n) hipLaunchKernelGGL(k_fq_counts, grid_for(n, 256), dim3(256), 0, g.stream, d_recs, a, n, nb, sb);
        g.memset0(nb + n, 4);
        g.memset0(sb + n, 4);
        excl_sum(g, nb, noff, n + 1);
        excl_sum(g, sb, soff, n + 1);
        uint32_t tot[2];
        g.download(&tot[0], noff + n, 1);
        g.download(&tot[1], soff + n, 1);
        g.sync();
        sizes[0] = tot[0];
        sizes[1] = tot[1];
        sizes[2] = d_qual ? tot[1] : 0;
        if (d_names && d_seq && n) {
            hipLaunchKernelGGL(k_fq_gather, grid_for(n * 64, 256), dim3(256), 0, g.stream, d_text, d_recs,
                               a, n, noff, soff, d_names, d_seq, d_qual);
            FQZ5_HIP(hipGetLastError());
            if (h_flag) {
                uint32_t *fl = g.arena.alloc_n<uint32_t>(size_t(n));
                hipLaunchKernelGGL(k_fq_flags, grid_for(n, 256), dim3(256), 0, g.stream, d_recs, a, n,
                                   d_names, noff, nb, fl);
                FQZ5_HIP(hipGetLastError());
                g.download(h_flag, fl, n);
            }
            if (h_len) g.download(h_len, sb, n);
        }
        g.reset();
        return 0;
    } catch (const std::exception &e) {
        fqz5_set_error(e.what());
        try { if (gp) gp->reset(); } catch (...) {}
        return -1;
    }
}

static int format_impl(const uint8_t *d_names, uint64_t name_len, const uint8_t *d_seq,
                       const uint8_t *d_qual, const uint32_t *h_len, uint64_t nrec, int plus_name,
                       uint8_t *d_out, uint64_t out_cap, uint64_t *out_len, uint64_t *r1_len) {
    GpuCtx *gp = nullptr;
    try {
        GpuCtx &g = gpu();
        gp = &g;
        uint64_t nz = 0;
        uint64_t *z = find_delims(g, d_names, name_len, 0, &nz);
        if (nz < nrec) throw GpuError("fastq_format: fewer names than records");
        std::vector<uint64_t> hz(size_t(nrec) + 1), ooff(size_t(nrec) + 1), soff(size_t(nrec) + 1);
        if (nrec) g.download(hz.data(), z, nrec);
        g.sync();
        uint64_t o = 0, s = 0, prev = uint64_t(-1);
        for (uint64_t k = 0; k < nrec; k++) {
            const uint64_t nl = hz[k] - (prev + 1);
            ooff[k] = o;
            soff[k] = s;
            o += d_qual ? 1 + nl + 1 + h_len[k] + 2 + (plus_name ? nl : 0) + 1 + h_len[k] + 1
                        : 1 + nl + 1 + h_len[k] + 1;
            s += h_len[k];
            prev = hz[k];
        }
        if (r1_len) {
            // output_fastq_deinterleaved (fqzcomp5.c:3612-3676): even records
            // to the first text, odd ones to the second, placed after it
            uint64_t t1 = 0;
            for (uint64_t k = 0; k < nrec; k += 2) t1 += (k + 1 < nrec ? ooff[k + 1] : o) - ooff[k];
            uint64_t o1 = 0, o2 = t1;
            for (uint64_t k = 0; k < nrec; k++) {
                const uint64_t sz = (k + 1 < nrec ? ooff[k + 1] : o) - ooff[k];
                uint64_t &w = (k & 1) ? o2 : o1;
                ooff[k] = w;
                w += sz;
            }
            *r1_len = t1;
        }
        *out_len = o;
        if (!d_out) { g.reset(); return 0; }
        if (o > out_cap) throw GpuError("fastq_format: output larger than out_cap");
        const uint64_t *d_oo = g.upload(ooff.data(), nrec);
        const uint64_t *d_so = g.upload(soff.data(), nrec);
        const uint32_t *d_l = g.upload(h_len, nrec);
        if (nrec)
            hipLaunchKernelGGL(k_fq_format, grid_for(nrec * 64, 256), dim3(256), 0, g.stream, d_names, z,
                               d_seq, d_qual, d_so, d_l, d_oo, nrec, plus_name, d_out);
        FQZ5_HIP(hipGetLastError());
        g.reset();
        return 0;
    } catch (const std::exception &e) {
        fqz5_set_error(e.what());
        try { if (gp) gp->reset(); } catch (...) {}
        return -1;
    }
}

int fqz5_fastq_format(const uint8_t *d_names, uint64_t name_len, const uint8_t *d_seq,
                      const uint8_t *d_qual, const uint32_t *h_len, uint64_t nrec, int plus_name,
                      uint8_t *d_out, uint64_t out_cap, uint64_t *out_len) {
    return format_impl(d_names, name_len, d_seq, d_qual, h_len, nrec, plus_name, d_out, out_cap,
                       out_len, nullptr);
}

int fqz5_fastq_format_pairs(const uint8_t *d_names, uint64_t name_len, const uint8_t *d_seq,
                            const uint8_t *d_qual, const uint32_t *h_len, uint64_t nrec,
                            int plus_name, uint8_t *d_out, uint64_t out_cap, uint64_t *out_len,
                            uint64_t *r1_len) {
    uint64_t dummy = 0;
    return format_impl(d_names, name_len, d_seq, d_qual, h_len, nrec, plus_name, d_out, out_cap,
                       out_len, r1_len ? r1_len : &dummy);
}

}  // extern "C"
