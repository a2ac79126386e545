/*
 * fqz5_mi355x.h — C-ABI of the MI355X-native fqzcomp5 block codec.
 *
 * Part 1 re-exports the htscodecs entry points that fqzcomp5 binds, with
 * identical names, argument meaning, ownership and error behaviour, so a
 * fqzcomp5 build links this library in place of htscodecs' CPU objects:
 *   rANS 4x16/32x16  /root/reference/htscodecs/rANS_static4x16.h:41-66
 *   fqzcomp_qual     /root/reference/htscodecs/fqzcomp_qual.h:59-170
 *                    (the fork's ABI: fqz_slice carries the sequences)
 *   arith_dynamic    /root/reference/htscodecs/arith_dynamic.h:41-54
 *
 * Part 2 is the batched, device-resident API used by the block codec and
 * the benchmark: many streams per call, inputs and outputs in HBM.
 *
 * Every entry point runs its byte work on the GPU.  There is no CPU path:
 * without a visible HIP device the calls fail (NULL / negative status) and
 * fqz5_last_error() says why.
 */
#ifndef FQZ5_MI355X_H
#define FQZ5_MI355X_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- Part 1: htscodecs drop-in (rANS_static4x16.h:41-66) -------------- */

/* Replaces rans_compress_bound_4x16 (rANS_static4x16pr.c:93). */
unsigned int rans_compress_bound_4x16(unsigned int size, int order);

/* Replaces rans_compress_to_4x16 (rANS_static4x16pr.c:1224).
 * out == NULL: a buffer of rans_compress_bound_4x16() bytes is malloc()ed
 * and returned (caller free()s).  Otherwise *out_size is the capacity on
 * entry and the used size on return.  NULL and *out_size = 0 on failure. */
unsigned char *rans_compress_to_4x16(unsigned char *in, unsigned int in_size,
                                     unsigned char *out, unsigned int *out_size,
                                     int order);

/* Replaces rans_compress_4x16 (rANS_static4x16pr.c:1602). */
unsigned char *rans_compress_4x16(unsigned char *in, unsigned int in_size,
                                  unsigned int *out_size, int order);

/* Replaces rans_uncompress_to_4x16 (rANS_static4x16pr.c:1607). */
unsigned char *rans_uncompress_to_4x16(unsigned char *in, unsigned int in_size,
                                       unsigned char *out, unsigned int *out_size);

/* Replaces rans_uncompress_4x16 (rANS_static4x16pr.c:1896). */
unsigned char *rans_uncompress_4x16(unsigned char *in, unsigned int in_size,
                                    unsigned int *out_size);

/* Replaces rans_set_cpu (rANS_static4x16pr.c:1212).  Accepted and ignored:
 * the GPU kernels produce the same bytes as every reference CPU variant. */
void rans_set_cpu(int opts);

/* ---- fqzcomp_qual (htscodecs/fqzcomp_qual.h) -------------------------- */

#define FQZ_FREVERSE 16          /* fqzcomp_qual.h:37 */
#define FQZ_FREAD2 128           /* fqzcomp_qual.h:38 */
#define FQZ_VERS 5

/* fqzcomp_qual.h:59-64 (fork ABI): per-record lengths, flags (READ2 /
 * REVERSE; bits 16+ are used as selectors during fqz_compress) and the
 * record sequences (for sequence-context strategies, may be NULL). */
typedef struct {
    int num_records;
    uint32_t *len;
    uint32_t *flags;
    unsigned char **seq;
} fqz_slice;

/* fqzcomp_qual.h:92-139: one parameter block / the global parameters. */
typedef struct {
    uint16_t context;
    unsigned int pflags;
    unsigned int do_sel, do_dedup, store_qmap, fixed_len;
    unsigned char use_qtab, use_dtab, use_ptab;
    unsigned int qbits, qloc;
    unsigned int pbits, ploc;
    unsigned int dbits, dloc;
    unsigned int sbits, sloc;
    unsigned int bbits, bloc, boff;
    int max_sym, nsym, max_sel;
    unsigned int qmap[256];
    unsigned int qtab[256];
    unsigned int ptab[1024];
    unsigned int dtab[256];
    int qshift;
    int pshift;
    int dshift;
    int sshift;
    unsigned int qmask;
    int do_r2, do_qa;
} fqz_param;

typedef struct {
    int vers;
    unsigned int gflags;
    int nparam;
    int max_sel;
    unsigned int stab[256];
    int max_sym;
    fqz_param *p;
} fqz_gparams;

/* Replaces fqz_compress (fqzcomp_qual.c:1636).  Encodes in_size quality
 * bytes (values q-33) of s->num_records records.  Like the reference it
 * may rewrite s->len[] to fit in_size and uses the top 16 bits of
 * s->flags[] as selectors while running (cleared on return).  gp == NULL
 * picks parameters from the data (strat 0..4); a caller-supplied gp is used
 * as is (and, as in the reference, its position / delta tables are
 * shifted in place).  Returns a malloc()ed stream (caller frees), NULL on
 * failure. */
char *fqz_compress(int vers, fqz_slice *s, char *in, size_t in_size,
                   size_t *out_size, int strat, fqz_gparams *gp);

/* Replaces fqz_decompress (fqzcomp_qual.c:1642).  lengths[0..nlengths)
 * receive the record lengths; s may carry the decoded sequences for
 * sequence-context streams.  malloc()ed result, NULL on failure. */
char *fqz_decompress(char *in, size_t in_size, size_t *out_size,
                     int *lengths, int nlengths, fqz_slice *s);

/* ---- sequence context model (fqzcomp5.c:1073-1406) --------------------- */

/* Replaces encode_seq (fqzcomp5.c:1073): the SEQ10 .. SEQ14B coder of a
 * sequence section (ctx_size 10..14 in fqzcomp5; 1..14 here), len[] the
 * record lengths whose starts reset the k-mer contexts.  Same bytes as the
 * reference; NULL when the records run out before the data (as the
 * reference) or on a device error.  malloc()ed result, caller frees. */
char *fqz5_seq_encode(unsigned char *in, unsigned int in_size, unsigned int *len,
                      int nrecords, int both_strands, int ctx_size,
                      unsigned int *out_size);

/* Replaces decode_seq (fqzcomp5.c:1272): out_size bytes from a stream of
 * fqz5_seq_encode / encode_seq.  NULL on a damaged stream. */
char *fqz5_seq_decode(unsigned char *in, unsigned int in_size, unsigned int *len,
                      int nrecords, int both_strands, int ctx_size,
                      unsigned int out_size);

/* ---- the same decoders on a host core (host_dec.cpp) ------------------- */

/* fqz_decompress and fqz5_seq_decode on the calling thread's host core:
 * same arguments, same bytes, same NULL cases.  One block is one dependent
 * chain, which one host core runs 5-15x faster than one GPU wave; the block
 * decoder uses them for its adaptive-model sections when
 * fqz5_set_host_decode asks for it. */
char *fqz5_fqz_decompress_host(char *in, size_t in_size, size_t *out_size,
                               int *lengths, int nlengths, fqz_slice *s);
char *fqz5_seq_decode_host(unsigned char *in, unsigned int in_size, unsigned int *len,
                           int nrecords, int both_strands, int ctx_size,
                           unsigned int out_size);

/* Where fqz5_decode_sections (fqz5_block.h) runs the adaptive-model chains
 * (fqz quality sections, SEQ10..SEQ14B sequence sections): 0 = on the GPU,
 * 1 = on host cores (up to $FQZ5_HOST_THREADS threads) beside the GPU's
 * rANS, LZP and name work, 2 = each chain where its measured cost finishes
 * the call soonest (the default; $FQZ5_HOST_DECODE overrides it); 3 =
 * every other chain on host cores (tests of the mixed placement).  Output
 * bytes do not depend on it.  Returns the previous setting. */
int fqz5_set_host_decode(int mode);
/* The host threads of the library's pools: this rank's share of the cores
 * (the affinity mask / $LOCAL_WORLD_SIZE, capped by $OMP_NUM_THREADS and 16;
 * $FQZ5_HOST_THREADS overrides). */
int fqz5_host_threads(void);
/* The host-buffer encoder's trial batches (rans_compress_4x16 with a
 * callee-allocated output): out3[0] calls taken by that path, out3[1] calls
 * answered with an output a batch coded ahead, out3[2] batches of more than
 * one order.  $FQZ5_NO_TRIAL_BATCH turns the path off. */
void fqz5_trial_batch_stats(uint64_t *out3);
/* Adaptive-model chains fqz5_decode_sections placed so far: out2[0] on host
 * cores, out2[1] on the GPU. */
void fqz5_decode_chain_counts(uint64_t *out2);

/* ---- CRC32 (zlib crc32, fqzcomp5.c:2268-2269, :2310-2311, :4443, :4670) --- */

/* zlib's crc32(crc, buf, len) computed on the GPU (same value; buf == NULL
 * returns 0, zlib's initial value).  On a device error it returns 0 with
 * fqz5_last_error() set. */
unsigned long fqz5_crc32(unsigned long crc, const unsigned char *buf, unsigned int len);

/* The same over device memory of any length: *out = crc32(crc, d_buf, len).
 * Returns 0, or -1 on a device error. */
int fqz5_crc32_dev(uint32_t crc, const uint8_t *d_buf, uint64_t len, uint32_t *out);

/* ---- arith_dynamic (arith_dynamic.h:41-54) ----------------------------- */

/* Replaces arith_compress_bound (arith_dynamic.c:77). */
unsigned int arith_compress_bound(unsigned int size, int order);

/* Replaces arith_compress_to (arith_dynamic.c:730).  order = 0/1 | PACK 0x80
 * | RLE 0x40 | CAT 0x20 | NOSZ 0x10 | STRIPE 0x08 (stripes in bits 8-15);
 * EXT 0x04 (bzip2) fails as in a reference build without libbz2.
 * out == NULL: a buffer of arith_compress_bound() bytes is malloc()ed. */
unsigned char *arith_compress_to(unsigned char *in, unsigned int in_size,
                                 unsigned char *out, unsigned int *out_size,
                                 int order);

/* Replaces arith_compress (arith_dynamic.c:1027). */
unsigned char *arith_compress(unsigned char *in, unsigned int in_size,
                              unsigned int *out_size, int order);

/* Replaces arith_uncompress_to (arith_dynamic.c:1032). */
unsigned char *arith_uncompress_to(unsigned char *in, unsigned int in_size,
                                   unsigned char *out, unsigned int *out_sz);

/* Replaces arith_uncompress (arith_dynamic.c:1279). */
unsigned char *arith_uncompress(unsigned char *in, unsigned int in_size,
                                unsigned int *out_size);

/* ---- tok3 read-name tokeniser (tokenise_name3.h:43-75) ----------------- */

/* Replaces tok3_encode_names (tokenise_name3.c:1451).  `blk` holds names
 * terminated by '\n' or '\0' (rewritten to '\0' in place).  level 1-9
 * selects the per-type rANS / arith method lists of compress()
 * (tokenise_name3.c:1281-1358); use_arith codes the streams with
 * arith_dynamic.  Returns a malloc()ed buffer of *out_len bytes, or NULL
 * (more than 128 tokens, a byte >= 0x80, a codec failure).  *last_start_p
 * (when not NULL) receives the offset after the last terminator. */
uint8_t *tok3_encode_names(char *blk, int len, int level, int use_arith,
                           int *out_len, int *last_start_p);

/* Replaces tok3_decode_names (tokenise_name3.c:1675).  Returns the
 * '\0'-terminated names, malloc()ed, *out_len bytes; NULL on a malformed
 * stream. */
uint8_t *tok3_decode_names(uint8_t *in, uint32_t sz, uint32_t *out_len);

/* ---- Part 2: batched device API --------------------------------------- */

/* One stream.  `in`/`out` are device pointers. */
typedef struct {
    const uint8_t *in;
    uint8_t *out;
    uint32_t in_size;
    uint32_t out_cap;    /* compress: capacity (0 = bound); decompress: size */
    int32_t order;       /* compress only: htscodecs order word */
    uint32_t out_size;   /* result */
    int32_t status;      /* result: 0 ok, -1 failed (reference NULL) */
    int32_t pad;
} fqz5_rans_job;

/* Compress / decompress `n` streams in one batch on the calling thread's
 * GPU context; returns 0, or -1 on a device error (see fqz5_last_error). */
int fqz5_rans_compress_batch(fqz5_rans_job *jobs, int n);
int fqz5_rans_uncompress_batch(fqz5_rans_job *jobs, int n);

/* HIP stream (hipStream_t) that the calling thread's batches run on. */
void *fqz5_stream(void);

/* Ordering contract of the device-pointer entry points (fqz5_crc32_dev,
 * fqz5_rans_*_batch, fqz5_sections_*, fqz5_encode_sections,
 * fqz5_decode_sections, fqz5_blocks_assemble, fqz5_block_parse,
 * fqz5_block_lengths, fqz5_fastq_*):
 *  - inputs: they read device buffers on fqz5_stream().  A buffer written on
 *    another stream must be complete first: synchronise that stream, or call
 *    fqz5_stream_wait(producer) before the entry point (device-side wait,
 *    the host does not block);
 *  - outputs: every device output is written when the call returns (the
 *    calls synchronise fqz5_stream() before returning), so any stream may
 *    read it afterwards.
 * fqz5_stream_wait: the calling thread's fqz5_stream() — and every stream
 * the calling thread's entry points hand work to (its helper contexts,
 * existing or created later) — waits for all work enqueued on `stream` (a
 * hipStream_t; NULL = the null stream) so far.  Returns 0 or -1. */
int fqz5_stream_wait(void *stream);

/* 1 if a HIP device is usable, else 0 (and fqz5_last_error() is set). */
int fqz5_device_ok(void);

/* LZP pre-pass of fqzcomp5's LZP3 sequence method and of its LZP name
 * coding, on the GPU.
 *   fqz5_lzp   replaces lzp()   (lzp16e.h; lzp16e.c:113): same bytes, returns
 *              the output length (-1 on a device error).  `out` needs room for
 *              3 bytes per input byte in the worst case (escaped markers); the
 *              reference's callers allocate 2 * in_len + 1000, which the
 *              output of their inputs fits.
 *   fqz5_unlzp replaces unlzp() (lzp16e.c:166) with the output capacity the
 *              call sites know (fqzcomp5.c:2444 u_len, :1602 and :1667 the
 *              names buffers): returns the output length, or -1 if the
 *              stream is damaged or would write past out_cap (the reference
 *              would write past its buffer). */
int fqz5_lzp(unsigned char *in, int in_len, unsigned char *out);
int fqz5_unlzp(unsigned char *in, int in_len, unsigned char *out, int out_cap);

/* Last error message of the calling thread ("" if none). */
const char *fqz5_last_error(void);

/* Device bytes the arenas hold, process-wide: the chunks of every
 * thread's contexts, in use or idle in the shared pool (at most
 * $FQZ5_ARENA_IDLE_GB idle).  fqz5_arena_peak: the most held since the last
 * fqz5_arena_peak(1) (reset: 1 starts a new peak from the current holding).
 * fqz5_arena_use_peak: the most in use at once (held minus the idle chunks
 * kept for reuse) since the last fqz5_arena_use_peak(1). */
uint64_t fqz5_arena_bytes(void);
uint64_t fqz5_arena_peak(int reset);
uint64_t fqz5_arena_use_peak(int reset);

/* Kernel timing with HIP events on fqz5_stream() (benchmark roofline).
 * fqz5_profile(1) resets and enables; fqz5_profile_read fills
 * {enc_ms, enc_launches, enc_bytes, dec_ms, dec_launches, dec_bytes} for
 * the rANS chain kernels, bytes = algorithmic input + output bytes. */
void fqz5_profile(int on);
void fqz5_profile_read(double *out6);

/* The long kernels of every codec family, from every context of the
 * process (helper contexts included) since fqz5_profile(1): per kernel
 * {launch ms, launches, algorithmic bytes}, each launch timed by HIP events
 * around it on its own stream, in the order k_enc_chain (rANS encode, one
 * wave per chain), k_rans_dec, k_fqz_dec (both fqz decoders), k_fqz_rc (fqz
 * and sequence-model range chains), k_seq_dec, k_enc_chain2w (rANS encode,
 * two waves per chain), k_enc_replay (the emitting pass), k_seq_model,
 * k_fqz_model_hot (with its k_fqz_hot_list), k_fqz_ev_fill, k_lzp_dec,
 * k_enc_replay (the counting pass).  Fills min(nk, count) kernels; returns
 * the count. */
int fqz5_profile_read_all(double *out, int nk);

/* fqz encoder: quality models with at least `min_events` events in a block
 * are run one wavefront per model (the list in lanes); smaller ones one
 * lane per model.  0 disables the per-model wavefronts; the default is
 * 16384 (or $FQZ5_HOT_MIN).  Output bytes do not depend on it.  Returns the
 * previous value. */
unsigned fqz5_set_hot_min(unsigned min_events);

/* Hedged chain launches: the rANS decoder and the fqz range chain run each
 * dependent chain on 2-4 CUs at once while the copies fit one per CU, and
 * the first copy to finish wins (the same chain runs up to ~20 % slower on
 * some CUs).  Output bytes do not depend on it.  1 = on (default unless
 * $FQZ5_NO_HEDGE is set), 0 = off; returns the previous setting. */
int fqz5_set_hedge(int on);

/* The fqz decoder for small alphabets (at most 9 live symbols, qtab the
 * identity on them, no sequence context: Illumina 8-level and NovaSeq
 * data): 24-byte models in an LDS cache of ~6 280 sets instead of the
 * general decoder's 8 bytes per list slot.  Output bytes do not depend on
 * it.  1 = on (default unless $FQZ5_DEC_SMALL is "0"), 0 = off; returns
 * the previous setting. */
int fqz5_set_dec_small(int on);
/* Quality blocks decoded since the library was loaded: out2[0] by the
 * general fqz decoder, out2[1] by the small-alphabet one. */
void fqz5_fqz_dec_counts(uint64_t *out2);

/* Device check of the fqz decoder's division: floor(n / t) computed as
 * (u32)fma(n, recip(t), 2^-19) for every t < 2^16 and ~2000 n each.
 * Returns the number of mismatches (0), or -1 on a device error. */
long fqz5_fqz_div_selftest(void);

#ifdef __cplusplus
}
#endif
#endif
