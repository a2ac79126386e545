/*
 * fqz5_block.h — fqzcomp5 block-section coder on the GPU (C-ABI).
 *
 * Restates the per-section part of fqzcomp5's encode_block/decode_block
 * (fqzcomp5.c:2147-2547) for the sequence and quality sections: method
 * choice by the codec-trial state machine (metrics_method/metrics_update,
 * fqzcomp5.c:1899-1958), compress_with_methods' candidate loop
 * (fqzcomp5.c:1961-2144) and the section framing
 * [strat u8][u32 usize][u32 csize][stream] (fqzcomp5.c:2217-2257).
 * A caller hands over a run of blocks at once; the choices equal those of a
 * single-threaded reference run over the same blocks in the same order.
 * This build implements every method of the level presets: rANS (RANS0..
 * RANS193, RANSXN1), LZP3, the sequence context models SEQ10..SEQ14B, the
 * fqzcomp_qual methods FQZ0..FQZ4, and for name sections (FQZ5_SEC_NAME)
 * TLZP3, TOK3_3..9 and TOK3_3..9_LZP (encode_names, fqzcomp5.c:1408-1586).
 * A name section's output is encode_names' bytes [u32 name_len][u8 strat]
 * [u32 clen][payload] (no extra frame); its input is the block's names,
 * '\0' after each.  SEQ_CUSTOM is rejected.
 *
 * Blocks (encode_block / decode_block, fqzcomp5.c:2147-2547): the caller
 * codes the name, sequence and quality sections with the calls above, then
 * fqz5_blocks_assemble writes [u32 block_size][u32 nrec][u32 crc32] + names
 * + lengths + sequence + quality per block; fqz5_block_parse reads one back.
 */
#ifndef FQZ5_BLOCK_H
#define FQZ5_BLOCK_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define FQZ5_M_LAST 31            /* methods enum size, fqzcomp5.c:185-208 */
#define FQZ5_SEC_NAME 0           /* sections, fqzcomp5.c:177-183 */
#define FQZ5_SEC_LEN 1
#define FQZ5_SEC_SEQ 2
#define FQZ5_SEC_QUAL 3
#define FQZ5_SEC_LAST 4
#define FQZ5_METRICS_REVIEW 100   /* fqzcomp5.c:151 */
#define FQZ5_METRICS_TRIAL 3      /* fqzcomp5.c:152 */

typedef struct {                  /* the reference's `metrics` (fqzcomp5.c:221-225) */
    uint64_t usize[FQZ5_M_LAST], csize[FQZ5_M_LAST];
    int32_t review, trial;
    int32_t count[FQZ5_M_LAST];
    int32_t method_used;          /* method_used[sec] (fqzcomp5.c:232) */
} fqz5_section_stats;

typedef struct {
    fqz5_section_stats sec[FQZ5_SEC_LAST];
} fqz5_trial_state;

typedef struct {                  /* one section of one block (device data) */
    const uint8_t *in;            /* encode: raw bytes; decode: framed section */
    uint8_t *out;                 /* encode: framed section; decode: raw bytes */
    uint32_t in_size;
    uint32_t out_cap;
    uint32_t fixed_len;           /* fq->fixed_len (0 = variable) */
    int32_t sec;                  /* FQZ5_SEC_SEQ or FQZ5_SEC_QUAL */
    /* records of the block, for the FQZ methods (fqzcomp5.c:2071-2092):
     * host lengths and flags (flags may be NULL), and the block's sequence
     * bytes on the device, records back to back (NULL: no sequence) */
    const uint32_t *rec_len;
    const uint32_t *rec_flags;
    int32_t nrec;
    const uint8_t *seq;
} fqz5_section;

typedef struct {
    int32_t method;               /* chosen method (encode) */
    int32_t strat;                /* section strat byte */
    int32_t status;               /* 0 ok */
    uint32_t clen;                /* compressed stream bytes (excl. 9-byte frame) */
    uint32_t usize;               /* decoded bytes (decode) */
} fqz5_section_result;

void fqz5_trial_init(fqz5_trial_state *st);

/* Encode `n` sections given in block order; avail[sec] are the method masks
 * (1<<method).  st carries the trial state across calls.  Returns 0 or -1. */
int fqz5_encode_sections(const fqz5_section *secs, int n, const uint32_t *avail,
                         fqz5_trial_state *st, fqz5_section_result *res);

/* The same in four phases, for callers that replay the trial state over
 * sections held by several processes (multi-GPU, bench.py):
 *   schedule  host only: per section (file order) the method mask it tries,
 *             avail[sec] in trial / re-trial blocks and 0 elsewhere (their
 *             one method follows from the trial sizes); st is not changed;
 *   try       compress every method of masks[i] for each section;
 *             sizes[i*FQZ5_M_LAST+m] = candidate size, UINT32_MAX when not
 *             run (compress_with_methods' out_len); the candidates stay on
 *             the GPU until commit;
 *   replay    the host-only trial state machine over sections in file order;
 *   commit    encode the sections whose chosen method was not tried, then
 *             write every chosen stream, framed, to the outputs. */
void fqz5_trial_schedule(const int32_t *sec_ids, int n, const uint32_t *avail,
                         const fqz5_trial_state *st, uint32_t *masks_out);
int fqz5_sections_try(const fqz5_section *secs, int n, const uint32_t *masks,
                      uint32_t *sizes);
void fqz5_trial_replay(const int32_t *sec_ids, const uint32_t *in_sizes,
                       const uint32_t *sizes, int n, const uint32_t *avail,
                       fqz5_trial_state *st, int32_t *methods_out,
                       uint32_t *tried_out /* nullable: mask tried per section */);
int fqz5_sections_commit(const fqz5_section *secs, int n, const int32_t *methods,
                         fqz5_section_result *res);

/* Trial pruning (off by default).  When on, fqz5_sections_try skips the
 * range chain and bytes of an fqz candidate whose size is provably not below
 * the best rANS candidate: its lower bound 8 P >= sum log2(total/freq) - 8
 * (from the model pass) is at least the smallest exact rANS size in each of
 * the call's fqz sections and, summed over them, at least the smallest sum
 * of one rANS method.  rANS methods precede fqz ones, so they win ties: the
 * pruned candidate can never be chosen, and its reported size is the bound.
 * The caller turns it on only when the sections of the call that try fqz
 * are exactly one whole trial window (FQZ5_METRICS_TRIAL sections of one
 * section kind); otherwise the call does not prune.  Returns the previous
 * setting. */
int fqz5_set_trial_prune(int on);
/* Bounds-only tries for the large-block presets (encode_run_bounded): with
 * on = 1 every fqz and sequence-model candidate of a fqz5_sections_try skips
 * its range chain; `sizes` then holds its size lower bound (entropy of its
 * events) and fqz5_sections_try_upper its upper bound (entropy plus the
 * coder's slack, -log2(1 - total / 2^24) per event), every other entry
 * equal in both.  The caller decides the trial when the intervals separate
 * the candidates (fqzcomp5.c:1972-2127: per section the first smallest
 * size; the trial window's smallest (csize + 1) / usize, :1913-1924) and
 * commits the winners; otherwise it tries again with on = 0.  Returns the
 * previous setting. */
int fqz5_set_trial_bounds(int on);
/* The upper-bound sizes matrix (nsec * FQZ5_M_LAST) of this thread's last
 * fqz5_sections_try, which had `nsec` sections; -1 if there was none. */
int fqz5_sections_try_upper(uint32_t *upper, int nsec);
/* End this thread's try session (its candidates are dropped) and free the
 * device arenas of the thread's GPU context and helper contexts, after
 * synchronising them.  The large-block path calls it between its tries and
 * its commit, whose candidates run on other contexts. */
int fqz5_arenas_release(void);
/* {fqz candidates tried, of which pruned} since the library was loaded. */
void fqz5_trial_counts(uint64_t *out2);

/* Decode framed sections (strat 0 = rANS) into their outputs. */
int fqz5_decode_sections(const fqz5_section *secs, int n, fqz5_section_result *res);

/* ---- blocks (fqzcomp5.c:2147-2547) ------------------------------------ */

#define FQZ5_FREAD2 128           /* fqzcomp_qual.h:45 */

/* Per-record flags the way load_seqs_kseq sets them (fqzcomp5.c:518-527):
 * FQZ5_FREAD2 when the name (with its comment) ends in "/2" or equals the
 * previous name of the block.  names: host, '\0' after each. */
void fqz5_name_flags(const char *names, uint32_t name_len, int nrec, uint32_t *flags);

/* The lengths section (fqzcomp5.c:2189-2214): [nb][varint fixed_len] when
 * fixed_len != 0 (fq->fixed_len: -1 for a block without records), else
 * [0][u32 size][varint per record].  Returns its size (<= 5 + 5 nrec), or
 * -1 if cap is too small. */
int fqz5_block_lengths(const uint32_t *len, int nrec, int32_t fixed_len, uint8_t *out,
                       uint32_t cap);

typedef struct {                  /* one block's coded parts */
    int32_t nrec;
    const uint8_t *name;          /* device: encode_names' bytes */
    uint32_t name_size;
    const uint8_t *lengths;       /* host: fqz5_block_lengths' bytes */
    uint32_t lengths_size;
    const uint8_t *seq;           /* device: framed sequence section */
    uint32_t seq_size;
    const uint8_t *qual;          /* device: framed quality section; NULL for */
    uint32_t qual_size;           /*   FASTA (9 zero bytes are written) */
} fqz5_block_parts;

/* Write n blocks, block i at d_out + off[i] (device); size[i] receives its
 * bytes (12 + parts; the caller sizes off[] with fqz5_block_size).  The
 * CRC32 of bytes 12.. is computed on the device.  Returns 0 or -1. */
uint64_t fqz5_block_size(const fqz5_block_parts *p);
int fqz5_blocks_assemble(const fqz5_block_parts *parts, int n, uint8_t *d_out,
                         const uint64_t *off, uint32_t *size);

typedef struct {                  /* one block read back (decode_block) */
    uint32_t block_size;          /* bytes after the block_size field */
    uint32_t nrec;
    int32_t crc_ok;               /* stored CRC equals the CRC of the block */
    uint32_t name_off, name_size; /* encode_names' bytes, offsets in the block */
    uint32_t name_ulen;           /* names' decoded size */
    int32_t fixed_len;            /* 0: variable lengths */
    uint32_t seq_off, seq_size;   /* framed sections */
    uint32_t seq_ulen;
    uint32_t qual_off, qual_size; /* qual_size 9 with qual_ulen 0: FASTA */
    uint32_t qual_ulen;
} fqz5_block_view;

/* Parse the block at d_block (device, `avail` bytes readable): the layout,
 * the CRC check and, when lens != NULL (nrec entries), the record lengths.
 * Returns 0, or -1 on a malformed block: a field past the block, a quality
 * section whose u_len is not the sequence u_len (FASTA's 9 zero bytes
 * aside), or record lengths that do not sum to the sequence u_len (the
 * section outputs are sized from these fields). */
int fqz5_block_parse(const uint8_t *d_block, uint64_t avail, fqz5_block_view *v,
                     uint32_t *lens, uint32_t lens_cap);

/* The same for a block of any container version the reference decodes
 * (read_header, fqzcomp5.c:2576-2602; decode_block :2290-2318):
 * FQZ5_V11 `FQZ5\1\1\0\0` blocks carry [u32 size][u32 nrec][u32 crc32];
 * FQZ5_V10 `FQZ5\1\0\0\0` and FQZ5_VOLD (no file header) blocks have no CRC
 * field ([u32 size][u32 nrec], the name section at offset 8) and report
 * crc_ok = 1, as the reference skips the check for them.
 * fqz5_block_parse(...) is fqz5_block_parse_v(..., FQZ5_V11, ...). */
enum { FQZ5_V11 = 0, FQZ5_V10 = 1, FQZ5_VOLD = 2 };
int fqz5_block_parse_v(const uint8_t *d_block, uint64_t avail, int version,
                       fqz5_block_view *v, uint32_t *lens, uint32_t lens_cap);

/* The same parse for n blocks at once (d_blocks[i], avail[i] bytes; lens[i]
 * with lens_cap[i] entries, or NULL): every block's header reads of one kind
 * share one round trip (5 for the batch, instead of ~6 per block).
 * status[i] = 0 or -1 per block; returns -1 when any block failed
 * (fqz5_last_error: the first failure).  Replaces a loop of decode_block's
 * header reads (fqzcomp5.c:2300-2487) over the blocks. */
int fqz5_blocks_parse_v(const uint8_t *const *d_blocks, const uint64_t *avail, int n,
                        int version, fqz5_block_view *views, uint32_t *const *lens,
                        const uint32_t *lens_cap, int32_t *status);

#ifdef __cplusplus
}
#endif
#endif
