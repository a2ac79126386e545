/*
 * fqz5_fastq.h — FASTQ text in device memory to fqzcomp5 blocks and back
 * (SURVEY §8 f3), on the GPU:
 *
 *   fqz5_fastq_index    load_seqs_kseq's record parse (fqzcomp5.c:423-623,
 *                       kseq.h:178-218) for 4-line FASTQ: name up to the
 *                       first isspace(), comment to the line end, one
 *                       sequence line, '+' line, one quality line, a
 *                       trailing '\r' dropped as kseq drops it.  Text whose
 *                       first byte is '>' is FASTA: a record per header
 *                       line, its sequence lines joined as kseq joins them
 *                       (kseq.h:194-198; no quality section in its blocks,
 *                       fqzcomp5.c:575-578, :2258-2264).  Other text fails
 *                       (multi-line FASTQ); it is never parsed on the host.
 *   fqz5_fastq_blocks   the block split rule (fqzcomp5.c:471-479): a record
 *                       that would take a non-empty block past blk_size
 *                       (name.l + 1 + seq.l + qual.l per record) starts the
 *                       next block.
 *   fqz5_fastq_gather   one block's section inputs: names (name [' '
 *                       comment] '\0'), bases, qualities - 33 (device), the
 *                       record lengths and READ2 flags (host).
 *   fqz5_fastq_format(_pairs) output_fastq (fqzcomp5.c:3441-3480) of a decoded
 *                       block: '@' name '\n' seq '\n' '+' [name] '\n'
 *                       qual + 33 '\n'; without qualities output_fasta
 *                       (:3503-3517): '>' name '\n' seq '\n'.
 *
 * Offsets are bytes into the text.  Calls return 0 (fqz5_fastq_index: 1 for
 * FASTA text; fqz5_fastq_blocks: the block count) or -1 with
 * fqz5_last_error() set.
 */
#ifndef FQZ5_FASTQ_H
#define FQZ5_FASTQ_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct {                  /* one record of the text */
    uint64_t name, comment, seq, qual;        /* offsets */
    uint32_t name_len, comment_len, seq_len;  /* kseq's name.l, comment.l, seq.l */
    uint32_t fasta;                           /* 1: FASTA, its sequence lines
                                                 in [seq, qual); 2: wrapped
                                                 FASTQ, sequence and quality
                                                 lines from seq and qual */
    uint64_t end;                             /* the record's text end */
} fqz5_fastq_rec;

/* Index the records of d_text[0..len) (device) into d_recs (device, max_rec
 * entries; len / 6 + 1 always suffice); *nrec receives their number and
 * h_rec_size (host, max_rec entries, may be NULL) each record's
 * load_seqs_kseq size. */
int fqz5_fastq_index(const uint8_t *d_text, uint64_t len, fqz5_fastq_rec *d_recs,
                     uint64_t max_rec, uint64_t *nrec, uint32_t *h_rec_size);

/* fqz5_fastq_index for every layout kseq_read reads (kseq.h:178-218): 4-line
 * FASTQ, FASTA, and wrapped FASTQ (sequence and quality split over several
 * lines each; records with fasta = 2).  fqz5_fastq_index itself takes 4-line
 * FASTQ and FASTA only (the multi-GPU windows count records in lines). */
int fqz5_fastq_index_any(const uint8_t *d_text, uint64_t len, fqz5_fastq_rec *d_recs,
                         uint64_t max_rec, uint64_t *nrec, uint32_t *h_rec_size);

/* The ends (exclusive text offsets, increasing) of the complete FASTQ
 * records of d_text[0..len) (device; 4-line or wrapped): a record that the
 * text cuts off is left out unless eof (then the text end closes the last
 * one).  h_ends (host) holds up to max_ends; *n_ends receives the count.
 * Returns 0, or -1 on text that is not FASTQ kseq reads the same way. */
int fqz5_fastq_record_ends(const uint8_t *d_text, uint64_t len, int eof, uint64_t *h_ends,
                           uint64_t max_ends, uint64_t *n_ends);

/* Block starts (host): first[k] = the first record of block k, first[n] =
 * nrec.  Returns n, or -1 when more than max_blocks. */
int fqz5_fastq_blocks(const uint32_t *rec_size, uint64_t nrec, uint32_t blk_size,
                      uint64_t *first, int max_blocks);

/* Records [a, b) as one block.  sizes[3] receives the bytes of the names,
 * bases and qualities; with d_names / d_seq NULL only the sizes are
 * computed; d_qual NULL (FASTA): no qualities (sizes[2] = 0).  h_len / h_flag (host, b - a entries, may be NULL): record
 * lengths and FQZ5 READ2 flags (fqzcomp5.c:518-527). */
int fqz5_fastq_gather(const uint8_t *d_text, const fqz5_fastq_rec *d_recs, uint64_t a,
                      uint64_t b, uint8_t *d_names, uint8_t *d_seq, uint8_t *d_qual,
                      uint32_t *h_len, uint32_t *h_flag, uint64_t *sizes);

/* FASTQ text of a block (names '\0' after each, bases, qualities - 33 on
 * the device; lengths on the host) into d_out (out_cap bytes); *out_len its
 * size.  d_qual NULL: FASTA text.  d_out NULL: the size only. */
int fqz5_fastq_format(const uint8_t *d_names, uint64_t name_len, const uint8_t *d_seq,
                      const uint8_t *d_qual, const uint32_t *h_len, uint64_t nrec,
                      int plus_name, uint8_t *d_out, uint64_t out_cap, uint64_t *out_len);

/* Paired output (fqzcomp5 -d in out1 out2: output_fastq_deinterleaved /
 * output_fasta_deinterleaved, fqzcomp5.c:3535-3549, :3612-3676): as
 * fqz5_fastq_format, the block's even records (R1) first and its odd
 * records (R2) after them; *r1_len the first text's size. */
int fqz5_fastq_format_pairs(const uint8_t *d_names, uint64_t name_len, const uint8_t *d_seq,
                            const uint8_t *d_qual, const uint32_t *h_len, uint64_t nrec,
                            int plus_name, uint8_t *d_out, uint64_t out_cap, uint64_t *out_len,
                            uint64_t *r1_len);

#ifdef __cplusplus
}
#endif
#endif
