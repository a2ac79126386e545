// seq_cm.h — work descriptors of the sequence context model kernels
// (seq_cm.hip): fqzcomp5's SEQ10 .. SEQ14B methods, fqzcomp5.c:1073-1406.
// All pointers are device pointers.
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>

namespace fqz5 {

constexpr uint32_t SEQ_K_MAX = 14;      // 4^14 contexts x 4 count bytes = 1 GiB

// Encoder.  The block becomes coding events in stream order:
//   per run of one class (uppercase ACGT / lowercase acgt / other bytes):
//     the run length as 255-digits (run-length model of the class),
//     the run's symbols (k-mer context model, or the literal model),
//     the class switch (2-symbol state model of the class), except at the end;
//   and, when the block does not start with ACGT, an empty uppercase run and
//   its switch first (the coder starts in the uppercase state).
// The symbol at byte p is event p + lead + run_off[r] + D_r (r its run, D_r
// the run's digit count, run_off the exclusive scan of D + 1 over the runs).
struct SeqJob {
    const uint8_t *in;
    uint32_t n, k, both, mask;          // mask = 4^k - 1
    uint32_t lead;                      // 2 when the block starts with another class
                                        // (an empty uppercase run and its switch), else 0
    uint32_t nrun, nseg, nkeys;         // nkeys = n (one strand) or 2n (both)
    const uint32_t *seg;                // record starts where contexts restart, seg[nseg] = n
    uint32_t *flag, *ex;                // per byte: run head, exclusive scan of the heads
    uint32_t *run_start;                // per run (nrun)
    uint32_t *cnt, *run_off;            // per run D + 1 (and 0 at nrun), its exclusive scan
    uint32_t *key;                      // per context event (interleaved fw/rv): context id
    uint64_t *val;                      //   (2e + rv) << 8 | symbol, e the event index of
                                        //   the forward symbol of the byte
    const uint32_t *skey;               // the same, sorted by context
    const uint64_t *sval;
    uint4 *rec;                         // per coding event: {RN(1/total) (2 words), freq, cum}
};

hipError_t launch_seq_heads(const SeqJob &j, hipStream_t s);
hipError_t launch_seq_runs(const SeqJob &j, hipStream_t s);       // run starts, cnt
hipError_t launch_seq_ctx(const SeqJob &j, hipStream_t s);        // keys / values
hipError_t launch_seq_model(const SeqJob &j, hipStream_t s);      // context events -> rec
hipError_t launch_seq_side(const SeqJob &j, hipStream_t s);       // run / literal / state -> rec

// Decoder: one chain per block.
struct SeqDecJob {
    const uint8_t *in;
    uint32_t in_len, n, k, both;
    uint32_t mask, nseg;
    const uint32_t *seg;
    uint32_t *models;                   // 4^k x 4 counts
    uint8_t *out;
    int32_t *status;                    // 0 ok, -1 damaged stream
};
hipError_t launch_seq_models_init(uint32_t *models, size_t nctx, hipStream_t s);
// one workgroup per job (device array)
// lookahead: k >= 3, the decoder that loads each base's counts three
// bases ahead (k_seq_dec_la); else the one-step decoder
hipError_t launch_seq_dec(const SeqDecJob *d_jobs, int njobs, hipStream_t s, bool lookahead);

}  // namespace fqz5
