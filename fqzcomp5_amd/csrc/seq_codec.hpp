// seq_codec.hpp — the sequence context model (SEQ10 .. SEQ14B,
// fqzcomp5.c:1073-1406) on device-resident blocks (seq_codec.cpp), for the
// section coder (block.cpp) and fqz5_seq_encode / fqz5_seq_decode.
#pragma once
#include <memory>
#include <vector>

#include "gpu_ctx.hpp"
#include "rans_codec.hpp"

namespace fqz5 {

struct SeqEncReq {
    const uint8_t *d_in = nullptr;      // device bases
    uint32_t n = 0;
    const uint32_t *lens = nullptr;     // host record lengths
    int nrec = 0;
    int both = 0, k = 12;
    // results
    bool ok = false;                    // false: the records run out (encode_seq's NULL)
    Layout out;                         // the coder bytes (device)
    std::shared_ptr<struct SeqWork> w;  // between prepare and finish
};
// prepare: every block's events and model pass (one block after another,
// every phase a parallel kernel) and its size lower bound; finish: the range
// chains of the requests not in `skip` in one launch, and their bytes.
void seq_encode_prepare(GpuCtx &g, std::vector<SeqEncReq> &reqs);
void seq_encode_finish(GpuCtx &g, std::vector<SeqEncReq> &reqs, const std::vector<char> *skip);
// Output size lower bound after prepare (entropy of the events), 0 if none.
uint64_t seq_size_lower_bound(const SeqEncReq &r);
// ... and the upper bound (entropy plus the coder's slack), 0 if none.
uint64_t seq_size_upper_bound(const SeqEncReq &r);
void seq_encode_batch(GpuCtx &g, std::vector<SeqEncReq> &reqs);

struct SeqDecReq {
    const uint8_t *d_in = nullptr;      // device stream
    uint32_t in_size = 0;
    const uint32_t *lens = nullptr;
    int nrec = 0;
    int both = 0, k = 12;
    uint8_t *d_out = nullptr;           // device output of n bytes
    uint32_t n = 0;
    bool ok = false;
};
// every block's chain in one launch
void seq_decode_batch(GpuCtx &g, std::vector<SeqDecReq> &reqs);

}  // namespace fqz5
