// fqz_codec.hpp — batched fqzcomp_qual encode / decode on device-resident
// blocks (fqz_codec.cpp).  fqz_compress / fqz_decompress (capi.cpp) are
// one-block batches over host buffers; the section coder (block.cpp) runs
// every block of a batch together: each serial kernel (model pass, range
// chain, carry, decoder) is one launch over all blocks.
#pragma once
#include <memory>
#include <vector>

#include "../../include/fqz5_mi355x.h"
#include "gpu_ctx.hpp"
#include "rans_codec.hpp"

namespace fqz5 {

struct FqzEncReq {
    const uint8_t *d_in = nullptr;      // device quality bytes
    size_t n = 0;
    int nrec = 0;
    uint32_t *lens = nullptr;           // host; may be rewritten to fit n (fqzcomp_qual.c:829-837)
    uint32_t *flags = nullptr;          // host; selector bits are set and cleared again
    const uint8_t *d_seq = nullptr;     // device: the records' bases back to back, or
    unsigned char **h_seq = nullptr;    //   host per-record pointers, or neither
    int vers = 4, strat = 0;
    fqz_gparams *gp = nullptr;
    // results
    bool ok = false;
    Layout out;                         // [varint size + parameters (host)][coder bytes (device)]
    struct Work;
    std::shared_ptr<Work> w;
};
uint32_t fqz_hot_min();
uint32_t fqz_set_hot_min(uint32_t v);
void fqz_encode_batch(GpuCtx &g, std::vector<FqzEncReq> &reqs);
// fqz_encode_batch in two halves: prepare runs every stage up to the model
// pass and sets each parallel request's size lower bound (entropy of its
// events; fqz_size_lower_bound, 0 if unknown); finish runs the range chain
// and the bytes of the requests not marked in skip (skipped ones get no
// output, ok = false).
void fqz_encode_prepare(GpuCtx &g, std::vector<FqzEncReq> &reqs);
void fqz_encode_finish(GpuCtx &g, std::vector<FqzEncReq> &reqs, const std::vector<char> *skip);
uint64_t fqz_size_lower_bound(const FqzEncReq &r);
// ... and its upper bound (the coder's slack over the entropy), 0 if unknown
uint64_t fqz_size_upper_bound(const FqzEncReq &r);
// coder bytes from the entropy sum (and slack sum) of a range-coded event list
uint64_t rc_bytes_lower(double bits);
uint64_t rc_bytes_upper(double bits, double slack);
struct FqzEvJob;
// The range coder back end shared by fqz and the sequence model: for jobs
// whose rec[] (stream order), nev, out and out_len are set, the range
// chain, the shift scan and the big-number bytes (*out_len = size).
void rc_backend(GpuCtx &g, std::vector<FqzEvJob *> &js);

struct FqzDecReq {
    const uint8_t *h_in = nullptr;      // host copy of the stream (parameters)
    const uint8_t *d_in = nullptr;      // device copy of the same bytes
    size_t in_size = 0;
    int *lengths = nullptr;             // host out: the first nlengths record lengths
    int nlengths = 0;
    int nrec = 0;                       // records of the sequence layout below
    const uint32_t *lens = nullptr;     // host: their lengths (sequence offsets)
    const uint8_t *d_seq = nullptr;     // device: bases back to back, or
    unsigned char **h_seq = nullptr;    //   host per-record pointers, or neither
    uint8_t *d_out = nullptr;           // device output, or nullptr (arena)
    size_t out_cap = 0;
    // results
    bool ok = false;
    size_t out_size = 0;
    struct Work;
    std::shared_ptr<Work> w;
};
void fqz_decode_batch(GpuCtx &g, std::vector<FqzDecReq> &reqs);

}  // namespace fqz5
