// lzp_codec.hpp — fqzcomp5's LZP pre-pass (lzp16e.c) on device-resident
// blocks (lzp_codec.cpp): the first stage of the LZP3 sequence method
// (fqzcomp5.c:2013-2021 encode, :2431-2445 decode), and fqz5_lzp /
// fqz5_unlzp on host buffers.
#pragma once
#include <vector>

#include "gpu_ctx.hpp"

namespace fqz5 {

struct LzpEncReq {
    const uint8_t *d_in = nullptr;      // device bytes
    uint32_t n = 0;
    // results (device output in the context arena, valid until its reset)
    uint8_t *d_out = nullptr;
    uint32_t out_len = 0;
};
// every block's parallel passes, then one sync for the output lengths
void lzp_encode_batch(GpuCtx &g, std::vector<LzpEncReq> &reqs);

struct LzpDecReq {
    const uint8_t *d_in = nullptr;      // device lzp stream
    uint32_t in_len = 0;
    uint8_t *d_out = nullptr;           // device output of cap bytes
    uint32_t cap = 0;
    // results
    bool ok = false;
    uint32_t out_len = 0;
};
// every block's decoder in one launch (one wave each)
void lzp_decode_batch(GpuCtx &g, std::vector<LzpDecReq> &reqs);

}  // namespace fqz5
