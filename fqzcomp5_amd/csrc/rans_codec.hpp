// rans_codec.hpp — batched rANS 4x16/32x16 compressor/decompressor on the
// GPU.  A batch holds any number of independent streams; every stage of
// every stream in the batch is issued as one launch per stage, so the
// per-stream dependent rANS chains of all streams run concurrently.
#pragma once
#include <algorithm>
#include <thread>
#include <mutex>
#include <exception>
#include <atomic>
#include <cstdint>
#include <vector>

#include "gpu_ctx.hpp"
#include "host_dec.hpp"

namespace fqz5 {

// Host-side table construction (encoder: normalise_freq, O1 shift choice,
// serialised tables; decoder: slot tables) spread over up to 16 threads: a
// -3/-5 batch has thousands of stripe jobs.  fn(i) must touch item i only.
template <class F> inline void host_parallel(size_t n, F fn) {
    const size_t hw = size_t(host::threads());
    if (n < 64 || hw == 1) {
        for (size_t i = 0; i < n; i++) fn(i);
        return;
    }
    std::atomic<size_t> next{0};
    std::exception_ptr err;
    std::mutex mu;
    auto work = [&] {
        try {
            for (size_t i; (i = next.fetch_add(16)) < n;)
                for (size_t k = i; k < std::min(n, i + 16); k++) fn(k);
        } catch (...) {
            std::lock_guard<std::mutex> lk(mu);
            if (!err) err = std::current_exception();
        }
    };
    std::vector<std::thread> th;
    for (size_t t = 1; t < hw; t++) th.emplace_back(work);
    work();
    for (auto &t : th) t.join();
    if (err) std::rethrow_exception(err);
}



// A part of an output stream: host bytes or a device range.
struct Piece {
    std::vector<uint8_t> host;
    const uint8_t *dev = nullptr;
    uint32_t len = 0;
    uint32_t size() const { return dev ? len : uint32_t(host.size()); }
};
using Layout = std::vector<Piece>;

inline uint32_t layout_size(const Layout &l) {
    uint32_t s = 0;
    for (auto &p : l) s += p.size();
    return s;
}

struct CompressReq {
    const uint8_t *d_in = nullptr;  // device input
    uint32_t n = 0;
    int order = 0;
    uint32_t cap = 0;               // output capacity (0 => bound)
    // results
    bool ok = false;
    Layout out;
};

// Compress all requests (rans_compress_to_4x16 semantics, byte-exact).
// Layout pieces may point into the context arena: consume them (e.g. with
// write_layouts) before the next batch on this thread.
void compress_batch(GpuCtx &g, std::vector<CompressReq> &reqs);

// Copy each layout to a device destination (one copy launch for all).
void write_layouts_dev(GpuCtx &g, const std::vector<const Layout *> &ls,
                       const std::vector<uint8_t *> &dsts);
// Copy a layout to host memory.
void write_layout_host(GpuCtx &g, const Layout &l, uint8_t *dst);

struct DecompressReq {
    const uint8_t *h_in = nullptr;  // host copy of the stream (headers)
    const uint8_t *d_in = nullptr;  // device copy of the same bytes
    uint32_t in_size = 0;
    uint32_t out_cap = 0;           // expected/maximum output size
    uint8_t *d_out = nullptr;       // device output (out_cap bytes)
    // results
    bool ok = false;
    uint32_t out_size = 0;
};

// rans_uncompress_to_4x16 semantics.
void decompress_batch(GpuCtx &g, std::vector<DecompressReq> &reqs);

}  // namespace fqz5
