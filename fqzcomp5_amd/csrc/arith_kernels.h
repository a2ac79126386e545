// arith_kernels.h — the arith_dynamic entropy coders on the GPU
// (arith_kernels.hip); the dispatcher is arith_codec.cpp.
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>

namespace fqz5 {

// One entropy-coded stream: encode n input bytes into at most cap coder
// bytes, or decode in_len coder bytes into n output bytes.  m = the byte
// models' symbol count (max symbol + 1).
struct ArithJob {
    const uint8_t *in;
    uint8_t *out;
    uint8_t *models;            // model lists in HBM (nullptr: in LDS)
    uint32_t *out_len;          // encode: coder bytes written
    int32_t *status;            // 0, or -1 (output full / input exhausted)
    uint32_t n, in_len, cap, m, o1, rle;
};

uint32_t arith_model_bytes(uint32_t m, bool o1, bool rle);
bool arith_models_in_lds(uint32_t m, bool o1, bool rle);
hipError_t launch_arith(const ArithJob *d_jobs, int njobs, bool decode, bool global_models,
                        uint32_t lds_bytes, hipStream_t s);

// the dispatcher (arith_codec.cpp): host buffers, GPU work
uint32_t arith_compress_bound_ref(uint32_t size, int order);
uint8_t *arith_compress_gpu(const uint8_t *in, uint32_t in_size, uint8_t *out, uint32_t *out_size,
                            int order);
uint8_t *arith_uncompress_gpu(const uint8_t *in, uint32_t in_size, uint8_t *out,
                              uint32_t *out_size);

}  // namespace fqz5
