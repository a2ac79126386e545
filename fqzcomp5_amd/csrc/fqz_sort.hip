// fqz_sort.hip — device-wide scan and stable radix sort (hipCUB / rocPRIM)
// for the parallel fqzcomp_qual encoder (fqz_kernels.hip): the exclusive
// scan of per-record event counts, the carry scan of the output columns and
// the stable sort of events by model.
// Each call with tmp == nullptr only reports the scratch size.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include "fqz_kernels.h"

namespace fqz5 {

hipError_t fqz_exclusive_scan(const uint32_t *in, uint32_t *out, int n, void *tmp, size_t &bytes,
                              hipStream_t s) {
    return hipcub::DeviceScan::ExclusiveSum(tmp, bytes, in, out, n, s);
}

namespace {
// b after a: a generating or killing word decides the carry out, a
// propagating one passes on what came in
struct CarryCompose {
    __device__ uint8_t operator()(uint8_t a, uint8_t b) const {
        return b == FQZ_CARRY_PROP ? a : b;
    }
};
}  // namespace

hipError_t fqz_carry_scan(const uint8_t *in, uint8_t *out, int n, void *tmp, size_t &bytes,
                          hipStream_t s) {
    return hipcub::DeviceScan::InclusiveScan(tmp, bytes, in, out, CarryCompose(), n, s);
}

hipError_t fqz_sort_by_model(const uint32_t *k_in, uint32_t *k_out, const uint64_t *v_in,
                             uint64_t *v_out, int n, int key_bits, void *tmp, size_t &bytes,
                             hipStream_t s) {
    return hipcub::DeviceRadixSort::SortPairs(tmp, bytes, k_in, k_out, v_in, v_out, n, 0,
                                              key_bits, s);
}

}  // namespace fqz5
