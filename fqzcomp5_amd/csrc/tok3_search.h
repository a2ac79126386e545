// tok3_search.h — the tok3 trie search on the GPU for a batch of name blocks
// (tok3_search.hip; the host orchestration is tok3_search_batch, tok3.cpp).
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>

namespace fqz5 {

constexpr uint32_t T3_NONE = 0xffffffffu;
constexpr uint32_t T3_LSET_BITS = 1024;   // name lengths kept per block (longer: every depth)
constexpr uint32_t T3_KEY_BITS = 56;      // sort key: a 56-bit prefix hash

// search_trie's results for one name (block-local name numbers; pnum -1:
// none, as the host Trie::search)
struct T3Found { int pnum, exact, is_fixed, fixed_len; };

// The batch: the blocks' bytes back to back (each cut after its last
// terminator), and the device work arrays.
struct T3Batch {
    const uint8_t *bytes;
    uint32_t nbytes, nblk, nnames, npairs;
    const uint32_t *off;       // nblk + 1: each block's first byte, then nbytes
    const uint8_t *split;      // per block: a name section whose read ids are searched
    uint32_t *term, *tix;      // per byte: a terminator; terminators before it
    uint32_t *end;             // per name: its terminator
    uint32_t *st, *len, *sec;  // per name: first byte, length (of its id), block
    uint32_t *name0;           // per block: its first name
    uint32_t *lset;            // per block: T3_LSET_BITS bits, the names' lengths
    uint32_t *cnt, *poff;      // per name: its pairs, the first one
    uint64_t *key;             // per pair: the prefix hash
    uint32_t *val;             // per pair: its number
    const uint64_t *skey;      // sorted
    const uint32_t *sval;
    uint32_t *pname, *pdepth;  // per pair: its name and depth
    uint32_t *V;               // per pair: V(name, depth)
    int4 *fmt;                 // per name: prefix_len, is_fixed, fixed_len
    T3Found *found;            // per name
    uint32_t *bad;             // per block: refused, or a check failed
};

// stages 0: terminators / refused bytes; 1: name ends, blocks' first names
// (after the scan of term into tix); 2: extents, length sets, pair counts;
// 3: the pairs (after the scan of cnt into poff); 4: V and the results (after
// the sort)
hipError_t t3_launch(const T3Batch &b, int stage, hipStream_t s);
hipError_t t3_scan(const uint32_t *in, uint32_t *out, uint32_t n, void *tmp, size_t &bytes,
                   hipStream_t s);
// stable sort of (key, val) pairs; tmp == nullptr: the scratch size
hipError_t t3_sort(const uint64_t *k_in, uint64_t *k_out, const uint32_t *v_in, uint32_t *v_out,
                   uint32_t n, void *tmp, size_t &bytes, hipStream_t s);

}  // namespace fqz5
