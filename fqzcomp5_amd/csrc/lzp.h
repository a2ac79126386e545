// lzp.h — work descriptors of the LZP kernels (lzp.hip): fqzcomp5's LZP
// pre-pass (lzp16e.c:113-214) behind the LZP3 sequence method
// (fqzcomp5.c:2013-2021, :2431-2445).  All pointers are device pointers.
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>

namespace fqz5 {

constexpr uint32_t LZP_HASH_BITS = 16;          // lzp16e.c:43-45
constexpr uint32_t LZP_MIN_LEN = 3;             // lzp16e.c:50-52
constexpr uint32_t LZP_MARK = 233;              // lzp16e.c:54
constexpr uint32_t LZP_MAX_LEN = 65535;         // lzp16e.c:121
constexpr uint32_t LZP_CHUNK = 8192;            // positions per speculative parse chunk

// Encoder, one block: every position i gets its hash h_i (a function of the
// 4 bytes before it), its prediction pred_i (the last j < i with h_j == h_i,
// 0 = none) and its match length; the token starts are the positions the
// serial parse visits, found by speculative chunk parses joined by one
// walk; each token is then written at its scanned offset.
struct LzpEncJob {
    const uint8_t *in;
    uint32_t n, nchunk;
    uint32_t *key, *skey;          // n: hash per position, sorted
    uint32_t *val, *sval;          // n: position, sorted by hash (stable)
    uint32_t *pred;                // n
    uint32_t *rev;                 // n: stop positions in reverse order (UINT32_MAX: linked)
    uint32_t *nxt;                 // n: inclusive min-scan of rev
    uint32_t *base;                // n: length at a stop position
    uint16_t *ml;                  // n: match length (0: literal)
    uint8_t *spec;                 // n: on its chunk's speculative path
    uint8_t *walk;                 // n: visited by the joining walk
    uint32_t *exitp, *conv;        // nchunk: speculative exit; where the true path joins
    uint32_t *size, *off;          // n: token bytes at a token start, their exclusive scan
    uint8_t *out;                  // >= 3 n bytes
    uint32_t *out_len;             // 1
};

hipError_t launch_lzp_hash(const LzpEncJob &j, hipStream_t s);
hipError_t launch_lzp_pred(const LzpEncJob &j, hipStream_t s);
hipError_t launch_lzp_stops(const LzpEncJob &j, hipStream_t s);
hipError_t launch_lzp_endscan(const LzpEncJob &j, hipStream_t s);
hipError_t launch_lzp_resolve(const LzpEncJob &j, hipStream_t s);
hipError_t launch_lzp_lengths(const LzpEncJob &j, hipStream_t s);
hipError_t launch_lzp_parse(const LzpEncJob &j, hipStream_t s);      // chunks + walk
hipError_t launch_lzp_sizes(const LzpEncJob &j, hipStream_t s);
hipError_t launch_lzp_emit(const LzpEncJob &j, hipStream_t s);
// device-wide helpers (hipCUB); tmp == nullptr reports the scratch size
hipError_t lzp_sort(const LzpEncJob &j, void *tmp, size_t &bytes, hipStream_t s);
hipError_t lzp_min_scan(const LzpEncJob &j, void *tmp, size_t &bytes, hipStream_t s);
hipError_t lzp_size_scan(const LzpEncJob &j, void *tmp, size_t &bytes, hipStream_t s);
hipError_t lzp_sort_ends(const LzpEncJob &j, void *tmp, size_t &bytes, hipStream_t s);  // key/val by distance
hipError_t lzp_end_scan(const LzpEncJob &j, void *tmp, size_t &bytes, hipStream_t s);   // val -> off

// Decoder: one wave per block.  Literal runs go 64 bytes per step; each
// marker byte looks up the hash table (65536 u32, zeroed) of its position.
struct LzpDecJob {
    const uint8_t *in;
    uint32_t in_len, cap;
    uint8_t *out;
    uint32_t *ht;
    uint32_t *out_len;
    int32_t *status;               // 0 ok, -1 damaged (token cut short / past cap)
};
hipError_t launch_lzp_dec(const LzpDecJob *d_jobs, int njobs, hipStream_t s);

}  // namespace fqz5
