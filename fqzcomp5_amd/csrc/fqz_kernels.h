// fqz_kernels.h — work descriptors of the fqzcomp_qual kernels
// (fqz_kernels.hip).  All pointers are device pointers.
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>

namespace fqz5 {

constexpr int FQZ_CTX = 65536;          // CTX_SIZE, fqzcomp_qual.c:73-74
constexpr int FQZ_QSYMS = 96;           // QMAX, fqzcomp_qual.c:84
constexpr int FQZ_QMODEL_BYTES = 304;   // sizeof(FList<96>): u32 + 99 u16 + 99 u8, padded
constexpr int FQZ_MAX_PARAMS = 4;

// One parameter block as the kernels use it: position / delta tables
// already shifted to their context location (fqzcomp_qual.c:1067-1076).
struct FqzDevParam {
    uint32_t ctx0, qshift, qloc, sloc, bbits, bloc, boff, qmask;
    uint32_t sel, dedup, fixed, pad;
    uint32_t qtab[256];
    uint32_t ptab[1024];
    uint32_t dtab[256];
    uint8_t qmap[256];
};

struct FqzDevGlobal {
    uint32_t gflags, nparam, max_sel, max_sym;
    uint8_t stab[256];
    FqzDevParam p[FQZ_MAX_PARAMS];
};

struct FqzStatJob {
    const uint8_t *q;           // quality bytes
    const uint64_t *off;        // record offsets
    const uint32_t *len;        // record lengths
    const uint32_t *flags;      // record flags (READ2 = 128)
    uint32_t nrec;              // records walked by the statistics
    uint32_t pad;
    uint32_t *rec_avg;          // out: per-record average quality (tenths)
    uint32_t *avg_hist;         // out: [2560]
    uint32_t *dups;             // out: duplicate-record count
    const uint2 *chunks;        // histogram work: record ranges
    uint32_t *h1, *h2;          // out: [128][256] READ1 / READ2
    const uint32_t *amap;       // [2560] average -> class (qbin pass)
    uint32_t *b4;               // out: [4][128][256] per class
};

struct FqzEncJob {
    const FqzDevGlobal *g;
    const uint8_t *q;
    uint64_t n;
    const uint32_t *len, *sel, *flags;
    uint32_t nrec, pad;
    const uint8_t *seq;         // per-record sequence bytes or nullptr
    const uint64_t *seq_off;
    uint8_t *models;            // FQZ_CTX quality models
    uint8_t *out;               // range-coder bytes
    uint32_t *out_len;
};

struct FqzDecJob {
    const FqzDevGlobal *g;
    const uint8_t *in;          // range-coder bytes
    uint64_t in_len;
    uint64_t n;                 // decoded size
    const uint8_t *seq;
    const uint64_t *seq_off;
    uint32_t nseq, nlengths, max_rec, pad;
    uint8_t *models;
    uint8_t *out;
    uint32_t *lengths;          // out: record lengths (nlengths)
    uint8_t *rev;               // GFLAG_DO_REV bookkeeping (max_rec)
    uint32_t *rlen;
    int32_t *status;
    uint32_t *nrec_out;
};

hipError_t launch_fqz_records(const FqzStatJob &j, hipStream_t s);
hipError_t launch_fqz_hist(const FqzStatJob &j, int nchunks, int mode, hipStream_t s);
hipError_t launch_fqz_model_init(uint8_t *models, int live, hipStream_t s);
hipError_t launch_fqz_encode(const FqzEncJob &j, hipStream_t s);
hipError_t launch_fqz_decode(const FqzDecJob &j, hipStream_t s);

}  // namespace fqz5
