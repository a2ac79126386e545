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
    uint32_t nseq, nlengths;
    uint8_t *out;
    uint32_t *lengths;          // out: record lengths (nlengths)
    int32_t *status;
    uint32_t *nrec_out;
    // the decoder (fqz_decode.hip) keeps quality models in an LDS cache
    // backed by FQZ_CTX x ment bytes in HBM; qmap / duplicate / reversal
    // fix-ups are applied afterwards from the record lists it writes.
    uint8_t *back;
    uint32_t *back_hi;          // live > 62: list slots past lane 63, FQZ_CTX x 64 words
    uint32_t *hi_bits;          //   and which contexts' are written (FQZ_CTX bits, zeroed)
    uint32_t ment, nsets;       // cached model bytes, direct-mapped sets
    uint32_t cap_list, pad2;    // capacity of each record list
    uint4 *recs;                // nparam > 1: non-duplicate records {start, len, param, 0}
    uint2 *dups;                // duplicate records {start, len}
    uint2 *revs;                // reversed records {start, len}
    uint32_t *counts;           // out: [nrecs, ndups, nrevs, misses, slow symbols]
    // hedged (not null): copies of the block decode on other CUs with their
    // own backing store, everything else shared (identical writes); the
    // first copy to finish sets *done and the others leave
    uint32_t *done;
};

// Bytes of one cached quality model for `live` symbols: slots of 8 bytes
// {e, w}, read by the decoder's lane j as one 64-bit word: slot 0 a guard
// (e = 0xffff), then the sorted list (e = freq | cum << 16, w = qtab value |
// symbol << 24) up to lane 63, then the sentinel (e = context | total << 16).
// With more than 62 live symbols the list slots past lane 63 stay in HBM.
constexpr uint32_t fqz_dec_model_bytes(uint32_t live) {
    return 8u * ((live < 63u ? live : 63u) + 2u);
}
constexpr uint32_t FQZ_DEC_CACHE_BYTES = 163840u - 35088u - 1024u;
constexpr uint32_t FQZ_DEC_MAX_LIVE = 126u;   // guard + slots + sentinel in two lane registers (slow path)

// The small-alphabet decoder (fqz_decode_small.hip): models of at most 9
// live symbols as 24 bytes (u16 cumulative counts of slots 1..8, the tag,
// the total, the slots' symbols as nibbles) in a 4-way set-associative LDS
// cache (FqzDecJob::nsets counts sets of FQZ_SMALL_WAYS models) after
// FQZ_SMALL_LDS_FIXED bytes and FQZ_SMALL_PARAM_BYTES per parameter block;
// the backing store is FQZ_CTX models of 24 bytes.
constexpr uint32_t FQZ_SMALL_MAX_LIVE = 9u;
constexpr uint32_t FQZ_SMALL_MODEL_BYTES = 24u;
constexpr uint32_t FQZ_SMALL_WAYS = 4u;
constexpr uint32_t FQZ_SMALL_LDS_FIXED = 10512u;
constexpr uint32_t FQZ_SMALL_PARAM_BYTES = 2560u;
constexpr uint32_t fqz_small_sets(uint32_t nparam) {
    return (163840u - FQZ_SMALL_LDS_FIXED - nparam * FQZ_SMALL_PARAM_BYTES) /
           (FQZ_SMALL_WAYS * FQZ_SMALL_MODEL_BYTES);
}

// Parallel encoder (fqz_kernels.hip): the block becomes a list of coding
// events (record headers and quality symbols) in stream order; events are
// stably sorted by the model they use, every model runs over its own
// events in parallel to produce (cum, freq, total), and one lane range-codes
// the events in stream order.  Model ids: quality contexts 0..65535, then:
constexpr uint32_t FQZ_M_SEL = 65536, FQZ_M_LEN = 65537, FQZ_M_REV = 65541,
                   FQZ_M_DUP = 65542, FQZ_NMODELS = 65543, FQZ_MODEL_BITS = 17;

struct FqzEvJob {
    const FqzDevGlobal *g;
    const uint8_t *q;
    const uint64_t *off;        // record offsets
    const uint32_t *len, *sel, *flags;
    uint32_t nrec, nev;
    const uint8_t *seq;
    const uint64_t *seq_off;
    uint32_t *nev_rec;          // per-record event counts
    const uint32_t *ev_off;     // their exclusive scan
    uint8_t *dup;               // per-record duplicate flag
    uint32_t *key;              // events: model id
    uint64_t *val;              // events: index << 8 | symbol
    const uint32_t *skey;       // events sorted by model
    const uint64_t *sval;
    uint32_t *seg_lo, *seg_hi;  // per model: its range in the sorted order
    uint64_t *code;             // per sorted event: cum | freq << 16 | total << 32
    uint8_t *scratch;           // the non-quality models
    uint4 *rec;                 // per event: {RN(1/total) (2 words), freq, cum}; the range
                                // chain turns the first two into total's magic number, shift
    uint32_t *addend;           // per event: cum * (range / total)
    uint32_t *shifts;           // per event: coder byte shifts, then their scan
    const uint32_t *pos;        // exclusive scan of shifts
    uint32_t *nshift;           // total shifts
    unsigned long long *acc;    // little-endian 32-bit columns of the sum
    uint32_t nwords;
    uint32_t pad2;
    uint8_t *out;
    uint32_t *out_len;
    uint32_t *done;             // hedged range chain: claim word (zeroed; ~0 = a copy finished)
    uint32_t *ck;               // range chain: the range before every 64th event
};
// records of room J.rec needs past nev (the range chain's last loads)
constexpr uint32_t RC_PAD = 128;

hipError_t launch_fqz_events(const FqzEvJob &j, int phase, hipStream_t s);
// batched over the blocks of a request list: d_jobs in device memory
// hot: per job a list of stride words (zeroed); models with at least hot_min
// events go to the one-wave-per-model kernel (hot_min = 0: none do)
constexpr uint32_t FQZ_HOT_GRID = 64;            // waves per job for hot models
constexpr uint32_t FQZ_HOT_GRID_MAX = 2048;     // at most, one per hot model
constexpr uint32_t FQZ_HOT_MIN = 16384;
// (the hot models first, then the pass over the rest: launch_fqz_model_hot
// before launch_fqz_model_pass on the same stream)
hipError_t launch_fqz_model_hot(const FqzEvJob *d_jobs, int njobs, uint32_t *hot,
                                uint32_t stride, uint32_t hot_min, hipStream_t s);
hipError_t launch_fqz_model_pass(const FqzEvJob *d_jobs, int njobs, uint32_t hot_min,
                                 hipStream_t s);
// the range chain of d_jobs[0, njobs) (hedge copies after the first nbase):
// phase 0 the records' totals into multipliers, 1 the chain, 2 every
// event's q and byte shifts (max_nev: the most events of a job)
hipError_t launch_fqz_rc(const FqzEvJob *d_jobs, int njobs, int nbase, uint32_t max_nev,
                         int phase, hipStream_t s);
// per workgroup b: sum over its events of log2(total / freq) (after the model
// pass) in partial[b], of -log2(1 - total 2^-24) in partial[nblk + b]
hipError_t launch_fqz_entropy(const FqzEvJob &j, double *partial, uint32_t nblk, hipStream_t s);
hipError_t launch_rec_entropy(const uint4 *rec, uint32_t nev, double *partial, uint32_t nblk,
                              hipStream_t s);
// carry normalisation of the output columns: phase 1 writes s_w and the
// carry code per word, phase 2 (code = the scanned prefix codes) the digits
constexpr uint8_t FQZ_CARRY_KILL = 0, FQZ_CARRY_PROP = 1, FQZ_CARRY_GEN = 2;
hipError_t launch_fqz_norm(const FqzEvJob &j, int phase, uint32_t *sw, uint8_t *code,
                           hipStream_t s);
hipError_t launch_fqz_expand(const FqzEvJob &j, hipStream_t s);
hipError_t launch_fqz_bytes(const FqzEvJob &j, int phase, hipStream_t s);
// fqz_sort.hip
hipError_t fqz_exclusive_scan(const uint32_t *in, uint32_t *out, int n, void *tmp, size_t &bytes,
                              hipStream_t s);
// inclusive scan of the carry codes (the composition of kill / propagate /
// generate maps of a carry bit)
hipError_t fqz_carry_scan(const uint8_t *in, uint8_t *out, int n, void *tmp, size_t &bytes,
                          hipStream_t s);
hipError_t fqz_sort_by_model(const uint32_t *k_in, uint32_t *k_out, const uint64_t *v_in,
                             uint64_t *v_out, int n, int key_bits, void *tmp, size_t &bytes,
                             hipStream_t s);

hipError_t launch_fqz_records(const FqzStatJob &j, hipStream_t s);
hipError_t launch_fqz_hist(const FqzStatJob &j, int nchunks, int mode, hipStream_t s);
hipError_t launch_fqz_model_init(uint8_t *models, int live, hipStream_t s);
hipError_t launch_fqz_encode(const FqzEncJob &j, hipStream_t s);
// fqz_decode.hip: ne = lane registers per model (live + 2 <= 64 ? 1 : 2),
// seq = sequence bases in the context, qid = one qtab shared by every
// parameter block (its values ride in the cached models); map_mode 0 none / 1 one qmap / 2 per record
hipError_t launch_fqz_dec(const FqzDecJob *d_jobs, int njobs, int ne, bool seq, bool qid,
                          hipStream_t s);
hipError_t launch_fqz_dec_fix(const FqzDecJob &j, int map_mode, bool dups, bool revs, hipStream_t s);
// fqz_decode_small.hip: jobs with ment = FQZ_SMALL_MODEL_BYTES, nsets <=
// fqz_small_sets(nparam) and a backing store filled by launch_fqz_small_back;
// dt = some parameter block has delta terms
hipError_t launch_fqz_dec_small(const FqzDecJob *d_jobs, int njobs, bool dt, hipStream_t s);
hipError_t launch_fqz_small_back(uint8_t *back, uint32_t live, hipStream_t s);
hipError_t fqz_div_selftest(uint32_t *d_bad, hipStream_t s);

}  // namespace fqz5
