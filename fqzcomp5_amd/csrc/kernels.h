// kernels.h — work descriptors shared by the host planner (rans_codec.cpp)
// and the gfx950 kernels (rans_kernels.hip).  All pointers are device
// pointers.
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>

namespace fqz5 {

#define RANS_LOW_D (1u << 15)

// One slice [begin, end) of segment `seg`; counts[seg*512 + 0..255] receive
// the byte histogram, counts[seg*512 + 256..511] the repeat counts.
struct HistItem {
    const uint8_t *data;
    uint32_t begin, end;
    uint32_t seg, pad;
};

// Order-1 pair histogram slice over an A-symbol compacted alphabet.
struct Hist1Item {
    const uint8_t *data;
    const uint8_t *remap;   // 256 entries, byte -> alphabet index
    uint32_t begin, end;
    uint32_t A;
    uint32_t out_off;       // offset (u32 units) of the A*A result block
};

struct PackItem {
    const uint8_t *in;
    uint8_t *out;
    const uint8_t *code;    // pack: byte -> code; unpack: code -> byte
    uint32_t n;             // pack: input symbols; unpack: output symbols
    int32_t per;            // symbols per byte (0, 2, 4, 8)
};

struct StripeItem {
    const uint8_t *in;
    uint8_t *out;
    uint32_t n, N;
    int32_t dir;            // 0 transpose, 1 untranspose
    int32_t pad;
};

struct CopyItem {
    const uint8_t *src;
    uint8_t *dst;
    uint32_t len;
    uint32_t pad;
};

struct EncSym;  // rans_format.hpp

struct EncJob {
    const uint8_t *in;
    const EncSym *tab;      // O0: [256]; O1: [A*A] (remap[ctx]*A + remap[sym])
    const uint8_t *remap;   // O1: byte -> alphabet index (nullptr for O0)
    uint8_t *out_end;       // 2-byte aligned; stream grows downward
    uint32_t *out_len;      // bytes written below out_end
    uint32_t *ck;           // (nchunks + 1) * nx state checkpoints
    uint32_t *cnt;          // nchunks word counts, then exclusive offsets
    uint32_t n;
    int32_t nx;             // 4 or 32
    int32_t bits;           // 12 (O0) or 10/12 (O1)
    int32_t A;              // O1 alphabet size
    uint32_t nchunks;       // ceil(steps / enc_chunk_steps(nx))
};

// O1 encoder tables of more than ENC_TAB_LDS_MAX bytes at 16 B per entry
// (alphabets over 64) stay in global memory, compact: 4 B per (context,
// symbol), freq | start << 13 (freq <= 4096, start < 4096), expanded to the
// 16-B symbol when the chain's entries are staged and in the replay, with
// the reciprocal of each frequency from an LDS table (enc_rcp_lds).  A
// quarter of the bytes per symbol read, and a 256-symbol table (256 KB)
// stays in the XCD's L2 beside the other streams' (1 MB each did not).
constexpr uint32_t ENC_TAB_LDS_MAX = 65536;
constexpr uint32_t ENC_RCP_N = 4097;                      // frequencies 0..4096
__host__ __device__ inline bool enc_tab_compact(bool o1, uint32_t A) { return o1 && A * A * 16u > ENC_TAB_LDS_MAX; }

// Encoder chunk: steps between state checkpoints (chain and replay agree).
inline uint32_t enc_chunk_steps(int nx) { return 1024u / uint32_t(nx); }
// Replay: chunks handled by one 1024-thread workgroup.
inline uint32_t enc_replay_chunks(int nx) { return 16u * uint32_t(64 / nx); }

// out[i] = *src[i]: single bytes fetched for host decisions.
struct GatherItem {
    const uint8_t *src;
};

struct DecJob {
    const uint8_t *in;      // payload: NX states then 16-bit words
    const uint32_t *tab;    // rows of 2^bits entries; O0 one row, O1 one
                            // row per context in alphabet order
    const uint8_t *alpha;   // O1: row index -> byte value (nullptr for O0)
    uint8_t *out;
    int32_t *status;
    uint32_t in_len;
    uint32_t n;
    int32_t nx;
    int32_t bits;
    uint32_t rows;          // table rows (1 for O0)
    uint32_t mode;          // DEC_TAB_* (dec_table_mode)
    uint32_t *done;         // hedged launch: claim word, zeroed; ~0 = a copy finished (or nullptr)
    // O0 NX=4 with at most DEC_REG_MAX symbols covering all 2^bits slots:
    // the symbols' start | f << 16 in slot order (the register decoder,
    // rans_chain.hip dec4_lean_body); nreg = 0 otherwise.  nx = 0 marks a
    // padding job of an XCD-grouped launch (exits at once).
    uint32_t nreg;
    uint32_t reg[8];
    // O1 NX=4 with at most DEC_O1KEY_MAX (context, symbol) pairs, rows <= 8
    // (bits 12) or 16 (bits <= 10): the replicated-state register decoder
    // (rans_chain.hip dec4_o1reg_body).  okeys: 16 * (pairs / 16 rounded up)
    // keys ctx << rowsh | start << 16 | (0xffff - ((f-1) << 4 | sym)), the
    // last group padded with key 0; 0: not this decoder.
    uint32_t okeys;
    uint32_t rowsh;
    uint32_t okey[64];
};
constexpr uint32_t DEC_REG_MAX = 8;
constexpr uint32_t DEC_O1KEY_MAX = 64;
constexpr uint32_t DEC_O1REG_LDS_BYTES = 16384;

// Decoder table placement (rans_chain.hip).  Per slot of a row of 2^bits:
//   LDS / GLOBAL  u32 (f-1) << (bits+8) | (slot - start) << 8 | symbol
//                 (alphabet index for O1), in LDS or read from global memory;
//   SPLIT (O1)    u8 symbol per slot, then u32 (f-1) << 16 | start per
//                 (context, symbol) in rows of 2^dec_rp_log(rows) entries.
enum : uint32_t { DEC_TAB_LDS = 0, DEC_TAB_GLOBAL = 1, DEC_TAB_SPLIT = 2 };
constexpr uint32_t DEC_TAB_LDS_MAX = 147456;
__host__ __device__ inline uint32_t dec_rp_log(uint32_t rows) {
    uint32_t r = 0;
    while ((1u << r) < rows) r++;
    return r;
}
// 32-bit words of the table image for a mode
__host__ __device__ inline uint32_t dec_tab_words(uint32_t mode, uint32_t rows, int bits) {
    const uint32_t slots = rows << bits;
    if (mode == DEC_TAB_SPLIT) return slots / 4 + (rows << dec_rp_log(rows));
    return slots;
}
// NX=4 streams whose table fits the lean decoder's 16-byte entries in LDS
// (rans_chain.hip dec4_lean_body): O0, and O1 with rows x 2^bits <= 8192.
constexpr uint32_t DEC_LEAN_ENTRIES = 8192;
__host__ __device__ inline bool dec_lean(uint32_t rows, int bits) {
    return (uint64_t(rows) << bits) <= DEC_LEAN_ENTRIES;
}

inline uint32_t dec_table_mode(bool o1, uint32_t rows, int bits) {
    if (dec_tab_words(DEC_TAB_LDS, rows, bits) * 4u <= DEC_TAB_LDS_MAX) return DEC_TAB_LDS;
    if (o1 && dec_tab_words(DEC_TAB_SPLIT, rows, bits) * 4u <= DEC_TAB_LDS_MAX)
        return DEC_TAB_SPLIT;
    return DEC_TAB_GLOBAL;
}

// RLE encode of one leaf input; saved[] marks the RLE symbols.
struct RleItem {
    const uint8_t *in;
    const uint8_t *saved;
    uint8_t *lits;
    uint8_t *runs;
    uint32_t n;
    uint32_t pad;
};

// RLE decode: literals + run varints -> nout bytes.
struct UnRleItem {
    const uint8_t *lits;
    const uint8_t *runs;
    const uint8_t *saved;
    uint32_t *vend;         // scratch, one entry per varint
    uint8_t *out;
    uint32_t nlit, nrun, nvarint, nout;
};

constexpr uint32_t RLE_CHUNK = 65536;

hipError_t launch_rle_count(const RleItem *items, const uint32_t *chunk_item,
                            int nchunks, uint32_t *cstat, hipStream_t s);
hipError_t launch_rle_emit(const RleItem *items, const uint32_t *chunk_item,
                           int nchunks, const uint32_t *cmeta, hipStream_t s);
hipError_t launch_unrle_count(const UnRleItem *items, const uint32_t *chunk_item,
                              int nchunks, uint32_t *cstat, int what, hipStream_t s);
hipError_t launch_unrle_vend(const UnRleItem *items, const uint32_t *chunk_item,
                             int nchunks, const uint32_t *coff, hipStream_t s);
hipError_t launch_unrle_expand(const UnRleItem *items, const uint32_t *chunk_item,
                               int nchunks, const uint32_t *coff, uint32_t *cstat,
                               int what, hipStream_t s);

hipError_t launch_gather(const GatherItem *items, int n, uint8_t *out, hipStream_t s);
// Order-1 encoder table of one job, built on the GPU: f[A*A] the normalised
// frequencies over the compacted alphabet (row = context), out[A*A] the
// EncSym of every (context, symbol) (rans_compress.cpp build_o1).
struct EncTabItem {
    const uint16_t *f;
    EncSym *out;
    uint32_t A;
    uint32_t bits;
};
hipError_t launch_enc_tab(const EncTabItem *d_items, int nitems, hipStream_t s);
hipError_t launch_hist0(const HistItem *d_items, int nitems, uint32_t *d_counts,
                        hipStream_t s);
// big: items with A*A >= 16384 (16-bit LDS counters; slices < 65536 bytes)
hipError_t launch_hist1(const Hist1Item *d_items, int nitems, uint32_t *d_counts, bool big,
                        hipStream_t s);
hipError_t launch_pack(const PackItem *d_items, int nitems, uint32_t max_out,
                       bool unpack, hipStream_t s);
hipError_t launch_stripe(const StripeItem *d_items, int nitems, uint32_t max_n,
                         hipStream_t s);
hipError_t launch_copy(const CopyItem *d_items, int nitems, hipStream_t s);
// One launch for all jobs; O1 jobs are the ones with remap / alpha set.
// `lds` = dynamic LDS bytes: the maximum of enc_lds_bytes/dec_lds_bytes
// over the launch's jobs.
uint32_t enc_lds_bytes(int o1, uint32_t A);
uint32_t enc_replay_lds_bytes(int o1, uint32_t A);
bool enc_chain_2w(int o1, int nx, uint32_t A);       // runs k_enc_chain2w
uint32_t enc_2w_lds_bytes(int o1, uint32_t A);
hipError_t launch_enc_chain2w(const EncJob *d_jobs, int njobs, uint32_t lds, hipStream_t s);
uint32_t dec_lds_bytes(uint32_t rows, int bits, int mode);
hipError_t launch_enc_chain(const EncJob *d_jobs, int njobs, uint32_t lds, hipStream_t s);
// d_items: uint32 pairs {job index, first chunk}
hipError_t launch_enc_replay(const EncJob *d_jobs, const uint32_t *d_items, int nitems,
                             bool emit, uint32_t lds, hipStream_t s);
hipError_t launch_enc_scan(const EncJob *d_jobs, int njobs, hipStream_t s);
hipError_t launch_dec(const DecJob *d_jobs, int njobs, uint32_t lds, hipStream_t s);

}  // namespace fqz5
