// tok3.hpp — the tok3 name tokeniser in stages, so that a caller can code
// the token streams of many name blocks (every name candidate of a run of
// fqzcomp5 blocks) as one GPU batch:
//
//   encode  tok3_tokenise (host) -> tok3_add_requests (uploads, candidate
//           rANS requests appended to the caller's batch) -> compress_batch
//           -> tok3_assemble (smallest candidate per stream, duplicate
//           streams, serialisation: tok3_encode_names' bytes)
//   decode  tok3_dec_parse (host) -> tok3_dec_add_requests -> decompress_batch
//           -> tok3_dec_finish (names rebuilt: tok3_decode_names' bytes)
//
// tok3_encode_names / tok3_decode_names (tok3.cpp) are these stages over a
// batch of one.  use_arith streams are coded inside tok3_assemble /
// tok3_dec_finish (arith_dynamic on the GPU), not through the batch.
#pragma once
#include <cstdint>
#include <utility>
#include <vector>

#include "rans_codec.hpp"
#include "tok3_search.h"

namespace fqz5 {

struct Tok3Enc {
    int level = 0, use_arith = 0;
    int nreads = 0, last_start = 0, max_tok = 1;
    std::vector<std::vector<uint8_t>> desc;                  // [128 * 16], empty = absent
    std::vector<std::vector<std::pair<int, int>>> cand;      // per stream: (method, request)
};

// Tokenise `len` bytes of names ('\n' or '\0' terminated; terminators are
// rewritten to '\0' in place).  false where tok3_encode_names returns NULL.
// pipelined: the trie searches on a second thread, ahead of the coding
// (for callers with host cores to spare; the same result).
// found (optional): every name's trie search done beforehand
// (tok3_search_batch), so only the coding runs here.
bool tok3_tokenise(char *blk, int len, int level, int use_arith, Tok3Enc &T,
                   bool pipelined = false, const T3Found *found = nullptr);

// The trie searches of a batch of name blocks on the GPU (tok3_search.hip):
// per block its names' search results, or ok = false (a block the tokenise
// loop refuses, or one whose checks found a hash collision: search it on
// the host).  h_blk: the block's bytes on the host (its names' extents come
// from there); d_blk: a device copy (or nullptr: h_blk is uploaded).
// h_pinned: a pinned host copy to upload from instead.  split: the block is
// a name section ('\0' after each name) of which the read ids are searched
// (strat 2: name_split's ids, without building them); d_blk required.
struct Tok3SearchJob {
    const char *h_blk = nullptr;
    const uint8_t *d_blk = nullptr;
    const uint8_t *h_pinned = nullptr;
    uint32_t len = 0;
    bool split = false;
    std::vector<T3Found> found;
    bool ok = false;
};
// The names of a block as the tokenise loop visits them (:1487-1505): false
// when the loop fails (a byte that is neither a name byte nor '\0' / '\n')
// or create_context would (no names, more than 10M).
bool tok3_name_extents(const char *blk, uint32_t len, std::vector<uint32_t> &st,
                       std::vector<uint32_t> &ln);
void tok3_search_batch(GpuCtx &g, std::vector<Tok3SearchJob *> &jobs);
// Each stream's candidate methods (compress(), tokenise_name3.c:1268-1417) as
// rANS requests appended to `reqs` (no requests when use_arith).
void tok3_add_requests(GpuCtx &g, Tok3Enc &T, std::vector<CompressReq> &reqs);
// After compress_batch over `reqs`: the serialised tok3 stream.  false where
// the reference fails (a codec returning NULL).
bool tok3_assemble(GpuCtx &g, const Tok3Enc &T, const std::vector<CompressReq> &reqs,
                   std::vector<uint8_t> &out);

struct Tok3Dec {
    const uint8_t *in = nullptr;
    uint32_t sz = 0;
    int ulen0 = 0, nreads = 0, use_arith = 0, max_tok = 1;
    struct Coded { int i; uint32_t off, clen, ulen; };
    std::vector<Coded> coded;
    std::vector<std::pair<int, int>> order;                  // (0 coded / 1 copy / 2 col0, index)
    std::vector<std::pair<int, int>> copies;                 // (to, from)
    size_t req0 = 0;                                         // first request in the batch
    uint8_t *d_out = nullptr;                                // the decoded streams, back to back
    std::vector<size_t> out_off;
    size_t out_tot = 0;
    std::vector<std::vector<uint8_t>> dec;                   // tok3_dec_fetch: host copies
    bool fetched = false;
};

// Parse the stream layout (tokenise_name3.c:1679-1809); false = NULL.
bool tok3_dec_parse(const uint8_t *in, uint32_t sz, Tok3Dec &D);
// The coded streams as rANS decode requests (d_in: a device copy of `in`,
// or nullptr to upload it); none when use_arith.
void tok3_dec_add_requests(GpuCtx &g, Tok3Dec &D, const uint8_t *d_in,
                           std::vector<DecompressReq> &reqs);
// After decompress_batch: the names, '\0' after each; false = NULL.
// = tok3_dec_fetch (the decoded streams to the host; arith streams decoded)
// + tok3_dec_rebuild (host only: any thread).
bool tok3_dec_finish(GpuCtx &g, Tok3Dec &D, const std::vector<DecompressReq> &reqs,
                     std::vector<uint8_t> &out);
bool tok3_dec_fetch(GpuCtx &g, Tok3Dec &D, const std::vector<DecompressReq> &reqs);
bool tok3_dec_rebuild(Tok3Dec &D, std::vector<uint8_t> &out);

// Host copies of device layouts: one gather on the device, one copy down.
void download_layouts(GpuCtx &g, const std::vector<const Layout *> &ls,
                      const std::vector<uint8_t *> &dsts);

}  // namespace fqz5
