// names.hpp — fqzcomp5's name section (encode_names / decode_names,
// fqzcomp5.c:1408-1794) in stages, so that every name candidate of a run of
// blocks shares one LZP batch and one rANS batch on the GPU:
//
//   strat 0 (TLZP3)        lzp of the names, rANS order 5
//   strat 1 (TOK3_n)       tok3 of the names at level n
//   strat 2 (TOK3_n_LZP)   tok3 of the read ids, rANS order 129 of the
//                          per-record flags (/1 /2 suffix, comment, space
//                          or tab), lzp + rANS order 5 of the comments
//
// Section bytes: [u32 name_len][u8 strat][u32 clen][payload], strat 2's
// payload [u32 clen1][u32 clenf][tok3][flags][comments].
#pragma once
#include <cstdint>
#include <functional>
#include <vector>

#include "lzp_codec.hpp"
#include "rans_codec.hpp"
#include "tok3.hpp"

namespace fqz5 {

// fqzcomp5.c:190-199
constexpr int M_TLZP3 = 11, M_TOK3_3 = 12, M_TOK3_9 = 15, M_TOK3_3_LZP = 16, M_TOK3_9_LZP = 19;
inline bool is_name_method(int m) { return m >= M_TLZP3 && m <= M_TOK3_9_LZP; }
// compress_with_methods' encode_names arguments (fqzcomp5.c:2023-2045)
inline int name_strat(int m) { return m == M_TLZP3 ? 0 : m <= M_TOK3_9 ? 1 : 2; }
inline int name_level(int m) {
    return m == M_TLZP3 ? (m - M_TOK3_3) * 2 + 3 : m <= M_TOK3_9 ? (m - M_TOK3_3) * 2 + 3
                                                                  : (m - M_TOK3_3_LZP) * 2 + 3;
}

struct NameEnc {
    int strat = 0, level = 0;
    uint32_t name_len = 0;
    bool ok = false;                 // false: encode_names returns NULL
    Tok3Enc tok;
    bool tok_ok = false;
    std::vector<char> ids;           // strat 1: the names; strat 2: the read ids
    std::vector<char> comments;      // strat 2
    std::vector<uint8_t> flag;       // strat 2: one byte per record
    int lzp = -1;                    // its lzp request
    int req_main = -1, req_flag = -1;
    std::vector<uint8_t> out;        // the section bytes
};

// Host stage (any thread): copy / split and tokenise.  h_names: the block's
// names ('\0' after each), len bytes.
void name_prepare(const uint8_t *h_names, uint32_t len, int strat, int level, NameEnc &E,
                  bool pipelined = false);
// = name_split (the copy / split into E.ids) + name_tokenise (found: the
// names' trie searches done beforehand, tok3_search_batch)
void name_split(const uint8_t *h_names, uint32_t len, int strat, int level, NameEnc &E);
void name_tokenise(NameEnc &E, bool pipelined, const T3Found *found);
// Device stage 1: the lzp inputs (strat 0: the names at d_names; strat 2:
// the comments, uploaded).
void name_add_lzp(GpuCtx &g, NameEnc &E, const uint8_t *d_names, std::vector<LzpEncReq> &lz);
// Stage 2, after lzp_encode_batch: every rANS request (tok3 streams, lzp
// outputs at order 5, flags at order 129).  lead: a strat-2 candidate of the
// same section whose requests E shares for everything but the tok3 streams
// (E's level differs).
void name_add_requests(GpuCtx &g, NameEnc &E, const std::vector<LzpEncReq> &lz,
                       std::vector<CompressReq> &reqs, const NameEnc *lead = nullptr);
// Stage 3, after compress_batch: E.out, E.ok.
void name_assemble(GpuCtx &g, NameEnc &E, const std::vector<CompressReq> &reqs);
// All stages for a set of candidates on context g (hosts stages on up to
// 16 threads).  h_names[k] / d_names[k]: candidate k's names; ready[k]
// (optional): an event after which h_names[k] holds them (a download still
// in flight when the batch starts).
void names_encode_batch(GpuCtx &g, std::vector<NameEnc> &jobs,
                        const std::vector<const uint8_t *> &h_names,
                        const std::vector<const uint8_t *> &d_names,
                        const std::vector<uint32_t> &lens, const std::vector<int> &methods,
                        const std::vector<hipEvent_t> *ready = nullptr);

struct NameDec {
    const uint8_t *comp = nullptr;   // host: the payload after [u_len][strat][c_len]
    const uint8_t *d_comp = nullptr; // device copy (or nullptr)
    uint32_t c_len = 0, u_len = 0;
    int strat = 0;
    bool ok = false;
    Tok3Dec tok;
    uint32_t clen1 = 0, clenf = 0, clen2 = 0;
    int req_main = -1, req_flag = -1;    // strat 0: the lzp stream; strat 2: comments / flags
    uint8_t *d_rout = nullptr, *d_flag = nullptr;
    uint32_t rout_len = 0, flag_len = 0;
    int lzp = -1;
    uint8_t *d_lout = nullptr;
    // The host buffers below live in the fetching context's pinned staging
    // (name_dec_fetch; valid until that context's reset): the decoded names
    // of a -5 NovaSeq run are ~590 MB a step, and as fresh pageable vectors
    // their page faults and unmapping cost ~90 ms after the decode's last
    // kernel (and their upload ran at pageable speed).
    uint8_t *names = nullptr;        // u_len bytes (strat 2: room for the stitch)
    std::vector<uint32_t> flags;     // strat 2: FQZ_FREAD2 per decoded record
    int nrec = 0;                    // strat 2: decode_names' *out_num_records
    bool fetched = false;            // name_dec_fetch: the device outputs on the host
    uint8_t *fl = nullptr, *out2 = nullptr;   // strat 2: flag bytes, comments
    uint32_t fl_len = 0, out2_len = 0;
};

// decode_names (fqzcomp5.c:1588-1794) in stages over a batch.
bool name_dec_parse(NameDec &D);
void name_dec_add_requests(GpuCtx &g, NameDec &D, std::vector<DecompressReq> &reqs);
void name_dec_add_lzp(GpuCtx &g, NameDec &D, const std::vector<DecompressReq> &reqs,
                      std::vector<LzpDecReq> &lz);
// = name_dec_fetch (downloads; serial per context) + name_dec_rebuild
// (host only: any thread).
void name_dec_finish(GpuCtx &g, NameDec &D, const std::vector<DecompressReq> &reqs,
                     const std::vector<LzpDecReq> &lz);
void name_dec_fetch(GpuCtx &g, NameDec &D, const std::vector<DecompressReq> &reqs,
                    const std::vector<LzpDecReq> &lz);
void name_dec_rebuild(NameDec &D);
// fetched (optional) runs once the GPU work is done, before the host rebuild
void names_decode_batch(GpuCtx &g, std::vector<NameDec> &jobs,
                        const std::function<void()> &fetched = {});

}  // namespace fqz5
