// rans_decompress.cpp — host planner for batched GPU decompression with the
// semantics of htscodecs rans_uncompress_to_4x16 (rANS_static4x16pr.c:
// 1607-1894).  Stream headers are parsed on the host; the rANS chains,
// RLE expansion, un-packing and stripe interleave run on the GPU, one
// launch per stage for the whole batch:
//   A  O0 chains of compressed order-1 tables   (only when present)
//   B  all O0 / O1 chains (main data and RLE meta-data)
//   C  RLE expansion, D  un-packing, E  stripe interleave.
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <algorithm>
#include <climits>
#include <cstring>

#include "kernels.h"
#include "rans_codec.hpp"
#include "rans_format.hpp"

namespace fqz5 {

namespace {

struct DJ {                         // one entropy stream to decode
    const uint8_t *h = nullptr;     // host view of the stream (table first)
    const uint8_t *d = nullptr;     // device view
    uint32_t len = 0;               // bytes from the table to the stream end
    uint32_t n = 0;                 // decoded size
    bool o1 = false;
    int nx = 4;
    uint8_t *d_out = nullptr;
    // parsed
    int bits = 12;
    uint32_t tab_len = 0;           // bytes before the rANS states
    int hdr_dj = -1;                // O1 with a compressed table
    std::vector<uint8_t> hdr;       // decoded table bytes (host)
    std::vector<uint32_t> F;        // normalised freqs: rows x 256
    std::vector<uint8_t> alpha;     // O1 contexts
    bool ok = true;
};

struct Node {
    const uint8_t *h = nullptr, *d = nullptr;
    uint32_t len = 0;
    uint8_t *d_out = nullptr;
    uint32_t out_cap = 0;
    bool ok = false;
    uint32_t out_size = 0;
    // STRIPE
    bool stripe = false;
    unsigned N = 0;
    uint32_t ulen = 0;
    std::vector<int> kids;
    uint8_t *d_tmp = nullptr;
    // leaf
    bool pack = false, rle = false, cat = false;
    int per = 1;
    uint8_t map[256] = {0};
    uint32_t osz = 0, ent_n = 0;    // final size, entropy-stage size
    uint32_t lit_len = 0, meta_len = 0;
    const uint8_t *h_meta = nullptr;   // raw meta on host
    const uint8_t *d_meta = nullptr;   // meta on device (raw or decoded)
    int dj_meta = -1, dj_main = -1;
    uint8_t *d_ent = nullptr;       // entropy-stage output
    uint8_t *d_unrle = nullptr;     // RLE-stage output
    const uint8_t *d_cat = nullptr; // CAT payload (device)
    uint32_t unrle_len = 0;
};

class Decompressor {
  public:
    explicit Decompressor(GpuCtx &g) : g_(g) {}
    void run(std::vector<DecompressReq> &reqs);

  private:
    GpuCtx &g_;
    std::vector<Node> nodes_;
    std::vector<DJ> djs_;

    int parse(const uint8_t *h, const uint8_t *d, uint32_t len, uint8_t *d_out,
              uint32_t out_cap, int depth);
    int add_dj(const uint8_t *h, const uint8_t *d, uint32_t len, uint32_t n, bool o1,
               int nx, uint8_t *d_out);
    bool parse_o0_table(DJ &j, const uint8_t *p, const uint8_t *end, uint32_t *used);
    bool parse_o1_table(DJ &j, const uint8_t *p, const uint8_t *end);
    void run_djs(const std::vector<int> &ids);
};

int Decompressor::add_dj(const uint8_t *h, const uint8_t *d, uint32_t len, uint32_t n,
                         bool o1, int nx, uint8_t *d_out) {
    djs_.emplace_back();
    DJ &j = djs_.back();
    j.h = h;
    j.d = d;
    j.len = len;
    j.n = n;
    j.o1 = o1;
    j.nx = nx;
    j.d_out = d_out;
    const int id = int(djs_.size()) - 1;
    if (!n) return id;
    if (!o1) {
        j.ok = parse_o0_table(j, h, h + len, &j.tab_len);
    } else {
        // O1 header byte: shift<<4 | compressed (rANS_static4x16pr.c:572-587)
        if (len < 1) { j.ok = false; return id; }
        j.bits = h[0] >> 4;
        if (j.bits != 10 && j.bits != 12) { j.ok = false; return id; }
        if (h[0] & 1) {
            uint32_t u, c, p = 1;
            p += varint_get(h + p, h + len, &u);
            p += varint_get(h + p, h + len, &c);
            if (c > len - p) { j.ok = false; return id; }
            j.tab_len = p + c;
            uint8_t *d_hdr = g_.arena.alloc_n<uint8_t>(u + 1);
            int hid = add_dj(h + p, d + p, c, u, false, 4, d_hdr);
            djs_[id].hdr_dj = hid;
        } else {
            DJ &jj = djs_[id];
            jj.ok = parse_o1_table(jj, h + 1, h + len);
        }
    }
    return id;
}

// decode_freq + normalise_freq_shift (rANS_static4x16pr.c:261-285)
bool Decompressor::parse_o0_table(DJ &j, const uint8_t *p, const uint8_t *end,
                                  uint32_t *used) {
    uint32_t F[256] = {0}, tot = 0;
    int k = get_freq0(p, end, F, &tot);
    if (!k) return false;
    scale_pow2(F, tot, 4096);
    uint32_t x = 0;
    for (int s = 0; s < 256; s++) x += F[s];
    if (x != 4096) return false;
    j.bits = 12;
    j.F.assign(F, F + 256);
    *used = uint32_t(k);
    return true;
}

// decode_freq1 (rANS_static16_int.h:468-536).  Sets tab_len for the
// uncompressed case.
bool Decompressor::parse_o1_table(DJ &j, const uint8_t *p0, const uint8_t *end) {
    const uint8_t *p = p0;
    uint32_t A[256] = {0};
    int k = get_alphabet(p, end, A);
    if (!k) return false;
    p += k;
    if (p >= end) return false;
    j.alpha.clear();
    for (int s = 0; s < 256; s++)
        if (A[s]) j.alpha.push_back(uint8_t(s));
    if (j.alpha.empty() || j.alpha[0] != 0) return false;
    j.F.assign(j.alpha.size() * 256, 0);
    for (size_t r = 0; r < j.alpha.size(); r++) {
        uint32_t F[256] = {0}, T = 0;
        k = get_freq_row(p, end, A, F, &T);
        if (!k) return false;
        p += k;
        if (!T) continue;
        scale_pow2(F, T, 1u << j.bits);
        uint32_t x = 0;
        for (int s = 0; s < 256; s++) x += F[s];
        if (x != (1u << j.bits)) return false;
        std::memcpy(&j.F[r * 256], F, sizeof F);
    }
    if (j.hdr_dj < 0) j.tab_len = 1 + uint32_t(p - p0);
    return true;
}

// Parse one stream (rans_uncompress_to_4x16).  out_cap is *out_size: the
// output capacity, and the size itself for NOSZ streams.
int Decompressor::parse(const uint8_t *h, const uint8_t *d, uint32_t len, uint8_t *d_out,
                        uint32_t out_cap, int depth) {
    nodes_.emplace_back();
    const int id = int(nodes_.size()) - 1;
    {
        Node &N = nodes_[id];
        N.h = h; N.d = d; N.len = len; N.d_out = d_out; N.out_cap = out_cap;
    }
    if (!len) return id;
    const uint8_t *end = h + len;
    if (h[0] & ORD_STRIPE) {                     // :1615-1694
        if (depth > 0) return id;                // fqzcomp5 never nests stripes
        uint32_t ulen, p = 1;
        p += varint_get(h + p, end, &ulen);
        if (p >= len) return id;
        unsigned N = h[p++];
        if (N < 1 || ulen != out_cap) return id;
        uint32_t clen[256], ulenN[256], idxN[256];
        uint64_t ctot = 0;
        for (unsigned i = 0; i < N; i++) {
            ulenN[i] = ulen / N + ((ulen % N) > i);
            idxN[i] = i ? idxN[i - 1] + ulenN[i - 1] : 0;
            p += varint_get(h + p, end, &clen[i]);
            ctot += clen[i];
            if (p > len || clen[i] > len || clen[i] < 1) return id;
        }
        if (p + ctot > len) return id;
        const uint32_t lim = uint32_t(p + ctot);
        uint8_t *d_tmp = g_.arena.alloc_n<uint8_t>(ulen + 1);
        std::vector<int> kids;
        for (unsigned i = 0; i < N; i++) {
            kids.push_back(parse(h + p, d + p, lim - p, d_tmp + idxN[i], ulenN[i], depth + 1));
            p += clen[i];
        }
        Node &S = nodes_[id];
        S.stripe = true;
        S.N = N;
        S.ulen = ulen;
        S.kids = std::move(kids);
        S.d_tmp = d_tmp;
        S.ok = true;
        return id;
    }
    const int order = h[0];
    uint32_t p = 1;
    uint32_t osz;
    if (!(order & ORD_NOSZ)) p += varint_get(h + p, end, &osz);
    else osz = out_cap;
    if (osz > out_cap) return id;
    Node L;
    L.h = h; L.d = d; L.len = len; L.d_out = d_out; L.out_cap = out_cap;
    L.osz = osz;
    L.pack = order & ORD_PACK;
    L.rle = order & ORD_RLE;
    L.cat = order & ORD_CAT;
    const bool x32 = order & ORD_X32, o1 = order & 1;
    uint32_t ent_n = osz;
    if (L.pack) {                                // hts_unpack_meta (pack.c:161)
        if (p >= len) return id;
        unsigned ns = h[p] ? h[p] : 256;
        L.per = ns <= 1 ? 0 : ns <= 2 ? 8 : ns <= 4 ? 4 : ns <= 16 ? 2 : 1;
        if (L.per != 1) {
            if (p + 1 + ns > len) return id;
            std::memcpy(L.map, h + p + 1, ns);
            p += 1 + ns;
        } else {
            p += 1;
        }
        uint32_t pl;
        p += varint_get(h + p, end, &pl);
        if (pl > osz) return id;
        ent_n = pl;
    }
    if (L.rle) {                                 // :1810-1834
        uint32_t um, rl, cm;
        p += varint_get(h + p, end, &um);
        p += varint_get(h + p, end, &rl);
        if (rl > ent_n) return id;
        if (um & 1) {
            L.meta_len = um / 2;
            if (L.meta_len > len - p) L.meta_len = len - p;
            L.h_meta = h + p;
            L.d_meta = d + p;
            cm = L.meta_len;
        } else {
            p += varint_get(h + p, end, &cm);
            L.meta_len = um / 2;
            if (cm > len - p) return id;
            uint8_t *d_m = g_.arena.alloc_n<uint8_t>(L.meta_len + 1);
            L.dj_meta = add_dj(h + p, d + p, len - p, L.meta_len, false, x32 ? 32 : 4, d_m);
            L.d_meta = d_m;
        }
        if (cm > len - p) return id;
        p += cm;
        L.lit_len = rl;
        ent_n = rl;
    }
    L.ent_n = ent_n;
    const uint32_t rest = len - p;
    if (!rest) {
        L.ent_n = 0;
    } else if (L.cat) {
        if (ent_n > rest) return id;
        L.d_cat = d + p;
    }
    // entropy stage output: straight to d_out when nothing follows
    if (L.pack || L.rle) L.d_ent = g_.arena.alloc_n<uint8_t>(L.ent_n + 1);
    else L.d_ent = d_out;
    if (rest && !L.cat && L.ent_n)
        L.dj_main = add_dj(h + p, d + p, rest, L.ent_n, o1, x32 ? 32 : 4, L.d_ent);
    else if (rest && !L.cat && !L.ent_n)
        L.dj_main = -1;
    L.ok = true;
    nodes_[id] = std::move(L);
    return id;
}

// $FQZ5_NO_REGDEC / $FQZ5_NO_XCD_GROUP: the table-in-LDS O0 decoder and the
// plain hedge order instead (A/B measurements)
static bool reg_decoder() {
    static const bool on = std::getenv("FQZ5_NO_REGDEC") == nullptr;
    return on;
}
static bool xcd_grouping() {
    static const bool on = std::getenv("FQZ5_NO_XCD_GROUP") == nullptr;
    return on;
}

// The O1 register decoder's keys (rans_chain.hip dec4_o1reg_body): every
// context row complete (its frequencies cover the 2^bits slots), at most 8
// contexts with 12-bit slots or 16 with <= 10, at most DEC_O1KEY_MAX (context,
// symbol) pairs.  Off unless $FQZ5_O1REG=1: measured slower than the LDS
// table step (NovaSeq qualities, one stream: 101.7 against 65.8 ns per
// step; the -5 launch 146 against 94), DESIGN.md section 4.
static bool o1reg_decoder() {
    static const bool on = [] {
        const char *e = std::getenv("FQZ5_O1REG");
        return e && e[0] == '1';
    }();
    return on;
}
static bool o1_keys(const DJ &j, DecJob &d) {
    const uint32_t rows = uint32_t(j.alpha.size()), M = 1u << j.bits;
    if (j.bits > 12 || rows > (j.bits == 12 ? 8u : 16u)) return false;
    const uint32_t rowsh = j.bits == 12 ? 29u : 28u;
    uint32_t nk = 0;
    for (uint32_t r = 0; r < rows; r++) {
        const uint32_t *F = &j.F[size_t(r) * 256];
        uint32_t x = 0;
        for (uint32_t s = 0; s < 256; s++) {
            if (!F[s]) continue;
            const auto it = std::lower_bound(j.alpha.begin(), j.alpha.end(), uint8_t(s));
            if (it == j.alpha.end() || *it != s || nk >= DEC_O1KEY_MAX || F[s] > M) return false;
            const uint32_t sym = uint32_t(it - j.alpha.begin());
            d.okey[nk++] = r << rowsh | x << 16 | (0xffffu - ((F[s] - 1) << 4 | sym));
            x += F[s];
        }
        if (x != M) return false;
    }
    if (!nk) return false;
    const uint32_t nk16 = (nk + 15) & ~15u;
    for (uint32_t k = nk; k < nk16; k++) d.okey[k] = d.okey[0];
    d.okeys = nk16;
    d.rowsh = rowsh;
    return true;
}

void Decompressor::run_djs(const std::vector<int> &ids) {
    std::vector<uint32_t> tabs;
    std::vector<uint8_t> alphas;
    struct Off { size_t tab, alpha; };
    std::vector<Off> offs;
    std::vector<int> used;
    // table image offsets first, then every job's table in parallel
    for (int id : ids) {
        DJ &j = djs_[id];
        if (!j.ok || !j.n) continue;
        const size_t rows = j.o1 ? j.alpha.size() : 1;
        const uint32_t mode = dec_table_mode(j.o1, uint32_t(rows), j.bits);
        Off o{tabs.size(), alphas.size()};
        tabs.resize(tabs.size() + dec_tab_words(mode, uint32_t(rows), j.bits), 0);
        if (j.o1) alphas.insert(alphas.end(), j.alpha.begin(), j.alpha.end());
        offs.push_back(o);
        used.push_back(id);
    }
    host_parallel(used.size(), [&](size_t k) {
        DJ &j = djs_[used[k]];
        const uint32_t M = 1u << j.bits;
        const size_t rows = j.o1 ? j.alpha.size() : 1;
        const uint32_t mode = dec_table_mode(j.o1, uint32_t(rows), j.bits);
        uint32_t *t = &tabs[offs[k].tab];
        // LDS/GLOBAL: [u32 per slot];  SPLIT: [u8 per slot][u32 fb]
        uint8_t *tsym = reinterpret_cast<uint8_t *>(t);
        uint32_t *tfb = t + rows * M / 4;
        const uint32_t rpl = dec_rp_log(uint32_t(rows));
        for (size_t r = 0; r < rows; r++) {
            const uint32_t *F = &j.F[r * 256];
            uint32_t x = 0;
            for (int s = 0; s < 256; s++) {
                if (!F[s]) continue;
                uint32_t sym = s;
                if (j.o1) {    // alphabet index of s
                    auto it = std::lower_bound(j.alpha.begin(), j.alpha.end(), uint8_t(s));
                    if (it == j.alpha.end() || *it != s) { j.ok = false; break; }
                    sym = uint32_t(it - j.alpha.begin());
                }
                if (mode == DEC_TAB_SPLIT) tfb[(r << rpl) + sym] = ((F[s] - 1) << 16) | x;
                for (uint32_t y = 0; y < F[s] && x + y < M; y++) {
                    if (mode == DEC_TAB_SPLIT)
                        tsym[r * M + x + y] = uint8_t(sym);
                    else
                        t[r * M + x + y] = ((F[s] - 1) << (j.bits + 8)) | (y << 8) | sym;
                }
                x += F[s];
            }
        }
    });
    if (used.empty()) return;
    const uint32_t *d_tabs = g_.upload(tabs);
    const uint8_t *d_alpha = alphas.empty() ? nullptr : g_.upload(alphas);
    int32_t *d_status = g_.arena.alloc_n<int32_t>(used.size());
    g_.memset0(d_status, used.size() * 4);
    // One launch: every stream is a latency-bound chain on its own wave, so
    // occupancy does not matter and the launch carries the largest table.
    std::vector<DecJob> djs;
    uint32_t lds = 0;
    std::vector<size_t> ord;
    for (size_t k = 0; k < used.size(); k++) {
        DJ &j = djs_[used[k]];
        if (j.len < j.tab_len + 4u * j.nx) { j.ok = false; continue; }
        ord.push_back(k);
    }
    // longest chains first so they start in the first dispatch wave
    std::stable_sort(ord.begin(), ord.end(), [&](size_t a, size_t b) {
        return djs_[used[a]].n / djs_[used[a]].nx > djs_[used[b]].n / djs_[used[b]].nx;
    });
    double bytes = 0;
    for (size_t k : ord) {
        DJ &j = djs_[used[k]];
        const uint32_t rows = j.o1 ? uint32_t(j.alpha.size()) : 1u;
        const uint32_t mode = dec_table_mode(j.o1, rows, j.bits);
        djs.push_back(DecJob{j.d + j.tab_len, d_tabs + offs[k].tab,
                             j.o1 ? d_alpha + offs[k].alpha : nullptr, j.d_out, d_status + k,
                             j.len - j.tab_len, j.n, j.nx, j.bits, rows, mode, nullptr, 0, {}});
        if (!j.o1 && j.nx == 4 && reg_decoder()) {
            // the register decoder: <= 8 symbols that cover every slot
            DecJob &d = djs.back();
            uint32_t k2 = 0, x = 0;
            for (int s = 0; s < 256 && k2 <= DEC_REG_MAX; s++) {
                if (!j.F[s]) continue;
                if (k2 < DEC_REG_MAX) d.reg[k2] = x | (j.F[s] << 16);
                k2++;
                x += j.F[s];
            }
            if (k2 >= 1 && k2 <= DEC_REG_MAX && x == (1u << j.bits)) d.nreg = k2;
        }
        if (j.o1 && j.nx == 4 && o1reg_decoder() && o1_keys(j, djs.back()))
            lds = std::max(lds, DEC_O1REG_LDS_BYTES);
        bytes += double(j.n) + (j.len - j.tab_len);
        lds = std::max(lds, dec_lds_bytes(rows, j.bits, int(mode)));
    }
    EventPair ev((g_.prof.on || prof_on()) && !ord.empty(), g_.stream);
    // hedge: the long streams several times on different CUs, while the
    // copies fit one per CU (hedge_plan)
    // a chain's cost: its steps, those of the table decoders weighted by
    // their time per step against the O0 register decoder's
    // ($FQZ5_HEDGE_TABW; 1 = by steps alone)
    static const double tabw = [] {
        const char *e = std::getenv("FQZ5_HEDGE_TABW");
        return e ? std::atof(e) : 1.0;
    }();
    std::vector<double> steps;
    for (const DecJob &d : djs)
        steps.push_back(double(d.n / uint32_t(d.nx)) * (d.nreg ? 1.0 : tabw));
    HedgeShare share(size_t(g_.cus));          // held until the launch is synchronised
    const std::vector<int> cp = hedge_plan(steps, share.cus);
    if (std::any_of(cp.begin(), cp.end(), [](int c) { return c > 1; })) {
        const size_t nj = djs.size();
        uint32_t *d_done = g_.arena.alloc_n<uint32_t>(nj);
        g_.memset0(d_done, nj * 4);
        for (size_t k = 0; k < nj; k++) djs[k].done = d_done + k;
        // every copy of a stream on one XCD (xcd_layout), padding jobs nx = 0
        const std::vector<int> pos = xcd_grouping() ? xcd_layout(cp, share.cus)
                                                    : std::vector<int>();
        if (!pos.empty()) {
            std::vector<DecJob> laid(pos.size());
            for (size_t i = 0; i < pos.size(); i++) {
                if (pos[i] >= 0) laid[i] = djs[size_t(pos[i])];
                else { laid[i] = djs[0]; laid[i].nx = 0; }
            }
            djs.swap(laid);
        } else {
            for (size_t k = 0; k < nj; k++)
                for (int c = 1; c < cp[k]; c++) djs.push_back(djs[k]);
        }
    }
    lds = g_.chain_lds(lds, djs.size());
    if (!djs.empty()) FQZ5_HIP(launch_dec(g_.upload(djs), int(djs.size()), lds, g_.stream));
    ev.stop(g_.stream);
    std::vector<int32_t> st(used.size());
    g_.download(st.data(), d_status, st.size());
    g_.sync();
    if (ev.on) {
        const double ms = ev.ms();
        g_.prof.dec_ms += ms;
        g_.prof.dec_launches += 1;
        g_.prof.dec_bytes += bytes;
        if (prof_on()) prof_add(PK_RANS_DEC, ms, bytes);
    }
    for (size_t k = 0; k < used.size(); k++)
        if (st[k]) djs_[used[k]].ok = false;
}

// $FQZ5_STEP_TRACE: host wall time of the decode phases on stderr
static bool step_trace() {
    static const bool on = std::getenv("FQZ5_STEP_TRACE") != nullptr;
    return on;
}
static double now_ms() {
    return std::chrono::duration<double, std::milli>(
               std::chrono::steady_clock::now().time_since_epoch()).count();
}

void Decompressor::run(std::vector<DecompressReq> &reqs) {
    const double t0 = step_trace() ? now_ms() : 0;
    std::vector<int> roots;
    for (auto &r : reqs) {
        r.ok = false;
        r.out_size = 0;
        roots.push_back(parse(r.h_in, r.d_in, r.in_size, r.d_out, r.out_cap, 0));
    }
    const double t1 = step_trace() ? now_ms() : 0;
    // A: compressed order-1 tables
    std::vector<int> hdr;
    for (size_t i = 0; i < djs_.size(); i++)
        if (djs_[i].hdr_dj >= 0) hdr.push_back(djs_[i].hdr_dj);
    if (!hdr.empty()) {
        run_djs(hdr);
        for (size_t i = 0; i < djs_.size(); i++) {
            DJ &j = djs_[i];
            if (j.hdr_dj < 0) continue;
            DJ &hj = djs_[j.hdr_dj];
            if (!hj.ok) { j.ok = false; continue; }
            j.hdr.resize(hj.n);
            g_.download(j.hdr.data(), hj.d_out, hj.n);
        }
        g_.sync();
        for (size_t i = 0; i < djs_.size(); i++) {
            DJ &j = djs_[i];
            if (j.hdr_dj < 0 || !j.ok) continue;
            j.ok = parse_o1_table(j, j.hdr.data(), j.hdr.data() + j.hdr.size());
        }
    }
    // B: all remaining chains
    std::vector<int> rest;
    std::vector<char> is_hdr(djs_.size(), 0);
    for (int h : hdr) is_hdr[h] = 1;
    for (size_t i = 0; i < djs_.size(); i++)
        if (!is_hdr[i]) rest.push_back(int(i));
    const double t2 = step_trace() ? now_ms() : 0;
    run_djs(rest);
    const double t3 = step_trace() ? now_ms() : 0;

    // CAT payloads
    std::vector<CopyItem> cps;
    for (auto &N : nodes_) {
        if (N.stripe || !N.ok) continue;
        if (N.dj_main >= 0 && !djs_[N.dj_main].ok) N.ok = false;
        if (N.dj_meta >= 0 && !djs_[N.dj_meta].ok) N.ok = false;
        if (N.d_cat)
            for (uint32_t o = 0; o < N.ent_n; o += 65536)
                cps.push_back({N.d_cat + o, N.d_ent + o, std::min<uint32_t>(65536, N.ent_n - o), 0});
    }
    if (!cps.empty()) FQZ5_HIP(launch_copy(g_.upload(cps), int(cps.size()), g_.stream));

    // C: RLE expansion (rle.c:142-189).  Meta = [nsyms][syms][run varints].
    std::vector<int> rl;
    std::vector<const uint8_t *> probes;
    for (size_t i = 0; i < nodes_.size(); i++) {
        Node &N = nodes_[i];
        if (!N.stripe && N.ok && N.rle) {
            if (!N.meta_len) { N.ok = false; continue; }
            rl.push_back(int(i));
        }
    }
    if (!rl.empty()) {
        // RLE symbol lists (first bytes of each meta block) to the host
        std::vector<std::vector<uint8_t>> mh(rl.size());
        for (size_t k = 0; k < rl.size(); k++) {
            Node &N = nodes_[rl[k]];
            uint32_t m = std::min<uint32_t>(N.meta_len, 257);
            mh[k].resize(m);
            if (N.h_meta) std::memcpy(mh[k].data(), N.h_meta, m);
            else g_.download(mh[k].data(), N.d_meta, m);
        }
        g_.sync();
        std::vector<UnRleItem> items;
        std::vector<uint8_t> saved;
        std::vector<int> who;
        std::vector<uint32_t> ci_lit, ci_run;
        for (size_t k = 0; k < rl.size(); k++) {
            Node &N = nodes_[rl[k]];
            unsigned ns = mh[k][0] ? mh[k][0] : 256;
            if (N.meta_len < 1 + ns) { N.ok = false; continue; }
            uint8_t sv[256] = {0};
            for (unsigned s = 0; s < ns; s++) sv[mh[k][1 + s]] = 1;
            saved.insert(saved.end(), sv, sv + 256);
            const uint32_t nrun = N.meta_len - 1 - ns;
            N.d_unrle = N.pack ? g_.arena.alloc_n<uint8_t>(N.osz + 1) : N.d_out;
            UnRleItem it{N.d_ent, N.d_meta + 1 + ns, nullptr,
                         g_.arena.alloc_n<uint32_t>(nrun + 1), N.d_unrle,
                         N.ent_n, nrun, 0, N.osz};
            const uint32_t w = uint32_t(items.size());
            for (uint32_t c = 0; c * RLE_CHUNK < std::max<uint32_t>(N.ent_n, 1); c++) {
                ci_lit.push_back(w);
                ci_lit.push_back(c);
            }
            for (uint32_t c = 0; c * RLE_CHUNK < nrun; c++) {
                ci_run.push_back(w);
                ci_run.push_back(c);
            }
            items.push_back(it);
            who.push_back(rl[k]);
        }
        if (!items.empty()) {
            uint8_t *d_saved = g_.upload(saved);
            for (size_t k = 0; k < items.size(); k++) items[k].saved = d_saved + 256 * k;
            const int nl = int(ci_lit.size() / 2), nr = int(ci_run.size() / 2);
            // pass 1: RLE literals per literal chunk; terminators per run chunk
            UnRleItem *d_items = g_.upload(items);
            uint32_t *d_cil = g_.upload(ci_lit), *d_cir = g_.upload(ci_run);
            uint32_t *d_cl = g_.arena.alloc_n<uint32_t>(nl + 1);
            uint32_t *d_cr = g_.arena.alloc_n<uint32_t>(nr + 1);
            FQZ5_HIP(launch_unrle_count(d_items, d_cil, nl, d_cl, 0, g_.stream));
            FQZ5_HIP(launch_unrle_count(d_items, d_cir, nr, d_cr, 1, g_.stream));
            std::vector<uint32_t> cl(nl), cr(nr);
            g_.download(cl.data(), d_cl, nl);
            g_.download(cr.data(), d_cr, nr);
            g_.sync();
            // scans per item
            std::vector<uint32_t> coff_lit(2 * size_t(nl)), coff_run(nr);
            {
                std::vector<uint64_t> acc(items.size(), 0);
                for (int c = 0; c < nr; c++) {
                    uint32_t w = ci_run[2 * c];
                    coff_run[c] = uint32_t(acc[w]);
                    acc[w] += cr[c];
                }
                for (size_t k = 0; k < items.size(); k++) items[k].nvarint = uint32_t(acc[k]);
                std::fill(acc.begin(), acc.end(), 0);
                for (int c = 0; c < nl; c++) {
                    uint32_t w = ci_lit[2 * c];
                    coff_lit[2 * c] = uint32_t(acc[w]);
                    acc[w] += cl[c];
                }
            }
            d_items = g_.upload(items);
            FQZ5_HIP(launch_unrle_vend(d_items, d_cir, nr, g_.upload(coff_run), g_.stream));
            // pass 3: output size per literal chunk
            uint32_t *d_coff = g_.upload(coff_lit);
            FQZ5_HIP(launch_unrle_expand(d_items, d_cil, nl, d_coff, d_cl, 0, g_.stream));
            g_.download(cl.data(), d_cl, nl);
            g_.sync();
            {
                std::vector<uint64_t> acc(items.size(), 0);
                for (int c = 0; c < nl; c++) {
                    uint32_t w = ci_lit[2 * c];
                    coff_lit[2 * c + 1] = uint32_t(acc[w]);
                    acc[w] += cl[c];
                }
                for (size_t k = 0; k < items.size(); k++) {
                    Node &N = nodes_[who[k]];
                    N.unrle_len = uint32_t(acc[k]);
                    if (acc[k] > N.osz) N.ok = false;     // rle.c:171 overflow
                }
            }
            FQZ5_HIP(launch_unrle_expand(d_items, d_cil, nl, g_.upload(coff_lit), d_cl, 1,
                                         g_.stream));
        }
    }
    // D: un-packing (pack.c:207-344)
    {
        std::vector<PackItem> items;
        std::vector<uint8_t> maps;
        uint32_t max_n = 0;
        for (auto &N : nodes_) {
            if (N.stripe || !N.ok || !N.pack) continue;
            const uint8_t *src = N.rle ? N.d_unrle : N.d_ent;
            const uint32_t srclen = N.rle ? N.unrle_len : N.ent_n;
            if (N.per == 1) {   // >16 symbols: stored raw
                items.push_back({src, N.d_out, nullptr, srclen, -1});
                N.out_size = srclen;
            } else {
                if (N.per && (uint64_t(N.osz) + N.per - 1) / N.per > srclen) { N.ok = false; continue; }
                items.push_back({src, N.d_out, nullptr, N.osz, N.per});
                N.out_size = N.osz;
            }
            maps.insert(maps.end(), N.map, N.map + 256);
            max_n = std::max(max_n, items.back().n);
        }
        if (!items.empty()) {
            uint8_t *d_maps = g_.upload(maps);
            std::vector<CopyItem> raw;
            std::vector<PackItem> real;
            for (size_t k = 0; k < items.size(); k++) {
                items[k].code = d_maps + 256 * k;
                if (items[k].per < 0) {
                    for (uint32_t o = 0; o < items[k].n; o += 65536)
                        raw.push_back({items[k].in + o, items[k].out + o,
                                       std::min<uint32_t>(65536, items[k].n - o), 0});
                } else {
                    real.push_back(items[k]);
                }
            }
            if (!real.empty())
                FQZ5_HIP(launch_pack(g_.upload(real), int(real.size()), max_n, true, g_.stream));
            if (!raw.empty()) FQZ5_HIP(launch_copy(g_.upload(raw), int(raw.size()), g_.stream));
        }
    }
    for (auto &N : nodes_) {
        if (N.stripe || !N.ok || N.pack) continue;
        N.out_size = N.rle ? N.unrle_len : N.ent_n;
    }
    // E: stripe interleave (utils.h:79 unstripe)
    std::vector<StripeItem> si;
    uint32_t max_n = 0;
    for (auto &S : nodes_) {
        if (!S.stripe || !S.ok) continue;
        for (unsigned i = 0; i < S.N; i++) {
            Node &K = nodes_[S.kids[i]];
            const uint32_t want = S.ulen / S.N + ((S.ulen % S.N) > i);
            if (!K.ok || K.out_size != want) S.ok = false;
        }
        if (!S.ok) continue;
        si.push_back({S.d_tmp, S.d_out, S.ulen, S.N, 1, 0});
        max_n = std::max(max_n, S.ulen);
        S.out_size = S.ulen;
    }
    if (!si.empty()) FQZ5_HIP(launch_stripe(g_.upload(si), int(si.size()), max_n, g_.stream));
    g_.sync();
    if (step_trace())
        std::fprintf(stderr, "decode: parse %.1f ms, o1 headers %.1f ms, chains %.1f ms, "
                     "post %.1f ms (%zu streams, %zu chains)\n", t1 - t0, t2 - t1, t3 - t2,
                     now_ms() - t3, reqs.size(), djs_.size());
    for (size_t i = 0; i < reqs.size(); i++) {
        Node &N = nodes_[roots[i]];
        reqs[i].ok = N.ok;
        reqs[i].out_size = N.ok ? N.out_size : 0;
    }
}

}  // namespace

void decompress_batch(GpuCtx &g, std::vector<DecompressReq> &reqs) {
    Decompressor d(g);
    d.run(reqs);
}

}  // namespace fqz5
