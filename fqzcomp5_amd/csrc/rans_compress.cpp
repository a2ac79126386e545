// rans_compress.cpp — host planner for batched GPU compression with the
// exact byte semantics of htscodecs rans_compress_to_4x16
// (rANS_static4x16pr.c:1224-1600).
//
// Every request is decomposed into "leaves" (one non-STRIPE, non-CAT call
// of the reference function; a STRIPE request has one leaf per stripe and
// candidate sub-order) and every leaf into at most two "entropy jobs" (the
// main O0/O1 stream and the O0 stream of its RLE meta-data), plus one O0
// job per order-1 table big enough to be compressed.  Stages:
//   1 stripe transpose + byte histograms     (GPU) -> PACK decision (host)
//   2 bit-packing + histograms               (GPU) -> RLE symbols   (host)
//   3 RLE literal/run counting               (GPU) -> RLE accept    (host)
//   4 RLE emit, O0/O1 histograms             (GPU) -> tables        (host)
//   5 the rANS chains of every job            (GPU, one launch per order)
//   6 layout: CAT fallback, stripe best-of, capacity rules          (host)
// Each stage is one launch over all streams of the batch.  The reference's
// capacity failures (NULL returns) are decided in stage 6 from sizes: they
// never change the bytes of a successful call.
#include <sys/syscall.h>
#include <unistd.h>
#include <algorithm>
#include <map>
#include <chrono>
#include <climits>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <atomic>
#include <exception>
#include <memory>
#include <mutex>
#include <thread>
#include <vector>

#include "kernels.h"
#include "rans_codec.hpp"
#include "rans_format.hpp"

namespace fqz5 {

namespace {

constexpr uint32_t HIST_SLICE = 1u << 17;
constexpr uint32_t HIST1_BIG_SLICE = 1u << 22;   // 16-bit counters that spill (k_hist1<true>)
constexpr uint32_t NONE32 = 0xffffffffu;

struct EJ {                       // one rANS entropy stream to encode
    const uint8_t *d_in = nullptr;
    std::vector<uint8_t> h_in;    // input produced on the host (O1 tables)
    uint32_t n = 0;
    bool o1 = false;
    int nx = 4;
    bool needs_hist = false;
    uint32_t F0[256] = {0};       // order-0 histogram of the input
    // order-1
    int A = 0;
    uint8_t remap[256] = {0};
    uint32_t f1_off = 0;
    uint8_t seg_first[32] = {0};  // in[z*isz] for z >= 1
    uint8_t last_byte = 0;
    // tables
    int bits = 12;
    std::vector<uint8_t> table;   // serialised frequency table
    std::vector<EncSym> syms;     // O0 (host-built)
    std::vector<uint16_t> f1;     // O1: normalised frequencies [A*A], the table is built on the GPU
    int hdr_job = -1;             // O1: job compressing table[1..]
    // kernel output
    uint8_t *d_end = nullptr;
    uint32_t payload = 0;
    Layout layout;                // this job's bytes (table + payload)
};

struct Leaf {
    const uint8_t *d_in = nullptr;
    uint32_t n = 0;
    int order = 0;                // after the entry-point flag adjustments
    uint32_t hist[256] = {0}, eq[256] = {0};
    // PACK
    bool pack = false;
    int per = 0, pmeta_len = 0;
    uint8_t pmeta[257] = {0};
    uint8_t code[256] = {0};
    uint32_t plen = 0;
    uint8_t *d_packed = nullptr;
    uint32_t phist[256] = {0}, peq[256] = {0};
    // data entering RLE / the entropy coder
    const uint8_t *d_cur = nullptr;
    uint32_t n_cur = 0;
    bool x32 = false;
    // RLE
    bool rle = false;
    int nsyms = 0;
    uint8_t saved[256] = {0}, syms[256] = {0};
    uint32_t nchunks = 0, chunk0 = 0;
    uint64_t llen = 0, runs_len = 0;
    uint32_t rmeta = 0;
    uint8_t *d_lits = nullptr, *d_meta = nullptr;
    // entropy
    bool o1 = false;
    int ej_main = -1, ej_meta = -1;
};

struct StripeReq {
    unsigned N = 0;
    uint32_t plen[256] = {0}, pidx[256] = {0};
    uint8_t *d_tr = nullptr;
    std::vector<std::vector<int>> leaves;   // per stripe, in candidate order
};

// varint_put with the reference's end-of-buffer refusal (varint.h:173).
inline int vput(uint8_t *buf, uint32_t pos, uint32_t cap, uint32_t v) {
    uint32_t room = cap > pos ? cap - pos : 0;
    if (room < 5 && room < uint32_t(varint_len(v))) return 0;
    return varint_put(buf + pos, nullptr, v);
}

// Flag adjustments made on entry of rans_compress_to_4x16 (:1256-1265).
inline int entry_flags(int order, uint32_t n) {
    if ((order & ORD_SIMD_AUTO) && n >= 50000 && !(order & ORD_STRIPE)) order |= ORD_X32;
    if (n <= 20) order &= ~ORD_STRIPE;
    if (n <= 1000) order &= ~ORD_X32;
    return order;
}

class Compressor {
  public:
    explicit Compressor(GpuCtx &g) : g_(g) {}
    void run(std::vector<CompressReq> &reqs);
    size_t njobs() const { return jobs_.size(); }

  private:
    GpuCtx &g_;
    std::vector<Leaf> leaves_;
    std::vector<StripeReq> stripes_;
    std::vector<EJ> jobs_;

    int add_leaf(const uint8_t *d, uint32_t n, int order) {
        leaves_.emplace_back();
        Leaf &L = leaves_.back();
        L.d_in = d;
        L.n = n;
        L.order = order;
        return int(leaves_.size()) - 1;
    }
    int add_job(const uint8_t *d, uint32_t n, bool o1, int nx) {
        jobs_.emplace_back();
        EJ &j = jobs_.back();
        j.d_in = d;
        j.n = n;
        j.o1 = o1;
        j.nx = nx;
        return int(jobs_.size()) - 1;
    }

    void hist0(const std::vector<std::pair<const uint8_t *, uint32_t>> &segs,
               std::vector<uint32_t> &counts);
    void gather(const std::vector<const uint8_t *> &ptrs, std::vector<uint8_t> &out);
    void stage_pack();
    void stage_rle();
    void stage_tables();
    void build_o0(EJ &j);
    void build_o1(EJ &j, const uint32_t *cnt);
    void stage_encode();
    void finish_job(EJ &j);
    bool leaf_layout(const Leaf &L, uint32_t cap, Layout &out) const;
    bool stripe_layout(const StripeReq &S, const CompressReq &r, Layout &out) const;
};

// ---------------------------------------------------------------------------
void Compressor::hist0(const std::vector<std::pair<const uint8_t *, uint32_t>> &segs,
                       std::vector<uint32_t> &counts) {
    counts.assign(segs.size() * 512, 0);
    if (segs.empty()) return;
    // the candidates of one section share their input: count each distinct
    // (pointer, length) once
    std::map<std::pair<const uint8_t *, uint32_t>, uint32_t> uniq;
    std::vector<uint32_t> of(segs.size());
    std::vector<HistItem> items;
    for (uint32_t s = 0; s < segs.size(); s++) {
        auto ins = uniq.emplace(segs[s], uint32_t(uniq.size()));
        of[s] = ins.first->second;
        if (!ins.second) continue;
        for (uint32_t b = 0; b < segs[s].second; b += HIST_SLICE)
            items.push_back({segs[s].first, b, std::min(segs[s].second, b + HIST_SLICE), of[s], 0});
    }
    std::vector<uint32_t> u(uniq.size() * 512);
    uint32_t *d_counts = g_.arena.alloc_n<uint32_t>(u.size());
    g_.memset0(d_counts, u.size() * 4);
    if (!items.empty())
        FQZ5_HIP(launch_hist0(g_.upload(items), int(items.size()), d_counts, g_.stream));
    g_.download(u.data(), d_counts, u.size());
    g_.sync();
    for (uint32_t s = 0; s < segs.size(); s++)
        std::memcpy(&counts[size_t(s) * 512], &u[size_t(of[s]) * 512], 2048);
}

void Compressor::gather(const std::vector<const uint8_t *> &ptrs, std::vector<uint8_t> &out) {
    out.assign(ptrs.size(), 0);
    if (ptrs.empty()) return;
    std::vector<GatherItem> items(ptrs.size());
    for (size_t i = 0; i < ptrs.size(); i++) items[i].src = ptrs[i];
    uint8_t *d_out = g_.arena.alloc_n<uint8_t>(ptrs.size());
    FQZ5_HIP(launch_gather(g_.upload(items), int(items.size()), d_out, g_.stream));
    g_.download(out.data(), d_out, out.size());
    g_.sync();
}

// Stages 1-2: byte histograms of every leaf input, the PACK decision
// (pack.c:56-94, entry at rANS_static4x16pr.c:1429-1462) and packing.
void Compressor::stage_pack() {
    std::vector<std::pair<const uint8_t *, uint32_t>> segs;
    for (auto &L : leaves_) segs.push_back({L.d_in, L.n});
    std::vector<uint32_t> cnt;
    hist0(segs, cnt);
    std::vector<PackItem> items;
    std::vector<uint8_t> codes;
    uint32_t max_out = 0;
    // leaves packing the same input (e.g. RANS129 and RANS193 of a section)
    // share one packed copy: same histogram, same codes
    std::map<std::pair<const uint8_t *, uint32_t>, uint8_t *> packed;
    for (size_t i = 0; i < leaves_.size(); i++) {
        Leaf &L = leaves_[i];
        std::memcpy(L.hist, &cnt[i * 512], 1024);
        std::memcpy(L.eq, &cnt[i * 512 + 256], 1024);
        L.d_cur = L.d_in;
        L.n_cur = L.n;
        L.x32 = (L.order & ORD_X32) != 0;
        if (!(L.order & ORD_PACK) || !L.n) continue;
        int ns = 0;
        for (int s = 0; s < 256; s++)
            if (L.hist[s]) { L.code[s] = uint8_t(ns++); L.pmeta[ns] = uint8_t(s); }
        L.pmeta[0] = uint8_t(ns);
        if (ns > 16) continue;
        L.pack = true;
        L.pmeta_len = ns + 1;
        L.per = ns > 4 ? 2 : ns > 2 ? 4 : ns > 1 ? 8 : 0;
        L.plen = L.per ? (L.n + L.per - 1) / L.per : 0;
        auto ins = packed.emplace(std::make_pair(L.d_in, L.n), nullptr);
        if (!ins.second) {
            L.d_packed = ins.first->second;
            continue;
        }
        L.d_packed = ins.first->second = g_.arena.alloc_n<uint8_t>(L.plen + 1);
        if (L.per) {
            codes.insert(codes.end(), L.code, L.code + 256);
            items.push_back({L.d_in, L.d_packed, nullptr, L.n, L.per});
            max_out = std::max(max_out, L.plen);
        }
    }
    if (!items.empty()) {
        uint8_t *d_codes = g_.upload(codes);
        for (size_t k = 0; k < items.size(); k++) items[k].code = d_codes + 256 * k;
        FQZ5_HIP(launch_pack(g_.upload(items), int(items.size()), max_out, false, g_.stream));
    }
    segs.clear();
    std::vector<int> who;
    for (size_t i = 0; i < leaves_.size(); i++) {
        Leaf &L = leaves_[i];
        if (!L.pack) continue;
        L.d_cur = L.d_packed;
        L.n_cur = L.plen;
        if (L.x32 && L.plen < 32) L.x32 = false;   // :1455-1458
        segs.push_back({L.d_packed, L.plen});
        who.push_back(int(i));
    }
    hist0(segs, cnt);
    for (size_t k = 0; k < who.size(); k++) {
        std::memcpy(leaves_[who[k]].phist, &cnt[k * 512], 1024);
        std::memcpy(leaves_[who[k]].peq, &cnt[k * 512 + 256], 1024);
    }
}

// Stages 3-4a: RLE (rle.c:48-138, entry at rANS_static4x16pr.c:1464-1536).
void Compressor::stage_rle() {
    std::vector<int> who;
    for (size_t i = 0; i < leaves_.size(); i++) {
        Leaf &L = leaves_[i];
        if (!(L.order & ORD_RLE) || !L.n_cur) continue;
        const uint32_t *h = L.pack ? L.phist : L.hist;
        const uint32_t *e = L.pack ? L.peq : L.eq;
        // rle_find_syms: +1 per repeat, -1 per non-repeat, keep if > 0
        L.nsyms = 0;
        for (int s = 0; s < 256; s++) {
            int64_t score = 2 * int64_t(e[s]) - int64_t(h[s]);
            L.saved[s] = score > 0;
            if (score > 0) L.syms[L.nsyms++] = uint8_t(s);
        }
        L.nchunks = (L.n_cur + RLE_CHUNK - 1) / RLE_CHUNK;
        who.push_back(int(i));
    }
    if (who.empty()) return;
    std::vector<uint8_t> saved(who.size() * 256);
    std::vector<RleItem> items;
    std::vector<uint32_t> chunk_item;
    uint32_t nch = 0;
    for (size_t k = 0; k < who.size(); k++) {
        Leaf &L = leaves_[who[k]];
        std::memcpy(&saved[k * 256], L.saved, 256);
        L.chunk0 = nch;
        for (uint32_t c = 0; c < L.nchunks; c++) {
            chunk_item.push_back(uint32_t(k));
            chunk_item.push_back(c);
        }
        nch += L.nchunks;
        items.push_back({L.d_cur, nullptr, nullptr, nullptr, L.n_cur, 0});
    }
    uint8_t *d_saved = g_.upload(saved);
    for (size_t k = 0; k < items.size(); k++) items[k].saved = d_saved + 256 * k;
    uint32_t *d_cstat = g_.arena.alloc_n<uint32_t>(5 * size_t(nch));
    FQZ5_HIP(launch_rle_count(g_.upload(items), g_.upload(chunk_item), int(nch), d_cstat,
                              g_.stream));
    std::vector<uint32_t> cs(5 * size_t(nch));
    g_.download(cs.data(), d_cstat, cs.size());
    g_.sync();

    // host scan of the per-chunk totals
    std::vector<uint32_t> cmeta(3 * size_t(nch));
    for (size_t k = 0; k < who.size(); k++) {
        Leaf &L = leaves_[who[k]];
        uint32_t next = L.n_cur;
        for (uint32_t c = L.nchunks; c-- > 0;) {      // successor of each chunk
            cmeta[3 * (L.chunk0 + c) + 2] = next;
            uint32_t f = cs[5 * (L.chunk0 + c) + 1];
            if (f != NONE32) next = f;
        }
        uint64_t lo = 0, ro = 0;
        for (uint32_t c = 0; c < L.nchunks; c++) {
            const uint32_t *st = &cs[5 * (L.chunk0 + c)];
            uint32_t *cm = &cmeta[3 * (L.chunk0 + c)];
            cm[0] = uint32_t(lo);
            cm[1] = uint32_t(ro);
            lo += st[0];
            ro += st[3];
            if (st[2] != NONE32 && st[4]) ro += varint_len(cm[2] - st[2] - 1);
        }
        L.llen = lo;
        L.runs_len = ro;
        L.rmeta = uint32_t(ro + L.nsyms + 1);
        // :1485 — keep RLE only if it saves at least 1%
        L.rle = double(L.llen + L.rmeta) < .99 * double(L.n_cur);
    }
    // emit the accepted ones; meta = [nsyms][syms][run varints]
    std::vector<RleItem> eitems;
    std::vector<uint32_t> ci2, cm2;
    std::vector<uint8_t> heads;
    std::vector<std::pair<size_t, Leaf *>> head_of;
    for (size_t k = 0; k < who.size(); k++) {
        Leaf &L = leaves_[who[k]];
        if (!L.rle) continue;
        L.d_lits = g_.arena.alloc_n<uint8_t>(L.llen + 1);
        L.d_meta = g_.arena.alloc_n<uint8_t>(L.rmeta + 1);
        head_of.push_back({heads.size(), &L});
        heads.push_back(uint8_t(L.nsyms));
        heads.insert(heads.end(), L.syms, L.syms + L.nsyms);
        RleItem it = items[k];
        it.lits = L.d_lits;
        it.runs = L.d_meta + 1 + L.nsyms;
        for (uint32_t c = 0; c < L.nchunks; c++) {
            ci2.push_back(uint32_t(eitems.size()));
            ci2.push_back(c);
            for (int t = 0; t < 3; t++) cm2.push_back(cmeta[3 * (L.chunk0 + c) + t]);
        }
        eitems.push_back(it);
    }
    if (eitems.empty()) return;
    uint8_t *d_heads = g_.upload(heads);
    std::vector<CopyItem> cps;
    for (auto &h : head_of)
        cps.push_back({d_heads + h.first, h.second->d_meta, uint32_t(1 + h.second->nsyms), 0});
    FQZ5_HIP(launch_copy(g_.upload(cps), int(cps.size()), g_.stream));
    FQZ5_HIP(launch_rle_emit(g_.upload(eitems), g_.upload(ci2), int(ci2.size() / 2),
                             g_.upload(cm2), g_.stream));
}

// ---------------------------------------------------------------------------
// O0 table: rans_compress_O0_4x16 (:146-170), identical for 32x16 (:100-128).
void Compressor::build_o0(EJ &j) {
    uint32_t F[256];
    std::memcpy(F, j.F0, sizeof F);
    uint32_t mv = pow2_ceil(j.n);
    if (mv > 4096) mv = 4096;
    normalise_freq(F, int(j.n), mv);
    j.table.assign(1024, 0);
    j.table.resize(put_freq0(j.table.data(), F));
    normalise_freq(F, int(mv), 4096);
    j.bits = 12;
    j.syms.assign(256, EncSym{0, 0, 0, 0});
    for (uint32_t s = 0, x = 0; s < 256; s++)
        if (F[s]) { j.syms[s] = make_encsym(x, F[s], 12); x += F[s]; }
}

// O1 table: encode_freq1 (rANS_static16_int.h:312-421) with the histogram
// quirks of hist1_4 (utils.h:280-357).
void Compressor::build_o1(EJ &j, const uint32_t *cnt) {
    std::vector<uint32_t> Fm(256 * 256, 0);
    auto F = reinterpret_cast<uint32_t(*)[256]>(Fm.data());
    uint8_t alpha[256];
    for (int s = 0; s < 256; s++)
        if (s == 0 || j.F0[s]) alpha[j.remap[s]] = uint8_t(s);
    for (int a = 0; a < j.A; a++)
        for (int b = 0; b < j.A; b++) F[alpha[a]][alpha[b]] = cnt[a * j.A + b];
    uint32_t T[256] = {0};
    for (int i = 0; i < 256; i++)
        for (int k = 0; k < 256; k++) T[i] += F[i][k];
    T[j.last_byte]++;                                   // utils.h:311
    for (int z = 1; z < j.nx; z++) F[0][j.seg_first[z]]++;  // :325-326
    T[0] += j.nx - 1;

    std::vector<uint8_t> &h = j.table;
    h.assign(1 + 300 + 256 * 700, 0);
    uint32_t p = 1;
    uint32_t t0 = T[0];
    T[0] = 1;
    p += put_alphabet(&h[p], T);
    T[0] = t0;
    uint32_t rowmax[256] = {0};
    const int shift = o1_pick_shift(T, F, rowmax);
    j.bits = shift;
    // Per context, the normalised frequencies over the compacted alphabet;
    // k_enc_tab turns them into the EncSym table (start = the running sum
    // in byte order).  Every symbol with a frequency is in the alphabet (it
    // occurs in the input, or is 0).
    j.f1.assign(size_t(j.A) * j.A, 0);
    for (int i = 0; i < 256; i++) {
        if (!T[i]) continue;
        uint32_t mv = rowmax[i];
        if (shift == 10 && mv > 1024) mv = 1024;
        normalise_freq(F[i], int(T[i]), mv);
        p += put_freq_row(&h[p], T, F[i]);
        scale_pow2(F[i], mv, 1u << shift);
        const size_t row = size_t(j.remap[i]) * j.A;
        for (uint32_t s = 0; s < 256; s++) {
            if (!F[i][s]) continue;
            if (s != 0 && !j.F0[s])
                throw GpuError("rANS O1: a frequency outside the alphabet");
            j.f1[row + j.remap[s]] = uint16_t(F[i][s]);
        }
    }
    h.resize(p);
    h[0] = uint8_t(shift << 4);
}

void Compressor::stage_tables() {
    static const bool trace = std::getenv("FQZ5_STEP_TRACE") != nullptr;
    auto now = [] {
        return std::chrono::duration<double, std::milli>(
                   std::chrono::steady_clock::now().time_since_epoch()).count();
    };
    const double ta = trace ? now() : 0;
    // byte histograms of job inputs made in stage 4 (RLE literals, meta)
    std::vector<std::pair<const uint8_t *, uint32_t>> segs;
    std::vector<int> who;
    for (size_t i = 0; i < jobs_.size(); i++)
        if (jobs_[i].needs_hist) { segs.push_back({jobs_[i].d_in, jobs_[i].n}); who.push_back(int(i)); }
    std::vector<uint32_t> cnt;
    hist0(segs, cnt);
    for (size_t k = 0; k < who.size(); k++) std::memcpy(jobs_[who[k]].F0, &cnt[k * 512], 1024);

    // order-1 pair histograms over the compacted alphabet (always incl. 0)
    std::vector<int> o1jobs;
    uint32_t total = 0;
    for (size_t i = 0; i < jobs_.size(); i++) {
        EJ &j = jobs_[i];
        if (!j.o1) continue;
        j.A = 0;
        for (int s = 0; s < 256; s++)
            if (s == 0 || j.F0[s]) j.remap[s] = uint8_t(j.A++);
        j.f1_off = total;
        total += uint32_t(j.A) * uint32_t(j.A);
        o1jobs.push_back(int(i));
    }
    if (o1jobs.empty()) return;
    std::vector<uint8_t> remaps(o1jobs.size() * 256);
    for (size_t k = 0; k < o1jobs.size(); k++)
        std::memcpy(&remaps[k * 256], jobs_[o1jobs[k]].remap, 256);
    uint8_t *d_remaps = g_.upload(remaps);
    std::vector<Hist1Item> items, big;
    std::vector<const uint8_t *> probes;
    for (size_t k = 0; k < o1jobs.size(); k++) {
        EJ &j = jobs_[o1jobs[k]];
        const bool isbig = uint32_t(j.A) * uint32_t(j.A) >= 16384;
        const uint32_t sl = isbig ? HIST1_BIG_SLICE : HIST_SLICE;
        for (uint32_t b = 0; b < j.n; b += sl)
            (isbig ? big : items).push_back({j.d_in, d_remaps + 256 * k, b, std::min(j.n, b + sl),
                                             uint32_t(j.A), j.f1_off});
        uint32_t isz = j.n / j.nx;
        for (int z = 1; z < j.nx; z++) probes.push_back(j.d_in + size_t(z) * isz);
        probes.push_back(j.d_in + j.n - 1);
    }
    uint32_t *d_cnt = g_.arena.alloc_n<uint32_t>(total);
    g_.memset0(d_cnt, size_t(total) * 4);
    if (!items.empty()) FQZ5_HIP(launch_hist1(g_.upload(items), int(items.size()), d_cnt, false, g_.stream));
    if (!big.empty()) FQZ5_HIP(launch_hist1(g_.upload(big), int(big.size()), d_cnt, true, g_.stream));
    std::vector<uint32_t> h(total);
    g_.download(h.data(), d_cnt, total);
    std::vector<uint8_t> pb;
    gather(probes, pb);   // syncs
    size_t q = 0;
    for (int ji : o1jobs) {
        EJ &j = jobs_[ji];
        for (int z = 1; z < j.nx; z++) j.seg_first[z] = pb[q++];
        j.last_byte = pb[q++];
    }
    const double tb = trace ? now() : 0;
    host_parallel(o1jobs.size(), [&](size_t k) { build_o1(jobs_[o1jobs[k]], &h[jobs_[o1jobs[k]].f1_off]); });
    if (trace)
        std::fprintf(stderr, "[tid %ld] tables: o1 hist %.1f ms, build_o1 %.1f ms (%zu jobs, %u pairs)\n", long(syscall(SYS_gettid)),
                     tb - ta, now() - tb, o1jobs.size(), total);
}

// Stage 5: all rANS chains.  O1 tables above 1000 bytes get their own
// O0-4x16 job (rANS_static16_int.h:397-412) in the same launch.
void Compressor::stage_encode() {
    static const bool trace = std::getenv("FQZ5_STEP_TRACE") != nullptr;
    auto now = [] {
        return std::chrono::duration<double, std::milli>(
                   std::chrono::steady_clock::now().time_since_epoch()).count();
    };
    const double ta = trace ? now() : 0;
    const size_t nmain = jobs_.size();
    host_parallel(nmain, [&](size_t i) { if (!jobs_[i].o1) build_o0(jobs_[i]); });
    for (size_t i = 0; i < nmain; i++) {
        if (!jobs_[i].o1 || jobs_[i].table.size() <= 1000) continue;
        EJ h;
        h.h_in.assign(jobs_[i].table.begin() + 1, jobs_[i].table.end());
        h.n = uint32_t(h.h_in.size());
        h.nx = 4;
        for (uint8_t b : h.h_in) h.F0[b]++;
        build_o0(h);
        jobs_.push_back(std::move(h));
        jobs_[i].hdr_job = int(jobs_.size()) - 1;
    }
    // Chain pass: two launches on two queues, jobs whose tables fit a small
    // LDS footprint (many waves per CU) and the rest.  Then the replay
    // passes over all chunks of all jobs (rans_chain.hip).
    std::vector<EncJob> ejs, ejb, eall;
    std::vector<uint32_t> items;
    uint32_t lds_s = 0, lds_b = 0, lds_r = 0;
    std::vector<int> order;
    for (size_t i = 0; i < jobs_.size(); i++)
        if (jobs_[i].n) order.push_back(int(i));
    // longest chains first so they start in the first dispatch wave
    std::stable_sort(order.begin(), order.end(), [&](int a, int b) {
        return jobs_[a].n / jobs_[a].nx > jobs_[b].n / jobs_[b].nx;
    });
    uint32_t *d_lens = g_.arena.alloc_n<uint32_t>(jobs_.size());
    // every job's symbol table and O1 remap in one upload each (a stripe
    // candidate set is thousands of small jobs)
    // O0 tables from the host; O1 tables built on the GPU from their
    // frequencies (k_enc_tab), into one device array
    std::vector<size_t> tab_off(jobs_.size()), rm_off(jobs_.size()), f1_off(jobs_.size());
    std::vector<EncSym> all_syms;
    std::vector<uint16_t> all_f1;
    std::vector<uint8_t> all_rm;
    size_t nsyms = 0;
    for (int i : order) {
        const EJ &j = jobs_[i];
        if (j.o1) {
            tab_off[i] = nsyms;
            nsyms += j.f1.size();
            f1_off[i] = all_f1.size();
            all_f1.insert(all_f1.end(), j.f1.begin(), j.f1.end());
        }
        rm_off[i] = all_rm.size();
        if (j.o1) all_rm.insert(all_rm.end(), j.remap, j.remap + 256);
    }
    for (int i : order) {
        const EJ &j = jobs_[i];
        if (j.o1) continue;
        tab_off[i] = nsyms + all_syms.size();
        all_syms.insert(all_syms.end(), j.syms.begin(), j.syms.end());
    }
    const double tb = trace ? now() : 0;
    EncSym *d_syms = g_.arena.alloc_n<EncSym>(std::max<size_t>(nsyms + all_syms.size(), 1));
    if (!all_syms.empty()) {
        uint8_t *st = g_.staging.alloc(all_syms.size() * sizeof(EncSym));
        std::memcpy(st, all_syms.data(), all_syms.size() * sizeof(EncSym));
        FQZ5_HIP(hipMemcpyAsync(d_syms + nsyms, st, all_syms.size() * sizeof(EncSym),
                                hipMemcpyHostToDevice, g_.stream));
    }
    if (!all_f1.empty()) {
        const uint16_t *d_f1 = g_.upload(all_f1);
        std::vector<EncTabItem> ti;
        for (int i : order)
            if (jobs_[i].o1)
                ti.push_back({d_f1 + f1_off[i], d_syms + tab_off[i], uint32_t(jobs_[i].A),
                              uint32_t(jobs_[i].bits)});
        FQZ5_HIP(launch_enc_tab(g_.upload(ti), int(ti.size()), g_.stream));
    }
    const uint8_t *d_rms = all_rm.empty() ? nullptr : g_.upload(all_rm);
    for (int i : order) {
        EJ &j = jobs_[i];
        if (!j.h_in.empty()) j.d_in = g_.upload(j.h_in);
        const EncSym *d_tab = d_syms + tab_off[i];
        const size_t cap = 2 * size_t(j.n) + 16 * size_t(j.nx) + 1088;
        uint8_t *base = g_.arena.alloc_n<uint8_t>(cap);
        j.d_end = base + (cap & ~size_t(15));
        const uint8_t *d_remap = j.o1 ? d_rms + rm_off[i] : nullptr;
        const uint32_t steps = j.o1 ? j.n - uint32_t(j.nx - 1) * (j.n / uint32_t(j.nx))
                                    : (j.n + uint32_t(j.nx) - 1) / uint32_t(j.nx);
        const uint32_t S = enc_chunk_steps(j.nx);
        const uint32_t nch = (steps + S - 1) / S;
        uint32_t *d_ck = g_.arena.alloc_n<uint32_t>(size_t(nch + 1) * uint32_t(j.nx));
        uint32_t *d_cnt = g_.arena.alloc_n<uint32_t>(nch);
        const EncJob e{j.d_in, d_tab, d_remap, j.d_end, d_lens + i, d_ck, d_cnt,
                       j.n, j.nx, j.bits, j.A, nch};
        // ejs: two-wave chains (NX=4, table in LDS: the long ones);
        // ejb: the rest (X32, O1 tables too big for LDS)
        if (enc_chain_2w(j.o1, j.nx, uint32_t(j.A))) {
            ejs.push_back(e);
            lds_s = std::max(lds_s, enc_2w_lds_bytes(j.o1, uint32_t(j.A)));
        } else {
            ejb.push_back(e);
            lds_b = std::max(lds_b, enc_lds_bytes(j.o1, uint32_t(j.A)));
        }
        const uint32_t per = enc_replay_chunks(j.nx);
        for (uint32_t c0 = 0; c0 < nch; c0 += per) {
            items.push_back(uint32_t(eall.size()));
            items.push_back(c0);
        }
        eall.push_back(e);
        lds_r = std::max(lds_r, enc_replay_lds_bytes(j.o1, uint32_t(j.A)));
    }
    EventPair ev(g_.prof.on && !order.empty(), g_.stream);
    lds_s = g_.chain_lds(lds_s, ejs.size() + ejb.size());
    lds_b = g_.chain_lds(lds_b, ejs.size() + ejb.size());
    // per-kernel spans (fqz5_profile_read_all): their bytes once the
    // output lengths are known, below
    long tk_2w = -1, tk_1w = -1, tk_r0 = -1, tk_r1 = -1;
    if (!ejs.empty()) {
        const EncJob *d = g_.upload(ejs);
        const EncJob *db = ejb.empty() ? nullptr : g_.upload(ejb);
        g_.fork();
        {
            ProfSpan sp(PK_ENC_CHAIN2W, g_.stream2);
            FQZ5_HIP(launch_enc_chain2w(d, int(ejs.size()), lds_s, g_.stream2));
            tk_2w = sp.end(0);
        }
        if (db) {
            ProfSpan sp(PK_ENC_CHAIN, g_.stream);
            FQZ5_HIP(launch_enc_chain(db, int(ejb.size()), lds_b, g_.stream));
            tk_1w = sp.end(0);
        }
        g_.join();
    } else if (!ejb.empty()) {
        const EncJob *db = g_.upload(ejb);
        ProfSpan sp(PK_ENC_CHAIN, g_.stream);
        FQZ5_HIP(launch_enc_chain(db, int(ejb.size()), lds_b, g_.stream));
        tk_1w = sp.end(0);
    }
    if (!eall.empty()) {
        const EncJob *d_all = g_.upload(eall);
        const uint32_t *d_items = g_.upload(items);
        const int nit = int(items.size() / 2);
        {
            ProfSpan sp(PK_ENC_REPLAY0, g_.stream);
            FQZ5_HIP(launch_enc_replay(d_all, d_items, nit, false, lds_r, g_.stream));
            tk_r0 = sp.end(0);
        }
        FQZ5_HIP(launch_enc_scan(d_all, int(eall.size()), g_.stream));
        ProfSpan sp(PK_ENC_REPLAY, g_.stream);
        FQZ5_HIP(launch_enc_replay(d_all, d_items, nit, true, lds_r, g_.stream));
        tk_r1 = sp.end(0);
    }
    ev.stop(g_.stream);
    const double tc = trace ? now() : 0;
    std::vector<uint32_t> lens(jobs_.size(), 0);
    g_.download(lens.data(), d_lens, jobs_.size());
    g_.sync();
    const double td = trace ? now() : 0;
    if (ev.on || tk_r1 >= 0) {
        double bytes = 0, b2w = 0, b1w = 0;
        for (int i : order) {
            const double b = double(jobs_[i].n) + lens[i];
            bytes += b;
            (enc_chain_2w(jobs_[i].o1, jobs_[i].nx, uint32_t(jobs_[i].A)) ? b2w : b1w) += b;
        }
        prof_bytes(tk_2w, b2w);
        prof_bytes(tk_1w, b1w);
        prof_bytes(tk_r0, bytes);
        prof_bytes(tk_r1, bytes);
        if (ev.on) {
            g_.prof.enc_ms += ev.ms();
            g_.prof.enc_launches += 1;
            g_.prof.enc_bytes += bytes;
        }
    }
    for (size_t i = 0; i < jobs_.size(); i++) jobs_[i].payload = jobs_[i].n ? lens[i] : 0;
    for (size_t i = nmain; i < jobs_.size(); i++) finish_job(jobs_[i]);
    for (size_t i = 0; i < nmain; i++) finish_job(jobs_[i]);
    if (trace)
        std::fprintf(stderr, "[tid %ld] encode: tables %.1f ms (%zu syms), uploads+launch %.1f ms, "
                     "wait %.1f ms, finish %.1f ms\n", long(syscall(SYS_gettid)), tb - ta, nsyms + all_syms.size(), tc - tb,
                     td - tc, now() - td);
}

void Compressor::finish_job(EJ &j) {
    j.layout.clear();
    if (!j.n) return;   // empty O0 stream is zero bytes (:139-140, :225-229)
    Piece tab;
    tab.host = j.table;
    if (j.hdr_job >= 0) {
        const EJ &h = jobs_[j.hdr_job];
        const uint32_t c = layout_size(h.layout), raw = uint32_t(j.table.size());
        if (c + 6 < raw) {      // keep the compressed table
            uint8_t tmp[12];
            tab.host.assign(1, uint8_t(j.table[0] | 1));
            int k = varint_put(tmp, nullptr, raw - 1);
            tab.host.insert(tab.host.end(), tmp, tmp + k);
            k = varint_put(tmp, nullptr, c);
            tab.host.insert(tab.host.end(), tmp, tmp + k);
            j.layout.push_back(std::move(tab));
            for (auto &p : h.layout) j.layout.push_back(p);
            tab = Piece();
        }
    }
    if (!tab.host.empty()) j.layout.push_back(std::move(tab));
    Piece pl;
    pl.dev = j.d_end - j.payload;
    pl.len = j.payload;
    j.layout.push_back(pl);
}

// ---------------------------------------------------------------------------
// Stage 6: the non-STRIPE path of rans_compress_to_4x16 (:1411-1599) for a
// given capacity; false where the reference returns NULL.
bool Compressor::leaf_layout(const Leaf &L, uint32_t cap, Layout &out) const {
    out.clear();
    if (cap == 0) return false;
    uint8_t h[320];
    uint32_t out_size = cap;
    const int no_size = L.order & ORD_NOSZ;
    h[0] = uint8_t(L.order);
    uint32_t hb = 1;                       // header bytes
    if (!no_size) hb += vput(h, 1, cap, L.n);
    uint32_t n = L.n;
    if ((L.order & ORD_PACK) && L.n) {
        if (hb + 256 > out_size) return false;
        if (!L.pack) {
            h[0] &= ~ORD_PACK;
        } else {
            std::memcpy(&h[hb], L.pmeta, L.pmeta_len);
            hb += L.pmeta_len;
            int vs = vput(h, hb, cap, L.plen);
            hb += vs;
            out_size -= vs;                 // reference quirk (:1453)
            n = L.plen;
        }
    } else if (L.order & ORD_PACK) {
        h[0] &= ~ORD_PACK;
    }
    uint32_t hl = hb;                      // header incl. RLE meta bytes
    Layout meta;
    if ((L.order & ORD_RLE) && n) {
        if (!L.rle) {
            h[0] &= ~ORD_RLE;
        } else {
            int sz = vput(h, hb, cap, L.rmeta * 2);
            sz += vput(h, hb + sz, cap, uint32_t(L.llen));
            if (hb + sz + 5 > out_size) return false;
            const uint32_t cm_cap = out_size - (hb + sz + 5);
            if (compress_bound(L.rmeta, 0) - 20 > cm_cap) return false;
            const EJ &mj = jobs_[L.ej_meta];
            uint32_t cm = layout_size(mj.layout);
            int sz2;
            if (cm < L.rmeta) {
                sz2 = vput(h, hb + sz, cap, cm);
                meta = mj.layout;
            } else {                        // stored raw (:1519-1525)
                sz = vput(h, hb, cap, L.rmeta * 2 + 1);
                sz2 = vput(h, hb + sz, cap, uint32_t(L.llen));
                Piece p;
                p.dev = L.d_meta;
                p.len = L.rmeta;
                meta.push_back(p);
                cm = L.rmeta;
            }
            hb += sz + sz2;
            hl = hb + cm;
            n = uint32_t(L.llen);
        }
    } else if (L.order & ORD_RLE) {
        h[0] &= ~ORD_RLE;
    }
    if ((L.order & ORD_X32) && !L.x32) h[0] &= ~ORD_X32;   // :1455-1458, :1504-1507
    if (hl > out_size) return false;
    out_size -= hl;
    if ((L.order & 3) && n < 8) h[0] &= ~1;                 // :1547-1550
    if (compress_bound(n, L.o1 ? 1 : 0) - 20 > out_size) return false;
    const EJ &ej = jobs_[L.ej_main];
    const uint32_t es = layout_size(ej.layout);
    Layout body;
    if (es >= n) {                                          // CAT fallback (:1560-1574)
        h[0] &= ~3;
        h[0] |= ORD_CAT | no_size;
        if (hl + n > cap) return false;
        if (n) {
            Piece p;
            p.dev = ej.d_in;
            p.len = n;
            body.push_back(p);
        }
    } else {
        body = ej.layout;
    }
    out.push_back(Piece{std::vector<uint8_t>(h, h + hb), nullptr, 0});
    for (auto &p : meta) out.push_back(p);
    for (auto &p : body) out.push_back(p);
    return true;
}

// STRIPE (:1266-1393): best of the candidate sub-orders per stripe, where a
// candidate that would not fit the remaining capacity is skipped.
bool Compressor::stripe_layout(const StripeReq &S, const CompressReq &r, Layout &out) const {
    out.clear();
    const uint32_t cap = r.cap;
    const int order = entry_flags(r.order, r.n);
    std::vector<uint8_t> h(7 + 5 * 256 + 16, 0);
    h[0] = uint8_t(order & ~ORD_NOSZ);
    uint32_t hl = 1 + vput(h.data(), 1, cap, r.n);
    if (hl >= cap) return false;
    h[hl++] = uint8_t(S.N);
    uint32_t pos = 7 + 5 * S.N;
    Layout body;
    for (unsigned i = 0; i < S.N; i++) {
        uint32_t best = UINT32_MAX;
        Layout best_l;
        for (int li : S.leaves[i]) {
            if (pos > cap) continue;
            Layout l;
            if (!leaf_layout(leaves_[li], cap - pos, l)) continue;
            const uint32_t sz = layout_size(l);
            if (sz && best > sz) { best = sz; best_l = std::move(l); }
        }
        if (best == UINT32_MAX) return false;
        pos += best;
        hl += vput(h.data(), hl, cap, best);
        for (auto &p : best_l) body.push_back(std::move(p));
    }
    h.resize(hl);
    out.push_back(Piece{h, nullptr, 0});
    for (auto &p : body) out.push_back(std::move(p));
    return true;
}

// ---------------------------------------------------------------------------
void Compressor::run(std::vector<CompressReq> &reqs) {
    const double t_enter = std::chrono::duration<double, std::milli>(
                               std::chrono::steady_clock::now().time_since_epoch()).count();
    std::vector<int> req_leaf(reqs.size(), -1), req_stripe(reqs.size(), -1);
    std::vector<StripeItem> sitems;
    uint32_t max_n = 0;
    for (size_t i = 0; i < reqs.size(); i++) {
        CompressReq &r = reqs[i];
        r.ok = false;
        r.out.clear();
        if (!r.cap) r.cap = compress_bound(r.n, r.order);
        if (r.n > uint32_t(INT_MAX)) continue;
        const int order = entry_flags(r.order, r.n);
        if (order & ORD_STRIPE) {
            stripes_.emplace_back();
            StripeReq &S = stripes_.back();
            unsigned N = (order >> 8) & 0xff;
            if (!N) N = 4;
            if (N > r.n) N = r.n;
            S.N = N;
            for (unsigned k = 0; k < N; k++) {
                S.plen[k] = r.n / N + ((r.n % N) > k);
                S.pidx[k] = k ? S.pidx[k - 1] + S.plen[k - 1] : 0;
            }
            S.d_tr = g_.arena.alloc_n<uint8_t>(r.n);
            sitems.push_back({r.d_in, S.d_tr, r.n, N, 0, 0});
            max_n = std::max(max_n, r.n);
            S.leaves.resize(N);
            const int cand[4] = {1, 64, 128, 0};
            for (unsigned k = 0; k < N; k++)
                for (int m : cand) {
                    if ((order & m) != m) continue;
                    if ((order & ORD_STRIPE_NO0) && !(m & 1)) continue;
                    const int co = entry_flags(m | ORD_NOSZ | (order & ORD_X32), S.plen[k]);
                    S.leaves[k].push_back(add_leaf(S.d_tr + S.pidx[k], S.plen[k], co));
                }
            req_stripe[i] = int(stripes_.size()) - 1;
        } else if (!(order & ORD_CAT)) {
            req_leaf[i] = add_leaf(r.d_in, r.n, order);
        }
    }
    if (!sitems.empty())
        FQZ5_HIP(launch_stripe(g_.upload(sitems), int(sitems.size()), max_n, g_.stream));
    static const bool trace = std::getenv("FQZ5_STEP_TRACE") != nullptr;
    auto now = [] {
        return std::chrono::duration<double, std::milli>(
                   std::chrono::steady_clock::now().time_since_epoch()).count();
    };
    const double t0 = trace ? now() : 0;
    if (trace) std::fprintf(stderr, "[tid %ld] compress: leaves %.1f ms\n", long(syscall(SYS_gettid)), t0 - t_enter);
    stage_pack();
    const double t1 = trace ? now() : 0;
    stage_rle();
    const double t2 = trace ? now() : 0;
    for (auto &L : leaves_) {
        uint32_t n = L.n_cur;
        if (L.rle) {
            n = uint32_t(L.llen);
            if (L.x32 && (L.rmeta < 32 || L.llen < 32)) L.x32 = false;  // :1504-1507
        }
        L.o1 = (L.order & 1) && n >= 8;
        const int nx = L.x32 ? 32 : 4;
        if (L.rle) {
            L.ej_meta = add_job(L.d_meta, L.rmeta, false, nx);
            jobs_[L.ej_meta].needs_hist = true;
            L.ej_main = add_job(L.d_lits, n, L.o1, nx);
            jobs_[L.ej_main].needs_hist = true;
        } else {
            L.ej_main = add_job(L.d_cur, n, L.o1, nx);
            std::memcpy(jobs_[L.ej_main].F0, L.pack ? L.phist : L.hist, 1024);
        }
    }
    const double t3 = trace ? now() : 0;
    stage_tables();
    const double t4 = trace ? now() : 0;
    stage_encode();
    const double t5 = trace ? now() : 0;
    if (trace)
        std::fprintf(stderr, "[tid %ld] compress: pack %.1f ms, rle %.1f ms, jobs %.1f ms, tables %.1f ms, "
                     "encode %.1f ms (%zu requests, %zu jobs)\n", long(syscall(SYS_gettid)), t1 - t0, t2 - t1, t3 - t2,
                     t4 - t3, t5 - t4, reqs.size(), jobs_.size());
    struct Done {
        bool on;
        double t;
        ~Done() {
            if (on)
                std::fprintf(stderr, "[tid %ld] compress: layouts %.1f ms\n", long(syscall(SYS_gettid)),
                             std::chrono::duration<double, std::milli>(
                                 std::chrono::steady_clock::now().time_since_epoch()).count() - t);
        }
    } done_{trace, t5};
    for (size_t i = 0; i < reqs.size(); i++) {
        CompressReq &r = reqs[i];
        if (r.n > uint32_t(INT_MAX)) continue;
        if (req_stripe[i] >= 0) {
            r.ok = stripe_layout(stripes_[req_stripe[i]], r, r.out);
        } else if (req_leaf[i] >= 0) {
            r.ok = leaf_layout(leaves_[req_leaf[i]], r.cap, r.out);
        } else {                                   // CAT (:1395-1409)
            uint8_t h[8];
            h[0] = ORD_CAT;
            const uint32_t hl = 1 + vput(h, 1, r.cap, r.n);
            if (hl + r.n > r.cap) continue;
            r.out.push_back(Piece{std::vector<uint8_t>(h, h + hl), nullptr, 0});
            if (r.n) {
                Piece p;
                p.dev = r.d_in;
                p.len = r.n;
                r.out.push_back(p);
            }
            r.ok = true;
        }
    }
}

}  // namespace

void compress_batch(GpuCtx &g, std::vector<CompressReq> &reqs) {
    static const bool trace = std::getenv("FQZ5_STEP_TRACE") != nullptr;
    auto now = [] {
        return std::chrono::duration<double, std::milli>(
                   std::chrono::steady_clock::now().time_since_epoch()).count();
    };
    std::unique_ptr<Compressor> c(new Compressor(g));
    c->run(reqs);
    const double t0 = trace ? now() : 0;
    // A batch of thousands of jobs frees ~100 MB of host tables and
    // layouts (130 ms at -5, mostly munmap); the results no longer refer to
    // them, so a detached thread frees them off the caller's critical path.
    if (c->njobs() > 1000) std::thread([p = c.release()] { delete p; }).detach();
    else c.reset();
    if (trace) std::fprintf(stderr, "[tid %ld] compress: teardown %.1f ms\n", long(syscall(SYS_gettid)), now() - t0);
}

// ---------------------------------------------------------------------------
void write_layouts_dev(GpuCtx &g, const std::vector<const Layout *> &ls,
                       const std::vector<uint8_t *> &dsts) {
    std::vector<uint8_t> hostbytes;
    struct Pend { size_t off; uint8_t *dst; uint32_t len; };
    std::vector<Pend> hp;
    std::vector<CopyItem> items;
    for (size_t i = 0; i < ls.size(); i++) {
        uint8_t *dst = dsts[i];
        for (const Piece &p : *ls[i]) {
            if (p.dev) {
                for (uint32_t o = 0; o < p.len; o += 65536)
                    items.push_back({p.dev + o, dst + o, std::min<uint32_t>(65536, p.len - o), 0});
                dst += p.len;
            } else if (!p.host.empty()) {
                hp.push_back({hostbytes.size(), dst, uint32_t(p.host.size())});
                hostbytes.insert(hostbytes.end(), p.host.begin(), p.host.end());
                dst += p.host.size();
            }
        }
    }
    if (!hostbytes.empty()) {
        const uint8_t *d_h = g.upload(hostbytes);
        for (auto &q : hp)
            for (uint32_t o = 0; o < q.len; o += 65536)
                items.push_back({d_h + q.off + o, q.dst + o, std::min<uint32_t>(65536, q.len - o), 0});
    }
    if (!items.empty())
        FQZ5_HIP(launch_copy(g.upload(items), int(items.size()), g.stream));
}

void write_layout_host(GpuCtx &g, const Layout &l, uint8_t *dst) {
    for (const Piece &p : l) {
        if (p.dev) {
            g.download(dst, p.dev, p.len);
            dst += p.len;
        } else {
            std::memcpy(dst, p.host.data(), p.host.size());
            dst += p.host.size();
        }
    }
    g.sync();
}

}  // namespace fqz5
