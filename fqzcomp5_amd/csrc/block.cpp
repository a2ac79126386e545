// block.cpp — fqzcomp5's per-block section coder for the sequence and
// quality sections (fqzcomp5.c:1899-2280), driving the batched GPU rANS
// codec.
//
// The reference encodes one block at a time per worker thread, trying every
// method of the section's mask while the codec trial is running
// (metrics_method / compress_with_methods, fqzcomp5.c:1899-2144).  Here a
// whole run of blocks is handed over at once: every candidate method of
// every block is compressed speculatively in ONE GPU batch (the chains run
// side by side, so the extra candidates cost little wall time), then the
// trial state machine is replayed on the host in block order, which gives
// exactly the choices of a single-threaded (-t1) reference run.
#include <atomic>
#include <chrono>
#include <cstdio>
#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <exception>
#include <functional>
#include <thread>
#include <deque>
#include <memory>
#include <vector>

#include "../../include/fqz5_block.h"
#include "rans_codec.hpp"
#include "fqz_codec.hpp"
#include "seq_codec.hpp"
#include "lzp_codec.hpp"
#include "names.hpp"
#include "host_dec.hpp"
#include "rans_format.hpp"

namespace fqz5 {

GpuCtx &gpu();
void fqz5_set_error(const char *msg);

namespace {

// fqzcomp5.c:185-208
enum Method {
    RANS0 = 1, RANS1, RANS64, RANS65, RANS128, RANS129, RANS192, RANS193,
    RANSXN1, LZP3, SEQ10 = 20, SEQ12, SEQ12B, SEQ13B, SEQ14B, SEQ_CUSTOM,
    FQZ0 = 26, FQZ1, FQZ2, FQZ3, FQZ4, M_LAST = 31
};
constexpr uint32_t RANS_MASK =
    (1u << RANS0) | (1u << RANS1) | (1u << RANS64) | (1u << RANS65) |
    (1u << RANS128) | (1u << RANS129) | (1u << RANS192) | (1u << RANS193) |
    (1u << RANSXN1);
constexpr uint32_t FQZ_MASK =
    (1u << FQZ0) | (1u << FQZ1) | (1u << FQZ2) | (1u << FQZ3) | (1u << FQZ4);

constexpr uint32_t SEQ_MASK =
    (1u << SEQ10) | (1u << SEQ12) | (1u << SEQ12B) | (1u << SEQ13B) | (1u << SEQ14B);
constexpr uint32_t NAME_MASK = ((1u << (M_TOK3_9_LZP + 1)) - 1) & ~((1u << M_TLZP3) - 1);

bool is_fqz(int m) { return m >= FQZ0 && m <= FQZ4; }
bool is_seqcm(int m) { return m >= SEQ10 && m <= SEQ14B; }

// encode_seq's parameters per method and the section strat byte
// (k << 4) | (both << 3) | 1 (fqzcomp5.c:2047-2062)
SeqEncReq seq_req(const fqz5_section &S, int m) {
    static const int slevel[] = {10, 12, 12, 13, 14}, both[] = {0, 0, 1, 1, 1};
    SeqEncReq r;
    r.d_in = S.in;
    r.n = S.in_size;
    r.lens = S.rec_len;
    r.nrec = S.nrec;
    r.k = slevel[m - SEQ10];
    r.both = both[m - SEQ10];
    return r;
}
int seq_strat(int m) {
    static const int slevel[] = {10, 12, 12, 13, 14}, both[] = {0, 0, 1, 1, 1};
    return (slevel[m - SEQ10] << 4) | (both[m - SEQ10] << 3) | 1;
}

// order word per rANS method (fqzcomp5.c:1992-2010)
int method_order(int m, uint32_t fixed_len) {
    static const int ord[] = {0, 1, 64, 65, 128, 129, 192, 193};
    if (m >= RANS0 && m <= RANS193) return ord[m - RANS0];
    return int((fixed_len << 8) + 9);   // RANSXN1, incl. the >=256 aliasing
}

// metrics_method (fqzcomp5.c:1899-1946)
uint32_t metrics_method(fqz5_trial_state &st, int sec, uint32_t avail) {
    fqz5_section_stats &s = st.sec[sec];
    if (s.review <= 0) {
        s.review = FQZ5_METRICS_REVIEW;
        s.trial = FQZ5_METRICS_TRIAL;
        std::memset(s.usize, 0, sizeof s.usize);
        std::memset(s.csize, 0, sizeof s.csize);
        std::memset(s.count, 0, sizeof s.count);
    }
    if (s.trial > 0) return avail;
    if (s.trial > -99999) {
        int best_m = 0;
        double best = 1e30;
        for (int m = 0; m < FQZ5_M_LAST; m++) {
            if (s.usize[m] && best > (s.csize[m] + 1.0) / s.usize[m]) {
                best = (s.csize[m] + 1.0) / s.usize[m];
                best_m = m;
            }
        }
        s.method_used = best_m;
        s.trial = -99999;
        return 1u << best_m;
    }
    s.review--;
    return 1u << s.method_used;
}

}  // namespace

// Speculative candidates of the last fqz5_sections_try on this thread; they
// live in the thread's GPU arena until fqz5_sections_commit.
struct TrySession {
    std::vector<CompressReq> reqs;
    std::vector<std::vector<int>> req_of;
    std::vector<FqzEncReq> fqz;                   // FQZ candidates
    std::vector<uint64_t> fqz_lb;                 // pruned candidates: size lower bound (else 0)
    std::vector<std::vector<int>> fqz_of;
    std::vector<SeqEncReq> seq;                   // sequence CM candidates
    std::vector<uint64_t> seq_lb;                 // pruned candidates: size lower bound (else 0)
    std::vector<uint64_t> fqz_ub, seq_ub;         // pruned candidates: size upper bound
    std::vector<char> fqz_skip, seq_skip;         // range chain skipped: no bytes yet
    std::vector<std::vector<int>> seq_of;
    std::vector<uint32_t> upper;                  // the sizes matrix with upper bounds
    std::deque<std::vector<uint32_t>> recs;       // their (rewritable) lengths / flags
    std::vector<NameEnc> names;                   // name-section candidates (host bytes)
    std::vector<std::vector<int>> name_of;
    bool open = false;
    bool aux = false;                             // candidates live in the helper contexts
};

// fqz_compress(4, slice, in, size, &len, m - FQZ0, NULL) for a section
// (compress_with_methods, fqzcomp5.c:2071-2092)
FqzEncReq fqz_req(const fqz5_section &S, int m, std::deque<std::vector<uint32_t>> &keep) {
    FqzEncReq r;
    r.d_in = S.in;
    r.n = S.in_size;
    r.nrec = S.nrec;
    keep.emplace_back(S.rec_len, S.rec_len + std::max(S.nrec, 0));
    r.lens = keep.back().data();
    if (S.rec_flags)
        keep.emplace_back(S.rec_flags, S.rec_flags + std::max(S.nrec, 0));
    else
        keep.emplace_back(size_t(std::max(S.nrec, 0)), 0u);
    r.flags = keep.back().data();
    r.d_seq = S.seq;
    r.vers = 4;
    r.strat = m - FQZ0;
    return r;
}
thread_local TrySession t_sess;

// Name-section candidates (encode_names, fqzcomp5.c:1408-1586) of sections
// `which` x methods `meth`, on context g: the names come down once per
// section, are split / tokenised on host threads, and every lzp pass and
// rANS stream of all candidates runs as one batch each.
void encode_name_jobs(GpuCtx &g, const fqz5_section *secs, const std::vector<int> &which,
                      const std::vector<int> &meth, std::vector<NameEnc> &out) {
    out.assign(which.size(), NameEnc());
    if (which.empty()) return;
    // into the pinned staging arena (kept until the context's reset): a
    // pageable copy of a -5 run's 38 name blocks (570 MB) took ~0.5 s
    // Each block's tokenising starts when its own download is done (an
    // event per block), not after all of them.
    std::vector<const uint8_t *> host;
    std::vector<hipEvent_t> evs;
    std::vector<int> host_of(which.size());
    std::vector<int> seen;
    struct Events {
        std::vector<hipEvent_t> &e;
        ~Events() { for (auto x : e) (void)hipEventDestroy(x); }
    } keep_{evs};
    for (size_t k = 0; k < which.size(); k++) {
        auto it = std::find(seen.begin(), seen.end(), which[k]);
        if (it != seen.end()) { host_of[k] = int(it - seen.begin()); continue; }
        host_of[k] = int(seen.size());
        seen.push_back(which[k]);
        const fqz5_section &S = secs[which[k]];
        uint8_t *hb = g.staging.alloc(S.in_size + 1);
        g.download(hb, S.in, S.in_size);
        hipEvent_t e;
        FQZ5_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
        evs.push_back(e);
        FQZ5_HIP(hipEventRecord(e, g.stream));
        host.push_back(hb);
    }
    std::vector<const uint8_t *> h(which.size()), d(which.size());
    std::vector<uint32_t> lens(which.size());
    std::vector<hipEvent_t> ready(which.size());
    for (size_t k = 0; k < which.size(); k++) {
        h[k] = host[size_t(host_of[k])];
        ready[k] = evs[size_t(host_of[k])];
        d[k] = secs[which[k]].in;
        lens[k] = secs[which[k]].in_size;
    }
    names_encode_batch(g, out, h, d, lens, meth, &ready);
    g.sync();
}

// Trial pruning (fqz5_set_trial_prune): an fqz or sequence-model candidate
// whose size is provably not below the best rANS candidate's, in every trial
// section and summed over the trial window, cannot be chosen (rANS methods
// come first, so they win ties); its range chain and bytes are skipped and
// its lower bound stands in for its size.  The caller enables it only when
// the sections of this call that try such methods form one whole trial
// window per section kind.
std::atomic<int> g_prune{0};
// Bounds-only tries (fqz5_set_trial_bounds): every fqz and sequence-model
// candidate skips its range chain and reports its size as the interval
// [lower, upper] (entropy, entropy plus the coder's slack): the caller
// decides the trial from the intervals when they separate the candidates,
// and codes the winners at commit (encode_run_bounded).
std::atomic<int> g_bounds{0};
std::atomic<uint64_t> g_fqz_tried{0}, g_fqz_pruned{0};
std::atomic<uint64_t> g_chains_host{0}, g_chains_gpu{0};   // fqz5_decode_chain_counts

// Which requests of one family of work candidates (fqz methods FQZ0..FQZ4 on
// quality sections, or the sequence models SEQ10..SEQ14B) to skip, from the
// exact sizes of the earlier (rANS) methods and the family's lower bounds.
// of[i][m]: the request index of method m in section i (-1 if none); lb(k):
// request k's size lower bound (0 if unknown).
template <class LB>
std::vector<char> prune_plan(const std::vector<CompressReq> &reqs,
                             const std::vector<std::vector<int>> &of, int mlo, int mhi,
                             size_t nreq, LB lb) {
    std::vector<char> skip(nreq, 0);
    const int nsec = int(of.size());
    std::vector<int> F;                                 // sections trying the family
    for (int i = 0; i < nsec; i++)
        for (int m = mlo; m <= mhi; m++)
            if (of[i][m] >= 0) { F.push_back(i); break; }
    // one whole trial window: every method's usize is then the same, and the
    // window's pick (min (csize + 1) / usize) compares plain sums
    if (F.size() != size_t(FQZ5_METRICS_TRIAL)) return skip;
    auto rsize = [&](int i, int m) -> int64_t {          // exact rANS size, -1 if none
        const int ri = t_sess.req_of[i][m];
        return ri >= 0 && reqs[size_t(ri)].ok ? int64_t(layout_size(reqs[size_t(ri)].out)) : -1;
    };
    std::vector<int64_t> best(F.size(), -1);            // per section: min earlier size
    for (size_t k = 0; k < F.size(); k++)
        for (int m = 1; m < mlo; m++) {
            const int64_t z = rsize(F[k], m);
            if (z >= 0 && (best[k] < 0 || z < best[k])) best[k] = z;
        }
    int64_t best_sum = -1;                              // min over methods tried everywhere
    for (int m = 1; m < mlo; m++) {
        int64_t sum = 0;
        bool all = true;
        for (int i : F) {
            const int64_t z = rsize(i, m);
            if (z < 0) { all = false; break; }
            sum += z;
        }
        if (all && (best_sum < 0 || sum < best_sum)) best_sum = sum;
    }
    for (int m = mlo; m <= mhi; m++) {
        bool ok = true;
        int64_t lbsum = 0;
        for (size_t k = 0; k < F.size() && ok; k++) {
            const int fi = of[F[k]][m];
            if (fi < 0) { ok = false; break; }            // must be tried in the whole window
            const int64_t b = int64_t(lb(size_t(fi)));
            ok = b > 0 && best[k] >= 0 && b >= best[k];
            lbsum += b;
        }
        if (!ok || !(best_sum >= 0 && lbsum >= best_sum)) continue;
        for (int i : F)
            if (of[i][m] >= 0) skip[size_t(of[i][m])] = 1;
    }
    return skip;
}

// LZP3 candidates of sections `which`: their lzp output (device, this
// context's arena) joins `reqs` as an order-5 rANS request; of[i][LZP3]
// gets its index.
void add_lzp3(GpuCtx &g, const fqz5_section *secs, const std::vector<int> &which,
              std::vector<CompressReq> &reqs, std::vector<std::vector<int>> &of) {
    if (which.empty()) return;
    std::vector<LzpEncReq> lz(which.size());
    for (size_t k = 0; k < which.size(); k++) {
        lz[k].d_in = secs[which[k]].in;
        lz[k].n = secs[which[k]].in_size;
    }
    lzp_encode_batch(g, lz);
    for (size_t k = 0; k < which.size(); k++) {
        CompressReq r;
        r.d_in = lz[k].d_out;
        r.n = lz[k].out_len;
        r.order = 5;
        r.cap = compress_bound(r.n, r.order);
        of[size_t(which[k])][LZP3] = int(reqs.size());
        reqs.push_back(std::move(r));
    }
}

}  // namespace fqz5

using namespace fqz5;

extern "C" {

void fqz5_trial_init(fqz5_trial_state *st) { std::memset(st, 0, sizeof *st); }

int fqz5_set_trial_prune(int on) { return g_prune.exchange(on ? 1 : 0); }

int fqz5_set_trial_bounds(int on) { return g_bounds.exchange(on ? 1 : 0); }

int fqz5_arenas_release(void) {
    try {
        t_sess = TrySession();
        gpu_release_all();
        return 0;
    } catch (const std::exception &e) {
        fqz5_set_error(e.what());
        return -1;
    }
}

int fqz5_sections_try_upper(uint32_t *upper, int nsec) {
    if (nsec < 0 || size_t(nsec) * FQZ5_M_LAST != t_sess.upper.size()) {
        fqz5_set_error("fqz5_sections_try_upper: no try of that many sections on this thread");
        return -1;
    }
    std::memcpy(upper, t_sess.upper.data(), t_sess.upper.size() * sizeof(uint32_t));
    return 0;
}

void fqz5_decode_chain_counts(uint64_t *out2) {
    out2[0] = g_chains_host.load();
    out2[1] = g_chains_gpu.load();
}

void fqz5_trial_counts(uint64_t *out2) {
    out2[0] = g_fqz_tried.load();
    out2[1] = g_fqz_pruned.load();
}

void fqz5_trial_schedule(const int32_t *sec_ids, int nsec, const uint32_t *avail,
                         const fqz5_trial_state *st, uint32_t *masks_out) {
    // metrics_method's counters without the sizes: which sections try every
    // method (trial and re-trial blocks) does not depend on the outcomes
    fqz5_trial_state s = *st;
    for (int i = 0; i < nsec; i++) {
        fqz5_section_stats &ss = s.sec[sec_ids[i]];
        if (ss.review <= 0) {
            ss.review = FQZ5_METRICS_REVIEW;
            ss.trial = FQZ5_METRICS_TRIAL;
        }
        masks_out[i] = 0;
        if (ss.trial > 0) {
            masks_out[i] = avail[sec_ids[i]];
            ss.trial--;
        } else if (ss.trial > -99999) {
            ss.trial = -99999;
        } else {
            ss.review--;
        }
    }
}

static bool step_trace() {
    static const bool on = std::getenv("FQZ5_STEP_TRACE") != nullptr;
    return on;
}
static double now_ms() {
    return std::chrono::duration<double, std::milli>(
               std::chrono::steady_clock::now().time_since_epoch()).count();
}

int fqz5_sections_try(const fqz5_section *secs, int nsec, const uint32_t *masks,
                      uint32_t *sizes) {
    const double t0 = step_trace() ? now_ms() : 0;
    try {
        GpuCtx &g = gpu();
        if (t_sess.open) {
            g.reset();
            gpu_aux_reset_all();
        }
        t_sess = TrySession();
        for (int i = 0; i < nsec; i++) {
            if (masks[i] & ~(RANS_MASK | FQZ_MASK | SEQ_MASK | NAME_MASK | (1u << LZP3)))
                throw GpuError("fqz5_sections_try: method mask has SEQ_CUSTOM (not in this build)");
            if ((masks[i] & NAME_MASK) && secs[i].sec != FQZ5_SEC_NAME)
                throw GpuError("fqz5_sections_try: name methods need a name section");
            if (secs[i].sec == FQZ5_SEC_NAME && (masks[i] & ~NAME_MASK))
                throw GpuError("fqz5_sections_try: a name section takes name methods only");
            if ((masks[i] & SEQ_MASK) && (secs[i].sec != FQZ5_SEC_SEQ || !secs[i].rec_len))
                throw GpuError("fqz5_sections_try: SEQ methods need a sequence section with records");
            if ((masks[i] & FQZ_MASK) && (secs[i].sec != FQZ5_SEC_QUAL || !secs[i].rec_len))
                throw GpuError("fqz5_sections_try: FQZ methods need a quality section with records");
        }
        std::vector<CompressReq> &reqs = t_sess.reqs;
        t_sess.req_of.assign(nsec, std::vector<int>(FQZ5_M_LAST, -1));
        t_sess.fqz_of.assign(nsec, std::vector<int>(FQZ5_M_LAST, -1));
        t_sess.seq_of.assign(nsec, std::vector<int>(FQZ5_M_LAST, -1));
        t_sess.name_of.assign(nsec, std::vector<int>(FQZ5_M_LAST, -1));
        std::vector<int> name_sec, name_meth;             // name candidates
        std::vector<int> lzp_sec;                         // sections trying LZP3
        std::vector<CompressReq> sreq;                    // RANSXN1 (stripe) candidates
        std::vector<int> sreq_sec;
        for (int i = 0; i < nsec; i++) {
            const fqz5_section &S = secs[i];
            for (int m = 1; m < FQZ5_M_LAST; m++) {
                if (!(masks[i] & (1u << m))) continue;
                if (is_fqz(m)) {
                    t_sess.fqz_of[i][m] = int(t_sess.fqz.size());
                    t_sess.fqz.push_back(fqz_req(S, m, t_sess.recs));
                    continue;
                }
                if (is_seqcm(m)) {
                    t_sess.seq_of[i][m] = int(t_sess.seq.size());
                    t_sess.seq.push_back(seq_req(S, m));
                    continue;
                }
                if (is_name_method(m)) {
                    t_sess.name_of[i][m] = int(name_sec.size());
                    name_sec.push_back(i);
                    name_meth.push_back(m);
                    continue;
                }
                if (m == RANSXN1 && !S.fixed_len) continue;   // out = NULL (:2004-2007)
                if (m == LZP3) {                               // after the lzp pass, below
                    lzp_sec.push_back(i);
                    continue;
                }
                CompressReq r;
                r.d_in = S.in;
                r.n = S.in_size;
                r.order = method_order(m, S.fixed_len);
                r.cap = compress_bound(r.n, r.order);
                if (m == RANSXN1) {          // thousands of short stripe chains
                    sreq_sec.push_back(i);
                    sreq.push_back(std::move(r));
                    continue;
                }
                t_sess.req_of[i][m] = int(reqs.size());
                reqs.push_back(std::move(r));
            }
        }
        // The candidates whose cost grows with their work (trial blocks only)
        // run on the thread's helper contexts from helper threads, beside the
        // rANS candidates (a few long chains that leave most of the GPU
        // idle): LZP3 (the lzp pass, then rANS order 5 of its output,
        // fqzcomp5.c:2013-2021), the fqz and the sequence-model model passes.
        // Then the fqz / sequence-model candidates that provably lose the
        // trial are pruned, and the others' range chains run.
        static const bool no_aux = std::getenv("FQZ5_NO_AUX") != nullptr;
        std::vector<FqzEncReq> &fq = t_sess.fqz;
        std::vector<SeqEncReq> &sq = t_sess.seq;
        auto join_stripes = [&] {          // the stripe candidates join the batch
            for (size_t k = 0; k < sreq.size(); k++) {
                t_sess.req_of[size_t(sreq_sec[k])][RANSXN1] = int(reqs.size());
                reqs.push_back(std::move(sreq[k]));
            }
            sreq.clear();
        };
        if ((!fq.empty() || !sq.empty() || !lzp_sec.empty() || !sreq.empty() || !name_sec.empty()) &&
            !no_aux) {
            t_sess.aux = true;
            GpuCtx &ga = gpu_aux(0), &gb = gpu_aux(2), &gc = gpu_aux(1);
            // sequence-model candidates: one helper context each (their
            // passes are latency-bound and overlap well), up to AUX_NSEQ
            // (each runs one block at a time with ~120 B of device memory per
            // base while it prepares: as many side by side as fit a quarter of
            // HBM; -9's 1 GB blocks take them one after another)
            size_t nsq = std::min<size_t>(sq.size(), size_t(AUX_NSEQ));
            {
                uint64_t mx = 1;
                for (const SeqEncReq &q : sq) mx = std::max<uint64_t>(mx, q.n);
                size_t fr = 0, tot = 0;
                if (hipMemGetInfo(&fr, &tot) != hipSuccess || !tot) tot = size_t(64) << 30;
                const uint64_t fit = (uint64_t(tot) / 4) / (120 * mx);
                nsq = std::max<size_t>(1, std::min<size_t>(nsq, size_t(fit)));
            }
            std::vector<std::vector<SeqEncReq>> sqg(nsq);
            for (size_t k = 0; k < sq.size(); k++) sqg[k % std::max<size_t>(nsq, 1)].push_back(sq[k]);
            std::vector<CompressReq> lzr;
            std::vector<std::vector<int>> lzr_of(size_t(nsec), std::vector<int>(FQZ5_M_LAST, -1));
            std::vector<std::exception_ptr> err(2 + nsq);
            auto on = [t0](GpuCtx &c, std::exception_ptr &e, auto &&fn) {
                return std::thread([&c, &e, fn, t0] {
                    try {
                        FQZ5_HIP(hipSetDevice(c.device));
                        fn();
                        if (step_trace())
                            std::fprintf(stderr, "sections_try: helper context %p done at %.1f ms\n",
                                         static_cast<void *>(&c), now_ms() - t0);
                    } catch (...) {
                        e = std::current_exception();
                    }
                });
            };
            std::vector<std::thread> th;
            th.push_back(on(gc, err[0], [&] {
                add_lzp3(gc, secs, lzp_sec, lzr, lzr_of);
                if (!lzr.empty()) compress_batch(gc, lzr);
            }));
            th.push_back(on(ga, err[1], [&] { if (!fq.empty()) fqz_encode_prepare(ga, fq); }));
            // The RANSXN1 candidates (150 stripes x 4 orders per quality
            // section: most of a batch's jobs, and most of its host work on
            // tables) run as their own batch on a helper context, so that
            // their host work overlaps the long chains of the other rANS
            // candidates on the GPU.
            GpuCtx &gs = gpu_aux(AUX_STRIPES);
            std::exception_ptr serr;
            std::thread ts = on(gs, serr, [&] { if (!sreq.empty()) compress_batch(gs, sreq); });
            // the name candidates: host tokenising, then their own batches
            // (t_sess is thread_local: the helper thread gets the caller's
            // vector by reference)
            GpuCtx &gn = gpu_aux(AUX_NAMES);
            std::exception_ptr nerr;
            std::vector<NameEnc> &nres = t_sess.names;
            std::thread tn = on(gn, nerr, [&] {
                encode_name_jobs(gn, secs, name_sec, name_meth, nres);
            });
            for (size_t k = 0; k < nsq; k++) {
                GpuCtx &gk = gpu_aux(int(AUX_SEQ0 + k));
                std::vector<SeqEncReq> &grp = sqg[k];
                th.push_back(on(gk, err[2 + k], [&gk, &grp] { seq_encode_prepare(gk, grp); }));
            }
            // The plain O0/O1 candidates (RANS0/RANS1: the longest chains,
            // one step per 4 input bytes) need no PACK / RLE pass: they run
            // as a batch of their own on a helper context, so that their
            // chains start while this thread packs and run-length codes the
            // others' inputs (the packed chains are half as long or less).
            std::vector<size_t> plain_at;
            std::vector<char> is_plain(reqs.size(), 0);
            std::vector<CompressReq> plain, rest;
            for (size_t k = 0; k < reqs.size(); k++)
                if ((reqs[k].order & ~1) == 0 && reqs[k].n >= (1u << 20)) plain_at.push_back(k);
            if (plain_at.size() == reqs.size()) plain_at.clear();
            for (size_t k : plain_at) is_plain[k] = 1;
            if (!plain_at.empty())
                for (size_t k = 0; k < reqs.size(); k++)
                    (is_plain[k] ? plain : rest).push_back(std::move(reqs[k]));
            GpuCtx &gp = gpu_aux(AUX_PLAIN);
            gp.prof.on = g.prof.on;
            std::exception_ptr perr;
            std::thread tp = on(gp, perr, [&] { if (!plain.empty()) compress_batch(gp, plain); });
            double tc = 0, tpl = 0;
            try {
                compress_batch(g, plain_at.empty() ? reqs : rest);
                if (!plain_at.empty()) {             // back in request order
                    size_t q = 0;
                    for (size_t k = 0; k < reqs.size(); k++)
                        if (!is_plain[k]) reqs[k] = std::move(rest[q++]);
                }
                tc = step_trace() ? now_ms() : 0;
                tp.join();
                tpl = step_trace() ? now_ms() : 0;
            } catch (...) {
                if (tp.joinable()) tp.join();
                for (auto &t : th) t.join();
                ts.join();
                tn.join();
                throw;
            }
            if (perr) {
                for (auto &t : th) t.join();
                ts.join();
                tn.join();
                std::rethrow_exception(perr);
            }
            for (size_t q = 0; q < plain_at.size(); q++) reqs[plain_at[q]] = std::move(plain[q]);
            g.prof.enc_ms += gp.prof.enc_ms;
            g.prof.enc_launches += gp.prof.enc_launches;
            g.prof.enc_bytes += gp.prof.enc_bytes;
            gp.prof = KernelProfile();
            if (step_trace() && !plain_at.empty())
                std::fprintf(stderr, "sections_try: %zu plain rANS candidates on a helper, "
                             "done %.1f ms after the others\n", plain_at.size(), tpl - tc);
            tc = std::max(tc, tpl);
            for (auto &t : th) t.join();
            ts.join();
            tn.join();
            if (serr) std::rethrow_exception(serr);
            if (nerr) std::rethrow_exception(nerr);
            join_stripes();
            if (step_trace())
                std::fprintf(stderr, "sections_try: rANS candidates %.1f ms, helpers waited "
                             "%.1f ms more\n", tc - t0, now_ms() - tc);
            for (auto &e : err)
                if (e) std::rethrow_exception(e);
            for (size_t k = 0; k < sq.size(); k++)          // their work back in request order
                sq[k] = std::move(sqg[k % std::max<size_t>(nsq, 1)][k / std::max<size_t>(nsq, 1)]);
            for (int i : lzp_sec) {                     // the LZP3 streams join the batch
                t_sess.req_of[size_t(i)][LZP3] = int(reqs.size());
                reqs.push_back(std::move(lzr[size_t(lzr_of[size_t(i)][LZP3])]));
            }
            std::vector<char> skip_f(fq.size(), 0), skip_s(sq.size(), 0);
            if (g_bounds.load()) {
                for (size_t k = 0; k < fq.size(); k++) skip_f[k] = fqz_size_lower_bound(fq[k]) > 0;
                for (size_t k = 0; k < sq.size(); k++) skip_s[k] = seq_size_upper_bound(sq[k]) > 0;
            } else if (g_prune.load()) {
                skip_f = prune_plan(reqs, t_sess.fqz_of, FQZ0, FQZ4, fq.size(),
                                    [&](size_t k) { return fqz_size_lower_bound(fq[k]); });
                skip_s = prune_plan(reqs, t_sess.seq_of, SEQ10, SEQ14B, sq.size(),
                                    [&](size_t k) { return seq_size_lower_bound(sq[k]); });
            }
            std::exception_ptr ferr;
            std::thread tf = on(ga, ferr, [&] { if (!fq.empty()) fqz_encode_finish(ga, fq, &skip_f); });
            try {
                FQZ5_HIP(hipSetDevice(gb.device));
                if (!sq.empty()) seq_encode_finish(gb, sq, &skip_s);
            } catch (...) {
                tf.join();
                throw;
            }
            tf.join();
            if (ferr) std::rethrow_exception(ferr);
            t_sess.fqz_skip.insert(t_sess.fqz_skip.end(), skip_f.begin(), skip_f.end());
            t_sess.seq_skip.insert(t_sess.seq_skip.end(), skip_s.begin(), skip_s.end());
            for (size_t k = 0; k < fq.size(); k++) {
                t_sess.fqz_lb.push_back(skip_f[k] ? fqz_size_lower_bound(fq[k]) : 0);
                t_sess.fqz_ub.push_back(skip_f[k] ? fqz_size_upper_bound(fq[k]) : 0);
            }
            for (size_t k = 0; k < sq.size(); k++) {
                t_sess.seq_lb.push_back(skip_s[k] ? seq_size_lower_bound(sq[k]) : 0);
                t_sess.seq_ub.push_back(skip_s[k] ? seq_size_upper_bound(sq[k]) : 0);
            }
            g_fqz_tried += fq.size() + sq.size();
            for (char c : skip_f) g_fqz_pruned += c ? 1 : 0;
            for (char c : skip_s) g_fqz_pruned += c ? 1 : 0;
        } else {
            join_stripes();
            add_lzp3(g, secs, lzp_sec, reqs, t_sess.req_of);
            compress_batch(g, reqs);
            encode_name_jobs(g, secs, name_sec, name_meth, t_sess.names);
            if (!fq.empty()) fqz_encode_batch(g, fq);
            if (!sq.empty()) seq_encode_batch(g, sq);
            t_sess.fqz_lb.assign(fq.size(), 0);
            t_sess.seq_lb.assign(sq.size(), 0);
            t_sess.fqz_ub.assign(fq.size(), 0);
            t_sess.seq_ub.assign(sq.size(), 0);
            t_sess.fqz_skip.assign(fq.size(), 0);
            t_sess.seq_skip.assign(sq.size(), 0);
            g_fqz_tried += fq.size() + sq.size();
        }
        t_sess.open = true;
        if (step_trace())
            std::fprintf(stderr, "sections_try: %.1f ms (device / pinned allocations so far %llu, "
                         "frees %llu)\n", now_ms() - t0,
                         (unsigned long long)ChunkPool::alloc_calls().load(),
                         (unsigned long long)ChunkPool::free_calls().load());
        // sizes as compress_with_methods sees them: UINT_MAX when not run,
        // 0 when the codec returned NULL (out_len = *out_size = 0); a
        // skipped candidate's lower bound here, its upper bound in `upper`
        t_sess.upper.assign(size_t(nsec) * FQZ5_M_LAST, 0);
        for (int i = 0; i < nsec; i++) {
            // encode_names returns NULL without writing *out_size, so a
            // failing name candidate is seen with the size the previous name
            // candidate of this section wrote (fqzcomp5.c:2036-2044, :1433-
            // 1440); never strictly the best, but it enters the trial's
            // totals (metrics_update) and can win the later blocks
            uint32_t stale = UINT32_MAX;
            for (int m = 0; m < FQZ5_M_LAST; m++) {
                const int ri = t_sess.req_of[i][m], fi = t_sess.fqz_of[i][m];
                const int si = t_sess.seq_of[i][m], ni = t_sess.name_of[i][m];
                uint32_t sz = UINT32_MAX;
                if (ri >= 0) sz = reqs[ri].ok ? layout_size(reqs[ri].out) : 0;
                // a name candidate's size is its whole section (encode_names'
                // *out_size)
                if (ni >= 0) {
                    if (t_sess.names[size_t(ni)].ok)
                        stale = sz = uint32_t(t_sess.names[size_t(ni)].out.size());
                    else
                        sz = stale;
                }
                if (si >= 0) {
                    const uint64_t lb = t_sess.seq_lb[size_t(si)];   // pruned: its lower bound
                    sz = t_sess.seq[size_t(si)].ok ? layout_size(t_sess.seq[size_t(si)].out)
                         : lb ? uint32_t(std::min<uint64_t>(lb, UINT32_MAX - 1)) : 0;
                }
                if (fi >= 0) {
                    const uint64_t lb = t_sess.fqz_lb[size_t(fi)];   // pruned: its lower bound
                    sz = t_sess.fqz[size_t(fi)].ok ? layout_size(t_sess.fqz[size_t(fi)].out)
                         : lb ? uint32_t(std::min<uint64_t>(lb, UINT32_MAX - 1)) : 0;
                }
                uint32_t up = sz;
                if (si >= 0 && !t_sess.seq[size_t(si)].ok && t_sess.seq_ub[size_t(si)])
                    up = uint32_t(std::min<uint64_t>(t_sess.seq_ub[size_t(si)], UINT32_MAX - 1));
                if (fi >= 0 && !t_sess.fqz[size_t(fi)].ok && t_sess.fqz_ub[size_t(fi)])
                    up = uint32_t(std::min<uint64_t>(t_sess.fqz_ub[size_t(fi)], UINT32_MAX - 1));
                sizes[size_t(i) * FQZ5_M_LAST + m] = sz;
                t_sess.upper[size_t(i) * FQZ5_M_LAST + m] = up;
            }
        }
        return 0;
    } catch (const std::exception &e) {
        fqz5_set_error(e.what());
        t_sess = TrySession();
        try { gpu().reset(); } catch (...) {}
        try { gpu_aux_reset_all(); } catch (...) {}
        return -1;
    }
}

void fqz5_trial_replay(const int32_t *sec_ids, const uint32_t *in_sizes,
                       const uint32_t *sizes, int nsec, const uint32_t *avail,
                       fqz5_trial_state *st, int32_t *methods_out,
                       uint32_t *tried_out) {
    for (int i = 0; i < nsec; i++) {
        const int sec = sec_ids[i];
        fqz5_section_stats &ss = st->sec[sec];
        const uint32_t methods = metrics_method(*st, sec, avail[sec]);
        const bool in_trial = ss.trial > 0;           // compress_with_methods
        uint32_t best_sz = UINT32_MAX;
        int best_m = 0;
        for (int m = 0; m < FQZ5_M_LAST; m++) {
            if (!(methods & (1u << m))) continue;
            const uint32_t out_len = sizes[size_t(i) * FQZ5_M_LAST + m];
            if (best_sz > out_len) { best_sz = out_len; best_m = m; }
        }
        // outside the trial the one method is run whatever its size (the
        // caller encodes it at commit: its size is not known here)
        if (!in_trial && __builtin_popcount(methods) == 1) best_m = __builtin_ctz(methods);
        if (in_trial) {                                 // metrics_update, :2121-2130
            for (int m = 0; m < FQZ5_M_LAST; m++) {
                if (!(methods & (1u << m)) || ss.trial <= 0) continue;
                ss.usize[m] += in_sizes[i];
                ss.csize[m] += sizes[size_t(i) * FQZ5_M_LAST + m];
                ss.count[m]++;
            }
            ss.trial--;
        }
        methods_out[i] = best_m;
        if (tried_out) tried_out[i] = methods;
    }
}

int fqz5_sections_commit(const fqz5_section *secs, int nsec, const int32_t *methods,
                         fqz5_section_result *res) {
    const double t0 = step_trace() ? now_ms() : 0;
    try {
        GpuCtx &g = gpu();
        if (!t_sess.open || int(t_sess.req_of.size()) != nsec)
            throw GpuError("fqz5_sections_commit: no matching fqz5_sections_try");
        // sections outside the trial: their one method, encoded now
        std::vector<CompressReq> late;
        std::vector<int> late_of(nsec, -1), late_fqz_of(nsec, -1), late_seq_of(nsec, -1);
        std::vector<FqzEncReq> late_fqz;
        std::vector<SeqEncReq> late_seq;
        std::vector<int> late_lzp;
        std::vector<std::vector<int>> late_lzp_of(nsec, std::vector<int>(FQZ5_M_LAST, -1));
        std::vector<int> late_name_sec, late_name_meth, late_name_of(nsec, -1);
        // a candidate the session tried with its range chain skipped (a
        // bounds-only try or a pruned one) has no bytes: coded now, as a
        // method the session did not try
        auto coded_fqz = [&](int i, int m) {
            const int f = t_sess.fqz_of[i][m];
            return f >= 0 && !(size_t(f) < t_sess.fqz_skip.size() && t_sess.fqz_skip[size_t(f)]);
        };
        auto coded_seq = [&](int i, int m) {
            const int q = t_sess.seq_of[i][m];
            return q >= 0 && !(size_t(q) < t_sess.seq_skip.size() && t_sess.seq_skip[size_t(q)]);
        };
        for (int i = 0; i < nsec; i++) {
            const int m = methods[i];
            if (m <= 0 || m >= FQZ5_M_LAST || t_sess.req_of[i][m] >= 0 || coded_fqz(i, m) ||
                coded_seq(i, m) || t_sess.name_of[i][m] >= 0)
                continue;
            if (is_name_method(m) && secs[i].sec == FQZ5_SEC_NAME) {
                late_name_of[i] = int(late_name_sec.size());
                late_name_sec.push_back(i);
                late_name_meth.push_back(m);
                continue;
            }
            if (is_seqcm(m) && secs[i].sec == FQZ5_SEC_SEQ && secs[i].rec_len) {
                late_seq_of[i] = int(late_seq.size());
                late_seq.push_back(seq_req(secs[i], m));
                continue;
            }
            if (is_fqz(m) && secs[i].sec == FQZ5_SEC_QUAL && secs[i].rec_len) {
                late_fqz_of[i] = int(late_fqz.size());
                late_fqz.push_back(fqz_req(secs[i], m, t_sess.recs));
                continue;
            }
            if (m == LZP3 && secs[i].sec == FQZ5_SEC_SEQ) {
                late_lzp.push_back(i);
                continue;
            }
            if (!(RANS_MASK & (1u << m)) || (m == RANSXN1 && !secs[i].fixed_len)) continue;
            CompressReq r;
            r.d_in = secs[i].in;
            r.n = secs[i].in_size;
            r.order = method_order(m, secs[i].fixed_len);
            r.cap = compress_bound(r.n, r.order);
            late_of[i] = int(late.size());
            late.push_back(std::move(r));
        }
        // The late fqz encodes (-5 Illumina: every block's quality section;
        // their range chains, ~1.2 s for a 100 MB block, are the commit's
        // long pole) start first, in groups on the helper contexts (the
        // sequence models' ones, idle now), so that each group's chains start
        // when its own model pass is done, and the other late encodes run
        // beside them on this thread.
        static const bool no_aux = std::getenv("FQZ5_NO_AUX") != nullptr;
        std::vector<std::vector<FqzEncReq>> fgrp;
        std::vector<std::exception_ptr> ferr;
        std::vector<std::thread> fth;
        struct JoinAll {
            std::vector<std::thread> &t;
            ~JoinAll() { for (auto &x : t) if (x.joinable()) x.join(); }
        } join_f{fth};
        const bool fqz_aux = !late_fqz.empty() && !no_aux;
        if (fqz_aux) {
            const size_t ng = std::min<size_t>(late_fqz.size(), size_t(AUX_NSEQ));
            fgrp.resize(ng);
            ferr.resize(ng);
            for (size_t k = 0; k < late_fqz.size(); k++) fgrp[k % ng].push_back(std::move(late_fqz[k]));
            for (size_t q = 0; q < ng; q++) {
                GpuCtx &c = gpu_aux(int(AUX_SEQ0 + q));
                fth.emplace_back([&c, &grp = fgrp[q], &e = ferr[q]] {
                    try {
                        FQZ5_HIP(hipSetDevice(c.device));
                        fqz_encode_batch(c, grp);
                    } catch (...) {
                        e = std::current_exception();
                    }
                });
            }
        }
        add_lzp3(g, secs, late_lzp, late, late_lzp_of);
        for (int i : late_lzp) late_of[i] = late_lzp_of[size_t(i)][LZP3];
        if (!late.empty()) compress_batch(g, late);
        if (!late_fqz.empty() && !fqz_aux) fqz_encode_batch(g, late_fqz);
        if (!late_seq.empty()) seq_encode_batch(g, late_seq);
        std::vector<NameEnc> late_names;
        encode_name_jobs(g, secs, late_name_sec, late_name_meth, late_names);
        if (fqz_aux) {
            for (auto &t : fth) t.join();
            for (auto &e : ferr)
                if (e) std::rethrow_exception(e);
            const size_t ng = fgrp.size();
            for (size_t k = 0; k < late_fqz.size(); k++) late_fqz[k] = std::move(fgrp[k % ng][k / ng]);
        }
        std::vector<const Layout *> ls;
        std::vector<uint8_t *> dsts;
        std::vector<Layout> framed(nsec);
        for (int i = 0; i < nsec; i++) {
            const fqz5_section &S = secs[i];
            fqz5_section_result &R = res[i];
            const int m = methods[i];
            const int ri = (m > 0 && m < FQZ5_M_LAST) ? t_sess.req_of[i][m] : -1;
            const int fi = (m > 0 && m < FQZ5_M_LAST) ? t_sess.fqz_of[i][m] : -1;
            const int si = (m > 0 && m < FQZ5_M_LAST) ? t_sess.seq_of[i][m] : -1;
            const int ni = (m > 0 && m < FQZ5_M_LAST) ? t_sess.name_of[i][m] : -1;
            if (S.sec == FQZ5_SEC_NAME) {             // encode_names' bytes, unframed
                const NameEnc *E = ni >= 0 ? &t_sess.names[size_t(ni)]
                                   : late_name_of[i] >= 0 ? &late_names[size_t(late_name_of[i])]
                                                          : nullptr;
                R.method = m;
                R.strat = is_name_method(m) ? name_strat(m) : 0;
                R.status = -1;
                R.clen = 0;
                R.usize = S.in_size;
                if (!E || !E->ok) continue;
                R.clen = uint32_t(E->out.size());
                if (E->out.size() > S.out_cap) continue;
                Piece p;
                p.host = E->out;
                framed[i].push_back(std::move(p));
                ls.push_back(&framed[i]);
                dsts.push_back(S.out);
                R.status = 0;
                continue;
            }
            const Layout *lay = nullptr;
            if (ri >= 0 && t_sess.reqs[ri].ok) lay = &t_sess.reqs[ri].out;
            if (late_of[i] >= 0 && late[late_of[i]].ok) lay = &late[late_of[i]].out;
            if (fi >= 0 && t_sess.fqz[size_t(fi)].ok) lay = &t_sess.fqz[size_t(fi)].out;
            if (late_fqz_of[i] >= 0 && late_fqz[late_fqz_of[i]].ok) lay = &late_fqz[late_fqz_of[i]].out;
            if (si >= 0 && t_sess.seq[size_t(si)].ok) lay = &t_sess.seq[size_t(si)].out;
            if (late_seq_of[i] >= 0 && late_seq[late_seq_of[i]].ok) lay = &late_seq[late_seq_of[i]].out;
            R.method = m;
            // compress_with_methods' *strat (fqzcomp5.c:1994-2069)
            R.strat = is_fqz(m) ? 1 : is_seqcm(m) ? seq_strat(m) : m == LZP3 ? LZP3 : 0;
            R.status = -1;
            R.clen = 0;
            R.usize = S.in_size;
            if (!lay) continue;
            const uint32_t clen = layout_size(*lay);
            R.clen = clen;
            if (9ull + clen > S.out_cap) continue;
            // section framing [strat u8][u32 usize][u32 csize] (:2224-2229)
            Piece h;
            h.host.resize(9);
            h.host[0] = uint8_t(R.strat);
            std::memcpy(&h.host[1], &S.in_size, 4);
            std::memcpy(&h.host[5], &clen, 4);
            framed[i].push_back(std::move(h));
            for (auto &p : *lay) framed[i].push_back(p);
            ls.push_back(&framed[i]);
            dsts.push_back(S.out);
            R.status = 0;
        }
        const double t1 = step_trace() ? now_ms() : 0;
        write_layouts_dev(g, ls, dsts);
        const double t2 = step_trace() ? now_ms() : 0;
        g.reset();
        const double t3 = step_trace() ? now_ms() : 0;
        // the fqz candidates of the try live in the aux arena: rewind it too,
        // or every step's trial buffers take fresh chunks (the r01 bench OOM)
        if (t_sess.aux || fqz_aux) gpu_aux_reset_all();
        // the session's host buffers (candidate tables, layouts, the name
        // candidates' token streams: ~100 MB, mostly munmap) are freed by a
        // detached thread, off the caller's path; nothing refers to them now
        std::thread([old = std::make_unique<TrySession>(std::move(t_sess))]() mutable {
            old.reset();
        }).detach();
        t_sess = TrySession();
        if (step_trace())
            std::fprintf(stderr, "sections_commit: late encodes %.1f ms, write %.1f ms, sync "
                         "%.1f ms, release %.1f ms\n", t1 - t0, t2 - t1, t3 - t2, now_ms() - t3);
        return 0;
    } catch (const std::exception &e) {
        fqz5_set_error(e.what());
        t_sess = TrySession();
        try { gpu().reset(); } catch (...) {}
        return -1;
    }
}

int fqz5_encode_sections(const fqz5_section *secs, int nsec, const uint32_t *avail,
                         fqz5_trial_state *st, fqz5_section_result *res) {
    std::vector<uint32_t> sizes(size_t(nsec) * FQZ5_M_LAST), masks(nsec);
    std::vector<int32_t> ids(nsec), meth(nsec);
    std::vector<uint32_t> ins(nsec);
    for (int i = 0; i < nsec; i++) { ids[i] = secs[i].sec; ins[i] = secs[i].in_size; }
    // every method of every section in one launch (see sections.encode_run)
    for (int i = 0; i < nsec; i++) masks[i] = avail[secs[i].sec];
    if (fqz5_sections_try(secs, nsec, masks.data(), sizes.data())) return -1;
    fqz5_trial_replay(ids.data(), ins.data(), sizes.data(), nsec, avail, st, meth.data(),
                      nullptr);
    return fqz5_sections_commit(secs, nsec, meth.data(), res);
}

int fqz5_decode_sections(const fqz5_section *secs, int nsec, fqz5_section_result *res) {
    // (trace) entry to exit, the locals' destructors included
    struct ExitTrace {
        double t;
        ~ExitTrace() {
            if (t) std::fprintf(stderr, "decode_sections: entry to exit %.1f ms\n", now_ms() - t);
        }
    } exit_trace{step_trace() ? now_ms() : 0.0};
    try {
        GpuCtx &g = gpu();
        static const bool trace = std::getenv("FQZ5_STEP_TRACE") != nullptr;
        const auto t0 = std::chrono::steady_clock::now();
        // section headers to the host, then the rANS payloads
        size_t tot = 0;
        for (int i = 0; i < nsec; i++) tot += secs[i].in_size;
        // into the pinned staging arena (kept until g.reset() below): a
        // pageable copy of a -5 run's 600 MB took 125 ms, this one ~5x less
        uint8_t *host = g.staging.alloc(tot + 1);
        size_t off = 0;
        for (int i = 0; i < nsec; i++) {
            g.download(host + off, secs[i].in, secs[i].in_size);
            off += secs[i].in_size;
        }
        g.sync();
        std::vector<DecompressReq> reqs;
        std::vector<FqzDecReq> fqz;
        std::vector<SeqDecReq> seqd;
        std::vector<int> who, who_fqz, who_seq;
        std::vector<LzpDecReq> lzd;
        std::vector<int> who_lzp;                     // section of each lzd entry
        std::vector<size_t> lzp_rans;                 // its rANS stage in reqs
        std::vector<NameDec> nd;                      // name sections (decode_names)
        std::vector<int> who_name;
        std::vector<const uint8_t *> seq_h;           // host stream of each seqd entry
        off = 0;
        for (int i = 0; i < nsec; i++) {
            const uint8_t *h = host + off;
            off += secs[i].in_size;
            res[i].status = -1;
            if (secs[i].in_size < 9) continue;
            if (secs[i].sec == FQZ5_SEC_NAME) {       // [u32 u_len][u8 strat][u32 c_len] (:2325-2327)
                NameDec D;
                std::memcpy(&D.u_len, h, 4);
                D.strat = h[4];
                std::memcpy(&D.c_len, h + 5, 4);
                res[i].strat = D.strat;
                res[i].clen = D.c_len;
                if (9ull + D.c_len > secs[i].in_size || D.u_len > secs[i].out_cap) continue;
                D.comp = h + 9;
                D.d_comp = secs[i].in + 9;
                nd.push_back(D);
                who_name.push_back(i);
                continue;
            }
            uint32_t ulen, clen;
            std::memcpy(&ulen, h + 1, 4);
            std::memcpy(&clen, h + 5, 4);
            res[i].strat = h[0];
            res[i].clen = clen;
            if (9ull + clen > secs[i].in_size || ulen > secs[i].out_cap) continue;
            if (h[0] == 1 && secs[i].sec == FQZ5_SEC_QUAL) {   // fqz_decompress (:2498-2530)
                FqzDecReq f;
                f.h_in = h + 9;
                f.d_in = secs[i].in + 9;
                f.in_size = clen;
                f.nrec = secs[i].rec_len ? secs[i].nrec : 0;
                f.lens = secs[i].rec_len;
                f.d_seq = secs[i].seq;
                f.d_out = secs[i].out;
                f.out_cap = secs[i].out_cap;
                fqz.push_back(f);
                who_fqz.push_back(i);
                continue;
            }
            if ((h[0] & 7) == 1 && secs[i].sec == FQZ5_SEC_SEQ) {   // decode_seq (:2421-2430)
                seq_h.push_back(h + 9);
                SeqDecReq q;
                q.d_in = secs[i].in + 9;
                q.in_size = clen;
                q.lens = secs[i].rec_len;
                q.nrec = secs[i].nrec;
                q.k = h[0] >> 4;
                q.both = (h[0] >> 3) & 1;
                q.d_out = secs[i].out;
                q.n = ulen;
                seqd.push_back(q);
                who_seq.push_back(i);
                continue;
            }
            if (h[0] == LZP3 && secs[i].sec == FQZ5_SEC_SEQ) {   // rANS, then unlzp (:2431-2445)
                const uint8_t *hs = h + 9;
                uint32_t rsz = 0;
                if (clen < 2 || (hs[0] & ORD_NOSZ) || !varint_get(hs + 1, hs + clen, &rsz)) continue;
                DecompressReq r;
                r.h_in = hs;
                r.d_in = secs[i].in + 9;
                r.in_size = clen;
                r.out_cap = rsz;
                r.d_out = g.arena.alloc_n<uint8_t>(size_t(rsz) + 1);
                LzpDecReq z;
                z.d_in = r.d_out;
                z.d_out = secs[i].out;
                z.cap = ulen;
                lzp_rans.push_back(reqs.size());
                reqs.push_back(r);
                who.push_back(-1);
                lzd.push_back(z);
                who_lzp.push_back(i);
                continue;
            }
            if (h[0] != 0) continue;
            DecompressReq r;
            r.h_in = h + 9;
            r.d_in = secs[i].in + 9;
            r.in_size = clen;
            r.out_cap = ulen;
            r.d_out = secs[i].out;
            reqs.push_back(r);
            who.push_back(i);
        }
        const auto t1 = std::chrono::steady_clock::now();
        // ---- where each adaptive-model chain decodes (host_decode_mode():
        // 0 the GPU, 1 host cores, 2 by the chains' measured costs,
        // host::plan).  A quality chain with a sequence context waits for
        // its block's bases; when those come from a host chain it runs on
        // the host too (its bases are there) ----------------------------------
        const int hmode = host_decode_mode();
        std::vector<int> fqz_kind(fqz.size(), host::CK_FQZ), fqz_src(fqz.size(), -1);
        for (size_t k = 0; k < fqz.size(); k++) {
            const FqzDecReq &f = fqz[k];
            uint32_t tl = 0;
            const int vk = varint_get(f.h_in, f.h_in + f.in_size, &tl);
            if (vk > 0 && size_t(vk) + 1 < f.in_size && (f.h_in[vk + 1] & 8u) && f.d_seq) {
                fqz_kind[k] = host::CK_FQZ_SEQ;
                for (size_t m = 0; m < seqd.size(); m++)
                    if (seqd[m].d_out == f.d_seq) fqz_src[k] = int(m);
            }
        }
        std::vector<char> seq_on_host(seqd.size(), hmode == 1), fqz_on_host(fqz.size(), hmode == 1);
        if (hmode == 3) {                 // (tests: every other chain on the host)
            for (size_t m = 0; m < seqd.size(); m++) seq_on_host[m] = m % 2 == 0;
            for (size_t k = 0; k < fqz.size(); k++) fqz_on_host[k] = (seqd.size() + k) % 2 == 0;
        }
        if (hmode == 2 && !(seqd.empty() && fqz.empty())) {
            std::vector<uint64_t> n;
            std::vector<int> kind;
            for (const SeqDecReq &q : seqd) { n.push_back(q.n); kind.push_back(host::CK_SEQ); }
            for (size_t k = 0; k < fqz.size(); k++) { n.push_back(fqz[k].out_cap); kind.push_back(fqz_kind[k]); }
            const std::vector<char> on = host::plan(n, kind, host::threads());
            for (size_t m = 0; m < seqd.size(); m++) seq_on_host[m] = on[m];
            for (size_t k = 0; k < fqz.size(); k++) fqz_on_host[k] = on[seqd.size() + k];
        }
        for (size_t k = 0; k < fqz.size(); k++)
            if (fqz_src[k] >= 0 && seq_on_host[size_t(fqz_src[k])]) fqz_on_host[k] = 1;
        g_chains_host += uint64_t(std::count(seq_on_host.begin(), seq_on_host.end(), 1) +
                                  std::count(fqz_on_host.begin(), fqz_on_host.end(), 1));
        g_chains_gpu += uint64_t(std::count(seq_on_host.begin(), seq_on_host.end(), 0) +
                                 std::count(fqz_on_host.begin(), fqz_on_host.end(), 0));
        // ---- the host chains: sequence-model sections and quality sections
        // without a sequence context start now, beside the GPU's rANS and
        // names; quality sections with one wait for their block's bases
        struct HostChain { uint8_t *buf = nullptr; size_t cap = 0, n = 0; int sec = -1; bool ok = false; };
        std::vector<HostChain> hc;
        std::vector<size_t> hc_idx;                   // seqd / fqz index of each host chain
        std::vector<int> hc_kind;                     // host::ChainKind
        for (size_t k = 0; k < seqd.size(); k++) {
            if (!seq_on_host[k]) continue;
            HostChain c;
            c.cap = c.n = seqd[k].n;
            c.buf = g.staging.alloc(c.cap + 1);
            c.sec = who_seq[k];
            hc.push_back(c);
            hc_idx.push_back(k);
            hc_kind.push_back(host::CK_SEQ);
        }
        for (size_t k = 0; k < fqz.size(); k++) {
            if (!fqz_on_host[k]) continue;
            HostChain c;
            c.cap = fqz[k].out_cap;
            c.buf = g.staging.alloc(c.cap + 1);
            c.sec = who_fqz[k];
            hc.push_back(c);
            hc_idx.push_back(k);
            hc_kind.push_back(fqz_kind[k]);
        }
        auto timed = [](int kind, size_t n, const std::function<bool()> &fn) {
            const auto a = std::chrono::steady_clock::now();
            const bool ok = fn();
            const double ns = std::chrono::duration<double, std::nano>(std::chrono::steady_clock::now() - a).count();
            if (ok && n >= (1u << 20)) host::chain_measured(kind, false, ns / double(n));
            return ok;
        };
        host::Jobs hjobs;
        std::vector<size_t> early_h;                  // host chains that start now
        for (size_t j = 0; j < hc.size(); j++)
            if (hc_kind[j] != host::CK_FQZ_SEQ) early_h.push_back(j);
        hjobs.start(early_h.size(), [&](size_t t) {
            const size_t j = early_h[t];
            HostChain &c = hc[j];
            if (hc_kind[j] == host::CK_SEQ) {
                const SeqDecReq &q = seqd[hc_idx[j]];
                c.ok = timed(host::CK_SEQ, q.n, [&] {
                    return host::seq_decode(seq_h[hc_idx[j]], q.in_size, q.lens, q.nrec, q.both, q.k,
                                            c.buf, q.n) == 0;
                });
            } else {
                const FqzDecReq &f = fqz[hc_idx[j]];
                c.ok = timed(host::CK_FQZ, c.cap, [&] {
                    return host::fqz_decode(f.h_in, f.in_size, c.buf, c.cap, &c.n, nullptr, 0, nullptr, 0) == 0;
                });
            }
        });
        // the name sections on their helper context, beside the chains: their
        // host rebuild overlaps the GPU's rANS / fqz / sequence decoding
        // The name sections decode on their helper context beside the chains.
        // Each hedged chain copy holds a CU (its LDS), so while the names run
        // they count as a second hedging caller: the chains' copies take half
        // the CUs and the names' short kernels find the rest free (their
        // host rebuild needs no CU at all).
        std::exception_ptr nerr;
        double t_names_up = 0;                        // (trace) the names' upload done
        std::thread tn;
        GpuCtx *gn = nullptr;
        std::unique_ptr<HedgeShare> nshare;
        if (!nd.empty()) {
            gn = &gpu_aux(AUX_NAMES);
            nshare = std::make_unique<HedgeShare>(size_t(g.cus));
            tn = std::thread([&] {
                try {
                    FQZ5_HIP(hipSetDevice(gn->device));
                    names_decode_batch(*gn, nd);
                    // the names to their sections now, on the names context,
                    // while the chains still run (after them, on the main
                    // stream, -5 NovaSeq's 590 MB of names added ~50 ms)
                    for (size_t k = 0; k < nd.size(); k++)
                        if (nd[k].ok && nd[k].u_len)
                            FQZ5_HIP(hipMemcpyAsync(secs[who_name[k]].out, nd[k].names,
                                                    nd[k].u_len, hipMemcpyHostToDevice, gn->stream));
                    gn->sync();                       // (nd's buffers are the sources)
                    if (trace) t_names_up = now_ms();
                } catch (...) {
                    nerr = std::current_exception();
                }
            });
        }
        struct Join {                                 // joined on every exit
            std::thread &t;
            ~Join() { if (t.joinable()) t.join(); }
        } join_names{tn};
        // a GPU batch's time over its longest chain: the chain cost the plan reads
        auto gpu_timed = [](int kind, uint64_t longest, const std::function<void()> &fn) {
            const auto a = std::chrono::steady_clock::now();
            fn();
            const double ns = std::chrono::duration<double, std::nano>(std::chrono::steady_clock::now() - a).count();
            if (longest >= (1u << 20)) host::chain_measured(kind, true, ns / double(longest));
        };
        // GPU quality sections without a sequence context need nothing else
        // of this call: they decode on the fqz helper context from a thread
        // of their own, beside the rANS / LZP / sequence-model work, instead
        // of after it (a -5 Illumina step waited ~0.6 s for the rANS batch
        // before its 8 s fqz launch).  Those with one wait for the bases.
        std::vector<FqzDecReq> fqz_early;
        std::vector<size_t> early_of;                 // fqz index of each early request
        std::vector<char> is_early(fqz.size(), 0);
        uint64_t early_longest = 0;
        for (size_t k = 0; k < fqz.size(); k++) {
            if (fqz_on_host[k] || fqz_kind[k] == host::CK_FQZ_SEQ) continue;
            fqz_early.push_back(fqz[k]);
            early_of.push_back(k);
            is_early[k] = 1;
            early_longest = std::max<uint64_t>(early_longest, fqz[k].out_cap);
        }
        std::exception_ptr ferr;
        std::thread tf;
        GpuCtx *gf = nullptr;
        if (!fqz_early.empty()) {
            gf = &gpu_aux(0);
            tf = std::thread([&] {
                try {
                    FQZ5_HIP(hipSetDevice(gf->device));
                    gpu_timed(host::CK_FQZ, early_longest, [&] { fqz_decode_batch(*gf, fqz_early); });
                } catch (...) {
                    ferr = std::current_exception();
                }
            });
        }
        Join join_fqz{tf};
        // the GPU's sequence-model sections likewise (their own helper context)
        std::vector<SeqDecReq> seq_gpu;
        std::vector<size_t> seq_gpu_of;
        uint64_t seq_longest = 0;
        for (size_t m = 0; m < seqd.size(); m++)
            if (!seq_on_host[m]) {
                seq_gpu.push_back(seqd[m]);
                seq_gpu_of.push_back(m);
                seq_longest = std::max<uint64_t>(seq_longest, seqd[m].n);
            }
        std::exception_ptr serr;
        std::thread ts;
        GpuCtx *gs = nullptr;
        if (!seq_gpu.empty()) {
            gs = &gpu_aux(AUX_SEQ0);
            ts = std::thread([&] {
                try {
                    FQZ5_HIP(hipSetDevice(gs->device));
                    gpu_timed(host::CK_SEQ, seq_longest, [&] { seq_decode_batch(*gs, seq_gpu); });
                } catch (...) {
                    serr = std::current_exception();
                }
            });
        }
        Join join_seq{ts};
        decompress_batch(g, reqs);
        const double t_rans = trace ? now_ms() : 0;
        if (trace)
            std::fprintf(stderr, "decode_sections: %zu bytes to host in %.1f ms, rANS %.1f ms\n", tot,
                         std::chrono::duration<double, std::milli>(t1 - t0).count(),
                         std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t1).count());
        if (!lzd.empty()) {
            std::vector<LzpDecReq> run;
            std::vector<int> run_who;
            for (size_t k = 0; k < lzd.size(); k++) {
                const DecompressReq &r = reqs[lzp_rans[k]];
                if (!r.ok) continue;
                lzd[k].in_len = r.out_size;
                run.push_back(lzd[k]);
                run_who.push_back(who_lzp[k]);
            }
            lzp_decode_batch(g, run);
            for (size_t k = 0; k < run.size(); k++) {
                fqz5_section_result &R = res[run_who[k]];
                R.status = run[k].ok ? 0 : -1;
                R.usize = run[k].out_len;
            }
        }
        if (ts.joinable()) ts.join();
        if (serr) std::rethrow_exception(serr);
        for (size_t i = 0; i < seq_gpu.size(); i++) seqd[seq_gpu_of[i]] = seq_gpu[i];
        // after the rANS and sequence sections: a quality section's sequence
        // context may be the output of this call's sequence section (a GPU
        // one: host-decoded bases make their quality chain a host chain)
        {
            std::vector<FqzDecReq> late;
            std::vector<size_t> late_of;
            uint64_t longest = 0;
            for (size_t k = 0; k < fqz.size(); k++)
                if (!is_early[k] && !fqz_on_host[k]) {
                    late.push_back(fqz[k]);
                    late_of.push_back(k);
                    longest = std::max<uint64_t>(longest, fqz[k].out_cap);
                }
            if (!late.empty()) {
                gpu_timed(host::CK_FQZ_SEQ, longest, [&] { fqz_decode_batch(g, late); });
                for (size_t k = 0; k < late.size(); k++) fqz[late_of[k]] = late[k];
            }
        }
        if (tf.joinable()) tf.join();
        if (ferr) std::rethrow_exception(ferr);
        for (size_t k = 0; k < fqz_early.size(); k++) fqz[early_of[k]] = fqz_early[k];
        if (!hc.empty()) {
            hjobs.join();
            // the quality chains with a sequence context: their block's bases
            // on the host (a host-decoded sequence section's buffer, or a copy
            // of the GPU's output), per record pointers as the reference's s->seq
            std::vector<std::vector<const uint8_t *>> recp(hc.size());
            for (size_t j = 0; j < hc.size(); j++) {
                if (hc_kind[j] != host::CK_FQZ_SEQ) continue;
                const FqzDecReq &f = fqz[hc_idx[j]];
                const uint8_t *bases = nullptr;
                bool host_src = false;
                for (size_t m = 0; m < hc.size(); m++)
                    if (hc_kind[m] == host::CK_SEQ && secs[hc[m].sec].out == f.d_seq) {
                        bases = hc[m].ok ? hc[m].buf : nullptr;
                        host_src = true;
                    }
                uint64_t nb = 0;
                for (int r = 0; r < f.nrec; r++) nb += f.lens[r];
                if (!bases) {
                    uint8_t *b = g.staging.alloc(nb + 1);
                    if (!host_src) g.download(b, f.d_seq, nb);
                    else std::memset(b, 0, nb + 1);   // (its sequence chain failed)
                    bases = b;
                }
                recp[j].resize(size_t(std::max(f.nrec, 1)));
                uint64_t o = 0;
                for (int r = 0; r < f.nrec; r++) {
                    recp[j][size_t(r)] = bases + o;
                    o += f.lens[r];
                }
            }
            g.sync();
            host::Jobs hb;
            std::vector<size_t> late;
            for (size_t j = 0; j < hc.size(); j++)
                if (hc_kind[j] == host::CK_FQZ_SEQ) late.push_back(j);
            hb.start(late.size(), [&](size_t t) {
                HostChain &c = hc[late[t]];
                const FqzDecReq &f = fqz[hc_idx[late[t]]];
                c.ok = timed(host::CK_FQZ_SEQ, c.cap, [&] {
                    return host::fqz_decode(f.h_in, f.in_size, c.buf, c.cap, &c.n, nullptr, 0,
                                            recp[late[t]].data(), f.nrec) == 0;
                });
            });
            hb.join();
            for (HostChain &c : hc) {
                fqz5_section_result &R = res[c.sec];
                R.status = c.ok ? 0 : -1;
                R.usize = uint32_t(c.n);
                if (c.ok && c.n)
                    FQZ5_HIP(hipMemcpyAsync(secs[c.sec].out, c.buf, c.n, hipMemcpyHostToDevice, g.stream));
            }
        }
        const double t_hc = trace ? now_ms() : 0;
        if (tn.joinable()) tn.join();
        nshare.reset();
        if (nerr) std::rethrow_exception(nerr);
        const double t_nj = trace ? now_ms() : 0;
        for (size_t k = 0; k < nd.size(); k++) {
            fqz5_section_result &R = res[who_name[k]];
            if (!nd[k].ok) continue;                    // (uploaded by the names thread)
            R.status = 0;
            R.usize = nd[k].u_len;
        }
        for (size_t k = 0; k < reqs.size(); k++) {
            if (who[k] < 0) continue;                   // an LZP3 section's rANS stage
            fqz5_section_result &R = res[who[k]];
            R.status = reqs[k].ok ? 0 : -1;
            R.usize = reqs[k].out_size;
        }
        for (size_t k = 0; k < seqd.size(); k++) {
            if (seq_on_host[k]) continue;
            fqz5_section_result &R = res[who_seq[k]];
            R.status = seqd[k].ok ? 0 : -1;
            R.usize = seqd[k].n;
        }
        for (size_t k = 0; k < fqz.size(); k++) {
            if (fqz_on_host[k]) continue;
            fqz5_section_result &R = res[who_fqz[k]];
            R.status = fqz[k].ok ? 0 : -1;
            R.usize = uint32_t(fqz[k].out_size);
        }
        g.reset();
        if (gn) gn->reset();
        if (gf) gf->reset();
        if (gs) gs->reset();
        if (trace) {
            const double tb = std::chrono::duration<double, std::milli>(t0.time_since_epoch()).count();
            std::fprintf(stderr, "decode_sections: from its start: rANS done %.1f, host chains joined "
                         "%.1f, names uploaded %.1f, names joined %.1f, reset %.1f ms\n", t_rans - tb,
                         t_hc - tb, t_names_up ? t_names_up - tb : -1.0, t_nj - tb, now_ms() - tb);
        }
        return 0;
    } catch (const std::exception &e) {
        fqz5_set_error(e.what());
        try { gpu().reset(); } catch (...) {}
        try { gpu_aux_reset_all(); } catch (...) {}
        return -1;
    }
}

}  // extern "C"
