// capi.cpp — extern "C" entry points (include/fqz5_mi355x.h).
#include <algorithm>
#include <atomic>
#include <climits>
#include <cstdlib>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <cstdio>
#include <string>
#include <csignal>
#include <execinfo.h>
#include <unistd.h>
#include <sys/syscall.h>
#include <chrono>

#include "../../include/fqz5_mi355x.h"
#include "rans_codec.hpp"
#include "rans_format.hpp"
#include "fqz_kernels.h"
#include "arith_kernels.h"
#include "fqz_codec.hpp"
#include "host_dec.hpp"

// $FQZ5_SEGV_TRACE: on SIGSEGV print the native call stack (library offsets,
// for llvm-symbolizer) before the default action (a diagnostic for faults in
// host code, which the Python fault handler shows only as its own frames)
namespace {
void segv_trace(int sig) {
    void *bt[64];
    const int n = backtrace(bt, 64);
    const char msg[] = "[fqz5] native stack at the fault:\n";
    (void)!write(2, msg, sizeof msg - 1);
    backtrace_symbols_fd(bt, n, 2);
    std::signal(sig, SIG_DFL);
    std::raise(sig);
}
__attribute__((constructor)) void segv_trace_install() {
    if (std::getenv("FQZ5_SEGV_TRACE")) std::signal(SIGSEGV, segv_trace);
}
}  // namespace

namespace fqz5 {

// The trial's helper contexts (gpu_aux) each own streams that must run
// beside the calling thread's; HIP's default of 4 hardware queues per
// process makes them share queues and serialise.  Raise it when the process
// (e.g. the relinked CLI) loads this library before anything touched HIP:
// FQZ5_HW_QUEUES, when set, is used as given (experiments, fewer queues
// included); otherwise an unset GPU_MAX_HW_QUEUES or HIP's default of 4 is
// raised to 20, and any other value the caller chose is kept.  Not 32: once
// the helper contexts had mapped 32 queues, every later long kernel ran
// ~30 % slower (a 44.5M-symbol fqz decode 180 -> 232 ns per symbol after a
// -5 encode, 180 with 4, 8, 16 or 20 queues): the
// scheduler time-slices more queues than the hardware maps at once, and the
// running waves are preempted and restored.
__attribute__((constructor)) static void hw_queues_default() {
    const char *v = std::getenv("GPU_MAX_HW_QUEUES");
    const char *w = std::getenv("FQZ5_HW_QUEUES");
    if (w) {
        setenv("GPU_MAX_HW_QUEUES", w, 1);
        return;
    }
    if (!v || !*v || std::atoi(v) == 4) setenv("GPU_MAX_HW_QUEUES", "20", 1);
}

static thread_local std::string g_err;

// the process-wide kernel profile (gpu_ctx.hpp: ProfKernel)
static std::mutex g_prof_mu;
static double g_prof[PK_N][3];
static std::atomic<bool> g_prof_on{false};
void prof_add(int kernel, double ms, double bytes) {
    std::lock_guard<std::mutex> lk(g_prof_mu);
    g_prof[kernel][0] += ms;
    g_prof[kernel][1] += 1;
    g_prof[kernel][2] += bytes;
}
bool prof_on() { return g_prof_on.load(); }

struct ProfPending { int kernel; hipEvent_t a, b; double bytes; };
static std::vector<ProfPending> g_prof_pend;          // under g_prof_mu
ProfSpan::ProfSpan(int k, hipStream_t st) : s(st) {
    if (!prof_on()) return;
    if (hipEventCreate(&a) != hipSuccess) { a = nullptr; return; }
    if (hipEventRecord(a, s) != hipSuccess) { (void)hipEventDestroy(a); a = nullptr; return; }
    kernel = k;
}
long ProfSpan::end(double bytes) {
    if (kernel < 0) return -1;
    hipEvent_t b = nullptr;
    if (hipEventCreate(&b) != hipSuccess || hipEventRecord(b, s) != hipSuccess) {
        if (b) (void)hipEventDestroy(b);
        return -1;
    }
    std::lock_guard<std::mutex> lk(g_prof_mu);
    g_prof_pend.push_back({kernel, a, b, bytes});
    a = nullptr;
    kernel = -1;
    return long(g_prof_pend.size()) - 1;
}
ProfSpan::~ProfSpan() {
    if (a) (void)hipEventDestroy(a);
}
void prof_bytes(long token, double bytes) {
    if (token < 0) return;
    std::lock_guard<std::mutex> lk(g_prof_mu);
    if (size_t(token) < g_prof_pend.size()) g_prof_pend[size_t(token)].bytes = bytes;
}
// the queued spans into the table (their events complete first); under g_prof_mu
static void prof_drain() {
    for (ProfPending &p : g_prof_pend) {
        float ms = 0;
        if (hipEventSynchronize(p.b) == hipSuccess && hipEventElapsedTime(&ms, p.a, p.b) == hipSuccess) {
            g_prof[p.kernel][0] += ms;
            g_prof[p.kernel][1] += 1;
            g_prof[p.kernel][2] += p.bytes;
        }
        (void)hipEventDestroy(p.a);
        (void)hipEventDestroy(p.b);
    }
    g_prof_pend.clear();
}
static thread_local std::unique_ptr<GpuCtx> g_ctx;

static const auto g_t_load = std::chrono::steady_clock::now();
static double since_load_ms() {
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - g_t_load)
        .count();
}
bool call_trace_on() {
    static const bool on = [] {
        const char *e = std::getenv("FQZ5_CALL_TRACE");
        return e && e[0] && e[0] != '0';
    }();
    return on;
}
CallTrace::CallTrace(const char *f, size_t bytes) : fn(f), n(bytes) {
    if (!call_trace_on()) return;
    t[0] = since_load_ms();
    tag[0] = "enter";
    k = 1;
}
void CallTrace::mark(const char *what) {
    if (!k || k >= 9) return;
    t[k] = since_load_ms();
    tag[k++] = what;
}
CallTrace::~CallTrace() {
    if (!k) return;
    t[k] = since_load_ms();
    tag[k++] = "exit";
    char line[512];
    int p = std::snprintf(line, sizeof line, "[call] tid=%ld %s n=%zu", long(syscall(SYS_gettid)),
                          fn, n);
    for (int i = 0; i < k && p < int(sizeof line) - 40; i++)
        p += std::snprintf(line + p, sizeof line - size_t(p), " %s=%.2f", tag[i], t[i]);
    std::fprintf(stderr, "%s\n", line);
}

GpuCtx &gpu() {
    if (!g_ctx) g_ctx.reset(new GpuCtx());
    return *g_ctx;
}

#ifdef FQZ5_COPY_STATS
// diagnostics build (tools/build_variant.sh): host<->device copies per call site
struct CopyStats {
    std::mutex mu;
    std::map<std::string, uint64_t> n;
    ~CopyStats() {
        for (auto &kv : n) std::fprintf(stderr, "copies %8llu %s\n", (unsigned long long)kv.second, kv.first.c_str());
    }
};
static CopyStats g_cs;
void GpuCtx::copy_stat(const char *kind, const char *file, int line) {
    std::lock_guard<std::mutex> lk(g_cs.mu);
    g_cs.n[std::string(kind) + " " + file + ":" + std::to_string(line)]++;
}
#endif

static std::atomic<int> g_hedge{-1};
static std::atomic<int> g_hedging{0};
HedgeShare::HedgeShare(size_t all) {
    const int k = g_hedging.fetch_add(1) + 1;
    cus = std::max<size_t>(1, all / size_t(k));
}
HedgeShare::~HedgeShare() { g_hedging.fetch_sub(1); }

bool hedge_chains() {
    int v = g_hedge.load();
    if (v < 0) {
        v = std::getenv("FQZ5_NO_HEDGE") == nullptr ? 1 : 0;
        g_hedge.store(v);
    }
    return v != 0;
}

static std::atomic<int> g_dec_small{-1};
bool small_decoder_on() {
    int v = g_dec_small.load();
    if (v < 0) {
        const char *e = std::getenv("FQZ5_DEC_SMALL");   // on unless "0"
        v = e && e[0] == '0' ? 0 : 1;
        g_dec_small.store(v);
    }
    return v != 0;
}

static std::atomic<int> g_host_dec{-1};
int host_decode_mode() {
    int v = g_host_dec.load();
    if (v < 0) {
        const char *e = std::getenv("FQZ5_HOST_DECODE");
        v = e ? std::atoi(e) : 2;
        if (v < 0 || v > 3) v = 2;
        g_host_dec.store(v);
    }
    return v;
}

// The calling thread's helper contexts: their own streams and arenas, for
// work the thread hands to helper threads to run beside its own
// (fqz5_sections_try: LZP3, fqz and sequence-model candidates beside the
// rANS candidates).
static thread_local std::unique_ptr<GpuCtx> g_aux[AUX_CTXS];
// fqz5_stream_wait's event, once recorded: a helper context created later
// waits for it too (its streams then see the caller's producer work)
static thread_local hipEvent_t g_wait_ev = nullptr;
static thread_local bool g_wait_armed = false;
static void ctx_wait(GpuCtx &c, hipEvent_t ev) {
    FQZ5_HIP(hipStreamWaitEvent(c.stream, ev, 0));
    if (c.stream2) FQZ5_HIP(hipStreamWaitEvent(c.stream2, ev, 0));   // (a later one forks from stream)
}
GpuCtx &gpu_aux(int k) {
    if (!g_aux[k]) {
        // Normal priority, as this thread's context ($FQZ5_AUX_HIGH_PRIO=1:
        // the device's highest, rounds 2-4).  With the helpers at high
        // priority the -3 encode's pack stage waited ~220 ms behind the plain
        // rANS helper's chain in about half the steps (encode 300 ms on
        // average, 230-400; all at normal priority 254, 228-296); the -5
        // items were within their noise either way.
        // ($FQZ5_FQZ_HIGH_PRIO=1: the fqz helper alone at high priority,
        // for experiments on the -5 try's fqz statistics round trips)
        const bool high = std::getenv("FQZ5_AUX_HIGH_PRIO") != nullptr ||
                          (k == 0 && std::getenv("FQZ5_FQZ_HIGH_PRIO") != nullptr);
        g_aux[k].reset(new GpuCtx(high));
        if (g_wait_armed) ctx_wait(*g_aux[k], g_wait_ev);
    }
    return *g_aux[k];
}
void gpu_aux_reset_all() {
    for (auto &a : g_aux)
        if (a) a->reset();
}
static void release_ctx(GpuCtx &c) {
    c.sync();
    if (c.stream2) FQZ5_HIP(hipStreamSynchronize(c.stream2));
    c.arena.release();
    c.fqz_tmp.release();
    c.lzp_tmp.release();
    c.sort_tmp.release();
    c.ev_tmp.release();
    c.staging.reset();
}
void gpu_release_all() {
    if (g_ctx) release_ctx(*g_ctx);
    for (auto &a : g_aux)
        if (a) release_ctx(*a);
}
static uint64_t arena_bytes() { return ChunkPool::get().held(); }

// Size a stream decodes to, from its header (needed when the caller did
// not give an output buffer).  0 with ok=false if it cannot be known.
static uint32_t header_size(const uint8_t *in, uint32_t len, bool *ok) {
    *ok = false;
    if (!len) return 0;
    if ((in[0] & ORD_NOSZ) && !(in[0] & ORD_STRIPE)) return 0;
    uint32_t v = 0;
    if (!varint_get(in + 1, in + len, &v)) return 0;
    *ok = true;
    return v;
}

// ---------------------------------------------------------------------------
// The trial batch of the host-buffer encoder (the drop-in's
// rans_compress_4x16).  fqzcomp5's compress_with_methods tries a section's
// methods one call after another on the same input buffer while the codec
// trial runs (fqzcomp5.c:1979-2012: RANS0, RANS1, RANS129, RANS193, then
// RANSXN1 for qualities), and each call is a serial rANS chain of ~11M steps
// on the GPU.  So a call on an input that this thread saw before, or on a
// new input after one that was asked for several orders, codes the orders
// the last trial asked for as one batch (their chains run side by side on
// different CUs), returns the one asked for and keeps the others; a later
// call on the same bytes (memcmp against the kept copy) for one of those
// orders returns its kept output.  Outputs are the bytes a call of that
// order returns (the same deterministic coder); only calls with out == NULL
// (rans_compress_4x16, callee-allocated) take this path, so the capacity
// semantics of rans_compress_to_4x16 are untouched.  $FQZ5_NO_TRIAL_BATCH
// turns it off.
struct TrialCache {
    std::vector<uint8_t> in;      // the input's bytes: the upload source and the comparison
    uint32_t n = 0;
    bool valid = false;
    std::vector<int> asked;       // orders asked for on this input, in call order
    // coded ahead, not yet asked: kept in device memory (its own arena) and
    // brought down only when asked (a batch call brings down one output)
    std::map<int, std::pair<uint8_t *, uint32_t>> ready;
    DevArena dev;
    void drop_ready() {                      // (no queued work uses dev: batches sync)
        ready.clear();
        dev.reset();
    }
};
static thread_local TrialCache t_trial;
static thread_local std::vector<int> t_pat;            // this thread's last multi-order input
static std::mutex g_pat_mu;
static std::vector<int> g_pat;                         // the last multi-order input of any thread
// Before any input was asked for several orders: the preset trials' rANS
// orders (RANS0, RANS1, RANS129, RANS193), which compress_with_methods
// starts with RANS0 (the lowest method bit, fqzcomp5.c:1979-1998)
static const std::vector<int> k_trial_default{0, 1, 129, 193};
static std::atomic<uint64_t> g_trial_stats[3];         // calls, served from a batch, batches > 1
static bool trial_batch_on() {
    static const bool on = std::getenv("FQZ5_NO_TRIAL_BATCH") == nullptr;
    return on;
}
constexpr uint32_t TRIAL_MIN_BYTES = 1u << 16;         // smaller inputs: the plain call

static unsigned char *rans_compress_trial(const unsigned char *in, unsigned int in_size,
                                          unsigned int *out_size, int order, CallTrace &ct) {
    TrialCache &c = t_trial;
    g_trial_stats[0]++;
    const bool same = c.valid && c.n == in_size && std::memcmp(c.in.data(), in, in_size) == 0;
    std::vector<int> want{order};
    if (same) {
        if (std::find(c.asked.begin(), c.asked.end(), order) == c.asked.end())
            c.asked.push_back(order);
        auto it = c.ready.find(order);
        if (it != c.ready.end()) {
            const uint32_t sz = it->second.second;
            auto *r = static_cast<unsigned char *>(malloc(compress_bound(in_size, order)));
            if (!r) { *out_size = 0; return nullptr; }
            if (sz) FQZ5_HIP(hipMemcpy(r, it->second.first, sz, hipMemcpyDeviceToHost));
            *out_size = sz;
            c.ready.erase(it);
            g_trial_stats[1]++;
            return r;
        }
        // a trial the last pattern did not foresee: the preset orders as well
        for (int o : {0, 1, 129, 193})
            if (std::find(c.asked.begin(), c.asked.end(), o) == c.asked.end() && !c.ready.count(o))
                want.push_back(o);
    } else {
        if (c.valid && c.asked.size() >= 2) {
            t_pat = c.asked;
            std::lock_guard<std::mutex> lk(g_pat_mu);
            g_pat = c.asked;
        }
        c.drop_ready();
        c.valid = false;
        if (c.in.size() < in_size) c.in.resize(in_size);
        std::memcpy(c.in.data(), in, in_size);
        c.n = in_size;
        c.valid = true;
        c.asked.assign(1, order);
        // a trial asks its orders in a fixed sequence: a call for the first
        // order of the last trial seen (this thread's, else any thread's,
        // else the presets') starts another, and the rest is coded with it.
        // A block past the trial asks one order, its section's winner, on
        // each input: only when that winner is the trial's first order is
        // the batch coded for nothing (beside a chain at least as long).
        std::vector<int> pat = t_pat;
        if (pat.empty()) {
            std::lock_guard<std::mutex> lk(g_pat_mu);
            pat = g_pat.empty() ? k_trial_default : g_pat;
        }
        if (!pat.empty() && pat[0] == order)
            for (int o : pat)
                if (o != order) want.push_back(o);
    }
    if (want.size() > 1) g_trial_stats[2]++;
    ct.mark("copy");
    GpuCtx &g = gpu();
    const uint8_t *d_in = g.upload_sync(c.in.data(), in_size);
    if (ct.k) { g.sync(); ct.mark("up"); }
    std::vector<CompressReq> reqs(want.size());
    for (size_t i = 0; i < want.size(); i++) {
        reqs[i].d_in = d_in;
        reqs[i].n = in_size;
        reqs[i].order = want[i];
        reqs[i].cap = compress_bound(in_size, want[i]);
    }
    compress_batch(g, reqs);
    if (ct.k) { g.sync(); ct.mark("run"); }
    unsigned char *asked = nullptr;
    uint32_t asked_sz = 0;
    std::vector<const Layout *> keep;
    std::vector<uint8_t *> keep_at;
    for (size_t i = 0; i < reqs.size(); i++) {
        if (!reqs[i].ok) continue;                     // (a speculated order: not kept)
        const uint32_t sz = layout_size(reqs[i].out);
        if (i == 0) {
            auto *dst = static_cast<unsigned char *>(malloc(compress_bound(in_size, want[i])));
            if (!dst) continue;
            write_layout_host(g, reqs[i].out, dst);
            asked = dst;
            asked_sz = sz;
        } else {
            uint8_t *d = c.dev.alloc_n<uint8_t>(std::max<uint32_t>(sz, 1));
            keep.push_back(&reqs[i].out);
            keep_at.push_back(d);
            c.ready[want[i]] = {d, sz};
        }
    }
    if (!keep.empty()) {                               // one copy launch for all of them
        write_layouts_dev(g, keep, keep_at);
        g.sync();
    }
    ct.mark("down");
    g.reset();
    if (!asked) {
        *out_size = 0;
        return nullptr;
    }
    *out_size = asked_sz;
    return asked;
}

}  // namespace fqz5

using namespace fqz5;

#define GUARD_BEGIN try {
#define GUARD_END(failret)                                                    \
    }                                                                         \
    catch (const std::exception &e) {                                         \
        g_err = e.what();                                                     \
        try { if (g_ctx) g_ctx->reset(); } catch (...) {}                     \
        return failret;                                                       \
    }

namespace fqz5 {
void fqz5_set_error(const char *msg) { g_err = msg; }
// fqz_codec.cpp
uint8_t *fqz_encode_gpu(int vers, fqz_slice *s, const uint8_t *in, size_t n, size_t *out_size,
                        int strat, fqz_gparams *gp);
uint8_t *fqz_decode_gpu(const uint8_t *in, size_t in_size, size_t *out_size, int *lengths,
                        int nlengths, fqz_slice *s);
}

extern "C" {

char *fqz_compress(int vers, fqz_slice *s, char *in, size_t in_size, size_t *out_size,
                   int strat, fqz_gparams *gp) {
    GUARD_BEGIN
    if (!s || !out_size || (!in && in_size)) return nullptr;
    CallTrace ct("fqz_compress", in_size);
    return reinterpret_cast<char *>(fqz_encode_gpu(
        vers, s, reinterpret_cast<const uint8_t *>(in), in_size, out_size, strat, gp));
    GUARD_END(nullptr)
}

char *fqz_decompress(char *in, size_t in_size, size_t *out_size, int *lengths, int nlengths,
                     fqz_slice *s) {
    GUARD_BEGIN
    if (!in || !out_size) return nullptr;
    CallTrace ct("fqz_decompress", in_size);
    return reinterpret_cast<char *>(fqz_decode_gpu(
        reinterpret_cast<const uint8_t *>(in), in_size, out_size, lengths, nlengths, s));
    GUARD_END(nullptr)
}

unsigned int rans_compress_bound_4x16(unsigned int size, int order) {
    return compress_bound(size, order);
}

unsigned char *rans_compress_to_4x16(unsigned char *in, unsigned int in_size,
                                     unsigned char *out, unsigned int *out_size,
                                     int order) {
    if (in_size > unsigned(INT_MAX) || (out && *out_size == 0)) {
        *out_size = 0;
        return nullptr;
    }
    GUARD_BEGIN
    CallTrace ct("rans_compress", in_size);
    if (!out && in && in_size >= TRIAL_MIN_BYTES && trial_batch_on()) {
        return rans_compress_trial(in, in_size, out_size, order, ct);
    }
    GpuCtx &g = gpu();
    std::vector<CompressReq> reqs(1);
    reqs[0].d_in = g.upload_sync(in, in_size);
    if (ct.k) { g.sync(); ct.mark("up"); }
    reqs[0].n = in_size;
    reqs[0].order = order;
    reqs[0].cap = out ? *out_size : compress_bound(in_size, order);
    compress_batch(g, reqs);
    if (ct.k) { g.sync(); ct.mark("run"); }
    if (!reqs[0].ok) {
        g.reset();
        *out_size = 0;
        return nullptr;
    }
    const uint32_t sz = layout_size(reqs[0].out);
    unsigned char *dst = out;
    if (!dst) {
        dst = static_cast<unsigned char *>(malloc(compress_bound(in_size, order)));
        if (!dst) { g.reset(); *out_size = 0; return nullptr; }
    }
    write_layout_host(g, reqs[0].out, dst);
    g.reset();
    *out_size = sz;
    return dst;
    GUARD_END((*out_size = 0, nullptr))
}

unsigned char *rans_compress_4x16(unsigned char *in, unsigned int in_size,
                                  unsigned int *out_size, int order) {
    return rans_compress_to_4x16(in, in_size, nullptr, out_size, order);
}

unsigned char *rans_uncompress_to_4x16(unsigned char *in, unsigned int in_size,
                                       unsigned char *out, unsigned int *out_size) {
    if (!in_size) return nullptr;
    GUARD_BEGIN
    uint32_t cap;
    if (out) {
        cap = *out_size;
    } else {
        bool ok;
        cap = header_size(in, in_size, &ok);
        if (!ok || cap >= unsigned(INT_MAX)) return nullptr;
    }
    CallTrace ct("rans_uncompress", in_size);
    GpuCtx &g = gpu();
    std::vector<DecompressReq> reqs(1);
    reqs[0].h_in = in;
    reqs[0].d_in = g.upload_sync(in, in_size);
    if (ct.k) { g.sync(); ct.mark("up"); }
    reqs[0].in_size = in_size;
    reqs[0].out_cap = cap;
    reqs[0].d_out = g.arena.alloc_n<uint8_t>(size_t(cap) + 1);
    decompress_batch(g, reqs);
    if (ct.k) { g.sync(); ct.mark("run"); }
    if (!reqs[0].ok) { g.reset(); return nullptr; }
    unsigned char *dst = out;
    if (!dst) {
        dst = static_cast<unsigned char *>(malloc(cap ? cap : 1));
        if (!dst) { g.reset(); return nullptr; }
    }
    g.download(dst, reqs[0].d_out, reqs[0].out_size);
    g.reset();
    *out_size = reqs[0].out_size;
    return dst;
    GUARD_END(nullptr)
}

unsigned char *rans_uncompress_4x16(unsigned char *in, unsigned int in_size,
                                    unsigned int *out_size) {
    return rans_uncompress_to_4x16(in, in_size, nullptr, out_size);
}

void rans_set_cpu(int) {}

unsigned int arith_compress_bound(unsigned int size, int order) {
    return arith_compress_bound_ref(size, order);
}

unsigned char *arith_compress_to(unsigned char *in, unsigned int in_size, unsigned char *out,
                                 unsigned int *out_size, int order) {
    GUARD_BEGIN
    return arith_compress_gpu(in, in_size, out, out_size, order);
    GUARD_END(nullptr)
}

unsigned char *arith_compress(unsigned char *in, unsigned int in_size, unsigned int *out_size,
                              int order) {
    return arith_compress_to(in, in_size, nullptr, out_size, order);
}

unsigned char *arith_uncompress_to(unsigned char *in, unsigned int in_size, unsigned char *out,
                                   unsigned int *out_sz) {
    GUARD_BEGIN
    return arith_uncompress_gpu(in, in_size, out, out_sz);
    GUARD_END(nullptr)
}

unsigned char *arith_uncompress(unsigned char *in, unsigned int in_size,
                                unsigned int *out_size) {
    return arith_uncompress_to(in, in_size, nullptr, out_size);
}

int fqz5_rans_compress_batch(fqz5_rans_job *jobs, int n) {
    GUARD_BEGIN
    GpuCtx &g = gpu();
    std::vector<CompressReq> reqs(n);
    for (int i = 0; i < n; i++) {
        reqs[i].d_in = jobs[i].in;
        reqs[i].n = jobs[i].in_size;
        reqs[i].order = jobs[i].order;
        reqs[i].cap = jobs[i].out_cap;
    }
    compress_batch(g, reqs);
    std::vector<const Layout *> ls;
    std::vector<uint8_t *> dsts;
    for (int i = 0; i < n; i++) {
        jobs[i].status = reqs[i].ok ? 0 : -1;
        jobs[i].out_size = reqs[i].ok ? layout_size(reqs[i].out) : 0;
        if (reqs[i].ok) {
            ls.push_back(&reqs[i].out);
            dsts.push_back(jobs[i].out);
        }
    }
    write_layouts_dev(g, ls, dsts);
    g.reset();
    return 0;
    GUARD_END(-1)
}

int fqz5_rans_uncompress_batch(fqz5_rans_job *jobs, int n) {
    GUARD_BEGIN
    GpuCtx &g = gpu();
    // headers are parsed on the host: bring the compressed bytes over
    size_t tot = 0;
    for (int i = 0; i < n; i++) tot += jobs[i].in_size;
    std::vector<uint8_t> host(tot + 1);
    std::vector<DecompressReq> reqs(n);
    size_t off = 0;
    for (int i = 0; i < n; i++) {
        g.download(host.data() + off, jobs[i].in, jobs[i].in_size);
        reqs[i].h_in = host.data() + off;
        reqs[i].d_in = jobs[i].in;
        reqs[i].in_size = jobs[i].in_size;
        reqs[i].out_cap = jobs[i].out_cap;
        reqs[i].d_out = jobs[i].out;
        off += jobs[i].in_size;
    }
    g.sync();
    decompress_batch(g, reqs);
    for (int i = 0; i < n; i++) {
        jobs[i].status = reqs[i].ok ? 0 : -1;
        jobs[i].out_size = reqs[i].out_size;
    }
    g.reset();
    return 0;
    GUARD_END(-1)
}

int fqz5_stream_wait(void *stream) {
    try {
        // one event per thread, re-recorded: every stream of the calling
        // thread's contexts (its own and the helper contexts the entry
        // points hand work to) waits for the work enqueued on `stream` so
        // far (device-side, no host sync)
        GpuCtx &g = gpu();
        if (!g_wait_ev) FQZ5_HIP(hipEventCreateWithFlags(&g_wait_ev, hipEventDisableTiming));
        FQZ5_HIP(hipEventRecord(g_wait_ev, static_cast<hipStream_t>(stream)));
        ctx_wait(g, g_wait_ev);
        for (auto &a : g_aux)
            if (a) ctx_wait(*a, g_wait_ev);
        g_wait_armed = true;
        return 0;
    } catch (const std::exception &e) {
        g_err = e.what();
        return -1;
    }
}

void *fqz5_stream(void) {
    try {
        return gpu().stream;
    } catch (const std::exception &e) {
        g_err = e.what();
        return nullptr;
    }
}

int fqz5_device_ok(void) {
    try {
        gpu();
        return 1;
    } catch (const std::exception &e) {
        g_err = e.what();
        return 0;
    }
}

const char *fqz5_last_error(void) { return g_err.c_str(); }

uint64_t fqz5_arena_bytes(void) { return arena_bytes(); }
uint64_t fqz5_arena_peak(int reset) { return ChunkPool::get().peak(reset != 0); }
uint64_t fqz5_arena_use_peak(int reset) { return ChunkPool::get().use_peak(reset != 0); }

unsigned fqz5_set_hot_min(unsigned min_events) { return fqz_set_hot_min(min_events); }

int fqz5_host_threads(void) { return host::threads(); }

void fqz5_trial_batch_stats(uint64_t *out3) {
    for (int i = 0; i < 3; i++) out3[i] = g_trial_stats[i].load();
}

int fqz5_set_host_decode(int mode) {
    const int prev = host_decode_mode();
    g_host_dec.store(mode < 0 || mode > 3 ? 2 : mode);
    return prev;
}

void fqz5_fqz_dec_counts(uint64_t *out2) {
    out2[0] = fqz_dec_blocks(false);
    out2[1] = fqz_dec_blocks(true);
}

int fqz5_set_dec_small(int on) {
    const int prev = small_decoder_on() ? 1 : 0;
    g_dec_small.store(on ? 1 : 0);
    return prev;
}

int fqz5_set_hedge(int on) {
    const int prev = hedge_chains() ? 1 : 0;
    g_hedge.store(on ? 1 : 0);
    return prev;
}

void fqz5_profile(int on) {
    try {
        GpuCtx &g = gpu();
        g.prof = KernelProfile();
        g.prof.on = on != 0;
        {
            std::lock_guard<std::mutex> lk(g_prof_mu);
            prof_drain();
            for (int k = 0; k < PK_N; k++) g_prof[k][0] = g_prof[k][1] = g_prof[k][2] = 0;
        }
        g_prof_on.store(on != 0);
    } catch (const std::exception &e) {
        g_err = e.what();
    }
}

int fqz5_profile_read_all(double *out, int nk) {
    std::lock_guard<std::mutex> lk(g_prof_mu);
    prof_drain();
    const int n = nk < int(PK_N) ? nk : int(PK_N);
    for (int k = 0; k < n; k++)
        for (int j = 0; j < 3; j++) out[3 * k + j] = g_prof[k][j];
    return int(PK_N);
}

void fqz5_profile_read(double *out6) {
    try {
        const KernelProfile &p = gpu().prof;
        out6[0] = p.enc_ms; out6[1] = p.enc_launches; out6[2] = p.enc_bytes;
        out6[3] = p.dec_ms; out6[4] = p.dec_launches; out6[5] = p.dec_bytes;
    } catch (const std::exception &e) {
        g_err = e.what();
    }
}

long fqz5_fqz_div_selftest(void) {
    try {
        GpuCtx &g = gpu();
        g.reset();
        uint32_t *d = g.arena.alloc_n<uint32_t>(1);
        g.memset0(d, sizeof(uint32_t));
        FQZ5_HIP(fqz_div_selftest(d, g.stream));
        uint32_t bad = 0;
        g.download(&bad, d, 1);
        g.sync();
        g.reset();
        return long(bad);
    } catch (const std::exception &e) {
        g_err = e.what();
        return -1;
    }
}

}  // extern "C"
