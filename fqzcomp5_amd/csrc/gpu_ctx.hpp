// gpu_ctx.hpp — per-host-thread GPU context: one HIP stream plus a device
// bump arena that is reset after every batch.  The htscodecs entry points
// are re-entrant and called from many worker threads at once
// (fqzcomp5.c:2721-2729); giving each host thread its own
// stream and arena keeps concurrent calls independent.
#pragma once
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <atomic>
#include <mutex>
#include <stdexcept>
#include <string>
#include <utility>
#include <vector>

namespace fqz5 {

struct GpuError : std::runtime_error {
    using std::runtime_error::runtime_error;
};

#define FQZ5_HIP(expr)                                                        \
    do {                                                                      \
        hipError_t e_ = (expr);                                               \
        if (e_ != hipSuccess)                                                 \
            throw ::fqz5::GpuError(std::string(#expr) + ": " +               \
                                   hipGetErrorString(e_));                    \
    } while (0)

// Device memory: one process-wide pool of chunks shared by every context's
// arena.  An arena takes chunks from the pool as it grows and gives them all
// back at reset() (after its stream has drained), so the device footprint
// is the peak of what the contexts use at the same time, not the sum of each
// context's own peak.  Idle chunks beyond keep_idle()
// (a quarter of the device's memory or the work's peak, whichever is more)
// go back to the device.
class ChunkPool {
  public:
    static ChunkPool &get() {
        static ChunkPool *p = new ChunkPool();   // never destroyed (thread exits use it)
        return *p;
    }
    // a chunk of at least `need` bytes (its size in *got)
    void *take(size_t need, size_t *got) {
        {
            std::lock_guard<std::mutex> lk(m_);
            auto it = idle_.lower_bound(need);
            if (it != idle_.end()) {
                void *b = it->second;
                const size_t sz = it->first;
                idle_.erase(it);
                *got = sz;
                idle_bytes_ -= sz;
                use(sz);
                return b;
            }
        }
        void *b = nullptr;
        alloc_calls().fetch_add(1, std::memory_order_relaxed);
        hipError_t e = hipMalloc(&b, need);
        if (e != hipSuccess) {              // the idle chunks back to the device, once more
            trim(0);
            FQZ5_HIP(hipMalloc(&b, need));
        }
        std::lock_guard<std::mutex> lk(m_);
        held_ += need;
        peak_ = std::max(peak_, held_);
        use(need);
        *got = need;
        return b;
    }
    void give(void *b, size_t sz) {
        bool over;
        size_t keep;
        {
            std::lock_guard<std::mutex> lk(m_);
            idle_.emplace(sz, b);
            idle_bytes_ += sz;
            in_use_ -= sz;
            keep = keep_idle();
            over = idle_bytes_ > keep;
        }
        if (over) trim(keep);
    }
    void drop(void *b, size_t sz) {
        (void)hipFree(b);
        std::lock_guard<std::mutex> lk(m_);
        held_ -= sz;
        in_use_ -= sz;
    }
    // idle chunks back to the device until at most `keep` bytes stay idle
    // hipMalloc / hipHostMalloc / hipFree calls so far (FQZ5_STEP_TRACE:
    // calls inside a step can stall it)
    static std::atomic<uint64_t> &alloc_calls() { static std::atomic<uint64_t> n{0}; return n; }
    static std::atomic<uint64_t> &free_calls() { static std::atomic<uint64_t> n{0}; return n; }
    void trim(size_t keep) {
        std::vector<std::pair<size_t, void *>> out;
        {
            std::lock_guard<std::mutex> lk(m_);
            while (idle_bytes_ > keep && !idle_.empty()) {
                auto it = std::prev(idle_.end());        // the largest first
                out.emplace_back(it->first, it->second);
                idle_bytes_ -= it->first;
                held_ -= it->first;
                idle_.erase(it);
            }
        }
        free_calls().fetch_add(out.size(), std::memory_order_relaxed);
        for (auto &c : out) (void)hipFree(c.second);
    }
    size_t held() { std::lock_guard<std::mutex> lk(m_); return held_; }
    size_t peak(bool reset) {
        std::lock_guard<std::mutex> lk(m_);
        const size_t p = peak_;
        if (reset) peak_ = held_;
        return p;
    }
    // the most bytes in use at once (held minus idle: what the work itself
    // needed, without the chunks kept idle for reuse)
    size_t use_peak(bool reset) {
        std::lock_guard<std::mutex> lk(m_);
        const size_t p = use_peak_;
        if (reset) use_peak_ = in_use_;
        return p;
    }

  private:
    // Idle chunks kept for reuse: a quarter of the device's memory, or the
    // most the work has had in use at once when that is more (at most 70 %
    // of the device); $FQZ5_ARENA_IDLE_GB fixes it.  Trimming calls hipFree,
    // which waits for every kernel on the device to finish: a trim in the
    // middle of a step stalls the calling thread behind the longest chain
    // (measured: the names helper of a -3 step blocked ~150 ms), and a pool
    // trimmed below a step's peak allocates it again next step (-5 NovaSeq:
    // peak 102 GB in use against a 72 GB cap), so steady state must not trim.
    static size_t dev_total() {
        static const size_t t = [] {
            size_t fr = 0, tot = 0;
            if (hipMemGetInfo(&fr, &tot) != hipSuccess || !tot) tot = size_t(64) << 30;
            return tot;
        }();
        return t;
    }
    size_t keep_idle() const {   // under m_
        static const long fixed = [] {
            const char *e = std::getenv("FQZ5_ARENA_IDLE_GB");
            return e ? long(std::atof(e) * 1e9) : -1L;
        }();
        if (fixed >= 0) return size_t(fixed);
        const size_t tot = dev_total();
        return std::min(tot / 10 * 7, std::max(tot / 4, max_use_));
    }
    void use(size_t n) {   // under m_
        in_use_ += n;
        use_peak_ = std::max(use_peak_, in_use_);
        max_use_ = std::max(max_use_, in_use_);
    }
    std::mutex m_;
    std::multimap<size_t, void *> idle_;
    size_t idle_bytes_ = 0, held_ = 0, peak_ = 0, in_use_ = 0, use_peak_ = 0, max_use_ = 0;
};

// A bump arena over pool chunks; reset() rewinds and returns the chunks.
class DevArena {
  public:
    ~DevArena() {
        for (auto &c : chunks_) ChunkPool::get().drop(c.base, c.size);
    }
    void *alloc(size_t n, size_t align = 256, const char *file = __builtin_FILE(),
                int line = __builtin_LINE()) {
        if (n == 0) n = 1;
        if (trace_on()) trace(n, file, line);
        for (; cur_ < chunks_.size(); cur_++) {
            Chunk &c = chunks_[cur_];
            size_t off = (c.used + align - 1) & ~(align - 1);
            if (off + n <= c.size) {
                c.used = off + n;
                return static_cast<uint8_t *>(c.base) + off;
            }
        }
        const size_t need = n + align > (size_t(256) << 20) ? n + align : (size_t(256) << 20);
        Chunk c{nullptr, 0, 0};
        c.base = ChunkPool::get().take(need, &c.size);
        chunks_.push_back(c);
        cur_ = chunks_.size() - 1;
        chunks_[cur_].used = n;
        return c.base;
    }
    template <class T> T *alloc_n(size_t n, const char *file = __builtin_FILE(),
                                  int line = __builtin_LINE()) {
        return static_cast<T *>(alloc(n * sizeof(T), alignof(T) > 256 ? alignof(T) : 256, file,
                                      line));
    }
    // (only once nothing queued uses the arena any more)
    void reset() {
        if (trace_on()) trace_dump();
        if (!shared()) {                 // $FQZ5_ARENA_POOL=0: keep them (rewind only)
            for (auto &c : chunks_) c.used = 0;
            cur_ = 0;
            return;
        }
        for (auto &c : chunks_) ChunkPool::get().give(c.base, c.size);
        chunks_.clear();
        cur_ = 0;
    }
    // every chunk and the pool's idle ones back to the device
    void release() {
        if (trace_on()) trace_dump();
        for (auto &c : chunks_) ChunkPool::get().drop(c.base, c.size);
        chunks_.clear();
        cur_ = 0;
        ChunkPool::get().trim(0);
    }
    // device bytes held (all chunks, used or not)
    size_t bytes() const {
        size_t t = 0;
        for (auto &c : chunks_) t += c.size;
        return t;
    }

  private:
    struct Chunk { void *base; size_t size, used; };
    std::vector<Chunk> chunks_;
    size_t cur_ = 0;
    static bool shared() {
        static const bool on = [] {
            const char *e = std::getenv("FQZ5_ARENA_POOL");
            return !(e && e[0] == '0');
        }();
        return on;
    }
    // FQZ5_ARENA_TRACE=<MB>: per call site, the bytes taken between two
    // resets, printed at the reset when their sum is at least <MB> (a
    // diagnostic for the footprint per input byte)
    std::vector<std::pair<std::string, size_t>> sites_;
    static size_t trace_on() {
        static const size_t mb = [] {
            const char *e = std::getenv("FQZ5_ARENA_TRACE");
            return e ? size_t(std::strtoull(e, nullptr, 10)) : size_t(0);
        }();
        return mb;
    }
    void trace(size_t n, const char *file, int line) {
        const char *b = std::strrchr(file, '/');
        std::string k = std::string(b ? b + 1 : file) + ":" + std::to_string(line);
        for (auto &s : sites_)
            if (s.first == k) { s.second += n; return; }
        sites_.emplace_back(k, n);
    }
    void trace_dump() {
        size_t tot = 0;
        for (auto &s : sites_) tot += s.second;
        if (tot >= (trace_on() << 20)) {
            std::sort(sites_.begin(), sites_.end(),
                      [](const auto &a, const auto &b) { return a.second > b.second; });
            std::fprintf(stderr, "[arena] %.3f GB (pool %.3f GB, peak %.3f GB):", tot / 1e9,
                         ChunkPool::get().held() / 1e9, ChunkPool::get().peak(false) / 1e9);
            for (size_t i = 0; i < sites_.size() && i < 14; i++)
                std::fprintf(stderr, " %s=%.3f", sites_[i].first.c_str(), sites_[i].second / 1e9);
            std::fprintf(stderr, "\n");
        }
        sites_.clear();
    }
};

// Pinned host staging: every host->device upload is first copied here so
// the caller's buffer may die before the asynchronous copy runs.
class PinnedArena {
  public:
    ~PinnedArena() {
        for (auto &c : chunks_) (void)hipHostFree(c.base);
    }
    uint8_t *alloc(size_t n) {
        n = (n + 63) & ~size_t(63);
        for (; cur_ < chunks_.size(); cur_++) {
            Chunk &c = chunks_[cur_];
            if (c.used + n <= c.size) {
                uint8_t *p = c.base + c.used;
                c.used += n;
                return p;
            }
        }
        // (8 MB chunks: pinning 64 MB on a thread's first upload took ~100-200 ms
        // with several new threads at once, the drop-in CLI's workers)
        size_t sz = n > (size_t(8) << 20) ? n : (size_t(8) << 20);
        Chunk c{nullptr, sz, n};
        ChunkPool::alloc_calls().fetch_add(1, std::memory_order_relaxed);
        FQZ5_HIP(hipHostMalloc(reinterpret_cast<void **>(&c.base), sz, hipHostMallocDefault));
        chunks_.push_back(c);
        cur_ = chunks_.size() - 1;
        return c.base;
    }
    void reset() {
        for (auto &c : chunks_) c.used = 0;
        cur_ = 0;
    }

  private:
    struct Chunk { uint8_t *base; size_t size, used; };
    std::vector<Chunk> chunks_;
    size_t cur_ = 0;
};

// Live per-kernel timing (HIP events on the launching context's stream),
// read by the benchmark to find the dominant kernel of a step and its
// roofline.  One process-wide table of the chain kernels of every codec
// family, filled from every context (helper contexts included) while
// fqz5_profile(1) is on: launch time, launches, algorithmic bytes (the
// kernel's input plus output of its jobs).
enum ProfKernel {
    PK_ENC_CHAIN, PK_RANS_DEC, PK_FQZ_DEC, PK_FQZ_RC, PK_SEQ_DEC,           // (the first five: r01-r04)
    PK_ENC_CHAIN2W, PK_ENC_REPLAY, PK_SEQ_MODEL, PK_FQZ_MODEL_HOT, PK_FQZ_EV_FILL, PK_LZP_DEC,
    PK_ENC_REPLAY0, PK_N
};
void prof_add(int kernel, double ms, double bytes);
bool prof_on();
// One kernel launch timed on its own stream: begin() records an event before
// the launch, end() one after it and queues the pair; fqz5_profile_read_all
// synchronises the queued events and adds their spans (so no launch site
// waits for its kernel).  `bytes` (algorithmic input + output) may be set
// after end() with prof_bytes(token) once known.  No-ops while profiling is
// off (token -1).
struct ProfSpan {
    int kernel = -1;
    hipStream_t s = nullptr;
    hipEvent_t a = nullptr;
    ProfSpan(int k, hipStream_t st);
    long end(double bytes);
    ProfSpan(const ProfSpan &) = delete;
    ProfSpan &operator=(const ProfSpan &) = delete;
    ~ProfSpan();
};
void prof_bytes(long token, double bytes);

// $FQZ5_CALL_TRACE=1: one stderr line per host-buffer C-ABI call (the
// drop-in's entry points): the thread, the call, its input size, and the
// milliseconds since the library loaded at entry, at each stage mark and at
// exit (the marks sync the stream first, so the stages do not overlap).
bool call_trace_on();
struct CallTrace {
    const char *fn;
    size_t n;
    double t[10];
    const char *tag[10];
    int k = 0;
    CallTrace(const char *f, size_t bytes);
    void mark(const char *what);            // a stage ends here
    ~CallTrace();
};

struct KernelProfile {
    bool on = false;
    double enc_ms = 0, dec_ms = 0;
    double enc_launches = 0, dec_launches = 0;
    double enc_bytes = 0, dec_bytes = 0;   // algorithmic: input + output
};

// Brackets one launch with events when profiling is on.
struct EventPair {
    hipEvent_t a = nullptr, b = nullptr;
    bool on = false;
    EventPair(bool enable, hipStream_t s) : on(enable) {
        if (!on) return;
        FQZ5_HIP(hipEventCreate(&a));
        FQZ5_HIP(hipEventCreate(&b));
        FQZ5_HIP(hipEventRecord(a, s));
    }
    void stop(hipStream_t s) {
        if (on) FQZ5_HIP(hipEventRecord(b, s));
    }
    double ms() {   // after the stream has been synchronised
        if (!on) return 0;
        float t = 0;
        FQZ5_HIP(hipEventElapsedTime(&t, a, b));
        return t;
    }
    ~EventPair() {
        if (a) (void)hipEventDestroy(a);
        if (b) (void)hipEventDestroy(b);
    }
};

struct GpuCtx {
    KernelProfile prof;
    hipStream_t stream = nullptr;
    hipStream_t stream2 = nullptr;   // second queue for concurrent launches (fork() makes it)
    hipEvent_t fork_ev = nullptr, join_ev = nullptr;
    DevArena arena;
    // scratch of one codec's batch (its event tables, sort and scan
    // buffers), returned to the pool as soon as the batch's outputs exist
    // (tmp_done), so a try session holds its candidates' outputs only
    // (fqz: the unsorted events and the sort's buffers die with the sort,
    // the sorted events and their codes with the expansion into records)
    DevArena fqz_tmp, lzp_tmp, sort_tmp, ev_tmp;
    PinnedArena staging;
    int device = 0;
    int cus = 256;                   // compute units (MI355X: 256)
    int prio_ = 0;                   // the streams' priority

    // Dynamic LDS for a launch of `jobs` single-wave chain workgroups: while
    // there are no more chains than CUs, ask for more than half a CU's LDS
    // so that no two chains share a CU (measured: 20 chains of one launch
    // ran ~15 % slower per step than one alone when allowed to pack).
    // LDS of a launch of one-wave chain workgroups, padded so that no two
    // chains share a SIMD: one workgroup per CU while they fit, else at most
    // four per CU (the dispatcher gives them four different SIMDs).  Two
    // chains on one SIMD share its issue slots and each runs at half speed
    // (measured: 46 such pairs in a 393-workgroup -5 decode launch).
    uint32_t chain_lds(uint32_t lds, size_t jobs) const {
        constexpr uint32_t HALF_CU = 80 * 1024 + 16, FIFTH_CU = 32 * 1024 + 16;
        if (jobs <= size_t(cus)) return lds < HALF_CU ? HALF_CU : lds;
        if (jobs <= 4 * size_t(cus)) return lds < FIFTH_CU ? FIFTH_CU : lds;
        return lds;
    }

    // high_prio: the streams get the device's highest priority
    // ($FQZ5_AUX_HIGH_PRIO=1 for the helper contexts, gpu_aux).
    explicit GpuCtx(bool high_prio = false) {
        int n = 0;
        if (hipGetDeviceCount(&n) != hipSuccess || n <= 0)
            throw GpuError("fqz5: no HIP device visible (this library has no CPU path)");
        FQZ5_HIP(hipGetDevice(&device));
        FQZ5_HIP(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device));
        int lo = 0, hi = 0;
        FQZ5_HIP(hipDeviceGetStreamPriorityRange(&lo, &hi));
        prio_ = high_prio ? hi : lo;
        FQZ5_HIP(hipStreamCreateWithPriority(&stream, hipStreamNonBlocking, prio_));
        FQZ5_HIP(hipEventCreateWithFlags(&fork_ev, hipEventDisableTiming));
        FQZ5_HIP(hipEventCreateWithFlags(&join_ev, hipEventDisableTiming));
    }
    ~GpuCtx() {
        if (fork_ev) (void)hipEventDestroy(fork_ev);
        if (join_ev) (void)hipEventDestroy(join_ev);
        if (stream2) (void)hipStreamDestroy(stream2);
        if (stream) (void)hipStreamDestroy(stream);
    }
    // stream2 waits for everything queued on stream so far.  stream2 is
    // made here, on first use: HIP maps streams onto a fixed number of
    // hardware queues, and an idle stream2 per context would take one that
    // a working stream then has to share (its kernels queue behind the
    // other stream's: -5 NovaSeq's quality chains waited ~330 ms behind a
    // sequence model).
    void fork() {
        if (!stream2) FQZ5_HIP(hipStreamCreateWithPriority(&stream2, hipStreamNonBlocking, prio_));
        FQZ5_HIP(hipEventRecord(fork_ev, stream));
        FQZ5_HIP(hipStreamWaitEvent(stream2, fork_ev, 0));
    }
    // stream waits for everything queued on stream2 so far
    void join() {
        if (!stream2) return;
        FQZ5_HIP(hipEventRecord(join_ev, stream2));
        FQZ5_HIP(hipStreamWaitEvent(stream, join_ev, 0));
    }
    void sync() { FQZ5_HIP(hipStreamSynchronize(stream)); }

#ifdef FQZ5_COPY_STATS
    static void copy_stat(const char *kind, const char *file, int line);
#define FQZ5_CS_ARGS , const char *file_ = __builtin_FILE(), int line_ = __builtin_LINE()
#define FQZ5_CS(kind) copy_stat(kind, file_, line_)
#else
#define FQZ5_CS_ARGS
#define FQZ5_CS(kind)
#endif
    template <class T> T *upload(const T *h, size_t n FQZ5_CS_ARGS) {
        FQZ5_CS("up");
        T *d = arena.alloc_n<T>(n ? n : 1);
        if (n) {
            uint8_t *st = staging.alloc(n * sizeof(T));
            std::memcpy(st, h, n * sizeof(T));
            FQZ5_HIP(hipMemcpyAsync(d, st, n * sizeof(T), hipMemcpyHostToDevice, stream));
        }
        return d;
    }
    // A host-buffer call's input (the drop-in entry points, an idle stream):
    // copied from the caller's memory through the runtime's shared staging
    // and waited for, so the caller's buffer may die after it.  Large
    // inputs through the thread's own pinned staging instead meant pinning
    // a chunk of their size (hipHostMalloc) on each worker thread's first
    // call: 150-570 ms with the drop-in CLI's workers starting together
    // (profiles/r06_dropin_*).  Small ones keep the staging (cheap).
    template <class T> T *upload_sync(const T *h, size_t n) {
        if (n * sizeof(T) < (size_t(1) << 20)) return upload(h, n);
        T *d = arena.alloc_n<T>(n);
        FQZ5_HIP(hipMemcpyAsync(d, h, n * sizeof(T), hipMemcpyHostToDevice, stream));
        sync();
        return d;
    }
    // Rewind both arenas; only after everything queued has completed.
    void reset() {
        sync();
        if (stream2) FQZ5_HIP(hipStreamSynchronize(stream2));   // (its chunks go to the pool)
        arena.reset();
        fqz_tmp.reset();
        lzp_tmp.reset();
        sort_tmp.reset();
        ev_tmp.reset();
        staging.reset();
    }
    // a scratch arena back to the pool once the streams have drained
    void tmp_done(DevArena &a) {
        sync();
        if (stream2) FQZ5_HIP(hipStreamSynchronize(stream2));
        a.reset();
    }
    template <class T> T *upload(const std::vector<T> &v FQZ5_CS_ARGS) {
#ifdef FQZ5_COPY_STATS
        return upload(v.data(), v.size(), file_, line_);
#else
        return upload(v.data(), v.size());
#endif
    }
    template <class T> void download(T *h, const T *d, size_t n FQZ5_CS_ARGS) {
        FQZ5_CS("down");
        if (n) FQZ5_HIP(hipMemcpyAsync(h, d, n * sizeof(T), hipMemcpyDeviceToHost, stream));
    }
    void memset0(void *d, size_t n) {
        if (n) FQZ5_HIP(hipMemsetAsync(d, 0, n, stream));
    }
};

// Hedged chain launches (rANS decode, fqz range chain): on unless
// $FQZ5_NO_HEDGE is set or fqz5_set_hedge(0).
bool hedge_chains();
// the small-alphabet fqz decoder (fqz5_set_dec_small, $FQZ5_DEC_SMALL)
bool small_decoder_on();
// the block decoder's adaptive-model chains on host cores (fqz5_set_host_decode)
int host_decode_mode();
// quality blocks decoded by the general (false) / small (true) fqz decoder
uint64_t fqz_dec_blocks(bool small);
int small_copies();   // hedged copies of a small-decoder block
// Copies of each of `jobs` chains: up to 4 while they fit one per CU.
inline size_t hedge_copies(size_t jobs, size_t cus) {
    if (!hedge_chains() || !jobs) return 1;
    const size_t c = cus / jobs;
    return c < 1 ? 1 : (c > 4 ? 4 : c);
}
// Copies per chain of a launch, from the chains' costs (steps, or steps
// times the decoder's time per step): one each, then the CUs left over, one
// copy at a time, to the chain of at least half the largest cost with the
// most cost per copy (equal costs: in turn), up to HEDGE_MAX copies each.
// Those chains set the launch time (a cheaper chain finishes in time on any
// CU). The slowest CUs run a chain ~40 % slower than the fastest (DESIGN.md
// section 4), so the costly chains gain the most from more draws.  All ones
// when hedging is off.
constexpr int HEDGE_MAX = 24;   // copies of one chain at most
inline std::vector<int> hedge_plan(const std::vector<double> &cost, size_t cus) {
    std::vector<int> c(cost.size(), 1);
    static const size_t cap_waves = [] {   // experiments: $FQZ5_HEDGE_WAVES caps the launch
        const char *e = std::getenv("FQZ5_HEDGE_WAVES");
        return e ? size_t(std::strtoul(e, nullptr, 10)) : size_t(0);
    }();
    if (cap_waves && cap_waves < cus) cus = cap_waves;
    if (!hedge_chains() || cost.empty() || cost.size() >= cus) return c;
    double mx = 0;
    for (double s : cost) mx = s > mx ? s : mx;
    std::vector<size_t> longs;
    for (size_t i = 0; i < cost.size(); i++)
        if (2 * cost[i] >= mx) longs.push_back(i);
    for (size_t spare = cus - cost.size(); spare; spare--) {
        size_t best = longs.size();
        for (size_t k = 0; k < longs.size(); k++) {
            const size_t i = longs[k];
            if (c[i] >= HEDGE_MAX) continue;
            if (best == longs.size() ||
                cost[i] * c[longs[best]] > cost[longs[best]] * c[i]) best = k;
        }
        if (best == longs.size()) break;
        c[longs[best]]++;
    }
    return c;
}
inline std::vector<int> hedge_plan(const std::vector<uint64_t> &steps, size_t cus) {
    return hedge_plan(std::vector<double>(steps.begin(), steps.end()), cus);
}

// XCD-grouped layout of a hedged launch: workgroup b runs on XCD b % 8
// (observed dispatch order, MI355X_MICROARCH.md "Workgroup dispatch"), so a
// job placed at positions of one residue has all its copies on one XCD and
// the copies' reads of the same stream share that XCD's L2 instead of each
// fetching it from HBM.  Jobs (longest first) go to the XCD with the fewest
// hedged jobs, then the fewest jobs; each XCD's cus/8 slots are dealt one per
// job, then the rest round-robin to its hedged jobs up to their copies in
// `cp`.  Returns the job index per position, -1 for padding (empty when
// nothing is hedged: keep the plain order).
constexpr int XCDS = 8;
inline std::vector<int> xcd_layout(const std::vector<int> &cp, size_t cus) {
    std::vector<int> pos;
    if (cp.empty() || std::all_of(cp.begin(), cp.end(), [](int c) { return c <= 1; })) return pos;
    const size_t cap = cus / XCDS;
    if (cp.size() > cap * XCDS) return pos;
    std::vector<std::vector<int>> bk(XCDS);
    std::vector<int> nh(XCDS, 0);
    for (size_t k = 0; k < cp.size(); k++) {     // jobs arrive longest first
        int b = 0;
        for (int i = 1; i < XCDS; i++) {
            const bool hk = cp[k] > 1;
            const auto key = [&](int j) { return std::make_pair(hk ? nh[j] : 0, bk[j].size()); };
            if (key(i) < key(b)) b = i;
        }
        bk[b].push_back(int(k));
        nh[b] += cp[k] > 1;
    }
    size_t rows = 0;
    std::vector<std::vector<int>> slots(XCDS);
    for (int b = 0; b < XCDS; b++) {
        std::vector<int> got(bk[b].size(), 1);
        size_t spare = cap - bk[b].size();
        for (bool more = true; more && spare;) {
            more = false;
            for (size_t i = 0; i < bk[b].size() && spare; i++)
                if (got[i] < cp[bk[b][i]]) { got[i]++; spare--; more = true; }
        }
        for (size_t i = 0; i < bk[b].size(); i++)
            for (int c = 0; c < got[i]; c++) slots[b].push_back(bk[b][i]);
        rows = std::max(rows, slots[b].size());
    }
    pos.assign(rows * XCDS, -1);
    for (int b = 0; b < XCDS; b++)
        for (size_t r = 0; r < slots[b].size(); r++) pos[r * XCDS + b] = slots[b][r];
    return pos;
}

// Hedged launches in flight in this process (decode chains, fqz range
// chains).  Concurrent callers (the drop-in CLI's thread pool, several host
// threads) share the spare CUs: each plans its copies for cus / active.
struct HedgeShare {
    size_t cus;
    explicit HedgeShare(size_t all);
    ~HedgeShare();
};

// The calling thread's context (created on first use).
GpuCtx &gpu();
// Helper contexts of the calling thread (k < AUX_CTXS), for work run by
// helper threads concurrently with the thread's own (created on first use),
// and a rewind of every one that exists.
constexpr int AUX_CTXS = 11;  // 0 fqz, 1 LZP3, 2..7 sequence models, 8 stripes, 9 names,
                              // 10 plain rANS candidates
constexpr int AUX_SEQ0 = 2, AUX_NSEQ = 6, AUX_STRIPES = 8, AUX_NAMES = 9, AUX_PLAIN = 10;
GpuCtx &gpu_aux(int k = 0);
void gpu_aux_reset_all();
// After synchronising them, free the device arenas of the calling thread's
// context and of its helper contexts (their high-water marks otherwise stay
// held: -7 tries and commits on different contexts would add them up).
void gpu_release_all();

}  // namespace fqz5
