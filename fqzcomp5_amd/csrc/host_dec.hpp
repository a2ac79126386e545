// host_dec.hpp — the adaptive-model decode chains on host cores (host_dec.cpp)
#pragma once
#include <atomic>
#include <cstddef>
#include <cstdint>
#include <functional>
#include <thread>
#include <algorithm>
#include <vector>

namespace fqz5 {
namespace host {

// uncompress_block_fqz2f (fqzcomp_qual.c:1410-1634) of `in` into out (at
// most out_cap bytes; *out_size the decoded size).  lengths: the first
// nlengths record lengths out.  seq: per record its bases (the reference's
// s->seq[rec], nrec of them; nullptr: none).  Returns 0 or -1.
int fqz_decode(const uint8_t *in, size_t in_size, uint8_t *out, size_t out_cap, size_t *out_size,
               int *lengths, int nlengths, const uint8_t *const *seq, int nrec);

// decode_seq (fqzcomp5.c:1272-1406): n bases of records lens[nrec] with a
// k-mer context model (both: both strands update).  Returns 0 or -1.
int seq_decode(const uint8_t *in, uint32_t in_size, const uint32_t *lens, int nrec, int both, int k,
               uint8_t *out, uint32_t n);

// Host threads of the library's pools (the decode chains, the name
// tokenisers, the table builders): $FQZ5_HOST_THREADS, else this rank's
// share of the cores: the process's affinity mask divided by
// $LOCAL_WORLD_SIZE, capped by $OMP_NUM_THREADS and at 16 (the CPU share of
// one GPU on the MI355X boxes).
int threads();
// the cores share above without the cap of 16
int cores_of_rank();

// Which adaptive-model decode chains of a fqz5_decode_sections call run on
// host cores and which on the GPU (host_decode_mode() 2, the default).  A
// chain is serial whichever side runs it: on a host core it costs
// n x host_ns, and a host core takes one chain at a time; on the GPU each
// chain has a wave of its own (the launch lasts as long as its longest
// chain, n x gpu_ns).  The per-symbol costs start at committed measurements
// (profiles/r04_fqz_dec_bench.txt) and follow what this
// process measures: every host chain's time, and every GPU batch's time over
// its longest chain.  plan() places the chains longest first, each where the
// call's finish time (the later of the host cores' and the GPU's) grows
// least; ties go to the host.
enum ChainKind { CK_SEQ = 0, CK_FQZ = 1, CK_FQZ_SEQ = 2, CK_N };
double chain_ns(int kind, bool gpu);
void chain_measured(int kind, bool gpu, double ns_per_symbol);
std::vector<char> plan(const std::vector<uint64_t> &n, const std::vector<int> &kind, int threads);

// fn(i) for i in [0, n) on up to threads() host threads, started by start()
// and waited for by join() (or the destructor); the work list is shared, so
// long and short jobs balance.
class Jobs {
  public:
    void start(size_t n, std::function<void(size_t)> fn) {
        fn_ = std::move(fn);
        n_ = n;
        next_ = 0;
        const size_t t = std::min<size_t>(n, size_t(threads()));
        for (size_t k = 0; k < t; k++)
            th_.emplace_back([this] {
                for (size_t i; (i = next_.fetch_add(1)) < n_;) fn_(i);
            });
    }
    void join() {
        for (auto &t : th_) t.join();
        th_.clear();
    }
    ~Jobs() { join(); }

  private:
    std::function<void(size_t)> fn_;
    size_t n_ = 0;
    std::atomic<size_t> next_{0};
    std::vector<std::thread> th_;
};

}  // namespace host
}  // namespace fqz5
