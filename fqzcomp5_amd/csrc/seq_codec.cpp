// seq_codec.cpp — fqzcomp5's sequence context model (SEQ10 .. SEQ14B) on the
// GPU, behind fqz5_seq_encode / fqz5_seq_decode: the drop-ins of fqzcomp5.c's
// encode_seq (:1073-1270) and decode_seq (:1272-1406), same arguments, same
// bytes, same NULL cases (include/fqz5_mi355x.h).
#include <cstdlib>
#include <cstring>
#include <vector>

#include "../../include/fqz5_mi355x.h"
#include "fqz_codec.hpp"
#include "fqz_kernels.h"
#include "seq_cm.h"
#include "seq_codec.hpp"

namespace fqz5 {

GpuCtx &gpu();
void fqz5_set_error(const char *msg);

namespace {

// Record segments (fqzcomp5.c:1127-1128, :1210-1219): the contexts restart
// at every record start.  The reference counts a record down in an int, so a
// record of length 0 (or >= 2^31) is never seen to end: no later boundary.
// false: a boundary is due but the records are used up (the reference
// returns NULL there).
bool seq_segments(const uint32_t *len, int nrec, uint32_t n, std::vector<uint32_t> &seg) {
    seg.assign(1, 0u);
    if (n && nrec > 0) {
        uint64_t pos = 0;
        int64_t left = int32_t(len[0]);
        int next = 1;
        while (left > 0) {
            const uint64_t b = pos + uint64_t(left);
            if (b >= n) break;
            if (next >= nrec) return false;
            seg.push_back(uint32_t(b));
            pos = b;
            left = int32_t(len[next++]);
        }
    }
    seg.push_back(n);
    return true;
}

bool seq_class_uc(uint8_t c) { return c == 'A' || c == 'C' || c == 'G' || c == 'T'; }

}  // namespace

// One block: events, context and side models, then the range coder back end.
// Returns the device output and its size.
static uint8_t *seq_encode_dev(GpuCtx &g, const uint8_t *d_in, uint32_t n,
                               const std::vector<uint32_t> &seg, int both, int k,
                               uint32_t *out_len) {
    SeqJob J{};
    J.in = d_in;
    J.n = n;
    J.k = uint32_t(k);
    J.both = both ? 1u : 0u;
    J.mask = uint32_t((1ull << (2 * k)) - 1);
    J.nseg = uint32_t(seg.size() - 1);
    J.seg = g.upload(seg);
    uint32_t nev = 0;
    if (n) {
        J.flag = g.arena.alloc_n<uint32_t>(n);
        J.ex = g.arena.alloc_n<uint32_t>(n);
        FQZ5_HIP(launch_seq_heads(J, g.stream));
        size_t tb = 0;
        FQZ5_HIP(fqz_exclusive_scan(J.flag, J.ex, int(n), nullptr, tb, g.stream));
        void *tmp = g.arena.alloc_n<uint8_t>(tb);
        FQZ5_HIP(fqz_exclusive_scan(J.flag, J.ex, int(n), tmp, tb, g.stream));
        uint32_t last[2];
        uint8_t first = 0;
        g.download(&last[0], J.ex + n - 1, 1);
        g.download(&last[1], J.flag + n - 1, 1);
        g.download(&first, d_in, 1);
        g.sync();
        J.nrun = last[0] + last[1];
        J.lead = seq_class_uc(first) ? 0u : 2u;
        J.run_start = g.arena.alloc_n<uint32_t>(J.nrun);
        J.cnt = g.arena.alloc_n<uint32_t>(J.nrun + 1);
        J.run_off = g.arena.alloc_n<uint32_t>(J.nrun + 1);
        FQZ5_HIP(launch_seq_runs(J, g.stream));
        tb = 0;
        FQZ5_HIP(fqz_exclusive_scan(J.cnt, J.run_off, int(J.nrun + 1), nullptr, tb, g.stream));
        tmp = g.arena.alloc_n<uint8_t>(tb);
        FQZ5_HIP(fqz_exclusive_scan(J.cnt, J.run_off, int(J.nrun + 1), tmp, tb, g.stream));
        uint32_t tot = 0;
        g.download(&tot, J.run_off + J.nrun, 1);
        g.sync();
        // symbols + lead pair + (digits + switch) per run - the last switch
        const uint64_t ne = uint64_t(n) + J.lead + tot - 1ull;
        if (ne >= (1ull << 31)) throw GpuError("fqz5_seq_encode: block too large");
        nev = uint32_t(ne);

        J.nkeys = n * (J.both + 1u);
        J.key = g.arena.alloc_n<uint32_t>(J.nkeys);
        J.val = g.arena.alloc_n<uint64_t>(J.nkeys);
        FQZ5_HIP(launch_seq_ctx(J, g.stream));
        uint32_t *skey = g.arena.alloc_n<uint32_t>(J.nkeys);
        uint64_t *sval = g.arena.alloc_n<uint64_t>(J.nkeys);
        tb = 0;
        const int kb = 2 * k + 1;
        FQZ5_HIP(fqz_sort_by_model(J.key, skey, J.val, sval, int(J.nkeys), kb, nullptr, tb, g.stream));
        tmp = g.arena.alloc_n<uint8_t>(tb);
        FQZ5_HIP(fqz_sort_by_model(J.key, skey, J.val, sval, int(J.nkeys), kb, tmp, tb, g.stream));
        J.skey = skey;
        J.sval = sval;
    }
    J.rec = g.arena.alloc_n<uint4>(nev ? nev : 1);
    FQZ5_HIP(launch_seq_model(J, g.stream));
    FQZ5_HIP(launch_seq_side(J, g.stream));

    FqzEvJob E{};
    E.nev = nev;
    E.rec = J.rec;
    // each event shifts the coder at most twice (range >= 2^24 / 65519 >= 256 after it)
    uint8_t *out = g.arena.alloc_n<uint8_t>(2 * size_t(nev) + 16);
    E.out = out;
    E.out_len = g.arena.alloc_n<uint32_t>(1);
    std::vector<FqzEvJob *> js{&E};
    rc_backend(g, js);
    g.download(out_len, E.out_len, 1);
    g.sync();
    return out;
}

void seq_encode_batch(GpuCtx &g, std::vector<SeqEncReq> &reqs) {
    for (SeqEncReq &R : reqs) {
        R.ok = false;
        R.out.clear();
        if (R.k < 1 || R.k > int(SEQ_K_MAX)) throw GpuError("seq: context size out of range (1..14)");
        std::vector<uint32_t> seg;
        if (!R.lens || !seq_segments(R.lens, R.nrec, R.n, seg)) continue;
        uint32_t len = 0;
        Piece p;
        p.dev = seq_encode_dev(g, R.d_in, R.n, seg, R.both, R.k, &len);
        p.len = len;
        R.out.push_back(p);
        R.ok = true;
    }
}

void seq_decode_batch(GpuCtx &g, std::vector<SeqDecReq> &reqs) {
    std::vector<SeqDecJob> js;
    std::vector<size_t> who;
    for (size_t i = 0; i < reqs.size(); i++) {
        SeqDecReq &R = reqs[i];
        R.ok = false;
        if (R.k < 1 || R.k > int(SEQ_K_MAX)) continue;
        std::vector<uint32_t> seg;
        if (!R.lens || !seq_segments(R.lens, R.nrec, R.n, seg)) continue;
        SeqDecJob J{};
        J.in = R.d_in;
        J.in_len = R.in_size;
        J.n = R.n;
        J.k = uint32_t(R.k);
        J.both = R.both ? 1u : 0u;
        J.mask = uint32_t((1ull << (2 * R.k)) - 1);
        J.nseg = uint32_t(seg.size() - 1);
        J.seg = g.upload(seg);
        const size_t nctx = size_t(J.mask) + 1;
        J.models = g.arena.alloc_n<uint32_t>(nctx);
        FQZ5_HIP(launch_seq_models_init(J.models, nctx, g.stream));
        J.out = R.d_out;
        J.status = g.arena.alloc_n<int32_t>(1);
        js.push_back(J);
        who.push_back(i);
    }
    if (js.empty()) return;
    FQZ5_HIP(launch_seq_dec(g.upload(js), int(js.size()), g.stream));
    std::vector<int32_t> st(js.size(), -1);
    for (size_t k = 0; k < js.size(); k++) g.download(&st[k], js[k].status, 1);
    g.sync();
    for (size_t k = 0; k < js.size(); k++) reqs[who[k]].ok = st[k] == 0;
}

}  // namespace fqz5

using namespace fqz5;

extern "C" {

char *fqz5_seq_encode(unsigned char *in, unsigned int in_size, unsigned int *len, int nrecords,
                      int both_strands, int ctx_size, unsigned int *out_size) {
    GpuCtx *gp = nullptr;
    try {
        if (!out_size || (!in && in_size) || !len || nrecords < 1) return nullptr;
        if (ctx_size < 1 || ctx_size > int(SEQ_K_MAX))
            throw GpuError("fqz5_seq_encode: context size out of range (1..14)");
        if (in_size > (1u << 30)) throw GpuError("fqz5_seq_encode: block too large");
        std::vector<uint32_t> seg;
        if (!seq_segments(len, nrecords, in_size, seg)) return nullptr;
        GpuCtx &g = gpu();
        gp = &g;
        const uint8_t *d_in = g.upload(in, in_size);
        uint32_t n_out = 0;
        uint8_t *d_out = seq_encode_dev(g, d_in, in_size, seg, both_strands, ctx_size, &n_out);
        char *out = static_cast<char *>(std::malloc(n_out ? n_out : 1));
        if (!out) throw GpuError("fqz5_seq_encode: out of host memory");
        g.download(reinterpret_cast<uint8_t *>(out), d_out, n_out);
        g.reset();
        *out_size = n_out;
        return out;
    } catch (const std::exception &e) {
        fqz5_set_error(e.what());
        try { if (gp) gp->reset(); } catch (...) {}
        return nullptr;
    }
}

char *fqz5_seq_decode(unsigned char *in, unsigned int in_size, unsigned int *len, int nrecords,
                      int both_strands, int ctx_size, unsigned int out_size) {
    GpuCtx *gp = nullptr;
    try {
        if ((!in && in_size) || !len || nrecords < 1) return nullptr;
        if (ctx_size < 1 || ctx_size > int(SEQ_K_MAX))
            throw GpuError("fqz5_seq_decode: context size out of range (1..14)");
        std::vector<uint32_t> seg;
        if (!seq_segments(len, nrecords, out_size, seg)) return nullptr;
        GpuCtx &g = gpu();
        gp = &g;
        std::vector<SeqDecReq> rq(1);
        rq[0].d_in = g.upload(in, in_size);
        rq[0].in_size = in_size;
        rq[0].lens = len;
        rq[0].nrec = nrecords;
        rq[0].both = both_strands;
        rq[0].k = ctx_size;
        rq[0].n = out_size;
        rq[0].d_out = g.arena.alloc_n<uint8_t>(out_size ? out_size : 1);
        seq_decode_batch(g, rq);
        char *out = static_cast<char *>(std::malloc(out_size ? out_size : 1));
        if (!out) throw GpuError("fqz5_seq_decode: out of host memory");
        g.download(reinterpret_cast<uint8_t *>(out), rq[0].d_out, out_size);
        g.reset();
        const int32_t st = rq[0].ok ? 0 : -1;
        if (st != 0) {
            std::free(out);
            fqz5_set_error("fqz5_seq_decode: damaged stream");
            return nullptr;
        }
        return out;
    } catch (const std::exception &e) {
        fqz5_set_error(e.what());
        try { if (gp) gp->reset(); } catch (...) {}
        return nullptr;
    }
}

}  // extern "C"
