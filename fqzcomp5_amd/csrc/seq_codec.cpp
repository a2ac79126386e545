// seq_codec.cpp — fqzcomp5's sequence context model (SEQ10 .. SEQ14B) on the
// GPU, behind fqz5_seq_encode / fqz5_seq_decode: the drop-ins of fqzcomp5.c's
// encode_seq (:1073-1270) and decode_seq (:1272-1406), same arguments, same
// bytes, same NULL cases (include/fqz5_mi355x.h).
#include <algorithm>
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

struct SeqWork {
    SeqJob J{};
    FqzEvJob E{};
    uint32_t nev = 0;
    uint64_t lb = 0;                    // output bytes >= lb
    uint64_t ub = 0;                    // output bytes <= ub
    uint32_t clen = 0;
    bool ready = false;                 // events built (records did not run out)
};

// One block: events, context and side models; the coder records J.rec in
// stream order and the entropy partial sums into `part` (EB doubles).
static void seq_prepare_dev(GpuCtx &g, SeqWork &W, const uint8_t *d_in, uint32_t n,
                            const std::vector<uint32_t> &seg, int both, int k, double *part,
                            uint32_t EB) {
    SeqJob &J = W.J;
    J.in = d_in;
    J.n = n;
    J.k = uint32_t(k);
    J.both = both ? 1u : 0u;
    J.mask = uint32_t((1ull << (2 * k)) - 1);
    J.nseg = uint32_t(seg.size() - 1);
    J.seg = g.upload(seg);
    uint32_t nev = 0;
    if (n) {
        J.flag = g.ev_tmp.alloc_n<uint32_t>(n);
        J.ex = g.ev_tmp.alloc_n<uint32_t>(n);
        FQZ5_HIP(launch_seq_heads(J, g.stream));
        size_t tb = 0;
        FQZ5_HIP(fqz_exclusive_scan(J.flag, J.ex, int(n), nullptr, tb, g.stream));
        void *tmp = g.ev_tmp.alloc_n<uint8_t>(tb);
        FQZ5_HIP(fqz_exclusive_scan(J.flag, J.ex, int(n), tmp, tb, g.stream));
        uint32_t last[2];
        uint8_t first = 0;
        g.download(&last[0], J.ex + n - 1, 1);
        g.download(&last[1], J.flag + n - 1, 1);
        g.download(&first, d_in, 1);
        g.sync();
        J.nrun = last[0] + last[1];
        J.lead = seq_class_uc(first) ? 0u : 2u;
        J.run_start = g.ev_tmp.alloc_n<uint32_t>(J.nrun);
        J.cnt = g.ev_tmp.alloc_n<uint32_t>(J.nrun + 1);
        J.run_off = g.ev_tmp.alloc_n<uint32_t>(J.nrun + 1);
        FQZ5_HIP(launch_seq_runs(J, g.stream));
        tb = 0;
        FQZ5_HIP(fqz_exclusive_scan(J.cnt, J.run_off, int(J.nrun + 1), nullptr, tb, g.stream));
        tmp = g.ev_tmp.alloc_n<uint8_t>(tb);
        FQZ5_HIP(fqz_exclusive_scan(J.cnt, J.run_off, int(J.nrun + 1), tmp, tb, g.stream));
        uint32_t tot = 0;
        g.download(&tot, J.run_off + J.nrun, 1);
        g.sync();
        // symbols + lead pair + (digits + switch) per run - the last switch
        const uint64_t ne = uint64_t(n) + J.lead + tot - 1ull;
        if (ne >= (1ull << 31)) throw GpuError("fqz5_seq_encode: block too large");
        nev = uint32_t(ne);

        J.nkeys = n * (J.both + 1u);
        J.key = g.ev_tmp.alloc_n<uint32_t>(J.nkeys);
        J.val = g.ev_tmp.alloc_n<uint64_t>(J.nkeys);
        FQZ5_HIP(launch_seq_ctx(J, g.stream));
        uint32_t *skey = g.ev_tmp.alloc_n<uint32_t>(J.nkeys);
        uint64_t *sval = g.ev_tmp.alloc_n<uint64_t>(J.nkeys);
        tb = 0;
        const int kb = 2 * k + 1;
        FQZ5_HIP(fqz_sort_by_model(J.key, skey, J.val, sval, int(J.nkeys), kb, nullptr, tb, g.stream));
        tmp = g.ev_tmp.alloc_n<uint8_t>(tb);
        FQZ5_HIP(fqz_sort_by_model(J.key, skey, J.val, sval, int(J.nkeys), kb, tmp, tb, g.stream));
        J.skey = skey;
        J.sval = sval;
    }
    J.rec = g.fqz_tmp.alloc_n<uint4>(nev + RC_PAD);
    {
        ProfSpan sp(PK_SEQ_MODEL, g.stream);
        FQZ5_HIP(launch_seq_model(J, g.stream));
        sp.end(double(n));
    }
    FQZ5_HIP(launch_seq_side(J, g.stream));
    FQZ5_HIP(launch_rec_entropy(J.rec, nev, part, EB, g.stream));
    W.nev = nev;
    // the heads, runs and sorted contexts back to the pool (the records are
    // what the coder needs): one block's, not every block's, at the peak
    g.tmp_done(g.ev_tmp);
}

void seq_encode_prepare(GpuCtx &g, std::vector<SeqEncReq> &reqs) {
    constexpr uint32_t EB = 256;   // per request: EB entropy partials, then EB slack partials
    double *part = g.arena.alloc_n<double>(2 * size_t(EB) * std::max<size_t>(reqs.size(), 1));
    g.memset0(part, 2 * size_t(EB) * std::max<size_t>(reqs.size(), 1) * sizeof(double));
    for (size_t i = 0; i < reqs.size(); i++) {
        SeqEncReq &R = reqs[i];
        R.ok = false;
        R.out.clear();
        R.w = std::make_shared<SeqWork>();
        if (R.k < 1 || R.k > int(SEQ_K_MAX)) throw GpuError("seq: context size out of range (1..14)");
        std::vector<uint32_t> seg;
        if (!R.lens || !seq_segments(R.lens, R.nrec, R.n, seg)) continue;
        seq_prepare_dev(g, *R.w, R.d_in, R.n, seg, R.both, R.k, part + 2 * i * EB, EB);
        R.w->ready = true;
    }
    std::vector<double> hp(2 * size_t(EB) * reqs.size());
    g.download(hp.data(), part, hp.size());
    g.sync();
    for (size_t i = 0; i < reqs.size(); i++) {
        SeqWork &W = *reqs[i].w;
        if (!W.ready) continue;
        double bits = 0, slack = 0;
        for (uint32_t b = 0; b < EB; b++) {
            bits += hp[2 * i * EB + b];
            slack += hp[(2 * i + 1) * EB + b];
        }
        // the coder's P bytes and its 5 flush bytes
        W.lb = rc_bytes_lower(bits);
        W.ub = rc_bytes_upper(bits, slack) + 5;
    }
}

void seq_encode_finish(GpuCtx &g, std::vector<SeqEncReq> &reqs, const std::vector<char> *skip) {
    std::vector<FqzEvJob *> js;
    std::vector<SeqEncReq *> run;
    for (size_t i = 0; i < reqs.size(); i++) {
        SeqEncReq &R = reqs[i];
        if (!R.w || !R.w->ready || (skip && (*skip)[i])) continue;
        SeqWork &W = *R.w;
        W.E = FqzEvJob{};
        W.E.nev = W.nev;
        W.E.rec = W.J.rec;
        // each event shifts the coder at most twice (range >= 2^24 / 65519 >= 256 after it)
        W.E.out = g.arena.alloc_n<uint8_t>(2 * size_t(W.nev) + 16);
        W.E.out_len = g.arena.alloc_n<uint32_t>(1);
        js.push_back(&W.E);
        run.push_back(&R);
    }
    rc_backend(g, js);
    for (SeqEncReq *R : run) g.download(&R->w->clen, R->w->E.out_len, 1);
    // (the event records of blocks prepared on this context and the coder's
    // buffers back to the pool; outputs stay)
    g.tmp_done(g.fqz_tmp);
    for (SeqEncReq *R : run) {
        SeqWork &W = *R->w;
        if (W.lb > W.clen)   // the entropy bound is a theorem
            throw GpuError("seq: size below its entropy bound");
        if (W.ub < W.clen)   // and so is the slack bound
            throw GpuError("seq: size above its upper bound");
        Piece p;
        p.dev = W.E.out;
        p.len = W.clen;
        R->out.push_back(p);
        R->ok = true;
    }
}

uint64_t seq_size_lower_bound(const SeqEncReq &r) { return r.w && r.w->ready ? r.w->lb : 0; }
uint64_t seq_size_upper_bound(const SeqEncReq &r) { return r.w && r.w->ready ? r.w->ub : 0; }

void seq_encode_batch(GpuCtx &g, std::vector<SeqEncReq> &reqs) {
    seq_encode_prepare(g, reqs);
    seq_encode_finish(g, reqs, nullptr);
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
    EventPair ev(prof_on(), g.stream);
    // k >= 3: the lookahead decoder; the rest (k = 1, 2) the one-step one
    std::vector<SeqDecJob> la, one;
    for (const SeqDecJob &J : js) (J.k >= 3 ? la : one).push_back(J);
    if (!la.empty()) FQZ5_HIP(launch_seq_dec(g.upload(la), int(la.size()), g.stream, true));
    if (!one.empty()) FQZ5_HIP(launch_seq_dec(g.upload(one), int(one.size()), g.stream, false));
    ev.stop(g.stream);
    std::vector<int32_t> st(js.size(), -1);
    for (size_t k = 0; k < js.size(); k++) g.download(&st[k], js[k].status, 1);
    g.sync();
    if (ev.on) {   // compressed bytes in, bases out
        double b = 0;
        for (const SeqDecJob &J : js) b += double(J.in_len) + double(J.n);
        prof_add(PK_SEQ_DEC, ev.ms(), b);
    }
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
        std::vector<SeqEncReq> rq(1);
        rq[0].d_in = g.upload(in, in_size);
        rq[0].n = in_size;
        rq[0].lens = len;
        rq[0].nrec = nrecords;
        rq[0].both = both_strands;
        rq[0].k = ctx_size;
        seq_encode_batch(g, rq);
        if (!rq[0].ok) { g.reset(); return nullptr; }
        const uint32_t n_out = rq[0].out[0].len;
        const uint8_t *d_out = rq[0].out[0].dev;
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
