// lzp_codec.cpp — host side of the LZP kernels (lzp.hip): the LZP pre-pass
// of fqzcomp5's LZP3 sequence method on device-resident blocks, and the
// host-buffer entry points fqz5_lzp / fqz5_unlzp (lzp16e.c:113 lzp,
// :166 unlzp; include/fqz5_mi355x.h).
#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "../../include/fqz5_mi355x.h"
#include "lzp.h"
#include "lzp_codec.hpp"

namespace fqz5 {

GpuCtx &gpu();
void fqz5_set_error(const char *msg);

void lzp_encode_batch(GpuCtx &g, std::vector<LzpEncReq> &reqs) {
    std::vector<uint32_t *> lens(reqs.size(), nullptr);
    for (size_t r = 0; r < reqs.size(); r++) {
        LzpEncReq &R = reqs[r];
        const uint32_t n = R.n;
        if (n > (1u << 31)) throw GpuError("lzp: block too large");
        LzpEncJob J{};
        J.in = R.d_in;
        J.n = n;
        J.nchunk = (n + LZP_CHUNK - 1) / LZP_CHUNK;
        J.out = g.arena.alloc_n<uint8_t>(3 * size_t(n) + 16);
        J.out_len = g.arena.alloc_n<uint32_t>(1);
        lens[r] = J.out_len;
        R.d_out = J.out;
        if (!n) {
            g.memset0(J.out_len, 4);
            continue;
        }
        J.key = g.lzp_tmp.alloc_n<uint32_t>(n);
        J.skey = g.lzp_tmp.alloc_n<uint32_t>(n);
        J.val = g.lzp_tmp.alloc_n<uint32_t>(n);
        J.sval = g.lzp_tmp.alloc_n<uint32_t>(n);
        J.pred = g.lzp_tmp.alloc_n<uint32_t>(n);
        J.rev = g.lzp_tmp.alloc_n<uint32_t>(n);
        J.nxt = g.lzp_tmp.alloc_n<uint32_t>(n);
        J.base = g.lzp_tmp.alloc_n<uint32_t>(n);
        J.ml = g.lzp_tmp.alloc_n<uint16_t>(n);
        J.spec = g.lzp_tmp.alloc_n<uint8_t>(n);
        J.walk = g.lzp_tmp.alloc_n<uint8_t>(n);
        J.exitp = g.lzp_tmp.alloc_n<uint32_t>(J.nchunk);
        J.conv = g.lzp_tmp.alloc_n<uint32_t>(J.nchunk);
        J.size = g.lzp_tmp.alloc_n<uint32_t>(n);
        J.off = g.lzp_tmp.alloc_n<uint32_t>(n);
        g.memset0(J.spec, n);
        g.memset0(J.walk, n);
        FQZ5_HIP(hipMemsetAsync(J.conv, 0xff, size_t(J.nchunk) * 4, g.stream));
        FQZ5_HIP(launch_lzp_hash(J, g.stream));
        size_t tb = 0, t2 = 0, t3 = 0, t4 = 0, t5 = 0;
        FQZ5_HIP(lzp_sort(J, nullptr, tb, g.stream));
        FQZ5_HIP(lzp_min_scan(J, nullptr, t2, g.stream));
        FQZ5_HIP(lzp_size_scan(J, nullptr, t3, g.stream));
        FQZ5_HIP(lzp_sort_ends(J, nullptr, t4, g.stream));
        FQZ5_HIP(lzp_end_scan(J, nullptr, t5, g.stream));
        const size_t tmax = std::max({tb, t2, t3, t4, t5});
        void *tmp = g.lzp_tmp.alloc_n<uint8_t>(tmax);
        tb = t2 = t3 = t4 = t5 = tmax;
        FQZ5_HIP(lzp_sort(J, tmp, tb, g.stream));
        FQZ5_HIP(launch_lzp_pred(J, g.stream));
        FQZ5_HIP(launch_lzp_stops(J, g.stream));
        // segment-end lengths: ends sorted by (distance, position), each run
        // measured up to the next end of its distance, then linked
        FQZ5_HIP(lzp_sort_ends(J, tmp, t4, g.stream));
        FQZ5_HIP(launch_lzp_endscan(J, g.stream));
        FQZ5_HIP(lzp_end_scan(J, tmp, t5, g.stream));
        FQZ5_HIP(launch_lzp_resolve(J, g.stream));
        FQZ5_HIP(lzp_min_scan(J, tmp, t2, g.stream));
        FQZ5_HIP(launch_lzp_lengths(J, g.stream));
        FQZ5_HIP(launch_lzp_parse(J, g.stream));
        FQZ5_HIP(launch_lzp_sizes(J, g.stream));
        FQZ5_HIP(lzp_size_scan(J, tmp, t3, g.stream));
        FQZ5_HIP(launch_lzp_emit(J, g.stream));
    }
    std::vector<uint32_t> L(reqs.size(), 0);
    for (size_t r = 0; r < reqs.size(); r++) g.download(&L[r], lens[r], 1);
    g.tmp_done(g.lzp_tmp);                 // (syncs) the parse buffers back to the pool
    for (size_t r = 0; r < reqs.size(); r++) reqs[r].out_len = L[r];
}

void lzp_decode_batch(GpuCtx &g, std::vector<LzpDecReq> &reqs) {
    if (reqs.empty()) return;
    std::vector<LzpDecJob> js(reqs.size());
    uint32_t *lens = g.arena.alloc_n<uint32_t>(reqs.size());
    int32_t *st = g.arena.alloc_n<int32_t>(reqs.size());
    uint32_t *ht = g.arena.alloc_n<uint32_t>(reqs.size() << LZP_HASH_BITS);
    g.memset0(ht, (reqs.size() << LZP_HASH_BITS) * 4);
    for (size_t r = 0; r < reqs.size(); r++) {
        LzpDecJob &J = js[r];
        J.in = reqs[r].d_in;
        J.in_len = reqs[r].in_len;
        J.cap = reqs[r].cap;
        J.out = reqs[r].d_out;
        J.ht = ht + (r << LZP_HASH_BITS);
        J.out_len = lens + r;
        J.status = st + r;
    }
    const LzpDecJob *d_js = g.upload(js);
    ProfSpan sp(PK_LZP_DEC, g.stream);
    FQZ5_HIP(launch_lzp_dec(d_js, int(js.size()), g.stream));
    double b = 0;
    for (const LzpDecReq &r : reqs) b += double(r.in_len) + r.cap;
    sp.end(b);
    std::vector<uint32_t> L(reqs.size());
    std::vector<int32_t> S(reqs.size());
    g.download(L.data(), lens, L.size());
    g.download(S.data(), st, S.size());
    g.sync();
    for (size_t r = 0; r < reqs.size(); r++) {
        reqs[r].ok = S[r] == 0;
        reqs[r].out_len = L[r];
    }
}

}  // namespace fqz5

using namespace fqz5;

extern "C" {

int fqz5_lzp(unsigned char *in, int in_len, unsigned char *out) {
    GpuCtx *gp = nullptr;
    try {
        if (in_len < 0 || (!in && in_len) || !out) return -1;
        GpuCtx &g = gpu();
        gp = &g;
        std::vector<LzpEncReq> rq(1);
        rq[0].d_in = g.upload(in, size_t(in_len));
        rq[0].n = uint32_t(in_len);
        lzp_encode_batch(g, rq);
        g.download(out, rq[0].d_out, rq[0].out_len);
        g.reset();
        return int(rq[0].out_len);
    } catch (const std::exception &e) {
        fqz5_set_error(e.what());
        try { if (gp) gp->reset(); } catch (...) {}
        return -1;
    }
}

int fqz5_unlzp(unsigned char *in, int in_len, unsigned char *out, int out_cap) {
    GpuCtx *gp = nullptr;
    try {
        if (in_len < 0 || out_cap < 0 || (!in && in_len) || (!out && out_cap)) return -1;
        GpuCtx &g = gpu();
        gp = &g;
        std::vector<LzpDecReq> rq(1);
        rq[0].d_in = g.upload(in, size_t(in_len));
        rq[0].in_len = uint32_t(in_len);
        rq[0].cap = uint32_t(out_cap);
        rq[0].d_out = g.arena.alloc_n<uint8_t>(size_t(out_cap) + 4);
        lzp_decode_batch(g, rq);
        if (!rq[0].ok) {
            g.reset();
            fqz5_set_error("fqz5_unlzp: damaged stream or output past out_cap");
            return -1;
        }
        g.download(out, rq[0].d_out, rq[0].out_len);
        g.reset();
        return int(rq[0].out_len);
    } catch (const std::exception &e) {
        fqz5_set_error(e.what());
        try { if (gp) gp->reset(); } catch (...) {}
        return -1;
    }
}

}  // extern "C"
