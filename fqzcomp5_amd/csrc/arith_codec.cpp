// arith_codec.cpp — arith_compress_to / arith_uncompress_to (htscodecs
// arith_dynamic.c:730-1277) on the GPU.  The control flow is the
// reference's, step for step (its buffer arithmetic included: the CAT
// block falls through, the packed-size varint is subtracted from the
// capacity twice, stripe candidates are written at offset 7 + 5N); the
// bytes are produced by kernels: histograms for the maximum symbol and the
// pack map, pack / unpack, stripe transposes, and the entropy coders
// (arith_kernels.hip).  Headers are assembled on the host.
#include <climits>
#include <cstring>
#include <vector>

#include "arith_kernels.h"
#include "gpu_ctx.hpp"
#include "kernels.h"
#include "rans_format.hpp"

namespace fqz5 {
namespace {

constexpr int AX_PACK = 0x80, AX_RLE = 0x40, AX_CAT = 0x20, AX_NOSZ = 0x10, AX_STRIPE = 0x08,
              AX_EXT = 0x04;

// byte histogram of a device buffer
void hist(GpuCtx &g, const uint8_t *d, uint32_t n, uint32_t cnt[256]) {
    std::memset(cnt, 0, 256 * sizeof(uint32_t));
    if (!n) return;
    uint32_t *dc = g.arena.alloc_n<uint32_t>(512);
    g.memset0(dc, 512 * 4);
    std::vector<HistItem> items;
    for (uint32_t b = 0; b < n; b += 1u << 20)
        items.push_back(HistItem{d, b, std::min(n, b + (1u << 20)), 0, 0});
    FQZ5_HIP(launch_hist0(g.upload(items), int(items.size()), dc, g.stream));
    g.download(cnt, dc, 256);
    g.sync();
}

// the four entropy coders: out = [m][coder bytes]
bool ent_compress(GpuCtx &g, const uint8_t *d_in, uint32_t n, uint8_t *out, uint32_t *out_size,
                  bool o1, bool rle) {
    const int bound = int(arith_compress_bound_ref(n, 0)) - 5;
    if (bound > int(*out_size)) return false;
    uint32_t cnt[256];
    hist(g, d_in, n, cnt);
    uint32_t m = 0;
    for (uint32_t s = 0; s < 256; s++)
        if (cnt[s]) m = s;
    m++;
    out[0] = uint8_t(m);
    ArithJob J{};
    J.in = d_in;
    J.n = n;
    J.cap = *out_size - 1;
    J.m = m;
    J.o1 = o1;
    J.rle = rle;
    J.out = g.arena.alloc_n<uint8_t>(J.cap + 1);
    J.out_len = g.arena.alloc_n<uint32_t>(1);
    J.status = g.arena.alloc_n<int32_t>(1);
    const bool in_lds = arith_models_in_lds(m, o1, rle);
    const uint32_t mb = arith_model_bytes(m, o1, rle);
    if (!in_lds) J.models = g.arena.alloc_n<uint8_t>(mb);
    FQZ5_HIP(launch_arith(g.upload(&J, 1), 1, false, !in_lds, mb, g.stream));
    int32_t st = 0;
    uint32_t len = 0;
    g.download(&st, J.status, 1);
    g.download(&len, J.out_len, 1);
    g.sync();
    if (st) return false;
    g.download(out + 1, J.out, len);
    g.sync();
    *out_size = len + 1;
    return true;
}

bool ent_uncompress(GpuCtx &g, const uint8_t *h_in, uint32_t in_size, uint8_t *d_out, uint32_t n,
                    bool o1, bool rle) {
    ArithJob J{};
    J.m = h_in[0] ? h_in[0] : 256u;
    J.in = g.upload(h_in + 1, in_size - 1);
    J.in_len = in_size - 1;
    J.n = n;
    J.o1 = o1;
    J.rle = rle;
    J.out = d_out;
    J.out_len = g.arena.alloc_n<uint32_t>(1);
    J.status = g.arena.alloc_n<int32_t>(1);
    const bool in_lds = arith_models_in_lds(J.m, o1, rle);
    const uint32_t mb = arith_model_bytes(J.m, o1, rle);
    if (!in_lds) J.models = g.arena.alloc_n<uint8_t>(mb);
    FQZ5_HIP(launch_arith(g.upload(&J, 1), 1, true, !in_lds, mb, g.stream));
    int32_t st = 0;
    g.download(&st, J.status, 1);
    g.sync();
    return st == 0;
}

void stripe(GpuCtx &g, const uint8_t *in, uint8_t *out, uint32_t n, uint32_t N, int dir) {
    if (!n) return;
    StripeItem it{in, out, n, N, dir, 0};
    FQZ5_HIP(launch_stripe(g.upload(&it, 1), 1, n, g.stream));
}

// arith_compress_to on a device input, into a host buffer of *out_size
bool compress_to(GpuCtx &g, const uint8_t *d_in, uint32_t in_size, uint8_t *out,
                 uint32_t *out_size, int order) {
    if (in_size > INT_MAX || *out_size == 0) return false;
    uint8_t *out_end = out + *out_size;
    uint32_t c_meta_len;
    if (in_size <= 20) order &= ~AX_STRIPE;
    if (order & AX_CAT) {                         // (:743-752, falls through)
        out[0] = AX_CAT;
        c_meta_len = 1 + uint32_t(varint_put(&out[1], out_end, in_size));
        if (c_meta_len + in_size > *out_size) return false;
        g.download(out + c_meta_len, d_in, in_size);
        g.sync();
        *out_size = in_size + c_meta_len;
    }
    if (order & AX_STRIPE) {                      // (:754-869)
        uint32_t N = uint32_t((order >> 8) & 0xff);
        if (N == 0) N = 4;
        if (N > in_size) N = in_size;
        uint32_t part[256], idx[256];
        for (uint32_t i = 0; i < N; i++) {
            part[i] = in_size / N + ((in_size % N) > i);
            idx[i] = i ? idx[i - 1] + part[i - 1] : 0;
        }
        uint8_t *tr = g.arena.alloc_n<uint8_t>(in_size);
        stripe(g, d_in, tr, in_size, N, 0);
        c_meta_len = 1;
        out[0] = uint8_t(order & ~AX_NOSZ);
        c_meta_len += uint32_t(varint_put(out + c_meta_len, out_end, in_size));
        if (c_meta_len >= *out_size) return false;
        out[c_meta_len++] = uint8_t(N);
        uint8_t *out2 = out + 7 + 5 * N, *out2_start = out2;
        static const int M[4][4] = {{3, 1, 64, 0}, {2, 1, 0}, {2, 1, 128}, {2, 1, 128}};
        for (uint32_t s = 0; s < N; s++) {
            const int *m = M[s < 3 ? s : 3];
            int j, best_j = 0;
            uint32_t best_sz = INT_MAX, olen2 = 0;
            for (j = 1; j <= m[0]; j++) {
                if (out2 - out > long(*out_size)) continue;
                olen2 = *out_size - uint32_t(out2 - out);
                if ((order & 3) == 0 && (m[j] & 1)) continue;
                const bool r = compress_to(g, tr + idx[s], part[s], out2, &olen2, m[j] | AX_NOSZ);
                if (r && olen2 && best_sz > olen2) {
                    best_sz = olen2;
                    best_j = j;
                }
            }
            if (best_sz == uint32_t(INT_MAX)) return false;
            if (best_j != j - 1) {
                olen2 = *out_size - uint32_t(out2 - out);
                if (!compress_to(g, tr + idx[s], part[s], out2, &olen2, m[best_j] | AX_NOSZ))
                    return false;
            }
            out2 += olen2;
            c_meta_len += uint32_t(varint_put(out + c_meta_len, out_end, olen2));
        }
        std::memmove(out + c_meta_len, out2_start, size_t(out2 - out2_start));
        *out_size = c_meta_len + uint32_t(out2 - out2_start);
        return true;
    }
    int do_pack = order & AX_PACK, do_rle = order & AX_RLE;
    const int no_size = order & AX_NOSZ, do_ext = order & AX_EXT;
    out[0] = uint8_t(order);
    c_meta_len = 1;
    if (!no_size) c_meta_len += uint32_t(varint_put(&out[1], out_end, in_size));
    order &= 3;
    const uint8_t *d = d_in;
    if (do_pack && in_size) {                     // hts_pack (pack.c:56-147)
        if (c_meta_len + 256 > *out_size) return false;
        uint32_t cnt[256];
        hist(g, d_in, in_size, cnt);
        uint8_t code[256] = {0};
        int ns = 0;
        uint8_t *meta = out + c_meta_len;
        for (int s = 0; s < 256; s++)
            if (cnt[s]) {
                code[s] = uint8_t(ns++);
                meta[ns] = uint8_t(s);
            }
        meta[0] = uint8_t(ns);
        if (ns > 16) {
            out[0] &= uint8_t(~AX_PACK);
            do_pack = 0;
        } else {
            const int per = ns > 4 ? 2 : ns > 2 ? 4 : ns > 1 ? 8 : 0;
            const uint32_t plen = per ? (in_size + uint32_t(per) - 1) / uint32_t(per) : 0;
            uint8_t *packed = g.arena.alloc_n<uint8_t>(std::max<uint32_t>(plen, 1));
            if (plen) {
                PackItem it{d_in, packed, g.upload(code, 256), in_size, per};
                FQZ5_HIP(launch_pack(g.upload(&it, 1), 1, plen, false, g.stream));
            }
            d = packed;
            in_size = plen;
            c_meta_len += uint32_t(ns + 1);
            const int sz = varint_put(out + c_meta_len, out_end, in_size);
            c_meta_len += uint32_t(sz);
            *out_size -= uint32_t(sz);
        }
    } else if (do_pack) {
        out[0] &= uint8_t(~AX_PACK);
    }
    if (do_rle && !in_size) out[0] &= uint8_t(~AX_RLE);
    *out_size -= c_meta_len;
    if (order && in_size < 8) {
        out[0] &= uint8_t(~3);
        order &= ~3;
    }
    if (do_ext) return false;                     // no libbz2 in the reference build
    if (!ent_compress(g, d, in_size, out + c_meta_len, out_size, order == 1, do_rle != 0))
        return false;
    if (*out_size >= in_size) {                   // (:980-993)
        out[0] &= uint8_t(~(3 | AX_EXT));
        out[0] |= uint8_t(AX_CAT | no_size);
        if (out + c_meta_len + in_size > out_end) return false;
        g.download(out + c_meta_len, d, in_size);
        g.sync();
        *out_size = in_size;
    }
    *out_size += c_meta_len;
    return true;
}

// arith_uncompress_to of host bytes into device memory.  has_out: the
// caller gave an output buffer of *out_size (d_out); otherwise one is made
// (returned through d_out).
bool uncompress_to(GpuCtx &g, const uint8_t *in, uint32_t in_size, uint8_t *&d_out,
                   uint32_t *out_size, bool has_out) {
    const uint8_t *in_end = in + in_size;
    if (in_size == 0) return false;
    if (*in & AX_STRIPE) {                        // (:1040-1122)
        uint32_t ulen = 0, c_meta_len = 1;
        uint64_t clen_tot = 0;
        c_meta_len += uint32_t(varint_get(in + c_meta_len, in_end, &ulen));
        if (c_meta_len >= in_size) return false;
        const uint32_t N = in[c_meta_len++];
        if (N < 1) return false;
        uint32_t clenN[256], ulenN[256], idxN[256];
        if (!has_out) {
            if (ulen >= uint32_t(INT_MAX)) return false;
            d_out = g.arena.alloc_n<uint8_t>(std::max<uint32_t>(ulen, 1));
            *out_size = ulen;
            has_out = true;
        }
        if (ulen != *out_size) return false;
        for (uint32_t i = 0; i < N; i++) {
            ulenN[i] = ulen / N + ((ulen % N) > i);
            idxN[i] = i ? idxN[i - 1] + ulenN[i - 1] : 0;
            c_meta_len += uint32_t(varint_get(in + c_meta_len, in_end, &clenN[i]));
            clen_tot += clenN[i];
            if (c_meta_len > in_size || clenN[i] > in_size || clenN[i] < 1) return false;
        }
        if (c_meta_len + clen_tot > in_size) return false;
        in_size = c_meta_len + uint32_t(clen_tot);
        uint8_t *outN = g.arena.alloc_n<uint8_t>(std::max<uint32_t>(ulen, 1));
        for (uint32_t i = 0; i < N; i++) {
            uint32_t olen = ulenN[i];
            uint8_t *dst = outN + idxN[i];
            if (in_size < c_meta_len ||
                !uncompress_to(g, in + c_meta_len, in_size - c_meta_len, dst, &olen, true) ||
                olen != ulenN[i])
                return false;
            c_meta_len += clenN[i];
        }
        stripe(g, outN, d_out, ulen, N, 1);       // unstripe (utils.h:79-138)
        *out_size = ulen;
        return true;
    }
    int order = *in++;
    in_size--;
    const int do_pack = order & AX_PACK, do_rle = order & AX_RLE, do_cat = order & AX_CAT;
    const int no_size = order & AX_NOSZ, do_ext = order & AX_EXT;
    order &= 3;
    int sz = 0;
    uint32_t osz = 0;
    if (!no_size)
        sz = varint_get(in, in_end, &osz);
    else
        osz = *out_size;
    in += sz;
    in_size -= uint32_t(sz);
    if (osz >= uint32_t(INT_MAX)) return false;
    if (no_size && !has_out) return false;
    if (!has_out) {
        *out_size = osz;
        d_out = g.arena.alloc_n<uint8_t>(std::max<uint32_t>(osz, 1));
    } else {
        if (*out_size < osz) return false;
        *out_size = osz;
    }
    uint32_t tmp1_size = *out_size;
    uint8_t *tmp1 = d_out;
    uint8_t map[256] = {0};
    int per = 0;
    uint64_t unpacked_sz = 0;
    if (do_pack) {                                // hts_unpack_meta (pack.c:161-199)
        tmp1 = g.arena.alloc_n<uint8_t>(std::max<uint32_t>(*out_size, 1));
        if (in_size == 0) return false;
        uint32_t ns = in[0] ? in[0] : 256u;
        uint32_t c_meta = 1;
        per = ns <= 1 ? 0 : ns <= 2 ? 8 : ns <= 4 ? 4 : ns <= 16 ? 2 : 1;
        if (per != 1) {
            if (in_size <= 1 || in_size < 1 + ns) return false;
            std::memcpy(map, in + 1, ns);
            c_meta = 1 + ns;
        }
        unpacked_sz = osz;
        in += c_meta;
        in_size -= c_meta;
        uint32_t o2 = 0;
        sz = varint_get(in, in_end, &o2);
        in += sz;
        in_size -= uint32_t(sz);
        if (o2 > tmp1_size) return false;
        tmp1_size = o2;
    }
    if (in_size) {
        if (do_cat) {
            if (tmp1_size > in_size || tmp1_size > *out_size) return false;
            if (tmp1_size) {
                const uint8_t *src = g.upload(in, tmp1_size);
                FQZ5_HIP(hipMemcpyAsync(tmp1, src, tmp1_size, hipMemcpyDeviceToDevice, g.stream));
            }
        } else if (do_ext) {
            return false;
        } else if (!ent_uncompress(g, in, in_size, tmp1, tmp1_size, order == 1, do_rle != 0)) {
            return false;
        }
    } else {
        tmp1_size = 0;
    }
    uint32_t tmp2_size = tmp1_size;
    if (do_pack) {                                // hts_unpack (pack.c:207-344)
        if (per == 1) unpacked_sz = tmp1_size;
        if (per == 1) {
            if (tmp1_size)
                FQZ5_HIP(hipMemcpyAsync(d_out, tmp1, tmp1_size, hipMemcpyDeviceToDevice, g.stream));
        } else {
            if (per && (unpacked_sz + uint32_t(per) - 1) / uint32_t(per) > tmp1_size) return false;
            if (unpacked_sz) {
                PackItem it{tmp1, d_out, g.upload(map, 256), uint32_t(unpacked_sz), per};
                FQZ5_HIP(launch_pack(g.upload(&it, 1), 1, uint32_t(unpacked_sz), true, g.stream));
            }
        }
        tmp2_size = uint32_t(unpacked_sz);
    }
    *out_size = tmp2_size;
    return true;
}

}  // namespace

uint32_t arith_compress_bound_ref(uint32_t size, int order) {
    int N = (order >> 8) & 0xff;
    if (!N) N = 4;
    return uint32_t((order == 0 ? 1.05 * size + 257 * 3 + 4
                                : 1.05 * size + 257 * 257 * 3 + 4 + 257 * 3 + 4) +
                    5 + ((order & AX_PACK) ? 1 : 0) + ((order & AX_RLE) ? 1 + 257 * 3 + 4 : 0) +
                    ((order & AX_STRIPE) ? 7 + 5 * N : 0));
}

// host buffers (the C-ABI): out == nullptr => malloc of the bound
uint8_t *arith_compress_gpu(const uint8_t *in, uint32_t in_size, uint8_t *out, uint32_t *out_size,
                            int order) {
    if (in_size > uint32_t(INT_MAX) || (out && *out_size == 0)) {
        *out_size = 0;
        return nullptr;
    }
    GpuCtx &g = gpu();
    g.reset();
    uint8_t *own = nullptr;
    if (!out) {
        *out_size = arith_compress_bound_ref(in_size, order);
        own = out = static_cast<uint8_t *>(std::malloc(*out_size ? *out_size : 1));
        if (!out) {
            *out_size = 0;
            return nullptr;
        }
    }
    const uint8_t *d_in = g.upload(in, in_size);
    if (!compress_to(g, d_in, in_size, out, out_size, order)) {
        std::free(own);
        *out_size = 0;
        g.reset();
        return nullptr;
    }
    g.reset();
    return out;
}

uint8_t *arith_uncompress_gpu(const uint8_t *in, uint32_t in_size, uint8_t *out,
                              uint32_t *out_size) {
    GpuCtx &g = gpu();
    g.reset();
    uint8_t *d_out = out ? g.arena.alloc_n<uint8_t>(std::max<uint32_t>(*out_size, 1)) : nullptr;
    uint32_t sz = out ? *out_size : 0;
    if (!uncompress_to(g, in, in_size, d_out, &sz, out != nullptr)) {
        g.reset();
        return nullptr;
    }
    uint8_t *dst = out;
    if (!dst) {
        dst = static_cast<uint8_t *>(std::malloc(sz ? sz : 1));
        if (!dst) {
            g.reset();
            return nullptr;
        }
    }
    g.download(dst, d_out, sz);
    g.sync();
    *out_size = sz;
    g.reset();
    return dst;
}

}  // namespace fqz5
