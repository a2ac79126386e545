// blocks.cpp — fqzcomp5's block framing around the coded sections
// (encode_block / decode_block, fqzcomp5.c:2147-2547): the lengths section,
// the 12-byte block header with its CRC32 (computed on the device over the
// block as it lies in HBM), and the parse of a block back into its parts.
// The sections themselves are coded by block.cpp (fqz5_sections_*).
#include <algorithm>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/fqz5_block.h"
#include "gpu_ctx.hpp"
#include "rans_format.hpp"

namespace fqz5 {
GpuCtx &gpu();
void fqz5_set_error(const char *msg);
void crc32_dev(GpuCtx &g, uint32_t crc, const uint8_t *d_in, uint64_t n, uint32_t *d_out);
}  // namespace fqz5

using namespace fqz5;

extern "C" {

void fqz5_name_flags(const char *names, uint32_t name_len, int nrec, uint32_t *flags) {
    // load_seqs_kseq (fqzcomp5.c:518-527): the name buffer holds name [' '
    // comment] '\0' per record; kseq's name.l is the part before the space
    uint32_t p = 0;
    const char *last = nullptr;
    for (int i = 0; i < nrec; i++) {
        const char *nm = names + p;
        uint32_t l = 0;
        while (p + l < name_len && nm[l]) l++;
        uint32_t name_l = 0;
        while (name_l < l && nm[name_l] != ' ') name_l++;
        uint32_t f = 0;
        if (name_l > 1 && l >= 2 && nm[l - 1] == '2' && nm[l - 2] == '/') f = FQZ5_FREAD2;
        if (last && std::strcmp(nm, last) == 0) f = FQZ5_FREAD2;
        flags[i] = f;
        last = nm;
        p += l + 1;
    }
}

int fqz5_block_lengths(const uint32_t *len, int nrec, int32_t fixed_len, uint8_t *out,
                       uint32_t cap) {
    if (fixed_len) {                                   // [nb][varint] (:2190-2197)
        uint8_t v[8];
        const int nb = varint_put(v, nullptr, uint32_t(fixed_len));
        if (cap < uint32_t(nb) + 1) return -1;
        out[0] = uint8_t(nb);
        std::memcpy(out + 1, v, size_t(nb));
        return nb + 1;
    }
    if (cap < 5 + 5ull * uint32_t(std::max(nrec, 0))) return -1;   // [0][u32 size][varints]
    uint32_t nb = 5;
    out[0] = 0;
    for (int i = 0; i < nrec; i++) nb += uint32_t(varint_put(out + nb, nullptr, len[i]));
    const uint32_t body = nb - 5;
    std::memcpy(out + 1, &body, 4);
    return int(nb);
}

uint64_t fqz5_block_size(const fqz5_block_parts *p) {
    return 12ull + p->name_size + p->lengths_size + p->seq_size + (p->qual ? p->qual_size : 9u);
}

int fqz5_blocks_assemble(const fqz5_block_parts *parts, int n, uint8_t *d_out,
                         const uint64_t *off, uint32_t *size) {
    GpuCtx *gp = nullptr;
    try {
        GpuCtx &g = gpu();
        gp = &g;
        uint32_t *d_crc = g.arena.alloc_n<uint32_t>(size_t(std::max(n, 1)));
        for (int i = 0; i < n; i++) {
            const fqz5_block_parts &P = parts[i];
            uint8_t *b = d_out + off[i];
            uint64_t o = 12;
            auto d2d = [&](const uint8_t *src, uint32_t len) {
                if (len) FQZ5_HIP(hipMemcpyAsync(b + o, src, len, hipMemcpyDeviceToDevice, g.stream));
                o += len;
            };
            d2d(P.name, P.name_size);
            if (P.lengths_size) {
                uint8_t *st = g.staging.alloc(P.lengths_size);
                std::memcpy(st, P.lengths, P.lengths_size);
                FQZ5_HIP(hipMemcpyAsync(b + o, st, P.lengths_size, hipMemcpyHostToDevice, g.stream));
                o += P.lengths_size;
            }
            d2d(P.seq, P.seq_size);
            if (P.qual) {
                d2d(P.qual, P.qual_size);
            } else {                                   // FASTA: 9 zero bytes (:2258-2264)
                g.memset0(b + o, 9);
                o += 9;
            }
            if (o > UINT32_MAX) throw GpuError("fqz5_blocks_assemble: block over 4 GB");
            size[i] = uint32_t(o);
            crc32_dev(g, 0, b + 12, o - 12, d_crc + i);   // crc32 of bytes 12.. (:2268-2269)
        }
        std::vector<uint32_t> crc(size_t(std::max(n, 1)));
        g.download(crc.data(), d_crc, size_t(n));
        g.sync();
        uint8_t *hdr = g.staging.alloc(12ull * size_t(std::max(n, 1)));
        for (int i = 0; i < n; i++) {
            const uint32_t bs = size[i] - 4, nr = uint32_t(parts[i].nrec);
            std::memcpy(hdr + 12 * i, &bs, 4);
            std::memcpy(hdr + 12 * i + 4, &nr, 4);
            std::memcpy(hdr + 12 * i + 8, &crc[size_t(i)], 4);
            FQZ5_HIP(hipMemcpyAsync(d_out + off[i], hdr + 12 * i, 12, hipMemcpyHostToDevice, g.stream));
        }
        g.reset();
        return 0;
    } catch (const std::exception &e) {
        fqz5_set_error(e.what());
        try { if (gp) gp->reset(); } catch (...) {}
        return -1;
    }
}

int fqz5_block_parse(const uint8_t *d_block, uint64_t avail, fqz5_block_view *v,
                     uint32_t *lens, uint32_t lens_cap) {
    return fqz5_block_parse_v(d_block, avail, FQZ5_V11, v, lens, lens_cap);
}

int fqz5_block_parse_v(const uint8_t *d_block, uint64_t avail, int version,
                       fqz5_block_view *v, uint32_t *lens, uint32_t lens_cap) {
    GpuCtx *gp = nullptr;
    try {
        if (version < FQZ5_V11 || version > FQZ5_VOLD)
            throw GpuError("fqz5_block_parse: unknown container version");
        GpuCtx &g = gpu();
        gp = &g;
        std::memset(v, 0, sizeof *v);
        // the name section's offset: after [size][nrec][crc] (v1.1), or
        // after [size][nrec] (v1.0 and the headerless format have no CRC
        // field, fqzcomp5.c:2300-2318)
        const uint64_t hd = version == FQZ5_V11 ? 12 : 8;
        auto get = [&](uint64_t at, uint64_t n, uint8_t *dst) {   // GET (:2282-2288)
            if (at + n > avail) throw GpuError("fqz5_block_parse: block truncated");
            g.download(dst, d_block + at, n);
            g.sync();
        };
        uint8_t h[21];
        get(0, hd + 9, h);
        std::memcpy(&v->block_size, h, 4);
        std::memcpy(&v->nrec, h + 4, 4);
        uint32_t c_len;
        if (uint64_t(v->block_size) + 4 > avail || v->block_size < hd - 4)
            throw GpuError("fqz5_block_parse: block size past the data");
        const uint64_t end = uint64_t(v->block_size) + 4;
        if (version == FQZ5_V11) {
            uint32_t crc_stored;
            std::memcpy(&crc_stored, h + 8, 4);
            uint32_t *d_crc = g.arena.alloc_n<uint32_t>(1);
            crc32_dev(g, 0, d_block + 12, v->block_size - 8, d_crc);   // (:2309-2317)
            uint32_t crc = 0;
            g.download(&crc, d_crc, 1);
            g.sync();
            v->crc_ok = crc == crc_stored;
        } else {
            v->crc_ok = 1;                             // (no check, :2306)
        }
        std::memcpy(&v->name_ulen, h + hd, 4);
        std::memcpy(&c_len, h + hd + 5, 4);
        v->name_off = uint32_t(hd);
        v->name_size = 9 + c_len;
        uint64_t o = hd + 9 + c_len;
        uint8_t lh[6];
        uint64_t lens_sum = 0;
        get(o, 1, lh);
        if (lh[0] > 0) {                               // fixed length (:2385-2395)
            const uint64_t k = std::min<uint64_t>(5, end - std::min(end, o + 1));
            get(o + 1, k, lh + 1);
            uint32_t fl = 0;
            const int vl = varint_get(lh + 1, lh + 1 + k, &fl);
            if (!vl) throw GpuError("fqz5_block_parse: bad fixed length");
            v->fixed_len = int32_t(fl);
            if (lens)
                for (uint32_t i = 0; i < std::min(v->nrec, lens_cap); i++) lens[i] = fl;
            lens_sum = uint64_t(fl) * v->nrec;
            o += 1 + uint64_t(vl);
        } else {                                       // [0][u32 blen][varints] (:2396-2408)
            uint8_t b4[4];
            get(o + 1, 4, b4);
            o += 5;
            const uint64_t k = std::min<uint64_t>(5ull * v->nrec, end - std::min(end, o));
            std::vector<uint8_t> vb(size_t(k) + 1);
            if (k) get(o, k, vb.data());
            const uint8_t *p = vb.data(), *pe = vb.data() + k;
            for (uint32_t i = 0; i < v->nrec; i++) {
                uint32_t x = 0;
                const int vl = varint_get(p, pe, &x);
                if (!vl) throw GpuError("fqz5_block_parse: bad length varint");
                if (lens && i < lens_cap) lens[i] = x;
                lens_sum += x;
                p += vl;
            }
            o += uint64_t(p - vb.data());
        }
        uint8_t m[9];
        get(o, 9, m);                                  // seq (:2415-2419)
        std::memcpy(&v->seq_ulen, m + 1, 4);
        std::memcpy(&c_len, m + 5, 4);
        v->seq_off = uint32_t(o);
        v->seq_size = 9 + c_len;
        o += 9ull + c_len;
        get(o, 9, m);                                  // qual (:2471-2487)
        std::memcpy(&v->qual_ulen, m + 1, 4);
        std::memcpy(&c_len, m + 5, 4);
        v->qual_off = uint32_t(o);
        v->qual_size = 9 + c_len;
        o += 9ull + c_len;
        if (o > end) throw GpuError("fqz5_block_parse: sections past the block end");
        // the decoders write u_len bytes into outputs sized from these
        // fields: a quality section (not FASTA's 9 zero bytes) decodes to one
        // byte per base, and the record lengths cover the bases exactly
        const bool fasta = v->qual_ulen == 0 && v->qual_size == 9;
        if (!fasta && v->qual_ulen != v->seq_ulen)
            throw GpuError("fqz5_block_parse: quality and sequence sizes differ");
        if (lens_sum != v->seq_ulen)
            throw GpuError("fqz5_block_parse: record lengths do not sum to the bases");
        g.reset();
        return 0;
    } catch (const std::exception &e) {
        fqz5_set_error(e.what());
        try { if (gp) gp->reset(); } catch (...) {}
        return -1;
    }
}

// Many blocks at once: the same fields as fqz5_block_parse_v, with every
// block's header reads of one kind batched into one round trip (5 syncs for
// the whole batch instead of ~6 per block; a -5 decode of 38 blocks parsed
// them one call per block).
int fqz5_blocks_parse_v(const uint8_t *const *d_blocks, const uint64_t *avail, int n,
                        int version, fqz5_block_view *views, uint32_t *const *lens,
                        const uint32_t *lens_cap, int32_t *status) {
    GpuCtx *gp = nullptr;
    try {
        if (version < FQZ5_V11 || version > FQZ5_VOLD)
            throw GpuError("fqz5_block_parse: unknown container version");
        GpuCtx &g = gpu();
        gp = &g;
        const size_t N = size_t(std::max(n, 0));
        const uint64_t hd = version == FQZ5_V11 ? 12 : 8;
        std::vector<std::string> err(N);
        std::vector<uint64_t> end(N), o(N), lens_sum(N);
        auto fail = [&](size_t i, const char *m) { if (err[i].empty()) err[i] = m; };
        auto ok = [&](size_t i) { return err[i].empty(); };
        // host staging for the reads of one round
        auto round = [&](const std::vector<uint64_t> &at, const std::vector<uint64_t> &len,
                         std::vector<std::vector<uint8_t>> &out) {
            out.assign(N, {});
            for (size_t i = 0; i < N; i++) {
                if (!ok(i) || !len[i]) continue;
                if (at[i] + len[i] > avail[i]) { fail(i, "fqz5_block_parse: block truncated"); continue; }
                out[i].resize(len[i]);
                g.download(out[i].data(), d_blocks[i] + at[i], len[i]);
            }
        };
        std::vector<std::vector<uint8_t>> h;
        std::vector<uint64_t> at(N, 0), len(N, hd + 9);
        round(at, len, h);
        g.sync();
        uint32_t *d_crc = g.arena.alloc_n<uint32_t>(std::max<size_t>(N, 1));
        std::vector<uint32_t> crc_stored(N, 0), crc(N, 0);
        for (size_t i = 0; i < N; i++) {
            fqz5_block_view *v = &views[i];
            std::memset(v, 0, sizeof *v);
            if (!ok(i)) continue;
            std::memcpy(&v->block_size, h[i].data(), 4);
            std::memcpy(&v->nrec, h[i].data() + 4, 4);
            if (uint64_t(v->block_size) + 4 > avail[i] || v->block_size < hd - 4) {
                fail(i, "fqz5_block_parse: block size past the data");
                continue;
            }
            end[i] = uint64_t(v->block_size) + 4;
            if (version == FQZ5_V11) {
                std::memcpy(&crc_stored[i], h[i].data() + 8, 4);
                crc32_dev(g, 0, d_blocks[i] + 12, v->block_size - 8, d_crc + i);   // (:2309-2317)
            } else {
                v->crc_ok = 1;                         // (no check, :2306)
            }
            uint32_t c_len;
            std::memcpy(&v->name_ulen, h[i].data() + hd, 4);
            std::memcpy(&c_len, h[i].data() + hd + 5, 4);
            v->name_off = uint32_t(hd);
            v->name_size = 9 + c_len;
            o[i] = hd + 9 + c_len;
        }
        // the lengths section's first bytes (and the CRCs)
        for (size_t i = 0; i < N; i++) {
            at[i] = o[i];
            len[i] = ok(i) ? std::min<uint64_t>(6, end[i] - std::min(end[i], o[i])) : 0;
            if (ok(i) && !len[i]) fail(i, "fqz5_block_parse: block truncated");
        }
        round(at, len, h);
        if (version == FQZ5_V11 && N) g.download(crc.data(), d_crc, N);
        g.sync();
        std::vector<uint64_t> vat(N, 0), vlen(N, 0);
        std::vector<char> varlen(N, 0);
        for (size_t i = 0; i < N; i++) {
            fqz5_block_view *v = &views[i];
            if (version == FQZ5_V11) v->crc_ok = crc[i] == crc_stored[i];
            if (!ok(i)) continue;
            const uint8_t *lh = h[i].data();
            if (lh[0] > 0) {                           // fixed length (:2385-2395)
                uint32_t fl = 0;
                const int vl = varint_get(lh + 1, lh + h[i].size(), &fl);
                if (!vl) { fail(i, "fqz5_block_parse: bad fixed length"); continue; }
                v->fixed_len = int32_t(fl);
                if (lens[i])
                    for (uint32_t r = 0; r < std::min(v->nrec, lens_cap[i]); r++) lens[i][r] = fl;
                lens_sum[i] = uint64_t(fl) * v->nrec;
                o[i] += 1 + uint64_t(vl);
            } else {                                   // [0][u32 blen][varints] (:2396-2408)
                if (h[i].size() < 5) { fail(i, "fqz5_block_parse: block truncated"); continue; }
                varlen[i] = 1;
                o[i] += 5;
                vat[i] = o[i];
                vlen[i] = std::min<uint64_t>(5ull * v->nrec, end[i] - std::min(end[i], o[i]));
            }
        }
        round(vat, vlen, h);                           // variable lengths' varints
        g.sync();
        for (size_t i = 0; i < N; i++) {
            fqz5_block_view *v = &views[i];
            if (!ok(i) || !vlen[i]) {
                if (ok(i) && varlen[i] && v->nrec) fail(i, "fqz5_block_parse: bad length varint");
                continue;
            }
            const uint8_t *p = h[i].data(), *pe = p + h[i].size();
            uint64_t sum = 0;
            for (uint32_t r = 0; r < v->nrec; r++) {
                uint32_t x = 0;
                const int vl = varint_get(p, pe, &x);
                if (!vl) { fail(i, "fqz5_block_parse: bad length varint"); break; }
                if (lens[i] && r < lens_cap[i]) lens[i][r] = x;
                sum += x;
                p += vl;
            }
            lens_sum[i] = sum;
            o[i] += uint64_t(p - h[i].data());
        }
        for (size_t i = 0; i < N; i++) { at[i] = o[i]; len[i] = ok(i) ? 9 : 0; }
        round(at, len, h);                             // seq (:2415-2419)
        g.sync();
        for (size_t i = 0; i < N; i++) {
            fqz5_block_view *v = &views[i];
            if (!ok(i)) continue;
            uint32_t c_len;
            std::memcpy(&v->seq_ulen, h[i].data() + 1, 4);
            std::memcpy(&c_len, h[i].data() + 5, 4);
            v->seq_off = uint32_t(o[i]);
            v->seq_size = 9 + c_len;
            o[i] += 9ull + c_len;
            at[i] = o[i];
        }
        round(at, len, h);                             // qual (:2471-2487)
        g.sync();
        int bad = 0;
        for (size_t i = 0; i < N; i++) {
            fqz5_block_view *v = &views[i];
            if (ok(i)) {
                uint32_t c_len;
                std::memcpy(&v->qual_ulen, h[i].data() + 1, 4);
                std::memcpy(&c_len, h[i].data() + 5, 4);
                v->qual_off = uint32_t(o[i]);
                v->qual_size = 9 + c_len;
                o[i] += 9ull + c_len;
                if (o[i] > end[i]) fail(i, "fqz5_block_parse: sections past the block end");
            }
            if (ok(i)) {
                const bool fasta = v->qual_ulen == 0 && v->qual_size == 9;
                if (!fasta && v->qual_ulen != v->seq_ulen)
                    fail(i, "fqz5_block_parse: quality and sequence sizes differ");
                else if (lens_sum[i] != v->seq_ulen)
                    fail(i, "fqz5_block_parse: record lengths do not sum to the bases");
            }
            status[i] = ok(i) ? 0 : -1;
            if (!ok(i) && !bad++) fqz5_set_error(err[i].c_str());
        }
        g.reset();
        return bad ? -1 : 0;
    } catch (const std::exception &e) {
        fqz5_set_error(e.what());
        try { if (gp) gp->reset(); } catch (...) {}
        return -1;
    }
}

}  // extern "C"
