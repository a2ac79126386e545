// names.cpp — fqzcomp5's name section (encode_names / decode_names,
// fqzcomp5.c:1408-1794) over batches of candidates: the host splits and
// tokenises (tok3.cpp), the GPU runs every lzp pass, every rANS stream (tok3
// columns, lzp outputs, flag bytes) and every decode as one batch each.
#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <exception>
#include <mutex>
#include <thread>

#include "host_dec.hpp"
#include "names.hpp"
#include "rans_format.hpp"

namespace fqz5 {

namespace {
void put32(uint8_t *p, uint32_t v) { std::memcpy(p, &v, 4); }
uint32_t get32(const uint8_t *p) { uint32_t v; std::memcpy(&v, p, 4); return v; }

// fn(i) for i < n on up to 16 host threads
template <class F> void on_threads(size_t n, F fn) {
    const size_t hw = size_t(host::threads());
    if (n <= 1 || hw == 1) {
        for (size_t i = 0; i < n; i++) fn(i);
        return;
    }
    std::atomic<size_t> next{0};
    std::exception_ptr err;
    std::mutex mu;
    auto work = [&] {
        try {
            for (size_t i; (i = next.fetch_add(1)) < n;) fn(i);
        } catch (...) {
            std::lock_guard<std::mutex> lk(mu);
            if (!err) err = std::current_exception();
        }
    };
    std::vector<std::thread> th;
    for (size_t t = 1; t < std::min(hw, n); t++) th.emplace_back(work);
    work();
    for (auto &t : th) t.join();
    if (err) std::rethrow_exception(err);
}
bool trace() {
    static const bool on = std::getenv("FQZ5_STEP_TRACE") != nullptr;
    return on;
}
double now_ms() {
    return std::chrono::duration<double, std::milli>(
               std::chrono::steady_clock::now().time_since_epoch()).count();
}
}  // namespace

void name_prepare(const uint8_t *h, uint32_t name_len, int strat, int level, NameEnc &E,
                  bool pipelined) {
    name_split(h, name_len, strat, level, E);
    name_tokenise(E, pipelined, nullptr);
}

void name_tokenise(NameEnc &E, bool pipelined, const T3Found *found) {
    if (E.strat == 0) return;
    E.tok_ok = tok3_tokenise(E.ids.data(), int(E.ids.size()), E.level, 0, E.tok, pipelined, found);
}

void name_split(const uint8_t *h, uint32_t name_len, int strat, int level, NameEnc &E) {
    E = NameEnc();
    E.strat = strat;
    E.level = level;
    E.name_len = name_len;
    if (strat == 0) return;                         // lzp + rANS only
    if (strat == 1) {
        E.ids.assign(h, h + name_len);
        return;
    }
    // strat 2: split each name into the read id (less a /1 or /2 suffix),
    // a flag byte and the comment after the first space or tab
    // (fqzcomp5.c:1462-1515)
    E.ids.resize(name_len + 1);
    E.comments.resize(name_len + 1);
    char *cp1 = E.ids.data(), *cp2 = E.comments.data();
    const char *nb = reinterpret_cast<const char *>(h);
    uint32_t i = 0;
    while (i < name_len) {
        uint32_t j, w1end = 0, w2start = 0, w2end = 0;
        int f = 0;
        for (j = i; j < name_len; j++) {
            if (nb[j] == '\0') {
                w2end = j;
                break;
            }
            if (!w2start && (nb[j] == ' ' || nb[j] == '\t')) {
                w1end = j;
                w2start = j + 1;
                f |= 4;                                 // has a comment
            }
        }
        if (!w1end) w1end = j;                         // (also when the space was at 0)
        if (!w2end) w2end = j;
        if (w2start) f |= nb[w2start - 1] == ' ' ? 0 : 8;
        if (w1end > 1 && nb[w1end - 2] == '/') {
            if (nb[w1end - 1] == '1') f |= 1, w1end -= 2;
            else if (nb[w1end - 1] == '2') f |= 3, w1end -= 2;
        }
        E.flag.push_back(uint8_t(f));
        std::memcpy(cp1, nb + i, w1end - i);
        cp1[w1end - i] = 0;
        cp1 += w1end - i + 1;
        if (w2start) {
            std::memcpy(cp2, nb + w2start, w2end - w2start);
            cp2[w2end - w2start] = 0;
            cp2 += w2end - w2start + 1;
        }
        i = j + 1;
    }
    E.ids.resize(size_t(cp1 - E.ids.data()));
    E.comments.resize(size_t(cp2 - E.comments.data()));
}

void name_add_lzp(GpuCtx &g, NameEnc &E, const uint8_t *d_names, std::vector<LzpEncReq> &lz) {
    const uint8_t *src = nullptr;
    uint32_t n = 0;
    if (E.strat == 0) {
        src = d_names;
        n = E.name_len;
    } else if (E.strat == 2 && !E.comments.empty() && E.tok_ok) {
        src = g.upload(reinterpret_cast<const uint8_t *>(E.comments.data()), E.comments.size());
        n = uint32_t(E.comments.size());
    } else {
        return;
    }
    LzpEncReq r;
    r.d_in = src;
    r.n = n;
    E.lzp = int(lz.size());
    lz.push_back(r);
}

void name_add_requests(GpuCtx &g, NameEnc &E, const std::vector<LzpEncReq> &lz,
                       std::vector<CompressReq> &reqs, const NameEnc *lead) {
    if (lead) {                                     // the same comments and flags
        E.lzp = lead->lzp;
        E.req_main = lead->req_main;
        E.req_flag = lead->req_flag;
        if (E.tok_ok) tok3_add_requests(g, E.tok, reqs);
        return;
    }
    if (E.lzp >= 0) {                               // rans_compress_4x16(lzp_out, .., 5)
        CompressReq r;
        r.d_in = lz[size_t(E.lzp)].d_out;
        r.n = lz[size_t(E.lzp)].out_len;
        r.order = 5;
        r.cap = compress_bound(r.n, r.order);
        E.req_main = int(reqs.size());
        reqs.push_back(std::move(r));
    }
    if (E.strat == 0 || !E.tok_ok) return;
    tok3_add_requests(g, E.tok, reqs);
    if (E.strat == 2) {                             // rans_compress_4x16(flag, nr, .., 129)
        CompressReq r;
        r.d_in = g.upload(E.flag.data(), E.flag.size());
        r.n = uint32_t(E.flag.size());
        r.order = 129;
        r.cap = compress_bound(r.n, r.order);
        E.req_flag = int(reqs.size());
        reqs.push_back(std::move(r));
    }
}

void name_assemble(GpuCtx &g, NameEnc &E, const std::vector<CompressReq> &reqs) {
    E.ok = false;
    E.out.clear();
    const CompressReq *main = E.req_main >= 0 ? &reqs[size_t(E.req_main)] : nullptr;
    const CompressReq *fl = E.req_flag >= 0 ? &reqs[size_t(E.req_flag)] : nullptr;
    if ((main && !main->ok) || (fl && !fl->ok)) return;
    std::vector<uint8_t> t3;
    if (E.strat != 0) {
        if (!E.tok_ok || !tok3_assemble(g, E.tok, reqs, t3)) return;
    }
    const uint32_t cm = main ? layout_size(main->out) : 0, cf = fl ? layout_size(fl->out) : 0;
    uint32_t clen = 0;
    if (E.strat == 0) clen = cm;
    else if (E.strat == 1) clen = uint32_t(t3.size());
    else clen = uint32_t(t3.size()) + cf + cm + 8;
    E.out.resize(9 + size_t(clen));
    uint8_t *cp = E.out.data();
    put32(cp, E.name_len);
    cp[4] = uint8_t(E.strat);
    put32(cp + 5, clen);
    cp += 9;
    std::vector<const Layout *> ls;
    std::vector<uint8_t *> dst;
    if (E.strat == 0) {
        ls.push_back(&main->out);
        dst.push_back(cp);
    } else if (E.strat == 1) {
        std::memcpy(cp, t3.data(), t3.size());
    } else {
        put32(cp, uint32_t(t3.size()));
        put32(cp + 4, cf);
        cp += 8;
        std::memcpy(cp, t3.data(), t3.size());
        cp += t3.size();
        ls.push_back(&fl->out);
        dst.push_back(cp);
        if (main) {
            ls.push_back(&main->out);
            dst.push_back(cp + cf);
        }
    }
    if (!ls.empty()) download_layouts(g, ls, dst);
    E.ok = true;
}

void names_encode_batch(GpuCtx &g, std::vector<NameEnc> &jobs,
                        const std::vector<const uint8_t *> &h_names,
                        const std::vector<const uint8_t *> &d_names,
                        const std::vector<uint32_t> &lens, const std::vector<int> &methods,
                        const std::vector<hipEvent_t> *ready) {
    const double t0 = trace() ? now_ms() : 0;
    // TLZP3 candidates (strat 0) need no tokenising: their lzp pass and
    // rANS stream run on the GPU (one helper thread) while the host threads
    // tokenise the others; the comment lzp passes of strat 2 follow.
    std::vector<size_t> early, late;
    for (size_t k = 0; k < jobs.size(); k++)
        (name_strat(methods[k]) == 0 ? early : late).push_back(k);
    std::vector<LzpEncReq> lz0, lz1;
    std::vector<CompressReq> rq0, rq1;
    // tok3's tokens do not depend on its level (the level only picks each
    // stream's rANS methods, tokenise_name3.c:1275-1366): candidates of one
    // section and strategy tokenise once and copy the rest
    std::vector<std::vector<size_t>> groups;
    for (size_t k : late) {
        auto same = [&](const std::vector<size_t> &gr) {
            const size_t j = gr[0];
            return h_names[j] == h_names[k] && lens[j] == lens[k] &&
                   name_strat(methods[j]) == name_strat(methods[k]);
        };
        auto it = std::find_if(groups.begin(), groups.end(), same);
        if (it == groups.end()) groups.push_back({k});
        else it->push_back(k);
    }
    // every section's trie searches in one GPU batch (tok3_search.hip), so
    // the host threads only code the tokens; a section the batch could not
    // take searches on the host ($FQZ5_TOK3_GPU=0: all of them)
    static const bool gpu_search = [] {
        const char *e = std::getenv("FQZ5_TOK3_GPU");
        return !e || std::atoi(e) != 0;
    }();
    std::vector<Tok3SearchJob> sj(groups.size());
    for (size_t i = 0; i < groups.size(); i++) {
        // the sections themselves, on the device: strat 2 searches the read
        // ids in place (split mode), strat 1 the names
        const size_t k = groups[i][0];
        sj[i].h_blk = reinterpret_cast<const char *>(h_names[k]);
        sj[i].d_blk = d_names[k];
        sj[i].len = lens[k];
        sj[i].split = name_strat(methods[k]) == 2;
    }
    // the ids (strat 2) or names (strat 1) of each section on the host, on
    // the host threads; the batch search waits for the sections' host
    // copies only through h_blk's last bytes
    on_threads(groups.size(), [&](size_t i) {
        const size_t k = groups[i][0];
        if (ready) FQZ5_HIP(hipEventSynchronize((*ready)[k]));
        name_split(h_names[k], lens[k], name_strat(methods[k]), name_level(methods[k]), jobs[k]);
    });
    const double ts = trace() ? now_ms() : 0;
    if (gpu_search && !groups.empty()) {
        std::vector<Tok3SearchJob *> sp;
        for (size_t i = 0; i < groups.size(); i++)
            if (lens[groups[i][0]]) sp.push_back(&sj[i]);
        if (!sp.empty()) tok3_search_batch(g, sp);
    }
    const double tsd = trace() ? now_ms() : 0;
    size_t on_host = 0;
    for (size_t i = 0; i < groups.size(); i++) on_host += !sj[i].ok;
    // the comments' lzp passes (strat 2) need the split only: their inputs go
    // up now and the passes run on the GPU thread below while the host
    // tokenises (a candidate whose tokenising then fails is dropped at
    // assembly, as before)
    // (the requests here, their uploads on the GPU thread: a ~200 MB pageable
    // copy on this thread delayed the tokenising by ~50 ms at -5)
    std::vector<const char *> lz1_host;
    for (const auto &gr : groups) {
        NameEnc &E = jobs[gr[0]];
        if (E.strat != 2 || E.comments.empty()) continue;
        LzpEncReq r;
        r.d_in = nullptr;
        r.n = uint32_t(E.comments.size());
        E.lzp = int(lz1.size());
        lz1.push_back(r);
        lz1_host.push_back(E.comments.data());
    }
    double t_early = 0;
    std::exception_ptr err0;
    std::thread gpu_early([&] {
        try {
            // a new thread starts on device 0: g's arena may grow (hipMalloc
            // on the current device) and must land on g's device
            FQZ5_HIP(hipSetDevice(g.device));
            for (size_t k : early) {
                name_prepare(h_names[k], lens[k], 0, name_level(methods[k]), jobs[k]);
                name_add_lzp(g, jobs[k], d_names[k], lz0);
            }
            if (!lz0.empty()) lzp_encode_batch(g, lz0);
            for (size_t i = 0; i < lz1.size(); i++)
                lz1[i].d_in = g.upload(reinterpret_cast<const uint8_t *>(lz1_host[i]), lz1[i].n);
            if (!lz1.empty()) lzp_encode_batch(g, lz1);
            for (size_t k : early) name_add_requests(g, jobs[k], lz0, rq0);
            if (!rq0.empty()) compress_batch(g, rq0);
            if (trace()) t_early = now_ms();
        } catch (...) {
            err0 = std::current_exception();
        }
    });
    // fewer host-searched sections than host threads: each tokenises on two
    // (its trie searches ahead on the second), so its names take ~60 % as long
    const size_t hw = size_t(host::threads());
    const bool pipelined = on_host < hw;
    try {
        on_threads(groups.size(), [&](size_t i) {
            const std::vector<size_t> &gr = groups[i];
            const size_t k = gr[0];
            name_tokenise(jobs[k], pipelined, sj[i].ok ? sj[i].found.data() : nullptr);
            for (size_t x = 1; x < gr.size(); x++) {
                NameEnc &E = jobs[gr[x]];
                E = jobs[k];
                E.level = E.tok.level = name_level(methods[gr[x]]);
            }
        });
    } catch (...) {
        gpu_early.join();
        throw;
    }
    const double t1 = trace() ? now_ms() : 0;
    gpu_early.join();
    if (err0) std::rethrow_exception(err0);
    const double t1b = trace() ? now_ms() : 0;
    const double t2 = t1b;
    for (const auto &gr : groups)
        for (size_t x = 0; x < gr.size(); x++)
            name_add_requests(g, jobs[gr[x]], lz1, rq1, x ? &jobs[gr[0]] : nullptr);
    if (!rq1.empty()) compress_batch(g, rq1);
    const double t3 = trace() ? now_ms() : 0;
    for (size_t k : early) name_assemble(g, jobs[k], rq0);
    for (size_t k : late) name_assemble(g, jobs[k], rq1);
    if (trace())
        std::fprintf(stderr, "names encode: %zu candidates, split %.1f ms, GPU trie searches "
                     "%.1f ms (%zu of %zu sections on the host), tokenise %.1f ms (TLZP3 and the "
                     "comment lzp passes on the GPU beside it: done at %.1f ms), waited %.1f ms, "
                     "lzp %.1f ms, %zu rANS "
                     "streams %.1f ms, assemble %.1f ms\n", jobs.size(), ts - t0, tsd - ts, on_host,
                     groups.size(), t1 - tsd, t_early ? t_early - t0 : 0.0, t1b - t1,
                     t2 - t1b, rq0.size() + rq1.size(), t3 - t2, now_ms() - t3);
}

// ---------------------------------------------------------------------------
bool name_dec_parse(NameDec &D) {
    D.ok = false;
    if (D.strat == 0) return true;
    if (D.strat == 1) return tok3_dec_parse(D.comp, D.c_len, D.tok);
    if (D.c_len < 8) return false;
    D.clen1 = get32(D.comp);
    D.clenf = get32(D.comp + 4);
    if (uint64_t(D.c_len) < uint64_t(D.clen1) + D.clenf + 8) return false;   // :1623
    D.clen2 = D.c_len - D.clen1 - D.clenf - 8;
    return tok3_dec_parse(D.comp + 8, D.clen1, D.tok);
}

namespace {
// a rANS stream's decoded size from its header (rans_uncompress_4x16's
// allocation), or false
bool rans_usize(const uint8_t *s, uint32_t n, uint32_t *u) {
    return n >= 2 && !(s[0] & ORD_NOSZ) && varint_get(s + 1, s + n, u) > 0;
}
}  // namespace

void name_dec_add_requests(GpuCtx &g, NameDec &D, std::vector<DecompressReq> &reqs) {
    if (!D.d_comp) D.d_comp = g.upload(D.comp, D.c_len);
    auto add = [&](uint32_t off, uint32_t n, uint8_t **d_out, uint32_t *ulen) -> int {
        if (!rans_usize(D.comp + off, n, ulen)) return -1;
        DecompressReq r;
        r.h_in = D.comp + off;
        r.d_in = D.d_comp + off;
        r.in_size = n;
        r.out_cap = *ulen;
        *d_out = g.arena.alloc_n<uint8_t>(size_t(*ulen) + 1);
        r.d_out = *d_out;
        reqs.push_back(r);
        return int(reqs.size()) - 1;
    };
    if (D.strat == 0) {
        D.req_main = add(0, D.c_len, &D.d_rout, &D.rout_len);
        return;
    }
    if (D.strat == 1) {
        tok3_dec_add_requests(g, D.tok, D.d_comp, reqs);
        return;
    }
    tok3_dec_add_requests(g, D.tok, D.d_comp + 8, reqs);
    D.req_flag = add(8 + D.clen1, D.clenf, &D.d_flag, &D.flag_len);
    if (D.clen2) D.req_main = add(8 + D.clen1 + D.clenf, D.clen2, &D.d_rout, &D.rout_len);
}

void name_dec_add_lzp(GpuCtx &g, NameDec &D, const std::vector<DecompressReq> &reqs,
                      std::vector<LzpDecReq> &lz) {
    if (D.req_main < 0 || !reqs[size_t(D.req_main)].ok) return;
    LzpDecReq z;
    z.d_in = D.d_rout;
    z.in_len = reqs[size_t(D.req_main)].out_size;
    z.cap = D.u_len;                                 // out = malloc(u_len) (:1597,1659)
    D.d_lout = g.arena.alloc_n<uint8_t>(size_t(D.u_len) + 4);
    z.d_out = D.d_lout;
    D.lzp = int(lz.size());
    lz.push_back(z);
}

void name_dec_fetch(GpuCtx &g, NameDec &D, const std::vector<DecompressReq> &reqs,
                    const std::vector<LzpDecReq> &lz) {
    D.fetched = false;
    D.ok = false;
    D.names = D.fl = D.out2 = nullptr;
    D.fl_len = D.out2_len = 0;
    if (D.strat == 0) {
        if (D.lzp < 0 || !lz[size_t(D.lzp)].ok) return;
        const uint32_t n = std::min(lz[size_t(D.lzp)].out_len, D.u_len);
        D.names = g.staging.alloc(size_t(D.u_len) + 1);
        g.download(D.names, D.d_lout, n);
        g.sync();
        std::memset(D.names + n, 0, D.u_len - n);
        D.fetched = true;
        return;
    }
    if (!tok3_dec_fetch(g, D.tok, reqs)) return;
    if (D.strat == 2) {
        if (D.req_flag < 0 || !reqs[size_t(D.req_flag)].ok) return;
        if (D.clen2 && (D.lzp < 0 || !lz[size_t(D.lzp)].ok)) return;
        D.fl_len = reqs[size_t(D.req_flag)].out_size;
        D.fl = g.staging.alloc(size_t(D.fl_len) + 1);
        g.download(D.fl, D.d_flag, D.fl_len);
        if (D.clen2) {
            D.out2_len = lz[size_t(D.lzp)].out_len;
            D.out2 = g.staging.alloc(size_t(D.out2_len) + 1);
            g.download(D.out2, D.d_lout, D.out2_len);
        }
        g.sync();
        // the stitch writes up to u_len + 2 bytes a record (fqzcomp5.c:1683-1777)
        D.names = g.staging.alloc(size_t(D.u_len) + size_t(D.fl_len) * 2 + 1);
    } else {
        D.names = g.staging.alloc(size_t(D.u_len) + 1);
    }
    D.fetched = true;
}

void name_dec_rebuild(NameDec &D) {
    D.ok = false;
    if (!D.fetched) return;
    if (D.strat == 0) {
        D.ok = true;
        return;
    }
    std::vector<uint8_t> out1;
    if (!tok3_dec_rebuild(D.tok, out1)) return;
    if (D.strat == 1) {
        const size_t n = std::min<size_t>(out1.size(), D.u_len);
        std::memcpy(D.names, out1.data(), n);
        std::memset(D.names + n, 0, D.u_len - n);
        D.ok = true;
        return;
    }
    // stitch id + flag + comment (fqzcomp5.c:1683-1777), straight into the
    // names buffer (its first u_len bytes are the section's)
    const uint32_t u_lenf = D.fl_len;
    const size_t out_size = size_t(D.u_len) + size_t(u_lenf) * 2;
    const uint8_t *cp1 = out1.data(), *cp1_end = cp1 + out1.size();
    const uint8_t *cpf = D.fl, *cpf_end = cpf + D.fl_len;
    const uint8_t *cp2 = D.clen2 ? D.out2 : nullptr;
    const uint8_t *cp2_end = cp2 + (cp2 ? D.out2_len : 0);
    uint8_t *cp = D.names, *cp_end = cp + out_size, *last_cp = nullptr;
    int rec = 0;
    D.flags.assign(u_lenf, 0);
    while (cp < cp_end) {
        while (cp1 < cp1_end && cp < cp_end && *cp1) *cp++ = *cp1++;
        cp1++;
        int flag = 0;
        if (cpf < cpf_end) flag = *cpf++;
        if ((flag & 1) && cp + 1 < cp_end) {
            *cp++ = '/';
            *cp++ = (flag & 2) ? '2' : '1';
        }
        if ((flag & 4) && cp < cp_end) *cp++ = (flag & 8) ? '\t' : ' ';
        if (cp2) {
            while (cp2 < cp2_end && cp < cp_end && *cp2) *cp++ = *cp2++;
            cp2++;
        }
        if (rec < int(u_lenf)) D.flags[size_t(rec)] = (flag & 3) == 3 ? 128u : 0u;   // FQZ_FREAD2
        rec++;
        if (cp == last_cp) break;                    // ran out of data
        if (cp < cp_end) *cp++ = 0;
        else return;                                 // goto err (:1763-1775)
        last_cp = cp;
    }
    D.nrec = rec;
    if (cp < D.names + D.u_len) std::memset(cp, 0, size_t(D.names + D.u_len - cp));
    D.ok = true;
}

void name_dec_finish(GpuCtx &g, NameDec &D, const std::vector<DecompressReq> &reqs,
                     const std::vector<LzpDecReq> &lz) {
    name_dec_fetch(g, D, reqs, lz);
    name_dec_rebuild(D);
}

void names_decode_batch(GpuCtx &g, std::vector<NameDec> &jobs,
                        const std::function<void()> &fetched) {
    const double t0 = trace() ? now_ms() : 0;
    std::vector<DecompressReq> reqs;
    std::vector<char> good(jobs.size());
    for (size_t k = 0; k < jobs.size(); k++) {
        good[k] = name_dec_parse(jobs[k]);
        if (good[k]) name_dec_add_requests(g, jobs[k], reqs);
    }
    if (!reqs.empty()) decompress_batch(g, reqs);
    std::vector<LzpDecReq> lz;
    for (size_t k = 0; k < jobs.size(); k++)
        if (good[k]) name_dec_add_lzp(g, jobs[k], reqs, lz);
    if (!lz.empty()) lzp_decode_batch(g, lz);
    const double t1 = trace() ? now_ms() : 0;
    for (size_t k = 0; k < jobs.size(); k++)
        if (good[k]) name_dec_fetch(g, jobs[k], reqs, lz);
        else jobs[k].fetched = false;
    const double t2 = trace() ? now_ms() : 0;
    if (fetched) fetched();
    on_threads(jobs.size(), [&](size_t k) { name_dec_rebuild(jobs[k]); });
    if (trace())
        std::fprintf(stderr, "names decode: %zu sections, %zu rANS streams + lzp %.1f ms, "
                     "fetch %.1f ms, rebuild %.1f ms\n", jobs.size(), reqs.size(), t1 - t0,
                     t2 - t1, now_ms() - t2);
}

}  // namespace fqz5
