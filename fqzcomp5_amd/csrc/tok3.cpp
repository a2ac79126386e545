// tok3.cpp — the read-name tokeniser (htscodecs tokenise_name3.c, the
// TOK3 name methods of fqzcomp5) behind its own C-ABI:
// tok3_encode_names / tok3_decode_names, byte-identical to the reference.
//
// A block of names becomes up to 128 x 16 byte streams ("descriptors"): per
// token position, the token types and one stream per type's values, each
// name tokenised against an earlier name found through a trie of all names
// (search_trie, tokenise_name3.c:591-695).  The tokenising is a short serial
// pass over the names on the host (a name's tokens depend on the earlier
// name and on per-column running counts); the descriptors are then entropy
// coded as one batch of rANS 4x16 candidates on the GPU (compress():
// every method the level lists for the stream's type, smallest kept, first
// on ties, tokenise_name3.c:1268-1417), and decoded as one batch of rANS
// streams before the names are rebuilt.  use_arith (never set by fqzcomp5,
// fqzcomp5.c:1433,1490) codes them with arith_dynamic, also on the GPU.
#include <algorithm>
#include <cctype>
#include <climits>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <thread>
#include <vector>

#include "../../include/fqz5_mi355x.h"
#include "rans_codec.hpp"
#include "rans_format.hpp"
#include "tok3.hpp"
#include "tok3_search.h"
#include "names.hpp"

namespace fqz5 {
void fqz5_set_error(const char *msg);   // capi.cpp
namespace {

constexpr int MAX_TOKENS = 128;                 // tokenise_name3.c:75-76
constexpr int MAX_TBLOCKS = MAX_TOKENS << 4;

enum NameType : int {                           // :81-82
    N_TYPE = 0, N_ALPHA, N_CHAR, N_DIGITS0, N_DZLEN, N_DUP, N_DIFF,
    N_DIGITS, N_DDELTA, N_DDELTA0, N_MATCH, N_NOP, N_END, N_ALL
};

// <ctype.h> classes of the C locale, for 7-bit bytes (the names are 7-bit)
inline bool c_alpha(uint8_t c) { return uint8_t((c | 32) - 'a') < 26; }
inline bool c_digit(uint8_t c) { return uint8_t(c - '0') < 10; }
inline bool c_space(uint8_t c) { return c == ' ' || uint8_t(c - 9) < 5; }
inline bool c_punct(uint8_t c) { return c > 32 && c < 127 && !c_alpha(c) && !c_digit(c); }
inline bool c_xdigit(uint8_t c) { return c_digit(c) || uint8_t((c | 32) - 'a') < 6; }

// punctuation or space (the trie search's from_punct bytes), by byte
struct PsTable {
    uint8_t t[256];
    PsTable() {
        for (int c = 0; c < 256; c++) t[c] = (c_punct(uint8_t(c)) || c_space(uint8_t(c))) ? 1 : 0;
    }
};
const PsTable PS_TAB;
const uint8_t *const PS = PS_TAB.t;

struct Tok { int type = 0, ival = 0, sval = 0; };    // last_context_tok
// last_context: a name's tokens live in one arena per block (a finished
// name's tokens never change, so a duplicate shares its original's)
struct Last {
    const char *name = nullptr;
    int ntok = 0;
    uint32_t off = 0;                                  // first token in the arena
};

// ---------------------------------------------------------------------------
// The name formats search_trie special-cases (:600-644): the prefix length
// whose trie node picks the name to compare against, and a fixed-length
// leading token.
int name_format(const char *data, size_t len, int *is_fixed, int *fixed_len) {
    *fixed_len = 0;
    *is_fixed = 0;
    const char *d = *data == '@' ? data + 1 : data;
    const int l = *data == '@' ? int(len) - 1 : int(len);
    const int f = (*data == '>') ? 1 : 0;
    auto xd = [](char c) { return c_xdigit(uint8_t(c)); };
    if (l > 70 && d[f + 0] == 'm' && d[7] == '_' && d[f + 14] == '_' && d[f + 61] == '/')
        return 60;                                     // PacBio
    if (l == 17 && d[f + 5] == ':' && d[f + 11] == ':') {
        *fixed_len = 6;                                // IonTorrent
        *is_fixed = 1;
        return 6;
    }
    if (l >= 36 && d[f + 8] == '-' && d[f + 13] == '-' && d[f + 18] == '-' && d[f + 23] == '-' &&
        xd(d[f + 0]) && xd(d[f + 7]) && xd(d[f + 9]) && xd(d[f + 12]) && xd(d[f + 14]) &&
        xd(d[f + 17]) && xd(d[f + 19]) && xd(d[f + 22]) && xd(d[f + 24]) && xd(d[f + 35])) {
        *fixed_len = 36;                               // ONT uuid
        *is_fixed = 1;
        return 36;
    }
    int colons = 0;                                    // Illumina: lane:tile:x:y
    size_t i = 0;
    for (i = 0; i < len && data[i] > ' '; i++) {}
    while (i > 0 && colons < 4)
        if (data[--i] == ':') colons++;
    if (colons == 4) {
        *fixed_len = int(i) + 1;
        *is_fixed = 1;
        return int(i) + 1;
    }
    return INT_MAX;
}

// Trie over all names of the block (build_trie / search_trie, :477-695): a
// node keeps the index of the last name that walked through it (24 bits, as
// the reference's bitfield), initially the one that created it.  Fused with
// build_trie: the reference builds the trie of every name first (a node
// holding its first name) and then searches name by name (each visit
// leaving the visitor's number), so at name n's visit a node holds the last
// earlier name through it, or n itself when n is the first.  A node created
// on first sight holds n: the same values in one pass.
//
// Stored as a radix trie: an edge carries a run of characters (a slice of
// the name that made it) whose one-character nodes would all hold the same
// name, since every visit walks a whole prefix.  A visit that ends or turns
// off inside an edge splits it: the walked part takes the visitor, the rest
// keeps its name.  A name thus costs a character compare per byte and a few
// node operations instead of a node (and a sibling scan) per byte.
struct Trie {
    struct Node {
        const char *s = nullptr;                       // the edge's characters
        uint32_t len = 0, n = 0;
        int child = -1, sib = -1;
        char fc = 0;                                   // s[0]
    };
    std::vector<Node> nodes{Node()};                   // node 0: the root
    std::vector<uint32_t> ps{0};                       // punct / space bytes before p

    // -> the name to tokenise against, or -1 (:591-695)
    int search(const char *data, size_t len, uint32_t n, int *exact, int *is_fixed,
               int *fixed_len) {
        *exact = 0;
        const int prefix_len = name_format(data, len, is_fixed, fixed_len);
        const uint32_t nn = n & 0xffffffu;
        // the walk reads to the first byte <= '\n'; a byte >= 0x80 ends it
        // with -1 after the bytes before it were walked (:654-674)
        size_t L = 0;
        bool high = false;
        if (ps.size() < len + 1) ps.resize(len + 1);
        while (L < len && uint8_t(data[L]) > '\n') {
            if (uint8_t(data[L]) & 0x80) { high = true; break; }
            ps[L + 1] = ps[L] + PS[uint8_t(data[L])];
            L++;
        }
        int from = -1, from_punct = -1, p3 = -1;
        // the bytes [a, b) (b > a) walked through nodes that held val, in
        // order: per byte p the reference sets from = val, from_punct = val
        // if byte p is punctuation or space and val is not this name, and p3
        // = val if p + 1 is the prefix length
        auto run = [&](size_t a, size_t b, uint32_t val) {
            from = int(val);
            if (val != nn && ps[b] != ps[a]) from_punct = int(val);
            if (int64_t(prefix_len) > int64_t(a) && int64_t(prefix_len) <= int64_t(b)) p3 = int(val);
        };
        auto leaf = [&](int parent, size_t i) {       // the rest of the name, new
            Node w;
            w.s = data + i;
            w.len = uint32_t(L - i);
            w.n = nn;
            w.fc = data[i];
            w.sib = nodes[size_t(parent)].child;
            nodes.push_back(w);
            nodes[size_t(parent)].child = int(nodes.size()) - 1;
            if (i < L) run(i, L, nn);
        };
        int t = 0;
        size_t i = 0;
        while (i < L) {
            const char c = data[i];
            int x = nodes[size_t(t)].child, l = -1;
            while (x >= 0 && nodes[size_t(x)].fc != c) { l = x; x = nodes[size_t(x)].sib; }
            if (x < 0) {
                leaf(t, i);
                break;
            }
            if (l >= 0) {                              // to the front (order is immaterial)
                nodes[size_t(l)].sib = nodes[size_t(x)].sib;
                nodes[size_t(x)].sib = nodes[size_t(t)].child;
                nodes[size_t(t)].child = x;
            }
            const Node e = nodes[size_t(x)];
            const size_t m = std::min<size_t>(e.len, L - i);
            size_t k = 1;
            while (k < m && e.s[k] == data[i + k]) k++;
            run(i, i + k, e.n);
            if (k == e.len) {                          // the whole edge
                nodes[size_t(x)].n = nn;
                t = x;
                i += k;
                continue;
            }
            Node mid;                                  // split: [0, k) walked, [k, len) kept
            mid.s = e.s;
            mid.len = uint32_t(k);
            mid.n = nn;
            mid.fc = e.fc;
            mid.child = x;
            mid.sib = e.sib;
            nodes[size_t(x)].s = e.s + k;
            nodes[size_t(x)].len = e.len - uint32_t(k);
            nodes[size_t(x)].fc = e.s[k];
            nodes[size_t(x)].sib = -1;
            nodes.push_back(mid);
            const int y = int(nodes.size()) - 1;
            nodes[size_t(t)].child = y;                // x was at the front
            i += k;
            if (i < L) leaf(y, i);
            break;
        }
        if (high) return -1;
        *exact = (int(nn) != from) && len;
        return *exact ? from : (p3 != -1 ? p3 : from_punct);
    }
};

// search_trie's results for one name (Trie::search here, or k_t3_find)
using Found = T3Found;

// ---------------------------------------------------------------------------
struct Encoder {
    std::vector<std::vector<uint8_t>> desc = std::vector<std::vector<uint8_t>>(MAX_TBLOCKS);
    int dcount[MAX_TOKENS] = {0}, icount[MAX_TOKENS] = {0};
    int max_tok = 1;                                 // create_context (:204)
    int counter = 0;
    std::vector<Last> lc;
    std::vector<Tok> toks;                             // every name's tokens
    Trie trie;

    void grow_tok(int ntok) {                          // the reference's max_tok resets
        for (int t = max_tok; t <= ntok; t++) {
            for (int k = 0; k < 16; k++) desc[size_t(t << 4 | k)].clear();
            dcount[t] = icount[t] = 0;
        }
        max_tok = ntok + 1;
    }
    void type(int ntok, int ty) { desc[size_t(ntok << 4)].push_back(uint8_t(ty)); }
    void tint(int ntok, int ty, uint32_t v) {          // encode_token_int
        type(ntok, ty);
        auto &b = desc[size_t(ntok << 4 | ty)];
        for (int k = 0; k < 4; k++) b.push_back(uint8_t(v >> (8 * k)));
    }
    void tint1(int ntok, int ty, uint32_t v) {         // encode_token_int1
        type(ntok, ty);
        desc[size_t(ntok << 4 | ty)].push_back(uint8_t(v));
    }
    void tint1_(int ntok, int ty, uint32_t v) {        // encode_token_int1_ (no type)
        desc[size_t(ntok << 4 | ty)].push_back(uint8_t(v));
    }
    void alpha(int ntok, const char *s, int len) {
        type(ntok, N_ALPHA);
        auto &b = desc[size_t(ntok << 4 | N_ALPHA)];
        b.insert(b.end(), s, s + len);
        b.push_back(0);
    }
    void chr(int ntok, char c) {
        type(ntok, N_CHAR);
        desc[size_t(ntok << 4 | N_CHAR)].push_back(uint8_t(c));
    }

    // encode_name (:697-1020), mode 1
    bool name(char *nm, int len) {
        Found f;
        f.pnum = trie.search(nm, size_t(len), uint32_t(counter), &f.exact, &f.is_fixed, &f.fixed_len);
        return name(nm, len, f);
    }
    // ... with the trie search's results for this name
    bool name(char *nm, int len, const Found &f) {
        int is_fixed = f.is_fixed;
        const int fixed_len = f.fixed_len, exact = f.exact;
        const int cnum = counter++;
        int pnum = f.pnum;
        if (pnum < 0) pnum = cnum ? cnum - 1 : 0;
        Last &C = lc[size_t(cnum)];
        const Last &P = lc[size_t(pnum)];
        if (exact && size_t(len) == std::strlen(P.name)) {
            tint(0, N_DUP, uint32_t(cnum - pnum));
            C.name = nm;
            C.ntok = P.ntok;
            C.off = P.off;
            return true;
        }
        C.off = uint32_t(toks.size());
        // slot t of this name exists before any pointer into the arena is
        // taken for step t (growing it moves the arena)
        auto ensure = [&](int t) {
            if (toks.size() < size_t(C.off) + size_t(t) + 1) toks.resize(size_t(C.off) + size_t(t) + 1);
        };
        auto ct = [&](int t) -> Tok & { return toks[size_t(C.off) + size_t(t)]; };
        tint(0, N_DIFF, uint32_t(cnum - pnum));
        int ntok = 1, i;
        auto ptok = [&](int t) -> const Tok * {
            return (pnum < cnum && t < P.ntok) ? &toks[size_t(P.off) + size_t(t)] : nullptr;
        };
        if (fixed_len == 36) {                         // ONT uuid (:735-752)
            if (37 >= max_tok) grow_tok(37);
            for (i = 0; i < 36; i++, ntok++) {
                chr(ntok, nm[i]);
                ensure(ntok);
                ct(ntok) = {N_CHAR, nm[i], 0};
            }
            is_fixed = 0;
            i = 36;
        } else if (is_fixed) {                         // :753-773
            if (ntok >= max_tok) grow_tok(ntok);
            ensure(ntok);
            const Tok *pt = ptok(ntok);
            if (pt && pt->type == N_ALPHA && pt->ival == fixed_len &&
                std::memcmp(nm, P.name, size_t(fixed_len)) == 0)
                type(ntok, N_MATCH);
            else
                alpha(ntok, nm, fixed_len);
            ct(ntok++) = {N_ALPHA, fixed_len, 0};
            i = fixed_len;
        } else {
            i = 0;
        }
        for (; i < len; i++) {
            if (ntok >= max_tok) {
                if (max_tok >= MAX_TOKENS) return false;
                grow_tok(ntok);
            }
            ensure(ntok);
            const uint8_t ci = uint8_t(nm[i]);
            bool as_char = false;
            if (c_alpha(ci)) {                         // :791-838
                int s = i + 1;
                while (s < len && (c_alpha(uint8_t(nm[s])) || c_punct(uint8_t(nm[s])))) s++;
                if (s - i == 1) {
                    as_char = true;
                } else {
                    const Tok *pt = ptok(ntok);
                    if (pt && pt->type == N_ALPHA && s - i == pt->ival &&
                        std::memcmp(&nm[i], &P.name[pt->sval], size_t(s - i)) == 0)
                        type(ntok, N_MATCH);
                    else
                        alpha(ntok, &nm[i], s - i);
                    ct(ntok) = {N_ALPHA, s - i, i};
                    i = s - 1;
                }
            } else if (c_digit(ci)) {
                // digits (:839-943); a leading 0, or the previous name's
                // token being DIGITS0 of the same length, codes DIGITS0
                uint32_t s = uint32_t(i), v = 0;
                while (s < uint32_t(len) && c_digit(uint8_t(nm[s])) && s - uint32_t(i) < 9) {
                    v = v * 10 + uint32_t(nm[s] - '0');
                    s++;
                }
                const uint32_t dl = s - uint32_t(i);
                const Tok *pt = ptok(ntok);
                const bool zero = ci == '0' || (pt && pt->type == N_DIGITS0 && uint32_t(pt->sval) == dl);
                if (zero) {
                    if (pt && pt->type == N_DIGITS0) {
                        const int d = int(v - uint32_t(pt->ival));
                        if (d == 0 && uint32_t(pt->sval) == dl) {
                            type(ntok, N_MATCH);
                        } else if (d < 256 && d >= 0 && uint32_t(pt->sval) == dl) {
                            tint1(ntok, N_DDELTA0, uint32_t(d));
                        } else {
                            tint1_(ntok, N_DZLEN, dl);
                            tint(ntok, N_DIGITS0, v);
                        }
                    } else {
                        tint1_(ntok, N_DZLEN, dl);
                        tint(ntok, N_DIGITS0, v);
                    }
                    ct(ntok) = {N_DIGITS0, int(v), int(dl)};
                } else {
                    if (pt && pt->type == N_DIGITS) {
                        const int d = int(v - uint32_t(pt->ival));
                        if (d == 0) {
                            type(ntok, N_MATCH);
                        } else if (d < 256 && d >= 0 && (5 + dcount[ntok]) > icount[ntok]) {
                            tint1(ntok, N_DDELTA, uint32_t(d));
                            dcount[ntok]++;
                        } else {
                            tint(ntok, N_DIGITS, v);
                            icount[ntok]++;
                        }
                    } else {
                        tint(ntok, N_DIGITS, v);
                    }
                    // token_str keeps whatever this slot held (:939-941)
                    ct(ntok).type = N_DIGITS;
                    ct(ntok).ival = int(v);
                }
                i = int(s) - 1;
            } else {
                as_char = true;
            }
            if (as_char) {                             // n_char (:944-967)
                const Tok *pt = ptok(ntok);
                if (pt && pt->type == N_CHAR && nm[i] == char(pt->ival))
                    type(ntok, N_MATCH);
                else
                    chr(ntok, nm[i]);
                ct(ntok).type = N_CHAR;
                ct(ntok).ival = nm[i];
            }
            ntok++;
        }
        if (ntok >= max_tok) {
            if (max_tok >= MAX_TOKENS) return false;
            grow_tok(ntok);
        }
        type(ntok, N_END);
        ensure(ntok);
        C.name = nm;
        C.ntok = ntok;
        return true;
    }
};

// compress()'s method lists (:1281-1358), by level (1-9 -> 0-4) and type
const int METH[5][N_ALL][7] = {
    {{1, 128}, {1, 129}, {1, 0}, {1, 8}, {1, 0}, {1, 8}, {1, 8}, {1, 8}, {1, 0}, {1, 128},
     {1, 0}, {1, 0}, {1, 0}},
    {{2, 192, 0}, {2, 129, 1}, {1, 0}, {2, 128 + 8, 0}, {1, 0}, {1, 192 + 8}, {1, 128 + 8},
     {1, 192 + 8}, {1, 0}, {1, 128}, {1, 0}, {1, 0}, {1, 0}},
    {{2, 192, 0}, {4, 1, 128, 0, 129}, {1, 0}, {2, 200, 0}, {1, 0}, {1, 200}, {2, 192, 200},
     {2, 132, 201}, {1, 0}, {1, 128}, {1, 0}, {1, 0}, {1, 0}},
    {{3, 193, 0, 1}, {5, 128, 1, 128, 0, 129}, {2, 1, 0}, {2, 200, 0}, {1, 0}, {1, 201},
     {2, 192, 200}, {2, 132, 201}, {1, 0}, {1, 128}, {1, 0}, {1, 0}, {1, 0}},
    {{6, 192, 0, 1, 65, 193, 132}, {4, 132, 1, 0, 129}, {3, 1, 0, 192}, {4, 201, 0, 192, 64},
     {3, 0, 128, 1}, {1, 201}, {3, 192, 201, 65}, {6, 132, 201, 1, 192, 129, 193},
     {3, 1, 0, 192}, {3, 192, 1, 0}, {1, 0}, {1, 0}, {1, 0}},
};

#define GUARD_BEGIN try {
#define GUARD_END(failret)                                                    \
    }                                                                         \
    catch (const std::exception &e) {                                         \
        fqz5_set_error(e.what());                                             \
        return failret;                                                       \
    }

int put_varint(uint8_t *out, uint32_t v) {
    uint8_t tmp[8];
    const int k = varint_put(tmp, nullptr, v);
    std::memcpy(out, tmp, size_t(k));
    return k;
}

}  // namespace

// The names loop in two threads: the trie search of each name (~60 % of the
// time, cache misses) runs ahead on a helper thread and publishes its
// results in batches; this thread codes each name once its search is done.
// The same names in the same order, so the same streams.
static bool tokenise_pipelined(Encoder &E, char *blk, int len) {
    std::vector<uint32_t> st, ln;                      // names (:1487-1505)
    for (int i = 0, j = 0; i < len; j = ++i) {
        while (i < len && static_cast<signed char>(blk[i]) >= ' ') i++;
        if (i >= len) break;
        if (blk[i] != '\0' && blk[i] != '\n') return false;
        blk[i] = '\0';
        st.push_back(uint32_t(j));
        ln.push_back(uint32_t(i - j));
    }
    const size_t nn = st.size();
    std::vector<Found> found(nn);
    std::atomic<size_t> done{0};
    std::atomic<bool> stop{false};
    constexpr size_t BATCH = 256;
    std::thread th([&] {
        for (size_t k = 0; k < nn && !stop.load(std::memory_order_relaxed); k++) {
            Found &f = found[k];
            f.pnum = E.trie.search(blk + st[k], ln[k], uint32_t(k), &f.exact, &f.is_fixed, &f.fixed_len);
            if ((k + 1) % BATCH == 0 || k + 1 == nn) done.store(k + 1, std::memory_order_release);
        }
    });
    bool ok = true;
    for (size_t k = 0; k < nn && ok; k++) {
        while (done.load(std::memory_order_acquire) <= k) std::this_thread::yield();
        ok = E.name(blk + st[k], int(ln[k]), found[k]);
    }
    stop.store(true);
    th.join();
    return ok;
}

bool tok3_tokenise(char *blk, int len, int level, int use_arith, Tok3Enc &T, bool pipelined,
                   const T3Found *found) {
    T = Tok3Enc();
    T.level = level;
    T.use_arith = use_arith;
    T.last_start = -1;
    if (len < 0) return false;
    int nreads = 0, last_start = 0, i, j;
    for (i = 0; i < len; i++)
        if (blk[i] <= '\n') nreads++;
    if (nreads <= 0 || nreads > 10000000) return false;     // create_context (:172-187)
    Encoder E;
    E.lc.resize(size_t(nreads) + 1);
    if (!found) E.trie.nodes.reserve(size_t(len) / 4 + 16);
    // the trie of all names (:1469-1482) is built inside the search (Trie::
    // search); its loop's line ends give last_start (it cannot fail: its
    // lines hold no byte >= 0x80)
    for (i = len - 1; i >= 0; i--)
        if (blk[i] <= '\n') { last_start = i + 1; break; }
    T.last_start = last_start;
    if (found) {                                      // the searches done (tok3_search_batch)
        size_t k = 0;
        for (i = j = 0; i < len; j = ++i) {
            while (i < len && static_cast<signed char>(blk[i]) >= ' ') i++;
            if (i >= len) break;
            if (blk[i] != '\0' && blk[i] != '\n') return false;
            blk[i] = '\0';
            if (!E.name(&blk[j], i - j, found[k++])) return false;
        }
    } else if (!pipelined) {
        for (i = j = 0; i < len; j = ++i) {            // names (:1487-1505)
            while (i < len && static_cast<signed char>(blk[i]) >= ' ') i++;
            if (i >= len) break;
            if (blk[i] != '\0' && blk[i] != '\n') return false;
            blk[i] = '\0';
            if (!E.name(&blk[j], i - j)) return false;
        }
    } else if (!tokenise_pipelined(E, blk, len)) {
        return false;
    }
    // drop the type stream of a column that is all MATCH bar its first
    // entry while the column has other streams (:1531-1553)
    for (i = 0; i < E.max_tok * 16; i += 16) {
        std::vector<uint8_t> &b = E.desc[size_t(i)];
        if (b.empty()) continue;
        size_t z = 1;
        while (z < b.size() && b[z] == N_MATCH) z++;
        if (z == b.size()) {
            int k = 1;
            while (k < 16 && E.desc[size_t(i + k)].empty()) k++;
            if (k < 16) b.clear();
        }
    }
    T.nreads = nreads;
    T.max_tok = E.max_tok;
    T.desc = std::move(E.desc);
    return true;
}

bool tok3_name_extents(const char *blk, uint32_t len, std::vector<uint32_t> &st,
                       std::vector<uint32_t> &ln) {
    st.clear();
    ln.clear();
    for (uint32_t i = 0, j = 0; i < len; j = ++i) {
        while (i < len && static_cast<signed char>(blk[i]) >= ' ') i++;
        if (i >= len) break;
        if (blk[i] != '\0' && blk[i] != '\n') return false;
        st.push_back(j);
        ln.push_back(i - j);
    }
    return !st.empty() && st.size() <= 10000000u;    // create_context's limits (:172-187)
}

void tok3_search_batch(GpuCtx &g, std::vector<Tok3SearchJob *> &jobs) {
    // each block up to its last terminator (the loop ignores the rest)
    std::vector<uint32_t> off;
    std::vector<Tok3SearchJob *> run;
    uint64_t nbytes = 0;
    for (Tok3SearchJob *J : jobs) {
        J->ok = false;
        J->found.clear();
        uint32_t tl = J->len;
        while (tl > 0 && J->h_blk[tl - 1] != '\0' && J->h_blk[tl - 1] != '\n') tl--;
        // (split: the section's last name must end in '\0', as name_split's
        // last id does)
        if (J->split && (tl != J->len || !J->d_blk)) continue;
        if (!tl || nbytes + tl + 64 >= (1ull << 31)) continue;
        off.push_back(uint32_t(nbytes));
        nbytes += tl;
        J->len = tl;
        run.push_back(J);
    }
    if (run.empty()) return;
    off.push_back(uint32_t(nbytes));
    // (FQZ5_STEP_TRACE: the stages' GPU time from events on the stream)
    static const bool trace = std::getenv("FQZ5_STEP_TRACE") != nullptr;
    std::vector<hipEvent_t> ev;
    auto mark = [&] {
        if (!trace) return;
        hipEvent_t e;
        FQZ5_HIP(hipEventCreate(&e));
        FQZ5_HIP(hipEventRecord(e, g.stream));
        ev.push_back(e);
    };
    const auto h0 = std::chrono::steady_clock::now();
    mark();
    const uint32_t B = uint32_t(nbytes), S = uint32_t(run.size());
    T3Batch b{};
    uint8_t *bytes = g.arena.alloc_n<uint8_t>(size_t(B) + 64);
    g.memset0(bytes + B, 64);
    for (size_t r = 0; r < run.size(); r++) {
        Tok3SearchJob &J = *run[r];
        if (J.d_blk) {
            FQZ5_HIP(hipMemcpyAsync(bytes + off[r], J.d_blk, J.len, hipMemcpyDeviceToDevice, g.stream));
        } else if (J.h_pinned) {
            FQZ5_HIP(hipMemcpyAsync(bytes + off[r], J.h_pinned, J.len, hipMemcpyHostToDevice, g.stream));
        } else {
            uint8_t *h = g.staging.alloc(J.len);
            std::memcpy(h, J.h_blk, J.len);
            FQZ5_HIP(hipMemcpyAsync(bytes + off[r], h, J.len, hipMemcpyHostToDevice, g.stream));
        }
    }
    mark();
    b.bytes = bytes;
    b.nbytes = B;
    b.nblk = S;
    b.off = g.upload(off);
    std::vector<uint8_t> split(S);
    for (size_t r = 0; r < run.size(); r++) split[r] = run[r]->split ? 1 : 0;
    b.split = g.upload(split);
    b.term = g.arena.alloc_n<uint32_t>(B);
    b.tix = g.arena.alloc_n<uint32_t>(B);
    b.bad = g.arena.alloc_n<uint32_t>(S);
    b.name0 = g.arena.alloc_n<uint32_t>(S);
    b.lset = g.arena.alloc_n<uint32_t>(size_t(S) * (T3_LSET_BITS / 32));
    g.memset0(b.bad, S * 4);
    g.memset0(b.lset, size_t(S) * (T3_LSET_BITS / 32) * 4);
    auto scan = [&](const uint32_t *in, uint32_t *out, uint32_t n) {
        size_t tb = 0;
        FQZ5_HIP(t3_scan(in, out, n, nullptr, tb, g.stream));
        void *tmp = g.arena.alloc_n<uint8_t>(tb);
        FQZ5_HIP(t3_scan(in, out, n, tmp, tb, g.stream));
    };
    auto total = [&](const uint32_t *ex, const uint32_t *in, uint32_t n) {   // ex[n-1] + in[n-1]
        uint32_t t[2];
        g.download(&t[0], ex + n - 1, 1);
        g.download(&t[1], in + n - 1, 1);
        g.sync();
        return t[0] + t[1];
    };
    FQZ5_HIP(t3_launch(b, 0, g.stream));
    scan(b.term, b.tix, B);
    const uint32_t N = total(b.tix, b.term, B);        // (the buffer ends with a terminator)
    b.nnames = N;
    b.end = g.arena.alloc_n<uint32_t>(N);
    b.st = g.arena.alloc_n<uint32_t>(N);
    b.len = g.arena.alloc_n<uint32_t>(N);
    b.sec = g.arena.alloc_n<uint32_t>(N);
    b.cnt = g.arena.alloc_n<uint32_t>(N);
    b.poff = g.arena.alloc_n<uint32_t>(N);
    FQZ5_HIP(t3_launch(b, 1, g.stream));
    FQZ5_HIP(t3_launch(b, 2, g.stream));
    scan(b.cnt, b.poff, N);
    const uint32_t P = total(b.poff, b.cnt, N);
    mark();
    b.npairs = P;
    b.key = g.arena.alloc_n<uint64_t>(P);
    b.val = g.arena.alloc_n<uint32_t>(P);
    uint64_t *skey = g.arena.alloc_n<uint64_t>(P);
    uint32_t *sval = g.arena.alloc_n<uint32_t>(P);
    b.skey = skey;
    b.sval = sval;
    b.pname = g.arena.alloc_n<uint32_t>(P);
    b.pdepth = g.arena.alloc_n<uint32_t>(P);
    b.V = g.arena.alloc_n<uint32_t>(P);
    b.fmt = g.arena.alloc_n<int4>(N);
    b.found = g.arena.alloc_n<T3Found>(N);
    FQZ5_HIP(t3_launch(b, 3, g.stream));
    mark();
    size_t tb = 0;
    FQZ5_HIP(t3_sort(b.key, skey, b.val, sval, P, nullptr, tb, g.stream));
    void *tmp = g.arena.alloc_n<uint8_t>(tb);
    FQZ5_HIP(t3_sort(b.key, skey, b.val, sval, P, tmp, tb, g.stream));
    mark();
    FQZ5_HIP(t3_launch(b, 4, g.stream));
    mark();
    std::vector<T3Found> found(N);
    std::vector<uint32_t> bad(S), name0(S);
    g.download(found.data(), b.found, N);
    g.download(bad.data(), b.bad, S);
    g.download(name0.data(), b.name0, S);
    mark();
    g.sync();
    if (trace) {
        float ms[6] = {0};
        for (size_t i = 0; i + 1 < ev.size() && i < 6; i++) FQZ5_HIP(hipEventElapsedTime(&ms[i], ev[i], ev[i + 1]));
        for (hipEvent_t e : ev) (void)hipEventDestroy(e);
        std::fprintf(stderr, "tok3 search: %u blocks, %u names, %u bytes, %u pairs: uploads %.1f, "
                     "names %.1f, pairs %.1f, sort %.1f, find %.1f, download %.1f ms; %.1f ms in all\n",
                     S, N, B, P, ms[0], ms[1], ms[2], ms[3], ms[4], ms[5],
                     std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - h0).count());
    }
    for (size_t r = 0; r < run.size(); r++) {
        if (bad[r]) continue;                           // refused, or a hash collision: the host trie
        const size_t a = name0[r], e = r + 1 < run.size() ? name0[r + 1] : N;
        run[r]->found.assign(found.begin() + long(a), found.begin() + long(e));
        run[r]->ok = true;
    }
}

void tok3_add_requests(GpuCtx &g, Tok3Enc &T, std::vector<CompressReq> &reqs) {
    const int lv = std::min(std::max((T.level - 1) / 2, 0), 4);
    T.cand.assign(size_t(T.max_tok * 16), {});
    for (int i = 0; i < T.max_tok * 16; i++) {
        const std::vector<uint8_t> &b = T.desc[size_t(i)];
        if (b.empty()) continue;
        int meth[7];
        std::memcpy(meth, METH[lv][i & 15], sizeof(meth));
        if (T.use_arith && lv == 1 && (i & 15) == N_DIGITS) meth[1] = 201;   // :1364
        const uint32_t ocap = uint32_t(1.5 * arith_compress_bound(unsigned(b.size()), 1));
        const uint8_t *d_in = T.use_arith ? nullptr : g.upload(b.data(), b.size());
        for (int m = 1; m <= meth[0]; m++) {
            int mm = meth[m];
            if (!T.use_arith && (mm & 4)) mm &= ~4;
            if (b.size() % 4 != 0 && (mm & 8)) continue;
            if (T.use_arith) {                          // coded in tok3_assemble
                T.cand[size_t(i)].push_back({mm, -1});
                continue;
            }
            CompressReq r;
            r.d_in = d_in;
            r.n = uint32_t(b.size());
            r.order = mm;
            r.cap = ocap > 6 ? ocap - 6 : 0;           // rans_encode's *out_len - 6 (:1242)
            T.cand[size_t(i)].push_back({mm, int(reqs.size())});
            reqs.push_back(std::move(r));
        }
    }
}

void download_layouts(GpuCtx &g, const std::vector<const Layout *> &ls,
                      const std::vector<uint8_t *> &dsts) {
    size_t tot = 0;
    std::vector<size_t> off(ls.size());
    for (size_t k = 0; k < ls.size(); k++) {
        off[k] = tot;
        tot += layout_size(*ls[k]);
    }
    if (!tot) return;
    uint8_t *d = g.arena.alloc_n<uint8_t>(tot);
    std::vector<uint8_t *> dd(ls.size());
    for (size_t k = 0; k < ls.size(); k++) dd[k] = d + off[k];
    write_layouts_dev(g, ls, dd);
    uint8_t *h = g.staging.alloc(tot);
    g.download(h, d, tot);
    g.sync();
    for (size_t k = 0; k < ls.size(); k++)
        std::memcpy(dsts[k], h + off[k], layout_size(*ls[k]));
}

bool tok3_assemble(GpuCtx &g, const Tok3Enc &T, const std::vector<CompressReq> &reqs,
                   std::vector<uint8_t> &out) {
    const int nd = T.max_tok * 16;
    int i, j;
    std::vector<std::vector<uint8_t>> comp(static_cast<size_t>(nd));
    if (!T.use_arith) {
        std::vector<const Layout *> ls;
        std::vector<uint8_t *> dst;
        for (i = 0; i < nd; i++) {
            if (T.desc[size_t(i)].empty()) continue;
            int best = -1;
            uint64_t best_sz = UINT64_MAX;
            for (auto &c : T.cand[size_t(i)]) {
                const CompressReq &r = reqs[size_t(c.second)];
                if (!r.ok) return false;                // rans_encode failed (:1383-1386)
                uint8_t v[8];
                const uint32_t olen = layout_size(r.out);
                const uint64_t sz = uint64_t(olen) + uint64_t(put_varint(v, olen));
                if (best_sz > sz) { best_sz = sz; best = c.second; }
            }
            if (best < 0) return false;
            const uint32_t olen = layout_size(reqs[size_t(best)].out);
            std::vector<uint8_t> &o = comp[size_t(i)];
            o.resize(8 + size_t(olen));
            const int nb = put_varint(o.data(), olen);
            o.resize(size_t(nb) + olen);
            ls.push_back(&reqs[size_t(best)].out);
            dst.push_back(o.data() + nb);
        }
        download_layouts(g, ls, dst);
    } else {
        for (i = 0; i < nd; i++) {
            const std::vector<uint8_t> &b = T.desc[size_t(i)];
            if (b.empty()) continue;
            uint64_t best_sz = UINT64_MAX;
            const uint32_t ocap = uint32_t(1.5 * arith_compress_bound(unsigned(b.size()), 1));
            std::vector<uint8_t> o(ocap + 8);
            std::vector<uint8_t> in(b);
            for (auto &c : T.cand[size_t(i)]) {          // arith_encode (:1214-1224)
                unsigned olen = ocap - 6;
                if (!arith_compress_to(in.data(), unsigned(in.size()), o.data() + 6, &olen, c.first))
                    return false;
                uint8_t v[8];
                const int nb = put_varint(v, olen);
                if (best_sz > uint64_t(olen) + uint64_t(nb)) {
                    best_sz = uint64_t(olen) + uint64_t(nb);
                    comp[size_t(i)].assign(v, v + nb);
                    comp[size_t(i)].insert(comp[size_t(i)].end(), o.data() + 6, o.data() + 6 + olen);
                }
            }
        }
    }
    // serialise, with streams equal to an earlier one as references (:1559-1657)
    uint32_t tot = 9;
    std::vector<int> dup(size_t(nd), -1);
    for (i = 0; i < nd; i++) {
        if (T.desc[size_t(i)].empty()) continue;
        const std::vector<uint8_t> &ci = comp[size_t(i)];
        for (j = 0; j < i; j++) {
            const std::vector<uint8_t> &cj = comp[size_t(j)];
            if (T.desc[size_t(j)].empty() || ci.size() != cj.size() || ci.size() <= 4) continue;
            if (std::memcmp(ci.data(), cj.data(), ci.size()) == 0) break;
        }
        if (j < i) { dup[size_t(i)] = j; tot += 3; }
        else tot += uint32_t(ci.size()) + 1;
    }
    out.resize(tot);
    uint8_t *cp = out.data();
    for (int k = 0; k < 4; k++) *cp++ = uint8_t(uint32_t(T.last_start) >> (8 * k));
    for (int k = 0; k < 4; k++) *cp++ = uint8_t(uint32_t(T.nreads) >> (8 * k));
    *cp++ = uint8_t(T.use_arith);
    int last_tnum = -1;
    for (i = 0; i < nd; i++) {
        if (T.desc[size_t(i)].empty()) continue;
        uint8_t t8 = uint8_t(i & 15);
        if ((i >> 4) != last_tnum) { t8 |= 128; last_tnum = i >> 4; }
        if (dup[size_t(i)] >= 0) {
            *cp++ = t8 | 64;
            *cp++ = uint8_t(dup[size_t(i)] >> 4);
            *cp++ = uint8_t(dup[size_t(i)] & 15);
        } else {
            *cp++ = t8;
            std::memcpy(cp, comp[size_t(i)].data(), comp[size_t(i)].size());
            cp += comp[size_t(i)].size();
        }
    }
    return true;
}

bool tok3_dec_parse(const uint8_t *in, uint32_t sz, Tok3Dec &D) {
    D = Tok3Dec();
    if (sz < 9) return false;
    D.in = in;
    D.sz = sz;
    D.ulen0 = int(uint32_t(in[0]) | uint32_t(in[1]) << 8 | uint32_t(in[2]) << 16 |
                  uint32_t(in[3]) << 24);
    if (D.ulen0 < 0 || D.ulen0 >= INT_MAX - 1024) return false;
    D.nreads = int(uint32_t(in[4]) | uint32_t(in[5]) << 8 | uint32_t(in[6]) << 16 |
                   uint32_t(in[7]) << 24);
    D.use_arith = in[8];
    if (D.nreads <= 0 || D.nreads > 10000000) return false;   // create_context (:172-187)
    // the streams in order: coded, copies of earlier ones, and elided type
    // streams regenerated from the first type of the column (:1704-1809)
    int tnum = -1;
    uint32_t o = 9;
    while (o < sz) {
        const uint8_t tt = in[o++];
        if (tt & 64) {
            if (o + 2 > sz) return false;
            int j = in[o++] << 4;
            j += in[o++];
            if (tt & 128) {
                if (++tnum >= MAX_TOKENS) return false;
                D.max_tok = tnum + 1;
            }
            if ((tt & 15) != 0 && (tt & 128)) {
                if (tnum < 0) return false;
                D.order.push_back({2, tnum << 4 | (tt & 15)});
            }
            if (tnum < 0) return false;
            const int i = (tnum << 4) | (tt & 15);
            if (j >= i) return false;
            D.copies.push_back({i, j});
            D.order.push_back({1, int(D.copies.size()) - 1});
            continue;
        }
        if (tt & 128) {
            if (++tnum >= MAX_TOKENS) return false;
            D.max_tok = tnum + 1;
        }
        if ((tt & 15) != 0 && (tt & 128)) {
            if (tnum < 0) return false;
            D.order.push_back({2, tnum << 4 | (tt & 15)});
        }
        // uncompressed_size (:1419-1429): varint clen, then the codec's order
        // byte and its varint size
        uint32_t clen = 0, ul = 0;
        const int nb = varint_get(in + o, in + sz, &clen);
        if (!nb || o + uint32_t(nb) + 1 > sz) return false;
        if (!varint_get(in + o + nb + 1, in + sz, &ul)) return false;
        if (tnum < 0 || ul >= uint32_t(INT_MAX)) return false;
        const int i = (tnum << 4) | (tt & 15);
        // the codec sees the rest of the block (:1792); clen only advances
        D.coded.push_back({i, o + uint32_t(nb), sz - o - uint32_t(nb), ul});
        D.order.push_back({0, int(D.coded.size()) - 1});
        if (uint64_t(o) + uint64_t(nb) + clen >= sz) break;
        o += uint32_t(nb) + clen;
    }
    return true;
}

void tok3_dec_add_requests(GpuCtx &g, Tok3Dec &D, const uint8_t *d_in,
                           std::vector<DecompressReq> &reqs) {
    D.req0 = reqs.size();
    if (D.use_arith || D.coded.empty()) return;
    if (!d_in) d_in = g.upload(D.in, D.sz);
    D.out_off.resize(D.coded.size());
    D.out_tot = 0;
    for (size_t k = 0; k < D.coded.size(); k++) {
        D.out_off[k] = D.out_tot;
        D.out_tot += size_t(D.coded[k].ulen) + 1;
    }
    D.d_out = g.arena.alloc_n<uint8_t>(D.out_tot);
    for (size_t k = 0; k < D.coded.size(); k++) {
        const Tok3Dec::Coded &c = D.coded[k];
        DecompressReq r;
        r.h_in = D.in + c.off;
        r.d_in = d_in + c.off;
        r.in_size = c.clen;
        r.out_cap = c.ulen;
        r.d_out = D.d_out + D.out_off[k];
        reqs.push_back(r);
    }
}

bool tok3_dec_fetch(GpuCtx &g, Tok3Dec &D, const std::vector<DecompressReq> &reqs) {
    D.fetched = false;
    D.dec.assign(D.coded.size(), {});
    std::vector<std::vector<uint8_t>> &dec = D.dec;
    if (!D.use_arith) {
        for (size_t k = 0; k < D.coded.size(); k++) {
            const DecompressReq &r = reqs[D.req0 + k];
            if (!r.ok || r.out_size != D.coded[k].ulen) return false;
        }
        if (D.out_tot) {
            uint8_t *h = g.staging.alloc(D.out_tot);
            g.download(h, D.d_out, D.out_tot);
            g.sync();
            for (size_t k = 0; k < D.coded.size(); k++)
                dec[k].assign(h + D.out_off[k], h + D.out_off[k] + D.coded[k].ulen);
        }
    } else {
        for (size_t k = 0; k < D.coded.size(); k++) {
            unsigned ol = D.coded[k].ulen;
            dec[k].resize(size_t(ol) + 1);
            if (!arith_uncompress_to(const_cast<uint8_t *>(D.in) + D.coded[k].off, D.coded[k].clen,
                                     dec[k].data(), &ol) ||
                ol != D.coded[k].ulen)
                return false;
            dec[k].resize(ol);
        }
    }
    D.fetched = true;
    return true;
}

bool tok3_dec_finish(GpuCtx &g, Tok3Dec &D, const std::vector<DecompressReq> &reqs,
                     std::vector<uint8_t> &out) {
    return tok3_dec_fetch(g, D, reqs) && tok3_dec_rebuild(D, out);
}

bool tok3_dec_rebuild(Tok3Dec &D, std::vector<uint8_t> &out) {
    if (!D.fetched) return false;
    struct Desc { std::vector<uint8_t> buf; size_t l = 0; bool have = false; };
    std::vector<Desc> desc(MAX_TBLOCKS);
    const int nreads = D.nreads, max_tok = D.max_tok;
    std::vector<std::vector<uint8_t>> &dec = D.dec;
    for (auto &e : D.order) {                          // in stream order, as the reference
        if (e.first == 2) {                            // an elided type stream: ty then MATCH
            Desc &c = desc[size_t(e.second & ~15)];
            c.buf.assign(size_t(nreads), uint8_t(N_MATCH));
            c.buf[0] = uint8_t(e.second & 15);
            c.have = true;
            c.l = 0;
        } else if (e.first == 1) {
            const auto &c = D.copies[size_t(e.second)];
            if (!desc[size_t(c.second)].have) return false;
            desc[size_t(c.first)].buf = desc[size_t(c.second)].buf;
            desc[size_t(c.first)].have = true;
            desc[size_t(c.first)].l = 0;
        } else {
            const Tok3Dec::Coded &c = D.coded[size_t(e.second)];
            desc[size_t(c.i)].buf = std::move(dec[size_t(e.second)]);
            desc[size_t(c.i)].have = true;
            desc[size_t(c.i)].l = 0;
        }
    }
    using D_ = Desc;
    // decode_name per name (:1023-1212)
    auto dtype = [&](int ntok) -> int {
        D_ &d = desc[size_t(ntok << 4)];
        if (d.l >= d.buf.size()) return -1;
        return d.buf[d.l++];
    };
    auto dint = [&](int ntok, int ty, uint32_t *v) -> bool {
        D_ &d = desc[size_t(ntok << 4 | ty)];
        if (d.l + 4 > d.buf.size()) return false;
        const uint8_t *p = d.buf.data() + d.l;
        *v = uint32_t(p[0]) | uint32_t(p[1]) << 8 | uint32_t(p[2]) << 16 | uint32_t(p[3]) << 24;
        d.l += 4;
        return true;
    };
    auto dint1 = [&](int ntok, int ty, uint32_t *v) -> bool {
        D_ &d = desc[size_t(ntok << 4 | ty)];
        if (d.l >= d.buf.size()) return false;
        *v = d.buf[d.l++];
        return true;
    };
    auto fixed = [](char *cp, uint32_t v, uint8_t l) -> int {   // append_uint32_fixed (:233)
        if (l <= 9) {
            uint32_t p = 1;
            for (int k = 1; k < l; k++) p *= 10;
            for (; p; p /= 10) { *cp++ = char(v / p + '0'); v %= p; }
        }
        return l;
    };
    auto var = [](char *cp, uint32_t v) {              // append_uint32_var (v = 0 writes nothing)
        char t[12];
        int n = 0;
        while (v) { t[n++] = char('0' + v % 10); v /= 10; }
        for (int k = 0; k < n; k++) cp[k] = t[n - 1 - k];
        return n;
    };
    int64_t ulen = int64_t(D.ulen0) + 1024;
    // the names go straight into `out` (no second buffer and copy)
    out.assign(static_cast<size_t>(ulen), 0);
    char *outb = reinterpret_cast<char *>(out.data());
    std::vector<Last> lc(size_t(nreads) + 1);          // max_names = nreads + 1 (:190)
    std::vector<Tok> toks;
    size_t osz = 0;
    int counter = 0, ret = 0;
    for (;;) {
        char *nm = outb + osz;
        const int64_t nlen = ulen;
        ret = -1;
        const int cnum = counter++;
        if (cnum > nreads) { ret = -1; break; }
        const int t0 = dtype(0);
        if (t0 < 0 || t0 >= max_tok * 16) { ret = 0; break; }
        uint32_t dist;
        if (!dint(0, t0, &dist) || int64_t(dist) > cnum) break;
        int pnum = cnum - int(dist);
        if (pnum < 0) pnum = 0;
        Last &C = lc[size_t(cnum)];
        const Last &P = lc[size_t(pnum)];
        if (t0 == N_DUP) {
            if (pnum == cnum) break;
            const size_t pl = std::strlen(P.name);
            if (int64_t(pl) + 1 >= nlen) break;
            std::memcpy(nm, P.name, pl + 1);
            C.name = nm;
            C.ntok = P.ntok;
            C.off = P.off;
            ret = int(pl) + 1;
        } else {
            *nm = 0;
            int64_t len = 0;
            C.off = uint32_t(toks.size());
            int ntok;
            bool done = false, bad = false;
            for (ntok = 1; ntok < MAX_TOKENS && ntok < max_tok && !done && !bad; ntok++) {
                uint32_t v, vl;
                const int tok = dtype(ntok);
                C.ntok = 0;
                if (toks.size() < size_t(C.off) + size_t(ntok) + 1)
                    toks.resize(size_t(C.off) + size_t(ntok) + 1);
                Tok &T = toks[size_t(C.off) + size_t(ntok)];
                const Tok *pt = ntok < P.ntok ? &toks[size_t(P.off) + size_t(ntok)] : nullptr;
                switch (tok) {
                case N_CHAR:
                    if (len + 1 >= nlen || !dint1(ntok, N_CHAR, &v)) { bad = true; break; }
                    nm[len] = char(v);
                    T.type = N_CHAR;
                    T.ival = nm[len++];
                    break;
                case N_ALPHA: {
                    D_ &d = desc[size_t(ntok << 4 | N_ALPHA)];
                    if (d.l >= d.buf.size()) { bad = true; break; }
                    int64_t l2 = 0;
                    char c;
                    const int64_t maxl = nlen - len;
                    do {
                        c = char(d.buf[d.l++]);
                        nm[len + l2++] = c;
                    } while (c && l2 < maxl && d.l < d.buf.size());
                    T.type = N_ALPHA;
                    T.sval = int(len);
                    T.ival = int(l2 - 1);
                    len += l2 - 1;
                    break;
                }
                case N_DIGITS0:
                    if (!dint1(ntok, N_DZLEN, &vl) || !dint(ntok, N_DIGITS0, &v)) { bad = true; break; }
                    if (len + 20 + int64_t(vl) >= nlen) { bad = true; break; }
                    len += fixed(nm + len, v, uint8_t(vl));
                    T = {N_DIGITS0, int(v), int(vl)};
                    break;
                case N_DDELTA0:
                    if (!pt || !dint1(ntok, N_DDELTA0, &v)) { bad = true; break; }
                    v += uint32_t(pt->ival);
                    if (len + pt->sval + 1 >= nlen) { bad = true; break; }
                    len += fixed(nm + len, v, uint8_t(pt->sval));
                    T = {N_DIGITS0, int(v), pt->sval};
                    break;
                case N_DIGITS:
                    if (!dint(ntok, N_DIGITS, &v) || len + 20 >= nlen) { bad = true; break; }
                    len += var(nm + len, v);
                    T.type = N_DIGITS;
                    T.ival = int(v);
                    break;
                case N_DDELTA:
                    if (!pt || !dint1(ntok, N_DDELTA, &v)) { bad = true; break; }
                    v += uint32_t(pt->ival);
                    if (len + 20 >= nlen) { bad = true; break; }
                    len += var(nm + len, v);
                    T.type = N_DIGITS;
                    T.ival = int(v);
                    break;
                case N_NOP:
                    T.type = N_NOP;
                    break;
                case N_MATCH:
                    if (!pt) { bad = true; break; }
                    switch (pt->type) {
                    case N_CHAR:
                        if (len + 1 >= nlen) { bad = true; break; }
                        nm[len++] = char(pt->ival);
                        T.type = N_CHAR;
                        T.ival = pt->ival;
                        break;
                    case N_ALPHA:
                        if (pt->ival < 0 || len + pt->ival >= nlen) { bad = true; break; }
                        std::memcpy(nm + len, P.name + pt->sval, size_t(pt->ival));
                        T = {N_ALPHA, pt->ival, int(len)};
                        len += pt->ival;
                        break;
                    case N_DIGITS:
                        if (len + 20 >= nlen) { bad = true; break; }
                        len += var(nm + len, uint32_t(pt->ival));
                        T.type = N_DIGITS;
                        T.ival = pt->ival;
                        break;
                    case N_DIGITS0:
                        if (len + pt->sval >= nlen) { bad = true; break; }
                        len += fixed(nm + len, uint32_t(pt->ival), uint8_t(pt->sval));
                        T = {N_DIGITS0, pt->ival, pt->sval};
                        break;
                    default:
                        bad = true;
                    }
                    break;
                default:                                // an elided N_END
                case N_END:
                    if (len + 1 >= nlen) { bad = true; break; }
                    nm[len++] = 0;
                    T.type = N_END;
                    C.name = nm;
                    C.ntok = ntok;
                    done = true;
                    ret = int(len);
                    break;
                }
            }
            if (!done) ret = -1;
        }
        if (ret <= 0) break;
        osz += size_t(ret);
        ulen -= ret;
    }
    if (ret < 0) return false;
    out.resize(osz);
    return true;
}

}  // namespace fqz5

using namespace fqz5;

extern "C" {

// Host stage only (no GPU call): tokenise a copy of `blk` and return the
// bytes of its token streams, -1 where tok3_encode_names returns NULL.  For
// timing the tokeniser (tools/tok3_time.py).
long long fqz5_tok3_tokenise_bytes(const char *blk, int len, int level) {
    std::vector<char> b(blk, blk + std::max(len, 0));
    Tok3Enc T;
    if (!tok3_tokenise(b.data(), len, level, 0, T)) return -1;
    long long tot = 0;
    for (auto &d : T.desc) tot += (long long)d.size();
    return tot;
}

// Host stage only: FNV-1a of every token stream (index, size, bytes) of
// `blk`, for CPU regression tests of the tokeniser; 0 on failure.
unsigned long long fqz5_tok3_tokenise_digest_mode(const char *blk, int len, int level, int pipelined);
unsigned long long fqz5_tok3_tokenise_digest(const char *blk, int len, int level) {
    return fqz5_tok3_tokenise_digest_mode(blk, len, level, 0);
}
// (tests: pipelined 1 runs the trie searches on a second thread)
unsigned long long fqz5_tok3_tokenise_digest_mode(const char *blk, int len, int level, int pipelined) {
    std::vector<char> b(blk, blk + std::max(len, 0));
    Tok3Enc T;
    if (!tok3_tokenise(b.data(), len, level, 0, T, pipelined != 0)) return 0;
    uint64_t h = 1469598103934665603ull;
    auto mix = [&](uint8_t v) { h = (h ^ v) * 1099511628211ull; };
    for (size_t i = 0; i < T.desc.size(); i++) {
        const auto &d = T.desc[i];
        if (d.empty()) continue;
        for (int k = 0; k < 4; k++) mix(uint8_t(i >> (8 * k)));
        for (int k = 0; k < 4; k++) mix(uint8_t(d.size() >> (8 * k)));
        for (uint8_t v : d) mix(v);
    }
    mix(uint8_t(T.max_tok));
    return h;
}

uint8_t *tok3_encode_names(char *blk, int len, int level, int use_arith, int *out_len,
                           int *last_start_p) {
    fqz5::CallTrace ct("tok3_encode_names", size_t(len > 0 ? len : 0));
    if (len < 0) {
        *out_len = 0;
        return nullptr;
    }
    GpuCtx *gp = nullptr;
    GUARD_BEGIN
    Tok3Enc T;
    const bool ok = tok3_tokenise(blk, len, level, use_arith, T);
    ct.mark("tok");
    if (last_start_p && T.last_start >= 0) *last_start_p = T.last_start;
    if (!ok) return nullptr;
    GpuCtx &g = gpu();
    gp = &g;
    std::vector<CompressReq> reqs;
    tok3_add_requests(g, T, reqs);
    if (!reqs.empty()) compress_batch(g, reqs);
    if (ct.k) { g.sync(); ct.mark("run"); }
    std::vector<uint8_t> o;
    const bool good = tok3_assemble(g, T, reqs, o);
    g.reset();
    if (!good) return nullptr;
    uint8_t *out = static_cast<uint8_t *>(malloc(o.size() + 13));
    if (!out) return nullptr;
    std::memcpy(out, o.data(), o.size());
    *out_len = int(o.size());
    return out;
    GUARD_END((gp ? (void)gp->reset() : (void)0, nullptr))
}

uint8_t *tok3_decode_names(uint8_t *in, uint32_t sz, uint32_t *out_len) {
    fqz5::CallTrace ct("tok3_decode_names", sz);
    GpuCtx *gp = nullptr;
    GUARD_BEGIN
    Tok3Dec D;
    if (!tok3_dec_parse(in, sz, D)) return nullptr;
    GpuCtx &g = gpu();
    gp = &g;
    ct.mark("ctx");
    std::vector<DecompressReq> reqs;
    tok3_dec_add_requests(g, D, nullptr, reqs);
    if (!reqs.empty()) decompress_batch(g, reqs);
    if (ct.k) { g.sync(); ct.mark("run"); }
    std::vector<uint8_t> o;
    const bool good = tok3_dec_finish(g, D, reqs, o);
    g.reset();
    if (!good) return nullptr;
    uint8_t *out = static_cast<uint8_t *>(malloc(std::max<size_t>(o.size(), 1)));
    if (!out) return nullptr;
    std::memcpy(out, o.data(), o.size());
    *out_len = uint32_t(o.size());
    return out;
    GUARD_END((gp ? (void)gp->reset() : (void)0, nullptr))
}

// (tests) the GPU batch search against the host trie on `nblk` blocks back
// to back (lens[i] bytes each): mismatching names, or -1 - i when block i's
// GPU search was refused or failed its checks.  split: the blocks are name
// sections, searched in split mode against the host trie over name_split's
// read ids.
long long fqz5_tok3_search_check(const char *blks, const uint32_t *lens, int nblk, int split) {
    GUARD_BEGIN
    GpuCtx &g = gpu();
    std::vector<std::vector<char>> copy(size_t(std::max(nblk, 0)));
    std::vector<Tok3SearchJob> jobs(copy.size());
    std::vector<Tok3SearchJob *> jp;
    size_t off = 0;
    for (size_t i = 0; i < copy.size(); i++) {
        copy[i].assign(blks + off, blks + off + lens[i]);
        off += lens[i];
        jobs[i].h_blk = copy[i].data();
        jobs[i].len = lens[i];
        jobs[i].split = split != 0;
        if (split) jobs[i].d_blk = g.upload(reinterpret_cast<const uint8_t *>(copy[i].data()), lens[i]);
        jp.push_back(&jobs[i]);
    }
    tok3_search_batch(g, jp);
    g.reset();
    long long bad = 0;
    for (size_t i = 0; i < copy.size(); i++) {
        if (!jobs[i].ok) return -1 - (long long)i;
        std::vector<char> ids = copy[i];
        if (split) {
            NameEnc E;
            name_split(reinterpret_cast<const uint8_t *>(copy[i].data()), lens[i], 2, 3, E);
            ids = E.ids;
        }
        std::vector<uint32_t> st, ln;
        if (!tok3_name_extents(ids.data(), uint32_t(ids.size()), st, ln)) return -1 - (long long)i;
        if (st.size() != jobs[i].found.size()) return -1000 - (long long)i;
        Trie t;
        for (size_t k = 0; k < st.size(); k++) {
            char *nm = ids.data() + st[k];
            nm[ln[k]] = '\0';
            Found f;
            f.pnum = t.search(nm, ln[k], uint32_t(k), &f.exact, &f.is_fixed, &f.fixed_len);
            const T3Found &G = jobs[i].found[k];
            bad += (f.pnum != G.pnum || f.exact != G.exact || f.is_fixed != G.is_fixed ||
                    f.fixed_len != G.fixed_len);
        }
    }
    return bad;
    GUARD_END(-1000000)
}

}  // extern "C"
