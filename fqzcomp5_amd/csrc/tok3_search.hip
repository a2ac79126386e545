// tok3_search.hip — the trie search of the tok3 tokeniser (search_trie,
// tokenise_name3.c:591-695; the host form is Trie::search in tok3.cpp) for
// every name of a batch of name blocks at once.
//
// The trie leaves at each node the number of the last name that walked
// through it, so what a name reads at depth d of its walk is
//   V(n, d) = the last earlier name m < n whose first d bytes are n's
// (or n itself when there is none).  The search then returns
//   exact       V(n, L) != n                    (L = n's length > 0)
//   from        V(n, L)
//   p3          V(n, P)                          (name_format's prefix P <= L)
//   from_punct  V(n, p + 1) for the last punctuation / space byte p of n
//               with V(n, p + 1) != n
//   -> exact ? from : p3 != -1 ? p3 : from_punct
// Only these depths are read, so a name m enters pairs (hash of its first d
// bytes, m) at the depths another name could read in it: its punctuation
// depths (a name sharing m's first d bytes has the same punctuation there),
// the lengths of the block's names (exact), the fixed prefixes 6, 36, 60 of
// name_format (its Illumina prefix ends at a ':'), and its own length.  A
// stable sort by hash puts the pairs of equal prefixes together in name
// order, so V(n, d) is the pair sorted just before n's pair at depth d, when
// its hash is the same.  A hash can collide, never miss: every V the result
// uses is checked byte for byte, and a block with a failed check goes back
// to the host trie (tok3_search_batch in tok3.cpp).
//
// The blocks lie back to back, each cut after its last terminator (the
// tokenise loop ignores what follows it), so the names are the runs before
// each '\0' / '\n' of the whole buffer.  A block in split mode is a name
// section ('\0' after each name) whose read ids are what is tokenised
// (fqzcomp5's TOK3_n_LZP, fqzcomp5.c:1462-1515, names.cpp name_split): each
// name's walk is its id, a prefix of it, so the section itself is searched
// and no id block is built or uploaded.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include "tok3_search.h"

namespace fqz5 {

namespace {
__device__ __forceinline__ uint64_t mix64(uint64_t z) {      // splitmix64's finaliser
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
    return z ^ (z >> 31);
}
__device__ __forceinline__ bool c_alpha(uint8_t c) { return uint8_t((c | 32) - 'a') < 26; }
__device__ __forceinline__ bool c_digit(uint8_t c) { return uint8_t(c - '0') < 10; }
__device__ __forceinline__ bool c_xdigit(uint8_t c) { return c_digit(c) || uint8_t((c | 32) - 'a') < 6; }
__device__ __forceinline__ bool c_space(uint8_t c) { return c == ' ' || uint8_t(c - 9) < 5; }
__device__ __forceinline__ bool c_punct(uint8_t c) { return c > 32 && c < 127 && !c_alpha(c) && !c_digit(c); }
__device__ __forceinline__ bool ps(uint8_t c) { return c_punct(c) || c_space(c); }

// name_format (tok3.cpp, tokenise_name3.c:600-644): prefix_len, and the
// fixed leading token
__device__ int name_format(const uint8_t *data, uint32_t len, int *is_fixed, int *fixed_len) {
    *fixed_len = 0;
    *is_fixed = 0;
    const uint8_t *d = data[0] == '@' ? data + 1 : data;
    const int l = data[0] == '@' ? int(len) - 1 : int(len);
    const int f = data[0] == '>' ? 1 : 0;
    if (l > 70 && d[f + 0] == 'm' && d[7] == '_' && d[f + 14] == '_' && d[f + 61] == '/')
        return 60;
    if (l == 17 && d[f + 5] == ':' && d[f + 11] == ':') {
        *fixed_len = 6;
        *is_fixed = 1;
        return 6;
    }
    if (l >= 36 && d[f + 8] == '-' && d[f + 13] == '-' && d[f + 18] == '-' && d[f + 23] == '-' &&
        c_xdigit(d[f + 0]) && c_xdigit(d[f + 7]) && c_xdigit(d[f + 9]) && c_xdigit(d[f + 12]) &&
        c_xdigit(d[f + 14]) && c_xdigit(d[f + 17]) && c_xdigit(d[f + 19]) && c_xdigit(d[f + 22]) &&
        c_xdigit(d[f + 24]) && c_xdigit(d[f + 35])) {
        *fixed_len = 36;
        *is_fixed = 1;
        return 36;
    }
    int colons = 0;
    uint32_t i = 0;
    for (i = 0; i < len && data[i] > ' '; i++) {}
    while (i > 0 && colons < 4)
        if (data[--i] == ':') colons++;
    if (colons == 4) {
        *fixed_len = int(i) + 1;
        *is_fixed = 1;
        return int(i) + 1;
    }
    return 0x7fffffff;
}

__device__ __forceinline__ uint32_t block_of(const T3Batch &B, uint32_t p) {   // byte -> block
    uint32_t lo = 0, hi = B.nblk;                       // off[lo] <= p < off[hi]
    while (hi - lo > 1) {
        const uint32_t m = (lo + hi) / 2;
        if (B.off[m] <= p) lo = m;
        else hi = m;
    }
    return lo;
}

__global__ void k_t3_bytes(T3Batch B) {                 // terminators, refused bytes
    const uint32_t p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= B.nbytes) return;
    const uint8_t c = B.bytes[p];
    const uint32_t s = block_of(B, p);
    if (B.split[s]) {
        // ids: a '\n' would end an id mid-name (the host split handles
        // that); other refused bytes are checked per id (k_t3_names)
        B.term[p] = c == 0;
        if (c == '\n') B.bad[s] = 1u;
        return;
    }
    const bool term = c == 0 || c == '\n';
    B.term[p] = term;
    if (!term && (c < 0x20 || c >= 0x80)) B.bad[s] = 1u;
}

__global__ void k_t3_ends(T3Batch B) {                  // name k ends at its terminator
    const uint32_t p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p < B.nbytes && B.term[p]) B.end[B.tix[p]] = p;
}

__global__ void k_t3_blocks(T3Batch B) {                // each block's first name
    const uint32_t s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s < B.nblk) B.name0[s] = B.tix[B.off[s]];
}

__device__ __forceinline__ uint32_t name_block(const T3Batch &B, uint32_t k) {
    uint32_t lo = 0, hi = B.nblk;
    while (hi - lo > 1) {
        const uint32_t m = (lo + hi) / 2;
        if (B.name0[m] <= k) lo = m;
        else hi = m;
    }
    return lo;
}

// per name: its extent and block, the block's length set.  Split mode: the
// read id, as name_split cuts it: up to the first space or tab (a space at
// the block's first byte does not count, :1471), less a "/1" or "/2" (the
// bytes before an id are a terminator, never '/')
__global__ void k_t3_names(T3Batch B) {
    const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= B.nnames) return;
    const uint32_t st = k ? B.end[k - 1] + 1 : 0, e = B.end[k], s = name_block(B, k);
    uint32_t L = e - st;
    if (B.split[s]) {
        const uint32_t o = B.off[s];                   // absolute positions in the block
        uint32_t w1 = e;
        for (uint32_t j = st; j < e; j++) {
            const uint8_t c = B.bytes[j];
            if (c == ' ' || c == '\t') { w1 = j; break; }
        }
        if (w1 == o) w1 = e;
        if (w1 - o > 1 && B.bytes[w1 - 2] == '/' && (B.bytes[w1 - 1] == '1' || B.bytes[w1 - 1] == '2'))
            w1 -= 2;
        L = w1 - st;
        for (uint32_t j = st; j < w1; j++) {
            const uint8_t c = B.bytes[j];
            if (c < 0x20 || c >= 0x80) { B.bad[s] = 1u; break; }
        }
    }
    B.st[k] = st;
    B.len[k] = L;
    B.sec[k] = s;
    // the length set: most names of a block share a few lengths, so the bit
    // is read first and set only when it is still clear (one atomic per new
    // length, not one per name on the same word: -5 NovaSeq, ~24 ms a launch)
    if (L < T3_LSET_BITS) {
        uint32_t *w = &B.lset[s * (T3_LSET_BITS / 32) + L / 32];
        const uint32_t bit = 1u << (L % 32);
        if (!(__hip_atomic_load(w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) & bit)) atomicOr(w, bit);
    }
}

// the depths at which name k enters a pair (its walk has L bytes)
// (c: the name's byte d - 1)
__device__ __forceinline__ bool t3_depth(const T3Batch &B, const uint32_t *lset, uint8_t c,
                                         uint32_t d, uint32_t L) {
    return d == L || ps(c) || d == 6 || d == 36 || d == 60 || d >= T3_LSET_BITS ||
           ((lset[d / 32] >> (d % 32)) & 1u);
}

__global__ void k_t3_count(T3Batch B) {
    const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= B.nnames) return;
    const uint32_t st = B.st[k], L = B.len[k];
    const uint32_t *lset = B.lset + B.sec[k] * (T3_LSET_BITS / 32);
    const uint8_t *s = B.bytes + st;
    uint32_t c = 0;
    for (uint32_t d = 1; d <= L; d++) c += t3_depth(B, lset, s[d - 1], d, L);
    B.cnt[k] = c;
}

// per name: its pairs (key, pair number) in depth order, each pair's name
// and depth; name_format's results.  A wave takes 64 names, whose pairs are
// one contiguous range; per window of T3W pairs each lane walks its own name
// (the prefix hash is serial) into LDS and the wave writes the window out
// as whole lines.  The walks read the names' bytes from an LDS copy of the
// wave's first T3NB bytes (the names lie back to back), past it from HBM.
// (Round 6: one thread per name writing its own pairs made every store touch
// 64 lines: 14.4 GB of HBM traffic in the -5 NovaSeq dispatch, 11.4 GB of it
// writes, profiles/r06_pmc_l5.json.)
constexpr uint32_t T3W = 1024, T3NB = 4096;
__global__ __launch_bounds__(64) void k_t3_pairs(T3Batch B) {
    __shared__ uint64_t wkey[T3W];
    __shared__ uint32_t wdep[T3W];
    __shared__ uint8_t wln[T3W];
    __shared__ uint32_t nb32[T3NB / 4];
    const uint32_t lane = threadIdx.x;
    const uint32_t k0 = blockIdx.x * 64u;
    const uint32_t k = k0 + lane;
    const bool act = k < B.nnames;
    const uint32_t kend = min(k0 + 64u, B.nnames);
    const uint32_t Q0 = B.poff[k0];
    const uint32_t Q1 = kend < B.nnames ? B.poff[kend] : B.npairs;
    uint32_t q = act ? B.poff[k] : Q1;
    const uint32_t st = act ? B.st[k] : 0u, L = act ? B.len[k] : 0u, sec = act ? B.sec[k] : 0u;
    const uint32_t *lset = B.lset + sec * (T3_LSET_BITS / 32);
    const uint8_t *s = B.bytes + st;
    if (act) {
        int is_fixed, fixed_len;
        const int pl = name_format(s, L, &is_fixed, &fixed_len);
        B.fmt[k] = make_int4(pl, is_fixed, fixed_len, 0);
    }
    const uint32_t st0 = B.st[k0];
    for (uint32_t i = lane; i < T3NB / 4; i += 64u) {
        const uint32_t a = st0 + 4u * i;
        uint32_t v = 0;
        if (uint64_t(a) + 4 <= B.nbytes) {
            v = *reinterpret_cast<const uint32_t *>(B.bytes + a);
        } else {
            for (uint32_t j = 0; j < 4; j++)
                if (a + j < B.nbytes) v |= uint32_t(B.bytes[a + j]) << (8 * j);
        }
        nb32[i] = v;
    }
    __syncthreads();
    const uint8_t *nb = reinterpret_cast<const uint8_t *>(nb32);
    const uint32_t rel = st - st0;
    uint64_t h = 0x9e3779b97f4a7c15ull ^ (uint64_t(sec) * 0xd6e8feb86659fd93ull);
    uint32_t d = 1;
    for (uint32_t w0 = Q0; w0 < Q1; w0 += T3W) {
        const uint32_t wend = min(w0 + T3W, Q1);
        for (; q < wend && d <= L; d++) {
            const uint32_t c = rel + d - 1 < T3NB ? nb[rel + d - 1] : s[d - 1];
            h = (h + c + 1) * 0x100000001b3ull;
            h ^= h >> 29;
            if (!t3_depth(B, lset, uint8_t(c), d, L)) continue;
            wkey[q - w0] = mix64(h + uint64_t(d) * 0x9fb21c651e98df25ull) >> (64 - T3_KEY_BITS);
            wdep[q - w0] = d;
            wln[q - w0] = uint8_t(lane);
            q++;
        }
        __syncthreads();
        for (uint32_t i = lane; i < wend - w0; i += 64u) {
            const uint32_t qq = w0 + i;
            B.key[qq] = wkey[i];
            B.val[qq] = qq;
            B.pname[qq] = k0 + wln[i];
            B.pdepth[qq] = wdep[i];
        }
        __syncthreads();
    }
}

// per sorted pair: V of its (name, depth) = the name of the pair before it
// with the same key, or none
__global__ void k_t3_pred(T3Batch B) {
    const uint32_t q = blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= B.npairs) return;
    const uint64_t key = B.skey[q];
    B.V[B.sval[q]] = (q > 0 && B.skey[q - 1] == key) ? B.pname[B.sval[q - 1]] : T3_NONE;
}

// byte-for-byte: the first d bytes of names m and k are equal
__device__ bool same_prefix(const T3Batch &B, uint32_t m, uint32_t k, uint32_t d) {
    const uint32_t sm = B.st[m], sk = B.st[k];
    if (B.len[m] < d || B.len[k] < d) return false;
    const uint8_t *a = B.bytes + sm, *b = B.bytes + sk;
    for (uint32_t i = 0; i < d; i++)
        if (a[i] != b[i]) return false;
    return true;
}

// per name: search_trie's result (block-local name numbers)
__global__ void k_t3_find(T3Batch B) {
    const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= B.nnames) return;
    const uint32_t st = B.st[k], L = B.len[k], sec = B.sec[k], n0 = B.name0[sec];
    const uint32_t q0 = B.poff[k], q1 = q0 + B.cnt[k];  // its pairs, depths ascending
    const int4 fm = B.fmt[k];
    const int self = int(k - n0);
    bool ok = true;
    int from = -1, p3 = -1, from_punct = -1, exact = 0;
    if (L > 0) {                                       // the last pair is at depth L
        const uint32_t v = B.V[q1 - 1];
        exact = v != T3_NONE;
        from = exact ? int(v - n0) : self;
        // v == k: a collision of the name with itself at another depth (the
        // prefix check passes trivially there): the host trie decides
        if (exact && (v == k || !same_prefix(B, v, k, L))) ok = false;
    }
    if (!exact && fm.x >= 1 && uint32_t(fm.x) <= L) {
        uint32_t v = T3_NONE;
        bool seen = false;
        for (uint32_t q = q0; q < q1; q++)
            if (B.pdepth[q] == uint32_t(fm.x)) { v = B.V[q]; seen = true; break; }
        if (!seen) ok = false;                         // (cannot happen: P is a pair depth)
        p3 = v != T3_NONE ? int(v - n0) : self;
        if (v != T3_NONE && (v == k || !same_prefix(B, v, k, uint32_t(fm.x)))) ok = false;
    }
    if (!exact && p3 == -1) {
        const uint8_t *s = B.bytes + st;
        for (uint32_t q = q1; q-- > q0;) {
            const uint32_t d = B.pdepth[q], v = B.V[q];
            if (v == T3_NONE || !ps(s[d - 1])) continue;
            from_punct = int(v - n0);
            if (v == k || !same_prefix(B, v, k, d)) ok = false;
            break;
        }
    }
    T3Found r;
    r.pnum = exact ? from : (p3 != -1 ? p3 : from_punct);
    r.exact = exact;
    r.is_fixed = fm.y;
    r.fixed_len = fm.z;
    B.found[k] = r;
    if (!ok) B.bad[sec] = 1u;
}

dim3 grid(uint64_t n) { return dim3(unsigned((n + 255) / 256)); }
}  // namespace

hipError_t t3_scan(const uint32_t *in, uint32_t *out, uint32_t n, void *tmp, size_t &bytes,
                   hipStream_t s) {
    return hipcub::DeviceScan::ExclusiveSum(tmp, bytes, in, out, int(n), s);
}

hipError_t t3_sort(const uint64_t *k_in, uint64_t *k_out, const uint32_t *v_in, uint32_t *v_out,
                   uint32_t n, void *tmp, size_t &bytes, hipStream_t s) {
    return hipcub::DeviceRadixSort::SortPairs(tmp, bytes, k_in, k_out, v_in, v_out, int(n), 0,
                                              int(T3_KEY_BITS), s);
}

hipError_t t3_launch(const T3Batch &b, int stage, hipStream_t s) {
    switch (stage) {
    case 0:
        if (b.nbytes) hipLaunchKernelGGL(k_t3_bytes, grid(b.nbytes), dim3(256), 0, s, b);
        break;
    case 1:
        if (b.nbytes) hipLaunchKernelGGL(k_t3_ends, grid(b.nbytes), dim3(256), 0, s, b);
        if (b.nblk) hipLaunchKernelGGL(k_t3_blocks, grid(b.nblk), dim3(256), 0, s, b);
        break;
    case 2:
        if (b.nnames) {
            hipLaunchKernelGGL(k_t3_names, grid(b.nnames), dim3(256), 0, s, b);
            hipLaunchKernelGGL(k_t3_count, grid(b.nnames), dim3(256), 0, s, b);
        }
        break;
    case 3:
        if (b.nnames) hipLaunchKernelGGL(k_t3_pairs, dim3((b.nnames + 63) / 64), dim3(64), 0, s, b);
        break;
    case 4:
        if (b.npairs) hipLaunchKernelGGL(k_t3_pred, grid(b.npairs), dim3(256), 0, s, b);
        if (b.nnames) hipLaunchKernelGGL(k_t3_find, grid(b.nnames), dim3(256), 0, s, b);
        break;
    }
    return hipGetLastError();
}

}  // namespace fqz5
