// chain_probe.hip — cycle breakdown (s_memtime) of the encoder chain kernel
// on one synthetic O0 stream: staging vs chain per chunk.  Builds the
// library's kernel source with FQZ5_CHAIN_PROBE.
#define FQZ5_CHAIN_PROBE 1
#include "../fqzcomp5_amd/csrc/rans_chain.hip"
#include <cstdio>
#include <vector>
#include <random>

using namespace fqz5;

int main(int argc, char **argv) {
    const uint32_t n = argc > 1 ? uint32_t(atoi(argv[1])) : 43500000u;
    std::vector<uint8_t> in(n);
    std::mt19937 rng(1);
    const char al[5] = {'A', 'C', 'G', 'T', 'N'};
    for (auto &b : in) { uint32_t r = rng() % 1000; b = al[r < 5 ? 4 : r % 4]; }
    uint32_t F[256] = {0};
    F['A'] = 1020; F['C'] = 1020; F['G'] = 1020; F['T'] = 1030; F['N'] = 6;
    std::vector<EncSym> tab(256);
    uint32_t st = 0;
    for (int s = 0; s < 256; s++) { if (F[s]) tab[s] = make_encsym(st, F[s], 12); st += F[s]; }
    const uint32_t T = (n + 3) / 4, S = enc_chunk_steps(4), nch = (T + S - 1) / S;
    uint8_t *d_in, *d_out; EncSym *d_tab; uint32_t *d_ck, *d_cnt, *d_len; EncJob *d_job;
    (void)hipMalloc(&d_in, n); (void)hipMalloc(&d_out, 2 * size_t(n) + 4096);
    (void)hipMalloc(&d_tab, 256 * 16); (void)hipMalloc(&d_ck, (nch + 1) * 16);
    (void)hipMalloc(&d_cnt, nch * 4); (void)hipMalloc(&d_len, 4); (void)hipMalloc(&d_job, sizeof(EncJob));
    (void)hipMemcpy(d_in, in.data(), n, hipMemcpyHostToDevice);
    (void)hipMemcpy(d_tab, tab.data(), 256 * 16, hipMemcpyHostToDevice);
    EncJob J{d_in, d_tab, nullptr, d_out + 2 * size_t(n) + 2048, d_len, d_ck, d_cnt, n, 4, 12, 0, nch};
    (void)hipMemcpy(d_job, &J, sizeof J, hipMemcpyHostToDevice);
    for (int rep = 0; rep < 2; rep++) {
        uint64_t z[8] = {0};
        (void)hipMemcpyToSymbol(HIP_SYMBOL(g_probe), z, sizeof z);
        hipEvent_t a, b; (void)hipEventCreate(&a); (void)hipEventCreate(&b);
        (void)hipEventRecord(a);
        (void)launch_enc_chain(d_job, 1, enc_lds_bytes(0, 0), 0);
        (void)hipEventRecord(b); (void)hipEventSynchronize(b);
        float ms; (void)hipEventElapsedTime(&ms, a, b);
        (void)hipMemcpyFromSymbol(z, HIP_SYMBOL(g_probe), sizeof z);
        printf("n=%u steps=%u  %.2f ms  %.2f ns/step  stage %.1f cyc/step  chain %.1f cyc/step\n",
               n, T, ms, ms * 1e6 / T, double(z[0]) / T, double(z[1]) / T);
    }
    return 0;
}
