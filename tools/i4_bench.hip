// tools/i4_bench.hip — latency of i4_block (jmh_i4.h: one Intra4x4 block on one wave) alone and
// under load: every workgroup (one wave) runs the 16 blocks of a random macroblock in decoding
// order and stamps s_memtime around each block.  Prints the mean shader cycles per block over the
// workgroups and a checksum of the decisions (costs, modes, levels, reconstruction), so that
// variants of i4_block (built with -D...) can be compared for speed and for identical results.
//   hipcc -O3 --offload-arch=gfx950 -I h264-jm-commentary_amd/csrc tools/i4_bench.hip -o tools/i4_bench
//   tools/i4_bench [workgroups] [repeats]
#include "jmh_i4.h"
#include <cstdio>
#include <cstdlib>
#include <vector>

__global__ __launch_bounds__(64) void k_i4_bench(DevParams d, const uint8_t *src, MbScratch *scr, unsigned long long *cyc, int reps,
                                                  unsigned long long *stamps) {
    __shared__ IntraS<uint8_t> s;
    const int lane = threadIdx.x, b = blockIdx.x;
    const uint8_t *p = src + (size_t)b * 512;
    MbScratch *sc = scr + b;
    unsigned long long tot = 0;
    for (int r = 0; r < reps; r++) {
        for (int i = lane; i < 256; i += 64) s.org[i] = p[i];
        if (lane < 24) s.nb.rtop[lane] = p[256 + lane];
        if (lane < 16) { s.nb.rleft[lane] = p[280 + lane]; s.ipred_cur[lane] = -1; }
        if (lane < 10) s.bd.ipm[lane] = (int8_t)(p[300 + lane] % 10) - 1;
        __syncthreads();
        const int qpk = q_round(d.qsel, 15 + d.qp / 6);
        int tabr[2];
        i4_tabrow(lane, tabr);
        int acc[3] = {0, 0, 0};
        const unsigned long long t0 = __builtin_amdgcn_s_memtime();
        for (int blk = 0; blk < 16; blk++) {
            const int bx4 = 2 * ((blk >> 2) & 1) + (blk & 1), by4 = 2 * (blk >> 3) + ((blk >> 1) & 1);
            // stamps (argument 3): i4_block's sub-phase clocks [52..57] of block blk, last repeat of WG 0
            unsigned long long *pst = stamps && b == 0 && r == reps - 1 ? stamps + 6 * blk - 52 : nullptr;
            i4_block(d, s, sc, 0, bx4, by4, tabr, true, true, true, true, qpk, acc, pst);
        }
        const unsigned long long t1 = __builtin_amdgcn_s_memtime();
        tot += t1 - t0;
        if (lane == 0) { sc->i4cost = acc[0]; sc->i4cbp = acc[1]; sc->i4blk = acc[2]; }
        if (lane < 16) sc->ipred[lane] = s.ipred_cur[lane];
        reinterpret_cast<uint32_t *>(sc->i4rec)[lane] = reinterpret_cast<const uint32_t *>(s.rec)[lane];
        __syncthreads();
    }
    if (lane == 0) cyc[b] = tot / reps;
}

int main(int argc, char **argv) {
    const int nwg = argc > 1 ? atoi(argv[1]) : 1, reps = argc > 2 ? atoi(argv[2]) : 20, stamp = argc > 3;
    std::vector<uint8_t> h((size_t)nwg * 512);
    unsigned x = 12345;
    for (auto &v : h) { x = x * 1103515245u + 12345u; v = (uint8_t)(x >> 16); }
    for (int b = 0; b < nwg; b++)   // smooth-ish content: average neighbours so that several modes compete
        for (int i = 1; i < 256; i++) h[(size_t)b * 512 + i] = (uint8_t)((h[(size_t)b * 512 + i] + 3 * h[(size_t)b * 512 + i - 1]) / 4);
    DevParams d{};
    d.lambda_mode = 25; d.qp = 28; d.qpbd = 0; d.use_hadamard = 1; d.maxv = 255; d.qsel = 1;
    uint8_t *dsrc; MbScratch *dscr; unsigned long long *dcyc, *dst = nullptr;
    if (stamp && hipMalloc(&dst, 16 * 6 * 8)) return 1;
    if (hipMalloc(&dsrc, h.size()) || hipMalloc(&dscr, (size_t)nwg * sizeof(MbScratch)) || hipMalloc(&dcyc, nwg * 8)) return 1;
    (void)hipMemcpy(dsrc, h.data(), h.size(), hipMemcpyHostToDevice);
    (void)hipMemset(dscr, 0, (size_t)nwg * sizeof(MbScratch));
    hipLaunchKernelGGL(k_i4_bench, dim3(nwg), dim3(64), 0, 0, d, dsrc, dscr, dcyc, reps, dst);
    if (hipDeviceSynchronize() != hipSuccess) { fprintf(stderr, "kernel failed\n"); return 1; }
    std::vector<unsigned long long> c(nwg);
    std::vector<MbScratch> r(nwg);
    (void)hipMemcpy(c.data(), dcyc, nwg * 8, hipMemcpyDeviceToHost);
    (void)hipMemcpy(r.data(), dscr, (size_t)nwg * sizeof(MbScratch), hipMemcpyDeviceToHost);
    double mean = 0;
    for (auto v : c) mean += (double)v;
    mean /= nwg;
    unsigned long long ck = 1469598103934665603ull;
    for (auto &m : r) {
        const uint8_t *q = reinterpret_cast<const uint8_t *>(&m.i4cost);
        for (size_t i = 0; i < 12; i++) ck = (ck ^ q[i]) * 1099511628211ull;
        for (int i = 0; i < 16; i++) ck = (ck ^ (uint8_t)m.ipred[i]) * 1099511628211ull;
        for (int i = 0; i < 256; i++) ck = (ck ^ (uint16_t)m.i4lev[i / 16][i % 16]) * 1099511628211ull;
        for (int i = 0; i < 256; i++) ck = (ck ^ m.i4rec[i]) * 1099511628211ull;
    }
    if (stamp) {   // per sub-phase wall-clock (100 MHz) deltas averaged over the 16 blocks, in ns
        std::vector<unsigned long long> st(96);
        (void)hipMemcpy(st.data(), dst, 96 * 8, hipMemcpyDeviceToHost);
        double ph[5] = {0};
        for (int k = 0; k < 16; k++)
            for (int q = 0; q < 5; q++) ph[q] += (double)(st[6 * k + q + 1] - st[6 * k + q]) * 10.0 / 16;
        printf("sub-phases ns: fetch %.0f predict+decide %.0f winner %.0f fwd+quant %.0f inv+store %.0f; block to block %.0f\n", ph[0], ph[1],
               ph[2], ph[3], ph[4], (double)(st[90] - st[0]) * 10.0 / 15);
    }
    printf("{\"workgroups\": %d, \"reps\": %d, \"cycles_per_mb\": %.0f, \"cycles_per_block\": %.1f, \"checksum\": \"%016llx\"}\n", nwg, reps,
           mean, mean / 16, ck);
    return 0;
}
