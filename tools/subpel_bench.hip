// tools/subpel_bench.hip — latency of k_mb_analyse's subpel_wave (SubPelBlockMotionSearch on one
// wave, jmh_analyse.hip) for a 4x4 (with its forwarded MVP) and an 8x8 block, on one workgroup
// alone or on many: wave 0 of every workgroup runs the search `reps` times on synthetic planes and
// stamps s_memtime around them.  Prints the mean shader cycles per search and a checksum of the
// results, so that variants (built with -D...) can be compared for speed and identical results.
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -I h264-jm-commentary_amd/csrc tools/subpel_bench.hip -o tools/subpel_bench
//   tools/subpel_bench [workgroups] [reps]
#include "jmh_analyse.hip"
#include <cstdio>
#include <cstdlib>
#include <vector>

__global__ __launch_bounds__(NTA, 4) void k_subpel_bench(DevParams d, const uint8_t *src, unsigned long long *cyc, int *res, int reps) {
    __shared__ MeS s;
    const int tid = threadIdx.x, wave = tid >> 6, b = blockIdx.x;
    const uint8_t *p = src + (size_t)b * 4096;
    for (int i = tid; i < 4 * PLS; i += NTA) s.planes[i] = p[i & 4095] ^ (uint8_t)(i >> 12);
    if (tid < 256) s.org[tid] = p[tid * 7 & 4095];
    if (tid < 10) { s.bd.ref[tid] = tid == 5 ? -2 : 0; s.bd.mv[tid][0] = (int16_t)(p[tid] % 9 - 4); s.bd.mv[tid][1] = (int16_t)(p[tid + 16] % 9 - 4); }
    for (int i = tid; i < 8 * 16 * 2; i += NTA) (&s.all_mv[0][0][0])[i] = (int16_t)(p[i] % 7 - 3);
    if (tid < 32) (&s.motion_cost[0][0])[tid] = 0;
    // full-pel winners: spiral order 1 + (b % 60) around the window centre
    if (tid < (NTS / 64) * MAXNS) (&s.red[0][0])[tid] = (100u << 13) | (unsigned)(1 + (b + tid) % 60);
    __syncthreads();
    unsigned long long t0 = 0, t1 = 0;
    const SDesc q4 = {7, 1, 0, 0, 7, 0, 1, 0}, q8 = {4, 0, 0, 0, 0, 0, 0, 0};
    if (wave == 0) {
        t0 = __builtin_amdgcn_s_memtime();
        for (int r = 0; r < reps; r++) subpel_wave(d, s, 0, q4, 5, -3, 2, -1, 0, 0);
        t1 = __builtin_amdgcn_s_memtime();
        if (__lane_id() == 0) cyc[2 * b] = (t1 - t0) / reps;
        t0 = __builtin_amdgcn_s_memtime();
        for (int r = 0; r < reps; r++) subpel_wave(d, s, 0, q8, 5, -3, 2, -1, 0, 0);
        t1 = __builtin_amdgcn_s_memtime();
        if (__lane_id() == 0) cyc[2 * b + 1] = (t1 - t0) / reps;
    }
    __syncthreads();
    if (tid < 64) res[b * 64 + tid] = s.all_mv[7][tid & 15][0] + 7 * s.all_mv[4][tid & 15][1] + s.motion_cost[7][0] + s.pmv[0][0] * 3 + s.pmv[0][1];
}

int main(int argc, char **argv) {
    const int nwg = argc > 1 ? atoi(argv[1]) : 1, reps = argc > 2 ? atoi(argv[2]) : 50;
    std::vector<uint8_t> h((size_t)nwg * 4096);
    unsigned x = 777;
    for (auto &v : h) { x = x * 1103515245u + 12345u; v = (uint8_t)(x >> 16); }
    // spiral-index -> position table (ordtab_fill's second part) at ORDTAB_SPOS
    std::vector<uint32_t> ot((size_t)ORDTAB_SPOS + 65 * 65, 0);
    for (int k = 0; k < 65 * 65; k++) {
        int px = 0, py = 0;   // host restatement of spiral_pos
        if (k) {
            int l = 1;
            while ((2 * l + 1) * (2 * l + 1) <= k) l++;
            const int o = k - (2 * l - 1) * (2 * l - 1);
            if (o < 2 * (2 * l - 1)) { px = (o >> 1) - l + 1; py = (o & 1) ? l : -l; }
            else { const int o2 = o - 2 * (2 * l - 1); py = (o2 >> 1) - l; px = (o2 & 1) ? l : -l; }
        }
        ot[(size_t)ORDTAB_SPOS + k] = ((uint32_t)px & 0xFFFFu) | (uint32_t)py << 16;
    }
    DevParams d{};
    d.sr = 32; d.side = 65; d.npos = 65 * 65; d.lambda_motion = 12; d.use_hadamard = 1; d.slice_type = JMH_P_SLICE;
    d.maxv = 255; d.isr = 0xFE; d.mbw = 120; d.mbh = 68; d.slice_mbs = 8160;
    uint8_t *dsrc; unsigned long long *dcyc; int *dres; uint32_t *dot;
    if (hipMalloc(&dsrc, h.size()) || hipMalloc(&dcyc, (size_t)nwg * 16) || hipMalloc(&dres, (size_t)nwg * 256) ||
        hipMalloc(&dot, ot.size() * 4))
        return 1;
    (void)hipMemcpy(dsrc, h.data(), h.size(), hipMemcpyHostToDevice);
    (void)hipMemcpy(dot, ot.data(), ot.size() * 4, hipMemcpyHostToDevice);
    d.ordtab = dot;
    hipLaunchKernelGGL(k_subpel_bench, dim3(nwg), dim3(NTA), 0, 0, d, dsrc, dcyc, dres, reps);
    if (hipDeviceSynchronize() != hipSuccess) { fprintf(stderr, "kernel failed\n"); return 1; }
    std::vector<unsigned long long> c((size_t)nwg * 2);
    std::vector<int> r((size_t)nwg * 64);
    (void)hipMemcpy(c.data(), dcyc, c.size() * 8, hipMemcpyDeviceToHost);
    (void)hipMemcpy(r.data(), dres, r.size() * 4, hipMemcpyDeviceToHost);
    double m4 = 0, m8 = 0;
    for (int b = 0; b < nwg; b++) { m4 += (double)c[2 * b]; m8 += (double)c[2 * b + 1]; }
    unsigned long long ck = 1469598103934665603ull;
    for (int v : r) ck = (ck ^ (uint32_t)v) * 1099511628211ull;
    printf("{\"workgroups\": %d, \"reps\": %d, \"cycles_4x4\": %.0f, \"cycles_8x8\": %.0f, \"checksum\": \"%016llx\"}\n", nwg, reps,
           m4 / nwg, m8 / nwg, ck);
    return 0;
}
