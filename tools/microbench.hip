// tools/microbench.hip — latency probes for the macroblock kernels' building blocks on gfx950:
// cost of one barrier-separated phase (LDS write -> s_barrier -> LDS read) at 512 / 768 threads,
// an LDS round trip, a DPP row reduction, and a global load round trip. Debug tool, not product.
//   hipcc --offload-arch=gfx950 -O3 tools/microbench.hip -o /tmp/mb && /tmp/mb
#include <hip/hip_runtime.h>
#include <stdio.h>

template <int NT>
__global__ __launch_bounds__(NT) void k_phase(int iters, int *out, unsigned long long *t) {
    __shared__ int x[NT];
    int v = threadIdx.x;
    unsigned long long t0 = wall_clock64();
    for (int i = 0; i < iters; i++) {
        x[threadIdx.x] = v;
        __syncthreads();
        v += x[(threadIdx.x + 1) % NT];
        __syncthreads();
    }
    unsigned long long t1 = wall_clock64();
    out[blockIdx.x * NT + threadIdx.x] = v;
    if (threadIdx.x == 0) t[blockIdx.x] = t1 - t0;
}

__global__ __launch_bounds__(64) void k_lds_chain(int iters, int *out, unsigned long long *t) {
    __shared__ int x[64];
    x[threadIdx.x] = threadIdx.x;
    __syncthreads();
    int v = threadIdx.x;
    unsigned long long t0 = wall_clock64();
    for (int i = 0; i < iters; i++) v = x[v & 63];
    unsigned long long t1 = wall_clock64();
    out[threadIdx.x] = v;
    if (threadIdx.x == 0) t[0] = t1 - t0;
}

__global__ __launch_bounds__(64) void k_global_chain(int iters, const int *p, int *out, unsigned long long *t) {
    int v = threadIdx.x;
    unsigned long long t0 = wall_clock64();
    for (int i = 0; i < iters; i++) v = p[v & 1023];
    unsigned long long t1 = wall_clock64();
    out[threadIdx.x] = v;
    if (threadIdx.x == 0) t[0] = t1 - t0;
}

__global__ __launch_bounds__(64) void k_bperm_chain(int iters, int *out, unsigned long long *t) {
    int v = threadIdx.x;
    unsigned long long t0 = wall_clock64();
    for (int i = 0; i < iters; i++) v = __shfl(v, (v + 1) & 63, 64);
    unsigned long long t1 = wall_clock64();
    out[threadIdx.x] = v;
    if (threadIdx.x == 0) t[0] = t1 - t0;
}

__global__ __launch_bounds__(64) void k_dpp_chain(int iters, int *out, unsigned long long *t) {
    int v = threadIdx.x;
    unsigned long long t0 = wall_clock64();
    for (int i = 0; i < iters; i++) {
        v += __builtin_amdgcn_update_dpp(v, v, 0xB1, 0xF, 0xF, false);
        v += __builtin_amdgcn_update_dpp(v, v, 0x4E, 0xF, 0xF, false);
        v += __builtin_amdgcn_update_dpp(v, v, 0x141, 0xF, 0xF, false);
        v += __builtin_amdgcn_update_dpp(v, v, 0x140, 0xF, 0xF, false);
    }
    unsigned long long t1 = wall_clock64();
    out[threadIdx.x] = v;
    if (threadIdx.x == 0) t[0] = t1 - t0;
}

int main() {
    int *out, *p;
    unsigned long long *t, h[256];
    hipMalloc(&out, 256 * 1024 * 4);
    hipMalloc(&p, 1024 * 4);
    hipMemset(p, 0, 4096);
    hipMalloc(&t, 256 * 8);
    int rate = 0;
    hipDeviceGetAttribute(&rate, hipDeviceAttributeWallClockRate, 0);
    const double ns = 1e6 / rate;   // ns per tick
    const int it = 2000;
    auto run = [&](const char *name, int n, int div) {
        hipDeviceSynchronize();
        hipMemcpy(h, t, n * 8, hipMemcpyDeviceToHost);
        unsigned long long m = 0;
        for (int i = 0; i < n; i++) m = h[i] > m ? h[i] : m;
        printf("%-34s %8.1f ns per step\n", name, m * ns / div);
    };
    hipLaunchKernelGGL(k_phase<512>, dim3(32), dim3(512), 0, 0, it, out, t);
    run("barrier phase, 512 thr, 32 WGs", 32, 2 * it);
    hipLaunchKernelGGL(k_phase<768>, dim3(32), dim3(768), 0, 0, it, out, t);
    run("barrier phase, 768 thr, 32 WGs", 32, 2 * it);
    hipLaunchKernelGGL(k_phase<256>, dim3(32), dim3(256), 0, 0, it, out, t);
    run("barrier phase, 256 thr, 32 WGs", 32, 2 * it);
    hipLaunchKernelGGL(k_lds_chain, dim3(1), dim3(64), 0, 0, it, out, t);
    run("dependent LDS load", 1, it);
    hipLaunchKernelGGL(k_global_chain, dim3(1), dim3(64), 0, 0, it, p, out, t);
    run("dependent global load (L2 hit)", 1, it);
    hipLaunchKernelGGL(k_bperm_chain, dim3(1), dim3(64), 0, 0, it, out, t);
    run("dependent ds_bpermute", 1, it);
    hipLaunchKernelGGL(k_dpp_chain, dim3(1), dim3(64), 0, 0, it, out, t);
    run("row16 DPP sum (4 steps)", 1, it);
    printf("wall clock %d kHz\n", rate);
    return 0;
}
