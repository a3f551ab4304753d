// Host cost of hipLaunchKernelGGL against the kernel-argument size (16 B .. 4 KB): the lencod
// main thread issues ~48 launches per 1080p picture with 4 KB TickArgs.
//   hipcc --offload-arch=gfx950 -O2 tools/launch_cost.hip -o tools/launch_cost_bin
#include <hip/hip_runtime.h>
#include <chrono>
#include <stdio.h>

template <int N>
struct Args { int v[N / 4]; };

template <int N>
__global__ void k_args(const Args<N> a, int *out) {
    if (threadIdx.x == 0 && blockIdx.x == 0) out[0] = a.v[N / 4 - 1];
}

template <int N>
static double cost_us(hipStream_t st, int *d, int reps) {
    Args<N> a{};
    for (int i = 0; i < 3; i++) hipLaunchKernelGGL(k_args<N>, dim3(1), dim3(64), 0, st, a, d);
    hipStreamSynchronize(st);
    auto t0 = std::chrono::steady_clock::now();
    for (int i = 0; i < reps; i++) { a.v[0] = i; hipLaunchKernelGGL(k_args<N>, dim3(1), dim3(64), 0, st, a, d); }
    auto t1 = std::chrono::steady_clock::now();
    hipStreamSynchronize(st);
    return std::chrono::duration<double, std::micro>(t1 - t0).count() / reps;
}

int main() {
    hipStream_t st;
    hipStreamCreateWithFlags(&st, hipStreamNonBlocking);
    int *d;
    hipMalloc(&d, 64);
    printf("{\"launch_us\": {\"16\": %.2f, \"256\": %.2f, \"1024\": %.2f, \"2048\": %.2f, \"4064\": %.2f}}\n",
           cost_us<16>(st, d, 2000), cost_us<256>(st, d, 2000), cost_us<1024>(st, d, 2000), cost_us<2048>(st, d, 2000),
           cost_us<4064>(st, d, 2000));
    return 0;
}
