// fetch_calib.hip -- calibrates rocprofv3's FETCH_SIZE on gfx950 against known byte counts for
// the load widths the wavefront kernels use (the MI355X guide calibrates only 16-byte
// per-lane streaming reads, at exactly 1/2).  One launch per width streams a 1 GiB buffer (beyond
// the 256 MiB Infinity Cache, evicted between launches by a 512 MiB write) exactly once:
//   k_read<16>  global_load_dwordx4 per lane    k_read<4>  global_load_dword per lane
//   k_read<1>   global_load_ubyte per lane      k_read<2>  global_load_ushort per lane
// Run:  rocprofv3 --pmc FETCH_SIZE --kernel-trace -d OUT -o fc --output-format csv -- ./fetch_calib
// then tools/fetch_calib.py OUT: FETCH_SIZE (KB) x 1024 / bytes per kernel = the factor.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

template <int BYTES>
__global__ void k_read(const uint8_t *__restrict__ p, size_t n, uint32_t *__restrict__ out) {
    const size_t stride = (size_t)gridDim.x * blockDim.x * BYTES;
    uint32_t acc = 0;
    for (size_t i = ((size_t)blockIdx.x * blockDim.x + threadIdx.x) * BYTES; i < n; i += stride) {
        if constexpr (BYTES == 16) {
            const uint4 v = *reinterpret_cast<const uint4 *>(p + i);
            acc += v.x + v.y + v.z + v.w;
        } else if constexpr (BYTES == 4) acc += *reinterpret_cast<const uint32_t *>(p + i);
        else if constexpr (BYTES == 2) acc += *reinterpret_cast<const uint16_t *>(p + i);
        else acc += p[i];
    }
    if (acc == 0x7FFFFFFEu) out[0] = acc;   // keeps the loads (a sum the data never gives)
}
__global__ void k_evict(uint32_t *__restrict__ p, size_t n) {
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) p[i] = (uint32_t)i;
}

int main() {
    const size_t n = (size_t)1 << 30, ne = ((size_t)512 << 20) / 4;
    uint8_t *buf;
    uint32_t *ev, *out;
    if (hipMalloc(&buf, n) != hipSuccess || hipMalloc(&ev, ne * 4) != hipSuccess || hipMalloc(&out, 4) != hipSuccess) return 1;
    if (hipMemset(buf, 1, n) != hipSuccess) return 1;
    const dim3 g(256 * 8), b(256);
    auto evict = [&] { hipLaunchKernelGGL(k_evict, g, b, 0, 0, ev, ne); };
    evict(); hipLaunchKernelGGL(k_read<16>, g, b, 0, 0, buf, n, out);
    evict(); hipLaunchKernelGGL(k_read<4>, g, b, 0, 0, buf, n, out);
    evict(); hipLaunchKernelGGL(k_read<2>, g, b, 0, 0, buf, n, out);
    evict(); hipLaunchKernelGGL(k_read<1>, g, b, 0, 0, buf, n, out);
    if (hipDeviceSynchronize() != hipSuccess) return 2;
    printf("{\"bytes_per_kernel\": %zu}\n", n);
    (void)hipFree(buf); (void)hipFree(ev); (void)hipFree(out);
    return 0;
}
