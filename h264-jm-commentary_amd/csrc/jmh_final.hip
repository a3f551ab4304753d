// jmh_final.hip — k_mb_final: the second half of encode_one_macroblock [J] (RDO off) for every
// macroblock of one wavefront diagonal, after k_mb_analyse (and k_mb_intra8 in the High profile):
// the mode decision over the analysis costs, then the residual coding of the chosen mode with
// 16-lane transform groups (LumaResidualCoding / dct_luma_16x16 / dct_chroma + reconstruction),
// or, with Transform8x8Mode, TransformDecision and dct_luma8x8 on one wave per 8x8 block, and the
// outputs the next diagonal depends on (reconstruction, MVs, reference indices, intra modes).
#include "jmh_final.h"

// OCC workgroups per CU (see jmh_final.h)
template <int OCC, class pel, bool T8>
__global__ __launch_bounds__(NT, OCC) void k_mb_final(const TickArgs t) {
    __shared__ FinS<pel> s;
    const unsigned long long bt0 = t.bprof_fin ? wall_clock64() : 0;
    const int m = xcd_block(blockIdx.x, t.pre[t.npic]);       // XCD-aware (jmh_device.h)
    if (m >= t.pre[t.npic]) return;                           // padding block (whole workgroup)
    final_mb<OCC, pel, T8>(t, s, m, threadIdx.x, blockIdx.x, bt0);
}

// one MB per 512-thread workgroup (final_core's luma and chroma coding side by side), two per CU
template <class pel, bool T8>
__global__ __launch_bounds__(2 * NT, 4) void k_mb_final512(const TickArgs t) {
    __shared__ FinS<pel> s;
    const unsigned long long bt0 = t.bprof_fin ? wall_clock64() : 0;
    const int m = xcd_block(blockIdx.x, t.pre[t.npic]);       // XCD-aware (jmh_device.h)
    if (m >= t.pre[t.npic]) return;                           // padding block (whole workgroup)
    final_mb<5, pel, T8, 2 * NT>(t, s, m, threadIdx.x, blockIdx.x, bt0);
}

hipError_t jmh_launch_final(const TickArgs &t, hipStream_t st) {
    static const bool occ8 = getenv("JMH_FINAL_OCC8") != nullptr;   // A/B: the 8-per-CU build always
    static const char *f512 = getenv("JMH_FINAL512");               // A/B: 0 = the 256-thread five-per-CU build
    const int n = t.pre[t.npic];
    if (!occ8 && t.bd == 8 && !t.t8 && n <= 2 * 256 && !(f512 && atoi(f512) == 0))
        hipLaunchKernelGGL((k_mb_final512<uint8_t, false>), dim3(xcd_grid(n)), dim3(2 * NT), 0, st, t);
    else if (t.bd > 8) hipLaunchKernelGGL((k_mb_final<8, uint16_t, true>), dim3(xcd_grid(n)), dim3(NT), 0, st, t);
    else if (occ8 || n > 5 * 256) hipLaunchKernelGGL((k_mb_final<8, uint8_t, true>), dim3(xcd_grid(n)), dim3(NT), 0, st, t);
    else if (t.t8) hipLaunchKernelGGL((k_mb_final<5, uint8_t, true>), dim3(xcd_grid(n)), dim3(NT), 0, st, t);
    else hipLaunchKernelGGL((k_mb_final<5, uint8_t, false>), dim3(xcd_grid(n)), dim3(NT), 0, st, t);
    return hipGetLastError();
}
