// jmh_intra8.hip — k_mb_intra8: the Intra8x8 macroblock decision of the High profile
// (Transform8x8Mode = 1) for every macroblock of one wavefront tick, between k_mb_analyse and
// k_mb_final.  Restates JM FRExt rdopt.c › Mode_Decision_for_Intra8x8Macroblock /
// Mode_Decision_for_new_8x8IntraBlocks (RDO off) [J] as pinned in docs/JM_SEMANTICS.md items 26-28:
// the four 8x8 blocks in order, each with the nine Intra_8x8 predictions (8.3.2.2, reference
// sample filtering 8.3.2.2.1) scored by HadamardSAD8x8 + (mode != MPM ? 4λ : 0), then dct_luma8x8
// of the winner and its reconstruction, which the next block predicts from.
//
// One workgroup (4 waves) per macroblock: wave w scores modes w, w + 4, w + 8 with one lane per
// sample of the 8x8 block (64-lane Hadamard by lane exchanges), and wave 0 transforms the winner.
// Results land in MbScratch (i8cost, i8cbp, i8modes, i8lev, i8rec) for k_mb_final's decision.
#include "jmh_intra8.h"

__global__ __launch_bounds__(NT, 8) void k_mb_intra8(const TickArgs t) {
    __shared__ I8S<uint8_t> s;   // bit depth 8 (FFS / full-search ticks)
    const int mi = xcd_block(blockIdx.x, t.pre[t.npic]);      // XCD-aware (jmh_device.h)
    if (mi >= t.pre[t.npic]) return;
    intra8_mb<uint8_t>(t, s, mi);
}

hipError_t jmh_launch_intra8(const TickArgs &t, hipStream_t st) {
    hipLaunchKernelGGL(k_mb_intra8, dim3(xcd_grid(t.pre[t.npic])), dim3(NT), 0, st, t);
    return hipGetLastError();
}
