// jmh_hbd.hip — the High 10 (9 / 10-bit luma, config 5) unit seams on 16-bit samples
// (include/jmhip.h jmh_*_u16; JM >= 10 FRExt with imgpel = unsigned short [J]):
//
//  k_sad_table_u16  SetupFastFullPelSearch's 4x4 BlockSAD table: one thread per (macroblock,
//                   window position), the 16 4x4 SADs by v_sad_u16 on packed sample pairs (a 4x4
//                   SAD <= 16 * 1023 fits the u16 table as at 8 bits)
//  k_tq4x4_u16      dct_luma at qp + QpBdOffsetY on 16-lane groups (the macroblock kernels'
//                   lane_fwd4x4 / lane_quant / lane_inv4x4), reconstruction clipped to 2^bd - 1
//  k_tq8x8_u16      dct_luma8x8 likewise on one wave per block; int32 headroom at 10 bits: the
//                   largest |coefficient| x quant_coef8 is 64 * 1023 * 20972 + (1 << 26) / 3 < 2^31
//
// The per-block search at 10 bits is k_block_search<uint16_t> (jmh_block.hip).
#include "jmh_common.h"

// pack two samples into one dword (low = first)
__device__ __forceinline__ uint32_t pk2(int a, int b) { return (uint32_t)a | ((uint32_t)b << 16); }

__global__ __launch_bounds__(256) void k_sad_table_u16(const uint16_t *__restrict__ org, const uint16_t *__restrict__ ref, int W, int H, int sr,
                                                       const int32_t *mb_xy, const int32_t *centres, uint16_t *out) {
    const int i = blockIdx.y;
    const int side = 2 * sr + 1, npos = side * side;
    const int r = blockIdx.x * 256 + threadIdx.x;
    if (r >= npos) return;
    const int px = 16 * mb_xy[2 * i], py = 16 * mb_xy[2 * i + 1];
    const int dx = r % side - sr + centres[2 * i], dy = r / side - sr + centres[2 * i + 1];
#pragma unroll 1
    for (int b = 0; b < 16; b++) {
        const int ox = (b & 3) * 4, oy = (b >> 2) * 4;
        uint32_t sad = 0;
#pragma unroll
        for (int y = 0; y < 4; y++) {
            const uint16_t *o = org + (py + oy + y) * W + px + ox;
            const int ry = iclip(0, H - 1, py + dy + oy + y) * W, rx = px + dx + ox;
            const uint32_t r01 = pk2(ref[ry + iclip(0, W - 1, rx)], ref[ry + iclip(0, W - 1, rx + 1)]);
            const uint32_t r23 = pk2(ref[ry + iclip(0, W - 1, rx + 2)], ref[ry + iclip(0, W - 1, rx + 3)]);
            sad = __builtin_amdgcn_sad_u16(pk2(o[0], o[1]), r01, sad);
            sad = __builtin_amdgcn_sad_u16(pk2(o[2], o[3]), r23, sad);
        }
        out[((size_t)i * 16 + b) * npos + r] = (uint16_t)sad;
    }
}

__global__ __launch_bounds__(256) void k_tq4x4_u16(int n, const int16_t *resid, const uint16_t *pred, int qpb, int qsel, int maxv,
                                                   int16_t *levels, uint16_t *recon, int32_t *coeff_cost, int32_t *nonzero) {
    const int blk = blockIdx.x * 16 + (threadIdx.x >> 4), l = threadIdx.x & 15;
    const bool act = blk < n;
    const int bi = act ? blk : 0;
    const int c = lane_fwd4x4(resid[16 * bi + l], l);
    int lev, dq, cc;
    const int q_bits = 15 + qpb / 6;
    const unsigned nz = lane_quant(c, l, qpb, q_round(qsel, q_bits), false, lev, dq, cc);
    const int rv = lane_inv4x4(dq, l, pred[16 * bi + l], maxv);
    if (act) {
        levels[16 * blk + l] = (int16_t)lev;
        recon[16 * blk + l] = (uint16_t)rv;
        if (l == 0) { coeff_cost[blk] = cc; nonzero[blk] = nz != 0; }
    }
}

__global__ __launch_bounds__(256) void k_tq8x8_u16(int n, const int16_t *resid, const uint16_t *pred, int qpb, int qsel, int maxv,
                                                   int16_t *levels, uint16_t *recon, int32_t *coeff_cost, int32_t *nonzero) {
    const int blk = blockIdx.x * 4 + (threadIdx.x >> 6), l = threadIdx.x & 63;
    if (blk >= n) return;                        // whole waves only: no workgroup barrier below
    const int q_bits = 16 + qpb / 6;
    const int c = wave_fwd8x8(resid[64 * blk + l], l);
    int lev, dq, cc;
    const unsigned long long nz = wave_quant8(c, l, qpb, q_round(qsel, q_bits), lev, dq, cc);
    recon[64 * blk + l] = (uint16_t)wave_inv8x8(dq, l, pred[64 * blk + l], maxv);
    levels[64 * blk + l] = (int16_t)lev;
    if (l == 0) { coeff_cost[blk] = cc; nonzero[blk] = nz != 0; }
}

hipError_t jmh_launch_sad_table_u16(const uint16_t *org, const uint16_t *ref, int W, int H, int sr, int n_mb, const int32_t *mb_xy,
                                    const int32_t *centres, uint16_t *out, hipStream_t st) {
    const int side = 2 * sr + 1, npos = side * side;
    hipLaunchKernelGGL(k_sad_table_u16, dim3((npos + 255) / 256, n_mb), dim3(256), 0, st, org, ref, W, H, sr, mb_xy, centres, out);
    return hipGetLastError();
}
hipError_t jmh_launch_tq4x4_u16(int n, const int16_t *resid, const uint16_t *pred, int qp, int qsel, int bit_depth, int16_t *levels,
                                uint16_t *recon, int32_t *cc, int32_t *nz, hipStream_t st) {
    hipLaunchKernelGGL(k_tq4x4_u16, dim3((n + 15) / 16), dim3(256), 0, st, n, resid, pred, qp + 6 * (bit_depth - 8), qsel,
                       (1 << bit_depth) - 1, levels, recon, cc, nz);
    return hipGetLastError();
}
hipError_t jmh_launch_tq8x8_u16(int n, const int16_t *resid, const uint16_t *pred, int qp, int qsel, int bit_depth, int16_t *levels,
                                uint16_t *recon, int32_t *cc, int32_t *nz, hipStream_t st) {
    hipLaunchKernelGGL(k_tq8x8_u16, dim3((n + 3) / 4), dim3(256), 0, st, n, resid, pred, qp + 6 * (bit_depth - 8), qsel,
                       (1 << bit_depth) - 1, levels, recon, cc, nz);
    return hipGetLastError();
}
