// jmh_kernels.hip — gfx950 kernels outside the macroblock wavefront:
//
//  k_interp      UnifiedOneForthPix [J] / H.264 8.4.2.2.1: 16 quarter-pel phase planes of the
//                reference (HBM-bound; one thread per padded integer position, all 16 phases),
//                for the jmh_read_qpel seam (a1).  The macroblock kernels interpolate on the fly
//                (LDS planes in k_mb_analyse, qpel_direct in k_mb_final), so a picture can be
//                searched while its reference is still being reconstructed (pipelining).
//  k_sad_table / k_tq4x4   unit seams (jmh_ffs_sad_table / jmh_tq4x4_batch); k_tq4x4 runs the
//                same 16-lane TQ primitive the macroblock kernels use.
//
// The macroblock wavefront itself is k_mb_analyse (jmh_analyse.hip) + k_mb_final (jmh_final.hip).
#include "jmh_common.h"

// ======================================================================================
//  quarter-pel interpolation (H.264 8.4.2.2.1), spec coordinate clamping
// ======================================================================================
// rpx / hb1 / vh1: jmh_common.h

__global__ __launch_bounds__(256) void k_interp(const uint8_t *__restrict__ ref, int W, int H, uint8_t *__restrict__ qpel, int qstride,
                                                int qplane) {
    int px = blockIdx.x * 64 + (threadIdx.x & 63);
    int py = blockIdx.y * 4 + (threadIdx.x >> 6);
    if (px >= qstride || py >= H + 2 * QPAD) return;
    int x = px - QPAD, y = py - QPAD;
    int G = rpx(ref, W, H, x, y), Hn = rpx(ref, W, H, x + 1, y), M = rpx(ref, W, H, x, y + 1);
    int b = clip255((hb1(ref, W, H, x, y) + 16) >> 5);
    int hh = clip255((vh1(ref, W, H, x, y) + 16) >> 5);
    int s = clip255((hb1(ref, W, H, x, y + 1) + 16) >> 5);
    int m = clip255((vh1(ref, W, H, x + 1, y) + 16) >> 5);
    int j1 = tap6(vh1(ref, W, H, x - 2, y), vh1(ref, W, H, x - 1, y), vh1(ref, W, H, x, y), vh1(ref, W, H, x + 1, y), vh1(ref, W, H, x + 2, y),
                  vh1(ref, W, H, x + 3, y));
    int j = clip255((j1 + 512) >> 10);
    uint8_t v[16];
    v[0] = G;                  v[1] = (G + b + 1) >> 1;   v[2] = b;                  v[3] = (Hn + b + 1) >> 1;
    v[4] = (G + hh + 1) >> 1;  v[5] = (b + hh + 1) >> 1;  v[6] = (b + j + 1) >> 1;   v[7] = (b + m + 1) >> 1;
    v[8] = hh;                 v[9] = (hh + j + 1) >> 1;  v[10] = j;                 v[11] = (j + m + 1) >> 1;
    v[12] = (M + hh + 1) >> 1; v[13] = (hh + s + 1) >> 1; v[14] = (j + s + 1) >> 1;  v[15] = (m + s + 1) >> 1;
    size_t o = (size_t)py * qstride + px;
#pragma unroll
    for (int ph = 0; ph < 16; ph++) qpel[(size_t)ph * qplane + o] = v[ph];
}

// ======================================================================================
//  unit seams
// ======================================================================================
__global__ __launch_bounds__(256) void k_sad_table(const uint8_t *__restrict__ org, const uint8_t *__restrict__ ref, int W, int H, int sr,
                                                   const int32_t *mb_xy, const int32_t *centres, uint16_t *out) {
    int i = blockIdx.y;
    int side = 2 * sr + 1, npos = side * side;
    int r = blockIdx.x * 256 + threadIdx.x;
    if (r >= npos) return;
    int px = 16 * mb_xy[2 * i], py = 16 * mb_xy[2 * i + 1];
    int dx = r % side - sr + centres[2 * i], dy = r / side - sr + centres[2 * i + 1];
    for (int b = 0; b < 16; b++) {
        int ox = (b & 3) * 4, oy = (b >> 2) * 4, sad = 0;
        for (int y = 0; y < 4; y++)
            for (int x = 0; x < 4; x++)
                sad += abs(org[(py + oy + y) * W + px + ox + x] - ref[iclip(0, H - 1, py + dy + oy + y) * W + iclip(0, W - 1, px + dx + ox + x)]);
        out[((size_t)i * 16 + b) * npos + r] = (uint16_t)sad;
    }
}

// the macroblock kernel's 16-lane dct_luma on independent blocks (16 lanes per block)
__global__ __launch_bounds__(256) void k_tq4x4(int n, const int16_t *resid, const uint8_t *pred, int qp, int qsel, int16_t *levels,
                                               uint8_t *recon, int32_t *coeff_cost, int32_t *nonzero) {
    const int blk = blockIdx.x * 16 + (threadIdx.x >> 4), l = threadIdx.x & 15;
    const bool act = blk < n;
    const int bi = act ? blk : 0;
    const int c = lane_fwd4x4(resid[16 * bi + l], l);
    int lev, dq, cc;
    const int q_bits = 15 + qp / 6;
    unsigned nz = lane_quant(c, l, qp, q_round(qsel, q_bits), false, lev, dq, cc);
    const int rv = lane_inv4x4(dq, l, pred[16 * bi + l]);
    if (act) {
        levels[16 * blk + l] = (int16_t)lev;
        recon[16 * blk + l] = (uint8_t)rv;
        if (l == 0) { coeff_cost[blk] = cc; nonzero[blk] = nz != 0; }
    }
}

// the macroblock kernels' one-wave dct_luma8x8 on independent blocks (4 blocks per workgroup)
__global__ __launch_bounds__(256) void k_tq8x8(int n, const int16_t *resid, const uint8_t *pred, int qp, int qsel, int16_t *levels,
                                               uint8_t *recon, int32_t *coeff_cost, int32_t *nonzero) {
    const int blk = blockIdx.x * 4 + (threadIdx.x >> 6), l = threadIdx.x & 63;
    if (blk >= n) return;                        // whole waves only: no workgroup barrier below
    const int q_bits = 16 + qp / 6;
    const int c = wave_fwd8x8(resid[64 * blk + l], l);
    int lev, dq, cc;
    const unsigned long long nz = wave_quant8(c, l, qp, q_round(qsel, q_bits), lev, dq, cc);
    recon[64 * blk + l] = (uint8_t)wave_inv8x8(dq, l, pred[64 * blk + l]);
    levels[64 * blk + l] = (int16_t)lev;
    if (l == 0) { coeff_cost[blk] = cc; nonzero[blk] = nz != 0; }
}

// ---- launchers (host side, same translation unit) --------------------------------------
hipError_t jmh_launch_interp(const uint8_t *ref, int W, int H, uint8_t *qpel, int qstride, int qplane, hipStream_t st) {
    dim3 grid((qstride + 63) / 64, (H + 2 * QPAD + 3) / 4);
    hipLaunchKernelGGL(k_interp, grid, dim3(256), 0, st, ref, W, H, qpel, qstride, qplane);
    return hipGetLastError();
}
hipError_t jmh_launch_sad_table(const uint8_t *org, const uint8_t *ref, int W, int H, int sr, int n_mb, const int32_t *mb_xy,
                                const int32_t *centres, uint16_t *out, hipStream_t st) {
    int side = 2 * sr + 1, npos = side * side;
    hipLaunchKernelGGL(k_sad_table, dim3((npos + 255) / 256, n_mb), dim3(256), 0, st, org, ref, W, H, sr, mb_xy, centres, out);
    return hipGetLastError();
}
hipError_t jmh_launch_tq8x8(int n, const int16_t *resid, const uint8_t *pred, int qp, int qsel, int16_t *levels, uint8_t *recon,
                            int32_t *cc, int32_t *nz, hipStream_t st) {
    hipLaunchKernelGGL(k_tq8x8, dim3((n + 3) / 4), dim3(256), 0, st, n, resid, pred, qp, qsel, levels, recon, cc, nz);
    return hipGetLastError();
}
hipError_t jmh_launch_tq4x4(int n, const int16_t *resid, const uint8_t *pred, int qp, int qsel, int16_t *levels, uint8_t *recon,
                            int32_t *cc, int32_t *nz, hipStream_t st) {
    hipLaunchKernelGGL(k_tq4x4, dim3((n + 15) / 16), dim3(256), 0, st, n, resid, pred, qp, qsel, levels, recon, cc, nz);
    return hipGetLastError();
}
