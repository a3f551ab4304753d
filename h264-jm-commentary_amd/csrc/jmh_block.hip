// jmh_block.hip — k_block_search: one BlockMotionSearch [J] call per request (JM 8.6
// mv-search.c › BlockMotionSearch → FastFullPelBlockMotionSearch / FullPelBlockMotionSearch →
// SubPelBlockMotionSearch), the per-block seam behind the host's JM-named call surface
// (host/jm86.c BlockMotionSearch / PartitionMotionSearch) and an RDO-on loop.
//
// The wavefront kernels search whole macroblocks with the MVP derived on the device; here the
// caller supplies the MVP, the window centre, the (restricted) range and lambda, exactly the
// arguments BlockMotionSearch works from, so any loop order the host chooses is served.
// One 256-thread workgroup per request:
//   * full pel: the spiral's (2R+1)^2 positions around the centre spread over the threads, SAD
//     straight from the reference (clamped coordinates = UMV), cost = SAD + MV_COST(lambda_factor,
//     2, ...), key = (cost + KOFF) << 13 | JM order (FFS: 0 for the (0,0) pre-check, else spiral
//     index + 1; full search: spiral index, the 16x16 zero-vector bias applied), block minimum;
//   * sub pel: half- then quarter-pel pass, one thread per (candidate, 4x4 sub-block) with the
//     quarter samples computed from the reference (qpel_direct), SATD, LDS candidate sums, the
//     candidate scan with strict '<' on one thread (JM order).
#include "jmh_common.h"

#define BKOFF 8192                       // cost offset: the zero-vector bias can make a cost negative

__device__ __forceinline__ int mv_cost_lf(int lf, int shift, int cx, int cy, int px, int py) {
    return (lf * (mvbits(cx * (1 << shift) - px) + mvbits(cy * (1 << shift) - py))) >> 16;   // MV_COST [J]
}

// T: uint8_t (8-bit) or uint16_t (High 10 seam, jmh_block_motion_search_u16: maxv = 2^bd - 1, the
// quarter-pel samples clipped to it; a 16x16 cost needs 19 bits, the key's 13-bit order still fits)
template <class T>
__global__ __launch_bounds__(256) void k_block_search(const jmh_block_search *reqs, jmh_block_result *out, const T *cur, const T *ref,
                                                      int W, int H, int had, int maxv) {
    __shared__ T org[256];
    __shared__ unsigned red[4];
    __shared__ int csum[9];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const jmh_block_search &q = reqs[blockIdx.x];
    const int bt = q.blocktype, bw = c_blc[bt][0], bh = c_blc[bt][1];
    const int px0 = 16 * q.mb_x + 4 * q.block_x, py0 = 16 * q.mb_y + 4 * q.block_y;   // block origin (pixels)
    const int lf = q.lambda_factor, pmx = q.pred_mv[0], pmy = q.pred_mv[1];
    const bool ffs = q.search_mode == 0;
    const bool check00 = !ffs && bt == 1 && q.slice_p;
    if (tid < bw * bh) org[tid] = cur[(py0 + tid / bw) * W + px0 + tid % bw];
    __syncthreads();
    // ---- full pel
    const int npos = (2 * q.search_range + 1) * (2 * q.search_range + 1);
    unsigned best = 0xFFFFFFFFu;
    for (int k = tid - (ffs ? 1 : 0); k < npos; k += 256) {
        int mx, my;
        if (k < 0) { mx = 0; my = 0; }                          // FFS: the (0,0) pre-check, order 0
        else { int sx, sy; spiral_pos(k, sx, sy); mx = q.centre[0] + sx; my = q.centre[1] + sy; }
        int cost = mv_cost_lf(lf, 2, mx, my, pmx, pmy);
        if (check00 && mx == 0 && my == 0) cost -= (lf * 16) >> 16;   // WEIGHTED_COST(lambda_factor, 16)
        for (int y = 0; y < bh; y++)
            for (int x = 0; x < bw; x++) cost += abs((int)org[y * bw + x] - rpx(ref, W, H, px0 + mx + x, py0 + my + y));
        const unsigned order = k < 0 ? 0u : (unsigned)(ffs ? k + 1 : k);
        best = min(best, ((unsigned)(cost + BKOFF) << 13) | order);
    }
    best = wave_min_u32(best);
    if (lane == 0) red[wave] = best;
    __syncthreads();
    best = min(min(red[0], red[1]), min(red[2], red[3]));
    const unsigned order = best & 8191u;
    int fmx, fmy;
    if (ffs && order == 0) { fmx = 0; fmy = 0; }
    else { int sx, sy; spiral_pos((int)order - (ffs ? 1 : 0), sx, sy); fmx = q.centre[0] + sx; fmy = q.centre[1] + sy; }
    const int fcost = (int)(best >> 13) - BKOFF;
    // ---- sub pel (SubPelBlockMotionSearch [J], search_pos2 = search_pos4 = 9)
    int min_mcost = had ? BIGCOST : fcost;
    const bool check_pos0 = bt == 1 && fmx == 0 && fmy == 0 && had && q.slice_p;
    const int nsx = bw >> 2, nsub = nsx * (bh >> 2);
    int qx = 4 * fmx, qy = 4 * fmy;
    for (int pass = 0; pass < 2; pass++) {
        const int step = pass == 0 ? 2 : 1, min_pos = pass == 0 ? (had ? 0 : 1) : 1;
        if (tid < 9) csum[tid] = 0;
        __syncthreads();
        for (int task = tid; task < 9 * nsub; task += 256) {
            const int c = task / nsub, sb = task - c * nsub;
            if (c < min_pos) continue;
            const int cx = qx + step * sp9x(c), cy = qy + step * sp9y(c);
            const int ox = 4 * (sb % nsx), oy = 4 * (sb / nsx);
            int d[16];
#pragma unroll
            for (int y = 0; y < 4; y++)
#pragma unroll
                for (int x = 0; x < 4; x++)
                    d[4 * y + x] = (int)org[(oy + y) * bw + ox + x] - qpel_direct(ref, W, H, 4 * (px0 + ox + x) + cx, 4 * (py0 + oy + y) + cy, maxv);
            atomicAdd(&csum[c], satd4x4(d, had));
        }
        __syncthreads();
        if (tid == 0) {
            int bpos = 0;
            for (int c = min_pos; c < 9; c++) {
                const int cx = qx + step * sp9x(c), cy = qy + step * sp9y(c);
                int mcost = mv_cost_lf(lf, 0, cx, cy, pmx, pmy);
                if (pass == 0 && check_pos0 && c == 0) mcost -= (lf * 16) >> 16;
                mcost += csum[c];
                if (mcost < min_mcost) { min_mcost = mcost; bpos = c; }
            }
            csum[0] = bpos;                                     // broadcast (read after the barrier)
            red[0] = (unsigned)min_mcost;
        }
        __syncthreads();
        const int bpos = csum[0];
        min_mcost = (int)red[0];
        qx += step * sp9x(bpos);
        qy += step * sp9y(bpos);
        __syncthreads();
    }
    if (tid == 0) {
        jmh_block_result &r = out[blockIdx.x];
        r.mv[0] = qx; r.mv[1] = qy;
        r.min_mcost = min_mcost;
        r.fullpel_mv[0] = fmx; r.fullpel_mv[1] = fmy;
        r.fullpel_cost = fcost;
    }
}

hipError_t jmh_launch_block_search(int n, const jmh_block_search *reqs, jmh_block_result *out, const uint8_t *cur, const uint8_t *ref, int W,
                                   int H, int had, hipStream_t st) {
    hipLaunchKernelGGL(k_block_search<uint8_t>, dim3(n), dim3(256), 0, st, reqs, out, cur, ref, W, H, had, 255);
    return hipGetLastError();
}
hipError_t jmh_launch_block_search_u16(int n, const jmh_block_search *reqs, jmh_block_result *out, const uint16_t *cur, const uint16_t *ref,
                                       int W, int H, int had, int bit_depth, hipStream_t st) {
    hipLaunchKernelGGL(k_block_search<uint16_t>, dim3(n), dim3(256), 0, st, reqs, out, cur, ref, W, H, had, (1 << bit_depth) - 1);
    return hipGetLastError();
}
