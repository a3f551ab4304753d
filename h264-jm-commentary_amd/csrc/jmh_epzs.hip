// jmh_epzs.hip — k_mb_epzs: the motion-search half of encode_one_macroblock [J] with SearchMode 3
// (EPZSPelBlockMotionSearch as restated in oracle/encode.c epzs_search, docs/JM_SEMANTICS.md
// items 33-40), ONE WAVE per P macroblock.
//
// EPZS evaluates few positions per search (41 ordered predictors, then a handful of diamond
// rounds) but its 41 searches are strictly sequential (MVP, spatial memory and earlier-type
// predictors read the searches before).  So the search is latency-bound, and one wave per MB with
// wave-synchronous LDS (no workgroup barrier anywhere) beats a workgroup of waves meeting at
// barriers:
//   * full pel: lane i evaluates predictor i (i < 41) — the whole block SAD per lane from the
//     LDS window by aligned dwords + v_alignbyte + v_sad_u8 — one wave minimum of
//     (cost << 6 | i) keys is JM's strict '<' scan in list order; a refinement round is one
//     pattern point per lane (4 or 12 lanes) and one wave minimum;
//   * sub pel: the block's b / h / j neighbourhood at its full-pel MV in three small planes (b
//     and j from unclipped horizontal taps, so j is one vertical 6-tap per sample; G is the window),
//     lane task = (candidate, 4x4 sub-block) with a packed int16 Hadamard, DPP sums over the
//     candidate's lanes, one wave minimum per pass.
// LDS: a 120x120 window (+ ~4.5 KB state = 18.6 KB: eight macroblocks per CU, so a 2160p tick's
// ~2,000 P macroblocks run in one round).  A block's reach is MB +- (2 SR + 4) when each search
// centres on its own MVP; the window covers MB +- 52 around the MB's 16x16 MVP / 4 (the centre
// of most searches), i.e. everything when 2 SR + 4 <= 52, and a sample outside it is read from
// the reference picture in global memory instead (UMV-clamped, as the window load clamps): per
// lane in the full-pel SADs, per search (into a small neighbourhood plane) for the sub-pel planes.
// Results land in MbScratch exactly like the other search kernels (the intra workgroups and
// k_mb_final are shared).
// High 10 (pel = uint16_t): the same kernel on 16-bit samples -- two samples per dword, v_sad_u16
// for the SADs, the packed-int16 Hadamard on 16-bit differences (|d| <= 1023 keeps every stage in
// range), int32 horizontal taps, and the EPZS thresholds times 1 << (BitDepthY - 8).
#include "jmh_epzs.h"

// JM10X: built with JM >= 10's EPZS options (EPZSDualRefinement, EPZSSubPelME, the adaptive
// thresholds: items 46, 61, 62); the instantiation without them (all off, e.g. config 3's JM 8.6
// EPZS) constant-folds those branches away instead of testing them at run time
template <class pel, bool JM10X>
__global__ __launch_bounds__(NTE) void k_mb_epzs(const TickArgs t) {
    __shared__ EpzS<pel> s;
    const int b = xcd_block(blockIdx.x, t.pre[t.nP]), lane = threadIdx.x;   // XCD-aware (jmh_device.h)
    if (b >= t.pre[t.nP]) return;
    const int e = tick_entry(t, b);
    DevParams d = tick_params(t, e);
    if constexpr (!JM10X) { d.epzs_dual = 0; d.epzs_subpel = 0; d.epzs_maxts = 0; }
    if constexpr (sizeof(pel) == 1) { d.maxv = 255; d.qpbd = 0; }   // 8-bit samples: constants
    const int mby = d.y_min + (b - t.pre[e]), mbx = d.diag - 2 * mby;
    MbScratch *scr = d.scr + mby * d.mbw + mbx;
    const bool prof = d.prof && lane == 0 && d.prof_mb == mby * d.mbw + mbx;
    const unsigned long long bt0 = t.bprof ? wall_clock64() : 0;   // debug (JMH_BLOCK_PROF): role 4
    if (prof) d.prof[32] = wall_clock64();
    const EWin<pel> wn = epzs_load_mb(d, s, mbx, mby, lane);
    wave_lds_sync();
    if (prof) d.prof[33] = wall_clock64();
    // PartitionMotionSearch [J] order: 16x16, 16x8 (2), 8x16 (2), then per 8x8 block the sub-modes
    // 4..7 and its best sub-mode (read through best8x8)
    int best8x8 = 0, cost8x8 = 0;
    epzs_block<1>(d, s, wn, 0, 0, 0, 0, 0, prof);
    if (prof) d.prof[34] = wall_clock64();
    epzs_block<2>(d, s, wn, 0, 0, 0, 0, 0, prof);
    epzs_block<2>(d, s, wn, 0, 2, 1, 0, 0, prof);
    epzs_block<3>(d, s, wn, 0, 0, 0, 0, 0, prof);
    epzs_block<3>(d, s, wn, 2, 0, 1, 0, 0, prof);
    if (prof) d.prof[35] = wall_clock64();
#pragma unroll 1
    for (int b8 = 0; b8 < 4; b8++) {
        const int X = 2 * (b8 & 1), Y = 2 * (b8 >> 1);
        epzs_block<4>(d, s, wn, X, Y, b8, b8, best8x8, prof);
        epzs_block<5>(d, s, wn, X, Y, b8, b8, best8x8, prof);
        epzs_block<5>(d, s, wn, X, Y + 1, b8, b8, best8x8, prof);
        epzs_block<6>(d, s, wn, X, Y, b8, b8, best8x8, prof);
        epzs_block<6>(d, s, wn, X + 1, Y, b8, b8, best8x8, prof);
        epzs_block<7>(d, s, wn, X, Y, b8, b8, best8x8, prof);
        epzs_block<7>(d, s, wn, X + 1, Y, b8, b8, best8x8, prof);
        epzs_block<7>(d, s, wn, X, Y + 1, b8, b8, best8x8, prof);
        epzs_block<7>(d, s, wn, X + 1, Y + 1, b8, b8, best8x8, prof);
        int mc8 = BIGCOST, bm = 0;
        for (int mode = 4; mode <= 7; mode++) {
            if (!inter_on(d.isr, mode)) continue;
            const int c = s.motion_cost[mode][b8];
            if (c < mc8) { mc8 = c; bm = mode; }
        }
        best8x8 |= bm << (4 * b8);
        cost8x8 += mc8;
        if (prof) d.prof[36 + b8] = wall_clock64();
    }
    // results: MVs and partition costs of types 1..7, P8x8 decision, FindSkipModeMotionVector
    for (int i = lane; i < 7 * 32; i += NTE) {
        const int m = 1 + i / 32, k = (i & 31) >> 1, c = i & 1;
        scr->all_mv[m][k][c] = s.all_mv[m][k][c];
    }
    if (d.epzs_maxts)                                   // item 61: the full-pel costs for the neighbours
        for (int i = lane; i < 7 * 16; i += NTE) scr->fpc[i >> 4][i & 15] = s.fpc[i >> 4][i & 15];
    if (lane < 28) scr->motion_cost[1 + lane / 4][lane & 3] = s.motion_cost[1 + lane / 4][lane & 3];
    else if (lane == 32) { scr->best8x8 = best8x8; scr->cost8x8 = cost8x8; }
    else if (lane == 48) {
        int pcx, pcy;
        set_mvp(NbBorder{s.bd}, 0, 0, 16, 16, pcx, pcy);
        NbBorder nbv{s.bd};
        int ra = -1, ax = 0, ay = 0, rb = -1, bx = 0, by = 0;
        const bool aa = nbv(-1, 0, ra, ax, ay), ab = nbv(0, -1, rb, bx, by);
        const bool zl = !aa || (ra == 0 && ax == 0 && ay == 0), za = !ab || (rb == 0 && bx == 0 && by == 0);
        scr->skipx = (za || zl) ? 0 : pcx;
        scr->skipy = (za || zl) ? 0 : pcy;
    }
    if (prof) d.prof[40] = wall_clock64();
    if (t.bprof && lane == 0) {
        t.bprof[3 * blockIdx.x] = bt0;
        t.bprof[3 * blockIdx.x + 1] = wall_clock64();
        t.bprof[3 * blockIdx.x + 2] = 4;
    }
}

hipError_t jmh_launch_epzs(const TickArgs &t, hipStream_t st) {
    if (t.pre[t.nP] == 0) return hipSuccess;
    const dim3 g(xcd_grid(t.pre[t.nP]));
    const bool x = t.epzs_dual || t.epzs_subpel || t.epzs_maxts;
    if (t.bd > 8) {
        if (x) hipLaunchKernelGGL((k_mb_epzs<uint16_t, true>), g, dim3(NTE), 0, st, t);
        else hipLaunchKernelGGL((k_mb_epzs<uint16_t, false>), g, dim3(NTE), 0, st, t);
    } else {
        if (x) hipLaunchKernelGGL((k_mb_epzs<uint8_t, true>), g, dim3(NTE), 0, st, t);
        else hipLaunchKernelGGL((k_mb_epzs<uint8_t, false>), g, dim3(NTE), 0, st, t);
    }
    return hipGetLastError();
}
