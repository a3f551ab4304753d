// jmh_device.h — device-side types and constants shared by the MI355X kernels (gfx950 only).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "../../include/jmhip.h"

#define SRMAX 32                         // LDS-resident FFS window: SearchRange <= 32
#define SIDE_MAX (2 * SRMAX + 1)
#define NPOS_MAX (SIDE_MAX * SIDE_MAX)   // 4225 search positions
#define QPAD 4                           // quarter-pel plane padding (== oracle JMO_PAD)
#define NT 256                           // threads per finalize / unit workgroup
#define NTA 512                          // threads per analysis workgroup (8 waves, 2 per SIMD)
#define BIGCOST (1 << 20)

// Per-macroblock analysis results, written by k_mb_analyse (three roles on separate
// workgroups) and consumed by k_mb_final on the same wavefront diagonal.
struct MbScratch {
    int16_t all_mv[8][16][2];            // best MV per block type (1..7) and 4x4 block
    int32_t motion_cost[8][4];           // per block type: partition cost (16x8/8x16 block, P8x8 b8)
    int32_t best8x8;                     // P8x8 sub-mode per b8, 4 bits each
    int32_t cost8x8;
    int32_t skipx, skipy;                // FindSkipModeMotionVector
    int32_t i4cost, i4cbp, i4blk;        // Intra4x4 decision (with its reconstruction)
    int32_t i16cost, i16mode, c_mode;
    int8_t ipred[16];
    int16_t i4lev[16][16];               // Intra4x4 levels in scan order
    uint8_t i4rec[256];                  // Intra4x4 reconstruction of the MB
};

struct DevParams {
    int W, H, Wc, Hc, mbw, mbh;
    int sr, side, npos;
    int search_mode, use_hadamard, restrict_sr;
    int inter_search[8];
    int qstride, qplane;
    const uint8_t *orgY, *orgU, *orgV;
    const uint8_t *refY, *refU, *refV;
    const uint8_t *qpel;
    uint8_t *recY, *recU, *recV;
    uint8_t *dbkY, *dbkU, *dbkV;   // deblocked reconstruction (null: no deblocking on the device)
    int lf_disable, lf_offA, lf_offB;   // disable_deblocking_filter_idc, FilterOffsetA/B (= 2 x div2)
    int16_t *mv;
    int8_t *refidx;
    int8_t *ipred;
    jmh_mb_result *res;
    MbScratch *scr;
    unsigned long long *prof;   // debug phase timestamps (null: off)
    int prof_mb;
    int slice_type, qp, lambda_mode, lambda_motion, cqp_off;
    int diag, y_min, ndiag;     // wavefront diagonal of this launch: mbx + 2*mby == diag, ndiag MBs
};
