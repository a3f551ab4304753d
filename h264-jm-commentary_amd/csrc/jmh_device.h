// jmh_device.h — device-side types and constants shared by the MI355X kernels (gfx950 only).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "../../include/jmhip.h"

#define SRMAX 32                         // LDS-resident FFS window: SearchRange <= 32
#define SIDE_MAX (2 * SRMAX + 1)
#define NPOS_MAX (SIDE_MAX * SIDE_MAX)   // 4225 search positions
#define WIN_MAX (2 * SRMAX + 16)         // 80x80 integer reference window
#define WSTRIDE 84                       // window row stride: >= WIN_MAX + 3 (aligned over-read)
#define QPAD 4                           // quarter-pel plane padding (== oracle JMO_PAD)
#define NT 256                           // threads per macroblock workgroup (4 waves)
#define BIGCOST (1 << 20)

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
    int16_t *mv;
    int8_t *refidx;
    int8_t *ipred;
    jmh_mb_result *res;
    const int16_t *spiral;      // [npos][2] (x, y)
    const int16_t *spiral_of;   // window raster index -> spiral index
    int slice_type, qp, lambda_mode, lambda_motion, cqp_off;
    int diag, y_min;            // wavefront diagonal of this launch: mbx + 2*mby == diag
};
