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
// JMH_I4WAVE 1: a P macroblock's intra decisions run on wave 7 of its motion-search workgroup on
// their own schedule (the seven search waves meet at LDS-counter barriers, never at s_barrier, which
// would wait for wave 7), so the Intra4x4 chain is off the search's stage chain; 0: the Intra4x4
// steps ride in the stages' sub-pel phases on waves 6 and 7 (A/B: -DJMH_I4WAVE=0).  The variant
// measured slower (1143 vs 1168 MP/s, profiles/r8a_i4wave_ab.txt) and is kept for A/B only: it is
// correct only while intra_wave and every search stage after the split are free of __syncthreads
// (an s_barrier would pair arrivals of unrelated program points), and no test builds it.
#ifndef JMH_I4WAVE
#define JMH_I4WAVE 0
#endif
#if JMH_I4WAVE && !defined(JMH_I4WAVE_AB)
#error "JMH_I4WAVE is an A/B-only variant: define JMH_I4WAVE_AB to build it (see the comment above)"
#endif
#define NTS (JMH_I4WAVE ? 448 : NTA)     // threads of the FFS position strips (the search waves)
#define NPK (JMH_I4WAVE ? 11 : 10)       // FFS search positions per search thread (a column strip):
                                         //   65 x ceil(65 / NPK) strips <= NTS
#define NPK2 ((NPK + 1) / 2)             // packed order-key pairs per thread
#define ORDTAB_SPOS (NPK2 * NTA)         // ordtab: the spiral-index -> position table after the keys
#define BIGCOST (1 << 20)
#define PMAX 33                          // pictures per wavefront tick (pipelined pictures in flight;
                                         // 2160p needs 508 / PIPE_LAG + 1 = 33)
// A picture's macroblock (x, y) reads its reference (the previous picture, deblocked) at pixel
// offsets -68..+83 from the MB origin: window centre |MVP/4| <= SR, positions +-SR around it,
// +-3/4 sub-pel, the 6-tap support and the LDS window margin (SR 32).  The farthest samples, rows
// and columns 0..3 of MB (x+5, y+5), are final once that MB's own final kernel (DeblockMb of its
// left and top edges) has run; samples 13..15 of MBs x+4 / y+4 wait for the same MB.  So picture q
// may run diagonal d once picture q-1 has completed diagonal (x+5) + 2(y+5) = d + 15: a lag of
// PIPE_LAG diagonals (tests/test_gpu_parity.py checks pipelined == sequential at the window edge).
#define PIPE_LAG 16
// SearchRange > 32 (EPZS only, up to 64): the same argument with the reach 16 + 2 SR + 3 pixels, i.e.
// MB (x + R, y + R), R = (19 + 2 SR) / 16 (5 at SR 32, 9 at SR 64): a lag of 3 R + 1 diagonals (the
// RD stage schedule's lag follows the same reach, jmhip_abi.hip rdo_schedule)
__host__ __device__ __forceinline__ int ref_reach(int sr) { return sr <= SRMAX ? 5 : (19 + 2 * sr) / 16; }
__host__ __device__ __forceinline__ int pipe_lag(int sr) { return sr <= SRMAX ? PIPE_LAG : 3 * ref_reach(sr) + 1; }

// Per-macroblock analysis results, written by k_mb_analyse (three roles on separate
// workgroups) and consumed by k_mb_final on the same wavefront diagonal.
struct MbScratch {
    int16_t all_mv[8][16][2];            // best MV per block type (1..7) and 4x4 block
    uint16_t fpc[7][16];                 // EPZS: each search's full-pel cost per block type 1..7 and
                                         //   4x4, saturated (the neighbours' distortion of item 61)
    int32_t motion_cost[8][4];           // per block type: partition cost (16x8/8x16 block, P8x8 b8)
    int32_t best8x8;                     // P8x8 sub-mode per b8, 4 bits each
    int32_t cost8x8;
    int32_t skipx, skipy;                // FindSkipModeMotionVector
    int32_t i4cost, i4cbp, i4blk;        // Intra4x4 decision (with its reconstruction)
    int32_t i16cost, i16mode, c_mode;
    int8_t ipred[16];
    int16_t i4lev[16][16];               // Intra4x4 levels in scan order
    alignas(4) uint8_t i4rec[512];       // Intra4x4 reconstruction of the MB (256 samples of pel)
    // Intra8x8 decision (k_mb_intra8, Transform8x8Mode only)
    int32_t i8cost, i8cbp, i8modes;      // i8modes: 4 bits per 8x8 block
    int16_t i8lev[16][16];               // levels in the CAVLC interleave (jmh_mb_result.luma)
    alignas(4) uint8_t i8rec[512];
};

// RDOptimization 1: the per-picture RD state, stored right after the picture's MbScratch array
// (PicParams.scr + mbw * mbh) so that the kernel arguments stay within 4 KB: the lambdas from the
// host, the slices' CABAC states (contexts + codIRange, jmh_cabac_rate.h) and what every coded
// macroblock leaves for its neighbours' context selection
struct jmr_mbinfo;
struct RdoPic {
    double lambda;                       // lambda_mode (jmh_frame_params.lambda_rd)
    int32_t lf;                          // LAMBDA_FACTOR(sqrt(lambda_mode)) of the motion searches
    int32_t pad;
    uint8_t *cab;                        // [slice][JMR_NCTX] context states (state << 1 | valMPS)
    uint32_t *range;                     // [slice] codIRange (CAVLC: the mb_skip_run so far)
    jmr_mbinfo *mbi;                     // [MB]
};

// byte offset of the RdoPic in a picture's MbScratch allocation (16-aligned)
__host__ __device__ __forceinline__ size_t rdo_pic_offset(size_t nmb) { return (nmb * sizeof(MbScratch) + 15) & ~(size_t)15; }

struct DevParams {
    int W, H, Wc, Hc, mbw, mbh;
    int sr, side, npos;
    int search_mode, use_hadamard, restrict_sr;
    int isr;                    // InterSearch16x16..4x4 as bits 1..7 (a mask: a per-thread array
                                // indexed at run time would put the whole DevParams in scratch)
    int t8;                     // Transform8x8Mode (High profile)
    int epzs_dual;              // EPZSDualRefinement (SearchMode 3)
    int epzs_subpel;            // EPZSSubPelME (item 62) and its EPZSSubPelThresScale
    int epzs_spts;
    int epzs_mints, epzs_maxts; // EPZSMinThresScale / EPZSMaxThresScale (item 61; maxts 0: off)
    int slice_mbs;              // SliceMode 1: MBs per slice (the whole picture for one slice)
    int maxv, qpbd;             // (1 << bit depth) - 1 (Clip1), QpBdOffsetY = QpBdOffsetC = 6 (bit depth - 8)
    // plane pointers are byte addresses of uint8_t (bit depth 8) or uint16_t (9 / 10) samples:
    // the kernels templated on the sample type cast them (spl<pel>)
    const uint8_t *orgY, *orgU, *orgV;
    const uint8_t *refY, *refU, *refV;
    uint8_t *recY, *recU, *recV;
    uint8_t *dbkY, *dbkU, *dbkV;   // deblocked reconstruction (null: no deblocking on the device)
    int lf_disable, lf_offA, lf_offB;   // disable_deblocking_filter_idc, FilterOffsetA/B (= 2 x div2)
    int16_t *mv;
    int8_t *refidx;
    int8_t *ipred;
    const int16_t *tmv;         // EPZS temporal predictors: the previous picture's MVs / ref_idx
    const int8_t *tref;         //   (null: no previous picture)
    const uint32_t *ordtab;     // FFS: JM order keys of every thread's positions (ordtab_fill)
    jmh_mb_result *res;
    MbScratch *scr;
    unsigned long long *prof;   // debug phase timestamps (null: off)
    int prof_mb;
    int slice_type, qp, lambda_mode, lambda_motion, cqp_off;
    int qsel;                   // quantisation rounding selector of this slice (q_round, jmh_common.h)
    int diag, y_min;            // wavefront diagonal of this picture in the launch: mbx + 2*mby == diag
                                //   (RDOptimization 1: diag = the stage of the RD schedule)
    int rdo;                    // RDOptimization 1 (the RD kernels; no 16x16 zero-vector biases)
    int lf;                     // LAMBDA_FACTOR of the motion searches: 65536 * lambda_motion (RDO
                                //   off, integer lambda), the host's RDO one (RDOptimization 1)
    double lambda_rd;           // RDOptimization 1: lambda_mode
    int cavlc;                  // RDOptimization 1 with SymbolMode 0: CAVLC rates (jmh_cavlc_rate.h, item 64);
                                //   RdoPic.range[slice] then holds the slice's mb_skip_run so far
    const RdoPic *rp;           // RDOptimization 1: the picture's RD state
    int cip;                    // UseConstrainedIntraPred: intra prediction from intra neighbours only (intra_avail)
    int i16c;                   // k_mb_flow: the P macroblock's Intra16x16 / chroma decisions run on
                                //   me_mb's idle waves (intra slot 11); 0: k_mb_analyse's intra roles do them
};

// Neighbour MB availability (6.4.8 / JM getNeighbour): inside the picture and in the current
// slice.  Slices are runs of slice_mbs MBs in raster order and every neighbour precedes the MB,
// so "same slice" is "address >= the slice's first MB".  One slice: the picture-edge rules.
struct MbAvail { bool L, T, TL, TR; };
__device__ __forceinline__ MbAvail mb_avail(const DevParams &d, int mbx, int mby) {
    const int a = mby * d.mbw + mbx, first = a - a % d.slice_mbs;
    MbAvail v;
    v.L = mbx > 0 && a - 1 >= first;
    v.T = mby > 0 && a - d.mbw >= first;
    v.TL = mbx > 0 && mby > 0 && a - d.mbw - 1 >= first;
    v.TR = mby > 0 && mbx + 1 < d.mbw && a - d.mbw + 1 >= first;
    return v;
}
// ... for intra prediction (samples and the Intra4x4 / 8x8 mode prediction): with
// UseConstrainedIntraPred an inter (or skipped) neighbour is "not available for Intra prediction"
// (8.3.1.1 dcPredModePredictedFlag, 8.3.1.2, 8.3.2, 8.3.3, 8.3.4); its refidx (-1: intra) is final
// by the time the MB's intra analysis runs
__device__ __forceinline__ MbAvail intra_avail(const DevParams &d, int mbx, int mby) {
    MbAvail v = mb_avail(d, mbx, mby);
    if (d.cip && d.slice_type == JMH_P_SLICE) {
        const int W4 = d.W >> 2, a = 4 * mby * W4 + 4 * mbx;   // the MB's top-left 4x4
        v.L = v.L && d.refidx[a - 1] < 0;
        v.T = v.T && d.refidx[a - W4] < 0;
        v.TL = v.TL && d.refidx[a - W4 - 1] < 0;
        v.TR = v.TR && d.refidx[a - W4 + 4] < 0;
    }
    return v;
}

// One wavefront tick: the same diagonal step for up to PMAX pictures in flight, each on its own
// diagonal (kernel argument, by value; ~2.4 KB).  Entries [0, nP) are P pictures.
struct PicParams {
    const uint8_t *org, *ref;            // 4:2:0 pictures, Y then U then V
    uint8_t *rec, *dbk;                  // dbk null: no deblocking
    int16_t *mv;
    int8_t *refidx, *ipred;
    const int16_t *tmv;                  // previous picture's motion field (EPZS temporal predictors)
    const int8_t *tref;
    jmh_mb_result *res;
    MbScratch *scr;
    int32_t lambda_mode, lambda_motion;
    int16_t diag, y_min;
    int16_t qsel;                        // q_round selector (JM 8.6 !P / JM >= 10 2 + quant_offset)
    int8_t slice_type, qp, cqp_off, lf_disable, lf_offA, lf_offB;   // packed: PMAX entries fit 4 KB
};
struct TickArgs {
    int W, H, mbw, mbh, sr, search_mode, use_hadamard, restrict_sr;
    int inter_search[8];
    unsigned long long *prof;
    int prof_mb;
    unsigned long long *bprof;           // debug (JMH_BLOCK_PROF): per-block start / end / role
    unsigned long long *bprof_fin;       //   ... of k_mb_final (role 3)
    int me_in_analyse;                   // 1: k_mb_analyse runs the FFS searches; 0: k_mb_me_full did
                                         //   (full search, SearchMode -1, or EPZS, SearchMode 3)
    int t8;                              // Transform8x8Mode: k_mb_intra8 ran, k_mb_final decides 4x4 / 8x8
    int epzs_dual;                       // EPZSDualRefinement (k_mb_epzs)
    int epzs_subpel, epzs_spts;          // EPZSSubPelME, EPZSSubPelThresScale
    int epzs_mints, epzs_maxts;          // EPZSMinThresScale, EPZSMaxThresScale
    int slice_mbs;                       // SliceMode 1: MBs per slice (>= 1; mbw * mbh for one slice)
    int cip;                             // UseConstrainedIntraPred
    int bd;                              // bit depth: 8 (uint8_t samples) or 9 / 10 (uint16_t, High 10)
    int rdo;                             // RDOptimization 1: k_rdo_inter + k_rdo_intra + k_rdo_final on the stage
                                         //   (1: CABAC rates, 2: CAVLC rates, SymbolMode 0)
    const int32_t *sched, *soff;         //   schedule: MB addresses in stage order, offsets per stage
    void *rscr;                          //   the tick's candidate scratch (RdoScr per tick MB)
    void *ffs;                           //   SearchMode 0: the tick MBs' SAD tables (null: the searches scan)
    unsigned long long ffs_slot;         //   ... bytes per tick MB (ffs_slot_bytes)
    const uint32_t *ordtab;              // FFS order keys, [NPK2][NTA] packed pairs (jmh_create)
    int npic, nP;
    int pre[PMAX + 1];                   // MB prefix sums over the entries
    PicParams p[PMAX];
};
// RDOptimization 1 + SearchMode 0: bytes of one tick MB's SAD table (jmh_epzs.h ffs_table_build)
__host__ __device__ __forceinline__ size_t ffs_slot_bytes(int sr) {
    const size_t np = (size_t)(2 * sr + 1) * (2 * sr + 1);
    return np * 5 * 8;                   // five phases of four u16 SADs per position
}
static_assert(sizeof(TickArgs) <= 4096, "TickArgs is passed by value in the kernel argument segment");

// ---------------------------------------------------------------------------------------------
//  Dataflow wavefront (k_mb_flow, SearchMode 0 with 8-bit samples, RDO off): one persistent launch
//  per segment of ticks.  The host flattens the segment's ticks into a list of macroblocks in tick
//  order; a workgroup claims the next one with an atomic ticket, waits until the macroblocks it
//  depends on are done (per-MB flags), and runs its whole encode_one_macroblock -- motion search,
//  intra decisions, the final -- before publishing its own flag.  Every dependency precedes the
//  MB in tick order, and every claimed ticket belongs to a resident workgroup, so the wait always
//  ends.
// ---------------------------------------------------------------------------------------------
// per ring entry, copied to the device with each segment: the picture's parameters and the flag
// generations that mark its macroblocks (and its reference picture's) done
struct FlowPic {
    PicParams pp;
    uint32_t gen;                        // flags[entry][mb] >= gen: MB done (the entry's use count)
    int32_t ref_entry;                   // ring entry of the reference picture (-1: none / explicit buffer)
    uint32_t ref_gen;
    int32_t pad;
};
struct FlowArgs {
    int W, H, mbw, mbh, sr, search_mode, use_hadamard, restrict_sr;
    int isr;                             // InterSearch bits 1..7
    int slice_mbs;
    const uint32_t *ordtab;
    unsigned long long *prof;
    int prof_mb;
    const FlowPic *pics;                 // [nring]
    const uint32_t *items;               // the segment's MBs in tick order: entry << 24 | mby << 12 | mbx
    int nitems;
    int nmb, nring;
    unsigned *head;                      // ticket counter (monotonic over launches)
    unsigned base;                       // its value at this launch's first ticket
    uint32_t *flags;                     // [nring][nmb] generations
    unsigned *err;                       // host-visible: [0] 1 = a dependency wait timed out, 2 = a ticket /
                                         //   item out of range ([1] ticket, [2] item)
    unsigned long long *fprof;           // debug (JMH_FLOW_PROF=<launch>): per ticket 6 words -- start,
                                         //   dependencies met, analysis done, final done, flag stored,
                                         //   hardware id << 32 | item (null: off)
};
#define FLOW_ITEM(e, x, y) (((uint32_t)(e) << 24) | ((uint32_t)(y) << 12) | (uint32_t)(x))

// XCD-aware block order.  Workgroups are dispatched round-robin over the 8 XCDs (hardware block b
// runs on XCD b % 8), each with its own L2.  A launch of n logical blocks uses 8 * ceil(n / 8)
// hardware blocks and gives every XCD one contiguous run of the logical list, whose consecutive
// entries are neighbouring MBs of one picture's diagonal (search windows and MC reads overlap), so
// they share that XCD's L2.  Returns the logical block (>= n: idle).
#define NXCD 8
__device__ __forceinline__ int xcd_block(int b, int n) { return (b % NXCD) * ((n + NXCD - 1) / NXCD) + b / NXCD; }
__host__ __device__ __forceinline__ int xcd_grid(int n) { return NXCD * ((n + NXCD - 1) / NXCD); }

// entry of MB index idx (pre[e] <= idx < pre[e + 1]); uniform scalar loop
__device__ __forceinline__ int tick_entry(const TickArgs &t, int idx) {
    int e = 0;
    while (e + 1 < t.npic && t.pre[e + 1] <= idx) e++;
    return e;
}
__device__ __forceinline__ bool inter_on(int isr, int mode) { return (isr >> mode) & 1; }
__device__ __forceinline__ DevParams tick_params(const TickArgs &t, int e) {
    DevParams d;
    const PicParams &q = t.p[e];
    d.W = t.W; d.H = t.H; d.Wc = t.W >> 1; d.Hc = t.H >> 1; d.mbw = t.mbw; d.mbh = t.mbh;
    d.sr = t.sr; d.side = 2 * t.sr + 1; d.npos = d.side * d.side;
    d.search_mode = t.search_mode; d.use_hadamard = t.use_hadamard; d.restrict_sr = t.restrict_sr;
    d.isr = 0;
#pragma unroll
    for (int i = 1; i < 8; i++) d.isr |= (t.inter_search[i] != 0) << i;
    d.t8 = t.t8;
    d.epzs_dual = t.epzs_dual;
    d.epzs_subpel = t.epzs_subpel; d.epzs_spts = t.epzs_spts;
    d.epzs_mints = t.epzs_mints; d.epzs_maxts = t.epzs_maxts;
    d.slice_mbs = t.slice_mbs;
    d.maxv = (1 << t.bd) - 1; d.qpbd = 6 * (t.bd - 8);
    const int ps = t.bd > 8 ? 2 : 1, ls = t.W * t.H * ps, lc = ls >> 2;
    d.orgY = q.org; d.orgU = q.org + ls; d.orgV = q.org + ls + lc;
    d.refY = q.ref; d.refU = q.ref + ls; d.refV = q.ref + ls + lc;
    d.recY = q.rec; d.recU = q.rec + ls; d.recV = q.rec + ls + lc;
    d.dbkY = q.dbk; d.dbkU = q.dbk ? q.dbk + ls : nullptr; d.dbkV = q.dbk ? q.dbk + ls + lc : nullptr;
    d.lf_disable = q.lf_disable; d.lf_offA = q.lf_offA; d.lf_offB = q.lf_offB;
    d.mv = q.mv; d.refidx = q.refidx; d.ipred = q.ipred; d.res = q.res; d.scr = q.scr;
    d.tmv = q.tmv; d.tref = q.tref; d.ordtab = t.ordtab;
    d.prof = e == 0 ? t.prof : nullptr; d.prof_mb = t.prof_mb;
    d.slice_type = q.slice_type; d.qp = q.qp; d.lambda_mode = q.lambda_mode; d.lambda_motion = q.lambda_motion;
    d.cqp_off = q.cqp_off; d.qsel = q.qsel; d.diag = q.diag; d.y_min = q.y_min;
    d.rdo = t.rdo;
    d.cavlc = t.rdo == 2;
    d.i16c = 0;
    d.cip = t.cip;
    d.lf = q.lambda_motion << 16;
    d.lambda_rd = 0;
    d.rp = nullptr;
    if (t.rdo) {
        d.rp = reinterpret_cast<const RdoPic *>(reinterpret_cast<const uint8_t *>(q.scr) + rdo_pic_offset((size_t)t.mbw * t.mbh));
        d.lf = d.rp->lf;
        d.lambda_rd = d.rp->lambda;
    }
    return d;
}

// the macroblock of tick MB index m (entry e): the diagonal mbx + 2 mby == diag of the RDO-off
// wavefront, or the RD stage schedule's list (RDOptimization 1)
__device__ __forceinline__ void tick_mb(const TickArgs &t, const DevParams &d, int e, int m, int &mbx, int &mby) {
    if (t.rdo) {
        const int a = t.sched[t.soff[d.diag] + (m - t.pre[e])];
        mby = a / d.mbw;
        mbx = a - mby * d.mbw;
    } else {
        mby = d.y_min + (m - t.pre[e]);
        mbx = d.diag - 2 * mby;
    }
}

// sample-typed view of a DevParams plane pointer (bytes of uint8_t or uint16_t samples)
template <class pel> __device__ __forceinline__ pel *spl(uint8_t *p) { return reinterpret_cast<pel *>(p); }
template <class pel> __device__ __forceinline__ const pel *spl(const uint8_t *p) { return reinterpret_cast<const pel *>(p); }
