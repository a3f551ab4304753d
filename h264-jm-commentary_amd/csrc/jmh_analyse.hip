// jmh_analyse.hip — k_mb_analyse: the decision half of encode_one_macroblock [J] (RDO off) for
// every macroblock of one wavefront tick (SearchMode 0, fast full search), on 512-thread
// workgroups of two kinds:
//
//   motion search (one per P macroblock): all 41 BlockMotionSearch calls -- 16x16, 16x8, 8x16 and
//           the P8x8 sub-modes of the four 8x8 blocks -- plus FindSkipModeMotionVector, with the
//           MB's Intra4x4 decision on waves 6 and 7 between the search stages (intra_slot)
//   intra (four MBs per workgroup, 128 threads each): Intra16x16 and chroma intra-mode decisions,
//           and Intra4x4 for MBs without a motion-search workgroup (I pictures)
//
// k_mb_intra (end of file) runs the intra decisions for ticks whose search has its own kernel
// (SearchMode -1: k_mb_me_full, 3: k_mb_epzs).
//
// JM runs the 41 searches of a P macroblock one after another. The only coupling between them is
// the motion vector predictor, which reads MVs already stored inside the MB. Enumerating those
// reads (getLuma4x4Neighbour + the C-availability rules of SetMotionVectorPredictor): a 16x16 /
// 16x8 / 8x16 search reads only MB neighbours and the same partition type's earlier block; a
// P8x8 sub-mode search in 8x8 block b8 reads MB neighbours, the final (best sub-mode) MVs of the
// 8x8 blocks before b8 and the same sub-mode's earlier blocks in b8. So the 41 searches form 16
// dependent stages (the 16x16-type searches inside block 0's first two), each a set of
// independent searches evaluated together, with results identical to JM's sequential order.
// Per-mode MV arrays provide the exact neighbour view. Likewise the 16 Intra4x4 blocks only read
// blocks on earlier (x4 + 2*y4) diagonals, so they run as 10 steps of up to two blocks.
//
// Motion search data path per workgroup:
//   * 88x88 reference window (+4 margin for the 6-tap filter) and its b, h, j half-pel planes in
//     LDS, computed once per MB (SubPelBlockMotionSearch reads only LDS);
//   * SetupFastFullPelSearch's SADs of every integer position in REGISTERS, only those the next
//     searches read: each thread owns a column strip of NPK positions and keeps 2 packed u16 pairs
//     per position -- first the four 8x8 SADs (16x16 / 16x8 / 8x16 are sums of them; kept in LDS
//     for block 0's stages), then per 8x8 block its four 4x4 SADs (recomputed per block).  Any
//     partition reduces with plain 32-bit adds of packed pairs (no carries: a half never exceeds
//     2 x 16320).  The small table keeps the workgroup at 128 VGPRs (two per CU);
//   * cost = SAD + (lambda * mvbits)(x) + (lambda * mvbits)(y) from one u16 LDS table, key =
//     cost << 13 | JM order (0 for the (0,0) pre-check, else spiral index + 1), DPP wave min;
//   * sub-pel on one wave per search: a quad of lanes per candidate, DPP butterflies / packed
//     int16 Hadamard, one wave minimum per half / quarter pass.
#include "jmh_common.h"
#ifndef JMH_EXP
#define JMH_EXP 0                             // tools/valu_split.sh builds variants without parts
#endif
#include "jmh_intra8.h"
#include "jmh_intra.h"
#include "jmh_i4.h"
#ifdef JMH_FLOW_TU
#include "jmh_final.h"          // k_mb_flow (jmh_flow.hip compiles this file with JMH_FLOW_TU)
#endif

#define MVB_OFF 544                           // mvbits LUT: |4*(centre+offset) - pmv| <= 256 + 259
#define MVB_LEN 1104
#define PLS (WIN_DIM_MAX * WST + 32)          // stride between the G, b, h, j planes
#define MAXNS 7                               // searches per stage (block 0 stage 0: 3 + 4)

struct MeS {
    uint8_t org[256];
    Border bd;
    IntraNb<uint8_t> nb;
    int16_t all_mv[8][16][2];
    int motion_cost[8][4];
    unsigned red[NTS / 64][MAXNS];            // per search wave, per search of the stage: argmin keys
    int pmv[MAXNS][2];                        // MVPs of the next stage's searches (forwarded)
    uint16_t mvc[MVB_LEN];                    // lambda * mvbits(v) at [v + MVB_OFF] (|v| <= 4*2*SR + 259)
    uint8_t planes[4 * PLS];                  // G (the window), b, h, j
    union {
        int16_t h1[WIN_DIM_MAX * WST];        // unclipped vertical 6-tap intermediates (planes only)
        uint2 sad8[NPK * NTS];                // then: the 8x8 SADs of every thread's positions,
    } hs;                                     //   [k][thread] (16x16 / 16x8 / 8x16 searches)
    unsigned long long *pst;                  // debug: per-stage stamps (thread 0), null when off
    int pn;
    unsigned bar;                             // JMH_I4WAVE: arrivals at the search waves' barriers (search_sync)
    IntraS<uint8_t> in;                       // the MB's intra decisions, run by waves 6 and 7
};
union AnalyseS {
    MeS me;
    IntraS<uint8_t> in[4];
};

__device__ __forceinline__ void sstamp(MeS &s, int wave) {
    if (wave == 0 && __lane_id() == 0 && s.pst && s.pn < 44) s.pst[s.pn++] = wall_clock64();
}

// ======================================================================================
//  motion search
// ======================================================================================
// neighbour view of a motion search of block type bt in 8x8 block b8 (see header comment)
struct NbMe {
    const MeS &s;
    int bt, b8, best8x8;
    __device__ bool operator()(int xN, int yN, int &ref, int &mx, int &my) const {
        if (yN > 15 || (xN > 15 && yN >= 0)) return false;
        if (xN < 0 || yN < 0) {
            int c = border_cell(xN, yN);
            if (c < 0 || s.bd.ref[c] == -2) return false;
            ref = s.bd.ref[c]; mx = s.bd.mv[c][0]; my = s.bd.mv[c][1];
            return true;
        }
        int k = (yN >> 2) * 4 + (xN >> 2), cb8 = ((yN >> 3) << 1) | (xN >> 3);
        int m = (bt <= 3 || cb8 == b8) ? bt : (best8x8 >> (4 * cb8)) & 15;
        ref = 0; mx = s.all_mv[m][k][0]; my = s.all_mv[m][k][1];
        return true;
    }
};

// SAD of partition (BT, BX, BY) from the 2 packed pair registers of one position.
// Role 1: r[h] = 8x8 blocks (0, h) low, (1, h) high.  Role 2 (8x8 block at 4x4 coords X, Y even):
// r[ly] = 4x4 blocks (X, Y + ly) low, (X + 1, Y + ly) high.
template <int BT, int BX, int BY>
__device__ __forceinline__ unsigned psum(const uint32_t (&r)[2]) {
    uint32_t v;
    if constexpr (BT == 1 || BT == 4) v = r[0] + r[1];
    else if constexpr (BT == 2) v = r[BY >> 1];
    else if constexpr (BT == 5) v = r[BY & 1];
    else if constexpr (BT == 3) { v = r[0] + r[1]; return (BX >> 1) ? v >> 16 : v & 0xFFFFu; }
    else if constexpr (BT == 6) { v = r[0] + r[1]; return (BX & 1) ? v >> 16 : v & 0xFFFFu; }
    else { v = r[BY & 1]; return (BX & 1) ? v >> 16 : v & 0xFFFFu; }
    return (v & 0xFFFFu) + (v >> 16);
}

// per-thread search state: SADs of the thread's NPK positions and their JM order keys
struct PosState {
    uint32_t sadp[NPK][2];
    uint32_t ordk2[NPK2];    // JM order of positions 2i (low half) and 2i+1 (high half): 0 = (0,0)
                             // pre-check, else spiral index + 1; 0xFFFF for slots outside the table
    int dx, dy0;
    int scx, scy;            // window centre (full pel, relative to the MB)
    unsigned bgen;           // JMH_I4WAVE: arrivals search_sync waits for (wave-uniform)
};

// optimisation fence on the register-resident search state, once per stage: keeps the compiler
// from hoisting unpacked partition sums of later stages (doubling the live registers)
__device__ __forceinline__ void fence_state(PosState &ps) {
#pragma unroll
    for (int k = 0; k < NPK; k++) {
#pragma unroll
        for (int q = 0; q < 2; q++) asm volatile("" : "+v"(ps.sadp[k][q]));
    }
#pragma unroll
    for (int k = 0; k < NPK2; k++) asm volatile("" : "+v"(ps.ordk2[k]));
    asm volatile("" : "+v"(ps.dx), "+v"(ps.dy0));   // nor position arithmetic (RestrictSearchRange 0)
}

// order key of position k, sign-extended: a slot outside the table gives 0xFFFFFFFF, which ORed
// into any key loses every comparison
__device__ __forceinline__ uint32_t ordk_of(const PosState &ps, int k) {
    const uint32_t w = ps.ordk2[k >> 1];
    return (k & 1) ? (uint32_t)((int)w >> 16) : (uint32_t)(int)(int16_t)(w & 0xFFFFu);
}

// this thread's best key for a search of partition (BT, BX, BY) with predictor (pmx, pmy):
// cost = SAD + lambda*(mvbits(x) + mvbits(y)) from the LDS mvbits table; 'range' < sr only with
// RestrictSearchRange 0 (positions outside are skipped, the (0,0) pre-check never is)
template <int BT, int BX, int BY>
__device__ __forceinline__ unsigned eval_search(const MeS &s, const PosState &ps, const uint32_t (&sp)[NPK][2], int sr, int range, int pmx,
                                                int pmy, int scx, int scy) {
    const unsigned cxv = s.mvc[4 * (scx - sr + ps.dx) - pmx + MVB_OFF];
    const uint16_t *cy = s.mvc + 4 * (scy - sr + ps.dy0) - pmy + MVB_OFF;
    unsigned b = 0xFFFFFFFFu;
    if (range >= sr) {
#pragma unroll
        for (int k = 0; k < NPK; k++) {
            const unsigned cost = psum<BT, BX, BY>(sp[k]) + cxv + cy[4 * k];
            b = min(b, (cost << 13) | ordk_of(ps, k));
        }
    } else {
        const int rx = abs(ps.dx - sr);
#pragma unroll
        for (int k = 0; k < NPK; k++) {
            const unsigned cost = psum<BT, BX, BY>(sp[k]) + cxv + cy[4 * k];
            const uint32_t o = ordk_of(ps, k);
            const bool in = max(rx, abs(ps.dy0 + k - sr)) <= range || o == 0;
            b = min(b, in ? (cost << 13) | o : 0xFFFFFFFFu);
        }
    }
    return b;
}

__device__ __forceinline__ int search_range(const DevParams &d, int bt) { return d.restrict_sr == 0 ? d.sr / min(2, bt) : d.sr; }

// one search of a stage: block type, position (4x4 units), partition index of motion_cost, and
// the next-stage search whose MVP depends only on this result and on final MVs (fbt 0: none),
// which the sub-pel wave computes into pmv[fslot]
struct SDesc {
    int bt, bx4, by4, mc;
    int fbt, fbx4, fby4, fslot;
};

// SATD() [J] of one 4x4 sub-block against the sub-pel prediction at quarter-pel offset (ox, oy)
// from the full-pel position; wbase = window offset of the sub-block's top-left sample there.
// One lane does the whole block: rows of 4 samples as dwords (two aligned LDS reads +
// v_alignbyte per plane), the rounding average of the two planes per byte.
__device__ __forceinline__ uint32_t lds_u32_at(const uint8_t *p) { return lds_u32_any(p); }
typedef short s16x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ s16x2 as_s2(uint32_t v) { return __builtin_bit_cast(s16x2, v); }
__device__ __forceinline__ uint32_t as_u32(s16x2 v) { return __builtin_bit_cast(uint32_t, v); }
__device__ __forceinline__ s16x2 abs2(s16x2 v) { return __builtin_elementwise_max(v, (s16x2)(0) - v); }
__device__ __forceinline__ s16x2 lo16(uint32_t w) { return as_s2(__builtin_amdgcn_perm(0u, w, 0x0c010c00u)); }   // bytes 0, 1
__device__ __forceinline__ s16x2 hi16(uint32_t w) { return as_s2(__builtin_amdgcn_perm(0u, w, 0x0c030c02u)); }   // bytes 2, 3
__device__ __forceinline__ s16x2 tap6_2(s16x2 a, s16x2 b, s16x2 c, s16x2 d, s16x2 e, s16x2 f) {
    return (a + f) + (s16x2)(20) * (c + d) - (s16x2)(5) * (b + e);
}
__device__ __forceinline__ s16x2 clip5(s16x2 v) {   // clip255((v + 16) >> 5)
    return __builtin_elementwise_min(__builtin_elementwise_max((v + (s16x2)(16)) >> (s16x2)(5), (s16x2)(0)), (s16x2)(255));
}
__device__ __forceinline__ uint32_t pack4(s16x2 lo, s16x2 hi) { return __builtin_amdgcn_perm(as_u32(hi), as_u32(lo), 0x06040200u); }

// HALF: a half-pel (or full-pel) position, whose sample is one plane's (A == B): B is not read
template <bool HALF>
__device__ __forceinline__ int subblock_satd(const MeS &s, int wbase, int obase, int ox, int oy, int had) {
#if JMH_EXP & 1   // instruction-count experiment (tools/valu_split.sh): no sub-pel SATD
    return 0;
#endif
    const int off = qoff((oy & 3) * 4 + (ox & 3));
    const int xa = (off >> 12) & 15, ya = (off >> 8) & 15, xb = (off >> 4) & 15, yb = off & 15;
    const int oA = ((xa & 1) + 2 * (ya & 1)) * PLS + (ya >> 1) * WST + (xa >> 1);
    const int oB = ((xb & 1) + 2 * (yb & 1)) * PLS + (yb >> 1) * WST + (xb >> 1);
    const uint8_t *r0 = s.planes + wbase + (oy >> 2) * WST + (ox >> 2);
    uint32_t O[4], P[4];
#pragma unroll
    for (int yy = 0; yy < 4; yy++) {
        const uint32_t A = lds_u32_at(r0 + yy * WST + oA);
        if constexpr (HALF) P[yy] = A;
        else {
            const uint32_t B = lds_u32_at(r0 + yy * WST + oB);
            P[yy] = (A | B) - (((A ^ B) >> 1) & 0x7F7F7F7Fu);   // per byte (a + b + 1) >> 1
        }
        O[yy] = *reinterpret_cast<const uint32_t *>(s.org + obase + 16 * yy);
    }
    if (!had) {
        uint32_t sad = 0;
#pragma unroll
        for (int yy = 0; yy < 4; yy++) sad = __builtin_amdgcn_sad_u8(O[yy], P[yy], sad);
        return (int)sad;
    }
    // 4x4 Hadamard on packed int16 pairs (|coefficient| <= 16 * 255): r[y][h] = columns 2h, 2h+1
    s16x2 r[4][2];
#pragma unroll
    for (int yy = 0; yy < 4; yy++) {
        r[yy][0] = as_s2(__builtin_amdgcn_perm(0u, O[yy], 0x0c010c00u)) - as_s2(__builtin_amdgcn_perm(0u, P[yy], 0x0c010c00u));
        r[yy][1] = as_s2(__builtin_amdgcn_perm(0u, O[yy], 0x0c030c02u)) - as_s2(__builtin_amdgcn_perm(0u, P[yy], 0x0c030c02u));
    }
    s16x2 m[4][2];
#pragma unroll
    for (int h = 0; h < 2; h++) {   // vertical
        const s16x2 a0 = r[0][h] + r[3][h], a1 = r[1][h] + r[2][h], a2 = r[1][h] - r[2][h], a3 = r[0][h] - r[3][h];
        m[0][h] = a0 + a1; m[2][h] = a0 - a1; m[1][h] = a2 + a3; m[3][h] = a3 - a2;
    }
    s16x2 acc = (s16x2)(0);
#pragma unroll
    for (int p = 0; p < 2; p++) {   // horizontal, rows 2p and 2p+1 packed together
        const uint32_t u0 = as_u32(m[2 * p][0]), v0 = as_u32(m[2 * p + 1][0]);
        const uint32_t u1 = as_u32(m[2 * p][1]), v1 = as_u32(m[2 * p + 1][1]);
        const s16x2 x0 = as_s2(__builtin_amdgcn_perm(v0, u0, 0x05040100u)), x1 = as_s2(__builtin_amdgcn_perm(v0, u0, 0x07060302u));
        const s16x2 x2 = as_s2(__builtin_amdgcn_perm(v1, u1, 0x05040100u)), x3 = as_s2(__builtin_amdgcn_perm(v1, u1, 0x07060302u));
        // last butterfly: |a + b| + |a - b| = 2 max(|a|, |b|), so SATD = sum of the maxima
        const s16x2 a0 = x0 + x3, a1 = x1 + x2, a2 = x1 - x2, a3 = x0 - x3;
        acc += __builtin_elementwise_max(abs2(a0), abs2(a1)) + __builtin_elementwise_max(abs2(a2), abs2(a3));   // <= 4 * 4080 per half
    }
    const uint32_t t = as_u32(acc);
    return (int)((t & 0xFFFFu) + (t >> 16));
}

// one row (row = lane & 3) of a 4x4 SATD on a quad of lanes: the vertical transform crosses the
// quad by DPP, the result is this row's share (the quad sum is the block's SATD)
template <bool HALF>
__device__ __forceinline__ int quad_row_satd(const MeS &s, int wbase, int obase, int ox, int oy, int row, int had) {
#if JMH_EXP & 1
    return 0;
#endif
    const int off = qoff((oy & 3) * 4 + (ox & 3));
    const int xa = (off >> 12) & 15, ya = (off >> 8) & 15, xb = (off >> 4) & 15, yb = off & 15;
    const int oA = ((xa & 1) + 2 * (ya & 1)) * PLS + (ya >> 1) * WST + (xa >> 1);
    const int oB = ((xb & 1) + 2 * (yb & 1)) * PLS + (yb >> 1) * WST + (xb >> 1);
    const uint8_t *rr = s.planes + wbase + (oy >> 2) * WST + (ox >> 2) + row * WST;
    const uint32_t A = lds_u32_at(rr + oA);
    uint32_t P = A;
    if constexpr (!HALF) {
        const uint32_t B = lds_u32_at(rr + oB);
        P = (A | B) - (((A ^ B) >> 1) & 0x7F7F7F7Fu);
    }
    const uint32_t O = *reinterpret_cast<const uint32_t *>(s.org + obase + 16 * row);
    if (!had) return (int)__builtin_amdgcn_sad_u8(O, P, 0u);
    s16x2 p0 = as_s2(__builtin_amdgcn_perm(0u, O, 0x0c010c00u)) - as_s2(__builtin_amdgcn_perm(0u, P, 0x0c010c00u));
    s16x2 p1 = as_s2(__builtin_amdgcn_perm(0u, O, 0x0c030c02u)) - as_s2(__builtin_amdgcn_perm(0u, P, 0x0c030c02u));
    {   // rows (0,3), (1,2): sums on rows 0, 1, differences on rows 2, 3
        const s16x2 q0 = as_s2((uint32_t)dpp<0x1B>((int)as_u32(p0))), q1 = as_s2((uint32_t)dpp<0x1B>((int)as_u32(p1)));
        p0 = row < 2 ? p0 + q0 : q0 - p0;
        p1 = row < 2 ? p1 + q1 : q1 - p1;
    }
    {   // rows (0,1), (2,3)
        const s16x2 q0 = as_s2((uint32_t)dpp<0xB1>((int)as_u32(p0))), q1 = as_s2((uint32_t)dpp<0xB1>((int)as_u32(p1)));
        p0 = (row & 1) == 0 ? p0 + q0 : q0 - p0;
        p1 = (row & 1) == 0 ? p1 + q1 : q1 - p1;
    }
    // horizontal: (x0, x1) = p0, (x2, x3) = p1 -> (x0 + x3, x1 + x2), (x0 - x3, x1 - x2)
    const s16x2 sw = as_s2(__builtin_amdgcn_alignbit(as_u32(p1), as_u32(p1), 16));
    const uint32_t t = as_u32(abs2(p0 + sw)), u = as_u32(abs2(p0 - sw));
    return (int)(max(t & 0xFFFFu, t >> 16) + max(u & 0xFFFFu, u >> 16));
}

// SubPelBlockMotionSearch [J] of search j of the stage on ONE wave: full-pel winner from the
// per-wave keys, then half-pel (9 candidates) and quarter-pel (8) passes.  Lane task = (candidate,
// 4x4 sub-block), aligned groups of nsub lanes sum a candidate, the wave minimum of
// (cost, candidate) keys is JM's strict '<' scan in candidate order.  No workgroup barrier.
#define KOFF 4096
__device__ __forceinline__ void subpel_wave(const DevParams &d, MeS &s, int j, const SDesc q, int pmvx, int pmvy, int scx, int scy, int b8,
                                            int best8x8) {
    const int lane = __lane_id();
    const int sr = d.sr, lam = d.lambda_motion, had = d.use_hadamard;
    unsigned best = s.red[0][j];
#pragma unroll
    for (int w = 1; w < NTS / 64; w++) best = min(best, s.red[w][j]);
    const unsigned order = best & 8191u;
    int rx, ry;
    if (order == 0) { rx = -scx; ry = -scy; }
    else {   // spiral index -> position from the context's table (a scalar load, no sqrt)
        const uint32_t e = d.ordtab[ORDTAB_SPOS + order - 1];
        rx = (int)(int16_t)(e & 0xFFFFu);
        ry = (int)e >> 16;
    }
    const int fmx = scx + rx, fmy = scy + ry;
    int min_mcost = had ? BIGCOST : (int)(best >> 13);
    const int lw4 = lw4_of(q.bt), lns = lw4 + lh4_of(q.bt), nsub = 1 << lns;
    const bool check0 = q.bt == 1 && fmx == 0 && fmy == 0 && had && d.slice_type == JMH_P_SLICE;
    const int wb0 = (WM + sr + ry) * WST + WM + sr + rx;   // window offset of MB pixel (0,0) at the full-pel MV
    int qx = 0, qy = 0;
#pragma unroll
    for (int pass = 0; pass < 2; pass++) {
        const int step = pass == 0 ? 2 : 1;
        const int min_pos = pass == 0 ? (had ? 0 : 1) : 1;
        unsigned kb = 0xFFFFFFFFu;
        if (lns <= 1) {   // 4x4 / 8x4 / 4x8: a quad per candidate, one row per lane -- of both 4x4
                          // sub-blocks for 8x4 / 4x8, so the nine candidates take one pass of the wave
            const int row = lane & 3, c = lane >> 2;
            const bool val = c < 9 && c >= min_pos;
            const int ox = qx + step * sp9x(c), oy = qy + step * sp9y(c);
            int sat = 0;
            if (c < 9) {   // quad-uniform
                const int bxs1 = q.bx4 + lw4, bys1 = q.by4 + (lns - lw4);   // the second sub-block
                sat = pass == 0 ? quad_row_satd<true>(s, wb0 + 4 * q.by4 * WST + 4 * q.bx4, 64 * q.by4 + 4 * q.bx4, ox, oy, row, had)
                                : quad_row_satd<false>(s, wb0 + 4 * q.by4 * WST + 4 * q.bx4, 64 * q.by4 + 4 * q.bx4, ox, oy, row, had);
                if (lns)
                    sat += pass == 0 ? quad_row_satd<true>(s, wb0 + 4 * bys1 * WST + 4 * bxs1, 64 * bys1 + 4 * bxs1, ox, oy, row, had)
                                     : quad_row_satd<false>(s, wb0 + 4 * bys1 * WST + 4 * bxs1, 64 * bys1 + 4 * bxs1, ox, oy, row, had);
            }
            sat += dpp<0xB1>(sat);   // the quad's rows
            sat += dpp<0x4E>(sat);
            if (val && row == 0) {
                int cost = sat + (int)__umul24(lam, mvbits(4 * fmx + ox - pmvx) + mvbits(4 * fmy + oy - pmvy));
                if (pass == 0 && check0 && c == 0) cost -= 16 * lam;
                kb = min(kb, ((unsigned)(cost + KOFF) << 4) | (unsigned)c);
            }
        } else {   // 8x8 and larger: a quad per candidate, lane g of it takes the 4x4 sub-blocks
                   // g * spl .. g * spl + spl - 1 (spl = nsub / 4), so one pass of the wave
            const int g = lane & 3, c = lane >> 2, lspl = lns - 2;
            const bool val = c < 9 && c >= min_pos;
            const int ox = qx + step * sp9x(c), oy = qy + step * sp9y(c);
            int sat = 0;
            if (val) {
#pragma unroll
                for (int k = 0; k < 4; k++) {
                    if (k >= (1 << lspl)) break;
                    const int sub = (g << lspl) + k;
                    const int bxs = q.bx4 + (sub & ((1 << lw4) - 1)), bys = q.by4 + (sub >> lw4);
                    sat += pass == 0 ? subblock_satd<true>(s, wb0 + 4 * bys * WST + 4 * bxs, 64 * bys + 4 * bxs, ox, oy, had)
                                     : subblock_satd<false>(s, wb0 + 4 * bys * WST + 4 * bxs, 64 * bys + 4 * bxs, ox, oy, had);
                }
            }
            sat += dpp<0xB1>(sat);   // the quad
            sat += dpp<0x4E>(sat);
            if (val && g == 0) {
                int cost = sat + (int)__umul24(lam, mvbits(4 * fmx + ox - pmvx) + mvbits(4 * fmy + oy - pmvy));
                if (pass == 0 && check0 && c == 0) cost -= 16 * lam;
                kb = min(kb, ((unsigned)(cost + KOFF) << 4) | (unsigned)c);
            }
        }
        kb = wave_min_u32(kb);
        if (kb != 0xFFFFFFFFu && (int)(kb >> 4) - KOFF < min_mcost) {
            const int c = kb & 15;
            min_mcost = (int)(kb >> 4) - KOFF;
            qx += step * sp9x(c);
            qy += step * sp9y(c);
        }
    }
    if (lane < nsub) {
        const int k = (q.by4 + (lane >> lw4)) * 4 + q.bx4 + (lane & ((1 << lw4) - 1));
        s.all_mv[q.bt][k][0] = (int16_t)(4 * fmx + qx);
        s.all_mv[q.bt][k][1] = (int16_t)(4 * fmy + qy);
    }
    if (lane == 0) s.motion_cost[q.bt][q.mc] += min_mcost;
    if (q.fbt) {   // forwarded MVP of the next stage's search (reads the MVs just stored)
        int mx, my;
        set_mvp(NbMe{s, q.fbt, b8, best8x8}, q.fbx4, q.fby4, 4 << lw4_of(q.fbt), 4 << lh4_of(q.fbt), mx, my);
        if (lane == 0) { s.pmv[q.fslot][0] = mx; s.pmv[q.fslot][1] = my; }
    }
}

// one stage of NS independent searches: MVPs (FWD: forwarded by the previous stage's sub-pel
// waves through LDS; else lane j of every wave computes search j's, then readlane), the full-pel
// argmin over all positions by every thread (EV fills bk[] from pmx/pmy), per-wave minima -> LDS
// -> barrier, sub-pel search j on wave j (+ forwarded MVPs), barrier.
// the wave of a stage's search j: waves 0, 1, 4, 5 (SIMDs 0 and 1) first, so that the Intra4x4
// waves 6 and 7 (SIMDs 2 and 3) share their SIMDs with no sub-pel wave of the workgroup in stages
// of up to four searches
#ifndef JMH_SWMAP
#define JMH_SWMAP 1
#endif
__device__ __forceinline__ constexpr int search_wave(int j) { return JMH_SWMAP ? (0x6325410 >> (4 * j)) & 15 : j; }

// barrier of the search waves.  JMH_I4WAVE: the seven search waves count their arrivals in LDS
// (one monotonic counter, the release / acquire fences order the stage's LDS writes and reads
// around it) -- an s_barrier would also wait for the intra wave 7, which runs its own chain.  Every
// search wave reaches every barrier, so the poll always ends.
__device__ __forceinline__ void search_sync(MeS &s, PosState &ps) {
#if JMH_I4WAVE
    ps.bgen += NTS / 64;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    if (__lane_id() == 0) __hip_atomic_fetch_add(&s.bar, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    while (__builtin_amdgcn_readfirstlane(__hip_atomic_load(&s.bar, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)) < ps.bgen)
        __builtin_amdgcn_s_sleep(1);
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
#else
    (void)s; (void)ps;
    __syncthreads();
#endif
}

template <int NS, bool FWD, class EV, class IDLE>
__device__ __forceinline__ void me_stage(const DevParams &d, MeS &s, PosState &ps, const SDesc (&sd)[NS], int b8, int best8x8, EV ev,
                                         int islot, IDLE idle, int wave) {
    const int lane = __lane_id();
    fence_state(ps);
    int pmx[NS], pmy[NS];
    unsigned bk[NS];
    if constexpr (FWD) {
#pragma unroll
        for (int j = 0; j < NS; j++) {   // uniform: SGPRs
            pmx[j] = __builtin_amdgcn_readfirstlane(s.pmv[j][0]);
            pmy[j] = __builtin_amdgcn_readfirstlane(s.pmv[j][1]);
        }
    } else {
        // wave j computes search j's MVP (wave-uniform code for a constant block), then LDS
#pragma unroll
        for (int j = 0; j < NS; j++)
            if (wave == search_wave(j)) {
                int mx, my;
                set_mvp(NbMe{s, sd[j].bt, b8, best8x8}, sd[j].bx4, sd[j].by4, 4 << lw4_of(sd[j].bt), 4 << lh4_of(sd[j].bt), mx, my);
                if (lane == 0) { s.pmv[j][0] = mx; s.pmv[j][1] = my; }
            }
        search_sync(s, ps);
#pragma unroll
        for (int j = 0; j < NS; j++) {   // uniform: SGPRs
            pmx[j] = __builtin_amdgcn_readfirstlane(s.pmv[j][0]);
            pmy[j] = __builtin_amdgcn_readfirstlane(s.pmv[j][1]);
        }
    }
    ev(bk, pmx, pmy);
#pragma unroll
    for (int j = 0; j < NS; j++) {
        const unsigned v = wave_min_u32(bk[j]);
        if (lane == 0) s.red[wave][j] = v;
    }
    search_sync(s, ps);
    sstamp(s, wave);
#pragma unroll
    for (int j = 0; j < NS; j++)
        if (wave == search_wave(j)) subpel_wave(d, s, j, sd[j], pmx[j], pmy[j], ps.scx, ps.scy, b8, best8x8);
#if !JMH_I4WAVE
    if constexpr (NS <= 6) {
        if (islot >= 0 && wave >= 6) idle(islot, wave - 6);   // the MB's Intra4x4 on otherwise idle waves
    } else {
        if (islot >= 0 && wave == 7) idle(islot, 0);          // one free wave: a one-block step
    }
#else
    (void)islot; (void)idle;
#endif
    search_sync(s, ps);
    sstamp(s, wave);
}

#define EV(J, BT, BX, BY) bk[J] = eval_search<BT, BX, BY>(s, ps, ps.sadp, sr, search_range(d, BT), pmx[J], pmy[J], ps.scx, ps.scy)

// up to three searches on the 8x8 SADs kept in LDS (16x16 / 16x8 / 8x16): one LDS read per
// position shared by the searches, so only two SAD registers are live at a time.  Search j is
// (BT[j], BX[j], BY[j]); keys as eval_search.
template <int N, int BT0, int BX0, int BY0, int BT1, int BX1, int BY1, int BT2 = 0, int BX2 = 0, int BY2 = 0>
__device__ __forceinline__ void eval_sad8(const MeS &s, const PosState &ps, int tid, int sr, const int (&range)[N], const int *pmx,
                                          const int *pmy, unsigned *out) {
    unsigned cxv[N];
    const uint16_t *cy[N];
    bool full = true;
#pragma unroll
    for (int j = 0; j < N; j++) {
        cxv[j] = s.mvc[4 * (ps.scx - sr + ps.dx) - pmx[j] + MVB_OFF];
        cy[j] = s.mvc + 4 * (ps.scy - sr + ps.dy0) - pmy[j] + MVB_OFF;
        out[j] = 0xFFFFFFFFu;
        full = full && range[j] >= sr;
    }
    auto loop = [&](auto restricted) {
        const int rx = abs(ps.dx - sr);
#pragma unroll
        for (int k = 0; k < NPK; k++) {
            const uint2 v = s.hs.sad8[k * NTS + tid];
            const uint32_t r[2] = {v.x, v.y};
            const uint32_t o = ordk_of(ps, k);
            unsigned c[3];
            c[0] = psum<BT0, BX0, BY0>(r);
            c[1] = psum<BT1, BX1, BY1>(r);
            if constexpr (N > 2) c[2] = psum<BT2, BX2, BY2>(r);
#pragma unroll
            for (int j = 0; j < N; j++) {
                const unsigned key = ((c[j] + cxv[j] + cy[j][4 * k]) << 13) | o;
                if constexpr (decltype(restricted)::value)
                    out[j] = min(out[j], (max(rx, abs(ps.dy0 + k - sr)) <= range[j] || o == 0) ? key : 0xFFFFFFFFu);
                else
                    out[j] = min(out[j], key);
            }
        }
    };
    if (full) loop(std::false_type{});
    else loop(std::true_type{});   // RestrictSearchRange 0: positions outside a type's range
}

// SADs at this thread's NPK positions (column strip dx, rows dy0..dy0+NPK-1 of the window) of the
// 8x8 org block at pixel (OX, OY).  EIGHT: the 8x8 SAD into half HI of ps.sadp[k][SLOT] (role 1);
// else the four 4x4 SADs, rows 0..3 into ps.sadp[k][0] and 4..7 into [1] (role 2).  One 8-pixel
// column at a time keeps the unrolled window rows (3 dwords each) within the register budget.
template <bool EIGHT, int OX, int OY, int SLOT, int HI>
__device__ __forceinline__ void sad_strip(const MeS &s, PosState &ps) {
#if JMH_EXP & 4   // instruction-count experiment: no SAD strips
    return;
#endif
    const int wx = ps.dx + WM + OX;
    const uint32_t sel = wx & 3;
    const uint8_t *wb = s.planes + (ps.dy0 + WM + OY) * WST + (wx & ~3);
    uint32_t acc[NPK][2];
#pragma unroll
    for (int k = 0; k < NPK; k++) acc[k][0] = acc[k][1] = 0;
#pragma unroll
    for (int r = 0; r < 8 + NPK - 1; r++) {
        const uint32_t *w32 = reinterpret_cast<const uint32_t *>(wb + r * WST);
        const uint32_t a0 = w32[0], a1 = w32[1], a2 = w32[2];
        const uint32_t w0 = __builtin_amdgcn_alignbyte(a1, a0, sel), w1 = __builtin_amdgcn_alignbyte(a2, a1, sel);
#pragma unroll
        for (int k = 0; k < NPK; k++) {
            const int mr = r - k;
            if (mr < 0 || mr > 7) continue;
            const uint2 o = *reinterpret_cast<const uint2 *>(s.org + (OY + mr) * 16 + OX);
            if constexpr (EIGHT) {
                acc[k][0] = __builtin_amdgcn_sad_u8(w1, o.y, __builtin_amdgcn_sad_u8(w0, o.x, acc[k][0]));
                if (mr == 7) ps.sadp[k][SLOT] = HI ? (ps.sadp[k][SLOT] | (acc[k][0] << 16)) : acc[k][0];
            } else {
                acc[k][0] = __builtin_amdgcn_sad_u8(w0, o.x, acc[k][0]);
                acc[k][1] = __builtin_amdgcn_sad_u8(w1, o.y, acc[k][1]);
                if ((mr & 3) == 3) {
                    ps.sadp[k][mr >> 2] = acc[k][0] | (acc[k][1] << 16);
                    acc[k][0] = acc[k][1] = 0;
                }
            }
        }
    }
}

// one 8x8 block of P8x8: its 4x4 SADs, 4 stages (sub-modes 4..7 in parallel, then the 4x4
// chain), then the P8x8 sub-mode decision for the block (its MVs are read through best8x8).
// Every block leaves its 8x8 SAD (the sum of its 4x4 SADs) in the LDS 8x8 table, so block 3 also
// runs the 16x16 / 16x8 / 8x16 searches, which are independent of P8x8: the first blocks of each
// type in its stage 0, the second ones in its stage 1.  Intra4x4 slots 0..10 (waves 6, 7) run in
// the sub-pel phases of the stages listed below.
template <int B8, class IDLE>
__device__ __forceinline__ void p8x8_block(const DevParams &d, MeS &s, PosState &ps, int &best8x8, int &cost8x8, IDLE idle, int wave, int tid) {
    constexpr int X = 2 * (B8 & 1), Y = 2 * (B8 >> 1);
    // Intra4x4 slots (diagonal steps 0..9, 10 = the results) in the stages whose sub-pel phase is
    // long enough to hide a step: the multi-search stages 0 and 1 of every block (block 3's stage
    // 0 has one free wave, so its step, 8, is a one-block step), two steps in single-search stages
    constexpr int IS0 = 3 * B8 - (B8 == 3 ? 1 : 0), IS1 = IS0 + 1;
    // (k_mb_flow: block 2's stage 2, slot 11, the Intra16x16 and chroma intra-mode decisions)
    constexpr int IS2 = B8 <= 1 ? 3 * B8 + 2 : B8 == 3 ? 10 : 11, IS3 = -1;
    const int sr = d.sr;
    fence_state(ps);
    sad_strip<false, 4 * X, 4 * Y, 0, 0>(s, ps);        // the four 4x4 SADs of this 8x8 block
    // this block's 8x8 SAD into its 16-bit half of the 8x8 table entry (each thread reads only its
    // own entries: no barrier)
#pragma unroll
    for (int k = 0; k < NPK; k++) {
        const uint32_t a = ps.sadp[k][0], b = ps.sadp[k][1];
        reinterpret_cast<uint16_t *>(&s.hs.sad8[k * NTS + tid])[B8] = (uint16_t)((a & 0xFFFFu) + (a >> 16) + (b & 0xFFFFu) + (b >> 16));
    }
    if constexpr (B8 == 3) {
        // stage 0: 8x8, 8x4 upper, 4x8 left, 4x4 top-left + 16x16, 16x8 upper, 8x16 left
        const SDesc sd[7] = {{4, X, Y, B8, 0, 0, 0, 0},
                             {5, X, Y, B8, 5, X, Y + 1, 0},
                             {6, X, Y, B8, 6, X + 1, Y, 1},
                             {7, X, Y, B8, 7, X + 1, Y, 2},
                             {1, 0, 0, 0, 0, 0, 0, 0},
                             {2, 0, 0, 0, 2, 0, 2, 3},
                             {3, 0, 0, 0, 3, 2, 0, 4}};
        me_stage<7, false>(d, s, ps, sd, B8, best8x8, [&](unsigned (&bk)[7], const int (&pmx)[7], const int (&pmy)[7]) {
            EV(0, 4, X, Y); EV(1, 5, X, Y); EV(2, 6, X, Y); EV(3, 7, X, Y);
            const int rg[3] = {search_range(d, 1), search_range(d, 2), search_range(d, 3)};
            eval_sad8<3, 1, 0, 0, 2, 0, 0, 3, 0, 0>(s, ps, tid, sr, rg, pmx + 4, pmy + 4, bk + 4);
        }, IS0, idle, wave);
        // stage 1: 8x4 lower, 4x8 right, 4x4 top-right + 16x8 lower, 8x16 right
        const SDesc sd1[5] = {{5, X, Y + 1, B8, 0, 0, 0, 0}, {6, X + 1, Y, B8, 0, 0, 0, 0}, {7, X + 1, Y, B8, 7, X, Y + 1, 0},
                              {2, 0, 2, 1, 0, 0, 0, 0}, {3, 2, 0, 1, 0, 0, 0, 0}};
        me_stage<5, true>(d, s, ps, sd1, B8, best8x8, [&](unsigned (&bk)[5], const int (&pmx)[5], const int (&pmy)[5]) {
            EV(0, 5, X, Y + 1); EV(1, 6, X + 1, Y); EV(2, 7, X + 1, Y);
            const int rg[2] = {search_range(d, 2), search_range(d, 3)};
            eval_sad8<2, 2, 0, 2, 3, 2, 0>(s, ps, tid, sr, rg, pmx + 3, pmy + 3, bk + 3);
        }, IS1, idle, wave);
    } else {
        {   // stage 0: 8x8, 8x4 upper, 4x8 left, 4x4 top-left
            const SDesc sd[4] = {{4, X, Y, B8, 0, 0, 0, 0},
                                 {5, X, Y, B8, 5, X, Y + 1, 0},
                                 {6, X, Y, B8, 6, X + 1, Y, 1},
                                 {7, X, Y, B8, 7, X + 1, Y, 2}};
            me_stage<4, false>(d, s, ps, sd, B8, best8x8, [&](unsigned (&bk)[4], const int (&pmx)[4], const int (&pmy)[4]) {
                EV(0, 4, X, Y); EV(1, 5, X, Y); EV(2, 6, X, Y); EV(3, 7, X, Y);
            }, IS0, idle, wave);
        }
        {   // stage 1: 8x4 lower, 4x8 right, 4x4 top-right
            const SDesc sd[3] = {{5, X, Y + 1, B8, 0, 0, 0, 0}, {6, X + 1, Y, B8, 0, 0, 0, 0}, {7, X + 1, Y, B8, 7, X, Y + 1, 0}};
            me_stage<3, true>(d, s, ps, sd, B8, best8x8, [&](unsigned (&bk)[3], const int (&pmx)[3], const int (&pmy)[3]) {
                EV(0, 5, X, Y + 1); EV(1, 6, X + 1, Y); EV(2, 7, X + 1, Y);
            }, IS1, idle, wave);
        }
    }
    {   // stage 2: 4x4 bottom-left
        const SDesc sd[1] = {{7, X, Y + 1, B8, 7, X + 1, Y + 1, 0}};
        me_stage<1, true>(d, s, ps, sd, B8, best8x8, [&](unsigned (&bk)[1], const int (&pmx)[1], const int (&pmy)[1]) { EV(0, 7, X, Y + 1); },
                          IS2, idle, wave);
    }
    {   // stage 3: 4x4 bottom-right
        const SDesc sd[1] = {{7, X + 1, Y + 1, B8, 0, 0, 0, 0}};
        me_stage<1, true>(d, s, ps, sd, B8, best8x8, [&](unsigned (&bk)[1], const int (&pmx)[1], const int (&pmy)[1]) { EV(0, 7, X + 1, Y + 1); },
                          IS3, idle, wave);
    }
    int mc8 = BIGCOST, bm = 0;
    for (int mode = 4; mode <= 7; mode++) {
        if (!inter_on(d.isr, mode)) continue;
        const int c = s.motion_cost[mode][B8];
        if (c < mc8) { mc8 = c; bm = mode; }
    }
    best8x8 = __builtin_amdgcn_readfirstlane(best8x8 | bm << (4 * B8));   // uniform: SGPRs
    cost8x8 = __builtin_amdgcn_readfirstlane(cost8x8 + mc8);
}

// ======================================================================================
//  intra decisions
// ======================================================================================
// the Intra16x16 decision of the RDO-off wavefront (MbScratch i16cost / i16mode)
template <class pel>
__device__ __forceinline__ void i16_decision(const DevParams &d, const pel *org, const IntraNb<pel> &nb, MbScratch *scr, int lane, bool avL, bool avT,
                                             bool avTL) {
    int best, i16mode;
    i16_pick(d, org, nb, lane, avL, avT, avTL, best, i16mode);
    if (lane == 0) { scr->i16cost = best; scr->i16mode = i16mode; }
}

// IntraChromaPrediction8x8 mode decision on one wave: 4 modes x 2 components x 4 blocks.  A lane's
// DC and plane parameters once, then each sample selected without branching (a per-lane mode
// switch ran all four paths, the plane's parameters per sample)
template <class pel>
__device__ __forceinline__ void chroma_decision(const DevParams &d, const IntraNb<pel> &nb, MbScratch *scr, int lane, bool avL, bool avT, bool avTL) {
    int sat = 0;
    if (lane < 32) {
        const int m = lane >> 3, uv = (lane >> 2) & 1, b = lane & 3, xo = (b & 1) * 4, yo = (b >> 1) * 4;
        const pel *T = nb.ctop[uv] + 1, *L = nb.cleft[uv];
        const int Pc = nb.ctop[uv][0];
        const int dcv = chroma_dc(T, L, avT, avL, b, (d.maxv + 1) >> 1);
        int ih = 0, iv = 0;
#pragma unroll
        for (int i = 1; i <= 4; i++) {
            ih += i * (T[3 + i] - (3 - i >= 0 ? T[3 - i] : Pc));
            iv += i * (L[3 + i] - (3 - i >= 0 ? L[3 - i] : Pc));
        }
        const int ib = (34 * ih + 32) >> 6, ic = (34 * iv + 32) >> 6, iaa = 16 * (L[7] + T[7]);
        int df[16];
#pragma unroll
        for (int y = 0; y < 4; y++)
#pragma unroll
            for (int x = 0; x < 4; x++) {
                const int px = xo + x, py = yo + y;
                const int pl = clipmx((iaa + (px - 3) * ib + (py - 3) * ic + 16) >> 5, d.maxv);
                const int p = m == 0 ? dcv : m == 1 ? (int)L[py] : m == 2 ? (int)T[px] : pl;
                df[4 * y + x] = nb.orgc[uv][py * 8 + px] - p;
            }
        sat = satd4x4(df, d.use_hadamard);
    }
    const bool cav[4] = {true, avL, avT, avT && avL && avTL};
    int minc = BIGCOST, c_mode = 0;
#pragma unroll
    for (int m = 0; m < 4; m++) {
        int c = 0;
#pragma unroll
        for (int q = 0; q < 8; q++) c += __builtin_amdgcn_readlane(sat, 8 * m + q);
        if (cav[m] && c < minc) { minc = c; c_mode = m; }
    }
    if (lane == 0) scr->c_mode = c_mode;
}

// ======================================================================================
//  motion search of one P macroblock (all 41 searches)
// ======================================================================================
__device__ __forceinline__ void intra_slot(const DevParams &d, IntraS<uint8_t> &s, MbScratch *scr, int k, int w, int mbx, int mby);
__device__ __forceinline__ void intra_wave(const DevParams &d, IntraS<uint8_t> &s, MbScratch *scr, int mbx, int mby);

// the part of me_mb's setup that reads no other workgroup's output (the source block, the lambda *
// mvbits table, zeroed accumulators): k_mb_flow runs it while its dependencies finish (pre = true
// then skips it in me_mb)
__device__ __forceinline__ void me_prologue(const DevParams &d, MeS &s, int mbx, int mby) {
    const int tid = threadIdx.x;
    if (tid < 256) s.in.org[tid] = s.org[tid] = d.orgY[(16 * mby + (tid >> 4)) * d.W + 16 * mbx + (tid & 15)];
    else if (tid >= 472 && tid < 478) s.in.part[(tid - 472) / 3][(tid - 472) % 3] = 0;
    else if (tid >= 480 && tid < 512) s.motion_cost[(tid - 480) >> 2][tid & 3] = 0;
    for (int i = tid; i < MVB_LEN; i += NTA) s.mvc[i] = (uint16_t)__umul24(d.lambda_motion, mvbits(i - MVB_OFF));
}

__device__ __forceinline__ void me_mb(const DevParams &d, MeS &s, int mbx, int mby, bool pre = false) {
    const int tid = threadIdx.x;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);   // an SGPR: tid itself dies after the setup
    const int W = d.W, sr = d.sr, side = d.side;
    const int pix_x = 16 * mbx, pix_y = 16 * mby;
    const bool prof = prof_mb_here(d, mbx, mby);
    PSTAMP(0);
    MbScratch *scr = d.scr + mby * d.mbw + mbx;
    if (tid == 0) { s.pst = prof ? d.prof + 20 : nullptr; s.pn = 0; s.bar = 0; }
    if (tid < 256) { if (!pre) s.in.org[tid] = s.org[tid] = d.orgY[(pix_y + (tid >> 4)) * W + pix_x + (tid & 15)]; }
#if JMH_I4WAVE
    else if (tid < 384) load_orgc(d, s.in.nb, tid - 256, mbx, mby);   // the intra wave's chroma decision
#endif
    else if (tid >= 384 && tid < 394) { load_border(d, s.bd, tid - 384, mbx, mby); load_border(d, s.in.bd, tid - 384, mbx, mby); }
    else if (!pre && tid >= 472 && tid < 478) s.in.part[(tid - 472) / 3][(tid - 472) % 3] = 0;
    else if (!pre && tid >= 480 && tid < 512) s.motion_cost[(tid - 480) >> 2][tid & 3] = 0;
    // the MB's Intra4x4 decision (10 diagonal steps, then the results) runs on waves 6 and 7
    // while the motion search's sub-pel waves work: slots 0..10 (intra_slot)
#if JMH_EXP & 2   // instruction-count experiment: no Intra4x4 in the search workgroup
    auto idle = [&](int, int) {};
#else
    auto idle = [&](int k, int w) { intra_slot(d, s.in, scr, k, w, mbx, mby); };
#endif
    (void)scr;
    if (!pre)
        for (int i = tid; i < MVB_LEN; i += NTA) s.mvc[i] = (uint16_t)__umul24(d.lambda_motion, mvbits(i - MVB_OFF));
    int pcx = 0, pcy = 0, scx = 0, scy = 0;
    uint8_t *G = s.planes;
    const int wdim = 2 * sr + 16 + 2 * WM;
    {
        // SetupFastFullPelSearch: centre = 16x16 MVP / 4 (trunc), clamped to +-SR; the window
        // load starts right away (its centre depends only on the border cells).  One LDS dword
        // per task: two aligned global dwords + v_alignbyte inside the picture, clamped bytes
        // at its edges; columns >= wdim are zero.
        __syncthreads();
        set_mvp(NbBorder{s.bd}, 0, 0, 16, 16, pcx, pcy);
        scx = iclip(-sr, sr, pcx / 4); scy = iclip(-sr, sr, pcy / 4);
        const int X0 = pix_x + scx - sr - WM, Y0 = pix_y + scy - sr - WM;
        constexpr int ND4 = WST / 4, NWT = (WIN_DIM_MAX * ND4 + NTA - 1) / NTA;
        // all global loads first (interior dwords; edge tasks fall back to clamped bytes below)
        uint32_t lo_[NWT], hi_[NWT];
        bool fast[NWT];
#pragma unroll
        for (int i = 0; i < NWT; i++) {
            const int task = tid + i * NTA;
            const int y = task / ND4, j = task - y * ND4, x0 = X0 + 4 * j;
            fast[i] = task < wdim * ND4 && 4 * j + 3 < wdim && x0 >= 0 && x0 + 3 < W;
            const uint32_t *p = reinterpret_cast<const uint32_t *>(d.refY + iclip(0, d.H - 1, Y0 + y) * W + (fast[i] ? (x0 & ~3) : 0));
            lo_[i] = p[0];
            hi_[i] = (fast[i] && (x0 & 3)) ? p[1] : 0u;
        }
#pragma unroll
        for (int i = 0; i < NWT; i++) {
            const int task = tid + i * NTA;
            if (task >= wdim * ND4) break;
            const int y = task / ND4, j = task - y * ND4, x0 = X0 + 4 * j;
            uint32_t v;
            if (fast[i]) v = __builtin_amdgcn_alignbyte(hi_[i], lo_[i], x0 & 3);
            else {
                const uint8_t *row = d.refY + iclip(0, d.H - 1, Y0 + y) * W;
                v = 0;
#pragma unroll
                for (int q = 0; q < 4; q++)
                    if (4 * j + q < wdim) v |= (uint32_t)row[iclip(0, W - 1, x0 + q)] << (8 * q);
            }
            *reinterpret_cast<uint32_t *>(G + y * WST + 4 * j) = v;
        }
        if (tid < 32) G[wdim * WST + tid] = 0;
        // intra neighbourhood (first read in intra slot 0, after the next barriers)
        if (tid >= 128 && tid < 199) load_intra_nb(d, s.in.nb, tid - 128, mbx, mby);
    }
    __syncthreads();
    PSTAMP(1);
    {
        // ---- this thread's column strip of NPK positions: SADs (registers) and JM order keys
        PosState ps;
        const int nstrips = (side + NPK - 1) / NPK;
        const bool sact = tid < side * nstrips;
        ps.dx = sact ? tid % side : 0;
        ps.dy0 = sact ? (tid / side) * NPK : 0;
        ps.scx = scx; ps.scy = scy;
        ps.bgen = 0;
        // (the 8x8 SADs of the 16x16 / 16x8 / 8x16 searches come from each 8x8 block's 4x4 SADs,
        // p8x8_block)
        PSTAMP(8);
        // JM order keys of the strip from the per-context table (first read in the first stage, so
        // the loads overlap the half-pel planes); the (0,0) pre-check position, order 0, depends on
        // the MB's window centre
#pragma unroll
        for (int k2 = 0; k2 < NPK2; k2++) ps.ordk2[k2] = d.ordtab[k2 * NTA + tid];
        {
            const int k0 = sr - scy - ps.dy0;   // strip slot of the pre-check position
            const bool mine = sact && ps.dx == sr - scx;
#pragma unroll
            for (int k2 = 0; k2 < NPK2; k2++)
                if (mine && (k0 >> 1) == k2) ps.ordk2[k2] &= (k0 & 1) ? 0x0000FFFFu : 0xFFFF0000u;
        }
        PSTAMP(9);
        // ---- half-pel planes over window rows / columns [3, 2sr+21): four columns (one dword) per
        //      thread: h1 (unclipped vertical taps, int16) and h by a sliding column run, b from
        //      the row's dwords; then j from h1
        {
            const int lo = WM - 1, n = 2 * sr + 18;
            uint8_t *PB = s.planes + PLS, *PH = s.planes + 2 * PLS, *PJ = s.planes + 3 * PLS;
            constexpr int NG = WIN_DIM_MAX / 4, NR = NTA / NG;        // 22 column groups x 23 row runs
            const int g = tid % NG, rb = tid / NG, c0 = 4 * g;
            const int run = (n + NR - 1) / NR, y0 = lo + rb * run, y1 = rb < NR ? min(lo + n, y0 + run) : y0;
            if (y0 < y1) {
                const uint32_t *gc = reinterpret_cast<const uint32_t *>(G + c0);
                constexpr int WS4 = WST / 4;
                uint32_t w0 = gc[(y0 - 2) * WS4], w1 = gc[(y0 - 1) * WS4], w2 = gc[y0 * WS4], w3 = gc[(y0 + 1) * WS4], w4 = gc[(y0 + 2) * WS4];
                for (int y = y0; y < y1; y++) {
                    const uint32_t w5 = gc[(y + 3) * WS4];
                    const uint32_t L = gc[y * WS4 - 1], R = gc[y * WS4 + 1];
                    int hv[4];
                    uint32_t ph = 0, pb = 0;
#pragma unroll
                    for (int i = 0; i < 4; i++) {
                        const int sh = 8 * i;
                        hv[i] = tap6((int)((w0 >> sh) & 255u), (int)((w1 >> sh) & 255u), (int)((w2 >> sh) & 255u), (int)((w3 >> sh) & 255u),
                                     (int)((w4 >> sh) & 255u), (int)((w5 >> sh) & 255u));
                        ph |= (uint32_t)clip255((hv[i] + 16) >> 5) << sh;
                    }
                    // b: bytes c0-2 .. c0+6 of row y (w2) from L | w2 | R
                    const uint64_t mr = ((uint64_t)R << 32) | w2;
                    int bx[9];
                    bx[0] = (int)((L >> 16) & 255u); bx[1] = (int)(L >> 24);
#pragma unroll
                    for (int k = 0; k < 7; k++) bx[2 + k] = (int)((mr >> (8 * k)) & 255u);
#pragma unroll
                    for (int i = 0; i < 4; i++)
                        pb |= (uint32_t)clip255((tap6(bx[i], bx[i + 1], bx[i + 2], bx[i + 3], bx[i + 4], bx[i + 5]) + 16) >> 5) << (8 * i);
#pragma unroll
                    for (int i = 0; i < 4; i++) {
                        const int cx = c0 + i;
                        s.hs.h1[y * WST + cx] = (int16_t)hv[i];
                        { PH[y * WST + cx] = (uint8_t)(ph >> (8 * i)); PB[y * WST + cx] = (uint8_t)(pb >> (8 * i)); }
                    }
                    w0 = w1; w1 = w2; w2 = w3; w3 = w4; w4 = w5;
                }
            }
            __syncthreads();
            PSTAMP(10);
            for (int y = y0; y < y1; y++) {   // j = clip((6-tap of h1 + 512) >> 10), 32-bit taps
                const uint32_t *hr = reinterpret_cast<const uint32_t *>(s.hs.h1 + y * WST + c0);
                const uint32_t q0 = hr[-1], q1 = hr[0], q2 = hr[1], q3 = hr[2], q4 = hr[3];
                const int x[9] = {(int)(int16_t)q0, (int)q0 >> 16, (int)(int16_t)q1, (int)q1 >> 16, (int)(int16_t)q2,
                                  (int)q2 >> 16, (int)(int16_t)q3, (int)q3 >> 16, (int)(int16_t)q4};
                uint32_t jv = 0;
#pragma unroll
                for (int i = 0; i < 4; i++)
                    jv |= (uint32_t)clip255((tap6(x[i], x[i + 1], x[i + 2], x[i + 3], x[i + 4], x[i + 5]) + 512) >> 10) << (8 * i);
#pragma unroll
                for (int i = 0; i < 4; i++)
                    PJ[y * WST + c0 + i] = (uint8_t)(jv >> (8 * i));
            }
        }
        __syncthreads();   // h1 is dead: its LDS holds the 8x8 SADs from here on
        PSTAMP(2);
#if JMH_I4WAVE
        if (wave == NTS / 64) {   // the last s_barrier this wave meets: the intra decisions from here on
#if !(JMH_EXP & 2)
            intra_wave(d, s.in, scr, mbx, mby);
#endif
            return;
        }
#endif
        {   // ---- P8x8 (4 x 4 stages), the 16x16 / 16x8 / 8x16 searches inside block 3's stages 0, 1
            int best8x8 = 0, cost8x8 = 0;
            p8x8_block<0>(d, s, ps, best8x8, cost8x8, idle, wave, tid);
            PSTAMP(3);
            p8x8_block<1>(d, s, ps, best8x8, cost8x8, idle, wave, tid);
            PSTAMP(4);
            p8x8_block<2>(d, s, ps, best8x8, cost8x8, idle, wave, tid);
            PSTAMP(5);
            p8x8_block<3>(d, s, ps, best8x8, cost8x8, idle, wave, tid);
            // results: MVs of types 1..7, partition costs, P8x8 modes, FindSkipModeMotionVector
            if (tid < 224) {
                const int m = 1 + tid / 32, k = (tid & 31) >> 1, c = tid & 1;
                scr->all_mv[m][k][c] = s.all_mv[m][k][c];
            } else if (tid < 252) {
                const int m = 1 + (tid - 224) / 4, k = tid & 3;
                scr->motion_cost[m][k] = s.motion_cost[m][k];
            } else if (tid == 256) {
                scr->best8x8 = best8x8; scr->cost8x8 = cost8x8;
            } else if (tid == 320) {
                NbBorder nbv{s.bd};
                int ra = -1, ax = 0, ay = 0, rb = -1, bx = 0, by = 0;
                const bool aa = nbv(-1, 0, ra, ax, ay), ab = nbv(0, -1, rb, bx, by);
                const bool zl = !aa || (ra == 0 && ax == 0 && ay == 0), za = !ab || (rb == 0 && bx == 0 && by == 0);
                scr->skipx = (za || zl) ? 0 : pcx;
                scr->skipy = (za || zl) ? 0 : pcy;
            }
            PSTAMP(6);
        }
    }
}

// one MB on 128 threads (tid = 0..127, waves 0 and 1 of the group); every thread of the
// workgroup reaches the same barriers (act: the group has an MB)
template <class pel>
__device__ __forceinline__ void intra_role(const DevParams &d, IntraS<pel> &s, int mbx, int mby, int tid, bool act, bool i4) {
    const int wave = tid >> 6, lane = tid & 63;
    const int pix_x = 16 * mbx, pix_y = 16 * mby, W = d.W;
    const MbAvail mav = intra_avail(d, mbx, mby);
    const bool avL = mav.L, avT = mav.T, avTL = mav.TL, avTR = mav.TR;
    const bool prof = act && prof_mb_here(d, mbx, mby);
    PSTAMP(12);
    if (act) {
        const pel *orgY = spl<pel>(d.orgY);
        s.org[tid] = orgY[(pix_y + (tid >> 4)) * W + pix_x + (tid & 15)];
        s.org[tid + 128] = orgY[(pix_y + 8 + (tid >> 4)) * W + pix_x + (tid & 15)];
        load_orgc(d, s.nb, tid, mbx, mby);
        if (tid < 10) load_border(d, s.bd, tid, mbx, mby);
        else if (tid >= 16 && tid < 16 + 71) load_intra_nb(d, s.nb, tid - 16, mbx, mby);
    }
    MbScratch *scr = d.scr + mby * d.mbw + mbx;
    const int q_bits = 15 + (d.qp + d.qpbd) / 6;
    const int qpk = q_round(d.qsel, q_bits);
    int tabr[2];
    i4_tabrow(lane, tabr);
    int acc[3] = {0, 0, 0};                   // cost, cbp (per b8), block mask
    __syncthreads();
    for (int dg = 0; dg < 10; dg++) {         // blocks with bx4 + 2*by4 == dg, by4 ascending
        const int by_lo = dg > 3 ? (dg - 2) >> 1 : 0;
        const int by4 = by_lo + wave, bx4 = dg - 2 * by4;
        if (act && i4 && by4 <= 3 && bx4 >= 0 && bx4 <= 3) i4_block(d, s, scr, wave, bx4, by4, tabr, avL, avT, avTL, avTR, qpk, acc);
        __syncthreads();
    }
    if (act && lane == 0) { s.part[wave][0] = acc[0]; s.part[wave][1] = acc[1]; s.part[wave][2] = acc[2]; }
    __syncthreads();
    if (!act) return;
    if (i4 && tid == 0) {
        scr->i4cost = 24 * d.lambda_mode + s.part[0][0] + s.part[1][0];   // 4 x (int)floor(6*lambda+0.4999)
        scr->i4cbp = s.part[0][1] | s.part[1][1];
        scr->i4blk = s.part[0][2] | s.part[1][2];
    }
    if (i4 && tid < 16) scr->ipred[tid] = s.ipred_cur[tid];
    if (i4 && tid < (int)sizeof(s.rec) / 4) reinterpret_cast<uint32_t *>(scr->i4rec)[tid] = reinterpret_cast<const uint32_t *>(s.rec)[tid];
    PSTAMP(13);
    // Intra16x16 (wave 0) and intra chroma mode (wave 1) decisions
    if (wave == 0) i16_decision(d, s.org, s.nb, scr, lane, avL, avT, avTL);
    else chroma_decision(d, s.nb, scr, lane, avL, avT, avTL);
    PSTAMP(14);
}

// the Intra4x4 decision inside a motion-search workgroup, on its waves 6 and 7 (w = wave - 6; wave
// 7 as w = 0 in block 3's first stage) while the sub-pel waves of a stage work; steps are separated
// by the stage barriers.  Slot
// k = 0..9: diagonal k of the 4x4 grid; slot 10: the totals and results.
__device__ __forceinline__ void intra_slot(const DevParams &d, IntraS<uint8_t> &s, MbScratch *scr, int k, int w, int mbx, int mby) {
    const int lane = threadIdx.x & 63;
    const MbAvail mav = intra_avail(d, mbx, mby);
    const bool avL = mav.L, avT = mav.T, avTL = mav.TL, avTR = mav.TR;
    if (k == 11) {                                       // k_mb_flow: Intra16x16 (wave 6), chroma (wave 7)
        if (d.i16c) {
            if (w == 0) i16_decision(d, s.org, s.nb, scr, lane, avL, avT, avTL);
            else chroma_decision(d, s.nb, scr, lane, avL, avT, avTL);
        }
    } else if (k < 10) {
        const int q_bits = 15 + d.qp / 6;
        const int qpk = q_round(d.qsel, q_bits);
        int tabr[2];
        i4_tabrow(lane, tabr);
        const int by_lo = k > 3 ? (k - 2) >> 1 : 0;
        const int by4 = by_lo + w, bx4 = k - 2 * by4;
        if (by4 <= 3 && bx4 >= 0 && bx4 <= 3) {   // the wave's running cost / cbp / block mask live in LDS
            int acc[3] = {s.part[w][0], s.part[w][1], s.part[w][2]};
            unsigned long long *pst = (k == 4 && w == 0 && d.prof && d.prof_mb == mby * d.mbw + mbx) ? d.prof : nullptr;   // debug stamps
            i4_block(d, s, scr, w, bx4, by4, tabr, avL, avT, avTL, avTR, qpk, acc, pst);
            if (lane == 0) { s.part[w][0] = acc[0]; s.part[w][1] = acc[1]; s.part[w][2] = acc[2]; }
        }
    } else if (w == 0) {
        if (lane == 0) {
            scr->i4cost = 24 * d.lambda_mode + s.part[0][0] + s.part[1][0];   // 4 x (int)floor(6*lambda+0.4999)
            scr->i4cbp = s.part[0][1] | s.part[1][1];
            scr->i4blk = s.part[0][2] | s.part[1][2];
        }
        if (lane < 16) scr->ipred[lane] = s.ipred_cur[lane];
        reinterpret_cast<uint32_t *>(scr->i4rec)[lane] = reinterpret_cast<const uint32_t *>(s.rec)[lane];
    }
}

// JMH_I4WAVE: the intra decisions of a P macroblock on wave 7 of its motion-search workgroup, on
// a schedule of their own (the search waves synchronise among themselves, search_sync): Intra4x4
// over the 16 blocks in JM's decoding order on one wave (each block's neighbours are earlier in
// it; the LDS writes of one wave are seen by its later reads), then the Intra16x16 and chroma
// intra-mode decisions, so that no intra workgroup runs for a P picture's MBs
__device__ __forceinline__ void intra_wave(const DevParams &d, IntraS<uint8_t> &s, MbScratch *scr, int mbx, int mby) {
    const int lane = __lane_id();
    const bool prof = prof_mb_here(d, mbx, mby, NTS / 64);   // debug (JMH_PHASE_PROF): stamps 60..62
    PSTAMP(60);
    const MbAvail mav = intra_avail(d, mbx, mby);
    const int qpk = q_round(d.qsel, 15 + d.qp / 6);
    int tabr[2];
    i4_tabrow(lane, tabr);
    int acc[3] = {0, 0, 0};                   // cost, cbp (per b8), block mask
    for (int blk = 0; blk < 16; blk++) {
        const int bx4 = 2 * ((blk >> 2) & 1) + (blk & 1), by4 = 2 * (blk >> 3) + ((blk >> 1) & 1);
        i4_block(d, s, scr, 0, bx4, by4, tabr, mav.L, mav.T, mav.TL, mav.TR, qpk, acc);
    }
    if (lane == 0) {
        scr->i4cost = 24 * d.lambda_mode + acc[0];   // 4 x (int)floor(6*lambda+0.4999)
        scr->i4cbp = acc[1];
        scr->i4blk = acc[2];
    }
    if (lane < 16) scr->ipred[lane] = s.ipred_cur[lane];
    reinterpret_cast<uint32_t *>(scr->i4rec)[lane] = reinterpret_cast<const uint32_t *>(s.rec)[lane];
    PSTAMP(61);
    i16_decision(d, s.org, s.nb, scr, lane, mav.L, mav.T, mav.TL);
    chroma_decision(d, s.nb, scr, lane, mav.L, mav.T, mav.TL);
    PSTAMP(62);
}

#ifndef JMH_FLOW_TU   // the tick kernels (jmh_flow.hip builds k_mb_flow from the same device functions)
__global__ __launch_bounds__(NTA, 4) void k_mb_analyse(const TickArgs t) {
    __shared__ AnalyseS s;
    // blocks: [0, nPm) the motion search of each P picture MB with its Intra4x4 decision (longest,
    // dispatched first), then intra workgroups over every MB, four MBs (128 threads each) per
    // workgroup: Intra16x16 + chroma decisions, and Intra4x4 for MBs without a motion-search
    // workgroup (I pictures; SearchMode -1, where k_mb_me_full searched)
    const int nPm = t.me_in_analyse ? t.pre[t.nP] : 0, nPg = xcd_grid(nPm), tot = t.pre[t.npic], b = blockIdx.x;
    const unsigned long long t0 = t.bprof ? wall_clock64() : 0;
    const bool first_thread = threadIdx.x == 0;   // a lane mask: threadIdx itself dies early
    const int role = b < nPg ? 2 : 0;
    unsigned long long tag = role;                            // debug (JMH_BLOCK_PROF): role | MB << 4 | entry << 32
    if (role == 2) {
        const int m = xcd_block(b, nPm);                      // XCD-aware: neighbouring MBs share an L2
        if (m >= nPm) return;                                 // padding block (whole workgroup)
        const int e = tick_entry(t, m);
        const DevParams d = tick_params(t, e);
        const int mby = d.y_min + (m - t.pre[e]), mbx = d.diag - 2 * mby;
        tag = 2u | (unsigned long long)(mby * d.mbw + mbx) << 4 | (unsigned long long)e << 32;
        me_mb(d, s.me, mbx, mby);
    } else {
        const int q = __builtin_amdgcn_readfirstlane((JMH_I4WAVE ? nPm : 0) + 4 * (b - nPg) + (int)(threadIdx.x >> 7));
        const bool act = q < tot;
        const int e = tick_entry(t, act ? q : 0);
        const DevParams d = tick_params(t, e);
        const int mby = d.y_min + ((act ? q : t.pre[e]) - t.pre[e]), mbx = d.diag - 2 * mby;
        intra_role(d, s.in[threadIdx.x >> 7], mbx, mby, threadIdx.x & 127, act, q >= nPm);
    }
    if (t.bprof) {
        __syncthreads();
        if (first_thread) {
            t.bprof[3 * b] = t0;
            t.bprof[3 * b + 1] = wall_clock64();
            t.bprof[3 * b + 2] = tag;
        }
    }
}

// The intra analysis of a tick whose motion search has its own kernel (SearchMode -1: k_mb_me_full,
// 3: k_mb_epzs): every MB's Intra4x4 + Intra16x16 + chroma decisions (intra_role, two MBs per
// 256-thread workgroup) and, in the High profile, its Intra8x8 decision (intra8_mb, one MB per
// workgroup) in ONE launch of small workgroups -- instead of k_mb_analyse's 512-thread, 78 KB LDS
// workgroups followed by k_mb_intra8 -- so the two independent decisions share the CUs (eight
// workgroups per CU): blocks [0, nRg) the intra roles (longest, first), then the Intra8x8 blocks.
#ifndef JMH_INTRA_OCC
#define JMH_INTRA_OCC 8                       // waves per SIMD the register budget targets (A/B: -D)
#endif
template <class pel>
__global__ __launch_bounds__(NT, JMH_INTRA_OCC) void k_mb_intra(const TickArgs t) {
    __shared__ union {
        IntraS<pel> in[2];
        I8S<pel> i8;
    } s;
    const int tot = t.pre[t.npic], nR = (tot + 1) / 2, nRg = xcd_grid(nR), b = blockIdx.x;
    if (b < nRg) {
        const int r = xcd_block(b, nR);
        if (r >= nR) return;                                   // padding block (whole workgroup)
        const int q = __builtin_amdgcn_readfirstlane(2 * r + (int)(threadIdx.x >> 7));
        const bool act = q < tot;
        const int e = tick_entry(t, act ? q : 0);
        const DevParams d = tick_params(t, e);
        const int mby = d.y_min + ((act ? q : t.pre[e]) - t.pre[e]), mbx = d.diag - 2 * mby;
        intra_role(d, s.in[threadIdx.x >> 7], mbx, mby, threadIdx.x & 127, act, true);
    } else {
        const int mi = xcd_block(b - nRg, tot);
        if (mi >= tot) return;
        intra8_mb<pel>(t, s.i8, mi);
    }
}

hipError_t jmh_launch_intra(const TickArgs &t, hipStream_t st) {
    const int tot = t.pre[t.npic];
    const int nblocks = xcd_grid((tot + 1) / 2) + (t.t8 ? xcd_grid(tot) : 0);
    if (t.bd > 8) hipLaunchKernelGGL(k_mb_intra<uint16_t>, dim3(nblocks), dim3(NT), 0, st, t);
    else hipLaunchKernelGGL(k_mb_intra<uint8_t>, dim3(nblocks), dim3(NT), 0, st, t);
    return hipGetLastError();
}

hipError_t jmh_launch_analyse(const TickArgs &t, hipStream_t st) {
    const int nPm = t.me_in_analyse ? t.pre[t.nP] : 0;   // JMH_I4WAVE: their intra decisions ran on wave 7
    const int nblocks = xcd_grid(nPm) + (t.pre[t.npic] - (JMH_I4WAVE ? nPm : 0) + 3) / 4;
    if (nblocks == 0) return hipSuccess;
    hipLaunchKernelGGL(k_mb_analyse, dim3(nblocks), dim3(NTA), 0, st, t);
    return hipGetLastError();
}
#endif

#ifdef JMH_FLOW_TU
// ======================================================================================
//  k_mb_flow: the dataflow wavefront (jmh_device.h FlowArgs)
// ======================================================================================
__device__ __forceinline__ DevParams flow_params(const FlowArgs &f, const PicParams &q) {
    DevParams d;
    d.W = f.W; d.H = f.H; d.Wc = f.W >> 1; d.Hc = f.H >> 1; d.mbw = f.mbw; d.mbh = f.mbh;
    d.sr = f.sr; d.side = 2 * f.sr + 1; d.npos = d.side * d.side;
    d.search_mode = f.search_mode; d.use_hadamard = f.use_hadamard; d.restrict_sr = f.restrict_sr;
    d.isr = f.isr;
    d.t8 = 0;
    d.epzs_dual = 0; d.epzs_subpel = 0; d.epzs_spts = 0; d.epzs_mints = 0; d.epzs_maxts = 0;
    d.slice_mbs = f.slice_mbs;
    d.maxv = 255; d.qpbd = 0;
    const int ls = f.W * f.H, lc = ls >> 2;
    d.orgY = q.org; d.orgU = q.org + ls; d.orgV = q.org + ls + lc;
    d.refY = q.ref; d.refU = q.ref + ls; d.refV = q.ref + ls + lc;
    d.recY = q.rec; d.recU = q.rec + ls; d.recV = q.rec + ls + lc;
    d.dbkY = q.dbk; d.dbkU = q.dbk ? q.dbk + ls : nullptr; d.dbkV = q.dbk ? q.dbk + ls + lc : nullptr;
    d.lf_disable = q.lf_disable; d.lf_offA = q.lf_offA; d.lf_offB = q.lf_offB;
    d.mv = q.mv; d.refidx = q.refidx; d.ipred = q.ipred; d.res = q.res; d.scr = q.scr;
    d.tmv = nullptr; d.tref = nullptr; d.ordtab = f.ordtab;
    d.prof = f.prof; d.prof_mb = f.prof_mb;
    d.slice_type = q.slice_type; d.qp = q.qp; d.lambda_mode = q.lambda_mode; d.lambda_motion = q.lambda_motion;
    d.cqp_off = q.cqp_off; d.qsel = q.qsel; d.diag = q.diag; d.y_min = q.y_min;
    d.rdo = 0; d.cavlc = 0;
    d.i16c = 1;
    d.cip = 0;                                           // (the dataflow path runs without UseConstrainedIntraPred)
    d.lf = q.lambda_motion << 16;
    d.lambda_rd = 0;
    d.rp = nullptr;
    return d;
}

// k_mb_flow's luma MC: the quarter-pel sample at (X, Y) from the P macroblock's search window
// planes still in LDS (G, b, h, j at window coordinates; ox / oy: the window origin in the
// picture), the same values as qpel_direct (the window is the clamped reference and the planes
// its 6-tap half samples).  The final's MVs are the searches' results, within +-(SR + 3/4) of the
// window centre, so every sample lies in the planes' rows / columns [3, 2 SR + 21).
struct PlaneMC {
    uint32_t g;                                // LDS byte address of the G plane
    int ox, oy;
    __device__ __forceinline__ int at(int plane, int x, int y) const {
        return ((lds_cu8 *)(uintptr_t)(g + plane * PLS + y * WST + x))[0];
    }
    __device__ __forceinline__ int operator()(int X, int Y) const {
        const int x = (X >> 2) - ox, y = (Y >> 2) - oy, fx = X & 3, fy = Y & 3;
        if (fy == 0) {
            const int G = at(0, x, y);
            if (fx == 0) return G;
            const int b = at(1, x, y);
            return fx == 2 ? b : ((fx == 1 ? G : at(0, x + 1, y)) + b + 1) >> 1;
        }
        if (fx == 0) {
            const int h = at(2, x, y);
            return fy == 2 ? h : ((fy == 1 ? at(0, x, y) : at(0, x, y + 1)) + h + 1) >> 1;
        }
        if ((fx & 1) && (fy & 1)) return (at(1, x, fy == 1 ? y : y + 1) + at(2, fx == 1 ? x : x + 1, y) + 1) >> 1;   // e g p r
        const int j = at(3, x, y);
        if (fx == 2 && fy == 2) return j;
        const int o = fx == 2 ? at(1, x, fy == 1 ? y : y + 1) : at(2, fx == 1 ? x : x + 1, y);   // f q / i k
        return (j + o + 1) >> 1;
    }
};

#define FLOW_SPIN_MAX (1 << 17)               // polls before a dependency wait gives up (~0.1 s; a wait
                                              // lasts a few macroblocks, ~0.2 ms, at most)
__device__ __forceinline__ bool flow_done(const FlowArgs &f, int e, int mb, uint32_t gen) {
    return __hip_atomic_load(f.flags + (size_t)e * f.nmb + mb, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= gen;
}

// Persistent: every workgroup claims tickets until the segment is exhausted.  Per macroblock: its
// left and top-right (top at the right edge) neighbours and the reference picture's MB (x+5, y+5)
// (PIPE_LAG's reach, clamped) must be done -- the rest of the wavefront's dependencies follow from
// theirs; then the P macroblock's me_mb (41 searches + Intra4x4), its Intra16x16 / chroma
// decisions on waves 0 / 1 (or an I macroblock's intra_role), and final_core on all 512 threads.
// Publication: every wave's stores drained, the workgroup barrier, one agent-scope release, the
// flag; a waiter polls relaxed, then one agent-scope acquire before the workgroup reads
// (MI355X_MICROARCH.md, inter-workgroup visibility).
// One workgroup per macroblock of the segment (grid = the segment's MB count), which claims its
// macroblock by an atomic ticket when it starts, so the MBs run in tick order as the hardware
// dispatches workgroups into freed slots.  Per macroblock: its left and top-right (top at the
// right edge) neighbours and the reference picture's MB (x+5, y+5) (PIPE_LAG's reach, clamped) must
// be done -- the rest of the wavefront's dependencies follow from theirs; a claimed ticket belongs
// to a running workgroup and waits only on smaller tickets, so every wait ends.  Then the P
// macroblock's me_mb (41 searches + Intra4x4), its Intra16x16 / chroma decisions on waves 0 / 1 (an
// I macroblock: intra_role), and final_core on all 512 threads.  Publication: every wave's stores
// drained, the workgroup barrier, one agent-scope release, the flag; a waiter polls relaxed, then
// one agent-scope acquire before the workgroup reads (MI355X_MICROARCH.md, inter-workgroup
// visibility).
__global__ __launch_bounds__(NTA, 4) void k_mb_flow(const FlowArgs f) {
    // the final's LDS beside the analysis' (81.1 KB: still two workgroups per CU), so that it reads
    // the MB's source, intra neighbourhood and search window planes where the analysis left them
    __shared__ struct {
        FinS<uint8_t> fin;
        AnalyseS a;
    } s;
    __shared__ int s_item;
    __shared__ unsigned s_tk;
    const int tid = threadIdx.x;
    const unsigned long long t0 = f.fprof ? wall_clock64() : 0;
    if (tid == 0) {
        const unsigned n = atomicAdd(f.head, 1u) - f.base;   // < nitems: one ticket per workgroup
        s_tk = n;
        int item = n < (unsigned)f.nitems ? (int)f.items[n] : -1;
        // (never expected) a ticket or item out of range: reported, the workgroup does nothing
        if (item < 0 || (item >> 24) >= f.nring || ((item >> 12) & 0xFFF) >= f.mbh || (item & 0xFFF) >= f.mbw) {
            __hip_atomic_store(f.err + 1, n, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            __hip_atomic_store(f.err + 2, (unsigned)item, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            __hip_atomic_store(f.err, 2u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            item = -1;
        }
        s_item = item;
    }
    __syncthreads();
    const int item = __builtin_amdgcn_readfirstlane(s_item);   // uniform: the parameters stay scalar loads
    if (item < 0) return;
    const int e = item >> 24, mby = (item >> 12) & 0xFFF, mbx = item & 0xFFF;
    const bool pslice = f.pics[e].pp.slice_type == JMH_P_SLICE;
    if (pslice) {   // what reads no other workgroup's output, while the dependencies finish
        const DevParams d = flow_params(f, f.pics[e].pp);
        me_prologue(d, s.a.me, mbx, mby);
        if (tid >= 256 && tid < 384) load_orgc(d, s.a.me.in.nb, tid - 256, mbx, mby);   // the chroma decision's source
    }
    if (tid == 0) {
        const FlowPic &P = f.pics[e];
        const uint32_t g = P.gen;
        const int mb = mby * f.mbw + mbx;
        const int re = pslice ? P.ref_entry : -1;
        const int rmb = min(mby + 5, f.mbh - 1) * f.mbw + min(mbx + 5, f.mbw - 1);
        const int tmb = mby > 0 ? (mbx + 1 < f.mbw ? mb - f.mbw + 1 : mb - f.mbw) : -1;
        // bounded: after FLOW_SPIN_MAX polls (or once any wait of the launch has timed out) the
        // workgroup goes on and the host reports the launch as failed
        int spin = 0;
        while (!((mbx == 0 || flow_done(f, e, mb - 1, g)) && (tmb < 0 || flow_done(f, e, tmb, g)) &&
                 (re < 0 || flow_done(f, re, rmb, P.ref_gen)))) {
            __builtin_amdgcn_s_sleep(2);
            if (++spin > FLOW_SPIN_MAX) { __hip_atomic_store(f.err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM); break; }
            if ((spin & 63) == 0 && __hip_atomic_load(f.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM)) break;
        }
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __syncthreads();
    // debug stamps (JMH_FLOW_PROF): the slot is re-derived at each use, nothing stays live across me_mb
#define FLOW_FP (f.fprof ? f.fprof + 6 * (size_t)__builtin_amdgcn_readfirstlane(s_tk) : nullptr)
    if (unsigned long long *fp = FLOW_FP; fp && tid == 0) {
        fp[0] = t0;
        fp[1] = wall_clock64();
        const unsigned hw = __builtin_amdgcn_s_getreg((4 << 0) | (0 << 6) | (15 << 11));    // HW_ID bits 0..15
        const unsigned xcc = __builtin_amdgcn_s_getreg((20 << 0) | (0 << 6) | (3 << 11));   // XCC_ID bits 0..3
        fp[5] = (unsigned long long)(hw | xcc << 16) << 32 | (unsigned)item;
    }
    {   // the analysis (DevParams scoped per phase: one set live across me_mb spills)
        const DevParams d = flow_params(f, f.pics[e].pp);
        if (pslice) me_mb(d, s.a.me, mbx, mby, true);
        else intra_role(d, s.a.in[tid >> 7], mbx, mby, tid & 127, tid < 128, true);
    }
    if (unsigned long long *fp = FLOW_FP; fp && tid == 0) fp[2] = wall_clock64();
    asm volatile("" ::: "memory");                            // re-read the parameters below
    {
        const DevParams d = flow_params(f, f.pics[e].pp);
        const bool prof = prof_mb_here(d, mbx, mby);
        PSTAMP(56);
        __syncthreads();                                      // MbScratch complete
        PSTAMP(58);
        int pcx = 0, pcy = 0;                                 // me_mb's window origin (SetupFastFullPelSearch centre)
        if (pslice) set_mvp(NbBorder{s.a.me.bd}, 0, 0, 16, 16, pcx, pcy);
        const int scx = iclip(-d.sr, d.sr, pcx / 4), scy = iclip(-d.sr, d.sr, pcy / 4);
        const PlaneMC mc{(uint32_t)(uintptr_t)(lds_cu8 *)s.a.me.planes, 16 * mbx + scx - d.sr - WM, 16 * mby + scy - d.sr - WM};
        IntraS<uint8_t> &in = pslice ? s.a.me.in : s.a.in[0];  // (I macroblocks: no MC)
        final_core<5, uint8_t, false, NTA>(d, s.fin, mbx, mby, tid, mc, in.org, &in.nb);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0) {
        unsigned long long *fp = FLOW_FP;
        if (fp) fp[3] = wall_clock64();
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __hip_atomic_store(f.flags + (size_t)e * f.nmb + mby * f.mbw + mbx, f.pics[e].gen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (fp) fp[4] = wall_clock64();
    }
#undef FLOW_FP
}

hipError_t jmh_launch_flow(const FlowArgs &f, hipStream_t st) {
    if (f.nitems <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_mb_flow, dim3(f.nitems), dim3(NTA), 0, st, f);
    return hipGetLastError();
}
#endif

#ifdef JMH_ISA_PROBE
// ISA inspection only (hipcc -DJMH_ISA_PROBE -S): one sub-pel search of a 4x4 and of an 8x8 block
__global__ __launch_bounds__(NTA, 4) void k_probe_subpel(const TickArgs t, int j) {
    __shared__ MeS s;
    const DevParams d = tick_params(t, 0);
    const SDesc q4 = {7, 1, 0, 0, 7, 0, 1, 0}, q8 = {4, 0, 0, 0, 0, 0, 0, 0};
    if (j) subpel_wave(d, s, 0, q4, t.W, t.H, 3, -2, 0, 0);
    else subpel_wave(d, s, 0, q8, t.W, t.H, 3, -2, 0, 0);
    __syncthreads();
    if (threadIdx.x < 64) d.mv[threadIdx.x] = s.all_mv[j ? 7 : 4][threadIdx.x & 15][threadIdx.x >> 4 & 1] + s.motion_cost[4][0] + s.pmv[0][0];
}
#endif
