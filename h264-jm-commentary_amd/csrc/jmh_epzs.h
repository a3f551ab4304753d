// jmh_epzs.h -- the EPZS motion search of one macroblock on one wave (k_mb_epzs, k_rdo_inter):
// LDS state, predictor list, full-pel SADs, refinement, sub-pel (see jmh_epzs.hip's header).
#pragma once
#include "jmh_common.h"

// WEIGHTED_COST(lambda_factor, bits) [J]: lambda * bits for the integer RDO-off lambda (24-bit
// multiply), (LAMBDA_FACTOR * bits) >> 16 with the RDO lambda factor (RDOptimization 1)
__device__ __forceinline__ int wcost(const DevParams &d, int bits) {
    return d.rdo ? (int)(((unsigned)d.lf * (unsigned)bits) >> 16) : (int)__umul24(d.lambda_motion, bits);
}

#define NTE 64                                // one wave per macroblock
#ifndef EOFF_L                                // (-DEOFF_L=...: A/B builds)
#define EOFF_L 48                             // LDS window margin around the MB (or 2 SR + 4 if less;
                                              //   A/B on config 3: profiles/r7j_window_ab.txt)
#endif
// window loads in flight per lane (one batch of global loads per round trip)
#ifndef EPZS_NB8
#define EPZS_NB8 32
#endif
#ifndef EPZS_NB16
#define EPZS_NB16 16
#endif
#ifndef EPZS_FB_ROWS
#define EPZS_FB_ROWS 4                        // k_rdo_inter: block rows per batch of global loads when a SAD
#endif                                        //   leaves the window (k_mb_epzs: 1; A/B profiles/r7x_fallback_ab.txt)
#ifndef EPZS_EDGE
#define EPZS_EDGE 0                           // samples a window SAD needs right of its block: none -- the extra
#endif                                        //   dword a row reads for v_alignbyte only feeds unused bytes, and
                                              //   past the window's last row it stays inside EpzS (gn follows g)
#ifndef EOFF_L16
#define EOFF_L16 40                           // ... for 16-bit samples: 30.4 KB k_rdo_inter, five MBs per CU (A/B: profiles/r5r_window_ab.txt)
#endif
// window geometry per sample type: margin, rows (= row stride) of the LDS window
template <class pel>
struct EGeo {
    static constexpr int off = sizeof(pel) == 2 ? EOFF_L16 : EOFF_L;
    static constexpr int ew = 16 + 2 * off;
    static_assert(off % 2 == 0, "window rows must be whole dwords");
    // ffs_build_phase reads every table position straight from the window, with no global
    // fallback: the margin must cover SRMAX + 3 (the 6-tap reach) around the FFS centre
    static_assert(off >= SRMAX + 3, "the FFS SAD table (RDO + SearchMode 0) needs a window margin >= SRMAX + 3");
};
#define NPRED 41                              // EPZS predictor slots (oracle epzs_predictors)
#define HPS 20                                // sub-pel plane stride (>= 18 + 2 alignment slack)
#define HPR 18                                // sub-pel plane rows (block + 1 on each side)
#define HPL (HPR * HPS + 8)                   // sub-pel plane size (b, h, j)
#define EKOFF 4096                            // sub-pel cost offset in keys (16x16 zero-vector bias)
#define GNX 8                                 // sub-pel neighbourhood plane (a search whose reach leaves
#define GNY 5                                 //   the window): block-relative x in [-GNX, 4 w4 + 2 + GNX),
#define GNS 36                                //   y in [-GNY, 4 h4 + 2 + GNY), stride GNS
#define GNR (18 + 2 * GNY)

template <class pel> struct EpzTap { typedef int16_t type; };   // unclipped 6-tap sums: |.| <= 42 * maxv
template <> struct EpzTap<uint16_t> { typedef int32_t type; };
template <class pel>
struct EpzS {
    alignas(4) pel g[EGeo<pel>::ew * EGeo<pel>::ew];           // the window
    alignas(4) pel gn[GNR * GNS + 8];         // a search's integer-sample neighbourhood read from global
    alignas(8) pel org[256];
    Border bd;
    int16_t all_mv[8][16][2];
    int motion_cost[8][4];
    int16_t tmv[6][6][2];                     // previous picture's MVs around the MB (4x4 units,
    int8_t tref[6][6];                        //   MB origin at [1][1]; -1: none)
    int16_t mem[7][16][2];                    // spatial memory: the left MB's searches (types 1..7)
    int memok;
    int scx, scy;                             // RDO with FFS (item 65): the MB's window centre
    uint16_t fpc[7][16];                      // item 61: this MB's full-pel costs per type and 4x4,
    uint16_t fpb[7][10];                      //   the neighbour MBs' at the border cells (1..9)
    alignas(4) pel hp[3][HPL];                // b, h, j of the block's [-1, w] x [-1, h] at its MV
    typename EpzTap<pel>::type b1[HPR + 5][HPR];   // unclipped horizontal taps, rows -3 .. h + 1
};

// neighbour view of a search of block type bt in 8x8 block b8 (as NbMe in jmh_analyse.hip)
template <class S>
struct NbEpz {
    const S &s;
    int bt, b8, best8x8;
    __device__ __forceinline__ bool operator()(int xN, int yN, int &ref, int &mx, int &my) const {
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

__device__ __forceinline__ uint32_t eld_u32(const void *p) { return lds_u32_any(p); }   // 4 bytes at any LDS address

// the LDS window: picture position of its sample (0, 0) and window position of the MB origin
template <class pel>
struct EWin {
    const pel *ref;
    int W, H;
    int wx0, wy0, mx, my;
};
// reference sample at picture position (x, y), UMV-clamped (8.4.2.2.1), from global memory
template <class pel>
__device__ __forceinline__ uint32_t gref(const EWin<pel> &w, int x, int y) {
    return w.ref[iclip(0, w.H - 1, y) * w.W + iclip(0, w.W - 1, x)];
}

// the spatial neighbours A, B, C (or D) of a block as SetMotionVectorPredictor reads them (H.264
// 8.4.1.3), and the MVP from them (set_mvp's rules): EPZS predictors 2-4 are the same reads
struct MvpNb {   // scalar fields: a lane-indexed array would live in scratch
    int va, ra, xa, ya, vb, rb, xb, yb, vc, rc, xc, yc;
};
template <class NB>
__device__ __forceinline__ void set_mvp_nb(const NB &nb, int bx4, int bby4, int bsx, int bsy, int &px, int &py, MvpNb &n) {
    int ra = -1, rb = -1, rc = -1, rd = -1, ax = 0, ay = 0, bxv = 0, byv = 0, cx = 0, cy = 0, dx = 0, dy = 0;
    const int mb_x = 4 * bx4, mb_y = 4 * bby4;
    const bool av_a = nb(mb_x - 1, mb_y, ra, ax, ay);
    const bool av_b = nb(mb_x, mb_y - 1, rb, bxv, byv);
    bool av_c = nb(mb_x + bsx, mb_y - 1, rc, cx, cy);
    const bool av_d = nb(mb_x - 1, mb_y - 1, rd, dx, dy);
    if (mb_y > 0) {
        if (mb_x < 8) {
            if (mb_y == 8) { if (bsx == 16) av_c = false; }
            else if (mb_x + bsx == 8) av_c = false;
        } else if (mb_x + bsx == 16) av_c = false;
    }
    if (!av_c) { av_c = av_d; rc = rd; cx = dx; cy = dy; }
    n.va = av_a; n.ra = ra; n.xa = ax; n.ya = ay;
    n.vb = av_b; n.rb = rb; n.xb = bxv; n.yb = byv;
    n.vc = av_c; n.rc = rc; n.xc = cx; n.yc = cy;
    const int rL = av_a ? ra : -1, rU = av_b ? rb : -1, rUR = av_c ? rc : -1;
    int type = 0;
    if (rL == 0 && rU != 0 && rUR != 0) type = 1;
    else if (rL != 0 && rU == 0 && rUR != 0) type = 2;
    else if (rL != 0 && rU != 0 && rUR == 0) type = 3;
    if (bsx == 8 && bsy == 16) { if (mb_x == 0) { if (rL == 0) type = 1; } else if (rUR == 0) type = 3; }
    else if (bsx == 16 && bsy == 8) { if (mb_y == 0) { if (rU == 0) type = 2; } else if (rL == 0) type = 1; }
    const int A[2] = {av_a ? ax : 0, av_a ? ay : 0}, B[2] = {av_b ? bxv : 0, av_b ? byv : 0}, C[2] = {av_c ? cx : 0, av_c ? cy : 0};
    int p[2];
#pragma unroll
    for (int hv = 0; hv < 2; hv++) {
        const int a = A[hv], b = B[hv], c = C[hv];
        if (type == 1) p[hv] = a;
        else if (type == 2) p[hv] = b;
        else if (type == 3) p[hv] = c;
        else if (!(av_b || av_c)) p[hv] = a;
        else p[hv] = a + b + c - min(a, min(b, c)) - max(a, max(b, c));
    }
    px = p[0]; py = p[1];
}

// EPZS predictor i of a search (oracle/encode.c epzs_predictors order): 0 centre, 1 zero, 2-4
// spatial A / B / C (or D) (nb: the MVP's neighbour reads), 5-28 window rings R/4, R/2, R,
// 29-33 temporal (co-located, left, right, up, down), 34 spatial memory (left MB), 35-40 earlier
// block types.  False if not valid or outside the window around the centre.
template <class S>
__device__ __forceinline__ bool epzs_cand(const DevParams &d, const S &s, int i, int bt, int bx4, int by4, const MvpNb &nb,
                                          int range, int mvx0, int mvy0, int &x, int &y) {
    const int w4 = 1 << lw4_of(bt), h4 = 1 << lh4_of(bt), k0 = by4 * 4 + bx4;
    auto rnd = [](int v) { return (v + 2) >> 2; };
    bool v = true;
    x = 0; y = 0;
    if (i == 0) { x = mvx0; y = mvy0; }
    else if (i == 1) { }
    else if (i <= 4) {
        const int k = i - 2;
        // bit masks, not selects: a select of struct fields becomes an indexed scratch load
        const int m0 = -(k == 0), m1 = -(k == 1), m2 = -(k == 2);
        const int av = (nb.va & m0) | (nb.vb & m1) | (nb.vc & m2), ref = (nb.ra & m0) | (nb.rb & m1) | (nb.rc & m2);
        v = av && ref == 0;
        x = rnd((nb.xa & m0) | (nb.xb & m1) | (nb.xc & m2));
        y = rnd((nb.ya & m0) | (nb.yb & m1) | (nb.yc & m2));
    } else if (i <= 28) {
        const int ring = (i - 5) >> 3, k = (i - 5) & 7, rr = range >> (2 - ring);
        const int wx = k == 1 || k == 4 || k == 6 ? -1 : k == 2 || k == 5 || k == 7 ? 1 : 0;
        const int wy = k == 0 || k == 4 || k == 5 ? -1 : k == 3 || k == 6 || k == 7 ? 1 : 0;
        v = rr > 0; x = mvx0 + rr * wx; y = mvy0 + rr * wy;
    } else if (i <= 33) {
        const int k = i - 29;
        const int tx = 1 + bx4 + (k == 1 ? -1 : k == 2 ? w4 : 0), ty = 1 + by4 + (k == 3 ? -1 : k == 4 ? h4 : 0);
        v = s.tref[ty][tx] == 0;
        x = rnd(s.tmv[ty][tx][0]); y = rnd(s.tmv[ty][tx][1]);
    } else if (i == 34) {
        v = s.memok && inter_on(d.isr, bt);
        x = rnd(s.mem[bt - 1][k0][0]); y = rnd(s.mem[bt - 1][k0][1]);
    } else if (i < NPRED) {
        const int t = i - 34;
        v = t < bt && inter_on(d.isr, t);
        x = rnd(s.all_mv[t][k0][0]); y = rnd(s.all_mv[t][k0][1]);
    } else v = false;
    return v && abs(x - mvx0) <= range && abs(y - mvy0) <= range;
}

// offsets (dx + 4) | (dy + 4) << 4 of the 41 positions with |dx| + |dy| <= 4 (refinement batches)
// the 41 points with |dx| + |dy| <= 4 in raster order, (dy + 4) << 4 | (dx + 4), from the lane
// index by arithmetic (a per-lane table read is a vector memory round trip in every batch): row r
// (dy = r - 4) of the diamond starts after 0, 1, 4, 9, 16, 25, 32, 37, 40 points and its centre
// (dx = 0) is point 0, 2, 6, 12, 20, 28, 34, 38, 40 (6 bits each below)
__device__ __forceinline__ int dia41(int L) {
    const int r = (L >= 1) + (L >= 4) + (L >= 9) + (L >= 16) + (L >= 25) + (L >= 32) + (L >= 37) + (L >= 40);
    const int dx = L - (int)((0x289a2714306080ull >> (6 * r)) & 63);
    return r << 4 | (dx + 4);
}

// refinement pattern point e: small diamond (0,-1) (-1,0) (1,0) (0,1); extended diamond (0,-2)
// (-1,-1) (1,-1) (-2,0) (2,0) (-1,1) (1,1) (0,2) then the small diamond
__device__ __forceinline__ void epzs_pat(bool sd, int e, int &px, int &py) {
    if (sd) { px = e == 1 ? -1 : e == 2 ? 1 : 0; py = e == 0 ? -1 : e == 3 ? 1 : 0; return; }
    px = e < 8 ? (e == 1 || e == 5 ? -1 : e == 2 || e == 6 ? 1 : e == 3 ? -2 : e == 4 ? 2 : 0) : (e == 9 ? -1 : e == 10 ? 1 : 0);
    py = e < 8 ? (e == 0 ? -2 : e <= 2 ? -1 : e <= 4 ? 0 : e <= 6 ? 1 : 2) : (e == 8 ? -1 : e == 11 ? 1 : 0);
}

// SAD of the whole block (4 w4 x 4 h4 at 4x4 position bx4, by4) at full-pel displacement (x, y)
// on this lane: per row w4 + 1 aligned dwords, v_alignbyte, v_sad_u8 (16-bit samples: 2 w4 + 1
// dwords, v_sad_u16)
template <int LW4, int LH4, class pel, int FBR = 1>
__device__ __forceinline__ unsigned lane_block_sad(const EpzS<pel> &s, const EWin<pel> &wn, int bx4, int by4, int x, int y) {
    constexpr int W4 = 1 << LW4, H = 4 << LH4;
    static_assert(H % FBR == 0, "fallback row batches must tile the block");
    const int gx = wn.mx + 4 * bx4 + x, gy = wn.my + 4 * by4 + y;
    const uint32_t *org = reinterpret_cast<const uint32_t *>(s.org + (4 * by4) * 16 + 4 * bx4);
    uint32_t sad = 0;
    if constexpr (sizeof(pel) == 2) {
        constexpr int ND = 2 * W4;            // dwords of a block row
        if (gx >= 0 && gx + 4 * W4 + EPZS_EDGE <= EGeo<pel>::ew && gy >= 0 && gy + H <= EGeo<pel>::ew) {
            const int a = gy * EGeo<pel>::ew + gx;
            const uint32_t sel = (uint32_t)(a & 1) * 2;
            const uint32_t *base = reinterpret_cast<const uint32_t *>(s.g + (a & ~1));
#pragma unroll
            for (int r = 0; r < H; r++) {
                uint32_t w[ND + 1];
#pragma unroll
                for (int q = 0; q <= ND; q++) w[q] = base[r * (EGeo<pel>::ew / 2) + q];
#pragma unroll
                for (int q = 0; q < ND; q++) sad = __builtin_amdgcn_sad_u16(__builtin_amdgcn_alignbyte(w[q + 1], w[q], sel), org[r * 8 + q], sad);
            }
        } else {   // outside: the reference picture in global memory, clamped, FBR rows per round trip
            const int px = wn.wx0 + gx, py = wn.wy0 + gy;
#pragma unroll 1
            for (int r0 = 0; r0 < H; r0 += FBR) {
                uint32_t v[FBR][ND];
#pragma unroll
                for (int r = 0; r < FBR; r++)
#pragma unroll
                    for (int q = 0; q < ND; q++) v[r][q] = gref(wn, px + 2 * q, py + r0 + r) | gref(wn, px + 2 * q + 1, py + r0 + r) << 16;
#pragma unroll
                for (int r = 0; r < FBR; r++)
#pragma unroll
                    for (int q = 0; q < ND; q++) sad = __builtin_amdgcn_sad_u16(v[r][q], org[(r0 + r) * 8 + q], sad);
            }
        }
        return sad;
    }
    if (gx >= 0 && gx + 4 * W4 + EPZS_EDGE <= EGeo<pel>::ew && gy >= 0 && gy + H <= EGeo<pel>::ew) {   // inside the window
        const int a = gy * EGeo<pel>::ew + gx;
        const uint32_t sel = (uint32_t)(a & 3);
        const uint32_t *base = reinterpret_cast<const uint32_t *>(s.g + (a & ~3));
#pragma unroll
        for (int r = 0; r < H; r++) {
            uint32_t w[W4 + 1];
#pragma unroll
            for (int q = 0; q <= W4; q++) w[q] = base[r * (EGeo<pel>::ew / 4) + q];
#pragma unroll
            for (int q = 0; q < W4; q++) sad = __builtin_amdgcn_sad_u8(__builtin_amdgcn_alignbyte(w[q + 1], w[q], sel), org[r * 4 + q], sad);
        }
    } else {   // outside: the reference picture in global memory, clamped (far predictors), as above
        const int px = wn.wx0 + gx, py = wn.wy0 + gy;
#pragma unroll 1
        for (int r0 = 0; r0 < H; r0 += FBR) {
            uint32_t v[FBR][W4];
#pragma unroll
            for (int r = 0; r < FBR; r++)
#pragma unroll
                for (int q = 0; q < W4; q++) {
                    v[r][q] = 0;
#pragma unroll
                    for (int b = 0; b < 4; b++) v[r][q] |= gref(wn, px + 4 * q + b, py + r0 + r) << (8 * b);
                }
#pragma unroll
            for (int r = 0; r < FBR; r++)
#pragma unroll
                for (int q = 0; q < W4; q++) sad = __builtin_amdgcn_sad_u8(v[r][q], org[(r0 + r) * 4 + q], sad);
        }
    }
    return sad;
}

// ---- RDOptimization 1 with SearchMode 0 (item 65): SetupFastFullPelSearch's SAD table [J], shared
//      by the MB's 41 searches.  One table per tick MB in global memory (ffs_slot_bytes), raster over
//      the (2 SR + 1)^2 full-pel positions around the MB's FFS centre (the 16x16 MVP / 4, clamped),
//      five phases of one 8-byte entry per position: phase 0 the four 8x8 SADs, phase 1 + b8 the
//      four 4x4 SADs of 8x8 block b8, as u16 (an 8x8 SAD <= 64 x 1023 < 2^16) in raster order.  A
//      search sums the one, two or four it needs at read time (two v_perm + two v_sad_u16 against
//      zero): one dwordx2 store per position and phase instead of a store per block type, 169 KB
//      per MB at SR 32 (JM's nine-plus-five tables were 389 KB), and the nine searches of an 8x8
//      block read the same 34 KB.  The raster -> spiral-index map (the searches' tie order) follows
//      the spiral table in ordtab.
// entry of the search of block type bt at 4x4 position (bx4, by4): phase << 4 | selector (0: all
// four halves, 1: low dword, 2: high dword, 3: halves 0 + 2, 4: halves 1 + 3, 5 + k: half k)
__device__ __forceinline__ int ffs_tab_index(int bt, int bx4, int by4) {
    const int b8 = (by4 >> 1) * 2 + (bx4 >> 1);
    switch (bt) {
    case 1: return 0;
    case 2: return 1 + (by4 >> 1);
    case 3: return 3 + (bx4 >> 1);
    case 4: return (1 + b8) << 4;
    case 5: return (1 + b8) << 4 | (1 + (by4 & 1));
    case 6: return (1 + b8) << 4 | (3 + (bx4 & 1));
    default: return (1 + b8) << 4 | (5 + (by4 & 1) * 2 + (bx4 & 1));
    }
}
// the tables of one MB on its wave, centre (ccx, ccy), built before its first search: per 8x8 block
// b8 the four 4x4 SADs (phase 1 + b8), and their sum, the 8x8 SAD, into half b8 of phase 0 (the
// four 8x8 SADs: the 16x16 / 16x8 / 8x16 searches need no pass of their own).  Every position lies
// inside the LDS window (shifted to the same MVP, margin >= SR + 3).  Lane = column of positions;
// the window rows slide past the block: each reference row is read once and its SADs against the 8
// block rows go to the 8 positions (rows) in flight, a position completing every row.  A column
// past 64 (SR 32) a lane per position.
template <class pel>
__device__ __forceinline__ void ffs_build_phase(const DevParams &d, const EpzS<pel> &s, const EWin<pel> &wn, uint8_t *tab, int ccx, int ccy, int b8,
                                                int lane) {
    constexpr int EW = EGeo<pel>::ew, PPD = 4 / sizeof(pel);   // samples per dword
    constexpr int H = 8, ND = H / PPD, OD = 16 / PPD;    // block rows (and columns), dwords per block / MB row
    const int R = d.sr, side = 2 * R + 1, np = side * side;
    const int ox = 8 * (b8 & 1), oy = 8 * (b8 >> 1);
    uint2 *tb = reinterpret_cast<uint2 *>(tab) + (size_t)(1 + b8) * np;
    uint16_t *t0 = reinterpret_cast<uint16_t *>(tab) + b8;
    uint32_t o[H][ND];                                   // the block's rows (wave-uniform)
#pragma unroll
    for (int r = 0; r < H; r++)
#pragma unroll
        for (int q = 0; q < ND; q++) o[r][q] = reinterpret_cast<const uint32_t *>(s.org)[(oy + r) * OD + ox / PPD + q];
    // accumulator of block row k, dword q: the 4x4 (raster in the block)
    auto ai = [](int k, int q) { return (k >> 2) * 2 + q / (ND / 2); };
    auto sad = [](uint32_t r, uint32_t o, uint32_t c) {
        if constexpr (sizeof(pel) == 2) return __builtin_amdgcn_sad_u16(r, o, c);
        else return __builtin_amdgcn_sad_u8(r, o, c);
    };
    auto store = [&](int p, const uint32_t (&a)[4]) {
        tb[p] = make_uint2(a[0] | a[1] << 16, a[2] | a[3] << 16);
        t0[4 * p] = (uint16_t)(a[0] + a[1] + a[2] + a[3]);
    };
    const int wy0 = wn.my + ccy - R + oy, wx0 = wn.mx + ccx - R + ox;   // window position of position (0, 0)
    const int nc = min(side, NTE), c = min(lane, nc - 1), nrow = side + H - 1;
    {
        const int a0 = wy0 * EW + wx0 + c;
        const uint32_t sel = (uint32_t)(a0 & (PPD - 1)) * sizeof(pel);
        const uint32_t *base = reinterpret_cast<const uint32_t *>(s.g + (a0 & ~(PPD - 1)));
        uint32_t acc[H][4];
#pragma unroll 1
        for (int Y0 = 0; Y0 < nrow; Y0 += H) {
#pragma unroll
            for (int j = 0; j < H; j++) {
                const int Y = Y0 + j;                    // the window row read (position rows Y - H + 1 .. Y)
                if (Y >= nrow) break;                    // wave-uniform
#pragma unroll
                for (int i = 0; i < 4; i++) acc[j][i] = 0;   // position row Y starts
                uint32_t w[ND + 1], rf[ND];
#pragma unroll
                for (int q = 0; q <= ND; q++) w[q] = base[Y * (EW / PPD) + q];
#pragma unroll
                for (int q = 0; q < ND; q++) rf[q] = __builtin_amdgcn_alignbyte(w[q + 1], w[q], sel);
#pragma unroll
                for (int k = 0; k < H; k++)             // block row k <-> position row Y - k
#pragma unroll
                    for (int q = 0; q < ND; q++) acc[(j - k) & (H - 1)][ai(k, q)] = sad(rf[q], o[k][q], acc[(j - k) & (H - 1)][ai(k, q)]);
                const int y = Y - (H - 1);               // complete
                if (y >= 0 && y < side && lane < nc) store(y * side + c, acc[(j + 1) & (H - 1)]);
            }
        }
    }
#pragma unroll 1
    for (int cc = NTE; cc < side; cc++)                  // SR 32: column 64, a lane per row
        for (int y0 = 0; y0 < side; y0 += NTE) {
            const int y = min(y0 + lane, side - 1), a = (wy0 + y) * EW + wx0 + cc;
            const uint32_t sel = (uint32_t)(a & (PPD - 1)) * sizeof(pel);
            const uint32_t *base = reinterpret_cast<const uint32_t *>(s.g + (a & ~(PPD - 1)));
            uint32_t a4[4] = {0, 0, 0, 0};
#pragma unroll
            for (int k = 0; k < H; k++) {
                uint32_t w[ND + 1];
#pragma unroll
                for (int q = 0; q <= ND; q++) w[q] = base[k * (EW / PPD) + q];
#pragma unroll
                for (int q = 0; q < ND; q++) a4[ai(k, q)] = sad(__builtin_amdgcn_alignbyte(w[q + 1], w[q], sel), o[k][q], a4[ai(k, q)]);
            }
            if (y0 + lane < side) store(y * side + cc, a4);
        }
}
template <class pel>
__device__ __forceinline__ void ffs_table_build(const DevParams &d, const EpzS<pel> &s, const EWin<pel> &wn, uint8_t *tab, int ccx, int ccy, int lane) {
#pragma unroll 1
    for (int b8 = 0; b8 < 4; b8++) ffs_build_phase<pel>(d, s, wn, tab, ccx, ccy, b8, lane);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
}
// the full-pel search of one block from the table: every position of +-range around the centre,
// key = cost << 13 | spiral index (JM's scan order, strict '<'; the raster -> spiral map in ordtab),
// one wave minimum.  Lanes take the columns of a row (the row's MV-cost bits uniform; lanes past the
// last column repeat it), FFS_RB rows' loads in flight per round trip, and with them the column past
// 64 (SR 32) of those rows on lanes 0 .. FFS_RB - 1.  The entry's halves summed per selector class
// M (uniform): 0 all four (uint2, two v_sad_u16), 1 one dword's pair (u32, one v_sad_u16), 2 halves
// 0 + 2 or 1 + 3 (uint2, v_perm + v_sad_u16), 3 one half (u32, one shift or mask).
#ifndef FFS_RB
#define FFS_RB 22                                     // rows per round trip, 8-byte entries (M 0, 2)
#endif
#ifndef FFS_RB4
#define FFS_RB4 22                                    // ... 4-byte reads (M 1, 3)
#endif
template <int M>
__device__ __forceinline__ unsigned ffs_min_m(const DevParams &d, const uint8_t *tab_, int ph, int sel, int range, int ccx, int ccy, int pmx, int pmy, int lane) {
    const int R = d.sr, side = 2 * R + 1, np = side * side, n = 2 * range + 1, c0 = R - range;
    typedef typename std::conditional<M == 0 || M == 2, uint2, uint32_t>::type E;
    // the dword (M 1, 3) or the whole entry (M 0, 2)
    const E *tab = reinterpret_cast<const E *>(reinterpret_cast<const uint2 *>(tab_) + (size_t)ph * np) + ((M == 1 || M == 3) ? (sel >> 1) : 0);
    constexpr int ES = (M == 1 || M == 3) ? 2 : 1;       // entry stride in E
    const uint32_t pm = (sel & 1) ? 0x07060302u : 0x05040100u;   // M 2: halves 1 + 3 / 0 + 2
    const int sh = 16 * (sel & 1);                       // M 3: the half in its dword
    // the SAD plus t (the MV cost), v_sad_u16 against zero accumulating it
    auto val = [&](E v, unsigned t) -> unsigned {
        if constexpr (M == 0) return __builtin_amdgcn_sad_u16(v.y, 0u, __builtin_amdgcn_sad_u16(v.x, 0u, t));
        else if constexpr (M == 1) return __builtin_amdgcn_sad_u16(v, 0u, t);
        else if constexpr (M == 2) return __builtin_amdgcn_sad_u16(__builtin_amdgcn_perm(v.y, v.x, pm), 0u, t);
        else return ((v >> sh) & 0xFFFFu) + t;
    };
    const uint32_t *spr = d.ordtab + ORDTAB_SPOS + np;
    constexpr int RB = (M == 0 || M == 2) ? FFS_RB : FFS_RB4;
    unsigned kb = 0xFFFFFFFFu;
    const int lc = min(lane, n - 1);
    // WEIGHTED_COST under RDO, (lf x (bits_x + bits_y)) >> 16, as lf bits_x + lf bits_y (the row's
    // term uniform): no per-position multiply (products < 2^32 as in wcost)
    const unsigned lf = d.lf, lfx = lf * (unsigned)mvbits(4 * (ccx + lc - range) - pmx);
    const bool xc = n > NTE;                             // the column past 64 (wave-uniform)
    const unsigned lfc = lf * (unsigned)mvbits(4 * (ccx + NTE - range) - pmx);
#pragma unroll 1
    for (int r0 = 0; r0 < n; r0 += RB) {
        E sv[RB], xv{};
        uint32_t pv[RB], xp = 0;
        const int xr = min(r0 + lane, n - 1);
#pragma unroll
        for (int j = 0; j < RB; j++) {
            const int p = (min(r0 + j, n - 1) + c0) * side + c0 + lc;
            sv[j] = tab[(size_t)ES * p];
            pv[j] = spr[p];
        }
        if (xc) {
            const int p = (xr + c0) * side + c0 + NTE;
            xv = tab[(size_t)ES * p];
            xp = spr[p];
        }
#pragma unroll
        for (int j = 0; j < RB; j++) {
            const unsigned lfy = lf * (unsigned)mvbits(4 * (ccy + min(r0 + j, n - 1) - range) - pmy);   // uniform
            kb = min(kb, (val(sv[j], (lfx + lfy) >> 16) << 13) | pv[j]);
        }
        if (xc && lane < RB) {
            const unsigned lfr = lf * (unsigned)mvbits(4 * (ccy + xr - range) - pmy);
            kb = min(kb, (val(xv, (lfc + lfr) >> 16) << 13) | xp);
        }
    }
    return wave_min_u32(kb);
}
__device__ __forceinline__ unsigned ffs_table_min(const DevParams &d, const uint8_t *tab, int ti, int range, int ccx, int ccy, int pmx, int pmy, int lane) {
    const int ph = ti >> 4, sel = ti & 15;
    if (sel == 0) return ffs_min_m<0>(d, tab, ph, 0, range, ccx, ccy, pmx, pmy, lane);
    if (sel <= 2) return ffs_min_m<1>(d, tab, ph, 2 * (sel - 1), range, ccx, ccy, pmx, pmy, lane);
    if (sel <= 4) return ffs_min_m<2>(d, tab, ph, sel - 3, range, ccx, ccy, pmx, pmy, lane);
    return ffs_min_m<3>(d, tab, ph, sel - 5, range, ccx, ccy, pmx, pmy, lane);
}

// the full-pel argmins of NS searches over one table phase in one pass: searches whose MVPs need no
// other search of the group (SET 0: 16x16, 16x8 top, 8x16 left on phase 0; 8x8, 8x4 top, 4x8 left,
// 4x4 #0 on phase 1 + b8; SET 1, once those are done: 16x8 bottom, 8x16 right; 8x4 bottom, 4x8
// right, 4x4 #1), equal ranges (RestrictSearchRange != 0).  Search k of SET 0 sums all four halves,
// the low dword's pair, halves 0 + 2, half 0; of SET 1 the high dword's pair, halves 1 + 3, half 1.
// Keys as ffs_table_min (the argmin is bound by its round trips: one pass serves NS searches)
#ifndef FFS_GRB
#define FFS_GRB 13                                   // rows per round trip of a grouped pass (5 at SR 32: fewer
#endif                                               //   live registers beat fewer trips, profiles/r11a)
template <int NS, int SET = 0>
__device__ __forceinline__ void ffs_group_min(const DevParams &d, const uint8_t *tab_, int ph, int range, int ccx, int ccy, const int (&pmx)[4],
                                              const int (&pmy)[4], int lane, unsigned (&kb)[4]) {
    const int R = d.sr, side = 2 * R + 1, np = side * side, n = 2 * range + 1, c0 = R - range;
    const uint2 *tab = reinterpret_cast<const uint2 *>(tab_) + (size_t)ph * np;
    const uint32_t *spr = d.ordtab + ORDTAB_SPOS + np;
    constexpr int RB = FFS_GRB;
    const int lc = min(lane, n - 1);
    const unsigned lf = d.lf;
    const bool xc = n > NTE;
    unsigned lfx[NS], lfc[NS];
#pragma unroll
    for (int k = 0; k < NS; k++) {
        kb[k] = 0xFFFFFFFFu;
        lfx[k] = lf * (unsigned)mvbits(4 * (ccx + lc - range) - pmx[k]);
        lfc[k] = lf * (unsigned)mvbits(4 * (ccx + NTE - range) - pmx[k]);
    }
    auto val = [](int k, uint2 v, unsigned t) -> unsigned {
        if (SET == 1) {
            if (k == 0) return __builtin_amdgcn_sad_u16(v.y, 0u, t);
            if (k == 1) return __builtin_amdgcn_sad_u16(__builtin_amdgcn_perm(v.y, v.x, 0x07060302u), 0u, t);
            return (v.x >> 16) + t;
        }
        if (k == 0) return __builtin_amdgcn_sad_u16(v.y, 0u, __builtin_amdgcn_sad_u16(v.x, 0u, t));
        if (k == 1) return __builtin_amdgcn_sad_u16(v.x, 0u, t);
        if (k == 2) return __builtin_amdgcn_sad_u16(__builtin_amdgcn_perm(v.y, v.x, 0x05040100u), 0u, t);
        return (v.x & 0xFFFFu) + t;
    };
#pragma unroll 1
    for (int r0 = 0; r0 < n; r0 += RB) {
        uint2 sv[RB], xv = make_uint2(0, 0);
        uint32_t pv[RB], xp = 0;
        const int xr = min(r0 + lane, n - 1);
#pragma unroll
        for (int j = 0; j < RB; j++) {
            const int p = (min(r0 + j, n - 1) + c0) * side + c0 + lc;
            sv[j] = tab[p];
            pv[j] = spr[p];
        }
        if (xc) {
            const int p = (xr + c0) * side + c0 + NTE;
            xv = tab[p];
            xp = spr[p];
        }
#pragma unroll
        for (int j = 0; j < RB; j++) {
            const int y = ccy + min(r0 + j, n - 1) - range;
#pragma unroll
            for (int k = 0; k < NS; k++) {
                const unsigned lfy = lf * (unsigned)mvbits(4 * y - pmy[k]);   // uniform
                kb[k] = min(kb[k], (val(k, sv[j], (lfx[k] + lfy) >> 16) << 13) | pv[j]);
            }
        }
        if (xc && lane < RB) {
#pragma unroll
            for (int k = 0; k < NS; k++) {
                const unsigned lfr = lf * (unsigned)mvbits(4 * (ccy + xr - range) - pmy[k]);
                kb[k] = min(kb[k], (val(k, xv, (lfc[k] + lfr) >> 16) << 13) | xp);
            }
        }
    }
#pragma unroll
    for (int k = 0; k < NS; k++) kb[k] = wave_min_u32(kb[k]);
}

typedef short e16x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ e16x2 e_s2(uint32_t v) { return __builtin_bit_cast(e16x2, v); }
__device__ __forceinline__ uint32_t e_u32(e16x2 v) { return __builtin_bit_cast(uint32_t, v); }
__device__ __forceinline__ e16x2 e_abs2(e16x2 v) { return __builtin_elementwise_max(v, (e16x2)(0) - v); }
__device__ __forceinline__ int had_packed(const e16x2 (&r)[4][2]);

// row pointer and stride of half-grid plane pl (0 G = the window, 1 b, 2 h, 3 j) at block-
// relative integer position (rx, ry) (b / h / j sample [y][x] = position (x - 1, y - 1))
template <class pel>
__device__ __forceinline__ const pel *hp_row(const EpzS<pel> &s, int pl, const pel *gb, int gs, int rx, int ry, int &stride) {
    if (pl == 0) { stride = gs; return gb + ry * gs + rx; }
    stride = HPS;
    return s.hp[pl - 1] + (ry + 1) * HPS + rx + 1;
}

// SATD() [J] of one 4x4 sub-block at quarter-pel offset (ox, oy) in [-3, 3] from the full-pel
// MV (window position gx0, gy0 of the block origin): block-relative sub-block origin (sx, sy);
// rows as dwords from the phase's two half-grid planes, their rounding average per byte, packed
// int16 Hadamard (as subblock_satd)
template <class pel>
__device__ __forceinline__ int hp_satd(const EpzS<pel> &s, const pel *gb, int gs, int sx, int sy, int obase, int ox, int oy, int had) {
    const int off = qoff((oy & 3) * 4 + (ox & 3));
    const int xa = (off >> 12) & 15, ya = (off >> 8) & 15, xb = (off >> 4) & 15, yb = off & 15;
    const int rx = sx + (ox >> 2), ry = sy + (oy >> 2);
    int sa, sb;
    const pel *pA = hp_row(s, (xa & 1) + 2 * (ya & 1), gb, gs, rx + (xa >> 1), ry + (ya >> 1), sa);
    const pel *pB = hp_row(s, (xb & 1) + 2 * (yb & 1), gb, gs, rx + (xb >> 1), ry + (yb >> 1), sb);
    if constexpr (sizeof(pel) == 2) {
        // 16-bit samples: a row is two dwords; per sample (a + b + 1) >> 1, then the same packed
        // int16 Hadamard (differences |d| <= 1023: every stage stays within int16)
        uint32_t O[4][2], P[4][2];
#pragma unroll
        for (int yy = 0; yy < 4; yy++)
#pragma unroll
            for (int k = 0; k < 2; k++) {
                const uint32_t A = eld_u32(pA + yy * sa + 2 * k), B = eld_u32(pB + yy * sb + 2 * k);
                P[yy][k] = (A | B) - (((A ^ B) >> 1) & 0x7FFF7FFFu);
                O[yy][k] = *reinterpret_cast<const uint32_t *>(s.org + obase + 16 * yy + 2 * k);
            }
        if (!had) {
            uint32_t sad = 0;
#pragma unroll
            for (int yy = 0; yy < 4; yy++) {
                sad = __builtin_amdgcn_sad_u16(O[yy][0], P[yy][0], sad);
                sad = __builtin_amdgcn_sad_u16(O[yy][1], P[yy][1], sad);
            }
            return (int)sad;
        }
        e16x2 r[4][2];
#pragma unroll
        for (int yy = 0; yy < 4; yy++) {
            r[yy][0] = e_s2(O[yy][0]) - e_s2(P[yy][0]);
            r[yy][1] = e_s2(O[yy][1]) - e_s2(P[yy][1]);
        }
        return had_packed(r);
    }
    uint32_t O[4], P[4];
#pragma unroll
    for (int yy = 0; yy < 4; yy++) {
        const uint32_t A = eld_u32(pA + yy * sa), B = eld_u32(pB + yy * sb);
        P[yy] = (A | B) - (((A ^ B) >> 1) & 0x7F7F7F7Fu);   // per byte (a + b + 1) >> 1
        O[yy] = *reinterpret_cast<const uint32_t *>(s.org + obase + 16 * yy);
    }
    if (!had) {
        uint32_t sad = 0;
#pragma unroll
        for (int yy = 0; yy < 4; yy++) sad = __builtin_amdgcn_sad_u8(O[yy], P[yy], sad);
        return (int)sad;
    }
    e16x2 r[4][2];
#pragma unroll
    for (int yy = 0; yy < 4; yy++) {
        r[yy][0] = e_s2(__builtin_amdgcn_perm(0u, O[yy], 0x0c010c00u)) - e_s2(__builtin_amdgcn_perm(0u, P[yy], 0x0c010c00u));
        r[yy][1] = e_s2(__builtin_amdgcn_perm(0u, O[yy], 0x0c030c02u)) - e_s2(__builtin_amdgcn_perm(0u, P[yy], 0x0c030c02u));
    }
    return had_packed(r);
}

// SATD() of a 4x4 difference block held as packed int16 pairs r[row][0] = (d0, d1), r[row][1] =
// (d2, d3): vertical then horizontal butterflies, sum |.| via |a + b| + |a - b| = 2 max(|a|, |b|)
// (the >> 1 of SATD folded in)
__device__ __forceinline__ int had_packed(const e16x2 (&r)[4][2]) {
    e16x2 m[4][2];
#pragma unroll
    for (int h = 0; h < 2; h++) {
        const e16x2 a0 = r[0][h] + r[3][h], a1 = r[1][h] + r[2][h], a2 = r[1][h] - r[2][h], a3 = r[0][h] - r[3][h];
        m[0][h] = a0 + a1; m[2][h] = a0 - a1; m[1][h] = a2 + a3; m[3][h] = a3 - a2;
    }
    e16x2 acc = (e16x2)(0);
#pragma unroll
    for (int p = 0; p < 2; p++) {
        const uint32_t u0 = e_u32(m[2 * p][0]), v0 = e_u32(m[2 * p + 1][0]);
        const uint32_t u1 = e_u32(m[2 * p][1]), v1 = e_u32(m[2 * p + 1][1]);
        const e16x2 x0 = e_s2(__builtin_amdgcn_perm(v0, u0, 0x05040100u)), x1 = e_s2(__builtin_amdgcn_perm(v0, u0, 0x07060302u));
        const e16x2 x2 = e_s2(__builtin_amdgcn_perm(v1, u1, 0x05040100u)), x3 = e_s2(__builtin_amdgcn_perm(v1, u1, 0x07060302u));
        const e16x2 a0 = x0 + x3, a1 = x1 + x2, a2 = x1 - x2, a3 = x0 - x3;
        acc += __builtin_elementwise_max(e_abs2(a0), e_abs2(a1)) + __builtin_elementwise_max(e_abs2(a2), e_abs2(a3));
    }
    const uint32_t t = e_u32(acc);
    return (int)((t & 0xFFFFu) + (t >> 16));
}

// BlockMotionSearch [J] of one block on the wave: EPZS full pel + SubPelBlockMotionSearch;
// pmvo (k_rdo_inter; null in k_mb_epzs): receives the MVP each search used (the RD rate's mvd)
template <int BT, class pel, int FBR = 1>
__device__ __forceinline__ void epzs_block(const DevParams &d, EpzS<pel> &s, const EWin<pel> &wn, int bx4, int by4, int mc, int b8, int best8x8, bool prof,
                                           int16_t (*pmvo)[16][2] = nullptr, const uint8_t *ftab = nullptr, unsigned fkb = 0xFFFFFFFFu) {
    // debug (JMH_PHASE_PROF): steps of the MB's first 4x4 search into prof[41..46], of its 16x16
    // search into prof[47..52] (k_mb_epzs only)
    const bool sp = prof && ((BT == 7 && bx4 == 0 && by4 == 0) || BT == 1);
#define SSTAMP(k) do { if (sp) d.prof[(BT == 1 ? 47 : 41) + (k)] = wall_clock64(); } while (0)
    SSTAMP(0);
    constexpr int LW4 = BT <= 2 ? 2 : (BT <= 5 ? 1 : 0), LH4 = (BT == 1 || BT == 3) ? 2 : (BT == 2 || BT == 4 || BT == 6) ? 1 : 0;
    constexpr int W4 = 1 << LW4, H4 = 1 << LH4, LNS = LW4 + LH4, NSUB = 1 << LNS;
    const int lane = threadIdx.x;
    const int had = d.use_hadamard;
    const bool slice_p = d.slice_type == JMH_P_SLICE;
    const int range = d.restrict_sr == 0 ? d.sr / min(2, BT) : d.sr;
    int pmx, pmy;
    MvpNb nb;
    set_mvp_nb(NbEpz<EpzS<pel>>{s, BT, b8, best8x8}, bx4, by4, 4 * W4, 4 * H4, pmx, pmy, nb);
    pmx = __builtin_amdgcn_readfirstlane(pmx);
    pmy = __builtin_amdgcn_readfirstlane(pmy);
    const int mvx0 = iclip(-range, range, pmx / 4), mvy0 = iclip(-range, range, pmy / 4);
    const int med = 16 * W4 * H4 * ((d.maxv + 1) >> 8);   // medthres x pel_error_me (High 10)
    // the stop criterion after the predictors (wave-uniform): medthres, or EPZSDetermineStopCriterion
    // (item 61) from the same block type's full-pel costs at A, B and C (no D substitution)
    int stop = med;
    if (d.epzs_maxts) {
        const int pe = (d.maxv + 1) >> 8, npx = 16 * W4 * H4, mb_x = 4 * bx4, mb_y = 4 * by4, bsx = 4 * W4;
        auto fpn = [&](int xN, int yN, int &v) -> bool {
            if (yN > 15 || (xN > 15 && yN >= 0)) return false;
            if (xN >= 0 && yN >= 0) { v = s.fpc[BT - 1][(yN >> 2) * 4 + (xN >> 2)]; return true; }
            const int c = border_cell(xN, yN);
            if (c < 0 || s.bd.ref[c] == -2) return false;
            v = s.fpb[BT - 1][c];
            return true;
        };
        int sad = 0x7FFFFFFF, v = 0;
        if (fpn(mb_x - 1, mb_y, v)) sad = min(sad, v);
        if (fpn(mb_x, mb_y - 1, v)) sad = min(sad, v);
        bool cok = true;                                   // C inside the MB but later in decoding order
        if (mb_y > 0) {
            if (mb_x < 8) {
                if (mb_y == 8) { if (bsx == 16) cok = false; }
                else if (mb_x + bsx == 8) cok = false;
            } else if (mb_x + bsx == 16) cok = false;
        }
        if (cok && fpn(mb_x + bsx, mb_y - 1, v)) sad = min(sad, v);
        sad = min(max(sad, d.epzs_mints * npx * pe), d.epzs_maxts * npx * pe);
        stop = __builtin_amdgcn_readfirstlane((9 * max(med, sad) + 2 * med) >> 3);
    }
    SSTAMP(1);
    int bx = mvx0, by = mvy0, min_mcost;
    if (d.search_mode != 3) {
        // RDOptimization 1 with SearchMode 0 / -1 (k_rdo_inter, item 65): FastFullPelBlockMotionSearch
        // on the MB's window centred on the 16x16 MVP / 4 (clamped), or FullPelBlockMotionSearch on
        // the block's own centre; every position of +-range on a lane stride (SAD from the LDS window
        // or, outside it, from the reference picture), key = cost << 13 | spiral index (cost < 2^19:
        // 16x16 SAD < 2^18, no negative bias under RDO), one wave minimum; no (0,0) pre-check and no
        // zero-vector bias (!input->rdopt [J])
        if (BT == 1 && d.search_mode == 0) {
            if (lane == 0) { s.scx = iclip(-d.sr, d.sr, pmx / 4); s.scy = iclip(-d.sr, d.sr, pmy / 4); }
            wave_lds_sync();
        }
        const int ccx = d.search_mode == 0 ? s.scx : mvx0, ccy = d.search_mode == 0 ? s.scy : mvy0;
        const int side = 2 * range + 1, npos = side * side;
        unsigned kb = 0xFFFFFFFFu;
        if (ftab && d.search_mode == 0) {               // the MB's shared SAD table (ffs_table_build)
            // fkb: this search's key from a grouped pass (ffs_group_min), else its own argmin
            kb = fkb != 0xFFFFFFFFu ? fkb : ffs_table_min(d, ftab, ffs_tab_index(BT, bx4, by4), range, ccx, ccy, pmx, pmy, lane);
        } else {
#pragma unroll 1
        for (int p = lane; p < npos; p += NTE) {
            const int dy = p / side - range, dx = p - (dy + range) * side - range, x = ccx + dx, y = ccy + dy;
            const int c = (int)lane_block_sad<LW4, LH4, pel, FBR>(s, wn, bx4, by4, x, y) + wcost(d, mvbits(4 * x - pmx) + mvbits(4 * y - pmy));
            kb = min(kb, ((unsigned)c << 13) | (unsigned)spiral_index(dx, dy));
        }
        kb = wave_min_u32(kb);
        }
        int rx, ry;
        spiral_pos((int)(kb & 8191u), rx, ry);
        bx = ccx + rx; by = ccy + ry;
        min_mcost = (int)(kb >> 13);
    } else {
    // ---- full pel: predictor `lane`, then pattern rounds
    int cx, cy;
    const bool cv = epzs_cand(d, s, lane, BT, bx4, by4, nb, range, mvx0, mvy0, cx, cy);
    if (!cv) { cx = mvx0; cy = mvy0; }   // any valid position for the SAD (key discarded)
    const int c0 = (int)lane_block_sad<LW4, LH4, pel, FBR>(s, wn, bx4, by4, cx, cy) +
                   wcost(d, mvbits(4 * cx - pmx) + mvbits(4 * cy - pmy));
    const int cost0 = __builtin_amdgcn_readfirstlane(c0);   // predictor 0: the centre, always valid
    SSTAMP(2);
    min_mcost = cost0;
    if (cost0 >= med) {                                    // else: stop at the centre
        const unsigned m0 = wave_min_u32(cv ? ((unsigned)c0 << 6) | (unsigned)lane : 0xFFFFFFFFu);
        min_mcost = (int)(m0 >> 6);
        bx = __builtin_amdgcn_readlane(cx, m0 & 63);
        by = __builtin_amdgcn_readlane(cy, m0 & 63);
        if (min_mcost >= stop) {                           // pattern refinement until it stops
            // Rounds are resolved in batches: the cost of every position within |dx| + |dy| <= 4
            // of the batch centre (one per lane, 41 lanes), then up to 2 extended-diamond rounds
            // (each moves <= 2) or 4 small-diamond rounds (<= 1) on those costs, exactly as JM
            // scans them (pattern order, strict '<', window check); then a new batch.
            const bool sd = min_mcost < stop + ((3 * stop) >> 1);
            const int steps = sd ? 4 : 2;
            const int dia = lane < 41 ? dia41(lane) : 0x44;
            const int ddx = (dia & 15) - 4, ddy = (dia >> 4) - 4;
            auto refine = [&](int &rbx, int &rby, int &rcost) {
                for (bool done = false; !done;) {
                    const int x = rbx + ddx, y = rby + ddy;
                    const bool inw = lane < 41 && abs(x - mvx0) <= range && abs(y - mvy0) <= range;
                    int c = 0;
                    if (inw) c = (int)lane_block_sad<LW4, LH4, pel, FBR>(s, wn, bx4, by4, x, y) + wcost(d, mvbits(4 * x - pmx) + mvbits(4 * y - pmy));
                    for (int k = 0; k < steps; k++) {
                        const int rx = x - rbx, ry = y - rby;   // this lane's position relative to the current best
                        int e = 15;
                        if (sd) { if (abs(rx) <= 1 && abs(ry) <= 1) e = (int)((0xf3f2f1f0full >> (4 * ((ry + 1) * 3 + rx + 1))) & 15); }
                        else if (abs(rx) <= 2 && abs(ry) <= 2) {
                            const int i = (ry + 2) * 5 + rx + 2;
                            e = (int)((i < 16 ? 0xf4af93f281fff0ffull >> (4 * i) : 0xff7fff6b5ull >> (4 * (i - 16))) & 15);
                        }
                        const unsigned m = wave_min_u32(inw && e != 15 ? ((unsigned)c << 6) | (unsigned)e : 0xFFFFFFFFu);
                        if (m == 0xFFFFFFFFu || (int)(m >> 6) >= rcost) { done = true; break; }
                        rcost = (int)(m >> 6);
                        int px, py;
                        epzs_pat(sd, (int)(m & 63), px, py);
                        rbx += px; rby += py;
                    }
                }
            };
            const int pbx = bx, pby = by;                  // the best predictor
            refine(bx, by, min_mcost);
            if (d.epzs_dual) {
                // EPZSDualRefinement (item 46): the runner-up predictor -- the cheapest other lane,
                // lowest index on ties -- refined the same way; it wins only if strictly cheaper
                const unsigned m1 = wave_min_u32(cv && (unsigned)lane != (m0 & 63) ? ((unsigned)c0 << 6) | (unsigned)lane : 0xFFFFFFFFu);
                if (m1 != 0xFFFFFFFFu) {
                    int x2 = __builtin_amdgcn_readlane(cx, m1 & 63), y2 = __builtin_amdgcn_readlane(cy, m1 & 63), c2 = (int)(m1 >> 6);
                    if (x2 != pbx || y2 != pby) {
                        refine(x2, y2, c2);
                        if (c2 < min_mcost) { min_mcost = c2; bx = x2; by = y2; }
                    }
                }
            }
        }
    }
    }
    const int fmx = bx, fmy = by;
    if (lane < NSUB) {                                     // item 61: this search's full-pel cost
        const int k = (by4 + (lane >> LW4)) * 4 + bx4 + (lane & (W4 - 1));
        s.fpc[BT - 1][k] = (uint16_t)min(min_mcost, 65535);
    }
    if (had) min_mcost = BIGCOST;
    SSTAMP(3);
    // ---- sub-pel neighbourhood of the block at (fmx, fmy): b, h, j planes, sample [y][x] =
    //      block-relative (x - 1, y - 1); b1 = unclipped horizontal taps, row rr <-> y = rr - 2
    constexpr int PW = 4 * W4 + 2, PH = 4 * H4 + 2;
    const int gx0 = wn.mx + 4 * bx4 + fmx, gy0 = wn.my + 4 * by4 + fmy;   // window position of (0, 0)
    // integer samples around the block at its full-pel MV: the window, or when the reach
    // [-GNX, PW + GNX) x [-GNY, PH + GNY) leaves it, the neighbourhood plane read from global
    const pel *gb;
    int gs;
    if (gx0 - GNX >= 0 && gx0 + PW + GNX <= EGeo<pel>::ew && gy0 - GNY >= 0 && gy0 + PH + GNY <= EGeo<pel>::ew) {   // wave-uniform
        gb = s.g + gy0 * EGeo<pel>::ew + gx0; gs = EGeo<pel>::ew;
    } else {
        constexpr int NGN = (PH + 2 * GNY) * GNS;
#pragma unroll 1
        for (int i0 = 0; i0 < NGN; i0 += FBR * NTE) {   // FBR loads per lane in flight
            pel v[FBR];
#pragma unroll
            for (int k = 0; k < FBR; k++) {
                const int i = min(i0 + k * NTE + lane, NGN - 1), y = i / GNS, x = i - y * GNS;
                v[k] = (pel)gref(wn, wn.wx0 + gx0 + x - GNX, wn.wy0 + gy0 + y - GNY);
            }
#pragma unroll
            for (int k = 0; k < FBR; k++)
                if (i0 + k * NTE + lane < NGN) s.gn[i0 + k * NTE + lane] = v[k];
        }
        wave_lds_sync();
        gb = s.gn + GNY * GNS + GNX; gs = GNS;
    }
    auto G = [&](int x, int y) { return (int)gb[y * gs + x]; };
    for (int i = lane; i < PW * (PH + 5); i += NTE) {
        const int rr = i / PW, x = i - rr * PW, gx = x - 1, gy = rr - 3;
        const int h1 = tap6(G(gx - 2, gy), G(gx - 1, gy), G(gx, gy), G(gx + 1, gy), G(gx + 2, gy), G(gx + 3, gy));
        s.b1[rr][x] = (typename EpzTap<pel>::type)h1;
        if (rr >= 2 && rr < PH + 2) {
            s.hp[0][(rr - 2) * HPS + x] = (pel)clipmx((h1 + 16) >> 5, d.maxv);
            s.hp[1][(rr - 2) * HPS + x] =
                (pel)clipmx((tap6(G(gx, gy - 2), G(gx, gy - 1), G(gx, gy), G(gx, gy + 1), G(gx, gy + 2), G(gx, gy + 3)) + 16) >> 5, d.maxv);
        }
    }
    wave_lds_sync();
    for (int i = lane; i < PW * PH; i += NTE) {
        const int y = i / PW, x = i - y * PW;
        s.hp[2][y * HPS + x] =
            (pel)clipmx((tap6(s.b1[y][x], s.b1[y + 1][x], s.b1[y + 2][x], s.b1[y + 3][x], s.b1[y + 4][x], s.b1[y + 5][x]) + 512) >> 10, d.maxv);
    }
    wave_lds_sync();
    SSTAMP(4);
    // ---- half then quarter pel, JM order, strict '<'
    const bool check0 = BT == 1 && fmx == 0 && fmy == 0 && had && slice_p && !d.rdo;   // !input->rdopt [J]
    int qx = 0, qy = 0;
    if (d.epzs_subpel) {
        // EPZSSubPelBlockMotionSearch (item 62): small-diamond rounds, half pel inside F +- 2, then
        // quarter pel inside the half-pel result +- 1; a round = the 4 points x NSUB sub-blocks
        // (<= 64 lane tasks), one wave minimum of (cost, point) keys = strict '<' in pattern order
        auto round = [&](int cxq, int cyq, int step, int ox, int oy, bool centre) -> unsigned {
            const int m = lane >> LNS, sub = lane & (NSUB - 1);
            int px = cxq, py = cyq;
            if (!centre) {
                px += step * (m == 1 ? -1 : m == 2 ? 1 : 0);
                py += step * (m == 0 ? -1 : m == 3 ? 1 : 0);
            }
            const bool val = m < (centre ? 1 : 4) && abs(px - ox) <= step && abs(py - oy) <= step;
            int sat = 0;
            if (val) {
                const int sx = 4 * (sub & (W4 - 1)), sy = 4 * (sub >> LW4);
                sat = hp_satd(s, gb, gs, sx, sy, 64 * by4 + 4 * bx4 + 16 * sy + sx, px, py, had);
            }
            if constexpr (NSUB >= 2) sat += dpp<0xB1>(sat);
            if constexpr (NSUB >= 4) sat += dpp<0x4E>(sat);
            if constexpr (NSUB >= 8) sat += dpp<0x141>(sat);
            if constexpr (NSUB >= 16) sat += dpp<0x140>(sat);
            unsigned key = 0xFFFFFFFFu;
            if (val && sub == 0)
                key = ((unsigned)(sat + wcost(d, mvbits(4 * fmx + px - pmx) + mvbits(4 * fmy + py - pmy)) + EKOFF) << 4) | (unsigned)m;
            return wave_min_u32(key);
        };
        if (had) {                                         // the centre again, with SATD
            const unsigned k = round(0, 0, 0, 0, 0, true);
            if ((int)(k >> 4) - EKOFF < min_mcost) min_mcost = (int)(k >> 4) - EKOFF;
        }
        const int subthres = d.epzs_spts * 16 * NSUB * ((d.maxv + 1) >> 8);
        for (int stage = 0; stage < 2; stage++) {
            const int step = stage ? 1 : 2, ox = qx, oy = qy;
            if (stage && min_mcost < subthres) break;
            for (;;) {
                const unsigned k = round(qx, qy, step, ox, oy, false);
                if (k == 0xFFFFFFFFu || (int)(k >> 4) - EKOFF >= min_mcost) break;
                min_mcost = (int)(k >> 4) - EKOFF;
                const int m = k & 15;
                qx += step * (m == 1 ? -1 : m == 2 ? 1 : 0);
                qy += step * (m == 0 ? -1 : m == 3 ? 1 : 0);
            }
        }
    } else if constexpr (NSUB <= 2) {
        // blocks of one or two 4x4: the SATD of every position of the 7x7 quarter-pel grid around
        // the full-pel MV in one batch (lane task = (position, 4x4 sub-block)), then the half-pel
        // pass over the 9 even positions and the quarter-pel pass around its winner on the costs
        constexpr int NIT = (49 * NSUB + NTE - 1) / NTE;
        int cst[NIT];
#pragma unroll
        for (int it = 0; it < NIT; it++) {
            const int task = it * NTE + lane, p = task >> LNS, sub = task & (NSUB - 1);
            const int ox = p % 7 - 3, oy = p / 7 - 3;
            int sat = 0;
            if (p < 49) {
                const int sx = 4 * (sub & (W4 - 1)), sy = 4 * (sub >> LW4);
                sat = hp_satd(s, gb, gs, sx, sy, 64 * by4 + 4 * bx4 + 16 * sy + sx, ox, oy, had);
            }
            if constexpr (NSUB >= 2) sat += dpp<0xB1>(sat);
            if constexpr (NSUB >= 4) sat += dpp<0x4E>(sat);
            cst[it] = sat + wcost(d, mvbits(4 * fmx + ox - pmx) + mvbits(4 * fmy + oy - pmy));
        }
        // candidate index of offset (dx, dy) in {-1,0,1}^2 (spiral entries 0..8)
        auto c9 = [](int dx, int dy) { return (int)((0x827605413ull >> (4 * ((dy + 1) * 3 + dx + 1))) & 15); };
        const int min_pos = had ? 0 : 1;
        unsigned kb = 0xFFFFFFFFu;
#pragma unroll
        for (int it = 0; it < NIT; it++) {
            const int task = it * NTE + lane, p = task >> LNS, sub = task & (NSUB - 1);
            const int ox = p % 7 - 3, oy = p / 7 - 3;
            if (p < 49 && sub == 0 && !(ox & 1) && !(oy & 1) && abs(ox) <= 2 && abs(oy) <= 2) {
                const int c = c9(ox >> 1, oy >> 1);
                if (c >= min_pos) kb = min(kb, ((unsigned)(cst[it] - ((check0 && c == 0) ? wcost(d, 16) : 0) + EKOFF) << 4) | (unsigned)c);
            }
        }
        kb = wave_min_u32(kb);
        if (kb != 0xFFFFFFFFu && (int)(kb >> 4) - EKOFF < min_mcost) {
            min_mcost = (int)(kb >> 4) - EKOFF;
            qx = 2 * sp9x(kb & 15); qy = 2 * sp9y(kb & 15);
        }
        kb = 0xFFFFFFFFu;
#pragma unroll
        for (int it = 0; it < NIT; it++) {
            const int task = it * NTE + lane, p = task >> LNS, sub = task & (NSUB - 1);
            const int ox = p % 7 - 3, oy = p / 7 - 3;
            if (p < 49 && sub == 0 && abs(ox - qx) <= 1 && abs(oy - qy) <= 1 && (ox != qx || oy != qy))
                kb = min(kb, ((unsigned)(cst[it] + EKOFF) << 4) | (unsigned)c9(ox - qx, oy - qy));
        }
        kb = wave_min_u32(kb);
        if (kb != 0xFFFFFFFFu && (int)(kb >> 4) - EKOFF < min_mcost) {
            min_mcost = (int)(kb >> 4) - EKOFF;
            qx += sp9x(kb & 15); qy += sp9y(kb & 15);
        }
    } else {
        // 8x8 and larger blocks: the half pass, then the quarter pass around its winner; a pass's
        // tasks are (candidate min_pos..8) x NSUB sub-blocks, NSUB consecutive lanes per candidate,
        // so the quarter pass (8 candidates) is one round for 8x8, 16x8 and 8x16, two for 16x16
        // (8x8 in the 7x7 batch above took four)
#pragma unroll
        for (int pass = 0; pass < 2; pass++) {
            const int step = pass == 0 ? 2 : 1, min_pos = pass == 0 ? (had ? 0 : 1) : 1;
            const int ntask = (9 - min_pos) << LNS;
            unsigned kb = 0xFFFFFFFFu;
#pragma unroll
            for (int t0 = 0; t0 < (9 << LNS); t0 += NTE) {
                if (t0 >= ntask) break;                    // wave-uniform
                const int task = t0 + lane, c = min_pos + (task >> LNS), sub = task & (NSUB - 1);
                const bool val = c < 9;
                const int ox = qx + step * sp9x(c), oy = qy + step * sp9y(c);
                int sat = 0;
                if (val) {
                    const int sx = 4 * (sub & (W4 - 1)), sy = 4 * (sub >> LW4);
                    sat = hp_satd(s, gb, gs, sx, sy, 64 * by4 + 4 * bx4 + 16 * sy + sx, ox, oy, had);
                }
                sat += dpp<0xB1>(sat);
                sat += dpp<0x4E>(sat);
                if constexpr (NSUB >= 8) sat += dpp<0x141>(sat);
                if constexpr (NSUB >= 16) sat += dpp<0x140>(sat);
                if (val && sub == 0) {
                    int cost = sat + wcost(d, mvbits(4 * fmx + ox - pmx) + mvbits(4 * fmy + oy - pmy));
                    if (pass == 0 && check0 && c == 0) cost -= wcost(d, 16);
                    kb = min(kb, ((unsigned)(cost + EKOFF) << 4) | (unsigned)c);
                }
            }
            kb = wave_min_u32(kb);
            if (kb != 0xFFFFFFFFu && (int)(kb >> 4) - EKOFF < min_mcost) {
                const int c = kb & 15;
                min_mcost = (int)(kb >> 4) - EKOFF;
                qx += step * sp9x(c);
                qy += step * sp9y(c);
            }
        }
    }
    if (lane < NSUB) {
        const int k = (by4 + (lane >> LW4)) * 4 + bx4 + (lane & (W4 - 1));
        s.all_mv[BT][k][0] = (int16_t)(4 * fmx + qx);
        s.all_mv[BT][k][1] = (int16_t)(4 * fmy + qy);
        if (pmvo) { pmvo[BT][k][0] = (int16_t)pmx; pmvo[BT][k][1] = (int16_t)pmy; }
    }
    if (lane == 0) s.motion_cost[BT][mc] += min_mcost;
    wave_lds_sync();
    SSTAMP(5);
#undef SSTAMP
}


// the LDS window of a macroblock's searches: MB +- off, shifted to the MB's 16x16 MVP / 4 (clamped
// to +-SR; horizontally a multiple of 4) when off < 2 SR + 4 -- the centre most searches search
// around (the border cells in s.bd, synced)
template <class pel>
__device__ __forceinline__ EWin<pel> epzs_place(const DevParams &d, const EpzS<pel> &s, int mbx, int mby) {
    const int sr = d.sr, off = min(2 * sr + 4, EGeo<pel>::off);
    int wcx = 0, wcy = 0;
    if (off < 2 * sr + 4) {
        int pcx, pcy;
        set_mvp(NbBorder{s.bd}, 0, 0, 16, 16, pcx, pcy);
        wcx = __builtin_amdgcn_readfirstlane(iclip(-sr, sr, pcx / 4) & ~3);
        wcy = __builtin_amdgcn_readfirstlane(iclip(-sr, sr, pcy / 4));
    }
    return EWin<pel>{spl<pel>(d.refY), d.W, d.H, 16 * mbx + wcx - off, 16 * mby + wcy - off, off - wcx, off - wcy};
}
// ... its samples, NTH threads (dword per task: two aligned global dwords + v_alignbyte inside the
// picture, clamped samples at its edges: the spec's UMV access)
template <class pel, int NTH>
__device__ __forceinline__ void epzs_load_window(const DevParams &d, EpzS<pel> &s, const EWin<pel> &wn, int lane) {
    const int W = d.W, off = min(2 * d.sr + 4, EGeo<pel>::off), wdim = 16 + 2 * off;
    const pel *refY = wn.ref;
    if constexpr (sizeof(pel) == 2) {
        // 16-bit samples: two per dword; with off % 4 == 0 a dword is aligned in the picture and
        // wholly inside or outside it (as for bytes), else per-sample clamped reads
        constexpr int ND2 = EGeo<pel>::ew / 2, NB = EPZS_NB16;
        const int WX0 = wn.wx0, WY0 = wn.wy0, ntask = wdim * ND2;
        if ((off & 3) == 0) {
            for (int t0 = 0; t0 < ntask; t0 += NB * NTH) {
                uint32_t v[NB];
#pragma unroll
                for (int u = 0; u < NB; u++) {
                    const int task = t0 + u * NTH + lane, y = task / ND2, j = task - y * ND2, x0 = WX0 + 2 * j;
                    const pel *row = refY + iclip(0, d.H - 1, WY0 + y) * W;
                    const int xs = x0 < 0 ? 0 : x0 >= W ? W - 2 : x0;
                    v[u] = task < ntask ? *reinterpret_cast<const uint32_t *>(row + xs) : 0u;
                }
#pragma unroll
                for (int u = 0; u < NB; u++) {
                    const int task = t0 + u * NTH + lane, y = task / ND2, j = task - y * ND2, x0 = WX0 + 2 * j;
                    if (task >= ntask) continue;
                    uint32_t w = v[u];
                    if (x0 < 0) w = (w & 0xFFFFu) * 0x10001u;
                    else if (x0 >= W) w = (w >> 16) * 0x10001u;
                    if (2 * j >= wdim) w = 0;
                    *reinterpret_cast<uint32_t *>(s.g + y * EGeo<pel>::ew + 2 * j) = w;
                }
            }
        } else {
            for (int task = lane; task < ntask; task += NTH) {
                const int y = task / ND2, j = task - y * ND2, x0 = WX0 + 2 * j;
                const pel *row = refY + iclip(0, d.H - 1, WY0 + y) * W;
                uint32_t v = 0;
                for (int q = 0; q < 2; q++)
                    if (2 * j + q < wdim) v |= (uint32_t)row[iclip(0, W - 1, x0 + q)] << (16 * q);
                *reinterpret_cast<uint32_t *>(s.g + y * EGeo<pel>::ew + 2 * j) = v;
            }
        }
    } else {
        // with off % 4 == 0 the window's dwords are aligned in the picture (pix_x % 16 == 0, wcx %
        // 4 == 0) and lie wholly inside or wholly left / right of it (W % 16 == 0): an outside
        // dword is the replicated edge sample.  Two batches of 32 loads per lane in flight.
        constexpr int ND4 = EGeo<pel>::ew / 4, NB = EPZS_NB8;
        const int WX0 = wn.wx0, WY0 = wn.wy0, ntask = wdim * ND4;
        if ((off & 3) == 0) {
            for (int t0 = 0; t0 < ntask; t0 += NB * NTH) {
                uint32_t v[NB];
#pragma unroll
                for (int u = 0; u < NB; u++) {
                    const int task = t0 + u * NTH + lane, y = task / ND4, j = task - y * ND4, x0 = WX0 + 4 * j;
                    const uint8_t *row = refY + iclip(0, d.H - 1, WY0 + y) * W;
                    const int xs = x0 < 0 ? 0 : x0 >= W ? W - 4 : x0;
                    v[u] = task < ntask ? *reinterpret_cast<const uint32_t *>(row + xs) : 0u;
                }
#pragma unroll
                for (int u = 0; u < NB; u++) {
                    const int task = t0 + u * NTH + lane, y = task / ND4, j = task - y * ND4, x0 = WX0 + 4 * j;
                    if (task >= ntask) continue;
                    uint32_t w = v[u];
                    if (x0 < 0) w = (w & 0xFFu) * 0x01010101u;              // left of the picture
                    else if (x0 >= W) w = (w >> 24) * 0x01010101u;          // right of it
                    if (4 * j >= wdim) w = 0;
                    *reinterpret_cast<uint32_t *>(s.g + y * EGeo<pel>::ew + 4 * j) = w;
                }
            }
        } else {   // odd SearchRange: two aligned global dwords + v_alignbyte, clamped bytes at the edges
            for (int task = lane; task < ntask; task += NTH) {
                const int y = task / ND4, j = task - y * ND4, x0 = WX0 + 4 * j;
                const uint8_t *row = refY + iclip(0, d.H - 1, WY0 + y) * W;
                uint32_t v;
                if (4 * j + 3 < wdim && x0 >= 0 && x0 + 3 < W) {
                    const uint32_t *p = reinterpret_cast<const uint32_t *>(row + (x0 & ~3));
                    v = __builtin_amdgcn_alignbyte((x0 & 3) ? p[1] : 0u, p[0], x0 & 3);
                } else {
                    v = 0;
                    for (int q = 0; q < 4; q++)
                        if (4 * j + q < wdim) v |= (uint32_t)row[iclip(0, W - 1, x0 + q)] << (8 * q);
                }
                *reinterpret_cast<uint32_t *>(s.g + y * EGeo<pel>::ew + 4 * j) = v;
            }
        }
    }
}

// the inputs of one macroblock's searches on one wave (lane = 0..63): the MB (one dword per lane),
// border cells, the temporal neighbourhood, the left MB's searches, the window (dword per task: two
// aligned global dwords + v_alignbyte inside the picture, clamped bytes at its edges: the spec's
// UMV access).  Returns the window placement; the caller syncs the wave before reading s.
template <class pel>
__device__ __forceinline__ EWin<pel> epzs_load_mb(const DevParams &d, EpzS<pel> &s, int mbx, int mby, int lane) {
    const int pix_x = 16 * mbx, pix_y = 16 * mby, W = d.W, sr = d.sr;
    const int off = min(2 * sr + 4, EGeo<pel>::off);
    const int X0 = 4 * mbx, Y0 = 4 * mby, left = mb_avail(d, mbx, mby).L ? mby * d.mbw + mbx - 1 : -1;
    const pel *orgY = spl<pel>(d.orgY);
    if constexpr (sizeof(pel) == 1)
        reinterpret_cast<uint32_t *>(s.org)[lane] = *reinterpret_cast<const uint32_t *>(orgY + (pix_y + (lane >> 2)) * W + pix_x + 4 * (lane & 3));
    else
        for (int i = lane; i < 128; i += NTE)
            reinterpret_cast<uint32_t *>(s.org)[i] = *reinterpret_cast<const uint32_t *>(orgY + (pix_y + (i >> 3)) * W + pix_x + 2 * (i & 7));
    if (lane < 10) load_border(d, s.bd, lane, mbx, mby);
    if (lane < 32) s.motion_cost[lane >> 2][lane & 3] = 0;
    if (lane < 36) {
        const int ty = lane / 6, tx = lane - 6 * ty, px = X0 - 1 + tx, py = Y0 - 1 + ty;
        int ref = -1, mx = 0, my = 0;
        if (d.tref && px >= 0 && px < (W >> 2) && py >= 0 && py < (d.H >> 2)) {
            const int a = py * (W >> 2) + px;
            ref = d.tref[a]; mx = d.tmv[2 * a]; my = d.tmv[2 * a + 1];
        }
        s.tref[ty][tx] = (int8_t)ref; s.tmv[ty][tx][0] = (int16_t)mx; s.tmv[ty][tx][1] = (int16_t)my;
    }
    for (int i = lane; i < 7 * 32; i += NTE) {
        const int m = 1 + i / 32, k = (i & 31) >> 1, c = i & 1;
        s.mem[m - 1][k][c] = left >= 0 ? d.scr[left].all_mv[m][k][c] : 0;
    }
    if (lane == 0) s.memok = left >= 0;
    if (d.epzs_maxts && lane < 63) {              // item 61: the neighbours' full-pel costs, cells 1..9
        const int bt = lane / 9, cell = 1 + lane % 9;
        const MbAvail mav = mb_avail(d, mbx, mby);
        const bool av = cell <= 4 ? mav.T : cell == 5 ? mav.TR : mav.L;
        int v = 0;
        if (av) {
            const int a = cell <= 4 ? (mby - 1) * d.mbw + mbx : cell == 5 ? (mby - 1) * d.mbw + mbx + 1 : mby * d.mbw + mbx - 1;
            const int k = cell <= 4 ? 12 + cell - 1 : cell == 5 ? 12 : 4 * (cell - 6) + 3;
            v = d.scr[a].fpc[bt][k];
        }
        s.fpb[bt][cell] = (uint16_t)v;
    }
    if (off < 2 * sr + 4) wave_lds_sync();   // the border cells
    const EWin<pel> wn = epzs_place(d, s, mbx, mby);
    epzs_load_window<pel, NTE>(d, s, wn, lane);
    return wn;
}
