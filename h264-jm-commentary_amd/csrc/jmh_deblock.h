// jmh_deblock.h -- DeblockMb (JM 8.6 loopfilter.c [J], H.264 8.7) fused into the kernels that
// finish a macroblock (k_mb_final, k_rdo_final): this MB's left and top edges, in place on its
// already-filtered left / top neighbours in the deblocked picture (d.dbkY..).  MBs of one tick
// touch disjoint samples and every neighbour they read finished on an earlier tick (left, top and
// top-right precede the MB in both the diagonal wavefront and the RDO stage schedule), so the
// result equals JM's raster-order DeblockFrame.
#pragma once
#include "jmh_common.h"
#include <cstdlib>

// 8.7.2.2 thresholds (index = clip3(0, 51, qp + filter offset)) and tc0 (bS 1..3)
static __constant__ uint8_t c_alpha[52] = {0,  0,  0,  0,  0,  0,  0,  0,  0,  0,  0,  0,  0,   0,   0,   0,   4,   4,
                                           5,  6,  7,  8,  9,  10, 12, 13, 15, 17, 20, 22, 25,  28,  32,  36,  40,  45,
                                           50, 56, 63, 71, 80, 90, 101, 113, 127, 144, 162, 182, 203, 226, 255, 255};
static __constant__ uint8_t c_beta[52] = {0,  0,  0,  0,  0,  0,  0,  0,  0,  0,  0,  0,  0,  0,  0,  0,  2,  2,
                                          2,  3,  3,  3,  3,  4,  4,  4,  6,  6,  7,  7,  8,  8,  9,  9,  10, 10,
                                          11, 11, 12, 12, 13, 13, 14, 14, 15, 15, 16, 16, 17, 17, 18, 18};
static __constant__ uint8_t c_tc0[52][3] = {
    {0, 0, 0}, {0, 0, 0}, {0, 0, 0}, {0, 0, 0}, {0, 0, 0}, {0, 0, 0}, {0, 0, 0}, {0, 0, 0}, {0, 0, 0},
    {0, 0, 0}, {0, 0, 0}, {0, 0, 0}, {0, 0, 0}, {0, 0, 0}, {0, 0, 0}, {0, 0, 0}, {0, 0, 0}, {0, 0, 1},
    {0, 0, 1}, {0, 0, 1}, {0, 0, 1}, {0, 1, 1}, {0, 1, 1}, {1, 1, 1}, {1, 1, 1}, {1, 1, 1}, {1, 1, 1},
    {1, 1, 2}, {1, 1, 2}, {1, 1, 2}, {1, 1, 2}, {1, 2, 3}, {1, 2, 3}, {2, 2, 3}, {2, 2, 4}, {2, 3, 4},
    {2, 3, 4}, {3, 3, 5}, {3, 4, 6}, {3, 4, 6}, {4, 5, 7}, {4, 5, 8}, {4, 6, 9}, {5, 7, 10}, {6, 8, 11},
    {6, 8, 13}, {7, 10, 14}, {8, 11, 16}, {9, 12, 18}, {10, 13, 20}, {11, 15, 23}, {13, 17, 25}};

// one line of samples across an edge (8.7.2.3 / 8.7.2.4): q0 at q[0], p_k at q[-(k+1)*step];
// alpha / beta / tc0 already scaled by 1 << (BitDepth - 8), Clip1 to maxv
template <class pel>
__device__ __forceinline__ void filter_line(pel *q, int step, int bS, int alpha, int beta, int tc0, bool chroma, int maxv) {
    const int p0 = q[-step], p1 = q[-2 * step], q0 = q[0], q1 = q[step];
    if (!(abs(p0 - q0) < alpha && abs(p1 - p0) < beta && abs(q1 - q0) < beta)) return;
    if (chroma) {
        if (bS < 4) {
            const int tc = tc0 + 1;
            const int dl = iclip(-tc, tc, ((q0 - p0) * 4 + (p1 - q1) + 4) >> 3);
            q[-step] = (pel)clipmx(p0 + dl, maxv);
            q[0] = (pel)clipmx(q0 - dl, maxv);
        } else {
            q[-step] = (pel)((2 * p1 + p0 + q1 + 2) >> 2);
            q[0] = (pel)((2 * q1 + q0 + p1 + 2) >> 2);
        }
        return;
    }
    const int p2 = q[-3 * step], q2 = q[2 * step];
    const int ap = abs(p2 - p0), aq = abs(q2 - q0);
    if (bS < 4) {
        const int tc = tc0 + (ap < beta) + (aq < beta);
        const int dl = iclip(-tc, tc, ((q0 - p0) * 4 + (p1 - q1) + 4) >> 3);
        q[-step] = (pel)clipmx(p0 + dl, maxv);
        q[0] = (pel)clipmx(q0 - dl, maxv);
        if (ap < beta) q[-2 * step] = (pel)(p1 + iclip(-tc0, tc0, (p2 + ((p0 + q0 + 1) >> 1) - (p1 << 1)) >> 1));
        if (aq < beta) q[step] = (pel)(q1 + iclip(-tc0, tc0, (q2 + ((p0 + q0 + 1) >> 1) - (q1 << 1)) >> 1));
    } else {
        const int p3 = q[-4 * step], q3 = q[3 * step];
        const bool small = abs(p0 - q0) < ((alpha >> 2) + 2);
        if (ap < beta && small) {
            q[-step] = (pel)((p2 + 2 * p1 + 2 * p0 + 2 * q0 + q1 + 4) >> 3);
            q[-2 * step] = (pel)((p2 + p1 + p0 + q0 + 2) >> 2);
            q[-3 * step] = (pel)((2 * p3 + 3 * p2 + p1 + p0 + q0 + 4) >> 3);
        } else q[-step] = (pel)((2 * p1 + p0 + q1 + 2) >> 2);
        if (aq < beta && small) {
            q[0] = (pel)((p1 + 2 * p0 + 2 * q0 + 2 * q1 + q2 + 4) >> 3);
            q[step] = (pel)((p0 + q0 + q1 + q2 + 2) >> 2);
            q[2 * step] = (pel)((2 * q3 + 3 * q2 + q1 + q0 + p0 + 4) >> 3);
        } else q[0] = (pel)((2 * q1 + q0 + p1 + 2) >> 2);
    }
}



// LDS of the fused deblocking: the MB with 4 rows / columns of its (already filtered) top / left
// neighbours, boundary strengths
template <class pel>
struct DbkS {
    pel dy[20][20];                      // luma, rows / columns -4..15 -> [r + 4][c + 4]
    pel dc2[2][12][12];                  // chroma, rows / columns -4..7
    int8_t bs[2][4][4];                  // boundary strength [dir][edge][segment]
    int16_t nmv[2][4][2];                // deblock_prefetch: the left / top neighbour's MV of each
    int32_t nbits[2];                    //   edge segment's 4x4 block, its cbp_blk bits and intra flag
    int8_t nintra[2];
};

// DeblockMb's inputs from outside the macroblock -- the left and top neighbours' filtered samples
// (4 rows / columns, luma and chroma) and the mb_type / cbp_blk / MVs its boundary strengths read
// -- into LDS, NTH threads.  Final from the moment the MB's dependencies are done: only the MB
// itself, its left / top neighbours and the top-right one (done before it) write those samples, so
// the caller issues these loads early (final_core: with its own inputs) and deblock_mb<PRE> uses them.
template <class pel, int NTH>
__device__ __forceinline__ void deblock_prefetch(const DevParams &d, DbkS<pel> &s, int mbx, int mby, int tid) {
    const pel *dbkY = spl<pel>(d.dbkY), *dbkU = spl<pel>(d.dbkU), *dbkV = spl<pel>(d.dbkV);
    const int pix_x = 16 * mbx, pix_y = 16 * mby, W = d.W, Wc = d.Wc;
    const bool dbL = mbx > 0, dbT = mby > 0;
    for (int i = tid; i < 256 + 16; i += NTH) {
        if (i < 128) {                                   // luma: rows -4..-1 (i < 64), columns -4..-1
            const bool top = i < 64;
            const int a = i & 63, r = top ? (a >> 4) - 4 : a >> 2, c = top ? a & 15 : (a & 3) - 4;
            s.dy[r + 4][c + 4] = (top ? dbT : dbL) ? dbkY[(pix_y + r) * W + pix_x + c] : (pel)0;
        } else if (i < 256) {                            // chroma: per plane rows -4..-1, columns -4..-1
            const int j = i - 128, pl = j >> 6, a = j & 63;
            const bool top = a < 32;
            const int b = a & 31, r = top ? (b >> 3) - 4 : b >> 2, c = top ? b & 7 : (b & 3) - 4;
            s.dc2[pl][r + 4][c + 4] = (top ? dbT : dbL) ? (pl ? dbkV : dbkU)[((pix_y >> 1) + r) * Wc + (pix_x >> 1) + c] : (pel)0;
        } else {                                         // the neighbours' results (bS, 8.7.2.1)
            const int j = i - 256, dir = j >> 3, k = j & 7;
            const bool av = dir == 0 ? dbL : dbT;
            if (av) {
                const jmh_mb_result *rp = d.res + (dir == 0 ? mby * d.mbw + mbx - 1 : (mby - 1) * d.mbw + mbx);
                if (k < 4) {
                    const int bp = dir == 0 ? k * 4 + 3 : 12 + k;
                    s.nmv[dir][k][0] = rp->mv[bp][0];
                    s.nmv[dir][k][1] = rp->mv[bp][1];
                } else if (k == 4) {
                    s.nbits[dir] = rp->cbp_blk;
                } else if (k == 5) {
                    const int t = rp->mb_type;
                    s.nintra[dir] = t == JMH_I4MB || t == JMH_I16MB || t == JMH_I8MB;
                }
            }
        }
    }
}

// the MB's deblocking on NT threads (tid), after its reconstruction rec (LDS, 16x16) / cfin (LDS,
// 2 x 8x8) is final.  fmv: the MB's MVs per 4x4, cbp_blk: its coded 4x4 blocks, t8flag: 8x8
// transform (no 4x4 luma edges), qpy / qpcy: QPY and QPc (thresholds).  Every thread of the
// workgroup must call it (it synchronises).  NTH: threads of the workgroup (256, or 512 in the
// 512-thread final bodies: the sample loads / stores stride over all of them)
template <class pel, int NTH = NT, bool PRE = false>
__device__ __forceinline__ void deblock_mb(const DevParams &d, DbkS<pel> &s, const pel *rec, const pel (*cfin)[64], const int16_t (*fmv)[2],
                                           bool is_intra, int cbp_blk, bool t8flag, int qpy, int qpcy, int mbx, int mby, int tid) {
    pel *dbkY = spl<pel>(d.dbkY), *dbkU = spl<pel>(d.dbkU), *dbkV = spl<pel>(d.dbkV);
    const int pix_x = 16 * mbx, pix_y = 16 * mby, W = d.W, Wc = d.Wc, maxv = d.maxv;
    // deblocking filters across slice edges (disable_deblocking_filter_idc 0): picture edges only
    const bool dbL = mbx > 0, dbT = mby > 0;
    {
        const bool filt = d.lf_disable != 1;
        __syncthreads();                          // rec, cfin final
        for (int i = tid; i < 400 + 288; i += NTH) {
            if (i < 400) {
                const int r = i / 20 - 4, c = i % 20 - 4;
                int v = 0;
                if (r >= 0 && c >= 0) v = rec[16 * r + c];
                else if ((r < 0) != (c < 0)) {
                    if (PRE) continue;                   // deblock_prefetch loaded the borders
                    if ((r < 0 && dbT) || (c < 0 && dbL)) v = dbkY[(pix_y + r) * W + pix_x + c];
                }
                s.dy[r + 4][c + 4] = (pel)v;
            } else {
                const int j = i - 400, pl = j / 144, r = (j % 144) / 12 - 4, c = j % 12 - 4;
                int v = 0;
                if (r >= 0 && c >= 0) v = cfin[pl][8 * r + c];
                else if ((r < 0) != (c < 0)) {
                    if (PRE) continue;
                    if ((r < 0 && dbT) || (c < 0 && dbL)) v = (pl ? dbkV : dbkU)[((pix_y >> 1) + r) * Wc + (pix_x >> 1) + c];
                }
                s.dc2[pl][r + 4][c + 4] = (pel)v;
            }
        }
        if (tid < 32) {                           // boundary strength (8.7.2.1), frame MBs, one reference
            const int dir = tid >> 4, e = (tid >> 2) & 3, i = tid & 3;
            const bool mb_edge = e == 0;
            int bS = 0;
            if (filt && !(mb_edge && (dir == 0 ? !dbL : !dbT))) {
                const int bq = dir == 0 ? i * 4 + e : e * 4 + i;
                const int bp = dir == 0 ? (mb_edge ? i * 4 + 3 : bq - 1) : (mb_edge ? 12 + i : bq - 4);
                bool intra_p = is_intra, pcoef;
                int pref, pmx, pmy;
                const int qref = is_intra ? -1 : 0, qmx = fmv[bq][0], qmy = fmv[bq][1];
                const bool qcoef = (cbp_blk >> bq) & 1;
                if (mb_edge && PRE) {
                    intra_p = s.nintra[dir];
                    pcoef = (s.nbits[dir] >> bp) & 1;
                    pref = intra_p ? -1 : 0;
                    pmx = s.nmv[dir][i][0]; pmy = s.nmv[dir][i][1];
                } else if (mb_edge) {
                    const int nx = dir == 0 ? mbx - 1 : mbx, ny = dir == 0 ? mby : mby - 1;
                    const jmh_mb_result *rp = d.res + ny * d.mbw + nx;
                    intra_p = rp->mb_type == JMH_I4MB || rp->mb_type == JMH_I16MB || rp->mb_type == JMH_I8MB;
                    pcoef = (rp->cbp_blk >> bp) & 1;
                    pref = intra_p ? -1 : 0;
                    pmx = rp->mv[bp][0]; pmy = rp->mv[bp][1];
                } else {
                    pcoef = (cbp_blk >> bp) & 1;
                    pref = qref; pmx = fmv[bp][0]; pmy = fmv[bp][1];
                }
                if (intra_p || is_intra) bS = mb_edge ? 4 : 3;
                else if (pcoef || qcoef) bS = 2;
                else if (pref != qref || abs(pmx - qmx) >= 4 || abs(pmy - qmy) >= 4) bS = 1;
            }
            s.bs[dir][e][i] = (int8_t)bS;
        }
        __syncthreads();
        if (tid < 64 && filt) {                   // one wave: luma lines on lanes 0..15, chroma on 16..31
            // indices from QPY / QPc (8.7.2.2), thresholds times 1 << (BitDepth - 8) (8-457..8-470)
            const int offA = d.lf_offA, offB = d.lf_offB, bsc = 1 << (d.qpbd / 6);
            const int iA = iclip(0, 51, qpy + offA), iB = iclip(0, 51, qpy + offB);
            const int alpha = bsc * c_alpha[iA], beta = bsc * c_beta[iB];
            const int t1 = bsc * c_tc0[iA][0], t2 = bsc * c_tc0[iA][1], t3 = bsc * c_tc0[iA][2];
            const int cA = iclip(0, 51, qpcy + offA), cB = iclip(0, 51, qpcy + offB);
            const int calpha = bsc * c_alpha[cA], cbeta = bsc * c_beta[cB];
            const int u1 = bsc * c_tc0[cA][0], u2 = bsc * c_tc0[cA][1], u3 = bsc * c_tc0[cA][2];
            for (int dir = 0; dir < 2; dir++)
                for (int e = 0; e < 4; e++) {
                    if (tid < 16 && !((e & 1) && t8flag)) {             // 8x8 transform: no 4x4 luma edges
                        const int k = tid, b = s.bs[dir][e][k >> 2];
                        if (b) {
                            pel *q = dir == 0 ? &s.dy[k + 4][4 * e + 4] : &s.dy[4 * e + 4][k + 4];
                            filter_line(q, dir == 0 ? 1 : 20, b, alpha, beta, b == 1 ? t1 : b == 2 ? t2 : t3, false, maxv);
                        }
                    } else if (tid < 32 && !(e & 1)) {
                        const int pl = (tid - 16) >> 3, k = tid & 7, b = s.bs[dir][e][k >> 1];
                        if (b) {
                            pel *q = dir == 0 ? &s.dc2[pl][k + 4][2 * e + 4] : &s.dc2[pl][2 * e + 4][k + 4];
                            filter_line(q, dir == 0 ? 1 : 12, b, calpha, cbeta, b == 1 ? u1 : b == 2 ? u2 : u3, true, maxv);
                        }
                    }
                    wave_lds_sync();
                }
        }
        __syncthreads();
        for (int i = tid; i < 400 + 288; i += NTH) {
            if (i < 400) {
                const int r = i / 20 - 4, c = i % 20 - 4;
                if ((r >= 0 && c >= 0) || (r >= -3 && r < 0 && c >= 0 && dbT) || (c >= -3 && c < 0 && r >= 0 && dbL))
                    dbkY[(pix_y + r) * W + pix_x + c] = s.dy[r + 4][c + 4];
            } else {
                const int j = i - 400, pl = j / 144, r = (j % 144) / 12 - 4, c = j % 12 - 4;
                if ((r >= 0 && c >= 0) || (r == -1 && c >= 0 && c < 8 && dbT) || (c == -1 && r >= 0 && r < 8 && dbL))
                    if (r < 8 && c < 8) (pl ? dbkV : dbkU)[((pix_y >> 1) + r) * Wc + (pix_x >> 1) + c] = s.dc2[pl][r + 4][c + 4];
            }
        }
    }
}
