/*
 * deblock.c — H.264 8.7 deblocking of a reconstructed picture (frame MBs, one slice),
 * restating JM 8.6 loopfilter.c › DeblockFrame / DeblockMb / GetStrength / EdgeLoop [J].
 * Per MB in raster order: luma vertical edges left->right, then horizontal top->bottom;
 * chroma likewise, each filtered in place on already-filtered samples.
 * Host-side in this build (GPU deblocking is "next").
 */
#include <stdlib.h>
#include "jmhost.h"

static const uint8_t ALPHA[52] = {0,  0,  0,  0,  0,  0,  0,  0,  0,   0,   0,   0,   0,   0,   0,   0,   4,   4,
                                  5,  6,  7,  8,  9,  10, 12, 13, 15,  17,  20,  22,  25,  28,  32,  36,  40,  45,
                                  50, 56, 63, 71, 80, 90, 101, 113, 127, 144, 162, 182, 203, 226, 255, 255};
static const uint8_t BETA[52] = {0,  0,  0,  0,  0,  0,  0,  0,  0,  0,  0,  0,  0,  0,  0,  0,  2,  2,
                                 2,  3,  3,  3,  3,  4,  4,  4,  6,  6,  7,  7,  8,  8,  9,  9,  10, 10,
                                 11, 11, 12, 12, 13, 13, 14, 14, 15, 15, 16, 16, 17, 17, 18, 18};
static const uint8_t TC0[52][3] = {
    {0, 0, 0}, {0, 0, 0}, {0, 0, 0}, {0, 0, 0}, {0, 0, 0}, {0, 0, 0}, {0, 0, 0}, {0, 0, 0}, {0, 0, 0},
    {0, 0, 0}, {0, 0, 0}, {0, 0, 0}, {0, 0, 0}, {0, 0, 0}, {0, 0, 0}, {0, 0, 0}, {0, 0, 0}, {0, 0, 1},
    {0, 0, 1}, {0, 0, 1}, {0, 0, 1}, {0, 1, 1}, {0, 1, 1}, {1, 1, 1}, {1, 1, 1}, {1, 1, 1}, {1, 1, 1},
    {1, 1, 2}, {1, 1, 2}, {1, 1, 2}, {1, 1, 2}, {1, 2, 3}, {1, 2, 3}, {2, 2, 3}, {2, 2, 4}, {2, 3, 4},
    {2, 3, 4}, {3, 3, 5}, {3, 4, 6}, {3, 4, 6}, {4, 5, 7}, {4, 5, 8}, {4, 6, 9}, {5, 7, 10}, {6, 8, 11},
    {6, 8, 13}, {7, 10, 14}, {8, 11, 16}, {9, 12, 18}, {10, 13, 20}, {11, 15, 23}, {13, 17, 25}};
static const uint8_t QPC[52] = {0,  1,  2,  3,  4,  5,  6,  7,  8,  9,  10, 11, 12, 13, 14, 15, 16, 17,
                                18, 19, 20, 21, 22, 23, 24, 25, 26, 27, 28, 29, 29, 30, 31, 32, 32, 33,
                                34, 34, 35, 35, 36, 36, 37, 37, 37, 38, 38, 38, 39, 39, 39, 39};

static inline int clip3(int lo, int hi, int v) { return v < lo ? lo : v > hi ? hi : v; }
static inline int iabs_(int v) { return v < 0 ? -v : v; }

static int is_intra(const jmh_mb_result *r) { return r->mb_type == JMH_I4MB || r->mb_type == JMH_I16MB || r->mb_type == JMH_I8MB; }
static int has_coef(const jmh_mb_result *r, int blk) {   /* 4x4 luma block (raster) coded */
    if (r->mb_type == JMH_I16MB) return 1;              /* intra: bS >= 3 anyway            */
    return (r->cbp_blk >> blk) & 1;
}

/* bS for the edge between 4x4 block p (MB rp) and q (MB rq) (8.7.2.1, frame MBs, P slices) */
static int strength(const jmh_mb_result *rp, int bp, const jmh_mb_result *rq, int bq, int mb_edge) {
    if (is_intra(rp) || is_intra(rq)) return mb_edge ? 4 : 3;
    if (has_coef(rp, bp) || has_coef(rq, bq)) return 2;
    if (rp->ref_idx[((bp >> 3) << 1) + ((bp & 3) >> 1)] != rq->ref_idx[((bq >> 3) << 1) + ((bq & 3) >> 1)]) return 1;
    if (iabs_(rp->mv[bp][0] - rq->mv[bq][0]) >= 4 || iabs_(rp->mv[bp][1] - rq->mv[bq][1]) >= 4) return 1;
    return 0;
}

/* filter one line of samples across an edge; p[-k*step] = pk, p[k*step] = q_k (q0 at p[0]).
 * alpha, beta, tc0 already scaled by 1 << (BitDepth - 8) (8.7.2.2 / 8.7.2.3), Clip1 to maxv. */
#define FILTER_LINE(NAME, T)                                                                            \
    static void NAME(T *q0p, int step, int bS, int alpha, int beta, int tc0, int chroma, int maxv) {    \
        int p0 = q0p[-step], p1 = q0p[-2 * step], q0 = q0p[0], q1 = q0p[step];                        \
        if (!(iabs_(p0 - q0) < alpha && iabs_(p1 - p0) < beta && iabs_(q1 - q0) < beta)) return;     \
        if (chroma) {                                                                                  \
            if (bS < 4) {                                                                              \
                int tc = tc0 + 1;                                                                      \
                int d = clip3(-tc, tc, ((q0 - p0) * 4 + (p1 - q1) + 4) >> 3);                          \
                q0p[-step] = (T)clip3(0, maxv, p0 + d);                                                \
                q0p[0] = (T)clip3(0, maxv, q0 - d);                                                    \
            } else {                                                                                   \
                q0p[-step] = (T)((2 * p1 + p0 + q1 + 2) >> 2);                                         \
                q0p[0] = (T)((2 * q1 + q0 + p1 + 2) >> 2);                                             \
            }                                                                                          \
            return;                                                                                    \
        }                                                                                              \
        int p2 = q0p[-3 * step], q2 = q0p[2 * step];                                                   \
        int ap = iabs_(p2 - p0), aq = iabs_(q2 - q0);                                                  \
        if (bS < 4) {                                                                                  \
            int tc = tc0 + (ap < beta) + (aq < beta);                                                  \
            int d = clip3(-tc, tc, ((q0 - p0) * 4 + (p1 - q1) + 4) >> 3);                              \
            q0p[-step] = (T)clip3(0, maxv, p0 + d);                                                    \
            q0p[0] = (T)clip3(0, maxv, q0 - d);                                                        \
            if (ap < beta) q0p[-2 * step] = (T)(p1 + clip3(-tc0, tc0, (p2 + ((p0 + q0 + 1) >> 1) - (p1 << 1)) >> 1)); \
            if (aq < beta) q0p[step] = (T)(q1 + clip3(-tc0, tc0, (q2 + ((p0 + q0 + 1) >> 1) - (q1 << 1)) >> 1));     \
        } else {                                                                                       \
            int p3 = q0p[-4 * step], q3 = q0p[3 * step];                                               \
            int small = iabs_(p0 - q0) < ((alpha >> 2) + 2);                                           \
            if (ap < beta && small) {                                                                  \
                q0p[-step] = (T)((p2 + 2 * p1 + 2 * p0 + 2 * q0 + q1 + 4) >> 3);                       \
                q0p[-2 * step] = (T)((p2 + p1 + p0 + q0 + 2) >> 2);                                     \
                q0p[-3 * step] = (T)((2 * p3 + 3 * p2 + p1 + p0 + q0 + 4) >> 3);                        \
            } else q0p[-step] = (T)((2 * p1 + p0 + q1 + 2) >> 2);                                      \
            if (aq < beta && small) {                                                                  \
                q0p[0] = (T)((p1 + 2 * p0 + 2 * q0 + 2 * q1 + q2 + 4) >> 3);                           \
                q0p[step] = (T)((p0 + q0 + q1 + q2 + 2) >> 2);                                          \
                q0p[2 * step] = (T)((2 * q3 + 3 * q2 + q1 + q0 + p0 + 4) >> 3);                         \
            } else q0p[0] = (T)((2 * q1 + q0 + p1 + 2) >> 2);                                          \
        }                                                                                              \
    }
FILTER_LINE(filter_line8, uint8_t)
FILTER_LINE(filter_line16, uint16_t)
#undef FILTER_LINE

/* QPc (Table 8-15) of qPI = QPY + chroma_qp_index_offset clipped to [-QpBdOffsetC, 51] */
static int qpc_of(int qpi, int qpbd) {
    qpi = clip3(-qpbd, 51, qpi);
    return qpi < 0 ? qpi : QPC[qpi];
}

void jm_deblock_picture(jm_pic *p, const jm_seq *s, const jmh_mb_result *const *res, int qp) {
    if (s->lf_params_flag && s->lf_disable == 1) return;
    int offA = s->lf_params_flag ? 2 * s->lf_alpha : 0, offB = s->lf_params_flag ? 2 * s->lf_beta : 0;
    int W = p->w, Wc = p->w / 2;
    const int hbd = p->bd > 8, sc = hbd ? 1 << (p->bd - 8) : 1, maxv = hbd ? (1 << p->bd) - 1 : 255;
    int qpc = qpc_of(qp + s->chroma_qp_offset, 6 * (p->bd - 8));     /* deblocking uses QPc, not QP'c */
    for (int my = 0; my < s->mbh; my++)
        for (int mx = 0; mx < s->mbw; mx++) {
            const jmh_mb_result *rq = res[my * s->mbw + mx];
            for (int dir = 0; dir < 2; dir++) {       /* 0: vertical edges, 1: horizontal */
                for (int e = 0; e < 4; e++) {
                    int mb_edge = e == 0;
                    if ((e & 1) && rq->transform_8x8) continue;   /* 8x8 transform: no 4x4 luma edges */
                    const jmh_mb_result *rp = rq;
                    if (mb_edge) {
                        if (dir == 0 && mx == 0) continue;
                        if (dir == 1 && my == 0) continue;
                        rp = dir == 0 ? res[my * s->mbw + mx - 1] : res[(my - 1) * s->mbw + mx];
                    }
                    int bS[4];
                    for (int i = 0; i < 4; i++) {
                        int bq = dir == 0 ? i * 4 + e : e * 4 + i;
                        int bp = dir == 0 ? (mb_edge ? i * 4 + 3 : bq - 1) : (mb_edge ? 12 + i : bq - 4);
                        bS[i] = strength(rp, bp, rq, bq, mb_edge);
                    }
                    if (!bS[0] && !bS[1] && !bS[2] && !bS[3]) continue;
                    /* luma: qp of both MBs is the slice qp (no mb_qp_delta) */
                    int iA = clip3(0, 51, qp + offA), iB = clip3(0, 51, qp + offB);
                    int alpha = ALPHA[iA] * sc, beta = BETA[iB] * sc;
                    for (int k = 0; k < 16; k++) {
                        int b = bS[k >> 2];
                        if (!b) continue;
                        const size_t o = dir == 0 ? (size_t)(16 * my + k) * W + 16 * mx + 4 * e : (size_t)(16 * my + 4 * e) * W + 16 * mx + k;
                        const int tc0 = (b < 4 ? TC0[iA][b - 1] : 0) * sc;
                        if (hbd) filter_line16(p->Y + o, dir == 0 ? 1 : W, b, alpha, beta, tc0, 0, maxv);
                        else filter_line8(p->y + o, dir == 0 ? 1 : W, b, alpha, beta, tc0, 0, maxv);
                    }
                    if (e & 1) continue;                 /* chroma edges 0 and 2 (4:2:0) */
                    int cA = clip3(0, 51, qpc + offA), cB = clip3(0, 51, qpc + offB);
                    int ca = ALPHA[cA] * sc, cb = BETA[cB] * sc;
                    for (int pl = 0; pl < 2; pl++) {
                        for (int k = 0; k < 8; k++) {
                            int b = bS[k >> 1];
                            if (!b) continue;
                            const size_t o = dir == 0 ? (size_t)(8 * my + k) * Wc + 8 * mx + 2 * e : (size_t)(8 * my + 2 * e) * Wc + 8 * mx + k;
                            const int tc0 = (b < 4 ? TC0[cA][b - 1] : 0) * sc;
                            if (hbd) filter_line16((pl ? p->V : p->U) + o, dir == 0 ? 1 : Wc, b, ca, cb, tc0, 1, maxv);
                            else filter_line8((pl ? p->v : p->u) + o, dir == 0 ? 1 : Wc, b, ca, cb, tc0, 1, maxv);
                        }
                    }
                }
            }
        }
}
