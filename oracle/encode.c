/*
 * encode.c — oracle restatement of JM 8.6 lencod's RDO-off macroblock hot path
 * (TEST INFRASTRUCTURE ONLY; see jm_oracle.h for the parity status).
 *
 * Restated JM 8.6 functions [J] (no file:line exists: /root/reference holds README.md:1-4):
 *   rdopt.c      › encode_one_macroblock (RDO off), Mode_Decision_for_Intra4x4Macroblock,
 *                  Mode_Decision_for_8x8IntraBlocks, Mode_Decision_for_4x4IntraBlocks,
 *                  SetModesAndRefframeForBlocks, SetCoeffAndReconstruction8x8
 *   mv-search.c  › SetMotionVectorPredictor, FindSkipModeMotionVector, PartitionMotionSearch,
 *                  BlockMotionSearch, SetupFastFullPelSearch, SetupLargerBlocks,
 *                  FastFullPelBlockMotionSearch, FullPelBlockMotionSearch,
 *                  SubPelBlockMotionSearch
 *   block.c      › intrapred_luma, intrapred_luma_16x16, find_sad_16x16, dct_luma,
 *                  dct_luma_16x16, dct_chroma
 *   macroblock.c › LumaResidualCoding, LumaResidualCoding8x8, LumaPrediction4x4,
 *                  ChromaResidualCoding, OneComponentChromaPrediction4x4,
 *                  IntraChromaPrediction8x8
 * Normative pieces follow ITU-T H.264: 8.3.1/8.3.3/8.3.4 (intra prediction), 8.4.1.3 (MVP),
 * 8.4.1.1 (P_Skip MV), 8.4.2.2 (sample interpolation), 8.5.10-8.5.12 (inverse transforms).
 * Non-normative choices are listed in docs/JM_SEMANTICS.md.
 */
#include <stdlib.h>
#include "jmo_internal.h"


/* ====================================================================================== */
/*  neighbour access (getLuma4x4Neighbour / getNeighbour, H.264 6.4.11/6.4.12; neighbours
 *  outside the current slice are unavailable, 6.4.8 / JM_SEMANTICS item 47) */
/* ====================================================================================== */
int jmo_nb4(const mbs *s, int xN, int yN, int *idx) {
    const jmo_ctx *c = s->c;
    int mx, my;
    if (yN > 15) return 0;
    if (xN < 0) { mx = s->mbx - 1; my = yN < 0 ? s->mby - 1 : s->mby; }
    else if (xN <= 15) { mx = s->mbx; my = yN < 0 ? s->mby - 1 : s->mby; }
    else { if (yN >= 0) return 0; mx = s->mbx + 1; my = s->mby - 1; }
    if (mx < 0 || my < 0 || mx >= c->mbw || !jmo_same_slice(c, s->mby * c->mbw + s->mbx, my * c->mbw + mx)) return 0;
    *idx = ((s->pix_y + yN) >> 2) * (c->W >> 2) + ((s->pix_x + xN) >> 2);
    return 1;
}

/* the A, B, C neighbours of SetMotionVectorPredictor [J] / 8.4.1.3 (C replaced by D when not
 * available, including C inside the MB but later in decoding order); 4x4 picture indices */
static void mvp_neighbours(const mbs *s, int block_x, int block_y, int bsx, int bsy, int *av_a, int *av_b,
                           int *av_c, int *ia, int *ib, int *ic) {
    int mb_x = 4 * block_x, mb_y = 4 * block_y, id = 0;
    (void)bsy;
    *av_a = jmo_nb4(s, mb_x - 1, mb_y, ia);
    *av_b = jmo_nb4(s, mb_x, mb_y - 1, ib);
    *av_c = jmo_nb4(s, mb_x + bsx, mb_y - 1, ic);
    int av_d = jmo_nb4(s, mb_x - 1, mb_y - 1, &id);
    if (mb_y > 0) {                       /* C inside the MB but later in decoding order */
        if (mb_x < 8) {
            if (mb_y == 8) { if (bsx == 16) *av_c = 0; }
            else if (mb_x + bsx == 8) *av_c = 0;
        } else if (mb_x + bsx == 16) *av_c = 0;
    }
    if (!*av_c) { *av_c = av_d; *ic = id; }
}

/* SetMotionVectorPredictor [J] / H.264 8.4.1.3 (list 0). block_x/y in 4x4 units. */
void jmo_set_mvp(const mbs *s, int pmv[2], int ref, int block_x, int block_y, int bsx, int bsy) {
    const jmo_ctx *c = s->c;
    int ia = 0, ib = 0, ic = 0, av_a, av_b, av_c;
    mvp_neighbours(s, block_x, block_y, bsx, bsy, &av_a, &av_b, &av_c, &ia, &ib, &ic);
    int mb_x = 4 * block_x, mb_y = 4 * block_y;
    int rL = av_a ? c->refidx[ia] : -1;
    int rU = av_b ? c->refidx[ib] : -1;
    int rUR = av_c ? c->refidx[ic] : -1;
    enum { MEDIAN, PL, PU, PUR } type = MEDIAN;
    if (rL == ref && rU != ref && rUR != ref) type = PL;
    else if (rL != ref && rU == ref && rUR != ref) type = PU;
    else if (rL != ref && rU != ref && rUR == ref) type = PUR;
    if (bsx == 8 && bsy == 16) {
        if (mb_x == 0) { if (rL == ref) type = PL; }
        else if (rUR == ref) type = PUR;
    } else if (bsx == 16 && bsy == 8) {
        if (mb_y == 0) { if (rU == ref) type = PU; }
        else if (rL == ref) type = PL;
    }
    for (int hv = 0; hv < 2; hv++) {
        int a = av_a ? c->mv[2 * ia + hv] : 0;
        int b = av_b ? c->mv[2 * ib + hv] : 0;
        int cc = av_c ? c->mv[2 * ic + hv] : 0;
        int p;
        switch (type) {
        case PL: p = a; break;
        case PU: p = b; break;
        case PUR: p = cc; break;
        default:
            if (!(av_b || av_c)) p = a;
            else p = a + b + cc - imin(a, imin(b, cc)) - imax(a, imax(b, cc));
        }
        pmv[hv] = p;
    }
}

/* unit-test entry: the same rules on explicit neighbours (single MB, no picture) */
void jmo_mvp_median(int av_a, int rL, int ax, int ay, int av_b, int rU, int bx, int by,
                    int av_c, int rUR, int cx, int cy, int ref, int bsx, int bsy, int blk_x,
                    int blk_y, int32_t *pmv) {
    (void)blk_y;
    int type = 0;
    if (!av_a) rL = -1;
    if (!av_b) rU = -1;
    if (!av_c) rUR = -1;
    if (rL == ref && rU != ref && rUR != ref) type = 1;
    else if (rL != ref && rU == ref && rUR != ref) type = 2;
    else if (rL != ref && rU != ref && rUR == ref) type = 3;
    if (bsx == 8 && bsy == 16) { if (blk_x == 0) { if (rL == ref) type = 1; } else if (rUR == ref) type = 3; }
    else if (bsx == 16 && bsy == 8) { if (blk_y == 0) { if (rU == ref) type = 2; } else if (rL == ref) type = 1; }
    int va[2] = {av_a ? ax : 0, av_a ? ay : 0}, vb[2] = {av_b ? bx : 0, av_b ? by : 0},
        vc[2] = {av_c ? cx : 0, av_c ? cy : 0};
    for (int hv = 0; hv < 2; hv++) {
        int a = va[hv], b = vb[hv], cc = vc[hv];
        if (type == 1) pmv[hv] = a;
        else if (type == 2) pmv[hv] = b;
        else if (type == 3) pmv[hv] = cc;
        else if (!(av_b || av_c)) pmv[hv] = a;
        else pmv[hv] = a + b + cc - imin(a, imin(b, cc)) - imax(a, imax(b, cc));
    }
}

/* FindSkipModeMotionVector [J] / H.264 8.4.1.1 */
void jmo_find_skip_mv(mbs *s) {
    const jmo_ctx *c = s->c;
    int ia = 0, ib = 0;
    int av_a = jmo_nb4(s, -1, 0, &ia), av_b = jmo_nb4(s, 0, -1, &ib);
    int zl = !av_a ? 1 : (c->refidx[ia] == 0 && c->mv[2 * ia] == 0 && c->mv[2 * ia + 1] == 0);
    int za = !av_b ? 1 : (c->refidx[ib] == 0 && c->mv[2 * ib] == 0 && c->mv[2 * ib + 1] == 0);
    if (za || zl) { s->skip_mv[0] = s->skip_mv[1] = 0; }
    else {
        int pmv[2];
        jmo_set_mvp(s, pmv, 0, 0, 0, 16, 16);
        s->skip_mv[0] = pmv[0]; s->skip_mv[1] = pmv[1];
    }
}

/* ====================================================================================== */
/*  motion estimation                                                                        */
/* ====================================================================================== */
static inline int refpel(const jmo_ctx *c, int x, int y) {   /* UMV integer access (clamp) */
    return c->refY[iclip(0, c->H - 1, y) * c->W + iclip(0, c->W - 1, x)];
}
static inline int mv_cost(const mbs *s, int shift, int cx, int cy, int px, int py) {
    /* MV_COST(f,s,cx,cy,px,py) = (f*(mvbits[(cx<<s)-px]+mvbits[(cy<<s)-py])) >> 16 [J] */
    return (s->lf * (jmo_mvbits(cx * (1 << shift) - px) + jmo_mvbits(cy * (1 << shift) - py))) >> 16;
}

static int block_range(const mbs *s, int blocktype) {
    int sr = s->c->sr, rs = s->c->cfg.restrict_search_range;
    /* PartitionMotionSearch [J]: ref 0 -> (min(ref,1)+1) == 1 */
    if (rs == 2) return sr;
    if (rs == 1) return sr;
    return sr / imin(2, blocktype);
}

/* SetupFastFullPelSearch [J]: window centre = 16x16 MVP/4 (trunc), clamped to +-SR (RDO off);
 * 16 4x4 SADs per search position (stored in window raster order). */
static void ffs_setup_at(mbs *s, int scx, int scy) {
    jmo_ctx *c = s->c;
    int sr = c->sr, side = 2 * sr + 1;
    s->scx = scx;
    s->scy = scy;
    s->pos_00 = c->spiral_of[(-s->scy + sr) * side + (-s->scx + sr)];
    for (int dy = -sr; dy <= sr; dy++)
        for (int dx = -sr; dx <= sr; dx++) {
            int ax = s->pix_x + s->scx + dx, ay = s->pix_y + s->scy + dy;
            int r = (dy + sr) * side + (dx + sr);
            for (int b = 0; b < 16; b++) {
                int ox = (b & 3) * 4, oy = (b >> 2) * 4, sad = 0;
                for (int y = 0; y < 4; y++)
                    for (int x = 0; x < 4; x++)
                        sad += iabs(s->org[(oy + y) * 16 + ox + x] - refpel(c, ax + ox + x, ay + oy + y));
                c->blocksad[(size_t)b * c->npos + r] = (uint16_t)sad;
            }
        }
    s->setup_done = 1;
}
static void ffs_setup(mbs *s) {
    int sr = s->c->sr, pmv[2];
    jmo_set_mvp(s, pmv, 0, 0, 0, 16, 16);
    ffs_setup_at(s, iclip(-sr, sr, pmv[0] / 4), iclip(-sr, sr, pmv[1] / 4));
}

/* SetupLargerBlocks [J] equivalent: SAD of a bsx x bsy block at window raster index r */
static inline int block_sad_at(const mbs *s, int bx4, int by4, int w4, int h4, int r) {
    const jmo_ctx *c = s->c;
    int sum = 0;
    for (int y = 0; y < h4; y++)
        for (int x = 0; x < w4; x++)
            sum += c->blocksad[(size_t)((by4 + y) * 4 + bx4 + x) * c->npos + r];
    return sum;
}

/* FastFullPelBlockMotionSearch [J] */
static int ffs_search(mbs *s, int blocktype, int bx4, int by4, int pmvx, int pmvy, int range,
                      int *mvx, int *mvy) {
    jmo_ctx *c = s->c;
    int sr = c->sr, side = 2 * sr + 1;
    int w4 = jmo_blc_size[blocktype][0] >> 2, h4 = jmo_blc_size[blocktype][1] >> 2;
    int max_pos = (2 * range + 1) * (2 * range + 1);
    int min_mcost = BIGCOST, best_pos = 0;
    if (!s->setup_done) ffs_setup(s);
    if (!s->rdo) {   /* cost for (0,0)-vector first: RDO off only (!input->rdopt [J], item 65) */
        int r = (-s->scy + sr) * side + (-s->scx + sr);
        int mcost = block_sad_at(s, bx4, by4, w4, h4, r) + mv_cost(s, 2, 0, 0, pmvx, pmvy);
        if (mcost < min_mcost) { min_mcost = mcost; best_pos = s->pos_00; }
    }
    for (int pos = 0; pos < max_pos; pos++) {
        int dx = c->spiral_x[pos], dy = c->spiral_y[pos];
        int sad = block_sad_at(s, bx4, by4, w4, h4, (dy + sr) * side + (dx + sr));
        if (sad < min_mcost) {
            int mcost = sad + mv_cost(s, 2, s->scx + dx, s->scy + dy, pmvx, pmvy);
            if (mcost < min_mcost) { min_mcost = mcost; best_pos = pos; }
        }
    }
    *mvx = s->scx + c->spiral_x[best_pos];
    *mvy = s->scy + c->spiral_y[best_pos];
    return min_mcost;
}

/* FullPelBlockMotionSearch [J] (SearchMode -1): window centred on the block's own MVP */
static int full_search(mbs *s, int blocktype, int bx4, int by4, int pmvx, int pmvy, int range,
                       int *mvx, int *mvy) {
    jmo_ctx *c = s->c;
    int bsx = jmo_blc_size[blocktype][0], bsy = jmo_blc_size[blocktype][1];
    int max_pos = (2 * range + 1) * (2 * range + 1);
    int pic_x = s->pix_x + 4 * bx4, pic_y = s->pix_y + 4 * by4;
    int cxa = pic_x + *mvx, cya = pic_y + *mvy;
    int check_00 = (blocktype == 1 && s->slice_p && !s->rdo);   /* !input->rdopt [J] */
    int min_mcost = BIGCOST, best_pos = 0;
    for (int pos = 0; pos < max_pos; pos++) {
        int cx = cxa + c->spiral_x[pos], cy = cya + c->spiral_y[pos];
        int mcost = mv_cost(s, 2, cx - pic_x, cy - pic_y, pmvx, pmvy);
        if (check_00 && cx == pic_x && cy == pic_y) mcost -= (s->lf * 16) >> 16;
        if (mcost >= min_mcost) continue;
        for (int y = 0; y < bsy; y++)
            for (int x = 0; x < bsx; x++)
                mcost += iabs(s->org[(4 * by4 + y) * 16 + 4 * bx4 + x] - refpel(c, cx + x, cy + y));
        if (mcost < min_mcost) { best_pos = pos; min_mcost = mcost; }
    }
    *mvx += c->spiral_x[best_pos];
    *mvy += c->spiral_y[best_pos];
    return min_mcost;
}

/* ====================================================================================== */
/*  EPZS (SearchMode 3): me_epzs.c › EPZSPelBlockMotionSearch [J] as restated in             */
/*  docs/JM_SEMANTICS.md items 33-40 (JM parity unpinned: no JM source exists here)          */
/* ====================================================================================== */
static const int epzs_ed[12][2] = {{0, -2}, {-1, -1}, {1, -1}, {-2, 0}, {2, 0}, {-1, 1},   /* extended diamond */
                                   {1, 1},  {0, 2},   {0, -1}, {-1, 0}, {1, 0}, {0, 1}};
static const int epzs_sd[4][2] = {{0, -1}, {-1, 0}, {1, 0}, {0, 1}};                       /* small diamond   */
static const int epzs_win[8][2] = {{0, -1}, {-1, 0}, {1, 0}, {0, 1}, {-1, -1}, {1, -1}, {-1, 1}, {1, 1}};
static inline int rnd_fp(int v) { return (v + 2) >> 2; }          /* rshift_rnd_sf(mv, 2) [J] */

/* SAD of the block at full-pel displacement (mx, my) + MV_COST */
static int epzs_cost(const mbs *s, int bt, int bx4, int by4, int mx, int my, int pmvx, int pmvy) {
    const jmo_ctx *c = s->c;
    int bsx = jmo_blc_size[bt][0], bsy = jmo_blc_size[bt][1];
    int px = s->pix_x + 4 * bx4, py = s->pix_y + 4 * by4, sad = 0;
    for (int y = 0; y < bsy; y++)
        for (int x = 0; x < bsx; x++)
            sad += iabs(s->org[(4 * by4 + y) * 16 + 4 * bx4 + x] - refpel(c, px + mx + x, py + my + y));
    return sad + mv_cost(s, 2, mx, my, pmvx, pmvy);
}

/* the ordered EPZS predictor list of one search; returns its length (invalid entries flagged) */
static int epzs_predictors(const mbs *s, int bt, int bx4, int by4, int range, int c0x, int c0y,
                           int cand[41][2], int ok[41]) {
    const jmo_ctx *c = s->c;
    int n = 0, w4 = jmo_blc_size[bt][0] >> 2, h4 = jmo_blc_size[bt][1] >> 2;
#define ADD(v, x, y) do { ok[n] = (v); cand[n][0] = (x); cand[n][1] = (y); n++; } while (0)
    ADD(1, c0x, c0y);                                       /* 0: the search centre (median)   */
    ADD(1, 0, 0);                                           /* 1: zero vector                  */
    int av[3], ix[3];                                       /* 2-4: spatial A, B, C (or D)     */
    mvp_neighbours(s, bx4, by4, 4 * w4, 4 * h4, &av[0], &av[1], &av[2], &ix[0], &ix[1], &ix[2]);
    for (int k = 0; k < 3; k++) {
        int v = av[k] && c->refidx[ix[k]] == 0;
        ADD(v, v ? rnd_fp(c->mv[2 * ix[k]]) : 0, v ? rnd_fp(c->mv[2 * ix[k] + 1]) : 0);
    }
    for (int ring = 0; ring < 3; ring++) {                  /* 5-28: window rings R/4, R/2, R  */
        int r = range >> (2 - ring);
        for (int k = 0; k < 8; k++) ADD(r > 0, c0x + r * epzs_win[k][0], c0y + r * epzs_win[k][1]);
    }
    int W4 = c->W >> 2, H4 = c->H >> 2, X = (s->pix_x >> 2) + bx4, Y = (s->pix_y >> 2) + by4;
    const int tx[5] = {X, X - 1, X + w4, X, X}, ty[5] = {Y, Y, Y, Y - 1, Y + h4};
    for (int k = 0; k < 5; k++) {                           /* 29-33: temporal (co-located +4) */
        int in = tx[k] >= 0 && tx[k] < W4 && ty[k] >= 0 && ty[k] < H4;
        int i = in ? ty[k] * W4 + tx[k] : 0, v = in && c->tref[i] == 0;
        ADD(v, v ? rnd_fp(c->tmv[2 * i]) : 0, v ? rnd_fp(c->tmv[2 * i + 1]) : 0);
    }
    int k0 = by4 * 4 + bx4;                                 /* 34: spatial memory (left MB)    */
    int vm = s->mbx > 0 && jmo_same_slice(c, s->mby * c->mbw + s->mbx, s->mby * c->mbw + s->mbx - 1) && c->cfg.inter_search[bt];
    ADD(vm, vm ? rnd_fp(c->mem_mv[bt][k0][0]) : 0, vm ? rnd_fp(c->mem_mv[bt][k0][1]) : 0);
    static const int types[6] = {1, 2, 3, 4, 5, 6};         /* 35-40: earlier block types      */
    for (int k = 0; k < 6; k++) {
        int t = types[k], v = t < bt && c->cfg.inter_search[t];
        ADD(v, v ? rnd_fp(s->all_mv[t][k0][0]) : 0, v ? rnd_fp(s->all_mv[t][k0][1]) : 0);
    }
#undef ADD
    return n;
}

/* pattern refinement (item 37/38) from (bx, by) at cost *mc: small or extended diamond around the
 * current best, strict '<' in pattern order, move and repeat until no point improves */
static void epzs_refine(mbs *s, int bt, int bx4, int by4, int pmvx, int pmvy, int range, int c0x, int c0y, int sd,
                        int *bx, int *by, int *mc) {
    const int (*pat)[2] = sd ? epzs_sd : epzs_ed;
    int np = sd ? 4 : 12;
    for (;;) {
        int bi = -1, nbx = *bx, nby = *by;
        for (int i = 0; i < np; i++) {
            int mx = *bx + pat[i][0], my = *by + pat[i][1];
            if (iabs(mx - c0x) > range || iabs(my - c0y) > range) continue;
            int m = epzs_cost(s, bt, bx4, by4, mx, my, pmvx, pmvy);
            if (m < *mc) { *mc = m; bi = i; nbx = mx; nby = my; }
        }
        if (bi < 0) break;
        *bx = nbx; *by = nby;
    }
}

/* EPZSDetermineStopCriterion [J] restated (item 61): the stop criterion after the predictors from
 * the full-pel costs of the same block type's searches at the neighbours A (left), B (above), C
 * (above right, availability as SetMotionVectorPredictor's C but without the D substitution),
 * clamped to [minthres, maxthres], then (9 max(medthres, s) + 2 medthres) >> 3 */
static int epzs_stop_criterion(const mbs *s, int bt, int bx4, int by4, int w4, int h4, int med) {
    const jmo_ctx *c = s->c;
    const int pe = (c->maxv + 1) >> 8, npx = 16 * w4 * h4, mb_x = 4 * bx4, mb_y = 4 * by4, bsx = 4 * w4;
    const int minthres = c->cfg.epzs_min_thres_scale * npx * pe, maxthres = c->cfg.epzs_max_thres_scale * npx * pe;
    int ia = 0, ib = 0, ic = 0;
    int va = jmo_nb4(s, mb_x - 1, mb_y, &ia), vb = jmo_nb4(s, mb_x, mb_y - 1, &ib), vc = jmo_nb4(s, mb_x + bsx, mb_y - 1, &ic);
    if (mb_y > 0) {                       /* C inside the MB but later in decoding order */
        if (mb_x < 8) {
            if (mb_y == 8) { if (bsx == 16) vc = 0; }
            else if (mb_x + bsx == 8) vc = 0;
        } else if (mb_x + bsx == 16) vc = 0;
    }
    const uint16_t *fp = c->epzs_fp + (size_t)bt * (c->W >> 2) * (c->H >> 2);
    int sad = 0x7FFFFFFF;
    if (va && fp[ia] < sad) sad = fp[ia];
    if (vb && fp[ib] < sad) sad = fp[ib];
    if (vc && fp[ic] < sad) sad = fp[ic];
    sad = sad < minthres ? minthres : sad;
    sad = sad > maxthres ? maxthres : sad;
    return (9 * (med > sad ? med : sad) + 2 * med) >> 3;
}

static int epzs_search(mbs *s, int bt, int bx4, int by4, int pmvx, int pmvy, int range, int *mvx, int *mvy) {
    int c0x = *mvx, c0y = *mvy;
    /* medthres: EPZSMedThresScale 1, times pel_error_me = 1 << (bit depth - 8) (High 10) */
    int med = jmo_blc_size[bt][0] * jmo_blc_size[bt][1] * ((s->c->maxv + 1) >> 8);
    int cand[41][2], ok[41];
    int n = epzs_predictors(s, bt, bx4, by4, range, c0x, c0y, cand, ok);
    int min_mcost = epzs_cost(s, bt, bx4, by4, c0x, c0y, pmvx, pmvy), bx = c0x, by = c0y;
    /* the runner-up predictor (EPZSDualRefinement, item 46): the cheapest of the others,
     * earliest first on ties -- what a scan keeping best and second best ends with */
    int m2 = 0x7FFFFFFF, x2 = 0, y2 = 0;
    if (min_mcost >= med) {
        /* the stop criterion after the predictors: medthres, or the neighbour-adaptive one */
        int stop = med;
        if (s->c->cfg.epzs_max_thres_scale)
            stop = epzs_stop_criterion(s, bt, bx4, by4, jmo_blc_size[bt][0] >> 2, jmo_blc_size[bt][1] >> 2, med);
        for (int i = 1; i < n; i++) {                       /* predictors in order, strict '<' */
            if (!ok[i] || iabs(cand[i][0] - c0x) > range || iabs(cand[i][1] - c0y) > range) continue;
            int mc = epzs_cost(s, bt, bx4, by4, cand[i][0], cand[i][1], pmvx, pmvy);
            if (mc < min_mcost) { m2 = min_mcost; x2 = bx; y2 = by; min_mcost = mc; bx = cand[i][0]; by = cand[i][1]; }
            else if (mc < m2) { m2 = mc; x2 = cand[i][0]; y2 = cand[i][1]; }
        }
        if (min_mcost >= stop) {                            /* pattern refinement          */
            int sd = min_mcost < stop + ((3 * stop) >> 1);
            int pbx = bx, pby = by;
            epzs_refine(s, bt, bx4, by4, pmvx, pmvy, range, c0x, c0y, sd, &bx, &by, &min_mcost);
            if (s->c->cfg.epzs_dual_refinement && m2 != 0x7FFFFFFF && (x2 != pbx || y2 != pby)) {
                epzs_refine(s, bt, bx4, by4, pmvx, pmvy, range, c0x, c0y, sd, &x2, &y2, &m2);
                if (m2 < min_mcost) { min_mcost = m2; bx = x2; by = y2; }
            }
        }
    }
    *mvx = bx; *mvy = by;
    return min_mcost;
}

/* SATD of a block at a quarter-pel candidate (sum over its 4x4 sub-blocks) */
static int subpel_satd(const mbs *s, int bx4, int by4, int w4, int h4, int cmx, int cmy) {
    const jmo_ctx *c = s->c;
    int total = 0;
    for (int y4 = 0; y4 < h4; y4++)
        for (int x4 = 0; x4 < w4; x4++) {
            int32_t d[16];
            int ox = 4 * (bx4 + x4), oy = 4 * (by4 + y4);
            for (int y = 0; y < 4; y++)
                for (int x = 0; x < 4; x++)
                    d[4 * y + x] = s->org[(oy + y) * 16 + ox + x] -
                                   jmo_qpel_at(c, 4 * (s->pix_x + ox + x) + cmx, 4 * (s->pix_y + oy + y) + cmy);
            total += jmo_satd_block(d, c->cfg.use_hadamard);
        }
    return total;
}

/* SubPelBlockMotionSearch [J] with search_pos2 = search_pos4 = 9 */
static int subpel_search(mbs *s, int blocktype, int bx4, int by4, int pmvx, int pmvy, int *mvx,
                         int *mvy, int min_mcost) {
    jmo_ctx *c = s->c;
    int had = c->cfg.use_hadamard;
    int w4 = jmo_blc_size[blocktype][0] >> 2, h4 = jmo_blc_size[blocktype][1] >> 2;
    int check_position0 = (blocktype == 1 && *mvx == 0 && *mvy == 0 && had && s->slice_p && !s->rdo);
    int min_pos2 = had ? 0 : 1, max_pos2 = 9;
    int mx = *mvx * 4, my = *mvy * 4, best_pos = 0;
    for (int pos = min_pos2; pos < max_pos2; pos++) {          /* half-pel */
        int cx = mx + c->spiral_x[pos] * 2, cy = my + c->spiral_y[pos] * 2;
        int mcost = mv_cost(s, 0, cx, cy, pmvx, pmvy);
        if (check_position0 && pos == 0) mcost -= (s->lf * 16) >> 16;
        if (mcost >= min_mcost) continue;
        mcost += subpel_satd(s, bx4, by4, w4, h4, cx, cy);
        if (mcost < min_mcost) { min_mcost = mcost; best_pos = pos; }
    }
    if (best_pos) { mx += c->spiral_x[best_pos] * 2; my += c->spiral_y[best_pos] * 2; }
    best_pos = 0;
    for (int pos = 1; pos < 9; pos++) {                         /* quarter-pel */
        int cx = mx + c->spiral_x[pos], cy = my + c->spiral_y[pos];
        int mcost = mv_cost(s, 0, cx, cy, pmvx, pmvy);
        if (mcost >= min_mcost) continue;
        mcost += subpel_satd(s, bx4, by4, w4, h4, cx, cy);
        if (mcost < min_mcost) { min_mcost = mcost; best_pos = pos; }
    }
    if (best_pos) { mx += c->spiral_x[best_pos]; my += c->spiral_y[best_pos]; }
    *mvx = mx; *mvy = my;
    return min_mcost;
}

/* EPZSSubPelBlockMotionSearch [J] restated (EPZSSubPelME = 1, item 62): from the full-pel MV F, a
 * small diamond ((0,-1) (-1,0) (1,0) (0,1), strict '<' in that order, move to the best and repeat
 * until nothing improves) at half-pel steps inside F +- 2, then -- unless the cost is already below
 * EPZSSubPelThresScale x block pixels x pel_error -- at quarter-pel steps inside the half-pel
 * result +- 1.  Costs as SubPelBlockMotionSearch (item 8): MV cost + SATD (or SAD); with
 * UseHadamard the centre is first re-evaluated with SATD (the full-pel cost was SAD-based) */
static int epzs_subpel_search(mbs *s, int bt, int bx4, int by4, int pmvx, int pmvy, int *mvx, int *mvy, int min_mcost) {
    static const int dia[4][2] = {{0, -1}, {-1, 0}, {1, 0}, {0, 1}};
    jmo_ctx *c = s->c;
    const int w4 = jmo_blc_size[bt][0] >> 2, h4 = jmo_blc_size[bt][1] >> 2;
    const int subthres = c->cfg.epzs_subpel_thres_scale * 16 * w4 * h4 * ((c->maxv + 1) >> 8);
    int cx = *mvx * 4, cy = *mvy * 4;
    if (c->cfg.use_hadamard) {
        int m = mv_cost(s, 0, cx, cy, pmvx, pmvy) + subpel_satd(s, bx4, by4, w4, h4, cx, cy);
        if (m < min_mcost) min_mcost = m;
    }
    for (int stage = 0; stage < 2; stage++) {
        const int step = stage ? 1 : 2, ox = cx, oy = cy;
        if (stage && min_mcost < subthres) break;
        for (;;) {
            int moved = 0, nbx = cx, nby = cy;
            for (int k = 0; k < 4; k++) {
                int nx = cx + step * dia[k][0], ny = cy + step * dia[k][1];
                if (iabs(nx - ox) > step || iabs(ny - oy) > step) continue;   /* F +- 2, then +- 1 */
                int m = mv_cost(s, 0, nx, ny, pmvx, pmvy);
                if (m >= min_mcost) continue;
                m += subpel_satd(s, bx4, by4, w4, h4, nx, ny);
                if (m < min_mcost) { min_mcost = m; nbx = nx; nby = ny; moved = 1; }
            }
            if (!moved) break;
            cx = nbx; cy = nby;
        }
    }
    *mvx = cx; *mvy = cy;
    return min_mcost;
}

/* BlockMotionSearch [J] (list 0, ref 0) */
static int block_motion_search(mbs *s, int blocktype, int bx4, int by4, int range) {
    jmo_ctx *c = s->c;
    int bsx = jmo_blc_size[blocktype][0], bsy = jmo_blc_size[blocktype][1];
    int pmv[2];
    jmo_set_mvp(s, pmv, 0, bx4, by4, bsx, bsy);
    int mvx = iclip(-range, range, pmv[0] / 4), mvy = iclip(-range, range, pmv[1] / 4);
    int min_mcost;
    if (c->cfg.search_mode == 0) min_mcost = ffs_search(s, blocktype, bx4, by4, pmv[0], pmv[1], range, &mvx, &mvy);
    else if (c->cfg.search_mode == 3) min_mcost = epzs_search(s, blocktype, bx4, by4, pmv[0], pmv[1], range, &mvx, &mvy);
    else min_mcost = full_search(s, blocktype, bx4, by4, pmv[0], pmv[1], range, &mvx, &mvy);
    if (c->cfg.search_mode == 3) {               /* the neighbours' distortion of item 61 */
        uint16_t *fp = c->epzs_fp + (size_t)blocktype * (c->W >> 2) * (c->H >> 2);
        for (int y = 0; y < (bsy >> 2); y++)
            for (int x = 0; x < (bsx >> 2); x++)
                fp[((s->pix_y >> 2) + by4 + y) * (c->W >> 2) + (s->pix_x >> 2) + bx4 + x] = (uint16_t)(min_mcost < 65535 ? min_mcost : 65535);
    }
    if (c->cfg.use_hadamard) min_mcost = BIGCOST;
    if (c->cfg.search_mode == 3 && c->cfg.epzs_subpel_me)
        min_mcost = epzs_subpel_search(s, blocktype, bx4, by4, pmv[0], pmv[1], &mvx, &mvy, min_mcost);
    else min_mcost = subpel_search(s, blocktype, bx4, by4, pmv[0], pmv[1], &mvx, &mvy, min_mcost);
    for (int y = 0; y < (bsy >> 2); y++)
        for (int x = 0; x < (bsx >> 2); x++) {
            s->all_mv[blocktype][(by4 + y) * 4 + bx4 + x][0] = (int16_t)mvx;
            s->all_mv[blocktype][(by4 + y) * 4 + bx4 + x][1] = (int16_t)mvy;
            s->pmv[blocktype][(by4 + y) * 4 + bx4 + x][0] = (int16_t)pmv[0];   /* for the RD rate's mvd */
            s->pmv[blocktype][(by4 + y) * 4 + bx4 + x][1] = (int16_t)pmv[1];
        }
    return min_mcost;
}

/* the per-block seam (jmh_block_motion_search's oracle): BlockMotionSearch from explicit
 * arguments (MVP, centre, range, lambda_factor) on the pictures of jmo_search_pictures */
int jmo_search_pictures(jmo_ctx *c, const uint8_t *cur_y, const uint8_t *ref_y, int stride) {
    if (!c || !cur_y || !ref_y || stride < c->W) return JMH_E_INVALID_ARG;
    for (int y = 0; y < c->H; y++)
        for (int x = 0; x < c->W; x++) {
            c->orgY[(size_t)y * c->W + x] = cur_y[(size_t)y * stride + x];
            c->refY[(size_t)y * c->W + x] = ref_y[(size_t)y * stride + x];
        }
    jmo_build_qpel(c);
    c->have_ref = 1;
    return JMH_OK;
}

int jmo_block_motion_search(jmo_ctx *c, int n, const jmh_block_search *req, jmh_block_result *res) {
    if (!c || n <= 0 || !req || !res) return JMH_E_INVALID_ARG;
    for (int i = 0; i < n; i++) {
        const jmh_block_search *q = &req[i];
        if (q->blocktype < 1 || q->blocktype > 7 || q->search_range < 0 || q->search_range > c->sr) return JMH_E_INVALID_ARG;
        if (q->search_mode != 0 && q->search_mode != -1) return JMH_E_UNSUPPORTED_CFG;
        mbs S;
        mbs *s = &S;
        memset(s, 0, sizeof(*s));
        s->c = c; s->mbx = q->mb_x; s->mby = q->mb_y; s->pix_x = 16 * q->mb_x; s->pix_y = 16 * q->mb_y;
        s->lf = q->lambda_factor;
        s->slice_p = q->slice_p != 0;
        for (int y = 0; y < 16; y++) memcpy(s->org + 16 * y, c->orgY + (s->pix_y + y) * c->W + s->pix_x, 16 * sizeof(pel));
        int mvx = q->centre[0], mvy = q->centre[1], min_mcost;
        if (q->search_mode == 0) {
            ffs_setup_at(s, q->centre[0], q->centre[1]);
            min_mcost = ffs_search(s, q->blocktype, q->block_x, q->block_y, q->pred_mv[0], q->pred_mv[1], q->search_range, &mvx, &mvy);
        } else
            min_mcost = full_search(s, q->blocktype, q->block_x, q->block_y, q->pred_mv[0], q->pred_mv[1], q->search_range, &mvx, &mvy);
        res[i].fullpel_mv[0] = mvx; res[i].fullpel_mv[1] = mvy; res[i].fullpel_cost = min_mcost;
        if (c->cfg.use_hadamard) min_mcost = BIGCOST;
        min_mcost = subpel_search(s, q->blocktype, q->block_x, q->block_y, q->pred_mv[0], q->pred_mv[1], &mvx, &mvy, min_mcost);
        res[i].mv[0] = mvx; res[i].mv[1] = mvy; res[i].min_mcost = min_mcost;
    }
    return JMH_OK;
}

void jmo_write_enc_mv(mbs *s, int bx4, int by4, int w4, int h4, const int16_t (*mv)[2]) {
    jmo_ctx *c = s->c;
    int W4 = c->W >> 2;
    for (int y = 0; y < h4; y++)
        for (int x = 0; x < w4; x++) {
            int k = (by4 + y) * 4 + bx4 + x;
            int a = ((s->pix_y >> 2) + by4 + y) * W4 + (s->pix_x >> 2) + bx4 + x;
            c->mv[2 * a] = mv[k][0];
            c->mv[2 * a + 1] = mv[k][1];
            c->refidx[a] = 0;
        }
}

/* PartitionMotionSearch [J] (list 0, single reference) */
void jmo_partition_motion_search(mbs *s, int blocktype, int block8x8) {
    static const int bx0[5][4] = {{0, 0, 0, 0}, {0, 0, 0, 0}, {0, 0, 0, 0}, {0, 2, 0, 0}, {0, 2, 0, 2}};
    static const int by0[5][4] = {{0, 0, 0, 0}, {0, 0, 0, 0}, {0, 2, 0, 0}, {0, 0, 0, 0}, {0, 0, 2, 2}};
    int parttype = blocktype < 4 ? blocktype : 4;
    int step_h0 = jmo_blc_size[parttype][0] >> 2, step_v0 = jmo_blc_size[parttype][1] >> 2;
    int step_h = jmo_blc_size[blocktype][0] >> 2, step_v = jmo_blc_size[blocktype][1] >> 2;
    int range = block_range(s, blocktype);
    s->motion_cost[blocktype][block8x8] = 0;
    for (int v = by0[parttype][block8x8]; v < by0[parttype][block8x8] + step_v0; v += step_v)
        for (int h = bx0[parttype][block8x8]; h < bx0[parttype][block8x8] + step_h0; h += step_h) {
            s->motion_cost[blocktype][block8x8] += block_motion_search(s, blocktype, h, v, range);
            jmo_write_enc_mv(s, h, v, step_h, step_v, s->all_mv[blocktype]);
        }
}

/* ====================================================================================== */
/*  transform / quantisation                                                               */
/* ====================================================================================== */
/* dct_luma [J]: 4x4 forward, quant (deadzone qp_const), scan, dequant, inverse, recon */
int jmo_dct_luma4x4(const int32_t resid[16], const pel *pred, int ps, int qp, int intra_round,
                       int16_t levels[16], int *coeff_cost, pel *rec, int rs, int maxv) {
    int qp_per = qp / 6, qp_rem = qp % 6, q_bits = Q_BITS + qp_per;
    int qp_const = jmo_qround(intra_round, q_bits);
    int32_t m[16];
    memcpy(m, resid, sizeof(m));
    jmo_fwd4x4(m);
    int run = -1, nonzero = 0;
    for (int k = 0; k < 16; k++) {
        int pos = jmo_scan4x4[k];
        run++;
        int level = (iabs(m[pos]) * jmo_quant_coef[qp_rem][pos] + qp_const) >> q_bits;
        int ilev = 0;
        if (level != 0) {
            nonzero = 1;
            *coeff_cost += level > 1 ? MAX_VALUE : jmo_coeff_cost_tab[run];
            levels[k] = (int16_t)isign(level, m[pos]);
            run = -1;
            ilev = level * jmo_dequant_coef[qp_rem][pos] << qp_per;
        } else levels[k] = 0;
        m[pos] = isign(ilev, m[pos]);
    }
    jmo_inv4x4_add(m, pred, ps, rec, rs, maxv);
    return nonzero;
}

int jmo_tq4x4_batch(int n, const int16_t *resid, const uint8_t *pred, int qp, int intra,
                    int16_t *levels, uint8_t *recon, int32_t *coeff_cost, int32_t *nonzero) {
    if (n < 0 || qp < 0 || qp > 51 || intra < 0 || intra > JMO_RND_OFF(JMH_QOFFSET_MAX)) return JMH_E_INVALID_ARG;
    for (int i = 0; i < n; i++) {
        int32_t r[16];
        int cc = 0;
        pel p[16], o[16];
        for (int k = 0; k < 16; k++) { r[k] = resid[16 * i + k]; p[k] = pred[16 * i + k]; }
        nonzero[i] = jmo_dct_luma4x4(r, p, 4, qp, intra, levels + 16 * i, &cc, o, 4, 255);
        for (int k = 0; k < 16; k++) recon[16 * i + k] = (pel)o[k];
        coeff_cost[i] = cc;
    }
    return JMH_OK;
}

/* dct_luma8x8 [J] (JM FRExt block.c; forward8x8 + quant + dequant + inverse8x8): 8x8 core
 * transform, level = (|c|*quant_coef8 + qp_const) >> (16 + qp/6) with qp_const by slice type as
 * for 4x4 (docs/JM_SEMANTICS.md item 1), 8x8 frame zig-zag, COEFF_COST8x8 on the 64-scan runs,
 * dequantisation by the normative 8.5.13.1 formula on the signed level (flat scaling lists),
 * reconstruction clip((r + (pred<<6) + 32) >> 6).  levels[64] in scan order. */
int jmo_dct_luma8x8(const int32_t resid[64], const pel *pred, int ps, int qp, int intra_round,
                       int16_t levels[64], int *coeff_cost, pel *rec, int rs, int maxv) {
    int qp_per = qp / 6, qp_rem = qp % 6, q_bits = Q_BITS_8 + qp_per;
    int qp_const = jmo_qround(intra_round, q_bits);
    int scan[64];
    jmo_scan8x8(scan);
    int32_t m[64];
    memcpy(m, resid, sizeof(m));
    jmo_fwd8x8(m);
    int run = -1, nonzero = 0;
    for (int k = 0; k < 64; k++) {
        int pos = scan[k], cls = jmo_class8(pos & 7, pos >> 3);
        run++;
        int level = (iabs(m[pos]) * jmo_quant8_cls[qp_rem][cls] + qp_const) >> q_bits;
        int c = isign(level, m[pos]), d = 0;
        if (level != 0) {
            nonzero = 1;
            *coeff_cost += level > 1 ? MAX_VALUE : jmo_coeff_cost8(run);
            run = -1;
            int ls = 16 * jmo_dequant8_cls[qp_rem][cls];        /* LevelScale8x8, flat weights */
            d = qp >= 36 ? c * ls * (1 << (qp_per - 6)) : (c * ls + (1 << (5 - qp_per))) >> (6 - qp_per);
        }
        levels[k] = (int16_t)c;
        m[pos] = d;
    }
    jmo_inv8x8_add(m, pred, ps, rec, rs, maxv);
    return nonzero;
}

int jmo_tq8x8_batch(int n, const int16_t *resid, const uint8_t *pred, int qp, int intra,
                    int16_t *levels, uint8_t *recon, int32_t *coeff_cost, int32_t *nonzero) {
    if (n < 0 || qp < 0 || qp > 51 || intra < 0 || intra > JMO_RND_OFF(JMH_QOFFSET_MAX)) return JMH_E_INVALID_ARG;
    for (int i = 0; i < n; i++) {
        int32_t r[64];
        int cc = 0;
        pel p[64], o[64];
        for (int k = 0; k < 64; k++) { r[k] = resid[64 * i + k]; p[k] = pred[64 * i + k]; }
        nonzero[i] = jmo_dct_luma8x8(r, p, 8, qp, intra, levels + 64 * i, &cc, o, 8, 255);
        for (int k = 0; k < 64; k++) recon[64 * i + k] = (pel)o[k];
        coeff_cost[i] = cc;
    }
    return JMH_OK;
}
void jmo_forward8x8(const int32_t *in, int32_t *out) {
    memcpy(out, in, 64 * sizeof(int32_t));
    jmo_fwd8x8(out);
}

/* store an 8x8 block's scan-order levels as CAVLC's four interleaved 4x4 blocks (7.3.5.3.2) */
void jmo_put_levels8(int16_t luma[16][16], int b8, const int16_t lev[64]) {
    for (int j = 0; j < 4; j++) {
        int blk = (2 * (b8 >> 1) + (j >> 1)) * 4 + 2 * (b8 & 1) + (j & 1);
        for (int k = 0; k < 16; k++) luma[blk][k] = lev[4 * k + j];
    }
}

/* dct_chroma [J] for one component: 4 4x4 AC blocks + 2x2 DC; returns updated cr_cbp.
 * resid/pred raster 8x8.  DC reconstruction follows H.264 8.5.11.2 exactly. */
int jmo_dct_chroma(const int32_t resid[64], const pel pred[64], int qpc, int intra_round,
                      int cr_cbp, int16_t dc_out[4], int16_t ac_out[4][16], pel rec[64], int maxv) {
    int qp_per = qpc / 6, qp_rem = qpc % 6, q_bits = Q_BITS + qp_per;
    int qp_const = jmo_qround(intra_round, q_bits);
    int32_t m[4][16];
    for (int b = 0; b < 4; b++) {
        int ox = (b & 1) * 4, oy = (b >> 1) * 4;
        for (int y = 0; y < 4; y++)
            for (int x = 0; x < 4; x++) m[b][4 * y + x] = resid[(oy + y) * 8 + ox + x];
        jmo_fwd4x4(m[b]);
    }
    int m1[4] = {m[0][0] + m[1][0] + m[2][0] + m[3][0], m[0][0] - m[1][0] + m[2][0] - m[3][0],
                 m[0][0] + m[1][0] - m[2][0] - m[3][0], m[0][0] - m[1][0] - m[2][0] + m[3][0]};
    int dccoded = 0;
    for (int k = 0; k < 4; k++) {
        int level = (iabs(m1[k]) * jmo_quant_coef[qp_rem][0] + 2 * qp_const) >> (q_bits + 1);
        if (level != 0) { cr_cbp = imax(1, cr_cbp); dccoded = 1; }
        dc_out[k] = (int16_t)isign(level, m1[k]);
    }
    (void)dccoded;
    /* inverse 2x2 Hadamard of the levels and scaling (8.5.11.2): dcC = ((f*16v) << per) >> 5 */
    int c0 = dc_out[0], c1 = dc_out[1], c2 = dc_out[2], c3 = dc_out[3];
    int f[4] = {c0 + c1 + c2 + c3, c0 - c1 + c2 - c3, c0 + c1 - c2 - c3, c0 - c1 - c2 + c3};
    int v00 = jmo_dequant_coef[qp_rem][0];
    int coeff_cost = 0, ac_any = 0;
    for (int b = 0; b < 4; b++) {
        int run = -1;
        ac_out[b][0] = 0;
        for (int k = 1; k < 16; k++) {
            int pos = jmo_scan4x4[k];
            run++;
            int level = (iabs(m[b][pos]) * jmo_quant_coef[qp_rem][pos] + qp_const) >> q_bits;
            int ilev = 0;
            if (level != 0) {
                coeff_cost += level > 1 ? MAX_VALUE : jmo_coeff_cost_tab[run];
                ac_any = 1;
                run = -1;
                ilev = level * jmo_dequant_coef[qp_rem][pos] << qp_per;
            }
            ac_out[b][k] = (int16_t)isign(level, m[b][pos]);
            m[b][pos] = isign(ilev, m[b][pos]);
        }
    }
    if (coeff_cost < CHROMA_COEFF_COST) {                 /* reset chroma AC coeffs [J] */
        ac_any = 0;
        for (int b = 0; b < 4; b++)
            for (int k = 1; k < 16; k++) { ac_out[b][k] = 0; m[b][jmo_scan4x4[k]] = 0; }
    }
    if (ac_any) cr_cbp = 2;
    for (int b = 0; b < 4; b++) {
        m[b][0] = (f[b] * 16 * v00 * (1 << qp_per)) >> 5;   /* (x << per) of the spec: x * 2^per (x may be < 0) */
        int ox = (b & 1) * 4, oy = (b >> 1) * 4;
        jmo_inv4x4_add(m[b], pred + oy * 8 + ox, 8, rec + oy * 8 + ox, 8, maxv);
    }
    return cr_cbp;
}

/* dct_luma_16x16 [J]: returns luma cbp (15 if any AC level, else 0) */
int jmo_dct_luma_16x16(const int32_t resid[256], const pel pred[256], int qp, int rnd,
                          int16_t dc_out[16], int16_t ac_out[16][16], int *cbp_blk, pel rec[256], int maxv) {
    int qp_per = qp / 6, qp_rem = qp % 6, q_bits = Q_BITS + qp_per;
    int qp_const = jmo_qround(rnd, q_bits), qp_const2 = qp_const << 1;   /* JM 8.6: always / 3 */
    int32_t m[16][16];                     /* [4x4 block raster][coef raster] */
    for (int b = 0; b < 16; b++) {
        int ox = (b & 3) * 4, oy = (b >> 2) * 4;
        for (int y = 0; y < 4; y++)
            for (int x = 0; x < 4; x++) m[b][4 * y + x] = resid[(oy + y) * 16 + ox + x];
        jmo_fwd4x4(m[b]);
    }
    int32_t dc[16];                        /* DC matrix raster: [by*4+bx] */
    for (int b = 0; b < 16; b++) dc[b] = m[b][0];
    /* forward Hadamard, rows then columns with >>1 */
    for (int y = 0; y < 4; y++) {
        int32_t *r = dc + 4 * y;
        int a0 = r[0] + r[3], a3 = r[0] - r[3], a1 = r[1] + r[2], a2 = r[1] - r[2];
        r[0] = a0 + a1; r[2] = a0 - a1; r[1] = a3 + a2; r[3] = a3 - a2;
    }
    for (int x = 0; x < 4; x++) {
        int a0 = dc[x] + dc[12 + x], a3 = dc[x] - dc[12 + x];
        int a1 = dc[4 + x] + dc[8 + x], a2 = dc[4 + x] - dc[8 + x];
        dc[x] = (a0 + a1) >> 1; dc[8 + x] = (a0 - a1) >> 1;
        dc[4 + x] = (a3 + a2) >> 1; dc[12 + x] = (a3 - a2) >> 1;
    }
    int32_t lev[16];
    for (int k = 0; k < 16; k++) {
        int pos = jmo_scan4x4[k];
        int level = (iabs(dc[pos]) * jmo_quant_coef[qp_rem][0] + qp_const2) >> (q_bits + 1);
        dc_out[k] = (int16_t)isign(level, dc[pos]);
        lev[pos] = dc_out[k];
    }
    /* inverse Hadamard (8.5.10) + scaling ((f*v << per) + 2) >> 2 */
    int32_t t[16], f[16];
    for (int y = 0; y < 4; y++) {
        const int32_t *c = lev + 4 * y;
        int e0 = c[0] + c[2], e1 = c[0] - c[2], e2 = c[1] - c[3], e3 = c[1] + c[3];
        t[4 * y + 0] = e0 + e3; t[4 * y + 3] = e0 - e3; t[4 * y + 1] = e1 + e2; t[4 * y + 2] = e1 - e2;
    }
    for (int x = 0; x < 4; x++) {
        int e0 = t[x] + t[8 + x], e1 = t[x] - t[8 + x], e2 = t[4 + x] - t[12 + x], e3 = t[4 + x] + t[12 + x];
        f[x] = e0 + e3; f[12 + x] = e0 - e3; f[4 + x] = e1 + e2; f[8 + x] = e1 - e2;
    }
    int v00 = jmo_dequant_coef[qp_rem][0];
    int ac = 0;
    for (int b = 0; b < 16; b++) {
        int run = -1, nz = 0;
        (void)run;
        ac_out[b][0] = 0;
        for (int k = 1; k < 16; k++) {
            int pos = jmo_scan4x4[k];
            int level = (iabs(m[b][pos]) * jmo_quant_coef[qp_rem][pos] + qp_const) >> q_bits;
            if (level) { ac = 15; nz = 1; }
            ac_out[b][k] = (int16_t)isign(level, m[b][pos]);
            m[b][pos] = isign(level * jmo_dequant_coef[qp_rem][pos] << qp_per, m[b][pos]);
        }
        if (nz) *cbp_blk |= 1 << b;
        m[b][0] = (f[b] * v00 * (1 << qp_per) + 2) >> 2;
        int ox = (b & 3) * 4, oy = (b >> 2) * 4;
        jmo_inv4x4_add(m[b], pred + oy * 16 + ox, 16, rec + oy * 16 + ox, 16, maxv);
    }
    return ac;
}

/* ====================================================================================== */
/*  intra prediction (H.264 8.3)                                                            */
/* ====================================================================================== */
int jmo_mb_avail(const mbs *s, int dmx, int dmy) {
    int mx = s->mbx + dmx, my = s->mby + dmy;
    return mx >= 0 && my >= 0 && mx < s->c->mbw && my < s->c->mbh &&
           (my < s->mby || (my == s->mby && mx < s->mbx)) &&
           jmo_same_slice(s->c, s->mby * s->c->mbw + s->mbx, my * s->c->mbw + mx);
}
/* availability of a neighbour MB's samples for intra prediction: with UseConstrainedIntraPred
 * (constrained_intra_pred_flag, 8.3.1.2 / 8.3.2.2 / 8.3.3 / 8.3.4) an inter-coded neighbour's
 * samples are "not available for Intra prediction" */
static int intra_avail(const mbs *s, int dmx, int dmy) {
    return jmo_mb_avail(s, dmx, dmy) && (!s->c->cfg.constrained_intra_pred || s->c->mbintra[(s->mby + dmy) * s->c->mbw + s->mbx + dmx]);
}
/* luma sample availability at MB-relative (x,y) for intra prediction */
static int luma_avail(const mbs *s, int x, int y) {
    if (y > 15) return 0;
    if (x < 0) return intra_avail(s, -1, y < 0 ? -1 : 0);
    if (x <= 15) return y < 0 ? intra_avail(s, 0, -1) : 1;
    return y < 0 ? intra_avail(s, 1, -1) : 0;
}

/* intrapred_luma [J] / 8.3.1.2: the 9 Intra4x4 predictions of the 4x4 block at (bx,by)
 * (pixels, MB relative); pred[9][16]; avail[9] */
void jmo_intra4x4_pred(const mbs *s, int bx, int by, pel pred[9][16], int avail[9]) {
    const jmo_ctx *c = s->c;
    const pel *R = c->recY;
    int W = c->W, ax = s->pix_x + bx, ay = s->pix_y + by;
    int up = luma_avail(s, bx, by - 1), left = luma_avail(s, bx - 1, by);
    int ul = luma_avail(s, bx - 1, by - 1);
    int ur = luma_avail(s, bx + 4, by - 1) && !((bx == 4 || bx == 12) && (by == 4 || by == 12));
    int T[9], L[4];                      /* T[0] = p[-1,-1], T[1+x] = p[x,-1] */
    T[0] = ul ? R[(ay - 1) * W + ax - 1] : 0;
    for (int x = 0; x < 4; x++) T[1 + x] = up ? R[(ay - 1) * W + ax + x] : 0;
    for (int x = 4; x < 8; x++) T[1 + x] = up ? (ur ? R[(ay - 1) * W + ax + x] : T[4]) : 0;
    for (int y = 0; y < 4; y++) L[y] = left ? R[(ay + y) * W + ax - 1] : 0;
#define PT(x) T[1 + (x)]
#define PL(y) ((y) < 0 ? T[0] : L[y])
    int all = up && left && ul;
    for (int m = 0; m < 9; m++) avail[m] = 0;
    avail[2] = 1;
    avail[0] = avail[3] = avail[7] = up;
    avail[1] = avail[8] = left;
    avail[4] = avail[5] = avail[6] = all;
    for (int y = 0; y < 4; y++)
        for (int x = 0; x < 4; x++) {
            int k = 4 * y + x;
            pred[0][k] = (pel)PT(x);
            pred[1][k] = (pel)L[y];
            /* DDL */
            pred[3][k] = (pel)((x == 3 && y == 3) ? (PT(6) + 3 * PT(7) + 2) >> 2
                                                      : (PT(x + y) + 2 * PT(x + y + 1) + PT(x + y + 2) + 2) >> 2);
            /* DDR */
            if (x > y) pred[4][k] = (pel)((PT(x - y - 2) + 2 * PT(x - y - 1) + PT(x - y) + 2) >> 2);
            else if (x < y) pred[4][k] = (pel)((PL(y - x - 2) + 2 * PL(y - x - 1) + PL(y - x) + 2) >> 2);
            else pred[4][k] = (pel)((PT(0) + 2 * T[0] + PL(0) + 2) >> 2);
            /* VR */
            {
                int z = 2 * x - y, v;
                if (z >= 0 && !(z & 1)) v = (PT(x - (y >> 1) - 1) + PT(x - (y >> 1)) + 1) >> 1;
                else if (z >= 0) v = (PT(x - (y >> 1) - 2) + 2 * PT(x - (y >> 1) - 1) + PT(x - (y >> 1)) + 2) >> 2;
                else if (z == -1) v = (PL(0) + 2 * T[0] + PT(0) + 2) >> 2;
                else v = (PL(y - 1) + 2 * PL(y - 2) + PL(y - 3) + 2) >> 2;
                pred[5][k] = (pel)v;
            }
            /* HD */
            {
                int z = 2 * y - x, v;
                if (z >= 0 && !(z & 1)) v = (PL(y - (x >> 1) - 1) + PL(y - (x >> 1)) + 1) >> 1;
                else if (z >= 0) v = (PL(y - (x >> 1) - 2) + 2 * PL(y - (x >> 1) - 1) + PL(y - (x >> 1)) + 2) >> 2;
                else if (z == -1) v = (PL(0) + 2 * T[0] + PT(0) + 2) >> 2;
                else v = (PT(x - 1) + 2 * PT(x - 2) + PT(x - 3) + 2) >> 2;
                pred[6][k] = (pel)v;
            }
            /* VL */
            if (!(y & 1)) pred[7][k] = (pel)((PT(x + (y >> 1)) + PT(x + (y >> 1) + 1) + 1) >> 1);
            else pred[7][k] = (pel)((PT(x + (y >> 1)) + 2 * PT(x + (y >> 1) + 1) + PT(x + (y >> 1) + 2) + 2) >> 2);
            /* HU */
            {
                int z = x + 2 * y, v;
                if (z > 5) v = L[3];
                else if (z == 5) v = (L[2] + 3 * L[3] + 2) >> 2;
                else if (!(z & 1)) v = (L[y + (x >> 1)] + L[y + (x >> 1) + 1] + 1) >> 1;
                else v = (L[y + (x >> 1)] + 2 * L[y + (x >> 1) + 1] + L[y + (x >> 1) + 2] + 2) >> 2;
                pred[8][k] = (pel)v;
            }
        }
    /* DC */
    int dcv;
    if (up && left) dcv = (PT(0) + PT(1) + PT(2) + PT(3) + L[0] + L[1] + L[2] + L[3] + 4) >> 3;
    else if (left) dcv = (L[0] + L[1] + L[2] + L[3] + 2) >> 2;
    else if (up) dcv = (PT(0) + PT(1) + PT(2) + PT(3) + 2) >> 2;
    else dcv = (c->maxv + 1) >> 1;
    for (int k = 0; k < 16; k++) pred[2][k] = (pel)dcv;
#undef PT
#undef PL
}

/* Intra8x8 prediction (8.3.2.2, JM FRExt intrapred_luma8x8 [J]): reference sample filtering
 * (8.3.2.2.1) then the nine modes.  See jm_oracle.h for nb[] / avail. */
int jmo_intra8x8_pred(const int32_t nb[25], int avail, uint8_t pred[9][64]) {
    pel p[9][64];
    int ok = jmo_intra8x8_pred_px(nb, avail, p, 128);
    for (int m = 0; m < 9; m++)
        for (int k = 0; k < 64; k++) pred[m][k] = (uint8_t)p[m][k];
    return ok;
}
int jmo_intra8x8_pred_px(const int32_t nb[25], int avail, pel pred[9][64], int dc) {
    int left = avail & 1, up = (avail >> 1) & 1, ur = (avail >> 2) & 1, ul = (avail >> 3) & 1;
    int p[16], q[8], c = nb[0];                    /* raw top row (x = 0..15), left column, corner */
    for (int x = 0; x < 16; x++) p[x] = x < 8 || ur ? nb[1 + x] : nb[8];   /* substitution p[7,-1] */
    for (int y = 0; y < 8; y++) q[y] = nb[17 + y];
    int T[16] = {0}, L[8] = {0}, Q = c;                /* filtered p'[x,-1], p'[-1,y], p'[-1,-1] */
    if (up) {
        T[0] = ul ? (c + 2 * p[0] + p[1] + 2) >> 2 : (3 * p[0] + p[1] + 2) >> 2;
        for (int x = 1; x < 15; x++) T[x] = (p[x - 1] + 2 * p[x] + p[x + 1] + 2) >> 2;
        T[15] = (p[14] + 3 * p[15] + 2) >> 2;
    }
    if (ul) {
        if (up && left) Q = (p[0] + 2 * c + q[0] + 2) >> 2;
        else if (up) Q = (3 * c + p[0] + 2) >> 2;
        else if (left) Q = (3 * c + q[0] + 2) >> 2;
    }
    if (left) {
        L[0] = ul ? (c + 2 * q[0] + q[1] + 2) >> 2 : (3 * q[0] + q[1] + 2) >> 2;
        for (int y = 1; y < 7; y++) L[y] = (q[y - 1] + 2 * q[y] + q[y + 1] + 2) >> 2;
        L[7] = (q[6] + 3 * q[7] + 2) >> 2;
    }
#define PT(i) ((i) < 0 ? Q : T[i])
#define PL(j) ((j) < 0 ? Q : L[j])
    int dcv = dc, st = 0, sl = 0;
    for (int i = 0; i < 8; i++) { st += up ? T[i] : 0; sl += left ? L[i] : 0; }
    if (up && left) dcv = (st + sl + 8) >> 4;
    else if (up) dcv = (st + 4) >> 3;
    else if (left) dcv = (sl + 4) >> 3;
    int ok = (1 << 2) | (up ? (1 << 0) | (1 << 3) | (1 << 7) : 0) | (left ? (1 << 1) | (1 << 8) : 0) |
             (up && left && ul ? (1 << 4) | (1 << 5) | (1 << 6) : 0);
    for (int y = 0; y < 8; y++)
        for (int x = 0; x < 8; x++) {
            int k = 8 * y + x, v;
            pred[2][k] = (pel)dcv;
            if (up) {
                pred[0][k] = (pel)T[x];
                pred[3][k] = (pel)(x == 7 && y == 7 ? (T[14] + 3 * T[15] + 2) >> 2
                                                       : (T[x + y] + 2 * T[x + y + 1] + T[x + y + 2] + 2) >> 2);
                pred[7][k] = (pel)(!(y & 1) ? (T[x + (y >> 1)] + T[x + (y >> 1) + 1] + 1) >> 1
                                                : (T[x + (y >> 1)] + 2 * T[x + (y >> 1) + 1] + T[x + (y >> 1) + 2] + 2) >> 2);
            }
            if (left) {
                pred[1][k] = (pel)L[y];
                int z = x + 2 * y;
                if (z > 13) v = L[7];
                else if (z == 13) v = (L[6] + 3 * L[7] + 2) >> 2;
                else if (!(z & 1)) v = (L[y + (x >> 1)] + L[y + (x >> 1) + 1] + 1) >> 1;
                else v = (L[y + (x >> 1)] + 2 * L[y + (x >> 1) + 1] + L[y + (x >> 1) + 2] + 2) >> 2;
                pred[8][k] = (pel)v;
            }
            if (up && left && ul) {
                if (x > y) v = (PT(x - y - 2) + 2 * PT(x - y - 1) + PT(x - y) + 2) >> 2;
                else if (x < y) v = (PL(y - x - 2) + 2 * PL(y - x - 1) + PL(y - x) + 2) >> 2;
                else v = (PT(0) + 2 * Q + PL(0) + 2) >> 2;
                pred[4][k] = (pel)v;
                int z = 2 * x - y;
                if (z >= 0 && !(z & 1)) v = (PT(x - (y >> 1) - 1) + PT(x - (y >> 1)) + 1) >> 1;
                else if (z >= 0) v = (PT(x - (y >> 1) - 2) + 2 * PT(x - (y >> 1) - 1) + PT(x - (y >> 1)) + 2) >> 2;
                else if (z == -1) v = (PL(0) + 2 * Q + PT(0) + 2) >> 2;
                else v = (PL(y - 2 * x - 1) + 2 * PL(y - 2 * x - 2) + PL(y - 2 * x - 3) + 2) >> 2;
                pred[5][k] = (pel)v;
                z = 2 * y - x;
                if (z >= 0 && !(z & 1)) v = (PL(y - (x >> 1) - 1) + PL(y - (x >> 1)) + 1) >> 1;
                else if (z >= 0) v = (PL(y - (x >> 1) - 2) + 2 * PL(y - (x >> 1) - 1) + PL(y - (x >> 1)) + 2) >> 2;
                else if (z == -1) v = (PL(0) + 2 * Q + PT(0) + 2) >> 2;
                else v = (PT(x - 2 * y - 1) + 2 * PT(x - 2 * y - 2) + PT(x - 2 * y - 3) + 2) >> 2;
                pred[6][k] = (pel)v;
            }
        }
#undef PT
#undef PL
    return ok;
}

/* intrapred_luma_16x16 [J] / 8.3.3 */
void jmo_intra16_pred(const mbs *s, pel pred[4][256], int avail[4]) {
    const jmo_ctx *c = s->c;
    const pel *R = c->recY;
    int W = c->W, ax = s->pix_x, ay = s->pix_y;
    int up = intra_avail(s, 0, -1), left = intra_avail(s, -1, 0), ul = intra_avail(s, -1, -1);
    int T[16], L[16], P = ul ? R[(ay - 1) * W + ax - 1] : 0;
    for (int i = 0; i < 16; i++) {
        T[i] = up ? R[(ay - 1) * W + ax + i] : 0;
        L[i] = left ? R[(ay + i) * W + ax - 1] : 0;
    }
    avail[0] = up; avail[1] = left; avail[2] = 1; avail[3] = up && left && ul;
    int st = 0, sl = 0;
    for (int i = 0; i < 16; i++) { st += T[i]; sl += L[i]; }
    int dcv = (up && left) ? (st + sl + 16) >> 5 : up ? (st + 8) >> 4 : left ? (sl + 8) >> 4 : (c->maxv + 1) >> 1;
    int ih = 0, iv = 0;
    for (int i = 1; i <= 8; i++) {
        ih += i * (T[7 + i] - (7 - i >= 0 ? T[7 - i] : P));
        iv += i * (L[7 + i] - (7 - i >= 0 ? L[7 - i] : P));
    }
    int ib = (5 * ih + 32) >> 6, ic = (5 * iv + 32) >> 6, iaa = 16 * (L[15] + T[15]);
    for (int y = 0; y < 16; y++)
        for (int x = 0; x < 16; x++) {
            int k = 16 * y + x;
            pred[0][k] = (pel)T[x];
            pred[1][k] = (pel)L[y];
            pred[2][k] = (pel)dcv;
            pred[3][k] = (pel)clipv(c->maxv, (iaa + (x - 7) * ib + (y - 7) * ic + 16) >> 5);
        }
}

/* IntraChromaPrediction8x8 [J] / 8.3.4 for one component; pred[4][64] */
void jmo_intra_chroma_pred(const mbs *s, int uv, pel pred[4][64], int avail[4]) {
    const jmo_ctx *c = s->c;
    const pel *R = uv ? c->recV : c->recU;
    const int dc = (c->maxv + 1) >> 1;
    int W = c->Wc, ax = s->pix_x >> 1, ay = s->pix_y >> 1;
    int up = intra_avail(s, 0, -1), left = intra_avail(s, -1, 0), ul = intra_avail(s, -1, -1);
    int T[8], L[8], P = ul ? R[(ay - 1) * W + ax - 1] : 0;
    for (int i = 0; i < 8; i++) {
        T[i] = up ? R[(ay - 1) * W + ax + i] : 0;
        L[i] = left ? R[(ay + i) * W + ax - 1] : 0;
    }
    avail[0] = 1; avail[1] = left; avail[2] = up; avail[3] = up && left && ul;
    for (int b = 0; b < 4; b++) {          /* DC per 4x4 chroma block (8.3.4.1-3) */
        int xo = (b & 1) * 4, yo = (b >> 1) * 4;
        int s0 = 0, s1 = 0, s2 = 0, s3 = 0, sv = dc;
        for (int i = 0; i < 4; i++) { s0 += T[i]; s1 += T[4 + i]; s2 += L[i]; s3 += L[4 + i]; }
        if (b == 0) sv = (up && left) ? (s0 + s2 + 4) >> 3 : up ? (s0 + 2) >> 2 : left ? (s2 + 2) >> 2 : dc;
        else if (b == 1) sv = up ? (s1 + 2) >> 2 : left ? (s2 + 2) >> 2 : dc;
        else if (b == 2) sv = left ? (s3 + 2) >> 2 : up ? (s0 + 2) >> 2 : dc;
        else sv = (up && left) ? (s1 + s3 + 4) >> 3 : up ? (s1 + 2) >> 2 : left ? (s3 + 2) >> 2 : dc;
        for (int y = 0; y < 4; y++)
            for (int x = 0; x < 4; x++) pred[0][(yo + y) * 8 + xo + x] = (pel)sv;
    }
    int ih = 0, iv = 0;
    for (int i = 1; i <= 4; i++) {
        ih += i * (T[3 + i] - (3 - i >= 0 ? T[3 - i] : P));
        iv += i * (L[3 + i] - (3 - i >= 0 ? L[3 - i] : P));
    }
    int ib = (34 * ih + 32) >> 6, ic = (34 * iv + 32) >> 6, iaa = 16 * (L[7] + T[7]);
    for (int y = 0; y < 8; y++)
        for (int x = 0; x < 8; x++) {
            pred[1][y * 8 + x] = (pel)L[y];
            pred[2][y * 8 + x] = (pel)T[x];
            pred[3][y * 8 + x] = (pel)clipv(c->maxv, (iaa + (x - 3) * ib + (y - 3) * ic + 16) >> 5);
        }
}

/* find_sad_16x16 [J]: Hadamard cost of the 4 Intra16x16 predictions */
int jmo_find_sad_16x16(const mbs *s, pel pred[4][256], const int avail[4], int *mode) {
    int best = MAX_VALUE;
    *mode = 2;
    for (int k = 0; k < 4; k++) {
        if (!avail[k]) continue;
        int cost = 0, dc[16];
        for (int b = 0; b < 16; b++) {
            int ox = (b & 3) * 4, oy = (b >> 2) * 4;
            int m[16], t[16];
            for (int y = 0; y < 4; y++)
                for (int x = 0; x < 4; x++)
                    m[4 * y + x] = s->org[(oy + y) * 16 + ox + x] - pred[k][(oy + y) * 16 + ox + x];
            for (int y = 0; y < 4; y++) {
                int *r = m + 4 * y;
                int a0 = r[0] + r[3], a1 = r[1] + r[2], a2 = r[1] - r[2], a3 = r[0] - r[3];
                t[4 * y + 0] = a0 + a1; t[4 * y + 2] = a0 - a1; t[4 * y + 1] = a2 + a3; t[4 * y + 3] = a3 - a2;
            }
            for (int x = 0; x < 4; x++) {
                int a0 = t[x] + t[12 + x], a1 = t[4 + x] + t[8 + x], a2 = t[4 + x] - t[8 + x], a3 = t[x] - t[12 + x];
                m[x] = a0 + a1; m[8 + x] = a0 - a1; m[4 + x] = a2 + a3; m[12 + x] = a3 - a2;
            }
            for (int q = 1; q < 16; q++) cost += iabs(m[q]);
            dc[b] = m[0] / 4;
        }
        int t[16];
        for (int y = 0; y < 4; y++) {
            int *r = dc + 4 * y;
            int a0 = r[0] + r[3], a1 = r[1] + r[2], a2 = r[1] - r[2], a3 = r[0] - r[3];
            t[4 * y + 0] = a0 + a1; t[4 * y + 2] = a0 - a1; t[4 * y + 1] = a2 + a3; t[4 * y + 3] = a3 - a2;
        }
        for (int x = 0; x < 4; x++) {
            int a0 = t[x] + t[12 + x], a1 = t[4 + x] + t[8 + x], a2 = t[4 + x] - t[8 + x], a3 = t[x] - t[12 + x];
            cost += iabs(a0 + a1) + iabs(a0 - a1) + iabs(a2 + a3) + iabs(a3 - a2);
        }
        if (cost < best) { best = cost; *mode = k; }
    }
    return best / 2;
}

/* ====================================================================================== */
/*  motion compensation                                                                    */
/* ====================================================================================== */
void jmo_luma_pred_4x4(const mbs *s, int bx4, int by4, int mvx, int mvy, pel *out, int os) {
    for (int y = 0; y < 4; y++)
        for (int x = 0; x < 4; x++)
            out[y * os + x] = (pel)jmo_qpel_at(s->c, 4 * (s->pix_x + 4 * bx4 + x) + mvx,
                                                  4 * (s->pix_y + 4 * by4 + y) + mvy);
}
/* OneComponentChromaPrediction4x4 [J] / 8.4.2.2.2: pixel (i,j) uses the MV of luma 4x4 block
 * (i>>1, j>>1) */
void jmo_chroma_pred_mb(const mbs *s, int uv, const int16_t mv[16][2], pel pred[64]) {
    const jmo_ctx *c = s->c;
    const pel *R = uv ? c->refV : c->refU;
    int Wc = c->Wc, Hc = c->Hc;
    for (int j = 0; j < 8; j++)
        for (int i = 0; i < 8; i++) {
            const int16_t *v = mv[(j >> 1) * 4 + (i >> 1)];
            int ii = ((s->pix_x >> 1) + i) * 8 + v[0], jj = ((s->pix_y >> 1) + j) * 8 + v[1];
            int x0 = iclip(0, Wc - 1, ii >> 3), y0 = iclip(0, Hc - 1, jj >> 3);
            int x1 = iclip(0, Wc - 1, (ii + 7) >> 3), y1 = iclip(0, Hc - 1, (jj + 7) >> 3);
            int fx = ii & 7, fy = jj & 7;
            pred[j * 8 + i] = (pel)(((8 - fx) * (8 - fy) * R[y0 * Wc + x0] + fx * (8 - fy) * R[y0 * Wc + x1] +
                                         (8 - fx) * fy * R[y1 * Wc + x0] + fx * fy * R[y1 * Wc + x1] + 32) >> 6);
        }
}

/* ====================================================================================== */
/*  Intra8x8 decision (High profile): JM FRExt rdopt.c › Mode_Decision_for_Intra8x8Macroblock /  */
/*  Mode_Decision_for_new_8x8IntraBlocks, RDO off [J] (docs/JM_SEMANTICS.md items 26-28)      */
/* ====================================================================================== */
/* the 25 neighbour samples of 8x8 block b8 (inside the MB from rec, the MB's reconstruction so
 * far; outside from the picture) and their availability bits (1 left, 2 top, 4 top-right, 8
 * top-left), as jmo_intra8x8_pred_px takes them */
int jmo_i8_neighbours(const mbs *s, const pel rec[256], int b8, int32_t nb[25]) {
    const jmo_ctx *c = s->c;
    int bx = 8 * (b8 & 1), by = 8 * (b8 >> 1);
#define SMP(x, y) (((x) >= 0 && (x) < 16 && (y) >= 0 && (y) < 16) ? rec[(y) * 16 + (x)] \
                   : c->recY[(s->pix_y + (y)) * c->W + s->pix_x + (x)])
    int left = luma_avail(s, bx - 1, by), up = luma_avail(s, bx, by - 1);
    int ul = luma_avail(s, bx - 1, by - 1), ur = luma_avail(s, bx + 8, by - 1);
    for (int i = 0; i < 25; i++) nb[i] = 0;
    if (ul) nb[0] = SMP(bx - 1, by - 1);
    for (int x = 0; x < 16; x++) if (up && (x < 8 || ur)) nb[1 + x] = SMP(bx + x, by - 1);
    for (int y = 0; y < 8; y++) if (left) nb[17 + y] = SMP(bx - 1, by + y);
#undef SMP
    return left | up << 1 | ur << 2 | ul << 3;
}
/* predIntra8x8PredMode (8.3.2.1) of 8x8 block b8: neighbour 4x4 modes (I4: that block, I8:
 * repeated, else 2), modes[] of the current MB's earlier 8x8 blocks */
int jmo_i8_mpm(const mbs *s, int b8, const int modes[4]) {
    const jmo_ctx *c = s->c;
    int bx = 8 * (b8 & 1), by = 8 * (b8 >> 1);
    int ma = -1, mb = -1, ia = 0, ib = 0;
    if (bx) ma = modes[b8 - 1];
    else if (jmo_nb4(s, -1, by, &ia)) ma = c->ipred[ia];
    if (by) mb = modes[b8 - 2];
    else if (jmo_nb4(s, bx, -1, &ib)) mb = c->ipred[ib];
    return (ma < 0 || mb < 0) ? 2 : imin(ma, mb);
}

int jmo_intra8x8_decision(mbs *s, int qp, int lambda, int intra_round, pel rec[256],
                             int16_t lev[4][64], int modes[4], int *cbp) {
    const jmo_ctx *c = s->c;
    int cost = 6 * lambda;                                 /* (int)floor(6*lambda+0.4999), once */
    *cbp = 0;
    for (int b8 = 0; b8 < 4; b8++) {
        int bx = 8 * (b8 & 1), by = 8 * (b8 >> 1);
        int32_t nb[25];
        int av = jmo_i8_neighbours(s, rec, b8, nb);
        pel pred[9][64];
        int ok = jmo_intra8x8_pred_px(nb, av, pred, (c->maxv + 1) >> 1);
        int mpm = jmo_i8_mpm(s, b8, modes);
        int best = 2, bcost = BIGCOST;
        for (int m = 0; m < 9; m++) {
            if (!((ok >> m) & 1)) continue;
            int32_t d[64];
            for (int y = 0; y < 8; y++)
                for (int x = 0; x < 8; x++) d[8 * y + x] = s->org[(by + y) * 16 + bx + x] - pred[m][8 * y + x];
            int mc = (m == mpm ? 0 : 4 * lambda) + jmo_satd8x8(d, c->cfg.use_hadamard);
            if (mc < bcost) { bcost = mc; best = m; }
        }
        modes[b8] = best;
        int32_t r[64];
        for (int y = 0; y < 8; y++)
            for (int x = 0; x < 8; x++) r[8 * y + x] = s->org[(by + y) * 16 + bx + x] - pred[best][8 * y + x];
        int dummy = 0;
        if (jmo_dct_luma8x8(r, pred[best], 8, qp, intra_round, lev[b8], &dummy, rec + by * 16 + bx, 16, c->maxv)) *cbp |= 1 << b8;
        cost += bcost;
    }
    return cost;
}

/* TransformDecision [J] (RDO off): over the final prediction of the MB, sum of the 16 4x4 SATDs
 * against the sum of the four 8x8 SATDs; 8x8 if strictly smaller (item 29) */
int jmo_transform_decision(const mbs *s, const pel pred[256]) {
    int had = s->c->cfg.use_hadamard, cost4 = 0, cost8 = 0;
    for (int b8 = 0; b8 < 4; b8++) {
        int bx = 8 * (b8 & 1), by = 8 * (b8 >> 1);
        int32_t d[64];
        for (int y = 0; y < 8; y++)
            for (int x = 0; x < 8; x++) d[8 * y + x] = s->org[(by + y) * 16 + bx + x] - pred[(by + y) * 16 + bx + x];
        cost8 += jmo_satd8x8(d, had);
        for (int q = 0; q < 4; q++) {
            int32_t e[16];
            for (int y = 0; y < 4; y++)
                for (int x = 0; x < 4; x++) e[4 * y + x] = d[(4 * (q >> 1) + y) * 8 + 4 * (q & 1) + x];
            cost4 += jmo_satd_block(e, had);
        }
    }
    return cost8 < cost4;
}

/* ====================================================================================== */
/*  encode_one_macroblock (RDO off)                                                         */
/* ====================================================================================== */
void jmo_store_rec_luma(jmo_ctx *c, const mbs *s, const pel rec[256]) {
    for (int y = 0; y < 16; y++) memcpy(c->recY + (s->pix_y + y) * c->W + s->pix_x, rec + 16 * y, 16 * sizeof(pel));
}

void jmo_encode_mb(jmo_ctx *c, int mbx, int mby) {
    mbs S;
    mbs *s = &S;
    memset(s, 0, sizeof(*s));
    s->c = c; s->mbx = mbx; s->mby = mby; s->pix_x = 16 * mbx; s->pix_y = 16 * mby;
    s->mb_addr = mby * c->mbw + mbx;
    s->lambda = c->fp.lambda_motion;
    s->lf = 65536 * s->lambda;
    s->slice_p = c->fp.slice_type == JMH_P_SLICE;
    /* quantisation at QP'Y = QPY + QpBdOffsetY (8.5.x; JM >= 10 bitdepth_luma_qp_scale [J]) */
    const int qpy = c->fp.qp, qp = qpy + c->qpbd, lambda = c->fp.lambda_mode, maxv = c->maxv;
    /* JM 8.6: qp_const by slice type, Intra16x16 always / 3 [J]; JM >= 10: the slice's flat
     * OffsetMatrix entry for every block (items 1, 45) */
    const int jm10 = c->cfg.jm_version >= 10;
    int intra_round = jm10 ? JMO_RND_OFF(c->cfg.quant_offset[s->slice_p]) : !s->slice_p;
    int i16_round = jm10 ? intra_round : JMO_RND_I;
    int W = c->W, W4 = W >> 2;
    for (int y = 0; y < 16; y++) memcpy(s->org + 16 * y, c->orgY + (s->pix_y + y) * W + s->pix_x, 16 * sizeof(pel));
    for (int y = 0; y < 8; y++) {
        memcpy(s->orgc[0] + 8 * y, c->orgU + ((s->pix_y >> 1) + y) * c->Wc + (s->pix_x >> 1), 8 * sizeof(pel));
        memcpy(s->orgc[1] + 8 * y, c->orgV + ((s->pix_y >> 1) + y) * c->Wc + (s->pix_x >> 1), 8 * sizeof(pel));
    }
    jmh_mb_result *res = &c->res[s->mb_addr];
    memset(res, 0, sizeof(*res));
    const int *isr = c->cfg.inter_search;
    int valid[9] = {0};
    int intra_only = !s->slice_p;
    for (int m = 1; m <= 7; m++) valid[m] = !intra_only && isr[m];
    valid[8] = valid[4] || valid[5] || valid[6] || valid[7];

    int min_cost = BIGCOST, best_mode = 1;
    int best8x8mode[4] = {0, 0, 0, 0};
    int W4i = W4;
    (void)W4i;
    if (!intra_only) {
        /* ===== 16x16, 16x8, 8x16 ===== */
        for (int mode = 1; mode < 4; mode++) {
            if (!valid[mode]) continue;
            int cost = 0;
            for (int block = 0; block < (mode == 1 ? 1 : 2); block++) {
                jmo_partition_motion_search(s, mode, block);
                cost += s->motion_cost[mode][block];   /* + (int)(2*lambda*min(ref,1)) == 0 */
            }
            if (cost < min_cost) { best_mode = mode; min_cost = cost; }
        }
        /* ===== P8x8 ===== */
        if (valid[8]) {
            int cost8x8 = 0;
            for (int block = 0; block < 4; block++) {
                int min_cost8x8 = BIGCOST;
                for (int mode = 4; mode <= 7; mode++) {
                    if (!valid[mode]) continue;
                    jmo_partition_motion_search(s, mode, block);
                    int cost = s->motion_cost[mode][block];
                    if (cost < min_cost8x8) { min_cost8x8 = cost; best8x8mode[block] = mode; }
                }
                cost8x8 += min_cost8x8;
                /* reset stored motion vectors of this 8x8 to its best sub-mode */
                int mode = best8x8mode[block];
                if (mode > 0) jmo_write_enc_mv(s, (block & 1) * 2, (block >> 1) * 2, 2, 2, s->all_mv[mode]);
            }
            if (cost8x8 < min_cost) { best_mode = JMH_P8x8; min_cost = cost8x8; }
        }
        jmo_find_skip_mv(s);
        memcpy(c->mem_mv, s->all_mv, sizeof(c->mem_mv));   /* EPZS spatial memory of the next MB */
    }

    /* ===== Intra 8x8 decision (Transform8x8Mode; before Intra4x4, "<=") ===== */
    const int t8 = c->cfg.transform_8x8_mode;
    pel i8rec[256];
    int16_t i8lev[4][64];
    int i8modes[4] = {2, 2, 2, 2}, i8cbp = 0;
    if (t8) {
        int i8cost = jmo_intra8x8_decision(s, qp, lambda, intra_round, i8rec, i8lev, i8modes, &i8cbp);
        if (i8cost <= min_cost) { min_cost = i8cost; best_mode = JMH_I8MB; }
    }
    /* ===== Intra 4x4 decision (with TQ + recon of every 4x4 in coding order) ===== */
    pel i4rec[256];
    int16_t i4lev[16][16];
    int i4modes[16];
    int i4cbp = 0, i4cbpblk = 0, i4cost = 0;
    {
        int W4l = c->W >> 2;
        /* save the recon area: Mode_Decision_for_Intra4x4Macroblock writes enc_picture */
        for (int b8 = 0; b8 < 4; b8++) {
            int cost8 = 6 * lambda;                         /* (int)floor(6*lambda+0.4999) */
            for (int b4 = 0; b4 < 4; b4++) {
                int bx = 8 * (b8 & 1) + 4 * (b4 & 1), by = 8 * (b8 >> 1) + 4 * (b4 >> 1);
                int blk = (by >> 2) * 4 + (bx >> 2);
                int ia = 0, ib = 0;
                int av_l = jmo_nb4(s, bx - 1, by, &ia), av_u = jmo_nb4(s, bx, by - 1, &ib);
                int upMode = av_u ? c->ipred[ib] : -1, leftMode = av_l ? c->ipred[ia] : -1;
                int mpm = (upMode < 0 || leftMode < 0) ? 2 : imin(upMode, leftMode);
                pel pred[9][16];
                int avail[9];
                jmo_intra4x4_pred(s, bx, by, pred, avail);
                int best = 0, bcost = BIGCOST;
                for (int m = 0; m < 9; m++) {
                    if (!avail[m]) continue;
                    int32_t d[16];
                    for (int y = 0; y < 4; y++)
                        for (int x = 0; x < 4; x++)
                            d[4 * y + x] = s->org[(by + y) * 16 + bx + x] - pred[m][4 * y + x];
                    int cost = (m == mpm) ? 0 : 4 * lambda;      /* (int)floor(4*lambda) */
                    cost += jmo_satd_block(d, c->cfg.use_hadamard);
                    if (cost < bcost) { best = m; bcost = cost; }
                }
                c->ipred[((s->pix_y + by) >> 2) * W4l + ((s->pix_x + bx) >> 2)] = (int8_t)best;
                i4modes[blk] = best;
                int32_t r[16];
                for (int y = 0; y < 4; y++)
                    for (int x = 0; x < 4; x++)
                        r[4 * y + x] = s->org[(by + y) * 16 + bx + x] - pred[best][4 * y + x];
                int dummy = 0;
                pel *dst = c->recY + (s->pix_y + by) * c->W + s->pix_x + bx;
                if (jmo_dct_luma4x4(r, pred[best], 4, qp, intra_round, i4lev[blk], &dummy, dst, c->W, maxv)) {
                    i4cbp |= 1 << b8;
                    i4cbpblk |= 1 << blk;
                }
                cost8 += bcost;
            }
            i4cost += cost8;
        }
        for (int y = 0; y < 16; y++) memcpy(i4rec + 16 * y, c->recY + (s->pix_y + y) * c->W + s->pix_x, 16 * sizeof(pel));
    }
    if (i4cost <= min_cost) { min_cost = i4cost; best_mode = JMH_I4MB; }
    /* ===== Intra 16x16 ===== */
    pel i16pred[4][256];
    int i16avail[4], i16mode = 2;
    jmo_intra16_pred(s, i16pred, i16avail);
    int i16cost = jmo_find_sad_16x16(s, i16pred, i16avail, &i16mode);
    if (i16cost < min_cost) { min_cost = i16cost; best_mode = JMH_I16MB; }

    /* ===== final macroblock parameters ===== */
    int is_intra = best_mode == JMH_I4MB || best_mode == JMH_I16MB || best_mode == JMH_I8MB;
    int16_t fmv[16][2];
    memset(fmv, 0, sizeof(fmv));
    int b8mode[4];
    for (int b = 0; b < 4; b++) b8mode[b] = best_mode == JMH_P8x8 ? best8x8mode[b] : best_mode;
    if (best_mode == JMH_I4MB) for (int b = 0; b < 4; b++) b8mode[b] = JMH_IBLOCK;
    if (best_mode == JMH_I16MB) for (int b = 0; b < 4; b++) b8mode[b] = 0;
    if (best_mode == JMH_I8MB) for (int b = 0; b < 4; b++) b8mode[b] = JMH_I8MB;
    if (!is_intra)
        for (int k = 0; k < 16; k++) {
            int b8 = ((k >> 3) << 1) + ((k & 3) >> 1);
            fmv[k][0] = s->all_mv[b8mode[b8]][k][0];
            fmv[k][1] = s->all_mv[b8mode[b8]][k][1];
        }
    int cbp = 0, cbp_blk = 0, tr8 = 0;
    pel rec[256];
    if (best_mode == JMH_I8MB) {
        cbp = i8cbp; tr8 = 1;
        memcpy(rec, i8rec, sizeof(rec));
        for (int b8 = 0; b8 < 4; b8++) {
            jmo_put_levels8(res->luma, b8, i8lev[b8]);
            if ((cbp >> b8) & 1) cbp_blk |= 0x33 << ((b8 >> 1) * 8 + (b8 & 1) * 2);
        }
        for (int k = 0; k < 16; k++) res->ipred[k] = (int8_t)i8modes[((k >> 3) << 1) + ((k & 3) >> 1)];
    } else if (best_mode == JMH_I4MB) {
        cbp = i4cbp; cbp_blk = i4cbpblk;
        memcpy(rec, i4rec, sizeof(rec));
        for (int k = 0; k < 16; k++) { res->ipred[k] = (int8_t)i4modes[k]; memcpy(res->luma[k], i4lev[k], 32); }
    } else if (best_mode == JMH_I16MB) {
        int32_t r[256];
        for (int k = 0; k < 256; k++) r[k] = s->org[k] - i16pred[i16mode][k];
        cbp = jmo_dct_luma_16x16(r, i16pred[i16mode], qp, i16_round, res->luma_dc, res->luma, &cbp_blk, rec, maxv);
        res->i16mode = (int8_t)i16mode;
    } else {
        /* LumaResidualCoding / LumaResidualCoding8x8 (also SetCoeffAndReconstruction8x8) */
        pel pred[256];
        int sum_cnt_nonz = 0;
        for (int k = 0; k < 16; k++) jmo_luma_pred_4x4(s, k & 3, k >> 2, fmv[k][0], fmv[k][1], pred + 4 * (k >> 2) * 16 + 4 * (k & 3), 16);
        if (t8 && (best_mode <= 3 || (b8mode[0] == 4 && b8mode[1] == 4 && b8mode[2] == 4 && b8mode[3] == 4)))
            tr8 = jmo_transform_decision(s, pred);
        for (int b8 = 0; b8 < 4; b8++) {
            int coeff_cost = 0, cbp8 = 0, blk8 = 0;
            if (tr8) {                                    /* dct_luma8x8 path */
                int bx = 8 * (b8 & 1), by = 8 * (b8 >> 1);
                int32_t r[64];
                int16_t lv[64];
                for (int y = 0; y < 8; y++)
                    for (int x = 0; x < 8; x++) r[8 * y + x] = s->org[(by + y) * 16 + bx + x] - pred[(by + y) * 16 + bx + x];
                if (jmo_dct_luma8x8(r, pred + by * 16 + bx, 16, qp, intra_round, lv, &coeff_cost, rec + by * 16 + bx, 16, maxv)) {
                    cbp8 = 1;
                    blk8 = 0x33 << ((b8 >> 1) * 8 + (b8 & 1) * 2);
                }
                jmo_put_levels8(res->luma, b8, lv);
            }
            for (int b4 = 0; b4 < 4 && !tr8; b4++) {
                int bx4 = 2 * (b8 & 1) + (b4 & 1), by4 = 2 * (b8 >> 1) + (b4 >> 1);
                int k = by4 * 4 + bx4;
                int32_t r[16];
                for (int y = 0; y < 4; y++)
                    for (int x = 0; x < 4; x++)
                        r[4 * y + x] = s->org[(4 * by4 + y) * 16 + 4 * bx4 + x] - pred[(4 * by4 + y) * 16 + 4 * bx4 + x];
                if (jmo_dct_luma4x4(r, pred + 4 * by4 * 16 + 4 * bx4, 16, qp, intra_round, res->luma[k], &coeff_cost,
                                rec + 4 * by4 * 16 + 4 * bx4, 16, maxv)) {
                    blk8 |= 1 << k;
                    cbp8 = 1;
                }
            }
            if (coeff_cost <= LUMA_COEFF_COST) {          /* discard "expensive" single coeffs */
                coeff_cost = 0;
                cbp8 = 0; blk8 = 0;
                for (int b4 = 0; b4 < 4; b4++) {
                    int bx4 = 2 * (b8 & 1) + (b4 & 1), by4 = 2 * (b8 >> 1) + (b4 >> 1);
                    memset(res->luma[by4 * 4 + bx4], 0, 32);
                    for (int y = 0; y < 4; y++)
                        memcpy(rec + (4 * by4 + y) * 16 + 4 * bx4, pred + (4 * by4 + y) * 16 + 4 * bx4, 4 * sizeof(pel));
                }
            }
            if (cbp8) cbp |= 1 << b8;
            cbp_blk |= blk8;
            sum_cnt_nonz += coeff_cost;
        }
        if (sum_cnt_nonz <= LUMA_MB_COEFF_COST) {
            cbp = 0; cbp_blk = 0;
            memset(res->luma, 0, sizeof(res->luma));
            memcpy(rec, pred, sizeof(rec));
        }
    }
    jmo_store_rec_luma(c, s, rec);

    /* ===== chroma: IntraChromaPrediction8x8 (intra MBs) + ChromaResidualCoding ===== */
    int c_mode = 0;
    pel cpred[2][4][64];
    if (is_intra) {
        int cav[4];
        jmo_intra_chroma_pred(s, 0, cpred[0], cav);
        jmo_intra_chroma_pred(s, 1, cpred[1], cav);
        int min_c = BIGCOST;
        for (int m = 0; m < 4; m++) {                 /* DC, H, V, Plane */
            if (!cav[m]) continue;
            int cost = 0;
            for (int uv = 0; uv < 2; uv++)
                for (int b = 0; b < 4; b++) {
                    int32_t d[16];
                    int xo = (b & 1) * 4, yo = (b >> 1) * 4;
                    for (int y = 0; y < 4; y++)
                        for (int x = 0; x < 4; x++)
                            d[4 * y + x] = s->orgc[uv][(yo + y) * 8 + xo + x] - cpred[uv][m][(yo + y) * 8 + xo + x];
                    cost += jmo_satd_block(d, c->cfg.use_hadamard);
                }
            if (cost < min_c) { min_c = cost; c_mode = m; }
        }
    }
    /* QP'c = QPc(Clip3(-QpBdOffsetC, 51, QPY + chroma_qp_index_offset)) + QpBdOffsetC (8.5.8) */
    int qpc = jmo_qpc(qpy + c->fp.chroma_qp_offset, c->qpbd) + c->qpbd;
    int cr_cbp = 0;
    for (int uv = 0; uv < 2; uv++) {
        pel pred[64], crec[64];
        if (is_intra) memcpy(pred, cpred[uv][c_mode], sizeof(pred));
        else jmo_chroma_pred_mb(s, uv, fmv, pred);
        int32_t r[64];
        for (int k = 0; k < 64; k++) r[k] = s->orgc[uv][k] - pred[k];
        cr_cbp = jmo_dct_chroma(r, pred, qpc, intra_round, cr_cbp, res->chroma_dc[uv], res->chroma_ac[uv], crec, maxv);
        pel *R = uv ? c->recV : c->recU;
        for (int y = 0; y < 8; y++) memcpy(R + ((s->pix_y >> 1) + y) * c->Wc + (s->pix_x >> 1), crec + 8 * y, 8 * sizeof(pel));
    }
    cbp |= cr_cbp << 4;

    /* ===== results, picture arrays, P_Skip detection ===== */
    int mb_type = best_mode;
    if (s->slice_p && best_mode == 1 && cbp == 0 && fmv[0][0] == s->skip_mv[0] && fmv[0][1] == s->skip_mv[1])
        mb_type = JMH_PSKIP;
    res->mb_type = (int16_t)mb_type;
    res->transform_8x8 = (int8_t)(tr8 && (best_mode == JMH_I8MB || (cbp & 15)));
    res->cbp = (int16_t)cbp;
    res->cbp_blk = cbp_blk;
    res->c_ipred_mode = (int8_t)(is_intra ? c_mode : 0);
    res->min_cost = min_cost;
    for (int b = 0; b < 4; b++) {
        res->b8mode[b] = (int8_t)(mb_type == JMH_PSKIP ? 0 : b8mode[b]);
        res->ref_idx[b] = (int8_t)(is_intra ? -1 : 0);
    }
    memcpy(res->mv, fmv, sizeof(fmv));
    for (int k = 0; k < 16; k++) {
        int a = ((s->pix_y >> 2) + (k >> 2)) * W4 + (s->pix_x >> 2) + (k & 3);
        c->mv[2 * a] = fmv[k][0];
        c->mv[2 * a + 1] = fmv[k][1];
        c->refidx[a] = (int8_t)(is_intra ? -1 : 0);
        if (best_mode == JMH_I8MB) c->ipred[a] = res->ipred[k];
        else if (best_mode != JMH_I4MB) {
            res->ipred[k] = 2;
            /* predIntraNxNPredMode (8.3.1.1): an inter neighbour under constrained_intra_pred sets
             * dcPredModePredictedFlag, as an unavailable one (-1 here) */
            c->ipred[a] = (int8_t)(!is_intra && c->cfg.constrained_intra_pred ? -1 : 2);
        }
    }
    c->mbintra[s->mb_addr] = (int8_t)is_intra;
}
