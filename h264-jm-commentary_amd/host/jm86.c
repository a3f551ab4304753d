/*
 * jm86.c — the JM 8.6 call surface of the hot path (jmhost.h): encode_one_macroblock,
 * PartitionMotionSearch, BlockMotionSearch and dct_luma with JM 8.6 signatures over JM-shaped
 * state (img), so lencod's slice loop — start_macroblock → encode_one_macroblock →
 * write_one_macroblock per macroblock (JM 8.6 slice.c › encode_one_slice [J]) — runs unchanged
 * on top of the device.
 *
 * Restated JM 8.6 functions [J] (no file:line exists: /root/reference holds README.md:1-4):
 *   rdopt.c     › encode_one_macroblock (RDO off: the inter part, modes 1..3 then P8x8 with
 *                 the per-8x8 sub-mode decision, strict '<')
 *   mv-search.c › PartitionMotionSearch (RestrictSearchRange), BlockMotionSearch,
 *                 SetMotionVectorPredictor (8.4.1.3), SetupFastFullPelSearch's window centre
 *   block.c     › dct_luma
 *   macroblock.c› start_macroblock, write_one_macroblock
 * The arithmetic of the searches and the transform runs on the device (jmh_block_motion_search,
 * jmh_tq4x4_batch) through the backend; this file holds only JM's control flow and state.
 */
#include <math.h>
#include <stdlib.h>
#include <string.h>
#include "jmhost.h"

__thread jm86_img *img = NULL;

static const int blc_size[8][2] = {{16, 16}, {16, 16}, {16, 8}, {8, 16}, {8, 8}, {8, 4}, {4, 8}, {4, 4}};

int jm86_init(jm86_img *im, const jm_input *inp, jm_backend *be, int width, int height) {
    memset(im, 0, sizeof(*im));
    im->width = width; im->height = height;
    im->mbw = width / 16; im->mbh = height / 16;
    im->input = inp;
    im->be = be;
    size_t n4 = (size_t)width * height / 16;
    im->mb_data = (jmh_mb_result *)calloc((size_t)im->mbw * im->mbh, sizeof(jmh_mb_result));
    im->enc_mv = (int16_t *)calloc(2 * n4, sizeof(int16_t));
    im->enc_ref = (int8_t *)malloc(n4);
    im->enc_imgY = (uint8_t *)calloc((size_t)width * height, 1);
    if (!im->mb_data || !im->enc_mv || !im->enc_ref || !im->enc_imgY) { jm86_free(im); return JMH_E_OOM; }
    img = im;
    return JMH_OK;
}

void jm86_free(jm86_img *im) {
    free(im->mb_data); free(im->enc_mv); free(im->enc_ref); free(im->enc_imgY);
    im->mb_data = NULL; im->enc_mv = NULL; im->enc_ref = NULL; im->enc_imgY = NULL;
    if (img == im) img = NULL;
}

static int surface_on(const jm86_img *im) {
    const jm_input *inp = im->input;
    return inp->jm_call_surface && im->type == JMH_P_SLICE && (inp->search_mode == 0 || inp->search_mode == -1) &&
           im->be->block_search && im->be->search_pictures;
}

int jm86_start_picture(jm86_img *im, const jmh_frame_params *fp, const jm_pic *cur, const jm_pic *ref, jm_slice_writer *writer) {
    img = im;
    im->type = fp->slice_type;
    im->qp = fp->qp;
    im->lambda_mode = fp->lambda_mode;
    im->lambda_motion = fp->lambda_motion;
    im->writer = writer;
    im->slice_first = 0;
    memset(im->enc_mv, 0, (size_t)im->width * im->height / 16 * 2 * sizeof(int16_t));
    memset(im->enc_ref, -1, (size_t)im->width * im->height / 16);
    if (surface_on(im)) return im->be->search_pictures(im->be->ctx, cur, ref);
    return JMH_OK;
}

/* macroblock.c › start_macroblock [J]: position of img->current_mb_nr */
void start_macroblock(void) {
    img->mb_x = img->current_mb_nr % img->mbw;
    img->mb_y = img->current_mb_nr / img->mbw;
    img->pix_x = 16 * img->mb_x;
    img->pix_y = 16 * img->mb_y;
    img->setup_done = 0;
    memset(img->all_mv, 0, sizeof(img->all_mv));
    memset(img->motion_cost, 0, sizeof(img->motion_cost));
}

/* ---- SetMotionVectorPredictor [J] / H.264 8.4.1.3 over enc_picture (list 0) ------------- */
/* neighbour 4x4 of the current MB at luma offset (xN, yN): available + picture 4x4 index */
static int nb4(int xN, int yN, int *idx) {
    int mx, my;
    if (yN > 15) return 0;
    if (xN < 0) { mx = img->mb_x - 1; my = yN < 0 ? img->mb_y - 1 : img->mb_y; }
    else if (xN <= 15) { mx = img->mb_x; my = yN < 0 ? img->mb_y - 1 : img->mb_y; }
    else { if (yN >= 0) return 0; mx = img->mb_x + 1; my = img->mb_y - 1; }
    /* raster order: the rest is coded; outside the current slice is unavailable (6.4.8) */
    if (mx < 0 || my < 0 || mx >= img->mbw || my * img->mbw + mx < img->slice_first) return 0;
    *idx = ((img->pix_y + yN) >> 2) * (img->width >> 2) + ((img->pix_x + xN) >> 2);
    return 1;
}

static void SetMotionVectorPredictor(int pmv[2], int ref, int mb_x, int mb_y, int bsx, int bsy) {
    int ia = 0, ib = 0, ic = 0, id = 0;
    int av_a = nb4(mb_x - 1, mb_y, &ia), av_b = nb4(mb_x, mb_y - 1, &ib);
    int av_c = nb4(mb_x + bsx, mb_y - 1, &ic), av_d = nb4(mb_x - 1, mb_y - 1, &id);
    if (mb_y > 0) {   /* C inside the MB but later in decoding order */
        if (mb_x < 8) { if (mb_y == 8) { if (bsx == 16) av_c = 0; } else if (mb_x + bsx == 8) av_c = 0; }
        else if (mb_x + bsx == 16) av_c = 0;
    }
    if (!av_c) { av_c = av_d; ic = id; }
    const int rL = av_a ? img->enc_ref[ia] : -1, rU = av_b ? img->enc_ref[ib] : -1, rUR = av_c ? img->enc_ref[ic] : -1;
    int type = 0;   /* 0 median, 1 left, 2 up, 3 up-right */
    if (rL == ref && rU != ref && rUR != ref) type = 1;
    else if (rL != ref && rU == ref && rUR != ref) type = 2;
    else if (rL != ref && rU != ref && rUR == ref) type = 3;
    if (bsx == 8 && bsy == 16) { if (mb_x == 0) { if (rL == ref) type = 1; } else if (rUR == ref) type = 3; }
    else if (bsx == 16 && bsy == 8) { if (mb_y == 0) { if (rU == ref) type = 2; } else if (rL == ref) type = 1; }
    for (int hv = 0; hv < 2; hv++) {
        const int a = av_a ? img->enc_mv[2 * ia + hv] : 0, b = av_b ? img->enc_mv[2 * ib + hv] : 0;
        const int c = av_c ? img->enc_mv[2 * ic + hv] : 0;
        int p;
        if (type == 1) p = a;
        else if (type == 2) p = b;
        else if (type == 3) p = c;
        else if (!(av_b || av_c)) p = a;
        else {
            const int mn = a < b ? (a < c ? a : c) : (b < c ? b : c), mx = a > b ? (a > c ? a : c) : (b > c ? b : c);
            p = a + b + c - mn - mx;
        }
        pmv[hv] = p;
    }
}

static int clampi(int lo, int hi, int v) { return v < lo ? lo : v > hi ? hi : v; }

/* mv-search.c › BlockMotionSearch [J]: one block (list 0, ref 0); mb_x / mb_y: the block's
 * luma offset inside the macroblock.  Stores the MV in img->all_mv, returns min_mcost. */
int BlockMotionSearch(int ref, int list, int mb_x, int mb_y, int blocktype, int search_range, double lambda) {
    const jm_input *inp = img->input;
    const int bsx = blc_size[blocktype][0], bsy = blc_size[blocktype][1];
    int pmv[2];
    SetMotionVectorPredictor(pmv, ref, mb_x, mb_y, bsx, bsy);
    jmh_block_search q;
    memset(&q, 0, sizeof(q));
    q.mb_x = img->mb_x; q.mb_y = img->mb_y;
    q.blocktype = blocktype;
    q.block_x = mb_x >> 2; q.block_y = mb_y >> 2;
    q.pred_mv[0] = pmv[0]; q.pred_mv[1] = pmv[1];
    q.search_range = search_range;
    q.lambda_factor = (int)(65536.0 * lambda + 0.5);   /* LAMBDA_FACTOR [J] */
    q.search_mode = inp->search_mode;
    q.slice_p = img->type == JMH_P_SLICE;
    if (inp->search_mode == 0) {
        if (!img->setup_done) {   /* SetupFastFullPelSearch: 16x16 MVP / 4, clamped to +-SearchRange */
            int p16[2];
            SetMotionVectorPredictor(p16, ref, 0, 0, 16, 16);
            img->search_centre[0] = clampi(-inp->search_range, inp->search_range, p16[0] / 4);
            img->search_centre[1] = clampi(-inp->search_range, inp->search_range, p16[1] / 4);
            img->setup_done = 1;
        }
        q.centre[0] = img->search_centre[0]; q.centre[1] = img->search_centre[1];
    } else {   /* search centre = MVP / 4, the (0,0) vector kept inside (RDO off) */
        q.centre[0] = clampi(-search_range, search_range, pmv[0] / 4);
        q.centre[1] = clampi(-search_range, search_range, pmv[1] / 4);
    }
    jmh_block_result r;
    int st = img->be->block_search(img->be->ctx, 1, &q, &r);
    if (st) { fprintf(stderr, "BlockMotionSearch: backend status %d\n", st); return 1 << 20; }
    img->surface_searches++;
    (void)list;
    for (int y = 0; y < (bsy >> 2); y++)
        for (int x = 0; x < (bsx >> 2); x++) {
            const int k = ((mb_y >> 2) + y) * 4 + (mb_x >> 2) + x;
            img->all_mv[blocktype][k][0] = (int16_t)r.mv[0];
            img->all_mv[blocktype][k][1] = (int16_t)r.mv[1];
        }
    return r.min_mcost;
}

/* enc_picture->mv / ref_idx of a block of the current MB (for the MVPs that follow) */
static void set_enc_mv(int bx4, int by4, int w4, int h4, const int16_t (*mv)[2], int ref) {
    const int W4 = img->width >> 2;
    for (int y = 0; y < h4; y++)
        for (int x = 0; x < w4; x++) {
            const int k = (by4 + y) * 4 + bx4 + x, a = ((img->pix_y >> 2) + by4 + y) * W4 + (img->pix_x >> 2) + bx4 + x;
            img->enc_mv[2 * a] = mv ? mv[k][0] : 0;
            img->enc_mv[2 * a + 1] = mv ? mv[k][1] : 0;
            img->enc_ref[a] = (int8_t)ref;
        }
}

/* mv-search.c › PartitionMotionSearch [J] (list 0, one reference frame) */
void PartitionMotionSearch(int blocktype, int block8x8, double lambda) {
    static const int bx0[5][4] = {{0, 0, 0, 0}, {0, 0, 0, 0}, {0, 0, 0, 0}, {0, 2, 0, 0}, {0, 2, 0, 2}};
    static const int by0[5][4] = {{0, 0, 0, 0}, {0, 0, 0, 0}, {0, 2, 0, 0}, {0, 0, 0, 0}, {0, 0, 2, 2}};
    const jm_input *inp = img->input;
    const int parttype = blocktype < 4 ? blocktype : 4;
    const int step_h0 = blc_size[parttype][0] >> 2, step_v0 = blc_size[parttype][1] >> 2;
    const int step_h = blc_size[blocktype][0] >> 2, step_v = blc_size[blocktype][1] >> 2;
    const int ref = 0;
    /* RestrictSearchRange (input->full_search): 2 whole range, 1 / (min(ref,1)+1), 0 also / min(2, blocktype) */
    int search_range = inp->search_range;
    if (inp->restrict_search_range == 1) search_range /= (ref < 1 ? ref : 1) + 1;
    else if (inp->restrict_search_range == 0) search_range /= ((ref < 1 ? ref : 1) + 1) * (blocktype < 2 ? blocktype : 2);
    img->motion_cost[blocktype][block8x8] = 0;
    for (int v = by0[parttype][block8x8]; v < by0[parttype][block8x8] + step_v0; v += step_v)
        for (int h = bx0[parttype][block8x8]; h < bx0[parttype][block8x8] + step_h0; h += step_h) {
            img->motion_cost[blocktype][block8x8] += BlockMotionSearch(ref, 0, 4 * h, 4 * v, blocktype, search_range, lambda);
            set_enc_mv(h, v, step_h, step_v, (const int16_t (*)[2])img->all_mv[blocktype], ref);
        }
}

/* the RDO-off inter part of rdopt.c › encode_one_macroblock [J]: returns the best inter mode
 * (1..3, 8 = P8x8) and its cost; best8x8[b8] = the sub-mode of each 8x8 block */
static int inter_searches(int *best_cost, int best8x8[4]) {
    const int *isr = img->input->inter_search;
    const double lambda = img->lambda_motion;
    int min_cost = 1 << 20, best_mode = 1;
    for (int mode = 1; mode < 4; mode++) {
        if (!isr[mode]) continue;
        int cost = 0;
        for (int block = 0; block < (mode == 1 ? 1 : 2); block++) {
            PartitionMotionSearch(mode, block, lambda);
            cost += img->motion_cost[mode][block];   /* + (int)(2*lambda*min(ref,1)) == 0 */
        }
        if (cost < min_cost) { best_mode = mode; min_cost = cost; }
    }
    if (isr[4] || isr[5] || isr[6] || isr[7]) {
        int cost8x8 = 0;
        for (int block = 0; block < 4; block++) {
            int min8 = 1 << 20;
            best8x8[block] = 0;
            for (int mode = 4; mode <= 7; mode++) {
                if (!isr[mode]) continue;
                PartitionMotionSearch(mode, block, lambda);
                if (img->motion_cost[mode][block] < min8) { min8 = img->motion_cost[mode][block]; best8x8[block] = mode; }
            }
            cost8x8 += min8;
            /* the 8x8 block's MVs for the MVPs that follow: its best sub-mode */
            if (best8x8[block]) set_enc_mv((block & 1) * 2, (block >> 1) * 2, 2, 2, (const int16_t (*)[2])img->all_mv[best8x8[block]], 0);
        }
        if (cost8x8 < min_cost) { best_mode = JMH_P8x8; min_cost = cost8x8; }
    }
    *best_cost = min_cost;
    return best_mode;
}

/* the decision of the backend against the call surface's inter searches: an inter decision
 * must be the best inter mode with its cost and MVs; an intra one must not cost more */
static int check_decision(const jmh_mb_result *r, int best_mode, int best_cost, const int best8x8[4]) {
    const int t = r->mb_type;
    if (t == JMH_I4MB || t == JMH_I8MB) return r->min_cost <= best_cost;
    if (t == JMH_I16MB) return r->min_cost < best_cost;
    const int mode = t == JMH_PSKIP ? 1 : t;
    if (mode != best_mode || r->min_cost != best_cost) return 0;
    for (int k = 0; k < 16; k++) {
        const int b8 = ((k >> 3) << 1) + ((k & 3) >> 1), m = mode == JMH_P8x8 ? best8x8[b8] : mode;
        if (mode == JMH_P8x8 && r->b8mode[b8] != m) return 0;
        if (r->mv[k][0] != img->all_mv[m][k][0] || r->mv[k][1] != img->all_mv[m][k][1]) return 0;
    }
    return 1;
}

/* rdopt.c › encode_one_macroblock [J] (RDO off) for img->current_mb_nr */
void encode_one_macroblock(void) {
    const int a = img->current_mb_nr;
    const jmh_mb_result *r = img->res ? &img->res[a] : img->be->mb_result(img->be->ctx, a);
    if (surface_on(img)) {
        int best_cost = 0, best8x8[4] = {0, 0, 0, 0};
        const int best_mode = inter_searches(&best_cost, best8x8);
        img->surface_checked++;
        if (!check_decision(r, best_mode, best_cost, best8x8)) {
            img->surface_mismatches++;
            fprintf(stderr, "encode_one_macroblock: MB %d: decision (type %d, cost %d) disagrees with the call surface's "
                            "inter searches (mode %d, cost %d)\n", a, r->mb_type, r->min_cost, best_mode, best_cost);
        }
    }
    if (r != &img->mb_data[a]) img->mb_data[a] = *r;
    /* the final MVs become enc_picture's (intra: ref_idx -1) */
    const int intra = r->mb_type == JMH_I4MB || r->mb_type == JMH_I16MB || r->mb_type == JMH_I8MB;
    set_enc_mv(0, 0, 4, 4, intra ? NULL : (const int16_t (*)[2])r->mv, intra ? -1 : 0);
}

/* macroblock.c › write_one_macroblock [J]: CAVLC of the current macroblock */
void write_one_macroblock(void) { jm_slice_write_mb(img->writer, img->current_mb_nr, &img->mb_data[img->current_mb_nr]); }

/* block.c › dct_luma [J]: the 4x4 block at luma offset (block_x, block_y) of the current MB:
 * forward transform + quantisation of img->m7, levels (frame zig-zag) into the MB's cofAC
 * (mb_data.luma), dequantisation + inverse + reconstruction over img->mpr into enc_picture's
 * imgY; *coeff_cost += the block's COEFF_COST; returns the nonzero flag.  The rounding offset
 * follows the slice type (docs/JM_SEMANTICS.md item 1); old_intra_mode is not used (it serves
 * JM's lossless coding only). */
int dct_luma(int block_x, int block_y, int *coeff_cost, int old_intra_mode) {
    (void)old_intra_mode;
    int16_t resid[16], lev[16];
    uint8_t pred[16], rec[16];
    int32_t cc = 0, nz = 0;
    for (int y = 0; y < 4; y++)
        for (int x = 0; x < 4; x++) {
            resid[4 * y + x] = (int16_t)img->m7[block_y + y][block_x + x];
            pred[4 * y + x] = img->mpr[block_y + y][block_x + x];
        }
    if (!img->be->tq4x4 || img->be->tq4x4(img->be->ctx, 1, resid, pred, img->qp, img->type == JMH_I_SLICE, lev, rec, &cc, &nz)) {
        fprintf(stderr, "dct_luma: backend failed\n");
        return 0;
    }
    const int blk = (block_y >> 2) * 4 + (block_x >> 2);
    memcpy(img->mb_data[img->current_mb_nr].luma[blk], lev, sizeof(lev));
    for (int y = 0; y < 4; y++)
        memcpy(img->enc_imgY + (size_t)(img->pix_y + block_y + y) * img->width + img->pix_x + block_x, rec + 4 * y, 4);
    *coeff_cost += cc;
    return nz;
}
