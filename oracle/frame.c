/*
 * frame.c — oracle picture driver (TEST INFRASTRUCTURE ONLY).
 * Restates JM 8.6 image.c › code_a_picture / slice.c › encode_one_slice's macroblock loop
 * (one slice, raster order) around encode_one_macroblock, and exposes the unit seams that
 * tests compare the GPU path against.
 */
#include <stdio.h>
#include <stdlib.h>
#include "jmo_internal.h"

static int cfg_ok(const jmh_config *cfg) {
    if (!cfg || cfg->width <= 0 || cfg->height <= 0 || (cfg->width & 15) || (cfg->height & 15))
        return JMH_E_INVALID_ARG;
    if (cfg->search_range < 1 || cfg->search_range > JMO_MAX_SR) return JMH_E_INVALID_ARG;
    if (cfg->search_mode != 0 && cfg->search_mode != -1 && cfg->search_mode != 3) return JMH_E_UNSUPPORTED_CFG;
    if (cfg->num_ref_frames != 1) return JMH_E_UNSUPPORTED_CFG;
    if (cfg->constrained_intra_pred != 0 && cfg->constrained_intra_pred != 1) return JMH_E_INVALID_ARG;
    if (cfg->restrict_search_range < 0 || cfg->restrict_search_range > 2) return JMH_E_INVALID_ARG;
    if (cfg->transform_8x8_mode != 0 && cfg->transform_8x8_mode != 1) return JMH_E_UNSUPPORTED_CFG;
    if (cfg->jm_version < 0 || cfg->jm_version == 9 || cfg->jm_version > 99) return JMH_E_UNSUPPORTED_CFG;
    if (cfg->epzs_dual_refinement != 0 && cfg->epzs_dual_refinement != 1) return JMH_E_UNSUPPORTED_CFG;
    if (cfg->slice_mbs < 0) return JMH_E_INVALID_ARG;
    if ((cfg->epzs_subpel_me != 0 && cfg->epzs_subpel_me != 1) || cfg->epzs_subpel_thres_scale < 0 ||
        cfg->epzs_subpel_thres_scale > JMH_EPZS_SCALE_MAX || cfg->epzs_min_thres_scale < 0 || cfg->epzs_min_thres_scale > JMH_EPZS_SCALE_MAX ||
        cfg->epzs_max_thres_scale < 0 || cfg->epzs_max_thres_scale > JMH_EPZS_SCALE_MAX) return JMH_E_INVALID_ARG;
    if (cfg->bit_depth != 0 && (cfg->bit_depth < 8 || cfg->bit_depth > 10)) return JMH_E_UNSUPPORTED_CFG;
    /* RDOptimization 1: CABAC rate, 4x4 transform (docs/JM_SEMANTICS.md items 53-60) */
    if (cfg->rdo != 0 && cfg->rdo != 1) return JMH_E_UNSUPPORTED_CFG;
    if (cfg->jm_version >= 10 && (cfg->quant_offset[0] < 0 || cfg->quant_offset[0] > JMH_QOFFSET_MAX || cfg->quant_offset[1] < 0 ||
                                  cfg->quant_offset[1] > JMH_QOFFSET_MAX)) return JMH_E_INVALID_ARG;
    return JMH_OK;
}

int jmo_create(const jmh_config *cfg, jmo_ctx **out) {
    int st = cfg_ok(cfg);
    if (st) return st;
    jmo_ctx *c = (jmo_ctx *)calloc(1, sizeof(jmo_ctx));
    if (!c) return JMH_E_OOM;
    c->cfg = *cfg;
    c->W = cfg->width; c->H = cfg->height; c->Wc = c->W / 2; c->Hc = c->H / 2;
    c->mbw = c->W / 16; c->mbh = c->H / 16;
    c->bd = cfg->bit_depth ? cfg->bit_depth : 8;
    c->maxv = (1 << c->bd) - 1;
    c->qpbd = 6 * (c->bd - 8);
    c->sr = cfg->search_range;
    c->npos = (2 * c->sr + 1) * (2 * c->sr + 1);
    jmo_init_spiral(c);
    size_t ls = (size_t)c->W * c->H, cs = (size_t)c->Wc * c->Hc, n4 = ls / 16;
    c->orgY = malloc(ls * sizeof(pel)); c->orgU = malloc(cs * sizeof(pel)); c->orgV = malloc(cs * sizeof(pel));
    c->refY = malloc(ls * sizeof(pel)); c->refU = malloc(cs * sizeof(pel)); c->refV = malloc(cs * sizeof(pel));
    c->recY = calloc(ls, sizeof(pel)); c->recU = calloc(cs, sizeof(pel)); c->recV = calloc(cs, sizeof(pel));
    c->qstride = c->W + 2 * JMO_PAD;
    c->qplane = c->qstride * (c->H + 2 * JMO_PAD);
    c->qpel = malloc((size_t)16 * c->qplane * sizeof(pel));
    c->mv = calloc(2 * n4, sizeof(int16_t));
    c->refidx = calloc(n4, 1);
    c->ipred = calloc(n4, 1);
    c->tmv = calloc(2 * n4, sizeof(int16_t));
    c->tref = malloc(n4);
    c->mbintra = calloc((size_t)c->mbw * c->mbh, 1);
    c->res = calloc((size_t)c->mbw * c->mbh, sizeof(jmh_mb_result));
    c->blocksad = malloc(sizeof(uint16_t) * 16 * (size_t)c->npos);
    c->cabi = calloc((size_t)c->mbw * c->mbh, sizeof(jmo_cabmbi));
    c->cab_mvd = calloc((size_t)(c->W / 4) * (c->H / 4) * 2, sizeof(int16_t));
    c->cav_tc = calloc((size_t)c->mbw * c->mbh, 24);
    c->epzs_fp = calloc(8 * n4, sizeof(uint16_t));
    if (!c->orgY || !c->qpel || !c->res || !c->blocksad || !c->tmv || !c->tref || !c->cabi || !c->cab_mvd || !c->cav_tc || !c->epzs_fp) { jmo_destroy(c); return JMH_E_OOM; }
    memset(c->refidx, -1, n4);                             /* no previous picture: no motion */
    *out = c;
    return JMH_OK;
}

void jmo_destroy(jmo_ctx *c) {
    if (!c) return;
    free(c->spiral_x); free(c->spiral_y); free(c->spiral_of);
    free(c->orgY); free(c->orgU); free(c->orgV);
    free(c->refY); free(c->refU); free(c->refV);
    free(c->recY); free(c->recU); free(c->recV);
    free(c->qpel); free(c->mv); free(c->refidx); free(c->ipred); free(c->mbintra);
    free(c->res); free(c->blocksad); free(c->tmv); free(c->tref); free(c->cabi); free(c->cab_mvd); free(c->cav_tc); free(c->epzs_fp);
    free(c);
}

/* pictures enter as 8-bit (uint8_t entry points, bit depth 8) or 16-bit samples (the _u16 ones,
 * High 10): stored as pel either way; a sample above (1 << bit depth) - 1 is an argument error */
static int copy_plane(pel *dst, int dw, int dh, const void *src, int stride, int wide, int maxv) {
    for (int y = 0; y < dh; y++)
        for (int x = 0; x < dw; x++) {
            int v = wide ? ((const uint16_t *)src)[(size_t)y * stride + x] : ((const uint8_t *)src)[(size_t)y * stride + x];
            if (v > maxv) return JMH_E_INVALID_ARG;
            dst[(size_t)y * dw + x] = (pel)v;
        }
    return JMH_OK;
}
static int copy_pic(const jmo_ctx *c, pel *Y, pel *U, pel *V, const void *y, const void *u, const void *v, int sy, int sc,
                    int wide) {
    if ((c->bd > 8) != wide) return JMH_E_UNSUPPORTED_CFG;    /* 8-bit entry points <-> bit depth 8 */
    int r = copy_plane(Y, c->W, c->H, y, sy, wide, c->maxv);
    if (!r) r = copy_plane(U, c->Wc, c->Hc, u, sc, wide, c->maxv);
    if (!r) r = copy_plane(V, c->Wc, c->Hc, v, sc, wide, c->maxv);
    return r;
}

static int set_reference(jmo_ctx *c, const void *y, const void *u, const void *v, int stride_y, int stride_c, int wide) {
    if (!c || !y || !u || !v) return JMH_E_INVALID_ARG;
    int r = copy_pic(c, c->refY, c->refU, c->refV, y, u, v, stride_y, stride_c, wide);
    if (r) return r;
    jmo_build_qpel(c);
    c->have_ref = 1;
    return JMH_OK;
}
int jmo_set_reference(jmo_ctx *c, const uint8_t *y, const uint8_t *u, const uint8_t *v, int stride_y, int stride_c) {
    return set_reference(c, y, u, v, stride_y, stride_c, 0);
}
int jmo_set_reference_u16(jmo_ctx *c, const uint16_t *y, const uint16_t *u, const uint16_t *v, int stride_y, int stride_c) {
    return set_reference(c, y, u, v, stride_y, stride_c, 1);
}

int jmo_load_current(jmo_ctx *c, const uint8_t *y, const uint8_t *u, const uint8_t *v,
                     int stride_y, int stride_c) {
    if (!c || !y || !u || !v) return JMH_E_INVALID_ARG;
    return copy_pic(c, c->orgY, c->orgU, c->orgV, y, u, v, stride_y, stride_c, 0);
}

static int encode_frame(jmo_ctx *c, const void *y, const void *u, const void *v, int stride_y, int stride_c,
                        const jmh_frame_params *fp, int wide) {
    if (!c || !y || !u || !v || !fp) return JMH_E_INVALID_ARG;
    if (fp->slice_type != JMH_P_SLICE && fp->slice_type != JMH_I_SLICE) return JMH_E_UNSUPPORTED_CFG;
    if (fp->slice_type == JMH_P_SLICE && !c->have_ref) return JMH_E_STATE;
    if (fp->qp < 0 || fp->qp > 51) return JMH_E_INVALID_ARG;
    int r = copy_pic(c, c->orgY, c->orgU, c->orgV, y, u, v, stride_y, stride_c, wide);
    if (r) return r;
    c->fp = *fp;
    size_t n4 = (size_t)c->W * c->H / 16;
    memcpy(c->tmv, c->mv, 2 * n4 * sizeof(int16_t));     /* EPZS temporal predictors: the last */
    memcpy(c->tref, c->refidx, n4);                       /* encoded picture's motion field     */
    memset(c->mv, 0, 2 * n4 * sizeof(int16_t));
    memset(c->refidx, -1, n4);
    memset(c->ipred, 2, n4);
    for (int my = 0; my < c->mbh; my++)
        for (int mx = 0; mx < c->mbw; mx++) {
            if (c->cfg.rdo) jmo_encode_mb_rdo(c, mx, my);
            else jmo_encode_mb(c, mx, my);
        }
    return JMH_OK;
}
int jmo_encode_frame(jmo_ctx *c, const uint8_t *y, const uint8_t *u, const uint8_t *v, int stride_y, int stride_c,
                     const jmh_frame_params *fp) {
    return encode_frame(c, y, u, v, stride_y, stride_c, fp, 0);
}
int jmo_encode_frame_u16(jmo_ctx *c, const uint16_t *y, const uint16_t *u, const uint16_t *v, int stride_y,
                         int stride_c, const jmh_frame_params *fp) {
    return encode_frame(c, y, u, v, stride_y, stride_c, fp, 1);
}

const jmh_mb_result *jmo_mb_result(const jmo_ctx *c, int mb_addr) {
    if (!c || mb_addr < 0 || mb_addr >= c->mbw * c->mbh) return NULL;
    return &c->res[mb_addr];
}

static void out_plane(void *dst, int stride, const pel *src, int w, int h, int wide) {
    for (int y = 0; y < h; y++)
        for (int x = 0; x < w; x++) {
            if (wide) ((uint16_t *)dst)[(size_t)y * stride + x] = src[(size_t)y * w + x];
            else ((uint8_t *)dst)[(size_t)y * stride + x] = (uint8_t)src[(size_t)y * w + x];
        }
}
static int read_recon(const jmo_ctx *c, void *y, void *u, void *v, int stride_y, int stride_c, int wide) {
    if (!c) return JMH_E_INVALID_ARG;
    if ((c->bd > 8) != wide) return JMH_E_UNSUPPORTED_CFG;
    out_plane(y, stride_y, c->recY, c->W, c->H, wide);
    out_plane(u, stride_c, c->recU, c->Wc, c->Hc, wide);
    out_plane(v, stride_c, c->recV, c->Wc, c->Hc, wide);
    return JMH_OK;
}
int jmo_read_recon(const jmo_ctx *c, uint8_t *y, uint8_t *u, uint8_t *v, int stride_y, int stride_c) {
    return read_recon(c, y, u, v, stride_y, stride_c, 0);
}
int jmo_read_recon_u16(const jmo_ctx *c, uint16_t *y, uint16_t *u, uint16_t *v, int stride_y, int stride_c) {
    return read_recon(c, y, u, v, stride_y, stride_c, 1);
}

int jmo_read_qpel(const jmo_ctx *c, uint8_t *out) {
    if (!c || !c->have_ref) return JMH_E_STATE;
    if (c->bd > 8) return JMH_E_UNSUPPORTED_CFG;
    for (size_t i = 0; i < (size_t)16 * c->qplane; i++) out[i] = (uint8_t)c->qpel[i];
    return JMH_OK;
}

/* SetupFastFullPelSearch's 4x4 SAD table for explicit window centres (unit seam) */
int jmo_ffs_sad_table(jmo_ctx *c, int n_mb, const int32_t *mb_xy, const int32_t *centres,
                      uint16_t *out) {
    if (!c || n_mb < 0) return JMH_E_INVALID_ARG;
    int sr = c->sr, side = 2 * sr + 1;
    for (int i = 0; i < n_mb; i++) {
        int px = 16 * mb_xy[2 * i], py = 16 * mb_xy[2 * i + 1];
        if (mb_xy[2 * i] < 0 || mb_xy[2 * i] >= c->mbw || mb_xy[2 * i + 1] < 0 || mb_xy[2 * i + 1] >= c->mbh)
            return JMH_E_INVALID_ARG;
        int cx = centres[2 * i], cy = centres[2 * i + 1];
        uint16_t *o = out + (size_t)i * 16 * c->npos;
        for (int dy = -sr; dy <= sr; dy++)
            for (int dx = -sr; dx <= sr; dx++) {
                int r = (dy + sr) * side + dx + sr;
                for (int b = 0; b < 16; b++) {
                    int ox = (b & 3) * 4, oy = (b >> 2) * 4, sad = 0;
                    for (int y = 0; y < 4; y++)
                        for (int x = 0; x < 4; x++) {
                            int ax = iclip(0, c->W - 1, px + cx + dx + ox + x);
                            int ay = iclip(0, c->H - 1, py + cy + dy + oy + y);
                            sad += iabs(c->orgY[(py + oy + y) * c->W + px + ox + x] - c->refY[ay * c->W + ax]);
                        }
                    o[(size_t)b * c->npos + r] = (uint16_t)sad;
                }
            }
    }
    return JMH_OK;
}
