/*
 * hbd.c — the High 10 (9 / 10-bit luma) restatement of the per-block seams (TEST
 * INFRASTRUCTURE ONLY; see jm_oracle.h).  JM >= 10 builds with imgpel = unsigned short and
 * carries the bit depth through img->bitdepth_luma, img->max_imgpel_value and
 * img->bitdepth_luma_qp_scale [J]; the hot-path arithmetic is the 8-bit one on wider samples:
 *   - SAD / SATD (mv-search.c › FastFullPelBlockMotionSearch / FullPelBlockMotionSearch /
 *     SubPelBlockMotionSearch, SATD) on 16-bit differences;
 *   - quarter-pel samples of H.264 8.4.2.2.1 with Clip1Y = clip(0, (1 << BitDepthY) - 1);
 *   - dct_luma / dct_luma8x8 (block.c) at qp + QpBdOffsetY (qp_per / qp_rem / q_bits from
 *     qp + 6 * (bit_depth - 8)), the rounding offsets of the 8-bit restatement (JM_SEMANTICS
 *     item 1), reconstruction clipped to (1 << bit_depth) - 1 (JM_SEMANTICS items 41-44).
 * Written independently of the 8-bit functions in encode.c / common.c (shared: transform
 * cores, tables, spiral, mvbits), so bit_depth 8 on 16-bit samples cross-checks both.
 * JM parity unpinned: no JM source exists in /root/reference.
 */
#include <stdlib.h>
#include "jmo_internal.h"

struct jmo_hbd {
    int W, H, sr, bd, maxv;
    uint16_t *cur, *ref;                  /* coded-size luma, stride W */
    int32_t *sx, *sy;                     /* spiral of the context's search range */
};

int jmo_hbd_create(int W, int H, int sr, jmo_hbd **out) {
    if (!out || W <= 0 || H <= 0 || (W & 15) || (H & 15) || sr < 0 || sr > JMO_MAX_SR) return JMH_E_INVALID_ARG;
    jmo_hbd *h = (jmo_hbd *)calloc(1, sizeof(jmo_hbd));
    if (!h) return JMH_E_OOM;
    h->W = W; h->H = H; h->sr = sr; h->bd = 8; h->maxv = 255;
    const int np = (2 * sr + 1) * (2 * sr + 1);
    h->cur = (uint16_t *)calloc((size_t)W * H, 2);
    h->ref = (uint16_t *)calloc((size_t)W * H, 2);
    h->sx = (int32_t *)malloc(np * sizeof(int32_t));
    h->sy = (int32_t *)malloc(np * sizeof(int32_t));
    if (!h->cur || !h->ref || !h->sx || !h->sy) { jmo_hbd_destroy(h); return JMH_E_OOM; }
    jmo_spiral(sr, h->sx, h->sy);
    *out = h;
    return JMH_OK;
}

void jmo_hbd_destroy(jmo_hbd *h) {
    if (!h) return;
    free(h->cur); free(h->ref); free(h->sx); free(h->sy);
    free(h);
}

int jmo_hbd_pictures(jmo_hbd *h, const uint16_t *cur, const uint16_t *ref, int stride, int bit_depth) {
    if (!h || !cur || !ref || stride < h->W || bit_depth < 8 || bit_depth > 10) return JMH_E_INVALID_ARG;
    h->bd = bit_depth;
    h->maxv = (1 << bit_depth) - 1;
    for (int y = 0; y < h->H; y++)
        for (int x = 0; x < h->W; x++) {
            h->cur[y * h->W + x] = cur[(size_t)y * stride + x];
            h->ref[y * h->W + x] = ref[(size_t)y * stride + x];
        }
    return JMH_OK;
}

static inline int rp(const jmo_hbd *h, int x, int y) { return h->ref[iclip(0, h->H - 1, y) * h->W + iclip(0, h->W - 1, x)]; }
static inline int t6(int a, int b, int c, int d, int e, int f) { return a - 5 * b + 20 * c + 20 * d - 5 * e + f; }
static inline int hclip(const jmo_hbd *h, int v) { return iclip(0, h->maxv, v); }
static int hb1(const jmo_hbd *h, int x, int y) { return t6(rp(h, x - 2, y), rp(h, x - 1, y), rp(h, x, y), rp(h, x + 1, y), rp(h, x + 2, y), rp(h, x + 3, y)); }
static int vh1(const jmo_hbd *h, int x, int y) { return t6(rp(h, x, y - 2), rp(h, x, y - 1), rp(h, x, y), rp(h, x, y + 1), rp(h, x, y + 2), rp(h, x, y + 3)); }

/* luma sample at quarter-pel position (X, Y) of the reference (H.264 8.4.2.2.1, Clip1Y) */
int jmo_hbd_qpel(const jmo_hbd *h, int X, int Y) {
    const int x = X >> 2, y = Y >> 2, fx = X & 3, fy = Y & 3;
    const int G = rp(h, x, y);
    if (!fx && !fy) return G;
    const int b = hclip(h, (hb1(h, x, y) + 16) >> 5), hh = hclip(h, (vh1(h, x, y) + 16) >> 5);
    const int s = hclip(h, (hb1(h, x, y + 1) + 16) >> 5), m = hclip(h, (vh1(h, x + 1, y) + 16) >> 5);
    const int j = hclip(h, (t6(vh1(h, x - 2, y), vh1(h, x - 1, y), vh1(h, x, y), vh1(h, x + 1, y), vh1(h, x + 2, y), vh1(h, x + 3, y)) + 512) >> 10);
    switch (fy * 4 + fx) {
    case 1: return (G + b + 1) >> 1;
    case 2: return b;
    case 3: return (rp(h, x + 1, y) + b + 1) >> 1;
    case 4: return (G + hh + 1) >> 1;
    case 5: return (b + hh + 1) >> 1;
    case 6: return (b + j + 1) >> 1;
    case 7: return (b + m + 1) >> 1;
    case 8: return hh;
    case 9: return (hh + j + 1) >> 1;
    case 10: return j;
    case 11: return (j + m + 1) >> 1;
    case 12: return (rp(h, x, y + 1) + hh + 1) >> 1;
    case 13: return (hh + s + 1) >> 1;
    case 14: return (j + s + 1) >> 1;
    default: return (m + s + 1) >> 1;
    }
}

static int mvc(int lf, int shift, int cx, int cy, int px, int py) {   /* MV_COST [J] */
    return (lf * (jmo_mvbits(cx * (1 << shift) - px) + jmo_mvbits(cy * (1 << shift) - py))) >> 16;
}

/* SAD of the w x h block at picture position (px0, py0) displaced by (mx, my) (UMV clamping) */
static int block_sad(const jmo_hbd *h, int px0, int py0, int w, int hh, int mx, int my) {
    int sad = 0;
    for (int y = 0; y < hh; y++)
        for (int x = 0; x < w; x++) sad += iabs(h->cur[(py0 + y) * h->W + px0 + x] - rp(h, px0 + mx + x, py0 + my + y));
    return sad;
}

/* BlockMotionSearch [J] for one request on the 16-bit pictures: full pel (FFS: the (0,0)
 * pre-check, then the spiral around the centre, strict '<'; full search: the spiral around the
 * block's own centre with the 16x16 zero-vector bias), then SubPelBlockMotionSearch (half-pel
 * pass 9 candidates, quarter-pel pass 8, SATD summed over the 4x4 sub-blocks, strict '<') */
static void hbd_search(const jmo_hbd *h, int had, const jmh_block_search *q, jmh_block_result *r) {
    const int bt = q->blocktype, bw = jmo_blc_size[bt][0], bh = jmo_blc_size[bt][1];
    const int px0 = 16 * q->mb_x + 4 * q->block_x, py0 = 16 * q->mb_y + 4 * q->block_y;
    const int lf = q->lambda_factor, pmx = q->pred_mv[0], pmy = q->pred_mv[1];
    const int np = (2 * q->search_range + 1) * (2 * q->search_range + 1);
    int min_mcost = BIGCOST, fmx = 0, fmy = 0;
    if (q->search_mode == 0) {
        min_mcost = block_sad(h, px0, py0, bw, bh, 0, 0) + mvc(lf, 2, 0, 0, pmx, pmy);   /* (0,0) first */
        for (int p = 0; p < np; p++) {
            const int mx = q->centre[0] + h->sx[p], my = q->centre[1] + h->sy[p];
            const int c = block_sad(h, px0, py0, bw, bh, mx, my) + mvc(lf, 2, mx, my, pmx, pmy);
            if (c < min_mcost) { min_mcost = c; fmx = mx; fmy = my; }
        }
    } else {
        const int check00 = bt == 1 && q->slice_p;
        for (int p = 0; p < np; p++) {
            const int mx = q->centre[0] + h->sx[p], my = q->centre[1] + h->sy[p];
            int c = mvc(lf, 2, mx, my, pmx, pmy);
            if (check00 && mx == 0 && my == 0) c -= (lf * 16) >> 16;
            c += block_sad(h, px0, py0, bw, bh, mx, my);
            if (c < min_mcost) { min_mcost = c; fmx = mx; fmy = my; }
        }
    }
    r->fullpel_mv[0] = fmx; r->fullpel_mv[1] = fmy; r->fullpel_cost = min_mcost;
    if (had) min_mcost = BIGCOST;
    const int check0 = bt == 1 && fmx == 0 && fmy == 0 && had && q->slice_p;
    int qx = 4 * fmx, qy = 4 * fmy;
    for (int pass = 0; pass < 2; pass++) {
        const int step = pass == 0 ? 2 : 1, min_pos = pass == 0 ? (had ? 0 : 1) : 1;
        int best = 0;
        for (int pos = min_pos; pos < 9; pos++) {
            const int cx = qx + step * h->sx[pos], cy = qy + step * h->sy[pos];
            int c = mvc(lf, 0, cx, cy, pmx, pmy);
            if (pass == 0 && check0 && pos == 0) c -= (lf * 16) >> 16;
            for (int by = 0; by < bh; by += 4)
                for (int bx = 0; bx < bw; bx += 4) {
                    int32_t d[16];
                    for (int y = 0; y < 4; y++)
                        for (int x = 0; x < 4; x++)
                            d[4 * y + x] = h->cur[(py0 + by + y) * h->W + px0 + bx + x] -
                                           jmo_hbd_qpel(h, 4 * (px0 + bx + x) + cx, 4 * (py0 + by + y) + cy);
                    c += jmo_satd_block(d, had);
                }
            if (c < min_mcost) { min_mcost = c; best = pos; }
        }
        qx += step * h->sx[best];
        qy += step * h->sy[best];
    }
    r->mv[0] = qx; r->mv[1] = qy; r->min_mcost = min_mcost;
}

int jmo_hbd_block_motion_search(const jmo_hbd *h, int had, int n, const jmh_block_search *req, jmh_block_result *res) {
    if (!h || n <= 0 || !req || !res) return JMH_E_INVALID_ARG;
    for (int i = 0; i < n; i++) {
        const jmh_block_search *q = &req[i];
        if (q->blocktype < 1 || q->blocktype > 7 || q->search_range < 0 || q->search_range > h->sr) return JMH_E_INVALID_ARG;
        if (q->search_mode != 0 && q->search_mode != -1) return JMH_E_UNSUPPORTED_CFG;
        hbd_search(h, had, q, &res[i]);
    }
    return JMH_OK;
}

/* SetupFastFullPelSearch's 4x4 BlockSAD table: out[n_mb][16][(2 sr + 1)^2], window raster */
int jmo_hbd_sad_table(const jmo_hbd *h, int n_mb, const int32_t *mb_xy, const int32_t *centres, uint16_t *out) {
    if (!h || n_mb <= 0 || !mb_xy || !centres || !out) return JMH_E_INVALID_ARG;
    const int sr = h->sr, side = 2 * sr + 1, np = side * side;
    for (int i = 0; i < n_mb; i++) {
        const int px = 16 * mb_xy[2 * i], py = 16 * mb_xy[2 * i + 1];
        for (int r = 0; r < np; r++) {
            const int dx = r % side - sr + centres[2 * i], dy = r / side - sr + centres[2 * i + 1];
            for (int b = 0; b < 16; b++)
                out[((size_t)i * 16 + b) * np + r] = (uint16_t)block_sad(h, px + (b & 3) * 4, py + (b >> 2) * 4, 4, 4, dx, dy);
        }
    }
    return JMH_OK;
}

/* dct_luma [J] at qp + QpBdOffsetY: levels (scan order), recon clipped to (1 << bd) - 1 */
int jmo_hbd_tq4x4_batch(int n, const int16_t *resid, const uint16_t *pred, int qp, int intra, int bd, int16_t *levels, uint16_t *recon,
                        int32_t *coeff_cost, int32_t *nonzero) {
    if (n < 0 || qp < 0 || qp > 51 || bd < 8 || bd > 10 || intra < 0 || intra > JMO_RND_OFF(JMH_QOFFSET_MAX)) return JMH_E_INVALID_ARG;
    const int qpb = qp + 6 * (bd - 8), maxv = (1 << bd) - 1;
    const int qp_per = qpb / 6, qp_rem = qpb % 6, q_bits = Q_BITS + qp_per;
    const int qp_const = jmo_qround(intra, q_bits);
    for (int i = 0; i < n; i++) {
        int32_t m[16], rr[16];
        for (int k = 0; k < 16; k++) m[k] = resid[16 * i + k];
        jmo_fwd4x4(m);
        int run = -1, nz = 0, cc = 0;
        for (int k = 0; k < 16; k++) {
            const int pos = jmo_scan4x4[k];
            run++;
            const int level = (iabs(m[pos]) * jmo_quant_coef[qp_rem][pos] + qp_const) >> q_bits;
            int ilev = 0;
            levels[16 * i + k] = 0;
            if (level) {
                nz = 1;
                cc += level > 1 ? MAX_VALUE : jmo_coeff_cost_tab[run];
                levels[16 * i + k] = (int16_t)isign(level, m[pos]);
                run = -1;
                ilev = level * jmo_dequant_coef[qp_rem][pos] << qp_per;
            }
            m[pos] = isign(ilev, m[pos]);
        }
        jmo_inverse4x4(m, rr);
        for (int k = 0; k < 16; k++)
            recon[16 * i + k] = (uint16_t)iclip(0, maxv, (rr[k] + (pred[16 * i + k] << DQ_BITS) + DQ_ROUND) >> DQ_BITS);
        coeff_cost[i] = cc;
        nonzero[i] = nz;
    }
    return JMH_OK;
}

/* dct_luma8x8 [J] at qp + QpBdOffsetY: normative 8.5.13.1 dequantisation, recon clipped */
int jmo_hbd_tq8x8_batch(int n, const int16_t *resid, const uint16_t *pred, int qp, int intra, int bd, int16_t *levels, uint16_t *recon,
                        int32_t *coeff_cost, int32_t *nonzero) {
    if (n < 0 || qp < 0 || qp > 51 || bd < 8 || bd > 10 || intra < 0 || intra > JMO_RND_OFF(JMH_QOFFSET_MAX)) return JMH_E_INVALID_ARG;
    const int qpb = qp + 6 * (bd - 8), maxv = (1 << bd) - 1;
    const int qp_per = qpb / 6, qp_rem = qpb % 6, q_bits = Q_BITS_8 + qp_per;
    const int qp_const = jmo_qround(intra, q_bits);
    int scan[64];
    jmo_scan8x8(scan);
    for (int i = 0; i < n; i++) {
        int32_t m[64], rr[64];
        for (int k = 0; k < 64; k++) m[k] = resid[64 * i + k];
        jmo_fwd8x8(m);
        int run = -1, nz = 0, cc = 0;
        for (int k = 0; k < 64; k++) {
            const int pos = scan[k], cls = jmo_class8(pos & 7, pos >> 3);
            run++;
            const int level = (int)(((int64_t)iabs(m[pos]) * jmo_quant8_cls[qp_rem][cls] + qp_const) >> q_bits);
            const int c = isign(level, m[pos]);
            int dq = 0;
            if (level) {
                nz = 1;
                cc += level > 1 ? MAX_VALUE : jmo_coeff_cost8(run);
                run = -1;
                const int ls = 16 * jmo_dequant8_cls[qp_rem][cls];
                dq = qpb >= 36 ? c * ls * (1 << (qp_per - 6)) : (c * ls + (1 << (5 - qp_per))) >> (6 - qp_per);
            }
            levels[64 * i + k] = (int16_t)c;
            m[pos] = dq;
        }
        jmo_inverse8x8(m, rr);
        for (int k = 0; k < 64; k++)
            recon[64 * i + k] = (uint16_t)iclip(0, maxv, (rr[k] + (pred[64 * i + k] << DQ_BITS) + DQ_ROUND) >> DQ_BITS);
        coeff_cost[i] = cc;
        nonzero[i] = nz;
    }
    return JMH_OK;
}
