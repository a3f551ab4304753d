/*
 * jm86_check.c — TEST INFRASTRUCTURE: drives the product's JM 8.6 call surface (host/jm86.c:
 * dct_luma, BlockMotionSearch, PartitionMotionSearch) on the MI355X backend (libjmhip.so) and
 * checks every call against this oracle.
 *   jm86_check            exit 0 = every call bit-exact; prints one summary line
 * dct_luma: random residual / prediction blocks at every QP, both rounding offsets, against
 * jmo_tq4x4_batch.  BlockMotionSearch: JM-ordered PartitionMotionSearch calls over a P picture
 * of a synthetic sequence in MB raster order through encode_one_macroblock, on the device,
 * with the oracle's decisions as the backend result: each P macroblock's inter mode, cost and
 * MVs must equal the device searches' (enc_picture follows the oracle's decisions).
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include "jm_oracle.h"
#include "jmhost.h"

static int g_tq(void *ctx, int n, const int16_t *resid, const uint8_t *pred, int qp, int intra, int16_t *lev, uint8_t *rec,
                int32_t *cc, int32_t *nz) {
    return jmh_tq4x4_batch((jmh_ctx *)ctx, n, resid, pred, qp, intra, lev, rec, cc, nz);
}
static int g_search_pictures(void *ctx, const jm_pic *cur, const jm_pic *ref) {
    return jmh_search_pictures((jmh_ctx *)ctx, cur->y, ref->y, cur->w);
}
static int g_block_search(void *ctx, int n, const jmh_block_search *q, jmh_block_result *r) {
    return jmh_block_motion_search((jmh_ctx *)ctx, n, q, r);
}
static jmo_ctx *g_oracle;   /* the backend's decisions come from the oracle (be.ctx is the device's) */
static const jmh_mb_result *o_res(void *c, int a) { (void)c; return jmo_mb_result(g_oracle, a); }

static uint64_t rng = 0x9E3779B97F4A7C15ull;
static uint32_t rnd(void) { rng ^= rng << 13; rng ^= rng >> 7; rng ^= rng << 17; return (uint32_t)(rng >> 11); }

int main(void) {
    const int W = 176, H = 144, SR = 16;
    jm_input inp;
    jm_input_defaults(&inp);
    inp.width = W; inp.height = H; inp.search_range = SR; inp.jm_call_surface = 0;
    jmh_config cfg;
    jm_fill_config(&inp, &cfg);
    jmh_ctx *g = NULL;
    jmo_ctx *o = NULL;
    int r = jmh_create(&cfg, 0, &g);
    if (r) { printf("jmh_create: %s\n", jmh_strerror(r)); return 2; }
    if (jmo_create(&cfg, &o)) { printf("jmo_create failed\n"); return 2; }
    g_oracle = o;
    jm_backend be;
    memset(&be, 0, sizeof(be));
    be.name = "mi355x-hip"; be.ctx = g; be.mb_result = o_res;
    be.tq4x4 = g_tq; be.search_pictures = g_search_pictures; be.block_search = g_block_search;
    jm86_img im;
    if (jm86_init(&im, &inp, &be, W, H)) return 2;
    int bad = 0, calls = 0;
    /* ---- dct_luma vs jmo_tq4x4_batch ---- */
    for (int qp = 0; qp <= 51; qp++)
        for (int intra = 0; intra < 2; intra++) {
            jmh_frame_params fp;
            memset(&fp, 0, sizeof(fp));
            fp.slice_type = intra ? JMH_I_SLICE : JMH_P_SLICE; fp.qp = qp;
            fp.lambda_mode = fp.lambda_motion = jm_lambda_rdo_off(qp);
            jm86_start_picture(&im, &fp, NULL, NULL, NULL);
            img->current_mb_nr = (qp * 7) % (im.mbw * im.mbh);
            start_macroblock();
            for (int b = 0; b < 16; b++) {
                int bx = 4 * (b & 3), by = 4 * (b >> 2);
                int16_t resid[16];
                uint8_t pred[16];
                for (int k = 0; k < 16; k++) {
                    int amp = b < 4 ? 255 : 1 + (int)(rnd() % 64);
                    resid[k] = (int16_t)((int)(rnd() % (2 * amp + 1)) - amp);
                    pred[k] = (uint8_t)(rnd() & 255);
                    img->m7[by + (k >> 2)][bx + (k & 3)] = resid[k];
                    img->mpr[by + (k >> 2)][bx + (k & 3)] = pred[k];
                }
                int cost = 0;
                int nz = dct_luma(bx, by, &cost, 0);
                int16_t lev[16];
                uint8_t rec[16];
                int32_t occ = 0, onz = 0;
                jmo_tq4x4_batch(1, resid, pred, qp, intra, lev, rec, &occ, &onz);
                calls++;
                int ok = nz == onz && cost == occ && !memcmp(lev, img->mb_data[img->current_mb_nr].luma[b], sizeof(lev));
                for (int y = 0; y < 4; y++)
                    ok = ok && !memcmp(rec + 4 * y, img->enc_imgY + (size_t)(img->pix_y + by + y) * W + img->pix_x + bx, 4);
                if (!ok) { if (bad < 5) printf("dct_luma mismatch qp %d intra %d block %d\n", qp, intra, b); bad++; }
            }
        }
    /* ---- BlockMotionSearch / PartitionMotionSearch over a P picture, raster MB order ---- */
    jm_pic cur, ref;
    jm_pic_alloc(&cur, W, H); jm_pic_alloc(&ref, W, H);
    jm_synth_frame(&ref, W, H, 3, 0);
    jm_synth_frame(&cur, W, H, 3, 1);
    jmh_frame_params fp;
    memset(&fp, 0, sizeof(fp));
    fp.slice_type = JMH_I_SLICE; fp.qp = 28; fp.lambda_mode = fp.lambda_motion = jm_lambda_rdo_off(28);
    jmo_encode_frame(o, ref.y, ref.u, ref.v, W, W / 2, &fp);   /* oracle decisions: reference = its I recon */
    jm_pic rec;
    jm_pic_alloc(&rec, W, H);
    jmo_read_recon(o, rec.y, rec.u, rec.v, W, W / 2);
    jmo_set_reference(o, rec.y, rec.u, rec.v, W, W / 2);
    fp.slice_type = JMH_P_SLICE;
    jmo_encode_frame(o, cur.y, cur.u, cur.v, W, W / 2, &fp);
    inp.jm_call_surface = 1;
    jm86_start_picture(&im, &fp, &cur, &rec, NULL);
    int searches0 = 0, mbs = 0;
    for (int a = 0; a < im.mbw * im.mbh; a++) {
        img->current_mb_nr = a;
        start_macroblock();
        int before = img->surface_searches;
        encode_one_macroblock();   /* the inter searches on the device, checked against the oracle's decision */
        searches0 += img->surface_searches - before;
        mbs++;
    }
    printf("jm86_check: dct_luma %d calls, %d mismatches; %d P MBs, %d BlockMotionSearch calls on the device, "
           "%d decisions inconsistent\n", calls, bad, mbs, searches0, img->surface_mismatches);
    int fail = bad || img->surface_mismatches || searches0 == 0;
    jm86_free(&im);
    jmh_destroy(g); jmo_destroy(o);
    jm_pic_free(&cur); jm_pic_free(&ref); jm_pic_free(&rec);
    return fail ? 1 : 0;
}
