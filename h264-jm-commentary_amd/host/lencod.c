/*
 * lencod.c — product encoder binary: JM 8.6 lencod.c › main [J] with the macroblock hot path
 * bound to the MI355X C ABI (libjmhip.so).  There is no CPU fallback: if no HIP device is
 * usable the run fails with the jmh_* status, as JM's error() would.
 */
#include <stdlib.h>
#include <string.h>
#include "jmhost.h"

/* 8-bit pictures through the uint8_t entry points, High 10 ones through the _u16 ones */
static int gpu_set_ref(void *ctx, const jm_pic *p) {
    if (p->bd > 8) return jmh_set_reference_u16((jmh_ctx *)ctx, 0, 0, p->Y, p->U, p->V, p->w, p->w / 2);
    return jmh_set_reference((jmh_ctx *)ctx, 0, 0, p->y, p->u, p->v, p->w, p->w / 2);
}
static int gpu_encode(void *ctx, const jm_pic *cur, const jmh_frame_params *fp) {
    int r = cur->bd > 8 ? jmh_frame_submit_u16((jmh_ctx *)ctx, cur->Y, cur->U, cur->V, cur->w, cur->w / 2, fp)
                        : jmh_frame_submit((jmh_ctx *)ctx, cur->y, cur->u, cur->v, cur->w, cur->w / 2, fp);
    return r ? r : jmh_frame_wait((jmh_ctx *)ctx);
}
static const jmh_mb_result *gpu_res(void *ctx, int a) { return jmh_get_mb_result((const jmh_ctx *)ctx, a); }
static int gpu_recon(void *ctx, jm_pic *p) {
    if (p->bd > 8) return jmh_read_recon_u16((jmh_ctx *)ctx, p->Y, p->U, p->V, p->w, p->w / 2);
    return jmh_read_recon((jmh_ctx *)ctx, p->y, p->u, p->v, p->w, p->w / 2);
}
static void gpu_destroy(void *ctx) { jmh_destroy((jmh_ctx *)ctx); }
static int gpu_deblocked(void *ctx, jm_pic *p) {
    if (p->bd > 8) return jmh_read_deblocked_u16((jmh_ctx *)ctx, p->Y, p->U, p->V, p->w, p->w / 2);
    return jmh_read_deblocked((jmh_ctx *)ctx, p->y, p->u, p->v, p->w, p->w / 2);
}
static int gpu_ref_deblocked(void *ctx) { return jmh_set_reference_slot((jmh_ctx *)ctx, -2); }
static int gpu_push(void *ctx, const jm_pic *cur, const jmh_frame_params *fp) {
    if (cur->bd > 8) return jmh_frame_push_u16((jmh_ctx *)ctx, cur->Y, cur->U, cur->V, cur->w, cur->w / 2, fp);
    return jmh_frame_push((jmh_ctx *)ctx, cur->y, cur->u, cur->v, cur->w, cur->w / 2, fp);
}
static int gpu_pop(void *ctx) { return jmh_frame_pop((jmh_ctx *)ctx); }
static int gpu_search_pictures(void *ctx, const jm_pic *cur, const jm_pic *ref) {
    return jmh_search_pictures((jmh_ctx *)ctx, cur->y, ref->y, cur->w);
}
static int gpu_block_search(void *ctx, int n, const jmh_block_search *q, jmh_block_result *r) {
    return jmh_block_motion_search((jmh_ctx *)ctx, n, q, r);
}
static int gpu_tq4x4(void *ctx, int n, const int16_t *resid, const uint8_t *pred, int qp, int intra, int16_t *lev, uint8_t *rec,
                     int32_t *cc, int32_t *nz) {
    return jmh_tq4x4_batch((jmh_ctx *)ctx, n, resid, pred, qp, intra, lev, rec, cc, nz);
}

int main(int argc, char **argv) {
    jm_input inp;
    char err[1024];
    jm_input_defaults(&inp);
    if (jm_configure(&inp, argc, argv, err, sizeof(err))) { fprintf(stderr, "%s\n", err); return 1; }
    jmh_config cfg;
    jm_fill_config(&inp, &cfg);
    /* device deblocking: only the deblocked picture comes back (the recon file, PSNR and the
       next reference are the filtered picture, as in JM) */
    if (!getenv("JMH_HOST_DEBLOCK")) cfg.flags |= JMH_FLAG_NO_RECON_READBACK;
    jmh_ctx *ctx = NULL;
    int r = jmh_create(&cfg, inp.hip_device, &ctx);
    if (r) { fprintf(stderr, "jmh_create failed: %s\n", jmh_strerror(r)); return 2; }
    jm_backend be = {"mi355x-hip", ctx, gpu_set_ref, gpu_encode, gpu_res, gpu_recon, gpu_destroy,
                     gpu_deblocked, gpu_ref_deblocked, gpu_push, gpu_pop, jmh_pipeline_depth(ctx),
                     gpu_search_pictures, gpu_block_search, gpu_tq4x4};
    if (getenv("JMH_HOST_DEBLOCK")) be.read_deblocked = NULL, be.reference_deblocked = NULL;
    jm_stats st;
    r = jm_encode_sequence(&inp, &be, &st, stdout);
    double mp = (double)inp.width * inp.height * st.frames / 1e6;
    if (!r && st.me_tq_ms > 0)
        printf(" ME+TQ throughput (host-observed, incl. PCIe): %.2f MP/s\n", mp / (st.me_tq_ms / 1e3));
    be.destroy(ctx);
    return r ? 3 : 0;
}
