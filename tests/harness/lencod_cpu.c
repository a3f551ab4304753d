/*
 * lencod_cpu.c — CPU reference encoder (TEST INFRASTRUCTURE / CPU BASELINE ONLY).
 * The product's host plumbing (libjmhost.a: encoder.cfg, frame loop, CAVLC, deblocking) with
 * the macroblock hot path bound to this oracle instead of libjmhip.so.  Its .264 and recon are
 * the parity reference for the MI355X encoder on the same encoder.cfg.
 */
#include <stdlib.h>
#include "jm_oracle.h"
#include "jmhost.h"

static int o_set_ref(void *c, const jm_pic *p) {
    if (p->bd > 8) return jmo_set_reference_u16((jmo_ctx *)c, p->Y, p->U, p->V, p->w, p->w / 2);
    return jmo_set_reference((jmo_ctx *)c, p->y, p->u, p->v, p->w, p->w / 2);
}
static int o_encode(void *c, const jm_pic *p, const jmh_frame_params *fp) {
    if (p->bd > 8) return jmo_encode_frame_u16((jmo_ctx *)c, p->Y, p->U, p->V, p->w, p->w / 2, fp);
    return jmo_encode_frame((jmo_ctx *)c, p->y, p->u, p->v, p->w, p->w / 2, fp);
}
static const jmh_mb_result *o_res(void *c, int a) { return jmo_mb_result((const jmo_ctx *)c, a); }
static int o_recon(void *c, jm_pic *p) {
    if (p->bd > 8) return jmo_read_recon_u16((const jmo_ctx *)c, p->Y, p->U, p->V, p->w, p->w / 2);
    return jmo_read_recon((const jmo_ctx *)c, p->y, p->u, p->v, p->w, p->w / 2);
}
static void o_destroy(void *c) { jmo_destroy((jmo_ctx *)c); }
/* the per-call seams of the JM call surface; jmo_search_pictures loads the same current and
 * reference luma the picture was encoded with (the oracle encodes one picture at a time) */
static int o_search_pictures(void *c, const jm_pic *cur, const jm_pic *ref) {
    return jmo_search_pictures((jmo_ctx *)c, cur->y, ref->y, cur->w);
}
static int o_block_search(void *c, int n, const jmh_block_search *q, jmh_block_result *r) {
    return jmo_block_motion_search((jmo_ctx *)c, n, q, r);
}
static int o_tq4x4(void *c, int n, const int16_t *resid, const uint8_t *pred, int qp, int intra, int16_t *lev, uint8_t *rec,
                   int32_t *cc, int32_t *nz) {
    (void)c;
    return jmo_tq4x4_batch(n, resid, pred, qp, intra, lev, rec, cc, nz);
}

int main(int argc, char **argv) {
    jm_input inp;
    char err[1024];
    jm_input_defaults(&inp);
    if (jm_configure(&inp, argc, argv, err, sizeof(err))) { fprintf(stderr, "%s\n", err); return 1; }
    jmh_config cfg;
    jm_fill_config(&inp, &cfg);
    jmo_ctx *ctx = NULL;
    int r = jmo_create(&cfg, &ctx);
    if (r) { fprintf(stderr, "jmo_create failed: %d\n", r); return 2; }
    jm_backend be = {"cpu-oracle", ctx, o_set_ref, o_encode, o_res, o_recon, o_destroy, NULL, NULL, NULL, NULL, 1,
                     o_search_pictures, o_block_search, o_tq4x4};
    jm_stats st;
    r = jm_encode_sequence(&inp, &be, &st, stdout);
    double mp = (double)inp.width * inp.height * st.frames / 1e6;
    if (!r && st.me_tq_ms > 0) printf(" ME+TQ throughput (1 core): %.4f MP/s\n", mp / (st.me_tq_ms / 1e3));
    be.destroy(ctx);
    return r ? 3 : 0;
}
