/*
 * lencod_cpu.c — CPU reference encoder (TEST INFRASTRUCTURE / CPU BASELINE ONLY).
 * The product's host plumbing (libjmhost.a: encoder.cfg, frame loop, CAVLC, deblocking) with
 * the macroblock hot path bound to this oracle instead of libjmhip.so.  Its .264 and recon are
 * the parity reference for the MI355X encoder on the same encoder.cfg.
 */
#include <stdlib.h>
#include "jm_oracle.h"
#include "jmhost.h"

static int o_set_ref(void *c, const jm_pic *p) { return jmo_set_reference((jmo_ctx *)c, p->y, p->u, p->v, p->w, p->w / 2); }
static int o_encode(void *c, const jm_pic *p, const jmh_frame_params *fp) {
    return jmo_encode_frame((jmo_ctx *)c, p->y, p->u, p->v, p->w, p->w / 2, fp);
}
static const jmh_mb_result *o_res(void *c, int a) { return jmo_mb_result((const jmo_ctx *)c, a); }
static int o_recon(void *c, jm_pic *p) { return jmo_read_recon((const jmo_ctx *)c, p->y, p->u, p->v, p->w, p->w / 2); }
static void o_destroy(void *c) { jmo_destroy((jmo_ctx *)c); }

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
    jm_backend be = {"cpu-oracle", ctx, o_set_ref, o_encode, o_res, o_recon, o_destroy, NULL, NULL, NULL, NULL, 1};
    jm_stats st;
    r = jm_encode_sequence(&inp, &be, &st, stdout);
    double mp = (double)inp.width * inp.height * st.frames / 1e6;
    if (!r && st.me_tq_ms > 0) printf(" ME+TQ throughput (1 core): %.4f MP/s\n", mp / (st.me_tq_ms / 1e3));
    be.destroy(ctx);
    return r ? 3 : 0;
}
