// jmhip_abi.hip — the extern "C" boundary (include/jmhip.h) over the gfx950 kernels.
// One context = one HIP device + one HIP stream; device buffers are sized once at create.
// Per picture: H2D of the source (pinned staging) -> 254 wavefront launches at 1080p (one per
// diagonal mbx + 2*mby) -> D2H of the macroblock results and the unfiltered reconstruction.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <vector>
#include "jmh_device.h"

hipError_t jmh_launch_interp(const uint8_t *ref, int W, int H, uint8_t *qpel, int qstride, int qplane, hipStream_t st);
hipError_t jmh_launch_analyse(const DevParams &p, hipStream_t st);
hipError_t jmh_launch_final(const DevParams &p, hipStream_t st);
hipError_t jmh_launch_sad_table(const uint8_t *org, const uint8_t *ref, int W, int H, int sr, int n_mb, const int32_t *mb_xy,
                                const int32_t *centres, uint16_t *out, hipStream_t st);
hipError_t jmh_launch_tq4x4(int n, const int16_t *resid, const uint8_t *pred, int qp, int intra, int16_t *levels, uint8_t *recon,
                            int32_t *cc, int32_t *nz, hipStream_t st);

// JMH_FLAG_KERNEL_TIMING brackets every KT_STRIDE-th diagonal's two launches with events: the
// averages are sampled uniformly over the picture while the event packets stay off most launches
#define KT_STRIDE 8
// ring of begin/end event pairs; completed pairs are folded into `sum` (ms)
struct EvRing {
    std::vector<hipEvent_t> a, b;
    int cap = 0, head = 0, count = 0, n = 0;
    float sum = 0;
};
static int ring_init(EvRing &r, int cap) {
    r.cap = cap; r.head = r.count = r.n = 0; r.sum = 0;
    r.a.assign(cap, nullptr); r.b.assign(cap, nullptr);
    for (int i = 0; i < cap; i++)
        if (hipEventCreate(&r.a[i]) != hipSuccess || hipEventCreate(&r.b[i]) != hipSuccess) return -1;
    return 0;
}
static void ring_free(EvRing &r) {
    for (int i = 0; i < r.cap; i++) {
        if (r.a[i]) (void)hipEventDestroy(r.a[i]);
        if (r.b[i]) (void)hipEventDestroy(r.b[i]);
    }
    r.cap = 0;
}
static void ring_fold_oldest(EvRing &r) {
    int i = (r.head - r.count + r.cap) % r.cap;
    float ms = 0;
    if (hipEventSynchronize(r.b[i]) == hipSuccess && hipEventElapsedTime(&ms, r.a[i], r.b[i]) == hipSuccess) {
        r.sum += ms;
        r.n++;
    }
    r.count--;
}
static hipError_t ring_begin(EvRing &r, hipStream_t st) {
    if (r.count == r.cap) ring_fold_oldest(r);
    return hipEventRecord(r.a[r.head], st);
}
static hipError_t ring_end(EvRing &r, hipStream_t st) {
    hipError_t e = hipEventRecord(r.b[r.head], st);
    r.head = (r.head + 1) % r.cap;
    r.count++;
    return e;
}
static void ring_drain(EvRing &r, float &sum, int &n) {
    while (r.count) ring_fold_oldest(r);
    sum = r.sum; n = r.n;
    r.sum = 0; r.n = 0;
}

struct jmh_ctx {
    jmh_config cfg;
    int dev;
    hipStream_t st;
    int W, H, Wc, Hc, mbw, mbh, sr, side, npos, qstride, qplane;
    size_t fsize;                        // bytes of one 4:2:0 picture (Y then U then V)
    uint8_t *d_cur, *d_ref, *d_qpel, *d_rec, *d_slots;
    uint8_t *d_dbk;                      // deblocked reconstruction (next reference); swapped with d_ref
    int nslots;
    int16_t *d_mv;
    int8_t *d_refidx, *d_ipred;
    jmh_mb_result *d_res;
    MbScratch *d_scr;
    unsigned long long *d_prof;          // JMH_PHASE_PROF=<mb>: per-phase wall clock of one MB
    int prof_mb;
    jmh_mb_result *h_res;
    uint8_t *h_rec, *h_dbk, *h_stage_cur, *h_stage_ref;
    int have_ref, pending, have_results, have_total;
    int dbk_dev, dbk_host;               // d_dbk / h_dbk hold the last picture's deblocking
    hipEvent_t ev_t0, ev_t1;
    EvRing ring_interp, ring_mb, ring_an, ring_fin;   // ring_an / ring_fin: JMH_FLAG_KERNEL_TIMING
    jmh_timing timing;
    std::vector<int> dcount, dymin;
};

#define HCHK(x)                                                                  \
    do {                                                                         \
        hipError_t e_ = (x);                                                     \
        if (e_ != hipSuccess) {                                                  \
            fprintf(stderr, "jmhip: %s failed: %s\n", #x, hipGetErrorString(e_)); \
            return JMH_E_HIP;                                                    \
        }                                                                        \
    } while (0)

extern "C" {

int jmh_abi_version(void) { return JMH_ABI_VERSION; }

const char *jmh_strerror(int s) {
    switch (s) {
    case JMH_OK: return "ok";
    case JMH_E_INVALID_ARG: return "invalid argument";
    case JMH_E_HIP: return "HIP runtime error";
    case JMH_E_OOM: return "out of memory";
    case JMH_E_UNSUPPORTED_CFG: return "unsupported configuration";
    case JMH_E_STATE: return "invalid call order";
    case JMH_E_NO_DEVICE: return "no HIP device";
    }
    return "unknown status";
}

int jmh_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}

void jmh_destroy(jmh_ctx *c) {
    if (!c) return;
    (void)hipSetDevice(c->dev);
    if (c->st) (void)hipStreamSynchronize(c->st);
    void *dev_bufs[] = {c->d_cur, c->d_ref, c->d_qpel, c->d_rec, c->d_dbk, c->d_slots, c->d_mv, c->d_refidx,
                        c->d_ipred, c->d_res, c->d_scr, c->d_prof};
    for (void *p : dev_bufs) if (p) (void)hipFree(p);
    void *host_bufs[] = {c->h_res, c->h_rec, c->h_dbk, c->h_stage_cur, c->h_stage_ref};
    for (void *p : host_bufs) if (p) (void)hipHostFree(p);
    if (c->ev_t0) (void)hipEventDestroy(c->ev_t0);
    if (c->ev_t1) (void)hipEventDestroy(c->ev_t1);
    ring_free(c->ring_interp);
    ring_free(c->ring_mb);
    ring_free(c->ring_an);
    ring_free(c->ring_fin);
    if (c->st) (void)hipStreamDestroy(c->st);
    delete c;
}

int jmh_create(const jmh_config *cfg, int hip_device, jmh_ctx **out) {
    if (!cfg || !out) return JMH_E_INVALID_ARG;
    *out = nullptr;
    if (cfg->width <= 0 || cfg->height <= 0 || (cfg->width & 15) || (cfg->height & 15)) return JMH_E_INVALID_ARG;
    if (cfg->search_range < 1 || cfg->search_range > 64) return JMH_E_INVALID_ARG;
    if (cfg->search_range > SRMAX) return JMH_E_UNSUPPORTED_CFG;            // LDS-resident window
    if (cfg->search_mode != 0) return JMH_E_UNSUPPORTED_CFG;                // FFS (SearchMode 0)
    if (cfg->num_ref_frames != 1 || cfg->constrained_intra_pred) return JMH_E_UNSUPPORTED_CFG;
    if (cfg->restrict_search_range < 0 || cfg->restrict_search_range > 2) return JMH_E_INVALID_ARG;
    int ndev = jmh_device_count();
    if (ndev <= 0) return JMH_E_NO_DEVICE;
    if (hip_device < 0 || hip_device >= ndev) return JMH_E_INVALID_ARG;
    jmh_ctx *c = new jmh_ctx();
    memset((void *)&c->cfg, 0, sizeof(c->cfg));
    c->cfg = *cfg;
    c->dev = hip_device;
    HCHK(hipSetDevice(hip_device));
    c->W = cfg->width; c->H = cfg->height; c->Wc = c->W / 2; c->Hc = c->H / 2;
    c->mbw = c->W / 16; c->mbh = c->H / 16;
    c->sr = cfg->search_range; c->side = 2 * c->sr + 1; c->npos = c->side * c->side;
    c->qstride = c->W + 2 * QPAD; c->qplane = c->qstride * (c->H + 2 * QPAD);
    c->fsize = (size_t)c->W * c->H * 3 / 2;
    c->nslots = cfg->num_frame_slots > 0 ? cfg->num_frame_slots : 1;
    int st = JMH_OK;
#define ALLOC(p, n) do { if (hipMalloc((void **)&(p), (n)) != hipSuccess) { st = JMH_E_OOM; goto fail; } } while (0)
#define HALLOC(p, n) do { if (hipHostMalloc((void **)&(p), (n), hipHostMallocDefault) != hipSuccess) { st = JMH_E_OOM; goto fail; } } while (0)
    {
        if (hipStreamCreateWithFlags(&c->st, hipStreamNonBlocking) != hipSuccess) { st = JMH_E_HIP; goto fail; }
        size_t n4 = (size_t)c->W * c->H / 16, nmb = (size_t)c->mbw * c->mbh;
        ALLOC(c->d_cur, c->fsize); ALLOC(c->d_ref, c->fsize); ALLOC(c->d_rec, c->fsize); ALLOC(c->d_dbk, c->fsize);
        ALLOC(c->d_qpel, (size_t)16 * c->qplane);
        ALLOC(c->d_slots, c->fsize * c->nslots);
        ALLOC(c->d_mv, n4 * 2 * sizeof(int16_t)); ALLOC(c->d_refidx, n4); ALLOC(c->d_ipred, n4);
        ALLOC(c->d_res, nmb * sizeof(jmh_mb_result));
        ALLOC(c->d_scr, nmb * sizeof(MbScratch));
        c->prof_mb = -1;
        if (const char *e = getenv("JMH_PHASE_PROF")) {
            c->prof_mb = atoi(e);
            ALLOC(c->d_prof, 64 * sizeof(unsigned long long));
            if (hipMemset(c->d_prof, 0, 64 * sizeof(unsigned long long)) != hipSuccess) { st = JMH_E_HIP; goto fail; }
        }
        HALLOC(c->h_res, nmb * sizeof(jmh_mb_result)); HALLOC(c->h_rec, c->fsize); HALLOC(c->h_dbk, c->fsize);
        HALLOC(c->h_stage_cur, c->fsize); HALLOC(c->h_stage_ref, c->fsize);
        if (hipMemset(c->d_rec, 0, c->fsize) != hipSuccess || hipMemset(c->d_ref, 0, c->fsize) != hipSuccess) { st = JMH_E_HIP; goto fail; }
        if (hipEventCreate(&c->ev_t0) != hipSuccess || hipEventCreate(&c->ev_t1) != hipSuccess ||
            ring_init(c->ring_interp, 64) || ring_init(c->ring_mb, 64) ||
            ((cfg->flags & JMH_FLAG_KERNEL_TIMING) && (ring_init(c->ring_an, 2048) || ring_init(c->ring_fin, 2048)))) { st = JMH_E_HIP; goto fail; }
        int nd = (c->mbw - 1) + 2 * (c->mbh - 1) + 1;
        c->dcount.resize(nd); c->dymin.resize(nd);
        for (int dg = 0; dg < nd; dg++) {
            int ymin = dg - (c->mbw - 1) > 0 ? (dg - (c->mbw - 1) + 1) / 2 : 0;
            int ymax = dg / 2 < c->mbh - 1 ? dg / 2 : c->mbh - 1;
            c->dymin[dg] = ymin;
            c->dcount[dg] = ymax >= ymin ? ymax - ymin + 1 : 0;
        }
    }
#undef ALLOC
#undef HALLOC
    *out = c;
    return JMH_OK;
fail:
    jmh_destroy(c);
    return st;
}

static void pack_planes(uint8_t *dst, int W, int H, const uint8_t *y, const uint8_t *u, const uint8_t *v, int sy, int sc) {
    for (int r = 0; r < H; r++) memcpy(dst + (size_t)r * W, y + (size_t)r * sy, W);
    uint8_t *du = dst + (size_t)W * H, *dv = du + (size_t)W * H / 4;
    for (int r = 0; r < H / 2; r++) {
        memcpy(du + (size_t)r * (W / 2), u + (size_t)r * sc, W / 2);
        memcpy(dv + (size_t)r * (W / 2), v + (size_t)r * sc, W / 2);
    }
}

static int run_interp(jmh_ctx *c, const uint8_t *d_refY) {
    HCHK(ring_begin(c->ring_interp, c->st));
    HCHK(jmh_launch_interp(d_refY, c->W, c->H, c->d_qpel, c->qstride, c->qplane, c->st));
    HCHK(ring_end(c->ring_interp, c->st));
    c->have_ref = 1;
    return JMH_OK;
}

int jmh_set_reference(jmh_ctx *c, int list, int ref_idx, const uint8_t *y, const uint8_t *u, const uint8_t *v, int sy, int sc) {
    if (!c || !y || !u || !v || sy < c->W || sc < c->Wc) return JMH_E_INVALID_ARG;
    if (list != 0 || ref_idx != 0) return JMH_E_UNSUPPORTED_CFG;
    HCHK(hipSetDevice(c->dev));
    HCHK(hipStreamSynchronize(c->st));   // staging buffer reuse
    pack_planes(c->h_stage_ref, c->W, c->H, y, u, v, sy, sc);
    HCHK(hipMemcpyAsync(c->d_ref, c->h_stage_ref, c->fsize, hipMemcpyHostToDevice, c->st));
    return run_interp(c, c->d_ref);
}

int jmh_set_reference_slot(jmh_ctx *c, int slot) {
    if (!c || slot < -2 || slot >= c->nslots) return JMH_E_INVALID_ARG;
    HCHK(hipSetDevice(c->dev));
    if (slot == -2) {   // the device deblocking becomes the reference: swap buffers, no copy
        if (!c->dbk_dev) return JMH_E_STATE;
        uint8_t *t = c->d_ref; c->d_ref = c->d_dbk; c->d_dbk = t;
        c->dbk_dev = 0;
        return run_interp(c, c->d_ref);
    }
    const uint8_t *src = slot < 0 ? c->d_rec : c->d_slots + (size_t)slot * c->fsize;
    HCHK(hipMemcpyAsync(c->d_ref, src, c->fsize, hipMemcpyDeviceToDevice, c->st));
    return run_interp(c, c->d_ref);
}

static int enqueue_encode(jmh_ctx *c, const uint8_t *d_pic, const jmh_frame_params *fp) {
    if (fp->slice_type != JMH_P_SLICE && fp->slice_type != JMH_I_SLICE) return JMH_E_UNSUPPORTED_CFG;
    if (fp->qp < 0 || fp->qp > 51 || fp->lambda_mode < 0 || fp->lambda_motion < 0) return JMH_E_INVALID_ARG;
    if (fp->slice_type == JMH_P_SLICE && !c->have_ref) return JMH_E_STATE;
    DevParams p;
    memset(&p, 0, sizeof(p));
    p.W = c->W; p.H = c->H; p.Wc = c->Wc; p.Hc = c->Hc; p.mbw = c->mbw; p.mbh = c->mbh;
    p.sr = c->sr; p.side = c->side; p.npos = c->npos;
    p.search_mode = c->cfg.search_mode; p.use_hadamard = c->cfg.use_hadamard; p.restrict_sr = c->cfg.restrict_search_range;
    for (int i = 0; i < 8; i++) p.inter_search[i] = c->cfg.inter_search[i];
    p.qstride = c->qstride; p.qplane = c->qplane;
    size_t ls = (size_t)c->W * c->H;
    p.orgY = d_pic; p.orgU = d_pic + ls; p.orgV = d_pic + ls + ls / 4;
    p.refY = c->d_ref; p.refU = c->d_ref + ls; p.refV = c->d_ref + ls + ls / 4;
    p.qpel = c->d_qpel;
    p.recY = c->d_rec; p.recU = c->d_rec + ls; p.recV = c->d_rec + ls + ls / 4;
    p.mv = c->d_mv; p.refidx = c->d_refidx; p.ipred = c->d_ipred; p.res = c->d_res; p.scr = c->d_scr;
    p.prof = c->d_prof; p.prof_mb = c->prof_mb;
    p.slice_type = fp->slice_type; p.qp = fp->qp; p.lambda_mode = fp->lambda_mode; p.lambda_motion = fp->lambda_motion;
    p.cqp_off = fp->chroma_qp_offset;
    if (fp->deblock) {   // DeblockFrame fused into k_mb_final, into d_dbk (never aliases d_ref)
        if (fp->lf_disable < 0 || fp->lf_disable > 2 || fp->lf_alpha_div2 < -6 || fp->lf_alpha_div2 > 6 ||
            fp->lf_beta_div2 < -6 || fp->lf_beta_div2 > 6) return JMH_E_INVALID_ARG;
        p.dbkY = c->d_dbk; p.dbkU = c->d_dbk + ls; p.dbkV = c->d_dbk + ls + ls / 4;
        p.lf_disable = fp->lf_disable;   // idc 2 == 0 with one slice per picture
        p.lf_offA = 2 * fp->lf_alpha_div2; p.lf_offB = 2 * fp->lf_beta_div2;
    }
    c->dbk_dev = fp->deblock != 0;
    HCHK(ring_begin(c->ring_mb, c->st));
    for (size_t dg = 0; dg < c->dcount.size(); dg++) {
        if (!c->dcount[dg]) continue;
        p.diag = (int)dg; p.y_min = c->dymin[dg]; p.ndiag = c->dcount[dg];
        const bool kt = c->ring_an.cap > 0 && dg % KT_STRIDE == 0;   // sampled per-launch timing
        if (kt) HCHK(ring_begin(c->ring_an, c->st));
        HCHK(jmh_launch_analyse(p, c->st));
        if (kt) { HCHK(ring_end(c->ring_an, c->st)); HCHK(ring_begin(c->ring_fin, c->st)); }
        HCHK(jmh_launch_final(p, c->st));
        if (kt) HCHK(ring_end(c->ring_fin, c->st));
    }
    HCHK(ring_end(c->ring_mb, c->st));
    int nl = 0;
    for (int n : c->dcount) nl += 2 * (n > 0);
    c->timing.mb_launches = nl;
    return JMH_OK;
}

int jmh_frame_submit(jmh_ctx *c, const uint8_t *y, const uint8_t *u, const uint8_t *v, int sy, int sc, const jmh_frame_params *fp) {
    if (!c || !y || !u || !v || !fp || sy < c->W || sc < c->Wc) return JMH_E_INVALID_ARG;
    HCHK(hipSetDevice(c->dev));
    HCHK(hipStreamSynchronize(c->st));
    pack_planes(c->h_stage_cur, c->W, c->H, y, u, v, sy, sc);
    HCHK(hipEventRecord(c->ev_t0, c->st));
    HCHK(hipMemcpyAsync(c->d_cur, c->h_stage_cur, c->fsize, hipMemcpyHostToDevice, c->st));
    int r = enqueue_encode(c, c->d_cur, fp);
    if (r) return r;
    HCHK(hipMemcpyAsync(c->h_res, c->d_res, (size_t)c->mbw * c->mbh * sizeof(jmh_mb_result), hipMemcpyDeviceToHost, c->st));
    HCHK(hipMemcpyAsync(c->h_rec, c->d_rec, c->fsize, hipMemcpyDeviceToHost, c->st));
    if (c->dbk_dev) HCHK(hipMemcpyAsync(c->h_dbk, c->d_dbk, c->fsize, hipMemcpyDeviceToHost, c->st));
    c->dbk_host = c->dbk_dev;
    HCHK(hipEventRecord(c->ev_t1, c->st));
    c->pending = 1;
    c->have_total = 1;
    c->have_results = 0;
    return JMH_OK;
}

int jmh_frame_wait(jmh_ctx *c) {
    if (!c) return JMH_E_INVALID_ARG;
    if (!c->pending) return JMH_E_STATE;
    HCHK(hipSetDevice(c->dev));
    HCHK(hipStreamSynchronize(c->st));
    c->pending = 0;
    c->have_results = 1;
    return JMH_OK;
}

const jmh_mb_result *jmh_get_mb_result(const jmh_ctx *c, int mb_addr) {
    if (!c || !c->have_results || mb_addr < 0 || mb_addr >= c->mbw * c->mbh) return nullptr;
    return &c->h_res[mb_addr];
}

static void unpack_planes(const uint8_t *src, int W, int H, uint8_t *y, uint8_t *u, uint8_t *v, int sy, int sc) {
    size_t ls = (size_t)W * H;
    for (int r = 0; r < H; r++) memcpy(y + (size_t)r * sy, src + (size_t)r * W, W);
    for (int r = 0; r < H / 2; r++) {
        memcpy(u + (size_t)r * sc, src + ls + (size_t)r * (W / 2), W / 2);
        memcpy(v + (size_t)r * sc, src + ls + ls / 4 + (size_t)r * (W / 2), W / 2);
    }
}

int jmh_read_recon(jmh_ctx *c, uint8_t *y, uint8_t *u, uint8_t *v, int sy, int sc) {
    if (!c || !y || !u || !v || sy < c->W || sc < c->Wc) return JMH_E_INVALID_ARG;
    if (!c->have_results) return JMH_E_STATE;
    unpack_planes(c->h_rec, c->W, c->H, y, u, v, sy, sc);
    return JMH_OK;
}

int jmh_read_deblocked(jmh_ctx *c, uint8_t *y, uint8_t *u, uint8_t *v, int sy, int sc) {
    if (!c || !y || !u || !v || sy < c->W || sc < c->Wc) return JMH_E_INVALID_ARG;
    if (!c->have_results || !c->dbk_host) return JMH_E_STATE;
    unpack_planes(c->h_dbk, c->W, c->H, y, u, v, sy, sc);
    return JMH_OK;
}

int jmh_load_frame(jmh_ctx *c, int slot, const uint8_t *y, const uint8_t *u, const uint8_t *v, int sy, int sc) {
    if (!c || slot < 0 || slot >= c->nslots || !y || !u || !v || sy < c->W || sc < c->Wc) return JMH_E_INVALID_ARG;
    HCHK(hipSetDevice(c->dev));
    HCHK(hipStreamSynchronize(c->st));
    pack_planes(c->h_stage_cur, c->W, c->H, y, u, v, sy, sc);
    HCHK(hipMemcpyAsync(c->d_slots + (size_t)slot * c->fsize, c->h_stage_cur, c->fsize, hipMemcpyHostToDevice, c->st));
    HCHK(hipStreamSynchronize(c->st));
    return JMH_OK;
}

int jmh_encode_slot(jmh_ctx *c, int slot, const jmh_frame_params *fp) {
    if (!c || !fp || slot < 0 || slot >= c->nslots) return JMH_E_INVALID_ARG;
    HCHK(hipSetDevice(c->dev));
    return enqueue_encode(c, c->d_slots + (size_t)slot * c->fsize, fp);
}

int jmh_sync(jmh_ctx *c) {
    if (!c) return JMH_E_INVALID_ARG;
    HCHK(hipSetDevice(c->dev));
    HCHK(hipStreamSynchronize(c->st));
    if (c->d_prof) {   // debug: phase timestamps of MB prof_mb from the last picture
        unsigned long long h[64];
        int rate_khz = 0;
        HCHK(hipMemcpy(h, c->d_prof, sizeof(h), hipMemcpyDeviceToHost));
        HCHK(hipDeviceGetAttribute(&rate_khz, hipDeviceAttributeWallClockRate, c->dev));
        double us = rate_khz > 0 ? 1e3 / rate_khz : 0.01;
        unsigned long long t0 = ~0ull;
        for (int k = 0; k < 20; k++) if (h[k] && h[k] < t0) t0 = h[k];
        fprintf(stderr, "jmh_phase mb=%d us since first stamp:", c->prof_mb);
        for (int k = 0; k < 64; k++) if (h[k]) fprintf(stderr, " [%d]%.2f", k, (double)(h[k] - t0) * us);
        fprintf(stderr, "\n");
        HCHK(hipMemset(c->d_prof, 0, sizeof(h)));
    }
    return JMH_OK;
}

int jmh_get_timing(jmh_ctx *c, jmh_timing *t) {
    if (!c || !t) return JMH_E_INVALID_ARG;
    HCHK(hipSetDevice(c->dev));
    HCHK(hipStreamSynchronize(c->st));
    float ms = 0;
    ring_drain(c->ring_interp, c->timing.interp_ms, c->timing.interps);
    ring_drain(c->ring_mb, c->timing.mb_ms, c->timing.pictures);
    if (c->ring_an.cap) {
        ring_drain(c->ring_an, c->timing.analyse_ms, c->timing.analyse_launches);
        ring_drain(c->ring_fin, c->timing.final_ms, c->timing.final_launches);
    }
    if (c->have_total && hipEventElapsedTime(&ms, c->ev_t0, c->ev_t1) == hipSuccess) c->timing.total_ms = ms;
    *t = c->timing;
    return JMH_OK;
}

int jmh_ffs_sad_table(jmh_ctx *c, int n_mb, const int32_t *mb_xy, const int32_t *centres, uint16_t *out) {
    if (!c || n_mb <= 0 || !mb_xy || !centres || !out) return JMH_E_INVALID_ARG;
    for (int i = 0; i < n_mb; i++)
        if (mb_xy[2 * i] < 0 || mb_xy[2 * i] >= c->mbw || mb_xy[2 * i + 1] < 0 || mb_xy[2 * i + 1] >= c->mbh) return JMH_E_INVALID_ARG;
    if (!c->have_ref) return JMH_E_STATE;
    HCHK(hipSetDevice(c->dev));
    int32_t *d_xy = nullptr, *d_c = nullptr;
    uint16_t *d_out = nullptr;
    size_t on = (size_t)n_mb * 16 * c->npos;
    HCHK(hipMalloc((void **)&d_xy, n_mb * 8));
    HCHK(hipMalloc((void **)&d_c, n_mb * 8));
    HCHK(hipMalloc((void **)&d_out, on * 2));
    HCHK(hipMemcpyAsync(d_xy, mb_xy, n_mb * 8, hipMemcpyHostToDevice, c->st));
    HCHK(hipMemcpyAsync(d_c, centres, n_mb * 8, hipMemcpyHostToDevice, c->st));
    HCHK(jmh_launch_sad_table(c->d_slots, c->d_ref, c->W, c->H, c->sr, n_mb, d_xy, d_c, d_out, c->st));
    HCHK(hipMemcpyAsync(out, d_out, on * 2, hipMemcpyDeviceToHost, c->st));
    HCHK(hipStreamSynchronize(c->st));
    HCHK(hipFree(d_xy)); HCHK(hipFree(d_c)); HCHK(hipFree(d_out));
    return JMH_OK;
}

int jmh_tq4x4_batch(jmh_ctx *c, int n, const int16_t *resid, const uint8_t *pred, int qp, int intra, int16_t *levels,
                    uint8_t *recon, int32_t *coeff_cost, int32_t *nonzero) {
    if (!c || n <= 0 || !resid || !pred || !levels || !recon || !coeff_cost || !nonzero || qp < 0 || qp > 51) return JMH_E_INVALID_ARG;
    HCHK(hipSetDevice(c->dev));
    int16_t *dr, *dl;
    uint8_t *dp, *drec;
    int32_t *dcc, *dnz;
    HCHK(hipMalloc((void **)&dr, n * 32)); HCHK(hipMalloc((void **)&dl, n * 32));
    HCHK(hipMalloc((void **)&dp, n * 16)); HCHK(hipMalloc((void **)&drec, n * 16));
    HCHK(hipMalloc((void **)&dcc, n * 4)); HCHK(hipMalloc((void **)&dnz, n * 4));
    HCHK(hipMemcpyAsync(dr, resid, n * 32, hipMemcpyHostToDevice, c->st));
    HCHK(hipMemcpyAsync(dp, pred, n * 16, hipMemcpyHostToDevice, c->st));
    HCHK(jmh_launch_tq4x4(n, dr, dp, qp, intra, dl, drec, dcc, dnz, c->st));
    HCHK(hipMemcpyAsync(levels, dl, n * 32, hipMemcpyDeviceToHost, c->st));
    HCHK(hipMemcpyAsync(recon, drec, n * 16, hipMemcpyDeviceToHost, c->st));
    HCHK(hipMemcpyAsync(coeff_cost, dcc, n * 4, hipMemcpyDeviceToHost, c->st));
    HCHK(hipMemcpyAsync(nonzero, dnz, n * 4, hipMemcpyDeviceToHost, c->st));
    HCHK(hipStreamSynchronize(c->st));
    HCHK(hipFree(dr)); HCHK(hipFree(dl)); HCHK(hipFree(dp)); HCHK(hipFree(drec)); HCHK(hipFree(dcc)); HCHK(hipFree(dnz));
    return JMH_OK;
}

/* test seam: quarter-pel planes of the current reference, [16][H+8][W+8] */
int jmh_read_qpel(jmh_ctx *c, uint8_t *out) {
    if (!c || !out) return JMH_E_INVALID_ARG;
    if (!c->have_ref) return JMH_E_STATE;
    HCHK(hipSetDevice(c->dev));
    HCHK(hipMemcpyAsync(out, c->d_qpel, (size_t)16 * c->qplane, hipMemcpyDeviceToHost, c->st));
    HCHK(hipStreamSynchronize(c->st));
    return JMH_OK;
}

}  // extern "C"
