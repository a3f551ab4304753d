// jmhip_abi.hip — the extern "C" boundary (include/jmhip.h) over the gfx950 kernels.
// One context = one HIP device + one HIP stream; device buffers are sized once at create.
//
// Pictures run as a pipeline of wavefront ticks.  A picture walks its 254 diagonals (1080p;
// mbx + 2*mby == d); a tick launches k_mb_analyse + k_mb_final once for the next diagonal of
// every picture in flight.  A picture that references the previous one starts once that one is
// PIPE_LAG diagonals ahead, so in steady state ~254/PIPE_LAG pictures share each launch and the
// chip sees hundreds of macroblocks per dispatch instead of <= 34.  Ticks are issued lazily
// from the host (push issues until the new picture has started; pop / sync drain), all on one
// stream, so stream order is the only synchronisation.
//
// Per-picture device state lives in a ring of nring = depth + 2 entries (source, recon,
// deblocked recon, MV / ref_idx / ipred maps, results, MbScratch); an entry is reused only once
// no picture in flight reads or writes it and its results were popped.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <deque>
#include <vector>
#include <algorithm>
#include "jmh_device.h"
#include "jmh_cabac_rate.h"

hipError_t jmh_launch_interp(const uint8_t *ref, int W, int H, uint8_t *qpel, int qstride, int qplane, hipStream_t st);
hipError_t jmh_launch_analyse(const TickArgs &t, hipStream_t st);
hipError_t jmh_launch_intra(const TickArgs &t, hipStream_t st);
hipError_t jmh_launch_final(const TickArgs &t, hipStream_t st);
hipError_t jmh_launch_intra8(const TickArgs &t, hipStream_t st);
hipError_t jmh_launch_me_full(const TickArgs &t, hipStream_t st);
hipError_t jmh_launch_epzs(const TickArgs &t, hipStream_t st);
hipError_t jmh_launch_flow(const FlowArgs &f, hipStream_t st);
hipError_t jmh_launch_rdo(const TickArgs &t, hipStream_t st, hipStream_t side, hipEvent_t fork, hipEvent_t join);
size_t jmh_rdo_scratch_bytes();
hipError_t jmh_launch_block_search_u16(int n, const jmh_block_search *reqs, jmh_block_result *out, const uint16_t *cur, const uint16_t *ref,
                                       int W, int H, int had, int bit_depth, hipStream_t st);
hipError_t jmh_launch_sad_table_u16(const uint16_t *org, const uint16_t *ref, int W, int H, int sr, int n_mb, const int32_t *mb_xy,
                                    const int32_t *centres, uint16_t *out, hipStream_t st);
hipError_t jmh_launch_tq4x4_u16(int n, const int16_t *resid, const uint16_t *pred, int qp, int qsel, int bit_depth, int16_t *levels,
                                uint16_t *recon, int32_t *cc, int32_t *nz, hipStream_t st);
hipError_t jmh_launch_tq8x8_u16(int n, const int16_t *resid, const uint16_t *pred, int qp, int qsel, int bit_depth, int16_t *levels,
                                uint16_t *recon, int32_t *cc, int32_t *nz, hipStream_t st);
hipError_t jmh_launch_sad_table(const uint8_t *org, const uint8_t *ref, int W, int H, int sr, int n_mb, const int32_t *mb_xy,
                                const int32_t *centres, uint16_t *out, hipStream_t st);
hipError_t jmh_launch_tq8x8(int n, const int16_t *resid, const uint8_t *pred, int qp, int qsel, int16_t *levels, uint8_t *recon,
                            int32_t *cc, int32_t *nz, hipStream_t st);
hipError_t jmh_launch_block_search(int n, const jmh_block_search *reqs, jmh_block_result *out, const uint8_t *cur, const uint8_t *ref, int W,
                                   int H, int had, hipStream_t st);
hipError_t jmh_launch_tq4x4(int n, const int16_t *resid, const uint8_t *pred, int qp, int qsel, int16_t *levels, uint8_t *recon,
                            int32_t *cc, int32_t *nz, hipStream_t st);

// quantisation rounding selector of a slice (q_round, jmh_common.h; docs/JM_SEMANTICS.md items 1
// and 45): JM 8.6 = 1 in I slices, 0 in P slices; JMVersion >= 10 = 2 + the slice's OffsetMatrix entry
static int q_selector(const jmh_config &cfg, bool i_slice) {
    return cfg.jm_version >= 10 ? 2 + cfg.quant_offset[i_slice ? 0 : 1] : i_slice ? 1 : 0;
}

// JMH_FLAG_KERNEL_TIMING brackets every KT_STRIDE-th tick's two launches with events: the
// averages are sampled uniformly while the event packets stay off most launches
#define KT_STRIDE 32                      // an event pair between two launches costs ~7 us on that tick
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


// one ring entry: everything one picture in flight owns
struct PicBuf {
    uint8_t *src, *rec, *dbk;            // device: source (jmh_frame_push), recon, deblocked recon
    int16_t *mv;
    int8_t *refidx, *ipred;
    jmh_mb_result *res;
    MbScratch *scr;
    jmh_mb_result *h_res;                // pinned host copies (allocated on first readback use)
    uint8_t *h_src, *h_rec, *h_dbk;
    hipEvent_t ev_src, ev_t0, ev_done;   // staging reuse / push..done timing
    hipEvent_t ev_fin;                   // the picture's last tick (the copy stream's readback waits)
    uint8_t *cab;                        // RDOptimization 1: the slices' context states,
    uint32_t *range;                     //   codIRange, the MBs' context-selection records
    jmr_mbinfo *mbi;
    RdoPic *h_rp;                        //   pinned staging of the entry's RdoPic (after scr)
    hipEvent_t ev_rp;                    //   its H2D copy (h_rp is rewritten only after it completes)
    int recon_read;                      // h_rec holds the occupant's reconstruction
    int unpopped;                        // readback picture not yet popped
    int deblocked;                       // the occupant was deblocked on the device (dbk valid)
    uint32_t gen;                        // dataflow: occupants so far (the flag value of its MBs)
};

// a picture in flight (not yet fully issued)
struct Flight {
    int id, entry, ref_entry;            // ref_entry: ring entry read as reference (-1: d_ref / none)
    int tmv_entry;                       // ring entry whose motion field EPZS reads (-1: none)
    int pred_id;                         // picture it must trail by PIPE_LAG diagonals (-1: none)
    int stage, started, readback;
    PicParams pp;
};

enum { REF_NONE, REF_BUF, REF_REC, REF_DBK };

struct jmh_ctx {
    jmh_config cfg;
    int dev;
    hipStream_t st;                      // the wavefront ticks (and source uploads)
    hipStream_t cst;                     // readback of finished pictures, overlapping later ticks
    hipStream_t sst = nullptr;           // RDO on: k_rdo_intra beside k_rdo_inter (JMH_RDO_SIDE=0: off)
    hipEvent_t ev_fork = nullptr, ev_join = nullptr;
    int W, H, Wc, Hc, mbw, mbh, sr, side, npos, qstride, qplane, nd;
    size_t fsize, n4, nmb;               // bytes of one 4:2:0 picture (Y then U then V)
    uint8_t *d_ref, *d_qpel, *d_slots;   // explicit reference (set_reference), a1 seam, slots
    uint8_t *d_scur, *d_sref;            // luma pictures of the per-block searches (jmh_search_pictures)
    uint32_t *d_ordtab;                  // FFS order keys of the analysis threads' strips (ordtab_fill)
    uint16_t *d_scur16, *d_sref16;       // 16-bit luma pictures of the High 10 seams (jmh_search_pictures_u16)
    int bd, ps, maxv;                    // picture bit depth, bytes per sample (1, 2), (1 << bd) - 1
    int hbd_bits;                        //   and their bit depth
    int nslots;
    int depth, nring;
    std::vector<PicBuf> ring;
    std::deque<Flight> fl;               // issued-incompletely pictures, oldest first
    std::deque<int> popq;                // readback pictures (ring entries) not yet popped
    int next_id, next_entry;
    int last_id, last_entry;             // the last pushed picture
    int ref_kind, ref_entry;             // the reference of the next pushed picture
    int cur_entry;                       // results visible through get_mb_result / read_*
    unsigned long long *d_prof;          // JMH_PHASE_PROF=<mb>: per-phase wall clock of one MB
    int prof_mb;
    unsigned long long *d_bprof;         // JMH_BLOCK_PROF=<tick>: k_mb_analyse block start/end/role
    int bprof_tick, bprof_blocks;
    uint8_t *h_stage_ref;
    EvRing ring_interp, ring_mb, ring_an, ring_fin;   // ring_an / ring_fin: JMH_FLAG_KERNEL_TIMING
    jmh_timing timing;
    int ticks_total;
    std::vector<int> dcount, dymin;
    int lag;                             // stages a picture trails its reference picture by
    // RDOptimization 1: the RD stage schedule (MB addresses in stage order, offsets per stage),
    // the tick's candidate scratch, slices per picture
    int32_t *d_sched, *d_soff;
    void *d_rscr;
    void *d_ffs;                         // RDO + SearchMode 0: the tick MBs' SAD tables (k_rdo_inter)
    int nslice;
    // dataflow wavefront (k_mb_flow): ticks are not launched one by one but
    // collected into a segment of macroblocks in tick order, launched as one grid on a flush
    bool flow = false;
    int seg_max = 0;                     // ticks per segment before a flush (JMH_FLOW_SEG)
    int seg_min = 0;                     // ... or, once the device is idle, this many (JMH_FLOW_SEG_MIN)
    hipEvent_t ev_flow = nullptr;        // the last segment launch's end: a segment of >= seg_min ticks
                                         //   is flushed as soon as the device has run out of work
    std::vector<FlowPic> fpic;           // per ring entry: parameters + flag generations
    std::vector<uint32_t> seg;           // the pending segment's macroblocks (FLOW_ITEM)
    unsigned long long seg_mask = 0;     // ring entries the pending segment reads or writes
    int seg_ticks = 0;
    size_t seg_cap = 0;                  // items the device / staging buffers hold
    // segment buffers, alternating: pinned staging -> device on the upload stream, beside the
    // previous segment's launch (a buffer is rewritten once the launch that read it has ended)
    uint8_t *d_seg[2] = {nullptr, nullptr};   // device: FlowPic[nring], then the items
    uint8_t *h_seg[2] = {nullptr, nullptr};   // pinned staging
    hipEvent_t ev_seg[2] = {nullptr, nullptr};   // the upload out of h_seg[i] / into d_seg[i] done
    hipEvent_t ev_kseg[2] = {nullptr, nullptr};  // the launch that read d_seg[i] done
    hipStream_t ust = nullptr;           // the segment uploads
    int seg_slot = 0;
    uint32_t *d_flags = nullptr;         // [nring][nmb] generations of the finished MBs
    unsigned *d_head = nullptr;          // ticket counter
    unsigned head_base = 0;
    unsigned *h_err = nullptr;           // pinned, device-written: a dependency wait timed out
    int fprof_launch = -1, flow_count = 0;   // debug: JMH_FLOW_PROF=<launch> -> JMH_FLOW_PROF_OUT (raw u64)
    unsigned long long *d_fprof = nullptr;
    size_t fprof_n = 0;
    std::vector<uint32_t> fprof_items;
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

}  // extern "C"

static void free_entry(PicBuf &b) {
    void *dev_bufs[] = {b.src, b.rec, b.dbk, b.mv, b.refidx, b.ipred, b.res, b.scr, b.cab, b.range, b.mbi};
    for (void *p : dev_bufs) if (p) (void)hipFree(p);
    void *host_bufs[] = {b.h_res, b.h_src, b.h_rec, b.h_dbk, b.h_rp};
    for (void *p : host_bufs) if (p) (void)hipHostFree(p);
    hipEvent_t evs[] = {b.ev_src, b.ev_t0, b.ev_done, b.ev_fin, b.ev_rp};
    for (hipEvent_t e : evs) if (e) (void)hipEventDestroy(e);
}

static int alloc_entry(jmh_ctx *c, PicBuf &b) {
    memset((void *)&b, 0, sizeof(b));
#define ALLOC(p, n) do { if (hipMalloc((void **)&(p), (n)) != hipSuccess) return JMH_E_OOM; } while (0)
    ALLOC(b.src, c->fsize); ALLOC(b.rec, c->fsize); ALLOC(b.dbk, c->fsize);
    ALLOC(b.mv, c->n4 * 2 * sizeof(int16_t)); ALLOC(b.refidx, c->n4); ALLOC(b.ipred, c->n4);
    ALLOC(b.res, c->nmb * sizeof(jmh_mb_result));
    // RDOptimization 1: the picture's RdoPic sits right after its MbScratch array (jmh_device.h)
    ALLOC(b.scr, c->cfg.rdo ? rdo_pic_offset(c->nmb) + sizeof(RdoPic) : c->nmb * sizeof(MbScratch));
    if (c->cfg.rdo) {
        ALLOC(b.cab, (size_t)c->nslice * JMR_NCTX);
        ALLOC(b.range, (size_t)c->nslice * sizeof(uint32_t));
        ALLOC(b.mbi, c->nmb * sizeof(jmr_mbinfo));
        if (hipHostMalloc((void **)&b.h_rp, sizeof(RdoPic), hipHostMallocDefault) != hipSuccess) return JMH_E_OOM;
        b.h_rp->lambda = 0; b.h_rp->lf = 0; b.h_rp->pad = 0;
        b.h_rp->cab = b.cab; b.h_rp->range = b.range; b.h_rp->mbi = b.mbi;
        if (hipEventCreateWithFlags(&b.ev_rp, hipEventDisableTiming) != hipSuccess) return JMH_E_HIP;
    }
#undef ALLOC
    if (hipMemset(b.rec, 0, c->fsize) != hipSuccess || hipMemset(b.dbk, 0, c->fsize) != hipSuccess) return JMH_E_HIP;
    if (hipEventCreate(&b.ev_src) != hipSuccess || hipEventCreate(&b.ev_t0) != hipSuccess ||
        hipEventCreate(&b.ev_done) != hipSuccess || hipEventCreateWithFlags(&b.ev_fin, hipEventDisableTiming) != hipSuccess)
        return JMH_E_HIP;
    return JMH_OK;
}

// pinned readback / staging, on first use: all four buffers or none (a partial allocation is
// released, so a later call retries instead of seeing a half-initialised entry)
static int alloc_host(jmh_ctx *c, PicBuf &b) {
    if (b.h_res && b.h_src && b.h_rec && b.h_dbk) return JMH_OK;
    void **bufs[4] = {(void **)&b.h_res, (void **)&b.h_src, (void **)&b.h_rec, (void **)&b.h_dbk};
    const size_t sizes[4] = {c->nmb * sizeof(jmh_mb_result), c->fsize, c->fsize, c->fsize};
    for (int i = 0; i < 4; i++)
        if (!*bufs[i] && hipHostMalloc(bufs[i], sizes[i], hipHostMallocDefault) != hipSuccess) {
            *bufs[i] = nullptr;
            for (int k = 0; k < 4; k++)
                if (*bufs[k]) { (void)hipHostFree(*bufs[k]); *bufs[k] = nullptr; }
            return JMH_E_OOM;
        }
    return JMH_OK;
}

// device temporaries of the unit seams: freed on every return path
struct DevTemps {
    std::vector<void *> p;
    ~DevTemps() { for (void *q : p) if (q) (void)hipFree(q); }
    template <class T> hipError_t alloc(T **out, size_t n) {
        void *q = nullptr;
        hipError_t e = hipMalloc(&q, n);
        if (e == hipSuccess) p.push_back(q);
        *out = (T *)q;
        return e;
    }
};

static void ordtab_fill(std::vector<uint32_t> &tab, int sr);

// RDOptimization 1: the RD stage schedule.  A macroblock's stage is one more than
// the latest of its left, top and top-right neighbours (prediction, deblocking) and of its
// predecessor in the slice (the CABAC coding state): with one MB row per slice the diagonals
// x + 2y, with one slice per picture raster order.  A picture trails its reference picture by
// lag = 1 + max over MBs of (latest stage in the MB's reference reach [0, x + R] x [0, y + R] (R = ref_reach: 5 up to SR 32) -
// its own stage) stages (PIPE_LAG's derivation, jmh_device.h).  Fills order (MB addresses by
// stage, raster within a stage), off (stage offsets), c->dcount, c->nd, c->lag; non-zero when
// the schedule's stages do not fit PicParams.diag (int16).
static int rdo_schedule(jmh_ctx *c, std::vector<int> &order, std::vector<int> &off) {
    const int mbw = c->mbw, mbh = c->mbh, n = mbw * mbh, k = c->cfg.slice_mbs > 0 ? c->cfg.slice_mbs : n;
    std::vector<int> stage(n);
    int nd = 0;
    for (int a = 0; a < n; a++) {
        const int x = a % mbw, y = a / mbw;
        int s = 0;
        if (x > 0) s = std::max(s, stage[a - 1] + 1);
        if (y > 0) s = std::max(s, stage[a - mbw] + 1);
        if (y > 0 && x + 1 < mbw) s = std::max(s, stage[a - mbw + 1] + 1);
        if (a % k != 0) s = std::max(s, stage[a - 1] + 1);
        stage[a] = s;
        nd = std::max(nd, s + 1);
    }
    if (nd > 32767) return -1;
    c->nd = nd;
    c->dcount.assign(nd, 0);
    for (int a = 0; a < n; a++) c->dcount[stage[a]]++;
    off.assign(nd + 1, 0);
    for (int s = 0; s < nd; s++) off[s + 1] = off[s] + c->dcount[s];
    order.assign(n, 0);
    std::vector<int> fill(off.begin(), off.end() - 1);
    for (int a = 0; a < n; a++) order[fill[stage[a]]++] = a;
    std::vector<int> pm(n);                           // prefix maximum of the stages
    for (int y = 0; y < mbh; y++)
        for (int x = 0; x < mbw; x++) {
            int v = stage[y * mbw + x];
            if (x > 0) v = std::max(v, pm[y * mbw + x - 1]);
            if (y > 0) v = std::max(v, pm[(y - 1) * mbw + x]);
            pm[y * mbw + x] = v;
        }
    int lag = 1;
    const int R = ref_reach(c->sr);
    for (int y = 0; y < mbh; y++)
        for (int x = 0; x < mbw; x++) {
            const int X = std::min(x + R, mbw - 1), Y = std::min(y + R, mbh - 1);
            lag = std::max(lag, pm[Y * mbw + X] - stage[y * mbw + x] + 1);
        }
    c->lag = lag;
    return 0;
}

extern "C" {

void jmh_destroy(jmh_ctx *c) {
    if (!c) return;
    (void)hipSetDevice(c->dev);
    if (c->st) (void)hipStreamSynchronize(c->st);
    if (c->cst) (void)hipStreamSynchronize(c->cst);
    if (c->sst) (void)hipStreamSynchronize(c->sst);
    for (PicBuf &b : c->ring) free_entry(b);
    void *dev_bufs[] = {c->d_ref, c->d_qpel, c->d_slots, c->d_prof, c->d_bprof, c->d_scur, c->d_sref, c->d_ordtab, c->d_scur16,
                        c->d_sref16, c->d_sched, c->d_soff, c->d_rscr, c->d_ffs, c->d_seg[0], c->d_seg[1], c->d_flags, c->d_head,
                        c->d_fprof};
    for (void *p : dev_bufs) if (p) (void)hipFree(p);
    if (c->h_stage_ref) (void)hipHostFree(c->h_stage_ref);
    for (int i = 0; i < 2; i++) {
        if (c->h_seg[i]) (void)hipHostFree(c->h_seg[i]);
        if (c->ev_seg[i]) (void)hipEventDestroy(c->ev_seg[i]);
        if (c->ev_kseg[i]) (void)hipEventDestroy(c->ev_kseg[i]);
    }
    if (c->ust) { (void)hipStreamSynchronize(c->ust); (void)hipStreamDestroy(c->ust); }
    if (c->h_err) (void)hipHostFree(c->h_err);
    if (c->ev_flow) (void)hipEventDestroy(c->ev_flow);
    ring_free(c->ring_interp);
    ring_free(c->ring_mb);
    ring_free(c->ring_an);
    ring_free(c->ring_fin);
    if (c->st) (void)hipStreamDestroy(c->st);
    if (c->cst) (void)hipStreamDestroy(c->cst);
    if (c->sst) (void)hipStreamDestroy(c->sst);
    if (c->ev_fork) (void)hipEventDestroy(c->ev_fork);
    if (c->ev_join) (void)hipEventDestroy(c->ev_join);
    delete c;
}

int jmh_create(const jmh_config *cfg, int hip_device, jmh_ctx **out) {
    if (!cfg || !out) return JMH_E_INVALID_ARG;
    *out = nullptr;
    if (cfg->width <= 0 || cfg->height <= 0 || (cfg->width & 15) || (cfg->height & 15)) return JMH_E_INVALID_ARG;
    if (cfg->search_range < 1 || cfg->search_range > 64) return JMH_E_INVALID_ARG;
    // SearchRange > 32: EPZS only (its window falls back to the reference in global memory; the FFS
    // and full-search windows are LDS-resident at SRMAX)
    if (cfg->search_range > SRMAX && cfg->search_mode != 3) return JMH_E_UNSUPPORTED_CFG;
    if (cfg->search_mode != 0 && cfg->search_mode != -1 && cfg->search_mode != 3) return JMH_E_UNSUPPORTED_CFG;   // FFS / full / EPZS
    if (cfg->num_ref_frames != 1) return JMH_E_UNSUPPORTED_CFG;
    if (cfg->constrained_intra_pred != 0 && cfg->constrained_intra_pred != 1) return JMH_E_INVALID_ARG;
    if (cfg->restrict_search_range < 0 || cfg->restrict_search_range > 2) return JMH_E_INVALID_ARG;
    if (cfg->pipeline_depth < 0 || cfg->pipeline_depth > PMAX) return JMH_E_INVALID_ARG;
    if (cfg->transform_8x8_mode != 0 && cfg->transform_8x8_mode != 1) return JMH_E_UNSUPPORTED_CFG;
    if (cfg->jm_version < 0 || cfg->jm_version == 9 || cfg->jm_version > 99) return JMH_E_UNSUPPORTED_CFG;   // 0 / 8: JM 8.6, 10..: JM >= 10
    if (cfg->epzs_dual_refinement != 0 && cfg->epzs_dual_refinement != 1) return JMH_E_UNSUPPORTED_CFG;
    if ((cfg->epzs_subpel_me != 0 && cfg->epzs_subpel_me != 1) || cfg->epzs_subpel_thres_scale < 0 ||
        cfg->epzs_subpel_thres_scale > JMH_EPZS_SCALE_MAX || cfg->epzs_min_thres_scale < 0 || cfg->epzs_min_thres_scale > JMH_EPZS_SCALE_MAX ||
        cfg->epzs_max_thres_scale < 0 || cfg->epzs_max_thres_scale > JMH_EPZS_SCALE_MAX) return JMH_E_INVALID_ARG;
    if (cfg->slice_mbs < 0) return JMH_E_INVALID_ARG;
    if (cfg->bit_depth != 0 && (cfg->bit_depth < 8 || cfg->bit_depth > 10)) return JMH_E_UNSUPPORTED_CFG;
    // High 10 pictures: the EPZS wavefront (k_mb_epzs / k_mb_intra / k_mb_final on 16-bit samples)
    // RDOptimization 1: the CABAC rate, EPZS searches, either transform mode (k_rdo_inter / k_rdo_intra / k_rdo_final)
    if (cfg->rdo != 0 && (cfg->rdo != 1 || cfg->symbol_mode < 0 || cfg->symbol_mode > 1))
        return JMH_E_UNSUPPORTED_CFG;
    if (cfg->jm_version >= 10 && (cfg->quant_offset[0] < 0 || cfg->quant_offset[0] > JMH_QOFFSET_MAX || cfg->quant_offset[1] < 0 ||
                                  cfg->quant_offset[1] > JMH_QOFFSET_MAX)) return JMH_E_INVALID_ARG;
    int ndev = jmh_device_count();
    if (ndev <= 0) return JMH_E_NO_DEVICE;
    if (hip_device < 0 || hip_device >= ndev) return JMH_E_INVALID_ARG;
    jmh_ctx *c = new jmh_ctx();
    c->cfg = *cfg;
    c->dev = hip_device;
    HCHK(hipSetDevice(hip_device));
    c->W = cfg->width; c->H = cfg->height; c->Wc = c->W / 2; c->Hc = c->H / 2;
    c->mbw = c->W / 16; c->mbh = c->H / 16;
    c->sr = cfg->search_range; c->side = 2 * c->sr + 1; c->npos = c->side * c->side;
    c->qstride = c->W + 2 * QPAD; c->qplane = c->qstride * (c->H + 2 * QPAD);
    c->bd = cfg->bit_depth > 8 ? cfg->bit_depth : 8; c->ps = c->bd > 8 ? 2 : 1; c->maxv = (1 << c->bd) - 1;
    c->fsize = (size_t)c->W * c->H * 3 / 2 * c->ps;
    c->n4 = (size_t)c->W * c->H / 16; c->nmb = (size_t)c->mbw * c->mbh;
    c->nslots = cfg->num_frame_slots > 0 ? cfg->num_frame_slots : 1;
    c->nd = (c->mbw - 1) + 2 * (c->mbh - 1) + 1;
    c->lag = pipe_lag(c->sr);
    c->nslice = cfg->slice_mbs > 0 ? (int)((c->nmb + cfg->slice_mbs - 1) / cfg->slice_mbs) : 1;
    std::vector<int> rd_order, rd_off;
    if (cfg->rdo && rdo_schedule(c, rd_order, rd_off)) { delete c; return JMH_E_UNSUPPORTED_CFG; }
    // enough pictures to cover the wavefront: one starts every lag stages
    int auto_depth = (c->nd + c->lag - 1) / c->lag + 1;
    c->depth = cfg->pipeline_depth > 0 ? cfg->pipeline_depth : (auto_depth < PMAX ? auto_depth : PMAX);
    // dataflow wavefront: FFS on 8-bit samples, RDO off, no 8x8 transform (k_mb_analyse's search +
    // k_mb_final); JMH_FLOW=0 keeps the tick launches, as does the per-tick block profile
    {
        const char *fe = getenv("JMH_FLOW");
        c->flow = cfg->search_mode == 0 && c->bd == 8 && !cfg->rdo && !cfg->transform_8x8_mode && !cfg->constrained_intra_pred &&
                  !(fe && atoi(fe) == 0) &&
                  !getenv("JMH_BLOCK_PROF") && c->mbw < 4096 && c->mbh < 4096;
        const char *sg = getenv("JMH_FLOW_SEG");
        const char *sm = getenv("JMH_FLOW_SEG_MIN");
        c->seg_min = sm && atoi(sm) > 0 ? atoi(sm) : 8;
        c->seg_max = sg && atoi(sg) > 0 ? std::min(atoi(sg), 256) : 128;   // (<= 256: nring stays < 64, seg_mask's bits)   // A/B 64 / 128 / 256: 1392.6 / 1402.4 / 1401.4 MP/s (profiles/r10g_flow_seg_ab.txt)
    }
    // (dataflow: enough more entries that an entry's next occupant never falls into a segment that
    // still finishes its previous one, which would force a flush: a segment of seg_max ticks spans
    // seg_max / lag pictures)
    c->nring = c->depth + 2 + (c->flow ? (c->seg_max + c->lag - 1) / c->lag + 2 : 0);
    c->next_id = 0; c->next_entry = 0; c->last_id = -1; c->last_entry = -1;
    c->ref_kind = REF_NONE; c->ref_entry = -1; c->cur_entry = -1;
    c->prof_mb = -1;
    int st = JMH_OK;
#define ALLOC(p, n) do { if (hipMalloc((void **)&(p), (n)) != hipSuccess) { st = JMH_E_OOM; goto fail; } } while (0)
    {
        if (hipStreamCreateWithFlags(&c->st, hipStreamNonBlocking) != hipSuccess ||
            hipStreamCreateWithFlags(&c->cst, hipStreamNonBlocking) != hipSuccess) { st = JMH_E_HIP; goto fail; }
        // RDO on: the intra role on a side stream, concurrent with the inter role (the inter
        // workgroups' LDS leaves room for intra ones beside them); joined before k_rdo_final.
        // RDO off with a separate search kernel (EPZS, full search, High 10 FFS): k_mb_intra on the
        // side stream beside k_mb_epzs / k_mb_me_full, joined before k_mb_final (A/B knobs:
        // JMH_RDO_SIDE=0, JMH_INTRA_SIDE=0)
        const char *side = getenv(cfg->rdo ? "JMH_RDO_SIDE" : "JMH_INTRA_SIDE");
        const bool sep_search = cfg->rdo || cfg->search_mode != 0 || (cfg->bit_depth > 8);
        if (sep_search && !(side && atoi(side) == 0)) {
            if (hipStreamCreateWithFlags(&c->sst, hipStreamNonBlocking) != hipSuccess ||
                hipEventCreateWithFlags(&c->ev_fork, hipEventDisableTiming) != hipSuccess ||
                hipEventCreateWithFlags(&c->ev_join, hipEventDisableTiming) != hipSuccess) { st = JMH_E_HIP; goto fail; }
        }
        ALLOC(c->d_ref, c->fsize);
        ALLOC(c->d_qpel, (size_t)16 * c->qplane);
        ALLOC(c->d_slots, c->fsize * c->nslots);
        {
            std::vector<uint32_t> ot;
            ordtab_fill(ot, c->sr);
            ALLOC(c->d_ordtab, ot.size() * sizeof(uint32_t));
            if (hipMemcpy(c->d_ordtab, ot.data(), ot.size() * sizeof(uint32_t), hipMemcpyHostToDevice) != hipSuccess) { st = JMH_E_HIP; goto fail; }
        }
        c->ring.resize(c->nring);
        for (PicBuf &b : c->ring) {
            if ((st = alloc_entry(c, b))) goto fail;
            if (hipEventRecord(b.ev_src, c->st) != hipSuccess) { st = JMH_E_HIP; goto fail; }
        }
        c->bprof_tick = -1;
        if (const char *e = getenv("JMH_BLOCK_PROF")) {
            c->bprof_tick = atoi(e);
            ALLOC(c->d_bprof, ((size_t)3 * 3 * PMAX * c->mbh + 64) * sizeof(unsigned long long));
        }
        if (const char *e = getenv("JMH_PHASE_PROF")) {
            c->prof_mb = atoi(e);
            ALLOC(c->d_prof, 64 * sizeof(unsigned long long));
            if (hipMemset(c->d_prof, 0, 64 * sizeof(unsigned long long)) != hipSuccess) { st = JMH_E_HIP; goto fail; }
        }
        if (hipHostMalloc((void **)&c->h_stage_ref, c->fsize, hipHostMallocDefault) != hipSuccess) { st = JMH_E_OOM; goto fail; }
        if (c->flow) {
            // segment buffers: seg_max ticks of at most PMAX diagonals each
            c->seg_cap = (size_t)c->seg_max * PMAX * (size_t)std::min(c->mbh, (c->mbw + 1) / 2 + 1) + 1;
            const size_t sb = (size_t)c->nring * sizeof(FlowPic) + c->seg_cap * sizeof(uint32_t);
            ALLOC(c->d_seg[0], sb);
            ALLOC(c->d_seg[1], sb);
            if (hipStreamCreateWithFlags(&c->ust, hipStreamNonBlocking) != hipSuccess) { st = JMH_E_HIP; goto fail; }
            ALLOC(c->d_flags, (size_t)c->nring * c->nmb * sizeof(uint32_t));
            ALLOC(c->d_head, sizeof(unsigned));
            for (int i = 0; i < 2; i++)
                if (hipHostMalloc((void **)&c->h_seg[i], sb, hipHostMallocDefault) != hipSuccess ||
                    hipEventCreateWithFlags(&c->ev_seg[i], hipEventDisableTiming) != hipSuccess ||
                    hipEventCreateWithFlags(&c->ev_kseg[i], hipEventDisableTiming) != hipSuccess) { st = JMH_E_OOM; goto fail; }
            if (hipHostMalloc((void **)&c->h_err, 4 * sizeof(unsigned), hipHostMallocCoherent | hipHostMallocMapped) != hipSuccess) { st = JMH_E_OOM; goto fail; }
            if (hipEventCreateWithFlags(&c->ev_flow, hipEventDisableTiming) != hipSuccess) { st = JMH_E_HIP; goto fail; }
            memset(c->h_err, 0, 4 * sizeof(unsigned));
            // on the context's stream: a plain hipMemset of device memory may still be pending on the
            // null stream, which the non-blocking stream does not wait for, when the first segment
            // claims its tickets (seen with two processes on one GPU)
            if (hipMemsetAsync(c->d_flags, 0, (size_t)c->nring * c->nmb * sizeof(uint32_t), c->st) != hipSuccess ||
                hipMemsetAsync(c->d_head, 0, sizeof(unsigned), c->st) != hipSuccess) { st = JMH_E_HIP; goto fail; }
            c->fpic.assign(c->nring, FlowPic{});
            c->seg.reserve(c->seg_cap);
            if (const char *e = getenv("JMH_FLOW_PROF")) {
                c->fprof_launch = atoi(e);
                ALLOC(c->d_fprof, c->seg_cap * 6 * sizeof(unsigned long long));
            }
        }
        if (hipMemset(c->d_ref, 0, c->fsize) != hipSuccess) { st = JMH_E_HIP; goto fail; }
        if (ring_init(c->ring_interp, 64) || ring_init(c->ring_mb, 64) ||
            ((cfg->flags & JMH_FLAG_KERNEL_TIMING) && (ring_init(c->ring_an, 2048) || ring_init(c->ring_fin, 2048)))) { st = JMH_E_HIP; goto fail; }
        if (cfg->rdo) {   // the RD stage schedule (rdo_schedule), the tick's candidate scratch
            c->dymin.assign(c->nd, 0);
            int maxc = 0;
            for (int sg = 0; sg < c->nd; sg++) maxc = std::max(maxc, c->dcount[sg]);
            ALLOC(c->d_sched, rd_order.size() * sizeof(int32_t));
            ALLOC(c->d_soff, rd_off.size() * sizeof(int32_t));
            ALLOC(c->d_rscr, (size_t)PMAX * maxc * jmh_rdo_scratch_bytes());
            // SearchMode 0: one SAD table per tick MB (JMH_RDO_FFS_TABLE=0: every search scans, A/B)
            const char *ft = getenv("JMH_RDO_FFS_TABLE");
            // (a failed allocation leaves d_ffs null: the searches then scan, with identical results)
            if (cfg->search_mode == 0 && !(ft && atoi(ft) == 0) &&
                hipMalloc(&c->d_ffs, (size_t)PMAX * maxc * ffs_slot_bytes(c->sr)) != hipSuccess) {
                c->d_ffs = nullptr;
                (void)hipGetLastError();
            }
            if (hipMemcpy(c->d_sched, rd_order.data(), rd_order.size() * sizeof(int32_t), hipMemcpyHostToDevice) != hipSuccess ||
                hipMemcpy(c->d_soff, rd_off.data(), rd_off.size() * sizeof(int32_t), hipMemcpyHostToDevice) != hipSuccess) { st = JMH_E_HIP; goto fail; }
        } else {
            c->dcount.resize(c->nd); c->dymin.resize(c->nd);
            for (int dg = 0; dg < c->nd; dg++) {
                int ymin = dg - (c->mbw - 1) > 0 ? (dg - (c->mbw - 1) + 1) / 2 : 0;
                int ymax = dg / 2 < c->mbh - 1 ? dg / 2 : c->mbh - 1;
                c->dymin[dg] = ymin;
                c->dcount[dg] = ymax >= ymin ? ymax - ymin + 1 : 0;
            }
        }
    }
#undef ALLOC
    // every initialising memset (null stream, possibly still pending: hipMemset of device memory
    // returns before it completes) done before the context's non-blocking streams run
    if (hipDeviceSynchronize() != hipSuccess) { st = JMH_E_HIP; goto fail; }
    *out = c;
    return JMH_OK;
fail:
    jmh_destroy(c);
    return st;
}

int jmh_pipeline_depth(const jmh_ctx *c) { return c ? c->depth : JMH_E_INVALID_ARG; }

}  // extern "C"

// JM spiral order (Init_Motion_Search_Module [J]) of relative position (x, y)
static int host_spiral_index(int x, int y) {
    const int ax = x < 0 ? -x : x, ay = y < 0 ? -y : y, l = ax > ay ? ax : ay;
    if (l == 0) return 0;
    const int base = (2 * l - 1) * (2 * l - 1);
    if (ay == l && ax < l) return base + 2 * (x + l - 1) + (y > 0);
    return base + 2 * (2 * l - 1) + 2 * (y + l) + (x > 0);
}

// order keys of the FFS analysis threads (k_mb_analyse): thread t owns window column t % side,
// rows (t / side) * NPK .. + NPK - 1; key = spiral index + 1 (0 is the (0,0) pre-check, set per
// MB in the kernel), 0xFFFF outside the window.  [NPK2][NTA] packed pairs (low = even slot); only
// the NTS search threads own strips.  Then the inverse, ORDTAB_SPOS: spiral index -> position
// (x & 0xFFFF | y << 16), read with one scalar load where a search's winner is decoded.
static void ordtab_fill(std::vector<uint32_t> &tab, int sr) {
    const int side = 2 * sr + 1, nstrips = (side + NPK - 1) / NPK;
    static_assert(SIDE_MAX * ((SIDE_MAX + NPK - 1) / NPK) <= NTS, "the search threads cover every FFS position");
    // after the keys: spiral index -> position, then raster position -> spiral index (the RDO FFS
    // table's tie order, jmh_epzs.h ffs_table_min)
    tab.assign((size_t)ORDTAB_SPOS + (size_t)2 * side * side, 0);
    for (int y = -sr; y <= sr; y++)
        for (int x = -sr; x <= sr; x++) {
            tab[(size_t)ORDTAB_SPOS + host_spiral_index(x, y)] = ((uint32_t)x & 0xFFFFu) | (uint32_t)y << 16;
            tab[(size_t)ORDTAB_SPOS + (size_t)side * side + (size_t)(y + sr) * side + x + sr] = (uint32_t)host_spiral_index(x, y);
        }
    for (int t = 0; t < NTA; t++) {
        const bool sact = t < side * nstrips && t < NTS;
        const int dx = sact ? t % side : 0, dy0 = sact ? (t / side) * NPK : 0;
        for (int k = 0; k < NPK; k++) {
            const int dy = dy0 + k;
            const uint32_t o = (!sact || dy >= side) ? 0xFFFFu : (uint32_t)(host_spiral_index(dx - sr, dy - sr) + 1);
            tab[(size_t)(k >> 1) * NTA + t] |= o << (16 * (k & 1));
        }
    }
}

// planar 4:2:0 packing of ps-byte samples (strides in samples).  16-bit samples are range-checked
// on the way (the kernels' cost keys and transform headroom assume every sample <= maxv): false
// when one exceeds maxv = (1 << bit depth) - 1, with dst then partially written.
static inline uint16_t pack_row16(uint16_t *d, const uint16_t *s, int n) {
    uint16_t acc = 0;
    for (int x = 0; x < n; x++) { d[x] = s[x]; acc |= s[x]; }
    return acc;
}
static bool pack_planes(uint8_t *dst, int W, int H, const void *yv, const void *uv, const void *vv, int sy, int sc, int ps,
                        int maxv) {
    const uint8_t *y = (const uint8_t *)yv, *u = (const uint8_t *)uv, *v = (const uint8_t *)vv;
    uint8_t *du = dst + (size_t)W * H * ps, *dv = du + (size_t)W * H / 4 * ps;
    if (ps == 1) {
        for (int r = 0; r < H; r++) memcpy(dst + (size_t)r * W, y + (size_t)r * sy, (size_t)W);
        for (int r = 0; r < H / 2; r++) {
            memcpy(du + (size_t)r * (W / 2), u + (size_t)r * sc, (size_t)(W / 2));
            memcpy(dv + (size_t)r * (W / 2), v + (size_t)r * sc, (size_t)(W / 2));
        }
        return true;
    }
    const uint16_t *y16 = (const uint16_t *)y, *u16 = (const uint16_t *)u, *v16 = (const uint16_t *)v;
    uint16_t acc = 0;
    for (int r = 0; r < H; r++) acc |= pack_row16((uint16_t *)dst + (size_t)r * W, y16 + (size_t)r * sy, W);
    for (int r = 0; r < H / 2; r++) {
        acc |= pack_row16((uint16_t *)du + (size_t)r * (W / 2), u16 + (size_t)r * sc, W / 2);
        acc |= pack_row16((uint16_t *)dv + (size_t)r * (W / 2), v16 + (size_t)r * sc, W / 2);
    }
    return (acc & ~maxv) == 0;   // maxv = 2^bd - 1: every sample <= maxv iff no bit above it is set
}

static void unpack_planes(const uint8_t *src, int W, int H, void *yv, void *uv, void *vv, int sy, int sc, int ps) {
    uint8_t *y = (uint8_t *)yv, *u = (uint8_t *)uv, *v = (uint8_t *)vv;
    size_t ls = (size_t)W * H * ps;
    for (int r = 0; r < H; r++) memcpy(y + (size_t)r * sy * ps, src + (size_t)r * W * ps, (size_t)W * ps);
    for (int r = 0; r < H / 2; r++) {
        memcpy(u + (size_t)r * sc * ps, src + ls + (size_t)r * (W / 2) * ps, (size_t)(W / 2) * ps);
        memcpy(v + (size_t)r * sc * ps, src + ls + ls / 4 + (size_t)r * (W / 2) * ps, (size_t)(W / 2) * ps);
    }
}

// the entry point's sample width matches the context (the sample range of a 16-bit picture is
// checked while it is packed into staging, pack_planes)
static int check_pic(const jmh_ctx *c, bool wide) {
    return (c->bd > 8) != wide ? JMH_E_UNSUPPORTED_CFG : JMH_OK;
}

// ---------------------------------------------------------------------------------------------
//  the tick scheduler
// ---------------------------------------------------------------------------------------------
static int skip_empty(const jmh_ctx *c, int stage) {
    while (stage < c->nd && c->dcount[stage] == 0) stage++;
    return stage;
}

// dataflow: launch the pending segment -- the FlowPic table and the items into the device
// buffer (pinned staging, alternating; a staging buffer is rewritten only after its copy ran), then
// one k_mb_flow grid of one workgroup per macroblock.  Stream order covers everything before and
// after the segment; inside it the per-MB flags do.
static int flow_flush(jmh_ctx *c) {
    if (!c->flow || c->seg.empty()) return JMH_OK;
    const int sl = c->seg_slot;
    c->seg_slot ^= 1;
    HCHK(hipEventSynchronize(c->ev_seg[sl]));
    const size_t pb = (size_t)c->nring * sizeof(FlowPic), ib = c->seg.size() * sizeof(uint32_t);
    if (c->seg.size() > c->seg_cap) return JMH_E_STATE;   // (never expected: seg_max ticks of <= PMAX diagonals)
    for (uint32_t it : c->seg) {
        const int e = (int)(it >> 24);
        if (e >= c->nring || c->fpic[e].gen == 0) { fprintf(stderr, "jmhip: flow segment item 0x%08x without a picture\n", it); return JMH_E_STATE; }
    }
    memcpy(c->h_seg[sl], c->fpic.data(), pb);
    memcpy(c->h_seg[sl] + pb, c->seg.data(), ib);
    HCHK(hipStreamWaitEvent(c->ust, c->ev_kseg[sl], 0));   // the launch two segments back read d_seg[sl]
    HCHK(hipMemcpyAsync(c->d_seg[sl], c->h_seg[sl], pb + ib, hipMemcpyHostToDevice, c->ust));
    HCHK(hipEventRecord(c->ev_seg[sl], c->ust));
    HCHK(hipStreamWaitEvent(c->st, c->ev_seg[sl], 0));
    FlowArgs f;
    memset(&f, 0, sizeof(f));
    f.W = c->W; f.H = c->H; f.mbw = c->mbw; f.mbh = c->mbh; f.sr = c->sr;
    f.search_mode = c->cfg.search_mode; f.use_hadamard = c->cfg.use_hadamard; f.restrict_sr = c->cfg.restrict_search_range;
    for (int i = 1; i < 8; i++) f.isr |= (c->cfg.inter_search[i] != 0) << i;
    f.slice_mbs = c->cfg.slice_mbs > 0 ? c->cfg.slice_mbs : c->mbw * c->mbh;
    f.ordtab = c->d_ordtab;
    f.prof = c->d_prof; f.prof_mb = c->prof_mb;
    f.pics = reinterpret_cast<const FlowPic *>(c->d_seg[sl]);
    f.items = reinterpret_cast<const uint32_t *>(c->d_seg[sl] + pb);
    f.nitems = (int)c->seg.size();
    f.nmb = (int)c->nmb; f.nring = c->nring;
    f.head = c->d_head; f.base = c->head_base;
    f.flags = c->d_flags;
    f.err = c->h_err;
    if (c->d_fprof && c->flow_count == c->fprof_launch) {
        f.fprof = c->d_fprof;
        c->fprof_n = c->seg.size();
        c->fprof_items = c->seg;
    }
    c->flow_count++;
    const bool kt = c->ring_an.cap > 0;
    HCHK(ring_begin(c->ring_mb, c->st));
    if (kt) HCHK(ring_begin(c->ring_an, c->st));
    HCHK(jmh_launch_flow(f, c->st));
    if (kt) HCHK(ring_end(c->ring_an, c->st));
    HCHK(ring_end(c->ring_mb, c->st));
    HCHK(hipEventRecord(c->ev_flow, c->st));
    HCHK(hipEventRecord(c->ev_kseg[sl], c->st));
    c->head_base += (unsigned)c->seg.size();
    c->timing.flow_launches++;
    c->timing.flow_mbs += (int)c->seg.size();
    c->seg.clear();
    c->seg_mask = 0;
    c->seg_ticks = 0;
    return JMH_OK;
}

// a dependency wait of k_mb_flow that timed out (never expected: every wait ends by construction);
// debug: the profiled launch's stamps to JMH_FLOW_PROF_OUT once it has run
static int flow_check(jmh_ctx *c) {
    if (c->fprof_n && c->flow_count > c->fprof_launch) {
        std::vector<unsigned long long> h(6 * c->fprof_n);
        HCHK(hipStreamSynchronize(c->st));
        HCHK(hipMemcpy(h.data(), c->d_fprof, h.size() * 8, hipMemcpyDeviceToHost));
        int rate_khz = 0;
        HCHK(hipDeviceGetAttribute(&rate_khz, hipDeviceAttributeWallClockRate, c->dev));
        const char *path = getenv("JMH_FLOW_PROF_OUT");
        if (FILE *fo = fopen(path ? path : "flow_prof.bin", "wb")) {
            const unsigned long long hdr[4] = {(unsigned long long)c->fprof_n, (unsigned long long)rate_khz, (unsigned long long)c->mbw,
                                               (unsigned long long)c->mbh};
            fwrite(hdr, 8, 4, fo);
            fwrite(h.data(), 8, h.size(), fo);
            fwrite(c->fprof_items.data(), 4, c->fprof_items.size(), fo);
            fclose(fo);
        }
        c->fprof_n = 0;
    }
    if (c->flow && c->h_err && __atomic_load_n(c->h_err, __ATOMIC_ACQUIRE)) {
        if (c->h_err[0] == 2) fprintf(stderr, "jmhip: k_mb_flow ticket %u item 0x%08x out of range (results invalid)\n", c->h_err[1], c->h_err[2]);
        else fprintf(stderr, "jmhip: k_mb_flow dependency wait timed out (results invalid)\n");
        return JMH_E_HIP;
    }
    return JMH_OK;
}

// after a picture's last tick: its readback on the copy stream (the D2H overlaps the ticks of
// the pictures still in flight; the entry's device buffers are not written again before the host
// has popped the picture, which waits for ev_done), then the done event
static int finish_picture(jmh_ctx *c, const Flight &f) {
    c->timing.pictures_done++;
    if (!f.readback) return JMH_OK;
    int r = flow_flush(c);                // the picture's last MBs before its events
    if (r) return r;
    PicBuf &b = c->ring[f.entry];
    HCHK(hipEventRecord(b.ev_fin, c->st));
    HCHK(hipStreamWaitEvent(c->cst, b.ev_fin, 0));
    HCHK(hipMemcpyAsync(b.h_res, b.res, c->nmb * sizeof(jmh_mb_result), hipMemcpyDeviceToHost, c->cst));
    b.recon_read = !(f.pp.dbk && (c->cfg.flags & JMH_FLAG_NO_RECON_READBACK));
    if (b.recon_read) HCHK(hipMemcpyAsync(b.h_rec, b.rec, c->fsize, hipMemcpyDeviceToHost, c->cst));
    if (f.pp.dbk) HCHK(hipMemcpyAsync(b.h_dbk, b.dbk, c->fsize, hipMemcpyDeviceToHost, c->cst));
    HCHK(hipEventRecord(b.ev_done, c->cst));
    return JMH_OK;
}

// one tick: the next diagonal of every picture whose dependencies are met (oldest first)
static int issue_tick(jmh_ctx *c) {
    TickArgs t;
    memset(&t, 0, sizeof(t));
    t.W = c->W; t.H = c->H; t.mbw = c->mbw; t.mbh = c->mbh; t.sr = c->sr;
    t.search_mode = c->cfg.search_mode; t.use_hadamard = c->cfg.use_hadamard; t.restrict_sr = c->cfg.restrict_search_range;
    for (int i = 0; i < 8; i++) t.inter_search[i] = c->cfg.inter_search[i];
    t.prof = c->d_prof; t.prof_mb = c->prof_mb;
    t.me_in_analyse = c->cfg.search_mode == 0 && c->bd == 8;   // High 10 FFS: k_mb_me_full<uint16_t, true>
    t.t8 = c->cfg.transform_8x8_mode;
    t.epzs_dual = c->cfg.epzs_dual_refinement;
    t.epzs_subpel = c->cfg.epzs_subpel_me; t.epzs_spts = c->cfg.epzs_subpel_thres_scale;
    t.epzs_mints = c->cfg.epzs_min_thres_scale; t.epzs_maxts = c->cfg.epzs_max_thres_scale;
    t.slice_mbs = c->cfg.slice_mbs > 0 ? c->cfg.slice_mbs : c->mbw * c->mbh;
    t.cip = c->cfg.constrained_intra_pred;
    t.bd = c->bd;
    t.ordtab = c->d_ordtab;
    t.rdo = c->cfg.rdo ? (c->cfg.symbol_mode ? 1 : 2) : 0;   // 2: CAVLC rates
    t.sched = c->d_sched; t.soff = c->d_soff; t.rscr = c->d_rscr;
    t.ffs = c->d_ffs; t.ffs_slot = ffs_slot_bytes(c->sr);
    int act[PMAX], nact = 0, nP = 0;
    const int nf = (int)c->fl.size();
    std::vector<int> before(nf);
    for (int i = 0; i < nf; i++) before[i] = c->fl[i].stage = skip_empty(c, c->fl[i].stage);
    for (int i = 0; i < nf && nact < PMAX; i++) {
        const Flight &f = c->fl[i];
        if (f.stage >= c->nd) continue;
        if (f.pred_id >= 0 && i > 0 && c->fl[i - 1].id == f.pred_id &&
            before[i - 1] < c->nd && before[i - 1] - f.stage < c->lag) continue;
        act[nact++] = i;
        nP += f.pp.slice_type == JMH_P_SLICE;
    }
    // entries: P pictures first (role 2 runs on those only)
    int k = 0, mbs = 0;
    for (int pass = 0; pass < 2; pass++)
        for (int a = 0; a < nact; a++) {
            Flight &f = c->fl[act[a]];
            if ((f.pp.slice_type == JMH_P_SLICE) != (pass == 0)) continue;
            t.p[k] = f.pp;
            t.p[k].diag = f.stage;
            t.p[k].y_min = c->dymin[f.stage];
            t.pre[k] = mbs;
            mbs += c->dcount[f.stage];
            k++;
        }
    t.npic = k; t.nP = nP; t.pre[k] = mbs;
    if (c->d_bprof && c->ticks_total == c->bprof_tick) {
        t.bprof = c->d_bprof;
        // the analysis blocks: k_mb_analyse's (roles 0 / 2), or the separate search kernel's (role 4)
        // RDO: k_rdo_inter's blocks (role 4), then k_rdo_intra's (role 1)
        const int na = t.rdo ? xcd_grid(t.pre[nP]) + xcd_grid(t.pre[k])
                             : t.me_in_analyse ? xcd_grid(t.pre[nP]) + (t.pre[k] + 3) / 4 : xcd_grid(t.pre[nP]);
        t.bprof_fin = c->d_bprof + 3 * na;
        HCHK(hipMemsetAsync(c->d_bprof, 0, ((size_t)3 * 3 * PMAX * c->mbh + 64) * sizeof(unsigned long long), c->st));
        c->bprof_blocks = na + xcd_grid(t.pre[k]);
    }
    if (nact && c->flow) {
        // dataflow: the tick's macroblocks join the pending segment in tick order (P pictures
        // first, diagonal MBs top to bottom, as the tick kernels' block order)
        for (int pass = 0; pass < 2; pass++)
            for (int a = 0; a < nact; a++) {
                const Flight &f = c->fl[act[a]];
                if ((f.pp.slice_type == JMH_P_SLICE) != (pass == 0)) continue;
                const int y0 = c->dymin[f.stage], n = c->dcount[f.stage];
                for (int i = 0; i < n; i++) c->seg.push_back(FLOW_ITEM(f.entry, f.stage - 2 * (y0 + i), y0 + i));
                c->seg_mask |= 1ull << f.entry;
                if (f.ref_entry >= 0) c->seg_mask |= 1ull << f.ref_entry;
            }
        c->seg_ticks++;
        c->ticks_total++;
        c->timing.ticks++;
        c->timing.tick_mbs += mbs;
        c->timing.mb_launches += 1;
    } else if (nact) {
        const bool kt = c->ring_an.cap > 0 && c->ticks_total % KT_STRIDE == 0;   // sampled per-launch timing
        if (kt) HCHK(ring_begin(c->ring_an, c->st));
        if (t.rdo) {                                    // RDOptimization 1: analyse + final
            HCHK(jmh_launch_rdo(t, c->st, c->sst, c->ev_fork, c->ev_join));
        } else if (t.me_in_analyse) {                   // FFS: motion search + intra in k_mb_analyse
            HCHK(jmh_launch_analyse(t, c->st));
            if (t.t8) HCHK(jmh_launch_intra8(t, c->st));   // Intra8x8 decision (High profile)
        } else {                                        // EPZS (one wave per MB) / SearchMode -1 / High 10 FFS
            // the intra decisions (independent of the searches) on the side stream: its workgroups
            // take the CUs the search workgroups leave as they finish; joined before k_mb_final
            const bool side = c->sst && nP > 0;
            if (side) { HCHK(hipEventRecord(c->ev_fork, c->st)); HCHK(hipStreamWaitEvent(c->sst, c->ev_fork, 0)); }
            if (t.search_mode == 3) HCHK(jmh_launch_epzs(t, c->st));
            else HCHK(jmh_launch_me_full(t, c->st));
            HCHK(jmh_launch_intra(t, side ? c->sst : c->st));   // all intra decisions incl. Intra8x8
            if (side) { HCHK(hipEventRecord(c->ev_join, c->sst)); HCHK(hipStreamWaitEvent(c->st, c->ev_join, 0)); }
        }
        if (kt) { HCHK(ring_end(c->ring_an, c->st)); HCHK(ring_begin(c->ring_fin, c->st)); }
        if (!t.rdo) HCHK(jmh_launch_final(t, c->st));
        if (kt) HCHK(ring_end(c->ring_fin, c->st));
        c->ticks_total++;
        c->timing.ticks++;
        c->timing.tick_mbs += mbs;
        c->timing.mb_launches += 2;
    }
    for (int a = 0; a < nact; a++) {
        Flight &f = c->fl[act[a]];
        f.started = 1;
        f.stage = skip_empty(c, f.stage + 1);
    }
    while (!c->fl.empty() && skip_empty(c, c->fl.front().stage) >= c->nd) {
        int r = finish_picture(c, c->fl.front());
        c->fl.pop_front();
        if (r) return r;
    }
    // flush at seg_max ticks, or earlier once the device has finished every launched segment (so
    // that it starts soon after the host resumes issuing and segments stay as long as the host's
    // lead allows: each launch boundary drains the device)
    if (c->flow && (c->seg_ticks >= c->seg_max || (c->seg_ticks >= c->seg_min && hipEventQuery(c->ev_flow) == hipSuccess)))
        return flow_flush(c);
    return JMH_OK;
}

static bool entry_busy(const jmh_ctx *c, int e) {
    for (const Flight &f : c->fl)
        if (f.entry == e || f.ref_entry == e || f.tmv_entry == e) return true;
    return false;
}

// issue ticks while cond() holds, bracketed by one mb-timing event pair
template <class Cond>
static int issue_while(jmh_ctx *c, Cond cond) {
    if (!cond()) return JMH_OK;
    if (c->flow) {   // the launches happen at flushes (flow_flush brackets them with ring_mb)
        int r = JMH_OK;
        while (!r && cond()) {
            if (c->fl.empty()) return JMH_E_STATE;
            r = issue_tick(c);
        }
        return r;
    }
    HCHK(ring_begin(c->ring_mb, c->st));
    int r = JMH_OK;
    while (!r && cond()) {
        if (c->fl.empty()) { r = JMH_E_STATE; break; }   // cannot progress (never expected)
        r = issue_tick(c);
    }
    HCHK(ring_end(c->ring_mb, c->st));
    return r;
}

static int drain(jmh_ctx *c) {
    int r = issue_while(c, [c] { return !c->fl.empty(); });
    return r ? r : flow_flush(c);
}

static const uint8_t *ref_ptr(const jmh_ctx *c) {
    if (c->ref_kind == REF_REC) return c->ring[c->ref_entry].rec;
    if (c->ref_kind == REF_DBK) return c->ring[c->ref_entry].dbk;
    return c->d_ref;
}

// queue one picture (src: device 4:2:0 picture that stays valid until it is fully issued)
static int push_picture(jmh_ctx *c, const uint8_t *src, int entry, const jmh_frame_params *fp, bool readback) {
    const bool p_slice = fp->slice_type == JMH_P_SLICE;
    PicBuf &b = c->ring[entry];
    Flight f;
    memset(&f, 0, sizeof(f));
    f.id = c->next_id++;
    f.entry = entry;
    f.ref_entry = p_slice && (c->ref_kind == REF_REC || c->ref_kind == REF_DBK) ? c->ref_entry : -1;
    f.pred_id = -1;
    // EPZS temporal predictors read the motion field of the picture pushed last (the reference
    // itself when it is the previous picture on the device; otherwise a completed picture)
    f.tmv_entry = p_slice && c->cfg.search_mode == 3 && c->last_id >= 0 ? c->last_entry : -1;
    if (f.ref_entry >= 0)
        for (const Flight &g : c->fl)
            if (g.entry == f.ref_entry) f.pred_id = g.id;
    // the chained predecessor must be the picture right before this one in the flight list
    if (f.pred_id >= 0 && (c->fl.empty() || c->fl.back().id != f.pred_id)) {
        int r = drain(c);
        if (r) return r;
        f.pred_id = -1;
    }
    f.readback = readback;
    PicParams &q = f.pp;
    q.org = src; q.ref = ref_ptr(c);
    q.rec = b.rec; q.dbk = fp->deblock ? b.dbk : nullptr;
    q.mv = b.mv; q.refidx = b.refidx; q.ipred = b.ipred; q.res = b.res; q.scr = b.scr;
    q.tmv = f.tmv_entry >= 0 ? c->ring[f.tmv_entry].mv : nullptr;
    q.tref = f.tmv_entry >= 0 ? c->ring[f.tmv_entry].refidx : nullptr;
    q.slice_type = fp->slice_type; q.qp = fp->qp; q.lambda_mode = fp->lambda_mode; q.lambda_motion = fp->lambda_motion;
    q.cqp_off = fp->chroma_qp_offset;
    q.qsel = (int16_t)q_selector(c->cfg, fp->slice_type != JMH_P_SLICE);
    q.lf_disable = fp->lf_disable; q.lf_offA = 2 * fp->lf_alpha_div2; q.lf_offB = 2 * fp->lf_beta_div2;
    b.unpopped = readback;
    b.deblocked = fp->deblock != 0;
    if (c->cfg.rdo) {   // the picture's lambdas into its RdoPic (stream order: before its ticks)
        // the entry's previous occupant may have been queued without any host wait since (the
        // jmh_encode_slot path): its copy out of h_rp must have run before h_rp is rewritten
        HCHK(hipEventSynchronize(b.ev_rp));
        b.h_rp->lambda = fp->lambda_rd;
        b.h_rp->lf = fp->lambda_factor_rd;
        HCHK(hipMemcpyAsync(reinterpret_cast<uint8_t *>(b.scr) + rdo_pic_offset(c->nmb), b.h_rp, sizeof(RdoPic), hipMemcpyHostToDevice, c->st));
        HCHK(hipEventRecord(b.ev_rp, c->st));
    }
    if (c->flow) {
        FlowPic &fp2 = c->fpic[entry];
        fp2.pp = q;
        fp2.gen = ++b.gen;
        fp2.ref_entry = f.ref_entry;
        fp2.ref_gen = f.ref_entry >= 0 ? c->ring[f.ref_entry].gen : 0;
    }
    c->fl.push_back(f);
    c->last_id = f.id;
    c->last_entry = entry;
    c->timing.pictures++;
    const int id = f.id;
    // run until the new picture has started (older pictures advance up to PIPE_LAG diagonals)
    return issue_while(c, [c, id] {
        for (const Flight &g : c->fl)
            if (g.id == id) return !g.started;
        return false;
    });
}

static int check_params(const jmh_ctx *c, const jmh_frame_params *fp) {
    if (fp->slice_type != JMH_P_SLICE && fp->slice_type != JMH_I_SLICE) return JMH_E_UNSUPPORTED_CFG;
    if (fp->qp < 0 || fp->qp > 51 || fp->lambda_mode < 0 || fp->lambda_motion < 0 || fp->lambda_mode > JMH_LAMBDA_MAX ||
        fp->lambda_motion > JMH_LAMBDA_MAX) return JMH_E_INVALID_ARG;
    if (fp->deblock && (fp->lf_disable < 0 || fp->lf_disable > 2 || fp->lf_alpha_div2 < -6 || fp->lf_alpha_div2 > 6 ||
                        fp->lf_beta_div2 < -6 || fp->lf_beta_div2 > 6)) return JMH_E_INVALID_ARG;
    if (fp->slice_type == JMH_P_SLICE && c->ref_kind == REF_NONE) return JMH_E_STATE;
    // RDOptimization 1: lambda_mode > 0 and its factor (jm_lambda_rdo_on at QP 51 + QpBdOffset 12:
    // lambda = 0.85 * 2^((63 - 12) / 3) = 0.85 * 2^17, factor = 65536 * sqrt(lambda) ~ 2.2e7 < 2^25,
    // kept below 2^31 / 64 so that factor * mvbits fits the searches' 32-bit costs)
    if (c->cfg.rdo && !(fp->lambda_rd > 0 && fp->lambda_rd < 1e9 && fp->lambda_factor_rd > 0 && fp->lambda_factor_rd < (1 << 25)))
        return JMH_E_INVALID_ARG;
    return JMH_OK;
}

// claim the next ring entry: nothing in flight may touch it, its results must have been popped,
// and a reference that lives in it is copied out first
static int claim_entry(jmh_ctx *c, int *out) {
    const int e = c->next_entry;
    if (c->ring[e].unpopped) return JMH_E_STATE;
    int r = issue_while(c, [c, e] { return entry_busy(c, e); });
    if (r) return r;
    if (c->flow && ((c->seg_mask >> e) & 1) && (r = flow_flush(c))) return r;   // its last readers before its rewrite
    if ((c->ref_kind == REF_REC || c->ref_kind == REF_DBK) && c->ref_entry == e) {
        if ((r = drain(c))) return r;   // pictures in flight may still read d_ref
        HCHK(hipMemcpyAsync(c->d_ref, ref_ptr(c), c->fsize, hipMemcpyDeviceToDevice, c->st));
        c->ref_kind = REF_BUF;
        c->ref_entry = -1;
    }
    c->next_entry = (e + 1) % c->nring;
    *out = e;
    return JMH_OK;
}

extern "C" {

}  // extern "C"
static int set_reference_any(jmh_ctx *c, int list, int ref_idx, const void *y, const void *u, const void *v, int sy, int sc, bool wide) {
    if (!c || !y || !u || !v || sy < c->W || sc < c->Wc) return JMH_E_INVALID_ARG;
    if (list != 0 || ref_idx != 0) return JMH_E_UNSUPPORTED_CFG;
    int r = check_pic(c, wide);
    if (r) return r;
    HCHK(hipSetDevice(c->dev));
    r = drain(c);   // pictures in flight may read d_ref
    if (r) return r;
    HCHK(hipStreamSynchronize(c->st));   // staging buffer reuse
    if (!pack_planes(c->h_stage_ref, c->W, c->H, y, u, v, sy, sc, c->ps, c->maxv)) return JMH_E_INVALID_ARG;
    HCHK(hipMemcpyAsync(c->d_ref, c->h_stage_ref, c->fsize, hipMemcpyHostToDevice, c->st));
    c->ref_kind = REF_BUF; c->ref_entry = -1;
    return JMH_OK;
}
extern "C" {
int jmh_set_reference(jmh_ctx *c, int list, int ref_idx, const uint8_t *y, const uint8_t *u, const uint8_t *v, int sy, int sc) {
    return set_reference_any(c, list, ref_idx, y, u, v, sy, sc, false);
}
int jmh_set_reference_u16(jmh_ctx *c, int list, int ref_idx, const uint16_t *y, const uint16_t *u, const uint16_t *v, int sy, int sc) {
    return set_reference_any(c, list, ref_idx, y, u, v, sy, sc, true);
}

int jmh_set_reference_slot(jmh_ctx *c, int slot) {
    if (!c || slot < -2 || slot >= c->nslots) return JMH_E_INVALID_ARG;
    HCHK(hipSetDevice(c->dev));
    if (slot < 0) {   // the last pushed picture (its recon, or its device deblocking): no copy
        if (c->last_id < 0 || (slot == -2 && !c->ring[c->last_entry].deblocked)) return JMH_E_STATE;
        c->ref_kind = slot == -1 ? REF_REC : REF_DBK;
        c->ref_entry = c->last_entry;
        return JMH_OK;
    }
    int r = drain(c);
    if (r) return r;
    HCHK(hipMemcpyAsync(c->d_ref, c->d_slots + (size_t)slot * c->fsize, c->fsize, hipMemcpyDeviceToDevice, c->st));
    c->ref_kind = REF_BUF; c->ref_entry = -1;
    return JMH_OK;
}

}  // extern "C"
static int frame_push_any(jmh_ctx *c, const void *y, const void *u, const void *v, int sy, int sc, const jmh_frame_params *fp, bool wide) {
    if (!c || !y || !u || !v || !fp || sy < c->W || sc < c->Wc) return JMH_E_INVALID_ARG;
    int r = check_params(c, fp);
    if (r) return r;
    if ((r = check_pic(c, wide))) return r;
    if ((int)c->popq.size() >= c->depth) return JMH_E_STATE;
    HCHK(hipSetDevice(c->dev));
    int e;
    if ((r = claim_entry(c, &e))) return r;
    PicBuf &b = c->ring[e];
    if ((r = alloc_host(c, b))) return r;
    HCHK(hipEventSynchronize(b.ev_src));   // the previous H2D out of this staging buffer
    // an out-of-range sample rejects the picture before its own copy or ticks are queued: the
    // claimed entry stays free (nothing refers to it).  Not side-effect free: claiming the entry
    // may already have issued ticks of earlier pictures (legal progress of their wavefronts)
    if (!pack_planes(b.h_src, c->W, c->H, y, u, v, sy, sc, c->ps, c->maxv)) return JMH_E_INVALID_ARG;
    HCHK(hipEventRecord(b.ev_t0, c->st));
    HCHK(hipMemcpyAsync(b.src, b.h_src, c->fsize, hipMemcpyHostToDevice, c->st));
    HCHK(hipEventRecord(b.ev_src, c->st));
    c->popq.push_back(e);
    return push_picture(c, b.src, e, fp, true);
}
extern "C" {
int jmh_frame_push(jmh_ctx *c, const uint8_t *y, const uint8_t *u, const uint8_t *v, int sy, int sc, const jmh_frame_params *fp) {
    return frame_push_any(c, y, u, v, sy, sc, fp, false);
}
int jmh_frame_push_u16(jmh_ctx *c, const uint16_t *y, const uint16_t *u, const uint16_t *v, int sy, int sc, const jmh_frame_params *fp) {
    return frame_push_any(c, y, u, v, sy, sc, fp, true);
}

int jmh_frame_pop(jmh_ctx *c) {
    if (!c) return JMH_E_INVALID_ARG;
    if (c->popq.empty()) return JMH_E_STATE;
    HCHK(hipSetDevice(c->dev));
    const int e = c->popq.front();
    int r = issue_while(c, [c, e] {
        for (const Flight &f : c->fl)
            if (f.entry == e) return true;
        return false;
    });
    if (r) return r;
    // look-ahead: a lag of ticks more before waiting, so the device keeps working while the
    // caller writes the popped picture and reads the next one (the next push then needs that many
    // fewer ticks to start its picture; results are unchanged: ticks only advance legal diagonals)
    int ahead = PIPE_LAG;
    if ((r = issue_while(c, [c, &ahead] { return ahead-- > 0 && !c->fl.empty(); }))) return r;
    HCHK(hipEventSynchronize(c->ring[e].ev_done));
    if ((r = flow_check(c))) return r;
    c->popq.pop_front();
    c->ring[e].unpopped = 0;
    c->cur_entry = e;
    float ms = 0;
    if (hipEventElapsedTime(&ms, c->ring[e].ev_t0, c->ring[e].ev_done) == hipSuccess) c->timing.total_ms = ms;
    return JMH_OK;
}

int jmh_frame_submit(jmh_ctx *c, const uint8_t *y, const uint8_t *u, const uint8_t *v, int sy, int sc, const jmh_frame_params *fp) {
    return jmh_frame_push(c, y, u, v, sy, sc, fp);
}
int jmh_frame_submit_u16(jmh_ctx *c, const uint16_t *y, const uint16_t *u, const uint16_t *v, int sy, int sc, const jmh_frame_params *fp) {
    return jmh_frame_push_u16(c, y, u, v, sy, sc, fp);
}

int jmh_frame_wait(jmh_ctx *c) { return jmh_frame_pop(c); }

const jmh_mb_result *jmh_get_mb_result(const jmh_ctx *c, int mb_addr) {
    if (!c || c->cur_entry < 0 || mb_addr < 0 || mb_addr >= c->mbw * c->mbh) return nullptr;
    return &c->ring[c->cur_entry].h_res[mb_addr];
}

}  // extern "C"
static int read_pic(jmh_ctx *c, void *y, void *u, void *v, int sy, int sc, bool wide, bool dbk) {
    if (!c || !y || !u || !v || sy < c->W || sc < c->Wc) return JMH_E_INVALID_ARG;
    if ((c->bd > 8) != wide) return JMH_E_UNSUPPORTED_CFG;
    if (c->cur_entry < 0 || !(dbk ? c->ring[c->cur_entry].deblocked : c->ring[c->cur_entry].recon_read)) return JMH_E_STATE;
    const PicBuf &b = c->ring[c->cur_entry];
    unpack_planes(dbk ? b.h_dbk : b.h_rec, c->W, c->H, y, u, v, sy, sc, c->ps);
    return JMH_OK;
}
static int load_frame_any(jmh_ctx *c, int slot, const void *y, const void *u, const void *v, int sy, int sc, bool wide) {
    if (!c || slot < 0 || slot >= c->nslots || !y || !u || !v || sy < c->W || sc < c->Wc) return JMH_E_INVALID_ARG;
    int r = check_pic(c, wide);
    if (r) return r;
    HCHK(hipSetDevice(c->dev));
    r = drain(c);   // pictures in flight may read the slot
    if (r) return r;
    HCHK(hipStreamSynchronize(c->st));
    if (!pack_planes(c->h_stage_ref, c->W, c->H, y, u, v, sy, sc, c->ps, c->maxv)) return JMH_E_INVALID_ARG;
    HCHK(hipMemcpyAsync(c->d_slots + (size_t)slot * c->fsize, c->h_stage_ref, c->fsize, hipMemcpyHostToDevice, c->st));
    HCHK(hipStreamSynchronize(c->st));
    return JMH_OK;
}
extern "C" {
int jmh_read_recon(jmh_ctx *c, uint8_t *y, uint8_t *u, uint8_t *v, int sy, int sc) { return read_pic(c, y, u, v, sy, sc, false, false); }
int jmh_read_recon_u16(jmh_ctx *c, uint16_t *y, uint16_t *u, uint16_t *v, int sy, int sc) { return read_pic(c, y, u, v, sy, sc, true, false); }
int jmh_read_deblocked(jmh_ctx *c, uint8_t *y, uint8_t *u, uint8_t *v, int sy, int sc) { return read_pic(c, y, u, v, sy, sc, false, true); }
int jmh_read_deblocked_u16(jmh_ctx *c, uint16_t *y, uint16_t *u, uint16_t *v, int sy, int sc) { return read_pic(c, y, u, v, sy, sc, true, true); }
int jmh_load_frame(jmh_ctx *c, int slot, const uint8_t *y, const uint8_t *u, const uint8_t *v, int sy, int sc) {
    return load_frame_any(c, slot, y, u, v, sy, sc, false);
}
int jmh_load_frame_u16(jmh_ctx *c, int slot, const uint16_t *y, const uint16_t *u, const uint16_t *v, int sy, int sc) {
    return load_frame_any(c, slot, y, u, v, sy, sc, true);
}

int jmh_encode_slot(jmh_ctx *c, int slot, const jmh_frame_params *fp) {
    if (!c || !fp || slot < 0 || slot >= c->nslots) return JMH_E_INVALID_ARG;
    int r = check_params(c, fp);
    if (r) return r;
    HCHK(hipSetDevice(c->dev));
    int e;
    if ((r = claim_entry(c, &e))) return r;
    return push_picture(c, c->d_slots + (size_t)slot * c->fsize, e, fp, false);
}

int jmh_sync(jmh_ctx *c) {
    if (!c) return JMH_E_INVALID_ARG;
    HCHK(hipSetDevice(c->dev));
    int r = drain(c);
    if (r) return r;
    HCHK(hipStreamSynchronize(c->st));
    if ((r = flow_check(c))) return r;
    if (c->d_bprof && c->bprof_blocks) {   // debug: block durations of one tick, per role
        std::vector<unsigned long long> h(3 * c->bprof_blocks);
        HCHK(hipMemcpy(h.data(), c->d_bprof, h.size() * 8, hipMemcpyDeviceToHost));
        int rate_khz = 0;
        HCHK(hipDeviceGetAttribute(&rate_khz, hipDeviceAttributeWallClockRate, c->dev));
        double us = rate_khz > 0 ? 1e3 / rate_khz : 0.01;
        unsigned long long t0 = ~0ull, t1 = 0;
        double sum[5] = {0, 0, 0, 0, 0}, mx[5] = {0, 0, 0, 0, 0};
        std::vector<double> durs[5];
        std::vector<std::pair<double, unsigned long long>> slow;   // role-2 blocks: (duration, i)
        int n[5] = {0, 0, 0, 0, 0};
        unsigned long long f0 = ~0ull, f1 = 0, r0[5], r1[5];
        for (int r = 0; r < 5; r++) { r0[r] = ~0ull; r1[r] = 0; }
        for (int i = 0; i < c->bprof_blocks; i++) {
            unsigned long long a = h[3 * i], b = h[3 * i + 1];
            int role = (int)(h[3 * i + 2] & 15);                   // k_mb_analyse: | MB << 4 | entry << 32
            if (!a || role < 0 || role > 4 || b < a) continue;   // 0: padding block, not written
            if (role == 2) slow.push_back({(double)(b - a) * us, (unsigned long long)i});
            if (role == 3) { f0 = a < f0 ? a : f0; f1 = b > f1 ? b : f1; }
            r0[role] = a < r0[role] ? a : r0[role]; r1[role] = b > r1[role] ? b : r1[role];
            t0 = a < t0 ? a : t0; t1 = b > t1 ? b : t1;
            double dur = (double)(b - a) * us;
            sum[role] += dur; n[role]++; mx[role] = dur > mx[role] ? dur : mx[role];
            durs[role].push_back(dur);
        }
        fprintf(stderr, "jmh_blocks tick=%d blocks=%d span=%.1fus", c->bprof_tick, c->bprof_blocks, (double)(t1 - t0) * us);
        for (int r = 0; r < 5; r++)
            if (n[r]) {
                std::sort(durs[r].begin(), durs[r].end());
                fprintf(stderr, " role%d: n=%d mean=%.1fus p50=%.1f p90=%.1f max=%.1fus (from %.1f to %.1fus)", r, n[r], sum[r] / n[r],
                        durs[r][n[r] / 2], durs[r][(9 * n[r]) / 10], mx[r], (double)(r0[r] - t0) * us, (double)(r1[r] - t0) * us);
            }
        if (f1) fprintf(stderr, " final: first start %.1fus after the analysis' first, span %.1fus", (double)(f0 - t0) * us, (double)(f1 - f0) * us);
        fprintf(stderr, "\n");
        if (!slow.empty()) {                                    // the slowest motion-search blocks: which MBs
            std::sort(slow.begin(), slow.end());
            fprintf(stderr, "jmh_blocks slowest role2 (mbx,mby,entry start+dur us):");
            for (size_t k = slow.size() > 12 ? slow.size() - 12 : 0; k < slow.size(); k++) {
                const unsigned long long i = slow[k].second, tg = h[3 * i + 2];
                const int mb = (int)((tg >> 4) & 0xFFFFFFFu), en = (int)(tg >> 32);
                fprintf(stderr, " (%d,%d,%d %.1f+%.1f)", mb % c->mbw, mb / c->mbw, en, (double)(h[3 * i] - t0) * us, slow[k].first);
            }
            double xs[8] = {0}, xm[8] = {0};                     // per XCD (hardware block % 8)
            int xn[8] = {0};
            for (auto &q : slow) { const int x = (int)(q.second % 8); xs[x] += q.first; xn[x]++; xm[x] = q.first > xm[x] ? q.first : xm[x]; }
            fprintf(stderr, " per XCD mean/max:");
            for (int x = 0; x < 8; x++) if (xn[x]) fprintf(stderr, " %d:%.1f/%.1f", x, xs[x] / xn[x], xm[x]);
            fprintf(stderr, " fastest:");
            for (size_t k = 0; k < slow.size() && k < 6; k++) {
                const unsigned long long i = slow[k].second, tg = h[3 * i + 2];
                const int mb = (int)((tg >> 4) & 0xFFFFFFFu), en = (int)(tg >> 32);
                fprintf(stderr, " (%d,%d,%d %.1f+%.1f)", mb % c->mbw, mb / c->mbw, en, (double)(h[3 * i] - t0) * us, slow[k].first);
            }
            fprintf(stderr, "\n");
        }
        c->bprof_blocks = 0;
    }
    if (c->d_prof) {   // debug: phase timestamps of MB prof_mb (first picture of a tick)
        unsigned long long h[64];
        int rate_khz = 0;
        HCHK(hipMemcpy(h, c->d_prof, sizeof(h), hipMemcpyDeviceToHost));
        HCHK(hipDeviceGetAttribute(&rate_khz, hipDeviceAttributeWallClockRate, c->dev));
        double us = rate_khz > 0 ? 1e3 / rate_khz : 0.01;
        unsigned long long t0 = ~0ull;
        for (int k = 0; k < 64; k++) if (k != 31 && h[k] && h[k] < t0) t0 = h[k];   // [31]: a count
        fprintf(stderr, "jmh_phase mb=%d us since first stamp:", c->prof_mb);
        for (int k = 0; k < 64; k++)
            if (k == 31 && h[k]) fprintf(stderr, " [31]#%llu", h[k]);
            else if (h[k]) fprintf(stderr, " [%d]%.2f", k, (double)(h[k] - t0) * us);
        fprintf(stderr, "\n");
        HCHK(hipMemset(c->d_prof, 0, sizeof(h)));
    }
    return JMH_OK;
}

int jmh_wait_issued(jmh_ctx *c) {
    if (!c) return JMH_E_INVALID_ARG;
    HCHK(hipSetDevice(c->dev));
    int r = flow_flush(c);
    if (r) return r;
    HCHK(hipStreamSynchronize(c->st));
    return flow_check(c);
}

int jmh_get_timing(jmh_ctx *c, jmh_timing *t) {
    if (!c || !t) return JMH_E_INVALID_ARG;
    HCHK(hipSetDevice(c->dev));
    int r = flow_flush(c);
    if (r) return r;
    HCHK(hipStreamSynchronize(c->st));   // the issued launches only: pictures in flight stay
    int npic = 0;
    ring_drain(c->ring_interp, c->timing.interp_ms, c->timing.interps);
    ring_drain(c->ring_mb, c->timing.mb_ms, npic);
    if (c->ring_an.cap) {
        ring_drain(c->ring_an, c->timing.analyse_ms, c->timing.analyse_launches);
        ring_drain(c->ring_fin, c->timing.final_ms, c->timing.final_launches);
    }
    *t = c->timing;
    // counters restart (total_ms stays: the last popped picture)
    c->timing.pictures = 0; c->timing.mb_launches = 0; c->timing.ticks = 0; c->timing.tick_mbs = 0;
    c->timing.pictures_done = 0;
    c->timing.flow_launches = 0; c->timing.flow_mbs = 0;
    return flow_check(c);
}

int jmh_ffs_sad_table(jmh_ctx *c, int n_mb, const int32_t *mb_xy, const int32_t *centres, uint16_t *out) {
    if (!c || n_mb <= 0 || !mb_xy || !centres || !out) return JMH_E_INVALID_ARG;
    for (int i = 0; i < n_mb; i++)
        if (mb_xy[2 * i] < 0 || mb_xy[2 * i] >= c->mbw || mb_xy[2 * i + 1] < 0 || mb_xy[2 * i + 1] >= c->mbh) return JMH_E_INVALID_ARG;
    if (c->ref_kind == REF_NONE) return JMH_E_STATE;
    if (c->bd > 8) return JMH_E_UNSUPPORTED_CFG;   // the 8-bit SAD-table seam (High 10: jmh_ffs_sad_table_u16)
    HCHK(hipSetDevice(c->dev));
    int r = drain(c);
    if (r) return r;
    int32_t *d_xy = nullptr, *d_c = nullptr;
    uint16_t *d_out = nullptr;
    size_t on = (size_t)n_mb * 16 * c->npos;
    DevTemps tmp;
    HCHK(tmp.alloc(&d_xy, n_mb * 8));
    HCHK(tmp.alloc(&d_c, n_mb * 8));
    HCHK(tmp.alloc(&d_out, on * 2));
    HCHK(hipMemcpyAsync(d_xy, mb_xy, n_mb * 8, hipMemcpyHostToDevice, c->st));
    HCHK(hipMemcpyAsync(d_c, centres, n_mb * 8, hipMemcpyHostToDevice, c->st));
    HCHK(jmh_launch_sad_table(c->d_slots, ref_ptr(c), c->W, c->H, c->sr, n_mb, d_xy, d_c, d_out, c->st));
    HCHK(hipMemcpyAsync(out, d_out, on * 2, hipMemcpyDeviceToHost, c->st));
    HCHK(hipStreamSynchronize(c->st));
    return JMH_OK;
}

int jmh_tq4x4_batch(jmh_ctx *c, int n, const int16_t *resid, const uint8_t *pred, int qp, int intra, int16_t *levels,
                    uint8_t *recon, int32_t *coeff_cost, int32_t *nonzero) {
    if (!c || n <= 0 || !resid || !pred || !levels || !recon || !coeff_cost || !nonzero || qp < 0 || qp > 51) return JMH_E_INVALID_ARG;
    HCHK(hipSetDevice(c->dev));
    int16_t *dr, *dl;
    uint8_t *dp, *drec;
    int32_t *dcc, *dnz;
    DevTemps tmp;
    HCHK(tmp.alloc(&dr, (size_t)n * 32)); HCHK(tmp.alloc(&dl, (size_t)n * 32));
    HCHK(tmp.alloc(&dp, (size_t)n * 16)); HCHK(tmp.alloc(&drec, (size_t)n * 16));
    HCHK(tmp.alloc(&dcc, (size_t)n * 4)); HCHK(tmp.alloc(&dnz, (size_t)n * 4));
    HCHK(hipMemcpyAsync(dr, resid, n * 32, hipMemcpyHostToDevice, c->st));
    HCHK(hipMemcpyAsync(dp, pred, n * 16, hipMemcpyHostToDevice, c->st));
    HCHK(jmh_launch_tq4x4(n, dr, dp, qp, q_selector(c->cfg, intra != 0), dl, drec, dcc, dnz, c->st));
    HCHK(hipMemcpyAsync(levels, dl, n * 32, hipMemcpyDeviceToHost, c->st));
    HCHK(hipMemcpyAsync(recon, drec, n * 16, hipMemcpyDeviceToHost, c->st));
    HCHK(hipMemcpyAsync(coeff_cost, dcc, n * 4, hipMemcpyDeviceToHost, c->st));
    HCHK(hipMemcpyAsync(nonzero, dnz, n * 4, hipMemcpyDeviceToHost, c->st));
    HCHK(hipStreamSynchronize(c->st));
    return JMH_OK;
}

int jmh_tq8x8_batch(jmh_ctx *c, int n, const int16_t *resid, const uint8_t *pred, int qp, int intra, int16_t *levels,
                    uint8_t *recon, int32_t *coeff_cost, int32_t *nonzero) {
    if (!c || n <= 0 || !resid || !pred || !levels || !recon || !coeff_cost || !nonzero || qp < 0 || qp > 51) return JMH_E_INVALID_ARG;
    HCHK(hipSetDevice(c->dev));
    int16_t *dr, *dl;
    uint8_t *dp, *drec;
    int32_t *dcc, *dnz;
    DevTemps tmp;
    HCHK(tmp.alloc(&dr, (size_t)n * 128)); HCHK(tmp.alloc(&dl, (size_t)n * 128));
    HCHK(tmp.alloc(&dp, (size_t)n * 64)); HCHK(tmp.alloc(&drec, (size_t)n * 64));
    HCHK(tmp.alloc(&dcc, (size_t)n * 4)); HCHK(tmp.alloc(&dnz, (size_t)n * 4));
    HCHK(hipMemcpyAsync(dr, resid, n * 128, hipMemcpyHostToDevice, c->st));
    HCHK(hipMemcpyAsync(dp, pred, n * 64, hipMemcpyHostToDevice, c->st));
    HCHK(jmh_launch_tq8x8(n, dr, dp, qp, q_selector(c->cfg, intra != 0), dl, drec, dcc, dnz, c->st));
    HCHK(hipMemcpyAsync(levels, dl, n * 128, hipMemcpyDeviceToHost, c->st));
    HCHK(hipMemcpyAsync(recon, drec, n * 64, hipMemcpyDeviceToHost, c->st));
    HCHK(hipMemcpyAsync(coeff_cost, dcc, n * 4, hipMemcpyDeviceToHost, c->st));
    HCHK(hipMemcpyAsync(nonzero, dnz, n * 4, hipMemcpyDeviceToHost, c->st));
    HCHK(hipStreamSynchronize(c->st));
    return JMH_OK;
}

int jmh_search_pictures(jmh_ctx *c, const uint8_t *cur_y, const uint8_t *ref_y, int sy) {
    if (!c || !cur_y || !ref_y || sy < c->W) return JMH_E_INVALID_ARG;
    HCHK(hipSetDevice(c->dev));
    const size_t ls = (size_t)c->W * c->H;
    if (!c->d_scur) {
        if (hipMalloc((void **)&c->d_scur, ls) != hipSuccess) return JMH_E_OOM;
        if (hipMalloc((void **)&c->d_sref, ls) != hipSuccess) { (void)hipFree(c->d_scur); c->d_scur = nullptr; return JMH_E_OOM; }
    }
    HCHK(hipStreamSynchronize(c->st));   // an earlier search may still read the buffers
    HCHK(hipMemcpy2DAsync(c->d_scur, c->W, cur_y, sy, c->W, c->H, hipMemcpyHostToDevice, c->st));
    HCHK(hipMemcpy2DAsync(c->d_sref, c->W, ref_y, sy, c->W, c->H, hipMemcpyHostToDevice, c->st));
    HCHK(hipStreamSynchronize(c->st));
    return JMH_OK;
}

static int check_block_requests(const jmh_ctx *c, int n, const jmh_block_search *req) {
    for (int i = 0; i < n; i++) {   // the kernel's block and window assumptions, checked on the host
        const jmh_block_search &q = req[i];
        if (q.blocktype < 1 || q.blocktype > 7 || q.mb_x < 0 || q.mb_x >= c->mbw || q.mb_y < 0 || q.mb_y >= c->mbh) return JMH_E_INVALID_ARG;
        static const int bw4[8] = {4, 4, 4, 2, 2, 2, 1, 1}, bh4[8] = {4, 4, 2, 4, 2, 1, 2, 1};
        if (q.block_x < 0 || q.block_y < 0 || q.block_x + bw4[q.blocktype] > 4 || q.block_y + bh4[q.blocktype] > 4) return JMH_E_INVALID_ARG;
        if (q.search_range < 0 || q.search_range > c->sr) return JMH_E_INVALID_ARG;
        if (q.search_range > SRMAX) return JMH_E_UNSUPPORTED_CFG;   // 13-bit spiral order keys: (2 SR + 1)^2 < 8192
        if (q.lambda_factor < 0 || q.lambda_factor > (1 << 24)) return JMH_E_INVALID_ARG;
        if (q.search_mode != 0 && q.search_mode != -1) return JMH_E_UNSUPPORTED_CFG;
        if (abs(q.centre[0]) > 2048 || abs(q.centre[1]) > 2048 || abs(q.pred_mv[0]) > 8192 || abs(q.pred_mv[1]) > 8192) return JMH_E_INVALID_ARG;
    }
    return JMH_OK;
}
int jmh_block_motion_search(jmh_ctx *c, int n, const jmh_block_search *req, jmh_block_result *res) {
    if (!c || n <= 0 || !req || !res) return JMH_E_INVALID_ARG;
    if (!c->d_scur) return JMH_E_STATE;
    int r = check_block_requests(c, n, req);
    if (r) return r;
    HCHK(hipSetDevice(c->dev));
    DevTemps tmp;
    jmh_block_search *d_req;
    jmh_block_result *d_res;
    HCHK(tmp.alloc(&d_req, (size_t)n * sizeof(jmh_block_search)));
    HCHK(tmp.alloc(&d_res, (size_t)n * sizeof(jmh_block_result)));
    HCHK(hipMemcpyAsync(d_req, req, (size_t)n * sizeof(jmh_block_search), hipMemcpyHostToDevice, c->st));
    HCHK(jmh_launch_block_search(n, d_req, d_res, c->d_scur, c->d_sref, c->W, c->H, c->cfg.use_hadamard, c->st));
    HCHK(hipMemcpyAsync(res, d_res, (size_t)n * sizeof(jmh_block_result), hipMemcpyDeviceToHost, c->st));
    HCHK(hipStreamSynchronize(c->st));
    return JMH_OK;
}

// ---- High 10 seams (16-bit samples) ----------------------------------------------------------
int jmh_search_pictures_u16(jmh_ctx *c, const uint16_t *cur_y, const uint16_t *ref_y, int sy, int bit_depth) {
    if (!c || !cur_y || !ref_y || sy < c->W || bit_depth < 8 || bit_depth > 10) return JMH_E_INVALID_ARG;
    const int maxv = (1 << bit_depth) - 1;
    for (int y = 0; y < c->H; y++)   // out-of-range samples would break the 19-bit cost keys
        for (int x = 0; x < c->W; x++)
            if (cur_y[(size_t)y * sy + x] > maxv || ref_y[(size_t)y * sy + x] > maxv) return JMH_E_INVALID_ARG;
    HCHK(hipSetDevice(c->dev));
    const size_t ls = (size_t)c->W * c->H * 2;
    if (!c->d_scur16) {
        if (hipMalloc((void **)&c->d_scur16, ls) != hipSuccess) return JMH_E_OOM;
        if (hipMalloc((void **)&c->d_sref16, ls) != hipSuccess) { (void)hipFree(c->d_scur16); c->d_scur16 = nullptr; return JMH_E_OOM; }
    }
    HCHK(hipStreamSynchronize(c->st));   // an earlier search may still read the buffers
    HCHK(hipMemcpy2DAsync(c->d_scur16, (size_t)c->W * 2, cur_y, (size_t)sy * 2, (size_t)c->W * 2, c->H, hipMemcpyHostToDevice, c->st));
    HCHK(hipMemcpy2DAsync(c->d_sref16, (size_t)c->W * 2, ref_y, (size_t)sy * 2, (size_t)c->W * 2, c->H, hipMemcpyHostToDevice, c->st));
    HCHK(hipStreamSynchronize(c->st));
    c->hbd_bits = bit_depth;
    return JMH_OK;
}
int jmh_block_motion_search_u16(jmh_ctx *c, int n, const jmh_block_search *req, jmh_block_result *res) {
    if (!c || n <= 0 || !req || !res) return JMH_E_INVALID_ARG;
    if (!c->d_scur16) return JMH_E_STATE;
    int r = check_block_requests(c, n, req);
    if (r) return r;
    HCHK(hipSetDevice(c->dev));
    DevTemps tmp;
    jmh_block_search *d_req;
    jmh_block_result *d_res;
    HCHK(tmp.alloc(&d_req, (size_t)n * sizeof(jmh_block_search)));
    HCHK(tmp.alloc(&d_res, (size_t)n * sizeof(jmh_block_result)));
    HCHK(hipMemcpyAsync(d_req, req, (size_t)n * sizeof(jmh_block_search), hipMemcpyHostToDevice, c->st));
    HCHK(jmh_launch_block_search_u16(n, d_req, d_res, c->d_scur16, c->d_sref16, c->W, c->H, c->cfg.use_hadamard, c->hbd_bits, c->st));
    HCHK(hipMemcpyAsync(res, d_res, (size_t)n * sizeof(jmh_block_result), hipMemcpyDeviceToHost, c->st));
    HCHK(hipStreamSynchronize(c->st));
    return JMH_OK;
}
int jmh_ffs_sad_table_u16(jmh_ctx *c, int n_mb, const int32_t *mb_xy, const int32_t *centres, uint16_t *out) {
    if (!c || n_mb <= 0 || !mb_xy || !centres || !out) return JMH_E_INVALID_ARG;
    for (int i = 0; i < n_mb; i++)
        if (mb_xy[2 * i] < 0 || mb_xy[2 * i] >= c->mbw || mb_xy[2 * i + 1] < 0 || mb_xy[2 * i + 1] >= c->mbh ||
            abs(centres[2 * i]) > c->sr || abs(centres[2 * i + 1]) > c->sr) return JMH_E_INVALID_ARG;
    if (!c->d_scur16) return JMH_E_STATE;
    HCHK(hipSetDevice(c->dev));
    int32_t *d_xy = nullptr, *d_c = nullptr;
    uint16_t *d_out = nullptr;
    const size_t on = (size_t)n_mb * 16 * c->npos;
    DevTemps tmp;
    HCHK(tmp.alloc(&d_xy, n_mb * 8));
    HCHK(tmp.alloc(&d_c, n_mb * 8));
    HCHK(tmp.alloc(&d_out, on * 2));
    HCHK(hipMemcpyAsync(d_xy, mb_xy, n_mb * 8, hipMemcpyHostToDevice, c->st));
    HCHK(hipMemcpyAsync(d_c, centres, n_mb * 8, hipMemcpyHostToDevice, c->st));
    HCHK(jmh_launch_sad_table_u16(c->d_scur16, c->d_sref16, c->W, c->H, c->sr, n_mb, d_xy, d_c, d_out, c->st));
    HCHK(hipMemcpyAsync(out, d_out, on * 2, hipMemcpyDeviceToHost, c->st));
    HCHK(hipStreamSynchronize(c->st));
    return JMH_OK;
}
}  // extern "C"
// dct_luma / dct_luma8x8 at bit_depth (EL = 16 or 64 samples per block)
template <int EL>
static int tq_batch_u16(jmh_ctx *c, int n, const int16_t *resid, const uint16_t *pred, int qp, int intra, int bit_depth, int16_t *levels,
                        uint16_t *recon, int32_t *coeff_cost, int32_t *nonzero) {
    if (!c || n <= 0 || !resid || !pred || !levels || !recon || !coeff_cost || !nonzero || qp < 0 || qp > 51 || bit_depth < 8 ||
        bit_depth > 10) return JMH_E_INVALID_ARG;
    const int maxv = (1 << bit_depth) - 1;
    for (size_t k = 0; k < (size_t)n * EL; k++)   // the int32 headroom of the quantiser assumes these ranges
        if (pred[k] > maxv || resid[k] > maxv || resid[k] < -maxv) return JMH_E_INVALID_ARG;
    HCHK(hipSetDevice(c->dev));
    int16_t *dr, *dl;
    uint16_t *dp, *drec;
    int32_t *dcc, *dnz;
    DevTemps tmp;
    HCHK(tmp.alloc(&dr, (size_t)n * EL * 2)); HCHK(tmp.alloc(&dl, (size_t)n * EL * 2));
    HCHK(tmp.alloc(&dp, (size_t)n * EL * 2)); HCHK(tmp.alloc(&drec, (size_t)n * EL * 2));
    HCHK(tmp.alloc(&dcc, (size_t)n * 4)); HCHK(tmp.alloc(&dnz, (size_t)n * 4));
    HCHK(hipMemcpyAsync(dr, resid, (size_t)n * EL * 2, hipMemcpyHostToDevice, c->st));
    HCHK(hipMemcpyAsync(dp, pred, (size_t)n * EL * 2, hipMemcpyHostToDevice, c->st));
    if (EL == 16) HCHK(jmh_launch_tq4x4_u16(n, dr, dp, qp, q_selector(c->cfg, intra != 0), bit_depth, dl, drec, dcc, dnz, c->st));
    else HCHK(jmh_launch_tq8x8_u16(n, dr, dp, qp, q_selector(c->cfg, intra != 0), bit_depth, dl, drec, dcc, dnz, c->st));
    HCHK(hipMemcpyAsync(levels, dl, (size_t)n * EL * 2, hipMemcpyDeviceToHost, c->st));
    HCHK(hipMemcpyAsync(recon, drec, (size_t)n * EL * 2, hipMemcpyDeviceToHost, c->st));
    HCHK(hipMemcpyAsync(coeff_cost, dcc, (size_t)n * 4, hipMemcpyDeviceToHost, c->st));
    HCHK(hipMemcpyAsync(nonzero, dnz, (size_t)n * 4, hipMemcpyDeviceToHost, c->st));
    HCHK(hipStreamSynchronize(c->st));
    return JMH_OK;
}
extern "C" {
int jmh_tq4x4_batch_u16(jmh_ctx *c, int n, const int16_t *resid, const uint16_t *pred, int qp, int intra, int bit_depth, int16_t *levels,
                        uint16_t *recon, int32_t *coeff_cost, int32_t *nonzero) {
    return tq_batch_u16<16>(c, n, resid, pred, qp, intra, bit_depth, levels, recon, coeff_cost, nonzero);
}
int jmh_tq8x8_batch_u16(jmh_ctx *c, int n, const int16_t *resid, const uint16_t *pred, int qp, int intra, int bit_depth, int16_t *levels,
                        uint16_t *recon, int32_t *coeff_cost, int32_t *nonzero) {
    return tq_batch_u16<64>(c, n, resid, pred, qp, intra, bit_depth, levels, recon, coeff_cost, nonzero);
}

/* test seam: quarter-pel planes of the current reference, [16][H+8][W+8] (UnifiedOneForthPix) */
int jmh_read_qpel(jmh_ctx *c, uint8_t *out) {
    if (!c || !out) return JMH_E_INVALID_ARG;
    if (c->ref_kind == REF_NONE) return JMH_E_STATE;
    if (c->bd > 8) return JMH_E_UNSUPPORTED_CFG;   // 8-bit phase planes
    HCHK(hipSetDevice(c->dev));
    int r = drain(c);
    if (r) return r;
    HCHK(ring_begin(c->ring_interp, c->st));
    HCHK(jmh_launch_interp(ref_ptr(c), c->W, c->H, c->d_qpel, c->qstride, c->qplane, c->st));
    HCHK(ring_end(c->ring_interp, c->st));
    HCHK(hipMemcpyAsync(out, c->d_qpel, (size_t)16 * c->qplane, hipMemcpyDeviceToHost, c->st));
    HCHK(hipStreamSynchronize(c->st));
    return JMH_OK;
}

}  // extern "C"
