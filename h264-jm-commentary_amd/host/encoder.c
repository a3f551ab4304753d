/*
 * encoder.c — sequence / picture driver, restating JM 8.6 lencod.c › main frame loop and
 * image.c › encode_one_frame [J]: read (or synthesise) the picture, choose I/P, run the
 * macroblock hot path through the backend (encode_one_macroblock for every MB), write the
 * slice (CAVLC), deblock the reconstruction, make it the reference (UnifiedOneForthPix runs in
 * the backend), write the recon, print JM's per-frame report line.
 */
#include <math.h>
#include <pthread.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
#include "jmhost.h"

static double now_ms(void) {
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return ts.tv_sec * 1e3 + ts.tv_nsec * 1e-6;
}

int jm_lambda_rdo_off(int qp) {
    static const int QP2QUANT[40] = {1, 1, 1, 1, 2, 2, 2, 2, 3, 3, 3, 4, 4, 4,
                                     5, 6, 6, 7, 8, 9, 10, 11, 13, 14, 16, 18, 20, 23,
                                     25, 29, 32, 36, 40, 45, 51, 57, 64, 72, 81, 91};
    int i = qp - 12;
    return QP2QUANT[i < 0 ? 0 : i];
}

/* RDOptimization 1 (rdopt.c encode_one_macroblock [J], no B pictures): lambda_mode = 0.85 *
   2^((QP - SHIFT_QP) / 3) at QP + QpBdOffsetY (JM >= 13 init_lambda's bitdepth_luma_qp_scale),
   lambda_motion = sqrt(lambda_mode), LAMBDA_FACTOR = (int)(65536 * lambda_motion + 0.5) */
double jm_lambda_rdo_on(int qp, int bit_depth, int *lambda_factor) {
    const int qpbd = bit_depth > 8 ? 6 * (bit_depth - 8) : 0;
    const double lam = 0.85 * pow(2.0, (double)(qp + qpbd - 12) / 3.0);
    if (lambda_factor) *lambda_factor = (int)(65536.0 * sqrt(lam) + 0.5);
    return lam;
}

/* squared error summed in integers (per row in 32 bits: 65025 * w < 2^32 for w < 66051; 64-bit
   rows at High 10), so the value equals JM's double accumulation of integer squares exactly; the
   peak is (1 << bit depth) - 1 (JM >= 10 img->max_imgpel_value [J]) */
static double psnr_pl(const jm_pic *a, const jm_pic *b, int pl, int w, int h) {
    uint64_t se = 0;
    const int st = pl ? a->w / 2 : a->w;
    const size_t off = pl == 0 ? 0 : (size_t)a->w * a->h + (size_t)(pl - 1) * (a->w / 2) * (a->h / 2);
    for (int y = 0; y < h; y++) {
        uint64_t r = 0;
        if (a->bd > 8) {
            const uint16_t *pa = a->Y + off + (size_t)y * st, *pb = b->Y + off + (size_t)y * st;
            for (int x = 0; x < w; x++) { const int d = pa[x] - pb[x]; r += (uint64_t)(d * d); }
        } else {
            const uint8_t *pa = a->y + off + (size_t)y * st, *pb = b->y + off + (size_t)y * st;
            uint32_t r32 = 0;
            for (int x = 0; x < w; x++) { const int d = pa[x] - pb[x]; r32 += (uint32_t)(d * d); }
            r = r32;
        }
        se += r;
    }
    if (se == 0) return 99.0;
    const double peak = a->bd > 8 ? (double)((1 << a->bd) - 1) : 255.0;
    return 10.0 * log10(peak * peak * w * h / (double)se);
}

/* slice.c › encode_one_slice [J]: the macroblock loop of one slice through the JM 8.6 call
 * surface (host/jm86.c): start_macroblock, encode_one_macroblock, write_one_macroblock.
 * image.c › code_a_picture [J] runs it for every slice of the picture (SliceMode 1: SliceArgument
 * MBs each, raster order); each slice is its own NAL unit, appended to out.  One slice writer
 * serves the picture (jm_slice_restart between slices). */
static void encode_one_slice(const jm_seq *s, int first) {
    const int nmb = s->mbw * s->mbh, end = s->slice_mbs > 0 && first + s->slice_mbs < nmb ? first + s->slice_mbs : nmb;
    img->slice_first = first;
    for (int a = first; a < end; a++) {
        img->current_mb_nr = a;
        start_macroblock();
        encode_one_macroblock();
        write_one_macroblock();
    }
}
static int encode_picture_slices(jm86_img *im, const jm_seq *s, const jm_slice *sl0, const jmh_frame_params *fp,
                                 const jm_pic *cur, const jm_pic *ref, jm_bits *out) {
    const int nmb = s->mbw * s->mbh, step = s->slice_mbs > 0 ? s->slice_mbs : nmb;
    const long len0 = out->len;
    jm_slice sl = *sl0;
    sl.first_mb = 0;
    jm_bits rbsp[2];             /* the slice being written and the next one (alternating) */
    int k = 0, nslices = 0;
    long bins = 0;
    jm_bits_init(&rbsp[0]);
    jm_slice_writer *w = jm_slice_begin(&rbsp[0], s, &sl);
    if (!w) { jm_bits_free(&rbsp[0]); return JMH_E_OOM; }
    int r = jm86_start_picture(im, fp, cur, ref, w);
    if (r) { jm_slice_end(w); jm_bits_free(&rbsp[0]); return r; }
    for (int first = 0; first < nmb; first += step) {
        encode_one_slice(s, first);
        if (first + step >= nmb) {
            long chk, bad;
            jm_slice_rate_check(w, &chk, &bad);
            im->rate_checked += chk;
            im->rate_mismatches += bad;
            bins = jm_slice_end(w);
        } else {
            jm_bits_init(&rbsp[k ^ 1]);
            sl.first_mb = first + step;
            jm_slice_restart(w, &rbsp[k ^ 1], &sl);
        }
        jm_write_nal(out, sl0->idr ? 3 : 2, sl0->idr ? 5 : 1, &rbsp[k]);
        jm_bits_free(&rbsp[k]);
        nslices++;
        k ^= 1;
    }
    im->writer = NULL;
    if (s->entropy_coding) {
        /* cabac_zero_words (7.4.2.10, 9.3.4.6): BinCountsInNALunits <= 32/3 * NumBytesInVclNALunits
           + RawMbBits * PicSizeInMbs / 32 (4:2:0: RawMbBits = 256 * BitDepthY + 128 * BitDepthC, 3072 at
           8 bits, 3840 at High 10); scaled by 3, so 3 * RawMbBits / 32 = 36 * BitDepth per MB.  Each word
           appended to the last slice is 0x000003 in the byte stream (emulation prevention). */
        const long bytes = out->len - len0 - 4L * nslices;          /* NAL units, no start codes */
        const int bd = s->bit_depth > 8 ? s->bit_depth : 8;
        const long excess = 3 * bins - 36L * bd * nmb - 32 * bytes;
        for (long z = excess > 0 ? (excess + 95) / 96 : 0; z > 0; z--) {
            static const uint8_t zw[3] = {0, 0, 3};
            jm_bits t = {(uint8_t *)zw, 3, 3, 0, 0};
            jm_bits_append(out, &t);
        }
    }
    return JMH_OK;
}

/* ---- parallel slice writing (WriterThreads > 0, pipelined device backend) -------------------
 * The slices of different pictures are independent once their macroblock results exist (one
 * slice per picture, device deblocking), so popped pictures are written by a pool of threads,
 * each with its own JM state (img is thread-local), and emitted in picture order.  The main
 * thread keeps the device busy: pop, copy the results and the deblocked picture into a job,
 * push the next picture. */
typedef struct wjob {
    jm86_img im;                 /* the job's JM state; im.mb_data holds the picture's results   */
    jm_pic rec;                  /* its deblocked reconstruction                                 */
    const jm_pic *cur;           /* its source (pend slot, not refilled before the job is flushed) */
    jmh_frame_params fp;
    jm_slice sl;
    int f, is_i;
    double met;                  /* backend time charged to the picture (report line)           */
    jm_bits out;                 /* NAL unit                                                     */
    long pic_bits;
    double py, pu, pv, write_ms;
    int status, state;           /* state: 0 idle, 1 queued, 2 running, 3 done                   */
} wjob_t;

typedef struct wpool {
    pthread_mutex_t mu;
    pthread_cond_t cv_work, cv_done;
    wjob_t *jobs;
    int nj, stop;
    int *queue, qh, qt;          /* job indices, FIFO */
    const jm_seq *s;
    const jm_input *inp;
    pthread_t *th;
    int nth;
} wpool_t;

static int encode_picture_slices(jm86_img *im, const jm_seq *s, const jm_slice *sl0, const jmh_frame_params *fp,
                                 const jm_pic *cur, const jm_pic *ref, jm_bits *out);

static void job_run(wpool_t *P, wjob_t *j) {
    const jm_seq *s = P->s;
    const jm_input *inp = P->inp;
    const int W = s->width;
    double t0 = now_ms();
    j->out.len = 0;
    j->status = encode_picture_slices(&j->im, s, &j->sl, &j->fp, j->cur, &j->rec, &j->out);
    j->pic_bits = j->out.len * 8;
    j->py = psnr_pl(j->cur, &j->rec, 0, inp->width, inp->height);
    j->pu = psnr_pl(j->cur, &j->rec, 1, inp->width / 2, inp->height / 2);
    j->pv = psnr_pl(j->cur, &j->rec, 2, inp->width / 2, inp->height / 2);
    (void)W;
    j->write_ms = now_ms() - t0;
}

static void *writer_main(void *arg) {
    wpool_t *P = (wpool_t *)arg;
    for (;;) {
        pthread_mutex_lock(&P->mu);
        while (!P->stop && P->qh == P->qt) pthread_cond_wait(&P->cv_work, &P->mu);
        if (P->qh == P->qt) { pthread_mutex_unlock(&P->mu); return NULL; }   /* stop, queue drained */
        wjob_t *j = &P->jobs[P->queue[P->qh % P->nj]];
        P->qh++;
        j->state = 2;
        pthread_mutex_unlock(&P->mu);
        job_run(P, j);
        pthread_mutex_lock(&P->mu);
        j->state = 3;
        pthread_cond_broadcast(&P->cv_done);
        pthread_mutex_unlock(&P->mu);
    }
}

static void pool_submit(wpool_t *P, int k) {
    pthread_mutex_lock(&P->mu);
    P->jobs[k].state = 1;
    P->queue[P->qt % P->nj] = k;
    P->qt++;
    pthread_cond_signal(&P->cv_work);
    pthread_mutex_unlock(&P->mu);
}

static void pool_wait(wpool_t *P, int k) {
    pthread_mutex_lock(&P->mu);
    while (P->jobs[k].state != 3) pthread_cond_wait(&P->cv_done, &P->mu);
    pthread_mutex_unlock(&P->mu);
}

/* job state is shared with the writer threads: read and reset it under the pool lock only */
static int job_busy(wpool_t *P, int k) {
    pthread_mutex_lock(&P->mu);
    const int st = P->jobs[k].state;
    pthread_mutex_unlock(&P->mu);
    return st != 0;
}
static void job_release(wpool_t *P, int k) {
    pthread_mutex_lock(&P->mu);
    P->jobs[k].state = 0;
    pthread_mutex_unlock(&P->mu);
}

int jm_encode_sequence(const jm_input *inp, jm_backend *be, jm_stats *st, FILE *log) {
    memset(st, 0, sizeof(*st));
    jmh_config cfg;
    jm_fill_config(inp, &cfg);
    int W = cfg.width, H = cfg.height;
    jm_seq s;
    memset(&s, 0, sizeof(s));
    s.width = W; s.height = H; s.disp_w = inp->width; s.disp_h = inp->height;
    s.mbw = W / 16; s.mbh = H / 16;
    s.profile_idc = inp->profile_idc; s.level_idc = inp->level_idc;
    s.num_ref_frames = inp->num_ref_frames;
    s.log2_max_frame_num = 8; s.log2_max_poc_lsb = 8;
    s.chroma_qp_offset = inp->chroma_qp_offset;
    s.lf_params_flag = inp->lf_params_flag; s.lf_disable = inp->lf_disable;
    s.slice_mbs = inp->slice_mode == 1 ? inp->slice_arg : 0;
    s.lf_alpha = inp->lf_alpha; s.lf_beta = inp->lf_beta;
    s.constrained_intra = inp->constrained_intra;
    s.transform_8x8_mode = inp->transform_8x8_mode;
    s.entropy_coding = inp->symbol_mode;
    s.bit_depth = inp->bit_depth_luma;
    const int bd = inp->bit_depth_luma;
    s.cabac_init_idc = inp->model_number;
    s.rdo = inp->rdopt;

    FILE *fin = NULL, *fout = NULL, *frec = NULL;
    uint64_t seed = 0;
    int synthetic = !strncmp(inp->infile, "synthetic:", 10);
    if (synthetic) seed = strtoull(inp->infile + 10, NULL, 10);
    else if (!(fin = fopen(inp->infile, "rb"))) { fprintf(stderr, "Input file %s does not exist\n", inp->infile); return JMH_E_INVALID_ARG; }
    if (!(fout = fopen(inp->outfile, "wb"))) { fprintf(stderr, "Cannot open output file %s\n", inp->outfile); if (fin) fclose(fin); return JMH_E_INVALID_ARG; }
    if (inp->reconfile[0] && !(frec = fopen(inp->reconfile, "wb"))) { fprintf(stderr, "Cannot open recon file %s\n", inp->reconfile); fclose(fout); if (fin) fclose(fin); return JMH_E_INVALID_ARG; }

    /* pictures waiting for their results: depth > 1 when the backend pipelines (jmh_frame_push /
       jmh_frame_pop, lencod.c); their sources stay here for the PSNR */
    const int dev_dbk = be->read_deblocked && be->reference_deblocked;
    const int pipelined = dev_dbk && be->push && be->pop && be->depth > 1;
    const int depth = pipelined ? be->depth : 1;
    /* parallel slice writing: pipelined device backend, not with the call surface's per-MB
       device searches (those share the context with the frame loop) */
    const int nwr = (pipelined && !inp->jm_call_surface) ? inp->writer_threads : 0;
    const int nj = nwr ? 2 * nwr : 0;                  /* jobs in flight: queued + running + done */
    const int plen = depth + nj + 1;                   /* source slots: a job's source stays put */
    typedef struct { jm_pic cur; jmh_frame_params fp; int f, is_i, frame_num; } pend_t;
    pend_t *pend = (pend_t *)calloc(plen, sizeof(pend_t));
    jm_pic rec;
    memset(&rec, 0, sizeof(rec));
    int alloc_fail = !pend || jm_pic_alloc_bd(&rec, W, H, bd);
    for (int k = 0; k < plen && !alloc_fail; k++) alloc_fail = jm_pic_alloc_bd(&pend[k].cur, W, H, bd);
    if (alloc_fail) {
        if (pend) for (int k = 0; k < plen; k++) jm_pic_free(&pend[k].cur);
        free(pend);
        jm_pic_free(&rec);
        if (fin) fclose(fin);
        fclose(fout);
        if (frec) fclose(frec);
        return JMH_E_OOM;
    }
    int nmb = s.mbw * s.mbh;
    const jmh_mb_result **res = (const jmh_mb_result **)malloc(sizeof(*res) * nmb);
    jm86_img im;
    memset(&im, 0, sizeof(im));
    wpool_t pool;
    memset(&pool, 0, sizeof(pool));
    int st_ret = 0, njobs_init = 0, nstarted = 0, pool_sync = 0;
    long jseq = 0, jflushed = 0;   /* jobs submitted / emitted (picture order) */
    double copy_ms = 0, write_ms = 0;
    double read_ms = 0, push_ms = 0, pop_ms = 0, flush_ms = 0;   /* main thread, for the summary */
    jm_bits out, rbsp;
    jm_bits_init(&out); jm_bits_init(&rbsp);
    if (!res || jm86_init(&im, inp, be, W, H)) { st_ret = JMH_E_OOM; goto cleanup; }
    if (nwr) {
        pool.nj = nj; pool.s = &s; pool.inp = inp; pool.nth = nwr;
        pool.jobs = (wjob_t *)calloc(nj, sizeof(wjob_t));
        pool.queue = (int *)calloc(nj, sizeof(int));
        pool.th = (pthread_t *)calloc(nwr, sizeof(pthread_t));
        if (!pool.jobs || !pool.queue || !pool.th) { st_ret = JMH_E_OOM; goto cleanup; }
        for (; njobs_init < nj; njobs_init++) {
            wjob_t *j = &pool.jobs[njobs_init];
            jm_bits_init(&j->out);
            if (jm86_init(&j->im, inp, be, W, H) || jm_pic_alloc_bd(&j->rec, W, H, bd)) { njobs_init++; st_ret = JMH_E_OOM; goto cleanup; }
            j->im.res = j->im.mb_data;   /* results copied in at pop */
        }
        img = &im;   /* jm86_init of the jobs set this thread's img */
        pthread_mutex_init(&pool.mu, NULL);
        pthread_cond_init(&pool.cv_work, NULL);
        pthread_cond_init(&pool.cv_done, NULL);
        pool_sync = 1;
        for (; nstarted < nwr; nstarted++)
            if (pthread_create(&pool.th[nstarted], NULL, writer_main, &pool)) { st_ret = JMH_E_OOM; goto cleanup; }
    }
    jm_write_sps(&rbsp, &s); jm_write_nal(&out, 3, 7, &rbsp); jm_bits_free(&rbsp);
    jm_write_pps(&rbsp, &s); jm_write_nal(&out, 3, 8, &rbsp); jm_bits_free(&rbsp);
    long header_bits = out.len * 8;
    fwrite(out.buf, 1, out.len, fout);
    st->bits += header_bits;
    out.len = 0;
    if (log) {
        fprintf(log, "------------------------------- MI355X jm-hot-path lencod (%s) -------------------------------\n", be->name);
        if (pipelined) fprintf(log, " (%d pictures in flight%s)\n", depth, nwr ? ", parallel slice writing" : "");
        if (nwr) fprintf(log, " (%d slice-writer threads)\n", nwr);
        fprintf(log, " Frame  Bit/pic  QP   SnrY    SnrU    SnrV    Time(ms) MET(ms) Frm/Fld  I D\n");
    }
    double t_start = now_ms();
    int frame_num = 0, head = 0, count = 0;
    /* the rest of encode_one_frame for a picture whose macroblock results are available:
       slice (CAVLC), deblocking / next reference, recon file, PSNR, report line */
    /* emit a finished job: NAL unit, recon, statistics, report line (picture order) */
    #define FLUSH_JOB(J)                                                                           \
    do {                                                                                           \
        wjob_t *fj_ = (J);                                                                          \
        double tf_ = now_ms();                                                                      \
        pool_wait(&pool, (int)(fj_ - pool.jobs));                                                   \
        if (fj_->status) { st_ret = fj_->status; break; }                                           \
        fwrite(fj_->out.buf, 1, fj_->out.len, fout);                                                 \
        if (frec) jm_write_yuv_frame(frec, &fj_->rec, inp->width, inp->height);                     \
        st->psnr_y += fj_->py; st->psnr_u += fj_->pu; st->psnr_v += fj_->pv;                          \
        st->bits += fj_->pic_bits;                                                                  \
        im.rate_checked += fj_->im.rate_checked; im.rate_mismatches += fj_->im.rate_mismatches;     \
        fj_->im.rate_checked = fj_->im.rate_mismatches = 0;                                         \
        st->frames++;                                                                              \
        st->entropy_ms += fj_->write_ms;                                                            \
        write_ms += fj_->write_ms;                                                                  \
        if (log)                                                                                   \
            fprintf(log, "%4d(%s) %8ld   %2d %7.4f %7.4f %7.4f %9.1f %7.1f    FRM\n", fj_->f,          \
                    fj_->is_i ? "IDR" : " P ", fj_->pic_bits, fj_->fp.qp, fj_->py, fj_->pu, fj_->pv,       \
                    fj_->write_ms + fj_->met, fj_->met);                                              \
        job_release(&pool, (int)(fj_ - pool.jobs));                                                 \
        jflushed++;                                                                                \
        flush_ms += now_ms() - tf_;                                                                 \
    } while (0)
    /* hand a popped picture to the writer pool: its results and deblocked picture into a job */
    #define SUBMIT(P, MET_MS)                                                                      \
    do {                                                                                           \
        pend_t *p_ = (P);                                                                          \
        wjob_t *j_ = &pool.jobs[jseq % nj];                                                       \
        if (job_busy(&pool, (int)(j_ - pool.jobs))) { FLUSH_JOB(j_); if (st_ret) break; }          \
        double t1 = now_ms();                                                                      \
        const jmh_mb_result *r0_ = be->mb_result(be->ctx, 0);                                      \
        if (nmb > 1 && be->mb_result(be->ctx, nmb - 1) != r0_ + (nmb - 1)) { st_ret = JMH_E_STATE; break; } \
        memcpy(j_->im.mb_data, r0_, (size_t)nmb * sizeof(jmh_mb_result));                         \
        int r_ = be->read_deblocked(be->ctx, &j_->rec);                                            \
        if (r_) { fprintf(stderr, "read_deblocked failed: %d\n", r_); st_ret = r_; break; }       \
        copy_ms += now_ms() - t1;                                                                  \
        st->deblock_ms += now_ms() - t1;                                                           \
        j_->cur = &p_->cur; j_->fp = p_->fp; j_->f = p_->f; j_->is_i = p_->is_i; j_->met = (MET_MS); \
        j_->sl.idr = p_->f == 0; j_->sl.slice_type = p_->fp.slice_type; j_->sl.frame_num = p_->frame_num; \
        j_->sl.poc_lsb = 2 * p_->f; j_->sl.idr_pic_id = 0; j_->sl.qp = p_->fp.qp; j_->sl.first_mb = 0; \
        pool_submit(&pool, (int)(j_ - pool.jobs));                                                 \
        jseq++;                                                                                    \
    } while (0)
    #define EMIT(P, MET_MS)                                                                          \
    do {                                                                                           \
        if (nwr) { SUBMIT(P, MET_MS); break; }                                                     \
        pend_t *p_ = (P);                                                                          \
        double t1 = now_ms();                                                                      \
        for (int a = 0; a < nmb; a++) res[a] = be->mb_result(be->ctx, a);                          \
        jm_slice sl;                                                                               \
        sl.idr = p_->f == 0; sl.slice_type = p_->fp.slice_type; sl.frame_num = p_->frame_num;      \
        sl.poc_lsb = 2 * p_->f; sl.idr_pic_id = 0; sl.qp = p_->fp.qp;                              \
        sl.first_mb = 0;                                                                           \
        { int e_ = encode_picture_slices(&im, &s, &sl, &p_->fp, &p_->cur, &rec, &out); if (e_) { st_ret = e_; break; } } \
        double t2 = now_ms();                                                                      \
        st->entropy_ms += t2 - t1;                                                                 \
        long pic_bits = out.len * 8;                                                               \
        fwrite(out.buf, 1, out.len, fout);                                                         \
        out.len = 0;                                                                               \
        int r_;                                                                                    \
        if (dev_dbk) r_ = be->read_deblocked(be->ctx, &rec);                                       \
        else {                                                                                     \
            be->read_recon(be->ctx, &rec);                                                         \
            jm_deblock_picture(&rec, &s, res, p_->fp.qp);                                          \
            r_ = be->set_reference(be->ctx, &rec);                                                 \
        }                                                                                          \
        double t3 = now_ms();                                                                      \
        st->deblock_ms += t3 - t2;                                                                 \
        if (r_) { fprintf(stderr, "set_reference failed: %d\n", r_); st_ret = r_; break; }         \
        if (frec) jm_write_yuv_frame(frec, &rec, inp->width, inp->height);                         \
        double py = psnr_pl(&p_->cur, &rec, 0, inp->width, inp->height);                           \
        double pu = psnr_pl(&p_->cur, &rec, 1, inp->width / 2, inp->height / 2);                   \
        double pv = psnr_pl(&p_->cur, &rec, 2, inp->width / 2, inp->height / 2);                   \
        st->psnr_y += py; st->psnr_u += pu; st->psnr_v += pv;                                      \
        st->bits += pic_bits;                                                                      \
        st->frames++;                                                                              \
        if (log)                                                                                   \
            fprintf(log, "%4d(%s) %8ld   %2d %7.4f %7.4f %7.4f %9.1f %7.1f    FRM\n", p_->f,          \
                    p_->is_i ? "IDR" : " P ", pic_bits, p_->fp.qp, py, pu, pv, t3 - t1 + (MET_MS), (MET_MS)); \
    } while (0)
    for (int f = 0; f < inp->frames && !st_ret; f++) {
        if (pipelined && count == depth) {   /* the oldest picture's results */
            double t0 = now_ms();
            int r = be->pop(be->ctx);
            double met = now_ms() - t0;
            if (r) { fprintf(stderr, "hot path backend '%s' failed: status %d\n", be->name, r); st_ret = r; break; }
            st->me_tq_ms += met;
            pop_ms += met;
            EMIT(&pend[head], met);
            if (st_ret) break;
            head = (head + 1) % plen;
            count--;
        }
        pend_t *p = &pend[(head + count) % plen];
        int idx = inp->start_frame + f;
        double tr = now_ms();
        if (synthetic) jm_synth_frame(&p->cur, inp->width, inp->height, seed, idx);
        else if (jm_read_yuv_frame(fin, &p->cur, inp->width, inp->height, idx)) { fprintf(stderr, "ReadOneFrame: cannot read frame %d\n", idx); st_ret = JMH_E_INVALID_ARG; break; }
        read_ms += now_ms() - tr;
        p->f = f;
        p->is_i = f == 0 || (inp->intra_period && f % inp->intra_period == 0);
        p->frame_num = frame_num++;
        jmh_frame_params *fp = &p->fp;
        memset(fp, 0, sizeof(*fp));
        fp->slice_type = p->is_i ? JMH_I_SLICE : JMH_P_SLICE;
        fp->qp = p->is_i ? inp->qp_i : inp->qp_p;
        fp->lambda_mode = fp->lambda_motion = jm_lambda_rdo_off(fp->qp);
        if (inp->rdopt) fp->lambda_rd = jm_lambda_rdo_on(fp->qp, inp->bit_depth_luma, &fp->lambda_factor_rd);
        fp->chroma_qp_offset = inp->chroma_qp_offset;
        if (dev_dbk) {   /* same parameters jm_deblock_picture derives from the slice header */
            fp->deblock = 1;
            fp->lf_disable = s.lf_params_flag ? s.lf_disable : 0;
            fp->lf_alpha_div2 = s.lf_params_flag ? s.lf_alpha : 0;
            fp->lf_beta_div2 = s.lf_params_flag ? s.lf_beta : 0;
        }
        double t0 = now_ms();
        int r = 0;
        if (dev_dbk && !p->is_i) r = be->reference_deblocked(be->ctx);   /* previous picture, on the device */
        if (!r) r = pipelined ? be->push(be->ctx, &p->cur, fp) : be->encode_frame(be->ctx, &p->cur, fp);
        double met = now_ms() - t0;
        if (r) { fprintf(stderr, "hot path backend '%s' failed: status %d\n", be->name, r); st_ret = r; break; }
        st->me_tq_ms += met;
        push_ms += met;
        if (pipelined) count++;
        else EMIT(p, met);
    }
    while (pipelined && count && !st_ret) {
        double t0 = now_ms();
        int r = be->pop(be->ctx);
        double met = now_ms() - t0;
        if (r) { fprintf(stderr, "hot path backend '%s' failed: status %d\n", be->name, r); st_ret = r; break; }
        st->me_tq_ms += met;
        EMIT(&pend[head], met);
        head = (head + 1) % plen;
        count--;
    }
    while (nwr && jflushed < jseq && !st_ret) FLUSH_JOB(&pool.jobs[jflushed % nj]);
    #undef EMIT
    #undef SUBMIT
    #undef FLUSH_JOB
    st->total_ms = now_ms() - t_start;
cleanup:
    /* one teardown for every exit: stop and join the writer threads that started, free what
       was allocated (also after a partial setup) */
    if (nstarted) {
        pthread_mutex_lock(&pool.mu);
        pool.stop = 1;
        pthread_cond_broadcast(&pool.cv_work);
        pthread_mutex_unlock(&pool.mu);
        for (int k = 0; k < nstarted; k++) pthread_join(pool.th[k], NULL);
    }
    for (int k = 0; k < njobs_init; k++) { jm86_free(&pool.jobs[k].im); jm_pic_free(&pool.jobs[k].rec); jm_bits_free(&pool.jobs[k].out); }
    if (pool_sync) {
        pthread_mutex_destroy(&pool.mu);
        pthread_cond_destroy(&pool.cv_work);
        pthread_cond_destroy(&pool.cv_done);
    }
    free(pool.jobs); free(pool.queue); free(pool.th);
    img = &im;
    st->surface_checked = im.surface_checked;
    st->surface_searches = im.surface_searches;
    st->surface_mismatches = im.surface_mismatches;
    if (log && inp->jm_call_surface)
        fprintf(log, " JM call surface: %d P macroblocks through PartitionMotionSearch / BlockMotionSearch (%d backend "
                     "searches), %d inconsistent with the wavefront decision\n",
                im.surface_checked, im.surface_searches, im.surface_mismatches);
    if (!st_ret && im.surface_mismatches) st_ret = JMH_E_STATE;
    st->rate_checked = im.rate_checked;
    st->rate_mismatches = im.rate_mismatches;
    if (log && inp->rdopt)
        fprintf(log, " RD rate check: %ld macroblocks, %ld whose RD rate differs from the bits written (CABAC or CAVLC)\n",
                im.rate_checked, im.rate_mismatches);
    if (!st_ret && im.rate_mismatches) st_ret = JMH_E_STATE;
    jm86_free(&im);
    if (st->frames) { st->psnr_y /= st->frames; st->psnr_u /= st->frames; st->psnr_v /= st->frames; }
    if (log && st->frames)
        fprintf(log, " Total encoding time for the seq.  : %.3f sec\n Total ME+TQ time (backend)        : %.3f sec\n"
                     " SNR Y(dB) %.4f U %.4f V %.4f   bits %ld\n",
                st->total_ms / 1e3, st->me_tq_ms / 1e3, st->psnr_y, st->psnr_u, st->psnr_v, st->bits);
    if (log && st->frames)
        fprintf(log, " Host per picture: slice writing + PSNR %.2f ms (%s), results + readback (+ host deblocking) %.2f ms, wall %.2f ms\n",
                st->entropy_ms / st->frames, nwr ? "writer threads" : "main thread", st->deblock_ms / st->frames,
                st->total_ms / st->frames);
    if (log && st->frames)
        fprintf(log, " Main thread per picture: read %.2f ms, push %.2f, pop (wait) %.2f, results to writer %.2f, flush %.2f\n",
                read_ms / st->frames, push_ms / st->frames, pop_ms / st->frames, copy_ms / st->frames, flush_ms / st->frames);
    jm_bits_free(&out);
    free(res);
    for (int k = 0; k < plen; k++) jm_pic_free(&pend[k].cur);
    free(pend);
    jm_pic_free(&rec);
    if (fin) fclose(fin);
    fclose(fout);
    if (frec) fclose(frec);
    return st_ret;
}
