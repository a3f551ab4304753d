/*
 * encoder.c — sequence / picture driver, restating JM 8.6 lencod.c › main frame loop and
 * image.c › encode_one_frame [J]: read (or synthesise) the picture, choose I/P, run the
 * macroblock hot path through the backend (encode_one_macroblock for every MB), write the
 * slice (CAVLC), deblock the reconstruction, make it the reference (UnifiedOneForthPix runs in
 * the backend), write the recon, print JM's per-frame report line.
 */
#include <math.h>
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

static double psnr(const uint8_t *a, int sa, const uint8_t *b, int sb, int w, int h) {
    double se = 0;
    for (int y = 0; y < h; y++)
        for (int x = 0; x < w; x++) {
            int d = a[y * sa + x] - b[y * sb + x];
            se += d * d;
        }
    if (se == 0) return 99.0;
    return 10.0 * log10(255.0 * 255.0 * w * h / se);
}

/* slice.c › encode_one_slice [J]: the macroblock loop of one picture (one slice) through the JM
 * 8.6 call surface (host/jm86.c): start_macroblock, encode_one_macroblock, write_one_macroblock */
static int encode_one_slice(jm86_img *im, const jm_seq *s, const jm_slice *sl, const jmh_frame_params *fp, const jm_pic *cur,
                            const jm_pic *ref, jm_bits *rbsp) {
    jm_slice_writer *w = jm_slice_begin(rbsp, s, sl);
    if (!w) return JMH_E_OOM;
    int r = jm86_start_picture(im, fp, cur, ref, w);
    if (r) { jm_slice_end(w); return r; }
    for (int a = 0; a < s->mbw * s->mbh; a++) {
        img->current_mb_nr = a;
        start_macroblock();
        encode_one_macroblock();
        write_one_macroblock();
    }
    jm_slice_end(w);
    return JMH_OK;
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
    s.lf_alpha = inp->lf_alpha; s.lf_beta = inp->lf_beta;
    s.constrained_intra = inp->constrained_intra;
    s.transform_8x8_mode = inp->transform_8x8_mode;

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
    typedef struct { jm_pic cur; jmh_frame_params fp; int f, is_i, frame_num; } pend_t;
    pend_t *pend = (pend_t *)calloc(depth, sizeof(pend_t));
    jm_pic rec;
    int alloc_fail = !pend || jm_pic_alloc(&rec, W, H);
    for (int k = 0; k < depth && !alloc_fail; k++) alloc_fail = jm_pic_alloc(&pend[k].cur, W, H);
    if (alloc_fail) return JMH_E_OOM;
    int nmb = s.mbw * s.mbh;
    const jmh_mb_result **res = (const jmh_mb_result **)malloc(sizeof(*res) * nmb);
    jm86_img im;
    if (!res || jm86_init(&im, inp, be, W, H)) return JMH_E_OOM;
    jm_bits out, rbsp;
    jm_bits_init(&out); jm_bits_init(&rbsp);
    jm_write_sps(&rbsp, &s); jm_write_nal(&out, 3, 7, &rbsp); jm_bits_free(&rbsp);
    jm_write_pps(&rbsp, &s); jm_write_nal(&out, 3, 8, &rbsp); jm_bits_free(&rbsp);
    long header_bits = out.len * 8;
    fwrite(out.buf, 1, out.len, fout);
    st->bits += header_bits;
    out.len = 0;
    if (log) {
        fprintf(log, "------------------------------- MI355X jm-hot-path lencod (%s) -------------------------------\n", be->name);
        if (pipelined) fprintf(log, " (%d pictures in flight)\n", depth);
        fprintf(log, " Frame  Bit/pic  QP   SnrY    SnrU    SnrV    Time(ms) MET(ms) Frm/Fld  I D\n");
    }
    double t_start = now_ms();
    int st_ret = 0, frame_num = 0, head = 0, count = 0;
    /* the rest of encode_one_frame for a picture whose macroblock results are available:
       slice (CAVLC), deblocking / next reference, recon file, PSNR, report line */
    #define EMIT(P, MET_MS)                                                                          \
    do {                                                                                           \
        pend_t *p_ = (P);                                                                          \
        double t1 = now_ms();                                                                      \
        for (int a = 0; a < nmb; a++) res[a] = be->mb_result(be->ctx, a);                          \
        jm_slice sl;                                                                               \
        sl.idr = p_->f == 0; sl.slice_type = p_->fp.slice_type; sl.frame_num = p_->frame_num;      \
        sl.poc_lsb = 2 * p_->f; sl.idr_pic_id = 0; sl.qp = p_->fp.qp;                              \
        jm_bits_init(&rbsp);                                                                       \
        if (encode_one_slice(&im, &s, &sl, &p_->fp, &p_->cur, &rec, &rbsp)) { st_ret = JMH_E_OOM; break; } \
        jm_write_nal(&out, sl.idr ? 3 : 2, sl.idr ? 5 : 1, &rbsp);                                 \
        jm_bits_free(&rbsp);                                                                       \
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
        double py = psnr(p_->cur.y, W, rec.y, W, inp->width, inp->height);                         \
        double pu = psnr(p_->cur.u, W / 2, rec.u, W / 2, inp->width / 2, inp->height / 2);         \
        double pv = psnr(p_->cur.v, W / 2, rec.v, W / 2, inp->width / 2, inp->height / 2);         \
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
            EMIT(&pend[head], met);
            if (st_ret) break;
            head = (head + 1) % depth;
            count--;
        }
        pend_t *p = &pend[(head + count) % depth];
        int idx = inp->start_frame + f;
        if (synthetic) jm_synth_frame(&p->cur, inp->width, inp->height, seed, idx);
        else if (jm_read_yuv_frame(fin, &p->cur, inp->width, inp->height, idx)) { fprintf(stderr, "ReadOneFrame: cannot read frame %d\n", idx); st_ret = JMH_E_INVALID_ARG; break; }
        p->f = f;
        p->is_i = f == 0 || (inp->intra_period && f % inp->intra_period == 0);
        p->frame_num = frame_num++;
        jmh_frame_params *fp = &p->fp;
        memset(fp, 0, sizeof(*fp));
        fp->slice_type = p->is_i ? JMH_I_SLICE : JMH_P_SLICE;
        fp->qp = p->is_i ? inp->qp_i : inp->qp_p;
        fp->lambda_mode = fp->lambda_motion = jm_lambda_rdo_off(fp->qp);
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
        head = (head + 1) % depth;
        count--;
    }
    #undef EMIT
    st->total_ms = now_ms() - t_start;
    st->surface_checked = im.surface_checked;
    st->surface_searches = im.surface_searches;
    st->surface_mismatches = im.surface_mismatches;
    if (log && inp->jm_call_surface)
        fprintf(log, " JM call surface: %d P macroblocks through PartitionMotionSearch / BlockMotionSearch (%d backend "
                     "searches), %d inconsistent with the wavefront decision\n",
                im.surface_checked, im.surface_searches, im.surface_mismatches);
    if (!st_ret && im.surface_mismatches) st_ret = JMH_E_STATE;
    jm86_free(&im);
    if (st->frames) { st->psnr_y /= st->frames; st->psnr_u /= st->frames; st->psnr_v /= st->frames; }
    if (log && st->frames)
        fprintf(log, " Total encoding time for the seq.  : %.3f sec\n Total ME+TQ time (backend)        : %.3f sec\n"
                     " SNR Y(dB) %.4f U %.4f V %.4f   bits %ld\n",
                st->total_ms / 1e3, st->me_tq_ms / 1e3, st->psnr_y, st->psnr_u, st->psnr_v, st->bits);
    jm_bits_free(&out);
    free(res);
    for (int k = 0; k < depth; k++) jm_pic_free(&pend[k].cur);
    free(pend);
    jm_pic_free(&rec);
    if (fin) fclose(fin);
    fclose(fout);
    if (frec) fclose(frec);
    return st_ret;
}
