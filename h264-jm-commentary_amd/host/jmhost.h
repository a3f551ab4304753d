/*
 * jmhost.h — lencod-compatible host plumbing around the jmh_* hot path.
 *
 * Mirrors the JM 8.6 lencod structure [J] (no file:line exists: /root/reference holds only
 * README.md:1-4): configfile.c (encoder.cfg, Map[], -d/-f/-p), lencod.c main + frame loop,
 * image.c encode_one_frame, slice.c/header.c/parset.c/nalu.c (slice + parameter sets + NAL),
 * vlc.c + macroblock.c writers (CAVLC), loopfilter.c (deblocking).  The macroblock hot path is
 * a pluggable backend: the product binary binds it to libjmhip.so (MI355X); the test-only CPU
 * reference binary (oracle/lencod_cpu) binds it to the oracle.
 */
#ifndef JMHOST_H
#define JMHOST_H

#include <stdint.h>
#include <stdio.h>
#include "../../include/jmhip.h"

#ifdef __cplusplus
extern "C" {
#endif

/* ---- encoder.cfg (JM 8.6 keys, with JM>=10 spellings accepted as aliases) -------------- */
typedef struct jm_input {
    char infile[512];          /* InputFile ("synthetic:<seed>" = built-in generator)         */
    char outfile[512];         /* OutputFile (.264 Annex B)                                   */
    char reconfile[512];       /* ReconFile ("" = none)                                       */
    int  frames;               /* FramesToBeEncoded                                           */
    int  start_frame;          /* StartFrame                                                  */
    int  width, height;        /* SourceWidth / SourceHeight (displayed size)                 */
    int  intra_period;         /* IntraPeriod (0: only the first picture is intra)           */
    int  qp_i, qp_p;           /* QPFirstFrame (QPISlice) / QPRemainingFrame (QPPSlice)       */
    int  search_range;         /* SearchRange                                                 */
    int  search_mode;          /* SearchMode: -1 full, 0 fast full (UseFME=0 == 0)             */
    int  use_hadamard;         /* UseHadamard                                                 */
    int  num_ref_frames;       /* NumberReferenceFrames                                       */
    int  restrict_search_range;/* RestrictSearchRange                                         */
    int  inter_search[8];      /* InterSearch16x16 .. InterSearch4x4 ([1..7])                 */
    int  rdopt;                /* RDOptimization: 0, or 1 with SymbolMode 1 (CABAC rate)       */
    int  profile_idc;          /* ProfileIDC (66 Baseline, 100 High)                          */
    int  transform_8x8_mode;   /* Transform8x8Mode (0, 1; needs ProfileIDC 100)               */
    int  jm_version;           /* JMVersion: 8 (JM 8.6 rules, default) or >= 10 (JM >= 10
                                  quantisation offsets, docs/JM_SEMANTICS.md item 45)          */
    int  qoff_intra, qoff_inter;/* QOffsetIntra / QOffsetInter: flat OffsetMatrix entries at
                                  OffsetBits 11 (JMVersion >= 10; -1 = JM defaults 682 / 342) */
    int  adaptive_rounding;    /* AdaptiveRounding (must be 0)                                */
    int  epzs_dual;            /* EPZSDualRefinement (0, 1; SearchMode 3)                      */
    int  slice_mode;           /* SliceMode (0: one slice per picture, 1: SliceArgument MBs)   */
    int  slice_arg;            /* SliceArgument (MBs per slice with SliceMode 1)               */
    int  epzs_subpel;          /* EPZSSubPelME (0, 1; SearchMode 3; JM_SEMANTICS item 62)      */
    int  epzs_subpel_thres;    /* EPZSSubPelThresScale (item 62)                               */
    int  epzs_min_thres;       /* EPZSMinThresScale (item 61)                                  */
    int  epzs_max_thres;       /* EPZSMaxThresScale (item 61; 0: the fixed medthres stop)      */
    int  offset_matrix_present;/* OffsetMatrixPresentFlag (must be 0: flat lists only)         */
    int  level_idc;            /* LevelIDC                                                    */
    int  symbol_mode;          /* SymbolMode (0 = CAVLC, 1 = CABAC)                            */
    int  bit_depth_luma;       /* SourceBitDepthLuma (JM >= 10 FRExt): 8, 9, 10                 */
    int  bit_depth_chroma;     /* SourceBitDepthChroma: equal to the luma bit depth            */
    int  context_init_method;  /* ContextInitMethod (0: fixed; 1 adaptive is rejected)          */
    int  model_number;         /* FixedModelNumber: cabac_init_idc of P slices (0)              */
    int  lf_params_flag;       /* LoopFilterParametersFlag                                    */
    int  lf_disable;           /* LoopFilterDisable                                           */
    int  lf_alpha, lf_beta;    /* LoopFilterAlphaC0Offset / LoopFilterBetaOffset              */
    int  chroma_qp_offset;     /* ChromaQPOffset                                              */
    int  constrained_intra;    /* UseConstrainedIntraPred                                     */
    int  frame_rate;           /* FrameRate (report only)                                     */
    int  hip_device;           /* (this build) HIP device index                               */
    int  pipeline_depth;       /* (this build) pictures in flight on the device (0 = auto)   */
    int  writer_threads;       /* (this build) slice-writer threads (0: the frame loop writes;
                                  used with a pipelined device backend)                       */
    int  jm_call_surface;      /* (this build) 1: every P macroblock also runs JM 8.6's inter
                                  searches through PartitionMotionSearch / BlockMotionSearch
                                  (the per-block device seam), checked against the wavefront
                                  decision (host/jm86.c)                                      */
    int  verbose;
} jm_input;

void jm_input_defaults(jm_input *inp);
/* JM Configure(): argv "-d file", "-f file", "-p Key=Value", "-h"; returns 0 or -1 (message
 * printed).  Unknown keys are an error (as in JM ParameterNameToMapIndex). */
int  jm_configure(jm_input *inp, int argc, char **argv, char *err, int errlen);
int  jm_parse_content(jm_input *inp, const char *buf, char *err, int errlen);
int  jm_set_param(jm_input *inp, const char *key, const char *val, char *err, int errlen);
int  jm_patch_input(jm_input *inp, char *err, int errlen);   /* PatchInp() */

/* ---- pictures ---------------------------------------------------------------------------- */
typedef struct jm_pic {
    int w, h;                  /* coded (multiple of 16) */
    uint8_t *y, *u, *v;        /* contiguous planes, stride = w / w/2 (bit depth 8)              */
    int bd;                    /* bit depth: 8 (y, u, v) or 9 / 10 (Y, U, V, 16-bit samples)     */
    uint16_t *Y, *U, *V;       /* High 10 planes (JM >= 10 imgpel = unsigned short [J])          */
} jm_pic;
int  jm_pic_alloc(jm_pic *p, int w, int h);
int  jm_pic_alloc_bd(jm_pic *p, int w, int h, int bd);
void jm_pic_free(jm_pic *p);

/* deterministic synthetic 4:2:0 source: integer-only texture, global
 * quarter-pel motion, moving rectangles, per-frame noise.  Writes the displayed w x h into the
 * coded picture and pads to the coded size by edge replication (JM PaddAutoCropBorders). */
void jm_synth_frame(jm_pic *p, int disp_w, int disp_h, uint64_t seed, int frame);
/* the same picture at bit depth bd (9 / 10) in 16-bit samples: each 8-bit sample v becomes
   v << (bd - 8) plus (bd - 8) low bits of per-sample noise (10-bit texture range 64..943) */
void jm_synth_frame_hbd(uint16_t *y, uint16_t *u, uint16_t *v, int w, int h, int disp_w, int disp_h, uint64_t seed,
                        int frame, int bd);
/* read frame `index` of a planar I420 file (displayed size) into the coded picture */
int  jm_read_yuv_frame(FILE *f, jm_pic *p, int disp_w, int disp_h, int index);
int  jm_write_yuv_frame(FILE *f, const jm_pic *p, int disp_w, int disp_h);
void jm_pad_picture(jm_pic *p, int disp_w, int disp_h);

/* ---- bitstream writer ------------------------------------------------------------------ */
typedef struct jm_bits {
    uint8_t *buf;
    long cap, len;             /* bytes */
    uint64_t acc;
    int nacc;
} jm_bits;
void jm_bits_init(jm_bits *b);
void jm_bits_free(jm_bits *b);
void jm_put(jm_bits *b, uint32_t val, int n);
void jm_put_ue(jm_bits *b, uint32_t v);
void jm_put_se(jm_bits *b, int32_t v);
void jm_trailing_bits(jm_bits *b);
void jm_bits_align_flush(jm_bits *b);
void jm_bits_append(jm_bits *b, const jm_bits *src);   /* whole bytes of src (byte aligned b) */

typedef struct jm_seq {
    int width, height;         /* coded */
    int disp_w, disp_h;
    int mbw, mbh;
    int profile_idc, level_idc;
    int num_ref_frames;
    int log2_max_frame_num, log2_max_poc_lsb;
    int chroma_qp_offset;
    int lf_params_flag, lf_disable, lf_alpha, lf_beta;
    int constrained_intra;
    int transform_8x8_mode;    /* PPS transform_8x8_mode_flag (High profile)                   */
    int slice_mbs;             /* MBs per slice, raster order (SliceMode 1); 0: one slice      */
    int bit_depth;             /* BitDepthLuma = BitDepthChroma (High 10: 9 / 10)              */
    int entropy_coding;        /* PPS entropy_coding_mode_flag: 0 CAVLC, 1 CABAC (SymbolMode)  */
    int cabac_init_idc;        /* cabac_init_idc of P slices (FixedModelNumber)                */
    int rdo;                   /* RDOptimization 1: the writer checks each macroblock's RD rate
                                  (jmh_mb_result.min_cost) against the CABAC bits it writes     */
} jm_seq;

/* NAL unit (Annex B start code + emulation prevention) appended to out */
void jm_write_nal(jm_bits *out, int nal_ref_idc, int nal_type, const jm_bits *rbsp);
void jm_write_sps(jm_bits *rbsp, const jm_seq *s);
void jm_write_pps(jm_bits *rbsp, const jm_seq *s);

typedef struct jm_slice {
    int idr, slice_type, frame_num, poc_lsb, idr_pic_id, qp;
    int first_mb;              /* first_mb_in_slice                                             */
} jm_slice;
/* slice header + CAVLC slice data for a whole picture (one slice); results in raster order */
int  jm_write_slice(jm_bits *rbsp, const jm_seq *s, const jm_slice *sl,
                    const jmh_mb_result *const *res);
/* the same, one macroblock at a time (write_one_macroblock), macroblocks in raster order */
typedef struct jm_slice_writer jm_slice_writer;
jm_slice_writer *jm_slice_begin(jm_bits *rbsp, const jm_seq *s, const jm_slice *sl);
void jm_slice_write_mb(jm_slice_writer *w, int mb_addr, const jmh_mb_result *r);
/* closes the last slice; returns the CABAC bins of the picture's slices (0 with CAVLC) */
long jm_slice_end(jm_slice_writer *w);
/* RDOptimization 1 + CABAC: macroblocks written so far and those whose RD rate differed */
void jm_slice_rate_check(const jm_slice_writer *w, long *checked, long *bad);
/* close the current slice's data in its rbsp and start the next slice (header into rbsp), keeping
   the picture's neighbour buffers (SliceMode 1: one writer per picture, one rbsp per slice) */
void jm_slice_restart(jm_slice_writer *w, jm_bits *rbsp, const jm_slice *sl);

/* ---- deblocking (H.264 8.7), in place on the reconstructed picture ---------------------- */
void jm_deblock_picture(jm_pic *p, const jm_seq *s, const jmh_mb_result *const *res, int qp);

/* ---- hot-path backend ------------------------------------------------------------------ */
typedef struct jm_backend {
    const char *name;
    void *ctx;
    int (*set_reference)(void *ctx, const jm_pic *ref);
    int (*encode_frame)(void *ctx, const jm_pic *cur, const jmh_frame_params *fp); /* sync */
    const jmh_mb_result *(*mb_result)(void *ctx, int mb_addr);
    int (*read_recon)(void *ctx, jm_pic *rec);
    void (*destroy)(void *ctx);
    /* optional (NULL: DeblockFrame runs on the host, jm_deblock_picture): the backend deblocks
       while encoding (jmh_frame_params.deblock), returns the filtered picture and makes it the
       next reference without a host round trip */
    int (*read_deblocked)(void *ctx, jm_pic *rec);
    int (*reference_deblocked)(void *ctx);
    /* optional pipelining (NULL / depth <= 1: one picture at a time): push queues a picture,
       pop waits for the oldest one and makes its results current; up to depth in flight */
    int (*push)(void *ctx, const jm_pic *cur, const jmh_frame_params *fp);
    int (*pop)(void *ctx);
    int depth;
    /* optional per-call seams of the JM 8.6 call surface (host/jm86.c): BlockMotionSearch on
       the luma pictures given to search_pictures, dct_luma on explicit residual blocks */
    int (*search_pictures)(void *ctx, const jm_pic *cur, const jm_pic *ref);
    int (*block_search)(void *ctx, int n, const jmh_block_search *req, jmh_block_result *res);
    int (*tq4x4)(void *ctx, int n, const int16_t *resid, const uint8_t *pred, int qp, int intra,
                 int16_t *levels, uint8_t *recon, int32_t *coeff_cost, int32_t *nonzero);
} jm_backend;

typedef struct jm_stats {
    int frames;
    double me_tq_ms;           /* backend encode_frame wall time (ME + TQ + recon)            */
    double total_ms;
    double entropy_ms, deblock_ms;
    long bits;
    double psnr_y, psnr_u, psnr_v;   /* averages                                              */
    int surface_checked, surface_searches, surface_mismatches;   /* JMCallSurface (jm86.c)      */
    long rate_checked, rate_mismatches;                          /* RDOptimization 1 (writer)   */
} jm_stats;

/* ---- the JM 8.6 call surface (host/jm86.c) ------------------------------------------------
 * JM 8.6 lencod keeps its state in globals (global.h: img, input, enc_picture) and calls, per
 * macroblock of a slice, start_macroblock → encode_one_macroblock → write_one_macroblock
 * (slice.c › encode_one_slice); encode_one_macroblock (rdopt.c) calls PartitionMotionSearch →
 * BlockMotionSearch (mv-search.c) and, through the residual coding, dct_luma (block.c) [J].
 * Those functions exist here with JM 8.6 signatures over the subset of that state the hot path
 * reads and writes (jm86_img):
 *   encode_one_macroblock()  the decision of macroblock img->current_mb_nr: the backend's result
 *                            (the device computed the whole picture's encode_one_macroblock
 *                            calls in one wavefront); with JMCallSurface = 1 a P macroblock
 *                            also runs JM's RDO-off inter searches through
 *                            PartitionMotionSearch / BlockMotionSearch (one device search per
 *                            call) and checks the decision's inter mode, cost and MVs against
 *                            them (jm86_img.surface_mismatches)
 *   PartitionMotionSearch / BlockMotionSearch  one device search per block (jmh_block_motion_
 *                            search), MVP from enc_picture's MVs (SetMotionVectorPredictor)
 *   dct_luma                 the 4x4 TQ + reconstruction of img->m7 / img->mpr (jmh_tq4x4_batch)
 */
typedef struct jm86_img {
    int current_mb_nr, mb_x, mb_y, pix_x, pix_y;
    int width, height, mbw, mbh;
    int type;                         /* slice type of the picture (JMH_P_SLICE / JMH_I_SLICE) */
    int qp, lambda_mode, lambda_motion;
    jmh_mb_result *mb_data;           /* img->mb_data (+ cofAC / cofDC / mv) per macroblock     */
    int16_t all_mv[8][16][2];         /* img->all_mv[.][.][LIST_0][ref 0][blocktype] (this MB)  */
    int motion_cost[8][4];            /* motion_cost[blocktype][LIST_0][ref 0][block]           */
    int search_centre[2];             /* SetupFastFullPelSearch's window centre (this MB)      */
    int setup_done;
    int m7[16][16];                   /* img->m7: residual of the block dct_luma codes          */
    uint8_t mpr[16][16];              /* img->mpr: its prediction                               */
    int16_t *enc_mv;                  /* enc_picture->mv[LIST_0], per 4x4 of the picture [2]    */
    int8_t *enc_ref;                  /*   and ->ref_idx (-1: intra / not coded yet)            */
    uint8_t *enc_imgY;                /* enc_picture->imgY (dct_luma's reconstruction)          */
    int surface_searches;             /* BlockMotionSearch calls made (statistics)              */
    int surface_checked, surface_mismatches;   /* P MBs checked / found inconsistent            */
    long rate_checked, rate_mismatches;        /* RDOptimization 1: MB rates checked by the writer */
    const jm_input *input;
    jm_backend *be;
    jm_slice_writer *writer;
    int slice_first;                  /* first MB of the current slice (neighbour availability) */
    const jmh_mb_result *res;         /* the picture's results (NULL: the backend's current ones) */
} jm86_img;
extern __thread jm86_img *img;       /* JM's global img, one per slice-writing thread */

int  jm86_init(jm86_img *im, const jm_input *inp, jm_backend *be, int width, int height);
void jm86_free(jm86_img *im);
/* start a picture: its slice type, QP, lambdas; with the call surface on, the luma pictures
   of the per-block searches (cur, and ref for a P picture) */
int  jm86_start_picture(jm86_img *im, const jmh_frame_params *fp, const jm_pic *cur, const jm_pic *ref,
                        jm_slice_writer *writer);
void start_macroblock(void);
void encode_one_macroblock(void);
void write_one_macroblock(void);
int  BlockMotionSearch(int ref, int list, int mb_x, int mb_y, int blocktype, int search_range, double lambda);
void PartitionMotionSearch(int blocktype, int block8x8, double lambda);
int  dct_luma(int block_x, int block_y, int *coeff_cost, int old_intra_mode);

void jm_fill_config(const jm_input *inp, jmh_config *cfg);
int  jm_lambda_rdo_off(int qp);    /* QP2QUANT[max(0,qp-12)] */
double jm_lambda_rdo_on(int qp, int bit_depth, int *lambda_factor);   /* 0.85*2^((qp+QpBdOffsetY-12)/3) */
/* encode the whole sequence: returns 0 or a negative status */
int  jm_encode_sequence(const jm_input *inp, jm_backend *be, jm_stats *st, FILE *log);

#ifdef __cplusplus
}
#endif
#endif
