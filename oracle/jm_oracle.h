/*
 * jm_oracle.h — CPU restatement of the JM lencod hot path (TEST INFRASTRUCTURE ONLY).
 *
 * This directory is the oracle: plain C, written from the ITU-T H.264 normative clauses and
 * from JM 8.6 lencod's non-normative encoder semantics (docs/JM_SEMANTICS.md).  It is used
 * only by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg, as the checker and
 * the CPU baseline.  The product (h264-jm-commentary_amd/) never links or calls it.
 *
 * PARITY STATUS: the mounted reference holds only README.md:1-4 (no JM source, no tests, no
 * fixtures, no binary), so parity of this restatement with JM's own output is UNPINNED.
 * What IS pinned: (1) the normative parts by spec known-answer tests and by the independent
 * closed-loop decoder in oracle/decoder.c (decoder output == encoder recon, byte for byte);
 * (2) the GPU path by bit-exact equality with this oracle.  Every JM function restated here is
 * cited as "JM 8.6 <file> › <function> [J]"; no file:line exists.
 */
#ifndef JM_ORACLE_H
#define JM_ORACLE_H

#include <stdint.h>
#include "../include/jmhip.h"

#ifdef __cplusplus
extern "C" {
#endif

#define JMO_PAD 4            /* qpel-plane padding (JM IMG_PAD_SIZE [J]); >= 3 makes UMV
                                clamping identical to the spec's coordinate clamping       */
#define JMO_MAX_SR 64

typedef struct jmo_ctx jmo_ctx;

/* ---- backend API (mirrors jmh_*) ----------------------------------------------------- */
int  jmo_create(const jmh_config *cfg, jmo_ctx **out);
void jmo_destroy(jmo_ctx *c);
int  jmo_set_reference(jmo_ctx *c, const uint8_t *y, const uint8_t *u, const uint8_t *v,
                       int stride_y, int stride_c);
int  jmo_encode_frame(jmo_ctx *c, const uint8_t *y, const uint8_t *u, const uint8_t *v,
                      int stride_y, int stride_c, const jmh_frame_params *fp);
const jmh_mb_result *jmo_mb_result(const jmo_ctx *c, int mb_addr);
/* High 10 pictures (cfg.bit_depth 9 / 10): 16-bit samples; the uint8_t entry points serve bit depth 8 */
int  jmo_set_reference_u16(jmo_ctx *c, const uint16_t *y, const uint16_t *u, const uint16_t *v, int stride_y,
                           int stride_c);
int  jmo_encode_frame_u16(jmo_ctx *c, const uint16_t *y, const uint16_t *u, const uint16_t *v, int stride_y,
                          int stride_c, const jmh_frame_params *fp);
int  jmo_read_recon_u16(const jmo_ctx *c, uint16_t *y, uint16_t *u, uint16_t *v, int stride_y, int stride_c);
int  jmo_read_recon(const jmo_ctx *c, uint8_t *y, uint8_t *u, uint8_t *v, int stride_y,
                    int stride_c);
/* copy the 16 quarter-pel phase planes: out[16][(H+2P)][(W+2P)], phase = 4*yfrac + xfrac  */
int  jmo_read_qpel(const jmo_ctx *c, uint8_t *out);
/* load the current picture without encoding (for jmo_ffs_sad_table)                       */
int  jmo_load_current(jmo_ctx *c, const uint8_t *y, const uint8_t *u, const uint8_t *v,
                      int stride_y, int stride_c);

/* ---- unit entry points (known-answer + GPU unit parity) ------------------------------ */
/* per-block BlockMotionSearch seam (the oracle of jmh_block_motion_search); jmo_search_pictures
 * replaces the context's current and reference luma                                        */
int  jmo_search_pictures(jmo_ctx *c, const uint8_t *cur_y, const uint8_t *ref_y, int stride);
int  jmo_block_motion_search(jmo_ctx *c, int n, const jmh_block_search *req, jmh_block_result *res);
int  jmo_ffs_sad_table(jmo_ctx *c, int n_mb, const int32_t *mb_xy, const int32_t *centres,
                       uint16_t *out);
/* TQ seams: `intra` is the rounding selector of jmo_internal.h (0: JM 8.6 P-slice / 6, 1: I-slice
 * / 3, 2 + o: JM >= 10 flat OffsetMatrix entry o at OffsetBits 11), here and in jmo_tq8x8_batch /
 * jmo_hbd_tq*_batch                                                                         */
int  jmo_tq4x4_batch(int n, const int16_t *resid, const uint8_t *pred, int qp, int intra,
                     int16_t *levels, uint8_t *recon, int32_t *coeff_cost, int32_t *nonzero);
/* spec luma sample at quarter-pel position (X,Y) of an integer plane (clamped coords)   */
int  jmo_luma_qpel_sample(const uint8_t *p, int w, int h, int stride, int X, int Y);
void jmo_spiral(int range, int32_t *sx, int32_t *sy);           /* (2R+1)^2 entries       */
int  jmo_mvbits(int v);
int  jmo_satd4x4(const int32_t *diff, int use_hadamard);
void jmo_forward4x4(const int32_t *in, int32_t *out);             /* raster in/out         */
void jmo_inverse4x4(const int32_t *in, int32_t *out);             /* no rounding shift     */
int  jmo_qp2quant(int qp);
/* 8x8 transform unit seams (known answers; GPU unit parity) */
void jmo_forward8x8(const int32_t *in, int32_t *out);             /* raster in/out         */
void jmo_inverse8x8(const int32_t *in, int32_t *out);             /* no rounding shift     */
int  jmo_satd8x8(const int32_t d[64], int use_hadamard);
int  jmo_tq8x8_batch(int n, const int16_t *resid, const uint8_t *pred, int qp, int intra,
                     int16_t *levels, uint8_t *recon, int32_t *coeff_cost, int32_t *nonzero);
/* Intra8x8 prediction (8.3.2.2) of one block from its 25 unfiltered neighbours
 * nb[0] = p[-1,-1], nb[1..16] = p[0..15,-1], nb[17..24] = p[-1,0..7]; avail bits: 1 left,
 * 2 top, 4 top-right, 8 top-left.  pred[9][64]; returns the bitmask of available modes.   */
int  jmo_intra8x8_pred(const int32_t nb[25], int avail, uint8_t pred[9][64]);
int  jmo_qp_scale_cr(int qp);
/* median MV predictor of the spec on explicit neighbours (unit tests)                     */
void jmo_mvp_median(int avail_a, int ref_a, int mva_x, int mva_y,
                    int avail_b, int ref_b, int mvb_x, int mvb_y,
                    int avail_c, int ref_c, int mvc_x, int mvc_y,
                    int ref, int bsx, int bsy, int blk_x, int blk_y, int32_t *pmv);

/* ---- High 10 per-block seams (hbd.c): the oracles of jmh_*_u16 -------------------------- */
typedef struct jmo_hbd jmo_hbd;
int  jmo_hbd_create(int W, int H, int sr, jmo_hbd **out);
void jmo_hbd_destroy(jmo_hbd *h);
int  jmo_hbd_pictures(jmo_hbd *h, const uint16_t *cur, const uint16_t *ref, int stride, int bit_depth);
int  jmo_hbd_qpel(const jmo_hbd *h, int X, int Y);
int  jmo_hbd_block_motion_search(const jmo_hbd *h, int use_hadamard, int n, const jmh_block_search *req,
                                 jmh_block_result *res);
int  jmo_hbd_sad_table(const jmo_hbd *h, int n_mb, const int32_t *mb_xy, const int32_t *centres, uint16_t *out);
int  jmo_hbd_tq4x4_batch(int n, const int16_t *resid, const uint16_t *pred, int qp, int intra, int bit_depth,
                         int16_t *levels, uint16_t *recon, int32_t *coeff_cost, int32_t *nonzero);
int  jmo_hbd_tq8x8_batch(int n, const int16_t *resid, const uint16_t *pred, int qp, int intra, int bit_depth,
                         int16_t *levels, uint16_t *recon, int32_t *coeff_cost, int32_t *nonzero);

/* ---- closed-loop decoder (Baseline CAVLC subset emitted by the host encoder) --------- */
typedef struct jmo_dec jmo_dec;
int  jmo_dec_create(jmo_dec **out);
void jmo_dec_destroy(jmo_dec *d);
/* decode a whole Annex-B stream; frames are appended to out (cropped 4:2:0 I420), returns
 * number of frames decoded or a negative error.  out_cap in bytes.                        */
int  jmo_decode_annexb(jmo_dec *d, const uint8_t *buf, long len, uint8_t *out, long out_cap,
                       int *width, int *height);
const char *jmo_dec_error(const jmo_dec *d);
int jmo_dec_bit_depth(const jmo_dec *d);   /* of the last SPS (0: none yet); output samples are 16-bit LE above 8 */

#ifdef __cplusplus
}
#endif
#endif
