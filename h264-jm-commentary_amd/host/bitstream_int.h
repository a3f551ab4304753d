/*
 * bitstream_int.h — state shared by the slice writer's two entropy coders (bitstream.c: CAVLC,
 * cabac.c: CABAC): the picture's neighbour buffers and the normative MVP / MPM derivations
 * both coders code against.  Internal to the host library.
 */
#ifndef JM_BITSTREAM_INT_H
#define JM_BITSTREAM_INT_H

#include "jmhost.h"

typedef struct {
    const jm_seq *s;
    int16_t *mv;        /* per 4x4 [2] of the picture, final values (written MBs) */
    int8_t *ref;        /* per 4x4, -1 intra / not yet written                      */
    int8_t *ipm;        /* per 4x4 Intra4x4PredMode, -1: MB not I4x4               */
    uint32_t *written;  /* per MB: the stamp of the slice that wrote it             */
    uint32_t stamp;     /* the current slice's stamp (neighbours of other slices are not
                           available, 6.4.8; the buffers serve every slice of a picture) */
    uint8_t *tc;        /* per MB: 16 luma + 4 Cb + 4 Cr total_coeff (CAVLC nC)     */
} wctx;

/* MB (mx,my) is available: inside the picture and written by the current slice */
int  jm_w_mb_ok(const wctx *w, int mx, int my);
/* normative MVP (8.4.1.3) of the partition at (bx,by) size bw x bh (pixels, MB relative); the
   current MB's mv/ref entries must already hold its final values */
void jm_w_mvp(const wctx *w, int mx, int my, int bx, int by, int bw, int bh, int *p);
/* predIntra4x4PredMode / predIntra8x8PredMode (8.3.1.1 / 8.3.2.1) of the 4x4 block (x4, y4) */
int  jm_w_mpm(const wctx *w, int mx, int my, int x4, int y4);
/* record the macroblock's final motion / intra data in the neighbour buffers and mark it
   written (its own MVP / MPM derivations read it) */
void jm_w_mark_mb(wctx *w, int mx, int my, const jmh_mb_result *r, int skip);

/* ---- CABAC (cabac.c; SymbolMode 1) ----------------------------------------------------- */
typedef struct jm_cabac jm_cabac;
jm_cabac *jm_cabac_new(const jm_seq *s);
void jm_cabac_free(jm_cabac *c);
/* slice_data start: cabac_alignment_one_bit, context initialisation (9.3.1.1), engine init */
void jm_cabac_slice_start(jm_cabac *c, jm_bits *b, int slice_type, int qp);
/* one macroblock (mb_skip_flag in P slices, macroblock_layer), end_of_slice_flag of the
   previous one first */
void jm_cabac_write_mb(jm_cabac *c, wctx *w, int mx, int my, const jmh_mb_result *r, int slice_p);
/* bits of the last jm_cabac_write_mb (arienco_bits_written delta, no end_of_slice_flag): the RD rate
   of that macroblock (RDOptimization 1 reports it in jmh_mb_result.min_cost) */
long jm_cabac_mb_bits(const jm_cabac *c);
/* end_of_slice_flag = 1 of the slice's last macroblock, flush (its last bit is the
   rbsp_stop_one_bit), alignment; returns the slice's bin count */
long jm_cabac_slice_end(jm_cabac *c);

#endif
