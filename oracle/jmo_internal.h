/* jmo_internal.h — oracle internals (TEST INFRASTRUCTURE ONLY; see jm_oracle.h header). */
#ifndef JMO_INTERNAL_H
#define JMO_INTERNAL_H

#include <stdint.h>
#include <string.h>
#include "jm_oracle.h"

#define MAX_VALUE 999999          /* JM 8.6 defines.h MAX_VALUE [J]                       */
#define Q_BITS 15                 /* JM 8.6 defines.h Q_BITS [J]                          */
#define DQ_BITS 6
#define DQ_ROUND 32
#define LUMA_COEFF_COST 4         /* _LUMA_COEFF_COST_    (8x8 block, "<=") [J]            */
#define LUMA_MB_COEFF_COST 5      /* sum_cnt_nonz "<= 5" in LumaResidualCoding [J]         */
#define CHROMA_COEFF_COST 4       /* _CHROMA_COEFF_COST_  ("<") [J]                         */
#define SHIFT_QP 12
#define BIGCOST (1 << 20)         /* JM max_value / min_cost initialisers [J]              */

extern const int jmo_quant_coef[6][16];    /* raster [y*4+x] */
extern const int jmo_dequant_coef[6][16];
extern const int jmo_scan4x4[16];          /* zig-zag frame scan -> raster index */
extern const int jmo_qp2quant_tab[40];
extern const int jmo_qp_scale_cr_tab[52];
extern const int jmo_coeff_cost_tab[16];
extern const int jmo_blc_size[8][2];       /* JM input->blc_size [J]: {w,h} per blocktype */

static inline int iabs(int a) { return a < 0 ? -a : a; }
static inline int imin(int a, int b) { return a < b ? a : b; }
static inline int imax(int a, int b) { return a > b ? a : b; }
static inline int iclip(int lo, int hi, int v) { return v < lo ? lo : (v > hi ? hi : v); }
static inline int clip255(int v) { return v < 0 ? 0 : (v > 255 ? 255 : v); }

/* samples: 16-bit storage for every bit depth (8: values 0..255; High 10: 0..1023, JM >= 10 imgpel
 * = unsigned short [J]); Clip1 = clip to (1 << bit_depth) - 1 */
typedef uint16_t pel;
static inline int clipv(int maxv, int v) { return v < 0 ? 0 : (v > maxv ? maxv : v); }
static inline int isign(int a, int b) { return b < 0 ? -iabs(a) : iabs(a); } /* JM sign(a,b) */

/* ---- the oracle's CABAC coder for RD rates (cabac_enc.c; the tables are decoder.c's) ------- */
#define JMO_NCTX 460                 /* spec ctxIdx 0..459 (frame coding, 4:2:0)                 */
extern const uint8_t jmo_lps_range[64][4];   /* Table 9-44 rangeTabLPS                         */
extern const uint8_t jmo_lps_next[64];       /*            transIdxLPS                         */
extern const uint8_t jmo_sig8x8_inc[63], jmo_last8x8_inc[63];   /* Table 9-43 (frame)          */
void jmo_cabac_init_models(int slice_i, int qp, uint8_t *st, uint8_t *mps);   /* 9.3.1.1        */
typedef struct jmo_cab {
    uint8_t st[JMO_NCTX], mps[JMO_NCTX];     /* pStateIdx, valMPS                               */
    uint32_t low, range;                     /* codILow, codIRange                              */
    int first, outstanding;                  /* firstBitFlag, bitsOutstanding                   */
    long put;                                /* bits PutBit emitted (the first one included)    */
} jmo_cab;
typedef struct jmo_cabmbi {                  /* a coded macroblock, for its neighbours' ctxIdxInc */
    uint8_t skip, intra, i16, nxn, t8;       /* P_Skip, intra, I_16x16, I_NxN, transform_size_8x8_flag */
    uint8_t cbp, cmode, cbf_dc, cbfc[2];     /* cbp; intra_chroma_pred_mode; coded_block_flags: DC
                                                (bit 0 luma, 1 Cb, 2 Cr), chroma AC (2x2 raster)  */
    uint16_t cbf4;                           /* luma 4x4 coded_block_flags (raster; an 8x8-transform
                                                block's inferred 1 on its four)                    */
} jmo_cabmbi;
typedef struct jmo_cabnb {                   /* the current macroblock's neighbours A, B          */
    const jmo_cabmbi *A, *B;                 /* NULL: not available                              */
    int16_t mvdA[4][2], mvdB[4][2];          /* mvd_l0 of A's right column, of B's bottom row     */
} jmo_cabnb;
typedef struct jmo_cabsyn {                  /* the syntax of a macroblock candidate               */
    int mb_type, cbp, t8, i16mode, cmode;
    int b8mode[4];
    int ipm[16];                             /* I4MB raster / I8MB on each 8x8's top-left: -1 = the
                                                predicted mode, else rem_intra_pred_mode           */
    int16_t mvd[16][2];                      /* the mvd of the partition covering each 4x4 (raster) */
    const int16_t (*luma)[16];               /* as jmh_mb_result.luma / luma_dc / chroma_*        */
    const int16_t *luma_dc;
    const int16_t (*cdc)[4];
    const int16_t (*cac)[4][16];
} jmo_cabsyn;
typedef struct jmo_cabcur {                  /* the P8x8 RD loop's running macroblock state        */
    int16_t mvd[16][2];
    uint16_t cbf4;
    uint8_t cbpl;
} jmo_cabcur;
void jmo_cab_start(jmo_cab *e, int slice_i, int qp);
long jmo_cab_bits(const jmo_cab *e);         /* JM's arienco_bits_written                         */
void jmo_cab_decision(jmo_cab *e, int ctx, int bin);
void jmo_cab_bypass(jmo_cab *e, int bin);
void jmo_cab_terminate(jmo_cab *e, int bin);
void jmo_cab_skip(jmo_cab *e, const jmo_cabnb *nb);
void jmo_cab_mb(jmo_cab *e, const jmo_cabnb *nb, const jmo_cabsyn *m, int slice_p, int t8mode, jmo_cabmbi *out,
                int16_t mvd_out[16][2]);
void jmo_cab_b8(jmo_cab *e, const jmo_cabnb *nb, jmo_cabcur *cur, int b8, int sm, const int16_t (*mvd4)[2], int coded,
                const int16_t (*lev4)[16]);
void jmo_cab_i4(jmo_cab *e, const jmo_cabnb *nb, int x4, int y4, int code, const int16_t *lev);
void jmo_cab_i8(jmo_cab *e, int code, const int16_t *lev64);

/* ---- the oracle's CAVLC bit count for RD rates (cavlc_bits.c; the tables are decoder.c's) --- */
extern const uint8_t jmo_ct_len[3][4][17], jmo_ctdc_len[4][5], jmo_tz_len[15][16], jmo_tzdc_len[3][4], jmo_rb_len[7][15];
extern const uint8_t jmo_cbp_intra[48], jmo_cbp_inter[48];   /* Table 9-4: codeNum -> cbp       */
typedef struct jmo_cavnb {                   /* TotalCoeff of the neighbours A, B (NULL: not available):
                                                16 luma (4x4 raster), 4 Cb, 4 Cr (2x2 raster)     */
    const uint8_t *A, *B;
} jmo_cavnb;
int jmo_cavlc_block_bits(const int16_t *coef, int n, int nC, int *total_coeff);
int jmo_cavlc_mb_bits(const jmo_cavnb *nb, const jmo_cabsyn *m, int slice_p, int t8mode, int skip_run, uint8_t tc_out[24]);
int jmo_cavlc_b8_bits(const jmo_cavnb *nb, uint8_t cur_tc[24], int b8, int sm, const int16_t (*mvd4)[2], int coded,
                      const int16_t (*lev4)[16]);
int jmo_cavlc_skip_bits(int skip_run, int last_in_picture);
int jmo_cavlc_i4_bits(const jmo_cavnb *nb, uint8_t cur_tc[24], int x4, int y4, int code, const int16_t *lev);
int jmo_cavlc_i8_bits(const jmo_cavnb *nb, uint8_t cur_tc[24], int b8, int code, const int16_t *lev64);

/* Test hook (tests/harness/rate_xcheck.c): every RD rate the oracle computes, with the coder state,
 * neighbours and syntax it was computed from and the state after; NULL in normal use */
enum { JMO_RATE_SKIP, JMO_RATE_MB, JMO_RATE_B8, JMO_RATE_I4, JMO_RATE_I8 };
typedef struct jmo_rate_event {
    int kind, slice_p, t8mode;
    const jmo_cab *before, *after;
    const jmo_cabnb *nb;
    const jmo_cabsyn *syn;                   /* JMO_RATE_MB                                       */
    const jmo_cabcur *cur_before;            /* JMO_RATE_B8                                       */
    int b8, sm, coded;
    const int16_t (*mvd4)[2];
    const int16_t (*lev4)[16];
    int x4, y4, code;                        /* JMO_RATE_I4 (JMO_RATE_I8: code, lev[64])          */
    const int16_t *lev;
    long bits;                               /* the oracle's rate                                 */
    /* SymbolMode 0 (CAVLC): no coder state; the neighbours' TotalCoeff, the current MB's so far (B8,
       I4, I8) and the slice's pending mb_skip_run (MB) */
    int cavlc, skip_run, b8i;                /* b8i: JMO_RATE_I8's 8x8 block                       */
    int last_mb;                             /* JMO_RATE_SKIP: the last MB of the picture          */
    const jmo_cavnb *cnb;
    const uint8_t *tc_before;
} jmo_rate_event;
extern void (*jmo_rate_hook)(const jmo_rate_event *ev);

/* ---- encoder state (replaces JM's img/enc_picture globals for the hot path) ------------ */
struct jmo_ctx {
    jmh_config cfg;
    int W, H, Wc, Hc, mbw, mbh;
    int bd, maxv, qpbd;              /* bit depth, (1 << bd) - 1, QpBdOffsetY = QpBdOffsetC = 6 (bd - 8) */
    int sr;                          /* max search range                                       */
    int npos;                        /* (2sr+1)^2                                              */
    int32_t *spiral_x, *spiral_y;    /* JM spiral_search_x/y [J]                               */
    int32_t *spiral_of;              /* window raster (dy+sr)*(2sr+1)+(dx+sr) -> spiral index   */
    /* current picture (coded size) */
    pel *orgY, *orgU, *orgV;
    /* reference: integer planes + 16 quarter-pel phase planes (padded by JMO_PAD) */
    pel *refY, *refU, *refV;
    pel *qpel;                       /* [16][H+2P][W+2P]                                        */
    int qstride, qplane;
    int have_ref;
    /* unfiltered reconstruction (enc_picture->imgY / imgUV) */
    pel *recY, *recU, *recV;
    /* per-4x4 picture arrays (enc_picture->mv / ref_idx, img->ipredmode) */
    int16_t *mv;                     /* [(H/4)*(W/4)][2] */
    int8_t *refidx;                  /* [(H/4)*(W/4)]    */
    int8_t *ipred;                   /* [(H/4)*(W/4)]    */
    int8_t *mbintra;                 /* per MB: 1 if intra                                      */
    jmh_mb_result *res;
    jmh_frame_params fp;
    /* per-MB scratch */
    uint16_t *blocksad;              /* [16][npos] 4x4 SADs (window raster order)               */
    /* EPZS (SearchMode 3): the previous picture's motion field (temporal predictors) and the
       left macroblock's per-blocktype search results (spatial memory predictors) */
    int16_t *tmv;                    /* [(H/4)*(W/4)][2], snapshot of mv at picture start        */
    int8_t *tref;                    /* [(H/4)*(W/4)], -1: intra / no previous picture          */
    int16_t mem_mv[8][16][2];        /* all_mv of the MB to the left (valid when mbx > 0)       */
    uint16_t *epzs_fp;               /* [8][(H/4)*(W/4)]: each search's full-pel cost (saturated at
                                        65535) per block type and 4x4: the neighbours' distortion of
                                        EPZSDetermineStopCriterion (item 61)                     */
    /* RDOptimization = 1: the slice's CABAC coder (cabac_enc.c), what every coded macroblock leaves
       for its neighbours' context selection, and the mvd_l0 of every 4x4 block */
    jmo_cab cab;
    jmo_cabmbi *cabi;
    int16_t *cab_mvd;                /* [(H/4)*(W/4)][2] */
    /* ... with SymbolMode 0: the slice's pending mb_skip_run and every MB's 24 TotalCoeff */
    int cav_run;
    uint8_t *cav_tc;                 /* [mbw*mbh][24] */
};

/* SliceMode 1 (SliceArgument MBs per slice, raster order): MB addresses a and n lie in one slice.
 * Neighbours precede the current MB, so this is "n >= the slice's first MB" (6.4.8).          */
static inline int jmo_same_slice(const jmo_ctx *c, int a, int n) {
    int k = c->cfg.slice_mbs;
    return k <= 0 || n >= a - a % k;
}

/* common.c */
void jmo_init_spiral(jmo_ctx *c);
void jmo_build_qpel(jmo_ctx *c);
int  jmo_qpel_at(const jmo_ctx *c, int X, int Y);   /* from the phase planes (clamped)   */
int  jmo_satd_block(const int32_t d[16], int use_hadamard);
void jmo_fwd4x4(int32_t m[16]);                       /* in-place, raster                 */
void jmo_inv4x4_add(const int32_t m[16], const pel *pred, int pstride, pel *out, int ostride, int maxv);
/* spec luma sample at quarter-pel (X,Y) of a pel plane (8.4.2.2.1, Clip1 to maxv)            */
int  jmo_qpel_px(const pel *p, int w, int h, int stride, int X, int Y, int maxv);
/* QPc of a luma QP + chroma offset (8.5.8, Table 8-15), qPI clipped to [-qpbd, 51]: negative
 * values map to themselves (high bit depth); add qpbd for QP'c                              */
int  jmo_qpc(int qp_plus_offset, int qpbd);

/* 8x8 transform (High profile) */
#define Q_BITS_8 16               /* JM FRExt Q_BITS_8 [J]                                 */

/* Quantisation rounding selector (docs/JM_SEMANTICS.md items 1 and 45), the `intra_round` argument
 * of the dct_* functions and the oracle's TQ seams: JMO_RND_P / JMO_RND_I are JM 8.6's
 * (1 << q_bits) / 6 and / 3; JMO_RND_OFF(o) is a JM >= 10 flat OffsetMatrix entry o at OffsetBits 11
 * (q_offsets.c CalculateOffsetParam: LevelOffset = OffsetList << (q_bits - OffsetBits)) [J] */
#define JMO_RND_P 0
#define JMO_RND_I 1
#define JMO_RND_OFF(o) (2 + (o))
#define OFFSET_BITS 11
static inline int jmo_qround(int rnd, int q_bits) {
    return rnd >= 2 ? (rnd - 2) << (q_bits - OFFSET_BITS) : rnd ? (1 << q_bits) / 3 : (1 << q_bits) / 6;
}
extern const int jmo_quant8_cls[6][6];
extern const int jmo_dequant8_cls[6][6];
int  jmo_class8(int x, int y);
int  jmo_coeff_cost8(int run);
void jmo_scan8x8(int scan[64]);
void jmo_fwd8x8(int32_t m[64]);
void jmo_inverse8x8(const int32_t *in, int32_t *out);
void jmo_inv8x8_add(const int32_t m[64], const pel *pred, int pstride, pel *out, int ostride, int maxv);
/* Intra8x8 prediction on pel samples (jmo_intra8x8_pred's body); dc = 1 << (bd - 1)          */
int  jmo_intra8x8_pred_px(const int32_t nb[25], int avail, pel pred[9][64], int dc);
int  jmo_satd8x8(const int32_t d[64], int use_hadamard);

/* encode.c */
void jmo_encode_mb(jmo_ctx *c, int mbx, int mby);

/* ---- encode.c internals shared with the RD mode decision (rdo.c) ------------------------ */
typedef struct {
    jmo_ctx *c;
    int mbx, mby, pix_x, pix_y, mb_addr;
    int lambda;                /* RDO off: lambda_mode == lambda_motion (integer)                  */
    int lf;                    /* LAMBDA_FACTOR(lambda_motion): 65536*lambda (RDO off), RDO on the
                                  host's (int)(65536 * sqrt(lambda_mode) + 0.5)                      */
    int rdo;                   /* RDOptimization 1: no 16x16 zero-vector biases (!input->rdopt [J]) */
    int slice_p;
    pel org[256];              /* imgY_org of the MB                                       */
    pel orgc[2][64];
    /* FFS state (SetupFastFullPelSearch) */
    int setup_done, scx, scy, pos_00;
    int16_t all_mv[8][16][2];  /* img->all_mv[.][.][LIST_0][ref 0][blocktype]               */
    int16_t pmv[8][16][2];     /* the MVP each search used (its partition's mvd = mv - pmv)   */
    int motion_cost[8][4];
    int skip_mv[2];
} mbs;
int  jmo_nb4(const mbs *s, int xN, int yN, int *idx);
void jmo_set_mvp(const mbs *s, int pmv[2], int ref, int block_x, int block_y, int bsx, int bsy);
void jmo_find_skip_mv(mbs *s);
void jmo_write_enc_mv(mbs *s, int bx4, int by4, int w4, int h4, const int16_t (*mv)[2]);
void jmo_partition_motion_search(mbs *s, int blocktype, int block8x8);
int  jmo_dct_luma4x4(const int32_t resid[16], const pel *pred, int ps, int qp, int intra_round, int16_t levels[16],
                     int *coeff_cost, pel *rec, int rs, int maxv);
int  jmo_dct_luma8x8(const int32_t resid[64], const pel *pred, int ps, int qp, int intra_round, int16_t levels[64],
                     int *coeff_cost, pel *rec, int rs, int maxv);
void jmo_put_levels8(int16_t luma[16][16], int b8, const int16_t lev[64]);
int  jmo_dct_chroma(const int32_t resid[64], const pel pred[64], int qpc, int intra_round, int cr_cbp, int16_t dc_out[4],
                    int16_t ac_out[4][16], pel rec[64], int maxv);
int  jmo_dct_luma_16x16(const int32_t resid[256], const pel pred[256], int qp, int rnd, int16_t dc_out[16],
                        int16_t ac_out[16][16], int *cbp_blk, pel rec[256], int maxv);
int  jmo_mb_avail(const mbs *s, int dmx, int dmy);
void jmo_intra4x4_pred(const mbs *s, int bx, int by, pel pred[9][16], int avail[9]);
void jmo_intra16_pred(const mbs *s, pel pred[4][256], int avail[4]);
void jmo_intra_chroma_pred(const mbs *s, int uv, pel pred[4][64], int avail[4]);
int  jmo_find_sad_16x16(const mbs *s, pel pred[4][256], const int avail[4], int *mode);
void jmo_luma_pred_4x4(const mbs *s, int bx4, int by4, int mvx, int mvy, pel *out, int os);
void jmo_chroma_pred_mb(const mbs *s, int uv, const int16_t mv[16][2], pel pred[64]);
void jmo_store_rec_luma(jmo_ctx *c, const mbs *s, const pel rec[256]);
int  jmo_i8_neighbours(const mbs *s, const pel rec[256], int b8, int32_t nb[25]);
int  jmo_i8_mpm(const mbs *s, int b8, const int modes[4]);

/* rdo.c: encode_one_macroblock with RDOptimization = 1 (CABAC rate) */
void jmo_encode_mb_rdo(jmo_ctx *c, int mbx, int mby);

#endif
