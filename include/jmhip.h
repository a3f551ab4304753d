/*
 * jmhip.h — C ABI of the MI355X-native JM (lencod) hot path:
 *           motion estimation + integer transform / quantisation / reconstruction.
 *
 * This is the drop-in boundary.  JM has no plugin/FFI API; its seams are the
 * C functions of lencod.  Each entry point below replaces one of them:
 *
 *   JM 8.6 lencod seam [J]                                  replaced by
 *   ----------------------------------------------------    -----------------------------------
 *   image.c  › UnifiedOneForthPix(enc_frame_picture)        jmh_set_reference()
 *   image.c  › code_a_picture → encode_one_slice →
 *              per MB encode_one_macroblock()  (rdopt.c)    jmh_frame_submit() + jmh_frame_wait()
 *              (+ mv-search.c › PartitionMotionSearch /         then, per MB, jmh_get_mb_result()
 *               BlockMotionSearch / SetupFastFullPelSearch /
 *               FastFullPelBlockMotionSearch / SubPelBlock-
 *               MotionSearch, block.c › dct_luma / dct_chroma /
 *               dct_luma_16x16, macroblock.c › LumaResidual-
 *               Coding / ChromaResidualCoding)
 *   enc_picture->imgY / imgUV (unfiltered reconstruction)   jmh_read_recon()
 *   mv-search.c › SetupFastFullPelSearch (BlockSAD table)    jmh_ffs_sad_table()   (unit seam)
 *   block.c › dct_luma (4x4 TQ + recon)                     jmh_tq4x4_batch()     (unit seam)
 *   block.c › dct_luma8x8 (JM FRExt, High profile)          jmh_tq8x8_batch()     (unit seam)
 *   mv-search.c › BlockMotionSearch (one block, caller's MVP,   jmh_search_pictures() +
 *               centre, range and lambda: the per-call seam    jmh_block_motion_search()
 *               of host/jm86.c BlockMotionSearch /
 *               PartitionMotionSearch and of an RDO-on loop)
 *   the same seams at 9 / 10 bits (JM >= 10 imgpel = u16)   jmh_*_u16()
 *
 * Reference citations: the mounted reference (/root/reference) holds only README.md:1-4 (an
 * annotated-JM commentary with no source), so no file:line into JM source exists; the JM
 * function names above are the JM 8.6 names (tag [J]).  docs/JM_SEMANTICS.md
 * pins every non-normative choice.
 *
 * Conventions: plain C types only; 0 = OK, negative JMH_E_* on error; nothing throws or aborts
 * across this boundary.  One context = one HIP device + one HIP stream; a context is not
 * thread-safe (JM is single threaded).  Multi-GPU = one process (and one context) per GPU.
 */
#ifndef JMHIP_H
#define JMHIP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define JMH_ABI_VERSION 14
#define JMH_LAMBDA_MAX 1023   /* jmh_frame_params lambdas: lambda * mvbits fits the u16 cost tables */
#define JMH_QOFFSET_MAX 2047  /* jmh_config.quant_offset: OffsetBits 11 (1 << 11 = a whole step)    */

/* ---- status codes ---------------------------------------------------------------------- */
#define JMH_OK                 0
#define JMH_E_INVALID_ARG     (-1)
#define JMH_E_HIP             (-2)
#define JMH_E_OOM             (-3)
#define JMH_E_UNSUPPORTED_CFG (-4)
#define JMH_E_STATE           (-5)
#define JMH_E_NO_DEVICE       (-6)

/* ---- slice types (H.264 slice_type % 5) ------------------------------------------------- */
#define JMH_P_SLICE 0
#define JMH_I_SLICE 2

/* ---- macroblock types: JM 8.6 defines.h numbering [J] ------------------------------------ */
#define JMH_PSKIP  0   /* P_Skip (P slice, 16x16, ref 0, skip MV, cbp 0)  */
#define JMH_P16x16 1
#define JMH_P16x8  2
#define JMH_P8x16  3
#define JMH_SMB8x8 4   /* sub-macroblock types 4..7 = 8x8, 8x4, 4x8, 4x4 (b8mode[] only) */
#define JMH_SMB8x4 5
#define JMH_SMB4x8 6
#define JMH_SMB4x4 7
#define JMH_P8x8   8
#define JMH_I4MB   9
#define JMH_I16MB  10
#define JMH_IBLOCK 11  /* b8mode[] of an I4MB */
#define JMH_I8MB   13  /* Intra8x8 (High profile, Transform8x8Mode; JM FRExt numbering [J])       */

/* ---- encoder configuration (encoder.cfg subset that the hot path reads) ----------------- */
typedef struct jmh_config {
    int32_t width;                  /* coded luma width  (multiple of 16)                        */
    int32_t height;                 /* coded luma height (multiple of 16)                        */
    int32_t search_range;           /* SearchRange (full-pel), 1..32 (LDS-resident window; larger
                                       values return JMH_E_UNSUPPORTED_CFG)                       */
    int32_t search_mode;            /* 0 = fast full search (FFS, JM _FAST_FULL_ME_), -1 = full   */
    int32_t use_hadamard;           /* UseHadamard                                                */
    int32_t restrict_search_range;  /* RestrictSearchRange 0 / 1 / 2                              */
    int32_t inter_search[8];        /* [1..7] = InterSearch16x16 .. InterSearch4x4 ([0] unused)   */
    int32_t num_ref_frames;         /* NumberReferenceFrames (this build: 1)                      */
    int32_t constrained_intra_pred; /* UseConstrainedIntraPred 0 / 1 (constrained_intra_pred_flag) */
    int32_t num_frame_slots;        /* device-resident input frame slots (bench / pipelining)     */
    int32_t flags;                  /* JMH_FLAG_* (0 for the defaults)                            */
    int32_t pipeline_depth;         /* pictures in flight at once (0: enough to fill the device,  */
                                    /*   1: one picture at a time); see jmh_frame_push            */
    int32_t transform_8x8_mode;     /* Transform8x8Mode: 0 off, 1 adaptive 4x4 / 8x8 (High profile) */
    int32_t jm_version;             /* JMVersion: 0 or 8 = JM 8.6 quantisation rounding ((1 << q_bits)
                                       / 3 in I slices, / 6 in P slices, Intra16x16 always / 3);
                                       >= 10 = JM >= 10 q_offsets.c: every block of a slice rounds
                                       with quant_offset[slice] << (q_bits - 11) (docs/JM_SEMANTICS.md
                                       items 1, 45; AdaptiveRounding off)                           */
    int32_t quant_offset[2];        /* JMVersion >= 10: flat OffsetMatrix entries at OffsetBits 11 for
                                       [0] I slices, [1] P slices, 0..JMH_QOFFSET_MAX (JM defaults
                                       682, 342: Offset_intra_default_intra / _inter) [J]          */
    int32_t epzs_dual_refinement;   /* EPZSDualRefinement (SearchMode 3): 0 off, 1 refine the runner-up
                                       predictor too (docs/JM_SEMANTICS.md item 46)                 */
    int32_t slice_mbs;              /* SliceMode 1 / SliceArgument: macroblocks per slice in raster
                                       order (0: one slice per picture).  Intra prediction, MV
                                       prediction and the EPZS spatial memory see only neighbours of
                                       the same slice (H.264 6.4.8, docs/JM_SEMANTICS.md item 47);
                                       deblocking still crosses slice edges (idc 0)                 */
    int32_t bit_depth;              /* BitDepthLuma = BitDepthChroma: 0 or 8 (8-bit pictures, the
                                       uint8_t entry points), 9 or 10 (High 10: 16-bit samples through
                                       the *_u16 picture entry points; SearchMode 0, -1 or 3; quantisation
                                       at QP + QpBdOffset, Clip1 to (1 << bit_depth) - 1, deblocking
                                       thresholds scaled by 1 << (bit_depth - 8); docs/JM_SEMANTICS.md
                                       items 49-52)                                                  */
    int32_t rdo;                    /* RDOptimization: 0 off (the cost-based decision of rdopt.c's RDO-off
                                       branch), 1 on: encode_one_macroblock's rate-distortion loop
                                       (RDCost_for_macroblocks / RDCost_for_8x8blocks / RDCost_for_4x4
                                       IntraBlocks / RDCost_for_8x8IntraBlocks [J]: SSD + lambda_rd *
                                       rate, the rate from the CABAC coding state of the slice,
                                       csrc/jmh_cabac_rate.h, or with symbol_mode 0 the CAVLC bit count,
                                       csrc/jmh_cavlc_rate.h); with SearchMode 3, 0 or -1
                                       (docs/JM_SEMANTICS.md items 53-60, 63, 64, 65)                 */
    int32_t symbol_mode;            /* SymbolMode: 0 CAVLC, 1 CABAC (the RD rate's entropy coder)     */
    /* JM >= 10 EPZS options (SearchMode 3; docs/JM_SEMANTICS.md items 61, 62); zero keeps items 36, 39 */
    int32_t epzs_subpel_me;         /* EPZSSubPelME: 0 SubPelBlockMotionSearch, 1 the EPZS sub-pel
                                       pattern search (small diamond at half, then quarter pel)      */
    int32_t epzs_subpel_thres_scale;/* EPZSSubPelThresScale, 0..JMH_EPZS_SCALE_MAX: the quarter-pel
                                       stage is skipped below scale x block pixels x pel_error (0:
                                       never)                                                       */
    int32_t epzs_min_thres_scale;   /* EPZSMinThresScale, 0..JMH_EPZS_SCALE_MAX                      */
    int32_t epzs_max_thres_scale;   /* EPZSMaxThresScale, 0..JMH_EPZS_SCALE_MAX: 0 = the fixed medthres
                                       stop after the predictors (item 36); >= 1 the stop criterion
                                       from the neighbours' full-pel costs clamped to [min, max] x
                                       block pixels x pel_error (EPZSDetermineStopCriterion, item 61) */
} jmh_config;
#define JMH_EPZS_SCALE_MAX 63       /* keeps every threshold below 2^16 at 10 bits */
/* per-launch HIP-event timing of the two wavefront kernels on every 8th diagonal (jmh_timing
 * analyse_ms / final_ms and their launch counts: averages per launch, sampled uniformly)     */
#define JMH_FLAG_KERNEL_TIMING 1
/* pictures deblocked on the device (jmh_frame_params.deblock) skip the readback of the
   reconstruction before deblocking: jmh_read_recon returns JMH_E_STATE for them (lencod with
   device deblocking reads only jmh_read_deblocked) */
#define JMH_FLAG_NO_RECON_READBACK 2

/* ---- per-picture parameters ------------------------------------------------------------- */
typedef struct jmh_frame_params {
    int32_t slice_type;        /* JMH_P_SLICE / JMH_I_SLICE                                      */
    int32_t qp;                /* slice QP (0..51), constant over the picture (no rate control)  */
    int32_t lambda_mode;       /* RDO off: QP2QUANT[max(0,qp-12)] (integer, computed on host);   */
    int32_t lambda_motion;     /* RDO off: == lambda_mode.  Both 0..JMH_LAMBDA_MAX (JM: <= 91)   */
    int32_t chroma_qp_offset;  /* chroma_qp_index_offset                                         */
    int32_t deblock;           /* 1: also deblock (DeblockFrame, 8.7) on the device into the     */
                               /*    next reference (jmh_read_deblocked, set_reference_slot(-2)) */
    int32_t lf_disable;        /* disable_deblocking_filter_idc (1: copy, no filtering)          */
    int32_t lf_alpha_div2;     /* slice_alpha_c0_offset_div2                                     */
    int32_t lf_beta_div2;      /* slice_beta_offset_div2                                         */
    int32_t lambda_factor_rd;  /* RDO on: LAMBDA_FACTOR(lambda_motion) = (int)(65536 * sqrt(lambda_rd)
                                  + 0.5), the motion searches' lambda (computed on the host, libm)   */
    double  lambda_rd;         /* RDO on: lambda_mode = 0.85 * 2^((QP + QpBdOffsetY - 12) / 3) (P and
                                  I slices, no B pictures), the J = D + lambda * R multiplier        */
} jmh_frame_params;

/* ---- per-macroblock result (what encode_one_macroblock leaves behind) ------------------- */
typedef struct jmh_mb_result {
    int16_t mb_type;           /* JMH_PSKIP .. JMH_I16MB                                          */
    int16_t cbp;               /* luma bits 0..3 (8x8 blocks), chroma (0/1/2) << 4                */
    int32_t cbp_blk;           /* bit (4*by+bx): 4x4 luma block has non-zero levels (I16: AC);
                                  transform_8x8: all four bits of an 8x8 block with any level      */
    int8_t  b8mode[4];         /* per 8x8: sub-mb type 4..7 for P8x8, mb_type otherwise           */
    int8_t  ref_idx[4];        /* per 8x8, list 0; -1 for intra                                  */
    int8_t  i16mode;           /* Intra16x16 prediction mode 0..3 (I16MB only)                   */
    int8_t  c_ipred_mode;      /* intra chroma prediction mode 0..3 (intra MBs)                  */
    int8_t  transform_8x8;     /* transform_size_8x8_flag (0 unless the MB codes luma with 8x8)   */
    int8_t  pad0;
    int8_t  ipred[16];         /* Intra4x4 modes, 4x4 raster order (by*4+bx); I8MB: the Intra8x8
                                  mode of the 8x8 block, repeated on its four 4x4; 2 (DC) otherwise */
    int16_t mv[16][2];         /* final list-0 MV per 4x4 block (raster), quarter-pel            */
    int16_t luma[16][16];      /* per 4x4 block (raster): levels in frame zig-zag scan order;
                                  I16MB: AC only, [k][0] = 0.  transform_8x8: the 8x8 block's 64
                                  levels in 8x8 zig-zag order, interleaved as CAVLC codes them
                                  (7.3.5.3.2): luma[4x4 j of the 8x8][k] = level8x8[4k + j], j in
                                  0 TL, 1 TR, 2 BL, 3 BR                                            */
    int16_t luma_dc[16];       /* I16MB DC levels, zig-zag scan order                             */
    int16_t chroma_dc[2][4];   /* [uv][k] 2x2 DC levels, raster c0..c3                            */
    int16_t chroma_ac[2][4][16]; /* [uv][4x4 blk raster][scan]; [..][0] = 0                       */
    int32_t min_cost;          /* diagnostic: cost of the chosen mode                             */
    int32_t reserved;
} jmh_mb_result;

/* ---- kernel timing (HIP events on the context stream), summed since the previous
 *      jmh_get_timing call (which resets the sums).  jmh_get_timing waits for the launches
 *      issued so far and does NOT drain pictures in flight (the pipeline stays primed).  ---- */
typedef struct jmh_timing {
    float interp_ms;           /* sum of quarter-pel interpolations (jmh_set_reference*)       */
    float mb_ms;               /* sum of whole macroblock wavefronts (first to last dispatch)  */
    float total_ms;            /* last jmh_frame_submit: H2D + wavefront + D2H                 */
    int32_t mb_launches;       /* wavefront launches (dispatches) per picture                  */
    int32_t pictures;          /* pictures summed in mb_ms                                     */
    int32_t interps;           /* interpolations summed in interp_ms                           */
    float analyse_ms;          /* JMH_FLAG_KERNEL_TIMING: sum of sampled k_mb_analyse launches   */
    int32_t analyse_launches;  /*   ... and the number of launches summed                       */
    float final_ms;            /* JMH_FLAG_KERNEL_TIMING: sum of k_mb_final launch durations    */
    int32_t final_launches;
    int32_t ticks;             /* wavefront ticks (one k_mb_analyse + one k_mb_final each; a tick
                                  runs one diagonal of every picture in flight)                   */
    int32_t tick_mbs;          /* macroblocks processed by those ticks                          */
    int32_t pictures_done;     /* pictures whose last tick was issued (completed once the
                                  issued work has drained: jmh_wait_issued)                      */
    int32_t flow_launches;     /* ABI 14: dataflow launches (k_mb_flow: one per segment of ticks,
                                  SearchMode 0 at 8 bits, RDO off); analyse_ms / analyse_launches
                                  then time those launches                                        */
    int32_t flow_mbs;          /*   ... and the macroblocks they processed                        */
} jmh_timing;

typedef struct jmh_ctx jmh_ctx;

/* ---- lifecycle -------------------------------------------------------------------------- */
int  jmh_create(const jmh_config *cfg, int hip_device, jmh_ctx **out);
void jmh_destroy(jmh_ctx *ctx);
const char *jmh_strerror(int status);
int  jmh_abi_version(void);
int  jmh_device_count(void);

/* ---- reference picture (replaces UnifiedOneForthPix on the deblocked recon) --------------
 * list must be 0 and ref_idx 0 in this build.  Planes are 8-bit, coded size, 4:2:0.        */
int  jmh_set_reference(jmh_ctx *ctx, int list, int ref_idx,
                       const uint8_t *y, const uint8_t *u, const uint8_t *v,
                       int stride_y, int stride_c);

/* ---- one picture of encode_one_macroblock() calls ----------------------------------------
 * The caller's planes must stay valid until jmh_frame_submit returns (copied to the device).
 * Results and recon become host-visible after jmh_frame_wait; pointers returned by
 * jmh_get_mb_result stay valid until the next submit / pop.                                     */
int  jmh_frame_submit(jmh_ctx *ctx, const uint8_t *y, const uint8_t *u, const uint8_t *v,
                      int stride_y, int stride_c, const jmh_frame_params *fp);
int  jmh_frame_wait(jmh_ctx *ctx);
/* ---- pipelined pictures (the frame loop of lencod.c › main with pictures in flight) --------
 * jmh_frame_push queues a picture against the current reference and returns at once; a P
 * picture whose reference is the previous picture (jmh_set_reference_slot -1 / -2) runs each
 * wavefront diagonal d once that picture has finished diagonal d + PIPE_LAG (jmh_device.h), so
 * up to jmh_pipeline_depth() pictures share every launch.  jmh_frame_pop waits for the oldest
 * pushed picture; jmh_get_mb_result / jmh_read_recon / jmh_read_deblocked then return its
 * results (submit == push, wait == pop).  Results are identical to one picture at a time.
 * Push returns JMH_E_STATE when jmh_pipeline_depth() pictures are waiting to be popped.       */
int  jmh_frame_push(jmh_ctx *ctx, const uint8_t *y, const uint8_t *u, const uint8_t *v,
                    int stride_y, int stride_c, const jmh_frame_params *fp);
int  jmh_frame_pop(jmh_ctx *ctx);
int  jmh_pipeline_depth(const jmh_ctx *ctx);
const jmh_mb_result *jmh_get_mb_result(const jmh_ctx *ctx, int mb_addr);
int  jmh_read_recon(jmh_ctx *ctx, uint8_t *y, uint8_t *u, uint8_t *v, int stride_y, int stride_c);
/* the deblocked picture of the last jmh_frame_submit with deblock = 1 (replaces DeblockFrame)  */
int  jmh_read_deblocked(jmh_ctx *ctx, uint8_t *y, uint8_t *u, uint8_t *v, int stride_y, int stride_c);

/* ---- device-resident variants (inputs already in HBM; used by bench.py) ------------------ */
int  jmh_load_frame(jmh_ctx *ctx, int slot, const uint8_t *y, const uint8_t *u, const uint8_t *v,
                    int stride_y, int stride_c);
int  jmh_set_reference_slot(jmh_ctx *ctx, int slot);   /* slot -1: the last picture's recon,    */
                                                         /* -2: its device deblocking (deblock=1) */
int  jmh_encode_slot(jmh_ctx *ctx, int slot, const jmh_frame_params *fp); /* pipelined, no D2H */
int  jmh_sync(jmh_ctx *ctx);           /* drain: every picture in flight runs to completion  */
/* wait for the launches issued so far WITHOUT issuing more: pictures in flight stay in flight
 * (partially encoded), so a timed region can start and end with the pipeline full            */
int  jmh_wait_issued(jmh_ctx *ctx);
int  jmh_get_timing(jmh_ctx *ctx, jmh_timing *t);

/* ---- unit seams (minimum slice; tests call these directly) ------------------------------
 * jmh_ffs_sad_table: SetupFastFullPelSearch's 4x4 BlockSAD table for n_mb macroblocks of the
 *   picture in resident slot 0 (jmh_load_frame) against the current reference.  mb_xy[2*i] = (mb_x, mb_y); centres[2*i] = absolute full-pel window centre
 *   offset (cx, cy) relative to the MB.  out[i][blk(16)][(2R+1)^2] in window raster order
 *   (dy outer, dx inner, dy,dx in [-R,R]).                                                  */
int  jmh_ffs_sad_table(jmh_ctx *ctx, int n_mb, const int32_t *mb_xy, const int32_t *centres,
                       uint16_t *out);
/* jmh_tq4x4_batch: dct_luma on n independent 4x4 residual blocks.  resid[n][16] (raster),
 *   pred[n][16] (raster), levels[n][16] (scan order), recon[n][16] (raster); nonzero[n].
 *   intra selects the I-slice rounding offset vs the P-slice one: JM 8.6 (1<<q_bits)/3 vs /6,
 *   or with jm_version >= 10 the context's quant_offset[0] vs [1] << (q_bits - 11).          */
int  jmh_tq4x4_batch(jmh_ctx *ctx, int n, const int16_t *resid, const uint8_t *pred, int qp,
                     int intra, int16_t *levels, uint8_t *recon, int32_t *coeff_cost,
                     int32_t *nonzero);
/* jmh_tq8x8_batch: dct_luma8x8 (High profile, a12) on n independent 8x8 blocks, the same
 *   one-wave-per-block primitive as the macroblock kernels.  resid[n][64] (raster), pred[n][64]
 *   (raster), levels[n][64] (8x8 zig-zag scan order), recon[n][64] (raster); coeff_cost[n]
 *   (COEFF_COST8x8), nonzero[n].  intra selects the rounding offset as for jmh_tq4x4_batch. */
int  jmh_tq8x8_batch(jmh_ctx *ctx, int n, const int16_t *resid, const uint8_t *pred, int qp,
                     int intra, int16_t *levels, uint8_t *recon, int32_t *coeff_cost,
                     int32_t *nonzero);
/* ---- per-block motion search: JM 8.6 mv-search.c › BlockMotionSearch [J] for one block per
 * request, from the arguments BlockMotionSearch works from (the caller derives the MVP with
 * SetMotionVectorPredictor, the centre with SetupFastFullPelSearch / the MVP, the range with
 * RestrictSearchRange): full pel (FFS: (0,0) pre-check then the spiral around the MB's window
 * centre; full search: the spiral around the block's own centre with the 16x16 zero-vector
 * bias) and SubPelBlockMotionSearch (half then quarter pel, SATD with UseHadamard of the
 * context's configuration).  Searches the luma pictures given to jmh_search_pictures.        */
typedef struct jmh_block_search {
    int32_t mb_x, mb_y;         /* macroblock, in MBs                                              */
    int32_t blocktype;          /* 1..7: 16x16, 16x8, 8x16, 8x8, 8x4, 4x8, 4x4                      */
    int32_t block_x, block_y;   /* block position inside the MB, 4x4 units                        */
    int32_t pred_mv[2];         /* the block's MVP, quarter pel                                   */
    int32_t centre[2];          /* full-pel search centre (an MV): FFS the MB's window centre,    */
                                /*   full search pred_mv / 4 clamped to +-search_range            */
    int32_t search_range;       /* 0..SearchRange: the spiral's first (2R+1)^2 positions          */
    int32_t lambda_factor;      /* LAMBDA_FACTOR(lambda_motion) = (int)(65536 * lambda + 0.5)     */
    int32_t search_mode;        /* 0 fast full search, -1 full search                             */
    int32_t slice_p;            /* 1: P slice (the 16x16 zero-vector biases apply)                */
} jmh_block_search;
typedef struct jmh_block_result {
    int32_t mv[2];              /* quarter pel (what BlockMotionSearch stores in all_mv)          */
    int32_t min_mcost;          /* BlockMotionSearch's return value                               */
    int32_t fullpel_mv[2];      /* the full-pel winner                                            */
    int32_t fullpel_cost;
} jmh_block_result;
/* current and reference luma pictures (coded size) of the per-block searches (copied)         */
int  jmh_search_pictures(jmh_ctx *ctx, const uint8_t *cur_y, const uint8_t *ref_y, int stride_y);
/* n independent requests in one launch (n = 1 for a JM-shaped call); res[n]                   */
int  jmh_block_motion_search(jmh_ctx *ctx, int n, const jmh_block_search *req, jmh_block_result *res);

/* ---- High 10 (config 5, BitDepthLuma 9 / 10) sample path: the same seams on 16-bit samples
 * 0 .. (1 << bit_depth) - 1, bit_depth 8..10 (8 gives exactly the 8-bit seams' results).
 * JM >= 10 FRExt [J] (imgpel = unsigned short): SAD / SATD on the wider samples, quarter-pel
 * interpolation clipped to (1 << bit_depth) - 1 (H.264 8.4.2.2.1 Clip1Y), quantisation at
 * qp + QpBdOffsetY (6 * (bit_depth - 8), qp_per / qp_rem / q_bits of block.c › dct_luma /
 * dct_luma8x8), reconstruction clipped to (1 << bit_depth) - 1.  The whole-picture wavefront
 * stays 8-bit (docs/JM_SEMANTICS.md items 41-44).                        */
/* luma pictures (coded size, 16-bit samples) of the 10-bit per-block searches (copied)        */
int  jmh_search_pictures_u16(jmh_ctx *ctx, const uint16_t *cur_y, const uint16_t *ref_y, int stride_y,
                             int bit_depth);
/* jmh_block_motion_search on the pictures of jmh_search_pictures_u16 (costs need 19 bits:
   a 16x16 SAD reaches 256 * 1023)                                                            */
int  jmh_block_motion_search_u16(jmh_ctx *ctx, int n, const jmh_block_search *req, jmh_block_result *res);
/* SetupFastFullPelSearch's 4x4 BlockSAD table (as jmh_ffs_sad_table, a 4x4 SAD <= 16 * 1023
   fits 16 bits) on the pictures of jmh_search_pictures_u16, by v_sad_u16 on sample pairs       */
int  jmh_ffs_sad_table_u16(jmh_ctx *ctx, int n_mb, const int32_t *mb_xy, const int32_t *centres,
                           uint16_t *out);
/* dct_luma / dct_luma8x8 on 16-bit predictions and reconstructions; qp 0..51 is the slice QP
   (QpBdOffsetY is added from bit_depth); resid within +-((1 << bit_depth) - 1)                */
int  jmh_tq4x4_batch_u16(jmh_ctx *ctx, int n, const int16_t *resid, const uint16_t *pred, int qp,
                         int intra, int bit_depth, int16_t *levels, uint16_t *recon,
                         int32_t *coeff_cost, int32_t *nonzero);
int  jmh_tq8x8_batch_u16(jmh_ctx *ctx, int n, const int16_t *resid, const uint16_t *pred, int qp,
                         int intra, int bit_depth, int16_t *levels, uint16_t *recon,
                         int32_t *coeff_cost, int32_t *nonzero);

/* ---- High 10 pictures (jmh_config.bit_depth 9 / 10): the picture entry points above on 16-bit
 * samples 0 .. (1 << bit_depth) - 1, same semantics, strides in samples.  The whole wavefront
 * (motion search, intra, mode decision, TQ + reconstruction, deblocking) runs on them.  A context
 * with bit_depth 9 / 10 accepts only these for pictures (the uint8_t ones return
 * JMH_E_UNSUPPORTED_CFG) and vice versa.                                                      */
int  jmh_set_reference_u16(jmh_ctx *ctx, int list, int ref_idx, const uint16_t *y, const uint16_t *u,
                           const uint16_t *v, int stride_y, int stride_c);
int  jmh_frame_submit_u16(jmh_ctx *ctx, const uint16_t *y, const uint16_t *u, const uint16_t *v,
                          int stride_y, int stride_c, const jmh_frame_params *fp);
int  jmh_frame_push_u16(jmh_ctx *ctx, const uint16_t *y, const uint16_t *u, const uint16_t *v,
                        int stride_y, int stride_c, const jmh_frame_params *fp);
int  jmh_read_recon_u16(jmh_ctx *ctx, uint16_t *y, uint16_t *u, uint16_t *v, int stride_y, int stride_c);
int  jmh_read_deblocked_u16(jmh_ctx *ctx, uint16_t *y, uint16_t *u, uint16_t *v, int stride_y, int stride_c);
int  jmh_load_frame_u16(jmh_ctx *ctx, int slot, const uint16_t *y, const uint16_t *u, const uint16_t *v,
                        int stride_y, int stride_c);

/* jmh_read_qpel: the 16 quarter-pel phase planes of the current reference (test seam for
 *   UnifiedOneForthPix), out[16][H+8][W+8], phase = 4*yfrac + xfrac, 4-sample padding.      */
int  jmh_read_qpel(jmh_ctx *ctx, uint8_t *out);

#ifdef __cplusplus
}
#endif
#endif /* JMHIP_H */
