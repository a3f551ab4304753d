/*
 * bitstream.c — Annex B NAL packaging, SPS/PPS/slice header and the CAVLC macroblock layer.
 * Restates JM 8.6 nalu.c / parset.c › GenerateSeq_parameter_set_rbsp / GeneratePic_parameter_set
 * _rbsp, header.c › SliceHeader, macroblock.c › writeMBLayer / writeMotionInfo2NAL /
 * writeCBPandLumaCoeff / writeChromaCoeff, vlc.c › ue_v / se_v / writeSyntaxElement_NumCoeff
 * TrailingOnes / _TotalZeros / _Run / _Level_VLC1 / _Level_VLCN [J].  Syntax and tables follow
 * ITU-T H.264 7.3 and 9.1/9.2 (Tables 9-4, 9-5, 9-7..9-10).  Header field choices: see
 * docs/JM_SEMANTICS.md §Headers.
 */
#include <stdlib.h>
#include <string.h>
#include "bitstream_int.h"

/* ---- bit writer ---------------------------------------------------------------------- */
void jm_bits_init(jm_bits *b) { memset(b, 0, sizeof(*b)); }
void jm_bits_free(jm_bits *b) { free(b->buf); memset(b, 0, sizeof(*b)); }
static void put_byte(jm_bits *b, uint8_t v) {
    if (b->len >= b->cap) {
        b->cap = b->cap ? 2 * b->cap : 4096;
        b->buf = (uint8_t *)realloc(b->buf, b->cap);
    }
    b->buf[b->len++] = v;
}
void jm_put(jm_bits *b, uint32_t val, int n) {
    for (int i = n - 1; i >= 0; i--) {
        b->acc = (b->acc << 1) | ((val >> i) & 1);
        if (++b->nacc == 8) { put_byte(b, (uint8_t)b->acc); b->acc = 0; b->nacc = 0; }
    }
}
void jm_put_ue(jm_bits *b, uint32_t v) {
    uint32_t x = v + 1;
    int len = 31 - __builtin_clz(x);
    jm_put(b, 0, len);
    jm_put(b, x, len + 1);
}
void jm_put_se(jm_bits *b, int32_t v) { jm_put_ue(b, v > 0 ? (uint32_t)(2 * v - 1) : (uint32_t)(-2 * v)); }
void jm_trailing_bits(jm_bits *b) {
    jm_put(b, 1, 1);
    while (b->nacc) jm_put(b, 0, 1);
}
void jm_bits_align_flush(jm_bits *b) { while (b->nacc) jm_put(b, 0, 1); }
void jm_bits_append(jm_bits *b, const jm_bits *src) { for (long i = 0; i < src->len; i++) put_byte(b, src->buf[i]); }

void jm_write_nal(jm_bits *out, int nal_ref_idc, int nal_type, const jm_bits *rbsp) {
    put_byte(out, 0); put_byte(out, 0); put_byte(out, 0); put_byte(out, 1);
    put_byte(out, (uint8_t)((nal_ref_idc << 5) | nal_type));
    int zeros = 0;
    for (long i = 0; i < rbsp->len; i++) {
        uint8_t v = rbsp->buf[i];
        if (zeros >= 2 && v <= 3) { put_byte(out, 3); zeros = 0; }
        put_byte(out, v);
        zeros = v == 0 ? zeros + 1 : 0;
    }
}

/* ---- parameter sets ------------------------------------------------------------------- */
void jm_write_sps(jm_bits *b, const jm_seq *s) {
    jm_put(b, s->profile_idc, 8);
    jm_put(b, 0, 8);                         /* constraint_set0..3 = 0, reserved_zero_4bits */
    jm_put(b, s->level_idc, 8);
    jm_put_ue(b, 0);                         /* seq_parameter_set_id */
    if (s->profile_idc >= 100) {             /* High / High 10: 4:2:0, no scaling matrices */
        const int bd = s->bit_depth > 8 ? s->bit_depth : 8;
        jm_put_ue(b, 1);                     /* chroma_format_idc */
        jm_put_ue(b, bd - 8);                /* bit_depth_luma_minus8 */
        jm_put_ue(b, bd - 8);                /* bit_depth_chroma_minus8 */
        jm_put(b, 0, 1);                     /* qpprime_y_zero_transform_bypass_flag */
        jm_put(b, 0, 1);                     /* seq_scaling_matrix_present_flag */
    }
    jm_put_ue(b, s->log2_max_frame_num - 4);
    jm_put_ue(b, 0);                         /* pic_order_cnt_type */
    jm_put_ue(b, s->log2_max_poc_lsb - 4);
    jm_put_ue(b, s->num_ref_frames);
    jm_put(b, 0, 1);                         /* gaps_in_frame_num_value_allowed_flag */
    jm_put_ue(b, s->mbw - 1);
    jm_put_ue(b, s->mbh - 1);
    jm_put(b, 1, 1);                         /* frame_mbs_only_flag */
    jm_put(b, 1, 1);                         /* direct_8x8_inference_flag */
    int crop = s->disp_w != s->width || s->disp_h != s->height;
    jm_put(b, crop, 1);
    if (crop) {
        jm_put_ue(b, 0);
        jm_put_ue(b, (s->width - s->disp_w) / 2);
        jm_put_ue(b, 0);
        jm_put_ue(b, (s->height - s->disp_h) / 2);
    }
    jm_put(b, 0, 1);                         /* vui_parameters_present_flag */
    jm_trailing_bits(b);
}

void jm_write_pps(jm_bits *b, const jm_seq *s) {
    jm_put_ue(b, 0);                         /* pic_parameter_set_id */
    jm_put_ue(b, 0);                         /* seq_parameter_set_id */
    jm_put(b, s->entropy_coding ? 1 : 0, 1); /* entropy_coding_mode_flag (0 CAVLC, 1 CABAC) */
    jm_put(b, 0, 1);                         /* pic_order_present_flag */
    jm_put_ue(b, 0);                         /* num_slice_groups_minus1 */
    jm_put_ue(b, s->num_ref_frames - 1);     /* num_ref_idx_l0_active_minus1 */
    jm_put_ue(b, 0);                         /* num_ref_idx_l1_active_minus1 */
    jm_put(b, 0, 1);                         /* weighted_pred_flag */
    jm_put(b, 0, 2);                         /* weighted_bipred_idc */
    jm_put_se(b, 0);                         /* pic_init_qp_minus26 */
    jm_put_se(b, 0);                         /* pic_init_qs_minus26 */
    jm_put_se(b, s->chroma_qp_offset);
    jm_put(b, s->lf_params_flag, 1);         /* deblocking_filter_control_present_flag */
    jm_put(b, s->constrained_intra, 1);
    jm_put(b, 0, 1);                         /* redundant_pic_cnt_present_flag */
    if (s->profile_idc >= 100) {             /* PPS range extension (High) */
        jm_put(b, s->transform_8x8_mode ? 1 : 0, 1);   /* transform_8x8_mode_flag */
        jm_put(b, 0, 1);                     /* pic_scaling_matrix_present_flag */
        jm_put_se(b, s->chroma_qp_offset);   /* second_chroma_qp_index_offset */
    }
    jm_trailing_bits(b);
}

/* ---- CAVLC tables (H.264 Tables 9-5, 9-7, 9-8, 9-9a, 9-10) ---------------------------- */
static const uint8_t ct_len[3][4][17] = {
    {{1, 6, 8, 9, 10, 11, 13, 13, 13, 14, 14, 15, 15, 16, 16, 16, 16},
     {0, 2, 6, 8, 9, 10, 11, 13, 13, 14, 14, 15, 15, 15, 16, 16, 16},
     {0, 0, 3, 7, 8, 9, 10, 11, 13, 13, 14, 14, 15, 15, 16, 16, 16},
     {0, 0, 0, 5, 6, 7, 8, 9, 10, 11, 13, 14, 14, 15, 15, 16, 16}},
    {{2, 6, 6, 7, 8, 8, 9, 11, 11, 12, 12, 12, 13, 13, 13, 14, 14},
     {0, 2, 5, 6, 6, 7, 8, 9, 11, 11, 12, 12, 13, 13, 14, 14, 14},
     {0, 0, 3, 6, 6, 7, 8, 9, 11, 11, 12, 12, 13, 13, 13, 14, 14},
     {0, 0, 0, 4, 4, 5, 6, 6, 7, 9, 11, 11, 12, 13, 13, 13, 14}},
    {{4, 6, 6, 6, 7, 7, 7, 7, 8, 8, 9, 9, 9, 10, 10, 10, 10},
     {0, 4, 5, 5, 5, 5, 6, 6, 7, 8, 8, 9, 9, 9, 10, 10, 10},
     {0, 0, 4, 5, 5, 5, 6, 6, 7, 7, 8, 8, 9, 9, 10, 10, 10},
     {0, 0, 0, 4, 4, 4, 4, 4, 5, 6, 7, 8, 8, 9, 10, 10, 10}}};
static const uint8_t ct_code[3][4][17] = {
    {{1, 5, 7, 7, 7, 7, 15, 11, 8, 15, 11, 15, 11, 15, 11, 7, 4},
     {0, 1, 4, 6, 6, 6, 6, 14, 10, 14, 10, 14, 10, 1, 14, 10, 6},
     {0, 0, 1, 5, 5, 5, 5, 5, 13, 9, 13, 9, 13, 9, 13, 9, 5},
     {0, 0, 0, 3, 3, 4, 4, 4, 4, 4, 12, 12, 8, 12, 8, 12, 8}},
    {{3, 11, 7, 7, 7, 4, 7, 15, 11, 15, 11, 8, 15, 11, 7, 9, 7},
     {0, 2, 7, 10, 6, 6, 6, 6, 14, 10, 14, 10, 14, 10, 11, 8, 6},
     {0, 0, 3, 9, 5, 5, 5, 5, 13, 9, 13, 9, 13, 9, 6, 10, 5},
     {0, 0, 0, 5, 4, 6, 8, 4, 4, 4, 12, 8, 12, 12, 8, 1, 4}},
    {{15, 15, 11, 8, 15, 11, 9, 8, 15, 11, 15, 11, 8, 13, 9, 5, 1},
     {0, 14, 15, 12, 10, 8, 14, 10, 14, 14, 10, 14, 10, 7, 12, 8, 4},
     {0, 0, 13, 14, 11, 9, 13, 9, 13, 10, 13, 9, 13, 9, 11, 7, 3},
     {0, 0, 0, 12, 11, 10, 9, 8, 13, 12, 12, 12, 8, 12, 10, 6, 2}}};
static const uint8_t ctdc_len[4][5] = {{2, 6, 6, 6, 6}, {0, 1, 6, 7, 8}, {0, 0, 3, 7, 8}, {0, 0, 0, 6, 7}};
static const uint8_t ctdc_code[4][5] = {{1, 7, 4, 3, 2}, {0, 1, 6, 3, 3}, {0, 0, 1, 2, 2}, {0, 0, 0, 5, 0}};
static const uint8_t tz_len[15][16] = {
    {1, 3, 3, 4, 4, 5, 5, 6, 6, 7, 7, 8, 8, 9, 9, 9}, {3, 3, 3, 3, 3, 4, 4, 4, 4, 5, 5, 6, 6, 6, 6},
    {4, 3, 3, 3, 4, 4, 3, 3, 4, 5, 5, 6, 5, 6},       {5, 3, 4, 4, 3, 3, 3, 4, 3, 4, 5, 5, 5},
    {4, 4, 4, 3, 3, 3, 3, 3, 4, 5, 4, 5},             {6, 5, 3, 3, 3, 3, 3, 3, 4, 3, 6},
    {6, 5, 3, 3, 3, 2, 3, 4, 3, 6},                   {6, 4, 5, 3, 2, 2, 3, 3, 6},
    {6, 6, 4, 2, 2, 3, 2, 5},                         {5, 5, 3, 2, 2, 2, 4},
    {4, 4, 3, 3, 1, 3},                               {4, 4, 2, 1, 3},
    {3, 3, 1, 2},                                     {2, 2, 1},
    {1, 1}};
static const uint8_t tz_code[15][16] = {
    {1, 3, 2, 3, 2, 3, 2, 3, 2, 3, 2, 3, 2, 3, 2, 1}, {7, 6, 5, 4, 3, 5, 4, 3, 2, 3, 2, 3, 2, 1, 0},
    {5, 7, 6, 5, 4, 3, 4, 3, 2, 3, 2, 1, 1, 0},       {3, 7, 5, 4, 6, 5, 4, 3, 3, 2, 2, 1, 0},
    {5, 4, 3, 7, 6, 5, 4, 3, 2, 1, 1, 0},             {1, 1, 7, 6, 5, 4, 3, 2, 1, 1, 0},
    {1, 1, 5, 4, 3, 3, 2, 1, 1, 0},                   {1, 1, 1, 3, 3, 2, 2, 1, 0},
    {1, 0, 1, 3, 2, 1, 1, 1},                         {1, 0, 1, 3, 2, 1, 1},
    {0, 1, 1, 2, 1, 3},                               {0, 1, 1, 1, 1},
    {0, 1, 1, 1},                                     {0, 1, 1},
    {0, 1}};
static const uint8_t tzdc_len[3][4] = {{1, 2, 3, 3}, {1, 2, 2, 0}, {1, 1, 0, 0}};
static const uint8_t tzdc_code[3][4] = {{1, 1, 1, 0}, {1, 1, 0, 0}, {1, 0, 0, 0}};
static const uint8_t rb_len[7][15] = {
    {1, 1}, {1, 2, 2}, {2, 2, 2, 2}, {2, 2, 2, 3, 3}, {2, 2, 3, 3, 3, 3}, {2, 3, 3, 3, 3, 3, 3},
    {3, 3, 3, 3, 3, 3, 3, 4, 5, 6, 7, 8, 9, 10, 11}};
static const uint8_t rb_code[7][15] = {
    {1, 0}, {1, 1, 0}, {3, 2, 1, 0}, {3, 2, 1, 1, 0}, {3, 2, 3, 2, 1, 0}, {3, 0, 1, 3, 2, 5, 4},
    {7, 6, 5, 4, 3, 2, 1, 1, 1, 1, 1, 1, 1, 1, 1}};
/* Table 9-4 (ChromaArrayType 1): coded_block_pattern -> codeNum, intra (I_NxN) and inter */
static const uint8_t cbp_intra_code[48] = {
    3, 29, 30, 17, 31, 18, 37, 8, 32, 38, 19, 9, 20, 10, 11, 2, 16, 33, 34, 21, 35, 22, 39, 4,
    36, 40, 23, 5, 24, 6, 7, 1, 41, 42, 43, 25, 44, 26, 46, 12, 45, 47, 27, 13, 28, 14, 15, 0};
static const uint8_t cbp_inter_code[48] = {
    0, 2, 3, 7, 4, 8, 17, 13, 5, 18, 9, 14, 10, 15, 16, 11, 1, 32, 33, 36, 34, 37, 44, 40,
    35, 45, 38, 41, 39, 42, 43, 19, 6, 24, 25, 20, 26, 21, 46, 28, 27, 47, 22, 29, 23, 30, 31, 12};

/* residual_block_cavlc (7.3.5.3.2 / 9.2); coeffs[0..n) in scan order; nC = -1: chroma DC.
 * Returns TotalCoeff. */
static int write_residual_block(jm_bits *b, const int16_t *coeffs, int n, int nC) {
    int pos[16], lev[16], tc = 0;
    for (int i = n - 1; i >= 0; i--)          /* reverse scan order */
        if (coeffs[i]) { pos[tc] = i; lev[tc] = coeffs[i]; tc++; }
    int t1 = 0;
    while (t1 < tc && t1 < 3 && (lev[t1] == 1 || lev[t1] == -1)) t1++;
    if (nC == -1) jm_put(b, ctdc_code[t1][tc], ctdc_len[t1][tc]);
    else if (nC >= 8) jm_put(b, tc == 0 ? 3 : (uint32_t)(((tc - 1) << 2) | t1), 6);
    else {
        int t = nC < 2 ? 0 : nC < 4 ? 1 : 2;
        jm_put(b, ct_code[t][t1][tc], ct_len[t][t1][tc]);
    }
    if (!tc) return 0;
    int sl = (tc > 10 && t1 < 3) ? 1 : 0;
    for (int i = 0; i < tc; i++) {
        if (i < t1) { jm_put(b, lev[i] < 0, 1); continue; }
        int v = lev[i];
        int code = v > 0 ? 2 * v - 2 : -2 * v - 1;
        if (i == t1 && t1 < 3) code -= 2;
        if (sl == 0 && code < 14) jm_put(b, 1, code + 1);
        else if (sl == 0 && code < 30) { jm_put(b, 1, 15); jm_put(b, code - 14, 4); }
        else if (sl > 0 && code < (15 << sl)) { jm_put(b, 1, (code >> sl) + 1); jm_put(b, code & ((1 << sl) - 1), sl); }
        else {   /* level_prefix >= 15 (9.2.2.1): prefix 15 takes 12 suffix bits, each further one 1 more */
            int rest = code - (sl == 0 ? 30 : 15 << sl), prefix = 15;
            while (rest >= (1 << (prefix - 3))) { rest -= 1 << (prefix - 3); prefix++; }
            jm_put(b, 0, prefix); jm_put(b, 1, 1); jm_put(b, (uint32_t)rest, prefix - 3);
        }
        if (sl == 0) sl = 1;
        int a = v < 0 ? -v : v;
        if (a > (3 << (sl - 1)) && sl < 6) sl++;
    }
    int total_zeros = pos[0] + 1 - tc;          /* pos[0] = highest nonzero index */
    if (tc < n) {
        if (nC == -1) jm_put(b, tzdc_code[tc - 1][total_zeros], tzdc_len[tc - 1][total_zeros]);
        else jm_put(b, tz_code[tc - 1][total_zeros], tz_len[tc - 1][total_zeros]);
    }
    int zl = total_zeros;
    for (int i = 0; i < tc - 1 && zl > 0; i++) {
        int run = pos[i] - pos[i + 1] - 1;
        int t = zl > 6 ? 6 : zl - 1;
        jm_put(b, rb_code[t][run], rb_len[t][run]);
        zl -= run;
    }
    return tc;
}

/* ---- slice ----------------------------------------------------------------------------- */
int jm_w_mb_ok(const wctx *w, int mx, int my) {
    return mx >= 0 && my >= 0 && mx < w->s->mbw && my < w->s->mbh && w->written[my * w->s->mbw + mx] == w->stamp;
}
#define mb_ok jm_w_mb_ok
/* neighbour 4x4 in luma pixels relative to MB (mx,my): returns availability + 4x4 index */
static int nb(const wctx *w, int mx, int my, int xN, int yN, int *idx, int cur_ok) {
    int tx, ty;
    if (yN > 15) return 0;
    if (xN < 0) { tx = mx - 1; ty = yN < 0 ? my - 1 : my; }
    else if (xN <= 15) { tx = mx; ty = yN < 0 ? my - 1 : my; }
    else { if (yN >= 0) return 0; tx = mx + 1; ty = my - 1; }
    if (tx == mx && ty == my) { if (!cur_ok) return 0; }
    else if (!mb_ok(w, tx, ty)) return 0;
    int W4 = w->s->mbw * 4;
    *idx = ((16 * my + yN) >> 2) * W4 + ((16 * mx + xN) >> 2);
    return 1;
}

/* normative MVP (8.4.1.3) of the partition at (bx,by) size bw x bh (pixels, MB relative);
 * the current MB's mv/ref entries must already hold its final values. */
void jm_w_mvp(const wctx *w, int mx, int my, int bx, int by, int bw, int bh, int *p) {
    int ia = 0, ib = 0, ic = 0, id = 0;
    int aa = nb(w, mx, my, bx - 1, by, &ia, 1), ab = nb(w, mx, my, bx, by - 1, &ib, 1);
    int ac = nb(w, mx, my, bx + bw, by - 1, &ic, 1), ad = nb(w, mx, my, bx - 1, by - 1, &id, 1);
    if (by > 0) {                         /* C inside the MB, not yet decoded */
        if (bx < 8) { if (by == 8) { if (bw == 16) ac = 0; } else if (bx + bw == 8) ac = 0; }
        else if (bx + bw == 16) ac = 0;
    }
    if (!ac) { ac = ad; ic = id; }
    int rA = aa ? w->ref[ia] : -1, rB = ab ? w->ref[ib] : -1, rC = ac ? w->ref[ic] : -1;
    int type = 0;
    if (rA == 0 && rB != 0 && rC != 0) type = 1;
    else if (rA != 0 && rB == 0 && rC != 0) type = 2;
    else if (rA != 0 && rB != 0 && rC == 0) type = 3;
    if (bw == 8 && bh == 16) { if (bx == 0) { if (rA == 0) type = 1; } else if (rC == 0) type = 3; }
    else if (bw == 16 && bh == 8) { if (by == 0) { if (rB == 0) type = 2; } else if (rA == 0) type = 1; }
    for (int hv = 0; hv < 2; hv++) {
        int a = aa ? w->mv[2 * ia + hv] : 0, b = ab ? w->mv[2 * ib + hv] : 0, c = ac ? w->mv[2 * ic + hv] : 0;
        int v;
        if (type == 1) v = a;
        else if (type == 2) v = b;
        else if (type == 3) v = c;
        else if (!ab && !ac) v = a;
        else { int mn = a < b ? a : b; mn = mn < c ? mn : c; int mxv = a > b ? a : b; mxv = mxv > c ? mxv : c; v = a + b + c - mn - mxv; }
        p[hv] = v;
    }
}

static void put_mvd(jm_bits *b, const wctx *w, int mx, int my, const jmh_mb_result *r, int bx, int by, int bw, int bh) {
    int p[2];
    jm_w_mvp(w, mx, my, bx, by, bw, bh, p);
    int k = (by >> 2) * 4 + (bx >> 2);
    jm_put_se(b, r->mv[k][0] - p[0]);
    jm_put_se(b, r->mv[k][1] - p[1]);
}

/* nC for a luma (comp 0) or chroma (comp 1/2) 4x4 block at 4x4 coords (x4,y4) in the MB */
static int calc_nc(const wctx *w, int mx, int my, int comp, int x4, int y4, const uint8_t *cur_tc) {
    int lim = comp ? 1 : 3, base = comp ? 16 + 4 * (comp - 1) : 0, st = comp ? 2 : 4;
    int na = 0, nb_ = 0, aa = 0, ab = 0;
    if (x4 > 0) { aa = 1; na = cur_tc[base + y4 * st + x4 - 1]; }
    else if (mb_ok(w, mx - 1, my)) { aa = 1; na = w->tc[(my * w->s->mbw + mx - 1) * 24 + base + y4 * st + lim]; }
    if (y4 > 0) { ab = 1; nb_ = cur_tc[base + (y4 - 1) * st + x4]; }
    else if (mb_ok(w, mx, my - 1)) { ab = 1; nb_ = w->tc[((my - 1) * w->s->mbw + mx) * 24 + base + lim * st + x4]; }
    if (aa && ab) return (na + nb_ + 1) >> 1;
    if (aa) return na;
    if (ab) return nb_;
    return 0;
}

/* predIntra4x4PredMode / predIntra8x8PredMode (8.3.1.1 / 8.3.2.1): DC unless both the left and
 * the upper neighbour exist (and, with constrained_intra_pred_flag, are intra); a neighbour that
 * is not I_NxN counts as DC (2) */
int jm_w_mpm(const wctx *w, int mx, int my, int x4, int y4) {
    int ia = 0, ib = 0;
    int aa = nb(w, mx, my, 4 * x4 - 1, 4 * y4, &ia, 1), ab = nb(w, mx, my, 4 * x4, 4 * y4 - 1, &ib, 1);
    if (!aa || !ab) return 2;
    if (w->s->constrained_intra && (w->ref[ia] >= 0 || w->ref[ib] >= 0)) return 2;
    int ma = w->ipm[ia] < 0 ? 2 : w->ipm[ia], mb = w->ipm[ib] < 0 ? 2 : w->ipm[ib];
    return ma < mb ? ma : mb;
}

void jm_w_mark_mb(wctx *w, int mx, int my, const jmh_mb_result *r, int skip) {
    int mbt = r->mb_type, W4 = w->s->mbw * 4;
    int is_i4 = !skip && (mbt == JMH_I4MB || mbt == JMH_I8MB), is_intra = !skip && (is_i4 || mbt == JMH_I16MB);
    for (int k = 0; k < 16; k++) {
        int a = (my * 4 + (k >> 2)) * W4 + mx * 4 + (k & 3);
        w->mv[2 * a] = is_intra ? 0 : r->mv[k][0];
        w->mv[2 * a + 1] = is_intra ? 0 : r->mv[k][1];
        w->ref[a] = is_intra ? -1 : 0;
        w->ipm[a] = is_i4 ? r->ipred[k] : -1;
    }
    w->written[my * w->s->mbw + mx] = w->stamp;
}

static int write_mb(jm_bits *b, wctx *w, int mx, int my, const jmh_mb_result *r, int slice_p) {
    int mbt = r->mb_type, cbp = r->cbp;
    int is_i8 = mbt == JMH_I8MB, is_i4 = mbt == JMH_I4MB || is_i8, is_i16 = mbt == JMH_I16MB;
    int is_intra = is_i4 || is_i16, t8 = r->transform_8x8;   /* is_i4: I_NxN (4x4 or 8x8) */
    int cbpl = cbp & 15, cbpc = cbp >> 4;
    /* mark the MB's final motion / intra data (needed by its own MVP / MPM derivations) */
    jm_w_mark_mb(w, mx, my, r, 0);
    int ue_type;
    if (is_i16) {
        int t = 1 + r->i16mode + 4 * cbpc + (cbpl ? 12 : 0);
        ue_type = slice_p ? 5 + t : t;
    } else if (is_i4) ue_type = slice_p ? 5 : 0;
    else if (mbt == JMH_P8x8) ue_type = 3;
    else ue_type = mbt - 1;
    jm_put_ue(b, ue_type);
    if (mbt == JMH_P8x8)
        for (int i = 0; i < 4; i++) jm_put_ue(b, r->b8mode[i] - 4);
    if (is_i4 && w->s->transform_8x8_mode) jm_put(b, is_i8, 1);   /* transform_size_8x8_flag */
    if (is_i4) {   /* prev_intra4x4_pred_mode_flag / rem (16 blocks), or the 8x8 ones (4 blocks) */
        for (int blk = 0; blk < 16; blk += is_i8 ? 4 : 1) {
            int x4 = ((blk >> 2) & 1) * 2 + (blk & 1), y4 = (blk >> 3) * 2 + ((blk >> 1) & 1);
            int pred = jm_w_mpm(w, mx, my, x4, y4), m = r->ipred[y4 * 4 + x4];
            if (m == pred) jm_put(b, 1, 1);
            else { jm_put(b, 0, 1); jm_put(b, m < pred ? m : m - 1, 3); }
        }
    }
    if (is_intra) jm_put_ue(b, r->c_ipred_mode);
    if (!is_intra) {
        if (mbt == JMH_P16x16) put_mvd(b, w, mx, my, r, 0, 0, 16, 16);
        else if (mbt == JMH_P16x8) { put_mvd(b, w, mx, my, r, 0, 0, 16, 8); put_mvd(b, w, mx, my, r, 0, 8, 16, 8); }
        else if (mbt == JMH_P8x16) { put_mvd(b, w, mx, my, r, 0, 0, 8, 16); put_mvd(b, w, mx, my, r, 8, 0, 8, 16); }
        else {
            for (int i = 0; i < 4; i++) {
                int ox = (i & 1) * 8, oy = (i >> 1) * 8, sm = r->b8mode[i];
                int sw = (sm == 4 || sm == 5) ? 8 : 4, sh = (sm == 4 || sm == 6) ? 8 : 4;
                for (int y = 0; y < 8; y += sh)
                    for (int x = 0; x < 8; x += sw) put_mvd(b, w, mx, my, r, ox + x, oy + y, sw, sh);
            }
        }
    }
    if (!is_i16) jm_put_ue(b, is_i4 ? cbp_intra_code[cbp] : cbp_inter_code[cbp]);
    /* transform_size_8x8_flag of inter MBs: luma coded, no sub-8x8 partitions (7.3.5) */
    if (!is_intra && cbpl && w->s->transform_8x8_mode &&
        (mbt != JMH_P8x8 || (r->b8mode[0] == 4 && r->b8mode[1] == 4 && r->b8mode[2] == 4 && r->b8mode[3] == 4)))
        jm_put(b, t8, 1);
    uint8_t *tc = w->tc + (size_t)(my * w->s->mbw + mx) * 24;
    memset(tc, 0, 24);
    if (cbp > 0 || is_i16) {
        jm_put_se(b, 0);                    /* mb_qp_delta */
        if (is_i16) write_residual_block(b, r->luma_dc, 16, calc_nc(w, mx, my, 0, 0, 0, tc));
        for (int blk = 0; blk < 16; blk++) {
            int b8 = blk >> 2;
            int x4 = (b8 & 1) * 2 + (blk & 1), y4 = (b8 >> 1) * 2 + ((blk >> 1) & 1);
            if (!(cbpl & (1 << b8))) continue;
            int nC = calc_nc(w, mx, my, 0, x4, y4, tc);
            const int16_t *lv = r->luma[y4 * 4 + x4];
            tc[y4 * 4 + x4] = (uint8_t)(is_i16 ? write_residual_block(b, lv + 1, 15, nC)
                                                : write_residual_block(b, lv, 16, nC));
        }
        if (cbpc) {
            write_residual_block(b, r->chroma_dc[0], 4, -1);
            write_residual_block(b, r->chroma_dc[1], 4, -1);
        }
        if (cbpc == 2)
            for (int uv = 0; uv < 2; uv++)
                for (int k = 0; k < 4; k++) {
                    int nC = calc_nc(w, mx, my, 1 + uv, k & 1, k >> 1, tc);
                    tc[16 + 4 * uv + k] = (uint8_t)write_residual_block(b, r->chroma_ac[uv][k] + 1, 15, nC);
                }
    }
    return 0;
}

/* the slice writer, one macroblock at a time (JM 8.6 slice.c › encode_one_slice calls
 * macroblock.c › write_one_macroblock after encode_one_macroblock for every MB [J]) */
struct jm_slice_writer {
    jm_bits *b;
    wctx w;
    int skip_run, slice_p;
    int open;                  /* header written and buffers allocated */
    jm_cabac *cab;             /* SymbolMode 1: the CABAC coder (NULL: CAVLC)                 */
    long bins;                 /* CABAC bins of the picture's slices                           */
    long rate_checked, rate_bad;   /* RDOptimization 1: macroblocks whose RD rate was checked    */
};

/* slice_header (7.3.3) */
static void write_slice_header(jm_bits *b, const jm_seq *s, const jm_slice *sl) {
    jm_put_ue(b, sl->first_mb);                       /* first_mb_in_slice */
    jm_put_ue(b, sl->slice_type);                     /* 0 = P, 2 = I            */
    jm_put_ue(b, 0);                                  /* pic_parameter_set_id    */
    jm_put(b, sl->frame_num & ((1 << s->log2_max_frame_num) - 1), s->log2_max_frame_num);
    if (sl->idr) jm_put_ue(b, sl->idr_pic_id);
    jm_put(b, sl->poc_lsb & ((1 << s->log2_max_poc_lsb) - 1), s->log2_max_poc_lsb);
    if (sl->slice_type == JMH_P_SLICE) {
        jm_put(b, 0, 1);                              /* num_ref_idx_active_override_flag */
        jm_put(b, 0, 1);                              /* ref_pic_list_reordering_flag_l0  */
    }
    if (sl->idr) { jm_put(b, 0, 1); jm_put(b, 0, 1); } /* no_output_of_prior_pics, long_term */
    else jm_put(b, 0, 1);                             /* adaptive_ref_pic_marking_mode_flag */
    if (s->entropy_coding && sl->slice_type != JMH_I_SLICE)
        jm_put_ue(b, s->cabac_init_idc);              /* cabac_init_idc (FixedModelNumber) */
    jm_put_se(b, sl->qp - 26);                        /* slice_qp_delta */
    if (s->lf_params_flag) {
        jm_put_ue(b, s->lf_disable);
        /* LoopFilterAlphaC0Offset / LoopFilterBetaOffset are the div2 values [J] */
        if (s->lf_disable != 1) { jm_put_se(b, s->lf_alpha); jm_put_se(b, s->lf_beta); }
    }
}

jm_slice_writer *jm_slice_begin(jm_bits *b, const jm_seq *s, const jm_slice *sl) {
    jm_slice_writer *sw = calloc(1, sizeof(*sw));
    if (!sw) return NULL;
    write_slice_header(b, s, sl);
    /* slice_data (7.3.4); neighbour state of the picture (entries are read only for MBs that
       carry the current slice's stamp, so no clearing between slices) */
    int nmb = s->mbw * s->mbh, W4 = s->mbw * 4, H4 = s->mbh * 4;
    wctx *w = &sw->w;
    sw->b = b;
    w->s = s;
    w->mv = malloc((size_t)W4 * H4 * 2 * sizeof(int16_t));
    w->ref = malloc((size_t)W4 * H4);
    w->ipm = malloc((size_t)W4 * H4);
    w->written = calloc(nmb, sizeof(uint32_t));
    w->tc = malloc((size_t)nmb * 24);
    if (!w->mv || !w->ref || !w->ipm || !w->written || !w->tc) { jm_slice_end(sw); return NULL; }
    w->stamp = 1;
    sw->slice_p = sl->slice_type == JMH_P_SLICE;
    sw->open = 1;
    if (s->entropy_coding) {
        if (!(sw->cab = jm_cabac_new(s))) { sw->open = 0; jm_slice_end(sw); return NULL; }
        jm_cabac_slice_start(sw->cab, b, sl->slice_type, sl->qp);
    }
    return sw;
}

static void close_slice_data(jm_slice_writer *sw) {
    if (sw->cab) { sw->bins += jm_cabac_slice_end(sw->cab); return; }   /* ends with the stop bit */
    if (sw->slice_p && sw->skip_run) jm_put_ue(sw->b, sw->skip_run);
    sw->skip_run = 0;
    jm_trailing_bits(sw->b);
}

void jm_slice_restart(jm_slice_writer *sw, jm_bits *b, const jm_slice *sl) {
    close_slice_data(sw);
    write_slice_header(b, sw->w.s, sl);
    sw->b = b;
    sw->w.stamp++;
    sw->slice_p = sl->slice_type == JMH_P_SLICE;
    if (sw->cab) jm_cabac_slice_start(sw->cab, b, sl->slice_type, sl->qp);
}

void jm_slice_write_mb(jm_slice_writer *sw, int a, const jmh_mb_result *r) {
    wctx *w = &sw->w;
    const jm_seq *s = w->s;
    int mx = a % s->mbw, my = a / s->mbw, W4 = s->mbw * 4;
    if (sw->cab) {
        jm_cabac_write_mb(sw->cab, w, mx, my, r, sw->slice_p);
        if (s->rdo) {   /* the backend's RD rate of the chosen candidate == the bits written for it */
            sw->rate_checked++;
            sw->rate_bad += jm_cabac_mb_bits(sw->cab) != r->min_cost;
        }
        return;
    }
    if (sw->slice_p && r->mb_type == JMH_PSKIP) {
        for (int k = 0; k < 16; k++) {
            int i = (my * 4 + (k >> 2)) * W4 + mx * 4 + (k & 3);
            w->mv[2 * i] = r->mv[k][0]; w->mv[2 * i + 1] = r->mv[k][1];
            w->ref[i] = 0; w->ipm[i] = -1;
        }
        w->written[a] = w->stamp;
        memset(w->tc + (size_t)a * 24, 0, 24);
        sw->skip_run++;
        if (s->rdo) {   /* nothing written yet -- except the run itself at the picture's last MB (item 64(a)) */
            long expect = 0;
            if (a == s->mbw * s->mbh - 1) for (unsigned v = (unsigned)sw->skip_run + 1u; v; v >>= 1) expect += 2;   /* ue */
            if (expect) expect--;
            sw->rate_checked++;
            sw->rate_bad += r->min_cost != expect;
        }
        return;
    }
    const long bit0 = 8 * sw->b->len + sw->b->nacc;
    if (sw->slice_p) { jm_put_ue(sw->b, sw->skip_run); sw->skip_run = 0; }
    write_mb(sw->b, w, mx, my, r, sw->slice_p);
    if (s->rdo) {   /* the backend's CAVLC RD rate of the chosen candidate == the bits written for it */
        sw->rate_checked++;
        sw->rate_bad += 8 * sw->b->len + sw->b->nacc - bit0 != r->min_cost;
    }
}

void jm_slice_rate_check(const jm_slice_writer *sw, long *checked, long *bad) {
    *checked = sw ? sw->rate_checked : 0;
    *bad = sw ? sw->rate_bad : 0;
}

long jm_slice_end(jm_slice_writer *sw) {
    if (!sw) return 0;
    if (sw->open) close_slice_data(sw);
    const long bins = sw->bins;
    jm_cabac_free(sw->cab);
    free(sw->w.mv); free(sw->w.ref); free(sw->w.ipm); free(sw->w.written); free(sw->w.tc);
    free(sw);
    return bins;
}

int jm_write_slice(jm_bits *b, const jm_seq *s, const jm_slice *sl, const jmh_mb_result *const *res) {
    jm_slice_writer *sw = jm_slice_begin(b, s, sl);
    if (!sw) return JMH_E_OOM;
    for (int a = 0; a < s->mbw * s->mbh; a++) jm_slice_write_mb(sw, a, res[a]);
    jm_slice_end(sw);
    return 0;
}
