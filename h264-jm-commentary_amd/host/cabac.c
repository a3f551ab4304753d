/*
 * cabac.c — CABAC slice data (SymbolMode = 1), restating JM lencod's cabac.c (writeMB_typeInfo
 * _CABAC, writeB8_typeInfo_CABAC, writeMVD_CABAC, writeCBP_CABAC, writeCBP_BIT_CABAC, write_and
 * _store_CBP_block_bit, write_significance_map, write_significant_coefficients, writeIntraPred
 * Mode_CABAC, writeCIPredMode_CABAC, writeDquant_CABAC, writeMB_skip_flagInfo_CABAC, writeMB
 * Transform_size_CABAC), biariencode.c (arienco_start_encoding, biari_encode_symbol, biari
 * _encode_symbol_eq_prob, biari_encode_symbol_final, arienco_done_encoding) and context_ini.c
 * (init_contexts with a fixed model) [J] — no file:line exists: /root/reference holds only
 * README.md:1-4.  Arithmetic, binarisations and context selection follow ITU-T
 * H.264 9.3 (9.3.1.1 initialisation, 9.3.2 binarisation, 9.3.3.1 ctxIdx derivation, 9.3.4
 * arithmetic encoding); the initialisation values (m, n) are those of Tables 9-12 .. 9-33 for
 * the I slices and for cabac_init_idc 0, restated from the standard (docs/JM_SEMANTICS.md item
 * 48: parity with JM unpinned, the independent decoder oracle/decoder.c carries its own copy).
 * Scope: frame macroblocks, 4:2:0, 8-bit, one reference (no ref_idx), mb_qp_delta 0, no I_PCM.
 */
#include <stdlib.h>
#include <string.h>
#include "bitstream_int.h"

/* ---- Table 9-44: rangeTabLPS, transIdxLPS -------------------------------------------------- */
static const uint8_t rangeTabLPS[64][4] = {
    {128, 176, 208, 240}, {128, 167, 197, 227}, {128, 158, 187, 216}, {123, 150, 178, 205}, {116, 142, 169, 195},
    {111, 135, 160, 185}, {105, 128, 152, 175}, {100, 122, 144, 166}, {95, 116, 137, 158},  {90, 110, 130, 150},
    {85, 104, 123, 142},  {81, 99, 117, 135},   {77, 94, 111, 128},   {73, 89, 105, 122},   {69, 85, 100, 116},
    {66, 80, 95, 110},    {62, 76, 90, 104},    {59, 72, 86, 99},     {56, 69, 81, 94},     {53, 65, 77, 89},
    {51, 62, 73, 85},     {48, 59, 69, 80},     {46, 56, 66, 76},     {43, 53, 63, 72},     {41, 50, 59, 69},
    {39, 48, 56, 65},     {37, 45, 54, 62},     {35, 43, 51, 59},     {33, 41, 48, 56},     {32, 39, 46, 53},
    {30, 37, 43, 50},     {29, 35, 41, 48},     {27, 33, 39, 45},     {26, 31, 37, 43},     {24, 30, 35, 41},
    {23, 28, 33, 39},     {22, 27, 32, 37},     {21, 26, 30, 35},     {20, 24, 29, 33},     {19, 23, 27, 31},
    {18, 22, 26, 30},     {17, 21, 25, 28},     {16, 20, 23, 27},     {15, 19, 22, 25},     {14, 18, 21, 24},
    {14, 17, 20, 23},     {13, 16, 19, 22},     {12, 15, 18, 21},     {12, 14, 17, 20},     {11, 14, 16, 19},
    {11, 13, 15, 18},     {10, 12, 15, 17},     {10, 12, 14, 16},     {9, 11, 13, 15},      {9, 11, 12, 14},
    {8, 10, 12, 14},      {8, 9, 11, 13},       {7, 9, 11, 12},       {7, 9, 10, 12},       {7, 8, 10, 11},
    {6, 8, 9, 11},        {6, 7, 9, 10},        {6, 7, 8, 9},         {2, 2, 2, 2}};
static const uint8_t transIdxLPS[64] = {
    0,  0,  1,  2,  2,  4,  4,  5,  6,  7,  8,  9,  9,  11, 11, 12, 13, 13, 15, 15, 16, 16,
    18, 18, 19, 19, 21, 21, 22, 22, 23, 24, 24, 25, 26, 26, 27, 27, 28, 29, 29, 30, 30, 30,
    31, 32, 32, 33, 33, 33, 34, 34, 35, 35, 35, 36, 36, 36, 37, 37, 37, 38, 38, 63};

/* ---- Tables 9-12 .. 9-33: (m, n) per ctxIdx, I slices and cabac_init_idc 0 -----------------
 * Only the contexts this scope codes are listed (mb_type / skip / sub_mb_type 0..23, mvd and
 * ref_idx 40..59, mb_qp_delta / intra modes 60..69, cbp / coded_block_flag 73..104, frame
 * significance / last / levels 105..275, transform_size_8x8_flag and the 8x8 frame residual
 * 399..435); the rest stay (0, 0) and are never coded.                                      */
#define NCTX 460
static const int8_t init_I[NCTX][2] = {
    /* 0..10: mb_type (SI prefix, I) */
    [0] = {20, -15}, {2, 54}, {3, 74}, {20, -15}, {2, 54}, {3, 74}, {-28, 127}, {-23, 104}, {-6, 53}, {-1, 54}, {7, 51},
    /* 60..69: mb_qp_delta, intra_chroma_pred_mode, prev_intra_pred_mode_flag, rem_intra_pred_mode */
    [60] = {0, 41}, {0, 63}, {0, 63}, {0, 63}, {-9, 83}, {4, 86}, {0, 97}, {-7, 72}, {13, 41}, {3, 62},
    /* 70..72 mb_field_decoding_flag, 73..84 coded_block_pattern, 85..104 coded_block_flag */
    [70] = {0, 11}, {1, 55}, {0, 69}, {-17, 127}, {-13, 102}, {0, 82}, {-7, 74}, {-21, 107}, {-27, 127}, {-31, 127},
    {-24, 127}, {-18, 95}, {-27, 127}, {-21, 114}, {-30, 127}, {-17, 123}, {-12, 115}, {-16, 122},
    [88] = {-11, 115}, {-12, 63}, {-2, 68}, {-15, 84}, {-13, 104}, {-3, 70}, {-8, 93}, {-10, 90}, {-30, 127}, {-1, 74},
    {-6, 97}, {-7, 91}, {-20, 127}, {-4, 56}, {-5, 82}, {-7, 76}, {-22, 125},
    /* 105..165: significant_coeff_flag (frame) */
    [105] = {-7, 93}, {-11, 87}, {-3, 77}, {-5, 71}, {-4, 63}, {-4, 68}, {-12, 84}, {-7, 62}, {-7, 65}, {8, 61}, {5, 56},
    {-2, 66}, {1, 64}, {0, 61}, {-2, 78}, {1, 50}, {7, 52}, {10, 35}, {0, 44}, {11, 38}, {1, 45}, {0, 46}, {5, 44},
    {31, 17}, {1, 51}, {7, 50}, {28, 19}, {16, 33}, {14, 62}, {-13, 108}, {-15, 100},
    [136] = {-13, 101}, {-13, 91}, {-12, 94}, {-10, 88}, {-16, 84}, {-10, 86}, {-7, 83}, {-13, 87}, {-19, 94}, {1, 70},
    {0, 72}, {-5, 74}, {18, 59}, {-8, 102}, {-15, 100}, {0, 95}, {-4, 75}, {2, 72}, {-11, 75}, {-3, 71}, {15, 46},
    {-13, 69}, {0, 62}, {0, 65}, {21, 37}, {-15, 72}, {9, 57}, {16, 54}, {0, 62}, {12, 72},
    /* 166..226: last_significant_coeff_flag (frame) */
    [166] = {24, 0}, {15, 9}, {8, 25}, {13, 18}, {15, 9}, {13, 19}, {10, 37}, {12, 18}, {6, 29}, {20, 33}, {15, 30},
    {4, 45}, {1, 58}, {0, 62}, {7, 61}, {12, 38}, {11, 45}, {15, 39}, {11, 42}, {13, 44}, {16, 45}, {12, 41}, {10, 49},
    {30, 34}, {18, 42}, {10, 55}, {17, 51}, {17, 46}, {0, 89}, {26, -19}, {22, -17},
    [197] = {26, -17}, {30, -25}, {28, -20}, {33, -23}, {37, -27}, {33, -23}, {40, -28}, {38, -17}, {33, -11}, {40, -15},
    {41, -6}, {38, 1}, {41, 17}, {30, -6}, {27, 3}, {26, 22}, {37, -16}, {35, -4}, {38, -8}, {38, -3}, {37, 3}, {38, 5},
    {42, 0}, {35, 16}, {39, 22}, {14, 48}, {27, 37}, {21, 60}, {12, 68}, {2, 97},
    /* 227..275: coeff_abs_level_minus1 */
    [227] = {-3, 71}, {-6, 42}, {-5, 50}, {-3, 54}, {-2, 62}, {0, 58}, {1, 63}, {-2, 72}, {-1, 74}, {-9, 91}, {-5, 67},
    {-5, 27}, {-3, 39}, {-2, 44}, {0, 46}, {-16, 64}, {-8, 68}, {-10, 78}, {-6, 77}, {-10, 86}, {-12, 92}, {-15, 55},
    {-10, 60}, {-6, 62}, {-4, 65},
    [252] = {-12, 73}, {-8, 76}, {-7, 80}, {-9, 88}, {-17, 110}, {-11, 97}, {-20, 84}, {-11, 79}, {-6, 73}, {-4, 74},
    {-13, 86}, {-13, 96}, {-11, 97}, {-19, 117}, {-8, 78}, {-5, 33}, {-4, 48}, {-2, 53}, {-3, 62}, {-13, 71}, {-10, 79},
    {-12, 86}, {-13, 90}, {-14, 97},
    /* 399..401 transform_size_8x8_flag, 402..416 / 417..425 / 426..435: 8x8 residual (frame) */
    [399] = {31, 21}, {31, 31}, {25, 50},
    [402] = {-17, 120}, {-20, 112}, {-18, 114}, {-11, 85}, {-15, 92}, {-14, 89}, {-26, 71}, {-15, 81}, {-14, 80}, {0, 68},
    {-14, 70}, {-24, 56}, {-23, 68}, {-24, 50}, {-11, 74},
    [417] = {23, -13}, {26, -13}, {40, -15}, {49, -14}, {44, 3}, {45, 6}, {44, 34}, {33, 54}, {19, 82},
    [426] = {-3, 75}, {-1, 23}, {1, 34}, {1, 43}, {0, 54}, {-2, 55}, {0, 61}, {1, 64}, {0, 68}, {-9, 92},
};
static const int8_t init_P0[NCTX][2] = {
    [0] = {20, -15}, {2, 54}, {3, 74}, {20, -15}, {2, 54}, {3, 74}, {-28, 127}, {-23, 104}, {-6, 53}, {-1, 54}, {7, 51},
    /* 11..13 mb_skip_flag, 14..20 mb_type (P prefix / suffix), 21..23 sub_mb_type */
    [11] = {23, 33}, {23, 2}, {21, 0}, {1, 9}, {0, 49}, {-37, 118}, {5, 57}, {-13, 78}, {-11, 65}, {1, 62}, {12, 49},
    {-4, 73}, {17, 50},
    /* 24..39 (B slices) */
    [24] = {18, 64}, {9, 43}, {29, 0}, {26, 67}, {16, 90}, {9, 104}, {-46, 127}, {-20, 104}, {1, 67}, {-13, 78},
    {-11, 65}, {1, 62}, {-6, 86}, {-17, 95}, {-6, 61}, {9, 45},
    /* 40..46 mvd_l0[][][0], 47..53 mvd_l0[][][1], 54..59 ref_idx */
    [40] = {-3, 69}, {-6, 81}, {-11, 96}, {6, 55}, {7, 67}, {-5, 86}, {2, 88}, {0, 58}, {-3, 76}, {-10, 94}, {5, 54},
    {4, 69}, {-3, 81}, {0, 88},
    [54] = {-7, 67}, {-5, 74}, {-4, 74}, {-5, 80}, {-7, 72}, {1, 58},
    [60] = {0, 41}, {0, 63}, {0, 63}, {0, 63}, {-9, 83}, {4, 86}, {0, 97}, {-7, 72}, {13, 41}, {3, 62},
    [70] = {0, 45}, {-4, 78}, {-3, 96}, {-27, 126}, {-28, 98}, {-25, 101}, {-23, 67}, {-28, 82}, {-20, 94}, {-16, 83},
    {-22, 110}, {-21, 91}, {-18, 102}, {-13, 93}, {-29, 127}, {-7, 92}, {-5, 89}, {-7, 96}, {-13, 108}, {-3, 46},
    {-1, 65}, {-1, 57}, {-9, 93}, {-3, 74}, {-9, 92}, {-8, 87}, {-23, 126}, {5, 54}, {6, 60}, {6, 59}, {6, 69},
    {-1, 48}, {0, 68}, {-4, 69}, {-8, 88},
    [105] = {-2, 85}, {-6, 78}, {-1, 75}, {-7, 77}, {2, 54}, {5, 50}, {-3, 68}, {1, 50}, {6, 42}, {-4, 81}, {1, 63},
    {-4, 70}, {0, 67}, {2, 57}, {-2, 76}, {11, 35}, {4, 64}, {1, 61}, {11, 35}, {18, 25}, {12, 24}, {13, 29}, {13, 36},
    {-10, 93}, {-7, 73}, {-2, 73}, {13, 46}, {9, 49}, {-7, 100}, {9, 53}, {2, 53}, {5, 53}, {-2, 61}, {0, 56}, {0, 56},
    {-13, 63}, {-5, 60}, {-1, 62}, {4, 57}, {-6, 69}, {4, 57}, {14, 39}, {4, 51}, {13, 68}, {3, 64}, {1, 61}, {9, 63},
    {7, 50}, {16, 39}, {5, 44}, {4, 52}, {11, 48}, {-5, 60}, {-1, 59}, {0, 59}, {22, 33}, {5, 44}, {14, 43}, {-1, 78},
    {0, 60}, {9, 69},
    [166] = {11, 28}, {2, 40}, {3, 44}, {0, 49}, {0, 46}, {2, 44}, {2, 51}, {0, 47}, {4, 39}, {2, 62}, {6, 46}, {0, 54},
    {3, 54}, {2, 58}, {4, 63}, {6, 51}, {6, 57}, {7, 53}, {6, 52}, {6, 55}, {11, 45}, {14, 36}, {8, 53}, {-1, 82},
    {7, 55}, {-3, 78}, {15, 46}, {22, 31}, {-1, 84}, {25, 7}, {30, -7}, {28, 3}, {28, 4}, {32, 0}, {34, -1}, {30, 6},
    {30, 6}, {32, 9}, {31, 19}, {26, 27}, {26, 30}, {37, 20}, {28, 34}, {17, 70}, {1, 67}, {5, 59}, {9, 67}, {16, 30},
    {18, 32}, {18, 35}, {22, 29}, {24, 31}, {23, 38}, {18, 43}, {20, 41}, {11, 63}, {9, 59}, {9, 64}, {-1, 94},
    {-2, 89}, {-9, 108},
    [227] = {-6, 76}, {-2, 44}, {0, 45}, {0, 52}, {-3, 64}, {-2, 59}, {-4, 70}, {-4, 75}, {-8, 82}, {-17, 102}, {-9, 77},
    {3, 24}, {0, 42}, {0, 48}, {0, 55}, {-6, 59}, {-7, 71}, {-12, 83}, {-11, 87}, {-30, 119}, {1, 58}, {-3, 29},
    {-1, 36}, {1, 38}, {2, 43}, {-6, 55}, {0, 58}, {0, 64}, {-3, 74}, {-10, 90}, {0, 70}, {-4, 29}, {5, 31}, {7, 42},
    {1, 59}, {-2, 58}, {-3, 72}, {-3, 81}, {-11, 97}, {0, 58}, {8, 5}, {10, 14}, {14, 18}, {13, 27}, {2, 40}, {0, 58},
    {-3, 70}, {-6, 79}, {-8, 85},
    [399] = {12, 40}, {11, 51}, {14, 59},
    [402] = {-4, 79}, {-7, 71}, {-5, 69}, {-9, 70}, {-8, 66}, {-10, 68}, {-19, 73}, {-12, 69}, {-16, 70}, {-15, 67},
    {-20, 62}, {-19, 70}, {-16, 66}, {-22, 65}, {-20, 63},
    [417] = {9, -2}, {26, -9}, {33, -9}, {39, -7}, {41, -2}, {45, 3}, {49, 9}, {45, 27}, {36, 59},
    [426] = {-6, 66}, {-7, 35}, {-7, 42}, {-8, 45}, {-5, 48}, {-12, 56}, {-6, 60}, {-5, 62}, {-8, 66}, {-8, 76},
};

/* accessors for tests (tests/test_cabac.py checks the table shapes) */
const int8_t *jm_cabac_init_table(int slice_i) { return slice_i ? &init_I[0][0] : &init_P0[0][0]; }
const uint8_t *jm_cabac_range_lps(void) { return &rangeTabLPS[0][0]; }
const uint8_t *jm_cabac_trans_lps(void) { return transIdxLPS; }

/* ---- per-macroblock state the context selection reads (9.3.3.1.1) ----------------------- */
enum { K_SKIP = 0, K_INTER = 1, K_INXN = 2, K_I16 = 3 };
typedef struct {
    uint8_t kind;       /* K_*                                                                  */
    uint8_t cbp;        /* coded_block_pattern (luma | chroma << 4), 0 for P_Skip              */
    uint8_t t8;         /* transform_size_8x8_flag                                              */
    uint8_t cmode;      /* intra_chroma_pred_mode (0 for inter macroblocks)                     */
    uint8_t cbf_dc;     /* coded_block_flag: bit 0 luma DC (I16), bit 1 Cb DC, bit 2 Cr DC       */
    uint8_t cbf_cac[2]; /* chroma AC blocks (2x2 raster)                                        */
    uint16_t cbf_l;     /* luma 4x4 blocks (4x4 raster): the 4x4 block's flag (I16: its AC block),
                           8x8 transform: the 8x8 block's cbp bit (its flag is inferred, 7.4.5.3.3) */
} cmb;

struct jm_cabac {
    const jm_seq *s;
    jm_bits *b;
    uint32_t low, range;
    int outstanding, first;
    long bins, pic_bins;
    long nbits;         /* arienco_bits_written: one per renormalisation step and bypass bin     */
    long mb_bits;       /* of the last macroblock (mb_skip_flag .. residual, no end_of_slice_flag) */
    uint8_t state[NCTX], mps[NCTX];
    cmb *mb;
    int16_t *mvd;       /* per 4x4 of the picture [2]: mvd_l0 of the partition covering it      */
    int pending_eos;    /* a macroblock of the slice awaits its end_of_slice_flag = 0          */
};

jm_cabac *jm_cabac_new(const jm_seq *s) {
    jm_cabac *c = calloc(1, sizeof(*c));
    if (!c) return NULL;
    c->s = s;
    c->mb = calloc((size_t)s->mbw * s->mbh, sizeof(cmb));
    c->mvd = calloc((size_t)s->mbw * s->mbh * 32, sizeof(int16_t));
    if (!c->mb || !c->mvd) { jm_cabac_free(c); return NULL; }
    return c;
}
void jm_cabac_free(jm_cabac *c) {
    if (!c) return;
    free(c->mb); free(c->mvd); free(c);
}

/* ---- arithmetic encoder (9.3.4.2 .. 9.3.4.5) -------------------------------------------- */
static void put_bit(jm_cabac *c, int bit) {
    if (c->first) c->first = 0;
    else jm_put(c->b, (uint32_t)bit, 1);
    for (; c->outstanding > 0; c->outstanding--) jm_put(c->b, (uint32_t)(1 - bit), 1);
}
static void renorm(jm_cabac *c) {
    while (c->range < 256) {
        if (c->low < 256) put_bit(c, 0);
        else if (c->low >= 512) { c->low -= 512; put_bit(c, 1); }
        else { c->low -= 256; c->outstanding++; }
        c->range <<= 1;
        c->low <<= 1;
        c->nbits++;
    }
}
static void enc(jm_cabac *c, int ctx, int bin) {
    const uint32_t lps = rangeTabLPS[c->state[ctx]][(c->range >> 6) & 3];
    c->range -= lps;
    if (bin != c->mps[ctx]) {
        c->low += c->range;
        c->range = lps;
        if (c->state[ctx] == 0) c->mps[ctx] ^= 1;
        c->state[ctx] = transIdxLPS[c->state[ctx]];
    } else if (c->state[ctx] < 62) c->state[ctx]++;
    renorm(c);
    c->bins++;
}
static void enc_bypass(jm_cabac *c, int bin) {
    c->low <<= 1;
    if (bin) c->low += c->range;
    if (c->low >= 1024) { put_bit(c, 1); c->low -= 1024; }
    else if (c->low < 512) put_bit(c, 0);
    else { c->low -= 512; c->outstanding++; }
    c->bins++;
    c->nbits++;
}
static void enc_terminate(jm_cabac *c, int bin) {
    c->range -= 2;
    c->bins++;
    if (!bin) { renorm(c); return; }
    c->low += c->range;
    c->range = 2;                                    /* EncodeFlush (9.3.4.5) */
    renorm(c);
    put_bit(c, (c->low >> 9) & 1);
    jm_put(c->b, ((c->low >> 7) & 3) | 1, 2);        /* its last bit is the rbsp_stop_one_bit */
}

void jm_cabac_slice_start(jm_cabac *c, jm_bits *b, int slice_type, int qp) {
    c->b = b;
    while (b->nacc) jm_put(b, 1, 1);                 /* cabac_alignment_one_bit */
    const int8_t (*t)[2] = slice_type == JMH_I_SLICE ? init_I : init_P0;
    const int q = qp < 0 ? 0 : qp > 51 ? 51 : qp;
    for (int i = 0; i < NCTX; i++) {                /* 9.3.1.1 */
        int pre = ((t[i][0] * q) >> 4) + t[i][1];
        pre = pre < 1 ? 1 : pre > 126 ? 126 : pre;
        if (pre <= 63) { c->state[i] = (uint8_t)(63 - pre); c->mps[i] = 0; }
        else { c->state[i] = (uint8_t)(pre - 64); c->mps[i] = 1; }
    }
    c->low = 0; c->range = 510; c->first = 1; c->outstanding = 0;   /* 9.3.4.1 */
    c->bins = 0;
    c->pending_eos = 0;
}

long jm_cabac_slice_end(jm_cabac *c) {
    if (c->pending_eos) enc_terminate(c, 1);        /* end_of_slice_flag = 1 + flush */
    c->pending_eos = 0;
    while (c->b->nacc) jm_put(c->b, 0, 1);           /* rbsp_alignment_zero_bit */
    c->pic_bins += c->bins;
    return c->bins;
}

/* ---- binarisations ----------------------------------------------------------------------- */
/* UEGk suffix (9.3.2.3): Exp-Golomb of order k in bypass bins */
static void exp_golomb_bypass(jm_cabac *c, unsigned v, int k) {
    for (;;) {
        if (v >= (1u << k)) { enc_bypass(c, 1); v -= 1u << k; k++; }
        else {
            enc_bypass(c, 0);
            while (k--) enc_bypass(c, (v >> k) & 1);
            return;
        }
    }
}

/* neighbouring macroblocks A (left) and B (above): index or -1 when not available */
static int nb_mb(const wctx *w, int mx, int my, int left) {
    int x = left ? mx - 1 : mx, y = left ? my : my - 1;
    return jm_w_mb_ok(w, x, y) ? y * w->s->mbw + x : -1;
}

/* coded_block_flag condTermFlagN (9.3.3.1.1.9) of a neighbouring block in macroblock n (-1: not
 * available); cur_intra: the current macroblock is intra; coded: that block exists in n (the
 * transBlockN derivation), flag: its coded_block_flag */
static int cbf_term(int n, int cur_intra, int coded, int flag) {
    if (n < 0) return cur_intra;
    return coded ? flag : 0;
}
/* the same for luma 4x4 / I16 AC blocks: 4x4 (x4, y4) of macroblock n */
static int cbf_luma_term(const jm_cabac *c, int n, int cur_intra, int x4, int y4) {
    if (n < 0) return cur_intra;
    const cmb *m = &c->mb[n];
    if (m->kind == K_SKIP) return 0;
    const int b8 = (y4 >> 1) * 2 + (x4 >> 1);
    if (!((m->cbp >> b8) & 1)) return 0;
    return (m->cbf_l >> (y4 * 4 + x4)) & 1;
}

/* residual_block_cabac (7.3.5.3.3) with the ctxIdx of 9.3.3.1.3: coef[0..n) in scan order;
 * cat 0..4 (ctxBlockCat), 5 = luma 8x8; cbf_ctx < 0: no coded_block_flag (8x8). Returns the
 * coded_block_flag. */
static const uint8_t sig8x8_inc[63] = {0,  1,  2,  3,  4,  5,  5,  4,  4,  3,  3,  4,  4,  4,  5,  5,  4,  4,  4,  4,  3,
                                      3,  6,  7,  7,  7,  8,  9,  10, 9,  8,  7,  7,  6,  11, 12, 13, 11, 6,  7,  8,  9,
                                      14, 10, 9,  8,  6,  11, 12, 13, 11, 6,  9,  14, 10, 9,  11, 12, 13, 11, 14, 10, 12};
static const uint8_t last8x8_inc[63] = {0, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 2, 2, 2, 2, 2, 2,
                                       2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 3, 3, 3, 3, 3, 3, 3, 3, 4, 4, 4, 4,
                                       4, 4, 4, 4, 5, 5, 5, 5, 6, 6, 6, 6, 7, 7, 7, 7, 8, 8, 8};
static int residual_block(jm_cabac *c, const int16_t *coef, int n, int cat, int cbf_ctx) {
    static const int sig_off[5] = {0, 15, 29, 44, 47}, abs_off[5] = {0, 10, 20, 30, 39};
    int last = -1;
    for (int i = 0; i < n; i++) if (coef[i]) last = i;
    const int cbf = last >= 0;
    if (cbf_ctx >= 0) enc(c, cbf_ctx, cbf);
    if (!cbf) return 0;
    const int sig_base = cat == 5 ? 402 : 105 + sig_off[cat], last_base = cat == 5 ? 417 : 166 + sig_off[cat];
    const int abs_base = cat == 5 ? 426 : 227 + abs_off[cat];
    for (int i = 0; i < n - 1; i++) {           /* significance map */
        const int si = cat == 5 ? sig8x8_inc[i] : cat == 3 ? (i < 2 ? i : 2) : i;
        const int li = cat == 5 ? last8x8_inc[i] : cat == 3 ? (i < 2 ? i : 2) : i;
        enc(c, sig_base + si, coef[i] != 0);
        if (coef[i]) {
            enc(c, last_base + li, i == last);
            if (i == last) break;
        }
    }
    int eq1 = 0, gt1 = 0;
    for (int i = last; i >= 0; i--) {           /* levels, reverse scan order */
        if (!coef[i]) continue;
        const int a = coef[i] < 0 ? -coef[i] : coef[i], v = a - 1;
        enc(c, abs_base + (gt1 ? 0 : (1 + eq1 < 4 ? 1 + eq1 : 4)), v > 0);
        if (v > 0) {
            const int ctx = abs_base + 5 + (gt1 < 4 - (cat == 3) ? gt1 : 4 - (cat == 3));
            int k = 1;
            for (; k < v && k < 14; k++) enc(c, ctx, 1);
            if (v < 14) enc(c, ctx, 0);
            else exp_golomb_bypass(c, (unsigned)(v - 14), 0);
        }
        enc_bypass(c, coef[i] < 0);
        if (a == 1) eq1++;
        else gt1++;
    }
    return 1;
}

/* mvd_l0 (9.3.2.3 UEG3, signed, uCoff 9; ctxIdxInc of bin 0 from absMvdComp of A + B) */
static void write_mvd_comp(jm_cabac *c, int v, int sum, int comp) {
    const int base = comp ? 47 : 40, a = v < 0 ? -v : v;
    enc(c, base + (sum < 3 ? 0 : sum > 32 ? 2 : 1), a != 0);
    if (a) {
        static const int inc[9] = {0, 3, 4, 5, 6, 6, 6, 6, 6};
        int k = 1;
        for (; k < a && k < 9; k++) enc(c, base + inc[k], 1);
        if (a < 9) enc(c, base + inc[k], 0);
        else exp_golomb_bypass(c, (unsigned)(a - 9), 3);
        enc_bypass(c, v < 0);
    }
}
static void write_mvd(jm_cabac *c, wctx *w, int mx, int my, int ma, int mb, const jmh_mb_result *r, int bx, int by,
                      int bw, int bh) {
    int p[2];
    jm_w_mvp(w, mx, my, bx, by, bw, bh, p);
    const int W4 = w->s->mbw * 4, k = (by >> 2) * 4 + (bx >> 2);
    const int gx = mx * 4 + (bx >> 2), gy = my * 4 + (by >> 2);
    /* neighbouring partitions A (x - 1, y) and B (x, y - 1) of the partition's top-left sample;
       unavailable, P_Skip or intra give 0 (their mvd entries are 0) */
    const int ia = bx > 0 ? gy * W4 + gx - 1 : (ma >= 0 ? gy * W4 + gx - 1 : -1);
    const int ib = by > 0 ? (gy - 1) * W4 + gx : (mb >= 0 ? (gy - 1) * W4 + gx : -1);
    const int d[2] = {r->mv[k][0] - p[0], r->mv[k][1] - p[1]};
    for (int comp = 0; comp < 2; comp++) {
        const int sa = ia >= 0 ? abs(c->mvd[2 * ia + comp]) : 0, sb = ib >= 0 ? abs(c->mvd[2 * ib + comp]) : 0;
        write_mvd_comp(c, d[comp], sa + sb, comp);
    }
    for (int y = gy; y < gy + (bh >> 2); y++)
        for (int x = gx; x < gx + (bw >> 2); x++) { c->mvd[2 * (y * W4 + x)] = (int16_t)d[0]; c->mvd[2 * (y * W4 + x) + 1] = (int16_t)d[1]; }
}

/* 8x8 levels in zig-zag order from jmh_mb_result's CAVLC interleave (luma[4x4 j][k] = lev[4k + j]) */
static void level8x8(const jmh_mb_result *r, int b8, int16_t *out) {
    for (int j = 0; j < 4; j++) {
        const int x4 = (b8 & 1) * 2 + (j & 1), y4 = (b8 >> 1) * 2 + (j >> 1);
        for (int k = 0; k < 16; k++) out[4 * k + j] = r->luma[y4 * 4 + x4][k];
    }
}

static void write_mb_body(jm_cabac *c, wctx *w, int mx, int my, const jmh_mb_result *r, int slice_p);
void jm_cabac_write_mb(jm_cabac *c, wctx *w, int mx, int my, const jmh_mb_result *r, int slice_p) {
    if (c->pending_eos) enc_terminate(c, 0);         /* end_of_slice_flag of the previous MB */
    c->pending_eos = 1;
    const long nb0 = c->nbits;
    write_mb_body(c, w, mx, my, r, slice_p);
    c->mb_bits = c->nbits - nb0;
}
long jm_cabac_mb_bits(const jm_cabac *c) { return c->mb_bits; }

static void write_mb_body(jm_cabac *c, wctx *w, int mx, int my, const jmh_mb_result *r, int slice_p) {
    const jm_seq *s = w->s;
    const int a = my * s->mbw + mx, W4 = s->mbw * 4;
    const int na = nb_mb(w, mx, my, 1), nbb = nb_mb(w, mx, my, 0);
    const cmb *A = na >= 0 ? &c->mb[na] : NULL, *B = nbb >= 0 ? &c->mb[nbb] : NULL;
    cmb *m = &c->mb[a];
    memset(m, 0, sizeof(*m));
    for (int k = 0; k < 16; k++) {
        const int i = (my * 4 + (k >> 2)) * W4 + mx * 4 + (k & 3);
        c->mvd[2 * i] = c->mvd[2 * i + 1] = 0;
    }
    const int mbt = r->mb_type;
    const int skip = slice_p && mbt == JMH_PSKIP;
    if (slice_p)                                      /* mb_skip_flag: ctxIdx 11..13 */
        enc(c, 11 + (A && A->kind != K_SKIP) + (B && B->kind != K_SKIP), skip);
    jm_w_mark_mb(w, mx, my, r, skip);
    if (skip) { m->kind = K_SKIP; return; }

    const int is_i8 = mbt == JMH_I8MB, is_nxn = mbt == JMH_I4MB || is_i8, is_i16 = mbt == JMH_I16MB;
    const int intra = is_nxn || is_i16, cbp = r->cbp, cbpl = cbp & 15, cbpc = cbp >> 4;
    m->kind = is_i16 ? K_I16 : is_nxn ? K_INXN : K_INTER;
    m->cbp = (uint8_t)cbp;
    /* ---- mb_type (9.3.2.5, Tables 9-36 / 9-37; ctxIdx 3..10 in I slices, 14..20 in P) ---- */
    if (intra) {
        int base;                                     /* ctxIdx of the I-type bins 0, 2, 3, 4/5, 6 */
        if (slice_p) { enc(c, 14, 1); base = 17; }    /* prefix: intra in a P slice */
        else base = 3;
        const int inc0 = slice_p ? 0 : (A && A->kind != K_INXN) + (B && B->kind != K_INXN);
        enc(c, base + inc0, is_i16);
        if (is_i16) {
            enc_terminate(c, 0);                      /* not I_PCM */
            enc(c, base + 1 + !slice_p * 2, cbpl != 0);
            enc(c, base + 2 + !slice_p * 2, cbpc != 0);
            if (cbpc) enc(c, base + (slice_p ? 2 : 5), cbpc == 2);
            enc(c, base + (slice_p ? 3 : 6), r->i16mode >> 1);
            enc(c, base + (slice_p ? 3 : 7), r->i16mode & 1);
        }
    } else {
        /* P_L0_16x16 000, P_L0_L0_16x8 011, P_L0_L0_8x16 010, P_8x8 001 */
        const int b1 = mbt == JMH_P16x8 || mbt == JMH_P8x16;
        const int b2 = mbt == JMH_P16x8 || mbt == JMH_P8x8;
        enc(c, 14, 0);
        enc(c, 15, b1);
        enc(c, 16 + b1, b2);
    }
    if (mbt == JMH_P8x8)                               /* sub_mb_type: 8x8 1, 8x4 00, 4x8 011, 4x4 010 */
        for (int i = 0; i < 4; i++) {
            const int sm = r->b8mode[i];
            enc(c, 21, sm == JMH_SMB8x8);
            if (sm == JMH_SMB8x8) continue;
            enc(c, 22, sm != JMH_SMB8x4);
            if (sm != JMH_SMB8x4) enc(c, 23, sm == JMH_SMB4x8);
        }
    /* transform_size_8x8_flag of I_NxN (ctxIdx 399..401) */
    if (is_nxn && s->transform_8x8_mode) {
        enc(c, 399 + (A && A->t8) + (B && B->t8), is_i8);
        m->t8 = (uint8_t)is_i8;
    }
    if (is_nxn) {                                     /* prev_intra_pred_mode_flag / rem (68, 69) */
        for (int blk = 0; blk < 16; blk += is_i8 ? 4 : 1) {
            const int x4 = ((blk >> 2) & 1) * 2 + (blk & 1), y4 = (blk >> 3) * 2 + ((blk >> 1) & 1);
            const int pred = jm_w_mpm(w, mx, my, x4, y4), mode = r->ipred[y4 * 4 + x4];
            enc(c, 68, mode == pred);
            if (mode != pred) {
                const int rem = mode < pred ? mode : mode - 1;
                for (int bit = 0; bit < 3; bit++) enc(c, 69, (rem >> bit) & 1);   /* FL, LSB first */
            }
        }
    }
    if (intra) {                                      /* intra_chroma_pred_mode: TU cMax 3 (64..67) */
        const int cm = r->c_ipred_mode;
        const int inc = (A && (A->kind == K_INXN || A->kind == K_I16) && A->cmode) +
                        (B && (B->kind == K_INXN || B->kind == K_I16) && B->cmode);
        enc(c, 64 + inc, cm > 0);
        if (cm > 0) { enc(c, 67, cm > 1); if (cm > 1) enc(c, 67, cm > 2); }
        m->cmode = (uint8_t)cm;
    } else if (mbt == JMH_P16x16) write_mvd(c, w, mx, my, na, nbb, r, 0, 0, 16, 16);
    else if (mbt == JMH_P16x8) { write_mvd(c, w, mx, my, na, nbb, r, 0, 0, 16, 8); write_mvd(c, w, mx, my, na, nbb, r, 0, 8, 16, 8); }
    else if (mbt == JMH_P8x16) { write_mvd(c, w, mx, my, na, nbb, r, 0, 0, 8, 16); write_mvd(c, w, mx, my, na, nbb, r, 8, 0, 8, 16); }
    else {
        for (int i = 0; i < 4; i++) {
            const int ox = (i & 1) * 8, oy = (i >> 1) * 8, sm = r->b8mode[i];
            const int sw = (sm == 4 || sm == 5) ? 8 : 4, sh = (sm == 4 || sm == 6) ? 8 : 4;
            for (int y = 0; y < 8; y += sh)
                for (int x = 0; x < 8; x += sw) write_mvd(c, w, mx, my, na, nbb, r, ox + x, oy + y, sw, sh);
        }
    }
    /* ---- coded_block_pattern: luma FL 4 bins (73..76), chroma TU cMax 2 (77..84) ---------- */
    if (!is_i16) {
        for (int b8 = 0; b8 < 4; b8++) {
            const int bx = b8 & 1, by = b8 >> 1;
            int ta, tb;       /* condTermFlagN: 1 when the neighbouring 8x8 block codes no luma */
            if (bx) ta = !((cbpl >> (b8 - 1)) & 1);
            else ta = A ? !((A->cbp >> (b8 + 1)) & 1) : 0;
            if (by) tb = !((cbpl >> (b8 - 2)) & 1);
            else tb = B ? !((B->cbp >> (b8 + 2)) & 1) : 0;
            enc(c, 73 + ta + 2 * tb, (cbpl >> b8) & 1);
        }
        const int ca = A ? A->cbp >> 4 : 0, cb = B ? B->cbp >> 4 : 0;
        enc(c, 77 + (ca != 0) + 2 * (cb != 0), cbpc != 0);
        if (cbpc) enc(c, 81 + (ca == 2) + 2 * (cb == 2), cbpc == 2);
    }
    /* transform_size_8x8_flag of inter macroblocks: luma coded, no sub-8x8 partitions (7.3.5) */
    if (!intra && cbpl && s->transform_8x8_mode &&
        (mbt != JMH_P8x8 || (r->b8mode[0] == 4 && r->b8mode[1] == 4 && r->b8mode[2] == 4 && r->b8mode[3] == 4))) {
        enc(c, 399 + (A && A->t8) + (B && B->t8), r->transform_8x8 != 0);
        m->t8 = r->transform_8x8 != 0;
    }
    if (!(cbp > 0 || is_i16)) return;
    enc(c, 60, 0);                                   /* mb_qp_delta = 0 (the previous one is 0 too) */
    /* ---- residual (7.3.5.3) ---- */
    if (is_i16) {                                    /* Intra16x16DCLevel: ctxBlockCat 0 */
        const int ta = A ? (A->kind == K_I16 ? A->cbf_dc & 1 : 0) : 1;
        const int tb = B ? (B->kind == K_I16 ? B->cbf_dc & 1 : 0) : 1;
        m->cbf_dc |= (uint8_t)residual_block(c, r->luma_dc, 16, 0, 85 + ta + 2 * tb);
    }
    for (int b8 = 0; b8 < 4; b8++) {
        if (!((cbpl >> b8) & 1)) continue;
        if (m->t8) {                                 /* 8x8 block (cat 5), flag inferred 1 */
            int16_t lv[64];
            level8x8(r, b8, lv);
            residual_block(c, lv, 64, 5, -1);
            const int x4 = (b8 & 1) * 2, y4 = (b8 >> 1) * 2;
            m->cbf_l |= (uint16_t)(0x33 << (y4 * 4 + x4));
            continue;
        }
        for (int i4 = 0; i4 < 4; i4++) {
            const int x4 = (b8 & 1) * 2 + (i4 & 1), y4 = (b8 >> 1) * 2 + (i4 >> 1);
            const int ta = x4 ? (m->cbf_l >> (y4 * 4 + x4 - 1)) & 1 : cbf_luma_term(c, na, intra, 3, y4);
            const int tb = y4 ? (m->cbf_l >> ((y4 - 1) * 4 + x4)) & 1 : cbf_luma_term(c, nbb, intra, x4, 3);
            const int16_t *lv = r->luma[y4 * 4 + x4];
            const int f = is_i16 ? residual_block(c, lv + 1, 15, 1, 85 + 4 + ta + 2 * tb)
                                 : residual_block(c, lv, 16, 2, 85 + 8 + ta + 2 * tb);
            m->cbf_l |= (uint16_t)(f << (y4 * 4 + x4));
        }
    }
    if (cbpc) {                                       /* chroma DC (cat 3) */
        for (int uv = 0; uv < 2; uv++) {
            const int ta = cbf_term(na, intra, A && (A->cbp >> 4) != 0, A ? (A->cbf_dc >> (1 + uv)) & 1 : 0);
            const int tb = cbf_term(nbb, intra, B && (B->cbp >> 4) != 0, B ? (B->cbf_dc >> (1 + uv)) & 1 : 0);
            m->cbf_dc |= (uint8_t)(residual_block(c, r->chroma_dc[uv], 4, 3, 85 + 12 + ta + 2 * tb) << (1 + uv));
        }
    }
    if (cbpc == 2) {                                  /* chroma AC (cat 4) */
        for (int uv = 0; uv < 2; uv++)
            for (int k = 0; k < 4; k++) {
                const int bx = k & 1, by = k >> 1;
                const int ta = bx ? (m->cbf_cac[uv] >> (k - 1)) & 1
                                  : cbf_term(na, intra, A && (A->cbp >> 4) == 2, A ? (A->cbf_cac[uv] >> (k + 1)) & 1 : 0);
                const int tb = by ? (m->cbf_cac[uv] >> (k - 2)) & 1
                                  : cbf_term(nbb, intra, B && (B->cbp >> 4) == 2, B ? (B->cbf_cac[uv] >> (k + 2)) & 1 : 0);
                const int f = residual_block(c, r->chroma_ac[uv][k] + 1, 15, 4, 85 + 16 + ta + 2 * tb);
                m->cbf_cac[uv] |= (uint8_t)(f << k);
            }
    }
}
