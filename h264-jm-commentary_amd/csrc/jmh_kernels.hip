// jmh_kernels.hip — hand-written CDNA4 (gfx950) kernels of the JM lencod hot path.
//
//  k_interp      UnifiedOneForthPix [J] / H.264 8.4.2.2.1: 16 quarter-pel phase planes of the
//                reference (HBM-bound; one thread per padded integer position, all 16 phases).
//  k_mb_encode   encode_one_macroblock [J] (RDO off) for every macroblock of one wavefront
//                diagonal (mbx + 2*mby == diag): one 256-thread workgroup per macroblock.
//                  - SetupFastFullPelSearch: 80x80 reference window staged in LDS, the
//                    16 x (2R+1)^2 table of 4x4 SADs built with v_sad_u8 on v_alignbyte'd dwords
//                    and kept in LDS (135 KB at R = 32 -> one workgroup per CU);
//                  - FastFullPelBlockMotionSearch: argmin of (cost<<13 | spiral order) keys,
//                    wave shuffle + LDS min reduction (strict '<' + JM tie order preserved);
//                  - SubPelBlockMotionSearch: 9 half + 8 quarter candidates x 4x4 sub-blocks
//                    evaluated in parallel (Hadamard SATD), JM candidate order resolved serially;
//                  - Intra4x4 / Intra16x16 decisions, luma/chroma residual coding
//                    (dct_luma / dct_luma_16x16 / dct_chroma) with JM's coefficient-cost rules.
//  k_sad_table / k_tq4x4   unit seams (jmh_ffs_sad_table / jmh_tq4x4_batch).
//
// The wavefront order preserves JM's raster-order semantics exactly: an MB depends only on its
// left, top-left, top and top-right neighbours, all on earlier diagonals (earlier launches).
// Reference citations: JM 8.6 function names [J]; /root/reference holds README.md:1-4 only.
#include "jmh_device.h"

__constant__ int c_quant[6][16] = {
    {13107, 8066, 13107, 8066, 8066, 5243, 8066, 5243, 13107, 8066, 13107, 8066, 8066, 5243, 8066, 5243},
    {11916, 7490, 11916, 7490, 7490, 4660, 7490, 4660, 11916, 7490, 11916, 7490, 7490, 4660, 7490, 4660},
    {10082, 6554, 10082, 6554, 6554, 4194, 6554, 4194, 10082, 6554, 10082, 6554, 6554, 4194, 6554, 4194},
    {9362, 5825, 9362, 5825, 5825, 3647, 5825, 3647, 9362, 5825, 9362, 5825, 5825, 3647, 5825, 3647},
    {8192, 5243, 8192, 5243, 5243, 3355, 5243, 3355, 8192, 5243, 8192, 5243, 5243, 3355, 5243, 3355},
    {7282, 4559, 7282, 4559, 4559, 2893, 4559, 2893, 7282, 4559, 7282, 4559, 4559, 2893, 4559, 2893}};
__constant__ int c_dequant[6][16] = {
    {10, 13, 10, 13, 13, 16, 13, 16, 10, 13, 10, 13, 13, 16, 13, 16},
    {11, 14, 11, 14, 14, 18, 14, 18, 11, 14, 11, 14, 14, 18, 14, 18},
    {13, 16, 13, 16, 16, 20, 16, 20, 13, 16, 13, 16, 16, 20, 16, 20},
    {14, 18, 14, 18, 18, 23, 18, 23, 14, 18, 14, 18, 18, 23, 18, 23},
    {16, 20, 16, 20, 20, 25, 20, 25, 16, 20, 16, 20, 20, 25, 20, 25},
    {18, 23, 18, 23, 23, 29, 23, 29, 18, 23, 18, 23, 23, 29, 23, 29}};
__constant__ int c_scan[16] = {0, 1, 4, 8, 5, 2, 3, 6, 9, 12, 13, 10, 7, 11, 14, 15};
__constant__ int c_coeff_cost[16] = {3, 2, 2, 1, 1, 1, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
__constant__ int c_qpc[52] = {0,  1,  2,  3,  4,  5,  6,  7,  8,  9,  10, 11, 12, 13, 14, 15, 16, 17,
                              18, 19, 20, 21, 22, 23, 24, 25, 26, 27, 28, 29, 29, 30, 31, 32, 32, 33,
                              34, 34, 35, 35, 36, 36, 37, 37, 37, 38, 38, 38, 39, 39, 39, 39};
__constant__ int c_blc[8][2] = {{16, 16}, {16, 16}, {16, 8}, {8, 16}, {8, 8}, {8, 4}, {4, 8}, {4, 4}};
// sub-pel candidate offsets = spiral entries 0..8
__constant__ int c_sp9[9][2] = {{0, 0}, {0, -1}, {0, 1}, {-1, -1}, {1, -1}, {-1, 0}, {1, 0}, {-1, 1}, {1, 1}};

#define MAX_VALUE 999999

__device__ __forceinline__ int iclip(int lo, int hi, int v) { return v < lo ? lo : (v > hi ? hi : v); }
__device__ __forceinline__ int clip255(int v) { return v < 0 ? 0 : (v > 255 ? 255 : v); }
__device__ __forceinline__ int isign(int a, int b) { return b < 0 ? -abs(a) : abs(a); }
__device__ __forceinline__ int mvbits(int v) { return v == 0 ? 1 : 2 * (31 - __clz(abs(v))) + 3; }

// ======================================================================================
//  quarter-pel interpolation (H.264 8.4.2.2.1), spec coordinate clamping
// ======================================================================================
__device__ __forceinline__ int rpx(const uint8_t *p, int w, int h, int x, int y) {
    return p[iclip(0, h - 1, y) * w + iclip(0, w - 1, x)];
}
__device__ __forceinline__ int tap6(int a, int b, int c, int d, int e, int f) { return a - 5 * b + 20 * c + 20 * d - 5 * e + f; }
__device__ __forceinline__ int hb1(const uint8_t *p, int w, int h, int x, int y) {
    return tap6(rpx(p, w, h, x - 2, y), rpx(p, w, h, x - 1, y), rpx(p, w, h, x, y), rpx(p, w, h, x + 1, y),
                rpx(p, w, h, x + 2, y), rpx(p, w, h, x + 3, y));
}
__device__ __forceinline__ int vh1(const uint8_t *p, int w, int h, int x, int y) {
    return tap6(rpx(p, w, h, x, y - 2), rpx(p, w, h, x, y - 1), rpx(p, w, h, x, y), rpx(p, w, h, x, y + 1),
                rpx(p, w, h, x, y + 2), rpx(p, w, h, x, y + 3));
}

// one thread = one padded integer position; writes its sample in all 16 phase planes
__global__ __launch_bounds__(256) void k_interp(const uint8_t *__restrict__ ref, int W, int H,
                                                uint8_t *__restrict__ qpel, int qstride, int qplane) {
    int px = blockIdx.x * 64 + (threadIdx.x & 63);
    int py = blockIdx.y * 4 + (threadIdx.x >> 6);
    if (px >= qstride || py >= H + 2 * QPAD) return;
    int x = px - QPAD, y = py - QPAD;
    int G = rpx(ref, W, H, x, y), Hn = rpx(ref, W, H, x + 1, y), M = rpx(ref, W, H, x, y + 1);
    int b = clip255((hb1(ref, W, H, x, y) + 16) >> 5);
    int hh = clip255((vh1(ref, W, H, x, y) + 16) >> 5);
    int s = clip255((hb1(ref, W, H, x, y + 1) + 16) >> 5);
    int m = clip255((vh1(ref, W, H, x + 1, y) + 16) >> 5);
    int j1 = tap6(vh1(ref, W, H, x - 2, y), vh1(ref, W, H, x - 1, y), vh1(ref, W, H, x, y), vh1(ref, W, H, x + 1, y),
                  vh1(ref, W, H, x + 2, y), vh1(ref, W, H, x + 3, y));
    int j = clip255((j1 + 512) >> 10);
    uint8_t v[16];
    v[0] = G;                     v[1] = (G + b + 1) >> 1;  v[2] = b;                 v[3] = (Hn + b + 1) >> 1;
    v[4] = (G + hh + 1) >> 1;     v[5] = (b + hh + 1) >> 1; v[6] = (b + j + 1) >> 1;  v[7] = (b + m + 1) >> 1;
    v[8] = hh;                    v[9] = (hh + j + 1) >> 1; v[10] = j;                v[11] = (j + m + 1) >> 1;
    v[12] = (M + hh + 1) >> 1;    v[13] = (hh + s + 1) >> 1; v[14] = (j + s + 1) >> 1; v[15] = (m + s + 1) >> 1;
    size_t o = (size_t)py * qstride + px;
#pragma unroll
    for (int ph = 0; ph < 16; ph++) qpel[(size_t)ph * qplane + o] = v[ph];
}

// ======================================================================================
//  transform / quantisation helpers (single-thread, one block), JM 8.6 block.c [J]
// ======================================================================================
__device__ void fwd4x4(int m[16]) {
#pragma unroll
    for (int y = 0; y < 4; y++) {
        int *r = m + 4 * y;
        int p0 = r[0] + r[3], p3 = r[0] - r[3], p1 = r[1] + r[2], p2 = r[1] - r[2];
        r[0] = p0 + p1; r[2] = p0 - p1; r[1] = 2 * p3 + p2; r[3] = p3 - 2 * p2;
    }
#pragma unroll
    for (int x = 0; x < 4; x++) {
        int p0 = m[x] + m[12 + x], p3 = m[x] - m[12 + x], p1 = m[4 + x] + m[8 + x], p2 = m[4 + x] - m[8 + x];
        m[x] = p0 + p1; m[8 + x] = p0 - p1; m[4 + x] = 2 * p3 + p2; m[12 + x] = p3 - 2 * p2;
    }
}
// inverse 4x4 (8.5.12.2) + recon clip((r + (pred<<6) + 32) >> 6)
__device__ void inv4x4_add(const int m[16], const uint8_t *pred, int ps, uint8_t *out, int os) {
    int t[16];
#pragma unroll
    for (int y = 0; y < 4; y++) {
        const int *d = m + 4 * y;
        int e0 = d[0] + d[2], e1 = d[0] - d[2], e2 = (d[1] >> 1) - d[3], e3 = d[1] + (d[3] >> 1);
        t[4 * y] = e0 + e3; t[4 * y + 1] = e1 + e2; t[4 * y + 2] = e1 - e2; t[4 * y + 3] = e0 - e3;
    }
#pragma unroll
    for (int x = 0; x < 4; x++) {
        int d0 = t[x], d1 = t[4 + x], d2 = t[8 + x], d3 = t[12 + x];
        int e0 = d0 + d2, e1 = d0 - d2, e2 = (d1 >> 1) - d3, e3 = d1 + (d3 >> 1);
        int r[4] = {e0 + e3, e1 + e2, e1 - e2, e0 - e3};
#pragma unroll
        for (int y = 0; y < 4; y++) out[y * os + x] = (uint8_t)clip255((r[y] + (pred[y * ps + x] << 6) + 32) >> 6);
    }
}
// dct_luma [J]: returns nonzero; levels in scan order; accumulates coeff cost
__device__ int dct_luma4x4(const int resid[16], const uint8_t *pred, int ps, int qp, int intra_round, int16_t *levels,
                           int *coeff_cost, uint8_t *rec, int rs) {
    int qp_per = qp / 6, qp_rem = qp % 6, q_bits = 15 + qp_per;
    int qp_const = intra_round ? (1 << q_bits) / 3 : (1 << q_bits) / 6;
    int m[16];
#pragma unroll
    for (int k = 0; k < 16; k++) m[k] = resid[k];
    fwd4x4(m);
    int run = -1, nonzero = 0;
    for (int k = 0; k < 16; k++) {
        int pos = c_scan[k];
        run++;
        int level = (abs(m[pos]) * c_quant[qp_rem][pos] + qp_const) >> q_bits;
        int ilev = 0;
        if (level != 0) {
            nonzero = 1;
            *coeff_cost += level > 1 ? MAX_VALUE : c_coeff_cost[run];
            levels[k] = (int16_t)isign(level, m[pos]);
            run = -1;
            ilev = level * c_dequant[qp_rem][pos] << qp_per;
        } else levels[k] = 0;
        m[pos] = isign(ilev, m[pos]);
    }
    inv4x4_add(m, pred, ps, rec, rs);
    return nonzero;
}
// SATD() [J]: 4x4 Hadamard sum >> 1, or SAD
__device__ int satd4x4(const int d[16], int had) {
    int s = 0;
    if (!had) {
#pragma unroll
        for (int k = 0; k < 16; k++) s += abs(d[k]);
        return s;
    }
    int m[16];
#pragma unroll
    for (int x = 0; x < 4; x++) {
        int a0 = d[x] + d[12 + x], a1 = d[4 + x] + d[8 + x], a2 = d[4 + x] - d[8 + x], a3 = d[x] - d[12 + x];
        m[x] = a0 + a1; m[8 + x] = a0 - a1; m[4 + x] = a2 + a3; m[12 + x] = a3 - a2;
    }
#pragma unroll
    for (int y = 0; y < 4; y++) {
        int *r = m + 4 * y;
        int a0 = r[0] + r[3], a1 = r[1] + r[2], a2 = r[1] - r[2], a3 = r[0] - r[3];
        s += abs(a0 + a1) + abs(a0 - a1) + abs(a2 + a3) + abs(a3 - a2);
    }
    return s >> 1;
}

// ======================================================================================
//  macroblock kernel shared state
// ======================================================================================
struct MeBuf {
    uint8_t win[WIN_MAX * WSTRIDE + 16];
    uint16_t sad[16 * NPOS_MAX];          // [4x4 block][window raster position]
};
struct FinBuf {
    uint8_t i4pred[9][16];
    int i4cost[9];
    int i4P[13];
    int i4av[9];
    int16_t i4lev[16][16];
    uint8_t i16pred[4][256];
    int i16ac[4][16];
    int i16dcv[4][16];
    int i16cost[4];
    int i16av[4];
    uint8_t pred[256];
    int16_t lev[16][16];
    int bcost[16];
    int bnz[16];
    int dc[16];
    int dcdq[16];
    int16_t dclev[16];
    uint8_t cpred[2][4][64];
    int cav[4];
    int ccost[4][8];
    int cm[2][4][16];
    int16_t cdc[2][4];
    int16_t cac[2][4][16];
    int cfcost[2];
    int cdcq[2][4];
    uint8_t crec[2][64];
    uint8_t cfin[2][64];
};
struct Smem {
    uint8_t org[256];
    uint8_t orgc[2][64];
    uint8_t rec[256];
    int16_t enc_mv[16][2];
    int8_t enc_ref[16];
    int8_t ipred_cur[16];
    int16_t all_mv[8][16][2];
    int16_t fmv[16][2];
    int motion_cost[8][4];
    int satd[9][16];
    int ccand[9];
    unsigned red[NT / 64];
    int sc[32];
    union {
        MeBuf me;
        FinBuf fin;
    } u;
};
// scalar slots in Smem::sc
enum { S_SCX, S_SCY, S_POS00, S_PMVX, S_PMVY, S_MVX, S_MVY, S_MINC, S_BEST, S_CHK0, S_MINPOS2, S_MPM, S_BESTMODE,
       S_MINCOST, S_I4CBP, S_I4BLK, S_I16MODE, S_CMODE, S_CBP, S_CBPBLK, S_CRCBP, S_SKIPX, S_SKIPY, S_I4COST, S_I16COST };

__device__ unsigned block_min_u32(unsigned v, unsigned *red) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = min(v, (unsigned)__shfl_xor((int)v, o, 64));
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
    __syncthreads();
    unsigned r = red[0];
#pragma unroll
    for (int i = 1; i < NT / 64; i++) r = min(r, red[i]);
    __syncthreads();
    return r;
}

// getLuma4x4Neighbour [J] for MVP purposes: reads the current MB's enc_picture state from LDS
__device__ bool nb4(const DevParams &d, const Smem &s, int mbx, int mby, int xN, int yN, int &ref, int &mx_, int &my_) {
    int tx, ty;
    if (yN > 15) return false;
    if (xN < 0) { tx = mbx - 1; ty = yN < 0 ? mby - 1 : mby; }
    else if (xN <= 15) { tx = mbx; ty = yN < 0 ? mby - 1 : mby; }
    else { if (yN >= 0) return false; tx = mbx + 1; ty = mby - 1; }
    if (tx < 0 || ty < 0 || tx >= d.mbw) return false;
    if (tx == mbx && ty == mby) {
        int k = (yN >> 2) * 4 + (xN >> 2);
        ref = s.enc_ref[k]; mx_ = s.enc_mv[k][0]; my_ = s.enc_mv[k][1];
        return true;
    }
    int a = ((16 * mby + yN) >> 2) * (d.W >> 2) + ((16 * mbx + xN) >> 2);
    ref = d.refidx[a]; mx_ = d.mv[2 * a]; my_ = d.mv[2 * a + 1];
    return true;
}

// SetMotionVectorPredictor [J] / H.264 8.4.1.3 (list 0, ref 0); thread-serial
__device__ void set_mvp(const DevParams &d, const Smem &s, int mbx, int mby, int bx4, int by4, int bsx, int bsy, int &px, int &py) {
    int mb_x = 4 * bx4, mb_y = 4 * by4;
    int ra = -1, rb = -1, rc = -1, rd = -1, ax = 0, ay = 0, bxv = 0, byv = 0, cx = 0, cy = 0, dx = 0, dy = 0;
    bool av_a = nb4(d, s, mbx, mby, mb_x - 1, mb_y, ra, ax, ay);
    bool av_b = nb4(d, s, mbx, mby, mb_x, mb_y - 1, rb, bxv, byv);
    bool av_c = nb4(d, s, mbx, mby, mb_x + bsx, mb_y - 1, rc, cx, cy);
    bool av_d = nb4(d, s, mbx, mby, mb_x - 1, mb_y - 1, rd, dx, dy);
    if (mb_y > 0) {
        if (mb_x < 8) {
            if (mb_y == 8) { if (bsx == 16) av_c = false; }
            else if (mb_x + bsx == 8) av_c = false;
        } else if (mb_x + bsx == 16) av_c = false;
    }
    if (!av_c) { av_c = av_d; rc = rd; cx = dx; cy = dy; }
    int rL = av_a ? ra : -1, rU = av_b ? rb : -1, rUR = av_c ? rc : -1;
    int type = 0;
    if (rL == 0 && rU != 0 && rUR != 0) type = 1;
    else if (rL != 0 && rU == 0 && rUR != 0) type = 2;
    else if (rL != 0 && rU != 0 && rUR == 0) type = 3;
    if (bsx == 8 && bsy == 16) { if (mb_x == 0) { if (rL == 0) type = 1; } else if (rUR == 0) type = 3; }
    else if (bsx == 16 && bsy == 8) { if (mb_y == 0) { if (rU == 0) type = 2; } else if (rL == 0) type = 1; }
    int A[2] = {av_a ? ax : 0, av_a ? ay : 0}, B[2] = {av_b ? bxv : 0, av_b ? byv : 0}, C[2] = {av_c ? cx : 0, av_c ? cy : 0};
    int p[2];
#pragma unroll
    for (int hv = 0; hv < 2; hv++) {
        int a = A[hv], b = B[hv], c = C[hv];
        if (type == 1) p[hv] = a;
        else if (type == 2) p[hv] = b;
        else if (type == 3) p[hv] = c;
        else if (!(av_b || av_c)) p[hv] = a;
        else p[hv] = a + b + c - min(a, min(b, c)) - max(a, max(b, c));
    }
    px = p[0]; py = p[1];
}

__device__ __forceinline__ int qpel_at(const DevParams &d, int X, int Y) {
    int x = iclip(-QPAD, d.W - 1 + QPAD, X >> 2), y = iclip(-QPAD, d.H - 1 + QPAD, Y >> 2);
    int ph = (Y & 3) * 4 + (X & 3);
    return d.qpel[(size_t)ph * d.qplane + (size_t)(y + QPAD) * d.qstride + (x + QPAD)];
}

// ======================================================================================
//  motion search (one block), all threads participate
// ======================================================================================
__device__ void block_motion_search(const DevParams &d, Smem &s, int mbx, int mby, int bt, int bx4, int by4) {
    const int tid = threadIdx.x;
    const int bsx = c_blc[bt][0], bsy = c_blc[bt][1], w4 = bsx >> 2, h4 = bsy >> 2;
    const int sr = d.sr, side = d.side;
    int range = sr;
    if (d.restrict_sr == 0) range = sr / min(2, bt);
    const int lf = 65536 * d.lambda_motion;
    if (tid == 0) {
        int px, py;
        set_mvp(d, s, mbx, mby, bx4, by4, bsx, bsy, px, py);
        s.sc[S_PMVX] = px; s.sc[S_PMVY] = py;
    }
    __syncthreads();
    const int pmvx = s.sc[S_PMVX], pmvy = s.sc[S_PMVY];
    const int scx = s.sc[S_SCX], scy = s.sc[S_SCY], pos00 = s.sc[S_POS00];
    // ---- FastFullPelBlockMotionSearch: keys = cost << 13 | order (order 0 = the (0,0) pre-check)
    unsigned best = 0xFFFFFFFFu;
    for (int r = tid; r < d.npos; r += NT) {
        int dx = r % side - sr, dy = r / side - sr;
        if (abs(dx) > range || abs(dy) > range) continue;
        int sad = 0;
        for (int y = 0; y < h4; y++)
            for (int x = 0; x < w4; x++) sad += s.u.me.sad[((by4 + y) * 4 + bx4 + x) * NPOS_MAX + r];
        int cost = sad + ((lf * (mvbits(((scx + dx) << 2) - pmvx) + mvbits(((scy + dy) << 2) - pmvy))) >> 16);
        int sp = d.spiral_of[r];
        unsigned order = sp == pos00 ? 0u : (unsigned)sp + 1u;
        best = min(best, ((unsigned)cost << 13) | order);
    }
    if (tid == 0) {   // the (0,0) pre-check is evaluated even outside a restricted range
        int r = (-scy + sr) * side + (-scx + sr);
        int sad = 0;
        for (int y = 0; y < h4; y++)
            for (int x = 0; x < w4; x++) sad += s.u.me.sad[((by4 + y) * 4 + bx4 + x) * NPOS_MAX + r];
        int cost = sad + ((lf * (mvbits(-pmvx) + mvbits(-pmvy))) >> 16);
        best = min(best, (unsigned)cost << 13);
    }
    best = block_min_u32(best, s.red);
    // ---- SubPelBlockMotionSearch (search_pos2 = search_pos4 = 9)
    unsigned order = best & 8191u;
    int bsp = order == 0 ? pos00 : (int)order - 1;
    int fmx = scx + d.spiral[2 * bsp], fmy = scy + d.spiral[2 * bsp + 1];
    int min_mcost = (int)(best >> 13);
    const int had = d.use_hadamard;
    const int check0 = (bt == 1 && fmx == 0 && fmy == 0 && had && d.slice_type == JMH_P_SLICE);
    if (had) min_mcost = BIGCOST;
    const int nsub = w4 * h4;
    int cmx = fmx << 2, cmy = fmy << 2;
    for (int pass = 0; pass < 2; pass++) {
        const int step = pass == 0 ? 2 : 1;
        const int min_pos = pass == 0 ? (had ? 0 : 1) : 1;
        if (tid < 9 * nsub) {
            int cand = tid / nsub, sub = tid % nsub;
            if (cand >= min_pos) {
                int vx = cmx + step * c_sp9[cand][0], vy = cmy + step * c_sp9[cand][1];
                int ox = 4 * (bx4 + sub % w4), oy = 4 * (by4 + sub / w4);
                int df[16];
#pragma unroll
                for (int y = 0; y < 4; y++)
#pragma unroll
                    for (int x = 0; x < 4; x++)
                        df[4 * y + x] = s.org[(oy + y) * 16 + ox + x] -
                                        qpel_at(d, 4 * (16 * mbx + ox + x) + vx, 4 * (16 * mby + oy + y) + vy);
                s.satd[cand][sub] = satd4x4(df, had);
            }
        }
        __syncthreads();
        if (tid < 9) {
            int cand = tid;
            int vx = cmx + step * c_sp9[cand][0], vy = cmy + step * c_sp9[cand][1];
            int mc = (lf * (mvbits(vx - pmvx) + mvbits(vy - pmvy))) >> 16;
            if (pass == 0 && check0 && cand == 0) mc -= (lf * 16) >> 16;
            int sum = 0;
            for (int k = 0; k < nsub; k++) sum += s.satd[cand][k];
            s.ccand[cand] = mc + sum;
        }
        __syncthreads();
        // JM: candidates in order, strict '<' against the running minimum (mvcost-only
        // pruning is result-neutral)
        int bpos = 0;
        for (int cand = min_pos; cand < 9; cand++) {
            int c = s.ccand[cand];
            if (c < min_mcost) { min_mcost = c; bpos = cand; }
        }
        cmx += step * c_sp9[bpos][0];
        cmy += step * c_sp9[bpos][1];
        __syncthreads();
    }
    // ---- store (BlockMotionSearch / PartitionMotionSearch bookkeeping)
    if (tid < w4 * h4) {
        int k = (by4 + tid / w4) * 4 + bx4 + tid % w4;
        s.all_mv[bt][k][0] = (int16_t)cmx; s.all_mv[bt][k][1] = (int16_t)cmy;
        s.enc_mv[k][0] = (int16_t)cmx; s.enc_mv[k][1] = (int16_t)cmy;
        s.enc_ref[k] = 0;
    }
    if (tid == 0) s.sc[S_MINC] = min_mcost;
    __syncthreads();
}

__constant__ int bx0[5][4] = {{0, 0, 0, 0}, {0, 0, 0, 0}, {0, 0, 0, 0}, {0, 2, 0, 0}, {0, 2, 0, 2}};
__constant__ int by0[5][4] = {{0, 0, 0, 0}, {0, 0, 0, 0}, {0, 2, 0, 0}, {0, 0, 0, 0}, {0, 0, 2, 2}};
// PartitionMotionSearch [J] (single reference)
__device__ void partition_motion_search(const DevParams &d, Smem &s, int mbx, int mby, int bt, int b8) {
    int pt = bt < 4 ? bt : 4;
    int sh0 = c_blc[pt][0] >> 2, sv0 = c_blc[pt][1] >> 2, sh = c_blc[bt][0] >> 2, sv = c_blc[bt][1] >> 2;
    int cost = 0;
    for (int v = by0[pt][b8]; v < by0[pt][b8] + sv0; v += sv)
        for (int h = bx0[pt][b8]; h < bx0[pt][b8] + sh0; h += sh) {
            block_motion_search(d, s, mbx, mby, bt, h, v);
            cost += s.sc[S_MINC];
        }
    if (threadIdx.x == 0) s.motion_cost[bt][b8] = cost;
    __syncthreads();
}

// ======================================================================================
//  intra helpers
// ======================================================================================
__device__ __forceinline__ bool mb_avail(const DevParams &d, int mbx, int mby, int dmx, int dmy) {
    int mx = mbx + dmx, my = mby + dmy;
    return mx >= 0 && my >= 0 && mx < d.mbw && my < d.mbh && (my < mby || (my == mby && mx < mbx));
}
// luma sample of the current picture recon at MB-relative (x,y): current MB from LDS
__device__ __forceinline__ int rec_luma(const DevParams &d, const Smem &s, int mbx, int mby, int x, int y) {
    if (x >= 0 && x < 16 && y >= 0 && y < 16) return s.rec[16 * y + x];
    return d.recY[(16 * mby + y) * d.W + 16 * mbx + x];
}

// Intra4x4 predictions of block at (bx,by) (thread m computes mode m); P[] gathered by thread 0
__device__ void i4_pred_mode(const int *P, int up, int left, int m, uint8_t out[16]) {
#define PT(x) P[1 + (x)]
#define PL(y) ((y) < 0 ? P[0] : P[9 + (y)])
    for (int y = 0; y < 4; y++)
        for (int x = 0; x < 4; x++) {
            int v = 0;
            switch (m) {
            case 0: v = PT(x); break;
            case 1: v = PL(y); break;
            case 2:
                if (up && left) v = (PT(0) + PT(1) + PT(2) + PT(3) + PL(0) + PL(1) + PL(2) + PL(3) + 4) >> 3;
                else if (left) v = (PL(0) + PL(1) + PL(2) + PL(3) + 2) >> 2;
                else if (up) v = (PT(0) + PT(1) + PT(2) + PT(3) + 2) >> 2;
                else v = 128;
                break;
            case 3: v = (x == 3 && y == 3) ? (PT(6) + 3 * PT(7) + 2) >> 2 : (PT(x + y) + 2 * PT(x + y + 1) + PT(x + y + 2) + 2) >> 2; break;
            case 4:
                if (x > y) v = (PT(x - y - 2) + 2 * PT(x - y - 1) + PT(x - y) + 2) >> 2;
                else if (x < y) v = (PL(y - x - 2) + 2 * PL(y - x - 1) + PL(y - x) + 2) >> 2;
                else v = (PT(0) + 2 * P[0] + PL(0) + 2) >> 2;
                break;
            case 5: {
                int z = 2 * x - y;
                if (z >= 0 && !(z & 1)) v = (PT(x - (y >> 1) - 1) + PT(x - (y >> 1)) + 1) >> 1;
                else if (z >= 0) v = (PT(x - (y >> 1) - 2) + 2 * PT(x - (y >> 1) - 1) + PT(x - (y >> 1)) + 2) >> 2;
                else if (z == -1) v = (PL(0) + 2 * P[0] + PT(0) + 2) >> 2;
                else v = (PL(y - 1) + 2 * PL(y - 2) + PL(y - 3) + 2) >> 2;
                break;
            }
            case 6: {
                int z = 2 * y - x;
                if (z >= 0 && !(z & 1)) v = (PL(y - (x >> 1) - 1) + PL(y - (x >> 1)) + 1) >> 1;
                else if (z >= 0) v = (PL(y - (x >> 1) - 2) + 2 * PL(y - (x >> 1) - 1) + PL(y - (x >> 1)) + 2) >> 2;
                else if (z == -1) v = (PL(0) + 2 * P[0] + PT(0) + 2) >> 2;
                else v = (PT(x - 1) + 2 * PT(x - 2) + PT(x - 3) + 2) >> 2;
                break;
            }
            case 7:
                v = (y & 1) ? (PT(x + (y >> 1)) + 2 * PT(x + (y >> 1) + 1) + PT(x + (y >> 1) + 2) + 2) >> 2
                            : (PT(x + (y >> 1)) + PT(x + (y >> 1) + 1) + 1) >> 1;
                break;
            default: {
                int z = x + 2 * y;
                if (z > 5) v = PL(3);
                else if (z == 5) v = (PL(2) + 3 * PL(3) + 2) >> 2;
                else if (!(z & 1)) v = (PL(y + (x >> 1)) + PL(y + (x >> 1) + 1) + 1) >> 1;
                else v = (PL(y + (x >> 1)) + 2 * PL(y + (x >> 1) + 1) + PL(y + (x >> 1) + 2) + 2) >> 2;
            }
            }
            out[4 * y + x] = (uint8_t)v;
        }
#undef PT
#undef PL
}

// chroma DC prediction for one 4x4 chroma block (8.3.4.1-3)
__device__ int chroma_dc(const int *T, const int *L, int up, int left, int b) {
    int s0 = 0, s1 = 0, s2 = 0, s3 = 0;
    for (int i = 0; i < 4; i++) { s0 += T[i]; s1 += T[4 + i]; s2 += L[i]; s3 += L[4 + i]; }
    if (b == 0) return (up && left) ? (s0 + s2 + 4) >> 3 : up ? (s0 + 2) >> 2 : left ? (s2 + 2) >> 2 : 128;
    if (b == 1) return up ? (s1 + 2) >> 2 : left ? (s2 + 2) >> 2 : 128;
    if (b == 2) return left ? (s3 + 2) >> 2 : up ? (s0 + 2) >> 2 : 128;
    return (up && left) ? (s1 + s3 + 4) >> 3 : up ? (s1 + 2) >> 2 : left ? (s3 + 2) >> 2 : 128;
}

// ======================================================================================
//  k_mb_encode: encode_one_macroblock for every MB of diagonal d.diag
// ======================================================================================
__global__ __launch_bounds__(NT) void k_mb_encode(DevParams d) {
    __shared__ Smem s;
    const int tid = threadIdx.x;
    const int mby = d.y_min + blockIdx.x;
    const int mbx = d.diag - 2 * mby;
    const int pix_x = 16 * mbx, pix_y = 16 * mby;
    const int W = d.W, Wc = d.Wc, W4 = d.W >> 2;
    const int slice_p = d.slice_type == JMH_P_SLICE;
    const int qp = d.qp, lambda = d.lambda_mode;
    const int intra_round = !slice_p;
    const int sr = d.sr, side = d.side;

    // ---- load the original MB, init per-MB state
    s.org[tid] = d.orgY[(pix_y + (tid >> 4)) * W + pix_x + (tid & 15)];
    if (tid < 128) {
        int uv = tid >> 6, k = tid & 63;
        s.orgc[uv][k] = (uv ? d.orgV : d.orgU)[((pix_y >> 1) + (k >> 3)) * Wc + (pix_x >> 1) + (k & 7)];
    }
    if (tid < 16) { s.enc_ref[tid] = -1; s.enc_mv[tid][0] = s.enc_mv[tid][1] = 0; }
    if (tid < 32) s.motion_cost[tid >> 2][tid & 3] = 0;
    __syncthreads();

    int min_cost = BIGCOST, best_mode = 1;
    int best8x8[4] = {0, 0, 0, 0};
    int skipx = 0, skipy = 0;
    int valid[9];
    for (int m = 1; m <= 7; m++) valid[m] = slice_p && d.inter_search[m];
    valid[8] = valid[4] || valid[5] || valid[6] || valid[7];

    if (slice_p) {
        // ---- SetupFastFullPelSearch: centre = 16x16 MVP / 4 (trunc), clamped to +-SR
        if (tid == 0) {
            int px, py;
            set_mvp(d, s, mbx, mby, 0, 0, 16, 16, px, py);
            int cx = iclip(-sr, sr, px / 4), cy = iclip(-sr, sr, py / 4);
            s.sc[S_SCX] = cx; s.sc[S_SCY] = cy;
            s.sc[S_POS00] = d.spiral_of[(-cy + sr) * side + (-cx + sr)];
        }
        __syncthreads();
        const int scx = s.sc[S_SCX], scy = s.sc[S_SCY];
        const int wdim = 2 * sr + 16;
        const int X0 = pix_x + scx - sr, Y0 = pix_y + scy - sr;
        for (int i = tid; i < wdim * WSTRIDE; i += NT) {
            int y = i / WSTRIDE, x = i % WSTRIDE;
            s.u.me.win[i] = x < wdim ? d.refY[iclip(0, d.H - 1, Y0 + y) * W + iclip(0, W - 1, X0 + x)] : 0;
        }
        if (tid < 16) s.u.me.win[wdim * WSTRIDE + tid] = 0;
        __syncthreads();
        // 16 4x4 SADs per position: v_sad_u8 on dword-aligned (v_alignbyte) reference rows
        const uint32_t *org32 = reinterpret_cast<const uint32_t *>(s.org);
        for (int r = tid; r < d.npos; r += NT) {
            int dx = r % side, dy = r / side;
            uint32_t acc[16];
#pragma unroll
            for (int b = 0; b < 16; b++) acc[b] = 0;
#pragma unroll
            for (int row = 0; row < 16; row++) {
                const uint8_t *wr = s.u.me.win + (dy + row) * WSTRIDE;
                const uint32_t *w32 = reinterpret_cast<const uint32_t *>(wr + (dx & ~3));
                const uint32_t sel = dx & 3;    // v_alignbyte byte select
                uint32_t a0 = w32[0], a1 = w32[1], a2 = w32[2], a3 = w32[3], a4 = w32[4];
                uint32_t r0 = __builtin_amdgcn_alignbyte(a1, a0, sel);
                uint32_t r1 = __builtin_amdgcn_alignbyte(a2, a1, sel);
                uint32_t r2 = __builtin_amdgcn_alignbyte(a3, a2, sel);
                uint32_t r3 = __builtin_amdgcn_alignbyte(a4, a3, sel);
                int br = (row >> 2) * 4;
                acc[br + 0] = __builtin_amdgcn_sad_u8(r0, org32[row * 4 + 0], acc[br + 0]);
                acc[br + 1] = __builtin_amdgcn_sad_u8(r1, org32[row * 4 + 1], acc[br + 1]);
                acc[br + 2] = __builtin_amdgcn_sad_u8(r2, org32[row * 4 + 2], acc[br + 2]);
                acc[br + 3] = __builtin_amdgcn_sad_u8(r3, org32[row * 4 + 3], acc[br + 3]);
            }
#pragma unroll
            for (int b = 0; b < 16; b++) s.u.me.sad[b * NPOS_MAX + r] = (uint16_t)acc[b];
        }
        __syncthreads();
        // ---- 16x16, 16x8, 8x16
        for (int mode = 1; mode < 4; mode++) {
            if (!valid[mode]) continue;
            int cost = 0;
            for (int block = 0; block < (mode == 1 ? 1 : 2); block++) {
                partition_motion_search(d, s, mbx, mby, mode, block);
                cost += s.motion_cost[mode][block];
            }
            if (cost < min_cost) { best_mode = mode; min_cost = cost; }
        }
        // ---- P8x8
        if (valid[8]) {
            int cost8x8 = 0;
            for (int block = 0; block < 4; block++) {
                int mc8 = BIGCOST;
                for (int mode = 4; mode <= 7; mode++) {
                    if (!valid[mode]) continue;
                    partition_motion_search(d, s, mbx, mby, mode, block);
                    int cost = s.motion_cost[mode][block];
                    if (cost < mc8) { mc8 = cost; best8x8[block] = mode; }
                }
                cost8x8 += mc8;
                int mode = best8x8[block];
                if (tid < 4 && mode > 0) {   // reset stored motion vectors of this 8x8
                    int k = ((block >> 1) * 2 + (tid >> 1)) * 4 + (block & 1) * 2 + (tid & 1);
                    s.enc_mv[k][0] = s.all_mv[mode][k][0]; s.enc_mv[k][1] = s.all_mv[mode][k][1]; s.enc_ref[k] = 0;
                }
                __syncthreads();
            }
            if (cost8x8 < min_cost) { best_mode = JMH_P8x8; min_cost = cost8x8; }
        }
        // ---- FindSkipModeMotionVector
        if (tid == 0) {
            int ra, ax, ay, rb, bx, by;
            bool aa = nb4(d, s, mbx, mby, -1, 0, ra, ax, ay), ab = nb4(d, s, mbx, mby, 0, -1, rb, bx, by);
            bool zl = !aa || (ra == 0 && ax == 0 && ay == 0), za = !ab || (rb == 0 && bx == 0 && by == 0);
            int px = 0, py = 0;
            if (!(za || zl)) set_mvp(d, s, mbx, mby, 0, 0, 16, 16, px, py);
            s.sc[S_SKIPX] = px; s.sc[S_SKIPY] = py;
        }
        __syncthreads();
        skipx = s.sc[S_SKIPX]; skipy = s.sc[S_SKIPY];
    }
    __syncthreads();   // the ME buffers are dead from here on (union reuse)

    FinBuf &f = s.u.fin;
    // ======== Intra 4x4 decision with TQ + recon per block (Mode_Decision_for_Intra4x4Macroblock)
    int i4cost = 0, i4cbp = 0, i4blk = 0;
    for (int b8 = 0; b8 < 4; b8++) {
        int cost8 = 6 * lambda;
        for (int b4 = 0; b4 < 4; b4++) {
            int bx = 8 * (b8 & 1) + 4 * (b4 & 1), by = 8 * (b8 >> 1) + 4 * (b4 >> 1);
            int blk = (by >> 2) * 4 + (bx >> 2);
            if (tid == 0) {
                // MPM
                int upM = -1, leftM = -1;
                if (bx > 0) leftM = s.ipred_cur[blk - 1];
                else if (mb_avail(d, mbx, mby, -1, 0)) leftM = d.ipred[((pix_y + by) >> 2) * W4 + (pix_x >> 2) - 1];
                if (by > 0) upM = s.ipred_cur[blk - 4];
                else if (mb_avail(d, mbx, mby, 0, -1)) upM = d.ipred[((pix_y >> 2) - 1) * W4 + ((pix_x + bx) >> 2)];
                s.sc[S_MPM] = (upM < 0 || leftM < 0) ? 2 : min(upM, leftM);
                // neighbour samples
                bool up = by > 0 || mb_avail(d, mbx, mby, 0, -1);
                bool left = bx > 0 || mb_avail(d, mbx, mby, -1, 0);
                bool ul = (bx > 0 && by > 0) || (bx == 0 && by > 0 && mb_avail(d, mbx, mby, -1, 0)) ||
                          (bx > 0 && by == 0 && mb_avail(d, mbx, mby, 0, -1)) || (bx == 0 && by == 0 && mb_avail(d, mbx, mby, -1, -1));
                bool ur;
                if (by == 0) ur = (bx + 4 <= 15) ? mb_avail(d, mbx, mby, 0, -1) : mb_avail(d, mbx, mby, 1, -1);
                else ur = bx + 4 <= 15;
                if ((bx == 4 || bx == 12) && (by == 4 || by == 12)) ur = false;
                f.i4P[0] = ul ? rec_luma(d, s, mbx, mby, bx - 1, by - 1) : 0;
                for (int i = 0; i < 4; i++) f.i4P[1 + i] = up ? rec_luma(d, s, mbx, mby, bx + i, by - 1) : 0;
                for (int i = 4; i < 8; i++) f.i4P[1 + i] = up ? (ur ? rec_luma(d, s, mbx, mby, bx + i, by - 1) : f.i4P[4]) : 0;
                for (int i = 0; i < 4; i++) f.i4P[9 + i] = left ? rec_luma(d, s, mbx, mby, bx - 1, by + i) : 0;
                int all = up && left && ul;
                f.i4av[0] = f.i4av[3] = f.i4av[7] = up;
                f.i4av[1] = f.i4av[8] = left;
                f.i4av[2] = 1;
                f.i4av[4] = f.i4av[5] = f.i4av[6] = all;
                s.sc[S_BEST] = (up ? 1 : 0) | (left ? 2 : 0);
            }
            __syncthreads();
            if (tid < 9) {
                int m = tid;
                int c = BIGCOST + 1;
                if (f.i4av[m]) {
                    i4_pred_mode(f.i4P, s.sc[S_BEST] & 1, (s.sc[S_BEST] >> 1) & 1, m, f.i4pred[m]);
                    int df[16];
                    for (int y = 0; y < 4; y++)
                        for (int x = 0; x < 4; x++) df[4 * y + x] = s.org[(by + y) * 16 + bx + x] - f.i4pred[m][4 * y + x];
                    c = (m == s.sc[S_MPM] ? 0 : 4 * lambda) + satd4x4(df, d.use_hadamard);
                }
                f.i4cost[m] = c;
            }
            __syncthreads();
            if (tid == 0) {
                int best = 0, bc = BIGCOST;
                for (int m = 0; m < 9; m++)
                    if (f.i4av[m] && f.i4cost[m] < bc) { bc = f.i4cost[m]; best = m; }
                s.ipred_cur[blk] = (int8_t)best;
                int rr[16], dummy = 0;
                for (int y = 0; y < 4; y++)
                    for (int x = 0; x < 4; x++) rr[4 * y + x] = s.org[(by + y) * 16 + bx + x] - f.i4pred[best][4 * y + x];
                int nz = dct_luma4x4(rr, f.i4pred[best], 4, qp, intra_round, f.i4lev[blk], &dummy, s.rec + by * 16 + bx, 16);
                s.sc[S_MINC] = bc;
                s.sc[S_I4BLK] = nz;
            }
            __syncthreads();
            cost8 += s.sc[S_MINC];
            if (s.sc[S_I4BLK]) { i4cbp |= 1 << b8; i4blk |= 1 << blk; }
        }
        i4cost += cost8;
    }
    if (i4cost <= min_cost) { min_cost = i4cost; best_mode = JMH_I4MB; }

    // ======== Intra 16x16 (intrapred_luma_16x16 + find_sad_16x16)
    {
        const bool up = mb_avail(d, mbx, mby, 0, -1), left = mb_avail(d, mbx, mby, -1, 0), ul = mb_avail(d, mbx, mby, -1, -1);
        if (tid == 0) { f.i16av[0] = up; f.i16av[1] = left; f.i16av[2] = 1; f.i16av[3] = up && left && ul; }
        // DC / plane parameters (every thread computes them; 33 loads each, cached)
        int st = 0, sl = 0, ih = 0, iv = 0;
        int Pc = ul ? d.recY[(pix_y - 1) * W + pix_x - 1] : 0;
        for (int i = 0; i < 16; i++) {
            st += up ? d.recY[(pix_y - 1) * W + pix_x + i] : 0;
            sl += left ? d.recY[(pix_y + i) * W + pix_x - 1] : 0;
        }
        for (int i = 1; i <= 8; i++) {
            int ta = up ? d.recY[(pix_y - 1) * W + pix_x + 7 + i] : 0;
            int tb = 7 - i >= 0 ? (up ? d.recY[(pix_y - 1) * W + pix_x + 7 - i] : 0) : Pc;
            int la = left ? d.recY[(pix_y + 7 + i) * W + pix_x - 1] : 0;
            int lb = 7 - i >= 0 ? (left ? d.recY[(pix_y + 7 - i) * W + pix_x - 1] : 0) : Pc;
            ih += i * (ta - tb); iv += i * (la - lb);
        }
        int dcv = (up && left) ? (st + sl + 16) >> 5 : up ? (st + 8) >> 4 : left ? (sl + 8) >> 4 : 128;
        int ib = (5 * ih + 32) >> 6, ic = (5 * iv + 32) >> 6;
        int iaa = 16 * ((left ? d.recY[(pix_y + 15) * W + pix_x - 1] : 0) + (up ? d.recY[(pix_y - 1) * W + pix_x + 15] : 0));
        int x = tid & 15, y = tid >> 4;
        f.i16pred[0][tid] = (uint8_t)(up ? d.recY[(pix_y - 1) * W + pix_x + x] : 0);
        f.i16pred[1][tid] = (uint8_t)(left ? d.recY[(pix_y + y) * W + pix_x - 1] : 0);
        f.i16pred[2][tid] = (uint8_t)dcv;
        f.i16pred[3][tid] = (uint8_t)clip255((iaa + (x - 7) * ib + (y - 7) * ic + 16) >> 5);
        __syncthreads();
        if (tid < 64) {
            int m = tid >> 4, b = tid & 15, ox = (b & 3) * 4, oy = (b >> 2) * 4;
            int mm[16], t[16];
            for (int yy = 0; yy < 4; yy++)
                for (int xx = 0; xx < 4; xx++) mm[4 * yy + xx] = s.org[(oy + yy) * 16 + ox + xx] - f.i16pred[m][(oy + yy) * 16 + ox + xx];
            for (int yy = 0; yy < 4; yy++) {
                int *r = mm + 4 * yy;
                int a0 = r[0] + r[3], a1 = r[1] + r[2], a2 = r[1] - r[2], a3 = r[0] - r[3];
                t[4 * yy] = a0 + a1; t[4 * yy + 2] = a0 - a1; t[4 * yy + 1] = a2 + a3; t[4 * yy + 3] = a3 - a2;
            }
            int acs = 0, dcc = 0;
            for (int xx = 0; xx < 4; xx++) {
                int a0 = t[xx] + t[12 + xx], a1 = t[4 + xx] + t[8 + xx], a2 = t[4 + xx] - t[8 + xx], a3 = t[xx] - t[12 + xx];
                int o0 = a0 + a1, o2 = a0 - a1, o1 = a2 + a3, o3 = a3 - a2;
                if (xx == 0) dcc = o0; else acs += abs(o0);
                acs += abs(o1) + abs(o2) + abs(o3);
            }
            f.i16ac[m][b] = acs;
            f.i16dcv[m][b] = dcc / 4;
        }
        __syncthreads();
        if (tid < 4) {
            int m = tid, cost = 0;
            int t[16];
            for (int b = 0; b < 16; b++) cost += f.i16ac[m][b];
            const int *dcv4 = f.i16dcv[m];
            for (int yy = 0; yy < 4; yy++) {
                const int *r = dcv4 + 4 * yy;
                int a0 = r[0] + r[3], a1 = r[1] + r[2], a2 = r[1] - r[2], a3 = r[0] - r[3];
                t[4 * yy] = a0 + a1; t[4 * yy + 2] = a0 - a1; t[4 * yy + 1] = a2 + a3; t[4 * yy + 3] = a3 - a2;
            }
            for (int xx = 0; xx < 4; xx++) {
                int a0 = t[xx] + t[12 + xx], a1 = t[4 + xx] + t[8 + xx], a2 = t[4 + xx] - t[8 + xx], a3 = t[xx] - t[12 + xx];
                cost += abs(a0 + a1) + abs(a0 - a1) + abs(a2 + a3) + abs(a3 - a2);
            }
            f.i16cost[m] = cost;
        }
        __syncthreads();
    }
    int i16mode = 2;
    {
        int best = MAX_VALUE;
        for (int k = 0; k < 4; k++)
            if (f.i16av[k] && f.i16cost[k] < best) { best = f.i16cost[k]; i16mode = k; }
        int i16cost = best / 2;
        if (i16cost < min_cost) { min_cost = i16cost; best_mode = JMH_I16MB; }
    }

    // ======== final macroblock parameters
    const int is_intra = best_mode == JMH_I4MB || best_mode == JMH_I16MB;
    int b8mode[4];
    for (int b = 0; b < 4; b++) b8mode[b] = best_mode == JMH_P8x8 ? best8x8[b] : best_mode;
    if (best_mode == JMH_I4MB) for (int b = 0; b < 4; b++) b8mode[b] = JMH_IBLOCK;
    if (best_mode == JMH_I16MB) for (int b = 0; b < 4; b++) b8mode[b] = 0;
    if (tid < 16) {
        int k = tid, b8 = ((k >> 3) << 1) + ((k & 3) >> 1);
        s.fmv[k][0] = is_intra ? 0 : s.all_mv[b8mode[b8]][k][0];
        s.fmv[k][1] = is_intra ? 0 : s.all_mv[b8mode[b8]][k][1];
    }
    __syncthreads();
    int cbp = 0, cbp_blk = 0;
    if (best_mode == JMH_I4MB) {
        cbp = i4cbp; cbp_blk = i4blk;
        if (tid < 16) for (int k = 0; k < 16; k++) f.lev[tid][k] = f.i4lev[tid][k];
    } else if (best_mode == JMH_I16MB) {
        // dct_luma_16x16 [J]
        const int qp_per = qp / 6, qp_rem = qp % 6, q_bits = 15 + qp_per;
        const int qp_const = (1 << q_bits) / 3, qp_const2 = qp_const << 1;
        int m[16];
        if (tid < 16) {
            int b = tid, ox = (b & 3) * 4, oy = (b >> 2) * 4;
            for (int yy = 0; yy < 4; yy++)
                for (int xx = 0; xx < 4; xx++) m[4 * yy + xx] = s.org[(oy + yy) * 16 + ox + xx] - f.i16pred[i16mode][(oy + yy) * 16 + ox + xx];
            fwd4x4(m);
            f.dc[b] = m[0];
        }
        __syncthreads();
        if (tid == 0) {
            int *dc = f.dc;
            for (int yy = 0; yy < 4; yy++) {
                int *r = dc + 4 * yy;
                int a0 = r[0] + r[3], a3 = r[0] - r[3], a1 = r[1] + r[2], a2 = r[1] - r[2];
                r[0] = a0 + a1; r[2] = a0 - a1; r[1] = a3 + a2; r[3] = a3 - a2;
            }
            for (int xx = 0; xx < 4; xx++) {
                int a0 = dc[xx] + dc[12 + xx], a3 = dc[xx] - dc[12 + xx], a1 = dc[4 + xx] + dc[8 + xx], a2 = dc[4 + xx] - dc[8 + xx];
                dc[xx] = (a0 + a1) >> 1; dc[8 + xx] = (a0 - a1) >> 1; dc[4 + xx] = (a3 + a2) >> 1; dc[12 + xx] = (a3 - a2) >> 1;
            }
            int lev[16];
            for (int k = 0; k < 16; k++) {
                int pos = c_scan[k];
                int level = (abs(dc[pos]) * c_quant[qp_rem][0] + qp_const2) >> (q_bits + 1);
                f.dclev[k] = (int16_t)isign(level, dc[pos]);
                lev[pos] = f.dclev[k];
            }
            int t[16];
            for (int yy = 0; yy < 4; yy++) {
                const int *c = lev + 4 * yy;
                int e0 = c[0] + c[2], e1 = c[0] - c[2], e2 = c[1] - c[3], e3 = c[1] + c[3];
                t[4 * yy] = e0 + e3; t[4 * yy + 3] = e0 - e3; t[4 * yy + 1] = e1 + e2; t[4 * yy + 2] = e1 - e2;
            }
            int v00 = c_dequant[qp_rem][0];
            for (int xx = 0; xx < 4; xx++) {
                int e0 = t[xx] + t[8 + xx], e1 = t[xx] - t[8 + xx], e2 = t[4 + xx] - t[12 + xx], e3 = t[4 + xx] + t[12 + xx];
                int fv[4] = {e0 + e3, e1 + e2, e1 - e2, e0 - e3};
                for (int yy = 0; yy < 4; yy++) f.dcdq[4 * yy + xx] = ((fv[yy] * v00 << qp_per) + 2) >> 2;
            }
        }
        __syncthreads();
        if (tid < 16) {
            int b = tid, nz = 0;
            f.lev[b][0] = 0;
            for (int k = 1; k < 16; k++) {
                int pos = c_scan[k];
                int level = (abs(m[pos]) * c_quant[qp_rem][pos] + qp_const) >> q_bits;
                if (level) nz = 1;
                f.lev[b][k] = (int16_t)isign(level, m[pos]);
                m[pos] = isign(level * c_dequant[qp_rem][pos] << qp_per, m[pos]);
            }
            m[0] = f.dcdq[b];
            f.bnz[b] = nz;
            int ox = (b & 3) * 4, oy = (b >> 2) * 4;
            inv4x4_add(m, f.i16pred[i16mode] + oy * 16 + ox, 16, s.rec + oy * 16 + ox, 16);
        }
        __syncthreads();
        for (int b = 0; b < 16; b++)
            if (f.bnz[b]) { cbp = 15; cbp_blk |= 1 << b; }
    } else {
        // LumaResidualCoding / LumaResidualCoding8x8 (+ SetCoeffAndReconstruction8x8)
        if (tid < 16) {
            int k = tid, bx4 = k & 3, by4 = k >> 2;
            int mvx = s.fmv[k][0], mvy = s.fmv[k][1];
            uint8_t *pr = f.pred + 4 * by4 * 16 + 4 * bx4;
            int rr[16];
            for (int y = 0; y < 4; y++)
                for (int x = 0; x < 4; x++) {
                    int p = qpel_at(d, 4 * (pix_x + 4 * bx4 + x) + mvx, 4 * (pix_y + 4 * by4 + y) + mvy);
                    pr[y * 16 + x] = (uint8_t)p;
                    rr[4 * y + x] = s.org[(4 * by4 + y) * 16 + 4 * bx4 + x] - p;
                }
            int cc = 0;
            f.bnz[k] = dct_luma4x4(rr, pr, 16, qp, intra_round, f.lev[k], &cc, s.rec + 4 * by4 * 16 + 4 * bx4, 16);
            f.bcost[k] = cc;
        }
        __syncthreads();
        int sum_cnt = 0, keep8 = 0;
        for (int b8 = 0; b8 < 4; b8++) {
            int base = (b8 >> 1) * 8 + (b8 & 1) * 2;
            int cc = f.bcost[base] + f.bcost[base + 1] + f.bcost[base + 4] + f.bcost[base + 5];
            int nz = f.bnz[base] | f.bnz[base + 1] | f.bnz[base + 4] | f.bnz[base + 5];
            if (cc <= 4) cc = 0;
            else {
                keep8 |= 1 << b8;
                if (nz) cbp |= 1 << b8;
                for (int q = 0; q < 4; q++) {
                    int k = base + (q & 1) + (q >> 1) * 4;
                    if (f.bnz[k]) cbp_blk |= 1 << k;
                }
            }
            sum_cnt += cc;
        }
        if (sum_cnt <= 5) { keep8 = 0; cbp = 0; cbp_blk = 0; }
        if (tid < 16) {
            int k = tid, b8 = ((k >> 3) << 1) + ((k & 3) >> 1);
            if (!((keep8 >> b8) & 1)) {
                for (int q = 0; q < 16; q++) f.lev[k][q] = 0;
                int bx4 = k & 3, by4 = k >> 2;
                for (int y = 0; y < 4; y++)
                    for (int x = 0; x < 4; x++) s.rec[(4 * by4 + y) * 16 + 4 * bx4 + x] = f.pred[(4 * by4 + y) * 16 + 4 * bx4 + x];
            }
        }
    }
    __syncthreads();

    // ======== chroma: IntraChromaPrediction8x8 (intra MBs) + ChromaResidualCoding
    {
        int c_mode = 0;
        if (is_intra) {
            const bool up = mb_avail(d, mbx, mby, 0, -1), left = mb_avail(d, mbx, mby, -1, 0), ul = mb_avail(d, mbx, mby, -1, -1);
            if (tid < 128) {
                int uv = tid >> 6, k = tid & 63, x = k & 7, y = k >> 3;
                const uint8_t *R = uv ? d.recV : d.recU;
                int cx = pix_x >> 1, cy = pix_y >> 1;
                int T[8], L[8], Pc = ul ? R[(cy - 1) * Wc + cx - 1] : 0;
                for (int i = 0; i < 8; i++) {
                    T[i] = up ? R[(cy - 1) * Wc + cx + i] : 0;
                    L[i] = left ? R[(cy + i) * Wc + cx - 1] : 0;
                }
                f.cpred[uv][0][k] = (uint8_t)chroma_dc(T, L, up, left, (y >> 2) * 2 + (x >> 2));
                f.cpred[uv][1][k] = (uint8_t)L[y];
                f.cpred[uv][2][k] = (uint8_t)T[x];
                int ih = 0, iv = 0;
                for (int i = 1; i <= 4; i++) {
                    ih += i * (T[3 + i] - (3 - i >= 0 ? T[3 - i] : Pc));
                    iv += i * (L[3 + i] - (3 - i >= 0 ? L[3 - i] : Pc));
                }
                int ib = (34 * ih + 32) >> 6, ic = (34 * iv + 32) >> 6, iaa = 16 * (L[7] + T[7]);
                f.cpred[uv][3][k] = (uint8_t)clip255((iaa + (x - 3) * ib + (y - 3) * ic + 16) >> 5);
            }
            if (tid == 0) { f.cav[0] = 1; f.cav[1] = left; f.cav[2] = up; f.cav[3] = up && left && ul; }
            __syncthreads();
            if (tid < 32) {
                int m = tid >> 3, uv = (tid >> 2) & 1, b = tid & 3, xo = (b & 1) * 4, yo = (b >> 1) * 4;
                int df[16];
                for (int y = 0; y < 4; y++)
                    for (int x = 0; x < 4; x++) df[4 * y + x] = s.orgc[uv][(yo + y) * 8 + xo + x] - f.cpred[uv][m][(yo + y) * 8 + xo + x];
                f.ccost[m][uv * 4 + b] = satd4x4(df, d.use_hadamard);
            }
            __syncthreads();
            int minc = BIGCOST;
            for (int m = 0; m < 4; m++) {
                if (!f.cav[m]) continue;
                int c = 0;
                for (int q = 0; q < 8; q++) c += f.ccost[m][q];
                if (c < minc) { minc = c; c_mode = m; }
            }
        } else if (tid < 128) {
            // OneComponentChromaPrediction4x4 [J] / 8.4.2.2.2
            int uv = tid >> 6, k = tid & 63, i = k & 7, j = k >> 3;
            const uint8_t *R = uv ? d.refV : d.refU;
            int vx = s.fmv[(j >> 1) * 4 + (i >> 1)][0], vy = s.fmv[(j >> 1) * 4 + (i >> 1)][1];
            int ii = ((pix_x >> 1) + i) * 8 + vx, jj = ((pix_y >> 1) + j) * 8 + vy;
            int x0 = iclip(0, Wc - 1, ii >> 3), y0 = iclip(0, d.Hc - 1, jj >> 3);
            int x1 = iclip(0, Wc - 1, (ii + 7) >> 3), y1 = iclip(0, d.Hc - 1, (jj + 7) >> 3);
            int fx = ii & 7, fy = jj & 7;
            f.cpred[uv][0][k] = (uint8_t)(((8 - fx) * (8 - fy) * R[y0 * Wc + x0] + fx * (8 - fy) * R[y0 * Wc + x1] +
                                           (8 - fx) * fy * R[y1 * Wc + x0] + fx * fy * R[y1 * Wc + x1] + 32) >> 6);
        }
        __syncthreads();
        // dct_chroma [J] per component
        const int qpc = c_qpc[iclip(0, 51, qp + d.cqp_off)];
        const int qp_per = qpc / 6, qp_rem = qpc % 6, q_bits = 15 + qp_per;
        const int qp_const = intra_round ? (1 << q_bits) / 3 : (1 << q_bits) / 6;
        if (tid < 8) {
            int uv = tid >> 2, b = tid & 3, xo = (b & 1) * 4, yo = (b >> 1) * 4;
            const uint8_t *pr = f.cpred[uv][is_intra ? c_mode : 0];
            int *m = f.cm[uv][b];
            for (int y = 0; y < 4; y++)
                for (int x = 0; x < 4; x++) m[4 * y + x] = s.orgc[uv][(yo + y) * 8 + xo + x] - pr[(yo + y) * 8 + xo + x];
            fwd4x4(m);
        }
        __syncthreads();
        if (tid < 2) {
            int uv = tid;
            int(*m)[16] = f.cm[uv];
            int m1[4] = {m[0][0] + m[1][0] + m[2][0] + m[3][0], m[0][0] - m[1][0] + m[2][0] - m[3][0],
                         m[0][0] + m[1][0] - m[2][0] - m[3][0], m[0][0] - m[1][0] - m[2][0] + m[3][0]};
            int dcnz = 0;
            for (int k = 0; k < 4; k++) {
                int level = (abs(m1[k]) * c_quant[qp_rem][0] + 2 * qp_const) >> (q_bits + 1);
                if (level) dcnz = 1;
                f.cdc[uv][k] = (int16_t)isign(level, m1[k]);
            }
            int c0 = f.cdc[uv][0], c1 = f.cdc[uv][1], c2 = f.cdc[uv][2], c3 = f.cdc[uv][3];
            int fv[4] = {c0 + c1 + c2 + c3, c0 - c1 + c2 - c3, c0 + c1 - c2 - c3, c0 - c1 - c2 + c3};
            int v00 = c_dequant[qp_rem][0];
            for (int k = 0; k < 4; k++) f.cdcq[uv][k] = ((fv[k] * 16 * v00) << qp_per) >> 5;
            int coeff_cost = 0, acany = 0;
            for (int b = 0; b < 4; b++) {
                int run = -1;
                f.cac[uv][b][0] = 0;
                for (int k = 1; k < 16; k++) {
                    int pos = c_scan[k];
                    run++;
                    int level = (abs(m[b][pos]) * c_quant[qp_rem][pos] + qp_const) >> q_bits;
                    int ilev = 0;
                    if (level) {
                        coeff_cost += level > 1 ? MAX_VALUE : c_coeff_cost[run];
                        acany = 1;
                        run = -1;
                        ilev = level * c_dequant[qp_rem][pos] << qp_per;
                    }
                    f.cac[uv][b][k] = (int16_t)isign(level, m[b][pos]);
                    m[b][pos] = isign(ilev, m[b][pos]);
                }
            }
            if (coeff_cost < 4) {
                acany = 0;
                for (int b = 0; b < 4; b++)
                    for (int k = 1; k < 16; k++) { f.cac[uv][b][k] = 0; m[b][c_scan[k]] = 0; }
            }
            f.cfcost[uv] = (acany ? 2 : 0) | (dcnz ? 1 : 0);
        }
        __syncthreads();
        if (tid < 8) {
            int uv = tid >> 2, b = tid & 3, xo = (b & 1) * 4, yo = (b >> 1) * 4;
            int *m = f.cm[uv][b];
            m[0] = f.cdcq[uv][b];
            const uint8_t *pr = f.cpred[uv][is_intra ? c_mode : 0];
            inv4x4_add(m, pr + yo * 8 + xo, 8, f.cfin[uv] + yo * 8 + xo, 8);
        }
        __syncthreads();
        int cr = 0;
        for (int uv = 0; uv < 2; uv++) {
            if (f.cfcost[uv] & 1) cr = max(cr, 1);
            if (f.cfcost[uv] & 2) cr = 2;
        }
        cbp |= cr << 4;
        // ======== outputs
        jmh_mb_result *res = d.res + mby * d.mbw + mbx;
        int mb_type = best_mode;
        if (slice_p && best_mode == 1 && cbp == 0 && s.fmv[0][0] == skipx && s.fmv[0][1] == skipy) mb_type = JMH_PSKIP;
        if (tid == 0) {
            res->mb_type = (int16_t)mb_type;
            res->cbp = (int16_t)cbp;
            res->cbp_blk = cbp_blk;
            for (int b = 0; b < 4; b++) {
                res->b8mode[b] = (int8_t)(mb_type == JMH_PSKIP ? 0 : b8mode[b]);
                res->ref_idx[b] = (int8_t)(is_intra ? -1 : 0);
            }
            res->i16mode = (int8_t)(best_mode == JMH_I16MB ? i16mode : 0);
            res->c_ipred_mode = (int8_t)(is_intra ? c_mode : 0);
            res->pad0[0] = res->pad0[1] = 0;
            res->min_cost = min_cost;
            res->reserved = 0;
        }
        if (tid < 16) {
            int k = tid;
            int ip = best_mode == JMH_I4MB ? s.ipred_cur[k] : 2;
            res->ipred[k] = (int8_t)ip;
            res->mv[k][0] = s.fmv[k][0]; res->mv[k][1] = s.fmv[k][1];
            for (int q = 0; q < 16; q++) res->luma[k][q] = f.lev[k][q];
            res->luma_dc[k] = best_mode == JMH_I16MB ? f.dclev[k] : 0;
            int a = ((pix_y >> 2) + (k >> 2)) * W4 + (pix_x >> 2) + (k & 3);
            d.mv[2 * a] = s.fmv[k][0]; d.mv[2 * a + 1] = s.fmv[k][1];
            d.refidx[a] = (int8_t)(is_intra ? -1 : 0);
            d.ipred[a] = (int8_t)ip;
        }
        if (tid < 8) { int uv = tid >> 2, k = tid & 3; res->chroma_dc[uv][k] = f.cdc[uv][k]; }
        if (tid < 128) {
            int uv = tid >> 6, b = (tid >> 4) & 3, q = tid & 15;
            res->chroma_ac[uv][b][q] = f.cac[uv][b][q];
            int k = tid & 63;
            (uv ? d.recV : d.recU)[((pix_y >> 1) + (k >> 3)) * Wc + (pix_x >> 1) + (k & 7)] = f.cfin[uv][k];
        }
        d.recY[(pix_y + (tid >> 4)) * W + pix_x + (tid & 15)] = s.rec[tid];
    }
}

// ======================================================================================
//  unit seams
// ======================================================================================
__global__ __launch_bounds__(256) void k_sad_table(const uint8_t *__restrict__ org, const uint8_t *__restrict__ ref, int W, int H,
                                                   int sr, const int32_t *mb_xy, const int32_t *centres, uint16_t *out) {
    int i = blockIdx.y;
    int side = 2 * sr + 1, npos = side * side;
    int r = blockIdx.x * 256 + threadIdx.x;
    if (r >= npos) return;
    int px = 16 * mb_xy[2 * i], py = 16 * mb_xy[2 * i + 1];
    int dx = r % side - sr + centres[2 * i], dy = r / side - sr + centres[2 * i + 1];
    for (int b = 0; b < 16; b++) {
        int ox = (b & 3) * 4, oy = (b >> 2) * 4, sad = 0;
        for (int y = 0; y < 4; y++)
            for (int x = 0; x < 4; x++)
                sad += abs(org[(py + oy + y) * W + px + ox + x] -
                           ref[iclip(0, H - 1, py + dy + oy + y) * W + iclip(0, W - 1, px + dx + ox + x)]);
        out[((size_t)i * 16 + b) * npos + r] = (uint16_t)sad;
    }
}

__global__ __launch_bounds__(256) void k_tq4x4(int n, const int16_t *resid, const uint8_t *pred, int qp, int intra, int16_t *levels,
                                               uint8_t *recon, int32_t *coeff_cost, int32_t *nonzero) {
    int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    int r[16], cc = 0;
    for (int k = 0; k < 16; k++) r[k] = resid[16 * i + k];
    nonzero[i] = dct_luma4x4(r, pred + 16 * i, 4, qp, intra, levels + 16 * i, &cc, recon + 16 * i, 4);
    coeff_cost[i] = cc;
}

// ---- launchers (host side, same translation unit) --------------------------------------
hipError_t jmh_launch_interp(const uint8_t *ref, int W, int H, uint8_t *qpel, int qstride, int qplane, hipStream_t st) {
    dim3 grid((qstride + 63) / 64, (H + 2 * QPAD + 3) / 4);
    hipLaunchKernelGGL(k_interp, grid, dim3(256), 0, st, ref, W, H, qpel, qstride, qplane);
    return hipGetLastError();
}
hipError_t jmh_launch_mb(const DevParams &p, int nblocks, hipStream_t st) {
    hipLaunchKernelGGL(k_mb_encode, dim3(nblocks), dim3(NT), 0, st, p);
    return hipGetLastError();
}
hipError_t jmh_launch_sad_table(const uint8_t *org, const uint8_t *ref, int W, int H, int sr, int n_mb, const int32_t *mb_xy,
                                const int32_t *centres, uint16_t *out, hipStream_t st) {
    int side = 2 * sr + 1, npos = side * side;
    hipLaunchKernelGGL(k_sad_table, dim3((npos + 255) / 256, n_mb), dim3(256), 0, st, org, ref, W, H, sr, mb_xy, centres, out);
    return hipGetLastError();
}
hipError_t jmh_launch_tq4x4(int n, const int16_t *resid, const uint8_t *pred, int qp, int intra, int16_t *levels, uint8_t *recon,
                            int32_t *cc, int32_t *nz, hipStream_t st) {
    hipLaunchKernelGGL(k_tq4x4, dim3((n + 255) / 256), dim3(256), 0, st, n, resid, pred, qp, intra, levels, recon, cc, nz);
    return hipGetLastError();
}
