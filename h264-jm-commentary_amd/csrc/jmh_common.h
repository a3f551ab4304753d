// jmh_common.h — device helpers shared by the gfx950 kernels: JM tables, H.264 integer
// arithmetic, 16-lane transform primitives (wave shuffles / DPP), SATD, MV prediction.
// Every translation unit gets its own (static) copy of the constant tables.
#pragma once
#include "jmh_device.h"

#define MAX_VALUE 999999
#define WM 4                                  // window margin (6-tap support of sub-pel samples)
#define WIN_DIM_MAX (2 * SRMAX + 16 + 2 * WM) // 88
#define WST 92                                // window row stride (>= WIN_DIM_MAX + 3, mult of 4)

// quantisation / dequantisation coefficients by class: (even,even), (odd,odd), mixed
static __constant__ int c_q3[6][3] = {{13107, 5243, 8066}, {11916, 4660, 7490}, {10082, 4194, 6554},
                                      {9362, 3647, 5825},  {8192, 3355, 5243},  {7282, 2893, 4559}};
static __constant__ int c_dq3[6][3] = {{10, 16, 13}, {11, 18, 14}, {13, 20, 16}, {14, 23, 18}, {16, 25, 20}, {18, 29, 23}};
static __constant__ int c_qpc[52] = {0,  1,  2,  3,  4,  5,  6,  7,  8,  9,  10, 11, 12, 13, 14, 15, 16, 17,
                                     18, 19, 20, 21, 22, 23, 24, 25, 26, 27, 28, 29, 29, 30, 31, 32, 32, 33,
                                     34, 34, 35, 35, 36, 36, 37, 37, 37, 38, 38, 38, 39, 39, 39, 39};
static __constant__ int c_blc[8][2] = {{16, 16}, {16, 16}, {16, 8}, {8, 16}, {8, 8}, {8, 4}, {4, 8}, {4, 4}};
// sub-pel candidate offsets = spiral entries 0..8 (Init_Motion_Search_Module [J])
static __constant__ int c_sp9[9][2] = {{0, 0}, {0, -1}, {0, 1}, {-1, -1}, {1, -1}, {-1, 0}, {1, 0}, {-1, 1}, {1, 1}};
// quarter-pel sample = average of two half-pel-grid samples A, B per phase ((G+b+1)>>1 ...
// (m+s+1)>>1, H.264 8.4.2.2.1; a full/half sample has A == B). Offsets in half-grid units
// packed as nibbles dxA, dyA, dxB, dyB (high to low); phase = (qy & 3) * 4 + (qx & 3).
static __constant__ uint16_t c_qoff[16] = {
    0x0000, 0x0010, 0x1010, 0x2010,   // G, a, b, c
    0x0001, 0x1001, 0x1011, 0x1021,   // d, e, f, g
    0x0101, 0x0111, 0x1111, 0x1121,   // h, i, j, k
    0x0201, 0x0112, 0x1112, 0x2112};  // n, p, q, r
// the same two tables as immediates (no memory access; index may vary across lanes)
__device__ __forceinline__ int sp9x(int c) { return ((0x22215 >> (2 * c)) & 3) - 1; }
__device__ __forceinline__ int sp9y(int c) { return ((0x29421 >> (2 * c)) & 3) - 1; }
__device__ __forceinline__ int qoff(int ph) {
    const uint64_t q = ph < 8 ? (ph < 4 ? 0x2010101000100000ULL : 0x1021101110010001ULL)
                              : (ph < 12 ? 0x1121111101110101ULL : 0x2112111201120201ULL);
    return (int)((q >> (16 * (ph & 3))) & 0xFFFF);
}
// block type (1..7 = 16x16, 16x8, 8x16, 8x8, 8x4, 4x8, 4x4) -> log2 of width / 4 and height / 4
__device__ __forceinline__ int lw4_of(int bt) { return bt <= 2 ? 2 : (bt <= 5 ? 1 : 0); }
__device__ __forceinline__ int lh4_of(int bt) { return (bt == 1 || bt == 3) ? 2 : (bt == 2 || bt == 4 || bt == 6) ? 1 : 0; }
// 4x4 frame zig-zag (scan position -> raster), packed as nibbles
#define SCAN_PACKED 0xFEB7ADC963258410ULL
__device__ __forceinline__ int scan_of(int k) { return (int)((SCAN_PACKED >> (4 * k)) & 15); }

__device__ __forceinline__ int iclip(int lo, int hi, int v) { return v < lo ? lo : (v > hi ? hi : v); }
__device__ __forceinline__ int clip255(int v) { return v < 0 ? 0 : (v > 255 ? 255 : v); }
__device__ __forceinline__ int clipmx(int v, int maxv) { return v < 0 ? 0 : (v > maxv ? maxv : v); }   // Clip1
__device__ __forceinline__ int isign(int a, int b) { return b < 0 ? -abs(a) : abs(a); }
__device__ __forceinline__ int mvbits(int v) { return v == 0 ? 1 : 2 * (31 - __clz(abs(v))) + 3; }
__device__ __forceinline__ int tap6(int a, int b, int c, int d, int e, int f) { return a - 5 * b + 20 * c + 20 * d - 5 * e + f; }
// JM spiral index of relative position (x, y) (Init_Motion_Search_Module ordering)
// ---- quarter-pel samples straight from the reference (H.264 8.4.2.2.1, spec clamping) ----
template <class T>
__device__ __forceinline__ int rpx(const T *p, int w, int h, int x, int y) { return p[iclip(0, h - 1, y) * w + iclip(0, w - 1, x)]; }
__device__ __forceinline__ int hb1(const uint8_t *p, int w, int h, int x, int y) {
    return tap6(rpx(p, w, h, x - 2, y), rpx(p, w, h, x - 1, y), rpx(p, w, h, x, y), rpx(p, w, h, x + 1, y), rpx(p, w, h, x + 2, y),
                rpx(p, w, h, x + 3, y));
}
__device__ __forceinline__ int vh1(const uint8_t *p, int w, int h, int x, int y) {
    return tap6(rpx(p, w, h, x, y - 2), rpx(p, w, h, x, y - 1), rpx(p, w, h, x, y), rpx(p, w, h, x, y + 1), rpx(p, w, h, x, y + 2),
                rpx(p, w, h, x, y + 3));
}
// one luma sample at quarter-pel position (X, Y) (units of 1/4 pel) from integer samples px(x, y):
// only the half-pel samples the phase needs (G, b, h, s, m, j of Figure 8-4), same values as
// k_interp's 16 planes; maxv = (1 << BitDepthY) - 1 (Clip1Y).  SERIAL_J: the centre sample j's six
// columns one loop iteration at a time (six loads live instead of 36: no spills in a 64-VGPR kernel)
template <class PX, bool SERIAL_J = false>
__device__ __forceinline__ int qpel_from(PX px, int X, int Y, int maxv = 255) {
    const int x = X >> 2, y = Y >> 2, fx = X & 3, fy = Y & 3;
    auto hb1p = [&](int xx, int yy) { return tap6(px(xx - 2, yy), px(xx - 1, yy), px(xx, yy), px(xx + 1, yy), px(xx + 2, yy), px(xx + 3, yy)); };
    auto vh1p = [&](int xx, int yy) { return tap6(px(xx, yy - 2), px(xx, yy - 1), px(xx, yy), px(xx, yy + 1), px(xx, yy + 2), px(xx, yy + 3)); };
    auto hb = [&](int xx, int yy) { return iclip(0, maxv, (hb1p(xx, yy) + 16) >> 5); };
    auto vb = [&](int xx, int yy) { return iclip(0, maxv, (vh1p(xx, yy) + 16) >> 5); };
    if (fy == 0) {
        const int G = px(x, y);
        if (fx == 0) return G;
        const int b = hb(x, y);
        return fx == 2 ? b : ((fx == 1 ? G : px(x + 1, y)) + b + 1) >> 1;
    }
    if (fx == 0) {
        const int h = vb(x, y);
        return fy == 2 ? h : ((fy == 1 ? px(x, y) : px(x, y + 1)) + h + 1) >> 1;
    }
    if ((fx & 1) && (fy & 1)) return (hb(x, fy == 1 ? y : y + 1) + vb(fx == 1 ? x : x + 1, y) + 1) >> 1;   // e g p r
    int j1 = 0;
    if constexpr (SERIAL_J) {
#pragma unroll 1
        for (int k = 0; k < 6; k++) j1 += (k == 0 || k == 5 ? 1 : (k == 1 || k == 4 ? -5 : 20)) * vh1p(x - 2 + k, y);
    } else {
#pragma unroll
        for (int k = 0; k < 6; k++) j1 += (k == 0 || k == 5 ? 1 : (k == 1 || k == 4 ? -5 : 20)) * vh1p(x - 2 + k, y);
    }
    const int j = iclip(0, maxv, (j1 + 512) >> 10);
    if (fx == 2 && fy == 2) return j;
    const int o = fx == 2 ? hb(x, fy == 1 ? y : y + 1) : vb(fx == 1 ? x : x + 1, y);   // f q / i k
    return (j + o + 1) >> 1;
}
// ... straight from the reference picture in HBM, spec coordinate clamping (k_mb_final MC)
template <class T, bool SERIAL_J = false>
__device__ __forceinline__ int qpel_direct(const T *ref, int W, int H, int X, int Y, int maxv = 255) {
    auto px = [&](int x, int y) { return rpx(ref, W, H, x, y); };
    return qpel_from<decltype(px), SERIAL_J>(px, X, Y, maxv);
}

__device__ __forceinline__ int spiral_index(int x, int y) {
    int ax = abs(x), ay = abs(y), l = max(ax, ay);
    if (l == 0) return 0;
    int base = (2 * l - 1) * (2 * l - 1);
    if (ay == l && ax < l) return base + 2 * (x + l - 1) + (y > 0);
    return base + 2 * (2 * l - 1) + 2 * (y + l) + (x > 0);
}
__device__ __forceinline__ void spiral_pos(int k, int &x, int &y) {
    if (k == 0) { x = y = 0; return; }
    int l = max(1, (int)((sqrtf((float)k) + 1.0f) * 0.5f));   // ring: (2l-1)^2 <= k < (2l+1)^2
    if ((2 * l + 1) * (2 * l + 1) <= k) l++;
    if ((2 * l - 1) * (2 * l - 1) > k) l--;
    int o = k - (2 * l - 1) * (2 * l - 1);
    if (o < 2 * (2 * l - 1)) { x = (o >> 1) - l + 1; y = (o & 1) ? l : -l; }
    else { o -= 2 * (2 * l - 1); y = (o >> 1) - l; x = (o & 1) ? l : -l; }
}
// COEFF_COST [J] of a |level| == 1 coefficient by preceding zero run
__device__ __forceinline__ int coeff_cost_run(int run) { return run == 0 ? 3 : run <= 2 ? 2 : run <= 5 ? 1 : 0; }

// 4 bytes at any byte address of LDS: two aligned LDS dwords + v_alignbyte.  The pointer is cast
// to the LDS address space before its low bits are taken: through a generic integer the reads
// become flat loads (the vector memory path, waited on with vmcnt) instead of one ds_read2_b32.
// Every caller passes an LDS address.
typedef __attribute__((address_space(3))) const uint32_t lds_cu32;
typedef __attribute__((address_space(3))) const uint8_t lds_cu8;
__device__ __forceinline__ uint32_t lds_u32_any(const void *p) {
    const uint32_t a = (uint32_t)(uintptr_t)(lds_cu8 *)p;
    lds_cu32 *q = (lds_cu32 *)(uintptr_t)(a & ~3u);
    return __builtin_amdgcn_alignbyte(q[1], q[0], a & 3);
}

// ---- cross-lane helpers ----------------------------------------------------------------
// DPP lane moves: quad_perm [1,0,3,2] (0xB1), [2,3,0,1] (0x4E), [3,2,1,0] (0x1B),
// row_half_mirror (0x141), row_mirror (0x140), row_ror:8 (0x128) — all within a 16-lane row
// A disabled source lane reads 0 (bound_ctrl): with that (or an identity old value, dpp_umin)
// the compiler folds the move into the consuming v_add / v_sub / v_min as a DPP operand, one
// instruction instead of a copy, a v_mov_dpp and the operation.  Every caller runs its rows fully
// active (a lane's result is used only where every lane its reduction reads was active).
#ifndef JMH_DPP_FOLD
#define JMH_DPP_FOLD 1                        // A/B: 0 = the earlier update_dpp(v, v) moves
#endif
template <int CTRL>
__device__ __forceinline__ int dpp(int v) {
#if JMH_DPP_FOLD
    return __builtin_amdgcn_update_dpp(0, v, CTRL, 0xF, 0xF, true);
#else
    return __builtin_amdgcn_update_dpp(v, v, CTRL, 0xF, 0xF, false);
#endif
}
// min(v, v of the DPP source lane) with 0xFFFFFFFF as the old value: folds into v_min_u32_dpp, and
// a disabled source lane leaves v unchanged
template <int CTRL>
__device__ __forceinline__ unsigned dpp_umin(unsigned v) {
#if JMH_DPP_FOLD
    return min(v, (unsigned)__builtin_amdgcn_update_dpp(-1, (int)v, CTRL, 0xF, 0xF, false));
#else
    return min(v, (unsigned)__builtin_amdgcn_update_dpp((int)v, (int)v, CTRL, 0xF, 0xF, false));
#endif
}
// sum over each aligned 16-lane row (all 16 lanes must be active); every lane gets the sum
__device__ __forceinline__ int row16_sum(int v) {
    v += dpp<0xB1>(v);
    v += dpp<0x4E>(v);
    v += dpp<0x141>(v);
    v += dpp<0x140>(v);
    return v;
}
// 4x4 Hadamard of a block held one sample per lane (l = 4y + x) of a 16-lane row: four
// butterfly stages over lane ^1, ^2 (quad_perm), ^4 (half_mirror + quad reverse), ^8 (row_ror:8).
// Outputs are the 16 Walsh coefficients in butterfly order (sums of |.| are order-free).
__device__ __forceinline__ int row16_had(int v, int l) {
    int p = dpp<0xB1>(v);
    v = (l & 1) ? p - v : v + p;
    p = dpp<0x4E>(v);
    v = (l & 2) ? p - v : v + p;
    p = dpp<0x1B>(dpp<0x141>(v));
    v = (l & 4) ? p - v : v + p;
    p = dpp<0x128>(v);
    v = (l & 8) ? p - v : v + p;
    return v;
}
// minimum over the whole (fully active) wave, wave-uniform result
__device__ __forceinline__ unsigned wave_min_u32(unsigned v) {
    v = dpp_umin<0xB1>(v);
    v = dpp_umin<0x4E>(v);
    v = dpp_umin<0x141>(v);
    v = dpp_umin<0x140>(v);
    unsigned a = __builtin_amdgcn_readlane(v, 0), b = __builtin_amdgcn_readlane(v, 16);
    unsigned c = __builtin_amdgcn_readlane(v, 32), e = __builtin_amdgcn_readlane(v, 48);
    return min(min(a, b), min(c, e));
}
// compiler + hardware ordering of LDS traffic between lanes of one wave (wave-synchronous code)
__device__ __forceinline__ void wave_lds_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// ======================================================================================
//  16-lane 4x4 transform primitives (lane l of a 16-lane group holds raster element l)
// ======================================================================================
__device__ __forceinline__ int g16(int v, int src) { return __shfl(v, (int)(threadIdx.x & 48) + src, 64); }

// The output of a 4x4 butterfly stage at position k (a lane's x or y) is one expression with per-lane coefficients: a ?: chain
// over four different sums compiles to divergent branches.
//   forward, position k of (p0, p1, p2, p3) = (v0 + v3, v1 + v2, v1 - v2, v0 - v3):
//     k 0: p0 + p1, 1: 2 p3 + p2, 2: p0 - p1, 3: p3 - 2 p2  =  ca * (k odd ? p3 : p0) + cb * (k odd ? p2 : p1)
__device__ __forceinline__ int fwd_tap(int p0, int p1, int p2, int p3, int k) {
    const int a = (k & 1) ? p3 : p0, b = (k & 1) ? p2 : p1;
    const int ca = k == 1 ? 2 : 1, cb = k < 2 ? 1 : k == 2 ? -1 : -2;
    return ca * a + cb * b;
}
//   inverse, (e0, e1, e2, e3) = (d0 + d2, d0 - d2, (d1 >> 1) - d3, d1 + (d3 >> 1)):
//     k 0: e0 + e3, 1: e1 + e2, 2: e1 - e2, 3: e0 - e3  =  (k 0/3 ? e0 : e1) +- (k 0/3 ? e3 : e2)
__device__ __forceinline__ int inv_tap(int e0, int e1, int e2, int e3, int k) {
    const bool outer = k == 0 || k == 3;
    const int a = outer ? e0 : e1, b = outer ? e3 : e2;
    return k < 2 ? a + b : a - b;
}
#ifndef JMH_LANE_TAPS
#define JMH_LANE_TAPS 1                       // A/B: 0 = the ?: chains in lane_fwd4x4 / lane_inv4x4
#endif
// forward 4x4 core transform (dct_luma [J]): rows then columns
__device__ __forceinline__ int lane_fwd4x4(int r, int l) {
    int y = l >> 2, x = l & 3;
    int v0 = g16(r, 4 * y), v1 = g16(r, 4 * y + 1), v2 = g16(r, 4 * y + 2), v3 = g16(r, 4 * y + 3);
    int p0 = v0 + v3, p3 = v0 - v3, p1 = v1 + v2, p2 = v1 - v2;
#if JMH_LANE_TAPS
    const int t = fwd_tap(p0, p1, p2, p3, x);
    const int u0 = g16(t, x), u1 = g16(t, 4 + x), u2 = g16(t, 8 + x), u3 = g16(t, 12 + x);
    return fwd_tap(u0 + u3, u1 + u2, u1 - u2, u0 - u3, y);
#else
    int t = x == 0 ? p0 + p1 : x == 1 ? 2 * p3 + p2 : x == 2 ? p0 - p1 : p3 - 2 * p2;
    int u0 = g16(t, x), u1 = g16(t, 4 + x), u2 = g16(t, 8 + x), u3 = g16(t, 12 + x);
    p0 = u0 + u3; p3 = u0 - u3; p1 = u1 + u2; p2 = u1 - u2;
    return y == 0 ? p0 + p1 : y == 1 ? 2 * p3 + p2 : y == 2 ? p0 - p1 : p3 - 2 * p2;
#endif
}
// inverse 4x4 (8.5.12.2, rows first) + reconstruction clip((x + (pred << 6) + 32) >> 6) to maxv
__device__ __forceinline__ int lane_inv4x4(int dq, int l, int pred, int maxv = 255) {
    int y = l >> 2, x = l & 3;
    int d0 = g16(dq, 4 * y), d1 = g16(dq, 4 * y + 1), d2 = g16(dq, 4 * y + 2), d3 = g16(dq, 4 * y + 3);
    int e0 = d0 + d2, e1 = d0 - d2, e2 = (d1 >> 1) - d3, e3 = d1 + (d3 >> 1);
#if JMH_LANE_TAPS
    const int t = inv_tap(e0, e1, e2, e3, x);
    const int f0 = g16(t, x), f1 = g16(t, 4 + x), f2 = g16(t, 8 + x), f3 = g16(t, 12 + x);
    const int o = inv_tap(f0 + f2, f0 - f2, (f1 >> 1) - f3, f1 + (f3 >> 1), y);
#else
    int t = x == 0 ? e0 + e3 : x == 1 ? e1 + e2 : x == 2 ? e1 - e2 : e0 - e3;
    int f0 = g16(t, x), f1 = g16(t, 4 + x), f2 = g16(t, 8 + x), f3 = g16(t, 12 + x);
    e0 = f0 + f2; e1 = f0 - f2; e2 = (f1 >> 1) - f3; e3 = f1 + (f3 >> 1);
    int o = y == 0 ? e0 + e3 : y == 1 ? e1 + e2 : y == 2 ? e1 - e2 : e0 - e3;
#endif
    return iclip(0, maxv, (o + (pred << 6) + 32) >> 6);
}
// quantisation rounding offset at q_bits (docs/JM_SEMANTICS.md items 1 and 45; oracle jmo_qround):
//   sel 0 / 1 = JM 8.6 (1 << q_bits) / 6 (P slice) / 3 (I slice, and Intra16x16 always);
//   sel 2 + o = JM >= 10 flat OffsetMatrix entry o at OffsetBits 11: o << (q_bits - 11)
__device__ __forceinline__ int q_round(int sel, int q_bits) {
    return sel >= 2 ? (sel - 2) << (q_bits - 11) : sel ? (1 << q_bits) / 3 : (1 << q_bits) / 6;
}
// the Intra16x16 selector: JM 8.6 always rounds dct_luma_16x16 with / 3
__device__ __forceinline__ int q_sel16(int sel) { return sel >= 2 ? sel : 1; }
// quantisation (dct_luma / dct_chroma AC [J]) of coefficient c at raster l.
//   lev_scan: signed level at SCAN position l; dq: dequantised coefficient at raster l;
//   cost: COEFF_COST sum over the block (all 16 lanes); returns the scan-order non-zero mask.
__device__ __forceinline__ unsigned lane_quant(int c, int l, int qp, int qp_const, bool ac_only, int &lev_scan, int &dq, int &cost) {
    const int qp_per = qp / 6, qp_rem = qp % 6, q_bits = 15 + qp_per;
    const int x = l & 3, y = l >> 2;
    const int cls = ((x | y) & 1) == 0 ? 0 : ((x & y) & 1) ? 1 : 2;
    // the three scalings of qp_rem as wave-uniform values (scalar loads), then a per-lane select:
    // without the readfirstlane the compiler folds the select into a per-lane indexed load, a
    // vector memory round trip inside every block's dependent chain
    const int q0 = __builtin_amdgcn_readfirstlane(c_q3[qp_rem][0]), q1 = __builtin_amdgcn_readfirstlane(c_q3[qp_rem][1]);
    const int q2 = __builtin_amdgcn_readfirstlane(c_q3[qp_rem][2]);
    const int d0 = __builtin_amdgcn_readfirstlane(c_dq3[qp_rem][0]), d1 = __builtin_amdgcn_readfirstlane(c_dq3[qp_rem][1]);
    const int d2 = __builtin_amdgcn_readfirstlane(c_dq3[qp_rem][2]);
    const int qc = cls == 0 ? q0 : cls == 1 ? q1 : q2;
    const int dqc = cls == 0 ? d0 : cls == 1 ? d1 : d2;
    int level = (abs(c) * qc + qp_const) >> q_bits;
    if (ac_only && l == 0) level = 0;
    const int dqm = level * dqc << qp_per;    // |level| x scale: the sign of c, 0 for a zero level
    dq = c < 0 ? -dqm : dqm;
    const int sr = scan_of(l);
    const int lvs = g16(level, sr), cs = g16(c, sr);
    const unsigned long long bal = __ballot(lvs != 0);
    const unsigned m = (unsigned)(bal >> (threadIdx.x & 48)) & 0xFFFFu;
    int k = 0;
    if (lvs) {
        unsigned below = m & ((1u << l) - 1u);
        int prev = below ? 31 - __clz(below) : (ac_only ? 0 : -1);
        k = lvs > 1 ? MAX_VALUE : coeff_cost_run(l - prev - 1);
    }
    cost = row16_sum(k);
    lev_scan = lvs ? isign(lvs, cs) : 0;
    return m;
}

// single-thread SATD() [J]: 4x4 Hadamard sum >> 1, or SAD
__device__ __forceinline__ int satd4x4(const int d[16], int had) {
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
// 16-lane sum of |4x4 Hadamard| (no >>1); every lane of the (fully active) row gets the sum
__device__ __forceinline__ int lane_had_abs(int dv, int l) { return row16_sum(abs(row16_had(dv, l))); }
// 16-lane SATD() [J]
__device__ __forceinline__ int lane_satd(int dv, int l, int had) {
    return had ? lane_had_abs(dv, l) >> 1 : row16_sum(abs(dv));
}

// SetMotionVectorPredictor [J] / H.264 8.4.1.3 (list 0, ref 0). NB(xN, yN, ref, mx, my)
// returns the availability of the 4x4 neighbour covering MB-relative pixel (xN, yN).
template <class NB>
__device__ __forceinline__ void set_mvp(const NB &nb, int bx4, int by4, int bsx, int bsy, int &px, int &py) {
    int mb_x = 4 * bx4, mb_y = 4 * by4;
    int ra = -1, rb = -1, rc = -1, rd = -1, ax = 0, ay = 0, bxv = 0, byv = 0, cx = 0, cy = 0, dx = 0, dy = 0;
    bool av_a = nb(mb_x - 1, mb_y, ra, ax, ay);
    bool av_b = nb(mb_x, mb_y - 1, rb, bxv, byv);
    bool av_c = nb(mb_x + bsx, mb_y - 1, rc, cx, cy);
    bool av_d = nb(mb_x - 1, mb_y - 1, rd, dx, dy);
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

// neighbour k (0 A, 1 B, 2 C, or D when C is not available, as in set_mvp) of a block
template <class NB>
__device__ __forceinline__ bool mvp_nbr(const NB &nb, int bx4, int by4, int bsx, int k, int &ref, int &mx, int &my) {
    const int mb_x = 4 * bx4, mb_y = 4 * by4;
    if (k == 0) return nb(mb_x - 1, mb_y, ref, mx, my);
    if (k == 1) return nb(mb_x, mb_y - 1, ref, mx, my);
    bool av_c = nb(mb_x + bsx, mb_y - 1, ref, mx, my);
    if (mb_y > 0) {
        if (mb_x < 8) {
            if (mb_y == 8) { if (bsx == 16) av_c = false; }
            else if (mb_x + bsx == 8) av_c = false;
        } else if (mb_x + bsx == 16) av_c = false;
    }
    if (!av_c) av_c = nb(mb_x - 1, mb_y - 1, ref, mx, my);
    return av_c;
}

// border neighbour cells of an MB: 0..5 = row y4 = -1 (x4 = -1..4), 6..9 = column x4 = -1 (y4 = 0..3)
struct Border {
    int16_t mv[10][2];
    int8_t ref[10];                      // -2: not available, -1: intra, 0: ref 0
    int8_t ipm[10];                      // Intra4x4PredMode, -1 unavailable
};
__device__ __forceinline__ int border_cell(int xN, int yN) {   // -1: inside the MB or unavailable
    if (yN < 0) { int b = xN >> 2; return b > 4 ? -1 : b + 1; }
    if (xN < 0) return yN > 15 ? -1 : 6 + (yN >> 2);
    return -1;
}
// prefetch by threads t < 10 of the workgroup
__device__ __forceinline__ void load_border(const DevParams &d, Border &b, int t, int mbx, int mby) {
    const int W4 = d.W >> 2;
    int by4 = t < 6 ? -1 : t - 6, bx4 = t < 6 ? t - 1 : -1;
    const MbAvail m = mb_avail(d, mbx, mby);
    bool av = by4 < 0 ? (bx4 < 0 ? m.TL : bx4 > 3 ? m.TR : m.T) : m.L;
    int ref = -2, mx = 0, my = 0, ipm = -1;
    if (av) {
        int a = (4 * mby + by4) * W4 + 4 * mbx + bx4;
        ref = d.refidx[a]; mx = d.mv[2 * a]; my = d.mv[2 * a + 1]; ipm = d.ipred[a];
        if (d.cip && ref >= 0) ipm = -1;   // UseConstrainedIntraPred: an inter neighbour sets dcPredModePredictedFlag
    }
    b.ref[t] = (int8_t)ref; b.mv[t][0] = (int16_t)mx; b.mv[t][1] = (int16_t)my; b.ipm[t] = (int8_t)ipm;
}
// neighbour view with only border cells (16x16 MVP, skip MV)
struct NbBorder {
    const Border &b;
    __device__ __forceinline__ bool operator()(int xN, int yN, int &ref, int &mx, int &my) const {
        if (yN > 15 || (xN > 15 && yN >= 0)) return false;
        int c = border_cell(xN, yN);
        if (c < 0 || b.ref[c] == -2) return false;
        ref = b.ref[c]; mx = b.mv[c][0]; my = b.mv[c][1];
        return true;
    }
};

// Intra4x4 prediction sample (8.3.1.2) of mode m at pixel (x,y); P[0] = p[-1,-1],
// P[1+i] = p[i,-1] (i = 0..7), P[9+j] = p[-1,j]
__device__ __forceinline__ int i4_pred_px(const int *P, int up, int left, int m, int x, int y) {
#define PT(i) P[1 + (i)]
#define PL(j) ((j) < 0 ? P[0] : P[9 + (j)])
    switch (m) {
    case 0: return PT(x);
    case 1: return PL(y);
    case 2:
        if (up && left) return (PT(0) + PT(1) + PT(2) + PT(3) + PL(0) + PL(1) + PL(2) + PL(3) + 4) >> 3;
        if (left) return (PL(0) + PL(1) + PL(2) + PL(3) + 2) >> 2;
        if (up) return (PT(0) + PT(1) + PT(2) + PT(3) + 2) >> 2;
        return 128;
    case 3: return (x == 3 && y == 3) ? (PT(6) + 3 * PT(7) + 2) >> 2 : (PT(x + y) + 2 * PT(x + y + 1) + PT(x + y + 2) + 2) >> 2;
    case 4:
        if (x > y) return (PT(x - y - 2) + 2 * PT(x - y - 1) + PT(x - y) + 2) >> 2;
        if (x < y) return (PL(y - x - 2) + 2 * PL(y - x - 1) + PL(y - x) + 2) >> 2;
        return (PT(0) + 2 * P[0] + PL(0) + 2) >> 2;
    case 5: {
        int z = 2 * x - y;
        if (z >= 0 && !(z & 1)) return (PT(x - (y >> 1) - 1) + PT(x - (y >> 1)) + 1) >> 1;
        if (z >= 0) return (PT(x - (y >> 1) - 2) + 2 * PT(x - (y >> 1) - 1) + PT(x - (y >> 1)) + 2) >> 2;
        if (z == -1) return (PL(0) + 2 * P[0] + PT(0) + 2) >> 2;
        return (PL(y - 1) + 2 * PL(y - 2) + PL(y - 3) + 2) >> 2;
    }
    case 6: {
        int z = 2 * y - x;
        if (z >= 0 && !(z & 1)) return (PL(y - (x >> 1) - 1) + PL(y - (x >> 1)) + 1) >> 1;
        if (z >= 0) return (PL(y - (x >> 1) - 2) + 2 * PL(y - (x >> 1) - 1) + PL(y - (x >> 1)) + 2) >> 2;
        if (z == -1) return (PL(0) + 2 * P[0] + PT(0) + 2) >> 2;
        return (PT(x - 1) + 2 * PT(x - 2) + PT(x - 3) + 2) >> 2;
    }
    case 7:
        return (y & 1) ? (PT(x + (y >> 1)) + 2 * PT(x + (y >> 1) + 1) + PT(x + (y >> 1) + 2) + 2) >> 2
                       : (PT(x + (y >> 1)) + PT(x + (y >> 1) + 1) + 1) >> 1;
    default: {
        int z = x + 2 * y;
        if (z > 5) return PL(3);
        if (z == 5) return (PL(2) + 3 * PL(3) + 2) >> 2;
        if (!(z & 1)) return (PL(y + (x >> 1)) + PL(y + (x >> 1) + 1) + 1) >> 1;
        return (PL(y + (x >> 1)) + 2 * PL(y + (x >> 1) + 1) + PL(y + (x >> 1) + 2) + 2) >> 2;
    }
    }
#undef PT
#undef PL
}

// chroma DC prediction of one 4x4 chroma block (8.3.4.1-3); dcd = 1 << (BitDepthC - 1)
template <class pel>
__device__ __forceinline__ int chroma_dc(const pel *T, const pel *L, int up, int left, int b, int dcd) {
    int s0 = 0, s1 = 0, s2 = 0, s3 = 0;
    for (int i = 0; i < 4; i++) { s0 += T[i]; s1 += T[4 + i]; s2 += L[i]; s3 += L[4 + i]; }
    if (b == 0) return (up && left) ? (s0 + s2 + 4) >> 3 : up ? (s0 + 2) >> 2 : left ? (s2 + 2) >> 2 : dcd;
    if (b == 1) return up ? (s1 + 2) >> 2 : left ? (s2 + 2) >> 2 : dcd;
    if (b == 2) return left ? (s3 + 2) >> 2 : up ? (s0 + 2) >> 2 : dcd;
    return (up && left) ? (s1 + s3 + 4) >> 3 : up ? (s1 + 2) >> 2 : left ? (s3 + 2) >> 2 : dcd;
}
// chroma intra prediction (8.3.4) of mode m at pixel (x, y) of one component (Clip1C to maxv)
template <class pel>
__device__ __forceinline__ int chroma_pred_px(const pel *T, const pel *L, int Pc, int up, int left, int m, int x, int y, int maxv = 255) {
    if (m == 0) return chroma_dc(T, L, up, left, (y >> 2) * 2 + (x >> 2), (maxv + 1) >> 1);
    if (m == 1) return L[y];
    if (m == 2) return T[x];
    int ih = 0, iv = 0;
    for (int i = 1; i <= 4; i++) {
        ih += i * (T[3 + i] - (3 - i >= 0 ? T[3 - i] : Pc));
        iv += i * (L[3 + i] - (3 - i >= 0 ? L[3 - i] : Pc));
    }
    int ib = (34 * ih + 32) >> 6, ic = (34 * iv + 32) >> 6, iaa = 16 * (L[7] + T[7]);
    return clipmx((iaa + (x - 3) * ib + (y - 3) * ic + 16) >> 5, maxv);
}
// Intra16x16 prediction (8.3.3): mode-independent parameters, then per-pixel samples.
// T = row y = -1 (T[-1] is the corner p[-1,-1]), L = column x = -1.
struct I16Par { int dcv, ib, ic, iaa; };
template <class pel>
__device__ __forceinline__ I16Par i16_params(const pel *T, const pel *L, int up, int left, int dcd = 128) {
    int st = 0, sl = 0, ih = 0, iv = 0;
    for (int i = 0; i < 16; i++) { st += T[i]; sl += L[i]; }
    for (int i = 1; i <= 8; i++) {
        ih += i * (T[7 + i] - T[7 - i]);
        iv += i * (L[7 + i] - (7 - i >= 0 ? L[7 - i] : T[-1]));
    }
    I16Par p;
    p.dcv = (up && left) ? (st + sl + 16) >> 5 : up ? (st + 8) >> 4 : left ? (sl + 8) >> 4 : dcd;
    p.ib = (5 * ih + 32) >> 6; p.ic = (5 * iv + 32) >> 6; p.iaa = 16 * (L[15] + T[15]);
    return p;
}
template <class pel>
__device__ __forceinline__ int i16_pred(const I16Par &p, const pel *T, const pel *L, int m, int x, int y, int maxv = 255) {
    if (m == 0) return T[x];
    if (m == 1) return L[y];
    if (m == 2) return p.dcv;
    return clipmx((p.iaa + (x - 7) * p.ib + (y - 7) * p.ic + 16) >> 5, maxv);
}

// ======================================================================================
//  64-lane 8x8 primitives (High profile, Transform8x8Mode): one wave per 8x8 block, lane
//  l = 8y + x holds raster element l.  dct_luma8x8 / HadamardSAD8x8 / Intra8x8 [J]
// ======================================================================================
// normAdjust8x8 class (8.5.9) of raster position (x, y) and the per-class JM tables
__device__ __forceinline__ int class8(int x, int y) {
    if (!(x & 3) && !(y & 3)) return 0;
    if ((x & 1) && (y & 1)) return 1;
    if ((x & 3) == 2 && (y & 3) == 2) return 2;
    if ((!(x & 3) && (y & 1)) || ((x & 1) && !(y & 3))) return 3;
    if ((!(x & 3) && (y & 3) == 2) || ((x & 3) == 2 && !(y & 3))) return 4;
    return 5;
}
static __constant__ int c_q8[6][6] = {{13107, 11428, 20972, 12222, 16777, 15481}, {11916, 10826, 19174, 11058, 14980, 14290},
                                      {10082, 8943, 15978, 9675, 12710, 11985},   {9362, 8228, 14913, 8931, 11984, 11259},
                                      {8192, 7346, 13159, 7740, 10486, 9777},     {7282, 6428, 11570, 6830, 9118, 8640}};
static __constant__ int c_dq8[6][6] = {{20, 18, 32, 19, 25, 24}, {22, 19, 35, 21, 28, 26}, {26, 23, 42, 24, 33, 31},
                                       {28, 25, 45, 26, 35, 33}, {32, 28, 51, 30, 40, 38}, {36, 32, 58, 34, 46, 43}};
// 8x8 frame zig-zag: scan index -> raster (8y + x)
static __constant__ uint8_t c_scan8[64] = {0,  1,  8,  16, 9,  2,  3,  10, 17, 24, 32, 25, 18, 11, 4,  5,
                                           12, 19, 26, 33, 40, 48, 41, 34, 27, 20, 13, 6,  7,  14, 21, 28,
                                           35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23, 30, 37, 44, 51,
                                           58, 59, 52, 45, 38, 31, 39, 46, 53, 60, 61, 54, 47, 55, 62, 63};
// the same as immediates (no memory access: the index varies across lanes), eight per qword
__device__ __forceinline__ int scan8_of(int l) {
    const int g = l >> 3;
    const uint64_t q = g < 4 ? (g < 2 ? (g == 0 ? 0x0a03020910080100ull : 0x05040b1219201811ull) : (g == 2 ? 0x22293028211a130cull : 0x1c150e07060d141bull))
                             : (g < 6 ? (g == 4 ? 0x242b323938312a23ull : 0x332c251e170f161dull) : (g == 6 ? 0x2e271f262d343b3aull : 0x3f3e372f363d3c35ull));
    return (int)((q >> (8 * (l & 7))) & 63);
}
// one of six per-class values of a wave-uniform table row (scalar loads + a per-lane select)
__device__ __forceinline__ int pick6(const int *row, int cls) {
    const int a0 = __builtin_amdgcn_readfirstlane(row[0]), a1 = __builtin_amdgcn_readfirstlane(row[1]);
    const int a2 = __builtin_amdgcn_readfirstlane(row[2]), a3 = __builtin_amdgcn_readfirstlane(row[3]);
    const int a4 = __builtin_amdgcn_readfirstlane(row[4]), a5 = __builtin_amdgcn_readfirstlane(row[5]);
    return cls < 3 ? (cls == 0 ? a0 : cls == 1 ? a1 : a2) : (cls == 3 ? a3 : cls == 4 ? a4 : a5);
}
// COEFF_COST8x8 [J] of a |level| == 1 coefficient by preceding zero run (64-scan)
__device__ __forceinline__ int coeff_cost8_run(int run) { return run < 4 ? 3 : run < 12 ? 2 : run < 24 ? 1 : 0; }

// sum over the whole (fully active) wave; every lane gets the sum
__device__ __forceinline__ int wave_sum(int v) {
    v = row16_sum(v);
    return __builtin_amdgcn_readlane(v, 0) + __builtin_amdgcn_readlane(v, 16) + __builtin_amdgcn_readlane(v, 32) +
           __builtin_amdgcn_readlane(v, 48);
}
__device__ __forceinline__ int w64(int v, int src) { return __shfl(v, src, 64); }

// one 8-point butterfly of the forward 8x8 (JM forward8x8 [J]); returns output k
__device__ __forceinline__ int fwd8_pick(int x0, int x1, int x2, int x3, int x4, int x5, int x6, int x7, int k) {
    const int a0 = x0 + x7, a1 = x1 + x6, a2 = x2 + x5, a3 = x3 + x4;
    const int b0 = a0 + a3, b1 = a1 + a2, b2 = a0 - a3, b3 = a1 - a2;
    const int a4 = x0 - x7, a5 = x1 - x6, a6 = x2 - x5, a7 = x3 - x4;
    const int b4 = a5 + a6 + ((a4 >> 1) + a4), b5 = a4 - a7 - ((a6 >> 1) + a6);
    const int b6 = a4 + a7 - ((a5 >> 1) + a5), b7 = a5 - a6 + ((a7 >> 1) + a7);
    switch (k) {
    case 0: return b0 + b1;
    case 1: return b4 + (b7 >> 2);
    case 2: return b2 + (b3 >> 1);
    case 3: return b5 + (b6 >> 2);
    case 4: return b0 - b1;
    case 5: return b6 - (b5 >> 2);
    case 6: return (b2 >> 1) - b3;
    default: return (b4 >> 2) - b7;
    }
}
// one 8-point inverse (8.5.13.2); returns output k
__device__ __forceinline__ int inv8_pick(int d0, int d1, int d2, int d3, int d4, int d5, int d6, int d7, int k) {
    const int a0 = d0 + d4, a4 = d0 - d4, a2 = (d2 >> 1) - d6, a6 = d2 + (d6 >> 1);
    const int b0 = a0 + a6, b2 = a4 + a2, b4 = a4 - a2, b6 = a0 - a6;
    const int a1 = -d3 + d5 - d7 - (d7 >> 1), a3 = d1 + d7 - d3 - (d3 >> 1);
    const int a5 = -d1 + d7 + d5 + (d5 >> 1), a7 = d3 + d5 + d1 + (d1 >> 1);
    const int b1 = a1 + (a7 >> 2), b7 = a7 - (a1 >> 2), b3 = a3 + (a5 >> 2), b5 = (a3 >> 2) - a5;
    switch (k) {
    case 0: return b0 + b7;
    case 1: return b2 + b5;
    case 2: return b4 + b3;
    case 3: return b6 + b1;
    case 4: return b6 - b1;
    case 5: return b4 - b3;
    case 6: return b2 - b5;
    default: return b0 - b7;
    }
}
// forward 8x8 core transform: rows then columns (lanes exchange by ds_bpermute)
__device__ __forceinline__ int wave_fwd8x8(int r, int l) {
    const int x = l & 7, y = l >> 3, rb = 8 * y;
    const int t = fwd8_pick(w64(r, rb), w64(r, rb + 1), w64(r, rb + 2), w64(r, rb + 3), w64(r, rb + 4), w64(r, rb + 5),
                            w64(r, rb + 6), w64(r, rb + 7), x);
    return fwd8_pick(w64(t, x), w64(t, 8 + x), w64(t, 16 + x), w64(t, 24 + x), w64(t, 32 + x), w64(t, 40 + x), w64(t, 48 + x),
                     w64(t, 56 + x), y);
}
// inverse 8x8 (rows first) + reconstruction clip((x + (pred << 6) + 32) >> 6) to maxv
__device__ __forceinline__ int wave_inv8x8(int dq, int l, int pred, int maxv = 255) {
    const int x = l & 7, y = l >> 3, rb = 8 * y;
    const int t = inv8_pick(w64(dq, rb), w64(dq, rb + 1), w64(dq, rb + 2), w64(dq, rb + 3), w64(dq, rb + 4), w64(dq, rb + 5),
                            w64(dq, rb + 6), w64(dq, rb + 7), x);
    const int o = inv8_pick(w64(t, x), w64(t, 8 + x), w64(t, 16 + x), w64(t, 24 + x), w64(t, 32 + x), w64(t, 40 + x), w64(t, 48 + x),
                            w64(t, 56 + x), y);
    return iclip(0, maxv, (o + (pred << 6) + 32) >> 6);
}
// quantisation of coefficient c at raster l (dct_luma8x8 [J]): lev_scan = signed level at SCAN
// position l, dq = normative 8.5.13.1 dequantisation of the signed level at raster l (flat
// weights), cost = COEFF_COST8x8 sum (wave-uniform); returns the scan-order non-zero mask.
__device__ __forceinline__ unsigned long long wave_quant8(int c, int l, int qp, int qp_const, int &lev_scan, int &dq, int &cost) {
    const int qp_per = qp / 6, qp_rem = qp % 6, q_bits = 16 + qp_per;
    const int cls = class8(l & 7, l >> 3);
    const int level = (abs(c) * pick6(c_q8[qp_rem], cls) + qp_const) >> q_bits;
    const int sl = c < 0 ? -level : level;
    const int ls = 16 * pick6(c_dq8[qp_rem], cls);
    dq = !level ? 0 : qp >= 36 ? sl * ls * (1 << (qp_per - 6)) : (sl * ls + (1 << (5 - qp_per))) >> (6 - qp_per);
    const int lvs = w64(sl, scan8_of(l));
    const unsigned long long m = __ballot(lvs != 0);
    int k = 0;
    if (lvs) {
        const unsigned long long below = m & ((1ull << l) - 1ull);
        const int prev = below ? 63 - __clzll(below) : -1;
        k = abs(lvs) > 1 ? MAX_VALUE : coeff_cost8_run(l - prev - 1);
    }
    cost = wave_sum(k);
    lev_scan = lvs;
    return m;
}
// sum over the wave of |Hadamard| of the 8x8 block (h = 1, 2, 4, 8, 16, 32) or, with quad4, of
// the four 4x4 blocks (h = 1, 2, 8, 16); wave-uniform
__device__ __forceinline__ int wave_had_abs(int v, int l, bool quad4) {
#pragma unroll
    for (int h = 1; h < 64; h <<= 1) {
        if (quad4 && (h == 4 || h == 32)) continue;
        const int p = __shfl_xor(v, h, 64);
        v = (l & h) ? p - v : v + p;
    }
    return wave_sum(abs(v));
}
// SATD of an 8x8 block (HadamardSAD8x8 [J]: (sum + 2) >> 2) and the sum of its four 4x4 SATD()
__device__ __forceinline__ int wave_satd8(int dv, int l, int had) { return had ? (wave_had_abs(dv, l, false) + 2) >> 2 : wave_sum(abs(dv)); }
__device__ __forceinline__ int wave_satd4x4s(int dv, int l, int had) { return had ? wave_had_abs(dv, l, true) >> 1 : wave_sum(abs(dv)); }
// scan index k of an 8x8 block b8 -> (raster 4x4 block of the CAVLC interleave, entry)
__device__ __forceinline__ int il_blk(int b8, int k) { const int j = k & 3; return (2 * (b8 >> 1) + (j >> 1)) * 4 + 2 * (b8 & 1) + (j & 1); }

// Intra8x8 prediction (8.3.2.2) of mode m at (x, y) from the filtered reference edge f[0..24]:
// f[7 - y] = p'[-1, y], f[8] = p'[-1, -1], f[9 + x] = p'[x, -1]
__device__ __forceinline__ int i8_pred_px(const int *f, int dcv, int m, int x, int y) {
#define TAP(c) ((f[(c) - 1] + 2 * f[c] + f[(c) + 1] + 2) >> 2)
    int z;
    switch (m) {
    case 0: return f[9 + x];
    case 1: return f[7 - y];
    case 2: return dcv;
    case 3: return x + y < 14 ? TAP(10 + x + y) : (f[23] + 3 * f[24] + 2) >> 2;
    case 4: return TAP(8 + x - y);
    case 5:
        z = 2 * x - y;
        if (z >= 0 && !(z & 1)) return (f[8 + x - (y >> 1)] + f[9 + x - (y >> 1)] + 1) >> 1;
        return z > 0 ? TAP(8 + x - (y >> 1)) : TAP(9 + z);
    case 6:
        z = 2 * y - x;
        if (z >= 0 && !(z & 1)) return (f[8 - y + (x >> 1)] + f[7 - y + (x >> 1)] + 1) >> 1;
        return z > 0 ? TAP(8 - y + (x >> 1)) : TAP(7 - z);
    case 7:
        return (y & 1) ? (f[9 + x + (y >> 1)] + 2 * f[10 + x + (y >> 1)] + f[11 + x + (y >> 1)] + 2) >> 2
                       : (f[9 + x + (y >> 1)] + f[10 + x + (y >> 1)] + 1) >> 1;
    default:
        z = x + 2 * y;
        if (z > 13) return f[0];
        if (z == 13) return (f[1] + 3 * f[0] + 2) >> 2;
        if (!(z & 1)) return (f[7 - y - (x >> 1)] + f[6 - y - (x >> 1)] + 1) >> 1;
        return (f[7 - y - (x >> 1)] + 2 * f[6 - y - (x >> 1)] + f[5 - y - (x >> 1)] + 2) >> 2;
    }
#undef TAP
}

// debug phase profiling of one macroblock (DevParams::prof): lane 0 of wave w of the matching group
__device__ __forceinline__ bool prof_mb_here(const DevParams &d, int mbx, int mby, int w = 0) {
    return d.prof && threadIdx.x == 64 * w && d.prof_mb == mby * d.mbw + mbx;
}
#define PSTAMP(k) do { if (prof) d.prof[k] = wall_clock64(); } while (0)
