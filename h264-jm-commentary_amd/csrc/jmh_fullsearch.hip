// jmh_fullsearch.hip — k_mb_me_full: the motion-search half of encode_one_macroblock [J] with
// SearchMode = -1 (FullPelBlockMotionSearch), one 256-thread workgroup per P macroblock (EPZS,
// SearchMode 3, has its own one-wave kernel: jmh_epzs.hip).
//
// Unlike FFS, every search centres its window on its OWN predictor (MVP/4 clamped to its range),
// so there is no shared SAD table: each of the 41 searches computes the SAD of its block at all
// (2*range+1)^2 positions straight from an LDS window that covers every block's reach (MB +-
// (2*SR + 4): block offset <= range + |centre| <= 2*SR, sub-pel and 6-tap margin).  cost =
// lambda*(mvbits(x) + mvbits(y)) - 16*lambda for the 16x16 zero vector + SAD, key = cost <<
// 13 | spiral index, strict '<' (FullPelBlockMotionSearch [J]).  Sub-pel samples come from the
// same window through the 6-tap on the fly (qpel_from), candidate SATD sums by LDS atomics.
//
// The searches run in JM's order (16x16, 16x8, 8x16, then per 8x8 block the sub-modes 4..7),
// which is dependency-exact by construction.  The results land in MbScratch exactly like
// k_mb_analyse's FFS search, so the intra workgroups and k_mb_final are shared.
//
// Templated on the sample type and the search: pel = uint16_t is High 10 (two samples per dword,
// v_sad_u16, Clip1 to (1 << BitDepth) - 1 in the half-pel planes; a 16x16 SAD < 2^18, so the
// `cost << 13` keys still fit 32 bits), and FFS = true is SearchMode 0 for those pictures
// (FastFullPelBlockMotionSearch [J]: every search of the MB on the window centred on the 16x16
// MVP / 4 clamped to +-SR, the (0,0) vector checked first -- order key 0, the spiral positions
// 1.. -- and no 16x16 zero-vector bias in full pel).  8-bit FFS keeps k_mb_analyse's shared 4x4
// SAD table; here each search sums its block directly (7x the SAD work, on the 10-bit path only).
#include "jmh_common.h"

#define NTF 256                               // threads per full-search workgroup
#define FOFF_MAX (2 * SRMAX + 4)              // window margin around the MB
#define FW_MAX (16 + 2 * FOFF_MAX)            // 152
#define FST 156                               // window row stride (>= FW_MAX + 4, multiple of 4)
#define FKOFF 4096                            // cost offset in keys (16x16 zero-vector bias)


template <class pel>
struct FullS {
    pel g[FW_MAX * FST + 16];
    pel org[256];
    Border bd;
    int16_t all_mv[8][16][2];
    int motion_cost[8][4];
    unsigned red[2][NTF / 64];
    int ccost[2][9];
    int cost0;
    pel hp[3][18][20];                         // half-pel b / h / j around the block at its full-pel MV
    int scx, scy;                              // FFS: the window centre (16x16 MVP / 4, clamped)
};

// half-grid sample (hx, hy) relative to the block origin at its full-pel MV (window (gx0, gy0)):
// even / even = integer sample, odd x = b, odd y = h, both odd = j (8.4.2.2.1)
template <class pel>
__device__ __forceinline__ int hg_at(const FullS<pel> &s, int gx0, int gy0, int hx, int hy) {
    if (!((hx | hy) & 1)) return s.g[(gy0 + (hy >> 1)) * FST + gx0 + (hx >> 1)];
    const int pl = (hx & hy & 1) ? 2 : (hx & 1) ? 0 : 1;
    return s.hp[pl][(hy >> 1) + 1][(hx >> 1) + 1];
}

// neighbour view of a search of block type bt in 8x8 block b8 (as NbMe in jmh_analyse.hip)
template <class pel>
struct NbFull {
    const FullS<pel> &s;
    int bt, b8, best8x8;
    __device__ __forceinline__ bool operator()(int xN, int yN, int &ref, int &mx, int &my) const {
        if (yN > 15 || (xN > 15 && yN >= 0)) return false;
        if (xN < 0 || yN < 0) {
            int c = border_cell(xN, yN);
            if (c < 0 || s.bd.ref[c] == -2) return false;
            ref = s.bd.ref[c]; mx = s.bd.mv[c][0]; my = s.bd.mv[c][1];
            return true;
        }
        int k = (yN >> 2) * 4 + (xN >> 2), cb8 = ((yN >> 3) << 1) | (xN >> 3);
        int m = (bt <= 3 || cb8 == b8) ? bt : (best8x8 >> (4 * cb8)) & 15;
        ref = 0; mx = s.all_mv[m][k][0]; my = s.all_mv[m][k][1];
        return true;
    }
};

__device__ __forceinline__ uint32_t lds_u32(const void *p) { return lds_u32_any(p); }   // 4 bytes at any LDS address

// workgroup minimum of per-thread keys (double-buffered slot: consecutive calls need no second
// barrier); every thread returns the minimum
template <class pel>
__device__ __forceinline__ unsigned wg_min(FullS<pel> &s, unsigned k, int &slot) {
    k = wave_min_u32(k);
    if ((threadIdx.x & 63) == 0) s.red[slot][threadIdx.x >> 6] = k;
    __syncthreads();
    unsigned m = s.red[slot][0];
#pragma unroll
    for (int w = 1; w < NTF / 64; w++) m = min(m, s.red[slot][w]);
    slot ^= 1;
    return m;
}

// BlockMotionSearch [J] for one block: full-pel full search (FFS: on the MB's common window) +
// SubPelBlockMotionSearch
template <class pel, bool FFS>
__device__ __forceinline__ void full_block_search(const DevParams &d, FullS<pel> &s, int off, int bt, int bx4, int by4, int mc, int b8,
                                                           int best8x8, int X0, int Y0, int pslot) {
    const int tid = threadIdx.x;
    const bool prof = pslot >= 0 && pslot < 28 && d.prof && tid == 0 && d.prof_mb == (Y0 >> 2) * d.mbw + (X0 >> 2);
    const int lam = d.lambda_motion, had = d.use_hadamard;
    const bool slice_p = d.slice_type == JMH_P_SLICE;
    const int range = d.restrict_sr == 0 ? d.sr / min(2, bt) : d.sr;
    const int lw4 = lw4_of(bt), lh4 = lh4_of(bt), w4 = 1 << lw4, h4 = 1 << lh4, lns = lw4 + lh4, nsub = 1 << lns;
    int pmx, pmy;
    set_mvp(NbFull<pel>{s, bt, b8, best8x8}, bx4, by4, 4 * w4, 4 * h4, pmx, pmy);
    if (FFS && bt == 1) {                              // SetupFastFullPelSearch: the MB's window centre
        if (tid == 0) { s.scx = iclip(-d.sr, d.sr, pmx / 4); s.scy = iclip(-d.sr, d.sr, pmy / 4); }
        __syncthreads();
    }
    const int mvx0 = FFS ? s.scx : iclip(-range, range, pmx / 4), mvy0 = FFS ? s.scy : iclip(-range, range, pmy / 4);
    int fmx, fmy, min_mcost;
    {
    // ---- full pel: every thread a stride of positions, SADs by dword v_sad_u8 / v_sad_u16
    constexpr int PD = 4 / (int)sizeof(pel);           // samples per dword
    const int side = 2 * range + 1, npos = side * side;
    // the block's SAD + MV cost at MV (cx, cy) (window position = MB origin + block + MV)
    auto cost_at = [&](int cx, int cy) {
        int cost = lam * (mvbits(4 * cx - pmx) + mvbits(4 * cy - pmy));
        if (!FFS && bt == 1 && slice_p && cx == 0 && cy == 0) cost -= 16 * lam;
        const int wx = off + 4 * bx4 + cx, wy = off + 4 * by4 + cy;
        uint32_t sad = 0;
        for (int r = 0; r < 4 * h4; r++) {
            const pel *row = s.g + (wy + r) * FST + wx;
            const uint32_t *org = reinterpret_cast<const uint32_t *>(s.org + (4 * by4 + r) * 16 + 4 * bx4);
            for (int q = 0; q < 4 * w4 / PD; q++) {
                if constexpr (sizeof(pel) == 1) sad = __builtin_amdgcn_sad_u8(lds_u32(row + PD * q), org[q], sad);
                else sad = __builtin_amdgcn_sad_u16(lds_u32(row + PD * q), org[q], sad);
            }
        }
        return cost + (int)sad;
    };
    // key = cost << 13 | JM order: full search the spiral index; FFS 0 for its (0,0) pre-check,
    // spiral index + 1 for the positions
    unsigned kb = 0xFFFFFFFFu;
    for (int p = tid; p < npos; p += NTF) {
        const int dy = p / side - range, dx = p - (dy + range) * side - range;
        kb = min(kb, ((unsigned)(cost_at(mvx0 + dx, mvy0 + dy) + FKOFF) << 13) | (unsigned)(spiral_index(dx, dy) + FFS));
    }
    if (FFS && tid == NTF - 1) kb = min(kb, (unsigned)(cost_at(0, 0) + FKOFF) << 13);
    int slot = 0;
    const unsigned best = wg_min(s, kb, slot);
    int rx, ry;
    if (FFS && (best & 8191u) == 0) { rx = -mvx0; ry = -mvy0; }
    else spiral_pos((int)(best & 8191u) - FFS, rx, ry);
    fmx = mvx0 + rx; fmy = mvy0 + ry;
    min_mcost = had ? BIGCOST : (int)(best >> 13) - FKOFF;
    }
    // ---- sub pel (half then quarter): half-pel b / h / j planes of the block's neighbourhood
    // (x, y in [-1, w] x [-1, h] around its full-pel position) built once, then every quarter
    // sample is the average of two half-grid samples; one 16-lane group per (candidate, 4x4)
    const bool check0 = bt == 1 && fmx == 0 && fmy == 0 && had && slice_p;
    auto px = [&](int x, int y) { return (int)s.g[y * FST + x]; };
    const int maxv = d.maxv;
    const int gx0 = off + 4 * bx4 + fmx, gy0 = off + 4 * by4 + fmy;
    {
        const int PW = 4 * w4 + 2, PH = 4 * h4 + 2;
        for (int i = tid; i < PW * PH; i += NTF) {
            const int y = i / PW, x = i - y * PW, gx = gx0 + x - 1, gy = gy0 + y - 1;
            s.hp[0][y][x] = (pel)iclip(0, maxv, (tap6(px(gx - 2, gy), px(gx - 1, gy), px(gx, gy), px(gx + 1, gy), px(gx + 2, gy), px(gx + 3, gy)) + 16) >> 5);
            s.hp[1][y][x] = (pel)iclip(0, maxv, (tap6(px(gx, gy - 2), px(gx, gy - 1), px(gx, gy), px(gx, gy + 1), px(gx, gy + 2), px(gx, gy + 3)) + 16) >> 5);
            int v[6];
#pragma unroll
            for (int k = 0; k < 6; k++) {
                const int xx = gx - 2 + k;
                v[k] = tap6(px(xx, gy - 2), px(xx, gy - 1), px(xx, gy), px(xx, gy + 1), px(xx, gy + 2), px(xx, gy + 3));
            }
            s.hp[2][y][x] = (pel)iclip(0, maxv, (tap6(v[0], v[1], v[2], v[3], v[4], v[5]) + 512) >> 10);
        }
    }
    const int grp = tid >> 4, l = tid & 15;
    if (tid < 18) s.ccost[tid / 9][tid % 9] = 0;
    __syncthreads();
    int qx = 0, qy = 0;
    for (int pass = 0; pass < 2; pass++) {
        const int step = pass == 0 ? 2 : 1, min_pos = pass == 0 ? (had ? 0 : 1) : 1;
        for (int task = grp; task < (9 << lns); task += NTF / 16) {   // group-uniform
            const int c = task >> lns, sub = task & (nsub - 1);
            if (c < min_pos) continue;
            const int ox = qx + step * sp9x(c), oy = qy + step * sp9y(c);
            const int pxl = 4 * (sub & (w4 - 1)) + (l & 3), pyl = 4 * (sub >> lw4) + (l >> 2);
            const int Qx = 4 * pxl + ox, Qy = 4 * pyl + oy, xi = Qx >> 2, yi = Qy >> 2;
            const int q = qoff(((Qy & 3) << 2) | (Qx & 3));
            const int a = hg_at(s, gx0, gy0, 2 * xi + ((q >> 12) & 15), 2 * yi + ((q >> 8) & 15));
            const int b = hg_at(s, gx0, gy0, 2 * xi + ((q >> 4) & 15), 2 * yi + (q & 15));
            const int dv = s.org[(4 * by4 + pyl) * 16 + 4 * bx4 + pxl] - ((a + b + 1) >> 1);
            const int sat = lane_satd(dv, l, had);
            if (l == 0) atomicAdd(&s.ccost[pass][c], sat);
        }
        __syncthreads();
        int bpos = 0;
        for (int c = min_pos; c < 9; c++) {   // JM order, strict '<'
            const int ox = qx + step * sp9x(c), oy = qy + step * sp9y(c);
            int v = s.ccost[pass][c] + lam * (mvbits(4 * fmx + ox - pmx) + mvbits(4 * fmy + oy - pmy));
            if (pass == 0 && check0 && c == 0) v -= 16 * lam;
            if (v < min_mcost) { min_mcost = v; bpos = c; }
        }
        qx += step * sp9x(bpos);
        qy += step * sp9y(bpos);
    }
    if (tid < nsub) {
        const int k = (by4 + (tid >> lw4)) * 4 + bx4 + (tid & (w4 - 1));
        s.all_mv[bt][k][0] = (int16_t)(4 * fmx + qx);
        s.all_mv[bt][k][1] = (int16_t)(4 * fmy + qy);
    }
    if (tid == 0) s.motion_cost[bt][mc] += min_mcost;
    __syncthreads();
    if (prof) d.prof[35 + pslot] = wall_clock64();
}

template <class pel, bool FFS>
__global__ __launch_bounds__(NTF, sizeof(pel) == 1 ? 6 : 3) void k_mb_me_full(const TickArgs t) {   // 16-bit: LDS allows 3 per CU
    __shared__ FullS<pel> s;
    const int b = xcd_block(blockIdx.x, t.pre[t.nP]), tid = threadIdx.x;   // XCD-aware (jmh_device.h)
    if (b >= t.pre[t.nP]) return;
    const int e = tick_entry(t, b);
    const DevParams d = tick_params(t, e);
    const int mby = d.y_min + (b - t.pre[e]), mbx = d.diag - 2 * mby;
    const int pix_x = 16 * mbx, pix_y = 16 * mby, W = d.W, sr = d.sr;
    const int off = 2 * sr + 4, wdim = 16 + 2 * off;
    MbScratch *scr = d.scr + mby * d.mbw + mbx;
    const int X0 = 4 * mbx, Y0 = 4 * mby;
    if (d.prof && tid == 0 && d.prof_mb == mby * d.mbw + mbx) d.prof[32] = wall_clock64();
    s.org[tid] = spl<pel>(d.orgY)[(pix_y + (tid >> 4)) * W + pix_x + (tid & 15)];
    if (tid < 10) load_border(d, s.bd, tid, mbx, mby);
    else if (tid >= 32 && tid < 64) s.motion_cost[(tid - 32) >> 2][tid & 3] = 0;
    {   // window: MB pixel (0,0) at (off, off); per-coordinate clamping is the spec's UMV access
        constexpr int PD = 4 / (int)sizeof(pel), ND4 = FST / PD, SB = 8 * (int)sizeof(pel);
        const int X0 = pix_x - off, Y0 = pix_y - off;
        for (int task = tid; task < wdim * ND4; task += NTF) {
            const int y = task / ND4, j = task - y * ND4, x0 = X0 + PD * j;
            const pel *row = spl<pel>(d.refY) + iclip(0, d.H - 1, Y0 + y) * W;
            uint32_t v;
            if (PD * j + PD - 1 < wdim && x0 >= 0 && x0 + PD - 1 < W) {
                if constexpr (sizeof(pel) == 1) {
                    const uint32_t *p = reinterpret_cast<const uint32_t *>(row + (x0 & ~3));
                    v = __builtin_amdgcn_alignbyte((x0 & 3) ? p[1] : 0u, p[0], x0 & 3);
                } else {
                    v = *reinterpret_cast<const uint32_t *>(row + x0);   // x0 even: pix_x - 2 SR - 4 + 2 j
                }
            } else {
                v = 0;
                for (int q = 0; q < PD; q++)
                    if (PD * j + q < wdim) v |= (uint32_t)row[iclip(0, W - 1, x0 + q)] << (SB * q);
            }
            *reinterpret_cast<uint32_t *>(s.g + y * FST + PD * j) = v;
        }
    }
    __syncthreads();
    if (d.prof && tid == 0 && d.prof_mb == mby * d.mbw + mbx) d.prof[33] = wall_clock64();
    // PartitionMotionSearch [J] order: 16x16, 16x8 (2), 8x16 (2), then per 8x8 block the sub-modes
    // 4..7 and its best sub-mode (read through best8x8).  One call site (a loop over the 41
    // searches) so the search inlines once: no call frames / register spills to scratch.
    int best8x8 = 0, cost8x8 = 0;
#pragma unroll 1
    for (int i = 0; i < 41; i++) {
        int bt, bx4, by4, mc, b8;
        if (i < 5) {   // 16x16; 16x8 upper, lower; 8x16 left, right
            bt = i == 0 ? 1 : i <= 2 ? 2 : 3;
            bx4 = i == 4 ? 2 : 0; by4 = i == 2 ? 2 : 0; mc = (i == 2 || i == 4) ? 1 : 0; b8 = 0;
        } else {       // 8x8; 8x4 x2; 4x8 x2; 4x4 x4 of 8x8 block b8
            const int j = (i - 5) % 9;
            b8 = (i - 5) / 9; mc = b8;
            bt = j == 0 ? 4 : j <= 2 ? 5 : j <= 4 ? 6 : 7;
            const int sx = j == 4 || j == 6 || j == 8 ? 1 : 0, sy = j == 2 || j == 7 || j == 8 ? 1 : 0;
            bx4 = 2 * (b8 & 1) + sx; by4 = 2 * (b8 >> 1) + sy;
        }
        full_block_search<pel, FFS>(d, s, off, bt, bx4, by4, mc, b8, i < 5 ? 0 : best8x8, X0, Y0, i < 14 ? 2 * i : -1);
        if (i >= 5 && (i - 5) % 9 == 8) {
            int mc8 = BIGCOST, bm = 0;
            for (int mode = 4; mode <= 7; mode++) {
                if (!inter_on(d.isr, mode)) continue;
                const int c = s.motion_cost[mode][b8];
                if (c < mc8) { mc8 = c; bm = mode; }
            }
            best8x8 |= bm << (4 * b8);
            cost8x8 += mc8;
        }
    }
    // results: MVs and partition costs of types 1..7, P8x8 decision, FindSkipModeMotionVector
    for (int i = tid; i < 7 * 32; i += NTF) {
        const int m = 1 + i / 32, k = (i & 31) >> 1, c = i & 1;
        scr->all_mv[m][k][c] = s.all_mv[m][k][c];
    }
    if (tid < 28) scr->motion_cost[1 + tid / 4][tid & 3] = s.motion_cost[1 + tid / 4][tid & 3];
    else if (tid == 64) { scr->best8x8 = best8x8; scr->cost8x8 = cost8x8; }
    else if (tid == 128) {
        int pcx, pcy;
        set_mvp(NbBorder{s.bd}, 0, 0, 16, 16, pcx, pcy);
        NbBorder nbv{s.bd};
        int ra = -1, ax = 0, ay = 0, rb = -1, bx = 0, by = 0;
        const bool aa = nbv(-1, 0, ra, ax, ay), ab = nbv(0, -1, rb, bx, by);
        const bool zl = !aa || (ra == 0 && ax == 0 && ay == 0), za = !ab || (rb == 0 && bx == 0 && by == 0);
        scr->skipx = (za || zl) ? 0 : pcx;
        scr->skipy = (za || zl) ? 0 : pcy;
    }
}

hipError_t jmh_launch_me_full(const TickArgs &t, hipStream_t st) {
    if (t.pre[t.nP] == 0) return hipSuccess;
    typedef void (*Kern)(const TickArgs);
    const bool ffs = t.search_mode == 0;   // 8-bit FFS runs in k_mb_analyse
    const Kern k = t.bd > 8 ? (ffs ? k_mb_me_full<uint16_t, true> : k_mb_me_full<uint16_t, false>) : k_mb_me_full<uint8_t, false>;
    hipLaunchKernelGGL(k, dim3(xcd_grid(t.pre[t.nP])), dim3(NTF), 0, st, t);
    return hipGetLastError();
}
