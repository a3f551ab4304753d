/*
 * yuv.c — picture buffers, planar I420 I/O (JM image.c › ReadOneFrame [J]) with edge
 * replication to the coded size, and the deterministic synthetic source of SURVEY.md §8d.
 *
 * Synthetic source: integer-only, so every host produces the same bytes.  Texture = 4 octaves
 * of lattice value noise + 2 triangle gratings + a gradient, sampled on a quarter-pel grid;
 * global motion (+3,-1) pel/frame plus a quarter-pel phase cycle; 12 rectangles (32..256 px)
 * with their own texture and velocities up to +-20 pel/frame; fresh +-2 noise per frame;
 * xorshift64*-derived hashing with seed 0x5EED0000 + stream id.
 */
#include <stdlib.h>
#include <string.h>
#include "jmhost.h"

int jm_pic_alloc_bd(jm_pic *p, int w, int h, int bd) {
    memset(p, 0, sizeof(*p));
    p->w = w; p->h = h; p->bd = bd > 8 ? bd : 8;
    size_t ls = (size_t)w * h, cs = ls / 4;
    if (p->bd > 8) {
        p->Y = (uint16_t *)malloc((ls + 2 * cs) * sizeof(uint16_t));
        if (!p->Y) return -1;
        p->U = p->Y + ls;
        p->V = p->U + cs;
        return 0;
    }
    p->y = (uint8_t *)malloc(ls + 2 * cs);
    if (!p->y) return -1;
    p->u = p->y + ls;
    p->v = p->u + cs;
    return 0;
}
int jm_pic_alloc(jm_pic *p, int w, int h) { return jm_pic_alloc_bd(p, w, h, 8); }
void jm_pic_free(jm_pic *p) {
    free(p->y); p->y = p->u = p->v = NULL;
    free(p->Y); p->Y = p->U = p->V = NULL;
}

/* PaddAutoCropBorders-style edge replication of the displayed area to the coded size */
#define PAD_PLANES(T, Y, U, V)                                                                          \
    do {                                                                                                \
        int w = p->w, h = p->h;                                                                         \
        for (int y = 0; y < dh; y++)                                                                    \
            for (int x = dw; x < w; x++) Y[y * w + x] = Y[y * w + dw - 1];                              \
        for (int y = dh; y < h; y++) memcpy(Y + (size_t)y * w, Y + (size_t)(dh - 1) * w, w * sizeof(T)); \
        int cw = w / 2, ch = h / 2, cdw = dw / 2, cdh = dh / 2;                                         \
        T *pl[2] = {U, V};                                                                              \
        for (int k = 0; k < 2; k++) {                                                                   \
            for (int y = 0; y < cdh; y++)                                                               \
                for (int x = cdw; x < cw; x++) pl[k][y * cw + x] = pl[k][y * cw + cdw - 1];             \
            for (int y = cdh; y < ch; y++)                                                              \
                memcpy(pl[k] + (size_t)y * cw, pl[k] + (size_t)(cdh - 1) * cw, cw * sizeof(T));          \
        }                                                                                               \
    } while (0)
void jm_pad_picture(jm_pic *p, int dw, int dh) {
    if (p->bd > 8) PAD_PLANES(uint16_t, p->Y, p->U, p->V);
    else PAD_PLANES(uint8_t, p->y, p->u, p->v);
}

/* High 10 files: 16-bit little-endian samples (JM >= 10 ReadOneFrame with symbol_size_in_bytes 2 [J]) */
static int read_hbd(FILE *f, jm_pic *p, int dw, int dh, int index) {
    long fs = (long)dw * dh * 3 / 2 * 2;
    if (fseek(f, fs * index, SEEK_SET)) return -1;
    for (int y = 0; y < dh; y++)
        if (fread(p->Y + (size_t)y * p->w, 2, dw, f) != (size_t)dw) return -1;
    for (int y = 0; y < dh / 2; y++)
        if (fread(p->U + (size_t)y * (p->w / 2), 2, dw / 2, f) != (size_t)(dw / 2)) return -1;
    for (int y = 0; y < dh / 2; y++)
        if (fread(p->V + (size_t)y * (p->w / 2), 2, dw / 2, f) != (size_t)(dw / 2)) return -1;
    const int maxv = (1 << p->bd) - 1;
    for (size_t i = 0; i < (size_t)p->w * p->h * 3 / 2; i++)
        if (p->Y[i] > maxv) p->Y[i] = (uint16_t)maxv;     /* samples beyond the bit depth: Clip1 */
    jm_pad_picture(p, dw, dh);
    return 0;
}

int jm_read_yuv_frame(FILE *f, jm_pic *p, int dw, int dh, int index) {
    if (p->bd > 8) return read_hbd(f, p, dw, dh, index);
    long fs = (long)dw * dh * 3 / 2;
    if (fseek(f, fs * index, SEEK_SET)) return -1;
    if (p->w == dw) {   /* rows contiguous in the planes: one read per plane (no stdio buffering) */
        if (fread(p->y, 1, (size_t)dw * dh, f) != (size_t)dw * dh) return -1;
        if (fread(p->u, 1, (size_t)(dw / 2) * (dh / 2), f) != (size_t)(dw / 2) * (dh / 2)) return -1;
        if (fread(p->v, 1, (size_t)(dw / 2) * (dh / 2), f) != (size_t)(dw / 2) * (dh / 2)) return -1;
    } else {
        for (int y = 0; y < dh; y++)
            if (fread(p->y + (size_t)y * p->w, 1, dw, f) != (size_t)dw) return -1;
        for (int y = 0; y < dh / 2; y++)
            if (fread(p->u + (size_t)y * (p->w / 2), 1, dw / 2, f) != (size_t)(dw / 2)) return -1;
        for (int y = 0; y < dh / 2; y++)
            if (fread(p->v + (size_t)y * (p->w / 2), 1, dw / 2, f) != (size_t)(dw / 2)) return -1;
    }
    jm_pad_picture(p, dw, dh);
    return 0;
}

int jm_write_yuv_frame(FILE *f, const jm_pic *p, int dw, int dh) {
    if (p->bd > 8) {
        for (int y = 0; y < dh; y++) fwrite(p->Y + (size_t)y * p->w, 2, dw, f);
        for (int y = 0; y < dh / 2; y++) fwrite(p->U + (size_t)y * (p->w / 2), 2, dw / 2, f);
        for (int y = 0; y < dh / 2; y++) fwrite(p->V + (size_t)y * (p->w / 2), 2, dw / 2, f);
        return 0;
    }
    for (int y = 0; y < dh; y++) fwrite(p->y + (size_t)y * p->w, 1, dw, f);
    for (int y = 0; y < dh / 2; y++) fwrite(p->u + (size_t)y * (p->w / 2), 1, dw / 2, f);
    for (int y = 0; y < dh / 2; y++) fwrite(p->v + (size_t)y * (p->w / 2), 1, dw / 2, f);
    return 0;
}

/* ---- synthetic source ------------------------------------------------------------------ */
static inline uint64_t mix64(uint64_t x) {       /* xorshift64* step used as a hash */
    x ^= x >> 12; x ^= x << 25; x ^= x >> 27;
    return x * 0x2545F4914F6CDD1DULL;
}
static inline uint32_t hash3(uint64_t seed, int32_t a, int32_t b, int32_t c) {
    uint64_t x = seed ^ ((uint64_t)(uint32_t)a * 0x9E3779B97F4A7C15ULL) ^
                 ((uint64_t)(uint32_t)b * 0xC2B2AE3D27D4EB4FULL) ^ ((uint64_t)(uint32_t)c << 17);
    return (uint32_t)(mix64(mix64(x | 1)) >> 32);
}
static inline int floordiv(int a, int b) { return a >= 0 ? a / b : -((-a + b - 1) / b); }

/* value noise at quarter-pel coordinate (X,Y), lattice cell `cell` pels, result 0..255 */
static int vnoise(uint64_t seed, int oct, int X, int Y, int cell) {
    int q = 4 * cell;
    int ix = floordiv(X, q), iy = floordiv(Y, q);
    int fx = X - ix * q, fy = Y - iy * q;             /* 0..q-1 */
    int v00 = hash3(seed, ix, iy, oct) & 255, v10 = hash3(seed, ix + 1, iy, oct) & 255;
    int v01 = hash3(seed, ix, iy + 1, oct) & 255, v11 = hash3(seed, ix + 1, iy + 1, oct) & 255;
    int top = v00 * (q - fx) + v10 * fx, bot = v01 * (q - fx) + v11 * fx;
    return (top * (q - fy) + bot * fy) / (q * q);
}
static inline int tri(int t, int period) {            /* triangle wave 0..255, t in qpel */
    int p4 = 4 * period;
    int m = t % p4;
    if (m < 0) m += p4;
    int h = p4 / 2;
    return m < h ? (m * 255) / h : ((p4 - m) * 255) / h;
}
static int texture(uint64_t seed, int X, int Y, int plane) {
    int v = 0;
    v += vnoise(seed, 0 + plane, X, Y, 61) * 40;
    v += vnoise(seed, 1 + plane, X, Y, 23) * 28;
    v += vnoise(seed, 2 + plane, X, Y, 9) * 18;
    v += vnoise(seed, 3 + plane, X, Y, 4) * 14;
    v /= 100;
    int g1 = tri(X + 2 * Y, 37 + 5 * plane), g2 = tri(3 * X - Y, 17 + 3 * plane);
    v = (v * 6 + g1 * 2 + g2 * 2) / 10;
    v += (X / 4 + Y / 4) / 64;                          /* gentle gradient */
    return v;
}

typedef struct { int x, y, w, h, vx, vy; } rect_t;    /* pos/vel in quarter pels */

static void synth8(jm_pic *p, int dw, int dh, uint64_t seed, int t);
void jm_synth_frame(jm_pic *p, int dw, int dh, uint64_t seed, int t) {
    if (p->bd <= 8) { synth8(p, dw, dh, seed, t); return; }
    jm_synth_frame_hbd(p->Y, p->U, p->V, p->w, p->h, dw, dh, seed, t, p->bd);
}

void jm_synth_frame_hbd(uint16_t *Y, uint16_t *U, uint16_t *V, int w, int h, int dw, int dh, uint64_t seed, int t, int bd) {
    jm_pic q;
    if (jm_pic_alloc(&q, w, h)) return;
    synth8(&q, dw, dh, seed, t);
    const uint64_t s = 0x5EED0000ULL + seed + 77;
    const int sh = bd - 8, lo = (1 << sh) - 1;
    for (int y = 0; y < dh; y++)
        for (int x = 0; x < dw; x++)
            Y[(size_t)y * w + x] = (uint16_t)((q.y[(size_t)y * w + x] << sh) | (hash3(s, x, y, 2 * t) & lo));
    for (int y = 0; y < dh / 2; y++)
        for (int x = 0; x < dw / 2; x++) {
            const size_t i = (size_t)y * (w / 2) + x;
            U[i] = (uint16_t)((q.u[i] << sh) | (hash3(s, x, y, 2 * t + 1) & lo));
            V[i] = (uint16_t)((q.v[i] << sh) | (hash3(s, y, x, 2 * t + 1) & lo));
        }
    jm_pic_free(&q);
    jm_pic view;
    memset(&view, 0, sizeof(view));
    view.w = w; view.h = h; view.bd = bd; view.Y = Y; view.U = U; view.V = V;
    jm_pad_picture(&view, dw, dh);
}

static void synth8(jm_pic *p, int dw, int dh, uint64_t seed, int t) {
    uint64_t s = 0x5EED0000ULL + seed;
    rect_t R[12];
    for (int k = 0; k < 12; k++) {
        uint32_t a = hash3(s, k, 1, 99), b = hash3(s, k, 2, 99), c = hash3(s, k, 3, 99);
        R[k].w = 32 + (int)(a % 225);
        R[k].h = 32 + (int)(b % 225);
        R[k].vx = (int)(c % 161) - 80;                    /* +-20 pel/frame in qpel */
        R[k].vy = (int)((c >> 8) % 161) - 80;
        int x0 = (int)(hash3(s, k, 4, 99) % (uint32_t)dw), y0 = (int)(hash3(s, k, 5, 99) % (uint32_t)dh);
        int span_x = 4 * (dw + R[k].w), span_y = 4 * (dh + R[k].h);
        int px = (4 * x0 + R[k].vx * t) % span_x, py = (4 * y0 + R[k].vy * t) % span_y;
        if (px < 0) px += span_x;
        if (py < 0) py += span_y;
        R[k].x = px - 4 * R[k].w;                          /* wraps through the picture */
        R[k].y = py - 4 * R[k].h;
    }
    int gx = 12 * t + (t % 4), gy = -4 * t + ((t / 2) % 4);   /* global motion, qpel */
    for (int y = 0; y < dh; y++)
        for (int x = 0; x < dw; x++) {
            int X = 4 * x, Y = 4 * y, v = -1;
            for (int k = 11; k >= 0 && v < 0; k--)
                if (X >= R[k].x && X < R[k].x + 4 * R[k].w && Y >= R[k].y && Y < R[k].y + 4 * R[k].h)
                    v = texture(s + 1000 + k, X - R[k].x, Y - R[k].y, 0);
            if (v < 0) v = texture(s, X - gx, Y - gy, 0);
            v = 16 + (v * 219) / 255 + (int)(hash3(s, x, y, 7 + 3 * t) % 5) - 2;
            p->y[(size_t)y * p->w + x] = (uint8_t)(v < 16 ? 16 : v > 235 ? 235 : v);
        }
    for (int pl = 0; pl < 2; pl++) {
        uint8_t *P = pl ? p->v : p->u;
        int cw = p->w / 2;
        for (int y = 0; y < dh / 2; y++)
            for (int x = 0; x < dw / 2; x++) {
                int X = 8 * x, Y = 8 * y, v = -1;
                for (int k = 11; k >= 0 && v < 0; k--)
                    if (X >= R[k].x && X < R[k].x + 4 * R[k].w && Y >= R[k].y && Y < R[k].y + 4 * R[k].h)
                        v = texture(s + 1000 + k, X - R[k].x, Y - R[k].y, 8 + 4 * pl);
                if (v < 0) v = texture(s, X - gx, Y - gy, 8 + 4 * pl);
                v = 16 + (v * 224) / 255 + (int)(hash3(s, x, y, 1000 + 3 * t + pl) % 5) - 2;
                P[(size_t)y * cw + x] = (uint8_t)(v < 16 ? 16 : v > 240 ? 240 : v);
            }
    }
    jm_pad_picture(p, dw, dh);
}
