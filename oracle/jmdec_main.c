/* jmdec_main.c — closed-loop decoder CLI (TEST INFRASTRUCTURE ONLY): jmdec in.264 out.yuv */
#include <stdio.h>
#include <stdlib.h>
#include "jm_oracle.h"

int main(int argc, char **argv) {
    if (argc < 3) { fprintf(stderr, "usage: jmdec in.264 out.yuv\n"); return 1; }
    FILE *f = fopen(argv[1], "rb");
    if (!f) { perror(argv[1]); return 1; }
    fseek(f, 0, SEEK_END);
    long n = ftell(f);
    fseek(f, 0, SEEK_SET);
    unsigned char *buf = malloc(n > 0 ? n : 1);
    if (!buf || fread(buf, 1, n, f) != (size_t)n) { free(buf); fclose(f); return 1; }
    fclose(f);
    long cap = 64L * 1024 * 1024 * 16;
    unsigned char *out = malloc(cap);
    jmo_dec *d = NULL;
    if (!out || jmo_dec_create(&d)) { free(buf); free(out); return 1; }
    int w = 0, h = 0;
    int frames = jmo_decode_annexb(d, buf, n, out, cap, &w, &h);
    free(buf);
    if (frames < 0) { fprintf(stderr, "decode error: %s\n", jmo_dec_error(d)); jmo_dec_destroy(d); free(out); return 2; }
    FILE *o = fopen(argv[2], "wb");
    if (!o) { perror(argv[2]); jmo_dec_destroy(d); free(out); return 1; }
    const int bd = jmo_dec_bit_depth(d);
    fwrite(out, 1, (size_t)frames * w * h * 3 / 2 * (bd > 8 ? 2 : 1), o);   /* 16-bit LE above 8 bits */
    fclose(o);
    printf("decoded %d frames %dx%d bit depth %d\n", frames, w, h, bd);
    jmo_dec_destroy(d);
    free(out);
    return 0;
}
