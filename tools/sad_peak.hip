// tools/sad_peak.hip — issue-rate microbenchmark of the gfx950 sum-of-absolute-differences
// instructions, to price the VALU roofline of the FFS SAD table (BASELINE.md:
// "the v_sad_u8 peak, which is microbenchmarked on the node").
//
// Each lane runs 8 independent accumulator chains of one instruction (inline asm, so nothing is
// hoisted or folded), the whole chip full of waves.  Reports per instruction: lane-ops/s, absolute
// differences/s (AD per lane-op: v_sad_u8 / v_msad_u8 / v_sad_hi_u8 4, v_sad_u16 2, the quad forms
// v_qsad_pk_u16_u8 / v_mqsad_pk_u16_u8 / v_mqsad_u32_u8 16) and lane-ops per CU per shader clock
// (the clock measured in-kernel: s_memtime / s_memrealtime).  Prints one JSON object.
//   hipcc --offload-arch=gfx950 -O3 tools/sad_peak.hip -o tools/sad_peak_bin && tools/sad_peak_bin
#include <hip/hip_runtime.h>
#include <stdio.h>

typedef unsigned v4u __attribute__((ext_vector_type(4)));
typedef unsigned long long u64;

#define NT 256
#define ITERS 2048

enum Op { SAD_U8, MSAD_U8, SAD_HI_U8, SAD_U16, QSAD_PK, MQSAD_PK, MQSAD_U32, V_ADD_U32, NOPS };
static const char *kName[NOPS] = {"v_sad_u8", "v_msad_u8", "v_sad_hi_u8", "v_sad_u16", "v_qsad_pk_u16_u8",
                                  "v_mqsad_pk_u16_u8", "v_mqsad_u32_u8", "v_add_u32"};
static const int kAd[NOPS] = {4, 4, 4, 2, 16, 16, 16, 0};

template <int OP>
__global__ __launch_bounds__(NT) void k_sad(unsigned seed, unsigned *out, u64 *clk) {
    const unsigned t = blockIdx.x * NT + threadIdx.x;
    unsigned a = t * 2654435761u ^ seed, b = a * 40503u + 17u;
    u64 q = ((u64)a << 32) | b;
    u64 t0 = 0, r0 = 0;
    if (threadIdx.x == 0) { t0 = __builtin_amdgcn_s_memtime(); r0 = __builtin_amdgcn_s_memrealtime(); }
    unsigned s = 0;
    if (OP == MQSAD_U32) {
        v4u c[8];
        for (int k = 0; k < 8; k++) c[k] = (v4u){a + k, b, a ^ k, b + k};
        for (int i = 0; i < ITERS; i++) {
#pragma unroll
            for (int k = 0; k < 8; k++) asm volatile("v_mqsad_u32_u8 %0, %1, %2, %0" : "+v"(c[k]) : "v"(q), "v"(b));
#pragma unroll
            for (int k = 0; k < 8; k++) asm volatile("v_mqsad_u32_u8 %0, %1, %2, %0" : "+v"(c[k]) : "v"(q), "v"(a));
        }
        for (int k = 0; k < 8; k++) s += c[k].x + c[k].y + c[k].z + c[k].w;
    } else if (OP == QSAD_PK || OP == MQSAD_PK) {
        u64 c[8];
        for (int k = 0; k < 8; k++) c[k] = q + k;
        for (int i = 0; i < ITERS; i++) {
#pragma unroll
            for (int k = 0; k < 8; k++) {
                if (OP == QSAD_PK) asm volatile("v_qsad_pk_u16_u8 %0, %1, %2, %0" : "+v"(c[k]) : "v"(q), "v"(b));
                else asm volatile("v_mqsad_pk_u16_u8 %0, %1, %2, %0" : "+v"(c[k]) : "v"(q), "v"(b));
            }
#pragma unroll
            for (int k = 0; k < 8; k++) {
                if (OP == QSAD_PK) asm volatile("v_qsad_pk_u16_u8 %0, %1, %2, %0" : "+v"(c[k]) : "v"(q), "v"(a));
                else asm volatile("v_mqsad_pk_u16_u8 %0, %1, %2, %0" : "+v"(c[k]) : "v"(q), "v"(a));
            }
        }
        for (int k = 0; k < 8; k++) s += (unsigned)c[k] + (unsigned)(c[k] >> 32);
    } else {
        unsigned c[8];
        for (int k = 0; k < 8; k++) c[k] = a + k;
        for (int i = 0; i < ITERS; i++) {
#pragma unroll
            for (int k = 0; k < 8; k++) {
                if (OP == SAD_U8) asm volatile("v_sad_u8 %0, %1, %2, %0" : "+v"(c[k]) : "v"(a), "v"(b));
                if (OP == MSAD_U8) asm volatile("v_msad_u8 %0, %1, %2, %0" : "+v"(c[k]) : "v"(a), "v"(b));
                if (OP == SAD_HI_U8) asm volatile("v_sad_hi_u8 %0, %1, %2, %0" : "+v"(c[k]) : "v"(a), "v"(b));
                if (OP == SAD_U16) asm volatile("v_sad_u16 %0, %1, %2, %0" : "+v"(c[k]) : "v"(a), "v"(b));
                if (OP == V_ADD_U32) asm volatile("v_add_u32 %0, %1, %0" : "+v"(c[k]) : "v"(a));
            }
#pragma unroll
            for (int k = 0; k < 8; k++) {
                if (OP == SAD_U8) asm volatile("v_sad_u8 %0, %1, %2, %0" : "+v"(c[k]) : "v"(b), "v"(a));
                if (OP == MSAD_U8) asm volatile("v_msad_u8 %0, %1, %2, %0" : "+v"(c[k]) : "v"(b), "v"(a));
                if (OP == SAD_HI_U8) asm volatile("v_sad_hi_u8 %0, %1, %2, %0" : "+v"(c[k]) : "v"(b), "v"(a));
                if (OP == SAD_U16) asm volatile("v_sad_u16 %0, %1, %2, %0" : "+v"(c[k]) : "v"(b), "v"(a));
                if (OP == V_ADD_U32) asm volatile("v_add_u32 %0, %1, %0" : "+v"(c[k]) : "v"(b));
            }
        }
        for (int k = 0; k < 8; k++) s += c[k];
    }
    out[t] = s;
    if (threadIdx.x == 0 && blockIdx.x == 0) {
        clk[0] = __builtin_amdgcn_s_memtime() - t0;
        clk[1] = __builtin_amdgcn_s_memrealtime() - r0;
    }
}

#define CHK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); return 1; } } while (0)

template <int OP>
static int run(int blocks, unsigned *out, u64 *clk, double *ops_per_s, double *ghz) {
    hipEvent_t e0, e1;
    CHK(hipEventCreate(&e0)); CHK(hipEventCreate(&e1));
    hipLaunchKernelGGL(k_sad<OP>, dim3(blocks), dim3(NT), 0, 0, 1u, out, clk);   // warm-up
    CHK(hipDeviceSynchronize());
    float best = 1e30f;
    for (int rep = 0; rep < 5; rep++) {
        CHK(hipEventRecord(e0, 0));
        hipLaunchKernelGGL(k_sad<OP>, dim3(blocks), dim3(NT), 0, 0, 2u + rep, out, clk);
        CHK(hipEventRecord(e1, 0));
        CHK(hipEventSynchronize(e1));
        float ms = 0;
        CHK(hipEventElapsedTime(&ms, e0, e1));
        if (ms < best) best = ms;
    }
    u64 h[2];
    CHK(hipMemcpy(h, clk, sizeof(h), hipMemcpyDeviceToHost));
    *ghz = h[1] ? (double)h[0] / (double)h[1] * 0.1 : 0.0;   // s_memrealtime runs at 100 MHz
    *ops_per_s = (double)blocks * NT * ITERS * 16 / (best * 1e-3);
    CHK(hipEventDestroy(e0)); CHK(hipEventDestroy(e1));
    return 0;
}

int main() {
    hipDeviceProp_t prop;
    CHK(hipGetDeviceProperties(&prop, 0));
    const int cus = prop.multiProcessorCount;
    const int blocks = cus * 32;   // 8 waves per SIMD requested; residency decides the rest
    unsigned *out;
    u64 *clk;
    CHK(hipMalloc(&out, (size_t)blocks * NT * 4));
    CHK(hipMalloc(&clk, 16));
    double ops[NOPS], ghz[NOPS];
    int r = 0;
    r |= run<SAD_U8>(blocks, out, clk, &ops[SAD_U8], &ghz[SAD_U8]);
    r |= run<MSAD_U8>(blocks, out, clk, &ops[MSAD_U8], &ghz[MSAD_U8]);
    r |= run<SAD_HI_U8>(blocks, out, clk, &ops[SAD_HI_U8], &ghz[SAD_HI_U8]);
    r |= run<SAD_U16>(blocks, out, clk, &ops[SAD_U16], &ghz[SAD_U16]);
    r |= run<QSAD_PK>(blocks, out, clk, &ops[QSAD_PK], &ghz[QSAD_PK]);
    r |= run<MQSAD_PK>(blocks, out, clk, &ops[MQSAD_PK], &ghz[MQSAD_PK]);
    r |= run<MQSAD_U32>(blocks, out, clk, &ops[MQSAD_U32], &ghz[MQSAD_U32]);
    r |= run<V_ADD_U32>(blocks, out, clk, &ops[V_ADD_U32], &ghz[V_ADD_U32]);
    if (r) return 1;
    printf("{\"device\": \"%s\", \"cus\": %d, \"blocks\": %d, \"threads_per_block\": %d, \"ops\": {", prop.gcnArchName, cus, blocks, NT);
    for (int o = 0; o < NOPS; o++) {
        const double per_cu_clk = ops[o] / cus / (ghz[o] * 1e9);
        printf("%s\"%s\": {\"lane_ops_per_s\": %.4e, \"ad_per_lane_op\": %d, \"ad_per_s\": %.4e, \"clock_ghz\": %.3f, "
               "\"lane_ops_per_cu_per_clk\": %.2f, \"ad_per_s_at_2p4ghz\": %.4e}",
               o ? ", " : "", kName[o], ops[o], kAd[o], ops[o] * kAd[o], ghz[o], per_cu_clk, per_cu_clk * cus * 2.4e9 * kAd[o]);
    }
    printf("}}\n");
    return 0;
}
