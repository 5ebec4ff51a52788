// mfma_shape.hip — A/B of the two f16 MFMA shapes under the H = 50 backward's instruction mix.
//
// The backward cell (fcr_bwd.h) issues, per 16-trajectory wave and cell, ~227 v_mfma_f32_16x16x32_f16 beside ~653
// other VALU (~105 of them 8-cycle transcendentals), two waves per SIMD (profiles/round3c_stall_counters.txt). The
// 32x32x16 form would give a wave 32 trajectories: the same MFMA count per wave for twice the work (each 32x32x16
// holds issue 8 of its 32 cycles instead of 8 of 16), twice the VALU per wave, half the waves. This kernel runs that
// mix on random f16 operands with the MFMA -> VALU -> MFMA dependencies of the cell (accumulators consumed by the
// VALU streams, whose values become the next operands), sustained back to back, and reports wall time per unit of
// work and the in-kernel clock (s_memtime / s_memrealtime, MI355X_MICROARCH.md DVFS item 6) for:
//   s16: 16x16x32, 4 chains, V VALU + T transcendental per MFMA, 4096 waves (2 per SIMD, two rounds)
//   s32: 32x32x16, 2 chains, 2V VALU + 2T transcendental per MFMA, 2048 waves (2 per SIMD, one round)
// equal total MFMA FLOP and equal total VALU. It models the issue port and the clock, not the register pressure
// (the real 32-trajectory cell doubles the per-lane state: DESIGN.md §6).
//   hipcc -O3 --offload-arch=gfx950 -o mfma_shape mfma_shape.hip && ./mfma_shape
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#include <utility>

typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

#define CHECK(x)                                                                         \
    do {                                                                                 \
        hipError_t e = (x);                                                              \
        if (e != hipSuccess) {                                                           \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e));    \
            exit(1);                                                                     \
        }                                                                                \
    } while (0)

constexpr int kSteps = 8;   // MFMA steps per iteration (one dependency round trip per iteration)

// SH: 16 or 32. V / T: plain VALU and transcendentals per MFMA (times 16 to allow fractions: V16 = 16 V).
template <int SH, int V16, int T16, int ILP, int WPB = 8>
__global__ __launch_bounds__(64 * WPB, WPB == 8 ? 2 : 1) void mix_kernel(const _Float16 *__restrict__ src, float *__restrict__ dst, int iters,
                                                     unsigned long long *clk) {
    constexpr int CH = SH == 16 ? 4 : 2;             // independent accumulator chains
    constexpr int NV = (V16 * CH * kSteps) / 16;     // plain VALU per iteration
    constexpr int NT = (T16 * CH * kSteps) / 16;     // transcendentals per iteration
    constexpr int NS = SH == 16 ? ILP : 2 * ILP;     // independent VALU streams per lane: twice the units per lane at 32
    const int lane = threadIdx.x & 63;
    const size_t wid = (size_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    const _Float16 *s = src + (wid * 64 + lane) % 4096 * 32;
    f16x8 a[CH], b[CH];
    for (int c = 0; c < CH; ++c)
        for (int j = 0; j < 8; ++j) {
            a[c][j] = s[c * 8 + j];
            b[c][j] = s[(c * 8 + j + 5) % 32];
        }
    float v[NS];
    for (int k = 0; k < NS; ++k) v[k] = (float)s[k] + 1.5f;
    f32x4 acc16[4] = {};
    f32x16 acc32[2] = {};
    unsigned long long t0 = 0, r0 = 0;
    if (lane == 0) {
        t0 = __builtin_amdgcn_s_memtime();
        r0 = __builtin_amdgcn_s_memrealtime();
    }
    for (int it = 0; it < iters; ++it) {
        // kSteps MFMA steps, each one MFMA per chain with its share of the VALU streams interleaved (the shares are
        // compile-time per step, so the totals are exact: NV, NT per iteration)
        auto step = [&](auto stc) {
            constexpr int st = decltype(stc)::value;
            constexpr int nv = (st + 1) * NV / kSteps - st * NV / kSteps;
            constexpr int nt = (st + 1) * NT / kSteps - st * NT / kSteps;
#pragma unroll
            for (int c = 0; c < CH; ++c) {
                if constexpr (SH == 16) acc16[c] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a[c], b[c], acc16[c], 0, 0, 0);
                else acc32[c] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a[c], b[c], acc32[c], 0, 0, 0);
            }
#pragma unroll
            for (int k = 0; k < nv; ++k) v[(st * 7 + k) % NS] = fmaf(v[(st * 7 + k) % NS], 0.999f, 0.001f);
#pragma unroll
            for (int k = 0; k < nt; ++k) v[(st * 5 + k + 3) % NS] = __builtin_amdgcn_rcpf(v[(st * 5 + k + 3) % NS]);
            constexpr int per = (nv + nt + CH - 1) / CH;
#pragma unroll
            for (int c = 0; c < CH; ++c) {
                __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);     // one MFMA
                __builtin_amdgcn_sched_group_barrier(0x002, per, 0);   // then its VALU share
            }
        };
        [&]<int... S>(std::integer_sequence<int, S...>) { (step(std::integral_constant<int, S>{}), ...); }
        (std::make_integer_sequence<int, kSteps>{});
        // dependency round trip: accumulators into the VALU streams, the streams into the next B operands
#pragma unroll
        for (int c = 0; c < CH; ++c) {
            const float x = SH == 16 ? acc16[c][c] : acc32[c][c];
            v[c] += x * 1e-9f;
            b[c][c] = (_Float16)v[c + CH];
        }
    }
    float r = 0.0f;
    for (int k = 0; k < NS; ++k) r += v[k];
    for (int c = 0; c < CH; ++c) r += SH == 16 ? acc16[c][0] + acc16[c][3] : acc32[c][0] + acc32[c][15];
    dst[wid * 64 + lane] = r;
    if (lane == 0 && (threadIdx.x >> 6) == 0) {
        clk[2 * blockIdx.x] = __builtin_amdgcn_s_memtime() - t0;
        clk[2 * blockIdx.x + 1] = __builtin_amdgcn_s_memrealtime() - r0;
    }
}

// WPB 8: eight waves per workgroup, two per SIMD; WPB 4 with 160 KB of (unused) LDS: one workgroup per CU, one wave per
// SIMD — what a 32-trajectory cell whose state needs more than 256 registers would run at. PAD16: MFMA work per unit of
// useful work x 16 (the 32x32 tile covers 8 units: 56 for H = 50 against 52 on 16x16 tiles, 17/16 ~ 1.077 -> the
// VALU of a variant with padding is its unpadded VALU / 1.077, and its useful FLOP the executed / 1.077).
template <int SH, int V16, int T16, int ILP = 8, int WPB = 8, int PAD16 = 16>
void run(const char *tag, const _Float16 *src, float *dst, unsigned long long *clk, int iters, double target_s) {
    const int waves = SH == 16 ? 4096 : 2048;
    const int blocks = waves / WPB;
    const int lds = WPB == 8 ? 0 : 160 * 1024;
    if (lds) CHECK(hipFuncSetAttribute((const void *)mix_kernel<SH, V16, T16, ILP, WPB>, hipFuncAttributeMaxDynamicSharedMemorySize, lds));
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    // warm-up and sizing
    hipLaunchKernelGGL((mix_kernel<SH, V16, T16, ILP, WPB>), dim3(blocks), dim3(64 * WPB), lds, 0, src, dst, iters, clk);
    CHECK(hipDeviceSynchronize());
    CHECK(hipEventRecord(e0));
    hipLaunchKernelGGL((mix_kernel<SH, V16, T16, ILP, WPB>), dim3(blocks), dim3(64 * WPB), lds, 0, src, dst, iters, clk);
    CHECK(hipEventRecord(e1));
    CHECK(hipEventSynchronize(e1));
    float ms1 = 0.0f;
    CHECK(hipEventElapsedTime(&ms1, e0, e1));
    int reps = (int)(target_s * 1e3 / ms1);
    if (reps < 3) reps = 3;
    CHECK(hipEventRecord(e0));
    for (int r = 0; r < reps; ++r)
        hipLaunchKernelGGL((mix_kernel<SH, V16, T16, ILP, WPB>), dim3(blocks), dim3(64 * WPB), lds, 0, src, dst, iters, clk);
    CHECK(hipEventRecord(e1));
    CHECK(hipEventSynchronize(e1));
    float ms = 0.0f;
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    ms /= reps;
    unsigned long long *h = (unsigned long long *)malloc(16 * blocks);
    CHECK(hipMemcpy(h, clk, 16 * blocks, hipMemcpyDeviceToHost));
    double ghz = 0.0;
    for (int b = 0; b < blocks; ++b) ghz += (double)h[2 * b] / (double)h[2 * b + 1] * 0.1;   // memrealtime: 100 MHz
    ghz /= blocks;
    free(h);
    constexpr int CH = SH == 16 ? 4 : 2;
    const double flop = (double)waves * iters * kSteps * CH * (SH == 16 ? 16.0 * 16 * 32 : 32.0 * 32 * 16) * 2;
    const double useful_ms = ms * PAD16 / 16.0;   // time per unit of useful work, padding charged
    printf("{\"tag\": \"%s\", \"waves_per_simd\": %d, \"pad\": %.3f, \"ms_per_useful\": %.4f, \"ilp\": %d, \"shape\": \"%dx%dx%d\", \"valu_per_mfma\": %.3f, \"trans_per_mfma\": %.3f, \"waves\": %d, "
           "\"ms\": %.4f, \"tflops\": %.1f, \"clock_ghz\": %.3f, \"cycles_per_mfma_per_simd\": %.2f}\n",
           tag, WPB == 8 ? 2 : 1, PAD16 / 16.0, useful_ms, SH == 16 ? ILP : 2 * ILP, SH, SH, SH == 16 ? 32 : 16, V16 / 16.0, T16 / 16.0, waves, ms, flop / (ms * 1e-3) / 1e12, ghz,
           ghz * 1e9 * ms * 1e-3 / ((double)waves / 1024 * iters * kSteps * CH));
    fflush(stdout);
}

int main(int argc, char **argv) {
    const int iters = argc > 1 ? atoi(argv[1]) : 400;
    const double target_s = argc > 2 ? atof(argv[2]) : 2.0;
    const size_t n = 4096 * 32;
    _Float16 *h = (_Float16 *)malloc(n * 2);
    srand(1);
    for (size_t i = 0; i < n; ++i) h[i] = (_Float16)((rand() / (float)RAND_MAX) * 2.0f - 1.0f);   // random operands
    _Float16 *src;
    float *dst;
    unsigned long long *clk;
    CHECK(hipMalloc(&src, n * 2));
    CHECK(hipMalloc(&dst, 4096 * 64 * 4));
    CHECK(hipMalloc(&clk, 16 * 512));
    CHECK(hipMemcpy(src, h, n * 2, hipMemcpyHostToDevice));
    // the backward's mix: 653 VALU (105 transcendental) per 227 MFMA per wave-cell -> V = 2.41, T = 0.46 per 16x16x32
    // (16ths: V16 = 39, T16 = 7); the 32-trajectory wave twice that per 32x32x16. Bare MFMA loops for reference.
    run<16, 0, 0>("bare", src, dst, clk, iters, target_s);
    run<32, 0, 0>("bare", src, dst, clk, iters, target_s);
    run<16, 39, 7>("bwd_mix", src, dst, clk, iters, target_s);
    run<32, 78, 14>("bwd_mix", src, dst, clk, iters, target_s);
    // the forward's mix: 298 VALU (101 transcendental) per 108 MFMA -> V = 1.82, T = 0.94
    run<16, 29, 15>("fwd_mix", src, dst, clk, iters, target_s);
    run<32, 58, 30>("fwd_mix", src, dst, clk, iters, target_s);
    // less independent VALU work per lane (the real cell's chains are short: 64 % issue efficiency at two waves)
    run<16, 39, 7, 4>("bwd_mix_ilp", src, dst, clk, iters, target_s);
    run<32, 78, 14, 4>("bwd_mix_ilp", src, dst, clk, iters, target_s);
    // the 32-trajectory cell as it would be built: 56 units on 32x32 tiles against 52 (MFMA work x 17/16 per useful
    // work, its VALU unchanged per useful work: 78 / (17/16) = 73, 14 -> 13), at two and at one wave per SIMD
    run<32, 73, 13, 8, 8, 17>("bwd_mix_pad", src, dst, clk, iters, target_s);
    run<32, 73, 13, 8, 4, 17>("bwd_mix_pad_1wave", src, dst, clk, iters, target_s);
    run<32, 73, 13, 4, 4, 17>("bwd_mix_pad_1wave_ilp", src, dst, clk, iters, target_s);
    // order reversed (DVFS drift check)
    run<32, 78, 14>("bwd_mix_rev", src, dst, clk, iters, target_s);
    run<16, 39, 7>("bwd_mix_rev", src, dst, clk, iters, target_s);
    return 0;
}
