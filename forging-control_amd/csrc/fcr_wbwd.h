// fcr_wbwd.h — H > 52 (config 5): the backward cell's gradient product [input grad | dh_{t-1}] = dG · [W_ih | W_hh]
// as ONE hand-written split-f16 MFMA GEMM (in place of rocBLAS gemm16_bwd's Cijk kernels where the shapes allow,
// fcr_abi.hip wide_hwbwd_ok). Reference: the autograd backward of nn.LSTM inside loss.backward() (Functions.py:325, :655).
//
// out[b][n] = sum_r dG[b][r] W[r][n] over the 4H gate rows r, fp32-accurate from f16 halves: with dG = dG_hi +
// dG_lo (the cell kernel's split of dG * scale, wide_cell_bwd_kernel) and W = W_hi + W_lo,
//   out = W_lo dG_hi + W_hi dG_lo + W_hi dG_hi      (three MFMAs per k-block; the dropped lo·lo is <= 2^-22)
// Against rocBLAS on the K-concatenated [hi | lo | hi] rows (K = 12H) every hi fragment is read ONCE for its two
// products, so a workgroup stages 4 halves per (row, k) instead of 6, and the dgate rows need no third copy.
//
// Operands (row-major, k contiguous): A = W^T split, [NO][lda] hi and lo (row n = output column: W_ih column n
// for n < H, W_hh column n - H — wide_split_bt_kernel); B = the dgate rows [B][ldb] hi, lo at +lo_off.
// MFMA roles: A = W^T (M = output columns), B = dG^T (N = trajectories), D[m][n] = out[b = n][col = m]: a lane's
// D fragment is 4 consecutive columns of one trajectory row, one 16-B store.
// Tile: a workgroup owns 256 output columns x 128 trajectories; 8 waves (4 along M x 2 along N), each 64 x 64 =
// 4 x 4 D tiles; K in steps of 32 (one k-block) through a 3-stage LDS-DMA ring (global_load_lds, 16 B per lane,
// two steps of prefetch, a bare s_barrier per step) — the staging of fcr_wgemm.h, with hi and lo stages. A stage
// is 256 + 256 + 128 + 128 rows of 64 B = 48 KB; 3 stages = 144 KB: one workgroup (8 waves, 2 per SIMD) per CU.
// XCD-aware order: a trajectory block's output-column blocks run on one XCD, so its dgate rows are read from HBM
// once into that XCD's L2.
#pragma once
#include "fcr_common.h"
#include "fcr_f16.h"

namespace fcr {

constexpr int kWbM = 256;                 // output columns per workgroup
constexpr int kWbN = 128;                 // trajectories per workgroup
constexpr int kWbK = 32;                  // k per step
constexpr int kWbWM = 4, kWbWN = 2;       // waves along the output columns x along the trajectories
constexpr int kWbWaves = kWbWM * kWbWN;
constexpr int kWbTM = kWbM / kWbWM / 16, kWbTN = kWbN / kWbWN / 16;   // D tiles per wave
constexpr int kWbThreads = 64 * kWbWaves;
constexpr int kWbStageA = kWbM * kWbK * 2;                // bytes of one split half of A
constexpr int kWbStageB = kWbN * kWbK * 2;
constexpr int kWbStage = 2 * kWbStageA + 2 * kWbStageB;   // hi A | lo A | hi B | lo B
constexpr int kWbStages = 3;
constexpr int kWbLds = kWbStages * kWbStage;
constexpr int kWbPieces = kWbStage / 1024 / kWbWaves;     // 1 KB LDS-DMA pieces per wave per stage
static_assert(kWbStage % (1024 * kWbWaves) == 0, "DMA pieces");
static_assert(kWbLds <= 163840, "LDS");

struct WbArgs {
    const _Float16 *Ahi, *Alo;   // [NO][lda]
    const _Float16 *B;           // dgate rows [B][ldb], hi at +0, lo at +lo_off halves
    float *out;                  // [B][ldo], columns [0, NO)
    const float *rs;             // [B] per-row factor applied to the output (the dgate rows' own inverse scales), or null
    int lda, ldb, lo_off, ldo, NB, NO, K;
};

// byte offset of 16-B chunk c of 64-B LDS row r: the swizzle puts the 8 rows of a fragment read's 8-lane phase
// on distinct 16-B slots of a 128-B bank line (fcr_wgemm.h wg_off)
__device__ __forceinline__ uint32_t wb_off(int r, int c) { return (uint32_t)(r * 64 + ((c ^ ((r >> 1) & 3)) << 4)); }

__global__ __launch_bounds__(kWbThreads, 1) void wide_bwd_gemm_kernel(WbArgs a) {
    static_assert(kWbPieces == 6 || kWbPieces == 12, "vmcnt immediates");
    extern __shared__ __attribute__((aligned(16))) char lds[];
    const int tid = threadIdx.x, lane = tid & 63;
    const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wm = wv % kWbWM, wn = wv / kWbWM;            // column slice, trajectory slice
    const int ny = (a.NO + kWbM - 1) / kWbM, total = gridDim.x, id = blockIdx.x;
    const int xcd = id & 7, loc = id >> 3, q8 = total >> 3, rr = total & 7;
    const int wg = (xcd < rr ? xcd * (q8 + 1) : rr * (q8 + 1) + (xcd - rr) * q8) + loc;
    const int m0 = (wg % ny) * kWbM;                       // first output column
    const int b0 = (wg / ny) * kWbN;                       // first trajectory
    const int nk = a.K / kWbK;

    // DMA piece j of a stage: 16 rows x 64 B of [A hi (16 pieces) | A lo (16) | B hi (8) | B lo (8)]; lane i lands
    // at +16 i (row i >> 2, slot i & 3) and fetches the global chunk the row's swizzle puts in that slot
    const _Float16 *gsrc[kWbPieces];
    uint32_t ldst[kWbPieces];
#pragma unroll
    for (int p = 0; p < kWbPieces; ++p) {
        const int j = wv + kWbWaves * p;
        const int part = j < 16 ? 0 : j < 32 ? 1 : j < 40 ? 2 : 3;
        const int base = part == 0 ? 0 : part == 1 ? 16 : part == 2 ? 32 : 40;
        const int r = 16 * (j - base) + (lane >> 2);
        const int c = (lane & 3) ^ ((r >> 1) & 3);
        if (part < 2) {
            int n = m0 + r;
            if (n >= a.NO) n = a.NO - 1;                   // tail columns recompute the last one (not stored)
            gsrc[p] = (part == 0 ? a.Ahi : a.Alo) + (size_t)n * a.lda + 8 * c;
        } else {
            int b = b0 + r;
            if (b >= a.NB) b = a.NB - 1;                   // tail rows recompute the last trajectory (not stored)
            gsrc[p] = a.B + (size_t)b * a.ldb + (part == 3 ? a.lo_off : 0) + 8 * c;
        }
        ldst[p] = (uint32_t)j * 1024;
    }
    auto dma = [&](int ks, int buf) {
#pragma unroll
        for (int p = 0; p < kWbPieces; ++p)
            __builtin_amdgcn_global_load_lds(
                (const __attribute__((address_space(1))) void *)(gsrc[p] + ks * kWbK),
                (__attribute__((address_space(3))) void *)((__attribute__((address_space(3))) char *)lds + buf * kWbStage +
                                                           ldst[p]),
                16, 0, 0);
    };

    f32x4 acc[kWbTM][kWbTN];
#pragma unroll
    for (int i = 0; i < kWbTM; ++i)
#pragma unroll
        for (int j = 0; j < kWbTN; ++j) acc[i][j] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
    const int fr = lane & 15, fq = lane >> 4;
    // two steps of prefetch: stage ks is waited for with step ks + 1's pieces still in flight (vmcnt counts this
    // wave's DMA in issue order); a bare s_barrier publishes every wave's pieces (fcr_wgemm.h)
    dma(0, 0);
    if (nk > 1) dma(1, 1);
    int buf = 0;
    for (int ks = 0; ks < nk; ++ks) {
        if (ks + 1 < nk) {
            if constexpr (kWbPieces == 6) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
            else asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
        } else {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
        const char *st = lds + buf * kWbStage;
        f16x8 ah[kWbTM], al[kWbTM], bh[kWbTN], bl[kWbTN];
#pragma unroll
        for (int j = 0; j < kWbTN; ++j) {
            const int r = 16 * (kWbTN * wn + j) + fr;
            bh[j] = *reinterpret_cast<const f16x8 *>(st + 2 * kWbStageA + wb_off(r, fq));
            bl[j] = *reinterpret_cast<const f16x8 *>(st + 2 * kWbStageA + kWbStageB + wb_off(r, fq));
        }
#pragma unroll
        for (int i = 0; i < kWbTM; ++i) {
            const int r = 16 * (kWbTM * wm + i) + fr;
            ah[i] = *reinterpret_cast<const f16x8 *>(st + wb_off(r, fq));
            al[i] = *reinterpret_cast<const f16x8 *>(st + kWbStageA + wb_off(r, fq));
        }
        const int nb = buf == 0 ? 2 : buf - 1;            // (ks + 2) % 3: every wave finished reading it at ks - 1
        if (ks + 2 < nk) dma(ks + 2, nb);
#pragma unroll
        for (int i = 0; i < kWbTM; ++i)
#pragma unroll
            for (int j = 0; j < kWbTN; ++j) acc[i][j] = mma3(ah[i], al[i], bh[j], bl[j], acc[i][j]);
        buf = buf == 2 ? 0 : buf + 1;
    }
    // ---- epilogue: lane = trajectory b0 + 16 (TN wn + j) + (lane & 15), columns m0 + 16 (TM wm + i) + 4 (lane >> 4) .. +3
#pragma unroll
    for (int j = 0; j < kWbTN; ++j) {
        const int b = b0 + 16 * (kWbTN * wn + j) + fr;
        if (b >= a.NB) continue;
        float *row = a.out + (size_t)b * a.ldo;
        const float f = a.rs ? a.rs[b] : 1.0f;
#pragma unroll
        for (int i = 0; i < kWbTM; ++i) {
            const int col = m0 + 16 * (kWbTM * wm + i) + 4 * fq;
            if (col < a.NO) *reinterpret_cast<f32x4 *>(row + col) = acc[i][j] * f;
        }
    }
}

// A of the gradient product, transposed and split: dst_hi / dst_lo [NO][4H], row n = output column n of
// [W_ih | W_hh] (layers >= 1, NO = 2H; `wih` null for layer 0: W_hh only, NO = H), column r = gate row r.
__global__ void wide_split_bt_kernel(const float *__restrict__ wih, const float *__restrict__ whh, int H, int NO,
                                     _Float16 *dst_hi, _Float16 *dst_lo) {
    const size_t idx = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int K = 4 * H;
    if (idx >= (size_t)NO * K) return;
    const int n = (int)(idx / K), r = (int)(idx % K);
    const float v = (wih && n < H) ? wih[(size_t)r * H + n] : whh[(size_t)r * H + (wih ? n - H : n)];
    const _Float16 hi = (_Float16)v;
    dst_hi[idx] = hi;
    dst_lo[idx] = (_Float16)(v - (float)hi);
}

}  // namespace fcr
