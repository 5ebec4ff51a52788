// fcr_wgemm.h — H > 52 (config 5): one LSTM cell of the whole batch as ONE hand-written split-f16 MFMA GEMM
// with the cell update in its epilogue (in place of rocBLAS gemm16_fwd + wide_cell_kernel, every layer).
// Used for every layer when H % 64 == 0: at config 5 it took the step from 703 to 657 ms (forward 219 -> 180
// ms), equal to the rocBLAS path within 2e-7 relative.
//
// Product: G[b][r] = sum_k XB[b][k] A[r][k], the K-concatenated split operands of fcr_wide.h (A = [Wih_hi |
// Wih_hi | Wih_lo | Whh_hi | Whh_hi | Whh_lo] rows r = gate*H + unit, XB = [x_hi | x_lo | x_hi | h_hi | h_lo |
// h_hi] rows b = trajectory), fp32 accumulate. A workgroup owns 64 units x 128 trajectories: its 256 A rows
// are taken unit-major, gate-minor (LDS row 4 u + gate), so an MFMA D fragment (16 rows x 16 trajectories;
// lane = trajectory lane & 15, rows 4 (lane >> 4) .. +3) holds the four gates i, f, g, o of ONE unit of ONE
// trajectory: the cell update runs on the accumulators, and the 4H x B gate matrix never goes to HBM.
//
// Tile walk: 4 waves (2 x 2), each 128 rows (32 units) x 64 trajectories = 8 x 4 D tiles (LDS reads 0.023
// B per MFMA flop, under the 0.031 one CU's LDS sustains at the MFMA peak); K in steps of 32 (one 16x16x32
// f16 k-block), A and XB chunks staged into LDS by LDS-DMA through a 3-stage ring, one barrier per step;
// 72 KB of LDS (the epilogue's tiles) lets two workgroups share a CU, so one's epilogue and barriers
// overlap the other's MFMAs. LDS rows are 64 B; their 16-B chunks are XOR-swizzled by (row >> 1) & 3, so
// the 8 rows of a ds_read_b128 phase land on distinct 16-B bank groups. (8 waves x 128 x 32 measured the
// same; K steps of 64 at one workgroup per CU 13 % slower; B fragments loaded straight from global memory
// into registers (64-B row pieces) 22 % slower; a second register set for a two-step prefetch 5 % slower.
// Diagnostic builds bound the loop: cache-hot operand loads gain 6 %, no loads and LDS stores at all 33 %:
// the staging (LDS write traffic and the wait before it), not HBM, is what the loop loses to. LDS-DMA
// (global_load_lds) was 2 % faster than the register round trip; a 3-stage ring with the next step's fragment
// reads overlapping the MFMAs 5 % slower; the 3-stage ring with two steps of DMA prefetch and a bare
// s_barrier (round 2f) took the config-5 forward from 191.9 to 188.0 ms, bit-identical — the loop is not
// waiting on HBM latency so much as on its per-step barrier and LDS traffic. The register-staged and 2-stage
// forms are in the history.)
#pragma once
#include "fcr_common.h"
#include "fcr_f16.h"

namespace fcr {

constexpr int kWgU = 64;                  // units per workgroup
constexpr int kWgM = 4 * kWgU;            // A rows per workgroup
constexpr int kWgN = 128;                 // trajectories per workgroup
constexpr int kWgK = 32;                  // K per step: 32 keeps the workgroup at 72 KB of LDS, two per CU
constexpr int kWgC = kWgK / 8;            // 16-B chunks per LDS row
constexpr int kWgWaves = 4;               // 2 x kWgWC waves; each 128 rows x kWgN / kWgWC trajectories
constexpr int kWgWC = kWgWaves / 2;
constexpr int kWgNT = kWgN / kWgWC / 16;  // D tiles per wave along the trajectories
constexpr int kWgThreads = 64 * kWgWaves;
constexpr int kWgStageA = kWgM * kWgK * 2;   // bytes
constexpr int kWgStageB = kWgN * kWgK * 2;
constexpr int kWgEpi = kWgN * ((kWgU + 4) * 4 + 2 * (kWgU + 8) * 2);   // the epilogue's c / hi / lo tiles
// LDS stages of the DMA mainloop: 3 = two steps of prefetch (the ring fits in the 72 KB the epilogue's tiles take
// anyway), the stage wait is vmcnt(pieces of one step), not vmcnt(0)
constexpr int kWgStages = 3;
constexpr int kWgLds = kWgStages * (kWgStageA + kWgStageB) > kWgEpi ? kWgStages * (kWgStageA + kWgStageB) : kWgEpi;

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

struct WgArgs {
    const _Float16 *A;     // [4H][lda]
    const _Float16 *XB;    // [B][ldb]
    int lda, ldb, K, B, H;
    const float *c_prev;   // [B][H] or null (t = 0)
    float *c_out;          // [B][H]
    float *h_out;          // [B][H] or null
    float *preact;         // [B][4H] or null: the gate pre-activations (the backward's recompute keeps them)
    _Float16 *xb_h;        // next cell's operand row h part (3H halves at +u, +H+u, +2H+u), stride sh, or null
    _Float16 *xb_x;        // layer above's operand row x part, stride sx, or null
    int sh, sx;
};

// byte offset of 16-B chunk c of LDS row r in a stage; the swizzle puts the 8 rows of a fragment read's
// 8-lane phase on the 8 distinct 16-B slots of a 128-B bank line
__device__ __forceinline__ uint32_t wg_off(int r, int c) { return (uint32_t)(r * 64 + ((c ^ ((r >> 1) & 3)) << 4)); }

__global__ __launch_bounds__(kWgThreads, 2) void wide_gemm_cell_kernel(WgArgs a) {
    extern __shared__ __attribute__((aligned(16))) char lds[];
    const int tid = threadIdx.x, lane = tid & 63;
    const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wr = wv / kWgWC, wc = wv % kWgWC;         // wave's 128-row half, trajectory slice
    const int H = a.H;
    // XCD-aware walk (consecutive workgroup ids go to different XCDs, each with its own L2): the ids an XCD
    // receives are renumbered contiguously and walk the unit blocks fastest, so a trajectory block's operand
    // rows come from HBM once into that XCD's L2 and serve its 4H / 256 unit blocks (bijective for any count)
    const int ny = H / kWgU, total = gridDim.x, id = blockIdx.x;
    const int xcd = id & 7, loc = id >> 3, q = total >> 3, rr = total & 7;
    const int wg = (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + loc;
    const int u0 = (wg % ny) * kWgU;                   // first unit of the workgroup
    const int b0 = (wg / ny) * kWgN;                   // first trajectory
    const int nk = a.K / kWgK;

    // LDS-DMA staging (global_load_lds, 16 B per lane): one wave instruction fills one 1 KB piece of a stage
    // = 16 rows x 64 B; lane i lands at +16 i, i.e. row i >> 2, slot i & 3, so it fetches the global chunk
    // that the row's swizzle puts in that slot. A stage is 16 A pieces + 8 B pieces, 6 per wave.
    constexpr int NPC = (kWgStageA + kWgStageB) / 1024 / kWgWaves;
    static_assert(kWgC == 4 && (kWgStageA + kWgStageB) % (1024 * kWgWaves) == 0, "DMA pieces");
    const _Float16 *gsrc[NPC];
    uint32_t ldst[NPC];
#pragma unroll
    for (int q = 0; q < NPC; ++q) {
        const int j = wv + kWgWaves * q;                  // piece of the stage
        const bool isA = j < kWgStageA / 1024;
        const int r = 16 * (isA ? j : j - kWgStageA / 1024) + (lane >> 2);
        const int c = (lane & 3) ^ ((r >> 1) & 3);
        if (isA) {
            gsrc[q] = a.A + (size_t)((r & 3) * H + u0 + (r >> 2)) * a.lda + 8 * c;
        } else {
            int b = b0 + r;
            if (b >= a.B) b = a.B - 1;                     // tail rows recompute the last trajectory (not stored)
            gsrc[q] = a.XB + (size_t)b * a.ldb + 8 * c;
        }
        ldst[q] = (uint32_t)j * 1024;
    }
    auto dma = [&](int ks, int buf) {
#pragma unroll
        for (int q = 0; q < NPC; ++q)
            __builtin_amdgcn_global_load_lds(
                (const __attribute__((address_space(1))) void *)(gsrc[q] + ks * kWgK),
                (__attribute__((address_space(3))) void *)((__attribute__((address_space(3))) char *)lds +
                                                           buf * (kWgStageA + kWgStageB) + ldst[q]),
                16, 0, 0);
    };

    f32x4 acc[8][kWgNT];
#pragma unroll
    for (int m = 0; m < 8; ++m)
#pragma unroll
        for (int n = 0; n < kWgNT; ++n) acc[m][n] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
    const int fr = lane & 15, fq = lane >> 4;
    // two steps of prefetch: stage ks is waited for with step ks + 1's pieces still in flight (vmcnt counts
    // this wave's DMA in issue order), and the barrier is a bare s_barrier: __syncthreads()'s release fence
    // would drain every outstanding load (vmcnt(0)). The empty asm statements keep the compiler's LDS
    // accesses on their side of it.
    dma(0, 0);
    if (nk > 1) dma(1, 1);
    int buf = 0;
    for (int ks = 0; ks < nk; ++ks) {
        if (ks + 1 < nk) {
            static_assert(NPC == 6, "vmcnt immediate");
            asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
        } else {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
        const char *base = lds + buf * (kWgStageA + kWgStageB);
        f16x8 af[8], bf[kWgNT];
#pragma unroll
        for (int n = 0; n < kWgNT; ++n)
            bf[n] = *reinterpret_cast<const f16x8 *>(base + kWgStageA + wg_off(16 * (kWgNT * wc + n) + fr, fq));
#pragma unroll
        for (int m = 0; m < 8; ++m) af[m] = *reinterpret_cast<const f16x8 *>(base + wg_off(128 * wr + 16 * m + fr, fq));
        const int nb = buf == 0 ? 2 : buf - 1;       // (ks + 2) % 3: the stage every wave finished reading at ks - 1
        if (ks + 2 < nk) dma(ks + 2, nb);
#pragma unroll
        for (int m = 0; m < 8; ++m)
#pragma unroll
            for (int n = 0; n < kWgNT; ++n) acc[m][n] = mfma16(af[m], bf[n], acc[m][n]);
        buf = buf == 2 ? 0 : buf + 1;
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    // ---- epilogue: the cell update (wide_cell_kernel's arithmetic) on the accumulators, through LDS ----
    // A lane holds (trajectory, unit) pairs scattered over 16 rows; the slabs want whole rows. So the c_prev
    // tile comes in by rows, each lane updates its pairs in LDS tiles [trajectory][unit] (rows padded by 16 B:
    // 2-way bank conflicts at most, chunks stay 16-B aligned), and c, the operand halves and (keep_act) the
    // pre-activations go out by rows again.
    constexpr int CSTR = kWgU + 4;            // floats per c row
    constexpr int HSTR = kWgU + 8;            // halves per hi / lo row
    float *cs = reinterpret_cast<float *>(lds);                                   // [128][CSTR]
    _Float16 *hs = reinterpret_cast<_Float16 *>(lds + kWgN * CSTR * 4);           // [128][HSTR]
    _Float16 *ls = hs + kWgN * HSTR;                                              // [128][HSTR]
    constexpr int ERS = kWgThreads / 16;      // row-wise passes: ERS rows x 16 chunks per pass
    const int er = tid >> 4, ec = tid & 15;
    auto row_b = [&](int r) { return b0 + r; };
    if (a.c_prev) {
#pragma unroll
        for (int p = 0; p < kWgN / ERS; ++p) {
            const int r = er + ERS * p, b = row_b(r);
            if (b < a.B)
                *reinterpret_cast<f32x4 *>(cs + r * CSTR + 4 * ec) =
                    *reinterpret_cast<const f32x4 *>(a.c_prev + (size_t)b * H + u0 + 4 * ec);
        }
    }
    __syncthreads();
#pragma unroll
    for (int n = 0; n < kWgNT; ++n) {
        const int r = 16 * (kWgNT * wc + n) + fr;
#pragma unroll
        for (int m = 0; m < 8; ++m) {
            const int ul = 32 * wr + 4 * m + fq;
            const f32x4 g4 = acc[m][n];
            const float cp = a.c_prev ? cs[r * CSTR + ul] : 0.0f;
            const float i = sigm(g4[0]), f = sigm(g4[1]), g = tanhf(g4[2]), o = sigm(g4[3]);
            const float c = (a.c_prev ? f * cp : 0.0f) + i * g;
            const float h = o * tanhf(c);
            const _Float16 hi = (_Float16)h;
            cs[r * CSTR + ul] = c;
            hs[r * HSTR + ul] = hi;
            ls[r * HSTR + ul] = (_Float16)(h - (float)hi);
            const int b = b0 + r;
            if (a.h_out && b < a.B) a.h_out[(size_t)b * H + u0 + ul] = h;   // the readout's cell only
        }
    }
    __syncthreads();
#pragma unroll
    for (int p = 0; p < kWgN / ERS; ++p) {
        const int r = er + ERS * p, b = row_b(r);
        if (b >= a.B) continue;
        *reinterpret_cast<f32x4 *>(a.c_out + (size_t)b * H + u0 + 4 * ec) = *reinterpret_cast<const f32x4 *>(cs + r * CSTR + 4 * ec);
        if (ec < 8) {   // 8 chunks of 8 halves per row: the hi and lo halves of 64 units
            const u32x4 hv = *reinterpret_cast<const u32x4 *>(hs + r * HSTR + 8 * ec);
            const u32x4 lv = *reinterpret_cast<const u32x4 *>(ls + r * HSTR + 8 * ec);
            if (a.xb_h) {
                _Float16 *q = a.xb_h + (size_t)b * a.sh + u0 + 8 * ec;
                *reinterpret_cast<u32x4 *>(q) = hv;
                *reinterpret_cast<u32x4 *>(q + H) = lv;
                *reinterpret_cast<u32x4 *>(q + 2 * H) = hv;
            }
            if (a.xb_x) {
                _Float16 *q = a.xb_x + (size_t)b * a.sx + u0 + 8 * ec;
                *reinterpret_cast<u32x4 *>(q) = hv;
                *reinterpret_cast<u32x4 *>(q + H) = lv;
                *reinterpret_cast<u32x4 *>(q + 2 * H) = hv;
            }
        }
    }
    if (a.preact) {   // gate by gate through the c tile: rows of 64 pre-activations
#pragma unroll
        for (int gt = 0; gt < 4; ++gt) {
            __syncthreads();
#pragma unroll
            for (int n = 0; n < kWgNT; ++n)
#pragma unroll
                for (int m = 0; m < 8; ++m) cs[(16 * (kWgNT * wc + n) + fr) * CSTR + 32 * wr + 4 * m + fq] = acc[m][n][gt];
            __syncthreads();
#pragma unroll
            for (int p = 0; p < kWgN / ERS; ++p) {
                const int r = er + ERS * p, b = row_b(r);
                if (b < a.B)
                    *reinterpret_cast<f32x4 *>(a.preact + (size_t)b * 4 * H + gt * H + u0 + 4 * ec) =
                        *reinterpret_cast<const f32x4 *>(cs + r * CSTR + 4 * ec);
            }
        }
    }
}

}  // namespace fcr
