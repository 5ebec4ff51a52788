// fcr_wgemm.h — H > 52 (config 5): one LSTM cell of the whole batch as ONE hand-written split-f16 MFMA GEMM
// with the cell update in its epilogue (in place of rocBLAS gemm16_fwd + wide_cell_kernel for layers >= 1).
// Experimental, built with FCR_WIDE_FUSED=1 (fcr_abi.hip): correct, but its mainloop is ~2x slower than
// rocBLAS's Tensile kernel at this shape — the deep-pipelined 256^2 structure of cdna_hip_programming.md §5
// is what it would need before the fused epilogue (no 4H x B gate matrix in HBM) pays.
//
// Product: G[b][r] = sum_k XB[b][k] A[r][k], the K-concatenated split operands of fcr_wide.h (A = [Wih_hi |
// Wih_hi | Wih_lo | Whh_hi | Whh_hi | Whh_lo] rows r = gate*H + unit, XB = [x_hi | x_lo | x_hi | h_hi | h_lo |
// h_hi] rows b = trajectory), fp32 accumulate. A workgroup owns 64 units x 128 trajectories: its 256 A rows
// are taken unit-major, gate-minor (LDS row 4 u + gate), so an MFMA D fragment (16 rows x 16 trajectories;
// lane = trajectory lane & 15, rows 4 (lane >> 4) .. +3) holds the four gates i, f, g, o of ONE unit of ONE
// trajectory: the cell update runs on the accumulators, and the 4H x B gate matrix never goes to HBM.
//
// Tile walk: 8 waves (2 x 4), each 128 rows (32 units) x 32 trajectories = 8 x 2 D tiles; K in steps of 64
// (two 16x16x32 f16 k-blocks), A and XB chunks staged global -> registers -> LDS, double-buffered, one
// barrier per step. LDS rows are 128 B; their 16-B chunks are XOR-swizzled by (row & 7), so the 16 rows
// one ds_read_b128 touches land on distinct banks.
#pragma once
#include "fcr_common.h"
#include "fcr_f16.h"

namespace fcr {

constexpr int kWgU = 64;                  // units per workgroup
constexpr int kWgM = 4 * kWgU;            // A rows per workgroup
constexpr int kWgN = 128;                 // trajectories per workgroup
constexpr int kWgK = 64;                  // K per step
constexpr int kWgThreads = 512;
constexpr int kWgStageA = kWgM * kWgK * 2;   // bytes
constexpr int kWgStageB = kWgN * kWgK * 2;
constexpr int kWgLds = 2 * (kWgStageA + kWgStageB);

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

// byte offset of 16-B chunk c (0..7) of LDS row r in a stage
__device__ __forceinline__ uint32_t wg_off(int r, int c) { return (uint32_t)(r * 128 + ((c ^ (r & 7)) << 4)); }

__global__ __launch_bounds__(kWgThreads, 2) void wide_gemm_cell_kernel(WgArgs a) {
    extern __shared__ __attribute__((aligned(16))) char lds[];
    const int tid = threadIdx.x, lane = tid & 63;
    const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wr = wv >> 2, wc = wv & 3;               // wave's 128-row half, 32-trajectory quarter
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

    // global -> register chunk assignment: A 256 rows x 8 chunks (4 per thread), XB 128 rows x 8 chunks (2)
    typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
    const int cch = tid & 7;
    const _Float16 *gA[4];
    uint32_t oA[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int r = (tid >> 3) + 64 * i;            // LDS row = 4 * unit + gate
        const int grow = (r & 3) * H + u0 + (r >> 2);  // torch row gate * H + unit
        gA[i] = a.A + (size_t)grow * a.lda + cch * 8;
        oA[i] = wg_off(r, cch);
    }
    const _Float16 *gB[2];
    uint32_t oB[2];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
        const int r = (tid >> 3) + 64 * i;
        int b = b0 + r;
        if (b >= a.B) b = a.B - 1;                     // tail rows recompute the last trajectory (not stored)
        gB[i] = a.XB + (size_t)b * a.ldb + cch * 8;
        oB[i] = (uint32_t)kWgStageA + wg_off(r, cch);
    }
    u32x4 ra[4], rb[2];
    auto gload = [&](int ks) {
#pragma unroll
        for (int i = 0; i < 4; ++i) ra[i] = *reinterpret_cast<const u32x4 *>(gA[i] + ks * kWgK);
#pragma unroll
        for (int i = 0; i < 2; ++i) rb[i] = *reinterpret_cast<const u32x4 *>(gB[i] + ks * kWgK);
    };
    auto lstore = [&](int buf) {
        char *base = lds + buf * (kWgStageA + kWgStageB);
#pragma unroll
        for (int i = 0; i < 4; ++i) *reinterpret_cast<u32x4 *>(base + oA[i]) = ra[i];
#pragma unroll
        for (int i = 0; i < 2; ++i) *reinterpret_cast<u32x4 *>(base + oB[i]) = rb[i];
    };

    f32x4 acc[8][2];
#pragma unroll
    for (int m = 0; m < 8; ++m) acc[m][0] = acc[m][1] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};

    // fragment reads: A tile m rows 128 wr + 16 m + (lane & 15), k chunk 4 kb + (lane >> 4); B likewise
    const int fr = lane & 15, fq = lane >> 4;
    gload(0);
    lstore(0);
    __syncthreads();
    for (int ks = 0; ks < nk; ++ks) {
        const int buf = ks & 1;
        if (ks + 1 < nk) gload(ks + 1);
        const char *base = lds + buf * (kWgStageA + kWgStageB);
#pragma unroll
        for (int kb = 0; kb < 2; ++kb) {
            f16x8 bf[2];
#pragma unroll
            for (int n = 0; n < 2; ++n) {
                const int r = 32 * wc + 16 * n + fr;
                bf[n] = *reinterpret_cast<const f16x8 *>(base + kWgStageA + wg_off(r, 4 * kb + fq));
            }
#pragma unroll
            for (int m = 0; m < 8; ++m) {
                const int r = 128 * wr + 16 * m + fr;
                const f16x8 af = *reinterpret_cast<const f16x8 *>(base + wg_off(r, 4 * kb + fq));
                acc[m][0] = mfma16(af, bf[0], acc[m][0]);
                acc[m][1] = mfma16(af, bf[1], acc[m][1]);
            }
        }
        if (ks + 1 < nk) lstore(buf ^ 1);
        __syncthreads();
    }

    // ---- epilogue: the cell update (wide_cell_kernel's arithmetic) on the accumulators ----
#pragma unroll
    for (int n = 0; n < 2; ++n) {
        const int b = b0 + 32 * wc + 16 * n + fr;
        if (b >= a.B) continue;
#pragma unroll
        for (int m = 0; m < 8; ++m) {
            const int u = u0 + 32 * wr + 4 * m + fq;
            const f32x4 g4 = acc[m][n];
            const size_t idx = (size_t)b * H + u;
            const float cp = a.c_prev ? a.c_prev[idx] : 0.0f;
            const float i = sigm(g4[0]), f = sigm(g4[1]), g = tanhf(g4[2]), o = sigm(g4[3]);
            const float c = (a.c_prev ? f * cp : 0.0f) + i * g;
            const float h = o * tanhf(c);
            const _Float16 hi = (_Float16)h;
            const _Float16 lo = (_Float16)(h - (float)hi);
            a.c_out[idx] = c;
            if (a.h_out) a.h_out[idx] = h;
            if (a.xb_h) {
                _Float16 *p = a.xb_h + (size_t)b * a.sh + u;
                p[0] = hi;
                p[H] = lo;
                p[2 * H] = hi;
            }
            if (a.xb_x) {
                _Float16 *p = a.xb_x + (size_t)b * a.sx + u;
                p[0] = hi;
                p[H] = lo;
                p[2 * H] = hi;
            }
            if (a.preact) {
                float *p = a.preact + (size_t)b * 4 * H + u;
                p[0] = g4[0];
                p[H] = g4[1];
                p[2 * H] = g4[2];
                p[3 * H] = g4[3];
            }
        }
    }
}

}  // namespace fcr
