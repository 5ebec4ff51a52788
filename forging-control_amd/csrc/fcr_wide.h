// fcr_wide.h — device kernels of the rollout for hidden sizes above the LDS-resident tiers (H > 52;
// H = 256, N = 25). There a layer's weights (4H x (in+H) fp32, 2 MB at H = 256)
// no longer fit in LDS next to anything else, and one cell of one trajectory is a 1 MFLOP GEMV, so each cell
// runs batch-wide: the gate GEMM with the cell update in its epilogue (fcr_wgemm.h), the backward cell as one fused
// kernel (fcr_wbwd.h); everything around them — window rows, controller, readout, costs, their backward — is here,
// one thread per trajectory (or a few lanes per trajectory), batch-major so every access is coalesced. All of it runs
// at Hp, H padded to whole 64-unit blocks with zero-weight units (fcr_abi.hip wide_hp).
//
// Data (fcr_abi.hip WideLayout), row-major with the batch index outermost inside a slice:
//   WR  [10][B][64] halves   layer-0 window records [hi | lo] of the current window (Functions.py:1395-1396, 1433-1434)
//   HR  [2][10][B][2Hp]      h records [hi | lo] of two layers' cells (layer l in slot l & 1)
//   Cs  [3][10][Hp/8][B][8]  c_t of every cell of the current window (k8 rows, below)
//   Act [3][10][B][Hp][4]    gate activations i, f, g, o of every cell (the backward's dgates read them)
//   rowg [N+9][B][5]         d loss / d (extended window row r): every window's layer-0 input gradient
//                            lands in rows j..j+9 — the row-gradient bookkeeping of fcr_bwd.h, batch-wide
// The backward keeps nothing from the forward but xhat, the predictions and the kept windows: it recomputes each
// other window's cells (a checkpoint per window) before running that window's reverse pass.
#pragma once
#include "fcr_common.h"

namespace fcr {

struct WideArgs {
    int B, N, H, CH;
    float alpha;
    const float *X, *u0, *states, *noise;
    const float *fcw, *fcb, *cwi, *cbi, *cwo;
    float *xhat, *pred, *tot, *cmd, *err;
    float *Hs, *Cs, *Act, *dH, *dC, *rowg, *dv;
    const float *dloss;
    _Float16 *wr;    // split-f16 rollout: layer 0's window records [10][B][2 kWgRecX0] (hi | lo), else null
    const float *wsc;   // window-column scales of the split's range guard (fcr_pack.h)
};

// "k8" rows of the fp32 per-unit arrays the backward cells stream K step by K step — c, dh, the input gradients, dc
// (fcr_wbwd.h): element (b, u) of a B x n array at ((u >> 3) B + b) 8 + (u & 7), i.e. [n / 8][B][8]. A K step's 8
// units of consecutive trajectories are contiguous, so the 32 B one trajectory needs per step share a 128-B line with
// three neighbours' instead of with its own next three steps' (which L1 does not keep that long).
__host__ __device__ __forceinline__ size_t k8(int B, int b, int u) { return ((size_t)(u >> 3) * B + b) * 8 + (u & 7); }

// layer 0's window record (the x part of its cell products, fcr_wgemm.h): [hi (32) | lo (32)] halves per
// trajectory and row, the 5 window columns first, zero after
constexpr int kWideRecX0 = 32;
static_assert(kIn <= kWideRecX0, "window columns exceed their record block");

// controller (FNNModel.forward, Functions.py:261-289) pre-Hardtanh output, and its ReLU inputs' signs
__device__ __forceinline__ float wide_fnn(const WideArgs &a, float x0, float x3, float ref) {
    float v = 0.0f;
    for (int k = 0; k < a.CH; ++k) {
        const float z = a.cwi[k * kCtrlIn + 0] * x0 + a.cwi[k * kCtrlIn + 1] * x3 + a.cwi[k * kCtrlIn + 2] * ref + a.cbi[k];
        v += a.cwo[k] * relu(z);
    }
    return v;
}

// extended window row r of trajectory b: rows 0..9 = states (row 9 col 4 = u0), row 10+m = (xhat_m, u_{m+1})
__device__ __forceinline__ float ext_row(const WideArgs &a, int b, int r, int col) {
    if (r < kL) {
        if (r == kL - 1 && col == kIn - 1) return a.pred[(size_t)b * a.N];   // u_0 (prediction[:, 0])
        return a.states[((size_t)b * kL + r) * kIn + col];
    }
    const int m = r - kL;
    return col < kOut ? a.xhat[((size_t)b * a.N + m) * kOut + col] : a.pred[(size_t)b * a.N + m + 1];
}

// Window j of the forward: the controller call that produces u_j (j > 0, Functions.py:1421-1430), the
// command cost (:1405, :1446), and the window's layer-0 input rows. CTRL = false: rows only (recompute).
template <bool CTRL>
__global__ void wide_window_kernel(WideArgs a, int j) {
    const int b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= a.B) return;
    if (CTRL) {
        const float ref = a.X[(size_t)b * kCtrlIn + 2];
        float u, cmd;
        if (j == 0) {
            u = a.u0[b];
            cmd = a.alpha * sq(a.states[((size_t)b * kL + kL - 2) * kIn + kIn - 1] - u);
            a.tot[b] = cmd;
            a.cmd[b] = cmd;
            a.err[b] = 0.0f;
        } else {
            const float *xh = a.xhat + ((size_t)b * a.N + j - 1) * kOut;
            u = hardtanh(wide_fnn(a, xh[0], xh[3], ref));
            cmd = a.alpha * sq(a.pred[(size_t)b * a.N + j - 1] - u);
            a.tot[b] += cmd;
            a.cmd[b] += cmd;
        }
        a.pred[(size_t)b * a.N + j] = u;
    }
    for (int t = 0; t < kL; ++t) {
        float x[kIn];
        for (int col = 0; col < kIn; ++col) x[col] = ext_row(a, b, j + t, col);
        if (a.wr) {
            typedef _Float16 h8 __attribute__((ext_vector_type(8)));
            h8 hi = {}, lo = {};
#pragma unroll
            for (int col = 0; col < kIn; ++col) {
                const float v = x[col] * a.wsc[col];   // range guard (fcr_pack.h): v 2^-s_c against W_ih0 2^s_c
                hi[col] = (_Float16)v;
                lo[col] = (_Float16)(v - (float)hi[col]);
            }
            h8 *p = reinterpret_cast<h8 *>(a.wr + ((size_t)t * a.B + b) * 2 * kWideRecX0);
            const h8 z = {};
#pragma unroll
            for (int k = 0; k < kWideRecX0 / 8; ++k) {
                p[k] = k == 0 ? hi : z;
                p[kWideRecX0 / 8 + k] = k == 0 ? lo : z;
            }
        }
    }
}

// Readout fc(h_9 of layer 2) (Functions.py:377), noise (:1400-1402), and the step's error and
// constraint costs (:1405-1414, :1443-1452).
// kRoLanes lanes per trajectory: each lane reads a strided slice of the trajectory's h row (the group's
// loads of one row are contiguous: coalesced), partial dot products reduced across the group by shuffles.
constexpr int kRoLanes = 16;
__global__ void wide_readout_kernel(WideArgs a, int j, const float *__restrict__ h) {
    const size_t gid = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int b = (int)(gid / kRoLanes), q = (int)(gid % kRoLanes);
    const bool live = b < a.B;
    float xo[kOut];
    for (int o = 0; o < kOut; ++o) {
        float s = 0.0f;
        if (live)
            for (int u = q; u < a.H; u += kRoLanes) s += a.fcw[o * a.H + u] * h[(size_t)b * a.H + u];
#pragma unroll
        for (int m = kRoLanes / 2; m > 0; m >>= 1) s += __shfl_xor(s, m, kRoLanes);
        xo[o] = s;
    }
    if (!live || q != 0) return;
    for (int o = 0; o < kOut; ++o) {
        xo[o] += a.fcb[o] + (a.noise ? a.noise[((size_t)b * a.N + j) * kOut + o] : 0.0f);
        a.xhat[((size_t)b * a.N + j) * kOut + o] = xo[o];
    }
    const float ref = a.X[(size_t)b * kCtrlIn + 2];
    const float err = sq(xo[0] - ref);
    const float con = relu(-xo[1]) + relu(-xo[2]) + relu(xo[1] - kP1Max) + relu(xo[2] - kP2Max);
    a.tot[b] += err + con;
    a.err[b] += err;
}

// per-trajectory outputs (Functions.py:1458-1460)
__global__ void wide_finish_kernel(WideArgs a, float *cost, float *command, float *error, float *xhat_user) {
    const int b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= a.B) return;
    cost[b] = a.tot[b] / (float)a.N;
    command[b] = a.cmd[b] / (float)a.N;
    error[b] = a.err[b] / (float)a.N;
    if (xhat_user)
        for (int k = 0; k < a.N * kOut; ++k) xhat_user[(size_t)b * a.N * kOut + k] = a.xhat[(size_t)b * a.N * kOut + k];
}

// Backward head of window j: d loss / d xhat_j from the step costs and from every later window that
// read row 10+j (rowg), the controller's backward at (xhat_j[0], xhat_j[3], ref) (stores dv for the
// parameter gradients), and dh_9 of layer 2 = fc.Wᵀ dxhat_j into dH. Same algebra as fcr_bwd.h.
// kRoLanes lanes per trajectory: the group's first lane runs the scalar algebra, all of them write dH.
__device__ __forceinline__ void wide_head_dxhat(const WideArgs &a, int j, int b, float (&d)[kOut]) {
    const int N = a.N;
    const float wgt = a.dloss[0] / ((float)a.B * (float)N);
    const float ref = a.X[(size_t)b * kCtrlIn + 2];
    const float *xh = a.xhat + ((size_t)b * N + j) * kOut;
    float d0 = wgt * 2.0f * (xh[0] - ref);
    float d1 = wgt * ((-xh[1] > 0.0f ? -1.0f : 0.0f) + (xh[1] - kP1Max > 0.0f ? 1.0f : 0.0f));
    float d2 = wgt * ((-xh[2] > 0.0f ? -1.0f : 0.0f) + (xh[2] - kP2Max > 0.0f ? 1.0f : 0.0f));
    float d3 = 0.0f;
    if (j <= N - 2) {
        const float *G = a.rowg + ((size_t)(kL + j) * a.B + b) * kIn;
        d0 += G[0];
        d1 += G[1];
        d2 += G[2];
        d3 += G[3];
        const float *pr = a.pred + (size_t)b * N;
        float du = 2.0f * a.alpha * wgt * (pr[j + 1] - pr[j]);
        if (j + 2 < N) du += 2.0f * a.alpha * wgt * (pr[j + 1] - pr[j + 2]);
        du += G[4];
        const float v = wide_fnn(a, xh[0], xh[3], ref);
        const float dv = (v > -1.0f && v < 1.0f) ? du : 0.0f;
        float dca = 0.0f, dcb = 0.0f;
        for (int k = 0; k < a.CH; ++k) {
            const float z = a.cwi[k * kCtrlIn + 0] * xh[0] + a.cwi[k * kCtrlIn + 1] * xh[3] + a.cwi[k * kCtrlIn + 2] * ref + a.cbi[k];
            const float dz = z > 0.0f ? dv * a.cwo[k] : 0.0f;
            dca += dz * a.cwi[k * kCtrlIn + 0];
            dcb += dz * a.cwi[k * kCtrlIn + 1];
        }
        a.dv[(size_t)b * N + j] = dv;
        d0 += dca;
        d3 += dcb;
    } else {
        a.dv[(size_t)b * N + j] = 0.0f;
    }
    d[0] = d0;
    d[1] = d1;
    d[2] = d2;
    d[3] = d3;
}
// rmh (the fused backward, fcr_wbwd.h), or null: the row bound max_u |dH[b][u]| into rmh[b]
__global__ void wide_head_kernel(WideArgs a, int j, float *rmh) {
    const size_t gid = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int b = (int)(gid / kRoLanes), q = (int)(gid % kRoLanes);
    const bool live = b < a.B;
    float d[kOut] = {0.0f, 0.0f, 0.0f, 0.0f};
    if (live && q == 0) wide_head_dxhat(a, j, b, d);
#pragma unroll
    for (int k = 0; k < kOut; ++k) d[k] = __shfl(d[k], 0, kRoLanes);
    float m = 0.0f;
    if (live)
        for (int u = q; u < a.H; u += kRoLanes) {
            const float v = a.fcw[u] * d[0] + a.fcw[a.H + u] * d[1] + a.fcw[2 * a.H + u] * d[2] + a.fcw[3 * a.H + u] * d[3];
            a.dH[k8(a.B, b, u)] = v;
            m = fmaxf(m, fabsf(v));
        }
    if (!rmh) return;
#pragma unroll
    for (int s = kRoLanes / 2; s > 0; s >>= 1) m = fmaxf(m, __shfl_xor(m, s, kRoLanes));
    if (live && q == 0) rmh[b] = m;   // slot 0: the layer-2 cell at t = 9 reads one slot (WbArgs.nrh = 1)
}

// The per-row dgate scale of the fused backward cell (fcr_wbwd.h) is 2^(kWideDgExp - e), e the exponent of a bound m on
// the row's |dc_t| (m >= |dc| + |dh|): the i, g, o rows are |dc_t| or |dh| times a local derivative <= 1, so below
// 2^kWideDgExp scaled; the forget row is dc_t c_{t-1} f (1 - f) with |c_{t-1}| <= t <= kL - 1 (|c_t| <= |c_{t-1}| + 1
// from c = 0), so it reaches (kL - 1) / 4 * 2^kWideDgExp (18 432 at kL = 10): a finite f16, with that margin only.
// |c_{t-1}| <= t holds because EVERY window's LSTM starts from h = c = 0 (Functions.py:349-350): the rollout never
// carries a state into a window, and no ABI entry takes an initial c; a path that did would need its own bound here.
// The bound is formed with fmaxf, which drops a NaN row maximum: the NaN dgates themselves still propagate into the
// products, so a non-finite gradient stays non-finite (tests/test_gpu_parity.py
// test_wide_forget_dgates_near_their_f16_margin drives the forget row to 2 of the 9/4 this allows).
constexpr int kWideDgExp = 13;
static_assert((kL - 1) * (1 << kWideDgExp) / 4 < 65504, "f16 overflow of the forget-gate dgates: lower kWideDgExp");

// fc.W [4][H] -> [4][Hp] with zero padding units: the rollout's readout and head run at the padded size
__global__ void wide_pad_fc_kernel(const float *__restrict__ fcw, int H, int Hp, float *__restrict__ dst) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= kOut * Hp) return;
    const int o = i / Hp, u = i % Hp;
    dst[i] = u < H ? fcw[(size_t)o * H + u] : 0.0f;
}

// d loss / d u0 (Functions.py:1396 row 9 col 4, and the command costs cmd_0, cmd_1)
__global__ void wide_gu0_kernel(WideArgs a, float *g_u0) {
    const int b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= a.B) return;
    const float wgt = a.dloss[0] / ((float)a.B * (float)a.N);
    const float *pr = a.pred + (size_t)b * a.N;
    const float s84 = a.states[((size_t)b * kL + kL - 2) * kIn + kIn - 1];
    float du0 = 2.0f * a.alpha * wgt * (pr[0] - s84);
    if (a.N > 1) du0 += 2.0f * a.alpha * wgt * (pr[0] - pr[1]);
    g_u0[b] = a.rowg[((size_t)(kL - 1) * a.B + b) * kIn + kIn - 1] + du0;
}

}  // namespace fcr
