// fcr_wide.h — device kernels of the rollout for hidden sizes above the LDS-resident tiers (H > 52;
// H = 256, N = 25). There a layer's weights (4H x (in+H) fp32, 2 MB at H = 256)
// no longer fit in LDS next to anything else, and one cell of one trajectory is a 1 MFLOP GEMV, so the
// cell product is done batch-wide as a plain fp32 GEMM on rocBLAS (M = B trajectories) and everything
// around it — cell update, window build, controller, readout, costs, their backward — is hand-written
// here, one thread per (trajectory, unit) or per trajectory, batch-major so every access is coalesced.
//
// Data (fcr_abi.hip, wide layout), all row-major with the batch index outermost inside a slice:
//   X0  [10][B][5]        layer-0 input rows of the current window (Functions.py:1395-1396, 1433-1434)
//   Hs, Cs [3][10][B][H]  h_t, c_t of every cell of the current window
//   Act [3][10][B][4H]    gate activations (i, f, g, o) of the window, kept by the backward's recompute
//   G   [B][4H]           gate pre-activations (forward) / d loss / d pre-activations (backward)
//   rowg [N+9][B][5]      d loss / d (extended window row r): every window's layer-0 input gradient
//                         lands in rows j..j+9 — the row-gradient bookkeeping of fcr_bwd.h, batch-wide
// The backward keeps nothing from the forward but xhat and the predictions: it recomputes each
// window's cells (a checkpoint per window) before running that window's reverse pass.
#pragma once
#include "fcr_common.h"

namespace fcr {

struct WideArgs {
    int B, N, H, CH;
    float alpha;
    const float *X, *u0, *states, *noise;
    const float *fcw, *fcb, *cwi, *cbi, *cwo;
    float *xhat, *pred, *tot, *cmd, *err;
    float *X0, *Hs, *Cs, *Act, *G, *dH, *dC, *rowg, *dv;
    const float *dloss;
    _Float16 *xb0;   // split-f16 rollout: layer-0 operand rows (slot stride B 6H, row stride xb0_ld), else null
    const float *wsc;   // window-column scales of the split's range guard (fcr_pack.h)
};

// layer 0's K = 5 window-row input as the last kX16 columns of its split-f16 operand rows and weights:
// [x_hi (5) | x_lo (5) | x_hi (5) | 0] against [Wih_hi | Wih_hi | Wih_lo | 0]; 32 columns keep layer 0's K
// (3H + kX16, or kX16 at t = 0) a whole number of the fused cell kernel's K steps (fcr_wgemm.h)
constexpr int kX16 = 32;
static_assert(3 * kIn < kX16, "layer-0 input split exceeds its padded block");
// row stride of layer 0's operand rows [h part 3H | x part kX16], padded to whole 128-B lines (rows that
// straddle lines cost the GEMM's operand loads)
__host__ __device__ constexpr int xb0_ld(int H) { return (3 * H + kX16 + 63) / 64 * 64; }


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
        for (int col = 0; col < kIn; ++col) {
            x[col] = ext_row(a, b, j + t, col);
            a.X0[((size_t)t * a.B + b) * kIn + col] = x[col];
        }
        if (a.xb0) {
            _Float16 *p = a.xb0 + (size_t)t * a.B * 6 * a.H + (size_t)b * xb0_ld(a.H) + 3 * a.H;
            for (int col = 0; col < kIn; ++col) {
                const float v = x[col] * a.wsc[col];   // range guard (fcr_pack.h): v 2^-s_c against W_ih0 2^s_c
                const _Float16 hi = (_Float16)v;
                p[col] = hi;
                p[kIn + col] = (_Float16)(v - (float)hi);
                p[2 * kIn + col] = hi;
            }
            for (int k = 3 * kIn; k < kX16; ++k) p[k] = (_Float16)0.0f;
        }
    }
}

// Cell update from the gate pre-activations G [B][4H] (torch gate order i|f|g|o): c, h; and, for the
// backward's recompute, the activations. tanh is the library's (a few ulp RELATIVE to tanh): these
// memory-bound kernels can afford it, and the weight gradients of the surrogate step need it when the
// hidden states are small (1 - 2/(1 + e^{2x}) is only accurate to ~1e-7 absolute).
// xb_h / xb_x (split-f16 path, else null): the GEMM operand rows that take this h — the h part of the
// same layer's next cell and the x part of the layer above's cell t — as (hi, lo, hi), row strides sh / sx.
// V consecutive units per thread (V = 4 when H % 4 == 0: 16-B gate / state accesses, 8-B f16 stores —
// the kernel is HBM-bound and the wide accesses are what it runs at; V = 2 for even H, else 1).
template <int V>
struct WideVec {
    typedef float F __attribute__((ext_vector_type(V)));
    typedef _Float16 h __attribute__((ext_vector_type(V)));
    static __device__ __forceinline__ F ld(const float *p) { return *(const F *)p; }
    static __device__ __forceinline__ void st(float *p, F v) { *(F *)p = v; }
    static __device__ __forceinline__ void st16(_Float16 *p, h v) { *(h *)p = v; }
};

template <int V>
__global__ void wide_cell_kernel(const float *__restrict__ G, const float *__restrict__ c_prev, float *c_out,
                                 float *h_out, float *act, _Float16 *xb_h, int sh, _Float16 *xb_x, int sx, int B,
                                 int H) {
    using W = WideVec<V>;
    const int HV = H / V;
    const size_t iv = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (iv >= (size_t)B * HV) return;
    const size_t b = iv / HV, u = (iv % HV) * V, idx = b * H + u;
    const float *g4 = G + b * 4 * H + u;
    const typename W::F gi = W::ld(g4), gf = W::ld(g4 + H), gg = W::ld(g4 + 2 * H), go = W::ld(g4 + 3 * H);
    typename W::F cp = {}, i, f, g, o, c, h;
    if (c_prev) cp = W::ld(c_prev + idx);
    typename W::h hi, lo;
#pragma unroll
    for (int k = 0; k < V; ++k) {
        i[k] = sigm(gi[k]);
        f[k] = sigm(gf[k]);
        g[k] = tanhf(gg[k]);
        o[k] = sigm(go[k]);
        c[k] = (c_prev ? f[k] * cp[k] : 0.0f) + i[k] * g[k];
        h[k] = o[k] * tanhf(c[k]);
        hi[k] = (_Float16)h[k];
        lo[k] = (_Float16)(h[k] - (float)hi[k]);
    }
    W::st(c_out + idx, c);
    if (h_out) W::st(h_out + idx, h);
    if (xb_h) {
        _Float16 *p = xb_h + b * sh + u;
        W::st16(p, hi);
        W::st16(p + H, lo);
        W::st16(p + 2 * H, hi);
    }
    if (xb_x) {
        _Float16 *p = xb_x + b * sx + u;
        W::st16(p, hi);
        W::st16(p + H, lo);
        W::st16(p + 2 * H, hi);
    }
    if (act) {
        float *a4 = act + b * 4 * H + u;
        W::st(a4, i);
        W::st(a4 + H, f);
        W::st(a4 + 2 * H, g);
        W::st(a4 + 3 * H, o);
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
// rmh (the fused backward, fcr_wbwd.h), or null: the row bound max_u |dH[b][u]| into rmh[b] (rmh[B + b] = 0: the
// second column block's slot)
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
            a.dH[(size_t)b * a.H + u] = v;
            m = fmaxf(m, fabsf(v));
        }
    if (!rmh) return;
#pragma unroll
    for (int s = kRoLanes / 2; s > 0; s >>= 1) m = fmaxf(m, __shfl_xor(m, s, kRoLanes));
    if (live && q == 0) {
        rmh[b] = m;
        rmh[a.B + b] = 0.0f;
    }
}

// Backward of one cell: from the activations, c_t, c_{t-1}, the incoming dh (carried dH + din from the
// layer above; see dh_scaled) and the carried dc: d loss / d (gate pre-activations) into dG, and dc_{t-1} into dC.
// act: the gate activations (i, f, g, o) kept by the recompute, or with PRE their pre-activations (the
// split-f16 rollout keeps the GEMM output per cell instead of writing a second 4H-wide array), from which
// the activations are rebuilt with the forward's arithmetic. dG (fp32) may be null when only dgsp is used.
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
// With PRE, c_t is recomputed from the pre-activations and c_{t-1} rather than loaded (round 3d: bit-identical,
// backward -2.4 % at config 5).
template <bool PRE, int V, int T = 1>
__global__ __launch_bounds__(256) void wide_cell_bwd_kernel(const float *__restrict__ act, const float *__restrict__ c,
                                     const float *__restrict__ c_prev, const float *__restrict__ dH,
                                     const float *__restrict__ din, float *dC, float *dG, _Float16 *dgsp,
                                     const float *__restrict__ consts, int dh_scaled, int ldh, int ldx, int B,
                                     int H, int dg3, const float *__restrict__ wih0 = nullptr, float *rowg = nullptr) {
    using W = WideVec<V>;
    // with consts (split-f16 rollout) din, and dH unless it is the head's, come from gemm16_bwd in the
    // scaled units of the dgates: back by 1/scale = consts[0], one fp32 product each
    const float c0 = consts ? consts[0] : 1.0f, mh = dh_scaled ? c0 : 1.0f;
    const int HV = H / V;
    // a thread owns V units of T consecutive trajectories (T > 1 only for layer 0's row gradient: its W_ih0
    // rows, 4 V kIn floats, are loaded once for the T trajectories instead of once per trajectory)
    const size_t iv = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (iv >= ((size_t)B + T - 1) / T * HV) return;
    const size_t bg = iv / HV, u = (iv % HV) * V;
    float wr[4][V * kIn];
    if (rowg) {
        static_assert(V * kIn % 4 == 0 || V == 1 || V == 2, "row block in 16-B pieces");
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            // V consecutive rows of kIn floats: V * kIn / 4 16-B loads (80 B at V = 4, 16-B aligned as u % 4 == 0)
            if constexpr (V == 4) {
                const f32x4 *w4 = reinterpret_cast<const f32x4 *>(wih0 + ((size_t)k * H + u) * kIn);
#pragma unroll
                for (int q = 0; q < V * kIn / 4; ++q) {
                    const f32x4 v = w4[q];
                    wr[k][4 * q] = v[0]; wr[k][4 * q + 1] = v[1]; wr[k][4 * q + 2] = v[2]; wr[k][4 * q + 3] = v[3];
                }
            } else {
#pragma unroll
                for (int q = 0; q < V * kIn; ++q) wr[k][q] = wih0[((size_t)k * H + u) * kIn + q];
            }
        }
    }
    for (int t = 0; t < T; ++t) {
        const size_t b = bg * T + t, idx = b * H + u;
        if (b >= (size_t)B) break;   // uniform over the trajectory's H / V threads
        const float *a4 = act + b * 4 * H + u;
        const typename W::F ai = W::ld(a4), af = W::ld(a4 + H), ag = W::ld(a4 + 2 * H), ao = W::ld(a4 + 3 * H);
        const typename W::F dhv = W::ld(dH + b * ldh + u), dcv = W::ld(dC + idx);
        typename W::F cp = {}, dn = {}, dg[4], dco, cv;
        if (c_prev) cp = W::ld(c_prev + idx);
        if (!PRE) cv = W::ld(c + idx);
        if (din) dn = W::ld(din + b * ldx + u);
#pragma unroll
        for (int k = 0; k < V; ++k) {
            const float i = PRE ? sigm(ai[k]) : ai[k], f = PRE ? sigm(af[k]) : af[k], g = PRE ? tanhf(ag[k]) : ag[k],
                        o = PRE ? sigm(ao[k]) : ao[k];
            // c_t rebuilt as the forward's cell formed it (fcr_wgemm.h epilogue: f c_{t-1} + i g) instead of read: 1 of the
            // ~14 KB a trajectory row moves through this HBM-bound kernel
            const float tc = tanhf(PRE ? (c_prev ? f * cp[k] : 0.0f) + i * g : cv[k]);
            const float dh = dhv[k] * mh + dn[k] * c0;
            const float dct = dcv[k] + dh * o * (1.0f - tc * tc);
            dg[0][k] = dct * g * i * (1.0f - i);
            dg[1][k] = dct * cp[k] * f * (1.0f - f);
            dg[2][k] = dct * i * (1.0f - g * g);
            dg[3][k] = dh * tc * o * (1.0f - o);
            dco[k] = dct * f;
        }
        if (dG) {
            float *d4 = dG + b * 4 * H + u;
#pragma unroll
            for (int k = 0; k < 4; ++k) W::st(d4 + k * H, dg[k]);
        }
        if (dgsp) {   // split-f16 operand row [hi | lo | hi] of W^T dG, scaled into the f16 range (wide_bscale_kernel)
            const float sc = consts[3];
            _Float16 *o16 = dgsp + b * 12 * H + u;
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                typename W::h hi, lo;
#pragma unroll
                for (int e = 0; e < V; ++e) {
                    const float v = dg[k][e] * sc;
                    hi[e] = (_Float16)v;
                    lo[e] = (_Float16)(v - (float)hi[e]);
                }
                W::st16(o16 + k * H, hi);
                W::st16(o16 + (4 + k) * H, lo);
                if (dg3) W::st16(o16 + (8 + k) * H, hi);
            }
        }
        W::st(dC + idx, dco);
        if (rowg) {   // layer 0: the window-row gradient sum_r dG[b][r] W_ih0[r][c] (c < kIn), fp32 from these
            // dgates, reduced over the trajectory's H / V threads (one aligned segment of a wave: the host checks
            // 64 % (H / V) == 0) — in place of kIn + 3 more columns in the backward product
            float pc[kIn] = {};
#pragma unroll
            for (int k = 0; k < 4; ++k)
#pragma unroll
                for (int e = 0; e < V; ++e)
#pragma unroll
                    for (int cc = 0; cc < kIn; ++cc) pc[cc] = fmaf(dg[k][e], wr[k][e * kIn + cc], pc[cc]);
            // (a DPP form of the first four butterfly levels measured within the noise, round 2g)
#pragma unroll
            for (int cc = 0; cc < kIn; ++cc)
                for (int o = 1; o < HV; o <<= 1) pc[cc] += __shfl_xor(pc[cc], o);
            if (u == 0)
#pragma unroll
                for (int cc = 0; cc < kIn; ++cc) rowg[b * kIn + cc] += pc[cc];
        }
    }
}

// Split-f16 operands of the config-5 gate GEMMs (fp32-accurate on the matrix cores, as fcr_f16.h does
// for the fused kernels): every product a.b becomes a_hi b_hi + a_hi b_lo + a_lo b_hi, laid out as ONE
// K-concatenated GEMM per cell so the fp32 gate matrix is written once (C traffic, not the MFMA, bounded
// the per-term calls). Forward A, row-major [4H][6H] = [Wih_hi | Wih_hi | Wih_lo | Whh_hi | Whh_hi | Whh_lo]
// against operand rows [x_hi | x_lo | x_hi | h_hi | h_lo | h_hi] (layer 0: [h part | x part of kX16 columns]);
// backward A (below) stacks [W_hi ; W_hi ; W_lo] (12H rows) against the dgate rows [dG_hi | dG_lo | dG_hi].
__global__ void wide_split_fa_kernel(const float *__restrict__ Wih, const float *__restrict__ Whh, int H, int layer0,
                                     const float *__restrict__ wsc, _Float16 *dst) {
    const int KA = layer0 ? 3 * H + kX16 : 6 * H;
    const size_t idx = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= (size_t)4 * H * KA) return;
    const int r = (int)(idx / KA), k = (int)(idx % KA);
    float v;
    int term;
    if (layer0) {
        if (k < 3 * H) {
            term = k / H;
            v = Whh[(size_t)r * H + k % H];
        } else {
            const int kk = k - 3 * H;
            if (kk >= 3 * kIn) {
                dst[idx] = (_Float16)0.0f;
                return;
            }
            term = kk / kIn;
            v = Wih[(size_t)r * kIn + kk % kIn] / wsc[kk % kIn];   // range guard (fcr_pack.h): exact
        }
    } else {
        const int part = k / (3 * H), kk = k % (3 * H), u = kk % H;
        term = kk / H;
        v = (part == 0 ? Wih : Whh)[(size_t)r * H + u];
    }
    const _Float16 hi = (_Float16)v;
    dst[idx] = term < 2 ? hi : (_Float16)(v - (float)hi);
}

// Layer 0's backward A, row-major [12H][H + 8]: per split row the W_hh row (H columns), then the W_ih row
// (kIn columns) and zero padding — ONE product gives dh_{t-1} and the window-row gradient of the cell.
__global__ void wide_split_bx0_kernel(const float *__restrict__ Wih, const float *__restrict__ Whh, int H,
                                      const float *__restrict__ wsc, _Float16 *dst) {
    const int ld = H + 8;
    const size_t idx = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= (size_t)12 * H * ld) return;
    const int r = (int)(idx / ld), col = (int)(idx % ld), term = r / (4 * H), g = r % (4 * H);
    float v = 0.0f;
    if (col < H) v = Whh[(size_t)g * H + col];
    else if (col < H + kIn) v = Wih[(size_t)g * kIn + col - H] / wsc[col - H];
    const _Float16 hi = (_Float16)v;
    dst[idx] = term < 2 ? hi : (_Float16)(v - (float)hi);
}
// Layers >= 1: backward A row-major [12H][2H], per split row [W_ih row | W_hh row] — ONE product gives the
// cell's input gradient (the layer below's incoming dh) and dh_{t-1}, side by side in rows of 2H.
__global__ void wide_split_bcat_kernel(const float *__restrict__ Wih, const float *__restrict__ Whh, int H,
                                       _Float16 *dst) {
    const size_t idx = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= (size_t)24 * H * H) return;
    const int r = (int)(idx / (2 * H)), col = (int)(idx % (2 * H)), term = r / (4 * H), g = r % (4 * H);
    const float v = col < H ? Wih[(size_t)g * H + col] : Whh[(size_t)g * H + col - H];
    const _Float16 hi = (_Float16)v;
    dst[idx] = term < 2 ? hi : (_Float16)(v - (float)hi);
}
// rowg row += the window-row gradient part of layer 0's backward product (scaled units, see dh_scaled; the
// range guard's column scale back, fcr_pack.h)
__global__ void wide_rowg_kernel(const float *__restrict__ E, int ldE, const float *__restrict__ consts,
                                 const float *__restrict__ wsc, float *rowg, int B) {
    const size_t idx = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= (size_t)B * kIn) return;
    const size_t b = idx / kIn, col = idx % kIn;
    rowg[idx] += consts[0] * E[b * ldE + col] * wsc[col];
}

// The dgates are split as dG * 2^k / dloss (|dG| ~ dloss / (B N): without it they would sit in the f16
// subnormals); the backward GEMMs' outputs stay in those units and wide_cell_bwd_kernel scales them back by
// consts[0] = dloss * 2^-k on load (no host sync for dloss). consts = [1/scale, 0, 1, scale].
__global__ void wide_bscale_kernel(const float *__restrict__ dloss, int k, float *consts) {
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    // dloss = 0: every gradient is 0 (no 0 * inf). A non-finite dloss must come out non-finite (as torch's
    // would, for GradScaler / anomaly detection): the NaN scale turns every dgate operand into NaN.
    const float d = dloss[0];
    consts[0] = d != 0.0f ? ldexpf(d, -k) : 0.0f;
    consts[1] = 0.0f;
    consts[2] = 1.0f;
    consts[3] = !isfinite(d) ? __builtin_nanf("") : d != 0.0f ? ldexpf(1.0f, k) / d : 0.0f;
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
