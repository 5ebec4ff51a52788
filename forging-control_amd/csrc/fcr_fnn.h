// fcr_fnn.h — the caller's controller call `output = model(X)` (Functions.py:643) on gfx950:
// FNNModel.forward (Functions.py:261-289) at the reference's shape, Linear(3 -> hidden) + ReLU,
// Linear(hidden -> 1, no bias) + Hardtanh (UL/Main.py:188), and its autograd backward.
//
// Torch ran this as rocBLAS GEMMs whose backward reduces over the whole batch on a handful of
// workgroups (~0.33 ms per B = 65 536 step, 3 % of the training step). Here: one lane per sample for
// the forward; the backward recomputes the forward per sample (dpre = g·1[-1 < pre < 1]), stages
// (x, dpre) in LDS and turns the lanes into hidden units for the parameter sums (the ctrl_grad_kernel
// pattern, fcr_pack.h), then grad_reduce_kernel sums the per-block partials in a fixed order.
#pragma once
#include "fcr_common.h"
#include "fcr_pack.h"

namespace fcr {
namespace fnn {

constexpr int kFnnBlock = 256;
constexpr int kFnnMaxHidden = 64;   // one wave's lanes are the hidden units in the backward
constexpr int kFnnItems = 256;      // samples per backward block

// params -> LDS records [k][W0 W1 W2 b wout]
__device__ __forceinline__ void load_params(float (*sp)[5], int hidden, const float *W, const float *bi,
                                            const float *wo) {
    for (int i = threadIdx.x; i < hidden * 5; i += blockDim.x) {
        const int k = i / 5, p = i % 5;
        sp[k][p] = p < 3 ? W[k * kCtrlIn + p] : (p == 3 ? bi[k] : wo[k]);
    }
}

// pre-Hardtanh output of one sample (z_k = W_k·x + b_k; pre = Σ_k wout_k relu(z_k))
__device__ __forceinline__ float fnn_sample(const float (*sp)[5], int hidden, float x0, float x1, float x2) {
    float acc = 0.0f;
    for (int k = 0; k < hidden; ++k) {
        const float z = fmaf(sp[k][2], x2, fmaf(sp[k][1], x1, sp[k][0] * x0)) + sp[k][3];
        acc = fmaf(sp[k][4], relu(z), acc);
    }
    return acc;
}

__global__ __launch_bounds__(kFnnBlock) void fnn_fwd_kernel(int B, int hidden, const float *__restrict__ X,
                                                            const float *W, const float *bi, const float *wo,
                                                            float *__restrict__ u) {
    __shared__ float sp[kFnnMaxHidden][5];
    load_params(sp, hidden, W, bi, wo);
    __syncthreads();
    const int b = blockIdx.x * kFnnBlock + threadIdx.x;
    if (b >= B) return;
    const float *x = X + (size_t)b * kCtrlIn;
    u[b] = hardtanh(fnn_sample(sp, hidden, x[0], x[1], x[2]));   // Functions.py:287
}

// Per-block partial sums [block][k][dW0 dW1 dW2 db dwout] of the parameter gradients, and g_X
// (optional) = Σ_k dz_k W_k. Hardtanh'(pre) = 1 on (-1, 1), 0 elsewhere; ReLU'(0) = 0 (torch).
__global__ __launch_bounds__(kFnnBlock) void fnn_bwd_kernel(int B, int hidden, const float *__restrict__ X,
                                                            const float *W, const float *bi, const float *wo,
                                                            const float *__restrict__ g, float *__restrict__ gX,
                                                            float *__restrict__ part, float *gwi = nullptr,
                                                            float *gbi = nullptr, float *gwo = nullptr) {
    __shared__ float sp[kFnnMaxHidden][5];
    __shared__ float sx[3][kFnnItems], sd[kFnnItems];
    __shared__ float red[kFnnBlock / kWave][kFnnMaxHidden][5];
    load_params(sp, hidden, W, bi, wo);
    __syncthreads();
    const int i0 = blockIdx.x * kFnnItems;
    const int n = B - i0 < kFnnItems ? B - i0 : kFnnItems;
    for (int i = threadIdx.x; i < n; i += kFnnBlock) {
        const float *x = X + (size_t)(i0 + i) * kCtrlIn;
        const float x0 = x[0], x1 = x[1], x2 = x[2];
        const float pre = fnn_sample(sp, hidden, x0, x1, x2);
        const float d = (pre > -1.0f && pre < 1.0f) ? g[i0 + i] : 0.0f;
        sx[0][i] = x0;
        sx[1][i] = x1;
        sx[2][i] = x2;
        sd[i] = d;
        if (gX) {
            float g0 = 0.0f, g1 = 0.0f, g2 = 0.0f;
            for (int k = 0; k < hidden; ++k) {
                const float z = fmaf(sp[k][2], x2, fmaf(sp[k][1], x1, sp[k][0] * x0)) + sp[k][3];
                const float dz = z > 0.0f ? d * sp[k][4] : 0.0f;
                g0 = fmaf(dz, sp[k][0], g0);
                g1 = fmaf(dz, sp[k][1], g1);
                g2 = fmaf(dz, sp[k][2], g2);
            }
            float *o = gX + (size_t)(i0 + i) * kCtrlIn;
            o[0] = g0;
            o[1] = g1;
            o[2] = g2;
        }
    }
    __syncthreads();
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int k = lane < hidden ? lane : 0;
    const float W0 = sp[k][0], W1 = sp[k][1], W2 = sp[k][2], bk = sp[k][3], wk = sp[k][4];
    float a0 = 0.0f, a1 = 0.0f, a2 = 0.0f, a3 = 0.0f, a4 = 0.0f;
    for (int i = w; i < n; i += kFnnBlock / kWave) {
        const float x0 = sx[0][i], x1 = sx[1][i], x2 = sx[2][i], d = sd[i];
        const float z = fmaf(W2, x2, fmaf(W1, x1, W0 * x0)) + bk;
        const float dz = z > 0.0f ? d * wk : 0.0f;
        a0 = fmaf(dz, x0, a0);
        a1 = fmaf(dz, x1, a1);
        a2 = fmaf(dz, x2, a2);
        a3 += dz;
        a4 = fmaf(d, relu(z), a4);
    }
    red[w][lane][0] = a0;
    red[w][lane][1] = a1;
    red[w][lane][2] = a2;
    red[w][lane][3] = a3;
    red[w][lane][4] = a4;
    __syncthreads();
    if (w == 0 && lane < hidden) {
#pragma unroll
        for (int p = 0; p < 5; ++p) {
            float s = 0.0f;
#pragma unroll
            for (int ww = 0; ww < kFnnBlock / kWave; ++ww) s += red[ww][lane][p];
            grad_out5(part, hidden, lane, p, s, gwi, gbi, gwo);
        }
    }
}

}  // namespace fnn
}  // namespace fcr
