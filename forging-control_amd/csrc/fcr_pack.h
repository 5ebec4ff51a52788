// fcr_pack.h — small-parameter packing (controller, readout) and fixed-order reductions. The LSTM
// weights are packed by pack_fwd16_kernel (fcr_f16.h) and pack_img_kernel (fcr_img.h).
#pragma once
#include "fcr_common.h"

namespace fcr {

struct PackArgs {
    int H, HS, CH;
    const float *wih[3], *whh[3], *fcw, *fcb, *cwi, *cbi, *cwo;
    float *fcp, *fcbo, *fnp;
};

__global__ void pack_misc_kernel(PackArgs a) {
    const int idx = blockIdx.x * blockDim.x + threadIdx.x;
    const int H = a.H, HS = a.HS;
    const int nfc = kOut * HS * 4;
    if (idx < nfc) {
        const int q = idx & 3, r = (idx >> 2) % HS, o = (idx >> 2) / HS;
        const int u = 4 * r + q;
        a.fcp[idx] = u < H ? a.fcw[o * H + u] : 0.0f;
    }
    if (idx < kOut) a.fcbo[idx] = a.fcb[idx];
    const int nf = kMS * 4 * kFnpStride;
    if (idx < nf) {
        const int p = idx % kFnpStride, q = (idx / kFnpStride) & 3, m = idx / (kFnpStride * 4);
        const int k = 4 * m + q;
        float v = 0.0f;
        if (k < a.CH) {
            if (p < 3) v = a.cwi[k * kCtrlIn + p];
            else if (p == 3) v = a.cbi[k];
            else if (p == 4) v = a.cwo[k];
        }
        a.fnp[idx] = v;
    }
}

// loss = sum(loss_part[0..nw)) / B, fixed order (one block)
__global__ void loss_reduce_kernel(const float *part, int nw, int B, float *loss) {
    __shared__ float red[256];
    float s = 0.0f;
    for (int i = threadIdx.x; i < nw; i += blockDim.x) s += part[i];
    red[threadIdx.x] = s;
    __syncthreads();
    for (int w = 128; w > 0; w >>= 1) {
        if ((int)threadIdx.x < w) red[threadIdx.x] += red[threadIdx.x + w];
        __syncthreads();
    }
    if (threadIdx.x == 0) loss[0] = red[0] / (float)B;
}

// Controller parameter gradients (the in-loss controller calls, Functions.py:1424-1430), from the dv
// the backward kernel stored per (trajectory, step): z = W_inp·[x0, x3, ref] + b is recomputed from
// the stored xhat with the same arithmetic as fnn_pre; dz = dv·w_out·1[z>0]. One block per chunk of
// (trajectory, step) items; a wave's lanes are the hidden units; fixed-order sums everywhere.
constexpr int kCtrlBlock = 256;
constexpr int kCtrlItems = 1024;   // items per block
__global__ __launch_bounds__(kCtrlBlock) void ctrl_grad_kernel(const float *X, const float *xhat, const float *dv,
                                                               const float *fnp, int B, int N, int hidden,
                                                               float *part) {
    __shared__ float sx0[kCtrlItems], sx3[kCtrlItems], sref[kCtrlItems], sdv[kCtrlItems];
    __shared__ float red[kCtrlBlock / kWave][64][5];
    const long long items = (long long)B * N;
    const long long i0 = (long long)blockIdx.x * kCtrlItems;
    const int n = (int)((items - i0) < kCtrlItems ? (items - i0) : kCtrlItems);
    for (int i = threadIdx.x; i < n; i += blockDim.x) {
        const long long it = i0 + i;
        const int bb = (int)(it / N);
        sx0[i] = xhat[it * kOut + 0];
        sx3[i] = xhat[it * kOut + 3];
        sref[i] = X[(size_t)bb * kCtrlIn + 2];
        sdv[i] = dv[it];
    }
    __syncthreads();
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int k = lane;   // hidden unit
    float W0 = 0.0f, W1 = 0.0f, W2 = 0.0f, bk = 0.0f, wo = 0.0f;
    if (k < hidden) {
        const float *p = fnp + ((k >> 2) * 4 + (k & 3)) * kFnpStride;
        W0 = p[0]; W1 = p[1]; W2 = p[2]; bk = p[3]; wo = p[4];
    }
    float g0 = 0.0f, g1 = 0.0f, g2 = 0.0f, g3 = 0.0f, g4 = 0.0f;
    for (int i = w; i < n; i += kCtrlBlock / kWave) {
        const float a = sx0[i], b3 = sx3[i], r = sref[i], d = sdv[i];
        const float z = W0 * a + W1 * b3 + W2 * r + bk;    // == fnn_pre's z
        const float dz = z > 0.0f ? d * wo : 0.0f;
        g0 += dz * a;
        g1 += dz * b3;
        g2 += dz * r;
        g3 += dz;
        g4 += d * (z > 0.0f ? z : 0.0f);
    }
    red[w][lane][0] = g0; red[w][lane][1] = g1; red[w][lane][2] = g2; red[w][lane][3] = g3; red[w][lane][4] = g4;
    __syncthreads();
    if (w == 0 && k < hidden) {
#pragma unroll
        for (int p = 0; p < 5; ++p) {
            float s = 0.0f;
#pragma unroll
            for (int ww = 0; ww < kCtrlBlock / kWave; ++ww) s += red[ww][lane][p];
            part[((size_t)blockIdx.x * hidden + k) * 5 + p] = s;
        }
    }
}

// grads: one block per (unit k, param p); sum over waves in fixed order
__global__ void grad_reduce_kernel(const float *part, int nw, int hidden, float *gwi, float *gbi,
                                   float *gwo) {
    __shared__ float red[256];
    const int kp = blockIdx.x, k = kp / 5, p = kp % 5;
    float s = 0.0f;
    for (int i = threadIdx.x; i < nw; i += blockDim.x) s += part[((size_t)i * hidden + k) * 5 + p];
    red[threadIdx.x] = s;
    __syncthreads();
    for (int w = 128; w > 0; w >>= 1) {
        if ((int)threadIdx.x < w) red[threadIdx.x] += red[threadIdx.x + w];
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        const float v = red[0];
        if (p < 3) gwi[k * kCtrlIn + p] = v;
        else if (p == 3) gbi[k] = v;
        else gwo[k] = v;
    }
}

}  // namespace fcr
