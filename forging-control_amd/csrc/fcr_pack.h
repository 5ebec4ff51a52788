// fcr_pack.h — weight packing into MFMA fragment order, and fixed-order reductions.
#pragma once
#include "fcr_common.h"

namespace fcr {

struct PackArgs {
    int H, HS, CH;
    const float *wih[3], *whh[3], *fcw, *fcb, *cwi, *cbi, *cwo;
    float *fa[3], *ba[3], *fcp, *fcbo, *fnp;
};

// Forward fragment, layout [r][k/4][lane][k%4]: element (r, s, lane) is A[rho][k] of k-step s with
// rho = lane&15 -> unit 4r+(rho>>2), gate rho&3 (torch row gate*H + unit); k = lane>>4 -> input
// index of k-step s (layer 0: s<2 window column 4s+k, else h unit 4(s-2)+k; layer>=1: s<HS
// layer-below unit 4s+k, else h unit 4(s-HS)+k). Padding (unit >= H, column >= 5, s >= KS) is 0.
__global__ void pack_fwd_kernel(PackArgs a, int l) {
    const int H = a.H, HS = a.HS;
    const int KS = l == 0 ? 2 + HS : 2 * HS;
    const int KQ = (KS + 3) / 4 * 4;
    const int n = HS * KQ * kWave;
    const int idx = blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= n) return;
    const int e = idx & 3, lane = (idx >> 2) & 63, rq = idx >> 8;
    const int qd = rq % (KQ / 4), r = rq / (KQ / 4);
    const int s = 4 * qd + e;
    const int rho = lane & 15, kq = lane >> 4;
    const int unit = 4 * r + (rho >> 2), gate = rho & 3;
    float v = 0.0f;
    if (unit < H && s < KS) {
        const int grow = gate * H + unit;
        if (l == 0) {
            if (s < 2) {
                const int col = 4 * s + kq;
                if (col < kIn) v = a.wih[0][grow * kIn + col];
            } else {
                const int u = 4 * (s - 2) + kq;
                if (u < H) v = a.whh[0][grow * H + u];
            }
        } else {
            if (s < HS) {
                const int u = 4 * s + kq;
                if (u < H) v = a.wih[l][grow * H + u];
            } else {
                const int u = 4 * (s - HS) + kq;
                if (u < H) v = a.whh[l][grow * H + u];
            }
        }
    }
    a.fa[l][idx] = v * (gate == 2 ? kTwoLog2e : kNegLog2e);   // exp2 argument scaling, see fwd_pointwise
}

// Backward fragment, layout [tau][r][lane][gamma]: element is A'[rho][k] of k-step s' = 4r+gamma
// with rho = lane&15 -> output slot sigma = 4tau+(rho&3) in lane group qo = rho>>2, and
// k = lane>>4 -> gate row gamma*H + 4r + k. Output slots: layer>=1: sigma<HS dx unit 4sigma+qo
// (W_ih column), HS<=sigma<2HS dh_prev unit 4(sigma-HS)+qo (W_hh column); layer 0: sigma<HS dh_prev,
// sigma==HS dx column qo, sigma==HS+1 dx column 4 (qo==0 only).
__global__ void pack_bwd_kernel(PackArgs a, int l) {
    const int H = a.H, HS = a.HS;
    const int NB = l == 0 ? (HS + 2 + 3) / 4 : (2 * HS + 3) / 4;
    const int n = NB * HS * kWave * 4;
    const int idx = blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= n) return;
    const int gate = idx & 3, lane = (idx >> 2) & 63, tr = idx >> 8;
    const int r = tr % HS, tau = tr / HS;
    const int rho = lane & 15, kq = lane >> 4;
    const int sigma = 4 * tau + (rho & 3), qo = rho >> 2;
    const int unit_k = 4 * r + kq;
    float v = 0.0f;
    if (unit_k < H) {
        const int grow = gate * H + unit_k;
        if (l == 0) {
            if (sigma < HS) {
                const int u = 4 * sigma + qo;
                if (u < H) v = a.whh[0][grow * H + u];
            } else if (sigma == HS) {
                v = a.wih[0][grow * kIn + qo];
            } else if (sigma == HS + 1 && qo == 0) {
                v = a.wih[0][grow * kIn + 4];
            }
        } else {
            if (sigma < HS) {
                const int u = 4 * sigma + qo;
                if (u < H) v = a.wih[l][grow * H + u];
            } else if (sigma < 2 * HS) {
                const int u = 4 * (sigma - HS) + qo;
                if (u < H) v = a.whh[l][grow * H + u];
            }
        }
    }
    a.ba[l][idx] = v;
}

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
