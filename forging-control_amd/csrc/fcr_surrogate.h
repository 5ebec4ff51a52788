// fcr_surrogate.h — kernels of the LSTM surrogate's own training step.
//
// Reference: Model_NN/Main.py:218-242 trains LSTMModel(5, 50, 4, 3) (Model_NN/Functions.py:255-330,
// no LSTM bias, fc readout of the last step) with nn.MSELoss and AdamW through
// NeuralNetwork.train_model (Model_NN/Functions.py:520-569): forward on a (B, 10, 5) window batch,
// loss.backward() for EVERY weight, optimizer.step().
//
// H > 52 runs the rollout's wide kernels over one window (fcr_wgemm.h forward cells, fcr_wbwd.h backward cells that
// also write each cell's dgates) and the weight gradients as ONE reduction per weight matrix over all 10·B
// (window step, sample) rows (fcr_wgrad.h):
//   dW_ih[l] = Σ_t dG_t^T · x_t        (k = 10·B),    dW_hh[l] = Σ_{t>=1} dG_t^T · h_{t-1}   (k = 9·B).
// H <= 52 runs the fused cells of fcr_sur.h.
// The kernels here are the glue: batch-first <-> time-major window transposes and the fc readout.
#pragma once
#include <hip/hip_runtime.h>

#include "fcr_common.h"

namespace fcr {
namespace surrogate {

constexpr int kSurBlock = 256;

// (B, L, F) batch-first -> (L, B, F) time-major (inverse = true: the other way)
__global__ __launch_bounds__(kSurBlock) void window_transpose_kernel(const float *__restrict__ src,
                                                                     float *__restrict__ dst, int B, int F,
                                                                     bool inverse) {
    const long long e = (long long)blockIdx.x * kSurBlock + threadIdx.x;
    if (e >= (long long)B * kL * F) return;
    const int f = (int)(e % F);
    const long long r = e / F;                   // row index in the destination layout
    long long s;
    if (!inverse) {                              // dst (t, b): source (b, t)
        const int t = (int)(r / B), b = (int)(r % B);
        s = ((long long)b * kL + t) * F + f;
    } else {                                     // dst (b, t): source (t, b)
        const int b = (int)(r / kL), t = (int)(r % kL);
        s = ((long long)t * B + b) * F + f;
    }
    dst[e] = src[s];
}

// y[b][o] = fc.W[o] · h[b] + fc.b[o]   (Model_NN/Functions.py:330: self.fc(out[:, -1, :]))
__global__ __launch_bounds__(kSurBlock) void readout_kernel(const float *__restrict__ h,
                                                            const float *__restrict__ fcw,
                                                            const float *__restrict__ fcb, float *__restrict__ y,
                                                            int B, int H) {
    const int b = blockIdx.x * kSurBlock + threadIdx.x;
    if (b >= B) return;
    const float *hb = h + (size_t)b * H;
    float acc[kOut];
#pragma unroll
    for (int o = 0; o < kOut; ++o) acc[o] = 0.0f;
    for (int j = 0; j < H; ++j) {
        const float v = hb[j];
#pragma unroll
        for (int o = 0; o < kOut; ++o) acc[o] = fmaf(fcw[o * H + j], v, acc[o]);
    }
#pragma unroll
    for (int o = 0; o < kOut; ++o) y[(size_t)b * kOut + o] = acc[o] + fcb[o];
}

// dh of the top layer's last step = dy · fc.W   (B x 4)(4 x H)
__global__ __launch_bounds__(kSurBlock) void readout_bwd_kernel(const float *__restrict__ dy,
                                                                const float *__restrict__ fcw, float *__restrict__ dh,
                                                                int B, int H) {
    const long long e = (long long)blockIdx.x * kSurBlock + threadIdx.x;
    if (e >= (long long)B * H) return;
    const int b = (int)(e / H), j = (int)(e % H);
    float acc = 0.0f;
#pragma unroll
    for (int o = 0; o < kOut; ++o) acc = fmaf(dy[(size_t)b * kOut + o], fcw[o * H + j], acc);
    dh[e] = acc;
}

// d fc.b = Σ_b dy[b]: one block per output, fixed-order tree (deterministic)
__global__ __launch_bounds__(kSurBlock) void bias_grad_kernel(const float *__restrict__ dy, float *__restrict__ g,
                                                              int B) {
    __shared__ float part[kSurBlock];
    const int o = blockIdx.x;
    float acc = 0.0f;
    for (int b = threadIdx.x; b < B; b += kSurBlock) acc += dy[(size_t)b * kOut + o];
    part[threadIdx.x] = acc;
    __syncthreads();
    for (int w = kSurBlock / 2; w > 0; w >>= 1) {
        if ((int)threadIdx.x < w) part[threadIdx.x] += part[threadIdx.x + w];
        __syncthreads();
    }
    if (threadIdx.x == 0) g[o] = part[0];
}

}  // namespace surrogate
}  // namespace fcr
