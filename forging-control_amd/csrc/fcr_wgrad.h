// fcr_wgrad.h — the LSTM surrogate's weight gradients at H > 52: the autograd weight
// gradients of nn.LSTM inside loss.backward() (Model_NN/Functions.py:520-569, :325):
//   dW_ih[l] = sum_{t, b} dG_l[t][b]^T x_l[t][b]          (n = 10 B rows)
//   dW_hh[l] = sum_{t >= 1, b} dG_l[t][b]^T h_l[t-1][b]   (n = 9 B rows)
// as ONE reduction per weight over all (window step, sample) rows n: C[r][k] = sum_n A[n][r] X[n][k], A the fp32
// dgate rows the fused backward cells write (fcr_wbwd.h WbArgs.dg, rows of 4 Hp in the padded gate order
// gate Hp + unit), X either fp32 rows (layer 0's window values) or the forward's split h records [hi (Hp) | lo (Hp)]
// whose sum is h (fcr_wgemm.h). The products are exact fp32 products of their operands on the matrix cores
// (v_mfma_f32_16x16x4_f32, fp32 in and out: the dgates of a reduction over 10 B rows span many powers of two, which an
// f16 split would have to rescale per row), fp32 accumulation, deterministic: the n range is split over S workgroups
// into fixed partial slabs summed in a fixed order (wgrad_sum_pad_kernel). The X operand of layers >= 1 is NOT the
// forward's fp32 h: it is rebuilt as hi + lo from the f16 record (hi = f16(h), lo = f16(h - hi)), which carries
// |h - (hi + lo)| <= 2^-11 |h - hi| <= 2^-22 |h| (lo rounds to 11 bits; a lo in f16's subnormal range, |h - hi| <
// 2^-14, adds at most 2^-25 absolute) — the same split error the forward's own products see, so the gradients match
// the fp64 oracle at the tests' 1e-5 (tests/test_surrogate.py) without an fp32 copy of every h.
// Tile: a workgroup owns 128 r x 128 k of C, 4 waves of 64 x 64 (4 x 4 tiles of 16 x 16); the n loop stages 16 rows
// of A and X (8 KB each) through LDS per step, so each MFMA operand element is loaded once per workgroup.
#pragma once
#include "fcr_common.h"
#include "fcr_wide.h"

namespace fcr {

constexpr int kWgrT = 128;                 // C tile (r and k) per workgroup
constexpr int kWgrN = 32;                  // n rows per staged step (8 MFMA k-steps of 4)
constexpr int kWgrThreads = 256;
constexpr int kWgrLd = kWgrT + 4;          // LDS row stride (floats): consecutive rows shift by 4 banks
constexpr int kWgrSmallK = 16;             // K up to this: wgrad_small_kernel (layer 0's 5 window columns)

struct WgradArgs {
    const float *A;            // [n][lda] fp32 dgate rows
    int lda;
    const float *X;            // fp32 rows [n][ldx], or null
    const _Float16 *XR;        // split records [n][2 Hx] (hi | lo), or null
    int ldx, Hx;               // fp32 row stride; the records' half width
    long long n;               // rows
    int R, K;                  // C rows (padded gate rows 4 Hp) and columns (real input width)
    long long n_per;           // rows per n slice (the split over blockIdx.z); a multiple of kWgrN
    float *part;               // [S][R][K] partial sums (slice s at + s R K)
};

// Round 5 (second session): 32 rows per step staged through two LDS buffers with ONE barrier per step, the next
// step's rows loaded into registers (16-B loads: 4 A quads and 2 + 2 record quads per thread) while the current one
// multiplies — the first form loaded, barriered, stored, barriered and multiplied 16 rows at a time, exposing every
// load's latency (48 TF/s on the surrogate's H = 256 step, 68 % of it).
__global__ __launch_bounds__(kWgrThreads, 2) void wgrad_kernel(WgradArgs a) {
    extern __shared__ __attribute__((aligned(16))) float wgs[];   // [2][As | Xs], each [kWgrN][kWgrLd]
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const int r0 = blockIdx.x * kWgrT, k0 = blockIdx.y * kWgrT;
    const long long nb = (long long)blockIdx.z * a.n_per, ne = nb + a.n_per < a.n ? nb + a.n_per : a.n;
    const int wr = (wv >> 1) * 64, wk = (wv & 1) * 64;   // the wave's 64 x 64 sub-tile
    f32x4 acc[4][4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
    // staging: thread -> row tid / 8 of the 32, 16 consecutive columns (tid % 8) * 16 of the 128
    const int sr = tid >> 3, sc = (tid & 7) * 16;
    f32x4 av[4], xv[4];
    auto load = [&](long long n0) {
        const long long n = n0 + sr;
        const bool live = n < ne;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int r = r0 + sc + 4 * q, k = k0 + sc + 4 * q;
            av[q] = (live && r + 3 < a.R) ? *reinterpret_cast<const f32x4 *>(a.A + n * a.lda + r) : f32x4{0, 0, 0, 0};
            if (a.X) {
                f32x4 v = {0, 0, 0, 0};
                if (live)
#pragma unroll
                    for (int e = 0; e < 4; ++e) v[e] = k + e < a.K ? a.X[n * a.ldx + k + e] : 0.0f;
                xv[q] = v;
            }
        }
        if (!a.X) {   // records: 16 hi and 16 lo halves = 2 + 2 quads (halves past K are zero padding units, and
                      // their columns are not stored)
            typedef _Float16 h8 __attribute__((ext_vector_type(8)));
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                const int k = k0 + sc + 8 * h;
                h8 hi = {}, lo = {};
                if (live && k < a.K) {
                    const _Float16 *rec = a.XR + n * 2 * a.Hx;
                    hi = *reinterpret_cast<const h8 *>(rec + k);
                    lo = *reinterpret_cast<const h8 *>(rec + a.Hx + k);
                }
#pragma unroll
                for (int e = 0; e < 8; ++e) xv[2 * h + e / 4][e % 4] = (float)hi[e] + (float)lo[e];
            }
        }
    };
    auto store = [&](int buf) {
        float *As = wgs + buf * 2 * kWgrN * kWgrLd, *Xs = As + kWgrN * kWgrLd;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            *reinterpret_cast<f32x4 *>(As + sr * kWgrLd + sc + 4 * q) = av[q];
            *reinterpret_cast<f32x4 *>(Xs + sr * kWgrLd + sc + 4 * q) = xv[q];
        }
    };
    long long n0 = nb;
    if (n0 < ne) {
        load(n0);
        store(0);
        if (n0 + kWgrN < ne) load(n0 + kWgrN);
    }
    for (int buf = 0; n0 < ne; n0 += kWgrN, buf ^= 1) {
        __syncthreads();   // buffer buf written; buffer buf ^ 1 no longer read (step - 1)
        if (n0 + kWgrN < ne) {
            store(buf ^ 1);                                   // rows of the next step, loaded during this one
            if (n0 + 2 * kWgrN < ne) load(n0 + 2 * kWgrN);   // and the step after, in flight across it
        }
        const float *As = wgs + buf * 2 * kWgrN * kWgrLd, *Xs = As + kWgrN * kWgrLd;
#pragma unroll
        for (int kk = 0; kk < kWgrN; kk += 4) {
            // 16x16x4 f32: lane l supplies A[i = l % 16][kk + l / 16] and X[kk + l / 16][j = l % 16]
            const int q = kk + (lane >> 4), i = lane & 15;
            float fa[4], fx[4];
#pragma unroll
            for (int t = 0; t < 4; ++t) {
                fa[t] = As[q * kWgrLd + wr + 16 * t + i];
                fx[t] = Xs[q * kWgrLd + wk + 16 * t + i];
            }
#pragma unroll
            for (int ti = 0; ti < 4; ++ti)
#pragma unroll
                for (int tj = 0; tj < 4; ++tj) acc[ti][tj] = mfma(fa[ti], fx[tj], acc[ti][tj]);
        }
    }
    // D: lane l holds C[4 (l / 16) + v][l % 16] of each 16 x 16 tile (v = 0..3)
    float *out = a.part + (long long)blockIdx.z * a.R * a.K;
#pragma unroll
    for (int ti = 0; ti < 4; ++ti)
#pragma unroll
        for (int tj = 0; tj < 4; ++tj)
#pragma unroll
            for (int v = 0; v < 4; ++v) {
                const int r = r0 + wr + 16 * ti + 4 * (lane >> 4) + v, k = k0 + wk + 16 * tj + (lane & 15);
                if (r < a.R && k < a.K) out[(long long)r * a.K + k] = acc[ti][tj][v];
            }
}
constexpr int kWgrLds = 2 * 2 * kWgrN * kWgrLd * 4;   // bytes

// The same reduction for K <= kWgrSmallK fp32 columns (layer 0's W_ih: the 5 window columns), where a 128-wide k tile
// would multiply zeros: one thread per gate row r and n slice, all K columns in registers, partials [S][R][K]
__global__ __launch_bounds__(256) void wgrad_small_kernel(WgradArgs a) {
    const int r = blockIdx.x * 256 + threadIdx.x;
    if (r >= a.R) return;
    const long long nb = (long long)blockIdx.y * a.n_per, ne = nb + a.n_per < a.n ? nb + a.n_per : a.n;
    float s[kWgrSmallK] = {};
#pragma unroll 8
    for (long long n = nb; n < ne; ++n) {
        const float g = a.A[n * a.lda + r];
#pragma unroll
        for (int k = 0; k < kWgrSmallK; ++k)
            if (k < a.K) s[k] = fmaf(g, a.X[n * a.ldx + k], s[k]);
    }
    float *out = a.part + (long long)blockIdx.y * a.R * a.K + (long long)r * a.K;
#pragma unroll
    for (int k = 0; k < kWgrSmallK; ++k)
        if (k < a.K) out[k] = s[k];
}

// dW (torch layout [4H][K], real units only) = sum over the S slices of the padded partials [S][4Hp][K], in slice
// order (deterministic)
__global__ void wgrad_sum_pad_kernel(const float *__restrict__ part, int S, int H, int Hp, int K, float *__restrict__ dW) {
    const long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= (long long)4 * H * K) return;
    const int k = (int)(e % K), tr = (int)(e / K), gate = tr / H, unit = tr % H;
    const long long src = (long long)(gate * Hp + unit) * K + k, RK = (long long)4 * Hp * K;
    float s = 0.0f;
    for (int i = 0; i < S; ++i) s += part[i * RK + src];
    dW[e] = s;
}

// The readout's gradients at H > 52: d fc.W [4][H] = sum_b dy[b] h[b] (h the fp32 top-layer h_9, rows of Hp), per
// column block of 64 units and slice of the batch into partials [S][4][Hp], then summed in slice order
__global__ __launch_bounds__(256) void fc_wgrad_part_kernel(const float *__restrict__ dy, const float *__restrict__ h,
                                                            int B, int Hp, int b_per, float *__restrict__ part) {
    const int u = blockIdx.x * 256 + threadIdx.x;
    if (u >= Hp) return;
    const int b0 = blockIdx.y * b_per, b1 = b0 + b_per < B ? b0 + b_per : B;
    float s[kOut] = {};
    for (int b = b0; b < b1; ++b) {
        const float hv = h[(size_t)b * Hp + u];
#pragma unroll
        for (int o = 0; o < kOut; ++o) s[o] = fmaf(dy[(size_t)b * kOut + o], hv, s[o]);
    }
#pragma unroll
    for (int o = 0; o < kOut; ++o) part[((size_t)blockIdx.y * kOut + o) * Hp + u] = s[o];
}
__global__ void fc_wgrad_sum_kernel(const float *__restrict__ part, int S, int H, int Hp, float *__restrict__ g) {
    const int e = blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= kOut * H) return;
    const int o = e / H, u = e % H;
    float s = 0.0f;
    for (int i = 0; i < S; ++i) s += part[((size_t)i * kOut + o) * Hp + u];
    g[e] = s;
}

// dh_9 of the top layer = dy fc.W (k8 rows of Hp, fcr_wide.h; fc.W padded with zero units)
__global__ void sur_head_kernel(const float *__restrict__ dy, const float *__restrict__ fcw, int B, int Hp,
                                float *__restrict__ dH) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= (size_t)B * Hp) return;
    const size_t b = i / Hp, u = i % Hp;
    float v = 0.0f;
#pragma unroll
    for (int o = 0; o < kOut; ++o) v = fmaf(dy[b * kOut + o], fcw[(size_t)o * Hp + u], v);
    dH[k8(B, (int)b, (int)u)] = v;
}

// the surrogate's window records at H > 52: layer 0's x part of the forward cells (fcr_wgemm.h), [10][B][2 kWideRecX0]
// halves, from the (B, 10, 5) window batch with the range guard's column scales (fcr_pack.h); and the same rows fp32
// time-major [10][B][5] for the weight gradient of W_ih0
__global__ void sur_window_rec_kernel(const float *__restrict__ x, const float *__restrict__ wsc, int B,
                                      _Float16 *__restrict__ wr, float *__restrict__ xt) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= B * kL) return;
    const int b = i / kL, t = i % kL;
    typedef _Float16 h8 __attribute__((ext_vector_type(8)));
    h8 hi = {}, lo = {};
#pragma unroll
    for (int c = 0; c < kIn; ++c) {
        const float v0 = x[((size_t)b * kL + t) * kIn + c];
        xt[((size_t)t * B + b) * kIn + c] = v0;
        const float v = v0 * wsc[c];
        hi[c] = (_Float16)v;
        lo[c] = (_Float16)(v - (float)hi[c]);
    }
    h8 *p = reinterpret_cast<h8 *>(wr + ((size_t)t * B + b) * 2 * kWideRecX0);
    const h8 z = {};
#pragma unroll
    for (int k = 0; k < kWideRecX0 / 8; ++k) {
        p[k] = k == 0 ? hi : z;
        p[kWideRecX0 / 8 + k] = k == 0 ? lo : z;
    }
}

}  // namespace fcr
