// fcr_small.h — small-batch rollout kernels (the reference trains at B = 15, UL/Main.py:84,297).
//
// The fused kernels (fcr_fwd.h, fcr_bwd.h) give each 16-trajectory group ONE wave that runs every
// cell of the rollout itself: below ~16 k trajectories (one wave per SIMD) the step time is that
// wave's sequential latency, ~3 ms whatever B is. Here a group gets a workgroup of NQ = ceil(HS/4)
// waves, one per SIMD, and wave w owns the unit slots of record quad w (slots 4w .. 4w+3):
//   forward  — wave w computes the gate tiles of its slots (fwd16_cell over that tile range), keeps
//              their c, and the cell's h_t is exchanged through LDS (one barrier per cell) so every
//              wave has the whole h_{t-1} for the next cell's B operand;
//   backward — wave w recomputes its tiles, forms the dgates of its slots and the partial transposed
//              product W[its gate rows]ᵀ·dgates for all output tiles (bwd_cell<..., PART>); the
//              partials are summed through LDS in a fixed order (two barriers per cell), and each
//              wave takes the dx / dh_prev of its own slots.
// Slab layout (hseq, cseq, xw, dseq) is that of the fused kernels — each wave writes its own quads
// of a record, and a record is read whole only across a phase barrier — so a split forward and a fused
// backward (or the reverse) are interchangeable; the backward's window-row gradients go to a per-wave
// copy of dxrow (every wave needs them at the window head), so nothing global is handed between waves
// inside a phase. Results equal the fused kernels' up to the fp32 order of the partial sums.
#pragma once
#include "fcr_bwd.h"
#include "fcr_fwd.h"

namespace fcr {

template <int HS>
struct Small {
    static constexpr int NQ = (HS + 3) / 4;                       // waves per workgroup = record quads
    static constexpr int XBUF = 2 * NQ * kWave * 16;              // h exchange, double-buffered
    static constexpr int LDS_FWD = Geo16<HS>::LDS_FWD + XBUF;
    static constexpr int NB = Img<HS, false>::NB > Img<HS, true>::NB ? Img<HS, false>::NB : Img<HS, true>::NB;
    static constexpr int RED = NQ * NB * kWave * 16;              // partial transposed products
    static constexpr int LDS_BWD = BwdLds<HS, false>::BYTES + RED;
    static_assert(LDS_FWD <= 163840 && LDS_BWD <= 163840, "small-batch LDS exceeds 160 KiB");
    static_assert(Geo16<HS>::LDS_FWD % 16 == 0 && BwdLds<HS, false>::BYTES % 16 == 0, "16-B aligned buffers");
};

template <int V>
struct IC {
    static constexpr int v = V;
};
// f(IC<w>) for the wave-uniform w: every quad's code is a compile-time instance (register arrays stay
// statically indexed)
template <int HS, class F>
__device__ __forceinline__ void by_quad(int w, F &&f) {
    if constexpr (HS > 12) {
        if (w == 3) { f(IC<3>{}); return; }
    }
    if constexpr (HS > 8) {
        if (w == 2) { f(IC<2>{}); return; }
    }
    if constexpr (HS > 4) {
        if (w == 1) { f(IC<1>{}); return; }
    }
    f(IC<0>{});
}
template <int HS, int W>
struct QR {   // slot range of quad W
    static constexpr int R0 = 4 * W, R1 = 4 * W + 4 < HS ? 4 * W + 4 : HS;
};

// quad k of a compact record (store_quads' layout: full quads, then the HS%4 tail slots per lane)
template <int HS, int k>
__device__ __forceinline__ void store_quad(f32x4 *dst, const float (&v)[HS], int lane) {
    constexpr int FQ = HS / 4, TS = HS % 4;
    if constexpr (k < FQ) {
        dst[k * kWave + lane] = f32x4{v[4 * k], v[4 * k + 1], v[4 * k + 2], v[4 * k + 3]};
    } else {
        float *t = reinterpret_cast<float *>(dst + FQ * kWave) + lane * TS;
        if constexpr (TS == 1) {
            t[0] = v[4 * FQ];
        } else if constexpr (TS == 2) {
            *reinterpret_cast<f32x2 *>(t) = f32x2{v[4 * FQ], v[4 * FQ + 1]};
        } else {
            typedef float f32x3 __attribute__((ext_vector_type(3)));
            *reinterpret_cast<f32x3 *>(t) = f32x3{v[4 * FQ], v[4 * FQ + 1], v[4 * FQ + 2]};
        }
    }
}

// LDS-only workgroup barrier: the wave's LDS writes are complete, its global loads stay in flight
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }
// before a barrier that hands global slab records between waves: this wave's stores are complete
__device__ __forceinline__ void vm_drain() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

// h exchange: wave W publishes its slots of h_t, every wave reads the whole vector back
template <int HS, int W>
__device__ __forceinline__ void xchg_put(f32x4 *xb, const float (&h)[HS], int lane) {
    using Q = QR<HS, W>;
    f32x4 v = {0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
    for (int e = 0; e < 4; ++e)
        if (Q::R0 + e < Q::R1) v[e] = h[Q::R0 + e];
    xb[W * kWave + lane] = v;
}
template <int HS>
__device__ __forceinline__ void xchg_get(const f32x4 *xb, float (&h)[HS], int lane) {
#pragma unroll
    for (int k = 0; k < Small<HS>::NQ; ++k) {
        const f32x4 v = xb[k * kWave + lane];
#pragma unroll
        for (int e = 0; e < 4; ++e)
            if (4 * k + e < HS) h[4 * k + e] = v[e];
    }
}

// ---------------------------------------------------------------------------------------------------
// forward: the fused forward kernel's program (fcr_fwd.h) with the cell's tiles split over the waves
// ---------------------------------------------------------------------------------------------------
template <int HS, bool STORE>
__global__ __launch_bounds__(Small<HS>::NQ * kWave, 1) void fcr_sfwd_kernel(FwdArgs a) {
    using G = Geo16<HS>;
    constexpr int NQ = Small<HS>::NQ;
    extern __shared__ __attribute__((aligned(16))) float lw[];
    // [layer 1|2 fragments, refilled per phase | layer 0 | misc | h exchange]
    float *lw0 = lw + G::FA1;
    float *lfnp = lw0 + G::FA0;
    float *lfcp = lfnp + G::FNP;
    float *lfcb = lfcp + G::FCP;
    f32x4 *xbuf = reinterpret_cast<f32x4 *>(lw + G::LDS_FWD / 4);
    lds_copy(lw0, a.p.fa[0], G::FA0);
    lds_copy(lfnp, a.p.fnp, G::FNP);
    lds_copy(lfcp, a.p.fcp, G::FCP);
    lds_copy(lfcb, a.p.fcb, 4);
    const int lane = threadIdx.x & 63;
    const int q = lane >> 4, sl = lane & 15;
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int grp = blockIdx.x;   // the fused kernels' wave index: same slab regions
    const int b = grp * kTile + sl;
    const bool valid = b < a.B;
    const bool lead = w == 0;     // writes the per-trajectory outputs
    const int bc = valid ? b : a.B - 1;
    const int N = a.N;
    const float alpha = a.alpha;

    const float ref = a.X[(size_t)bc * kCtrlIn + 2];                 // Functions.py:1392
    const float *st = a.states + (size_t)bc * kL * kIn;
    float w0[kL], w1[kL];
    const float scq = a.p.wsc[q], sc4 = a.p.wsc[4];
#pragma unroll
    for (int t = 0; t < kL; ++t) {
        w0[t] = st[t * kIn + q] * scq;
        w1[t] = (q == 0) ? st[t * kIn + 4] * sc4 : 0.0f;
    }
    const float u0 = a.u0[bc];
    if (q == 0) w1[kL - 1] = u0 * sc4;                                // Functions.py:1396
    float u_prev = u0;
    float cmd_j = alpha * sq(st[(kL - 2) * kIn + 4] - u0);            // Functions.py:1405
    float cmd_sum = 0.0f, err_sum = 0.0f, tot_sum = 0.0f;
    float xh0 = 0.0f, xh1 = 0.0f, xh2 = 0.0f, xh3 = 0.0f;

    float c[HS], hout[HS], hp[HS], xc[HS], xn[HS];
#pragma unroll
    for (int r = 0; r < HS; ++r) c[r] = hout[r] = hp[r] = xc[r] = xn[r] = 0.0f;
    const size_t qcell = (size_t)Geo<HS>::QC;
    const size_t wseq = (size_t)grp * N * kLayers * kL * qcell;
    f32x4 *hs_wave = a.hseq + wseq;
    f32x4 *cs_wave = a.cseq + wseq;
    f32x2 *xw_wave = a.xw + (size_t)grp * N * kL * kWave;
    Pace turn;
    turn.turn = 0;
    turn.me = w;
    turn.cnt = turn.other = 0;
    turn.prog = nullptr;
    __syncthreads();

    for (int j = 0; j < N; ++j) {
        const float *lfnp_j = opaque(lfnp), *lfcp_j = opaque(lfcp), *lfcb_j = opaque(lfcb);
        float pred = u0;
        if (j > 0) {                                                   // Functions.py:1421-1434
            float z[kMS];
            const float un = hardtanh(fnn_pre(lfnp_j, q, xh0, xh3, ref, z));
            cmd_j = alpha * sq(u_prev - un);                           // Functions.py:1446
#pragma unroll
            for (int k = 0; k < kL - 1; ++k) {
                w0[k] = w0[k + 1];
                w1[k] = w1[k + 1];
            }
            w0[kL - 1] = sel4(q, xh0, xh1, xh2, xh3) * scq;
            w1[kL - 1] = (q == 0) ? un * sc4 : 0.0f;
            u_prev = un;
            pred = un;
        }
        if (lead && valid && q == 0) a.prediction[(size_t)b * N + j] = pred;   // Functions.py:1455,1466

        f32x4 *hsj = hs_wave + (size_t)j * kLayers * kL * qcell;
        f32x4 *csj = cs_wave + (size_t)j * kLayers * kL * qcell;
#define SEQ_H(l, t) (hsj + (size_t)((l) * kL + (t)) * qcell)
#define SEQ_C(l, t) (csj + (size_t)((l) * kL + (t)) * qcell)
        // ---- layer 0 (Functions.py:374) ----
        for (int t = 0; t < kL; ++t) {
            const float x0 = w0[0], x1 = w1[0];
            rot_left(w0);
            rot_left(w1);
            by_quad<HS>(w, [&](auto Wc) {
                constexpr int W = decltype(Wc)::v;
                using Q = QR<HS, W>;
                if (t == 0) fwd16_cell<HS, true, true, false, Q::R0, Q::R1>(lw0, lane, x0, x1, hp, hp, c, hout, turn);
                else fwd16_cell<HS, true, false, false, Q::R0, Q::R1>(lw0, lane, x0, x1, hp, hp, c, hout, turn);
                store_quad<HS, W>(SEQ_H(0, t), hout, lane);
                if (STORE && t + 1 < kL) store_quad<HS, W>(SEQ_C(0, t), c, lane);   // c_9 is never a c_{t-1}
                if (t + 1 < kL) xchg_put<HS, W>(xbuf + (t & 1) * NQ * kWave, hout, lane);
            });
            if (STORE && lead) xw_wave[((size_t)j * kL + t) * kWave + lane] = f32x2{x0, x1};
            if (t + 1 < kL) {
                lds_barrier();
                xchg_get<HS>(xbuf + (t & 1) * NQ * kWave, hp, lane);
            }
        }
        // ---- layers 1, 2: input sequence from the slab records the workgroup wrote ----
#pragma unroll
        for (int l = 1; l < kLayers; ++l) {
            const bool keep_h = l == 1 || STORE;
            vm_drain();   // this wave's quads of the layer-below records are in memory before the barrier
            lds_fill<G::FA1 * 4, NQ>(lw, a.p.fa[l]);
            load_quads<HS>(xc, SEQ_H(l - 1, 0), lane);
            for (int t = 0; t < kL; ++t) {
                load_quads<HS>(xn, SEQ_H(l - 1, t + 1 < kL ? t + 1 : t), lane);
                const bool xch = t + 1 < kL || l == kLayers - 1;   // the readout needs the whole h_9 of layer 2
                by_quad<HS>(w, [&](auto Wc) {
                    constexpr int W = decltype(Wc)::v;
                    using Q = QR<HS, W>;
                    if (t == 0) fwd16_cell<HS, false, true, false, Q::R0, Q::R1>(lw, lane, 0.0f, 0.0f, xc, hp, c, hout, turn);
                    else fwd16_cell<HS, false, false, false, Q::R0, Q::R1>(lw, lane, 0.0f, 0.0f, xc, hp, c, hout, turn);
                    if (keep_h && !(l == 2 && t + 1 == kL)) store_quad<HS, W>(SEQ_H(l, t), hout, lane);
                    if (STORE && t + 1 < kL) store_quad<HS, W>(SEQ_C(l, t), c, lane);
                    if (xch) xchg_put<HS, W>(xbuf + (t & 1) * NQ * kWave, hout, lane);
                });
                if (xch) {
                    lds_barrier();
                    xchg_get<HS>(xbuf + (t & 1) * NQ * kWave, hp, lane);
                }
#pragma unroll
                for (int r = 0; r < HS; ++r) xc[r] = xn[r];
            }
        }
#undef SEQ_H
#undef SEQ_C
        // ---- readout fc(h_9 of layer 2) (Functions.py:377), identical in every wave ----
        float xo[kOut];
#pragma unroll
        for (int o = 0; o < kOut; ++o) {
            float p = 0.0f;
#pragma unroll
            for (int r = 0; r < HS; ++r) p += lfcp_j[(o * HS + r) * 4 + q] * hp[r];
            xo[o] = xor_sum_q(p) + lfcb_j[o];
        }
        if (a.noise) {                                                 // Functions.py:1400-1402
            const float *nz = a.noise + ((size_t)bc * N + j) * kOut;
#pragma unroll
            for (int o = 0; o < kOut; ++o) xo[o] += nz[o];
        }
        xh0 = xo[0];
        xh1 = xo[1];
        xh2 = xo[2];
        xh3 = xo[3];
        if (lead && valid) {
            const float mine = sel4(q, xh0, xh1, xh2, xh3);
            a.xhat_ws[((size_t)b * N + j) * kOut + q] = mine;
            if (a.xhat_user) a.xhat_user[((size_t)b * N + j) * kOut + q] = mine;
        }
        const float err = sq(xh0 - ref);                              // Functions.py:1405-1414, 1443-1452
        const float con = relu(-xh1) + relu(-xh2) + relu(xh1 - kP1Max) + relu(xh2 - kP2Max);
        tot_sum += (err + cmd_j) + con;
        err_sum += err;
        cmd_sum += cmd_j;
    }
    const float cost = tot_sum / (float)N;                             // Functions.py:1458-1460
    if (lead && valid && q == 0) {
        a.cost[b] = cost;
        a.command[b] = cmd_sum / (float)N;
        a.error[b] = err_sum / (float)N;
    }
    float part = (valid && q == 0) ? cost : 0.0f;
#pragma unroll
    for (int m = 1; m < 64; m <<= 1) part += __shfl_xor(part, m);
    if (lead && lane == 0) a.loss_part[grp] = part;
}

// ---------------------------------------------------------------------------------------------------
// backward: the fused backward kernel's program (fcr_bwd.h) with each cell's slots split over the waves
// ---------------------------------------------------------------------------------------------------
// Partial products of one cell -> the sums this wave needs: dh_prev of its slots (L0: combined slots σ =
// s; else σ = HS + s), dx of its slots (layers >= 1: σ = s, into its dseq quad) and, for L0, the window
// columns σ = HS, HS+1 (every wave: the row gradients feed each wave's window head).
template <int HS, bool L0, int W>
__device__ __forceinline__ void small_reduce(f32x4 *red, const f32x4 (&part)[Small<HS>::NB], int lane, float (&dh)[HS],
                                             float (&dxo)[HS], float &dxq, float &dx4) {
    using Q = QR<HS, W>;
    constexpr int NQ = Small<HS>::NQ, NB = Small<HS>::NB;
    constexpr int NBL = Img<HS, L0>::NB;
    asm volatile("s_barrier" ::: "memory");   // every wave has read the previous cell's partials
#pragma unroll
    for (int tau = 0; tau < NBL; ++tau) red[(W * NB + tau) * kWave + lane] = part[tau];
    lds_barrier();
    auto need = [&](int tau) {
        bool n = false;
        for (int s = Q::R0; s < Q::R1; ++s) {
            if ((s >> 2) == tau && !L0) n = true;                      // dx of own slots
            if (((L0 ? s : HS + s) >> 2) == tau) n = true;             // dh_prev of own slots
        }
        if (L0 && (HS >> 2 == tau || (HS + 1) >> 2 == tau)) n = true;  // window columns
        return n;
    };
    f32x4 sum[NB];
#pragma unroll
    for (int tau = 0; tau < NBL; ++tau) {
        if (!need(tau)) continue;
        f32x4 s = red[tau * kWave + lane];
#pragma unroll
        for (int v = 1; v < NQ; ++v) s += red[(v * NB + tau) * kWave + lane];
        sum[tau] = s;
    }
#pragma unroll
    for (int s = Q::R0; s < Q::R1; ++s) {
        const int sh = L0 ? s : HS + s;
        dh[s] = sum[sh >> 2][sh & 3];
        if (!L0) dxo[s] = sum[s >> 2][s & 3];
    }
    if (L0) {
        dxq = sum[HS >> 2][HS & 3];
        dx4 = sum[(HS + 1) >> 2][(HS + 1) & 3];
    }
}

template <int HS, bool L0, bool DIN, bool FIRST, bool NX_L0, bool NX_HC, bool NX_DIN>
__device__ __forceinline__ void sbwd_cell(int w, uint32_t fb, uint32_t tb, int lane, const float (&ext)[HS],
                                          float (&dh)[HS], float (&dc)[HS], float (&dxo)[HS], float &dxq, float &dx4,
                                          CellIn<HS> &ci, const NextIn &nx, Stamps &sp, f32x4 *red, f32x4 *dseq_cell) {
    by_quad<HS>(w, [&](auto Wc) {
        constexpr int W = decltype(Wc)::v;
        using Q = QR<HS, W>;
        f32x4 part[Small<HS>::NB];
        bwd_cell<HS, L0, DIN, FIRST, NX_L0, NX_HC, NX_DIN, false, Q::R0, Q::R1, true>(fb, tb, lane, ext, dh, dc, dxo, dxq,
                                                                                     dx4, ci, nx, sp, part);
        small_reduce<HS, L0, W>(red, part, lane, dh, dxo, dxq, dx4);
        if (!L0) store_quad<HS, W>(dseq_cell, dxo, lane);
    });
}

template <int HS>
__global__ __launch_bounds__(Small<HS>::NQ * kWave, 1) void fcr_sbwd_kernel(BwdArgs a) {
    using LD = BwdLds<HS, false>;
    using I1 = Img<HS, false>;
    using I0 = Img<HS, true>;
    constexpr int NQ = Small<HS>::NQ;
    extern __shared__ __attribute__((aligned(16))) float lw[];
    float *lfnp = lw + LD::REGION / 4;
    float *lfcp = lfnp + LD::FNP;
    f32x4 *red = reinterpret_cast<f32x4 *>(lw + LD::BYTES / 4);
    lds_copy(lfnp, a.p.fnp, LD::FNP);
    lds_copy(lfcp, a.p.fcp, LD::FCP);
    __syncthreads();
    const int lane = threadIdx.x & 63;
    const int q = lane >> 4, sl = lane & 15;
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int grp = blockIdx.x;
    const int b = grp * kTile + sl;
    const bool valid = b < a.B;
    const bool lead = w == 0;
    const int bc = valid ? b : a.B - 1;
    const int N = a.N;
    const float alpha = a.alpha;
    const float wgt = valid ? a.dloss[0] / ((float)a.B * (float)N) : 0.0f;   // Functions.py:1458, 1463
    const float ref = a.X[(size_t)bc * kCtrlIn + 2];
    const float scq = a.p.wsc[q], sc4 = a.p.wsc[4];
    const float s84 = a.states[(size_t)bc * kL * kIn + (kL - 2) * kIn + 4];
    const float *pred = a.prediction + (size_t)bc * N;
    const float *xh = a.xhat + (size_t)bc * N * kOut;
    const ImgLane<I1::U> L1 = img_lane<I1::U>(lds_offset(lw), lane);
    const ImgLane<I0::U> L0 = img_lane<I0::U>(lds_offset(lw), lane);

    // this wave's own copy of the window-row gradients (dxrow holds NQ copies per group)
    const __amdgpu_buffer_rsrc_t rr =
        wave_rsrc(a.dxrow + ((size_t)grp * NQ + w) * N * kL * kWave, (size_t)N * kL * kWave * 8);
    auto row_grad = [&](int rho) {
        f32x2 acc2 = {0.0f, 0.0f};
        const int w_hi = rho < N - 1 ? rho : N - 1;
        const int w_lo = rho - (kL - 1) > 0 ? rho - (kL - 1) : 0;
        for (int v = w_hi; v >= w_lo; --v) acc2 += buf_ld2(rr, lane * 8, (uint32_t)((v * kL + (rho - v)) * kWave * 8));
        return acc2;
    };
    float dh[HS], dc[HS], dxo[HS], dab[HS];
#pragma unroll
    for (int r = 0; r < HS; ++r) dh[r] = dc[r] = dxo[r] = dab[r] = 0.0f;

    const size_t qcell = (size_t)Geo<HS>::QC;
    const size_t seq_sz = (size_t)N * kLayers * kL * qcell;
    const size_t dseq_sz = (size_t)N * 2 * kL * qcell;
    NextIn nb;
    nb.rh = wave_rsrc(a.hseq + (size_t)grp * seq_sz, seq_sz * 16);
    nb.rc = wave_rsrc(a.cseq + (size_t)grp * seq_sz, seq_sz * 16);
    nb.rx = wave_rsrc(a.xw + (size_t)grp * N * kL * kWave, (size_t)N * kL * kWave * 8);
    nb.rd = wave_rsrc(a.dseq + (size_t)grp * dseq_sz, dseq_sz * 16);
    f32x4 *dseq_w = a.dseq + (size_t)grp * dseq_sz;
    auto hoff = [&](int j, int l, int t) { return (uint32_t)(((size_t)(j * kLayers + l) * kL + t) * qcell * 16); };
    auto doff = [&](int j, int lfrom, int t) { return ((size_t)(j * 2 + (2 - lfrom)) * kL + t) * qcell; };
    auto next_of = [&](int j, int l, int t) {   // the cell processed after (j, l, t)
        NextIn n = nb;
        int nj = j, nl = l, nt = t - 1;
        if (t == 0) {
            nt = kL - 1;
            nl = l - 1;
            if (l == 0) { nl = 2; nj = j - 1; }
        }
        if (nj < 0) { nj = 0; nl = 2; nt = 9; }
        n.x = nl == 0 ? (uint32_t)((nj * kL + nt) * kWave * 8) : hoff(nj, nl > 0 ? nl - 1 : 0, nt);
        n.h = hoff(nj, nl, nt > 0 ? nt - 1 : 0);
        n.c = n.h;
        n.d = (uint32_t)((nl < 2 ? doff(nj, nl + 1, nt) : 0) * 16);
        return n;
    };
    Stamps sp = {{0, 0, 0, 0, 0, 0, 0, 0}};
    CellIn<HS> ci;
    {
        const NextIn f = next_of(N - 1, 2, kL);
        load_xhd<HS, false, true, false>(ci, f, lane);
        ld_quads<HS>(ci.c, f.rc, f.c, lane);
    }
    float dxq = 0.0f, dx4 = 0.0f;

    for (int j = N - 1; j >= 0; --j) {
        const float *lfnp_j = opaque(lfnp), *lfcp_j = opaque(lfcp);
        // layer 2's image; the barriers also order the previous window's row-gradient stores
        lds_fill<I1::BYTES, NQ>(lw, a.p.img[2]);
        const float x0 = xh[j * kOut + 0], x1 = xh[j * kOut + 1], x2 = xh[j * kOut + 2], x3 = xh[j * kOut + 3];
        float d0 = wgt * 2.0f * (x0 - ref);                             // Functions.py:1443-1452
        float d1 = wgt * ((-x1 > 0.0f ? -1.0f : 0.0f) + (x1 - kP1Max > 0.0f ? 1.0f : 0.0f));
        float d2 = wgt * ((-x2 > 0.0f ? -1.0f : 0.0f) + (x2 - kP2Max > 0.0f ? 1.0f : 0.0f));
        float d3 = 0.0f;
        if (j <= N - 2) {
            const f32x2 Gr = row_grad(kL + j);
            d0 += __shfl(Gr[0], sl);
            d1 += __shfl(Gr[0], sl + 16);
            d2 += __shfl(Gr[0], sl + 32);
            d3 += __shfl(Gr[0], sl + 48);
            const float g4 = __shfl(Gr[1], sl);
            const float uj = pred[j], uj1 = pred[j + 1];
            float du = 2.0f * alpha * wgt * (uj1 - uj);
            if (j + 2 < N) du += 2.0f * alpha * wgt * (uj1 - pred[j + 2]);
            du += g4;
            float z[kMS];                                               // Functions.py:1424-1430
            const float v = fnn_pre(lfnp_j, q, x0, x3, ref, z);
            const float dv = (v > -1.0f && v < 1.0f) ? du : 0.0f;
            float dca = 0.0f, dcb = 0.0f;
#pragma unroll
            for (int m = 0; m < kMS; ++m) {
                const float *p = lfnp_j + (m * 4 + q) * kFnpStride;
                const float dz = (z[m] > 0.0f) ? dv * p[4] : 0.0f;
                dca += dz * p[0];
                dcb += dz * p[1];
            }
            if (lead && valid && q == 0) a.dv[(size_t)b * N + j] = dv;
            d0 += xor_sum_q(dca);
            d3 += xor_sum_q(dcb);
        } else if (lead && valid && q == 0) {
            a.dv[(size_t)b * N + j] = 0.0f;
        }
        float dh_out[HS];
#pragma unroll
        for (int r = 0; r < HS; ++r) {
            const float *fp = lfcp_j + r * 4 + q;
            dh_out[r] = fp[0] * d0 + fp[HS * 4] * d1 + fp[2 * HS * 4] * d2 + fp[3 * HS * 4] * d3;
        }
        // ---- layer 2 ----
#pragma unroll
        for (int r = 0; r < HS; ++r) dh[r] = dc[r] = 0.0f;
        for (int t = kL - 1; t >= 2; --t) {
#pragma unroll
            for (int r = 0; r < HS; ++r) dab[r] = (t == kL - 1) ? dh_out[r] : 0.0f;
            sbwd_cell<HS, false, false, false, false, true, false>(w, L1.fb, L1.tb, lane, dab, dh, dc, dxo, dxq, dx4, ci,
                                                                   next_of(j, 2, t), sp, red, dseq_w + doff(j, 2, t));
        }
#pragma unroll
        for (int r = 0; r < HS; ++r) dab[r] = 0.0f;
        sbwd_cell<HS, false, false, false, false, false, false>(w, L1.fb, L1.tb, lane, dab, dh, dc, dxo, dxq, dx4, ci,
                                                                next_of(j, 2, 1), sp, red, dseq_w + doff(j, 2, 1));
        sbwd_cell<HS, false, false, true, false, true, true>(w, L1.fb, L1.tb, lane, dab, dh, dc, dxo, dxq, dx4, ci,
                                                             next_of(j, 2, 0), sp, red, dseq_w + doff(j, 2, 0));
        // ---- layer 1 ----
        lds_fill<I1::BYTES, NQ>(lw, a.p.img[1]);
#pragma unroll
        for (int r = 0; r < HS; ++r) dh[r] = dc[r] = 0.0f;
        for (int t = kL - 1; t >= 2; --t)
            sbwd_cell<HS, false, true, false, false, true, true>(w, L1.fb, L1.tb, lane, dab, dh, dc, dxo, dxq, dx4, ci,
                                                                 next_of(j, 1, t), sp, red, dseq_w + doff(j, 1, t));
        sbwd_cell<HS, false, true, false, false, false, true>(w, L1.fb, L1.tb, lane, dab, dh, dc, dxo, dxq, dx4, ci,
                                                              next_of(j, 1, 1), sp, red, dseq_w + doff(j, 1, 1));
        sbwd_cell<HS, false, true, true, true, true, true>(w, L1.fb, L1.tb, lane, dab, dh, dc, dxo, dxq, dx4, ci,
                                                           next_of(j, 1, 0), sp, red, dseq_w + doff(j, 1, 0));
        // ---- layer 0: dx -> window-row gradients (this wave's copy) ----
        lds_fill<I0::BYTES, NQ>(lw, a.p.img[0]);
#pragma unroll
        for (int r = 0; r < HS; ++r) dh[r] = dc[r] = 0.0f;
        for (int t = kL - 1; t >= 2; --t) {
            sbwd_cell<HS, true, true, false, true, true, true>(w, L0.fb, L0.tb, lane, dab, dh, dc, dxo, dxq, dx4, ci,
                                                               next_of(j, 0, t), sp, red, nullptr);
            buf_st2(rr, lane * 8, (uint32_t)((j * kL + t) * kWave * 8), f32x2{dxq * scq, dx4 * sc4});   // row j+t
        }
        sbwd_cell<HS, true, true, false, true, false, true>(w, L0.fb, L0.tb, lane, dab, dh, dc, dxo, dxq, dx4, ci,
                                                            next_of(j, 0, 1), sp, red, nullptr);
        buf_st2(rr, lane * 8, (uint32_t)((j * kL + 1) * kWave * 8), f32x2{dxq * scq, dx4 * sc4});       // row j+1
        sbwd_cell<HS, true, true, true, false, true, false>(w, L0.fb, L0.tb, lane, dab, dh, dc, dxo, dxq, dx4, ci,
                                                            next_of(j, 0, 0), sp, red, nullptr);
        buf_st2(rr, lane * 8, (uint32_t)((j * kL) * kWave * 8), f32x2{dxq * scq, dx4 * sc4});           // row j
    }
    const float g_u0_rows = row_grad(kL - 1)[1];   // row 9, col 4 = u0 (Functions.py:1396)
    float du0 = 2.0f * alpha * wgt * (pred[0] - s84);
    if (N > 1) du0 += 2.0f * alpha * wgt * (pred[0] - pred[1]);
    if (lead && valid && q == 0) a.g_u0[b] = g_u0_rows + du0;
}

}  // namespace fcr
