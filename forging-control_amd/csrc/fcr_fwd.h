// fcr_fwd.h — forward rollout kernel (MPCLoss.forward, Functions.py:1353-1472).
//
// One wave = 16 trajectories; one workgroup = kFwdWaves waves sharing one LDS-resident layer of
// MFMA fragments. Each window (horizon step) runs three layer PHASES (layer-major): the current
// layer's fragments are copied into LDS, then the wave steps t = 0..9 through that layer. The layer's
// 10 outputs go to a per-wave global slab (written once, read once, prefetched one cell ahead by the
// next phase), which keeps the live state small enough for 2 waves per SIMD.
#pragma once
#include "fcr_common.h"
#include "fcr_f16.h"

namespace fcr {

// Cell update for one unit slot: a = D fragment (i,f,g,o pre-activations of unit 4r+q).
template <bool FIRST, bool STORE>
__device__ __forceinline__ void fwd_pointwise(f32x4 a, float &c, float &h, f32x4 *gs, f32x2 *cs,
                                              int lane) {
    // The packed weights carry the exp2 scaling (pack_fwd_kernel): a = (-x log2e) for i, f, o and
    // (2 x log2e) for g, so each activation is exp2 + add + rcp (+ one fma for tanh).
    const float i = sigm_pre(a[0]);
    const float f = sigm_pre(a[1]);
    const float g = tanh_pre(a[2]);
    const float o = sigm_pre(a[3]);
    const float gi = g * i;
    const float cf = FIRST ? 0.0f : f * c;            // c_{-1} = 0 (Functions.py:349-350)
    const float cn = cf + gi;
    c = cn;
    const float tc = tanh_f(cn);
    h = o * tc;
    if (STORE) {   // local derivatives for the backward (fcr_bwd.h cell_grad), 24 B per slot:
        // dh/dc = o(1-tc^2), dh/do_pre = tc o(1-o), dc/di_pre = g i(1-i), dc/df_pre = c_{t-1} f(1-f),
        // dc/dg_pre = i(1-g^2), and f — each one fma from products already formed
        gs[lane] = f32x4{fmaf(-h, tc, o), fmaf(-h, o, h), fmaf(-gi, i, gi), fmaf(-cf, f, cf)};
        cs[lane] = f32x2{fmaf(-gi, g, i), f};
    }
}

// One LSTM cell for 16 trajectories. L0: input is the window row (x0: column q in lane group q,
// x1: column 4 in lane group 0); otherwise x = the layer-below h_t. FIRST: t = 0 (h_{t-1} = 0, so the
// recurrent product is skipped). lw = this layer's fragments in LDS, [r][k-quad][lane][4]: one
// ds_read_b128 feeds four MFMAs. Each k-quad is its own scheduling region (bounded register use);
// the cell update of tile r-1 is issued in the first region of tile r, beside its MFMAs.
template <int HS, bool L0, bool FIRST, bool STORE>
__device__ __forceinline__ void fwd_cell(const float *__restrict__ lw, int lane, float x0, float x1,
                                         const float (&x)[HS], const float (&hp)[HS], float (&c)[HS],
                                         float (&hout)[HS], f32x4 *gs, f32x2 *cs) {
    constexpr int NX = L0 ? 2 : HS;                 // k-steps over the input
    constexpr int NK = FIRST ? NX : NX + HS;        // k-steps used (h_{t-1} part skipped at t = 0)
    constexpr int QR = (NX + HS + 3) / 4;           // k-quads per fragment row
    constexpr int QN = (NK + 3) / 4;                // k-quads used
#if FCR_FWD_TILE_REGION
    f32x4 qb[2][QN];
#pragma unroll
    for (int qd = 0; qd < QN; ++qd) qb[0][qd] = lds_quad(lw, qd, lane);
    f32x4 prev = {0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
    for (int r = 0; r < HS; ++r) {
        sched_fence();
        if (r + 1 < HS) {
#pragma unroll
            for (int qd = 0; qd < QN; ++qd) qb[(r + 1) & 1][qd] = lds_quad(lw, (r + 1) * QR + qd, lane);
        }
        f32x4 va[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) va[u] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
        for (int s = 0; s < NK; ++s) {
            float bop;
            if (s < NX) bop = L0 ? (s == 0 ? x0 : x1) : x[s < NX ? s : 0];
            else bop = hp[s - NX < HS ? s - NX : 0];
            va[s & 3] = mfma(qb[r & 1][s >> 2][s & 3], bop, va[s & 3]);
        }
        if (r > 0)
            fwd_pointwise<FIRST, STORE>(prev, c[r - 1], hout[r - 1], gs + (r - 1) * kWave,
                                        cs + (r - 1) * kWave, lane);
        prev = (va[0] + va[1]) + (va[2] + va[3]);
    }
#else
    f32x4 cur = lds_quad(lw, 0, lane);
    f32x4 pv[4];   // the previous tile's chains: summed one region later, once their MFMAs have landed
#pragma unroll
    for (int u = 0; u < 4; ++u) pv[u] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
    for (int r = 0; r < HS; ++r) {
        f32x4 va[4];   // FCR_FWD_CHAINS accumulation chains over the k-steps (MFMA dependent latency)
#pragma unroll
        for (int u = 0; u < 4; ++u) va[u] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
        for (int qd = 0; qd < QN; ++qd) {
            sched_fence();
            f32x4 nxt = cur;
            if (qd + 1 < QN) nxt = lds_quad(lw, r * QR + qd + 1, lane);
            else if (r + 1 < HS) nxt = lds_quad(lw, (r + 1) * QR, lane);
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const int s = 4 * qd + e;
                if (s < NK) {
                    float bop;
                    if (s < NX) bop = L0 ? (s == 0 ? x0 : x1) : x[s < NX ? s : 0];
                    else bop = hp[s - NX < HS ? s - NX : 0];
                    va[e % FCR_FWD_CHAINS] = mfma(cur[e], bop, va[e % FCR_FWD_CHAINS]);
                }
            }
            if (qd == 0 && r > 0) {
                const f32x4 prev = FCR_FWD_CHAINS == 4 ? (pv[0] + pv[1]) + (pv[2] + pv[3]) : pv[0] + pv[1];
                fwd_pointwise<FIRST, STORE>(prev, c[r - 1], hout[r - 1], gs + (r - 1) * kWave,
                                            cs + (r - 1) * kWave, lane);
            }
            cur = nxt;
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) pv[u] = va[u];
    }
    const f32x4 prev = FCR_FWD_CHAINS == 4 ? (pv[0] + pv[1]) + (pv[2] + pv[3]) : pv[0] + pv[1];
#endif
    sched_fence();
    fwd_pointwise<FIRST, STORE>(prev, c[HS - 1], hout[HS - 1], gs + (HS - 1) * kWave,
                                cs + (HS - 1) * kWave, lane);
}

__device__ __forceinline__ void rot_left(float (&w)[kL]) {
    const float t0 = w[0];
#pragma unroll
    for (int k = 0; k < kL - 1; ++k) w[k] = w[k + 1];
    w[kL - 1] = t0;
}

// The same cell on the f16 matrix cores (fcr_f16.h): fragments [r][kb][hi|lo][lane][8 halves].
// The B operands (this cell's inputs and h_{t-1}) are split once per cell and shared by all tiles;
// each k-block is its own scheduling region with the next block's two fragment reads in flight.
template <int HS, bool L0, bool FIRST, bool STORE>
__device__ __forceinline__ void fwd16_cell(const float *__restrict__ lw, int lane, float x0, float x1,
                                           const float (&x)[HS], const float (&hp)[HS], float (&c)[HS],
                                           float (&hout)[HS], f32x4 *gs, f32x2 *cs) {
    using G = Geo16<HS>;
    constexpr int KBH = G::KBH;
    constexpr int KB = L0 ? G::KB0 : G::KB1;
    // active k-blocks: at t = 0 the h_{t-1} blocks are all zero
    constexpr int KLO = (L0 && FIRST) ? G::XBLK : 0;
    constexpr int KHI = FIRST ? (L0 ? G::XBLK + 1 : KBH) : KB;
    f16x8 bh[KB], bl[KB];
#pragma unroll
    for (int kb = KLO; kb < KHI; ++kb) {
        float v[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            float e = 0.0f;
            if (L0) {
                const int s = 8 * kb + j;
                if (kb < KBH && s < HS) e = FIRST ? 0.0f : hp[s < HS ? s : 0];
                else if (kb == G::XBLK && j == 5) e = x0;
                else if (kb == G::XBLK && j == 6) e = x1;
            } else if (kb < KBH) {
                const int s = 8 * kb + j;
                if (s < HS) e = x[s < HS ? s : 0];
            } else {
                const int s = 8 * (kb - KBH) + j;
                if (s < HS) e = hp[s < HS ? s : 0];
            }
            v[j] = e;
        }
        split8(v, bh[kb], bl[kb]);
    }
    f16x8 ah = lds_frag16(lw, (0 * KB + KLO) * 2, lane), al = lds_frag16(lw, (0 * KB + KLO) * 2 + 1, lane);
    f32x4 prev = {0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
    for (int r = 0; r < HS; ++r) {
        f32x4 acc = {0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
        for (int kb = KLO; kb < KHI; ++kb) {
            sched_fence();
            f16x8 nh = ah, nl = al;
            if (kb + 1 < KHI) {
                nh = lds_frag16(lw, (r * KB + kb + 1) * 2, lane);
                nl = lds_frag16(lw, (r * KB + kb + 1) * 2 + 1, lane);
            } else if (r + 1 < HS) {
                nh = lds_frag16(lw, ((r + 1) * KB + KLO) * 2, lane);
                nl = lds_frag16(lw, ((r + 1) * KB + KLO) * 2 + 1, lane);
            }
            acc = mma3(ah, al, bh[kb], bl[kb], acc);
            if (kb == KLO && r > 0)
                fwd_pointwise<FIRST, STORE>(prev, c[r - 1], hout[r - 1], gs + (r - 1) * kWave,
                                            cs + (r - 1) * kWave, lane);
            ah = nh;
            al = nl;
        }
        prev = acc;
    }
    sched_fence();
    fwd_pointwise<FIRST, STORE>(prev, c[HS - 1], hout[HS - 1], gs + (HS - 1) * kWave,
                                cs + (HS - 1) * kWave, lane);
}

#if FCR_F16
#define FCR_FWD_CELL fwd16_cell
#define FCR_FGEO Geo16
#else
#define FCR_FWD_CELL fwd_cell
#define FCR_FGEO Geo
#endif

template <int HS, bool STORE>
__global__ __launch_bounds__(kFwdWaves * kWave, kFwdWaves / 4) void fcr_fwd_kernel(FwdArgs a) {
    using G = FCR_FGEO<HS>;
    extern __shared__ __attribute__((aligned(16))) float lw[];
    float *lw0 = lw + G::FA1;                   // resident layer-0 fragments
    float *lfnp = lw0 + G::FA0;                 // resident controller records
    float *lfcp = lfnp + G::FNP;                // resident fc.weight (lane layout) and fc.bias
    float *lfcb = lfcp + G::FCP;
    lds_copy(lw0, a.p.fa[0], G::FA0);
    lds_copy(lfnp, a.p.fnp, G::FNP);
    lds_copy(lfcp, a.p.fcp, G::FCP);
    lds_copy(lfcb, a.p.fcb, 4);
    const int lane = threadIdx.x & 63;
    const int q = lane >> 4, sl = lane & 15;
    // wave-uniform by construction; readfirstlane lets the compiler keep every address base in SGPRs
    const int wave = blockIdx.x * kFwdWaves + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int b = wave * kTile + sl;
    const bool valid = b < a.B;
    const int bc = valid ? b : a.B - 1;   // out-of-range lanes recompute the last trajectory
    const int N = a.N;
    const float alpha = a.alpha;

    const float ref = a.X[(size_t)bc * kCtrlIn + 2];                 // Functions.py:1392
    const float *st = a.states + (size_t)bc * kL * kIn;
    float w0[kL], w1[kL];                                             // window ring, B-operand layout
#pragma unroll
    for (int t = 0; t < kL; ++t) {
        w0[t] = st[t * kIn + q];
        w1[t] = (q == 0) ? st[t * kIn + 4] : 0.0f;
    }
    const float u0 = a.u0[bc];
    if (q == 0) w1[kL - 1] = u0;                                      // Functions.py:1396
    float u_prev = u0;
    float cmd_j = alpha * sq(st[(kL - 2) * kIn + 4] - u0);            // Functions.py:1405
    float cmd_sum = 0.0f, err_sum = 0.0f, tot_sum = 0.0f;
    float xh0 = 0.0f, xh1 = 0.0f, xh2 = 0.0f, xh3 = 0.0f;

    float c[HS], hout[HS], hp[HS], xc[HS], xn[HS];
    const size_t cell = (size_t)HS * kWave;
    const size_t cells_per_wave = (size_t)N * kLayers * kL;
    // h-sequence hand-off slab [wave][j][layer 0|1][t][slot][64]: each address written once, read once
    const size_t qcell = (size_t)Geo<HS>::HQ * kWave;    // one cell of a sequence slab, in quads
    f32x4 *hs_wave = a.hseq + (size_t)wave * N * 2 * kL * qcell;

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
            w0[kL - 1] = sel4(q, xh0, xh1, xh2, xh3);
            w1[kL - 1] = (q == 0) ? un : 0.0f;
            u_prev = un;
            pred = un;
        }
        if (valid && q == 0) a.prediction[(size_t)b * N + j] = pred;   // Functions.py:1455,1466

        f32x4 *gs = a.gates;
        f32x2 *cs = a.cstore;
        if (STORE) {
            const size_t base = ((size_t)wave * cells_per_wave + (size_t)j * kLayers * kL) * cell;
            gs += base;
            cs += base;
        }
#define FCR_G(l, t) (gs + (STORE ? (size_t)((l) * kL + (t)) * cell : 0))
#define FCR_C(l, t) (cs + (STORE ? (size_t)((l) * kL + (t)) * cell : 0))
        f32x4 *hs0 = hs_wave + (size_t)j * 2 * kL * qcell;  // layer-0 outputs, t-major
        f32x4 *hs1 = hs0 + (size_t)kL * qcell;              // layer-1 outputs
        // ---- layer 0 over the window (Functions.py:374) ----
        __syncthreads();   // resident blocks are in place (first window) — no refill for layer 0
        stagger();
        {
            const float x0 = w0[0], x1 = w1[0];
            rot_left(w0);
            rot_left(w1);
            FCR_FWD_CELL<HS, true, true, STORE>(lw0, lane, x0, x1, hp, hp, c, hout, FCR_G(0, 0), FCR_C(0, 0));
            store_quads<HS>(hs0, hout, lane);
#pragma unroll
            for (int r = 0; r < HS; ++r) hp[r] = hout[r];
        }
        for (int t = 1; t < kL; ++t) {
            const float x0 = w0[0], x1 = w1[0];
            rot_left(w0);
            rot_left(w1);
            FCR_FWD_CELL<HS, true, false, STORE>(lw0, lane, x0, x1, hp, hp, c, hout, FCR_G(0, t), FCR_C(0, t));
            store_quads<HS>(hs0 + (size_t)t * qcell, hout, lane);
#pragma unroll
            for (int r = 0; r < HS; ++r) hp[r] = hout[r];
        }
        // ---- layers 1, 2: input sequence streamed back from the slab, one cell ahead ----
#pragma unroll
        for (int l = 1; l < kLayers; ++l) {
            const f32x4 *src = (l == 1) ? hs0 : hs1;
            lds_fill(lw, a.p.fa[l], G::FA1);
            stagger();
            load_quads<HS>(xc, src, lane);
            load_quads<HS>(xn, src + qcell, lane);
            FCR_FWD_CELL<HS, false, true, STORE>(lw, lane, 0.0f, 0.0f, xc, hp, c, hout, FCR_G(l, 0), FCR_C(l, 0));
            if (l == 1) store_quads<HS>(hs1, hout, lane);
#pragma unroll
            for (int r = 0; r < HS; ++r) {
                hp[r] = hout[r];
                xc[r] = xn[r];
            }
            for (int t = 1; t < kL; ++t) {
                load_quads<HS>(xn, src + (size_t)(t + 1 < kL ? t + 1 : t) * qcell, lane);
                FCR_FWD_CELL<HS, false, false, STORE>(lw, lane, 0.0f, 0.0f, xc, hp, c, hout, FCR_G(l, t),
                                                  FCR_C(l, t));
                if (l == 1) store_quads<HS>(hs1 + (size_t)t * qcell, hout, lane);
#pragma unroll
                for (int r = 0; r < HS; ++r) {
                    hp[r] = hout[r];
                    xc[r] = xn[r];
                }
            }
        }
#undef FCR_G
#undef FCR_C
        // ---- readout fc(h_9 of layer 2) (Functions.py:377) ----
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
        if (valid) {
            const float mine = sel4(q, xh0, xh1, xh2, xh3);
            a.xhat_ws[((size_t)b * N + j) * kOut + q] = mine;
            if (a.xhat_user) a.xhat_user[((size_t)b * N + j) * kOut + q] = mine;
        }
        // ---- step cost (Functions.py:1405-1414, 1443-1452) ----
        const float err = sq(xh0 - ref);
        const float con = relu(-xh1) + relu(-xh2) + relu(xh1 - kP1Max) + relu(xh2 - kP2Max);
        tot_sum += (err + cmd_j) + con;
        err_sum += err;
        cmd_sum += cmd_j;
    }
    const float cost = tot_sum / (float)N;                             // Functions.py:1458-1460
    if (valid && q == 0) {
        a.cost[b] = cost;
        a.command[b] = cmd_sum / (float)N;
        a.error[b] = err_sum / (float)N;
    }
    float part = (valid && q == 0) ? cost : 0.0f;                      // per-wave loss partial
#pragma unroll
    for (int m = 1; m < 64; m <<= 1) part += __shfl_xor(part, m);
    if (lane == 0) a.loss_part[wave] = part;
}

}  // namespace fcr
