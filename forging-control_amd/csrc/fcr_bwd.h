// fcr_bwd.h — backward of the rollout (what loss.backward(), Functions.py:655, computes for the
// controller): reverse over windows; per window three layer phases (2 -> 1 -> 0), each reverse over
// t = 9..0 with that layer's transposed MFMA fragments resident in LDS.
//
// Per cell the stored activations (i,f,g,o,c_t) and c_{t-1} come back from HBM one cell ahead of use
// (prefetch into VGPRs; the weights come from LDS on lgkmcnt, so no weight read ever waits behind the
// in-order vmcnt of these HBM loads).
#pragma once
#include "fcr_common.h"

namespace fcr {

// d loss / d (gate pre-activations) of one unit slot, and the carried dc (torch LSTM semantics), from
// the coefficients the forward stored: P = (dh/dc, dh/do_pre, dc/di_pre, dc/df_pre), Q = (dc/dg_pre, f).
__device__ __forceinline__ void cell_grad(const f32x4 P, const f32x2 Q, float dh, float &dc_rec, float &di,
                                          float &df, float &dg, float &dO) {
    const float dc = dc_rec + dh * P[0];
    dO = dh * P[1];
    di = dc * P[2];
    df = dc * P[3];
    dg = dc * Q[0];
    dc_rec = dc * Q[1];
}

// Stored coefficients of one cell — (dh/dc, dh/do, dc/di, dc/df) and (dc/dg, f) per unit slot — and the incoming dh
// from the layer above (dx of layer l+1 at this t, handed over through a per-wave global slab in
// 4-slot quads). A single buffer rolls through the cells: right after slot r of the current cell is
// consumed, slot r of the NEXT cell (in reverse order) is loaded into the same registers, so every HBM
// load is in flight for one cell. Per cell that is 2*HS + ceil(HS/4) loads: within vmcnt's 63.
template <int HS>
struct CellBuf {
    f32x4 g[HS];
    f32x2 cc[HS];
    f32x4 dq[Geo<HS>::HQ];     // din quads (only read by cells whose layer has an input from above)
    __device__ __forceinline__ float din(int r) const { return dq[r >> 2][r & 3]; }
};

struct NextCell {              // where the next cell's data lives
    const f32x4 *g;
    const f32x2 *c;
    const f32x4 *din;          // always a valid address; unused by layer-2 cells
};

// Nothing here may touch the loaded values (a use at load time would make the wave wait for them).
template <int HS>
__device__ __forceinline__ void load_slot(CellBuf<HS> &cb, const NextCell &n, int r, int lane) {
    cb.g[r] = n.g[r * kWave + lane];
    cb.cc[r] = n.c[r * kWave + lane];
    if ((r & 3) == 3 || r == HS - 1) cb.dq[r >> 2] = n.din[(r >> 2) * kWave + lane];   // quad consumed
}

// One backward cell: [dx ; dh_prev] = W^T . dgates over NB output tiles. dh (in: carried dh from
// t+1; out: dh_prev), dc carried in place. The incoming dh from above is cb.din (DIN) or ext.
// L0: outputs dxq (col q) and dx4 (col 4, lane group 0); else dxo (unit slots of the layer-below h).
// lw = transposed fragments [tau][r][lane][gamma]: one ds_read_b128 per output tile and unit slot
// feeds the four gate k-steps. cb holds this cell on entry and the next cell on exit.
template <int HS, bool L0, bool DIN>
__device__ __forceinline__ void bwd_cell(const float *__restrict__ lw, int lane, const float (&ext)[HS],
                                         float (&dh)[HS], float (&dc)[HS], float (&dxo)[HS], float &dxq,
                                         float &dx4, CellBuf<HS> &cb, const NextCell &nx) {
    constexpr int NB = L0 ? Geo<HS>::NB0 : Geo<HS>::NB1;
    f32x4 acc[NB];
#pragma unroll
    for (int k = 0; k < NB; ++k) acc[k] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
#if FCR_BWD_PIPE == 1
    // software pipeline: region r issues slot r's MFMAs while the VALU computes slot r+1's gradients
    // (and its fragment reads land), so the in-order issue never waits on a VALU chain.
    f32x4 w[2][NB];
    float d[2][4];
#pragma unroll
    for (int k = 0; k < NB; ++k) w[0][k] = lds_quad(lw, k * HS, lane);
    cell_grad(cb.g[0], cb.cc[0], dh[0] + (DIN ? cb.din(0) : ext[0]), dc[0], d[0][0], d[0][1],
              d[0][2], d[0][3]);
#pragma unroll
    for (int r = 0; r < HS; ++r) {
        sched_fence();
        const int cu = r & 1, nu = cu ^ 1;
        if (r + 1 < HS) {
#pragma unroll
            for (int k = 0; k < NB; ++k) w[nu][k] = lds_quad(lw, k * HS + r + 1, lane);
            cell_grad(cb.g[r + 1], cb.cc[r + 1], dh[r + 1] + (DIN ? cb.din(r + 1) : ext[r + 1]),
                      dc[r + 1], d[nu][0], d[nu][1], d[nu][2], d[nu][3]);
        }
#pragma unroll
        for (int gm = 0; gm < 4; ++gm)
#pragma unroll
            for (int k = 0; k < NB; ++k) acc[k] = mfma(w[cu][k][gm], d[cu][gm], acc[k]);
        load_slot<HS>(cb, nx, r, lane);
    }
#elif FCR_BWD_PIPE == 2
    // single-buffered pipeline: slot r+1's gradients beside slot r's MFMAs; slot r+1's fragment reads
    // are issued after slot r's last MFMA (fenced), so they can reuse the operand registers.
    f32x4 w[NB];
    float d[4];
#pragma unroll
    for (int k = 0; k < NB; ++k) w[k] = lds_quad(lw, k * HS, lane);
    cell_grad(cb.g[0], cb.cc[0], dh[0] + (DIN ? cb.din(0) : ext[0]), dc[0], d[0], d[1], d[2], d[3]);
#pragma unroll
    for (int r = 0; r < HS; ++r) {
        sched_fence();
        float dn[4] = {0.0f, 0.0f, 0.0f, 0.0f};
        if (r + 1 < HS)
            cell_grad(cb.g[r + 1], cb.cc[r + 1], dh[r + 1] + (DIN ? cb.din(r + 1) : ext[r + 1]), dc[r + 1],
                      dn[0], dn[1], dn[2], dn[3]);
#pragma unroll
        for (int gm = 0; gm < 4; ++gm)
#pragma unroll
            for (int k = 0; k < NB; ++k) acc[k] = mfma(w[k][gm], d[gm], acc[k]);
        sched_fence();
        if (r + 1 < HS) {
#pragma unroll
            for (int k = 0; k < NB; ++k) w[k] = lds_quad(lw, k * HS + r + 1, lane);
        }
        load_slot<HS>(cb, nx, r, lane);
#pragma unroll
        for (int gm = 0; gm < 4; ++gm) d[gm] = dn[gm];
    }
#else
#pragma unroll
    for (int r = 0; r < HS; ++r) {
        sched_fence();
        f32x4 w[NB];   // issued first; the cell-gradient VALU below covers the LDS latency
#pragma unroll
        for (int k = 0; k < NB; ++k) w[k] = lds_quad(lw, k * HS + r, lane);
        float d[4];
        cell_grad(cb.g[r], cb.cc[r], dh[r] + (DIN ? cb.din(r) : ext[r]), dc[r], d[0], d[1],
                  d[2], d[3]);
#pragma unroll
        for (int gm = 0; gm < 4; ++gm)
#pragma unroll
            for (int k = 0; k < NB; ++k) acc[k] = mfma(w[k][gm], d[gm], acc[k]);
        load_slot<HS>(cb, nx, r, lane);
    }
#endif
    sched_fence();
    if (L0) {
#pragma unroll
        for (int s = 0; s < HS; ++s) dh[s] = acc[s >> 2][s & 3];
        dxq = acc[HS >> 2][HS & 3];
        dx4 = acc[(HS + 1) >> 2][(HS + 1) & 3];
    } else {
#pragma unroll
        for (int s = 0; s < HS; ++s) {
            dxo[s] = acc[s >> 2][s & 3];
            dh[s] = acc[(HS + s) >> 2][(HS + s) & 3];
        }
    }
}

template <int HS>
__global__ __launch_bounds__(kBwdWaves * kWave, kBwdWaves / 4) void fcr_bwd_kernel(BwdArgs a) {
    using G = Geo<HS>;
    extern __shared__ __attribute__((aligned(16))) float lw[];
    float *lw0 = lw + G::BA1;                   // resident layer-0 fragments
    float *lfnp = lw0 + G::BA0;                 // resident controller records
    float *lfcp = lfnp + G::FNP;                // resident fc.weight (lane layout)
    lds_copy(lw0, a.p.ba[0], G::BA0);
    lds_copy(lfnp, a.p.fnp, G::FNP);
    lds_copy(lfcp, a.p.fcp, G::FCP);
    __syncthreads();
    const int lane = threadIdx.x & 63;
    const int q = lane >> 4, sl = lane & 15;
    const int wave = blockIdx.x * kBwdWaves + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int b = wave * kTile + sl;
    const bool valid = b < a.B;
    const int bc = valid ? b : a.B - 1;
    const int N = a.N;
    const float alpha = a.alpha;
    // d loss / d (one step-cost term) = dloss / (B N)   (Functions.py:1458, 1463)
    const float wgt = valid ? a.dloss[0] / ((float)a.B * (float)N) : 0.0f;
    const float ref = a.X[(size_t)bc * kCtrlIn + 2];
    const float s84 = a.states[(size_t)bc * kL * kIn + (kL - 2) * kIn + 4];
    const float *pred = a.prediction + (size_t)bc * N;
    const float *xh = a.xhat + (size_t)bc * N * kOut;

    // window-row gradients dx(w, t) (lane group q: column q; lane group 0 also column 4) go to a
    // per-wave slab; row rho = w + t of the extended sequence sums the windows that contained it.
    f32x2 *dxr = a.dxrow + (size_t)wave * N * kL * kWave;
    auto row_grad = [&](int rho) {   // sum over windows w = max(0, rho-9) .. min(N-1, rho) of dx(w, rho-w)
        f32x2 acc2 = {0.0f, 0.0f};
        const int w_hi = rho < N - 1 ? rho : N - 1;
        const int w_lo = rho - (kL - 1) > 0 ? rho - (kL - 1) : 0;
        for (int w = w_hi; w >= w_lo; --w) acc2 += dxr[((size_t)w * kL + (rho - w)) * kWave + lane];
        return acc2;
    };
    float dh[HS], dc[HS], dxo[HS], dab[HS];

    const size_t cell = (size_t)HS * kWave;
    const size_t wave_base = (size_t)wave * N * kLayers * kL * cell;
    const size_t qcell = (size_t)Geo<HS>::HQ * kWave;   // one cell of the dx slab, in quads
    const size_t seq_base = (size_t)wave * N * 2 * kL * qcell;
    // stored activations of cell (j, l, t); dx handed from layer src+... : slab (j, l_from, t), l_from = 2 or 1
    auto gcell = [&](int j, int l, int t) { return wave_base + ((size_t)(j * kLayers + l) * kL + t) * cell; };
    auto scell = [&](int j, int lfrom, int t) { return seq_base + ((size_t)(j * 2 + (2 - lfrom)) * kL + t) * qcell; };
    auto next_of = [&](int j, int l, int t) {   // the cell processed after (j, l, t)
        NextCell n;
        int nj = j, nl = l, nt = t - 1;
        if (t == 0) {
            nt = kL - 1;
            nl = l - 1;
            if (l == 0) { nl = 2; nj = j - 1; }
        }
        if (nj < 0) { nj = 0; nl = 0; nt = 0; }   // past the last cell: reload it (harmless)
        const size_t gb = gcell(nj, nl, nt);
        n.g = a.gates + gb;
        n.c = a.cstore + gb;
        n.din = a.dseq + (nl < 2 ? scell(nj, nl + 1, nt) : seq_base);
        return n;
    };
    CellBuf<HS> cb;
    {
        NextCell first = next_of(N - 1, 2, kL);   // t = kL -> (N-1, 2, 9)
#pragma unroll
        for (int r = 0; r < HS; ++r) load_slot<HS>(cb, first, r, lane);
    }

    for (int j = N - 1; j >= 0; --j) {
        const float *lfnp_j = opaque(lfnp), *lfcp_j = opaque(lfcp);
        const float x0 = xh[j * kOut + 0], x1 = xh[j * kOut + 1], x2 = xh[j * kOut + 2],
                    x3 = xh[j * kOut + 3];
        // direct cost gradients of step j (Functions.py:1443-1452)
        float d0 = wgt * 2.0f * (x0 - ref);
        float d1 = wgt * ((-x1 > 0.0f ? -1.0f : 0.0f) + (x1 - kP1Max > 0.0f ? 1.0f : 0.0f));
        float d2 = wgt * ((-x2 > 0.0f ? -1.0f : 0.0f) + (x2 - kP2Max > 0.0f ? 1.0f : 0.0f));
        float d3 = 0.0f;
        if (j <= N - 2) {
            // row 10+j = (xhat_j, u_{j+1}) is complete once windows j+1 .. j+10 are done
            const f32x2 G = row_grad(kL + j);   // row 10+j = (xhat_j, u_{j+1})
            d0 += __shfl(G[0], sl);
            d1 += __shfl(G[0], sl + 16);
            d2 += __shfl(G[0], sl + 32);
            d3 += __shfl(G[0], sl + 48);
            const float g4 = __shfl(G[1], sl);
            const float uj = pred[j], uj1 = pred[j + 1];
            float du = 2.0f * alpha * wgt * (uj1 - uj);                       // cmd_{j+1}
            if (j + 2 < N) du += 2.0f * alpha * wgt * (uj1 - pred[j + 2]);    // cmd_{j+2}
            du += g4;
            // controller backward at (xhat_j[0], xhat_j[3], ref) (Functions.py:1424-1430)
            float z[kMS];
            const float v = fnn_pre(lfnp_j, q, x0, x3, ref, z);
            const float dv = (v > -1.0f && v < 1.0f) ? du : 0.0f;            // Hardtanh'
            float dca = 0.0f, dcb = 0.0f;
#pragma unroll
            for (int m = 0; m < kMS; ++m) {
                const float *p = lfnp_j + (m * 4 + q) * kFnpStride;
                const float dz = (z[m] > 0.0f) ? dv * p[4] : 0.0f;               // ReLU'
                dca += dz * p[0];
                dcb += dz * p[1];
            }
            // the controller's parameter gradients are finished by ctrl_grad_kernel from dv
            if (valid && q == 0) a.dv[(size_t)b * N + j] = dv;
            d0 += xor_sum_q(dca);
            d3 += xor_sum_q(dcb);
        } else if (valid && q == 0) {
            a.dv[(size_t)b * N + j] = 0.0f;   // the last step feeds no controller call
        }
        // ---- layer 2: dh_9 = fc.W^T dxhat (Functions.py:377) ----
        float dh_out[HS];
#pragma unroll
        for (int r = 0; r < HS; ++r) {
            const float *fp = lfcp_j + r * 4 + q;
            dh_out[r] = fp[0] * d0 + fp[HS * 4] * d1 + fp[2 * HS * 4] * d2 + fp[3 * HS * 4] * d3;
        }
        float unused0, unused1;
        lds_fill(lw, a.p.ba[2], G::BA1);
        stagger();
#pragma unroll
        for (int r = 0; r < HS; ++r) dh[r] = dc[r] = 0.0f;
        for (int t = kL - 1; t >= 0; --t) {
#pragma unroll
            for (int r = 0; r < HS; ++r) dab[r] = (t == kL - 1) ? dh_out[r] : 0.0f;
            bwd_cell<HS, false, false>(lw, lane, dab, dh, dc, dxo, unused0, unused1, cb, next_of(j, 2, t));
            store_quads<HS>(a.dseq + scell(j, 2, t), dxo, lane);
        }
        // ---- layer 1 ----
        lds_fill(lw, a.p.ba[1], G::BA1);
        stagger();
#pragma unroll
        for (int r = 0; r < HS; ++r) dh[r] = dc[r] = 0.0f;
        for (int t = kL - 1; t >= 0; --t) {
            bwd_cell<HS, false, true>(lw, lane, dab, dh, dc, dxo, unused0, unused1, cb, next_of(j, 1, t));
            store_quads<HS>(a.dseq + scell(j, 1, t), dxo, lane);
        }
        // ---- layer 0: dx -> window-row gradients ----
#pragma unroll
        for (int r = 0; r < HS; ++r) dh[r] = dc[r] = 0.0f;
        for (int t = kL - 1; t >= 0; --t) {
            float dxq, dx4;
            bwd_cell<HS, true, true>(lw0, lane, dab, dh, dc, dxo, dxq, dx4, cb, next_of(j, 0, t));
            dxr[((size_t)j * kL + t) * kWave + lane] = f32x2{dxq, dx4};   // row j+t
        }
    }
    const float g_u0_rows = row_grad(kL - 1)[1];   // row 9, col 4 = u0 (Functions.py:1396)
    // command-cost terms of u0: cmd_0 = a(s84 - u0)^2, cmd_1 = a(u0 - u1)^2
    float du0 = 2.0f * alpha * wgt * (pred[0] - s84);
    if (N > 1) du0 += 2.0f * alpha * wgt * (pred[0] - pred[1]);
    if (valid && q == 0) a.g_u0[b] = g_u0_rows + du0;
}

}  // namespace fcr
