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

// d loss / d (gate pre-activations) of one unit slot, and the carried dc (torch LSTM semantics).
__device__ __forceinline__ void cell_grad(const f32x4 g, float ct, float cp, float dh, float &dc_rec,
                                          float &di, float &df, float &dg, float &dO) {
    const float i = g[0], f = g[1], gg = g[2], o = g[3];
    const float tc = tanh_f(ct);
    const float dc = dc_rec + dh * o * (1.0f - tc * tc);
    di = dc * gg * i * (1.0f - i);
    df = dc * cp * f * (1.0f - f);
    dg = dc * i * (1.0f - gg * gg);
    dO = dh * tc * o * (1.0f - o);
    dc_rec = dc * f;
}

// Stored activations of one cell (i,f,g,o, c_t), c_{t-1}, and the incoming dh from the layer above
// (dx of layer l+1 at this t, handed over through a per-wave global slab). A single buffer rolls
// through the cells: right after slot r of the current cell is consumed, slot r of the NEXT cell (in
// reverse order) is loaded into the same registers, so every HBM load is in flight for one cell.
template <int HS>
struct CellBuf {
    f32x4 g[HS];
    float ct[HS], cp[HS], din[HS];
};

struct NextCell {              // where the next cell's data lives
    const f32x4 *g;
    const float *c;
    const float *din;
    bool prev, has_din;
};

template <int HS>
__device__ __forceinline__ void load_slot(CellBuf<HS> &cb, const NextCell &n, int r, int lane) {
    const float *pc = n.prev ? n.c - (size_t)HS * kWave : n.c;   // keep addresses valid when unused
    cb.g[r] = n.g[r * kWave + lane];
    cb.ct[r] = n.c[r * kWave + lane];
    const float v = pc[r * kWave + lane];
    cb.cp[r] = n.prev ? v : 0.0f;
    const float dv = __builtin_nontemporal_load(n.din + r * kWave + lane);
    cb.din[r] = n.has_din ? dv : 0.0f;
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
#pragma unroll
    for (int r = 0; r < HS; ++r) {
        sched_fence();
        f32x4 w[NB];   // issued first; the cell-gradient VALU below covers the LDS latency
#pragma unroll
        for (int k = 0; k < NB; ++k) w[k] = lds_quad(lw, k * HS + r, lane);
        float d[4];
        cell_grad(cb.g[r], cb.ct[r], cb.cp[r], dh[r] + (DIN ? cb.din[r] : ext[r]), dc[r], d[0], d[1],
                  d[2], d[3]);
#pragma unroll
        for (int gm = 0; gm < 4; ++gm)
#pragma unroll
            for (int k = 0; k < NB; ++k) acc[k] = mfma(w[k][gm], d[gm], acc[k]);
        load_slot<HS>(cb, nx, r, lane);
    }
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

// Reduce-scatter of 80 per-lane values over the 16 trajectory lanes (xor 8,4,2,1): afterwards lane
// sl holds the sums of values 5*sl .. 5*sl+4 (controller unit m = sl, params p = 0..4).
__device__ __forceinline__ void reduce_scatter16(float (&v)[80], int sl, float (&out)[5]) {
#pragma unroll
    for (int i = 0; i < 40; ++i) {
        const bool hi = sl & 8;
        const float keep = hi ? v[i + 40] : v[i], send = hi ? v[i] : v[i + 40];
        v[i] = keep + __shfl_xor(send, 8);
    }
#pragma unroll
    for (int i = 0; i < 20; ++i) {
        const bool hi = sl & 4;
        const float keep = hi ? v[i + 20] : v[i], send = hi ? v[i] : v[i + 20];
        v[i] = keep + __shfl_xor(send, 4);
    }
#pragma unroll
    for (int i = 0; i < 10; ++i) {
        const bool hi = sl & 2;
        const float keep = hi ? v[i + 10] : v[i], send = hi ? v[i] : v[i + 10];
        v[i] = keep + __shfl_xor(send, 2);
    }
#pragma unroll
    for (int i = 0; i < 5; ++i) {
        const bool hi = sl & 1;
        const float keep = hi ? v[i + 5] : v[i], send = hi ? v[i] : v[i + 5];
        out[i] += keep + __shfl_xor(send, 1);
    }
}

__device__ __forceinline__ void rot_right(float (&w)[kL]) {
    const float t9 = w[kL - 1];
#pragma unroll
    for (int k = kL - 1; k > 0; --k) w[k] = w[k - 1];
    w[0] = t9;
}

template <int HS>
__global__ __launch_bounds__(kBwdWaves * kWave, 1) void fcr_bwd_kernel(BwdArgs a) {
    using G = Geo<HS>;
    extern __shared__ __attribute__((aligned(16))) float lw[];
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

    float Ra[kL], Rb[kL];     // window-row gradient ring (lane group q: col q; group 0 also col 4)
#pragma unroll
    for (int t = 0; t < kL; ++t) Ra[t] = Rb[t] = 0.0f;
    float Gq = 0.0f, G4 = 0.0f;   // completed gradient of row 10+j
    float g_u0_rows = 0.0f;
    float facc[5] = {0.0f, 0.0f, 0.0f, 0.0f, 0.0f};
    float dh[HS], dc[HS], dxo[HS], dab[HS];

    const size_t cell = (size_t)HS * kWave;
    const size_t wave_base = (size_t)wave * N * kLayers * kL * cell;
    const size_t seq_base = (size_t)wave * N * 2 * kL * cell;
    // stored activations of cell (j, l, t); dx handed from layer src+... : slab (j, l_from, t), l_from = 2 or 1
    auto gcell = [&](int j, int l, int t) { return wave_base + ((size_t)(j * kLayers + l) * kL + t) * cell; };
    auto scell = [&](int j, int lfrom, int t) { return seq_base + ((size_t)(j * 2 + (2 - lfrom)) * kL + t) * cell; };
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
        n.prev = nt > 0;
        n.has_din = nl < 2;
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
        const float x0 = xh[j * kOut + 0], x1 = xh[j * kOut + 1], x2 = xh[j * kOut + 2],
                    x3 = xh[j * kOut + 3];
        // direct cost gradients of step j (Functions.py:1443-1452)
        float d0 = wgt * 2.0f * (x0 - ref);
        float d1 = wgt * ((-x1 > 0.0f ? -1.0f : 0.0f) + (x1 - kP1Max > 0.0f ? 1.0f : 0.0f));
        float d2 = wgt * ((-x2 > 0.0f ? -1.0f : 0.0f) + (x2 - kP2Max > 0.0f ? 1.0f : 0.0f));
        float d3 = 0.0f;
        if (j <= N - 2) {
            // row 10+j = (xhat_j, u_{j+1}) is complete once windows j+1 .. j+10 are done
            d0 += __shfl(Gq, sl);
            d1 += __shfl(Gq, sl + 16);
            d2 += __shfl(Gq, sl + 32);
            d3 += __shfl(Gq, sl + 48);
            const float g4 = __shfl(G4, sl);
            const float uj = pred[j], uj1 = pred[j + 1];
            float du = 2.0f * alpha * wgt * (uj1 - uj);                       // cmd_{j+1}
            if (j + 2 < N) du += 2.0f * alpha * wgt * (uj1 - pred[j + 2]);    // cmd_{j+2}
            du += g4;
            // controller backward at (xhat_j[0], xhat_j[3], ref) (Functions.py:1424-1430)
            float z[kMS];
            const float v = fnn_pre(a.p.fnp, q, x0, x3, ref, z);
            const float dv = (v > -1.0f && v < 1.0f) ? du : 0.0f;            // Hardtanh'
            float vals[80];
            float dca = 0.0f, dcb = 0.0f;
#pragma unroll
            for (int m = 0; m < kMS; ++m) {
                const float *p = a.p.fnp + (m * 4 + q) * kFnpStride;
                const float dz = (z[m] > 0.0f) ? dv * p[4] : 0.0f;               // ReLU'
                vals[m * 5 + 0] = dz * x0;
                vals[m * 5 + 1] = dz * x3;
                vals[m * 5 + 2] = dz * ref;
                vals[m * 5 + 3] = dz;
                vals[m * 5 + 4] = dv * relu(z[m]);
                dca += dz * p[0];
                dcb += dz * p[1];
            }
#pragma unroll
            for (int i = kMS * 5; i < 80; ++i) vals[i] = 0.0f;
            reduce_scatter16(vals, sl, facc);
            d0 += xor_sum_q(dca);
            d3 += xor_sum_q(dcb);
        }
        // ---- layer 2: dh_9 = fc.W^T dxhat (Functions.py:377) ----
        float dh_out[HS];
#pragma unroll
        for (int r = 0; r < HS; ++r) {
            const float *fp = a.p.fcp + r * 4 + q;
            dh_out[r] = fp[0] * d0 + fp[HS * 4] * d1 + fp[2 * HS * 4] * d2 + fp[3 * HS * 4] * d3;
        }
        float unused0, unused1;
        lds_fill(lw, a.p.ba[2], G::BA1);
#pragma unroll
        for (int r = 0; r < HS; ++r) dh[r] = dc[r] = 0.0f;
        for (int t = kL - 1; t >= 0; --t) {
#pragma unroll
            for (int r = 0; r < HS; ++r) dab[r] = (t == kL - 1) ? dh_out[r] : 0.0f;
            bwd_cell<HS, false, false>(lw, lane, dab, dh, dc, dxo, unused0, unused1, cb, next_of(j, 2, t));
            float *dst = a.dseq + scell(j, 2, t);
#pragma unroll
            for (int r = 0; r < HS; ++r) dst[r * kWave + lane] = dxo[r];
        }
        // ---- layer 1 ----
        lds_fill(lw, a.p.ba[1], G::BA1);
#pragma unroll
        for (int r = 0; r < HS; ++r) dh[r] = dc[r] = 0.0f;
        for (int t = kL - 1; t >= 0; --t) {
            bwd_cell<HS, false, true>(lw, lane, dab, dh, dc, dxo, unused0, unused1, cb, next_of(j, 1, t));
            float *dst = a.dseq + scell(j, 1, t);
#pragma unroll
            for (int r = 0; r < HS; ++r) dst[r * kWave + lane] = dxo[r];
        }
        // ---- layer 0: dx -> window-row gradients ----
        lds_fill(lw, a.p.ba[0], G::BA0);
#pragma unroll
        for (int r = 0; r < HS; ++r) dh[r] = dc[r] = 0.0f;
        for (int t = kL - 1; t >= 0; --t) {
            float dxq, dx4;
            bwd_cell<HS, true, true>(lw, lane, dab, dh, dc, dxo, dxq, dx4, cb, next_of(j, 0, t));
            Ra[kL - 1] += dxq;   // row j+t of the extended sequence
            Rb[kL - 1] += dx4;
            rot_right(Ra);
            rot_right(Rb);
        }
        // row j+9 leaves the ring complete; shift the ring to window j-1
        const float outa = Ra[kL - 1], outb = Rb[kL - 1];
#pragma unroll
        for (int k = kL - 1; k > 0; --k) {
            Ra[k] = Ra[k - 1];
            Rb[k] = Rb[k - 1];
        }
        Ra[0] = Rb[0] = 0.0f;
        if (j > 0) {
            Gq = outa;
            G4 = outb;
        } else {
            g_u0_rows = outb;   // row 9, col 4 = u0 (Functions.py:1396)
        }
    }
    // command-cost terms of u0: cmd_0 = a(s84 - u0)^2, cmd_1 = a(u0 - u1)^2
    float du0 = 2.0f * alpha * wgt * (pred[0] - s84);
    if (N > 1) du0 += 2.0f * alpha * wgt * (pred[0] - pred[1]);
    if (valid && q == 0) a.g_u0[b] = g_u0_rows + du0;
    // controller parameter partials of this wave: unit k = 4*sl + q, params (W0, W1, W2, b, wout)
    const int k = 4 * sl + q;
    if (sl < kMS && k < a.hidden) {
        float *dst = a.fnn_part + ((size_t)wave * a.hidden + k) * 5;
#pragma unroll
        for (int p = 0; p < 5; ++p) dst[p] = facc[p];
    }
}

}  // namespace fcr
