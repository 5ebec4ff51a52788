// fcr_bwd.h — backward of the rollout (what loss.backward(), Functions.py:655, computes for the
// controller): reverse over windows; per window three layer phases (2 -> 1 -> 0), each reverse over
// t = 9..0 with that layer's transposed MFMA fragments resident in LDS.
//
// Per cell the stored activations (i,f,g,o,c_t) and c_{t-1} come back from HBM one cell ahead of use
// (prefetch into VGPRs; the weights come from LDS on lgkmcnt, so no weight read ever waits behind the
// in-order vmcnt of these HBM loads).
#pragma once
#include "fcr_common.h"
#include "fcr_f16.h"

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

// Where the next cell's data lives: buffer descriptors over this wave's own regions (wave-uniform,
// SGPRs) and the cell's byte offsets in them (SGPRs), so every load's address is one shared lane
// offset VGPR — no 64-bit address pairs per slot for the compiler to keep live.
struct NextCell {
    __amdgpu_buffer_rsrc_t rg, rc, rd;   // gates (P), cstore (Q), dseq (din) regions of this wave
    uint32_t g, c, din;                  // byte offsets of the cell; din always valid (layer 2 ignores it)
    bool ld_din;                         // the cell reads a din (layers 0, 1): only then fetch it — a
                                         // fetched-but-unused register is reused at once, i.e. waited for
};

// Nothing here may touch the loaded values (a use at load time would make the wave wait for them).
template <int HS, bool DQ = true>
__device__ __forceinline__ void load_slot(CellBuf<HS> &cb, const NextCell &n, int r, int lane) {
    cb.g[r] = buf_ld4(n.rg, lane * 16, n.g + r * kWave * 16);
    cb.cc[r] = buf_ld2(n.rc, lane * 8, n.c + r * kWave * 8);
    if (DQ && ((r & 3) == 3 || r == HS - 1))   // quad consumed
        cb.dq[r >> 2] = buf_ld4(n.rd, lane * 16, n.din + (r >> 2) * kWave * 16);
}
template <int HS>
__device__ __forceinline__ void load_din(CellBuf<HS> &cb, const NextCell &n, int lane) {
#pragma unroll
    for (int k = 0; k < Geo<HS>::HQ; ++k) cb.dq[k] = buf_ld4(n.rd, lane * 16, n.din + k * kWave * 16);
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

// The same cell on the f16 matrix cores (fcr_f16.h). k-block kb = unit slots 2kb, 2kb+1 x gates; the
// lane's own dgates of those slots are its B operand, so no data moves between lanes. The dgates of a
// trajectory are scaled by 2^(13-e) (e = exponent of the largest |dh|+|dc| over its slots, which bounds
// every dgate) before the hi/lo split, and the products scaled back: both exact powers of two.
// Region kb issues block kb's MFMAs beside the VALU work of block kb+1 (gradients, scale, split).
#ifndef FCR_B16_AT
#define FCR_B16_AT 0      // tile step of region kb that builds block kb+1's operands
#endif
#ifndef FCR_B16_FINE
#define FCR_B16_FINE 1    // one scheduling region per (kb, tile) instead of per kb
#endif
template <int HS, bool L0, bool DIN>
__device__ __forceinline__ void bwd16_cell(const float *__restrict__ lw, int lane, const float (&ext)[HS],
                                           float (&dh)[HS], float (&dc)[HS], float (&dxo)[HS], float &dxq,
                                           float &dx4, CellBuf<HS> &cb, const NextCell &nx) {
    using G = Geo16<HS>;
    constexpr int NB = L0 ? G::NB0 : G::NB1;
    constexpr int KBB = G::KBB;
    float m = 0.0f;
#pragma unroll
    for (int r = 0; r < HS; ++r) {
        dh[r] += DIN ? cb.din(r) : ext[r];
        m = fmaxf(m, fabsf(dh[r]) + fabsf(dc[r]));
    }
    // every din is consumed: the next cell's come in now, a whole cell ahead of the wait for them
    if (nx.ld_din) load_din<HS>(cb, nx, lane);
    m = fmaxf(m, __shfl_xor(m, 16));
    m = fmaxf(m, __shfl_xor(m, 32));
    const int e = max(__builtin_amdgcn_frexp_expf(m), -100);   // m < 2^e; all-zero -> e = 0
    const float up = __builtin_amdgcn_ldexpf(1.0f, 13 - e), down = __builtin_amdgcn_ldexpf(1.0f, e - 13);
    // B operand of block kb: scaled dgates of slots 2kb, 2kb+1 (j = 4*(slot&1) + gate)
    auto block = [&](int kb, f16x8 &bh, f16x8 &bl) {
        float v[8];
#pragma unroll
        for (int u = 0; u < 2; ++u) {
            const int r = 2 * kb + u;
            if (r < HS) {
                float dcs = dc[r] * up;
                cell_grad(cb.g[r], cb.cc[r], dh[r] * up, dcs, v[4 * u], v[4 * u + 1], v[4 * u + 2], v[4 * u + 3]);
                dc[r] = dcs * down;
            } else {
                v[4 * u] = v[4 * u + 1] = v[4 * u + 2] = v[4 * u + 3] = 0.0f;
            }
        }
        split8(v, bh, bl);
    };
    f32x4 acc[NB];
#pragma unroll
    for (int k = 0; k < NB; ++k) acc[k] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
    f16x8 bh[2], bl[2];
    block(0, bh[0], bl[0]);
    f16x8 ah = lds_frag16(lw, 0, lane), al = lds_frag16(lw, 1, lane);
#pragma unroll
    for (int kb = 0; kb < KBB; ++kb) {
        const int cu = kb & 1, nu = cu ^ 1;
#pragma unroll
        for (int t = 0; t < NB; ++t) {
            // one scheduling region per (kb, tile): fragment (t, kb) is in (ah, al); the next one in
            // (tau, kb) order is fetched beside its MFMAs, and block kb+1 is built in the first region
            if (FCR_B16_FINE || t == 0) sched_fence();
            f16x8 nh = ah, nl = al;
            const int nt = t + 1 < NB ? t + 1 : 0, nk = t + 1 < NB ? kb : kb + 1;
            if (nk < KBB) {
                nh = lds_frag16(lw, (nt * KBB + nk) * 2, lane);
                nl = lds_frag16(lw, (nt * KBB + nk) * 2 + 1, lane);
            }
            if (t == (FCR_B16_AT < NB ? FCR_B16_AT : NB - 1) && kb + 1 < KBB) block(kb + 1, bh[nu], bl[nu]);
            // the products only feed the cell's outputs, so IR passes would sink every MFMA to the
            // end of the cell (all fragments live at once); naming the accumulator here keeps block
            // kb-1's MFMAs ahead of this point (issued ~NB*3 MFMAs ago: no hazard wait)
            if (kb > 0) asm volatile("" : "+v"(acc[t]));
            acc[t] = mma3(ah, al, bh[cu], bl[cu], acc[t]);
            ah = nh;
            al = nl;
        }
        // slots 2kb+2, 2kb+3 were consumed by block(kb+1): their next-cell records may load now
#pragma unroll
        for (int u = 0; u < 2; ++u) {
            const int r = 2 * (kb + 1) + u;
            if (kb == 0 && u == 0) {
                load_slot<HS, false>(cb, nx, 0, lane);
                load_slot<HS, false>(cb, nx, 1, lane);
            }
            if (r < HS) load_slot<HS, false>(cb, nx, r, lane);
        }
    }
    sched_fence();
    if (L0) {
#pragma unroll
        for (int s = 0; s < HS; ++s) dh[s] = acc[s >> 2][s & 3] * down;
        dxq = acc[HS >> 2][HS & 3] * down;
        dx4 = acc[(HS + 1) >> 2][(HS + 1) & 3] * down;
    } else {
#pragma unroll
        for (int s = 0; s < HS; ++s) {
            dxo[s] = acc[s >> 2][s & 3] * down;
            dh[s] = acc[(HS + s) >> 2][(HS + s) & 3] * down;
        }
    }
}

#if FCR_F16
#define FCR_BWD_CELL bwd16_cell
#define FCR_BGEO Geo16
#else
#define FCR_BWD_CELL bwd_cell
#define FCR_BGEO Geo
#endif

template <int HS>
__global__ __launch_bounds__(kBwdWaves * kWave, kBwdWaves / 4) void fcr_bwd_kernel(BwdArgs a) {
    using G = FCR_BGEO<HS>;
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
    const __amdgpu_buffer_rsrc_t rx = wave_rsrc(a.dxrow + (size_t)wave * N * kL * kWave, (size_t)N * kL * kWave * 8);
    auto row_grad = [&](int rho) {   // sum over windows w = max(0, rho-9) .. min(N-1, rho) of dx(w, rho-w)
        f32x2 acc2 = {0.0f, 0.0f};
        const int w_hi = rho < N - 1 ? rho : N - 1;
        const int w_lo = rho - (kL - 1) > 0 ? rho - (kL - 1) : 0;
        for (int w = w_hi; w >= w_lo; --w) acc2 += buf_ld2(rx, lane * 8, (uint32_t)((w * kL + (rho - w)) * kWave * 8));
        return acc2;
    };
    float dh[HS], dc[HS], dxo[HS], dab[HS];

    const size_t cell = (size_t)HS * kWave;
    const size_t wave_base = (size_t)wave * N * kLayers * kL * cell;
    const size_t qcell = (size_t)Geo<HS>::HQ * kWave;   // one cell of the dx slab, in quads
    const size_t seq_base = (size_t)wave * N * 2 * kL * qcell;
    // stored activations of cell (j, l, t); dx handed from layer src+... : slab (j, l_from, t), l_from = 2 or 1
    // cell offsets inside this wave's regions (elements), and the absolute slab cell for stores
    auto gcell = [&](int j, int l, int t) { return ((size_t)(j * kLayers + l) * kL + t) * cell; };
    auto srel = [&](int j, int lfrom, int t) { return ((size_t)(j * 2 + (2 - lfrom)) * kL + t) * qcell; };
    const size_t wave_cells = (size_t)N * kLayers * kL * cell;
    const __amdgpu_buffer_rsrc_t rg = wave_rsrc(a.gates + wave_base, wave_cells * 16);
    const __amdgpu_buffer_rsrc_t rc = wave_rsrc(a.cstore + wave_base, wave_cells * 8);
    const __amdgpu_buffer_rsrc_t rd = wave_rsrc(a.dseq + seq_base, (size_t)N * 2 * kL * qcell * 16);
    auto next_of = [&](int j, int l, int t) {   // the cell processed after (j, l, t)
        NextCell n;
        n.rg = rg;
        n.rc = rc;
        n.rd = rd;
        int nj = j, nl = l, nt = t - 1;
        if (t == 0) {
            nt = kL - 1;
            nl = l - 1;
            if (l == 0) { nl = 2; nj = j - 1; }
        }
        if (nj < 0) { nj = 0; nl = 0; nt = 0; }   // past the last cell: reload it (harmless)
        const size_t gb = gcell(nj, nl, nt);
        n.g = (uint32_t)(gb * 16);
        n.c = (uint32_t)(gb * 8);
        n.din = (uint32_t)((nl < 2 ? srel(nj, nl + 1, nt) : 0) * 16);
        n.ld_din = nl < 2;
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
            FCR_BWD_CELL<HS, false, false>(lw, lane, dab, dh, dc, dxo, unused0, unused1, cb, next_of(j, 2, t));
            store_quads<HS>(a.dseq + seq_base + srel(j, 2, t), dxo, lane);
        }
        // ---- layer 1 ----
        lds_fill(lw, a.p.ba[1], G::BA1);
        stagger();
#pragma unroll
        for (int r = 0; r < HS; ++r) dh[r] = dc[r] = 0.0f;
        for (int t = kL - 1; t >= 0; --t) {
            FCR_BWD_CELL<HS, false, true>(lw, lane, dab, dh, dc, dxo, unused0, unused1, cb, next_of(j, 1, t));
            store_quads<HS>(a.dseq + seq_base + srel(j, 1, t), dxo, lane);
        }
        // ---- layer 0: dx -> window-row gradients ----
#pragma unroll
        for (int r = 0; r < HS; ++r) dh[r] = dc[r] = 0.0f;
        for (int t = kL - 1; t >= 0; --t) {
            float dxq, dx4;
            FCR_BWD_CELL<HS, true, true>(lw0, lane, dab, dh, dc, dxo, dxq, dx4, cb, next_of(j, 0, t));
            buf_st2(rx, lane * 8, (uint32_t)((j * kL + t) * kWave * 8), f32x2{dxq, dx4});   // row j+t
        }
    }
    const float g_u0_rows = row_grad(kL - 1)[1];   // row 9, col 4 = u0 (Functions.py:1396)
    // command-cost terms of u0: cmd_0 = a(s84 - u0)^2, cmd_1 = a(u0 - u1)^2
    float du0 = 2.0f * alpha * wgt * (pred[0] - s84);
    if (N > 1) du0 += 2.0f * alpha * wgt * (pred[0] - pred[1]);
    if (valid && q == 0) a.g_u0[b] = g_u0_rows + du0;
}

}  // namespace fcr
