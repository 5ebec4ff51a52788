// fcr_sur.h — the LSTM surrogate's training step on the rollout's fused split-f16 kernels,
// H <= 52: LSTMModel(5, H, 4, 3) forward on a (B, 10, 5) window batch and the gradient of EVERY weight
// (Model_NN/Functions.py:520-569 driven by Model_NN/Main.py:218-242; the model is Functions.py:255-330).
//
// A window batch is the rollout's window 0 with the rows given instead of generated, so the two cell loops are the
// rollout's (fcr_fwd.h fwd16_cell, fcr_bwd.h bwd_cell) over one window, with the same packed fragments and weight
// images (fcr_f16.h, fcr_img.h) and the same range guard on the window columns (fcr_pack.h):
//   sur_fwd_kernel    3 layer phases x 10 cells per wave of 16 windows; keeps h (split records), c and the window
//                     rows like the rollout's forward; y = fc(h_9 of layer 2) and h_9 (fp32, the readout's gradient).
//   sur_bwd_kernel    dh_9 = fc.W^T dy, then the rollout's recompute-in-backward cells (layers 2, 1, 0), each of
//                     which also stores its scaled dgate blocks and its per-trajectory unscaling factor (DgOut);
//                     the window-row gradients are dL/dx when the caller asks for them.
//   sur_wgrad_kernel  the weight gradients of one layer, dW = sum over (window, step) of dgates^T [x_t | h_{t-1}]: a
//                     split-K product over k-blocks of 64 rows (16 windows x 2 steps of two backward waves), the
//                     dgates re-scaled per row and re-split, both operands read transposed (ds_read_b64_tr_b16)
//                     from a natural row layout in LDS, v_mfma_f32_16x16x32_f16 into per-workgroup partials.
//   sur_part_sum_kernel, sur_wgrad_finish_kernel  the fixed-order sum of the partials, decoded into the W_ih / W_hh
//                     gradients (deterministic).
#pragma once
#include "fcr_bwd.h"
#include "fcr_fwd.h"

namespace fcr {

struct SurArgs {
    int B, H;
    const float *x;      // (B, 10, 5) windows, batch-first (Model_NN/Functions.py:328)
    float *y;            // (B, 4)
    float *htop;         // (B, H): h_9 of layer 2, fp32 (the readout's weight gradient)
    f32x4 *hseq, *cseq;  // [wave][layer][t][record]: h (split records) and c of every cell
    f32x2 *xw;           // [wave][t][64]: the range-guarded window rows (column q, column 4)
    const float *dy;     // (B, 4) = dL/dy
    float *g_x;          // (B, 10, 5) = dL/dx, or null
    f32x4 *dseq;         // [wave][2][t][record]: dx of layers 2, 1
    char *dgs;           // [wave][layer][t][KBB][hi|lo][64 lanes][16 B]: the cells' scaled dgate blocks
    float *dsc;          // [wave][layer][t][16]: per-trajectory unscaling factor of those blocks (0: no gradient)
    Packed p;
};

template <int HS>
struct SurGeo {
    static constexpr int KBB = (HS + 1) / 2;
    static constexpr int QC = Geo<HS>::QC;                       // 16-B units per cell record
    static constexpr size_t SEQ = (size_t)kLayers * kL * QC;      // per wave, in 16-B units
    static constexpr size_t DSEQ = (size_t)2 * kL * QC;
    static constexpr size_t DG = (size_t)kLayers * kL * KBB * 2048;   // bytes per wave
    static constexpr size_t DSC = (size_t)kLayers * kL * 16;          // floats per wave
    static constexpr int LDS_FWD = (Geo16<HS>::FA1 + Geo16<HS>::FA0 + Geo16<HS>::FCP + 4) * 4;
    static constexpr int LDS_BWD = BwdLds<HS, false>::REGION + Geo16<HS>::FCP * 4;
};

// ---------------------------------------------------------------------------------------------------------------
// forward: fcr_fwd_kernel's window body for j = 0, the window rows read from x
template <int HS, bool STORE>
__global__ __launch_bounds__(kFwdWaves * kWave, kFwdWaves / 4) void sur_fwd_kernel(SurArgs a) {
    using G = Geo16<HS>;
    extern __shared__ __attribute__((aligned(16))) float lw[];
    float *lw0 = lw + G::FA1;     // resident layer-0 fragments; layers 1, 2 are refilled into lw per phase
    float *lfcp = lw0 + G::FA0;   // fc.weight (lane layout), fc.bias
    float *lfcb = lfcp + G::FCP;
    lds_copy(lw0, a.p.fa[0], G::FA0);
    lds_copy(lfcp, a.p.fcp, G::FCP);
    lds_copy(lfcb, a.p.fcb, 4);
    const int lane = threadIdx.x & 63;
    const int q = lane >> 4, sl = lane & 15;
    const int wave = blockIdx.x * kFwdWaves + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int b = wave * kTile + sl;
    const bool valid = b < a.B;
    const int bc = valid ? b : a.B - 1;   // out-of-range lanes recompute the last window (never stored as y)
    const float *xb = a.x + (size_t)bc * kL * kIn;
    const float scq = a.p.wsc[q], sc4 = a.p.wsc[4];
    float w0[kL], w1[kL];   // window rows in the B-operand layout (column q; column 4 in lane group 0)
#pragma unroll
    for (int t = 0; t < kL; ++t) {
        w0[t] = xb[t * kIn + q] * scq;
        w1[t] = (q == 0) ? xb[t * kIn + 4] * sc4 : 0.0f;
    }
    float c[HS], hout[HS], hp[HS], xc[HS], xn[HS];
    constexpr size_t qcell = (size_t)Geo<HS>::QC;
    const __amdgpu_buffer_rsrc_t rh = wave_rsrc(a.hseq + (size_t)wave * SurGeo<HS>::SEQ, SurGeo<HS>::SEQ * 16);
    const __amdgpu_buffer_rsrc_t rc = wave_rsrc(a.cseq + (size_t)wave * SurGeo<HS>::SEQ, SurGeo<HS>::SEQ * 16);
    const __amdgpu_buffer_rsrc_t rx = wave_rsrc(a.xw + (size_t)wave * kL * kWave, (size_t)kL * kWave * 8);
#define SEQ_O(l, t) ((uint32_t)(((l) * kL + (t)) * qcell * 16))
    Pace turn;
    turn.turn = (threadIdx.x >> 8) & 1;
    __syncthreads();
    // ---- layer 0 (Model_NN/Functions.py:327) ----
    {
        const float x0 = w0[0], x1 = w1[0];
        rot_left(w0);
        rot_left(w1);
        fwd16_cell<HS, true, true, false>(lw0, lane, x0, x1, hp, hp, c, hout, turn);
        split_rec<HS>(hout, hp);
        buf_store_quads<HS>(rh, SEQ_O(0, 0), hp, lane);
        if (STORE) {
            buf_st2(rx, lane * 8, 0u, f32x2{x0, x1});
            buf_store_quads<HS>(rc, SEQ_O(0, 0), c, lane);
        }
    }
    for (int t = 1; t < kL; ++t) {
        const float x0 = w0[0], x1 = w1[0];
        rot_left(w0);
        rot_left(w1);
        fwd16_cell<HS, true, false, false>(lw0, lane, x0, x1, hp, hp, c, hout, turn);
        split_rec<HS>(hout, hp);
        buf_store_quads<HS>(rh, SEQ_O(0, t), hp, lane);
        if (STORE) {
            buf_st2(rx, lane * 8, (uint32_t)(t * kWave * 8), f32x2{x0, x1});
            if (t + 1 < kL) buf_store_quads<HS>(rc, SEQ_O(0, t), c, lane);
        }
    }
    // ---- layers 1, 2 ----
#pragma unroll
    for (int l = 1; l < kLayers; ++l) {
        lds_fill<G::FA1 * 4, kFwdWaves>(lw, a.p.fa[l]);
        buf_load_quads<HS>(xc, rh, SEQ_O(l - 1, 0), lane);
        buf_load_quads<HS>(xn, rh, SEQ_O(l - 1, 1), lane);
        fwd16_cell<HS, false, true, false>(lw, lane, 0.0f, 0.0f, xc, hp, c, hout, turn);
        split_rec<HS>(hout, hp);
        if (l == 1 || STORE) buf_store_quads<HS>(rh, SEQ_O(l, 0), hp, lane);
        if (STORE) buf_store_quads<HS>(rc, SEQ_O(l, 0), c, lane);
#pragma unroll
        for (int r = 0; r < HS; ++r) xc[r] = xn[r];
#pragma unroll 3
        for (int t = 1; t < kL; ++t) {
            buf_load_quads<HS>(xn, rh, SEQ_O(l - 1, t + 1 < kL ? t + 1 : t), lane);
            fwd16_cell<HS, false, false, false>(lw, lane, 0.0f, 0.0f, xc, hp, c, hout, turn);
            if (!(l == 2 && t + 1 == kL)) {   // h_9 of layer 2 only feeds the readout (fp32 hout)
                split_rec<HS>(hout, hp);
                if (l == 1 || STORE) buf_store_quads<HS>(rh, SEQ_O(l, t), hp, lane);
            }
            if (STORE && t + 1 < kL) buf_store_quads<HS>(rc, SEQ_O(l, t), c, lane);
#pragma unroll
            for (int r = 0; r < HS; ++r) xc[r] = xn[r];
        }
    }
#undef SEQ_O
    // ---- readout fc(out[:, -1, :]) (Model_NN/Functions.py:330) ----
    float xo[kOut];
#pragma unroll
    for (int o = 0; o < kOut; ++o) {
        float p = 0.0f;
#pragma unroll
        for (int r = 0; r < HS; ++r) p += lfcp[(o * HS + r) * 4 + q] * hout[r];
        xo[o] = xor_sum_q(p) + lfcb[o];
    }
    if (valid) {
        a.y[(size_t)b * kOut + q] = sel4(q, xo[0], xo[1], xo[2], xo[3]);
        if (STORE) {
#pragma unroll
            for (int r = 0; r < HS; ++r)
                if (4 * r + q < a.H) a.htop[(size_t)b * a.H + 4 * r + q] = hout[r];
        }
    }
}

// ---------------------------------------------------------------------------------------------------------------
// backward: fcr_bwd_kernel's window body for j = 0 (dh_9 from dy instead of the rollout's cost terms), every cell
// with DG: its dgate blocks and unscaling factor into the wave's dgs / dsc regions
template <int HS>
__global__ __launch_bounds__(kBwdWaves * kWave, kBwdWaves / 4) void sur_bwd_kernel(SurArgs a) {
    using LD = BwdLds<HS, false>;
    using I1 = Img<HS, false>;
    using I0 = Img<HS, true>;
    using SG = SurGeo<HS>;
    extern __shared__ __attribute__((aligned(16))) float lw[];
    float *lfcp = lw + LD::REGION / 4;
    lds_copy(lfcp, a.p.fcp, Geo16<HS>::FCP);
    __syncthreads();
    const int lane = threadIdx.x & 63;
    const int q = lane >> 4, sl = lane & 15;
    const int wave = blockIdx.x * kBwdWaves + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int b = wave * kTile + sl;
    const bool valid = b < a.B;
    const float scq = a.p.wsc[q], sc4 = a.p.wsc[4];   // d/dx = 2^-s_c d/dx' (fcr_pack.h)
    const ImgLane<I1::U> L1 = img_lane<I1::U>(lds_offset(lw), lane);
    const ImgLane<I0::U> L0 = img_lane<I0::U>(lds_offset(lw), lane);
    // dh_9 = fc.W^T dy (Model_NN/Functions.py:330); padding windows carry no gradient
    float dyo[kOut];
#pragma unroll
    for (int o = 0; o < kOut; ++o) dyo[o] = valid ? a.dy[(size_t)b * kOut + o] : 0.0f;
    float dh_out[HS];
#pragma unroll
    for (int r = 0; r < HS; ++r) {
        const float *fp = lfcp + r * 4 + q;
        dh_out[r] = fp[0] * dyo[0] + fp[HS * 4] * dyo[1] + fp[2 * HS * 4] * dyo[2] + fp[3 * HS * 4] * dyo[3];
    }
    float dh[HS], dc[HS], dxo[HS], dab[HS];
    constexpr size_t qcell = (size_t)Geo<HS>::QC;
    NextIn nb;
    nb.rh = wave_rsrc(a.hseq + (size_t)wave * SG::SEQ, SG::SEQ * 16);
    nb.rc = wave_rsrc(a.cseq + (size_t)wave * SG::SEQ, SG::SEQ * 16);
    nb.rx = wave_rsrc(a.xw + (size_t)wave * kL * kWave, (size_t)kL * kWave * 8);
    nb.rd = wave_rsrc(a.dseq + (size_t)wave * SG::DSEQ, SG::DSEQ * 16);
    auto hoff = [&](int l, int t) { return (uint32_t)(((size_t)l * kL + t) * qcell * 16); };
    auto doff = [&](int lfrom, int t) { return ((size_t)(2 - lfrom) * kL + t) * qcell; };
    auto next_of = [&](int l, int t) {   // the cell processed after (l, t)
        NextIn n = nb;
        int nl = l, nt = t - 1;
        if (t == 0) {
            nt = kL - 1;
            nl = l - 1;
        }
        if (nl < 0) { nl = 2; nt = kL - 1; }   // past the last cell: reload a valid one (harmless)
        n.x = nl == 0 ? (uint32_t)(nt * kWave * 8) : hoff(nl > 0 ? nl - 1 : 0, nt);
        n.h = hoff(nl, nt > 0 ? nt - 1 : 0);
        n.c = n.h;
        n.o = hoff(nl, nt);
        n.d = (uint32_t)((nl < 2 ? doff(nl + 1, nt) : 0) * 16);
        return n;
    };
    DgOut dg;
    dg.r = wave_rsrc(a.dgs + (size_t)wave * SG::DG, SG::DG);
    dg.rs = wave_rsrc(a.dsc + (size_t)wave * SG::DSC, SG::DSC * 4);
    auto dg_at = [&](int l, int t) {
        DgOut d = dg;
        d.off = (uint32_t)(((size_t)l * kL + t) * SG::KBB * 2048);
        d.soff = (uint32_t)((l * kL + t) * 64);
        return d;
    };
    Stamps sp = {{0, 0, 0, 0, (unsigned long long)((threadIdx.x >> 8) & 1), 0, 0, 0}};
    CellIn<HS> ci;
    {
        const NextIn f = next_of(2, kL);   // t = kL -> (2, 9)
        load_xhd<HS, false, true, false>(ci, f, lane);
        ld_quads<HS>(ci.c, f.rc, f.c, lane);
    }
    float unused0, unused1;
    // ---- layer 2 ----
    lds_fill<I1::BYTES, kBwdWaves>(lw, a.p.img[2]);
#pragma unroll
    for (int r = 0; r < HS; ++r) dh[r] = dc[r] = dab[r] = 0.0f;
    {
        const DgOut d = dg_at(2, kL - 1);
        bwd_cell<HS, false, false, false, false, true, false, false, false, true, true>(
            L1.fb, L1.tb, lane, dh_out, dh, dc, dxo, unused0, unused1, ci, next_of(2, kL - 1), sp, &d);
        buf_store_quads<HS>(nb.rd, (uint32_t)((doff(2, kL - 1)) * 16), dxo, lane);
    }
    for (int t = kL - 2; t >= 2; --t) {
        const DgOut d = dg_at(2, t);
        bwd_cell<HS, false, false, false, false, true, false, false, true, true, true>(
            L1.fb, L1.tb, lane, dab, dh, dc, dxo, unused0, unused1, ci, next_of(2, t), sp, &d);
        buf_store_quads<HS>(nb.rd, (uint32_t)((doff(2, t)) * 16), dxo, lane);
    }
    {
        const DgOut d1 = dg_at(2, 1);
        bwd_cell<HS, false, false, false, false, false, false, false, true, true, true>(
            L1.fb, L1.tb, lane, dab, dh, dc, dxo, unused0, unused1, ci, next_of(2, 1), sp, &d1);
        buf_store_quads<HS>(nb.rd, (uint32_t)((doff(2, 1)) * 16), dxo, lane);
        const DgOut d0 = dg_at(2, 0);
        bwd_cell<HS, false, false, true, false, true, true, false, true, true, true>(
            L1.fb, L1.tb, lane, dab, dh, dc, dxo, unused0, unused1, ci, next_of(2, 0), sp, &d0);
        buf_store_quads<HS>(nb.rd, (uint32_t)((doff(2, 0)) * 16), dxo, lane);
    }
    // ---- layer 1 ----
    lds_fill<I1::BYTES, kBwdWaves>(lw, a.p.img[1]);
#pragma unroll
    for (int r = 0; r < HS; ++r) dh[r] = dc[r] = 0.0f;
    for (int t = kL - 1; t >= 2; --t) {
        const DgOut d = dg_at(1, t);
        bwd_cell<HS, false, true, false, false, true, true, false, true, true, true>(
            L1.fb, L1.tb, lane, dab, dh, dc, dxo, unused0, unused1, ci, next_of(1, t), sp, &d);
        buf_store_quads<HS>(nb.rd, (uint32_t)((doff(1, t)) * 16), dxo, lane);
    }
    {
        const DgOut d1 = dg_at(1, 1);
        bwd_cell<HS, false, true, false, false, false, true, false, true, true, true>(
            L1.fb, L1.tb, lane, dab, dh, dc, dxo, unused0, unused1, ci, next_of(1, 1), sp, &d1);
        buf_store_quads<HS>(nb.rd, (uint32_t)((doff(1, 1)) * 16), dxo, lane);
        const DgOut d0 = dg_at(1, 0);
        bwd_cell<HS, false, true, true, true, true, true, false, true, true, true>(
            L1.fb, L1.tb, lane, dab, dh, dc, dxo, unused0, unused1, ci, next_of(1, 0), sp, &d0);
        buf_store_quads<HS>(nb.rd, (uint32_t)((doff(1, 0)) * 16), dxo, lane);
    }
    // ---- layer 0: the window-row gradients are dL/dx ----
    lds_fill<I0::BYTES, kBwdWaves>(lw, a.p.img[0]);
#pragma unroll
    for (int r = 0; r < HS; ++r) dh[r] = dc[r] = 0.0f;
    float *gx = (a.g_x && valid) ? a.g_x + (size_t)b * kL * kIn : nullptr;
    auto put_gx = [&](int t, float dxq, float dx4) {
        if (gx) {
            gx[t * kIn + q] = dxq * scq;
            if (q == 0) gx[t * kIn + 4] = dx4 * sc4;
        }
    };
    for (int t = kL - 1; t >= 2; --t) {
        float dxq, dx4;
        const DgOut d = dg_at(0, t);
        bwd_cell<HS, true, true, false, true, true, true, false, true, true, true>(
            L0.fb, L0.tb, lane, dab, dh, dc, dxo, dxq, dx4, ci, next_of(0, t), sp, &d);
        put_gx(t, dxq, dx4);
    }
    {
        float dxq, dx4;
        const DgOut d1 = dg_at(0, 1);
        bwd_cell<HS, true, true, false, true, false, true, false, true, true, true>(
            L0.fb, L0.tb, lane, dab, dh, dc, dxo, dxq, dx4, ci, next_of(0, 1), sp, &d1);
        put_gx(1, dxq, dx4);
        const DgOut d0 = dg_at(0, 0);
        bwd_cell<HS, true, true, true, false, true, false, false, true, false, true>(
            L0.fb, L0.tb, lane, dab, dh, dc, dxo, dxq, dx4, ci, next_of(0, 0), sp, &d0);
        put_gx(0, dxq, dx4);
    }
}

// ---------------------------------------------------------------------------------------------------------------
// weight gradients of layer l: D[R][n] = sum over rows k of dG[k][R] in[k][n]
//   R = 16 slot + 4 c + gate: gate row (gate, unit 4 slot + c) — the forward D-tile order (m-tile = slot);
//   n = 16 nt + 4 c + e: record half 4a + e of lane group c, a = nt (x record: the layer-below h_t) or nt - RA (h
//       record: h_{t-1}; zero at t = 0). A record half p < HS is the hi half of slot p, HS <= p < 2HS the lo half of
//       slot p - HS, so the hi and lo parts of every input are separate columns and their sum is the input — the B
//       operand needs no split of its own. Layer 0: the h record, then one tile of the window columns
//       (hi x_c, lo x_c, hi x_4, lo x_4) per group c (x_4 in group 0 only).
// A k-block is 64 rows, k = 32 ws + 16 cs + trajectory: two backward waves (ws) x two steps 2tp + cs; its inputs
// (~82 KB at H = 50) are loaded into registers one k-block ahead, so every CU has that much in flight under the
// products of the previous one. Each row's dgates come back from their scaled halves times the row's `down` and the
// workgroup's common scale S (1 / the largest `down` of its rows, so every value stays in f16's range; exact
// powers of two), then are split again.
// LDS (natural row layouts, 8-B units of 4 consecutive R or n): A rows at sur_rowA(k) (544-B stride plus 128-B
// shifts per 8 and per 16 rows), B rows at sur_rowB(k) (768-B stride, 8-B swizzle): the 32 lanes of each half of a
// transposed read land on 32 distinct bank pairs (checked by tests/test_sur_layout.py).
constexpr int kSurKW = 2, kSurKC = 2;                   // backward waves x steps per k-block
constexpr int kSurKR = 16 * kSurKW * kSurKC;             // rows per k-block
__host__ __device__ constexpr int sur_rowA(int k) { return k * 544 + 128 * ((k >> 3) & 1) + 128 * (k >> 4); }
__host__ __device__ constexpr int sur_rowB(int k) { return k * 768 + 8 * ((k & 3) + 4 * ((k >> 3) & 1)); }
template <int HS, bool L0>
struct SurWg {
    static constexpr int KBB = (HS + 1) / 2;
    static constexpr int MT = HS;                     // m-tiles
    static constexpr int RA = (2 * HS + 3) / 4;       // 4-half units per record
    static constexpr int NT = L0 ? RA + 1 : 2 * RA;   // n-tiles
    static constexpr int MW = (MT + 1) / 2;           // m-tiles per wave (2 m-groups)
    static constexpr int NW = (NT + 3) / 4;           // n-tiles per wave (4 n-groups)
    static constexpr int SA = 544, SB = 768;
    static constexpr int A_BYTES = sur_rowA(kSurKR - 1) + 32 * 2 * KBB;   // the last row's start + its length
    static constexpr int A_PAD = (A_BYTES + 255) / 256 * 256;
    static constexpr int B_OFF = 2 * A_PAD;
    static constexpr int LDS = B_OFF + kSurKR * SB;
    static constexpr int ROWS_N = 16 * NT;            // partial row length (floats)
    static constexpr int PART = 16 * MT * ROWS_N;     // floats per workgroup partial
    static_assert(LDS <= 163840, "LDS");
};
constexpr int kSurWgThreads = 512;
constexpr int kSurWgMaxGroups = 256;

template <int HS, bool L0>
__global__ __launch_bounds__(kSurWgThreads, 1) void sur_wgrad_kernel(SurArgs a, int l, int nkb, float *part) {
    using W = SurWg<HS, L0>;
    using SG = SurGeo<HS>;
    typedef _Float16 f16x4v __attribute__((ext_vector_type(4)));
    extern __shared__ __attribute__((aligned(16))) char sm[];
    __shared__ float red[kSurWgThreads / 64];
    const int tid = threadIdx.x, lane = tid & 63;
    const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int G = gridDim.x;
    const int kb0 = (int)((long long)nkb * blockIdx.x / G), kb1 = (int)((long long)nkb * (blockIdx.x + 1) / G);
    constexpr int NTP = kL / kSurKC;   // k-blocks (step groups) per backward-wave group
    // ---- the workgroup's common scale: the largest `down` over its rows ----
    float m = 0.0f;
    for (int e = tid; e < kSurKR * (kb1 - kb0); e += kSurWgThreads) {
        const int kb = kb0 + e / kSurKR, r = e % kSurKR;
        const int w = (kb / NTP) * kSurKW + r / (16 * kSurKC), tp = kb % NTP;
        m = fmaxf(m, a.dsc[(size_t)w * SG::DSC + (size_t)(l * kL + kSurKC * tp) * 16 + r % (16 * kSurKC)]);
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o));
    if (lane == 0) red[wv] = m;
    __syncthreads();
    m = red[0];
#pragma unroll
    for (int i = 1; i < kSurWgThreads / 64; ++i) m = fmaxf(m, red[i]);
    const float S = m > 0.0f ? 1.0f / m : 1.0f;   // exact: m is a power of two

    // ---- staging items of a k-block: dgate pieces (waves x steps x KBB blocks x 64 lanes; hi and lo 16 B each) and
    // one input record per thread: (wave ws, step cs, record rr, lane lam) ----
    constexpr int NDG = kSurKW * kSurKC * W::KBB * 64;
    constexpr int DGI = (NDG + kSurWgThreads - 1) / kSurWgThreads;
    static_assert(kSurKW * kSurKC * 2 * 64 == kSurWgThreads, "one input record per thread");
    f32x4 gh[DGI], gl[DGI];
    float gs[DGI];
    float rec[16];
    f32x2 win = {0.0f, 0.0f};
    const int rlam = tid & 63, rrr = (tid >> 6) & 1, rcs = (tid >> 7) % kSurKC, rws = tid / (128 * kSurKC);
    auto load = [&](int kb) {
        const int w0 = (kb / NTP) * kSurKW, tp = kb % NTP;
#pragma unroll
        for (int i = 0; i < DGI; ++i) {
            const int it = tid + i * kSurWgThreads;
            if (it < NDG) {
                const int lam = it & 63, kbb = (it >> 6) % W::KBB, cs = (it / (64 * W::KBB)) % kSurKC,
                          ws = it / (64 * W::KBB * kSurKC);
                const int w = w0 + ws, t = kSurKC * tp + cs;
                const char *src = a.dgs + (size_t)w * SG::DG + ((size_t)(l * kL + t) * W::KBB + kbb) * 2048 + lam * 16;
                gh[i] = *reinterpret_cast<const f32x4 *>(src);
                gl[i] = *reinterpret_cast<const f32x4 *>(src + 1024);
                gs[i] = a.dsc[(size_t)w * SG::DSC + (size_t)(l * kL + t) * 16 + (lam & 15)];
            }
        }
        const int w = w0 + rws, t = kSurKC * tp + rcs;
#pragma unroll
        for (int e = 0; e < 16; ++e) rec[e] = 0.0f;
        // record rrr = 0: the layer input at t (layer >= 1: layer l-1's h_t; layer 0: the window row),
        // rrr = 1: h_{t-1} of layer l (none at t = 0)
        if (L0 && rrr == 0) {
            win = a.xw[((size_t)w * kL + t) * kWave + rlam];
        } else if (!(rrr == 1 && t == 0)) {
            const int ll = rrr == 0 ? l - 1 : l, tt = rrr == 0 ? t : t - 1;
            const f32x4 *cellp = a.hseq + (size_t)w * SG::SEQ + (size_t)(ll * kL + tt) * SG::QC;
            constexpr int FQ = HS / 4, TS = HS % 4;
#pragma unroll
            for (int k = 0; k < FQ; ++k) {
                const f32x4 v = cellp[k * kWave + rlam];
#pragma unroll
                for (int e = 0; e < 4; ++e) rec[4 * k + e] = v[e];
            }
            const float *tail = reinterpret_cast<const float *>(cellp + FQ * kWave) + rlam * TS;
#pragma unroll
            for (int e = 0; e < TS; ++e) rec[4 * FQ + e] = tail[e];
        }
    };
    char *lA = sm, *lAl = sm + W::A_PAD, *lB = sm + W::B_OFF;
    auto stage = [&]() {
#pragma unroll
        for (int i = 0; i < DGI; ++i) {
            const int it = tid + i * kSurWgThreads;
            if (it < NDG) {
                const int lam = it & 63, kbb = (it >> 6) % W::KBB, cs = (it / (64 * W::KBB)) % kSurKC,
                          ws = it / (64 * W::KBB * kSurKC);
                const int k = 32 * ws + 16 * cs + (lam & 15), qq = lam >> 4;
                const float sc = gs[i] * S;
                const f16x8 h = __builtin_bit_cast(f16x8, gh[i]), lo = __builtin_bit_cast(f16x8, gl[i]);
                float v[8];
#pragma unroll
                for (int j = 0; j < 8; ++j) v[j] = ((float)h[j] + (float)lo[j]) * sc;
                f16x8 nh, nl;
                split8(v, nh, nl);
                const int o0 = sur_rowA(k) + 32 * (2 * kbb) + 8 * qq;
                f16x4v h0, h1, l0, l1;
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    h0[j] = nh[j];
                    h1[j] = nh[4 + j];
                    l0[j] = nl[j];
                    l1[j] = nl[4 + j];
                }
                *reinterpret_cast<f16x4v *>(lA + o0) = h0;
                *reinterpret_cast<f16x4v *>(lA + o0 + 32) = h1;
                *reinterpret_cast<f16x4v *>(lAl + o0) = l0;
                *reinterpret_cast<f16x4v *>(lAl + o0 + 32) = l1;
            }
        }
        {
            const int k = 32 * rws + 16 * rcs + (rlam & 15), qq = rlam >> 4;
            // layer >= 1: x record at +0, h record at +256; layer 0: h record at +0, window unit at +256
            const int region = L0 ? (rrr == 0 ? 256 : 0) : 256 * rrr;
            char *dst = lB + sur_rowB(k) + region + 64 * qq;
            if (L0 && rrr == 0) {
                f16x4v u;
                const _Float16 h0 = (_Float16)win[0], h1 = (_Float16)win[1];
                u[0] = h0;
                u[1] = (_Float16)(win[0] - (float)h0);
                u[2] = h1;
                u[3] = (_Float16)(win[1] - (float)h1);
                *reinterpret_cast<f16x4v *>(dst) = u;
            } else {
#pragma unroll
                for (int k4 = 0; k4 < 4; ++k4)
                    *reinterpret_cast<f32x4 *>(dst + 16 * k4) =
                        f32x4{rec[4 * k4], rec[4 * k4 + 1], rec[4 * k4 + 2], rec[4 * k4 + 3]};
            }
        }
    };

    // ---- products: wave (mg, ng) owns m-tiles [mg MW, ..) x n-tiles [ng NW, ..) ----
    const int mg = wv & 1, ng = wv >> 1;
    const int g = lane >> 4, er = (lane >> 2) & 3, c = lane & 3;
    // lane bases of the transposed reads for the rows 8g + er (+ 4h, + 32kk: instruction offsets)
    const uint32_t la = lds_offset(lA) + (uint32_t)(sur_rowA(8 * g + er) + 8 * c);
    const uint32_t lb = lds_offset(lB) + (uint32_t)(sur_rowB(8 * g + er) + 64 * c);
    f32x4 acc[W::MW][W::NW];
#pragma unroll
    for (int i = 0; i < W::MW; ++i)
#pragma unroll
        for (int j = 0; j < W::NW; ++j) acc[i][j] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
    auto frag = [&](uint32_t addr, uint32_t step) {
        const f16x4 p0 = lds_tr_f16(addr), p1 = lds_tr_f16(addr + step);
        f16x8 f;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            f[j] = p0[j];
            f[4 + j] = p1[j];
        }
        return f;
    };
    if (kb0 < kb1) load(kb0);
    for (int kb = kb0; kb < kb1; ++kb) {
        __syncthreads();   // the previous k-block's reads are done
        stage();
        __syncthreads();
        if (kb + 1 < kb1) load(kb + 1);   // in flight under this k-block's products
#pragma unroll
        for (int kk = 0; kk < kSurKR / 32; ++kk) {
            // rows 32kk + 8g + er + 4h: sur_rowA / sur_rowB differ from the lane base by constants
            const uint32_t oA = (uint32_t)(sur_rowA(32 * kk) - sur_rowA(0)), oB = (uint32_t)(sur_rowB(32 * kk) - sur_rowB(0));
            const uint32_t hA = (uint32_t)(sur_rowA(4) - sur_rowA(0)), hB = (uint32_t)(sur_rowB(4) - sur_rowB(0));
            f16x8 bf[W::NW];
#pragma unroll
            for (int j = 0; j < W::NW; ++j) {
                const int nt = ng * W::NW + j;
                if (nt < W::NT) {
                    const int rg = nt < W::RA ? 0 : 256;
                    const int aa = nt < W::RA ? nt : nt - W::RA;
                    bf[j] = frag(lb + oB + rg + 8 * aa, hB);
                }
            }
#pragma unroll
            for (int i = 0; i < W::MW; ++i) {
                const int mt = mg * W::MW + i;
                if (mt < W::MT) {
                    const f16x8 ah = frag(la + oA + 32 * mt, hA);
                    const f16x8 al = frag(la + W::A_PAD + oA + 32 * mt, hA);
#pragma unroll
                    for (int j = 0; j < W::NW; ++j) {
                        if (ng * W::NW + j < W::NT) {
                            acc[i][j] = mfma16(al, bf[j], acc[i][j]);
                            acc[i][j] = mfma16(ah, bf[j], acc[i][j]);
                        }
                    }
                }
            }
        }
    }
    // ---- partial of this workgroup, unscaled (exact): rows R, columns n ----
    float *pw = part + (size_t)blockIdx.x * W::PART;
    const float inv = m > 0.0f ? m : 0.0f;
#pragma unroll
    for (int i = 0; i < W::MW; ++i) {
        const int mt = mg * W::MW + i;
#pragma unroll
        for (int j = 0; j < W::NW; ++j) {
            const int nt = ng * W::NW + j;
            if (mt < W::MT && nt < W::NT) {
#pragma unroll
                for (int e = 0; e < 4; ++e)
                    pw[(size_t)(16 * mt + 4 * g + e) * W::ROWS_N + 16 * nt + (lane & 15)] = acc[i][j][e] * inv;
            }
        }
    }
}

// dW of layer l from the G partials (fixed order): thread per (torch gate row, input column); layer >= 1: columns
// [W_ih (H) | W_hh (H)], layer 0: [W_ih (5) | W_hh (H)]. The packed rows carry the exp2 pre-scale kappa of their
// gate and the window columns the range guard 2^-s_c: dW = kappa sum(D) (/ wsc for the window columns).
template <int HS, bool L0>
__global__ __launch_bounds__(256) void sur_wgrad_finish_kernel(const float *__restrict__ part, int G, int H,
                                                               const float *__restrict__ wsc, float *g_ih,
                                                               float *g_hh) {
    using W = SurWg<HS, L0>;
    const int nin = L0 ? kIn : H;
    const int idx = blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= 4 * H * (nin + H)) return;
    const int gr = idx / (nin + H), col = idx % (nin + H);
    const int gate = gr / H, unit = gr % H;
    const int R = 16 * (unit >> 2) + 4 * (unit & 3) + gate;
    const float kappa = gate == 2 ? kTwoLog2e : kNegLog2e;
    int n_hi, n_lo;
    float f = kappa;
    auto rec_cols = [&](int rec, int u) {   // columns of the hi and lo halves of input unit u of a record
        const int s = u >> 2, cc = u & 3;
        const int ph = s, pl = HS + s;
        n_hi = 16 * (rec * W::RA + (ph >> 2)) + 4 * cc + (ph & 3);
        n_lo = 16 * (rec * W::RA + (pl >> 2)) + 4 * cc + (pl & 3);
    };
    const bool ih = col < nin;
    if (L0) {
        if (ih) {   // window column col
            const int cc = col < 4 ? col : 0, e = col < 4 ? 0 : 2;
            n_hi = 16 * W::RA + 4 * cc + e;
            n_lo = n_hi + 1;
            f = kappa / wsc[col];
        } else {
            rec_cols(0, col - nin);
        }
    } else {
        rec_cols(ih ? 0 : 1, ih ? col : col - nin);
    }
    float s = 0.0f;
    for (int gi = 0; gi < G; ++gi) {
        const float *p = part + (size_t)gi * W::PART + (size_t)R * W::ROWS_N;
        s += p[n_hi] + p[n_lo];
    }
    if (ih) g_ih[(size_t)gr * nin + col] = s * f;
    else g_hh[(size_t)gr * H + (col - nin)] = s * f;
}

// the G workgroup partials summed in place into partial 0, in fixed order: a thread per 4 consecutive elements, the
// loads of 8 partials issued ahead of their (ordered) adds
__global__ __launch_bounds__(256) void sur_part_sum_kernel(float *part, int G, int n) {
    const int e = 4 * (blockIdx.x * blockDim.x + threadIdx.x);
    if (e >= n) return;   // n % 4 == 0 (16 x 16 tiles)
    f32x4 s = {0.0f, 0.0f, 0.0f, 0.0f};
    int g = 0;
    for (; g + 8 <= G; g += 8) {
        f32x4 v[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) v[i] = *reinterpret_cast<const f32x4 *>(part + (size_t)(g + i) * n + e);
#pragma unroll
        for (int i = 0; i < 8; ++i) s += v[i];
    }
    for (; g < G; ++g) s += *reinterpret_cast<const f32x4 *>(part + (size_t)g * n + e);
    *reinterpret_cast<f32x4 *>(part + e) = s;
}

// The readout's gradients d fc.weight[o][u] = sum_b dy[b][o] h_9[b][u] and d fc.bias[o] = sum_b dy[b][o]: per block
// a tile of kFcRows windows staged in LDS (coalesced), one thread per output, partials [block][4H + 4]; then a
// fixed-order sum over the blocks (sur_fc_final_kernel). Deterministic.
constexpr int kFcRows = 128;
__global__ __launch_bounds__(256) void sur_fc_partial_kernel(const float *__restrict__ dy, const float *__restrict__ htop,
                                                             int B, int H, float *part) {
    __shared__ float sh[kFcRows * 52];
    __shared__ float sdy[kFcRows * kOut];
    const int b0 = blockIdx.x * kFcRows;
    const int nr = B - b0 < kFcRows ? B - b0 : kFcRows;
    for (int e = threadIdx.x; e < nr * H; e += 256) sh[e] = htop[(size_t)b0 * H + e];
    for (int e = threadIdx.x; e < nr * kOut; e += 256) sdy[e] = dy[(size_t)b0 * kOut + e];
    __syncthreads();
    const int t = threadIdx.x, nout = kOut * H + kOut;
    if (t >= nout) return;
    float s = 0.0f;
    if (t < kOut * H) {
        const int o = t / H, u = t % H;
        for (int r = 0; r < nr; ++r) s = fmaf(sdy[r * kOut + o], sh[r * H + u], s);
    } else {
        for (int r = 0; r < nr; ++r) s += sdy[r * kOut + (t - kOut * H)];
    }
    part[(size_t)blockIdx.x * nout + t] = s;
}
// one block per output: a strided fixed-order sum per thread, then a fixed tree
__global__ __launch_bounds__(256) void sur_fc_final_kernel(const float *__restrict__ part, int nblk, int H, float *g_fc_w,
                                                           float *g_fc_b) {
    __shared__ float red[256];
    const int t = blockIdx.x, nout = kOut * H + kOut;
    float s = 0.0f;
    for (int b = threadIdx.x; b < nblk; b += 256) s += part[(size_t)b * nout + t];
    red[threadIdx.x] = s;
    __syncthreads();
    for (int w = 128; w > 0; w >>= 1) {
        if ((int)threadIdx.x < w) red[threadIdx.x] += red[threadIdx.x + w];
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        if (t < kOut * H) g_fc_w[t] = red[0];
        else g_fc_b[t - kOut * H] = red[0];
    }
}

}  // namespace fcr
