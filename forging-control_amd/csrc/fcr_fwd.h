// fcr_fwd.h — forward rollout kernel (MPCLoss.forward, Functions.py:1353-1472).
//
// One wave = 16 trajectories; one workgroup = kFwdWaves waves sharing one LDS-resident layer of
// MFMA fragments. Each window (horizon step) runs three layer PHASES (layer-major): the current
// layer's fragments are copied into LDS, then the wave steps t = 0..9 through that layer. Each cell's
// h goes to a per-wave global slab (the next phase reads it back one cell ahead), and — when the
// backward will run — so do c and the layer-0 window rows: the backward recomputes every gate from
// (x_t, h_{t-1}, c_{t-1}) instead of reading stored activations (fcr_bwd.h), so the forward writes
// 8 B per unit slot and cell instead of the 24 B of local derivatives.
#pragma once
#include "fcr_common.h"
#include "fcr_f16.h"

namespace fcr {

__device__ __forceinline__ void rot_left(float (&w)[kL]) {
    const float t0 = w[0];
#pragma unroll
    for (int k = 0; k < kL - 1; ++k) w[k] = w[k + 1];
    w[kL - 1] = t0;
}

// One LSTM cell for 16 trajectories on the f16 matrix cores (fcr_f16.h): fragments
// [r][kb][hi|lo][lane][8 halves]. L0: input is the window row (x0: column q in lane group q, x1:
// column 4 in lane group 0); otherwise x = the split record of the layer-below h_t. hp = the split
// record of h_{t-1} (fcr_f16.h, split_rec); hout = this cell's h (fp32). FIRST: t = 0 (h_{t-1} = 0: those
// k-blocks are skipped). The B operands are split once per cell and shared by all tiles. Tiles go in
// pairs, one accumulator each (a dependent 16x16x32 MFMA chain issues back to back): one scheduling region
// per k-block with the next block's fragment reads in flight, and the previous pair's cell update spread over
// this pair's regions beside its MFMAs.
// Issue-priority pacing of the two waves that share a SIMD (waves w and w+4 of the workgroup): they alternate the
// higher priority cell by cell. Every layer phase ends at a workgroup barrier (the fragment refill), so a wave that
// runs ahead only waits there while its partner runs alone on the SIMD. (Giving it always to the younger wave, or
// taking it from the wave that is ahead of its partner by published progress, measured 3 % slower: DESIGN.md §6.)
struct Pace {
    unsigned turn;
};
__device__ __forceinline__ void pace_cell(Pace &p) {
    if (p.turn & 1) __builtin_amdgcn_s_setprio(1);
    else __builtin_amdgcn_s_setprio(0);
    p.turn ^= 1;
}

// R0, R1: the tile (unit slot) range this wave computes — the whole cell by default; the small-batch
// kernels (fcr_small.h) split a cell's tiles over the waves of a workgroup (R0 even).
template <int HS, bool L0, bool FIRST, bool LP, int R0 = 0, int R1 = HS>
__device__ __forceinline__ void fwd16_cell(const float *__restrict__ lw, int lane, float x0, float x1,
                                           const float (&x)[HS], const float (&hp)[HS], float (&c)[HS],
                                           float (&hout)[HS], Pace &turn) {
    pace_cell(turn);
    using G = Geo16<HS>;
    constexpr int KB = L0 ? G::KB0 : G::KB1;
    constexpr int KLO = (L0 && FIRST) ? G::XBLK : 0;
    constexpr int KHI = FIRST ? (L0 ? G::XBLK + 1 : G::KX1) : KB;
    constexpr int P0 = R0 / 2, P1 = (R1 + 1) / 2;   // tile pairs [P0, P1)
    static_assert(R0 % 2 == 0 && R0 < R1 && R1 <= HS, "tile range");
    // packed tail block (fcr_f16.h): one MFMA on the tail fragment, no lo fragment
    constexpr bool TAIL = !L0 && G::TAIL1;
    constexpr int KT = TAIL ? KB - 1 : KB;   // lo fragments per tile
    f16x8 bh[KB], bl[KB] = {};
#pragma unroll
    for (int kb = KLO; kb < KHI; ++kb) rec_operand<HS, L0, FIRST, LP>(kb, x0, x1, x, hp, bh[kb], bl[kb]);
    if (TAIL && KHI == KB) bh[KB - 1] = tail_operand<LP>(bh[KB - 1], bl[KB - 1]);
    // fragment reads of (tile r, block kb): hi, lo
    auto rd = [&](int r, int kb, f16x8 &h, f16x8 &l) {   // split-major fragments (pack_fwd16_kernel)
        h = lds_frag16(lw, r * KB + kb, lane);
        if (!LP && !(TAIL && kb == KB - 1)) l = lds_frag16(lw, HS * KB + r * KT + kb, lane);
    };
    f16x8 ah[2], al[2] = {};
    rd(R0, KLO, ah[0], al[0]);
    if (R0 + 1 < R1) rd(R0 + 1, KLO, ah[1], al[1]);
    f32x4 prev[2] = {{0.0f, 0.0f, 0.0f, 0.0f}, {0.0f, 0.0f, 0.0f, 0.0f}};
    constexpr int R = KHI - KLO;   // regions per tile pair
    float po[2] = {0.0f, 0.0f};    // exp2 of the previous pair's output-gate pre-activations between the stages
#pragma unroll
    for (int p = P0; p < P1; ++p) {
        const int r0 = 2 * p, r1 = 2 * p + 1;
        const bool two = r1 < R1;
        f32x4 acc[2] = {{0.0f, 0.0f, 0.0f, 0.0f}, {0.0f, 0.0f, 0.0f, 0.0f}};
#pragma unroll
        for (int kb = KLO; kb < KHI; ++kb) {
            sched_fence();
            // next region's fragments: (same pair, kb+1), else (next pair, KLO)
            f16x8 nh[2] = {ah[0], ah[1]}, nl[2] = {al[0], al[1]};
            if (kb + 1 < KHI) {
                rd(r0, kb + 1, nh[0], nl[0]);
                if (two) rd(r1, kb + 1, nh[1], nl[1]);
            } else if (p + 1 < P1) {
                rd(r0 + 2, KLO, nh[0], nl[0]);
                if (r1 + 2 < R1) rd(r1 + 2, KLO, nh[1], nl[1]);
            }
            if (TAIL && kb == KB - 1) {
                acc[0] = mfma16(ah[0], bh[kb], acc[0]);
                if (two) acc[1] = mfma16(ah[1], bh[kb], acc[1]);
            } else {
                acc[0] = mma_p<LP>(ah[0], al[0], bh[kb], bl[kb], acc[0]);
                if (two) acc[1] = mma_p<LP>(ah[1], al[1], bh[kb], bl[kb], acc[1]);
            }
            if (p > P0) {
                // the previous pair's pointwise, spread over this pair's regions beside its MFMAs
                // (R >= 3: gates of slot r0 | gates of slot r1 | both h; R = 2: both gates | both h)
                const int qr = kb - KLO;
                if (R == 1 || (R == 2 && qr == 0) || (R >= 3 && qr == 0))
                    lstm_point_a<FIRST>(prev[0], c[r0 - 2], c[r0 - 2], po[0]);
                if (R == 1 || (R == 2 && qr == 0) || (R >= 3 && qr == 1))
                    lstm_point_a<FIRST>(prev[1], c[r1 - 2], c[r1 - 2], po[1]);
                if (R == 1 || (R == 2 && qr == 1) || (R >= 3 && qr == 2)) {
                    lstm_point_b(c[r0 - 2], po[0], hout[r0 - 2]);
                    lstm_point_b(c[r1 - 2], po[1], hout[r1 - 2]);
                }
            }
#pragma unroll
            for (int u = 0; u < 2; ++u) {
                ah[u] = nh[u];
                al[u] = nl[u];
            }
        }
        prev[0] = acc[0];
        prev[1] = acc[1];
    }
    sched_fence();
    lstm_point<FIRST>(prev[0], c[2 * P1 - 2], c[2 * P1 - 2], hout[2 * P1 - 2]);
    if (2 * P1 - 1 < R1) lstm_point<FIRST>(prev[1], c[2 * P1 - 1], c[2 * P1 - 1], hout[2 * P1 - 1]);
}

#ifndef FCR_STAMP
#define FCR_STAMP 0
#endif
__device__ __forceinline__ unsigned long long fstamp() {
#if FCR_STAMP
    return __builtin_amdgcn_s_memtime();
#else
    return 0;
#endif
}

template <int HS, bool STORE, bool LP>
__global__ __launch_bounds__(kFwdWaves * kWave, kFwdWaves / 4) void fcr_fwd_kernel(FwdArgs a) {
    using G = Geo16<HS>;
    extern __shared__ __attribute__((aligned(16))) float lw[];
    // fp32 mode: [layer 1|2 fragments, refilled per phase | layer 0 | misc];
    // f16 mode:  [layer 1 hi | layer 2 hi | layer 0 hi | misc], all resident
    constexpr int F0 = LP ? G::FA0 / 2 : G::FA0;
    float *lw0 = lw + (LP ? 2 * G::FH1 : G::FA1);   // resident layer-0 fragments
    float *lfnp = lw0 + F0;                     // resident controller records
    float *lfcp = lfnp + G::FNP;                // resident fc.weight (lane layout) and fc.bias
    float *lfcb = lfcp + G::FCP;
    float *lwl[3] = {lw0, lw, lw + G::FH1};
    if (LP) {
        lds_copy(lwl[1], a.p.fa[1], G::FH1);
        lds_copy(lwl[2], a.p.fa[2], G::FH1);
    }
    lds_copy(lw0, a.p.fa[0], F0);
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
    const float scq = a.p.wsc[q], sc4 = a.p.wsc[4];   // range guard (fcr_pack.h): the ring holds v 2^-s_c
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

    float c[HS], hout[HS], hp[HS], xc[HS], xn[HS];   // hp, xc, xn: split records (fcr_f16.h)
    constexpr int kRW = rec_words<HS, LP>();         // words of an h record (hi halves only in the f16 mode)
    // sequence slabs [wave][j][layer][t][quad][64]: the split record of h of every cell (layers 0, 1: the
    // next phase's input; with STORE also layer 2) and, with STORE, c; plus the window rows [wave][j][t][64]
    const size_t qcell = (size_t)Geo<HS>::QC;    // one cell of a sequence slab, in 16-B units
    const size_t wseq = (size_t)wave * N * kLayers * kL * qcell;
    // the wave's slab regions as buffer descriptors: every record access is (lane offset, SGPR cell offset)
    const __amdgpu_buffer_rsrc_t rh = wave_rsrc(a.hseq + wseq, (size_t)N * kLayers * kL * qcell * 16);
    const __amdgpu_buffer_rsrc_t rc = wave_rsrc(a.cseq + wseq, (size_t)N * kLayers * kL * qcell * 16);
    const __amdgpu_buffer_rsrc_t rx = wave_rsrc(a.xw + (size_t)wave * N * kL * kWave, (size_t)N * kL * kWave * 8);

    unsigned long long st_fill = 0, st_l0 = 0, st_l2 = 0, st_head = 0;
    Pace turn;
    turn.turn = (threadIdx.x >> 8) & 1;   // waves w and w+4 share a SIMD: start out of phase
    const unsigned long long st_k0 = fstamp();
    for (int j = 0; j < N; ++j) {
        const unsigned long long st_w0 = fstamp();
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
        if (valid && q == 0) a.prediction[(size_t)b * N + j] = pred;   // Functions.py:1455,1466

        const uint32_t oj = (uint32_t)((size_t)j * kLayers * kL * qcell * 16);   // window j's cells, [layer][t]
#define SEQ_O(l, t) (oj + (uint32_t)(((l) * kL + (t)) * qcell * 16))
        const unsigned long long st_w1 = fstamp();
        st_head += st_w1 - st_w0;
        // ---- layers 0 and 1 together, time-major (Functions.py:374): layer 1's input h_t leaves layer 0's cell
        // already split in registers, so the slab holds it only for the backward; layer 1's fragments sit beside
        // the resident layer 0 for the phase, layer 2's replace them after it ----
        {
            const unsigned long long st_f0 = fstamp();
            if (!LP) lds_fill<G::FA1 * 4, kFwdWaves>(lw, a.p.fa[1]);   // its first barrier also publishes the resident blocks
            else if (j == 0) __syncthreads();   // f16 mode: every layer resident, never refilled
            const unsigned long long st_f1 = fstamp();
            st_fill += st_f1 - st_f0;
            const float *lw1 = LP ? lwl[1] : lw;
            float c1[HS], h1[HS];   // layer 1's c and the split record of its h
            float c2[LP ? HS : 1], h2[LP ? HS : 1];   // f16 mode: layer 2's
            {
                const float x0 = w0[0], x1 = w1[0];
                rot_left(w0);
                rot_left(w1);
                fwd16_cell<HS, true, true, LP>(lw0, lane, x0, x1, hp, hp, c, hout, turn);
                split_rec<HS, LP>(hout, hp);
                if (STORE) {
                    buf_store_rec<kRW>(rh, SEQ_O(0, 0), hp, lane);
                    buf_st2(rx, lane * 8, (uint32_t)(j * kL * kWave * 8), f32x2{x0, x1});
                    c_store<HS, LP>(rc, SEQ_O(0, 0), c, lane);
                }
                fwd16_cell<HS, false, true, LP>(lw1, lane, 0.0f, 0.0f, hp, h1, c1, hout, turn);
                split_rec<HS, LP>(hout, h1);
                if (STORE || !LP) buf_store_rec<kRW>(rh, SEQ_O(1, 0), h1, lane);   // f16 mode: layer 2 is in this phase
                if (STORE) c_store<HS, LP>(rc, SEQ_O(1, 0), c1, lane);
                if constexpr (LP) {   // every layer resident: layer 2 joins the phase (its h_t from registers as well)
                    fwd16_cell<HS, false, true, LP>(lwl[2], lane, 0.0f, 0.0f, h1, h2, c2, hout, turn);
                    split_rec<HS, LP>(hout, h2);
                    if (STORE) {
                        buf_store_rec<kRW>(rh, SEQ_O(2, 0), h2, lane);
                        c_store<HS, LP>(rc, SEQ_O(2, 0), c2, lane);
                    }
                }
            }
            for (int t = 1; t < kL; ++t) {
                const float x0 = w0[0], x1 = w1[0];
                rot_left(w0);
                rot_left(w1);
                fwd16_cell<HS, true, false, LP>(lw0, lane, x0, x1, hp, hp, c, hout, turn);
                split_rec<HS, LP>(hout, hp);
                if (STORE) {
                    buf_store_rec<kRW>(rh, SEQ_O(0, t), hp, lane);
                    buf_st2(rx, lane * 8, (uint32_t)((j * kL + t) * kWave * 8), f32x2{x0, x1});
                    if (t + 1 < kL) c_store<HS, LP>(rc, SEQ_O(0, t), c, lane);   // c_9 is never a c_{t-1}
                }
                fwd16_cell<HS, false, false, LP>(lw1, lane, 0.0f, 0.0f, hp, h1, c1, hout, turn);
                split_rec<HS, LP>(hout, h1);
                if (STORE || !LP) buf_store_rec<kRW>(rh, SEQ_O(1, t), h1, lane);
                if (STORE && t + 1 < kL) c_store<HS, LP>(rc, SEQ_O(1, t), c1, lane);
                if constexpr (LP) {
                    fwd16_cell<HS, false, false, LP>(lwl[2], lane, 0.0f, 0.0f, h1, h2, c2, hout, turn);
                    if (t + 1 < kL) {   // h_9 of layer 2 only feeds the readout (fp32 hout)
                        split_rec<HS, LP>(hout, h2);
                        if (STORE) {
                            buf_store_rec<kRW>(rh, SEQ_O(2, t), h2, lane);
                            c_store<HS, LP>(rc, SEQ_O(2, t), c2, lane);
                        }
                    }
                }
            }
            st_l0 += fstamp() - st_f1;
        }
        // ---- layer 2: its input sequence (layer 1's h) streamed back from the slab, one cell ahead ----
        if constexpr (!LP) {
            constexpr int l = 2;
            const unsigned long long st_f0 = fstamp();
            lds_fill<G::FA1 * 4, kFwdWaves>(lw, a.p.fa[l]);
            const float *lwc = lw;
            const unsigned long long st_f1 = fstamp();
            st_fill += st_f1 - st_f0;
            buf_load_quads<HS>(xc, rh, SEQ_O(l - 1, 0), lane);
            buf_load_quads<HS>(xn, rh, SEQ_O(l - 1, 1), lane);
            fwd16_cell<HS, false, true, LP>(lwc, lane, 0.0f, 0.0f, xc, hp, c, hout, turn);
            split_rec<HS, LP>(hout, hp);
            if (STORE) buf_store_rec<kRW>(rh, SEQ_O(l, 0), hp, lane);
            if (STORE) c_store<HS, LP>(rc, SEQ_O(l, 0), c, lane);
#pragma unroll
            for (int r = 0; r < HS; ++r) xc[r] = xn[r];
#pragma unroll 3
            for (int t = 1; t < kL; ++t) {
                buf_load_quads<HS>(xn, rh, SEQ_O(l - 1, t + 1 < kL ? t + 1 : t), lane);
                fwd16_cell<HS, false, false, LP>(lwc, lane, 0.0f, 0.0f, xc, hp, c, hout, turn);
                if (t + 1 < kL) {   // h_9 of layer 2 only feeds the readout (fp32 hout)
                    split_rec<HS, LP>(hout, hp);
                    if (STORE) buf_store_rec<kRW>(rh, SEQ_O(l, t), hp, lane);
                }
                if (STORE && t + 1 < kL) c_store<HS, LP>(rc, SEQ_O(l, t), c, lane);
#pragma unroll
                for (int r = 0; r < HS; ++r) xc[r] = xn[r];
            }
            st_l2 += fstamp() - st_f1;
        }
#undef SEQ_O
        // ---- readout fc(h_9 of layer 2) (Functions.py:377) ----
        float xo[kOut];
#pragma unroll
        for (int o = 0; o < kOut; ++o) {
            float p = 0.0f;
#pragma unroll
            for (int r = 0; r < HS; ++r) p += lfcp_j[(o * HS + r) * 4 + q] * hout[r];
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
#if FCR_STAMP
    if (lane == 0) {
        unsigned long long *o = a.stamp + (size_t)wave * 8;
        o[0] = st_head;
        o[1] = st_l0;
        o[2] = st_fill;
        o[3] = st_l2;
        o[4] = fstamp() - st_k0;
        o[5] = o[6] = o[7] = 0;
    }
#endif
}

}  // namespace fcr
