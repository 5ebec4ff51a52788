// fcr_pipe.h — layer- and window-pipelined small-batch rollout (config 1: the reference trains at B = 15,
// UL/Main.py:84,297).
//
// The small-batch kernels (fcr_small.h) give a 16-trajectory group ONE workgroup that walks every cell of the rollout
// in sequence: per window 30 dependent cells (3 layers x 10 steps) plus two weight-image refills, in both passes. Here
// a group gets, per window set, one workgroup per LSTM layer in the backward (3 S) and two in the forward (2 S: layers
// 0 and 1 time-major in one, their fragments fit one LDS together; layer 2 and the heads in the other), each holding
// its layers' weights resident in LDS (no refills). Set s of S takes the windows j = s, s + S, ... (forward; backward N-1-s, N-1-s-S, ...): every window is an
// LSTM run from zero state, so the windows of different sets run at once and the layers run as a wavefront across
// workgroups — cell (j, l, t) needs (j, l, t - 1) of its own workgroup and, from the layer below (forward) or above
// (backward), the same cell's input, handed over through the sequence slabs (the layout fcr_small.h / the fused
// kernels use) and a per-workgroup progress counter (pipe_wait / pipe_signal, fcr_small.h).
// What remains serial is the prediction feedback. Forward: window j's row t is row j + t of the extended sequence,
// for j + t >= 10 the output (x_hat, u) of window j + t - 10, handed from that window's layer-2 workgroup as a row;
// so the chain is one cell per layer per window (j, t = 9) -> the head -> (j + 1, 9), with two hand-offs (layer 1 ->
// layer 2, the head's row -> layer 0). Backward: window j's head needs
// the row gradient of row j + 10, i.e. the first layer-0 cells of windows j + 1 .. j + S.
// Within a workgroup, cells run exactly as fcr_small.h runs them (wave w owns the slots of record quad w; the same
// fwd16_cell / sb_step arithmetic, the same LDS exchange and fixed-order reductions), and the cost sums are formed
// in window order from the rows at the end, so results are bit-identical to the small-batch kernels' for every S.
// Co-residency: a workgroup may wait on another of its launch, so the host runs this family only when every
// workgroup fits the device at once (<= 3 S x groups <= CUs / 2; a CU holds at least one) and bounds every wait.
// Placement: the workgroups of a group get block ids of one residue mod 8, i.e. one XCD (one L2).
#pragma once
#include "fcr_small.h"

namespace fcr {

template <int HS>
struct Pipe {
    static constexpr int NQ = Small<HS>::NQ;
    // per window set, one progress counter per producing workgroup (the count of its cells whose outputs are
    // signalled): forward layer 0, layer 1, the layer-2 workgroup's hand-off rows; backward layers 0, 1, 2
    static constexpr int F0 = 0, F1 = 1, ROW = 2, BWD = 3, PER_SET = 6;
    static constexpr int MAX_SETS = 4;       // forward (2 workgroups per set)
    static constexpr int MAX_SETS_BWD = 3;   // backward (3 workgroups per set)
    static_assert(MAX_SETS * PER_SET <= kPipeAbort - 2, "pipe counters");
    // forward, layers 0 + 1: [layer 0's fragments | layer 1's | h exchange (one record slot per layer)];
    //          layer 2:      [layer 2's fragments | controller records | fc.weight | fc.bias | h exchange]
    static constexpr int LDS_FWD01 = (Geo16<HS>::FA0 + Geo16<HS>::FA1) * 4 + Small<HS>::XBUF;
    static constexpr int LDS_FWD2 = (Geo16<HS>::FA1 + Geo16<HS>::FNP + Geo16<HS>::FCP + 4) * 4 + Small<HS>::XBUF;
    static constexpr int LDS_FWD = LDS_FWD01 > LDS_FWD2 ? LDS_FWD01 : LDS_FWD2;
    // backward: [layer image (resident) | controller records | fc.weight | partial products]
    static constexpr int LDS_BWD = BwdLds<HS, false>::BYTES + Small<HS>::RED;
    static_assert(LDS_FWD <= 163840 && LDS_BWD <= 163840, "pipe LDS");   // at least one workgroup per CU
};
// the hand-off row of window j, per trajectory: x_hat_j (floats 0..3, lane group q's column q), u_{j+1} (4), and the
// step's cost terms err_j (5), con_j (6) for the in-order sums at the end
constexpr int kPipeRow = 8;   // floats per trajectory and window

struct PipeArgs {
    unsigned *flags;   // [groups][kPipeFlags], zeroed before each launch
    float *rows;       // [groups][N][16][kPipeRow]
    int groups;
    float *loss;       // forward: the batch mean (the last group to finish reduces the per-group sums)
};

// The counters are zeroed by each forward call's pack_all_kernel (fcr_abi.hip), ahead of the forward and its backward
// on the call's stream, by a kernel rather than hipMemsetAsync: a memset captured into a HIP graph left stale counters
// in replays (the consumers ran ahead on the previous replay's rows: profiles/round6_b15_pipe_graph.log); a kernel node
// has the ordering and the release / acquire of any kernel boundary. A backward leaves its own counters zeroed (the
// last of a group's workgroups to arrive resets them), so a second backward of the same forward starts clean.
constexpr int kPipeArrive = kPipeAbort - 1;   // backward: the group's workgroups that have finished
constexpr int kPipeLossArrive = kPipeAbort - 2;   // forward, group 0's word: the groups whose cost sums are stored

// block id -> (group, role, window set), R roles per set (forward 2: layers 0 + 1, layer 2; backward 3: one per
// layer): the ids of one group share their residue mod 8 (one XCD); -1: an unused id
template <int S, int R>
__device__ __forceinline__ int pipe_role(int groups, int &role, int &set) {
    const int id = blockIdx.x, xcd = id & 7, k = id >> 3;
    const int rs = k % (R * S);
    role = rs % R;
    set = rs / R;
    const int grp = xcd + 8 * (k / (R * S));
    return grp < groups ? grp : -1;
}
// windows of set s: ceil((N - s) / S) (the host keeps S <= N, so every set has one)
template <int S>
__device__ __forceinline__ int pipe_windows(int N, int s) { return (N - s + S - 1) / S; }

// ---------------------------------------------------------------------------------------------------
// forward. Two workgroups per (group, window set): layers 0 and 1 time-major in one (layer 1's input is the record
// layer 0 just made, in registers, as in the fused kernel's first phase: no hand-off between them), layer 2 and the
// window heads in the other. Per cell (local index m = i * 10 + t over the workgroup's windows j = s + S i): the gates
// of this wave's slots, the h exchange through LDS (one barrier), then this wave's quad of the h record (and c) — the
// layer-1 record write-through, as the layer-2 workgroup reads it — and at the NEXT cell's barrier, all four waves
// having drained those stores, one lane signals m + 1 layer-1 cells done; a window's last cell (on the cross-window
// chain) is published at once. Layer 2 prefetches its input records (sc1) up to two cells ahead, as far as published.
// ---------------------------------------------------------------------------------------------------
template <int HS, bool STORE, int S>
__global__ __launch_bounds__(Small<HS>::NQ * kWave, 1) void fcr_pfwd_kernel(FwdArgs a, PipeArgs pa) {
    using G = Geo16<HS>;
    using P = Pipe<HS>;
    int role, set;
    const int grp = pipe_role<S, 2>(pa.groups, role, set);
    if (grp < 0) return;   // uniform over the workgroup
    const int layer = role == 0 ? 0 : 2;   // 0: layers 0 and 1, 2: layer 2 and the heads
    extern __shared__ __attribute__((aligned(16))) float lw[];
    float *lw1 = lw + G::FA0;               // (layers 0 + 1) layer 1's fragments
    float *lfnp = lw + G::FA1;              // (layer 2) controller records, fc.weight, fc.bias
    float *lfcp = lfnp + G::FNP;
    float *lfcb = lfcp + G::FCP;
    f32x4 *xbuf = reinterpret_cast<f32x4 *>(layer == 0 ? lw + G::FA0 + G::FA1 : lfcb + 4);
    constexpr int RECB = Geo<HS>::QC * 16;
    if (layer == 0) {
        lds_copy(lw, a.p.fa[0], G::FA0);
        lds_copy(lw1, a.p.fa[1], G::FA1);
    } else {
        lds_copy(lw, a.p.fa[2], G::FA1);
        lds_copy(lfnp, a.p.fnp, G::FNP);
        lds_copy(lfcp, a.p.fcp, G::FCP);
        lds_copy(lfcb, a.p.fcb, 4);
    }
    const int lane = threadIdx.x & 63;
    const int q = lane >> 4, sl = lane & 15;
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int b = grp * kTile + sl;
    const bool valid = b < a.B;
    const bool lead = w == 0;
    const int bc = valid ? b : a.B - 1;
    const int N = a.N;
    const int nwin = pipe_windows<S>(N, set);
    const int NC = nwin * kL;   // cells of the workgroup per layer (its windows)
    const float alpha = a.alpha;
    unsigned *fl = pa.flags + (size_t)grp * kPipeFlags;
    unsigned *fs = fl + set * P::PER_SET;   // this window set's counters
    float *rowbuf = pa.rows + (size_t)grp * N * kTile * kPipeRow;
    auto row_of = [&](int j) { return rowbuf + ((size_t)j * kTile + sl) * kPipeRow; };   // window j's hand-off row
    auto row_ready = [&](int j) { pipe_wait(fl, fl + (j % S) * P::PER_SET + P::ROW, (unsigned)(j / S + 1)); };

    const float ref = a.X[(size_t)bc * kCtrlIn + 2];                 // Functions.py:1392
    const float *st = a.states + (size_t)bc * kL * kIn;
    const float scq = a.p.wsc[q], sc4 = a.p.wsc[4];
    const float u0 = a.u0[bc];

    float c[HS], hout[HS], hp[HS];
#pragma unroll
    for (int r = 0; r < HS; ++r) c[r] = hout[r] = hp[r] = 0.0f;
    const size_t qcell = (size_t)Geo<HS>::QC;
    const size_t seq = (size_t)N * kLayers * kL * qcell;
    f32x4 *hs_wave = a.hseq + (size_t)grp * seq;
    f32x4 *cs_wave = a.cseq + (size_t)grp * seq;
    const __amdgpu_buffer_rsrc_t rh = wave_rsrc(a.hseq + (size_t)grp * seq, seq * 16);
    f32x2 *xw_wave = a.xw + (size_t)grp * N * kL * kWave;
    auto hoff = [&](int n, int l) {   // byte offset of cell n = j * 10 + t of layer l in the group's h slab
        return (uint32_t)((((size_t)(n / kL) * kLayers + l) * kL + n % kL) * qcell * 16);
    };
    auto nglob = [&](int m) { return (set + S * (m / kL)) * kL + m % kL; };   // local cell m -> cell index j * 10 + t
    Pace turn;
    turn.turn = 0;
    __syncthreads();
    if (layer == 0) {
        // ---- layers 0 and 1. Layer 0's input: the window's rows (B-operand layout), rotated so the current cell's
        // row is at [0]; a row of the extended sequence past row 9 is a hand-off row, loaded when its cell comes (the
        // last S rows of a window) ----
        float c1[HS], hout1[HS], hp1[HS];
#pragma unroll
        for (int r = 0; r < HS; ++r) c1[r] = hout1[r] = hp1[r] = 0.0f;
        float w0[kL], w1[kL];
#pragma unroll
        for (int t = 0; t < kL; ++t) {
            const int r = set + t;   // the first window's rows below 10: the states, u0 in row 9 (Functions.py:1395-1396)
            w0[t] = r < kL ? st[(r < kL ? r : 0) * kIn + q] * scq : 0.0f;
            w1[t] = (q == 0 && r < kL) ? (r == kL - 1 ? u0 : st[(r < kL ? r : 0) * kIn + 4]) * sc4 : 0.0f;
        }
        char *xb0 = reinterpret_cast<char *>(xbuf), *xb1 = xb0 + RECB;   // one exchange slot per layer
        for (int i = 0; i < nwin; ++i) {
            const int j = set + S * i;
            if (i > 0) {   // Functions.py:1433-1434: the window slides by S rows between this workgroup's windows
#pragma unroll
                for (int k = 0; k + S < kL; ++k) {
                    w0[k] = w0[k + S];
                    w1[k] = w1[k + S];
                }
            }
            for (int t = 0; t < kL; ++t) {
                const int m = i * kL + t, n = j * kL + t;
                if (t >= kL - S && j + t >= kL) {   // row j + t = (x_hat, u) of window j + t - 10
                    const int src = j + t - kL;
                    row_ready(src);
                    const float *rw = row_of(src);
                    const float xq = __hip_atomic_load(rw + q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    const float uj = __hip_atomic_load(rw + 4, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    w0[0] = xq * scq;                                  // x_hat, column q
                    w1[0] = (q == 0) ? uj * sc4 : 0.0f;                // u
                }
                const float x0 = w0[0], x1 = w1[0];
                rot_left(w0);
                rot_left(w1);
                // layer 0 (Functions.py:374)
                by_quad<HS>(w, [&](auto Wc) {
                    constexpr int W = decltype(Wc)::v;
                    using Q = QR<HS, W>;
                    if (t == 0) fwd16_cell<HS, true, true, false, Q::R0, Q::R1>(lw, lane, x0, x1, hp, hp, c, hout, turn);
                    else fwd16_cell<HS, true, false, false, Q::R0, Q::R1>(lw, lane, x0, x1, hp, hp, c, hout, turn);
                    xrec_put<HS, W>(xb0, hout, lane);
                });
                pipe_drain();   // this wave's record stores of the previous cells (long complete)
                lds_barrier();
                pipe_signal(fs + P::F1, (unsigned)m);
                load_quads<HS>(hp, reinterpret_cast<const f32x4 *>(xb0), lane);   // the whole split record of h_t
                by_quad<HS>(w, [&](auto Wc) {
                    constexpr int W = decltype(Wc)::v;
                    store_quad<HS, W>(hs_wave + (size_t)hoff(n, 0) / 16, hp, lane);
                    if (STORE && t + 1 < kL) store_quad<HS, W>(cs_wave + (size_t)hoff(n, 0) / 16, c, lane);
                });
                if (STORE && lead) xw_wave[(size_t)n * kWave + lane] = f32x2{x0, x1};
                // layer 1, time-major: its input is layer 0's record of this step, in registers
                by_quad<HS>(w, [&](auto Wc) {
                    constexpr int W = decltype(Wc)::v;
                    using Q = QR<HS, W>;
                    if (t == 0) fwd16_cell<HS, false, true, false, Q::R0, Q::R1>(lw1, lane, 0.0f, 0.0f, hp, hp1, c1, hout1, turn);
                    else fwd16_cell<HS, false, false, false, Q::R0, Q::R1>(lw1, lane, 0.0f, 0.0f, hp, hp1, c1, hout1, turn);
                    xrec_put<HS, W>(xb1, hout1, lane);
                });
                lds_barrier();
                load_quads<HS>(hp1, reinterpret_cast<const f32x4 *>(xb1), lane);
                by_quad<HS>(w, [&](auto Wc) {
                    constexpr int W = decltype(Wc)::v;
                    st_quad_sc1<HS, W>(rh, hoff(n, 1), hp1, lane);   // the layer-2 workgroup's input
                    if (STORE && t + 1 < kL) store_quad<HS, W>(cs_wave + (size_t)hoff(n, 1) / 16, c1, lane);
                });
                if (t == kL - 1) {   // the window's last cell is on the cross-window chain: published at once
                    pipe_drain();
                    lds_barrier();
                    pipe_signal(fs + P::F1, (unsigned)(m + 1));
                }
            }
        }
        pipe_drain();
        __syncthreads();
        pipe_signal(fs + P::F1, (unsigned)NC);
        return;
    }
    // ---- layer 2: input records from layer 1 (sc1), up to two cells ahead ----
    constexpr bool keep_h = STORE;
    unsigned *below = fs + P::F1;
    if (set == 0 && lead && valid && q == 0) a.prediction[(size_t)b * N] = u0;   // Functions.py:1455
    // the input records of cells m, m + 1, m + 2, prefetched as far as the layer below has published them (a record
    // that was late is waited for at its cell: a late input never stalls the cell before it)
    f32x4 xa[Geo<HS>::HQ], xn[Geo<HS>::HQ], xf[Geo<HS>::HQ];
#pragma unroll
    for (int k = 0; k < Geo<HS>::HQ; ++k) xn[k] = xf[k] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
    bool have_a = false, have_n = false;
    for (int i = 0; i < nwin; ++i) {
        const int j = set + S * i;
        for (int t = 0; t < kL; ++t) {
            const int m = i * kL + t, n = j * kL + t;
            if (!have_a) {
                pipe_wait(fl, below, (unsigned)(m + 1));
                ld_rec_sc1<HS>(xa, rh, hoff(nglob(m), layer - 1), lane);
            }
            const bool last = t + 1 == kL;   // h_9 of layer 2: the readout's, in fp32
            char *xb = reinterpret_cast<char *>(xbuf) + (t & 1) * RECB;
            float xc[HS];
#pragma unroll
            for (int r = 0; r < HS; ++r) xc[r] = xa[r >> 2][r & 3];
            by_quad<HS>(w, [&](auto Wc) {
                constexpr int W = decltype(Wc)::v;
                using Q = QR<HS, W>;
                if (t == 0) fwd16_cell<HS, false, true, false, Q::R0, Q::R1>(lw, lane, 0.0f, 0.0f, xc, hp, c, hout, turn);
                else fwd16_cell<HS, false, false, false, Q::R0, Q::R1>(lw, lane, 0.0f, 0.0f, xc, hp, c, hout, turn);
                if (last) xchg_put<HS, W>(reinterpret_cast<f32x4 *>(xb), hout, lane);
                else xrec_put<HS, W>(xb, hout, lane);
            });
            pipe_drain();   // this wave's record stores of the previous cell and its prefetches
            bool have_f = false;
            {
                const unsigned avail = pipe_count(below);
                if (!have_n && m + 1 < NC && avail >= (unsigned)(m + 2)) {
                    ld_rec_sc1<HS>(xn, rh, hoff(nglob(m + 1), layer - 1), lane);
                    have_n = true;
                }
                if (have_n && m + 2 < NC && avail >= (unsigned)(m + 3)) {
                    ld_rec_sc1<HS>(xf, rh, hoff(nglob(m + 2), layer - 1), lane);
                    have_f = true;
                }
            }
            lds_barrier();
            if (last) {
                xchg_get<HS>(reinterpret_cast<const f32x4 *>(xb), hout, lane);
            } else {
                load_quads<HS>(hp, reinterpret_cast<const f32x4 *>(xb), lane);
                if (keep_h)
                    by_quad<HS>(w, [&](auto Wc) { st_quad_sc1<HS, decltype(Wc)::v>(rh, hoff(n, layer), hp, lane); });
            }
            if (STORE && t + 1 < kL)
                by_quad<HS>(w, [&](auto Wc) {
                    store_quad<HS, decltype(Wc)::v>(cs_wave + (size_t)hoff(n, layer) / 16, c, lane);
                });
#pragma unroll
            for (int k = 0; k < Geo<HS>::HQ; ++k) {
                xa[k] = xn[k];
                xn[k] = xf[k];
            }
            have_a = have_n;
            have_n = have_f;
        }
        // ---- layer 2, end of window j: readout fc(h_9) (Functions.py:377), its cost terms, the next command ----
        const float *lfnp_j = opaque(lfnp), *lfcp_j = opaque(lfcp), *lfcb_j = opaque(lfcb);
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
        const float xh0 = xo[0], xh1 = xo[1], xh2 = xo[2], xh3 = xo[3];
        const float mine = sel4(q, xh0, xh1, xh2, xh3);
        if (lead && valid) {
            a.xhat_ws[((size_t)b * N + j) * kOut + q] = mine;
            if (a.xhat_user) a.xhat_user[((size_t)b * N + j) * kOut + q] = mine;
        }
        const float err = sq(xh0 - ref);                              // Functions.py:1405-1414, 1443-1452
        const float con = relu(-xh1) + relu(-xh2) + relu(xh1 - kP1Max) + relu(xh2 - kP2Max);
        float un = 0.0f;
        if (j + 1 < N) {                                               // Functions.py:1421-1434
            float z[kMS];
            un = hardtanh(fnn_pre(lfnp_j, q, xh0, xh3, ref, z));
            if (lead && valid && q == 0) a.prediction[(size_t)b * N + j + 1] = un;   // Functions.py:1466
        }
        if (lead) {   // the hand-off row of window j (write-through; only this wave stores it), then its counter
            float *rw = row_of(j);
            __hip_atomic_store(rw + q, mine, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (q == 0) {
                __hip_atomic_store(rw + 4, un, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                __hip_atomic_store(rw + 5, err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                __hip_atomic_store(rw + 6, con, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
            pipe_drain();
            pipe_signal(fs + P::ROW, (unsigned)(i + 1));
        }
    }
    // ---- the sums over the steps, in window order (Functions.py:1441-1460), by the workgroup of window N - 1 ----
    if (set != (N - 1) % S || !lead) return;
    for (int k = 0; k < S; ++k) pipe_wait(fl, fl + k * P::PER_SET + P::ROW, (unsigned)pipe_windows<S>(N, k));
    float u_prev = u0;
    float cmd_j = alpha * sq(st[(kL - 2) * kIn + 4] - u0);            // Functions.py:1405
    float cmd_sum = 0.0f, err_sum = 0.0f, tot_sum = 0.0f;
    for (int j = 0; j < N; ++j) {
        const float *rw = row_of(j);
        const float err = __hip_atomic_load(rw + 5, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const float con = __hip_atomic_load(rw + 6, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        tot_sum += (err + cmd_j) + con;
        err_sum += err;
        cmd_sum += cmd_j;
        if (j + 1 < N) {
            const float un = __hip_atomic_load(rw + 4, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            cmd_j = alpha * sq(u_prev - un);                           // Functions.py:1446
            u_prev = un;
        }
    }
    // every wait of the chains ends before this one: a timed-out one anywhere shows as NaN cost and loss
    const float cost = pipe_aborted(fl) ? __builtin_nanf("") : tot_sum / (float)N;   // Functions.py:1458-1460
    if (valid && q == 0) {
        a.cost[b] = cost;
        a.command[b] = cmd_sum / (float)N;
        a.error[b] = err_sum / (float)N;
    }
    float part = (valid && q == 0) ? cost : 0.0f;
#pragma unroll
    for (int m = 1; m < 64; m <<= 1) part += __shfl_xor(part, m);
    // the loss (no loss_reduce_kernel launch): each group's sum goes out write-through, then an arrival; the last group
    // to arrive sums them in loss_reduce_kernel's order (fcr_pack.h: its tree over 256 slots, of which the first
    // groups <= 32 are non-zero) and divides by B
    if (lane == 0) __hip_atomic_store(a.loss_part + grp, part, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    pipe_drain();
    unsigned prev = 0u;
    if (lane == 0) prev = __hip_atomic_fetch_add(pa.flags + kPipeLossArrive, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    prev = __builtin_amdgcn_readfirstlane(prev);
    if (prev + 1u != (unsigned)pa.groups) return;
    float v = lane < pa.groups ? __hip_atomic_load(a.loss_part + lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0.0f;
#pragma unroll
    for (int wd = 16; wd > 0; wd >>= 1) {
        const float o = __shfl_down(v, wd);
        if (lane < wd) v = v + o;
    }
    if (lane == 0) pa.loss[0] = v / (float)a.B;
}

// ---------------------------------------------------------------------------------------------------
// backward: each (layer, window set) workgroup runs fcr_sbwd_kernel's per-layer phases (sb_phase, PIPE) over its
// windows j = N-1-s, N-1-s-S, ...; layer 2's also their heads (cost gradients, the controller backward, dh_9), layer
// 0's the window-row gradients (each wave its own copy, fcr_small.h), and the layer-0 workgroup of window 0 g_u0
// ---------------------------------------------------------------------------------------------------
template <int HS, int S>
__global__ __launch_bounds__(Small<HS>::NQ * kWave, 1) void fcr_pbwd_kernel(BwdArgs a, PipeArgs pa) {
    using LD = BwdLds<HS, false>;
    using I1 = Img<HS, false>;
    using I0 = Img<HS, true>;
    using P = Pipe<HS>;
    constexpr int NQ = P::NQ;
    int layer, set;
    const int grp = pipe_role<S, 3>(pa.groups, layer, set);
    if (grp < 0) return;
    extern __shared__ __attribute__((aligned(16))) float lw[];
    float *lfnp = lw + LD::REGION / 4;
    float *lfcp = lfnp + LD::FNP;
    if (layer == 0) lds_copy(lw, a.p.img[0], I0::BYTES / 4);
    else lds_copy(lw, a.p.img[layer], I1::BYTES / 4);
    if (layer == 2) {
        lds_copy(lfnp, a.p.fnp, LD::FNP);
        lds_copy(lfcp, a.p.fcp, LD::FCP);
    }
    __syncthreads();
    const int lane = threadIdx.x & 63;
    const int q = lane >> 4, sl = lane & 15;
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int b = grp * kTile + sl;
    const bool valid = b < a.B;
    const bool lead = w == 0;
    const int bc = valid ? b : a.B - 1;
    const int N = a.N;
    const float alpha = a.alpha;
    const float wgt = valid ? a.dloss[0] / ((float)a.B * (float)N) : 0.0f;   // Functions.py:1458, 1463
    const float ref = a.X[(size_t)bc * kCtrlIn + 2];
    const float s84 = a.states[(size_t)bc * kL * kIn + (kL - 2) * kIn + 4];
    const float *pred = a.prediction + (size_t)bc * N;
    const float *xh = a.xhat + (size_t)bc * N * kOut;

    SbCtx<HS, true> x;
    {
        const ImgLane<I1::U> L1 = img_lane<I1::U>(lds_offset(lw), lane);
        const ImgLane<I0::U> L0 = img_lane<I0::U>(lds_offset(lw), lane);
        x.fb1 = L1.fb;
        x.tb1 = L1.tb;
        x.fb0 = L0.fb;
        x.tb0 = L0.tb;
    }
    x.lane = lane;
    x.N = N;
    Stamps sp = {{0, 0, 0, 0, 0, 0, 0, 0}};
    x.sp = &sp;
    x.scq = a.p.wsc[q];
    x.sc4 = a.p.wsc[4];
    x.red = reinterpret_cast<f32x4 *>(lw + LD::BYTES / 4);
    x.rr = wave_rsrc(a.dxrow + ((size_t)grp * NQ + w) * N * kL * kWave, (size_t)N * kL * kWave * 8);
    const size_t qcell = (size_t)Geo<HS>::QC;
    const size_t seq_sz = (size_t)N * kLayers * kL * qcell;
    const size_t dseq_sz = (size_t)N * 2 * kL * qcell;
    x.nb.rh = wave_rsrc(a.hseq + (size_t)grp * seq_sz, seq_sz * 16);
    x.nb.rc = wave_rsrc(a.cseq + (size_t)grp * seq_sz, seq_sz * 16);
    x.nb.rx = wave_rsrc(a.xw + (size_t)grp * N * kL * kWave, (size_t)N * kL * kWave * 8);
    x.nb.rd = wave_rsrc(a.dseq + (size_t)grp * dseq_sz, dseq_sz * 16);
    x.dseq_w = a.dseq + (size_t)grp * dseq_sz;
    unsigned *fl = pa.flags + (size_t)grp * kPipeFlags;
    x.flags = fl;
    x.S = S;
    x.din_pending = false;
    x.fl_own = set * P::PER_SET + P::BWD + layer;
    x.fl_above = layer < 2 ? set * P::PER_SET + P::BWD + layer + 1 : -1;
    const int nwin = pipe_windows<S>(N, set);
    const int j0 = N - 1 - set;   // this workgroup's first window (then j0 - S, ...)
    // the layer-0 counter of window v's set, and its count once v's cell t is done (x.done_after in that set's order)
    auto l0_done = [&](int v, int t) {
        pipe_wait(fl, fl + ((N - 1 - v) % S) * P::PER_SET + P::BWD, (unsigned)((N - 1 - v) / S * kL + (kL - 1 - t) + 1));
    };
    auto row_grad = [&](int rho) {   // sum over windows v = max(0, rho-9) .. min(N-1, rho) of dx(v, rho-v)
        f32x2 acc2 = {0.0f, 0.0f};
        const int w_hi = rho < N - 1 ? rho : N - 1;
        const int w_lo = rho - (kL - 1) > 0 ? rho - (kL - 1) : 0;
        // another workgroup's (layer 0's) write-through rows: sc1 loads
        for (int v = w_hi; v >= w_lo; --v) acc2 += buf_ld2_sc1(x.rr, lane * 8, (uint32_t)((v * kL + (rho - v)) * kWave * 8));
        return acc2;
    };
    float dh[HS], dc[HS];
#pragma unroll
    for (int r = 0; r < HS; ++r) dh[r] = dc[r] = 0.0f;
    CellIn<HS> ci;
    {   // the first cell (j0, layer, 9): its x, h (forward records), c and din (the layer above's first cell)
        if (layer < 2) pipe_wait(fl, fl + x.fl_above, x.done_after(j0, kL - 1));
        const NextIn f = x.next_of(j0 + S, layer, 0);   // the cell after (j0 + S, layer, 0) = (j0, layer, 9)
        by_quad<HS>(w, [&](auto Wc) {
            constexpr int W = decltype(Wc)::v;
            if (layer == 0) sb_load_a<HS, true, true>(ci, f, lane);
            else sb_load_a<HS, false, true>(ci, f, lane);
            if (layer < 2) sb_load_b<HS, W, true, true, true>(ci, f, lane);   // din: the layer above's (sc1)
            else sb_load_b<HS, W, true, false>(ci, f, lane);
        });
    }
    float dh_out[HS];
#pragma unroll
    for (int r = 0; r < HS; ++r) dh_out[r] = 0.0f;
    for (int j = j0; j >= 0; j -= S) {
        if (layer == 2) {   // ---- window head (Functions.py:1443-1452, 1424-1430, 377) ----
            const float *lfnp_j = opaque(lfnp), *lfcp_j = opaque(lfcp);
            const float x0 = xh[j * kOut + 0], x1 = xh[j * kOut + 1], x2 = xh[j * kOut + 2], x3 = xh[j * kOut + 3];
            const float uj = pred[j], uj1 = pred[j + 1 < N ? j + 1 : j], uj2 = pred[j + 2 < N ? j + 2 : j];
            float d0 = wgt * 2.0f * (x0 - ref);
            float d1 = wgt * ((-x1 > 0.0f ? -1.0f : 0.0f) + (x1 - kP1Max > 0.0f ? 1.0f : 0.0f));
            float d2 = wgt * ((-x2 > 0.0f ? -1.0f : 0.0f) + (x2 - kP2Max > 0.0f ? 1.0f : 0.0f));
            float d3 = 0.0f;
            if (j <= N - 2) {
                // row 10 + j sums dx(v, 10 + j - v) over windows v = j + 1 .. j + 10: each set's latest is among
                // v = j + 1 .. j + S (its cell t = 10 + j - v), the rest came before it in that set's order
                for (int v = j + 1; v <= j + S && v < N; ++v) l0_done(v, kL + j - v);
                const f32x2 Gr = row_grad(kL + j);
                d0 += __shfl(Gr[0], sl);
                d1 += __shfl(Gr[0], sl + 16);
                d2 += __shfl(Gr[0], sl + 32);
                d3 += __shfl(Gr[0], sl + 48);
                const float g4 = __shfl(Gr[1], sl);
                float du = 2.0f * alpha * wgt * (uj1 - uj);
                if (j + 2 < N) du += 2.0f * alpha * wgt * (uj1 - uj2);
                du += g4;
                float z[kMS];
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
#pragma unroll
            for (int r = 0; r < HS; ++r) {
                const float *fp = lfcp_j + r * 4 + q;
                dh_out[r] = fp[0] * d0 + fp[HS * 4] * d1 + fp[2 * HS * 4] * d2 + fp[3 * HS * 4] * d3;
            }
            by_quad<HS>(w, [&](auto Wc) { sb_phase<HS, 2, decltype(Wc)::v>(x, j, dh_out, ci, dh, dc); });
        } else if (layer == 1) {
            by_quad<HS>(w, [&](auto Wc) { sb_phase<HS, 1, decltype(Wc)::v>(x, j, dh_out, ci, dh, dc); });
        } else {
            by_quad<HS>(w, [&](auto Wc) { sb_phase<HS, 0, decltype(Wc)::v>(x, j, dh_out, ci, dh, dc); });
        }
    }
    pipe_drain();   // the last cell's outputs, signalled once every wave has drained them
    __syncthreads();
    pipe_signal(fl + x.fl_own, (unsigned)(nwin * kL));
    if (layer == 0 && set == (N - 1) % S) {
        // row 9 (its col 4 = u0, Functions.py:1396) sums dx(v, 9 - v) over windows 0 .. 9: every set's layer 0 done
        for (int k = 0; k < S; ++k) pipe_wait(fl, fl + k * P::PER_SET + P::BWD, (unsigned)(pipe_windows<S>(N, k) * kL));
        const float g_u0_rows = row_grad(kL - 1)[1];
        float du0 = 2.0f * alpha * wgt * (pred[0] - s84);
        if (N > 1) du0 += 2.0f * alpha * wgt * (pred[0] - pred[1]);
        // layer 0 ends the chain: a timed-out wait anywhere shows as NaN gradients
        if (lead && valid && q == 0) a.g_u0[b] = pipe_aborted(fl) ? __builtin_nanf("") : g_u0_rows + du0;
    }
    // every wave of this workgroup is past its last counter read: arrive; the group's last arrival zeroes the backward
    // counters for a later backward of the same forward
    __syncthreads();
    if (threadIdx.x == 0) {
        const unsigned prev = __hip_atomic_fetch_add(fl + kPipeArrive, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (prev == (unsigned)(3 * S - 1)) {
            for (int k = 0; k < S; ++k)
                for (int l = 0; l < 3; ++l)
                    __hip_atomic_store(fl + k * P::PER_SET + P::BWD + l, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(fl + kPipeArrive, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
}

}  // namespace fcr
