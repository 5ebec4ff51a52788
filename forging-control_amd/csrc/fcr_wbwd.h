// fcr_wbwd.h — H > 52 (config 5): ONE kernel per backward cell: the cell's gate gradients (the backward of the LSTM
// cell update) formed in the prologue of the gradient product
// [input grad | dh_{t-1}] = dG · [W_ih | W_hh], so the dgate rows never go to HBM. Reference: the autograd backward of
// nn.LSTM inside loss.backward() (Functions.py:325, :655).
//
// Product: out[b][n] = sum_r dG[b][r] W[r][n] over the 4H gate rows r, fp32-accurate from f16 halves: with dG = dG_hi
// + dG_lo (each trajectory row's dgates times its own power of two) and W = W_hi + W_lo,
//   out = (W_lo dG_hi + W_hi dG_lo + W_hi dG_hi) / scale_b    (three MFMAs per k-block; the dropped lo·lo <= 2^-22)
// A = W^T split, [NP][4H / 32][hi (32) | lo (32)] (row n = output column, W_ih column n for n < H, W_hh column n - H;
// layer 0: W_hh only; a K step's halves of one row are one 128-B line) with the K index UNIT-major, r' = 4 unit + gate
// (wide_split_bt_kernel), so a K step of 32 is 8 whole units: the dgates of one K step need only those units' inputs.
// Tile (WbG256, layer 0): a workgroup owns 256 output columns x 128 trajectories, and its 8 waves split by ROLE
// (round 4): waves 0-3 produce the B tiles (the step's dgates, hi | lo), waves 4-7 consume them (each 64 columns x all
// 128 trajectories = 4 x 8 D tiles; lane = trajectory, 4 consecutive columns: one 16-B store). Layers >= 1 run
// WbG256w (256 x 256, 4 + 8 waves, round 5). Wave w runs on SIMD w % 4, so every SIMD
// holds one producer and one consumer: the producer's transcendental chains issue while its partner's MFMAs run
// (with every wave doing both in turn, the step barrier lined the two waves of a SIMD up on the same phase, and the
// dgate chains were the critical path: 247 ms of backward against 168 ms with the activations stubbed out). K in
// steps of 32: A through a 2-stage LDS-DMA ring (W^T is L2-resident), in whole 128-B lines, issued by the producers
// for layers >= 1 (by the consumers for layer 0, whose producers carry the window-row gradient); the B tile of step
// ks + 1 is formed while the consumers multiply step ks. Producer thread (row r = tid / 2, half p = tid % 2) loads
// units 8s + 4p .. + 3 of its trajectory — their activations (the forward's [unit][gate] rows: 64 contiguous B) and
// c_{t-1}, dh, din, dc (k8 rows, fcr_wide.h: a step's units of consecutive trajectories contiguous), issued three
// steps ahead in rotating register sets — forms their 16 dgates and dc_{t-1}, splits them into the two 16-B chunks of
// its row half. With two column blocks (NO > 256) both form the same dgates; the first writes dc_{t-1}.
// Row scale: 2^(13 - e), e the exponent of a bound on the row's |dgates|: |dgate| <= |dc_t| <= |dc| + |dh_rec| +
// |din| (forget row: x (kL - 1) / 4, fcr_wide.h kWideDgExp). The three maxima come from the kernels that wrote those
// values (this kernel's epilogue and elementwise part of the previous cell, the head kernel), per row, so no pass
// over the row precedes the K loop.
#pragma once
#include <type_traits>

#include "fcr_common.h"
#include "fcr_f16.h"
#include "fcr_wide.h"

namespace fcr {

constexpr int kWbK = 32;                  // k per step (8 units x 4 gates)
constexpr int kWbProd = 4;                // producer (dgate) waves

// Workgroup geometry: M output columns x N trajectories, 4 producer and CONS consumer waves, U units per producer
// thread and K step (8 / U threads per trajectory row).
template <int M, int N, int CONS, int U>
struct WbGeo {
    static constexpr int kM = M, kN = N, kCons = CONS, kUnits = U;
    static constexpr int kWaves = kWbProd + CONS, kThreads = 64 * kWaves;
    static constexpr int kTM = M / CONS / 16, kTN = N / 16;   // D tiles per consumer wave
    static constexpr int kPPR = 8 / U;                          // producer threads per trajectory row
    static constexpr int kRPT = 8 * N / (64 * kWbProd * U);     // trajectory rows per producer thread
    static constexpr int kStage = M * kWbK * 4;                 // A rows of [hi (64 B) | lo (64 B)]
    static constexpr int kTileB = N * kWbK * 2;                 // one split half of the dgate tile
    static constexpr int kPieces = kStage / 1024 / CONS;        // LDS-DMA pieces per consumer wave per stage
    static constexpr int kOffB = 2 * kStage;                    // [A stage 0 | A stage 1 | B tile 0 hi, lo | B tile 1 ...]
    static constexpr int kOffDown = kOffB + 4 * kTileB;
    static constexpr int kOffW0 = kOffDown + N * 4;             // layer 0: W_ih0 as [unit][gate][kIn]
    static_assert(kStage % (1024 * CONS) == 0, "DMA pieces");
    static_assert(kRPT >= 1 && kRPT * 64 * kWbProd * U == 8 * N, "dgate mapping: a step's 8 units of every row");
    static_assert(U == 2 || U == 4, "units per producer thread");
};
// 256 columns x 128 trajectories, 4 + 4 waves (round 4): every layer; two column blocks at Hp = 256 form the same dgates
using WbG256 = WbGeo<256, 128, 4, 4>;
// 256 columns x 256 trajectories, 4 + 8 waves (layers >= 1 at B >= 32 768, fcr_abi.hip launch_fb): A staged once per 256
// trajectories (half the A bytes per trajectory of WbG256); each producer thread forms the dgates of two rows, each
// consumer 32 columns x 256 trajectories; 168 registers per wave (12 waves), 129 KB of LDS
using WbG256w = WbGeo<256, 256, 8, 4>;
constexpr int kWbW0LdsUnits = 768;                        // layer 0 with H above: W_ih0 read from global memory
constexpr int kWbLds256 = WbG256::kOffW0 + 4 * kWbW0LdsUnits * kIn * 4;
constexpr int kWbLds256w = WbG256w::kOffW0;               // layers >= 1 only (no W_ih0 block)
static_assert(kWbLds256 <= 163840 && kWbLds256w <= 163840, "LDS");
// LDS bytes of one launch: the W_ih0 block only for layer 0 with H <= kWbW0LdsUnits
template <class G>
__host__ __device__ constexpr int wb_lds_bytes(bool l0, int H) {
    return G::kOffW0 + (l0 && H <= kWbW0LdsUnits ? 4 * H * kIn * 4 : 0);
}

struct WbArgs {
    const _Float16 *A;           // [NP][4H / 32][hi (32) | lo (32)]: per output column and K step one 128-B line of
                                 // the f16 split of W^T (unit-major K, wide_split_bt_kernel)
    float *out;                  // k8 rows (fcr_wide.h) of NO columns; NO = 0: no product (layer 0, t = 0)
    int NO, NB, H;
    const float *act;            // [B][H][4] gate activations (i, f, g, o of each unit) of the cell, as its forward
                                 // evaluated and stored them (fcr_wgemm.h)
    // the per-unit rows below are k8 rows of H units ([H/8][NB][8], fcr_wide.h)
    const float *c_prev;         // c_{t-1}, or null (t = 0)
    const float *dh;             // incoming dh of the recurrence (the head's, or the next cell's product), or null: zero
                                 // (layers below the top at t = 9)
    const float *din;            // the layer above's input gradient at t, or null
    const float *dC;             // carried dc in, or null: zero (t = 9)
    float *dC_out;               // dc_{t-1} out (another buffer: the other column block still reads dC)
    const float *rm_c, *rm_h, *rm_d;   // row bounds in: max|dc| [B], max|dh| [nrh][B] (per column block of their
                                       // writer), max|din| [nrd][B]; each null where its rows are (zero or absent)
    int nrh, nrd;
    float *rm_c_out, *rm_h_out, *rm_d_out;   // row bounds out (or null): of dc_{t-1}, of the dh / input-grad columns,
                                             // [column block][B] (every block writes its slot, 0 where it has none)
    int h0, h1, d1;              // output columns [h0, h1) are dh_{t-1}, [0, d1) the layer below's input gradient
    const float *wih0;           // layer 0: W_ih0 packed [unit][gate][kIn] (the window-row gradient), else null
    float *dg;                   // [B][4H] the cell's dgates (fp32, rows gate H + unit), or null: the surrogate's weight
                                 // gradients (fcr_wgrad.h) read them; the rollout needs none
    float *rowg;                 // layer 0: [B][kIn] window-row gradient row (+=), else null
};

// Diagnostic build FCR_WB_STAMP=1 (scripts/stamp_wb.py; the stamps sit in the one-row producer of WbG256, i.e. runs at
// B < 32 768 or scripts/variants/wb_n128.json): per-wave s_memtime sums of the layer >= 1 kernel's K-step sections, added into fcr_wb_stamp by lane 0 (vector atomics) — consumers: barrier wait, A DMA issue, fragment reads +
// MFMA issue; producers: barrier wait, input load issue, dgates (including the wait for their inputs) + tile writes.
// Read the shares, never the build's run time (each stamp drains lgkmcnt).
#ifndef FCR_WB_STAMP
#define FCR_WB_STAMP 0
#endif
#if FCR_WB_STAMP
__device__ unsigned long long fcr_wb_stamp[16];
#define FCR_WB_ST(t)                                                                         \
    do {                                                                                     \
        __builtin_amdgcn_sched_barrier(0);                                                   \
        asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");           \
        __builtin_amdgcn_sched_barrier(0);                                                   \
    } while (0)
#else
#define FCR_WB_ST(t) ((void)0)
#endif

// byte offset of 16-B chunk c (0..3 hi, 4..7 lo) of 128-B LDS row r of an A stage: the XOR by (r >> 1) & 7 puts the 16
// lanes of each ds_read_b128 lane group (rows r, chunk c or c + 1) on 16 distinct 16-B slots of the 256-B bank row
__device__ __forceinline__ uint32_t wb_offa(int r, int c) { return (uint32_t)(r * 128 + ((c ^ ((r >> 1) & 7)) << 4)); }

// byte offset of 16-B chunk c of 64-B LDS row r: the swizzle puts the 8 rows of a fragment read's 8-lane phase
// on distinct 16-B slots of a 128-B bank line (fcr_wgemm.h wg_off)
__device__ __forceinline__ uint32_t wb_off(int r, int c) { return (uint32_t)(r * 64 + ((c ^ ((r >> 1) & 3)) << 4)); }

// one step's inputs of a producer thread: U consecutive units of one trajectory
template <int U>
struct WbIn {
    typedef float fU __attribute__((ext_vector_type(U)));
    f32x4 ac[U];   // i, f, g, o of each unit (the forward's [unit][gate] activation row)
    fU cp, dh, dn, dc;
};

// W0G: layer 0 at H > kWbW0LdsUnits reads W_ih0 from global memory (L1 / L2: every producer thread of a workgroup
// reads the same bytes per step) instead of staging it in LDS
template <class G, bool L0, bool W0G = false>
__global__ __launch_bounds__(G::kThreads, 1) void wide_bwd_fused_kernel(WbArgs a) {
    constexpr int kWbM = G::kM, kWbN = G::kN, kWbCons = G::kCons, kWbUnits = G::kUnits, kWbTM = G::kTM,
                  kWbTN = G::kTN, kWbThreads = G::kThreads, kWbStage = G::kStage,
                  kWbTileB = G::kTileB, kWbPieces = G::kPieces, kWbOffB = G::kOffB, kWbOffDown = G::kOffDown,
                  kWbOffW0 = G::kOffW0, kPPR = G::kPPR;
    using In = WbIn<kWbUnits>;
    // who stages A: the producers for layers >= 1 when they are as many waves as the consumers (the piece split
    // assumes kWbCons issuing waves), else the consumers
    constexpr bool kProdDma = !L0 && kWbProd == G::kCons;
    using fU = typename In::fU;
    extern __shared__ __attribute__((aligned(16))) char lds[];
    const int tid = threadIdx.x, lane = tid & 63;
    const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
    const bool producer = wv < kWbProd;                     // wave-uniform role
    const int cw = wv - kWbProd;                            // consumer: column slice
    const int H = a.H, K = 4 * H, nk = K / kWbK;
    const bool prod = a.NO > 0;
    const int ny = prod ? (a.NO + kWbM - 1) / kWbM : 1, total = gridDim.x, id = blockIdx.x;
    // XCD-aware order: consecutive ids go to different XCDs; each XCD's ids are renumbered contiguously and walk the
    // column blocks fastest, so a trajectory block's column blocks read its rows once into that XCD's L2
    const int xcd = id & 7, loc = id >> 3, q8 = total >> 3, rr = total & 7;
    const int wg = (xcd < rr ? xcd * (q8 + 1) : rr * (q8 + 1) + (xcd - rr) * q8) + loc;
    const int cb = wg % ny;                                 // column block
    const int m0 = cb * kWbM;                               // first output column
    const int b0 = (wg / ny) * kWbN;                        // first trajectory

    // ---- producer thread: its dgate rows (kRPT of them) and unit share; each row's scale from the producers' bounds
    constexpr int kRPT = G::kRPT;
    const int er0 = (tid / kPPR) & (kWbN / kRPT - 1), ep = tid % kPPR;   // (consumers: unused)
    int er[kRPT], eb[kRPT];
    bool elive[kRPT];
    float up[kRPT];
#pragma unroll
    for (int h = 0; h < kRPT; ++h) {
        er[h] = er0 + h * (kWbN / kRPT);
        eb[h] = b0 + er[h] < a.NB ? b0 + er[h] : a.NB - 1;   // tail rows recompute the last trajectory (not stored)
        elive[h] = b0 + er[h] < a.NB;
        up[h] = 0.0f;
    }
    if (producer) {
#pragma unroll
        for (int h = 0; h < kRPT; ++h) {
            float mh = 0.0f, md = 0.0f;
            if (a.rm_h)
                for (int k = 0; k < a.nrh; ++k) mh = fmaxf(mh, a.rm_h[(size_t)k * a.NB + eb[h]]);
            if (a.rm_d)
                for (int k = 0; k < a.nrd; ++k) md = fmaxf(md, a.rm_d[(size_t)k * a.NB + eb[h]]);
            const float m = (a.rm_c ? a.rm_c[eb[h]] : 0.0f) + mh + md;
            const int ex = m > 0.0f ? __builtin_amdgcn_frexp_expf(m) : 0;   // every |dgate| < 2^ex (x (kL-1)/4: forget)
            up[h] = __builtin_amdgcn_ldexpf(1.0f, kWideDgExp - ex);
            if (ep == 0)
                reinterpret_cast<float *>(lds + kWbOffDown)[er[h]] = __builtin_amdgcn_ldexpf(1.0f, ex - kWideDgExp);
        }
    }
    float *w0s = reinterpret_cast<float *>(lds + kWbOffW0);
    if constexpr (L0 && !W0G) {   // W_ih0, packed [unit][gate][kIn] by the host, into LDS as it is (16-B copies)
        const f32x4 *src = reinterpret_cast<const f32x4 *>(a.wih0);
        f32x4 *dst = reinterpret_cast<f32x4 *>(w0s);
        for (int i = tid; i < H * kIn; i += kWbThreads) dst[i] = src[i];   // 4 H kIn floats = H kIn quads
    }
    const float *w0l = W0G ? a.wih0 : w0s;

    // ---- consumers: A by LDS-DMA pieces (16 rows x 64 B of [A hi | A lo]; lane i lands at +16 i).
    // Issued from inline asm: with the intrinsic anywhere in the kernel the compiler's wait insertion drains every
    // outstanding load (vmcnt(0)) before the use of a prefetched value, the producers' included. The step barrier's
    // vmcnt(0) retires each consumer's own pieces. M0 carries the wave's LDS base; nothing else in the kernel uses it.
    const _Float16 *gsrc[kWbPieces];
    uint32_t ldst[kWbPieces];
#pragma unroll
    for (int q = 0; q < kWbPieces; ++q) {
        const int j = (producer ? wv : cw) + kWbCons * q;   // piece: rows 8 j .. 8 j + 7, whole 128-B lines
        const int r = 8 * j + (lane >> 3);
        const int c = (lane & 7) ^ ((r >> 1) & 7);         // the chunk wb_offa puts in lane's slot
        int n = m0 + r;
        if (n >= a.NO) n = a.NO > 0 ? a.NO - 1 : 0;        // tail columns recompute the last one (not stored)
        gsrc[q] = a.A + (size_t)n * 2 * K + 8 * c;
        ldst[q] = (uint32_t)j * 1024;
    }
    auto dma = [&](int ks, int buf) {
#pragma unroll
        for (int q = 0; q < kWbPieces; ++q) {
            const uint32_t la = __builtin_amdgcn_readfirstlane(
                (uint32_t)(uintptr_t)(__attribute__((address_space(3))) char *)(lds + buf * kWbStage + ldst[q]));
            const _Float16 *g = gsrc[q] + ks * 2 * kWbK;
#pragma clang diagnostic push
#pragma clang diagnostic ignored "-Winline-asm"
            asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off" :: "s"(la), "v"(g) : "memory", "m0");
#pragma clang diagnostic pop
        }
    };

    // ---- producers: inputs ahead, the tile one step ahead of the MFMAs ----
    // k8 rows: this thread's U units of step s at + s * 8 NB
    const size_t kso = (size_t)8 * a.NB;
    auto ldu = [](const float *p) { return *reinterpret_cast<const fU *>(p); };
    auto load_in = [&](int h, int s) {
        In x;
        const int u = 8 * s + kWbUnits * ep;
        const size_t so = s * kso + (size_t)eb[h] * 8 + kWbUnits * ep;
        const float *pre = a.act + (size_t)eb[h] * K;
#pragma unroll
        for (int k = 0; k < kWbUnits; ++k) x.ac[k] = *reinterpret_cast<const f32x4 *>(pre + 4 * (u + k));
        x.cp = a.c_prev ? ldu(a.c_prev + so) : fU{};
        x.dh = a.dh ? ldu(a.dh + so) : fU{};
        x.dn = a.din ? ldu(a.din + so) : fU{};
        x.dc = a.dC ? ldu(a.dC + so) : fU{};
        return x;
    };
    float mdc[kRPT];                       // max |dc_{t-1}| of this thread's units, per row
#pragma unroll
    for (int h = 0; h < kRPT; ++h) mdc[h] = 0.0f;
    float pc[kRPT][kIn] = {};              // layer 0: this thread's share of each row's window-row gradient
    // a row's dgates of step s: formed (and dc_{t-1}, the optional fp32 dgate rows, the dc bound), layer 0's
    // window-row gradient accumulated, split into the B tile
    auto form = [&](int h, int s, const In &x, float (&dg)[4 * kWbUnits]) {
        const bool wr_dc = cb == 0 && elive[h];   // every column block forms the same dc_{t-1}: the first stores it
        fU dco;
        const int u = 8 * s + kWbUnits * ep;
#pragma unroll
        for (int k = 0; k < kWbUnits; ++k) {
            const float i = x.ac[k][0], f = x.ac[k][1], g = x.ac[k][2], o = x.ac[k][3];   // the forward's activations
            const float cp = x.cp[k];
            const float tc = tanh_f(fmaf(f, cp, i * g));   // c_t rebuilt as the forward formed it (f c_{t-1} + i g)
            const float dh = x.dh[k] + x.dn[k];
            const float dct = fmaf(dh * o, 1.0f - tc * tc, x.dc[k]);
            dg[4 * k + 0] = dct * g * (i - i * i);
            dg[4 * k + 1] = dct * cp * (f - f * f);
            dg[4 * k + 2] = dct * i * (1.0f - g * g);
            dg[4 * k + 3] = dh * tc * (o - o * o);
            dco[k] = dct * f;
        }
        if (wr_dc) *reinterpret_cast<fU *>(a.dC_out + s * kso + (size_t)eb[h] * 8 + kWbUnits * ep) = dco;
        if (a.dg && wr_dc) {   // (column block 0 writes them: every block forms the same)
            float *d = a.dg + (size_t)eb[h] * K + u;
#pragma unroll
            for (int g = 0; g < 4; ++g) {
                fU v;
#pragma unroll
                for (int k = 0; k < kWbUnits; ++k) v[k] = dg[4 * k + g];
                *reinterpret_cast<fU *>(d + g * H) = v;
            }
        }
#pragma unroll
        for (int k = 0; k < kWbUnits; ++k) mdc[h] = fmaxf(mdc[h], fabsf(dco[k]));
    };
    // layer 0: sum_r dG[b][r] W_ih0[r][c] over this thread's 4 U gate rows, fp32, for its kRPT rows at once: each
    // unit's 20 W_ih0 values are read once for all rows, and unit by unit behind a scheduling fence (unrolled whole,
    // the compiler would hold all 20 U of them in registers)
    auto w0acc = [&](int s, const float (&dg)[kRPT][4 * kWbUnits]) {
        const int u = 8 * s + kWbUnits * ep;
#pragma unroll
        for (int k = 0; k < kWbUnits; ++k) {
            if constexpr (kRPT > 1) __builtin_amdgcn_sched_barrier(0);
            const f32x4 *w4 = reinterpret_cast<const f32x4 *>(w0l + (u + k) * 4 * kIn);   // [gate][column] of unit u + k
#pragma unroll
            for (int q = 0; q < 4 * kIn / 4; ++q) {
                const f32x4 wq = w4[q];
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    const int idx = 4 * q + e;   // (gate g, column c) = (idx / 5, idx % 5)
#pragma unroll
                    for (int h = 0; h < kRPT; ++h)
                        pc[h][idx % kIn] = fmaf(dg[h][4 * k + idx / kIn], wq[e], pc[h][idx % kIn]);
                }
            }
        }
    };
    auto tile = [&](int h, const float (&dg)[4 * kWbUnits], int buf) {
        if (!prod) return;
        // the split (fcr_f16.h mix_pair): hi = f16(up dg), lo = f16(up dg - hi); this thread's U units of the row's 8
        // are 16-B chunks U / 2 * ep .. of the row
        typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
        constexpr int NW = 2 * kWbUnits;   // 32-bit words of halves
        unsigned hw[NW], lw[NW];
#pragma unroll
        for (int p = 0; p < NW; ++p) mix_pair(dg[2 * p], up[h], dg[2 * p + 1], up[h], hw[p], lw[p]);
        char *bt = lds + kWbOffB + buf * 2 * kWbTileB;
#pragma unroll
        for (int c = 0; c < kWbUnits / 2; ++c) {
            const uint32_t o = wb_off(er[h], kWbUnits / 2 * ep + c);
            *reinterpret_cast<u32x4 *>(bt + o) = u32x4{hw[4 * c], hw[4 * c + 1], hw[4 * c + 2], hw[4 * c + 3]};
            *reinterpret_cast<u32x4 *>(bt + kWbTileB + o) = u32x4{lw[4 * c], lw[4 * c + 1], lw[4 * c + 2], lw[4 * c + 3]};
        }
    };
    // one row (the one-row producers)
    auto dgates = [&](int h, int s, const In &x, int buf) {
        float dg[kRPT][4 * kWbUnits];
        form(h, s, x, dg[0]);
        if constexpr (L0 && kRPT == 1) w0acc(s, dg);
        tile(h, dg[0], buf);
    };
    // every row of the thread (the two-row producers; layer 0 reads each W_ih0 value once for both)
    auto dgates_all = [&](int s, In (&x)[kRPT], int buf) {
        float dg[kRPT][4 * kWbUnits];
#pragma unroll
        for (int h = 0; h < kRPT; ++h) form(h, s, x[h], dg[h]);
        if constexpr (L0) w0acc(s, dg);
#pragma unroll
        for (int h = 0; h < kRPT; ++h) tile(h, dg[h], buf);
    };

    // The two roles run separate loops with the same barriers (one per K step, plus the prologue's and the
    // epilogue's): a shared loop would keep the consumers' accumulator registers live in the producers too.
    auto barrier = [] { asm volatile("s_waitcnt vmcnt(0)\n\ts_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); };
    const float *ldown = reinterpret_cast<const float *>(lds + kWbOffDown);
    float *red = reinterpret_cast<float *>(lds);   // epilogue: [cw][kWbN rows][2] (the A stages are retired)
    auto row_sum = [](float v) {   // over the kPPR producer threads of a row (consecutive lanes)
#pragma unroll
        for (int o = 1; o < kPPR; o <<= 1) v += __shfl_xor(v, o);
        return v;
    };
    auto row_max = [](float v) {
#pragma unroll
        for (int o = 1; o < kPPR; o <<= 1) v = fmaxf(v, __shfl_xor(v, o));
        return v;
    };
    if (producer) {
        // a producer's barrier waits only for its LDS tile writes: its input loads stay in flight across it, and the
        // compiler's own wait before their first use (exact counts: no DMA intrinsic in the kernel) is all
        auto pbarrier = [] { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); };
        if constexpr (kRPT == 2) {
            // two rows per thread (WbG256w): one register set per row, refilled for step ks + 2 right after step
            // ks + 1's dgates consumed it (a second set per row would not fit the 12-wave register budget); A is
            // staged by the consumers
            In x[kRPT];
#pragma unroll
            for (int h = 0; h < kRPT; ++h) x[h] = load_in(h, 0);
            barrier();   // W_ih0 and the row scales in LDS
            dgates_all(0, x, 0);
#pragma unroll
            for (int h = 0; h < kRPT; ++h)
                if (nk > 1) x[h] = load_in(h, 1);
            for (int ks = 0; ks < nk; ++ks) {
                pbarrier();   // tile ks published
                if (ks + 1 < nk) {
                    dgates_all(ks + 1, x, (ks & 1) ^ 1);
#pragma unroll
                    for (int h = 0; h < kRPT; ++h)
                        if (ks + 2 < nk) x[h] = load_in(h, ks + 2);
                }
            }
        } else if constexpr (!L0) {
            // Layers >= 1: the producers also stage A (the consumers then only read and multiply): step ks's pieces
            // of stage ks + 1 go out after its barrier (the slot every consumer finished reading at ks - 1), and
            // the step's barrier waits vmcnt(0) for them (and for the step's input loads: measured, the inputs
            // need no more than that one step in flight, round5_c5_bwd_pdma_ab.log)
            auto pbarrier_a = [] { asm volatile("s_waitcnt vmcnt(0)\n\ts_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); };
            if (kProdDma && prod) dma(0, 0);
            // inputs three steps ahead in rotating register sets (unrolled by three: a copy between sets would wait
            // for the loads)
            In x0 = load_in(0, 0), x1, x2;
            if (nk > 1) x1 = load_in(0, 1);
            if (nk > 2) x2 = load_in(0, 2);
            barrier();   // W_ih0 and the row scales in LDS
            dgates(0, 0, x0, 0);
            unsigned long long sw[4] = {0, 0, 0, 0}, tw0 = 0, tw1 = 0, tw2 = 0, tw3 = 0;
            (void)sw, (void)tw0, (void)tw1, (void)tw2, (void)tw3;
            auto pstep = [&](auto full, int ks, const In &xuse, In &xload) {
                constexpr bool FULL = decltype(full)::value;   // ks + 3 < nk: nothing conditional in the step
                FCR_WB_ST(tw0);
                pbarrier_a();                                  // tile ks published, stage ks landed
                FCR_WB_ST(tw1);
                if (FULL || ks + 3 < nk) xload = load_in(0, ks + 3);
                if (kProdDma && prod && ks + 1 < nk) dma(ks + 1, (ks + 1) & 1);
                FCR_WB_ST(tw2);
                if (FULL || ks + 1 < nk) dgates(0, ks + 1, xuse, (ks & 1) ^ 1);   // (its buffer was read at ks - 1)
                FCR_WB_ST(tw3);
                if (FCR_WB_STAMP) {
                    sw[0] += tw1 - tw0;
                    sw[1] += tw2 - tw1;
                    sw[2] += tw3 - tw2;
                    sw[3] += 1;
                }
            };
            using Full = std::integral_constant<bool, true>;
            using Tail = std::integral_constant<bool, false>;
            int ks = 0;
            for (; ks + 5 < nk; ks += 3) {   // step ks + t: dgates from set (t + 1) % 3, loads into set t
                pstep(Full{}, ks, x1, x0);
                pstep(Full{}, ks + 1, x2, x1);
                pstep(Full{}, ks + 2, x0, x2);
            }
            if (ks < nk) pstep(Tail{}, ks, x1, x0);   // the last 1..5 steps, the sets rotating on
            if (ks + 1 < nk) pstep(Tail{}, ks + 1, x2, x1);
            if (ks + 2 < nk) pstep(Tail{}, ks + 2, x0, x2);
            if (ks + 3 < nk) pstep(Tail{}, ks + 3, x1, x0);
            if (ks + 4 < nk) pstep(Tail{}, ks + 4, x2, x1);
#if FCR_WB_STAMP
            if (lane == 0)
                for (int k = 0; k < 4; ++k) atomicAdd(&fcr_wb_stamp[4 + k], sw[k]);
#endif
        } else {
            // layer 0 (the window-row gradient's W_ih0 reads and accumulators) has registers for one set ahead
            In xc = load_in(0, 0);
            barrier();
            dgates(0, 0, xc, 0);
            if (nk > 1) xc = load_in(0, 1);
            for (int ks = 0; ks < nk; ++ks) {
                pbarrier();
                In xn;
                if (ks + 2 < nk) xn = load_in(0, ks + 2);
                if (ks + 1 < nk) dgates(0, ks + 1, xc, (ks & 1) ^ 1);
                if (ks + 2 < nk) xc = xn;
            }
        }
        // per-row results: dc_{t-1} bound, layer 0's window-row gradient
#pragma unroll
        for (int h = 0; h < kRPT; ++h) {
            const float m = row_max(mdc[h]);
            if (a.rm_c_out && cb == 0 && elive[h] && ep == 0) a.rm_c_out[eb[h]] = m;
        }
        if constexpr (L0) {
#pragma unroll
            for (int h = 0; h < kRPT; ++h) {
#pragma unroll
                for (int c = 0; c < kIn; ++c) pc[h][c] = row_sum(pc[h][c]);
                if (a.rowg && elive[h] && cb == 0 && ep == 0)
#pragma unroll
                    for (int c = 0; c < kIn; ++c) a.rowg[(size_t)eb[h] * kIn + c] += pc[h][c];
            }
        }
        if (!prod) return;
        barrier();   // (the consumers' epilogue reuses the A stages)
        barrier();   // the consumers' row maxima are in `red`
    } else {
        f32x4 acc[kWbTM][kWbTN];
#pragma unroll
        for (int i = 0; i < kWbTM; ++i)
#pragma unroll
            for (int j = 0; j < kWbTN; ++j) acc[i][j] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
        const int fr = lane & 15, fq = lane >> 4;
        if (!kProdDma && prod) dma(0, 0);
        barrier();
        unsigned long long sc[4] = {0, 0, 0, 0}, tc0 = 0, tc1 = 0, tc2 = 0;
        (void)sc, (void)tc0, (void)tc1, (void)tc2;
        FCR_WB_ST(tc0);
        for (int ks = 0; ks < nk; ++ks) {
            const int buf = ks & 1;
            barrier();   // stage ks's A landed (its issuing waves waited for their pieces), tile ks written
            FCR_WB_ST(tc1);
            if (!prod) continue;
            if (!kProdDma && ks + 1 < nk) dma(ks + 1, buf ^ 1);   // into the stage every consumer finished reading at ks - 1
            FCR_WB_ST(tc2);
            if (FCR_WB_STAMP) {
                sc[0] += tc1 - tc0;
                sc[1] += tc2 - tc1;
            }
            const char *st = lds + buf * kWbStage;
            const char *bt = lds + kWbOffB + buf * 2 * kWbTileB;
            f16x8 ah[kWbTM], al[kWbTM];
#pragma unroll
            for (int i = 0; i < kWbTM; ++i) {
                const int r = 16 * (kWbTM * cw + i) + fr;
                ah[i] = *reinterpret_cast<const f16x8 *>(st + wb_offa(r, fq));
                al[i] = *reinterpret_cast<const f16x8 *>(st + wb_offa(r, 4 + fq));
            }
#pragma unroll
            for (int j = 0; j < kWbTN; ++j) {   // B tile by tile; the A fragments stay in registers across them
                const int r = 16 * j + fr;
                const f16x8 bh = *reinterpret_cast<const f16x8 *>(bt + wb_off(r, fq));
                const f16x8 bl = *reinterpret_cast<const f16x8 *>(bt + kWbTileB + wb_off(r, fq));
#pragma unroll
                for (int i = 0; i < kWbTM; ++i) acc[i][j] = mma3(ah[i], al[i], bh, bl, acc[i][j]);
            }
            FCR_WB_ST(tc0);
            if (FCR_WB_STAMP) {
                sc[2] += tc0 - tc2;
                sc[3] += 1;
            }
        }
#if FCR_WB_STAMP
        if (!L0 && lane == 0)
            for (int k = 0; k < 4; ++k) atomicAdd(&fcr_wb_stamp[k], sc[k]);
#endif
        if (!prod) return;
        // epilogue: lane = trajectory b0 + 16 j + (lane & 15), columns m0 + 16 (TM cw + i) + 4 (lane >> 4) .. +3, in
        // true units (x the row's down); and the row maxima of the dh and input-gradient columns
        barrier();
#pragma unroll
        for (int j = 0; j < kWbTN; ++j) {
            const int rl = 16 * j + fr, b = b0 + rl;
            const float f = ldown[rl];
            float mh = 0.0f, md = 0.0f;
#pragma unroll
            for (int i = 0; i < kWbTM; ++i) {
                const int col = m0 + 16 * (kWbTM * cw + i) + 4 * fq;
                const f32x4 v = acc[i][j] * f;
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    const float av = fabsf(v[e]);
                    if (col + e >= a.h0 && col + e < a.h1) mh = fmaxf(mh, av);
                    if (col + e < a.d1) md = fmaxf(md, av);
                }
                if (b < a.NB && col < a.NO) *reinterpret_cast<f32x4 *>(a.out + k8(a.NB, b, col)) = v;
            }
            mh = fmaxf(mh, __shfl_xor(mh, 16));
            mh = fmaxf(mh, __shfl_xor(mh, 32));
            md = fmaxf(md, __shfl_xor(md, 16));
            md = fmaxf(md, __shfl_xor(md, 32));
            if (fq == 0) {
                red[(cw * kWbN + rl) * 2] = mh;
                red[(cw * kWbN + rl) * 2 + 1] = md;
            }
        }
        barrier();
        return;
    }
    // the producers (threads 0 .. kWbN - 1 of them) reduce the consumers' row maxima over the column slices
    if (tid < kWbN && b0 + tid < a.NB) {
        float mh = 0.0f, md = 0.0f;
#pragma unroll
        for (int w = 0; w < kWbCons; ++w) {
            mh = fmaxf(mh, red[(w * kWbN + tid) * 2]);
            md = fmaxf(md, red[(w * kWbN + tid) * 2 + 1]);
        }
        const int b = b0 + tid;
        if (a.rm_h_out) a.rm_h_out[(size_t)cb * a.NB + b] = mh;
        if (a.rm_d_out) a.rm_d_out[(size_t)cb * a.NB + b] = md;
    }
}

// A of the gradient product, transposed and split: dst_hi / dst_lo [NO][4Hp], row n = output column n of
// [W_ih | W_hh] (layers >= 1, NO = 2Hp; `wih` null for layer 0: W_hh only, NO = Hp), column r' = 4 unit + gate
// (unit-major: a K step of the fused kernel is 8 whole units) holding torch's gate row gate H + unit; zero for the
// padding units (unit or column >= H) of the padded hidden size Hp.
__global__ void wide_split_bt_kernel(const float *__restrict__ wih, const float *__restrict__ whh, int H, int Hp,
                                     int NO, _Float16 *dst) {
    const size_t idx = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int K = 4 * Hp;
    if (idx >= (size_t)NO * K) return;
    const int n = (int)(idx / K), rp = (int)(idx % K);
    const int unit = rp >> 2, r = (rp & 3) * H + unit;
    const int col = (wih && n >= Hp) ? n - Hp : n;   // column of W_ih (n < Hp) or of W_hh
    float v = 0.0f;
    if (unit < H && col < H) v = (wih && n < Hp) ? wih[(size_t)r * H + col] : whh[(size_t)r * H + col];
    const _Float16 hi = (_Float16)v;
    _Float16 *d = dst + (size_t)n * 2 * K + (rp >> 5) * 64 + (rp & 31);   // K step rp / 32: [hi (32) | lo (32)]
    d[0] = hi;
    d[32] = (_Float16)(v - (float)hi);
}

}  // namespace fcr

namespace fcr {
// W_ih0 [4H][kIn] (torch) -> [unit][gate][kIn] over the padded Hp units (zero past H): the fused layer-0 cell's
// window-row gradient reads it by unit (fcr_wbwd.h)
__global__ void wide_pack_w0_kernel(const float *__restrict__ wih0, int H, int Hp, float *__restrict__ dst) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= 4 * Hp * kIn) return;
    const int u = i / (4 * kIn), g = (i / kIn) % 4, c = i % kIn;
    dst[i] = u < H ? wih0[((size_t)g * H + u) * kIn + c] : 0.0f;
}
}  // namespace fcr
