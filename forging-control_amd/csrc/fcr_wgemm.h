// fcr_wgemm.h — H > 52 (config 5): one LSTM cell of the whole batch as ONE hand-written split-f16 MFMA GEMM
// with the cell update in its epilogue. Every layer, every H: the host pads H to Hp, a multiple of 64, with
// zero-weight units (their gates stay i = f = o = 1/2, g = 0, so c = h = 0 and they add nothing to any product: the
// same padding the H <= 52 tiers use, fcr_abi.hip slot_tier).
//
// Product: G[b][r] = sum_k x[b][k] W[r][k] over the cell's two inputs, fp32-accurate from f16 halves
//   G = W_hi x_hi + W_hi x_lo + W_lo x_hi          (three MFMAs per 32-k block; the dropped lo.lo <= 2^-22)
// Operands (round 5): each input is a RECORD [b][hi (kx) | lo (kx)] — the h record the producing cell wrote ONCE
// (kx = Hp), or layer 0's window record (kx = 32: 5 window columns, zero padded; fcr_wide.h wide_window_kernel) — and
// the weights are split once per call into W_hi and W_lo, [4Hp][K] each, K = [x part | h part]. Against the former
// K-concatenated form ([x_hi|x_lo|x_hi|h_hi|h_lo|h_hi] operand rows that the cells wrote in two copies, against
// [W_hi|W_hi|W_lo|...]) this stages 4 halves per (row, k) instead of 6 and writes each h record once instead of
// twice (3 copies each): a third less LDS-DMA per MFMA and ~270 MB less HBM per cell at config 5.
// A workgroup owns 64 units x kWgN (256) trajectories: its 256 W rows are taken unit-major, gate-minor (LDS row 4 u +
// gate), so an MFMA D fragment (16 rows x 16 trajectories; lane = trajectory lane & 15, rows 4 (lane >> 4) .. +3)
// holds the four gates i, f, g, o of ONE unit of ONE trajectory: the cell update runs on the accumulators, and the
// 4H x B gate matrix never goes to HBM.
//
// Tile walk: kWgN / 32 waves (2 x kWgN / 64), each 128 rows (32 units) x 64 trajectories = 8 x 4 D tiles. A 32-k block
// is TWO ring steps of 32 KB (24 KB at kWgN = 128): step 2kb stages [W_hi | x_hi] and multiplies W_hi x_hi; step
// 2kb + 1 stages [W_lo | x_lo] and multiplies W_hi x_lo + W_lo x_hi (the hi fragments stay in registers across the
// two steps). Stages land by LDS-DMA through a 3-slot ring (two steps of prefetch, one barrier per step; the epilogue's
// tiles reuse it); at kWgN = 128 two workgroups share a CU (one's epilogue and barriers overlap the other's MFMAs), at
// 256 one workgroup per CU stages W once for twice the trajectories (round 5: −4.8 % forward). Round 5 also measured
// one 64 KB ring step per k-block (hi and lo together, 2 slots, one barrier per k-block): +1 % against the split
// steps at 256 (round5_c5_wg256_ab2_keepall.log). LDS rows are 64 B; their
// 16-B chunks are XOR-swizzled by (row >> 1) & 3, so the 8 rows of a ds_read_b128 phase land on distinct 16-B bank
// groups. (History, K-concatenated form: 8 waves x 128 x 32 measured the same; K steps of 64 at one workgroup per CU
// 13 % slower; B fragments straight from global memory 22 % slower; a 3-stage ring with two steps of DMA prefetch
// and a bare s_barrier took the config-5 forward from 191.9 to 188.0 ms; DMA every other step (a bounding build,
// half the staging) 203 -> 184 ms: the staging is what the loop pays for.)
#pragma once
#include "fcr_common.h"
#include "fcr_f16.h"
#include "fcr_wide.h"

namespace fcr {

constexpr int kWgU = 64;                  // units per workgroup (the host pads H to a multiple)
constexpr int kWgM = 4 * kWgU;            // W rows per workgroup
// trajectories per workgroup: 256 = 8 waves at one workgroup per CU (W staged once per 256 trajectories: config 5's
// forward −4.8 % every window kept, −1.9 % step at the default budget against 128 = 4 waves at two workgroups per CU,
// round5_c5_wg256_ab2_*.log; the code is generic over 128 | 256)
constexpr int kWgN = 256;
constexpr int kWgK = 32;                  // k per block (one 16x16x32 f16 MFMA k-block)
constexpr int kWgC = kWgK / 8;            // 16-B chunks per LDS row
constexpr int kWgWaves = kWgN / 32;       // 2 x kWgWC waves; each 128 rows x 64 trajectories
constexpr int kWgWC = kWgWaves / 2;
constexpr int kWgNT = kWgN / kWgWC / 16;  // D tiles per wave along the trajectories
constexpr int kWgThreads = 64 * kWgWaves;
constexpr int kWgStageA = kWgM * kWgK * 2;   // bytes: one split half of the W block
constexpr int kWgStageB = kWgN * kWgK * 2;   // one split half of the operand block
constexpr int kWgEpi = kWgN * (kWgU * 4 + 2 * kWgU * 2);   // the epilogue's c / hi / lo tiles (unpadded, swizzled rows)
constexpr int kWgStages = 3;              // ring slots: two steps of prefetch; the stage wait is vmcnt(one step's pieces)
constexpr int kWgLds = kWgStages * (kWgStageA + kWgStageB) > kWgEpi ? kWgStages * (kWgStageA + kWgStageB) : kWgEpi;
constexpr int kWgRecX0 = kWideRecX0;     // layer 0's window record: [hi (32) | lo (32)] halves, 5 columns used

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

struct WgArgs {
    const _Float16 *W;     // [2][4H][K]: W_hi then W_lo (at + 4 H K), rows torch order (gate H + unit), K = kx + H
    int K;
    const _Float16 *xr;    // x part records [B][2 kx] (hi | lo): the layer below's h records, or layer 0's window rows
    int kx;                // k of the x part (H, or kWgRecX0 for layer 0)
    const _Float16 *hr;    // h part records [B][2H] (hi | lo) of this layer's cell t - 1, or null (t = 0: x part only)
    int B, H;              // H: the padded hidden size (a multiple of kWgU)
    const float *c_prev;   // k8 rows [H/8][B][8] (fcr_wide.h) or null (t = 0)
    float *c_out;          // k8 rows [H/8][B][8]
    float *h_out;          // [B][H] fp32 or null (the readout's cell only)
    float *act;            // [B][H][4] or null: the gate activations i, f, g, o of each unit, as the cell update
                           // evaluated them
                           // (the backward's dgates read them: no sigmoid / tanh of its own but tanh(c_t))
    _Float16 *h_rec;       // [B][2H] this cell's h record (hi | lo): the next cell's and the layer above's operand
};

// byte offset of 16-B chunk c of LDS row r in a stage; the swizzle puts the 8 rows of a fragment read's
// 8-lane phase on the 8 distinct 16-B slots of a 128-B bank line
__device__ __forceinline__ uint32_t wg_off(int r, int c) { return (uint32_t)(r * 64 + ((c ^ ((r >> 1) & 3)) << 4)); }

__global__ __launch_bounds__(kWgThreads, kWgN == 128 ? 2 : 1) void wide_cell_fwd_kernel(WgArgs a) {
    extern __shared__ __attribute__((aligned(16))) char lds[];
    const int tid = threadIdx.x, lane = tid & 63;
    const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wr = wv / kWgWC, wc = wv % kWgWC;         // wave's 128-row half, trajectory slice
    const int H = a.H;
    // XCD-aware walk (consecutive workgroup ids go to different XCDs, each with its own L2): the ids an XCD
    // receives are renumbered contiguously and walk the unit blocks fastest, so a trajectory block's operand
    // records come from HBM once into that XCD's L2 and serve its H / 64 unit blocks (bijective for any count)
    const int ny = H / kWgU, total = gridDim.x, id = blockIdx.x;
    const int xcd = id & 7, loc = id >> 3, q8 = total >> 3, rr = total & 7;
    const int wg = (xcd < rr ? xcd * (q8 + 1) : rr * (q8 + 1) + (xcd - rr) * q8) + loc;
    const int u0 = (wg % ny) * kWgU;                   // first unit of the workgroup
    const int b0 = (wg / ny) * kWgN;                   // first trajectory
    const int nkx = a.kx / kWgK, nkb = nkx + (a.hr ? H / kWgK : 0), ns = 2 * nkb;

    // LDS-DMA staging (global_load_lds, 16 B per lane): one wave instruction fills one 1 KB piece of a stage
    // = 16 rows x 64 B; lane i lands at +16 i, i.e. row i >> 2, slot i & 3, so it fetches the global chunk
    // that the row's swizzle puts in that slot. A stage is 16 W pieces + 8 operand pieces, 6 per wave: pieces
    // q = 0..3 of a wave are W rows, q = 4, 5 operand rows.
    constexpr int NPC = (kWgStageA + kWgStageB) / 1024 / kWgWaves;
    constexpr int NW = kWgStageA / 1024 / kWgWaves;   // the wave's W pieces (then NPC - NW operand pieces)
    static_assert(kWgC == 4 && (NPC == 6 || NPC == 4) && NW * kWgWaves * 1024 == kWgStageA, "DMA pieces");
    const _Float16 *gw[NW];
    const _Float16 *gx[NPC - NW], *gh[NPC - NW];
    const size_t wlo = (size_t)4 * H * a.K;            // W_lo after W_hi
#pragma unroll
    for (int q = 0; q < NPC; ++q) {
        const int j = wv + kWgWaves * q;                  // piece of the stage
        const int r = 16 * (q < NW ? j : j - kWgStageA / 1024) + (lane >> 2);
        const int c = (lane & 3) ^ ((r >> 1) & 3);
        if (q < NW) {
            gw[q] = a.W + (size_t)((r & 3) * H + u0 + (r >> 2)) * a.K + 8 * c;
        } else {
            int b = b0 + r;
            if (b >= a.B) b = a.B - 1;                     // tail rows recompute the last trajectory (not stored)
            gx[q - NW] = a.xr + (size_t)b * 2 * a.kx + 8 * c;
            gh[q - NW] = a.hr ? a.hr + (size_t)b * 2 * H + 8 * c : gx[q - NW];
        }
    }
    // step s: k-block kb = s / 2, split half s % 2 (0: the hi halves, 1: the lo halves)
    auto dma = [&](int s, int buf) {
        const int kb = s >> 1, lo = s & 1;
        const bool xpart = kb < nkx;
        char *dst = lds + buf * (kWgStageA + kWgStageB);
#pragma unroll
        for (int q = 0; q < NPC; ++q) {
            const _Float16 *src;
            if (q < NW) src = gw[q] + kb * kWgK + (lo ? wlo : 0);
            else src = xpart ? gx[q - NW] + kb * kWgK + (lo ? a.kx : 0) : gh[q - NW] + (kb - nkx) * kWgK + (lo ? H : 0);
            __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void *)src,
                                             (__attribute__((address_space(3))) void *)(
                                                 (__attribute__((address_space(3))) char *)dst +
                                                 (uint32_t)(wv + kWgWaves * q) * 1024),
                                             16, 0, 0);
        }
    };

    f32x4 acc[8][kWgNT];
#pragma unroll
    for (int m = 0; m < 8; ++m)
#pragma unroll
        for (int n = 0; n < kWgNT; ++n) acc[m][n] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
    const int fr = lane & 15, fq = lane >> 4;
    // two steps of prefetch: stage s is waited for with step s + 1's pieces still in flight (vmcnt counts this
    // wave's DMA in issue order), and the barrier is a bare s_barrier: __syncthreads()'s release fence would drain
    // every outstanding load (vmcnt(0)). The barrier's lgkmcnt(0) retires this wave's fragment reads of step s - 1,
    // whose slot step s's DMA then refills.
    dma(0, 0);
    dma(1, 1);   // ns >= 2: every cell has at least one k-block
    f16x8 ah[8], bh[kWgNT];   // the hi fragments of the current k-block, kept from its first step to its second
    int buf = 0;
    auto wait_stage = [&](int s) {
        if (s + 1 < ns) {   // the next step's NPC pieces may stay in flight
            if constexpr (NPC == 6) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
            else asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
        }
        else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    };
    for (int s = 0; s < ns; s += 2) {
        // hi step: W_hi x_hi
        wait_stage(s);
        {
            const char *base = lds + buf * (kWgStageA + kWgStageB);
#pragma unroll
            for (int n = 0; n < kWgNT; ++n)
                bh[n] = *reinterpret_cast<const f16x8 *>(base + kWgStageA + wg_off(16 * (kWgNT * wc + n) + fr, fq));
#pragma unroll
            for (int m = 0; m < 8; ++m) ah[m] = *reinterpret_cast<const f16x8 *>(base + wg_off(128 * wr + 16 * m + fr, fq));
            if (s + 2 < ns) dma(s + 2, buf == 0 ? 2 : buf - 1);   // (s + 2) % 3: the slot every wave read at s - 1
#pragma unroll
            for (int m = 0; m < 8; ++m)
#pragma unroll
                for (int n = 0; n < kWgNT; ++n) acc[m][n] = mfma16(ah[m], bh[n], acc[m][n]);
            buf = buf == 2 ? 0 : buf + 1;
        }
        // lo step: W_hi x_lo + W_lo x_hi
        wait_stage(s + 1);
        {
            const char *base = lds + buf * (kWgStageA + kWgStageB);
            f16x8 bl[kWgNT];
#pragma unroll
            for (int n = 0; n < kWgNT; ++n)
                bl[n] = *reinterpret_cast<const f16x8 *>(base + kWgStageA + wg_off(16 * (kWgNT * wc + n) + fr, fq));
            if (s + 3 < ns) dma(s + 3, buf == 0 ? 2 : buf - 1);
#pragma unroll
            for (int m = 0; m < 8; ++m) {
                const f16x8 al = *reinterpret_cast<const f16x8 *>(base + wg_off(128 * wr + 16 * m + fr, fq));
#pragma unroll
                for (int n = 0; n < kWgNT; ++n) {
                    acc[m][n] = mfma16(al, bh[n], acc[m][n]);
                    acc[m][n] = mfma16(ah[m], bl[n], acc[m][n]);
                }
            }
            buf = buf == 2 ? 0 : buf + 1;
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    // ---- epilogue: the cell update on the accumulators, through LDS ----
    // A lane holds (trajectory, unit) pairs scattered over 16 rows; the records want whole rows. So the c_prev tile
    // comes in by rows, each lane updates its pairs in LDS tiles [trajectory][unit], and c and the h record go out by
    // rows again; the activations go straight from the registers ([unit][gate] rows, WgArgs.act).
    // Rows are unpadded (c: 256 B, hi / lo: 128 B) and swizzled (epi_cx / epi_sw): the 16-B chunks of row r XOR r & 7,
    // the elements inside a chunk XOR 2 where bit 3 of r is set. A per-element access (32 lanes = 16 rows x 2 units
    // on 32 banks) and every row-wise 16-B pass then hit distinct banks (scripts/wg_epi_banks.py: 320 -> 0 conflict
    // cycles per wave; the round-5 rows padded by 16 B measured 16 % of the kernel's LDS cycles as conflicts).
    constexpr int CSTR = kWgU;                // floats per c row
    constexpr int HSTR = kWgU;                // halves per hi / lo row
    float *cs = reinterpret_cast<float *>(lds);                                   // [kWgN][CSTR]
    _Float16 *hs = reinterpret_cast<_Float16 *>(lds + kWgN * CSTR * 4);           // [kWgN][HSTR]
    _Float16 *ls = hs + kWgN * HSTR;                                              // [kWgN][HSTR]
    auto epi_cx = [](int r) { return r & 7; };              // chunk swizzle of row r
    auto epi_sw = [](int r) { return ((r >> 3) & 1) << 1; }; // element swizzle inside a chunk of row r
    auto c_el = [&](int r, int ul) { return r * CSTR + 4 * ((ul >> 2) ^ epi_cx(r)) + ((ul & 3) ^ epi_sw(r)); };
    auto h_el = [&](int r, int ul) {
        return r * HSTR + 8 * ((ul >> 3) ^ epi_cx(r)) + 2 * (((ul >> 1) & 3) ^ epi_sw(r)) + (ul & 1);
    };
    constexpr int ERS = kWgThreads / 16;      // row-wise passes: ERS rows x 16 chunks per pass
    static_assert(ERS % 16 == 0, "a thread's rows share r & 15 (its swizzle)");
    const int er = tid >> 4, ec = tid & 15;
    const int ecx = ec ^ epi_cx(er), erx = (ec & 7) ^ epi_cx(er);   // the thread's physical c / h chunk
    const bool eswap = epi_sw(er) != 0;                           // its chunks' elements are stored z w x y
    if (a.c_prev) {
#pragma unroll
        for (int p = 0; p < kWgN / ERS; ++p) {
            const int r = er + ERS * p, b = b0 + r;
            if (b < a.B) {
                const f32x4 v = *reinterpret_cast<const f32x4 *>(a.c_prev + k8(a.B, b, u0 + 4 * ec));
                *reinterpret_cast<f32x4 *>(cs + r * CSTR + 4 * ecx) = eswap ? f32x4{v[2], v[3], v[0], v[1]} : v;
            }
        }
    }
    __syncthreads();
#pragma unroll
    for (int n = 0; n < kWgNT; ++n) {
        const int r = 16 * (kWgNT * wc + n) + fr;
#pragma unroll
        for (int m = 0; m < 8; ++m) {
            const int ul = 32 * wr + 4 * m + fq;
            const f32x4 g4 = acc[m][n];
            const float cp = a.c_prev ? cs[c_el(r, ul)] : 0.0f;
            const float i = sigm(g4[0]), f = sigm(g4[1]), g = tanhf(g4[2]), o = sigm(g4[3]);
            const int b = b0 + r;
            // the activations, [unit][gate] rows: a lane's four gates are one 16-B store, a fragment's 4 units x 16
            // trajectories 16 row pieces of 64 B (the next m fills the other half of each 128-B line)
            if (a.act && b < a.B) *reinterpret_cast<f32x4 *>(a.act + ((size_t)b * H + u0 + ul) * 4) = f32x4{i, f, g, o};
            const float c = (a.c_prev ? f * cp : 0.0f) + i * g;
            const float h = o * tanhf(c);
            const _Float16 hi = (_Float16)h;
            cs[c_el(r, ul)] = c;
            hs[h_el(r, ul)] = hi;
            ls[h_el(r, ul)] = (_Float16)(h - (float)hi);
            if (a.h_out && b < a.B) a.h_out[(size_t)b * H + u0 + ul] = h;   // the readout's cell only
        }
    }
    __syncthreads();
#pragma unroll
    for (int p = 0; p < kWgN / ERS; ++p) {
        const int r = er + ERS * p, b = b0 + r;
        if (b >= a.B) continue;
        const f32x4 cv = *reinterpret_cast<const f32x4 *>(cs + r * CSTR + 4 * ecx);
        *reinterpret_cast<f32x4 *>(a.c_out + k8(a.B, b, u0 + 4 * ec)) = eswap ? f32x4{cv[2], cv[3], cv[0], cv[1]} : cv;
        // 8 chunks of 8 halves per row and half: the hi halves of the 64 units (ec < 8), then the lo halves
        const int e = ec & 7;
        const u32x4 hv = *reinterpret_cast<const u32x4 *>((ec < 8 ? hs : ls) + r * HSTR + 8 * erx);
        *reinterpret_cast<u32x4 *>(a.h_rec + (size_t)b * 2 * H + (ec < 8 ? 0 : H) + u0 + 8 * e) =
            eswap ? u32x4{hv[2], hv[3], hv[0], hv[1]} : hv;
    }
}

// The split weights of one layer's forward cells: dst_hi / dst_lo [4Hp][K] (K = kx + Hp; kx = Hp for layers >= 1,
// kWgRecX0 for layer 0), row gate Hp + unit, columns [x part | h part]; zero outside the real H x in_dim block.
// Layer 0's window columns carry the range guard's power of two (fcr_pack.h): W_ih0 2^s_c against x 2^-s_c.
__global__ void wide_split_fw_kernel(const float *__restrict__ Wih, const float *__restrict__ Whh, int H, int Hp,
                                     int layer0, const float *__restrict__ wsc, _Float16 *dst_hi, _Float16 *dst_lo) {
    const int kx = layer0 ? kWgRecX0 : Hp, K = kx + Hp, nin = layer0 ? kIn : H;
    const size_t idx = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= (size_t)4 * Hp * K) return;
    const int r = (int)(idx / K), k = (int)(idx % K), gate = r / Hp, unit = r % Hp;
    float v = 0.0f;
    if (unit < H) {
        const int tr = gate * H + unit;   // torch's row
        if (k < kx) {
            if (k < nin) v = Wih[(size_t)tr * nin + k] / (layer0 ? wsc[k] : 1.0f);   // (exact: a power of two)
        } else if (k - kx < H) {
            v = Whh[(size_t)tr * H + (k - kx)];
        }
    }
    const _Float16 hi = (_Float16)v;
    dst_hi[idx] = hi;
    dst_lo[idx] = (_Float16)(v - (float)hi);
}

}  // namespace fcr
