// fcr_bwd.h — backward of the rollout (what loss.backward(), Functions.py:655, computes for the
// controller): reverse over windows; per window three layer phases (2 -> 1 -> 0), each reverse over
// t = 9..0, with that layer's weight image resident in LDS (fcr_img.h).
//
// Recompute, not store: each cell rebuilds its gate pre-activations from (x_t, h_{t-1}, c_{t-1}) —
// the forward kept h and c (8 B per unit slot) — with the very products and pointwise arithmetic of
// the forward kernel (rec_operand on the stored split records, mma3 in the same k order, lstm_point_grad), and feeds the local
// derivatives straight into the gradient product [dx ; dh_prev] = Wᵀ·dgates. Both products read the
// same LDS image: row reads for W·[x;h], ds_read_b64_tr_b16 for Wᵀ·dgates. Against storing the
// derivatives (24 B per slot written by the forward, read here), this halves the HBM traffic of
// the two kernels for 2x the matrix work of this one — the split-f16 matrix cores have it to spare.
#pragma once
#include "fcr_common.h"
#include "fcr_f16.h"
#include "fcr_img.h"

namespace fcr {

// Inputs of one backward cell, fetched one cell ahead: each register group is refilled for the next
// cell right after this cell consumed it (x, h_{t-1}, din at the top, c_{t-1} quad by quad).
template <int HS>
struct CellIn {
    f32x4 x[Geo<HS>::HQ];   // layer >= 1: split record of the layer-below h_t; layer 0: x[0] = (column q, column 4, -, -)
    f32x4 h[Geo<HS>::HQ];   // split record of h_{t-1} (fcr_f16.h)
    f32x4 c[Geo<HS>::HQ];   // c_{t-1}
    f32x4 d[Geo<HS>::HQ];   // din = dx of the layer above at t (layers 0, 1)
    f32x4 o[Geo<HS>::HQ];   // split record of the cell's own h_t (its tanh(c_t) = h_t / o_t: lstm_point_grad_h)
};

// Where the next cell's inputs live: buffer descriptors over this wave's own slab regions (SGPRs)
// and byte offsets (SGPRs), so every load's address is one shared lane-offset VGPR.
// What the next cell reads is known at compile time from where the current one sits in its phase
// (NX_L0: x from the window rows; NX_HC: t > 0, so h_{t-1}, c_{t-1} exist; NX_DIN: a din from above):
// only those are fetched. A fetched-but-unused register would be reused at once, i.e. waited for.
struct NextIn {
    __amdgpu_buffer_rsrc_t rh, rc, rx, rd;   // hseq, cseq, xw, dseq
    uint32_t x, h, c, d, o;
};

// Where a cell's scaled dgates go when the caller wants them (the surrogate's weight gradients, fcr_sur.h):
// every dgate block as it is formed — [block kbb][hi | lo][64 lanes][8 halves] from byte `off` — and the
// trajectory's unscaling factor (`down`, a power of two) at `soff` (lane group 0). Unused (DG = false) by the rollout.
struct DgOut {
    __amdgpu_buffer_rsrc_t r, rs;
    uint32_t off, soff;
};

template <int HS, int k = 0>
__device__ __forceinline__ void ld_quads(f32x4 (&dst)[Geo<HS>::HQ], __amdgpu_buffer_rsrc_t r, uint32_t off, int lane) {
    if constexpr (k < Geo<HS>::HQ) {
        dst[k] = buf_ldq<quad_n<HS, k>()>(r, quad_voff<HS, k>(lane), off + quad_soff<HS, k>());
        ld_quads<HS, k + 1>(dst, r, off, lane);
    }
}

// the first RW words of a record (buf_store_rec's layout) into the first quads of dst
template <int HS, int RW, int k = 0>
__device__ __forceinline__ void ld_rec(f32x4 (&dst)[Geo<HS>::HQ], __amdgpu_buffer_rsrc_t r, uint32_t off, int lane) {
    if constexpr (k < Geo<RW>::HQ) {
        dst[k] = buf_ldq<quad_n<RW, k>()>(r, quad_voff<RW, k>(lane), off + quad_soff<RW, k>());
        ld_rec<HS, RW, k + 1>(dst, r, off, lane);
    }
}

// quad k alone (a small-batch wave's own slots, fcr_small.h)
template <int HS, int k>
__device__ __forceinline__ void ld_quad(f32x4 (&dst)[Geo<HS>::HQ], __amdgpu_buffer_rsrc_t r, uint32_t off, int lane) {
    dst[k] = buf_ldq<quad_n<HS, k>()>(r, quad_voff<HS, k>(lane), off + quad_soff<HS, k>());
}

template <int HS, bool NX_L0, bool NX_HC, bool NX_DIN, bool LP = false>
__device__ __forceinline__ void load_xhd(CellIn<HS> &ci, const NextIn &n, int lane) {
    constexpr int RW = rec_words<HS, LP>();   // h records: hi halves only in the f16 mode
    if (NX_L0) {
        const f32x2 v = buf_ld2(n.rx, lane * 8, n.x);
        ci.x[0][0] = v[0];
        ci.x[0][1] = v[1];
    } else {
        ld_rec<HS, RW>(ci.x, n.rh, n.x, lane);
    }
    if (NX_HC) ld_rec<HS, RW>(ci.h, n.rh, n.h, lane);
    if (NX_DIN) ld_rec<HS, din_words<HS, LP>()>(ci.d, n.rd, n.d, lane);
}

// The f16 mode's d record (din_words): v 2^(14-e) as f16 halves, e = the exponent of the trajectory's largest |v| (over
// its four lanes: every scaled value is below 2^14), and e itself (an integer, exact in f16) in half HS. Relative to
// the trajectory's largest din the halves keep 2^-12 — the precision of the f16 dgates the products consume.
template <int HS>
__device__ __forceinline__ void din_store_lp(__amdgpu_buffer_rsrc_t r, uint32_t off, const float (&v)[HS], int lane) {
    typedef _Float16 f16x2 __attribute__((ext_vector_type(2)));
    constexpr int DW = din_words<HS, true>();
    float m = 0.0f;
#pragma unroll
    for (int s = 0; s < HS; ++s) m = fmaxf(m, fabsf(v[s]));
    m = max_q(m);
    const int e = max(__builtin_amdgcn_frexp_expf(m), -100);   // m < 2^e; all-zero -> e = 0
    const float sc = __builtin_amdgcn_ldexpf(1.0f, 14 - e);
    float w[HS];
#pragma unroll
    for (int d = 0; d < DW; ++d) {
        f16x2 p;
#pragma unroll
        for (int u = 0; u < 2; ++u) {
            const int i = 2 * d + u;
            p[u] = i < HS ? (_Float16)__builtin_fmaf(v[i < HS ? i : 0], sc, 0.0f) : i == HS ? (_Float16)(float)e : (_Float16)0.0f;
        }
        w[d] = __builtin_bit_cast(float, p);
    }
    buf_store_rec<DW>(r, off, w, lane);
}
template <int HS, bool LP>
__device__ __forceinline__ void din_store(__amdgpu_buffer_rsrc_t r, uint32_t off, const float (&v)[HS], int lane) {
    if constexpr (LP) din_store_lp<HS>(r, off, v, lane);
    else buf_store_quads<HS>(r, off, v, lane);
}
// c_{t-1} of slot r from the f16 mode's c record (c_store)
__device__ __forceinline__ float crec_lp(const f32x4 *c, int r) {
    typedef _Float16 f16x2 __attribute__((ext_vector_type(2)));
    const int w = r >> 1;
    const float wv = c[w >> 2][w & 3];   // (a plain element read: bit_cast of a vector element misreads, fcr_common.h)
    return (float)__builtin_bit_cast(f16x2, wv)[r & 1];
}
// din of slot r from the f16 mode's d record, given 2^(e-14) (dsc)
template <int HS>
__device__ __forceinline__ float din_lp(const f32x4 *d, int r, float dsc) {
    typedef _Float16 f16x2 __attribute__((ext_vector_type(2)));
    const int w = r >> 1;
    const float wv = d[w >> 2][w & 3];   // (a plain element read: bit_cast of a vector element misreads, fcr_common.h)
    return (float)__builtin_bit_cast(f16x2, wv)[r & 1] * dsc;
}
template <int HS>
__device__ __forceinline__ float din_scale_lp(const f32x4 *d) {
    typedef _Float16 f16x2 __attribute__((ext_vector_type(2)));
    constexpr int w = HS >> 1;
    const float wv = d[w >> 2][w & 3];
    return __builtin_amdgcn_ldexpf(1.0f, (int)(float)__builtin_bit_cast(f16x2, wv)[HS & 1] - 14);
}

// inverse exp2 pre-scales of the packed gate rows (fcr_img.h), folded into the dgate scaling
constexpr float kInvNegLog2e = 1.0f / kNegLog2e;

// One backward cell for 16 trajectories. L0: outputs dh_prev and the window-row gradients dxq (column
// q), dx4 (column 4, lane group 0); else dxo (layer-below h slots) and dh_prev. DIN: the incoming dh
// from above is ci.d (else ext). FIRST: t = 0 (h_{t-1} = c_{t-1} = 0). fb/tb: the lane's image
// addresses (fcr_img.h). On exit `ci` holds the next cell's inputs (or their loads are in flight).
//
// Per trajectory the dgates are scaled by 2^(13-e) (e = exponent of the largest |dh|+|dc| over its
// slots, which bounds every dgate) before the f16 split, and the products scaled back: both exact.
// Schedule: region kb issues the transposed products of dgate block kb (slots 2kb, 2kb+1) beside the
// recomputed forward tiles 2kb+2, 2kb+3 and their gradients, which form block kb+1.
// OWN: the cell's own h_t record is in ci.o (every cell but the first of a window's layer-2 phase, whose h_9
// only fed the readout): tanh(c_t) comes from it (lstm_point_grad_h) instead of being re-evaluated.
// NX_OWN: the next cell's is fetched. (The f16 mode's record holds f16(h) only: tanh(c_t) = h f16-rounded / o, the
// same accuracy against the fp64 oracle as re-evaluating tanh from the c record, scripts/f16_errs.py, and 5 % faster.)
#ifndef FCR_STAMP
#define FCR_STAMP 0   // diagnostic: per-wave s_memtime sums of the cell's sections (ws tail)
#endif
struct Stamps {
    unsigned long long t[8];   // prologue, regions, epilogue, cells, -, window head, fill 2, fill 1
};
__device__ __forceinline__ unsigned long long stamp_now() {
#if FCR_STAMP
    return __builtin_amdgcn_s_memtime();
#else
    return 0;
#endif
}

template <int HS, bool L0, bool DIN, bool FIRST, bool NX_L0, bool NX_HC, bool NX_DIN, bool LP, bool OWN = true,
          bool NX_OWN = true, bool DG = false>
__device__ __forceinline__ void bwd_cell(uint32_t fb, uint32_t tb, int lane, const float (&ext)[HS],
                                         float (&dh)[HS], float (&dc)[HS], float (&dxo)[HS], float &dxq,
                                         float &dx4, CellIn<HS> &ci, const NextIn &nx, Stamps &sp,
                                         const DgOut *dgo = nullptr) {
    const unsigned long long t0 = stamp_now();
    constexpr bool OWNH = OWN, NX_OWNH = NX_OWN;
    // the two waves of a SIMD take turns at the higher issue priority, cell by cell, so neither runs
    // ahead of the other between the phase barriers (oldest-first arbitration otherwise skews them)
    if (sp.t[4] & 1) __builtin_amdgcn_s_setprio(1);
    else __builtin_amdgcn_s_setprio(0);
    sp.t[4] ^= 1;
    using I = Img<HS, L0>;
    using G = Geo16<HS>;
    constexpr int KB = I::KB, NB = I::NB, KBB = I::KBB;
    constexpr uint32_t TILE = I::TILE;                  // one slot's 16 image rows
    constexpr uint32_t LO = I::HALF;                    // lo image
    constexpr int KLO = (L0 && FIRST) ? G::XBLK : 0;
    constexpr int KHI = FIRST ? (L0 ? G::XBLK + 1 : G::KX1) : KB;

    float up, down, sg0, sgg;   // the trajectory's power-of-two scale, set once the incoming dh is in
    float dgd = 0.0f;           // DG: down, or 0 when the trajectory has no gradient here (its dgates are zero)

    // packed tail block (fcr_f16.h, fcr_img.h): its hi-image row read is the packed fragment, and the
    // transposed product's last output tile reads W_lo of its two real rows from the hi image's padding rows
    constexpr bool TAIL = !L0 && G::TAIL1;
    constexpr bool TAILT = TAIL && !LP && (2 * HS) % 4 == 2;
    // ---- the recomputation's B operands (this cell's x_t and h_{t-1}) ----
    f16x8 bh[KB], bl[KB] = {};
    {
        float xv[HS], hv[HS];
#pragma unroll
        for (int s = 0; s < HS; ++s) {
            xv[s] = L0 ? 0.0f : ci.x[s >> 2][s & 3];
            hv[s] = FIRST ? 0.0f : ci.h[s >> 2][s & 3];
        }
        const float x0 = ci.x[0][0], x1 = ci.x[0][1];
#pragma unroll
        for (int kb = KLO; kb < KHI; ++kb) rec_operand<HS, L0, FIRST, LP>(kb, x0, x1, xv, hv, bh[kb], bl[kb]);
        if (TAIL && KHI == KB) bh[KB - 1] = tail_operand<LP>(bh[KB - 1], bl[KB - 1]);
    }

    // Recomputed forward tile r: its MFMA chain (one accumulator: a dependent 16x16x32 MFMA chain issues back to
    // back, MI355X_MICROARCH.md), issued two regions before its result is used.
    auto fwd_tile = [&](int r, f32x4 &a) {
        // the lo image through its own (opaque) base: its reads then also fit the 16-bit ds offset
        uint32_t fbl = fb + LO;
        asm volatile("" : "+v"(fbl));
        a = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
        for (int kb = KLO; kb < KHI; ++kb) {
            const uint32_t a0 = fb + 8u * (2 * kb) + r * TILE, a1 = fb + 8u * (2 * kb + 1) + r * TILE;
            const uint32_t b0 = fbl + 8u * (2 * kb) + r * TILE, b1 = fbl + 8u * (2 * kb + 1) + r * TILE;
            f16x8 ah, al = {};
            const f16x4 h0 = lds_b64_f16(a0), h1 = lds_b64_f16(a1);
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                ah[k] = h0[k];
                ah[4 + k] = h1[k];
            }
            const bool tail = TAIL && kb == KB - 1;
            if (!LP && !tail) {
                const f16x4 l0 = lds_b64_f16(b0), l1 = lds_b64_f16(b1);
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    al[k] = l0[k];
                    al[4 + k] = l1[k];
                }
            }
            a = tail ? mfma16(ah, bh[kb], a) : mma_p<LP>(ah, al, bh[kb], bl[kb], a);
        }
    };
    // pointwise + cell gradient of slot r from its pre-activations -> the 4 dgates as (scaled factor,
    // local derivative) pairs, multiplied inside the split (split8p): (dc s, dc/di), (dc s, dc/df),
    // (dc s_g, dc/dg), (dh s, dh/do) — s = the trajectory scale over the exp2 pre-scale of i, f, o rows,
    // s_g = -s/2 for the g rows (their pre-scale is -2x that of i, f, o: exact)
    auto slot_grad = [&](int r, f32x4 a, float *va, float *vb) {
        f32x4 P;
        f32x2 Q;
        const float cpv = FIRST ? 0.0f : (LP ? crec_lp(ci.c, r) : ci.c[r >> 2][r & 3]);
        if (OWNH) lstm_point_grad_h<FIRST>(a, cpv, rec_h<HS, LP>(ci.o, r), P, Q);
        else lstm_point_grad<FIRST>(a, cpv, P, Q);
        // torch LSTM semantics: dc = dc_carried + dh dh/dc; the carried dc of the cell below is dc f
        const float dcv = fmaf(dh[r], P[0], dc[r]);
        dc[r] = dcv * Q[1];
        const float dcs = dcv * sg0;
        va[0] = va[1] = dcs;
        va[2] = dcv * sgg;
        va[3] = dh[r] * sg0;
        vb[0] = P[2];
        vb[1] = P[3];
        vb[2] = Q[0];
        vb[3] = P[1];
        // c_{t-1} quad of slots 4k..4k+3 consumed (f16 mode: 8k..8k+7): the next cell's comes in
        if constexpr (LP) {
            constexpr int CW = rec_words<HS, true>(), CQ = Geo<CW>::HQ;
            static_assert(CQ <= 2, "f16 c record quads");
            if (NX_HC && CQ == 2 && r == 7)
                ci.c[0] = buf_ldq<quad_n<CW, 0>()>(nx.rc, quad_voff<CW, 0>(lane), nx.c + quad_soff<CW, 0>());
            if (NX_HC && r == HS - 1)
                ci.c[CQ - 1] = buf_ldq<quad_n<CW, CQ - 1>()>(nx.rc, quad_voff<CW, CQ - 1>(lane), nx.c + quad_soff<CW, CQ - 1>());
        } else {
            if (NX_HC && (r & 3) == 3)
                ci.c[r >> 2] = buf_ld4(nx.rc, lane * 16, nx.c + (r >> 2) * kWave * 16);
            if (NX_HC && r == HS - 1 && (r & 3) != 3)
                ci.c[r >> 2] = buf_ldq<quad_n<HS, (HS - 1) / 4>()>(nx.rc, quad_voff<HS, (HS - 1) / 4>(lane),
                                                                  nx.c + quad_soff<HS, (HS - 1) / 4>());
        }
    };
    // forward MFMAs of slot pair kbb into fa[.][0..1]
    auto fwd_pair = [&](int kbb, f32x4 (&fp)[2]) {
#pragma unroll
        for (int u = 0; u < 2; ++u)
            if (2 * kbb + u < HS) fwd_tile(2 * kbb + u, fp[u]);
    };
    // dgate block kbb (B operand of the transposed product) from the pair's pre-activations
    auto dgate_block = [&](int kbb, const f32x4 (&fp)[2], f16x8 &gh, f16x8 &gl) {
        float va[8], vb[8];
#pragma unroll
        for (int u = 0; u < 2; ++u) {
            const int r = 2 * kbb + u;
            if (r < HS) {
                slot_grad(r, fp[u], va + 4 * u, vb + 4 * u);
            } else {
#pragma unroll
                for (int k = 0; k < 4; ++k) va[4 * u + k] = vb[4 * u + k] = 0.0f;
            }
        }
        split_pp<LP>(va, vb, gh, gl);
    };

    // Pipeline: region kbb issues the forward MFMAs of pair kbb+2, the transposed products of dgate
    // block kbb, and the pointwise/gradient VALU of pair kbb+1 (whose MFMAs were issued a region ago).
    f32x4 acc[NB];
#pragma unroll
    for (int k = 0; k < NB; ++k) acc[k] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
    f32x4 fa[3][2];
    f16x8 gh[2], gl[2] = {};
    fwd_pair(0, fa[0]);
    if (KBB > 1) fwd_pair(1, fa[1]);
    // ---- incoming dh, and the trajectory's power-of-two scale: issued behind the first forward MFMAs,
    // which only need this cell's (prefetched) inputs, so the previous cell's tail overlaps them ----
    {
        float m = 0.0f;
        const float dsc = (DIN && LP) ? din_scale_lp<HS>(ci.d) : 0.0f;
#pragma unroll
        for (int r = 0; r < HS; ++r) {
            const float din = DIN ? (LP ? din_lp<HS>(ci.d, r, dsc) : ci.d[r >> 2][r & 3]) : ext[r];
            dh[r] = dh[r] + din;
            m = fmaxf(m, fabsf(dh[r]) + fabsf(dc[r]));
        }
        m = max_q(m);
        const int e = max(__builtin_amdgcn_frexp_expf(m), -100);   // m < 2^e; all-zero -> e = 0
        up = __builtin_amdgcn_ldexpf(1.0f, 13 - e);
        down = __builtin_amdgcn_ldexpf(1.0f, e - 13);
        sg0 = up * kInvNegLog2e;   // dgate scale of the i, f, o rows
        sgg = sg0 * -0.5f;         // and of the g rows
        if (DG) dgd = m > 0.0f ? down : 0.0f;
    }
    // OWN_REG: the next cell (t - 1, same phase) owns h_{t-1}, whose record this cell has in ci.h: kept in registers
    // for it instead of re-read from the slab (an L2 miss by then)
    constexpr bool OWN_REG = NX_OWNH && !FIRST;
    f32x4 hkeep[Geo<HS>::HQ];
    if constexpr (OWN_REG) {
#pragma unroll
        for (int k = 0; k < Geo<HS>::HQ; ++k) hkeep[k] = ci.h[k];
    }
    load_xhd<HS, NX_L0, NX_HC, NX_DIN, LP>(ci, nx, lane);   // x, h, din of this cell are consumed
    // DG: the block leaves as it is formed (two 16-B stores per lane), and the trajectory's `down`
    auto dg_store = [&](int kbb, f16x8 h, f16x8 l) {
        if constexpr (DG) {
            buf_st4(dgo->r, lane * 16, dgo->off + kbb * 2048, __builtin_bit_cast(f32x4, h));
            buf_st4(dgo->r, lane * 16, dgo->off + kbb * 2048 + 1024, __builtin_bit_cast(f32x4, l));
        }
    };
    if constexpr (DG) {
        if (lane < 16) buf_st1(dgo->rs, lane * 4, dgo->soff, dgd);
    }
    dgate_block(0, fa[0], gh[0], gl[0]);
    dg_store(0, gh[0], gl[0]);
    const unsigned long long t1 = stamp_now();
#pragma unroll
    for (int kbb = 0; kbb < KBB; ++kbb) {
        sched_fence();
        asm volatile("" : "+v"(fb), "+v"(tb));
        uint32_t tbl = tb + LO;   // lo image base (opaque: keeps the reads' offsets inside 16 bits)
        asm volatile("" : "+v"(tbl));
        const int cu = kbb & 1, nu = cu ^ 1;
        const bool two = 2 * kbb + 1 < HS;
        if (kbb + 2 < KBB) fwd_pair(kbb + 2, fa[(kbb + 2) % 3]);
#pragma unroll
        for (int tau = 0; tau < NB; ++tau) {
            const uint32_t ct = 8u * (2 * (tau >> 1) + (tau & 1)) + 2 * kbb * TILE;
            // the last tile of a packed-tail layer: its hi-image rows hold W_hi AND W_lo of the two real
            // inputs (fcr_img.h), so the lo image is not read and its W_lo·dgate_hi product is not issued
            const bool hi_only = TAILT && tau == NB - 1;
            f16x8 ah, al;
            const f16x4 h0 = lds_tr_f16(tb + ct), l0 = (LP || hi_only) ? f16x4{0, 0, 0, 0} : lds_tr_f16(tbl + ct);
            f16x4 h1 = {0, 0, 0, 0}, l1 = {0, 0, 0, 0};
            if (two) {
                h1 = lds_tr_f16(tb + ct + TILE);
                if (!LP && !hi_only) l1 = lds_tr_f16(tbl + ct + TILE);
            } else if (!LP) {
                // half block: the upper k-halves are read again instead of copied (a VGPR copy into an MFMA
                // operand costs two v_mov and an s_nop per tile): W_hi once more for the shared hi·hi | hi·lo
                // MFMA below, and W_lo once more as the (finite) partner of the padding slot's zero dgates
                uint32_t tbd = tb, tbld = tbl;
                asm volatile("" : "+v"(tbd), "+v"(tbld));
                h1 = lds_tr_f16(tbd + ct);
                if (!hi_only) l1 = lds_tr_f16(tbld + ct);
            }
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                ah[k] = h0[k];
                ah[4 + k] = h1[k];
                al[k] = l0[k];
                al[4 + k] = l1[k];
            }
            // the products only feed the cell's outputs, so IR passes would sink every MFMA to the end
            // of the cell (all fragments live at once); naming the accumulator keeps block kb-1's
            // MFMAs ahead of this point (issued ~NB*3 MFMAs ago: no hazard wait)
            if (kbb > 0) asm volatile("" : "+v"(acc[tau]));
            if (!two && !LP) {
                // half block (odd HS: its second slot is padding, k 4..7 of every group zero): the
                // hi·hi and hi·lo products share ONE MFMA over k = [W_hi d_hi | W_hi d_lo], then lo·hi
                typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
                const u32x4 h = __builtin_bit_cast(u32x4, gh[cu]), l = __builtin_bit_cast(u32x4, gl[cu]);
                acc[tau] = mfma16(ah, __builtin_bit_cast(f16x8, u32x4{h[0], h[1], l[0], l[1]}), acc[tau]);   // ah = [W_hi | W_hi]
                if (!hi_only) acc[tau] = mfma16(al, gh[cu], acc[tau]);
            } else if (hi_only) {
                acc[tau] = mfma16(ah, gl[cu], acc[tau]);
                acc[tau] = mfma16(ah, gh[cu], acc[tau]);
            } else {
                acc[tau] = mma_p<LP>(ah, al, gh[cu], gl[cu], acc[tau]);
            }
        }
        if (kbb + 1 < KBB) {
            dgate_block(kbb + 1, fa[(kbb + 1) % 3], gh[nu], gl[nu]);
            dg_store(kbb + 1, gh[nu], gl[nu]);
        }
        // every slot's own h consumed: the next cell's record comes in (an L2 hit: this cell read it as h_{t-1})
        if (NX_OWNH && kbb + 2 == KBB) {
            if constexpr (OWN_REG) {
#pragma unroll
                for (int k = 0; k < Geo<HS>::HQ; ++k) ci.o[k] = hkeep[k];
            } else {
                ld_rec<HS, rec_words<HS, LP>()>(ci.o, nx.rh, nx.o, lane);
            }
        }
    }
    sched_fence();
    const unsigned long long t2 = stamp_now();
    if (L0) {
#pragma unroll
        for (int s = 0; s < HS; ++s) dh[s] = acc[s >> 2][s & 3] * down;
        dxq = acc[HS >> 2][HS & 3] * down;
        dx4 = acc[(HS + 1) >> 2][(HS + 1) & 3] * down;
    } else {
        if (TAILT) {   // the last tile's padding rows 2HS, 2HS+1 carry the W_lo terms of rows 2HS-2, 2HS-1
            acc[NB - 1][0] += acc[NB - 1][2];
            acc[NB - 1][1] += acc[NB - 1][3];
        }
#pragma unroll
        for (int s = 0; s < HS; ++s) {
            dxo[s] = acc[s >> 2][s & 3] * down;
            dh[s] = acc[(HS + s) >> 2][(HS + s) & 3] * down;
        }
    }
    if (FCR_STAMP) {
        const unsigned long long t3 = stamp_now();
        sp.t[0] += t1 - t0;
        sp.t[1] += t2 - t1;
        sp.t[2] += t3 - t2;
        sp.t[3] += 1;
    }
}

// fp32 mode: [one image region, refilled per phase (layer 2, 1, 0: hi then lo) | misc];
// f16 mode:  [layer 2 hi | layer 1 hi | layer 0 hi | misc], all resident (no refills)
template <int HS, bool LP>
struct BwdLds {
    using I1 = Img<HS, false>;
    using I0 = Img<HS, true>;
    static constexpr int REGION = LP ? 2 * I1::HALF + I0::HALF : (I1::BYTES > I0::BYTES ? I1::BYTES : I0::BYTES);
    static constexpr int FNP = kMS * 4 * kFnpStride, FCP = kOut * HS * 4;
    static constexpr int BYTES = REGION + (FNP + FCP) * 4;
    static_assert(BYTES <= 163840, "weight images exceed the 160 KiB LDS");
    static_assert(I1::HALF % 16 == 0 && I0::HALF % 16 == 0, "images must be whole 16-B chunks");
};

template <int HS, bool LP>
__global__ __launch_bounds__(kBwdWaves * kWave, kBwdWaves / 4) void fcr_bwd_kernel(BwdArgs a) {
    using LD = BwdLds<HS, LP>;
    using I1 = Img<HS, false>;
    using I0 = Img<HS, true>;
    extern __shared__ __attribute__((aligned(16))) float lw[];
    float *lw1 = lw + (LP ? I1::HALF / 4 : 0);      // layer-1 image (f16 mode: resident beside layer 2's)
    float *lw0 = lw + (LP ? 2 * I1::HALF / 4 : 0);  // layer-0 image (fp32 mode: the same refilled region)
    float *lfnp = lw + LD::REGION / 4;              // resident controller records
    float *lfcp = lfnp + LD::FNP;                   // resident fc.weight (lane layout)
    if (LP) {
        lds_copy(lw, a.p.img[2], I1::HALF / 4);     // hi images only: the first half of each
        lds_copy(lw1, a.p.img[1], I1::HALF / 4);
        lds_copy(lw0, a.p.img[0], I0::HALF / 4);
    }
    lds_copy(lfnp, a.p.fnp, LD::FNP);
    lds_copy(lfcp, a.p.fcp, LD::FCP);
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
    const float scq = a.p.wsc[q], sc4 = a.p.wsc[4];   // range guard (fcr_pack.h): d/dv = 2^-s_c d/dv'
    const float s84 = a.states[(size_t)bc * kL * kIn + (kL - 2) * kIn + 4];
    const float *pred = a.prediction + (size_t)bc * N;
    const float *xh = a.xhat + (size_t)bc * N * kOut;
    const ImgLane<I1::U> L1 = img_lane<I1::U>(lds_offset(lw), lane);      // layer 2 (fp32: layers 2, 1)
    const ImgLane<I1::U> L1b = img_lane<I1::U>(lds_offset(lw1), lane);    // layer 1
    const ImgLane<I0::U> L0 = img_lane<I0::U>(lds_offset(lw0), lane);

    // window-row gradients dx(w, t) (lane group q: column q; lane group 0 also column 4) go to a
    // per-wave slab; row rho = w + t of the extended sequence sums the windows that contained it.
    const __amdgpu_buffer_rsrc_t rr = wave_rsrc(a.dxrow + (size_t)wave * N * kL * kWave, (size_t)N * kL * kWave * 8);
    auto row_grad = [&](int rho) {   // sum over windows w = max(0, rho-9) .. min(N-1, rho) of dx(w, rho-w)
        f32x2 acc2 = {0.0f, 0.0f};
        const int w_hi = rho < N - 1 ? rho : N - 1;
        const int w_lo = rho - (kL - 1) > 0 ? rho - (kL - 1) : 0;
        for (int w = w_hi; w >= w_lo; --w) acc2 += buf_ld2(rr, lane * 8, (uint32_t)((w * kL + (rho - w)) * kWave * 8));
        return acc2;
    };
    float dh[HS], dc[HS], dxo[HS], dab[HS];

    // this wave's slab regions
    const size_t qcell = (size_t)Geo<HS>::QC;   // one cell of a sequence slab, in 16-B units
    const size_t seq_sz = (size_t)N * kLayers * kL * qcell;
    const size_t dseq_sz = (size_t)N * 2 * kL * qcell;
    NextIn nb;
    nb.rh = wave_rsrc(a.hseq + (size_t)wave * seq_sz, seq_sz * 16);
    nb.rc = wave_rsrc(a.cseq + (size_t)wave * seq_sz, seq_sz * 16);
    nb.rx = wave_rsrc(a.xw + (size_t)wave * N * kL * kWave, (size_t)N * kL * kWave * 8);
    nb.rd = wave_rsrc(a.dseq + (size_t)wave * dseq_sz, dseq_sz * 16);
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
        if (nj < 0) { nj = 0; nl = 2; nt = 9; }   // past the last cell: reload a valid one (harmless)
        n.x = nl == 0 ? (uint32_t)((nj * kL + nt) * kWave * 8) : hoff(nj, nl > 0 ? nl - 1 : 0, nt);
        n.h = hoff(nj, nl, nt > 0 ? nt - 1 : 0);
        n.c = n.h;
        n.o = hoff(nj, nl, nt);   // the next cell's own h_t (not stored for layer 2's t = 9: not fetched then)
        n.d = (uint32_t)((nl < 2 ? doff(nj, nl + 1, nt) : 0) * 16);
        return n;
    };
    Stamps sp = {{0, 0, 0, 0, (unsigned long long)((threadIdx.x >> 8) & 1), 0, 0, 0}};
    const unsigned long long tk0 = stamp_now();
    CellIn<HS> ci;
    {
        const NextIn f = next_of(N - 1, 2, kL);   // t = kL -> (N-1, 2, 9)
        load_xhd<HS, false, true, false, LP>(ci, f, lane);
        ld_rec<HS, rec_words<HS, LP>()>(ci.c, f.rc, f.c, lane);   // (c records: f16 halves in the f16 mode)
    }

    for (int j = N - 1; j >= 0; --j) {
        const unsigned long long tw0 = stamp_now();
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
            const f32x2 G = row_grad(kL + j);
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
        const unsigned long long tw1 = stamp_now();
        if (!LP) {
            lds_fill<I1::BYTES, kBwdWaves>(lw, a.p.img[2]);
        }
        if (FCR_STAMP) {
            const unsigned long long tw2 = stamp_now();
            sp.t[5] += tw1 - tw0;
            sp.t[6] += tw2 - tw1;
        }
#pragma unroll
        for (int r = 0; r < HS; ++r) dh[r] = dc[r] = 0.0f;
        // t = 9 .. 2: the next cell is t-1 of the same layer; t = 1: the next is the FIRST cell (no
        // h, c); t = 0: the next is t = 9 of the layer below (or of layer 2 of the previous window)
        // t = 9: h_9 of layer 2 only fed the readout (no split record), so this cell re-evaluates tanh(c_9)
        bwd_cell<HS, false, false, false, false, true, false, LP, false>(L1.fb, L1.tb, lane, dh_out, dh, dc, dxo, unused0,
                                                                    unused1, ci, next_of(j, 2, kL - 1), sp);
        din_store<HS, LP>(nb.rd, (uint32_t)((doff(j, 2, kL - 1)) * 16), dxo, lane);
#pragma unroll
        for (int r = 0; r < HS; ++r) dab[r] = 0.0f;
        for (int t = kL - 2; t >= 2; --t) {
            bwd_cell<HS, false, false, false, false, true, false, LP>(L1.fb, L1.tb, lane, dab, dh, dc, dxo, unused0,
                                                                unused1, ci, next_of(j, 2, t), sp);
            din_store<HS, LP>(nb.rd, (uint32_t)((doff(j, 2, t)) * 16), dxo, lane);
        }
        bwd_cell<HS, false, false, false, false, false, false, LP>(L1.fb, L1.tb, lane, dab, dh, dc, dxo, unused0,
                                                             unused1, ci, next_of(j, 2, 1), sp);
        din_store<HS, LP>(nb.rd, (uint32_t)((doff(j, 2, 1)) * 16), dxo, lane);
        bwd_cell<HS, false, false, true, false, true, true, LP>(L1.fb, L1.tb, lane, dab, dh, dc, dxo, unused0,
                                                          unused1, ci, next_of(j, 2, 0), sp);
        din_store<HS, LP>(nb.rd, (uint32_t)((doff(j, 2, 0)) * 16), dxo, lane);
        // ---- layer 1 ----
        const unsigned long long tw3 = stamp_now();
        if (!LP) {
            lds_fill<I1::BYTES, kBwdWaves>(lw, a.p.img[1]);
        }
        if (FCR_STAMP) sp.t[7] += stamp_now() - tw3;
#pragma unroll
        for (int r = 0; r < HS; ++r) dh[r] = dc[r] = 0.0f;
        for (int t = kL - 1; t >= 2; --t) {
            bwd_cell<HS, false, true, false, false, true, true, LP>(L1b.fb, L1b.tb, lane, dab, dh, dc, dxo, unused0,
                                                              unused1, ci, next_of(j, 1, t), sp);
            din_store<HS, LP>(nb.rd, (uint32_t)((doff(j, 1, t)) * 16), dxo, lane);
        }
        bwd_cell<HS, false, true, false, false, false, true, LP>(L1b.fb, L1b.tb, lane, dab, dh, dc, dxo, unused0,
                                                           unused1, ci, next_of(j, 1, 1), sp);
        din_store<HS, LP>(nb.rd, (uint32_t)((doff(j, 1, 1)) * 16), dxo, lane);
        bwd_cell<HS, false, true, true, true, true, true, LP>(L1b.fb, L1b.tb, lane, dab, dh, dc, dxo, unused0,
                                                        unused1, ci, next_of(j, 1, 0), sp);
        din_store<HS, LP>(nb.rd, (uint32_t)((doff(j, 1, 0)) * 16), dxo, lane);
        // ---- layer 0: dx -> window-row gradients ----
        if (!LP) {
            lds_fill<I0::BYTES, kBwdWaves>(lw, a.p.img[0]);
        }
#pragma unroll
        for (int r = 0; r < HS; ++r) dh[r] = dc[r] = 0.0f;
        for (int t = kL - 1; t >= 2; --t) {
            float dxq, dx4;
            bwd_cell<HS, true, true, false, true, true, true, LP>(L0.fb, L0.tb, lane, dab, dh, dc, dxo, dxq, dx4, ci,
                                                            next_of(j, 0, t), sp);
            buf_st2(rr, lane * 8, (uint32_t)((j * kL + t) * kWave * 8), f32x2{dxq * scq, dx4 * sc4});   // row j+t
        }
        {
            float dxq, dx4;
            bwd_cell<HS, true, true, false, true, false, true, LP>(L0.fb, L0.tb, lane, dab, dh, dc, dxo, dxq, dx4, ci,
                                                             next_of(j, 0, 1), sp);
            buf_st2(rr, lane * 8, (uint32_t)((j * kL + 1) * kWave * 8), f32x2{dxq * scq, dx4 * sc4});   // row j+1
            bwd_cell<HS, true, true, true, false, true, false, LP, true, false>(L0.fb, L0.tb, lane, dab, dh, dc, dxo, dxq,
                                                                           dx4, ci, next_of(j, 0, 0), sp);
            buf_st2(rr, lane * 8, (uint32_t)((j * kL) * kWave * 8), f32x2{dxq * scq, dx4 * sc4});   // row j
        }
    }
    const float g_u0_rows = row_grad(kL - 1)[1];   // row 9, col 4 = u0 (Functions.py:1396)
    // command-cost terms of u0: cmd_0 = a(s84 - u0)^2, cmd_1 = a(u0 - u1)^2
    float du0 = 2.0f * alpha * wgt * (pred[0] - s84);
    if (N > 1) du0 += 2.0f * alpha * wgt * (pred[0] - pred[1]);
    if (valid && q == 0) a.g_u0[b] = g_u0_rows + du0;
    if (FCR_STAMP && lane == 0) {
        unsigned long long *o = a.stamp + (size_t)wave * 8;
        o[0] = sp.t[0];
        o[1] = sp.t[1];
        o[2] = sp.t[2];
        o[3] = sp.t[3];
        o[4] = stamp_now() - tk0;
        o[5] = sp.t[5];
        o[6] = sp.t[6];
        o[7] = sp.t[7];
    }
}

}  // namespace fcr
