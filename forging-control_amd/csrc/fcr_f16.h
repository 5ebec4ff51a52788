// fcr_f16.h — fp32-accurate gate products on the f16 matrix cores (v_mfma_f32_16x16x32_f16).
//
// Every fp32 operand v is split into two f16 halves, hi = f16(v), lo = f16(v - hi) (|v - hi - lo| <=
// 2^-22 |v| for normal values), and a product a·b is accumulated in fp32 as lo_a·hi_b + hi_a·lo_b +
// hi_a·hi_b (the dropped lo·lo term is <= 2^-22 |a b|). One 16x16x32 f16 MFMA does the work of eight
// 16x16x4 f32 MFMAs in half the cycles, so three of them cost 3/16 of the f32 matrix time at an
// accuracy comparable to fp32 (tests/test_gpu_parity.py holds the result to 1e-5 of the fp64 oracle).
//
// Forward operand geometry (k = 8·(lane>>4) + j inside a 32-wide k-block, j = 0..7 = the 8 halves a
// lane holds): tile r = D rows (units 4r..4r+3) x (gates i,f,g,o); the k index runs over the layer's
// input in "combined slots" σ = 8kb + j of lane group q = lane>>4 (unit 4σ'+q of the part σ falls in):
//   layer >= 1: σ < HS -> layer-below h_t slot σ, HS <= σ < 2HS -> h_{t-1} slot σ-HS;
//   layer 0:    σ < HS -> h_{t-1} slot σ, σ = HS -> window column q, σ = HS+1 -> column 4 (group 0).
// So every lane's B operand is its OWN registers — no cross-lane move — and the k layout is the column
// layout of the backward's weight image (fcr_img.h), which recomputes exactly these products.
// The backward scales each trajectory's dgates by a power of two before splitting (exact), so values
// never leave the f16 normal range; the products are scaled back exactly afterwards.
#pragma once
#include "fcr_common.h"
#include "fcr_pack.h"

namespace fcr {

typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));

// Packed tail block (layers >= 1 when 2·HS = 8·(KB1-1) + 2, i.e. HS = 13): the last k-block holds
// only combined slots 2HS-2, 2HS-1 (6 of its 8 k are zero padding), so its three split products go
// into ONE MFMA over k = [A_hi B_hi | A_lo B_hi | A_hi B_lo | 0 0]: the A fragment carries
// (hi σ0, hi σ1, lo σ0, lo σ1, hi σ0, hi σ1, 0, 0) and the B operand (hi, hi, hi, hi, lo, lo, 0, 0)
// of the two slots. 10 instead of 12 MFMAs per tile and 13 % less fragment LDS at H = 50. The lo copies
// sit at k positions 2, 3 — combined slots 2HS, 2HS+1 of the backward's weight image (fcr_img.h) — so the
// transposed product's last output tile, whose rows 2HS, 2HS+1 are padding, reads W_lo there from the hi
// image and gets the W_lo·dgate_hi term for free (fcr_bwd.h).
__host__ __device__ constexpr bool tail_packed(int HS) { return 2 * HS - 8 * ((2 * HS + 7) / 8 - 1) == 2; }

template <int HS>
struct Geo16 {
    static constexpr int KB0 = (HS + 2 + 7) / 8;                    // layer-0 k-blocks
    static constexpr int XBLK = HS >> 3;                            // layer-0 block holding the columns
    static constexpr int KB1 = (2 * HS + 7) / 8;                    // layers >= 1
    static constexpr int KX1 = (HS + 7) / 8;                        // layers >= 1: blocks holding x slots
    static constexpr bool TAIL1 = tail_packed(HS);                  // layers >= 1: packed last block
    static constexpr int QF0 = HS * KB0 * 2;                        // fragment quads (64 lanes x 16 B)
    static constexpr int QH1 = HS * KB1;                            // layers >= 1: hi quads (tail included)
    static constexpr int QF1 = QH1 + HS * (KB1 - (TAIL1 ? 1 : 0));  //   + lo quads
    static constexpr int FA0 = QF0 * kWave * 4, FA1 = QF1 * kWave * 4, FH1 = QH1 * kWave * 4;   // floats
    static constexpr int FNP = kMS * 4 * kFnpStride;
    static constexpr int FCP = kOut * HS * 4;
    static constexpr int MISC = FNP + FCP + 4;
    static constexpr int LDS_FWD = (FA1 + FA0 + MISC) * 4;   // bytes
    // f16 mode: the hi fragments of all three layers stay resident (no per-phase refills)
    static constexpr int LDS_FWD_LP = (2 * FH1 + FA0 / 2 + MISC) * 4;
    static_assert(LDS_FWD <= 163840 && LDS_FWD_LP <= 163840, "fragments exceed the 160 KiB LDS");
    static_assert((HS & 7) + 1 < 8, "window columns must share one k-block");
};

// B operand of the packed tail block from the block's split halves (elements 0, 1 are the two real
// slots): (hi, hi, hi, hi, lo, lo, 0, 0); the f16 mode keeps only the hi·hi part.
template <bool LP>
__device__ __forceinline__ f16x8 tail_operand(f16x8 bh, f16x8 bl) {
    typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
    const u32x4 h = __builtin_bit_cast(u32x4, bh), l = __builtin_bit_cast(u32x4, bl);
    return __builtin_bit_cast(f16x8, LP ? u32x4{h[0], 0u, 0u, 0u} : u32x4{h[0], h[0], l[0], 0u});
}

__device__ __forceinline__ f32x4 mfma16(f16x8 a, f16x8 b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ f16x8 lds_frag16(const float *lw, int idx, int lane) {
    return __builtin_bit_cast(f16x8, lds_quad(lw, idx, lane));
}

// The splits below are plain (_Float16)fmaf(a, b, c), which the backend selects as v_fma_mix* (~2.5
// instructions per value) with the MFMA operand hazards padded. (An inline-asm v_fma_mixlo/mixhi pair is 2, but
// the hazard recognizer does not look inside inline asm: an asm write of a VGPR an MFMA issued just before still
// reads went out unpadded, DESIGN.md §2 "Inline asm and MFMA hazards".)
// (hi, lo) of the products a·b for two values; hi = f16(a·b), lo = f16(a·b - hi), the product exact in the fma
__device__ __forceinline__ void mix_pair(float a0, float b0, float a1, float b1, unsigned &hp, unsigned &lp) {
    typedef _Float16 f16x2 __attribute__((ext_vector_type(2)));
    f16x2 h, l;
    h[0] = (_Float16)__builtin_fmaf(a0, b0, 0.0f);
    h[1] = (_Float16)__builtin_fmaf(a1, b1, 0.0f);
    l[0] = (_Float16)__builtin_fmaf(a0, b0, -(float)h[0]);
    l[1] = (_Float16)__builtin_fmaf(a1, b1, -(float)h[1]);
    hp = __builtin_bit_cast(unsigned, h);
    lp = __builtin_bit_cast(unsigned, l);
}
__device__ __forceinline__ unsigned mix_hi(float a0, float b0, float a1, float b1) {
    typedef _Float16 f16x2 __attribute__((ext_vector_type(2)));
    f16x2 h;
    h[0] = (_Float16)__builtin_fmaf(a0, b0, 0.0f);
    h[1] = (_Float16)__builtin_fmaf(a1, b1, 0.0f);
    return __builtin_bit_cast(unsigned, h);
}

// v -> (hi, lo) halves, 8 at a time
__device__ __forceinline__ void split8(const float (&v)[8], f16x8 &hi, f16x8 &lo) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        const _Float16 h = (_Float16)v[j];
        hi[j] = h;
        lo[j] = (_Float16)(v[j] - (float)h);
    }
}

// s·v -> (hi, lo) halves, 8 at a time, on the mixed-precision FMA: hi = f16(s·v) goes straight into a packed
// register and lo = f16(s·v - hi) (the product is exact inside the fma) — ~2.5 instructions per value, scale
// included, against ~3.5 for the scalar conversions the compiler emits for split8.
__device__ __forceinline__ void split8s(const float (&v)[8], float s, f16x8 &hi, f16x8 &lo) {
    typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
    u32x4 h, l;
    // a constant s = 1 would fold the fma away and lose the v_fma_mix form (cvt/sub/cvt instead)
    asm("" : "+v"(s));
#pragma unroll
    for (int p = 0; p < 4; ++p) {
        unsigned hp, lp;
        mix_pair(v[2 * p], s, v[2 * p + 1], s, hp, lp);
        h[p] = hp;
        l[p] = lp;
    }
    hi = __builtin_bit_cast(f16x8, h);
    lo = __builtin_bit_cast(f16x8, l);
}

// s·v -> hi = f16(s·v) only: the reduced-precision mode's operand (one product, no lo half)
__device__ __forceinline__ void cvt8s(const float (&v)[8], float s, f16x8 &hi) {
    typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
    u32x4 h;
#pragma unroll
    for (int p = 0; p < 4; ++p) {
        h[p] = mix_hi(v[2 * p], s, v[2 * p + 1], s);
    }
    hi = __builtin_bit_cast(f16x8, h);
}

// a·b -> (hi, lo) halves, 8 at a time: the product is formed exactly inside v_fma_mix, so hi = f16(a·b)
// and lo = f16(a·b - hi) cost the same two instructions per value as split8s with no separate multiply
// (the backward's dgates: a = the scaled dc or dh, b = the local derivative).
__device__ __forceinline__ void split8p(const float (&a)[8], const float (&b)[8], f16x8 &hi, f16x8 &lo) {
    typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
    u32x4 h, l;
#pragma unroll
    for (int p = 0; p < 4; ++p) {
        unsigned hp, lp;
        mix_pair(a[2 * p], b[2 * p], a[2 * p + 1], b[2 * p + 1], hp, lp);
        h[p] = hp;
        l[p] = lp;
    }
    hi = __builtin_bit_cast(f16x8, h);
    lo = __builtin_bit_cast(f16x8, l);
}
__device__ __forceinline__ void cvt8p(const float (&a)[8], const float (&b)[8], f16x8 &hi) {
    typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
    u32x4 h;
#pragma unroll
    for (int p = 0; p < 4; ++p) {
        h[p] = mix_hi(a[2 * p], b[2 * p], a[2 * p + 1], b[2 * p + 1]);
    }
    hi = __builtin_bit_cast(f16x8, h);
}

// Precision modes (fcr_dims.precision): LP = false — fp32-accurate split products (three MFMAs);
// LP = true — config 3's reduced-precision mode: f16 operands, ONE MFMA per product, fp32 accumulate
template <bool LP>
__device__ __forceinline__ void split_p(const float (&v)[8], float s, f16x8 &hi, f16x8 &lo) {
    if (LP) cvt8s(v, s, hi);
    else split8s(v, s, hi, lo);
}
template <bool LP>
__device__ __forceinline__ void split_pp(const float (&a)[8], const float (&b)[8], f16x8 &hi, f16x8 &lo) {
    if (LP) cvt8p(a, b, hi);
    else split8p(a, b, hi, lo);
}

// a·b with a = (ah, al), b = (bh, bl): small terms first, then the leading product
__device__ __forceinline__ f32x4 mma3(f16x8 ah, f16x8 al, f16x8 bh, f16x8 bl, f32x4 acc) {
    acc = mfma16(al, bh, acc);
    acc = mfma16(ah, bl, acc);
    return mfma16(ah, bh, acc);
}
template <bool LP>
__device__ __forceinline__ f32x4 mma_p(f16x8 ah, f16x8 al, f16x8 bh, f16x8 bl, f32x4 acc) {
    if (LP) return mfma16(ah, bh, acc);
    return mma3(ah, al, bh, bl, acc);
}

// B operand (8 combined slots of k-block kb) of a forward cell, from the lane's own registers.
// FIRST: h_{t-1} = 0. Identical in the forward kernel and the backward's recomputation.
template <int HS, bool L0, bool FIRST, bool LP>
__device__ __forceinline__ void fwd_operand(int kb, float x0, float x1, const float (&x)[HS],
                                            const float (&hp)[HS], f16x8 &bh, f16x8 &bl) {
    float v[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        const int s = 8 * kb + j;
        float e = 0.0f;
        if (L0) {
            if (s < HS) e = FIRST ? 0.0f : hp[s < HS ? s : 0];
            else if (s == HS) e = x0;
            else if (s == HS + 1) e = x1;
        } else {
            if (s < HS) e = x[s < HS ? s : 0];
            else if (s < 2 * HS) e = FIRST ? 0.0f : hp[(s >= HS && s < 2 * HS) ? s - HS : 0];
        }
        v[j] = e;
    }
    split_p<LP>(v, 1.0f, bh, bl);
}

// ---- split records ----
// A cell's h leaves the cell already split into the f16 halves every consumer multiplies with (the next
// cell's h_{t-1}, the layer above's x_t, the backward's recompute of both): its record (the compact slab
// record of fcr_common.h, HS 32-bit values per lane) holds the half array [hi(slot 0..HS-1) | lo(slot
// 0..HS-1)], hi = f16(h), lo = f16(h - hi), dword d = halves 2d (low) and 2d+1 (high). The B operands are
// then assembled from record dwords with alignbit / perm (compile-time selects) instead of re-splitting fp32
// values — the same halves, so the products are bit for bit those of a split at the consumer.
// LP (the f16 mode, whose products take the hi halves only): words d < ceil(HS / 2) = hi halves 2d, 2d + 1 — half the
// record's bytes; the remaining words are left as they are (never stored nor read).
template <int HS, bool LP = false>
__device__ __forceinline__ void split_rec(const float (&h)[HS], float (&r)[HS]) {
    typedef _Float16 f16x2 __attribute__((ext_vector_type(2)));
    if constexpr (LP) {
#pragma unroll
        for (int d = 0; d < (HS + 1) / 2; ++d) {
            f16x2 v;
            v[0] = (_Float16)h[2 * d];
            v[1] = 2 * d + 1 < HS ? (_Float16)h[2 * d + 1 < HS ? 2 * d + 1 : 0] : (_Float16)0.0f;
            r[d] = __builtin_bit_cast(float, v);
        }
        return;
    }
    float one = 1.0f;
    asm("" : "+v"(one));   // keeps the v_fma_mix form (a constant 1 folds the fma away)
    _Float16 hh[HS], ll[HS];
#pragma unroll
    for (int k = 0; k < HS; ++k) {
        hh[k] = (_Float16)__builtin_fmaf(h[k], one, 0.0f);
        ll[k] = (_Float16)__builtin_fmaf(h[k], one, -(float)hh[k]);
    }
#pragma unroll
    for (int d = 0; d < HS; ++d) {
        f16x2 v;
        v[0] = 2 * d < HS ? hh[2 * d < HS ? 2 * d : 0] : ll[2 * d >= HS ? 2 * d - HS : 0];
        v[1] = 2 * d + 1 < HS ? hh[2 * d + 1 < HS ? 2 * d + 1 : 0] : ll[2 * d + 1 >= HS ? 2 * d + 1 - HS : 0];
        r[d] = __builtin_bit_cast(float, v);
    }
}

// One 32-bit word of an operand from two halves, each (source, half index) with the source a record
// (1: x record, 2: h record) or the on-the-fly split window pair (3: hi pair, 4: lo pair), 0 = zero.
// Compile-time arguments: one alignbit or perm (or a plain register) per word.
struct HalfRef {
    int src, k;
};
template <int HS>
__device__ __forceinline__ uint32_t rec_word(HalfRef a, HalfRef b, const float (&xr)[HS], const float (&hr)[HS],
                                             uint32_t wh, uint32_t wl) {
    auto dw = [&](HalfRef h) -> uint32_t {
        if (h.src == 1) return __builtin_bit_cast(uint32_t, xr[h.k >> 1]);
        if (h.src == 2) return __builtin_bit_cast(uint32_t, hr[h.k >> 1]);
        return h.src == 3 ? wh : wl;
    };
    if (a.src == 0 && b.src == 0) return 0u;
    if (b.src == 0) return (a.k & 1) ? dw(a) >> 16 : dw(a) & 0xffffu;
    if (a.src == 0) return (b.k & 1) ? dw(b) & 0xffff0000u : dw(b) << 16;
    if (a.src == b.src && (b.k >> 1) == (a.k >> 1) && (a.k & 1) == 0 && (b.k & 1) == 1) return dw(a);
    if (a.src == b.src && (a.k & 1) == 1 && b.k == a.k + 1) return __builtin_amdgcn_alignbit(dw(b), dw(a), 16);
    // perm: bytes 0-3 select from the second source, 4-7 from the first
    const uint32_t sel = (uint32_t)(2 * (a.k & 1)) | (uint32_t)(2 * (a.k & 1) + 1) << 8 | (uint32_t)(4 + 2 * (b.k & 1)) << 16 |
                         (uint32_t)(5 + 2 * (b.k & 1)) << 24;
    return __builtin_amdgcn_perm(dw(b), dw(a), sel);
}

// B operand (8 combined slots of k-block kb) of a cell from the split records: layer >= 1 — x record (the
// layer below's h_t, σ < HS) and h record (h_{t-1}, σ - HS); layer 0 — h record (σ < HS) and the window
// columns x0 (σ = HS), x1 (σ = HS + 1), split here. FIRST: h_{t-1} = 0. Identical in the forward kernels
// and the backward's recomputation.
template <int HS, bool L0, bool FIRST, bool LP>
__device__ __forceinline__ void rec_operand(int kb, float x0, float x1, const float (&xr)[HS], const float (&hr)[HS],
                                            f16x8 &bh, f16x8 &bl) {
    typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
    typedef _Float16 f16x2 __attribute__((ext_vector_type(2)));
    uint32_t wh = 0u, wl = 0u;
    if (L0 && 8 * kb <= HS + 1 && HS < 8 * kb + 8) {   // the window columns fall in this block
        float one = 1.0f;
        asm("" : "+v"(one));
        f16x2 h, l;
        h[0] = (_Float16)__builtin_fmaf(x0, one, 0.0f);
        h[1] = (_Float16)__builtin_fmaf(x1, one, 0.0f);
        l[0] = (_Float16)__builtin_fmaf(x0, one, -(float)h[0]);
        l[1] = (_Float16)__builtin_fmaf(x1, one, -(float)h[1]);
        wh = __builtin_bit_cast(uint32_t, h);
        wl = __builtin_bit_cast(uint32_t, l);
    }
    auto ref = [&](int sg, bool lo) -> HalfRef {
        if (L0) {
            if (sg < HS) return FIRST ? HalfRef{0, 0} : HalfRef{2, lo ? HS + sg : sg};
            if (sg == HS) return HalfRef{lo ? 4 : 3, 0};
            if (sg == HS + 1) return HalfRef{lo ? 4 : 3, 1};
            return HalfRef{0, 0};
        }
        if (sg < HS) return HalfRef{1, lo ? HS + sg : sg};
        if (sg < 2 * HS) return FIRST ? HalfRef{0, 0} : HalfRef{2, lo ? sg : sg - HS};
        return HalfRef{0, 0};
    };
    u32x4 H, L;
#pragma unroll
    for (int p = 0; p < 4; ++p) {
        const int s0 = 8 * kb + 2 * p;
        H[p] = rec_word<HS>(ref(s0, false), ref(s0 + 1, false), xr, hr, wh, wl);
        L[p] = LP ? 0u : rec_word<HS>(ref(s0, true), ref(s0 + 1, true), xr, hr, wh, wl);
    }
    bh = __builtin_bit_cast(f16x8, H);
    bl = __builtin_bit_cast(f16x8, L);
}

// Cell update of one unit slot from its pre-activations a = (i, f, g, o), pre-scaled for exp2 (the
// packed weights carry -log2e for i, f, o and 2 log2e for g). The forward needs only c = f c_prev + i g
// and h = o tanh(c), so each of the two products shares ONE reciprocal (e_x = exp2 of a pre-activation):
//   i g      = (e_g - 1) / ((1 + e_i)(1 + e_g))          [fma(e_i, D_g, D_g), rcp, fma(e_g, r, -r)]
//   o tanh c = (e_c - 1) / ((1 + e_o)(1 + e_c))          [e_c = exp2(2 log2e c)]
// 8 transcendentals per slot instead of 10 (f keeps its own). Overflow: e_g is taken at min(a_g, 64), so
// e_g stays finite and an infinite denominator (e_i or e_o = inf: i or o = 0) gives the product 0, as the
// separate sigmoids do; |c| <= 10 (|c_t| <= |c_{t-1}| + 1 from zero), so e_c is finite. The backward's
// recompute (lstm_point_grad*) evaluates i, f, g, o separately, as its local derivatives need them.
// lstm_point_grad forms, from the same arithmetic, the six local derivatives the backward needs:
// P = (dh/dc, dh/do, dc/di, dc/df) and Q = (dc/dg, f), each one fma from products the cell has.
template <bool FIRST>
__device__ __forceinline__ float lstm_gi_c(f32x4 a, float c_prev) {
    const float f = sigm_pre(a[1]);
    const float ei = __builtin_amdgcn_exp2f(a[0]);
    // min(a_g, 64) as ONE v_med3_f32 (fminf adds a canonicalising v_max of the MFMA result in front of it)
    const float eg = __builtin_amdgcn_exp2f(__builtin_amdgcn_fmed3f(a[2], -1e30f, 64.0f));
    const float dg = 1.0f + eg;
    const float r = __builtin_amdgcn_rcpf(fmaf(ei, dg, dg));
    const float gi = fmaf(eg, r, -r);
    return FIRST ? gi : fmaf(f, c_prev, gi);           // c_{-1} = 0 (Functions.py:349-350)
}
__device__ __forceinline__ float lstm_h(float c, float eo) {
    const float ec = __builtin_amdgcn_exp2f(c * 2.8853900817779268f);
    const float dc = 1.0f + ec;
    const float r = __builtin_amdgcn_rcpf(fmaf(eo, dc, dc));
    return fmaf(ec, r, -r);
}
template <bool FIRST>
__device__ __forceinline__ void lstm_point(f32x4 a, float c_prev, float &c, float &h) {
    c = lstm_gi_c<FIRST>(a, c_prev);
    h = lstm_h(c, __builtin_amdgcn_exp2f(a[3]));
}
// lstm_point in two stages (the same arithmetic in the same order), so the forward cell can spread a
// tile pair's pointwise over the next pair's MFMA regions: A = gates and c (and e_o), B = h from (c, e_o)
template <bool FIRST>
__device__ __forceinline__ void lstm_point_a(f32x4 a, float c_prev, float &c, float &eo) {
    c = lstm_gi_c<FIRST>(a, c_prev);
    eo = __builtin_amdgcn_exp2f(a[3]);
}
__device__ __forceinline__ void lstm_point_b(float c, float eo, float &h) {
    h = lstm_h(c, eo);
}
template <bool FIRST>
__device__ __forceinline__ void lstm_point_grad(f32x4 a, float c_prev, f32x4 &P, f32x2 &Q) {
    const float i = sigm_pre(a[0]);
    const float f = sigm_pre(a[1]);
    const float g = tanh_pre(a[2]);
    const float o = sigm_pre(a[3]);
    const float gi = g * i;
    const float cf = FIRST ? 0.0f : f * c_prev;
    const float cn = cf + gi;
    const float tc = tanh_f(cn);
    const float h = o * tc;
    P = f32x4{fmaf(-h, tc, o), fmaf(-h, o, h), fmaf(-gi, i, gi), fmaf(-cf, f, cf)};
    Q = f32x2{fmaf(-gi, g, i), f};
}

// h of unit slot s from its split record (split_rec: hi at half s, lo at half HS + s of the record words):
// hi + lo in ONE v_fma_mix_f32 (f16 sources picked by op_sel; exact in fp32) — the compiler's form of the
// same sum is two conversions and an add. A VALU-to-VALU dependency: no MFMA operand hazard. s is a
// compile-time constant once the cell is unrolled: one of the four op_sel forms survives.
template <int HS, bool LP = false>
__device__ __forceinline__ float rec_h(const f32x4 *rec, int s) {
    if constexpr (LP) {   // the f16 mode's record: hi halves only
        typedef _Float16 f16x2 __attribute__((ext_vector_type(2)));
        const int wh = s >> 1;
        const float wv = rec[wh >> 2][wh & 3];   // (a plain element read: bit_cast of a vector element misreads)
        return (float)__builtin_bit_cast(f16x2, wv)[s & 1];
    }
    const int wh = s >> 1, wl = (HS + s) >> 1;
    const float a = rec[wh >> 2][wh & 3], b = rec[wl >> 2][wl & 3];
    float r;
#define FCR_MIX_H(SA, SB) asm("v_fma_mix_f32 %0, %1, 1.0, %2 op_sel:[" #SA ",0," #SB "] op_sel_hi:[1,0,1]" : "=v"(r) : "v"(a), "v"(b))
    if ((s & 1) == 0 && ((HS + s) & 1) == 0) FCR_MIX_H(0, 0);
    else if ((s & 1) == 0) FCR_MIX_H(0, 1);
    else if (((HS + s) & 1) == 0) FCR_MIX_H(1, 0);
    else FCR_MIX_H(1, 1);
#undef FCR_MIX_H
    return r;
}

// lstm_point_grad with tanh(c_t) recovered from the cell's own h_t (the forward's h_t = o tanh(c_t) with
// o = 1/(1 + e_o), so tanh(c_t) = h_t (1 + e_o), one multiply by the denominator the sigmoid already formed)
// instead of re-evaluated (exp2, rcp and three VALU): the same six local derivatives. h is the forward's h_t
// as its split record holds it (fp32-accurate; f16-subnormal h only perturbs P by the record's absolute
// 2^-25, below the gradients' fp32 level).
template <bool FIRST>
__device__ __forceinline__ void lstm_point_grad_h(f32x4 a, float c_prev, float h, f32x4 &P, f32x2 &Q) {
    const float i = sigm_pre(a[0]);
    const float f = sigm_pre(a[1]);
    const float g = tanh_pre(a[2]);
    // a_o at most 126 (one v_med3): a saturated output gate (the forward's e_o = inf, o = h = 0) keeps d_o finite,
    // so tc = h d_o is 0 there, not 0 * inf (tests/test_surrogate.py, range-guarded columns)
    const float d_o = 1.0f + __builtin_amdgcn_exp2f(__builtin_amdgcn_fmed3f(a[3], -1e30f, 126.0f));
    const float o = __builtin_amdgcn_rcpf(d_o);
    const float gi = g * i;
    const float cf = FIRST ? 0.0f : f * c_prev;
    const float tc = h * d_o;
    P = f32x4{fmaf(-h, tc, o), fmaf(-h, o, h), fmaf(-gi, i, gi), fmaf(-cf, f, cf)};
    Q = f32x2{fmaf(-gi, g, i), f};
}

// host-side geometry of the forward fragment blocks (bytes), matching Geo16
inline size_t f16_fwd_bytes(int HS, int l) {
    const int KB = l == 0 ? (HS + 2 + 7) / 8 : (2 * HS + 7) / 8;
    const int lo_blocks = (l > 0 && tail_packed(HS)) ? KB - 1 : KB;
    return (size_t)HS * (KB + lo_blocks) * kWave * 16;
}

// Scaled weight of the forward product: gate row (unit, gate) x combined slot s of lane group kq.
__device__ __forceinline__ float fwd16_weight(const PackArgs &a, int l, int unit, int gate, int s, int kq) {
    const int H = a.H, HS = a.HS;
    float v = 0.0f;
    if (unit < H) {
        const int grow = gate * H + unit;
        if (l == 0) {
            if (s < HS) {
                const int u = 4 * s + kq;
                if (u < H) v = a.whh[0][grow * H + u];
            } else if (s == HS) {
                v = a.wih[0][grow * kIn + kq] / a.wsc[kq];          // range guard (fcr_pack.h): exact
            } else if (s == HS + 1 && kq == 0) {
                v = a.wih[0][grow * kIn + 4] / a.wsc[4];
            }
        } else if (s < HS) {
            const int u = 4 * s + kq;
            if (u < H) v = a.wih[l][grow * H + u];
        } else if (s < 2 * HS) {
            const int u = 4 * (s - HS) + kq;
            if (u < H) v = a.whh[l][grow * H + u];
        }
    }
    return v * (gate == 2 ? kTwoLog2e : kNegLog2e);
}

// Forward fragments, f16 split: element (split, r, kb, lane, j) = hi|lo of A[rho][k] with rho = lane&15
// -> unit 4r+(rho>>2), gate rho&3 (torch row gate*H + unit), k = combined slot 8kb+j of lane group
// lane>>4 (see the header). Scaled for exp2 as the pointwise expects. Split-major: every hi fragment of
// the layer [r][kb], then every lo one [r][kb] (the f16 mode reads the first part); with a packed tail
// (tail_packed) the hi part's last block of each tile is the packed tail fragment and it has no lo.
__device__ __forceinline__ void pack_fwd16_item(const PackArgs &a, int l, _Float16 *dst, int idx) {
    const int HS = a.HS;
    const int KB = l == 0 ? (HS + 2 + 7) / 8 : (2 * HS + 7) / 8;
    const bool tail = l > 0 && tail_packed(HS);
    const int KL = tail ? KB - 1 : KB;   // lo blocks per tile
    const int n = HS * KB * kWave * 8;
    if (idx >= n) return;
    const int j = idx & 7, lane = (idx >> 3) & 63, rk = idx >> 9;
    const int kb = rk % KB, r = rk / KB;
    const int rho = lane & 15, kq = lane >> 4;
    const int unit = 4 * r + (rho >> 2), gate = rho & 3;
    if (tail && kb == KB - 1) {   // packed tail: (hi s0, hi s1, lo s0, lo s1, hi s0, hi s1, 0, 0)
        _Float16 out = (_Float16)0.0f;
        if (j < 6) {
            const float v = fwd16_weight(a, l, unit, gate, 8 * kb + (j & 1), kq);
            const _Float16 hi = (_Float16)v;
            out = (j == 2 || j == 3) ? (_Float16)(v - (float)hi) : hi;
        }
        dst[((size_t)rk * kWave + lane) * 8 + j] = out;
        return;
    }
    const float v = fwd16_weight(a, l, unit, gate, 8 * kb + j, kq);
    const _Float16 hi = (_Float16)v;
    const _Float16 lo = (_Float16)(v - (float)hi);
    const size_t nq = (size_t)HS * KB;
    dst[((size_t)rk * kWave + lane) * 8 + j] = hi;
    dst[((nq + (size_t)r * KL + kb) * kWave + lane) * 8 + j] = lo;
}
__global__ void pack_fwd16_kernel(PackArgs a, int l, _Float16 *dst) {
    pack_fwd16_item(a, l, dst, blockIdx.x * blockDim.x + threadIdx.x);
}

}  // namespace fcr
