// fcr_f16.h — fp32-accurate gate products on the f16 matrix cores (v_mfma_f32_16x16x32_f16).
//
// Every fp32 operand v is split into two f16 halves, hi = f16(v), lo = f16(v - hi) (|v - hi - lo| <=
// 2^-22 |v| for normal values), and a product a·b is accumulated in fp32 as lo_a·hi_b + hi_a·lo_b +
// hi_a·hi_b (the dropped lo·lo term is <= 2^-22 |a b|). One 16x16x32 f16 MFMA does the work of eight
// 16x16x4 f32 MFMAs in half the cycles, so three of them cost 3/16 of the f32 matrix time at an
// accuracy comparable to fp32 (tests/test_gpu_parity.py holds the result to 1e-5 of the fp64 oracle).
//
// Operand geometry (k = 8·(lane>>4) + j inside a 32-wide k-block, j = 0..7 = the 8 halves a lane holds):
//   forward tile r (D rows = units 4r..4r+3 x gates i,f,g,o, exactly as the f32 path), k-blocks over a
//   unit-slot vector: block kb, lane group q, j -> unit 4(8kb+j)+q, i.e. lane q's OWN slots 8kb..8kb+7;
//   layer 0 puts the 5 window columns at j = 5 (column q) and j = 6 (column 4, lane group 0) of the
//   block XBLK (the last h block when HS%8 <= 5 leaves those slots free);
//   backward k-block kb = unit slots 2kb, 2kb+1 x gates: j -> slot 2kb + (j>>2), gate j&3.
// The backward scales each trajectory's dgates by a power of two before splitting (exact), so values
// never leave the f16 normal range; the products are scaled back exactly afterwards.
#pragma once
#include "fcr_common.h"
#include "fcr_pack.h"

namespace fcr {

typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));

template <int HS>
struct Geo16 {
    static constexpr int KBH = (HS + 7) / 8;                       // k-blocks over a unit-slot vector
    static constexpr bool XIN = (HS % 8 >= 1) && (HS % 8 <= 5);     // window columns fit in the last h block
    static constexpr int KB0 = XIN ? KBH : KBH + 1;                 // layer-0 k-blocks
    static constexpr int XBLK = XIN ? KBH - 1 : KBH;                // layer-0 block holding the columns
    static constexpr int KB1 = 2 * KBH;                             // layers >= 1: x blocks, then h blocks
    static constexpr int KBB = (HS + 1) / 2;                        // backward k-blocks
    static constexpr int NB0 = (HS + 2 + 3) / 4;
    static constexpr int NB1 = (2 * HS + 3) / 4;
    static constexpr int QF0 = HS * KB0 * 2;                        // fragment quads (64 lanes x 16 B)
    static constexpr int QF1 = HS * KB1 * 2;
    static constexpr int QB0 = NB0 * KBB * 2;
    static constexpr int QB1 = NB1 * KBB * 2;
    static constexpr int FA0 = QF0 * kWave * 4, FA1 = QF1 * kWave * 4;   // floats
    static constexpr int BA0 = QB0 * kWave * 4, BA1 = QB1 * kWave * 4;
    static constexpr int FNP = kMS * 4 * kFnpStride;
    static constexpr int FCP = kOut * HS * 4;
    static constexpr int MISC = FNP + FCP + 4;
    static constexpr int LDS_FWD = (FA1 + FA0 + MISC) * 4;   // bytes
    static constexpr int LDS_BWD = (BA1 + BA0 + MISC) * 4;
    static_assert(LDS_FWD <= 163840 && LDS_BWD <= 163840, "fragments exceed the 160 KiB LDS");
};

__device__ __forceinline__ f32x4 mfma16(f16x8 a, f16x8 b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ f16x8 lds_frag16(const float *lw, int idx, int lane) {
    return __builtin_bit_cast(f16x8, lds_quad(lw, idx, lane));
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

// a·b with a = (ah, al), b = (bh, bl): small terms first, then the leading product
__device__ __forceinline__ f32x4 mma3(f16x8 ah, f16x8 al, f16x8 bh, f16x8 bl, f32x4 acc) {
    acc = mfma16(al, bh, acc);
    acc = mfma16(ah, bl, acc);
    return mfma16(ah, bh, acc);
}

// host-side geometry of the f16 fragment blocks (bytes), matching Geo16
inline size_t f16_fwd_bytes(int HS, int l) {
    const int KBH = (HS + 7) / 8;
    const bool xin = (HS % 8 >= 1) && (HS % 8 <= 5);
    const int KB = l == 0 ? (xin ? KBH : KBH + 1) : 2 * KBH;
    return (size_t)HS * KB * 2 * kWave * 16;
}
inline size_t f16_bwd_bytes(int HS, int l) {
    const int NB = l == 0 ? (HS + 2 + 3) / 4 : (2 * HS + 3) / 4;
    return (size_t)NB * ((HS + 1) / 2) * 2 * kWave * 16;
}

// Forward fragments, f16 split: element (r, kb, split, lane, j) = hi|lo of A[rho][k] with rho = lane&15
// -> unit 4r+(rho>>2), gate rho&3 (torch row gate*H + unit), k = 8*(lane>>4)+j inside k-block kb; the
// k index names an input unit/column as in the Geo16 comment. Scaled for exp2 like pack_fwd_kernel.
__global__ void pack_fwd16_kernel(PackArgs a, int l, _Float16 *dst) {
    const int H = a.H, HS = a.HS;
    const int KBH = (HS + 7) / 8;
    const bool xin = (HS % 8 >= 1) && (HS % 8 <= 5);
    const int XBLK = xin ? KBH - 1 : KBH;
    const int KB = l == 0 ? (xin ? KBH : KBH + 1) : 2 * KBH;
    const int n = HS * KB * kWave * 8;
    const int idx = blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= n) return;
    const int j = idx & 7, lane = (idx >> 3) & 63, rk = idx >> 9;
    const int kb = rk % KB, r = rk / KB;
    const int rho = lane & 15, kq = lane >> 4;
    const int unit = 4 * r + (rho >> 2), gate = rho & 3;
    float v = 0.0f;
    if (unit < H) {
        const int grow = gate * H + unit;
        if (l == 0) {
            const int s = 8 * kb + j, u = 4 * s + kq;
            if (kb < KBH && s < HS) {
                if (u < H) v = a.whh[0][grow * H + u];
            } else if (kb == XBLK && j == 5) {
                v = a.wih[0][grow * kIn + kq];
            } else if (kb == XBLK && j == 6 && kq == 0) {
                v = a.wih[0][grow * kIn + 4];
            }
        } else if (kb < KBH) {
            const int u = 4 * (8 * kb + j) + kq;
            if (u < H) v = a.wih[l][grow * H + u];
        } else {
            const int u = 4 * (8 * (kb - KBH) + j) + kq;
            if (u < H) v = a.whh[l][grow * H + u];
        }
    }
    v *= (gate == 2 ? kTwoLog2e : kNegLog2e);
    const _Float16 hi = (_Float16)v;
    const _Float16 lo = (_Float16)(v - (float)hi);
    const size_t frag = (size_t)rk * 2;
    dst[(frag * kWave + lane) * 8 + j] = hi;
    dst[((frag + 1) * kWave + lane) * 8 + j] = lo;
}

// Backward fragments, f16 split: element (tau, kb, split, lane, j) = hi|lo of A'[rho][k] with rho ->
// output slot sigma = 4tau+(rho&3) in lane group qo = rho>>2 (outputs as in pack_bwd_kernel) and
// k = 8*(lane>>4)+j -> gate row (j&3)*H + 4*(2kb+(j>>2)) + (lane>>4).
__global__ void pack_bwd16_kernel(PackArgs a, int l, _Float16 *dst) {
    const int H = a.H, HS = a.HS;
    const int NB = l == 0 ? (HS + 2 + 3) / 4 : (2 * HS + 3) / 4;
    const int KBB = (HS + 1) / 2;
    const int n = NB * KBB * kWave * 8;
    const int idx = blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= n) return;
    const int j = idx & 7, lane = (idx >> 3) & 63, tk = idx >> 9;
    const int kb = tk % KBB, tau = tk / KBB;
    const int rho = lane & 15, kq = lane >> 4;
    const int sigma = 4 * tau + (rho & 3), qo = rho >> 2;
    const int slot = 2 * kb + (j >> 2), gate = j & 3;
    const int unit_k = 4 * slot + kq;
    float v = 0.0f;
    if (slot < HS && unit_k < H) {
        const int grow = gate * H + unit_k;
        if (l == 0) {
            if (sigma < HS) {
                const int u = 4 * sigma + qo;
                if (u < H) v = a.whh[0][grow * H + u];
            } else if (sigma == HS) {
                v = a.wih[0][grow * kIn + qo];
            } else if (sigma == HS + 1 && qo == 0) {
                v = a.wih[0][grow * kIn + 4];
            }
        } else {
            if (sigma < HS) {
                const int u = 4 * sigma + qo;
                if (u < H) v = a.wih[l][grow * H + u];
            } else if (sigma < 2 * HS) {
                const int u = 4 * (sigma - HS) + qo;
                if (u < H) v = a.whh[l][grow * H + u];
            }
        }
    }
    const _Float16 hi = (_Float16)v;
    const _Float16 lo = (_Float16)(v - (float)hi);
    const size_t frag = (size_t)tk * 2;
    dst[(frag * kWave + lane) * 8 + j] = hi;
    dst[((frag + 1) * kWave + lane) * 8 + j] = lo;
}

}  // namespace fcr
