// fcr_img.h — one LDS image of a layer's weights that serves BOTH matrix products of the
// recompute-in-backward cell (fcr_bwd4.h):
//   forward  gates = W · [x ; h_{t-1}]        A operand = 8 consecutive INPUT columns of one gate row
//   backward [dx ; dh_prev] = Wᵀ · dgates     A operand = 8 consecutive GATE rows of one input column
// A fragment always holds 8 consecutive k per lane, so the two products need the weights contiguous
// along different axes. Storing W once as [gate row][input column] f16 (hi and lo images) and reading
// the backward operand with ds_read_b64_tr_b16 (a hardware 4x16 transpose per 16-lane group) gives
// both from one copy — two copies would not fit next to the resident layer-0 image in 160 KiB.
//
// Rows: R = 16*slot + 4*grp + gate for gate row (gate, unit 4*slot+grp) — the forward D tile `slot`
// (lane m = R&15) and, for the transposed read, gates 0..3 of one unit on 4 consecutive rows.
// Columns: the layer's input vector in "combined slots" σ (layer >= 1: x slots 0..HS-1, then h_{t-1}
// slots; layer 0: h_{t-1} slots, then window column q at σ = HS and column 4 at σ = HS+1, group 0),
// column = (σ>>3)*32 + grp*8 + (σ&7), i.e. k-block σ>>3, lane group grp, element σ&7 — the forward
// k layout of fwd16_cell, and 4 consecutive σ of one group are 4 consecutive columns (one 8-B unit).
// Row bytes RB = 64 * k-blocks, at least 128. Swizzle: the 8-B unit w of row R is stored at unit
// w ^ swz(R&15); swz only flips unit-index bits that the instruction (k-block, half, output tile)
// selects, so every lane's address is (its own base) XOR (an instruction constant), and both the
// forward row reads (ds_read_b64) and the transposed reads are free of LDS bank conflicts — checked
// exhaustively for H = 16, 32, 50 by scripts/img_swizzle_check.py.
#pragma once
#include "fcr_common.h"
#include "fcr_f16.h"
#include "fcr_pack.h"

namespace fcr {

template <int HS, bool L0>
struct Img {
    static constexpr int NSL = L0 ? HS + 2 : 2 * HS;              // combined input slots
    static constexpr int KB = (NSL + 7) / 8;                       // 32-column k-blocks
    static constexpr int RB = KB * 64 < 128 ? 128 : KB * 64;       // row bytes
    static constexpr int ROWS = 16 * HS;
    static constexpr int BYTES = 2 * ROWS * RB;                    // hi image, then lo image
    static constexpr int NB = (NSL + 3) / 4;                       // backward output tiles
    static constexpr int KBB = (HS + 1) / 2;                       // backward k-blocks (2 slots each)
};

// unit-index XOR of row position m (= R & 15) for row bytes RB (see the header comment)
__host__ __device__ constexpr int img_swz(int m, int RB) {
    return RB == 256 ? ((m & 1) | ((m >> 1) & 1) << 3 | ((m >> 2) & 1) << 4 | ((m >> 3) & 1) << 2)
                     : (((m >> 1) & 1) | ((m >> 2) & 1) << 3 | ((m >> 3) & 1) << 2);
}

inline size_t img_bytes(int HS, int l) {
    const int nsl = l == 0 ? HS + 2 : 2 * HS;
    const int kb = (nsl + 7) / 8;
    const int rb = kb * 64 < 128 ? 128 : kb * 64;
    return (size_t)2 * 16 * HS * rb;
}

// One thread per (image row, column): value W[gate*H + unit][input of (σ, grp)], pre-scaled for exp2
// like the forward fragments (the backward divides its dgates by the same per-gate factor). With a
// packed tail (tail_packed, fcr_f16.h) the hi image's last k-block carries, in its padding columns
// σ = 2HS .. 2HS+3, the copies (hi σ0, hi σ1, lo σ0, lo σ1) of its two real slots, so the recompute's
// row read of that block IS the packed tail fragment; the transposed product never reads those
// columns as anything but unused output rows, and the lo image keeps zeros there.
__global__ void pack_img_kernel(PackArgs a, int l, _Float16 *dst) {
    const int H = a.H, HS = a.HS;
    const int nsl = l == 0 ? HS + 2 : 2 * HS;
    const int kbn = (nsl + 7) / 8;
    const int RB = kbn * 64 < 128 ? 128 : kbn * 64;
    const int cols = RB / 2, rows = 16 * HS;
    const int idx = blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= rows * cols) return;
    const int col = idx % cols, R = idx / cols;
    const int slot = R >> 4, m = R & 15;
    const int unit = 4 * slot + (m >> 2), gate = m & 3;
    const int sg = (col >> 5) * 8 + (col & 7), grp = (col >> 3) & 3;   // combined slot, lane group
    auto weight = [&](int s) {
        float v = 0.0f;
        if (unit < H && s < nsl) {
            const int grow = gate * H + unit;
            if (l == 0) {
                if (s < HS) {
                    const int u = 4 * s + grp;
                    if (u < H) v = a.whh[0][grow * H + u];
                } else if (s == HS) {
                    v = a.wih[0][grow * kIn + grp];
                } else if (grp == 0) {   // s == HS + 1
                    v = a.wih[0][grow * kIn + 4];
                }
            } else if (s < HS) {
                const int u = 4 * s + grp;
                if (u < H) v = a.wih[l][grow * H + u];
            } else {
                const int u = 4 * (s - HS) + grp;
                if (u < H) v = a.whh[l][grow * H + u];
            }
        }
        return v * (gate == 2 ? kTwoLog2e : kNegLog2e);
    };
    _Float16 hi, lo;
    const int jt = sg - 8 * (kbn - 1);   // position inside the last k-block
    if (l > 0 && tail_packed(HS) && jt >= 2 && jt < 6) {
        const float v = weight(8 * (kbn - 1) + (jt & 1));
        const _Float16 vh = (_Float16)v;
        hi = jt < 4 ? vh : (_Float16)(v - (float)vh);
        lo = (_Float16)0.0f;
    } else {
        const float v = weight(sg);
        hi = (_Float16)v;
        lo = (_Float16)(v - (float)hi);
    }
    const int w = (col >> 2) ^ img_swz(m, RB);
    const size_t off = (size_t)R * (RB / 2) + w * 4 + (col & 3);   // in halves
    dst[off] = hi;
    dst[(size_t)rows * (RB / 2) + off] = lo;
}

typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;
typedef _Float16 f16x4 __attribute__((ext_vector_type(4)));

// LDS byte addresses. For an image at LDS byte offset `base` (a multiple of RB), lane l keeps
//   fb = base + m*RB + 8*((2q) ^ swz(m))           (m = l&15, q = l>>4: forward row reads)
//   tb = base + mt*RB + 8*((2p) ^ swz(mt))         (mt = 4*(l>>4) + ((l>>2)&3), p = l&3: transposed)
// The unit index of a read is (lane bits) | (instruction bits) with disjoint bit sets, so its address
// is fb ^ (8 * instruction bits) [+ 16*RB*slot as the ds offset]: one v_xor per distinct instruction
// part, shared by every slot; instruction bits = 8*kb + h0 (forward), 8*(tau>>1) + (tau&1) (transposed).
template <int RB>
struct ImgLane {
    uint32_t fb, tb;   // hi image; the lo image is ROWS*RB further
};

template <int RB>
__device__ __forceinline__ ImgLane<RB> img_lane(uint32_t base, int lane) {
    ImgLane<RB> L;
    const int m = lane & 15, q = lane >> 4;
    L.fb = base + m * RB + 8 * ((2 * q) ^ img_swz(m, RB));
    const int mt = 4 * (lane >> 4) + ((lane >> 2) & 3), p = lane & 3;
    L.tb = base + mt * RB + 8 * ((2 * p) ^ img_swz(mt, RB));
    return L;
}

// LDS byte offset of a pointer into the dynamic LDS array (generic -> LDS address space cast)
__device__ __forceinline__ uint32_t lds_offset(const void *p) {
    return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) char *)(p);
}

__device__ __forceinline__ f16x4 lds_b64_f16(uint32_t addr) {
    return *reinterpret_cast<const __attribute__((address_space(3))) f16x4 *>(
        (__attribute__((address_space(3))) char *)nullptr + addr);
}
__device__ __forceinline__ f16x4 lds_tr_f16(uint32_t addr) {
    return __builtin_bit_cast(f16x4, __builtin_amdgcn_ds_read_tr16_b64_v4i16(
                                         (lds_s16x4 *)((__attribute__((address_space(3))) char *)nullptr + addr)));
}

}  // namespace fcr
