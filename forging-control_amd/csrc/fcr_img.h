// fcr_img.h — one LDS image of a layer's weights that serves BOTH matrix products of the
// recompute-in-backward cell (fcr_bwd.h):
//   forward  gates = W · [x ; h_{t-1}]        A operand = 8 consecutive INPUT columns of one gate row
//   backward [dx ; dh_prev] = Wᵀ · dgates     A operand = 8 consecutive GATE rows of one input column
// A fragment always holds 8 consecutive k per lane, so the two products need the weights contiguous
// along different axes. Storing W once as [gate row][input column] f16 (hi and lo images) and reading
// the backward operand with ds_read_b64_tr_b16 (a hardware 4x16 transpose per 16-lane group) gives
// both from one copy — two copies would not fit in 160 KiB.
//
// Rows: R = 16*slot + 4*grp + gate for gate row (gate, unit 4*slot+grp) — the forward D tile `slot`
// (lane m = R&15) and, for the transposed read, gates 0..3 of one unit on 4 consecutive rows.
// Columns: the layer's input vector in "combined slots" σ (layer >= 1: x slots 0..HS-1, then h_{t-1}
// slots; layer 0: h_{t-1} slots, then window column q at σ = HS and column 4 at σ = HS+1, group 0),
// column = (σ>>3)*32 + grp*8 + (σ&7), i.e. k-block σ>>3, lane group grp, element σ&7 — the forward
// k layout of fwd16_cell, and 4 consecutive σ of one group are 4 consecutive columns (one 8-B unit).
// Layout (no swizzle, no address arithmetic in the kernel): a row holds U 8-B units (U = 32 when the
// layer has more than two k-blocks, else 16); the unit of (k-block kb, lane group q, half h0) is
// q*(U/4) + 2*kb + h0. The 16 rows of a slot's tile are STAGGERED: row m starts at img_row_start(m, U)
// units (33m, +8 from m = 8, for U = 32; rows paired into 32-unit blocks for U = 16), 4-5 % longer than
// packed rows. Every lane's address is then (its own base, img_lane) + (an instruction constant: tile,
// k-block, half, output tile) — the constant is the ds offset, so no per-read VALU — and both the forward
// row reads (ds_read_b64) and the transposed reads are free of LDS bank conflicts. Checked exhaustively
// (addresses, transposed-read semantics, banks) for H = 16, 32, 50 by scripts/img_layout_check.py.
#pragma once
#include "fcr_common.h"
#include "fcr_f16.h"
#include "fcr_pack.h"

namespace fcr {

__host__ __device__ constexpr int img_units(int kb) { return kb > 2 ? 32 : 16; }           // 8-B units per row
__host__ __device__ constexpr int img_tile_units(int U) { return U == 32 ? 536 : 268; }  // one slot's 16 rows
// unit offset of row m (0..15) of a tile: staggered so that rows land on distinct LDS bank groups
__host__ __device__ constexpr int img_row_start(int m, int U) {
    return U == 32 ? 33 * m + (m >= 8 ? 8 : 0)
                   : 33 * (m % 4 + 4 * (m / 8)) + (m >= 8 ? 4 : 0) + 16 * ((m / 4) % 2);
}
// unit of (k-block kb, lane group q, half h0) inside a row
__host__ __device__ constexpr int img_unit(int kb, int q, int h0, int U) { return q * (U / 4) + 2 * kb + h0; }

template <int HS, bool L0>
struct Img {
    static constexpr int NSL = L0 ? HS + 2 : 2 * HS;              // combined input slots
    static constexpr int KB = (NSL + 7) / 8;                       // 32-column k-blocks
    static constexpr int U = img_units(KB);                        // 8-B units per row
    static constexpr int TILE = 8 * img_tile_units(U);             // bytes per slot (16 staggered rows)
    static constexpr int HALF = HS * TILE;                         // hi image bytes; the lo image follows
    static constexpr int BYTES = (2 * HALF + 1023) / 1024 * 1024;  // whole 1 KiB chunks (LDS-DMA refills)
    static constexpr int NB = (NSL + 3) / 4;                       // backward output tiles
    static constexpr int KBB = (HS + 1) / 2;                       // backward k-blocks (2 slots each)
};

inline int img_kb(int HS, int l) { return ((l == 0 ? HS + 2 : 2 * HS) + 7) / 8; }
inline size_t img_bytes(int HS, int l) {
    const int U = img_units(img_kb(HS, l));
    return ((size_t)2 * HS * 8 * img_tile_units(U) + 1023) / 1024 * 1024;
}
// pack_img_kernel threads: one per (image row, logical column)
inline int img_pack_threads(int HS, int l) { return 16 * HS * 4 * img_units(img_kb(HS, l)); }

// One thread per (image row, column): value W[gate*H + unit][input of (σ, grp)], pre-scaled for exp2
// like the forward fragments (the backward divides its dgates by the same per-gate factor). With a
// packed tail (tail_packed, fcr_f16.h) the hi image's last k-block carries, in its padding columns
// σ = 2HS .. 2HS+3, the copies (lo σ0, lo σ1, hi σ0, hi σ1) of its two real slots σ0, σ1, so the
// recompute's row read of that block IS the packed tail fragment; the transposed product's last output
// tile reads rows σ0, σ1, 2HS, 2HS+1 of the hi image — W_hi and W_lo of the two real slots — so its
// hi-image products carry the W_lo·dgate term too (fcr_bwd.h); the lo image keeps zeros there.
__device__ __forceinline__ void pack_img_item(const PackArgs &a, int l, _Float16 *dst, int idx) {
    const int H = a.H, HS = a.HS;
    const int nsl = l == 0 ? HS + 2 : 2 * HS;
    const int kbn = (nsl + 7) / 8;
    const int U = img_units(kbn), TU = img_tile_units(U);
    const int cols = 4 * U, rows = 16 * HS;
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
                    v = a.wih[0][grow * kIn + grp] / a.wsc[grp];   // range guard (fcr_pack.h): exact
                } else if (grp == 0) {   // s == HS + 1
                    v = a.wih[0][grow * kIn + 4] / a.wsc[4];
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
        hi = jt < 4 ? (_Float16)(v - (float)vh) : vh;
        lo = (_Float16)0.0f;
    } else {
        const float v = weight(sg);
        hi = (_Float16)v;
        lo = (_Float16)(v - (float)hi);
    }
    // logical column col = (σ>>3)*32 + grp*8 + (σ&7): k-block σ>>3, group grp, half (σ&7)>>2, element σ&3
    const int u = img_unit(col >> 5, grp, (col >> 2) & 1, U);
    const size_t off = ((size_t)slot * TU + img_row_start(m, U) + u) * 4 + (col & 3);   // in halves
    dst[off] = hi;
    dst[(size_t)HS * TU * 4 + off] = lo;
}
__global__ void pack_img_kernel(PackArgs a, int l, _Float16 *dst) {
    pack_img_item(a, l, dst, blockIdx.x * blockDim.x + threadIdx.x);
}

typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;
typedef _Float16 f16x4 __attribute__((ext_vector_type(4)));

// LDS byte addresses. For an image at LDS byte offset `base`, lane l keeps
//   fb = base + 8*(row_start(m) + q*U/4)      (m = l&15, q = l>>4: forward row reads)
//   tb = base + 8*(row_start(mt) + p*U/4)     (mt = 4*(l>>4) + ((l>>2)&3), p = l&3: transposed reads)
// and a read adds an instruction constant (the ds offset): slot*TILE + 8*(2*kb + h0) for row reads,
// slot*TILE + 8*(2*(tau>>1) + (tau&1)) for transposed ones, + HALF for the lo image.
template <int U>
struct ImgLane {
    uint32_t fb, tb;   // hi image; the lo image is HALF further
};

template <int U>
__device__ __forceinline__ ImgLane<U> img_lane(uint32_t base, int lane) {
    ImgLane<U> L;
    const int m = lane & 15, q = lane >> 4;
    L.fb = base + 8 * (img_row_start(m, U) + q * (U / 4));
    const int mt = 4 * (lane >> 4) + ((lane >> 2) & 3), p = lane & 3;
    L.tb = base + 8 * (img_row_start(mt, U) + p * (U / 4));
    return L;
}

// LDS byte offset of a pointer into the dynamic LDS array (generic -> LDS address space cast)
__device__ __forceinline__ uint32_t lds_offset(const void *p) {
    return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) char *)(p);
}

// volatile: keeps every row read a single ds_read_b64 (base + 16-bit immediate offset) — the
// load/store optimiser would otherwise pair the two adjacent units of a fragment into ds_read2_b64,
// which is serviced in 16-lane groups on 32 banks (2-way conflicts on this layout) at half the rate
__device__ __forceinline__ f16x4 lds_b64_f16(uint32_t addr) {
    return *reinterpret_cast<const volatile __attribute__((address_space(3))) f16x4 *>(
        (__attribute__((address_space(3))) char *)nullptr + addr);
}
__device__ __forceinline__ f16x4 lds_tr_f16(uint32_t addr) {
    return __builtin_bit_cast(f16x4, __builtin_amdgcn_ds_read_tr16_b64_v4i16(
                                         (lds_s16x4 *)((__attribute__((address_space(3))) char *)nullptr + addr)));
}

}  // namespace fcr
