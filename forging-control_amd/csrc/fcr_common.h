// fcr_common.h — shared constants, device helpers and kernel argument blocks.
//
// Lane mapping: one wave = 16 trajectories (MFMA columns); hidden unit u = 4*slot + q lives in lane
// group q = lane>>4, register slot `slot` (HS = ceil(H/4) slots). Operand geometry: fcr_f16.h (forward
// fragments) and fcr_img.h (the backward's dual-use weight image).
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

namespace fcr {

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x2 __attribute__((ext_vector_type(2)));

constexpr int kWave = 64;
constexpr int kTile = 16;        // trajectories per wave (MFMA 16x16x4 column count)
constexpr int kL = 10;           // window rows (Functions.py:1434 hard-codes 1:10)
constexpr int kLayers = 3;       // UL/Main.py:147 (width_dim passed as layer_dim)
constexpr int kIn = 5;           // [y_dot, p1, p2, z, u]
constexpr int kOut = 4;          // [y_dot, p1, p2, z]
constexpr int kCtrlIn = 3;       // [y_dot, z, ref]
constexpr int kMS = 13;          // controller hidden slots (units 4m+q), hidden <= 52
constexpr int kFnpStride = 8;    // floats per (m, q) controller record: W0 W1 W2 b wout 0 0 0
constexpr int kFwdWaves = 8;     // waves per forward workgroup (2 per SIMD)
constexpr int kBwdWaves = 8;     // waves per backward workgroup (2 per SIMD)
constexpr float kP1Max = 2.122366f;  // Functions.py:1411 (32e6 / p1 max_abs_)
constexpr float kP2Max = 1.036233f;  // Functions.py:1411 (32e6 / p2 max_abs_)

template <int HS>
struct Geo {
    static constexpr int HQ = (HS + 3) / 4;   // registers (f32x4) per unit-slot vector
    static constexpr int QC = HS * 16;        // 16-B units per cell record of a sequence slab (64 lanes x 4·HS B)
};

struct Packed {                    // device pointers into the workspace
    const float *fa[3];            // forward fragments (fcr_f16.h) [r][kb][hi|lo][64][8 halves]
    const float *img[3];           // backward weight images (fcr_img.h) [hi|lo][row][RB bytes]
    const float *fcp;              // fc.weight in lane layout [o][slot][q]
    const float *fcb;              // fc.bias [4]
    const float *fnp;              // controller records [m][q][8]
    const float *wsc;              // window-column scales 2^-s_c [8] (range_final_kernel, fcr_pack.h)
};

// Sequence slabs (per wave, each address written once per call):
//   hseq, cseq [wave][j][layer][t][record]     h_t and c_t of every cell (compact records: store_quads)
//   xw         [wave][j][t][64]               layer-0 window row t of window j (col q, col 4)
//   dseq       [wave][j][2][t][record]         backward dx of layers 2, 1 (inputs of layers 1, 0)
//   dxrow      [wave][j][t][64]               backward window-row gradients (col q, col 4)
struct FwdArgs {
    int B, N;
    float alpha;
    const float *X, *u0, *states, *noise;
    float *cost, *command, *error, *prediction, *xhat_user, *xhat_ws, *loss_part;
    f32x4 *hseq;     // layers 0, 1 always (the next phase's input); layer 2 with `keep`
    f32x4 *cseq;     // with `keep` (null otherwise)
    f32x2 *xw;       // with `keep`
    unsigned long long *stamp;   // FCR_STAMP diagnostic builds only
    Packed p;
};

struct BwdArgs {
    int B, N, hidden;
    float alpha;
    const float *X, *states, *prediction, *xhat, *dloss;
    const f32x4 *hseq, *cseq;
    const f32x2 *xw;
    f32x4 *dseq;
    f32x2 *dxrow;
    float *g_u0;
    float *dv;       // [B][N] d loss / d (controller pre-Hardtanh output) of the call fed by step j
    unsigned long long *stamp;   // FCR_STAMP diagnostic builds only: per-wave cycle sums
    Packed p;
};

// ------------------------------------------------------------------------------------------------
// device helpers
// ------------------------------------------------------------------------------------------------
__device__ __forceinline__ f32x4 mfma(float a, float b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}
// logistic and tanh on v_exp_f32 / v_rcp_f32 (saturate correctly at +-inf)
__device__ __forceinline__ float sigm(float x) {
    return __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(x * -1.4426950408889634f));
}
__device__ __forceinline__ float tanh_f(float x) {
    return 1.0f - 2.0f * __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(x * 2.8853900817779268f));
}
// the same on an argument that is already scaled: sigm_pre(-x log2e) = sigm(x), tanh_pre(2x log2e) = tanh(x)
__device__ __forceinline__ float sigm_pre(float a) { return __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(a)); }
__device__ __forceinline__ float tanh_pre(float a) {
    return 1.0f - 2.0f * __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(a));
}
constexpr float kNegLog2e = -1.4426950408889634f;   // gate-row scales folded into the forward fragments
constexpr float kTwoLog2e = 2.8853900817779268f;
__device__ __forceinline__ float relu(float x) { return x > 0.0f ? x : 0.0f; }
__device__ __forceinline__ float sq(float x) { return x * x; }
__device__ __forceinline__ float hardtanh(float v) { return fminf(fmaxf(v, -1.0f), 1.0f); }
__device__ __forceinline__ float sel4(int q, float a, float b, float c, float d) {
    return q == 0 ? a : (q == 1 ? b : (q == 2 ? c : d));
}
// Sum / max over the 4 lane groups that share one trajectory (lanes l, l^16, l^32, l^48). (gfx950's
// v_permlane16/32_swap form measured +0.1..0.6 % in the backward, round 3d: the swaps' hazard s_nops eat the LDS
// round trip of the two ds_bpermutes.)
template <bool MAX>
__device__ __forceinline__ float reduce_q(float v) {
    auto op = [](float a, float b) { return MAX ? fmaxf(a, b) : a + b; };
    v = op(v, __shfl_xor(v, 16));
    return op(v, __shfl_xor(v, 32));
}
__device__ __forceinline__ float xor_sum_q(float v) { return reduce_q<false>(v); }
__device__ __forceinline__ float max_q(float v) { return reduce_q<true>(v); }
__device__ __forceinline__ void sched_fence() { __builtin_amdgcn_sched_barrier(0); }

// An LDS pointer the compiler cannot see through: stops it from hoisting loop-invariant LDS reads
// (e.g. the 65 controller parameters) out of the window loop into registers it does not have.
template <typename T>
__device__ __forceinline__ T *opaque(T *p) {
    int z = 0;
    asm volatile("" : "+s"(z));
    return p + z;
}

// ds_read_b128 of fragment quad `idx` (units of 16 B per lane-slot, i.e. element idx*64+lane of an
// f32x4 array). ds_* immediate offsets are 16-bit, so fragment blocks beyond 64 KB would each need a
// materialised address VGPR (which the compiler then hoists out of every loop and spills). Two
// bases, 48 KB apart, keep every compile-time offset inside the immediate field.
__device__ __forceinline__ f32x4 lds_quad(const float *lw, int idx, int lane) {
    constexpr int kSplit = 48 * 1024;
    const int byte = idx * kWave * 16;
    const char *lo = reinterpret_cast<const char *>(lw) + lane * 16;
    if (byte < kSplit) return *reinterpret_cast<const f32x4 *>(lo + byte);
    const char *hi = lo + kSplit;
    return *reinterpret_cast<const f32x4 *>(hi + (byte - kSplit));
}

// Raw buffer loads through a wave-uniform descriptor (base and size from SGPR values only, so no
// waterfall loop): the per-lane part is a 32-bit voffset, the rest an SGPR soffset.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t wave_rsrc(const void *base, size_t bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void *>(base), (short)0, (int)(uint32_t)bytes, 0x00020000);
}
__device__ __forceinline__ f32x4 buf_ld4(__amdgpu_buffer_rsrc_t r, uint32_t voff, uint32_t soff) {
    return __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(r, (int)voff, (int)soff, 0));
}
__device__ __forceinline__ f32x2 buf_ld2(__amdgpu_buffer_rsrc_t r, uint32_t voff, uint32_t soff) {
    return __builtin_bit_cast(f32x2, __builtin_amdgcn_raw_buffer_load_b64(r, (int)voff, (int)soff, 0));
}
// Quad k of a unit-slot vector with only its first n (1..4) slots loaded: a padding lane of a partial
// last quad that is loaded but never read is a register the compiler reuses at once — i.e. waits for.
template <int n>
__device__ __forceinline__ f32x4 buf_ldq(__amdgpu_buffer_rsrc_t r, uint32_t voff, uint32_t soff) {
    f32x4 q = {0.0f, 0.0f, 0.0f, 0.0f};
    if (n == 4) {
        q = buf_ld4(r, voff, soff);
    } else if (n == 3) {
        // the whole vector is cast: this compiler's __builtin_bit_cast of an ext_vector ELEMENT (v[1]) reads
        // element 0 (round 4: the f16 mode's 7-word h records came back as (w4, w4, w4) — DESIGN.md §2)
        typedef unsigned int u32x3 __attribute__((ext_vector_type(3)));
        typedef float f32x3 __attribute__((ext_vector_type(3)));
        const f32x3 v = __builtin_bit_cast(f32x3, __builtin_amdgcn_raw_buffer_load_b96(r, (int)voff, (int)soff, 0));
        q[0] = v[0];
        q[1] = v[1];
        q[2] = v[2];
    } else if (n == 2) {
        const f32x2 v = buf_ld2(r, voff, soff);
        q[0] = v[0];
        q[1] = v[1];
    } else {
        q[0] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, (int)voff, (int)soff, 0));
    }
    return q;
}
template <int HS, int k>
constexpr int quad_n() { return HS - 4 * k >= 4 ? 4 : HS - 4 * k; }
// per-lane byte offset and cell-relative byte offset of record quad k (the tail is packed, store_quads)
template <int HS, int k>
__device__ __forceinline__ uint32_t quad_voff(int lane) { return (uint32_t)lane * (quad_n<HS, k>() == 4 ? 16u : 4u * quad_n<HS, k>()); }
template <int HS, int k>
constexpr uint32_t quad_soff() { return (uint32_t)k * kWave * 16; }

__device__ __forceinline__ void buf_st2(__amdgpu_buffer_rsrc_t r, uint32_t voff, uint32_t soff, f32x2 v) {
    __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(__attribute__((ext_vector_type(2))) unsigned int, v), r,
                                          (int)voff, (int)soff, 0);
}

__device__ __forceinline__ void buf_st4(__amdgpu_buffer_rsrc_t r, uint32_t voff, uint32_t soff, f32x4 v) {
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(__attribute__((ext_vector_type(4))) unsigned int, v), r,
                                           (int)voff, (int)soff, 0);
}
__device__ __forceinline__ void buf_st1(__amdgpu_buffer_rsrc_t r, uint32_t voff, uint32_t soff, float v) {
    __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned int, v), r, (int)voff, (int)soff, 0);
}

// Copy a fragment block (global, L2-resident) into LDS; the caller brackets it with barriers.
__device__ __forceinline__ void lds_copy(float *lw, const float *__restrict__ src, int nfloats) {
    const float4 *s4 = reinterpret_cast<const float4 *>(src);
    float4 *d4 = reinterpret_cast<float4 *>(lw);
    for (int i = threadIdx.x; i < nfloats / 4; i += blockDim.x) d4[i] = s4[i];
}
// Refill the per-phase region. Every wave of the workgroup calls this at the same program point.
// Refill the per-phase LDS region with LDS-DMA (global_load_lds_dwordx4: each wave instruction moves
// one 1 KiB chunk straight into LDS, no VGPRs): after the barrier that retires the old image, every
// wave issues its chunks back to back; the barrier after them waits for the DMA (vmcnt) and publishes.
template <int NBYTES, int NWAVES>
__device__ __forceinline__ void lds_fill(float *lw, const float *__restrict__ src) {
    static_assert(NBYTES % 1024 == 0, "image must be whole 1 KiB chunks");
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
    __syncthreads();
    for (int c = wv; c < NBYTES / 1024; c += NWAVES)
        __builtin_amdgcn_global_load_lds(
            (const __attribute__((address_space(1))) void *)((const char *)src + c * 1024 + lane * 16),
            (__attribute__((address_space(3))) void *)((__attribute__((address_space(3))) char *)lw + c * 1024), 16,
            0, 0);
    __syncthreads();
}

// Unit-slot vectors <-> a compact cell record: HS/4 full 16-B quads [k][64 lanes] (slots 4k..4k+3),
// then the HS%4 tail slots packed per lane [64 lanes][HS%4] — 4·HS bytes per lane, no padding slots
// (a padded last quad cost 3/16 of the slab traffic at HS = 13, and the HBM traffic sets the clock
// the chip holds). A cell is Geo<HS>::QC quads; ceil(HS/4) memory instructions per cell.
template <int HS>
__device__ __forceinline__ void store_quads(f32x4 *dst, const float (&v)[HS], int lane) {
    constexpr int FQ = HS / 4, TS = HS % 4;
#pragma unroll
    for (int k = 0; k < FQ; ++k) dst[k * kWave + lane] = f32x4{v[4 * k], v[4 * k + 1], v[4 * k + 2], v[4 * k + 3]};
    if constexpr (TS > 0) {
        float *t = reinterpret_cast<float *>(dst + FQ * kWave) + lane * TS;
        if constexpr (TS == 1) {
            t[0] = v[4 * FQ];
        } else if constexpr (TS == 2) {
            *reinterpret_cast<f32x2 *>(t) = f32x2{v[4 * FQ], v[4 * FQ + 1]};
        } else {
            typedef float f32x3 __attribute__((ext_vector_type(3)));
            *reinterpret_cast<f32x3 *>(t) = f32x3{v[4 * FQ], v[4 * FQ + 1], v[4 * FQ + 2]};
        }
    }
}
template <int HS>
__device__ __forceinline__ void load_quads(float (&v)[HS], const f32x4 *src, int lane) {
    constexpr int FQ = HS / 4, TS = HS % 4;
#pragma unroll
    for (int k = 0; k < FQ; ++k) {
        const f32x4 q = src[k * kWave + lane];
#pragma unroll
        for (int e = 0; e < 4; ++e) v[4 * k + e] = q[e];
    }
    const float *t = reinterpret_cast<const float *>(src + FQ * kWave) + lane * TS;
#pragma unroll
    for (int e = 0; e < TS; ++e) v[4 * FQ + e] = t[e];
}

// store_quads / load_quads through a wave-uniform buffer descriptor (the layout above): the lane part is
// quad_voff, the cell's offset an SGPR soffset — no per-access 64-bit address arithmetic
template <int HS, int k = 0>
__device__ __forceinline__ void buf_store_quads(__amdgpu_buffer_rsrc_t r, uint32_t off, const float (&v)[HS], int lane) {
    if constexpr (k < Geo<HS>::HQ) {
        constexpr int n = quad_n<HS, k>();
        const uint32_t vo = quad_voff<HS, k>(lane), so = off + quad_soff<HS, k>();
        if constexpr (n == 4) {
            buf_st4(r, vo, so, f32x4{v[4 * k], v[4 * k + 1], v[4 * k + 2], v[4 * k + 3]});
        } else if constexpr (n == 3) {
            typedef unsigned int u32x3 __attribute__((ext_vector_type(3)));
            __builtin_amdgcn_raw_buffer_store_b96(u32x3{__builtin_bit_cast(unsigned, v[4 * k]), __builtin_bit_cast(unsigned, v[4 * k + 1]),
                                                        __builtin_bit_cast(unsigned, v[4 * k + 2])},
                                                  r, (int)vo, (int)so, 0);
        } else if constexpr (n == 2) {
            buf_st2(r, vo, so, f32x2{v[4 * k], v[4 * k + 1]});
        } else {
            buf_st1(r, vo, so, v[4 * k]);
        }
        buf_store_quads<HS, k + 1>(r, off, v, lane);
    }
}
// Words of a cell's h record: the fp32-accurate split record holds [hi | lo] (HS words per lane); the f16 mode's
// (LP) only the hi halves, ceil(HS / 2) words — its consumers never read a lo half (fcr_f16.h split_rec).
template <int HS, bool LP>
constexpr int rec_words() { return LP ? (HS + 1) / 2 : HS; }
// Words of a d record (din: the input gradient a layer hands to the one below at the same t): fp32 per slot; the f16
// mode's holds f16 halves scaled by a per-trajectory power of two whose exponent rides in half HS (fcr_bwd.h
// din_store_lp / the DIN read in bwd_cell) — half the bytes of the backward's largest slab stream.
template <int HS, bool LP>
constexpr int din_words() { return LP ? HS / 2 + 1 : HS; }
// The first RW words of a record array, stored in the compact layout of an RW-word record (a reader loads them
// with ld_rec<RW>): the cell's space is the HS-word layout's, so offsets are unchanged and only the bytes shrink.
template <int RW, int HS, int k = 0>
__device__ __forceinline__ void buf_store_rec(__amdgpu_buffer_rsrc_t r, uint32_t off, const float (&v)[HS], int lane) {
    static_assert(RW <= HS, "record words");
    if constexpr (k < Geo<RW>::HQ) {
        constexpr int n = quad_n<RW, k>();
        const uint32_t vo = quad_voff<RW, k>(lane), so = off + quad_soff<RW, k>();
        if constexpr (n == 4) {
            buf_st4(r, vo, so, f32x4{v[4 * k], v[4 * k + 1], v[4 * k + 2], v[4 * k + 3]});
        } else if constexpr (n == 3) {
            typedef unsigned int u32x3 __attribute__((ext_vector_type(3)));
            __builtin_amdgcn_raw_buffer_store_b96(u32x3{__builtin_bit_cast(unsigned, v[4 * k]), __builtin_bit_cast(unsigned, v[4 * k + 1]),
                                                        __builtin_bit_cast(unsigned, v[4 * k + 2])},
                                                  r, (int)vo, (int)so, 0);
        } else if constexpr (n == 2) {
            buf_st2(r, vo, so, f32x2{v[4 * k], v[4 * k + 1]});
        } else {
            buf_st1(r, vo, so, v[4 * k]);
        }
        buf_store_rec<RW, HS, k + 1>(r, off, v, lane);
    }
}
// A cell's c record: fp32 per slot; in the f16 mode (LP) f16 halves (slot 2w | 2w + 1 in word w, rec_words words) —
// |c_t| <= t + 1 (c_t = f c_{t-1} + i g from zero), so no scaling: the backward's c_{t-1} and its rebuilt c_t carry
// 2^-12 relative, as the f16 mode's h operands do.
template <int HS, bool LP>
__device__ __forceinline__ void c_store(__amdgpu_buffer_rsrc_t r, uint32_t off, const float (&v)[HS], int lane) {
    if constexpr (LP) {
        typedef _Float16 f16x2 __attribute__((ext_vector_type(2)));
        constexpr int CW = rec_words<HS, true>();
        float w[HS];
#pragma unroll
        for (int d = 0; d < CW; ++d) {
            f16x2 p;
            p[0] = (_Float16)v[2 * d];
            p[1] = 2 * d + 1 < HS ? (_Float16)v[2 * d + 1 < HS ? 2 * d + 1 : 0] : (_Float16)0.0f;
            w[d] = __builtin_bit_cast(float, p);
        }
        buf_store_rec<CW>(r, off, w, lane);
    } else {
        buf_store_quads<HS>(r, off, v, lane);
    }
}
template <int HS, int k = 0>
__device__ __forceinline__ void buf_load_quads(float (&v)[HS], __amdgpu_buffer_rsrc_t r, uint32_t off, int lane) {
    if constexpr (k < Geo<HS>::HQ) {
        constexpr int n = quad_n<HS, k>();
        const f32x4 q = buf_ldq<n>(r, quad_voff<HS, k>(lane), off + quad_soff<HS, k>());
#pragma unroll
        for (int e = 0; e < n; ++e) v[4 * k + e] = q[e];
        buf_load_quads<HS, k + 1>(v, r, off, lane);
    }
}

// Controller pre-activation (FNNModel.forward, Functions.py:261-289): lane group q evaluates hidden
// units 4m+q; returns the pre-Hardtanh output (identical arithmetic in forward and backward).
__device__ __forceinline__ float fnn_pre(const float *__restrict__ fnp, int q, float a, float b,
                                         float r, float (&z)[kMS]) {
    float part = 0.0f;
#pragma unroll
    for (int m = 0; m < kMS; ++m) {
        const float *p = fnp + (m * 4 + q) * kFnpStride;
        const float zz = p[0] * a + p[1] * b + p[2] * r + p[3];
        z[m] = zz;
        part += p[4] * relu(zz);
    }
    return xor_sum_q(part);
}

// Last store of a controller parameter-gradient kernel (ctrl_grad_kernel, fnn_bwd_kernel): the block's
// partial [block][k][p] for grad_reduce_kernel, or — launched as one block, with the outputs given — the
// gradient itself, as 0 + s: what grad_reduce_kernel's fixed-order sum makes of a single partial, bit for
// bit, one launch fewer (small batches are launch-bound)
__device__ __forceinline__ void grad_out5(float *part, int hidden, int k, int p, float s, float *gwi, float *gbi,
                                          float *gwo) {
    if (gwi) {
        const float v = 0.0f + s;
        if (p < 3) gwi[k * kCtrlIn + p] = v;
        else if (p == 3) gbi[k] = v;
        else gwo[k] = v;
    } else {
        part[((size_t)blockIdx.x * hidden + k) * 5 + p] = s;
    }
}

}  // namespace fcr
