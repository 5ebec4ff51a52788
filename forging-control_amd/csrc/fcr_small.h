// fcr_small.h — small-batch rollout kernels (the reference trains at B = 15, UL/Main.py:84,297).
//
// The fused kernels (fcr_fwd.h, fcr_bwd.h) give each 16-trajectory group ONE wave that runs every
// cell of the rollout itself: below ~16 k trajectories (one wave per SIMD) the step time is that
// wave's sequential latency, ~3 ms whatever B is. Here a group gets a workgroup of NQ = ceil(HS/4)
// waves, one per SIMD, and wave w owns the unit slots of record quad w (slots 4w .. 4w+3):
//   forward  — wave w computes the gate tiles of its slots (fwd16_cell over that tile range), keeps
//              their c, and the cell's h_t is exchanged through LDS (one barrier per cell) so every
//              wave has the whole h_{t-1} for the next cell's B operand;
//   backward — wave w recomputes its tiles, forms the dgates of its slots and the partial transposed
//              product W[its gate rows]ᵀ·dgates for all output tiles (sb_atile, sb_slot, sb_ttile: bwd_cell's
//              arithmetic); the partials are summed through LDS in a fixed order (two barriers per cell),
//              and each wave takes the dx / dh_prev of its own slots.
// Slab layout (hseq, cseq, xw, dseq) is that of the fused kernels — each wave writes its own quads
// of a record, and a record is read whole only across a phase barrier — so a split forward and a fused
// backward (or the reverse) are interchangeable; the backward's window-row gradients go to a per-wave
// copy of dxrow (every wave needs them at the window head), so nothing global is handed between waves
// inside a phase. Results equal the fused kernels' up to the fp32 order of the partial sums.
#pragma once
#include "fcr_bwd.h"
#include "fcr_fwd.h"

namespace fcr {

// Cross-workgroup hand-off of the layer-pipelined kernels (fcr_pipe.h), the R1 form of cdna_hip_programming.md Guideline 16
// (MI355X_MICROARCH.md § visibility, table row 1): every handed-off byte is stored write-through (sc1) by the wave that
// owns it; every storing wave drains its stores (s_waitcnt vmcnt(0)) before a workgroup barrier, after which ONE lane
// raises the workgroup's progress counter (an sc1 store); a consumer polls that one word relaxed and reads the payload
// with sc1 loads only, so no release or acquire fence (an L2 write-back / L1 invalidate, 1.7-6.5 us each) is needed.
// Polls are bounded (kPipeSpin, ~0.3 s): a partner that never arrives cannot hang the kernel — the first wait that gives
// up raises the group's abort word, after which every wait of the group returns at once, so the launch drains in about
// one bound (its outputs are then wrong, which the parity tests see).
constexpr int kPipeFlags = 32;     // words per group (128 B): progress counters, the abort word last
constexpr int kPipeAbort = kPipeFlags - 1;
constexpr int kPipeSpin = 1 << 20;
constexpr int kSc1 = 16;           // aux cache bits of a raw buffer access: sc1 (write-through store / L1-bypassing load)
__device__ __forceinline__ void pipe_drain() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }
__device__ __forceinline__ void pipe_signal(unsigned *f, unsigned v) {   // after the barrier that follows every drain
    if (threadIdx.x == 0) __hip_atomic_store(f, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// a producer's progress counter as it stands (no wait): prefetches take what is published and leave the rest
__device__ __forceinline__ unsigned pipe_count(const unsigned *f) {
    return __builtin_amdgcn_readfirstlane(__hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
}
// a wait of this launch timed out (its partner workgroup was not resident): the outputs are then poisoned with NaN
__device__ __forceinline__ bool pipe_aborted(const unsigned *blk) {
    return __builtin_amdgcn_readfirstlane(__hip_atomic_load(blk + kPipeAbort, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) != 0u;
}
__device__ __forceinline__ void pipe_wait(unsigned *blk, const unsigned *f, unsigned need) {
    for (int s = 0;; ++s) {
        if (__builtin_amdgcn_readfirstlane(__hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) >= need) break;
        if (__builtin_amdgcn_readfirstlane(__hip_atomic_load(blk + kPipeAbort, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)))
            break;
        if (s == kPipeSpin) {
            if ((threadIdx.x & 63) == 0) __hip_atomic_store(blk + kPipeAbort, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            break;
        }
        __builtin_amdgcn_s_sleep(1);
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");   // no instruction: keeps the payload loads below the poll
}
// sc1 record accesses in the compact record layout (store_quads): quad k of the record, or all of it
template <int HS, int k>
__device__ __forceinline__ void st_quad_sc1(__amdgpu_buffer_rsrc_t r, uint32_t off, const float (&v)[HS], int lane) {
    constexpr int n = quad_n<HS, k>();
    const uint32_t vo = quad_voff<HS, k>(lane), so = off + quad_soff<HS, k>();
    typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
    typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
    if constexpr (n == 4) {
        __builtin_amdgcn_raw_buffer_store_b128(u32x4{__builtin_bit_cast(unsigned, v[4 * k]), __builtin_bit_cast(unsigned, v[4 * k + 1]),
                                                     __builtin_bit_cast(unsigned, v[4 * k + 2]), __builtin_bit_cast(unsigned, v[4 * k + 3])},
                                               r, (int)vo, (int)so, kSc1);
    } else if constexpr (n == 2) {
        __builtin_amdgcn_raw_buffer_store_b64(u32x2{__builtin_bit_cast(unsigned, v[4 * k]), __builtin_bit_cast(unsigned, v[4 * k + 1])},
                                              r, (int)vo, (int)so, kSc1);
    } else {
        static_assert(n == 1, "the pipelined tiers: HS = 8, 13 (tail of 0 or 1 slot)");
        __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, v[4 * k]), r, (int)vo, (int)so, kSc1);
    }
}
template <int HS, int k = 0>
__device__ __forceinline__ void ld_rec_sc1(f32x4 (&dst)[Geo<HS>::HQ], __amdgpu_buffer_rsrc_t r, uint32_t off, int lane) {
    if constexpr (k < Geo<HS>::HQ) {
        constexpr int n = quad_n<HS, k>();
        const uint32_t vo = quad_voff<HS, k>(lane), so = off + quad_soff<HS, k>();
        if constexpr (n == 4) {
            dst[k] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(r, (int)vo, (int)so, kSc1));
        } else {
            static_assert(n == 1, "the pipelined tiers: HS = 8, 13 (tail of 0 or 1 slot)");
            f32x4 q = {0.0f, 0.0f, 0.0f, 0.0f};
            q[0] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, (int)vo, (int)so, kSc1));
            dst[k] = q;
        }
        ld_rec_sc1<HS, k + 1>(dst, r, off, lane);
    }
}
template <int HS, int k>
__device__ __forceinline__ void ld_quad_sc1(f32x4 (&dst)[Geo<HS>::HQ], __amdgpu_buffer_rsrc_t r, uint32_t off, int lane) {
    constexpr int n = quad_n<HS, k>();
    const uint32_t vo = quad_voff<HS, k>(lane), so = off + quad_soff<HS, k>();
    if constexpr (n == 4) {
        dst[k] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(r, (int)vo, (int)so, kSc1));
    } else {
        static_assert(n == 1, "the pipelined tiers: HS = 8, 13 (tail of 0 or 1 slot)");
        f32x4 q = {0.0f, 0.0f, 0.0f, 0.0f};
        q[0] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, (int)vo, (int)so, kSc1));
        dst[k] = q;
    }
}
__device__ __forceinline__ void buf_st2_sc1(__amdgpu_buffer_rsrc_t r, uint32_t voff, uint32_t soff, f32x2 v) {
    typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
    __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, v), r, (int)voff, (int)soff, kSc1);
}
__device__ __forceinline__ f32x2 buf_ld2_sc1(__amdgpu_buffer_rsrc_t r, uint32_t voff, uint32_t soff) {
    return __builtin_bit_cast(f32x2, __builtin_amdgcn_raw_buffer_load_b64(r, (int)voff, (int)soff, kSc1));
}


template <int HS>
struct Small {
    static constexpr int NQ = (HS + 3) / 4;                       // waves per workgroup = record quads
    static constexpr int XBUF = 2 * NQ * kWave * 16;              // h exchange (split record), double-buffered
    static constexpr int LDS_FWD = Geo16<HS>::LDS_FWD + XBUF;
    static constexpr int NB = Img<HS, false>::NB > Img<HS, true>::NB ? Img<HS, false>::NB : Img<HS, true>::NB;
    static constexpr int RED = NQ * NB * kWave * 16;              // partial transposed products
    static constexpr int LDS_BWD = BwdLds<HS, false>::BYTES + RED;
    static_assert(LDS_FWD <= 163840 && LDS_BWD <= 163840, "small-batch LDS exceeds 160 KiB");
    static_assert(XBUF >= 2 * Geo<HS>::QC * 16, "two split records fit the exchange buffer");
    static_assert(Geo16<HS>::LDS_FWD % 16 == 0 && BwdLds<HS, false>::BYTES % 16 == 0, "16-B aligned buffers");
};

template <int V>
struct IC {
    static constexpr int v = V;
};
// f(IC<w>) for the wave-uniform w: every quad's code is a compile-time instance (register arrays stay
// statically indexed)
template <int HS, class F>
__device__ __forceinline__ void by_quad(int w, F &&f) {
    if constexpr (HS > 12) {
        if (w == 3) { f(IC<3>{}); return; }
    }
    if constexpr (HS > 8) {
        if (w == 2) { f(IC<2>{}); return; }
    }
    if constexpr (HS > 4) {
        if (w == 1) { f(IC<1>{}); return; }
    }
    f(IC<0>{});
}
template <int HS, int W>
struct QR {   // slot range of quad W
    static constexpr int R0 = 4 * W, R1 = 4 * W + 4 < HS ? 4 * W + 4 : HS;
};

// quad k of a compact record (store_quads' layout: full quads, then the HS%4 tail slots per lane)
template <int HS, int k>
__device__ __forceinline__ void store_quad(f32x4 *dst, const float (&v)[HS], int lane) {
    constexpr int FQ = HS / 4, TS = HS % 4;
    if constexpr (k < FQ) {
        dst[k * kWave + lane] = f32x4{v[4 * k], v[4 * k + 1], v[4 * k + 2], v[4 * k + 3]};
    } else {
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

// LDS-only workgroup barrier: the wave's LDS writes are complete, its global loads stay in flight
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }
// before a barrier that hands global slab records between waves: this wave's stores are complete
__device__ __forceinline__ void vm_drain() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

// Per-phase image refill: LDS-DMA (lds_fill). With one workgroup per CU it is exposed (~2.7 k cycles per
// 109 KB image at B = 15); staging the image through registers with the global loads issued before the
// retiring barrier measured slower (round 2), so the DMA form stays.
template <int NBYTES, int NWAVES>
__device__ __forceinline__ void small_fill(float *lw, const float *__restrict__ src) {
    lds_fill<NBYTES, NWAVES>(lw, src);
}

// h exchange: wave W publishes its slots of h_t, every wave reads the whole vector back
template <int HS, int W>
__device__ __forceinline__ void xchg_put(f32x4 *xb, const float (&h)[HS], int lane) {
    using Q = QR<HS, W>;
    f32x4 v = {0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
    for (int e = 0; e < 4; ++e)
        if (Q::R0 + e < Q::R1) v[e] = h[Q::R0 + e];
    xb[W * kWave + lane] = v;
}
// split-record exchange: wave W writes the f16 halves of its slots (hi at half s, lo at half HS + s of the
// record, fcr_f16.h) into an LDS record laid out like a slab record (store_quads); every wave reads it whole
template <int HS>
__device__ __forceinline__ int rec_half_byte(int k, int lane) {   // byte of half k of this lane's record
    constexpr int FQ = HS / 4, TS = HS % 4;
    const int d = k >> 1;
    const int dw = d < 4 * FQ ? ((d >> 2) * kWave + lane) * 16 + (d & 3) * 4 : FQ * kWave * 16 + (lane * TS + d - 4 * FQ) * 4;
    return dw + 2 * (k & 1);
}
template <int HS, int W>
__device__ __forceinline__ void xrec_put(char *xb, const float (&h)[HS], int lane) {
    using Q = QR<HS, W>;
    float one = 1.0f;
    asm("" : "+v"(one));
#pragma unroll
    for (int s = Q::R0; s < Q::R1; ++s) {
        const _Float16 hi = (_Float16)__builtin_fmaf(h[s], one, 0.0f);
        const _Float16 lo = (_Float16)__builtin_fmaf(h[s], one, -(float)hi);
        *reinterpret_cast<_Float16 *>(xb + rec_half_byte<HS>(s, lane)) = hi;
        *reinterpret_cast<_Float16 *>(xb + rec_half_byte<HS>(HS + s, lane)) = lo;
    }
}

template <int HS>
__device__ __forceinline__ void xchg_get(const f32x4 *xb, float (&h)[HS], int lane) {
#pragma unroll
    for (int k = 0; k < Small<HS>::NQ; ++k) {
        const f32x4 v = xb[k * kWave + lane];
#pragma unroll
        for (int e = 0; e < 4; ++e)
            if (4 * k + e < HS) h[4 * k + e] = v[e];
    }
}

// ---------------------------------------------------------------------------------------------------
// forward: the fused forward kernel's program (fcr_fwd.h) with the cell's tiles split over the waves
// ---------------------------------------------------------------------------------------------------
template <int HS, bool STORE>
__global__ __launch_bounds__(Small<HS>::NQ * kWave, 1) void fcr_sfwd_kernel(FwdArgs a) {
    using G = Geo16<HS>;
    constexpr int NQ = Small<HS>::NQ;
    extern __shared__ __attribute__((aligned(16))) float lw[];
    // [layer 1|2 fragments, refilled per phase | layer 0 | misc | h exchange]
    float *lw0 = lw + G::FA1;
    float *lfnp = lw0 + G::FA0;
    float *lfcp = lfnp + G::FNP;
    float *lfcb = lfcp + G::FCP;
    f32x4 *xbuf = reinterpret_cast<f32x4 *>(lw + G::LDS_FWD / 4);
    constexpr int RECB = Geo<HS>::QC * 16;   // one split record (bytes); two of them double-buffer the exchange
    lds_copy(lw0, a.p.fa[0], G::FA0);
    lds_copy(lfnp, a.p.fnp, G::FNP);
    lds_copy(lfcp, a.p.fcp, G::FCP);
    lds_copy(lfcb, a.p.fcb, 4);
    const int lane = threadIdx.x & 63;
    const int q = lane >> 4, sl = lane & 15;
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int grp = blockIdx.x;   // the fused kernels' wave index: same slab regions
    const int b = grp * kTile + sl;
    const bool valid = b < a.B;
    const bool lead = w == 0;     // writes the per-trajectory outputs
    const int bc = valid ? b : a.B - 1;
    const int N = a.N;
    const float alpha = a.alpha;

    const float ref = a.X[(size_t)bc * kCtrlIn + 2];                 // Functions.py:1392
    const float *st = a.states + (size_t)bc * kL * kIn;
    float w0[kL], w1[kL];
    const float scq = a.p.wsc[q], sc4 = a.p.wsc[4];
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
#pragma unroll
    for (int r = 0; r < HS; ++r) c[r] = hout[r] = hp[r] = xc[r] = xn[r] = 0.0f;
    const size_t qcell = (size_t)Geo<HS>::QC;
    const size_t wseq = (size_t)grp * N * kLayers * kL * qcell;
    f32x4 *hs_wave = a.hseq + wseq;
    f32x4 *cs_wave = a.cseq + wseq;
    f32x2 *xw_wave = a.xw + (size_t)grp * N * kL * kWave;
    Pace turn;
    turn.turn = 0;
    unsigned long long sc[6] = {0, 0, 0, 0, 0, 0};   // FCR_STAMP: cells, exchanges, refills, count, head+readout, refill+first load
    const unsigned long long sk0 = fstamp();
    __syncthreads();

    for (int j = 0; j < N; ++j) {
        const unsigned long long sw0 = fstamp();
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
        if (lead && valid && q == 0) a.prediction[(size_t)b * N + j] = pred;   // Functions.py:1455,1466

        f32x4 *hsj = hs_wave + (size_t)j * kLayers * kL * qcell;
        f32x4 *csj = cs_wave + (size_t)j * kLayers * kL * qcell;
#define SEQ_H(l, t) (hsj + (size_t)((l) * kL + (t)) * qcell)
#define SEQ_C(l, t) (csj + (size_t)((l) * kL + (t)) * qcell)
        if (FCR_STAMP) sc[4] += fstamp() - sw0;   // window head
        // ---- layer 0 (Functions.py:374) ----
        for (int t = 0; t < kL; ++t) {
            const float x0 = w0[0], x1 = w1[0];
            rot_left(w0);
            rot_left(w1);
            char *xb = reinterpret_cast<char *>(xbuf) + (t & 1) * RECB;
            const unsigned long long s0 = fstamp();
            by_quad<HS>(w, [&](auto Wc) {
                constexpr int W = decltype(Wc)::v;
                using Q = QR<HS, W>;
                if (t == 0) fwd16_cell<HS, true, true, false, Q::R0, Q::R1>(lw0, lane, x0, x1, hp, hp, c, hout, turn);
                else fwd16_cell<HS, true, false, false, Q::R0, Q::R1>(lw0, lane, x0, x1, hp, hp, c, hout, turn);
                if (STORE && t + 1 < kL) store_quad<HS, W>(SEQ_C(0, t), c, lane);   // c_9 is never a c_{t-1}
                xrec_put<HS, W>(xb, hout, lane);
            });
            if (STORE && lead) xw_wave[((size_t)j * kL + t) * kWave + lane] = f32x2{x0, x1};
            const unsigned long long s1 = fstamp();
            lds_barrier();
            load_quads<HS>(hp, reinterpret_cast<const f32x4 *>(xb), lane);   // the whole split record of h_t
            by_quad<HS>(w, [&](auto Wc) { store_quad<HS, decltype(Wc)::v>(SEQ_H(0, t), hp, lane); });
            if (FCR_STAMP) {
                sc[0] += s1 - s0;
                sc[1] += fstamp() - s1;
                sc[3] += 1;
            }
        }
        // ---- layers 1, 2: input sequence from the slab records the workgroup wrote ----
#pragma unroll
        for (int l = 1; l < kLayers; ++l) {
            const bool keep_h = l == 1 || STORE;
            const unsigned long long sf0 = fstamp();
            vm_drain();   // this wave's chunks of the layer-below records are in memory before the barrier
            small_fill<G::FA1 * 4, NQ>(lw, a.p.fa[l]);
            if (FCR_STAMP) sc[2] += fstamp() - sf0;
            load_quads<HS>(xc, SEQ_H(l - 1, 0), lane);
            if (FCR_STAMP) {   // diagnostic: the first record's latency (the cell would wait for it anyway)
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                sc[5] += fstamp() - sf0;
            }
            for (int t = 0; t < kL; ++t) {
                load_quads<HS>(xn, SEQ_H(l - 1, t + 1 < kL ? t + 1 : t), lane);
                const bool last = l == kLayers - 1 && t + 1 == kL;   // h_9 of layer 2: the readout's, in fp32
                char *xb = reinterpret_cast<char *>(xbuf) + (t & 1) * RECB;
                const unsigned long long s0 = fstamp();
                by_quad<HS>(w, [&](auto Wc) {
                    constexpr int W = decltype(Wc)::v;
                    using Q = QR<HS, W>;
                    if (t == 0) fwd16_cell<HS, false, true, false, Q::R0, Q::R1>(lw, lane, 0.0f, 0.0f, xc, hp, c, hout, turn);
                    else fwd16_cell<HS, false, false, false, Q::R0, Q::R1>(lw, lane, 0.0f, 0.0f, xc, hp, c, hout, turn);
                    if (STORE && t + 1 < kL) store_quad<HS, W>(SEQ_C(l, t), c, lane);
                    if (last) xchg_put<HS, W>(reinterpret_cast<f32x4 *>(xb), hout, lane);
                    else xrec_put<HS, W>(xb, hout, lane);
                });
                const unsigned long long s1 = fstamp();
                lds_barrier();
                if (last) {
                    xchg_get<HS>(reinterpret_cast<const f32x4 *>(xb), hout, lane);
                } else {
                    load_quads<HS>(hp, reinterpret_cast<const f32x4 *>(xb), lane);
                    if (keep_h) by_quad<HS>(w, [&](auto Wc) { store_quad<HS, decltype(Wc)::v>(SEQ_H(l, t), hp, lane); });
                }
                if (FCR_STAMP) {
                    sc[0] += s1 - s0;
                    sc[1] += fstamp() - s1;
                    sc[3] += 1;
                }
#pragma unroll
                for (int r = 0; r < HS; ++r) xc[r] = xn[r];
            }
        }
#undef SEQ_H
#undef SEQ_C
        const unsigned long long sr0 = fstamp();
        // ---- readout fc(h_9 of layer 2) (Functions.py:377), identical in every wave ----
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
        if (lead && valid) {
            const float mine = sel4(q, xh0, xh1, xh2, xh3);
            a.xhat_ws[((size_t)b * N + j) * kOut + q] = mine;
            if (a.xhat_user) a.xhat_user[((size_t)b * N + j) * kOut + q] = mine;
        }
        const float err = sq(xh0 - ref);                              // Functions.py:1405-1414, 1443-1452
        const float con = relu(-xh1) + relu(-xh2) + relu(xh1 - kP1Max) + relu(xh2 - kP2Max);
        tot_sum += (err + cmd_j) + con;
        err_sum += err;
        cmd_sum += cmd_j;
        if (FCR_STAMP) sc[4] += fstamp() - sr0;   // readout and costs
    }
    const float cost = tot_sum / (float)N;                             // Functions.py:1458-1460
    if (lead && valid && q == 0) {
        a.cost[b] = cost;
        a.command[b] = cmd_sum / (float)N;
        a.error[b] = err_sum / (float)N;
    }
    float part = (valid && q == 0) ? cost : 0.0f;
#pragma unroll
    for (int m = 1; m < 64; m <<= 1) part += __shfl_xor(part, m);
    if (lead && lane == 0) a.loss_part[grp] = part;
    if (FCR_STAMP && lane == 0) {   // diagnostic builds: per (group, wave) cycle sums
        unsigned long long *o = a.stamp + ((size_t)grp * NQ + w) * 8;
        o[0] = sc[0];
        o[1] = sc[1];
        o[2] = sc[2];
        o[3] = sc[3];
        o[4] = fstamp() - sk0;
        o[5] = sc[4];
        o[6] = sc[5];
    }
}

// ---------------------------------------------------------------------------------------------------
// backward: the fused backward kernel's program (fcr_bwd.h) with each cell's slots split over the waves,
// software-pipelined across cells: a cell is A (recompute its gate pre-activations from the stored
// x_t, h_{t-1}) and B (cell gradients, dgates, the partial transposed product). A needs no gradient, so
// A(t-1) is issued between B(t) and the reduction of cell t: its MFMAs run while the wave waits at the
// reduction's barriers.
// ---------------------------------------------------------------------------------------------------
// Partial products of one cell -> the sums this wave needs: dh_prev of its slots (L0: combined slots σ =
// s; else σ = HS + s), dx of its slots (layers >= 1: σ = s, into its dseq quad) and, for L0, the window
// columns σ = HS, HS+1 (every wave: the row gradients feed each wave's window head).
// PUB (the layer-pipelined backward): after the first barrier — which every wave reached after draining its stores of
// the previous cell (din_ready_after) — one lane signals that cell's outputs: *pub = pub_v
template <int HS, bool L0, int W, bool PUB = false>
__device__ __forceinline__ void small_reduce(f32x4 *red, const f32x4 (&part)[Small<HS>::NB], int lane, float (&dh)[HS],
                                             float (&dxo)[HS], float &dxq, float &dx4, unsigned *pub = nullptr,
                                             unsigned pub_v = 0) {
    using Q = QR<HS, W>;
    constexpr int NQ = Small<HS>::NQ, NB = Small<HS>::NB;
    constexpr int NBL = Img<HS, L0>::NB;
    asm volatile("s_barrier" ::: "memory");   // every wave has read the previous cell's partials
    if constexpr (PUB) pipe_signal(pub, pub_v);
#pragma unroll
    for (int tau = 0; tau < NBL; ++tau) red[(W * NB + tau) * kWave + lane] = part[tau];
    lds_barrier();
    auto need = [&](int tau) {
        bool n = false;
        for (int s = Q::R0; s < Q::R1; ++s) {
            if ((s >> 2) == tau && !L0) n = true;                      // dx of own slots
            if (((L0 ? s : HS + s) >> 2) == tau) n = true;             // dh_prev of own slots
        }
        if (L0 && (HS >> 2 == tau || (HS + 1) >> 2 == tau)) n = true;  // window columns
        return n;
    };
    f32x4 sum[NB];
#pragma unroll
    for (int tau = 0; tau < NBL; ++tau) {
        if (!need(tau)) continue;
        f32x4 s = red[tau * kWave + lane];
#pragma unroll
        for (int v = 1; v < NQ; ++v) s += red[(v * NB + tau) * kWave + lane];
        sum[tau] = s;
    }
#pragma unroll
    for (int s = Q::R0; s < Q::R1; ++s) {
        const int sh = L0 ? s : HS + s;
        dh[s] = sum[sh >> 2][sh & 3];
        if (!L0) dxo[s] = sum[s >> 2][s & 3];
    }
    if (L0) {
        dxq = sum[HS >> 2][HS & 3];
        dx4 = sum[(HS + 1) >> 2][(HS + 1) & 3];
    }
}

// A's operands: the recomputation's B operand (x_t, h_{t-1} of the cell, split into f16 halves)
template <int HS, bool L0>
struct AOps {
    f16x8 bh[Img<HS, L0>::KB], bl[Img<HS, L0>::KB];
};
template <int HS, bool L0, bool FIRST>
struct ARange {
    using Gm = Geo16<HS>;
    static constexpr int KB = Img<HS, L0>::KB;
    static constexpr int KLO = (L0 && FIRST) ? Gm::XBLK : 0;
    static constexpr int KHI = FIRST ? (L0 ? Gm::XBLK + 1 : Gm::KX1) : KB;
    static constexpr bool TAIL = !L0 && Gm::TAIL1;
};
template <int HS, bool L0, bool FIRST>
__device__ __forceinline__ void sb_split(const CellIn<HS> &ci, AOps<HS, L0> &o) {
    using A = ARange<HS, L0, FIRST>;
    float xv[HS], hv[HS];
#pragma unroll
    for (int s = 0; s < HS; ++s) {
        xv[s] = L0 ? 0.0f : ci.x[s >> 2][s & 3];
        hv[s] = FIRST ? 0.0f : ci.h[s >> 2][s & 3];
    }
    const float x0 = ci.x[0][0], x1 = ci.x[0][1];
#pragma unroll
    for (int kb = 0; kb < A::KB; ++kb) o.bh[kb] = o.bl[kb] = f16x8{};
#pragma unroll
    for (int kb = A::KLO; kb < A::KHI; ++kb) rec_operand<HS, L0, FIRST, false>(kb, x0, x1, xv, hv, o.bh[kb], o.bl[kb]);
    if (A::TAIL && A::KHI == A::KB) o.bh[A::KB - 1] = tail_operand<false>(o.bh[A::KB - 1], o.bl[A::KB - 1]);
}
// A: gate pre-activations of this wave's tiles (the forward's products, the same k order), one tile at a
// time: its image rows (hi, lo per k-block) are read a chunk ahead of its MFMAs
template <int HS, bool L0>
struct AFrag {
    f16x8 h[Img<HS, L0>::KB], l[Img<HS, L0>::KB];
};
template <int HS, bool L0, bool FIRST>
__device__ __forceinline__ void sb_aread(uint32_t fb, int r, AFrag<HS, L0> &f) {
    using A = ARange<HS, L0, FIRST>;
    using I = Img<HS, L0>;
    constexpr uint32_t TILE = I::TILE, LO = I::HALF;
    uint32_t fbl = fb + LO;
    asm volatile("" : "+v"(fbl));
#pragma unroll
    for (int kb = A::KLO; kb < A::KHI; ++kb) {
        const f16x4 h0 = lds_b64_f16(fb + 8u * (2 * kb) + r * TILE), h1 = lds_b64_f16(fb + 8u * (2 * kb + 1) + r * TILE);
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            f.h[kb][k] = h0[k];
            f.h[kb][4 + k] = h1[k];
        }
        if (!(A::TAIL && kb == A::KB - 1)) {
            const f16x4 l0 = lds_b64_f16(fbl + 8u * (2 * kb) + r * TILE), l1 = lds_b64_f16(fbl + 8u * (2 * kb + 1) + r * TILE);
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                f.l[kb][k] = l0[k];
                f.l[kb][4 + k] = l1[k];
            }
        }
    }
}
template <int HS, bool L0, bool FIRST>
__device__ __forceinline__ f32x4 sb_atile(const AFrag<HS, L0> &f, const AOps<HS, L0> &o) {
    using A = ARange<HS, L0, FIRST>;
    f32x4 g = {0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
    for (int kb = A::KLO; kb < A::KHI; ++kb) {
        if (A::TAIL && kb == A::KB - 1) g = mfma16(f.h[kb], o.bh[kb], g);
        else g = mma3(f.h[kb], f.l[kb], o.bh[kb], o.bl[kb], g);
    }
    return g;
}

// B's scale: the incoming dh (+ din or ext) of this wave's slots and the power of two for the f16 split of
// its dgates (as in bwd_cell: 2^(13-e), e = exponent of the largest |dh| + |dc| of the trajectory's slots)
struct BScale {
    float sg0, sgg, down;
};
template <int HS, bool DIN, int R0, int R1>
__device__ __forceinline__ BScale sb_scale(const CellIn<HS> &ci, const float (&ext)[HS], float (&dh)[HS],
                                           const float (&dc)[HS]) {
    float m = 0.0f;
#pragma unroll
    for (int r = R0; r < R1; ++r) {
        dh[r] += DIN ? ci.d[r >> 2][r & 3] : ext[r];
        m = fmaxf(m, fabsf(dh[r]) + fabsf(dc[r]));
    }
    m = max_q(m);
    const int e = max(__builtin_amdgcn_frexp_expf(m), -100);   // m < 2^e; all-zero -> e = 0
    BScale b;
    b.sg0 = __builtin_amdgcn_ldexpf(1.0f, 13 - e) * kInvNegLog2e;
    b.sgg = b.sg0 * -0.5f;
    b.down = __builtin_amdgcn_ldexpf(1.0f, e - 13);
    return b;
}
// cell gradient of slot r from its pre-activations: the 4 dgates as (scaled factor, local derivative)
// pairs at va/vb[0..3] (multiplied inside the split, split8p)
template <int HS, bool FIRST>
__device__ __forceinline__ void sb_slot(int r, f32x4 g, const CellIn<HS> &ci, const BScale &sc, float (&dh)[HS],
                                        float (&dc)[HS], float *va, float *vb) {
    f32x4 P;
    f32x2 Q;
    lstm_point_grad<FIRST>(g, FIRST ? 0.0f : ci.c[r >> 2][r & 3], P, Q);
    const float dcv = fmaf(dh[r], P[0], dc[r]);   // dc = dc_carried + dh dh/dc
    dc[r] = dcv * Q[1];
    const float dcs = dcv * sc.sg0;
    va[0] = dcs;
    vb[0] = P[2];
    va[1] = dcs;
    vb[1] = P[3];
    va[2] = dcv * sc.sgg;
    vb[2] = Q[0];
    va[3] = dh[r] * sc.sg0;
    vb[3] = P[1];
}

// B's transposed product Wᵀ·dgates over THIS wave's gate rows for output tile tau: the image columns of
// its blocks (read a tile ahead) and 3 MFMAs per block (2 for a half block)
template <int HS, bool L0, int R0, int R1>
struct TFrag {
    static constexpr int NK = (R1 + 1) / 2 - R0 / 2;
    f16x4 h0[NK], l0[NK], h1[NK], l1[NK];
};
template <int HS, bool L0, int R0, int R1>
__device__ __forceinline__ void sb_tread(uint32_t tb, int tau, TFrag<HS, L0, R0, R1> &f) {
    using I = Img<HS, L0>;
    constexpr uint32_t TILE = I::TILE, LO = I::HALF;
    constexpr int K0 = R0 / 2, K1 = (R1 + 1) / 2;
    uint32_t tbl = tb + LO;
    asm volatile("" : "+v"(tbl));
#pragma unroll
    for (int kbb = K0; kbb < K1; ++kbb) {
        const uint32_t ct = 8u * (2 * (tau >> 1) + (tau & 1)) + 2 * kbb * TILE;
        f.h0[kbb - K0] = lds_tr_f16(tb + ct);
        f.l0[kbb - K0] = lds_tr_f16(tbl + ct);
        if (2 * kbb + 1 < R1) {
            f.h1[kbb - K0] = lds_tr_f16(tb + ct + TILE);
            f.l1[kbb - K0] = lds_tr_f16(tbl + ct + TILE);
        }
    }
}
template <int HS, bool L0, int R0, int R1>
__device__ __forceinline__ f32x4 sb_ttile(const TFrag<HS, L0, R0, R1> &f, const f16x8 (&gh)[2], const f16x8 (&gl)[2]) {
    constexpr int K0 = R0 / 2, K1 = (R1 + 1) / 2;
    f32x4 acc = {0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
    for (int kbb = K0; kbb < K1; ++kbb) {
        const int i = kbb - K0;
        if (2 * kbb + 1 >= R1) {
            // half block (its second slot is padding): hi·hi and hi·lo in ONE MFMA, then lo·hi
            typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
            const u32x4 h = __builtin_bit_cast(u32x4, gh[i]), l = __builtin_bit_cast(u32x4, gl[i]);
            f16x8 a2, al2 = {};
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                a2[k] = a2[4 + k] = f.h0[i][k];
                al2[k] = f.l0[i][k];
            }
            acc = mfma16(a2, __builtin_bit_cast(f16x8, u32x4{h[0], h[1], l[0], l[1]}), acc);
            acc = mfma16(al2, gh[i], acc);
        } else {
            f16x8 ah, al;
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                ah[k] = f.h0[i][k];
                ah[4 + k] = f.h1[i][k];
                al[k] = f.l0[i][k];
                al[4 + k] = f.l1[i][k];
            }
            acc = mma3(ah, al, gh[i], gl[i], acc);
        }
    }
    return acc;
}

// PIPE (fcr_pipe.h): one workgroup per (group, layer, window set) — set s of S takes windows N-1-s, N-1-s-S, ... — so
// the cell after (j, l, 0) is (j - S, l, 9), the din of a cell is waited for on the layer above's counters (same set),
// and each cell's outputs are published on this workgroup's counter
template <int HS, bool PIPE = false>
struct SbCtx {
    NextIn nb;                        // this group's slab descriptors
    f32x4 *dseq_w;                    // this group's dseq
    __amdgpu_buffer_rsrc_t rr;        // this wave's copy of the window-row gradients
    f32x4 *red;                       // LDS partial products
    uint32_t fb1, tb1, fb0, tb0;      // image lane addresses (layers >= 1 / layer 0 geometry)
    float scq, sc4;
    int lane, N;
    Stamps *sp;                       // FCR_STAMP diagnostic builds: [grad, recompute, reduce, cells, total, head+fills]
    __device__ uint32_t hoff(int j, int l, int t) const {
        return (uint32_t)(((size_t)(j * kLayers + l) * kL + t) * Geo<HS>::QC * 16);
    }
    __device__ size_t doff(int j, int lfrom, int t) const { return ((size_t)(j * 2 + (2 - lfrom)) * kL + t) * Geo<HS>::QC; }
    unsigned *flags;                  // PIPE: this group's counters (kPipeFlags)
    int fl_own, fl_above;             // PIPE: index of this workgroup's counter, of the layer above's (or -1)
    int S;                            // PIPE: window sets (the stride between this workgroup's windows)
    mutable bool din_pending;         // PIPE: the next cell's din was not yet published when it would have been prefetched
    __device__ NextIn next_of(int j, int l, int t) const {   // the cell processed after (j, l, t)
        NextIn n = nb;
        int nj = j, nl = l, nt = t - 1;
        if (t == 0) {
            nt = kL - 1;
            nl = PIPE ? l : l - 1;
            if (PIPE || l == 0) { nl = PIPE ? l : 2; nj = j - (PIPE ? S : 1); }
        }
        if (nj < 0) { nj = 0; nl = PIPE ? l : 2; nt = 9; }   // past the last cell: a valid one (harmless)
        n.x = nl == 0 ? (uint32_t)((nj * kL + nt) * kWave * 8) : hoff(nj, nl > 0 ? nl - 1 : 0, nt);
        n.h = hoff(nj, nl, nt > 0 ? nt - 1 : 0);
        n.c = n.h;
        n.d = (uint32_t)((nl < 2 ? doff(nj, nl + 1, nt) : 0) * 16);
        return n;
    }
    // PIPE: a layer workgroup's progress counter after cell (j, t) (its windows N-1-s, N-1-s-S, ..., t = 9 .. 0)
    __device__ unsigned done_after(int j, int t) const { return (unsigned)((N - 1 - j) / S * kL + (kL - 1 - t) + 1); }
    // PIPE, in cell (j, t) before prefetching the din of the cell after it: this wave's stores of the previous cell
    // are drained (they are signalled at this cell's first reduction barrier); true if the layer above has already
    // published that din (else the next cell waits for it at its start: a late din never stalls this cell)
    __device__ bool din_ready_after(int j, int t) const {
        pipe_drain();
        int nj = j, nt = t - 1;
        if (t == 0) { nj = j - S; nt = kL - 1; }
        return nj < 0 || fl_above < 0 || pipe_count(flags + fl_above) >= done_after(nj, nt);
    }
};

// inputs of the next A (x_t, h_{t-1}: whole records) and of the next B (c_{t-1}, din: this wave's quad)
template <int HS, bool NX_L0, bool NX_HC>
__device__ __forceinline__ void sb_load_a(CellIn<HS> &ci, const NextIn &n, int lane) {
    load_xhd<HS, NX_L0, NX_HC, false>(ci, n, lane);
}
template <int HS, int W, bool NX_HC, bool NX_DIN, bool PIPE = false>
__device__ __forceinline__ void sb_load_b(CellIn<HS> &ci, const NextIn &n, int lane) {
    if (NX_HC) ld_quad<HS, W>(ci.c, n.rc, n.c, lane);
    if (NX_DIN) {   // PIPE: another workgroup's record (sc1 load, the hand-off above)
        if constexpr (PIPE) ld_quad_sc1<HS, W>(ci.d, n.rd, n.d, lane);
        else ld_quad<HS, W>(ci.d, n.rd, n.d, lane);
    }
}

// One pipeline step of layer LAYER at cell t (t = 9 .. 0), in chunks that pair independent work so the
// MFMA pipe and the vector ALU overlap (one wave per SIMD: nothing else fills the MFMA shadows):
//   region 1, per own slot r: A(t-1)'s tile r (DO_A; FA: cell t-1 is the first) beside B(t)'s cell gradient
//             of slot r (FB: t = 0), the dgate split after each slot pair;
//   region 2, per output tile: B(t)'s transposed products beside a share of the operand split of A(t-2)
//             (DO_S; FS: t-2 = 0);
//   then the reduction of cell t and this wave's stores. Loads: B's next inputs (c, din of the cell after
//   t) after region 1, A's (x, h of the cell after t-2) after region 2 — a step ahead of their use.
template <int HS, int LAYER, int W, bool FB, bool DO_A, bool FA, bool DO_S, bool FS, bool S_NX_L0, bool S_NX_HC,
          bool B_NX_HC, bool B_NX_DIN, bool PIPE>
__device__ __forceinline__ void sb_step(const SbCtx<HS, PIPE> &x, int j, int t, const float (&ext)[HS], CellIn<HS> &ci,
                                        f32x4 (&G)[4], AOps<HS, LAYER == 0> &ops, float (&dh)[HS], float (&dc)[HS]) {
    using Q = QR<HS, W>;
    constexpr int R0 = Q::R0, R1 = Q::R1, NS = R1 - R0;
    constexpr bool L0 = LAYER == 0, DIN = LAYER < 2;
    constexpr int NB = Img<HS, L0>::NB;
    const uint32_t fb = L0 ? x.fb0 : x.fb1, tb = L0 ? x.tb0 : x.tb1;
    if constexpr (PIPE && DIN) {
        if (x.din_pending) {   // this cell's din was late at the prefetch: wait for it now
            pipe_wait(x.flags, x.flags + x.fl_above, x.done_after(j, t));
            ld_quad_sc1<HS, W>(ci.d, x.nb.rd, (uint32_t)(x.doff(j, LAYER + 1, t) * 16), x.lane);
            x.din_pending = false;
        }
    }
    const unsigned long long s0 = stamp_now();
    // ---- region 1 ----
    sched_fence();
    AFrag<HS, L0> fa[2];
    if constexpr (DO_A) sb_aread<HS, L0, FA>(fb, R0, fa[0]);
    const BScale sc = sb_scale<HS, DIN, R0, R1>(ci, ext, dh, dc);
    f32x4 Gn[4];
    f16x8 gh[2], gl[2];
    float va[8], vb[8];
#pragma unroll
    for (int u = 0; u < NS; ++u) {
        sched_fence();
        if constexpr (DO_A) {
            if (u + 1 < NS) sb_aread<HS, L0, FA>(fb, R0 + u + 1, fa[(u + 1) & 1]);
            Gn[u] = sb_atile<HS, L0, FA>(fa[u & 1], ops);
        }
        sb_slot<HS, FB>(R0 + u, G[u], ci, sc, dh, dc, va + 4 * (u & 1), vb + 4 * (u & 1));
        if ((u & 1) || u + 1 == NS) {
            if (!(u & 1)) {
#pragma unroll
                for (int k = 4; k < 8; ++k) va[k] = vb[k] = 0.0f;
            }
            split8p(va, vb, gh[u >> 1], gl[u >> 1]);
        }
    }
    sched_fence();
    if constexpr (PIPE) {   // the drain also for a cell with no din to prefetch
        const bool now = x.din_ready_after(j, t);
        const NextIn nx = x.next_of(j, LAYER, t);
        sb_load_b<HS, W, B_NX_HC, false, PIPE>(ci, nx, x.lane);
        if constexpr (B_NX_DIN) {
            if (now) ld_quad_sc1<HS, W>(ci.d, nx.rd, nx.d, x.lane);
            x.din_pending = !now;
        }
    } else {
        sb_load_b<HS, W, B_NX_HC, B_NX_DIN, PIPE>(ci, x.next_of(j, LAYER, t), x.lane);
    }
    const unsigned long long s1 = stamp_now();
    // ---- region 2 ----
    TFrag<HS, L0, R0, R1> tf[2];
    sb_tread<HS, L0, R0, R1>(tb, 0, tf[0]);
    f32x4 acc[Small<HS>::NB];
    // A(t-2)'s operand split spread over the output tiles: k-block kb goes with tile tau = kb * NB / KB
    using AR = ARange<HS, L0, FS>;
    float xv[HS], hv[HS];
#pragma unroll
    for (int s = 0; s < HS; ++s) {
        xv[s] = L0 ? 0.0f : ci.x[s >> 2][s & 3];
        hv[s] = FS ? 0.0f : ci.h[s >> 2][s & 3];
    }
    const float x0 = ci.x[0][0], x1 = ci.x[0][1];
#pragma unroll
    for (int tau = 0; tau < NB; ++tau) {
        sched_fence();
        if (tau + 1 < NB) sb_tread<HS, L0, R0, R1>(tb, tau + 1, tf[(tau + 1) & 1]);
        acc[tau] = sb_ttile<HS, L0, R0, R1>(tf[tau & 1], gh, gl);
        if constexpr (DO_S) {
#pragma unroll
            for (int kb = 0; kb < AR::KB; ++kb) {
                if (kb * NB / AR::KB != tau) continue;
                if (kb >= AR::KLO && kb < AR::KHI) rec_operand<HS, L0, FS, false>(kb, x0, x1, xv, hv, ops.bh[kb], ops.bl[kb]);
                else ops.bh[kb] = ops.bl[kb] = f16x8{};
                if (AR::TAIL && AR::KHI == AR::KB && kb == AR::KB - 1)
                    ops.bh[kb] = tail_operand<false>(ops.bh[kb], ops.bl[kb]);
            }
        }
    }
    sched_fence();
    if constexpr (DO_S) sb_load_a<HS, S_NX_L0, S_NX_HC>(ci, x.next_of(j, LAYER, t - 2), x.lane);
    if constexpr (DO_A) {
#pragma unroll
        for (int r = 0; r < NS; ++r) G[r] = Gn[r];
    }
    const unsigned long long s2 = stamp_now();
    f32x4 part[Small<HS>::NB];
#pragma unroll
    for (int tau = 0; tau < NB; ++tau) part[tau] = acc[tau] * sc.down;
    float dxo[HS], dxq = 0.0f, dx4 = 0.0f;
    // PIPE: signal the previous cell (done_after(j, t) - 1, this workgroup's order) at the first reduction barrier
    small_reduce<HS, L0, W, PIPE>(x.red, part, x.lane, dh, dxo, dxq, dx4, PIPE ? x.flags + x.fl_own : nullptr,
                                  PIPE ? x.done_after(j, t) - 1 : 0u);
    if (FCR_STAMP) {
        const unsigned long long s3 = stamp_now();
        x.sp->t[0] += s1 - s0;
        x.sp->t[1] += s2 - s1;
        x.sp->t[2] += s3 - s2;
        x.sp->t[3] += 1;
    }
    // this cell's outputs: the window-row gradients (layer 0) or the din of the layer below; PIPE: write-through, they
    // are another workgroup's inputs (signalled at the next cell's first reduction barrier)
    if constexpr (PIPE) {
        if (L0) buf_st2_sc1(x.rr, x.lane * 8, (uint32_t)((j * kL + t) * kWave * 8), f32x2{dxq * x.scq, dx4 * x.sc4});
        else st_quad_sc1<HS, W>(x.nb.rd, (uint32_t)(x.doff(j, LAYER, t) * 16), dxo, x.lane);
        if (t == kL - 1) {   // a window's first cell is on the cross-window chain (Pipe): published at once
            pipe_drain();
            lds_barrier();
            pipe_signal(x.flags + x.fl_own, x.done_after(j, t));
        }
    } else {
        if (L0) buf_st2(x.rr, x.lane * 8, (uint32_t)((j * kL + t) * kWave * 8), f32x2{dxq * x.scq, dx4 * x.sc4});   // row j+t
        else store_quad<HS, W>(x.dseq_w + x.doff(j, LAYER, t), dxo, x.lane);
    }
}

template <int HS, int LAYER, int W, bool PIPE = false>
__device__ __forceinline__ void sb_phase(const SbCtx<HS, PIPE> &x, int j, const float (&dh_out)[HS], CellIn<HS> &ci,
                                         float (&dh)[HS], float (&dc)[HS]) {
    using Q = QR<HS, W>;
    constexpr bool L0 = LAYER == 0, DIN = LAYER < 2;
    // the next phase's first cell: (j, LAYER - 1, 9), or (j - 1, 2, 9) after layer 0; PIPE: (j - 1, LAYER, 9)
    constexpr bool NEXT_L0 = PIPE ? L0 : LAYER == 1, NEXT_DIN = PIPE ? DIN : LAYER >= 1;
    float zero[HS];
#pragma unroll
    for (int r = 0; r < HS; ++r) zero[r] = 0.0f;
#pragma unroll
    for (int r = Q::R0; r < Q::R1; ++r) dh[r] = dc[r] = 0.0f;
    const unsigned long long p0 = stamp_now();
    // prologue: A(9), and A(8)'s operands (ci holds cell 9's x, h on entry)
    AOps<HS, L0> ops;
    f32x4 G[4];
    sb_split<HS, L0, false>(ci, ops);
    sb_load_a<HS, L0, true>(ci, x.next_of(j, LAYER, kL - 1), x.lane);
#pragma unroll
    for (int r = Q::R0; r < Q::R1; ++r) {
        AFrag<HS, L0> f;
        sb_aread<HS, L0, false>(L0 ? x.fb0 : x.fb1, r, f);
        G[r - Q::R0] = sb_atile<HS, L0, false>(f, ops);
    }
    sb_split<HS, L0, false>(ci, ops);
    sb_load_a<HS, L0, true>(ci, x.next_of(j, LAYER, kL - 2), x.lane);
    if (FCR_STAMP) x.sp->t[6] += stamp_now() - p0;
    //      <HS, LAYER, W, FB,   DO_A, FA,   DO_S, FS,   S_NX_L0, S_NX_HC, B_NX_HC, B_NX_DIN, PIPE>
    sb_step<HS, LAYER, W, false, true, false, true, false, L0, true, true, DIN, PIPE>(x, j, kL - 1, LAYER == 2 ? dh_out : zero,
                                                                                   ci, G, ops, dh, dc);
    for (int t = kL - 2; t >= 4; --t)
        sb_step<HS, LAYER, W, false, true, false, true, false, L0, true, true, DIN, PIPE>(x, j, t, zero, ci, G, ops, dh, dc);
    sb_step<HS, LAYER, W, false, true, false, true, false, L0, false, true, DIN, PIPE>(x, j, 3, zero, ci, G, ops, dh, dc);
    sb_step<HS, LAYER, W, false, true, false, true, true, NEXT_L0, true, true, DIN, PIPE>(x, j, 2, zero, ci, G, ops, dh, dc);
    sb_step<HS, LAYER, W, false, true, true, false, false, false, false, false, DIN, PIPE>(x, j, 1, zero, ci, G, ops, dh, dc);
    sb_step<HS, LAYER, W, true, false, false, false, false, false, false, true, NEXT_DIN, PIPE>(x, j, 0, zero, ci, G, ops, dh,
                                                                                              dc);
}

template <int HS>
__global__ __launch_bounds__(Small<HS>::NQ * kWave, 1) void fcr_sbwd_kernel(BwdArgs a) {
    using LD = BwdLds<HS, false>;
    using I1 = Img<HS, false>;
    using I0 = Img<HS, true>;
    constexpr int NQ = Small<HS>::NQ;
    extern __shared__ __attribute__((aligned(16))) float lw[];
    float *lfnp = lw + LD::REGION / 4;
    float *lfcp = lfnp + LD::FNP;
    lds_copy(lfnp, a.p.fnp, LD::FNP);
    lds_copy(lfcp, a.p.fcp, LD::FCP);
    __syncthreads();
    const int lane = threadIdx.x & 63;
    const int q = lane >> 4, sl = lane & 15;
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int grp = blockIdx.x;
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

    SbCtx<HS> x;
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
    const unsigned long long tk0 = stamp_now();
    x.scq = a.p.wsc[q];
    x.sc4 = a.p.wsc[4];
    x.red = reinterpret_cast<f32x4 *>(lw + LD::BYTES / 4);
    // this wave's own copy of the window-row gradients (dxrow holds NQ copies per group)
    x.rr = wave_rsrc(a.dxrow + ((size_t)grp * NQ + w) * N * kL * kWave, (size_t)N * kL * kWave * 8);
    const size_t qcell = (size_t)Geo<HS>::QC;
    const size_t seq_sz = (size_t)N * kLayers * kL * qcell;
    const size_t dseq_sz = (size_t)N * 2 * kL * qcell;
    x.nb.rh = wave_rsrc(a.hseq + (size_t)grp * seq_sz, seq_sz * 16);
    x.nb.rc = wave_rsrc(a.cseq + (size_t)grp * seq_sz, seq_sz * 16);
    x.nb.rx = wave_rsrc(a.xw + (size_t)grp * N * kL * kWave, (size_t)N * kL * kWave * 8);
    x.nb.rd = wave_rsrc(a.dseq + (size_t)grp * dseq_sz, dseq_sz * 16);
    x.dseq_w = a.dseq + (size_t)grp * dseq_sz;
    auto row_grad = [&](int rho) {   // sum over windows v = max(0, rho-9) .. min(N-1, rho) of dx(v, rho-v)
        f32x2 acc2 = {0.0f, 0.0f};
        const int w_hi = rho < N - 1 ? rho : N - 1;
        const int w_lo = rho - (kL - 1) > 0 ? rho - (kL - 1) : 0;
        for (int v = w_hi; v >= w_lo; --v) acc2 += buf_ld2(x.rr, lane * 8, (uint32_t)((v * kL + (rho - v)) * kWave * 8));
        return acc2;
    };
    float dh[HS], dc[HS];
#pragma unroll
    for (int r = 0; r < HS; ++r) dh[r] = dc[r] = 0.0f;
    CellIn<HS> ci;
    {
        const NextIn f = x.next_of(N - 1, 2, kL);   // t = kL -> (N-1, 2, 9)
        by_quad<HS>(w, [&](auto Wc) {
            constexpr int W = decltype(Wc)::v;
            sb_load_a<HS, false, true>(ci, f, lane);
            sb_load_b<HS, W, true, false>(ci, f, lane);
        });
    }

    for (int j = N - 1; j >= 0; --j) {
        const float *lfnp_j = opaque(lfnp), *lfcp_j = opaque(lfcp);
        // layer 2's image (the barriers also retire layer 0's reads of the previous window)
        const unsigned long long th0 = stamp_now();
        // the window head's global loads go out before the refill's barriers, which cover their latency
        const float x0 = xh[j * kOut + 0], x1 = xh[j * kOut + 1], x2 = xh[j * kOut + 2], x3 = xh[j * kOut + 3];
        const float uj = pred[j], uj1 = pred[j + 1 < N ? j + 1 : j], uj2 = pred[j + 2 < N ? j + 2 : j];
        const f32x2 Gr = j <= N - 2 ? row_grad(kL + j) : f32x2{0.0f, 0.0f};
        small_fill<I1::BYTES, NQ>(lw, a.p.img[2]);
        const unsigned long long th1 = stamp_now();
        float d0 = wgt * 2.0f * (x0 - ref);                             // Functions.py:1443-1452
        float d1 = wgt * ((-x1 > 0.0f ? -1.0f : 0.0f) + (x1 - kP1Max > 0.0f ? 1.0f : 0.0f));
        float d2 = wgt * ((-x2 > 0.0f ? -1.0f : 0.0f) + (x2 - kP2Max > 0.0f ? 1.0f : 0.0f));
        float d3 = 0.0f;
        if (j <= N - 2) {
            d0 += __shfl(Gr[0], sl);
            d1 += __shfl(Gr[0], sl + 16);
            d2 += __shfl(Gr[0], sl + 32);
            d3 += __shfl(Gr[0], sl + 48);
            const float g4 = __shfl(Gr[1], sl);
            float du = 2.0f * alpha * wgt * (uj1 - uj);
            if (j + 2 < N) du += 2.0f * alpha * wgt * (uj1 - uj2);
            du += g4;
            float z[kMS];                                               // Functions.py:1424-1430
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
        float dh_out[HS];
#pragma unroll
        for (int r = 0; r < HS; ++r) {
            const float *fp = lfcp_j + r * 4 + q;
            dh_out[r] = fp[0] * d0 + fp[HS * 4] * d1 + fp[2 * HS * 4] * d2 + fp[3 * HS * 4] * d3;
        }
        const unsigned long long th2 = stamp_now();
        by_quad<HS>(w, [&](auto Wc) { sb_phase<HS, 2, decltype(Wc)::v>(x, j, dh_out, ci, dh, dc); });
        const unsigned long long tf0 = stamp_now();
        small_fill<I1::BYTES, NQ>(lw, a.p.img[1]);
        const unsigned long long tf1 = stamp_now();
        by_quad<HS>(w, [&](auto Wc) { sb_phase<HS, 1, decltype(Wc)::v>(x, j, dh_out, ci, dh, dc); });
        const unsigned long long tf2 = stamp_now();
        small_fill<I0::BYTES, NQ>(lw, a.p.img[0]);
        if (FCR_STAMP) {
            sp.t[5] += (th1 - th0) + (tf1 - tf0) + (stamp_now() - tf2);   // three refills
            sp.t[7] += th2 - th1;                                         // window head
        }
        by_quad<HS>(w, [&](auto Wc) { sb_phase<HS, 0, decltype(Wc)::v>(x, j, dh_out, ci, dh, dc); });
    }
    if (FCR_STAMP && lane == 0) {   // diagnostic builds: per (group, wave) cycle sums
        unsigned long long *o = a.stamp + ((size_t)grp * NQ + w) * 8;
        o[0] = sp.t[0];
        o[1] = sp.t[1];
        o[2] = sp.t[2];
        o[3] = sp.t[3];
        o[4] = stamp_now() - tk0;
        o[5] = sp.t[5];
        o[6] = sp.t[6];
        o[7] = sp.t[7];
    }
    const float g_u0_rows = row_grad(kL - 1)[1];   // row 9, col 4 = u0 (Functions.py:1396)
    float du0 = 2.0f * alpha * wgt * (pred[0] - s84);
    if (N > 1) du0 += 2.0f * alpha * wgt * (pred[0] - pred[1]);
    if (lead && valid && q == 0) a.g_u0[b] = g_u0_rows + du0;
}

}  // namespace fcr
