// fcr_abi.hip — host side and C ABI (include/fcr.h) of the gfx950 rollout engine: the rollout's
// forward/backward (fused kernels for H <= 52, the per-cell path above) and the LSTM surrogate's
// training step; the plant, closed-loop and window entry points are in fcr_rows.hip.
//
// Replaces the torch work behind `loss_function(...)` / `loss.backward()` at
// /root/reference/Unsupervised Learning/Functions.py:646 and :655. All launches are stream-ordered on
// the caller's stream; nothing here allocates or synchronises.
#include <hip/hip_runtime.h>
#include <stdarg.h>
#include <stdint.h>
#include <stdio.h>

#include <atomic>
#include <mutex>

#include "fcr.h"
#include "fcr_bwd.h"
#include "fcr_common.h"
#include "fcr_fnn.h"
#include "fcr_fwd.h"
#include "fcr_img.h"
#include "fcr_pack.h"
#include "fcr_host.h"
#include "fcr_pipe.h"
#include "fcr_small.h"
#include "fcr_sur.h"
#include "fcr_surrogate.h"
#include "fcr_wide.h"
#include "fcr_wbwd.h"
#include "fcr_wgemm.h"
#include "fcr_wgrad.h"

namespace fcr {

thread_local char g_err[512] = "no error";

int fail(int code, const char *fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof(g_err), fmt, ap);
    va_end(ap);
    return code;
}

int launch_check(const char *what) {
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return fail(FCR_EHIP, "launch of %s failed: %s", what, hipGetErrorString(e));
    return FCR_OK;
}

// hipFuncSetAttribute(max dynamic LDS) once per (kernel instantiation, device): one bit per device in the caller's
// static mask. The mask is atomic (calls on several threads are allowed, include/fcr.h), two first calls that race
// both set the attribute (idempotent), and a second device in the process gets its own bit (devices past 63 set
// it on every call).
int lds_attr(const void *fn, int bytes, std::atomic<unsigned long long> &done, const char *what) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) dev = -1;
    const unsigned long long bit = (dev >= 0 && dev < 64) ? 1ull << dev : 0ull;
    if (bit && (done.load(std::memory_order_acquire) & bit)) return FCR_OK;
    const hipError_t e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
    if (e != hipSuccess) return fail(FCR_EHIP, "hipFuncSetAttribute(%s): %s", what, hipGetErrorString(e));
    done.fetch_or(bit, std::memory_order_release);
    return FCR_OK;
}

// window-column scales of the f16 split's range guard (fcr_pack.h) -> wsc[8], from the call's inputs
int launch_range(const fcr_dims *d, const float *states, const float *u0, const float *noise, const float *fcw,
                 const float *fcb, float *part, float *wsc, hipStream_t s) {
    const size_t rows = (size_t)d->B * (d->N > kL ? d->N : kL);
    if (rows <= 16 * kRangeThreads) {   // small batch: one block, the final step inside (one launch)
        hipLaunchKernelGGL(range_partial_kernel, dim3(1), dim3(kRangeThreads), 0, s, states, u0, noise, d->B, d->N,
                           part, fcw, fcb, d->H, wsc);
        return launch_check("range_partial_kernel");
    }
    hipLaunchKernelGGL(range_partial_kernel, dim3(kRangeBlocks), dim3(kRangeThreads), 0, s, states, u0, noise, d->B,
                       d->N, part, nullptr, nullptr, 0, nullptr);
    int rc = launch_check("range_partial_kernel");
    if (rc) return rc;
    hipLaunchKernelGGL(range_final_kernel, dim3(1), dim3(64), 0, s, (const float *)part, kRangeBlocks, fcw, fcb, d->H,
                       wsc);
    return launch_check("range_final_kernel");
}

namespace {

struct Layout {
    int HS, nw, nw_pad;
    size_t fa[3], img[3], fcp, fcb, fnp, wsc, rng, xhat, dv, loss_part, fnn_part, hseq, cseq, xw, dseq, dxrow, stamp, total;
    size_t pipe_flags, pipe_rows;   // the layer-pipelined small-batch kernels (fcr_pipe.h), L.nw <= kPipeMaxGroups
    int ctrl_blocks;
};

size_t align_up(size_t x) { return (x + 255) & ~(size_t)255; }

// Kernels are instantiated for 4, 8 and 13 unit slots (H <= 16, 32, 52); a smaller H runs in the next
// tier with its padding units' weights zero — their gates stay at i = f = o = 1/2, g = 0, so c = h = 0
// and they add nothing to any product (tests/test_gpu_parity.py: H = 40 against the oracle).
constexpr int kMaxSlots = 13;
constexpr int kMaxWideH = 2048;   // H > 4*kMaxSlots: the GEMM-per-cell path (fcr_wide.h)
bool is_wide(const fcr_dims *d) { return d->H > 4 * kMaxSlots; }
int slot_tier(int H) { return H <= 16 ? 4 : (H <= 32 ? 8 : 13); }

int check_dims(const fcr_dims *d) {
    if (!d) return fail(FCR_EINVAL, "dims is NULL");
    if (d->B < 1) return fail(FCR_EINVAL, "B=%d must be >= 1", d->B);
    if (d->N < 1) return fail(FCR_EINVAL, "N=%d must be >= 1", d->N);
    if (d->L != kL) return fail(FCR_EUNSUPPORTED, "L=%d: the rollout window is fixed at 10 rows", d->L);
    if (d->layers != kLayers) return fail(FCR_EUNSUPPORTED, "layers=%d: built for 3", d->layers);
    if (d->in_dim != kIn || d->out_dim != kOut || d->ctrl_in != kCtrlIn)
        return fail(FCR_EUNSUPPORTED, "in/out/ctrl_in = %d/%d/%d: built for 5/4/3", d->in_dim,
                    d->out_dim, d->ctrl_in);
    if (d->ctrl_hidden < 1 || d->ctrl_hidden > 4 * kMS)
        return fail(FCR_EUNSUPPORTED, "ctrl_hidden=%d: built for 1..52", d->ctrl_hidden);
    if (d->H < 1 || d->H > kMaxWideH)
        return fail(FCR_EUNSUPPORTED, "H=%d: built for 1..%d", d->H, kMaxWideH);
    if ((long long)d->B * d->N > (1LL << 31)) return fail(FCR_EINVAL, "B*N too large");
    if (d->precision == 2)
        return fail(FCR_EUNSUPPORTED, "precision=2 (f16 forward, fp32-accurate backward) is retired: it ran 1.08x the "
                    "fp32 step at the f16 mode's accuracy; use FCR_PRECISION_F16 (1) or FCR_PRECISION_FP32 (0)");
    if (d->precision != FCR_PRECISION_FP32 && d->precision != FCR_PRECISION_F16)
        return fail(FCR_EINVAL, "precision=%d: FCR_PRECISION_FP32 (0) or FCR_PRECISION_F16 (1)", d->precision);
    if (d->precision != FCR_PRECISION_FP32 && is_wide(d))
        return fail(FCR_EUNSUPPORTED, "reduced precision is built for H <= %d (the fused kernels)", 4 * kMaxSlots);
    return FCR_OK;
}

// the layer-pipelined small-batch kernels (fcr_pipe.h) run at most this many 16-trajectory groups (3 workgroups each)
constexpr int kPipeMaxGroups = 32;

Layout make_layout(const fcr_dims *d, int with_backward) {
    Layout L{};
    L.HS = slot_tier(d->H);
    L.nw = (d->B + kTile - 1) / kTile;
    constexpr int kPad = kFwdWaves > kBwdWaves ? kFwdWaves : kBwdWaves;
    L.nw_pad = (L.nw + kPad - 1) / kPad * kPad;  // covers both launch geometries
    size_t off = 0;
    auto take = [&](size_t bytes) {
        const size_t o = off;
        off += align_up(bytes);
        return o;
    };
    const int HS = L.HS;
    for (int l = 0; l < kLayers; ++l) L.fa[l] = take(f16_fwd_bytes(HS, l));
    if (with_backward)
        for (int l = 0; l < kLayers; ++l) L.img[l] = take(img_bytes(HS, l));
    L.fcp = take(sizeof(float) * kOut * HS * 4);
    L.fcb = take(sizeof(float) * kOut);
    L.fnp = take(sizeof(float) * kMS * 4 * kFnpStride);
    L.wsc = take(sizeof(float) * 8);
    L.rng = take(sizeof(float) * 8 * kRangeBlocks);
    L.xhat = take(sizeof(float) * (size_t)d->B * d->N * kOut);
    L.loss_part = take(sizeof(float) * L.nw_pad);
    L.dv = take(sizeof(float) * (size_t)d->B * d->N);
    L.ctrl_blocks = (int)(((long long)d->B * d->N + kCtrlItems - 1) / kCtrlItems);
    L.fnn_part = take(sizeof(float) * (size_t)L.ctrl_blocks * d->ctrl_hidden * 5);
    // sequence slabs (fcr_common.h): h of every cell always (layers 0, 1 are the next phase's input);
    // c, the window rows and the backward's dx / window-row-gradient slabs only with a backward
    const size_t qcells = (size_t)L.nw_pad * d->N * kLayers * kL * HS * 16;   // Geo<HS>::QC per cell
    L.hseq = take(sizeof(f32x4) * qcells);
    if (with_backward) {
        L.cseq = take(sizeof(f32x4) * qcells);
        L.xw = take(sizeof(f32x2) * (size_t)L.nw_pad * d->N * kL * kWave);
        L.dseq = take(sizeof(f32x4) * (size_t)L.nw_pad * d->N * 2 * kL * HS * 16);
        // the small-batch backward keeps one copy per wave of its group (fcr_small.h)
        const size_t rows_waves = L.nw_pad > 4 * L.nw ? L.nw_pad : 4 * L.nw;
        L.dxrow = take(sizeof(f32x2) * rows_waves * d->N * kL * kWave);
    }
#if FCR_STAMP
    L.stamp = take(sizeof(unsigned long long) * L.nw_pad * 16);   // [backward 8 | forward 8] per wave
#endif
    if (L.nw <= kPipeMaxGroups) {
        L.pipe_flags = take(sizeof(unsigned) * (size_t)L.nw * kPipeFlags);
        L.pipe_rows = take(sizeof(float) * (size_t)L.nw * d->N * kTile * kPipeRow);
    }
    L.total = off;
    return L;
}

Packed packed_ptrs(const Layout &L, char *ws) {
    Packed p;
    for (int l = 0; l < kLayers; ++l) {
        p.fa[l] = (const float *)(ws + L.fa[l]);
        p.img[l] = (const float *)(ws + L.img[l]);
    }
    p.fcp = (const float *)(ws + L.fcp);
    p.fcb = (const float *)(ws + L.fcb);
    p.fnp = (const float *)(ws + L.fnp);
    p.wsc = (const float *)(ws + L.wsc);
    return p;
}

template <int HS, bool STORE, bool LP>
int launch_fwd_t(const FwdArgs &fa, const Layout &L, hipStream_t s) {
    const int lds = LP ? Geo16<HS>::LDS_FWD_LP : Geo16<HS>::LDS_FWD;
    static std::atomic<unsigned long long> attr_done{0};
    if (const int rc = lds_attr((const void *)fcr_fwd_kernel<HS, STORE, LP>, lds, attr_done, "fwd")) return rc;
    hipLaunchKernelGGL((fcr_fwd_kernel<HS, STORE, LP>), dim3(L.nw_pad / kFwdWaves), dim3(kFwdWaves * kWave),
                       lds, s, fa);
    return launch_check("fcr_fwd_kernel");
}

template <int HS>
int launch_fwd(const FwdArgs &fa, const Layout &L, bool lp, hipStream_t s) {
    if (lp) return fa.cseq ? launch_fwd_t<HS, true, true>(fa, L, s) : launch_fwd_t<HS, false, true>(fa, L, s);
    return fa.cseq ? launch_fwd_t<HS, true, false>(fa, L, s) : launch_fwd_t<HS, false, false>(fa, L, s);
}

template <int HS, bool LP>
int launch_bwd_t(const BwdArgs &ba, const Layout &L, hipStream_t s) {
    const int lds = BwdLds<HS, LP>::BYTES;
    static std::atomic<unsigned long long> attr_done{0};
    if (const int rc = lds_attr((const void *)fcr_bwd_kernel<HS, LP>, lds, attr_done, "bwd")) return rc;
    hipLaunchKernelGGL((fcr_bwd_kernel<HS, LP>), dim3(L.nw_pad / kBwdWaves), dim3(kBwdWaves * kWave), lds, s, ba);
    return launch_check("fcr_bwd_kernel");
}

template <int HS>
int launch_bwd(const BwdArgs &ba, const Layout &L, bool lp, hipStream_t s) {
    return lp ? launch_bwd_t<HS, true>(ba, L, s) : launch_bwd_t<HS, false>(ba, L, s);
}

// Small-batch kernels (fcr_small.h): one workgroup of ceil(HS/4) waves per 16-trajectory group.
// Used for the fp32-accurate mode at HS = 8, 13 when B <= the call's small-batch limit (fcr_options; the
// process-wide default g_small_max_batch when it inherits): below one wave per SIMD the fused kernels run at one
// wave's sequential latency. A change between a forward and its backward is harmless: both families keep one
// workspace layout, and a mixed pair is valid (tested).
std::atomic<int> g_small_max_batch{8192};
int small_limit_of(const fcr_options *o) {
    return (o && o->small_batch_limit >= 0) ? o->small_batch_limit : g_small_max_batch.load(std::memory_order_relaxed);
}
bool use_small(const fcr_dims *d, const Layout &L, const fcr_options *o) {
    return d->precision == FCR_PRECISION_FP32 && (L.HS == 8 || L.HS == 13) && d->B <= small_limit_of(o);
}
void note_kernels(fcr_options *o, int family) {
    if (o) o->kernels = family;
}
// The small-batch family's layer-pipelined geometry (fcr_pipe.h: three workgroups per group that wait on each other)
// for B <= g_pipe_max_batch (default 512; 0 = never): only where every workgroup of the launch is resident at once —
// 3 per group, one per CU by LDS, within half the device's CUs (the other half for whatever else runs).
std::atomic<int> g_pipe_max_batch{512};
int device_cus() {
    static std::atomic<int> cus[64];
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 0;
    int n = cus[dev].load(std::memory_order_relaxed);
    if (n == 0) {
        if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) return 0;
        cus[dev].store(n, std::memory_order_relaxed);
    }
    return n;
}
bool use_pipe(const fcr_dims *d, const Layout &L, const fcr_options *o) {
    return use_small(d, L, o) && d->B <= g_pipe_max_batch.load(std::memory_order_relaxed) && L.nw <= kPipeMaxGroups &&
           6 * L.nw <= device_cus();
}
// window sets per group (fcr_pipe.h): up to `most` (forward 4, backward 3), as many as fit `per` S workgroups per group
// within half the CUs and S <= N; g_pipe_sets > 0 caps it (tests: every S gives the same bits)
std::atomic<int> g_pipe_sets{0};
int pipe_sets(const fcr_dims *d, const Layout &L, int most, int per) {
    const int fixed = g_pipe_sets.load(std::memory_order_relaxed);
    int S = fixed > 0 && fixed < most ? fixed : most;
    const int cus = device_cus();
    while (S > 1 && (2 * per * S * L.nw > cus || S > d->N)) --S;
    return S;
}
PipeArgs pipe_args(const Layout &L, char *base) {
    PipeArgs p;
    p.flags = (unsigned *)(base + L.pipe_flags);
    p.rows = (float *)(base + L.pipe_rows);
    p.groups = L.nw;
    p.loss = nullptr;
    return p;
}
// grid: 2 S (forward) / 3 S (backward) workgroups per group, the ids of a group one residue mod 8 apart (pipe_role)
template <int HS, bool STORE, int S>
int launch_pfwd_t(const FwdArgs &fa, const PipeArgs &pa, const Layout &L, hipStream_t s) {
    constexpr int lds = Pipe<HS>::LDS_FWD;
    static std::atomic<unsigned long long> attr_done{0};
    if (const int rc = lds_attr((const void *)fcr_pfwd_kernel<HS, STORE, S>, lds, attr_done, "pfwd")) return rc;
    // (the counters were zeroed by this call's pack_all_kernel)
    hipLaunchKernelGGL((fcr_pfwd_kernel<HS, STORE, S>), dim3(16 * S * ((L.nw + 7) / 8)), dim3(Small<HS>::NQ * kWave), lds,
                       s, fa, pa);
    return launch_check("fcr_pfwd_kernel");
}
template <int HS, bool STORE>
int launch_pfwd_s(const FwdArgs &fa, const PipeArgs &pa, const Layout &L, int S, hipStream_t s) {
    if (S == 4) return launch_pfwd_t<HS, STORE, 4>(fa, pa, L, s);
    if (S == 3) return launch_pfwd_t<HS, STORE, 3>(fa, pa, L, s);
    if (S == 2) return launch_pfwd_t<HS, STORE, 2>(fa, pa, L, s);
    return launch_pfwd_t<HS, STORE, 1>(fa, pa, L, s);
}
template <int HS, int S>
int launch_pbwd_t(const BwdArgs &ba, const PipeArgs &pa, const Layout &L, hipStream_t s) {
    constexpr int lds = Pipe<HS>::LDS_BWD;
    static std::atomic<unsigned long long> attr_done{0};
    if (const int rc = lds_attr((const void *)fcr_pbwd_kernel<HS, S>, lds, attr_done, "pbwd")) return rc;
    // (the counters were zeroed by the forward's pack_all_kernel; each backward leaves its own zeroed, fcr_pipe.h)
    hipLaunchKernelGGL((fcr_pbwd_kernel<HS, S>), dim3(24 * S * ((L.nw + 7) / 8)), dim3(Small<HS>::NQ * kWave), lds, s, ba,
                       pa);
    return launch_check("fcr_pbwd_kernel");
}
template <int HS>
int launch_pbwd_s(const BwdArgs &ba, const PipeArgs &pa, const Layout &L, int S, hipStream_t s) {
    if (S == 3) return launch_pbwd_t<HS, 3>(ba, pa, L, s);
    if (S == 2) return launch_pbwd_t<HS, 2>(ba, pa, L, s);
    return launch_pbwd_t<HS, 1>(ba, pa, L, s);
}

template <int HS, bool STORE>
int launch_sfwd_t(const FwdArgs &fa, const Layout &L, hipStream_t s) {
    constexpr int lds = Small<HS>::LDS_FWD;
    static std::atomic<unsigned long long> attr_done{0};
    if (const int rc = lds_attr((const void *)fcr_sfwd_kernel<HS, STORE>, lds, attr_done, "sfwd")) return rc;
    hipLaunchKernelGGL((fcr_sfwd_kernel<HS, STORE>), dim3(L.nw), dim3(Small<HS>::NQ * kWave), lds, s, fa);
    return launch_check("fcr_sfwd_kernel");
}

template <int HS>
int launch_sbwd_t(const BwdArgs &ba, const Layout &L, hipStream_t s) {
    constexpr int lds = Small<HS>::LDS_BWD;
    static std::atomic<unsigned long long> attr_done{0};
    if (const int rc = lds_attr((const void *)fcr_sbwd_kernel<HS>, lds, attr_done, "sbwd")) return rc;
    hipLaunchKernelGGL((fcr_sbwd_kernel<HS>), dim3(L.nw), dim3(Small<HS>::NQ * kWave), lds, s, ba);
    return launch_check("fcr_sbwd_kernel");
}

// ---------------------------------------------------------------------------------------------
// H > 52: the batch-wide path (fcr_wide.h, fcr_wgemm.h, fcr_wbwd.h)
// ---------------------------------------------------------------------------------------------
// Every kernel of the rollout's wide path runs at Hp = H padded to whole 64-unit blocks of the forward cell kernel
// (fcr_wgemm.h): the padding units have zero weights in and out, so their gates stay i = f = o = 1/2, g = 0, c = h = 0
// and every product they enter gains exact zeros (the H <= 52 tiers pad the same way, slot_tier). The split weights,
// the readout's fc.W and the window-row gradient's W_ih0 are packed padded per call; the caller's tensors keep H.
int wide_hp(int H) { return (H + kWgU - 1) / kWgU * kWgU; }
// The fused backward cell's column blocks (fcr_wbwd.h): 256 output columns per workgroup in every geometry (WbG256,
// WbG256w). (Round 5 measured 512 columns x 64 trajectories for layers >= 1 — each cell's dgates formed once instead
// of per column block, at twice the A reads per trajectory — 3 % slower at config 5; commit e9dc1d2 builds it with
// -DFCR_WB512=1.)
constexpr int kWbCols = WbG256::kM;
static_assert(WbG256w::kM == kWbCols, "every backward geometry has the same column blocks");
// row-bound slots: one per column block of the writing launch (every block writes its slot, 0 where it has no such
// columns). dh of layer l: its own cells' [0, 2 Hp) (layer 0: [0, Hp)); the input gradient: layer l + 1's [0, Hp)
int wb_hslots(int l, int Hp) { return ((l ? 2 * Hp : Hp) + kWbCols - 1) / kWbCols; }
int wb_dslots(int Hp) { return (Hp + kWbCols - 1) / kWbCols; }
// the slots allocated: the most any geometry writes
int wide_nslots(int Hp) { return (2 * Hp + WbG256::kM - 1) / WbG256::kM; }

struct WideLayout {
    int Hp, ns, keep, ctrl_blocks;
    size_t fcw, fcb, cwi, cbi, cwo, fcp, fcbo, fnp, wsc, rng, xhat, tot, cmd, err, Hs, Cs, WR, HR, total;
    size_t fw[3];   // forward split weights per layer: [2][4Hp][K] (W_hi, W_lo; K = kx + Hp, wide_split_fw_kernel)
    size_t bt[3];   // backward product A per layer: [NO][4Hp / 32][hi 32 | lo 32] (NO = Hp for layer 0, else 2Hp)
    size_t w0p;     // W_ih0 packed [Hp][4][kIn] (the fused layer-0 cell's window-row gradient)
    size_t Act, dH, dC, DC2, D[2], E0, RMc, RMh, RMd, rowg, dv, fnn_part;
    // kept windows (the last `keep` of N): the forward's gate pre-activations and c per cell
    // [keep][3][10][B][4Hp] / [keep][3][10][B][Hp], so the backward skips their recompute (wide_keep_fit)
    size_t KA, KC;
};

WideLayout make_wide(const fcr_dims *d, int with_backward, int keep = 0) {
    WideLayout L{};
    size_t off = 0;
    auto take = [&](size_t bytes) {
        const size_t o = off;
        off += align_up(bytes);
        return o;
    };
    const size_t B = d->B, N = d->N, F = sizeof(float), F16 = sizeof(_Float16);
    const size_t Hp = (size_t)wide_hp(d->H);
    L.Hp = (int)Hp;
    L.ns = wide_nslots((int)Hp);
    L.fcw = take(F * kOut * Hp);
    L.fcb = take(F * kOut);
    L.cwi = take(F * d->ctrl_hidden * kCtrlIn);
    L.cbi = take(F * d->ctrl_hidden);
    L.cwo = take(F * d->ctrl_hidden);
    L.fcp = take(F * kOut * kMaxSlots * 4);
    L.fcbo = take(F * kOut);
    L.fnp = take(F * kMS * 4 * kFnpStride);
    L.wsc = take(F * 8);
    L.rng = take(F * 8 * kRangeBlocks);
    L.xhat = take(F * B * N * kOut);
    L.tot = take(F * B);
    L.cmd = take(F * B);
    L.err = take(F * B);
    L.Hs = take(F * B * Hp);                               // fp32 h of the readout's cell (2, 9)
    L.Cs = take(F * kLayers * kL * B * Hp);                // c of every cell of the current window
    L.WR = take(F16 * kL * B * 2 * kWgRecX0);              // layer 0's window records
    L.HR = take(F16 * 2 * kL * B * 2 * Hp);                // h records of two layers (layer l in slot l & 1)
    for (int l = 0; l < kLayers; ++l) {
        const size_t K = (l == 0 ? kWgRecX0 : Hp) + Hp;
        L.fw[l] = take(F16 * 2 * 4 * Hp * K);
        if (with_backward) L.bt[l] = take(F16 * 2 * (l == 0 ? Hp : 2 * Hp) * 4 * Hp);
    }
    if (with_backward) {
        L.w0p = take(F * Hp * 4 * kIn);
        L.Act = take(F * kLayers * kL * B * 4 * Hp);
        L.dH = take(F * B * Hp);
        L.dC = take(F * B * Hp);
        L.DC2 = take(F * B * Hp);
        L.D[0] = take(F * kL * B * 2 * Hp);   // per t: [input gradient of the layer above | its dh_{t-1}]
        L.D[1] = take(F * kL * B * 2 * Hp);
        L.E0 = take(F * B * Hp);              // layer 0's dh_{t-1}
        L.RMc = take(F * 2 * B);              // [t & 1][B]            row bound of |dc|
        L.RMh = take(F * 2 * L.ns * B);       // [t & 1][slot][B]      of |dh|, per column block of its writer
        L.RMd = take(F * 2 * kL * L.ns * B);  // [l & 1][t][slot][B]   of |input gradient| for the layer below
        L.rowg = take(F * (N + kL - 1) * B * kIn);
        L.dv = take(F * B * N);
        L.ctrl_blocks = (int)(((long long)B * N + kCtrlItems - 1) / kCtrlItems);
        L.fnn_part = take(F * (size_t)L.ctrl_blocks * d->ctrl_hidden * 5);
        if (keep > 0) {
            L.keep = keep;
            L.KA = take(F * (size_t)keep * kLayers * kL * B * 4 * Hp);
            L.KC = take(F * (size_t)keep * kLayers * kL * B * Hp);
        }
    }
    L.total = off;
    return L;
}

// The number of kept windows a workspace of ws_bytes holds (the most that fit): the forward and the
// backward each derive it from the ws_bytes they are given, so they agree with no state between them.
int wide_keep_fit(const fcr_dims *d, size_t ws_bytes) {
    for (int k = d->N; k > 0; --k)
        if (make_wide(d, 1, k).total <= ws_bytes) return k;
    return 0;
}
// a kept window's slabs (window j of the last L.keep)
float *kept_act(const WideLayout &L, char *base, const fcr_dims *d, int j) {
    return (float *)(base + L.KA) + (size_t)(j - (d->N - L.keep)) * kLayers * kL * d->B * 4 * L.Hp;
}
float *kept_c(const WideLayout &L, char *base, const fcr_dims *d, int j) {
    return (float *)(base + L.KC) + (size_t)(j - (d->N - L.keep)) * kLayers * kL * d->B * L.Hp;
}
// fcr_set_wide_keep_budget: bytes of kept windows fcr_workspace_size may add; < 0 = the default policy
// (wide_default_cap). The process-wide default of fcr_options.wide_keep_budget.
std::atomic<long long> g_wide_keep_budget{-1};
long long keep_budget_of(const fcr_options *o) {
    if (o && o->wide_keep_budget != FCR_OPT_INHERIT) return o->wide_keep_budget < 0 ? -1 : o->wide_keep_budget;
    return g_wide_keep_budget.load();
}

// Default cap of a backward-enabled wide workspace: half of the memory that was FREE on the device the first
// time one was sized there (cached per device, so the count does not drift as torch's cache holds the last
// call's workspace), and never more than kWideDefaultFrac of the device's total. Ranks sharing a device each
// see what the others left; what exceeds the cap recomputes instead of keeping (the floor workspace stays).
constexpr double kWideDefaultFrac = 0.40;
long long wide_default_cap() {
    static std::mutex mu;
    static long long cap_of[64];
    static bool have[64];
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) dev = 0;
    std::lock_guard<std::mutex> lk(mu);
    if (!have[dev]) {
        size_t free_b = 0, total_b = 0;
        long long cap = 0;
        if (hipMemGetInfo(&free_b, &total_b) == hipSuccess) {
            cap = (long long)(free_b / 2);
            const long long lim = (long long)((double)total_b * kWideDefaultFrac);
            if (cap > lim) cap = lim;
        }
        cap_of[dev] = cap;
        have[dev] = true;
    }
    return cap_of[dev];
}

// The rollout's per-call packs of the current weights: forward split weights per layer, the backward product's A
// and W_ih0 (with_backward), the readout's fc.W, all at the padded Hp
int wide_pack(const fcr_weights *w, int H, const WideLayout &L, bool backward, char *base, const float *wsc,
              hipStream_t s) {
    const int Hp = L.Hp;
    int rc;
    auto grid = [](size_t n) { return dim3((unsigned)((n + 255) / 256)); };
    for (int l = 0; l < kLayers; ++l) {
        const size_t K = (l == 0 ? kWgRecX0 : Hp) + Hp, n = (size_t)4 * Hp * K;
        _Float16 *fw = (_Float16 *)(base + L.fw[l]);
        hipLaunchKernelGGL(wide_split_fw_kernel, grid(n), dim3(256), 0, s, w->w_ih[l], w->w_hh[l], H, Hp, (int)(l == 0),
                           wsc, fw, fw + n);
        if ((rc = launch_check("wide_split_fw_kernel"))) return rc;
        if (!backward) continue;
        const int NO = l == 0 ? Hp : 2 * Hp;
        const size_t nbt = (size_t)NO * 4 * Hp;
        _Float16 *bt = (_Float16 *)(base + L.bt[l]);
        hipLaunchKernelGGL(wide_split_bt_kernel, grid(nbt), dim3(256), 0, s, l == 0 ? (const float *)nullptr : w->w_ih[l],
                           w->w_hh[l], H, Hp, NO, bt);
        if ((rc = launch_check("wide_split_bt_kernel"))) return rc;
    }
    if (backward) {
        hipLaunchKernelGGL(wide_pack_w0_kernel, grid((size_t)4 * Hp * kIn), dim3(256), 0, s, w->w_ih[0], H, Hp,
                           (float *)(base + L.w0p));
        if ((rc = launch_check("wide_pack_w0_kernel"))) return rc;
    }
    hipLaunchKernelGGL(wide_pad_fc_kernel, grid((size_t)kOut * Hp), dim3(256), 0, s, w->fc_w, H, Hp, (float *)(base + L.fcw));
    return launch_check("wide_pad_fc_kernel");
}

WideArgs wide_args(const fcr_dims *d, const WideLayout &L, char *base) {
    WideArgs a{};
    a.B = d->B;
    a.N = d->N;
    a.H = L.Hp;   // every wide kernel runs at the padded size
    a.CH = d->ctrl_hidden;
    a.alpha = d->alpha;
    a.fcw = (const float *)(base + L.fcw);
    a.fcb = (const float *)(base + L.fcb);
    a.cwi = (const float *)(base + L.cwi);
    a.cbi = (const float *)(base + L.cbi);
    a.cwo = (const float *)(base + L.cwo);
    a.xhat = (float *)(base + L.xhat);
    a.tot = (float *)(base + L.tot);
    a.cmd = (float *)(base + L.cmd);
    a.err = (float *)(base + L.err);
    a.Hs = (float *)(base + L.Hs);
    a.Cs = (float *)(base + L.Cs);
    a.Act = L.Act ? (float *)(base + L.Act) : nullptr;
    a.dH = L.dH ? (float *)(base + L.dH) : nullptr;
    a.dC = L.dC ? (float *)(base + L.dC) : nullptr;
    a.rowg = L.rowg ? (float *)(base + L.rowg) : nullptr;
    a.dv = L.dv ? (float *)(base + L.dv) : nullptr;
    a.wsc = (const float *)(base + L.wsc);
    a.wr = (_Float16 *)(base + L.WR);
    return a;
}

// The per-call weight packs (pack_fwd16_item, pack_img_item, pack_misc_item) as jobs of one launch:
// block ranges in job order, 256 threads each, the same items the separate kernels ran
enum { kPackFwd16 = 0, kPackImg = 1, kPackMisc = 2 };
struct PackJob {
    int kind, l, blocks;
    _Float16 *dst;
};
struct PackAllArgs {
    PackArgs a;
    int njobs;
    PackJob job[2 * kLayers + 1];
    unsigned *clear;   // or null: the pipelined kernels' progress counters, zeroed by block 0 (fcr_pipe.h)
    int nclear;
};
__global__ __launch_bounds__(256) void pack_all_kernel(PackAllArgs p) {
    if (p.clear && blockIdx.x == 0)
        for (int i = (int)threadIdx.x; i < p.nclear; i += 256) p.clear[i] = 0u;
    int b = blockIdx.x, j = 0;
    while (j + 1 < p.njobs && b >= p.job[j].blocks) b -= p.job[j++].blocks;
    const int idx = b * 256 + (int)threadIdx.x;
    const PackJob &jb = p.job[j];
    if (jb.kind == kPackFwd16) pack_fwd16_item(p.a, jb.l, jb.dst, idx);
    else if (jb.kind == kPackImg) pack_img_item(p.a, jb.l, jb.dst, idx);
    else pack_misc_item(p.a, idx);
}

// One forward cell of the wide path: the cell's split-f16 GEMM and update as one hand-written kernel (fcr_wgemm.h)
int launch_wgemm_cell(const WgArgs &wa, hipStream_t s) {
    static std::atomic<unsigned long long> attr_done{0};
    if (const int rc = lds_attr((const void *)wide_cell_fwd_kernel, kWgLds, attr_done, "wgemm")) return rc;
    if (wa.H % kWgU || wa.kx % kWgK || wa.K != wa.kx + wa.H || wa.B <= 0 || !wa.W || !wa.xr || !wa.c_out || !wa.h_rec)
        return fail(FCR_EINVAL, "wide_cell_fwd_kernel: K %d kx %d H %d B %d off its tiling", wa.K, wa.kx, wa.H, wa.B);
    const int nx = (wa.B + kWgN - 1) / kWgN, ny = wa.H / kWgU;
    hipLaunchKernelGGL(wide_cell_fwd_kernel, dim3((unsigned)(nx * ny)), dim3(kWgThreads), kWgLds, s, wa);
    return launch_check("wide_cell_fwd_kernel");
}

// One backward cell of the fused path (fcr_wbwd.h): dgates formed in the product's prologue, out = dG [W_ih | W_hh]
// (columns [0, NO), NO = 0: the dgate part only) in true units. Geometries: layers >= 1 on 256 columns x 256
// trajectories (WbG256w: A staged once per 256 trajectories, backward −5.4 % at config 5, round5_c5_n256_ab_*.log)
// where its halved workgroup count still fills the chip (B >= 32 768: >= 256 workgroups at two column blocks; the
// surrogate's B = 256 step: 3.2 ms on WbG256 against 4.1) and the cell does not also write its dgates (the surrogate's
// B = 65 536 step 2 % slower on it); everything else, layer 0 included, on 256 x 128 (WbG256). (Layer 0 on WbG256w
// spills ~320 registers in its W_ih0 accumulation at the 12-wave budget: backward +57 %, round5_c5_l0w_ab_keepall.log;
// commit e9dc1d2 builds it with -DFCR_WB_L0_N256=1.)
int launch_fb(const WbArgs &wa, bool l0, hipStream_t s) {
    static std::atomic<unsigned long long> attr_done[4] = {{0}, {0}, {0}, {0}};
    const bool w0g = l0 && wa.H > kWbW0LdsUnits;   // layer 0 with W_ih0 read from global memory
    const bool n256 = !l0 && wa.NB >= 32768 && !wa.dg;
    enum { kL1 = 0, kL0 = 1, kL0Global = 2, kL1N256 = 3 };
    const int kind = l0 ? (w0g ? kL0Global : kL0) : (n256 ? kL1N256 : kL1);
    const void *fn = kind == kL1       ? (const void *)wide_bwd_fused_kernel<WbG256, false>
                     : kind == kL0     ? (const void *)wide_bwd_fused_kernel<WbG256, true, false>
                     : kind == kL1N256 ? (const void *)wide_bwd_fused_kernel<WbG256w, false>
                                       : (const void *)wide_bwd_fused_kernel<WbG256, true, true>;
    if (const int rc = lds_attr(fn, kind == kL1N256 ? kWbLds256w : kWbLds256, attr_done[kind], "wbwd")) return rc;
    if (wa.NO < 0 || wa.NO > 2 * wa.H || wa.NO % 8 || wa.H % 8 || wa.NB <= 0 || (wa.rm_h && wa.nrh < 1) ||
        (wa.rm_d && wa.nrd < 1) || (l0 && (!wa.wih0 || !wa.rowg)))
        return fail(FCR_EINVAL, "wide_bwd_fused_kernel: NO %d H %d B %d off its tiling", wa.NO, wa.H, wa.NB);
    const int N = kind == kL1N256 ? WbG256w::kN : WbG256::kN;
    const dim3 grid((unsigned)((wa.NB + N - 1) / N * (wa.NO > 0 ? (wa.NO + kWbCols - 1) / kWbCols : 1)));
    if (kind == kL1N256)
        hipLaunchKernelGGL((wide_bwd_fused_kernel<WbG256w, false>), grid, dim3(WbG256w::kThreads), wb_lds_bytes<WbG256w>(false, wa.H), s, wa);
    else if (kind == kL1)
        hipLaunchKernelGGL((wide_bwd_fused_kernel<WbG256, false>), grid, dim3(WbG256::kThreads), wb_lds_bytes<WbG256>(false, wa.H), s, wa);
    else if (kind == kL0)
        hipLaunchKernelGGL((wide_bwd_fused_kernel<WbG256, true, false>), grid, dim3(WbG256::kThreads), wb_lds_bytes<WbG256>(true, wa.H), s, wa);
    else
        hipLaunchKernelGGL((wide_bwd_fused_kernel<WbG256, true, true>), grid, dim3(WbG256::kThreads), wb_lds_bytes<WbG256>(true, wa.H), s, wa);
    return launch_check("wide_bwd_fused_kernel");
}

// |v| row maxima over the first n columns of B rows of stride ld, or of k8 rows (ld = 0; fcr_wide.h), one wave per
// row: the row bounds fcr_wide_bwd_cell hands the fused backward cell, which the rollout gets from the kernels that
// wrote those rows (the surrogate: its head's dh_9)
__global__ __launch_bounds__(256) void row_absmax_kernel(const float *__restrict__ v, int n, int ld, int B,
                                                         float *__restrict__ out) {
    const int b = blockIdx.x * 4 + (int)(threadIdx.x >> 6), lane = threadIdx.x & 63;
    if (b >= B) return;
    float m = 0.0f;
    for (int i = lane; i < n; i += 64) m = fmaxf(m, fabsf(v[ld ? (size_t)b * ld + i : k8(B, b, i)]));
#pragma unroll
    for (int o = 32; o; o >>= 1) m = fmaxf(m, __shfl_xor(m, o));
    if (lane == 0) out[b] = m;
}

// torch rows [B][ld] (first n columns) <-> k8 rows [n/8][B][8] (fcr_wide.h): the test hook's layout conversion
__global__ void k8_rows_kernel(const float *__restrict__ src, int B, int n, int ld, float *__restrict__ dst, int to_k8) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= (size_t)B * n) return;
    const int b = (int)(i / n), u = (int)(i % n);
    if (to_k8) dst[k8(B, b, u)] = src[(size_t)b * ld + u];
    else dst[(size_t)b * ld + u] = src[k8(B, b, u)];
}

// fcr_wide_bwd_cell (test hook): the scratch of one standalone fused backward cell
struct CellHookLayout {
    size_t bt, w0, rm, rows, total;
};
CellHookLayout cell_hook_layout(int B, int H, int layer0) {
    CellHookLayout L{};
    const size_t NP = layer0 ? H : 2 * (size_t)H;
    L.bt = 0;
    L.w0 = align_up(sizeof(_Float16) * 2 * NP * 4 * H);
    L.rm = L.w0 + align_up(sizeof(float) * 4 * H * kIn);
    L.rows = L.rm + align_up(sizeof(float) * 3 * (size_t)B);   // rm_c [B], rm_h [1][B], rm_d [1][B]
    // k8 copies of c_prev, dh, din, dc, dc_out (B H each) and out (B NP)
    L.total = L.rows + align_up(sizeof(float) * (size_t)B * (5 * (size_t)H + NP));
    return L;
}
int cell_hook_check(int B, int H) {
    if (B < 1) return fail(FCR_EINVAL, "fcr_wide_bwd_cell: B=%d", B);
    if (H < 8 || H % 8 || H > kMaxWideH)
        return fail(FCR_EUNSUPPORTED, "fcr_wide_bwd_cell: H=%d off the fused cell's tiling (a multiple of 8)", H);
    return FCR_OK;
}

// One backward cell of the H > 52 path exactly as wide_backward launches it (launch_fb, fcr_wbwd.h), on caller-given
// inputs: the standalone form the per-element tests of tests/test_wide_cell.py compare with an fp64 product
int wide_bwd_cell_hook(int B, int H, int layer0, const float *w_ih, const float *w_hh, const float *act,
                       const float *c_prev, const float *dh, const float *din, const float *dc, float *out,
                       float *dc_out, float *rowg, char *base, hipStream_t s) {
    const CellHookLayout L = cell_hook_layout(B, H, layer0);
    const int NP = layer0 ? H : 2 * H;
    const size_t nbt = (size_t)NP * 4 * H;
    _Float16 *bt = (_Float16 *)(base + L.bt);
    hipLaunchKernelGGL(wide_split_bt_kernel, dim3((unsigned)((nbt + 255) / 256)), dim3(256), 0, s,
                       layer0 ? (const float *)nullptr : w_ih, w_hh, H, H, NP, bt);
    int rc = launch_check("wide_split_bt_kernel");
    if (rc) return rc;
    float *w0 = (float *)(base + L.w0);
    if (layer0) {
        hipLaunchKernelGGL(wide_pack_w0_kernel, dim3((unsigned)((4 * H * kIn + 255) / 256)), dim3(256), 0, s, w_ih, H, H,
                           w0);
        if ((rc = launch_check("wide_pack_w0_kernel"))) return rc;
    }
    float *rm = (float *)(base + L.rm);
    float *rm_c = rm, *rm_h = rm + B, *rm_d = rm + 2 * (size_t)B;
    const dim3 rg((unsigned)((B + 3) / 4)), rb(256);
    hipLaunchKernelGGL(row_absmax_kernel, rg, rb, 0, s, dc, H, H, B, rm_c);
    hipLaunchKernelGGL(row_absmax_kernel, rg, rb, 0, s, dh, H, H, B, rm_h);
    if (din) hipLaunchKernelGGL(row_absmax_kernel, rg, rb, 0, s, din, H, H, B, rm_d);
    if ((rc = launch_check("row_absmax_kernel"))) return rc;
    // the cell reads and writes k8 rows: the caller's rows are converted around it
    float *rows = (float *)(base + L.rows);
    const size_t cell = (size_t)B * H;
    auto to_k8 = [&](const float *src, float *dst) -> const float * {
        if (!src) return nullptr;
        hipLaunchKernelGGL(k8_rows_kernel, dim3((unsigned)((cell + 255) / 256)), dim3(256), 0, s, src, B, H, H, dst, 1);
        return dst;
    };
    WbArgs wa{};
    wa.A = bt;
    wa.NB = B;
    wa.H = H;
    wa.act = act;
    wa.c_prev = to_k8(c_prev, rows);
    wa.dh = to_k8(dh, rows + cell);
    wa.din = to_k8(din, rows + 2 * cell);
    wa.dC = to_k8(dc, rows + 3 * cell);
    wa.dC_out = rows + 4 * cell;
    if ((rc = launch_check("k8_rows_kernel"))) return rc;
    wa.rm_c = rm_c;
    wa.rm_h = rm_h;
    wa.rm_d = din ? rm_d : nullptr;
    wa.nrh = 1;
    wa.nrd = 1;
    wa.out = rows + 5 * cell;
    if (!layer0) {   // [input gradient | dh_{t-1}] (t = 0, no c_prev: the former only)
        wa.NO = c_prev ? 2 * H : H;
        wa.h0 = H;
        wa.h1 = c_prev ? 2 * H : H;
        wa.d1 = H;
    } else {         // dh_{t-1} (none at t = 0) and the window-row gradient
        if (hipMemsetAsync(rowg, 0, sizeof(float) * kIn * (size_t)B, s) != hipSuccess)
            return fail(FCR_EHIP, "hipMemsetAsync failed");
        wa.NO = c_prev ? H : 0;
        wa.h0 = 0;
        wa.h1 = H;
        wa.d1 = 0;
        wa.wih0 = w0;
        wa.rowg = rowg;
    }
    if ((rc = launch_fb(wa, layer0 != 0, s))) return rc;
    hipLaunchKernelGGL(k8_rows_kernel, dim3((unsigned)((cell + 255) / 256)), dim3(256), 0, s, (const float *)wa.dC_out, B,
                       H, H, dc_out, 0);
    if (wa.NO > 0)
        hipLaunchKernelGGL(k8_rows_kernel, dim3((unsigned)(((size_t)B * wa.NO + 255) / 256)), dim3(256), 0, s,
                           (const float *)wa.out, B, wa.NO, layer0 ? H : 2 * H, out, 0);
    return launch_check("k8_rows_kernel");
}

// One window's 30 cells, forward (the rollout, and the backward's recompute of a window that was not kept): layer by
// layer, t = 0..9, each cell one wide_cell_fwd_kernel launch. keep_act: the cells' gate activations into `Act` (the
// backward's dgates read them, as autograd reads the activations its forward saved).
// fw: the layers' split weights; HR: h records of `slots` layers (layer l in slot l % slots: the rollout keeps two, the
// surrogate all three for its weight gradients)
int wide_cells(const WideArgs &a, const _Float16 *const *fw, _Float16 *HR, int Hp, int slots, bool keep_act,
               hipStream_t s) {
    const int B = a.B;
    const size_t cell = (size_t)B * Hp;
    auto rec = [&](int l, int t) { return HR + ((size_t)(l % slots) * kL + t) * B * 2 * Hp; };   // h record of (l, t)
    int rc;
    for (int l = 0; l < kLayers; ++l) {
        const size_t K = (l == 0 ? kWgRecX0 : Hp) + Hp;
        for (int t = 0; t < kL; ++t) {
            WgArgs wa{};
            wa.W = fw[l];
            wa.K = (int)K;
            wa.kx = l == 0 ? kWgRecX0 : Hp;
            wa.xr = l == 0 ? a.wr + (size_t)t * B * 2 * kWgRecX0 : rec(l - 1, t);
            wa.hr = t > 0 ? rec(l, t - 1) : nullptr;
            wa.B = B;
            wa.H = Hp;
            wa.c_prev = t > 0 ? a.Cs + ((size_t)l * kL + t - 1) * cell : nullptr;
            wa.c_out = a.Cs + ((size_t)l * kL + t) * cell;
            wa.h_out = (l == kLayers - 1 && t == kL - 1) ? a.Hs : nullptr;
            wa.act = keep_act ? a.Act + ((size_t)l * kL + t) * cell * 4 : nullptr;
            wa.h_rec = rec(l, t);
            if ((rc = launch_wgemm_cell(wa, s))) return rc;
        }
    }
    return FCR_OK;
}

// the rollout's window cells (two record slots)
int wide_window_cells(const WideArgs &a, const WideLayout &L, char *base, bool keep_act, hipStream_t s) {
    const _Float16 *fw[kLayers];
    for (int l = 0; l < kLayers; ++l) fw[l] = (const _Float16 *)(base + L.fw[l]);
    return wide_cells(a, fw, (_Float16 *)(base + L.HR), L.Hp, 2, keep_act, s);
}

int wide_forward(const fcr_dims *d, const fcr_weights *w, const float *X, const float *u0, const float *states,
                 const float *noise, float *loss, float *cost, float *command, float *error, float *prediction,
                 float *xhat, int with_backward, char *base, size_t ws_bytes, hipStream_t s) {
    const WideLayout L = make_wide(d, with_backward, with_backward ? wide_keep_fit(d, ws_bytes) : 0);
    const size_t F = sizeof(float);
    int rc;
    // private copies of every parameter the backward needs (fcr_backward takes no weights)
    auto cp = [&](size_t off, const float *src, size_t n) {
        return hipMemcpyAsync(base + off, src, n * F, hipMemcpyDeviceToDevice, s);
    };
    if (cp(L.fcb, w->fc_b, kOut) || cp(L.cwi, w->ctrl_w_inp, d->ctrl_hidden * kCtrlIn) ||
        cp(L.cbi, w->ctrl_b_inp, d->ctrl_hidden) || cp(L.cwo, w->ctrl_w_out, d->ctrl_hidden))
        return fail(FCR_EHIP, "hipMemcpyAsync (parameters) failed");
    PackArgs pa{};   // controller records for ctrl_grad_kernel (the fc part is unused on this path)
    pa.H = kMaxSlots * 4;
    pa.HS = kMaxSlots;
    pa.CH = d->ctrl_hidden;
    pa.fcw = w->fc_w;   // read only for units < 52 < H: in bounds
    pa.fcb = w->fc_b;
    pa.cwi = w->ctrl_w_inp;
    pa.cbi = w->ctrl_b_inp;
    pa.cwo = w->ctrl_w_out;
    pa.fcp = (float *)(base + L.fcp);
    pa.fcbo = (float *)(base + L.fcbo);
    pa.fnp = (float *)(base + L.fnp);
    hipLaunchKernelGGL(pack_misc_kernel, dim3(2), dim3(256), 0, s, pa);
    if ((rc = launch_check("pack_misc_kernel"))) return rc;
    if ((rc = launch_range(d, states, u0, noise, w->fc_w, w->fc_b, (float *)(base + L.rng), (float *)(base + L.wsc), s)))
        return rc;
    if ((rc = wide_pack(w, d->H, L, with_backward != 0, base, (const float *)(base + L.wsc), s))) return rc;
    WideArgs a = wide_args(d, L, base);
    a.X = X;
    a.u0 = u0;
    a.states = states;
    a.noise = noise;
    a.pred = prediction;
    const int nb = (d->B + 255) / 256;
    for (int j = 0; j < d->N; ++j) {
        hipLaunchKernelGGL(wide_window_kernel<true>, dim3(nb), dim3(256), 0, s, a, j);
        if ((rc = launch_check("wide_window_kernel"))) return rc;
        if (j >= d->N - L.keep) {   // kept window: pre-activations and c into its own slabs for the backward
            WideArgs ak = a;
            ak.Act = kept_act(L, base, d, j);
            ak.Cs = kept_c(L, base, d, j);
            if ((rc = wide_window_cells(ak, L, base, true, s))) return rc;
        } else if ((rc = wide_window_cells(a, L, base, false, s))) {
            return rc;
        }
        hipLaunchKernelGGL(wide_readout_kernel, dim3((unsigned)(((size_t)d->B * kRoLanes + 255) / 256)), dim3(256), 0, s, a, j,
                           (const float *)a.Hs);
        if ((rc = launch_check("wide_readout_kernel"))) return rc;
    }
    hipLaunchKernelGGL(wide_finish_kernel, dim3(nb), dim3(256), 0, s, a, cost, command, error, xhat);
    if ((rc = launch_check("wide_finish_kernel"))) return rc;
    hipLaunchKernelGGL(loss_reduce_kernel, dim3(1), dim3(256), 0, s, (const float *)cost, d->B, d->B, loss);
    return launch_check("loss_reduce_kernel");
}

int wide_backward(const fcr_dims *d, const float *X, const float *states, const float *prediction,
                  const float *dloss, float *g_u0, float *g_w_inp, float *g_b_inp, float *g_w_out, char *base,
                  size_t ws_bytes, hipStream_t s) {
    const WideLayout L = make_wide(d, 1, wide_keep_fit(d, ws_bytes));
    const int B = d->B, Hp = L.Hp, ns = L.ns, nd = wb_dslots(Hp);
    const size_t cell = (size_t)B * Hp;
    const int nb = (B + 255) / 256;
    int rc;
    WideArgs a = wide_args(d, L, base);
    a.X = X;
    a.states = states;
    a.pred = (float *)prediction;
    a.dloss = dloss;
    float *D[2] = {(float *)(base + L.D[0]), (float *)(base + L.D[1])};
    float *E0 = (float *)(base + L.E0);
    if (hipMemsetAsync(a.rowg, 0, sizeof(float) * (size_t)(d->N + kL - 1) * B * kIn, s) != hipSuccess)
        return fail(FCR_EHIP, "hipMemsetAsync failed");
    float *DC[2] = {a.dC, (float *)(base + L.DC2)};
    float *RMc = (float *)(base + L.RMc);
    float *RMh = (float *)(base + L.RMh);
    float *RMd = (float *)(base + L.RMd);
    for (int j = d->N - 1; j >= 0; --j) {
        hipLaunchKernelGGL(wide_head_kernel, dim3((unsigned)(((size_t)B * kRoLanes + 255) / 256)), dim3(256), 0, s, a, j,
                           RMh);   // slot 0 of parity (9 + 1) & 1 = 0: layer 2's t = 9 reads it
        if ((rc = launch_check("wide_head_kernel"))) return rc;
        if (j >= d->N - L.keep) {   // kept by the forward: no recompute
            a.Act = kept_act(L, base, d, j);
            a.Cs = kept_c(L, base, d, j);
        } else {
            a.Act = (float *)(base + L.Act);
            a.Cs = (float *)(base + L.Cs);
            hipLaunchKernelGGL(wide_window_kernel<false>, dim3(nb), dim3(256), 0, s, a, j);
            if ((rc = launch_check("wide_window_kernel"))) return rc;
            if ((rc = wide_window_cells(a, L, base, true, s))) return rc;   // checkpoint: recompute the window
        }
        for (int l = kLayers - 1; l >= 0; --l) {
            for (int t = kL - 1; t >= 0; --t) {
                const size_t c_off = ((size_t)l * kL + t) * cell;
                // dh_t below t = 9 comes from cell t+1's product: layer 0 columns 0..Hp-1 of E0, layers >= 1 columns
                // Hp..2Hp-1 of D[l-1] row t+1; the layer above's input gradient from D[l] row t
                // (t = 9: the head's dh for layer 2, zero below it, passed as null like the zero dc_9 and their bounds)
                const bool top9 = t == kL - 1 && l == kLayers - 1, zero9 = t == kL - 1 && l < kLayers - 1;
                // (D rows are k8 rows of 2Hp columns: column Hp starts at + Hp B = + cell)
                const float *dh_src = top9 ? a.dH : zero9 ? nullptr : l == 0 ? E0 : D[l - 1] + (size_t)(t + 1) * 2 * cell + cell;
                WbArgs wa{};
                wa.A = (const _Float16 *)(base + L.bt[l]);
                wa.NB = B;
                wa.H = Hp;
                wa.act = a.Act + c_off * 4;
                wa.c_prev = t > 0 ? a.Cs + c_off - cell : nullptr;
                wa.dh = dh_src;
                wa.din = l < kLayers - 1 ? D[l] + (size_t)t * 2 * cell : nullptr;
                wa.dC = t == kL - 1 ? nullptr : DC[(t + 1) & 1];   // t writes buffer t & 1
                wa.dC_out = DC[t & 1];
                wa.rm_c = t == kL - 1 ? nullptr : RMc + (size_t)((t + 1) & 1) * B;
                wa.rm_c_out = t > 0 ? RMc + (size_t)(t & 1) * B : nullptr;
                // dh's bound: the head's one slot at t = 9 (none below layer 2), else the column blocks of cell t + 1's
                // product
                wa.rm_h = zero9 ? nullptr : RMh + (size_t)((t + 1) & 1) * ns * B;
                wa.nrh = t == kL - 1 ? 1 : wb_hslots(l, Hp);
                wa.rm_h_out = t > 0 ? RMh + (size_t)(t & 1) * ns * B : nullptr;
                wa.rm_d = l < kLayers - 1 ? RMd + ((size_t)((l + 1) & 1) * kL + t) * ns * B : nullptr;
                wa.nrd = nd;
                wa.rm_d_out = l > 0 ? RMd + ((size_t)(l & 1) * kL + t) * ns * B : nullptr;
                if (l > 0) {   // [input gradient | dh_{t-1}] (t = 0: the former only) into D[l-1] row t
                    wa.out = D[l - 1] + (size_t)t * 2 * cell;
                    wa.NO = t > 0 ? 2 * Hp : Hp;
                    wa.h0 = Hp;
                    wa.h1 = t > 0 ? 2 * Hp : Hp;
                    wa.d1 = Hp;
                } else {       // dh_{t-1} into E0 (t = 0: none), and the window-row gradient into rowg row j + t
                    wa.out = E0;
                    wa.NO = t > 0 ? Hp : 0;
                    wa.h0 = 0;
                    wa.h1 = Hp;
                    wa.d1 = 0;
                    wa.wih0 = (const float *)(base + L.w0p);
                    wa.rowg = a.rowg + (size_t)(j + t) * B * kIn;
                }
                if ((rc = launch_fb(wa, l == 0, s))) return rc;
            }
        }
    }
    hipLaunchKernelGGL(wide_gu0_kernel, dim3(nb), dim3(256), 0, s, a, g_u0);
    if ((rc = launch_check("wide_gu0_kernel"))) return rc;
    float *part = (float *)(base + L.fnn_part);
    const bool one = L.ctrl_blocks == 1;   // one block writes the gradients itself (grad_out5)
    hipLaunchKernelGGL(ctrl_grad_kernel, dim3(L.ctrl_blocks), dim3(kCtrlBlock), 0, s, X, (const float *)a.xhat,
                       (const float *)a.dv, (const float *)(base + L.fnp), d->B, d->N, d->ctrl_hidden, part,
                       one ? g_w_inp : nullptr, one ? g_b_inp : nullptr, one ? g_w_out : nullptr);
    if ((rc = launch_check("ctrl_grad_kernel"))) return rc;
    if (one) return FCR_OK;
    hipLaunchKernelGGL(grad_reduce_kernel, dim3(d->ctrl_hidden * 5), dim3(256), 0, s, (const float *)part,
                       L.ctrl_blocks, d->ctrl_hidden, g_w_inp, g_b_inp, g_w_out);
    return launch_check("grad_reduce_kernel");
}

// ------------------------------------------------------------------------------------------------
// LSTM surrogate training step: LSTMModel forward on a window batch and the
// backward of ALL its weights (Model_NN/Functions.py:520-569), on the per-cell path.

int check_lstm_dims(const fcr_dims *d) {
    if (!d) return fail(FCR_EINVAL, "dims is NULL");
    if (d->B < 1) return fail(FCR_EINVAL, "B=%d must be >= 1", d->B);
    if (d->L != kL) return fail(FCR_EUNSUPPORTED, "L=%d: the window is fixed at 10 rows", d->L);
    if (d->layers != kLayers) return fail(FCR_EUNSUPPORTED, "layers=%d: built for 3", d->layers);
    if (d->in_dim != kIn || d->out_dim != kOut)
        return fail(FCR_EUNSUPPORTED, "in/out = %d/%d: built for 5/4", d->in_dim, d->out_dim);
    if (d->H < 1 || d->H > kMaxWideH) return fail(FCR_EUNSUPPORTED, "H=%d: built for 1..%d", d->H, kMaxWideH);
    if ((long long)d->B * kL * 4 * d->H > (1LL << 40)) return fail(FCR_EINVAL, "B*H too large");
    return FCR_OK;
}

// H > 52: the surrogate's step on the rollout's wide kernels (no vendor library): the forward cells of fcr_wgemm.h
// over the window batch (every cell's activations, c and h records kept), the fused backward cells of fcr_wbwd.h
// (which also write each cell's dgates), and the weight gradients as reductions over all 10 B (step, sample) rows
// on the fp32 matrix cores (fcr_wgrad.h). Hidden size padded to Hp as on the rollout's wide path.
struct SurWideLayout {
    int Hp, ns;
    size_t fcw, wsc, rng, xt, WR, HR, Cs, Act, Hs, fw[3], bt[3], w0p, dH, dC, DC2, D[2], E0, RMc, RMh, RMd, rowg, dG,
        fcpart, part, part_floats, total;
};
constexpr int kSurFcSlices = 64;   // batch slices of the readout's weight gradient (fixed: deterministic)

// n slices of one weight-gradient reduction: enough workgroups to fill the chip, whole kWgrN steps per slice
struct WgSplit {
    int S;
    long long n_per;
};
WgSplit wg_split(long long n, int R, int K) {
    // K <= kWgrSmallK (wgrad_small_kernel): one thread per row r, so many n slices for parallelism
    const bool small = K <= kWgrSmallK;
    const long long tiles = small ? (R + 255) / 256 : (long long)((R + kWgrT - 1) / kWgrT) * ((K + kWgrT - 1) / kWgrT);
    long long S = ((small ? 2048 : 512) + tiles - 1) / tiles;
    S = S < 1 ? 1 : (S > (small ? 1024 : 64) ? (small ? 1024 : 64) : S);
    long long per = (n + S - 1) / S;
    per = (per + kWgrN - 1) / kWgrN * kWgrN;
    return {(int)((n + per - 1) / per), per};
}

SurWideLayout make_surw(const fcr_dims *d, int with_backward) {
    SurWideLayout L{};
    size_t off = 0;
    auto take = [&](size_t bytes) {
        const size_t o = off;
        off += align_up(bytes);
        return o;
    };
    const size_t B = d->B, F = sizeof(float), F16 = sizeof(_Float16), Hp = (size_t)wide_hp(d->H);
    L.Hp = (int)Hp;
    L.ns = wide_nslots((int)Hp);
    L.fcw = take(F * kOut * Hp);
    L.wsc = take(F * 8);
    L.rng = take(F * 8 * kRangeBlocks);
    L.xt = take(F * kL * B * kIn);
    L.WR = take(F16 * kL * B * 2 * kWgRecX0);
    L.HR = take(F16 * kLayers * kL * B * 2 * Hp);
    L.Cs = take(F * kLayers * kL * B * Hp);
    // the gate activations only for the backward (the forward-only call's cells run with keep_act off)
    L.Act = with_backward ? take(F * kLayers * kL * B * 4 * Hp) : 0;
    L.Hs = take(F * B * Hp);
    for (int l = 0; l < kLayers; ++l) {
        L.fw[l] = take(F16 * 2 * 4 * Hp * ((l == 0 ? kWgRecX0 : Hp) + Hp));
        if (with_backward) L.bt[l] = take(F16 * 2 * (l == 0 ? Hp : 2 * Hp) * 4 * Hp);
    }
    if (with_backward) {
        L.w0p = take(F * Hp * 4 * kIn);
        L.dH = take(F * B * Hp);
        L.dC = take(F * B * Hp);
        L.DC2 = take(F * B * Hp);
        L.D[0] = take(F * kL * B * 2 * Hp);
        L.D[1] = take(F * kL * B * 2 * Hp);
        L.E0 = take(F * B * Hp);
        L.RMc = take(F * 2 * B);
        L.RMh = take(F * 2 * L.ns * B);
        L.RMd = take(F * 2 * kL * L.ns * B);
        L.rowg = take(F * kL * B * kIn);
        L.dG = take(F * kL * B * 4 * Hp);   // one layer's dgates, every step
        L.fcpart = take(F * kSurFcSlices * kOut * Hp);
        // the largest set of weight-gradient partials over every reduction surw_backward runs: n = 10 B rows (W_ih)
        // and 9 B rows (W_hh), K = kIn (layer 0's W_ih) and H. wg_split rounds each slice up to whole kWgrN steps,
        // so the 9 B reduction can take MORE slices than the 10 B one (H = 256, B = 110: 31 against 18)
        size_t pf = 0;
        for (long long n : {(long long)kL * B, (long long)(kL - 1) * B})
            for (int K : {kIn, d->H}) {
                const WgSplit w = wg_split(n, 4 * (int)Hp, K);
                const size_t a = (size_t)w.S * 4 * Hp * K;
                pf = a > pf ? a : pf;
            }
        L.part = take(F * pf);
        L.part_floats = pf;
    }
    L.total = off;
    return L;
}

int surw_forward(const fcr_dims *d, const fcr_weights *w, const float *x, float *y, int with_backward, char *base,
                 hipStream_t s) {
    const SurWideLayout L = make_surw(d, with_backward);
    const int B = d->B, Hp = L.Hp;
    int rc;
    // range guard of the window columns from the batch itself (as the H <= 52 step: u0 = x, fcr_pack.h)
    if ((rc = launch_range(d, x, x, nullptr, w->fc_w, w->fc_b, (float *)(base + L.rng), (float *)(base + L.wsc), s)))
        return rc;
    hipLaunchKernelGGL(sur_window_rec_kernel, dim3((unsigned)((B * kL + 255) / 256)), dim3(256), 0, s, x,
                       (const float *)(base + L.wsc), B, (_Float16 *)(base + L.WR), (float *)(base + L.xt));
    if ((rc = launch_check("sur_window_rec_kernel"))) return rc;
    auto grid = [](size_t n) { return dim3((unsigned)((n + 255) / 256)); };
    const _Float16 *fw[kLayers];
    for (int l = 0; l < kLayers; ++l) {
        const size_t K = (l == 0 ? kWgRecX0 : Hp) + Hp, n = (size_t)4 * Hp * K;
        _Float16 *p = (_Float16 *)(base + L.fw[l]);
        hipLaunchKernelGGL(wide_split_fw_kernel, grid(n), dim3(256), 0, s, w->w_ih[l], w->w_hh[l], d->H, Hp, (int)(l == 0),
                           (const float *)(base + L.wsc), p, p + n);
        if ((rc = launch_check("wide_split_fw_kernel"))) return rc;
        fw[l] = p;
    }
    hipLaunchKernelGGL(wide_pad_fc_kernel, grid((size_t)kOut * Hp), dim3(256), 0, s, w->fc_w, d->H, Hp, (float *)(base + L.fcw));
    if ((rc = launch_check("wide_pad_fc_kernel"))) return rc;
    WideArgs a{};
    a.B = B;
    a.N = 1;
    a.H = Hp;
    a.Cs = (float *)(base + L.Cs);
    a.Act = with_backward ? (float *)(base + L.Act) : nullptr;
    a.Hs = (float *)(base + L.Hs);
    a.wr = (_Float16 *)(base + L.WR);
    if ((rc = wide_cells(a, fw, (_Float16 *)(base + L.HR), Hp, kLayers, with_backward != 0, s))) return rc;
    hipLaunchKernelGGL(surrogate::readout_kernel, dim3((B + 255) / 256), dim3(256), 0, s, (const float *)a.Hs,
                       (const float *)(base + L.fcw), w->fc_b, y, B, Hp);
    return launch_check("readout_kernel");
}

// one weight gradient: dW [4H][K] = sum_n A[n][.] X[n][.] (fcr_wgrad.h), X fp32 rows or split records
int surw_wgrad(const float *A, long long n, int Hp, int H, int K, const float *X, int ldx, const _Float16 *XR,
               float *part, size_t part_floats, float *dW, hipStream_t s) {
    const WgSplit sp = wg_split(n, 4 * Hp, K);
    if ((size_t)sp.S * 4 * Hp * K > part_floats)   // make_surw sizes L.part for every (n, K) this runs with
        return fail(FCR_EWORKSPACE, "surrogate weight-gradient partials exceed their workspace slab");
    WgradArgs g{};
    g.A = A;
    g.lda = 4 * Hp;
    g.X = X;
    g.XR = XR;
    g.ldx = ldx;
    g.Hx = Hp;
    g.n = n;
    g.R = 4 * Hp;
    g.K = K;
    g.n_per = sp.n_per;
    g.part = part;
    int rc;
    if (K <= kWgrSmallK && X) {
        hipLaunchKernelGGL(wgrad_small_kernel, dim3((unsigned)((4 * Hp + 255) / 256), (unsigned)sp.S), dim3(256), 0, s, g);
        rc = launch_check("wgrad_small_kernel");
    } else {
        static std::atomic<unsigned long long> attr_done{0};
        if ((rc = lds_attr((const void *)wgrad_kernel, kWgrLds, attr_done, "wgrad"))) return rc;
        hipLaunchKernelGGL(wgrad_kernel, dim3((unsigned)((4 * Hp + kWgrT - 1) / kWgrT), (unsigned)((K + kWgrT - 1) / kWgrT),
                                              (unsigned)sp.S),
                           dim3(kWgrThreads), kWgrLds, s, g);
        rc = launch_check("wgrad_kernel");
    }
    if (rc) return rc;
    const long long e = (long long)4 * H * K;
    hipLaunchKernelGGL(wgrad_sum_pad_kernel, dim3((unsigned)((e + 255) / 256)), dim3(256), 0, s, (const float *)part, sp.S,
                       H, Hp, K, dW);
    return launch_check("wgrad_sum_pad_kernel");
}

int surw_backward(const fcr_dims *d, const fcr_weights *w, const float *dy, float *const *g_w_ih, float *const *g_w_hh,
                  float *g_fc_w, float *g_fc_b, float *g_x, char *base, hipStream_t s) {
    const SurWideLayout L = make_surw(d, 1);
    const int B = d->B, H = d->H, Hp = L.Hp, ns = L.ns, nd = wb_dslots(Hp);
    const size_t cell = (size_t)B * Hp;
    int rc;
    auto grid = [](size_t n) { return dim3((unsigned)((n + 255) / 256)); };
    // the backward's packs (the forward's split weights and padded fc.W are still in ws)
    for (int l = 0; l < kLayers; ++l) {
        const int NO = l == 0 ? Hp : 2 * Hp;
        const size_t nbt = (size_t)NO * 4 * Hp;
        _Float16 *bt = (_Float16 *)(base + L.bt[l]);
        hipLaunchKernelGGL(wide_split_bt_kernel, grid(nbt), dim3(256), 0, s, l == 0 ? (const float *)nullptr : w->w_ih[l],
                           w->w_hh[l], H, Hp, NO, bt);
        if ((rc = launch_check("wide_split_bt_kernel"))) return rc;
    }
    hipLaunchKernelGGL(wide_pack_w0_kernel, grid((size_t)4 * Hp * kIn), dim3(256), 0, s, w->w_ih[0], H, Hp,
                       (float *)(base + L.w0p));
    if ((rc = launch_check("wide_pack_w0_kernel"))) return rc;
    const float *Hs = (const float *)(base + L.Hs), *fcw = (const float *)(base + L.fcw);
    // readout: d fc.W = dy^T h_9 (fixed batch slices), d fc.b = sum dy, dh_9 = dy fc.W (its row bound: slot 0)
    const int b_per = (B + kSurFcSlices - 1) / kSurFcSlices;
    float *fcpart = (float *)(base + L.fcpart);
    hipLaunchKernelGGL(fc_wgrad_part_kernel, dim3((unsigned)((Hp + 255) / 256), kSurFcSlices), dim3(256), 0, s, dy, Hs, B,
                       Hp, b_per, fcpart);
    hipLaunchKernelGGL(fc_wgrad_sum_kernel, grid((size_t)kOut * H), dim3(256), 0, s, (const float *)fcpart,
                       kSurFcSlices, H, Hp, g_fc_w);
    hipLaunchKernelGGL(surrogate::bias_grad_kernel, dim3(kOut), dim3(surrogate::kSurBlock), 0, s, dy, g_fc_b, B);
    float *dH = (float *)(base + L.dH);
    float *RMc = (float *)(base + L.RMc), *RMh = (float *)(base + L.RMh), *RMd = (float *)(base + L.RMd);
    hipLaunchKernelGGL(sur_head_kernel, grid(cell), dim3(256), 0, s, dy, fcw, B, Hp, dH);
    hipLaunchKernelGGL(row_absmax_kernel, dim3((unsigned)((B + 3) / 4)), dim3(256), 0, s, (const float *)dH, Hp, 0, B, RMh);
    if ((rc = launch_check("readout backward"))) return rc;
    float *D[2] = {(float *)(base + L.D[0]), (float *)(base + L.D[1])};
    float *DC[2] = {(float *)(base + L.dC), (float *)(base + L.DC2)};
    float *E0 = (float *)(base + L.E0), *rowg = (float *)(base + L.rowg), *dG = (float *)(base + L.dG);
    float *part = (float *)(base + L.part);
    const float *Cs = (const float *)(base + L.Cs), *Act = (const float *)(base + L.Act);
    const _Float16 *HR = (const _Float16 *)(base + L.HR);
    if (hipMemsetAsync(rowg, 0, sizeof(float) * kL * B * kIn, s) != hipSuccess) return fail(FCR_EHIP, "hipMemsetAsync failed");
    for (int l = kLayers - 1; l >= 0; --l) {
        for (int t = kL - 1; t >= 0; --t) {   // the rollout's backward cells (wide_backward), one window
            const size_t c_off = ((size_t)l * kL + t) * cell;
            WbArgs wa{};
            wa.A = (const _Float16 *)(base + L.bt[l]);
            wa.NB = B;
            wa.H = Hp;
            wa.act = Act + c_off * 4;
            wa.c_prev = t > 0 ? Cs + c_off - cell : nullptr;
            const bool zero9 = t == kL - 1 && l < kLayers - 1;   // dh_9 below the top layer: zero (null)
            wa.dh = t == kL - 1 ? (zero9 ? nullptr : dH) : l == 0 ? E0 : D[l - 1] + (size_t)(t + 1) * 2 * cell + cell;
            wa.din = l < kLayers - 1 ? D[l] + (size_t)t * 2 * cell : nullptr;
            wa.dC = t == kL - 1 ? nullptr : DC[(t + 1) & 1];
            wa.dC_out = DC[t & 1];
            wa.rm_c = t == kL - 1 ? nullptr : RMc + (size_t)((t + 1) & 1) * B;
            wa.rm_c_out = t > 0 ? RMc + (size_t)(t & 1) * B : nullptr;
            wa.rm_h = zero9 ? nullptr : RMh + (size_t)((t + 1) & 1) * ns * B;
            wa.nrh = t == kL - 1 ? 1 : wb_hslots(l, Hp);
            wa.rm_h_out = t > 0 ? RMh + (size_t)(t & 1) * ns * B : nullptr;
            wa.rm_d = l < kLayers - 1 ? RMd + ((size_t)((l + 1) & 1) * kL + t) * ns * B : nullptr;
            wa.nrd = nd;
            wa.rm_d_out = l > 0 ? RMd + ((size_t)(l & 1) * kL + t) * ns * B : nullptr;
            wa.dg = dG + (size_t)t * cell * 4;
            if (l > 0) {
                wa.out = D[l - 1] + (size_t)t * 2 * cell;
                wa.NO = t > 0 ? 2 * Hp : Hp;
                wa.h0 = Hp;
                wa.h1 = t > 0 ? 2 * Hp : Hp;
                wa.d1 = Hp;
            } else {
                wa.out = E0;
                wa.NO = t > 0 ? Hp : 0;
                wa.h0 = 0;
                wa.h1 = Hp;
                wa.d1 = 0;
                wa.wih0 = (const float *)(base + L.w0p);
                wa.rowg = rowg + (size_t)t * B * kIn;   // dL/dx of window row t (the cell's window-row gradient)
            }
            if ((rc = launch_fb(wa, l == 0, s))) return rc;
        }
        // the layer's weight gradients over all (step, sample) rows: x_t = the window rows (layer 0, fp32) or the
        // layer below's h records; h_{t-1} = this layer's records of steps 0..8 against the dgates of steps 1..9
        const long long n10 = (long long)kL * B, n9 = (long long)(kL - 1) * B;
        if ((rc = surw_wgrad(dG, n10, Hp, H, l == 0 ? kIn : H, l == 0 ? (const float *)(base + L.xt) : nullptr, kIn,
                             l == 0 ? nullptr : HR + (size_t)(l - 1) * kL * B * 2 * Hp, part, L.part_floats, g_w_ih[l],
                             s)))
            return rc;
        if ((rc = surw_wgrad(dG + (size_t)B * 4 * Hp, n9, Hp, H, H, nullptr, 0, HR + (size_t)l * kL * B * 2 * Hp, part,
                             L.part_floats, g_w_hh[l], s)))
            return rc;
    }
    if (g_x) {   // the window-row gradients [t][B][5] -> (B, 10, 5)
        const long long nx = (long long)B * kL * kIn;
        hipLaunchKernelGGL(surrogate::window_transpose_kernel, dim3((unsigned)((nx + 255) / 256)), dim3(256), 0, s,
                           (const float *)rowg, g_x, B, kIn, true);
        if ((rc = launch_check("window_transpose_kernel"))) return rc;
    }
    return FCR_OK;
}

int lstm_weights_ok(const fcr_weights *w) {
    if (!w || !w->fc_w || !w->fc_b) return 0;
    for (int l = 0; l < kLayers; ++l)
        if (!w->w_ih[l] || !w->w_hh[l]) return 0;
    return 1;
}

// ------------------------------------------------------------------------------------------------
// LSTM surrogate, H <= 52: the rollout's fused split-f16 cells over one window (fcr_sur.h). Workspace:
// the packed fragments / images / readout as the rollout packs them, the window-batch slabs, and for the
// backward the dgate slab, its scales and the weight-gradient partials.
struct SurLayout {
    int HS, nw, nw_pad, groups;
    size_t fa[3], img[3], fcp, fcb, fnp, wsc, rng, hseq, cseq, xw, htop, dseq, dgs, dsc, part, total;
};
inline int sur_kbb(int HS) { return (HS + 1) / 2; }
// weight-gradient k-blocks: groups of kSurKW backward waves x kL / kSurKC step groups (a missing last wave of a
// group reads a padding wave of the slabs, whose dgates and scales the backward wrote as zero)
inline int sur_nkb(int nw) { return (nw + kSurKW - 1) / kSurKW * (kL / kSurKC); }
inline size_t sur_part_floats(int HS, bool l0) {
    const int RA = (2 * HS + 3) / 4, NT = l0 ? RA + 1 : 2 * RA;
    return (size_t)16 * HS * 16 * NT;
}
SurLayout make_sur(const fcr_dims *d, int with_backward) {
    SurLayout L{};
    L.HS = slot_tier(d->H);
    L.nw = (d->B + kTile - 1) / kTile;
    constexpr int kPad = kFwdWaves > kBwdWaves ? kFwdWaves : kBwdWaves;
    L.nw_pad = (L.nw + kPad - 1) / kPad * kPad;
    const int nkb = sur_nkb(L.nw);
    L.groups = nkb < kSurWgMaxGroups ? nkb : kSurWgMaxGroups;
    size_t off = 0;
    auto take = [&](size_t bytes) {
        const size_t o = off;
        off += align_up(bytes);
        return o;
    };
    const int HS = L.HS;
    const size_t cells = (size_t)L.nw_pad * kLayers * kL;
    for (int l = 0; l < kLayers; ++l) L.fa[l] = take(f16_fwd_bytes(HS, l));
    if (with_backward)
        for (int l = 0; l < kLayers; ++l) L.img[l] = take(img_bytes(HS, l));
    L.fcp = take(sizeof(float) * kOut * HS * 4);
    L.fcb = take(sizeof(float) * kOut);
    L.fnp = take(sizeof(float) * kMS * 4 * kFnpStride);   // written (zeros) by the shared pack job, unused
    L.wsc = take(sizeof(float) * 8);
    L.rng = take(sizeof(float) * 8 * kRangeBlocks);
    L.hseq = take(sizeof(f32x4) * cells * HS * 16);
    if (with_backward) {
        L.cseq = take(sizeof(f32x4) * cells * HS * 16);
        L.xw = take(sizeof(f32x2) * (size_t)L.nw_pad * kL * kWave);
        L.htop = take(sizeof(float) * (size_t)d->B * d->H);
        L.dseq = take(sizeof(f32x4) * (size_t)L.nw_pad * 2 * kL * HS * 16);
        L.dgs = take(cells * sur_kbb(HS) * 2048);
        L.dsc = take(sizeof(float) * cells * 16);
        const size_t pf = sur_part_floats(HS, false) > sur_part_floats(HS, true) ? sur_part_floats(HS, false)
                                                                                 : sur_part_floats(HS, true);
        const size_t fcf = (size_t)((d->B + kFcRows - 1) / kFcRows) * (kOut * d->H + kOut);   // readout partials
        const size_t wgf = (size_t)L.groups * pf;
        L.part = take(sizeof(float) * (wgf > fcf ? wgf : fcf));
    }
    L.total = off;
    return L;
}
SurArgs sur_args(const fcr_dims *d, const SurLayout &L, char *base) {
    SurArgs a{};
    a.B = d->B;
    a.H = d->H;
    a.hseq = (f32x4 *)(base + L.hseq);
    if (L.cseq) {
        a.cseq = (f32x4 *)(base + L.cseq);
        a.xw = (f32x2 *)(base + L.xw);
        a.htop = (float *)(base + L.htop);
        a.dseq = (f32x4 *)(base + L.dseq);
        a.dgs = base + L.dgs;
        a.dsc = (float *)(base + L.dsc);
    }
    for (int l = 0; l < kLayers; ++l) {
        a.p.fa[l] = (const float *)(base + L.fa[l]);
        a.p.img[l] = (const float *)(base + L.img[l]);
    }
    a.p.fcp = (const float *)(base + L.fcp);
    a.p.fcb = (const float *)(base + L.fcb);
    a.p.fnp = (const float *)(base + L.fnp);
    a.p.wsc = (const float *)(base + L.wsc);
    return a;
}

template <int HS>
int sur_forward_t(const SurArgs &a, const SurLayout &L, bool store, hipStream_t s) {
    constexpr int lds = SurGeo<HS>::LDS_FWD;
    static std::atomic<unsigned long long> attr_done[2] = {{0}, {0}};
    const void *fn = store ? (const void *)sur_fwd_kernel<HS, true> : (const void *)sur_fwd_kernel<HS, false>;
    if (const int rc = lds_attr(fn, lds, attr_done[store], "sur_fwd")) return rc;
    if (store) hipLaunchKernelGGL((sur_fwd_kernel<HS, true>), dim3(L.nw_pad / kFwdWaves), dim3(kFwdWaves * kWave), lds, s, a);
    else hipLaunchKernelGGL((sur_fwd_kernel<HS, false>), dim3(L.nw_pad / kFwdWaves), dim3(kFwdWaves * kWave), lds, s, a);
    return launch_check("sur_fwd_kernel");
}

template <int HS, bool L0>
int sur_wgrad_t(const SurArgs &a, const SurLayout &L, int l, float *part, float *g_ih, float *g_hh, hipStream_t s) {
    using W = SurWg<HS, L0>;
    static std::atomic<unsigned long long> attr_done{0};
    if (const int rc = lds_attr((const void *)sur_wgrad_kernel<HS, L0>, W::LDS, attr_done, "sur_wgrad")) return rc;
    const int nkb = sur_nkb(L.nw);
    hipLaunchKernelGGL((sur_wgrad_kernel<HS, L0>), dim3(L.groups), dim3(kSurWgThreads), W::LDS, s, a, l, nkb, part);
    int rc = launch_check("sur_wgrad_kernel");
    if (rc) return rc;
    if (L.groups > 1) {   // the partials summed into the first (coalesced, fixed order), then decoded from it
        hipLaunchKernelGGL(sur_part_sum_kernel, dim3((W::PART / 4 + 255) / 256), dim3(256), 0, s, part, L.groups, W::PART);
        if ((rc = launch_check("sur_part_sum_kernel"))) return rc;
    }
    const int nin = L0 ? kIn : a.H;
    const int n = 4 * a.H * (nin + a.H);
    hipLaunchKernelGGL((sur_wgrad_finish_kernel<HS, L0>), dim3((n + 255) / 256), dim3(256), 0, s, (const float *)part, 1,
                       a.H, a.p.wsc, g_ih, g_hh);
    return launch_check("sur_wgrad_finish_kernel");
}

template <int HS>
int sur_backward_t(const SurArgs &a, const SurLayout &L, float *const *g_w_ih, float *const *g_w_hh, float *part,
                   hipStream_t s) {
    constexpr int lds = SurGeo<HS>::LDS_BWD;
    static std::atomic<unsigned long long> attr_done{0};
    if (const int rc = lds_attr((const void *)sur_bwd_kernel<HS>, lds, attr_done, "sur_bwd")) return rc;
    hipLaunchKernelGGL((sur_bwd_kernel<HS>), dim3(L.nw_pad / kBwdWaves), dim3(kBwdWaves * kWave), lds, s, a);
    int rc = launch_check("sur_bwd_kernel");
    if (rc) return rc;
    if ((rc = sur_wgrad_t<HS, false>(a, L, 2, part, g_w_ih[2], g_w_hh[2], s))) return rc;
    if ((rc = sur_wgrad_t<HS, false>(a, L, 1, part, g_w_ih[1], g_w_hh[1], s))) return rc;
    return sur_wgrad_t<HS, true>(a, L, 0, part, g_w_ih[0], g_w_hh[0], s);
}

int sur_forward(const fcr_dims *d, const fcr_weights *w, const float *x, float *y, int with_backward, char *base,
                hipStream_t s) {
    const SurLayout L = make_sur(d, with_backward);
    int rc;
    // range guard of the window columns from the batch itself (u0 = x: its first B values are window values, so the
    // column-4 bound stays a bound)
    if ((rc = launch_range(d, x, x, nullptr, w->fc_w, w->fc_b, (float *)(base + L.rng), (float *)(base + L.wsc), s)))
        return rc;
    PackArgs pa{};
    pa.H = d->H;
    pa.HS = L.HS;
    pa.CH = 0;
    for (int l = 0; l < kLayers; ++l) {
        pa.wih[l] = w->w_ih[l];
        pa.whh[l] = w->w_hh[l];
    }
    pa.fcw = w->fc_w;
    pa.fcb = w->fc_b;
    pa.fcp = (float *)(base + L.fcp);
    pa.fcbo = (float *)(base + L.fcb);
    pa.fnp = (float *)(base + L.fnp);
    pa.wsc = (const float *)(base + L.wsc);
    PackAllArgs pk{};
    pk.a = pa;
    for (int l = 0; l < kLayers; ++l) {
        const int nf = L.HS * (l == 0 ? (L.HS + 2 + 7) / 8 : (2 * L.HS + 7) / 8) * kWave * 8;
        pk.job[pk.njobs++] = PackJob{kPackFwd16, l, (nf + 255) / 256, (_Float16 *)(base + L.fa[l])};
        if (with_backward)
            pk.job[pk.njobs++] = PackJob{kPackImg, l, (img_pack_threads(L.HS, l) + 255) / 256, (_Float16 *)(base + L.img[l])};
    }
    pk.job[pk.njobs++] = PackJob{kPackMisc, 0, 2, nullptr};
    int blocks = 0;
    for (int j = 0; j < pk.njobs; ++j) blocks += pk.job[j].blocks;
    hipLaunchKernelGGL(pack_all_kernel, dim3(blocks), dim3(256), 0, s, pk);
    if ((rc = launch_check("pack_all_kernel"))) return rc;
    SurArgs a = sur_args(d, L, base);
    a.x = x;
    a.y = y;
    switch (L.HS) {
        case 4: return sur_forward_t<4>(a, L, with_backward != 0, s);
        case 8: return sur_forward_t<8>(a, L, with_backward != 0, s);
        default: return sur_forward_t<13>(a, L, with_backward != 0, s);
    }
}

int sur_backward(const fcr_dims *d, const float *dy, float *const *g_w_ih, float *const *g_w_hh, float *g_fc_w,
                 float *g_fc_b, float *g_x, char *base, hipStream_t s) {
    const SurLayout L = make_sur(d, 1);
    SurArgs a = sur_args(d, L, base);
    a.dy = dy;
    a.g_x = g_x;
    float *part = (float *)(base + L.part);
    int rc;
    switch (L.HS) {
        case 4: rc = sur_backward_t<4>(a, L, g_w_ih, g_w_hh, part, s); break;
        case 8: rc = sur_backward_t<8>(a, L, g_w_ih, g_w_hh, part, s); break;
        default: rc = sur_backward_t<13>(a, L, g_w_ih, g_w_hh, part, s);
    }
    if (rc) return rc;
    // readout: d fc.W = dy^T h_9, d fc.b = sum dy (per-tile partials in the weight-gradient scratch, fixed-order sum)
    const int nfb = (d->B + kFcRows - 1) / kFcRows;
    hipLaunchKernelGGL(sur_fc_partial_kernel, dim3(nfb), dim3(256), 0, s, dy, (const float *)a.htop, d->B, d->H, part);
    if ((rc = launch_check("sur_fc_partial_kernel"))) return rc;
    hipLaunchKernelGGL(sur_fc_final_kernel, dim3(kOut * d->H + kOut), dim3(256), 0, s, (const float *)part, nfb, d->H, g_fc_w,
                       g_fc_b);
    return launch_check("sur_fc_final_kernel");
}

}  // namespace
}  // namespace fcr

using namespace fcr;

extern "C" {

const char *fcr_last_error(void) { return g_err; }

int fcr_abi_version(void) { return FCR_ABI_VERSION; }

int fcr_set_small_batch_limit(int32_t max_batch) {
    return g_small_max_batch.exchange(max_batch < 0 ? 0 : max_batch);
}

int fcr_get_small_batch_limit(void) { return g_small_max_batch.load(); }
int fcr_set_small_pipe_limit(int32_t max_batch) { return g_pipe_max_batch.exchange(max_batch < 0 ? 0 : max_batch); }
int fcr_get_small_pipe_limit(void) { return g_pipe_max_batch.load(); }
int fcr_set_small_pipe_sets(int32_t sets) {
    return g_pipe_sets.exchange(sets < 0 ? 0 : (sets > Pipe<13>::MAX_SETS ? Pipe<13>::MAX_SETS : sets));
}
int fcr_get_small_pipe_sets(void) { return g_pipe_sets.load(); }

int64_t fcr_set_wide_keep_budget(int64_t bytes) {
    return g_wide_keep_budget.exchange(bytes < 0 ? -1 : bytes);
}

int64_t fcr_get_wide_keep_budget(void) { return g_wide_keep_budget.load(); }

int fcr_wide_kept_windows(const fcr_dims *dims, size_t ws_bytes, int32_t *kept) {
    int rc = check_dims(dims);
    if (rc) return rc;
    if (!kept) return fail(FCR_EINVAL, "kept is NULL");
    *kept = is_wide(dims) ? wide_keep_fit(dims, ws_bytes) : 0;
    return FCR_OK;
}

#if FCR_STAMP
// diagnostic builds: byte offset (in ws) of the per-wave cycle sums [nw_pad][8] of the backward
size_t fcr_debug_stamp_offset(const fcr_dims *d) { return make_layout(d, 1).stamp; }
size_t fcr_debug_dseq_offset(const fcr_dims *d) { return make_layout(d, 1).dseq; }
size_t fcr_debug_dxrow_offset(const fcr_dims *d) { return make_layout(d, 1).dxrow; }
#endif

int fcr_wide_bwd_cell_workspace(int32_t B, int32_t H, int32_t layer0, size_t *bytes) {
    if (const int rc = cell_hook_check(B, H)) return rc;
    if (!bytes) return fail(FCR_EINVAL, "bytes is NULL");
    *bytes = cell_hook_layout(B, H, layer0).total;
    return FCR_OK;
}

int fcr_wide_bwd_cell(int32_t B, int32_t H, int32_t layer0, const float *w_ih, const float *w_hh, const float *act,
                      const float *c_prev, const float *dh, const float *din, const float *dc, float *out,
                      float *dc_out, float *rowg, void *ws, size_t ws_bytes, void *stream) {
    if (const int rc = cell_hook_check(B, H)) return rc;
    if (!w_hh || !act || !dh || !dc || !dc_out || !ws || (!layer0 && !w_ih) || (layer0 && (!w_ih || !rowg)) ||
        ((c_prev || !layer0) && !out))
        return fail(FCR_EINVAL, "fcr_wide_bwd_cell: a required pointer is NULL");
    if (((uintptr_t)ws) & 255) return fail(FCR_EINVAL, "fcr_wide_bwd_cell: ws must be 256-byte aligned");
    const size_t need = cell_hook_layout(B, H, layer0).total;
    if (ws_bytes < need) return fail(FCR_EWORKSPACE, "fcr_wide_bwd_cell: ws has %zu bytes, needs %zu", ws_bytes, need);
    return wide_bwd_cell_hook(B, H, layer0, w_ih, w_hh, act, c_prev, dh, din, dc, out, dc_out, rowg, (char *)ws,
                              (hipStream_t)stream);
}

int fcr_workspace_size(const fcr_dims *dims, const fcr_options *opts, int with_backward, size_t *bytes) {
    int rc = check_dims(dims);
    if (rc) return rc;
    if (!bytes) return fail(FCR_EINVAL, "bytes is NULL");
    if (!is_wide(dims)) {
        *bytes = make_layout(dims, with_backward).total;
        return FCR_OK;
    }
    int keep = 0;
    if (with_backward) {   // kept windows within the budget (fcr_set_wide_keep_budget)
        const size_t base = make_wide(dims, 1, 0).total;
        long long budget = keep_budget_of(opts);
        if (budget < 0) {   // default: the whole workspace within wide_default_cap()
            const long long cap = wide_default_cap();
            budget = cap > (long long)base ? cap - (long long)base : 0;
        }
        while (keep < dims->N && make_wide(dims, 1, keep + 1).total - base <= (size_t)budget) ++keep;
    }
    *bytes = make_wide(dims, with_backward, keep).total;
    return FCR_OK;
}

int fcr_forward(const fcr_dims *d, fcr_options *opts, const fcr_weights *w, const float *X, const float *u0,
                const float *states, const float *noise, float *loss, float *cost, float *command,
                float *error, float *prediction, float *xhat, int with_backward, void *ws,
                size_t ws_bytes, void *stream) {
    int rc = check_dims(d);
    if (rc) return rc;
    if (!w || !X || !u0 || !states || !loss || !cost || !command || !error || !prediction || !ws)
        return fail(FCR_EINVAL, "fcr_forward: a required pointer is NULL");
    for (int l = 0; l < kLayers; ++l)
        if (!w->w_ih[l] || !w->w_hh[l])
            return fail(FCR_EINVAL, "fcr_forward: LSTM weight of layer %d is NULL", l);
    if (!w->fc_w || !w->fc_b || !w->ctrl_w_inp || !w->ctrl_b_inp || !w->ctrl_w_out)
        return fail(FCR_EINVAL, "fcr_forward: a weight pointer is NULL");
    if (((uintptr_t)ws) & 255) return fail(FCR_EINVAL, "fcr_forward: ws must be 256-byte aligned");
    if (is_wide(d)) {
        const size_t need = make_wide(d, with_backward).total;
        if (ws_bytes < need) return fail(FCR_EWORKSPACE, "fcr_forward: ws has %zu bytes, needs %zu", ws_bytes, need);
        note_kernels(opts, FCR_KERNELS_WIDE);
        return wide_forward(d, w, X, u0, states, noise, loss, cost, command, error, prediction, xhat, with_backward,
                            (char *)ws, ws_bytes, (hipStream_t)stream);
    }
    const Layout L = make_layout(d, with_backward);
    if (ws_bytes < L.total)
        return fail(FCR_EWORKSPACE, "fcr_forward: ws has %zu bytes, needs %zu", ws_bytes, L.total);
    hipStream_t s = (hipStream_t)stream;
    char *base = (char *)ws;

    PackArgs pa{};
    pa.H = d->H;
    pa.HS = L.HS;
    pa.CH = d->ctrl_hidden;
    for (int l = 0; l < kLayers; ++l) {
        pa.wih[l] = w->w_ih[l];
        pa.whh[l] = w->w_hh[l];
    }
    pa.fcw = w->fc_w;
    pa.fcb = w->fc_b;
    pa.cwi = w->ctrl_w_inp;
    pa.cbi = w->ctrl_b_inp;
    pa.cwo = w->ctrl_w_out;
    pa.fcp = (float *)(base + L.fcp);
    pa.fcbo = (float *)(base + L.fcb);
    pa.fnp = (float *)(base + L.fnp);
    pa.wsc = (const float *)(base + L.wsc);
    if ((rc = launch_range(d, states, u0, noise, w->fc_w, w->fc_b, (float *)(base + L.rng), (float *)(base + L.wsc), s)))
        return rc;
    {   // every weight pack of the call in ONE launch (seven launches of ~4 us each were a step's overhead
        // at the reference's B = 15), and the pipelined kernels' counters zeroed for this forward and its backward
        PackAllArgs pk{};
        pk.a = pa;
        if (L.nw <= kPipeMaxGroups) {
            pk.clear = (unsigned *)(base + L.pipe_flags);
            pk.nclear = L.nw * kPipeFlags;
        }
        for (int l = 0; l < kLayers; ++l) {
            const int nf = L.HS * (l == 0 ? (L.HS + 2 + 7) / 8 : (2 * L.HS + 7) / 8) * kWave * 8;   // per (tile, block, lane, k)
            pk.job[pk.njobs++] = PackJob{kPackFwd16, l, (nf + 255) / 256, (_Float16 *)(base + L.fa[l])};
            if (with_backward)
                pk.job[pk.njobs++] = PackJob{kPackImg, l, (img_pack_threads(L.HS, l) + 255) / 256, (_Float16 *)(base + L.img[l])};
        }
        pk.job[pk.njobs++] = PackJob{kPackMisc, 0, 2, nullptr};
        int blocks = 0;
        for (int j = 0; j < pk.njobs; ++j) blocks += pk.job[j].blocks;
        hipLaunchKernelGGL(pack_all_kernel, dim3(blocks), dim3(256), 0, s, pk);
        if ((rc = launch_check("pack_all_kernel"))) return rc;
    }

    FwdArgs fa{};
    fa.B = d->B;
    fa.N = d->N;
    fa.alpha = d->alpha;
    fa.X = X;
    fa.u0 = u0;
    fa.states = states;
    fa.noise = noise;
    fa.cost = cost;
    fa.command = command;
    fa.error = error;
    fa.prediction = prediction;
    fa.xhat_user = xhat;
    fa.xhat_ws = (float *)(base + L.xhat);
    fa.loss_part = (float *)(base + L.loss_part);
    fa.hseq = (f32x4 *)(base + L.hseq);
    fa.cseq = with_backward ? (f32x4 *)(base + L.cseq) : nullptr;
    fa.xw = with_backward ? (f32x2 *)(base + L.xw) : nullptr;
    fa.p = packed_ptrs(L, base);
#if FCR_STAMP
    fa.stamp = (unsigned long long *)(base + L.stamp) + (size_t)L.nw_pad * 8;
#endif
    const bool small = use_small(d, L, opts);
    note_kernels(opts, small ? FCR_KERNELS_SMALL : FCR_KERNELS_FUSED);
    const bool piped = small && use_pipe(d, L, opts);
    if (piped) {
        PipeArgs pa = pipe_args(L, base);
        pa.loss = loss;
        const int S = pipe_sets(d, L, Pipe<13>::MAX_SETS, 2);
        if (L.HS == 8) rc = with_backward ? launch_pfwd_s<8, true>(fa, pa, L, S, s) : launch_pfwd_s<8, false>(fa, pa, L, S, s);
        else rc = with_backward ? launch_pfwd_s<13, true>(fa, pa, L, S, s) : launch_pfwd_s<13, false>(fa, pa, L, S, s);
    } else if (small) {
        if (L.HS == 8) rc = with_backward ? launch_sfwd_t<8, true>(fa, L, s) : launch_sfwd_t<8, false>(fa, L, s);
        else rc = with_backward ? launch_sfwd_t<13, true>(fa, L, s) : launch_sfwd_t<13, false>(fa, L, s);
    } else {
        switch (L.HS) {
            case 4: rc = launch_fwd<4>(fa, L, d->precision == FCR_PRECISION_F16, s); break;
            case 8: rc = launch_fwd<8>(fa, L, d->precision == FCR_PRECISION_F16, s); break;
            case 13: rc = launch_fwd<13>(fa, L, d->precision == FCR_PRECISION_F16, s); break;
            default: rc = fail(FCR_EUNSUPPORTED, "H=%d", d->H);
        }
    }
    if (rc) return rc;
    if (piped) return FCR_OK;   // the pipelined forward wrote the loss itself
    // the fused kernel writes a (zero) partial for every padded wave; the small one one per group
    hipLaunchKernelGGL(loss_reduce_kernel, dim3(1), dim3(256), 0, s, (const float *)fa.loss_part,
                       small ? L.nw : L.nw_pad, d->B, loss);
    return launch_check("loss_reduce_kernel");
}

int fcr_backward(const fcr_dims *d, fcr_options *opts, const float *X, const float *states, const float *prediction,
                 const float *dloss, float *g_u0, float *g_w_inp, float *g_b_inp, float *g_w_out,
                 void *ws, size_t ws_bytes, void *stream) {
    int rc = check_dims(d);
    if (rc) return rc;
    if (!X || !states || !prediction || !dloss || !g_u0 || !g_w_inp || !g_b_inp || !g_w_out || !ws)
        return fail(FCR_EINVAL, "fcr_backward: a required pointer is NULL");
    if (((uintptr_t)ws) & 255) return fail(FCR_EINVAL, "fcr_backward: ws must be 256-byte aligned");
    if (is_wide(d)) {
        const size_t need = make_wide(d, 1).total;
        if (ws_bytes < need) return fail(FCR_EWORKSPACE, "fcr_backward: ws has %zu bytes, needs %zu", ws_bytes, need);
        note_kernels(opts, FCR_KERNELS_WIDE);
        return wide_backward(d, X, states, prediction, dloss, g_u0, g_w_inp, g_b_inp, g_w_out, (char *)ws, ws_bytes,
                             (hipStream_t)stream);
    }
    const Layout L = make_layout(d, 1);
    if (ws_bytes < L.total)
        return fail(FCR_EWORKSPACE, "fcr_backward: ws has %zu bytes, needs %zu", ws_bytes, L.total);
    hipStream_t s = (hipStream_t)stream;
    char *base = (char *)ws;
    BwdArgs ba{};
    ba.B = d->B;
    ba.N = d->N;
    ba.hidden = d->ctrl_hidden;
    ba.alpha = d->alpha;
    ba.X = X;
    ba.states = states;
    ba.prediction = prediction;
    ba.xhat = (const float *)(base + L.xhat);
    ba.dloss = dloss;
    ba.hseq = (const f32x4 *)(base + L.hseq);
    ba.cseq = (const f32x4 *)(base + L.cseq);
    ba.xw = (const f32x2 *)(base + L.xw);
    ba.dseq = (f32x4 *)(base + L.dseq);
    ba.dxrow = (f32x2 *)(base + L.dxrow);
    ba.g_u0 = g_u0;
    ba.dv = (float *)(base + L.dv);
#if FCR_STAMP
    ba.stamp = (unsigned long long *)(base + L.stamp);
#endif
    ba.p = packed_ptrs(L, base);
    const bool small = use_small(d, L, opts);
    note_kernels(opts, small ? FCR_KERNELS_SMALL : FCR_KERNELS_FUSED);
    if (small && use_pipe(d, L, opts)) {
        const PipeArgs pa = pipe_args(L, base);
        const int S = pipe_sets(d, L, Pipe<13>::MAX_SETS_BWD, 3);
        rc = L.HS == 8 ? launch_pbwd_s<8>(ba, pa, L, S, s) : launch_pbwd_s<13>(ba, pa, L, S, s);
    } else if (small) {
        rc = L.HS == 8 ? launch_sbwd_t<8>(ba, L, s) : launch_sbwd_t<13>(ba, L, s);
    } else {
        switch (L.HS) {
            case 4: rc = launch_bwd<4>(ba, L, d->precision == FCR_PRECISION_F16, s); break;
            case 8: rc = launch_bwd<8>(ba, L, d->precision == FCR_PRECISION_F16, s); break;
            case 13: rc = launch_bwd<13>(ba, L, d->precision == FCR_PRECISION_F16, s); break;
            default: rc = fail(FCR_EUNSUPPORTED, "H=%d", d->H);
        }
    }
    if (rc) return rc;
    float *part = (float *)(base + L.fnn_part);
    const bool one = L.ctrl_blocks == 1;   // one block writes the gradients itself (grad_out5)
    hipLaunchKernelGGL(ctrl_grad_kernel, dim3(L.ctrl_blocks), dim3(kCtrlBlock), 0, s, X, ba.xhat,
                       (const float *)ba.dv, ba.p.fnp, d->B, d->N, d->ctrl_hidden, part,
                       one ? g_w_inp : nullptr, one ? g_b_inp : nullptr, one ? g_w_out : nullptr);
    if ((rc = launch_check("ctrl_grad_kernel"))) return rc;
    if (one) return FCR_OK;
    hipLaunchKernelGGL(grad_reduce_kernel, dim3(d->ctrl_hidden * 5), dim3(256), 0, s, (const float *)part,
                       L.ctrl_blocks, d->ctrl_hidden, g_w_inp, g_b_inp, g_w_out);
    return launch_check("grad_reduce_kernel");
}

int fcr_lstm_workspace_size(const fcr_dims *dims, int with_backward, size_t *bytes) {
    int rc = check_lstm_dims(dims);
    if (rc) return rc;
    if (!bytes) return fail(FCR_EINVAL, "bytes is NULL");
    *bytes = is_wide(dims) ? make_surw(dims, with_backward).total : make_sur(dims, with_backward).total;
    return FCR_OK;
}

int fcr_lstm_forward(const fcr_dims *d, const fcr_weights *w, const float *x, float *y, int with_backward, void *ws,
                     size_t ws_bytes, void *stream) {
    int rc = check_lstm_dims(d);
    if (rc) return rc;
    if (!x || !y || !ws) return fail(FCR_EINVAL, "fcr_lstm_forward: a required pointer is NULL");
    if (!lstm_weights_ok(w)) return fail(FCR_EINVAL, "fcr_lstm_forward: an LSTM/fc weight pointer is NULL");
    if (((uintptr_t)ws) & 255) return fail(FCR_EINVAL, "fcr_lstm_forward: ws must be 256-byte aligned");
    if (!is_wide(d)) {   // H <= 52: the fused kernels (fcr_sur.h)
        const size_t need = make_sur(d, with_backward).total;
        if (ws_bytes < need) return fail(FCR_EWORKSPACE, "fcr_lstm_forward: ws has %zu bytes, needs %zu", ws_bytes, need);
        return sur_forward(d, w, x, y, with_backward, (char *)ws, (hipStream_t)stream);
    }
    const size_t need = make_surw(d, with_backward).total;
    if (ws_bytes < need) return fail(FCR_EWORKSPACE, "fcr_lstm_forward: ws has %zu bytes, needs %zu", ws_bytes, need);
    return surw_forward(d, w, x, y, with_backward, (char *)ws, (hipStream_t)stream);
}

int fcr_lstm_backward(const fcr_dims *d, const fcr_weights *w, const float *dy, float *const *g_w_ih,
                      float *const *g_w_hh, float *g_fc_w, float *g_fc_b, float *g_x, void *ws, size_t ws_bytes,
                      void *stream) {
    int rc = check_lstm_dims(d);
    if (rc) return rc;
    if (!dy || !ws || !g_w_ih || !g_w_hh || !g_fc_w || !g_fc_b)
        return fail(FCR_EINVAL, "fcr_lstm_backward: a required pointer is NULL");
    for (int l = 0; l < kLayers; ++l)
        if (!g_w_ih[l] || !g_w_hh[l]) return fail(FCR_EINVAL, "fcr_lstm_backward: gradient of layer %d is NULL", l);
    if (!lstm_weights_ok(w)) return fail(FCR_EINVAL, "fcr_lstm_backward: an LSTM/fc weight pointer is NULL");
    if (((uintptr_t)ws) & 255) return fail(FCR_EINVAL, "fcr_lstm_backward: ws must be 256-byte aligned");
    if (!is_wide(d)) {
        const size_t need = make_sur(d, 1).total;
        if (ws_bytes < need) return fail(FCR_EWORKSPACE, "fcr_lstm_backward: ws has %zu bytes, needs %zu", ws_bytes, need);
        return sur_backward(d, dy, g_w_ih, g_w_hh, g_fc_w, g_fc_b, g_x, (char *)ws, (hipStream_t)stream);
    }
    const size_t need = make_surw(d, 1).total;
    if (ws_bytes < need) return fail(FCR_EWORKSPACE, "fcr_lstm_backward: ws has %zu bytes, needs %zu", ws_bytes, need);
    return surw_backward(d, w, dy, g_w_ih, g_w_hh, g_fc_w, g_fc_b, g_x, (char *)ws, (hipStream_t)stream);
}

int fcr_fnn_workspace_size(int32_t B, int32_t hidden, size_t *bytes) {
    if (B < 0 || hidden < 1 || hidden > fnn::kFnnMaxHidden)
        return fail(FCR_EINVAL, "fcr_fnn_workspace_size: B=%d, hidden=%d (1..%d)", B, hidden, fnn::kFnnMaxHidden);
    if (!bytes) return fail(FCR_EINVAL, "bytes is NULL");
    const size_t blocks = ((size_t)B + fnn::kFnnItems - 1) / fnn::kFnnItems;
    *bytes = blocks * (size_t)hidden * 5 * sizeof(float);
    return FCR_OK;
}

static int fnn_check(const char *what, int32_t B, int32_t in_dim, int32_t hidden) {
    if (B < 0) return fail(FCR_EINVAL, "%s: B=%d must be >= 0", what, B);
    if (in_dim != kCtrlIn) return fail(FCR_EUNSUPPORTED, "%s: in_dim=%d: built for %d (UL/Main.py:188)", what, in_dim, kCtrlIn);
    if (hidden < 1 || hidden > fnn::kFnnMaxHidden)
        return fail(FCR_EUNSUPPORTED, "%s: hidden=%d: built for 1..%d", what, hidden, fnn::kFnnMaxHidden);
    return FCR_OK;
}

int fcr_fnn_forward(int32_t B, int32_t in_dim, int32_t hidden, const float *X, const float *w_inp,
                    const float *b_inp, const float *w_out, float *u, void *stream) {
    int rc = fnn_check("fcr_fnn_forward", B, in_dim, hidden);
    if (rc) return rc;
    if (B == 0) return FCR_OK;
    if (!X || !w_inp || !b_inp || !w_out || !u) return fail(FCR_EINVAL, "fcr_fnn_forward: a required pointer is NULL");
    hipLaunchKernelGGL(fnn::fnn_fwd_kernel, dim3((B + fnn::kFnnBlock - 1) / fnn::kFnnBlock), dim3(fnn::kFnnBlock), 0,
                       (hipStream_t)stream, B, hidden, X, w_inp, b_inp, w_out, u);
    return launch_check("fnn_fwd_kernel");
}

int fcr_fnn_backward(int32_t B, int32_t in_dim, int32_t hidden, const float *X, const float *w_inp,
                     const float *b_inp, const float *w_out, const float *g_u, float *g_x, float *g_w_inp,
                     float *g_b_inp, float *g_w_out, void *ws, size_t ws_bytes, void *stream) {
    int rc = fnn_check("fcr_fnn_backward", B, in_dim, hidden);
    if (rc) return rc;
    if (!w_inp || !b_inp || !w_out || !g_w_inp || !g_b_inp || !g_w_out || (B && (!X || !g_u || !ws)))
        return fail(FCR_EINVAL, "fcr_fnn_backward: a required pointer is NULL");
    size_t need = 0;
    if ((rc = fcr_fnn_workspace_size(B, hidden, &need))) return rc;
    if (ws_bytes < need) return fail(FCR_EWORKSPACE, "fcr_fnn_backward: ws has %zu bytes, needs %zu", ws_bytes, need);
    hipStream_t s = (hipStream_t)stream;
    const int blocks = (int)((B + fnn::kFnnItems - 1) / fnn::kFnnItems);
    if (blocks) {
        const bool one = blocks == 1;   // one block writes the gradients itself (grad_out5)
        hipLaunchKernelGGL(fnn::fnn_bwd_kernel, dim3(blocks), dim3(fnn::kFnnBlock), 0, s, B, hidden, X, w_inp, b_inp,
                           w_out, g_u, g_x, (float *)ws, one ? g_w_inp : nullptr, one ? g_b_inp : nullptr,
                           one ? g_w_out : nullptr);
        if ((rc = launch_check("fnn_bwd_kernel"))) return rc;
        if (one) return FCR_OK;
    }
    hipLaunchKernelGGL(grad_reduce_kernel, dim3(hidden * 5), dim3(256), 0, s, (const float *)ws, blocks, hidden,
                       g_w_inp, g_b_inp, g_w_out);
    return launch_check("grad_reduce_kernel");
}

#if FCR_WB_STAMP
// diagnostic builds only (scripts/stamp_wb.py): the fused backward cell's section sums (fcr_wbwd.h), then zeroed
int fcr_debug_wb_stamp(unsigned long long *out16) {
    if (hipMemcpyFromSymbol(out16, HIP_SYMBOL(fcr_wb_stamp), 16 * sizeof(unsigned long long)) != hipSuccess)
        return FCR_EHIP;
    static const unsigned long long zero[16] = {};
    return hipMemcpyToSymbol(HIP_SYMBOL(fcr_wb_stamp), zero, sizeof(zero)) == hipSuccess ? FCR_OK : FCR_EHIP;
}
#endif
}  // extern "C"
