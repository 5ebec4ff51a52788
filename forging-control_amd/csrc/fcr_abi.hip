// fcr_abi.hip — host side and C ABI (include/fcr.h) of the gfx950 rollout engine.
//
// Replaces the torch work behind `loss_function(...)` / `loss.backward()` at
// /root/reference/Unsupervised Learning/Functions.py:646 and :655. All launches are stream-ordered on
// the caller's stream; nothing here allocates or synchronises.
#include <hip/hip_runtime.h>
#include <stdarg.h>
#include <stdint.h>
#include <stdio.h>

#include "fcr.h"
#include "fcr_bwd.h"
#include "fcr_common.h"
#include "fcr_fwd.h"
#include "fcr_img.h"
#include "fcr_pack.h"

namespace fcr {
namespace {

thread_local char g_err[512] = "no error";

int fail(int code, const char *fmt, ...) __attribute__((format(printf, 2, 3)));
int fail(int code, const char *fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof(g_err), fmt, ap);
    va_end(ap);
    return code;
}

struct Layout {
    int HS, nw, nw_pad;
    size_t fa[3], img[3], fcp, fcb, fnp, xhat, dv, loss_part, fnn_part, hseq, cseq, xw, dseq, dxrow, stamp, total;
    int ctrl_blocks;
};

size_t align_up(size_t x) { return (x + 255) & ~(size_t)255; }

// Kernels are instantiated for 4, 8 and 13 unit slots (H <= 16, 32, 52); a smaller H runs in the next
// tier with its padding units' weights zero — their gates stay at i = f = o = 1/2, g = 0, so c = h = 0
// and they add nothing to any product (tests/test_gpu_parity.py: H = 40 against the oracle).
constexpr int kMaxSlots = 13;
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
    if (d->H < 1 || d->H > 4 * kMaxSlots)
        return fail(FCR_EUNSUPPORTED, "H=%d: built for 1..%d (LDS-resident weight images)", d->H, 4 * kMaxSlots);
    if ((long long)d->B * d->N > (1LL << 31)) return fail(FCR_EINVAL, "B*N too large");
    return FCR_OK;
}

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
    L.xhat = take(sizeof(float) * (size_t)d->B * d->N * kOut);
    L.loss_part = take(sizeof(float) * L.nw_pad);
    L.dv = take(sizeof(float) * (size_t)d->B * d->N);
    L.ctrl_blocks = (int)(((long long)d->B * d->N + kCtrlItems - 1) / kCtrlItems);
    L.fnn_part = take(sizeof(float) * (size_t)L.ctrl_blocks * d->ctrl_hidden * 5);
    // sequence slabs (fcr_common.h): h of every cell always (layers 0, 1 are the next phase's input);
    // c, the window rows and the backward's dx / window-row-gradient slabs only with a backward
    const size_t qcells = (size_t)L.nw_pad * d->N * kLayers * kL * ((HS + 3) / 4) * kWave;
    L.hseq = take(sizeof(f32x4) * qcells);
    if (with_backward) {
        L.cseq = take(sizeof(f32x4) * qcells);
        L.xw = take(sizeof(f32x2) * (size_t)L.nw_pad * d->N * kL * kWave);
        L.dseq = take(sizeof(f32x4) * (size_t)L.nw_pad * d->N * 2 * kL * ((HS + 3) / 4) * kWave);
        L.dxrow = take(sizeof(f32x2) * (size_t)L.nw_pad * d->N * kL * kWave);
    }
#if FCR_STAMP
    L.stamp = take(sizeof(unsigned long long) * L.nw_pad * 8);
#endif
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
    return p;
}

int launch_check(const char *what) {
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return fail(FCR_EHIP, "launch of %s failed: %s", what, hipGetErrorString(e));
    return FCR_OK;
}

template <int HS, bool STORE>
int launch_fwd_t(const FwdArgs &fa, const Layout &L, hipStream_t s) {
    const int lds = Geo16<HS>::LDS_FWD;
    static bool attr_set = false;
    if (!attr_set) {
        const hipError_t e = hipFuncSetAttribute((const void *)fcr_fwd_kernel<HS, STORE>,
                                                 hipFuncAttributeMaxDynamicSharedMemorySize, lds);
        if (e != hipSuccess) return fail(FCR_EHIP, "hipFuncSetAttribute(fwd): %s", hipGetErrorString(e));
        attr_set = true;
    }
    hipLaunchKernelGGL((fcr_fwd_kernel<HS, STORE>), dim3(L.nw_pad / kFwdWaves), dim3(kFwdWaves * kWave),
                       lds, s, fa);
    return launch_check("fcr_fwd_kernel");
}

template <int HS>
int launch_fwd(const FwdArgs &fa, const Layout &L, hipStream_t s) {
    return fa.cseq ? launch_fwd_t<HS, true>(fa, L, s) : launch_fwd_t<HS, false>(fa, L, s);
}

template <int HS>
int launch_bwd(const BwdArgs &ba, const Layout &L, hipStream_t s) {
    const int lds = BwdLds<HS>::BYTES;
    static bool attr_set = false;
    if (!attr_set) {
        const hipError_t e = hipFuncSetAttribute((const void *)fcr_bwd_kernel<HS>,
                                                 hipFuncAttributeMaxDynamicSharedMemorySize, lds);
        if (e != hipSuccess) return fail(FCR_EHIP, "hipFuncSetAttribute(bwd): %s", hipGetErrorString(e));
        attr_set = true;
    }
    hipLaunchKernelGGL(fcr_bwd_kernel<HS>, dim3(L.nw_pad / kBwdWaves), dim3(kBwdWaves * kWave), lds, s, ba);
    return launch_check("fcr_bwd_kernel");
}

}  // namespace
}  // namespace fcr

using namespace fcr;

extern "C" {

const char *fcr_last_error(void) { return g_err; }

int fcr_abi_version(void) { return FCR_ABI_VERSION; }

#if FCR_STAMP
// diagnostic builds: byte offset (in ws) of the per-wave cycle sums [nw_pad][8] of the backward
size_t fcr_debug_stamp_offset(const fcr_dims *d) { return make_layout(d, 1).stamp; }
#endif

int fcr_workspace_size(const fcr_dims *dims, int with_backward, size_t *bytes) {
    int rc = check_dims(dims);
    if (rc) return rc;
    if (!bytes) return fail(FCR_EINVAL, "bytes is NULL");
    *bytes = make_layout(dims, with_backward).total;
    return FCR_OK;
}

int fcr_forward(const fcr_dims *d, const fcr_weights *w, const float *X, const float *u0,
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
    for (int l = 0; l < kLayers; ++l) {
        const int nf = (int)(f16_fwd_bytes(L.HS, l) / 4);   // one thread per (hi, lo) pair
        hipLaunchKernelGGL(pack_fwd16_kernel, dim3((nf + 255) / 256), dim3(256), 0, s, pa, l,
                           (_Float16 *)(base + L.fa[l]));
        if ((rc = launch_check("pack_fwd16_kernel"))) return rc;
        if (with_backward) {
            const int ni = (int)(img_bytes(L.HS, l) / 4);
            hipLaunchKernelGGL(pack_img_kernel, dim3((ni + 255) / 256), dim3(256), 0, s, pa, l,
                               (_Float16 *)(base + L.img[l]));
            if ((rc = launch_check("pack_img_kernel"))) return rc;
        }
    }
    hipLaunchKernelGGL(pack_misc_kernel, dim3(2), dim3(256), 0, s, pa);
    if ((rc = launch_check("pack_misc_kernel"))) return rc;

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
    switch (L.HS) {
        case 4: rc = launch_fwd<4>(fa, L, s); break;
        case 8: rc = launch_fwd<8>(fa, L, s); break;
        case 13: rc = launch_fwd<13>(fa, L, s); break;
        default: rc = fail(FCR_EUNSUPPORTED, "H=%d", d->H);
    }
    if (rc) return rc;
    hipLaunchKernelGGL(loss_reduce_kernel, dim3(1), dim3(256), 0, s, (const float *)fa.loss_part,
                       L.nw_pad, d->B, loss);
    return launch_check("loss_reduce_kernel");
}

int fcr_backward(const fcr_dims *d, const float *X, const float *states, const float *prediction,
                 const float *dloss, float *g_u0, float *g_w_inp, float *g_b_inp, float *g_w_out,
                 void *ws, size_t ws_bytes, void *stream) {
    int rc = check_dims(d);
    if (rc) return rc;
    if (!X || !states || !prediction || !dloss || !g_u0 || !g_w_inp || !g_b_inp || !g_w_out || !ws)
        return fail(FCR_EINVAL, "fcr_backward: a required pointer is NULL");
    if (((uintptr_t)ws) & 255) return fail(FCR_EINVAL, "fcr_backward: ws must be 256-byte aligned");
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
    switch (L.HS) {
        case 4: rc = launch_bwd<4>(ba, L, s); break;
        case 8: rc = launch_bwd<8>(ba, L, s); break;
        case 13: rc = launch_bwd<13>(ba, L, s); break;
        default: rc = fail(FCR_EUNSUPPORTED, "H=%d", d->H);
    }
    if (rc) return rc;
    float *part = (float *)(base + L.fnn_part);
    hipLaunchKernelGGL(ctrl_grad_kernel, dim3(L.ctrl_blocks), dim3(kCtrlBlock), 0, s, X, ba.xhat,
                       (const float *)ba.dv, ba.p.fnp, d->B, d->N, d->ctrl_hidden, part);
    if ((rc = launch_check("ctrl_grad_kernel"))) return rc;
    hipLaunchKernelGGL(grad_reduce_kernel, dim3(d->ctrl_hidden * 5), dim3(256), 0, s, (const float *)part,
                       L.ctrl_blocks, d->ctrl_hidden, g_w_inp, g_b_inp, g_w_out);
    return launch_check("grad_reduce_kernel");
}

}  // extern "C"
