/*
 * fcr.h — C ABI of the MI355X-native (gfx950) unsupervised-MPC rollout engine.
 *
 * This library replaces the work torch dispatches inside ONE Python call of the reference,
 *
 *     loss, loss_features = loss_function(simulator, model, X, output, z, device, enable_noise)
 *     ...
 *     loss.backward()
 *
 * at /root/reference/Unsupervised Learning/Functions.py:646 and :655 (MPCLoss.forward,
 * Functions.py:1353-1472, plus its autograd backward). The reference has no FFI of its own (it is
 * pure Python/PyTorch); the binding a maintainer adds is the ctypes stub in INTEGRATION.md, and the
 * Python drop-in `MPCLoss` in forging-control_amd/functions.py is that stub.
 *
 * Conventions (all entry points):
 *   - every pointer is caller-owned DEVICE memory (fp32, contiguous, batch-first exactly as the
 *     reference lays it out), except `dims`/`w` (host structs);
 *   - `stream` is a hipStream_t (passed as void* so this header needs no HIP headers); all work is
 *     stream-ordered on it, nothing synchronises the host;
 *   - no allocation inside a call: scratch comes from `ws` (size from fcr_workspace_size);
 *   - return FCR_OK (0) or a negative FCR_E* code; fcr_last_error() (thread-local) explains it.
 */
#ifndef FCR_H
#define FCR_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define FCR_ABI_VERSION 6   /* 6: kept wide windows hold gate activations; fcr_wide_bwd_cell */

enum {
    FCR_OK = 0,
    FCR_EINVAL = -1,      /* bad dims, null pointer, misalignment            */
    FCR_EWORKSPACE = -2,  /* ws too small                                      */
    FCR_EHIP = -3,        /* a HIP runtime call failed                         */
    FCR_EUNSUPPORTED = -4 /* dims valid for the reference but not built here   */
};

/* Problem shape. Reference values: L=10 (Functions.py:1434 hard-codes the 10-row window),
 * layers=3 / H=50 / in_dim=5 / out_dim=4 (UL/Main.py:144-154), ctrl 3->50->1 (UL/Main.py:183-188),
 * N = n_horizon = 10 (UL/template_mpc.py:20), alpha = 20.0 (UL/Main.py:192). */
typedef struct fcr_dims {
    int32_t B;           /* trajectories in the batch                         */
    int32_t N;           /* prediction horizon (MPCLoss.N)                    */
    int32_t L;           /* lookback rows of the LSTM window (must be 10)     */
    int32_t H;           /* LSTM hidden size: 1..52 fused kernels, 53..2048 per-cell GEMM path */
    int32_t layers;      /* LSTM layers (must be 3)                           */
    int32_t in_dim;      /* LSTM input features (must be 5)                   */
    int32_t out_dim;     /* LSTM outputs (must be 4)                          */
    int32_t ctrl_in;     /* controller inputs (must be 3)                     */
    int32_t ctrl_hidden; /* controller hidden units (<= 52)                   */
    float alpha;         /* MPCLoss.alpha, command-variation weight            */
    int32_t precision;   /* FCR_PRECISION_FP32 (0) or FCR_PRECISION_F16 (1), below */
} fcr_dims;

/* Arithmetic of the gate products (fcr_forward/fcr_backward; fcr_lstm_* ignore it and run fp32):
 *   FCR_PRECISION_FP32 — fp32-accurate: each operand split into two f16 halves, three f16 MFMAs per
 *                        product, fp32 accumulate (results within 1e-5 of an fp64 evaluation);
 *   FCR_PRECISION_F16  — config 3's reduced-precision mode ("bf16 storage/MFMA fwd"):
 *                        f16 operands (11-bit significand, more than bf16's 8; the backward's per-trajectory
 *                        power-of-two scaling keeps them in range), one MFMA per product, fp32 accumulate;
 *                        H <= 52 only;
 *   (2, the former FCR_PRECISION_F16_FWD — f16 forward, fp32-accurate backward — is retired in ABI v5 and refused
 *   with FCR_EUNSUPPORTED: it ran 1.08x the fp32 step at the all-f16 mode's accuracy, DESIGN.md §4 "Config 3".)
 * Both calls of one step must be given the same dims (the same precision value). */
#define FCR_PRECISION_FP32 0
#define FCR_PRECISION_F16 1

/* Weights, torch layouts (row-major, as state_dict holds them). */
typedef struct fcr_weights {
    const float *ctrl_w_inp; /* FNNModel.fc_inp.weight (ctrl_hidden, ctrl_in)  Functions.py:249 */
    const float *ctrl_b_inp; /* FNNModel.fc_inp.bias   (ctrl_hidden)                            */
    const float *ctrl_w_out; /* FNNModel.fc_out.weight (1, ctrl_hidden), no bias Functions.py:251 */
    const float *w_ih[3];    /* LSTMModel.lstm.weight_ih_l{0,1,2} (4H, in_dim | H)  :325        */
    const float *w_hh[3];    /* LSTMModel.lstm.weight_hh_l{0,1,2} (4H, H)                       */
    const float *fc_w;       /* LSTMModel.fc.weight (out_dim, H)                     :329        */
    const float *fc_b;       /* LSTMModel.fc.bias   (out_dim)                                    */
} fcr_weights;

/* Per-call kernel options of fcr_workspace_size / fcr_forward / fcr_backward (ABI v5). NULL = every field at
 * FCR_OPT_INHERIT. Two users of the library in one process (a training rollout and a validation rollout beside it,
 * on different streams or threads) each pass their own and see nothing of the other's; the process-wide setters
 * below only supply the defaults a field set to FCR_OPT_INHERIT takes. A forward and its backward should be given the
 * same options (both kernel families keep one workspace layout, so a mix is valid, only slower).
 *   small_batch_limit  B <= it runs the small-batch kernels (fp32-accurate mode, H 17..52), 0 = never;
 *                      negative (FCR_OPT_INHERIT): fcr_set_small_batch_limit's value
 *   wide_keep_budget   H > 52, read by fcr_workspace_size only: bytes of kept windows the workspace may add;
 *                      FCR_KEEP_AUTO (-1) the library's policy (fcr_set_wide_keep_budget below), FCR_OPT_INHERIT (-2)
 *                      the process-wide setting
 *   kernels            OUT, written by fcr_forward / fcr_backward: the kernel family the call launched
 *                      (FCR_KERNELS_SMALL, _FUSED or _WIDE) */
#define FCR_OPT_INHERIT (-2)
#define FCR_KEEP_AUTO (-1)
#define FCR_KERNELS_SMALL 1
#define FCR_KERNELS_FUSED 2
#define FCR_KERNELS_WIDE 3
typedef struct fcr_options {
    int32_t small_batch_limit;
    int32_t kernels;
    int64_t wide_keep_budget;
} fcr_options;

/* Bytes of scratch a forward (+ backward when with_backward != 0) needs for `dims` (and, H > 52, opts' keep budget). */
int fcr_workspace_size(const fcr_dims *dims, const fcr_options *opts, int with_backward, size_t *bytes);

/* H > 52: how many of the N windows a backward-enabled workspace of ws_bytes keeps (the forward and the backward
 * each derive this count from the ws_bytes they are given; 0 for H <= 52). */
int fcr_wide_kept_windows(const fcr_dims *dims, size_t ws_bytes, int32_t *kept);

/*
 * Forward rollout = MPCLoss.forward (Functions.py:1353-1472).
 *   X        (B,3)   input_controller [y_dot, z, ref]          (Functions.py:1353, ref = X[:,-1] :1392)
 *   u0       (B,1)   output_controller = controller(X)          (Functions.py:643)
 *   states   (B,L,5) LSTM window [y_dot,p1,p2,z,u]              (Functions.py:1395)
 *   noise    (B,N,4) additive LSTM-output noise, or NULL        (Functions.py:1400-1402,1438-1440)
 * Outputs:
 *   loss (1) mean cost; cost/command/error (B) = loss_features['loss'|'command'|'error'];
 *   prediction (B*N) sample-major = loss_features['prediction']  (Functions.py:1466);
 *   xhat (B,N,4) per-step LSTM predictions (closed-loop state trajectory), or NULL.
 * with_backward != 0 keeps the activations fcr_backward needs in `ws` (which must then not be
 * reused until fcr_backward has run).
 */
int fcr_forward(const fcr_dims *dims, fcr_options *opts, const fcr_weights *w,
                const float *X, const float *u0, const float *states, const float *noise,
                float *loss, float *cost, float *command, float *error,
                float *prediction, float *xhat,
                int with_backward, void *ws, size_t ws_bytes, void *stream);

/*
 * Backward of the last fcr_forward(with_backward=1) on the same `ws` = what loss.backward()
 * (Functions.py:655) delivers: d loss/d u0 (B,1) — handed back to the caller's controller(X) graph —
 * and the gradients of the controller parameters used inside the loss. `dloss` is a DEVICE pointer
 * to the incoming scalar gradient (no host sync). LSTM weight gradients are not computed (the
 * reference computes them but nothing reads them: UL/Main.py:195 optimises only the controller).
 * Parameter gradients are OVERWRITTEN (not accumulated); reduction order is fixed (deterministic).
 */
int fcr_backward(const fcr_dims *dims, fcr_options *opts,
                 const float *X, const float *states, const float *prediction,
                 const float *dloss,
                 float *g_u0, float *g_w_inp, float *g_b_inp, float *g_w_out,
                 void *ws, size_t ws_bytes, void *stream);

/*
 * The caller's controller call `output = model(X)` (Functions.py:643): FNNModel.forward
 * (Functions.py:261-289) at the reference's shape — Linear(in_dim=3 -> hidden) + ReLU,
 * Linear(hidden -> 1, no bias) + Hardtanh (UL/Main.py:188, width_dim = 1); hidden <= 64.
 *   X (B,3), w_inp (hidden,3), b_inp (hidden), w_out (1,hidden) -> u (B,1)
 * fcr_fnn_backward is its autograd backward for g_u = dL/du (B,1): the parameter gradients
 * (OVERWRITTEN, fixed reduction order) and g_x = dL/dX (B,3), or NULL to skip it. Hardtanh'(±1) = 0,
 * ReLU'(0) = 0 (torch). Scratch: fcr_fnn_workspace_size bytes.
 */
int fcr_fnn_workspace_size(int32_t B, int32_t hidden, size_t *bytes);
int fcr_fnn_forward(int32_t B, int32_t in_dim, int32_t hidden, const float *X, const float *w_inp,
                    const float *b_inp, const float *w_out, float *u, void *stream);
int fcr_fnn_backward(int32_t B, int32_t in_dim, int32_t hidden, const float *X, const float *w_inp,
                     const float *b_inp, const float *w_out, const float *g_u, float *g_x, float *g_w_inp,
                     float *g_b_inp, float *g_w_out, void *ws, size_t ws_bytes, void *stream);

/*
 * Batched forging-press plant: the state update x_{t+1} = F(x_t, u_t) of
 * FeasibilityRecovery.Ruge_Kuta (Functions.py:1743-1781) over the dynamics of forging_model
 * (Functions.py:1615-1740; smooth = 1: template_model.py:19-149, pressures floored by smooth_relu),
 * for B independent trajectories of S steps, in fp64.
 *   x0 (B,5)       initial states [y, y_dot, p1, p2, z]
 *   u  (B,S)       command held over each step
 *   x  (B,S+1,5)   x[:,0] = x0, x[:,t+1] = F(x[:,t], u[:,t])
 *   ts             step (the reference: TS = controller t_step = 0.001, template_mpc.py:23)
 *   substeps       RK4 stages per step (the reference: M = 4, Functions.py:1760)
 * B = 0 is a no-op. Buffers are fp64 device memory, 8-byte aligned.
 */
int fcr_plant_rk4(int32_t B, int32_t S, double ts, int32_t substeps, int32_t smooth,
                  const double *x0, const double *u, double *x, void *stream);

/*
 * Batched closed-loop evaluation (SURVEY.md §8(f) ranks 1 + 2): NeuralNetwork.loop (Functions.py:
 * 1075-1240) without feasibility recovery — per step the FNN controller on the MaxAbs-scaled
 * [y_dot, z, ref] (NN_make_step, :1560-1613; fp32 like torch) and the press advanced by the RK4
 * integrator of fcr_plant_rk4 (in place of do-mpc's CVODES) — for B trajectories × T steps, one launch.
 *   x0 (B,5), ref (B,T) unscaled speed references (NeuralNetwork.tvp_fun, :926-966, computed by the
 *   caller); controller weights as fcr_weights; in_scale = scalers['input'].scale_[0:2] (y_dot, z),
 *   ref_scale = scalers['y_dot'].scale_, out_scale = scalers['output'].scale_ (UL/Main.py:237-256);
 *   outputs x (B,T+1,5) with x[:,0] = x0 and u (B,T) the commands applied. fp64 buffers, fp32 weights.
 */
typedef struct fcr_closed_loop {
    int32_t B, T;
    double ts;
    int32_t substeps, smooth;
    const double *x0, *ref;
    const float *ctrl_w_inp, *ctrl_b_inp, *ctrl_w_out;
    int32_t ctrl_hidden;
    double in_scale[2];
    double ref_scale, out_scale;
    double *x, *u;
} fcr_closed_loop;

int fcr_closed_loop_run(const fcr_closed_loop *args, void *stream);

/*
 * Training-sample windows: the tables of the concatenated per-trajectory
 * SequenceDatasets (Functions.py:92-132, built by Data.get_individual_dataset :479-516 and
 * ConcatDataset, UL/Main.py:270-279), resident in device memory.
 *   X (rows, nx) features [y_dot, z, ref]; Y (rows, ny) target; Z (rows, nz) recurrent features;
 *   rows = trajectories · traj_len (T_TRAJ rows each); lookback = window rows (10, UL/Main.py:267).
 */
typedef struct fcr_windows {
    int64_t rows;
    int32_t traj_len;
    int32_t lookback;
    int32_t nx, ny, nz;
    const float *X, *Y, *Z;
} fcr_windows;

/*
 * Batch gather = SequenceDataset.__getitem__ (Functions.py:109-132) for every global index idx[b]
 * (trajectory k = idx / traj_len, row i = idx % traj_len):
 *   x[b] = X[i],  y[b] = Y[min(i+1, traj_len-1)],  z[b, j] = Z[max(i-lookback+1+j, 0)]   (rows of trajectory k)
 * into x (B,nx), y (B,ny), z (B,lookback,nz). `bad` (device int32) receives the number of indices outside
 * [0, rows) (their outputs are zero-filled) — the reference raises IndexError for them; the Python layer
 * checks it. Stream-ordered; B = 0 only clears `bad`.
 */
int fcr_window_gather(const fcr_windows *tables, int32_t B, const int64_t *idx,
                      float *x, float *y, float *z, int32_t *bad, void *stream);

/*
 * LSTM surrogate training step: what one iteration of
 * NeuralNetwork.train_model (Model_NN/Functions.py:520-569) asks of LSTMModel (Model_NN/Functions.py:
 * 255-330, trained by Model_NN/Main.py:218-242): the forward on a window batch and loss.backward() into
 * every weight. `dims` uses B, H, L (=10), layers (=3), in_dim (=5), out_dim (=4); the controller fields
 * are ignored. Weights: fcr_weights' w_ih/w_hh/fc_w/fc_b (the controller pointers are ignored).
 *   x  (B,10,5)  windows          y (B,4) = fc(h_9 of the top layer) + b
 * with_backward != 0 keeps every cell's state in `ws` for fcr_lstm_backward.
 */
int fcr_lstm_workspace_size(const fcr_dims *dims, int with_backward, size_t *bytes);
int fcr_lstm_forward(const fcr_dims *dims, const fcr_weights *w, const float *x, float *y,
                     int with_backward, void *ws, size_t ws_bytes, void *stream);

/*
 * Backward of the last fcr_lstm_forward(with_backward=1) on the same `ws` and weights, given dy = dL/dy
 * (B,4): gradients of weight_ih_l{0,1,2} (4H,5|H), weight_hh_l{0,1,2} (4H,H), fc.weight (4,H), fc.bias (4),
 * OVERWRITTEN, fixed reduction order; g_x (B,10,5) = dL/dx, or NULL to skip it.
 */
int fcr_lstm_backward(const fcr_dims *dims, const fcr_weights *w, const float *dy,
                      float *const *g_w_ih, float *const *g_w_hh, float *g_fc_w, float *g_fc_b, float *g_x,
                      void *ws, size_t ws_bytes, void *stream);

/*
 * Process-wide DEFAULTS of the per-call options (a field set to FCR_OPT_INHERIT takes them).
 * Small batches (fp32-accurate mode, H 17..52): B <= max_batch runs the small-batch kernels, which split each
 * 16-trajectory group's cell over the four waves of a workgroup (the reference trains at B = 15, UL/Main.py:84,297);
 * larger B runs the fused one-wave-per-group kernels. Default 8192; 0 = never (negative clamps to 0). Returns the
 * previous value; fcr_get_small_batch_limit reads it without changing it.
 */
int fcr_set_small_batch_limit(int32_t max_batch);
int fcr_get_small_batch_limit(void);

/* Within the small-batch family, B <= max_batch (and at most 32 groups of 16 trajectories, 3 workgroups each within
 * half the device's CUs) runs the layer-pipelined geometry (csrc/fcr_pipe.h: one workgroup per LSTM layer and window
 * set, the layers and windows as a wavefront; results bit-identical to the one-workgroup-per-group kernels). Default
 * 512; 0 = never.
 * Process-wide; returns the previous value; fcr_get_small_pipe_limit reads it. */
int fcr_set_small_pipe_limit(int32_t max_batch);
int fcr_get_small_pipe_limit(void);

/* The pipelined geometry's window sets S: set s takes windows s, s + S, ... so windows run concurrently (every window
 * is an LSTM run from zero state; only the prediction feedback is serial); the forward runs 2 S workgroups per group
 * (S <= 4), the backward 3 S (S <= 3). 0 (default) = the most that fit (within half the CUs, S <= N); k > 0 caps S at
 * k. Results are bit-identical for every S. Process-wide; returns the previous value; fcr_get_small_pipe_sets reads
 * it. */
int fcr_set_small_pipe_sets(int32_t sets);
int fcr_get_small_pipe_sets(void);

/*
 * H > 52 (the batch-wide GEMM path): how many bytes of "kept windows" fcr_workspace_size(with_backward = 1)
 * may add. The backward recomputes each window's cells from a per-window checkpoint (the rollout's memory
 * floor); a kept window instead holds the forward's gate activations and c for all its 30 cells
 * (30 B 5H floats: 10 GB at B = 65 536, H = 256 — torch's autograd keeps at least that for every window),
 * so its backward skips the recompute (config 5: a third of the step). The last windows are kept, as many
 * as the budget allows (fcr_wide_kept_windows).
 * bytes < 0 (FCR_KEEP_AUTO, the default): as many as keep the whole workspace within half of the memory that was
 * free on the device when a workspace was first sized there (cached per device: a stable count from call to call),
 * and within 40 % of the device's total memory; 0: keep none. The workspace stays allocated from the forward until
 * its backward has run (torch: until RolloutFn.backward releases it). Returns the previous budget.
 */
int64_t fcr_set_wide_keep_budget(int64_t bytes);
int64_t fcr_get_wide_keep_budget(void);

/*
 * TEST HOOK (not a reference interface; nothing on the rollout path calls it): ONE backward cell of the H > 52 path,
 * i.e. the autograd backward of one nn.LSTM cell (Functions.py:325, inside loss.backward() at :655), run by the same
 * kernel and launcher fcr_backward uses (wide_bwd_fused_kernel), on caller-given inputs, so a test can compare every
 * output element with an fp64 evaluation. H % 8 == 0, H <= 2048 (the fused cell's tiling). Per trajectory b:
 *   act (B,H,4) gate activations (i, f, g, o) = (sigmoid, sigmoid, tanh, sigmoid) of each unit's pre-activations, in
 *               the [unit][gate] layout the forward cell saves them;  c_prev (B,H) or NULL (t = 0);
 *   dh (B,H) incoming dh_t of the recurrence;  din (B,H) the layer above's input gradient at t, or NULL;
 *   dc (B,H) carried dc_t;  ->  dc_out (B,H) = dc_{t-1};
 *   layer0 == 0: out (B,2H) = dG [W_ih | W_hh] (input gradient | dh_{t-1}; only the first H columns without c_prev),
 *                w_ih (4H,H), w_hh (4H,H);
 *   layer0 != 0: out (B,H) = dG W_hh (dh_{t-1}; not written without c_prev), rowg (B,5) = dG W_ih0 (overwritten),
 *                w_ih = W_ih0 (4H,5), w_hh (4H,H).
 * dG are the gate gradients of the cell update c = f c_prev + i g, h = o tanh(c) for dh + din and dc. Scratch:
 * fcr_wide_bwd_cell_workspace bytes, 256-byte aligned.
 */
int fcr_wide_bwd_cell_workspace(int32_t B, int32_t H, int32_t layer0, size_t *bytes);
int fcr_wide_bwd_cell(int32_t B, int32_t H, int32_t layer0, const float *w_ih, const float *w_hh, const float *act,
                      const float *c_prev, const float *dh, const float *din, const float *dc, float *out,
                      float *dc_out, float *rowg, void *ws, size_t ws_bytes, void *stream);

/* Thread-local description of the last error (never NULL). */
const char *fcr_last_error(void);

/* FCR_ABI_VERSION of the loaded library. */
int fcr_abi_version(void);

#ifdef __cplusplus
}
#endif
#endif /* FCR_H */
