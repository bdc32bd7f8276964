/* fall3 — MI355X-native (gfx950) 3-stream fall-detection training step: C ABI.
 *
 * This is the drop-in boundary for the reference's model/step interface
 * (/root/reference/Multimodal_Fall3/model/...). Each entry point replaces one call of
 * the reference training loop (model/main.py:91-148):
 *
 *   f3_net_create      <- build_model(config)            model/build_model.py:5-19
 *   f3_net_entry       <- model.state_dict() keys/shapes  (same names, order, shapes)
 *   f3_net_forward     <- pred = model(data, sensor)      model/main.py:112, combination.py:37-46
 *   f3_net_loss        <- loss_fn(pred, label_onehot)     model/main.py:113,280 (CE, soft targets)
 *   f3_net_backward    <- loss.backward()                 model/main.py:115
 *   f3_rmsprop_step    <- optimizer.step()                model/main.py:127, optimizer.py:21
 *   f3_net_backward_rmsprop <- loss.backward(); optimizer.step()  (one GPU: the update per layer
 *                              as soon as its gradients are final)
 *
 * Conventions: plain pointers to device memory (HIP), sizes in elements, a HIP stream
 * passed as void*. No call allocates, frees or synchronises: every buffer (flat
 * parameters, flat grads, BN buffers, workspace) is owned by the caller, so a full
 * step can be captured into a HIP graph. Every function returns 0 on success or an
 * F3_E* status (never aborts); f3_status_string() names it.
 */
#ifndef FALL3_H
#define FALL3_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define F3_OK 0
#define F3_EINVAL 1001 /* bad argument / unsupported shape */
#define F3_EBATCH 1002 /* train-mode batch of 1: BatchNorm needs >1 value per channel */
#define F3_EHIP 1003   /* HIP launch error */
#define F3_ESTATE 1004 /* backward without a training forward on this workspace */
#define F3_EDEVICE 1005 /* a device-side check failed (a group barrier of the TARGCN GRU or the sensor CNN1D timed out) */

enum { F3_MODEL_TWO_STGCAN_BILSTM = 0, F3_MODEL_TWO_STGCAN = 1, F3_MODEL_STGCN = 2, F3_MODEL_BILSTM = 3 };
enum { F3_SENSOR_NONE = 0, F3_SENSOR_BILSTM = 1, F3_SENSOR_CNN_BILSTM = 2 };
enum { F3_NAMING_PACKAGE = 0, F3_NAMING_NOTEBOOK = 1 };
enum { F3_PRECISION_FP32 = 0, /* exact fp32 MFMA (v_mfma_f32_16x16x4_f32): parity mode */
       F3_PRECISION_BF16 = 1, /* bf16 GEMM operands in HBM, fp32 accumulate (v_mfma_f32_16x16x32_bf16) */
       F3_PRECISION_BF16_FP32IN = 2, /* kernel-level entries only: bf16 arithmetic on fp32 activations */
       F3_PRECISION_BF16X3 = 4 /* split-bf16 parity mode: fp32 activations, every GEMM operand split into
                                  bf16 hi + lo, products hi*hi + hi*lo + lo*hi on v_mfma_f32_16x16x32_bf16
                                  with fp32 accumulate (~2^-16 per product; gemm_x3.hip) */ };
enum { F3_ENTRY_PARAM = 0, F3_ENTRY_BUFFER = 1, F3_ENTRY_COUNTER = 2 };

typedef struct f3_config {
  int model;           /* F3_MODEL_*  (build_model.py:9-17 MODEL.NAME) */
  int num_node;        /* V: 14 coco_cut, 18 coco_mmpose (graph.py:24-49) */
  int num_partition;   /* K: 1 uniform, 2 distance, 3 spatial (graph.py:50-90) */
  int num_class;       /* DATA.NUM_CLASSES */
  int in_channels;     /* DATA.IN_CHANNELS (stgcn model) */
  int sensor;          /* F3_SENSOR_* */
  int sensor_dim;      /* DATA.SENSOR_DIM */
  int sensor_classes;  /* BiLSTM head width (package: num_class; UR notebook: 2) */
  int softmax_output;  /* notebook form returns softmax (GSTCAN_HAR_conv_10kfold.ipynb:444) */
  int naming;          /* F3_NAMING_* state_dict prefixes */
  int frames;          /* skeleton window T (30) */
  int sensor_frames;   /* IMU window Ts (30) */
  int precision;       /* F3_PRECISION_*: GEMM operand type of the skeleton streams' convs */
} f3_config;

typedef struct f3_net f3_net;

int f3_net_create(const f3_config* cfg, f3_net** out);
void f3_net_destroy(f3_net* net);

/* state_dict table: entries in reference order. kind = F3_ENTRY_*; offset indexes the
 * flat fp32 parameter array (PARAM), the flat fp32 buffer array (BUFFER: A, running
 * stats) or the flat int64 counter array (COUNTER: num_batches_tracked). */
int f3_net_num_entries(const f3_net* net);
int f3_net_entry(const f3_net* net, int i, const char** name, int* kind, int* ndim, int64_t* shape8,
                 int64_t* offset);
int64_t f3_net_param_count(const f3_net* net);
int64_t f3_net_buffer_count(const f3_net* net);
int64_t f3_net_counter_count(const f3_net* net);
int64_t f3_net_workspace_bytes(const f3_net* net, int batch);

/* Forward. skel f32[N,3,T,V] (reference layout), sensor f32[N,Ts,S] (ignored without a
 * sensor stream), out f32[N,C] (logits, or softmax for softmax_output). training=1 uses
 * batch statistics and updates running stats / num_batches_tracked in place (momentum
 * 0.1); training=0 uses running statistics. The workspace keeps what backward needs. */
int f3_net_forward(f3_net* net, int batch, int training, const float* params, float* buffers, int64_t* counters,
                   const float* skel, const float* sensor, float* out, void* workspace, void* stream);

/* loss = -(1/N) sum_i sum_c y_ic log_softmax(out_i)_c ; dout = dloss/dout. */
int f3_net_loss(f3_net* net, int batch, const float* out, const float* label, float* loss, float* dout,
                void* stream);

/* Backward of the last training forward on `workspace`: grads (flat, same layout as
 * params) are OVERWRITTEN with d(sum dout*out)/dparams. */
int f3_net_backward(f3_net* net, int batch, const float* params, const float* dout, float* grads,
                    void* workspace, void* stream);

/* Timing of the sensor CNN1D stages (GSTCAN_UR_conv.ipynb:493-514; models with the CNN1D
 * sensor branch only). enable=1 records HIP events around the Conv1D launches of every later
 * forward / backward on the sensor queue; ms (may be NULL) receives the last forward + backward's
 * 2 times in ms: both CNN1D layers forward, both backward (one cooperative launch each in
 * training; the per-layer launches in eval or under stream capture). No reference counterpart:
 * measurement only. */
int f3_net_sensor_times(f3_net* net, int enable, float* ms);

/* The same backward in two phases, for overlapping the data-parallel gradient all-reduce
 * with compute: phase 1 = zero grads, head, sensor branch and skeleton layers 4-6 (their
 * gradients, params[0 .. f3_net_grad_split) in the flat buffer); phase 2 = skeleton layers 0-3
 * and data_bn (the rest). phase 0 = both (f3_net_backward). Parameter offsets are laid out
 * phase-1-first; state_dict order is unchanged.
 * Phase 1 returns WITHOUT ordering `stream` after its private queues (the weight-gradient queues
 * keep draining while phase 2's critical path starts): make the all-reduce stream wait with
 * f3_net_wait_phase1 before reducing params[0 .. split). Phase 2 ends with `stream` ordered after
 * all work of both phases. */
int f3_net_backward_phase(f3_net* net, int batch, const float* params, const float* dout, float* grads,
                          void* workspace, int phase, void* stream);
int64_t f3_net_grad_split(const f3_net* net);
int f3_net_wait_phase1(f3_net* net, void* stream);

/* The single-GPU step's backward and optimizer in one call: f3_net_backward followed by
 * f3_rmsprop_step(params, square_avg, grads, nparam, lr, alpha, eps, 1.0) (loss.backward() +
 * optimizer.step(), model/main.py:115-127), except that each skeleton layer's RMSprop update is
 * issued on the queue that finishes that layer's gradients, as soon as they are final, instead of
 * after the whole backward; the rest (data_bn, sensor branch, head) follows the join. grads holds
 * the step's gradients afterwards as with f3_net_backward. Identical updates; not for data
 * parallelism (the all-reduce must come between the two). */
int f3_net_backward_rmsprop(f3_net* net, int batch, float* params, const float* dout, float* grads, float* square_avg,
                            void* workspace, float lr, float alpha, float eps, void* stream);
/* 1 if f3_net_backward_rmsprop issues the per-layer updates, 0 if it falls back to the backward
 * followed by one update (fixed by the parameter layout and precision; planned once per net). */
int f3_net_fused_rmsprop(f3_net* net);

/* The F3_PRECISION_* the net was created with (reads back f3_config.precision; -1 for NULL). */
int f3_net_precision(const f3_net* net);

/* Device status of the last training forward / backward (the sensor branch's cooperative CNN1D:
 * its group barriers time out instead of hanging when the workgroups cannot all be resident; the
 * launch then writes NaN into its outputs). Returns F3_EDEVICE if a copy of that error word flagged
 * a timeout (wait = 1: after every enqueued copy has completed; 0: those that have). Every
 * f3_net_forward / _backward* also returns F3_EDEVICE once when it finds a completed, flagged copy
 * from an earlier call. No reference counterpart: the reference's nn.Conv1d cannot fail this way
 * (GSTCAN_UR_conv.ipynb:493-514). */
int f3_net_status(f3_net* net, int wait);

/* torch.optim.RMSprop(lr, alpha, eps), no momentum / weight decay / centering, on
 * g = grad_scale * grads (1.0 = torch semantics; 1/world after a summed all-reduce):
 * sq = alpha*sq + (1-alpha)*g^2 ; p -= lr*g/(sqrt(sq)+eps). */
int f3_rmsprop_step(float* params, float* square_avg, const float* grads, int64_t n, float lr, float alpha,
                    float eps, float grad_scale, void* stream);

/* Kernel-level entries used by the unit tests and bench.py: out[N,T_out,V,Cout] = conv_(KT,1)(x)
 * with x [N,T_in,V,Cin] channels-last, w in reference layout [Cout][Cin][KT], bias [Cout]
 * (stgcan.py:24-31 tcn Conv2d). wpack is scratch of Cout*KT*Cin floats for the packed
 * operand; w == NULL reuses what a previous call packed there. precision = F3_PRECISION_*:
 * FP32 -> x/dy are fp32; BF16 -> x/dy are bf16 (the network's bf16 operand tensors);
 * BF16_FP32IN -> fp32 x/dy rounded to bf16 while staging; BF16X3 -> fp32 x/dy, split-bf16 products (wpack
 * then holds the bf16 hi and lo planes of the packed weight). f3_conv_forward also takes
 * F3_CONV_BF16_OUT (bf16 x, out written as bf16 [N,T_out,V,Cout]: the step's tcn output type). */
enum { F3_CONV_BF16_OUT = 3 };
int f3_conv_forward(const void* x, const float* w, const float* bias, float* out, float* wpack, int N, int T_in,
                    int V, int Cin, int Cout, int KT, int stride, int pad, int precision, void* stream);

/* Its gradients: dx = conv^T(dy) [N,T_in,V,Cin]; dw [Cout][Cin][KT] and db [Cout] (overwritten). */
int f3_conv_backward_data(const void* dy, const float* w, float* dx, float* wpack, int N, int T_in, int V, int Cin,
                          int Cout, int KT, int stride, int pad, int precision, void* stream);
int f3_conv_backward_weight(const void* dy, const void* x, float* dw, float* db, int N, int T_in, int V, int Cin,
                            int Cout, int KT, int stride, int pad, int precision, void* stream);
/* The bf16 weight-gradient kernel alone, as the training step launches it per layer: each
 * split of the rows writes its partial dW tile to slab[split][Cout][KT*Cin] (plain stores; the
 * step then sums the splits with a separate reduce launch, not done here). bf16 dy / x;
 * requires Cout % 64 == 0, Cin % 64 == 0, slab_floats >= Cout*KT*Cin. Used to time the kernel. */
int f3_conv_wgrad_packed(const void* dy, const void* x, float* slab, long long slab_floats, int N, int T_in, int V,
                         int Cin, int Cout, int KT, int stride, int pad, void* stream);

/* F3_PRECISION_BF16X3 as the training step runs it (the native split form on the bf16 LDS-DMA kernels):
 * f3_split_x3cat writes each fp32 row x[r][0..C) as the bf16 row of 2C made of 32-channel blocks
 * [x_hi 32 | x_lo 32] (hi = RNE bf16(x), lo = RNE bf16(x - hi)); the packed weight holds, per tap, the
 * blocks [W_hi 32 | W_lo 32] (prep code 4), and a k step issues x_hi W_hi + x_lo W_hi + x_hi W_lo (the
 * split product, ~2^-16 relative) from one staged row piece.
 * f3_conv_forward_x3cat / f3_conv_backward_data_x3cat: x3 / dy3 are such rows ([N,T,V,2Cin] /
 * [N,T_out,V,2Cout]); wpack is scratch of 2 * Cout*KT*Cin bf16 (w == NULL reuses it); out / dx
 * fp32 as f3_conv_forward / f3_conv_backward_data (bias required, epilogue + bias).
 * f3_conv_backward_weight_x3cat: the bf16 weight-gradient GEMM on the same rows, dy_hi x_hi + dy_lo
 * x_hi + dy_hi x_lo (split-K partials summed into dw [Cout][Cin][KT]; db from dy_hi + dy_lo; both
 * overwritten, db may be NULL). dw == NULL: the GEMM alone at the step's split count, partials left in
 * an internal slab (timing). Requires Cin, Cout multiples of 64.
 * f3_conv_step_x3cat: two GEMMs with the epilogues the step gives them, launched alone (measurement,
 * SURVEY §8d; bench.py roofline keys), through the step's own dispatch:
 *   kind F3_STEP_GCN_FWD (stgcan.py:50-56): the gcn 1x1 conv over the graph-mixed rows in3 = [Z_hi | Z_lo]
 *     of Cin = K*C_in channels, out = conv + bias_v[(row % V)][Cout] (the graph-mixed bias), the BN1
 *     batch sums of out added into st_sum / st_sq (fp64); w [Cout][Cin] (T = the frames);
 *   kind F3_STEP_TCN_DGRAD (stgcan.py:112-121, backward): the (9,1) tcn input gradient, stride 1, from
 *     in3 = dh rows of Cout channels into out = dv [N,T,V,Cin], masked where bn1(g) <= 0 (g fp32
 *     [N,T,V,Cin]; BN from gamma / beta and the batch sums bn_sum / bn_sq over bn_count values) with
 *     the BN1-backward sums sum(dv), sum(dv * g_hat) added into st_sum / st_sq; w [Cout][Cin][9].
 *   gcn-only / dgrad-only pointers may be NULL for the other kind. */
#define F3_STEP_GCN_FWD 0
#define F3_STEP_TCN_DGRAD 1
int f3_split_x3cat(const float* x, void* out, int64_t rows, int C, void* stream);
int f3_conv_forward_x3cat(const void* x3, const float* w, const float* bias, float* out, void* wpack, int N, int T_in,
                          int V, int Cin, int Cout, int KT, int stride, int pad, void* stream);
int f3_conv_backward_data_x3cat(const void* dy3, const float* w, float* dx, void* wpack, int N, int T_in, int V,
                                int Cin, int Cout, int KT, int stride, int pad, void* stream);
int f3_conv_backward_weight_x3cat(const void* dy3, const void* x3, float* dw, float* db, int N, int T_in, int V,
                                  int Cin, int Cout, int KT, int stride, int pad, void* stream);
int f3_conv_step_x3cat(int kind, const void* in3, const float* w, void* wpack, float* out, const float* bias_v,
                       const float* g, const float* gamma, const float* beta, const double* bn_sum,
                       const double* bn_sq, float bn_count, double* st_sum, double* st_sq, int N, int T, int V,
                       int Cin, int Cout, void* stream);

/* The 1x1 conv GEMM of the bf16 step with the step's epilogues (stgcan.py:50-56 gcn conv, its
 * input gradient; stgcan.py:123-144 stride-2 residual conv and its input gradient), through the
 * step's own dispatch (the weight-stationary pw_gemm kernel where the shape allows, else igemm).
 * x bf16 [N,T_in,V,Cin] rows; wpack bf16 [Cout][Cin]; out [N,T_out,V,Cout], bf16 (out_bf16 = 1) or
 * fp32. transposed = 0: forward, T_out = (T_in - 1) / stride + 1; transposed = 1: input gradient of a
 * stride-`stride` 1x1 conv whose input had T_out frames. epi: 0 plain, 1 + bias[Cout], 5 + bias with
 * BN sums, 6 + per-joint bias[V][Cout] with BN sums, 32 out += (fp32 out). st_sum / st_sq: fp64
 * [Cout] sums of the fp32 outputs, accumulated (+=). */
int f3_pointwise_conv(const void* x, const void* wpack, const float* bias, void* out, int out_bf16, double* st_sum,
                      double* st_sq, int N, int T_in, int T_out, int V, int Cin, int Cout, int stride, int transposed,
                      int epi, void* stream);

/* RGB spatial-conv branch (BUILD-DEFINED: the reference has RGB frames only in preprocessing,
 * 3_stream/har_create3.py:36-42,101-158, so its parity is unpinned; the north star names it).
 * frames bf16 [B][T][224][224][3]; wpack bf16 [64][192] (the Conv2d(3, 64, 8, stride 8) weight
 * [64][3][8][8] with k = (dy*8 + dx)*3 + ch); feat[B][64] = mean over frames and the 28 x 28 patch
 * grid of relu(conv + bias) (overwritten). The backward gives dw [64][192] (packed order) and
 * db [64] (overwritten) from dfeat [B][64]; scratch holds f3_rgb_scratch_floats(B, T) floats. */
long long f3_rgb_scratch_floats(int B, int T);
int f3_rgb_forward(const void* frames, const void* wpack, const float* bias, float* feat, int B, int T, void* stream);
int f3_rgb_backward(const void* frames, const void* wpack, const float* bias, const float* dfeat, float* dw, float* db,
                    float* scratch, long long scratch_floats, int B, int T, void* stream);

/* Graph mix of one st_gcan block (stgcan.py:54, applied to the gcn input):
 * z[f][w][k][ci] = sum_v A_eff[k][v][w] x[f][v][ci]; backward gives dx and dA_eff (overwritten). */
int f3_graph_mix_forward(const float* A_eff, const float* x, float* z, int frames, int K, int V, int Cin,
                         void* stream);
int f3_graph_mix_backward(const float* A_eff, const float* x, const float* dz, float* dx, float* dA, int frames, int K,
                          int V, int Cin, void* stream);
/* The same with the bf16 mode's operand types: F3_MIX_X_BF16 -> x (and, backward, dz) bf16;
 * F3_MIX_Z_BF16 -> forward z written bf16 (the gcn GEMM's operand, as the step stores it);
 * F3_MIX_X3 -> fp32 operands on the bf16x3 (split-bf16) MFMA kernels of F3_PRECISION_BF16X3;
 * F3_MIX_Z3 (with F3_MIX_X3) -> forward z written as the step stores it for the gcn GEMM: per (frame,
 * node) one bf16 row [z_hi | z_lo] of 2 K Cin (z_hi = RNE bf16(z), z_lo = RNE bf16(z - z_hi)). */
enum { F3_MIX_X_BF16 = 1, F3_MIX_Z_BF16 = 2, F3_MIX_X3 = 4, F3_MIX_Z3 = 8 };
int f3_graph_mix_forward_ex(const float* A_eff, const void* x, void* z, int frames, int K, int V, int Cin, int flags,
                            void* stream);
int f3_graph_mix_backward_ex(const float* A_eff, const void* x, const void* dz, float* dx, float* dA, int frames, int K,
                             int V, int Cin, int flags, void* stream);

const char* f3_status_string(int status);

/* ---- TARGCN skeleton model (BASELINE config 2; TRAGCN.py, EmbGCN.py, GRU.py, TA.py) ----
 * f3_targcn_create      <- TARGCN(adj=None, num_nodes=V)          TRAGCN.py:177-205
 *                          (the notebook's call, TARGCN_HAR_conv_10kfold.ipynb cell 3)
 * f3_targcn_entry       <- model.state_dict() keys/shapes (same names, order, shapes;
 *                          PARAM offsets 16-B aligned in the flat parameter array)
 * f3_targcn_forward     <- out = model(pts.permute(0,2,3,1))      TRAGCN.py:207-224
 * f3_targcn_backward    <- loss.backward()
 * f3_soft_ce            <- torch.nn.CrossEntropyLoss()(out, soft labels)
 * Optimizer: f3_rmsprop_step (the notebook's RMSprop). precision: F3_PRECISION_FP32 (exact fp32
 * MFMA, parity mode) or F3_PRECISION_BF16 (bf16 GEMM operands, fp32 accumulate and state). */
typedef struct f3_targcn_config {
  int num_node;   /* V (2..18) */
  int num_class;  /* fc output width */
  int precision;  /* F3_PRECISION_FP32 | F3_PRECISION_BF16 */
} f3_targcn_config;

typedef struct f3_targcn f3_targcn;

int f3_targcn_create(const f3_targcn_config* cfg, f3_targcn** out);
void f3_targcn_destroy(f3_targcn* net);
int f3_targcn_num_entries(const f3_targcn* net);
int f3_targcn_entry(const f3_targcn* net, int i, const char** name, int* kind, int* ndim, int64_t* shape8,
                    int64_t* offset);
int64_t f3_targcn_param_count(const f3_targcn* net);
int64_t f3_targcn_buffer_count(const f3_targcn* net);
int64_t f3_targcn_workspace_bytes(const f3_targcn* net, int batch);
/* source f32[B,T=30,V,3] (the notebook's pts.permute(0,2,3,1)), out f32[B,num_class] logits.
 * TARGCN has no batch statistics or dropout: train and eval forwards are the same computation;
 * the workspace keeps what backward needs. */
int f3_targcn_forward(f3_targcn* net, int batch, const float* params, const float* buffers, const float* source,
                      float* out, void* workspace, void* stream);
/* grads (flat, params layout) are OVERWRITTEN with d(sum dout*out)/dparams of the last forward. */
int f3_targcn_backward(f3_targcn* net, int batch, const float* params, const float* buffers, const float* dout,
                       float* grads, void* workspace, void* stream);
/* Stage timing (measurement aid, no reference counterpart): enable != 0 records HIP events around the
 * two GRU recurrences and the two TA layers of the following f3_targcn_forward / _backward calls on
 * their stream; ms != NULL (after such a pair) waits for them and writes 8 durations in ms:
 * gru_fwd l0, gru_fwd l1, ta_fwd l0, ta_fwd l1, ta_bwd l1, ta_bwd l0, gru_bwd l1, gru_bwd l0. */
int f3_targcn_stage_times(f3_targcn* net, int enable, float* ms);
/* Device-side status of the node-partitioned GRU recurrences (no reference counterpart: the
 * reference's GRU.py:17-27 loop has no inter-workgroup barrier). Each forward clears the barrier
 * error flag; after its recurrences the forward and the backward copy it to a host status word.
 * Returns F3_EDEVICE if a group barrier of the last forward / backward timed out (its outputs are
 * then wrong), F3_OK otherwise. wait = 1 first waits for that copy; wait = 0 reports only a copy
 * that has completed. Every f3_targcn_forward / _backward also returns F3_EDEVICE (and clears
 * the word) when it finds a completed copy flagged by an earlier call. Each call's copy has its own
 * host word (a ring), so a flag is reported once even when later calls run before the host asks. */
int f3_targcn_status(f3_targcn* net, int wait);
/* loss = -(1/N) sum_i sum_c y_ic log_softmax(out_i)_c (soft targets, not renormalised);
 * dout = dloss/dout. loss is overwritten. */
int f3_soft_ce(const float* out, const float* label, int N, int C, float* loss, float* dout, void* stream);

/* ---- musa_model.Model (the model root Multimodal_Fall3/main.py trains; model/musa_model.py) ----
 * f3_musa_create   <- Model(num_class=11, num_point=14, max_frame=300, graph=adjGraph('coco_cut',
 *                     'uniform'), bias=True, edge=True, block_size=41, embed_dim=64, n_stage=1,
 *                     act_type='tanh')                                      main.py:307-320, :492-559
 * f3_musa_entry    <- model.state_dict() keys/shapes (A included: a Parameter, requires_grad False)
 * f3_musa_forward  <- pred = model(data), x f32[N,3,T,V]                   musa_model.py:561-589
 * f3_musa_backward <- loss.backward()
 * Train mode: dropout != 0 enables the DropBlocks (keep_prob 0.9, block 41) and the head's
 * Dropout(0.2), all drawn from a counter hash of `seed` (oracle/musa_cpu.py reproduces it);
 * dropout == 0 is the reference with keep_prob 1 and p = 0. fp32 arithmetic (fp32 MFMA GEMMs). */
typedef struct f3_musa_config {
  int num_point;   /* V (13..18; 14 = coco_cut) */
  int frames;      /* T (8..64; the motion stream has T-1) */
  int num_class;   /* <= 64 */
  int precision;   /* F3_PRECISION_FP32 (0) or F3_PRECISION_BF16: the streams' 1x1 convs (graph conv,
                      residuals, point convs, Sep_TCN) on bf16 MFMA with fp32 accumulate, activations fp32
                      (the root main.py trains under bf16 autocast) */
} f3_musa_config;

typedef struct f3_musa f3_musa;

int f3_musa_create(const f3_musa_config* cfg, f3_musa** out);
void f3_musa_destroy(f3_musa* net);
int f3_musa_num_entries(const f3_musa* net);
int f3_musa_entry(const f3_musa* net, int i, const char** name, int* kind, int* ndim, int64_t* shape8,
                  int64_t* offset);
int64_t f3_musa_param_count(const f3_musa* net);
int64_t f3_musa_buffer_count(const f3_musa* net);
int64_t f3_musa_counter_count(const f3_musa* net);
int64_t f3_musa_workspace_bytes(const f3_musa* net, int batch);
int f3_musa_forward(f3_musa* net, int batch, int training, const float* params, float* buffers, int64_t* counters,
                    const float* x, float* out, void* workspace, unsigned seed, int dropout, void* stream);
/* grads (flat, params layout) are OVERWRITTEN; A and the SepTemporal blocks' edge get zeros (the
 * reference leaves their .grad None: A is frozen, those edges only shape DropBlock masks). */
int f3_musa_backward(f3_musa* net, int batch, const float* params, const float* buffers, const float* dout,
                     float* grads, void* workspace, void* stream);
/* Debug: with F3_MU_GUARD=<bytes> set before the library loads, the workspace plan puts a guard band
 * of that size after every region; this lists the guard offsets (returns the count; -1 on error). */
int f3_musa_guards(const f3_musa* net, int batch, int64_t* offsets, int max);
/* Kernel-level entry (tests, bench.py roofline): the depthwise temporal conv of SepTemporal_Block /
 * Sep_TCN, Conv2d(C, C, (K,1), (S,1), (P,0), groups=C) on channels-last x [N,T_in,V,C] -> y
 * [N,T_out,V,C], w [C][K], b [C]; sums (optional, [2C] fp64, accumulated): BatchNorm batch sums of y. */
int f3_dwconv_t_forward(const float* x, const float* w, const float* b, float* y, double* sums, int N, int T_in,
                        int V, int C, int K, int S, int P, void* stream);

/* ---- SkeletonTransformer (BASELINE config 5; skeleton_transformer.py) ----
 * f3_sktr_create     <- SkeletonTransformer(3, V, T, num_class, 32, 6, 16, 8)   :360-416
 *                       (GSTCAN_HAR_conv_kfold_trans.ipynb; V=14, T=30, 11 classes)
 * f3_sktr_entry      <- model.state_dict() keys/shapes (same names, order, shapes): PARAM
 *                       (16-B aligned offsets), BUFFER (BatchNorm3d running stats), COUNTER
 *                       (num_batches_tracked, int64)
 * f3_sktr_forward    <- out = model(x), x f32[N,3,T,V,M]                          :418-435
 * f3_sktr_backward   <- loss.backward()
 * Train mode randomness is explicit: sd = 18 stochastic-depth factors [block][spatial, temporal,
 * ffn] (torchvision StochasticDepth(p, "batch"): 0 or 1/(1-p); NULL = all 1), and the FFN
 * Dropout(dropout_p) mask comes from a counter hash of (dropout_seed, block, element) that the
 * oracle reproduces (oracle/sktr_cpu.py dropout_keep). Eval mode: running statistics, no
 * randomness. fp32 arithmetic throughout (fp32 MFMA GEMMs). */
typedef struct f3_sktr_config {
  int num_joint;   /* V: spatial attention length (14, 17, 18, 30, 32 supported) */
  int frames;      /* T: temporal attention length (same set) */
  int persons;     /* M >= 1 */
  int num_class;   /* <= 64 */
  int precision;   /* F3_PRECISION_FP32 (0) or F3_PRECISION_BF16: the 6 blocks' Linear layers (qkv, merge,
                      FFN) on bf16 MFMA with fp32 accumulate, activations fp32 in HBM (cfg 5 in bf16) */
} f3_sktr_config;

typedef struct f3_sktr f3_sktr;

int f3_sktr_create(const f3_sktr_config* cfg, f3_sktr** out);
void f3_sktr_destroy(f3_sktr* net);
int f3_sktr_num_entries(const f3_sktr* net);
int f3_sktr_entry(const f3_sktr* net, int i, const char** name, int* kind, int* ndim, int64_t* shape8,
                  int64_t* offset);
int64_t f3_sktr_param_count(const f3_sktr* net);
int64_t f3_sktr_buffer_count(const f3_sktr* net);
int64_t f3_sktr_counter_count(const f3_sktr* net);
int64_t f3_sktr_workspace_bytes(const f3_sktr* net, int batch);
int f3_sktr_forward(f3_sktr* net, int batch, int training, const float* params, float* buffers, int64_t* counters,
                    const float* x, float* out, void* workspace, const float* sd, unsigned dropout_seed,
                    float dropout_p, void* stream);
/* grads (flat, params layout) are OVERWRITTEN; needs the last forward to have been a training one. */
int f3_sktr_backward(f3_sktr* net, int batch, const float* params, const float* buffers, const float* dout,
                     float* grads, void* workspace, void* stream);

/* Debug accessor for tools/tests: device pointer of a per-layer workspace tensor
 * ("x","z","g","h","r","out","att","dh","dv","dg","dZ","dres","bn1_fsum",...) or NULL. */
void* f3_net_debug_tensor(f3_net* net, int batch, void* workspace, int stream, int layer, const char* what);

#ifdef __cplusplus
}
#endif
#endif /* FALL3_H */
