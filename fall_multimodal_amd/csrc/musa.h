// musa_model.Model (the model root Multimodal_Fall3/main.py trains) kernels: internal interface.
// Reference: /root/reference/Multimodal_Fall3/model/musa_model.py.
//
// Activations are channels-last rows [N][T][V][C] fp32 (row r = (n*T + t)*V + v). The 1x1
// convolutions run on the shared fp32 MFMA GEMM (f3_conv_gemm / f3_conv_wgrad, strided row maps
// for the stride-2 residual), the A*edge graph mix on f3_mix_fwd/bwd (one partition). This file
// holds the rest: the depthwise temporal convolution (the model's HBM-bound Conv1D) with its
// BatchNorm batch sums fused, BatchNorm+activation passes, the DropBlock statistics / masks
// (counter-hash draws shared with oracle/musa_cpu.py), the tanh(drop(z1) + drop(z2)) merge of
// every block, and the classifier head.
#pragma once
#include <hip/hip_runtime.h>

#include "common.h"

namespace f3 {
namespace mu {

enum : int { ACT_NONE = 0, ACT_RELU = 1, ACT_TANH = 2, ACT_LEAKY = 3 };
constexpr float kLeaky = 0.01f;
// Per-channel batch sums are reduced workgroup (LDS) -> one of kLanes fp32 lane rows (blockIdx %
// kLanes; memory-side f32 adds) -> fp64 totals in a small finalize launch that re-zeroes the
// lanes. Measured history (depthwise conv, C=128, B=256): thousands of workgroups adding into 2C
// fp64 addresses serialised (37 us of a 57 us launch); an in-kernel ticketed finalize (last
// arriver per XCD group, then last group) cost more than the separate launch (39.7 vs 27 + 5 us).
constexpr int kLanes = 256, kLaneRow = 512;   // 2C <= kLaneRow
constexpr size_t kLaneFloats = (size_t)kLanes * kLaneRow;

// depthwise temporal convolution (Conv2d(C, C, (K,1), (S,1), (P,0), groups=C)) over [N][T][V][C]
struct DwConvArgs {
  int N, T_in, T_out, V, C, K, S, P;
  const float* x;      // [N][T_in][V][C]
  const float* w;      // [C][K]   (reference [C][1][K][1])
  const float* b;      // [C]
  float* y;            // fwd out [N][T_out][V][C]
  double* sum; double* sumsq;   // fwd: BatchNorm batch sums of y (accumulated)
  float* lanes;        // fwd: lane scratch (kLaneFloats) when sum is set
  const float* dy;     // bwd in
  float* dx; int dx_add;        // bwd: input gradient (overwrite or +=)
  float* part;         // bwd: per-workgroup weight-gradient partial rows [grid][C*(K+1)]
  int part_rows;       // (out) rows written to part
  int grid, block;     // set by the launcher (kernels must not read gridDim / blockDim after their stores)
};

// y = act(BN(u)) (+ add)
struct BnActArgs {
  long long R; int C;
  const float* u;
  BnRef bn;
  int act;
  float* y;
  const float* add;
};

// backward of y = act(BN(u)): dz = dy * act'(BN(u)); du = BN'(dz) (+= add); gamma/beta grads
struct BnActBwdArgs {
  long long R; int C;
  const float* dy;
  const float* u;
  BnRef bn;
  int act;
  double* s_dz; double* s_dzx;  // [C] each (zeroed by the caller)
  float* lanes;                 // lane scratch (kLaneFloats)
  float* du; const float* add;
  float* g_gamma; float* g_beta;
  int grid;            // set by the launcher
};

// a[r] = sum_c |z[r][c]|, z = BN(u) (or u when bn_on == 0): DropBlock statistics
struct AbsStatArgs {
  long long R; int C;
  const float* u;
  BnRef bn; int bn_on;
  float* a;
};

// Randomized_DropBlock_Ske then Randomized_DropBlockT_1d as factors fS[n][v], fT[n][t]
struct DropMaskArgs {
  int N, T, V, C;
  const float* a;      // [N][T][V] sum_c |z|
  const float* Ae;     // [V][V] = A * edge
  unsigned seed; int call;
  float keep_prob; int block_size;
  float* fS; float* fT;
  float* scr;          // f3_mu_dropmask_scratch_floats(N, T, V) floats
};

// out = tanh(f1 * z1 + f2 * z2), z1 = BN1(u1), z2 = BN2(u2) or u2; f = fS[n][v] * fT[n][t] (or 1)
struct MergeArgs {
  int N, T, V, C;
  const float* u1; BnRef bn1; const float* fS1; const float* fT1;
  const float* u2; BnRef bn2; int bn2_on; const float* fS2; const float* fT2;
  float* out;
  // backward
  const float* dout;
  double* s1_dz; double* s1_dzx; double* s2_dz; double* s2_dzx;
  float* lanes;        // lane scratch (2 * kLaneFloats)
  float* du1; float* du2; int du2_add;
  float* g_gamma1; float* g_beta1; float* g_gamma2; float* g_beta2;
  int grid;            // set by the launcher
};

// column sums of rows (BatchNorm batch statistics of a tensor no producer epilogue covers)
struct ColStatArgs {
  long long R; int C;
  const float* x;
  double* sum; double* sumsq;
  float* lanes;        // lane scratch (kLaneFloats)
  int grid;            // set by the launcher
};

// tokens: pos [R][4] = (x, y, score, 0); mot [Rm][4] = (x[t] - x[t+1], y[t] - y[t+1], 0, 0)
struct TokenArgs {
  int N, T, V;
  const float* x;      // reference layout [N][3][T][V]
  float* pos; float* mot;
  float* rp;           // [N][3] mean of the raw positions over (T, V) (the head's res_pos)
};

// relu backward on the embedding: d_pre = d * (y > 0)
struct ReluBwdArgs {
  long long n;
  const float* y; const float* d; float* out;
};

// Classification_Module on [pooled pos (Cs) | pooled mot (Cs) | res_pos (3)]
struct HeadArgs {
  int N, Cs, TV1, TV2, NC;     // Cs = 256; TV = T*V rows per clip of each stream; NC classes
  const float* y1; const float* y2;   // stream outputs [N][TV][Cs]
  const float* x; int TVx;            // raw positions [N][3][T*V] (the head's res_pos = their mean)
  const float* w1; const float* b1;   // [128][2Cs+3]
  const float* lnw; const float* lnb; // [128]
  const float* w2; const float* b2;   // [NC][128]
  unsigned seed; float drop_p;        // Dropout(0.2) hash mask (train)
  float* feat;      // [N][2Cs+3]
  float* z1;        // [N][128] pre-activation of the first Linear
  float* stat;      // [N][2] LayerNorm mean, rstd
  float* h;         // [N][128] fc2 input (after dropout)
  float* out;       // [N][NC]
  // backward
  const float* dout;
  float* dz1;       // [N][128]
  float* dy1; float* dy2;   // [N][TV][Cs] stream output gradients (overwrite)
  float* g_lnw; float* g_lnb;
};

}  // namespace mu
}  // namespace f3

int f3_mu_dwconv_fwd(const f3::mu::DwConvArgs* a, hipStream_t s);
int f3_mu_dwconv_bwd(f3::mu::DwConvArgs* a, hipStream_t s);   // dx; weight partials in a->part
int f3_mu_dwconv_part_rows(const f3::mu::DwConvArgs* a);
int f3_mu_bn_act(const f3::mu::BnActArgs* a, hipStream_t s);
int f3_mu_bn_act_bwd(const f3::mu::BnActBwdArgs* a, hipStream_t s);
int f3_mu_absstat(const f3::mu::AbsStatArgs* a, hipStream_t s);
int f3_mu_dropmask(const f3::mu::DropMaskArgs* a, hipStream_t s);
int f3_mu_dropmask_scratch_floats(int N, int T, int V);
int f3_mu_merge_fwd(const f3::mu::MergeArgs* a, hipStream_t s);
int f3_mu_merge_bwd(const f3::mu::MergeArgs* a, hipStream_t s);
int f3_mu_colstat(const f3::mu::ColStatArgs* a, hipStream_t s);
int f3_mu_tokens(const f3::mu::TokenArgs* a, hipStream_t s);
int f3_mu_relu_bwd(const f3::mu::ReluBwdArgs* a, hipStream_t s);
int f3_mu_head_fwd(const f3::mu::HeadArgs* a, hipStream_t s);
int f3_mu_head_bwd(const f3::mu::HeadArgs* a, hipStream_t s);
