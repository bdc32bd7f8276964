// TARGCN (BASELINE config 2) kernels: graph-GRU recurrence with EmbGCN gates, temporal
// attention (TA) layers and the end_conv/pool/Linear head. Host launchers; the public C ABI is
// include/fall3.h (f3_targcn_*).
#pragma once
#include <hip/hip_runtime.h>
#include "common.h"

namespace f3 {
namespace tg {

constexpr int H = 64;     // rnn_units (TRAGCN.py:178)
constexpr int EMB = 64;   // embed_dim
constexpr int IP = 128;   // padded EmbGCN input width (dim_in + H <= 128)
constexpr int T = 30;     // frames = TA seq_len = horizon (TA.py:23, TRAGCN.py:178)
constexpr int C = 64;     // TA feature width (output_dim)
constexpr int CQ = 62;    // conv1/conv2 (1,3) output width
constexpr int VMAX = 18;  // nodes supported by the per-clip-tile LDS layout

// Packed EmbGCN operands of one (layer, part) (part: gate O=128, update O=64), in the
// GEMM operand type (bf16 or fp32):
//   Wf [V][O][IP]  node weights W_n = E . weights_pool, transposed (forward B operand)
//   Wb [V][IP][O]  W_n as [i][o] (input-gradient B operand)
//   Lf [O][IP]     linear.weight padded (forward static branch)
//   Lb [IP][O]     linear.weight transposed (input-gradient static branch)
//   bn [V][O]      fp32 node biases E . bias_pool
struct EmbOps {
  void* Wf;
  void* Wb;
  void* Lf;
  void* Lb;
  float* bn;
  const float* bl;  // linear.bias (param)
};

struct GruFwdArgs {
  int B, V, Din, I;
  const float* x;     // [B][T][V][Din]
  const float* S;     // [V][V] supports (I + softmax(relu(E E^T)))
  const float* cs;    // [V] static-branch node scale
  EmbOps g, u;        // gate (O = 2H), update (O = H)
  float* Hout;        // [R][H]  R = B*T*V rows (b*T + t)*V + n
  float* ZR;          // [R][2H] sigmoid(gate)
  float* SG;          // [R][2H] static pre-activation of the gate
  float* HC;          // [R][H]  tanh(update)
  float* SU;          // [R][H]  static pre-activation of the update
  void* XG;           // [R][IP] mixed gate input S.[x,h]      (operand type)
  void* XI;           // [R][IP] gate input [x,h]
  void* UG;           // [R][IP] mixed update input S.[x,r*h]
  void* UI;           // [R][IP] update input [x,r*h]
  long long* prof;    // optional phase stamps (F3_TG_PROF), [T][8]
  // node-partitioned recurrence (gru_fwd_node_kernel, bf16): per-step exchange of h and r*h
  // between the workgroups of a clip group, and the groups' barrier counters (zeroed per launch)
  unsigned short* hx;   // [B][V][H] bf16 h_t of every node
  unsigned short* rhx;  // [B][V][H] bf16 r*h of every node
  int* gsync;           // [GN_MAXG] counters, then an error flag
  int dbg_skip_arrive;  // test knob (F3_GN_SKIP_ARRIVE): workgroup 0 never arrives -> barrier timeout
};

constexpr int GN_BT = 32;     // clips per group of the node-partitioned recurrence
constexpr int GN_MAXG = 64;   // groups supported (B <= 2048)

struct GruBwdArgs {
  int B, V, Din, I;
  const float* S;
  const float* cs;
  EmbOps g, u;
  const float* Hout;
  const float* ZR;
  const float* SG;
  const float* HC;
  const float* SU;
  const float* dH;    // [R][H] gradient wrt this layer's outputs (from above)
  float* dX;          // [R][Din] input gradient (Din == H) or null
  void* DP;           // [R][2H] d gate pre-activation (operand type)
  void* DSG;          // [R][2H] cs * d gate static pre-activation
  void* DU;           // [R][H]
  void* DSU;          // [R][H]
  void* DXG;          // [R][IP] d(mixed gate input)
  void* DUG;          // [R][IP] d(mixed update input)
  long long* prof;    // optional phase stamps (F3_TG_PROF), [T][8]
  // node-partitioned backward (gru_bwd_node_kernel, bf16): the two per-step exchanges of every
  // node's d(mixed input) rows, and the group barrier counters (zeroed per launch)
  unsigned short* gx1;  // [B][V][IP] bf16 (update part)
  unsigned short* gx2;  // [B][V][IP] bf16 (gate part)
  int* gsync;           // [GN_MAXG] counters, then an error flag
  int dbg_skip_arrive;
};

struct TaArgs {
  int B, V;
  int b16;               // bf16 mode: the layer's products on bf16 MFMA (ta_fwd_mfma_kernel)
  const float* p;        // flat params
  long long off_vw, off_vb, off_c1w, off_c1b, off_c2w, off_c2b, off_lnw, off_lnb, off_lnffw, off_lnffb,
      off_f0w, off_f0b, off_f2w, off_f2b;
  const float* in;       // [B][T][V][C] layer input
  const float* pe;       // [T][C] added to the input (first layer) or null
  float* out;            // [B][T][V][C]
  float* save;           // [B*V][TA_SAVE] per-sequence saved tensors
  // backward
  const float* dout;     // [B][T][V][C]
  float* din;            // [B][T][V][C]
  float* grads;          // flat grads (same offsets as p), accumulated
  int dbg;               // (unused: kept for the argument layout)
  // backward weight gradients: each workgroup adds its waves' sums through LDS and stores them to
  // part[blockIdx][TA_PART] (plain stores); ta_part_reduce then adds the workgroups' rows into grads.
  // (Every wave's atomics into the same 64x64 matrices serialised at the end of the kernel.)
  float* part;           // [TA_MAX_WG][TA_PART] or null (per-wave atomics)
};

// the backward's per-workgroup gradient row (PART 1 fields, then reused by PART 2):
//   PART 1: dWf2 [64][64] | dWf0 [64][64] | lnffw lnffb f2b f0b lnw lnb [64] each
//   PART 2: dWv [64][64] | dW conv1 [T][T][3] | dW conv2 [T][T][3] | vb [64] | c1b [32] | c2b [32]
constexpr int TA_MAX_WG = 1024;
constexpr int TA_PART1 = 2 * 4096 + 6 * 64;
constexpr int TA_PART2 = 4096 + 2 * T * T * 3 + 64 + 2 * 32;
constexpr int TA_PART = (TA_PART2 > TA_PART1 ? TA_PART2 : TA_PART1) + 32;

// per-sequence saved block: q, k [T][CQ], v [T][C], P [T][T], xhat1 [T][C], u [T][C],
// fhat2 [T][C], rstd1 [T], rstd2 [T]
constexpr int TA_Q = 0, TA_K = TA_Q + T * CQ, TA_V = TA_K + T * CQ, TA_P = TA_V + T * C, TA_X1 = TA_P + T * T,
              TA_U = TA_X1 + T * C, TA_F2 = TA_U + T * C, TA_R1 = TA_F2 + T * C, TA_R2 = TA_R1 + T,
              TA_SAVE = TA_R2 + T;

struct PrepArgs {
  int V, I, O;
  const float* E;       // [V][EMB]
  const float* pool;    // weights_pool [EMB][I][O]
  const float* bpool;   // bias_pool [EMB][O]
  const float* lin;     // linear.weight [O][I]
  EmbOps ops;
};

// dSupp[n][m] += sum_r sum_{i<I} dxg[r][n][i] xin[r][m][i]  (two (dxg, xin) pairs, r = b*T + t)
struct SuppGradArgs {
  int V, I, rows;  // rows = B*T
  const void* dxg[2];
  const void* xin[2];
  float* dS;       // [V][V] accumulated
};

// dWpool / dbpool / dLin / dLin_b of one EmbGCN and its dE contribution (EmbGCN.py:65-68,81-82)
struct PoolGradArgs {
  int V, I, O;
  const float* E;
  const float* pool;     // [EMB][I][O]
  const float* bpool;    // [EMB][O]
  const float* cs;
  const float* dW;       // [V][O][IP]  per-node gconv weight gradient (sum_r dP x xg)
  const float* db;       // [V][O]
  const float* dWs;      // [V][O][IP]  per-node static weight gradient (sum_r cs dS x xin)
  const float* dbs;      // [V][O]      (sum_r cs dS)
  float* g_pool;         // [EMB][I][O]
  float* g_bpool;        // [EMB][O]
  float* g_lin;          // [O][I]
  float* g_linb;         // [O]
  float* g_E;            // [V][EMB] accumulated
};

}  // namespace tg
}  // namespace f3

int f3_tg_gru_lds_ok(int V);
int f3_tg_supports(const float* E, int V, float* S, float* cs, hipStream_t s);
int f3_tg_prep(const f3::tg::PrepArgs* a, int b16, hipStream_t s);
int f3_tg_gru_fwd(const f3::tg::GruFwdArgs* a, int b16, hipStream_t s);
int f3_tg_gru_bwd(const f3::tg::GruBwdArgs* a, int b16, hipStream_t s);
int f3_tg_supp_grad(const f3::tg::SuppGradArgs* a, int b16, hipStream_t s);
int f3_tg_pool_grad(const f3::tg::PoolGradArgs* a, hipStream_t s);
int f3_tg_supports_bwd(const float* E, int V, const float* dS, float* gE, hipStream_t s);
int f3_tg_endconv_mean(const float* W, const float* b, float* Wm, float* bm, hipStream_t s);
int f3_tg_pool_fwd(const float* Y, int B, int V, const float* Wm, const float* bm, float* xm, float* pooled,
                   hipStream_t s);
int f3_tg_pool_bwd(const float* dpooled, const float* xm, const float* Wm, int B, int V, float* dY, float* gW, float* gb,
                   hipStream_t s);
int f3_tg_ta_fwd(const f3::tg::TaArgs* a, hipStream_t s);
int f3_tg_ta_bwd(const f3::tg::TaArgs* a, hipStream_t s);
