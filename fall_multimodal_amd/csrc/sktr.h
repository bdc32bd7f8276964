// SkeletonTransformer (BASELINE config 5) kernels: internal launcher interface.
// Reference: /root/reference/skeleton_transformer.py (SkeletonTransformer(3,14,30,11,32,6,16,8)).
//
// Token layout: channels-last rows [N][M][T][V][32] (row r = ((n*M + m)*T + t)*V + v), fp32.
// The Linear layers run on the shared fp32 MFMA GEMM (f3_conv_gemm / f3_conv_wgrad with a
// 1x1 geometry); this file holds what is specific to the model: the token MLP embedding, the
// relative-position attention core over joints (spatial) or frames (temporal), the residual /
// BatchNorm3d / dropout elementwise passes and the pooled classifier.
#pragma once
#include <hip/hip_runtime.h>

#include "common.h"

namespace f3 {
namespace sk {

constexpr int EMB = 32;          // embedding_dim
constexpr int HEADS = 8, HD = 16;
constexpr int DM = HEADS * HD;   // 128 attention embed dims
constexpr int QKV = 3 * DM;      // 384
constexpr int FFN = 4 * EMB;     // 128
constexpr int HID0 = EMB / 2;    // 16: first embedding Linear
constexpr int CIN = 3;
constexpr int LMAX = 32;         // longest attention sequence supported (T or V)

struct EmbedArgs {
  int N, M, T, V;
  const float* x;      // reference layout [N][3][T][V][M]
  const float* w1;     // [16][3]
  const float* b1;
  const float* w2;     // [32][16]
  const float* b2;
  float* y;            // fwd out [R][32]
  const float* dy;     // bwd in [R][32]
  float* gw1; float* gb1; float* gw2; float* gb2;   // bwd: accumulated (+=)
};

// attention core on precomputed q|k|v rows
struct AttnArgs {
  int L;               // sequence length: V (spatial) or T (temporal)
  int temporal;        // 0: sequences (nm, t) over joints; 1: sequences (nm, v) over frames
  int nseq;            // N*M*T (spatial) or N*M*V (temporal)
  int T, V;
  float scale;         // embed_dims ** -0.5
  const float* qkv;    // [R][384]
  const float* table;  // relative_position_bias_table [2L-1][16]
  float* o;            // fwd out [R][128] (head-major channels h*16+d)
  const float* dout;   // bwd in [R][128]
  float* dqkv;         // bwd out [R][384]
  float* dtab;         // bwd out: per-sequence partial table gradients [nseq][2L-1][16]
};

// elementwise: u = a (+ b) + s * keep * f ; BatchNorm3d batch sums of u (fp64, accumulated)
struct ResidArgs {
  long long R;
  const float* a;
  const float* b;      // optional
  const float* f;
  float s;             // stochastic-depth factor of the branch
  unsigned seed;       // dropout (FFN branch): keep(e) from the counter hash, e = row*32 + c
  int block;
  float drop_p;        // 0: no dropout
  float* u;
  double* sum; double* sumsq;
};

struct BnApplyArgs {
  long long R;
  const float* u;
  BnRef bn;
  float* y;
};

// BatchNorm backward over rows: pass 1 accumulates sum(dy), sum(dy*xhat); pass 2 writes
// o1 = dU (+ add), o2 = s2 * keep * dU (optional), o3 = dU (optional), and the gamma/beta grads.
struct BnBwdArgs {
  long long R;
  const float* dy;
  const float* u;
  BnRef bn;
  double* s_dy; double* s_dyx;   // [32] each
  const float* add;
  float* o1; float* o2; float* o3;
  float s2;
  unsigned seed; int block; float drop_p;   // o2's dropout mask (FFN branch)
  float* g_gamma; float* g_beta;            // accumulated (+=)
};

struct GeluArgs {
  long long n;
  const float* h;
  float* g;          // fwd: gelu(h)
  const float* dg;   // bwd: dh = dg * gelu'(h)
  float* dh;
};

struct HeadArgs {
  int N, MTV, C;
  const float* y;      // [N][MTV][32]
  const float* w;      // fcn.0.weight [C][32]
  const float* b;
  float* pooled;       // [N][32]
  float* out;          // [N][C]
  const float* dout;   // bwd [N][C]
  float* dy;           // bwd [N][MTV][32]
  float* gw; float* gb;
};

}  // namespace sk
}  // namespace f3

// embedding: the forward keeps xt [R][4] (token-major input), a1/h1 [R][16], a2 [R][32]; the
// backward writes da1 [R][16], da2 [R][32] (weight gradients: wgrad GEMMs on those)
int f3_sk_embed_fwd_save(const f3::sk::EmbedArgs* a, float* xt, float* a1, float* h1, float* a2, hipStream_t s);
int f3_sk_embed_bwd_save(const f3::sk::EmbedArgs* a, const float* a1, const float* a2, float* da1, float* da2,
                         hipStream_t s);
bool f3_sk_attn_len_ok(int L);
int f3_sk_attn_fwd(const f3::sk::AttnArgs* a, hipStream_t s);
int f3_sk_attn_bwd(const f3::sk::AttnArgs* a, hipStream_t s);
int f3_sk_resid(const f3::sk::ResidArgs* a, hipStream_t s);
int f3_sk_bn_apply(const f3::sk::BnApplyArgs* a, hipStream_t s);
int f3_sk_bn_bwd(const f3::sk::BnBwdArgs* a, hipStream_t s);   // both passes
int f3_sk_gelu_fwd(const f3::sk::GeluArgs* a, hipStream_t s);
int f3_sk_gelu_bwd(const f3::sk::GeluArgs* a, hipStream_t s);
int f3_sk_head_fwd(const f3::sk::HeadArgs* a, hipStream_t s);
int f3_sk_head_bwd(const f3::sk::HeadArgs* a, hipStream_t s);
