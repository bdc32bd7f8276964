// Argument blocks of the IMU-branch kernels (sensor.hip).
#pragma once
#include "common.h"

namespace f3 {

constexpr int LSTM_NB = 4;  // clips per LSTM workgroup (LSTM_NB * H == 256 threads)

struct LstmArgs {
  int N, T, S;
  const float* x;             // [N][T][S]
  const float* w_ih[2];       // [4H][S]   (forward, reverse)
  const float* w_hh[2];       // [4H][H]
  const float* b_ih[2];
  const float* b_hh[2];
  float* seq;                 // [N][T][2H] hidden states
  float* gates;               // [2][N][T][4H] post-activation i,f,g,o
  float* cell;                // [2][N][T][H]
  float* hmean;               // [N][2H]
  // backward
  const float* dhmean;        // [N][2H]
  float* dx;                  // [N][T][S] (+=) or null
  float* g_w_ih[2];
  float* g_w_hh[2];
  float* g_b_ih[2];
  float* g_b_hh[2];
  // deterministic weight gradients: per (direction, clip tile) partial rows [2][tiles][4H (1 + S + H)]
  // (bias | w_ih | w_hh), summed in tile order by f3_colsum; null: float atomics
  float* wpart;
};

struct SHeadArgs {
  int N, Cs;
  const float* hmean;         // [N][128]
  BnRef bn;
  double* bn_sum;
  double* bn_sq;
  const float* W1; const float* b1;   // [16][128]
  const float* W2; const float* b2;   // [128][16]
  const float* W3; const float* b3;   // [Cs][128]
  float* ybn;                 // [N][128]
  float* a1;                  // [N][16]
  float* att;                 // [N][128]
  float* out;                 // [N][out_ld]
  int out_ld;
  // backward
  const float* dout;
  int dout_ld;
  float* dy;                  // scratch [N][128]
  float* dpre2;               // scratch [N][128]
  float* dpre1;               // scratch [N][16]
  float* dhmean;              // [N][128]
  float* g_W1; float* g_b1;
  float* g_W2; float* g_b2;
  float* g_W3; float* g_b3;
  float* g_gamma; float* g_beta;
};

struct Conv1dArgs {
  int N, T, Ci, Co;
  const float* x;             // [N][T][Ci]
  const float* w;             // [Co][Ci][5]
  const float* b;
  float* y;                   // [N][T][Co] conv output (pre-BN)
  double* st_sum;
  double* st_sq;
  BnRef bn;
  float* p;                   // [N][T/2][Co] pooled output
  // backward
  const float* dp;            // [N][T/2][Co]
  float* dy;                  // scratch [N][T][Co]
  double* bsum;
  double* bsq;
  float* g_gamma; float* g_beta;
  float* g_b; float* g_w;
  float* dx;                  // [N][T][Ci] (=) or null
};

// The two CNN1D layers as ONE cooperative launch per direction (f3_cnn1d_fwd / f3_cnn1d_bwd): a
// workgroup per clip (up to kCnnCoopG, clips walked n = b, b + G, ...), the BatchNorm statistics and
// the weight gradients reduced across workgroups in fixed order after group barriers (gn_barrier)
// instead of separate launches and float atomics.
constexpr int kCnnCoopG = 256;
struct CnnCoop {
  float* part;  // partial rows, f3_cnn1d_coop_part_floats(N, Ci1, Co1, Co2) floats
  int* sync;    // f3_cnn1d_coop_sync_ints() ints: barrier counters, error flag; zero at launch
};
int f3_cnn1d_coop_sync_ints();
size_t f3_cnn1d_coop_part_floats(int N, int Ci1, int Co1, int Co2);

struct HeadArgs {
  int N, C, nblk;
  const float* feat[3];       // feature blocks [N][ld_k]
  int width[3];
  int ld[3];
  const float* W;             // [C][sum(width)]
  const float* b;
  float* out;                 // [N][C]
  float* out2;                // [N][C] second copy of out (the caller's buffer), or null
  int softmax_out;
  // loss
  const float* label;         // [N][C] soft targets or null
  float* loss;                // scalar (+=)
  float* dout;                // [N][C] dLoss/dout (when label given)
  // backward
  const float* g_out;         // [N][C] gradient wrt out
  float* dlogits;             // scratch [N][C]
  float* dfeat[3];
  float* g_W; float* g_b;
};

}  // namespace f3

int f3_lstm_fwd(const f3::LstmArgs* a, hipStream_t s);
int f3_lstm_bwd(const f3::LstmArgs* a, hipStream_t s);
int f3_shead_fwd(const f3::SHeadArgs* a, hipStream_t s);
int f3_shead_bwd(const f3::SHeadArgs* a, hipStream_t s);
int f3_conv1d_fwd(const f3::Conv1dArgs* a, hipStream_t s);
int f3_bnrelupool_fwd(const f3::Conv1dArgs* a, hipStream_t s);
int f3_conv1d_bwd(const f3::Conv1dArgs* a, hipStream_t s);
// both CNN1D layers: the cooperative launch (training, `coop` given, not under stream capture,
// F3_CNN1D_COOP unset or 1), else the per-layer launches above (eval, capture)
int f3_cnn1d_fwd(const f3::Conv1dArgs* c1, const f3::Conv1dArgs* c2, const f3::CnnCoop* coop, hipStream_t s);
int f3_cnn1d_bwd(const f3::Conv1dArgs* c1, const f3::Conv1dArgs* c2, const f3::CnnCoop* coop, hipStream_t s);
int f3_head_fwd(const f3::HeadArgs* a, hipStream_t s);
int f3_ce(const f3::HeadArgs* a, hipStream_t s);
int f3_head_bwd(const f3::HeadArgs* a, hipStream_t s);  // f3_head_bwd_data, then f3_head_bwd_weight
// dlogits + feature gradients (the backward's critical path) / the Linear's weight gradients
int f3_head_bwd_data(const f3::HeadArgs* a, hipStream_t s);
int f3_head_bwd_weight(const f3::HeadArgs* a, hipStream_t s);
// zero na floats at a and nb floats at b (16-byte aligned) in one launch
int f3_zero2(float* a, long long na, float* b, long long nb, hipStream_t s);
// RMSprop over up to kRmsRanges ranges of one flat buffer in one launch (offsets and lengths in
// floats, multiples of 4: the entries of the flat parameter layout are 16-B aligned)
constexpr int kRmsRanges = 8;
struct RmsRanges {
  int n;
  long long lo[kRmsRanges], len[kRmsRanges];
};
int f3_rmsprop_ranges(float* p, float* sq, const float* g, const RmsRanges& r, float lr, float alpha, float eps,
                      float scale, hipStream_t s);
int f3_rmsprop(float* p, float* sq, const float* g, long long n, float lr, float alpha, float eps, float scale,
               hipStream_t s);
