// Argument blocks of the byte-moving layer kernels (layers.hip) and sensor/head kernels.
#pragma once
#include "common.h"

namespace f3 {

enum : int { PREP_MUL = 0, PREP_PACK_CONV, PREP_PACK_CONV_T, PREP_PACK_GCN, PREP_PACK_GCN_T, PREP_GCN_BIAS, PREP_COPY,
              PREP_UNPACK_CONV };

struct PrepJob {
  int type, n;
  float* dst;
  const float* s0;
  const float* s1;
  const float* s2;
  int d0, d1, d2;
  int bf16;  // dst type: 0 fp32, 1 bf16, 2 bf16 hi / lo planes,
             // 4 per-tap 32-channel blocks [hi 32 | lo 32] (bf16x3 native, ConvGemmArgs::x3n)
};

struct DataBnArgs {
  int N, T, V, C, motion;
  const float* skel;     // reference layout [N][3][T(+1)][V]
  float* out;            // [N][T][V][C] (bf16 when act16)
  int act16;
  BnRef bn;
  double* st_sum;
  double* st_sq;
  const float* dout;     // backward
  float* dgamma;
  float* dbeta;
  float* part;           // databn_bwd2: partial rows [blocks][2 VC] (gamma, beta), summed in order
};

struct MixArgs {
  int K, V, Cin, frames;
  const float* A;        // A_eff [K][V][V]
  const float* x;        // [frames][V][Cin] (bf16 when x16)
  int x16;
  float* z;              // [frames][V][K][Cin] (fwd out / bwd in)
  float* dx;             // bwd out
  float* dA;             // bwd accumulate [K][V][V]
  int accumulate;
  float* part;           // bwd scratch [kMixParts][K*V*V] (MFMA path)
  unsigned short* zb;    // fwd: write z as bf16 (bf16 mode GEMM operand) instead of fp32
  const unsigned short* dzb;  // bwd: dZ in bf16 (instead of z) — LDS mix path only
  int no_colsum;         // bwd: leave the dA partial rows in `part` (caller reduces: f3_mix_bwd_parts)
  int x3;                // bf16x3 mode: fp32 x / z / dz on the split-bf16 MFMA kernels (mix_*_x3)
  unsigned short* z3;    // bf16x3 fwd: Z as rows [hi | lo] of 2 K Cin bf16 (the bf16x3 gcn
                         // GEMM / weight-gradient operand) instead of fp32 z
};
constexpr int kMixParts = 1024;

// the first block's graph convolution (Cin <= 4, C = 64) in the bf16 mode (layer0.hip)
struct Gcn0Args {
  int frames, K, V, Ci;
  const float* A;               // A_eff [K][V][V]
  const unsigned short* x;      // bf16 [frames][V][Ci] (data_bn output)
  const unsigned short* w;      // bf16 packed gcn weight [64][K*Ci]
  const float* beff;            // graph-mixed bias [V][64]
  unsigned short* z;            // fwd out / bwd in: bf16 [frames][V][K][Ci]
  unsigned short* g;            // fwd out: bf16 [frames*V][64]
  double* st_sum;               // fwd: BN1 sums [64]
  double* st_sq;
  const unsigned short* dg;     // bwd in: bf16 [frames*V][64]
  float* dx;                    // bwd out: fp32 [frames][V][Ci]
  int accumulate;
  float* part_dA;               // bwd: per-block partial rows [blocks][K*V*V]
  float* part_dW;               // bwd: per-block partial rows [blocks][K*64*Ci] (gradient layout)
  // 1: fp32 operands and results (the bf16x3 mode: x, w, z, g, dg are float* behind these
  // pointers; products in fp32 on the VALU / fp32 MFMA instead of bf16)
  int f32;
};

struct GcnBiasBwdArgs {
  int K, V, C;
  const float* Aeff;
  const float* A;
  const float* G;        // [V][C] per-node column sums of dg
  const float* bias;     // gcn conv bias [K*C]
  float* db;
  const float* dAeff;
  float* dE;
};

enum : int { RES_NONE = 0, RES_ID = 1, RES_CONV = 2 };

constexpr int kCaMaxRowsPerThread = 4;  // channel attention: batch <= 1024 per GPU

struct BlockArgs {
  int N, TV, C, chunks, res_kind;
  int act16;             // h, r, x, out stored bf16
  float inv_tv;
  BnRef bn2, bnr;
  const float* h;        // tcn output before BN2 [M][C]
  const float* r;        // residual conv output before BN_r
  const float* x;        // block input (identity residual)
  const float* att;      // channel attention [N][C]
  float* out;            // block output [M][C]
  float* pool;           // [N][C] mean over (T,V) or null
  unsigned short* outb;  // optional bf16 copy of out (next block's residual-conv operand)
  // backward
  const float* dout;     // [M][C] or null when dout_nc is given
  const float* dout_nc;  // [N][C] gradient of the pooled mean (broadcast * inv_tv)
  float* P1;
  float* P2;
  float* Q2;             // conv residual: [N][C] per-clip sum dz*xhat_r (ca_bwd3 folds P1, Q2 into bnr_bsum/bsq)
  double* bnr_bsum;
  double* bnr_bsq;
  const double* bn2_bsum;
  const double* bn2_bsq;
  const float* e;        // [N][C] dgap / TV
  float* dh;
  float* dres;           // dr (conv) or dx (identity)
  unsigned short* dhb;   // bf16 mode: dh written as bf16 (GEMM operand) instead of fp32
  unsigned short* dresb; // bf16 mode, conv residual: dr as bf16 instead of fp32
  int x3;                // bf16x3 mode: dhb, dresb (backward) and outb (forward) receive rows
                         // [hi | lo] of 2C bf16 (the bf16x3 GEMM operands)
  float* dgamma2;
  float* dbeta2;
  // deterministic reductions: per-chunk partial rows of pool (forward, [chunks][N*C]) and of P1, P2,
  // Q2 (backward, three [chunks][N*C] blocks), summed in chunk order by f3_colsum; null: float atomics
  float* part;
  float* dgammar;
  float* dbetar;
  // block_bwd_apply (bf16x3): per (chunk, clip) column sums of the fp32 dh rows (the tcn bias gradient)
  // and, conv residual, of dres (its bias), rows [chunks][N][C | C] summed by the caller's colsum; the
  // weight-gradient kernels then run without their in-loop bias sums. null: not written
  float* dbpart;
  int no_colsum;  // block_bwd_reduce: leave P1 / P2 / Q2 in `part` (ca_bwd1x sums them, CaArgs::bpart)
};

struct BnBwdArgs {
  int N, TV, C, V, chunks;
  int act16;             // dv, g stored bf16
  BnRef bn;
  const double* bsum;
  const double* bsq;
  float* dgamma;
  float* dbeta;
  const float* dv;
  const float* g;
  float* dg;
  float* G;              // [V][C] (accumulated from Gpart by a column reduction)
  float* Gpart;          // [gridDim][V*C] per-workgroup partial rows
  unsigned short* dgb;   // bf16 mode: dg as bf16 (GEMM operand) instead of fp32
  int no_colsum;         // leave the G partial rows in Gpart (caller reduces with f3_colsum)
  int x3;                // bf16x3 mode: dgb receives dg as rows [hi | lo] of 2C bf16
};

struct BnReluArgs {      // u = relu(bn(g)) as bf16: the tcn GEMM operand of the bf16 mode
  int M, C;
  int g16;               // g stored bf16
  BnRef bn;
  const float* g;
  unsigned short* u;
  int x3;                // bf16x3 mode: u as rows [hi | lo] of 2C bf16 (fp32 g)
};

struct CaArgs {
  int N, C;
  float inv_tv;
  BnRef bn2, bnca;
  const float* W1;       // [C/4][C]
  const float* b1;
  const float* W2;       // [C][C/4]
  const float* b2;
  const float* gapsum;   // [N][C] sum over rows of the tcn output (pre-BN2)
  float* q1;             // [N][C/4]
  float* hid;            // [N][C/4]
  float* att;            // [N][C]
  double* ca_sum;
  double* ca_sq;
  // backward
  const float* P1;
  const float* P2;
  const float* Q2;       // conv residual (else null): per-clip sums for the residual BN backward
  double* bnr_bsum;
  double* bnr_bsq;
  float* dq2;
  float* dbn;
  float* dq1;
  float* e;
  double* bn2_bsum;
  double* bn2_bsq;
  float* g_bnca_gamma;
  float* g_bnca_beta;
  float* g_b1;
  float* g_W1;
  float* g_W2;
  float* g_b2;
  // deterministic weight gradients: per clip-group partial rows [groups][2 H C + C] (g_W1, g_W2, g_b2),
  // summed in group order by f3_colsum; null: float atomics
  float* wpart;
  // block_bwd_reduce's partial rows [chunks][3][N][C] (BlockArgs::no_colsum): ca_bwd1x sums each clip's
  // P1 / P2 / Q2 from them in the order f3_colsum uses and writes P1 / P2 / Q2; null: already summed
  const float* bpart;
  int bchunks;
};


struct BnRunJob {
  const double* sum;
  const double* sumsq;
  double count;
  int C;
  float* rmean;
  float* rvar;
  long long* nbt;
};

// job tables travel as kernel arguments (by value, < 4 KB), so a step needs no
// host->device copies and stays graph-capturable
constexpr int kMaxPrepJobs = 56;
struct PrepTable {
  int n;
  PrepJob jobs[kMaxPrepJobs];
};
constexpr int kMaxBnJobs = 56;
struct BnRunTable {
  int n;
  BnRunJob jobs[kMaxBnJobs];
};

}  // namespace f3

int f3_prep(const f3::PrepTable& t, hipStream_t s);
int f3_databn_fwd(const f3::DataBnArgs* a, hipStream_t s);
int f3_databn_bwd(const f3::DataBnArgs* a, hipStream_t s);
int f3_mix_fwd(const f3::MixArgs* a, hipStream_t s);
int f3_mix_bwd(const f3::MixArgs* a, hipStream_t s);
int f3_mix_bwd_parts(const f3::MixArgs* a);  // dA partial rows the LDS mix backward leaves (0: none)
bool f3_mix_lds_ok(int K, int V, int Cin);  // the LDS/MFMA mix path (takes bf16 dZ)
bool f3_mix_x3_ok(int K, int V, int Cin);   // the split-bf16 mix kernels (bf16x3 mode; MixArgs::z3)
int f3_split_x3(const float* x, unsigned short* out, long long rows, int C, hipStream_t s);  // [hi | lo] rows
int f3_gcn_bias_bwd(const f3::GcnBiasBwdArgs* a, hipStream_t s);
bool f3_gcn0_ok(int K, int V, int Ci, int C);
int f3_gcn0_fwd(const f3::Gcn0Args* a, hipStream_t s);
int f3_gcn0_bwd(const f3::Gcn0Args* a, hipStream_t s);
int f3_gcn0_bwd_parts(const f3::Gcn0Args* a);  // partial rows f3_gcn0_bwd leaves (caller: f3_colsum)
int f3_databn_bwd2(const f3::DataBnArgs* a, hipStream_t s);  // single-pass data_bn gamma/beta gradient
int f3_block_out(f3::BlockArgs a, hipStream_t s);
int f3_block_bwd_reduce(f3::BlockArgs a, hipStream_t s);
int f3_block_bwd_apply(f3::BlockArgs a, hipStream_t s);
int f3_bn_bwd_apply(f3::BnBwdArgs a, hipStream_t s);
int f3_bn_bwd_parts(int N, int TV, int V);  // Gpart rows f3_bn_bwd_apply writes
int f3_block_chunks(int TV);                 // row chunks per clip of the block kernels (dbpart rows: chunks * N)
int f3_bnrelu_bf16(const f3::BnReluArgs* a, hipStream_t s);
// several independent column sums in one launch (each as f3_colsum_ld)
constexpr int kColsumJobs = 10;
struct ColsumJob {
  const float* part;
  float* out;
  long long ld;
  int rows, cols;
};
int f3_colsum_multi(const ColsumJob* jobs, int n, hipStream_t s);
int f3_colsum(const float* part, int rows, int cols, float* out, hipStream_t s);  // out[c] += sum_r part[r][c]
// the same over rows `ld` floats apart (fixed summation order, as f3_colsum)
int f3_colsum_ld(const float* part, int rows, long long ld, int cols, float* out, hipStream_t s);
int f3_ca_fwd(const f3::CaArgs* a, hipStream_t s);
int f3_ca_bwd(const f3::CaArgs* a, hipStream_t s);          // input-gradient chain (ca_bwd1/2/3)
// W1/W2/b2 gradients (ca_bwd_w); with `defer`, the three column sums of its partial rows are appended
// to defer[*ndefer...] (ndefer advanced) for one batched f3_colsum_multi by the caller instead of launched
int f3_ca_bwd_weights(const f3::CaArgs* a, hipStream_t s, ColsumJob* defer = nullptr, int* ndefer = nullptr);
// the up-front-load channel-attention kernels apply (N <= 256, C % 64 == 0, F3_CA_X != 0) and can take
// block_bwd_reduce's partial rows of a T*V frame (chunks <= 16)
bool f3_ca_x_ok(int N, int C, int TV);
int f3_bn_running(const f3::BnRunTable& t, hipStream_t s);
