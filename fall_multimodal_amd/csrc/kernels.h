// Internal kernel-launcher interface (host side). The public C ABI is include/fall3.h.
#pragma once
#include <hip/hip_runtime.h>
#include "common.h"

namespace f3 {

// Row geometry of a temporal conv over [N][T][V][C] rows (row m = (n*T + t)*V + v).
struct ConvGeom {
  int M;            // output rows = N*T_out*V
  int Nc;           // output channels
  int Kc;           // input channels per tap
  int KT, S, P;     // taps, stride, zero padding
  int transposed;   // 1: input-gradient row map of a strided conv
  int T_out, T_in, V;
  int lda, ldo;     // row strides (elements) of input / output
};

enum : int {
  EPI_BIAS = 1,       // + bias[j]
  EPI_BIASV = 2,      // + bias[v][j]  (graph-mixed gcn bias)
  EPI_STATS = 4,      // fp64 sum / sum-of-squares per output channel (BN forward)
  EPI_GAP = 8,        // per (clip, channel) sum over the clip's rows (channel attention pool)
  EPI_RELUMASK = 16,  // zero where BN(aux)<=0, accumulate sum dv and sum dv*xhat(aux)
  EPI_ADD = 32,       // out += value
};

struct ConvGemmArgs {
  ConvGeom g;
  const float* in;
  const float* w;     // packed [Nc][KT*Kc]
  const unsigned short* wb;  // same, bf16; non-null selects the bf16 MFMA kernels
  const unsigned short* inb; // bf16 activations (instead of `in`); with wb: LDS-DMA kernel when shapes allow
  const unsigned short* zero;  // >= 16 zero bytes (rows outside the clip / tile for the LDS-DMA kernel)
  unsigned short* outb;        // LDS-DMA kernel: write the output as bf16 here instead of `out`
  float* out;
  BnRef pro_bn;       // prologue: relu(bn(x)) on input channels
  const float* bias;
  double* st_sum;
  double* st_sq;
  float* gap;         // [N][Nc]
  const float* aux;   // RELUMASK source rows
  int ldaux;
  const unsigned short* auxb;  // RELUMASK source rows stored bf16 (instead of aux)
  BnRef epi_bn;
  int x3;             // 1: split-bf16 kernel (fp32 in / out; wb = hi plane, wb + Nc*KT*Kc = lo plane)
  // bf16x3 native form (x3n = 1, igemm_bf16 / igemm_big / pw_gemm): the activation rows hold
  // [x_hi (Kc) | x_lo (Kc)] (lda >= 2 Kc), Kc = the real channel count, and the packed weights hold,
  // per tap, 32-channel blocks [W_hi (32) | W_lo (32)] (row length KT * 2 Kc). A k step covers one
  // 32-channel block: its staged 128-B row piece is [x_hi 32 | x_lo 32] and the wave issues the split
  // product's three MFMAs x_hi W_hi + x_lo W_hi + x_hi W_lo from the four fragments (x_hi read once
  // for two products), so the bytes staged and the fragments read per MFMA are 2/3 of the
  // K-concatenated form's
  int x3n;
};

enum : int { WG_OUT_CONV = 0, WG_OUT_GCN = 1 };

struct WgradArgs {
  ConvGeom g;         // geometry of the FORWARD conv (M = its output rows)
  const float* dy;    // [M][ldy]
  int ldy;
  const float* in;    // forward input rows
  float* dw;          // accumulated (+=)
  float* db;          // [Nc] accumulated (+=) or null
  int outmap;
  int gcn_cin;
  BnRef pro_bn;
  int rows_per_split;
  int bf16;           // 1: bf16 MFMA (operands rounded to bf16, fp32 accumulate)
  const unsigned short* dyb;  // bf16 dy (instead of dy)
  const unsigned short* inb;  // bf16 input rows (instead of in)
  const unsigned short* zero; // >= 16 zero bytes (LDS-DMA kernel)
  int xcd;                    // LDS-DMA kernel: XCD-aware 1-D grid (set by the launcher)
  // LDS-DMA kernel, WG_OUT_CONV: per-split partial tiles go to slab[split][Nc][KT*Kc] with plain
  // stores instead of fp32 atomics into dw (33 MB of memory-side atomics per layer-6 launch at
  // ~1.3 TB/s); the launcher then sums the splits into dw_ref (reference layout [Nc][Kc][KT], +=).
  // dw_ref == null: leave the partials in the slab (roofline timing of the kernel alone).
  float* slab;
  long long slab_cap;         // floats
  float* dw_ref;
  // Grouped launch (TARGCN per-node weight gradients): `groups` independent problems of the same
  // geometry, problem q reading dy + q*gs_dy, in + q*gs_in (elements) and accumulating into
  // dw + q*gs_dw, db + q*gs_db. groups <= 1: one problem. Atomics path only (slab == null).
  int groups;
  long long gs_dy, gs_in, gs_dw, gs_db;
  int wg_pct;                 // split sizing, percent of the resident workgroup slots (0: all)
  int taps_f;                 // (set by the launcher) wgrad_taps frame-chunk length
  float* dbpart;              // (set by the launcher) bias-gradient partial rows [splits][Nc] after the slab
                              // partials, summed in split order (deterministic); null: float atomics
  int x3;                     // 1: split-bf16 kernel on fp32 dy / in (gemm_x3.hip)
  // bf16x3 on the bf16 kernels by row segments (wgrad_big / wgrad_taps): dy / in are [hi | lo] rows
  // (ldy = 2 Nc, lda = 2 Kc) and the GEMM runs over 3 segments of the rows, (dY_hi, X_hi),
  // (dY_lo, X_hi), (dY_hi, X_lo) - the split product's three terms - with the split index
  // bz = row split * 3 + segment (the three segments of one row range on adjacent workgroups, i.e.
  // mostly one XCD: X_hi / dY_hi re-reads hit its L2); the bias sums the first two segments
  // (dY_hi + dY_lo). With gcn_cin > 0 (KT = 1, Ci = K gcn_cin) the slab reduce writes the gcn
  // weight's reference layout [K*C][gcn_cin] (column k gcn_cin + ci of the packed operand -> row k C + c).
  int x3seg;
};

// Apply a grouped launch's per-problem pointer offsets (no-op for groups <= 1).
F3_DEV void wgrad_group(WgradArgs& a, int grp) {
  if (a.groups <= 1) return;
  if (a.dy) a.dy += grp * a.gs_dy;
  if (a.in) a.in += grp * a.gs_in;
  if (a.dyb) a.dyb += grp * a.gs_dy;
  if (a.inb) a.inb += grp * a.gs_in;
  a.dw += grp * a.gs_dw;
  if (a.db) a.db += grp * a.gs_db;
}

}  // namespace f3

// Weight-gradient split-K sizing of the atomics-path kernels (gemm.hip, gemm_bf16.hip, gemm_x3.hip):
// target number of workgroups per launch. Each workgroup adds its whole output tile with float
// atomics (executed at the memory side, ~1.3 TB/s chip-wide), so more splits = more atomic traffic.
inline int f3_wgrad_target_wgs() { return 512; }

int f3_conv_gemm(const f3::ConvGemmArgs* a, int pro, int epi, hipStream_t s);
int f3_conv_wgrad(const f3::WgradArgs* a, int pro, hipStream_t s);
int f3_conv_gemm_bf16(const f3::ConvGemmArgs* a, int pro, int epi, hipStream_t s);
bool f3_igemm_ok(const f3::ConvGemmArgs& a);
int f3_igemm_bf16(const f3::ConvGemmArgs* a, int epi, hipStream_t s);
// weight-stationary 64-channel 9-tap tcn (tcn64.hip); f3_igemm_bf16 dispatches to it
bool f3_tcn64_ok(const f3::ConvGemmArgs& a, int epi);
int f3_tcn64(const f3::ConvGemmArgs* a, int epi, hipStream_t s);
// weight-stationary persistent 1x1 GEMM (pw_gemm.hip): gcn forward / input gradient, residual conv
bool f3_pw_ok(const f3::ConvGemmArgs& a, int epi);
int f3_pw_gemm(const f3::ConvGemmArgs* a, int epi, hipStream_t s);
bool f3_igemm_big_ok(const f3::ConvGemmArgs& a);
bool f3_igemm_big_win_ok(const f3::ConvGemmArgs& a);  // the clip-window form applies
int f3_igemm_big(const f3::ConvGemmArgs* a, int epi, hipStream_t s);
bool f3_wgrad_glds_ok(const f3::WgradArgs& a);
int f3_wgrad_glds_bf16(const f3::WgradArgs* a, hipStream_t s);
int f3_conv_wgrad_bf16(const f3::WgradArgs* a, int pro, hipStream_t s);
// split-bf16 (bf16x3) forms (gemm_x3.hip): fp32 activations, weights as pre-split bf16 hi / lo planes
int f3_conv_gemm_x3(const f3::ConvGemmArgs* a, int pro, int epi, hipStream_t s);
int f3_conv_wgrad_x3(const f3::WgradArgs* a, int pro, hipStream_t s);
