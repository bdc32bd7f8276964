// The first st_gcan block's graph convolution (stgcan.py:50-56 with in_channels = 3 joints
// coordinates, K = 3 partitions) in the bf16 mode, forward and backward, and data_bn's gamma / beta
// gradient (stgcan.py:213-218).
//
// Why separate kernels. With Cin = 3 the gcn GEMM has K*Cin = 9: the mixed input Z is 9 values per
// row and the 64 outputs per row are 9 multiply-adds each, so the layer is a few MB of HBM traffic.
// The general path spent ~150 us of launches on it per stream and step (the generic fp32 graph mix,
// a 64-wide GEMM tile for 9 columns, a weight-gradient GEMM over 9 columns) and it sits at the
// very end of the backward's critical path (profiles/r03_step_timeline.txt). Here:
//   gcn0_fwd   per block of 8 frames: x -> Z = A_eff-mix (same summation order as the generic mix,
//              stored bf16) -> g = Z . W^T + bias_eff[v] (fp32, BN1 sums in registers, stored bf16);
//   gcn0_bwd   per block of 8 frames: dZ = dg . W on bf16 MFMA (16 x 16 x 32, the 9 columns of one
//              tile), then dx = A_eff-mix^T(dZ) and the partial sums of dA_eff and of the gcn weight
//              gradient dW[k][c][ci] = sum dg[.][c] Z[.][k, ci]; the block's partial rows go to a
//              slab that f3_colsum adds into the gradients (no dZ in HBM, no weight-gradient GEMM);
//   databn_bwd2  one pass over the channels-last gradient rows (coalesced), per-(v, c) sums in
//              registers and LDS, one atomic per channel and block.
// F32 (Gcn0Args::f32, the bf16x3 mode): the same kernels on fp32 x / w / Z / g / dg, every product
// in fp32 (dZ on v_mfma_f32_16x16x4_f32): the generic path's mix + 9-column split GEMM + mix
// backward + weight-gradient GEMM took ~200 us per stream and step for this layer.
#include "layers.h"
#include "igemm.h"

#include <algorithm>

namespace f3 {

constexpr int G0_FB = 8;          // frames per block iteration
constexpr int G0_MAXKC = 12;      // K * Cin
constexpr int G0_MAXV = 25;
constexpr int G0_DWB = 12;        // gcn0_bwd: dg rows loaded together in the weight-gradient pass

F3_DEV float g0_bf(unsigned short u) { return __uint_as_float((unsigned)u << 16); }
F3_DEV unsigned short g0_rne(float f) {
  const __bf16 h = (__bf16)f;
  return __builtin_bit_cast(unsigned short, h);
}

// ---------------------------------------------------------------------------------------------
// forward
// ---------------------------------------------------------------------------------------------
template <int K, int Ci, bool F32>
__global__ __launch_bounds__(256) void gcn0_fwd_kernel(Gcn0Args a) {
  __shared__ float As[3 * G0_MAXV * G0_MAXV];
  __shared__ float xs[G0_FB * G0_MAXV * 4];
  __shared__ float zs[G0_FB * G0_MAXV * G0_MAXKC];
  __shared__ float bvs[G0_MAXV * 64];
  __shared__ float red[2][4][64];
  const int tid = threadIdx.x, c = tid & 63, rg = tid >> 6;
  constexpr int KC = K * Ci, C = 64;
  const int V = a.V;
  for (int i = tid; i < K * V * V; i += 256) As[i] = a.A[i];
  for (int i = tid; i < V * C; i += 256) bvs[i] = a.beff[i];
  const float* xf = reinterpret_cast<const float*>(a.x);
  const float* wf = reinterpret_cast<const float*>(a.w);
  float* zf = reinterpret_cast<float*>(a.z);
  float* gf = reinterpret_cast<float*>(a.g);
  float wv[KC];
#pragma unroll
  for (int j = 0; j < KC; ++j) wv[j] = F32 ? wf[c * KC + j] : g0_bf(a.w[c * KC + j]);
  float ssum = 0.f, ssq = 0.f;
  for (int f0 = blockIdx.x * G0_FB; f0 < a.frames; f0 += gridDim.x * G0_FB) {
    const int nf = min(G0_FB, a.frames - f0);
    __syncthreads();
    for (int i = tid; i < nf * V * Ci; i += 256) xs[i] = F32 ? xf[(size_t)f0 * V * Ci + i] : g0_bf(a.x[(size_t)f0 * V * Ci + i]);
    __syncthreads();
    // Z[f][w][k][ci] = sum_v A_eff[k][v][w] x[f][v][ci] (v ascending, as mix_fwd_kernel), bf16
    for (int o = tid; o < nf * V * KC; o += 256) {
      const int ci = o % Ci, t = o / Ci, k = t % K, t2 = t / K, w = t2 % V, fl = t2 / V;
      float acc = 0.f;
      for (int v = 0; v < V; ++v) acc += As[(k * V + v) * V + w] * xs[(fl * V + v) * Ci + ci];
      if (F32) {
        zf[(size_t)f0 * V * KC + o] = acc;
        zs[o] = acc;
      } else {
        const unsigned short zb = g0_rne(acc);
        a.z[(size_t)f0 * V * KC + o] = zb;
        zs[o] = g0_bf(zb);
      }
    }
    __syncthreads();
    // g[row][c] = sum_j Z[row][j] W[c][j] + bias_eff[v][c]
    for (int r = rg, w = rg; r < nf * V; r += 4) {
      float acc = 0.f;
#pragma unroll
      for (int j = 0; j < KC; ++j) acc += zs[r * KC + j] * wv[j];
      acc += bvs[w * C + c];
      w += 4;
      if (w >= V) w -= V;  // (V >= 4)
      if (F32) gf[((size_t)f0 * V + r) * C + c] = acc;
      else a.g[((size_t)f0 * V + r) * C + c] = g0_rne(acc);
      ssum += acc;
      ssq += acc * acc;
    }
  }
  red[0][rg][c] = ssum;
  red[1][rg][c] = ssq;
  __syncthreads();
  if (tid < 128) {
    const int q = tid >> 6;
    const float s = (red[q][0][c] + red[q][1][c]) + (red[q][2][c] + red[q][3][c]);
    atomic_add_d((q ? a.st_sq : a.st_sum) + c, (double)s);
  }
}

// ---------------------------------------------------------------------------------------------
// backward
// ---------------------------------------------------------------------------------------------
template <int K, int Ci, bool F32>
__global__ __launch_bounds__(256) void gcn0_bwd_kernel(Gcn0Args a) {
  __shared__ float As[3 * G0_MAXV * G0_MAXV];
  __shared__ float xs[G0_FB * G0_MAXV * 4];
  __shared__ float zs[G0_FB * G0_MAXV * G0_MAXKC];   // Z of the forward
  __shared__ float dzs[G0_FB * G0_MAXV * G0_MAXKC];  // dZ
  __shared__ float red[4][64 * G0_MAXKC];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, c = lane, rg = wave;
  constexpr int KC = K * Ci, C = 64;
  const int V = a.V, KVV = K * V * V;
  const int fr = lane & 15, fg = lane >> 4;
  for (int i = tid; i < KVV; i += 256) As[i] = a.A[i];
  // MFMA B operand (dZ = dg . W: k = c, n = j): lane (fg, fr) holds W[c = s*32 + fg*8 + e][j = fr]
  bf16x8 wb[2];
  // F32: v_mfma_f32_16x16x4_f32 steps s = 0..15, k slot fg of step s = channel c = fg*16 + s: lane
  // (fg, fr) holds W[fg*16 + s][fr] (A: dg[row fr][fg*16 + s], 16 consecutive floats per lane)
  float wf32[F32 ? 16 : 1];
  const float* wf = reinterpret_cast<const float*>(a.w);
  const float* xf = reinterpret_cast<const float*>(a.x);
  const float* zf = reinterpret_cast<const float*>(a.z);
  const float* dgf = reinterpret_cast<const float*>(a.dg);
  if (F32) {
#pragma unroll
    for (int s = 0; s < 16; ++s) wf32[s] = fr < KC ? wf[(fg * 16 + s) * KC + fr] : 0.f;
  } else {
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int cc = s * 32 + fg * 8 + e;
        const unsigned short u = fr < KC ? a.w[cc * KC + fr] : (unsigned short)0;
        wb[s][e] = __builtin_bit_cast(__bf16, u);
      }
  }
  float dacc[4] = {0.f, 0.f, 0.f, 0.f};  // dA_eff entries tid + 256 q
  float wacc[KC];                        // dW[.][c][.] over this thread's rows (j = k*Ci + ci)
#pragma unroll
  for (int j = 0; j < KC; ++j) wacc[j] = 0.f;
  int dv[4], dw[4], dk[4];  // (k, v, w) of the thread's dA_eff entries
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int idx = min(tid + q * 256, KVV - 1);
    dk[q] = idx / (V * V);
    const int r = idx - dk[q] * V * V;
    dv[q] = r / V;
    dw[q] = r - dv[q] * V;
  }
  for (int f0 = blockIdx.x * G0_FB; f0 < a.frames; f0 += gridDim.x * G0_FB) {
    const int nf = min(G0_FB, a.frames - f0), nr = nf * V;
    __syncthreads();
    for (int i = tid; i < nf * V * Ci; i += 256) xs[i] = F32 ? xf[(size_t)f0 * V * Ci + i] : g0_bf(a.x[(size_t)f0 * V * Ci + i]);
    for (int i = tid; i < nr * KC; i += 256) zs[i] = F32 ? zf[(size_t)f0 * V * KC + i] : g0_bf(a.z[(size_t)f0 * V * KC + i]);
    // dZ tiles of 16 rows: A fragment = 8 consecutive dg channels of row r0 + fr (16-B loads)
    for (int t = wave; t * 16 < nr; t += 4) {
      const int r = min(t * 16 + fr, nr - 1);
      f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
      if (F32) {
        const f32x4* dgr = reinterpret_cast<const f32x4*>(dgf + ((size_t)f0 * V + r) * C + fg * 16);
        f32x4 d[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) d[q] = dgr[q];
#pragma unroll
        for (int s = 0; s < 16; ++s) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(d[s >> 2][s & 3], wf32[s], acc, 0, 0, 0);
      } else {
        const unsigned short* dgr = a.dg + ((size_t)f0 * V + r) * C + fg * 8;
#pragma unroll
        for (int s = 0; s < 2; ++s) acc = mfma_bf16x(*reinterpret_cast<const bf16x8*>(dgr + s * 32), wb[s], acc);
      }
      // lane holds dZ[rows t*16 + 4fg + i][col fr]
      if (fr < KC)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int rr = t * 16 + fg * 4 + i;
          if (rr < nr) dzs[rr * KC + fr] = acc[i];
        }
    }
    __syncthreads();
    // dx[f][v][ci] (+)= sum_k sum_w A_eff[k][v][w] dZ[f][w][k][ci]
    for (int o = tid; o < nf * V * Ci; o += 256) {
      const int ci = o % Ci, t = o / Ci, v = t % V, fl = t / V;
      float acc = 0.f;
      for (int k = 0; k < K; ++k)
        for (int w = 0; w < V; ++w) acc += As[(k * V + v) * V + w] * dzs[(fl * V + w) * KC + k * Ci + ci];
      float* dst = a.dx + (size_t)f0 * V * Ci + o;
      if (a.accumulate) *dst += acc;
      else *dst = acc;
    }
    // dA_eff[k][v][w] += sum_{f, ci} x[f][v][ci] dZ[f][w][k][ci]
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      if (tid + q * 256 < KVV) {
        const int k = dk[q], v = dv[q], w = dw[q];
        float acc = 0.f;
        for (int fl = 0; fl < nf; ++fl)
#pragma unroll
          for (int ci = 0; ci < Ci; ++ci) acc += xs[(fl * V + v) * Ci + ci] * dzs[(fl * V + w) * KC + k * Ci + ci];
        dacc[q] += acc;
      }
    }
    // dW[k][c][ci] += sum_rows dg[row][c] Z[row][k*Ci + ci] (rows rg, rg + 4, ... in order; the rows'
    // dg loads issued G0_DWB at a time instead of one round trip per row)
    for (int rb = rg; rb < nr; rb += 4 * G0_DWB) {
      float d[G0_DWB];
#pragma unroll
      for (int i = 0; i < G0_DWB; ++i) {
        const int r = min(rb + 4 * i, nr - 1);
        d[i] = F32 ? dgf[((size_t)f0 * V + r) * C + c] : g0_bf(a.dg[((size_t)f0 * V + r) * C + c]);
      }
#pragma unroll
      for (int i = 0; i < G0_DWB; ++i) {
        const int r = rb + 4 * i;
        if (r < nr) {
#pragma unroll
          for (int j = 0; j < KC; ++j) wacc[j] += d[i] * zs[r * KC + j];
        }
      }
    }
  }
  // this block's partial rows: dA_eff [KVV] at part_dA[blockIdx], dW at part_dW[blockIdx] in the
  // gradient's layout [(k*C + c)*Ci + ci]
  float* pa = a.part_dA + (size_t)blockIdx.x * KVV;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int idx = tid + q * 256;
    if (idx < KVV) pa[idx] = dacc[q];
  }
  __syncthreads();
#pragma unroll
  for (int j = 0; j < KC; ++j) red[rg][c * KC + j] = wacc[j];
  __syncthreads();
  float* pw = a.part_dW + (size_t)blockIdx.x * C * KC;
  for (int e = tid; e < C * KC; e += 256) {
    const int k = e / (C * Ci), r = e - k * C * Ci, cc = r / Ci, ci = r - cc * Ci;
    const int src = cc * KC + k * Ci + ci;
    pw[e] = (red[0][src] + red[1][src]) + (red[2][src] + red[3][src]);
  }
}

// ---------------------------------------------------------------------------------------------
// data_bn gamma / beta gradients: channel (v, c) = index v*C + c of the channels-last rows
// ---------------------------------------------------------------------------------------------
constexpr int DB2_ROWS = 32;  // (n, t) rows per block
__global__ __launch_bounds__(256) void databn_bwd2_kernel(DataBnArgs a) {
  __shared__ double red[2][256];
  const int VC = a.V * a.C;  // <= 100
  const int tid = threadIdx.x, ch = tid % VC, grp = tid / VC, ngrp = 256 / VC;
  const int v = ch / a.C, c = ch - v * a.C;
  float sc, sh, mu, rs;
  bn_coeff(a.bn, ch, sc, sh, mu, rs);
  double s = 0.0, q = 0.0;
  const int NT = a.N * a.T, r0 = blockIdx.x * DB2_ROWS, r1 = min(NT, r0 + DB2_ROWS);
  if (grp < ngrp) {
    const int Ts = a.motion ? a.T + 1 : a.T;
    for (int e = r0 + grp; e < r1; e += ngrp) {
      const int n = e / a.T, t = e - n * a.T;
      const float* p = a.skel + (((size_t)n * 3 + c) * Ts + t) * a.V + v;
      const float x = a.motion ? (p[a.V] - p[0]) : p[0];
      const float dy = a.dout[(size_t)e * VC + ch];
      s += dy;
      q += (double)dy * ((x - mu) * rs);
    }
  }
  red[0][tid] = s;  // thread grp * VC + ch (the idle tail threads hold 0)
  red[1][tid] = q;
  __syncthreads();
  if (tid < VC) {
    double S = 0.0, Q = 0.0;
    for (int g2 = 0; g2 < ngrp; ++g2) { S += red[0][g2 * VC + tid]; Q += red[1][g2 * VC + tid]; }
    if (a.part) {  // this block's partial row [gamma (VC) | beta (VC)], summed in block order
      a.part[(size_t)blockIdx.x * 2 * VC + tid] = (float)Q;
      a.part[(size_t)blockIdx.x * 2 * VC + VC + tid] = (float)S;
    } else {
      atomic_add_f(a.dgamma + tid, (float)Q);
      atomic_add_f(a.dbeta + tid, (float)S);
    }
  }
}

}  // namespace f3

using namespace f3;

// instantiated: K = 3 partitions (the 'spatial' strategy) with 3 (positions) or 2 input channels
bool f3_gcn0_ok(int K, int V, int Ci, int C) {
  return C == 64 && K == 3 && (Ci == 2 || Ci == 3) && V >= 4 && V <= G0_MAXV &&
         K * V * V <= 1024;  // dA_eff: 4 entries per thread
}

// ~2 blocks of 8 frames each per workgroup: 1-2 resident workgroups per SIMD hide the LDS and
// integer latency the 1-per-CU form exposed (78 / 105 us alone -> see profiles/r03_layer0_ab.txt)
static int g0_grid(int frames) { return std::max(1, std::min(480, (frames + G0_FB - 1) / G0_FB)); }

int f3_gcn0_fwd(const Gcn0Args* a, hipStream_t s) {
  if (!f3_gcn0_ok(a->K, a->V, a->Ci, 64)) return F3_EINVAL;
  const dim3 grid(g0_grid(a->frames));
  if (a->f32) {
    if (a->Ci == 3) hipLaunchKernelGGL((gcn0_fwd_kernel<3, 3, true>), grid, dim3(256), 0, s, *a);
    else hipLaunchKernelGGL((gcn0_fwd_kernel<3, 2, true>), grid, dim3(256), 0, s, *a);
  } else {
    if (a->Ci == 3) hipLaunchKernelGGL((gcn0_fwd_kernel<3, 3, false>), grid, dim3(256), 0, s, *a);
    else hipLaunchKernelGGL((gcn0_fwd_kernel<3, 2, false>), grid, dim3(256), 0, s, *a);
  }
  F3_LAUNCH_CHECK();
  return F3_OK;
}

int f3_gcn0_bwd_parts(const Gcn0Args* a) { return g0_grid(a->frames); }

int f3_gcn0_bwd(const Gcn0Args* a, hipStream_t s) {
  if (!f3_gcn0_ok(a->K, a->V, a->Ci, 64) || !a->part_dA || !a->part_dW) return F3_EINVAL;
  const dim3 grid(g0_grid(a->frames));
  if (a->f32) {
    if (a->Ci == 3) hipLaunchKernelGGL((gcn0_bwd_kernel<3, 3, true>), grid, dim3(256), 0, s, *a);
    else hipLaunchKernelGGL((gcn0_bwd_kernel<3, 2, true>), grid, dim3(256), 0, s, *a);
  } else {
    if (a->Ci == 3) hipLaunchKernelGGL((gcn0_bwd_kernel<3, 3, false>), grid, dim3(256), 0, s, *a);
    else hipLaunchKernelGGL((gcn0_bwd_kernel<3, 2, false>), grid, dim3(256), 0, s, *a);
  }
  F3_LAUNCH_CHECK();
  return F3_OK;
}

int f3_databn_bwd2(const DataBnArgs* a, hipStream_t s) {
  if (a->V * a->C > 256 || a->C > 4) return F3_EINVAL;
  const int rows = a->N * a->T;
  const int blocks = (rows + DB2_ROWS - 1) / DB2_ROWS, VC = a->V * a->C;
  hipLaunchKernelGGL(databn_bwd2_kernel, dim3(blocks), dim3(256), 0, s, *a);
  F3_LAUNCH_CHECK();
  if (!a->part) return F3_OK;
  const ColsumJob j[2] = {{a->part, a->dgamma, 2LL * VC, blocks, VC}, {a->part + VC, a->dbeta, 2LL * VC, blocks, VC}};
  return f3_colsum_multi(j, 2, s);
}
