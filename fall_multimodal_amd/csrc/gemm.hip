// Implicit-GEMM temporal convolution over channels-last [N][T][V][C] activations,
// fp32 in / fp32 accumulate on the gfx950 matrix cores (v_mfma_f32_16x16x4_f32,
// exact f32: every product rounded once, fmaf-chain numerics).
//
// One template covers every channel contraction of an st_gcan block
// (Multimodal_Fall3/model/stgcan.py):
//   * gcn 1x1 conv after the graph mix  (KT=1)           stgcan.py:51
//   * tcn (9,1) conv, stride 1/2, pad 4                   stgcan.py:114-118
//   * residual 1x1 conv, stride 2                         stgcan.py:128-131
//   * their input-gradients (transposed row map)          autograd of the above
// and a second template computes the weight gradients (reduction over all rows,
// split across workgroups, f32 atomics into the reference-layout .grad buffer).
//
// Tile: 64 rows x 64 output channels per 256-thread workgroup (4 waves, 32x32 each,
// 2x2 MFMA 16x16 sub-tiles), K staged 16 at a time through LDS (double buffered,
// one barrier per K chunk). The MFMA k index inside a chunk is permuted
// (lane group g, step s -> k = 4g+s) so each lane's A and B fragments are one
// ds_read_b128; rows padded to 24 floats are bank-conflict free for that read.
#include "common.h"
#include "kernels.h"

namespace f3 {

constexpr int BM = 64, BN = 64, BK = 16, LDK = 24;

F3_DEV f32x4 mfma4(float a, float b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

// source row of output row m for temporal tap dt; -1 when the tap hits zero padding
F3_DEV int src_row(int n, int t, int v, int dt, const ConvGeom& g) {
  int ti;
  if (!g.transposed) {
    ti = t * g.S + dt - g.P;
    if (ti < 0 || ti >= g.T_in) return -1;
  } else {
    int num = t + g.P - dt;
    if (num < 0 || (num % g.S) != 0) return -1;
    ti = num / g.S;
    if (ti >= g.T_in) return -1;
  }
  return (n * g.T_in + ti) * g.V + v;
}

template <int PRO, int EPI>
__global__ __launch_bounds__(256) void conv_gemm_f32(ConvGemmArgs a) {
  __shared__ __attribute__((aligned(16))) float As[2][BM][LDK];
  __shared__ __attribute__((aligned(16))) float Bs[2][BN][LDK];
  __shared__ float pro_sc[256], pro_sh[256];
  __shared__ float epi_sc[BN], epi_sh[BN], epi_mu[BN], epi_rs[BN];
  __shared__ float red[2][2][BN];

  const ConvGeom& g = a.g;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int m0 = blockIdx.x * BM, j0 = blockIdx.y * BN;
  const int Ktot = g.KT * g.Kc;
  const int nchunk = (Ktot + BK - 1) / BK;
  const bool fastA = (g.Kc % BK) == 0 && (g.lda % 4) == 0;
  const bool fastB = (Ktot % BK) == 0;

  if (PRO) {
    for (int i = tid; i < g.Kc; i += 256) {
      float sc, sh, mu, rs;
      bn_coeff(a.pro_bn, i, sc, sh, mu, rs);
      pro_sc[i] = sc;
      pro_sh[i] = sh;
    }
  }
  if (EPI & EPI_RELUMASK) {
    if (tid < BN && j0 + tid < g.Nc) {
      float sc, sh, mu, rs;
      bn_coeff(a.epi_bn, j0 + tid, sc, sh, mu, rs);
      epi_sc[tid] = sc; epi_sh[tid] = sh; epi_mu[tid] = mu; epi_rs[tid] = rs;
    }
  }

  // loader assignment: one float4 of A and one of B per thread per chunk
  const int lr = tid >> 2, lk = (tid & 3) * 4;
  const int am = m0 + lr;
  int an = 0, at = 0, av = 0;
  const bool arow = am < g.M;
  if (arow) {
    int nt = am / g.V;
    av = am - nt * g.V;
    an = nt / g.T_out;
    at = nt - an * g.T_out;
  }
  const int bj = j0 + lr;

  float ra[4], rb[4];
  auto load_chunk = [&](int c) {
    const int k0 = c * BK + lk;
    // A
    if (fastA) {
      const int dt = k0 / g.Kc, i = k0 - dt * g.Kc;
      const int r = arow ? src_row(an, at, av, dt, g) : -1;
      if (r >= 0) {
        f32x4 v = *reinterpret_cast<const f32x4*>(a.in + (size_t)r * g.lda + i);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          float x = v[e];
          if (PRO) x = fmaxf(x * pro_sc[i + e] + pro_sh[i + e], 0.f);
          ra[e] = x;
        }
      } else {
#pragma unroll
        for (int e = 0; e < 4; ++e) ra[e] = 0.f;
      }
    } else {
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int k = k0 + e;
        float x = 0.f;
        if (arow && k < Ktot) {
          const int dt = k / g.Kc, i = k - dt * g.Kc;
          const int r = src_row(an, at, av, dt, g);
          if (r >= 0) {
            x = a.in[(size_t)r * g.lda + i];
            if (PRO) x = fmaxf(x * pro_sc[i] + pro_sh[i], 0.f);
          }
        }
        ra[e] = x;
      }
    }
    // B (packed [Nc][Ktot])
    if (bj < g.Nc && fastB) {
      f32x4 v = *reinterpret_cast<const f32x4*>(a.w + (size_t)bj * Ktot + k0);
#pragma unroll
      for (int e = 0; e < 4; ++e) rb[e] = v[e];
    } else {
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int k = k0 + e;
        rb[e] = (bj < g.Nc && k < Ktot) ? a.w[(size_t)bj * Ktot + k] : 0.f;
      }
    }
  };
  auto store_chunk = [&](int buf) {
    *reinterpret_cast<f32x4*>(&As[buf][lr][lk]) = f32x4{ra[0], ra[1], ra[2], ra[3]};
    *reinterpret_cast<f32x4*>(&Bs[buf][lr][lk]) = f32x4{rb[0], rb[1], rb[2], rb[3]};
  };

  if (PRO) __syncthreads();  // pro_sc ready before the first load
  load_chunk(0);
  store_chunk(0);
  __syncthreads();

  const int wm = wave >> 1, wj = wave & 1;
  const int fr = lane & 15, fg = lane >> 4;
  f32x4 acc[2][2];
#pragma unroll
  for (int x = 0; x < 2; ++x)
#pragma unroll
    for (int y = 0; y < 2; ++y) acc[x][y] = f32x4{0.f, 0.f, 0.f, 0.f};

  for (int c = 0; c < nchunk; ++c) {
    const int buf = c & 1;
    if (c + 1 < nchunk) load_chunk(c + 1);
    f32x4 fa[2], fb[2];
#pragma unroll
    for (int x = 0; x < 2; ++x)
      fa[x] = *reinterpret_cast<const f32x4*>(&As[buf][wm * 32 + x * 16 + fr][4 * fg]);
#pragma unroll
    for (int y = 0; y < 2; ++y)
      fb[y] = *reinterpret_cast<const f32x4*>(&Bs[buf][wj * 32 + y * 16 + fr][4 * fg]);
#pragma unroll
    for (int s = 0; s < 4; ++s)
#pragma unroll
      for (int x = 0; x < 2; ++x)
#pragma unroll
        for (int y = 0; y < 2; ++y) acc[x][y] = mfma4(fa[x][s], fb[y][s], acc[x][y]);
    if (c + 1 < nchunk) store_chunk(buf ^ 1);
    __syncthreads();
  }

  // ---------------- epilogue ----------------
  float ssum[2] = {0.f, 0.f}, ssq[2] = {0.f, 0.f};
  float gap0[2] = {0.f, 0.f}, gap1[2] = {0.f, 0.f};
  const int TV = g.T_out * g.V;
  const int nlo = m0 / TV;
#pragma unroll
  for (int y = 0; y < 2; ++y) {
    const int jl = wj * 32 + y * 16 + fr;
    const int j = j0 + jl;
    const bool jok = j < g.Nc;
#pragma unroll
    for (int x = 0; x < 2; ++x) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = m0 + wm * 32 + x * 16 + fg * 4 + r;
        if (!jok || m >= g.M) continue;
        float v = acc[x][y][r];
        if (EPI & EPI_BIAS) v += a.bias[j];
        if (EPI & EPI_BIASV) v += a.bias[(m % g.V) * g.Nc + j];
        if (EPI & EPI_RELUMASK) {
          const float gv = a.aux[(size_t)m * a.ldaux + j];
          if (gv * epi_sc[jl] + epi_sh[jl] <= 0.f) v = 0.f;
          const float xh = (gv - epi_mu[jl]) * epi_rs[jl];
          ssum[y] += v;
          ssq[y] += v * xh;
        } else if (EPI & EPI_STATS) {
          ssum[y] += v;
          ssq[y] += v * v;
        }
        if (EPI & EPI_GAP) {
          const int n = m / TV;
          if (n == nlo) gap0[y] += v;
          else if (n == nlo + 1) gap1[y] += v;
          else atomic_add_f(a.gap + (size_t)n * g.Nc + j, v);
        }
        float* o = a.out + (size_t)m * g.ldo + j;
        if (EPI & EPI_ADD) *o += v;
        else *o = v;
      }
    }
  }
  if (EPI & (EPI_STATS | EPI_RELUMASK | EPI_GAP)) {
    // reduce over the 4 lane groups (rows) of each column, then over the two row-waves
#pragma unroll
    for (int y = 0; y < 2; ++y) {
#pragma unroll
      for (int o = 16; o < 64; o <<= 1) {
        ssum[y] += __shfl_xor(ssum[y], o, 64);
        ssq[y] += __shfl_xor(ssq[y], o, 64);
        gap0[y] += __shfl_xor(gap0[y], o, 64);
        gap1[y] += __shfl_xor(gap1[y], o, 64);
      }
    }
    __shared__ float gred[2][2][BN];
    if (fg == 0) {
#pragma unroll
      for (int y = 0; y < 2; ++y) {
        const int jl = wj * 32 + y * 16 + fr;
        red[wm][0][jl] = ssum[y];
        red[wm][1][jl] = ssq[y];
        gred[wm][0][jl] = gap0[y];
        gred[wm][1][jl] = gap1[y];
      }
    }
    __syncthreads();
    if (tid < BN && j0 + tid < g.Nc) {
      const int j = j0 + tid;
      if (EPI & (EPI_STATS | EPI_RELUMASK)) {
        atomic_add_d(a.st_sum + j, (double)(red[0][0][tid] + red[1][0][tid]));
        atomic_add_d(a.st_sq + j, (double)(red[0][1][tid] + red[1][1][tid]));
      }
      if (EPI & EPI_GAP) {
        const float s0 = gred[0][0][tid] + gred[1][0][tid];
        const float s1 = gred[0][1][tid] + gred[1][1][tid];
        atomic_add_f(a.gap + (size_t)nlo * g.Nc + j, s0);
        if ((nlo + 1) * TV < g.M && s1 != 0.f) atomic_add_f(a.gap + (size_t)(nlo + 1) * g.Nc + j, s1);
      }
    }
  }
}

// dW[j][i'] = sum_m dY[m][j] * pro(In[src(m,dt)][i])   (split-K over rows, f32 atomics)
template <int PRO>
__global__ __launch_bounds__(256) void conv_wgrad_f32(WgradArgs a_) {
  WgradArgs a = a_;
  const int nsplit = (a.g.M + a.rows_per_split - 1) / a.rows_per_split;
  const int zsplit = blockIdx.z % nsplit;
  wgrad_group(a, blockIdx.z / nsplit);
  __shared__ __attribute__((aligned(16))) float Ys[2][BN][LDK];
  __shared__ __attribute__((aligned(16))) float Xs[2][BN][LDK];
  __shared__ float pro_sc[256], pro_sh[256];
  const ConvGeom& g = a.g;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int j0 = blockIdx.x * BN;
  const int itiles = (g.Kc + BN - 1) / BN;
  const int dt = blockIdx.y / itiles;
  const int i0 = (blockIdx.y - dt * itiles) * BN;
  const int r_begin = zsplit * a.rows_per_split;
  const int r_end = min(g.M, r_begin + a.rows_per_split);
  if (PRO) {
    for (int i = tid; i < g.Kc; i += 256) {
      float sc, sh, mu, rs;
      bn_coeff(a.pro_bn, i, sc, sh, mu, rs);
      pro_sc[i] = sc;
      pro_sh[i] = sh;
    }
    __syncthreads();
  }
  const bool fastY = (a.ldy % 4) == 0 && (g.Nc % 4) == 0;
  const bool fastX = (g.lda % 4) == 0 && (g.Kc % 4) == 0;
  const int lrow = tid >> 4, lq = (tid & 15) * 4;
  float ry[4], rx[4];
  auto load_chunk = [&](int r0) {
    const int m = r0 + lrow;
    const bool ok = m < r_end;
    const int j = j0 + lq;
    if (ok && fastY && j < g.Nc) {
      f32x4 v = *reinterpret_cast<const f32x4*>(a.dy + (size_t)m * a.ldy + j);
#pragma unroll
      for (int e = 0; e < 4; ++e) ry[e] = v[e];
    } else {
#pragma unroll
      for (int e = 0; e < 4; ++e) ry[e] = (ok && j + e < g.Nc) ? a.dy[(size_t)m * a.ldy + j + e] : 0.f;
    }
    int r = -1;
    if (ok) {
      int nt = m / g.V;
      int v = m - nt * g.V;
      int n = nt / g.T_out;
      int t = nt - n * g.T_out;
      r = src_row(n, t, v, dt, g);
    }
    const int i = i0 + lq;
    if (r >= 0 && fastX && i < g.Kc) {
      f32x4 v = *reinterpret_cast<const f32x4*>(a.in + (size_t)r * g.lda + i);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        float x = v[e];
        if (PRO) x = fmaxf(x * pro_sc[i + e] + pro_sh[i + e], 0.f);
        rx[e] = x;
      }
    } else {
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        float x = 0.f;
        if (r >= 0 && i + e < g.Kc) {
          x = a.in[(size_t)r * g.lda + i + e];
          if (PRO) x = fmaxf(x * pro_sc[i + e] + pro_sh[i + e], 0.f);
        }
        rx[e] = x;
      }
    }
  };
  auto store_chunk = [&](int buf) {
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      Ys[buf][lq + e][lrow] = ry[e];
      Xs[buf][lq + e][lrow] = rx[e];
    }
  };
  const int wm = wave >> 1, wj = wave & 1;
  const int fr = lane & 15, fg = lane >> 4;
  f32x4 acc[2][2];
#pragma unroll
  for (int x = 0; x < 2; ++x)
#pragma unroll
    for (int y = 0; y < 2; ++y) acc[x][y] = f32x4{0.f, 0.f, 0.f, 0.f};
  float dbacc = 0.f;
  const bool do_db = a.db && blockIdx.y == 0;

  if (r_begin < r_end) {
    load_chunk(r_begin);
    store_chunk(0);
    __syncthreads();
    int buf = 0;
    for (int r0 = r_begin; r0 < r_end; r0 += BK) {
      const bool more = r0 + BK < r_end;
      if (more) load_chunk(r0 + BK);
      f32x4 fa[2], fb[2];
#pragma unroll
      for (int x = 0; x < 2; ++x)
        fa[x] = *reinterpret_cast<const f32x4*>(&Ys[buf][wm * 32 + x * 16 + fr][4 * fg]);
#pragma unroll
      for (int y = 0; y < 2; ++y)
        fb[y] = *reinterpret_cast<const f32x4*>(&Xs[buf][wj * 32 + y * 16 + fr][4 * fg]);
#pragma unroll
      for (int s = 0; s < 4; ++s)
#pragma unroll
        for (int x = 0; x < 2; ++x)
#pragma unroll
          for (int y = 0; y < 2; ++y) acc[x][y] = mfma4(fa[x][s], fb[y][s], acc[x][y]);
      if (do_db && tid < BN) {
#pragma unroll
        for (int k = 0; k < BK; ++k) dbacc += Ys[buf][tid][k];
      }
      if (more) store_chunk(buf ^ 1);
      __syncthreads();
      buf ^= 1;
    }
  }
  if (do_db && tid < BN && j0 + tid < g.Nc && r_begin < r_end) atomic_add_f(a.db + j0 + tid, dbacc);
  // scatter-add into the reference weight layout
#pragma unroll
  for (int x = 0; x < 2; ++x) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int j = j0 + wm * 32 + x * 16 + fg * 4 + r;
      if (j >= g.Nc) continue;
#pragma unroll
      for (int y = 0; y < 2; ++y) {
        const int i = i0 + wj * 32 + y * 16 + fr;
        if (i >= g.Kc) continue;
        size_t idx;
        if (a.outmap == WG_OUT_CONV) {
          idx = ((size_t)j * g.Kc + i) * g.KT + dt;
        } else {  // gcn: i = k*Cin + ci  ->  W[k*C + j][ci]
          const int k = i / a.gcn_cin, ci = i - k * a.gcn_cin;
          idx = ((size_t)k * g.Nc + j) * a.gcn_cin + ci;
        }
        atomic_add_f(a.dw + idx, acc[x][y][r]);
      }
    }
  }
}

}  // namespace f3

using namespace f3;

int f3_conv_gemm(const ConvGemmArgs* args, int pro, int epi, hipStream_t s) {
  const ConvGemmArgs& a = *args;
  if (a.x3) return f3_conv_gemm_x3(args, pro, epi, s);
  if (a.wb) return f3_conv_gemm_bf16(args, pro, epi, s);
  if (a.g.M <= 0 || a.g.Nc <= 0) return F3_OK;
  if (pro && a.g.Kc > 256) return F3_EINVAL;
  dim3 grid((a.g.M + BM - 1) / BM, (a.g.Nc + BN - 1) / BN);
#define F3_GEMM_CASE(P, E)                                                   \
  if (pro == P && epi == (E)) {                                             \
    hipLaunchKernelGGL((conv_gemm_f32<P, (E)>), grid, dim3(256), 0, s, a); \
    F3_LAUNCH_CHECK();                                                       \
    return F3_OK;                                                            \
  }
  F3_GEMM_CASE(0, EPI_BIASV | EPI_STATS)                 // gcn forward
  F3_GEMM_CASE(1, EPI_BIAS | EPI_STATS | EPI_GAP)        // tcn forward
  F3_GEMM_CASE(0, EPI_BIAS | EPI_STATS)                  // residual forward
  F3_GEMM_CASE(0, EPI_RELUMASK)                          // tcn dgrad (+BN1 bwd sums)
  F3_GEMM_CASE(0, 0)                                     // gcn dgrad
  F3_GEMM_CASE(0, EPI_ADD)                               // residual dgrad
  F3_GEMM_CASE(0, EPI_BIAS)                              // plain conv (tests)
  F3_GEMM_CASE(1, 0)                                     // tests
#undef F3_GEMM_CASE
  return F3_EINVAL;
}

int f3_conv_wgrad(const WgradArgs* args, int pro, hipStream_t s) {
  if (args->x3) return f3_conv_wgrad_x3(args, pro, s);
  if (args->bf16) {
    if (!pro && f3_wgrad_glds_ok(*args)) return f3_wgrad_glds_bf16(args, s);
    return f3_conv_wgrad_bf16(args, pro, s);
  }
  WgradArgs a = *args;
  if (a.g.M <= 0) return F3_OK;
  if (pro && a.g.Kc > 256) return F3_EINVAL;
  const int gx = (a.g.Nc + BN - 1) / BN;
  const int gy = a.g.KT * ((a.g.Kc + BN - 1) / BN);
  int splits = (f3_wgrad_target_wgs() + gx * gy - 1) / (gx * gy);
  int rps = (a.g.M + splits - 1) / splits;
  rps = ((rps + BK - 1) / BK) * BK;
  if (rps < 4 * BK) rps = 4 * BK;
  splits = (a.g.M + rps - 1) / rps;
  a.rows_per_split = rps;
  dim3 grid(gx, gy, splits * std::max(1, a.groups));
  if (pro) hipLaunchKernelGGL(conv_wgrad_f32<1>, grid, dim3(256), 0, s, a);
  else hipLaunchKernelGGL(conv_wgrad_f32<0>, grid, dim3(256), 0, s, a);
  F3_LAUNCH_CHECK();
  return F3_OK;
}
