// bf16 MFMA (v_mfma_f32_16x16x32_bf16, fp32 accumulate) forms of the implicit-GEMM
// temporal convolution and its weight gradient — the throughput mode of the step.
//
// Activations stay fp32 in HBM (the fp32 parity mode reads the same buffers); each tile
// is converted to bf16 while it is staged into LDS, after the optional BN+ReLU prologue
// has been applied in fp32. Weights come pre-packed in bf16 from the prep kernel.
//
//   conv_gemm_bf16 : Out[m][j] = sum_{dt,i} pro(In[src(m,dt)][i]) W[j][dt*Kc+i]   (fwd / dgrad)
//     A tile [BM rows][32 k] and B tile [BN cols][32 k], k contiguous (96-B LDS rows:
//     the 16-lane x 16-B ds_read_b128 fragment pattern is conflict-free);
//   conv_wgrad_bf16: dW[j][i'] = sum_m dY[m][j] pro(In[src(m,dt)][i])
//     the reduction index m is the ROW index in memory, so both tiles are staged
//     row-major [32 m][cols] and read with ds_read_b64_tr_b16 (gfx950 transposed LDS
//     read: 4 rows x 16 columns per 16-lane group, column i to lane i).
#include "common.h"
#include "kernels.h"

namespace f3 {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef short s16x8 __attribute__((ext_vector_type(8)));

constexpr int HBK = 32;  // k (or m) per chunk
constexpr int HLD = 48;  // LDS row stride (bf16) of the k-contiguous tiles

F3_DEV f32x4 mfma_bf16(bf16x8 a, bf16x8 b, f32x4 c) { return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0); }

F3_DEV int src_row_b(int n, int t, int v, int dt, const ConvGeom& g) {
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

template <int PRO, int EPI, int WM, int WN>
__global__ __launch_bounds__(256) void conv_gemm_bf16(ConvGemmArgs a) {
  constexpr int BM = 32 * WM, BN = 32 * WN;
  constexpr int KPT = BM / 8;    // A values per thread per chunk (8 or 16)
  constexpr int TPR = HBK / KPT; // threads per A row
  constexpr int BPT = BN / 8;    // B values per thread per chunk (8 or 16)
  constexpr int TPB = HBK / BPT;
  __shared__ __attribute__((aligned(16))) __bf16 As[2][BM][HLD];
  __shared__ __attribute__((aligned(16))) __bf16 Bs[2][BN][HLD];
  __shared__ float pro_sc[256], pro_sh[256];
  __shared__ float epi_sc[BN], epi_sh[BN], epi_mu[BN], epi_rs[BN];
  __shared__ float red[2][2][BN], gred[2][2][BN];

  const ConvGeom& g = a.g;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int m0 = blockIdx.x * BM, j0 = blockIdx.y * BN;
  const int Ktot = g.KT * g.Kc;
  const int nchunk = (Ktot + HBK - 1) / HBK;
  const bool fastA = (g.Kc % HBK) == 0 && (g.lda % (a.inb ? 8 : 4)) == 0;
  const bool fastB = (Ktot % 8) == 0;
  const unsigned short* wb = reinterpret_cast<const unsigned short*>(a.wb);

  if (PRO) {
    for (int i = tid; i < g.Kc; i += 256) {
      float sc, sh, mu, rs;
      bn_coeff(a.pro_bn, i, sc, sh, mu, rs);
      pro_sc[i] = sc;
      pro_sh[i] = sh;
    }
  }
  if (EPI & EPI_RELUMASK) {
    for (int t = tid; t < BN; t += 256) {
      if (j0 + t < g.Nc) {
        float sc, sh, mu, rs;
        bn_coeff(a.epi_bn, j0 + t, sc, sh, mu, rs);
        epi_sc[t] = sc; epi_sh[t] = sh; epi_mu[t] = mu; epi_rs[t] = rs;
      }
    }
  }
  const int lr = tid / TPR, lk = (tid % TPR) * KPT;
  const int am = m0 + lr;
  int an = 0, at = 0, av = 0;
  const bool arow = am < g.M;
  if (arow) {
    int nt = am / g.V;
    av = am - nt * g.V;
    an = nt / g.T_out;
    at = nt - an * g.T_out;
  }
  const int br = tid / TPB, bk = (tid % TPB) * BPT;
  const int bj = j0 + br;

  float ra[KPT];
  unsigned short rb[BPT];
  auto load_chunk = [&](int c) {
    const int k0 = c * HBK + lk;
    if (fastA) {
      const int dt = k0 / g.Kc, i = k0 - dt * g.Kc;
      const int r = arow ? src_row_b(an, at, av, dt, g) : -1;
      if (r >= 0 && a.inb) {  // bf16 activations (alignment: lda % 8 == 0, checked by the launcher)
        const bf16x8* p = reinterpret_cast<const bf16x8*>(a.inb + (size_t)r * g.lda + i);
#pragma unroll
        for (int q = 0; q < KPT / 8; ++q) {
          const bf16x8 v = p[q];
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            float x = (float)v[e];
            if (PRO) x = fmaxf(x * pro_sc[i + 8 * q + e] + pro_sh[i + 8 * q + e], 0.f);
            ra[8 * q + e] = x;
          }
        }
      } else if (r >= 0) {
        const f32x4* p = reinterpret_cast<const f32x4*>(a.in + (size_t)r * g.lda + i);
#pragma unroll
        for (int q = 0; q < KPT / 4; ++q) {
          const f32x4 v = p[q];
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            float x = v[e];
            if (PRO) x = fmaxf(x * pro_sc[i + 4 * q + e] + pro_sh[i + 4 * q + e], 0.f);
            ra[4 * q + e] = x;
          }
        }
      } else {
#pragma unroll
        for (int e = 0; e < KPT; ++e) ra[e] = 0.f;
      }
    } else {
#pragma unroll
      for (int e = 0; e < KPT; ++e) {
        const int k = k0 + e;
        float x = 0.f;
        if (arow && k < Ktot) {
          const int dt = k / g.Kc, i = k - dt * g.Kc;
          const int r = src_row_b(an, at, av, dt, g);
          if (r >= 0) {
            x = a.inb ? (float)reinterpret_cast<const __bf16*>(a.inb)[(size_t)r * g.lda + i]
                      : a.in[(size_t)r * g.lda + i];
            if (PRO) x = fmaxf(x * pro_sc[i] + pro_sh[i], 0.f);
          }
        }
        ra[e] = x;
      }
    }
    const int kb = c * HBK + bk;
    if (bj < g.Nc && fastB && kb + BPT <= Ktot) {
      const uint4* p = reinterpret_cast<const uint4*>(wb + (size_t)bj * Ktot + kb);
#pragma unroll
      for (int q = 0; q < BPT / 8; ++q) {
        const uint4 v = p[q];
        const unsigned short* s = reinterpret_cast<const unsigned short*>(&v);
#pragma unroll
        for (int e = 0; e < 8; ++e) rb[8 * q + e] = s[e];
      }
    } else {
#pragma unroll
      for (int e = 0; e < BPT; ++e) {
        const int k = kb + e;
        rb[e] = (bj < g.Nc && k < Ktot) ? wb[(size_t)bj * Ktot + k] : (unsigned short)0;
      }
    }
  };
  auto store_chunk = [&](int buf) {
#pragma unroll
    for (int q = 0; q < KPT / 8; ++q) {
      bf16x8 v;
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = (__bf16)ra[8 * q + e];
      *reinterpret_cast<bf16x8*>(&As[buf][lr][lk + 8 * q]) = v;
    }
#pragma unroll
    for (int q = 0; q < BPT / 8; ++q) {
      uint4 v;
      unsigned short* s = reinterpret_cast<unsigned short*>(&v);
#pragma unroll
      for (int e = 0; e < 8; ++e) s[e] = rb[8 * q + e];
      *reinterpret_cast<uint4*>(&Bs[buf][br][bk + 8 * q]) = v;
    }
  };

  __syncthreads();  // prologue / epilogue coefficient tables
  load_chunk(0);
  store_chunk(0);
  __syncthreads();

  const int wm = wave >> 1, wj = wave & 1;
  const int fr = lane & 15, fg = lane >> 4;
  f32x4 acc[WM][WN];
#pragma unroll
  for (int x = 0; x < WM; ++x)
#pragma unroll
    for (int y = 0; y < WN; ++y) acc[x][y] = f32x4{0.f, 0.f, 0.f, 0.f};

  for (int c = 0; c < nchunk; ++c) {
    const int buf = c & 1;
    if (c + 1 < nchunk) load_chunk(c + 1);
    bf16x8 fa[WM], fb[WN];
#pragma unroll
    for (int x = 0; x < WM; ++x)
      fa[x] = *reinterpret_cast<const bf16x8*>(&As[buf][wm * 16 * WM + x * 16 + fr][8 * fg]);
#pragma unroll
    for (int y = 0; y < WN; ++y)
      fb[y] = *reinterpret_cast<const bf16x8*>(&Bs[buf][wj * 16 * WN + y * 16 + fr][8 * fg]);
#pragma unroll
    for (int x = 0; x < WM; ++x)
#pragma unroll
      for (int y = 0; y < WN; ++y) acc[x][y] = mfma_bf16(fa[x], fb[y], acc[x][y]);
    if (c + 1 < nchunk) store_chunk(buf ^ 1);
    __syncthreads();
  }

  // ---------------- epilogue (as conv_gemm_f32) ----------------
  float ssum[WN], ssq[WN], gap0[WN], gap1[WN];
#pragma unroll
  for (int y = 0; y < WN; ++y) ssum[y] = ssq[y] = gap0[y] = gap1[y] = 0.f;
  const int TV = g.T_out * g.V;
  const int nlo = m0 / TV;
#pragma unroll
  for (int y = 0; y < WN; ++y) {
    const int jl = wj * 16 * WN + y * 16 + fr;
    const int j = j0 + jl;
    const bool jok = j < g.Nc;
#pragma unroll
    for (int x = 0; x < WM; ++x) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = m0 + wm * 16 * WM + x * 16 + fg * 4 + r;
        if (!jok || m >= g.M) continue;
        float v = acc[x][y][r];
        if (EPI & EPI_BIAS) v += a.bias[j];
        if (EPI & EPI_BIASV) v += a.bias[(m % g.V) * g.Nc + j];
        if (EPI & EPI_RELUMASK) {
          const float gv = a.auxb ? bf2f(a.auxb[(size_t)m * a.ldaux + j]) : a.aux[(size_t)m * a.ldaux + j];
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
        if (!(EPI & EPI_ADD) && a.outb) {
          reinterpret_cast<__bf16*>(a.outb)[(size_t)m * g.ldo + j] = (__bf16)v;
        } else {
          float* o = a.out + (size_t)m * g.ldo + j;
          if (EPI & EPI_ADD) *o += v;
          else *o = v;
        }
      }
    }
  }
  if (EPI & (EPI_STATS | EPI_RELUMASK | EPI_GAP)) {
#pragma unroll
    for (int y = 0; y < WN; ++y) {
#pragma unroll
      for (int o = 16; o < 64; o <<= 1) {
        ssum[y] += __shfl_xor(ssum[y], o, 64);
        ssq[y] += __shfl_xor(ssq[y], o, 64);
        gap0[y] += __shfl_xor(gap0[y], o, 64);
        gap1[y] += __shfl_xor(gap1[y], o, 64);
      }
    }
    if (fg == 0) {
#pragma unroll
      for (int y = 0; y < WN; ++y) {
        const int jl = wj * 16 * WN + y * 16 + fr;
        red[wm][0][jl] = ssum[y];
        red[wm][1][jl] = ssq[y];
        gred[wm][0][jl] = gap0[y];
        gred[wm][1][jl] = gap1[y];
      }
    }
    __syncthreads();
    for (int t = tid; t < BN; t += 256) {
      const int j = j0 + t;
      if (j >= g.Nc) continue;
      if (EPI & (EPI_STATS | EPI_RELUMASK)) {
        atomic_add_d(a.st_sum + j, (double)(red[0][0][t] + red[1][0][t]));
        atomic_add_d(a.st_sq + j, (double)(red[0][1][t] + red[1][1][t]));
      }
      if (EPI & EPI_GAP) {
        const float s0 = gred[0][0][t] + gred[1][0][t];
        const float s1 = gred[0][1][t] + gred[1][1][t];
        atomic_add_f(a.gap + (size_t)nlo * g.Nc + j, s0);
        if ((nlo + 1) * TV < g.M && s1 != 0.f) atomic_add_f(a.gap + (size_t)(nlo + 1) * g.Nc + j, s1);
      }
    }
  }
}

// dW[j][i'] = sum_m dY[m][j] * pro(In[src(m,dt)][i]); split over rows, f32 atomics.
template <int PRO, int WM, int WN>
__global__ __launch_bounds__(256) void conv_wgrad_bf16(WgradArgs a) {
  constexpr int BJ = 32 * WM, BI = 32 * WN;
  constexpr int YLD = BJ + 8, XLD = BI + 8;  // 16-B pad: 2-way at worst for the tr reads
  constexpr int VPY = BJ / 8, VPX = BI / 8;  // values per thread per 32-row chunk (8 threads per row)
  __shared__ __attribute__((aligned(16))) __bf16 Ys[2][HBK][YLD];
  __shared__ __attribute__((aligned(16))) __bf16 Xs[2][HBK][XLD];
  __shared__ float pro_sc[256], pro_sh[256];
  const ConvGeom& g = a.g;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int j0 = blockIdx.x * BJ;
  const int itiles = (g.Kc + BI - 1) / BI;
  const int dt = blockIdx.y / itiles;
  const int i0 = (blockIdx.y - dt * itiles) * BI;
  const int r_begin = blockIdx.z * a.rows_per_split;
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
  const int lrow = tid >> 3;          // 0..31
  const int cy = (tid & 7) * VPY, cx = (tid & 7) * VPX;
  const bool fastY = (a.ldy % 4) == 0 && (g.Nc % 4) == 0;
  const bool fastX = (g.lda % 4) == 0 && (g.Kc % 4) == 0;
  const bool fastYb = (a.ldy % 8) == 0 && (g.Nc % 8) == 0;
  const bool fastXb = (g.lda % 8) == 0 && (g.Kc % 8) == 0;
  float ry[VPY], rx[VPX], dbp[VPY];
#pragma unroll
  for (int e = 0; e < VPY; ++e) dbp[e] = 0.f;
  const bool do_db = a.db && blockIdx.y == 0;
  auto load_chunk = [&](int r0) {
    const int m = r0 + lrow;
    const bool ok = m < r_end;
    const int j = j0 + cy;
    if (a.dyb) {  // bf16 dy
      const __bf16* yb = reinterpret_cast<const __bf16*>(a.dyb);
      if (ok && fastYb && j + VPY <= g.Nc) {
#pragma unroll
        for (int q = 0; q < VPY / 8; ++q) {
          const bf16x8 v = *reinterpret_cast<const bf16x8*>(yb + (size_t)m * a.ldy + j + 8 * q);
#pragma unroll
          for (int e = 0; e < 8; ++e) ry[8 * q + e] = (float)v[e];
        }
      } else {
#pragma unroll
        for (int e = 0; e < VPY; ++e) ry[e] = (ok && j + e < g.Nc) ? (float)yb[(size_t)m * a.ldy + j + e] : 0.f;
      }
    } else if (ok && fastY && j + VPY <= g.Nc) {
#pragma unroll
      for (int q = 0; q < VPY / 4; ++q) {
        const f32x4 v = *reinterpret_cast<const f32x4*>(a.dy + (size_t)m * a.ldy + j + 4 * q);
#pragma unroll
        for (int e = 0; e < 4; ++e) ry[4 * q + e] = v[e];
      }
    } else {
#pragma unroll
      for (int e = 0; e < VPY; ++e) ry[e] = (ok && j + e < g.Nc) ? a.dy[(size_t)m * a.ldy + j + e] : 0.f;
    }
    if (do_db) {
#pragma unroll
      for (int e = 0; e < VPY; ++e) dbp[e] += ry[e];
    }
    int r = -1;
    if (ok) {
      const int nt = m / g.V, v = m - nt * g.V, n = nt / g.T_out, t = nt - n * g.T_out;
      r = src_row_b(n, t, v, dt, g);
    }
    const int i = i0 + cx;
    if (a.inb) {  // bf16 input rows
      const __bf16* xb = reinterpret_cast<const __bf16*>(a.inb);
      if (r >= 0 && fastXb && i + VPX <= g.Kc) {
#pragma unroll
        for (int q = 0; q < VPX / 8; ++q) {
          const bf16x8 v = *reinterpret_cast<const bf16x8*>(xb + (size_t)r * g.lda + i + 8 * q);
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            float x = (float)v[e];
            if (PRO) x = fmaxf(x * pro_sc[i + 8 * q + e] + pro_sh[i + 8 * q + e], 0.f);
            rx[8 * q + e] = x;
          }
        }
      } else {
#pragma unroll
        for (int e = 0; e < VPX; ++e) {
          float x = 0.f;
          if (r >= 0 && i + e < g.Kc) {
            x = (float)xb[(size_t)r * g.lda + i + e];
            if (PRO) x = fmaxf(x * pro_sc[i + e] + pro_sh[i + e], 0.f);
          }
          rx[e] = x;
        }
      }
    } else if (r >= 0 && fastX && i + VPX <= g.Kc) {
#pragma unroll
      for (int q = 0; q < VPX / 4; ++q) {
        const f32x4 v = *reinterpret_cast<const f32x4*>(a.in + (size_t)r * g.lda + i + 4 * q);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          float x = v[e];
          if (PRO) x = fmaxf(x * pro_sc[i + 4 * q + e] + pro_sh[i + 4 * q + e], 0.f);
          rx[4 * q + e] = x;
        }
      }
    } else {
#pragma unroll
      for (int e = 0; e < VPX; ++e) {
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
    for (int q = 0; q < VPY / 8; ++q) {
      bf16x8 v;
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = (__bf16)ry[8 * q + e];
      *reinterpret_cast<bf16x8*>(&Ys[buf][lrow][cy + 8 * q]) = v;
    }
#pragma unroll
    for (int q = 0; q < VPX / 8; ++q) {
      bf16x8 v;
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = (__bf16)rx[8 * q + e];
      *reinterpret_cast<bf16x8*>(&Xs[buf][lrow][cx + 8 * q]) = v;
    }
  };
  const int wm = wave >> 1, wj = wave & 1;
  const int fr = lane & 15, fg = lane >> 4, tq = fr >> 2, tp = fr & 3;
  f32x4 acc[WM][WN];
#pragma unroll
  for (int x = 0; x < WM; ++x)
#pragma unroll
    for (int y = 0; y < WN; ++y) acc[x][y] = f32x4{0.f, 0.f, 0.f, 0.f};

  // transposed fragment: lane (fg, fr) gets column c0+fr of rows 8fg..8fg+7 of the tile
  auto tr_frag = [&](const __bf16* tile, int ld, int c0) {
    typedef __attribute__((address_space(3))) s16x4 lds_s16x4;
    const __bf16* p0 = tile + (8 * fg + tq) * ld + c0 + 4 * tp;
    const __bf16* p1 = p0 + 4 * ld;
    s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(p0));
    s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(p1));
    s16x8 v;
#pragma unroll
    for (int e = 0; e < 4; ++e) { v[e] = lo[e]; v[4 + e] = hi[e]; }
    return __builtin_bit_cast(bf16x8, v);
  };

  if (r_begin < r_end) {
    load_chunk(r_begin);
    store_chunk(0);
    __syncthreads();
    int buf = 0;
    for (int r0 = r_begin; r0 < r_end; r0 += HBK) {
      const bool more = r0 + HBK < r_end;
      if (more) load_chunk(r0 + HBK);
      bf16x8 fa[WM], fb[WN];
#pragma unroll
      for (int x = 0; x < WM; ++x) fa[x] = tr_frag(&Ys[buf][0][0], YLD, wm * 16 * WM + x * 16);
#pragma unroll
      for (int y = 0; y < WN; ++y) fb[y] = tr_frag(&Xs[buf][0][0], XLD, wj * 16 * WN + y * 16);
#pragma unroll
      for (int x = 0; x < WM; ++x)
#pragma unroll
        for (int y = 0; y < WN; ++y) acc[x][y] = mfma_bf16(fa[x], fb[y], acc[x][y]);
      if (more) store_chunk(buf ^ 1);
      __syncthreads();
      buf ^= 1;
    }
  }
  if (do_db && r_begin < r_end) {
    // reduce the per-thread column partials over the 32 row-threads sharing columns
#pragma unroll
    for (int e = 0; e < VPY; ++e) {
      float v = dbp[e];
      v += __shfl_xor(v, 8, 64);
      v += __shfl_xor(v, 16, 64);
      v += __shfl_xor(v, 32, 64);
      dbp[e] = v;
    }
    __shared__ float dbs[4][BJ];
    if ((lane >> 3) == 0) {
#pragma unroll
      for (int e = 0; e < VPY; ++e) dbs[wave][cy + e] = dbp[e];
    }
    __syncthreads();
    for (int t = tid; t < BJ; t += 256) {
      if (j0 + t < g.Nc) atomic_add_f(a.db + j0 + t, dbs[0][t] + dbs[1][t] + dbs[2][t] + dbs[3][t]);
    }
  }
#pragma unroll
  for (int x = 0; x < WM; ++x) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int j = j0 + wm * 16 * WM + x * 16 + fg * 4 + r;
      if (j >= g.Nc) continue;
#pragma unroll
      for (int y = 0; y < WN; ++y) {
        const int i = i0 + wj * 16 * WN + y * 16 + fr;
        if (i >= g.Kc) continue;
        size_t idx;
        if (a.outmap == WG_OUT_CONV) {
          idx = ((size_t)j * g.Kc + i) * g.KT + dt;
        } else {
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

template <int WM, int WN>
static int launch_gemm_bf16(const ConvGemmArgs& a, int pro, int epi, hipStream_t s) {
  dim3 grid((a.g.M + 32 * WM - 1) / (32 * WM), (a.g.Nc + 32 * WN - 1) / (32 * WN));
#define F3_BCASE(P, E)                                                                   \
  if (pro == P && epi == (E)) {                                                         \
    hipLaunchKernelGGL((conv_gemm_bf16<P, (E), WM, WN>), grid, dim3(256), 0, s, a);     \
    F3_LAUNCH_CHECK();                                                                   \
    return F3_OK;                                                                        \
  }
  F3_BCASE(0, EPI_BIASV | EPI_STATS)
  F3_BCASE(1, EPI_BIAS | EPI_STATS | EPI_GAP)
  F3_BCASE(0, EPI_BIAS | EPI_STATS)
  F3_BCASE(0, EPI_RELUMASK)
  F3_BCASE(0, 0)
  F3_BCASE(0, EPI_ADD)
  F3_BCASE(0, EPI_BIAS)
#undef F3_BCASE
  return F3_EINVAL;
}

int f3_conv_gemm_bf16(const ConvGemmArgs* args, int pro, int epi, hipStream_t s) {
  const ConvGemmArgs& a = *args;
  if (a.g.M <= 0 || a.g.Nc <= 0) return F3_OK;
  if (a.inb && !pro && f3_igemm_ok(a)) return f3_igemm_bf16(args, epi, s);
  if (a.x3n) return F3_EINVAL;  // (the bf16x3 operand forms exist on the LDS-DMA kernels only)
  if (pro && a.g.Kc > 256) return F3_EINVAL;
  if (!a.wb) return F3_EINVAL;
  // wide output channels: 128x128 tiles; narrow (64 / small gcn dgrad): 128x64
  if (a.g.Nc >= 128 && a.g.M >= 4096) return launch_gemm_bf16<4, 4>(a, pro, epi, s);
  return launch_gemm_bf16<4, 2>(a, pro, epi, s);
}

int f3_conv_wgrad_bf16(const WgradArgs* args, int pro, hipStream_t s) {
  WgradArgs a = *args;
  if (a.g.M <= 0) return F3_OK;
  if (pro && a.g.Kc > 256) return F3_EINVAL;
  const bool big = a.g.Nc >= 128 && a.g.Kc >= 128;
  const int BJ = big ? 128 : 64, BI = big ? 128 : 64;
  const int gx = (a.g.Nc + BJ - 1) / BJ;
  const int gy = a.g.KT * ((a.g.Kc + BI - 1) / BI);
  int splits = (f3_wgrad_target_wgs() + gx * gy - 1) / (gx * gy);
  int rps = (a.g.M + splits - 1) / splits;
  rps = ((rps + HBK - 1) / HBK) * HBK;
  if (rps < 4 * HBK) rps = 4 * HBK;
  splits = (a.g.M + rps - 1) / rps;
  a.rows_per_split = rps;
  dim3 grid(gx, gy, splits);
  if (big) {
    if (pro) hipLaunchKernelGGL((conv_wgrad_bf16<1, 4, 4>), grid, dim3(256), 0, s, a);
    else hipLaunchKernelGGL((conv_wgrad_bf16<0, 4, 4>), grid, dim3(256), 0, s, a);
  } else {
    if (pro) hipLaunchKernelGGL((conv_wgrad_bf16<1, 2, 2>), grid, dim3(256), 0, s, a);
    else hipLaunchKernelGGL((conv_wgrad_bf16<0, 2, 2>), grid, dim3(256), 0, s, a);
  }
  F3_LAUNCH_CHECK();
  return F3_OK;
}
