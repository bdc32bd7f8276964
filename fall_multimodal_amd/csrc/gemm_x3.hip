// Split-bf16 ("bf16x3") MFMA forms of the implicit-GEMM temporal convolution and its weight
// gradient: the parity mode of the step at bf16 matrix-core rates (F3_PRECISION_BF16X3).
//
// The reference computes this path in fp32 (Multimodal_Fall3/model/main.py:111 autocast fp32).
// gfx950 has exact fp32 MFMA only at 1/16 of the bf16 rate and no xf32, so every fp32 operand x is
// split into hi = RNE bf16(x) and lo = RNE bf16(x - hi) (x - hi is exact in fp32), and a product
// a*b is accumulated as lo_a*hi_b + hi_a*lo_b + hi_a*hi_b on v_mfma_f32_16x16x32_bf16 into one
// fp32 accumulator. |x - hi - lo| <= 2^-16 |x| and the dropped lo_a*lo_b <= 2^-16 |ab|, so each
// product carries ~2^-16 relative error against fp32's 2^-24: the logits stay within the north
// star's 1e-3 (tests/test_gpu_parity.py) while the MFMA work is 3/16 of the fp32 MFMA's.
//
// Activations stay fp32 in HBM (the same buffers and elementwise kernels as the fp32 mode). The
// activation operand is split while it is staged (register staging: global fp32 -> optional
// BN+ReLU prologue -> hi/lo -> LDS); the weight operand comes pre-split from the prep kernel as
// two bf16 planes (hi at wb, lo at wb + Nc*Ktot), so its staging is a plain copy.
//
//   conv_gemm_x3 : Out[m][j] = sum_{dt,i} pro(In[src(m,dt)][i]) W[j][dt*Kc+i]   (fwd / dgrad)
//     LDS rows of 128 B per tile row: 32 k of hi then 32 k of lo, 16-B chunks XOR-swizzled by
//     (row >> 1) & 7 so the 16-lane ds_read_b128 fragment reads are conflict-free.
//   conv_wgrad_x3: dW[j][i'] = sum_m dY[m][j] pro(In[src(m,dt)][i])
//     the reduction index is the memory row, so both tiles are staged row-major [32 m][cols]
//     (hi and lo planes) and read with ds_read_b64_tr_b16; split over rows, f32 atomics.
#include "common.h"
#include "kernels.h"

namespace f3 {

namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef short s16x4 __attribute__((ext_vector_type(4)));

constexpr int XBK = 32;  // k (or m) per chunk

F3_DEV f32x4 mfma_x(bf16x8 a, bf16x8 b, f32x4 c) { return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0); }

F3_DEV void split8(const float* x, bf16x8& hi, bf16x8& lo) {
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const __bf16 h = (__bf16)x[e];
    hi[e] = h;
    lo[e] = (__bf16)(x[e] - (float)h);
  }
}

F3_DEV int src_row_x(int n, int t, int v, int dt, const ConvGeom& g) {
  int ti;
  if (!g.transposed) {
    ti = t * g.S + dt - g.P;
    if (ti < 0 || ti >= g.T_in) return -1;
  } else {
    const int num = t + g.P - dt;
    if (num < 0 || (num % g.S) != 0) return -1;
    ti = num / g.S;
    if (ti >= g.T_in) return -1;
  }
  return (n * g.T_in + ti) * g.V + v;
}

// element offset (bf16 units) of 16-B chunk c (0-3 hi, 4-7 lo) of tile row r
F3_DEV int xoff(int r, int c) { return r * 64 + ((c ^ ((r >> 1) & 7)) << 3); }

// transposed LDS read (gfx950): 4 rows x 16 columns per 16-lane group, column i to lane i. Inline
// asm: the builtin carries no memory operand, and hipcc then waits vmcnt(0) (the register-staged
// prefetch of the next chunk) before it. Results are used only after x3_tr_wait.
typedef __attribute__((address_space(3))) const char lds_cchar;
F3_DEV s16x4 tr_read(const __bf16* p) {
  s16x4 r;
  const unsigned addr = (unsigned)(size_t)(lds_cchar*)p;
  asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(r) : "v"(addr));
  return r;
}

}  // namespace

// rows of the input tensor of a conv geometry (N * T_in * V); the lo plane of a pre-split operand
// starts this many rows (x lda) after the hi plane
F3_DEV size_t in_rows(const ConvGeom& g) { return (size_t)(g.M / (g.T_out * g.V)) * g.T_in * g.V; }

// AS: the activation operand arrives pre-split (a.inb = hi plane, lo plane in_rows * lda later;
// e.g. u = relu(bn1(g)) split once by bnrelu_x3 instead of once per tap here); no prologue
template <int PRO, int EPI, int WM, int WN, bool AS>
__global__ __launch_bounds__(256) void conv_gemm_x3(ConvGemmArgs a) {
  constexpr int BM = 32 * WM, BN = 32 * WN;
  constexpr int AIT = BM * 4 / 256;  // (row, k octet) items of the A tile per thread
  constexpr int BIT = BN * 4 / 256;
  __shared__ __attribute__((aligned(16))) __bf16 As[2][BM * 64];
  __shared__ __attribute__((aligned(16))) __bf16 Bs[2][BN * 64];
  __shared__ float pro_sc[256], pro_sh[256];
  __shared__ float epi_sc[BN], epi_sh[BN], epi_mu[BN], epi_rs[BN];
  __shared__ float red[2][2][BN], gred[2][2][BN];

  const ConvGeom& g = a.g;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int m0 = blockIdx.x * BM, j0 = blockIdx.y * BN;
  const int Ktot = g.KT * g.Kc;
  const int nchunk = (Ktot + XBK - 1) / XBK;
  const bool fastA = (g.Kc % 8) == 0 && (g.lda % 4) == 0;
  const bool fastB = (Ktot % 8) == 0;
  const unsigned short* wh = a.wb;
  const unsigned short* wl = a.wb + (size_t)g.Nc * Ktot;

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
  // per A item: tile row, k octet, row geometry
  int arow[AIT], aoct[AIT], an[AIT], at[AIT], av[AIT];
  bool aok[AIT];
#pragma unroll
  for (int q = 0; q < AIT; ++q) {
    const int idx = tid + 256 * q;
    arow[q] = idx >> 2;
    aoct[q] = idx & 3;
    const int am = m0 + arow[q];
    aok[q] = am < g.M;
    an[q] = at[q] = av[q] = 0;
    if (aok[q]) {
      const int nt = am / g.V;
      av[q] = am - nt * g.V;
      an[q] = nt / g.T_out;
      at[q] = nt - an[q] * g.T_out;
    }
  }
  float ra[AIT][8];
  uint4 rah[AIT], ral[AIT];
  uint4 rbh[BIT], rbl[BIT];
  const unsigned short* ah_plane = a.inb;
  const unsigned short* al_plane = AS ? a.inb + in_rows(g) * g.lda : nullptr;
  auto load_chunk = [&](int c) {
#pragma unroll
    for (int q = 0; q < AIT; ++q) {
      const int k0 = c * XBK + aoct[q] * 8;
      if constexpr (AS) {  // launcher guarantees Kc % 8 == 0 and lda % 8 == 0
        const int dt = k0 / g.Kc, i = k0 - dt * g.Kc;
        const int r = (aok[q] && k0 < Ktot) ? src_row_x(an[q], at[q], av[q], dt, g) : -1;
        const size_t o = (size_t)max(r, 0) * g.lda + i;
        const uint4 h = *reinterpret_cast<const uint4*>(ah_plane + o), l = *reinterpret_cast<const uint4*>(al_plane + o);
        const uint4 z = {0u, 0u, 0u, 0u};
        rah[q] = r >= 0 ? h : z;
        ral[q] = r >= 0 ? l : z;
      } else if (fastA) {
        const int dt = k0 / g.Kc, i = k0 - dt * g.Kc;
        const int r = (aok[q] && k0 < Ktot) ? src_row_x(an[q], at[q], av[q], dt, g) : -1;
        if (r >= 0) {
          const f32x4* p = reinterpret_cast<const f32x4*>(a.in + (size_t)r * g.lda + i);
          const f32x4 v0 = p[0], v1 = p[1];
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            ra[q][e] = v0[e];
            ra[q][4 + e] = v1[e];
          }
          if (PRO) {
#pragma unroll
            for (int e = 0; e < 8; ++e) ra[q][e] = fmaxf(ra[q][e] * pro_sc[i + e] + pro_sh[i + e], 0.f);
          }
        } else {
#pragma unroll
          for (int e = 0; e < 8; ++e) ra[q][e] = 0.f;
        }
      } else {
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const int k = k0 + e;
          float x = 0.f;
          if (aok[q] && k < Ktot) {
            const int dt = k / g.Kc, i = k - dt * g.Kc;
            const int r = src_row_x(an[q], at[q], av[q], dt, g);
            if (r >= 0) {
              x = a.in[(size_t)r * g.lda + i];
              if (PRO) x = fmaxf(x * pro_sc[i] + pro_sh[i], 0.f);
            }
          }
          ra[q][e] = x;
        }
      }
    }
#pragma unroll
    for (int q = 0; q < BIT; ++q) {
      const int idx = tid + 256 * q, brow = idx >> 2, boct = idx & 3;
      const int bj = j0 + brow, kb = c * XBK + boct * 8;
      if (bj < g.Nc && fastB && kb + 8 <= Ktot) {
        rbh[q] = *reinterpret_cast<const uint4*>(wh + (size_t)bj * Ktot + kb);
        rbl[q] = *reinterpret_cast<const uint4*>(wl + (size_t)bj * Ktot + kb);
      } else {
        unsigned short h[8], l[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const int k = kb + e;
          const bool ok = bj < g.Nc && k < Ktot;
          h[e] = ok ? wh[(size_t)bj * Ktot + k] : (unsigned short)0;
          l[e] = ok ? wl[(size_t)bj * Ktot + k] : (unsigned short)0;
        }
        rbh[q] = *reinterpret_cast<const uint4*>(h);
        rbl[q] = *reinterpret_cast<const uint4*>(l);
      }
    }
  };
  auto store_chunk = [&](int buf) {
#pragma unroll
    for (int q = 0; q < AIT; ++q) {
      if constexpr (AS) {
        *reinterpret_cast<uint4*>(&As[buf][xoff(arow[q], aoct[q])]) = rah[q];
        *reinterpret_cast<uint4*>(&As[buf][xoff(arow[q], 4 + aoct[q])]) = ral[q];
      } else {
        bf16x8 hi, lo;
        split8(ra[q], hi, lo);
        *reinterpret_cast<bf16x8*>(&As[buf][xoff(arow[q], aoct[q])]) = hi;
        *reinterpret_cast<bf16x8*>(&As[buf][xoff(arow[q], 4 + aoct[q])]) = lo;
      }
    }
#pragma unroll
    for (int q = 0; q < BIT; ++q) {
      const int idx = tid + 256 * q, brow = idx >> 2, boct = idx & 3;
      *reinterpret_cast<uint4*>(&Bs[buf][xoff(brow, boct)]) = rbh[q];
      *reinterpret_cast<uint4*>(&Bs[buf][xoff(brow, 4 + boct)]) = rbl[q];
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
    bf16x8 ah[WM], al[WM], bh[WN], bl[WN];
#pragma unroll
    for (int x = 0; x < WM; ++x) {
      const int r = wm * 16 * WM + x * 16 + fr;
      ah[x] = *reinterpret_cast<const bf16x8*>(&As[buf][xoff(r, fg)]);
      al[x] = *reinterpret_cast<const bf16x8*>(&As[buf][xoff(r, 4 + fg)]);
    }
#pragma unroll
    for (int y = 0; y < WN; ++y) {
      const int r = wj * 16 * WN + y * 16 + fr;
      bh[y] = *reinterpret_cast<const bf16x8*>(&Bs[buf][xoff(r, fg)]);
      bl[y] = *reinterpret_cast<const bf16x8*>(&Bs[buf][xoff(r, 4 + fg)]);
    }
    // the three products as three passes over the tile: consecutive MFMAs never share an accumulator
#pragma unroll
    for (int x = 0; x < WM; ++x)
#pragma unroll
      for (int y = 0; y < WN; ++y) acc[x][y] = mfma_x(al[x], bh[y], acc[x][y]);
#pragma unroll
    for (int x = 0; x < WM; ++x)
#pragma unroll
      for (int y = 0; y < WN; ++y) acc[x][y] = mfma_x(ah[x], bl[y], acc[x][y]);
#pragma unroll
    for (int x = 0; x < WM; ++x)
#pragma unroll
      for (int y = 0; y < WN; ++y) acc[x][y] = mfma_x(ah[x], bh[y], acc[x][y]);
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
// XS: the input rows arrive pre-split (a.inb hi plane, lo plane in_rows * lda later); no prologue
// YS: dY arrives pre-split (a.dyb hi plane, lo plane M * ldy later)
template <int PRO, int WM, int WN, bool XS, bool YS>
__global__ __launch_bounds__(256) void conv_wgrad_x3(WgradArgs a_) {
  WgradArgs a = a_;
  const int nsplit = (a.g.M + a.rows_per_split - 1) / a.rows_per_split;
  const int zsplit = blockIdx.z % nsplit;
  wgrad_group(a, blockIdx.z / nsplit);
  constexpr int BJ = 32 * WM, BI = 32 * WN;
  constexpr int YLD = BJ + 8, XLD = BI + 8;  // 16-B pad: 2-way at worst for the tr reads
  constexpr int VPY = BJ / 8, VPX = BI / 8;  // values per thread per 32-row chunk (8 threads per row)
  __shared__ __attribute__((aligned(16))) __bf16 Ys[2][2][XBK * YLD];  // [buf][hi, lo]
  __shared__ __attribute__((aligned(16))) __bf16 Xs[2][2][XBK * XLD];
  __shared__ float pro_sc[256], pro_sh[256];
  const ConvGeom& g = a.g;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int j0 = blockIdx.x * BJ;
  const int itiles = (g.Kc + BI - 1) / BI;
  const int dt = blockIdx.y / itiles;
  const int i0 = (blockIdx.y - dt * itiles) * BI;
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
  const int lrow = tid >> 3;  // 0..31
  const int cy = (tid & 7) * VPY, cx = (tid & 7) * VPX;
  const bool fastY = (a.ldy % 4) == 0 && (g.Nc % 4) == 0;
  const bool fastX = (g.lda % 4) == 0 && (g.Kc % 4) == 0;
  float ry[VPY], rx[VPX], dbp[VPY];
  uint4 rxh[VPX / 8], rxl[VPX / 8], ryh[VPY / 8], ryl[VPY / 8];
  const unsigned short* yh_plane = a.dyb;
  const unsigned short* yl_plane = YS ? a.dyb + (size_t)g.M * a.ldy : nullptr;
  const unsigned short* xh_plane = a.inb;
  const unsigned short* xl_plane = XS ? a.inb + in_rows(g) * g.lda : nullptr;
#pragma unroll
  for (int e = 0; e < VPY; ++e) dbp[e] = 0.f;
  const bool do_db = a.db && blockIdx.y == 0;
  auto load_chunk = [&](int r0) {
    const int m = r0 + lrow;
    const bool ok = m < r_end;
    const int j = j0 + cy;
    if constexpr (YS) {  // launcher guarantees Nc % BJ == 0 and ldy % 8 == 0
      const size_t o = (size_t)(ok ? m : r_begin) * a.ldy + j;
      const uint4 z = {0u, 0u, 0u, 0u};
#pragma unroll
      for (int q = 0; q < VPY / 8; ++q) {
        const uint4 h = *reinterpret_cast<const uint4*>(yh_plane + o + 8 * q);
        const uint4 l = *reinterpret_cast<const uint4*>(yl_plane + o + 8 * q);
        ryh[q] = ok ? h : z;
        ryl[q] = ok ? l : z;
        if (do_db) {  // the bias gradient from hi + lo in fp32
          const bf16x8 hv = __builtin_bit_cast(bf16x8, ryh[q]), lv = __builtin_bit_cast(bf16x8, ryl[q]);
#pragma unroll
          for (int e = 0; e < 8; ++e) ry[8 * q + e] = (float)hv[e] + (float)lv[e];
        }
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
      r = src_row_x(n, t, v, dt, g);
    }
    const int i = i0 + cx;
    if constexpr (XS) {  // launcher guarantees Kc % BI == 0 and lda % 8 == 0
      const size_t o = (size_t)max(r, 0) * g.lda + i;
      const uint4 z = {0u, 0u, 0u, 0u};
#pragma unroll
      for (int q = 0; q < VPX / 8; ++q) {
        const uint4 h = *reinterpret_cast<const uint4*>(xh_plane + o + 8 * q);
        const uint4 l = *reinterpret_cast<const uint4*>(xl_plane + o + 8 * q);
        rxh[q] = r >= 0 ? h : z;
        rxl[q] = r >= 0 ? l : z;
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
      if constexpr (YS) {
        *reinterpret_cast<uint4*>(&Ys[buf][0][lrow * YLD + cy + 8 * q]) = ryh[q];
        *reinterpret_cast<uint4*>(&Ys[buf][1][lrow * YLD + cy + 8 * q]) = ryl[q];
      } else {
        bf16x8 hi, lo;
        split8(&ry[8 * q], hi, lo);
        *reinterpret_cast<bf16x8*>(&Ys[buf][0][lrow * YLD + cy + 8 * q]) = hi;
        *reinterpret_cast<bf16x8*>(&Ys[buf][1][lrow * YLD + cy + 8 * q]) = lo;
      }
    }
#pragma unroll
    for (int q = 0; q < VPX / 8; ++q) {
      if constexpr (XS) {
        *reinterpret_cast<uint4*>(&Xs[buf][0][lrow * XLD + cx + 8 * q]) = rxh[q];
        *reinterpret_cast<uint4*>(&Xs[buf][1][lrow * XLD + cx + 8 * q]) = rxl[q];
      } else {
        bf16x8 hi, lo;
        split8(&rx[8 * q], hi, lo);
        *reinterpret_cast<bf16x8*>(&Xs[buf][0][lrow * XLD + cx + 8 * q]) = hi;
        *reinterpret_cast<bf16x8*>(&Xs[buf][1][lrow * XLD + cx + 8 * q]) = lo;
      }
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
  constexpr int NF = 2 * (WM + WN);  // (hi, lo) of every A and B fragment
  auto issue = [&](const __bf16* tile, int ld, int c0, s16x4& lo4, s16x4& hi4) {
    const __bf16* p0 = tile + (8 * fg + tq) * ld + c0 + 4 * tp;
    lo4 = tr_read(p0);
    hi4 = tr_read(p0 + 4 * ld);
  };

  if (r_begin < r_end) {
    load_chunk(r_begin);
    store_chunk(0);
    __syncthreads();
    int buf = 0;
    for (int r0 = r_begin; r0 < r_end; r0 += XBK) {
      const bool more = r0 + XBK < r_end;
      if (more) load_chunk(r0 + XBK);
      s16x4 lo4[NF], hi4[NF];
#pragma unroll
      for (int x = 0; x < WM; ++x) {
        issue(&Ys[buf][0][0], YLD, wm * 16 * WM + x * 16, lo4[2 * x], hi4[2 * x]);
        issue(&Ys[buf][1][0], YLD, wm * 16 * WM + x * 16, lo4[2 * x + 1], hi4[2 * x + 1]);
      }
#pragma unroll
      for (int y = 0; y < WN; ++y) {
        issue(&Xs[buf][0][0], XLD, wj * 16 * WN + y * 16, lo4[2 * WM + 2 * y], hi4[2 * WM + 2 * y]);
        issue(&Xs[buf][1][0], XLD, wj * 16 * WN + y * 16, lo4[2 * WM + 2 * y + 1], hi4[2 * WM + 2 * y + 1]);
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      bf16x8 f[NF];
#pragma unroll
      for (int k = 0; k < NF; ++k) {
        asm volatile("" : "+v"(lo4[k]), "+v"(hi4[k]));  // nothing reads them before the wait
        f[k] = __builtin_bit_cast(bf16x8, __builtin_shufflevector(lo4[k], hi4[k], 0, 1, 2, 3, 4, 5, 6, 7));
      }
#pragma unroll
      for (int p = 0; p < 3; ++p)  // lo*hi, hi*lo, hi*hi passes (no back-to-back accumulator reuse)
#pragma unroll
        for (int x = 0; x < WM; ++x)
#pragma unroll
          for (int y = 0; y < WN; ++y)
            acc[x][y] = mfma_x(f[2 * x + (p == 0)], f[2 * WM + 2 * y + (p == 1)], acc[x][y]);
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

template <int WM, int WN, bool AS>
static int launch_gemm_x3(const ConvGemmArgs& a, int pro, int epi, hipStream_t s) {
  dim3 grid((a.g.M + 32 * WM - 1) / (32 * WM), (a.g.Nc + 32 * WN - 1) / (32 * WN));
#define F3_XCASE(P, E)                                                                 \
  if (pro == P && epi == (E)) {                                                       \
    hipLaunchKernelGGL((conv_gemm_x3<P, (E), WM, WN, AS>), grid, dim3(256), 0, s, a); \
    F3_LAUNCH_CHECK();                                                                 \
    return F3_OK;                                                                      \
  }
  F3_XCASE(0, EPI_BIASV | EPI_STATS)           // gcn forward
  F3_XCASE(1, EPI_BIAS | EPI_STATS | EPI_GAP)  // tcn forward, BN1 + ReLU in the staging
  F3_XCASE(0, EPI_BIAS | EPI_STATS | EPI_GAP)  // tcn forward on the pre-split u
  F3_XCASE(0, EPI_BIAS | EPI_STATS)            // residual forward
  F3_XCASE(0, EPI_RELUMASK)                    // tcn dgrad (+BN1 bwd sums)
  F3_XCASE(0, 0)                               // gcn dgrad
  F3_XCASE(0, EPI_ADD)                         // residual dgrad
  F3_XCASE(0, EPI_BIAS)                        // plain conv (tests)
  F3_XCASE(1, 0)                               // tests
#undef F3_XCASE
  return F3_EINVAL;
}

int f3_conv_gemm_x3(const ConvGemmArgs* args, int pro, int epi, hipStream_t s) {
  const ConvGemmArgs& a = *args;
  if (a.g.M <= 0 || a.g.Nc <= 0) return F3_OK;
  // fp32 activations (in) or pre-split bf16 planes (inb: no prologue, Kc and lda multiples of 8);
  // split weight planes; fp32 output
  if (!a.wb || a.outb || (a.in != nullptr) == (a.inb != nullptr)) return F3_EINVAL;
  if (a.inb && (pro || a.g.Kc % 8 || a.g.lda % 8)) return F3_EINVAL;
  if (pro && a.g.Kc > 256) return F3_EINVAL;
  const bool wide = a.g.Nc >= 128 && a.g.M >= 4096;
  if (a.inb) return wide ? launch_gemm_x3<4, 4, true>(a, pro, epi, s) : launch_gemm_x3<4, 2, true>(a, pro, epi, s);
  return wide ? launch_gemm_x3<4, 4, false>(a, pro, epi, s) : launch_gemm_x3<4, 2, false>(a, pro, epi, s);
}

int f3_conv_wgrad_x3(const WgradArgs* args, int pro, hipStream_t s) {
  WgradArgs a = *args;
  if (a.g.M <= 0) return F3_OK;
  if (a.slab || (a.dy != nullptr) == (a.dyb != nullptr) || (a.in != nullptr) == (a.inb != nullptr)) return F3_EINVAL;
  if (pro && a.g.Kc > 256) return F3_EINVAL;
  const bool big = a.g.Nc >= 128 && a.g.Kc >= 128;
  const bool xs = a.inb != nullptr, ys = a.dyb != nullptr;
  if (xs && (pro || a.g.Kc % (big ? 128 : 64) || a.g.lda % 8)) return F3_EINVAL;
  if (ys && (a.g.Nc % (big ? 128 : 64) || a.ldy % 8 || (pro && !xs))) return F3_EINVAL;
  const int BJ = big ? 128 : 64, BI = big ? 128 : 64;
  const int gx = (a.g.Nc + BJ - 1) / BJ;
  const int gy = a.g.KT * ((a.g.Kc + BI - 1) / BI);
  int splits = (f3_wgrad_target_wgs() + gx * gy - 1) / (gx * gy);
  int rps = (a.g.M + splits - 1) / splits;
  rps = ((rps + XBK - 1) / XBK) * XBK;
  if (rps < 4 * XBK) rps = 4 * XBK;
  splits = (a.g.M + rps - 1) / rps;
  a.rows_per_split = rps;
  dim3 grid(gx, gy, splits * std::max(1, a.groups));
#define F3_XW(WM_, WN_)                                                                                      \
  if (xs && ys) hipLaunchKernelGGL((conv_wgrad_x3<0, WM_, WN_, true, true>), grid, dim3(256), 0, s, a);       \
  else if (xs) hipLaunchKernelGGL((conv_wgrad_x3<0, WM_, WN_, true, false>), grid, dim3(256), 0, s, a);       \
  else if (ys) hipLaunchKernelGGL((conv_wgrad_x3<0, WM_, WN_, false, true>), grid, dim3(256), 0, s, a);       \
  else if (pro) hipLaunchKernelGGL((conv_wgrad_x3<1, WM_, WN_, false, false>), grid, dim3(256), 0, s, a);     \
  else hipLaunchKernelGGL((conv_wgrad_x3<0, WM_, WN_, false, false>), grid, dim3(256), 0, s, a);
  if (big) {
    F3_XW(4, 4)
  } else {
    F3_XW(2, 2)
  }
#undef F3_XW
  F3_LAUNCH_CHECK();
  return F3_OK;
}
