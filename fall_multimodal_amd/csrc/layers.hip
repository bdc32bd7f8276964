// Per-layer byte-moving kernels of the st_gcan block and the skeleton stream ends:
// data_bn, graph mix (A_eff einsum), BatchNorm apply / backward, channel attention,
// residual + ReLU, average pool, weight packing and running-stat updates.
//
// Activations are channels-last rows [N][T][V][C] (row m = (n*T+t)*V + v). Elementwise
// kernels give each workgroup a chunk of ONE clip's rows, so per-(clip, channel)
// reductions (the channel-attention pool, its backward) finish in LDS and cost one
// atomic per channel per workgroup.
#include "common.h"
#include "layers.h"

#include <algorithm>
#include <cstring>
#include <type_traits>

namespace f3 {

typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

// ----------------------------------------------------------------------------
// prep: A_eff = A * E, gcn bias through the graph, weight packing  (one launch)
// ----------------------------------------------------------------------------
// bf16x3 native form (prep code 4, ConvGemmArgs::x3n): per tap, 32-channel blocks [W_hi (32) | W_lo (32)]
// (dst [rows][KT][2 inner], channel c of a tap at (c / 32) * 64 + c % 32, its lo 32 further on); the
// activation rows are [x_hi | x_lo] and the GEMM issues x_hi W_hi + x_lo W_hi + x_hi W_lo per block.
// inner % 32 == 0. j.n counts the dst elements (2 per source value).
F3_DEV void prep_x3n(const PrepJob& j, int e) {
  const bool gcn = j.type == PREP_PACK_GCN || j.type == PREP_PACK_GCN_T;
  const bool tr = j.type == PREP_PACK_CONV_T || j.type == PREP_PACK_GCN_T;
  const int J = j.d0, I = j.d1, KT = gcn ? 1 : j.d2;
  const int inner = gcn ? (tr ? J : j.d2 * I) : (tr ? J : I);
  const int row = e / (KT * inner), r = e - row * KT * inner, dt = r / inner, c = r - dt * inner;
  float val;
  if (gcn) {
    const int kc = tr ? row : c, cc = tr ? c : row, k = kc / I, ci = kc - k * I;
    val = j.s0[((size_t)k * J + cc) * I + ci];
  } else {
    val = tr ? j.s0[((size_t)c * I + row) * KT + dt] : j.s0[((size_t)row * I + c) * KT + dt];
  }
  const __bf16 hi = (__bf16)val;
  __bf16* d = reinterpret_cast<__bf16*>(j.dst) + ((size_t)row * KT + dt) * 2 * inner + (c >> 5) * 64 + (c & 31);
  d[0] = hi;
  d[32] = (__bf16)(val - (float)hi);
}

// The job table plus each job's first block: a 1-D grid whose blocks are shared out in proportion
// to the jobs' sizes (a fixed 64 blocks per job left the 256-channel packs to a few blocks looping
// ~100 times while the small jobs' blocks idled: 83 us per launch in the bf16x3 step)
struct PrepLaunch {
  PrepTable t;
  int boff[kMaxPrepJobs + 1];
};
static_assert(sizeof(PrepLaunch) <= 4096, "kernel argument block");

constexpr int kPrepVMax = 25;  // PREP_GCN_BIAS: joints whose column loads go out together
__global__ void prep_kernel(PrepLaunch L) {
  int jb = 0;
  while (jb + 1 < L.t.n && (int)blockIdx.x >= L.boff[jb + 1]) ++jb;
  const PrepJob j = L.t.jobs[jb];
  const int nb = L.boff[jb + 1] - L.boff[jb], lb = blockIdx.x - L.boff[jb];
  const int stride = nb * blockDim.x;
  if (j.bf16 == 4) {
    for (int e = lb * blockDim.x + threadIdx.x; e < j.n / 2; e += stride) prep_x3n(j, e);
    return;
  }
  for (int e = lb * blockDim.x + threadIdx.x; e < j.n; e += stride) {
    float val = 0.f;
    switch (j.type) {
      case PREP_MUL:
        val = j.s0[e] * j.s1[e];
        break;
      case PREP_COPY:
        val = j.s0[e];
        break;
      case PREP_PACK_CONV: {  // src [J][I][KT] -> dst [J][KT*I] (k = dt*I + i)
        const int I = j.d1, KT = j.d2;
        const int jj = e / (KT * I), r = e - jj * KT * I, dt = r / I, i = r - dt * I;
        val = j.s0[((size_t)jj * I + i) * KT + dt];
        break;
      }
      case PREP_UNPACK_CONV: {  // packed weight gradient [J][KT*I] -> reference layout [J][I][KT]
        const int I = j.d1, KT = j.d2;
        const int jj = e / (I * KT), r = e - jj * I * KT, i = r / KT, dt = r - i * KT;
        val = j.s0[(size_t)jj * KT * I + (size_t)dt * I + i];
        break;
      }
      case PREP_PACK_CONV_T: {  // dgrad operand: dst [I][KT*J] (k = dt*J + j)
        const int J = j.d0, I = j.d1, KT = j.d2;
        const int i = e / (KT * J), r = e - i * KT * J, dt = r / J, jj = r - dt * J;
        val = j.s0[((size_t)jj * I + i) * KT + dt];
        break;
      }
      case PREP_PACK_GCN: {  // W[k*C+c][ci] -> dst [C][K*Cin] (k-major then ci)
        const int C = j.d0, Cin = j.d1, K = j.d2;
        const int c = e / (K * Cin), r = e - c * K * Cin, k = r / Cin, ci = r - k * Cin;
        val = j.s0[((size_t)k * C + c) * Cin + ci];
        break;
      }
      case PREP_PACK_GCN_T: {  // dgrad operand: dst [K*Cin][C]
        const int C = j.d0, Cin = j.d1;
        const int kc = e / C, c = e - kc * C, k = kc / Cin, ci = kc - k * Cin;
        val = j.s0[((size_t)k * C + c) * Cin + ci];
        break;
      }
      case PREP_GCN_BIAS: {  // dst[w][c] = sum_k colsum(A*E)_k[w] * b[k*C+c]
        const int C = j.d0, V = j.d1, K = j.d2;
        const int w = e / C, c = e - w * C;
        float acc = 0.f;
        for (int k = 0; k < K; ++k) {
          float cs = 0.f;
          if (V <= kPrepVMax) {  // a column's loads issued together (the same sum, v ascending)
            float av[kPrepVMax], ev[kPrepVMax];
#pragma unroll
            for (int v = 0; v < kPrepVMax; ++v) {
              av[v] = v < V ? j.s0[(k * V + v) * V + w] : 0.f;
              ev[v] = v < V ? j.s1[(k * V + v) * V + w] : 0.f;
            }
#pragma unroll
            for (int v = 0; v < kPrepVMax; ++v)
              if (v < V) cs += av[v] * ev[v];
          } else {
            for (int v = 0; v < V; ++v) cs += j.s0[(k * V + v) * V + w] * j.s1[(k * V + v) * V + w];
          }
          acc += cs * j.s2[k * C + c];
        }
        val = acc;
        break;
      }
    }
    if (j.bf16 == 2) {  // bf16x3 mode: hi = RNE bf16(val) at [e], lo = RNE bf16(val - hi) at [n + e]
      const __bf16 hi = (__bf16)val;
      reinterpret_cast<__bf16*>(j.dst)[e] = hi;
      reinterpret_cast<__bf16*>(j.dst)[j.n + e] = (__bf16)(val - (float)hi);
    } else if (j.bf16) {
      reinterpret_cast<__bf16*>(j.dst)[e] = (__bf16)val;  // RNE (v_cvt_pk_bf16_f32)
    } else {
      j.dst[e] = val;
    }
  }
}

// ----------------------------------------------------------------------------
// data_bn (stgcan.py:213-218): BatchNorm1d over V*C channels (index v*C + c), stats
// over (N, T). The motion stream's input (combination.py:39) is formed on the fly.
// ----------------------------------------------------------------------------
F3_DEV float stream_in(const float* skel, int motion, int n, int c, int t, int v, int T, int V) {
  // skel is the reference layout [N][3][T][V]; motion: [N][2][T-1][V] = skel[t+1]-skel[t]
  const int Ts = motion ? T + 1 : T;
  const float* p = skel + (((size_t)n * 3 + c) * Ts + t) * V + v;
  return motion ? (p[V] - p[0]) : p[0];
}

// one 1024-thread workgroup per channel (a channel's N*T inputs are strided by V floats: latency,
// not bandwidth, bounds it), kDbnU inputs loaded per thread before they are summed
constexpr int kDbnU = 4;
__global__ __launch_bounds__(1024) void databn_stats_kernel(DataBnArgs a) {
  const int ch = blockIdx.x, v = ch / a.C, c = ch - v * a.C;
  const int NT = a.N * a.T;
  double s = 0.0, q = 0.0;
  for (int e0 = threadIdx.x; e0 < NT; e0 += kDbnU * blockDim.x) {
    float x[kDbnU];
#pragma unroll
    for (int u = 0; u < kDbnU; ++u) {
      const int e = e0 + u * blockDim.x;
      const int n = e / a.T, t = e - n * a.T;
      x[u] = e < NT ? stream_in(a.skel, a.motion, n, c, t, v, a.T, a.V) : 0.f;
    }
#pragma unroll
    for (int u = 0; u < kDbnU; ++u) {
      s += x[u];
      q += (double)x[u] * x[u];
    }
  }
  __shared__ double rs[2][16];
  s = warp_sum_d(s);
  q = warp_sum_d(q);
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) { rs[0][w] = s; rs[1][w] = q; }
  __syncthreads();
  if (threadIdx.x == 0) {
    double S = 0, Q = 0;
    for (int i = 0; i < (int)(blockDim.x >> 6); ++i) { S += rs[0][i]; Q += rs[1][i]; }
    a.st_sum[ch] = S;
    a.st_sq[ch] = Q;
  }
}

__global__ void databn_apply_kernel(DataBnArgs a) {
  const int total = a.N * a.T * a.V * a.C;
  for (int e = blockIdx.x * blockDim.x + threadIdx.x; e < total; e += gridDim.x * blockDim.x) {
    const int c = e % a.C, m = e / a.C, v = m % a.V, nt = m / a.V, t = nt % a.T, n = nt / a.T;
    float sc, sh, mu, rs;
    bn_coeff(a.bn, v * a.C + c, sc, sh, mu, rs);
    const float val = stream_in(a.skel, a.motion, n, c, t, v, a.T, a.V) * sc + sh;
    if (a.act16) reinterpret_cast<__bf16*>(a.out)[e] = (__bf16)val;
    else a.out[e] = val;
  }
}

// d gamma / d beta of data_bn from the gradient of its (channels-last) output
__global__ void databn_bwd_kernel(DataBnArgs a) {
  const int ch = blockIdx.x, v = ch / a.C, c = ch - v * a.C;
  float sc, sh, mu, rs;
  bn_coeff(a.bn, ch, sc, sh, mu, rs);
  double s = 0.0, q = 0.0;
  for (int e = threadIdx.x; e < a.N * a.T; e += blockDim.x) {
    const int n = e / a.T, t = e - n * a.T;
    const float x = stream_in(a.skel, a.motion, n, c, t, v, a.T, a.V);
    const float dy = a.dout[(((size_t)n * a.T + t) * a.V + v) * a.C + c];
    s += dy;
    q += (double)dy * ((x - mu) * rs);
  }
  __shared__ double rsd[2][16];
  s = warp_sum_d(s);
  q = warp_sum_d(q);
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) { rsd[0][w] = s; rsd[1][w] = q; }
  __syncthreads();
  if (threadIdx.x == 0) {
    double S = 0, Q = 0;
    for (int i = 0; i < (int)(blockDim.x >> 6); ++i) { S += rsd[0][i]; Q += rsd[1][i]; }
    a.dgamma[ch] += (float)Q;
    a.dbeta[ch] += (float)S;
  }
}

// ----------------------------------------------------------------------------
// graph mix (stgcan.py:54, reordered): Z[(f,w), k*Cin+ci] = sum_v A_eff[k,v,w] x[(f,v),ci]
// ----------------------------------------------------------------------------
__global__ __launch_bounds__(256) void mix_fwd_kernel(MixArgs a) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  float* As = sm;                       // [K][V][V]
  float* xs = sm + a.K * a.V * a.V;     // [V][Cin]
  const int KVV = a.K * a.V * a.V;
  for (int i = threadIdx.x; i < KVV; i += blockDim.x) As[i] = a.A[i];
  const int per = a.V * a.Cin;
  const int outs = a.V * a.K * a.Cin;
  for (int f = blockIdx.x; f < a.frames; f += gridDim.x) {
    __syncthreads();
    for (int i = threadIdx.x; i < per; i += blockDim.x) xs[i] = ld_act(a.x, (size_t)f * per + i, a.x16);
    __syncthreads();
    for (int o = threadIdx.x; o < outs; o += blockDim.x) {
      const int ci = o % a.Cin, wk = o / a.Cin, k = wk % a.K, w = wk / a.K;
      float acc = 0.f;
      for (int v = 0; v < a.V; ++v) acc += As[(k * a.V + v) * a.V + w] * xs[v * a.Cin + ci];
      if (a.zb) reinterpret_cast<__bf16*>(a.zb)[(size_t)f * outs + o] = (__bf16)acc;
      else a.z[(size_t)f * outs + o] = acc;
    }
  }
}

// dx[(f,v),ci] (+)= sum_{k,w} A_eff[k,v,w] dZ[(f,w),(k,ci)]
// dA[k,v,w]   += sum_{f,ci} x[(f,v),ci] dZ[(f,w),(k,ci)]
__global__ __launch_bounds__(256) void mix_bwd_kernel(MixArgs a) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  const int KVV = a.K * a.V * a.V;
  const int per = a.V * a.Cin, outs = a.V * a.K * a.Cin;
  float* As = sm;                 // [K][V][V]
  float* xs = As + KVV;           // [V][Cin]
  float* zs = xs + per;           // [V][K][Cin]
  for (int i = threadIdx.x; i < KVV; i += blockDim.x) As[i] = a.A[i];
  // dA accumulators: each thread owns up to 4 (k,v,w) entries
  float dacc[4] = {0.f, 0.f, 0.f, 0.f};
  for (int f = blockIdx.x; f < a.frames; f += gridDim.x) {
    __syncthreads();
    for (int i = threadIdx.x; i < per; i += blockDim.x) xs[i] = ld_act(a.x, (size_t)f * per + i, a.x16);
    for (int i = threadIdx.x; i < outs; i += blockDim.x) zs[i] = a.z[(size_t)f * outs + i];
    __syncthreads();
    for (int o = threadIdx.x; o < per; o += blockDim.x) {
      const int ci = o % a.Cin, v = o / a.Cin;
      float acc = 0.f;
      for (int k = 0; k < a.K; ++k)
        for (int w = 0; w < a.V; ++w) acc += As[(k * a.V + v) * a.V + w] * zs[(w * a.K + k) * a.Cin + ci];
      float* dst = a.dx + (size_t)f * per + o;
      if (a.accumulate) *dst += acc;
      else *dst = acc;
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int idx = threadIdx.x + q * blockDim.x;
      if (idx >= KVV) break;
      const int k = idx / (a.V * a.V), r = idx - k * a.V * a.V, v = r / a.V, w = r - v * a.V;
      const float* xr = xs + v * a.Cin;
      const float* zr = zs + (w * a.K + k) * a.Cin;
      float acc = 0.f;
      for (int ci = 0; ci < a.Cin; ++ci) acc += xr[ci] * zr[ci];
      dacc[q] += acc;
    }
  }
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int idx = threadIdx.x + q * blockDim.x;
    if (idx < KVV) atomic_add_f(a.dA + idx, dacc[q]);
  }
}

// ---------------------------------------------------------------------------
// MFMA forms of the graph mix (Cin % 16 == 0, K*V <= 64, V <= 32). Per frame f the mix
// is a tiny fixed left matrix times a [V x Cin] slab, so each wave keeps its fragments
// of A~[(w,k)][v] = A_eff[k][v][w] in registers and streams 16-channel column tiles.
//   fwd:  Z_f[(w,k)][ci] = sum_v  A~[(w,k)][v]  X_f[v][ci]
//   dx:   dX_f[v][ci]    = sum_wk A~[(w,k)][v]  dZ_f[(w,k)][ci]
//   dA:   dA[k][v][w]   += sum_{f,ci} X_f[v][ci] dZ_f[(w,k)][ci]
// (v_mfma_f32_16x16x4_f32; lane l: A[i=l&15][k=l>>4], B[k=l>>4][j=l&15],
//  D row 4*(l>>4)+r, col l&15)
// ---------------------------------------------------------------------------
F3_DEV f32x4 mfma16x4(float a, float b, f32x4 c) { return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0); }

F3_DEV float atil(const float* A, int K, int V, int wk, int v) {
  if (wk >= K * V || v >= V) return 0.f;
  const int w = wk / K, k = wk - w * K;
  return A[(k * V + v) * V + w];
}

// ---------------------------------------------------------------------------
// LDS-staged graph mix (Cin % 16 == 0, K*V <= 64, V <= 32): one frame at a time per
// workgroup, the frame's [V][Cin] input (and [K*V][Cin] gradient) loaded with coalesced
// 16-B reads into LDS (row stride Cin+20 floats: conflict-light scalar and b128 fragment
// reads), fp32 MFMA 16x16x4 with the fixed A~ fragments in registers, outputs written
// back through LDS as whole rows. The backward computes dX and dA from ONE read of dZ.
// ---------------------------------------------------------------------------

// Frame inputs are prefetched into registers one frame ahead as RAW 16-B / 8-B pieces
// (converted only when written to LDS, so the loads stay in flight during the previous
// frame's MFMAs); MFMA operand reads from LDS are unconditional (clamped row + 0/1 mask)
// so the compiler batches them.
// per-thread prefetch capacity (16-B x pieces / 8-B bf16 gradient pieces) for V <= 18, K <= 3
template <int CIN> struct MixCap {
  static constexpr int PX = (18 * CIN + 1023) / 1024;
  static constexpr int PZ = (54 * CIN + 1023) / 1024;
};

typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));

F3_DEV f32x4 bf4_to_f4(u32x2 r) {
  return f32x4{__uint_as_float(r.x << 16), __uint_as_float(r.x & 0xffff0000u), __uint_as_float(r.y << 16),
               __uint_as_float(r.y & 0xffff0000u)};
}

// Wave-per-frame graph mix forward: each wave owns whole frames (no workgroup barrier: a
// workgroup-per-frame form paid 3 barriers per frame), keeps its frame's [V][Cin] input in a
// wave-private LDS slab (bf16 when x is bf16), prefetches the next frame's input into registers
// during the MFMAs, and writes Z one 16-channel tile at a time through a [64][20] fp32 LDS tile
// as 16-B row pieces (L2 merges a wave's consecutive tiles into whole lines).
template <int CIN> struct MixWaveCap {
  static constexpr int PX = (18 * CIN / 4 + 63) / 64;  // 8-B (bf16) or 16-B (fp32) input pieces per lane
};

template <int KS, int CIN, bool XB>
__global__ __launch_bounds__(256) void mix_fwd_wave_kernel(MixArgs a) {
  using T = typename std::conditional<XB, unsigned short, float>::type;
  constexpr int PX = MixWaveCap<CIN>::PX;
  constexpr int S = CIN + (XB ? 8 : 4);    // LDS row stride (elements)
  constexpr int ZS = 20;                    // zt row stride (floats)
  constexpr int XW = 18 * S * (int)sizeof(T), ZW = 64 * ZS * 4;  // bytes per wave
  extern __shared__ __attribute__((aligned(16))) char smw[];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  T* xs = reinterpret_cast<T*>(smw + wave * (XW + ZW));
  float* zt = reinterpret_cast<float*>(smw + wave * (XW + ZW) + XW);
  const int fr = lane & 15, fg = lane >> 4;
  const int K = a.K, V = a.V, KV = K * V;
  // A_eff once per workgroup through LDS (coalesced), then each lane's 4*KS fragment values:
  // gathering them straight from global memory cost every wave 20 scattered loads
  {
    float* As = reinterpret_cast<float*>(smw + 4 * (XW + ZW));
    for (int i = threadIdx.x; i < K * V * V; i += 256) As[i] = a.A[i];
    __syncthreads();
  }
  const float* As = reinterpret_cast<const float*>(smw + 4 * (XW + ZW));
  float af[4][KS];
#pragma unroll
  for (int mt = 0; mt < 4; ++mt)
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) af[mt][ks] = atil(As, K, V, 16 * mt + fr, 4 * ks + fg);
  const int n4 = V * CIN / 4, C4 = CIN / 4;
  u32x2 rb[XB ? PX : 1];
  f32x4 rf[XB ? 1 : PX];
  auto prefetch = [&](int f) {  // unconditional loads from clamped indices
#pragma unroll
    for (int q = 0; q < PX; ++q) {
      const int i = min(lane + q * 64, n4 - 1);
      if constexpr (XB) rb[q] = reinterpret_cast<const u32x2*>(reinterpret_cast<const __bf16*>(a.x) + (size_t)f * V * CIN)[i];
      else rf[q] = reinterpret_cast<const f32x4*>(a.x + (size_t)f * V * CIN)[i];
    }
  };
  const int gw = blockIdx.x * 4 + wave, nw = gridDim.x * 4;
  if (gw < a.frames) prefetch(gw);
  for (int f = gw; f < a.frames; f += nw) {
#pragma unroll
    for (int q = 0; q < PX; ++q) {
      const int i = lane + q * 64;
      if (i < n4) {
        const int v = i / C4, c = (i - v * C4) * 4;
        if constexpr (XB) *reinterpret_cast<u32x2*>(xs + v * S + c) = rb[q];
        else *reinterpret_cast<f32x4*>(xs + v * S + c) = rf[q];
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    if (f + nw < a.frames) prefetch(f + nw);
    const size_t zoff = (size_t)f * KV * CIN;
#pragma unroll 1
    for (int t = 0; t < CIN / 16; ++t) {
      const int ci0 = t * 16;
      float b[KS];
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        const int v = 4 * ks + fg;
        const T raw = xs[min(v, V - 1) * S + ci0 + fr];
        float xv;
        if constexpr (XB) xv = __uint_as_float((unsigned)raw << 16);
        else xv = raw;
        b[ks] = v < V ? xv : 0.f;
      }
      f32x4 acc[4];
#pragma unroll
      for (int mt = 0; mt < 4; ++mt) acc[mt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < KS; ++ks)
#pragma unroll
        for (int mt = 0; mt < 4; ++mt) acc[mt] = mfma16x4(af[mt][ks], b[ks], acc[mt]);
#pragma unroll
      for (int mt = 0; mt < 4; ++mt)
#pragma unroll
        for (int r = 0; r < 4; ++r) zt[(16 * mt + 4 * fg + r) * ZS + fr] = acc[mt][r];
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      if (a.zb) {  // 16-B pieces: (row wk, half h) -> 8 bf16
        for (int p = lane; p < 2 * KV; p += 64) {
          const int wk = p >> 1, h = p & 1;
          const f32x4 u0 = *reinterpret_cast<const f32x4*>(zt + wk * ZS + 8 * h);
          const f32x4 u1 = *reinterpret_cast<const f32x4*>(zt + wk * ZS + 8 * h + 4);
          bf16x8 o;
#pragma unroll
          for (int e = 0; e < 4; ++e) { o[e] = (__bf16)u0[e]; o[4 + e] = (__bf16)u1[e]; }
          *reinterpret_cast<bf16x8*>(reinterpret_cast<__bf16*>(a.zb) + zoff + (size_t)wk * CIN + ci0 + 8 * h) = o;
        }
      } else {  // fp32 z: (row wk, quarter h) -> 4 floats
        for (int p = lane; p < 4 * KV; p += 64) {
          const int wk = p >> 2, h = p & 3;
          *reinterpret_cast<f32x4*>(a.z + zoff + (size_t)wk * CIN + ci0 + 4 * h) =
              *reinterpret_cast<const f32x4*>(zt + wk * ZS + 4 * h);
        }
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // zt is rewritten by the next tile
    }
  }
}

template <int KS, int CIN, bool ZB16, bool ACC>  // k steps over (w,k): ceil(K*V/4); ZB16: dZ is bf16;
__global__ __launch_bounds__(256) void mix_bwd_lds_kernel(MixArgs a) {  // ACC: dx += (identity residual)
  constexpr int kMixPX = MixCap<CIN>::PX, kMixPZ = MixCap<CIN>::PZ;
  extern __shared__ __attribute__((aligned(16))) float sm[];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, tid = threadIdx.x;
  const int fr = lane & 15, fg = lane >> 4;
  const int K = a.K, V = a.V, KV = K * V, KVV = KV * V;
  constexpr int Cin = CIN, S = CIN + 20;
  float* xs = sm;            // [V][S]
  float* zs = sm + V * S;    // [KV][S]
  float* ds = zs + KV * S;   // [V][S] current dx (accumulate: identity-residual gradient)
  float adx[2][KS];
#pragma unroll
  for (int mt = 0; mt < 2; ++mt)
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) adx[mt][ks] = atil(a.A, K, V, 4 * ks + fg, 16 * mt + fr);
  // dA tiles of this wave: (mt, nt) = (wave >> 1, 2*(wave & 1) + {0,1}) over [32 v][64 wk]
  const int dmt = wave >> 1, dnt0 = 2 * (wave & 1);
  f32x4 dacc[2] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};
  const int tiles = Cin / 16, n4x = V * Cin / 4, n4z = KV * Cin / 4, C4 = Cin / 4;
  constexpr bool zb16 = ZB16;
  // the bf16 mode stores x in bf16 as well (ZB16 <=> bf16 mode; the launcher checks x16)
  f32x4 rx[ZB16 ? 1 : kMixPX], rd[kMixPX];
  u32x2 rxb[ZB16 ? kMixPX : 1];
  u32x2 rz[ZB16 ? kMixPZ : 1];  // bf16 gradient pieces, raw
  auto prefetch = [&](int f) {  // unconditional loads from clamped indices (see mix_fwd_lds)
    const f32x4* dg = reinterpret_cast<const f32x4*>(a.dx + (size_t)f * V * Cin);
#pragma unroll
    for (int q = 0; q < kMixPX; ++q) {
      const int i = min(tid + q * 256, n4x - 1);
      if constexpr (ZB16) rxb[q] = reinterpret_cast<const u32x2*>(reinterpret_cast<const __bf16*>(a.x) + (size_t)f * V * Cin)[i];
      else rx[q] = reinterpret_cast<const f32x4*>(a.x + (size_t)f * V * Cin)[i];
      if constexpr (ACC) rd[q] = dg[i];
    }
    if constexpr (zb16) {
      const u32x2* zg = reinterpret_cast<const u32x2*>(a.dzb + (size_t)f * KV * Cin);
#pragma unroll
      for (int q = 0; q < kMixPZ; ++q) rz[q] = zg[min(tid + q * 256, n4z - 1)];
    }
  };
  if (blockIdx.x < a.frames) prefetch(blockIdx.x);
  for (int f = blockIdx.x; f < a.frames; f += gridDim.x) {
    __syncthreads();  // the previous frame is done with xs / zs / ds
#pragma unroll
    for (int q = 0; q < kMixPX; ++q) {
      const int i = tid + q * 256;
      if (i < n4x) {
        const int v = i / C4, c = (i - v * C4) * 4;
        if constexpr (ZB16) *reinterpret_cast<f32x4*>(xs + v * S + c) = bf4_to_f4(rxb[q]);
        else *reinterpret_cast<f32x4*>(xs + v * S + c) = rx[q];
        if (ACC) *reinterpret_cast<f32x4*>(ds + v * S + c) = rd[q];
      }
    }
    if constexpr (zb16) {
#pragma unroll
      for (int q = 0; q < kMixPZ; ++q) {
        const int i = tid + q * 256;
        if (i < n4z) {
          const int wk = i / C4, c = (i - wk * C4) * 4;
          *reinterpret_cast<f32x4*>(zs + wk * S + c) = bf4_to_f4(rz[q]);
        }
      }
    } else {  // fp32 mode: load the gradient frame now (batched: all loads, then the writes)
      const f32x4* zg = reinterpret_cast<const f32x4*>(a.z + (size_t)f * KV * Cin);
      for (int i0 = 0; i0 < n4z; i0 += 8 * 256) {
        f32x4 tmp[8];
#pragma unroll
        for (int q = 0; q < 8; ++q) {
          const int i = i0 + tid + q * 256;
          if (i < n4z) tmp[q] = zg[i];
        }
#pragma unroll
        for (int q = 0; q < 8; ++q) {
          const int i = i0 + tid + q * 256;
          if (i < n4z) {
            const int wk = i / C4, c = (i - wk * C4) * 4;
            *reinterpret_cast<f32x4*>(zs + wk * S + c) = tmp[q];
          }
        }
      }
    }
    __syncthreads();
    if (f + (int)gridDim.x < a.frames) prefetch(f + gridDim.x);
    // dX_f[v][ci] = sum_wk A~[v][wk] dZ_f[wk][ci]
    for (int t = wave; t < tiles; t += 4) {
      const int ci0 = t * 16;
      f32x4 acc[2] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};
      float b[KS];
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        const int wk = 4 * ks + fg;
        b[ks] = zs[min(wk, KV - 1) * S + ci0 + fr] * (wk < KV ? 1.f : 0.f);
      }
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        acc[0] = mfma16x4(adx[0][ks], b[ks], acc[0]);
        acc[1] = mfma16x4(adx[1][ks], b[ks], acc[1]);
      }
      float* dx = a.dx + (size_t)f * V * Cin + ci0 + fr;
#pragma unroll
      for (int mt = 0; mt < 2; ++mt)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int v = 16 * mt + 4 * fg + r;
          if (v < V) dx[(size_t)v * Cin] = acc[mt][r] + (ACC ? ds[v * S + ci0 + fr] : 0.f);
        }
    }
    // dA[v][wk] += sum_ci X_f[v][ci] dZ_f[wk][ci]   (k index of the MFMA = lane group,
    // the 4 components of each b128 read are 4 k-steps)
    {
      const int v = 16 * dmt + fr;
      const float mv = v < V ? 1.f : 0.f;
      const float* xrow = xs + min(v, V - 1) * S + 4 * fg;
      const int wk0 = 16 * dnt0 + fr, wk1 = wk0 + 16;
      const float m0 = wk0 < KV ? 1.f : 0.f, m1 = wk1 < KV ? 1.f : 0.f;
      const float* z0 = zs + min(wk0, KV - 1) * S + 4 * fg;
      const float* z1 = zs + min(wk1, KV - 1) * S + 4 * fg;
      for (int c16 = 0; c16 < Cin; c16 += 16) {
        const f32x4 xa = *reinterpret_cast<const f32x4*>(xrow + c16) * mv;
        const f32x4 za = *reinterpret_cast<const f32x4*>(z0 + c16) * m0;
        const f32x4 zb = *reinterpret_cast<const f32x4*>(z1 + c16) * m1;
#pragma unroll
        for (int s2 = 0; s2 < 4; ++s2) {
          dacc[0] = mfma16x4(xa[s2], za[s2], dacc[0]);
          dacc[1] = mfma16x4(xa[s2], zb[s2], dacc[1]);
        }
      }
    }
  }
  // workgroup partial row of dA (each (v, wk) has exactly one owner lane), then f3_colsum
  __syncthreads();
  float* red = sm;
  for (int i = tid; i < KVV; i += 256) red[i] = 0.f;
  __syncthreads();
#pragma unroll
  for (int q = 0; q < 2; ++q)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int v = 16 * dmt + 4 * fg + r, wk = 16 * (dnt0 + q) + fr;
      if (v < V && wk < KV) {
        const int w = wk / K, k = wk - w * K;
        red[(k * V + v) * V + w] = dacc[q][r];
      }
    }
  __syncthreads();
  float* row = a.part + (size_t)blockIdx.x * KVV;
  for (int i = tid; i < KVV; i += 256) row[i] = red[i];
}

// ----------------------------------------------------------------------------
// Graph-mix backward of the bf16 mode on bf16 MFMA (16x16x32). x and dZ are stored bf16, so
// dA = sum_{f,c} X_f[v][c] dZ_f[wk][c] takes them as MFMA operands with exact products and fp32
// accumulation (what the fp32 16x16x4 kernel computed, at 8x the MFMA rate); for
// dX = A~ . dZ the fp32 A~ is split into bf16 hi + lo (hi = its top 16 bits, lo = the rest
// rounded: |A~ - hi - lo| <= 2^-17 |A~|), two MFMAs per product. The fp32 16x16x4 kernel was
// bound by its MFMA work (~4 GFLOP padded per layer = ~25 us at the fp32 MFMA rate) and ran
// 53-107 us. One frame per loop trip: the frame's x [V][C] and dZ [KV][C] rows (bf16, prefetched
// into registers one frame ahead) land in LDS rows of 2C + 16 bytes (conflict-free 16-B row
// reads); dX's dZ fragments are transposed LDS reads (ds_read_b64_tr_b16), dA's fragments plain
// 16-B reads. dZ rows KV..63 are zero (they meet A~'s zero columns; garbage there could be NaN).
// Wave w: dX tiles nt = w, w + 4, ..; dA column tile wk 16w..16w+15 (all K*V <= 64) for both
// v tiles, accumulated over the workgroup's frames into one partial row (f3_colsum after).
// ----------------------------------------------------------------------------
typedef short mx_s16x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) const char mx_lds_t;
F3_DEV f32x4 mfma_bf16x(bf16x8 a, bf16x8 b, f32x4 c) { return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0); }

F3_DEV void a_split(float t, __bf16& hi, __bf16& lo) {
  const float h = __uint_as_float(__float_as_uint(t) & 0xffff0000u);
  hi = __builtin_bit_cast(__bf16, (unsigned short)(__float_as_uint(h) >> 16));
  lo = (__bf16)(t - h);
}

template <int CIN, bool ACC>
__global__ __launch_bounds__(256) void mix_bwd_bf16_kernel(MixArgs a) {
  constexpr int RB = 2 * CIN + 16, XR = 32, ZR = 64, C8 = CIN / 8;
  constexpr int PX = (18 * C8 + 255) / 256, PZ = (54 * C8 + 255) / 256;
  extern __shared__ __attribute__((aligned(16))) char smb[];
  char* xs = smb;            // [32][RB]
  char* zs = smb + XR * RB;  // [64][RB]
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, tid = threadIdx.x;
  const int fr = lane & 15, fg = lane >> 4;
  const int K = a.K, V = a.V, KV = K * V;
  const int nx = V * C8, nz = KV * C8;
  // A~ as the dX A operand: lane holds rows v = 16 mt + fr, k = wk = 32 ks + 8 fg + e
  bf16x8 ahi[2][2], alo[2][2];
#pragma unroll
  for (int mt = 0; mt < 2; ++mt)
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        __bf16 h, l;
        a_split(atil(a.A, K, V, 32 * ks + 8 * fg + e, 16 * mt + fr), h, l);
        ahi[mt][ks][e] = h;
        alo[mt][ks][e] = l;
      }
  for (int o = KV * RB + tid * 16; o < ZR * RB; o += 256 * 16)
    *reinterpret_cast<f32x4*>(zs + o) = f32x4{0.f, 0.f, 0.f, 0.f};
  f32x4 dacc[2] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};
  f32x4 rx[PX], rz[PZ];  // 16-B bf16 pieces of the next frame (unconditional, clamped loads)
  auto prefetch = [&](int f) {
    const f32x4* xg = reinterpret_cast<const f32x4*>(reinterpret_cast<const __bf16*>(a.x) + (size_t)f * V * CIN);
    const f32x4* zg = reinterpret_cast<const f32x4*>(reinterpret_cast<const __bf16*>(a.dzb) + (size_t)f * KV * CIN);
#pragma unroll
    for (int q = 0; q < PX; ++q) rx[q] = xg[min(tid + q * 256, nx - 1)];
#pragma unroll
    for (int q = 0; q < PZ; ++q) rz[q] = zg[min(tid + q * 256, nz - 1)];
  };
  if (blockIdx.x < a.frames) prefetch(blockIdx.x);
  for (int f = blockIdx.x; f < a.frames; f += gridDim.x) {
    __syncthreads();  // the previous frame's reads of xs / zs are done
#pragma unroll
    for (int q = 0; q < PX; ++q) {
      const int i = tid + q * 256;
      if (i < nx) *reinterpret_cast<f32x4*>(xs + (i / C8) * RB + (i % C8) * 16) = rx[q];
    }
#pragma unroll
    for (int q = 0; q < PZ; ++q) {
      const int i = tid + q * 256;
      if (i < nz) *reinterpret_cast<f32x4*>(zs + (i / C8) * RB + (i % C8) * 16) = rz[q];
    }
    __syncthreads();
    if (f + (int)gridDim.x < a.frames) prefetch(f + gridDim.x);
    // dX_f[v][c] = sum_wk A~[v][wk] dZ_f[wk][c]
    float* dxf = a.dx + (size_t)f * V * CIN;
    for (int nt = wave; nt < CIN / 16; nt += 4) {
      bf16x8 b[2];
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        const unsigned p = (unsigned)(size_t)(mx_lds_t*)(zs + (32 * ks + 8 * fg + (fr >> 2)) * RB + 32 * nt + 8 * (fr & 3));
        mx_s16x4 lo, hi;
        asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(lo) : "v"(p));
        asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(hi) : "v"(p), "n"(4 * RB));
        asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(lo), "+v"(hi)::"memory");
        b[ks] = __builtin_bit_cast(bf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
      }
      f32x4 acc[2] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};
#pragma unroll
      for (int mt = 0; mt < 2; ++mt)
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) {
          acc[mt] = mfma_bf16x(ahi[mt][ks], b[ks], acc[mt]);
          acc[mt] = mfma_bf16x(alo[mt][ks], b[ks], acc[mt]);
        }
      // lane holds v = 16 mt + 4 fg + r, c = 16 nt + fr; old values (identity residual) first
      float old[2][4];
#pragma unroll
      for (int mt = 0; mt < 2; ++mt)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int v = min(16 * mt + 4 * fg + r, V - 1);
          old[mt][r] = ACC ? dxf[(size_t)v * CIN + 16 * nt + fr] : 0.f;
        }
#pragma unroll
      for (int mt = 0; mt < 2; ++mt)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int v = 16 * mt + 4 * fg + r;
          if (v < V) dxf[(size_t)v * CIN + 16 * nt + fr] = acc[mt][r] + old[mt][r];
        }
    }
    // dA[v][wk] += sum_c X_f[v][c] dZ_f[wk][c]: this wave's wk tile, both v tiles
#pragma unroll 4
    for (int ks = 0; ks < CIN / 32; ++ks) {
      const int cb = (32 * ks + 8 * fg) * 2;
      const bf16x8 zb = *reinterpret_cast<const bf16x8*>(zs + (16 * wave + fr) * RB + cb);
      const bf16x8 x0 = *reinterpret_cast<const bf16x8*>(xs + fr * RB + cb);
      const bf16x8 x1 = *reinterpret_cast<const bf16x8*>(xs + (16 + fr) * RB + cb);
      dacc[0] = mfma_bf16x(x0, zb, dacc[0]);
      dacc[1] = mfma_bf16x(x1, zb, dacc[1]);
    }
  }
  // partial row of dA in the reference layout [k][v][w]: every (v < V, wk < KV) has one owner
  float* row = a.part + (size_t)blockIdx.x * K * V * V;
#pragma unroll
  for (int mt = 0; mt < 2; ++mt)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int v = 16 * mt + 4 * fg + r, wk = 16 * wave + fr;
      if (v < V && wk < KV) {
        const int w = wk / K, k = wk - w * K;
        row[(k * V + v) * V + w] = dacc[mt][r];
      }
    }
}

// Graph-mix forward of the bf16 mode on bf16 MFMA 16x16x32, in the backward kernel's form: one
// frame per loop trip (its x rows prefetched into registers one frame ahead, staged in LDS rows
// of 2C + 16 bytes), Z^T tiles out[c][wk] = sum_v x[v][c] A~[wk][v] with x fragments as
// transposed LDS reads and A~ (fp32) as bf16 hi + lo fragments held in registers, the tile
// written into an LDS image of the frame's Z [KV][C] (bf16, 8-B pieces: 4 channels of one row)
// and copied out as 16-B pieces of the contiguous frame. x rows V..31 are zero (they meet
// A~'s zero rows). Wave w: channel tiles w, w + 4, ...
template <int CIN>
__global__ __launch_bounds__(256) void mix_fwd_bf16_kernel(MixArgs a) {
  constexpr int RB = 2 * CIN + 16, XR = 32, C8 = CIN / 8;
  constexpr int PX = (18 * C8 + 255) / 256;
  extern __shared__ __attribute__((aligned(16))) char smb[];
  char* xs = smb;            // [32][RB]
  char* zt = smb + XR * RB;  // [64][RB]
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, tid = threadIdx.x;
  const int fr = lane & 15, fg = lane >> 4;
  const int K = a.K, V = a.V, KV = K * V;
  const int nx = V * C8, nz = KV * C8;
  // B operand: lane holds k = v = 8 fg + e, n = wk = 16 nt + fr
  bf16x8 bhi[4], blo[4];
#pragma unroll
  for (int nt = 0; nt < 4; ++nt)
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      __bf16 h, l;
      a_split(atil(a.A, K, V, 16 * nt + fr, 8 * fg + e), h, l);
      bhi[nt][e] = h;
      blo[nt][e] = l;
    }
  for (int o = V * RB + tid * 16; o < XR * RB; o += 256 * 16)
    *reinterpret_cast<f32x4*>(xs + o) = f32x4{0.f, 0.f, 0.f, 0.f};
  f32x4 rx[PX];
  auto prefetch = [&](int f) {
    const f32x4* xg = reinterpret_cast<const f32x4*>(reinterpret_cast<const __bf16*>(a.x) + (size_t)f * V * CIN);
#pragma unroll
    for (int q = 0; q < PX; ++q) rx[q] = xg[min(tid + q * 256, nx - 1)];
  };
  if (blockIdx.x < a.frames) prefetch(blockIdx.x);
  for (int f = blockIdx.x; f < a.frames; f += gridDim.x) {
    __syncthreads();  // the previous frame's xs reads and zt copy-out are done
#pragma unroll
    for (int q = 0; q < PX; ++q) {
      const int i = tid + q * 256;
      if (i < nx) *reinterpret_cast<f32x4*>(xs + (i / C8) * RB + (i % C8) * 16) = rx[q];
    }
    __syncthreads();
    if (f + (int)gridDim.x < a.frames) prefetch(f + gridDim.x);
    for (int mt = wave; mt < CIN / 16; mt += 4) {
      const unsigned p = (unsigned)(size_t)(mx_lds_t*)(xs + (8 * fg + (fr >> 2)) * RB + 32 * mt + 8 * (fr & 3));
      mx_s16x4 lo, hi;
      asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(lo) : "v"(p));
      asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(hi) : "v"(p), "n"(4 * RB));
      asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(lo), "+v"(hi)::"memory");
      const bf16x8 xa = __builtin_bit_cast(bf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) {
        f32x4 acc = mfma_bf16x(xa, bhi[nt], f32x4{0.f, 0.f, 0.f, 0.f});
        acc = mfma_bf16x(xa, blo[nt], acc);
        // lane holds Z[wk = 16 nt + fr][c = 16 mt + 4 fg + r], r = 0..3: one 8-B piece
        bf16x4 o;
#pragma unroll
        for (int r = 0; r < 4; ++r) o[r] = (__bf16)acc[r];
        *reinterpret_cast<bf16x4*>(zt + (16 * nt + fr) * RB + (16 * mt + 4 * fg) * 2) = o;
      }
    }
    __syncthreads();
    f32x4* zg = reinterpret_cast<f32x4*>(a.zb + (size_t)f * KV * CIN);
    for (int i = tid; i < nz; i += 256) zg[i] = *reinterpret_cast<const f32x4*>(zt + (i / C8) * RB + (i % C8) * 16);
  }
}

// ----------------------------------------------------------------------------
// Graph mix of the bf16x3 parity mode (F3_PRECISION_BF16X3: fp32 x / Z / dZ, gemm_x3.hip's split):
// the bf16 kernels' structure with BOTH operands split, x = x_hi + x_lo (hi = RNE bf16, lo = RNE
// bf16 of the rest) and A~ = hi + lo (a_split), each product as lo*hi + hi*lo + hi*hi on bf16
// MFMA into one fp32 accumulator (~2^-16 per product). The frame's fp32 rows are prefetched into
// registers one frame ahead and split while they are staged into two bf16 LDS planes (hi, lo) of
// rows of 2C + 16 bytes. The forward writes fp32 Z straight from the accumulators (a lane's 4
// consecutive channels: 16-B pieces); the backward as mix_bwd_bf16 (dX: A~ fragments in registers,
// dZ by transposed LDS reads; dA: x and dZ by 16-B LDS reads; per-workgroup dA partial rows).
// ----------------------------------------------------------------------------
F3_DEV void split4_store(const f32x4 v, char* hi, char* lo) {
  bf16x4 h, l;
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    h[e] = (__bf16)v[e];
    l[e] = (__bf16)(v[e] - (float)h[e]);
  }
  *reinterpret_cast<bf16x4*>(hi) = h;
  *reinterpret_cast<bf16x4*>(lo) = l;
}

F3_DEV f32x4 mfma_x3m(bf16x8 ah, bf16x8 al, bf16x8 bh, bf16x8 bl, f32x4 c) {
  c = mfma_bf16x(al, bh, c);
  c = mfma_bf16x(ah, bl, c);
  return mfma_bf16x(ah, bh, c);
}

// ZI (z3 output): the frame's Z rows [hi | lo] are assembled in an LDS image and leave as one
// contiguous V x 4 K CIN-byte block of 16-B pieces (the per-fragment stores wrote 32-B runs per row)
template <int CIN, bool ZI = false>
__global__ __launch_bounds__(256) void mix_fwd_x3_kernel(MixArgs a) {
  constexpr int RB = 2 * CIN + 16, XR = 32, C4 = CIN / 4;
  constexpr int PX = (18 * C4 + 255) / 256;
  extern __shared__ __attribute__((aligned(16))) char smb[];
  char* xh = smb;             // [32][RB] hi plane
  char* xl = smb + XR * RB;   // [32][RB] lo plane
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, tid = threadIdx.x;
  const int fr = lane & 15, fg = lane >> 4;
  const int K = a.K, V = a.V, KV = K * V;
  const int nx = V * C4;
  bf16x8 bhi[4], blo[4];  // B operand: lane holds k = v = 8 fg + e, n = wk = 16 nt + fr
#pragma unroll
  for (int nt = 0; nt < 4; ++nt)
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      __bf16 h, l;
      a_split(atil(a.A, K, V, 16 * nt + fr, 8 * fg + e), h, l);
      bhi[nt][e] = h;
      blo[nt][e] = l;
    }
  for (int o = V * RB + tid * 16; o < XR * RB; o += 256 * 16) {
    *reinterpret_cast<f32x4*>(xh + o) = f32x4{0.f, 0.f, 0.f, 0.f};
    *reinterpret_cast<f32x4*>(xl + o) = f32x4{0.f, 0.f, 0.f, 0.f};
  }
  f32x4 rx[PX];
  auto prefetch = [&](int f) {
    const f32x4* xg = reinterpret_cast<const f32x4*>(a.x + (size_t)f * V * CIN);
#pragma unroll
    for (int q = 0; q < PX; ++q) rx[q] = xg[min(tid + q * 256, nx - 1)];
  };
  if (blockIdx.x < a.frames) prefetch(blockIdx.x);
  for (int f = blockIdx.x; f < a.frames; f += gridDim.x) {
    __syncthreads();  // the previous frame's reads of the planes are done
#pragma unroll
    for (int q = 0; q < PX; ++q) {
      const int i = tid + q * 256;
      if (i < nx) {
        const int o = (i / C4) * RB + (i % C4) * 8;
        split4_store(rx[q], xh + o, xl + o);
      }
    }
    __syncthreads();
    if (f + (int)gridDim.x < a.frames) prefetch(f + gridDim.x);
    float* zf = a.z + (size_t)f * KV * CIN;
    char* zimg = smb + 2 * XR * RB;  // ZI: [V][2 K CIN] bf16
    for (int mt = wave; mt < CIN / 16; mt += 4) {
      const int o = (8 * fg + (fr >> 2)) * RB + 32 * mt + 8 * (fr & 3);
      const unsigned ph = (unsigned)(size_t)(mx_lds_t*)(xh + o), pl = (unsigned)(size_t)(mx_lds_t*)(xl + o);
      mx_s16x4 h0, h1, l0, l1;
      asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(h0) : "v"(ph));
      asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(h1) : "v"(ph), "n"(4 * RB));
      asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(l0) : "v"(pl));
      asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(l1) : "v"(pl), "n"(4 * RB));
      asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(h0), "+v"(h1), "+v"(l0), "+v"(l1)::"memory");
      const bf16x8 xah = __builtin_bit_cast(bf16x8, __builtin_shufflevector(h0, h1, 0, 1, 2, 3, 4, 5, 6, 7));
      const bf16x8 xal = __builtin_bit_cast(bf16x8, __builtin_shufflevector(l0, l1, 0, 1, 2, 3, 4, 5, 6, 7));
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) {
        const int wk = 16 * nt + fr;
        const f32x4 acc = mfma_x3m(xah, xal, bhi[nt], blo[nt], f32x4{0.f, 0.f, 0.f, 0.f});
        // lane holds Z[wk][c = 16 mt + 4 fg + r], r = 0..3: one 16-B piece of row wk
        if (wk < KV) {
          if (a.z3) {  // GEMM row (f, w = wk / K) of [hi | lo] over 2 K Cin, column k Cin + c
            const int w = wk / K, k = wk - w * K;
            char* row = ZI ? zimg + 2 * ((size_t)w * 2 * K * CIN + (size_t)k * CIN + 16 * mt + 4 * fg)
                           : reinterpret_cast<char*>(a.z3) +
                                 2 * (((size_t)f * V + w) * 2 * K * CIN + (size_t)k * CIN + 16 * mt + 4 * fg);
            bf16x4 h, l;
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              h[e] = (__bf16)acc[e];
              l[e] = (__bf16)(acc[e] - (float)h[e]);
            }
            *reinterpret_cast<bf16x4*>(row) = h;
            *reinterpret_cast<bf16x4*>(row + 2 * K * CIN) = l;
          } else {
            *reinterpret_cast<f32x4*>(zf + (size_t)wk * CIN + 16 * mt + 4 * fg) = acc;
          }
        }
      }
    }
    if constexpr (ZI) {  // the frame's image -> its contiguous Z rows
      __syncthreads();
      const int n16 = V * K * CIN / 4;  // V rows x 4 K CIN bytes / 16
      uint4* dst = reinterpret_cast<uint4*>(a.z3 + (size_t)f * V * 2 * K * CIN);
      const uint4* srcv = reinterpret_cast<const uint4*>(zimg);
      for (int i = tid; i < n16; i += 256) dst[i] = srcv[i];
    }
  }
}

template <int CIN, bool ACC>
__global__ __launch_bounds__(256) void mix_bwd_x3_kernel(MixArgs a) {
  constexpr int RB = 2 * CIN + 16, XR = 32, ZR = 64, C4 = CIN / 4;
  constexpr int PX = (18 * C4 + 255) / 256, PZ = (54 * C4 + 255) / 256;
  extern __shared__ __attribute__((aligned(16))) char smb[];
  char* xh = smb;                    // [32][RB]
  char* xl = xh + XR * RB;           // [32][RB]
  char* zh = xl + XR * RB;           // [64][RB]
  char* zl = zh + ZR * RB;           // [64][RB]
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, tid = threadIdx.x;
  const int fr = lane & 15, fg = lane >> 4;
  const int K = a.K, V = a.V, KV = K * V;
  const int nx = V * C4, nz = KV * C4;
  bf16x8 ahi[2][2], alo[2][2];  // A~ as the dX A operand: rows v = 16 mt + fr, k = wk = 32 ks + 8 fg + e
#pragma unroll
  for (int mt = 0; mt < 2; ++mt)
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        __bf16 h, l;
        a_split(atil(a.A, K, V, 32 * ks + 8 * fg + e, 16 * mt + fr), h, l);
        ahi[mt][ks][e] = h;
        alo[mt][ks][e] = l;
      }
  for (int o = KV * RB + tid * 16; o < ZR * RB; o += 256 * 16) {
    *reinterpret_cast<f32x4*>(zh + o) = f32x4{0.f, 0.f, 0.f, 0.f};
    *reinterpret_cast<f32x4*>(zl + o) = f32x4{0.f, 0.f, 0.f, 0.f};
  }
  f32x4 dacc[2] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};
  f32x4 rx[PX], rz[PZ];
  auto prefetch = [&](int f) {
    const f32x4* xg = reinterpret_cast<const f32x4*>(a.x + (size_t)f * V * CIN);
    const f32x4* zg = reinterpret_cast<const f32x4*>(a.z + (size_t)f * KV * CIN);
#pragma unroll
    for (int q = 0; q < PX; ++q) rx[q] = xg[min(tid + q * 256, nx - 1)];
#pragma unroll
    for (int q = 0; q < PZ; ++q) rz[q] = zg[min(tid + q * 256, nz - 1)];
  };
  if (blockIdx.x < a.frames) prefetch(blockIdx.x);
  for (int f = blockIdx.x; f < a.frames; f += gridDim.x) {
    __syncthreads();  // the previous frame's reads of the planes are done
#pragma unroll
    for (int q = 0; q < PX; ++q) {
      const int i = tid + q * 256;
      if (i < nx) {
        const int o = (i / C4) * RB + (i % C4) * 8;
        split4_store(rx[q], xh + o, xl + o);
      }
    }
#pragma unroll
    for (int q = 0; q < PZ; ++q) {
      const int i = tid + q * 256;
      if (i < nz) {
        const int o = (i / C4) * RB + (i % C4) * 8;
        split4_store(rz[q], zh + o, zl + o);
      }
    }
    __syncthreads();
    if (f + (int)gridDim.x < a.frames) prefetch(f + gridDim.x);
    // dX_f[v][c] = sum_wk A~[v][wk] dZ_f[wk][c]
    float* dxf = a.dx + (size_t)f * V * CIN;
    for (int nt = wave; nt < CIN / 16; nt += 4) {
      bf16x8 bh[2], bl[2];
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        const int o = (32 * ks + 8 * fg + (fr >> 2)) * RB + 32 * nt + 8 * (fr & 3);
        const unsigned ph = (unsigned)(size_t)(mx_lds_t*)(zh + o), pl = (unsigned)(size_t)(mx_lds_t*)(zl + o);
        mx_s16x4 h0, h1, l0, l1;
        asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(h0) : "v"(ph));
        asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(h1) : "v"(ph), "n"(4 * RB));
        asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(l0) : "v"(pl));
        asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(l1) : "v"(pl), "n"(4 * RB));
        asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(h0), "+v"(h1), "+v"(l0), "+v"(l1)::"memory");
        bh[ks] = __builtin_bit_cast(bf16x8, __builtin_shufflevector(h0, h1, 0, 1, 2, 3, 4, 5, 6, 7));
        bl[ks] = __builtin_bit_cast(bf16x8, __builtin_shufflevector(l0, l1, 0, 1, 2, 3, 4, 5, 6, 7));
      }
      f32x4 acc[2] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};
#pragma unroll
      for (int mt = 0; mt < 2; ++mt)
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) acc[mt] = mfma_x3m(ahi[mt][ks], alo[mt][ks], bh[ks], bl[ks], acc[mt]);
      float old[2][4];
#pragma unroll
      for (int mt = 0; mt < 2; ++mt)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int v = min(16 * mt + 4 * fg + r, V - 1);
          old[mt][r] = ACC ? dxf[(size_t)v * CIN + 16 * nt + fr] : 0.f;
        }
#pragma unroll
      for (int mt = 0; mt < 2; ++mt)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int v = 16 * mt + 4 * fg + r;
          if (v < V) dxf[(size_t)v * CIN + 16 * nt + fr] = acc[mt][r] + old[mt][r];
        }
    }
    // dA[v][wk] += sum_c X_f[v][c] dZ_f[wk][c]: this wave's wk tile, both v tiles
#pragma unroll 2
    for (int ks = 0; ks < CIN / 32; ++ks) {
      const int cb = (32 * ks + 8 * fg) * 2;
      const bf16x8 z_h = *reinterpret_cast<const bf16x8*>(zh + (16 * wave + fr) * RB + cb);
      const bf16x8 z_l = *reinterpret_cast<const bf16x8*>(zl + (16 * wave + fr) * RB + cb);
      const bf16x8 x0h = *reinterpret_cast<const bf16x8*>(xh + fr * RB + cb);
      const bf16x8 x0l = *reinterpret_cast<const bf16x8*>(xl + fr * RB + cb);
      const bf16x8 x1h = *reinterpret_cast<const bf16x8*>(xh + (16 + fr) * RB + cb);
      const bf16x8 x1l = *reinterpret_cast<const bf16x8*>(xl + (16 + fr) * RB + cb);
      dacc[0] = mfma_x3m(x0h, x0l, z_h, z_l, dacc[0]);
      dacc[1] = mfma_x3m(x1h, x1l, z_h, z_l, dacc[1]);
    }
  }
  float* row = a.part + (size_t)blockIdx.x * K * V * V;
#pragma unroll
  for (int mt = 0; mt < 2; ++mt)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int v = 16 * mt + 4 * fg + r, wk = 16 * wave + fr;
      if (v < V && wk < KV) {
        const int w = wk / K, k = wk - w * K;
        row[(k * V + v) * V + w] = dacc[mt][r];
      }
    }
}

// gcn bias through the graph + edge importance: db[k*C+c] += sum_w colsumAeff_k[w] G[w][c];
// dAeff[k,v,w] += sum_c b[k*C+c] G[w][c];  dE = A * dAeff. One launch: the first ceil(K C / 256)
// workgroups the bias gradient (A_eff staged in LDS with all threads, then the column sums), the
// next K V workgroups one (k, w) of dE each (the two parts are independent). Both run in the step's
// tail; the first version read A_eff column by column from L2 (18 dependent loads per thread).
__global__ __launch_bounds__(256) void gcn_bias_bwd_kernel(GcnBiasBwdArgs a) {
  __shared__ float sm[3072 + 1024];
  const int ndb = (a.K * a.C + 255) / 256, KV = a.K * a.V;
  if ((int)blockIdx.x < ndb) {
    float* Ae = sm;          // A_eff [K][V][V]
    float* cs = sm + 3072;   // colsum_k[w]
    for (int e = threadIdx.x; e < KV * a.V; e += blockDim.x) Ae[e] = a.Aeff[e];
    __syncthreads();
    for (int e = threadIdx.x; e < KV; e += blockDim.x) {
      const int k = e / a.V, w = e - k * a.V;
      float acc = 0.f;
      for (int v = 0; v < a.V; ++v) acc += Ae[(k * a.V + v) * a.V + w];
      cs[e] = acc;
    }
    __syncthreads();
    const int e = blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= a.K * a.C) return;
    const int k = e / a.C, c = e - k * a.C;
    float acc = 0.f;
#pragma unroll 6
    for (int w = 0; w < a.V; ++w) acc += cs[k * a.V + w] * a.G[w * a.C + c];
    a.db[e] += acc;
    return;
  }
  // (k, w): s = sum_c b[k*C+c] G[w][c]; dE[k][v][w] += A*(dAeff + s)
  float* red = sm;
  const int kw = blockIdx.x - ndb, k = kw / a.V, w = kw - k * a.V;
  float acc = 0.f;
  for (int c = threadIdx.x; c < a.C; c += blockDim.x) acc += a.bias[k * a.C + c] * a.G[w * a.C + c];
  acc = warp_sum(acc);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = acc;
  __syncthreads();
  const float sb = red[0] + red[1] + red[2] + red[3];
  for (int v = threadIdx.x; v < a.V; v += blockDim.x) {
    const int e = (k * a.V + v) * a.V + w;
    a.dE[e] += a.A[e] * (a.dAeff[e] + sb);
  }
}

// ----------------------------------------------------------------------------
// clip-chunk elementwise kernels. Thread t handles channel quad t % C4 of rows
// t / C4, t / C4 + RP, ... of its chunk (C4 = C/4, RP = 256/C4).
// ----------------------------------------------------------------------------
F3_DEV void chunk_rows(int TV, int chunks, int& r0, int& r1) {
  const int n = blockIdx.y, ch = blockIdx.x;
  const int per = (TV + chunks - 1) / chunks;
  r0 = n * TV + ch * per;
  r1 = min(n * TV + TV, r0 + per);
}

// reduce float4 partials over the RP row-lanes sharing a channel quad; returns in thread cq < C4
F3_DEV f32x4 quad_reduce(f32x4 v, float* lds, int C4) {
  const int tid = threadIdx.x;
  __syncthreads();
  reinterpret_cast<f32x4*>(lds)[tid] = v;
  __syncthreads();
  f32x4 r = {0.f, 0.f, 0.f, 0.f};
  if (tid < C4) {
    for (int i = tid; i < 256; i += C4) r += reinterpret_cast<f32x4*>(lds)[i];
  }
  return r;
}

// The row loops below take U = 4 rows per trip and issue all their loads before any use: at
// 2-4 workgroups per CU a one-row loop kept ~16 KB in flight per CU and ran the reduction at
// 2.2 TB/s. Rows past the chunk are clamped to its last row (loads stay in bounds, no branch
// around a load: hipcc waits vmcnt(0) per element for a conditional load) and masked out of
// the sums; their stores rewrite the last row with the same values. The residual kind and the
// pooled-gradient form are template parameters for the same reason.
constexpr int kRowU = 4;

// out = relu(bn2(h) * a[n,c] + res), res = bn_r(r) | x | 0 ; optional pooled mean
template <bool A16, int RES>
__global__ __launch_bounds__(256) void block_out_kernel(BlockArgs a) {
  __shared__ __attribute__((aligned(16))) float lds[1024];
  const int C = a.C, C4 = C / 4, RP = 256 / C4, tid = threadIdx.x;
  int r0, r1;
  chunk_rows(a.TV, a.chunks, r0, r1);
  const int n = blockIdx.y, cq = tid % C4, c0 = cq * 4;
  // the first pass's rows are loaded before the coefficient prologue (they do not depend on it)
  const int mb0 = r0 + tid / C4;
  f32x4 h[kRowU], res[kRowU];
  size_t off[kRowU];
#define F3_BO_LOADS(MB)                                                  \
  _Pragma("unroll") for (int u = 0; u < kRowU; ++u) {                    \
    off[u] = (size_t)min((MB) + u * RP, r1 - 1) * C + c0;                \
    h[u] = ld_act4<A16>(a.h, off[u]);                                    \
    if (RES == RES_CONV) res[u] = ld_act4<A16>(a.r, off[u]);             \
    else if (RES == RES_ID) res[u] = ld_act4<A16>(a.x, off[u]);          \
    else res[u] = f32x4{0.f, 0.f, 0.f, 0.f};                             \
  }
  F3_BO_LOADS(mb0)
  float sc2[4], sh2[4], scr[4], shr[4], mu[4], rs[4];
  bn_coeff4(a.bn2, c0, sc2, sh2, mu, rs);
  if (RES == RES_CONV) bn_coeff4(a.bnr, c0, scr, shr, mu, rs);
  const f32x4 av = *reinterpret_cast<const f32x4*>(a.att + (size_t)n * C + c0);
  f32x4 pool = {0.f, 0.f, 0.f, 0.f};
  for (int mb = mb0; mb < r1; mb += kRowU * RP) {
    if (mb != mb0) F3_BO_LOADS(mb)
#pragma unroll
    for (int u = 0; u < kRowU; ++u) {
      f32x4 o;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        float rv = res[u][e];
        if (RES == RES_CONV) rv = rv * scr[e] + shr[e];
        o[e] = fmaxf((h[u][e] * sc2[e] + sh2[e]) * av[e] + rv, 0.f);
      }
      st_act4<A16>(a.out, off[u], o);
      if (a.outb) {
        bf16x4 ob, lb;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          ob[e] = (__bf16)o[e];
          lb[e] = (__bf16)(o[e] - (float)ob[e]);
        }
        if (a.x3) {  // row [hi | lo] of 2C: the next block's bf16x3 residual-conv operand
          __bf16* row = reinterpret_cast<__bf16*>(a.outb) + 2 * (off[u] - c0) + c0;
          *reinterpret_cast<bf16x4*>(row) = ob;
          *reinterpret_cast<bf16x4*>(row + C) = lb;
        } else {
          *reinterpret_cast<bf16x4*>(reinterpret_cast<__bf16*>(a.outb) + off[u]) = ob;
        }
      }
      if (mb + u * RP < r1) pool += o;
    }
  }
#undef F3_BO_LOADS
  if (a.pool) {
    f32x4 r = quad_reduce(pool, lds, C4);
    if (tid < C4) {
      if (a.part) {  // this chunk's row of the pooled mean (f3_block_out sums the chunks in order)
        *reinterpret_cast<f32x4*>(a.part + ((size_t)blockIdx.x * a.N + n) * C + tid * 4) = r * a.inv_tv;
      } else {
#pragma unroll
        for (int e = 0; e < 4; ++e) atomic_add_f(a.pool + (size_t)n * C + tid * 4 + e, r[e] * a.inv_tv);
      }
    }
  }
}

// backward reductions over a block's output gradient:
//   dz = dout * (out > 0);  P1[n,c] = sum_tv dz;  P2[n,c] = sum_tv dz*xhat2
//   conv residual: R[c] += (sum dz, sum dz*xhat_r)
// DNC: the output gradient is the pooled-mean gradient dout_nc[n][c] broadcast * inv_tv
template <bool A16, int RES, bool DNC>
__global__ __launch_bounds__(256) void block_bwd_reduce_kernel(BlockArgs a) {
  __shared__ __attribute__((aligned(16))) float lds[1024];
  const int C = a.C, C4 = C / 4, RP = 256 / C4, tid = threadIdx.x;
  int r0, r1;
  chunk_rows(a.TV, a.chunks, r0, r1);
  const int n = blockIdx.y, cq = tid % C4, c0 = cq * 4;
  // the first pass's rows are loaded before the coefficient prologue (they do not depend on it)
  const int mb0 = r0 + tid / C4;
  f32x4 o[kRowU], d[kRowU], h[kRowU], rr[kRowU];
#define F3_BR_LOADS(MB)                                                          \
  _Pragma("unroll") for (int u = 0; u < kRowU; ++u) {                            \
    const size_t off = (size_t)min((MB) + u * RP, r1 - 1) * C + c0;              \
    o[u] = ld_act4<A16>(a.out, off);                                             \
    if (!DNC) d[u] = *reinterpret_cast<const f32x4*>(a.dout + off);              \
    h[u] = ld_act4<A16>(a.h, off);                                               \
    if (RES == RES_CONV) rr[u] = ld_act4<A16>(a.r, off);                         \
  }
  F3_BR_LOADS(mb0)
  float mu2[4], rs2[4], mur[4], rsr[4], sc[4], sh[4];
  bn_coeff4(a.bn2, c0, sc, sh, mu2, rs2);
  if (RES == RES_CONV) bn_coeff4(a.bnr, c0, sc, sh, mur, rsr);
  f32x4 p1 = {0, 0, 0, 0}, p2 = {0, 0, 0, 0}, q2 = {0, 0, 0, 0};
  f32x4 dbc = {0, 0, 0, 0};
  if (DNC) dbc = *reinterpret_cast<const f32x4*>(a.dout_nc + (size_t)n * C + c0) * a.inv_tv;
  for (int mb = mb0; mb < r1; mb += kRowU * RP) {
    if (mb != mb0) F3_BR_LOADS(mb)
#pragma unroll
    for (int u = 0; u < kRowU; ++u) {
      const float w = mb + u * RP < r1 ? 1.f : 0.f;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float dz = o[u][e] > 0.f ? (DNC ? dbc[e] : d[u][e]) * w : 0.f;
        p1[e] += dz;
        p2[e] += dz * ((h[u][e] - mu2[e]) * rs2[e]);
        if (RES == RES_CONV) q2[e] += dz * ((rr[u][e] - mur[e]) * rsr[e]);
      }
    }
  }
#undef F3_BR_LOADS
  // per-clip partial sums (a clip's chunks add into one row: <= chunks-way float atomics). The
  // residual BN's channel sums over all clips (sum dz = sum_n P1, sum dz*xhat_r = sum_n Q2) are
  // folded in by ca_bwd3, which walks the clips anyway: double atomics from every chunk of every
  // clip onto the same C addresses made the conv-residual form of this kernel 100 us.
  // (a.part: the chunk's partial rows, summed in chunk order by f3_block_bwd_reduce)
  // partial rows [chunk][P1 | P2 | Q2][N*C]
  const size_t pblk = (size_t)a.N * C, prow = (size_t)blockIdx.x * 3 * pblk + (size_t)n * C + tid * 4;
  f32x4 s1 = quad_reduce(p1, lds, C4);
  if (tid < C4) {
    if (a.part) {
      *reinterpret_cast<f32x4*>(a.part + prow) = s1;
    } else {
#pragma unroll
      for (int e = 0; e < 4; ++e) atomic_add_f(a.P1 + (size_t)n * C + tid * 4 + e, s1[e]);
    }
  }
  f32x4 s2 = quad_reduce(p2, lds, C4);
  if (tid < C4) {
    if (a.part) {
      *reinterpret_cast<f32x4*>(a.part + pblk + prow) = s2;
    } else {
#pragma unroll
      for (int e = 0; e < 4; ++e) atomic_add_f(a.P2 + (size_t)n * C + tid * 4 + e, s2[e]);
    }
  }
  if (RES == RES_CONV) {
    f32x4 t2 = quad_reduce(q2, lds, C4);
    if (tid < C4) {
      if (a.part) {
        *reinterpret_cast<f32x4*>(a.part + 2 * pblk + prow) = t2;
      } else {
#pragma unroll
        for (int e = 0; e < 4; ++e) atomic_add_f(a.Q2 + (size_t)n * C + tid * 4 + e, t2[e]);
      }
    }
  }
}

// dh = g2*rs2*(dz*a + e - D1/M - xhat2*D2/M);  residual: dr (conv) or dx = dz (identity)
template <bool A16, int RES, bool DNC>
__global__ __launch_bounds__(256) void block_bwd_apply_kernel(BlockArgs a) {
  const int C = a.C, C4 = C / 4, RP = 256 / C4, tid = threadIdx.x;
  const float invM = 1.f / (float)a.bn2.count;
  if (blockIdx.x == 0 && blockIdx.y == 0) {
    for (int c = tid; c < C; c += 256) {
      a.dgamma2[c] += (float)a.bn2_bsq[c];
      a.dbeta2[c] += (float)a.bn2_bsum[c];
      if (RES == RES_CONV) {
        a.dgammar[c] += (float)a.bnr_bsq[c];
        a.dbetar[c] += (float)a.bnr_bsum[c];
      }
    }
  }
  int r0, r1;
  chunk_rows(a.TV, a.chunks, r0, r1);
  const int n = blockIdx.y, cq = tid % C4, c0 = cq * 4;
  // the first pass's rows are loaded before the coefficient prologue (they do not depend on it)
  const int mb0 = r0 + tid / C4;
  f32x4 o[kRowU], d[kRowU], h[kRowU], rr[kRowU];
  size_t off[kRowU];
#define F3_BA_LOADS(MB)                                                          \
  _Pragma("unroll") for (int u = 0; u < kRowU; ++u) {                            \
    off[u] = (size_t)min((MB) + u * RP, r1 - 1) * C + c0;                        \
    o[u] = ld_act4<A16>(a.out, off[u]);                                          \
    if (!DNC) d[u] = *reinterpret_cast<const f32x4*>(a.dout + off[u]);           \
    h[u] = ld_act4<A16>(a.h, off[u]);                                            \
    if (RES == RES_CONV) rr[u] = ld_act4<A16>(a.r, off[u]);                      \
  }
  F3_BA_LOADS(mb0)
  float mu2[4], k2[4], m1[4], m2[4], rs2[4], mur[4], kr[4], n1[4], n2[4], rsr[4], sc[4], sh[4];
  double bs1[4], bs2[4], rs1[4], rsq[4];
#pragma unroll
  for (int e = 0; e < 4; ++e) {  // (loads first: see bn_coeff4)
    bs1[e] = a.bn2_bsum[c0 + e];
    bs2[e] = a.bn2_bsq[c0 + e];
    if (RES == RES_CONV) {
      rs1[e] = a.bnr_bsum[c0 + e];
      rsq[e] = a.bnr_bsq[c0 + e];
    }
  }
  bn_coeff4(a.bn2, c0, sc, sh, mu2, rs2);
  if (RES == RES_CONV) bn_coeff4(a.bnr, c0, sc, sh, mur, rsr);
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const int c = c0 + e;
    k2[e] = a.bn2.gamma[c] * rs2[e];
    m1[e] = (float)bs1[e] * invM;
    m2[e] = (float)bs2[e] * invM;
    if (RES == RES_CONV) {
      kr[e] = a.bnr.gamma[c] * rsr[e];
      n1[e] = (float)rs1[e] * invM;
      n2[e] = (float)rsq[e] * invM;
    }
  }
  const f32x4 av = *reinterpret_cast<const f32x4*>(a.att + (size_t)n * C + c0);
  const f32x4 ev = *reinterpret_cast<const f32x4*>(a.e + (size_t)n * C + c0);
  f32x4 dbc = {0, 0, 0, 0};
  if (DNC) dbc = *reinterpret_cast<const f32x4*>(a.dout_nc + (size_t)n * C + c0) * a.inv_tv;
  f32x4 sdh = {0, 0, 0, 0}, sdr = {0, 0, 0, 0};  // (dbpart) the chunk's column sums of dh / dres
  for (int mb = mb0; mb < r1; mb += kRowU * RP) {
    if (mb != mb0) F3_BA_LOADS(mb)
#pragma unroll
    for (int u = 0; u < kRowU; ++u) {
      f32x4 dh, dr;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float dz = o[u][e] > 0.f ? (DNC ? dbc[e] : d[u][e]) : 0.f;
        const float xh = (h[u][e] - mu2[e]) * rs2[e];
        dh[e] = k2[e] * (dz * av[e] + ev[e] - m1[e] - xh * m2[e]);
        if (RES == RES_CONV) {
          const float xr = (rr[u][e] - mur[e]) * rsr[e];
          dr[e] = kr[e] * (dz - n1[e] - xr * n2[e]);
        } else {
          dr[e] = dz;
        }
      }
      if (mb + u * RP < r1) {  // (rows past the chunk re-store its last row: summed once)
        sdh += dh;
        if (RES == RES_CONV) sdr += dr;
      }
      if (a.dhb) {
        bf16x4 hb, lb;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          hb[e] = (__bf16)dh[e];
          lb[e] = (__bf16)(dh[e] - (float)hb[e]);
        }
        if (a.x3) {  // row [hi | lo] of 2C (the bf16x3 tcn operand), lo = RNE bf16(dh - hi)
          __bf16* row = reinterpret_cast<__bf16*>(a.dhb) + 2 * (off[u] - c0) + c0;
          *reinterpret_cast<bf16x4*>(row) = hb;
          *reinterpret_cast<bf16x4*>(row + C) = lb;
        } else {
          *reinterpret_cast<bf16x4*>(reinterpret_cast<__bf16*>(a.dhb) + off[u]) = hb;
        }
      } else {
        *reinterpret_cast<f32x4*>(a.dh + off[u]) = dh;
      }
      if (RES == RES_CONV && a.dresb) {
        bf16x4 rb, rl;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          rb[e] = (__bf16)dr[e];
          rl[e] = (__bf16)(dr[e] - (float)rb[e]);
        }
        if (a.x3) {  // row [hi | lo] of 2C (the bf16x3 residual dgrad / wgrad operand)
          __bf16* row = reinterpret_cast<__bf16*>(a.dresb) + 2 * (off[u] - c0) + c0;
          *reinterpret_cast<bf16x4*>(row) = rb;
          *reinterpret_cast<bf16x4*>(row + C) = rl;
        } else {
          *reinterpret_cast<bf16x4*>(reinterpret_cast<__bf16*>(a.dresb) + off[u]) = rb;
        }
      } else if (RES != RES_NONE) {
        *reinterpret_cast<f32x4*>(a.dres + off[u]) = dr;
      }
    }
  }
#undef F3_BA_LOADS
  if (a.dbpart) {  // partial rows [chunk][n][C | C] (fixed-order sums in the caller's colsum)
    __shared__ __attribute__((aligned(16))) float lds[1024];
    float* row = a.dbpart + ((size_t)blockIdx.x * a.N + n) * 2 * C;
    const f32x4 s1 = quad_reduce(sdh, lds, C4);
    if (tid < C4) *reinterpret_cast<f32x4*>(row + tid * 4) = s1;
    if (RES == RES_CONV) {
      const f32x4 s2 = quad_reduce(sdr, lds, C4);
      if (tid < C4) *reinterpret_cast<f32x4*>(row + C + tid * 4) = s2;
    }
  }
}

// BN1 backward: dg = g1*rs1*(dv - S1/M - xhat1*S2/M), and the per-node column sums
// G[v][c] = sum_{n,t} dg (gcn bias / edge-importance gradients). One workgroup per
// (clip, FR frames); thread (v, 8-channel group) walks the frames, so each
// thread owns its G entries (no atomics) and a frame [V][C] is read contiguously. Each
// workgroup writes one partial row [V][C]; f3_colsum adds the rows into G.
// F3_BNBWD_FR: frames per workgroup (4 or 8; default 4), read in batches of 4 frames whose loads
// are all issued before any use
static int bn_bwd_frames() {
  static const int v = getenv("F3_BNBWD_FR") && atoi(getenv("F3_BNBWD_FR")) == 8 ? 8 : 4;
  return v;
}

// 8 activations at off: one 16-B load in the bf16 mode, two in fp32
template <bool A16>
F3_DEV void ld_act8(const void* p, size_t off, f32x4& x0, f32x4& x1) {
  if constexpr (A16) {
    const bf16x8 v = *reinterpret_cast<const bf16x8*>(reinterpret_cast<const __bf16*>(p) + off);
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      x0[e] = (float)v[e];
      x1[e] = (float)v[4 + e];
    }
  } else {
    x0 = *reinterpret_cast<const f32x4*>(reinterpret_cast<const float*>(p) + off);
    x1 = *reinterpret_cast<const f32x4*>(reinterpret_cast<const float*>(p) + off + 4);
  }
}

template <bool A16, int FR, bool HOIST = true>
__global__ __launch_bounds__(1024) void bn_bwd_apply_kernel(BnBwdArgs a) {
  __shared__ float mu[256], kk[256], m1[256], m2[256], rsv[256];
  const int C = a.C, CG = C / 8, V = a.V, T = a.TV / V, tid = threadIdx.x;
  const float invM = 1.f / (float)a.bn.count;
  const int v = tid / CG, c0 = (tid - v * CG) * 8;
  const int n = blockIdx.y, t0 = blockIdx.x * FR, t1 = min(T, t0 + FR);
  // the first batch's loads go out before the coefficient prologue (they do not depend on it), so
  // the prologue's parameter loads and barrier overlap them instead of preceding them
  f32x4 d0[4], d1[4], g0[4], g1[4];
  const int vl = min(v, V - 1);  // (threads past V load a valid row and return after the barrier)
  if (HOIST) {
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const size_t off = ((size_t)(n * T + min(t0 + u, t1 - 1)) * V + vl) * C + c0;
      ld_act8<A16>(a.dv, off, d0[u], d1[u]);
      ld_act8<A16>(a.g, off, g0[u], g1[u]);
    }
  }
  for (int c = tid; c < C; c += blockDim.x) {
    float sc, sh, rs;
    bn_coeff(a.bn, c, sc, sh, mu[c], rs);
    rsv[c] = rs;
    kk[c] = a.bn.gamma[c] * rs;
    m1[c] = (float)a.bsum[c] * invM;
    m2[c] = (float)a.bsq[c] * invM;
  }
  __syncthreads();
  if (blockIdx.x == 0 && blockIdx.y == 0) {
    for (int c = tid; c < C; c += blockDim.x) {
      a.dgamma[c] += (float)a.bsq[c];
      a.dbeta[c] += (float)a.bsum[c];
    }
  }
  if (v >= V) return;
  float acc[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) acc[e] = 0.f;
  float ck[8], cm1[8], cm2[8], cmu[8], crs[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    ck[e] = kk[c0 + e]; cm1[e] = m1[c0 + e]; cm2[e] = m2[c0 + e]; cmu[e] = mu[c0 + e]; crs[e] = rsv[c0 + e];
  }
#pragma unroll
  for (int b = 0; b < FR; b += 4) {
    // the batch's loads first (clamped to the last frame, masked out of the sums; see kRowU);
    // batch 0's went out before the prologue
    if (b > 0 || !HOIST) {
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const size_t off = ((size_t)(n * T + min(t0 + b + u, t1 - 1)) * V + v) * C + c0;
        ld_act8<A16>(a.dv, off, d0[u], d1[u]);
        ld_act8<A16>(a.g, off, g0[u], g1[u]);
      }
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int t = min(t0 + b + u, t1 - 1);
      const size_t off = ((size_t)(n * T + t) * V + v) * C + c0;
      const bool live = t0 + b + u < t1;
      float o[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float dv = e < 4 ? d0[u][e] : d1[u][e - 4];
        const float gv = e < 4 ? g0[u][e] : g1[u][e - 4];
        o[e] = ck[e] * (dv - cm1[e] - (gv - cmu[e]) * crs[e] * cm2[e]);
        if (live) acc[e] += o[e];
      }
      if (a.dgb) {
        bf16x8 ob, lb;
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          ob[e] = (__bf16)o[e];
          lb[e] = (__bf16)(o[e] - (float)ob[e]);
        }
        if (a.x3) {  // row [hi | lo] of 2C (the bf16x3 gcn dgrad / wgrad operand)
          __bf16* row = reinterpret_cast<__bf16*>(a.dgb) + 2 * (off - c0) + c0;
          *reinterpret_cast<bf16x8*>(row) = ob;
          *reinterpret_cast<bf16x8*>(row + C) = lb;
        } else {
          *reinterpret_cast<bf16x8*>(reinterpret_cast<__bf16*>(a.dgb) + off) = ob;
        }
      } else {
        *reinterpret_cast<f32x4*>(a.dg + off) = f32x4{o[0], o[1], o[2], o[3]};
        *reinterpret_cast<f32x4*>(a.dg + off + 4) = f32x4{o[4], o[5], o[6], o[7]};
      }
    }
  }
  float* row = a.Gpart + ((size_t)blockIdx.y * gridDim.x + blockIdx.x) * V * C + v * C + c0;
  *reinterpret_cast<f32x4*>(row) = f32x4{acc[0], acc[1], acc[2], acc[3]};
  *reinterpret_cast<f32x4*>(row + 4) = f32x4{acc[4], acc[5], acc[6], acc[7]};
}

// u = relu(g * scale + shift) in bf16 (BN1 + ReLU of the tcn input, bf16 mode). A thread owns
// one 8-channel group for the whole launch: the grid stride (gridDim * 256 * 8 elements) is a
// multiple of C, so its 8 scale / shift pairs are loaded once into registers; kBnReluU 16-B pieces
// are loaded before any is converted (one memory round trip per kBnReluU pieces); 4 workgroups
// per CU walk the rows so the per-workgroup coefficient prologue is paid ~4x per CU, not per piece.
constexpr int kBnReluU = 4;
template <bool G16, bool X3 = false>
__global__ __launch_bounds__(256) void bnrelu_bf16_kernel(BnReluArgs a) {
  __shared__ float scs[256], shs[256];
  for (int c = threadIdx.x; c < a.C; c += 256) {
    float mu, rs;
    bn_coeff(a.bn, c, scs[c], shs[c], mu, rs);
  }
  __syncthreads();
  const int c0 = (threadIdx.x * 8) % a.C;
  float sc[8], sh[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    sc[e] = scs[c0 + e];
    sh[e] = shs[c0 + e];
  }
  const long long total8 = (long long)a.M * a.C / 8, step = (long long)gridDim.x * 256;
  long long q = (long long)blockIdx.x * 256 + threadIdx.x;
  auto piece = [&](long long qq, f32x4& x0, f32x4& x1) __attribute__((always_inline)) {
    if constexpr (G16) {
      const bf16x8 v = *reinterpret_cast<const bf16x8*>(reinterpret_cast<const __bf16*>(a.g) + qq * 8);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        x0[e] = (float)v[e];
        x1[e] = (float)v[4 + e];
      }
    } else {
      x0 = *reinterpret_cast<const f32x4*>(a.g + qq * 8);
      x1 = *reinterpret_cast<const f32x4*>(a.g + qq * 8 + 4);
    }
  };
  auto put = [&](long long qq, const f32x4& x0, const f32x4& x1) __attribute__((always_inline)) {
    bf16x8 o, l;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const float u0 = fmaxf(x0[e] * sc[e] + sh[e], 0.f), u1 = fmaxf(x1[e] * sc[4 + e] + sh[4 + e], 0.f);
      o[e] = (__bf16)u0;
      o[4 + e] = (__bf16)u1;
      if constexpr (X3) {  // lo = RNE bf16(u - hi), exact difference (the split of gemm_x3.hip)
        l[e] = (__bf16)(u0 - (float)o[e]);
        l[4 + e] = (__bf16)(u1 - (float)o[4 + e]);
      }
    }
    if constexpr (X3) {  // row [hi | lo] of 2C (the bf16x3 tcn operand)
      const long long e0 = qq * 8, m = e0 / a.C, c = e0 - m * a.C;
      __bf16* row = reinterpret_cast<__bf16*>(a.u) + m * 2 * a.C + c;
      *reinterpret_cast<bf16x8*>(row) = o;
      *reinterpret_cast<bf16x8*>(row + a.C) = l;
    } else {
      *reinterpret_cast<bf16x8*>(reinterpret_cast<__bf16*>(a.u) + qq * 8) = o;
    }
  };
  for (; q + (kBnReluU - 1) * step < total8; q += kBnReluU * step) {
    f32x4 x0[kBnReluU], x1[kBnReluU];
#pragma unroll
    for (int u = 0; u < kBnReluU; ++u) piece(q + u * step, x0[u], x1[u]);
#pragma unroll
    for (int u = 0; u < kBnReluU; ++u) put(q + u * step, x0[u], x1[u]);
  }
  for (; q < total8; q += step) {
    f32x4 x0, x1;
    piece(q, x0, x1);
    put(q, x0, x1);
  }
}

// widths whose 8-channel groups do not tile 2048 threads (C % 8 == 0, 2048 % C != 0, e.g. 96 / 192):
// the piece's channel group is taken per piece (the pre-round-3 indexing)
template <bool G16>
__global__ __launch_bounds__(256) void bnrelu_bf16_any_kernel(BnReluArgs a) {
  __shared__ float scs[256], shs[256];
  for (int c = threadIdx.x; c < a.C; c += 256) {
    float mu, rs;
    bn_coeff(a.bn, c, scs[c], shs[c], mu, rs);
  }
  __syncthreads();
  const long long total8 = (long long)a.M * a.C / 8, step = (long long)gridDim.x * 256;
  for (long long q = (long long)blockIdx.x * 256 + threadIdx.x; q < total8; q += step) {
    const int c0 = (int)((q * 8) % a.C);
    float x[8];
    if constexpr (G16) {
      const bf16x8 v = *reinterpret_cast<const bf16x8*>(reinterpret_cast<const __bf16*>(a.g) + q * 8);
#pragma unroll
      for (int e = 0; e < 8; ++e) x[e] = (float)v[e];
    } else {
      const f32x4 x0 = *reinterpret_cast<const f32x4*>(a.g + q * 8), x1 = *reinterpret_cast<const f32x4*>(a.g + q * 8 + 4);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        x[e] = x0[e];
        x[4 + e] = x1[e];
      }
    }
    bf16x8 o;
#pragma unroll
    for (int e = 0; e < 8; ++e) o[e] = (__bf16)fmaxf(x[e] * scs[c0 + e] + shs[c0 + e], 0.f);
    *reinterpret_cast<bf16x8*>(reinterpret_cast<__bf16*>(a.u) + q * 8) = o;
  }
}

// out[c] += sum_r part[r][c], in a fixed order (the same bits every run): a workgroup owns 1024 / RG
// columns and all rows; its RG row groups (colsum_rg: fewer for few-row sums, up to 64 for tall narrow
// ones) sum rows rg, rg + RG, ... (four interleaved accumulators) and the RG partials are added in
// group order. (The
// first version split the rows over workgroups with one float atomic per column and workgroup:
// order-dependent sums.) One launch serves up to kColsumJobs independent sums (the workgroups of job
// j are blk[j] .. blk[j + 1] - 1): the reductions of one producer share a launch.
struct ColsumJobs {
  int n;
  const float* part[kColsumJobs];
  float* out[kColsumJobs];
  long long ld[kColsumJobs];
  int rows[kColsumJobs], cols[kColsumJobs], rg[kColsumJobs], blk[kColsumJobs + 1];
};
// row groups: the power of two <= rows up to 16, then up to 64 while the job has fewer than 256
// workgroups (tall, narrow sums: the BN-backward G rows are 2048 x 1152, 18 workgroups at 16 groups)
static int colsum_rg(int rows, int cols) {
  int rg = rows >= 16 ? 16 : rows >= 8 ? 8 : rows >= 4 ? 4 : rows >= 2 ? 2 : 1;
  while (rg < 64 && 2 * rg <= rows && (cols + 1024 / rg - 1) / (1024 / rg) < 256) rg *= 2;
  return rg;
}
__global__ __launch_bounds__(1024) void colsum_kernel(ColsumJobs J) {
  __shared__ float red[1024];
  int j = 0;
  while (j + 1 < J.n && (int)blockIdx.x >= J.blk[j + 1]) ++j;
  const float* part = J.part[j];
  const int rows = J.rows[j], cols = J.cols[j], RG = J.rg[j], CPB = 1024 / RG;
  const long long ld = J.ld[j];
  const int lane = threadIdx.x % CPB, rg = threadIdx.x / CPB;
  const int c = (blockIdx.x - J.blk[j]) * CPB + lane;
  float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;  // four loads in flight per thread
  if (c < cols) {
    int r = rg;
    for (; r + 3 * RG < rows; r += 4 * RG) {
      s0 += part[(size_t)r * ld + c];
      s1 += part[(size_t)(r + RG) * ld + c];
      s2 += part[(size_t)(r + 2 * RG) * ld + c];
      s3 += part[(size_t)(r + 3 * RG) * ld + c];
    }
    for (; r < rows; r += RG) s0 += part[(size_t)r * ld + c];
  }
  red[threadIdx.x] = (s0 + s1) + (s2 + s3);
  __syncthreads();
  if (rg == 0 && c < cols) {
    float t = 0.f;
    for (int g = 0; g < RG; ++g) t += red[g * CPB + lane];
    J.out[j][c] += t;
  }
}

// ----------------------------------------------------------------------------
// channel attention (stgcan.py:59-74)
// ----------------------------------------------------------------------------
F3_DEV float block_sum(float v, float* red) {
  v = warp_sum(v);
  const int w = threadIdx.x >> 6, nw = blockDim.x >> 6;
  __syncthreads();
  if ((threadIdx.x & 63) == 0) red[w] = v;
  __syncthreads();
  float s = 0.f;
  for (int i = 0; i < nw; ++i) s += red[i];
  return s;
}

// one workgroup per hidden unit j: q = W1 gap + b1, BN over the batch, ReLU.
// The batch here is only N values per unit and mean^2/var reaches ~1e3 in practice, so
// the variance is two-pass (sum (q-mean)^2), not E[q^2]-E[q]^2; the stats slots receive
// sum = N*mean and sumsq = N*(var + mean^2) in double for the running update/backward.
__global__ __launch_bounds__(256) void ca_fwd1_kernel(CaArgs a) {
  __shared__ float w1[256], sc2[256], sh2[256], red[8];
  const int j = blockIdx.x, C = a.C, H = C / 4;
  for (int c = threadIdx.x; c < C; c += 256) {
    float mu, rs;
    bn_coeff(a.bn2, c, sc2[c], sh2[c], mu, rs);
    w1[c] = a.W1[j * C + c];
  }
  __syncthreads();
  float qv[kCaMaxRowsPerThread];
  float s = 0.f;
#pragma unroll
  for (int r = 0; r < kCaMaxRowsPerThread; ++r) {
    const int n = threadIdx.x + r * 256;
    qv[r] = 0.f;
    if (n < a.N) {
      float q = a.b1[j];
      const float* gp = a.gapsum + (size_t)n * C;
      // (unrolled: the row's loads are independent of the sum; one load round trip per 8 channels)
#pragma unroll 8
      for (int c = 0; c < C; ++c) q += w1[c] * (gp[c] * a.inv_tv * sc2[c] + sh2[c]);
      a.q1[(size_t)n * H + j] = q;
      qv[r] = q;
      s += q;
    }
  }
  s = block_sum(s, red);
  const float mean_b = s / (float)a.N;
  float s2 = 0.f;
#pragma unroll
  for (int r = 0; r < kCaMaxRowsPerThread; ++r) {
    const int n = threadIdx.x + r * 256;
    if (n < a.N) s2 += (qv[r] - mean_b) * (qv[r] - mean_b);
  }
  s2 = block_sum(s2, red);
  const float var_b = s2 / (float)a.N;
  if (threadIdx.x == 0 && !a.bnca.eval) {
    a.ca_sum[j] = (double)mean_b * a.N;
    a.ca_sq[j] = ((double)var_b + (double)mean_b * mean_b) * a.N;
  }
  float mean, rstd;
  if (a.bnca.eval) {
    mean = a.bnca.rmean[j];
    rstd = rsqrtf(a.bnca.rvar[j] + kBnEps);
  } else {
    mean = mean_b;
    rstd = rsqrtf(var_b + kBnEps);
  }
  const float gm = a.bnca.gamma[j] * rstd, bt = a.bnca.beta[j] - mean * gm;
#pragma unroll
  for (int r = 0; r < kCaMaxRowsPerThread; ++r) {
    const int n = threadIdx.x + r * 256;
    if (n < a.N) a.hid[(size_t)n * H + j] = fmaxf(qv[r] * gm + bt, 0.f);
  }
}

// one workgroup per clip: a = sigmoid(W2 hid + b2)
__global__ __launch_bounds__(256) void ca_fwd2_kernel(CaArgs a) {
  __shared__ float hs[64];
  const int n = blockIdx.x, C = a.C, H = C / 4;
  if (threadIdx.x < H) hs[threadIdx.x] = a.hid[(size_t)n * H + threadIdx.x];
  __syncthreads();
  for (int c = threadIdx.x; c < C; c += 256) {
    float q = a.b2[c];
    const float* w = a.W2 + (size_t)c * H;
    for (int k = 0; k < H; ++k) q += w[k] * hs[k];
    a.att[(size_t)n * C + c] = sigmoidf_(q);
  }
}

// per clip: da = g2*P2 + b2*P1 ; dq2 = da*a*(1-a) ; dhid = W2^T dq2 ; dbn = dhid*(hid>0)
__global__ __launch_bounds__(256) void ca_bwd1_kernel(CaArgs a) {
  __shared__ float dq[256];
  const int n = blockIdx.x, C = a.C, H = C / 4;
  for (int c = threadIdx.x; c < C; c += 256) {
    const float da = a.bn2.gamma[c] * a.P2[(size_t)n * C + c] + a.bn2.beta[c] * a.P1[(size_t)n * C + c];
    const float at = a.att[(size_t)n * C + c];
    const float d = da * at * (1.f - at);
    dq[c] = d;
    a.dq2[(size_t)n * C + c] = d;
  }
  __syncthreads();
  // dhid: the four waves each take every fourth channel, partials summed through LDS
  __shared__ float part[4][64];
  const int j = threadIdx.x & 63, wv = threadIdx.x >> 6;
  if (j < H) {
    float acc0 = 0.f, acc1 = 0.f;
    int c = wv;
#pragma unroll 8
    for (; c + 4 < C; c += 8) {
      acc0 += dq[c] * a.W2[(size_t)c * H + j];
      acc1 += dq[c + 4] * a.W2[(size_t)(c + 4) * H + j];
    }
    if (c < C) acc0 += dq[c] * a.W2[(size_t)c * H + j];
    part[wv][j] = acc0 + acc1;
  }
  __syncthreads();
  if (threadIdx.x < H) {
    const float acc = (part[0][j] + part[1][j]) + (part[2][j] + part[3][j]);
    a.dbn[(size_t)n * H + j] = a.hid[(size_t)n * H + j] > 0.f ? acc : 0.f;
  }
}

// per hidden unit j: BN(batch) backward -> dq1; dW1, db1, dW2[:,j], db2, BN grads
__global__ __launch_bounds__(256) void ca_bwd2_kernel(CaArgs a) {
  __shared__ float dq1s[256], hs[256], red[8];
  __shared__ float sc2[256], sh2[256];
  const int j = blockIdx.x, C = a.C, H = C / 4, N = a.N;
  const double md = a.ca_sum[j] / N;
  const float mean = (float)md;
  const float var = (float)fmax(a.ca_sq[j] / N - md * md, 0.0);  // double: see ca_fwd1
  const float rstd = rsqrtf(var + kBnEps);
  float s1 = 0.f, s2 = 0.f;
  for (int n = threadIdx.x; n < N; n += 256) {
    const float d = a.dbn[(size_t)n * H + j];
    const float xh = (a.q1[(size_t)n * H + j] - mean) * rstd;
    s1 += d;
    s2 += d * xh;
  }
  s1 = block_sum(s1, red);
  s2 = block_sum(s2, red);
  const float k = a.bnca.gamma[j] * rstd;
  float db1 = 0.f;
  for (int n = threadIdx.x; n < N; n += 256) {
    const float d = a.dbn[(size_t)n * H + j];
    const float xh = (a.q1[(size_t)n * H + j] - mean) * rstd;
    const float dq = k * (d - s1 / N - xh * s2 / N);
    dq1s[n] = dq;
    a.dq1[(size_t)n * H + j] = dq;
    hs[n] = a.hid[(size_t)n * H + j];
    db1 += dq;
  }
  db1 = block_sum(db1, red);
  if (threadIdx.x == 0) {
    a.g_bnca_gamma[j] += s2;
    a.g_bnca_beta[j] += s1;
    a.g_b1[j] += db1;
  }
  (void)dq1s; (void)hs; (void)sc2; (void)sh2;
}

// channel-attention weight gradients as small GEMMs over the batch, one workgroup per
// (64 channels, kCaWClips clips): gW1[j][c] += sum_n dq1[n][j] gapn[n][c];
// gW2[c][j] += sum_n dq2[n][c] hid[n][j];  gb2[c] += sum_n dq2[n][c]
constexpr int kCaWClips = 8;
__global__ __launch_bounds__(256) void ca_bwd_w_kernel(CaArgs a) {
  __shared__ float dq1s[64][64];  // rows 0..31: dq1 tile, rows 32..63: hid tile; then the gW2 transpose
  float (*hs)[64] = dq1s + 32;
  const int C = a.C, H = C / 4, N = a.N;
  const int cl = threadIdx.x & 63, jg = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + cl, n0 = blockIdx.y * kCaWClips, n1 = min(N, n0 + kCaWClips);
  for (int i = threadIdx.x; i < kCaWClips * H; i += 256) {
    const int nn = i / H, j = i - nn * H, n = n0 + nn;
    dq1s[nn][j] = n < n1 ? a.dq1[(size_t)n * H + j] : 0.f;
    hs[nn][j] = n < n1 ? a.hid[(size_t)n * H + j] : 0.f;
  }
  __syncthreads();
  const bool cok = c < C;
  float sc = 0.f, sh = 0.f, mu, rs;
  if (cok) bn_coeff(a.bn2, c, sc, sh, mu, rs);
  float w1[16], w2[16], b2 = 0.f;
#pragma unroll
  for (int q = 0; q < 16; ++q) w1[q] = w2[q] = 0.f;
  // the group's gapsum / dq2 loads all go out before the sums (one round trip, not one per clip)
  float gv[kCaWClips], dv[kCaWClips];
#pragma unroll
  for (int m = 0; m < kCaWClips; ++m) {
    const bool ok = cok && n0 + m < n1;
    gv[m] = ok ? a.gapsum[(size_t)(n0 + m) * C + c] : 0.f;
    dv[m] = ok ? a.dq2[(size_t)(n0 + m) * C + c] : 0.f;
  }
#pragma unroll
  for (int m = 0; m < kCaWClips; ++m) {
    if (!cok || n0 + m >= n1) break;
    const float gap = gv[m] * a.inv_tv * sc + sh;
    const float d2 = dv[m];
    b2 += d2;
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      const int j = jg + 4 * q;
      if (j < H) {
        w1[q] += dq1s[m][j] * gap;
        w2[q] += d2 * hs[m][j];
      }
    }
  }
  // a.wpart: this clip group's partial row [g_W1 (H C) | g_W2 (C H) | g_b2 (C)], summed in group order
  float* wrow = a.wpart ? a.wpart + (size_t)blockIdx.y * (2 * H * C + C) : nullptr;
#pragma unroll
  for (int q = 0; q < 16; ++q) {
    const int j = jg + 4 * q;
    if (j < H && cok) {
      if (wrow) wrow[(size_t)j * C + c] = w1[q];
      else atomic_add_f(a.g_W1 + (size_t)j * C + c, w1[q]);  // lanes: consecutive c
    }
  }
  if (jg == 0 && cok) {
    if (wrow) wrow[2 * H * C + c] = b2;
    else atomic_add_f(a.g_b2 + c, b2);
  }
  // gW2 rows c0..c0+63 are one contiguous [64][H] block: transpose through LDS so the
  // atomics go out lane-contiguous
  float* t2 = &dq1s[0][0];  // 32*64 floats >= 64*H/2; use both arrays (64*H <= 4096)
  __syncthreads();
#pragma unroll
  for (int q = 0; q < 16; ++q) {
    const int j = jg + 4 * q;
    if (j < H) t2[cl * H + j] = w2[q];
  }
  __syncthreads();
  const int c0 = blockIdx.x * 64, nc = min(64, C - c0);
  for (int e = threadIdx.x; e < nc * H; e += 256) {
    if (wrow) wrow[H * C + (size_t)c0 * H + e] = t2[e];
    else atomic_add_f(a.g_W2 + (size_t)c0 * H + e, t2[e]);
  }
}

// per clip: dgap = W1^T dq1 ; e = dgap/TV ; BN2 backward sums D1, D2. kCaB3Clips clips per
// workgroup, their channel sums combined in registers before the (double) atomics, so each
// channel slot takes N/kCaB3Clips atomics instead of N.
constexpr int kCaB3Clips = 4;
// NCL = 1 (F3_CA_B3=1, A/B): one clip per workgroup of min(C, 256) threads - N workgroups instead
// of N / 4 with 3/4 of the threads idle at C = 64 (the kernel is a latency chain per thread)
template <int NCL>
__global__ __launch_bounds__(256) void ca_bwd3_kernel(CaArgs a) {
  constexpr int kCaB3Clips = NCL;
  __shared__ float dq[kCaB3Clips][64];
  const int n0 = blockIdx.x * kCaB3Clips, C = a.C, H = C / 4, N = a.N;
  for (int i = threadIdx.x; i < kCaB3Clips * H; i += blockDim.x) {
    const int nn = i / H, k = i - nn * H;
    dq[nn][k] = n0 + nn < N ? a.dq1[(size_t)(n0 + nn) * H + k] : 0.f;
  }
  __syncthreads();
  for (int c = threadIdx.x; c < C; c += blockDim.x) {
    float sc, sh, mu, rs;
    bn_coeff(a.bn2, c, sc, sh, mu, rs);
    // W1's column c read once for all the workgroup's clips (the clip loop outside re-read it
    // per clip: 4 dependent 64-long load chains); per clip the k order is unchanged
    float dgs[kCaB3Clips];
#pragma unroll
    for (int nn = 0; nn < kCaB3Clips; ++nn) dgs[nn] = 0.f;
#pragma unroll 8
    for (int k = 0; k < H; ++k) {
      const float wk = a.W1[(size_t)k * C + c];
#pragma unroll
      for (int nn = 0; nn < kCaB3Clips; ++nn) dgs[nn] += dq[nn][k] * wk;
    }
    double s1 = 0.0, s2 = 0.0, r1 = 0.0, r2 = 0.0;
#pragma unroll
    for (int nn = 0; nn < kCaB3Clips; ++nn) {
      if (n0 + nn >= N) break;
      const float dg = dgs[nn];
      const size_t o = (size_t)(n0 + nn) * C + c;
      a.e[o] = dg * a.inv_tv;
      const float at = a.att[o];
      const float xsum = (a.gapsum[o] - mu / a.inv_tv) * rs;  // sum_tv xhat2
      s1 += (double)(at * a.P1[o] + dg);
      s2 += (double)(at * a.P2[o] + dg * a.inv_tv * xsum);
      if (a.bnr_bsum) {  // conv residual BN: channel sums of dz and dz*xhat_r over the clips
        r1 += (double)a.P1[o];
        r2 += (double)a.Q2[o];
      }
    }
    atomic_add_d(a.bn2_bsum + c, s1);
    atomic_add_d(a.bn2_bsq + c, s2);
    if (a.bnr_bsum) {
      atomic_add_d(a.bnr_bsum + c, r1);
      atomic_add_d(a.bnr_bsq + c, r2);
    }
  }
}

// ----------------------------------------------------------------------------
// Channel attention with the loads of each phase issued up front (N <= 256, C % 64 == 0). The kernels
// above walk 16-256 long load chains per thread (a W1 / W2 row or column, a gapsum row, one element
// per iteration): on the main chains the five of them cost ~43 us per layer and stream in the serial
// step profile (ca_bwd3 alone 16.8 us), latency, not bytes. Here each thread's loads go out together
// and the sums run from registers / LDS; 1024-thread workgroups, four lanes per row (64-B pieces).
// ca_bwd3x keeps ca_bwd3's summation order (k sequential per clip, the clips of a workgroup added in
// clip order before its double atomics).
// ----------------------------------------------------------------------------
F3_DEV float block_sum16(float v, float* red) {  // 1024 threads
  v = warp_sum(v);
  const int w = threadIdx.x >> 6;
  __syncthreads();
  if ((threadIdx.x & 63) == 0) red[w] = v;
  __syncthreads();
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < 16; ++i) s += red[i];
  return s;
}

// one workgroup per hidden unit j; thread (n, p): clip n, channels 4p + 16i (float4 i)
__global__ __launch_bounds__(1024) void ca_fwd1x_kernel(CaArgs a) {
  __shared__ __attribute__((aligned(16))) float w1[256], sc2[256], sh2[256];
  __shared__ float red[16];
  const int j = blockIdx.x, C = a.C, H = C / 4, tid = threadIdx.x;
  const int n = tid >> 2, p = tid & 3, nv = C / 16;
  const bool live = n < a.N;
  f32x4 gv[16];
  const float* gp = a.gapsum + (size_t)(live ? n : 0) * C + 4 * p;
#pragma unroll
  for (int i = 0; i < 16; ++i)
    if (i < nv) gv[i] = *reinterpret_cast<const f32x4*>(gp + 16 * i);
  for (int c = tid; c < C; c += 1024) {
    float mu, rs;
    bn_coeff(a.bn2, c, sc2[c], sh2[c], mu, rs);
    w1[c] = a.W1[(size_t)j * C + c];
  }
  __syncthreads();
  float q = 0.f;
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    if (i >= nv) continue;
    const int c = 4 * p + 16 * i;
#pragma unroll
    for (int e = 0; e < 4; ++e) q += w1[c + e] * (gv[i][e] * a.inv_tv * sc2[c + e] + sh2[c + e]);
  }
  q += __shfl_xor(q, 1, 64);
  q += __shfl_xor(q, 2, 64);
  q += a.b1[j];
  const bool own = live && p == 0;
  const float s = block_sum16(own ? q : 0.f, red);
  const float mean_b = s / (float)a.N;
  const float s2 = block_sum16(own ? (q - mean_b) * (q - mean_b) : 0.f, red);
  const float var_b = s2 / (float)a.N;
  if (tid == 0 && !a.bnca.eval) {
    a.ca_sum[j] = (double)mean_b * a.N;
    a.ca_sq[j] = ((double)var_b + (double)mean_b * mean_b) * a.N;
  }
  float mean, rstd;
  if (a.bnca.eval) {
    mean = a.bnca.rmean[j];
    rstd = rsqrtf(a.bnca.rvar[j] + kBnEps);
  } else {
    mean = mean_b;
    rstd = rsqrtf(var_b + kBnEps);
  }
  const float gm = a.bnca.gamma[j] * rstd, bt = a.bnca.beta[j] - mean * gm;
  if (own) {
    a.q1[(size_t)n * H + j] = q;
    a.hid[(size_t)n * H + j] = fmaxf(q * gm + bt, 0.f);
  }
}

// one workgroup per clip: att = sigmoid(W2 hid + b2); thread (c, p): W2 row c, hidden units 4p + 16i
__global__ __launch_bounds__(1024) void ca_fwd2x_kernel(CaArgs a) {
  __shared__ float hs[64];
  const int n = blockIdx.x, C = a.C, H = C / 4, tid = threadIdx.x;
  const int c = tid >> 2, p = tid & 3, nv = H / 16;
  const bool live = c < C;
  f32x4 wv[4];
  const float* w = a.W2 + (size_t)(live ? c : 0) * H + 4 * p;
#pragma unroll
  for (int i = 0; i < 4; ++i)
    if (i < nv) wv[i] = *reinterpret_cast<const f32x4*>(w + 16 * i);
  if (tid < H) hs[tid] = a.hid[(size_t)n * H + tid];
  __syncthreads();
  float q = 0.f;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    if (i >= nv) continue;
#pragma unroll
    for (int e = 0; e < 4; ++e) q += wv[i][e] * hs[4 * p + 16 * i + e];
  }
  q += __shfl_xor(q, 1, 64);
  q += __shfl_xor(q, 2, 64);
  if (live && p == 0) a.att[(size_t)n * C + c] = sigmoidf_(a.b2[c] + q);
}

// sum of `rows` (<= 16) partial rows `ld` floats apart in colsum_kernel's order for such a column (row
// groups of the largest power of two <= rows, each group's rows in order, the groups in order, onto 0)
F3_DEV float colsum_few(const float* p, long long ld, int rows) {
  const int RG = rows >= 16 ? 16 : rows >= 8 ? 8 : rows >= 4 ? 4 : rows >= 2 ? 2 : 1;
  float t = 0.f;
  for (int g = 0; g < RG; ++g) {
    float s0 = 0.f;
    for (int r = g; r < rows; r += RG) s0 += p[(size_t)r * ld];
    t += (s0 + 0.f) + (0.f + 0.f);
  }
  return 0.f + t;
}

// per clip: dq2 = (g2 P2 + b2 P1) a (1 - a); dbn = (W2^T dq2) (hid > 0); thread (r, j) sums channels
// r + 16i of hidden unit j, the 16 partials added in r order
__global__ __launch_bounds__(1024) void ca_bwd1x_kernel(CaArgs a) {
  __shared__ float dq[256];
  __shared__ float part[16][64];
  const int n = blockIdx.x, C = a.C, H = C / 4, tid = threadIdx.x;
  const int j = tid & 63, r = tid >> 6, nci = C / 16;
  const bool jl = j < H;
  float wv[16];
#pragma unroll
  for (int i = 0; i < 16; ++i)
    if (i < nci) wv[i] = jl ? a.W2[(size_t)(r + 16 * i) * H + j] : 0.f;
  if (tid < C) {
    const size_t o = (size_t)n * C + tid;
    float p1, p2;
    if (a.bpart) {  // this clip's block sums from block_bwd_reduce's partial rows (no colsum launch)
      const long long nc = (long long)a.N * C, ld = 3 * nc;
      p1 = colsum_few(a.bpart + o, ld, a.bchunks);
      p2 = colsum_few(a.bpart + nc + o, ld, a.bchunks);
      const_cast<float*>(a.P1)[o] = p1;
      const_cast<float*>(a.P2)[o] = p2;
      if (a.bnr_bsum) const_cast<float*>(a.Q2)[o] = colsum_few(a.bpart + 2 * nc + o, ld, a.bchunks);
    } else {
      p1 = a.P1[o];
      p2 = a.P2[o];
    }
    const float da = a.bn2.gamma[tid] * p2 + a.bn2.beta[tid] * p1;
    const float at = a.att[o];
    const float d = da * at * (1.f - at);
    dq[tid] = d;
    a.dq2[o] = d;
  }
  __syncthreads();
  float acc = 0.f;
#pragma unroll
  for (int i = 0; i < 16; ++i)
    if (i < nci) acc += dq[r + 16 * i] * wv[i];
  part[r][j] = acc;
  __syncthreads();
  if (tid < H) {
    float t = 0.f;
#pragma unroll
    for (int q = 0; q < 16; ++q) t += part[q][tid];
    a.dbn[(size_t)n * H + tid] = a.hid[(size_t)n * H + tid] > 0.f ? t : 0.f;
  }
}

// per 4 clips: dgap = W1^T dq1, e = dgap / TV, BN2 (and residual BN) backward sums; thread (clip nn, c).
// FUSE2: ca_bwd2's attention-BN backward folded in. Every workgroup sums s1 = sum_n dbn and
// s2 = sum_n dbn xhat over all clips for each hidden unit (thread (r, j): clips r + 16i; the 16 partials
// added in r order), forms its own clips' dq1 rows (written for ca_bwd_w), and workgroup 0 adds the
// attention BN's gamma / beta and b1 gradients: one main-chain launch less per layer.
template <bool FUSE2>
__global__ __launch_bounds__(1024) void ca_bwd3x_kernel(CaArgs a) {
  __shared__ float dq[4][64];
  __shared__ double sred[4][4][256];  // [sum][clip][channel]
  const int n0 = blockIdx.x * 4, C = a.C, H = C / 4, N = a.N, tid = threadIdx.x;
  const int nn = tid >> 8, c = tid & 255, n = n0 + nn;
  const bool cl = c < C, live = cl && n < N;
  // this thread's (clip, channel) operands and BN2 coefficients: loaded first, so their round trips
  // overlap the FUSE2 part's loads and barriers (loads do not move across a barrier by themselves)
  const size_t o = (size_t)(live ? n : 0) * C + (cl ? c : 0);
  const float at = a.att[o], p1 = a.P1[o], p2 = a.P2[o], gs = a.gapsum[o];
  const float q2 = a.bnr_bsum ? a.Q2[o] : 0.f;
  float bsc = 0.f, bsh = 0.f, bmu = 0.f, brs = 0.f;
  if (live) bn_coeff(a.bn2, c, bsc, bsh, bmu, brs);
  if constexpr (FUSE2) {
    __shared__ float ps[2][16][64];
    __shared__ float s12[2][64], kk[64], mu[64], rsd[64];
    const int j = tid & 63, r = tid >> 6;
    const bool jl = j < H;
    float mean = 0.f, rstd = 0.f;
    if (jl) {
      const double md = a.ca_sum[j] / N;
      mean = (float)md;
      const float var = (float)fmax(a.ca_sq[j] / N - md * md, 0.0);  // double: see ca_fwd1
      rstd = rsqrtf(var + kBnEps);
    }
    float dv[16], xv[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int m = r + 16 * i;
      const bool ok = jl && m < N;
      dv[i] = ok ? a.dbn[(size_t)m * H + j] : 0.f;
      xv[i] = ok ? a.q1[(size_t)m * H + j] : 0.f;
    }
    float t1 = 0.f, t2 = 0.f;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      xv[i] = (xv[i] - mean) * rstd;
      t1 += dv[i];
      t2 += dv[i] * xv[i];
    }
    ps[0][r][j] = t1;
    ps[1][r][j] = t2;
    if (r == 0) {
      kk[j] = jl ? a.bnca.gamma[j] * rstd : 0.f;
      mu[j] = mean;
      rsd[j] = rstd;
    }
    __syncthreads();
    if (tid < 64) {
      float u1 = 0.f, u2 = 0.f;
#pragma unroll
      for (int g = 0; g < 16; ++g) {
        u1 += ps[0][g][tid];
        u2 += ps[1][g][tid];
      }
      s12[0][tid] = u1;
      s12[1][tid] = u2;
    }
    __syncthreads();
    if (tid < 4 * H) {  // this workgroup's clips' dq1 rows
      const int m = tid / H, k = tid - m * H;
      float v = 0.f;
      if (n0 + m < N) {
        const size_t q = (size_t)(n0 + m) * H + k;
        const float xh = (a.q1[q] - mu[k]) * rsd[k];
        v = kk[k] * (a.dbn[q] - s12[0][k] / N - xh * s12[1][k] / N);
        a.dq1[q] = v;
      }
      dq[m][k] = v;
    }
    if (blockIdx.x == 0) {  // (uniform) the attention BN's gamma / beta and b1 gradients
      const float S1 = s12[0][j], S2 = s12[1][j], kj = kk[j];
      float t3 = 0.f;
#pragma unroll
      for (int i = 0; i < 16; ++i)
        if (jl && r + 16 * i < N) t3 += kj * (dv[i] - S1 / N - xv[i] * S2 / N);
      ps[0][r][j] = t3;  // (ps[0] was last read before the barrier above)
      __syncthreads();
      if (tid < H) {
        float u = 0.f;
#pragma unroll
        for (int g = 0; g < 16; ++g) u += ps[0][g][tid];
        a.g_bnca_gamma[tid] += s12[1][tid];
        a.g_bnca_beta[tid] += s12[0][tid];
        a.g_b1[tid] += u;
      }
    }
  }
  float wk[64];
#pragma unroll
  for (int k = 0; k < 64; ++k)
    if (k < H) wk[k] = cl ? a.W1[(size_t)k * C + c] : 0.f;
  if (!FUSE2 && tid < 4 * H) {
    const int m = tid / H, k = tid - m * H;
    dq[m][k] = n0 + m < N ? a.dq1[(size_t)(n0 + m) * H + k] : 0.f;
  }
  __syncthreads();
  double s1 = 0.0, s2 = 0.0, r1 = 0.0, r2 = 0.0;
  if (live) {
    float dg = 0.f;
#pragma unroll
    for (int k = 0; k < 64; ++k)
      if (k < H) dg += dq[nn][k] * wk[k];
    a.e[o] = dg * a.inv_tv;
    const float xsum = (gs - bmu / a.inv_tv) * brs;  // sum_tv xhat2
    s1 = (double)(at * p1 + dg);
    s2 = (double)(at * p2 + dg * a.inv_tv * xsum);
    r1 = (double)p1;
    r2 = (double)q2;
  }
  sred[0][nn][c] = s1;
  sred[1][nn][c] = s2;
  sred[2][nn][c] = r1;
  sred[3][nn][c] = r2;
  __syncthreads();
  if (nn == 0 && cl) {
    double t1 = 0.0, t2 = 0.0, u1 = 0.0, u2 = 0.0;
#pragma unroll
    for (int m = 0; m < 4; ++m) {
      if (n0 + m >= N) break;
      t1 += sred[0][m][c];
      t2 += sred[1][m][c];
      u1 += sred[2][m][c];
      u2 += sred[3][m][c];
    }
    atomic_add_d(a.bn2_bsum + c, t1);
    atomic_add_d(a.bn2_bsq + c, t2);
    if (a.bnr_bsum) {
      atomic_add_d(a.bnr_bsum + c, u1);
      atomic_add_d(a.bnr_bsq + c, u2);
    }
  }
}

// ----------------------------------------------------------------------------
// BatchNorm running statistics (momentum 0.1, unbiased variance), all BNs at once
// ----------------------------------------------------------------------------
__global__ void bn_running_kernel(BnRunTable t) {
  const BnRunJob j = t.jobs[blockIdx.x];
  const double cnt = j.count;
  for (int c = threadIdx.x; c < j.C; c += blockDim.x) {
    const double m = j.sum[c] / cnt;
    double v = j.sumsq[c] / cnt - m * m;
    if (v < 0) v = 0;
    const double vu = cnt > 1 ? v * cnt / (cnt - 1) : v;
    j.rmean[c] = (float)(0.9 * j.rmean[c] + 0.1 * m);
    j.rvar[c] = (float)(0.9 * j.rvar[c] + 0.1 * vu);
  }
  if (threadIdx.x == 0 && j.nbt) j.nbt[0] += 1;
}

}  // namespace f3

using namespace f3;

int f3_prep(const PrepTable& t, hipStream_t s) {
  if (t.n <= 0) return F3_OK;
  if (t.n > kMaxPrepJobs) return F3_EINVAL;
  PrepLaunch L;
  L.t = t;
  L.boff[0] = 0;
  // items per thread (F3_PREP_IPT, default 4; 1..2048 blocks per job). The graph-mixed-bias job's
  // items are 2*K*V loads each: one item per thread (at four, its 3,584 items on four workgroups
  // were the launch's longest chain). 1 or 2 items per thread for the rest measured no faster (1:
  // +0.8 % step, the extra workgroups), r06_prep_ipt_ab.txt.
  static const int ipt = [] {
    const char* e = std::getenv("F3_PREP_IPT");
    const int v = e ? std::atoi(e) : 4;
    return v >= 1 && v <= 16 ? v : 4;
  }();
  for (int j = 0; j < t.n; ++j) {
    const long long items = t.jobs[j].bf16 == 4 ? t.jobs[j].n / 2 : t.jobs[j].n;
    const long long per = 256LL * (t.jobs[j].type == PREP_GCN_BIAS ? 1 : ipt);
    L.boff[j + 1] = L.boff[j] + (int)std::min<long long>(2048, std::max<long long>(1, (items + per - 1) / per));
  }
  hipLaunchKernelGGL(prep_kernel, dim3(L.boff[t.n]), dim3(256), 0, s, L);
  F3_LAUNCH_CHECK();
  return F3_OK;
}

int f3_databn_fwd(const DataBnArgs* a, hipStream_t s) {
  if (!a->bn.eval) {
    hipLaunchKernelGGL(databn_stats_kernel, dim3(a->V * a->C), dim3(1024), 0, s, *a);
    F3_LAUNCH_CHECK();
  }
  const int total = a->N * a->T * a->V * a->C;
  hipLaunchKernelGGL(databn_apply_kernel, dim3(min(2048, (total + 255) / 256)), dim3(256), 0, s, *a);
  F3_LAUNCH_CHECK();
  return F3_OK;
}

int f3_databn_bwd(const DataBnArgs* a, hipStream_t s) {
  hipLaunchKernelGGL(databn_bwd_kernel, dim3(a->V * a->C), dim3(256), 0, s, *a);
  F3_LAUNCH_CHECK();
  return F3_OK;
}

static size_t mix_lds(const MixArgs& a, bool bwd) {
  size_t f = (size_t)a.K * a.V * a.V + (size_t)a.V * a.Cin;
  if (bwd) f += (size_t)a.V * a.K * a.Cin;
  return f * sizeof(float);
}

// kernels with no static LDS may take up to the full 160 KiB as dynamic LDS (F3_LDS_LIMIT: once per
// kernel, a refusal returns F3_EHIP)
#define F3_BIG_LDS(fn) F3_LDS_LIMIT(fn, 160 * 1024)

static size_t mix_lds_bwd2(const MixArgs& a) {
  return sizeof(float) * std::max((size_t)(2 * a.V + a.K * a.V) * (a.Cin + 20), (size_t)a.K * a.V * a.V);
}

template <int KS, int CIN, bool XB>
static int launch_mix_fwd(const MixArgs* a, hipStream_t s) {
  F3_BIG_LDS((mix_fwd_wave_kernel<KS, CIN, XB>));
  // a wave per frame (the workgroup-per-frame mix_fwd_lds_kernel measured slower; a bf16-MFMA form
  // with 64-channel groups assembled in LDS measured slower too: 31 / 34 / 29 us vs 25 / 25 / 25 at
  // the three layer shapes: the fp32 MFMA work is not what bounds these kernels)
  const size_t per_wave = 18 * (CIN + (XB ? 8 : 4)) * (XB ? 2 : 4) + 64 * 20 * 4;
  const int grid = std::max(1, std::min((a->frames + 3) / 4, 1024));
  const size_t lds = 4 * per_wave + sizeof(float) * a->K * a->V * a->V;
  hipLaunchKernelGGL((mix_fwd_wave_kernel<KS, CIN, XB>), dim3(grid), dim3(256), lds, s, *a);
  F3_LAUNCH_CHECK();
  return F3_OK;
}

template <int CIN>
static int mix_fwd_ks(const MixArgs* a, hipStream_t s) {
  switch ((a->V + 3) / 4) {
    case 4: return a->x16 ? launch_mix_fwd<4, CIN, true>(a, s) : launch_mix_fwd<4, CIN, false>(a, s);
    case 5: return a->x16 ? launch_mix_fwd<5, CIN, true>(a, s) : launch_mix_fwd<5, CIN, false>(a, s);
    default: return -1;
  }
}

// LDS path: V in {13..18}, K <= 3, Cin in {64, 128, 256}; else the generic kernel
bool f3_mix_lds_ok(int K, int V, int Cin) {
  return (Cin == 64 || Cin == 128 || Cin == 256) && K <= 3 && V >= 13 && V <= 18;
}
static bool mix_lds_ok(const MixArgs& a) { return f3_mix_lds_ok(a.K, a.V, a.Cin); }

// bf16 mode (x and Z bf16): the bf16-MFMA kernel; F3_MIX_FWD_BF16=0 keeps the fp32-MFMA kernels
template <int CIN>
static int launch_mix_fwd_bf16(const MixArgs* a, hipStream_t s) {
  constexpr size_t lds = (size_t)96 * (2 * CIN + 16);
  F3_LDS_LIMIT(mix_fwd_bf16_kernel<CIN>, lds);
  static const int slots = [] {
    int per_cu = 0, dev = 0, cus = 256;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, (const void*)mix_fwd_bf16_kernel<CIN>, 256, lds) !=
            hipSuccess || per_cu < 1)
      per_cu = 1;
    if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    (void)hipGetLastError();
    return per_cu * cus;
  }();
  const int grid = std::max(1, std::min(a->frames, slots));
  hipLaunchKernelGGL(mix_fwd_bf16_kernel<CIN>, dim3(grid), dim3(256), lds, s, *a);
  F3_LAUNCH_CHECK();
  return F3_OK;
}

// bf16x3 mode: grid = one round of resident workgroups (occupancy at the kernel's LDS)
template <class KERN>
static int resident_slots(KERN k, size_t lds) {
  int per_cu = 0, dev = 0, cus = 256;
  (void)hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, (const void*)k, 256, lds) != hipSuccess || per_cu < 1)
    per_cu = 1;
  if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  (void)hipGetLastError();
  return per_cu * cus;
}
template <int CIN>
static size_t mix_x3_lds_fwd() { return (size_t)64 * (2 * CIN + 16); }
template <int CIN>
static size_t mix_x3_lds_bwd() { return (size_t)192 * (2 * CIN + 16); }
template <int CIN>
static int launch_mix_fwd_x3(const MixArgs* a, hipStream_t s) {
  // z3 output through the frame image (per-fragment stores measured 10.39 vs 10.22 ms/step,
  // profiles/r04_zimg_segminor_ab.txt)
  if (a->z3) {
    const size_t lds = mix_x3_lds_fwd<CIN>() + (size_t)a->V * 4 * a->K * CIN;
    if (lds > 160 * 1024) return F3_EINVAL;
    static size_t lds0 = lds;
    F3_BIG_LDS((mix_fwd_x3_kernel<CIN, true>));
    static const int slots = resident_slots(mix_fwd_x3_kernel<CIN, true>, lds0);
    const int grid = std::max(1, std::min(a->frames, lds == lds0 ? slots : 256));
    hipLaunchKernelGGL((mix_fwd_x3_kernel<CIN, true>), dim3(grid), dim3(256), lds, s, *a);
    F3_LAUNCH_CHECK();
    return F3_OK;
  }
  static const int slots = resident_slots(mix_fwd_x3_kernel<CIN>, mix_x3_lds_fwd<CIN>());
  const int grid = std::max(1, std::min(a->frames, slots));
  hipLaunchKernelGGL(mix_fwd_x3_kernel<CIN>, dim3(grid), dim3(256), mix_x3_lds_fwd<CIN>(), s, *a);
  F3_LAUNCH_CHECK();
  return F3_OK;
}
template <int CIN>
static int mix_bwd_x3_grid(const MixArgs* a) {
  static const int slots = [] {
    (void)resident_slots(mix_bwd_x3_kernel<CIN, false>, mix_x3_lds_bwd<CIN>());
    return resident_slots(mix_bwd_x3_kernel<CIN, true>, mix_x3_lds_bwd<CIN>());
  }();
  return std::max(1, std::min(std::min(a->frames, 768), slots));
}
template <int CIN>
static int launch_mix_bwd_x3(const MixArgs* a, hipStream_t s) {
  const int grid = mix_bwd_x3_grid<CIN>(a);
  if (a->accumulate)
    hipLaunchKernelGGL((mix_bwd_x3_kernel<CIN, true>), dim3(grid), dim3(256), mix_x3_lds_bwd<CIN>(), s, *a);
  else
    hipLaunchKernelGGL((mix_bwd_x3_kernel<CIN, false>), dim3(grid), dim3(256), mix_x3_lds_bwd<CIN>(), s, *a);
  F3_LAUNCH_CHECK();
  if (a->no_colsum) return F3_OK;
  return f3_colsum(a->part, grid, a->K * a->V * a->V, a->dA, s);
}
static bool mix_x3_ok(const MixArgs& a) {
  return a.x3 && !a.x16 && !a.zb && !a.dzb && (a.Cin == 64 || a.Cin == 128 || a.Cin == 256) && a.K * a.V <= 64 &&
         a.V <= 32;
}

// bf16x3 operand rows: out[r] = [hi | lo] of x[r] (2C bf16), hi = RNE bf16(x),
// lo = RNE bf16(x - hi). One thread per 4 channels: a 16-B read, two 8-B writes.
__global__ __launch_bounds__(256) void split_x3cat_kernel(const float* __restrict__ x, __bf16* __restrict__ out,
                                                          long long n4, int C4) {
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n4; i += (long long)gridDim.x * 256) {
    const long long r = i / C4;
    const int c = (int)(i - r * C4) * 4, C = C4 * 4;
    const f32x4 v = reinterpret_cast<const f32x4*>(x)[i];
    bf16x4 h, l;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      h[e] = (__bf16)v[e];
      l[e] = (__bf16)(v[e] - (float)h[e]);
    }
    __bf16* row = out + r * 2 * C + c;
    *reinterpret_cast<bf16x4*>(row) = h;
    *reinterpret_cast<bf16x4*>(row + C) = l;
  }
}

int f3_split_x3(const float* x, unsigned short* out, long long rows, int C, hipStream_t s) {
  if (C % 4 || rows < 0) return F3_EINVAL;
  const long long n4 = rows * (C / 4);
  if (n4 == 0) return F3_OK;
  const int grid = (int)std::min<long long>((n4 + 255) / 256, 8192);
  hipLaunchKernelGGL(split_x3cat_kernel, dim3(grid), dim3(256), 0, s, x, reinterpret_cast<__bf16*>(out), n4, C / 4);
  F3_LAUNCH_CHECK();
  return F3_OK;
}

bool f3_mix_x3_ok(int K, int V, int Cin) {
  MixArgs m;
  std::memset(&m, 0, sizeof(m));
  m.K = K; m.V = V; m.Cin = Cin; m.x3 = 1;
  return mix_x3_ok(m);
}

int f3_mix_fwd(const MixArgs* a, hipStream_t s) {
  if (a->z3 && !(a->x3 && mix_x3_ok(*a))) return F3_EINVAL;  // (only the split-bf16 kernel writes z3)
  if (a->x3 && mix_x3_ok(*a)) {  // (the first block's Cin = 2 / 3 mix stays on the fp32 kernels)
    if (a->frames <= 0) return F3_OK;
    return a->Cin == 64 ? launch_mix_fwd_x3<64>(a, s) : a->Cin == 128 ? launch_mix_fwd_x3<128>(a, s)
                                                         : launch_mix_fwd_x3<256>(a, s);
  }
  if (mix_lds_ok(*a) && a->x16 && a->zb && a->K * a->V <= 64 && a->V <= 32) {
    if (a->frames <= 0) return F3_OK;
    return a->Cin == 64 ? launch_mix_fwd_bf16<64>(a, s) : a->Cin == 128 ? launch_mix_fwd_bf16<128>(a, s)
                                                           : launch_mix_fwd_bf16<256>(a, s);
  }
  if (mix_lds_ok(*a)) {
    const int r = a->Cin == 64 ? mix_fwd_ks<64>(a, s) : a->Cin == 128 ? mix_fwd_ks<128>(a, s) : mix_fwd_ks<256>(a, s);
    if (r >= 0) return r;
  }
  F3_BIG_LDS(mix_fwd_kernel);
  if (mix_lds(*a, false) > 160 * 1024) return F3_EINVAL;
  const int grid = min(a->frames, 2048);
  hipLaunchKernelGGL(mix_fwd_kernel, dim3(grid), dim3(256), mix_lds(*a, false), s, *a);
  F3_LAUNCH_CHECK();
  return F3_OK;
}

template <int KS, int CIN, bool ZB16>
static int launch_mix_bwd(const MixArgs* a, hipStream_t s) {
  F3_BIG_LDS((mix_bwd_lds_kernel<KS, CIN, ZB16, false>));
  F3_BIG_LDS((mix_bwd_lds_kernel<KS, CIN, ZB16, true>));
  const int grid = std::min(a->frames, 768);  // resident workgroups loop over frames
  if (a->accumulate)
    hipLaunchKernelGGL((mix_bwd_lds_kernel<KS, CIN, ZB16, true>), dim3(grid), dim3(256), mix_lds_bwd2(*a), s, *a);
  else
    hipLaunchKernelGGL((mix_bwd_lds_kernel<KS, CIN, ZB16, false>), dim3(grid), dim3(256), mix_lds_bwd2(*a), s, *a);
  F3_LAUNCH_CHECK();
  if (a->no_colsum) return F3_OK;
  return f3_colsum(a->part, grid, a->K * a->V * a->V, a->dA, s);
}

// bf16 mode: the bf16-MFMA kernel (F3_MIX_BWD_BF16=0: the fp32 16x16x4 kernel). Grid = one
// round of resident workgroups (each loops over frames with its next frame prefetched), capped at
// 768 partial rows.
static bool mix_bwd_bf16_on() {
  static const bool v = !getenv("F3_MIX_BWD_BF16") || atoi(getenv("F3_MIX_BWD_BF16")) != 0;
  return v;
}
template <int CIN>
static size_t mix_bf16_lds() { return (size_t)96 * (2 * CIN + 16); }
template <int CIN>
static int mix_bwd_bf16_grid(const MixArgs* a) {
  F3_LDS_LIMIT((mix_bwd_bf16_kernel<CIN, false>), mix_bf16_lds<CIN>());
  F3_LDS_LIMIT((mix_bwd_bf16_kernel<CIN, true>), mix_bf16_lds<CIN>());
  static const int slots = [] {
    int per_cu = 0, dev = 0, cus = 256;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, (const void*)mix_bwd_bf16_kernel<CIN, true>, 256,
                                                     mix_bf16_lds<CIN>()) != hipSuccess || per_cu < 1)
      per_cu = 1;
    if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    (void)hipGetLastError();
    return per_cu * cus;
  }();
  return std::min(std::min(a->frames, 768), slots);
}
template <int CIN>
static int launch_mix_bwd_bf16(const MixArgs* a, hipStream_t s) {
  if (a->K * a->V > 64 || a->V > 32) return -1;
  const int grid = mix_bwd_bf16_grid<CIN>(a);
  if (a->accumulate)
    hipLaunchKernelGGL((mix_bwd_bf16_kernel<CIN, true>), dim3(grid), dim3(256), mix_bf16_lds<CIN>(), s, *a);
  else
    hipLaunchKernelGGL((mix_bwd_bf16_kernel<CIN, false>), dim3(grid), dim3(256), mix_bf16_lds<CIN>(), s, *a);
  F3_LAUNCH_CHECK();
  if (a->no_colsum) return F3_OK;
  return f3_colsum(a->part, grid, a->K * a->V * a->V, a->dA, s);
}

template <int CIN, bool ZB16>
static int mix_bwd_ks(const MixArgs* a, hipStream_t s) {
  if (ZB16 && mix_bwd_bf16_on()) {
    const int r = launch_mix_bwd_bf16<CIN>(a, s);
    if (r >= 0) return r;
  }
  switch ((a->K * a->V + 3) / 4) {
    case 4: return launch_mix_bwd<4, CIN, ZB16>(a, s);
    case 5: return launch_mix_bwd<5, CIN, ZB16>(a, s);
    case 7: return launch_mix_bwd<7, CIN, ZB16>(a, s);
    case 9: return launch_mix_bwd<9, CIN, ZB16>(a, s);
    case 11: return launch_mix_bwd<11, CIN, ZB16>(a, s);
    case 14: return launch_mix_bwd<14, CIN, ZB16>(a, s);
    default: return -1;
  }
}

template <int CIN>
static int mix_bwd_cin(const MixArgs* a, hipStream_t s) {
  if ((a->dzb != nullptr) != (a->x16 != 0)) return F3_EINVAL;  // bf16 dZ <=> bf16 x (the bf16 mode)
  return a->dzb ? mix_bwd_ks<CIN, true>(a, s) : mix_bwd_ks<CIN, false>(a, s);
}

int f3_mix_bwd_parts(const MixArgs* a) {  // rows of `part` the launch leaves (no_colsum callers sum them)
  if (a->x3 && mix_x3_ok(*a))
    return a->Cin == 64 ? mix_bwd_x3_grid<64>(a) : a->Cin == 128 ? mix_bwd_x3_grid<128>(a) : mix_bwd_x3_grid<256>(a);
  if (!mix_lds_ok(*a)) return 0;
  if (a->dzb && mix_bwd_bf16_on() && a->K * a->V <= 64 && a->V <= 32)
    return a->Cin == 64 ? mix_bwd_bf16_grid<64>(a) : a->Cin == 128 ? mix_bwd_bf16_grid<128>(a) : mix_bwd_bf16_grid<256>(a);
  return std::min(a->frames, 768);
}

int f3_mix_bwd(const MixArgs* a, hipStream_t s) {
  if (a->x3 && mix_x3_ok(*a)) {
    if (!a->part) return F3_EINVAL;
    if (a->frames <= 0) return F3_OK;
    return a->Cin == 64 ? launch_mix_bwd_x3<64>(a, s) : a->Cin == 128 ? launch_mix_bwd_x3<128>(a, s)
                                                         : launch_mix_bwd_x3<256>(a, s);
  }
  if (mix_lds_ok(*a)) {
    if (!a->part) return F3_EINVAL;
    const int r = a->Cin == 64 ? mix_bwd_cin<64>(a, s) : a->Cin == 128 ? mix_bwd_cin<128>(a, s) : mix_bwd_cin<256>(a, s);
    if (r >= 0) return r;
  }
  if (a->dzb) return F3_EINVAL;  // the generic kernel reads fp32 dZ
  F3_BIG_LDS(mix_bwd_kernel);
  if (a->K * a->V * a->V > 1024 || mix_lds(*a, true) > 160 * 1024) return F3_EINVAL;
  const int grid = min(a->frames, 1024);
  hipLaunchKernelGGL(mix_bwd_kernel, dim3(grid), dim3(256), mix_lds(*a, true), s, *a);
  F3_LAUNCH_CHECK();
  return F3_OK;
}

int f3_gcn_bias_bwd(const GcnBiasBwdArgs* a, hipStream_t s) {
  if (a->K * a->V * a->V > 3072 || a->K * a->V > 1024) return F3_EINVAL;
  hipLaunchKernelGGL(gcn_bias_bwd_kernel, dim3((a->K * a->C + 255) / 256 + a->K * a->V), dim3(256), 0, s, *a);
  F3_LAUNCH_CHECK();
  return F3_OK;
}

// rows per workgroup of the clip-chunk elementwise kernels (block_out, block_bwd_*): 96 (192 or 270
// measured no faster, profiles/r03_chunk_ab.txt)
static int chunks_for(int TV) { return max(1, (TV + 95) / 96); }
int f3_block_chunks(int TV) { return chunks_for(TV); }

// backward block kernels: instantiate on (activation type, residual kind, pooled gradient)
template <bool A16, int RES, bool DNC>
static void launch_block_bwd1(const BlockArgs& a, bool reduce, hipStream_t s) {
  const dim3 grid(a.chunks, a.N);
  if (reduce) hipLaunchKernelGGL((block_bwd_reduce_kernel<A16, RES, DNC>), grid, dim3(256), 0, s, a);
  else hipLaunchKernelGGL((block_bwd_apply_kernel<A16, RES, DNC>), grid, dim3(256), 0, s, a);
}
template <bool A16, int RES>
static void launch_block_bwd2(const BlockArgs& a, bool reduce, hipStream_t s) {
  if (a.dout_nc) launch_block_bwd1<A16, RES, true>(a, reduce, s);
  else launch_block_bwd1<A16, RES, false>(a, reduce, s);
}
template <bool REDUCE>
static void launch_block_bwd(const BlockArgs& a, hipStream_t s) {
  if (a.act16) {
    if (a.res_kind == RES_CONV) launch_block_bwd2<true, RES_CONV>(a, REDUCE, s);
    else if (a.res_kind == RES_ID) launch_block_bwd2<true, RES_ID>(a, REDUCE, s);
    else launch_block_bwd2<true, RES_NONE>(a, REDUCE, s);
  } else {
    if (a.res_kind == RES_CONV) launch_block_bwd2<false, RES_CONV>(a, REDUCE, s);
    else if (a.res_kind == RES_ID) launch_block_bwd2<false, RES_ID>(a, REDUCE, s);
    else launch_block_bwd2<false, RES_NONE>(a, REDUCE, s);
  }
}

int f3_block_out(BlockArgs a, hipStream_t s) {
  if (a.C % 4 || a.C > 256 || 256 % (a.C / 4)) return F3_EINVAL;
  a.chunks = chunks_for(a.TV);
  if (!a.pool) a.part = nullptr;
  const dim3 grid(a.chunks, a.N);
#define F3_BO(A, R) hipLaunchKernelGGL((block_out_kernel<A, R>), grid, dim3(256), 0, s, a)
  if (a.res_kind < RES_NONE || a.res_kind > RES_CONV) return F3_EINVAL;
  if (a.act16) {
    if (a.res_kind == RES_CONV) F3_BO(true, RES_CONV);
    else if (a.res_kind == RES_ID) F3_BO(true, RES_ID);
    else F3_BO(true, RES_NONE);
  } else {
    if (a.res_kind == RES_CONV) F3_BO(false, RES_CONV);
    else if (a.res_kind == RES_ID) F3_BO(false, RES_ID);
    else F3_BO(false, RES_NONE);
  }
#undef F3_BO
  F3_LAUNCH_CHECK();
  if (a.part) return f3_colsum(a.part, a.chunks, a.N * a.C, a.pool, s);
  return F3_OK;
}

int f3_block_bwd_reduce(BlockArgs a, hipStream_t s) {
  if (a.C % 4 || a.C > 256 || 256 % (a.C / 4)) return F3_EINVAL;
  a.chunks = chunks_for(a.TV);
  if (a.res_kind < RES_NONE || a.res_kind > RES_CONV) return F3_EINVAL;
  launch_block_bwd<true>(a, s);
  F3_LAUNCH_CHECK();
  if (!a.part || a.no_colsum) return F3_OK;
  const int nc = a.N * a.C, nseg = a.res_kind == RES_CONV ? 3 : 2;
  if (a.P2 == a.P1 + nc && (nseg == 2 || a.Q2 == a.P1 + 2 * nc))  // contiguous [P1 | P2 | Q2]: one launch
    return f3_colsum_ld(a.part, a.chunks, 3LL * nc, nseg * nc, a.P1, s);
  const ColsumJob j[3] = {{a.part, a.P1, 3LL * nc, a.chunks, nc},
                          {a.part + nc, a.P2, 3LL * nc, a.chunks, nc},
                          {a.part + 2 * nc, a.Q2, 3LL * nc, a.chunks, nc}};
  F3_TRY(f3_colsum_multi(j, nseg, s));
  return F3_OK;
}

int f3_block_bwd_apply(BlockArgs a, hipStream_t s) {
  if (a.C % 4 || a.C > 256 || 256 % (a.C / 4)) return F3_EINVAL;
  a.chunks = chunks_for(a.TV);
  if (a.res_kind < RES_NONE || a.res_kind > RES_CONV) return F3_EINVAL;
  launch_block_bwd<false>(a, s);
  F3_LAUNCH_CHECK();
  return F3_OK;
}

int f3_bn_bwd_parts(int N, int TV, int V) {
  const int fr = bn_bwd_frames();
  return ((TV / V + fr - 1) / fr) * N;
}

int f3_bn_bwd_apply(BnBwdArgs a, hipStream_t s) {
  if (a.C % 8 || a.C > 256 || a.TV % a.V || a.V * (a.C / 8) > 1024 || !a.Gpart) return F3_EINVAL;
  const int fr = bn_bwd_frames();
  const int T = a.TV / a.V, fch = (T + fr - 1) / fr;
  const int threads = ((a.V * (a.C / 8) + 63) / 64) * 64;
  if (fr == 8) {
    if (a.act16) hipLaunchKernelGGL((bn_bwd_apply_kernel<true, 8>), dim3(fch, a.N), dim3(threads), 0, s, a);
    else hipLaunchKernelGGL((bn_bwd_apply_kernel<false, 8>), dim3(fch, a.N), dim3(threads), 0, s, a);
  } else {
    if (a.act16) {
      hipLaunchKernelGGL((bn_bwd_apply_kernel<true, 4>), dim3(fch, a.N), dim3(threads), 0, s, a);
    } else {
      hipLaunchKernelGGL((bn_bwd_apply_kernel<false, 4>), dim3(fch, a.N), dim3(threads), 0, s, a);
    }
  }
  F3_LAUNCH_CHECK();
  if (a.no_colsum) return F3_OK;
  return f3_colsum(a.Gpart, fch * a.N, a.V * a.C, a.G, s);
}

int f3_colsum_multi(const ColsumJob* jobs, int n, hipStream_t s) {
  if (n < 0 || n > kColsumJobs) return F3_EINVAL;
  ColsumJobs J;
  J.n = 0;
  J.blk[0] = 0;
  for (int i = 0; i < n; ++i) {
    if (jobs[i].rows <= 0 || jobs[i].cols <= 0) continue;
    const int k = J.n++;
    J.part[k] = jobs[i].part;
    J.out[k] = jobs[i].out;
    J.ld[k] = jobs[i].ld;
    J.rows[k] = jobs[i].rows;
    J.cols[k] = jobs[i].cols;
    J.rg[k] = colsum_rg(jobs[i].rows, jobs[i].cols);
    const int cpb = 1024 / J.rg[k];
    J.blk[k + 1] = J.blk[k] + (jobs[i].cols + cpb - 1) / cpb;
  }
  if (J.n == 0) return F3_OK;
  hipLaunchKernelGGL(colsum_kernel, dim3(J.blk[J.n]), dim3(1024), 0, s, J);
  F3_LAUNCH_CHECK();
  return F3_OK;
}

int f3_colsum(const float* part, int rows, int cols, float* out, hipStream_t s) {
  const ColsumJob j{part, out, (long long)cols, rows, cols};
  return f3_colsum_multi(&j, 1, s);
}

int f3_colsum_ld(const float* part, int rows, long long ld, int cols, float* out, hipStream_t s) {
  const ColsumJob j{part, out, ld, rows, cols};
  return f3_colsum_multi(&j, 1, s);
}

int f3_bnrelu_bf16(const BnReluArgs* a, hipStream_t s) {
  if (a->C % 8 || a->C > 256) return F3_EINVAL;
  const size_t total8 = (size_t)a->M * a->C / 8;
  // (the main kernel needs 2048 % C == 0: a thread's channel group is fixed over its grid stride)
  if (2048 % a->C) {
    if (a->x3) return F3_EINVAL;
    const int grid = (int)std::min<size_t>((total8 + 255) / 256, 4096);
    if (a->g16) hipLaunchKernelGGL(bnrelu_bf16_any_kernel<true>, dim3(grid), dim3(256), 0, s, *a);
    else hipLaunchKernelGGL(bnrelu_bf16_any_kernel<false>, dim3(grid), dim3(256), 0, s, *a);
    F3_LAUNCH_CHECK();
    return F3_OK;
  }
  const int grid = (int)std::min<size_t>((total8 + 256 * kBnReluU - 1) / (256 * kBnReluU), 1024);
  if (a->x3) {
    if (a->g16) return F3_EINVAL;
    hipLaunchKernelGGL((bnrelu_bf16_kernel<false, true>), dim3(grid), dim3(256), 0, s, *a);
  } else if (a->g16) {
    hipLaunchKernelGGL(bnrelu_bf16_kernel<true>, dim3(grid), dim3(256), 0, s, *a);
  } else {
    hipLaunchKernelGGL(bnrelu_bf16_kernel<false>, dim3(grid), dim3(256), 0, s, *a);
  }
  F3_LAUNCH_CHECK();
  return F3_OK;
}

// F3_CA_X (default 1): the up-front-load channel-attention kernels where they fit (N <= 256, C % 64 == 0)
static bool ca_x(const CaArgs* a) {
  const char* e = getenv("F3_CA_X");  // (read per call: the A/B test flips it in one process)
  return !(e && atoi(e) == 0) && a->N <= 256 && a->C % 64 == 0;
}

// F3_CA_X=1: the x kernels with ca_bwd2 as its own launch (A/B); unset or 2: ca_bwd2 folded into ca_bwd3x
static bool ca_fuse2() {
  const char* e = getenv("F3_CA_X");
  return !(e && atoi(e) == 1);
}

bool f3_ca_x_ok(int N, int C, int TV) {
  CaArgs a;
  a.N = N;
  a.C = C;
  return ca_x(&a) && f3_block_chunks(TV) <= 16;
}

int f3_ca_fwd(const CaArgs* a, hipStream_t s) {
  if (a->C > 256 || a->N > 256 * kCaMaxRowsPerThread) return F3_EINVAL;
  if (ca_x(a)) {
    hipLaunchKernelGGL(ca_fwd1x_kernel, dim3(a->C / 4), dim3(1024), 0, s, *a);
    F3_LAUNCH_CHECK();
    hipLaunchKernelGGL(ca_fwd2x_kernel, dim3(a->N), dim3(1024), 0, s, *a);
    F3_LAUNCH_CHECK();
    return F3_OK;
  }
  hipLaunchKernelGGL(ca_fwd1_kernel, dim3(a->C / 4), dim3(256), 0, s, *a);
  F3_LAUNCH_CHECK();
  hipLaunchKernelGGL(ca_fwd2_kernel, dim3(a->N), dim3(256), 0, s, *a);
  F3_LAUNCH_CHECK();
  return F3_OK;
}

int f3_ca_bwd(const CaArgs* a, hipStream_t s) {
  if (a->C > 256 || a->N > 256) return F3_EINVAL;
  if (a->bpart && (!ca_x(a) || a->bchunks < 1 || a->bchunks > 16)) return F3_EINVAL;  // (f3_ca_x_ok decides)
  if (ca_x(a)) {
    hipLaunchKernelGGL(ca_bwd1x_kernel, dim3(a->N), dim3(1024), 0, s, *a);
    F3_LAUNCH_CHECK();
    if (ca_fuse2()) {
      hipLaunchKernelGGL(ca_bwd3x_kernel<true>, dim3((a->N + 3) / 4), dim3(1024), 0, s, *a);
      F3_LAUNCH_CHECK();
      return F3_OK;
    }
    hipLaunchKernelGGL(ca_bwd2_kernel, dim3(a->C / 4), dim3(256), 0, s, *a);
    F3_LAUNCH_CHECK();
    hipLaunchKernelGGL(ca_bwd3x_kernel<false>, dim3((a->N + 3) / 4), dim3(1024), 0, s, *a);
    F3_LAUNCH_CHECK();
    return F3_OK;
  }
  hipLaunchKernelGGL(ca_bwd1_kernel, dim3(a->N), dim3(256), 0, s, *a);
  F3_LAUNCH_CHECK();
  hipLaunchKernelGGL(ca_bwd2_kernel, dim3(a->C / 4), dim3(256), 0, s, *a);
  F3_LAUNCH_CHECK();
  // (one clip per workgroup measured no faster, profiles/r04_ca_b3_ab.txt)
  hipLaunchKernelGGL(ca_bwd3_kernel<kCaB3Clips>, dim3((a->N + kCaB3Clips - 1) / kCaB3Clips), dim3(256), 0, s, *a);
  F3_LAUNCH_CHECK();
  return F3_OK;
}

int f3_ca_bwd_weights(const CaArgs* a, hipStream_t s, ColsumJob* defer, int* ndefer) {
  if (a->C > 256 || a->N > 256) return F3_EINVAL;
  const int groups = (a->N + kCaWClips - 1) / kCaWClips, H = a->C / 4, C = a->C;
  hipLaunchKernelGGL(ca_bwd_w_kernel, dim3((a->C + 63) / 64, groups), dim3(256), 0, s, *a);
  F3_LAUNCH_CHECK();
  if (!a->wpart) return F3_OK;
  // the partial rows are [groups][2 H C + C]: sum each segment's columns over the groups
  const int ld = 2 * H * C + C;
  const ColsumJob j[3] = {{a->wpart, a->g_W1, ld, groups, H * C},
                          {a->wpart + H * C, a->g_W2, ld, groups, C * H},
                          {a->wpart + 2 * H * C, a->g_b2, ld, groups, C}};
  if (defer) {
    if (!ndefer || *ndefer + 3 > kColsumJobs) return F3_EINVAL;
    for (int i = 0; i < 3; ++i) defer[(*ndefer)++] = j[i];
    return F3_OK;
  }
  return f3_colsum_multi(j, 3, s);
}

int f3_bn_running(const BnRunTable& t, hipStream_t s) {
  if (t.n <= 0) return F3_OK;
  if (t.n > kMaxBnJobs) return F3_EINVAL;
  hipLaunchKernelGGL(bn_running_kernel, dim3(t.n), dim3(256), 0, s, t);
  F3_LAUNCH_CHECK();
  return F3_OK;
}
