// musa_model.Model kernels for gfx950 (reference: Multimodal_Fall3/model/musa_model.py).
//
// Per-channel reductions (BatchNorm sums, weight gradients of the depthwise conv) use one thread
// per (channel quad, row lane): nq = C/4 quads, 256/nq row lanes, float4 loads along the channels
// so a wave reads whole 512-B row segments; per-thread partials reduce through LDS float atomics,
// then once per workgroup into fp64 global sums. DropBlock masks: one 1024-thread workgroup per
// block call, every intermediate in LDS, draws from the counter hash of oracle/musa_cpu.py.
#include <math.h>

#include <algorithm>
#include <cstdlib>

#include "musa.h"

namespace f3 {
namespace mu {

F3_DEV float act_f(int a, float z) {
  switch (a) {
    case ACT_RELU: return fmaxf(z, 0.f);
    case ACT_TANH: return tanhf(z);
    case ACT_LEAKY: return z > 0.f ? z : kLeaky * z;
    default: return z;
  }
}
F3_DEV float act_d(int a, float z) {  // torch: relu' = (z > 0), leaky' = z > 0 ? 1 : slope
  switch (a) {
    case ACT_RELU: return z > 0.f ? 1.f : 0.f;
    case ACT_TANH: {
      const float t = tanhf(z);
      return 1.f - t * t;
    }
    case ACT_LEAKY: return z > 0.f ? 1.f : kLeaky;
    default: return 1.f;
  }
}

F3_DEV unsigned mix32(unsigned x) {
  x ^= x >> 16;
  x *= 0x7FEB352Du;
  x ^= x >> 15;
  x *= 0x846CA68Bu;
  x ^= x >> 16;
  return x;
}
// uniform24(seed, call, e) of oracle/musa_cpu.py
F3_DEV float uni24(unsigned seed, int call, unsigned e) {
  const unsigned base = mix32(seed ^ ((unsigned)call * 0x9E3779B9u));
  return (float)(mix32(e + base) >> 8) * (1.f / 16777216.f);
}

struct QuadLayout {
  int nq, rs, q, rl;
  bool act;
  F3_DEV QuadLayout(int C) {
    nq = C >> 2;
    rs = 256 / nq;
    q = threadIdx.x % nq;
    rl = threadIdx.x / nq;
    act = rl < rs;
  }
};

// per-channel sums of this workgroup's threads -> its fp32 lane (lanes[l][0..C) and [C..2C)),
// totalled in fp64 by mu_lane_finalize_kernel. Straight-line code behind raw barriers, and nb (the
// block size) from a kernel argument: a loop, a __syncthreads fence or a blockDim read (a vector
// load from the dispatch packet) ahead of the lane adds made hipcc wait vmcnt(0) for the
// workgroup's row stores first (7 us of a 27 us conv launch). Needs C <= 256 and nb >= C.
// STORE: the workgroup owns lane row blockIdx.x (grid <= kLanes) and writes its partial row with
// plain stores instead of memory-side adds (the depthwise conv's F3_DW_STORE form)
template <bool STORE = false>
F3_DEV void channel_flush(int C, int q, bool act, const float (&s1)[4], const float (&s2)[4], float* lanes, int nb) {
  __shared__ float r[512];
  const int t = threadIdx.x, n2 = 2 * C;
  if (t < n2) r[t] = 0.f;
  if (t + nb < n2) r[t + nb] = 0.f;
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  if (act)
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      atomicAdd(r + 4 * q + e, s1[e]);
      atomicAdd(r + C + 4 * q + e, s2[e]);
    }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  // one wave issues the lane adds (the others end here)
  if (t >= 64) return;
  float* l = lanes + (size_t)(blockIdx.x % kLanes) * kLaneRow;
  float v[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) v[i] = t + 64 * i < n2 ? r[t + 64 * i] : 0.f;
#pragma unroll
  for (int i = 0; i < 8; ++i)
    if (t + 64 * i < n2) {
      if constexpr (STORE) l[t + 64 * i] = v[i];
      else atomicAdd(l + t + 64 * i, v[i]);
    }
}
F3_DEV void channel_flush(int C, const QuadLayout& L, const float (&s1)[4], const float (&s2)[4], float* lanes) {
  channel_flush(C, L.q, L.act, s1, s2, lanes, 256);  // QuadLayout kernels run 256 threads
}

// totals of the lanes: g1[c] += sum_l lanes[l][c], g2[c] += sum_l lanes[l][C + c] (fp64); lanes
// re-zeroed. Workgroup w owns columns [64w, 64w + 64) of the 2C; its 16 lane groups of 64 threads
// walk every 16th lane with all loads independent (and the g1 / g2 read issued with them: one
// memory round trip), then the groups are summed in a fixed order.
constexpr int kFinCols = 64, kFinGroups = 16;
__global__ __launch_bounds__(kFinCols * kFinGroups) void mu_lane_finalize_kernel(float* lanes, int C, double* g1,
                                                                                 double* g2) {
  __shared__ double red[kFinGroups][kFinCols];
  const int n2 = 2 * C, j = threadIdx.x % kFinCols, grp = threadIdx.x / kFinCols;
  const int c = blockIdx.x * kFinCols + j;
  double s = 0.0, g = 0.0;
  if (c < n2) {
    constexpr int kPer = kLanes / kFinGroups;
    float v[kPer];
#pragma unroll
    for (int i = 0; i < kPer; ++i) v[i] = lanes[(size_t)(grp + i * kFinGroups) * kLaneRow + c];
    if (grp == 0) g = c < C ? g1[c] : g2[c - C];
#pragma unroll
    for (int i = 0; i < kPer; ++i) {
      lanes[(size_t)(grp + i * kFinGroups) * kLaneRow + c] = 0.f;
      s += (double)v[i];
    }
  }
  red[grp][j] = s;
  __syncthreads();
  if (grp == 0 && c < n2) {
    for (int k = 1; k < kFinGroups; ++k) s += red[k][j];
    if (c < C) g1[c] = g + s;
    else g2[c - C] = g + s;
  }
}

F3_DEV f32x4 ld4(const float* p) { return *reinterpret_cast<const f32x4*>(p); }
F3_DEV void st4(float* p, f32x4 v) { *reinterpret_cast<f32x4*>(p) = v; }

// ------------------------------------------------------------------------------------------
// depthwise temporal conv (SepTemporal_Block depth_conv / Sep_TCN sep31, sep11; :163-166, 429-436)
// ------------------------------------------------------------------------------------------
// One thread per (clip n, joint v, channel quad q, chunk of 8 output frames): the chunk's
// (8-1)*S + K input rows are loaded at once into registers, so every input row is read once per
// chunk (plus the K-S overlap with the neighbouring chunk) and consecutive threads read
// consecutive 16-B pieces of a row (joint-major rows of C channels: a wave covers 64 quads of one
// or two joints' rows). The grid is capped (1024 workgroups) and walks the items with a stride
// that is a multiple of the quad count, so a thread's BN partial sums stay per channel quad.
constexpr int kDwChunk = 8;

template <int K, int S, bool STORE>
__global__ __launch_bounds__(512) void mu_dwconv_fwd_kernel(DwConvArgs a) {
  const int nq = a.C >> 2;
  const int nchunk = (a.T_out + kDwChunk - 1) / kDwChunk;
  const int total = a.N * a.V * nq * nchunk;
  // blockDim is a multiple of nq, so a thread's channel quad is the same for every item it takes
  const int g0 = blockIdx.x * blockDim.x + threadIdx.x, G = gridDim.x * blockDim.x;
  const int q = g0 % nq;
  float s1[4] = {0.f, 0.f, 0.f, 0.f}, s2[4] = {0.f, 0.f, 0.f, 0.f};
  f32x4 w[K];
  const f32x4 b = ld4(a.b + 4 * q);
#pragma unroll
  for (int k = 0; k < K; ++k)
#pragma unroll
    for (int e = 0; e < 4; ++e) w[k][e] = a.w[(4 * q + e) * K + k];
  const int rstride = a.V * a.C;  // floats between consecutive frames of one joint
  for (int g = g0; g < total; g += G) {
    int rest = g / nq;
    const int v = rest % a.V;
    rest /= a.V;
    const int ch = rest % nchunk, n = rest / nchunk;
    const float* xb = a.x + ((size_t)n * a.T_in * a.V + v) * a.C + 4 * q;
    float* yb = a.y + ((size_t)n * a.T_out * a.V + v) * a.C + 4 * q;
    // the chunk's whole input window is loaded up front (clamped frames, zeroed after): every
    // load is in flight at once, and no load is conditional (a conditional load makes hipcc
    // wait vmcnt(0) per output)
    constexpr int NIN = (kDwChunk - 1) * S + K;
    const int t0 = ch * kDwChunk, nout = min(a.T_out - t0, kDwChunk);
    const int tb = t0 * S - a.P;
    f32x4 xw[NIN];
#pragma unroll
    for (int i = 0; i < NIN; ++i) xw[i] = ld4(xb + (size_t)min(max(tb + i, 0), a.T_in - 1) * rstride);
#pragma unroll
    for (int i = 0; i < NIN; ++i)
      if (tb + i < 0 || tb + i >= a.T_in) xw[i] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int o = 0; o < kDwChunk; ++o) {
      if (o < nout) {
        f32x4 acc = b;
#pragma unroll
        for (int k = 0; k < K; ++k)
#pragma unroll
          for (int e = 0; e < 4; ++e) acc[e] = fmaf(w[k][e], xw[o * S + k][e], acc[e]);
        st4(yb + (size_t)(t0 + o) * rstride, acc);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          s1[e] += acc[e];
          s2[e] = fmaf(acc[e], acc[e], s2[e]);
        }
      }
    }
  }
  if (a.sum) {
    channel_flush<STORE>(a.C, q, g0 < total, s1, s2, a.lanes, a.block);
  }
}

// dx[n][ti][v][c] = sum_k dy[n][to][v][c] w[c][k], ti = to*S + k - P
template <int K>
__global__ __launch_bounds__(256) void mu_dwconv_dx_kernel(DwConvArgs a) {
  const QuadLayout L(a.C);
  if (!L.act) return;
  f32x4 w[K];
#pragma unroll
  for (int k = 0; k < K; ++k)
#pragma unroll
    for (int e = 0; e < 4; ++e) w[k][e] = a.w[(4 * L.q + e) * K + k];
  const long long rows = (long long)a.N * a.T_in * a.V;
  for (long long r = (long long)blockIdx.x * L.rs + L.rl; r < rows; r += (long long)gridDim.x * L.rs) {
    const int v = (int)(r % a.V);
    const long long nt = r / a.V;
    const int ti = (int)(nt % a.T_in), n = (int)(nt / a.T_in);
    f32x4 acc = a.dx_add ? ld4(a.dx + (size_t)r * a.C + 4 * L.q) : f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int k = 0; k < K; ++k) {
      const int num = ti + a.P - k;
      if (num < 0 || num % a.S) continue;
      const int to = num / a.S;
      if (to >= a.T_out) continue;
      const f32x4 g = ld4(a.dy + (((size_t)n * a.T_out + to) * a.V + v) * a.C + 4 * L.q);
#pragma unroll
      for (int e = 0; e < 4; ++e) acc[e] = fmaf(w[k][e], g[e], acc[e]);
    }
    st4(a.dx + (size_t)r * a.C + 4 * L.q, acc);
  }
}

// weight / bias gradient partial rows: part[blk][c*K + k] and part[grid*C*K + blk*C + c]
template <int K>
__global__ __launch_bounds__(256) void mu_dwconv_dw_kernel(DwConvArgs a) {
  const QuadLayout L(a.C);
  __shared__ float red[256 * 6];
  for (int i = threadIdx.x; i < a.C * (K + 1); i += blockDim.x) red[i] = 0.f;
  __syncthreads();
  if (L.act) {
    f32x4 gw[K], gb = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int k = 0; k < K; ++k) gw[k] = f32x4{0.f, 0.f, 0.f, 0.f};
    const long long rows = (long long)a.N * a.T_out * a.V;
    for (long long r = (long long)blockIdx.x * L.rs + L.rl; r < rows; r += (long long)gridDim.x * L.rs) {
      const int v = (int)(r % a.V);
      const long long nt = r / a.V;
      const int to = (int)(nt % a.T_out), n = (int)(nt / a.T_out);
      const f32x4 g = ld4(a.dy + (size_t)r * a.C + 4 * L.q);
      gb += g;
#pragma unroll
      for (int k = 0; k < K; ++k) {
        const int ti = to * a.S + k - a.P;
        if (ti >= 0 && ti < a.T_in) {
          const f32x4 x = ld4(a.x + (((size_t)n * a.T_in + ti) * a.V + v) * a.C + 4 * L.q);
#pragma unroll
          for (int e = 0; e < 4; ++e) gw[k][e] = fmaf(g[e], x[e], gw[k][e]);
        }
      }
    }
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int c = 4 * L.q + e;
#pragma unroll
      for (int k = 0; k < K; ++k) atomicAdd(red + c * K + k, gw[k][e]);
      atomicAdd(red + a.C * K + c, gb[e]);
    }
  }
  __syncthreads();
  const size_t G = a.part_rows;  // == gridDim.x (set by the launcher)
  for (int i = threadIdx.x; i < a.C * K; i += 256) a.part[(size_t)blockIdx.x * a.C * K + i] = red[i];
  for (int c = threadIdx.x; c < a.C; c += 256) a.part[G * a.C * K + (size_t)blockIdx.x * a.C + c] = red[a.C * K + c];
}

// ------------------------------------------------------------------------------------------
// BatchNorm + activation
// ------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void mu_bn_act_kernel(BnActArgs a) {
  __shared__ float sc[256], sh[256];
  for (int c = threadIdx.x; c < a.C; c += blockDim.x) {
    float m, r;
    bn_coeff(a.bn, c, sc[c], sh[c], m, r);
  }
  __syncthreads();
  const long long n4 = a.R * a.C / 4;
  const int nq = a.C / 4;
  for (long long i = blockIdx.x * 256LL + threadIdx.x; i < n4; i += (long long)gridDim.x * 256) {
    const int c = (int)(i % nq) * 4;
    const f32x4 u = ld4(a.u + i * 4);
    f32x4 y;
#pragma unroll
    for (int e = 0; e < 4; ++e) y[e] = act_f(a.act, fmaf(u[e], sc[c + e], sh[c + e]));
    if (a.add) y += ld4(a.add + i * 4);
    st4(a.y + i * 4, y);
  }
}

__global__ __launch_bounds__(256) void mu_bn_act_bwd_reduce_kernel(BnActBwdArgs a) {
  __shared__ float sc[256], sh[256], mu_[256], rs_[256];
  for (int c = threadIdx.x; c < a.C; c += blockDim.x) bn_coeff(a.bn, c, sc[c], sh[c], mu_[c], rs_[c]);
  __syncthreads();
  const QuadLayout L(a.C);
  float s1[4] = {0.f, 0.f, 0.f, 0.f}, s2[4] = {0.f, 0.f, 0.f, 0.f};
  if (L.act) {
    const int c0 = 4 * L.q;
    for (long long r = (long long)blockIdx.x * L.rs + L.rl; r < a.R; r += (long long)gridDim.x * L.rs) {
      const f32x4 u = ld4(a.u + (size_t)r * a.C + c0), dy = ld4(a.dy + (size_t)r * a.C + c0);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float z = fmaf(u[e], sc[c0 + e], sh[c0 + e]);
        const float dz = dy[e] * act_d(a.act, z);
        s1[e] += dz;
        s2[e] = fmaf(dz, (u[e] - mu_[c0 + e]) * rs_[c0 + e], s2[e]);
      }
    }
  }
  channel_flush(a.C, L, s1, s2, a.lanes);
}

__global__ __launch_bounds__(256) void mu_bn_act_bwd_apply_kernel(BnActBwdArgs a) {
  __shared__ float sc[256], sh[256], mu_[256], rs_[256], m1[256], m2[256];
  for (int c = threadIdx.x; c < a.C; c += blockDim.x) {
    bn_coeff(a.bn, c, sc[c], sh[c], mu_[c], rs_[c]);
    m1[c] = (float)(a.s_dz[c] / (double)a.R);
    m2[c] = (float)(a.s_dzx[c] / (double)a.R);
    if (blockIdx.x == 0) {
      a.g_gamma[c] += (float)a.s_dzx[c];
      a.g_beta[c] += (float)a.s_dz[c];
    }
  }
  __syncthreads();
  const long long n4 = a.R * a.C / 4;
  const int nq = a.C / 4;
  for (long long i = blockIdx.x * 256LL + threadIdx.x; i < n4; i += (long long)gridDim.x * 256) {
    const int c = (int)(i % nq) * 4;
    const f32x4 u = ld4(a.u + i * 4), dy = ld4(a.dy + i * 4);
    f32x4 du;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const float z = fmaf(u[e], sc[c + e], sh[c + e]);
      const float dz = dy[e] * act_d(a.act, z);
      const float xh = (u[e] - mu_[c + e]) * rs_[c + e];
      du[e] = sc[c + e] * (dz - m1[c + e] - xh * m2[c + e]);
    }
    if (a.add) du += ld4(a.add + i * 4);
    st4(a.du + i * 4, du);
  }
}

__global__ __launch_bounds__(256) void mu_colstat_kernel(ColStatArgs a) {
  const QuadLayout L(a.C);
  float s1[4] = {0.f, 0.f, 0.f, 0.f}, s2[4] = {0.f, 0.f, 0.f, 0.f};
  if (L.act)
    for (long long r = (long long)blockIdx.x * L.rs + L.rl; r < a.R; r += (long long)gridDim.x * L.rs) {
      const f32x4 x = ld4(a.x + (size_t)r * a.C + 4 * L.q);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        s1[e] += x[e];
        s2[e] = fmaf(x[e], x[e], s2[e]);
      }
    }
  channel_flush(a.C, L, s1, s2, a.lanes);
}

// ------------------------------------------------------------------------------------------
// DropBlock (Randomized_DropBlock_Ske :39-70, Randomized_DropBlockT_1d :73-99)
// ------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void mu_absstat_kernel(AbsStatArgs a) {
  __shared__ float sc[256], sh[256], red[256];
  for (int c = threadIdx.x; c < a.C; c += blockDim.x) {
    float m, r;
    if (a.bn_on) bn_coeff(a.bn, c, sc[c], sh[c], m, r);
    else { sc[c] = 1.f; sh[c] = 0.f; }
  }
  __syncthreads();
  const QuadLayout L(a.C);
  // every workgroup walks whole rows: row lane rl of this pass handles row base + rl
  for (long long base = (long long)blockIdx.x * L.rs; base < a.R; base += (long long)gridDim.x * L.rs) {
    const long long r = base + L.rl;
    float s = 0.f;
    if (L.act && r < a.R) {
      const f32x4 u = ld4(a.u + (size_t)r * a.C + 4 * L.q);
#pragma unroll
      for (int e = 0; e < 4; ++e) s += fabsf(fmaf(u[e], sc[4 * L.q + e], sh[4 * L.q + e]));
    }
    red[threadIdx.x] = s;
    __syncthreads();
    if (L.act && L.q == 0 && r < a.R) {
      float t = 0.f;
      for (int j = 0; j < L.nq; ++j) t += red[L.rl * L.nq + j];
      a.a[r] = t;
    }
    __syncthreads();
  }
}

F3_DEV float block_sum(float v, float* scratch) {  // 1024 threads
  v = warp_sum(v);
  const int w = threadIdx.x >> 6;
  __syncthreads();
  if ((threadIdx.x & 63) == 0) scratch[w] = v;
  __syncthreads();
  float t = 0.f;
  for (int i = 0; i < (int)(blockDim.x >> 6); ++i) t += scratch[i];
  return t;
}

// The two DropBlocks run as three launches (one workgroup per clip for the per-clip reductions
// over a, then one workgroup for the global draws). The S-mask's rescale cS cancels in the T
// block's probabilities (bT / sum bT), so the per-clip T statistics use the 0/1 S mask.
// Scratch (DropMaskArgs::scr): sS [NV], rowS [N], mS [NV], rowM [N], bT [NT], rowT [N].
struct DropScr {
  float *sS, *rowS, *mS, *rowM, *bT, *rowT;
  F3_DEV DropScr(const DropMaskArgs& a) {
    const int NV = a.N * a.V, NT = a.N * a.T;
    sS = a.scr; rowS = sS + NV; mS = rowS + a.N; rowM = mS + NV; bT = rowM + a.N; rowT = bT + NT;
  }
};

// fixed-order sum of x[0..n) (identical in every workgroup of the same blockDim)
F3_DEV float ordered_sum(const float* x, int n, float* red) {
  float s = 0.f;
  for (int i = threadIdx.x; i < n; i += blockDim.x) s += x[i];
  red[threadIdx.x] = s;
  __syncthreads();
  for (int w = blockDim.x / 2; w > 0; w >>= 1) {
    if ((int)threadIdx.x < w) red[threadIdx.x] += red[threadIdx.x + w];
    __syncthreads();
  }
  const float t = red[0];
  __syncthreads();
  return t;
}

// Randomized_DropBlock_Ske input_abs per (n, v) = mean_{c,t} |z|, and its per-clip total
__global__ __launch_bounds__(256) void mu_drop_s_kernel(DropMaskArgs a) {
  __shared__ float sA[64 * 32];
  const DropScr d(a);
  const int n = blockIdx.x, TV = a.T * a.V;
  for (int i = threadIdx.x; i < TV; i += blockDim.x) sA[i] = a.a[(size_t)n * TV + i];
  __syncthreads();
  __shared__ float sv[32];
  if ((int)threadIdx.x < a.V) {
    const int v = threadIdx.x;
    float s = 0.f;
    for (int t = 0; t < a.T; ++t) s += sA[t * a.V + v];
    s /= (float)(a.C * a.T);
    sv[v] = s;
    d.sS[n * a.V + v] = s;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    float s = 0.f;
    for (int v = 0; v < a.V; ++v) s += sv[v];
    d.rowS[n] = s;
  }
}

// per clip: the S seed draws, M = (seed @ Ae) > 0.001, the 0/1 S mask, and the T block's
// input_abs per (n, t) = mean_{c,v} |z| * mask_S (unscaled)
__global__ __launch_bounds__(256) void mu_drop_t_kernel(DropMaskArgs a) {
  __shared__ float sA[64 * 32], Ae[32 * 32], red[256], seedm[32], msk[32], bt[64];
  const DropScr d(a);
  const int n = blockIdx.x, TV = a.T * a.V, V = a.V, NV = a.N * a.V;
  for (int i = threadIdx.x; i < TV; i += blockDim.x) sA[i] = a.a[(size_t)n * TV + i];
  for (int i = threadIdx.x; i < V * V; i += blockDim.x) Ae[i] = a.Ae[i];
  const float totS = ordered_sum(d.rowS, a.N, red);
  const float gamma = (1.f - a.keep_prob) / (1.f + 1.92f);
  if ((int)threadIdx.x < V) {
    const int i = n * V + threadIdx.x;
    const float p = fminf(d.sS[i] / totS * (float)NV * gamma, 1.f);
    seedm[threadIdx.x] = uni24(a.seed, 2 * a.call, (unsigned)i) < p ? 1.f : 0.f;
  }
  __syncthreads();
  if ((int)threadIdx.x < V) {
    const int w = threadIdx.x;
    float m = 0.f;
    for (int v = 0; v < V; ++v) m += seedm[v] * Ae[v * V + w];
    const float mask = m > 0.001f ? 0.f : 1.f;
    msk[w] = mask;
    d.mS[n * V + w] = mask;
  }
  __syncthreads();
  if ((int)threadIdx.x < a.T) {
    const int t = threadIdx.x;
    float s = 0.f;
    for (int v = 0; v < V; ++v) s += msk[v] * sA[t * V + v];
    s /= (float)(a.C * V);
    bt[t] = s;
    d.bT[n * a.T + t] = s;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    float m = 0.f, s = 0.f;
    for (int v = 0; v < V; ++v) m += msk[v];
    for (int t = 0; t < a.T; ++t) s += bt[t];
    d.rowM[n] = m;
    d.rowT[n] = s;
  }
}

// global part: fS = mask_S * NV / sum(mask_S); the T seed draws, the frame permutation (argsort of
// hashed keys: the reference's torch.randperm), max_pool1d, fT = mask_T * NT / sum(mask_T)
__global__ __launch_bounds__(1024) void mu_drop_final_kernel(DropMaskArgs a) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  const int N = a.N, T = a.T, NV = N * a.V, NT = N * T;
  const DropScr d(a);
  float* mT = sm;        // [NT] seed mask, then the permuted max-pool mask
  float* pT = mT + NT;   // [NT] max-pooled
  __shared__ float red[1024], keys[64];
  __shared__ int idx[64];
  const float cS = (float)NV / ordered_sum(d.rowM, N, red);
  for (int i = threadIdx.x; i < NV; i += blockDim.x) a.fS[i] = d.mS[i] * cS;
  const float totT = ordered_sum(d.rowT, N, red);
  const float gT = (1.f - a.keep_prob) / (float)a.block_size;
  for (int i = threadIdx.x; i < NT; i += blockDim.x) {
    const float p = fminf(d.bT[i] / totT * (float)NT * gT, 1.f);
    mT[i] = uni24(a.seed, 2 * a.call + 1, (unsigned)i) < p ? 1.f : 0.f;
  }
  if ((int)threadIdx.x < T) keys[threadIdx.x] = uni24(a.seed ^ 0x5BD1E995u, a.call, threadIdx.x);
  __syncthreads();
  if ((int)threadIdx.x < T) {
    const int t = threadIdx.x;
    int rank = 0;
    for (int j = 0; j < T; ++j) rank += (keys[j] < keys[t]) || (keys[j] == keys[t] && j < t);
    idx[rank] = t;
  }
  const int half = a.block_size / 2;
  for (int i = threadIdx.x; i < NT; i += blockDim.x) {  // max_pool1d(k = block_size, stride 1, pad = k/2)
    const int n = i / T, t = i - n * T;
    float m = 0.f;
    for (int j = max(0, t - half); j <= min(T - 1, t + half); ++j) m = fmaxf(m, mT[n * T + j]);
    pT[i] = m;
  }
  __syncthreads();
  float loc = 0.f;
  for (int i = threadIdx.x; i < NT; i += blockDim.x) {
    const int n = i / T, t = i - n * T;
    const float mask = 1.f - pT[n * T + idx[t]];
    mT[i] = mask;
    loc += mask;
  }
  const float cT = (float)NT / block_sum(loc, red);
  for (int i = threadIdx.x; i < NT; i += blockDim.x) a.fT[i] = mT[i] * cT;
}

// ------------------------------------------------------------------------------------------
// block merge: out = tanh(f1 z1 + f2 z2) (SpatialGraphConv :143-146, SepTemporal_Block :196-199)
// ------------------------------------------------------------------------------------------
struct MergeCoef {
  float sc1, sh1, mu1, rs1, sc2, sh2, mu2, rs2;
};

F3_DEV float drop_f(const float* fS, const float* fT, int n, int t, int v, int T, int V) {
  return fS ? fS[n * V + v] * fT[n * T + t] : 1.f;
}

__global__ __launch_bounds__(256) void mu_merge_fwd_kernel(MergeArgs a) {
  __shared__ float sc1[256], sh1[256], sc2[256], sh2[256];
  for (int c = threadIdx.x; c < a.C; c += blockDim.x) {
    float m, r;
    bn_coeff(a.bn1, c, sc1[c], sh1[c], m, r);
    if (a.bn2_on) bn_coeff(a.bn2, c, sc2[c], sh2[c], m, r);
    else { sc2[c] = 1.f; sh2[c] = 0.f; }
  }
  __syncthreads();
  const long long R = (long long)a.N * a.T * a.V;
  const int nq = a.C / 4;
  for (long long i = blockIdx.x * 256LL + threadIdx.x; i < R * nq; i += (long long)gridDim.x * 256) {
    const long long r = i / nq;
    const int c = (int)(i - r * nq) * 4;
    const int v = (int)(r % a.V), t = (int)((r / a.V) % a.T), n = (int)(r / ((long long)a.V * a.T));
    const float f1 = drop_f(a.fS1, a.fT1, n, t, v, a.T, a.V), f2 = drop_f(a.fS2, a.fT2, n, t, v, a.T, a.V);
    const f32x4 u1 = ld4(a.u1 + i * 4), u2 = ld4(a.u2 + i * 4);
    f32x4 o;
#pragma unroll
    for (int e = 0; e < 4; ++e)
      o[e] = tanhf(f1 * fmaf(u1[e], sc1[c + e], sh1[c + e]) + f2 * fmaf(u2[e], sc2[c + e], sh2[c + e]));
    st4(a.out + i * 4, o);
  }
}

__global__ __launch_bounds__(256) void mu_merge_bwd_reduce_kernel(MergeArgs a) {
  __shared__ float sc1[256], sh1[256], mu1[256], rs1[256], sc2[256], sh2[256], mu2[256], rs2[256];
  for (int c = threadIdx.x; c < a.C; c += blockDim.x) {
    bn_coeff(a.bn1, c, sc1[c], sh1[c], mu1[c], rs1[c]);
    if (a.bn2_on) bn_coeff(a.bn2, c, sc2[c], sh2[c], mu2[c], rs2[c]);
    else { sc2[c] = 1.f; sh2[c] = 0.f; mu2[c] = 0.f; rs2[c] = 1.f; }
  }
  __syncthreads();
  const QuadLayout L(a.C);
  float p1[4] = {0.f, 0.f, 0.f, 0.f}, q1[4] = {0.f, 0.f, 0.f, 0.f};
  float p2[4] = {0.f, 0.f, 0.f, 0.f}, q2[4] = {0.f, 0.f, 0.f, 0.f};
  const long long R = (long long)a.N * a.T * a.V;
  if (L.act) {
    const int c0 = 4 * L.q;
    for (long long r = (long long)blockIdx.x * L.rs + L.rl; r < R; r += (long long)gridDim.x * L.rs) {
      const int v = (int)(r % a.V), t = (int)((r / a.V) % a.T), n = (int)(r / ((long long)a.V * a.T));
      const float f1 = drop_f(a.fS1, a.fT1, n, t, v, a.T, a.V), f2 = drop_f(a.fS2, a.fT2, n, t, v, a.T, a.V);
      const f32x4 u1 = ld4(a.u1 + (size_t)r * a.C + c0), u2 = ld4(a.u2 + (size_t)r * a.C + c0);
      const f32x4 go = ld4(a.dout + (size_t)r * a.C + c0);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int c = c0 + e;
        const float o = tanhf(f1 * fmaf(u1[e], sc1[c], sh1[c]) + f2 * fmaf(u2[e], sc2[c], sh2[c]));
        const float dp = go[e] * (1.f - o * o);
        const float dz1 = dp * f1, dz2 = dp * f2;
        p1[e] += dz1;
        q1[e] = fmaf(dz1, (u1[e] - mu1[c]) * rs1[c], q1[e]);
        p2[e] += dz2;
        q2[e] = fmaf(dz2, (u2[e] - mu2[c]) * rs2[c], q2[e]);
      }
    }
  }
  channel_flush(a.C, L, p1, q1, a.lanes);
  if (a.bn2_on) {
    __syncthreads();
    channel_flush(a.C, L, p2, q2, a.lanes + kLaneFloats);
  }
}

__global__ __launch_bounds__(256) void mu_merge_bwd_apply_kernel(MergeArgs a) {
  __shared__ float sc1[256], sh1[256], mu1[256], rs1[256], sc2[256], sh2[256], mu2[256], rs2[256];
  __shared__ float m11[256], m12[256], m21[256], m22[256];
  const long long R = (long long)a.N * a.T * a.V;
  for (int c = threadIdx.x; c < a.C; c += blockDim.x) {
    bn_coeff(a.bn1, c, sc1[c], sh1[c], mu1[c], rs1[c]);
    m11[c] = (float)(a.s1_dz[c] / (double)R);
    m12[c] = (float)(a.s1_dzx[c] / (double)R);
    if (blockIdx.x == 0) {
      a.g_gamma1[c] += (float)a.s1_dzx[c];
      a.g_beta1[c] += (float)a.s1_dz[c];
    }
    if (a.bn2_on) {
      bn_coeff(a.bn2, c, sc2[c], sh2[c], mu2[c], rs2[c]);
      m21[c] = (float)(a.s2_dz[c] / (double)R);
      m22[c] = (float)(a.s2_dzx[c] / (double)R);
      if (blockIdx.x == 0) {
        a.g_gamma2[c] += (float)a.s2_dzx[c];
        a.g_beta2[c] += (float)a.s2_dz[c];
      }
    } else {
      sc2[c] = 1.f; sh2[c] = 0.f;
    }
  }
  __syncthreads();
  const int nq = a.C / 4;
  for (long long i = blockIdx.x * 256LL + threadIdx.x; i < R * nq; i += (long long)gridDim.x * 256) {
    const long long r = i / nq;
    const int c0 = (int)(i - r * nq) * 4;
    const int v = (int)(r % a.V), t = (int)((r / a.V) % a.T), n = (int)(r / ((long long)a.V * a.T));
    const float f1 = drop_f(a.fS1, a.fT1, n, t, v, a.T, a.V), f2 = drop_f(a.fS2, a.fT2, n, t, v, a.T, a.V);
    const f32x4 u1 = ld4(a.u1 + i * 4), u2 = ld4(a.u2 + i * 4), go = ld4(a.dout + i * 4);
    f32x4 d1, d2;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int c = c0 + e;
      const float o = tanhf(f1 * fmaf(u1[e], sc1[c], sh1[c]) + f2 * fmaf(u2[e], sc2[c], sh2[c]));
      const float dp = go[e] * (1.f - o * o);
      const float dz1 = dp * f1, dz2 = dp * f2;
      d1[e] = sc1[c] * (dz1 - m11[c] - (u1[e] - mu1[c]) * rs1[c] * m12[c]);
      d2[e] = a.bn2_on ? sc2[c] * (dz2 - m21[c] - (u2[e] - mu2[c]) * rs2[c] * m22[c]) : dz2;
    }
    st4(a.du1 + i * 4, d1);
    if (a.du2_add) d2 += ld4(a.du2 + i * 4);
    st4(a.du2 + i * 4, d2);
  }
}

// ------------------------------------------------------------------------------------------
// inputs, embedding ReLU backward
// ------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void mu_tokens_kernel(TokenArgs a) {
  const long long R = (long long)a.N * a.T * a.V;
  for (long long r = blockIdx.x * 256LL + threadIdx.x; r < R; r += (long long)gridDim.x * 256) {
    const int v = (int)(r % a.V), t = (int)((r / a.V) % a.T), n = (int)(r / ((long long)a.V * a.T));
    const size_t plane = (size_t)a.T * a.V;
    const float* xn = a.x + (size_t)n * 3 * plane;
    const float x0 = xn[(size_t)t * a.V + v], x1 = xn[plane + (size_t)t * a.V + v], x2 = xn[2 * plane + (size_t)t * a.V + v];
    st4(a.pos + r * 4, f32x4{x0, x1, x2, 0.f});
    if (t < a.T - 1) {  // mot = x[:, :2, :-1] - x[:, :2, 1:]
      const long long rm = ((long long)n * (a.T - 1) + t) * a.V + v;
      st4(a.mot + rm * 4, f32x4{x0 - xn[(size_t)(t + 1) * a.V + v], x1 - xn[plane + (size_t)(t + 1) * a.V + v], 0.f, 0.f});
    }
  }
}

__global__ __launch_bounds__(256) void mu_relu_bwd_kernel(ReluBwdArgs a) {
  for (long long i = blockIdx.x * 256LL + threadIdx.x; i < a.n / 4; i += (long long)gridDim.x * 256) {
    const f32x4 y = ld4(a.y + i * 4), d = ld4(a.d + i * 4);
    f32x4 o;
#pragma unroll
    for (int e = 0; e < 4; ++e) o[e] = y[e] > 0.f ? d[e] : 0.f;
    st4(a.out + i * 4, o);
  }
}

// ------------------------------------------------------------------------------------------
// head (Model.forward :575-589 + Classification_Module :476-490): one workgroup per clip
// ------------------------------------------------------------------------------------------
constexpr int HID = 128;

__global__ __launch_bounds__(256) void mu_head_fwd_kernel(HeadArgs a) {
  __shared__ float feat[2 * 256 + 4], z[HID], red[256];
  const int n = blockIdx.x, F = 2 * a.Cs + 3;
  for (int c = threadIdx.x; c < a.Cs; c += blockDim.x) {
    float s1 = 0.f, s2 = 0.f;
    const float* y1 = a.y1 + (size_t)n * a.TV1 * a.Cs + c;
    const float* y2 = a.y2 + (size_t)n * a.TV2 * a.Cs + c;
    for (int r = 0; r < a.TV1; ++r) s1 += y1[(size_t)r * a.Cs];
    for (int r = 0; r < a.TV2; ++r) s2 += y2[(size_t)r * a.Cs];
    feat[c] = s1 / (float)a.TV1;
    feat[a.Cs + c] = s2 / (float)a.TV2;
  }
  if (threadIdx.x < 3) {  // res_pos = mean of the raw positions over (T, V)
    float s = 0.f;
    const float* xp = a.x + ((size_t)n * 3 + threadIdx.x) * a.TVx;
    for (int i = 0; i < a.TVx; ++i) s += xp[i];
    feat[2 * a.Cs + threadIdx.x] = s / (float)a.TVx;
  }
  __syncthreads();
  for (int k = threadIdx.x; k < F; k += blockDim.x) a.feat[(size_t)n * F + k] = feat[k];
  float hval = 0.f;
  if (threadIdx.x < HID) {
    const int j = threadIdx.x;
    float acc = a.b1[j];
    const float* w = a.w1 + (size_t)j * F;
    for (int k = 0; k < F; ++k) acc = fmaf(w[k], feat[k], acc);
    a.z1[(size_t)n * HID + j] = acc;
    hval = acc > 0.f ? acc : kLeaky * acc;
  }
  red[threadIdx.x] = threadIdx.x < HID ? hval : 0.f;
  __syncthreads();
  if (threadIdx.x == 0) {
    float s = 0.f;
    for (int j = 0; j < HID; ++j) s += red[j];
    const float mean = s / HID;
    float q = 0.f;
    for (int j = 0; j < HID; ++j) q += (red[j] - mean) * (red[j] - mean);
    const float rstd = 1.f / sqrtf(q / HID + 1e-5f);
    a.stat[2 * n] = mean;
    a.stat[2 * n + 1] = rstd;
    z[0] = mean;
    z[1] = rstd;
  }
  __syncthreads();
  const float mean = z[0], rstd = z[1];
  __syncthreads();
  if (threadIdx.x < HID) {
    const int j = threadIdx.x;
    float l = (hval - mean) * rstd * a.lnw[j] + a.lnb[j];
    l = l > 0.f ? l : kLeaky * l;
    if (a.drop_p > 0.f) l = uni24(a.seed ^ 0x1B873593u, 0, (unsigned)(n * HID + j)) >= a.drop_p ? l / (1.f - a.drop_p) : 0.f;
    a.h[(size_t)n * HID + j] = l;
    z[j] = l;
  }
  __syncthreads();
  if (threadIdx.x < a.NC) {
    const int k = threadIdx.x;
    float o = a.b2[k];
    for (int j = 0; j < HID; ++j) o = fmaf(a.w2[k * HID + j], z[j], o);
    a.out[(size_t)n * a.NC + k] = o;
  }
}

__global__ __launch_bounds__(256) void mu_head_bwd_kernel(HeadArgs a) {
  __shared__ float dz[HID], red[2][HID], dfeat[2 * 256 + 4];
  const int n = blockIdx.x, F = 2 * a.Cs + 3;
  const float mean = a.stat[2 * n], rstd = a.stat[2 * n + 1];
  float xh = 0.f, dxh = 0.f, z1 = 0.f;
  if (threadIdx.x < HID) {
    const int j = threadIdx.x;
    float dh = 0.f;
    for (int k = 0; k < a.NC; ++k) dh = fmaf(a.dout[(size_t)n * a.NC + k], a.w2[k * HID + j], dh);
    if (a.drop_p > 0.f)
      dh = uni24(a.seed ^ 0x1B873593u, 0, (unsigned)(n * HID + j)) >= a.drop_p ? dh / (1.f - a.drop_p) : 0.f;
    z1 = a.z1[(size_t)n * HID + j];
    const float h1 = z1 > 0.f ? z1 : kLeaky * z1;
    xh = (h1 - mean) * rstd;
    const float l = xh * a.lnw[j] + a.lnb[j];
    const float dl = dh * (l > 0.f ? 1.f : kLeaky);
    atomicAdd(a.g_lnw + j, dl * xh);
    atomicAdd(a.g_lnb + j, dl);
    dxh = dl * a.lnw[j];
    red[0][j] = dxh;
    red[1][j] = dxh * xh;
  }
  __syncthreads();
  if (threadIdx.x < HID) {
    float s0 = 0.f, s1 = 0.f;
    for (int j = 0; j < HID; ++j) {
      s0 += red[0][j];
      s1 += red[1][j];
    }
    const int j = threadIdx.x;
    const float dh1 = rstd * (dxh - s0 / HID - xh * s1 / HID);
    const float d = dh1 * (z1 > 0.f ? 1.f : kLeaky);
    dz[j] = d;
    a.dz1[(size_t)n * HID + j] = d;
  }
  __syncthreads();
  for (int k = threadIdx.x; k < F; k += blockDim.x) {
    float s = 0.f;
    for (int j = 0; j < HID; ++j) s = fmaf(dz[j], a.w1[(size_t)j * F + k], s);
    dfeat[k] = s;
  }
  __syncthreads();
  const int nq = a.Cs / 4;
  for (int e = threadIdx.x; e < a.TV1 * nq; e += blockDim.x) {
    const int r = e / nq, c = (e - r * nq) * 4;
    const float s = 1.f / (float)a.TV1;
    st4(a.dy1 + ((size_t)n * a.TV1 + r) * a.Cs + c, f32x4{dfeat[c] * s, dfeat[c + 1] * s, dfeat[c + 2] * s, dfeat[c + 3] * s});
  }
  for (int e = threadIdx.x; e < a.TV2 * nq; e += blockDim.x) {
    const int r = e / nq, c = (e - r * nq) * 4;
    const float s = 1.f / (float)a.TV2;
    const float* d = dfeat + a.Cs;
    st4(a.dy2 + ((size_t)n * a.TV2 + r) * a.Cs + c, f32x4{d[c] * s, d[c + 1] * s, d[c + 2] * s, d[c + 3] * s});
  }
}

static int grid_for(long long items, int cap = 2048) {
  const long long g = (items + 255) / 256;
  return (int)(g < 1 ? 1 : (g > cap ? cap : g));
}
static int quad_grid(long long rows, int C, int cap) {
  const long long rs = 256 / (C / 4);
  const long long g = (rows + rs * 8 - 1) / (rs * 8);  // >= 8 rows per row lane
  return (int)(g < 1 ? 1 : (g > cap ? cap : g));
}

}  // namespace mu
}  // namespace f3

using namespace f3;
using namespace f3::mu;

static bool c_ok(int C) { return C % 4 == 0 && C >= 16 && C <= 256; }

#define F3_TRY_MU(x)              \
  do {                            \
    const int _st = (x);          \
    if (_st != F3_OK) return _st; \
  } while (0)


static int lane_finalize(float* lanes, int C, double* g1, double* g2, hipStream_t s) {
  hipLaunchKernelGGL(mu_lane_finalize_kernel, dim3((2 * C + kFinCols - 1) / kFinCols), dim3(kFinCols * kFinGroups), 0,
                     s, lanes, C, g1, g2);
  F3_LAUNCH_CHECK();
  return F3_OK;
}

int f3_mu_dwconv_part_rows(const DwConvArgs* a) {
  return quad_grid((long long)a->N * a->T_out * a->V, a->C, 512);
}

int f3_mu_dwconv_fwd(const DwConvArgs* a, hipStream_t s) {
  if (!c_ok(a->C)) return F3_EINVAL;
  const long long total = (long long)a->N * a->V * (a->C / 4) * ((a->T_out + kDwChunk - 1) / kDwChunk);
  if (total >= (1LL << 31)) return F3_EINVAL;
  // 256 threads per workgroup (rounded down to a multiple of the quad count, so a thread's channel
  // quad stays fixed over its grid-stride walk)
  const int nq = a->C / 4, block = 256 / nq * nq;
  const long long want = (total + block - 1) / block;
  // The workgroup cap. Measured (C=128, V=14, T=30, B=256, k3): the BN-sum epilogue costs ~2.3 ns per
  // wave of the grid at the launch's end (1024 x 256 threads: 28.3 vs 18.8 us without sums; 512 x
  // 256: 24.9 vs 19.9; 512-thread blocks or one wave issuing the lane adds: the same), so 512
  // workgroups of 256 threads, at most kLanes of them, each storing its BN partial row into its own
  // lane row (plain stores; the finalize adds the rows) instead of memory-side adds: k3/s1 48.8 ->
  // 51.3 % of HBM, k5/s2 46.4 -> 45.7 %, step unchanged (profiles/r04_musa_dwstore_ab.txt)
  constexpr int cap = 512;
  const bool st_rows = a->sum != nullptr;
  const int grid = (int)std::min<long long>(want, st_rows ? std::min(cap, kLanes) : cap);
  DwConvArgs b = *a;
  b.grid = grid;
  b.block = block;
  a = &b;
#define MU_DWF(K_, S_)                                                                                   \
  if (a->K == K_ && a->S == S_) {                                                                        \
    if (st_rows) hipLaunchKernelGGL((mu_dwconv_fwd_kernel<K_, S_, true>), dim3(grid), dim3(block), 0, s, *a); \
    else hipLaunchKernelGGL((mu_dwconv_fwd_kernel<K_, S_, false>), dim3(grid), dim3(block), 0, s, *a);      \
  } else
  MU_DWF(1, 1) MU_DWF(3, 1) MU_DWF(5, 1) MU_DWF(3, 2) MU_DWF(5, 2) return F3_EINVAL;
#undef MU_DWF
  F3_LAUNCH_CHECK();
  if (a->sum) return lane_finalize(a->lanes, a->C, a->sum, a->sumsq, s);
  return F3_OK;
}

int f3_mu_dwconv_bwd(DwConvArgs* a, hipStream_t s) {
  if (!c_ok(a->C)) return F3_EINVAL;
  const int gx = quad_grid((long long)a->N * a->T_in * a->V, a->C, 2048);
  const int gw = f3_mu_dwconv_part_rows(a);
  a->part_rows = gw;
  switch (a->K) {
#define MU_DW(K)                                                                          \
  case K:                                                                                 \
    if (a->dx) hipLaunchKernelGGL(mu_dwconv_dx_kernel<K>, dim3(gx), dim3(256), 0, s, *a); \
    hipLaunchKernelGGL(mu_dwconv_dw_kernel<K>, dim3(gw), dim3(256), 0, s, *a);           \
    break;
    MU_DW(1)
    MU_DW(3)
    MU_DW(5)
#undef MU_DW
    default: return F3_EINVAL;
  }
  F3_LAUNCH_CHECK();
  return F3_OK;
}

int f3_mu_bn_act(const BnActArgs* a, hipStream_t s) {
  if (!c_ok(a->C)) return F3_EINVAL;
  hipLaunchKernelGGL(mu_bn_act_kernel, dim3(grid_for(a->R * a->C / 4)), dim3(256), 0, s, *a);
  F3_LAUNCH_CHECK();
  return F3_OK;
}

int f3_mu_bn_act_bwd(const BnActBwdArgs* a, hipStream_t s) {
  if (!c_ok(a->C)) return F3_EINVAL;
  BnActBwdArgs b = *a;
  b.grid = quad_grid(a->R, a->C, 1024);
  hipLaunchKernelGGL(mu_bn_act_bwd_reduce_kernel, dim3(b.grid), dim3(256), 0, s, b);
  F3_LAUNCH_CHECK();
  F3_TRY_MU(lane_finalize(a->lanes, a->C, a->s_dz, a->s_dzx, s));
  hipLaunchKernelGGL(mu_bn_act_bwd_apply_kernel, dim3(grid_for(a->R * a->C / 4)), dim3(256), 0, s, *a);
  F3_LAUNCH_CHECK();
  return F3_OK;
}

int f3_mu_colstat(const ColStatArgs* a, hipStream_t s) {
  if (!c_ok(a->C)) return F3_EINVAL;
  ColStatArgs b = *a;
  b.grid = quad_grid(a->R, a->C, 1024);
  hipLaunchKernelGGL(mu_colstat_kernel, dim3(b.grid), dim3(256), 0, s, b);
  F3_LAUNCH_CHECK();
  return lane_finalize(a->lanes, a->C, a->sum, a->sumsq, s);
}

int f3_mu_absstat(const AbsStatArgs* a, hipStream_t s) {
  if (!c_ok(a->C)) return F3_EINVAL;
  hipLaunchKernelGGL(mu_absstat_kernel, dim3(quad_grid(a->R, a->C, 2048)), dim3(256), 0, s, *a);
  F3_LAUNCH_CHECK();
  return F3_OK;
}

int f3_mu_dropmask_scratch_floats(int N, int T, int V) { return 2 * N * V + N * T + 3 * N; }

int f3_mu_dropmask(const DropMaskArgs* a, hipStream_t s) {
  const size_t lds = sizeof(float) * 2 * (size_t)a->N * a->T;
  if (a->V > 32 || a->T > 64 || a->T * a->V > 64 * 32 || lds > 150 * 1024 || !a->scr) return F3_EINVAL;
  F3_LDS_LIMIT(mu_drop_final_kernel, 150 * 1024);
  hipLaunchKernelGGL(mu_drop_s_kernel, dim3(a->N), dim3(256), 0, s, *a);
  F3_LAUNCH_CHECK();
  hipLaunchKernelGGL(mu_drop_t_kernel, dim3(a->N), dim3(256), 0, s, *a);
  F3_LAUNCH_CHECK();
  hipLaunchKernelGGL(mu_drop_final_kernel, dim3(1), dim3(1024), lds, s, *a);
  F3_LAUNCH_CHECK();
  return F3_OK;
}

int f3_mu_merge_fwd(const MergeArgs* a, hipStream_t s) {
  if (!c_ok(a->C)) return F3_EINVAL;
  hipLaunchKernelGGL(mu_merge_fwd_kernel, dim3(grid_for((long long)a->N * a->T * a->V * a->C / 4)), dim3(256), 0, s, *a);
  F3_LAUNCH_CHECK();
  return F3_OK;
}

int f3_mu_merge_bwd(const MergeArgs* a, hipStream_t s) {
  if (!c_ok(a->C)) return F3_EINVAL;
  const long long R = (long long)a->N * a->T * a->V;
  MergeArgs b = *a;
  b.grid = quad_grid(R, a->C, 1024);
  hipLaunchKernelGGL(mu_merge_bwd_reduce_kernel, dim3(b.grid), dim3(256), 0, s, b);
  F3_LAUNCH_CHECK();
  F3_TRY_MU(lane_finalize(a->lanes, a->C, a->s1_dz, a->s1_dzx, s));
  if (a->bn2_on) F3_TRY_MU(lane_finalize(a->lanes + kLaneFloats, a->C, a->s2_dz, a->s2_dzx, s));
  hipLaunchKernelGGL(mu_merge_bwd_apply_kernel, dim3(grid_for(R * a->C / 4)), dim3(256), 0, s, *a);
  F3_LAUNCH_CHECK();
  return F3_OK;
}

int f3_mu_tokens(const TokenArgs* a, hipStream_t s) {
  hipLaunchKernelGGL(mu_tokens_kernel, dim3(grid_for((long long)a->N * a->T * a->V)), dim3(256), 0, s, *a);
  F3_LAUNCH_CHECK();
  return F3_OK;
}

int f3_mu_relu_bwd(const ReluBwdArgs* a, hipStream_t s) {
  hipLaunchKernelGGL(mu_relu_bwd_kernel, dim3(grid_for(a->n / 4)), dim3(256), 0, s, *a);
  F3_LAUNCH_CHECK();
  return F3_OK;
}

int f3_mu_head_fwd(const HeadArgs* a, hipStream_t s) {
  if (a->Cs > 256 || a->NC > 64) return F3_EINVAL;
  hipLaunchKernelGGL(mu_head_fwd_kernel, dim3(a->N), dim3(256), 0, s, *a);
  F3_LAUNCH_CHECK();
  return F3_OK;
}

int f3_mu_head_bwd(const HeadArgs* a, hipStream_t s) {
  if (a->Cs > 256 || a->NC > 64) return F3_EINVAL;
  hipLaunchKernelGGL(mu_head_bwd_kernel, dim3(a->N), dim3(256), 0, s, *a);
  F3_LAUNCH_CHECK();
  return F3_OK;
}
