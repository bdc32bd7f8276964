// SkeletonTransformer (BASELINE config 5) kernels for gfx950.
// Reference (file:line in /root/reference/skeleton_transformer.py):
//   embedding Linear(3,16)-GELU-Linear(16,32)-GELU            371-376, 421
//   RelativePositionalMultiHeadSelfAttention core             130-157
//   B2TSpatialTenporalTransformerBlock residual/BN3d/FFN      229-248
//   global pool + mean over persons + 1x1 Conv2d classifier   425-435
// Token rows are channels-last [N][M][T][V][32] fp32 (sktr.h). The attention core runs one
// workgroup per sequence: the sequence's k|v rows (and q|dO in the backward) are staged in LDS
// with coalesced 16-B loads, one thread per (head, query) row keeps q / o / dq in registers and
// its score / probability row in LDS (L <= 32, compile-time), and the backward's column sums
// (dk, dv, table) read the probability / score-gradient tiles back from LDS. Elementwise
// passes are float4 per thread.
#include <math.h>

#include "sktr.h"

namespace f3 {
namespace sk {

F3_DEV float gelu_f(float x) { return 0.5f * x * (1.f + erff(x * 0.70710678118654752f)); }
F3_DEV float gelu_d(float x) {
  return 0.5f * (1.f + erff(x * 0.70710678118654752f)) + x * 0.39894228040143268f * expf(-0.5f * x * x);
}

// counter-hash dropout mask, bit-for-bit the oracle's dropout_keep (oracle/sktr_cpu.py)
F3_DEV unsigned mix32(unsigned x) {
  x ^= x >> 16;
  x *= 0x7FEB352Du;
  x ^= x >> 15;
  x *= 0x846CA68Bu;
  x ^= x >> 16;
  return x;
}
F3_DEV unsigned drop_base(unsigned seed, int block) { return mix32(seed ^ ((unsigned)block * 0x9E3779B9u)); }
F3_DEV unsigned drop_thr(float p) {
  const float t = rintf(p * 16777216.f);
  return t >= 16777216.f ? 16777216u : (unsigned)t;
}
F3_DEV bool drop_keep(unsigned base, unsigned thr, unsigned e) { return (mix32(e + base) >> 8) >= thr; }

// ------------------------------------------------------------------------------------------
// embedding (skeleton_transformer.py:371-376): per token x[3] -> gelu(W1 x + b1)[16] ->
// gelu(W2 h + b2)[32]. The forward keeps the token-major input, both pre-activations and the
// hidden activation for the backward, whose weight gradients run on the shared wgrad GEMM.
// ------------------------------------------------------------------------------------------
struct EmbedSave {
  float* xt;   // [R][4] (4th column zero)
  float* a1;   // [R][16]
  float* h1;   // [R][16]
  float* a2;   // [R][32]
  float* da1;  // bwd [R][16]
  float* da2;  // bwd [R][32]
};

__global__ __launch_bounds__(256) void sk_embed_fwd_kernel(EmbedArgs a, EmbedSave sv) {
  __shared__ float w1[HID0 * CIN], b1[HID0], w2[EMB * HID0], b2[EMB];
  for (int e = threadIdx.x; e < EMB * HID0; e += 256) {
    w2[e] = a.w2[e];
    if (e < HID0 * CIN) w1[e] = a.w1[e];
    if (e < HID0) b1[e] = a.b1[e];
    if (e < EMB) b2[e] = a.b2[e];
  }
  __syncthreads();
  const long long R = (long long)a.N * a.M * a.T * a.V;
  for (long long r = blockIdx.x * 256LL + threadIdx.x; r < R; r += (long long)gridDim.x * 256) {
    const int v = (int)(r % a.V);
    const long long q = r / a.V;
    const int t = (int)(q % a.T);
    const long long nm = q / a.T;
    const int n = (int)(nm / a.M), m = (int)(nm - (long long)n * a.M);
    float x[CIN];
#pragma unroll
    for (int c = 0; c < CIN; ++c) x[c] = a.x[(((size_t)(n * CIN + c) * a.T + t) * a.V + v) * a.M + m];
    *reinterpret_cast<f32x4*>(sv.xt + r * 4) = f32x4{x[0], x[1], x[2], 0.f};
    float h[HID0];
#pragma unroll
    for (int k = 0; k < HID0; ++k) {
      float acc = b1[k];
#pragma unroll
      for (int c = 0; c < CIN; ++c) acc = fmaf(w1[k * CIN + c], x[c], acc);
      h[k] = acc;
    }
#pragma unroll
    for (int k = 0; k < HID0; k += 4) {
      *reinterpret_cast<f32x4*>(sv.a1 + r * HID0 + k) = f32x4{h[k], h[k + 1], h[k + 2], h[k + 3]};
#pragma unroll
      for (int u = 0; u < 4; ++u) h[k + u] = gelu_f(h[k + u]);
      *reinterpret_cast<f32x4*>(sv.h1 + r * HID0 + k) = f32x4{h[k], h[k + 1], h[k + 2], h[k + 3]};
    }
#pragma unroll 1
    for (int j0 = 0; j0 < EMB; j0 += 4) {
      f32x4 pre, out;
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        float acc = b2[j0 + u];
#pragma unroll
        for (int k = 0; k < HID0; ++k) acc = fmaf(w2[(j0 + u) * HID0 + k], h[k], acc);
        pre[u] = acc;
        out[u] = gelu_f(acc);
      }
      *reinterpret_cast<f32x4*>(sv.a2 + r * EMB + j0) = pre;
      *reinterpret_cast<f32x4*>(a.y + r * EMB + j0) = out;
    }
  }
}

// dA2 = dy * gelu'(a2); dA1 = (W2^T dA2) * gelu'(a1)
__global__ __launch_bounds__(256) void sk_embed_bwd_kernel(EmbedArgs a, EmbedSave sv) {
  __shared__ float w2[EMB * HID0];
  for (int e = threadIdx.x; e < EMB * HID0; e += 256) w2[e] = a.w2[e];
  __syncthreads();
  const long long R = (long long)a.N * a.M * a.T * a.V;
  for (long long r = blockIdx.x * 256LL + threadIdx.x; r < R; r += (long long)gridDim.x * 256) {
    float dh[HID0];
#pragma unroll
    for (int k = 0; k < HID0; ++k) dh[k] = 0.f;
#pragma unroll 1
    for (int j0 = 0; j0 < EMB; j0 += 4) {
      const f32x4 dy = *reinterpret_cast<const f32x4*>(a.dy + r * EMB + j0);
      const f32x4 pre = *reinterpret_cast<const f32x4*>(sv.a2 + r * EMB + j0);
      f32x4 d;
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        d[u] = dy[u] * gelu_d(pre[u]);
#pragma unroll
        for (int k = 0; k < HID0; ++k) dh[k] = fmaf(w2[(j0 + u) * HID0 + k], d[u], dh[k]);
      }
      *reinterpret_cast<f32x4*>(sv.da2 + r * EMB + j0) = d;
    }
#pragma unroll
    for (int k = 0; k < HID0; k += 4) {
      const f32x4 pre = *reinterpret_cast<const f32x4*>(sv.a1 + r * HID0 + k);
      f32x4 d;
#pragma unroll
      for (int u = 0; u < 4; ++u) d[u] = dh[k + u] * gelu_d(pre[u]);
      *reinterpret_cast<f32x4*>(sv.da1 + r * HID0 + k) = d;
    }
  }
}

// ------------------------------------------------------------------------------------------
// attention core (skeleton_transformer.py:143-151): per (sequence, head)
//   S = (q k^T) * scale + q . table[i - j + L - 1];  P = softmax_j(S);  o = P v
// ------------------------------------------------------------------------------------------
F3_DEV long long seq_row(const AttnArgs& a, int s, int l, int L) {
  if (a.temporal) {
    const int nm = s / a.V, v = s - nm * a.V;
    return ((long long)nm * a.T + l) * a.V + v;
  }
  return (long long)s * L + l;
}

// one thread per (head, query) row, rounded up to whole waves (the launch's block size)
constexpr int attn_threads(int L) { return (HEADS * L + 63) / 64 * 64; }

// 16-wide rows in LDS are read as four 16-B vectors (ds_read_b128)
F3_DEV f32x4 l4(const float* p) { return *reinterpret_cast<const f32x4*>(p); }
F3_DEV void load16(f32x4 (&r)[4], const float* p) {
#pragma unroll
  for (int u = 0; u < 4; ++u) r[u] = l4(p + 4 * u);
}
F3_DEV float dot16(const f32x4 (&a)[4], const float* p) {  // four independent chains
  f32x4 acc = a[0] * l4(p);
#pragma unroll
  for (int u = 1; u < 4; ++u) {
    const f32x4 b = l4(p + 4 * u);
#pragma unroll
    for (int e = 0; e < 4; ++e) acc[e] = fmaf(a[u][e], b[e], acc[e]);
  }
  return (acc[0] + acc[1]) + (acc[2] + acc[3]);
}
F3_DEV void axpy16(f32x4 (&acc)[4], float s, const float* p) {
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const f32x4 b = l4(p + 4 * u);
#pragma unroll
    for (int e = 0; e < 4; ++e) acc[u][e] = fmaf(s, b[e], acc[u][e]);
  }
}
F3_DEV void zero16(f32x4 (&r)[4]) {
#pragma unroll
  for (int u = 0; u < 4; ++u) r[u] = f32x4{0.f, 0.f, 0.f, 0.f};
}

template <int L>
__global__ __launch_bounds__(256) void sk_attn_fwd_kernel(AttnArgs a) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  constexpr int LP = L + 1;
  float* Ks = sm;                      // [L][128]
  float* Vs = Ks + L * DM;             // [L][128]
  float* Tb = Vs + L * DM;             // [2L-1][16]
  float* Ps = Tb + (2 * L - 1) * HD;   // [H][L][L+1] score / probability rows
  const int s = blockIdx.x;
  {  // all of the thread's 16-B loads in flight before the LDS writes
    constexpr int NPT = (L * 64 + attn_threads(L) - 1) / attn_threads(L);
    f32x4 buf[NPT];
#pragma unroll
    for (int q = 0; q < NPT; ++q) {
      const int e = min((int)threadIdx.x + q * (int)blockDim.x, L * 64 - 1);
      const int l = e >> 6, c4 = e & 63;
      buf[q] = *reinterpret_cast<const f32x4*>(a.qkv + seq_row(a, s, l, L) * QKV + DM + c4 * 4);
    }
#pragma unroll
    for (int q = 0; q < NPT; ++q) {
      const int e = threadIdx.x + q * blockDim.x;
      if (e < L * 64) {
        const int l = e >> 6, c4 = e & 63;
        float* dst = c4 < 32 ? Ks + l * DM + c4 * 4 : Vs + l * DM + (c4 - 32) * 4;
        *reinterpret_cast<f32x4*>(dst) = buf[q];
      }
    }
  }
  for (int e = threadIdx.x; e < (2 * L - 1) * HD; e += blockDim.x) Tb[e] = a.table[e];
  __syncthreads();
  const int h = threadIdx.x / L, i = threadIdx.x - h * L;
  if (h >= HEADS) return;
  const long long ri = seq_row(a, s, i, L);
  f32x4 q[4];
  load16(q, a.qkv + ri * QKV + h * HD);
  float* Sr = Ps + (h * L + i) * LP;
  float mx = -INFINITY;
#pragma unroll 2
  for (int j = 0; j < L; ++j) {
    const float sc = dot16(q, Ks + j * DM + h * HD) * a.scale + dot16(q, Tb + (i - j + L - 1) * HD);
    Sr[j] = sc;
    mx = fmaxf(mx, sc);
  }
  float sum = 0.f;
#pragma unroll 2
  for (int j = 0; j < L; ++j) {
    const float e = expf(Sr[j] - mx);
    Sr[j] = e;
    sum += e;
  }
  const float inv = 1.f / sum;
  f32x4 o[4];
  zero16(o);
#pragma unroll 2
  for (int j = 0; j < L; ++j) axpy16(o, Sr[j] * inv, Vs + j * DM + h * HD);
#pragma unroll
  for (int u = 0; u < 4; ++u) *reinterpret_cast<f32x4*>(a.o + ri * DM + h * HD + 4 * u) = o[u];
}

template <int L>
constexpr size_t attn_fwd_lds() {
  return sizeof(float) * (2 * L * DM + (2 * L - 1) * HD + HEADS * L * (L + 1));
}
template <int L>
constexpr size_t attn_bwd_lds() {
  return sizeof(float) * (4 * L * DM + (2 * L - 1) * HD + 2 * HEADS * L * (L + 1));
}

// backward: phase 1 rows (h, i): P, dP = dO v^T, dS = P (dP - rowsum(P dP)), dq;
// phase 2 columns (h, j): dk = scale dS^T q, dv = P^T dO; phase 3 (r, h): the table gradient
// sum_{i, j = i - r + L - 1} dS[h][i][j] q_i, summed over heads with LDS atomics.
template <int L>
__global__ __launch_bounds__(256) void sk_attn_bwd_kernel(AttnArgs a) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  float* Qs = sm;                       // [L][128]
  float* Ks = Qs + L * DM;
  float* Vs = Ks + L * DM;
  float* Os = Vs + L * DM;              // dO
  float* Tb = Os + L * DM;              // [2L-1][16]; the table gradient after phase 1
  float* Ps = Tb + (2 * L - 1) * HD;    // [H][L][L+1]
  float* Ss = Ps + HEADS * L * (L + 1); // [H][L][L+1]
  constexpr int LP = L + 1, NT = (2 * L - 1) * HD;
  const int s = blockIdx.x;
  {  // all of the thread's 16-B loads in flight before the LDS writes
    constexpr int NPT = (L * 128 + attn_threads(L) - 1) / attn_threads(L);
    f32x4 buf[NPT];
#pragma unroll
    for (int q = 0; q < NPT; ++q) {
      const int e = min((int)threadIdx.x + q * (int)blockDim.x, L * 128 - 1);
      const int l = e >> 7, c4 = e & 127;
      const long long r = seq_row(a, s, l, L);
      buf[q] = c4 < 96 ? *reinterpret_cast<const f32x4*>(a.qkv + r * QKV + c4 * 4)
                       : *reinterpret_cast<const f32x4*>(a.dout + r * DM + (c4 - 96) * 4);
    }
#pragma unroll
    for (int q = 0; q < NPT; ++q) {
      const int e = threadIdx.x + q * blockDim.x;
      if (e < L * 128) {
        const int l = e >> 7, c4 = e & 127;
        float* dst = c4 < 96 ? Qs + (c4 >> 5) * L * DM + l * DM + (c4 & 31) * 4 : Os + l * DM + (c4 - 96) * 4;
        *reinterpret_cast<f32x4*>(dst) = buf[q];
      }
    }
  }
  for (int e = threadIdx.x; e < NT; e += blockDim.x) Tb[e] = a.table[e];
  __syncthreads();
  const int h = threadIdx.x / L, i = threadIdx.x - h * L;
  const bool act = h < HEADS;
  if (act) {
    f32x4 q[4], go[4];
    load16(q, Qs + i * DM + h * HD);
    load16(go, Os + i * DM + h * HD);
    float* Pr = Ps + (h * L + i) * LP;
    float* Sr = Ss + (h * L + i) * LP;
    float mx = -INFINITY;
#pragma unroll 2
    for (int j = 0; j < L; ++j) {
      const float sc = dot16(q, Ks + j * DM + h * HD) * a.scale + dot16(q, Tb + (i - j + L - 1) * HD);
      Pr[j] = sc;
      mx = fmaxf(mx, sc);
    }
    float sum = 0.f;
#pragma unroll 2
    for (int j = 0; j < L; ++j) {
      const float e = expf(Pr[j] - mx);
      Pr[j] = e;
      sum += e;
    }
    const float inv = 1.f / sum;
    float dsum = 0.f;
#pragma unroll 2
    for (int j = 0; j < L; ++j) {
      const float p = Pr[j] * inv;
      Pr[j] = p;
      const float dp = dot16(go, Vs + j * DM + h * HD);
      Sr[j] = dp;
      dsum = fmaf(p, dp, dsum);
    }
    f32x4 dq[4], dqt[4];
    zero16(dq);
    zero16(dqt);
#pragma unroll 2
    for (int j = 0; j < L; ++j) {
      const float ds = Pr[j] * (Sr[j] - dsum);
      Sr[j] = ds;
      axpy16(dq, ds, Ks + j * DM + h * HD);
      axpy16(dqt, ds, Tb + (i - j + L - 1) * HD);
    }
    const long long ri = seq_row(a, s, i, L);
#pragma unroll
    for (int u = 0; u < 4; ++u) *reinterpret_cast<f32x4*>(a.dqkv + ri * QKV + h * HD + 4 * u) = dq[u] * a.scale + dqt[u];
  }
  __syncthreads();
  if (act) {
    const int j = i;
    f32x4 dk[4], dv[4];
    zero16(dk);
    zero16(dv);
#pragma unroll 2
    for (int ii = 0; ii < L; ++ii) {
      axpy16(dk, Ss[(h * L + ii) * LP + j], Qs + ii * DM + h * HD);
      axpy16(dv, Ps[(h * L + ii) * LP + j], Os + ii * DM + h * HD);
    }
    const long long rj = seq_row(a, s, j, L);
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      *reinterpret_cast<f32x4*>(a.dqkv + rj * QKV + DM + h * HD + 4 * u) = dk[u] * a.scale;
      *reinterpret_cast<f32x4*>(a.dqkv + rj * QKV + 2 * DM + h * HD + 4 * u) = dv[u];
    }
  }
  for (int e = threadIdx.x; e < NT; e += blockDim.x) Tb[e] = 0.f;   // table gradient accumulator
  __syncthreads();
  for (int idx = threadIdx.x; idx < (2 * L - 1) * HEADS; idx += blockDim.x) {
    const int r = idx / HEADS, hh = idx - r * HEADS;
    const int i0 = max(0, r - L + 1), i1 = min(L - 1, r);
    f32x4 acc[4];
    zero16(acc);
    for (int ii = i0; ii <= i1; ++ii) axpy16(acc, Ss[(hh * L + ii) * LP + ii - r + L - 1], Qs + ii * DM + hh * HD);
#pragma unroll
    for (int u = 0; u < 4; ++u)
#pragma unroll
      for (int e = 0; e < 4; ++e) atomicAdd(Tb + r * HD + 4 * u + e, acc[u][e]);
  }
  __syncthreads();
  float* dt = a.dtab + (long long)s * NT;
  for (int e = threadIdx.x; e < NT; e += blockDim.x) dt[e] = Tb[e];
}

// ------------------------------------------------------------------------------------------
// elementwise passes over [R][32] rows (one float4 per thread; a thread's channel quad is
// fixed across its grid-stride loop, so the BN sums reduce per quad then per workgroup)
// ------------------------------------------------------------------------------------------
F3_DEV void wg_channel_sums(const float (&s1)[4], const float (&s2)[4], double* g1, double* g2) {
  __shared__ float red[2][256][4];
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    red[0][threadIdx.x][e] = s1[e];
    red[1][threadIdx.x][e] = s2[e];
  }
  __syncthreads();
  if (threadIdx.x < 64) {
    const int which = threadIdx.x >> 5, c = threadIdx.x & 31, quad = c >> 2, e = c & 3;
    double acc = 0.0;
    for (int t = quad; t < 256; t += 8) acc += (double)red[which][t][e];
    if (which == 0) {
      if (g1) atomicAdd(g1 + c, acc);
    } else {
      if (g2) atomicAdd(g2 + c, acc);
    }
  }
}

__global__ __launch_bounds__(256) void sk_resid_kernel(ResidArgs a) {
  const long long n4 = a.R * (EMB / 4);
  const unsigned base = drop_base(a.seed, a.block), thr = drop_thr(a.drop_p);
  const float dscale = a.drop_p > 0.f ? a.s / (1.f - a.drop_p) : a.s;
  float s1[4] = {0.f, 0.f, 0.f, 0.f}, s2[4] = {0.f, 0.f, 0.f, 0.f};
  for (long long i = blockIdx.x * 256LL + threadIdx.x; i < n4; i += (long long)gridDim.x * 256) {
    f32x4 u = *reinterpret_cast<const f32x4*>(a.a + i * 4);
    if (a.b) u += *reinterpret_cast<const f32x4*>(a.b + i * 4);
    const f32x4 f = *reinterpret_cast<const f32x4*>(a.f + i * 4);
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      float k = dscale;
      if (a.drop_p > 0.f && !drop_keep(base, thr, (unsigned)(i * 4 + e))) k = 0.f;
      u[e] = fmaf(k, f[e], u[e]);
      s1[e] += u[e];
      s2[e] = fmaf(u[e], u[e], s2[e]);
    }
    *reinterpret_cast<f32x4*>(a.u + i * 4) = u;
  }
  if (a.sum) wg_channel_sums(s1, s2, a.sum, a.sumsq);
}

__global__ __launch_bounds__(256) void sk_bn_apply_kernel(BnApplyArgs a) {
  __shared__ float sc[EMB], sh[EMB];
  if (threadIdx.x < EMB) {
    float m, r;
    bn_coeff(a.bn, threadIdx.x, sc[threadIdx.x], sh[threadIdx.x], m, r);
  }
  __syncthreads();
  const long long n4 = a.R * (EMB / 4);
  for (long long i = blockIdx.x * 256LL + threadIdx.x; i < n4; i += (long long)gridDim.x * 256) {
    const int c = (int)(i & 7) * 4;
    const f32x4 u = *reinterpret_cast<const f32x4*>(a.u + i * 4);
    f32x4 y;
#pragma unroll
    for (int e = 0; e < 4; ++e) y[e] = fmaf(u[e], sc[c + e], sh[c + e]);
    *reinterpret_cast<f32x4*>(a.y + i * 4) = y;
  }
}

__global__ __launch_bounds__(256) void sk_bn_bwd_reduce_kernel(BnBwdArgs a) {
  __shared__ float mu[EMB], rs[EMB];
  if (threadIdx.x < EMB) {
    float sc, sh;
    bn_coeff(a.bn, threadIdx.x, sc, sh, mu[threadIdx.x], rs[threadIdx.x]);
  }
  __syncthreads();
  float s1[4] = {0.f, 0.f, 0.f, 0.f}, s2[4] = {0.f, 0.f, 0.f, 0.f};
  const long long n4 = a.R * (EMB / 4);
  for (long long i = blockIdx.x * 256LL + threadIdx.x; i < n4; i += (long long)gridDim.x * 256) {
    const int c = (int)(i & 7) * 4;
    const f32x4 dy = *reinterpret_cast<const f32x4*>(a.dy + i * 4);
    const f32x4 u = *reinterpret_cast<const f32x4*>(a.u + i * 4);
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      s1[e] += dy[e];
      s2[e] = fmaf(dy[e], (u[e] - mu[c + e]) * rs[c + e], s2[e]);
    }
  }
  wg_channel_sums(s1, s2, a.s_dy, a.s_dyx);
}

__global__ __launch_bounds__(256) void sk_bn_bwd_apply_kernel(BnBwdArgs a) {
  __shared__ float mu[EMB], rs[EMB], k1[EMB], mdy[EMB], mdx[EMB];
  if (threadIdx.x < EMB) {
    const int c = threadIdx.x;
    float sc, sh;
    bn_coeff(a.bn, c, sc, sh, mu[c], rs[c]);
    k1[c] = sc;  // gamma * rstd
    mdy[c] = (float)(a.s_dy[c] / (double)a.R);
    mdx[c] = (float)(a.s_dyx[c] / (double)a.R);
    if (blockIdx.x == 0) {
      a.g_gamma[c] += (float)a.s_dyx[c];
      a.g_beta[c] += (float)a.s_dy[c];
    }
  }
  __syncthreads();
  const unsigned base = drop_base(a.seed, a.block), thr = drop_thr(a.drop_p);
  const float dscale = a.drop_p > 0.f ? a.s2 / (1.f - a.drop_p) : a.s2;
  const long long n4 = a.R * (EMB / 4);
  for (long long i = blockIdx.x * 256LL + threadIdx.x; i < n4; i += (long long)gridDim.x * 256) {
    const int c = (int)(i & 7) * 4;
    const f32x4 dy = *reinterpret_cast<const f32x4*>(a.dy + i * 4);
    const f32x4 u = *reinterpret_cast<const f32x4*>(a.u + i * 4);
    f32x4 du, o2;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const float xh = (u[e] - mu[c + e]) * rs[c + e];
      du[e] = k1[c + e] * (dy[e] - mdy[c + e] - xh * mdx[c + e]);
      float k = dscale;
      if (a.drop_p > 0.f && !drop_keep(base, thr, (unsigned)(i * 4 + e))) k = 0.f;
      o2[e] = k * du[e];
    }
    if (a.o3) *reinterpret_cast<f32x4*>(a.o3 + i * 4) = du;
    if (a.o2) *reinterpret_cast<f32x4*>(a.o2 + i * 4) = o2;
    if (a.add) du += *reinterpret_cast<const f32x4*>(a.add + i * 4);
    *reinterpret_cast<f32x4*>(a.o1 + i * 4) = du;
  }
}

__global__ __launch_bounds__(256) void sk_gelu_fwd_kernel(GeluArgs a) {
  const long long n4 = a.n / 4;
  for (long long i = blockIdx.x * 256LL + threadIdx.x; i < n4; i += (long long)gridDim.x * 256) {
    f32x4 h = *reinterpret_cast<const f32x4*>(a.h + i * 4);
#pragma unroll
    for (int e = 0; e < 4; ++e) h[e] = gelu_f(h[e]);
    *reinterpret_cast<f32x4*>(a.g + i * 4) = h;
  }
}

__global__ __launch_bounds__(256) void sk_gelu_bwd_kernel(GeluArgs a) {
  const long long n4 = a.n / 4;
  for (long long i = blockIdx.x * 256LL + threadIdx.x; i < n4; i += (long long)gridDim.x * 256) {
    const f32x4 h = *reinterpret_cast<const f32x4*>(a.h + i * 4);
    f32x4 d = *reinterpret_cast<const f32x4*>(a.dg + i * 4);
#pragma unroll
    for (int e = 0; e < 4; ++e) d[e] *= gelu_d(h[e]);
    *reinterpret_cast<f32x4*>(a.dh + i * 4) = d;
  }
}

// ------------------------------------------------------------------------------------------
// head (skeleton_transformer.py:425-435): one workgroup per clip
// ------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void sk_head_fwd_kernel(HeadArgs a) {
  __shared__ float part[8][EMB], pooled[EMB];
  const int n = blockIdx.x, c = threadIdx.x & 31, g = threadIdx.x >> 5;
  const float* y = a.y + (size_t)n * a.MTV * EMB;
  float acc = 0.f;
  for (int t = g; t < a.MTV; t += 8) acc += y[(size_t)t * EMB + c];
  part[g][c] = acc;
  __syncthreads();
  if (threadIdx.x < EMB) {
    float s = 0.f;
#pragma unroll
    for (int q = 0; q < 8; ++q) s += part[q][c];
    pooled[c] = s / (float)a.MTV;
    a.pooled[(size_t)n * EMB + c] = pooled[c];
  }
  __syncthreads();
  if (threadIdx.x < a.C) {
    const int k = threadIdx.x;
    float o = a.b[k];
    for (int j = 0; j < EMB; ++j) o = fmaf(a.w[k * EMB + j], pooled[j], o);
    a.out[(size_t)n * a.C + k] = o;
  }
}

__global__ __launch_bounds__(256) void sk_head_bwd_kernel(HeadArgs a) {
  __shared__ float dp[EMB];
  const int n = blockIdx.x;
  if (threadIdx.x < EMB) {
    const int c = threadIdx.x;
    float s = 0.f;
    for (int k = 0; k < a.C; ++k) {
      const float g = a.dout[(size_t)n * a.C + k];
      s = fmaf(g, a.w[k * EMB + c], s);
      atomicAdd(a.gw + k * EMB + c, g * a.pooled[(size_t)n * EMB + c]);
    }
    dp[c] = s / (float)a.MTV;
  }
  if (threadIdx.x >= 64 && threadIdx.x < 64 + a.C) {
    const int k = threadIdx.x - 64;
    atomicAdd(a.gb + k, a.dout[(size_t)n * a.C + k]);
  }
  __syncthreads();
  float* dy = a.dy + (size_t)n * a.MTV * EMB;
  for (int e = threadIdx.x; e < a.MTV * (EMB / 4); e += 256) {
    const int c = (e & 7) * 4;
    *reinterpret_cast<f32x4*>(dy + (size_t)e * 4) = f32x4{dp[c], dp[c + 1], dp[c + 2], dp[c + 3]};
  }
}

static int grid_for(long long items, int cap = 2048) {
  const long long g = (items + 255) / 256;
  return (int)(g < 1 ? 1 : (g > cap ? cap : g));
}

template <int L>
static int launch_attn(const AttnArgs& a, bool bwd, hipStream_t s) {
  F3_LDS_LIMIT(sk_attn_fwd_kernel<L>, attn_fwd_lds<L>());
  F3_LDS_LIMIT(sk_attn_bwd_kernel<L>, attn_bwd_lds<L>());
  const int threads = attn_threads(L);
  if (bwd)
    hipLaunchKernelGGL(sk_attn_bwd_kernel<L>, dim3(a.nseq), dim3(threads), attn_bwd_lds<L>(), s, a);
  else
    hipLaunchKernelGGL(sk_attn_fwd_kernel<L>, dim3(a.nseq), dim3(threads), attn_fwd_lds<L>(), s, a);
  F3_LAUNCH_CHECK();
  return F3_OK;
}

static int attn_dispatch(const AttnArgs* a, bool bwd, hipStream_t s) {
  if (!a || a->nseq < 0 || !a->qkv || !a->table) return F3_EINVAL;
  if (a->nseq == 0) return F3_OK;
  switch (a->L) {
    case 14: return launch_attn<14>(*a, bwd, s);
    case 17: return launch_attn<17>(*a, bwd, s);
    case 18: return launch_attn<18>(*a, bwd, s);
    case 30: return launch_attn<30>(*a, bwd, s);
    case 32: return launch_attn<32>(*a, bwd, s);
    default: return F3_EINVAL;
  }
}

}  // namespace sk
}  // namespace f3

using namespace f3;
using namespace f3::sk;

bool f3_sk_attn_len_ok(int L) { return L == 14 || L == 17 || L == 18 || L == 30 || L == 32; }

int f3_sk_embed_fwd_save(const EmbedArgs* a, float* xt, float* a1, float* h1, float* a2, hipStream_t s) {
  EmbedSave sv{xt, a1, h1, a2, nullptr, nullptr};
  const long long R = (long long)a->N * a->M * a->T * a->V;
  hipLaunchKernelGGL(sk_embed_fwd_kernel, dim3(grid_for(R)), dim3(256), 0, s, *a, sv);
  F3_LAUNCH_CHECK();
  return F3_OK;
}

int f3_sk_embed_bwd_save(const EmbedArgs* a, const float* a1, const float* a2, float* da1, float* da2,
                         hipStream_t s) {
  EmbedSave sv{nullptr, const_cast<float*>(a1), nullptr, const_cast<float*>(a2), da1, da2};
  const long long R = (long long)a->N * a->M * a->T * a->V;
  hipLaunchKernelGGL(sk_embed_bwd_kernel, dim3(grid_for(R)), dim3(256), 0, s, *a, sv);
  F3_LAUNCH_CHECK();
  return F3_OK;
}

int f3_sk_attn_fwd(const AttnArgs* a, hipStream_t s) { return attn_dispatch(a, false, s); }
int f3_sk_attn_bwd(const AttnArgs* a, hipStream_t s) { return attn_dispatch(a, true, s); }

int f3_sk_resid(const ResidArgs* a, hipStream_t s) {
  hipLaunchKernelGGL(sk_resid_kernel, dim3(grid_for(a->R * (EMB / 4), 1024)), dim3(256), 0, s, *a);
  F3_LAUNCH_CHECK();
  return F3_OK;
}

int f3_sk_bn_apply(const BnApplyArgs* a, hipStream_t s) {
  hipLaunchKernelGGL(sk_bn_apply_kernel, dim3(grid_for(a->R * (EMB / 4))), dim3(256), 0, s, *a);
  F3_LAUNCH_CHECK();
  return F3_OK;
}

int f3_sk_bn_bwd(const BnBwdArgs* a, hipStream_t s) {
  hipLaunchKernelGGL(sk_bn_bwd_reduce_kernel, dim3(grid_for(a->R * (EMB / 4), 1024)), dim3(256), 0, s, *a);
  F3_LAUNCH_CHECK();
  hipLaunchKernelGGL(sk_bn_bwd_apply_kernel, dim3(grid_for(a->R * (EMB / 4))), dim3(256), 0, s, *a);
  F3_LAUNCH_CHECK();
  return F3_OK;
}

int f3_sk_gelu_fwd(const GeluArgs* a, hipStream_t s) {
  hipLaunchKernelGGL(sk_gelu_fwd_kernel, dim3(grid_for(a->n / 4)), dim3(256), 0, s, *a);
  F3_LAUNCH_CHECK();
  return F3_OK;
}

int f3_sk_gelu_bwd(const GeluArgs* a, hipStream_t s) {
  hipLaunchKernelGGL(sk_gelu_bwd_kernel, dim3(grid_for(a->n / 4)), dim3(256), 0, s, *a);
  F3_LAUNCH_CHECK();
  return F3_OK;
}

int f3_sk_head_fwd(const HeadArgs* a, hipStream_t s) {
  if (a->C > 64) return F3_EINVAL;
  hipLaunchKernelGGL(sk_head_fwd_kernel, dim3(a->N), dim3(256), 0, s, *a);
  F3_LAUNCH_CHECK();
  return F3_OK;
}

int f3_sk_head_bwd(const HeadArgs* a, hipStream_t s) {
  if (a->C > 64) return F3_EINVAL;
  hipLaunchKernelGGL(sk_head_bwd_kernel, dim3(a->N), dim3(256), 0, s, *a);
  F3_LAUNCH_CHECK();
  return F3_OK;
}
