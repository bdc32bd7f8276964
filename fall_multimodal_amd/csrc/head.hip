// Late fusion + loss + optimizer:
//   cat([pts256, mot256, sensor Cs]) -> Linear -> (softmax, notebook form)
//       Multimodal_Fall3/model/combination.py:45-46, GSTCAN_HAR_conv_10kfold.ipynb:432-444
//   CrossEntropyLoss with probability targets (no renormalisation)   model/main.py:113,280
//   RMSprop(lr) torch defaults (alpha .99, eps 1e-8 after sqrt)       model/optimizer.py:21
#include "common.h"
#include "sensor.h"

namespace f3 {

// one workgroup per clip: logits[c] = b[c] + sum_k W[c][k] feat[k]
__global__ __launch_bounds__(256) void head_fwd_kernel(HeadArgs a) {
  extern __shared__ float fs[];  // concatenated features
  __shared__ float z[64];
  const int n = blockIdx.x;
  int K = 0;
  if (a.width[0] <= (int)blockDim.x && a.width[1] <= (int)blockDim.x && a.width[2] <= (int)blockDim.x) {
    // blocks no wider than the workgroup: each thread's (up to three) loads go out together
    float v[3];
#pragma unroll
    for (int b = 0; b < 3; ++b)
      v[b] = b < a.nblk && (int)threadIdx.x < a.width[b] ? a.feat[b][(size_t)n * a.ld[b] + threadIdx.x] : 0.f;
#pragma unroll
    for (int b = 0; b < 3; ++b) {
      if (b < a.nblk && (int)threadIdx.x < a.width[b]) fs[K + threadIdx.x] = v[b];
      K += b < a.nblk ? a.width[b] : 0;
    }
  } else {
    for (int b = 0; b < a.nblk; ++b) {
      for (int k = threadIdx.x; k < a.width[b]; k += blockDim.x)
        fs[K + k] = a.feat[b][(size_t)n * a.ld[b] + k];
      K += a.width[b];
    }
  }
  __syncthreads();
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  for (int c = wave; c < a.C; c += blockDim.x >> 6) {
    float acc = 0.f;
#pragma unroll 4  // (unrolled: the weight loads of four k steps go out together; same sum order)
    for (int k = lane; k < K; k += 64) acc += a.W[(size_t)c * K + k] * fs[k];
    acc = warp_sum(acc);
    if (lane == 0) z[c] = acc + a.b[c];
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    if (a.softmax_out) {
      float mx = -INFINITY;
      for (int c = 0; c < a.C; ++c) mx = fmaxf(mx, z[c]);
      float s = 0.f;
      for (int c = 0; c < a.C; ++c) s += __expf(z[c] - mx);
      for (int c = 0; c < a.C; ++c) z[c] = __expf(z[c] - mx) / s;
    }
  }
  __syncthreads();
  // the module output, and the caller's copy of it (out2: no device-to-device copy afterwards)
  if (threadIdx.x < a.C) {
    a.out[(size_t)n * a.C + threadIdx.x] = z[threadIdx.x];
    if (a.out2) a.out2[(size_t)n * a.C + threadIdx.x] = z[threadIdx.x];
  }
}

// loss += -(1/N) sum_c y log_softmax(out);  dout = (softmax(out) * sum_c y - y) / N
constexpr int kCeOneBlock = 4096;  // batches up to this size: the single-workgroup form

// ONE: a single 256-thread workgroup walks every row and stores the mean loss (no zeroed loss word
// beforehand, no atomics: deterministic); otherwise one row per thread, atomics into a zeroed loss
constexpr int kCeRegs = 16;  // class counts up to this: the row is loaded into registers up front

template <bool ONE>
__global__ void ce_kernel(HeadArgs a) {
  float lsum = 0.f;
  const int n0 = ONE ? threadIdx.x : blockIdx.x * blockDim.x + threadIdx.x;
  for (int n = n0; n < a.N; n += ONE ? blockDim.x : a.N) {
    const float* o = a.out + (size_t)n * a.C;
    const float* y = a.label + (size_t)n * a.C;
    float* d = a.dout + (size_t)n * a.C;
    float l = 0.f;
    if (a.C <= kCeRegs) {
      // every load issued before the first use (clamped indices: no branches between them); the
      // same sequential sums as the loop form below, so the two agree bit for bit
      float ov[kCeRegs], yv[kCeRegs];
#pragma unroll
      for (int c = 0; c < kCeRegs; ++c) {
        const int cc = c < a.C ? c : a.C - 1;
        ov[c] = o[cc];
        yv[c] = y[cc];
      }
      float mx = -INFINITY;
#pragma unroll
      for (int c = 0; c < kCeRegs; ++c)
        if (c < a.C) mx = fmaxf(mx, ov[c]);
      float s = 0.f, ys = 0.f;
#pragma unroll
      for (int c = 0; c < kCeRegs; ++c)
        if (c < a.C) { s += expf(ov[c] - mx); ys += yv[c]; }
      const float lse = mx + logf(s);
#pragma unroll
      for (int c = 0; c < kCeRegs; ++c)
        if (c < a.C) {
          l -= yv[c] * (ov[c] - lse);
          d[c] = (expf(ov[c] - lse) * ys - yv[c]) / (float)a.N;
        }
    } else {
      float mx = -INFINITY;
      for (int c = 0; c < a.C; ++c) mx = fmaxf(mx, o[c]);
      float s = 0.f, ys = 0.f;
      for (int c = 0; c < a.C; ++c) { s += expf(o[c] - mx); ys += y[c]; }
      const float lse = mx + logf(s);
      for (int c = 0; c < a.C; ++c) {
        l -= y[c] * (o[c] - lse);
        d[c] = (expf(o[c] - lse) * ys - y[c]) / (float)a.N;
      }
    }
    lsum += l;
  }
  if constexpr (ONE) {
    __shared__ float red[4];
    for (int off = 32; off > 0; off >>= 1) lsum += __shfl_xor(lsum, off, 64);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = lsum;
    __syncthreads();
    if (threadIdx.x == 0) *a.loss = (red[0] + red[1] + red[2] + red[3]) / (float)a.N;
  } else {
    if (n0 < a.N) atomic_add_f(a.loss, lsum / (float)a.N);
  }
}

// dlogits from the gradient of the module output (softmax Jacobian for the notebook form)
__global__ void head_dlogits_kernel(HeadArgs a) {
  const int n = blockIdx.x * blockDim.x + threadIdx.x;
  if (n >= a.N) return;
  const float* g = a.g_out + (size_t)n * a.C;
  float* d = a.dlogits + (size_t)n * a.C;
  if (a.softmax_out) {
    const float* p = a.out + (size_t)n * a.C;
    float dot = 0.f;
    for (int c = 0; c < a.C; ++c) dot += p[c] * g[c];
    for (int c = 0; c < a.C; ++c) d[c] = p[c] * (g[c] - dot);
  } else {
    for (int c = 0; c < a.C; ++c) d[c] = g[c];
  }
}

// grid (ceil(K/64), C): dW[c][k] = sum_n dlog[n][c] feat[n][k], db[c]. A workgroup owns 64
// feature columns of one class; its 4 waves split the clips (coalesced 64-wide row reads,
// independent partial sums) and combine through LDS.
__global__ __launch_bounds__(256) void head_wgrad_kernel(HeadArgs a) {
  __shared__ float part[4][65];
  const int c = blockIdx.y, lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int K = a.width[0] + (a.nblk > 1 ? a.width[1] : 0) + (a.nblk > 2 ? a.width[2] : 0);
  const int k = blockIdx.x * 64 + lane;
  const float* f = nullptr;
  int ld = 0;
  if (k < K) {  // which concatenated block holds column k
    int off = 0;
    for (int b = 0; b < a.nblk; ++b) {
      if (k < off + a.width[b]) { f = a.feat[b] + (k - off); ld = a.ld[b]; break; }
      off += a.width[b];
    }
  }
  float acc = 0.f, accb = 0.f;
  for (int n = wave; n < a.N; n += 4) {
    const float d = a.dlogits[(size_t)n * a.C + c];
    if (f) acc += d * f[(size_t)n * ld];
    accb += d;
  }
  part[wave][lane] = acc;
  if (lane == 0) part[wave][64] = accb;
  __syncthreads();
  if (wave == 0) {
    const float s = part[0][lane] + part[1][lane] + part[2][lane] + part[3][lane];
    if (k < K) a.g_W[(size_t)c * K + k] += s;
    if (lane == 0 && blockIdx.x == 0) a.g_b[c] += part[0][64] + part[1][64] + part[2][64] + part[3][64];
  }
}

// grid (N): the clip's dlogits row (head_dlogits' arithmetic, in the same order; stored for
// head_wgrad), then dfeat[n][k] = sum_c dlog[n][c] W[c][k] from LDS
__global__ __launch_bounds__(256) void head_dfeat_kernel(HeadArgs a) {
  __shared__ float dl[64];
  __shared__ float pg[2][64];
  const int n = blockIdx.x;
  const int K = a.width[0] + (a.nblk > 1 ? a.width[1] : 0) + (a.nblk > 2 ? a.width[2] : 0);
  if (threadIdx.x < a.C) {
    pg[0][threadIdx.x] = a.softmax_out ? a.out[(size_t)n * a.C + threadIdx.x] : 0.f;
    pg[1][threadIdx.x] = a.g_out[(size_t)n * a.C + threadIdx.x];
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    if (a.softmax_out) {
      float dot = 0.f;
      for (int c = 0; c < a.C; ++c) dot += pg[0][c] * pg[1][c];
      for (int c = 0; c < a.C; ++c) dl[c] = pg[0][c] * (pg[1][c] - dot);
    } else {
      for (int c = 0; c < a.C; ++c) dl[c] = pg[1][c];
    }
  }
  __syncthreads();
  if (threadIdx.x < a.C) a.dlogits[(size_t)n * a.C + threadIdx.x] = dl[threadIdx.x];
  int off = 0;
  for (int b = 0; b < a.nblk; ++b) {
    if (a.dfeat[b]) {
      for (int k = threadIdx.x; k < a.width[b]; k += blockDim.x) {
        float acc = 0.f;
        for (int c = 0; c < a.C; ++c) acc += dl[c] * a.W[(size_t)c * K + off + k];
        a.dfeat[b][(size_t)n * a.width[b] + k] = acc;
      }
    }
    off += a.width[b];
  }
}

// zero two float ranges in one launch (the backward's gradient buffer and its zeroed workspace
// block); 16-byte aligned starts, float4 stores plus a scalar tail per range
__global__ __launch_bounds__(256) void zero2_kernel(float* __restrict__ a, long long na, float* __restrict__ b,
                                                   long long nb) {
  const long long stride = (long long)gridDim.x * blockDim.x;
  const long long t = blockIdx.x * (long long)blockDim.x + threadIdx.x;
  const long long a4 = na / 4, b4 = nb / 4;
  const f32x4 z = {0.f, 0.f, 0.f, 0.f};
  for (long long i = t; i < a4 + b4; i += stride) {
    if (i < a4) reinterpret_cast<f32x4*>(a)[i] = z;
    else reinterpret_cast<f32x4*>(b)[i - a4] = z;
  }
  if (t < na - a4 * 4) a[a4 * 4 + t] = 0.f;
  if (t < nb - b4 * 4) b[b4 * 4 + t] = 0.f;
}

__global__ void rmsprop_kernel(float* __restrict__ p, float* __restrict__ sq, const float* __restrict__ g,
                               long long n, float lr, float alpha, float eps, float scale) {
  const long long n4 = n / 4;
  const long long stride = (long long)gridDim.x * blockDim.x;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n4; i += stride) {
    f32x4 gv = reinterpret_cast<const f32x4*>(g)[i] * scale;
    f32x4 sv = reinterpret_cast<f32x4*>(sq)[i];
    f32x4 pv = reinterpret_cast<f32x4*>(p)[i];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      sv[e] = alpha * sv[e] + (1.f - alpha) * gv[e] * gv[e];
      pv[e] -= lr * gv[e] / (sqrtf(sv[e]) + eps);
    }
    reinterpret_cast<f32x4*>(sq)[i] = sv;
    reinterpret_cast<f32x4*>(p)[i] = pv;
  }
  for (long long i = n4 * 4 + blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n; i += stride) {
    const float gv = g[i] * scale;
    const float sv = alpha * sq[i] + (1.f - alpha) * gv * gv;
    sq[i] = sv;
    p[i] -= lr * gv / (sqrtf(sv) + eps);
  }
}

__global__ void rmsprop_ranges_kernel(float* __restrict__ p, float* __restrict__ sq, const float* __restrict__ g,
                                      RmsRanges r, long long n4, float lr, float alpha, float eps, float scale) {
  const long long stride = (long long)gridDim.x * blockDim.x;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n4; i += stride) {
    long long k = i, base = 0;
    int j = 0;
    for (; j < r.n - 1 && k >= r.len[j] / 4; ++j) k -= r.len[j] / 4;
    base = r.lo[j] / 4 + k;
    f32x4 gv = reinterpret_cast<const f32x4*>(g)[base] * scale;
    f32x4 sv = reinterpret_cast<f32x4*>(sq)[base];
    f32x4 pv = reinterpret_cast<f32x4*>(p)[base];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      sv[e] = alpha * sv[e] + (1.f - alpha) * gv[e] * gv[e];
      pv[e] -= lr * gv[e] / (sqrtf(sv[e]) + eps);
    }
    reinterpret_cast<f32x4*>(sq)[base] = sv;
    reinterpret_cast<f32x4*>(p)[base] = pv;
  }
}

}  // namespace f3

using namespace f3;

int f3_rmsprop_ranges(float* p, float* sq, const float* g, const RmsRanges& r, float lr, float alpha, float eps,
                      float scale, hipStream_t s) {
  if (r.n < 0 || r.n > kRmsRanges) return F3_EINVAL;
  long long n4 = 0;
  for (int j = 0; j < r.n; ++j) {
    if (r.lo[j] % 4 || r.len[j] % 4 || r.len[j] < 0) return F3_EINVAL;
    n4 += r.len[j] / 4;
  }
  if (n4 == 0) return F3_OK;
  const long long blocks = (n4 + 255) / 256;
  const int grid = (int)(blocks < 4096 ? blocks : 4096);
  hipLaunchKernelGGL(rmsprop_ranges_kernel, dim3(grid), dim3(256), 0, s, p, sq, g, r, n4, lr, alpha, eps, scale);
  F3_LAUNCH_CHECK();
  return F3_OK;
}

int f3_head_fwd(const HeadArgs* a, hipStream_t s) {
  if (a->C > 64) return F3_EINVAL;
  const int K = a->width[0] + (a->nblk > 1 ? a->width[1] : 0) + (a->nblk > 2 ? a->width[2] : 0);
  hipLaunchKernelGGL(head_fwd_kernel, dim3(a->N), dim3(256), (size_t)K * 4, s, *a);
  F3_LAUNCH_CHECK();
  return F3_OK;
}

int f3_ce(const HeadArgs* a, hipStream_t s) {
  if (a->N <= kCeOneBlock) {
    hipLaunchKernelGGL(ce_kernel<true>, dim3(1), dim3(256), 0, s, *a);
  } else {
    if (hipMemsetAsync(a->loss, 0, sizeof(float), s) != hipSuccess) return F3_EHIP;
    hipLaunchKernelGGL(ce_kernel<false>, dim3((a->N + 255) / 256), dim3(256), 0, s, *a);
  }
  F3_LAUNCH_CHECK();
  return F3_OK;
}

int f3_head_bwd_data(const HeadArgs* a, hipStream_t s) {
  if (a->C > 64) return F3_EINVAL;
  if (a->nblk > 0) {
    hipLaunchKernelGGL(head_dfeat_kernel, dim3(a->N), dim3(256), 0, s, *a);
  } else {
    hipLaunchKernelGGL(head_dlogits_kernel, dim3((a->N + 255) / 256), dim3(256), 0, s, *a);
  }
  F3_LAUNCH_CHECK();
  return F3_OK;
}

int f3_head_bwd_weight(const HeadArgs* a, hipStream_t s) {
  if (a->nblk == 0) return F3_OK;
  const int K = a->width[0] + (a->nblk > 1 ? a->width[1] : 0) + (a->nblk > 2 ? a->width[2] : 0);
  hipLaunchKernelGGL(head_wgrad_kernel, dim3((K + 63) / 64, a->C), dim3(256), 0, s, *a);
  F3_LAUNCH_CHECK();
  return F3_OK;
}

int f3_head_bwd(const HeadArgs* a, hipStream_t s) {
  F3_TRY(f3_head_bwd_data(a, s));
  return f3_head_bwd_weight(a, s);
}

int f3_zero2(float* a, long long na, float* b, long long nb, hipStream_t s) {
  if (na < 0 || nb < 0 || (na && !a) || (nb && !b) || ((uintptr_t)a | (uintptr_t)b) % 16) return F3_EINVAL;
  const long long n4 = na / 4 + nb / 4;
  if (n4 == 0 && na == 0 && nb == 0) return F3_OK;
  const long long blocks = (n4 + 255) / 256;
  const int grid = (int)(blocks < 2048 ? (blocks > 0 ? blocks : 1) : 2048);
  hipLaunchKernelGGL(zero2_kernel, dim3(grid), dim3(256), 0, s, a, na, b, nb);
  F3_LAUNCH_CHECK();
  return F3_OK;
}

int f3_rmsprop(float* p, float* sq, const float* g, long long n, float lr, float alpha, float eps, float scale,
               hipStream_t s) {
  if (n <= 0) return F3_OK;
  const long long blocks = ((n / 4) + 255) / 256;
  const int grid = (int)(blocks < 4096 ? (blocks > 0 ? blocks : 1) : 4096);
  hipLaunchKernelGGL(rmsprop_kernel, dim3(grid), dim3(256), 0, s, p, sq, g, n, lr, alpha, eps, scale);
  F3_LAUNCH_CHECK();
  return F3_OK;
}
