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
  for (int b = 0; b < a.nblk; ++b) {
    for (int k = threadIdx.x; k < a.width[b]; k += blockDim.x)
      fs[K + k] = a.feat[b][(size_t)n * a.ld[b] + k];
    K += a.width[b];
  }
  __syncthreads();
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  for (int c = wave; c < a.C; c += blockDim.x >> 6) {
    float acc = 0.f;
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
      for (int c = 0; c < a.C; ++c) a.out[(size_t)n * a.C + c] = __expf(z[c] - mx) / s;
    } else {
      for (int c = 0; c < a.C; ++c) a.out[(size_t)n * a.C + c] = z[c];
    }
  }
}

// loss += -(1/N) sum_c y log_softmax(out);  dout = (softmax(out) * sum_c y - y) / N
constexpr int kCeOneBlock = 4096;  // batches up to this size: the single-workgroup form

// ONE: a single 256-thread workgroup walks every row and stores the mean loss (no zeroed loss word
// beforehand, no atomics: deterministic); otherwise one row per thread, atomics into a zeroed loss
template <bool ONE>
__global__ void ce_kernel(HeadArgs a) {
  float lsum = 0.f;
  const int n0 = ONE ? threadIdx.x : blockIdx.x * blockDim.x + threadIdx.x;
  for (int n = n0; n < a.N; n += ONE ? blockDim.x : a.N) {
    const float* o = a.out + (size_t)n * a.C;
    const float* y = a.label + (size_t)n * a.C;
    float mx = -INFINITY;
    for (int c = 0; c < a.C; ++c) mx = fmaxf(mx, o[c]);
    float s = 0.f, ys = 0.f;
    for (int c = 0; c < a.C; ++c) { s += expf(o[c] - mx); ys += y[c]; }
    const float lse = mx + logf(s);
    float l = 0.f;
    for (int c = 0; c < a.C; ++c) {
      l -= y[c] * (o[c] - lse);
      a.dout[(size_t)n * a.C + c] = (expf(o[c] - lse) * ys - y[c]) / (float)a.N;
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

// grid (N): dfeat[n][k] = sum_c dlog[n][c] W[c][k]
__global__ __launch_bounds__(256) void head_dfeat_kernel(HeadArgs a) {
  const int n = blockIdx.x;
  const int K = a.width[0] + (a.nblk > 1 ? a.width[1] : 0) + (a.nblk > 2 ? a.width[2] : 0);
  int off = 0;
  for (int b = 0; b < a.nblk; ++b) {
    if (a.dfeat[b]) {
      for (int k = threadIdx.x; k < a.width[b]; k += blockDim.x) {
        float acc = 0.f;
        for (int c = 0; c < a.C; ++c) acc += a.dlogits[(size_t)n * a.C + c] * a.W[(size_t)c * K + off + k];
        a.dfeat[b][(size_t)n * a.width[b] + k] = acc;
      }
    }
    off += a.width[b];
  }
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

int f3_head_bwd(const HeadArgs* a, hipStream_t s) {
  hipLaunchKernelGGL(head_dlogits_kernel, dim3((a->N + 255) / 256), dim3(256), 0, s, *a);
  F3_LAUNCH_CHECK();
  if (a->nblk > 0) {
    const int K = a->width[0] + (a->nblk > 1 ? a->width[1] : 0) + (a->nblk > 2 ? a->width[2] : 0);
    hipLaunchKernelGGL(head_wgrad_kernel, dim3((K + 63) / 64, a->C), dim3(256), 0, s, *a);
    F3_LAUNCH_CHECK();
    hipLaunchKernelGGL(head_dfeat_kernel, dim3(a->N), dim3(256), 0, s, *a);
    F3_LAUNCH_CHECK();
  }
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
