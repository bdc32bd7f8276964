// Shared device helpers for the fall3 MI355X (gfx950) kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define F3_DEV __device__ __forceinline__

typedef float f32x4 __attribute__((ext_vector_type(4)));

namespace f3 {

constexpr float kBnEps = 1e-5f;

// Batch-norm coefficient source. Train mode derives mean/var from fp64 batch sums that
// the producing kernel accumulated in its epilogue; eval mode uses the running stats
// (nn.BatchNorm semantics: biased variance for normalisation).
struct BnRef {
  const double* sum;      // [C] sum x          (train)
  const double* sumsq;    // [C] sum x^2        (train)
  const float* gamma;     // [C]
  const float* beta;      // [C]
  const float* rmean;     // [C] running mean   (eval)
  const float* rvar;      // [C] running var    (eval)
  float count;            // elements per channel in the batch
  int eval;
};

// y = x*scale + shift ; also returns mean and 1/sqrt(var+eps) for backward formulas.
F3_DEV void bn_coeff(const BnRef& b, int c, float& scale, float& shift, float& mean, float& rstd) {
  if (b.eval) {
    mean = b.rmean[c];
    rstd = rsqrtf(b.rvar[c] + kBnEps);
  } else {
    double m = b.sum[c] / (double)b.count;
    double v = b.sumsq[c] / (double)b.count - m * m;
    if (v < 0) v = 0;
    mean = (float)m;
    rstd = (float)(1.0 / sqrt(v + (double)kBnEps));
  }
  scale = b.gamma[c] * rstd;
  shift = b.beta[c] - mean * scale;
}

// bn_coeff of channels c0 .. c0 + 3 with every load issued before any use (the per-channel calls
// in a row were a chain of dependent round trips ahead of the streaming kernels' first loads);
// the same arithmetic per channel, so bit-identical to four bn_coeff calls
F3_DEV void bn_coeff4(const BnRef& b, int c0, float* scale, float* shift, float* mean, float* rstd) {
  float g[4], be[4];
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    g[e] = b.gamma[c0 + e];
    be[e] = b.beta[c0 + e];
  }
  if (b.eval) {
    float rm[4], rv[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      rm[e] = b.rmean[c0 + e];
      rv[e] = b.rvar[c0 + e];
    }
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      mean[e] = rm[e];
      rstd[e] = rsqrtf(rv[e] + kBnEps);
    }
  } else {
    double sm[4], sq[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      sm[e] = b.sum[c0 + e];
      sq[e] = b.sumsq[c0 + e];
    }
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      double m = sm[e] / (double)b.count;
      double v = sq[e] / (double)b.count - m * m;
      if (v < 0) v = 0;
      mean[e] = (float)m;
      rstd[e] = (float)(1.0 / sqrt(v + (double)kBnEps));
    }
  }
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    scale[e] = g[e] * rstd[e];
    shift[e] = be[e] - mean[e] * scale[e];
  }
}

F3_DEV float warp_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

F3_DEV double warp_sum_d(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

F3_DEV void atomic_add_d(double* p, double v) { atomicAdd(p, v); }
F3_DEV void atomic_add_f(float* p, float v) { atomicAdd(p, v); }

F3_DEV float sigmoidf_(float x) { return 1.f / (1.f + __expf(-x)); }

// Activation storage. The bf16 mode keeps the layer activations (gcn / tcn / residual conv
// outputs, block outputs, the tcn input gradient) in bf16 in HBM; arithmetic stays fp32
// (BN statistics are taken in the producers' epilogues from the fp32 values). B16 selects
// the storage type; offsets are in elements.
typedef __bf16 act_bf16x4 __attribute__((ext_vector_type(4)));
F3_DEV float bf2f(unsigned short u) { return __uint_as_float((unsigned)u << 16); }
template <bool B16>
F3_DEV f32x4 ld_act4(const void* p, size_t off) {
  if constexpr (B16) {
    const act_bf16x4 v = *reinterpret_cast<const act_bf16x4*>(reinterpret_cast<const __bf16*>(p) + off);
    return f32x4{(float)v[0], (float)v[1], (float)v[2], (float)v[3]};
  } else {
    return *reinterpret_cast<const f32x4*>(reinterpret_cast<const float*>(p) + off);
  }
}
template <bool B16>
F3_DEV void st_act4(void* p, size_t off, f32x4 v) {
  if constexpr (B16) {
    act_bf16x4 o;
#pragma unroll
    for (int e = 0; e < 4; ++e) o[e] = (__bf16)v[e];
    *reinterpret_cast<act_bf16x4*>(reinterpret_cast<__bf16*>(p) + off) = o;
  } else {
    *reinterpret_cast<f32x4*>(reinterpret_cast<float*>(p) + off) = v;
  }
}
F3_DEV float ld_act(const void* p, size_t off, bool b16) {
  return b16 ? bf2f(reinterpret_cast<const unsigned short*>(p)[off]) : reinterpret_cast<const float*>(p)[off];
}

// Group barrier of co-resident workgroups (cooperative launches: the TARGCN node-partitioned GRU,
// the sensor CNN1D). Every workgroup of the group adds 1 to *cnt and waits until it reaches
// `target` (k x group size at the k-th barrier; *cnt zeroed before the launch). `arrive` false:
// this workgroup does not count itself (the F3_GN_SKIP_ARRIVE test knob, which makes the group's
// barriers time out). A barrier that does not complete within ~2^22 polls sets *err and stops
// waiting; once *err is set, every later barrier returns after the first poll that sees it, so a
// faulted launch drains quickly (the caller reports or poisons its outputs).
F3_DEV void gn_barrier(int* cnt, int target, int* err, bool arrive = true) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's exchange stores have reached L2
  __syncthreads();
  if (threadIdx.x == 0) {
    __threadfence();  // agent-scope release: the group's other XCDs see the stores
    if (arrive) __hip_atomic_fetch_add(cnt, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    int polls = 0;
    while (__hip_atomic_load(cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
      __builtin_amdgcn_s_sleep(1);
      ++polls;
      if ((polls & 1023) == 0 && __hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) break;
      if (polls > (1 << 22)) {
        __hip_atomic_store(err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        break;
      }
    }
    __threadfence();  // acquire: no stale lines of the exchanged rows survive in this CU / XCD
  }
  __syncthreads();
}

}  // namespace f3

// Error plumbing for the C ABI: never abort, return a status.
#define F3_OK 0
#define F3_EINVAL 1001
#define F3_EBATCH 1002   // train-mode batch of 1 (nn.BatchNorm: "Expected more than 1 value per channel")
#define F3_EHIP 1003

#include <stdio.h>
#include <stdlib.h>
// F3_DEBUG_SYNC=1 synchronises the device after every launch (debugging aid)
inline bool f3_debug_sync() {
  static const bool on = getenv("F3_DEBUG_SYNC") != nullptr;
  return on;
}
#ifndef F3_TRY
#define F3_TRY(x)               \
  do {                          \
    int _s = (x);               \
    if (_s != F3_OK) return _s; \
  } while (0)
#endif
#define F3_LAUNCH_CHECK()                                                              \
  do {                                                                                 \
    if (f3_debug_sync()) (void)hipDeviceSynchronize();                                 \
    hipError_t _e = hipGetLastError();                                                 \
    if (_e != hipSuccess) {                                                            \
      fprintf(stderr, "fall3: %s:%d launch failed: %s\n", __FILE__, __LINE__,          \
              hipGetErrorString(_e));                                                  \
      return F3_EHIP;                                                                  \
    }                                                                                  \
  } while (0)
// Raise a kernel's dynamic-LDS limit once per process (the result is cached per call site) and
// fail as F3_EHIP when the runtime refuses it, naming the attribute instead of the launch after it.
inline int f3_set_lds_limit(const void* fn, int bytes, const char* where, int line) {
  const hipError_t e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
  if (e == hipSuccess) return F3_OK;
  (void)hipGetLastError();  // the refusal must not surface as the next launch's error
  fprintf(stderr, "fall3: %s:%d hipFuncSetAttribute(MaxDynamicSharedMemorySize=%d) failed: %s\n", where, line, bytes,
          hipGetErrorString(e));
  return F3_EHIP;
}
#define F3_LDS_LIMIT(fn, bytes)                                                                  \
  do {                                                                                           \
    static const int _r = f3_set_lds_limit((const void*)(fn), (int)(bytes), __FILE__, __LINE__); \
    if (_r != F3_OK) return _r;                                                                  \
  } while (0)
