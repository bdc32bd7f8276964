// RGB spatial-conv branch (north star: "RGB spatial-conv branch" over 224x224 frames; SURVEY.md
// section 0.2 / 8a row R-RGB). The reference has RGB frames only in preprocessing
// (3_stream/har_create3.py:36-42,101-158), no model arithmetic, so this branch is BUILD-DEFINED and
// its parity is unpinned: its CPU restatement is oracle/rgb_cpu.py (the same definition in torch),
// not a reference. Definition (per clip b of T frames, frames channels-last bf16 [B][T][224][224][3]):
//   conv   = Conv2d(3, 64, kernel 8, stride 8) of each frame: a 28 x 28 grid of patches, each patch
//            192 values in (dy, dx, ch) order, times the packed weight [64][192] (+ bias)
//   feat   = mean over the T frames and 784 patches of relu(conv)               -> [B][64]
//   (the late-fusion logits feat . W_fc^T + b_fc are a torch Linear in rgb.py)
// The branch is HBM-bound: 301 KB of input per frame (2.3 GB per B = 256 step) against 20 MFLOP of
// convolution per frame. Neither kernel materialises the [B*T*784][64] conv output.
//   rgb_fwd:  a workgroup takes a run of frames; per 8-row strip of a frame (28 patches, one
//             contiguous 10.75 KB block of the image) the strip is staged in LDS (two strips ahead
//             in registers), the 4 waves each compute 16 output channels on bf16 MFMA with their
//             192 x 16 weight slice in registers, and add relu(conv + bias) into per-lane column
//             sums; one atomic per (clip, channel) and workgroup.
//   rgb_bwd:  the same walk recomputes the pre-activations, g = dfeat[b][c] / (T * 784) where
//             conv > 0, and accumulates dW[c][k] += sum_p g[p][c] patch[p][k] on MFMA (the strip is
//             also written transposed, [k][p], so the B fragments are 16-B reads) and db; each
//             workgroup stores its partial dW / db row to a slab that f3_colsum adds into the
//             gradients. No input gradient (the frames are inputs).
#include "rgb.h"

#include "igemm.h"

#include <algorithm>
#include <cstring>
#include <type_traits>

namespace f3 {

constexpr int RG_IMG = 224, RG_P = 8, RG_G = 28;                 // image side, patch, patches per side
constexpr int RG_ROWB = RG_IMG * 3 * 2;                          // bytes per image row (1344)
constexpr int RG_STRIP = RG_P * RG_ROWB;                         // bytes per 8-row strip (10752)
constexpr int RG_STRIP16 = RG_STRIP / 16;                        // 16-B pieces per strip (672)
constexpr int RG_PPT = (RG_STRIP16 + 255) / 256;                 // pieces per thread (3)
constexpr int RG_K = RG_P * RG_P * 3;                            // 192
constexpr int RG_KS = RG_K / 32;                                 // 6 MFMA k-steps
constexpr int RG_STRIPS = RG_G;                                  // strips per frame
constexpr int RG_BWD_MAXFPB = 15;                                // frames per backward workgroup (512 workgroups = 2 per CU at B=256, T=30)
typedef unsigned rg_u32x4 __attribute__((ext_vector_type(4)));  // (HIP's rg_u32x4 struct arrays went to scratch)

// patch p of a strip, k-group idx (8 consecutive k = one dy band's (dx, ch) 8-run): byte offset
F3_DEV int rg_off(int p, int idx) {
  const int dy = idx / 3, g = idx - dy * 3;
  return dy * RG_ROWB + p * 48 + g * 16;
}

// stage one strip: prefetched registers -> LDS (same byte layout as the image rows). Branch-free:
// the threads past the strip's 672 pieces rewrite the last piece with the same bytes (a conditional
// store made hipcc keep the prefetch registers in scratch)
F3_DEV void rg_store_strip(char* dst, const rg_u32x4 (&r)[RG_PPT]) {
#pragma unroll
  for (int i = 0; i < RG_PPT; ++i) {
    const int q = min((int)threadIdx.x + i * 256, RG_STRIP16 - 1);
    *reinterpret_cast<rg_u32x4*>(dst + q * 16) = r[i];
  }
}
F3_DEV void rg_load_strip(const char* src, rg_u32x4 (&r)[RG_PPT]) {
#pragma unroll
  for (int i = 0; i < RG_PPT; ++i) {
    const int q = min((int)threadIdx.x + i * 256, RG_STRIP16 - 1);
    r[i] = *reinterpret_cast<const rg_u32x4*>(src + q * 16);
  }
}

// the conv pre-activations of this wave's 16 channels for the strip in LDS: acc[t][i] =
// conv[p][c = 16w + fr] (without bias) for patch p = 16t + 4fg + i (PERM = false), or
// p = 8fg + 4t + i (PERM = true: lane fg then holds patches 8fg .. 8fg + 7 of its channel, which is
// the B-operand layout of a product that sums over patches). Rows p >= 28 are clamped duplicates.
template <bool PERM>
F3_DEV void rg_conv(const char* strip, const bf16x8 (&wf)[RG_KS], int fr, int fg, f32x4 (&acc)[2]) {
#pragma unroll
  for (int t = 0; t < 2; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int s = 0; s < RG_KS; ++s) {
    const int idx = s * 4 + fg;
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      const int p = min(PERM ? 8 * (fr >> 2) + 4 * t + (fr & 3) : t * 16 + fr, RG_G - 1);
      const bf16x8 fa = *reinterpret_cast<const bf16x8*>(strip + rg_off(p, idx));
      acc[t] = mfma_bf16x(fa, wf[s], acc[t]);
    }
  }
}

// weight slice of wave w: B fragments of W[c = 16w + fr][k = 32s + 8fg .. +8] (packed [64][192])
F3_DEV void rg_weights(const unsigned short* w, int wave, int fr, int fg, bf16x8 (&wf)[RG_KS]) {
  const unsigned short* wr = w + (size_t)(wave * 16 + fr) * RG_K + fg * 8;
#pragma unroll
  for (int s = 0; s < RG_KS; ++s) wf[s] = *reinterpret_cast<const bf16x8*>(wr + s * 32);
}

__global__ __launch_bounds__(256) void rgb_fwd_kernel(RgbArgs a) {
  __shared__ __attribute__((aligned(16))) char sbuf[2][RG_STRIP];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int fr = lane & 15, fg = lane >> 4;
  const int f0 = blockIdx.x * a.fpb, f1 = min(a.B * a.T, f0 + a.fpb);
  if (f0 >= f1) return;
  bf16x8 wf[RG_KS];
  rg_weights(a.w, wave, fr, fg, wf);
  const float bias = a.bias[wave * 16 + fr];
  const float inv = 1.f / (float)(a.T * RG_G * RG_G);
  const char* img = reinterpret_cast<const char*>(a.x);
  const int nstrip = (f1 - f0) * RG_STRIPS;
  auto strip_src = [&](int k) __attribute__((always_inline)) {  // k-th strip of the block (frame f0 + k / 28, strip k % 28)
    const int f = f0 + k / RG_STRIPS, sy = k % RG_STRIPS;
    return img + ((size_t)f * RG_IMG * RG_IMG * 3) * 2 + (size_t)sy * RG_STRIP;
  };
  rg_u32x4 pa[RG_PPT], pb[RG_PPT];  // strips k (even) and k + 1 (odd), two ahead of the LDS copy
  rg_load_strip(strip_src(0), pa);
  rg_load_strip(strip_src(min(1, nstrip - 1)), pb);
  float csum = 0.f;
  int fcur = f0 / a.T;  // clip of the current frame
  auto flush = [&](int clip) __attribute__((always_inline)) {
    float v = csum;
    v += __shfl_xor(v, 16, 64);
    v += __shfl_xor(v, 32, 64);
    if (fg == 0) atomic_add_f(a.feat + (size_t)clip * 64 + wave * 16 + fr, v * inv);
    csum = 0.f;
  };
  // one strip (even strips use sbuf[0] / pa, odd ones sbuf[1] / pb: a runtime index into a
  // prefetch array put it in scratch)
  auto step = [&](int k, char* buf, rg_u32x4 (&P)[RG_PPT]) __attribute__((always_inline)) {
    rg_store_strip(buf, P);
    rg_load_strip(strip_src(min(k + 2, nstrip - 1)), P);  // (unconditional: see rg_store_strip)
    __syncthreads();
    f32x4 acc[2];
    rg_conv<false>(buf, wf, fr, fg, acc);
    const int clip = (f0 + k / RG_STRIPS) / a.T;
    if (clip != fcur) {
      flush(fcur);
      fcur = clip;
    }
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int i = 0; i < 4; ++i)
        if (t * 16 + fg * 4 + i < RG_G) csum += fmaxf(acc[t][i] + bias, 0.f);
    __syncthreads();  // buf is restaged two strips later; every wave's reads of it are done
  };
  for (int k = 0; k < nstrip; k += 2) {
    step(k, sbuf[0], pa);
    if (k + 1 < nstrip) step(k + 1, sbuf[1], pb);
  }
  flush(fcur);
}

// dW^T[k][c] = sum_p X^T[k][p] mask[p][c] per strip, on bf16 MFMA 16x16x32 without any LDS copy
// besides the staged strip: A = X^T comes straight from the strip image through the transposed LDS
// read (ds_read_b64_tr_b16: a 16-lane group reads 4 patches x 16 consecutive k and each lane gets
// one k's 4 patches), B = the exact 0/1 relu mask, built in registers by the permuted conv
// (rg_conv<true>). The mask is constant-weighted within a clip (g = dfeat / (T*784) where the
// pre-activation is > 0), so the MFMAs accumulate the clip's unscaled sums and its df scales them
// in fp32 when the block moves to the next clip.
typedef short rg_s16x4 __attribute__((ext_vector_type(4)));
F3_DEV rg_s16x4 rg_tr_read(const char* p) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) rg_s16x4*)(p));
}

__global__ __launch_bounds__(256) void rgb_bwd_kernel(RgbArgs a) {
  __shared__ __attribute__((aligned(16))) char sbuf[2][RG_STRIP];
  __shared__ float dfs[RG_BWD_MAXFPB][64];  // dfeat / (T*784) of this block's clips
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int fr = lane & 15, fg = lane >> 4;
  const int f0 = blockIdx.x * a.fpb, f1 = min(a.B * a.T, f0 + a.fpb);
  bf16x8 wf[RG_KS];
  rg_weights(a.w, wave, fr, fg, wf);
  const float bias = a.bias[wave * 16 + fr];
  const float inv = 1.f / (float)(a.T * RG_G * RG_G);
  const char* img = reinterpret_cast<const char*>(a.x);
  const int nstrip = f0 < f1 ? (f1 - f0) * RG_STRIPS : 0;
  auto strip_src = [&](int k) __attribute__((always_inline)) {
    const int f = f0 + k / RG_STRIPS, sy = k % RG_STRIPS;
    return img + ((size_t)f * RG_IMG * RG_IMG * 3) * 2 + (size_t)sy * RG_STRIP;
  };
  // the upstream gradient of every clip this block touches (at most fpb clips), read once here so
  // the strip loop has no global load besides the strip prefetch
  const int clip0 = f0 / a.T;
  for (int i = tid; i < RG_BWD_MAXFPB * 64; i += 256) {
    const int cl = min(clip0 + i / 64, a.B - 1);
    dfs[i / 64][i % 64] = a.dfeat[(size_t)cl * 64 + i % 64] * inv;
  }
  // transposed-read addresses: lane (q = fr >> 2, r = fr & 3) of group fg points at patch
  // 8fg + 4h + q, k = 16j + 4r .. +3 (one dy band: 24 is a multiple of 4); patches past 27 clamp
  int troff[2][12];
#pragma unroll
  for (int h = 0; h < 2; ++h)
#pragma unroll
    for (int j = 0; j < 12; ++j) {
      const int p = min(8 * fg + 4 * h + (fr >> 2), RG_G - 1), kc = 16 * j + 4 * (fr & 3);
      const int dy = kc / 24;
      troff[h][j] = dy * RG_ROWB + p * 48 + (kc - dy * 24) * 2;
    }
  f32x4 dw[12];   // dW^T[k = 16j + 4fg + i][c = 16w + fr]
  f32x4 dwc[12];  // the current clip's unscaled mask^T x patch sums (scaled by its df at the clip's end)
#pragma unroll
  for (int j = 0; j < 12; ++j) dw[j] = dwc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
  int ccur = 0;  // clip of dwc (relative to clip0)
  auto flush = [&]() __attribute__((always_inline)) {
    const float dfc = dfs[ccur][wave * 16 + fr];
#pragma unroll
    for (int j = 0; j < 12; ++j) {
#pragma unroll
      for (int i = 0; i < 4; ++i) dw[j][i] = fmaf(dfc, dwc[j][i], dw[j][i]);
      dwc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
    }
  };
  float dbs = 0.f;
  rg_u32x4 pa[RG_PPT], pb[RG_PPT];
  if (nstrip > 0) {
    rg_load_strip(strip_src(0), pa);
    rg_load_strip(strip_src(min(1, nstrip - 1)), pb);
  }
  __syncthreads();
  auto step = [&](int k, char* buf, rg_u32x4 (&P)[RG_PPT]) __attribute__((always_inline)) {
    rg_store_strip(buf, P);
    rg_load_strip(strip_src(min(k + 2, nstrip - 1)), P);  // (unconditional: see rg_store_strip)
    __syncthreads();
    f32x4 acc[2];
    rg_conv<true>(buf, wf, fr, fg, acc);
    const int cl = (f0 + k / RG_STRIPS) / a.T - clip0;
    if (cl != ccur) {
      flush();
      ccur = cl;
    }
    const float df = dfs[cl][wave * 16 + fr];
    bf16x8 mk;  // B operand: mask[p = 8fg + e][c = fr]
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const bool on = 8 * fg + 4 * t + i < RG_G && acc[t][i] + bias > 0.f;
        dbs += on ? df : 0.f;
        mk[4 * t + i] = (__bf16)(on ? 1.f : 0.f);
      }
#pragma unroll
    for (int j = 0; j < 12; ++j) {
      const rg_s16x4 lo = rg_tr_read(buf + troff[0][j]), hi = rg_tr_read(buf + troff[1][j]);
      // (whole-vector bit cast: element-wise short -> __bf16 casts were mis-assembled by hipcc)
      const bf16x8 xa = __builtin_bit_cast(bf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
      dwc[j] = mfma_bf16x(xa, mk, dwc[j]);
    }
    __syncthreads();  // buf is restaged two strips later; every wave's reads of it are done
  };
  for (int k = 0; k < nstrip; k += 2) {
    step(k, sbuf[0], pa);
    if (k + 1 < nstrip) step(k + 1, sbuf[1], pb);
  }
  flush();
  // this workgroup's partial row: dW [64][192] then db [64]
  float* row = a.part + (size_t)blockIdx.x * (64 * RG_K + 64);
#pragma unroll
  for (int j = 0; j < 12; ++j)
    *reinterpret_cast<f32x4*>(row + (size_t)(wave * 16 + fr) * RG_K + j * 16 + fg * 4) = dw[j];
  dbs += __shfl_xor(dbs, 16, 64);
  dbs += __shfl_xor(dbs, 32, 64);
  if (fg == 0) row[64 * RG_K + wave * 16 + fr] = dbs;
}

}  // namespace f3

using namespace f3;

static bool rgb_ok(const RgbArgs* a) {
  return a && a->x && a->w && a->bias && a->B > 0 && a->T > 0 && a->fpb > 0;
}

int f3_rgb_fwd(RgbArgs a, hipStream_t s) {
  if (!rgb_ok(&a) || !a.feat) return F3_EINVAL;
  const int frames = a.B * a.T;
  hipLaunchKernelGGL(rgb_fwd_kernel, dim3((frames + a.fpb - 1) / a.fpb), dim3(256), 0, s, a);
  F3_LAUNCH_CHECK();
  return F3_OK;
}

int f3_rgb_bwd_blocks(const RgbArgs* a) { return (a->B * a->T + a->fpb - 1) / a->fpb; }

int f3_rgb_bwd(RgbArgs a, hipStream_t s) {
  if (!rgb_ok(&a) || !a.dfeat || !a.part) return F3_EINVAL;
  hipLaunchKernelGGL(rgb_bwd_kernel, dim3(f3_rgb_bwd_blocks(&a)), dim3(256), 0, s, a);
  F3_LAUNCH_CHECK();
  return F3_OK;
}

// ---------------------------------------------------------------------------------------------
// C ABI (include/fall3.h)
// ---------------------------------------------------------------------------------------------
// out[c] += sum_r part[r * stride + col0 + c] for c < cols: block = 64 columns x 4 row groups
__global__ __launch_bounds__(256) void rgb_colsum_kernel(const float* __restrict__ part, int rows, int stride,
                                                         int col0, int cols, float* __restrict__ out) {
  __shared__ float red[4][64];
  const int lane = threadIdx.x & 63, rg = threadIdx.x >> 6, c = blockIdx.x * 64 + lane;
  float acc0 = 0.f, acc1 = 0.f;
  if (c < cols) {
    int r = rg;
    for (; r + 4 < rows; r += 8) {
      acc0 += part[(size_t)r * stride + col0 + c];
      acc1 += part[(size_t)(r + 4) * stride + col0 + c];
    }
    if (r < rows) acc0 += part[(size_t)r * stride + col0 + c];
  }
  red[rg][lane] = acc0 + acc1;
  __syncthreads();
  if (rg == 0 && c < cols) out[c] += (red[0][lane] + red[1][lane]) + (red[2][lane] + red[3][lane]);
}

static int rgb_colsum(const float* part, int rows, int stride, int col0, int cols, float* out, hipStream_t s) {
  hipLaunchKernelGGL(rgb_colsum_kernel, dim3((cols + 63) / 64), dim3(256), 0, s, part, rows, stride, col0, cols, out);
  F3_LAUNCH_CHECK();
  return F3_OK;
}

static RgbArgs rgb_args(const void* frames, const void* wpack, const float* bias, int B, int T, int fpb) {
  RgbArgs a;
  std::memset(&a, 0, sizeof(a));
  a.B = B; a.T = T; a.fpb = fpb;
  a.x = reinterpret_cast<const unsigned short*>(frames);
  a.w = reinterpret_cast<const unsigned short*>(wpack);
  a.bias = bias;
  return a;
}

constexpr int kRgbFwdFpb = 6, kRgbBwdFpb = RG_BWD_MAXFPB;

extern "C" {

long long f3_rgb_scratch_floats(int B, int T) {
  if (B <= 0 || T <= 0) return 0;
  return (long long)((B * T + kRgbBwdFpb - 1) / kRgbBwdFpb) * (64 * RG_K + 64);
}

int f3_rgb_forward(const void* frames, const void* wpack, const float* bias, float* feat, int B, int T, void* stream) {
  if (!frames || !wpack || !bias || !feat || B <= 0 || T <= 0) return F3_EINVAL;
  hipStream_t s = (hipStream_t)stream;
  if (hipMemsetAsync(feat, 0, sizeof(float) * B * 64, s) != hipSuccess) return F3_EHIP;
  RgbArgs a = rgb_args(frames, wpack, bias, B, T, kRgbFwdFpb);
  a.feat = feat;
  return f3_rgb_fwd(a, s);
}

int f3_rgb_backward(const void* frames, const void* wpack, const float* bias, const float* dfeat, float* dw, float* db,
                    float* scratch, long long scratch_floats, int B, int T, void* stream) {
  if (!frames || !wpack || !bias || !dfeat || !dw || !db || !scratch || B <= 0 || T <= 0) return F3_EINVAL;
  if (scratch_floats < f3_rgb_scratch_floats(B, T)) return F3_EINVAL;
  hipStream_t s = (hipStream_t)stream;
  RgbArgs a = rgb_args(frames, wpack, bias, B, T, kRgbBwdFpb);
  a.dfeat = dfeat;
  a.part = scratch;
  const int rows = f3_rgb_bwd_blocks(&a);
  int st = f3_rgb_bwd(a, s);
  if (st != F3_OK) return st;
  if (hipMemsetAsync(dw, 0, sizeof(float) * 64 * RG_K, s) != hipSuccess) return F3_EHIP;
  if (hipMemsetAsync(db, 0, sizeof(float) * 64, s) != hipSuccess) return F3_EHIP;
  // the partial rows are [dW (64*192) | db (64)]: two column sums over the same rows (each output
  // element is written by one thread: plain adds, deterministic)
  st = rgb_colsum(scratch, rows, 64 * RG_K + 64, 0, 64 * RG_K, dw, s);
  if (st != F3_OK) return st;
  return rgb_colsum(scratch, rows, 64 * RG_K + 64, 64 * RG_K, 64, db, s);
}

}  // extern "C"
