// RGB spatial-conv branch (build-defined; see rgb.hip).
#pragma once
#include <hip/hip_runtime.h>

#include "common.h"

namespace f3 {

struct RgbArgs {
  int B, T;
  int fpb;                    // frames per workgroup
  const unsigned short* x;    // bf16 frames [B][T][224][224][3]
  const unsigned short* w;    // bf16 packed conv weight [64][192], k = (dy*8 + dx)*3 + ch
  const float* bias;          // [64]
  float* feat;                // fwd out [B][64] (accumulated: zeroed by the caller)
  const float* dfeat;         // bwd in [B][64]
  float* part;                // bwd out: per-workgroup partial rows [blocks][64*192 + 64]
};

}  // namespace f3

int f3_rgb_fwd(f3::RgbArgs a, hipStream_t s);
int f3_rgb_bwd(f3::RgbArgs a, hipStream_t s);
int f3_rgb_bwd_blocks(const f3::RgbArgs* a);
