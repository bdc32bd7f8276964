// Device helpers shared by the bf16 implicit-GEMM kernels (gemm_glds.hip, gemm_big.hip):
// MFMA wrapper, LDS chunk swizzle, XCD remap and the implicit-GEMM row maps.
#pragma once
#include "common.h"
#include "kernels.h"

namespace f3 {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __attribute__((address_space(3))) void lds_void_t;

constexpr int G_BK = 64;  // k depth of one LDS stage (64 bf16 = one 128-B row)

F3_DEV f32x4 mfma_bf16x(bf16x8 a, bf16x8 b, f32x4 c) { return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0); }

F3_DEV int g_src_row(int n, int t, int v, int dt, const ConvGeom& g) {
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

// 16-B chunk c of a 128-B LDS row r sits at position c ^ (r & 7): conflict-free ds_read_b128 fragment
// reads (16 consecutive rows x one chunk per half-wave group) at ANY first row, so tap-shifted window
// reads cost no bank conflicts (the former c ^ ((r >> 1) & 7) was conflict-free only at even 16-row
// offsets: 26 % of the window kernels' LDS cycles were conflicts)
F3_DEV int swz(int r, int c) { return c ^ (r & 7); }

// bf16x3 native form (ConvGemmArgs::x3n): the 16-B chunk cg (0..7) of the staged 128-B row piece of
// channel block i0 (32 channels) comes from the hi half (cg < 4: column i0 + 8 cg) or the lo half
// (cg >= 4: column C + i0 + 8 (cg - 4)) of a row [x_hi (C) | x_lo (C)]
F3_DEV int x3n_col(int C, int i0, int cg) { return i0 + 8 * cg + (cg >= 4 ? C - 32 : 0); }

// Parity-split rows for a stride-2 input gradient (see igemm_bf16). Measured on MI355X (B=256,
// V=18): tcn layer 5 (Kc=256) 162 -> 144 us, but layer 3 (Kc=128, 2 k-chunks per tap) 85 ->
// 94 us — with short per-tap k loops the halved MFMA work does not pay for the wider row
// footprint of a parity tile — so it is used from Kc >= 256, and for 1x1 convs (where the
// odd rows need no work at all).
__host__ __device__ inline bool igemm_parity(const ConvGeom& g) {
  return g.transposed && g.S == 2 && (g.KT == 1 || g.Kc >= 256);
}

// bijective XCD-aware remap: consecutive logical tiles land on one XCD (shared A panels)
F3_DEV int xcd_remap(int orig, int nwg) {
  const int xcd = orig & 7, q = nwg >> 3, r = nwg & 7;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (orig >> 3);
}

// Per staging row: branch-free source row for tap dt. Forward: ti = t*S + dt - P, valid in
// [0, T_in). Transposed (dgrad): x = t + P - dt, valid if x >= 0, x % S == 0, x / S < T_in
// (S is 1 or 2). base = first source row of the clip + v; q = t*S - P (fwd) or t + P (dgrad).
struct RowMap {
  int base, q;  // base < 0: row outside M
};

F3_DEV RowMap rowmap(int m, const ConvGeom& g) {
  RowMap r;
  if (m < 0 || m >= g.M) { r.base = -1; r.q = 0; return r; }
  const int nt = m / g.V, v = m - nt * g.V, n = nt / g.T_out, t = nt - n * g.T_out;
  r.base = n * g.T_in * g.V + v;
  r.q = g.transposed ? t + g.P : t * g.S - g.P;
  return r;
}

F3_DEV int rowmap_src(const RowMap& r, int dt, const ConvGeom& g) {
  int ti;
  bool ok;
  if (!g.transposed) {
    ti = r.q + dt;
    ok = ti >= 0 && ti < g.T_in;
  } else {
    const int x = r.q - dt;
    ti = g.S == 2 ? (x >> 1) : x;
    ok = x >= 0 && (g.S == 1 || (x & 1) == 0) && ti < g.T_in;
  }
  return (ok && r.base >= 0) ? r.base + ti * g.V : -1;
}

}  // namespace f3
