// Weight-stationary implicit GEMM for the 64-channel temporal convolutions of the skeleton
// streams (stgcan.py:112-121, the (9,1) tcn of the 64-channel blocks, stride 1): the forward
// h = conv(u) + bias with BN2 statistics and the channel-attention pool in the epilogue, and the
// input gradient dg = (conv^T(dh)) . [bn1(g) > 0] with the BN1-backward sums (RELUMASK).
//
// Why a separate kernel. At Kc = Nc = 64 the GEMM is small in K (9 taps x 64 = 576) and in N (64)
// and large in M (B*T*V = 138,240 rows): 10.2 GFLOP and ~35 MB of bf16 rows per launch, i.e. a few
// microseconds at the HBM or MFMA roofline. The tiled igemm_bf16 (128 x 64 tiles, 1080 workgroups,
// a 9-stage k loop each) spent ~50 us on it: every tile paid its prologue (the B panel, the window),
// a barrier per tap and an epilogue with fp64 atomics, with only ~3 workgroups per CU to hide them.
// Here each workgroup is persistent over a contiguous range of 128-row tiles:
//   - the 64 x 576 weight panel lives in REGISTERS for the whole launch (each of the 8 waves owns a
//     32-column slice: 2 column tiles x 18 k-steps of bf16x8 = 144 VGPRs), loaded once;
//   - the A operand of a tile is its input WINDOW, rows [m0 - P*V, m0 + 128 + P*V), staged once by
//     LDS-DMA (global_load_lds, 16-B pieces, XOR-swizzled 128-B rows) into one of two buffers while
//     the previous tile computes; the 9 taps read it shifted by whole frames, and rows whose frame
//     leaves the clip (temporal zero padding) are zeroed in the fragment;
//   - BN statistics stay in registers across tiles and are added once per workgroup; the pool
//     (GAP) and the bf16 output leave per tile through LDS (coalesced 16-B row stores, issued at
//     the start of the next tile so they drain under its MFMAs).
#include "igemm.h"

#include <algorithm>

namespace f3 {

constexpr int T64_BM = 128;                       // rows per tile
constexpr int T64_THREADS = 512;                  // 8 waves: wm = wave & 3 (32 rows), wj = wave >> 2 (32 cols)
constexpr int T64_KS = 18;                        // k-steps of 32: 9 taps x 64 channels
constexpr int T64_WROWS = T64_BM + 2 * 4 * 18;    // window capacity (P <= 4, V <= 18)
constexpr int T64_WIN = T64_WROWS * 128;          // bytes per window buffer
constexpr int T64_OTS = 64 + 8;                   // output staging row stride (bf16)
constexpr int T64_OT_OFF = 2 * T64_WIN;
constexpr int T64_RED_OFF = T64_OT_OFF + T64_BM * T64_OTS * 2;
constexpr int T64_LDS = T64_RED_OFF + 4 * 2 * 64 * 4;
static_assert(T64_LDS <= 160 * 1024, "tcn64 LDS");

template <int EPI>
__global__ __launch_bounds__(T64_THREADS) void tcn64_kernel(ConvGemmArgs a, int ntiles, int per_wg) {
  extern __shared__ __attribute__((aligned(16))) char t64_smem[];
  __bf16* ot = reinterpret_cast<__bf16*>(t64_smem + T64_OT_OFF);
  float* red = reinterpret_cast<float*>(t64_smem + T64_RED_OFF);  // [4 wm][2][64] pool partials
  const ConvGeom& g = a.g;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave & 3, wj = wave >> 2;
  const int fr = lane & 15, fg = lane >> 4;
  const int V = g.V, T = g.T_out, TV = T * V, PV = g.P * V, WR = T64_BM + 2 * PV;
  const int tile0 = blockIdx.x * per_wg, tile1 = min(ntiles, tile0 + per_wg);
  if (tile0 >= tile1) return;

  // this wave's weight slice, columns wj*32 + y*16 + fr, all 18 k-steps (packed [64][576] bf16):
  // 144 VGPRs, the MFMA B operands of every tile. (Holding the whole panel in one wave per SIMD —
  // 288 registers — made hipcc shuttle it through AGPRs with v_accvgpr_read before every MFMA.)
  bf16x8 wf[2][T64_KS];
#pragma unroll
  for (int y = 0; y < 2; ++y) {
    const unsigned short* wr = a.wb + (size_t)(wj * 32 + y * 16 + fr) * (T64_KS * 32) + fg * 8;
#pragma unroll
    for (int kk = 0; kk < T64_KS; ++kk) wf[y][kk] = *reinterpret_cast<const bf16x8*>(wr + kk * 32);
  }
  // per-column epilogue coefficients of the lane's two columns
  float bias[2] = {0.f, 0.f}, sc[2], sh[2], mu[2], rs[2];
#pragma unroll
  for (int y = 0; y < 2; ++y) {
    const int j = wj * 32 + y * 16 + fr;
    if (EPI & EPI_BIAS) bias[y] = a.bias[j];
    if (EPI & EPI_RELUMASK) bn_coeff(a.epi_bn, j, sc[y], sh[y], mu[y], rs[y]);
  }
  float ssum[2] = {0.f, 0.f}, ssq[2] = {0.f, 0.f};

  // window staging: 1-KiB DMA pieces (8 rows of 128 B), dealt round-robin over the 8 waves
  const int sub = lane >> 3, pch = lane & 7;
  auto load_win = [&](int tile, int buf) {
    const int m0 = tile * T64_BM, nwp = (WR + 7) >> 3;
    char* dst = t64_smem + buf * T64_WIN;
    for (int q = wave; q < nwp; q += 8) {
      const int rr = q * 8 + sub, gm = m0 - PV + rr;
      const bool ok = rr < WR && gm >= 0 && gm < g.M;
      const unsigned short* src = ok ? a.inb + (size_t)gm * g.lda + swz(rr, pch) * 8 : a.zero;
      __builtin_amdgcn_global_load_lds((const void*)src, (lds_void_t*)(dst + q * 1024), 16, 0, 0);
    }
  };
  // the staged bf16 output of a tile -> HBM (16-B row pieces; 128 rows x 8 pieces = 2 per thread)
  auto store_tile = [&](int tile) {
    const int m0 = tile * T64_BM;
    for (int q = tid; q < T64_BM * 8; q += T64_THREADS) {
      const int rl = q >> 3, c = q & 7, m = m0 + rl;
      if (m >= g.M) continue;
      *reinterpret_cast<uint4*>(reinterpret_cast<__bf16*>(a.outb) + (size_t)m * g.ldo + c * 8) =
          *reinterpret_cast<const uint4*>(ot + rl * T64_OTS + c * 8);
    }
  };

  load_win(tile0, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  int buf = 0;
  for (int tile = tile0; tile < tile1; ++tile, buf ^= 1) {
    const int m0 = tile * T64_BM;
    if (tile > tile0) store_tile(tile - 1);
    if (tile + 1 < tile1) load_win(tile + 1, buf ^ 1);
    // ---- 9 taps x 2 k-halves from the window ----
    const char* win = t64_smem + buf * T64_WIN;
    int tfr[2];
#pragma unroll
    for (int x = 0; x < 2; ++x) tfr[x] = ((m0 + wm * 32 + x * 16 + fr) / V) % T;
    f32x4 acc[2][2];
#pragma unroll
    for (int x = 0; x < 2; ++x)
#pragma unroll
      for (int y = 0; y < 2; ++y) acc[x][y] = f32x4{0.f, 0.f, 0.f, 0.f};
    // k-step s = (tap dt = s / 2, channel half h = s % 2)
#pragma unroll
    for (int s = 0; s < T64_KS; ++s) {
      const int dt = s >> 1, c = (s & 1) * 4 + fg;
      const int wo = (g.transposed ? 2 * g.P - dt : dt) * V, wsh = g.transposed ? g.P - dt : dt - g.P;
#pragma unroll
      for (int x = 0; x < 2; ++x) {
        const int r = wm * 32 + x * 16 + fr + wo;
        const bf16x8 v = *reinterpret_cast<const bf16x8*>(win + r * 128 + swz(r, c) * 16);
        const bf16x8 fa = (unsigned)(tfr[x] + wsh) < (unsigned)T ? v : bf16x8{};
#pragma unroll
        for (int y = 0; y < 2; ++y) acc[x][y] = mfma_bf16x(fa, wf[y][s], acc[x][y]);
      }
    }
    // RELUMASK source (bf16 g) of the lane's 8 rows x 2 columns. Loaded after the MFMAs: its wait
    // also waits for the next window's DMA (issued earlier; the DMA loop's count is not static),
    // which has had the whole k loop to land
    unsigned pre[2][4];  // two bf16 per register (columns y = 0, 1)
    if (EPI & EPI_RELUMASK) {
#pragma unroll
      for (int x = 0; x < 2; ++x)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int m = min(m0 + wm * 32 + x * 16 + fg * 4 + r, g.M - 1);
          const unsigned short* gr = a.auxb + (size_t)m * a.ldaux + wj * 32 + fr;
          pre[x][r] = (unsigned)gr[0] | ((unsigned)gr[16] << 16);
        }
    }
    // every thread's reads of `ot` (store_tile above) are done. A raw barrier: __syncthreads()
    // would also wait for the next window's DMA (vmcnt(0)), which should stay in flight
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    // ---- epilogue: bias / mask, statistics, pool, bf16 staging ----
    const int nlo = m0 / TV;
    float gp0[2] = {0.f, 0.f}, gp1[2] = {0.f, 0.f};
#pragma unroll
    for (int x = 0; x < 2; ++x)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int rl = wm * 32 + x * 16 + fg * 4 + r, m = m0 + rl;
        const bool ok = m < g.M;
        const int n = m / TV;
#pragma unroll
        for (int y = 0; y < 2; ++y) {
          float v = ok ? acc[x][y][r] : 0.f;
          if (EPI & EPI_BIAS) v = ok ? v + bias[y] : 0.f;
          if (EPI & EPI_RELUMASK) {
            const float gv = __uint_as_float(y == 0 ? pre[x][r] << 16 : pre[x][r] & 0xffff0000u);
            if (gv * sc[y] + sh[y] <= 0.f) v = 0.f;
            ssum[y] += v;
            ssq[y] += v * ((gv - mu[y]) * rs[y]);
          } else if (EPI & EPI_STATS) {
            ssum[y] += v;
            ssq[y] += v * v;
          }
          if (EPI & EPI_GAP) {
            if (n == nlo) gp0[y] += v;
            else gp1[y] += v;  // a 128-row tile spans at most two clips (T*V >= 128 checked by the launcher)
          }
          ot[rl * T64_OTS + wj * 32 + y * 16 + fr] = (__bf16)v;
        }
      }
    if (EPI & EPI_GAP) {
#pragma unroll
      for (int y = 0; y < 2; ++y) {
        gp0[y] += __shfl_xor(gp0[y], 16, 64);
        gp0[y] += __shfl_xor(gp0[y], 32, 64);
        gp1[y] += __shfl_xor(gp1[y], 16, 64);
        gp1[y] += __shfl_xor(gp1[y], 32, 64);
        if (fg == 0) {
          red[(wm * 2 + 0) * 64 + wj * 32 + y * 16 + fr] = gp0[y];
          red[(wm * 2 + 1) * 64 + wj * 32 + y * 16 + fr] = gp1[y];
        }
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    if ((EPI & EPI_GAP) && tid < 128) {
      const int half = tid >> 6, j = tid & 63;
      const float s = red[(0 * 2 + half) * 64 + j] + red[(1 * 2 + half) * 64 + j] + red[(2 * 2 + half) * 64 + j] +
                      red[(3 * 2 + half) * 64 + j];
      const int n = nlo + half;
      if (n * TV < g.M && (half == 0 || s != 0.f)) atomic_add_f(a.gap + (size_t)n * 64 + j, s);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the next window (and this tile's loads)
    __syncthreads();
  }
  store_tile(tile1 - 1);
  // ---- BN sums of the workgroup's tiles: lanes -> waves -> one fp64 add per column ----
  if (EPI & (EPI_STATS | EPI_RELUMASK)) {
#pragma unroll
    for (int y = 0; y < 2; ++y) {
      ssum[y] += __shfl_xor(ssum[y], 16, 64);
      ssum[y] += __shfl_xor(ssum[y], 32, 64);
      ssq[y] += __shfl_xor(ssq[y], 16, 64);
      ssq[y] += __shfl_xor(ssq[y], 32, 64);
    }
    __syncthreads();
    if (fg == 0) {
#pragma unroll
      for (int y = 0; y < 2; ++y) {
        red[(wm * 2 + 0) * 64 + wj * 32 + y * 16 + fr] = ssum[y];
        red[(wm * 2 + 1) * 64 + wj * 32 + y * 16 + fr] = ssq[y];
      }
    }
    __syncthreads();
    if (tid < 128) {
      const int q = tid >> 6, j = tid & 63;
      const float s = red[(0 * 2 + q) * 64 + j] + red[(1 * 2 + q) * 64 + j] + red[(2 * 2 + q) * 64 + j] +
                      red[(3 * 2 + q) * 64 + j];
      atomic_add_d((q == 0 ? a.st_sum : a.st_sq) + j, (double)s);
    }
  }
}

}  // namespace f3

using namespace f3;

// Shapes this kernel takes: 64 -> 64 channels, 9 taps, stride 1, "same" padding, T_in == T_out,
// bf16 in / out, a clip at least one tile long (a tile spans at most two clips), and the two
// epilogues of the bf16 step (tcn forward, tcn input gradient).
bool f3_tcn64_ok(const ConvGemmArgs& a, int epi) {
  const ConvGeom& g = a.g;
  if (!a.inb || !a.wb || !a.zero || !a.outb || a.x3n) return false;
  if (g.Kc != 64 || g.Nc != 64 || g.KT != 9 || g.S != 1 || g.P != 4 || g.T_in != g.T_out) return false;
  if (g.V > 18 || g.lda % 8 != 0 || g.ldo % 8 != 0 || g.T_out * g.V < T64_BM || g.M % (g.T_out * g.V) != 0) return false;
  if (epi == (EPI_BIAS | EPI_STATS | EPI_GAP)) return a.gap && a.st_sum && a.st_sq && a.bias;
  if (epi == EPI_RELUMASK) return a.auxb && a.st_sum && a.st_sq;
  return false;
}

int f3_tcn64(const ConvGemmArgs* args, int epi, hipStream_t s) {
  const ConvGemmArgs& a = *args;
  const int ntiles = (a.g.M + T64_BM - 1) / T64_BM;
  static int cus = [] {
    int dev = 0, n = 256;
    if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev);
    (void)hipGetLastError();
    return n;
  }();
  // tiles per workgroup: one round over the CUs
  const int per_wg = (ntiles + cus - 1) / cus;
  const int grid = (ntiles + per_wg - 1) / per_wg;
  if (epi == (EPI_BIAS | EPI_STATS | EPI_GAP)) {
    F3_LDS_LIMIT((tcn64_kernel<EPI_BIAS | EPI_STATS | EPI_GAP>), T64_LDS);
    hipLaunchKernelGGL((tcn64_kernel<EPI_BIAS | EPI_STATS | EPI_GAP>), dim3(grid), dim3(T64_THREADS), T64_LDS, s, a,
                       ntiles, per_wg);
  } else if (epi == EPI_RELUMASK) {
    F3_LDS_LIMIT(tcn64_kernel<EPI_RELUMASK>, T64_LDS);
    hipLaunchKernelGGL((tcn64_kernel<EPI_RELUMASK>), dim3(grid), dim3(T64_THREADS), T64_LDS, s, a, ntiles, per_wg);
  } else {
    return F3_EINVAL;
  }
  F3_LAUNCH_CHECK();
  return F3_OK;
}
