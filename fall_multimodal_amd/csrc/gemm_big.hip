// Large-tile bf16 implicit-GEMM temporal/graph convolution for the 128- and 256-channel
// layers: one 144-row (256 channels) or 288-row (128 channels) output tile per CU.
//
//   Out[m][j] = sum_{dt,i} In[src(m,dt)][i] * W[j][dt*Kc+i]     (fwd, or dgrad via the
//                                                                 transposed row map)
// Why a second kernel: at B=256, V=18 the 256-channel layers have M = 36864 output rows, so
// 128x128 tiles give 576 tiles = 2.25 per CU — two rounds with a 1/8-full tail, at 2
// workgroups per CU whose 2-stage vmcnt(0) loops leave the HBM/L2 latency exposed (measured
// 430-455 TF on the layer-6 tcn). Here a workgroup owns BM x Nc with BM = 144 (256 ch) or
// 288 (128 ch): M = 36864 is exactly 256 tiles, M = 69120 is 240 (one round either way).
// Each of the 8 waves (2 per SIMD, so one wave's LDS reads overlap the other's MFMAs) owns
// a 144 x 32 sub-tile (9 x 2 MFMA 16x16x32 tiles, 72 fp32 accumulators per lane): per 64-deep
// k step a wave issues 36 MFMAs against 22 KiB of LDS fragment reads. Staging is LDS-DMA
// (global_load_lds_dwordx4) into three stages with two in flight across raw barriers (counted
// vmcnt) — the ~1 workgroup/CU structure of cdna_hip_programming.md §5 "Pipelining across
// barriers". A stage is 1-KiB pieces (8 rows x 128 B, XOR-swizzled through the source address
// as in gemm_glds.hip), dealt round-robin to the 8 waves; where the pieces do not divide
// evenly a wave re-issues an earlier piece (identical bytes to the identical LDS address), so
// every wave's vmcnt count is the same constant.
// Row maps, the stride-2 parity split and the epilogues are those of igemm_bf16.
#include "igemm.h"

namespace f3 {

constexpr int BG_MT = 9, BG_NT = 2, BG_NST = 3;  // per-wave MFMA tiles (rows x cols), LDS stages
constexpr int BG_WAVES = 8, BG_THREADS = 64 * BG_WAVES;

// (Loading the weight fragments straight from global memory into registers, so the LDS stages carry
// the A rows only, measured slower: 67 -> 87 us on the layer-6 forward)
// WIN (clip window): for stride-1 temporal convs whose clips are exactly 144 rows (T*V = 144,
// the 256-channel layers at T = 8) a workgroup owns two whole clips x BN = 128 output channels.
// Each channel chunk's 288 input rows are staged ONCE (two 36-KiB A buffers) and all KT taps
// read them shifted by (dt - P) frames, rows falling outside the clip read as zero; only the
// weights are staged per (chunk, tap) step (16 KiB). Per workgroup that is 4 x 36 + 36 x 16 =
// 720 KiB of L2 -> LDS fill instead of 36 x 50 KiB = 1.8 MiB for the 144 x 256 tile.
typedef __attribute__((address_space(3))) const char lds_cchar_t;
constexpr int WIN_APS = 6;  // A pieces of the next chunk carried by one step (steps 2..7 of 9)
template <int WM, int WN, bool WIN = false>
struct BigCfg {
  static constexpr int BM = 16 * BG_MT * WM, BN = 16 * BG_NT * WN;
  static constexpr int AP = WIN ? WIN_APS : BM / 8, BP = BN / 8, NP = AP + BP;  // 1-KiB pieces per stage
  static constexpr int PPW = (NP + BG_WAVES - 1) / BG_WAVES;              // pieces per wave
  static constexpr int STAGE = WIN ? BN * 128 : NP * 1024;
  static constexpr int AWIN = WIN ? BM * 128 : 0;    // one A window buffer (WIN: two of them)
  static constexpr int SOFF = 2 * AWIN;              // byte offset of the per-step stages
  // the epilogue's output image (16 KiB + BM x (BN + 8) bf16) reuses the stages' bytes
  static constexpr int OT_NEED = 16 * 1024 + BM * (BN + 8) * 2;
  static constexpr int EPI_OFF = SOFF + BG_NST * STAGE > OT_NEED ? SOFF + BG_NST * STAGE : OT_NEED;
  static constexpr int ZOFF = EPI_OFF + 4 * BN * 4;  // WIN: one zero row, read for out-of-clip taps
  static constexpr int SMEM = ZOFF + (WIN ? 128 : 0);
};

// X3N: the bf16x3 native form (ConvGemmArgs::x3n): a k step is one 32-channel block, its staged row
// piece [x_hi 32 | x_lo 32] / [W_hi 32 | W_lo 32], and the wave issues x_hi W_hi + x_lo W_hi + x_hi W_lo
template <int EPI, int WM, int WN, bool WIN = false, bool X3N = false>
__global__ __launch_bounds__(BG_THREADS) void igemm_big(ConvGemmArgs a) {
  using Cfg = BigCfg<WM, WN, WIN>;
  static_assert(!(WIN && (WM != 2 || BG_MT * 16 != 144)), "WIN: two 144-row clips");
  constexpr int BM = Cfg::BM, BN = Cfg::BN, AP = Cfg::AP, NP = Cfg::NP, PPW = Cfg::PPW, STAGE = Cfg::STAGE;
  static_assert(WM * WN == BG_WAVES, "wave grid");
  static_assert(Cfg::SMEM <= 160 * 1024, "LDS");
  // ONE shared array (a second __shared__ object can de-pipeline LDS-DMA code)
  __shared__ __attribute__((aligned(16))) char smem[Cfg::SMEM];
  float* epi_sc = reinterpret_cast<float*>(smem + Cfg::EPI_OFF);
  float* epi_sh = epi_sc + BN;
  float* epi_mu = epi_sh + BN;
  float* epi_rs = epi_mu + BN;

  static_assert(!((EPI & EPI_ADD) && (EPI & (EPI_RELUMASK | EPI_BIASV))), "one preloaded epilogue operand");
  const ConvGeom& g = a.g;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  int tile = xcd_remap(blockIdx.x, gridDim.x);
  int n0 = 0;  // first output channel of the tile (WIN: Nc / BN column tiles, neighbours share rows)
  if (WIN) {
    const int ncol = g.Nc / BN;
    n0 = (tile % ncol) * BN;
    tile /= ncol;
  }
  const bool par = !WIN && igemm_parity(g);
  int p = 0, Tp = g.T_out, Mp = g.M;
  if (par) {
    const int nclip = g.M / (g.T_out * g.V), T0 = (g.T_out + 1) >> 1;
    const int tiles0 = (nclip * T0 * g.V + BM - 1) / BM;
    Tp = T0;
    if (tile >= tiles0) { p = 1; tile -= tiles0; Tp = g.T_out >> 1; }
    Mp = nclip * Tp * g.V;
  }
  auto phys = [&](int r) -> int {
    if (r >= Mp) return -1;
    if (!par) return r;
    const int nt = r / g.V, v = r - nt * g.V, n = nt / Tp, tt = nt - n * Tp;
    return (n * g.T_out + 2 * tt + p) * g.V + v;
  };
  const int m0 = tile * BM;
  constexpr int CB = X3N ? 32 : G_BK;                 // channels per k step
  const int Ktot = g.KT * g.Kc * (X3N ? 2 : 1);       // packed weight row length
  const int kpt = g.Kc / CB;
  const int dt0 = par ? ((p + g.P) & 1) : 0;
  const int ntap = par ? (g.KT - dt0 + 1) / 2 : g.KT;
  const int nchunk = ntap * kpt;
  // k step t -> (tap, channel chunk), tap-major (chunk-major order, all taps of a chunk back to back,
  // measured within 1 %: DESIGN.md §4.11)
  auto tapchunk = [&](int t, int& tap, int& i0) {
    tap = t / kpt;
    i0 = (t - tap * kpt) * CB;
  };
  // weight column of (tap dt, channel offset i0), A column of the lane's 16-B chunk cg
  auto wcol = [&](int dt, int i0) { return X3N ? dt * 2 * g.Kc + 2 * i0 : dt * g.Kc + i0; };
  auto acolx = [&](int i0, int cg) { return X3N ? x3n_col(g.Kc, i0, cg) : acol(a, i0) + cg * 8; };
  const unsigned short* in = a.inb;
  const unsigned short* wb = a.wb;

  if (EPI & EPI_RELUMASK) {
    for (int t = tid; t < BN; t += BG_THREADS) {
      float sc, sh, mu, rs;
      bn_coeff(a.epi_bn, n0 + t, sc, sh, mu, rs);
      epi_sc[t] = sc; epi_sh[t] = sh; epi_mu[t] = mu; epi_rs[t] = rs;
    }
  }

  // staging slots of this wave: piece q = (wave + 8 i) mod NP (A pieces, then B pieces); a
  // wrapped slot re-issues an earlier piece's identical copy (same bytes to the same LDS
  // address), so every wave issues PPW DMAs per stage and one vmcnt count serves all
  const int sub = lane >> 3, pch = lane & 7;
  RowMap amap[PPW];
  int boff[PPW];
#pragma unroll
  for (int i = 0; i < PPW; ++i) {
    if (WIN) break;
    const int q = (wave + BG_WAVES * i) % NP;
    amap[i].base = -1;
    amap[i].q = 0;
    boff[i] = 0;
    if (q < AP) {
      amap[i] = rowmap(phys(m0 + q * 8 + sub), g);
    } else {
      const int j = (q - AP) * 8 + sub;
      boff[i] = j * Ktot + swz(j, pch) * 8;
    }
  }
  auto stage = [&](int t, int buf) {
    int tap, i0;
    tapchunk(t, tap, i0);
    const int dt = par ? dt0 + 2 * tap : tap;
    const int k0 = wcol(dt, i0);
    char* sbase = smem + buf * STAGE;
#pragma unroll
    for (int i = 0; i < PPW; ++i) {
      const int q = (wave + BG_WAVES * i) % NP;
      const void* src;
      char* dst;
      if (q < AP) {
        const int r = rowmap_src(amap[i], dt, g);
        src = r >= 0 ? (const void*)(in + (size_t)r * g.lda + acolx(i0, swz(q * 8 + sub, pch))) : (const void*)a.zero;
        dst = sbase + q * 1024;
      } else {
        src = wb + boff[i] + k0;
        dst = sbase + q * 1024;
      }
      __builtin_amdgcn_global_load_lds(src, (lds_void_t*)dst, 16, 0, 0);
    }
  };

  const int wm = wave / WN, wn = wave % WN;
  const int fr = lane & 15, fg = lane >> 4;
  f32x4 acc[BG_MT][BG_NT];
#pragma unroll
  for (int x = 0; x < BG_MT; ++x)
#pragma unroll
    for (int y = 0; y < BG_NT; ++y) acc[x][y] = f32x4{0.f, 0.f, 0.f, 0.f};
  if constexpr (WIN) {
    // step u = (chunk c, tap dt), chunk-major: c = u / KT, dt = u % KT. Per step every wave
    // issues PPW DMAs: its B pieces of step u's weight stage, the 6 A pieces of chunk c + 1 that
    // step u carries (steps 2..7 of a chunk: the buffer they fill was last read in step c*KT - 1,
    // and a step is issued two steps ahead), and otherwise a re-issue of its first B piece.
    constexpr int KTW = 9;
    const int nstep = KTW * kpt;
    const int sgn = g.transposed ? -1 : 1;
    auto stage_w = [&](int u, int buf) {
      const int c = u / KTW, dt = u - c * KTW;
      const int k0 = wcol(dt, c * CB);
      char* sbase = smem + Cfg::SOFF + buf * STAGE;
      const void* src0 = wb + (size_t)(n0 + wave * 8 + sub) * Ktot + k0 + swz(wave * 8 + sub, pch) * 8;
#pragma unroll
      for (int i = 0; i < PPW; ++i) {
        const int q = wave + BG_WAVES * i;
        const void* src = src0;
        char* dst = sbase + wave * 1024;
        if (q < Cfg::BP) {
          src = wb + (size_t)(n0 + q * 8 + sub) * Ktot + k0 + swz(q * 8 + sub, pch) * 8;
          dst = sbase + q * 1024;
        } else if (q < NP && dt >= 2 && c + 1 < kpt) {
          const int pa = (dt - 2) * WIN_APS + (q - Cfg::BP);  // A piece of chunk c + 1
          if (pa < BM / 8) {
            src = in + (size_t)(m0 + pa * 8 + sub) * g.lda + acolx((c + 1) * CB, swz(pa * 8 + sub, pch));
            dst = smem + ((c + 1) & 1) * Cfg::AWIN + pa * 1024;
          }
        }
        __builtin_amdgcn_global_load_lds(src, (lds_void_t*)dst, 16, 0, 0);
      }
    };
    // chunk 0's A rows, then steps 0 and 1
    constexpr int A0W = (BM / 8 + BG_WAVES - 1) / BG_WAVES;
#pragma unroll
    for (int i = 0; i < A0W; ++i) {
      const int pa = (wave + BG_WAVES * i) % (BM / 8);
      // (the source computed outside the builtin's argument list: a lambda call inside it drops
      // the kernel's host stub without a diagnostic)
      const void* src = in + (size_t)(m0 + pa * 8 + sub) * g.lda + acolx(0, swz(pa * 8 + sub, pch));
      __builtin_amdgcn_global_load_lds(src, (lds_void_t*)(smem + pa * 1024), 16, 0, 0);
    }
    stage_w(0, 0);
    stage_w(1, 1);
    if (tid < 8) *reinterpret_cast<f32x4*>(smem + Cfg::ZOFF + tid * 16) = f32x4{0.f, 0.f, 0.f, 0.f};
    asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"n"(PPW) : "memory");
    __builtin_amdgcn_s_barrier();
    const int wrow = wm * 144;  // this wave's clip in the tile
    // fragment reads as inline asm: hipcc otherwise issues each ds_read_b128 just before the MFMA
    // that consumes it with its own lgkmcnt(0), exposing the LDS latency ~14 times per step. Both
    // k halves' 22 reads are issued at once; each half is released by a counted wait whose asm
    // also passes the fragments through (nothing can use them earlier). Out-of-clip tap rows read
    // a zero row instead of being masked.
    typedef unsigned u32x4_t __attribute__((ext_vector_type(4)));
    const unsigned lds0 = (unsigned)(size_t)(lds_cchar_t*)smem;
    const unsigned zaddr = lds0 + Cfg::ZOFF + fg * 16;
    for (int u = 0; u < nstep; ++u) {
      const int c = u / KTW, dt = u - c * KTW;
      const int sh = sgn * (dt - g.P) * g.V;  // row shift of this tap inside the clip
      if (u + 2 < nstep) stage_w(u + 2, (u + 2) % 3);
      const unsigned sa = lds0 + (c & 1) * Cfg::AWIN;
      const unsigned sb = lds0 + Cfg::SOFF + (u % 3) * STAGE;
      u32x4_t f[2][BG_NT + BG_MT];
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        const int cc = ks * 4 + fg;
#pragma unroll
        for (int y = 0; y < BG_NT; ++y) {
          const int r = wn * 32 + y * 16 + fr;
          asm volatile("ds_read_b128 %0, %1" : "=v"(f[ks][y]) : "v"(sb + r * 128 + swz(r, cc) * 16));
        }
#pragma unroll
        for (int x = 0; x < BG_MT; ++x) {
          const int rs = x * 16 + fr + sh, r = wrow + rs;
          const unsigned ad = (rs >= 0 && rs < 144) ? sa + r * 128 + swz(r, cc) * 16 : zaddr;
          asm volatile("ds_read_b128 %0, %1" : "=v"(f[ks][BG_NT + x]) : "v"(ad));
        }
      }
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        if (ks == 0) asm volatile("s_waitcnt lgkmcnt(%0)" ::"n"(BG_NT + BG_MT) : "memory");
        else asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
        for (int q = 0; q < BG_NT + BG_MT; ++q) asm volatile("" : "+v"(f[ks][q]));
#pragma unroll
        for (int x = 0; x < BG_MT; ++x)
#pragma unroll
          for (int y = 0; y < BG_NT; ++y) {
            // X3N: half 0 = the hi fragments (x_hi W_hi), half 1 = the lo ones (x_lo W_hi + x_hi W_lo)
            acc[x][y] = mfma_bf16x(__builtin_bit_cast(bf16x8, f[ks][BG_NT + x]),
                                   __builtin_bit_cast(bf16x8, f[X3N ? 0 : ks][y]), acc[x][y]);
            if (X3N && ks == 1)
              acc[x][y] = mfma_bf16x(__builtin_bit_cast(bf16x8, f[0][BG_NT + x]), __builtin_bit_cast(bf16x8, f[1][y]),
                                     acc[x][y]);
          }
        if (ks == 0) {  // pin the first half's MFMAs above the second wait (hipcc sinks them below it)
#pragma unroll
          for (int x = 0; x < BG_MT; ++x)
#pragma unroll
            for (int y = 0; y < BG_NT; ++y) asm volatile("" : "+v"(acc[x][y]));
        }
      }
      if (u + 2 < nstep) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(PPW) : "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
    }
  } else {
    if (nchunk == 0) {  // parity class without taps (1x1 stride-2 input gradient, odd rows)
      if (EPI & EPI_ADD) return;
      __syncthreads();
    } else {
      stage(0, 0);
      if (nchunk > 1) {
        stage(1, 1);
        asm volatile("s_waitcnt vmcnt(%0)" ::"n"(PPW) : "memory");
      } else {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      __builtin_amdgcn_s_barrier();
    }
    for (int t = 0; t < nchunk; ++t) {
      const int buf = t % 3;
      if (t + 2 < nchunk) stage(t + 2, (t + 2) % 3);
      const char* sa = smem + buf * STAGE;
      const char* sb = sa + AP * 1024;
      // (batched inline-asm fragment reads as in the WIN loop measured neutral here: DESIGN.md §4.6)
      if constexpr (X3N) {
        // the hi and lo fragments of the block (chunks fg and 4 + fg), three products
        bf16x8 fah[BG_MT], fal[BG_MT], fbh[BG_NT], fbl[BG_NT];
#pragma unroll
        for (int y = 0; y < BG_NT; ++y) {
          const int r = wn * 32 + y * 16 + fr;
          fbh[y] = *reinterpret_cast<const bf16x8*>(sb + r * 128 + swz(r, fg) * 16);
          fbl[y] = *reinterpret_cast<const bf16x8*>(sb + r * 128 + swz(r, 4 + fg) * 16);
        }
#pragma unroll
        for (int x = 0; x < BG_MT; ++x) {
          const int r = wm * 144 + x * 16 + fr;
          fah[x] = *reinterpret_cast<const bf16x8*>(sa + r * 128 + swz(r, fg) * 16);
          fal[x] = *reinterpret_cast<const bf16x8*>(sa + r * 128 + swz(r, 4 + fg) * 16);
        }
#pragma unroll
        for (int x = 0; x < BG_MT; ++x)
#pragma unroll
          for (int y = 0; y < BG_NT; ++y) {
            acc[x][y] = mfma_bf16x(fah[x], fbh[y], acc[x][y]);
            acc[x][y] = mfma_bf16x(fal[x], fbh[y], acc[x][y]);
            acc[x][y] = mfma_bf16x(fah[x], fbl[y], acc[x][y]);
          }
      } else {
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) {
          bf16x8 fa[BG_MT], fb[BG_NT];
          const int c = ks * 4 + fg;
#pragma unroll
          for (int y = 0; y < BG_NT; ++y) {
            const int r = wn * 32 + y * 16 + fr;
            fb[y] = *reinterpret_cast<const bf16x8*>(sb + r * 128 + swz(r, c) * 16);
          }
#pragma unroll
          for (int x = 0; x < BG_MT; ++x) {
            const int r = wm * 144 + x * 16 + fr;
            fa[x] = *reinterpret_cast<const bf16x8*>(sa + r * 128 + swz(r, c) * 16);
          }
#pragma unroll
          for (int x = 0; x < BG_MT; ++x)
#pragma unroll
            for (int y = 0; y < BG_NT; ++y) acc[x][y] = mfma_bf16x(fa[x], fb[y], acc[x][y]);
        }
      }
      if (t + 2 < nchunk) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(PPW) : "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
    }
  }
  __syncthreads();

  // ---------------- epilogue (as igemm_bf16) ----------------
  float* red = reinterpret_cast<float*>(smem);   // [WM][2][BN]  (stage 0 is free now)
  float* gred = red + 2 * WM * BN;               // [WM][2][BN]
  float ssum[BG_NT], ssq[BG_NT], gap0[BG_NT], gap1[BG_NT];
#pragma unroll
  for (int y = 0; y < BG_NT; ++y) ssum[y] = ssq[y] = gap0[y] = gap1[y] = 0.f;
  // bf16 outputs leave through an LDS image of the tile: the MFMA C layout gives a lane 4 rows of
  // ONE column (2-B scattered stores); the image is copied out as 16-B row chunks instead
  constexpr int OTS = BN + 8, OT_OFF = 16 * 1024;  // row stride (elements), byte offset past red/gred
  static_assert(OT_OFF + BM * OTS * 2 <= (int)sizeof(smem), "output staging tile");
  const bool stage_out = !(EPI & EPI_ADD) && a.outb && g.ldo % 8 == 0 && g.Nc % 8 == 0;
  __bf16* ot = reinterpret_cast<__bf16*>(smem + OT_OFF);
  const int TV = g.T_out * g.V;
  const int nlo = m0 / TV;  // GAP is forward-only (no parity split): m0 is the first output row
  // Per 16-row group x: the group's 4 output rows are resolved and every operand the epilogue
  // reads (RELUMASK source g, graph-mixed bias) is loaded for all 4 rows x BG_NT columns before
  // any use, from clamped in-bounds addresses. A per-element conditional load (row outside the
  // parity class, column past Nc, or the fp32/bf16 select) made hipcc wait vmcnt(0) on every
  // element: 72 dependent round trips per lane in the RELUMASK epilogue.
  const bool aux16 = a.auxb != nullptr;
  float biasj[BG_NT];  // EPI_BIAS: one value per column, loaded once
#pragma unroll
  for (int y = 0; y < BG_NT; ++y) biasj[y] = (EPI & EPI_BIAS) ? a.bias[min(n0 + wn * 32 + y * 16 + fr, g.Nc - 1)] : 0.f;
  // all groups' operands first: a load issued after the group's stores would make its first
  // use wait (vmcnt counts stores too) for every store before it
  float pre[BG_MT][4][BG_NT];
  auto preload = [&](auto load) {
#pragma unroll
    for (int x = 0; x < BG_MT; ++x)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int mc = max(phys(m0 + wm * 144 + x * 16 + fg * 4 + r), 0);
#pragma unroll
        for (int y = 0; y < BG_NT; ++y) pre[x][r][y] = load(mc, min(n0 + wn * 32 + y * 16 + fr, g.Nc - 1));
      }
  };
  if (EPI & EPI_RELUMASK) {
    if (aux16) preload([&](int mc, int jc) { return bf2f(a.auxb[(size_t)mc * a.ldaux + jc]); });
    else preload([&](int mc, int jc) { return a.aux[(size_t)mc * a.ldaux + jc]; });
  } else if (EPI & EPI_BIASV) {
    preload([&](int mc, int jc) { return a.bias[(mc % g.V) * g.Nc + jc]; });
  } else if (EPI & EPI_ADD) {
    preload([&](int mc, int jc) { return a.out[(size_t)mc * g.ldo + jc]; });
  }
#pragma unroll
  for (int x = 0; x < BG_MT; ++x) {
    int mrow[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) mrow[r] = phys(m0 + wm * 144 + x * 16 + fg * 4 + r);
#pragma unroll
    for (int y = 0; y < BG_NT; ++y) {
      const int jl = wn * 32 + y * 16 + fr, j = n0 + jl;  // tile-local / global column
      const bool jok = j < g.Nc;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = mrow[r];
        if (!jok || m < 0) continue;
        float v = acc[x][y][r];
        if (EPI & EPI_BIAS) v += biasj[y];
        if (EPI & EPI_BIASV) v += pre[x][r][y];
        if (EPI & EPI_RELUMASK) {
          const float gv = pre[x][r][y];
          if (gv * epi_sc[jl] + epi_sh[jl] <= 0.f) v = 0.f;
          const float xh = (gv - epi_mu[jl]) * epi_rs[jl];
          ssum[y] += v;
          ssq[y] += v * xh;
        } else if (EPI & EPI_STATS) {
          ssum[y] += v;
          ssq[y] += v * v;
        }
        if (EPI & EPI_GAP) {
          const int n = m / TV;
          if (n == nlo) gap0[y] += v;
          else if (n == nlo + 1) gap1[y] += v;
          else atomic_add_f(a.gap + (size_t)n * g.Nc + j, v);
        }
        if (!(EPI & EPI_ADD) && a.outb) {
          if (stage_out) ot[(wm * 144 + x * 16 + fg * 4 + r) * OTS + jl] = (__bf16)v;
          else reinterpret_cast<__bf16*>(a.outb)[(size_t)m * g.ldo + j] = (__bf16)v;
        } else {
          float* o = a.out + (size_t)m * g.ldo + j;
          if (EPI & EPI_ADD) *o = pre[x][r][y] + v;
          else *o = v;
        }
      }
    }
  }
  if (EPI & (EPI_STATS | EPI_RELUMASK | EPI_GAP)) {
#pragma unroll
    for (int y = 0; y < BG_NT; ++y) {
#pragma unroll
      for (int o = 16; o < 64; o <<= 1) {
        ssum[y] += __shfl_xor(ssum[y], o, 64);
        ssq[y] += __shfl_xor(ssq[y], o, 64);
        gap0[y] += __shfl_xor(gap0[y], o, 64);
        gap1[y] += __shfl_xor(gap1[y], o, 64);
      }
    }
    if (fg == 0) {
#pragma unroll
      for (int y = 0; y < BG_NT; ++y) {
        const int jl = wn * 32 + y * 16 + fr;
        red[(wm * 2 + 0) * BN + jl] = ssum[y];
        red[(wm * 2 + 1) * BN + jl] = ssq[y];
        gred[(wm * 2 + 0) * BN + jl] = gap0[y];
        gred[(wm * 2 + 1) * BN + jl] = gap1[y];
      }
    }
    __syncthreads();
    for (int t = tid; t < BN; t += BG_THREADS) {
      if (n0 + t >= g.Nc) continue;
      float s0 = 0.f, s1 = 0.f, g0 = 0.f, g1 = 0.f;
#pragma unroll
      for (int w = 0; w < WM; ++w) {
        s0 += red[(w * 2 + 0) * BN + t];
        s1 += red[(w * 2 + 1) * BN + t];
        g0 += gred[(w * 2 + 0) * BN + t];
        g1 += gred[(w * 2 + 1) * BN + t];
      }
      if (EPI & (EPI_STATS | EPI_RELUMASK)) {
        atomic_add_d(a.st_sum + n0 + t, (double)s0);
        atomic_add_d(a.st_sq + n0 + t, (double)s1);
      }
      if (EPI & EPI_GAP) {
        atomic_add_f(a.gap + (size_t)nlo * g.Nc + n0 + t, g0);
        if ((nlo + 1) * TV < g.M && g1 != 0.f) atomic_add_f(a.gap + (size_t)(nlo + 1) * g.Nc + n0 + t, g1);
      }
    }
  }
  if (stage_out) {
    __syncthreads();
    constexpr int CPR = BN / 8;  // 16-B chunks per tile row
    for (int q = tid; q < BM * CPR; q += blockDim.x) {
      const int rl = q / CPR, c = q - rl * CPR;
      const int m = phys(m0 + rl), j = n0 + c * 8;
      if (m < 0 || j >= g.Nc) continue;
      *reinterpret_cast<uint4*>(reinterpret_cast<__bf16*>(a.outb) + (size_t)m * g.ldo + j) =
          *reinterpret_cast<const uint4*>(ot + rl * OTS + c * 8);
    }
  }
}

}  // namespace f3

using namespace f3;

// Large tiles pay when the k loop is long enough to amortise the 3-stage prologue.
bool f3_igemm_big_ok(const ConvGemmArgs& a) {
  if (!f3_igemm_ok(a)) return false;
  if (a.g.Nc != 128 && a.g.Nc != 256) return false;
  return a.g.KT * a.g.Kc / (a.x3n ? 32 : G_BK) >= 6;
}

template <int WM, int WN, bool X3N>
static int launch_big(const ConvGemmArgs& a, int epi, hipStream_t s) {
  constexpr int BM = BigCfg<WM, WN>::BM;
  int tiles = (a.g.M + BM - 1) / BM;
  if (igemm_parity(a.g)) {
    if (a.g.M % (a.g.T_out * a.g.V) != 0 || (epi & (EPI_GAP | EPI_BIASV))) return F3_EINVAL;
    const int nclip = a.g.M / (a.g.T_out * a.g.V);
    const int M0 = nclip * ((a.g.T_out + 1) >> 1) * a.g.V, M1 = nclip * (a.g.T_out >> 1) * a.g.V;
    tiles = (M0 + BM - 1) / BM + (M1 + BM - 1) / BM;
  }
#define F3_BCASE(E)                                                                              \
  if (epi == (E)) {                                                                             \
    hipLaunchKernelGGL((igemm_big<(E), WM, WN, false, X3N>), dim3(tiles), dim3(BG_THREADS), 0, s, a); \
    F3_LAUNCH_CHECK();                                                                           \
    return F3_OK;                                                                                \
  }
  F3_BCASE(EPI_BIASV | EPI_STATS)            // gcn forward
  F3_BCASE(EPI_BIAS | EPI_STATS | EPI_GAP)   // tcn forward
  F3_BCASE(EPI_BIAS | EPI_STATS)             // residual forward
  F3_BCASE(EPI_RELUMASK)                     // tcn dgrad
  F3_BCASE(0)                                // gcn dgrad
  F3_BCASE(EPI_ADD)                          // residual dgrad
  F3_BCASE(EPI_BIAS)                         // plain conv (tests)
#undef F3_BCASE
  return F3_EINVAL;
}

// Clip-window form (WIN): stride-1 9-tap temporal convs (forward or input gradient) of the
// 256-channel layers at T = 8, where a clip is exactly one wave's 144 rows.
static bool big_win_ok(const ConvGemmArgs& a) {
  const ConvGeom& g = a.g;
  const int cb = a.x3n ? 32 : G_BK;
  return g.Nc % 128 == 0 && g.S == 1 && g.KT == 9 && 2 * g.P == g.KT - 1 && g.T_in == g.T_out &&
         g.T_out * g.V == 144 && g.M % 288 == 0 && g.Kc % cb == 0 && g.Kc / cb >= 2 && !igemm_parity(g);
}

// (a plain function: hipcc left the device stubs of the WIN instances undefined when they were
// launched from a function template)
static int launch_win(const ConvGemmArgs& a, int epi, hipStream_t s) {
  const int tiles = (a.g.M / 288) * (a.g.Nc / 128);
#define F3_WCASE(E)                                                                                   \
  if (epi == (E)) {                                                                                  \
    if (a.x3n) hipLaunchKernelGGL((igemm_big<(E), 2, 4, true, true>), dim3(tiles), dim3(BG_THREADS), 0, s, a); \
    else hipLaunchKernelGGL((igemm_big<(E), 2, 4, true, false>), dim3(tiles), dim3(BG_THREADS), 0, s, a);     \
    F3_LAUNCH_CHECK();                                                                                \
    return F3_OK;                                                                                     \
  }
  F3_WCASE(EPI_BIAS | EPI_STATS | EPI_GAP)   // tcn forward
  F3_WCASE(EPI_RELUMASK)                     // tcn dgrad
  F3_WCASE(EPI_BIAS)                         // plain conv (tests)
  F3_WCASE(0)                                // plain input gradient (tests)
#undef F3_WCASE
  return F3_EINVAL;
}

int f3_igemm_big(const ConvGemmArgs* args, int epi, hipStream_t s) {
  const ConvGemmArgs& a = *args;
  if (a.g.M <= 0) return F3_OK;
  if (!f3_igemm_big_ok(a)) return F3_EINVAL;
  if (big_win_ok(a)) {
    const int r = launch_win(a, epi, s);
    if (r != F3_EINVAL) return r;
  }
  if (a.g.Nc == 256) return a.x3n ? launch_big<1, 8, true>(a, epi, s) : launch_big<1, 8, false>(a, epi, s);
  return a.x3n ? launch_big<2, 4, true>(a, epi, s) : launch_big<2, 4, false>(a, epi, s);
}
