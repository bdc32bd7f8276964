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

#include <type_traits>

// F3_PROBE (tools/probe_build.sh only; 0 in the library): bit 1 drops the window loop's MFMAs, bit 2
// its weight / A-carry DMAs, bit 4 its LDS fragment reads — the bound each leg sets alone; bit 8 drops
// igemm_win1's per-step s_barrier, bit 16 its epilogue (timing only, results wrong; bits 1, 2, 4 apply
// to igemm_win1 too). (A static
// issue priority for waves 4-7, MI355X_MICROARCH.md "two waves per SIMD" item 4, measured within
// noise on l1d / l5d / l8d / l8f: profiles/r05_window_prio_ab.txt.) (Measured
// on l8d with this loop: 126 us full, 77 without MFMA, 55 without MFMA and DMA: the legs add up almost
// linearly. A software-pipelined loop (next step's hi fragments read under the current step's lo
// products) and a ping-pong of the SIMD partner waves (one loads while the other multiplies) were
// both 2-5 % SLOWER: the loading leg is instruction-issue bound, not latency bound.)
#ifndef F3_TILE_BATCH
#define F3_TILE_BATCH 1  // batched fragment reads in the tiled X3N loop (0: the hipcc-scheduled reads, A/B)
#endif
#ifndef F3_PROBE
#define F3_PROBE 0
#endif

namespace f3 {

constexpr int BG_MT = 9, BG_NT = 2, BG_NST = 3;  // per-wave MFMA tiles (rows x cols), LDS stages
constexpr int BG_WAVES = 8, BG_THREADS = 64 * BG_WAVES;

// (Loading the weight fragments straight from global memory into registers, so the LDS stages carry
// the A rows only, measured slower: 67 -> 87 us on the layer-6 forward)
// WIN (clip window, WIN = the clip rows of the layout): for 9-tap temporal convs a workgroup owns
// whole clips x BN = 128 output channels — two 144-row clips (WIN = 144, one per wave row: the
// 256-channel layers at T = 8) or one clip of up to 270 rows (WIN = 270: the 128-channel layers at
// T = 15). Per channel chunk the clips' input rows (the "window", 288 rows x 128 B) are staged ONCE
// and every tap reads them shifted by its frame offset, rows outside the clip reading a zero row;
// only the weights are staged per (chunk, tap) step (16 KiB). Three row maps share the engine:
//   stride 1 (fwd or input gradient): one window per chunk, tap dt shifts by +-(dt - P) frames;
//   stride-2 input gradient: a tile is one output-frame parity p of its clips; the window is the
//     clips' dY frames and only the taps dt = p + P (mod 2) contribute, shifted by (p + P - dt) / 2;
//   stride-2 forward: two windows per chunk, the even and the odd input frames; window q serves
//     the taps dt = P + q (mod 2), shifted by (dt - P - q) / 2.
// Per workgroup and chunk that is 36 KiB of A fill plus 16 KiB per tap instead of 52 KiB per tap.
// WIN = 540 (the 64-channel layers at T = 30): one clip of up to 540 rows x BN = 64 per workgroup
// (4 x 2 waves); the two channel chunks' windows (69 KiB each) leave room for two weight stages
// only, so steps are issued one ahead instead of two.
typedef __attribute__((address_space(3))) const char lds_cchar_t;
template <int WM, int WN, int WIN = 0>
struct BigCfg {
  static constexpr int BM = 16 * BG_MT * WM, BN = 16 * BG_NT * WN;
  static constexpr int NW = WM * WN;                                // waves
  // WIN: clips per workgroup (WIN = 144 with 4 waves: one clip x 128 channels, two workgroups per CU)
  static constexpr int CPW = WIN == 144 && WM == 2 ? 2 : 1;
  static constexpr int NPA = (CPW * WIN + 7) / 8;                // WIN: A pieces per window
  static constexpr int NST = (WIN == 540 || (WIN == 144 && WM == 1)) ? 2 : BG_NST, LA = NST - 1;  // weight stages, issued ahead
  // 1-KiB pieces per stage: A then B (WIN: slots for the next window's carried A pieces, <= 12 used
  // at two steps ahead, <= 8 at one)
  static constexpr int AP = WIN ? (WIN == 540 || WM == 1 ? 8 : 16) : BM / 8, BP = BN / 8, NP = AP + BP;
  static constexpr int PPW = (NP + NW - 1) / NW;                          // pieces per wave
  static constexpr int STAGE = WIN ? BN * 128 : NP * 1024;
  static constexpr int AWIN = NPA * 1024;            // one A window buffer (WIN: two of them)
  static constexpr int SOFF = 2 * AWIN;              // byte offset of the per-step stages
  // the epilogue's output image (16 KiB + BM x (BN + 8) bf16) reuses the stages' bytes
  static constexpr int OT_NEED = 16 * 1024 + BM * (BN + 8) * 2;
  static constexpr int EPI_OFF = SOFF + NST * STAGE > OT_NEED ? SOFF + NST * STAGE : OT_NEED;
  static constexpr int ZOFF = EPI_OFF + 4 * BN * 4;  // WIN: one zero row, read for out-of-clip taps
  static constexpr int DOFF = ZOFF + 128;            // WIN: 1-KiB sink of the idle DMA slots
  static constexpr int SMEM = WIN ? DOFF + 1024 : ZOFF;
};

// The epilogue of igemm_big and igemm_win1 (as igemm_bf16): bias / graph-mixed bias, BN statistics,
// channel-attention GAP, ReLU mask + BN-backward sums, accumulate; bf16 outputs through an LDS image.
// WIN: rows are clip-window rows (clip0, wmode / wpar as the kernels'); else phys(m0 + tile row).
template <int EPI, int WM, int WN, int WIN, class Phys>
F3_DEV __attribute__((always_inline)) void big_epilogue(const ConvGemmArgs& a, f32x4 (&acc)[BG_MT][BG_NT], char* smem,
                                                        int n0, int clip0, int nclip, int wmode, int wpar, int m0,
                                                        Phys phys) {
  using Cfg = BigCfg<WM, WN, WIN>;
  constexpr int NT = 64 * WM * WN, BM = Cfg::BM, BN = Cfg::BN, CPW = Cfg::CPW;
  const ConvGeom& g = a.g;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WN, wn = wave % WN;
  const int fr = lane & 15, fg = lane >> 4;
  float* epi_sc = reinterpret_cast<float*>(smem + Cfg::EPI_OFF);
  float* epi_sh = epi_sc + BN;
  float* epi_mu = epi_sh + BN;
  float* epi_rs = epi_mu + BN;
  // ---------------- epilogue (as igemm_bf16) ----------------
  float* red = reinterpret_cast<float*>(smem);   // [WM][2][BN]  (stage 0 is free now)
  float* gred = red + 2 * WM * BN;               // [WM][2][BN]
  float ssum[BG_NT], ssq[BG_NT], gap0[BG_NT], gap1[BG_NT];
#pragma unroll
  for (int y = 0; y < BG_NT; ++y) ssum[y] = ssq[y] = gap0[y] = gap1[y] = 0.f;
  // bf16 outputs leave through an LDS image of the tile: the MFMA C layout gives a lane 4 rows of
  // ONE column (2-B scattered stores); the image is copied out as 16-B row chunks instead
  constexpr int OTS = BN + 8, OT_OFF = 16 * 1024;  // row stride (elements), byte offset past red/gred
  static_assert(OT_OFF + BM * OTS * 2 <= Cfg::SMEM, "output staging tile");
  const bool stage_out = !(EPI & EPI_ADD) && a.outb && g.ldo % 8 == 0 && g.Nc % 8 == 0;
  __bf16* ot = reinterpret_cast<__bf16*>(smem + OT_OFF);
  const int TV = g.T_out * g.V;
  const int nlo = WIN ? clip0 : m0 / TV;  // first clip (GAP is forward-only: no parity split)
  // output row of tile row rl (-1: none)
  auto orow = [&](int rl) -> int {
    if constexpr (WIN != 0) {
      const int k = (CPW == 2 && rl >= WIN) ? 1 : 0, lo = rl - k * WIN, clip = clip0 + k;
      const int f = lo / g.V, v = lo - f * g.V, t = wmode == 1 ? 2 * f + wpar : f;
      if (lo >= WIN || t >= g.T_out || clip >= nclip) return -1;
      return (clip * g.T_out + t) * g.V + v;
    } else {
      return phys(m0 + rl);
    }
  };
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
        const int mc = max(orow(wm * 144 + x * 16 + fg * 4 + r), 0);
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
    for (int r = 0; r < 4; ++r) mrow[r] = orow(wm * 144 + x * 16 + fg * 4 + r);
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
    for (int t = tid; t < BN; t += NT) {
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
      const int m = orow(rl), j = n0 + c * 8;
      if (m < 0 || j >= g.Nc) continue;
      *reinterpret_cast<uint4*>(reinterpret_cast<__bf16*>(a.outb) + (size_t)m * g.ldo + j) =
          *reinterpret_cast<const uint4*>(ot + rl * OTS + c * 8);
    }
  }
}

// X3N: the bf16x3 native form (ConvGemmArgs::x3n): a k step is one 32-channel block, its staged row
// piece [x_hi 32 | x_lo 32] / [W_hi 32 | W_lo 32], and the wave issues x_hi W_hi + x_lo W_hi + x_hi W_lo
// K1 (tiled form, 1x1 convolutions: the gcn / residual GEMMs): every staging slot's source row is fixed
// for the launch and its column advances by one channel block per k step, so the slots' source pointers
// are computed once and a step adds a constant (the generic staging re-derives the tap, the row map and
// the column per slot and step: ~470 non-MFMA instructions per 54 MFMAs)
template <int EPI, int WM, int WN, int WIN = 0, bool X3N = false, bool K1 = false>
__global__ __launch_bounds__(64 * WM * WN) void igemm_big(ConvGemmArgs a) {
  using Cfg = BigCfg<WM, WN, WIN>;
  constexpr int NW = WM * WN, NT = 64 * NW;  // waves, threads
  static_assert(WIN == 0 || ((WIN == 144 || WIN == 270) && WM == 2 && WN == 4) || (WIN == 540 && WM == 4 && WN == 2) ||
                    (WIN == 144 && WM == 1 && WN == 4),
                "WIN layout");
  static_assert(BG_MT * 16 == 144, "a wave owns 144 rows");
  constexpr int BM = Cfg::BM, BN = Cfg::BN, AP = Cfg::AP, NP = Cfg::NP, PPW = Cfg::PPW, STAGE = Cfg::STAGE;
  static_assert(NW == BG_WAVES || (WIN == 144 && NW == 4), "wave grid");
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
  // WIN: first output channel (Nc / BN column tiles, neighbours share rows), output-frame parity of a
  // stride-2 input gradient, first clip; the row map (0 stride 1, 1 stride-2 dgrad, 2 stride-2 fwd)
  constexpr int CPW = Cfg::CPW, LA = Cfg::LA;  // clips per workgroup, steps issued ahead
  int n0 = 0, wpar = 0, clip0 = 0;
  const int wmode = g.S == 1 ? 0 : (g.transposed ? 1 : 2);
  const int nclip = WIN ? g.M / (g.T_out * g.V) : 0;
  if (WIN) {
    const int ncol = g.Nc / BN;
    n0 = (tile % ncol) * BN;
    tile /= ncol;
    if (wmode == 1) { wpar = tile & 1; tile >>= 1; }
    clip0 = tile * CPW;
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
  auto acolx = [&](int i0, int cg) { return X3N ? x3n_col(g.Kc, i0, cg) : i0 + cg * 8; };
  const unsigned short* in = a.inb;
  const unsigned short* wb = a.wb;

  if (EPI & EPI_RELUMASK) {
    for (int t = tid; t < BN; t += NT) {
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
  // K1: per slot the source of k step 0 and the element step per k step (0 for a zero row)
  const unsigned short* k1src[K1 ? PPW : 1];
  int k1step[K1 ? PPW : 1];
  if constexpr (K1) {
#pragma unroll
    for (int i = 0; i < PPW; ++i) {
      const int q = (wave + BG_WAVES * i) % NP;
      if (q < AP) {
        const int r = rowmap_src(amap[i], dt0, g);
        k1src[i] = r >= 0 ? in + (size_t)r * g.lda + acolx(0, swz(q * 8 + sub, pch)) : a.zero;
        k1step[i] = r >= 0 ? CB : 0;
      } else {
        k1src[i] = wb + boff[i] + wcol(dt0, 0);
        k1step[i] = X3N ? 2 * CB : CB;
      }
    }
  }
  auto stage = [&](int t, int buf) {
    if constexpr (K1) {
      char* sb = smem + buf * STAGE;
#pragma unroll
      for (int i = 0; i < PPW; ++i) {
        const int q = (wave + BG_WAVES * i) % NP;
        const void* src = k1src[i] + t * k1step[i];
        __builtin_amdgcn_global_load_lds(src, (lds_void_t*)(sb + q * 1024), 16, 0, 0);
      }
      return;
    }
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
  if constexpr (WIN != 0) {
    constexpr int CL = WIN, NPA = Cfg::NPA;  // window rows per clip, A pieces per window
    static_assert(Cfg::BP % NW == 0 && PPW * NW == Cfg::NP, "slots: B pieces, then A pieces");
    const int V = g.V, P = g.P, TVin = g.T_in * V;
    // taps of window q (q = input-frame parity for the stride-2 forward, else 0): dt = d0 + ds j,
    // j < nt, frame shift s0 + ss j. (Pairs of scalars, not arrays: a runtime-indexed private array
    // is promoted to LDS and costs a ds_read + wait per use.)
    int d00 = 0, d01 = 0, nt0 = g.KT, nt1 = 1, s00 = 0, s01 = 0, ds = 1, ss = 1;
    if (wmode == 0) {
      ss = g.transposed ? -1 : 1; s00 = -ss * P;
    } else {
      ds = 2;
      d00 = ((wmode == 1 ? wpar : 0) + P) & 1;
      d01 = (1 + P) & 1;
      nt0 = (g.KT - d00 + 1) >> 1;
      nt1 = (g.KT - d01 + 1) >> 1;
      ss = wmode == 1 ? -1 : 1;
      s00 = wmode == 1 ? (wpar + P - d00) >> 1 : (d00 - P) >> 1;
      s01 = (d01 - P - 1) >> 1;
    }
    const int NQ = wmode == 2 ? 2 : 1;  // windows per chunk
    const int nstep = (wmode == 2 ? g.KT : nt0) * kpt;
    // per window parity: A pieces per carrying step (nt - LA + 1 steps carry a window), valid rows
    const int ncar0 = nt0 - LA + 1, ncar1 = max(nt1 - LA + 1, 1);
    const int aps0 = (NPA + ncar0 - 1) / ncar0, aps1 = (NPA + ncar1 - 1) / ncar1;
    const int wlim0 = (NQ == 2 ? (g.T_in + 1) >> 1 : g.T_in) * V, wlim1 = (g.T_in >> 1) * V;
    const unsigned minv = (65536u + V - 1) / V;  // l / V as (l * minv) >> 16 (l < 2^9, V < 2^7)
    auto ntq = [&](int q) { return q ? nt1 : nt0; };
    // (chunk c, window q, tap j) of a step, advanced without divisions
    auto advance = [&](int& c, int& q, int& j) {
      if (++j == ntq(q)) {
        j = 0;
        if (NQ == 2 && q == 0) { q = 1; } else { q = 0; ++c; }
      }
    };
    // source of A piece pa (8 window rows) of window (c, q): clip row l of clip clip0 + k
    auto asrc = [&](int c, int q, int pa) -> const void* {
      const int R = pa * 8 + sub, k = (CPW == 2 && R >= CL) ? 1 : 0, l = R - k * CL, clip = clip0 + k;
      if (l >= (q ? wlim1 : wlim0) || clip >= nclip) return a.zero;
      int row = clip * TVin + l;
      if (NQ == 2) row += (int)(((unsigned)l * minv) >> 16) * V + q * V;  // input frame 2 f + q
      return in + (size_t)row * g.lda + acolx(c * CB, swz(R, pch));
    };
    // the lane's B piece offsets (slots i < BP / 8; the A slots follow)
    size_t boffw[Cfg::BP / NW];
#pragma unroll
    for (int i = 0; i < Cfg::BP / NW; ++i) {
      const int r = (wave + NW * i) * 8 + sub;
      boffw[i] = (size_t)(n0 + r) * Ktot + swz(r, pch) * 8;
    }
    // Per step every wave issues PPW DMAs: its B pieces of the step's weight stage, then A pieces of
    // the next window — step j >= LA of window w carries window w + 1's, step 0 of window w the last
    // group of its own (the buffer a window fills was last read by window w - 1, and a step is issued
    // LA steps ahead: steps LA .. nt(w) of window w's range are the ones that can) — and a sink DMA
    // of the zero row in slots left idle.
    auto stage_w = [&](int c, int q, int j, int buf) {
      const int k0 = wcol((q ? d01 : d00) + ds * j, c * CB);
      char* sbase = smem + Cfg::SOFF + buf * STAGE;
      bool car = false;
      int tc = c, tq = q, kk = 0, na = 0;
      if (j >= LA) {
        car = true; kk = j - LA; na = q ? aps1 : aps0;
        if (NQ == 2 && q == 0) tq = 1; else { tq = 0; tc = c + 1; }
      } else if (j == 0 && (c > 0 || q > 0)) {
        const int qp = NQ == 2 ? 1 - q : 0;
        car = true; kk = ntq(qp) - LA; na = qp ? aps1 : aps0;
      }
      car = car && tc < kpt;
      char* wdst = smem + ((tc * NQ + tq) & 1) * Cfg::AWIN;
#pragma unroll
      for (int i = 0; i < PPW; ++i) {
        const void* src;
        char* dst;
        if (i < Cfg::BP / NW) {
          src = wb + boffw[i] + k0;
          dst = sbase + (wave + NW * i) * 1024;
        } else {
          const int sl = wave + NW * i - Cfg::BP, pa = kk * na + sl;
          src = a.zero;
          dst = smem + Cfg::DOFF;
          if (car && sl < na && pa < NPA) {
            src = asrc(tc, tq, pa);
            dst = wdst + pa * 1024;
          }
        }
        __builtin_amdgcn_global_load_lds(src, (lds_void_t*)dst, 16, 0, 0);
      }
    };
    // window 0's A rows, then steps 0 and 1
    constexpr int A0W = (NPA + NW - 1) / NW;
#pragma unroll
    for (int i = 0; i < A0W; ++i) {
      const int pa = (wave + NW * i) % NPA;
      const void* src = asrc(0, 0, pa);
      __builtin_amdgcn_global_load_lds(src, (lds_void_t*)(smem + pa * 1024), 16, 0, 0);
    }
    int sc = 0, sq = 0, sj = 0;  // the step staged next
    stage_w(sc, sq, sj, 0);
    advance(sc, sq, sj);
    if (LA == 2 && nstep > 1) {
      stage_w(sc, sq, sj, 1);
      advance(sc, sq, sj);
    }
    if (tid < 8) *reinterpret_cast<f32x4*>(smem + Cfg::ZOFF + tid * 16) = f32x4{0.f, 0.f, 0.f, 0.f};
    if (LA == 2 && nstep > 1) asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"n"(PPW) : "memory");
    else asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    // the wave's rows: clip base row in the window and first output row of the clip
    const int cbase = CPW == 2 ? wm * 144 : 0, lo0 = CPW == 2 ? 0 : wm * 144;
    // fragment reads as inline asm: hipcc otherwise issues each ds_read_b128 just before the MFMA
    // that consumes it with its own lgkmcnt(0), exposing the LDS latency ~14 times per step. Both
    // k halves' 22 reads are issued at once; each half is released by a counted wait whose asm
    // also passes the fragments through (nothing can use them earlier). A fragment rows: the
    // lane's row of tile x is t + 16 x (t = first row + tap shift); swz(r, c) = c ^ (r & 7) is the
    // same for every x, so one base per k half plus an immediate 2 KiB x stride addresses them all,
    // and a row outside the clip reads the zero row (its address minus that stride).
    typedef unsigned u32x4_t __attribute__((ext_vector_type(4)));
    const unsigned lds0 = (unsigned)(size_t)(lds_cchar_t*)smem;
    const unsigned zrow = lds0 + Cfg::ZOFF;
    unsigned boffr[2][BG_NT];
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int y = 0; y < BG_NT; ++y) {
        const int r = wn * 32 + y * 16 + fr;
        boffr[ks][y] = lds0 + Cfg::SOFF + r * 128 + swz(r, ks * 4 + fg) * 16;
      }
    int c = 0, q = 0, j = 0;  // the step computed
    for (int u = 0; u < nstep; ++u) {
      const int t = lo0 + fr + ((q ? s01 : s00) + ss * j) * V;  // lane's tile-0 row in the clip, tap-shifted
      if (u + LA < nstep) {
        if (!(F3_PROBE & 2)) stage_w(sc, sq, sj, (u + LA) % Cfg::NST);
        advance(sc, sq, sj);
      }
      const unsigned rb = lds0 + ((c * NQ + q) & 1) * Cfg::AWIN + (unsigned)(cbase + t) * 128;
      const unsigned ab0 = rb + ((fg ^ (t & 7)) << 4), ab1 = rb + (((4 + fg) ^ (t & 7)) << 4);
      const unsigned soff = (u % Cfg::NST) * STAGE;
      u32x4_t f[2][BG_NT + BG_MT];
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
#pragma unroll
        for (int y = 0; y < BG_NT; ++y) {
          if (F3_PROBE & 4) { f[ks][y] = u32x4_t{0u, 0u, 0u, 0u}; continue; }
          asm volatile("ds_read_b128 %0, %1" : "=v"(f[ks][y]) : "v"(boffr[ks][y] + soff));
        }
        static_assert(BG_MT == 9, "F3_AREAD list");
#define F3_AREAD(X)                                                                                        \
  if (F3_PROBE & 4) f[ks][BG_NT + (X)] = u32x4_t{0u, 0u, 0u, 0u};                                         \
  else {                                                                                                   \
    const unsigned ad = (unsigned)(t + 16 * (X)) < (unsigned)CL ? (ks ? ab1 : ab0) : zrow - 2048u * (X);  \
    asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(f[ks][BG_NT + (X)]) : "v"(ad), "n"(2048 * (X))); \
  }
        F3_AREAD(0) F3_AREAD(1) F3_AREAD(2) F3_AREAD(3) F3_AREAD(4) F3_AREAD(5) F3_AREAD(6) F3_AREAD(7) F3_AREAD(8)
#undef F3_AREAD
      }
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        if (ks == 0) asm volatile("s_waitcnt lgkmcnt(%0)" ::"n"(BG_NT + BG_MT) : "memory");
        else asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
        for (int qq = 0; qq < BG_NT + BG_MT; ++qq) asm volatile("" : "+v"(f[ks][qq]));
#pragma unroll
        for (int x = 0; x < BG_MT; ++x)
#pragma unroll
          for (int y = 0; y < BG_NT; ++y) {
            if (F3_PROBE & 1) {  // probe build: fragments consumed, no MFMA
              asm volatile("" : "+v"(acc[x][y]) : "v"(f[ks][BG_NT + x]), "v"(f[ks][y]));
              continue;
            }
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
      if (LA == 2 && u + 2 < nstep) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(PPW) : "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      advance(c, q, j);
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
      // X3N: the 22 fragment reads of a step issued at once (inline asm, immediate row offsets: a
      // fragment's rows keep r & 7 over the 16-row tiles, so one swizzled base serves all), the hi
      // half's products under a counted wait, as the WIN loop. (In the round-2 bf16 form the batched
      // reads measured neutral here)
      if constexpr (X3N && F3_TILE_BATCH) {
        static_assert(BG_NT == 2 && BG_MT == 9, "batched tile reads");
        typedef unsigned u32x4_t __attribute__((ext_vector_type(4)));
        const unsigned l0 = (unsigned)(size_t)(lds_cchar_t*)smem + buf * STAGE;
        const int ra = wm * 144 + fr, rw = wn * 32 + fr;
        const unsigned ah[2] = {l0 + ra * 128 + swz(ra, fg) * 16, l0 + ra * 128 + swz(ra, 4 + fg) * 16};
        const unsigned bh[2] = {l0 + AP * 1024 + rw * 128 + swz(rw, fg) * 16,
                                l0 + AP * 1024 + rw * 128 + swz(rw, 4 + fg) * 16};
        u32x4_t f[2][BG_NT + BG_MT];
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) {
          asm volatile("ds_read_b128 %0, %1" : "=v"(f[ks][0]) : "v"(bh[ks]));
          asm volatile("ds_read_b128 %0, %1 offset:2048" : "=v"(f[ks][1]) : "v"(bh[ks]));
#define F3_TREAD(X) asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(f[ks][BG_NT + (X)]) : "v"(ah[ks]), "n"(2048 * (X)));
          F3_TREAD(0) F3_TREAD(1) F3_TREAD(2) F3_TREAD(3) F3_TREAD(4) F3_TREAD(5) F3_TREAD(6) F3_TREAD(7) F3_TREAD(8)
#undef F3_TREAD
        }
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) {
          if (ks == 0) asm volatile("s_waitcnt lgkmcnt(%0)" ::"n"(BG_NT + BG_MT) : "memory");
          else asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
          for (int qq = 0; qq < BG_NT + BG_MT; ++qq) asm volatile("" : "+v"(f[ks][qq]));
#pragma unroll
          for (int x = 0; x < BG_MT; ++x)
#pragma unroll
            for (int y = 0; y < BG_NT; ++y) {
              // half 0: x_hi W_hi; half 1: x_lo W_hi + x_hi W_lo (the products' order of the loop below)
              acc[x][y] = mfma_bf16x(__builtin_bit_cast(bf16x8, f[ks][BG_NT + x]), __builtin_bit_cast(bf16x8, f[0][y]),
                                     acc[x][y]);
              if (ks == 1)
                acc[x][y] = mfma_bf16x(__builtin_bit_cast(bf16x8, f[0][BG_NT + x]), __builtin_bit_cast(bf16x8, f[1][y]),
                                       acc[x][y]);
            }
          if (ks == 0) {
#pragma unroll
            for (int x = 0; x < BG_MT; ++x)
#pragma unroll
              for (int y = 0; y < BG_NT; ++y) asm volatile("" : "+v"(acc[x][y]));
          }
        }
      } else if constexpr (X3N) {
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

  big_epilogue<EPI, WM, WN, WIN>(a, acc, smem, n0, clip0, nclip, wmode, wpar, m0, phys);
}

// x through an empty asm: the compiler cannot move work that depends on it out of the step
F3_DEV int opaque_v(int x) {
  asm volatile("" : "+v"(x));
  return x;
}
// The window kernel's inline asm lives in these helpers: hipcc's host pass silently drops a kernel's
// launch stub when a lambda inside it holds a VGPR-constrained asm statement (found bisecting the
// undefined __device_stub__ symbols of the first igemm_win1 build).
typedef unsigned u32x4_t __attribute__((ext_vector_type(4)));
F3_DEV u32x4_t lds_rd128(unsigned addr) {
  u32x4_t v;
  asm volatile("ds_read_b128 %0, %1" : "=v"(v) : "v"(addr));
  return v;
}
template <int OFF>
F3_DEV u32x4_t lds_rd128o(unsigned addr) {
  u32x4_t v;
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(v) : "v"(addr), "n"(OFF));
  return v;
}
template <int N>
F3_DEV void wait_lgkm() { asm volatile("s_waitcnt lgkmcnt(%0)" ::"n"(N) : "memory"); }
template <int N>
F3_DEV void wait_vm() { asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory"); }
F3_DEV void pin_v(u32x4_t& v) { asm volatile("" : "+v"(v)); }
F3_DEV void pin_v(f32x4& v) { asm volatile("" : "+v"(v)); }

template <int I, int N, class F>
F3_DEV __attribute__((always_inline)) void static_for(F&& f) {
  if constexpr (I < N) {
    f(std::integral_constant<int, I>{});
    static_for<I + 1, N>(f);
  }
}

// The compile-time step schedule of one channel chunk of the clip-window GEMM (9 taps, pad 4):
//   MODE 0, stride 1 (forward or input gradient): one window, steps j = tap dt = j, frame shift
//     ss (j - 4) (ss = -1 for the input gradient, at run time);
//   MODE 1, stride-2 input gradient: the window is the clips' dY frames; a tile is one output-frame
//     parity p (NT = 5 - p steps): tap dt = p + 2 j, shift 2 - j;
//   MODE 2, stride-2 forward: two windows per chunk (q = 0 the even input frames, q = 1 the odd ones);
//     steps 0-4 window 0 with taps 0, 2, .. 8 (shift j - 2), steps 5-8 window 1 with taps 1, 3, 5, 7
//     (shift j - 7).
template <int MODE, int NT>
struct WinSched {
  static constexpr int NS = MODE == 1 ? NT : 9;                         // steps per chunk
  static constexpr int q(int j) { return MODE == 2 && j >= 5 ? 1 : 0; }
  static constexpr int jj(int j) { return MODE == 2 && j >= 5 ? j - 5 : j; }  // step within its window
  static constexpr int ntq(int qq) { return MODE == 2 ? (qq ? 4 : 5) : NS; }  // steps of window qq
  static constexpr int dt(int j) {
    return MODE == 0 ? j : MODE == 1 ? (5 - NT) + 2 * j : (q(j) ? 1 + 2 * jj(j) : 2 * jj(j));
  }
  static constexpr int shift(int j) { return MODE == 1 ? 2 - j : MODE == 2 ? jj(j) - 2 : j - 4; }  // x ss (MODE 0)
};

// igemm_win1: the clip-window GEMM in the bf16x3 native form with the tap schedule unrolled at compile
// time. igemm_big's window loop derives each step's (chunk, window, tap), its weight offset and the
// A-carry piece of the next window at run time (the carry decision alone is ~60 SALU / VALU
// instructions with exec-masked branches per step, ~300 non-MFMA instructions per 54 MFMAs in all:
// the load leg the probe builds found issue-bound). Here a chunk's steps are
// straight-line code: the tap, the LDS stage, which steps carry and which pieces a wave carries are
// constants; a wave issues its weight pieces plus ASL A-carry pieces per step (a slot with nothing to
// carry sinks the zero row, so the vmcnt count stays one constant). LDS layout, fragment reads, MFMA
// order and the epilogue are igemm_big's, so the two forms give bit-identical results.
//
// PP (ping-pong, F3_WIN1_PP=1): the two waves of a SIMD (wave w and w + NW/2) run in opposite phases, so
// one wave's fragment reads overlap the other's MFMAs (the probe builds found the two legs serialised,
// DESIGN.md §4.13). Every wave runs the same sequence per step, read | barrier | multiply | barrier;
// group B (waves NW/2 ..) starts one barrier late and skips the last one. Only group A issues the
// weight / carry DMAs (twice the pieces per wave), and every wave completes its reads (lgkmcnt 0)
// before the barrier that ends its read phase, so a stage is refilled only after both groups have
// read it. Each wave issues the same MFMAs in the same order as the plain form: bit-identical results.
template <int EPI, int WM, int WN, int WIN, int MODE, int NTP = 5, bool PP = false>
__global__ __launch_bounds__(64 * WM * WN) void igemm_win1(ConvGemmArgs a) {
  using Cfg = BigCfg<WM, WN, WIN>;
  constexpr int NW = WM * WN, NT = 64 * NW;
  constexpr int KT = 9, CL = WIN;
  constexpr int BN = Cfg::BN, STAGE = Cfg::STAGE, NST = Cfg::NST, LA = Cfg::LA, CPW = Cfg::CPW, NPA = Cfg::NPA;
  constexpr int NWS = PP ? NW / 2 : NW;                           // staging waves (PP: group A)
  constexpr int BSL = Cfg::BP / NWS;                              // weight pieces per wave and step
  constexpr int NQ = MODE == 2 ? 2 : 1;                           // windows per chunk
  // carry pieces per step: a window is carried by the LA.. steps of the window before it and that
  // window's step 0 (the last group): ntq - LA + 1 groups of aps pieces
  constexpr int APS_MAX = MODE == 0 ? (NPA + (KT - LA)) / (KT - LA + 1) : (NPA + (4 - LA)) / (4 - LA + 1);
  constexpr int ASL = (APS_MAX + NWS - 1) / NWS;                  // A slots per wave and step
  constexpr int DPS = BSL + ASL;                                  // DMAs per wave and step
  constexpr int A0W = (NPA + NW - 1) / NW;                        // window 0's pieces per wave
  static_assert(Cfg::BP % NWS == 0 && (LA == 1 || LA == 2) && (MODE == 0 || LA == 2), "win1 staging");
  static_assert(Cfg::SMEM <= 160 * 1024 && (NST - 1) * DPS < 64, "LDS / vmcnt");
  __shared__ __attribute__((aligned(16))) char smem[Cfg::SMEM];
  const ConvGeom& g = a.g;
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  int tile = xcd_remap(blockIdx.x, gridDim.x);
  const int ncol = g.Nc / BN;
  const int n0 = (tile % ncol) * BN;
  tile /= ncol;
  const int wpar = MODE == 1 ? 5 - NTP : 0;  // MODE 1: this launch's output-frame parity (NTP taps)
  const int clip0 = tile * CPW;
  const int nclip = g.M / (g.T_out * g.V);
  const int V = g.V, TVin = g.T_in * V, kpt = g.Kc / 32;
  const int ss = MODE == 0 ? (g.transposed ? -1 : 1) : 1;  // MODE 0: tap dt reads frame t + ss (dt - 4)
  // valid rows of window q (MODE 2: the even / odd input frames)
  const int wlim0 = (MODE == 2 ? (g.T_in + 1) >> 1 : g.T_in) * V, wlim1 = (g.T_in >> 1) * V;
  const unsigned minv = (65536u + V - 1) / V;  // l / V as (l * minv) >> 16 (l < 2^9, V < 2^7)
  if (EPI & EPI_RELUMASK) {
    float* epi_sc = reinterpret_cast<float*>(smem + Cfg::EPI_OFF);
    for (int t = tid; t < BN; t += NT) {
      float sc, sh, mu, rs;
      bn_coeff(a.epi_bn, n0 + t, sc, sh, mu, rs);
      epi_sc[t] = sc; epi_sc[BN + t] = sh; epi_sc[2 * BN + t] = mu; epi_sc[3 * BN + t] = rs;
    }
  }
  const unsigned short* in = a.inb;
  const unsigned short* wb = a.wb;
  const int sub = lane >> 3, pch = lane & 7;
  // the lane's 16-B chunk of a staged A row piece: swz(R, pch) with R & 7 == sub, in the x3n row
  const int sA = pch ^ sub, colA = 8 * sA + (sA >= 4 ? g.Kc - 32 : 0);
  const int Ktot = KT * g.Kc * 2;
  const unsigned short* bsrc[BSL];
#pragma unroll
  for (int i = 0; i < BSL; ++i) {
    const int r = ((PP ? wave % NWS : wave) + NWS * i) * 8 + sub;  // (PP: group B never stages)
    bsrc[i] = wb + (size_t)(n0 + r) * Ktot + swz(r, pch) * 8;
  }
  // window row R (= piece * 8 + sub) of chunk c, window q: clip row l of clip clip0 + k
  auto asrc = [&](int c, int qq, int R) -> const void* {
    const int k = (CPW == 2 && R >= CL) ? 1 : 0, l = R - k * CL, clip = clip0 + k;
    if (l >= (qq ? wlim1 : wlim0) || clip >= nclip) return a.zero;
    int row = clip * TVin + l;
    if (MODE == 2) row += (int)(((unsigned)l * minv) >> 16) * V + qq * V;  // input frame 2 f + q
    return in + (size_t)row * g.lda + c * 32 + colA;
  };

  using S = WinSched<MODE, NTP>;
  constexpr int NS = S::NS;
    // stage of step (c, J): the weight pieces of its tap, then the A carry: steps jj >= LA carry group
    // jj - LA of the next window, step jj = 0 (except the first window) its own window's last group
    auto stage = [&](const int J, int c) {
      const int Q = S::q(J), JJ = S::jj(J);
      char* sbase = smem + Cfg::SOFF + ((c * (NS % NST) + J) % NST) * STAGE;
      const int k0 = S::dt(J) * 2 * g.Kc + 64 * c;
#pragma unroll
      for (int i = 0; i < BSL; ++i) {
        const void* wsrc = bsrc[i] + k0;
        __builtin_amdgcn_global_load_lds(wsrc, (lds_void_t*)(sbase + (wave + NWS * i) * 1024), 16, 0, 0);
      }
      // target window (tc, tq), group kk, pieces per group na; carry == false: sink
      const bool NEXT = JJ >= LA, OWN = JJ == 0;
      const int TQ = NEXT ? (NQ == 2 && Q == 0 ? 1 : 0) : Q;
      const int QP = NQ == 2 ? 1 - Q : 0;  // the window before (OWN)
      const int KK = NEXT ? JJ - LA : S::ntq(QP) - LA;
      const int NCAR = (NEXT ? S::ntq(Q) : S::ntq(QP)) - LA + 1;
      const int NA = (NPA + NCAR - 1) / NCAR;  // (<= ASL * NW: APS_MAX)
      const int tc = NEXT && !(NQ == 2 && Q == 0) ? c + 1 : c;
      const bool car = (NEXT || OWN) && tc < kpt && !(OWN && c == 0 && Q == 0);
#pragma unroll
      for (int s2 = 0; s2 < ASL; ++s2) {
        const void* src = a.zero;
        char* dst = smem + Cfg::DOFF;
        const int sl = wave + NWS * s2, pa = KK * NA + sl;
        if (car && sl < NA && pa < NPA) {
          src = asrc(tc, TQ, opaque_v(wave * 8 + sub) + (KK * NA + NWS * s2) * 8);
          dst = smem + (NQ == 2 ? TQ : (tc & 1)) * Cfg::AWIN + pa * 1024;
        }
        __builtin_amdgcn_global_load_lds(src, (lds_void_t*)dst, 16, 0, 0);
      }
    };
    // window 0's rows (chunk 0, q 0), then the stages of steps 0 .. LA - 1 (they carry nothing)
#pragma unroll
    for (int i = 0; i < A0W; ++i) {
      const int pa = (wave + NW * i) % NPA;
      const void* src = asrc(0, 0, pa * 8 + sub);
      __builtin_amdgcn_global_load_lds(src, (lds_void_t*)(smem + pa * 1024), 16, 0, 0);
    }
    const bool grpB = PP && wave >= NWS;
    if (!grpB) {
      stage(0, 0);
      if constexpr (LA == 2) stage(1, 0);
    }
    if (tid < 8) *reinterpret_cast<f32x4*>(smem + Cfg::ZOFF + tid * 16) = f32x4{0.f, 0.f, 0.f, 0.f};
    if (LA == 2 && !grpB) wait_vm<DPS>();
    else wait_vm<0>();
    wait_lgkm<0>();
    __builtin_amdgcn_s_barrier();

    const int wm = wave / WN, wn = wave % WN;
    const int fr = lane & 15, fg = lane >> 4;
    f32x4 acc[BG_MT][BG_NT];
#pragma unroll
    for (int x = 0; x < BG_MT; ++x)
#pragma unroll
      for (int y = 0; y < BG_NT; ++y) acc[x][y] = f32x4{0.f, 0.f, 0.f, 0.f};
    const unsigned lds0 = (unsigned)(size_t)(lds_cchar_t*)smem;
    const unsigned zrow = lds0 + Cfg::ZOFF;
    unsigned boffr[2][BG_NT];
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int y = 0; y < BG_NT; ++y) {
        const int r = wn * 32 + y * 16 + fr;
        boffr[ks][y] = lds0 + Cfg::SOFF + r * 128 + swz(r, ks * 4 + fg) * 16;
      }
    // the wave's rows: clip base row in the window and first output row of the clip
    const int cbase = CPW == 2 ? wm * 144 : 0, lo0 = CPW == 2 ? 0 : wm * 144;
    u32x4_t f[2][BG_NT + BG_MT];
    if (grpB) __builtin_amdgcn_s_barrier();  // PP: group B runs one phase behind
#define F3_W1_READS                                                                                  \
  _Pragma("unroll") for (int ks = 0; ks < 2; ++ks) {                                                 \
    _Pragma("unroll") for (int y = 0; y < BG_NT; ++y)                                                \
      f[ks][y] = (F3_PROBE & 4) ? u32x4_t{0u, 0u, 0u, 0u} : lds_rd128(boffr[ks][y] + soff);           \
    F3_AREAD1(0) F3_AREAD1(1) F3_AREAD1(2) F3_AREAD1(3) F3_AREAD1(4) F3_AREAD1(5) F3_AREAD1(6)       \
    F3_AREAD1(7) F3_AREAD1(8)                                                                        \
  }
#define F3_AREAD1(X)                                                                                 \
  {                                                                                                  \
    const unsigned ad = (unsigned)(t + 16 * (X)) < (unsigned)CL ? (ks ? ab1 : ab0) : zrow - 2048u * (X); \
    f[ks][BG_NT + (X)] = (F3_PROBE & 4) ? u32x4_t{ad, 0u, 0u, 0u} : lds_rd128o<2048 * (X)>(ad);        \
  }
#define F3_W1_MFMAS                                                                                  \
  _Pragma("unroll") for (int ks = 0; ks < 2; ++ks) {                                                 \
    if (ks == 0) wait_lgkm<BG_NT + BG_MT>();                                                         \
    else wait_lgkm<0>();                                                                             \
    _Pragma("unroll") for (int qq = 0; qq < BG_NT + BG_MT; ++qq) pin_v(f[ks][qq]);                   \
    _Pragma("unroll") for (int x = 0; x < BG_MT; ++x)                                                \
      _Pragma("unroll") for (int y = 0; y < BG_NT; ++y) {                                            \
        if (F3_PROBE & 1) { /* probe build: fragments consumed, no MFMA */                           \
          acc[x][y][0] += __builtin_bit_cast(float, f[ks][BG_NT + x][0] ^ f[ks][y][1]);              \
          continue;                                                                                  \
        }                                                                                            \
        /* half 0: x_hi W_hi; half 1: x_lo W_hi + x_hi W_lo (igemm_big's order) */                   \
        acc[x][y] = mfma_bf16x(__builtin_bit_cast(bf16x8, f[ks][BG_NT + x]), __builtin_bit_cast(bf16x8, f[0][y]), \
                               acc[x][y]);                                                           \
        if (ks == 1)                                                                                 \
          acc[x][y] = mfma_bf16x(__builtin_bit_cast(bf16x8, f[0][BG_NT + x]),                        \
                                 __builtin_bit_cast(bf16x8, f[1][y]), acc[x][y]);                    \
      }                                                                                              \
    if (ks == 0) {                                                                                   \
      _Pragma("unroll") for (int x = 0; x < BG_MT; ++x)                                              \
        _Pragma("unroll") for (int y = 0; y < BG_NT; ++y) pin_v(acc[x][y]);                          \
    }                                                                                                \
  }
    for (int c = 0; c < kpt; ++c) {
      const bool more = c + 1 < kpt;
#pragma unroll
      for (int J = 0; J < NS; ++J) {  // unrolled: the schedule below folds to constants per step
        const int JS = (J + LA) % NS, CS = (J + LA) / NS;  // the step staged now: (c + CS, JS)
        const bool issue = CS == 0 || more;
        const unsigned wrow = lds0 + (NQ == 2 ? S::q(J) : (c & 1)) * Cfg::AWIN + (unsigned)cbase * 128;
        const int t = opaque_v(lo0 + fr) + (MODE == 0 ? ss * S::shift(J) : S::shift(J)) * V;  // tap-shifted row
        const unsigned rb = wrow + (unsigned)t * 128;
        const unsigned ab0 = rb + ((fg ^ (t & 7)) << 4), ab1 = rb + (((4 + fg) ^ (t & 7)) << 4);
        const unsigned soff = ((c * (NS % NST) + J) % NST) * STAGE;
        if constexpr (PP) {
          // read | barrier | multiply | barrier (group B one phase behind group A)
          if (!grpB && issue && !(F3_PROBE & 2)) stage(JS, c + CS);
          F3_W1_READS
          wait_lgkm<0>();
          __builtin_amdgcn_s_barrier();
          F3_W1_MFMAS
          if (!grpB) {
            if (LA == 2 && issue) wait_vm<DPS>();
            else wait_vm<0>();
          }
          if (!(grpB && J == NS - 1 && !more) && !(F3_PROBE & 8)) __builtin_amdgcn_s_barrier();
          continue;
        } else {
          if (issue && !(F3_PROBE & 2)) stage(JS, c + CS);
          F3_W1_READS
          F3_W1_MFMAS
        }
        // the step staged LA ahead must land before its compute: with LA = 2 this step's own DMAs
        // (the step after next) stay in flight
        if (LA == 2 && issue) wait_vm<DPS>();
        else wait_vm<0>();
        if (!(F3_PROBE & 8)) __builtin_amdgcn_s_barrier();
      }
    }
#undef F3_W1_READS
#undef F3_AREAD1
#undef F3_W1_MFMAS
    __syncthreads();
    auto none = [](int) { return -1; };
    if (F3_PROBE & 16) {  // probe build: no epilogue (one word per wave keeps the loop alive)
      if (lane == 0) a.out[blockIdx.x * NW + wave] = acc[0][0][0] + acc[BG_MT - 1][BG_NT - 1][3];
      return;
    }
    big_epilogue<EPI, WM, WN, WIN>(a, acc, smem, n0, clip0, nclip, MODE, wpar, 0, none);
}

}  // namespace f3

using namespace f3;

// Clip-window form (WIN): the clip rows of the window layout for a 9-tap temporal conv (stride 1
// forward or input gradient, stride-2 forward or input gradient) whose window and output frames
// fit 144 rows (two clips per tile) or 270 rows (one clip), else 0
static int big_win_rows(const ConvGemmArgs& a) {
  const ConvGeom& g = a.g;
  const int cb = a.x3n ? 32 : G_BK;
  if ((g.Nc % 128 && g.Nc != 64) || g.KT != 9 || 2 * g.P != g.KT - 1 || g.Kc % cb || g.T_out <= 0 || g.M % (g.T_out * g.V))
    return 0;
  int wf, of;  // window frames, output frames of one tile clip
  if (g.S == 1) {
    if (g.T_in != g.T_out) return 0;
    wf = of = g.T_in;
  } else if (g.S == 2) {
    wf = g.transposed ? g.T_in : (g.T_in + 1) / 2;
    of = g.transposed ? (g.T_out + 1) / 2 : g.T_out;
  } else {
    return 0;
  }
  const int rows = (wf > of ? wf : of) * g.V;
  if (g.Nc == 64) return g.S == 1 && rows <= 540 ? 540 : 0;
  return rows <= 144 ? 144 : rows <= 270 ? 270 : 0;
}

// Large tiles pay when the k loop is long enough to amortise the 3-stage prologue.
bool f3_igemm_big_ok(const ConvGemmArgs& a) {
  if (!f3_igemm_ok(a)) return false;
  if (a.g.Nc == 64) return big_win_rows(a) == 540;  // the window form only
  if (a.g.Nc != 128 && a.g.Nc != 256) return false;
  return a.g.KT * a.g.Kc / (a.x3n ? 32 : G_BK) >= 6;
}

// F3_K1=0 (A/B only): the 1x1 tiled GEMMs on the generic per-step staging (read per call)
static bool k1_enabled() {
  const char* e = getenv("F3_K1");
  return !e || atoi(e) != 0;
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
  const bool k1 = a.g.KT == 1 && k1_enabled();
#define F3_BCASE(E)                                                                              \
  if (epi == (E)) {                                                                             \
    if (k1) hipLaunchKernelGGL((igemm_big<(E), WM, WN, 0, X3N, true>), dim3(tiles), dim3(BG_THREADS), 0, s, a); \
    else hipLaunchKernelGGL((igemm_big<(E), WM, WN, 0, X3N>), dim3(tiles), dim3(BG_THREADS), 0, s, a); \
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

bool f3_igemm_big_win_ok(const ConvGemmArgs& a) { return f3_igemm_big_ok(a) && big_win_rows(a) != 0; }

// W4 (WIN = 144 only): a 4-wave form, one clip x 128 channels per workgroup, meant to run two
// independent workgroups per CU. Measured 1.5-1.75x SLOWER alone (l8d 134 -> 235 us) and the step
// 8.73 -> 9.36 ms (profiles/r05_win4_ab.txt); not dispatched, kept as the template's 4-wave case.
// F3_WIN1 (A/B only; read per call, the tests compare the forms): 0 = the window GEMMs on igemm_big's
// run-time tap schedule, 1 = igemm_win1 for stride 1 only, unset / 2 = igemm_win1 for every mode
static bool win1_enabled(int mode) {
  const char* e = getenv("F3_WIN1");
  const int v = e ? atoi(e) : 2;
  return mode == 0 ? v >= 1 : v >= 2;
}

// F3_WIN1_PP=1 (A/B; read per call): the ping-pong form of igemm_win1
static bool win1_pp() {
  const char* e = getenv("F3_WIN1_PP");
  return e && atoi(e) == 1;
}

template <int E, int WM, int WN, int CL, bool PP>
static void launch_win1_pp(const ConvGemmArgs& a, int mode, int tiles, hipStream_t s) {
  if constexpr (CL == 540) {  // (64-channel layers: stride 1 only)
    hipLaunchKernelGGL((igemm_win1<E, WM, WN, CL, 0, 5, PP>), dim3(tiles), dim3(64 * WM * WN), 0, s, a);
  } else {
    if (mode == 0) hipLaunchKernelGGL((igemm_win1<E, WM, WN, CL, 0, 5, PP>), dim3(tiles), dim3(64 * WM * WN), 0, s, a);
    else if (mode == 1) {  // one launch per output-frame parity (5 / 4 taps: a compile-time schedule each)
      hipLaunchKernelGGL((igemm_win1<E, WM, WN, CL, 1, 5, PP>), dim3(tiles / 2), dim3(64 * WM * WN), 0, s, a);
      hipLaunchKernelGGL((igemm_win1<E, WM, WN, CL, 1, 4, PP>), dim3(tiles / 2), dim3(64 * WM * WN), 0, s, a);
    }
    else hipLaunchKernelGGL((igemm_win1<E, WM, WN, CL, 2, 5, PP>), dim3(tiles), dim3(64 * WM * WN), 0, s, a);
  }
}

template <int E, int WM, int WN, int CL>
static void launch_win1(const ConvGemmArgs& a, int mode, int tiles, hipStream_t s) {
  if (win1_pp()) launch_win1_pp<E, WM, WN, CL, true>(a, mode, tiles, s);
  else launch_win1_pp<E, WM, WN, CL, false>(a, mode, tiles, s);
}

template <int CL, bool W4 = false>
static int launch_win(const ConvGemmArgs& a, int epi, hipStream_t s) {
  constexpr int WM = CL == 540 ? 4 : W4 ? 1 : 2, WN = CL == 540 ? 2 : 4, CPW = BigCfg<WM, WN, CL>::CPW;
  const int nclip = a.g.M / (a.g.T_out * a.g.V);
  const int tiles = (nclip + CPW - 1) / CPW * (a.g.S == 2 && a.g.transposed ? 2 : 1) * (a.g.Nc / (32 * WN));
  // 9 taps, pad 4, native split form: the compile-time tap schedule (igemm_win1). Alone
  // (tools/kbench.py, profiles/r06_win1_kbench.txt): T=8 fwd / dgrad 138 / 132 -> 114 / 110 us, T=15 75 /
  // 77 -> 67 / 66, T=30 dgrad 46 -> 43; the T=30 forward measured 43.6 -> 45.2 and stays on igemm_big.
  // Stride 2: MODE 1 (input gradient by output-frame parity), MODE 2 (forward, even / odd windows).
  const int mode = a.g.S == 1 ? 0 : a.g.transposed ? 1 : 2;
  const bool w1 = !W4 && a.x3n && a.g.KT == 9 && a.g.P == 4 && (CL != 540 || (a.g.transposed && mode == 0)) &&
                  win1_enabled(mode);
#define F3_WCASE(E)                                                                                   \
  if (epi == (E)) {                                                                                  \
    if (w1) launch_win1<(E), WM, WN, CL>(a, mode, tiles, s);                                          \
    else if (a.x3n) hipLaunchKernelGGL((igemm_big<(E), WM, WN, CL, true>), dim3(tiles), dim3(64 * WM * WN), 0, s, a); \
    else hipLaunchKernelGGL((igemm_big<(E), WM, WN, CL, false>), dim3(tiles), dim3(64 * WM * WN), 0, s, a);     \
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
  const int wrows = big_win_rows(a);
  if (wrows) {
    const int r = wrows == 144 ? launch_win<144>(a, epi, s)
                  : wrows == 270 ? launch_win<270>(a, epi, s) : launch_win<540>(a, epi, s);
    if (r != F3_EINVAL) return r;
  }
  if (a.g.Nc == 64) return F3_EINVAL;
  if (a.g.Nc == 256) return a.x3n ? launch_big<1, 8, true>(a, epi, s) : launch_big<1, 8, false>(a, epi, s);
  return a.x3n ? launch_big<2, 4, true>(a, epi, s) : launch_big<2, 4, false>(a, epi, s);
}
