// Weight-stationary persistent GEMM for the 1x1 convolutions of the skeleton streams: the gcn
// forward (g = conv1x1(Z) + graph-mixed bias, BN1 statistics; stgcan.py:50-56), the gcn input
// gradient (dZ = dg . W), the stride-2 residual conv forward (r = conv1x1(x[:, ::2]) + bias, BN
// statistics; stgcan.py:123-133) and its input gradient (dx[:, ::2] += dr . W, stgcan.py:143-144).
//
// Why a separate kernel. These GEMMs have K = 64-256 and N = 64-768 against M = 37k-138k rows: one
// to four 64-deep k chunks per output tile, so the tiled igemm_bf16 paid each tile's prologue (A and
// B from HBM), a barrier per chunk and an epilogue with fp64 statistic atomics (every tile into the
// same 2*Nc addresses) with 2 workgroups per CU to hide them: 33-64 us per launch for 26-88 MB of
// bf16 rows, i.e. 1.4-2.8 TB/s (profiles/r03_step_serial_kernels.txt). Here:
//   - a workgroup owns one column group of NT = 64*WN output columns (WN = 1, 2, 3, 4 or 6, chosen
//     so that one group covers as much of Nc as the registers allow) and keeps that slice of the
//     weight panel in REGISTERS for the whole launch (each of the 8 waves holds 16*WN columns x K:
//     WN*K/8 VGPRs, at most 128);
//   - it is persistent over a contiguous range of 64-row tiles; a tile's whole A block (64 rows x K,
//     bf16) is staged by LDS-DMA into a ring of NB buffers (as many as the LDS holds, 3-12), NB - 1
//     tiles ahead: at the end of a tile only the NEXT tile's block must have landed (a counted
//     vmcnt: every load is issued unconditionally, from the zero page past the range, so the count
//     is static), the NB - 2 after it stay in flight across the barrier;
//   - the output leaves through an LDS image (bf16, or the fp32 accumulated rows of EPI_ADD) as
//     16-B row pieces issued at the start of the next tile, so they drain under its MFMAs; BN
//     statistics stay in registers across the tiles and are added once per workgroup;
//   - the workgroups that share a row range (one per column group) get consecutive XCD-remapped
//     ids, so a range's A rows come from HBM once and from that XCD's L2 for the other groups.
// Epilogues: EPI_BIASV|EPI_STATS (gcn forward; the [V][NT] bias slice sits in LDS), EPI_BIAS|EPI_STATS
// (residual forward), EPI_BIAS (plain conv, tests), 0 (gcn input gradient), EPI_ADD (residual input
// gradient into the fp32 dx rows; stride 2 walks only the even output frames, the odd ones receive
// nothing). Output bf16 (non-accumulating) or fp32 (EPI_ADD).
#include "igemm.h"

#include <algorithm>
#include <type_traits>

namespace f3 {

constexpr int PW_LDS_BUDGET = 156 * 1024;
constexpr int PW_THREADS = 512;  // 8 waves: wm = wave & 1 (BM/2 rows), wj = wave >> 1 (16*WN columns)
constexpr int PW_VMAX = 18;      // joints of the BIASV table

// BM = rows per tile: 64, or 32 for K = 384 / 768 (a 64-row block of those is 48 / 96 KB)
template <int EPI, int KS, int WN, int BM, bool F32O = false>
struct PwLds {
  static constexpr bool ADD = (EPI & EPI_ADD) != 0;
  static constexpr bool WIDE = ADD || F32O;  // fp32 output image (accumulated, or plain fp32 rows)
  static constexpr int PW_BM = BM;
  static constexpr int K = KS * 32;
  static constexpr int NT = 64 * WN;            // columns per workgroup
  static constexpr int ABUF = PW_BM * K * 2;    // bytes per A buffer ([K/64][BM rows][128 B])
  static constexpr int OTS = WIDE ? NT + 4 : NT + 8;  // output image row stride (elements)
  static constexpr int ES = WIDE ? 4 : 2;             // image element size (fp32 / bf16)
  static constexpr int FIXED = PW_BM * OTS * ES + ((EPI & EPI_BIASV) ? PW_VMAX * NT * 4 : 0) +
                               ((EPI & EPI_STATS) ? 2 * 2 * NT * 4 : 0);
  // A ring depth: as many buffers as the LDS holds (NB - 2 tiles stay in flight across the end-of-
  // tile wait; ~72 KB per CU keeps HBM streaming, MI355X_MICROARCH.md 'gather into LDS'), capped at
  // 12; EPI_ADD keeps 3 (hipcc drains vmcnt before the preloaded rows anyway, see below)
  static constexpr int NB_FIT = (PW_LDS_BUDGET - FIXED) / ABUF;
  static constexpr int NB = ADD ? 3 : (NB_FIT > 12 ? 12 : NB_FIT);
  static constexpr int OT_OFF = NB * ABUF;
  static constexpr int BV_OFF = OT_OFF + PW_BM * OTS * ES;
  static constexpr int RED_OFF = BV_OFF + ((EPI & EPI_BIASV) ? PW_VMAX * NT * 4 : 0);
  static constexpr int BYTES = RED_OFF + ((EPI & EPI_STATS) ? 2 * 2 * NT * 4 : 0);
  // 16-B image pieces per tile, and per thread: PIECES each, or (TP < 512) one for threads < TP
  static constexpr int TP = PW_BM * NT * ES / 16;
  static constexpr int PIECES = TP >= PW_THREADS ? TP / PW_THREADS : 1;
  static constexpr int LPT = (KS / 2) * PW_BM / 64;  // DMA instructions per thread and tile
};

// s_waitcnt vmcnt(BASE + min(k, KMAX) * STEP) for a wave-uniform k (immediates only)
template <int BASE, int STEP, int KMAX>
F3_DEV void pw_wait_vm(int k) {
  if constexpr (KMAX == 0) {
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(BASE) : "memory");
  } else {
    if (k >= KMAX) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(BASE + KMAX * STEP) : "memory");
    else pw_wait_vm<BASE, STEP, KMAX - 1>(k);
  }
}

// F32O: fp32 output rows (a.out) instead of bf16 (the bf16x3 mode's fp32 activations). X3N: the bf16x3
// native form (ConvGemmArgs::x3n; the weight slices alternate hi / lo per 32-channel block, the A
// block's 128-B chunks are [x_hi 32 | x_lo 32], three MFMAs per block), fp32 output as F32O
template <int EPI, int KS, int WN, int BM, bool F32O = false, bool X3N = false>
__global__ __launch_bounds__(PW_THREADS) void pw_gemm_kernel(ConvGemmArgs a, int ncg, int per_wg) {
  using L = PwLds<EPI, KS, WN, BM, F32O>;
  constexpr int PW_BM = BM, MX = BM / 32;  // MX: 16-row MFMA tiles per wave
  constexpr int NT = L::NT, KC = KS / 2, OTS = L::OTS, NB = L::NB, LPT = L::LPT;
  constexpr bool ADD = L::ADD;
  static_assert(KS % 2 == 0 && NB >= 3 && L::BYTES <= 160 * 1024, "pw_gemm LDS");
  static_assert((BM == 64 || (BM == 32 && !ADD && KC % 2 == 0)) && LPT * 64 == KC * BM, "tile rows");
  static_assert((NB - 2) * (LPT + L::PIECES) < 64, "vmcnt immediate");
  static_assert(L::TP % 64 == 0 && (L::TP < PW_THREADS || L::TP % PW_THREADS == 0), "image pieces");
  extern __shared__ __attribute__((aligned(16))) char pw_smem[];
  char* img = pw_smem + L::OT_OFF;
  float* bv = reinterpret_cast<float*>(pw_smem + L::BV_OFF);   // [V][NT] graph-mixed bias slice
  float* red = reinterpret_cast<float*>(pw_smem + L::RED_OFF);  // [2 wm][2][NT] statistic partials
  const ConvGeom& g = a.g;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave & 1, wj = wave >> 1;
  const int fr = lane & 15, fg = lane >> 4;
  const int lin = xcd_remap(blockIdx.x, gridDim.x);
  const int cg = lin % ncg, range = lin / ncg;
  const int j0 = cg * NT;
  // stride-2 input gradient (EPI_ADD, the only accumulating use): the tile rows are the even
  // output frames
  constexpr bool par = ADD;
  const int Tp = par ? (g.T_out + 1) >> 1 : g.T_out;
  const int Mp = par ? (g.M / (g.T_out * g.V)) * Tp * g.V : g.M;
  const int ntiles = (Mp + PW_BM - 1) / PW_BM;
  const int tile0 = range * per_wg, tile1 = min(ntiles, tile0 + per_wg);
  if (tile0 >= tile1) return;
  auto phys = [&](int r) -> int {  // tile row -> output row (-1: none)
    if (r >= Mp) return -1;
    if (!par) return r;
    const int nt = r / g.V, v = r - nt * g.V, n = nt / Tp, tt = nt - n * Tp;
    return (n * g.T_out + 2 * tt) * g.V + v;
  };

  // this wave's weight slice: columns j0 + wj*16*WN + y*16 + fr, k = s*32 + fg*8 .. +8 (X3N: slice 2b
  // is block b's W_hi, 2b + 1 its W_lo; the packed row holds 2 Kc)
  bf16x8 wf[WN][KS];
  const int wld = X3N ? 2 * g.Kc : g.Kc;
#pragma unroll
  for (int y = 0; y < WN; ++y) {
    const unsigned short* wr = a.wb + (size_t)(j0 + wj * 16 * WN + y * 16 + fr) * wld + fg * 8;
#pragma unroll
    for (int s = 0; s < KS; ++s) wf[y][s] = *reinterpret_cast<const bf16x8*>(wr + s * 32);
  }
  float bias[WN];
#pragma unroll
  for (int y = 0; y < WN; ++y) bias[y] = (EPI & EPI_BIAS) ? a.bias[j0 + wj * 16 * WN + y * 16 + fr] : 0.f;
  if (EPI & EPI_BIASV)
    for (int i = tid; i < g.V * NT; i += PW_THREADS) bv[i] = a.bias[(i / NT) * g.Nc + j0 + i % NT];
  float ssum[WN], ssq[WN];
#pragma unroll
  for (int y = 0; y < WN; ++y) ssum[y] = ssq[y] = 0.f;
  // use the weight and bias registers here, before any DMA is issued: hipcc does not count loads and
  // LDS-DMA in order, so a first use after the prologue DMA made it wait vmcnt(0) for the whole ring
#pragma unroll
  for (int y = 0; y < WN; ++y) {
#pragma unroll
    for (int s = 0; s < KS; ++s) asm volatile("" ::"v"(wf[y][s]));
    asm volatile("" ::"v"(bias[y]));
  }

  // A staging: 1-KiB DMA pieces of 8 rows x 128 B, piece q = (64-channel chunk, row group); wave w
  // stages pieces w + 8i, i.e. row group w % (BM/8) of chunks (w + 8i) / (BM/8) (LPT instructions per
  // thread and tile, always issued: past the range from the zero page)
  constexpr int RGN = PW_BM / 8;
  const int sub = lane >> 3, pch = lane & 7, rr = (wave % RGN) * 8 + sub;
  auto load_tile = [&](int tile, int buf) {
    char* dst = pw_smem + buf * L::ABUF;
    const int m = tile < tile1 ? phys(tile * PW_BM + rr) : -1;
    const int r = m >= 0 ? rowmap_src(rowmap(m, g), 0, g) : -1;
    const unsigned short* src = r >= 0 ? a.inb + (size_t)r * g.lda : nullptr;
    const int cgl = swz(rr, pch);
#pragma unroll
    for (int i = 0; i < LPT; ++i) {
      const int q = wave + 8 * i, kc = q / RGN;
      const unsigned short* p = src ? src + (X3N ? x3n_col(g.Kc, kc * 32, cgl) : kc * 64 + cgl * 8) : a.zero;
      __builtin_amdgcn_global_load_lds((const void*)p, (lds_void_t*)(dst + q * 1024), 16, 0, 0);
    }
  };
  // the staged output of a tile -> HBM (16-B row pieces, L::PIECES per thread). FULL: every row of
  // the tile is valid (every tile but the problem's last), so the store count is static. The image
  // is read with inline asm and its own lgkmcnt wait: hipcc cannot tell a plain LDS read of the image
  // from one of the DMA destinations and waited vmcnt(0) before it, i.e. for the tile in flight.
  constexpr int CPR = NT * L::ES / 16;
  const unsigned img_lds = (unsigned)(size_t)(lds_void_t*)img;
  const bool storer = L::TP >= PW_THREADS || tid < L::TP;  // wave-uniform (TP % 64 == 0)
  auto store_tile = [&](int tile, auto full) {
    if (!storer) return;
#pragma unroll
    for (int i = 0; i < L::PIECES; ++i) {
      const int q = tid + i * PW_THREADS, rl = q / CPR, c = q - rl * CPR;
      const int m = phys(tile * PW_BM + rl);
      if (!decltype(full)::value && m < 0) continue;
      uint4 v;
      asm volatile("ds_read_b128 %0, %1\n\ts_waitcnt lgkmcnt(0)"
                   : "=v"(v)
                   : "v"(img_lds + (unsigned)((rl * OTS) * L::ES + c * 16))
                   : "memory");
      char* dst = L::WIDE ? reinterpret_cast<char*>(a.out + (size_t)m * g.ldo + j0)
                      : reinterpret_cast<char*>(reinterpret_cast<__bf16*>(a.outb) + (size_t)m * g.ldo + j0);
      *reinterpret_cast<uint4*>(dst + c * 16) = v;
    }
  };
  // EPI_ADD: the accumulated fp32 rows of a tile, loaded into registers one tile ahead (issued after
  // the end-of-tile barrier, so the next tile's stores and DMA are younger and stay in flight)
  float pre[2][4][WN];
  auto preload = [&](int tile) {
#pragma unroll
    for (int x = 0; x < 2; ++x)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = max(phys(tile * PW_BM + wm * 32 + x * 16 + fg * 4 + r), 0);
        const float* o = a.out + (size_t)m * g.ldo + j0 + wj * 16 * WN + fr;
#pragma unroll
        for (int y = 0; y < WN; ++y) pre[x][r][y] = o[y * 16];
      }
  };

#pragma unroll
  for (int i = 0; i < NB - 1; ++i) load_tile(tile0 + i, i);
  // tile0's block has landed (the other NB - 2 stay in flight) and the bias table is written. A raw
  // barrier: __syncthreads() would wait vmcnt(0)
  asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"n"((NB - 2) * LPT) : "memory");
  __builtin_amdgcn_s_barrier();
  if (ADD) preload(tile0);
  // One tile. Every vector-memory operation in it is unconditional (stores of full tiles, loads past
  // the range from the zero page, the preload clamped to the last tile) and the first tile (nothing
  // staged yet) is a separate instance of the body, so the end-of-tile wait counts exactly the
  // younger operations: tile t + 1's block was issued NB - 2 tiles before, each of which issued KC
  // loads and, after the first, L::PIECES stores. (EPI_ADD: the preloads are younger still, so the
  // count is conservative; hipcc waits vmcnt(0) before the preloaded rows' first use regardless: it
  // does not count loads of different kinds in order.)
  auto body = [&](int tile, auto first) {
    const int it = tile - tile0, buf = it % NB;
    if constexpr (!decltype(first)::value) store_tile(tile - 1, std::true_type{});
    load_tile(tile + NB - 1, (it + NB - 1) % NB);
    const char* A = pw_smem + buf * L::ABUF;
    f32x4 acc[MX][WN];
#pragma unroll
    for (int x = 0; x < MX; ++x)
#pragma unroll
      for (int y = 0; y < WN; ++y) acc[x][y] = f32x4{0.f, 0.f, 0.f, 0.f};
    if constexpr (X3N) {
#pragma unroll
      for (int b = 0; b < KS / 2; ++b) {
#pragma unroll
        for (int x = 0; x < MX; ++x) {
          const int r = wm * 16 * MX + x * 16 + fr;
          const bf16x8 fah = *reinterpret_cast<const bf16x8*>(A + (b * PW_BM + r) * 128 + swz(r, fg) * 16);
          const bf16x8 fal = *reinterpret_cast<const bf16x8*>(A + (b * PW_BM + r) * 128 + swz(r, 4 + fg) * 16);
#pragma unroll
          for (int y = 0; y < WN; ++y) {
            acc[x][y] = mfma_bf16x(fah, wf[y][2 * b], acc[x][y]);
            acc[x][y] = mfma_bf16x(fal, wf[y][2 * b], acc[x][y]);
            acc[x][y] = mfma_bf16x(fah, wf[y][2 * b + 1], acc[x][y]);
          }
        }
      }
    } else {
#pragma unroll
      for (int s = 0; s < KS; ++s) {
        const int kc = s >> 1, c = (s & 1) * 4 + fg;
#pragma unroll
        for (int x = 0; x < MX; ++x) {
          const int r = wm * 16 * MX + x * 16 + fr;
          const bf16x8 fa = *reinterpret_cast<const bf16x8*>(A + (kc * PW_BM + r) * 128 + swz(r, c) * 16);
#pragma unroll
          for (int y = 0; y < WN; ++y) acc[x][y] = mfma_bf16x(fa, wf[y][s], acc[x][y]);
        }
      }
    }
    // every thread's reads of the image (store_tile above) are done. A raw barrier: __syncthreads()
    // would also wait for the DMA in flight (vmcnt(0))
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
#pragma unroll
    for (int x = 0; x < MX; ++x)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int rl = wm * 16 * MX + x * 16 + fg * 4 + r, m = phys(tile * PW_BM + rl);
        const bool ok = m >= 0;
        const int vj = (EPI & EPI_BIASV) && ok ? m % g.V : 0;
#pragma unroll
        for (int y = 0; y < WN; ++y) {
          const int jl = wj * 16 * WN + y * 16 + fr;
          float v = acc[x][y][r];
          if (EPI & EPI_BIAS) v += bias[y];
          if (EPI & EPI_BIASV) v += bv[vj * NT + jl];
          if (!ok) v = 0.f;
          if (EPI & EPI_STATS) {
            ssum[y] += v;
            ssq[y] += v * v;
          }
          if (ADD) reinterpret_cast<float*>(img)[rl * OTS + jl] = pre[x][r][y] + v;
          else if (F32O) reinterpret_cast<float*>(img)[rl * OTS + jl] = v;
          else reinterpret_cast<__bf16*>(img)[rl * OTS + jl] = (__bf16)v;
        }
      }
    // the next tile's block has landed (the NB - 2 after it stay in flight) and the image is written
    if (storer) pw_wait_vm<(NB - 2) * LPT, L::PIECES, NB - 2>(it);
    else pw_wait_vm<(NB - 2) * LPT, 0, 0>(it);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    if (ADD) preload(min(tile + 1, tile1 - 1));
  };
  body(tile0, std::true_type{});
  for (int tile = tile0 + 1; tile < tile1; ++tile) body(tile, std::false_type{});
  store_tile(tile1 - 1, std::false_type{});
  // ---- BN sums of the workgroup's tiles: lanes -> waves -> one fp64 add per column ----
  if (EPI & EPI_STATS) {
#pragma unroll
    for (int y = 0; y < WN; ++y) {
      ssum[y] += __shfl_xor(ssum[y], 16, 64);
      ssum[y] += __shfl_xor(ssum[y], 32, 64);
      ssq[y] += __shfl_xor(ssq[y], 16, 64);
      ssq[y] += __shfl_xor(ssq[y], 32, 64);
    }
    if (fg == 0) {
#pragma unroll
      for (int y = 0; y < WN; ++y) {
        red[(wm * 2 + 0) * NT + wj * 16 * WN + y * 16 + fr] = ssum[y];
        red[(wm * 2 + 1) * NT + wj * 16 * WN + y * 16 + fr] = ssq[y];
      }
    }
    __syncthreads();
    for (int t = tid; t < 2 * NT; t += PW_THREADS) {
      const int q = t / NT, j = t - q * NT;
      const float s = red[(0 * 2 + q) * NT + j] + red[(1 * 2 + q) * NT + j];
      atomic_add_d((q == 0 ? a.st_sum : a.st_sq) + j0 + j, (double)s);
    }
  }
  // drain the DMA of the tiles past the range (zero page) before the workgroup ends
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

}  // namespace f3

using namespace f3;

// Instantiated (EPI, KS, WN) combinations: the step's shapes (and a plain conv for the unit test).
#define F3_PW_TABLE(X)                                                                                \
  X(EPI_BIASV | EPI_STATS, 6, 1) X(EPI_BIASV | EPI_STATS, 6, 2)                                       \
  X(EPI_BIASV | EPI_STATS, 12, 2) X(EPI_BIASV | EPI_STATS, 24, 1)                                     \
  X(EPI_BIAS | EPI_STATS, 2, 2) X(EPI_BIAS | EPI_STATS, 4, 4)                                         \
  X(EPI_BIAS, 2, 3)                                                                                   \
  X(0, 2, 3) X(0, 4, 3) X(0, 4, 6) X(0, 6, 1) X(0, 8, 3) X(0, 8, 4)                                   \
  X(EPI_ADD, 4, 1) X(EPI_ADD, 8, 2)
// the bf16x3 native form (KS = 2 Kc / 32): the gcn forwards at K Cin = 192 (KS 12, graph-mixed bias +
// BN sums; at K Cin = 384 a 32-row A block is 48 KB and the ring would hold two), the gcn input
// gradients (C = 64 / 128 / 256), the residual forwards and the 64-channel residual input gradient
// (EPI_ADD), all with fp32 output rows
#define F3_PW_TABLE_X3N(X)                                                                            \
  X(EPI_BIASV | EPI_STATS, 12, 1) X(EPI_BIASV | EPI_STATS, 12, 2)                                     \
  X(0, 4, 3) X(0, 8, 3) X(0, 16, 2) X(EPI_BIAS | EPI_STATS, 4, 2) X(EPI_BIAS | EPI_STATS, 8, 2)      \
  X(EPI_ADD, 8, 1)

// mode 0: bf16, 2: bf16x3 native (x3n)
static bool pw_has(int epi, int ks, int wn, int mode) {
#define F3_PW_HAS(E, KSV, WNV) \
  if (epi == (E) && ks == (KSV) && wn == (WNV)) return true;
  if (mode == 2) {
    F3_PW_TABLE_X3N(F3_PW_HAS)
  } else {
    F3_PW_TABLE(F3_PW_HAS)
  }
#undef F3_PW_HAS
  return false;
}

static int pw_mode(const ConvGemmArgs& a) { return a.x3n ? 2 : 0; }
// 32-deep k slices of the weight panel (x3n: hi and lo of every 32-channel block)
static int pw_ks(const ConvGemmArgs& a) { return (a.x3n ? 2 : 1) * a.g.Kc / 32; }

// column-group width: the widest 64*WN that divides Nc, keeps the weight slice within 128 VGPRs
// per lane and is instantiated (0 = none)
static int pw_wn(const ConvGemmArgs& a, int epi) {
  const int ks = pw_ks(a);
  for (int wn : {6, 4, 3, 2, 1})
    if (a.g.Nc % (64 * wn) == 0 && wn * ks * 4 <= 128 && pw_has(epi, ks, wn, pw_mode(a))) return wn;
  return 0;
}

// (the bf16x3 mode's 1x1 GEMMs run on this kernel too: 9.89 -> 9.84 ms/step in three of three
// interleaved rounds against the tiled kernels, profiles/r04_pw_x3_ab.txt)

// Shapes this kernel takes: 1x1 (KT = 1, P = 0) convs over bf16 rows with Kc in {64, 128, 192, 256}
// and an instantiated column group; the forward at stride 1 or 2, the input gradient (transposed)
// at stride 1 or, accumulating (EPI_ADD), stride 2.
bool f3_pw_ok(const ConvGemmArgs& a, int epi) {
  const ConvGeom& g = a.g;
  // bf16x3: the native form (x3n); fp32 out
  const bool x3 = a.x3n;
  if (!a.inb || !a.wb || !a.zero) return false;
  if (a.x3n && (g.Kc % 32 || g.lda < 2 * g.Kc)) return false;
  if (g.KT != 1 || g.P != 0 || (!a.x3n && g.Kc % 64 != 0) || g.Nc % 64 != 0 || g.lda % 8 != 0) return false;
  if (!a.x3n && g.Kc > 256 && g.Kc != 384 && g.Kc != 768) return false;
  if (!pw_wn(a, epi)) return false;
  const bool add = epi == EPI_ADD;
  if ((add || x3) ? (!a.out || (!add && a.outb)) : !a.outb) return false;
  if (g.ldo % ((add || x3) ? 4 : 8) != 0) return false;
  // EPI_ADD is the stride-2 input gradient (accumulating into the even frames only); the others
  // are forwards or stride-1 input gradients
  if (add != (g.transposed && g.S == 2)) return false;
  if (add && (!igemm_parity(g) || g.M % (g.T_out * g.V) != 0)) return false;
  if ((epi & EPI_STATS) && (!a.st_sum || !a.st_sq)) return false;
  if ((epi & (EPI_BIAS | EPI_BIASV)) && !a.bias) return false;
  if ((epi & EPI_BIASV) && g.V > PW_VMAX) return false;
  return true;
}

constexpr int pw_bm(int ks) { return ks > 8 ? 32 : 64; }

template <int EPI, int KS, int WN, bool F32O = false, bool X3N = false>
static int pw_launch(const ConvGemmArgs& a, int grid, int ncg, int per_wg, hipStream_t s) {
  constexpr int BM = pw_bm(KS);
  constexpr int lds = PwLds<EPI, KS, WN, BM, F32O>::BYTES;
  F3_LDS_LIMIT((pw_gemm_kernel<EPI, KS, WN, BM, F32O, X3N>), lds);
  hipLaunchKernelGGL((pw_gemm_kernel<EPI, KS, WN, BM, F32O, X3N>), dim3(grid), dim3(PW_THREADS), lds, s, a, ncg,
                     per_wg);
  return F3_OK;
}

int f3_pw_gemm(const ConvGemmArgs* args, int epi, hipStream_t s) {
  const ConvGemmArgs& a = *args;
  const ConvGeom& g = a.g;
  static int cus = [] {
    int dev = 0, n = 256;
    if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev);
    (void)hipGetLastError();
    return n;
  }();
  const int mode = pw_mode(a);
  const int wn = pw_wn(a, epi), ks = pw_ks(a);
  if (!wn) return F3_EINVAL;
  const int ncg = g.Nc / (64 * wn);
  const bool par = epi == EPI_ADD;
  const int Mp = par ? (g.M / (g.T_out * g.V)) * ((g.T_out + 1) >> 1) * g.V : g.M;
  const int bm = pw_bm(ks);
  const int ntiles = (Mp + bm - 1) / bm;
  // one round over the CUs: contiguous ranges of tiles, one workgroup per (range, column group)
  const int nr0 = std::max(1, cus / ncg);
  const int per_wg = (ntiles + nr0 - 1) / nr0;
  const int nranges = (ntiles + per_wg - 1) / per_wg;
  const int grid = ncg * nranges;
#define F3_PW_LAUNCH(E, KSV, WNV)                                 \
  if (epi == (E) && ks == (KSV) && wn == (WNV)) {                 \
    F3_TRY((pw_launch<(E), KSV, WNV>(a, grid, ncg, per_wg, s)));   \
    F3_LAUNCH_CHECK();                                            \
    return F3_OK;                                                 \
  }
#define F3_PW_LAUNCH_X3N(E, KSV, WNV)                                          \
  if (epi == (E) && ks == (KSV) && wn == (WNV)) {                              \
    F3_TRY((pw_launch<(E), KSV, WNV, (E) != EPI_ADD, true>(a, grid, ncg, per_wg, s))); \
    F3_LAUNCH_CHECK();                                                         \
    return F3_OK;                                                              \
  }
  if (mode == 2) {
    F3_PW_TABLE_X3N(F3_PW_LAUNCH_X3N)
  } else {
    F3_PW_TABLE(F3_PW_LAUNCH)
  }
#undef F3_PW_LAUNCH_X3N
#undef F3_PW_LAUNCH
  return F3_EINVAL;
}
