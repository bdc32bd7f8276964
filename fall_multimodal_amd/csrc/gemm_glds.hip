// bf16 implicit-GEMM temporal convolution with bf16 activations in HBM, staged by LDS-DMA
// (global_load_lds_dwordx4) — the throughput form of conv_gemm for the bf16 mode.
//
//   Out[m][j] = sum_{dt,i} In[src(m,dt)][i] * W[j][dt*Kc+i]      (fwd, or dgrad via the
//                                                                  transposed row map)
// In (bf16, row stride lda) is the GEMM operand tensor its producer wrote in bf16 (the
// tcn input is the materialised relu(bn1(g)), so there is no prologue here). W is the
// prep-packed bf16 operand [Nc][KT*Kc]. Requirements: Kc % 64 == 0 (a 64-deep k step never
// straddles two taps), lda % 8 == 0.
//
// Tile 128 x BN (BN = 128 or 64) x 64, 4 waves in 2x2 (each 64 x BN/2 = 4 x BN/32 MFMA
// 16x16x32 tiles), two LDS stages. Each stage is filled by 1-KiB LDS-DMA wave-instructions
// (8 rows x 128 B); a row's 16-B chunks are stored XOR-swizzled (chunk c of row r at
// c ^ (r & 7), igemm.h swz) through the per-lane SOURCE address, which makes the 16-lane
// ds_read_b128 fragment reads conflict-free at any row shift. The implicit-GEMM row gather is also in the source address:
// a row outside the clip (temporal zero padding) or past M reads a zero line.
// Epilogues as conv_gemm_f32 (bias, graph-mixed bias, BN statistics, channel-attention
// pooling, ReLU mask + BN-backward sums, accumulate).
#include "igemm.h"
#include "layers.h"

#include <algorithm>

namespace f3 {

constexpr int G_BM = 128;

// WIN (stride-1 temporal convs, forward or input gradient): the 9 taps of a row tile read the
// same input rows shifted by whole frames, so instead of staging a 128-row A tile per (tap,
// 64-channel chunk) the tile's input WINDOW — its rows plus P frames either side — is staged
// once per chunk and each tap reads its fragments at a row offset of dt*V. Rows whose shifted
// frame leaves the clip (temporal zero padding) are zeroed in the fragment, per lane and tap.
// A staging traffic drops from 9 x 128 to (128 + 2PV) rows per chunk (the 64-channel layers
// staged 2x more A than B bytes).
constexpr int G_WIN_ROWS = 128 + 2 * 4 * 18;  // window capacity: P <= 4, V <= 18 (3 workgroups per CU)

// X3N: the bf16x3 native form (ConvGemmArgs::x3n; see igemm_big)
template <int EPI, int WN, int NST, bool WIN = false, bool X3N = false>
__global__ __launch_bounds__(256) void igemm_bf16(ConvGemmArgs a) {
  constexpr int BM = G_BM, BN = 32 * WN;
  constexpr int A_BYTES = WIN ? 0 : BM * G_BK * 2, B_BYTES = BN * G_BK * 2, STAGE = A_BYTES + B_BYTES;
  constexpr int A_INSTR = A_BYTES / 1024 / 4, B_INSTR = B_BYTES / 1024 / 4;  // per wave
  constexpr int NPS = A_INSTR + B_INSTR;  // LDS-DMA instructions per wave per stage
  constexpr int WIN_OFF = NST * STAGE, WIN_BYTES = WIN ? G_WIN_ROWS * 128 : 0;
  constexpr int SMEM_MAIN = WIN_OFF + WIN_BYTES > 16 * 1024 + BM * (BN + 8) * 2 ? WIN_OFF + WIN_BYTES
                                                                                 : 16 * 1024 + BM * (BN + 8) * 2;
  // ONE shared array (a second __shared__ object can de-pipeline LDS-DMA code): NST
  // stages (and the window), then the epilogue coefficient tables; the reductions reuse stage 0.
  __shared__ __attribute__((aligned(16))) char smem[SMEM_MAIN + 4 * BN * 4];
  float* epi_sc = reinterpret_cast<float*>(smem + SMEM_MAIN);
  float* epi_sh = epi_sc + BN;
  float* epi_mu = epi_sh + BN;
  float* epi_rs = epi_mu + BN;

  static_assert(!((EPI & EPI_ADD) && (EPI & (EPI_RELUMASK | EPI_BIASV))), "one preloaded epilogue operand");
  const ConvGeom& g = a.g;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int ntn = (g.Nc + BN - 1) / BN;
  int tile = xcd_remap(blockIdx.x, gridDim.x);
  // Stride-2 input gradient: an output row t only receives taps dt = t + P (mod 2), so the
  // rows are split by the parity p of t (tiles of parity 0 first) and a tile walks only its
  // parity's taps (5 or 4 of 9) instead of multiplying zero rows.
  const bool par = igemm_parity(g);
  int p = 0, Tp = g.T_out, Mp = g.M;
  if (par) {
    const int nclip = g.M / (g.T_out * g.V), T0 = (g.T_out + 1) >> 1;
    const int tiles0 = ((nclip * T0 * g.V + BM - 1) / BM) * ntn;
    Tp = T0;
    if (tile >= tiles0) { p = 1; tile -= tiles0; Tp = g.T_out >> 1; }
    Mp = nclip * Tp * g.V;
  }
  auto phys = [&](int r) -> int {  // logical row of this tile's parity class -> output row (-1: none)
    if (r >= Mp) return -1;
    if (!par) return r;
    const int nt = r / g.V, v = r - nt * g.V, n = nt / Tp, tt = nt - n * Tp;
    return (n * g.T_out + 2 * tt + p) * g.V + v;
  };
  const int m0 = (tile / ntn) * BM, j0 = (tile % ntn) * BN;
  constexpr int CB = X3N ? 32 : G_BK;             // channels per k step
  const int Ktot = g.KT * g.Kc * (X3N ? 2 : 1);   // packed weight row length
  const int kpt = g.Kc / CB;                      // k chunks per tap
  const int dt0 = par ? ((p + g.P) & 1) : 0;      // first tap of this parity
  const int nchunk = (par ? (g.KT - dt0 + 1) / 2 : g.KT) * kpt;
  auto wcol = [&](int dt, int i0) { return X3N ? dt * 2 * g.Kc + 2 * i0 : dt * g.Kc + i0; };
  auto acolx = [&](int i0, int cg) { return X3N ? x3n_col(g.Kc, i0, cg) : i0 + cg * 8; };
  // window mode: stage t = (chunk t / KT, tap t % KT); window row of tile row r for tap dt:
  // r + wofs(dt) with wofs = dt*V (forward) or (2P - dt)*V (input gradient)
  const int PV = g.P * g.V, WR = BM + 2 * PV;
  auto wofs = [&](int dt) { return (g.transposed ? 2 * g.P - dt : dt) * g.V; };
  const unsigned short* in = a.inb;
  const unsigned short* wb = a.wb;

  if (EPI & EPI_RELUMASK) {
    for (int t = tid; t < BN; t += 256) {
      if (j0 + t < g.Nc) {
        float sc, sh, mu, rs;
        bn_coeff(a.epi_bn, j0 + t, sc, sh, mu, rs);
        epi_sc[t] = sc; epi_sh[t] = sh; epi_mu[t] = mu; epi_rs[t] = rs;
      }
    }
  }

  // per-lane staging rows (fixed for the whole k loop)
  const int sub = lane >> 3, pch = lane & 7;
  RowMap a_map[A_INSTR > 0 ? A_INSTR : 1];
  int a_c[A_INSTR > 0 ? A_INSTR : 1];  // the lane's 16-B chunk of its staging row (swizzled)
#pragma unroll
  for (int i = 0; i < A_INSTR; ++i) {
    const int rr = (wave * A_INSTR + i) * 8 + sub;
    a_c[i] = swz(rr, pch);
    a_map[i] = rowmap(phys(m0 + rr), g);
  }
  const unsigned short* b_row[B_INSTR];
#pragma unroll
  for (int i = 0; i < B_INSTR; ++i) {
    const int rb = (wave * B_INSTR + i) * 8 + sub;
    const int j = j0 + rb;
    b_row[i] = j < g.Nc ? wb + (size_t)j * Ktot + swz(rb, pch) * 8 : a.zero;
  }
  const int b_step = 1;  // (kept for clarity: zero rows never advance)
  (void)b_step;

  auto stage = [&](int t, int buf) {
    int tap = t / kpt, i0 = (t - tap * kpt) * CB;
    if (WIN) { tap = t % g.KT; i0 = (t / g.KT) * CB; }
    const int dt = par ? dt0 + 2 * tap : tap;
    const int k0 = wcol(dt, i0);
    char* sa = smem + buf * STAGE;
#pragma unroll
    for (int i = 0; i < A_INSTR; ++i) {
      const int r = rowmap_src(a_map[i], dt, g);
      const unsigned short* src = r >= 0 ? in + (size_t)r * g.lda + acolx(i0, a_c[i]) : a.zero;
      __builtin_amdgcn_global_load_lds((const void*)src, (lds_void_t*)(sa + (wave * A_INSTR + i) * 1024), 16, 0, 0);
    }
    char* sb = sa + A_BYTES;
#pragma unroll
    for (int i = 0; i < B_INSTR; ++i) {
      const unsigned short* src = b_row[i] == a.zero ? a.zero : b_row[i] + k0;
      __builtin_amdgcn_global_load_lds((const void*)src, (lds_void_t*)(sb + (wave * B_INSTR + i) * 1024), 16, 0, 0);
    }
  };

  // window staging: 1-KiB pieces of 8 rows, dealt round-robin to the 4 waves (waited with vmcnt(0))
  auto load_win = [&](int chunk) {
    const int i0 = chunk * CB, nwp = (WR + 7) >> 3;
    for (int q = wave; q < nwp; q += 4) {
      const int rr = q * 8 + sub, gm = m0 - PV + rr;
      const bool ok = rr < WR && gm >= 0 && gm < g.M;
      const unsigned short* src = ok ? in + (size_t)gm * g.lda + acolx(i0, swz(rr, pch)) : a.zero;
      __builtin_amdgcn_global_load_lds((const void*)src, (lds_void_t*)(smem + WIN_OFF + q * 1024), 16, 0, 0);
    }
  };

  const int wm = wave >> 1, wj = wave & 1;
  const int fr = lane & 15, fg = lane >> 4;
  int tfr[4];  // window mode: frame of each of the lane's 4 A rows (the row's clip-relative t)
#pragma unroll
  for (int x = 0; x < 4; ++x) tfr[x] = WIN ? ((m0 + wm * 64 + x * 16 + fr) / g.V) % g.T_out : 0;
  f32x4 acc[4][WN];
#pragma unroll
  for (int x = 0; x < 4; ++x)
#pragma unroll
    for (int y = 0; y < WN; ++y) acc[x][y] = f32x4{0.f, 0.f, 0.f, 0.f};

  if (nchunk == 0) {
    // a parity class with no taps (odd rows of a 1x1 stride-2 input gradient): zero rows,
    // nothing to do at all when accumulating (uniform across the workgroup)
    if (EPI & EPI_ADD) return;
    __syncthreads();  // epilogue coefficient tables
  } else if (NST == 2) {
    if (WIN) load_win(0);
    stage(0, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  } else {  // NST == 3: two stages in flight; raw barriers keep the newest one in flight
    if (WIN) load_win(0);  // (older than both stages: the counted wait below covers it)
    stage(0, 0);
    if (nchunk > 1) {
      stage(1, 1);
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NPS) : "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __builtin_amdgcn_s_barrier();
  }
  for (int t = 0; t < nchunk; ++t) {
    const int buf = NST == 2 ? (t & 1) : (t % 3);
    if (WIN && t > 0 && t % g.KT == 0) {  // next 64-channel chunk: restage the window
      load_win(t / g.KT);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
    }
    const int wdt = WIN ? t % g.KT : 0;
    const int wo = WIN ? wofs(wdt) : 0;
    const int wsh = WIN ? (g.transposed ? g.P - wdt : wdt - g.P) : 0;
    if (NST == 2) {
      if (t + 1 < nchunk) stage(t + 1, buf ^ 1);
    } else {
      if (t + 2 < nchunk) stage(t + 2, (t + 2) % 3);
    }
    const char* sa = smem + buf * STAGE;
    const char* sb = sa + A_BYTES;
    // the A / B fragments of chunk c (16-B chunk index within the staged 128-B row)
    auto frag_a = [&](int x, int c) -> bf16x8 {
      if (WIN) {
        const int r = wm * 64 + x * 16 + fr + wo;
        const bf16x8 v = *reinterpret_cast<const bf16x8*>(smem + WIN_OFF + r * 128 + swz(r, c) * 16);
        const bool ok = (unsigned)(tfr[x] + wsh) < (unsigned)g.T_out;
        return ok ? v : bf16x8{};
      }
      const int r = wm * 64 + x * 16 + fr;
      return *reinterpret_cast<const bf16x8*>(sa + r * 128 + swz(r, c) * 16);
    };
    auto frag_b = [&](int y, int c) -> bf16x8 {
      const int r = wj * 16 * WN + y * 16 + fr;
      return *reinterpret_cast<const bf16x8*>(sb + r * 128 + swz(r, c) * 16);
    };
    if constexpr (X3N) {  // hi fragments (chunk fg), lo fragments (chunk 4 + fg), three products
      bf16x8 fah[4], fal[4], fbh[WN], fbl[WN];
#pragma unroll
      for (int x = 0; x < 4; ++x) {
        fah[x] = frag_a(x, fg);
        fal[x] = frag_a(x, 4 + fg);
      }
#pragma unroll
      for (int y = 0; y < WN; ++y) {
        fbh[y] = frag_b(y, fg);
        fbl[y] = frag_b(y, 4 + fg);
      }
#pragma unroll
      for (int x = 0; x < 4; ++x)
#pragma unroll
        for (int y = 0; y < WN; ++y) {
          acc[x][y] = mfma_bf16x(fah[x], fbh[y], acc[x][y]);
          acc[x][y] = mfma_bf16x(fal[x], fbh[y], acc[x][y]);
          acc[x][y] = mfma_bf16x(fah[x], fbl[y], acc[x][y]);
        }
    } else {
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        bf16x8 fa[4], fb[WN];
        const int c = ks * 4 + fg;
#pragma unroll
        for (int x = 0; x < 4; ++x) fa[x] = frag_a(x, c);
#pragma unroll
        for (int y = 0; y < WN; ++y) fb[y] = frag_b(y, c);
#pragma unroll
        for (int x = 0; x < 4; ++x)
#pragma unroll
          for (int y = 0; y < WN; ++y) acc[x][y] = mfma_bf16x(fa[x], fb[y], acc[x][y]);
      }
    }
    if (NST == 2) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
    } else {
      if (t + 2 < nchunk) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NPS) : "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
    }
  }
  if (NST != 2) __syncthreads();

  // ---------------- epilogue ----------------
  float* red = reinterpret_cast<float*>(smem);   // [2][2][BN]  (stage 0 is free now)
  float* gred = red + 4 * BN;                    // [2][2][BN]
  float ssum[WN], ssq[WN], gap0[WN], gap1[WN];
#pragma unroll
  for (int y = 0; y < WN; ++y) ssum[y] = ssq[y] = gap0[y] = gap1[y] = 0.f;
  // bf16 outputs leave through an LDS image of the tile: the MFMA C layout gives a lane 4 rows of
  // ONE column (2-B scattered stores); the image is copied out as 16-B row chunks instead
  constexpr int OTS = BN + 8, OT_OFF = 16 * 1024;  // row stride (elements), byte offset past red/gred
  static_assert(OT_OFF + BM * OTS * 2 <= (int)sizeof(smem), "output staging tile");
  const bool stage_out = !(EPI & EPI_ADD) && a.outb && g.ldo % 8 == 0 && g.Nc % 8 == 0;
  __bf16* ot = reinterpret_cast<__bf16*>(smem + OT_OFF);
  const int TV = g.T_out * g.V;
  const int nlo = m0 / TV;
  // Per 16-row group x, every operand the epilogue reads (RELUMASK source, graph-mixed bias, the
  // accumulated output) is loaded for the group's 4 rows x WN columns before any use, from
  // clamped in-bounds addresses (see igemm_big: a conditional per-element load costs a
  // vmcnt(0) round trip each).
  const bool aux16 = a.auxb != nullptr;
  float biasj[WN];  // EPI_BIAS: one value per column, loaded once
#pragma unroll
  for (int y = 0; y < WN; ++y) biasj[y] = (EPI & EPI_BIAS) ? a.bias[min(j0 + wj * 16 * WN + y * 16 + fr, g.Nc - 1)] : 0.f;
  // all groups' operands first: a load issued after the group's stores would make its first
  // use wait (vmcnt counts stores too) for every store before it
  float pre[4][4][WN];
  auto preload = [&](auto load) {
#pragma unroll
    for (int x = 0; x < 4; ++x)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int mc = max(phys(m0 + wm * 64 + x * 16 + fg * 4 + r), 0);
#pragma unroll
        for (int y = 0; y < WN; ++y) pre[x][r][y] = load(mc, min(j0 + wj * 16 * WN + y * 16 + fr, g.Nc - 1));
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
  for (int x = 0; x < 4; ++x) {
    int mrow[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) mrow[r] = phys(m0 + wm * 64 + x * 16 + fg * 4 + r);
#pragma unroll
    for (int y = 0; y < WN; ++y) {
      const int jl = wj * 16 * WN + y * 16 + fr;
      const int j = j0 + jl;
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
          if (stage_out) ot[(wm * 64 + x * 16 + fg * 4 + r) * OTS + jl] = (__bf16)v;
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
    for (int y = 0; y < WN; ++y) {
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
      for (int y = 0; y < WN; ++y) {
        const int jl = wj * 16 * WN + y * 16 + fr;
        red[(wm * 2 + 0) * BN + jl] = ssum[y];
        red[(wm * 2 + 1) * BN + jl] = ssq[y];
        gred[(wm * 2 + 0) * BN + jl] = gap0[y];
        gred[(wm * 2 + 1) * BN + jl] = gap1[y];
      }
    }
    __syncthreads();
    for (int t = tid; t < BN; t += 256) {
      const int j = j0 + t;
      if (j >= g.Nc) continue;
      if (EPI & (EPI_STATS | EPI_RELUMASK)) {
        atomic_add_d(a.st_sum + j, (double)(red[0 * BN + t] + red[2 * BN + t]));
        atomic_add_d(a.st_sq + j, (double)(red[1 * BN + t] + red[3 * BN + t]));
      }
      if (EPI & EPI_GAP) {
        const float s0 = gred[0 * BN + t] + gred[2 * BN + t];
        const float s1 = gred[1 * BN + t] + gred[3 * BN + t];
        atomic_add_f(a.gap + (size_t)nlo * g.Nc + j, s0);
        if ((nlo + 1) * TV < g.M && s1 != 0.f) atomic_add_f(a.gap + (size_t)(nlo + 1) * g.Nc + j, s1);
      }
    }
  }
  if (stage_out) {
    __syncthreads();
    constexpr int CPR = BN / 8;  // 16-B chunks per tile row
    for (int q = tid; q < BM * CPR; q += blockDim.x) {
      const int rl = q / CPR, c = q - rl * CPR;
      const int m = phys(m0 + rl), j = j0 + c * 8;
      if (m < 0 || j >= g.Nc) continue;
      *reinterpret_cast<uint4*>(reinterpret_cast<__bf16*>(a.outb) + (size_t)m * g.ldo + j) =
          *reinterpret_cast<const uint4*>(ot + rl * OTS + c * 8);
    }
  }
}

}  // namespace f3

using namespace f3;

bool f3_igemm_ok(const ConvGemmArgs& a) {
  if (!a.inb || !a.wb || !a.zero || a.g.lda % 8 != 0) return false;
  if (a.x3n) return a.g.Kc % 32 == 0 && a.g.lda >= 2 * a.g.Kc;
  return a.g.Kc % G_BK == 0;
}

// Window mode (see igemm_bf16): stride-1 temporal convs with "same" padding whose output
// channels fit one column tile (64 or 128) and whose window fits the LDS reserve.
static bool igemm_win_ok(const ConvGemmArgs& a, int epi) {
  const ConvGeom& g = a.g;
  if (g.S != 1 || g.KT < 2 || 2 * g.P != g.KT - 1 || g.T_in != g.T_out) return false;
  // 128 channels: only the input gradient (77 vs 87-111 us for igemm_big at layer 4; the
  // forward measured 77 vs 58 us, and within noise on the bf16x3 operands)
  if (g.Nc != 64 && !(g.Nc == 128 && epi == EPI_RELUMASK)) return false;
  if (G_BM + 2 * g.P * g.V > G_WIN_ROWS || g.M % (g.T_out * g.V) != 0) return false;
  return epi == (EPI_BIAS | EPI_STATS | EPI_GAP) || epi == EPI_RELUMASK || epi == EPI_BIAS;
}

template <int WN, int NST, bool WIN = false, bool X3N = false>
static int launch_igemm(const ConvGemmArgs& a, int epi, hipStream_t s) {
  const int ntn = (a.g.Nc + 32 * WN - 1) / (32 * WN);
  int tiles = ((a.g.M + G_BM - 1) / G_BM) * ntn;
  if (igemm_parity(a.g)) {  // parity-split rows (see igemm_bf16)
    if (a.g.M % (a.g.T_out * a.g.V) != 0 || (epi & (EPI_GAP | EPI_BIASV))) return F3_EINVAL;
    const int nclip = a.g.M / (a.g.T_out * a.g.V);
    const int M0 = nclip * ((a.g.T_out + 1) >> 1) * a.g.V, M1 = nclip * (a.g.T_out >> 1) * a.g.V;
    tiles = ((M0 + G_BM - 1) / G_BM + (M1 + G_BM - 1) / G_BM) * ntn;
  }
#define F3_ICASE(E)                                                                   \
  if (epi == (E)) {                                                                  \
    hipLaunchKernelGGL((igemm_bf16<(E), WN, NST, WIN, X3N>), dim3(tiles), dim3(256), 0, s, a); \
    F3_LAUNCH_CHECK();                                                                \
    return F3_OK;                                                                     \
  }
  F3_ICASE(EPI_BIASV | EPI_STATS)            // gcn forward
  F3_ICASE(EPI_BIAS | EPI_STATS | EPI_GAP)   // tcn forward
  F3_ICASE(EPI_BIAS | EPI_STATS)             // residual forward
  F3_ICASE(EPI_RELUMASK)                     // tcn dgrad
  F3_ICASE(0)                                // gcn dgrad
  F3_ICASE(EPI_ADD)                          // residual dgrad
  F3_ICASE(EPI_BIAS)                         // plain conv (tests)
#undef F3_ICASE
  return F3_EINVAL;
}

int f3_igemm_bf16(const ConvGemmArgs* args, int epi, hipStream_t s) {
  const ConvGemmArgs& a = *args;
  if (a.g.M <= 0 || a.g.Nc <= 0) return F3_OK;
  if (!f3_igemm_ok(a)) return F3_EINVAL;
  if (f3_tcn64_ok(a, epi)) return f3_tcn64(args, epi, s);
  if (f3_pw_ok(a, epi)) return f3_pw_gemm(args, epi, s);
  // the clip-window form of igemm_big where it applies (whole clips per workgroup: 9-tap convs of
  // 64 channels at T*V <= 540, of 128 / 256 channels at T*V <= 270)
  if (f3_igemm_big_win_ok(a)) {
    const int r = f3_igemm_big(args, epi, s);
    if (r != F3_EINVAL) return r;
  }
  // two LDS stages (three measured slower for both the windows and the tiles)
  if (igemm_win_ok(a, epi)) {
    if (a.x3n) return a.g.Nc == 128 ? launch_igemm<4, 2, true, true>(a, epi, s) : launch_igemm<2, 2, true, true>(a, epi, s);
    return a.g.Nc == 128 ? launch_igemm<4, 2, true>(a, epi, s) : launch_igemm<2, 2, true>(a, epi, s);
  }
  if (f3_igemm_big_ok(a)) return f3_igemm_big(args, epi, s);
  // 128-wide column tiles unless they would leave a partial tile (Nc = 192: the gcn input
  // gradient of the 64-channel layers, where a second 128-wide tile is half empty)
  const bool wide = a.g.Nc > 64 && a.g.Nc % 128 == 0;
  if (a.x3n) return wide ? launch_igemm<4, 2, false, true>(a, epi, s) : launch_igemm<2, 2, false, true>(a, epi, s);
  return wide ? launch_igemm<4, 2>(a, epi, s) : launch_igemm<2, 2>(a, epi, s);
}

// ============================================================================
// Weight gradient, bf16 operands by LDS-DMA:
//   dW[j][dt*Kc+i] += sum_m dY[m][j] * In[src(m,dt)][i]
// GEMM over k = rows m (64 per stage): both tiles are staged row-major [64 m][128 cols]
// (1-KiB DMA pieces = 4 rows of 256 B, or 8 rows of 128 B for 64-wide tiles) and read as
// MFMA operands with the gfx950 transposed LDS read ds_read_b64_tr_b16. 32-B units of a row
// are XOR-swizzled (unit u of row r at u ^ f(r)) through the source address so each
// half-wave tr read (8 rows x 32 B) covers all 64 banks once.
// Output: WG_OUT_GCN -> the reference gcn layout directly; WG_OUT_CONV -> a packed
// [Nc][KT*Kc] accumulator (contiguous i for the atomics) that f3_unpack_conv_grad moves
// into the reference [Nc][Kc][KT] layout.
// ============================================================================
typedef short s16x4_t __attribute__((ext_vector_type(4)));
typedef short s16x8_t __attribute__((ext_vector_type(8)));

template <int U>
F3_DEV int wswz(int r) {  // unit permutation of row r (U 32-B units per row)
  if (U >= 8) return (r & 3) | (((r >> 3) & 1) << 2);  // 8 or 16 units
  return ((r >> 1) & 1) | (((r >> 3) & 1) << 1);
}

// Transposed LDS read issued from inline asm. The builtin (__builtin_amdgcn_ds_read_tr16_b64)
// carries no memory operand, so hipcc (ROCm 7.2) cannot tell it from a read of the LDS-DMA
// destination and waits vmcnt(0) before the first one of every stage: the stage just issued
// must land before the current one is consumed, which de-pipelines the ring (measured: the
// layer-6 wgrad spent 46 of 89 us in that wait). The asm read is invisible to the compiler's
// counters, so the caller waits lgkmcnt(0) itself (tr_wait) before using the results; the
// results pass through that asm so nothing can read them earlier.
typedef __attribute__((address_space(3))) const char lds_cchar_t;
F3_DEV s16x4_t tr_issue(const char* p) {
  s16x4_t r;
  const unsigned addr = (unsigned)(size_t)(lds_cchar_t*)p;
  asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(r) : "v"(addr));
  return r;
}
template <int NF>
F3_DEV void tr_wait(s16x4_t (&lo)[NF], s16x4_t (&hi)[NF]) {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
  for (int i = 0; i < NF; ++i) asm volatile("" : "+v"(lo[i]), "+v"(hi[i]));
}
F3_DEV bf16x8 tr_join(s16x4_t lo, s16x4_t hi) {
  s16x8_t v;
#pragma unroll
  for (int e = 0; e < 4; ++e) { v[e] = lo[e]; v[4 + e] = hi[e]; }
  return __builtin_bit_cast(bf16x8, v);
}

template <int TJ, int TI>  // tile widths: 128 or 64
__global__ __launch_bounds__(256) void wgrad_glds_bf16(WgradArgs a) {
  constexpr int UJ = TJ / 16, UI = TI / 16;         // 32-B units per row
  constexpr int Y_BYTES = 64 * TJ * 2, X_BYTES = 64 * TI * 2, STAGE = Y_BYTES + X_BYTES;
  constexpr int Y_INSTR = Y_BYTES / 1024 / 4, X_INSTR = X_BYTES / 1024 / 4;
  constexpr int YRPI = 1024 / (TJ * 2), XRPI = 1024 / (TI * 2);  // rows per DMA piece
  constexpr int WJ = TJ / 32, WI = TI / 32;          // MFMA tiles per wave (2x2 waves)
  __shared__ __attribute__((aligned(16))) char smem[2 * STAGE + TJ * 4];
  float* dbs = reinterpret_cast<float*>(smem + 2 * STAGE);   // [TJ]
  const ConvGeom& g = a.g;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  // xcd: 1-D grid, XCD-aware: the gx*gy workgroups of one row split (they all read that
  // split's dY and input rows) get consecutive logical ids, which xcd_remap keeps on one XCD,
  // so the split's rows come from HBM once and are re-read from that XCD's L2.
  const int itiles = (g.Kc + TI - 1) / TI;
  int bz = blockIdx.z, by = blockIdx.y, bx = blockIdx.x;
  if (a.xcd) {
    const int gx = (g.Nc + TJ - 1) / TJ, gy = g.KT * itiles;
    const int lin = xcd_remap(blockIdx.x, gridDim.x);
    bz = lin / (gx * gy);
    const int rem = lin - bz * gx * gy;
    by = rem / gx;
    bx = rem - by * gx;
  }
  const int j0 = bx * TJ;
  const int dt = by / itiles;
  const int i0 = (by - dt * itiles) * TI;
  const int r_begin = bz * a.rows_per_split;
  const int r_end = min(g.M, r_begin + a.rows_per_split);
  const bool do_db = a.db && by == 0;
  const __bf16* dyb = reinterpret_cast<const __bf16*>(a.dyb);
  const __bf16* xb = reinterpret_cast<const __bf16*>(a.inb);
  const __bf16* zero = reinterpret_cast<const __bf16*>(a.zero);

  // staging lanes: piece rows and the logical column each lane fetches
  const int ysub = lane / (TJ / 8), yph = lane % (TJ / 8);   // 16-B chunk index within the row
  const int xsub = lane / (TI / 8), xph = lane % (TI / 8);
  auto stage = [&](int r0, int buf) {
    char* sy = smem + buf * STAGE;
#pragma unroll
    for (int i = 0; i < Y_INSTR; ++i) {
      const int rr = (wave * Y_INSTR + i) * YRPI + ysub;
      const int m = r0 + rr;
      const int lu = (yph >> 1) ^ wswz<UJ>(rr);
      const int col = (lu * 2 + (yph & 1)) * 8;
      const __bf16* src = (m < r_end && j0 + col < g.Nc) ? dyb + (size_t)m * a.ldy + j0 + col : zero;
      __builtin_amdgcn_global_load_lds((const void*)src, (lds_void_t*)(sy + (wave * Y_INSTR + i) * 1024), 16, 0, 0);
    }
    char* sx = sy + Y_BYTES;
#pragma unroll
    for (int i = 0; i < X_INSTR; ++i) {
      const int rr = (wave * X_INSTR + i) * XRPI + xsub;
      const int m = r0 + rr;
      const int lu = (xph >> 1) ^ wswz<UI>(rr);
      const int col = (lu * 2 + (xph & 1)) * 8;
      int r = -1;
      if (m < r_end && i0 + col < g.Kc) {
        const int nt = m / g.V, v = m - nt * g.V, n = nt / g.T_out, t = nt - n * g.T_out;
        r = g_src_row(n, t, v, dt, g);
      }
      const __bf16* src = r >= 0 ? xb + (size_t)r * g.lda + i0 + col : zero;
      __builtin_amdgcn_global_load_lds((const void*)src, (lds_void_t*)(sx + (wave * X_INSTR + i) * 1024), 16, 0, 0);
    }
  };

  const int wm = wave >> 1, wn = wave & 1;
  const int fr = lane & 15, fg = lane >> 4, tq = fr >> 2, tp = fr & 3;
  // transposed fragment of a [64][cols] tile: lane (fg, fr) gets column c0+fr of rows
  // kb+8fg .. kb+8fg+7 (kb = 0 or 32)
  auto tr_frag = [&](const char* tile, int U, int c0, int kb, s16x4_t& lo, s16x4_t& hi) {
    const int r_lo = kb + 8 * fg + tq, r_hi = r_lo + 4;
    const int u = c0 >> 4;
    const int R = U * 32;
    const int f_lo = U == 8 ? wswz<8>(r_lo) : wswz<4>(r_lo);
    const int f_hi = U == 8 ? wswz<8>(r_hi) : wswz<4>(r_hi);
    lo = tr_issue(tile + r_lo * R + ((u ^ f_lo) * 32) + tp * 8);
    hi = tr_issue(tile + r_hi * R + ((u ^ f_hi) * 32) + tp * 8);
  };

  f32x4 acc[WJ][WI];
#pragma unroll
  for (int x = 0; x < WJ; ++x)
#pragma unroll
    for (int y = 0; y < WI; ++y) acc[x][y] = f32x4{0.f, 0.f, 0.f, 0.f};
  float dbp[WJ];
#pragma unroll
  for (int x = 0; x < WJ; ++x) dbp[x] = 0.f;

  const int nst = r_end > r_begin ? (r_end - r_begin + 63) / 64 : 0;
  if (nst > 0) {
    stage(r_begin, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }
  for (int t = 0; t < nst; ++t) {
    const int buf = t & 1;
    if (t + 1 < nst) stage(r_begin + (t + 1) * 64, buf ^ 1);
    const char* sy = smem + buf * STAGE;
    const char* sx = sy + Y_BYTES;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      bf16x8 fa[WJ], fb[WI];
      s16x4_t lo[WJ + WI], hi[WJ + WI];
#pragma unroll
      for (int x = 0; x < WJ; ++x) tr_frag(sy, UJ, wm * 16 * WJ + x * 16, ks * 32, lo[x], hi[x]);
#pragma unroll
      for (int y = 0; y < WI; ++y) tr_frag(sx, UI, wn * 16 * WI + y * 16, ks * 32, lo[WJ + y], hi[WJ + y]);
      tr_wait(lo, hi);
#pragma unroll
      for (int x = 0; x < WJ; ++x) fa[x] = tr_join(lo[x], hi[x]);
#pragma unroll
      for (int y = 0; y < WI; ++y) fb[y] = tr_join(lo[WJ + y], hi[WJ + y]);
      if (do_db && wn == 0) {
#pragma unroll
        for (int x = 0; x < WJ; ++x)
#pragma unroll
          for (int e = 0; e < 8; ++e) dbp[x] += (float)fa[x][e];
      }
#pragma unroll
      for (int x = 0; x < WJ; ++x)
#pragma unroll
        for (int y = 0; y < WI; ++y) acc[x][y] = mfma_bf16x(fa[x], fb[y], acc[x][y]);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }
  if (do_db) {
    // lane (fg, fr) holds column wm*16*WJ + x*16 + fr summed over its rows; add the 4 fg groups
#pragma unroll
    for (int x = 0; x < WJ; ++x) {
      dbp[x] += __shfl_xor(dbp[x], 16, 64);
      dbp[x] += __shfl_xor(dbp[x], 32, 64);
    }
    if (wn == 0 && fg == 0) {
#pragma unroll
      for (int x = 0; x < WJ; ++x) dbs[wm * 16 * WJ + x * 16 + fr] = dbp[x];
    }
    __syncthreads();
    for (int t = tid; t < TJ; t += 256) {
      if (j0 + t >= g.Nc) continue;
      if (a.dbpart) a.dbpart[(size_t)bz * g.Nc + j0 + t] = nst > 0 ? dbs[t] : 0.f;  // every (split, j) once
      else if (nst > 0) atomic_add_f(a.db + j0 + t, dbs[t]);
    }
  }
  const bool to_slab = a.slab != nullptr && a.outmap == WG_OUT_CONV;
  if (nst == 0 && !to_slab) return;  // (a slab tile is written even when empty: it is summed)
  float* slab = to_slab ? a.slab + (size_t)bz * g.Nc * g.KT * g.Kc : nullptr;
#pragma unroll
  for (int x = 0; x < WJ; ++x) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int j = j0 + wm * 16 * WJ + x * 16 + fg * 4 + r;
      if (j >= g.Nc) continue;
#pragma unroll
      for (int y = 0; y < WI; ++y) {
        const int i = i0 + wn * 16 * WI + y * 16 + fr;
        if (i >= g.Kc) continue;
        size_t idx;
        if (a.outmap == WG_OUT_GCN) {
          const int k = i / a.gcn_cin, ci = i - k * a.gcn_cin;
          idx = ((size_t)k * g.Nc + j) * a.gcn_cin + ci;
        } else {  // packed [Nc][KT*Kc]
          idx = (size_t)j * g.KT * g.Kc + (size_t)dt * g.Kc + i;
        }
        if (to_slab) slab[idx] = acc[x][y][r];
        else atomic_add_f(a.dw + idx, acc[x][y][r]);
      }
    }
  }
}

// The bias-gradient partial rows of a weight-gradient launch (WgradArgs::dbpart, one row of Nc per
// split) summed by the first ceil(Nc / 64) workgroups of its slab reduce (no separate launch):
// db[c] += sum_s dbpart[s][c], waves 0-3 over interleaved splits, combined in wave order.
F3_DEV void wgrad_bias_block(const float* __restrict__ dbpart, int splits, int Nc, float* __restrict__ db, int blk,
                             float (*part)[64]) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, c = blk * 64 + lane;
  float acc = 0.f;
  if (wave < 4 && c < Nc)
    for (int sp = wave; sp < splits; sp += 4) acc += dbpart[(size_t)sp * Nc + c];
  if (wave < 4) part[wave][lane] = acc;
  __syncthreads();
  if (wave == 0 && c < Nc) db[c] += ((part[0][lane] + part[1][lane]) + part[2][lane]) + part[3][lane];
}

// dw_ref[j][i][dt] += sum_s slab[s][j][dt*Kc + i]. A workgroup owns 64 consecutive slab
// elements (one (j, dt) row piece, Kc % 64 == 0); its 4 waves sum interleaved split subsets
// (coalesced 256-B reads, independent loads) and combine through LDS. With dbpart, the first
// nbias = ceil(Nc / 64) workgroups sum the bias rows instead (wgrad_bias_block).
__global__ __launch_bounds__(256) void wgrad_slab_reduce_kernel(const float* __restrict__ slab, int splits, int Nc,
                                                                int Kc, int KT, float* __restrict__ dw_ref,
                                                                int gcn_cin, const float* __restrict__ dbpart,
                                                                float* __restrict__ db) {
  __shared__ float part[4][64];
  const int nbias = dbpart ? (Nc + 63) / 64 : 0;
  if ((int)blockIdx.x < nbias) {
    wgrad_bias_block(dbpart, splits, Nc, db, blockIdx.x, part);
    return;
  }
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const size_t e = (size_t)(blockIdx.x - nbias) * 64 + lane;  // slab element (j, dt, i)
  const size_t stride = (size_t)Nc * KT * Kc;
  float acc0 = 0.f, acc1 = 0.f;
  int sp = wave;
  for (; sp + 4 < splits; sp += 8) {
    acc0 += slab[(size_t)sp * stride + e];
    acc1 += slab[(size_t)(sp + 4) * stride + e];
  }
  if (sp < splits) acc0 += slab[(size_t)sp * stride + e];
  part[wave][lane] = acc0 + acc1;
  __syncthreads();
  if (wave == 0) {
    const float v = part[0][lane] + part[1][lane] + part[2][lane] + part[3][lane];
    const int j = (int)(e / ((size_t)KT * Kc)), r = (int)(e - (size_t)j * KT * Kc), dt = r / Kc, i = r - dt * Kc;
    if (gcn_cin > 0) {  // gcn reference layout [K*Nc][gcn_cin] (KT = 1, i = k gcn_cin + ci)
      const int k = i / gcn_cin, ci = i - k * gcn_cin;
      dw_ref[((size_t)k * Nc + j) * gcn_cin + ci] += v;
    } else {
      dw_ref[((size_t)j * Kc + i) * KT + dt] += v;
    }
  }
}

// ----------------------------------------------------------------------------
// wgrad_big: the same weight-gradient GEMM for the 128/256-channel layers with 8 waves
// (512 threads, one workgroup per CU), a 3-stage LDS-DMA ring behind a counted vmcnt and raw
// s_barrier (the igemm_big structure: two 64-row stages stay in flight while the third is
// consumed), and tiles of TJ x TI = (WJW*16*MJ) x (WIW*16*MI). Staging pieces: 1-KiB DMA
// instructions, piece q = i*8 + wave (dY pieces first), so every wave issues the same count
// per stage and one vmcnt constant serves all. 32-B units are swizzled as in wgrad_glds_bf16
// (rows of 16 units use the 8-unit permutation: the half-wave tr read still covers 64 banks).
//
// The loop is kept lean in VALU work — at 2 waves per SIMD the per-stage address arithmetic,
// not the MFMA or the memory, bounded the first version (a loop with the loads and MFMAs
// removed still took half the time): every lane's LDS fragment offsets are fixed for the
// whole loop (the tr reads of a fragment differ only by immediates: +4 rows, +32 rows), and
// each staging lane walks its (clip, frame, joint) row coordinates incrementally instead of
// dividing by V and T per stage. Forward-geometry rows only (g.transposed == 0).
//
// NTW > 1 (tap groups): a workgroup computes NTW consecutive taps dt0 .. dt0 + NTW - 1 of its
// (j, i) tile from ONE staged copy of the dY rows — the input rows of each tap are staged into
// their own region — so the dY bytes staged per MFMA and the A-fragment LDS reads per MFMA
// drop by NTW (each wave holds NTW x MJ x MI accumulators). Taps past KT (the last group when
// NTW does not divide KT) are staged from the zero page and their MFMAs skipped.
// ----------------------------------------------------------------------------
// X3F (bf16x3, the three row segments fused): the staged rows carry both halves of the operands,
// [dY_hi (TJ) | dY_lo (TJ)] and [X_hi (TI) | X_lo (TI)], and the wave issues the split product's three
// MFMAs dY_hi X_hi + dY_lo X_hi + dY_hi X_lo per fragment set: one staging for all three terms instead
// of one per row segment (x3seg), 2/3 of the staged bytes per MFMA with the tap groups on top.
template <int WJW, int WIW, int MJ, int MI, int BK = 64, int NTW = 1, int NSTG = 3, bool X3F = false>
__global__ __launch_bounds__(WJW * WIW * 64) void wgrad_big(WgradArgs a_) {
  constexpr int NW = WJW * WIW;  // waves: 8 (one workgroup per CU) or 4 (the 64-wide tiles)
  constexpr int TJ = WJW * 16 * MJ, TI = WIW * 16 * MI;      // output tile
  constexpr int HS = X3F ? 2 : 1;                             // staged halves (hi | lo)
  constexpr int UJ = HS * TJ / 16, UI = HS * TI / 16;         // 32-B units per staged row
  constexpr int RJ = HS * TJ * 2, RI = HS * TI * 2;  // row bytes of the dY / input tiles
  constexpr int NKS = BK / 32;             // 32-deep MFMA k steps per stage
  constexpr int Y_BYTES = BK * RJ, X_BYTES = BK * RI, STAGE = Y_BYTES + NTW * X_BYTES;
  constexpr int YPW = Y_BYTES / 1024 / NW, XPW = X_BYTES / 1024 / NW, PPW = YPW + NTW * XPW;  // pieces per wave
  constexpr int YRPI = 1024 / RJ, XRPI = 1024 / RI;  // rows per piece
  constexpr int NST = NSTG;  // LDS stages in the ring (NST - 1 in flight)
  constexpr int NB = NTW * MI;  // B fragments per k step (all taps)
  static_assert(BK == 32 || BK == 64, "stage depth");
  static_assert(NTW >= 1 && NTW <= 3 && (NST - 1) * PPW < 64, "tap group");
  static_assert(NST == 3 || NST == 4, "ring depth");
  static_assert((NW == 8 || NW == 4) && YPW * NW * 1024 == Y_BYTES && XPW * NW * 1024 == X_BYTES, "whole pieces");
  static_assert(UJ >= 4 && UI >= 4, "64-column tiles at least");
  static_assert(NST * STAGE + TJ * 4 <= 160 * 1024, "LDS");
  static_assert(32 * RJ + 4 * RJ < 65536 && 32 * RI + 4 * RI < 65536, "ds offset immediates");
  __shared__ __attribute__((aligned(16))) char smem[NST * STAGE + TJ * 4];
  float* dbs = reinterpret_cast<float*>(smem + NST * STAGE);  // [TJ]
  const ConvGeom& g = a_.g;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int itiles = (g.Kc + TI - 1) / TI;
  const int gx = (g.Nc + TJ - 1) / TJ, gy = ((g.KT + NTW - 1) / NTW) * itiles;
  int lin = xcd_remap(blockIdx.x, gridDim.x);  // a row split's tiles stay on one XCD
  WgradArgs a = a_;
  if (a_.groups > 1) {  // grouped launch: problem-major over the 1-D grid
    const int per = gridDim.x / a_.groups;
    wgrad_group(a, lin / per);
    lin %= per;
  }
  const int bz = lin / (gx * gy);
  const int rem = lin - bz * gx * gy;
  const int by = rem / gx, bx = rem - by * gx;
  const int j0 = bx * TJ;
  const int grp = by / itiles, dt0 = grp * NTW;  // taps dt0 .. dt0 + NTW - 1
  const int i0 = (by - grp * itiles) * TI;
  // bf16x3 row segments (x3seg): split bz = row range bz / 3, segment seg = bz % 3, whose
  // operands sit at column offsets (0, 0) hi x hi, (Nc, 0) lo x hi, (0, Kc) hi x lo of the rows
  const int seg = (a.x3seg && !X3F) ? bz % 3 : 0;
  const int r_begin = ((a.x3seg && !X3F) ? bz / 3 : bz) * a.rows_per_split;
  const int r_end = min(g.M, r_begin + a.rows_per_split);
  const bool do_db = a.db && by == 0 && seg < 2;
  const __bf16* dyb = reinterpret_cast<const __bf16*>(a.dyb) + (seg == 1 ? g.Nc : 0);
  const __bf16* xb = reinterpret_cast<const __bf16*>(a.inb) + (seg == 2 ? g.Kc : 0);
  const __bf16* zero = reinterpret_cast<const __bf16*>(a.zero);
  const unsigned lds0 = (unsigned)(size_t)(lds_cchar_t*)smem;

  // ---- staging lanes: fixed column, rows walked 64 at a time ----
  const int ysub = lane / (HS * TJ / 8), yph = lane % (HS * TJ / 8);
  const int xsub = lane / (HS * TI / 8), xph = lane % (HS * TI / 8);
  // X3F: staged unit u < U/2 is the hi half's column j0 + 16 u, else the lo half's (offset Nc / Kc)
  int ycol[YPW], yrow[YPW];
  bool yok[YPW];
#pragma unroll
  for (int i = 0; i < YPW; ++i) {
    const int rr = (i * NW + wave) * YRPI + ysub;
    yrow[i] = r_begin + rr;
    const int u = (yph >> 1) ^ wswz<UJ>(rr), lo = X3F && u >= UJ / 2;
    const int cl = j0 + (lo ? u - UJ / 2 : u) * 16 + (yph & 1) * 8;  // logical column
    yok[i] = cl < g.Nc;
    ycol[i] = cl + (lo ? g.Nc : 0);
  }
  // input rows: m = (n*T_out + t)*V + v -> source (n*T_in + t*S + dt - P)*V + v
  const int dv = BK % g.V, dnt = BK / g.V;
  int xm[XPW], xv[XPW], xt[XPW], xn[XPW], xcol[XPW];
  bool xok[XPW];
#pragma unroll
  for (int i = 0; i < XPW; ++i) {
    const int rr = (i * NW + wave) * XRPI + xsub;
    const int m = r_begin + rr;
    xm[i] = m;
    const int nt = m / g.V;
    xv[i] = m - nt * g.V;
    xn[i] = nt / g.T_out;
    xt[i] = nt - xn[i] * g.T_out;
    const int u = (xph >> 1) ^ wswz<UI>(rr), lo = X3F && u >= UI / 2;
    const int cl = i0 + (lo ? u - UI / 2 : u) * 16 + (xph & 1) * 8;
    xok[i] = cl < g.Kc;
    xcol[i] = cl + (lo ? g.Kc : 0);
  }
  const int tshift = dt0 - g.P;
  const int ntap = min(NTW, g.KT - dt0);  // valid taps of this group
  auto stage = [&](int buf) {  // issue the next BK rows of every staging lane, then advance them
    const unsigned sy = lds0 + buf * STAGE;
#pragma unroll
    for (int i = 0; i < YPW; ++i) {
      const __bf16* src = (yrow[i] < r_end && yok[i]) ? dyb + (size_t)yrow[i] * a.ldy + ycol[i] : zero;
      __builtin_amdgcn_global_load_lds((const void*)src,
                                       (lds_void_t*)(size_t)(sy + (i * NW + wave) * 1024), 16, 0, 0);
      yrow[i] += BK;
    }
    const unsigned sx = sy + Y_BYTES;
#pragma unroll
    for (int i = 0; i < XPW; ++i) {
      const int tb = xt[i] * g.S + tshift;
      const bool okr = xm[i] < r_end && xok[i];
      const long long rb = (long long)(xn[i] * g.T_in + tb) * g.V + xv[i];
#pragma unroll
      for (int tt = 0; tt < NTW; ++tt) {  // tap dt0 + tt: input frame tb + tt (rows V apart)
        const int ti = tb + tt;
        const bool ok = okr && tt < ntap && ti >= 0 && ti < g.T_in;
        const __bf16* src = ok ? xb + (size_t)(rb + (long long)tt * g.V) * g.lda + xcol[i] : zero;
        __builtin_amdgcn_global_load_lds((const void*)src,
                                         (lds_void_t*)(size_t)(sx + tt * X_BYTES + (i * NW + wave) * 1024), 16, 0, 0);
      }
      xm[i] += BK;
      xv[i] += dv;
      xt[i] += dnt;
      if (xv[i] >= g.V) { xv[i] -= g.V; xt[i] += 1; }
      while (xt[i] >= g.T_out) { xt[i] -= g.T_out; xn[i] += 1; }
    }
  };

  // ---- fragment lanes: fixed LDS offsets ----
  const int wj = wave / WIW, wi = wave % WIW;
  const int fr = lane & 15, fg = lane >> 4, tq = fr >> 2, tp = fr & 3;
  const int r0 = 8 * fg + tq;                 // rows r0, r0+4 (lo/hi), +32 for the second k half
  const int fj = wswz<UJ>(r0), fi = wswz<UI>(r0);  // unchanged at r0 + 4, r0 + 32, r0 + 36
  // fragment h of tile x: X3F h = 0 the hi half, 1 the lo half (units U/2 further)
  constexpr int NH = HS;
  unsigned offa[NH][MJ], offb[NH][NB];
#pragma unroll
  for (int h = 0; h < NH; ++h) {
#pragma unroll
    for (int x = 0; x < MJ; ++x) offa[h][x] = r0 * RJ + (((h * UJ / 2 + wj * MJ + x) ^ fj) * 32) + tp * 8;
#pragma unroll
    for (int tt = 0; tt < NTW; ++tt)
#pragma unroll
      for (int y = 0; y < MI; ++y)
        offb[h][tt * MI + y] = Y_BYTES + tt * X_BYTES + r0 * RI + (((h * UI / 2 + wi * MI + y) ^ fi) * 32) + tp * 8;
  }

  f32x4 acc[MJ][NB];
#pragma unroll
  for (int x = 0; x < MJ; ++x)
#pragma unroll
    for (int y = 0; y < NB; ++y) acc[x][y] = f32x4{0.f, 0.f, 0.f, 0.f};
  float dbp[MJ];
#pragma unroll
  for (int x = 0; x < MJ; ++x) dbp[x] = 0.f;

  const int nst = r_end > r_begin ? (r_end - r_begin + BK - 1) / BK : 0;
  if (nst > 0) {
    stage(0);
    if (NST == 4 && nst > 2) {
      stage(1);
      stage(2);
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * PPW) : "memory");
    } else if (nst > 1) {
      stage(1);
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(PPW) : "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __builtin_amdgcn_s_barrier();
  }
  for (int t = 0; t < nst; ++t) {
    const int buf = t % NST;
    if (t + NST - 1 < nst) stage((t + NST - 1) % NST);
    const unsigned base = lds0 + buf * STAGE;
#pragma unroll
    for (int ks = 0; ks < NKS; ++ks) {
      // rows r0 / r0 + 4 of the fragment's 8 (lo / hi of the transposed read), + 32 for k step 1
      s16x4_t lo[NH * (MJ + NB)], hi[NH * (MJ + NB)];
#pragma unroll
      for (int h = 0; h < NH; ++h) {
#pragma unroll
        for (int x = 0; x < MJ; ++x) {
          const unsigned p = base + offa[h][x];
          const int q = h * (MJ + NB) + x;
          if (ks == 0) {
            asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(lo[q]) : "v"(p));
            asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(hi[q]) : "v"(p), "n"(4 * RJ));
          } else {
            asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(lo[q]) : "v"(p), "n"(32 * RJ));
            asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(hi[q]) : "v"(p), "n"(36 * RJ));
          }
        }
#pragma unroll
        for (int y = 0; y < NB; ++y) {
          const unsigned p = base + offb[h][y];
          const int q = h * (MJ + NB) + MJ + y;
          if (ks == 0) {
            asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(lo[q]) : "v"(p));
            asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(hi[q]) : "v"(p), "n"(4 * RI));
          } else {
            asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(lo[q]) : "v"(p), "n"(32 * RI));
            asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(hi[q]) : "v"(p), "n"(36 * RI));
          }
        }
      }
      tr_wait(lo, hi);
      bf16x8 fa[NH][MJ], fb[NH][NB];
#pragma unroll
      for (int h = 0; h < NH; ++h) {
#pragma unroll
        for (int x = 0; x < MJ; ++x) {
          const int q = h * (MJ + NB) + x;
          fa[h][x] = __builtin_bit_cast(bf16x8, __builtin_shufflevector(lo[q], hi[q], 0, 1, 2, 3, 4, 5, 6, 7));
        }
#pragma unroll
        for (int y = 0; y < NB; ++y) {
          const int q = h * (MJ + NB) + MJ + y;
          fb[h][y] = __builtin_bit_cast(bf16x8, __builtin_shufflevector(lo[q], hi[q], 0, 1, 2, 3, 4, 5, 6, 7));
        }
      }
      if (do_db && wi == 0) {  // (X3F: dY_hi + dY_lo)
#pragma unroll
        for (int h = 0; h < NH; ++h)
#pragma unroll
          for (int x = 0; x < MJ; ++x)
#pragma unroll
            for (int e = 0; e < 8; ++e) dbp[x] += (float)fa[h][x][e];
      }
#pragma unroll
      for (int tt = 0; tt < NTW; ++tt) {
        if (NTW > 1 && tt >= ntap) continue;  // (uniform) a tap past KT: zeros, skipped
#pragma unroll
        for (int x = 0; x < MJ; ++x)
#pragma unroll
          for (int y = 0; y < MI; ++y) {
            f32x4& d = acc[x][tt * MI + y];
            d = mfma_bf16x(fa[0][x], fb[0][tt * MI + y], d);
            if (X3F) {  // dY_lo X_hi + dY_hi X_lo
              d = mfma_bf16x(fa[NH - 1][x], fb[0][tt * MI + y], d);
              d = mfma_bf16x(fa[0][x], fb[NH - 1][tt * MI + y], d);
            }
          }
      }
    }
    // stage t + 1 must have landed: at most NST - 2 later stages still in flight
    if (t + NST - 1 < nst) asm volatile("s_waitcnt vmcnt(%0)" ::"n"((NST - 2) * PPW) : "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
  }
  if (do_db) {
#pragma unroll
    for (int x = 0; x < MJ; ++x) {
      dbp[x] += __shfl_xor(dbp[x], 16, 64);
      dbp[x] += __shfl_xor(dbp[x], 32, 64);
    }
    if (wi == 0 && fg == 0) {
#pragma unroll
      for (int x = 0; x < MJ; ++x) dbs[wj * 16 * MJ + x * 16 + fr] = dbp[x];
    }
    __syncthreads();
    if (!a.dbpart)
      for (int t = tid; t < TJ; t += NW * 64)
        if (j0 + t < g.Nc && nst > 0) atomic_add_f(a.db + j0 + t, dbs[t]);
  }
  if (a.dbpart && a.db && by == 0)  // every (split, column) row element written once (0: no bias terms)
    for (int t = tid; t < TJ; t += NW * 64)
      if (j0 + t < g.Nc) a.dbpart[(size_t)bz * g.Nc + j0 + t] = (do_db && nst > 0) ? dbs[t] : 0.f;
  const bool to_slab = a.slab != nullptr && a.outmap == WG_OUT_CONV;
  if (nst == 0 && !to_slab) return;
  float* slab = to_slab ? a.slab + (size_t)bz * g.Nc * g.KT * g.Kc : nullptr;
#pragma unroll
  for (int tt = 0; tt < NTW; ++tt) {
    if (tt >= ntap) continue;
    const int dt = dt0 + tt;
#pragma unroll
    for (int x = 0; x < MJ; ++x) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int j = j0 + wj * 16 * MJ + x * 16 + fg * 4 + r;
        if (j >= g.Nc) continue;
#pragma unroll
        for (int y = 0; y < MI; ++y) {
          const int i = i0 + wi * 16 * MI + y * 16 + fr;
          if (i >= g.Kc) continue;
          size_t idx;
          if (a.outmap == WG_OUT_GCN) {
            const int k = i / a.gcn_cin, ci = i - k * a.gcn_cin;
            idx = ((size_t)k * g.Nc + j) * a.gcn_cin + ci;
          } else {
            idx = (size_t)j * g.KT * g.Kc + (size_t)dt * g.Kc + i;
          }
          const float v = acc[x][tt * MI + y][r];
          if (to_slab) slab[idx] = v;
          else atomic_add_f(a.dw + idx, v);
        }
      }
    }
  }
}

// ----------------------------------------------------------------------------
// wgrad_taps: the stride-1 (9,1) tcn weight gradient with all 9 taps of a 64 co x 64 ci tile
// computed from ONE staged copy of each clip's rows. wgrad_big restages the dY and input rows
// once per tap (each tap is its own workgroup tile), so its L2 -> LDS fill is ~12x the
// algorithmic bytes and bounds it; here a workgroup stages a whole clip's dY rows [T*V][64 co]
// and input rows [T*V][64 ci] once, and tap dt reads the input tile shifted by dt*V rows. The
// input region keeps 4V zero rows above and below the clip (written once, never staged into),
// so a shifted window needs no masking; the dY region's rows past T*V (up to a 32-row multiple)
// stay zero, so the padded k steps add nothing. Fragments come from the same swizzled layout and
// transposed LDS reads as wgrad_big; the swizzle of a shifted row is taken per tap (it stays
// bank-conflict-free for any shift, checked exhaustively for V = 14 / 18).
// Waves: w & 3 picks the 16-column ci slice, w >> 2 the tap half (taps 0-4 or 5-8): the two waves
// sharing a SIMD issue 20 + 16 MFMAs per k step. Split-K over clips into slab[split] (plain
// stores), summed by wgrad_slab_reduce_kernel. One workgroup per CU (118 KiB of LDS), two stages.
// Needs: bf16 operands, forward geometry with S = 1, KT = 9, P = 4, T_in = T_out, V even,
// T*V % 8 == 0, roundup(T*V, 32) == 32*NKS, Nc % 64 == 0, Kc % 64 == 0.
// CH (frame chunks, the 64-channel layers at T = 30 / 29, whose 540-row clips do not fit two
// stages): the unit of work is a chunk of F = a.taps_f frames of a clip (F*V <= 32*NKS rows of dY)
// with its input rows from 4 frames before to 4 frames after — halo rows are real rows there,
// staged every unit (the zero page outside the clip), and dY rows past the chunk stage as zeros.
// ----------------------------------------------------------------------------
template <int NKS, bool CH = false>
__global__ __launch_bounds__(512) void wgrad_taps(WgradArgs a) {
  constexpr int R = 128;                    // row bytes of both tiles (64 bf16)
  constexpr int TVP = 32 * NKS;             // padded clip rows
  constexpr int VMAX = 18;
  constexpr int Y_BYTES = TVP * R, X_BYTES = (TVP + 8 * VMAX) * R, STAGE = Y_BYTES + X_BYTES;
  __shared__ __attribute__((aligned(16))) char smem[2 * STAGE];
  const ConvGeom& g = a.g;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int V = g.V, TV = g.T_out * g.V;
  const int jt = g.Nc / 64, tiles = jt * (g.Kc / 64);
  const int lin = xcd_remap(blockIdx.x, gridDim.x);  // a split's tiles stay on one XCD
  const int bz = lin / tiles, tile = lin - bz * tiles;
  const int j0 = (tile % jt) * 64, i0 = (tile / jt) * 64;
  // bf16x3 row segments (x3seg, as wgrad_big): (dY_hi, X_hi), (dY_lo, X_hi), (dY_hi, X_lo)
  const int seg = a.x3seg ? bz % 3 : 0;
  // units: whole clips, or (CH) chunks of F frames, upc per clip
  const int F = CH ? a.taps_f : g.T_out, upc = CH ? (g.T_out + F - 1) / F : 1;
  const int n_begin = (a.x3seg ? bz / 3 : bz) * a.rows_per_split;  // units per split
  const int n_end = min(g.M / TV * upc, n_begin + a.rows_per_split);
  const __bf16* dyb = reinterpret_cast<const __bf16*>(a.dyb) + (seg == 1 ? g.Nc : 0);
  const __bf16* xb = reinterpret_cast<const __bf16*>(a.inb) + (seg == 2 ? g.Kc : 0);
  const unsigned lds0 = (unsigned)(size_t)(lds_cchar_t*)smem;

  // ---- staging: 1-KiB pieces (8 rows), dY pieces then input pieces; a lane's slots are fixed ----
  // whole clips: TV / 8 dY pieces and as many input pieces (the halo rows stay zero); CH: all TVP / 8
  // dY pieces (rows past the chunk from the zero page) and the (F + 8) V rows of the input window
  const int npy = CH ? TVP / 8 : TV / 8, npx = CH ? ((F + 8) * V + 7) / 8 : TV / 8;
  const int np = npy + npx, ppw = (np + 7) / 8;
  const int sub = lane >> 3, ph = lane & 7;
  constexpr int PPW_MAX = CH ? (X_BYTES / R / 8 + TVP / 8 + 7) / 8 : (2 * TVP / 8 + 7) / 8;
  unsigned ldso[PPW_MAX];
  int srow[PPW_MAX], scol[PPW_MAX];  // the lane's row (clip-local dY row / window-local input row), column
  bool isy[PPW_MAX];
#pragma unroll
  for (int k = 0; k < PPW_MAX; ++k) {
    int piece = k * 8 + wave;
    if (piece >= np) piece %= np;  // the last round re-issues earlier pieces: same bytes, same place
    const bool y = piece < npy;
    const int pr = y ? piece : piece - npy;           // piece index within its tile
    const int crow = pr * 8 + sub;                    // dY row / (CH) input window row
    const int brow = y ? crow : (CH ? crow : 4 * V + crow);  // buffer row in its region
    const int u = (ph >> 1) ^ wswz<4>(brow);
    const int col = (u * 2 + (ph & 1)) * 8;
    isy[k] = y;
    ldso[k] = (unsigned)((y ? 0 : Y_BYTES) + brow * R + ph * 16);
    srow[k] = crow;
    scol[k] = y ? j0 + col : i0 + col;
  }
  auto stage = [&](int n, int buf) {
    // unit n: clip n / upc, frames f0 .. f0 + nf - 1 (CH); input window from frame f0 - 4
    const int clip = n / upc, f0 = (n - clip * upc) * F, nf = min(F, g.T_out - f0);
    const long long ybase = (long long)(clip * g.T_out + f0) * V;
    const long long xbase = (long long)(clip * g.T_in + f0 - (CH ? 4 : 0)) * V;
#pragma unroll
    for (int k = 0; k < PPW_MAX; ++k) {
      if (k < ppw) {
        const int r = srow[k];
        bool ok = true;
        if (CH) {
          const int xr = (f0 - 4) * V + r;  // clip-local input row of a window row
          ok = isy[k] ? r < nf * V : (r < (nf + 8) * V && xr >= 0 && xr < g.T_in * V);
        }
        const __bf16* src = !ok ? reinterpret_cast<const __bf16*>(a.zero)
                            : isy[k] ? dyb + (ybase + r) * a.ldy + scol[k] : xb + (xbase + r) * g.lda + scol[k];
        // the DMA writes lane L's 16 B at (M0 + instruction offset) + 16 L: pass the piece base
        __builtin_amdgcn_global_load_lds((const void*)src,
                                         (lds_void_t*)(size_t)(lds0 + buf * STAGE + ldso[k] - lane * 16), 16, 0, 0);
      }
    }
  };

  // ---- fragment lanes ----
  const int wi = wave & 3, kh = wave >> 2;
  const int ntap = kh == 0 ? 5 : 4, dt0 = kh * 5;
  const int fr = lane & 15, fg = lane >> 4, tq = fr >> 2, tp = fr & 3;
  const int r0 = 8 * fg + tq;
  const int fa = wswz<4>(r0);  // unchanged at r0 + 4 and r0 + 32*ks
  unsigned offa[4];
#pragma unroll
  for (int x = 0; x < 4; ++x) offa[x] = r0 * R + ((x ^ fa) * 32) + tp * 8;
  unsigned offl[5], offh[5];
  // every wave issues 5 tap reads (the second half's 5th repeats its 4th, unused): a read under a
  // wave-varying condition let hipcc repack the other reads' destination registers before the
  // lgkmcnt wait (measured: garbage in taps 2-3 whenever the LDS was slow, i.e. inside the step)
#pragma unroll
  for (int tt = 0; tt < 5; ++tt) {
    const int rl = r0 + (dt0 + min(tt, ntap - 1)) * V, rh = rl + 4;
    offl[tt] = Y_BYTES + rl * R + ((wi ^ wswz<4>(rl)) * 32) + tp * 8;
    offh[tt] = Y_BYTES + rh * R + ((wi ^ wswz<4>(rh)) * 32) + tp * 8;
  }

  f32x4 acc[5][4];
#pragma unroll
  for (int tt = 0; tt < 5; ++tt)
#pragma unroll
    for (int x = 0; x < 4; ++x) acc[tt][x] = f32x4{0.f, 0.f, 0.f, 0.f};
  // The second tap half has a free 5th MFMA column: with an all-ones B fragment it sums dY over
  // the rows, i.e. the bias gradient, at no extra issue (the first version summed the fragments
  // on the VALU in one wave, which held its workgroup's SIMD ~60 % longer per k step).
  typedef unsigned u32x4_t __attribute__((ext_vector_type(4)));
  const unsigned ones_m = kh ? 0xffffffffu : 0u;
  const u32x4_t ones_v = {0x3f803f80u & ones_m, 0x3f803f80u & ones_m, 0x3f803f80u & ones_m, 0x3f803f80u & ones_m};
  const u32x4_t keep_v = {~ones_m, ~ones_m, ~ones_m, ~ones_m};

  const int nst = n_end - n_begin;
  if (nst > 0) stage(n_begin, 0);
  // zero the rows no stage ever writes (dY padding past T*V, the input halo and tail), in both
  // buffers, while the first clip's DMA is in flight (disjoint bytes); CH: only the input rows past
  // the staged window
  if (CH) {
    const int xw = npx * 8;
#pragma unroll
    for (int b = 0; b < 2; ++b)
      for (int o = Y_BYTES + xw * R + tid * 16; o < STAGE; o += 512 * 16)
        *reinterpret_cast<f32x4*>(smem + b * STAGE + o) = f32x4{0.f, 0.f, 0.f, 0.f};
  } else {
    const int zr[3][2] = {{TV * R, Y_BYTES}, {Y_BYTES, Y_BYTES + 4 * V * R}, {Y_BYTES + (4 * V + TV) * R, STAGE}};
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int z = 0; z < 3; ++z)
        for (int o = zr[z][0] + tid * 16; o < zr[z][1]; o += 512 * 16)
          *reinterpret_cast<f32x4*>(smem + b * STAGE + o) = f32x4{0.f, 0.f, 0.f, 0.f};
  }
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
  __syncthreads();
  for (int t = 0; t < nst; ++t) {
    const int buf = t & 1;
    if (t + 1 < nst) stage(n_begin + t + 1, buf ^ 1);
    const unsigned base = lds0 + buf * STAGE;
    // k step ks + 1's 26 fragment reads are issued before k step ks's MFMAs (two register sets);
    // the loop is branch-free between every read and its wait, so no read destination can be
    // touched early (the second half's 5th tap is computed into an accumulator it discards)
    s16x4_t lo[2][9], hi[2][9];
    auto issue = [&](int ks, s16x4_t (&l)[9], s16x4_t (&h)[9]) {
#pragma unroll
      for (int x = 0; x < 4; ++x) {
        const unsigned p = base + offa[x] + ks * 32 * R;
        asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(l[x]) : "v"(p));
        asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(h[x]) : "v"(p), "n"(4 * R));
      }
#pragma unroll
      for (int tt = 0; tt < 5; ++tt) {
        asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(l[4 + tt]) : "v"(base + offl[tt] + ks * 32 * R));
        asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(h[4 + tt]) : "v"(base + offh[tt] + ks * 32 * R));
      }
    };
    issue(0, lo[0], hi[0]);
#pragma unroll
    for (int ks = 0; ks < NKS; ++ks) {
      const int c = ks & 1;
      tr_wait(lo[c], hi[c]);
      bf16x8 fa_[4];
#pragma unroll
      for (int x = 0; x < 4; ++x)
        fa_[x] = __builtin_bit_cast(bf16x8, __builtin_shufflevector(lo[c][x], hi[c][x], 0, 1, 2, 3, 4, 5, 6, 7));
      bf16x8 fbs[5];
#pragma unroll
      for (int tt = 0; tt < 5; ++tt)
        fbs[tt] = __builtin_bit_cast(bf16x8, __builtin_shufflevector(lo[c][4 + tt], hi[c][4 + tt], 0, 1, 2, 3, 4, 5, 6, 7));
      // second half: the 5th column is the ones fragment (bit select, no branch)
      fbs[4] = __builtin_bit_cast(bf16x8, (__builtin_bit_cast(u32x4_t, fbs[4]) & keep_v) | ones_v);
      if (ks + 1 < NKS) issue(ks + 1, lo[c ^ 1], hi[c ^ 1]);
#pragma unroll
      for (int tt = 0; tt < 5; ++tt)
#pragma unroll
        for (int x = 0; x < 4; ++x) acc[tt][x] = mfma_bf16x(fa_[x], fbs[tt], acc[tt][x]);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }
  // bias gradient: the ones column of wave (kh 1, wi 0) in the i0 == 0 tiles; lane (fg, fr = 0)
  // holds co = x*16 + fg*4 + r (all 16 columns carry the same sum); x3seg: dY_hi + dY_lo only
  if (a.db && i0 == 0 && kh == 1 && wi == 0 && fr == 0) {
    const bool any = seg < 2 && nst > 0;
#pragma unroll
    for (int x = 0; x < 4; ++x)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int j = j0 + x * 16 + fg * 4 + r;
        if (a.dbpart) a.dbpart[(size_t)bz * g.Nc + j] = any ? acc[4][x][r] : 0.f;  // every (split, j) once
        else if (any) atomic_add_f(a.db + j, acc[4][x][r]);
      }
  }
  // partials in fragment order, slab[split][tile][wi][dt][x][lane] as 16-B pieces: each store is
  // one contiguous KiB per wave (the reference-layout scatter took 80 4-B stores per lane at
  // the kernel's end, when every CU stores at once); wgrad_taps_reduce_kernel reorders
  f32x4* slab = reinterpret_cast<f32x4*>(a.slab) + ((size_t)(bz * tiles + tile) * 4 + wi) * 9 * 4 * 64 + lane;
#pragma unroll
  for (int tt = 0; tt < 5; ++tt) {
    if (tt < ntap) {
#pragma unroll
      for (int x = 0; x < 4; ++x) slab[((dt0 + tt) * 4 + x) * 64] = acc[tt][x];
    }
  }
}

// dw_ref[j][i][dt] += sum_s (wgrad_taps' fragment-order slab). Workgroup = one (tile, wi, x)
// block: 16 co x 16 ci x 9 taps. Wave dt, lane L sums the 16-B piece [dt][x][L] over the splits
// (each load a contiguous KiB per wave, 8 in flight), drops its 4 values into an LDS image
// [16 co][16 ci][9] that is exactly the reference layout of those 16 output rows (144
// contiguous floats each), and the workgroup adds it into dw_ref as 16-B pieces.
__global__ __launch_bounds__(576) void wgrad_taps_reduce_kernel(const float* __restrict__ slab, int splits, int Nc,
                                                                 int Kc, float* __restrict__ dw_ref,
                                                                 const float* __restrict__ dbpart,
                                                                 float* __restrict__ db) {
  __shared__ __attribute__((aligned(16))) float img[16 * 16 * 9];
  const int nbias = dbpart ? (Nc + 63) / 64 : 0;  // (the bias rows first, as wgrad_slab_reduce_kernel)
  if ((int)blockIdx.x < nbias) {
    wgrad_bias_block(dbpart, splits, Nc, db, blockIdx.x, reinterpret_cast<float (*)[64]>(img));
    return;
  }
  const int tiles = (Nc / 64) * (Kc / 64), jt = Nc / 64;
  const int b = blockIdx.x - nbias, tile = b >> 4, wi = (b >> 2) & 3, x = b & 3;
  const int j0 = (tile % jt) * 64 + x * 16, i0 = (tile / jt) * 64 + wi * 16;
  const int tid = threadIdx.x, dt = tid >> 6, lane = tid & 63, fr = lane & 15, fg = lane >> 4;
  const f32x4* p = reinterpret_cast<const f32x4*>(slab) + (((size_t)tile * 4 + wi) * 9 + dt) * 4 * 64 + x * 64 + lane;
  const size_t per = (size_t)tiles * 4 * 9 * 4 * 64;  // f32x4 per split
  f32x4 s = {0.f, 0.f, 0.f, 0.f};
  int sp = 0;
  for (; sp + 8 <= splits; sp += 8) {
    f32x4 v[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) v[q] = p[(size_t)(sp + q) * per];
#pragma unroll
    for (int q = 0; q < 8; ++q) s += v[q];
  }
  for (; sp < splits; ++sp) s += p[(size_t)sp * per];
#pragma unroll
  for (int r = 0; r < 4; ++r) img[((fg * 4 + r) * 16 + fr) * 9 + dt] = s[r];
  __syncthreads();
  // 16 rows x 36 float4 = 576 pieces, one per thread
  const int row = tid / 36, c4 = tid - row * 36;
  f32x4* o = reinterpret_cast<f32x4*>(dw_ref + ((size_t)(j0 + row) * Kc + i0) * 9) + c4;
  *o += *reinterpret_cast<const f32x4*>(img + row * 144 + c4 * 4);
}

// bf16x3 row segments are ordered segment-minor (split index = row range * 3 + segment: the three
// products of one row range on adjacent workgroups; 10.39 -> 10.25-10.32 ms/step against
// segment-major, profiles/r04_zimg_segminor_ab.txt)

// wgrad_taps applies (see its comment); nks = padded clip (or chunk) rows / 32, +16 for the chunked
// form, whose chunk frame count goes to a.taps_f
static int wgrad_taps_nks(WgradArgs& a) {
  const ConvGeom& g = a.g;
  if (!a.dyb || !a.inb || !a.slab || a.outmap != WG_OUT_CONV || a.groups > 1 || g.transposed) return 0;
  if (g.KT != 9 || g.S != 1 || g.P != 4 || g.T_in != g.T_out || g.V % 2 || g.V > 18) return 0;
  if (g.Nc % 64 || g.Kc % 64 || a.ldy % 8 || g.lda % 8) return 0;
  const int TV = g.T_out * g.V;
  if (g.M % TV) return 0;
  const int nks = (TV + 31) / 32;
  if (TV % 8 == 0 && (nks == 4 || nks == 5)) return nks;
  // frame chunks: the fewest chunks whose dY rows fit 6 k steps and whose window (F + 8 frames) fits
  // the input region (TVP + 8 * 18 rows). Only from 128 channels: on the 64-channel T = 30 layers (one
  // 64 x 64 tile, 231 splits) the chunked kernel took 66 us + a 19-56 us reduce over 16 workgroups
  // against wgrad_big's 63 + 10 (bf16x3, B = 256); the 128-channel T = 15 layer gains (85 vs 104 us)
  if (g.Nc < 128) return 0;
  for (int upc = 2; upc <= 8; ++upc) {
    const int F = (g.T_out + upc - 1) / upc, ks = (F * g.V + 31) / 32;
    if ((ks == 5 || ks == 6) && (F + 8) * g.V <= 32 * ks + 8 * 18) {
      a.taps_f = F;
      return 16 + ks;
    }
  }
  return 0;
}

static int launch_wgrad_taps(WgradArgs a, int nks, hipStream_t s) {
  const int TV = a.g.T_out * a.g.V;
  const int clips = a.g.M / TV * (nks > 16 ? (a.g.T_out + a.taps_f - 1) / a.taps_f : 1);  // units
  const int tiles = (a.g.Nc / 64) * (a.g.Kc / 64);
  const long long per_split = (long long)a.g.Nc * 9 * a.g.Kc;
  // one workgroup per CU, or the share wg_pct of them (side-queue launches beside the main chains)
  const int target = std::max(1, 256 * (a.wg_pct > 0 ? std::min(100, a.wg_pct) : 100) / 100);
  const int nseg = a.x3seg ? 3 : 1;  // bf16x3 row segments: `splits` clip splits per segment
  int splits = std::max(1, std::min(clips, target / (tiles * nseg)));
  splits = (int)std::min<long long>(splits, a.slab_cap / (per_split * nseg));
  if (splits < 1) return F3_EINVAL;
  const int cps = (clips + splits - 1) / splits;
  splits = (clips + cps - 1) / cps;
  a.rows_per_split = cps;  // clips per split
  splits *= nseg;
  // bias-gradient partial rows after the slab partials (deterministic order), where the slab has room
  a.dbpart = (a.db && (long long)splits * (per_split + a.g.Nc) <= a.slab_cap) ? a.slab + (size_t)splits * per_split
                                                                              : nullptr;
  const dim3 grid(tiles * splits);
  if (nks == 5) hipLaunchKernelGGL(wgrad_taps<5>, grid, dim3(512), 0, s, a);
  else if (nks == 4) hipLaunchKernelGGL(wgrad_taps<4>, grid, dim3(512), 0, s, a);
  else if (nks == 21) hipLaunchKernelGGL((wgrad_taps<5, true>), grid, dim3(512), 0, s, a);
  else hipLaunchKernelGGL((wgrad_taps<6, true>), grid, dim3(512), 0, s, a);
  F3_LAUNCH_CHECK();
  if (a.dw_ref) {  // (with the bias rows: no separate colsum launch)
    const int nbias = a.dbpart ? (a.g.Nc + 63) / 64 : 0;
    hipLaunchKernelGGL(wgrad_taps_reduce_kernel, dim3(nbias + tiles * 16), dim3(576), 0, s, a.slab, splits, a.g.Nc,
                       a.g.Kc, a.dw_ref, a.dbpart, a.db);
    F3_LAUNCH_CHECK();
    return F3_OK;
  }
  if (a.dbpart) return f3_colsum(a.dbpart, splits, a.g.Nc, a.db, s);
  return F3_OK;
}

bool f3_wgrad_glds_ok(const WgradArgs& a) {
  return a.dyb && a.inb && a.zero && a.g.Nc % 64 == 0 && a.g.Kc % 64 == 0 && a.ldy % 8 == 0 && a.g.lda % 8 == 0;
}

// dW accumulation target: WG_OUT_GCN writes the reference layout; WG_OUT_CONV writes the
// PACKED layout [Nc][KT*Kc] (caller unpacks with PREP_UNPACK_CONV).
// Resident workgroups of a kernel on the whole chip (occupancy x CUs), queried once.
static int resident_wgs(const void* fn, int threads) {
  int per_cu = 0, dev = 0, cus = 256;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, fn, threads, 0) != hipSuccess || per_cu < 1) per_cu = 2;
  if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  (void)hipGetLastError();
  return per_cu * cus;
}

template <int TJ, int TI, int THREADS, void (*KERNEL)(WgradArgs), int NTW = 1>
static int launch_wgrad(WgradArgs a, hipStream_t s) {
  const int gx = (a.g.Nc + TJ - 1) / TJ;
  const int gy = ((a.g.KT + NTW - 1) / NTW) * ((a.g.Kc + TI - 1) / TI);  // (tap groups of NTW)
  // Split-K over rows sized to ONE round of resident workgroups: rounding the split count up
  // (a ceil of 512 / tiles) put 513-540 workgroups on 512 slots on MI355X — a second round
  // for a handful of workgroups.
  static const int slots = resident_wgs((const void*)KERNEL, THREADS);
  // wg_pct (percent): size the splits to that share of the resident slots, leaving CUs to the main
  // chains the side-queue weight gradients run beside
  const int target = std::max(1, slots * (a.wg_pct > 0 ? std::min(100, a.wg_pct) : 100) / 100);
  const int groups = std::max(1, a.groups);  // grouped launches: wgrad_big, atomics (checked by the caller)
  // x3seg: three row segments, `splits` row splits each (one round of resident workgroups in all)
  const int nseg = a.x3seg ? 3 : 1;
  int splits = std::max(1, target / (gx * gy * groups * nseg));
  const bool to_slab = a.slab && a.outmap == WG_OUT_CONV;
  const long long per_split = (long long)a.g.Nc * a.g.KT * a.g.Kc;
  if (to_slab) {
    if (a.slab_cap < per_split * nseg) return F3_EINVAL;
    // (the slab grew for wgrad_taps; these tiles keep their measured split count)
    splits = (int)std::min<long long>(splits, std::min<long long>(a.slab_cap, a.x3seg ? a.slab_cap : 512LL * 128 * 128) /
                                                  (per_split * nseg));
  }
  int rps = (a.g.M + splits - 1) / splits;
  rps = ((rps + 63) / 64) * 64;
  if (rps < 256) rps = 256;
  splits = (a.g.M + rps - 1) / rps;
  a.rows_per_split = rps;
  splits *= nseg;  // slab partials (all segments)
  // bias-gradient partial rows after the slab partials (deterministic order), where the slab has room
  a.dbpart = (a.db && to_slab && (long long)splits * (per_split + a.g.Nc) <= a.slab_cap)
                 ? a.slab + (size_t)splits * per_split : nullptr;
  // XCD-aware 1-D grid: measured in the B=256 step, HBM fetch per launch 273 -> 40 MB (tcn layers
  // 0-2) and 171 -> 68 MB (layers 3-6) at unchanged kernel time against a round-robin 3-D grid
  a.xcd = 1;
  const dim3 grid(gx * gy * splits * groups);
  hipLaunchKernelGGL(KERNEL, grid, dim3(THREADS), 0, s, a);
  F3_LAUNCH_CHECK();
  if (to_slab && a.dw_ref) {  // (with the bias rows: no separate colsum launch)
    const int nbias = a.dbpart ? (a.g.Nc + 63) / 64 : 0;
    hipLaunchKernelGGL(wgrad_slab_reduce_kernel, dim3((unsigned)(nbias + per_split / 64)), dim3(256), 0, s, a.slab,
                       splits, a.g.Nc, a.g.Kc, a.g.KT, a.dw_ref, a.gcn_cin, a.dbpart, a.db);
    F3_LAUNCH_CHECK();
    return F3_OK;
  }
  if (a.dbpart) return f3_colsum(a.dbpart, splits, a.g.Nc, a.db, s);
  return F3_OK;
}

int f3_wgrad_glds_bf16(const WgradArgs* args, hipStream_t s) {
  const WgradArgs& a = *args;
  if (a.g.M <= 0) return F3_OK;
  if (!f3_wgrad_glds_ok(a)) return F3_EINVAL;
  // (dw_ref == null: the GEMM alone at the step's split count, partials left in the slab)
  if (a.x3seg && (!a.slab || a.outmap != WG_OUT_CONV || a.groups > 1 || a.g.transposed || a.ldy < 2 * a.g.Nc ||
                  a.g.lda < 2 * a.g.Kc))
    return F3_EINVAL;
  if (a.x3seg && a.gcn_cin > 0 && (a.g.KT != 1 || a.g.Kc % a.gcn_cin)) return F3_EINVAL;
  // 8-wave wide tiles for the 128/256-channel layers; the first 4-wave kernel (wgrad_glds_bf16) only
  // for transposed-geometry rows, which wgrad_big does not walk
  if (a.groups > 1 && (a.g.transposed || a.slab)) return F3_EINVAL;  // grouped: wgrad_big + atomics only
  const bool bigv = !a.g.transposed;
  if (bigv) {
    // all 9 taps of a clip-sized stride-1 layer from one staged copy of each clip (wgrad_taps); clip
    // segments with halo rows for the other (9,1) layers measured slower (61 vs 35 us)
    WgradArgs at = a;
    const int nks = wgrad_taps_nks(at);
    if (nks) return launch_wgrad_taps(at, nks, s);
  }
  if (a.x3seg && !bigv) return F3_EINVAL;  // (row segments: wgrad_taps / wgrad_big only)
  // Tile choice (layer-6 tcn weight gradient alone, B = 256, lean loop): 256 x 128 63 us,
  // 128 x 256 71 us, 256 x 256 (BK 32) 63 us, the 4-wave 128 x 128 kernel 99 us. The loop is
  // bound by the L2 -> LDS fill rate per CU, so the wider dY tile (each input row staged once
  // per 256 output channels) wins.
  // Tap groups (wgrad_big NTW > 1, the (9,1) tcn layers): the 256 x 128 tiles 2 taps (BK 32), the
  // 128 x 128 tiles 3 taps (BK 32). Measured on MI355X (bf16x3, B = 256): the layer-5 weight gradient
  // 0.260 -> 0.222 ms per launch pair with the 2-tap groups; both 9.90 -> 9.81 ms/step in four of four
  // rounds; 3-tap groups for the 64 x 64 tiles and 4-stage rings gave nothing (profiles/r04_ntw_ab.txt,
  // r04_last_ab.txt, r04_nst4_ab.txt)
  const bool taps9 = a.g.KT == 9;
  if (bigv && a.x3seg && !taps9 && a.g.Nc % 128 == 0 && a.g.Kc % 128 == 0) {
    // the 128 / 256-channel 1x1 (gcn, residual) bf16x3 weight gradients with the row segments fused (X3F):
    // 128 B of LDS fill per MFMA instead of 192 (profiles/r05_x3f8_ab.txt: step 8.75 -> 8.66 ms)
    WgradArgs af = a;
    af.x3seg = 0;
    if (a.g.Nc % 256 == 0) return launch_wgrad<256, 128, 512, wgrad_big<4, 2, 4, 4, 32, 1, 3, true>>(af, s);
    if (a.g.Kc % 256 == 0) return launch_wgrad<128, 256, 512, wgrad_big<2, 4, 4, 4, 32, 1, 3, true>>(af, s);
    return launch_wgrad<128, 128, 512, wgrad_big<2, 4, 4, 2, 32, 1, 3, true>>(af, s);
  }
  if (bigv && a.x3seg && taps9 && a.g.Nc % 128 == 0 && a.g.Kc % 128 == 0) {
    // the 9-tap bf16x3 weight gradients wgrad_taps does not take (the stride-2 layers), X3F: 256 x 128
    // tiles tap by tap (a 2-tap group of fused rows needs 192 KiB), 128 x 128 tiles in 2-tap groups.
    // Step 8.66-8.68 -> 8.52-8.59 ms (profiles/r05_x3f9_ab.txt; the 128-channel layer's share neutral)
    WgradArgs af = a;
    af.x3seg = 0;
    if (a.g.Nc % 256 == 0) return launch_wgrad<256, 128, 512, wgrad_big<4, 2, 4, 4, 32, 1, 3, true>>(af, s);
    return launch_wgrad<128, 128, 512, wgrad_big<2, 4, 4, 2, 32, 2, 3, true>, 2>(af, s);
  }
  if (bigv && a.g.Nc % 256 == 0 && a.g.Kc % 128 == 0) {
    if (taps9) return launch_wgrad<256, 128, 512, wgrad_big<4, 2, 4, 4, 32, 2>, 2>(a, s);
    return launch_wgrad<256, 128, 512, wgrad_big<4, 2, 4, 4>>(a, s);
  }
  if (bigv && a.g.Nc % 128 == 0 && a.g.Kc % 256 == 0)
    return launch_wgrad<128, 256, 512, wgrad_big<2, 4, 4, 4>>(a, s);
  if (bigv && a.g.Nc % 128 == 0 && a.g.Kc % 128 == 0) {
    if (taps9) return launch_wgrad<128, 128, 512, wgrad_big<2, 4, 4, 2, 32, 3>, 3>(a, s);
    return launch_wgrad<128, 128, 512, wgrad_big<2, 4, 4, 2>>(a, s);
  }
  if (bigv && a.x3seg && a.g.Nc % 64 == 0 && a.g.Kc % 64 == 0 && (a.g.Nc < 128 || a.g.Kc < 128)) {
    // bf16x3 on the 64-wide tiles: the three row segments fused into one staging (X3F, 32-row
    // stages: 48 KiB, three workgroups per CU). The 64-channel T=30 tcn weight gradient alone: 97.4 ->
    // 77.0 us, step 8.83-8.86 -> 8.73 ms; tap groups of 2 / 3 on top measured 87 / 110 us (fewer
    // workgroups per CU), profiles/r05_x3f_ab.txt
    WgradArgs af = a;
    af.x3seg = 0;
    if (a.g.Nc % 128 == 0) return launch_wgrad<128, 64, 256, wgrad_big<2, 2, 4, 2, 32, 1, 3, true>>(af, s);
    if (a.g.Kc % 128 == 0) return launch_wgrad<64, 128, 256, wgrad_big<2, 2, 2, 4, 32, 1, 3, true>>(af, s);
    // (64 x 64: 8 waves of 32 x 16 instead of 4 of 32 x 32 — same 73.8 us alone, step 8.52 -> 8.45 ms in
    // three of three rounds, more waves per CU beside the main chains; a 4-stage ring 86 us,
    // profiles/r05_w64_ab.txt)
    return launch_wgrad<64, 64, 512, wgrad_big<2, 4, 2, 1, 32, 1, 3, true>>(af, s);
  }
  if (bigv) {  // 64-wide tiles: 4 waves, same lean loop (64-channel tcn: 38 -> 28 us)
    if (a.g.Nc % 128 == 0) return launch_wgrad<128, 64, 256, wgrad_big<2, 2, 4, 2>>(a, s);
    if (a.g.Kc % 128 == 0) return launch_wgrad<64, 128, 256, wgrad_big<2, 2, 2, 4>>(a, s);
    return launch_wgrad<64, 64, 256, wgrad_big<2, 2, 2, 2>>(a, s);
  }
  const int TJ = a.g.Nc >= 128 ? 128 : 64, TI = a.g.Kc >= 128 ? 128 : 64;
  if (TJ == 128 && TI == 128) return launch_wgrad<128, 128, 256, wgrad_glds_bf16<128, 128>>(a, s);
  if (TJ == 128) return launch_wgrad<128, 64, 256, wgrad_glds_bf16<128, 64>>(a, s);
  if (TI == 128) return launch_wgrad<64, 128, 256, wgrad_glds_bf16<64, 128>>(a, s);
  return launch_wgrad<64, 64, 256, wgrad_glds_bf16<64, 64>>(a, s);
}
