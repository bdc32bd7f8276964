// TARGCN skeleton model (BASELINE config 2) on gfx950: EmbGCN-gated graph GRU, temporal
// attention, end_conv/pool/Linear head. Reference (file:line relative to /root/reference):
//   EmbGCN.forward       EmbGCN.py:69-89     (adaptive supports, node-specific weights, static branch)
//   GRU.forward          GRU.py:17-27
//   AVWDCRNN.forward     TRAGCN.py:150-169   (2 layers x 30 steps, then the TA layer)
//   Transform.forward    TA.py:40-69         (conv (1,3) q/k over T-as-channels, softmax over T, 2 LN)
//   TARGCN.forward       TRAGCN.py:207-224   (end_conv -> reshape -> avg pool -> Linear)
//
// Recurrence layout. The GRU mixes nodes (S . x) and applies node-specific weights, but never
// mixes clips, so one workgroup owns a tile of clips for all nodes and runs all 30 steps with no
// inter-workgroup communication. Per step, per node n, the EmbGCN products are MFMA GEMMs with
// the tile's clips as rows: [clips x I] . W_n[I x O] (gconv) and the static Linear
// [clips x I] . Lin^T; the mixed / raw inputs sit in LDS ([node][clip][k], 16-B padded rows),
// the packed weights stream from L2. The hidden state stays in registers of the wave that owns
// (node, 16-column tile) for both gate tiles (z and r columns) and the update tile, so the gate
// -> update -> h' chain needs no LDS round trip. Everything a weight gradient needs (mixed
// inputs, raw inputs, pre-activation gradients) is written once per row to HBM; the weight
// gradients themselves are large per-node GEMMs over B*T rows done after the recurrence.
#include "targcn.h"

#include <algorithm>

namespace f3 {
namespace tg {

typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));

template <bool B16>
struct Op;
template <>
struct Op<true> {
  typedef __bf16 T;
  static constexpr int KS = 32;       // k per MFMA (v_mfma_f32_16x16x32_bf16)
  static constexpr int XS = IP + 8;   // LDS row stride: 272-B rows, conflict-free b128 A reads
  static constexpr int BTF = 16;      // clips per workgroup, forward
  static constexpr int BTB = 8;       // backward (four [node][clip][k] buffers in LDS)
};
template <>
struct Op<false> {
  typedef float T;
  static constexpr int KS = 4;        // v_mfma_f32_16x16x4_f32 (exact fp32 products)
  static constexpr int XS = IP + 4;
  static constexpr int BTF = 4;
  static constexpr int BTB = 4;
};

template <bool B16>
F3_DEV f32x4 mma(const typename Op<B16>::T* a, const typename Op<B16>::T* b, f32x4 c) {
  if constexpr (B16) {
    const bf16x8_t av = *reinterpret_cast<const bf16x8_t*>(a);
    const bf16x8_t bv = *reinterpret_cast<const bf16x8_t*>(b);
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(av, bv, c, 0, 0, 0);
  } else {
    return __builtin_amdgcn_mfma_f32_16x16x4f32(*a, *b, c, 0, 0, 0);
  }
}

F3_DEV float silu_grad(float s) {  // d/ds s*sigmoid(s)
  const float g = sigmoidf_(s);
  return g * (1.f + s * (1.f - g));
}

// out[n][b][k] (+)= sum_m S'[n][m] in[m][b][k] for k < I (pairs of columns per thread);
// S' = S (forward mix, EmbGCN.py:84) or S^T (its input gradient).
template <typename TY, int BT, int XS, bool TRANS, bool ACC, int NT>
F3_DEV void node_mix(const TY* in, TY* out, const float* Sl, int V, int I, int tid) {
  const int kp = (I + 1) >> 1;
  for (int ci = tid; ci < BT * kp; ci += NT) {
    const int b = ci / kp, k = (ci - b * kp) * 2;
    float a0[VMAX], a1[VMAX];
#pragma unroll
    for (int n = 0; n < VMAX; ++n) a0[n] = a1[n] = 0.f;
    for (int m = 0; m < V; ++m) {
      const TY* src = in + (m * BT + b) * XS + k;
      const float x0 = (float)src[0], x1 = (float)src[1];
#pragma unroll
      for (int n = 0; n < VMAX; ++n) {
        if (n < V) {
          const float s = TRANS ? Sl[m * V + n] : Sl[n * V + m];
          a0[n] += s * x0;
          a1[n] += s * x1;
        }
      }
    }
#pragma unroll
    for (int n = 0; n < VMAX; ++n) {
      if (n < V) {
        TY* dst = out + (n * BT + b) * XS + k;
        if (ACC) {
          dst[0] = (TY)((float)dst[0] + a0[n]);
          dst[1] = (TY)((float)dst[1] + a1[n]);
        } else {
          dst[0] = (TY)a0[n];
          dst[1] = (TY)a1[n];
        }
      }
    }
  }
}

// LDS rows [n][b][0:IP] -> HBM rows ((b0+b)*T + t)*V + n of width IP (operand type), 16-B chunks
template <typename TY, int BT, int XS, int NT>
F3_DEV void store_rows(const TY* L, void* dst, int V, int B, int b0, int t, int tid) {
  constexpr int CH = IP * (int)sizeof(TY) / 16;
  for (int i = tid; i < V * BT * CH; i += NT) {
    const int row = i / CH, ch = i - row * CH;
    const int n = row / BT, b = row - n * BT;
    if (b0 + b >= B) continue;
    const size_t R = ((size_t)(b0 + b) * T + t) * V + n;
    const uint4 v = *reinterpret_cast<const uint4*>(reinterpret_cast<const char*>(L + row * XS) + ch * 16);
    *reinterpret_cast<uint4*>(reinterpret_cast<char*>(dst) + R * IP * sizeof(TY) + ch * 16) = v;
  }
}

constexpr int GRU_THREADS = 512;
constexpr int GRU_WAVES = GRU_THREADS / 64;
constexpr int NJ = (4 * VMAX + GRU_WAVES - 1) / GRU_WAVES;  // owned (node, 16-column tile) jobs per wave

// ---------------------------------------------------------------------------------------------
// Forward recurrence of one GRU layer (GRU.py:17-27 over TRAGCN.py:162-164's time loop).
// ---------------------------------------------------------------------------------------------
template <bool B16>
__global__ __launch_bounds__(GRU_THREADS) void gru_fwd_kernel(GruFwdArgs a) {
  using TT = typename Op<B16>::T;
  constexpr int BT = Op<B16>::BTF, XS = Op<B16>::XS, KS = Op<B16>::KS;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int V = a.V, Din = a.Din, I = a.I;
  TT* X = reinterpret_cast<TT*>(smem);
  TT* Y = X + V * BT * XS;
  float* Sl = reinterpret_cast<float*>(Y + V * BT * XS);
  float* csl = Sl + V * V;
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int b0 = blockIdx.x * BT;
  for (int i = tid; i < 2 * V * BT * XS; i += GRU_THREADS) X[i] = (TT)0.f;
  for (int i = tid; i < V * V; i += GRU_THREADS) Sl[i] = a.S[i];
  for (int i = tid; i < V; i += GRU_THREADS) csl[i] = a.cs[i];
  const int col = lane & 15, rq = lane >> 4;
  const int arow = (lane & 15) % BT;
  const int kofs = B16 ? 8 * (lane >> 4) : (lane >> 4);
  const int nks = (I + KS - 1) / KS;
  const int njobs = 4 * V;
  const TT* gWf = reinterpret_cast<const TT*>(a.g.Wf);
  const TT* gLf = reinterpret_cast<const TT*>(a.g.Lf);
  const TT* uWf = reinterpret_cast<const TT*>(a.u.Wf);
  const TT* uLf = reinterpret_cast<const TT*>(a.u.Lf);
  float hreg[NJ][4], zreg[NJ][4], rreg[NJ][4];
#pragma unroll
  for (int jj = 0; jj < NJ; ++jj)
#pragma unroll
    for (int r = 0; r < 4; ++r) hreg[jj][r] = zreg[jj][r] = rreg[jj][r] = 0.f;
  __syncthreads();
  for (int t = 0; t < T; ++t) {
    // x_t -> X[., ., 0:Din], h -> X[., ., Din:Din+H]
    for (int i = tid; i < BT * V * Din; i += GRU_THREADS) {
      const int b = i / (V * Din), rem = i - b * V * Din, n = rem / Din, c = rem - n * Din;
      const float v = (b0 + b < a.B) ? a.x[((size_t)(b0 + b) * T + t) * V * Din + rem] : 0.f;
      X[(n * BT + b) * XS + c] = (TT)v;
    }
#pragma unroll
    for (int jj = 0; jj < NJ; ++jj) {
      int q = wave + GRU_WAVES * jj;
      asm volatile("" : "+s"(q));  // per step: keep job addresses and biases out of loop-invariant registers
      if (q < njobs) {
        const int n = q >> 2, j = q & 3;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int b = rq * 4 + r;
          if (b < BT) X[(n * BT + b) * XS + Din + 16 * j + col] = (TT)hreg[jj][r];
        }
      }
    }
    __syncthreads();
    node_mix<TT, BT, XS, false, false, GRU_THREADS>(X, Y, Sl, V, I, tid);
    __syncthreads();
    store_rows<TT, BT, XS, GRU_THREADS>(X, a.XI, V, a.B, b0, t, tid);
    store_rows<TT, BT, XS, GRU_THREADS>(Y, a.XG, V, a.B, b0, t, tid);
    // gate: zr = sigmoid(S.x W_n + b_n + silu(cs*x Lin^T + b))   (EmbGCN.py:78-89, GRU.py:22)
#pragma unroll
    for (int jj = 0; jj < NJ; ++jj) {
      int q = wave + GRU_WAVES * jj;
      asm volatile("" : "+s"(q));  // per step: keep job addresses and biases out of loop-invariant registers
      if (q < njobs) {
        const int n = q >> 2, j = q & 3, cz = 16 * j + col;
        f32x4 gz = {0.f, 0.f, 0.f, 0.f}, gr = gz, sz = gz, sr = gz;
        const TT* ay = Y + (n * BT + arow) * XS + kofs;
        const TT* ax = X + (n * BT + arow) * XS + kofs;
        const TT* wz = gWf + ((size_t)n * 2 * H + cz) * IP + kofs;
        const TT* wr = wz + (size_t)H * IP;
        const TT* lz = gLf + (size_t)cz * IP + kofs;
        const TT* lr = lz + (size_t)H * IP;
#pragma unroll 1
        for (int ks = 0; ks < nks; ++ks) {
          const int o = ks * KS;
          gz = mma<B16>(ay + o, wz + o, gz);
          gr = mma<B16>(ay + o, wr + o, gr);
          sz = mma<B16>(ax + o, lz + o, sz);
          sr = mma<B16>(ax + o, lr + o, sr);
        }
        const float csn = csl[n];
        const float bnz = a.g.bn[n * 2 * H + cz], bnr = a.g.bn[n * 2 * H + H + cz];
        const float blz = a.g.bl[cz], blr = a.g.bl[H + cz];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int b = rq * 4 + r;
          const float s_z = sz[r] * csn + blz, s_r = sr[r] * csn + blr;
          const float z = sigmoidf_(gz[r] + bnz + s_z * sigmoidf_(s_z));
          const float rr = sigmoidf_(gr[r] + bnr + s_r * sigmoidf_(s_r));
          zreg[jj][r] = z;
          rreg[jj][r] = rr;
          if (b < BT && b0 + b < a.B) {
            const size_t R = ((size_t)(b0 + b) * T + t) * V + n;
            a.ZR[R * 2 * H + cz] = z;
            a.ZR[R * 2 * H + H + cz] = rr;
            a.SG[R * 2 * H + cz] = s_z;
            a.SG[R * 2 * H + H + cz] = s_r;
          }
        }
      }
    }
    __syncthreads();
    // candidate input [x, r*h] (GRU.py:24)
#pragma unroll
    for (int jj = 0; jj < NJ; ++jj) {
      int q = wave + GRU_WAVES * jj;
      asm volatile("" : "+s"(q));  // per step: keep job addresses and biases out of loop-invariant registers
      if (q < njobs) {
        const int n = q >> 2, j = q & 3;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int b = rq * 4 + r;
          if (b < BT) X[(n * BT + b) * XS + Din + 16 * j + col] = (TT)(rreg[jj][r] * hreg[jj][r]);
        }
      }
    }
    __syncthreads();
    node_mix<TT, BT, XS, false, false, GRU_THREADS>(X, Y, Sl, V, I, tid);
    __syncthreads();
    store_rows<TT, BT, XS, GRU_THREADS>(X, a.UI, V, a.B, b0, t, tid);
    store_rows<TT, BT, XS, GRU_THREADS>(Y, a.UG, V, a.B, b0, t, tid);
    // update: hc = tanh(EmbGCN_u([x, r*h])); h = z*h + (1-z)*hc   (GRU.py:25-26)
#pragma unroll
    for (int jj = 0; jj < NJ; ++jj) {
      int q = wave + GRU_WAVES * jj;
      asm volatile("" : "+s"(q));  // per step: keep job addresses and biases out of loop-invariant registers
      if (q < njobs) {
        const int n = q >> 2, j = q & 3, c = 16 * j + col;
        f32x4 gu = {0.f, 0.f, 0.f, 0.f}, su = gu;
        const TT* ay = Y + (n * BT + arow) * XS + kofs;
        const TT* ax = X + (n * BT + arow) * XS + kofs;
        const TT* wu = uWf + ((size_t)n * H + c) * IP + kofs;
        const TT* lu = uLf + (size_t)c * IP + kofs;
#pragma unroll 1
        for (int ks = 0; ks < nks; ++ks) {
          const int o = ks * KS;
          gu = mma<B16>(ay + o, wu + o, gu);
          su = mma<B16>(ax + o, lu + o, su);
        }
        const float csn = csl[n], bnu = a.u.bn[n * H + c], blu = a.u.bl[c];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int b = rq * 4 + r;
          const float s = su[r] * csn + blu;
          const float hc = tanhf(gu[r] + bnu + s * sigmoidf_(s));
          const float z = zreg[jj][r];
          const float h = z * hreg[jj][r] + (1.f - z) * hc;
          hreg[jj][r] = h;
          if (b < BT && b0 + b < a.B) {
            const size_t R = ((size_t)(b0 + b) * T + t) * V + n;
            a.HC[R * H + c] = hc;
            a.SU[R * H + c] = s;
            a.Hout[R * H + c] = h;
          }
        }
      }
    }
    __syncthreads();
  }
}

// ---------------------------------------------------------------------------------------------
// Backward recurrence (BPTT) of one GRU layer: the input-gradient chain only. Per step the
// pre-activation gradients (dP, cs*dSg, dU, cs*dSu) and the unmixed input gradients of both
// EmbGCN products (dXG, dUG) go to HBM for the post-recurrence weight / support gradients.
// ---------------------------------------------------------------------------------------------
template <bool B16>
__global__ __launch_bounds__(GRU_THREADS) void gru_bwd_kernel(GruBwdArgs a) {
  using TT = typename Op<B16>::T;
  constexpr int BT = Op<B16>::BTB, XS = Op<B16>::XS, KS = Op<B16>::KS;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int V = a.V, Din = a.Din, I = a.I;
  TT* AG = reinterpret_cast<TT*>(smem);   // [V][BT][XS] d pre-activation (gconv A operand)
  TT* AS = AG + V * BT * XS;              // cs * d static pre-activation (static A operand)
  TT* GX = AS + V * BT * XS;              // d mixed input (unmixed gconv input gradient)
  TT* DX = GX + V * BT * XS;              // d input = static part + S^T . GX
  float* Sl = reinterpret_cast<float*>(DX + V * BT * XS);
  float* csl = Sl + V * V;
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int b0 = blockIdx.x * BT;
  for (int i = tid; i < 4 * V * BT * XS; i += GRU_THREADS) AG[i] = (TT)0.f;
  for (int i = tid; i < V * V; i += GRU_THREADS) Sl[i] = a.S[i];
  for (int i = tid; i < V; i += GRU_THREADS) csl[i] = a.cs[i];
  const int col = lane & 15, rq = lane >> 4;
  const int arow = (lane & 15) % BT;
  const int kofs = B16 ? 8 * (lane >> 4) : (lane >> 4);
  const int njobs = 4 * V;
  const int nit = (I + 15) / 16;
  const bool has_dx = a.dX != nullptr && Din == H;
  const TT* gWb = reinterpret_cast<const TT*>(a.g.Wb);
  const TT* gLb = reinterpret_cast<const TT*>(a.g.Lb);
  const TT* uWb = reinterpret_cast<const TT*>(a.u.Wb);
  const TT* uLb = reinterpret_cast<const TT*>(a.u.Lb);
  TT* DP = reinterpret_cast<TT*>(a.DP);
  TT* DSG = reinterpret_cast<TT*>(a.DSG);
  TT* DU = reinterpret_cast<TT*>(a.DU);
  TT* DSU = reinterpret_cast<TT*>(a.DSU);
  float dh[NJ][4], dz[NJ][4], dxr[NJ][4];
#pragma unroll
  for (int jj = 0; jj < NJ; ++jj)
#pragma unroll
    for (int r = 0; r < 4; ++r) dh[jj][r] = dz[jj][r] = dxr[jj][r] = 0.f;
  __syncthreads();
  for (int t = T - 1; t >= 0; --t) {
    // h = z*hp + (1-z)*hc: dz, dhc -> dU (tanh), cs*dSu (silu)
#pragma unroll
    for (int jj = 0; jj < NJ; ++jj) {
      int q = wave + GRU_WAVES * jj;
      asm volatile("" : "+s"(q));  // per step: keep job addresses and biases out of loop-invariant registers
      if (q < njobs) {
        const int n = q >> 2, j = q & 3, c = 16 * j + col;
        const float csn = csl[n];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int b = rq * 4 + r;
          float dU = 0.f, dsu = 0.f;
          if (b < BT && b0 + b < a.B) {
            const size_t R = ((size_t)(b0 + b) * T + t) * V + n;
            const float g = dh[jj][r] + a.dH[R * H + c];
            const float z = a.ZR[R * 2 * H + c], hc = a.HC[R * H + c], su = a.SU[R * H + c];
            const float hp = t > 0 ? a.Hout[(R - V) * H + c] : 0.f;
            dz[jj][r] = g * (hp - hc);
            dU = g * (1.f - z) * (1.f - hc * hc);
            dsu = dU * silu_grad(su) * csn;
            dh[jj][r] = g * z;
            DU[R * H + c] = (TT)dU;
            DSU[R * H + c] = (TT)dsu;
          } else {
            dz[jj][r] = 0.f;
          }
          if (b < BT) {
            AG[(n * BT + b) * XS + c] = (TT)dU;
            AS[(n * BT + b) * XS + c] = (TT)dsu;
          }
        }
      }
    }
    __syncthreads();
    // update EmbGCN input gradient: GX = dU . W_n^T, DX = (cs dSu) . Lin
    for (int q = wave; q < V * nit; q += GRU_WAVES) {
      const int n = q / nit, i = 16 * (q - n * nit) + col;
      f32x4 gx = {0.f, 0.f, 0.f, 0.f}, sx = gx;
      const TT* aa = AG + (n * BT + arow) * XS + kofs;
      const TT* as = AS + (n * BT + arow) * XS + kofs;
      const TT* wb = uWb + ((size_t)n * IP + i) * H + kofs;
      const TT* lb = uLb + (size_t)i * H + kofs;
#pragma unroll 1
      for (int ks = 0; ks < H / KS; ++ks) {
        const int o = ks * KS;
        gx = mma<B16>(aa + o, wb + o, gx);
        sx = mma<B16>(as + o, lb + o, sx);
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int b = rq * 4 + r;
        if (b < BT) {
          GX[(n * BT + b) * XS + i] = (TT)gx[r];
          DX[(n * BT + b) * XS + i] = (TT)sx[r];
        }
      }
    }
    __syncthreads();
    node_mix<TT, BT, XS, true, true, GRU_THREADS>(GX, DX, Sl, V, I, tid);
    store_rows<TT, BT, XS, GRU_THREADS>(GX, a.DUG, V, a.B, b0, t, tid);
    __syncthreads();
    // d(r*h) -> dr, dh; gate pre-activation gradients
#pragma unroll
    for (int jj = 0; jj < NJ; ++jj) {
      int q = wave + GRU_WAVES * jj;
      asm volatile("" : "+s"(q));  // per step: keep job addresses and biases out of loop-invariant registers
      if (q < njobs) {
        const int n = q >> 2, j = q & 3, c = 16 * j + col;
        const float csn = csl[n];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int b = rq * 4 + r;
          float dPz = 0.f, dPr = 0.f, dsz = 0.f, dsr = 0.f;
          if (b < BT && b0 + b < a.B) {
            const size_t R = ((size_t)(b0 + b) * T + t) * V + n;
            const float drh = (float)DX[(n * BT + b) * XS + Din + c];
            const float z = a.ZR[R * 2 * H + c], rr = a.ZR[R * 2 * H + H + c];
            const float hp = t > 0 ? a.Hout[(R - V) * H + c] : 0.f;
            dh[jj][r] += drh * rr;
            if (has_dx) dxr[jj][r] = (float)DX[(n * BT + b) * XS + c];
            dPz = dz[jj][r] * z * (1.f - z);
            dPr = drh * hp * rr * (1.f - rr);
            dsz = dPz * silu_grad(a.SG[R * 2 * H + c]) * csn;
            dsr = dPr * silu_grad(a.SG[R * 2 * H + H + c]) * csn;
            DP[R * 2 * H + c] = (TT)dPz;
            DP[R * 2 * H + H + c] = (TT)dPr;
            DSG[R * 2 * H + c] = (TT)dsz;
            DSG[R * 2 * H + H + c] = (TT)dsr;
          }
          if (b < BT) {
            AG[(n * BT + b) * XS + c] = (TT)dPz;
            AG[(n * BT + b) * XS + H + c] = (TT)dPr;
            AS[(n * BT + b) * XS + c] = (TT)dsz;
            AS[(n * BT + b) * XS + H + c] = (TT)dsr;
          }
        }
      }
    }
    __syncthreads();
    // gate EmbGCN input gradient (K = 2H)
    for (int q = wave; q < V * nit; q += GRU_WAVES) {
      const int n = q / nit, i = 16 * (q - n * nit) + col;
      f32x4 gx = {0.f, 0.f, 0.f, 0.f}, sx = gx;
      const TT* aa = AG + (n * BT + arow) * XS + kofs;
      const TT* as = AS + (n * BT + arow) * XS + kofs;
      const TT* wb = gWb + ((size_t)n * IP + i) * 2 * H + kofs;
      const TT* lb = gLb + (size_t)i * 2 * H + kofs;
#pragma unroll 1
      for (int ks = 0; ks < 2 * H / KS; ++ks) {
        const int o = ks * KS;
        gx = mma<B16>(aa + o, wb + o, gx);
        sx = mma<B16>(as + o, lb + o, sx);
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int b = rq * 4 + r;
        if (b < BT) {
          GX[(n * BT + b) * XS + i] = (TT)gx[r];
          DX[(n * BT + b) * XS + i] = (TT)sx[r];
        }
      }
    }
    __syncthreads();
    node_mix<TT, BT, XS, true, true, GRU_THREADS>(GX, DX, Sl, V, I, tid);
    store_rows<TT, BT, XS, GRU_THREADS>(GX, a.DXG, V, a.B, b0, t, tid);
    __syncthreads();
#pragma unroll
    for (int jj = 0; jj < NJ; ++jj) {
      int q = wave + GRU_WAVES * jj;
      asm volatile("" : "+s"(q));  // per step: keep job addresses and biases out of loop-invariant registers
      if (q < njobs) {
        const int n = q >> 2, j = q & 3, c = 16 * j + col;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int b = rq * 4 + r;
          if (b < BT && b0 + b < a.B) {
            dh[jj][r] += (float)DX[(n * BT + b) * XS + Din + c];
            if (has_dx) {
              const size_t R = ((size_t)(b0 + b) * T + t) * V + n;
              a.dX[R * H + c] = dxr[jj][r] + (float)DX[(n * BT + b) * XS + c];
            }
          }
        }
      }
    }
  }
}

// ---------------------------------------------------------------------------------------------
// Per-step parameter preparation (TRAGCN.py's EmbGCN calls all share node_embeddings E):
//   S = I + softmax(relu(E E^T), 1)                                    EmbGCN.py:74-75
//   W_n = E . weights_pool, b_n = E . bias_pool (packed both ways)     EmbGCN.py:81-82
//   cs[m] = column sums of softmax(softmax(symnorm(ones + I/2)))        EmbGCN.py:14-26,63-64,78
// ---------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void tg_supports_kernel(const float* __restrict__ E, int V, float* S, float* cs) {
  __shared__ float Z[VMAX * VMAX];
  const int tid = threadIdx.x;
  for (int p = tid; p < V * V; p += 256) {
    const int n = p / V, m = p - n * V;
    float acc = 0.f;
    for (int d = 0; d < EMB; ++d) acc += E[n * EMB + d] * E[m * EMB + d];
    Z[p] = fmaxf(acc, 0.f);
  }
  __syncthreads();
  if (tid < V) {
    const int n = tid;
    float mx = -INFINITY;
    for (int m = 0; m < V; ++m) mx = fmaxf(mx, Z[n * V + m]);
    float s = 0.f;
    for (int m = 0; m < V; ++m) s += expf(Z[n * V + m] - mx);
    for (int m = 0; m < V; ++m) S[n * V + m] = expf(Z[n * V + m] - mx) / s + (m == n ? 1.f : 0.f);
  }
  if (tid == 0) {  // static adjacency with adj = ones (TRAGCN.py:191)
    const double dgn = 1.0 / ((double)V + 0.5), sq = sqrt(dgn);
    float M[VMAX * VMAX];
    for (int n = 0; n < V; ++n)
      for (int m = 0; m < V; ++m) M[n * V + m] = (float)(sq * ((n == m ? 1.5 : 1.0) * sq));
    for (int pass = 0; pass < 2; ++pass)  // softmax(dim=1) at init, softmax(dim=-1) in forward
      for (int n = 0; n < V; ++n) {
        float mx = -INFINITY, s = 0.f;
        for (int m = 0; m < V; ++m) mx = fmaxf(mx, M[n * V + m]);
        for (int m = 0; m < V; ++m) s += expf(M[n * V + m] - mx);
        for (int m = 0; m < V; ++m) M[n * V + m] = expf(M[n * V + m] - mx) / s;
      }
    for (int m = 0; m < V; ++m) {
      float s = 0.f;
      for (int n = 0; n < V; ++n) s += M[n * V + m];
      cs[m] = s;
    }
  }
}



// one thread per (n, i, o) of W_n (i < IP, zero padding for i >= I), plus the linear packs
template <bool B16>
__global__ __launch_bounds__(256) void tg_prep_kernel(PrepArgs a) {
  using TT = typename Op<B16>::T;
  const int V = a.V, I = a.I, O = a.O;
  const long long idx = blockIdx.x * 256ll + threadIdx.x;
  const long long nW = (long long)V * IP * O;
  TT* Wf = reinterpret_cast<TT*>(a.ops.Wf);
  TT* Wb = reinterpret_cast<TT*>(a.ops.Wb);
  if (idx < nW) {
    const int o = (int)(idx % O);
    const long long ni = idx / O;
    const int i = (int)(ni % IP), n = (int)(ni / IP);
    float acc = 0.f;
    if (i < I) {
      for (int d = 0; d < EMB; ++d) acc += a.E[n * EMB + d] * a.pool[((size_t)d * I + i) * O + o];
    }
    Wb[((size_t)n * IP + i) * O + o] = (TT)acc;
    Wf[((size_t)n * O + o) * IP + i] = (TT)acc;
    return;
  }
  long long k = idx - nW;
  if (k < (long long)O * IP) {
    const int o = (int)(k / IP), i = (int)(k % IP);
    const float w = i < I ? a.lin[(size_t)o * I + i] : 0.f;
    reinterpret_cast<TT*>(a.ops.Lf)[(size_t)o * IP + i] = (TT)w;
    reinterpret_cast<TT*>(a.ops.Lb)[(size_t)i * O + o] = (TT)w;
    return;
  }
  k -= (long long)O * IP;
  if (k < (long long)V * O) {
    const int n = (int)(k / O), o = (int)(k % O);
    float acc = 0.f;
    for (int d = 0; d < EMB; ++d) acc += a.E[n * EMB + d] * a.bpool[(size_t)d * O + o];
    a.ops.bn[k] = acc;
  }
}

// ---------------------------------------------------------------------------------------------
// Post-recurrence gradients.
// ---------------------------------------------------------------------------------------------
// dSupp[n][m] += sum_{r} sum_{i<I} dxg[r][n][i] * xin[r][m][i]  (two (dxg, xin) pairs, r = b*T+t)


template <bool B16>
__global__ __launch_bounds__(256) void tg_supp_grad_kernel(SuppGradArgs a) {
  using TT = typename Op<B16>::T;
  __shared__ float Ld[VMAX][IP + 1], Lx[VMAX][IP + 1];
  const int V = a.V, I = a.I, tid = threadIdx.x;
  float acc[2] = {0.f, 0.f};
  const int p0 = tid, p1 = tid + 256;
  for (int pr = 0; pr < 2; ++pr) {
    const TT* dg = reinterpret_cast<const TT*>(a.dxg[pr]);
    const TT* xi = reinterpret_cast<const TT*>(a.xin[pr]);
    for (int r = blockIdx.x; r < a.rows; r += gridDim.x) {
      __syncthreads();
      for (int e = tid; e < V * I; e += 256) {
        const int n = e / I, i = e - n * I;
        Ld[n][i] = (float)dg[((size_t)r * V + n) * IP + i];
        Lx[n][i] = (float)xi[((size_t)r * V + n) * IP + i];
      }
      __syncthreads();
      if (p0 < V * V) {
        const int n = p0 / V, m = p0 - n * V;
        float s = 0.f;
        for (int i = 0; i < I; ++i) s += Ld[n][i] * Lx[m][i];
        acc[0] += s;
      }
      if (p1 < V * V) {
        const int n = p1 / V, m = p1 - n * V;
        float s = 0.f;
        for (int i = 0; i < I; ++i) s += Ld[n][i] * Lx[m][i];
        acc[1] += s;
      }
    }
  }
  if (p0 < V * V) atomic_add_f(a.dS + p0, acc[0]);
  if (p1 < V * V) atomic_add_f(a.dS + p1, acc[1]);
}

// dWpool / dbpool / dLin / dLin_b of one EmbGCN and its dE contribution.


__global__ __launch_bounds__(256) void tg_pool_grad_kernel(PoolGradArgs a) {
  const int V = a.V, I = a.I, O = a.O;
  const long long idx = blockIdx.x * 256ll + threadIdx.x;
  const long long nP = (long long)EMB * I * O;
  if (idx < nP) {  // dWpool[d][i][o] = sum_n E[n][d] dW[n][o][i]
    const int o = (int)(idx % O);
    const long long di = idx / O;
    const int i = (int)(di % I), d = (int)(di / I);
    float acc = 0.f;
    for (int n = 0; n < V; ++n) acc += a.E[n * EMB + d] * a.dW[((size_t)n * O + o) * IP + i];
    a.g_pool[idx] = acc;
    return;
  }
  long long k = idx - nP;
  if (k < (long long)EMB * O) {  // dbpool[d][o] = sum_n E[n][d] db[n][o]
    const int d = (int)(k / O), o = (int)(k % O);
    float acc = 0.f;
    for (int n = 0; n < V; ++n) acc += a.E[n * EMB + d] * a.db[n * O + o];
    a.g_bpool[k] = acc;
    return;
  }
  k -= (long long)EMB * O;
  if (k < (long long)O * I) {  // dLin[o][i] = sum_n dWs[n][o][i]
    const int o = (int)(k / I), i = (int)(k % I);
    float acc = 0.f;
    for (int n = 0; n < V; ++n) acc += a.dWs[((size_t)n * O + o) * IP + i];
    a.g_lin[k] = acc;
    return;
  }
  k -= (long long)O * I;
  if (k < O) {  // dLin_b[o] = sum_n dbs[n][o] / cs[n]
    float acc = 0.f;
    for (int n = 0; n < V; ++n) acc += a.dbs[n * O + k] / a.cs[n];
    a.g_linb[k] = acc;
  }
}

// dE[n][d] += sum_{i,o} pool[d][i][o] dW[n][o][i] + sum_o bpool[d][o] db[n][o]; grid (V*EMB)
__global__ __launch_bounds__(256) void tg_pool_dE_kernel(PoolGradArgs a) {
  __shared__ float part[4];
  const int n = blockIdx.x / EMB, d = blockIdx.x % EMB;
  const int I = a.I, O = a.O;
  float acc = 0.f;
  for (int e = threadIdx.x; e < I * O; e += 256) {
    const int i = e / O, o = e - i * O;
    acc += a.pool[((size_t)d * I + i) * O + o] * a.dW[((size_t)n * O + o) * IP + i];
  }
  for (int o = threadIdx.x; o < O; o += 256) acc += a.bpool[(size_t)d * O + o] * a.db[n * O + o];
  acc = warp_sum(acc);
  if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) atomic_add_f(a.g_E + n * EMB + d, part[0] + part[1] + part[2] + part[3]);
}

// dE += (dZ + dZ^T) E through S = I + softmax(relu(E E^T), 1), dS given (one workgroup)
__global__ __launch_bounds__(256) void tg_supports_bwd_kernel(const float* __restrict__ E, int V,
                                                              const float* __restrict__ dS, float* g_E) {
  __shared__ float Z[VMAX * VMAX], P[VMAX * VMAX], dZ[VMAX * VMAX];
  const int tid = threadIdx.x;
  for (int p = tid; p < V * V; p += 256) {
    const int n = p / V, m = p - n * V;
    float acc = 0.f;
    for (int d = 0; d < EMB; ++d) acc += E[n * EMB + d] * E[m * EMB + d];
    Z[p] = acc;
  }
  __syncthreads();
  if (tid < V) {
    const int n = tid;
    float mx = -INFINITY, s = 0.f;
    for (int m = 0; m < V; ++m) mx = fmaxf(mx, fmaxf(Z[n * V + m], 0.f));
    for (int m = 0; m < V; ++m) s += expf(fmaxf(Z[n * V + m], 0.f) - mx);
    float dot = 0.f;
    for (int m = 0; m < V; ++m) {
      P[n * V + m] = expf(fmaxf(Z[n * V + m], 0.f) - mx) / s;
      dot += P[n * V + m] * dS[n * V + m];
    }
    for (int m = 0; m < V; ++m) {
      const float dA = P[n * V + m] * (dS[n * V + m] - dot);
      dZ[n * V + m] = Z[n * V + m] > 0.f ? dA : 0.f;
    }
  }
  __syncthreads();
  for (int p = tid; p < V * EMB; p += 256) {
    const int n = p / EMB, d = p - n * EMB;
    float acc = 0.f;
    for (int m = 0; m < V; ++m) acc += (dZ[n * V + m] + dZ[m * V + n]) * E[m * EMB + d];
    g_E[p] += acc;
  }
}

// ---------------------------------------------------------------------------------------------
// Head (TRAGCN.py:200-205,217-222). end_conv Conv2d(6, T*64, (1, H)) followed by the average
// pool over (T, N) of the reshaped [B, T, 64, N] output is linear, so the pooled feature is
//   pooled[b][c] = sum_k Wm[c][k] xm[b][k] + bm[c],
//   Wm[c][k] = mean_t W_end[t*64 + c][k],  bm[c] = mean_t b_end[t*64 + c],
//   xm[b][k = tin*H + h] = mean_n Y[b][T-6+tin][n][h]
// (exact reordering of the same sums); the 6.4 GFLOP end_conv at B=256 is never materialised.
// ---------------------------------------------------------------------------------------------
constexpr int KH = 6 * H;  // end_conv reduction width

__global__ __launch_bounds__(256) void tg_endconv_mean_kernel(const float* __restrict__ W, const float* __restrict__ bias,
                                                              float* Wm, float* bm) {
  const int idx = blockIdx.x * 256 + threadIdx.x;
  if (idx < C * KH) {
    const int c = idx / KH, k = idx - c * KH;
    float s = 0.f;
    for (int t = 0; t < T; ++t) s += W[(size_t)(t * C + c) * KH + k];
    Wm[idx] = s / (float)T;
  } else if (idx < C * KH + C) {
    const int c = idx - C * KH;
    float s = 0.f;
    for (int t = 0; t < T; ++t) s += bias[t * C + c];
    bm[c] = s / (float)T;
  }
}

// one workgroup per clip
__global__ __launch_bounds__(256) void tg_pool_fwd_kernel(const float* __restrict__ Y, int V, const float* __restrict__ Wm,
                                                          const float* __restrict__ bm, float* xm, float* pooled) {
  __shared__ float xs[KH];
  const int b = blockIdx.x;
  for (int k = threadIdx.x; k < KH; k += 256) {
    const int tin = k / H, h = k - tin * H;
    float s = 0.f;
    for (int n = 0; n < V; ++n) s += Y[(((size_t)b * T + (T - 6 + tin)) * V + n) * C + h];
    xs[k] = s / (float)V;
    xm[(size_t)b * KH + k] = xs[k];
  }
  __syncthreads();
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  for (int c = wave; c < C; c += 4) {
    float acc = 0.f;
    for (int k = lane; k < KH; k += 64) acc += Wm[c * KH + k] * xs[k];
    acc = warp_sum(acc);
    if (lane == 0) pooled[(size_t)b * C + c] = acc + bm[c];
  }
}

// dxm[b][k] = sum_c dpooled[b][c] Wm[c][k] -> dY[b][T-6+tin][n][h] = dxm / V (one workgroup per clip)
__global__ __launch_bounds__(256) void tg_pool_bwd_data_kernel(const float* __restrict__ dpooled, const float* __restrict__ Wm,
                                                               int V, float* dY) {
  __shared__ float dp[C];
  const int b = blockIdx.x;
  if (threadIdx.x < C) dp[threadIdx.x] = dpooled[(size_t)b * C + threadIdx.x];
  __syncthreads();
  for (int k = threadIdx.x; k < KH; k += 256) {
    float acc = 0.f;
    for (int c = 0; c < C; ++c) acc += dp[c] * Wm[c * KH + k];
    acc /= (float)V;
    const int tin = k / H, h = k - tin * H;
    for (int n = 0; n < V; ++n) dY[(((size_t)b * T + (T - 6 + tin)) * V + n) * C + h] = acc;
  }
}

// dWm[c][k] = sum_b dpooled[b][c] xm[b][k] -> g_W[t*64+c][k] = dWm / T ; g_b[t*64+c] = sum_b dpooled / T
__global__ __launch_bounds__(256) void tg_pool_bwd_weight_kernel(const float* __restrict__ dpooled, const float* __restrict__ xm,
                                                                 int B, float* gW, float* gb) {
  const int idx = blockIdx.x * 256 + threadIdx.x;
  if (idx < C * KH) {
    const int c = idx / KH, k = idx - c * KH;
    float s = 0.f;
    for (int b = 0; b < B; ++b) s += dpooled[(size_t)b * C + c] * xm[(size_t)b * KH + k];
    s /= (float)T;
    for (int t = 0; t < T; ++t) gW[(size_t)(t * C + c) * KH + k] = s;
  } else if (idx < C * KH + C) {
    const int c = idx - C * KH;
    float s = 0.f;
    for (int b = 0; b < B; ++b) s += dpooled[(size_t)b * C + c];
    s /= (float)T;
    for (int t = 0; t < T; ++t) gb[t * C + c] = s;
  }
}

// ---------------------------------------------------------------------------------------------
// Temporal attention layer (TA.py:40-69), one (clip, node) sequence X[T][C] at a time per
// workgroup (the layer never mixes sequences): q/k = Conv2d(T, T, (1,3)) over T-as-channels,
// v = Linear, A = softmax(q k^T / sqrt(C)) over T, o = LN(A v + x), y = LN(FF(o) + o).
// fp32 VALU with the layer's weights and the sequence's tensors in LDS.
// ---------------------------------------------------------------------------------------------
constexpr int TA_THREADS = 512;
constexpr int TA_W = 3 * C * C + 2 * T * T * 3 + 512;  // weight image (floats)
constexpr int VEC_CB1 = 0, VEC_CB2 = 30, VEC_BV = 64, VEC_BF1 = 128, VEC_BF2 = 192, VEC_G1 = 256, VEC_BE1 = 320,
              VEC_G2 = 384, VEC_BE2 = 448;
constexpr int TA_FWD_LDS = (TA_W + T * C + 2 * T * CQ + T * C + T * T + 3 * T * C + 64) * 4;
constexpr int TA_BWD_LDS = (TA_W + 8 * T * C + 2 * T * CQ + 2 * T * T + 64) * 4;
static_assert(TA_FWD_LDS <= 160 * 1024 && TA_BWD_LDS <= 160 * 1024, "TA LDS");

// weights into LDS; TRANSPOSED: Linear weights as [in][out] (forward), else [out][in]
template <bool TRANSPOSED>
F3_DEV void ta_load_weights(const TaArgs& a, float* sm, int tid) {
  const float* P = a.p;
  float* Wv = sm;
  float* W1 = Wv + C * C;
  float* W2 = W1 + C * C;
  float* cw1 = W2 + C * C;
  float* cw2 = cw1 + T * T * 3;
  float* vec = cw2 + T * T * 3;
  for (int i = tid; i < C * C; i += TA_THREADS) {
    const int o = i / C, k = i - o * C;
    const int d = TRANSPOSED ? k * C + o : i;
    Wv[d] = P[a.off_vw + i];
    W1[d] = P[a.off_f0w + i];
    W2[d] = P[a.off_f2w + i];
  }
  for (int i = tid; i < T * T * 3; i += TA_THREADS) {
    cw1[i] = P[a.off_c1w + i];
    cw2[i] = P[a.off_c2w + i];
  }
  for (int i = tid; i < 512; i += TA_THREADS) {
    float v = 0.f;
    if (i < 30) v = P[a.off_c1b + i];
    else if (i >= VEC_CB2 && i < VEC_CB2 + 30) v = P[a.off_c2b + i - VEC_CB2];
    else if (i >= VEC_BV && i < VEC_BV + C) v = P[a.off_vb + i - VEC_BV];
    else if (i >= VEC_BF1 && i < VEC_BF1 + C) v = P[a.off_f0b + i - VEC_BF1];
    else if (i >= VEC_BF2 && i < VEC_BF2 + C) v = P[a.off_f2b + i - VEC_BF2];
    else if (i >= VEC_G1 && i < VEC_G1 + C) v = P[a.off_lnw + i - VEC_G1];
    else if (i >= VEC_BE1 && i < VEC_BE1 + C) v = P[a.off_lnb + i - VEC_BE1];
    else if (i >= VEC_G2 && i < VEC_G2 + C) v = P[a.off_lnffw + i - VEC_G2];
    else if (i >= VEC_BE2 && i < VEC_BE2 + C) v = P[a.off_lnffb + i - VEC_BE2];
    vec[i] = v;
  }
}

__global__ __launch_bounds__(TA_THREADS) void ta_fwd_kernel(TaArgs a) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  ta_load_weights<true>(a, sm, tid);
  const float* WvT = sm;
  const float* W1T = WvT + C * C;
  const float* W2T = W1T + C * C;
  const float* cw1 = W2T + C * C;
  const float* cw2 = cw1 + T * T * 3;
  const float* vec = cw2 + T * T * 3;
  float* Xs = sm + TA_W;
  float* Q = Xs + T * C;
  float* K = Q + T * CQ;
  float* Vv = K + T * CQ;
  float* P = Vv + T * C;
  float* O1 = P + T * T;
  float* U = O1 + T * C;
  float* F = U + T * C;
  const int V = a.V;
  for (int sq = blockIdx.x; sq < a.B * V; sq += gridDim.x) {
    const int b = sq / V, n = sq - b * V;
    float* sv = a.save + (size_t)sq * TA_SAVE;
    __syncthreads();
    for (int i = tid; i < T * C; i += TA_THREADS) {
      const int t = i / C, c = i - t * C;
      float x = a.in[(((size_t)b * T + t) * V + n) * C + c];
      if (a.pe) x += a.pe[i];
      Xs[i] = x;
    }
    __syncthreads();
    for (int i = tid; i < 2 * T * CQ; i += TA_THREADS) {
      const int which = i / (T * CQ), rem = i - which * T * CQ, tq = rem / CQ, cq = rem - tq * CQ;
      const float* w = (which ? cw2 : cw1) + tq * T * 3;
      float acc = vec[(which ? VEC_CB2 : VEC_CB1) + tq];
      for (int t = 0; t < T; ++t) {
        const float* xr = Xs + t * C + cq;
        acc += w[t * 3] * xr[0] + w[t * 3 + 1] * xr[1] + w[t * 3 + 2] * xr[2];
      }
      (which ? K : Q)[rem] = acc;
    }
    for (int i = tid; i < T * C; i += TA_THREADS) {
      const int t = i / C, c = i - t * C;
      float acc = vec[VEC_BV + c];
      for (int k = 0; k < C; ++k) acc += WvT[k * C + c] * Xs[t * C + k];
      Vv[i] = acc;
    }
    __syncthreads();
    for (int i = tid; i < T * T; i += TA_THREADS) {
      const int t = i / T, u = i - t * T;
      float acc = 0.f;
      for (int k = 0; k < CQ; ++k) acc += Q[t * CQ + k] * K[u * CQ + k];
      P[i] = acc * 0.125f;  // / sqrt(C) (TA.py:57)
    }
    __syncthreads();
    for (int t = wave; t < T; t += TA_THREADS / 64) {
      const float x = lane < T ? P[t * T + lane] : -INFINITY;
      float mx = x;
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) mx = fmaxf(mx, __shfl_xor(mx, o, 64));
      const float e = lane < T ? expf(x - mx) : 0.f;
      const float ssum = warp_sum(e);
      if (lane < T) P[t * T + lane] = e / ssum;
    }
    __syncthreads();
    for (int i = tid; i < T * C; i += TA_THREADS) {
      const int t = i / C, c = i - t * C;
      float acc = Xs[i];
      for (int u = 0; u < T; ++u) acc += P[t * T + u] * Vv[u * C + c];
      O1[i] = acc;
    }
    __syncthreads();
    for (int t = wave; t < T; t += TA_THREADS / 64) {  // LayerNorm (TA.py:67)
      const float x = O1[t * C + lane];
      const float mean = warp_sum(x) * (1.f / C);
      const float d = x - mean;
      const float rstd = rsqrtf(warp_sum(d * d) * (1.f / C) + 1e-5f);
      const float xh = d * rstd;
      O1[t * C + lane] = xh * vec[VEC_G1 + lane] + vec[VEC_BE1 + lane];
      sv[TA_X1 + t * C + lane] = xh;
      if (lane == 0) sv[TA_R1 + t] = rstd;
    }
    __syncthreads();
    for (int i = tid; i < T * C; i += TA_THREADS) {
      const int t = i / C, k = i - t * C;
      float acc = vec[VEC_BF1 + k];
      for (int c = 0; c < C; ++c) acc += W1T[c * C + k] * O1[t * C + c];
      U[i] = fmaxf(acc, 0.f);
    }
    __syncthreads();
    for (int i = tid; i < T * C; i += TA_THREADS) {
      const int t = i / C, c = i - t * C;
      float acc = vec[VEC_BF2 + c] + O1[i];
      for (int k = 0; k < C; ++k) acc += W2T[k * C + c] * U[t * C + k];
      F[i] = acc;
    }
    __syncthreads();
    for (int t = wave; t < T; t += TA_THREADS / 64) {  // LayerNorm (TA.py:69)
      const float x = F[t * C + lane];
      const float mean = warp_sum(x) * (1.f / C);
      const float d = x - mean;
      const float rstd = rsqrtf(warp_sum(d * d) * (1.f / C) + 1e-5f);
      const float xh = d * rstd;
      a.out[(((size_t)b * T + t) * V + n) * C + lane] = xh * vec[VEC_G2 + lane] + vec[VEC_BE2 + lane];
      sv[TA_F2 + t * C + lane] = xh;
      if (lane == 0) sv[TA_R2 + t] = rstd;
    }
    for (int i = tid; i < 2 * T * CQ; i += TA_THREADS) sv[TA_Q + i] = Q[i];  // Q, K contiguous
    for (int i = tid; i < T * C; i += TA_THREADS) {
      sv[TA_V + i] = Vv[i];
      sv[TA_U + i] = U[i];
    }
    for (int i = tid; i < T * T; i += TA_THREADS) sv[TA_P + i] = P[i];
  }
}

__global__ __launch_bounds__(TA_THREADS) void ta_bwd_kernel(TaArgs a) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  ta_load_weights<false>(a, sm, tid);
  const float* Wv = sm;
  const float* W1 = Wv + C * C;
  const float* W2 = W1 + C * C;
  const float* cw1 = W2 + C * C;
  const float* cw2 = cw1 + T * T * 3;
  const float* vec = cw2 + T * T * 3;
  float* Xs = sm + TA_W;
  float* Q = Xs + T * C;
  float* K = Q + T * CQ;
  float* Vv = K + T * CQ;
  float* P = Vv + T * C;
  float* X1 = P + T * T;
  float* Y1 = X1 + T * C;
  float* U = Y1 + T * C;
  float* DY = U + T * C;
  float* G1 = DY + T * C;
  float* DX = G1 + T * C;
  float* dP = DX + T * C;
  float* R1 = dP + T * T;
  float* R2 = R1 + 32;
  // owned parameter-gradient accumulators
  const int ro = tid >> 3, co = (tid & 7) * 8;
  float gW2[8], gW1[8], gWv[8], gc1[6], gc2[6];
#pragma unroll
  for (int e = 0; e < 8; ++e) gW2[e] = gW1[e] = gWv[e] = 0.f;
#pragma unroll
  for (int e = 0; e < 6; ++e) gc1[e] = gc2[e] = 0.f;
  float gbv = 0.f, gbf1 = 0.f, gbf2 = 0.f, gg1 = 0.f, gbe1 = 0.f, gg2 = 0.f, gbe2 = 0.f, gcb = 0.f;
  const int V = a.V;
  for (int sq = blockIdx.x; sq < a.B * V; sq += gridDim.x) {
    const int b = sq / V, n = sq - b * V;
    const float* sv = a.save + (size_t)sq * TA_SAVE;
    __syncthreads();
    for (int i = tid; i < T * C; i += TA_THREADS) {
      const int t = i / C;
      const size_t g = (((size_t)b * T + t) * V + n) * C + (i - t * C);
      float x = a.in[g];
      if (a.pe) x += a.pe[i];
      Xs[i] = x;
      DY[i] = a.dout[g];
      Vv[i] = sv[TA_V + i];
      X1[i] = sv[TA_X1 + i];
      U[i] = sv[TA_U + i];
      G1[i] = sv[TA_F2 + i];
    }
    for (int i = tid; i < 2 * T * CQ; i += TA_THREADS) Q[i] = sv[TA_Q + i];
    for (int i = tid; i < T * T; i += TA_THREADS) P[i] = sv[TA_P + i];
    if (tid < T) {
      R1[tid] = sv[TA_R1 + tid];
      R2[tid] = sv[TA_R2 + tid];
    }
    __syncthreads();
    if (tid < C) {  // lnff affine gradients
      for (int t = 0; t < T; ++t) {
        gg2 += DY[t * C + tid] * G1[t * C + tid];
        gbe2 += DY[t * C + tid];
      }
    }
    __syncthreads();
    for (int t = wave; t < T; t += TA_THREADS / 64) {  // LayerNorm (lnff) backward -> dF
      const float fh = G1[t * C + lane];
      const float g = DY[t * C + lane] * vec[VEC_G2 + lane];
      const float m1 = warp_sum(g) * (1.f / C), m2 = warp_sum(g * fh) * (1.f / C);
      DY[t * C + lane] = R2[t] * (g - m1 - fh * m2);
    }
    for (int i = tid; i < T * C; i += TA_THREADS) {
      const int c = i % C;
      Y1[i] = X1[i] * vec[VEC_G1 + c] + vec[VEC_BE1 + c];
    }
    __syncthreads();
    // dW2[c][k] += sum_t dF[t][c] u[t][k]; dU = (dF W2) * (u > 0)
#pragma unroll 1
    for (int t = 0; t < T; ++t) {
      const float d = DY[t * C + ro];
#pragma unroll
      for (int e = 0; e < 8; ++e) gW2[e] += d * U[t * C + co + e];
    }
    if (tid < C)
      for (int t = 0; t < T; ++t) gbf2 += DY[t * C + tid];
    for (int i = tid; i < T * C; i += TA_THREADS) {
      const int t = i / C, k = i - t * C;
      float acc = 0.f;
      if (U[i] > 0.f)
        for (int c = 0; c < C; ++c) acc += DY[t * C + c] * W2[c * C + k];
      G1[i] = acc;
    }
    __syncthreads();
    // dW1[k][c] += sum_t dU[t][k] y1[t][c]; dY1 = dU W1 + dF (in place)
#pragma unroll 1
    for (int t = 0; t < T; ++t) {
      const float d = G1[t * C + ro];
#pragma unroll
      for (int e = 0; e < 8; ++e) gW1[e] += d * Y1[t * C + co + e];
    }
    if (tid < C)
      for (int t = 0; t < T; ++t) gbf1 += G1[t * C + tid];
    for (int i = tid; i < T * C; i += TA_THREADS) {
      const int t = i / C, c = i - t * C;
      float acc = DY[i];
      for (int k = 0; k < C; ++k) acc += G1[t * C + k] * W1[k * C + c];
      DY[i] = acc;
    }
    __syncthreads();
    if (tid < C) {  // ln affine gradients
      for (int t = 0; t < T; ++t) {
        gg1 += DY[t * C + tid] * X1[t * C + tid];
        gbe1 += DY[t * C + tid];
      }
    }
    __syncthreads();
    for (int t = wave; t < T; t += TA_THREADS / 64) {  // LayerNorm (ln) backward -> dO1
      const float xh = X1[t * C + lane];
      const float g = DY[t * C + lane] * vec[VEC_G1 + lane];
      const float m1 = warp_sum(g) * (1.f / C), m2 = warp_sum(g * xh) * (1.f / C);
      DY[t * C + lane] = R1[t] * (g - m1 - xh * m2);
    }
    __syncthreads();
    // o1 = P v + x: dX = dO1, dP = dO1 v^T, dV = P^T dO1 (into U)
    for (int i = tid; i < T * C; i += TA_THREADS) {
      const int u = i / C, c = i - u * C;
      DX[i] = DY[i];
      float acc = 0.f;
      for (int t = 0; t < T; ++t) acc += P[t * T + u] * DY[t * C + c];
      U[i] = acc;
    }
    for (int i = tid; i < T * T; i += TA_THREADS) {
      const int t = i / T, u = i - t * T;
      float acc = 0.f;
      for (int c = 0; c < C; ++c) acc += DY[t * C + c] * Vv[u * C + c];
      dP[i] = acc;
    }
    __syncthreads();
    for (int t = wave; t < T; t += TA_THREADS / 64) {  // softmax backward, / sqrt(C)
      const float p = lane < T ? P[t * T + lane] : 0.f;
      const float dp = lane < T ? dP[t * T + lane] : 0.f;
      const float dot = warp_sum(p * dp);
      if (lane < T) dP[t * T + lane] = p * (dp - dot) * 0.125f;
    }
#pragma unroll 1
    for (int t = 0; t < T; ++t) {  // dWv[c][c2] += sum_t dV[t][c] x[t][c2]
      const float d = U[t * C + ro];
#pragma unroll
      for (int e = 0; e < 8; ++e) gWv[e] += d * Xs[t * C + co + e];
    }
    if (tid < C)
      for (int t = 0; t < T; ++t) gbv += U[t * C + tid];
    for (int i = tid; i < T * C; i += TA_THREADS) {
      const int t = i / C, c2 = i - t * C;
      float acc = 0.f;
      for (int c = 0; c < C; ++c) acc += U[t * C + c] * Wv[c * C + c2];
      DX[i] += acc;
    }
    __syncthreads();
    // dq = dA k (into G1), dk = dA^T q (into Y1)
    for (int i = tid; i < 2 * T * CQ; i += TA_THREADS) {
      const int which = i / (T * CQ), rem = i - which * T * CQ, t = rem / CQ, cq = rem - t * CQ;
      float acc = 0.f;
      if (which == 0) {
        for (int u = 0; u < T; ++u) acc += dP[t * T + u] * K[u * CQ + cq];
        G1[rem] = acc;
      } else {
        for (int u = 0; u < T; ++u) acc += dP[u * T + t] * Q[u * CQ + cq];
        Y1[rem] = acc;
      }
    }
    __syncthreads();
#pragma unroll
    for (int e = 0; e < 6; ++e) {  // conv weight gradients dW[tq][t][j] += sum_c' d[tq][c'] x[t][c'+j]
      const int idx = tid + e * TA_THREADS;
      if (idx < T * T * 3) {
        const int tq = idx / (T * 3), r = idx - tq * T * 3, t = r / 3, j = r - t * 3;
        float s1 = 0.f, s2 = 0.f;
#pragma unroll 2
        for (int c = 0; c < CQ; ++c) {
          const float x = Xs[t * C + c + j];
          s1 += G1[tq * CQ + c] * x;
          s2 += Y1[tq * CQ + c] * x;
        }
        gc1[e] += s1;
        gc2[e] += s2;
      }
    }
    if (tid >= 64 && tid < 64 + T)
      for (int c = 0; c < CQ; ++c) gcb += G1[(tid - 64) * CQ + c];
    if (tid >= 128 && tid < 128 + T)
      for (int c = 0; c < CQ; ++c) gcb += Y1[(tid - 128) * CQ + c];
    for (int i = tid; i < T * C; i += TA_THREADS) {
      const int t = i / C, c = i - t * C;
      float acc = 0.f;
#pragma unroll 1
      for (int tq = 0; tq < T; ++tq) {
#pragma unroll
        for (int j = 0; j < 3; ++j) {
          const int cq = c - j;
          if (cq >= 0 && cq < CQ)
            acc += cw1[(tq * T + t) * 3 + j] * G1[tq * CQ + cq] + cw2[(tq * T + t) * 3 + j] * Y1[tq * CQ + cq];
        }
      }
      DX[i] += acc;
    }
    __syncthreads();
    for (int i = tid; i < T * C; i += TA_THREADS) {
      const int t = i / C;
      a.din[(((size_t)b * T + t) * V + n) * C + (i - t * C)] = DX[i];
    }
  }
  float* G = a.grads;
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    atomic_add_f(G + a.off_f2w + ro * C + co + e, gW2[e]);
    atomic_add_f(G + a.off_f0w + ro * C + co + e, gW1[e]);
    atomic_add_f(G + a.off_vw + ro * C + co + e, gWv[e]);
  }
#pragma unroll
  for (int e = 0; e < 6; ++e) {
    const int idx = tid + e * TA_THREADS;
    if (idx < T * T * 3) {
      atomic_add_f(G + a.off_c1w + idx, gc1[e]);
      atomic_add_f(G + a.off_c2w + idx, gc2[e]);
    }
  }
  if (tid < C) {
    atomic_add_f(G + a.off_vb + tid, gbv);
    atomic_add_f(G + a.off_f0b + tid, gbf1);
    atomic_add_f(G + a.off_f2b + tid, gbf2);
    atomic_add_f(G + a.off_lnw + tid, gg1);
    atomic_add_f(G + a.off_lnb + tid, gbe1);
    atomic_add_f(G + a.off_lnffw + tid, gg2);
    atomic_add_f(G + a.off_lnffb + tid, gbe2);
  }
  if (tid >= 64 && tid < 64 + T) atomic_add_f(G + a.off_c1b + tid - 64, gcb);
  if (tid >= 128 && tid < 128 + T) atomic_add_f(G + a.off_c2b + tid - 128, gcb);
}

}  // namespace tg
}  // namespace f3

using namespace f3;
using namespace f3::tg;

namespace {
template <typename K>
void allow_lds(K kernel, int bytes) {
  if (bytes > 64 * 1024) (void)hipFuncSetAttribute((const void*)kernel, hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
}
template <bool B16>
int gru_lds(int V, bool bwd) {
  using TT = typename Op<B16>::T;
  const int bt = bwd ? Op<B16>::BTB : Op<B16>::BTF;
  return (bwd ? 4 : 2) * V * bt * Op<B16>::XS * (int)sizeof(TT) + (V * V + V) * 4;
}
}  // namespace

int f3_tg_gru_lds_ok(int V) {
  return V >= 2 && V <= VMAX && gru_lds<true>(V, true) <= 160 * 1024 && gru_lds<true>(V, false) <= 160 * 1024 &&
         gru_lds<false>(V, true) <= 160 * 1024;
}

int f3_tg_supports(const float* E, int V, float* S, float* cs, hipStream_t s) {
  hipLaunchKernelGGL(tg_supports_kernel, dim3(1), dim3(256), 0, s, E, V, S, cs);
  F3_LAUNCH_CHECK();
  return F3_OK;
}

int f3_tg_prep(const PrepArgs* a, int b16, hipStream_t s) {
  const long long n = (long long)a->V * IP * a->O + (long long)a->O * IP + (long long)a->V * a->O;
  const dim3 grid((unsigned)((n + 255) / 256));
  if (b16) hipLaunchKernelGGL(tg_prep_kernel<true>, grid, dim3(256), 0, s, *a);
  else hipLaunchKernelGGL(tg_prep_kernel<false>, grid, dim3(256), 0, s, *a);
  F3_LAUNCH_CHECK();
  return F3_OK;
}

template <bool B16>
static int gru_fwd_launch(const GruFwdArgs& a, hipStream_t s) {
  const int lds = gru_lds<B16>(a.V, false);
  static bool once = (allow_lds(gru_fwd_kernel<B16>, 160 * 1024), true);
  (void)once;
  const int grid = (a.B + Op<B16>::BTF - 1) / Op<B16>::BTF;
  hipLaunchKernelGGL(gru_fwd_kernel<B16>, dim3(grid), dim3(GRU_THREADS), lds, s, a);
  F3_LAUNCH_CHECK();
  return F3_OK;
}

template <bool B16>
static int gru_bwd_launch(const GruBwdArgs& a, hipStream_t s) {
  const int lds = gru_lds<B16>(a.V, true);
  static bool once = (allow_lds(gru_bwd_kernel<B16>, 160 * 1024), true);
  (void)once;
  const int grid = (a.B + Op<B16>::BTB - 1) / Op<B16>::BTB;
  hipLaunchKernelGGL(gru_bwd_kernel<B16>, dim3(grid), dim3(GRU_THREADS), lds, s, a);
  F3_LAUNCH_CHECK();
  return F3_OK;
}

int f3_tg_gru_fwd(const GruFwdArgs* a, int b16, hipStream_t s) {
  if (!f3_tg_gru_lds_ok(a->V) || a->I > IP || a->B < 1) return F3_EINVAL;
  return b16 ? gru_fwd_launch<true>(*a, s) : gru_fwd_launch<false>(*a, s);
}

int f3_tg_gru_bwd(const GruBwdArgs* a, int b16, hipStream_t s) {
  if (!f3_tg_gru_lds_ok(a->V) || a->I > IP || a->B < 1) return F3_EINVAL;
  return b16 ? gru_bwd_launch<true>(*a, s) : gru_bwd_launch<false>(*a, s);
}

int f3_tg_supp_grad(const SuppGradArgs* a, int b16, hipStream_t s) {
  const int grid = std::min(1024, std::max(1, a->rows / 4));
  if (b16) hipLaunchKernelGGL(tg_supp_grad_kernel<true>, dim3(grid), dim3(256), 0, s, *a);
  else hipLaunchKernelGGL(tg_supp_grad_kernel<false>, dim3(grid), dim3(256), 0, s, *a);
  F3_LAUNCH_CHECK();
  return F3_OK;
}

int f3_tg_pool_grad(const PoolGradArgs* a, hipStream_t s) {
  const long long n = (long long)EMB * a->I * a->O + (long long)EMB * a->O + (long long)a->O * a->I + a->O;
  hipLaunchKernelGGL(tg_pool_grad_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, *a);
  F3_LAUNCH_CHECK();
  hipLaunchKernelGGL(tg_pool_dE_kernel, dim3(a->V * EMB), dim3(256), 0, s, *a);
  F3_LAUNCH_CHECK();
  return F3_OK;
}

int f3_tg_supports_bwd(const float* E, int V, const float* dS, float* gE, hipStream_t s) {
  hipLaunchKernelGGL(tg_supports_bwd_kernel, dim3(1), dim3(256), 0, s, E, V, dS, gE);
  F3_LAUNCH_CHECK();
  return F3_OK;
}

int f3_tg_endconv_mean(const float* W, const float* b, float* Wm, float* bm, hipStream_t s) {
  hipLaunchKernelGGL(tg_endconv_mean_kernel, dim3((C * KH + C + 255) / 256), dim3(256), 0, s, W, b, Wm, bm);
  F3_LAUNCH_CHECK();
  return F3_OK;
}

int f3_tg_pool_fwd(const float* Y, int B, int V, const float* Wm, const float* bm, float* xm, float* pooled,
                   hipStream_t s) {
  hipLaunchKernelGGL(tg_pool_fwd_kernel, dim3(B), dim3(256), 0, s, Y, V, Wm, bm, xm, pooled);
  F3_LAUNCH_CHECK();
  return F3_OK;
}

int f3_tg_pool_bwd(const float* dpooled, const float* xm, const float* Wm, int B, int V, float* dY, float* gW, float* gb,
                   hipStream_t s) {
  hipLaunchKernelGGL(tg_pool_bwd_data_kernel, dim3(B), dim3(256), 0, s, dpooled, Wm, V, dY);
  F3_LAUNCH_CHECK();
  hipLaunchKernelGGL(tg_pool_bwd_weight_kernel, dim3((C * KH + C + 255) / 256), dim3(256), 0, s, dpooled, xm, B, gW, gb);
  F3_LAUNCH_CHECK();
  return F3_OK;
}

static int ta_grid(const TaArgs& a) {
  int dev = 0, cus = 256;
  if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  (void)hipGetLastError();
  return std::max(1, std::min(cus, a.B * a.V));
}

int f3_tg_ta_fwd(const TaArgs* a, hipStream_t s) {
  static bool once = (allow_lds(ta_fwd_kernel, TA_FWD_LDS), true);
  (void)once;
  hipLaunchKernelGGL(ta_fwd_kernel, dim3(ta_grid(*a)), dim3(TA_THREADS), TA_FWD_LDS, s, *a);
  F3_LAUNCH_CHECK();
  return F3_OK;
}

int f3_tg_ta_bwd(const TaArgs* a, hipStream_t s) {
  static bool once = (allow_lds(ta_bwd_kernel, TA_BWD_LDS), true);
  (void)once;
  hipLaunchKernelGGL(ta_bwd_kernel, dim3(ta_grid(*a)), dim3(TA_THREADS), TA_BWD_LDS, s, *a);
  F3_LAUNCH_CHECK();
  return F3_OK;
}
