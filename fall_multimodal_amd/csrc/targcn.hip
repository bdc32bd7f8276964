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
#include <cstring>
#include <type_traits>

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
  static constexpr int BTF = 4;       // clips per workgroup, forward. MFMA rows 4-15 idle: the step
                                      // time of a workgroup is set by its weight stream, not its row
                                      // count, and fewer clips per workgroup spread the per-step
                                      // stores over more CUs (64 workgroups at B = 256)
  static constexpr int BTB = 3;       // backward (four [node][clip][k] buffers + the step's staged
                                      // fp32 inputs in LDS)
};
template <>
struct Op<false> {
  typedef float T;
  static constexpr int KS = 4;        // v_mfma_f32_16x16x4_f32 (exact fp32 products)
  static constexpr int XS = IP + 4;
  static constexpr int BTF = 4;
  static constexpr int BTB = 1;
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

F3_DEV bf16x8_t ld8(const __bf16* p) { return *reinterpret_cast<const bf16x8_t*>(p); }
F3_DEV f32x4 mfma8(bf16x8_t a, bf16x8_t b, f32x4 c) { return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0); }

F3_DEV float silu_grad(float s) {  // d/ds s*sigmoid(s)
  const float g = sigmoidf_(s);
  return g * (1.f + s * (1.f - g));
}

// out[n][b][k] (+)= sum_m S'[n][m] in[m][b][k] for k < I; S' = S (forward mix, EmbGCN.py:84)
// or S^T (its input gradient). Each thread owns one output node n (its S' row in registers) and
// walks 8-element chunks (b, k..k+7) with 16-B LDS reads: V reads + 8V FMAs per chunk.
template <typename TY, int BT, int XS, bool TRANS, bool ACC, int NT>
F3_DEV void node_mix(const TY* in, TY* out, const float* Sl, int V, int I, int tid) {
  const int tpn = NT / V;            // threads per output node
  int tl = tid;
  asm volatile("" : "+v"(tl));       // per call: keep the S row out of loop-invariant registers
  const int n = tl / tpn, sub = tl - n * tpn;
  if (n >= V) return;
  const int k8 = (I + 7) >> 3;
  const float* srow = Sl + (TRANS ? n : n * V);
  const int sstr = TRANS ? V : 1;
  for (int cidx = sub; cidx < BT * k8; cidx += tpn) {
    const int b = cidx / k8, k = (cidx - b * k8) * 8;
    float acc[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) acc[e] = 0.f;
#pragma unroll 2
    for (int m = 0; m < V; ++m) {
      const TY* src = in + (m * BT + b) * XS + k;
      const float sm = srow[m * sstr];
      float x[8];
      if constexpr (sizeof(TY) == 2) {
        const bf16x8_t v = *reinterpret_cast<const bf16x8_t*>(src);
#pragma unroll
        for (int e = 0; e < 8; ++e) x[e] = (float)v[e];
      } else {
        const f32x4 v0 = *reinterpret_cast<const f32x4*>(src), v1 = *reinterpret_cast<const f32x4*>(src + 4);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          x[e] = v0[e];
          x[e + 4] = v1[e];
        }
      }
#pragma unroll
      for (int e = 0; e < 8; ++e) acc[e] += sm * x[e];
    }
    TY* dst = out + (n * BT + b) * XS + k;
    if constexpr (sizeof(TY) == 2) {
      bf16x8_t o;
      if (ACC) {
        const bf16x8_t prev = *reinterpret_cast<const bf16x8_t*>(dst);
#pragma unroll
        for (int e = 0; e < 8; ++e) o[e] = (__bf16)((float)prev[e] + acc[e]);
      } else {
#pragma unroll
        for (int e = 0; e < 8; ++e) o[e] = (__bf16)acc[e];
      }
      *reinterpret_cast<bf16x8_t*>(dst) = o;
    } else {
      f32x4 o0, o1;
      if (ACC) {
        o0 = *reinterpret_cast<const f32x4*>(dst);
        o1 = *reinterpret_cast<const f32x4*>(dst + 4);
      } else {
        o0 = f32x4{0.f, 0.f, 0.f, 0.f};
        o1 = o0;
      }
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        o0[e] += acc[e];
        o1[e] += acc[e + 4];
      }
      *reinterpret_cast<f32x4*>(dst) = o0;
      *reinterpret_cast<f32x4*>(dst + 4) = o1;
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
    typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
    const u32x4 v = *reinterpret_cast<const u32x4*>(reinterpret_cast<const char*>(L + row * XS) + ch * 16);
    __builtin_nontemporal_store(v, reinterpret_cast<u32x4*>(reinterpret_cast<char*>(dst) + R * IP * sizeof(TY) + ch * 16));
  }
}

// F3_TG_PROF: workgroup 0 records wall-clock stamps at the recurrence's phase boundaries
#define F3_TG_STAMP(k) \
  do { if (a.prof && blockIdx.x == 0 && threadIdx.x == 0) a.prof[t * 8 + (k)] = wall_clock64(); } while (0)

constexpr int GRU_THREADS = 512;
constexpr int GRU_WAVES = GRU_THREADS / 64;
constexpr int NJ = (4 * VMAX + GRU_WAVES - 1) / GRU_WAVES;  // owned (node, 16-column tile) jobs per wave

// ---------------------------------------------------------------------------------------------
// Forward recurrence of one GRU layer (GRU.py:17-27 over TRAGCN.py:162-164's time loop).
// ---------------------------------------------------------------------------------------------
// Gate / update GEMM jobs of the forward recurrence. A job = (node n, 16-column tile j): the gate
// job computes the z and r column tiles of both EmbGCN products (4 MFMA tiles), the update job the
// candidate tile (2 MFMA tiles). Jobs are dealt round-robin over the 8 waves, so a wave's jobs all
// share j = wave % 4: the Linear (static-branch) weight tiles are the same for every job of a wave
// and stay in registers for the whole kernel; only the node weights W_n stream from L2. bf16: the
// K = IP reduction is 4 MFMA steps; all of a job's W_n fragments are loaded before its first MFMA,
// and job jj+1's fragments are issued before job jj computes and stores (vmcnt counts loads and
// stores in issue order, so a job never waits on the previous job's epilogue stores). fp32
// (parity mode): a plain k loop.
template <bool B16>
struct GateJob {  // node weights of the z and r column tiles (the shared Linear tiles stay resident)
  static constexpr int NW = B16 ? 2 * (IP / 32) : 1;
  typename std::conditional<B16, bf16x8_t, float>::type w[NW];
  float bv[2];
};
template <bool B16>
struct UpdJob {
  static constexpr int NW = B16 ? IP / 32 : 1;
  typename std::conditional<B16, bf16x8_t, float>::type w[NW];
  float bv;
};

template <bool B16>
__global__ __launch_bounds__(GRU_THREADS) void gru_fwd_kernel(GruFwdArgs a) {
  using TT = typename Op<B16>::T;
  constexpr int BT = Op<B16>::BTF, XS = Op<B16>::XS, KS = Op<B16>::KS;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int V = a.V, Din = a.Din, I = a.I;
  TT* X = reinterpret_cast<TT*>(smem);           // [V][BT][XS] EmbGCN input [x, h] / [x, r*h]
  TT* Y = X + V * BT * XS;                       // [V][BT][XS] S . input
  float* Hs = reinterpret_cast<float*>(Y + V * BT * XS);  // [V][BT][H] hidden state h (fp32)
  float* Zs = Hs + V * BT * H;                   // [V][BT][H] update gate z of this step
  float* Rs = Zs + V * BT * H;                   // [V][BT][H] reset gate r of this step
  float* Sl = Rs + V * BT * H;
  float* csl = Sl + V * V;
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int b0 = blockIdx.x * BT;
  for (int i = tid; i < 2 * V * BT * XS; i += GRU_THREADS) X[i] = (TT)0.f;
  for (int i = tid; i < 3 * V * BT * H; i += GRU_THREADS) Hs[i] = 0.f;  // h0 = 0 (TRAGCN.py:171-175)
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

  static_assert(GRU_WAVES % 4 == 0, "a wave's jobs share one column tile");
  const int jw = wave & 3, cw = 16 * jw + col;  // this wave's column tile / this lane's column
  // resident Linear tiles (gate z / r, update) and the Linear biases of this lane's column
  typename std::conditional<B16, bf16x8_t, float>::type lgz[B16 ? IP / 32 : 1], lgr[B16 ? IP / 32 : 1],
      lup[B16 ? IP / 32 : 1];
  if constexpr (B16) {
#pragma unroll
    for (int ks = 0; ks < IP / 32; ++ks) {
      lgz[ks] = ld8(gLf + (size_t)cw * IP + kofs + 32 * ks);
      lgr[ks] = ld8(gLf + (size_t)(H + cw) * IP + kofs + 32 * ks);
      lup[ks] = ld8(uLf + (size_t)cw * IP + kofs + 32 * ks);
    }
  }
  const float blz = a.g.bl[cw], blr = a.g.bl[H + cw], blu = a.u.bl[cw];

  auto gate_load = [&](int jj, GateJob<B16>& J) {
    int q = wave + GRU_WAVES * jj;
    asm volatile("" : "+s"(q));
    if (q < njobs) {
      const int n = q >> 2;
      if constexpr (B16) {
        const TT* wz = gWf + ((size_t)n * 2 * H + cw) * IP + kofs;
#pragma unroll
        for (int ks = 0; ks < IP / 32; ++ks) {
          J.w[ks] = ld8(wz + 32 * ks);
          J.w[IP / 32 + ks] = ld8(wz + (size_t)H * IP + 32 * ks);
        }
      }
      J.bv[0] = a.g.bn[n * 2 * H + cw];
      J.bv[1] = a.g.bn[n * 2 * H + H + cw];
    }
  };
  // zr = sigmoid(S.x W_n + b_n + silu(cs*x Lin^T + b))   (EmbGCN.py:78-89, GRU.py:22)
  auto gate_compute = [&](int jj, const GateJob<B16>& J, int t) {
    int q = wave + GRU_WAVES * jj;
    asm volatile("" : "+s"(q));
    if (q >= njobs) return;
    const int n = q >> 2;
    f32x4 gz = {0.f, 0.f, 0.f, 0.f}, gr = gz, sz = gz, sr = gz;
    const TT* ay = Y + (n * BT + arow) * XS + kofs;
    const TT* ax = X + (n * BT + arow) * XS + kofs;
    if constexpr (B16) {
#pragma unroll
      for (int ks = 0; ks < IP / 32; ++ks) {
        const bf16x8_t ya = ld8(ay + 32 * ks), xa = ld8(ax + 32 * ks);
        gz = mfma8(ya, J.w[ks], gz);
        gr = mfma8(ya, J.w[IP / 32 + ks], gr);
        sz = mfma8(xa, lgz[ks], sz);
        sr = mfma8(xa, lgr[ks], sr);
      }
    } else {
      const TT* wz = gWf + ((size_t)n * 2 * H + cw) * IP + kofs;
      const TT* lz = gLf + (size_t)cw * IP + kofs;
#pragma unroll 1
      for (int ks = 0; ks < nks; ++ks) {
        const int o = ks * KS;
        gz = mma<B16>(ay + o, wz + o, gz);
        gr = mma<B16>(ay + o, wz + (size_t)H * IP + o, gr);
        sz = mma<B16>(ax + o, lz + o, sz);
        sr = mma<B16>(ax + o, lz + (size_t)H * IP + o, sr);
      }
    }
    const float csn = csl[n];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int b = rq * 4 + r;
      if (b >= BT) continue;
      const float s_z = sz[r] * csn + blz, s_r = sr[r] * csn + blr;
      const float z = sigmoidf_(gz[r] + J.bv[0] + s_z * sigmoidf_(s_z));
      const float rr = sigmoidf_(gr[r] + J.bv[1] + s_r * sigmoidf_(s_r));
      Zs[(n * BT + b) * H + cw] = z;
      Rs[(n * BT + b) * H + cw] = rr;
      if (b0 + b < a.B) {
        const size_t R = ((size_t)(b0 + b) * T + t) * V + n;
        __builtin_nontemporal_store(z, &a.ZR[R * 2 * H + cw]);
        __builtin_nontemporal_store(rr, &a.ZR[R * 2 * H + H + cw]);
        __builtin_nontemporal_store(s_z, &a.SG[R * 2 * H + cw]);
        __builtin_nontemporal_store(s_r, &a.SG[R * 2 * H + H + cw]);
      }
    }
  };
  auto upd_load = [&](int jj, UpdJob<B16>& J) {
    int q = wave + GRU_WAVES * jj;
    asm volatile("" : "+s"(q));
    if (q < njobs) {
      const int n = q >> 2;
      if constexpr (B16) {
        const TT* wu = uWf + ((size_t)n * H + cw) * IP + kofs;
#pragma unroll
        for (int ks = 0; ks < IP / 32; ++ks) J.w[ks] = ld8(wu + 32 * ks);
      }
      J.bv = a.u.bn[n * H + cw];
    }
  };
  // hc = tanh(EmbGCN_u([x, r*h])); h = z*h + (1-z)*hc   (GRU.py:25-26)
  auto upd_compute = [&](int jj, const UpdJob<B16>& J, int t) {
    int q = wave + GRU_WAVES * jj;
    asm volatile("" : "+s"(q));
    if (q >= njobs) return;
    const int n = q >> 2;
    f32x4 gu = {0.f, 0.f, 0.f, 0.f}, su = gu;
    const TT* ay = Y + (n * BT + arow) * XS + kofs;
    const TT* ax = X + (n * BT + arow) * XS + kofs;
    if constexpr (B16) {
#pragma unroll
      for (int ks = 0; ks < IP / 32; ++ks) {
        gu = mfma8(ld8(ay + 32 * ks), J.w[ks], gu);
        su = mfma8(ld8(ax + 32 * ks), lup[ks], su);
      }
    } else {
      const TT* wu = uWf + ((size_t)n * H + cw) * IP + kofs;
      const TT* lu = uLf + (size_t)cw * IP + kofs;
#pragma unroll 1
      for (int ks = 0; ks < nks; ++ks) {
        const int o = ks * KS;
        gu = mma<B16>(ay + o, wu + o, gu);
        su = mma<B16>(ax + o, lu + o, su);
      }
    }
    const float csn = csl[n];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int b = rq * 4 + r;
      if (b >= BT) continue;
      const float s = su[r] * csn + blu;
      const float hc = tanhf(gu[r] + J.bv + s * sigmoidf_(s));
      const float z = Zs[(n * BT + b) * H + cw];
      float& hs = Hs[(n * BT + b) * H + cw];
      const float h = z * hs + (1.f - z) * hc;
      hs = h;
      if (b0 + b < a.B) {
        const size_t R = ((size_t)(b0 + b) * T + t) * V + n;
        __builtin_nontemporal_store(hc, &a.HC[R * H + cw]);
        __builtin_nontemporal_store(s, &a.SU[R * H + cw]);
        __builtin_nontemporal_store(h, &a.Hout[R * H + cw]);
      }
    }
  };

  __syncthreads();
  for (int t = 0; t < T; ++t) {
    F3_TG_STAMP(0);
    // x_t -> X[., ., 0:Din], h -> X[., ., Din:Din+H]
    if (Din % 4 == 0) {  // float4 loads, several in flight per thread
#pragma unroll 4
      for (int i = tid; i < BT * V * (Din / 4); i += GRU_THREADS) {
        const int b = i / (V * (Din / 4)), rem = i - b * V * (Din / 4), n = rem / (Din / 4), c = (rem - n * (Din / 4)) * 4;
        f32x4 v = {0.f, 0.f, 0.f, 0.f};
        if (b0 + b < a.B) v = *reinterpret_cast<const f32x4*>(a.x + ((size_t)(b0 + b) * T + t) * V * Din + rem * 4);
        TT* d = X + (n * BT + b) * XS + c;
#pragma unroll
        for (int e = 0; e < 4; ++e) d[e] = (TT)v[e];
      }
    } else {
#pragma unroll 4
      for (int i = tid; i < BT * V * Din; i += GRU_THREADS) {
        const int b = i / (V * Din), rem = i - b * V * Din, n = rem / Din, c = rem - n * Din;
        const float v = (b0 + b < a.B) ? a.x[((size_t)(b0 + b) * T + t) * V * Din + rem] : 0.f;
        X[(n * BT + b) * XS + c] = (TT)v;
      }
    }
    for (int i = tid; i < V * BT * (H / 4); i += GRU_THREADS) {
      const int row = i / (H / 4), c = (i - row * (H / 4)) * 4;
      const f32x4 h = *reinterpret_cast<const f32x4*>(Hs + row * H + c);
      TT* d = X + row * XS + Din + c;
#pragma unroll
      for (int e = 0; e < 4; ++e) d[e] = (TT)h[e];
    }
    __syncthreads();
    F3_TG_STAMP(1);
    node_mix<TT, BT, XS, false, false, GRU_THREADS>(X, Y, Sl, V, I, tid);
    __syncthreads();
    F3_TG_STAMP(2);
    store_rows<TT, BT, XS, GRU_THREADS>(X, a.XI, V, a.B, b0, t, tid);
    store_rows<TT, BT, XS, GRU_THREADS>(Y, a.XG, V, a.B, b0, t, tid);
    F3_TG_STAMP(7);
    {
      GateJob<B16> JA, JB;
      gate_load(0, JA);
#pragma unroll
      for (int jj = 0; jj < NJ; jj += 2) {
        if (jj + 1 < NJ) gate_load(jj + 1, JB);
        gate_compute(jj, JA, t);
        if (jj + 2 < NJ) gate_load(jj + 2, JA);
        if (jj + 1 < NJ) gate_compute(jj + 1, JB, t);
      }
    }
    __syncthreads();
    F3_TG_STAMP(3);
    // candidate input [x, r*h] (GRU.py:24)
    for (int i = tid; i < V * BT * (H / 4); i += GRU_THREADS) {
      const int row = i / (H / 4), c = (i - row * (H / 4)) * 4;
      const f32x4 h = *reinterpret_cast<const f32x4*>(Hs + row * H + c);
      const f32x4 r = *reinterpret_cast<const f32x4*>(Rs + row * H + c);
      TT* d = X + row * XS + Din + c;
#pragma unroll
      for (int e = 0; e < 4; ++e) d[e] = (TT)(r[e] * h[e]);
    }
    __syncthreads();
    F3_TG_STAMP(4);
    node_mix<TT, BT, XS, false, false, GRU_THREADS>(X, Y, Sl, V, I, tid);
    __syncthreads();
    F3_TG_STAMP(5);
    store_rows<TT, BT, XS, GRU_THREADS>(X, a.UI, V, a.B, b0, t, tid);
    store_rows<TT, BT, XS, GRU_THREADS>(Y, a.UG, V, a.B, b0, t, tid);
    {
      UpdJob<B16> JA, JB;
      upd_load(0, JA);
#pragma unroll
      for (int jj = 0; jj < NJ; jj += 2) {
        if (jj + 1 < NJ) upd_load(jj + 1, JB);
        upd_compute(jj, JA, t);
        if (jj + 2 < NJ) upd_load(jj + 2, JA);
        if (jj + 1 < NJ) upd_compute(jj + 1, JB, t);
      }
    }
    __syncthreads();
    F3_TG_STAMP(6);
  }
}

// ---------------------------------------------------------------------------------------------
// Node-partitioned forward recurrence (bf16 mode; always taken where its shape fits). gru_fwd_kernel keeps
// a clip tile and ALL nodes in one workgroup and re-streams the 17 node weight matrices from L2
// every step (816 KB per step; measured 19 us of gate GEMM + 14 us of update GEMM per 42 us step,
// profiles/r03_gru_phases.txt). Here a GROUP of V workgroups shares a tile of GN_BT clips and
// workgroup (g, n) owns node n: its W_n tiles (gate z, r and update) and the Linear tiles of the
// static branch stay in registers for all 30 steps (each of the 4 waves owns 16 hidden columns:
// 6 x 4 bf16x8 fragments = 96 VGPRs). The node mixing S.[x, h] needs every node's h, so h and r*h
// are exchanged through memory (hx, rhx) with two group barriers per step. The launch is
// cooperative (all workgroups co-resident, or the launch fails and the clip-tile kernel runs);
// a barrier that does not complete within ~2^22 polls sets the error flag (gsync[GN_MAXG]) and
// stops waiting, so a fault never hangs: the net copies the flag to a host status word after the
// launch and the next f3_targcn_* call (or f3_targcn_status) returns F3_EDEVICE.
// Numerics are those of gru_fwd_kernel: X = bf16([x, h]), Y = bf16(sum_m S[n][m] X_m) in fp32
// in m order, fp32 MFMA accumulation, fp32 epilogue and saved tensors.
// ---------------------------------------------------------------------------------------------
constexpr int GN_THREADS = 256;
constexpr int GN_XS = IP + 8;  // LDS row stride (bf16): 272-B rows

// (gn_barrier: common.h)

__global__ __launch_bounds__(GN_THREADS) void gru_fwd_node_kernel(GruFwdArgs a) {
  __shared__ __attribute__((aligned(16))) __bf16 Ys[GN_BT * GN_XS];  // S.[x, h] (gate) / S.[x, r*h] (update)
  __shared__ __attribute__((aligned(16))) __bf16 Xs[GN_BT * GN_XS];  // [x, h] / [x, r*h] of node n
  __shared__ float Sn[VMAX];
  const int V = a.V, Din = a.Din, I = a.I;
  const int NG = gridDim.x / V;
  const int g = blockIdx.x % NG, n = blockIdx.x / NG;
  const int b0 = g * GN_BT;
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int col = lane & 15, rq = lane >> 4, cw = 16 * w + col, kofs = 8 * rq;
  int* cnt = a.gsync + g;
  int* err = a.gsync + GN_MAXG;
  const bool arrive = !(a.dbg_skip_arrive && blockIdx.x == 0);
  for (int i = tid; i < GN_BT * GN_XS; i += GN_THREADS) {
    Ys[i] = (__bf16)0.f;
    Xs[i] = (__bf16)0.f;
  }
  for (int i = tid; i < V; i += GN_THREADS) Sn[i] = a.S[n * V + i];
  // resident weight fragments of this wave's columns (B operands: lane holds W[k = kofs + j][col])
  const __bf16* gWf = reinterpret_cast<const __bf16*>(a.g.Wf);
  const __bf16* gLf = reinterpret_cast<const __bf16*>(a.g.Lf);
  const __bf16* uWf = reinterpret_cast<const __bf16*>(a.u.Wf);
  const __bf16* uLf = reinterpret_cast<const __bf16*>(a.u.Lf);
  bf16x8_t wz[IP / 32], wr[IP / 32], wu[IP / 32], lz[IP / 32], lr[IP / 32], lu[IP / 32];
#pragma unroll
  for (int ks = 0; ks < IP / 32; ++ks) {
    wz[ks] = ld8(gWf + ((size_t)n * 2 * H + cw) * IP + kofs + 32 * ks);
    wr[ks] = ld8(gWf + ((size_t)n * 2 * H + H + cw) * IP + kofs + 32 * ks);
    wu[ks] = ld8(uWf + ((size_t)n * H + cw) * IP + kofs + 32 * ks);
    lz[ks] = ld8(gLf + (size_t)cw * IP + kofs + 32 * ks);
    lr[ks] = ld8(gLf + (size_t)(H + cw) * IP + kofs + 32 * ks);
    lu[ks] = ld8(uLf + (size_t)cw * IP + kofs + 32 * ks);
  }
  const float bz = a.g.bn[n * 2 * H + cw], br = a.g.bn[n * 2 * H + H + cw], bu = a.u.bn[n * H + cw];
  const float blz = a.g.bl[cw], blr = a.g.bl[H + cw], blu = a.u.bl[cw];
  const float csn = a.cs[n];
  float h[2][4], z[2][4];  // own node's h and z of this lane's column, rows x*16 + 4rq + i
#pragma unroll
  for (int x = 0; x < 2; ++x)
#pragma unroll
    for (int i = 0; i < 4; ++i) h[x][i] = z[x][i] = 0.f;
  __syncthreads();
  int nbar = 0;

  // Y h-part (columns Din..Din+H) = sum_m S[n][m] src[m] (bf16 rows [B][V][H]); one (clip, 8-column
  // chunk) per thread (GN_BT * H / 8 = 256)
  auto mix_h = [&](const unsigned short* src, bool zero) {
    const int b = tid >> 3, c8 = (tid & 7) * 8;
    float acc[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) acc[e] = 0.f;
    if (!zero && b0 + b < a.B) {
      const unsigned short* row = src + (size_t)(b0 + b) * V * H + c8;
#pragma unroll 2
      for (int m = 0; m < V; ++m) {
        const bf16x8_t v = ld8(reinterpret_cast<const __bf16*>(row + (size_t)m * H));
        const float sm = Sn[m];
#pragma unroll
        for (int e = 0; e < 8; ++e) acc[e] += sm * (float)v[e];
      }
    }
#pragma unroll
    for (int e = 0; e < 8; ++e) Ys[b * GN_XS + Din + c8 + e] = (__bf16)acc[e];
  };
  // Y x-part and X x-part of step t (x rows [B][T][V][Din] fp32, rounded to bf16 as X is)
  auto mix_x = [&](int t) {
    if (Din % 4 == 0) {  // 16-B rows pieces (layer 1: x = layer 0's h)
      const int D4 = Din / 4;
      for (int q = tid; q < GN_BT * D4; q += GN_THREADS) {
        const int b = q / D4, c = (q - b * D4) * 4;
        float acc[4] = {0.f, 0.f, 0.f, 0.f}, own[4] = {0.f, 0.f, 0.f, 0.f};
        if (b0 + b < a.B) {
          const float* xr = a.x + ((size_t)(b0 + b) * T + t) * V * Din + c;
#pragma unroll 3
          for (int m = 0; m < V; ++m) {
            const f32x4 v4 = *reinterpret_cast<const f32x4*>(xr + (size_t)m * Din);
            const float sm = Sn[m];
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              const float v = (float)(__bf16)v4[e];
              acc[e] += sm * v;
              if (m == n) own[e] = v;
            }
          }
        }
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          Ys[b * GN_XS + c + e] = (__bf16)acc[e];
          Xs[b * GN_XS + c + e] = (__bf16)own[e];
        }
      }
      return;
    }
    for (int q = tid; q < GN_BT * Din; q += GN_THREADS) {
      const int b = q / Din, c = q - b * Din;
      float acc = 0.f, own = 0.f;
      if (b0 + b < a.B) {
        const float* xr = a.x + ((size_t)(b0 + b) * T + t) * V * Din + c;
        for (int m = 0; m < V; ++m) {
          const float v = (float)(__bf16)xr[(size_t)m * Din];
          acc += Sn[m] * v;
          if (m == n) own = v;
        }
      }
      Ys[b * GN_XS + c] = (__bf16)acc;
      Xs[b * GN_XS + c] = (__bf16)own;
    }
  };
  // rows of Xs / Ys -> the saved [R][IP] operand rows of this node (16-B pieces)
  auto save_rows = [&](const __bf16* L, void* dst, int t) {
    for (int q = tid; q < GN_BT * (IP / 8); q += GN_THREADS) {
      const int b = q / (IP / 8), c = q - b * (IP / 8);
      if (b0 + b >= a.B) continue;
      const size_t R = ((size_t)(b0 + b) * T + t) * V + n;
      typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
      const u32x4 v = *reinterpret_cast<const u32x4*>(L + b * GN_XS + c * 8);
      __builtin_nontemporal_store(v, reinterpret_cast<u32x4*>(reinterpret_cast<__bf16*>(dst) + R * IP + c * 8));
    }
  };

  for (int t = 0; t < T; ++t) {
    // ---- gate input: X = [x_t, h_{t-1}] of node n, Y = S.[x_t, h_{t-1}] ----
    mix_x(t);
    mix_h(a.hx, t == 0);
#pragma unroll
    for (int x = 0; x < 2; ++x)
#pragma unroll
      for (int i = 0; i < 4; ++i) Xs[(x * 16 + 4 * rq + i) * GN_XS + Din + cw] = (__bf16)h[x][i];
    __syncthreads();
    save_rows(Xs, a.XI, t);
    save_rows(Ys, a.XG, t);
    // ---- gate: z, r of this wave's 16 columns ----
    float rh[2][4];
#pragma unroll
    for (int x = 0; x < 2; ++x) {
      f32x4 gz = {0.f, 0.f, 0.f, 0.f}, gr = gz, sz = gz, sr = gz;
      const __bf16* ay = Ys + (x * 16 + col) * GN_XS + kofs;
      const __bf16* ax = Xs + (x * 16 + col) * GN_XS + kofs;
#pragma unroll
      for (int ks = 0; ks < IP / 32; ++ks) {
        const bf16x8_t ya = ld8(ay + 32 * ks), xa = ld8(ax + 32 * ks);
        gz = mfma8(ya, wz[ks], gz);
        gr = mfma8(ya, wr[ks], gr);
        sz = mfma8(xa, lz[ks], sz);
        sr = mfma8(xa, lr[ks], sr);
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int b = x * 16 + 4 * rq + i;
        const float s_z = sz[i] * csn + blz, s_r = sr[i] * csn + blr;
        const float zz = sigmoidf_(gz[i] + bz + s_z * sigmoidf_(s_z));
        const float rr = sigmoidf_(gr[i] + br + s_r * sigmoidf_(s_r));
        z[x][i] = zz;
        rh[x][i] = rr * h[x][i];
        if (b0 + b < a.B) {
          const size_t R = ((size_t)(b0 + b) * T + t) * V + n;
          __builtin_nontemporal_store(zz, &a.ZR[R * 2 * H + cw]);
          __builtin_nontemporal_store(rr, &a.ZR[R * 2 * H + H + cw]);
          __builtin_nontemporal_store(s_z, &a.SG[R * 2 * H + cw]);
          __builtin_nontemporal_store(s_r, &a.SG[R * 2 * H + H + cw]);
          a.rhx[((size_t)(b0 + b) * V + n) * H + cw] = __builtin_bit_cast(unsigned short, (__bf16)rh[x][i]);
        }
      }
    }
    gn_barrier(cnt, V * ++nbar, err, arrive);  // every node's r*h (and every wave's reads of Xs / Ys) done
    // ---- update input: X = [x_t, r*h] of node n, Y = S.[x_t, r*h] (x parts unchanged) ----
    mix_h(a.rhx, false);
#pragma unroll
    for (int x = 0; x < 2; ++x)
#pragma unroll
      for (int i = 0; i < 4; ++i) Xs[(x * 16 + 4 * rq + i) * GN_XS + Din + cw] = (__bf16)rh[x][i];
    __syncthreads();
    save_rows(Xs, a.UI, t);
    save_rows(Ys, a.UG, t);
    // ---- update: hc, h ----
#pragma unroll
    for (int x = 0; x < 2; ++x) {
      f32x4 gu = {0.f, 0.f, 0.f, 0.f}, su = gu;
      const __bf16* ay = Ys + (x * 16 + col) * GN_XS + kofs;
      const __bf16* ax = Xs + (x * 16 + col) * GN_XS + kofs;
#pragma unroll
      for (int ks = 0; ks < IP / 32; ++ks) {
        gu = mfma8(ld8(ay + 32 * ks), wu[ks], gu);
        su = mfma8(ld8(ax + 32 * ks), lu[ks], su);
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int b = x * 16 + 4 * rq + i;
        const float sv = su[i] * csn + blu;
        const float hc = tanhf(gu[i] + bu + sv * sigmoidf_(sv));
        const float hn = z[x][i] * h[x][i] + (1.f - z[x][i]) * hc;
        h[x][i] = hn;
        if (b0 + b < a.B) {
          const size_t R = ((size_t)(b0 + b) * T + t) * V + n;
          __builtin_nontemporal_store(hc, &a.HC[R * H + cw]);
          __builtin_nontemporal_store(sv, &a.SU[R * H + cw]);
          __builtin_nontemporal_store(hn, &a.Hout[R * H + cw]);
          a.hx[((size_t)(b0 + b) * V + n) * H + cw] = __builtin_bit_cast(unsigned short, (__bf16)hn);
        }
      }
    }
    gn_barrier(cnt, V * ++nbar, err, arrive);  // every node's h_t (and every wave's reads of Xs / Ys) done
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
  // [7][V*BT][H] fp32: slots 0-4 this step's staged inputs (z; hc / r; su / s_z; h_{t-1}; dH / s_r),
  // 5 dz, 6 the update path's x gradient
  float* ST = reinterpret_cast<float*>(DX + V * BT * XS);
  float* Sl = ST + 7 * V * BT * H;
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
  const int nit2 = (I + 31) / 32;  // jobs of two 16-column input tiles
  const bool has_dx = a.dX != nullptr && Din == H;
  const TT* gWb = reinterpret_cast<const TT*>(a.g.Wb);
  const TT* gLb = reinterpret_cast<const TT*>(a.g.Lb);
  const TT* uWb = reinterpret_cast<const TT*>(a.u.Wb);
  const TT* uLb = reinterpret_cast<const TT*>(a.u.Lb);
  TT* DP = reinterpret_cast<TT*>(a.DP);
  TT* DSG = reinterpret_cast<TT*>(a.DSG);
  TT* DU = reinterpret_cast<TT*>(a.DU);
  TT* DSU = reinterpret_cast<TT*>(a.DSU);
  float dh[NJ][4];
#pragma unroll
  for (int jj = 0; jj < NJ; ++jj)
#pragma unroll
    for (int r = 0; r < 4; ++r) dh[jj][r] = 0.f;
  // Stage up to 5 per-row 64-float slices of this step's saved tensors into ST[slot] with every
  // 16-B load issued before the first LDS write (one round trip per phase instead of one per job).
  struct Src {
    const float* p;
    int ld, coff, tshift, slot;
  };
  auto stage = [&](const Src* src, int nsrc, int t) {
    constexpr int MAXK = (5 * VMAX * BT * (H / 4) + GRU_THREADS - 1) / GRU_THREADS;
    const int per = V * BT * (H / 4), total = nsrc * per;
    f32x4 v[MAXK];
#pragma unroll
    for (int k = 0; k < MAXK; ++k) {
      const int i = tid + k * GRU_THREADS;
      v[k] = f32x4{0.f, 0.f, 0.f, 0.f};
      if (i < total) {
        const int si = i / per, rem = i - si * per, row = rem / (H / 4), c4 = rem - row * (H / 4);
        const int n = row / BT, b = row - n * BT, tt = t + src[si].tshift;
        if (b0 + b < a.B && tt >= 0) {
          const size_t R = ((size_t)(b0 + b) * T + tt) * V + n;
          v[k] = *reinterpret_cast<const f32x4*>(src[si].p + R * src[si].ld + src[si].coff + 4 * c4);
        }
      }
    }
#pragma unroll
    for (int k = 0; k < MAXK; ++k) {
      const int i = tid + k * GRU_THREADS;
      if (i < total) {
        const int si = i / per, rem = i - si * per;
        *reinterpret_cast<f32x4*>(ST + (size_t)src[si].slot * V * BT * H + rem * 4) = v[k];
      }
    }
  };
  __syncthreads();
  for (int t = T - 1; t >= 0; --t) {
    F3_TG_STAMP(0);
    {  // z, hc, su, h_{t-1}, dH of this step
      const Src src[5] = {{a.ZR, 2 * H, 0, 0, 0}, {a.HC, H, 0, 0, 1}, {a.SU, H, 0, 0, 2}, {a.Hout, H, 0, -1, 3},
                          {a.dH, H, 0, 0, 4}};
      stage(src, 5, t);
    }
    F3_TG_STAMP(7);
    __syncthreads();
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
            const int o = (n * BT + b) * H + c, sl = V * BT * H;
            const float g = dh[jj][r] + ST[4 * sl + o];
            const float z = ST[o], hc = ST[sl + o], su = ST[2 * sl + o], hp = ST[3 * sl + o];
            ST[5 * sl + o] = g * (hp - hc);  // dz
            dU = g * (1.f - z) * (1.f - hc * hc);
            dsu = dU * silu_grad(su) * csn;
            dh[jj][r] = g * z;
            __builtin_nontemporal_store((TT)dU, &DU[R * H + c]);
            __builtin_nontemporal_store((TT)dsu, &DSU[R * H + c]);
          }
          if (b < BT) {
            AG[(n * BT + b) * XS + c] = (TT)dU;
            AS[(n * BT + b) * XS + c] = (TT)dsu;
          }
        }
      }
    }
    __syncthreads();
    F3_TG_STAMP(1);
    // update EmbGCN input gradient: GX = dU . W_n^T, DX = (cs dSu) . Lin
    for (int q = wave; q < V * nit2; q += GRU_WAVES) {
      const int n = q / nit2, i0 = 32 * (q - n * nit2) + col, i1 = i0 + 16;
      f32x4 gx0 = {0.f, 0.f, 0.f, 0.f}, gx1 = gx0, sx0 = gx0, sx1 = gx0;
      const TT* aa = AG + (n * BT + arow) * XS + kofs;
      const TT* as = AS + (n * BT + arow) * XS + kofs;
      const TT* wb0 = uWb + ((size_t)n * IP + i0) * H + kofs;
      const TT* wb1 = uWb + ((size_t)n * IP + i1) * H + kofs;
      const TT* lb0 = uLb + (size_t)i0 * H + kofs;
      const TT* lb1 = uLb + (size_t)i1 * H + kofs;
      if constexpr (B16) {  // all weight fragments of the job in flight before the first MFMA
        constexpr int NK = (H) / 32;
        bf16x8_t w0[NK], w1[NK], l0[NK], l1[NK];
#pragma unroll
        for (int ks = 0; ks < NK; ++ks) {
          w0[ks] = ld8(wb0 + 32 * ks);
          w1[ks] = ld8(wb1 + 32 * ks);
          l0[ks] = ld8(lb0 + 32 * ks);
          l1[ks] = ld8(lb1 + 32 * ks);
        }
#pragma unroll
        for (int ks = 0; ks < NK; ++ks) {
          const bf16x8_t ga = ld8(aa + 32 * ks), sa = ld8(as + 32 * ks);
          gx0 = mfma8(ga, w0[ks], gx0);
          gx1 = mfma8(ga, w1[ks], gx1);
          sx0 = mfma8(sa, l0[ks], sx0);
          sx1 = mfma8(sa, l1[ks], sx1);
        }
      } else {
#pragma unroll 1
        for (int ks = 0; ks < (H) / KS; ++ks) {
          const int o = ks * KS;
          gx0 = mma<B16>(aa + o, wb0 + o, gx0);
          gx1 = mma<B16>(aa + o, wb1 + o, gx1);
          sx0 = mma<B16>(as + o, lb0 + o, sx0);
          sx1 = mma<B16>(as + o, lb1 + o, sx1);
        }
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int b = rq * 4 + r;
        if (b < BT) {
          GX[(n * BT + b) * XS + i0] = (TT)gx0[r];
          DX[(n * BT + b) * XS + i0] = (TT)sx0[r];
          GX[(n * BT + b) * XS + i1] = (TT)gx1[r];
          DX[(n * BT + b) * XS + i1] = (TT)sx1[r];
        }
      }
    }
    __syncthreads();
    F3_TG_STAMP(2);
    node_mix<TT, BT, XS, true, true, GRU_THREADS>(GX, DX, Sl, V, I, tid);
    store_rows<TT, BT, XS, GRU_THREADS>(GX, a.DUG, V, a.B, b0, t, tid);
    __syncthreads();
    F3_TG_STAMP(3);
    {  // r, gate static pre-activations (z and h_{t-1} stay staged)
      const Src src[3] = {{a.ZR, 2 * H, H, 0, 1}, {a.SG, 2 * H, 0, 0, 2}, {a.SG, 2 * H, H, 0, 4}};
      stage(src, 3, t);
    }
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
            const int o = (n * BT + b) * H + c, sl = V * BT * H;
            const float drh = (float)DX[(n * BT + b) * XS + Din + c];
            const float z = ST[o], rr = ST[sl + o], hp = ST[3 * sl + o];
            dh[jj][r] += drh * rr;
            if (has_dx) ST[6 * sl + o] = (float)DX[(n * BT + b) * XS + c];
            dPz = ST[5 * sl + o] * z * (1.f - z);
            dPr = drh * hp * rr * (1.f - rr);
            dsz = dPz * silu_grad(ST[2 * sl + o]) * csn;
            dsr = dPr * silu_grad(ST[4 * sl + o]) * csn;
            __builtin_nontemporal_store((TT)dPz, &DP[R * 2 * H + c]);
            __builtin_nontemporal_store((TT)dPr, &DP[R * 2 * H + H + c]);
            __builtin_nontemporal_store((TT)dsz, &DSG[R * 2 * H + c]);
            __builtin_nontemporal_store((TT)dsr, &DSG[R * 2 * H + H + c]);
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
    F3_TG_STAMP(4);
    // gate EmbGCN input gradient (K = 2H)
    for (int q = wave; q < V * nit2; q += GRU_WAVES) {
      const int n = q / nit2, i0 = 32 * (q - n * nit2) + col, i1 = i0 + 16;
      f32x4 gx0 = {0.f, 0.f, 0.f, 0.f}, gx1 = gx0, sx0 = gx0, sx1 = gx0;
      const TT* aa = AG + (n * BT + arow) * XS + kofs;
      const TT* as = AS + (n * BT + arow) * XS + kofs;
      const TT* wb0 = gWb + ((size_t)n * IP + i0) * 2 * H + kofs;
      const TT* wb1 = gWb + ((size_t)n * IP + i1) * 2 * H + kofs;
      const TT* lb0 = gLb + (size_t)i0 * 2 * H + kofs;
      const TT* lb1 = gLb + (size_t)i1 * 2 * H + kofs;
      if constexpr (B16) {  // all weight fragments of the job in flight before the first MFMA
        constexpr int NK = (2 * H) / 32;
        bf16x8_t w0[NK], w1[NK], l0[NK], l1[NK];
#pragma unroll
        for (int ks = 0; ks < NK; ++ks) {
          w0[ks] = ld8(wb0 + 32 * ks);
          w1[ks] = ld8(wb1 + 32 * ks);
          l0[ks] = ld8(lb0 + 32 * ks);
          l1[ks] = ld8(lb1 + 32 * ks);
        }
#pragma unroll
        for (int ks = 0; ks < NK; ++ks) {
          const bf16x8_t ga = ld8(aa + 32 * ks), sa = ld8(as + 32 * ks);
          gx0 = mfma8(ga, w0[ks], gx0);
          gx1 = mfma8(ga, w1[ks], gx1);
          sx0 = mfma8(sa, l0[ks], sx0);
          sx1 = mfma8(sa, l1[ks], sx1);
        }
      } else {
#pragma unroll 1
        for (int ks = 0; ks < (2 * H) / KS; ++ks) {
          const int o = ks * KS;
          gx0 = mma<B16>(aa + o, wb0 + o, gx0);
          gx1 = mma<B16>(aa + o, wb1 + o, gx1);
          sx0 = mma<B16>(as + o, lb0 + o, sx0);
          sx1 = mma<B16>(as + o, lb1 + o, sx1);
        }
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int b = rq * 4 + r;
        if (b < BT) {
          GX[(n * BT + b) * XS + i0] = (TT)gx0[r];
          DX[(n * BT + b) * XS + i0] = (TT)sx0[r];
          GX[(n * BT + b) * XS + i1] = (TT)gx1[r];
          DX[(n * BT + b) * XS + i1] = (TT)sx1[r];
        }
      }
    }
    __syncthreads();
    F3_TG_STAMP(5);
    node_mix<TT, BT, XS, true, true, GRU_THREADS>(GX, DX, Sl, V, I, tid);
    store_rows<TT, BT, XS, GRU_THREADS>(GX, a.DXG, V, a.B, b0, t, tid);
    __syncthreads();
    F3_TG_STAMP(6);
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
              __builtin_nontemporal_store(ST[6 * V * BT * H + (n * BT + b) * H + c] + (float)DX[(n * BT + b) * XS + c],
                                          &a.dX[R * H + c]);
            }
          }
        }
      }
    }
  }
}

// ---------------------------------------------------------------------------------------------
// Node-partitioned backward recurrence (bf16 mode, where its shape fits): the layout of
// gru_fwd_node_kernel applied to gru_bwd_kernel's step. Workgroup (g, n) owns node n of a tile of
// GN_BT clips: its Wb / Lb tiles (the input-gradient B operands of both EmbGCN products) stay in
// registers, the element-wise epilogues touch only node n's rows, and the two S^T mixes of the
// d(mixed input) rows (update, then gate) read every node's rows from the exchange buffers gx1 /
// gx2 after a group barrier. Wave w owns hidden columns [16w, 16w+16) for the epilogues and
// input-gradient columns [32w, 32w+32) for the GEMMs. Numerics as gru_bwd_kernel: bf16 A operands
// and stored gradients, fp32 accumulation, DX = bf16(bf16(static) + sum_m S[m][n] GX_m).
// ---------------------------------------------------------------------------------------------
__global__ __launch_bounds__(GN_THREADS) void gru_bwd_node_kernel(GruBwdArgs a) {
  __shared__ __attribute__((aligned(16))) __bf16 AG[GN_BT * GN_XS];  // d pre-activation (gconv A)
  __shared__ __attribute__((aligned(16))) __bf16 AS[GN_BT * GN_XS];  // cs * d static pre-activation
  __shared__ __attribute__((aligned(16))) __bf16 GXs[GN_BT * GN_XS]; // this node's d mixed input
  __shared__ __attribute__((aligned(16))) __bf16 DXs[GN_BT * GN_XS]; // this node's d input
  __shared__ float Sc[VMAX];                                          // column n of S
  const int V = a.V, Din = a.Din, I = a.I;
  const int NG = gridDim.x / V;
  const int g = blockIdx.x % NG, n = blockIdx.x / NG;
  const int b0 = g * GN_BT;
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int col = lane & 15, rq = lane >> 4, cw = 16 * w + col, kofs = 8 * rq;
  const bool has_dx = a.dX != nullptr && Din == H;
  int* cnt = a.gsync + g;
  int* err = a.gsync + GN_MAXG;
  const bool arrive = !(a.dbg_skip_arrive && blockIdx.x == 0);
  for (int i = tid; i < GN_BT * GN_XS; i += GN_THREADS) {
    AG[i] = (__bf16)0.f;
    AS[i] = (__bf16)0.f;
    GXs[i] = (__bf16)0.f;
    DXs[i] = (__bf16)0.f;
  }
  for (int i = tid; i < V; i += GN_THREADS) Sc[i] = a.S[i * V + n];
  // resident B fragments: output columns i = 32w + 16y + col, k = o (update: H, gate: 2H)
  const __bf16* gWb = reinterpret_cast<const __bf16*>(a.g.Wb);
  const __bf16* gLb = reinterpret_cast<const __bf16*>(a.g.Lb);
  const __bf16* uWb = reinterpret_cast<const __bf16*>(a.u.Wb);
  const __bf16* uLb = reinterpret_cast<const __bf16*>(a.u.Lb);
  bf16x8_t wu[2][H / 32], lu[2][H / 32], wg[2][2 * H / 32], lg[2][2 * H / 32];
#pragma unroll
  for (int y = 0; y < 2; ++y) {
    const int i = 32 * w + 16 * y + col;
#pragma unroll
    for (int ks = 0; ks < H / 32; ++ks) {
      wu[y][ks] = ld8(uWb + ((size_t)n * IP + i) * H + kofs + 32 * ks);
      lu[y][ks] = ld8(uLb + (size_t)i * H + kofs + 32 * ks);
    }
#pragma unroll
    for (int ks = 0; ks < 2 * H / 32; ++ks) {
      wg[y][ks] = ld8(gWb + ((size_t)n * IP + i) * 2 * H + kofs + 32 * ks);
      lg[y][ks] = ld8(gLb + (size_t)i * 2 * H + kofs + 32 * ks);
    }
  }
  const float csn = a.cs[n];
  __bf16* DP = reinterpret_cast<__bf16*>(a.DP);
  __bf16* DSG = reinterpret_cast<__bf16*>(a.DSG);
  __bf16* DU = reinterpret_cast<__bf16*>(a.DU);
  __bf16* DSU = reinterpret_cast<__bf16*>(a.DSU);
  float dh[2][4], dz[2][4], dxu[2][4];
#pragma unroll
  for (int x = 0; x < 2; ++x)
#pragma unroll
    for (int i = 0; i < 4; ++i) dh[x][i] = dz[x][i] = dxu[x][i] = 0.f;
  __syncthreads();
  int nbar = 0;

  // GEMM: out[b][i] (i = 32w + 16y + col) = sum_k A[b][k] B[k][i] for the two products of one part
  // (gconv A=AG with Wb, static A=AS with Lb), then GXs / DXs (bf16) and the exchange / save rows
  auto part_gemm = [&](auto& wt, auto& lt, auto ksteps_tag) {
    constexpr int KS = decltype(ksteps_tag)::value;
#pragma unroll
    for (int x = 0; x < 2; ++x) {
      f32x4 gx[2], sx[2];
#pragma unroll
      for (int y = 0; y < 2; ++y) gx[y] = sx[y] = f32x4{0.f, 0.f, 0.f, 0.f};
      const __bf16* aa = AG + (x * 16 + col) * GN_XS + kofs;
      const __bf16* as = AS + (x * 16 + col) * GN_XS + kofs;
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        const bf16x8_t ga = ld8(aa + 32 * ks), sa = ld8(as + 32 * ks);
#pragma unroll
        for (int y = 0; y < 2; ++y) {
          gx[y] = mfma8(ga, wt[y][ks], gx[y]);
          sx[y] = mfma8(sa, lt[y][ks], sx[y]);
        }
      }
#pragma unroll
      for (int y = 0; y < 2; ++y)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int b = x * 16 + 4 * rq + i, c = 32 * w + 16 * y + col;
          GXs[b * GN_XS + c] = (__bf16)gx[y][i];
          DXs[b * GN_XS + c] = (__bf16)sx[y][i];
        }
    }
  };
  // this node's GXs rows -> the exchange buffer and the saved [R][IP] rows (16-B pieces)
  auto emit_gx = [&](unsigned short* xch, void* save, int t) {
    for (int q = tid; q < GN_BT * (IP / 8); q += GN_THREADS) {
      const int b = q / (IP / 8), c = q - b * (IP / 8);
      if (b0 + b >= a.B) continue;
      typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
      const u32x4 v = *reinterpret_cast<const u32x4*>(GXs + b * GN_XS + c * 8);
      *reinterpret_cast<u32x4*>(xch + ((size_t)(b0 + b) * V + n) * IP + c * 8) = v;
      const size_t R = ((size_t)(b0 + b) * T + t) * V + n;
      __builtin_nontemporal_store(v, reinterpret_cast<u32x4*>(reinterpret_cast<__bf16*>(save) + R * IP + c * 8));
    }
  };
  // DXs[b][i] = bf16(DXs + sum_m S[m][n] GX_m[b][i]) over every node's exchanged rows (fp32 sum in m order)
  auto mix_t = [&](const unsigned short* xch) {
    for (int q = tid; q < GN_BT * (IP / 8); q += GN_THREADS) {
      const int b = q / (IP / 8), c = (q - b * (IP / 8)) * 8;
      float acc[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) acc[e] = 0.f;
      if (b0 + b < a.B && c < I) {
        const unsigned short* rows = xch + (size_t)(b0 + b) * V * IP + c;
#pragma unroll 2
        for (int m = 0; m < V; ++m) {
          const bf16x8_t v = ld8(reinterpret_cast<const __bf16*>(rows + (size_t)m * IP));
          const float sm = Sc[m];
#pragma unroll
          for (int e = 0; e < 8; ++e) acc[e] += sm * (float)v[e];
        }
      }
      bf16x8_t o = ld8(DXs + b * GN_XS + c);
#pragma unroll
      for (int e = 0; e < 8; ++e) o[e] = (__bf16)((float)o[e] + acc[e]);
      *reinterpret_cast<bf16x8_t*>(DXs + b * GN_XS + c) = o;
    }
  };

  for (int t = T - 1; t >= 0; --t) {
    // ---- update part: h = z*hp + (1-z)*hc ----
    float z[2][4], hp[2][4];
#pragma unroll
    for (int x = 0; x < 2; ++x)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int b = x * 16 + 4 * rq + i;
        float dU = 0.f, dsu = 0.f;
        z[x][i] = hp[x][i] = 0.f;
        if (b0 + b < a.B) {
          const size_t R = ((size_t)(b0 + b) * T + t) * V + n;
          const float zz = a.ZR[R * 2 * H + cw], hc = a.HC[R * H + cw], su = a.SU[R * H + cw];
          const float hpp = t > 0 ? a.Hout[(R - V) * H + cw] : 0.f;
          const float gg = dh[x][i] + a.dH[R * H + cw];
          z[x][i] = zz;
          hp[x][i] = hpp;
          dz[x][i] = gg * (hpp - hc);
          dU = gg * (1.f - zz) * (1.f - hc * hc);
          dsu = dU * silu_grad(su) * csn;
          dh[x][i] = gg * zz;
          __builtin_nontemporal_store((__bf16)dU, &DU[R * H + cw]);
          __builtin_nontemporal_store((__bf16)dsu, &DSU[R * H + cw]);
        }
        AG[b * GN_XS + cw] = (__bf16)dU;
        AS[b * GN_XS + cw] = (__bf16)dsu;
      }
    __syncthreads();
    part_gemm(wu, lu, std::integral_constant<int, H / 32>{});
    __syncthreads();
    emit_gx(a.gx1, a.DUG, t);
    gn_barrier(cnt, V * ++nbar, err, arrive);  // every node's update-part GX rows
    mix_t(a.gx1);
    __syncthreads();
    // ---- gate part ----
#pragma unroll
    for (int x = 0; x < 2; ++x)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int b = x * 16 + 4 * rq + i;
        float dPz = 0.f, dPr = 0.f, dsz = 0.f, dsr = 0.f;
        if (b0 + b < a.B) {
          const size_t R = ((size_t)(b0 + b) * T + t) * V + n;
          const float rr = a.ZR[R * 2 * H + H + cw], sgz = a.SG[R * 2 * H + cw], sgr = a.SG[R * 2 * H + H + cw];
          const float drh = (float)DXs[b * GN_XS + Din + cw];
          dh[x][i] += drh * rr;
          if (has_dx) dxu[x][i] = (float)DXs[b * GN_XS + cw];
          dPz = dz[x][i] * z[x][i] * (1.f - z[x][i]);
          dPr = drh * hp[x][i] * rr * (1.f - rr);
          dsz = dPz * silu_grad(sgz) * csn;
          dsr = dPr * silu_grad(sgr) * csn;
          __builtin_nontemporal_store((__bf16)dPz, &DP[R * 2 * H + cw]);
          __builtin_nontemporal_store((__bf16)dPr, &DP[R * 2 * H + H + cw]);
          __builtin_nontemporal_store((__bf16)dsz, &DSG[R * 2 * H + cw]);
          __builtin_nontemporal_store((__bf16)dsr, &DSG[R * 2 * H + H + cw]);
        }
        AG[b * GN_XS + cw] = (__bf16)dPz;
        AG[b * GN_XS + H + cw] = (__bf16)dPr;
        AS[b * GN_XS + cw] = (__bf16)dsz;
        AS[b * GN_XS + H + cw] = (__bf16)dsr;
      }
    __syncthreads();
    part_gemm(wg, lg, std::integral_constant<int, 2 * H / 32>{});
    __syncthreads();
    emit_gx(a.gx2, a.DXG, t);
    gn_barrier(cnt, V * ++nbar, err, arrive);  // every node's gate-part GX rows
    mix_t(a.gx2);
    __syncthreads();
#pragma unroll
    for (int x = 0; x < 2; ++x)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int b = x * 16 + 4 * rq + i;
        if (b0 + b < a.B) {
          dh[x][i] += (float)DXs[b * GN_XS + Din + cw];
          if (has_dx) {
            const size_t R = ((size_t)(b0 + b) * T + t) * V + n;
            __builtin_nontemporal_store(dxu[x][i] + (float)DXs[b * GN_XS + cw], &a.dX[R * H + cw]);
          }
        }
      }
    __syncthreads();  // DXs / AG / AS are rewritten by the next step
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
  // static adjacency with adj = ones (TRAGCN.py:191): softmax(dim=1) at init, softmax(dim=-1)
  // in forward (one row per thread), then column sums
  __shared__ float M[VMAX * VMAX];
  if (tid < V) {
    const int n = tid;
    const double dgn = 1.0 / ((double)V + 0.5), sq = sqrt(dgn);
    for (int m = 0; m < V; ++m) M[n * V + m] = (float)(sq * ((n == m ? 1.5 : 1.0) * sq));
    for (int pass = 0; pass < 2; ++pass) {
      float mx = -INFINITY, s = 0.f;
      for (int m = 0; m < V; ++m) mx = fmaxf(mx, M[n * V + m]);
      for (int m = 0; m < V; ++m) s += expf(M[n * V + m] - mx);
      for (int m = 0; m < V; ++m) M[n * V + m] = expf(M[n * V + m] - mx) / s;
    }
  }
  __syncthreads();
  if (tid < V) {
    float s = 0.f;
    for (int n = 0; n < V; ++n) s += M[n * V + tid];
    cs[tid] = s;
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

// ---------------------------------------------------------------------------------------------
// Transform.forward on bf16 MFMA (the bf16 mode; TA.py:40-69). One WAVE per (clip, node) sequence:
// every product of the layer is a small GEMM over the sequence's 30 frames (padded to 32), done as
// v_mfma_f32_16x16x32_bf16 tiles with bf16 operands in LDS and fp32 accumulators:
//   Q = sum_j W1_j . X_j + b1   (conv1 (1,3) over T-as-channels: W1_j[t][t'] = conv1.weight[t][t'][0][j],
//                                X_j[t'][c'] = x[t'][c'+j], read as the transposed x shifted by j rows)
//   K likewise (conv2);  V = x . Wv^T + bv
//   A = softmax(Q K^T / sqrt(C)) over the 30 valid columns;  O1 = A . V + x
//   Y1 = LN(O1);  U = relu(Y1 . W0^T + b0);  F = U . W2^T + b2 + Y1;  out = LN(F)
// LayerNorm and softmax reduce a row across the 16 lanes that share it (MFMA C layout: lane l holds
// rows 4(l/16)+i of column l%16). The saved tensors are ta_fwd_kernel's (fp32, same layout), so the
// backward reads either forward's output.
// LDS: the layer's weights in bf16 once per workgroup, and per wave the sequence's x (row-major and
// transposed), Q, K, V^T, P; Y1 and U reuse x's and Q's space.
// ---------------------------------------------------------------------------------------------
constexpr int TAM_WAVES = 4;
constexpr int TAM_LD = 72;   // row stride (bf16) of [32][64] operands: 144-B rows, 16-B aligned
constexpr int TAM_LT = 40;   // row stride of [.][32] operands
constexpr int TAM_W1 = 3 * 32 * TAM_LT;          // one conv weight set [3][32 t][32 t'] (bf16)
constexpr int TAM_WL = 64 * TAM_LD;              // one Linear weight [64 out][64 in] (bf16)
constexpr int TAM_VEC = 10 * 64;                 // b1 b2 bv bf0 bf2 g1 be1 g2 be2 (fp32), 64 each
constexpr int TAM_SEQ = 32 * TAM_LD * 3 + 66 * TAM_LT + 64 * TAM_LT + 32 * TAM_LT;  // per-wave bf16
constexpr int TAM_LDS = (2 * TAM_W1 + 3 * TAM_WL) * 2 + TAM_VEC * 4 + TAM_WAVES * TAM_SEQ * 2;
static_assert(TAM_LDS <= 160 * 1024, "TA MFMA LDS");

// the wave's LDS writes complete (and are not moved) before its next LDS reads
F3_DEV void tam_wsync() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_wave_barrier();
}

F3_DEV f32x4 tam_mfma(bf16x8_t a, bf16x8_t b, f32x4 c) { return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0); }

// acc[x][y] (+)= A[32 x 32*KS] . B, A row-major (stride sa), B as Bt[n][k] row-major (stride sb)
template <int NT, int KSTEPS>
F3_DEV void tam_gemm(f32x4 (&acc)[2][NT], const __bf16* A, int sa, const __bf16* Bt, int sb, int fr, int fg) {
#pragma unroll
  for (int ks = 0; ks < KSTEPS; ++ks) {
    bf16x8_t fa[2], fb[NT];
#pragma unroll
    for (int x = 0; x < 2; ++x) fa[x] = *reinterpret_cast<const bf16x8_t*>(A + (x * 16 + fr) * sa + ks * 32 + fg * 8);
#pragma unroll
    for (int y = 0; y < NT; ++y) fb[y] = *reinterpret_cast<const bf16x8_t*>(Bt + (y * 16 + fr) * sb + ks * 32 + fg * 8);
#pragma unroll
    for (int x = 0; x < 2; ++x)
#pragma unroll
      for (int y = 0; y < NT; ++y) acc[x][y] = tam_mfma(fa[x], fb[y], acc[x][y]);
  }
}

template <int NT>
F3_DEV void tam_zero(f32x4 (&acc)[2][NT]) {
#pragma unroll
  for (int x = 0; x < 2; ++x)
#pragma unroll
    for (int y = 0; y < NT; ++y) acc[x][y] = f32x4{0.f, 0.f, 0.f, 0.f};
}

// sum over the 16 lanes that share a row (lanes 16g .. 16g+15)
F3_DEV float tam_rowsum(float v) {
#pragma unroll
  for (int o = 1; o < 16; o <<= 1) v += __shfl_xor(v, o, 64);
  return v;
}
F3_DEV float tam_rowmax(float v) {
#pragma unroll
  for (int o = 1; o < 16; o <<= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// LayerNorm over the 64 columns of each row of acc (4 tiles x 16 lanes); writes the normalised
// values back (xhat) and returns per-row rstd in rs[x][i]
F3_DEV void tam_layernorm(f32x4 (&acc)[2][4], float (&rs)[2][4]) {
#pragma unroll
  for (int x = 0; x < 2; ++x)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      float s = 0.f;
#pragma unroll
      for (int y = 0; y < 4; ++y) s += acc[x][y][i];
      const float mean = tam_rowsum(s) * (1.f / C);
      float q = 0.f;
#pragma unroll
      for (int y = 0; y < 4; ++y) {
        const float d = acc[x][y][i] - mean;
        acc[x][y][i] = d;
        q += d * d;
      }
      const float r = rsqrtf(tam_rowsum(q) * (1.f / C) + 1e-5f);
      rs[x][i] = r;
#pragma unroll
      for (int y = 0; y < 4; ++y) acc[x][y][i] *= r;
    }
}

__global__ __launch_bounds__(64 * TAM_WAVES) void ta_fwd_mfma_kernel(TaArgs a) {
  extern __shared__ __attribute__((aligned(16))) char tam_smem[];
  __bf16* W1 = reinterpret_cast<__bf16*>(tam_smem);     // [3][32][TAM_LT]
  __bf16* W2 = W1 + TAM_W1;
  __bf16* Wv = W2 + TAM_W1;                               // [64][TAM_LD], [out][in]
  __bf16* Wf0 = Wv + TAM_WL;
  __bf16* Wf2 = Wf0 + TAM_WL;
  float* vec = reinterpret_cast<float*>(Wf2 + TAM_WL);   // [10][64]
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform: scalar sequence pointers
  const float* P_ = a.p;
  for (int i = tid; i < 3 * 32 * 32; i += 64 * TAM_WAVES) {
    const int j = i / 1024, t = (i >> 5) & 31, u = i & 31;
    const bool ok = t < T && u < T;
    W1[j * 32 * TAM_LT + t * TAM_LT + u] = (__bf16)(ok ? P_[a.off_c1w + (t * T + u) * 3 + j] : 0.f);
    W2[j * 32 * TAM_LT + t * TAM_LT + u] = (__bf16)(ok ? P_[a.off_c2w + (t * T + u) * 3 + j] : 0.f);
  }
  for (int i = tid; i < C * C; i += 64 * TAM_WAVES) {
    const int o = i / C, k = i - o * C;
    Wv[o * TAM_LD + k] = (__bf16)P_[a.off_vw + i];
    Wf0[o * TAM_LD + k] = (__bf16)P_[a.off_f0w + i];
    Wf2[o * TAM_LD + k] = (__bf16)P_[a.off_f2w + i];
  }
  for (int i = tid; i < 64; i += 64 * TAM_WAVES) {
    vec[0 * 64 + i] = i < T ? P_[a.off_c1b + i] : 0.f;
    vec[1 * 64 + i] = i < T ? P_[a.off_c2b + i] : 0.f;
    vec[2 * 64 + i] = P_[a.off_vb + i];
    vec[3 * 64 + i] = P_[a.off_f0b + i];
    vec[4 * 64 + i] = P_[a.off_f2b + i];
    vec[5 * 64 + i] = P_[a.off_lnw + i];
    vec[6 * 64 + i] = P_[a.off_lnb + i];
    vec[7 * 64 + i] = P_[a.off_lnffw + i];
    vec[8 * 64 + i] = P_[a.off_lnffb + i];
  }
  // per-wave sequence buffers
  __bf16* xa = reinterpret_cast<__bf16*>(vec + TAM_VEC) + wave * TAM_SEQ;  // [32][LD] x, later Y1
  __bf16* Qs = xa + 32 * TAM_LD;                                            // [32][LD] Q, later U
  __bf16* Ks = Qs + 32 * TAM_LD;                                            // [32][LD]
  __bf16* xt = Ks + 32 * TAM_LD;                                            // [66][LT] x^T (rows 64, 65 zero)
  __bf16* Vt = xt + 66 * TAM_LT;                                            // [64][LT] V^T
  __bf16* Pm = Vt + 64 * TAM_LT;                                            // [32][LT] softmax
  const int fr = lane & 15, fg = lane >> 4;
  // zero the padding the GEMMs read but no sequence writes: x rows 30-31, x^T rows 64-65 and
  // columns 30-31, V^T columns 30-31 (NaN garbage would survive a multiply by zero)
  for (int i = lane; i < 2 * TAM_LD; i += 64) xa[30 * TAM_LD + i] = (__bf16)0.f;
  for (int i = lane; i < 66 * TAM_LT; i += 64) xt[i] = (__bf16)0.f;
  for (int i = lane; i < 64 * TAM_LT; i += 64) Vt[i] = (__bf16)0.f;
  __syncthreads();
  const int V = a.V, nseq = a.B * V;
  for (int sq = blockIdx.x * TAM_WAVES + wave; sq < nseq; sq += gridDim.x * TAM_WAVES) {
    // opaque copies of the lane coordinates (as in ta_bwd_mfma_kernel): the weight fragments are read
    // from LDS per sequence instead of being hoisted out of the loop, which held ~180 registers and
    // left none for the x rows below
    int fr = lane & 15, fg = lane >> 4;
    asm volatile("" : "+v"(fr), "+v"(fg));
    const int b = sq / V, n = sq - b * V;
    float* sv = a.save + (size_t)sq * TA_SAVE;
    const float* xin = a.in + ((size_t)b * T * V + n) * C;  // row t at xin + t*V*C
    const size_t rstride = (size_t)V * C;
    // x (+ PE) into LDS, row-major and transposed; lane = channel. All 30 rows are loaded before the
    // first is used (one memory round trip per sequence instead of 15 dependent pairs)
    float xr[T];
#pragma unroll
    for (int t = 0; t < T; ++t) xr[t] = xin[t * rstride + lane];
    if (a.pe) {
#pragma unroll
      for (int t = 0; t < T; ++t) xr[t] += a.pe[t * C + lane];
    }
#pragma unroll
    for (int t = 0; t < T; ++t) {
      const __bf16 h = (__bf16)xr[t];
      xa[t * TAM_LD + lane] = h;
      xt[lane * TAM_LT + t] = h;
    }
    tam_wsync();  // (each wave works on its own LDS: LDS order within the wave is enough)
    // ---- Q, K (conv (1,3) over T-as-channels), one at a time (register pressure) ----
#pragma unroll 1
    for (int w = 0; w < 2; ++w) {
      f32x4 q[2][4];
      tam_zero(q);
      const __bf16* Wc = w ? W2 : W1;
#pragma unroll
      for (int j = 0; j < 3; ++j) tam_gemm<4, 1>(q, Wc + j * 32 * TAM_LT, TAM_LT, xt + j * TAM_LT, TAM_LT, fr, fg);
      __bf16* dst = w ? Ks : Qs;
      float* svq = sv + (w ? TA_K : TA_Q);
#pragma unroll
      for (int x = 0; x < 2; ++x)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int t = x * 16 + fg * 4 + i;
          const float bt = vec[w * 64 + t];
#pragma unroll
          for (int y = 0; y < 4; ++y) {
            const int c = y * 16 + fr;
            const float qv = c < CQ ? q[x][y][i] + bt : 0.f;
            dst[t * TAM_LD + c] = (__bf16)qv;
            if (t < T && c < CQ) svq[t * CQ + c] = qv;
          }
        }
    }
    {  // V = x Wv^T + bv, stored transposed [c][u] (a lane's 4 rows of one column: 4 consecutive u)
      f32x4 v[2][4];
      tam_zero(v);
      tam_gemm<4, 2>(v, xa, TAM_LD, Wv, TAM_LD, fr, fg);
#pragma unroll
      for (int x = 0; x < 2; ++x)
#pragma unroll
        for (int y = 0; y < 4; ++y) {
          const int c = y * 16 + fr, u0 = x * 16 + fg * 4;
          const float bv = vec[2 * 64 + c];
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const float vv = v[x][y][i] + bv;
            const bool ok = u0 + i < T;
            Vt[c * TAM_LT + u0 + i] = ok ? (__bf16)vv : (__bf16)0.f;
            if (ok) sv[TA_V + (u0 + i) * C + c] = vv;
          }
        }
    }
    tam_wsync();
    // ---- A = softmax(Q K^T / sqrt(C)) over the valid 30 columns ----
    f32x4 s[2][2];
    tam_zero(s);
    tam_gemm<2, 2>(s, Qs, TAM_LD, Ks, TAM_LD, fr, fg);
#pragma unroll
    for (int x = 0; x < 2; ++x)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int t = x * 16 + fg * 4 + i;
        const float s0 = s[x][0][i] * 0.125f;                           // column fr < 16 <= 30
        const float s1 = fr + 16 < T ? s[x][1][i] * 0.125f : -INFINITY;  // column 16 + fr
        const float m = tam_rowmax(fmaxf(s0, s1));
        const float e0 = __expf(s0 - m), e1 = fr + 16 < T ? __expf(s1 - m) : 0.f;
        const float inv = 1.f / tam_rowsum(e0 + e1);
        const float p0 = e0 * inv, p1 = e1 * inv;
        Pm[t * TAM_LT + fr] = (__bf16)p0;
        Pm[t * TAM_LT + 16 + fr] = (__bf16)p1;
        if (t < T) {
          sv[TA_P + t * T + fr] = p0;
          if (fr + 16 < T) sv[TA_P + t * T + 16 + fr] = p1;
        }
      }
    tam_wsync();
    // ---- O1 = A V + x; Y1 = LN(O1) ----
    f32x4 o[2][4];
    tam_zero(o);
    tam_gemm<4, 1>(o, Pm, TAM_LT, Vt, TAM_LT, fr, fg);
#pragma unroll
    for (int x = 0; x < 2; ++x)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int t = min(x * 16 + fg * 4 + i, T - 1);  // rows 30, 31: any finite value
#pragma unroll
        for (int y = 0; y < 4; ++y) {
          const int c = y * 16 + fr;
          float xv = xin[t * rstride + c];
          if (a.pe) xv += a.pe[t * C + c];
          o[x][y][i] += xv;
        }
      }
    float r1[2][4];
    tam_layernorm(o, r1);
#pragma unroll
    for (int x = 0; x < 2; ++x)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int t = x * 16 + fg * 4 + i;
#pragma unroll
        for (int y = 0; y < 4; ++y) {
          const int c = y * 16 + fr;
          const float xh = o[x][y][i];
          const float y1 = xh * vec[5 * 64 + c] + vec[6 * 64 + c];
          if (t < T) sv[TA_X1 + t * C + c] = xh;
          o[x][y][i] = y1;                       // keep Y1 (fp32) for the residual
          xa[t * TAM_LD + c] = (__bf16)y1;       // and as the FF's A operand
        }
        if (t < T && fr == 0) sv[TA_R1 + t] = r1[x][i];
      }
    tam_wsync();
    // ---- U = relu(Y1 W0^T + b0) ----
    f32x4 u[2][4];
    tam_zero(u);
    tam_gemm<4, 2>(u, xa, TAM_LD, Wf0, TAM_LD, fr, fg);
#pragma unroll
    for (int x = 0; x < 2; ++x)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int t = x * 16 + fg * 4 + i;
#pragma unroll
        for (int y = 0; y < 4; ++y) {
          const int c = y * 16 + fr;
          const float uv = fmaxf(u[x][y][i] + vec[3 * 64 + c], 0.f);
          if (t < T) sv[TA_U + t * C + c] = uv;
          Qs[t * TAM_LD + c] = (__bf16)uv;
        }
      }
    tam_wsync();
    // ---- F = U W2^T + b2 + Y1; out = LN(F) ----
    f32x4 f[2][4];
#pragma unroll
    for (int x = 0; x < 2; ++x)
#pragma unroll
      for (int y = 0; y < 4; ++y) f[x][y] = o[x][y];
    tam_gemm<4, 2>(f, Qs, TAM_LD, Wf2, TAM_LD, fr, fg);
#pragma unroll
    for (int x = 0; x < 2; ++x)
#pragma unroll
      for (int y = 0; y < 4; ++y) {
        const float bb = vec[4 * 64 + y * 16 + fr];
#pragma unroll
        for (int i = 0; i < 4; ++i) f[x][y][i] += bb;
      }
    float r2[2][4];
    tam_layernorm(f, r2);
#pragma unroll
    for (int x = 0; x < 2; ++x)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int t = x * 16 + fg * 4 + i;
        if (t >= T) continue;
        float* orow = a.out + ((size_t)(b * T + t) * V + n) * C;
#pragma unroll
        for (int y = 0; y < 4; ++y) {
          const int c = y * 16 + fr;
          const float xh = f[x][y][i];
          sv[TA_F2 + t * C + c] = xh;
          orow[c] = xh * vec[7 * 64 + c] + vec[8 * 64 + c];
        }
        if (fr == 0) sv[TA_R2 + t] = r2[x][i];
      }
    tam_wsync();
  }
}

// ---------------------------------------------------------------------------------------------
// Transform backward on bf16 MFMA (the bf16 mode). One wave per sequence again, two waves per
// workgroup. Every operand is kept ONCE, row-major, in LDS: a product that reduces over the rows of
// an operand (the weight gradients, P^T dO, dS^T Q, the conv weight gradient) reads that operand's
// fragments with gfx950's transposed LDS read (ds_read_b64_tr_b16: lane i of a 16-lane group gets
// column i of 8 consecutive rows) instead of keeping transposed copies. The weight gradients of the
// layer accumulate in each wave's registers across its sequences and are added once per wave at the
// end (fp32 atomics); the input gradient is written per sequence.
//   FF:   dF = LN2'(dY);  dU = (dF Wf2) . [U > 0];  dY1 = dU Wf0 + dF;  dO1 = LN1'(dY1)
//         dWf2 += dF^T U;  dWf0 += dU^T Y1
//   attn: dP = dO1 V^T;  dV = P^T dO1;  dS = P . (dP - rowsum(P . dP)) / sqrt(C)
//         dQ = dS K;  dK = dS^T Q;  dWv += dV^T x;  dx = dO1 + dV Wv
//   conv: dW1_j += dQ X_j^T (X_j[t'][c'] = x[t'][c'+j]);  dx[t'][c] += sum_j,t W1_j[t][t'] dQ[t][c-j]
//         (and K with W2)
// ---------------------------------------------------------------------------------------------
constexpr int TAB_WAVES = 4;           // both halves use 256 VGPRs + ~220-256 AGPRs: one wave per SIMD
constexpr int TAB_R72 = 32 * TAM_LD;   // a [32][72] row-major operand (bf16)
constexpr int TAB_R40 = 32 * TAM_LT;   // a [32][40] operand
constexpr int TAB_T66 = 66 * TAM_LT;   // a [66][40] operand (two zero rows of padding)
constexpr int TAB_VEC = 4 * 64;        // g1, be1, g2 (fp32)
// PART 1: Wf0, Wf2, vec shared; per wave two [32][72] slots (dF then Y1; U then dU)
// PART 2: W1, W2, Wv shared; per wave S1..S3 [32][72], S4 [32][40], Sxt / Sdqt / Sdkt [66][40]
//         (S1: dO1 then dV;  S2: V then K;  S3: x;  S4: P then dS;  Sdkt: Q then dK^T)
constexpr int TAB_SH1 = 2 * TAM_WL * 2 + TAB_VEC * 4;
constexpr int TAB_SEQ1 = 2 * TAB_R72;
constexpr int TAB_SH2 = (2 * TAM_W1 + TAM_WL) * 2;
constexpr int TAB_SEQ2 = 3 * TAB_R72 + TAB_R40 + 3 * TAB_T66;
constexpr int TAB_LDS1 = TAB_SH1 + TAB_WAVES * TAB_SEQ1 * 2;
constexpr int TAB_LDS2 = TAB_SH2 + TAB_WAVES * TAB_SEQ2 * 2;
constexpr int TAB_RED_LDS = (4 * 4096 + 4 * 64 + 2 * 4 * 32) * 4;  // the workgroup gradient reduction
static_assert(TAB_LDS1 <= 160 * 1024 && TAB_LDS2 <= 160 * 1024, "TA MFMA backward LDS");
static_assert(TAB_R72 <= TAB_T66, "Q is staged in the dK^T slot");

typedef short tab_s16x4 __attribute__((ext_vector_type(4)));

// the two transposed reads of a B-style fragment: rows k0 + 8 fg .. +7 of column c0 + fr of a
// row-major bf16 matrix with row stride ld (elements). The builtin (unlike inline asm) lets the
// compiler fold the constant part of the address into the instruction's offset field and place the
// lgkmcnt waits itself; with asm every fragment address became a live VGPR hoisted out of the
// sequence loop and the kernel spilled. No global loads are in flight around these reads, so the
// conservative vmcnt wait the builtin brings costs nothing here.
typedef __attribute__((address_space(3))) tab_s16x4 tab_lds_s16x4;
F3_DEV void tab_tr(const __bf16* base, int ld, int k0, int c0, int fr, int fg, tab_s16x4& lo, tab_s16x4& hi) {
  const int tq = fr >> 2, tp = fr & 3;
  const __bf16* p0 = base + (k0 + 8 * fg + tq) * ld + c0 + 4 * tp;
  lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((tab_lds_s16x4*)(p0));
  hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((tab_lds_s16x4*)(p0 + 4 * ld));
}
template <int N>
F3_DEV void tab_trwait(tab_s16x4 (&)[N], tab_s16x4 (&)[N]) {}
F3_DEV bf16x8_t tab_join(tab_s16x4 lo, tab_s16x4 hi) {
  return __builtin_bit_cast(bf16x8_t, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
}

// acc[x][y] (+)= A . B over K = 32*KSTEPS. Fragments: A either normal (A row-major [m][k], stride
// sa) or transposed (A^T stored row-major [k][m]); B either normal (Bt row-major [n][k]) or
// transposed (B stored row-major [k][n]). MT x NT tiles of 16.
template <int MT, int NT, int KSTEPS, bool AT, bool BT>
F3_DEV void tab_gemm(f32x4 (&acc)[MT][NT], const __bf16* A, int sa, const __bf16* B, int sb, int fr, int fg,
                     int a_k0 = 0, int b_k0 = 0) {
#pragma unroll
  for (int ks = 0; ks < KSTEPS; ++ks) {
    bf16x8_t fa[MT], fb[NT];
    tab_s16x4 lo[MT + NT], hi[MT + NT];
#pragma unroll
    for (int x = 0; x < MT; ++x) {
      if (AT) tab_tr(A, sa, a_k0 + ks * 32, x * 16, fr, fg, lo[x], hi[x]);
      else fa[x] = *reinterpret_cast<const bf16x8_t*>(A + (x * 16 + fr) * sa + a_k0 + ks * 32 + fg * 8);
    }
#pragma unroll
    for (int y = 0; y < NT; ++y) {
      if (BT) tab_tr(B, sb, b_k0 + ks * 32, y * 16, fr, fg, lo[MT + y], hi[MT + y]);
      else fb[y] = *reinterpret_cast<const bf16x8_t*>(B + (y * 16 + fr) * sb + b_k0 + ks * 32 + fg * 8);
    }
    if (AT || BT) tab_trwait(lo, hi);
#pragma unroll
    for (int x = 0; x < MT; ++x)
      if (AT) fa[x] = tab_join(lo[x], hi[x]);
#pragma unroll
    for (int y = 0; y < NT; ++y)
      if (BT) fb[y] = tab_join(lo[MT + y], hi[MT + y]);
#pragma unroll
    for (int x = 0; x < MT; ++x)
#pragma unroll
      for (int y = 0; y < NT; ++y) acc[x][y] = tam_mfma(fa[x], fb[y], acc[x][y]);
  }
}

template <int MT, int NT>
F3_DEV void tab_zero(f32x4 (&acc)[MT][NT]) {
#pragma unroll
  for (int x = 0; x < MT; ++x)
#pragma unroll
    for (int y = 0; y < NT; ++y) acc[x][y] = f32x4{0.f, 0.f, 0.f, 0.f};
}

// store a [32 rows][16*NT cols] accumulator (rows x*16+4fg+i, cols y*16+fr) row-major as bf16
template <int NT>
F3_DEV void tab_store(__bf16* dst, int ld, const f32x4 (&acc)[2][NT], int fr, int fg) {
#pragma unroll
  for (int x = 0; x < 2; ++x)
#pragma unroll
    for (int y = 0; y < NT; ++y)
#pragma unroll
      for (int i = 0; i < 4; ++i) dst[(x * 16 + fg * 4 + i) * ld + y * 16 + fr] = (__bf16)acc[x][y][i];
}
// the same accumulator transposed ([col + roff][row], 4 consecutive rows of a lane = one 8-B store)
template <int NT>
F3_DEV void tab_store_t(__bf16* dst, int ld, int roff, const f32x4 (&acc)[2][NT], int fr, int fg) {
  typedef __bf16 bf16x4_t __attribute__((ext_vector_type(4)));
#pragma unroll
  for (int x = 0; x < 2; ++x)
#pragma unroll
    for (int y = 0; y < NT; ++y) {
      bf16x4_t v;
#pragma unroll
      for (int i = 0; i < 4; ++i) v[i] = (__bf16)acc[x][y][i];
      *reinterpret_cast<bf16x4_t*>(dst + (y * 16 + fr + roff) * ld + x * 16 + fg * 4) = v;
    }
}
// load an fp32 [rows < nrow][ncol] matrix (row stride lds) into the accumulator layout, 0 outside
template <int NT>
F3_DEV void tab_load(f32x4 (&acc)[2][NT], const float* src, int lds, int nrow, int ncol, int fr, int fg) {
#pragma unroll
  for (int x = 0; x < 2; ++x)
#pragma unroll
    for (int y = 0; y < NT; ++y)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int r = x * 16 + fg * 4 + i, c = y * 16 + fr;
        acc[x][y][i] = (r < nrow && c < ncol) ? src[r * lds + c] : 0.f;
      }
}

// add a per-lane column accumulator (summed over the lane's rows) across the 4 row groups, then
// one atomic per column
F3_DEV void tab_flush_cols(float v, float* dst, int fg) {
  v += __shfl_xor(v, 16, 64);
  v += __shfl_xor(v, 32, 64);
  if (fg == 0) atomic_add_f(dst, v);
}

// PART 1: the FF half (LN2', FF weight gradients, LN1') -> dO1 written into din (scratch);
// PART 2: the attention and conv half, reading dO1 from din and overwriting it with dx. Two launches
// keep each half's weight-gradient accumulators in registers without spilling.
template <int PART>
__global__ __launch_bounds__(64 * TAB_WAVES) void ta_bwd_mfma_kernel(TaArgs a) {
  extern __shared__ __attribute__((aligned(16))) char tab_smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const float* P_ = a.p;
  constexpr int NTH = 64 * TAB_WAVES;
  __bf16 *W1 = nullptr, *W2 = nullptr, *Wv = nullptr, *Wf0 = nullptr, *Wf2 = nullptr, *sq0;
  float* vec = nullptr;
  if constexpr (PART == 1) {
    Wf0 = reinterpret_cast<__bf16*>(tab_smem);  // [64 out][LD in]
    Wf2 = Wf0 + TAM_WL;
    vec = reinterpret_cast<float*>(Wf2 + TAM_WL);  // g1, be1, g2
    sq0 = reinterpret_cast<__bf16*>(tab_smem + TAB_SH1) + wave * TAB_SEQ1;
    for (int i = tid; i < C * C; i += NTH) {
      const int o = i / C, k = i - o * C;
      Wf0[o * TAM_LD + k] = (__bf16)P_[a.off_f0w + i];
      Wf2[o * TAM_LD + k] = (__bf16)P_[a.off_f2w + i];
    }
    for (int i = tid; i < 64; i += NTH) {
      vec[i] = P_[a.off_lnw + i];
      vec[64 + i] = P_[a.off_lnb + i];
      vec[128 + i] = P_[a.off_lnffw + i];
    }
  } else {
    W1 = reinterpret_cast<__bf16*>(tab_smem);  // [3][32 t][LT t'] (row-major W_j[t][t'])
    W2 = W1 + TAM_W1;
    Wv = W2 + TAM_W1;                         // [64 out][LD in]
    sq0 = reinterpret_cast<__bf16*>(tab_smem + TAB_SH2) + wave * TAB_SEQ2;
    for (int i = tid; i < 3 * 32 * 32; i += NTH) {
      const int j = i / 1024, t = (i >> 5) & 31, u = i & 31;
      const bool ok = t < T && u < T;
      W1[j * 32 * TAM_LT + t * TAM_LT + u] = (__bf16)(ok ? P_[a.off_c1w + (t * T + u) * 3 + j] : 0.f);
      W2[j * 32 * TAM_LT + t * TAM_LT + u] = (__bf16)(ok ? P_[a.off_c2w + (t * T + u) * 3 + j] : 0.f);
    }
    for (int i = tid; i < C * C; i += NTH) Wv[(i / C) * TAM_LD + i % C] = (__bf16)P_[a.off_vw + i];
  }
  // PART 1 slots
  __bf16* BdF = sq0;               // dF, then Y1
  __bf16* BU = sq0 + TAB_R72;      // U, then dU
  __bf16* BY1 = BdF;
  __bf16* BdU = BU;
  // PART 2 slots
  __bf16* Bdo = sq0;                       // S1: dO1, then dV
  __bf16* Bdv = Bdo;
  __bf16* Bv = sq0 + TAB_R72;              // S2: V, then K
  __bf16* Bk = Bv;
  __bf16* Bx = sq0 + 2 * TAB_R72;          // S3: x
  __bf16* Bp = sq0 + 3 * TAB_R72;          // S4: P [32][40], then dS
  __bf16* Bds = Bp;
  __bf16* Bxt = Bp + TAB_R40;              // x^T [66][40] (rows 64, 65 zero)
  __bf16* Bdqt = Bxt + TAB_T66;            // dQ^T at rows 2.. (rows 0, 1 zero)
  __bf16* Bdkt = Bdqt + TAB_T66;           // Q [32][72] first, then dK^T like dQ^T
  __bf16* Bq = Bdkt;
  const int fr = lane & 15, fg = lane >> 4;
  for (int i = lane; i < (PART == 1 ? TAB_SEQ1 : TAB_SEQ2); i += 64) sq0[i] = (__bf16)0.f;
  __syncthreads();
  // weight-gradient accumulators (this wave's sequences)
  f32x4 gA[4][4], gB[4][4];                 // PART 1: dWf2, dWf0;  PART 2: dWv (gA)
  f32x4 gC1[PART == 2 ? 3 : 1][2][2], gC2[PART == 2 ? 3 : 1][2][2];
  tab_zero(gA);
  tab_zero(gB);
#pragma unroll
  for (int j = 0; j < (PART == 2 ? 3 : 1); ++j) {
    tab_zero(gC1[j]);
    tab_zero(gC2[j]);
  }
  float cg2[4] = {}, cbe2[4] = {}, cbf2[4] = {}, cbf0[4] = {}, cg1[4] = {}, cbe1[4] = {}, cbv[4] = {};
  float rb1[2][4] = {}, rb2[2][4] = {};  // conv bias gradients per row t (summed over c')
  const int V = a.V, nseq = a.B * V;
  const size_t rstride = (size_t)V * C;
#pragma unroll 1
  for (int sq = blockIdx.x * TAB_WAVES + wave; sq < nseq; sq += gridDim.x * TAB_WAVES) {
    // opaque copies of the lane coordinates: every lane-derived address is then recomputed per
    // sequence instead of being hoisted out of the loop (dozens of live 64-bit offsets -> spills)
    int fr = lane & 15, fg = lane >> 4;
    asm volatile("" : "+v"(fr), "+v"(fg));
    const int b = sq / V, n = sq - b * V;
    const float* sv = a.save + (size_t)sq * TA_SAVE;
    const float* xin = a.in + ((size_t)b * T * V + n) * C;
    const float* dout = a.dout + ((size_t)b * T * V + n) * C;
    f32x4 dF[2][4];
    if constexpr (PART == 1) {
    // ---------------- FF ----------------
    f32x4 fh[2][4];
    tab_load(fh, sv + TA_F2, C, T, C, fr, fg);
#pragma unroll
    for (int x = 0; x < 2; ++x)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int t = x * 16 + fg * 4 + i;
        const float r2 = t < T ? sv[TA_R2 + t] : 0.f;
        float g[4], s1 = 0.f, s2 = 0.f;
#pragma unroll
        for (int y = 0; y < 4; ++y) {
          const int c = y * 16 + fr;
          const float dy = t < T ? dout[t * rstride + c] : 0.f;
          cg2[y] += dy * fh[x][y][i];
          cbe2[y] += dy;
          g[y] = dy * vec[128 + c];
          s1 += g[y];
          s2 += g[y] * fh[x][y][i];
        }
        const float m1 = tam_rowsum(s1) * (1.f / C), m2 = tam_rowsum(s2) * (1.f / C);
#pragma unroll
        for (int y = 0; y < 4; ++y) {
          dF[x][y][i] = r2 * (g[y] - m1 - fh[x][y][i] * m2);
          cbf2[y] += dF[x][y][i];
        }
      }
    {
      f32x4 u[2][4];
      tab_load(u, sv + TA_U, C, T, C, fr, fg);
      tab_store(BU, TAM_LD, u, fr, fg);  // the ReLU mask below reads U back (bf16 keeps the sign)
    }
    tab_store(BdF, TAM_LD, dF, fr, fg);
    tam_wsync();
    tab_gemm<4, 4, 1, true, true>(gA, BdF, TAM_LD, BU, TAM_LD, fr, fg);  // dWf2[c][k'] += sum_t dF[t][c] U[t][k']
    f32x4 du[2][4];
    tab_zero(du);
    tab_gemm<2, 4, 2, false, true>(du, BdF, TAM_LD, Wf2, TAM_LD, fr, fg);  // dF Wf2
#pragma unroll
    for (int x = 0; x < 2; ++x)
#pragma unroll
      for (int y = 0; y < 4; ++y)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const bool on = (float)BU[(x * 16 + fg * 4 + i) * TAM_LD + y * 16 + fr] > 0.f;
          du[x][y][i] = on ? du[x][y][i] : 0.f;
          cbf0[y] += du[x][y][i];
        }
    f32x4 y1[2][4];
    tab_load(y1, sv + TA_X1, C, T, C, fr, fg);  // xhat1 -> Y1 = g1 xhat1 + be1
#pragma unroll
    for (int x = 0; x < 2; ++x)
#pragma unroll
      for (int y = 0; y < 4; ++y)
#pragma unroll
        for (int i = 0; i < 4; ++i) y1[x][y][i] = y1[x][y][i] * vec[y * 16 + fr] + vec[64 + y * 16 + fr];
    tam_wsync();  // all lanes read their U (and the dF fragments) before dU / Y1 overwrite them
    tab_store(BdU, TAM_LD, du, fr, fg);
    tab_store(BY1, TAM_LD, y1, fr, fg);
    tam_wsync();
    tab_gemm<4, 4, 1, true, true>(gB, BdU, TAM_LD, BY1, TAM_LD, fr, fg);  // dWf0[k'][c] += sum_t dU[t][k'] Y1[t][c]
    tab_gemm<2, 4, 2, false, true>(dF, BdU, TAM_LD, Wf0, TAM_LD, fr, fg);  // dY1 = dF + dU Wf0
    // LN1 backward -> dO1 (into dF); y1 <- xhat1 again
    tab_load(y1, sv + TA_X1, C, T, C, fr, fg);
#pragma unroll
    for (int x = 0; x < 2; ++x)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int t = x * 16 + fg * 4 + i;
        const float r1 = t < T ? sv[TA_R1 + t] : 0.f;
        float g[4], s1 = 0.f, s2 = 0.f;
#pragma unroll
        for (int y = 0; y < 4; ++y) {
          const int c = y * 16 + fr;
          cg1[y] += dF[x][y][i] * y1[x][y][i];
          cbe1[y] += dF[x][y][i];
          g[y] = dF[x][y][i] * vec[c];
          s1 += g[y];
          s2 += g[y] * y1[x][y][i];
        }
        const float m1 = tam_rowsum(s1) * (1.f / C), m2 = tam_rowsum(s2) * (1.f / C);
#pragma unroll
        for (int y = 0; y < 4; ++y) dF[x][y][i] = r1 * (g[y] - m1 - y1[x][y][i] * m2);
      }
#pragma unroll
    for (int x = 0; x < 2; ++x)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int t = x * 16 + fg * 4 + i;
        if (t >= T) continue;
        float* drow = a.din + ((size_t)(b * T + t) * V + n) * C;
#pragma unroll
        for (int y = 0; y < 4; ++y) drow[y * 16 + fr] = dF[x][y][i];  // dO1 (scratch for PART 2)
      }
    tam_wsync();
    continue;
    } else {
    // dO1 from PART 1 (din is overwritten with dx below, by this same wave)
    tab_load(dF, a.din + ((size_t)b * T * V + n) * C, V * C, T, C, fr, fg);
    }
    // ---------------- attention ----------------
    tab_store(Bdo, TAM_LD, dF, fr, fg);
    f32x4 t4[2][4];
    tab_load(t4, sv + TA_V, C, T, C, fr, fg);
    tab_store(Bv, TAM_LD, t4, fr, fg);
#pragma unroll
    for (int x = 0; x < 2; ++x)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int t = min(x * 16 + fg * 4 + i, T - 1);
#pragma unroll
        for (int y = 0; y < 4; ++y) {
          float xv = xin[t * rstride + y * 16 + fr];
          if (a.pe) xv += a.pe[t * C + y * 16 + fr];
          t4[x][y][i] = x * 16 + fg * 4 + i < T ? xv : 0.f;
        }
      }
    tab_store(Bx, TAM_LD, t4, fr, fg);
    tab_store_t(Bxt, TAM_LT, 0, t4, fr, fg);
    f32x4 p[2][2];
    tab_load(p, sv + TA_P, T, T, T, fr, fg);
    tab_store(Bp, TAM_LT, p, fr, fg);
    tam_wsync();
    f32x4 dp[2][2];
    tab_zero(dp);
    tab_gemm<2, 2, 2, false, false>(dp, Bdo, TAM_LD, Bv, TAM_LD, fr, fg);  // dP = dO1 V^T
    f32x4 dv[2][4];
    tab_zero(dv);
    tab_gemm<2, 4, 1, true, true>(dv, Bp, TAM_LT, Bdo, TAM_LD, fr, fg);   // dV = P^T dO1
    // softmax backward (rows t, columns u; P is 0 outside the 30 x 30 block)
#pragma unroll
    for (int x = 0; x < 2; ++x)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float dot = tam_rowsum(p[x][0][i] * dp[x][0][i] + p[x][1][i] * dp[x][1][i]);
#pragma unroll
        for (int y = 0; y < 2; ++y) dp[x][y][i] = p[x][y][i] * (dp[x][y][i] - dot) * 0.125f;
      }
#pragma unroll
    for (int x = 0; x < 2; ++x)
#pragma unroll
      for (int y = 0; y < 4; ++y)
#pragma unroll
        for (int i = 0; i < 4; ++i) cbv[y] += dv[x][y][i];
    tam_wsync();  // dO1 / V / P fragments read by every lane: S1, S2, S4 are reused below
    tab_store(Bds, TAM_LT, dp, fr, fg);
    tab_store(Bdv, TAM_LD, dv, fr, fg);
    tab_load(t4, sv + TA_K, CQ, T, CQ, fr, fg);
    tab_store(Bk, TAM_LD, t4, fr, fg);
    tab_load(t4, sv + TA_Q, CQ, T, CQ, fr, fg);
    tab_store(Bq, TAM_LD, t4, fr, fg);
    tam_wsync();
    tab_gemm<4, 4, 1, true, true>(gA, Bdv, TAM_LD, Bx, TAM_LD, fr, fg);  // dWv[c][c2] += sum_u dV[u][c] x[u][c2]
    {
      f32x4 dq[2][4];  // dQ = dS K, then dK = dS^T Q in the same registers
      tab_zero(dq);
      tab_gemm<2, 4, 1, false, true>(dq, Bds, TAM_LT, Bk, TAM_LD, fr, fg);
#pragma unroll
      for (int x = 0; x < 2; ++x)
#pragma unroll
        for (int i = 0; i < 4; ++i)  // summed over this lane's columns; the 16 lanes of a row add up at the end
          rb1[x][i] += dq[x][0][i] + dq[x][1][i] + dq[x][2][i] + dq[x][3][i];
      tab_store_t(Bdqt, TAM_LT, 2, dq, fr, fg);
      tab_zero(dq);
      tab_gemm<2, 4, 1, true, true>(dq, Bds, TAM_LT, Bq, TAM_LD, fr, fg);
#pragma unroll
      for (int x = 0; x < 2; ++x)
#pragma unroll
        for (int i = 0; i < 4; ++i) rb2[x][i] += dq[x][0][i] + dq[x][1][i] + dq[x][2][i] + dq[x][3][i];
      tam_wsync();  // Q read by every lane before dK^T replaces it
      tab_store_t(Bdkt, TAM_LT, 2, dq, fr, fg);
      for (int i = lane; i < 2 * TAM_LT; i += 64) Bdkt[i] = (__bf16)0.f;  // the zero rows Q covered
    }
    tam_wsync();
    // conv weight gradients: dW_j[t][t'] += sum_c' dQ[t][c'] x[t'][c'+j] (A = dQ^T rows c'+2, B = x^T rows c'+j)
#pragma unroll
    for (int j = 0; j < (PART == 2 ? 3 : 0); ++j) {
      tab_gemm<2, 2, 2, true, true>(gC1[j], Bdqt, TAM_LT, Bxt, TAM_LT, fr, fg, 2, j);
      tab_gemm<2, 2, 2, true, true>(gC2[j], Bdkt, TAM_LT, Bxt, TAM_LT, fr, fg, 2, j);
    }
    // dx = dO1 (O1 = A V + x) + dV Wv + conv input gradients; dO1 in fp32 from din
    f32x4 dx[2][4];
    tab_load(dx, a.din + ((size_t)b * T * V + n) * C, V * C, T, C, fr, fg);
    tab_gemm<2, 4, 2, false, true>(dx, Bdv, TAM_LD, Wv, TAM_LD, fr, fg);
    // conv input gradients: dx[t'][c] += sum_j sum_t W_j[t][t'] dQ[t][c-j]  (B^T rows c-j+2 of dQ^T)
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      tab_gemm<2, 4, 1, true, false>(dx, W1 + j * 32 * TAM_LT, TAM_LT, Bdqt + (2 - j) * TAM_LT, TAM_LT, fr, fg);
      tab_gemm<2, 4, 1, true, false>(dx, W2 + j * 32 * TAM_LT, TAM_LT, Bdkt + (2 - j) * TAM_LT, TAM_LT, fr, fg);
    }
#pragma unroll
    for (int x = 0; x < 2; ++x)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int t = x * 16 + fg * 4 + i;
        if (t >= T) continue;
        float* drow = a.din + ((size_t)(b * T + t) * V + n) * C;
#pragma unroll
        for (int y = 0; y < 4; ++y) drow[y * 16 + fr] = dx[x][y][i];
      }
    tam_wsync();
  }
  // ---------------- flush this wave's weight gradients ----------------
  if (a.part) {  // workgroup sums through LDS -> this workgroup's row of the partial slab
    float* red = reinterpret_cast<float*>(tab_smem);  // [4 waves][4096] (the sequence slots are done)
    float* row = a.part + (size_t)blockIdx.x * TA_PART;
    auto wg_matrix = [&](const f32x4 (&g)[4][4], int field) {
      __syncthreads();
#pragma unroll
      for (int x = 0; x < 4; ++x)
#pragma unroll
        for (int y = 0; y < 4; ++y)
#pragma unroll
          for (int i = 0; i < 4; ++i) red[wave * 4096 + (x * 16 + fg * 4 + i) * C + y * 16 + fr] = g[x][y][i];
      __syncthreads();
      for (int e = tid; e < 4096; e += NTH) row[field + e] = (red[e] + red[4096 + e]) + (red[8192 + e] + red[12288 + e]);
    };
    auto wg_cols = [&](float v, int field, int c) {  // column sums over the lane's rows -> [64]
      v += __shfl_xor(v, 16, 64);
      v += __shfl_xor(v, 32, 64);
      if (fg == 0) red[16384 + wave * 64 + c] = v;
      return field;
    };
    auto wg_cols_out = [&](int field) {  // after a barrier: the 4 waves' column sums
      for (int e = tid; e < 64; e += NTH)
        row[field + e] = (red[16384 + e] + red[16384 + 64 + e]) + (red[16384 + 128 + e] + red[16384 + 192 + e]);
    };
    if constexpr (PART == 1) {
      wg_matrix(gA, 0);
      wg_matrix(gB, 4096);
      auto cols = [&](const float (&v)[4], int q) {  // (by reference: a pointer table forced scratch)
        __syncthreads();
#pragma unroll
        for (int y = 0; y < 4; ++y) wg_cols(v[y], 0, y * 16 + fr);
        __syncthreads();
        wg_cols_out(8192 + q * 64);
      };
      cols(cg2, 0);
      cols(cbe2, 1);
      cols(cbf2, 2);
      cols(cbf0, 3);
      cols(cg1, 4);
      cols(cbe1, 5);
    } else {
      wg_matrix(gA, 0);
#pragma unroll
      for (int cv = 0; cv < 2; ++cv) {
#pragma unroll
        for (int j = 0; j < 3; ++j) {
          __syncthreads();
#pragma unroll
          for (int x = 0; x < 2; ++x)
#pragma unroll
            for (int y = 0; y < 2; ++y)
#pragma unroll
              for (int i = 0; i < 4; ++i)
                red[wave * 1024 + (x * 16 + fg * 4 + i) * 32 + y * 16 + fr] = cv ? gC2[j][x][y][i] : gC1[j][x][y][i];
          __syncthreads();
          for (int e = tid; e < T * T; e += NTH) {
            const int t = e / T, u = e - t * T, k = t * 32 + u;
            row[4096 + cv * T * T * 3 + e * 3 + j] = (red[k] + red[1024 + k]) + (red[2048 + k] + red[3072 + k]);
          }
        }
      }
      __syncthreads();
#pragma unroll
      for (int y = 0; y < 4; ++y) wg_cols(cbv[y], 0, y * 16 + fr);
      // conv bias gradients: per-row sums of the 16 lanes of each row group
#pragma unroll
      for (int x = 0; x < 2; ++x)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int t = x * 16 + fg * 4 + i;
          const float s1 = tam_rowsum(rb1[x][i]), s2 = tam_rowsum(rb2[x][i]);
          if (fr == 0) {
            red[16384 + 256 + wave * 32 + t] = s1;
            red[16384 + 384 + wave * 32 + t] = s2;
          }
        }
      __syncthreads();
      const int fb = 4096 + 2 * T * T * 3;
      wg_cols_out(fb);
      for (int e = tid; e < 64; e += NTH) {
        const int which = e >> 5, t = e & 31;
        const float* r = red + 16384 + 256 + which * 128;
        row[fb + 64 + e] = t < T ? (r[t] + r[32 + t]) + (r[64 + t] + r[96 + t]) : 0.f;
      }
    }
    return;
  }
  float* G = a.grads;
  auto flush64 = [&](const f32x4 (&g)[4][4], long long off) {  // g rows = out (m), cols = in (n)
#pragma unroll
    for (int x = 0; x < 4; ++x)
#pragma unroll
      for (int y = 0; y < 4; ++y)
#pragma unroll
        for (int i = 0; i < 4; ++i) atomic_add_f(G + off + (x * 16 + fg * 4 + i) * C + y * 16 + fr, g[x][y][i]);
  };
  if constexpr (PART == 1) {
    flush64(gA, a.off_f2w);
    flush64(gB, a.off_f0w);
#pragma unroll
    for (int y = 0; y < 4; ++y) {
      const int c = y * 16 + fr;
      tab_flush_cols(cg2[y], G + a.off_lnffw + c, fg);
      tab_flush_cols(cbe2[y], G + a.off_lnffb + c, fg);
      tab_flush_cols(cbf2[y], G + a.off_f2b + c, fg);
      tab_flush_cols(cbf0[y], G + a.off_f0b + c, fg);
      tab_flush_cols(cg1[y], G + a.off_lnw + c, fg);
      tab_flush_cols(cbe1[y], G + a.off_lnb + c, fg);
    }
    return;
  }
  flush64(gA, a.off_vw);
#pragma unroll
  for (int j = 0; j < (PART == 2 ? 3 : 0); ++j)
#pragma unroll
    for (int x = 0; x < 2; ++x)
#pragma unroll
      for (int y = 0; y < 2; ++y)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int t = x * 16 + fg * 4 + i, u = y * 16 + fr;
          if (t < T && u < T) {
            atomic_add_f(G + a.off_c1w + (t * T + u) * 3 + j, gC1[j][x][y][i]);
            atomic_add_f(G + a.off_c2w + (t * T + u) * 3 + j, gC2[j][x][y][i]);
          }
        }
#pragma unroll
  for (int y = 0; y < 4; ++y) tab_flush_cols(cbv[y], G + a.off_vb + y * 16 + fr, fg);
#pragma unroll
  for (int x = 0; x < 2; ++x)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int t = x * 16 + fg * 4 + i;
      const float s1 = tam_rowsum(rb1[x][i]), s2 = tam_rowsum(rb2[x][i]);
      if (fr == 0 && t < T) {
        atomic_add_f(G + a.off_c1b + t, s1);
        atomic_add_f(G + a.off_c2b + t, s2);
      }
    }
}

}  // namespace tg
}  // namespace f3

using namespace f3;
using namespace f3::tg;

namespace {
template <bool B16>
int gru_lds(int V, bool bwd) {
  using TT = typename Op<B16>::T;
  const int bt = bwd ? Op<B16>::BTB : Op<B16>::BTF;
  return (bwd ? 4 : 2) * V * bt * Op<B16>::XS * (int)sizeof(TT) + (bwd ? 7 : 3) * V * bt * H * 4 + (V * V + V) * 4;
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
  F3_LDS_LIMIT(gru_fwd_kernel<B16>, 160 * 1024);
  const int grid = (a.B + Op<B16>::BTF - 1) / Op<B16>::BTF;
  hipLaunchKernelGGL(gru_fwd_kernel<B16>, dim3(grid), dim3(GRU_THREADS), lds, s, a);
  F3_LAUNCH_CHECK();
  return F3_OK;
}

template <bool B16>
static int gru_bwd_launch(const GruBwdArgs& a, hipStream_t s) {
  const int lds = gru_lds<B16>(a.V, true);
  F3_LDS_LIMIT(gru_bwd_kernel<B16>, 160 * 1024);
  const int grid = (a.B + Op<B16>::BTB - 1) / Op<B16>::BTB;
  hipLaunchKernelGGL(gru_bwd_kernel<B16>, dim3(grid), dim3(GRU_THREADS), lds, s, a);
  F3_LAUNCH_CHECK();
  return F3_OK;
}

// Workgroups of a node-partitioned kernel that are resident together: the occupancy query's answer
// per CU, capped at 6 (MI355X_MICROARCH.md "Residency and cooperative launch": the hardware admits
// floor(800 / (ceil(sgpr / 16) * 16 + 16)) 256-thread blocks per CU, 6 at these kernels' 94-106 SGPRs),
// times the CUs.
static int gn_resident(const void* kernel) {
  int per_cu = 0, dev = 0, cus = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kernel, GN_THREADS, 0) != hipSuccess || per_cu < 1 ||
      hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) !=
                                              hipSuccess) {
    (void)hipGetLastError();
    return 0;
  }
  return std::min(per_cu, 6) * cus;
}

// node-partitioned forward (see gru_fwd_node_kernel): bf16 mode, exchange buffers present, a launch
// of V x ceil(B / GN_BT) workgroups when they are all resident together (the group barriers need it);
// else false and the caller runs the clip-tile kernel. A plain launch, not hipLaunchCooperativeKernel:
// residency is the same (the occupancy check above is what the cooperative launch adds), the
// cooperative launch costs 15-20 us of queue latency per call, and a process that used it died with
// SIGSEGV in rocprofiler-sdk's exit handlers under rocprofv3.
static bool gru_fwd_node(const GruFwdArgs& a, hipStream_t s) {
  const int NG = (a.B + GN_BT - 1) / GN_BT;
  if (!a.hx || !a.rhx || !a.gsync || NG > GN_MAXG || a.V > VMAX || a.prof) return false;
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  if (hipStreamIsCapturing(s, &cs) != hipSuccess || cs != hipStreamCaptureStatusNone) {
    (void)hipGetLastError();
    return false;
  }
  if (hipMemsetAsync(a.gsync, 0, sizeof(int) * NG, s) != hipSuccess) return false;
  static const int resident = gn_resident((const void*)gru_fwd_node_kernel);
  if (NG * a.V > resident) return false;
  hipLaunchKernelGGL(gru_fwd_node_kernel, dim3(NG * a.V), dim3(GN_THREADS), 0, s, a);
  if (hipGetLastError() != hipSuccess) return false;
  return true;
}

int f3_tg_gru_fwd(const GruFwdArgs* a, int b16, hipStream_t s) {
  if (!f3_tg_gru_lds_ok(a->V) || a->I > IP || a->B < 1) return F3_EINVAL;
  if (b16 && gru_fwd_node(*a, s)) return F3_OK;
  return b16 ? gru_fwd_launch<true>(*a, s) : gru_fwd_launch<false>(*a, s);
}

static bool gru_bwd_node(const GruBwdArgs& a, hipStream_t s) {
  const int NG = (a.B + GN_BT - 1) / GN_BT;
  if (!a.gx1 || !a.gx2 || !a.gsync || NG > GN_MAXG || a.V > VMAX || a.prof) return false;
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  if (hipStreamIsCapturing(s, &cs) != hipSuccess || cs != hipStreamCaptureStatusNone) {
    (void)hipGetLastError();
    return false;
  }
  if (hipMemsetAsync(a.gsync, 0, sizeof(int) * NG, s) != hipSuccess) return false;
  static const int resident = gn_resident((const void*)gru_bwd_node_kernel);
  if (NG * a.V > resident) return false;
  hipLaunchKernelGGL(gru_bwd_node_kernel, dim3(NG * a.V), dim3(GN_THREADS), 0, s, a);
  if (hipGetLastError() != hipSuccess) return false;
  return true;
}

int f3_tg_gru_bwd(const GruBwdArgs* a, int b16, hipStream_t s) {
  if (!f3_tg_gru_lds_ok(a->V) || a->I > IP || a->B < 1) return F3_EINVAL;
  if (b16 && gru_bwd_node(*a, s)) return F3_OK;
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

// grads[seg.goff + e - seg.start] += sum over the workgroups' rows of part[.][e], for the fields of one
// backward half. Block = 64 fields x 4 row groups (each sums every 4th workgroup), LDS combine.
struct TaSeg {
  int start, len;
  long long goff;
};
struct TaSegs {
  TaSeg s[8];
  int n, total;
};
__global__ __launch_bounds__(256) void ta_part_reduce_kernel(const float* __restrict__ part, int nblk, TaSegs sg,
                                                             float* __restrict__ grads) {
  __shared__ float red[4][64];
  const int lane = threadIdx.x & 63, rg = threadIdx.x >> 6;
  const int e = blockIdx.x * 64 + lane;
  float acc0 = 0.f, acc1 = 0.f;
  if (e < sg.total) {
    int b = rg;
    for (; b + 4 < nblk; b += 8) {
      acc0 += part[(size_t)b * TA_PART + e];
      acc1 += part[(size_t)(b + 4) * TA_PART + e];
    }
    if (b < nblk) acc0 += part[(size_t)b * TA_PART + e];
  }
  red[rg][lane] = acc0 + acc1;
  __syncthreads();
  if (rg == 0 && e < sg.total) {
    const float v = (red[0][lane] + red[1][lane]) + (red[2][lane] + red[3][lane]);
    for (int k = 0; k < sg.n; ++k)
      if (e >= sg.s[k].start && e < sg.s[k].start + sg.s[k].len) grads[sg.s[k].goff + (e - sg.s[k].start)] += v;
  }
}

static int ta_grid(const TaArgs& a) {
  int dev = 0, cus = 256;
  if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  (void)hipGetLastError();
  return std::max(1, std::min(cus, a.B * a.V));
}

int f3_tg_ta_fwd(const TaArgs* a, hipStream_t s) {
  if (a->b16) {  // bf16 mode: one wave per sequence on bf16 MFMA
    F3_LDS_LIMIT(ta_fwd_mfma_kernel, TAM_LDS);
    const int grid = std::max(1, std::min(ta_grid(*a), (a->B * a->V + TAM_WAVES - 1) / TAM_WAVES));
    hipLaunchKernelGGL(ta_fwd_mfma_kernel, dim3(grid), dim3(64 * TAM_WAVES), TAM_LDS, s, *a);
    F3_LAUNCH_CHECK();
    return F3_OK;
  }
  F3_LDS_LIMIT(ta_fwd_kernel, TA_FWD_LDS);
  hipLaunchKernelGGL(ta_fwd_kernel, dim3(ta_grid(*a)), dim3(TA_THREADS), TA_FWD_LDS, s, *a);
  F3_LAUNCH_CHECK();
  return F3_OK;
}

int f3_tg_ta_bwd(const TaArgs* a_, hipStream_t s) {
  const TaArgs* a = a_;
  if (a->b16) {  // bf16 mode: one wave per sequence on bf16 MFMA
    F3_LDS_LIMIT(ta_bwd_mfma_kernel<1>, std::max(TAB_LDS1, TAB_RED_LDS));
    F3_LDS_LIMIT(ta_bwd_mfma_kernel<2>, std::max(TAB_LDS2, TAB_RED_LDS));
    const int grid = std::max(1, std::min({ta_grid(*a), (a->B * a->V + TAB_WAVES - 1) / TAB_WAVES, TA_MAX_WG}));
    // the workgroup reduction reuses the LDS as [4 waves][4096] + column sums
    const int lds1 = a->part ? std::max(TAB_LDS1, TAB_RED_LDS) : TAB_LDS1;
    const int lds2 = a->part ? std::max(TAB_LDS2, TAB_RED_LDS) : TAB_LDS2;
    hipLaunchKernelGGL(ta_bwd_mfma_kernel<1>, dim3(grid), dim3(64 * TAB_WAVES), lds1, s, *a);
    F3_LAUNCH_CHECK();
    if (a->part) {
      TaSegs sg;
      std::memset(&sg, 0, sizeof(sg));
      const long long g1[8] = {a->off_f2w, a->off_f0w, a->off_lnffw, a->off_lnffb, a->off_f2b, a->off_f0b, a->off_lnw,
                               a->off_lnb};
      const int l1[8] = {4096, 4096, 64, 64, 64, 64, 64, 64};
      int st = 0;
      for (int k = 0; k < 8; ++k) { sg.s[k] = TaSeg{st, l1[k], g1[k]}; st += l1[k]; }
      sg.n = 8; sg.total = st;
      hipLaunchKernelGGL(ta_part_reduce_kernel, dim3((sg.total + 63) / 64), dim3(256), 0, s, a->part, grid, sg, a->grads);
      F3_LAUNCH_CHECK();
    }
    hipLaunchKernelGGL(ta_bwd_mfma_kernel<2>, dim3(grid), dim3(64 * TAB_WAVES), lds2, s, *a);
    F3_LAUNCH_CHECK();
    if (a->part) {
      TaSegs sg;
      std::memset(&sg, 0, sizeof(sg));
      const long long g2[6] = {a->off_vw, a->off_c1w, a->off_c2w, a->off_vb, a->off_c1b, a->off_c2b};
      const int l2[6] = {4096, T * T * 3, T * T * 3, 64, T, T};
      const int s2[6] = {0, 4096, 4096 + T * T * 3, 4096 + 2 * T * T * 3, 4096 + 2 * T * T * 3 + 64,
                         4096 + 2 * T * T * 3 + 96};
      for (int k = 0; k < 6; ++k) sg.s[k] = TaSeg{s2[k], l2[k], g2[k]};
      sg.n = 6; sg.total = s2[5] + T;
      hipLaunchKernelGGL(ta_part_reduce_kernel, dim3((sg.total + 63) / 64), dim3(256), 0, s, a->part, grid, sg, a->grads);
      F3_LAUNCH_CHECK();
    }
    return F3_OK;
  }
  F3_LDS_LIMIT(ta_bwd_kernel, TA_BWD_LDS);
  hipLaunchKernelGGL(ta_bwd_kernel, dim3(ta_grid(*a)), dim3(TA_THREADS), TA_BWD_LDS, s, *a);
  F3_LAUNCH_CHECK();
  return F3_OK;
}
