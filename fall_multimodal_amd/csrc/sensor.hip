// IMU branch: (optional CNN1D front end) -> bidirectional LSTM -> mean over time ->
// BatchNorm1d -> channel attention MLP -> Linear.
//   BiLSTM            Multimodal_Fall3/model/bilstm.py:21-59 (nn.LSTM gate order i,f,g,o)
//   ChannelAttention  Multimodal_Fall3/model/bilstm.py:5-19
//   CNN1D             GSTCAN_UR_conv.ipynb cell 2 (:493-514)
//
// The recurrence is latency-bound (30 dependent steps): one persistent workgroup per
// (direction, group of LSTM_NB clips) keeps its gate rows of W_ih / W_hh in registers
// (thread g owns gate row g of 4H = 256) and walks all timesteps inside the kernel; the
// backward kernel runs BPTT in the same layout with W_hh staged in LDS for dh.
#include "common.h"
#include "sensor.h"
#include "layers.h"

#include <algorithm>

namespace f3 {

constexpr int H = 64, G4 = 256;

// ----------------------------------------------------------------------------
// LSTM forward: x [N][T][S] -> seq [N][T][2H] (saved h), gates [2][N][T][4H]
// (post-activation), cell [2][N][T][H], hmean [N][2H]
// ----------------------------------------------------------------------------
__global__ __launch_bounds__(256) void lstm_fwd_kernel(LstmArgs a) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  const int dir = blockIdx.y, n0 = blockIdx.x * LSTM_NB, S = a.S, T = a.T;
  float* xs = sm;                        // [NB][T][S]
  float* hs = xs + LSTM_NB * T * S;      // [NB][H]
  float* gs = hs + LSTM_NB * H;          // [NB][4H]
  const int tid = threadIdx.x;
  const float* wih = a.w_ih[dir];
  const float* whh = a.w_hh[dir];
  float wi[32], wh[H];
#pragma unroll
  for (int s = 0; s < 32; ++s) wi[s] = s < S ? wih[tid * S + s] : 0.f;
#pragma unroll
  for (int u = 0; u < H; ++u) wh[u] = whh[tid * H + u];
  const float bias = a.b_ih[dir][tid] + a.b_hh[dir][tid];
  for (int i = tid; i < LSTM_NB * T * S; i += 256) {
    const int b = i / (T * S), r = i - b * T * S;
    xs[i] = (n0 + b < a.N) ? a.x[(size_t)(n0 + b) * T * S + r] : 0.f;
  }
  for (int i = tid; i < LSTM_NB * H; i += 256) hs[i] = 0.f;
  const int cb = tid / H, cu = tid % H;  // cell-update ownership (LSTM_NB*H == 256)
  float c = 0.f, hsum = 0.f;
  const bool valid = n0 + cb < a.N;
  __syncthreads();
  for (int step = 0; step < T; ++step) {
    const int t = dir ? T - 1 - step : step;
#pragma unroll
    for (int b = 0; b < LSTM_NB; ++b) {
      float acc = bias;
      const float* xr = xs + (b * T + t) * S;
#pragma unroll
      for (int s = 0; s < 32; ++s)
        if (s < S) acc += wi[s] * xr[s];
      const float* hr = hs + b * H;
#pragma unroll
      for (int u = 0; u < H; ++u) acc += wh[u] * hr[u];
      const int gate = tid / H;  // 0 i, 1 f, 2 g, 3 o
      gs[b * G4 + tid] = gate == 2 ? tanhf(acc) : sigmoidf_(acc);
    }
    __syncthreads();
    const float gi = gs[cb * G4 + cu], gf = gs[cb * G4 + H + cu];
    const float gg = gs[cb * G4 + 2 * H + cu], go = gs[cb * G4 + 3 * H + cu];
    c = gf * c + gi * gg;
    const float h = go * tanhf(c);
    hs[cb * H + cu] = h;
    hsum += h;
    if (valid) {
      const size_t nt = (size_t)(n0 + cb) * T + t;
      a.seq[nt * 2 * H + dir * H + cu] = h;
      a.cell[((size_t)dir * a.N * T + nt) * H + cu] = c;
      float* gsv = a.gates + ((size_t)dir * a.N * T + nt) * G4;
      gsv[cu] = gi; gsv[H + cu] = gf; gsv[2 * H + cu] = gg; gsv[3 * H + cu] = go;
    }
    __syncthreads();
  }
  if (valid) a.hmean[(size_t)(n0 + cb) * 2 * H + dir * H + cu] = hsum / (float)T;
}

// ----------------------------------------------------------------------------
// LSTM backward (BPTT). dhmean [N][2H] -> weight grads (+= via atomics), dx (+=)
// ----------------------------------------------------------------------------
__global__ __launch_bounds__(256) void lstm_bwd_kernel(LstmArgs a) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  const int dir = blockIdx.y, n0 = blockIdx.x * LSTM_NB, S = a.S, T = a.T;
  float* whs = sm;                        // W_hh^T [H][4H + 4] (a unit's row of all gates: float4 reads)
  float* wis = whs + G4 * (H + 1);        // [4H][S]   (H * (4H + 4) == 4H * (H + 1))
  float* xs = wis + G4 * S;               // [NB][T][S]
  float* hp = xs + LSTM_NB * T * S;       // [NB][H] h_{prev}
  float* dgs = hp + LSTM_NB * H;          // [NB][4H]
  float* dhr = dgs + LSTM_NB * G4;        // [NB][H] recurrent dh
  const int tid = threadIdx.x;
  for (int i = tid; i < G4 * H; i += 256) whs[(i % H) * (G4 + 4) + i / H] = a.w_hh[dir][i];
  for (int i = tid; i < G4 * S; i += 256) wis[i] = a.w_ih[dir][i];
  for (int i = tid; i < LSTM_NB * T * S; i += 256) {
    const int b = i / (T * S), r = i - b * T * S;
    xs[i] = (n0 + b < a.N) ? a.x[(size_t)(n0 + b) * T * S + r] : 0.f;
  }
  for (int i = tid; i < LSTM_NB * H; i += 256) dhr[i] = 0.f;
  const int cb = tid / H, cu = tid % H;
  const bool valid = n0 + cb < a.N;
  const float dmean = valid ? a.dhmean[(size_t)(n0 + cb) * 2 * H + dir * H + cu] / (float)T : 0.f;
  float dc = 0.f;
  float gwh[H], gwi[32], gb = 0.f;
#pragma unroll
  for (int u = 0; u < H; ++u) gwh[u] = 0.f;
#pragma unroll
  for (int s = 0; s < 32; ++s) gwi[s] = 0.f;
  // the saved gates / cell / h of (clip cb, unit cu) at the time a processing step handles,
  // loaded one step ahead (unconditional loads from a clamped clip index: the recurrence chain
  // then never waits on global memory)
  struct StepVals { float gi, gf, gg, go, ct, cp, hprev; };
  const int cbc = min(n0 + cb, a.N - 1);
  auto load_step = [&](int step) {
    StepVals r;
    const int t = dir ? T - 1 - step : step, tp = dir ? t + 1 : t - 1;
    const int tpc = min(max(tp, 0), T - 1);
    const size_t nt = (size_t)cbc * T + t, ntp = (size_t)cbc * T + tpc;
    const float* gsv = a.gates + ((size_t)dir * a.N * T + nt) * G4;
    r.gi = gsv[cu]; r.gf = gsv[H + cu]; r.gg = gsv[2 * H + cu]; r.go = gsv[3 * H + cu];
    r.ct = a.cell[((size_t)dir * a.N * T + nt) * H + cu];
    r.cp = a.cell[((size_t)dir * a.N * T + ntp) * H + cu];
    r.hprev = a.seq[ntp * 2 * H + dir * H + cu];
    return r;
  };
  StepVals nxt = load_step(T - 1);
  __syncthreads();
  for (int step = T - 1; step >= 0; --step) {
    const int t = dir ? T - 1 - step : step;           // time of this processing step
    const bool has_prev = step > 0;
    const StepVals cur = nxt;
    if (step > 0) nxt = load_step(step - 1);
    // (b, u): cell backward
    {
      float gi = 0, gf = 0, gg = 0, go = 0, ct = 0, cp = 0;
      if (valid) {
        gi = cur.gi; gf = cur.gf; gg = cur.gg; go = cur.go;
        ct = cur.ct;
        if (has_prev) {
          cp = cur.cp;
          hp[cb * H + cu] = cur.hprev;
        } else {
          hp[cb * H + cu] = 0.f;
        }
      } else {
        hp[cb * H + cu] = 0.f;
      }
      const float dh = dmean + dhr[cb * H + cu];
      const float tc = tanhf(ct);
      const float dov = dh * tc;
      dc += dh * go * (1.f - tc * tc);
      const float div = dc * gg, dgv = dc * gi, dfv = dc * cp;
      dc = dc * gf;
      float* dg = dgs + cb * G4;
      dg[cu] = valid ? div * gi * (1.f - gi) : 0.f;
      dg[H + cu] = valid ? dfv * gf * (1.f - gf) : 0.f;
      dg[2 * H + cu] = valid ? dgv * (1.f - gg * gg) : 0.f;
      dg[3 * H + cu] = valid ? dov * go * (1.f - go) : 0.f;
    }
    __syncthreads();
    // thread = gate row: weight-gradient accumulation
#pragma unroll
    for (int b = 0; b < LSTM_NB; ++b) {
      const float d = dgs[b * G4 + tid];
      gb += d;
      const float* xr = xs + (b * T + t) * S;
#pragma unroll
      for (int s = 0; s < 32; ++s)
        if (s < S) gwi[s] += d * xr[s];
      const f32x4* hr = reinterpret_cast<const f32x4*>(hp + b * H);
#pragma unroll
      for (int u4 = 0; u4 < H / 4; ++u4) {
        const f32x4 h = hr[u4];
#pragma unroll
        for (int e = 0; e < 4; ++e) gwh[4 * u4 + e] += d * h[e];
      }
    }
    // (b, u'): recurrent dh = sum_g dgates[g] W_hh[g][u'] (16-B reads of both rows)
    {
      const f32x4* dg = reinterpret_cast<const f32x4*>(dgs + cb * G4);
      const f32x4* wr = reinterpret_cast<const f32x4*>(whs + cu * (G4 + 4));
      f32x4 acc4 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll 8
      for (int j = 0; j < G4 / 4; ++j) acc4 += dg[j] * wr[j];
      const float acc = (acc4[0] + acc4[1]) + (acc4[2] + acc4[3]);
      __syncthreads();  // everyone finished reading dhr of this step (dh above)
      dhr[cb * H + cu] = acc;
    }
    if (a.dx) {
      for (int i = tid; i < LSTM_NB * S; i += 256) {
        const int b = i / S, s = i - b * S;
        if (n0 + b >= a.N) continue;
        float acc = 0.f;
        for (int g = 0; g < G4; ++g) acc += dgs[b * G4 + g] * wis[g * S + s];
        atomic_add_f(a.dx + ((size_t)(n0 + b) * T + t) * S + s, acc);
      }
    }
    __syncthreads();
  }
  if (a.wpart) {  // this (direction, clip tile)'s partial row [bias | w_ih | w_hh], summed by f3_lstm_bwd
    float* row = a.wpart + ((size_t)dir * gridDim.x + blockIdx.x) * G4 * (1 + S + H);
    row[tid] = gb;
    for (int s = 0; s < S && s < 32; ++s) row[G4 + tid * S + s] = gwi[s];
#pragma unroll
    for (int u = 0; u < H; ++u) row[G4 * (1 + S) + tid * H + u] = gwh[u];
    return;
  }
  atomic_add_f(a.g_b_ih[dir] + tid, gb);
  atomic_add_f(a.g_b_hh[dir] + tid, gb);
  for (int s = 0; s < S && s < 32; ++s) atomic_add_f(a.g_w_ih[dir] + tid * S + s, gwi[s]);
#pragma unroll
  for (int u = 0; u < H; ++u) atomic_add_f(a.g_w_hh[dir] + tid * H + u, gwh[u]);
}

// ----------------------------------------------------------------------------
// sensor head: hmean -> BN1d(2H, batch stats) -> CA (2H->2H/8->2H) -> Linear(2H->Cs)
// ----------------------------------------------------------------------------
constexpr int HC = 2 * H, HR = HC / 8;

// Two launches: the BatchNorm1d batch statistics (one workgroup, 8 row slices per channel, fp64) and
// one workgroup of 128 threads per clip for BN -> CA -> Linear (a single workgroup walking every
// [N x 128] stage alone took 127 us at N = 256).
__global__ __launch_bounds__(1024) void shead_stats_kernel(SHeadArgs a) {
  __shared__ double rs[8][HC], rq[8][HC];
  const int c = threadIdx.x % HC, part = threadIdx.x / HC;
  double sum = 0.0, sq = 0.0;
  for (int n = part; n < a.N; n += 8) {
    const double v = a.hmean[(size_t)n * HC + c];
    sum += v;
    sq += v * v;
  }
  rs[part][c] = sum;
  rq[part][c] = sq;
  __syncthreads();
  if (part == 0) {
    for (int p = 1; p < 8; ++p) {
      sum += rs[p][c];
      sq += rq[p][c];
    }
    a.bn_sum[c] = sum;
    a.bn_sq[c] = sq;
  }
}

__global__ __launch_bounds__(128) void shead_clip_kernel(SHeadArgs a) {
  __shared__ float y[HC], h1[HR], yt[HC];
  const int n = blockIdx.x, c = threadIdx.x;
  float mean, rstd;
  if (a.bn.eval) {
    mean = a.bn.rmean[c];
    rstd = rsqrtf(a.bn.rvar[c] + kBnEps);
  } else {
    const double m = a.bn_sum[c] / a.N;
    double var = a.bn_sq[c] / a.N - m * m;
    if (var < 0) var = 0;
    mean = (float)m;
    rstd = (float)(1.0 / sqrt(var + kBnEps));
  }
  const float sc = a.bn.gamma[c] * rstd, sh = a.bn.beta[c] - mean * sc;
  const float yv = a.hmean[(size_t)n * HC + c] * sc + sh;
  a.ybn[(size_t)n * HC + c] = yv;
  y[c] = yv;
  __syncthreads();
  if (c < HR) {
    float q = a.b1[c];
    for (int k = 0; k < HC; ++k) q += a.W1[c * HC + k] * y[k];
    q = fmaxf(q, 0.f);
    h1[c] = q;
    a.a1[(size_t)n * HR + c] = q;
  }
  __syncthreads();
  float q = a.b2[c];
#pragma unroll
  for (int j = 0; j < HR; ++j) q += a.W2[c * HR + j] * h1[j];
  const float at = sigmoidf_(q);
  a.att[(size_t)n * HC + c] = at;
  yt[c] = yv * at;
  __syncthreads();
  for (int k = c; k < a.Cs; k += HC) {
    float o = a.b3[k];
    const float* w = a.W3 + (size_t)k * HC;
    for (int j = 0; j < HC; ++j) o += w[j] * yt[j];
    a.out[(size_t)n * a.out_ld + k] = o;
  }
}

// The backward as four launches whose outputs are spread over the whole chip (one thread per
// output, the batch reduction in a loop): a single-workgroup form took 640 us on one CU and
// delayed the motion stream's weight gradients queued behind it.
//
// Batch sums use 4 independent partial sums (n = u mod 4), so the loads of 4 clips are in
// flight together instead of one dependent add chain of N loads.
template <class F>
F3_DEV float batch_sum(int N, F f) {
  float p0 = 0.f, p1 = 0.f, p2 = 0.f, p3 = 0.f;
  int n = 0;
  for (; n + 4 <= N; n += 4) {
    p0 += f(n);
    p1 += f(n + 1);
    p2 += f(n + 2);
    p3 += f(n + 3);
  }
  for (; n < N; ++n) p0 += f(n);
  return (p0 + p1) + (p2 + p3);
}

__global__ __launch_bounds__(256) void shead_bwd_p1(SHeadArgs a) {  // W3 / b3 grads, dy, dpre2
  const int N = a.N, Cs = a.Cs;
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i < Cs * HC) {
    const int k = i / HC, c = i - k * HC;
    a.g_W3[i] += batch_sum(N, [&](int n) {
      return a.dout[(size_t)n * a.dout_ld + k] * a.ybn[(size_t)n * HC + c] * a.att[(size_t)n * HC + c];
    });
  } else if (i < Cs * HC + Cs) {
    const int k = i - Cs * HC;
    a.g_b3[k] += batch_sum(N, [&](int n) { return a.dout[(size_t)n * a.dout_ld + k]; });
  } else if (i < Cs * HC + Cs + N * HC) {
    const int e = i - Cs * HC - Cs, n = e / HC, c = e - n * HC;
    float d = 0.f;
    for (int k = 0; k < Cs; ++k) d += a.dout[(size_t)n * a.dout_ld + k] * a.W3[(size_t)k * HC + c];
    const float at = a.att[e];
    a.dy[e] = d * at;
    a.dpre2[e] = d * a.ybn[e] * at * (1.f - at);
  }
}

__global__ __launch_bounds__(256) void shead_bwd_p2(SHeadArgs a) {  // W2 / b2 grads, dpre1
  const int N = a.N;
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i < HC * HR) {
    const int c = i / HR, j = i - c * HR;
    a.g_W2[i] += batch_sum(N, [&](int n) { return a.dpre2[(size_t)n * HC + c] * a.a1[(size_t)n * HR + j]; });
    if (j == 0) a.g_b2[c] += batch_sum(N, [&](int n) { return a.dpre2[(size_t)n * HC + c]; });
  } else if (i < HC * HR + N * HR) {
    const int e = i - HC * HR, n = e / HR, j = e - n * HR;
    float acc = 0.f;
    for (int c = 0; c < HC; ++c) acc += a.dpre2[(size_t)n * HC + c] * a.W2[c * HR + j];
    a.dpre1[e] = a.a1[e] > 0.f ? acc : 0.f;
  }
}

__global__ __launch_bounds__(256) void shead_bwd_p3(SHeadArgs a) {  // W1 / b1 grads, dy += W1^T dpre1
  const int N = a.N;
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i < HR * HC) {
    const int j = i / HC, c = i - j * HC;
    a.g_W1[i] += batch_sum(N, [&](int n) { return a.dpre1[(size_t)n * HR + j] * a.ybn[(size_t)n * HC + c]; });
    if (c == 0) a.g_b1[j] += batch_sum(N, [&](int n) { return a.dpre1[(size_t)n * HR + j]; });
  } else if (i < HR * HC + N * HC) {
    const int e = i - HR * HC, n = e / HC, c = e - n * HC;
    float acc = 0.f;
    for (int j = 0; j < HR; ++j) acc += a.dpre1[(size_t)n * HR + j] * a.W1[j * HC + c];
    a.dy[e] += acc;
  }
}

__global__ __launch_bounds__(1024) void shead_bwd_p4(SHeadArgs a) {  // BatchNorm1d backward
  __shared__ float red1[HC], red2[HC], mean_s[HC], rstd_s[HC];
  const int tid = threadIdx.x, N = a.N;
  if (tid < HC) {
    const int c = tid;
    const double m = a.bn_sum[c] / N;
    double var = a.bn_sq[c] / N - m * m;
    if (var < 0) var = 0;
    const float rstd = (float)(1.0 / sqrt(var + kBnEps));
    const float mf = (float)m;
    const float s1 = batch_sum(N, [&](int n) { return a.dy[(size_t)n * HC + c]; });
    const float s2 = batch_sum(N, [&](int n) { return a.dy[(size_t)n * HC + c] * ((a.hmean[(size_t)n * HC + c] - mf) * rstd); });
    a.g_gamma[c] += s2;
    a.g_beta[c] += s1;
    red1[c] = s1 / N;
    red2[c] = s2 / N;
    mean_s[c] = mf;
    rstd_s[c] = rstd;
  }
  __syncthreads();
  for (int i = tid; i < N * HC; i += 1024) {
    const int c = i % HC;
    const float mean = mean_s[c], rstd = rstd_s[c];
    const float xh = (a.hmean[i] - mean) * rstd;
    a.dhmean[i] = a.bn.gamma[c] * rstd * (a.dy[i] - red1[c] - xh * red2[c]);
  }
}

// ----------------------------------------------------------------------------
// CNN1D: Conv1d(k5,p2) -> BN (batch stats) -> ReLU -> MaxPool1d(2), twice
// (GSTCAN_UR_conv.ipynb:493-514; layout [N][T][C] rows, time-major, channel contiguous).
// The tensors are tiny (B=256: 0.1-0.5 MB each), so these kernels are latency-bound; what they
// avoid is contention: a block walks several clips with a FIXED channel per thread
// (blockDim % Co == 0), keeps its BN / bias / weight-gradient partials in registers and adds
// them to HBM once per block (the first version added fp64 per element: 2 atomics x N*T*Co on
// Co addresses).
// ----------------------------------------------------------------------------
constexpr int C1D_THREADS = 256;
constexpr int C1D_GRID = 128;   // conv backward: blocks (each walks N / 128 clips)
constexpr int C1D_WMAX = 10;    // weight-gradient elements per thread: Co*Ci*5 <= 2560

// sum v over the threads of one channel (tid % Co == o) and add it to dst[o] (fp64)
F3_DEV void c1d_flush(float v, double* dst, float* red, int Co) {
  const int tid = threadIdx.x;
  __syncthreads();
  red[tid] = v;
  __syncthreads();
  if (tid < Co) {
    float s = 0.f;
    for (int i = tid; i < C1D_THREADS; i += Co) s += red[i];
    atomic_add_d(dst + tid, (double)s);
  }
}

// one block per clip; the clip's input rows and the weights in LDS
__global__ __launch_bounds__(C1D_THREADS) void conv1d_fwd_kernel(Conv1dArgs a) {
  extern __shared__ float c1d_sm[];
  float* ws = c1d_sm;                       // [Co][Ci][5]
  float* xs = ws + a.Co * a.Ci * 5;         // [T][Ci]
  float* red = xs + a.T * a.Ci;             // [256]
  const int tid = threadIdx.x, n = blockIdx.x, o = tid % a.Co, TCo = a.T * a.Co, TCi = a.T * a.Ci;
  for (int i = tid; i < a.Co * a.Ci * 5; i += C1D_THREADS) ws[i] = a.w[i];
  for (int i = tid; i < TCi; i += C1D_THREADS) xs[i] = a.x[(size_t)n * TCi + i];
  __syncthreads();
  float s1 = 0.f, s2 = 0.f;
  const float bo = a.b[o];
  for (int i = tid; i < TCo; i += C1D_THREADS) {  // i % Co == o for every i of this thread
    const int t = i / a.Co;
    float acc = bo;
    for (int k = 0; k < 5; ++k) {
      const int ti = t + k - 2;
      if (ti < 0 || ti >= a.T) continue;
      const float* xr = xs + ti * a.Ci;
      const float* wr = ws + o * a.Ci * 5 + k;
      for (int c = 0; c < a.Ci; ++c) acc += wr[c * 5] * xr[c];
    }
    a.y[(size_t)n * TCo + i] = acc;
    s1 += acc;
    s2 += acc * acc;
  }
  c1d_flush(s1, a.st_sum, red, a.Co);
  c1d_flush(s2, a.st_sq, red, a.Co);
}

__global__ __launch_bounds__(C1D_THREADS) void bnrelupool_fwd_kernel(Conv1dArgs a) {
  const int Tp = a.T / 2, tot = a.N * Tp * a.Co;
  for (int i = blockIdx.x * C1D_THREADS + threadIdx.x; i < tot; i += gridDim.x * C1D_THREADS) {
    const int o = i % a.Co, r = i / a.Co, n = r / Tp, tp = r - n * Tp;
    float sc, sh, mu, rs;
    bn_coeff(a.bn, o, sc, sh, mu, rs);
    const float* y = a.y + ((size_t)n * a.T + 2 * tp) * a.Co + o;
    a.p[i] = fmaxf(fmaxf(y[0] * sc + sh, 0.f), fmaxf(y[a.Co] * sc + sh, 0.f));
  }
}

// gradient through MaxPool + ReLU to the BN output, with the BN-backward sums (one block per clip)
__global__ __launch_bounds__(C1D_THREADS) void bnrelupool_bwd_kernel(Conv1dArgs a) {
  __shared__ float red[C1D_THREADS];
  const int tid = threadIdx.x, o = tid % a.Co, Tp = a.T / 2, TCo = a.T * a.Co, n = blockIdx.x;
  float sc, sh, mu, rs;
  bn_coeff(a.bn, o, sc, sh, mu, rs);
  float s1 = 0.f, s2 = 0.f;
  const float* yc = a.y + (size_t)n * TCo;
  for (int i = tid; i < TCo; i += C1D_THREADS) {
    const int t = i / a.Co;
    const float yv = yc[i];
    float d = 0.f;
    const int tp = t >> 1;
    if (tp < Tp) {
      const float v0 = fmaxf(yc[(2 * tp) * a.Co + o] * sc + sh, 0.f);
      const float v1 = fmaxf(yc[(2 * tp + 1) * a.Co + o] * sc + sh, 0.f);
      const int win = (v1 > v0) ? 1 : 0;  // first max wins ties (max_pool1d)
      const float me = fmaxf(yv * sc + sh, 0.f);
      if ((t & 1) == win && me > 0.f) d = a.dp[((size_t)n * Tp + tp) * a.Co + o];
    }
    a.dy[(size_t)n * TCo + i] = d;
    s1 += d;
    s2 += d * ((yv - mu) * rs);
  }
  c1d_flush(s1, a.bsum, red, a.Co);
  c1d_flush(s2, a.bsq, red, a.Co);
}

// BN apply backward, then the conv1d backward: dx per clip, dW and db as per-thread register
// partials over the block's clips (thread tid owns weight elements tid, tid + 256, ...)
__global__ __launch_bounds__(C1D_THREADS) void conv1d_bwd_kernel(Conv1dArgs a) {
  extern __shared__ float c1d_sm[];
  float* dcs = c1d_sm;                    // [T][Co] pre-BN gradient of the clip
  float* xs = dcs + a.T * a.Co;           // [T][Ci] the clip's conv input
  float* ws = xs + a.T * a.Ci;            // [Co][Ci][5]
  const int tid = threadIdx.x, TCo = a.T * a.Co, TCi = a.T * a.Ci, NW = a.Co * a.Ci * 5;
  const float M = a.bn.count;
  float gw[C1D_WMAX], gb = 0.f;
#pragma unroll
  for (int e = 0; e < C1D_WMAX; ++e) gw[e] = 0.f;
  for (int i = tid; i < NW; i += C1D_THREADS) ws[i] = a.w[i];
  if (blockIdx.x == 0) {
    for (int o = tid; o < a.Co; o += C1D_THREADS) {
      a.g_gamma[o] += (float)a.bsq[o];
      a.g_beta[o] += (float)a.bsum[o];
    }
  }
  for (int n = blockIdx.x; n < a.N; n += gridDim.x) {
    __syncthreads();  // the previous clip's readers are done
    for (int i = tid; i < TCo; i += C1D_THREADS) {
      const int o = i % a.Co;
      float sc, sh, mu, rs;
      bn_coeff(a.bn, o, sc, sh, mu, rs);
      const float xh = (a.y[(size_t)n * TCo + i] - mu) * rs;
      const float d = a.dy[(size_t)n * TCo + i];
      dcs[i] = a.bn.gamma[o] * rs * (d - (float)a.bsum[o] / M - xh * (float)a.bsq[o] / M);
    }
    for (int i = tid; i < TCi; i += C1D_THREADS) xs[i] = a.x[(size_t)n * TCi + i];
    __syncthreads();
    if (tid < a.Co)
      for (int t = 0; t < a.T; ++t) gb += dcs[t * a.Co + tid];
#pragma unroll
    for (int e = 0; e < C1D_WMAX; ++e) {
      const int i = tid + e * C1D_THREADS;
      if (i >= NW) break;
      const int o = i / (a.Ci * 5), r = i - o * a.Ci * 5, c = r / 5, k = r - c * 5;
      float acc = 0.f;
      for (int t = max(0, 2 - k); t < min(a.T, a.T + 2 - k); ++t) acc += dcs[t * a.Co + o] * xs[(t + k - 2) * a.Ci + c];
      gw[e] += acc;
    }
    if (a.dx) {
      for (int i = tid; i < TCi; i += C1D_THREADS) {
        const int ti = i / a.Ci, c = i - ti * a.Ci;
        float acc = 0.f;
        for (int k = 0; k < 5; ++k) {
          const int t = ti - k + 2;
          if (t < 0 || t >= a.T) continue;
          for (int o = 0; o < a.Co; ++o) acc += dcs[t * a.Co + o] * ws[(o * a.Ci + c) * 5 + k];
        }
        a.dx[(size_t)n * TCi + i] = acc;
      }
    }
  }
  if (tid < a.Co) atomic_add_f(a.g_b + tid, gb);
#pragma unroll
  for (int e = 0; e < C1D_WMAX; ++e) {
    const int i = tid + e * C1D_THREADS;
    if (i < NW) atomic_add_f(a.g_w + i, gw[e]);
  }
}


}  // namespace f3

using namespace f3;

static size_t lstm_fwd_lds(const LstmArgs& a) {
  return ((size_t)LSTM_NB * a.T * a.S + LSTM_NB * H + LSTM_NB * G4) * 4;
}
static size_t lstm_bwd_lds(const LstmArgs& a) {
  return ((size_t)G4 * (H + 1) + G4 * a.S + LSTM_NB * a.T * a.S + LSTM_NB * H + LSTM_NB * G4 + LSTM_NB * H) * 4;
}

int f3_lstm_fwd(const LstmArgs* a, hipStream_t s) {
  if (a->S > 32 || a->S < 1) return F3_EINVAL;
  dim3 grid((a->N + LSTM_NB - 1) / LSTM_NB, 2);
  hipLaunchKernelGGL(lstm_fwd_kernel, grid, dim3(256), lstm_fwd_lds(*a), s, *a);
  F3_LAUNCH_CHECK();
  return F3_OK;
}

int f3_lstm_bwd(const LstmArgs* a, hipStream_t s) {
  if (a->S > 32 || a->S < 1) return F3_EINVAL;
  dim3 grid((a->N + LSTM_NB - 1) / LSTM_NB, 2);
  const size_t lds = lstm_bwd_lds(*a);
  if (lds > 160 * 1024) return F3_EINVAL;
  static bool once = (hipFuncSetAttribute((const void*)lstm_bwd_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                                           160 * 1024), (void)hipGetLastError(), true);
  (void)once;
  hipLaunchKernelGGL(lstm_bwd_kernel, grid, dim3(256), lds, s, *a);
  F3_LAUNCH_CHECK();
  if (!a->wpart) return F3_OK;
  const int tiles = grid.x, S = a->S, row = G4 * (1 + S + H);
  for (int d = 0; d < 2; ++d) {
    const float* p = a->wpart + (size_t)d * tiles * row;
    F3_TRY(f3_colsum_ld(p, tiles, row, G4, a->g_b_ih[d], s));
    F3_TRY(f3_colsum_ld(p, tiles, row, G4, a->g_b_hh[d], s));
    F3_TRY(f3_colsum_ld(p + G4, tiles, row, G4 * S, a->g_w_ih[d], s));
    F3_TRY(f3_colsum_ld(p + G4 * (1 + S), tiles, row, G4 * H, a->g_w_hh[d], s));
  }
  return F3_OK;
}

int f3_shead_fwd(const SHeadArgs* a, hipStream_t s) {
  if (!a->bn.eval) {
    hipLaunchKernelGGL(shead_stats_kernel, dim3(1), dim3(1024), 0, s, *a);
    F3_LAUNCH_CHECK();
  }
  hipLaunchKernelGGL(shead_clip_kernel, dim3(a->N), dim3(HC), 0, s, *a);
  F3_LAUNCH_CHECK();
  return F3_OK;
}

int f3_shead_bwd(const SHeadArgs* a, hipStream_t s) {
  const int N = a->N, Cs = a->Cs;
  auto blocks = [](int n) { return dim3((n + 255) / 256); };
  hipLaunchKernelGGL(shead_bwd_p1, blocks(Cs * HC + Cs + N * HC), dim3(256), 0, s, *a);
  F3_LAUNCH_CHECK();
  hipLaunchKernelGGL(shead_bwd_p2, blocks(HC * HR + N * HR), dim3(256), 0, s, *a);
  F3_LAUNCH_CHECK();
  hipLaunchKernelGGL(shead_bwd_p3, blocks(HR * HC + N * HC), dim3(256), 0, s, *a);
  F3_LAUNCH_CHECK();
  hipLaunchKernelGGL(shead_bwd_p4, dim3(1), dim3(1024), 0, s, *a);
  F3_LAUNCH_CHECK();
  return F3_OK;
}

static int c1d_grid(const Conv1dArgs& a) { return std::max(1, std::min(a.N, C1D_GRID)); }
static bool c1d_ok(const Conv1dArgs& a) {
  return a.Co >= 1 && C1D_THREADS % a.Co == 0 && a.Co * a.Ci * 5 <= C1D_WMAX * C1D_THREADS && a.T >= 1;
}

int f3_conv1d_fwd(const Conv1dArgs* a, hipStream_t s) {
  if (!c1d_ok(*a)) return F3_EINVAL;
  const size_t lds = ((size_t)a->Co * a->Ci * 5 + (size_t)a->T * a->Ci + C1D_THREADS) * 4;
  hipLaunchKernelGGL(conv1d_fwd_kernel, dim3(a->N), dim3(C1D_THREADS), lds, s, *a);
  F3_LAUNCH_CHECK();
  return F3_OK;
}

int f3_bnrelupool_fwd(const Conv1dArgs* a, hipStream_t s) {
  const int tot = a->N * (a->T / 2) * a->Co;
  if (tot <= 0) return F3_OK;
  hipLaunchKernelGGL(bnrelupool_fwd_kernel, dim3(std::min((tot + C1D_THREADS - 1) / C1D_THREADS, 1024)),
                     dim3(C1D_THREADS), 0, s, *a);
  F3_LAUNCH_CHECK();
  return F3_OK;
}

int f3_conv1d_bwd(const Conv1dArgs* a, hipStream_t s) {
  if (!c1d_ok(*a)) return F3_EINVAL;
  hipLaunchKernelGGL(bnrelupool_bwd_kernel, dim3(a->N), dim3(C1D_THREADS), 0, s, *a);
  F3_LAUNCH_CHECK();
  hipLaunchKernelGGL(conv1d_bwd_kernel, dim3(c1d_grid(*a)), dim3(C1D_THREADS),
                     ((size_t)a->T * (a->Co + a->Ci) + (size_t)a->Co * a->Ci * 5) * 4, s, *a);
  F3_LAUNCH_CHECK();
  return F3_OK;
}

