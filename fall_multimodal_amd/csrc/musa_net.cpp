// musa_model.Model training step behind the C ABI (include/fall3.h f3_musa_*).
//
// Replaces, for the root driver Multimodal_Fall3/main.py (:307-320, train loop :79-132):
//   model = Model(num_class=11, num_point=14, max_frame=300, graph=adjGraph('coco_cut','uniform'),
//                 bias=True, edge=True, block_size=41, embed_dim=64, n_stage=1, act_type='tanh')
//                                                   -> f3_musa_create   (musa_model.py:492-559)
//   pred = model(data)                              -> f3_musa_forward  (:561-589)
//   loss.backward()                                 -> f3_musa_backward
//
// Each stream (positions, T=30; motion, T=29) runs SpatialGraphConv(64->128), SepTemporal_Block
// (k3 s1), SepTemporal_Block (k5 s2, strided residual), Sep_TCN(128->256) over channels-last
// rows. 1x1 convs: the shared fp32 MFMA GEMM (+bias, +BatchNorm sums in the epilogue); the graph
// mix: f3_mix_fwd (one partition); depthwise convs, BatchNorm/activation passes, DropBlock and the
// block merges: musa.hip.
#include <hip/hip_runtime.h>

#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "fall3.h"
#include "kernels.h"
#include "layers.h"
#include "musa.h"

using namespace f3;
using namespace f3::mu;

namespace {

struct Entry {
  std::string name;
  int kind;
  std::vector<int64_t> shape;
  int64_t off;
};

struct BnOff {
  int64_t w, b, rm, rv, nbt;
  int C, slot;
};

struct StreamOff {
  int64_t emb_w, emb_b;
  // SpatialGraphConv
  int64_t A0, e0, gcn_w, gcn_b, res0_w, res0_b;
  BnOff bn_h, bn_r0;
  // SepTemporal blocks 1 (k3 s1) and 2 (k5 s2)
  int64_t A[2], edge[2], dw_w[2], dw_b[2], pw_w[2], pw_b[2], res2_w, res2_b;
  BnOff bn_d[2], bn_p[2], bn_r2;
  // Sep_TCN
  int64_t d1_w, d1_b, p1_w, p1_b, d2_w, d2_b, p2_w, p2_b, sc_w, sc_b;
  BnOff bn1, bn2, bn3, bn4;
};

constexpr int E = 64, C1 = 128, CM = 192, C2 = 256, HIDDEN = 128;
constexpr float kKeepProb = 0.9f;   // musa_model.py:509
constexpr int kBlockSize = 41;      // main.py:316
constexpr float kHeadDrop = 0.2f;   // Classification_Module Dropout(0.2)

}  // namespace

struct f3_musa {
  int V, T, C;
  int prec = F3_PRECISION_FP32;  // F3_PRECISION_BF16: the stream 1x1 convs on bf16 MFMA (fp32 accumulate)
  std::vector<Entry> entries;
  int64_t nparam = 0, nbuf = 0, ncnt = 0;
  StreamOff st[2];
  int64_t fc0_w, fc0_b, ln_w, ln_b, fc5_w, fc5_b;
  std::vector<BnOff*> bns;
  // the last training forward's draws (the backward replays the masks it built)
  unsigned seed = 0;
  int drop = 0;
  int trained_batch = 0;

  int64_t add(const std::string& name, std::vector<int64_t> shape, int kind = F3_ENTRY_PARAM) {
    int64_t n = 1;
    for (auto d : shape) n *= d;
    Entry e{name, kind, shape, 0};
    if (kind == F3_ENTRY_PARAM) {
      e.off = nparam;
      nparam += (n + 3) / 4 * 4;
    } else if (kind == F3_ENTRY_BUFFER) {
      e.off = nbuf;
      nbuf += n;
    } else {
      e.off = ncnt;
      ncnt += 1;
    }
    entries.push_back(e);
    return e.off;
  }
  void add_bn(BnOff& o, const std::string& p, int C) {
    o.w = add(p + "weight", {C});
    o.b = add(p + "bias", {C});
    o.rm = add(p + "running_mean", {C}, F3_ENTRY_BUFFER);
    o.rv = add(p + "running_var", {C}, F3_ENTRY_BUFFER);
    o.nbt = add(p + "num_batches_tracked", {}, F3_ENTRY_COUNTER);
    o.C = C;
    o.slot = (int)bns.size();
    bns.push_back(&o);
  }
};

namespace {

struct StreamWs {
  int T, T2, cin;
  size_t tok, e0, r0, g, h, out1, d1, ee1, p1, out2, d2, ee2, p2, r2, out3;
  size_t td1, te1, tp1, te2, td2, te3, tp2, tres, out4;
  size_t fS[6], fT[6];
  size_t Ae[3];
  size_t dy4;  // head -> stream output gradient
};

struct Plan {
  StreamWs s[2];
  size_t a;            // DropBlock statistics scratch [R]
  size_t feat, z1, stat, h, dz1;
  size_t fsum, bsum;   // [22 BN][2][256] doubles
  size_t packT;        // transposed 1x1 weights for the input-gradient GEMMs (per stream)
  size_t packF;        // bf16 mode: the stream 1x1 weights as bf16 GEMM operands ([O][I], same slots)
  size_t ga, gb, gc, gd;  // backward scratch [R][256]
  size_t part;         // depthwise weight-gradient partials
  size_t mixpart;      // graph-mix dA partial rows
  size_t dmscr;        // DropBlock scratch (f3_mu_dropmask_scratch_floats)
  size_t lanes;        // per-channel reduction lanes (2 * kLaneFloats; finalize re-zeroes them)
  size_t total;
};

constexpr int kPackPerStream = C1 * E * 2 + C1 * C1 * 3 + CM * C1 + C2 * CM + C2 * C1;

// F3_MU_GUARD=<bytes> (debugging): a guard band after every region; f3_musa_guards lists them so a
// tool can fill the workspace with a pattern and find any kernel writing outside its region
size_t guard_bytes() {
  static const size_t g = getenv("F3_MU_GUARD") ? (size_t)atol(getenv("F3_MU_GUARD")) / 256 * 256 : 0;
  return g;
}

Plan plan(const f3_musa* net, int N, std::vector<size_t>* guards = nullptr) {
  Plan p;
  size_t o = 0;
  const size_t gb = guard_bytes();
  auto take = [&](size_t bytes) {
    const size_t at = o;
    o += (bytes + 255) / 256 * 256;
    if (gb) {
      if (guards) guards->push_back(o);
      o += gb;
    }
    return at;
  };
  const int V = net->V;
  size_t Rmax = 0;
  for (int si = 0; si < 2; ++si) {
    StreamWs& w = p.s[si];
    w.T = si == 0 ? net->T : net->T - 1;
    w.T2 = (w.T + 4 - 5) / 2 + 1;
    w.cin = si == 0 ? 3 : 2;
    const size_t R = (size_t)N * w.T * V, R2 = (size_t)N * w.T2 * V;
    Rmax = std::max(Rmax, R);
    w.tok = take(4 * R * 4);
    w.e0 = take(4 * R * E);
    for (size_t* t : {&w.r0, &w.g, &w.h, &w.out1, &w.d1, &w.ee1, &w.p1, &w.out2}) *t = take(4 * R * C1);
    for (size_t* t : {&w.d2, &w.ee2, &w.p2, &w.r2, &w.out3, &w.td1, &w.te1}) *t = take(4 * R2 * C1);
    for (size_t* t : {&w.tp1, &w.te2, &w.td2, &w.te3}) *t = take(4 * R2 * CM);
    for (size_t* t : {&w.tp2, &w.tres, &w.out4, &w.dy4}) *t = take(4 * R2 * C2);
    for (int k = 0; k < 6; ++k) {
      w.fS[k] = take(4 * (size_t)N * V);
      w.fT[k] = take(4 * (size_t)N * w.T);
    }
    for (int k = 0; k < 3; ++k) w.Ae[k] = take(4 * V * V);
  }
  p.a = take(4 * Rmax);
  const int F = 2 * C2 + 3;
  p.feat = take(4 * (size_t)N * F);
  p.z1 = take(4 * (size_t)N * HIDDEN);
  p.stat = take(4 * (size_t)N * 2);
  p.h = take(4 * (size_t)N * HIDDEN);
  p.dz1 = take(4 * (size_t)N * HIDDEN);
  p.fsum = take(8 * 22 * 512);
  p.bsum = take(8 * 22 * 512);
  p.packT = take(4 * 2 * (size_t)kPackPerStream);
  p.packF = net->prec == F3_PRECISION_BF16 ? take(4 * 2 * (size_t)kPackPerStream) : 0;
  p.ga = take(4 * Rmax * C2);
  p.gb = take(4 * Rmax * C2);
  p.gc = take(4 * Rmax * C2);
  p.gd = take(4 * Rmax * C2);
  p.part = take(4 * 512 * (size_t)CM * 6);
  p.mixpart = take(4 * (size_t)kMixParts * 1024);
  p.dmscr = take(4 * (size_t)f3_mu_dropmask_scratch_floats(N, net->T, V));
  p.lanes = take(4 * 2 * kLaneFloats);
  p.total = o;
  return p;
}

template <typename P>
P* at(void* ws, size_t off) {
  return reinterpret_cast<P*>(reinterpret_cast<char*>(ws) + off);
}

#define MU_TRY(x)                 \
  do {                            \
    const int _st = (x);          \
    if (_st != F3_OK) return _st; \
  } while (0)

// 1x1 conv over rows [N][T_in][V][I] -> [N][T_out][V][O] with stride S over T (fp32 MFMA GEMM)
ConvGemmArgs conv1x1(int N, int T_in, int T_out, int V, int I, int O, int S, const float* in, const float* W,
                     const float* bias, float* out) {
  ConvGemmArgs a;
  std::memset(&a, 0, sizeof(a));
  a.g.M = N * T_out * V; a.g.Nc = O; a.g.Kc = I; a.g.KT = 1; a.g.S = S; a.g.P = 0; a.g.transposed = 0;
  a.g.T_out = T_out; a.g.T_in = T_in; a.g.V = V; a.g.lda = I; a.g.ldo = O;
  a.in = in; a.w = W; a.out = out; a.bias = bias;
  return a;
}

// input gradient of that conv: dx[N][T_in][V][I] (+)= dy[N][T_out][V][O] . W, Wt = W^T [I][O]
// bf16: Wt holds the bf16 copy (bf16 MFMA on the fp32 dy, rounded as it is staged)
int conv1x1_dgrad(int N, int T_in, int T_out, int V, int I, int O, int S, const float* dy, const float* Wt, float* dx,
                  bool add, hipStream_t s, bool bf16 = false) {
  ConvGemmArgs a;
  std::memset(&a, 0, sizeof(a));
  a.g.M = N * T_in * V; a.g.Nc = I; a.g.Kc = O; a.g.KT = 1; a.g.S = S; a.g.P = 0; a.g.transposed = 1;
  a.g.T_out = T_in; a.g.T_in = T_out; a.g.V = V; a.g.lda = O; a.g.ldo = I;
  a.in = dy; a.w = bf16 ? nullptr : Wt; a.out = dx;
  a.wb = bf16 ? reinterpret_cast<const unsigned short*>(Wt) : nullptr;
  if (S == 1) {  // plain row map
    a.g.transposed = 0;
    a.g.T_out = a.g.T_in = T_in;
  }
  return f3_conv_gemm(&a, 0, add ? EPI_ADD : 0, s);
}

int conv1x1_wgrad(int N, int T_in, int T_out, int V, int I, int lda, int O, int S, const float* dy, const float* in,
                  float* dW, float* db, hipStream_t s, bool bf16 = false) {
  WgradArgs w;
  std::memset(&w, 0, sizeof(w));
  w.g.M = N * T_out * V; w.g.Nc = O; w.g.Kc = I; w.g.KT = 1; w.g.S = S; w.g.P = 0; w.g.transposed = 0;
  w.g.T_out = T_out; w.g.T_in = T_in; w.g.V = V; w.g.lda = lda; w.g.ldo = O;
  w.dy = dy; w.ldy = O; w.in = in; w.dw = dW; w.db = db; w.outmap = WG_OUT_CONV;
  w.bf16 = bf16;  // operands rounded to bf16 as they are staged, bf16 MFMA, fp32 accumulate
  return f3_conv_wgrad(&w, 0, s);
}

struct Ctx {
  f3_musa* net;
  const Plan& p;
  void* ws;
  const float* params;
  float* buffers;
  float* grads;
  bool train;
  int N;
  hipStream_t s;
  double* fsum(const BnOff& b) const { return at<double>(ws, p.fsum) + (size_t)b.slot * 512; }
  double* bsum(const BnOff& b) const { return at<double>(ws, p.bsum) + (size_t)b.slot * 512; }
  BnRef bn(const BnOff& b, long long R) const {
    BnRef r;
    r.sum = fsum(b);
    r.sumsq = r.sum + 256;
    r.gamma = params + b.w;
    r.beta = params + b.b;
    r.rmean = buffers + b.rm;
    r.rvar = buffers + b.rv;
    r.count = (float)R;
    r.eval = train ? 0 : 1;
    return r;
  }
  float* f(size_t off) const { return at<float>(ws, off); }
  float* lanes() const { return at<float>(ws, p.lanes); }
  bool hb() const { return net->prec == F3_PRECISION_BF16; }
};

// slot `which` of stream si's 1x1-weight area (0 gcn, 1 res0, 2 pw1, 3 pw2, 4 p1, 5 p2, 6 sc, 7 res2):
// transposed fp32/bf16 copies for the input gradients (packT) or bf16 forward operands (packF)
float* pack_slot(const Ctx& c, size_t region, int si, int which) {
  static const int sz[7] = {C1 * E, C1 * E, C1 * C1, C1 * C1, CM * C1, C2 * CM, C2 * C1};
  float* base = at<float>(c.ws, region) + (size_t)si * kPackPerStream;
  for (int i = 0; i < which; ++i) base += sz[i];
  return base;
}

// the forward 1x1 conv's weight operand: bf16 copy in the bf16 mode
ConvGemmArgs with_wb(const Ctx& c, ConvGemmArgs a, int si, int which) {
  if (c.hb()) {
    a.wb = reinterpret_cast<const unsigned short*>(pack_slot(c, c.p.packF, si, which));
    a.w = nullptr;
  }
  return a;
}

int gemm_fwd(const Ctx& c, ConvGemmArgs a, const BnOff* stats) {
  int epi = EPI_BIAS;
  if (stats && c.train) {
    a.st_sum = c.fsum(*stats);
    a.st_sq = a.st_sum + 256;
    epi |= EPI_STATS;
  }
  return f3_conv_gemm(&a, 0, epi, c.s);
}

// DropBlock factors of one branch (z = BN(u) or u) into fS/fT
int drop_masks(const Ctx& c, const StreamWs& w, const float* u, const BnOff* bn, long long R, int T, int C,
               const float* Ae, int call, float* fS, float* fT) {
  AbsStatArgs as;
  std::memset(&as, 0, sizeof(as));
  as.R = R; as.C = C; as.u = u; as.bn_on = bn != nullptr;
  if (bn) as.bn = c.bn(*bn, R);
  as.a = c.f(c.p.a);
  MU_TRY(f3_mu_absstat(&as, c.s));
  DropMaskArgs dm;
  dm.N = c.N; dm.T = T; dm.V = c.net->V; dm.C = C; dm.a = as.a; dm.Ae = Ae;
  dm.seed = c.net->seed; dm.call = call; dm.keep_prob = kKeepProb; dm.block_size = kBlockSize;
  dm.fS = fS; dm.fT = fT;
  dm.scr = c.f(c.p.dmscr);
  (void)w;
  return f3_mu_dropmask(&dm, c.s);
}

MergeArgs merge_args(const Ctx& c, int T, int C, const float* u1, const BnOff& b1, const float* u2, const BnOff* b2,
                     const StreamWs& w, int k1, long long R) {
  MergeArgs m;
  std::memset(&m, 0, sizeof(m));
  m.N = c.N; m.T = T; m.V = c.net->V; m.C = C;
  m.u1 = u1; m.bn1 = c.bn(b1, R);
  m.u2 = u2; m.bn2_on = b2 != nullptr;
  if (b2) m.bn2 = c.bn(*b2, R);
  if (c.train && c.net->drop) {
    m.fS1 = c.f(w.fS[k1]); m.fT1 = c.f(w.fT[k1]);
    m.fS2 = c.f(w.fS[k1 + 1]); m.fT2 = c.f(w.fT[k1 + 1]);
  }
  return m;
}

int stream_forward(const Ctx& c, int si) {
  f3_musa* net = c.net;
  const StreamOff& o = net->st[si];
  const StreamWs& w = c.p.s[si];
  const int N = c.N, V = net->V, T = w.T, T2 = w.T2;
  const long long R = (long long)N * T * V, R2 = (long long)N * T2 * V;
  const float* P = c.params;
  // embedding: relu(W x + b)
  {
    ConvGemmArgs a = conv1x1(N, T, T, V, w.cin, E, 1, c.f(w.tok), P + o.emb_w, P + o.emb_b, c.f(w.e0));
    a.g.lda = 4;  // token rows are padded to 4 floats
    MU_TRY(gemm_fwd(c, a, nullptr));
  }
  ReluBwdArgs rl;
  rl.n = R * E; rl.y = c.f(w.e0); rl.d = c.f(w.e0); rl.out = c.f(w.e0);  // relu in place
  MU_TRY(f3_mu_relu_bwd(&rl, c.s));
  // --- SpatialGraphConv(64 -> 128), musa_model.py:127-146
  {
    ConvGemmArgs a = with_wb(c, conv1x1(N, T, T, V, E, C1, 1, c.f(w.e0), P + o.gcn_w, P + o.gcn_b, c.f(w.g)), si, 0);
    ConvGemmArgs ar =
        with_wb(c, conv1x1(N, T, T, V, E, C1, 1, c.f(w.e0), P + o.res0_w, P + o.res0_b, c.f(w.r0)), si, 1);
    MU_TRY(gemm_fwd(c, a, nullptr));
    MU_TRY(gemm_fwd(c, ar, &o.bn_r0));
    MixArgs mx;
    std::memset(&mx, 0, sizeof(mx));
    mx.K = 1; mx.V = V; mx.Cin = C1; mx.frames = N * T; mx.A = c.f(w.Ae[0]); mx.x = c.f(w.g); mx.z = c.f(w.h);
    MU_TRY(f3_mix_fwd(&mx, c.s));
    if (c.train) {
      ColStatArgs cs;
      cs.R = R; cs.C = C1; cs.x = c.f(w.h); cs.sum = c.fsum(o.bn_h); cs.sumsq = cs.sum + 256;
      cs.lanes = c.lanes();
      MU_TRY(f3_mu_colstat(&cs, c.s));
    }
    if (c.train && net->drop) {
      const int call = si * 6;
      MU_TRY(drop_masks(c, w, c.f(w.h), &o.bn_h, R, T, C1, c.f(w.Ae[0]), call, c.f(w.fS[0]), c.f(w.fT[0])));
      MU_TRY(drop_masks(c, w, c.f(w.r0), &o.bn_r0, R, T, C1, c.f(w.Ae[0]), call + 1, c.f(w.fS[1]), c.f(w.fT[1])));
    }
    MergeArgs m = merge_args(c, T, C1, c.f(w.h), o.bn_h, c.f(w.r0), &o.bn_r0, w, 0, R);
    m.out = c.f(w.out1);
    MU_TRY(f3_mu_merge_fwd(&m, c.s));
  }
  // --- SepTemporal_Block(128, k3, s1) and (128, k5, s2), musa_model.py:185-199
  for (int b = 0; b < 2; ++b) {
    const int K = b == 0 ? 3 : 5, S = b == 0 ? 1 : 2, Ti = T, To = b == 0 ? T : T2;
    const long long Ro = (long long)N * To * V;
    const float* x = c.f(b == 0 ? w.out1 : w.out2);
    float* d = c.f(b == 0 ? w.d1 : w.d2);
    float* e = c.f(b == 0 ? w.ee1 : w.ee2);
    float* pp = c.f(b == 0 ? w.p1 : w.p2);
    DwConvArgs dw;
    std::memset(&dw, 0, sizeof(dw));
    dw.N = N; dw.T_in = Ti; dw.T_out = To; dw.V = V; dw.C = C1; dw.K = K; dw.S = S; dw.P = (K - 1) / 2;
    dw.x = x; dw.w = P + o.dw_w[b]; dw.b = P + o.dw_b[b]; dw.y = d;
    if (c.train) {
      dw.sum = c.fsum(o.bn_d[b]);
      dw.sumsq = dw.sum + 256;
      dw.lanes = c.lanes();
    }
    MU_TRY(f3_mu_dwconv_fwd(&dw, c.s));
    BnActArgs ba;
    std::memset(&ba, 0, sizeof(ba));
    ba.R = Ro; ba.C = C1; ba.u = d; ba.bn = c.bn(o.bn_d[b], Ro); ba.act = ACT_TANH; ba.y = e;
    MU_TRY(f3_mu_bn_act(&ba, c.s));
    MU_TRY(gemm_fwd(c, with_wb(c, conv1x1(N, To, To, V, C1, C1, 1, e, P + o.pw_w[b], P + o.pw_b[b], pp), si, 2 + b),
                    &o.bn_p[b]));
    const float* res = x;
    const BnOff* rbn = nullptr;
    if (b == 1) {
      MU_TRY(gemm_fwd(c, with_wb(c, conv1x1(N, Ti, To, V, C1, C1, 2, x, P + o.res2_w, P + o.res2_b, c.f(w.r2)), si, 7),
                      &o.bn_r2));
      res = c.f(w.r2);
      rbn = &o.bn_r2;
    }
    const int k1 = 2 + 2 * b;
    if (c.train && net->drop) {
      const int call = si * 6 + k1;
      MU_TRY(drop_masks(c, w, pp, &o.bn_p[b], Ro, To, C1, c.f(w.Ae[1 + b]), call, c.f(w.fS[k1]), c.f(w.fT[k1])));
      MU_TRY(drop_masks(c, w, res, rbn, Ro, To, C1, c.f(w.Ae[1 + b]), call + 1, c.f(w.fS[k1 + 1]),
                        c.f(w.fT[k1 + 1])));
    }
    MergeArgs m = merge_args(c, To, C1, pp, o.bn_p[b], res, rbn, w, k1, Ro);
    m.out = c.f(b == 0 ? w.out2 : w.out3);
    MU_TRY(f3_mu_merge_fwd(&m, c.s));
  }
  // --- Sep_TCN(128 -> 256), musa_model.py:461-474
  {
    const float* x = c.f(w.out3);
    MU_TRY(gemm_fwd(c, with_wb(c, conv1x1(N, T2, T2, V, C1, C2, 1, x, P + o.sc_w, P + o.sc_b, c.f(w.tres)), si, 6),
                    nullptr));
    DwConvArgs dw;
    std::memset(&dw, 0, sizeof(dw));
    dw.N = N; dw.T_in = T2; dw.T_out = T2; dw.V = V; dw.C = C1; dw.K = 3; dw.S = 1; dw.P = 1;
    dw.x = x; dw.w = P + o.d1_w; dw.b = P + o.d1_b; dw.y = c.f(w.td1);
    if (c.train) { dw.sum = c.fsum(o.bn1); dw.sumsq = dw.sum + 256; dw.lanes = c.lanes(); }
    MU_TRY(f3_mu_dwconv_fwd(&dw, c.s));
    BnActArgs ba;
    std::memset(&ba, 0, sizeof(ba));
    ba.R = R2; ba.C = C1; ba.u = c.f(w.td1); ba.bn = c.bn(o.bn1, R2); ba.act = ACT_LEAKY; ba.y = c.f(w.te1);
    MU_TRY(f3_mu_bn_act(&ba, c.s));
    MU_TRY(gemm_fwd(c, with_wb(c, conv1x1(N, T2, T2, V, C1, CM, 1, c.f(w.te1), P + o.p1_w, P + o.p1_b, c.f(w.tp1)), si, 4),
                    &o.bn2));
    ba.C = CM; ba.u = c.f(w.tp1); ba.bn = c.bn(o.bn2, R2); ba.act = ACT_RELU; ba.y = c.f(w.te2);
    MU_TRY(f3_mu_bn_act(&ba, c.s));
    std::memset(&dw, 0, sizeof(dw));
    dw.N = N; dw.T_in = T2; dw.T_out = T2; dw.V = V; dw.C = CM; dw.K = 1; dw.S = 1; dw.P = 0;
    dw.x = c.f(w.te2); dw.w = P + o.d2_w; dw.b = P + o.d2_b; dw.y = c.f(w.td2);
    if (c.train) { dw.sum = c.fsum(o.bn3); dw.sumsq = dw.sum + 256; dw.lanes = c.lanes(); }
    MU_TRY(f3_mu_dwconv_fwd(&dw, c.s));
    ba.C = CM; ba.u = c.f(w.td2); ba.bn = c.bn(o.bn3, R2); ba.act = ACT_LEAKY; ba.y = c.f(w.te3);
    MU_TRY(f3_mu_bn_act(&ba, c.s));
    MU_TRY(gemm_fwd(c, with_wb(c, conv1x1(N, T2, T2, V, CM, C2, 1, c.f(w.te3), P + o.p2_w, P + o.p2_b, c.f(w.tp2)), si, 5),
                    &o.bn4));
    ba.C = C2; ba.u = c.f(w.tp2); ba.bn = c.bn(o.bn4, R2); ba.act = ACT_RELU; ba.y = c.f(w.out4);
    ba.add = c.f(w.tres);
    MU_TRY(f3_mu_bn_act(&ba, c.s));
  }
  return F3_OK;
}

int bn_act_bwd(const Ctx& c, const BnOff& b, long long R, int C, const float* dy, const float* u, int act, float* du,
               const float* add) {
  BnActBwdArgs a;
  std::memset(&a, 0, sizeof(a));
  a.R = R; a.C = C; a.dy = dy; a.u = u; a.bn = c.bn(b, R); a.act = act;
  a.s_dz = c.bsum(b); a.s_dzx = a.s_dz + 256;
  a.lanes = c.lanes();
  a.du = du; a.add = add;
  a.g_gamma = c.grads + b.w; a.g_beta = c.grads + b.b;
  return f3_mu_bn_act_bwd(&a, c.s);
}

int dwconv_bwd(const Ctx& c, int N, int Ti, int To, int V, int C, int K, int S, const float* x, const float* dy,
               float* dx, bool add, int64_t w_off, int64_t b_off) {
  DwConvArgs dw;
  std::memset(&dw, 0, sizeof(dw));
  dw.N = N; dw.T_in = Ti; dw.T_out = To; dw.V = V; dw.C = C; dw.K = K; dw.S = S; dw.P = (K - 1) / 2;
  dw.x = x; dw.w = c.params + w_off; dw.dy = dy; dw.dx = dx; dw.dx_add = add;
  dw.part = c.f(c.p.part);
  MU_TRY(f3_mu_dwconv_bwd(&dw, c.s));
  MU_TRY(f3_colsum(dw.part, dw.part_rows, C * K, c.grads + w_off, c.s));
  return f3_colsum(dw.part + (size_t)dw.part_rows * C * K, dw.part_rows, C, c.grads + b_off, c.s);
}

// transposed copies [I][O] of the stream's 1x1 weights [O][I] (bf16 in the bf16 mode)
float* packT(const Ctx& c, int si, int which) { return pack_slot(c, c.p.packT, si, which); }

int stream_backward(const Ctx& c, int si, float* dres2T) {
  f3_musa* net = c.net;
  const StreamOff& o = net->st[si];
  const StreamWs& w = c.p.s[si];
  const int N = c.N, V = net->V, T = w.T, T2 = w.T2;
  const long long R = (long long)N * T * V, R2 = (long long)N * T2 * V;
  float* ga = c.f(c.p.ga);
  float* gb = c.f(c.p.gb);
  float* gc = c.f(c.p.gc);
  float* gd = c.f(c.p.gd);
  float* G = c.grads;
  const float* dy4 = c.f(w.dy4);
  // --- Sep_TCN
  MU_TRY(conv1x1_wgrad(N, T2, T2, V, C1, C1, C2, 1, dy4, c.f(w.out3), G + o.sc_w, G + o.sc_b, c.s, c.hb()));
  MU_TRY(conv1x1_dgrad(N, T2, T2, V, C1, C2, 1, dy4, packT(c, si, 6), gd, false, c.s, c.hb()));   // gd = d out3
  MU_TRY(bn_act_bwd(c, o.bn4, R2, C2, dy4, c.f(w.tp2), ACT_RELU, ga, nullptr));           // ga = d p2
  MU_TRY(conv1x1_wgrad(N, T2, T2, V, CM, CM, C2, 1, ga, c.f(w.te3), G + o.p2_w, G + o.p2_b, c.s, c.hb()));
  MU_TRY(conv1x1_dgrad(N, T2, T2, V, CM, C2, 1, ga, packT(c, si, 5), gb, false, c.s, c.hb()));    // gb = d e3
  MU_TRY(bn_act_bwd(c, o.bn3, R2, CM, gb, c.f(w.td2), ACT_LEAKY, ga, nullptr));           // ga = d d2
  MU_TRY(dwconv_bwd(c, N, T2, T2, V, CM, 1, 1, c.f(w.te2), ga, gb, false, o.d2_w, o.d2_b));  // gb = d e2
  MU_TRY(bn_act_bwd(c, o.bn2, R2, CM, gb, c.f(w.tp1), ACT_RELU, ga, nullptr));            // ga = d p1
  MU_TRY(conv1x1_wgrad(N, T2, T2, V, C1, C1, CM, 1, ga, c.f(w.te1), G + o.p1_w, G + o.p1_b, c.s, c.hb()));
  MU_TRY(conv1x1_dgrad(N, T2, T2, V, C1, CM, 1, ga, packT(c, si, 4), gb, false, c.s, c.hb()));    // gb = d e1
  MU_TRY(bn_act_bwd(c, o.bn1, R2, C1, gb, c.f(w.td1), ACT_LEAKY, ga, nullptr));           // ga = d d1
  MU_TRY(dwconv_bwd(c, N, T2, T2, V, C1, 3, 1, c.f(w.out3), ga, gd, true, o.d1_w, o.d1_b));  // gd += ...
  // --- SepTemporal blocks (2 then 1); gd holds d out3, then d out2
  for (int b = 1; b >= 0; --b) {
    const int K = b == 0 ? 3 : 5, S = b == 0 ? 1 : 2, Ti = T, To = b == 0 ? T : T2;
    const long long Ro = (long long)N * To * V;
    const float* x = c.f(b == 0 ? w.out1 : w.out2);
    const BnOff* rbn = b == 1 ? &o.bn_r2 : nullptr;
    const float* res = b == 1 ? c.f(w.r2) : x;
    const int k1 = 2 + 2 * b;
    MergeArgs m = merge_args(c, To, C1, c.f(b == 0 ? w.p1 : w.p2), o.bn_p[b], res, rbn, w, k1, Ro);
    m.dout = gd;
    m.lanes = c.lanes();
    m.s1_dz = c.bsum(o.bn_p[b]); m.s1_dzx = m.s1_dz + 256;
    if (rbn) { m.s2_dz = c.bsum(*rbn); m.s2_dzx = m.s2_dz + 256; }
    m.du1 = ga;                              // d p
    m.du2 = b == 1 ? gb : gc;                // d r2 (block 2) or d out1 via the identity (block 1)
    m.du2_add = 0;
    m.g_gamma1 = G + o.bn_p[b].w; m.g_beta1 = G + o.bn_p[b].b;
    if (rbn) { m.g_gamma2 = G + rbn->w; m.g_beta2 = G + rbn->b; }
    MU_TRY(f3_mu_merge_bwd(&m, c.s));
    float* dxin = gc;                        // d x of the block (x = out2 / out1) accumulates in gc
    if (b == 1) {  // strided residual: wgrad and dx = dr . W (transposed row map)
      MU_TRY(conv1x1_wgrad(N, Ti, To, V, C1, C1, C1, 2, gb, x, G + o.res2_w, G + o.res2_b, c.s, c.hb()));
      MU_TRY(conv1x1_dgrad(N, Ti, To, V, C1, C1, 2, gb, dres2T, gc, false, c.s, c.hb()));
    }
    MU_TRY(conv1x1_wgrad(N, To, To, V, C1, C1, C1, 1, ga, c.f(b == 0 ? w.ee1 : w.ee2), G + o.pw_w[b], G + o.pw_b[b],
                         c.s, c.hb()));
    MU_TRY(conv1x1_dgrad(N, To, To, V, C1, C1, 1, ga, packT(c, si, 2 + b), gb, false, c.s, c.hb()));   // gb = d e
    MU_TRY(bn_act_bwd(c, o.bn_d[b], Ro, C1, gb, c.f(b == 0 ? w.d1 : w.d2), ACT_TANH, ga, nullptr));  // ga = d d
    MU_TRY(dwconv_bwd(c, N, Ti, To, V, C1, K, S, x, ga, dxin, true, o.dw_w[b], o.dw_b[b]));
    std::swap(gc, gd);  // the block input's gradient becomes the next (earlier) block's output gradient
  }
  // --- SpatialGraphConv: gd = d out1
  {
    MergeArgs m = merge_args(c, T, C1, c.f(w.h), o.bn_h, c.f(w.r0), &o.bn_r0, w, 0, R);
    m.dout = gd;
    m.lanes = c.lanes();
    m.s1_dz = c.bsum(o.bn_h); m.s1_dzx = m.s1_dz + 256;
    m.s2_dz = c.bsum(o.bn_r0); m.s2_dzx = m.s2_dz + 256;
    m.du1 = ga; m.du2 = gb; m.du2_add = 0;
    m.g_gamma1 = G + o.bn_h.w; m.g_beta1 = G + o.bn_h.b; m.g_gamma2 = G + o.bn_r0.w; m.g_beta2 = G + o.bn_r0.b;
    MU_TRY(f3_mu_merge_bwd(&m, c.s));
    // graph mix backward: d g (gc) and d Ae
    float* dAe = c.f(c.p.a);  // scratch [V*V]
    if (hipMemsetAsync(dAe, 0, sizeof(float) * V * V, c.s) != hipSuccess) return F3_EHIP;
    MixArgs mx;
    std::memset(&mx, 0, sizeof(mx));
    mx.K = 1; mx.V = V; mx.Cin = C1; mx.frames = N * T; mx.A = c.f(w.Ae[0]); mx.x = c.f(w.g); mx.z = ga;
    mx.dx = gc; mx.dA = dAe; mx.accumulate = 0; mx.part = c.f(c.p.mixpart);
    MU_TRY(f3_mix_bwd(&mx, c.s));
    PrepTable t;  // d edge = d Ae * A
    t.n = 0;
    PrepJob& j = t.jobs[t.n++];
    std::memset(&j, 0, sizeof(j));
    j.type = PREP_MUL; j.n = V * V; j.dst = G + o.e0; j.s0 = dAe; j.s1 = c.params + o.A0;
    MU_TRY(f3_prep(t, c.s));
    MU_TRY(conv1x1_wgrad(N, T, T, V, E, E, C1, 1, gc, c.f(w.e0), G + o.gcn_w, G + o.gcn_b, c.s, c.hb()));
    MU_TRY(conv1x1_wgrad(N, T, T, V, E, E, C1, 1, gb, c.f(w.e0), G + o.res0_w, G + o.res0_b, c.s, c.hb()));
    MU_TRY(conv1x1_dgrad(N, T, T, V, E, C1, 1, gc, packT(c, si, 0), gd, false, c.s, c.hb()));
    MU_TRY(conv1x1_dgrad(N, T, T, V, E, C1, 1, gb, packT(c, si, 1), gd, true, c.s, c.hb()));   // gd = d e0
  }
  // --- embedding: relu backward, weight gradient on the token rows
  ReluBwdArgs rl;
  rl.n = R * E; rl.y = c.f(w.e0); rl.d = gd; rl.out = ga;
  MU_TRY(f3_mu_relu_bwd(&rl, c.s));
  return conv1x1_wgrad(N, T, T, V, w.cin, 4, E, 1, ga, c.f(w.tok), G + o.emb_w, G + o.emb_b, c.s);
}

}  // namespace

extern "C" {

int f3_musa_create(const f3_musa_config* cfg, f3_musa** out) {
  if (!cfg || !out) return F3_EINVAL;
  *out = nullptr;
  if (cfg->num_point < 13 || cfg->num_point > 18 || cfg->frames < 8 || cfg->frames > 64 || cfg->num_class < 1 ||
      cfg->num_class > 64)
    return F3_EINVAL;
  f3_musa* n = new f3_musa();
  n->V = cfg->num_point; n->T = cfg->frames; n->C = cfg->num_class;
  if (cfg->precision != F3_PRECISION_FP32 && cfg->precision != F3_PRECISION_BF16) { delete n; return F3_EINVAL; }
  n->prec = cfg->precision;
  const int V = n->V;
  n->bns.reserve(22);
  StreamOff* so[2] = {&n->st[0], &n->st[1]};
  so[0]->emb_w = n->add("joint_embed_pos.cnn.0.cnn.weight", {E, 3, 1, 1});
  so[0]->emb_b = n->add("joint_embed_pos.cnn.0.cnn.bias", {E});
  so[1]->emb_w = n->add("joint_embed_mos.cnn.0.cnn.weight", {E, 2, 1, 1});
  so[1]->emb_b = n->add("joint_embed_mos.cnn.0.cnn.bias", {E});
  for (int si = 0; si < 2; ++si) {
    StreamOff& o = *so[si];
    const std::string s = si == 0 ? "stream_pos." : "stream_mot.";
    std::string p = s + "0.";
    o.A0 = n->add(p + "A", {1, V, V});
    o.e0 = n->add(p + "edge", {1, V, V});
    o.gcn_w = n->add(p + "gcn.weight", {C1, E, 1, 1});
    o.gcn_b = n->add(p + "gcn.bias", {C1});
    n->add_bn(o.bn_h, p + "bn.", C1);
    o.res0_w = n->add(p + "residual.0.weight", {C1, E, 1, 1});
    o.res0_b = n->add(p + "residual.0.bias", {C1});
    n->add_bn(o.bn_r0, p + "residual.1.", C1);
    for (int b = 0; b < 2; ++b) {
      const int K = b == 0 ? 3 : 5;
      p = s + std::to_string(b + 1) + ".";
      o.A[b] = n->add(p + "A", {1, V, V});
      o.edge[b] = n->add(p + "edge", {1, V, V});
      o.dw_w[b] = n->add(p + "depth_conv.0.weight", {C1, 1, K, 1});
      o.dw_b[b] = n->add(p + "depth_conv.0.bias", {C1});
      n->add_bn(o.bn_d[b], p + "depth_conv.1.", C1);
      o.pw_w[b] = n->add(p + "point_conv.0.weight", {C1, C1, 1, 1});
      o.pw_b[b] = n->add(p + "point_conv.0.bias", {C1});
      n->add_bn(o.bn_p[b], p + "point_conv.1.", C1);
      if (b == 1) {
        o.res2_w = n->add(p + "residual.0.weight", {C1, C1, 1, 1});
        o.res2_b = n->add(p + "residual.0.bias", {C1});
        n->add_bn(o.bn_r2, p + "residual.1.", C1);
      }
    }
    p = s + "3.";
    o.d1_w = n->add(p + "sep31.seq.0.weight", {C1, 1, 3, 1});
    o.d1_b = n->add(p + "sep31.seq.0.bias", {C1});
    n->add_bn(o.bn1, p + "sep31.seq.1.", C1);
    o.p1_w = n->add(p + "sep31.seq.3.weight", {CM, C1, 1, 1});
    o.p1_b = n->add(p + "sep31.seq.3.bias", {CM});
    n->add_bn(o.bn2, p + "sep31.seq.4.", CM);
    o.d2_w = n->add(p + "sep11.seq.0.weight", {CM, 1, 1, 1});
    o.d2_b = n->add(p + "sep11.seq.0.bias", {CM});
    n->add_bn(o.bn3, p + "sep11.seq.1.", CM);
    o.p2_w = n->add(p + "sep11.seq.3.weight", {C2, CM, 1, 1});
    o.p2_b = n->add(p + "sep11.seq.3.bias", {C2});
    n->add_bn(o.bn4, p + "sep11.seq.4.", C2);
    o.sc_w = n->add(p + "shortcut.weight", {C2, C1, 1, 1});
    o.sc_b = n->add(p + "shortcut.bias", {C2});
  }
  n->fc0_w = n->add("fc.seq.0.weight", {HIDDEN, 2 * C2 + 3});
  n->fc0_b = n->add("fc.seq.0.bias", {HIDDEN});
  n->ln_w = n->add("fc.seq.2.weight", {HIDDEN});
  n->ln_b = n->add("fc.seq.2.bias", {HIDDEN});
  n->fc5_w = n->add("fc.seq.5.weight", {n->C, HIDDEN});
  n->fc5_b = n->add("fc.seq.5.bias", {n->C});
  *out = n;
  return F3_OK;
}

void f3_musa_destroy(f3_musa* net) { delete net; }
int f3_musa_num_entries(const f3_musa* net) { return net ? (int)net->entries.size() : 0; }

int f3_musa_entry(const f3_musa* net, int i, const char** name, int* kind, int* ndim, int64_t* shape8,
                  int64_t* offset) {
  if (!net || i < 0 || i >= (int)net->entries.size()) return F3_EINVAL;
  const Entry& e = net->entries[i];
  *name = e.name.c_str();
  *kind = e.kind;
  *ndim = (int)e.shape.size();
  for (int d = 0; d < 8; ++d) shape8[d] = d < (int)e.shape.size() ? e.shape[d] : 0;
  *offset = e.off;
  return F3_OK;
}

int64_t f3_musa_param_count(const f3_musa* net) { return net ? net->nparam : 0; }
int64_t f3_musa_buffer_count(const f3_musa* net) { return net ? net->nbuf : 0; }
int64_t f3_musa_counter_count(const f3_musa* net) { return net ? net->ncnt : 0; }
int64_t f3_musa_workspace_bytes(const f3_musa* net, int batch) {
  if (!net || batch < 1) return 0;
  return (int64_t)plan(net, batch).total;
}

int f3_musa_forward(f3_musa* net, int N, int training, const float* params, float* buffers, int64_t* counters,
                    const float* x, float* out, void* workspace, unsigned seed, int dropout, void* stream) {
  if (!net || N < 1 || !params || !buffers || !x || !out || !workspace) return F3_EINVAL;
  if (training && (N < 2 || !counters)) return training && N < 2 ? F3_EBATCH : F3_EINVAL;
  hipStream_t s = (hipStream_t)stream;
  const Plan p = plan(net, N);
  net->trained_batch = training ? N : 0;
  net->seed = seed;
  net->drop = training && dropout;
  Ctx c{net, p, workspace, params, buffers, nullptr, training != 0, N, s};
  if (training && hipMemsetAsync(at<char>(workspace, p.fsum), 0, 8 * 22 * 512, s) != hipSuccess) return F3_EHIP;
  if (training && hipMemsetAsync(at<char>(workspace, p.lanes), 0, 4 * 2 * kLaneFloats, s) != hipSuccess) return F3_EHIP;
  TokenArgs tk;
  std::memset(&tk, 0, sizeof(tk));
  tk.N = N; tk.T = net->T; tk.V = net->V; tk.x = x; tk.pos = c.f(p.s[0].tok); tk.mot = c.f(p.s[1].tok);
  MU_TRY(f3_mu_tokens(&tk, s));
  {  // A * edge of every graph-using block
    PrepTable t;
    t.n = 0;
    for (int si = 0; si < 2; ++si) {
      const StreamOff& o = net->st[si];
      const int64_t As[3] = {o.A0, o.A[0], o.A[1]}, Es[3] = {o.e0, o.edge[0], o.edge[1]};
      for (int k = 0; k < 3; ++k) {
        PrepJob& j = t.jobs[t.n++];
        std::memset(&j, 0, sizeof(j));
        j.type = PREP_MUL; j.n = net->V * net->V; j.dst = c.f(p.s[si].Ae[k]); j.s0 = params + As[k];
        j.s1 = params + Es[k];
      }
    }
    MU_TRY(f3_prep(t, s));
  }
  if (c.hb()) {  // bf16 mode: the stream 1x1 weights as bf16 GEMM operands ([O][I])
    PrepTable t;
    t.n = 0;
    auto job = [&](float* dst, const float* src, int O, int I) {
      PrepJob& j = t.jobs[t.n++];
      std::memset(&j, 0, sizeof(j));
      j.type = PREP_PACK_CONV; j.n = O * I; j.dst = dst; j.s0 = src; j.d0 = O; j.d1 = I; j.d2 = 1; j.bf16 = 1;
    };
    for (int si = 0; si < 2; ++si) {
      const StreamOff& o = net->st[si];
      const int64_t ws8[8] = {o.gcn_w, o.res0_w, o.pw_w[0], o.pw_w[1], o.p1_w, o.p2_w, o.sc_w, o.res2_w};
      const int O8[8] = {C1, C1, C1, C1, CM, C2, C2, C1}, I8[8] = {E, E, C1, C1, C1, CM, C1, C1};
      for (int k = 0; k < 8; ++k) job(pack_slot(c, p.packF, si, k), params + ws8[k], O8[k], I8[k]);
    }
    MU_TRY(f3_prep(t, s));
  }
  for (int si = 0; si < 2; ++si) MU_TRY(stream_forward(c, si));
  if (training) {
    BnRunTable t;
    t.n = 0;
    for (BnOff* b : net->bns) {
      // each BN's sums were taken over its own rows: the stream / stage decides the count
      BnRunJob& j = t.jobs[t.n++];
      j.sum = c.fsum(*b);
      j.sumsq = j.sum + 256;
      j.C = b->C;
      j.rmean = buffers + b->rm;
      j.rvar = buffers + b->rv;
      j.nbt = reinterpret_cast<long long*>(counters + b->nbt);
      j.count = 0;  // set below
    }
    // row counts per BN slot: stream-major order of add_bn (see f3_musa_create)
    int k = 0;
    for (int si = 0; si < 2; ++si) {
      const StreamWs& w = p.s[si];
      const double R = (double)N * w.T * net->V, R2 = (double)N * w.T2 * net->V;
      const double counts[11] = {R, R, R, R, R2, R2, R2, R2, R2, R2, R2};  // bn_h, r0, d1, p1, d2, p2, r2, tcn 1-4
      for (int q = 0; q < 11; ++q) t.jobs[k++].count = counts[q];
    }
    MU_TRY(f3_bn_running(t, s));
  }
  mu::HeadArgs h;
  std::memset(&h, 0, sizeof(h));
  h.N = N; h.Cs = C2; h.TV1 = p.s[0].T2 * net->V; h.TV2 = p.s[1].T2 * net->V; h.NC = net->C;
  h.y1 = c.f(p.s[0].out4); h.y2 = c.f(p.s[1].out4); h.x = x; h.TVx = net->T * net->V;
  h.w1 = params + net->fc0_w; h.b1 = params + net->fc0_b; h.lnw = params + net->ln_w; h.lnb = params + net->ln_b;
  h.w2 = params + net->fc5_w; h.b2 = params + net->fc5_b;
  h.seed = seed; h.drop_p = net->drop ? kHeadDrop : 0.f;
  h.feat = c.f(p.feat); h.z1 = c.f(p.z1); h.stat = c.f(p.stat); h.h = c.f(p.h); h.out = out;
  return f3_mu_head_fwd(&h, s);
}

int f3_musa_backward(f3_musa* net, int N, const float* params, const float* buffers, const float* dout, float* grads,
                     void* workspace, void* stream) {
  if (!net || N < 1 || !params || !buffers || !dout || !grads || !workspace) return F3_EINVAL;
  if (net->trained_batch != N) return F3_ESTATE;
  hipStream_t s = (hipStream_t)stream;
  const Plan p = plan(net, N);
  Ctx c{net, p, workspace, params, const_cast<float*>(buffers), grads, true, N, s};
  if (hipMemsetAsync(grads, 0, sizeof(float) * net->nparam, s) != hipSuccess) return F3_EHIP;
  if (hipMemsetAsync(at<char>(workspace, p.bsum), 0, 8 * 22 * 512, s) != hipSuccess) return F3_EHIP;
  if (hipMemsetAsync(at<char>(workspace, p.lanes), 0, 4 * 2 * kLaneFloats, s) != hipSuccess) return F3_EHIP;
  float* dres2T[2];
  {  // transposed 1x1 weights ([I][O] from [O][I]) for the input-gradient GEMMs
    PrepTable t;
    t.n = 0;
    auto job = [&](float* dst, const float* src, int O, int I) {
      PrepJob& j = t.jobs[t.n++];
      std::memset(&j, 0, sizeof(j));
      j.type = PREP_PACK_CONV_T; j.n = O * I; j.dst = dst; j.s0 = src; j.d0 = O; j.d1 = I; j.d2 = 1;
      j.bf16 = c.hb();
    };
    for (int si = 0; si < 2; ++si) {
      const StreamOff& o = net->st[si];
      job(packT(c, si, 0), params + o.gcn_w, C1, E);
      job(packT(c, si, 1), params + o.res0_w, C1, E);
      job(packT(c, si, 2), params + o.pw_w[0], C1, C1);
      job(packT(c, si, 3), params + o.pw_w[1], C1, C1);
      job(packT(c, si, 4), params + o.p1_w, CM, C1);
      job(packT(c, si, 5), params + o.p2_w, C2, CM);
      job(packT(c, si, 6), params + o.sc_w, C2, C1);
      dres2T[si] = packT(c, si, 7);
      job(dres2T[si], params + o.res2_w, C1, C1);
    }
    MU_TRY(f3_prep(t, s));
  }
  mu::HeadArgs h;
  std::memset(&h, 0, sizeof(h));
  h.N = N; h.Cs = C2; h.TV1 = p.s[0].T2 * net->V; h.TV2 = p.s[1].T2 * net->V; h.NC = net->C;
  h.w1 = params + net->fc0_w; h.lnw = params + net->ln_w; h.lnb = params + net->ln_b; h.w2 = params + net->fc5_w;
  h.seed = net->seed; h.drop_p = net->drop ? kHeadDrop : 0.f;
  h.z1 = c.f(p.z1); h.stat = c.f(p.stat);
  h.dout = dout; h.dz1 = c.f(p.dz1); h.dy1 = c.f(p.s[0].dy4); h.dy2 = c.f(p.s[1].dy4);
  h.g_lnw = grads + net->ln_w; h.g_lnb = grads + net->ln_b;
  MU_TRY(f3_mu_head_bwd(&h, s));
  const int F = 2 * C2 + 3;
  MU_TRY(conv1x1_wgrad(N, 1, 1, 1, F, F, HIDDEN, 1, c.f(p.dz1), c.f(p.feat), grads + net->fc0_w, grads + net->fc0_b, s));
  MU_TRY(conv1x1_wgrad(N, 1, 1, 1, HIDDEN, HIDDEN, net->C, 1, dout, c.f(p.h), grads + net->fc5_w, grads + net->fc5_b,
                       s));
  for (int si = 0; si < 2; ++si) MU_TRY(stream_backward(c, si, dres2T[si]));
  return F3_OK;
}

int f3_musa_guards(const f3_musa* net, int batch, int64_t* offsets, int max) {
  if (!net || batch < 1) return -1;
  std::vector<size_t> g;
  (void)plan(net, batch, &g);
  for (int i = 0; i < (int)g.size() && i < max; ++i) offsets[i] = (int64_t)g[i];
  return (int)g.size();
}

int f3_dwconv_t_forward(const float* x, const float* w, const float* b, float* y, double* sums, int N, int T_in,
                        int V, int C, int K, int S, int P, void* stream) {
  if (!x || !w || !b || !y || N < 1 || T_in < 1 || V < 1 || S < 1 || P < 0) return F3_EINVAL;
  DwConvArgs a;
  std::memset(&a, 0, sizeof(a));
  a.N = N; a.T_in = T_in; a.T_out = (T_in + 2 * P - K) / S + 1; a.V = V; a.C = C; a.K = K; a.S = S; a.P = P;
  if (a.T_out < 1) return F3_EINVAL;
  a.x = x; a.w = w; a.b = b; a.y = y;
  if (sums) {
    static float* lanes = nullptr;  // test / bench entry only: lane scratch kept for the process lifetime
    if (!lanes) {
      if (hipMalloc(&lanes, sizeof(float) * kLaneFloats) != hipSuccess) return F3_EHIP;
      if (hipMemset(lanes, 0, sizeof(float) * kLaneFloats) != hipSuccess) return F3_EHIP;
    }
    a.sum = sums; a.sumsq = sums + C; a.lanes = lanes;
  }
  return f3_mu_dwconv_fwd(&a, (hipStream_t)stream);
}

}  // extern "C"
