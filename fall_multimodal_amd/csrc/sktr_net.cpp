// SkeletonTransformer training step (BASELINE config 5) behind the C ABI (include/fall3.h f3_sktr_*).
//
// Replaces, for GSTCAN_HAR_conv_kfold_trans.ipynb / skeleton_transformer.py:
//   model = SkeletonTransformer(3, 14, 30, 11, 32, 6, 16, 8)  -> f3_sktr_create   (:360-416)
//   out = model(x)                                            -> f3_sktr_forward  (:418-435)
//   loss.backward()                                           -> f3_sktr_backward
//
// Per block (B2TSpatialTenporalTransformerBlock, :229-248), forward:
//   qkv GEMM -> spatial attention core -> merge GEMM -> u1 = y0 + sd*m, BN1 sums -> y1
//   qkv GEMM -> temporal attention core -> merge GEMM -> u2 = y1 + sd*m, BN2 sums -> y2
//   FFN1 GEMM -> GELU -> FFN2 GEMM -> u3 = y0 + y2 + sd*drop(f), BN3 sums -> y3 (next block's y0)
// The Linear layers are the shared fp32 MFMA GEMM over token rows (1x1 geometry); weight
// gradients the shared split-K wgrad GEMM (fp32 atomics into the flat gradient buffer).
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstring>
#include <string>
#include <vector>

#include "fall3.h"
#include "kernels.h"
#include "layers.h"
#include "sktr.h"

using namespace f3;
using namespace f3::sk;

namespace {

struct Entry {
  std::string name;
  int kind;
  std::vector<int64_t> shape;
  int64_t off;
};

struct AttnOff {
  int64_t table, wqkv, bqkv, wm, bm;
};
struct BnOff {
  int64_t w, b, rm, rv, nbt;
};
struct BlockOff {
  AttnOff at[2];   // spatial, temporal
  BnOff bn[3];
  int64_t w1, b1, w2, b2;
};

constexpr int NBLOCK = 6;

}  // namespace

struct f3_sktr {
  int V, T, M, C;
  int prec = F3_PRECISION_FP32;  // F3_PRECISION_BF16: the block Linears on bf16 MFMA (fp32 accumulate)
  std::vector<Entry> entries;
  int64_t nparam = 0, nbuf = 0, ncnt = 0;
  int64_t e_w1 = 0, e_b1 = 0, e_w2 = 0, e_b2 = 0, fc_w = 0, fc_b = 0;
  BlockOff blk[NBLOCK];
  // the last training forward's randomness (backward replays it)
  float sd[NBLOCK][3];
  unsigned seed = 0;
  float drop_p = 0.f;
  int trained_batch = 0;

  int64_t add(const std::string& name, std::vector<int64_t> shape, int kind = F3_ENTRY_PARAM) {
    int64_t n = 1;
    for (auto d : shape) n *= d;
    Entry e{name, kind, shape, 0};
    if (kind == F3_ENTRY_PARAM) {
      e.off = nparam;
      nparam += (n + 3) / 4 * 4;  // 16-B aligned entries (float4 RMSprop)
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
};

namespace {

struct BlockWs {
  size_t qkv[2], o[2], u[3], y1, y2, yout, h, g;
};

struct Plan {
  size_t xt, a1, h1, a2, y0;
  BlockWs b[NBLOCK];
  size_t mtmp, pooled;
  size_t fsum;      // [18 BN][2][32] doubles, forward batch sums
  size_t bsum;      // [18 BN][2][32] doubles, backward sums
  size_t packT;     // transposed weights for the input-gradient GEMMs, per block 6 matrices
  size_t packF;     // bf16 mode: the forward weights as bf16 GEMM operands, same slots
  size_t du3, dy2, dy1, dm, dbig, dqkv, dya, dyb, da1, da2, dtab;
  size_t total;
};

constexpr int kPackPerBlock = 2 * (QKV * EMB + DM * EMB) + 2 * FFN * EMB;

Plan plan(const f3_sktr* net, int N) {
  Plan p;
  size_t o = 0;
  auto take = [&](size_t bytes) {
    const size_t at = o;
    o += (bytes + 255) / 256 * 256;
    return at;
  };
  const size_t R = (size_t)N * net->M * net->T * net->V;
  const size_t r32 = 4 * R * EMB, r128 = 4 * R * DM, r384 = 4 * R * QKV;
  p.xt = take(4 * R * 4);
  p.a1 = take(4 * R * HID0);
  p.h1 = take(4 * R * HID0);
  p.a2 = take(r32);
  p.y0 = take(r32);
  for (int b = 0; b < NBLOCK; ++b) {
    BlockWs& w = p.b[b];
    for (int k = 0; k < 2; ++k) {
      w.qkv[k] = take(r384);
      w.o[k] = take(r128);
    }
    for (int k = 0; k < 3; ++k) w.u[k] = take(r32);
    w.y1 = take(r32);
    w.y2 = take(r32);
    w.yout = take(r32);
    w.h = take(r128);
    w.g = take(r128);
  }
  p.mtmp = take(r32);
  p.pooled = take(4 * (size_t)N * EMB);
  p.fsum = take(8 * 18 * 64);
  p.bsum = take(8 * 18 * 64);
  p.packT = take(4 * (size_t)NBLOCK * kPackPerBlock);
  p.packF = net->prec == F3_PRECISION_BF16 ? take(4 * (size_t)NBLOCK * kPackPerBlock) : 0;
  p.du3 = take(r32);
  p.dy2 = take(r32);
  p.dy1 = take(r32);
  p.dm = take(r32);
  p.dbig = take(r128);
  p.dqkv = take(r384);
  p.dya = take(r32);
  p.dyb = take(r32);
  p.da1 = take(4 * R * HID0);
  p.da2 = take(r32);
  const size_t nseq = std::max((size_t)N * net->M * net->T * (2 * net->V - 1),
                               (size_t)N * net->M * net->V * (2 * net->T - 1));
  p.dtab = take(4 * nseq * HD);
  p.total = o;
  return p;
}

template <typename P>
P* at(void* ws, size_t off) {
  return reinterpret_cast<P*>(reinterpret_cast<char*>(ws) + off);
}

#define SK_TRY(x)                 \
  do {                            \
    const int _st = (x);          \
    if (_st != F3_OK) return _st; \
  } while (0)

// token-row Linear: out[R][O] = in[R][I] . W^T (+ bias) ; W packed [O][I] (nn.Linear layout)
// wb (bf16 mode): the same weight as a bf16 operand; fp32 activations are rounded to bf16 as
// they are staged (conv_gemm_bf16), accumulation and outputs stay fp32
int linear(const float* in, int I, const float* W, const float* bias, float* out, int O, long long R, int epi,
           hipStream_t s, const void* wb = nullptr) {
  ConvGemmArgs a;
  std::memset(&a, 0, sizeof(a));
  a.g.M = (int)R; a.g.Nc = O; a.g.Kc = I; a.g.KT = 1; a.g.S = 1; a.g.P = 0; a.g.transposed = 0;
  a.g.T_out = 1; a.g.T_in = 1; a.g.V = 1; a.g.lda = I; a.g.ldo = O;
  a.in = in; a.w = W; a.out = out; a.bias = bias;
  a.wb = reinterpret_cast<const unsigned short*>(wb);
  return f3_conv_gemm(&a, 0, epi, s);
}

// weight gradient of a token-row Linear: dW[O][I] += dy[R][O]^T in[R][I] ; db[O] += sum dy
// bf16 != 0: operands rounded to bf16 as they are staged, bf16 MFMA, fp32 accumulate (conv_wgrad_bf16)
int linear_wgrad(const float* dy, int O, const float* in, int I, int lda, float* dW, float* db, long long R,
                 hipStream_t s, int bf16 = 0) {
  WgradArgs w;
  std::memset(&w, 0, sizeof(w));
  w.g.M = (int)R; w.g.Nc = O; w.g.Kc = I; w.g.KT = 1; w.g.S = 1; w.g.P = 0; w.g.transposed = 0;
  w.g.T_out = 1; w.g.T_in = 1; w.g.V = 1; w.g.lda = lda; w.g.ldo = O;
  w.dy = dy; w.ldy = O; w.in = in; w.dw = dW; w.db = db; w.outmap = WG_OUT_CONV; w.bf16 = bf16;
  return f3_conv_wgrad(&w, 0, s);
}

BnRef bnref(const f3_sktr* net, const Plan& p, void* ws, const float* params, const float* buffers, int b, int k,
            long long R, bool train) {
  const BnOff& o = net->blk[b].bn[k];
  BnRef r;
  const int idx = b * 3 + k;
  r.sum = at<double>(ws, p.fsum) + idx * 64;
  r.sumsq = r.sum + 32;
  r.gamma = params + o.w;
  r.beta = params + o.b;
  r.rmean = buffers + o.rm;
  r.rvar = buffers + o.rv;
  r.count = (float)R;
  r.eval = train ? 0 : 1;
  return r;
}

// transposed weight slots of block b: Wqkv^T [32][384] and Wm^T [128][32] per attention, W1^T [32][128], W2^T [128][32]
float* packT(void* ws, const Plan& p, int b, int which, bool fwd = false) {
  float* base = at<float>(ws, fwd ? p.packF : p.packT) + (size_t)b * kPackPerBlock;
  const size_t sz[6] = {QKV * EMB, DM * EMB, QKV * EMB, DM * EMB, FFN * EMB, FFN * EMB};
  for (int i = 0; i < which; ++i) base += sz[i];
  return base;
}

}  // namespace

extern "C" {

int f3_sktr_create(const f3_sktr_config* cfg, f3_sktr** out) {
  if (!cfg || !out) return F3_EINVAL;
  *out = nullptr;
  if (!f3_sk_attn_len_ok(cfg->num_joint) || !f3_sk_attn_len_ok(cfg->frames) || cfg->persons < 1 ||
      cfg->num_class < 1 || cfg->num_class > 64)
    return F3_EINVAL;
  f3_sktr* n = new f3_sktr();
  n->V = cfg->num_joint; n->T = cfg->frames; n->M = cfg->persons; n->C = cfg->num_class;
  if (cfg->precision != F3_PRECISION_FP32 && cfg->precision != F3_PRECISION_BF16) { delete n; return F3_EINVAL; }
  n->prec = cfg->precision;
  // state_dict order of SkeletonTransformer (checked against the reference by tools/gen_golden.py)
  n->e_w1 = n->add("embedding.0.weight", {HID0, CIN});
  n->e_b1 = n->add("embedding.0.bias", {HID0});
  n->e_w2 = n->add("embedding.2.weight", {EMB, HID0});
  n->e_b2 = n->add("embedding.2.bias", {EMB});
  for (int b = 0; b < NBLOCK; ++b) {
    const std::string p = "extractor." + std::to_string(b) + ".";
    BlockOff& B = n->blk[b];
    for (int k = 0; k < 2; ++k) {
      const std::string q = p + (k == 0 ? "multi_head_spatial_self_attention." : "multi_head_temporal_self_attention.");
      const int L = k == 0 ? n->V : n->T;
      AttnOff& A = B.at[k];
      A.table = n->add(q + "relative_position_bias_table", {2 * L - 1, HD});
      A.wqkv = n->add(q + "w_qkv.weight", {QKV, EMB});
      A.bqkv = n->add(q + "w_qkv.bias", {QKV});
      A.wm = n->add(q + "merge.weight", {EMB, DM});
      A.bm = n->add(q + "merge.bias", {EMB});
      const std::string nb = p + (k == 0 ? "norm1." : "norm2.");
      BnOff& o = B.bn[k];
      o.w = n->add(nb + "weight", {EMB});
      o.b = n->add(nb + "bias", {EMB});
      o.rm = n->add(nb + "running_mean", {EMB}, F3_ENTRY_BUFFER);
      o.rv = n->add(nb + "running_var", {EMB}, F3_ENTRY_BUFFER);
      o.nbt = n->add(nb + "num_batches_tracked", {}, F3_ENTRY_COUNTER);
    }
    B.w1 = n->add(p + "feed_forward_network.0.weight", {FFN, EMB});
    B.b1 = n->add(p + "feed_forward_network.0.bias", {FFN});
    B.w2 = n->add(p + "feed_forward_network.2.weight", {EMB, FFN});
    B.b2 = n->add(p + "feed_forward_network.2.bias", {EMB});
    BnOff& o = B.bn[2];
    o.w = n->add(p + "norm3.weight", {EMB});
    o.b = n->add(p + "norm3.bias", {EMB});
    o.rm = n->add(p + "norm3.running_mean", {EMB}, F3_ENTRY_BUFFER);
    o.rv = n->add(p + "norm3.running_var", {EMB}, F3_ENTRY_BUFFER);
    o.nbt = n->add(p + "norm3.num_batches_tracked", {}, F3_ENTRY_COUNTER);
  }
  n->fc_w = n->add("fcn.0.weight", {n->C, EMB, 1, 1});
  n->fc_b = n->add("fcn.0.bias", {n->C});
  for (auto& r : n->sd)
    for (float& v : r) v = 1.f;
  *out = n;
  return F3_OK;
}

void f3_sktr_destroy(f3_sktr* net) { delete net; }
int f3_sktr_num_entries(const f3_sktr* net) { return net ? (int)net->entries.size() : 0; }

int f3_sktr_entry(const f3_sktr* net, int i, const char** name, int* kind, int* ndim, int64_t* shape8,
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

int64_t f3_sktr_param_count(const f3_sktr* net) { return net ? net->nparam : 0; }
int64_t f3_sktr_buffer_count(const f3_sktr* net) { return net ? net->nbuf : 0; }
int64_t f3_sktr_counter_count(const f3_sktr* net) { return net ? net->ncnt : 0; }

int64_t f3_sktr_workspace_bytes(const f3_sktr* net, int batch) {
  if (!net || batch < 1) return 0;
  return (int64_t)plan(net, batch).total;
}

int f3_sktr_forward(f3_sktr* net, int N, int training, const float* params, float* buffers, int64_t* counters,
                    const float* x, float* out, void* workspace, const float* sd, unsigned dropout_seed,
                    float dropout_p, void* stream) {
  if (!net || N < 1 || !params || !buffers || !x || !out || !workspace) return F3_EINVAL;
  if (training && !counters) return F3_EINVAL;
  if (dropout_p < 0.f || dropout_p >= 1.f) return F3_EINVAL;
  const long long R = (long long)N * net->M * net->T * net->V;
  if (training && R < 2) return F3_EBATCH;
  hipStream_t s = (hipStream_t)stream;
  const Plan p = plan(net, N);
  void* ws = workspace;
  const bool tr = training != 0;
  if (tr) {
    for (int b = 0; b < NBLOCK; ++b)
      for (int k = 0; k < 3; ++k) net->sd[b][k] = sd ? sd[b * 3 + k] : 1.f;
    net->seed = dropout_seed;
    net->drop_p = dropout_p;
    net->trained_batch = N;
    if (hipMemsetAsync(at<char>(ws, p.fsum), 0, 8 * 18 * 64, s) != hipSuccess) return F3_EHIP;
  } else {
    net->trained_batch = 0;
  }
  EmbedArgs ea;
  std::memset(&ea, 0, sizeof(ea));
  ea.N = N; ea.M = net->M; ea.T = net->T; ea.V = net->V; ea.x = x;
  ea.w1 = params + net->e_w1; ea.b1 = params + net->e_b1; ea.w2 = params + net->e_w2; ea.b2 = params + net->e_b2;
  ea.y = at<float>(ws, p.y0);
  SK_TRY(f3_sk_embed_fwd_save(&ea, at<float>(ws, p.xt), at<float>(ws, p.a1), at<float>(ws, p.h1), at<float>(ws, p.a2),
                              s));
  const bool hb = net->prec == F3_PRECISION_BF16;
  if (hb) {  // the block Linears' weights as bf16 GEMM operands ([O][I], nn.Linear layout)
    PrepTable t;
    t.n = 0;
    auto job = [&](float* dst, const float* src, int O, int I) {
      PrepJob& j = t.jobs[t.n++];
      std::memset(&j, 0, sizeof(j));
      j.type = PREP_PACK_CONV; j.n = O * I; j.dst = dst; j.s0 = src; j.d0 = O; j.d1 = I; j.d2 = 1; j.bf16 = 1;
    };
    for (int b = 0; b < NBLOCK; ++b) {
      const BlockOff& B = net->blk[b];
      for (int k = 0; k < 2; ++k) {
        job(packT(ws, p, b, 2 * k, true), params + B.at[k].wqkv, QKV, EMB);
        job(packT(ws, p, b, 2 * k + 1, true), params + B.at[k].wm, EMB, DM);
      }
      job(packT(ws, p, b, 4, true), params + B.w1, FFN, EMB);
      job(packT(ws, p, b, 5, true), params + B.w2, EMB, FFN);
    }
    SK_TRY(f3_prep(t, s));
  }
  auto wbf = [&](int b, int which) -> const void* { return hb ? packT(ws, p, b, which, true) : nullptr; };
  const float scale = 1.f / std::sqrt((float)DM);
  float* mt = at<float>(ws, p.mtmp);
  const float* yin = at<float>(ws, p.y0);
  for (int b = 0; b < NBLOCK; ++b) {
    const BlockOff& B = net->blk[b];
    const BlockWs& W = p.b[b];
    const float* ycur = yin;
    for (int k = 0; k < 2; ++k) {  // spatial (over joints), temporal (over frames)
      const AttnOff& A = B.at[k];
      float* qkv = at<float>(ws, W.qkv[k]);
      float* o = at<float>(ws, W.o[k]);
      SK_TRY(linear(ycur, EMB, params + A.wqkv, params + A.bqkv, qkv, QKV, R, EPI_BIAS, s, wbf(b, 2 * k)));
      AttnArgs aa;
      std::memset(&aa, 0, sizeof(aa));
      aa.L = k == 0 ? net->V : net->T;
      aa.temporal = k;
      aa.nseq = (int)(k == 0 ? (long long)N * net->M * net->T : (long long)N * net->M * net->V);
      aa.T = net->T; aa.V = net->V; aa.scale = scale;
      aa.qkv = qkv; aa.table = params + A.table; aa.o = o;
      SK_TRY(f3_sk_attn_fwd(&aa, s));
      SK_TRY(linear(o, DM, params + A.wm, params + A.bm, mt, EMB, R, EPI_BIAS, s, wbf(b, 2 * k + 1)));
      BnRef bn = bnref(net, p, ws, params, buffers, b, k, R, tr);
      ResidArgs ra;
      std::memset(&ra, 0, sizeof(ra));
      ra.R = R; ra.a = ycur; ra.f = mt; ra.s = tr ? net->sd[b][k] : 1.f;
      ra.u = at<float>(ws, W.u[k]);
      ra.sum = tr ? const_cast<double*>(bn.sum) : nullptr;
      ra.sumsq = tr ? const_cast<double*>(bn.sumsq) : nullptr;
      SK_TRY(f3_sk_resid(&ra, s));
      BnApplyArgs ba;
      ba.R = R; ba.u = ra.u; ba.bn = bn; ba.y = at<float>(ws, k == 0 ? W.y1 : W.y2);
      SK_TRY(f3_sk_bn_apply(&ba, s));
      ycur = ba.y;
    }
    // feed-forward network (Linear 32->128, GELU, Linear 128->32, Dropout)
    float* h = at<float>(ws, W.h);
    float* g = at<float>(ws, W.g);
    SK_TRY(linear(ycur, EMB, params + B.w1, params + B.b1, h, FFN, R, EPI_BIAS, s, wbf(b, 4)));
    GeluArgs ga;
    std::memset(&ga, 0, sizeof(ga));
    ga.n = R * FFN; ga.h = h; ga.g = g;
    SK_TRY(f3_sk_gelu_fwd(&ga, s));
    SK_TRY(linear(g, FFN, params + B.w2, params + B.b2, mt, EMB, R, EPI_BIAS, s, wbf(b, 5)));
    BnRef bn = bnref(net, p, ws, params, buffers, b, 2, R, tr);
    ResidArgs ra;
    std::memset(&ra, 0, sizeof(ra));
    ra.R = R; ra.a = yin; ra.b = ycur; ra.f = mt; ra.s = tr ? net->sd[b][2] : 1.f;
    ra.seed = net->seed; ra.block = b; ra.drop_p = tr ? net->drop_p : 0.f;
    ra.u = at<float>(ws, W.u[2]);
    ra.sum = tr ? const_cast<double*>(bn.sum) : nullptr;
    ra.sumsq = tr ? const_cast<double*>(bn.sumsq) : nullptr;
    SK_TRY(f3_sk_resid(&ra, s));
    BnApplyArgs ba;
    ba.R = R; ba.u = ra.u; ba.bn = bn; ba.y = at<float>(ws, W.yout);
    SK_TRY(f3_sk_bn_apply(&ba, s));
    yin = ba.y;
  }
  if (tr) {  // running statistics (momentum 0.1, unbiased variance) and num_batches_tracked
    BnRunTable t;
    t.n = 0;
    for (int b = 0; b < NBLOCK; ++b)
      for (int k = 0; k < 3; ++k) {
        const BnOff& o = net->blk[b].bn[k];
        BnRunJob& j = t.jobs[t.n++];
        j.sum = at<double>(ws, p.fsum) + (b * 3 + k) * 64;
        j.sumsq = j.sum + 32;
        j.count = (double)R;
        j.C = EMB;
        j.rmean = buffers + o.rm;
        j.rvar = buffers + o.rv;
        j.nbt = reinterpret_cast<long long*>(counters + o.nbt);
      }
    SK_TRY(f3_bn_running(t, s));
  }
  sk::HeadArgs hd;
  std::memset(&hd, 0, sizeof(hd));
  hd.N = N; hd.MTV = net->M * net->T * net->V; hd.C = net->C;
  hd.y = yin; hd.w = params + net->fc_w; hd.b = params + net->fc_b;
  hd.pooled = at<float>(ws, p.pooled); hd.out = out;
  return f3_sk_head_fwd(&hd, s);
}

int f3_sktr_backward(f3_sktr* net, int N, const float* params, const float* buffers, const float* dout,
                     float* grads, void* workspace, void* stream) {
  if (!net || N < 1 || !params || !buffers || !dout || !grads || !workspace) return F3_EINVAL;
  if (net->trained_batch != N) return F3_ESTATE;
  hipStream_t s = (hipStream_t)stream;
  const Plan p = plan(net, N);
  void* ws = workspace;
  const long long R = (long long)N * net->M * net->T * net->V;
  if (hipMemsetAsync(grads, 0, sizeof(float) * net->nparam, s) != hipSuccess) return F3_EHIP;
  if (hipMemsetAsync(at<char>(ws, p.bsum), 0, 8 * 18 * 64, s) != hipSuccess) return F3_EHIP;
  {  // transposed weights for the input-gradient GEMMs
    PrepTable t;
    t.n = 0;
    auto job = [&](float* dst, const float* src, int O, int I) {  // dst[I][O] = src[O][I]
      PrepJob& j = t.jobs[t.n++];
      std::memset(&j, 0, sizeof(j));
      j.type = PREP_PACK_CONV_T; j.n = O * I; j.dst = dst; j.s0 = src; j.d0 = O; j.d1 = I; j.d2 = 1;
      j.bf16 = net->prec == F3_PRECISION_BF16;  // bf16 mode: the transposed copies are bf16 operands
    };
    for (int b = 0; b < NBLOCK; ++b) {
      const BlockOff& B = net->blk[b];
      for (int k = 0; k < 2; ++k) {
        job(packT(ws, p, b, 2 * k), params + B.at[k].wqkv, QKV, EMB);
        job(packT(ws, p, b, 2 * k + 1), params + B.at[k].wm, EMB, DM);
      }
      job(packT(ws, p, b, 4), params + B.w1, FFN, EMB);
      job(packT(ws, p, b, 5), params + B.w2, EMB, FFN);
    }
    SK_TRY(f3_prep(t, s));
  }
  // classifier + pool: dY of the last block's output
  float* dy_cur = at<float>(ws, p.dya);
  float* dy_next = at<float>(ws, p.dyb);
  {
    sk::HeadArgs hd;
    std::memset(&hd, 0, sizeof(hd));
    hd.N = N; hd.MTV = net->M * net->T * net->V; hd.C = net->C;
    hd.w = params + net->fc_w; hd.pooled = at<float>(ws, p.pooled);
    hd.dout = dout; hd.dy = dy_cur; hd.gw = grads + net->fc_w; hd.gb = grads + net->fc_b;
    SK_TRY(f3_sk_head_bwd(&hd, s));
  }
  const float scale = 1.f / std::sqrt((float)DM);
  float* du3 = at<float>(ws, p.du3);
  float* dy2 = at<float>(ws, p.dy2);
  float* dy1 = at<float>(ws, p.dy1);
  float* dm = at<float>(ws, p.dm);
  float* dbig = at<float>(ws, p.dbig);
  float* dqkv = at<float>(ws, p.dqkv);
  const int hb = net->prec == F3_PRECISION_BF16;
  // the input-gradient GEMMs' B operand: fp32 transposed weights, or their bf16 copies (same slots)
  auto lin_t = [&](const float* dy, int O, int b, int which, float* out, int I, int epi) {
    const float* wt = packT(ws, p, b, which);
    return linear(dy, O, hb ? nullptr : wt, nullptr, out, I, R, epi, s, hb ? (const void*)wt : nullptr);
  };
  for (int b = NBLOCK - 1; b >= 0; --b) {
    const BlockOff& B = net->blk[b];
    const BlockWs& W = p.b[b];
    const float* yin = b == 0 ? at<float>(ws, p.y0) : at<float>(ws, p.b[b - 1].yout);
    auto bnb = [&](int k, const float* dy, const float* u, const float* add, float* o1, float* o2, float* o3, float s2,
                   float drop_p) {
      sk::BnBwdArgs a;
      std::memset(&a, 0, sizeof(a));
      a.R = R; a.dy = dy; a.u = u;
      a.bn = bnref(net, p, ws, params, buffers, b, k, R, true);
      a.s_dy = at<double>(ws, p.bsum) + (b * 3 + k) * 64;
      a.s_dyx = a.s_dy + 32;
      a.add = add; a.o1 = o1; a.o2 = o2; a.o3 = o3; a.s2 = s2;
      a.seed = net->seed; a.block = b; a.drop_p = drop_p;
      a.g_gamma = grads + B.bn[k].w; a.g_beta = grads + B.bn[k].b;
      return f3_sk_bn_bwd(&a, s);
    };
    // BN3: dU3 -> dy2 (its skip into y2) and du3 (kept for y0); dF = sd * drop'(dU3)
    SK_TRY(bnb(2, dy_cur, at<float>(ws, W.u[2]), nullptr, dy2, dm, du3, net->sd[b][2], net->drop_p));
    // FFN backward
    SK_TRY(linear_wgrad(dm, EMB, at<float>(ws, W.g), FFN, FFN, grads + B.w2, grads + B.b2, R, s, hb));
    SK_TRY(lin_t(dm, EMB, b, 5, dbig, FFN, 0));   // dG = dF W2
    GeluArgs ga;
    std::memset(&ga, 0, sizeof(ga));
    ga.n = R * FFN; ga.h = at<float>(ws, W.h); ga.dg = dbig; ga.dh = dbig;
    SK_TRY(f3_sk_gelu_bwd(&ga, s));
    SK_TRY(linear_wgrad(dbig, FFN, at<float>(ws, W.y2), EMB, EMB, grads + B.w1, grads + B.b1, R, s, hb));
    SK_TRY(lin_t(dbig, FFN, b, 4, dy2, EMB, EPI_ADD));   // dy2 += dH W1
    // temporal then spatial attention
    for (int k = 1; k >= 0; --k) {
      const AttnOff& A = B.at[k];
      const float* dyk = k == 1 ? dy2 : dy1;
      float* o1 = k == 1 ? dy1 : dy_next;           // dU + (skip): y1's / y0's gradient so far
      const float* add = k == 1 ? nullptr : du3;    // y0 also feeds u3 directly
      SK_TRY(bnb(k, dyk, at<float>(ws, W.u[k]), add, o1, dm, nullptr, net->sd[b][k], 0.f));
      const float* xin = k == 1 ? at<float>(ws, W.y1) : yin;
      SK_TRY(linear_wgrad(dm, EMB, at<float>(ws, W.o[k]), DM, DM, grads + A.wm, grads + A.bm, R, s, hb));
      SK_TRY(lin_t(dm, EMB, b, 2 * k + 1, dbig, DM, 0));   // dO = dM Wm
      AttnArgs aa;
      std::memset(&aa, 0, sizeof(aa));
      aa.L = k == 0 ? net->V : net->T;
      aa.temporal = k;
      aa.nseq = (int)(k == 0 ? (long long)N * net->M * net->T : (long long)N * net->M * net->V);
      aa.T = net->T; aa.V = net->V; aa.scale = scale;
      aa.qkv = at<float>(ws, W.qkv[k]); aa.table = params + A.table;
      aa.dout = dbig; aa.dqkv = dqkv; aa.dtab = at<float>(ws, p.dtab);
      SK_TRY(f3_sk_attn_bwd(&aa, s));
      SK_TRY(f3_colsum(aa.dtab, aa.nseq, (2 * aa.L - 1) * HD, grads + A.table, s));
      SK_TRY(linear_wgrad(dqkv, QKV, xin, EMB, EMB, grads + A.wqkv, grads + A.bqkv, R, s, hb));
      SK_TRY(lin_t(dqkv, QKV, b, 2 * k, o1, EMB, EPI_ADD));   // += dQKV Wqkv
    }
    std::swap(dy_cur, dy_next);
  }
  // embedding
  EmbedArgs ea;
  std::memset(&ea, 0, sizeof(ea));
  ea.N = N; ea.M = net->M; ea.T = net->T; ea.V = net->V;
  ea.w1 = params + net->e_w1; ea.b1 = params + net->e_b1; ea.w2 = params + net->e_w2; ea.b2 = params + net->e_b2;
  ea.dy = dy_cur;
  float* da1 = at<float>(ws, p.da1);
  float* da2 = at<float>(ws, p.da2);
  SK_TRY(f3_sk_embed_bwd_save(&ea, at<float>(ws, p.a1), at<float>(ws, p.a2), da1, da2, s));
  SK_TRY(linear_wgrad(da2, EMB, at<float>(ws, p.h1), HID0, HID0, grads + net->e_w2, grads + net->e_b2, R, s));
  return linear_wgrad(da1, HID0, at<float>(ws, p.xt), CIN, 4, grads + net->e_w1, grads + net->e_b1, R, s);
}

}  // extern "C"
