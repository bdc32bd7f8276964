// TARGCN training step (BASELINE config 2) behind the C ABI in include/fall3.h (f3_targcn_*).
//
// Replaces, for the skeleton-only TARGCN notebook (TARGCN_HAR_conv_10kfold.ipynb cell 3):
//   model = TARGCN(adj=None).to(device)          -> f3_targcn_create        (TRAGCN.py:177-205)
//   out = model(pts.permute(0, 2, 3, 1))          -> f3_targcn_forward       (TRAGCN.py:207-224)
//   loss.backward()                               -> f3_targcn_backward
//   (CrossEntropyLoss / RMSprop: f3_soft_ce / f3_rmsprop_step)
//
// Forward launches: supports + static scale, 4 EmbGCN weight packs, end_conv mean, GRU layer 0,
// GRU layer 1 (persistent per clip tile, 30 steps each), TA layer 0, TA layer 1, pool, Linear.
// Backward: Linear, pool, TA 1, TA 0, GRU 1 BPTT -> its per-node weight gradients (grouped
// MFMA GEMMs over B*T rows) and support gradient, GRU 0 likewise, then the E / pool reductions.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>
#include <string>
#include <vector>

#include "fall3.h"
#include "kernels.h"
#include "sensor.h"
#include "status_ring.h"
#include "targcn.h"

using namespace f3;
using namespace f3::tg;

namespace {

struct Entry {
  std::string name;
  int kind;
  std::vector<int64_t> shape;
  int64_t off;
};

struct EmbOff {
  int64_t pool, bpool, lin, linb;
  int I, O;
};

struct TaOff {
  int64_t vw, vb, c1w, c1b, c2w, c2b, lnw, lnb, lnffw, lnffb, f0w, f0b, f2w, f2b;
};

constexpr int DIN0 = 3;

}  // namespace

struct f3_targcn {
  int V, C, prec;
  std::vector<Entry> entries;
  int64_t nparam = 0, nbuf = 0;
  int64_t E = 0;
  EmbOff emb[2][2];  // [layer][gate, update]
  TaOff ta[2];
  int64_t end_w = 0, end_b = 0, fc_w = 0, fc_b = 0, pe = 0;
  // f3_targcn_stage_times: timing events around the recurrences and the TA layers (0 = off)
  int timing = 0;
  hipEvent_t tev[11] = {};
  // GRU group-barrier error flag: copied after the recurrences of every call into a pinned ring
  // (status_ring.h), reported once as F3_EDEVICE
  StatusRing status;
  // F3_TG_PROF (debugging aid): the GRU forward / backward per-phase stamp buffers, owned here so they are
  // released by f3_targcn_destroy, never by an exit-time destructor after the HIP runtime's teardown
  long long* prof[2] = {nullptr, nullptr};
  ~f3_targcn() {
    for (auto& e : tev) if (e) (void)hipEventDestroy(e);
    for (auto& p : prof) if (p) (void)hipFree(p);
  }

  int64_t add(const std::string& name, std::vector<int64_t> shape, int kind = F3_ENTRY_PARAM) {
    int64_t n = 1;
    for (auto d : shape) n *= d;
    Entry e{name, kind, shape, 0};
    if (kind == F3_ENTRY_PARAM) {
      e.off = nparam;
      nparam += (n + 3) / 4 * 4;  // 16-B aligned entries (float4 RMSprop)
    } else {
      e.off = nbuf;
      nbuf += n;
    }
    entries.push_back(e);
    return e.off;
  }
};

namespace {

// Workspace plan for one batch size: byte offsets, 256-B aligned.
struct Plan {
  size_t S, cs, Wm, bm;
  size_t ops[2][2][5];  // Wf, Wb, Lf, Lb, bn
  size_t H[2], ZR[2], SG[2], HC[2], SU[2], XG[2], XI[2], UG[2], UI[2];
  size_t ta_out0, ta_out1, ta_save[2], ta_part, xm, pooled;
  size_t hx, rhx, gsync, gx1, gx2;  // node-partitioned recurrences: exchange buffers, barrier counters
  // backward
  size_t dlog, dpooled, dY0, dH1, dH0, DP, DSG, DU, DSU, DXG, DUG;
  size_t zero_begin, dW[2][2][4], dS, dY1, zpage, zero_end;
  size_t total;
};

Plan plan(const f3_targcn* net, int B) {
  Plan p;
  size_t o = 0;
  auto take = [&](size_t bytes) {
    const size_t at = o;
    o += (bytes + 255) / 256 * 256;
    return at;
  };
  const int V = net->V;
  const size_t es = net->prec == F3_PRECISION_FP32 ? 4 : 2;
  const size_t R = (size_t)B * T * V;
  p.S = take(4 * V * V);
  p.cs = take(4 * V);
  p.Wm = take(4 * C * 6 * H);
  p.bm = take(4 * C);
  for (int l = 0; l < 2; ++l)
    for (int q = 0; q < 2; ++q) {
      const int O = q == 0 ? 2 * H : H;
      p.ops[l][q][0] = take(es * V * O * IP);
      p.ops[l][q][1] = take(es * V * IP * O);
      p.ops[l][q][2] = take(es * O * IP);
      p.ops[l][q][3] = take(es * IP * O);
      p.ops[l][q][4] = take(4 * V * O);
    }
  for (int l = 0; l < 2; ++l) {
    p.H[l] = take(4 * R * H);
    p.ZR[l] = take(4 * R * 2 * H);
    p.SG[l] = take(4 * R * 2 * H);
    p.HC[l] = take(4 * R * H);
    p.SU[l] = take(4 * R * H);
    p.XG[l] = take(es * R * IP);
    p.XI[l] = take(es * R * IP);
    p.UG[l] = take(es * R * IP);
    p.UI[l] = take(es * R * IP);
  }
  p.hx = take(2 * (size_t)B * V * H);
  p.rhx = take(2 * (size_t)B * V * H);
  p.gsync = take(4 * (GN_MAXG + 1));
  p.gx1 = take(2 * (size_t)B * V * IP);
  p.gx2 = take(2 * (size_t)B * V * IP);
  p.ta_out0 = take(4 * R * C);
  p.ta_out1 = take(4 * R * C);
  for (int l = 0; l < 2; ++l) p.ta_save[l] = take(4 * (size_t)B * V * TA_SAVE);
  p.ta_part = take(4 * (size_t)TA_MAX_WG * TA_PART);
  p.xm = take(4 * (size_t)B * 6 * H);
  p.pooled = take(4 * (size_t)B * C);
  p.dlog = take(4 * (size_t)B * net->C);
  p.dpooled = take(4 * (size_t)B * C);
  p.dY0 = take(4 * R * C);
  p.dH1 = take(4 * R * H);
  p.dH0 = take(4 * R * H);
  p.DP = take(es * R * 2 * H);
  p.DSG = take(es * R * 2 * H);
  p.DU = take(es * R * H);
  p.DSU = take(es * R * H);
  p.DXG = take(es * R * IP);
  p.DUG = take(es * R * IP);
  p.zero_begin = o;
  for (int l = 0; l < 2; ++l)
    for (int q = 0; q < 2; ++q) {
      const int O = q == 0 ? 2 * H : H;
      p.dW[l][q][0] = take(4 * (size_t)V * O * IP);
      p.dW[l][q][1] = take(4 * (size_t)V * O);
      p.dW[l][q][2] = take(4 * (size_t)V * O * IP);
      p.dW[l][q][3] = take(4 * (size_t)V * O);
    }
  p.dS = take(4 * V * V);
  p.dY1 = take(4 * R * C);
  p.zpage = take(4096);
  p.zero_end = o;
  p.total = o;
  return p;
}

template <typename P>
P* at(void* ws, size_t off) {
  return reinterpret_cast<P*>(reinterpret_cast<char*>(ws) + off);
}

EmbOps ops_of(const f3_targcn* net, const Plan& p, void* ws, const float* params, int l, int q) {
  EmbOps o;
  o.Wf = at<void>(ws, p.ops[l][q][0]);
  o.Wb = at<void>(ws, p.ops[l][q][1]);
  o.Lf = at<void>(ws, p.ops[l][q][2]);
  o.Lb = at<void>(ws, p.ops[l][q][3]);
  o.bn = at<float>(ws, p.ops[l][q][4]);
  o.bl = params + net->emb[l][q].linb;
  return o;
}

TaArgs ta_args(const f3_targcn* net, int l, int B, const float* params) {
  TaArgs a;
  std::memset(&a, 0, sizeof(a));
  a.B = B;
  a.V = net->V;
  a.b16 = net->prec == F3_PRECISION_BF16;
  a.p = params;
  const TaOff& t = net->ta[l];
  a.off_vw = t.vw; a.off_vb = t.vb; a.off_c1w = t.c1w; a.off_c1b = t.c1b; a.off_c2w = t.c2w; a.off_c2b = t.c2b;
  a.off_lnw = t.lnw; a.off_lnb = t.lnb; a.off_lnffw = t.lnffw; a.off_lnffb = t.lnffb;
  a.off_f0w = t.f0w; a.off_f0b = t.f0b; a.off_f2w = t.f2w; a.off_f2b = t.f2b;
  return a;
}

// stage timing marks (f3_targcn_stage_times): forward 0 | gru0 | 1 | gru1 | 2 | ta0 | 3 | ta1 | 4,
// backward 5 | ta1 | 6 | ta0 | 7 | gru1 | 8 ... 9 | gru0 | 10
inline void mark(f3_targcn* n, int i, hipStream_t s) {
  if (n->timing && n->tev[i]) (void)hipEventRecord(n->tev[i], s);
}

#define TG_TRY(x)                 \
  do {                            \
    const int _st = (x);          \
    if (_st != F3_OK) return _st; \
  } while (0)

}  // namespace

namespace {

// F3_GN_SKIP_ARRIVE: test knob, workgroup 0 of the node-partitioned recurrences never arrives at
// the group barriers (they time out and raise the flag): 1 in the forward and backward recurrences,
// 2 in the backward ones only
int gn_skip_arrive(bool backward) {
  const char* e = getenv("F3_GN_SKIP_ARRIVE");
  const int v = e ? atoi(e) : 0;
  return v == 1 || (v == 2 && backward);
}

int take_status(f3_targcn* net, bool wait) { return net->status.take(wait); }

// enqueue the copy of the flag (gsync[GN_MAXG]); the node-partitioned path is off under capture
int post_status(f3_targcn* net, const int* gsync, hipStream_t s) { return net->status.post(gsync + GN_MAXG, s); }

}  // namespace

extern "C" {

int f3_targcn_create(const f3_targcn_config* cfg, f3_targcn** out) {
  if (!cfg || !out) return F3_EINVAL;
  *out = nullptr;
  if (!f3_tg_gru_lds_ok(cfg->num_node) || cfg->num_class < 1 || cfg->num_class > 64) return F3_EINVAL;
  if (cfg->precision != F3_PRECISION_FP32 && cfg->precision != F3_PRECISION_BF16) return F3_EINVAL;
  f3_targcn* n = new f3_targcn();
  n->V = cfg->num_node;
  n->C = cfg->num_class;
  n->prec = cfg->precision;
  // state_dict order of TARGCN(adj=None, num_nodes=V) (TRAGCN.py:194-205)
  n->E = n->add("node_embeddings", {n->V, EMB});
  for (int l = 0; l < 2; ++l) {
    const int din = l == 0 ? DIN0 : H;
    for (int q = 0; q < 2; ++q) {
      const int O = q == 0 ? 2 * H : H, I = din + H;
      const std::string p = "encoder.dcrnn_cells." + std::to_string(l) + (q == 0 ? ".gate." : ".update.");
      EmbOff& e = n->emb[l][q];
      e.I = I;
      e.O = O;
      e.pool = n->add(p + "weights_pool", {EMB, I, O});
      e.bpool = n->add(p + "bias_pool", {EMB, O});
      e.lin = n->add(p + "linear.weight", {O, I});
      e.linb = n->add(p + "linear.bias", {O});
    }
  }
  for (int l = 0; l < 2; ++l) {
    const std::string p = "encoder.trans_layer_T.trans_layers." + std::to_string(l) + ".";
    TaOff& t = n->ta[l];
    t.vw = n->add(p + "vff.weight", {C, C});
    t.vb = n->add(p + "vff.bias", {C});
    t.c1w = n->add(p + "conv1.weight", {T, T, 1, 3});
    t.c1b = n->add(p + "conv1.bias", {T});
    t.c2w = n->add(p + "conv2.weight", {T, T, 1, 3});
    t.c2b = n->add(p + "conv2.bias", {T});
    t.lnw = n->add(p + "ln.weight", {C});
    t.lnb = n->add(p + "ln.bias", {C});
    t.lnffw = n->add(p + "lnff.weight", {C});
    t.lnffb = n->add(p + "lnff.bias", {C});
    t.f0w = n->add(p + "ff.0.weight", {C, C});
    t.f0b = n->add(p + "ff.0.bias", {C});
    t.f2w = n->add(p + "ff.2.weight", {C, C});
    t.f2b = n->add(p + "ff.2.bias", {C});
  }
  n->pe = n->add("encoder.trans_layer_T.PE.pe", {1, T, 1, C}, F3_ENTRY_BUFFER);
  n->end_w = n->add("end_conv.weight", {T * C, 6, 1, H});
  n->end_b = n->add("end_conv.bias", {T * C});
  n->fc_w = n->add("fc.2.weight", {n->C, C});
  n->fc_b = n->add("fc.2.bias", {n->C});
  *out = n;
  return F3_OK;
}

void f3_targcn_destroy(f3_targcn* net) { delete net; }

int f3_targcn_num_entries(const f3_targcn* net) { return net ? (int)net->entries.size() : 0; }

int f3_targcn_entry(const f3_targcn* net, int i, const char** name, int* kind, int* ndim, int64_t* shape8,
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

int64_t f3_targcn_param_count(const f3_targcn* net) { return net ? net->nparam : 0; }
int64_t f3_targcn_buffer_count(const f3_targcn* net) { return net ? net->nbuf : 0; }

int64_t f3_targcn_workspace_bytes(const f3_targcn* net, int batch) {
  if (!net || batch < 1) return 0;
  return (int64_t)plan(net, batch).total;
}

int f3_targcn_forward(f3_targcn* net, int B, const float* params, const float* buffers, const float* source,
                      float* out, void* workspace, void* stream) {
  if (!net || B < 1 || !params || !buffers || !source || !out || !workspace) return F3_EINVAL;
  hipStream_t s = (hipStream_t)stream;
  const Plan p = plan(net, B);
  void* ws = workspace;
  const int V = net->V, b16 = net->prec == F3_PRECISION_BF16;
  TG_TRY(take_status(net, false));
  // clear the barrier counters and the error flag once per forward (each recurrence launch
  // re-zeroes only its counters, so a flag raised by layer 0 survives to the status copy)
  if (hipMemsetAsync(at<char>(ws, p.gsync), 0, sizeof(int) * (GN_MAXG + 1), s) != hipSuccess) return F3_EHIP;
  const float* E = params + net->E;
  float* S = at<float>(ws, p.S);
  float* cs = at<float>(ws, p.cs);
  TG_TRY(f3_tg_supports(E, V, S, cs, s));
  for (int l = 0; l < 2; ++l)
    for (int q = 0; q < 2; ++q) {
      const EmbOff& e = net->emb[l][q];
      PrepArgs pa;
      pa.V = V; pa.I = e.I; pa.O = e.O;
      pa.E = E; pa.pool = params + e.pool; pa.bpool = params + e.bpool; pa.lin = params + e.lin;
      pa.ops = ops_of(net, p, ws, params, l, q);
      TG_TRY(f3_tg_prep(&pa, b16, s));
    }
  TG_TRY(f3_tg_endconv_mean(params + net->end_w, params + net->end_b, at<float>(ws, p.Wm), at<float>(ws, p.bm), s));
  mark(net, 0, s);
  for (int l = 0; l < 2; ++l) {  // AVWDCRNN (TRAGCN.py:159-166)
    GruFwdArgs g;
    std::memset(&g, 0, sizeof(g));
    g.B = B; g.V = V; g.Din = l == 0 ? DIN0 : H; g.I = g.Din + H;
    g.x = l == 0 ? source : at<float>(ws, p.H[0]);
    g.S = S; g.cs = cs;
    g.g = ops_of(net, p, ws, params, l, 0);
    g.u = ops_of(net, p, ws, params, l, 1);
    g.Hout = at<float>(ws, p.H[l]); g.ZR = at<float>(ws, p.ZR[l]); g.SG = at<float>(ws, p.SG[l]);
    g.HC = at<float>(ws, p.HC[l]); g.SU = at<float>(ws, p.SU[l]);
    g.XG = at<void>(ws, p.XG[l]); g.XI = at<void>(ws, p.XI[l]); g.UG = at<void>(ws, p.UG[l]); g.UI = at<void>(ws, p.UI[l]);
    g.hx = at<unsigned short>(ws, p.hx); g.rhx = at<unsigned short>(ws, p.rhx); g.gsync = at<int>(ws, p.gsync);
    g.dbg_skip_arrive = gn_skip_arrive(false);
    long long*& prof = net->prof[0];
    if (getenv("F3_TG_PROF") && !prof && hipMalloc(&prof, T * 8 * sizeof(long long)) != hipSuccess) prof = nullptr;
    g.prof = getenv("F3_TG_PROF") ? prof : nullptr;
    TG_TRY(f3_tg_gru_fwd(&g, b16, s));
    mark(net, 1 + l, s);
    if (g.prof) {  // debugging aid: per-phase microseconds of workgroup 0, averaged over the steps
      long long h[T * 8];
      (void)hipStreamSynchronize(s);
      (void)hipMemcpy(h, prof, sizeof(h), hipMemcpyDeviceToHost);
      double ph[8] = {0};
      // stamps: 0 step start, 1 fill, 2 mix, 7 row stores, 3 gate, 4 r*h, 5 mix, 6 update
      const int ord[8] = {0, 1, 2, 7, 3, 4, 5, 6};
      for (int t = 0; t < T; ++t)
        for (int k = 1; k < 8; ++k) ph[k] += (h[t * 8 + ord[k]] - h[t * 8 + ord[k - 1]]) * 0.01 / T;  // 100 MHz
      fprintf(stderr, "gru_fwd layer %d per-step phases (us) fill/mix/stores/gate/rh/mix/stores+update:", l);
      for (int k = 1; k < 8; ++k) fprintf(stderr, " %.2f", ph[k]);
      fprintf(stderr, "\n");
    }
  }
  if (b16) TG_TRY(post_status(net, at<int>(ws, p.gsync), s));
  for (int l = 0; l < 2; ++l) {  // transformer_layer (TA.py:101-108)
    TaArgs a = ta_args(net, l, B, params);
    a.in = l == 0 ? at<float>(ws, p.H[1]) : at<float>(ws, p.ta_out0);
    a.pe = l == 0 ? buffers + net->pe : nullptr;
    a.out = at<float>(ws, l == 0 ? p.ta_out0 : p.ta_out1);
    a.save = at<float>(ws, p.ta_save[l]);
    TG_TRY(f3_tg_ta_fwd(&a, s));
    mark(net, 3 + l, s);
  }
  TG_TRY(f3_tg_pool_fwd(at<float>(ws, p.ta_out1), B, V, at<float>(ws, p.Wm), at<float>(ws, p.bm), at<float>(ws, p.xm),
                        at<float>(ws, p.pooled), s));
  HeadArgs h;
  std::memset(&h, 0, sizeof(h));
  h.N = B; h.C = net->C; h.nblk = 1;
  h.feat[0] = at<float>(ws, p.pooled); h.width[0] = C; h.ld[0] = C;
  h.W = params + net->fc_w; h.b = params + net->fc_b; h.out = out;
  return f3_head_fwd(&h, s);
}

int f3_targcn_backward(f3_targcn* net, int B, const float* params, const float* buffers, const float* dout,
                       float* grads, void* workspace, void* stream) {
  if (!net || B < 1 || !params || !buffers || !dout || !grads || !workspace) return F3_EINVAL;
  hipStream_t s = (hipStream_t)stream;
  const Plan p = plan(net, B);
  void* ws = workspace;
  const int V = net->V, b16 = net->prec == F3_PRECISION_BF16;
  TG_TRY(take_status(net, false));
  if (hipMemsetAsync(grads, 0, sizeof(float) * net->nparam, s) != hipSuccess) return F3_EHIP;
  if (hipMemsetAsync(at<char>(ws, p.zero_begin), 0, p.zero_end - p.zero_begin, s) != hipSuccess) return F3_EHIP;
  // Linear(64 -> C)
  HeadArgs h;
  std::memset(&h, 0, sizeof(h));
  h.N = B; h.C = net->C; h.nblk = 1;
  h.feat[0] = at<float>(ws, p.pooled); h.width[0] = C; h.ld[0] = C;
  h.W = params + net->fc_w; h.b = params + net->fc_b;
  h.g_out = dout; h.dlogits = at<float>(ws, p.dlog);
  h.dfeat[0] = at<float>(ws, p.dpooled);
  h.g_W = grads + net->fc_w; h.g_b = grads + net->fc_b;
  TG_TRY(f3_head_bwd(&h, s));
  TG_TRY(f3_tg_pool_bwd(at<float>(ws, p.dpooled), at<float>(ws, p.xm), at<float>(ws, p.Wm), B, V, at<float>(ws, p.dY1),
                        grads + net->end_w, grads + net->end_b, s));
  mark(net, 5, s);
  for (int l = 1; l >= 0; --l) {
    TaArgs a = ta_args(net, l, B, params);
    a.in = l == 0 ? at<float>(ws, p.H[1]) : at<float>(ws, p.ta_out0);
    a.pe = l == 0 ? buffers + net->pe : nullptr;
    a.save = at<float>(ws, p.ta_save[l]);
    a.dout = at<float>(ws, l == 1 ? p.dY1 : p.dY0);
    a.din = at<float>(ws, l == 1 ? p.dY0 : p.dH1);
    a.grads = grads;
    a.part = at<float>(ws, p.ta_part);
    TG_TRY(f3_tg_ta_bwd(&a, s));
    mark(net, 7 - l, s);
  }
  const float* S = at<float>(ws, p.S);
  const float* cs = at<float>(ws, p.cs);
  const float* E = params + net->E;
  float* dS = at<float>(ws, p.dS);
  const unsigned short* zpage = at<unsigned short>(ws, p.zpage);
  for (int l = 1; l >= 0; --l) {
    GruBwdArgs g;
    std::memset(&g, 0, sizeof(g));
    g.B = B; g.V = V; g.Din = l == 0 ? DIN0 : H; g.I = g.Din + H;
    g.S = S; g.cs = cs;
    g.g = ops_of(net, p, ws, params, l, 0);
    g.u = ops_of(net, p, ws, params, l, 1);
    g.Hout = at<float>(ws, p.H[l]); g.ZR = at<float>(ws, p.ZR[l]); g.SG = at<float>(ws, p.SG[l]);
    g.HC = at<float>(ws, p.HC[l]); g.SU = at<float>(ws, p.SU[l]);
    g.dH = at<float>(ws, l == 1 ? p.dH1 : p.dH0);
    g.dX = l == 1 ? at<float>(ws, p.dH0) : nullptr;
    g.DP = at<void>(ws, p.DP); g.DSG = at<void>(ws, p.DSG); g.DU = at<void>(ws, p.DU); g.DSU = at<void>(ws, p.DSU);
    g.DXG = at<void>(ws, p.DXG); g.DUG = at<void>(ws, p.DUG);
    g.gx1 = at<unsigned short>(ws, p.gx1); g.gx2 = at<unsigned short>(ws, p.gx2); g.gsync = at<int>(ws, p.gsync);
    g.dbg_skip_arrive = gn_skip_arrive(true);
    long long*& prof = net->prof[1];
    if (getenv("F3_TG_PROF") && !prof && hipMalloc(&prof, T * 8 * sizeof(long long)) != hipSuccess) prof = nullptr;
    g.prof = getenv("F3_TG_PROF") ? prof : nullptr;
    mark(net, l == 1 ? 7 : 9, s);
    TG_TRY(f3_tg_gru_bwd(&g, b16, s));
    mark(net, l == 1 ? 8 : 10, s);
    if (g.prof) {
      long long h[T * 8];
      (void)hipStreamSynchronize(s);
      (void)hipMemcpy(h, prof, sizeof(h), hipMemcpyDeviceToHost);
      double ph[8] = {0};
      const int ord[8] = {0, 7, 1, 2, 3, 4, 5, 6};
      for (int t = 0; t < T; ++t)
        for (int k = 1; k < 8; ++k) ph[k] += (h[t * 8 + ord[k]] - h[t * 8 + ord[k - 1]]) * 0.01 / T;
      fprintf(stderr, "gru_bwd layer %d per-step phases (us) stage/upd-epi/upd-gemm/mixT/gate-epi/gate-gemm/mixT:", l);
      for (int k = 1; k < 8; ++k) fprintf(stderr, " %.2f", ph[k]);
      fprintf(stderr, "\n");
    }
    // per-node weight gradients over the B*T rows of each node (grouped GEMMs, one group per node)
    struct Job { size_t dy, x; int O; size_t dw, db; };
    const Job jobs[4] = {{p.DP, p.XG[l], 2 * H, p.dW[l][0][0], p.dW[l][0][1]},
                         {p.DSG, p.XI[l], 2 * H, p.dW[l][0][2], p.dW[l][0][3]},
                         {p.DU, p.UG[l], H, p.dW[l][1][0], p.dW[l][1][1]},
                         {p.DSU, p.UI[l], H, p.dW[l][1][2], p.dW[l][1][3]}};
    for (const Job& j : jobs) {
      WgradArgs w;
      std::memset(&w, 0, sizeof(w));
      const int M = B * T;
      w.g.M = M; w.g.Nc = j.O; w.g.Kc = IP; w.g.KT = 1; w.g.S = 1; w.g.P = 0; w.g.transposed = 0;
      w.g.T_out = M; w.g.T_in = M; w.g.V = 1; w.g.lda = V * IP; w.g.ldo = j.O;
      w.ldy = V * j.O;
      w.dw = at<float>(ws, j.dw); w.db = at<float>(ws, j.db);
      w.outmap = WG_OUT_CONV;
      w.groups = V; w.gs_dy = j.O; w.gs_in = IP; w.gs_dw = (long long)j.O * IP; w.gs_db = j.O;
      w.bf16 = b16;
      if (b16) {
        w.dyb = at<const unsigned short>(ws, j.dy);
        w.inb = at<const unsigned short>(ws, j.x);
        w.zero = zpage;
        if (!f3_wgrad_glds_ok(w)) return F3_EINVAL;
      } else {
        w.dy = at<const float>(ws, j.dy);
        w.in = at<const float>(ws, j.x);
      }
      TG_TRY(f3_conv_wgrad(&w, 0, s));
    }
    SuppGradArgs sg;
    sg.V = V; sg.I = g.I; sg.rows = B * T;
    sg.dxg[0] = at<void>(ws, p.DXG); sg.xin[0] = at<void>(ws, p.XI[l]);
    sg.dxg[1] = at<void>(ws, p.DUG); sg.xin[1] = at<void>(ws, p.UI[l]);
    sg.dS = dS;
    TG_TRY(f3_tg_supp_grad(&sg, b16, s));
  }
  if (b16) TG_TRY(post_status(net, at<int>(ws, p.gsync), s));
  for (int l = 0; l < 2; ++l)
    for (int q = 0; q < 2; ++q) {
      const EmbOff& e = net->emb[l][q];
      PoolGradArgs a;
      a.V = V; a.I = e.I; a.O = e.O;
      a.E = E; a.pool = params + e.pool; a.bpool = params + e.bpool; a.cs = cs;
      a.dW = at<float>(ws, p.dW[l][q][0]); a.db = at<float>(ws, p.dW[l][q][1]);
      a.dWs = at<float>(ws, p.dW[l][q][2]); a.dbs = at<float>(ws, p.dW[l][q][3]);
      a.g_pool = grads + e.pool; a.g_bpool = grads + e.bpool; a.g_lin = grads + e.lin; a.g_linb = grads + e.linb;
      a.g_E = grads + net->E;
      TG_TRY(f3_tg_pool_grad(&a, s));
    }
  return f3_tg_supports_bwd(E, V, dS, grads + net->E, s);
}

int f3_targcn_stage_times(f3_targcn* net, int enable, float* ms) {
  if (!net) return F3_EINVAL;
  if (enable && !net->timing) {
    for (auto& e : net->tev)
      if (!e && hipEventCreate(&e) != hipSuccess) return F3_EHIP;
  }
  if (ms) {  // the last forward + backward: gru_fwd l0, l1, ta_fwd l0, l1, ta_bwd l1, l0, gru_bwd l1, l0
    if (!net->timing) return F3_ESTATE;
    const int pairs[8][2] = {{0, 1}, {1, 2}, {2, 3}, {3, 4}, {5, 6}, {6, 7}, {7, 8}, {9, 10}};
    for (int i = 0; i < 8; ++i) {
      if (hipEventSynchronize(net->tev[pairs[i][1]]) != hipSuccess ||
          hipEventElapsedTime(&ms[i], net->tev[pairs[i][0]], net->tev[pairs[i][1]]) != hipSuccess)
        return F3_EHIP;
    }
  }
  net->timing = enable;
  return F3_OK;
}

int f3_targcn_status(f3_targcn* net, int wait) {
  if (!net) return F3_EINVAL;
  return take_status(net, wait != 0);
}

int f3_soft_ce(const float* out, const float* label, int N, int C, float* loss, float* dout, void* stream) {
  if (!out || !label || !loss || !dout || N < 1 || C < 1) return F3_EINVAL;
  hipStream_t s = (hipStream_t)stream;
  // (f3_ce stores the loss; larger batches zero it and accumulate)
  HeadArgs h;
  std::memset(&h, 0, sizeof(h));
  h.N = N; h.C = C; h.out = const_cast<float*>(out); h.label = label; h.loss = loss; h.dout = dout;
  return f3_ce(&h, s);
}

}  // extern "C"
