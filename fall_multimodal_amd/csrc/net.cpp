// Native network plan + step schedule behind the C ABI (include/fall3.h).
//
// The plan mirrors the reference module tree (build_model.py:5-19 ->
// combination.py TwoStreamSTGCAN(_BiLSTM) / stgcan.py STGCAN / bilstm.py BiLSTM and the
// UR notebook CNN_BiLSTM) as a flat parameter table whose names, order and shapes are
// exactly the reference state_dict, so checkpoints interchange. Parameters, buffers and
// gradients live in flat arrays owned by the caller; activations, saved tensors, packed
// weights and reduction scratch live in one caller-provided workspace whose layout is a
// pure function of the batch size.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <functional>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "common.h"
#include "status_ring.h"
#include "kernels.h"
#include "layers.h"
#include "sensor.h"
#include "fall3.h"

using namespace f3;

namespace {

struct Entry {
  std::string name;
  int kind;
  std::vector<int64_t> shape;
  int64_t offset, numel;
  int phase;  // params: backward phase that finalises the gradient (1 = head side, 2 = input side)
};

// Backward runs in two phases so DP can all-reduce the first phase's gradients while the
// second computes: phase 1 = head, sensor branch and skeleton layers >= kSplitLayer;
// phase 2 = skeleton layers < kSplitLayer and data_bn. Parameter OFFSETS in the flat buffer
// are assigned phase-1-first (state_dict ORDER is unchanged), so each phase's gradients
// form one contiguous range.
constexpr int kSplitLayer = 4;

struct BnIdx {
  int w = -1, b = -1, rm = -1, rv = -1, nbt = -1, C = 0;
};

struct LayerIdx {
  int cin, cout, stride, res, T_in, T_out;
  int gcn_w, gcn_b, tcn_w, tcn_b, res_w = -1, res_b = -1, ca_w1, ca_b1, ca_w2, ca_b2, edge;
  BnIdx bn1, bn2, bnr, bnca;
};

struct StreamIdx {
  int cin, T, motion, A;
  BnIdx dbn;
  LayerIdx L[7];
  int cls_w = -1, cls_b = -1;
};

struct LstmIdx {
  int wih[2], whh[2], bih[2], bhh[2];
  BnIdx bn;
  int ca_w1, ca_b1, ca_w2, ca_b2, fc_w, fc_b;
  int S, Cs;
};

struct CnnIdx {
  int w1, b1, w2, b2, fcw, fcb;
  BnIdx bn1, bn2;
};

const int kChan[7][4] = {{-1, 64, 1, RES_NONE}, {64, 64, 1, RES_ID},    {64, 64, 1, RES_ID},
                         {64, 128, 2, RES_CONV}, {128, 128, 1, RES_ID}, {128, 256, 2, RES_CONV},
                         {256, 256, 1, RES_ID}};  // stgcan.py:182-194

}  // namespace

struct f3_net {
  // branch concurrency: the position stream runs on the caller's stream, the motion stream
  // and the sensor branch on two private streams forked/joined with events (capturable)
  // aux[0]: motion stream, aux[1]: sensor branch, aux[2]: weight-gradient side stream (both
  // skeleton streams' wgrad / gcn-bias work, off the backward critical path)
  hipStream_t aux[3] = {nullptr, nullptr, nullptr};
  hipEvent_t ev[4] = {nullptr, nullptr, nullptr, nullptr};
  hipEvent_t ev_main[2][7] = {};  // per (skeleton stream, layer) main -> side hand-offs
  // end of backward phase 1 on each queue it used ([0..2] aux, [3] the caller's stream): the
  // gradient all-reduce of the phase-1 bucket waits on these instead of the caller's stream
  // joining every queue, so phase 2's critical path starts while phase 1's weight gradients drain
  hipEvent_t ev_p1[4] = {nullptr, nullptr, nullptr, nullptr};
  int p1_mask = 0;  // bit i: ev_p1[i] recorded by the last phase-1 backward
  bool par_init = false, par_ok = false;
  // f3_net_sensor_times: events around the sensor CNN1D launches (0 = off): 0 | forward | 1,
  // 2 | backward | 3
  int stiming = 0;
  hipEvent_t sev[4] = {};
  // the cooperative CNN1D's group-barrier error word (sync[0] of its forward / backward launch),
  // copied to the host after each launch; reported once as F3_EDEVICE by the next f3_net_forward /
  // backward call or f3_net_status (status_ring.h)
  StatusRing cstatus;
  void smark(int i, hipStream_t s) {
    if (stiming && sev[i]) (void)hipEventRecord(sev[i], s);
  }
  ~f3_net() {
    for (auto& e : sev) if (e) (void)hipEventDestroy(e);
    for (auto& a : aux) if (a) (void)hipStreamDestroy(a);
    for (auto& e : ev) if (e) (void)hipEventDestroy(e);
    for (auto& e : ev_p1) if (e) (void)hipEventDestroy(e);
    for (int i = 0; i < 2; ++i)
      for (int l = 0; l < 7; ++l) {
        if (ev_main[i][l]) (void)hipEventDestroy(ev_main[i][l]);
      }
  }
  f3_config cfg;
  std::vector<Entry> entries;
  int64_t nparam = 0, nbuf = 0, ncnt = 0;
  int nstreams = 0;
  StreamIdx st[2];
  bool has_sensor = false, has_cnn = false;
  LstmIdx lstm;
  CnnIdx cnn;
  int fc_w = -1, fc_b = -1;
  int K, V;

  int cur_phase = 1;
  int64_t nparam_phase1 = 0;
  // f3_net_backward_rmsprop's plan, fixed by the parameter layout: computed once (first call)
  int fused_opt = -1;                  // -1 unknown, 0 one update after the backward, 1 per layer
  std::vector<RmsRanges> rest_ranges;  // parameters outside the skeleton layers' ranges
  int add(const std::string& name, int kind, std::vector<int64_t> shape) {
    Entry e;
    e.name = name;
    e.kind = kind;
    e.phase = cur_phase;
    e.shape = shape;
    e.numel = 1;
    for (auto d : shape) e.numel *= d;
    int64_t* ctr = kind == F3_ENTRY_PARAM ? &nparam : (kind == F3_ENTRY_BUFFER ? &nbuf : &ncnt);
    e.offset = *ctr;
    *ctr += e.numel;
    entries.push_back(e);
    return (int)entries.size() - 1;
  }
  void finalize_offsets() {  // phase-1 parameters first; every entry 16-B aligned (float4 RMSprop)
    int64_t off = 0;
    for (int ph = 1; ph <= 2; ++ph) {
      for (auto& e : entries)
        if (e.kind == F3_ENTRY_PARAM && e.phase == ph) {
          e.offset = off;
          off += (e.numel + 3) / 4 * 4;
        }
      if (ph == 1) nparam_phase1 = off;
    }
    nparam = off;  // includes the alignment padding (zero gradients, RMSprop leaves it at 0)
  }
  BnIdx add_bn(const std::string& p, int C) {
    BnIdx b;
    b.C = C;
    b.w = add(p + ".weight", F3_ENTRY_PARAM, {C});
    b.b = add(p + ".bias", F3_ENTRY_PARAM, {C});
    b.rm = add(p + ".running_mean", F3_ENTRY_BUFFER, {C});
    b.rv = add(p + ".running_var", F3_ENTRY_BUFFER, {C});
    b.nbt = add(p + ".num_batches_tracked", F3_ENTRY_COUNTER, {});
    return b;
  }
  void add_stream(StreamIdx& s, const std::string& pre, int cin, int motion, int num_class) {
    const std::string layers = cfg.naming == F3_NAMING_NOTEBOOK ? "st_gcn_networks" : "st_gcan_networks";
    s.cin = cin;
    s.motion = motion;
    s.T = motion ? cfg.frames - 1 : cfg.frames;
    s.A = add(pre + "A", F3_ENTRY_BUFFER, {K, V, V});
    cur_phase = 2;
    s.dbn = add_bn(pre + "data_bn", cin * V);
    int T = s.T;
    for (int i = 0; i < 7; ++i) {
      LayerIdx& L = s.L[i];
      L.cin = kChan[i][0] < 0 ? cin : kChan[i][0];
      L.cout = kChan[i][1];
      L.stride = kChan[i][2];
      L.res = kChan[i][3];
      L.T_in = T;
      L.T_out = (T - 1) / L.stride + 1;  // (T + 2*4 - 9)/s + 1
      T = L.T_out;
      const int ci = L.cin, co = L.cout;
      const std::string p = pre + layers + "." + std::to_string(i) + ".";
      cur_phase = i >= kSplitLayer ? 1 : 2;
      L.gcn_w = add(p + "gcn.conv.weight", F3_ENTRY_PARAM, {K * co, ci, 1, 1});
      L.gcn_b = add(p + "gcn.conv.bias", F3_ENTRY_PARAM, {K * co});
      L.bn1 = add_bn(p + "tcn.0", co);
      L.tcn_w = add(p + "tcn.2.weight", F3_ENTRY_PARAM, {co, co, 9, 1});
      L.tcn_b = add(p + "tcn.2.bias", F3_ENTRY_PARAM, {co});
      L.bn2 = add_bn(p + "tcn.3", co);
      if (L.res == RES_CONV) {
        L.res_w = add(p + "residual.0.weight", F3_ENTRY_PARAM, {co, ci, 1, 1});
        L.res_b = add(p + "residual.0.bias", F3_ENTRY_PARAM, {co});
        L.bnr = add_bn(p + "residual.1", co);
      }
      const std::string q = p + "channel_attention_module.atten.";
      L.ca_w1 = add(q + "1.weight", F3_ENTRY_PARAM, {co / 4, co, 1, 1});
      L.ca_b1 = add(q + "1.bias", F3_ENTRY_PARAM, {co / 4});
      L.bnca = add_bn(q + "2", co / 4);
      L.ca_w2 = add(q + "4.weight", F3_ENTRY_PARAM, {co, co / 4, 1, 1});
      L.ca_b2 = add(q + "4.bias", F3_ENTRY_PARAM, {co});
    }
    for (int i = 0; i < 7; ++i) {
      cur_phase = i >= kSplitLayer ? 1 : 2;
      s.L[i].edge = add(pre + "edge_importance." + std::to_string(i), F3_ENTRY_PARAM, {K, V, V});
    }
    cur_phase = 1;
    if (num_class > 0) {
      s.cls_w = add(pre + "cls.weight", F3_ENTRY_PARAM, {num_class, 256, 1, 1});
      s.cls_b = add(pre + "cls.bias", F3_ENTRY_PARAM, {num_class});
    }
  }
  void add_bilstm(const std::string& p, int S, int C) {
    const int H = 64;
    lstm.S = S;
    lstm.Cs = C;
    const char* sfx[2] = {"", "_reverse"};
    for (int d = 0; d < 2; ++d) {
      lstm.wih[d] = add(p + "lstm1.weight_ih_l0" + sfx[d], F3_ENTRY_PARAM, {4 * H, S});
      lstm.whh[d] = add(p + "lstm1.weight_hh_l0" + sfx[d], F3_ENTRY_PARAM, {4 * H, H});
      lstm.bih[d] = add(p + "lstm1.bias_ih_l0" + sfx[d], F3_ENTRY_PARAM, {4 * H});
      lstm.bhh[d] = add(p + "lstm1.bias_hh_l0" + sfx[d], F3_ENTRY_PARAM, {4 * H});
    }
    lstm.bn = add_bn(p + "batchnorm", 2 * H);
    lstm.ca_w1 = add(p + "channelattention.attention.0.weight", F3_ENTRY_PARAM, {2 * H / 8, 2 * H});
    lstm.ca_b1 = add(p + "channelattention.attention.0.bias", F3_ENTRY_PARAM, {2 * H / 8});
    lstm.ca_w2 = add(p + "channelattention.attention.2.weight", F3_ENTRY_PARAM, {2 * H, 2 * H / 8});
    lstm.ca_b2 = add(p + "channelattention.attention.2.bias", F3_ENTRY_PARAM, {2 * H});
    lstm.fc_w = add(p + "fc.1.weight", F3_ENTRY_PARAM, {C, 2 * H});
    lstm.fc_b = add(p + "fc.1.bias", F3_ENTRY_PARAM, {C});
  }
  void add_cnn(const std::string& p, int S, int T) {
    cnn.w1 = add(p + "layer1.0.weight", F3_ENTRY_PARAM, {16, S, 5});
    cnn.b1 = add(p + "layer1.0.bias", F3_ENTRY_PARAM, {16});
    cnn.bn1 = add_bn(p + "layer1.1", 16);
    cnn.w2 = add(p + "layer2.0.weight", F3_ENTRY_PARAM, {32, 16, 5});
    cnn.b2 = add(p + "layer2.0.bias", F3_ENTRY_PARAM, {32});
    cnn.bn2 = add_bn(p + "layer2.1", 32);
    cnn.fcw = add(p + "fc.weight", F3_ENTRY_PARAM, {32, 32 * ((T / 2) / 2)});  // unused in forward
    cnn.fcb = add(p + "fc.bias", F3_ENTRY_PARAM, {32});
  }
};

namespace {

struct Arena {
  char* base;
  size_t off = 0;
  template <class T>
  T* take(size_t n) {
    off = (off + 255) & ~(size_t)255;
    T* p = base ? reinterpret_cast<T*>(base + off) : nullptr;
    off += n * sizeof(T);
    return p;
  }
};

// slab capacity: one round of resident 128x128 weight-gradient tiles (2 per CU x 256 CUs), or 16
// splits of the 256 x 256 x 9 tcn weight (wgrad_taps: 16 tiles x 16 splits = one workgroup per
// CU); the launchers cap the split count to it
// capacity of a stream's weight-gradient split-K slab (floats; the bf16x3 launches use 4x this)
constexpr long long kWgradSlabFloats = std::max(512LL * 128 * 128, 16LL * 256 * 256 * 9);

struct BnWs {
  double *fsum = nullptr, *fsq = nullptr, *bsum = nullptr, *bsq = nullptr;
};

struct LayerWs {
  const float* x = nullptr;  // block input (previous block output or data_bn output)
  float *z, *g, *h, *r = nullptr, *out, *q1, *hid, *att, *gap;
  float *gw, *gwT, *tw, *twT, *rw = nullptr, *rwT = nullptr, *aeff, *beff;
  BnWs bn1, bn2, bnr, bnca;
  float *P1, *P2, *Q2, *G, *dAeff, *dq2, *dbn, *dq1, *e;
  // bf16 mode: u = relu(bn1(g)) (tcn GEMM operand, saved for its wgrad), a bf16 copy of the
  // block output when the next block has a residual conv, the packed tcn weight gradient
  unsigned short *u = nullptr, *outb = nullptr;
  const unsigned short* xb = nullptr;  // bf16 copy of the block input (RES_CONV blocks)
  // per-layer backward tensors the side stream's weight gradients read (dh: tcn output
  // gradient, dg: gcn output gradient, dres: residual-conv output gradient): never re-used
  // by another layer, so the main stream needs no wait on the side stream before the join
  float *dh = nullptr, *dg = nullptr, *dres = nullptr;
  // per-layer partial rows of the BN1-backward node sums (G) and the graph-mix dA, reduced on
  // the side stream
  float *gpart = nullptr, *mixpart = nullptr;
  float* dbpart = nullptr;  // bf16x3: block_bwd_apply's dh / dres column-sum rows (tcn / residual bias grads)
};

struct StreamWs {
  float *x0, *pool, *A;  // A: copy of the adjacency buffer (backward has no buffer pointer)
  BnWs dbn;
  LayerWs L[7];
  float *dv, *dZ, *dx[2], *dpool;
  float* slab;  // bf16 weight-gradient split partials (see WgradArgs::slab); one per skeleton stream
  // deterministic reductions: partial rows summed in a fixed order (f3_colsum) instead of float atomics,
  // one region for the stream's main queue (pool, P1/P2/Q2, data_bn) and one for its side queue (CA weights)
  float* detm;
  float* dets;
};

struct Ws {
  StreamWs st[2];
  // sensor
  float *y1, *p1, *y2, *p2, *dy1, *dp1, *dy2, *dp2;
  BnWs cbn1, cbn2, sbn;
  float* cpart = nullptr;                          // cooperative CNN1D partial rows
  int *csyncf = nullptr, *csyncb = nullptr;        // its barrier counter + error flag (zeroed regions)
  float *seq, *gates, *cell, *hmean, *ybn, *a1, *satt, *sout, *sdy, *sdpre2, *sdpre1, *dhmean;
  float* lwpart;  // LSTM weight-gradient partial rows (LstmArgs::wpart)
  // head
  float *out, *dlogits, *ds;
  float *skel, *sensor;  // copies of the step's inputs (backward re-reads them)
  char *zf0, *zf1, *zb0, *zb1;
  const unsigned short* zero;  // 256 zero bytes (LDS-DMA GEMM padding rows)
  size_t bytes;
};

void bn_take(Arena& A, BnWs& b, int C) {
  b.fsum = A.take<double>(C);
  b.fsq = A.take<double>(C);
}
void bn_take_b(Arena& A, BnWs& b, int C) {
  b.bsum = A.take<double>(C);
  b.bsq = A.take<double>(C);
}

Ws plan(const f3_net& net, int N, char* base) {
  Ws w;
  std::memset(&w, 0, sizeof(w));
  Arena A{base};
  const int K = net.K, V = net.V;
  const bool cnn = net.has_cnn;
  const int Ts = net.cfg.sensor_frames;
  const int Tl = cnn ? (Ts / 2) / 2 : Ts;
  const bool hb = net.cfg.precision == F3_PRECISION_BF16;
  const bool x3 = net.cfg.precision == F3_PRECISION_BF16X3;
  // ---- zero-at-forward region ----
  w.zf0 = A.take<char>(0);
  w.zero = reinterpret_cast<const unsigned short*>(A.take<char>(256));
  for (int si = 0; si < net.nstreams; ++si) {
    const StreamIdx& S = net.st[si];
    StreamWs& W = w.st[si];
    bn_take(A, W.dbn, S.cin * V);
    W.pool = A.take<float>((size_t)N * 256);
    for (int l = 0; l < 7; ++l) {
      const LayerIdx& L = S.L[l];
      LayerWs& X = W.L[l];
      bn_take(A, X.bn1, L.cout);
      bn_take(A, X.bn2, L.cout);
      if (L.res == RES_CONV) bn_take(A, X.bnr, L.cout);
      bn_take(A, X.bnca, L.cout / 4);
      X.gap = A.take<float>((size_t)N * L.cout);
    }
  }
  if (net.has_sensor) {
    if (cnn) {
      bn_take(A, w.cbn1, 16);
      bn_take(A, w.cbn2, 32);
      w.csyncf = A.take<int>(f3_cnn1d_coop_sync_ints());
    }
    bn_take(A, w.sbn, 128);
  }
  w.zf1 = A.take<char>(0);
  // ---- zero-at-backward region ----
  w.zb0 = A.take<char>(0);
  for (int si = 0; si < net.nstreams; ++si) {
    const StreamIdx& S = net.st[si];
    StreamWs& W = w.st[si];
    for (int l = 0; l < 7; ++l) {
      const LayerIdx& L = S.L[l];
      LayerWs& X = W.L[l];
      bn_take_b(A, X.bn1, L.cout);
      bn_take_b(A, X.bn2, L.cout);
      if (L.res == RES_CONV) bn_take_b(A, X.bnr, L.cout);
      // [P1 | P2 | Q2] contiguous: f3_block_bwd_reduce sums their partial rows in one launch
      X.P1 = A.take<float>((size_t)3 * N * L.cout);
      X.P2 = X.P1 + (size_t)N * L.cout;
      X.Q2 = L.res == RES_CONV ? X.P1 + (size_t)2 * N * L.cout : nullptr;
      X.G = A.take<float>((size_t)V * L.cout);
      X.dAeff = A.take<float>((size_t)K * V * V);
    }
  }
  if (net.has_sensor && cnn) {
    bn_take_b(A, w.cbn1, 16);
    bn_take_b(A, w.cbn2, 32);
    w.csyncb = A.take<int>(f3_cnn1d_coop_sync_ints());
    w.dp2 = A.take<float>((size_t)N * Tl * 32);
  }
  w.zb1 = A.take<char>(0);
  // ---- saved activations, packed weights, scratch ----
  for (int si = 0; si < net.nstreams; ++si) {
    const StreamIdx& S = net.st[si];
    StreamWs& W = w.st[si];
    W.x0 = A.take<float>((size_t)N * S.T * V * S.cin);
    W.A = A.take<float>((size_t)K * V * V);
    size_t maxMC = 0, maxZ = 0;
    const float* xin = W.x0;
    const unsigned short* xinb = nullptr;
    for (int l = 0; l < 7; ++l) {
      const LayerIdx& L = S.L[l];
      LayerWs& X = W.L[l];
      const size_t Mi = (size_t)N * L.T_in * V, Mo = (size_t)N * L.T_out * V;
      const int C = L.cout, Ci = L.cin;
      // bf16x3 with the split-bf16 graph mix (Ci = 64 / 128 / 256): the gcn GEMM operands Z and dg
      // as rows [hi | lo] of 2 K Ci / 2C bf16 (the fp32 slot), the packed weights in the native form
      const bool gcat = x3 && f3_mix_x3_ok(K, V, Ci);
      X.x = xin;
      X.xb = xinb;
      X.z = gcat ? reinterpret_cast<float*>(A.take<unsigned short>(2 * Mi * K * Ci)) : A.take<float>(Mi * K * Ci);
      X.g = A.take<float>(Mi * C);
      // u = relu(bn1(g)): bf16 (bf16 mode) or rows [hi | lo] of 2C bf16 (bf16x3 mode)
      if (hb || x3) X.u = A.take<unsigned short>((x3 ? 2 : 1) * Mi * C);
      X.h = A.take<float>(Mo * C);
      if (L.res == RES_CONV) X.r = A.take<float>(Mo * C);
      X.out = A.take<float>(Mo * C);
      X.q1 = A.take<float>((size_t)N * C / 4);
      X.hid = A.take<float>((size_t)N * C / 4);
      X.att = A.take<float>((size_t)N * C);
      // packed GEMM weights: the fp32 slot (2 bf16 per weight) holds every form: fp32, bf16, the split
      // hi / lo planes, and the bf16x3 native [W_hi 32 | W_lo 32] blocks (prep code 4)
      X.gw = reinterpret_cast<float*>(A.take<unsigned short>((size_t)C * K * Ci * 2));
      X.gwT = reinterpret_cast<float*>(A.take<unsigned short>((size_t)C * K * Ci * 2));
      X.tw = reinterpret_cast<float*>(A.take<unsigned short>((size_t)C * 9 * C * 2));
      X.twT = reinterpret_cast<float*>(A.take<unsigned short>((size_t)C * 9 * C * 2));
      if (L.res == RES_CONV) {
        X.rw = reinterpret_cast<float*>(A.take<unsigned short>((size_t)C * Ci * 2));
        X.rwT = reinterpret_cast<float*>(A.take<unsigned short>((size_t)C * Ci * 2));
      }
      X.aeff = A.take<float>((size_t)K * V * V);
      X.beff = A.take<float>((size_t)V * C);
      X.dq2 = A.take<float>((size_t)N * C);
      X.dbn = A.take<float>((size_t)N * C / 4);
      X.dq1 = A.take<float>((size_t)N * C / 4);
      X.e = A.take<float>((size_t)N * C);
      X.dh = reinterpret_cast<float*>(A.take<unsigned short>(Mo * C * 2));  // x3: [hi | lo] rows
      X.dg = gcat ? reinterpret_cast<float*>(A.take<unsigned short>(2 * Mi * C)) : A.take<float>(Mi * C);
      X.gpart = A.take<float>((size_t)f3_bn_bwd_parts(N, L.T_in * V, V) * V * C);
      if (x3) X.dbpart = A.take<float>((size_t)f3_block_chunks(L.T_out * V) * N * 2 * C);
      X.mixpart = A.take<float>((size_t)kMixParts * K * V * V);
      // (bf16x3: dres as rows [hi | lo] of 2C bf16)
      if (L.res == RES_CONV) X.dres = x3 ? reinterpret_cast<float*>(A.take<unsigned short>(2 * Mo * C)) : A.take<float>(Mo * C);
      xin = X.out;
      // bf16 mode: the block output itself is stored bf16 (the next block's residual-conv operand);
      // bf16x3: a [hi | lo] copy of it when the next block has a residual conv
      xinb = hb ? reinterpret_cast<const unsigned short*>(X.out) : nullptr;
      if (x3 && l < 6 && S.L[l + 1].res == RES_CONV) xinb = X.outb = A.take<unsigned short>(2 * Mo * C);
      maxMC = std::max(maxMC, std::max(Mi * C, Mi * Ci));
      maxMC = std::max(maxMC, Mo * C);
      maxZ = std::max(maxZ, Mi * K * Ci);
    }

    W.dv = A.take<float>(maxMC);
    W.slab = A.take<float>(kWgradSlabFloats * (x3 ? 4 : 1));  // x3: [2C][9][2C] partials

    W.dZ = A.take<float>(maxZ);
    W.dx[0] = A.take<float>(maxMC);
    W.dx[1] = A.take<float>(maxMC);
    W.dpool = A.take<float>((size_t)N * 256);
    {  // partial-row regions (see StreamWs::detm / dets)
      size_t m = (size_t)((S.T * V + 95) / 96) * N * 256;  // pool partials of the last block
      size_t d = 0;
      for (int l = 0; l < 7; ++l) {
        const LayerIdx& L = S.L[l];
        const size_t ch = (size_t)(L.T_out * V + 95) / 96;  // f3_block_* chunks per clip
        m = std::max(m, 3 * ch * N * L.cout);
        d = std::max(d, (size_t)((N + 7) / 8) * (2 * (L.cout / 4) * L.cout + L.cout));
      }
      m = std::max(m, (size_t)((N * S.T + 31) / 32) * 2 * V * S.cin);  // data_bn gamma / beta partials
      W.detm = A.take<float>(m);
      W.dets = A.take<float>(d);
    }
  }
  if (net.has_sensor) {
    if (cnn) {
      w.y1 = A.take<float>((size_t)N * Ts * 16);
      w.p1 = A.take<float>((size_t)N * (Ts / 2) * 16);
      w.y2 = A.take<float>((size_t)N * (Ts / 2) * 32);
      w.p2 = A.take<float>((size_t)N * Tl * 32);
      w.dy1 = A.take<float>((size_t)N * Ts * 16);
      w.dp1 = A.take<float>((size_t)N * (Ts / 2) * 16);
      w.dy2 = A.take<float>((size_t)N * (Ts / 2) * 32);
      w.cpart = A.take<float>(f3_cnn1d_coop_part_floats(N, net.cfg.sensor_dim, 16, 32));
    }
    w.seq = A.take<float>((size_t)N * Tl * 128);
    w.gates = A.take<float>((size_t)2 * N * Tl * 256);
    w.cell = A.take<float>((size_t)2 * N * Tl * 64);
    w.lwpart = A.take<float>((size_t)2 * ((N + LSTM_NB - 1) / LSTM_NB) * 256 * (1 + (net.has_cnn ? 32 : net.lstm.S) + 64));
    w.hmean = A.take<float>((size_t)N * 128);
    w.ybn = A.take<float>((size_t)N * 128);
    w.a1 = A.take<float>((size_t)N * 16);
    w.satt = A.take<float>((size_t)N * 128);
    w.sout = A.take<float>((size_t)N * net.lstm.Cs);
    w.sdy = A.take<float>((size_t)N * 128);
    w.sdpre2 = A.take<float>((size_t)N * 128);
    w.sdpre1 = A.take<float>((size_t)N * 16);
    w.dhmean = A.take<float>((size_t)N * 128);
    w.ds = A.take<float>((size_t)N * net.lstm.Cs);
  }
  if (net.nstreams) w.skel = A.take<float>((size_t)N * 3 * net.cfg.frames * V);
  if (net.has_sensor) w.sensor = A.take<float>((size_t)N * Ts * net.cfg.sensor_dim);
  w.out = A.take<float>((size_t)N * net.cfg.num_class);
  w.dlogits = A.take<float>((size_t)N * net.cfg.num_class);
  w.bytes = (A.off + 255) & ~(size_t)255;
  return w;
}

struct Ptrs {
  const f3_net& net;
  const float* P;
  float* B;
  int64_t* C;
  float* G;
  // f3_net_backward_rmsprop: RMSprop(lr, alpha, eps) on params / square_avg, each skeleton layer's
  // range issued on the queue that finishes its gradients (opt_p == null: no fused update)
  float* opt_p = nullptr;
  float* opt_sq = nullptr;
  float lr = 0.f, alpha = 0.f, eps = 0.f;
  const float* p(int i) const { return P + net.entries[i].offset; }
  float* g(int i) const { return G + net.entries[i].offset; }
  float* b(int i) const { return B + net.entries[i].offset; }
  long long* c(int i) const { return reinterpret_cast<long long*>(C + net.entries[i].offset); }
  BnRef ref(const BnIdx& bi, const BnWs& w, float count, int eval) const {
    BnRef r;
    r.sum = w.fsum;
    r.sumsq = w.fsq;
    r.gamma = p(bi.w);
    r.beta = p(bi.b);
    r.rmean = B ? b(bi.rm) : nullptr;
    r.rvar = B ? b(bi.rv) : nullptr;
    r.count = count;
    r.eval = eval;
    return r;
  }
};


ConvGeom geom(int M, int Nc, int Kc, int KT, int S, int P, int tr, int T_out, int T_in, int V, int lda, int ldo) {
  ConvGeom g;
  g.M = M; g.Nc = Nc; g.Kc = Kc; g.KT = KT; g.S = S; g.P = P; g.transposed = tr;
  g.T_out = T_out; g.T_in = T_in; g.V = V; g.lda = lda; g.ldo = ldo;
  return g;
}

void add_job(PrepTable& t, int type, int n, float* dst, const float* s0, const float* s1, const float* s2, int d0,
             int d1, int d2, int bf16 = 0) {
  PrepJob& j = t.jobs[t.n++];
  j.type = type; j.n = n; j.dst = dst; j.s0 = s0; j.s1 = s1; j.s2 = s2; j.d0 = d0; j.d1 = d1; j.d2 = d2;
  j.bf16 = bf16;
}

// bf16 view of a packed operand (the fp32-sized slot holds the bf16 copy in bf16 mode)
inline const unsigned short* bf(const float* p, int on) { return on ? reinterpret_cast<const unsigned short*>(p) : nullptr; }
// bf16x3 mode (F3_PRECISION_BF16X3, the default): fp32 activations as in the fp32 mode; GEMM operands
// as bf16 rows [x_hi | x_lo] written by their producers and weights packed per tap in 32-channel
// blocks [W_hi | W_lo] (prep code 4), three bf16 MFMA products per block (x3_gemm below)
inline int is_x3(const f3_net& n) { return n.cfg.precision == F3_PRECISION_BF16X3; }
// Side-queue weight gradients of layers >= 2 are split for 75 % of the chip's workgroup slots, so the
// main chains running beside them keep CUs (a whole-chip wgrad_big grid holds every CU's LDS until it
// drains: the main queues sat idle 190-335 us behind the layer-5 weight gradient,
// profiles/r04_x3_step_timeline.txt); layers 0-1 (the step's tail, main chains done) keep the whole
// chip. Measured (bf16x3 step): 10.17 -> 10.07 ms at 50 or 75 %, flat over 50-90 % and the first split
// layer 0-2 (profiles/r04_ntw_ab.txt, r04_frac_ab.txt)
inline int side_pct(bool split, int l) { return split && l >= 2 ? 75 : 0; }
// bf16x3: the first block's gcn (Cin = 3: a 9-column GEMM, too narrow for the bf16 implicit-GEMM kernels)
// runs on layer0.hip's fused kernels in their fp32 form (mix + GEMM + bias + BN1 sums in one pass;
// backward dZ, dx, dA and dW partials in one pass): 10.14 -> 9.92 ms/step against the generic mix +
// split GEMMs (profiles/r04_gcn0_x3_ab.txt)
// bf16x3 GEMMs on the bf16 kernels in the native form (ConvGemmArgs::x3n, prep code 4: [x_hi | x_lo]
// rows staged once, three MFMAs per 32-channel block). The round-4 K-concatenated form (Kc = 3C,
// [W_hi | W_hi | W_lo], the third K segment re-staging x_hi) measured 8 % slower per step (9.97-10.02
// vs 9.11-9.12 ms, profiles/r05_x3n_ab.txt) and is gone.
constexpr int x3code() { return 4; }
// packed size (bf16 elements) of n weights in a prep code
inline int x3mul(int code) { return code == 4 ? 2 : 1; }
// set a bf16x3 GEMM on [hi | lo] rows of C channels (lda 2C)
inline void x3_gemm(ConvGemmArgs& a, int C) {
  a.x3n = 1;
  a.g.lda = 2 * C;
}

// prep code of the packed GEMM weights: 0 fp32, 1 bf16, 2 split hi / lo planes
inline int wcode(const f3_net& n) { return n.cfg.precision == F3_PRECISION_BF16 ? 1 : is_x3(n) ? 2 : 0; }
// bf16 view of an activation slot (bf16 mode stores GEMM operand tensors as bf16)
inline unsigned short* bfa(float* p, int on) { return on ? reinterpret_cast<unsigned short*>(p) : nullptr; }

void add_bnrun(BnRunTable& t, const Ptrs& q, const BnIdx& bi, const double* sum, const double* sq, double count) {
  BnRunJob& j = t.jobs[t.n++];
  j.sum = sum; j.sumsq = sq; j.count = count; j.C = bi.C;
  j.rmean = q.b(bi.rm); j.rvar = q.b(bi.rv); j.nbt = q.c(bi.nbt);
}

// Forward of one skeleton stream in stages: stage -1 = weight prep + data_bn, stage l = block l.
// The caller interleaves the two streams' stages so both branch queues are fed from the start
// (host submission, eager or graph replay, walks the launches in issue order).
int stream_forward_layer(const f3_net& net, int si, int N, int train, const Ptrs& q, Ws& w, BnRunTable& run,
                         hipStream_t s, int l);

int stream_forward(const f3_net& net, int si, int N, int train, const Ptrs& q, Ws& w, const float* skel,
                   BnRunTable& run, hipStream_t s, int stage) {
  if (stage >= 0) return stream_forward_layer(net, si, N, train, q, w, run, s, stage);
  const StreamIdx& S = net.st[si];
  StreamWs& W = w.st[si];
  const int K = net.K, V = net.V, eval = !train;
  const int hb = net.cfg.precision == F3_PRECISION_BF16;
  const int wc = wcode(net);
  // weights: A_eff, gcn bias through the graph, packed GEMM operands
  PrepTable pt;
  pt.n = 0;
  add_job(pt, PREP_COPY, K * V * V, W.A, q.b(S.A), nullptr, nullptr, 0, 0, 0);
  for (int l = 0; l < 7; ++l) {
    const LayerIdx& L = S.L[l];
    LayerWs& X = W.L[l];
    const int C = L.cout, Ci = L.cin;
    add_job(pt, PREP_MUL, K * V * V, X.aeff, q.b(S.A), q.p(L.edge), nullptr, 0, 0, 0);
    add_job(pt, PREP_GCN_BIAS, V * C, X.beff, q.b(S.A), q.p(L.edge), q.p(L.gcn_b), C, V, K);
    // bf16x3 with the split-bf16 mix: native-form gcn weights (code 4) for the bf16 kernels
    const bool l0f = wc == 2 && f3_gcn0_ok(K, V, Ci, C);  // fp32 weights (layer0.hip)
    // bf16x3: the bf16 implicit-GEMM kernels' packing (native [hi 32 | lo 32] blocks, code 4)
    const int xc = wc == 2 ? x3code() : wc;
    const int gc = wc == 2 && f3_mix_x3_ok(K, V, Ci) ? xc : (l0f ? 0 : wc);
    add_job(pt, PREP_PACK_GCN, C * K * Ci * x3mul(gc), X.gw, q.p(L.gcn_w), nullptr, nullptr, C, Ci, K, gc);
    add_job(pt, PREP_PACK_CONV, C * 9 * C * x3mul(xc), X.tw, q.p(L.tcn_w), nullptr, nullptr, C, C, 9, xc);
    if (train) {
      add_job(pt, PREP_PACK_GCN_T, C * K * Ci * x3mul(gc), X.gwT, q.p(L.gcn_w), nullptr, nullptr, C, Ci, K, gc);
      add_job(pt, PREP_PACK_CONV_T, C * 9 * C * x3mul(xc), X.twT, q.p(L.tcn_w), nullptr, nullptr, C, C, 9, xc);
    }
    if (L.res == RES_CONV) {
      add_job(pt, PREP_PACK_CONV, C * Ci * x3mul(xc), X.rw, q.p(L.res_w), nullptr, nullptr, C, Ci, 1, xc);
      if (train) add_job(pt, PREP_PACK_CONV_T, C * Ci * x3mul(xc), X.rwT, q.p(L.res_w), nullptr, nullptr, C, Ci, 1, xc);
    }
  }
  F3_TRY(f3_prep(pt, s));
  // data_bn
  DataBnArgs d;
  std::memset(&d, 0, sizeof(d));
  d.N = N; d.T = S.T; d.V = V; d.C = S.cin; d.motion = S.motion; d.skel = skel; d.out = W.x0;
  d.bn = q.ref(S.dbn, W.dbn, (float)(N * S.T), eval);
  d.st_sum = W.dbn.fsum; d.st_sq = W.dbn.fsq;
  d.act16 = hb;  // bf16 mode: activations stored bf16
  F3_TRY(f3_databn_fwd(&d, s));
  if (train) add_bnrun(run, q, S.dbn, W.dbn.fsum, W.dbn.fsq, (double)N * S.T);
  return F3_OK;
}

int stream_forward_layer(const f3_net& net, int si, int N, int train, const Ptrs& q, Ws& w, BnRunTable& run,
                         hipStream_t s, int l) {
  const StreamIdx& S = net.st[si];
  StreamWs& W = w.st[si];
  const int K = net.K, V = net.V, eval = !train;
  const int hb = net.cfg.precision == F3_PRECISION_BF16;
  const int x3 = is_x3(net), wq = hb || x3;
  {
    const LayerIdx& L = S.L[l];
    LayerWs& X = W.L[l];
    const int C = L.cout, Ci = L.cin, Ti = L.T_in, To = L.T_out;
    const int Mi = N * Ti * V, Mo = N * To * V;
    const BnRef bn1 = q.ref(L.bn1, X.bn1, (float)Mi, eval);
    const BnRef bn2 = q.ref(L.bn2, X.bn2, (float)Mo, eval);
    BnRef bnr;
    std::memset(&bnr, 0, sizeof(bnr));
    if (L.res == RES_CONV) bnr = q.ref(L.bnr, X.bnr, (float)Mo, eval);
    // graph mix then 1x1 conv (stgcan.py:50-56)
    if ((hb || x3) && f3_gcn0_ok(K, V, Ci, C)) {  // the 3-channel first block: one kernel (layer0.hip)
      Gcn0Args g0;
      std::memset(&g0, 0, sizeof(g0));
      g0.frames = N * Ti; g0.K = K; g0.V = V; g0.Ci = Ci; g0.A = X.aeff;
      g0.x = reinterpret_cast<const unsigned short*>(X.x); g0.w = bf(X.gw, 1); g0.beff = X.beff;
      g0.z = bfa(X.z, 1); g0.g = bfa(X.g, 1); g0.st_sum = X.bn1.fsum; g0.st_sq = X.bn1.fsq;
      g0.f32 = x3;  // bf16x3: fp32 x / w / Z / g behind the same pointers
      F3_TRY(f3_gcn0_fwd(&g0, s));
    } else {
      MixArgs mx;
      std::memset(&mx, 0, sizeof(mx));
      mx.K = K; mx.V = V; mx.Cin = Ci; mx.frames = N * Ti; mx.A = X.aeff; mx.x = X.x; mx.z = X.z;
      mx.zb = bfa(X.z, hb); mx.x16 = hb; mx.x3 = x3;
      const bool gcat = x3 && f3_mix_x3_ok(K, V, Ci);
      mx.z3 = bfa(X.z, gcat);
      F3_TRY(f3_mix_fwd(&mx, s));
      ConvGemmArgs ga;
      std::memset(&ga, 0, sizeof(ga));
      ga.g = geom(Mi, C, K * Ci, 1, 1, 0, 0, Ti, Ti, V, K * Ci, C);
      ga.in = hb ? nullptr : X.z; ga.inb = bfa(X.z, hb); ga.zero = w.zero;
      ga.w = X.gw; ga.wb = bf(X.gw, wq); ga.out = X.g; ga.outb = bfa(X.g, hb); ga.x3 = x3;
      ga.bias = X.beff; ga.st_sum = X.bn1.fsum; ga.st_sq = X.bn1.fsq;
      if (gcat) {  // the [Z_hi | Z_lo] rows of K Ci channels on the bf16 kernels
        ga.x3 = 0; ga.in = nullptr; ga.inb = bfa(X.z, 1);
        x3_gemm(ga, K * Ci);
      }
      F3_TRY(f3_conv_gemm(&ga, 0, EPI_BIASV | EPI_STATS, s));
    }
    if (L.res == RES_CONV) {  // residual conv (stgcan.py:128-131)
      ConvGemmArgs ra;
      std::memset(&ra, 0, sizeof(ra));
      ra.g = geom(Mo, C, Ci, 1, L.stride, 0, 0, To, Ti, V, Ci, C);
      ra.in = hb ? nullptr : X.x; ra.inb = hb ? X.xb : nullptr; ra.zero = w.zero;
      if (hb && !X.xb) return F3_ESTATE;
      ra.w = X.rw; ra.wb = bf(X.rw, wq); ra.out = X.r; ra.outb = bfa(X.r, hb); ra.x3 = x3;
      ra.bias = q.p(L.res_b); ra.st_sum = X.bnr.fsum; ra.st_sq = X.bnr.fsq;
      if (x3) {  // the previous block's [x_hi | x_lo] copy
        if (!X.xb) return F3_ESTATE;
        ra.x3 = 0; ra.in = nullptr; ra.inb = X.xb;
        x3_gemm(ra, Ci);
      }
      F3_TRY(f3_conv_gemm(&ra, 0, EPI_BIAS | EPI_STATS, s));
    }
    // tcn: BN1 + ReLU prologue, (9,1) conv, bias, BN2 stats + channel-attention pool epilogue
    ConvGemmArgs ta;
    std::memset(&ta, 0, sizeof(ta));
    ta.g = geom(Mo, C, C, 9, L.stride, 4, 0, To, Ti, V, C, C);
    ta.w = X.tw; ta.wb = bf(X.tw, wq); ta.out = X.h; ta.outb = bfa(X.h, hb); ta.bias = q.p(L.tcn_b);
    ta.st_sum = X.bn2.fsum; ta.st_sq = X.bn2.fsq; ta.gap = X.gap;
    if (hb || x3) {  // materialise u = relu(bn1(g)) once (also the tcn wgrad operand): bf16, or
      // (bf16x3) rows [u_hi | u_lo | u_hi] against the packed [W_hi | W_hi | W_lo]: the bf16 LDS-DMA
      // implicit-GEMM kernels then compute u_hi W_hi + u_lo W_hi + u_hi W_lo over K = 9 x 3C
      BnReluArgs br;
      std::memset(&br, 0, sizeof(br));
      br.M = Mi; br.C = C; br.bn = bn1; br.g = X.g; br.u = X.u; br.g16 = hb; br.x3 = x3;
      F3_TRY(f3_bnrelu_bf16(&br, s));
      if (x3) x3_gemm(ta, C);
      ta.inb = X.u; ta.zero = w.zero;
      F3_TRY(f3_conv_gemm(&ta, 0, EPI_BIAS | EPI_STATS | EPI_GAP, s));
    } else {
      ta.in = X.g; ta.pro_bn = bn1;
      F3_TRY(f3_conv_gemm(&ta, 1, EPI_BIAS | EPI_STATS | EPI_GAP, s));
    }
    // channel attention (stgcan.py:59-74)
    CaArgs ca;
    std::memset(&ca, 0, sizeof(ca));
    ca.N = N; ca.C = C; ca.inv_tv = 1.f / (float)(To * V); ca.bn2 = bn2;
    ca.bnca = q.ref(L.bnca, X.bnca, (float)N, eval);
    ca.W1 = q.p(L.ca_w1); ca.b1 = q.p(L.ca_b1); ca.W2 = q.p(L.ca_w2); ca.b2 = q.p(L.ca_b2);
    ca.gapsum = X.gap; ca.q1 = X.q1; ca.hid = X.hid; ca.att = X.att; ca.ca_sum = X.bnca.fsum; ca.ca_sq = X.bnca.fsq;
    F3_TRY(f3_ca_fwd(&ca, s));
    // residual add + ReLU (stgcan.py:143-144), pooled mean after the last block (stgcan.py:224)
    BlockArgs ba;
    std::memset(&ba, 0, sizeof(ba));
    ba.N = N; ba.TV = To * V; ba.C = C; ba.res_kind = L.res; ba.inv_tv = 1.f / (float)(To * V);
    ba.bn2 = bn2; ba.bnr = bnr; ba.h = X.h; ba.r = X.r; ba.x = X.x; ba.att = X.att; ba.out = X.out;
    ba.pool = l == 6 ? W.pool : nullptr;
    ba.part = W.detm;
    ba.act16 = hb;
    if (x3 && X.outb) { ba.outb = X.outb; ba.x3 = 1; }
    F3_TRY(f3_block_out(ba, s));
    if (train) {
      add_bnrun(run, q, L.bn1, X.bn1.fsum, X.bn1.fsq, Mi);
      add_bnrun(run, q, L.bn2, X.bn2.fsum, X.bn2.fsq, Mo);
      if (L.res == RES_CONV) add_bnrun(run, q, L.bnr, X.bnr.fsum, X.bnr.fsq, Mo);
      add_bnrun(run, q, L.bnca, X.bnca.fsum, X.bnca.fsq, N);
    }
  }
  return F3_OK;
}

// The flat-parameter ranges of one skeleton layer: [gcn.conv.weight .. channel_attention ... 4.bias]
// (contiguous: entries are laid out in creation order within a phase group, 16-B aligned) and its
// edge_importance entry (created after the stream's layers).
RmsRanges layer_ranges(const f3_net& n, const LayerIdx& L) {
  RmsRanges r;
  r.n = 2;
  const Entry &a = n.entries[L.gcn_w], &b = n.entries[L.ca_b2], &e = n.entries[L.edge];
  r.lo[0] = a.offset;
  r.len[0] = b.offset + (b.numel + 3) / 4 * 4 - a.offset;
  r.lo[1] = e.offset;
  r.len[1] = (e.numel + 3) / 4 * 4;
  return r;
}

// debugging aid: F3_DEBUG_BWD_STOP="stream,layer" ends the backward right after that
// layer's tcn input-gradient so its scratch tensors can be inspected (f3_net_debug_tensor)
bool debug_stop(int si, int l) {
  static const char* e = getenv("F3_DEBUG_BWD_STOP");
  if (!e) return false;
  int a = -1, b = -1;
  sscanf(e, "%d,%d", &a, &b);
  return a == si && b == l;
}

// Backward of layers l_hi..l_lo (descending); data_bn after layer 0. Layer l writes its
// input gradient to W.dx[(6-l)&1] and reads layer l+1's from W.dx[(5-l)&1].
// Main stream s: the chain that carries the input gradient down the layers. Side stream ss
// (== s when not parallel): the layer's weight gradients (tcn / gcn / residual wgrad, gcn
// bias + edge importance), which nothing downstream waits for. Layer l's side work starts after
// ev_main[si][l]. It reads only
// per-layer tensors, so the only side -> main edge is the final join. (Main also waiting on the side stream per layer — double-buffered scratch —
// made HIP's stream-capture end fault on ROCm 7.2.)
int stream_backward(const f3_net& net, int si, int N, const Ptrs& q, Ws& w, const float* skel, hipStream_t s,
                    int l_hi, int l_lo, hipStream_t ss = nullptr, int call_hi = 6, int part = 3) {
  if (!ss) ss = s;
  (void)call_hi;
  const bool split = ss != s;
  const StreamIdx& S = net.st[si];
  StreamWs& W = w.st[si];
  const int K = net.K, V = net.V;
  const int hb = net.cfg.precision == F3_PRECISION_BF16;
  const int x3 = is_x3(net), wq = hb || x3;
  const float* dout = l_hi == 6 ? nullptr : W.dx[(5 - l_hi) & 1];
  int pp = (6 - l_hi) & 1;
  for (int l = l_hi; l >= l_lo; --l) {
    const LayerIdx& L = S.L[l];
    LayerWs& X = W.L[l];
    const int C = L.cout, Ci = L.cin, Ti = L.T_in, To = L.T_out;
    const int Mi = N * Ti * V, Mo = N * To * V;
    float* dx = W.dx[pp];
    float* const dh = X.dh;
    float* const dg = X.dg;
    float* const dres = X.dres;
    ColsumJob cj[kColsumJobs];  // side-queue column sums, launched together before the gcn bias step
    int ncj = 0;
    const BnRef bn1 = q.ref(L.bn1, X.bn1, (float)Mi, 0);
    const BnRef bn2 = q.ref(L.bn2, X.bn2, (float)Mo, 0);
    BnRef bnr;
    std::memset(&bnr, 0, sizeof(bnr));
    if (L.res == RES_CONV) bnr = q.ref(L.bnr, X.bnr, (float)Mo, 0);
    BlockArgs ba;
    std::memset(&ba, 0, sizeof(ba));
    ba.N = N; ba.TV = To * V; ba.C = C; ba.res_kind = L.res; ba.inv_tv = 1.f / (float)(To * V);
    ba.bn2 = bn2; ba.bnr = bnr; ba.h = X.h; ba.r = X.r; ba.x = X.x; ba.att = X.att; ba.out = X.out;
    ba.dout = dout; ba.dout_nc = l == 6 ? W.dpool : nullptr; ba.act16 = hb;
    ba.P1 = X.P1; ba.P2 = X.P2; ba.Q2 = X.Q2; ba.bnr_bsum = X.bnr.bsum; ba.bnr_bsq = X.bnr.bsq;
    ba.bn2_bsum = X.bn2.bsum; ba.bn2_bsq = X.bn2.bsq; ba.e = X.e; ba.dh = dh;
    ba.dres = L.res == RES_CONV ? dres : (L.res == RES_ID ? dx : nullptr);
    ba.dhb = bfa(dh, hb || x3);  // bf16x3: dh as split hi / lo planes (the tcn dgrad / wgrad operand)
    ba.x3 = x3;
    ba.dresb = L.res == RES_CONV ? bfa(dres, hb || x3) : nullptr;  // bf16x3: [hi | lo] rows
    ba.dgamma2 = q.g(L.bn2.w); ba.dbeta2 = q.g(L.bn2.b);
    if (L.res == RES_CONV) { ba.dgammar = q.g(L.bnr.w); ba.dbetar = q.g(L.bnr.b); }
    ba.part = W.detm;
    // the block sums P1 / P2 / Q2 summed by ca_bwd1x from the partial rows (one launch less per layer)
    const bool ca_sums = f3_ca_x_ok(N, C, To * V);
    ba.no_colsum = ca_sums;
    if (part & 1) F3_TRY(f3_block_bwd_reduce(ba, s));
    ba.no_colsum = 0;
    ba.dbpart = x3 ? X.dbpart : nullptr;  // (block_bwd_apply only: the bias-gradient rows)
    CaArgs ca;
    std::memset(&ca, 0, sizeof(ca));
    ca.N = N; ca.C = C; ca.inv_tv = 1.f / (float)(To * V); ca.bn2 = bn2;
    ca.bnca = q.ref(L.bnca, X.bnca, (float)N, 0);
    ca.W1 = q.p(L.ca_w1); ca.b1 = q.p(L.ca_b1); ca.W2 = q.p(L.ca_w2); ca.b2 = q.p(L.ca_b2);
    ca.gapsum = X.gap; ca.q1 = X.q1; ca.hid = X.hid; ca.att = X.att; ca.ca_sum = X.bnca.fsum; ca.ca_sq = X.bnca.fsq;
    ca.P1 = X.P1; ca.P2 = X.P2; ca.dq2 = X.dq2; ca.dbn = X.dbn; ca.dq1 = X.dq1; ca.e = X.e;
    ca.Q2 = X.Q2; ca.bnr_bsum = L.res == RES_CONV ? X.bnr.bsum : nullptr; ca.bnr_bsq = L.res == RES_CONV ? X.bnr.bsq : nullptr;
    ca.bn2_bsum = X.bn2.bsum; ca.bn2_bsq = X.bn2.bsq;
    ca.g_bnca_gamma = q.g(L.bnca.w); ca.g_bnca_beta = q.g(L.bnca.b);
    ca.g_b1 = q.g(L.ca_b1); ca.g_W1 = q.g(L.ca_w1); ca.g_W2 = q.g(L.ca_w2); ca.g_b2 = q.g(L.ca_b2);
    if (ca_sums) { ca.bpart = W.detm; ca.bchunks = f3_block_chunks(To * V); }
    if (part & 1) F3_TRY(f3_ca_bwd(&ca, s));  // the W1/W2 gradients (ca_bwd_w) go to the side stream
    if (part & 1) F3_TRY(f3_block_bwd_apply(ba, s));
    // (Starting the tcn / residual / CA weight gradients right after block_bwd_apply instead of after
    // the layer's whole main chain measured slower, 5.69 vs 5.54 ms/step, profiles/r03_side_early_ab.txt:
    // the side work then takes CUs from the main chain, the step's critical path.)
    // tcn input gradient (transposed conv) with ReLU mask + BN1-backward sums
    ConvGemmArgs td;
    std::memset(&td, 0, sizeof(td));
    td.g = geom(Mi, C, C, 9, L.stride, 4, 1, Ti, To, V, C, C);
    td.in = (hb || x3) ? nullptr : dh; td.inb = bfa(dh, hb || x3); td.zero = w.zero;
    td.w = X.twT; td.wb = bf(X.twT, wq); td.out = W.dv; td.aux = X.g; td.ldaux = C; td.epi_bn = bn1;
    if (x3) x3_gemm(td, C);  // dh rows [hi | lo]
    td.outb = bfa(W.dv, hb); td.auxb = hb ? reinterpret_cast<const unsigned short*>(X.g) : nullptr;
    td.st_sum = X.bn1.bsum; td.st_sq = X.bn1.bsq;
    if (part & 1) F3_TRY(f3_conv_gemm(&td, 0, EPI_RELUMASK, s));
    if (debug_stop(si, l)) return F3_OK;
    BnBwdArgs bb;
    std::memset(&bb, 0, sizeof(bb));
    bb.N = N; bb.TV = Ti * V; bb.C = C; bb.V = V; bb.bn = bn1; bb.bsum = X.bn1.bsum; bb.bsq = X.bn1.bsq;
    bb.dgamma = q.g(L.bn1.w); bb.dbeta = q.g(L.bn1.b); bb.dv = W.dv; bb.g = X.g; bb.dg = dg; bb.G = X.G;
    bb.Gpart = X.gpart; bb.dgb = bfa(dg, hb); bb.act16 = hb; bb.no_colsum = split;
    const bool gcat = x3 && f3_mix_x3_ok(K, V, Ci);  // dg as [hi | lo] rows (see plan)
    if (gcat) { bb.dgb = bfa(dg, 1); bb.x3 = 1; }
    if (part & 1) F3_TRY(f3_bn_bwd_apply(bb, s));
    // gcn: dZ = dg W^T ; dW ; mix^T ; bias/edge grads
    const bool g0 = (hb || x3) && f3_gcn0_ok(K, V, Ci, C);  // the 3-channel first block (layer0.hip)
    Gcn0Args b0;
    std::memset(&b0, 0, sizeof(b0));
    int g0_parts = 0;
    if (g0) {
      b0.frames = N * Ti; b0.K = K; b0.V = V; b0.Ci = Ci; b0.A = X.aeff;
      b0.x = reinterpret_cast<const unsigned short*>(X.x); b0.w = bf(X.gw, 1); b0.z = bfa(X.z, 1);
      b0.dg = bfa(dg, 1); b0.dx = dx; b0.accumulate = L.res == RES_ID;
      b0.f32 = x3;  // bf16x3: fp32 x / w / Z / dg
      g0_parts = f3_gcn0_bwd_parts(&b0);
      if ((size_t)g0_parts * (K * V * V + K * C * Ci) > (size_t)kMixParts * K * V * V) return F3_EINVAL;
      b0.part_dA = X.mixpart;
      b0.part_dW = X.mixpart + (size_t)g0_parts * K * V * V;
    }
    ConvGemmArgs gd;
    std::memset(&gd, 0, sizeof(gd));
    gd.g = geom(Mi, K * Ci, C, 1, 1, 0, 0, Ti, Ti, V, C, K * Ci);
    gd.in = hb ? nullptr : dg; gd.inb = bfa(dg, hb); gd.zero = w.zero;
    gd.w = X.gwT; gd.wb = bf(X.gwT, wq); gd.x3 = x3; gd.out = W.dZ;
    if (gcat) {  // dg rows [hi | lo]
      gd.x3 = 0; gd.in = nullptr; gd.inb = bfa(dg, 1);
      x3_gemm(gd, C);
    }
    const bool dzb = hb && f3_mix_lds_ok(K, V, Ci);  // bf16 dZ feeds the LDS graph-mix backward
    if (dzb) {
      if (!f3_igemm_ok(gd)) return F3_EINVAL;
      gd.outb = bfa(W.dZ, 1);
    }
    if ((part & 1) && !g0) F3_TRY(f3_conv_gemm(&gd, 0, 0, s));
    MixArgs mx;
    std::memset(&mx, 0, sizeof(mx));
    mx.K = K; mx.V = V; mx.Cin = Ci; mx.frames = N * Ti; mx.A = X.aeff; mx.x = X.x; mx.z = W.dZ;
    mx.dx = dx; mx.dA = X.dAeff; mx.accumulate = L.res == RES_ID; mx.part = X.mixpart; mx.x16 = hb;
    mx.no_colsum = split; mx.x3 = x3;
    mx.dzb = dzb ? bfa(W.dZ, 1) : nullptr;
    if (part & 1) F3_TRY(g0 ? f3_gcn0_bwd(&b0, s) : f3_mix_bwd(&mx, s));
    if (L.res == RES_CONV) {
      ConvGemmArgs rd;
      std::memset(&rd, 0, sizeof(rd));
      rd.g = geom(Mi, Ci, C, 1, L.stride, 0, 1, Ti, To, V, C, Ci);
      rd.in = hb ? nullptr : dres; rd.inb = bfa(dres, hb); rd.zero = w.zero;
      rd.w = X.rwT; rd.wb = bf(X.rwT, wq); rd.x3 = x3; rd.out = dx;
      if (x3) {  // dres rows [hi | lo]
        rd.x3 = 0; rd.in = nullptr; rd.inb = bfa(dres, 1);
        x3_gemm(rd, C);
      }
      if (part & 1) F3_TRY(f3_conv_gemm(&rd, 0, EPI_ADD, s));
    }
    // ---- side stream: this layer's weight gradients ----
    if (split && (part & 1) && hipEventRecord(net.ev_main[si][l], s) != hipSuccess) return F3_EHIP;
    if (split && (part & 2) && hipStreamWaitEvent(ss, net.ev_main[si][l], 0) != hipSuccess) return F3_EHIP;
    WgradArgs tw;
    std::memset(&tw, 0, sizeof(tw));
    tw.wg_pct = side_pct(split, l);
    tw.g = geom(Mo, C, C, 9, L.stride, 4, 0, To, Ti, V, C, C);
    tw.ldy = C; tw.dw = q.g(L.tcn_w); tw.db = q.g(L.tcn_b);
    tw.outmap = WG_OUT_CONV; tw.bf16 = hb; tw.x3 = x3;
    if (hb) {  // bf16 operands dh, u; split partials in the stream's slab, summed into the grads
      tw.dyb = bfa(dh, 1); tw.inb = X.u; tw.zero = w.zero;
      tw.slab = W.slab; tw.slab_cap = kWgradSlabFloats; tw.dw_ref = q.g(L.tcn_w);
      if (!f3_wgrad_glds_ok(tw)) return F3_EINVAL;
      if (part & 2) F3_TRY(f3_conv_wgrad(&tw, 0, ss));
    } else if (x3) {  // on the bf16 kernels over the [hi | lo] rows of dh and u: three row segments
      // (dh_hi u_hi, dh_lo u_hi, dh_hi u_lo). (One GEMM on [dh_hi | dh_lo] x [u_hi | u_lo] whose
      // quadrants a fold adds computes the unused lo*lo quadrant too: 11.31 vs 10.78 ms/step.)
      tw.x3 = 0; tw.bf16 = 1;
      tw.ldy = 2 * C; tw.dyb = bfa(dh, 1); tw.inb = X.u; tw.zero = w.zero;
      tw.slab = W.slab; tw.slab_cap = kWgradSlabFloats * 4; tw.dw_ref = q.g(L.tcn_w);
      tw.g = geom(Mo, C, C, 9, L.stride, 4, 0, To, Ti, V, 2 * C, C);
      tw.x3seg = 1;
      tw.db = nullptr;  // the bias gradient from block_bwd_apply's dh rows (colsum below)
      if (!f3_wgrad_glds_ok(tw)) return F3_EINVAL;
      if (part & 2) F3_TRY(f3_conv_wgrad(&tw, 0, ss));
      if (part & 2) {
        const int rows = f3_block_chunks(To * V) * N;
        cj[ncj++] = {X.dbpart, q.g(L.tcn_b), 2LL * C, rows, C};
        if (L.res == RES_CONV) cj[ncj++] = {X.dbpart + C, q.g(L.res_b), 2LL * C, rows, C};
      }
    } else {
      tw.dy = dh; tw.in = X.g; tw.pro_bn = bn1;
      if (part & 2) F3_TRY(f3_conv_wgrad(&tw, 1, ss));
    }
    ca.wpart = W.dets;
    if (part & 2) F3_TRY(f3_ca_bwd_weights(&ca, ss, cj, &ncj));
    if (L.res == RES_CONV) {
      WgradArgs rw;
      std::memset(&rw, 0, sizeof(rw));
      rw.wg_pct = side_pct(split, l);
      rw.g = geom(Mo, C, Ci, 1, L.stride, 0, 0, To, Ti, V, Ci, C);
      rw.ldy = C; rw.dw = q.g(L.res_w); rw.db = q.g(L.res_b); rw.outmap = WG_OUT_CONV; rw.bf16 = hb; rw.x3 = x3;
      if (hb) {
        rw.dyb = bfa(dres, 1); rw.inb = X.xb; rw.zero = w.zero;
        rw.slab = W.slab; rw.slab_cap = kWgradSlabFloats; rw.dw_ref = q.g(L.res_w);
      } else if (x3) {  // row segments as the tcn's
        rw.x3 = 0; rw.bf16 = 1;
        rw.ldy = 2 * C; rw.dyb = bfa(dres, 1); rw.inb = X.xb; rw.zero = w.zero;
        rw.slab = W.slab; rw.slab_cap = kWgradSlabFloats * 4; rw.dw_ref = q.g(L.res_w);
        rw.g = geom(Mo, C, Ci, 1, L.stride, 0, 0, To, Ti, V, 2 * Ci, C);
        rw.x3seg = 1;
        rw.db = nullptr;  // summed from block_bwd_apply's dres rows with the tcn bias
        if (!f3_wgrad_glds_ok(rw)) return F3_EINVAL;
      } else {
        rw.dy = dres; rw.in = X.x;
      }
      if (part & 2) F3_TRY(f3_conv_wgrad(&rw, 0, ss));
    }
    if (split) {  // reductions whose results only feed weight gradients
      const int T = L.T_in, fch = f3_bn_bwd_parts(N, T * V, V);
      if (part & 2) cj[ncj++] = {X.gpart, X.G, (long long)V * C, fch, V * C};
      const int mparts = g0 ? 0 : f3_mix_bwd_parts(&mx);
      if (mparts && (part & 2)) cj[ncj++] = {X.mixpart, X.dAeff, (long long)K * V * V, mparts, K * V * V};
    }
    if (g0 && (part & 2)) {  // the first block's dA_eff and gcn weight gradient partial rows
      cj[ncj++] = {b0.part_dA, X.dAeff, (long long)K * V * V, g0_parts, K * V * V};
      cj[ncj++] = {b0.part_dW, q.g(L.gcn_w), (long long)K * C * Ci, g0_parts, K * C * Ci};
    }
    // this layer's side-queue column sums (attention weights, tcn / residual biases, BN G, dA_eff,
    // layer-0 gcn rows) as one launch; each job's summation order is that of its own f3_colsum
    if (ncj > kColsumJobs) return F3_EINVAL;
    F3_TRY(f3_colsum_multi(cj, ncj, ss));
    ncj = 0;
    WgradArgs gw;
    std::memset(&gw, 0, sizeof(gw));
    gw.wg_pct = side_pct(split, l);
    gw.g = geom(Mi, C, K * Ci, 1, 1, 0, 0, Ti, Ti, V, K * Ci, C);
    gw.ldy = C; gw.dw = q.g(L.gcn_w); gw.db = nullptr;
    if (hb) {
      gw.dyb = bfa(dg, 1); gw.inb = bfa(X.z, 1); gw.zero = w.zero;
    } else {
      gw.dy = dg; gw.in = X.z;
    }
    gw.outmap = WG_OUT_GCN; gw.gcn_cin = Ci; gw.bf16 = hb; gw.x3 = x3;
    if (gcat) {  // row segments into the slab, reduced into the gcn layout
      gw.x3 = 0; gw.bf16 = 1; gw.outmap = WG_OUT_CONV;
      gw.ldy = 2 * C; gw.dyb = bfa(dg, 1); gw.inb = bfa(X.z, 1); gw.zero = w.zero; gw.dy = nullptr; gw.in = nullptr;
      gw.slab = W.slab; gw.slab_cap = kWgradSlabFloats * 4; gw.dw_ref = q.g(L.gcn_w); gw.dw = nullptr;
      gw.g = geom(Mi, C, K * Ci, 1, 1, 0, 0, Ti, Ti, V, 2 * K * Ci, C);
      gw.x3seg = 1;
      if (!f3_wgrad_glds_ok(gw)) return F3_EINVAL;
    }
    if ((part & 2) && !g0) F3_TRY(f3_conv_wgrad(&gw, 0, ss));
    GcnBiasBwdArgs gb;
    gb.K = K; gb.V = V; gb.C = C; gb.Aeff = X.aeff; gb.A = W.A; gb.G = X.G; gb.bias = q.p(L.gcn_b);
    gb.db = q.g(L.gcn_b); gb.dAeff = X.dAeff; gb.dE = q.g(L.edge);
    if (part & 2) F3_TRY(f3_gcn_bias_bwd(&gb, ss));
    // fused optimizer: every gradient of this layer is final here on ss (its main-chain parts were
    // waited for through ev_main), and nothing later in the backward reads these parameters
    if (q.opt_p && (part & 2))
      F3_TRY(f3_rmsprop_ranges(q.opt_p, q.opt_sq, q.G, layer_ranges(net, L), q.lr, q.alpha, q.eps, 1.f, ss));
    dout = dx;
    pp ^= 1;
  }
  if (l_lo > 0) return F3_OK;
  DataBnArgs d;
  std::memset(&d, 0, sizeof(d));
  d.N = N; d.T = S.T; d.V = V; d.C = S.cin; d.motion = S.motion; d.skel = skel;
  d.bn = q.ref(S.dbn, W.dbn, (float)(N * S.T), 0);
  d.dout = dout; d.dgamma = q.g(S.dbn.w); d.dbeta = q.g(S.dbn.b);
  d.part = W.detm;
  if (part & 1) {  // the coalesced single-pass data_bn gradient where its shape fits, else the per-channel one
    const int st = f3_databn_bwd2(&d, s);
    if (st == F3_EINVAL) F3_TRY(f3_databn_bwd(&d, s));
    else if (st != F3_OK) return st;
  }
  return F3_OK;
}

void sensor_args(const f3_net& net, int N, int train, const Ptrs& q, Ws& w, const float* sensor, LstmArgs& la,
                 SHeadArgs& sa, Conv1dArgs& c1, Conv1dArgs& c2) {
  const int Ts = net.cfg.sensor_frames;
  const int eval = !train;
  std::memset(&la, 0, sizeof(la));
  std::memset(&sa, 0, sizeof(sa));
  std::memset(&c1, 0, sizeof(c1));
  std::memset(&c2, 0, sizeof(c2));
  if (net.has_cnn) {
    c1.N = N; c1.T = Ts; c1.Ci = net.cfg.sensor_dim; c1.Co = 16; c1.x = sensor; c1.w = q.p(net.cnn.w1);
    c1.b = q.p(net.cnn.b1); c1.y = w.y1; c1.st_sum = w.cbn1.fsum; c1.st_sq = w.cbn1.fsq;
    c1.bn = q.ref(net.cnn.bn1, w.cbn1, (float)(N * Ts), eval); c1.p = w.p1;
    c1.dp = w.dp1; c1.dy = w.dy1; c1.bsum = w.cbn1.bsum; c1.bsq = w.cbn1.bsq;
    c1.g_gamma = q.G ? q.g(net.cnn.bn1.w) : nullptr; c1.g_beta = q.G ? q.g(net.cnn.bn1.b) : nullptr;
    c1.g_b = q.G ? q.g(net.cnn.b1) : nullptr; c1.g_w = q.G ? q.g(net.cnn.w1) : nullptr; c1.dx = nullptr;
    c2 = c1;
    c2.T = Ts / 2; c2.Ci = 16; c2.Co = 32; c2.x = w.p1; c2.w = q.p(net.cnn.w2); c2.b = q.p(net.cnn.b2);
    c2.y = w.y2; c2.st_sum = w.cbn2.fsum; c2.st_sq = w.cbn2.fsq;
    c2.bn = q.ref(net.cnn.bn2, w.cbn2, (float)(N * (Ts / 2)), eval); c2.p = w.p2;
    c2.dp = w.dp2; c2.dy = w.dy2; c2.bsum = w.cbn2.bsum; c2.bsq = w.cbn2.bsq;
    c2.g_gamma = q.G ? q.g(net.cnn.bn2.w) : nullptr; c2.g_beta = q.G ? q.g(net.cnn.bn2.b) : nullptr;
    c2.g_b = q.G ? q.g(net.cnn.b2) : nullptr; c2.g_w = q.G ? q.g(net.cnn.w2) : nullptr; c2.dx = w.dp1;
  }
  la.N = N;
  la.T = net.has_cnn ? (Ts / 2) / 2 : Ts;
  la.S = net.has_cnn ? 32 : net.lstm.S;
  la.x = net.has_cnn ? w.p2 : sensor;
  for (int d = 0; d < 2; ++d) {
    la.w_ih[d] = q.p(net.lstm.wih[d]); la.w_hh[d] = q.p(net.lstm.whh[d]);
    la.b_ih[d] = q.p(net.lstm.bih[d]); la.b_hh[d] = q.p(net.lstm.bhh[d]);
    if (q.G) {
      la.g_w_ih[d] = q.g(net.lstm.wih[d]); la.g_w_hh[d] = q.g(net.lstm.whh[d]);
      la.g_b_ih[d] = q.g(net.lstm.bih[d]); la.g_b_hh[d] = q.g(net.lstm.bhh[d]);
      la.wpart = w.lwpart;
    }
  }
  la.seq = w.seq; la.gates = w.gates; la.cell = w.cell; la.hmean = w.hmean;
  la.dhmean = w.dhmean; la.dx = net.has_cnn ? w.dp2 : nullptr;
  sa.N = N; sa.Cs = net.lstm.Cs; sa.hmean = w.hmean;
  sa.bn = q.ref(net.lstm.bn, w.sbn, (float)N, eval); sa.bn_sum = w.sbn.fsum; sa.bn_sq = w.sbn.fsq;
  sa.W1 = q.p(net.lstm.ca_w1); sa.b1 = q.p(net.lstm.ca_b1); sa.W2 = q.p(net.lstm.ca_w2); sa.b2 = q.p(net.lstm.ca_b2);
  sa.W3 = q.p(net.lstm.fc_w); sa.b3 = q.p(net.lstm.fc_b);
  sa.ybn = w.ybn; sa.a1 = w.a1; sa.att = w.satt; sa.out = w.sout; sa.out_ld = net.lstm.Cs;
  sa.dout = w.ds; sa.dout_ld = net.lstm.Cs; sa.dy = w.sdy; sa.dpre2 = w.sdpre2; sa.dpre1 = w.sdpre1;
  sa.dhmean = w.dhmean;
  if (q.G) {
    sa.g_W1 = q.g(net.lstm.ca_w1); sa.g_b1 = q.g(net.lstm.ca_b1); sa.g_W2 = q.g(net.lstm.ca_w2);
    sa.g_b2 = q.g(net.lstm.ca_b2); sa.g_W3 = q.g(net.lstm.fc_w); sa.g_b3 = q.g(net.lstm.fc_b);
    sa.g_gamma = q.g(net.lstm.bn.w); sa.g_beta = q.g(net.lstm.bn.b);
  }
}

void head_args(const f3_net& net, int N, const Ptrs& q, Ws& w, HeadArgs& h) {
  std::memset(&h, 0, sizeof(h));
  h.N = N;
  h.C = net.cfg.num_class;
  h.softmax_out = net.cfg.softmax_output;
  h.out = w.out;
  h.dlogits = w.dlogits;
  const int m = net.cfg.model;
  if (m == F3_MODEL_STGCN) {
    h.nblk = 1;
    h.feat[0] = w.st[0].pool; h.width[0] = 256; h.ld[0] = 256; h.dfeat[0] = w.st[0].dpool;
    h.W = q.p(net.st[0].cls_w); h.b = q.p(net.st[0].cls_b);
    if (q.G) { h.g_W = q.g(net.st[0].cls_w); h.g_b = q.g(net.st[0].cls_b); }
  } else if (m == F3_MODEL_BILSTM) {
    h.nblk = 0;
  } else {
    h.nblk = net.has_sensor ? 3 : 2;
    for (int i = 0; i < 2; ++i) {
      h.feat[i] = w.st[i].pool; h.width[i] = 256; h.ld[i] = 256; h.dfeat[i] = w.st[i].dpool;
    }
    if (net.has_sensor) {
      h.feat[2] = w.sout; h.width[2] = net.lstm.Cs; h.ld[2] = net.lstm.Cs; h.dfeat[2] = w.ds;
    }
    h.W = q.p(net.fc_w); h.b = q.p(net.fc_b);
    if (q.G) { h.g_W = q.g(net.fc_w); h.g_b = q.g(net.fc_b); }
  }
}

// flags of the events that fork / join the branch queues. They order work between queues of ONE
// device, so a device-scope release is all they need (hipEventRecord's default is a system-scope
// fence: L2 writeback + invalidate at every record; 5.56-5.57 -> 5.55-5.56 ms/step,
// profiles/r03_event_scope_ab.txt).
static unsigned branch_event_flags() { return hipEventDisableTiming | hipEventReleaseToDevice; }

// Private branch streams, created on the first eager call (never during a capture: there the
// branches stay on the caller's stream). F3_SERIAL=1 keeps everything on one stream.
bool ensure_parallel(f3_net& n, hipStream_t s) {
  if (n.par_init) return n.par_ok;
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  if (hipStreamIsCapturing(s, &cs) != hipSuccess || cs != hipStreamCaptureStatusNone) {
    (void)hipGetLastError();
    return false;
  }
  n.par_init = true;
  if (getenv("F3_SERIAL")) return n.par_ok = false;
  const unsigned evf = branch_event_flags();
  bool ok = true;
  // (the side queues at the lowest or highest stream priority measured within noise, r04_queue_ab.txt)
  for (int i = 0; i < 3; ++i) ok = ok && hipStreamCreateWithFlags(&n.aux[i], hipStreamNonBlocking) == hipSuccess;
  for (auto& e : n.ev) ok = ok && hipEventCreateWithFlags(&e, evf) == hipSuccess;
  for (auto& e : n.ev_p1) ok = ok && hipEventCreateWithFlags(&e, evf) == hipSuccess;
  for (int i = 0; i < 2; ++i)
    for (int l = 0; l < 7; ++l) {
      ok = ok && hipEventCreateWithFlags(&n.ev_main[i][l], evf) == hipSuccess;
    }
  (void)hipGetLastError();
  return n.par_ok = ok;
}

// Fork `k` branch streams off s (they see all work queued on s so far) / join them back.
// Only the branch streams that will receive work are forked (mask bit i = aux[i]): a
// forked-but-empty branch in a stream capture breaks HIP graph instantiation.
enum : int { BR_MOTION = 1, BR_SENSOR = 2, BR_SIDE = 4 };
struct Branches {
  f3_net& n;
  hipStream_t s;
  bool par;
  int mask = BR_MOTION | BR_SENSOR | BR_SIDE;
  hipStream_t at(int i) const { return par && i > 0 && (mask >> (i - 1) & 1) ? n.aux[i - 1] : s; }
  hipStream_t side() const { return par && (mask & BR_SIDE) ? n.aux[2] : s; }
  // weight-gradient queue of skeleton stream si: the motion stream's goes to the sensor queue,
  // idle once the (short) sensor backward is done, so the two streams' weight gradients drain
  // in parallel at the end of the backward instead of one after the other on aux[2]
  hipStream_t side(int si) const {
    return si == 1 && par && (mask & BR_SIDE) && (mask & BR_SENSOR) ? n.aux[1] : side();
  }
  int fork() {
    if (!par || !mask) return F3_OK;
    if (hipEventRecord(n.ev[0], s) != hipSuccess) return F3_EHIP;
    for (int i = 0; i < 3; ++i)
      if ((mask >> i & 1) && hipStreamWaitEvent(n.aux[i], n.ev[0], 0) != hipSuccess) return F3_EHIP;
    return F3_OK;
  }
  int join() {
    if (!par) return F3_OK;
    for (int i = 0; i < 3; ++i) {
      if (!(mask >> i & 1)) continue;
      if (hipEventRecord(n.ev[1 + i], n.aux[i]) != hipSuccess) return F3_EHIP;
      if (hipStreamWaitEvent(s, n.ev[1 + i], 0) != hipSuccess) return F3_EHIP;
    }
    return F3_OK;
  }
  // end of backward phase 1: record where every queue is instead of joining them into s. Under
  // stream capture the queues are joined instead: a capture must end with every forked queue
  // joined back, and events recorded inside one capture are not re-recorded by its replay (the
  // caller orders its all-reduce after the replaying stream, train.py TrainStep.__call__).
  int mark_phase1() {
    n.p1_mask = 0;
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    if (hipStreamIsCapturing(s, &cs) != hipSuccess) return F3_EHIP;
    if (cs != hipStreamCaptureStatusNone) return join();
    for (auto& e : n.ev_p1)  // (serial mode never created the branch events)
      if (!e && hipEventCreateWithFlags(&e, branch_event_flags()) != hipSuccess) return F3_EHIP;
    for (int i = 0; i < 3 && par; ++i) {
      if (!(mask >> i & 1)) continue;
      if (hipEventRecord(n.ev_p1[i], n.aux[i]) != hipSuccess) return F3_EHIP;
      n.p1_mask |= 1 << i;
    }
    if (hipEventRecord(n.ev_p1[3], s) != hipSuccess) return F3_EHIP;
    n.p1_mask |= 8;
    return F3_OK;
  }
};

// stream `t` waits for everything backward phase 1 queued (no-op after a serial phase 1, whose
// work is all on the caller's stream)
int wait_phase1(f3_net& n, hipStream_t t) {
  for (int i = 0; i < 4; ++i)
    if ((n.p1_mask >> i & 1) && hipStreamWaitEvent(t, n.ev_p1[i], 0) != hipSuccess) return F3_EHIP;
  return F3_OK;
}

}  // namespace

// ============================================================================
// C ABI
// ============================================================================
extern "C" {

int f3_net_create(const f3_config* cfg, f3_net** out) {
  if (!cfg || !out) return F3_EINVAL;
  if (cfg->num_node < 2 || cfg->num_partition < 1 || cfg->num_class < 1 || cfg->num_class > 64) return F3_EINVAL;
  if (cfg->frames < 2 || cfg->model < 0 || cfg->model > 3) return F3_EINVAL;
  if (cfg->num_partition * cfg->num_node * cfg->num_node > 1024) return F3_EINVAL;
  if (cfg->precision != F3_PRECISION_FP32 && cfg->precision != F3_PRECISION_BF16 &&
      cfg->precision != F3_PRECISION_BF16X3)
    return F3_EINVAL;  // not 2 (kernel-level entries only)
  f3_net* n = new f3_net();
  n->cfg = *cfg;
  n->K = cfg->num_partition;
  n->V = cfg->num_node;
  const bool nb = cfg->naming == F3_NAMING_NOTEBOOK;
  const std::string p1 = nb ? "pts_stream." : "stgcan_1.", p2 = nb ? "mot_stream." : "stgcan_2.";
  const std::string ps = nb ? "sensor." : "lstm.", pf = nb ? "fcn." : "fc.";
  const int Cs = cfg->sensor_classes > 0 ? cfg->sensor_classes : cfg->num_class;
  switch (cfg->model) {
    case F3_MODEL_STGCN:
      n->nstreams = 1;
      n->add_stream(n->st[0], "", cfg->in_channels, 0, cfg->num_class);
      break;
    case F3_MODEL_BILSTM:
      n->has_sensor = true;
      if (cfg->sensor == F3_SENSOR_CNN_BILSTM) {  // sensor-only CNN_BiLSTM (GSTCAN_UR_sensor.ipynb:572-586)
        n->has_cnn = true;
        n->add_cnn("cnn.", cfg->sensor_dim, cfg->sensor_frames);
        n->add_bilstm("bilstm.", 32, cfg->num_class);
        break;
      }
      if (cfg->sensor_dim > 32) { delete n; return F3_EINVAL; }
      n->add_bilstm("", cfg->sensor_dim, cfg->num_class);
      break;
    default: {
      n->nstreams = 2;
      n->add_stream(n->st[0], p1, 3, 0, 0);
      n->add_stream(n->st[1], p2, 2, 1, 0);
      const bool sens = cfg->model == F3_MODEL_TWO_STGCAN_BILSTM;
      n->has_sensor = sens;
      n->has_cnn = sens && cfg->sensor == F3_SENSOR_CNN_BILSTM;
      if (sens && !n->has_cnn && cfg->sensor_dim > 32) { delete n; return F3_EINVAL; }
      auto add_sensor = [&]() {
        if (!sens) return;
        if (n->has_cnn) {
          n->add_cnn(ps + "cnn.", cfg->sensor_dim, cfg->sensor_frames);
          n->add_bilstm(ps + "bilstm.", 32, Cs);
        } else {
          n->add_bilstm(ps, cfg->sensor_dim, Cs);
        }
      };
      auto add_fc = [&]() {
        n->fc_w = n->add(pf + "weight", F3_ENTRY_PARAM, {cfg->num_class, 512 + (sens ? Cs : 0)});
        n->fc_b = n->add(pf + "bias", F3_ENTRY_PARAM, {cfg->num_class});
      };
      if (nb) { add_fc(); add_sensor(); } else { add_sensor(); add_fc(); }
    }
  }
  n->finalize_offsets();
  *out = n;
  return F3_OK;
}

void f3_net_destroy(f3_net* net) { delete net; }

int f3_net_num_entries(const f3_net* net) { return net ? (int)net->entries.size() : 0; }

int f3_net_entry(const f3_net* net, int i, const char** name, int* kind, int* ndim, int64_t* shape8, int64_t* offset) {
  if (!net || i < 0 || i >= (int)net->entries.size()) return F3_EINVAL;
  const Entry& e = net->entries[i];
  if (name) *name = e.name.c_str();
  if (kind) *kind = e.kind;
  if (ndim) *ndim = (int)e.shape.size();
  if (shape8) for (size_t d = 0; d < e.shape.size() && d < 8; ++d) shape8[d] = e.shape[d];
  if (offset) *offset = e.offset;
  return F3_OK;
}

int64_t f3_net_param_count(const f3_net* net) { return net ? net->nparam : 0; }
int64_t f3_net_buffer_count(const f3_net* net) { return net ? net->nbuf : 0; }
int64_t f3_net_counter_count(const f3_net* net) { return net ? net->ncnt : 0; }

int64_t f3_net_workspace_bytes(const f3_net* net, int batch) {
  if (!net || batch < 1) return 0;
  return (int64_t)plan(*net, batch, nullptr).bytes;
}

int f3_net_forward(f3_net* net, int N, int training, const float* params, float* buffers, int64_t* counters,
                   const float* skel, const float* sensor, float* out, void* workspace, void* stream) {
  if (!net || !params || !buffers || !out || !workspace || N < 1) return F3_EINVAL;
  if (training && N < 2) return F3_EBATCH;
  F3_TRY(net->cstatus.take(false));
  hipStream_t s = (hipStream_t)stream;
  Ws w = plan(*net, N, (char*)workspace);
  Ptrs q{*net, params, buffers, counters, nullptr};
  if (training && !counters) return F3_EINVAL;
  if (hipMemsetAsync(w.zf0, 0, w.zf1 - w.zf0, s) != hipSuccess) return F3_EHIP;
  if (net->nstreams) {
    if (!skel) return F3_EINVAL;
    if (hipMemcpyAsync(w.skel, skel, sizeof(float) * N * 3 * net->cfg.frames * net->V, hipMemcpyDeviceToDevice, s) !=
        hipSuccess)
      return F3_EHIP;
  }
  if (net->has_sensor) {
    if (!sensor) return F3_EINVAL;
    if (hipMemcpyAsync(w.sensor, sensor, sizeof(float) * N * net->cfg.sensor_frames * net->cfg.sensor_dim,
                       hipMemcpyDeviceToDevice, s) != hipSuccess)
      return F3_EHIP;
  }
  BnRunTable run;
  run.n = 0;
  Branches br{*net, s, ensure_parallel(*net, s)};
  br.mask = (net->nstreams > 1 ? BR_MOTION : 0) | (net->has_sensor ? BR_SENSOR : 0);
  F3_TRY(br.fork());
  // the skeleton streams' weight prep + data_bn first (the motion stream's queue waited ~130 us for
  // the host to submit the sensor branch ahead of it), then the sensor branch (small, latency-bound),
  // then the skeleton streams stage by stage, interleaved, so every branch queue is fed early
  for (int si = 0; si < net->nstreams; ++si)
    F3_TRY(stream_forward(*net, si, N, training, q, w, w.skel, run, br.at(si), -1));
  if (net->has_sensor) {
    const hipStream_t ss = br.at(2);
    LstmArgs la;
    SHeadArgs sa;
    Conv1dArgs c1, c2;
    sensor_args(*net, N, training, q, w, w.sensor, la, sa, c1, c2);
    if (net->has_cnn) {
      const CnnCoop coop{w.cpart, w.csyncf};
      net->smark(0, ss);
      F3_TRY(f3_cnn1d_fwd(&c1, &c2, &coop, ss));
      net->smark(1, ss);
      if (training) F3_TRY(net->cstatus.post(w.csyncf, ss));
      if (training) {
        add_bnrun(run, q, net->cnn.bn1, w.cbn1.fsum, w.cbn1.fsq, (double)N * net->cfg.sensor_frames);
        add_bnrun(run, q, net->cnn.bn2, w.cbn2.fsum, w.cbn2.fsq, (double)N * (net->cfg.sensor_frames / 2));
      }
    }
    F3_TRY(f3_lstm_fwd(&la, ss));
    F3_TRY(f3_shead_fwd(&sa, ss));
    if (training) add_bnrun(run, q, net->lstm.bn, w.sbn.fsum, w.sbn.fsq, N);
  }
  for (int stage = 0; stage < 7; ++stage)
    for (int si = 0; si < net->nstreams; ++si)
      F3_TRY(stream_forward(*net, si, N, training, q, w, w.skel, run, br.at(si), stage));
  F3_TRY(br.join());
  HeadArgs h;
  head_args(*net, N, q, w, h);
  if (net->cfg.model == F3_MODEL_BILSTM) {
    if (hipMemcpyAsync(w.out, w.sout, sizeof(float) * N * net->cfg.num_class, hipMemcpyDeviceToDevice, s) != hipSuccess)
      return F3_EHIP;
    if (hipMemcpyAsync(out, w.out, sizeof(float) * N * net->cfg.num_class, hipMemcpyDeviceToDevice, s) != hipSuccess)
      return F3_EHIP;
  } else {
    h.out2 = out;  // the head writes the caller's copy itself
    F3_TRY(f3_head_fwd(&h, s));
  }
  if (training) F3_TRY(f3_bn_running(run, s));
  return F3_OK;
}

int f3_net_loss(f3_net* net, int N, const float* out, const float* label, float* loss, float* dout, void* stream) {
  if (!net || !out || !label || !loss || !dout) return F3_EINVAL;
  hipStream_t s = (hipStream_t)stream;
  // (f3_ce stores the loss; larger batches zero it and accumulate)
  HeadArgs h;
  std::memset(&h, 0, sizeof(h));
  h.N = N; h.C = net->cfg.num_class; h.out = const_cast<float*>(out); h.label = label; h.loss = loss; h.dout = dout;
  return f3_ce(&h, s);
}

int f3_net_backward(f3_net* net, int N, const float* params, const float* dout, float* grads, void* workspace,
                    void* stream) {
  return f3_net_backward_phase(net, N, params, dout, grads, workspace, 0, stream);
}

int64_t f3_net_grad_split(const f3_net* net) { return net ? net->nparam_phase1 : 0; }

}  // extern "C"

namespace {
struct FusedOpt {
  float *p, *sq;
  float lr, alpha, eps;
};

int net_backward(f3_net* net, int N, const float* params, const float* dout, float* grads, void* workspace, int phase,
                 void* stream, const FusedOpt* opt);

// the skeleton layers' ranges cover exactly their own parameter entries (the fused optimizer's
// per-layer launches rely on it; checked once per call, ~300 entries)
bool layer_ranges_ok(const f3_net& n) {
  for (int si = 0; si < n.nstreams; ++si)
    for (int l = 0; l < 7; ++l) {
      const LayerIdx& L = n.st[si].L[l];
      const RmsRanges r = layer_ranges(n, L);
      long long sum = 0;
      for (int i = L.gcn_w; i <= L.ca_b2; ++i) {
        const Entry& e = n.entries[i];
        if (e.kind != F3_ENTRY_PARAM) continue;
        if (e.offset < r.lo[0] || e.offset >= r.lo[0] + r.len[0]) return false;
        sum += (e.numel + 3) / 4 * 4;
      }
      if (sum != r.len[0]) return false;
    }
  return true;
}

// f3_net_backward_rmsprop's plan: whether the per-layer updates apply (a layout whose layer entries are
// not contiguous cannot be updated per layer) and the leftover ranges updated after the join
void fused_opt_plan(f3_net& n) {
  n.fused_opt = layer_ranges_ok(n);
  n.rest_ranges.clear();
  if (!n.fused_opt) return;
  std::vector<std::pair<long long, long long>> done, rest;
  for (int si = 0; si < n.nstreams; ++si)
    for (int l = 0; l < 7; ++l) {
      const RmsRanges r = layer_ranges(n, n.st[si].L[l]);
      for (int j = 0; j < r.n; ++j) done.push_back({r.lo[j], r.lo[j] + r.len[j]});
    }
  for (const Entry& e : n.entries) {
    if (e.kind != F3_ENTRY_PARAM) continue;
    bool in = false;
    for (auto& d : done) in = in || (e.offset >= d.first && e.offset < d.second);
    if (in) continue;
    const long long lo = e.offset, hi = e.offset + (e.numel + 3) / 4 * 4;
    if (!rest.empty() && rest.back().second == lo) rest.back().second = hi;
    else rest.push_back({lo, hi});
  }
  RmsRanges r;
  r.n = 0;
  for (size_t i = 0; i < rest.size(); ++i) {
    r.lo[r.n] = rest[i].first;
    r.len[r.n] = rest[i].second - rest[i].first;
    if (++r.n == kRmsRanges || i + 1 == rest.size()) {
      n.rest_ranges.push_back(r);
      r.n = 0;
    }
  }
}
}  // namespace

extern "C" {

int f3_net_backward_rmsprop(f3_net* net, int N, float* params, const float* dout, float* grads, float* square_avg,
                            void* workspace, float lr, float alpha, float eps, void* stream) {
  if (!net || !params || !square_avg) return F3_EINVAL;
  hipStream_t s = (hipStream_t)stream;
  // (a layout without contiguous per-layer ranges: one update after the backward, as f3_net_backward +
  // f3_rmsprop_step)
  if (net->fused_opt < 0) fused_opt_plan(*net);
  if (!net->fused_opt) {
    F3_TRY(net_backward(net, N, params, dout, grads, workspace, 0, stream, nullptr));
    return f3_rmsprop(params, square_avg, grads, net->nparam, lr, alpha, eps, 1.f, s);
  }
  const FusedOpt o{params, square_avg, lr, alpha, eps};
  F3_TRY(net_backward(net, N, params, dout, grads, workspace, 0, stream, &o));
  // every parameter outside the layers' ranges (data_bn, sensor branch, head), after the join
  for (const RmsRanges& r : net->rest_ranges)
    F3_TRY(f3_rmsprop_ranges(params, square_avg, grads, r, lr, alpha, eps, 1.f, s));
  return F3_OK;
}

int f3_net_fused_rmsprop(f3_net* net) {
  if (!net) return -1;
  if (net->fused_opt < 0) fused_opt_plan(*net);
  return net->fused_opt;
}

int f3_net_precision(const f3_net* net) { return net ? net->cfg.precision : -1; }

int f3_net_status(f3_net* net, int wait) {
  if (!net) return F3_EINVAL;
  return net->cstatus.take(wait != 0);
}

int f3_net_backward_phase(f3_net* net, int N, const float* params, const float* dout, float* grads, void* workspace,
                          int phase, void* stream) {
  return net_backward(net, N, params, dout, grads, workspace, phase, stream, nullptr);
}

}  // extern "C"

namespace {
int net_backward(f3_net* net, int N, const float* params, const float* dout, float* grads, void* workspace, int phase,
                 void* stream, const FusedOpt* opt) {
  if (!net || !params || !grads || !workspace || N < 2 || phase < 0 || phase > 2) return F3_EINVAL;
  if (phase != 2 && !dout) return F3_EINVAL;
  F3_TRY(net->cstatus.take(false));
  if (opt && phase != 0) return F3_EINVAL;
  hipStream_t s = (hipStream_t)stream;
  Ws w = plan(*net, N, (char*)workspace);
  Ptrs q{*net, params, nullptr, nullptr, grads};
  if (opt) {
    q.opt_p = opt->p; q.opt_sq = opt->sq; q.lr = opt->lr; q.alpha = opt->alpha; q.eps = opt->eps;
  }
  // skeleton streams layer by layer, interleaved (see stream_forward)
  // after_first: called once the first layer's main chains are submitted (the sensor backward, so its
  // host submission does not hold back the skeleton streams' first layer)
  auto skeleton = [&](Branches& br, int l_hi, int l_lo, const std::function<int()>& after_first) -> int {
    // Each layer's main chains are submitted before the previous layer's side-stream work (the
    // weight gradients): the host can be held up submitting to the long side queue, and the
    // main queues should already hold their next layer by then (neutral in time since the side
    // split, kept: it removed 150-490 us idle stretches of the main queues before it)
    const bool defer = br.side() != br.s;
    // Every layer's weight gradients run on the side queues. (A former F3_TAIL_SIDE=0 option ran
    // layer 0's on the stream's own queue: measured neutral to 1 % slower, and it raced with the
    // side queue's layer-1 launch on the stream's shared split-K slab, so it is gone.)
    auto side_of = [&](int si, int) { return br.side(si); };
    for (int l = l_hi; l >= l_lo; --l) {
      for (int si = 0; si < net->nstreams; ++si) {
        F3_TRY(stream_backward(*net, si, N, q, w, w.skel, br.at(si), l, l, side_of(si, l), l_hi,
                               defer ? 1 : 3));
        if (debug_stop(si, l)) return F3_OK;  // leave the scratch as is for f3_net_debug_tensor
      }
      if (l == l_hi && after_first) F3_TRY(after_first());
      if (defer && l < l_hi)
        for (int si = 0; si < net->nstreams; ++si)
          F3_TRY(stream_backward(*net, si, N, q, w, w.skel, br.at(si), l + 1, l + 1, side_of(si, l + 1),
                                 l_hi, 2));
    }
    if (defer)
      for (int si = 0; si < net->nstreams; ++si)
        F3_TRY(stream_backward(*net, si, N, q, w, w.skel, br.at(si), l_lo, l_lo, side_of(si, l_lo), l_hi, 2));
    return F3_OK;
  };
  if (phase == 2) {
    Branches br{*net, s, ensure_parallel(*net, s)};
    // the same queue assignment as phase 1 (mask incl. the sensor queue, which carries the motion
    // stream's weight gradients): a stream's split-K slab is then only ever used from one queue,
    // so phase 2's weight gradients cannot overlap phase 1's still-draining ones on that slab
    br.mask = (net->nstreams > 1 ? BR_MOTION : 0) | (net->has_sensor ? BR_SENSOR : 0) |
              (net->nstreams > 0 ? BR_SIDE : 0);
    F3_TRY(br.fork());
    F3_TRY(skeleton(br, kSplitLayer - 1, 0, nullptr));
    F3_TRY(br.join());
    F3_TRY(wait_phase1(*net, s));  // phase 1's queues (e.g. the sensor queue) are done too
    net->p1_mask = 0;
    return F3_OK;
  }
  // the gradient buffer and the backward's zeroed workspace block: one launch when both are float
  // ranges on 16-byte boundaries (the usual case), else two memsets
  const size_t zb = w.zb1 - w.zb0;
  if (zb % 4 == 0 && ((uintptr_t)grads | (uintptr_t)w.zb0) % 16 == 0) {
    F3_TRY(f3_zero2(grads, net->nparam, reinterpret_cast<float*>(w.zb0), (long long)(zb / 4), s));
  } else {
    if (hipMemsetAsync(grads, 0, sizeof(float) * net->nparam, s) != hipSuccess) return F3_EHIP;
    if (hipMemsetAsync(w.zb0, 0, zb, s) != hipSuccess) return F3_EHIP;
  }
  HeadArgs h;
  head_args(*net, N, q, w, h);
  h.g_out = dout;
  LstmArgs la;
  SHeadArgs sa;
  Conv1dArgs c1, c2;
  if (net->has_sensor) sensor_args(*net, N, 1, q, w, w.sensor, la, sa, c1, c2);
  if (net->cfg.model == F3_MODEL_BILSTM) {
    sa.dout = dout;
    sa.dout_ld = net->cfg.num_class;
  } else {
    F3_TRY(f3_head_bwd_data(&h, s));  // dlogits + feature gradients: what the streams' backward waits for
  }
  Branches br{*net, s, ensure_parallel(*net, s)};
  br.mask = (net->nstreams > 1 ? BR_MOTION : 0) | (net->has_sensor ? BR_SENSOR : 0) | (net->nstreams > 0 ? BR_SIDE : 0);
  F3_TRY(br.fork());
  // the head Linear's weight gradients off the critical path, at the front of the side queue (which
  // then waits for the first layer's data gradients anyway)
  if (net->cfg.model != F3_MODEL_BILSTM) F3_TRY(f3_head_bwd_weight(&h, br.side()));
  auto sensor_bwd = [&]() -> int {
    if (!net->has_sensor) return F3_OK;
    const hipStream_t ss = br.at(2);
    F3_TRY(f3_shead_bwd(&sa, ss));
    F3_TRY(f3_lstm_bwd(&la, ss));
    if (net->has_cnn) {
      const CnnCoop coop{w.cpart, w.csyncb};
      net->smark(2, ss);
      F3_TRY(f3_cnn1d_bwd(&c1, &c2, &coop, ss));
      net->smark(3, ss);
      F3_TRY(net->cstatus.post(w.csyncb, ss));
    }
    return F3_OK;
  };
  // the skeleton streams' first layer is submitted before the sensor backward; a sensor-only model has
  // no skeleton layer to wait for
  if (net->nstreams == 0) F3_TRY(sensor_bwd());
  F3_TRY(skeleton(br, 6, phase == 1 ? kSplitLayer : 0,
                  net->nstreams == 0 ? std::function<int()>() : std::function<int()>(sensor_bwd)));
  if (phase == 1) return br.mark_phase1();  // the caller orders its all-reduce after f3_net_wait_phase1
  F3_TRY(br.join());
  return F3_OK;
}
}  // namespace

extern "C" {

int f3_net_sensor_times(f3_net* net, int enable, float* ms) {
  if (!net) return F3_EINVAL;
  if (!net->has_cnn) return F3_EINVAL;
  if (enable && !net->stiming) {
    for (auto& e : net->sev)
      if (!e && hipEventCreate(&e) != hipSuccess) return F3_EHIP;
  }
  if (ms) {  // forward, backward (ms)
    if (!net->stiming) return F3_ESTATE;
    const int pairs[2][2] = {{0, 1}, {2, 3}};
    for (int i = 0; i < 2; ++i) {
      if (hipEventSynchronize(net->sev[pairs[i][1]]) != hipSuccess ||
          hipEventElapsedTime(&ms[i], net->sev[pairs[i][0]], net->sev[pairs[i][1]]) != hipSuccess)
        return F3_EHIP;
    }
  }
  net->stiming = enable;
  return F3_OK;
}

int f3_net_wait_phase1(f3_net* net, void* stream) {
  if (!net) return F3_EINVAL;
  return wait_phase1(*net, (hipStream_t)stream);
}

int f3_rmsprop_step(float* params, float* square_avg, const float* grads, int64_t n, float lr, float alpha,
                    float eps, float grad_scale, void* stream) {
  if (!params || !square_avg || !grads) return F3_EINVAL;
  return f3_rmsprop(params, square_avg, grads, n, lr, alpha, eps, grad_scale, (hipStream_t)stream);
}

// test-entry scratch (kept for the process lifetime; the network uses its workspace)
static const unsigned short* test_zero_page() {
  static void* z = nullptr;
  if (!z && hipMalloc(&z, 4096) == hipSuccess) (void)hipMemset(z, 0, 4096);
  return (const unsigned short*)z;
}
static float* test_scratch(size_t n) {
  static float* p = nullptr;
  static size_t cap = 0;
  if (n > cap) {
    if (p) (void)hipFree(p);
    p = nullptr;
    if (hipMalloc(&p, n * sizeof(float)) != hipSuccess) return nullptr;
    cap = n;
  }
  return p;
}

int f3_conv_forward(const void* x, const float* w, const float* bias, float* out, float* wpack, int N, int T_in,
                    int V, int Cin, int Cout, int KT, int stride, int pad, int precision, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  if (precision < 0 || precision > F3_PRECISION_BF16X3) return F3_EINVAL;
  const bool bf_out = precision == F3_CONV_BF16_OUT;
  if (bf_out) precision = F3_PRECISION_BF16;
  const int x3 = precision == F3_PRECISION_BF16X3;
  const int hb = precision != F3_PRECISION_FP32;
  if (w) {  // w == NULL: wpack already holds the packed operand (timing the GEMM alone)
    PrepTable t;
    t.n = 0;
    add_job(t, PREP_PACK_CONV, Cout * KT * Cin, wpack, w, nullptr, nullptr, Cout, Cin, KT, x3 ? 2 : hb);
    F3_TRY(f3_prep(t, s));
  }
  const int T_out = (T_in + 2 * pad - KT) / stride + 1;
  ConvGemmArgs a;
  std::memset(&a, 0, sizeof(a));
  a.g = geom(N * T_out * V, Cout, Cin, KT, stride, pad, 0, T_out, T_in, V, Cin, Cout);
  if (precision == F3_PRECISION_BF16) {
    a.inb = (const unsigned short*)x;
    a.zero = test_zero_page();
  } else {
    a.in = (const float*)x;
  }
  a.w = wpack; a.wb = bf(wpack, hb); a.out = out; a.bias = bias; a.x3 = x3;
  if (bf_out) a.outb = reinterpret_cast<unsigned short*>(out);
  return f3_conv_gemm(&a, 0, EPI_BIAS, s);
}

int f3_conv_backward_data(const void* dy, const float* w, float* dx, float* wpack, int N, int T_in, int V, int Cin,
                          int Cout, int KT, int stride, int pad, int precision, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  if (precision < 0 || (precision > 2 && precision != F3_PRECISION_BF16X3)) return F3_EINVAL;
  const int x3 = precision == F3_PRECISION_BF16X3;
  const int hb = precision != F3_PRECISION_FP32;
  PrepTable t;
  t.n = 0;
  add_job(t, PREP_PACK_CONV_T, Cout * KT * Cin, wpack, w, nullptr, nullptr, Cout, Cin, KT, x3 ? 2 : hb);
  F3_TRY(f3_prep(t, s));
  const int T_out = (T_in + 2 * pad - KT) / stride + 1;
  ConvGemmArgs a;
  std::memset(&a, 0, sizeof(a));
  a.g = geom(N * T_in * V, Cin, Cout, KT, stride, pad, 1, T_in, T_out, V, Cout, Cin);
  if (precision == F3_PRECISION_BF16) {
    a.inb = (const unsigned short*)dy;
    a.zero = test_zero_page();
  } else {
    a.in = (const float*)dy;
  }
  a.w = wpack; a.wb = bf(wpack, hb); a.out = dx; a.x3 = x3;
  return f3_conv_gemm(&a, 0, 0, s);
}

int f3_pointwise_conv(const void* x, const void* wpack, const float* bias, void* out, int out_bf16, double* st_sum,
                      double* st_sq, int N, int T_in, int T_out, int V, int Cin, int Cout, int stride, int transposed,
                      int epi, void* stream) {
  if (!x || !wpack || !out || N <= 0 || T_in <= 0 || T_out <= 0 || V <= 0 || (stride != 1 && stride != 2)) return F3_EINVAL;
  if (epi != 0 && epi != EPI_BIAS && epi != (EPI_BIAS | EPI_STATS) && epi != (EPI_BIASV | EPI_STATS) && epi != EPI_ADD)
    return F3_EINVAL;
  if (transposed ? (T_in != (T_out - 1) / stride + 1) : (T_out != (T_in - 1) / stride + 1)) return F3_EINVAL;
  if ((epi & EPI_ADD) && out_bf16) return F3_EINVAL;
  if ((epi & EPI_STATS) && (!st_sum || !st_sq)) return F3_EINVAL;
  if ((epi & (EPI_BIAS | EPI_BIASV)) && !bias) return F3_EINVAL;
  ConvGemmArgs a;
  std::memset(&a, 0, sizeof(a));
  a.g = geom(N * T_out * V, Cout, Cin, 1, stride, 0, transposed, T_out, T_in, V, Cin, Cout);
  a.inb = (const unsigned short*)x;
  a.wb = (const unsigned short*)wpack;
  a.zero = test_zero_page();
  if (out_bf16) a.outb = (unsigned short*)out;
  else a.out = (float*)out;
  a.bias = bias; a.st_sum = st_sum; a.st_sq = st_sq;
  if (!f3_igemm_ok(a)) return F3_EINVAL;
  return f3_igemm_bf16(&a, epi, (hipStream_t)stream);
}

// ---- bf16x3 on the bf16 kernels, as the step launches them ([hi | lo] operand rows, native form) ----
int f3_split_x3cat(const float* x, void* out, int64_t rows, int C, void* stream) {
  if (!x || !out || rows < 0 || C <= 0 || C % 4) return F3_EINVAL;
  return f3_split_x3(x, static_cast<unsigned short*>(out), rows, C, (hipStream_t)stream);
}

static bool x3cat_shape_ok(int N, int T_in, int V, int Cin, int Cout, int KT, int stride, int pad) {
  return N > 0 && T_in > 0 && V > 0 && Cin > 0 && Cout > 0 && KT > 0 && (stride == 1 || stride == 2) && pad >= 0 &&
         (T_in + 2 * pad - KT) / stride + 1 > 0 && Cin % 8 == 0 && Cout % 8 == 0;
}

int f3_conv_forward_x3cat(const void* x3, const float* w, const float* bias, float* out, void* wpack, int N, int T_in,
                          int V, int Cin, int Cout, int KT, int stride, int pad, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  if (!x3 || !bias || !out || !wpack || !x3cat_shape_ok(N, T_in, V, Cin, Cout, KT, stride, pad)) return F3_EINVAL;
  if (w) {  // the step's packing (native [W_hi 32 | W_lo 32] blocks; w == NULL: wpack already packed)
    PrepTable t;
    t.n = 0;
    add_job(t, PREP_PACK_CONV, Cout * KT * Cin * x3mul(x3code()), static_cast<float*>(wpack), w, nullptr, nullptr,
            Cout, Cin, KT, x3code());
    F3_TRY(f3_prep(t, s));
  }
  const int T_out = (T_in + 2 * pad - KT) / stride + 1;
  ConvGemmArgs a;
  std::memset(&a, 0, sizeof(a));
  a.g = geom(N * T_out * V, Cout, Cin, KT, stride, pad, 0, T_out, T_in, V, 2 * Cin, Cout);
  x3_gemm(a, Cin);
  a.inb = static_cast<const unsigned short*>(x3); a.zero = test_zero_page();
  a.wb = static_cast<const unsigned short*>(wpack); a.out = out; a.bias = bias;
  if (!f3_igemm_ok(a)) return F3_EINVAL;
  return f3_conv_gemm(&a, 0, EPI_BIAS, s);
}

int f3_conv_backward_data_x3cat(const void* dy3, const float* w, float* dx, void* wpack, int N, int T_in, int V,
                                int Cin, int Cout, int KT, int stride, int pad, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  if (!dy3 || !dx || !wpack || !x3cat_shape_ok(N, T_in, V, Cin, Cout, KT, stride, pad)) return F3_EINVAL;
  if (w) {  // the transposed packing, as the step's
    PrepTable t;
    t.n = 0;
    add_job(t, PREP_PACK_CONV_T, Cout * KT * Cin * x3mul(x3code()), static_cast<float*>(wpack), w, nullptr, nullptr,
            Cout, Cin, KT, x3code());
    F3_TRY(f3_prep(t, s));
  }
  const int T_out = (T_in + 2 * pad - KT) / stride + 1;
  ConvGemmArgs a;
  std::memset(&a, 0, sizeof(a));
  a.g = geom(N * T_in * V, Cin, Cout, KT, stride, pad, 1, T_in, T_out, V, 2 * Cout, Cin);
  x3_gemm(a, Cout);
  a.inb = static_cast<const unsigned short*>(dy3); a.zero = test_zero_page();
  a.wb = static_cast<const unsigned short*>(wpack); a.out = dx;
  if (!f3_igemm_ok(a)) return F3_EINVAL;
  return f3_conv_gemm(&a, 0, 0, s);
}

int f3_conv_step_x3cat(int kind, const void* in3, const float* w, void* wpack, float* out, const float* bias_v,
                       const float* g, const float* gamma, const float* beta, const double* bn_sum,
                       const double* bn_sq, float bn_count, double* st_sum, double* st_sq, int N, int T, int V,
                       int Cin, int Cout, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  const bool gcn = kind == F3_STEP_GCN_FWD, dgrad = kind == F3_STEP_TCN_DGRAD;
  if ((!gcn && !dgrad) || !in3 || !wpack || !out || !st_sum || !st_sq) return F3_EINVAL;
  if (gcn && !bias_v) return F3_EINVAL;
  if (dgrad && (!g || !gamma || !beta || !bn_sum || !bn_sq || bn_count <= 0.f)) return F3_EINVAL;
  const int KT = gcn ? 1 : 9, pad = gcn ? 0 : 4;
  if (!x3cat_shape_ok(N, T, V, Cin, Cout, KT, 1, pad)) return F3_EINVAL;
  if (w) {  // the step's packing (w == NULL: wpack already packed)
    PrepTable t;
    t.n = 0;
    add_job(t, gcn ? PREP_PACK_CONV : PREP_PACK_CONV_T, Cout * KT * Cin * x3mul(x3code()), static_cast<float*>(wpack),
            w, nullptr, nullptr, Cout, Cin, KT, x3code());
    F3_TRY(f3_prep(t, s));
  }
  ConvGemmArgs a;
  std::memset(&a, 0, sizeof(a));
  a.inb = static_cast<const unsigned short*>(in3); a.zero = test_zero_page();
  a.wb = static_cast<const unsigned short*>(wpack); a.out = out; a.st_sum = st_sum; a.st_sq = st_sq;
  if (gcn) {  // stream_forward_layer's gcn GEMM: [Z_hi | Z_lo] rows of K Ci channels, graph-mixed bias, BN1 sums
    a.g = geom(N * T * V, Cout, Cin, 1, 1, 0, 0, T, T, V, Cin, Cout);
    x3_gemm(a, Cin);
    a.bias = bias_v;
    if (!f3_igemm_ok(a)) return F3_EINVAL;
    return f3_conv_gemm(&a, 0, EPI_BIASV | EPI_STATS, s);
  }
  // stream_backward's tcn input gradient: dh rows [hi | lo] of Cout channels (the tcn's output) into
  // dv[M][Cin]; ReLU mask of bn1(g) and the BN1-backward sums in the epilogue (RELUMASK)
  a.g = geom(N * T * V, Cin, Cout, KT, 1, pad, 1, T, T, V, Cout, Cin);
  x3_gemm(a, Cout);
  a.aux = g; a.ldaux = Cin;
  a.epi_bn.sum = bn_sum; a.epi_bn.sumsq = bn_sq; a.epi_bn.gamma = gamma; a.epi_bn.beta = beta;
  a.epi_bn.count = bn_count; a.epi_bn.eval = 0;
  if (!f3_igemm_ok(a)) return F3_EINVAL;
  return f3_conv_gemm(&a, 0, EPI_RELUMASK, s);
}

int f3_conv_backward_weight_x3cat(const void* dy3, const void* x3, float* dw, float* db, int N, int T_in, int V,
                                  int Cin, int Cout, int KT, int stride, int pad, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  if (!dy3 || !x3 || !x3cat_shape_ok(N, T_in, V, Cin, Cout, KT, stride, pad)) return F3_EINVAL;
  const int T_out = (T_in + 2 * pad - KT) / stride + 1;
  const long long cap = kWgradSlabFloats * 4;  // the step's x3 slab (plan: W.slab)
  float* slab = test_scratch((size_t)cap + 2 * Cout);
  if (!slab) return F3_EHIP;
  WgradArgs a;
  std::memset(&a, 0, sizeof(a));
  a.ldy = 2 * Cout; a.outmap = WG_OUT_CONV; a.bf16 = 1;
  a.dyb = static_cast<const unsigned short*>(dy3); a.inb = static_cast<const unsigned short*>(x3);
  a.zero = test_zero_page(); a.slab = slab; a.slab_cap = cap;
  a.g = geom(N * T_out * V, Cout, Cin, KT, stride, pad, 0, T_out, T_in, V, 2 * Cin, Cout);
  a.x3seg = 1;
  if (dw) {  // dw == NULL: the GEMM alone (partials left in the slab)
    if (hipMemsetAsync(dw, 0, sizeof(float) * Cout * Cin * KT, s) != hipSuccess) return F3_EHIP;
    a.dw_ref = dw;
    if (db) {
      if (hipMemsetAsync(db, 0, sizeof(float) * Cout, s) != hipSuccess) return F3_EHIP;
      a.db = db;
    }
  }
  if (!f3_wgrad_glds_ok(a)) return F3_EINVAL;
  return f3_conv_wgrad(&a, 0, s);
}

int f3_conv_backward_weight(const void* dy, const void* x, float* dw, float* db, int N, int T_in, int V, int Cin,
                            int Cout, int KT, int stride, int pad, int precision, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  if (precision < 0 || (precision > 2 && precision != F3_PRECISION_BF16X3)) return F3_EINVAL;
  const int T_out = (T_in + 2 * pad - KT) / stride + 1;
  if (hipMemsetAsync(dw, 0, sizeof(float) * Cout * Cin * KT, s) != hipSuccess) return F3_EHIP;
  if (db && hipMemsetAsync(db, 0, sizeof(float) * Cout, s) != hipSuccess) return F3_EHIP;
  WgradArgs a;
  std::memset(&a, 0, sizeof(a));
  a.g = geom(N * T_out * V, Cout, Cin, KT, stride, pad, 0, T_out, T_in, V, Cin, Cout);
  a.ldy = Cout; a.dw = dw; a.db = db; a.outmap = WG_OUT_CONV;
  a.x3 = precision == F3_PRECISION_BF16X3;
  a.bf16 = precision != F3_PRECISION_FP32 && !a.x3;
  if (precision == F3_PRECISION_BF16) {
    a.dyb = (const unsigned short*)dy;
    a.inb = (const unsigned short*)x;
    a.zero = test_zero_page();
    if (f3_wgrad_glds_ok(a)) {  // split partials in a scratch slab, summed into dw (the step's path)
      const long long cap = kWgradSlabFloats;
      float* slab = test_scratch((size_t)cap);
      if (!slab) return F3_EHIP;
      a.slab = slab; a.slab_cap = cap; a.dw_ref = dw;
      return f3_conv_wgrad(&a, 0, s);
    }
  } else {
    a.dy = (const float*)dy;
    a.in = (const float*)x;
  }
  return f3_conv_wgrad(&a, 0, s);
}

int f3_conv_wgrad_packed(const void* dy, const void* x, float* slab, long long slab_floats, int N, int T_in, int V,
                         int Cin, int Cout, int KT, int stride, int pad, void* stream) {
  if (!dy || !x || !slab || N < 1) return F3_EINVAL;
  const int T_out = (T_in + 2 * pad - KT) / stride + 1;
  WgradArgs a;
  std::memset(&a, 0, sizeof(a));
  a.g = geom(N * T_out * V, Cout, Cin, KT, stride, pad, 0, T_out, T_in, V, Cin, Cout);
  a.ldy = Cout; a.dw = nullptr; a.db = nullptr; a.outmap = WG_OUT_CONV; a.bf16 = 1;
  a.slab = slab; a.slab_cap = slab_floats; a.dw_ref = nullptr;  // the kernel alone: partials stay in the slab
  a.dyb = (const unsigned short*)dy; a.inb = (const unsigned short*)x; a.zero = test_zero_page();
  if (!f3_wgrad_glds_ok(a)) return F3_EINVAL;
  return f3_conv_wgrad(&a, 0, (hipStream_t)stream);
}

int f3_graph_mix_forward(const float* A_eff, const float* x, float* z, int frames, int K, int V, int Cin,
                         void* stream) {
  MixArgs m;
  std::memset(&m, 0, sizeof(m));
  m.K = K; m.V = V; m.Cin = Cin; m.frames = frames; m.A = A_eff; m.x = x; m.z = z;
  return f3_mix_fwd(&m, (hipStream_t)stream);
}

int f3_graph_mix_backward(const float* A_eff, const float* x, const float* dz, float* dx, float* dA, int frames, int K,
                          int V, int Cin, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  if (hipMemsetAsync(dA, 0, sizeof(float) * K * V * V, s) != hipSuccess) return F3_EHIP;
  MixArgs m;
  std::memset(&m, 0, sizeof(m));
  m.K = K; m.V = V; m.Cin = Cin; m.frames = frames; m.A = A_eff; m.x = x; m.z = const_cast<float*>(dz);
  m.dx = dx; m.dA = dA; m.accumulate = 0;
  static float* part = nullptr;  // test entry only: scratch kept for the process lifetime
  if (!part && hipMalloc(&part, sizeof(float) * kMixParts * 1024) != hipSuccess) return F3_EHIP;
  m.part = part;
  return f3_mix_bwd(&m, s);
}

int f3_graph_mix_forward_ex(const float* A_eff, const void* x, void* z, int frames, int K, int V, int Cin, int flags,
                            void* stream) {
  if (!A_eff || !x || !z || frames < 0 || (flags & ~15) || ((flags & F3_MIX_X3) && (flags & 3))) return F3_EINVAL;
  if ((flags & F3_MIX_Z3) && !(flags & F3_MIX_X3)) return F3_EINVAL;
  MixArgs m;
  std::memset(&m, 0, sizeof(m));
  m.K = K; m.V = V; m.Cin = Cin; m.frames = frames; m.A = A_eff;
  m.x = static_cast<const float*>(x); m.x16 = flags & F3_MIX_X_BF16; m.x3 = (flags & F3_MIX_X3) != 0;
  m.z = static_cast<float*>(z);
  if (flags & F3_MIX_Z_BF16) m.zb = static_cast<unsigned short*>(z);
  if (flags & F3_MIX_Z3) m.z3 = static_cast<unsigned short*>(z);
  return f3_mix_fwd(&m, (hipStream_t)stream);
}

int f3_graph_mix_backward_ex(const float* A_eff, const void* x, const void* dz, float* dx, float* dA, int frames, int K,
                             int V, int Cin, int flags, void* stream) {
  if (!A_eff || !x || !dz || !dx || !dA || frames < 0 || (flags & ~5) || ((flags & F3_MIX_X3) && (flags & 1)))
    return F3_EINVAL;
  hipStream_t s = (hipStream_t)stream;
  if (hipMemsetAsync(dA, 0, sizeof(float) * K * V * V, s) != hipSuccess) return F3_EHIP;
  MixArgs m;
  std::memset(&m, 0, sizeof(m));
  m.K = K; m.V = V; m.Cin = Cin; m.frames = frames; m.A = A_eff; m.x = static_cast<const float*>(x);
  m.dx = dx; m.dA = dA; m.accumulate = 0; m.x3 = (flags & F3_MIX_X3) != 0;
  if (flags & F3_MIX_X_BF16) {
    m.x16 = 1;
    m.dzb = static_cast<const unsigned short*>(dz);
  } else {
    m.z = const_cast<float*>(static_cast<const float*>(dz));
  }
  static float* part = nullptr;  // test entry only: scratch kept for the process lifetime
  if (!part && hipMalloc(&part, sizeof(float) * kMixParts * 1024) != hipSuccess) return F3_EHIP;
  m.part = part;
  return f3_mix_bwd(&m, s);
}

// debug accessor (tests/tools only): device pointer of a named per-layer workspace tensor
void* f3_net_debug_tensor(f3_net* net, int batch, void* workspace, int stream, int layer, const char* what) {
  if (!net || stream < 0 || stream >= net->nstreams || layer < 0 || layer > 6) return nullptr;
  Ws w = plan(*net, batch, (char*)workspace);
  StreamWs& W = w.st[stream];
  LayerWs& X = W.L[layer];
  const std::string k(what);
  if (k == "x") return (void*)X.x;
  if (k == "z") return X.z;
  if (k == "g") return X.g;
  if (k == "h") return X.h;
  if (k == "r") return X.r;
  if (k == "out") return X.out;
  if (k == "att") return X.att;
  if (k == "dh") return X.dh;
  if (k == "u") return X.u;
  if (k == "dv") return W.dv;
  if (k == "dg") return X.dg;
  if (k == "dZ") return W.dZ;
  if (k == "dres") return X.dres;
  if (k == "dx0") return W.dx[0];
  if (k == "dx1") return W.dx[1];
  if (k == "bn1_fsum") return X.bn1.fsum;
  if (k == "bn1_fsq") return X.bn1.fsq;
  if (k == "bn1_bsum") return X.bn1.bsum;
  if (k == "bn1_bsq") return X.bn1.bsq;
  if (k == "twT") return X.twT;
  if (k == "P1") return X.P1;
  if (k == "P2") return X.P2;
  if (k == "e") return X.e;
  if (k == "gap") return X.gap;
  if (k == "q1") return X.q1;
  if (k == "hid") return X.hid;
  if (k == "dq1") return X.dq1;
  if (k == "dq2") return X.dq2;
  if (k == "dbn") return X.dbn;
  if (k == "bn2_fsum") return X.bn2.fsum;
  if (k == "bn2_fsq") return X.bn2.fsq;
  if (k == "bn2_bsum") return X.bn2.bsum;
  if (k == "bn2_bsq") return X.bn2.bsq;
  if (k == "ca_fsum") return X.bnca.fsum;
  if (k == "ca_fsq") return X.bnca.fsq;
  if (k == "dpool") return W.dpool;
  if (k == "pool") return W.pool;
  return nullptr;
}

const char* f3_status_string(int st) {
  switch (st) {
    case F3_OK: return "ok";
    case F3_EINVAL: return "invalid argument or unsupported shape";
    case F3_EBATCH: return "Expected more than 1 value per channel when training";
    case F3_EHIP: return "HIP launch error";
    case F3_ESTATE: return "backward without a training forward";
    case F3_EDEVICE: return "device-side check failed (a group barrier timed out: TARGCN GRU or sensor CNN1D; outputs are invalid)";
    default: return "unknown status";
  }
}

}  // extern "C"
