#!/usr/bin/env python3
"""Generate golden vectors by running the REFERENCE's own modules (build container only).

Run:  PYTHONDONTWRITEBYTECODE=1 python tools/gen_golden.py [--targcn-only | --sktr-only | --musa-only]
Writes: tests/golden/*.npz  (small, committed; the reference itself never travels).

How the reference is imported: the packaged 3-stream model lives in
/root/reference/Multimodal_Fall3/model/{stgcan,graph,bilstm,combination}.py, but
combination.py:5-6 imports a non-existent `model.st_gcn` subpackage, so that name is
aliased to the real modules. The UR notebook model is obtained by exec'ing cells 1-2
of GSTCAN_UR_conv.ipynb on CPU. Nothing is copied into this repo: only inputs,
outputs, gradients and post-step parameter samples are stored.

Weights come from oracle/prng.py (seeded per parameter name), so a fixture stores
only the seed; `load_state_dict(strict=True)` also proves that the oracle's
parameter table has the reference's exact state_dict keys and shapes.
"""
from __future__ import annotations

import contextlib
import importlib
import io
import json
import os
import sys
import types

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
sys.path.insert(0, REPO)
from oracle import model_cpu as oc  # noqa: E402
from oracle import musa_cpu as mu  # noqa: E402
from oracle import sktr_cpu as sk  # noqa: E402
from oracle import targcn_cpu as tg  # noqa: E402
from oracle.prng import synthetic_batch  # noqa: E402

REF = "/root/reference"
OUT = os.path.join(REPO, "tests", "golden")
FULL_LIMIT = 128    # tensors up to this many elements are stored whole
SAMPLES = 32


def import_reference():
    sys.path.insert(0, REF + "/Multimodal_Fall3")
    stg = importlib.import_module("model.stgcan")
    gr = importlib.import_module("model.graph")
    pkg = types.ModuleType("model.st_gcn")
    pkg.__path__ = []
    sys.modules.update({"model.st_gcn": pkg, "model.st_gcn.stgcan": stg, "model.st_gcn.graph": gr})
    comb = importlib.import_module("model.combination")
    bil = importlib.import_module("model.bilstm")
    nb = json.load(open(REF + "/GSTCAN_UR_conv.ipynb"))
    ns = {"__name__": "nbmod", "device": torch.device("cpu")}
    exec(compile("\n".join("".join(nb["cells"][i]["source"]) for i in (1, 2)), "nb_ur", "exec"), ns)
    return stg, gr, comb, bil, ns


def sample_idx(n):
    if n <= SAMPLES:
        return np.arange(n)
    return (np.arange(SAMPLES) * (n // SAMPLES) + 7) % n


def pack(prefix, d, t):
    a = t.detach().double().numpy().reshape(-1)
    if a.size <= FULL_LIMIT:
        d[prefix] = a.astype(np.float32)
    else:
        d[prefix + "@norm"] = np.array([np.linalg.norm(a)])
        d[prefix + "@sum"] = np.array([a.sum()])
        d[prefix + "@val"] = a[sample_idx(a.size)].astype(np.float32)


def run_case(tag, module, spec, forward_fn, batch, seed, frames=30, sensor_frames=30):
    torch.manual_seed(0)
    state = oc.init_state(spec, seed, sensor_frames)
    module.load_state_dict(state, strict=True)
    module.train()
    V = state[next(k for k in state if k.endswith("A"))].shape[-1] if spec.model != "bilstm" else 14
    skel, sensor, label = synthetic_batch(batch, V, spec.num_class, spec.sensor_dim, seed + 1,
                                          frames=frames, sensor_frames=sensor_frames)
    sk, se, lb = (torch.from_numpy(x) for x in (skel, sensor, label))
    opt = torch.optim.RMSprop(module.parameters(), lr=1e-3)
    opt.zero_grad()
    with contextlib.redirect_stdout(io.StringIO()):
        out = forward_fn(module, sk, se)
    loss = torch.nn.CrossEntropyLoss()(out, lb)
    loss.backward()
    d = {"seed": np.array([seed]), "skel": skel, "sensor": sensor, "label": label,
         "out": out.detach().numpy(), "loss": np.array([loss.item()]),
         "spec": np.array([json.dumps(spec.__dict__)])}
    nparams = 0
    for name, p in module.named_parameters():
        nparams += p.numel()
        if p.grad is None:  # e.g. CNN1D.fc is built but never used (GSTCAN_UR_conv.ipynb cell 2)
            d["nograd:" + name] = np.array([1])
            continue
        pack("grad:" + name, d, p.grad)
    opt.step()
    for name, p in module.named_parameters():
        pack("post:" + name, d, p)
    for name, b in module.named_buffers():
        if name.endswith(("running_mean", "running_var")):
            pack("buf:" + name, d, b)
    d["nparams"] = np.array([nparams])
    path = os.path.join(OUT, f"model_{tag}.npz")
    np.savez_compressed(path, **d)
    print(f"{tag}: params={nparams} loss={loss.item():.6f} -> {path} ({os.path.getsize(path)//1024} KB)")
    return nparams


def import_targcn():
    """TRAGCN.py imports `TRAGCN.GRU` / `TRAGCN.TA` (the notebook's package name,
    TARGCN_HAR_conv_10kfold.ipynb cell 3): alias a package of that name to the reference root."""
    tp = types.ModuleType("TRAGCN")
    tp.__path__ = [REF]
    sys.modules["TRAGCN"] = tp
    with contextlib.redirect_stdout(io.StringIO()):
        return importlib.import_module("TRAGCN.TRAGCN")


def run_targcn_case(tag, T, V, batch, seed, lr=1e-5):
    """TARGCN(adj=None, num_nodes=V) train step as the notebook runs it: out = model(pts.permute(0,2,3,1)),
    CrossEntropyLoss(out, soft labels), RMSprop(lr=1e-5). weights_pool / bias_pool are
    uninitialised memory in the reference (EmbGCN.py:67-68): every parameter is loaded from the
    portable PRNG instead."""
    torch.manual_seed(0)
    model = T.TARGCN(adj=None, num_nodes=V)
    state = tg.init_state(V, seed)
    model.load_state_dict(state, strict=True)
    model.train()
    src, label = tg.synthetic_source(batch, V, 11, seed + 1)
    x, lb = torch.from_numpy(src), torch.from_numpy(label)
    opt = torch.optim.RMSprop(model.parameters(), lr=lr)
    opt.zero_grad()
    out = model(x)
    loss = torch.nn.CrossEntropyLoss()(out, lb)
    loss.backward()
    d = {"seed": np.array([seed]), "V": np.array([V]), "source": src, "label": label, "lr": np.array([lr]),
         "out": out.detach().numpy(), "loss": np.array([loss.item()])}
    nparams = 0
    for name, p in model.named_parameters():
        nparams += p.numel()
        pack("grad:" + name, d, p.grad)
    opt.step()
    for name, p in model.named_parameters():
        pack("post:" + name, d, p)
    d["nparams"] = np.array([nparams])
    path = os.path.join(OUT, f"targcn_{tag}.npz")
    np.savez_compressed(path, **d)
    print(f"targcn {tag}: params={nparams} loss={loss.item():.6f} -> {path} ({os.path.getsize(path)//1024} KB)")
    return nparams


def import_sktr():
    """skeleton_transformer.py imports torchvision (absent here) for ops.StochasticDepth: stub it as
    the identity, which is what the reference computes in eval mode and what a
    train-mode step computes with every stochastic-depth draw kept at scale 1."""
    tv = types.ModuleType("torchvision")
    ops = types.ModuleType("torchvision.ops")

    class StochasticDepth(torch.nn.Module):
        def __init__(self, p, mode):
            super().__init__()
            self.p, self.mode = p, mode

        def forward(self, x):
            return x

    ops.StochasticDepth = StochasticDepth
    tv.ops = ops
    sys.modules.setdefault("torchvision", tv)
    sys.modules.setdefault("torchvision.ops", ops)
    sys.path.insert(0, REF)
    return importlib.import_module("skeleton_transformer")


def run_sktr_case(tag, S, batch, seed, M=1, V=14, T=30, lr=1e-3):
    """SkeletonTransformer(3, V, T, 11, 32, 6, 16, 8) train step (GSTCAN_HAR_conv_kfold_trans.ipynb):
    CE(out, soft labels), RMSprop(lr). Stochastic depth = identity (torchvision stub) and the FFN
    Dropout(0.5) set to p=0, so the step is deterministic; the oracle covers both with explicit
    draws. Also records eval-mode logits of the initial model (running statistics 0 / 1): after
    the step the biases that feed a BatchNorm have moved by RMSprop's +-10*lr on rounding-level
    gradients, which eval mode (no batch statistics to cancel them) would amplify."""
    torch.manual_seed(0)
    model = S.SkeletonTransformer(3, V, T, 11, 32, 6, 16, 8)
    for m in model.modules():
        if isinstance(m, torch.nn.Dropout):
            m.p = 0.0
    state = sk.init_state(seed, V, T)
    assert list(model.state_dict().keys()) == list(state.keys()), "oracle state_dict order differs"
    model.load_state_dict(state, strict=True)
    xs, label = sk.synthetic_clips(batch, V, 11, seed + 1, T=T, M=M)
    x, lb = torch.from_numpy(xs), torch.from_numpy(label)
    model.eval()
    with torch.no_grad():
        eval_out = model(x).numpy()
    model.train()
    opt = torch.optim.RMSprop(model.parameters(), lr=lr)
    opt.zero_grad()
    out = model(x)
    loss = torch.nn.CrossEntropyLoss()(out, lb)
    loss.backward()
    d = {"seed": np.array([seed]), "V": np.array([V]), "T": np.array([T]), "M": np.array([M]), "x": xs,
         "label": label, "lr": np.array([lr]), "out": out.detach().numpy(), "loss": np.array([loss.item()])}
    nparams = 0
    for name, p in model.named_parameters():
        nparams += p.numel()
        pack("grad:" + name, d, p.grad)
    opt.step()
    for name, p in model.named_parameters():
        pack("post:" + name, d, p)
    for name, b in model.named_buffers():
        if name.endswith(("running_mean", "running_var")):
            pack("buf:" + name, d, b)
    d["eval_out"] = eval_out
    d["nparams"] = np.array([nparams])
    path = os.path.join(OUT, f"sktr_{tag}.npz")
    np.savez_compressed(path, **d)
    print(f"sktr {tag}: params={nparams} loss={loss.item():.6f} -> {path} ({os.path.getsize(path)//1024} KB)")
    return nparams


def import_musa():
    sys.path.insert(0, REF + "/Multimodal_Fall3/model")
    return importlib.import_module("musa_model")


def run_musa_case(tag, Mm, batch, seed, lr=1e-3):
    """musa_model.Model as root Multimodal_Fall3/main.py:307-320 builds it, one train step with
    CrossEntropyLoss and RMSprop(lr). DropBlock off (keep_prob = 1 on every block, so the modules
    return their input) and the classifier's Dropout p = 0: the step is deterministic; the oracle
    covers the random parts with hash draws shared with the kernels."""
    import warnings
    torch.manual_seed(0)
    g = Mm.adjGraph(layout="coco_cut", strategy="uniform")
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        model = Mm.Model(num_class=11, num_point=14, max_frame=300, graph=g, bias=True, edge=True, block_size=41,
                         embed_dim=64, n_stage=1, act_type="tanh")
    for m in model.modules():
        if hasattr(m, "keep_prob"):
            m.keep_prob = 1.0
        if isinstance(m, torch.nn.Dropout):
            m.p = 0.0
    state = mu.init_state(seed)
    assert list(model.state_dict().keys()) == list(state.keys()), "oracle state_dict order differs"
    for k, v in model.state_dict().items():
        assert tuple(v.shape) == tuple(state[k].shape), k
        if k.endswith(".A"):
            assert torch.equal(v, state[k]), "adjGraph A differs from the oracle's"
    model.load_state_dict(state, strict=True)
    skel, _, label = synthetic_batch(batch, 14, 11, 1, seed + 1)
    x, lb = torch.from_numpy(skel), torch.from_numpy(label)
    model.eval()
    with torch.no_grad():
        eval_out = model(x).numpy()
    model.train()
    opt = torch.optim.RMSprop([p for p in model.parameters() if p.requires_grad], lr=lr)
    opt.zero_grad()
    out = model(x)
    loss = torch.nn.CrossEntropyLoss()(out, lb)
    loss.backward()
    d = {"seed": np.array([seed]), "x": skel, "label": label, "lr": np.array([lr]), "out": out.detach().numpy(),
         "loss": np.array([loss.item()]), "eval_out": eval_out}
    nparams = 0
    for name, p in model.named_parameters():
        nparams += p.numel()
        if p.grad is None:
            d["nograd:" + name] = np.array([1])
            continue
        pack("grad:" + name, d, p.grad)
    opt.step()
    for name, p in model.named_parameters():
        pack("post:" + name, d, p)
    for name, b in model.named_buffers():
        if name.endswith(("running_mean", "running_var")):
            pack("buf:" + name, d, b)
    d["nparams"] = np.array([nparams])
    path = os.path.join(OUT, f"musa_{tag}.npz")
    np.savez_compressed(path, **d)
    print(f"musa {tag}: params={nparams} loss={loss.item():.6f} -> {path} ({os.path.getsize(path)//1024} KB)")
    return nparams


def main():
    os.makedirs(OUT, exist_ok=True)
    if "--musa-only" in sys.argv:
        Mm = import_musa()
        kat = json.load(open(os.path.join(OUT, "param_counts.json")))
        kat["musa"] = run_musa_case("b4", Mm, 4, 9001)
        with open(os.path.join(OUT, "param_counts.json"), "w") as f:
            json.dump(kat, f, indent=1, sort_keys=True)
        return
    if "--sktr-only" in sys.argv:
        S = import_sktr()
        kat = json.load(open(os.path.join(OUT, "param_counts.json")))
        kat["sktr"] = run_sktr_case("m1", S, 4, 8001)
        run_sktr_case("m2", S, 3, 8002, M=2)
        with open(os.path.join(OUT, "param_counts.json"), "w") as f:
            json.dump(kat, f, indent=1, sort_keys=True)
        return
    if "--targcn-only" in sys.argv:
        T = import_targcn()
        kat = json.load(open(os.path.join(OUT, "param_counts.json")))
        kat["targcn_v14"] = run_targcn_case("v14", T, 14, 4, 7001)
        kat["targcn_v17"] = run_targcn_case("v17", T, 17, 3, 7002)
        with open(os.path.join(OUT, "param_counts.json"), "w") as f:
            json.dump(kat, f, indent=1, sort_keys=True)
        return
    stg, gr, comb, bil, ns = import_reference()

    # graph adjacency for every layout x strategy (graph.py:20-126)
    graphs = {}
    for layout in ("coco_cut", "coco_mmpose"):
        for strat in ("uniform", "distance", "spatial"):
            graphs[f"{layout}:{strat}"] = gr.Graph(layout=layout, strategy=strat).A.astype(np.float64)
    np.savez_compressed(os.path.join(OUT, "graphs.npz"), **graphs)

    kat = {}
    fwd_pkg = lambda m, sk, se: m(sk, se)  # noqa: E731

    def fwd_two(m, sk, se):  # reference TwoStreamSTGCAN.forward has a missing-arg bug (§0.7)
        mot = sk[:, :2, 1:] - sk[:, :2, :-1]
        return m.fc(torch.cat((m.stgcan_1(sk, None), m.stgcan_2(mot, None)), dim=-1))

    cases = []
    spec = oc.Spec(model="two_stgcan_bilstm", layout="coco_cut", num_class=11, sensor_dim=15)
    cases.append(("har", comb.TwoStreamSTGCAN_BiLSTM(3, {"layout": "coco_cut", "strategy": "spatial"}, 11,
                                                      bilstm_input_size=15), spec, fwd_pkg, 4, 1234))
    spec = oc.Spec(model="two_stgcan_bilstm", layout="coco_mmpose", num_class=11, sensor_dim=6)
    cases.append(("ns", comb.TwoStreamSTGCAN_BiLSTM(3, {"layout": "coco_mmpose", "strategy": "spatial"}, 11,
                                                     bilstm_input_size=6), spec, fwd_pkg, 4, 2345))
    spec = oc.Spec(model="two_stgcan", layout="coco_cut", num_class=11, sensor="none")
    cases.append(("two", comb.TwoStreamSTGCAN(3, {"layout": "coco_cut", "strategy": "spatial"}, 11),
                  spec, fwd_two, 4, 3456))
    spec = oc.Spec(model="stgcn", layout="coco_cut", num_class=11, sensor="none")
    cases.append(("stgcn", stg.STGCAN(3, {"layout": "coco_cut", "strategy": "spatial"}, num_class=11),
                  spec, lambda m, sk, se: m(sk, None), 3, 4567))
    spec = oc.Spec(model="bilstm", num_class=11, sensor_dim=15)
    cases.append(("bilstm", bil.BiLSTM(input_size=15, hidden_size=64, num_layers=1, dropout_prob=0.3,
                                       num_classes=11, feature="mean"),
                  spec, lambda m, sk, se: m(None, se), 5, 5678))
    spec = oc.Spec(model="two_stgcan_bilstm", layout="coco_cut", num_class=2, sensor="cnn_bilstm",
                   sensor_dim=4, sensor_classes=2, softmax_output=True, naming="notebook")
    cases.append(("ur_nb", ns["TwoStreamSpatialTemporalGraph"]({"strategy": "spatial"}, 2),
                  spec, lambda m, sk, se: m((sk, sk[:, :2, 1:] - sk[:, :2, :-1], se)), 4, 6789))
    for tag, mod, spec, fn, b, seed in cases:
        kat[tag] = run_case(tag, mod, spec, fn, b, seed)
    # BASELINE config 1: the sensor-only CNN_BiLSTM of GSTCAN_UR_sensor.ipynb (cell 2, called at :4142)
    nbs = json.load(open(REF + "/GSTCAN_UR_sensor.ipynb"))
    nss = {"__name__": "nbsensor", "device": torch.device("cpu")}
    exec(compile("".join(nbs["cells"][2]["source"]), "nb_ur_sensor", "exec"), nss)
    spec = oc.Spec(model="bilstm", num_class=2, sensor="cnn_bilstm", sensor_dim=4)
    kat["ur_sensor"] = run_case("ur_sensor", nss["CNN_BiLSTM"](hidden_size=16, num_layers=1, dropout_prob=0.3,
                                                              num_classes=2, feature="mean"),
                                spec, lambda m, sk, se: m(se), 8, 7890)
    T = import_targcn()
    kat["targcn_v14"] = run_targcn_case("v14", T, 14, 4, 7001)
    kat["targcn_v17"] = run_targcn_case("v17", T, 17, 3, 7002)
    S = import_sktr()
    kat["sktr"] = run_sktr_case("m1", S, 4, 8001)
    run_sktr_case("m2", S, 3, 8002, M=2)
    kat["musa"] = run_musa_case("b4", import_musa(), 4, 9001)
    with open(os.path.join(OUT, "param_counts.json"), "w") as f:
        json.dump(kat, f, indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
