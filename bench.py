#!/usr/bin/env python3
"""Benchmark: clips/s of the 3-stream fall-detection training step (fwd + CE + bwd +
RMSprop, + gradient all-reduce for N > 1) on MI355X, one process per GPU.

Workload (BASELINE.json north star / configs[3] per GPU): synthetic clips with B=256 per
GPU, T=30 frames, J=17 COCO joints + centre node (coco_mmpose, V=18), 3-channel skeleton
+ 6-axis IMU at the frame rate (Ts=30), 11 classes; random-init weights of the reference
architecture (TwoStreamSTGCAN_BiLSTM, combination.py:27-46). The reference has no RGB model
arithmetic; the build-defined RGB spatial-conv branch is timed beside the headline
(`rgb_branch`: its kernels alone, and the whole north-star step WITH it, skeleton + IMU + RGB as
one step), its parity unpinned.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--batch B] [--graph]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N

`bench.py --gpus N` without a torch.distributed environment starts the N ranks itself (one per
GPU, torch.distributed.run as a child process) and fails if the node has fewer than N GPUs.

Prints ONE JSON line (rank 0) with value = global clips/s over the timed region (max over
ranks) in the parity-meeting bf16x3 mode (split-bf16 products on bf16 MFMA, fp32 activations: logits
within 1e-3 of the fp64 oracle, identical argmax), the roofline of the dominant kernel (the
temporal-conv input-gradient clip-window GEMM, measured live with HIP events on the stream it runs on;
HBM traffic from profiles/r06_roofline_pmc.json) and the CPU baseline (the oracle timed on this host's
cores on a bounded sample). The bf16 and fp32 modes' step times are reported beside it
(bf16_mode, fp32_mode); `--precision bf16` makes the faster, lower-precision bf16 mode the line.
"""
import argparse
import json
import math
import subprocess
import os
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

PEAK_MFMA_TFLOPS = {"fp32": 157.3,    # MI355X_MICROARCH.md: dense FP32 matrix peak (spec)
                    "bf16": 2500.0,   # MI355X_MICROARCH.md: BF16 MFMA ~2.5 PF dense (no sparsity)
                    "bf16x3": 2500.0}  # split-bf16 runs on the bf16 MFMA: priced at 3 bf16 products per FLOP
# bf16 MFMA products per algorithmic (fp32-equivalent) FLOP of a mode: the split product x_hi w_hi +
# x_lo w_hi + x_hi w_lo costs three
PRODUCTS = {"fp32": 1, "bf16": 1, "bf16x3": 3}
PEAK_HBM_GBS = 8000.0
FLOP_PER_CLIP = {(18, 6): 5.118e9, (14, 15): 3.946e9}  # 3-stream fwd+bwd GEMM FLOPs per clip


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=5)
    p.add_argument("--batch", type=int, default=256, help="clips per GPU")
    p.add_argument("--layout", default="coco_mmpose")
    p.add_argument("--sensor-dim", type=int, default=6)
    p.add_argument("--precision", default=None, choices=("bf16x3", "bf16", "fp32"),
                   help="GEMM arithmetic. bf16x3 (the fall3 default, the parity-meeting mode): fp32 activations, "
                        "split-bf16 products on bf16 MFMA; bf16: bf16 operands, fp32 accumulate (faster, logits "
                        "~4e-3 off); fp32: fp32 MFMA. The other --model legs default to bf16")
    p.add_argument("--graph", action="store_true",
                   help="replay the step as HIP graphs (measured slower on ROCm 7.2 for this multi-stream "
                        "step: 10.1 vs 8.15 ms at B=256; see DESIGN.md)")
    p.add_argument("--no-graph", action="store_true", help=argparse.SUPPRESS)  # the default; kept for old commands
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--model", default="fall3", choices=("fall3", "targcn", "sktr", "musa"),
                   help="fall3: the headline 3-stream step (default). targcn / sktr: BASELINE config 2 / 5 alone; "
                        "musa: the root main.py's musa_model")
    p.add_argument("--no-targcn", action="store_true", help="skip the config-2 TARGCN and config-5 lines in the default run")
    p.add_argument("--cpu-seconds", type=float, default=24.0)
    p.add_argument("--launch-check", action="store_true",
                   help="start the --gpus N ranks exactly as a bench run does, all-reduce each rank's id over gloo and "
                        "print the ranks seen; touches no GPU (tests/test_bench_launch.py)")
    a = p.parse_args()
    if a.precision is None:
        a.precision = "bf16x3" if a.model == "fall3" else "bf16"
    return a


def launch_ranks(a):
    """`bench.py --gpus N` with no torch.distributed environment: start N ranks (one per GPU) with
    torch.distributed.run as a CHILD process and exit with its status (never exec: this process
    must not have touched the GPU, and it has not - torch.cuda.device_count() does not initialise
    it). Fails loudly when the node has fewer than N GPUs instead of silently timing one."""
    import socket
    import subprocess
    if not a.launch_check:
        have = torch.cuda.device_count()
        if have < a.gpus:
            raise SystemExit(f"bench.py --gpus {a.gpus}: this node has {have} GPU(s); refusing to report a "
                             f"{a.gpus}-GPU number from fewer ranks")
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={a.gpus}",
           "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY=os.environ.get("HSA_ENABLE_IPC_MODE_LEGACY", "0"))
    return subprocess.call(cmd, env=env)


def launch_check(world, rank):
    """Each rank contributes its id over gloo: rank 0 prints the world and the ranks seen."""
    dist.init_process_group("gloo")
    ids = torch.zeros(world, dtype=torch.int64)
    ids[rank] = rank + 1
    dist.all_reduce(ids)
    if rank == 0:
        print(json.dumps({"launch_check": True, "world": dist.get_world_size(),
                          "ranks_seen": [int(i) - 1 for i in ids.tolist()]}), flush=True)
    dist.destroy_process_group()


ROOFLINE_PMC = os.path.join(ROOT, "profiles", "r06_roofline_pmc.json")
RGB_PMC = os.path.join(ROOT, "profiles", "r04_rgb_pmc.json")


def _time_launch(fn, reps=20):
    """Average duration of one launch, HIP events on torch's current stream — the stream the
    library launches on (_lib.stream_handle)."""
    for _ in range(3):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


def roofline_kernels(dev, batch, V, precision, only=None):
    """The step's GEMM kernels on the layer-6 tcn shape (C=256, T=8, 9 taps, B clips), each
    launched alone through the C ABI exactly as the step launches it:
    * "wgrad": the tcn weight gradient as the step computes it: wgrad_taps<5> (all 9 taps of a
      64x64 tile from one staged copy of each clip; split-K partials into the slab) + wgrad_slab_reduce (partials summed into dW[Cout][Cin][KT]);
      f3_conv_backward_weight(bf16). The headline roofline (the step's largest kernel share,
      profiles/r01_bf16_kernel_summary.txt);
    * "wgrad_kernel": the GEMM kernel alone (partials left in the slab), for the kernel's own fraction;
    * "tcn_fwd": the forward implicit GEMM with bf16 output (the step writes the tcn output bf16;
      its launch adds the BN-statistics/pool epilogue, EPI 13): igemm_big<1,2,4,false,true>, the
      clip-window form (two clips x 128 channels per workgroup, each channel chunk's rows staged
      once for all 9 taps).
    Algorithmic FLOP per launch = 2*M*N*K = 2 * (B*8*V) * 256 * (9*256) for all three."""
    if precision == "bf16x3":
        return roofline_kernels_x3(dev, batch, V, only)
    import fall_multimodal_amd._lib as L
    lib = L.lib()
    N, T, C, KT = batch, 8, 256, 9
    flop = 2.0 * (N * T * V) * C * (KT * C)
    peak = PEAK_MFMA_TFLOPS[precision]
    st = L.stream_handle()
    out = {}
    x = torch.randn(N, T, V, C, device=dev)
    dy = torch.randn(N, T, V, C, device=dev)
    bf = precision == "bf16"
    if bf:  # the network's bf16 GEMM operand tensors are bf16 in HBM
        x, dy = x.to(torch.bfloat16), dy.to(torch.bfloat16)
    w = torch.randn(C, C, KT, device=dev) / 48.0
    b = torch.zeros(C, device=dev)
    y = torch.empty(N, T, V, C, device=dev, dtype=torch.bfloat16 if bf else torch.float32)
    wp = torch.empty(C * KT * C, device=dev)
    prec = 3 if bf else 0  # F3_CONV_BF16_OUT: bf16 in, bf16 out (as the step)
    L.check(lib.f3_conv_forward(L.ptr(x), L.ptr(w), L.ptr(b), L.ptr(y), L.ptr(wp), N, T, V, C, C, KT, 1, 4, prec, st),
            "conv")  # packs w into wp; the timed launches reuse it (the GEMM alone)
    ms = _time_launch(lambda: lib.f3_conv_forward(L.ptr(x), None, L.ptr(b), L.ptr(y), L.ptr(wp), N, T, V, C, C, KT, 1,
                                                  4, prec, st))
    win = (N * T * V) % 288 == 0 and T * V == 144
    fname = "igemm_big<1,2,4,true> (clip window)" if win else "igemm_big<1,1,8>"
    out["tcn_fwd"] = {"kernel": f"{fname + ' bf16-out' if bf else 'conv_gemm_f32'} (tcn 9x1 fwd, C=256, T=8, "
                                f"N={N}, V={V})", "ms": ms}
    if bf:
        dw = torch.empty(C, C, KT, device=dev)
        ms = _time_launch(lambda: lib.f3_conv_backward_weight(L.ptr(dy), L.ptr(x), L.ptr(dw), None, N, T, V, C, C, KT,
                                                              1, 4, 1, st))
        taps = V % 2 == 0
        kname = "wgrad_taps<5>" if taps else "wgrad_big<4,2,4,4,64>"
        out["wgrad"] = {"kernel": f"{kname} + slab reduce (tcn 9x1 weight gradient incl. the "
                                  f"split-K reduce, C=256, T=8, N={N}, V={V})", "ms": ms}
        # the step's slab (net.cpp wgrad_slab_floats)
        cap = max(512 * 128 * 128, 16 * 256 * 256 * 9)
        slab = torch.empty(cap, device=dev)
        L.check(lib.f3_conv_wgrad_packed(L.ptr(dy), L.ptr(x), L.ptr(slab), cap, N, T, V, C, C, KT, 1, 4, st), "wgrad")
        ms = _time_launch(lambda: lib.f3_conv_wgrad_packed(L.ptr(dy), L.ptr(x), L.ptr(slab), cap, N, T, V, C, C, KT, 1, 4,
                                                           st))
        out["wgrad_kernel"] = {"kernel": f"{kname} alone (partials left in the slab, C=256, T=8, N={N}, "
                                         f"V={V})", "ms": ms}
        # the step's largest kernel share (profiles/r03_step_kernel_summary.txt): wgrad_big<4,2,4,4,64>,
        # whose largest launch is tcn layer 5's weight gradient (stride 2, T 15 -> 8, C 256): the same
        # 2*M*N*K as layer 6 (M = B*8*V output rows, K = 9*256)
        T5 = 15
        x5 = torch.randn(N, T5, V, C, device=dev).to(torch.bfloat16)
        ms = _time_launch(lambda: lib.f3_conv_backward_weight(L.ptr(dy), L.ptr(x5), L.ptr(dw), None, N, T5, V, C, C,
                                                              KT, 2, 4, 1, st))
        out["wgrad_l5"] = {"kernel": f"wgrad_big<4,2,4,4,64> + slab reduce (tcn 9x1 weight gradient incl. the split-K "
                                     f"reduce, stride 2, C=256, T=15->8, N={N}, V={V})", "ms": ms}
    return _roofline_records(out, flop, peak)


def roofline_kernels_x3(dev, batch, V, only=None):
    """bf16x3 (the headline mode): the step's largest GEMM families (the serial step profiles,
    profiles/r05_x3_step_serial_kernels_final.txt, r06_colsum_batch_serial_kernels.txt), each launched alone
    through the C ABI exactly as
    the step launches it, on operand rows [hi | lo] (f3_split_x3cat, done once outside the timing, as the
    step's producers write them) in the native split form (three bf16 MFMA products per algorithmic FLOP):
    * "dgrad_l8": the 256-channel T=8 stride-1 tcn input gradient, the clip-window form with the
      compile-time tap schedule (igemm_win1: two clips x 128 channels per workgroup, the 9 taps reading
      one staged window) and the RELUMASK epilogue the step runs — the HEADLINE: the WIN=144 input
      gradient was the step's largest serial family in round 5 (600 us/step; 3 instances and 680 us
      per step in round 6, the stride-2 ones split by output-frame parity);
    * "wgrad_l1": the 64-channel T=30 tcn weight gradient (layers 0-3), wgrad_big<2,4,2,1,32> X3F (the
      three products dy_hi x_hi, dy_lo x_hi, dy_hi x_lo from one staging of [hi | lo] rows) + the slab
      reduce — the third (500 us/step; the second is the WIN=144 forward, "tcn_fwd");
    * "wgrad_l5": the 256-channel stride-2 (T 15 -> 8) weight gradient, wgrad_big<4,2,4,4,32> X3F;
    * "wgrad" / "wgrad_kernel": the T=8 stride-1 weight gradient (wgrad_taps<5>, all 9 taps from one
      staged copy of each clip) with / without its reduce;
    * "tcn_fwd": the T=8 stride-1 forward (clip window, fp32 out + bias).
    Algorithmic FLOP per launch = 2*M*N*K of the reference's conv (M output rows, K = 9 Cin), priced
    against the dense bf16 MFMA peak; mfma_issue_frac counts the 3 products. Algorithmic bytes (the
    stored formats: [hi | lo] rows = 4 B per element, fp32 outputs and weights): wgrad = dY + X + dW,
    dgrad = dY + W + dX, fwd = X + W + Y. `only`: one key (the per-key PMC passes of
    tools/roofline_pmc.py)."""
    import fall_multimodal_amd._lib as L
    lib = L.lib()
    N, T, C, KT = batch, 8, 256, 9
    peak = PEAK_MFMA_TFLOPS["bf16x3"]
    st = L.stream_handle()
    want = (lambda k: only is None or k == only)

    def split(t):
        rows, c = t.numel() // t.shape[-1], t.shape[-1]
        out = torch.empty(rows, 2 * c, device=dev, dtype=torch.bfloat16)
        L.check(lib.f3_split_x3cat(L.ptr(t), L.ptr(out), rows, c, st), "split")
        return out

    def conv_flop(rows, cout, cin):
        return 2.0 * rows * cout * KT * cin

    out = {}
    x3 = split(torch.randn(N, T, V, C, device=dev))
    dy3 = split(torch.randn(N, T, V, C, device=dev))
    w = torch.randn(C, C, KT, device=dev) / 48.0
    b = torch.zeros(C, device=dev)
    wp = torch.empty(C * KT * C, device=dev)
    row8, row15, wbytes = N * T * V * C * 4, N * 15 * V * C * 4, C * C * KT * 4  # [hi | lo] rows: 4 B / element
    if want("tcn_fwd"):
        y = torch.empty(N, T, V, C, device=dev)
        L.check(lib.f3_conv_forward_x3cat(L.ptr(x3), L.ptr(w), L.ptr(b), L.ptr(y), L.ptr(wp), N, T, V, C, C, KT, 1, 4,
                                          st), "conv")  # packs w; the timed launches reuse it (the GEMM alone)
        ms = _time_launch(lambda: lib.f3_conv_forward_x3cat(L.ptr(x3), None, L.ptr(b), L.ptr(y), L.ptr(wp), N, T, V, C,
                                                            C, KT, 1, 4, st))
        out["tcn_fwd"] = {"kernel": f"igemm_win1<1,2,4,144,0,5> clip window, compile-time tap schedule (tcn 9x1 fwd, bf16x3, C=256, T=8, N={N}, "
                                    f"V={V})", "ms": ms, "bytes": row8 + row8 + wbytes, "flop": conv_flop(N * T * V, C, C)}
    if want("dgrad_l8"):
        # the instance the step runs (stream_backward's td): the RELUMASK epilogue reads g (fp32) and
        # BN1's coefficients, masks dv where bn1(g) <= 0 and adds the BN1-backward sums
        dx = torch.empty(N, T, V, C, device=dev)
        g = torch.randn(N, T, V, C, device=dev)
        gam, bet = torch.rand(C, device=dev) + 0.5, torch.randn(C, device=dev) * 0.1
        gd = g.reshape(-1, C).double()
        bsum, bsq = gd.sum(0), (gd * gd).sum(0)
        ssum, ssq = torch.zeros(C, dtype=torch.float64, device=dev), torch.zeros(C, dtype=torch.float64, device=dev)
        args = (L.ptr(dx), None, L.ptr(g), L.ptr(gam), L.ptr(bet), L.ptr(bsum), L.ptr(bsq), float(N * T * V),
                L.ptr(ssum), L.ptr(ssq), N, T, V, C, C, st)
        L.check(lib.f3_conv_step_x3cat(1, L.ptr(dy3), L.ptr(w), L.ptr(wp), *args), "dgrad relumask")
        ms = _time_launch(lambda: lib.f3_conv_step_x3cat(1, L.ptr(dy3), None, L.ptr(wp), *args))
        out["dgrad_l8"] = {"kernel": f"igemm_win1<16,2,4,144,0,5> clip window, compile-time tap schedule, RELUMASK epilogue (tcn 9x1 input "
                                     f"gradient as the step runs it, bf16x3, C=256, T=8, N={N}, V={V})", "ms": ms,
                           "bytes": row8 + row8 + wbytes + N * T * V * C * 4,  # + the mask operand g (fp32)
                           "flop": conv_flop(N * T * V, C, C)}
    for key, Tg, Cg in (("gcn_l5", 15, 128), ("gcn_l6", 8, 256)):
        if not want(key):
            continue
        # the 1x1 GCN contraction (stgcan.py:50-56) of skeleton layers 5 / 6 as the step runs it: the
        # graph-mixed rows [Z_hi | Z_lo] of K * C_in = 3 * Cg channels -> 256, graph-mixed bias + BN1 sums
        Kc = 3 * Cg
        z3 = split(torch.randn(N, Tg, V, Kc, device=dev))
        wg = torch.randn(C, Kc, device=dev) / math.sqrt(Kc)
        wpg = torch.empty(C * Kc, device=dev)
        og = torch.empty(N, Tg, V, C, device=dev)
        bv = torch.randn(V, C, device=dev) * 0.1
        ssum, ssq = torch.zeros(C, dtype=torch.float64, device=dev), torch.zeros(C, dtype=torch.float64, device=dev)
        args = (L.ptr(og), L.ptr(bv), None, None, None, None, None, 0.0, L.ptr(ssum), L.ptr(ssq), N, Tg, V, Kc, C, st)
        L.check(lib.f3_conv_step_x3cat(0, L.ptr(z3), L.ptr(wg), L.ptr(wpg), *args), "gcn")
        ms = _time_launch(lambda: lib.f3_conv_step_x3cat(0, L.ptr(z3), None, L.ptr(wpg), *args))
        M = N * Tg * V
        nb = M * Kc * 4 + C * Kc * 4 + M * C * 4 + V * C * 4  # Z [hi | lo], W packed, g fp32, bias
        out[key] = {"kernel": f"1x1 gcn GEMM, graph-mixed bias + BN1 sums (bf16x3, K*Cin={Kc} -> {C}, T={Tg}, "
                              f"N={N}, V={V}; igemm_big<6,1,8,0,x3n>)",
                    "ms": ms, "bytes": nb, "flop": 2.0 * M * C * Kc}
    dw = torch.empty(C, C, KT, device=dev)
    db = torch.empty(C, device=dev)
    if want("wgrad"):
        ms = _time_launch(lambda: lib.f3_conv_backward_weight_x3cat(L.ptr(dy3), L.ptr(x3), L.ptr(dw), L.ptr(db), N, T, V,
                                                                    C, C, KT, 1, 4, st))
        out["wgrad"] = {"kernel": f"wgrad_taps<5> x 3 row segments + reduce (tcn 9x1 weight gradient, bf16x3, C=256, "
                                  f"T=8, N={N}, V={V})", "ms": ms, "bytes": row8 + row8 + wbytes,
                        "flop": conv_flop(N * T * V, C, C)}
    if want("wgrad_kernel"):
        ms = _time_launch(lambda: lib.f3_conv_backward_weight_x3cat(L.ptr(dy3), L.ptr(x3), None, None, N, T, V, C, C, KT,
                                                                    1, 4, st))
        out["wgrad_kernel"] = {"kernel": f"wgrad_taps<5> x 3 row segments alone (bf16x3, partials left in the slab, "
                                         f"C=256, T=8, N={N}, V={V})", "ms": ms, "bytes": row8 + row8 + wbytes,
                               "flop": conv_flop(N * T * V, C, C)}
    if want("wgrad_l5"):
        x5 = split(torch.randn(N, 15, V, C, device=dev))
        ms = _time_launch(lambda: lib.f3_conv_backward_weight_x3cat(L.ptr(dy3), L.ptr(x5), L.ptr(dw), L.ptr(db), N, 15,
                                                                    V, C, C, KT, 2, 4, st))
        out["wgrad_l5"] = {"kernel": f"wgrad_big<4,2,4,4,32,X3F> + slab reduce (tcn 9x1 weight gradient, bf16x3, "
                                     f"stride 2, C=256, T=15->8, N={N}, V={V})", "ms": ms,
                           "bytes": row8 + row15 + wbytes, "flop": conv_flop(N * T * V, C, C)}
    if want("wgrad_l1"):
        C1, T1 = 64, 30
        x1 = split(torch.randn(N, T1, V, C1, device=dev))
        dy1 = split(torch.randn(N, T1, V, C1, device=dev))
        dw1 = torch.empty(C1, C1, KT, device=dev)
        db1 = torch.empty(C1, device=dev)
        ms = _time_launch(lambda: lib.f3_conv_backward_weight_x3cat(L.ptr(dy1), L.ptr(x1), L.ptr(dw1), L.ptr(db1), N, T1,
                                                                    V, C1, C1, KT, 1, 4, st))
        row30 = N * T1 * V * C1 * 4
        out["wgrad_l1"] = {"kernel": f"wgrad_big<2,4,2,1,32,X3F> + slab reduce (tcn 9x1 weight gradient, bf16x3, "
                                     f"C=64, T=30, N={N}, V={V})", "ms": ms,
                           "bytes": row30 + row30 + C1 * C1 * KT * 4, "flop": conv_flop(N * T1 * V, C1, C1)}
    return _roofline_records(out, None, peak, products=3)


def _gcn_roofline(roofs):
    """The north star's "MFMA utilisation for the graph GEMM against gfx950 peak": the 1x1 GCN contraction
    of skeleton layers 5 and 6 (stgcan.py:50-56) as the step launches it, MFMA fractions as the other keys
    plus its fraction of the HBM peak (the bf16x3 operand rows make it HBM-leaning: 77-128 FLOP per
    algorithmic byte against a ridge of 312 bf16 / 104 bf16x3-product FLOP per byte)."""
    if not roofs or "gcn_l5" not in roofs:
        return None
    res = {}
    for k in ("gcn_l5", "gcn_l6"):
        r = dict(roofs[k])
        if r.get("algorithmic_bytes"):
            gbs = r["algorithmic_bytes"] / (r["ms_per_launch"] * 1e-3) / 1e9
            r["hbm_achieved_gbs"] = round(gbs, 1)
            r["hbm_frac"] = round(gbs / PEAK_HBM_GBS, 4)
        res[k[4:]] = r
    return res


def _roofline_records(out, flop, peak, products=1):
    """flop: ALGORITHMIC FLOPs per launch (2*M*N*K of the reference's conv). `achieved` / `frac` are
    algorithmic: flop / time / the dense bf16 (or fp32) MFMA peak. bf16x3 issues `products` = 3 bf16
    MFMA products per algorithmic FLOP; `mfma_issue_frac` = products x frac is the matrix cores' issue
    utilisation (what rounds <= 4 reported as frac). `algorithmic_bytes`: each operand read once and
    the result written once, in the stored formats (r["bytes"]); `traffic` the PMC bytes per launch."""
    pmc = {}
    if os.path.exists(ROOFLINE_PMC):
        with open(ROOFLINE_PMC) as f:
            pmc = json.load(f)
    res = {}
    for key, r in out.items():
        fl = r.get("flop", flop)  # per-key FLOPs where the keys' shapes differ
        achieved = fl / (r["ms"] * 1e-3) / 1e12
        t = pmc.get(key, {})
        traffic = t.get("bytes_per_launch") if t.get("kernel") == r["kernel"] else None
        res[key] = {"kernel": r["kernel"], "bound": "mfma", "achieved": round(achieved, 2), "peak": peak,
                    "unit": "TFLOP/s", "frac": round(achieved / peak, 4), "traffic": traffic,
                    "flop_per_launch": fl, "ms_per_launch": round(r["ms"], 4),
                    "products_per_flop": products, "mfma_issue_frac": round(products * achieved / peak, 4),
                    "algorithmic_bytes": r.get("bytes"),
                    "traffic_over_algorithmic": None if (traffic is None or not r.get("bytes")) else
                    round(traffic / r["bytes"], 3)}
    return res


def mix_roofline(dev, batch, V, precision):
    """Graph mix of a st_gcan block (stgcan.py:54; R-GCN's A-contraction, HBM-bound) on the
    layer-1 shape (Cin=64, K=3, T=30, B clips), launched alone with the step's operand types.
    Algorithmic bytes: fwd = x + z (+A); bwd = x + dz + dx (+A, dA)."""
    import fall_multimodal_amd._lib as L
    lib = L.lib()
    K, Cin, T = 3, 64, 30
    frames = batch * T
    bf = precision == "bf16"
    x3f = 4 if precision == "bf16x3" else 0  # F3_MIX_X3: fp32 operands on the split-bf16 MFMA kernels
    et = torch.bfloat16 if bf else torch.float32
    es = 2 if bf else 4
    A = torch.rand(K, V, V, device=dev) / V
    x = torch.randn(frames, V, Cin, device=dev).to(et)
    z = torch.empty(frames, V, K, Cin, device=dev, dtype=et)
    dx = torch.empty(frames, V, Cin, device=dev)
    dA = torch.empty(K, V, V, device=dev)
    st = L.stream_handle()
    ffl = ((1 if bf else 0) | (2 if bf else 0)) | x3f
    ms_f = _time_launch(lambda: lib.f3_graph_mix_forward_ex(L.ptr(A), L.ptr(x), L.ptr(z), frames, K, V, Cin, ffl, st))
    ms_b = _time_launch(lambda: lib.f3_graph_mix_backward_ex(L.ptr(A), L.ptr(x), L.ptr(z), L.ptr(dx), L.ptr(dA), frames,
                                                             K, V, Cin, (1 if bf else 0) | x3f, st))
    nx = frames * V * Cin
    bytes_f = nx * es + nx * K * es + K * V * V * 4
    bytes_b = nx * es + nx * K * es + nx * 4 + 2 * K * V * V * 4
    bwd_kern = ("mix_bwd_bf16 (bf16 MFMA) + colsum" if bf and os.environ.get("F3_MIX_BWD_BF16", "1") != "0"
                else "mix_bwd_x3 (split-bf16 MFMA) + colsum" if x3f else "mix_bwd_lds (fp32 MFMA) + colsum")
    res = {}
    fwd_kern = ("mix_fwd_bf16 (bf16 MFMA)" if bf
                else "mix_fwd_x3 (split-bf16 MFMA, fp32 z)" if x3f else "mix_fwd_wave (fp32 MFMA)")
    for key, byt, ms, kern in (("fwd", bytes_f, ms_f, fwd_kern), ("bwd", bytes_b, ms_b, bwd_kern)):
        gbs = byt / (ms * 1e-3) / 1e9
        res[key] = {"kernel": f"{kern} (K=3, V={V}, Cin=64, frames={frames}, {precision})", "bound": "hbm",
                    "achieved": round(gbs, 1), "peak": PEAK_HBM_GBS, "unit": "GB/s",
                    "frac": round(gbs / PEAK_HBM_GBS, 4), "bytes_per_launch": byt, "ms_per_launch": round(ms, 4)}
    # the backward at the other two layer shapes of the step (128 ch at T=15, 256 ch at T=8)
    res["bwd_other_shapes"] = {}
    for cin, t in ((128, 15), (256, 8)):
        fr = batch * t
        x2 = torch.randn(fr, V, cin, device=dev).to(et)
        z2 = torch.randn(fr, V, K, cin, device=dev).to(et)
        dx2 = torch.empty(fr, V, cin, device=dev)
        ms2 = _time_launch(lambda: lib.f3_graph_mix_backward_ex(L.ptr(A), L.ptr(x2), L.ptr(z2), L.ptr(dx2), L.ptr(dA),
                                                                fr, K, V, cin, (1 if bf else 0) | x3f, st))
        n2 = fr * V * cin
        b2 = n2 * es + n2 * K * es + n2 * 4 + 2 * K * V * V * 4
        res["bwd_other_shapes"][f"Cin{cin}_T{t}"] = {"ms_per_launch": round(ms2, 4), "bytes_per_launch": b2,
                                                     "frac": round(b2 / (ms2 * 1e-3) / 1e9 / PEAK_HBM_GBS, 4)}
    return res


def sensor_bench(dev, precision="fp32"):
    """The sensor models on their own: BASELINE config 1 (sensor-only CNN_BiLSTM, UR-Fall, S=4,
    B=32, GSTCAN_UR_sensor.ipynb:572-586) training-step throughput, and the north-star sensor
    branch's BiLSTM (bilstm.py:21-59, S=6, T=30, B=256) per-recurrent-step latency: the
    BiLSTM-only model's forward and fwd+bwd step divided by the 30 dependent steps (each
    direction runs concurrently; the head kernels are included, so these are upper bounds)."""
    import fall_multimodal_amd as f3
    res = {}
    g = torch.Generator().manual_seed(5)
    for name, model, B, S in (("cfg1_cnn_bilstm", f3.CNN_BiLSTM(device=dev), 32, 4),
                              ("bilstm_S6", f3.BiLSTM(6, num_classes=11, device=dev), 256, 6)):
        C = model.spec.num_class
        x = torch.randn(B, 30, S, generator=g).to(dev)
        lab = torch.softmax(torch.randn(B, C, generator=g), 1).to(dev)
        step = f3.TrainStep(model, B, lr=1e-3)
        out = torch.empty(B, C, device=dev)
        ws = step.ws
        for _ in range(3):
            step(None, x, lab)
        torch.cuda.synchronize()
        reps = 50
        t0 = time.perf_counter()
        for _ in range(reps):
            step(None, x, lab)
        torch.cuda.synchronize()
        dt_step = (time.perf_counter() - t0) / reps
        t0 = time.perf_counter()
        for _ in range(reps):
            model.native_forward(None, x, out, ws, True)
        torch.cuda.synchronize()
        dt_fwd = (time.perf_counter() - t0) / reps
        res[name] = {"batch": B, "sensor_dim": S, "clips_per_s": round(B / dt_step, 1),
                     "ms_per_step": round(dt_step * 1e3, 4), "fwd_ms": round(dt_fwd * 1e3, 4),
                     "lstm_fwd_us_per_recurrent_step": round(dt_fwd * 1e6 / 30, 2),
                     "lstm_step_us_per_recurrent_step": round(dt_step * 1e6 / 30, 2)}
        if name == "cfg1_cnn_bilstm":
            res[name]["cnn1d"] = cnn1d_stage_times(model, step, x, lab, B, S)
    m256 = f3.CNN_BiLSTM(device=dev)
    x256 = torch.randn(256, 30, 4, generator=g).to(dev)
    lab256 = torch.softmax(torch.randn(256, m256.spec.num_class, generator=g), 1).to(dev)
    res["cnn1d_B256"] = cnn1d_stage_times(m256, f3.TrainStep(m256, 256, lr=1e-3), x256, lab256, 256, 4)
    return res


def cnn1d_stage_times(model, step, x, lab, B, S, T=30, reps=20):
    """Time of the sensor CNN1D (GSTCAN_UR_conv.ipynb:493-514: Conv1d(S->16,k5) BN ReLU MaxPool,
    Conv1d(16->32,k5) BN ReLU MaxPool) in the training step, from HIP events around its launches on
    the sensor queue (f3_net_sensor_times), mean over `reps` steps. Since round 5 each direction is
    ONE cooperative launch (sensor.hip cnn1d_coop_*: the BatchNorm statistics and weight gradients
    reduced across workgroups after group barriers). Algorithmic bytes (fp32, each tensor once):
    forward x + w1 + y1 + p1 + w2 + y2 + p2; backward dp2 + y2 + dy2 + p1 + w2 + dW2 + y1 + dy1 + x +
    dW1. The tensors are 0.02-1 MB, so the launches are latency-bound (barriers, not bytes)."""
    import ctypes
    import fall_multimodal_amd._lib as FL
    L, check = FL.lib(), FL.check
    h = model._native.h
    f32 = 4
    acc = [0.0] * 2
    check(L.f3_net_sensor_times(h, 1, None), "sensor times on")
    for _ in range(3):
        step(None, x, lab)
    torch.cuda.synchronize()
    ms = (ctypes.c_float * 2)()
    for _ in range(reps):
        step(None, x, lab)
        check(L.f3_net_sensor_times(h, 1, ms), "sensor times")
        for i in range(2):
            acc[i] += ms[i] / reps
    check(L.f3_net_sensor_times(h, 0, None), "sensor times off")
    T2, T3 = T // 2, (T // 2) // 2
    xb, y1, p1, y2, p2 = (B * T * S * f32, B * T * 16 * f32, B * T2 * 16 * f32, B * T2 * 32 * f32,
                          B * T3 * 32 * f32)
    w1, w2 = 16 * S * 5 * f32, 32 * 16 * 5 * f32
    nbytes = {"forward": xb + w1 + y1 + p1 + w2 + y2 + p2,
              "backward": p2 + 2 * y2 + p1 + 2 * w2 + 2 * y1 + xb + 2 * w1}
    out = {}
    for i, nm in enumerate(nbytes):
        us = acc[i] * 1e3
        out[nm] = {"us": round(us, 2), "bytes": nbytes[nm], "GBps": round(nbytes[nm] / (us * 1e-6) / 1e9, 1)}
    out["total_us"] = round(sum(acc) * 1e3, 2)
    out["batch"] = B
    out["form"] = "one cooperative launch per direction (group barriers for the BatchNorm statistics)"
    out["note"] = ("HIP events around the launch on the sensor queue; latency-bound (tensors of 0.02-1 MB): "
                   "GB/s against 8 TB/s is not a meaningful fraction here")
    return out


def eval_throughput(model, sk, se, reps=20):
    """Eval step: the eval-mode forward (BN running statistics) of the same
    B clips, as model/main.py's valid/test loops run it; clips/s over `reps` forwards."""
    B = sk.shape[0]
    out = torch.empty(B, model.spec.num_class, device=sk.device)
    ws = torch.empty(model._native.workspace_bytes(B), dtype=torch.uint8, device=sk.device)
    for _ in range(3):
        model.native_forward(sk, se, out, ws, False)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        model.native_forward(sk, se, out, ws, False)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / reps
    return {"clips_per_s": round(B / dt, 1), "ms_per_batch": round(dt * 1e3, 3), "batch": B}


def autograd_path_bench(model, sk, se, lb, steps=5):
    """The reference driver's loop body unchanged (model/main.py:112-127): out = model(data, sensor)
    through the fall3::net_forward custom op, CrossEntropyLoss, loss.backward() (fall3::net_backward),
    optimizer.step() with fall3 RMSprop (one fall3::rmsprop_ over the flat parameter range), zero_grad."""
    import fall_multimodal_amd as f3
    opt = f3.RMSprop(model.parameters(), lr=1e-3)
    loss_fn = torch.nn.CrossEntropyLoss()

    def one():
        opt.zero_grad()
        loss = loss_fn(model(sk, se), lb)
        loss.backward()
        opt.step()

    for _ in range(3):
        one()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        one()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / steps
    return {"ms_per_step": round(dt * 1e3, 3), "clips_per_s": round(sk.shape[0] / dt, 1), "steps": steps,
            "path": "model(data, sensor) -> CrossEntropyLoss -> backward -> RMSprop.step (torch.library ops)"}


def replica_seconds(fn, steps, warmup):
    """Seconds per step of fn over `steps` timed calls after `warmup`, bracketed by barrier +
    synchronize on both sides and maxed over ranks when torch.distributed is initialised (the
    replicas-only configs: every rank runs its own independent step, no collective)."""
    world = dist.get_world_size() if dist.is_available() and dist.is_initialized() else 1
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        fn()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([dt], device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    return dt / steps, world


def targcn_bench(dev, B=256, V=17, steps=10, warmup=3, precision="bf16", cpu_seconds=0.0):
    """BASELINE config 2: skeleton-only TARGCN (TRAGCN.py:177-224, V=17 joints, T=30, bf16 GEMM
    operands) training step (fwd + CE + bwd + RMSprop) at B=256 on one GPU, synthetic clips,
    random-init weights. ms_per_step is the whole step; the recurrence is 2 layers x 30 dependent
    GRU steps forward and backward (per-kernel times: profiles/r02_targcn_kernel_summary.txt)."""
    import fall_multimodal_amd as f3
    from oracle import targcn_cpu as tg
    src, lab = tg.synthetic_source(B, V, 11, 3)
    model = f3.TARGCN(num_nodes=V, device=dev, precision=precision)
    step = f3.TargcnStep(model, B, lr=1e-5)
    x, y = torch.from_numpy(src).to(dev), torch.from_numpy(lab).to(dev)
    dt, world = replica_seconds(lambda: step(x, y), steps, warmup)
    stages = targcn_stage_times(model, step, x, y, B, V, precision)
    rec = {"metric": "clips/sec (fwd+bwd) TARGCN skeleton-only, B=256, 1 GPU", "value": round(world * B / dt, 1),
           "unit": "clips/s", "n_gpus": world, "scaling": "weak", "ms_per_step": round(dt * 1e3, 3),
           "dtype": precision, "steps": steps,
           "config": {"workload": f"targcn_V{V}_T30_B{B}", "global_batch": world * B, "joints": V, "frames": 30,
                      "gru_layers": 2, "hidden": 64, "ta_layers": 2, "parallelism": f"replicas{world}"},
           "final_loss": round(float(step.loss.item()), 5), "stages": stages}
    if cpu_seconds > 0:  # the oracle (pinned bit-exactly to the reference) on this host's cores
        threads = cpu_threads()
        torch.set_num_threads(threads)
        st = tg.init_state(V, 7)
        Bc = B
        s_c, l_c = (torch.from_numpy(a) for a in tg.synthetic_source(Bc, V, 11, 1))
        tg.train_step(st, s_c, l_c)
        t0, n = time.perf_counter(), 0
        while n < 1 or (time.perf_counter() - t0 < cpu_seconds and n < 20):
            tg.train_step(st, s_c, l_c)
            n += 1
        rec["cpu_baseline"] = {"value": round(Bc * n / (time.perf_counter() - t0), 2), "unit": "clips/s",
                               "cores": threads, "kind": "port",
                               "sample": f"{n} oracle train steps of B={Bc}, V={V}, fp32, torch CPU"}
    return rec


def targcn_stage_times(model, step, x, y, B, V, precision, reps=5):
    """The recurrences and TA layers of one TARGCN step, timed with HIP events on the step's stream
    (f3_targcn_stage_times), averaged over `reps` steps. R-GRU is latency-bound: its
    figure is us per recurrent step (kernel time / 30 dependent steps); the achieved GB/s of each
    recurrence kernel is also given, from its algorithmic bytes: every row it must read and write once
    (R = B*T*V rows; forward writes H, sigmoid gates, static gate, tanh update, static update (fp32)
    and the four EmbGCN operand rows (operand type, 128 wide); backward reads the five saved fp32
    tensors and dH, writes the four pre-activation gradients and two mixed-input gradients (operand
    type) and dX (layer 1))."""
    import ctypes
    import fall_multimodal_amd._lib as L
    lib, h = L.lib(), model._native.h
    acc = np.zeros(8)
    L.check(lib.f3_targcn_stage_times(h, 1, None), "stage times")
    for _ in range(reps):
        step(x, y)
        ms = (ctypes.c_float * 8)()
        L.check(lib.f3_targcn_stage_times(h, 1, ms), "stage times")
        acc += np.array(ms[:])
    L.check(lib.f3_targcn_stage_times(h, 0, None), "stage times")
    acc /= reps
    R, T, es = B * 30 * V, 30, (2 if precision == "bf16" else 4)
    fwd_row = [4 * 3 + 4 * (64 + 128 + 128 + 64 + 64) + es * 4 * 128, 4 * 64 + 4 * (64 + 128 + 128 + 64 + 64) + es * 4 * 128]
    bwd_row = [4 * (64 + 128 + 128 + 64 + 64) + 4 * 64 + es * (128 * 2 + 64 * 2 + 2 * 128),
               4 * (64 + 128 + 128 + 64 + 64) + 4 * 64 + es * (128 * 2 + 64 * 2 + 2 * 128) + 4 * 64]
    out = {}
    for i, (name, row) in enumerate((("gru_fwd_l0", fwd_row[0]), ("gru_fwd_l1", fwd_row[1]))):
        out[name] = {"ms": round(acc[i], 4), "us_per_recurrent_step": round(acc[i] * 1e3 / T, 2),
                     "GBps": round(R * row / (acc[i] * 1e-3) / 1e9, 1), "bytes": R * row}
    for i, name in ((6, "gru_bwd_l1"), (7, "gru_bwd_l0")):
        row = bwd_row[1] if name.endswith("l1") else bwd_row[0]
        out[name] = {"ms": round(acc[i], 4), "us_per_recurrent_step": round(acc[i] * 1e3 / T, 2),
                     "GBps": round(R * row / (acc[i] * 1e-3) / 1e9, 1), "bytes": R * row}
    for i, name in ((2, "ta_fwd_l0"), (3, "ta_fwd_l1"), (4, "ta_bwd_l1"), (5, "ta_bwd_l0")):
        out[name] = {"ms": round(acc[i], 4)}
    out["note"] = ("HIP events around each launch on the step's stream (f3_targcn_stage_times), mean of "
                   f"{reps} steps; R-GRU is latency-bound: 30 dependent steps per layer")
    return out


def sktr_bench(dev, B=256, steps=10, warmup=3, cpu_seconds=0.0, precision="bf16"):
    """BASELINE config 5: SkeletonTransformer(3, 14, 30, 11, 32, 6, 16, 8) training step (fwd + CE +
    bwd + RMSprop, train-mode FFN dropout and stochastic depth) at B=256 on one GPU, synthetic clips,
    random-init weights. precision "bf16" (BASELINE cfg 5): the block Linears on bf16 MFMA, fp32
    accumulate; "fp32": fp32 MFMA (the parity mode, also reported). The 10-fold CV shards folds over
    GPUs as independent replicas (no collective), so per-GPU throughput is the whole story."""
    import fall_multimodal_amd as f3
    from fall_multimodal_amd.cv import folds_of_rank, kfold_indices
    from oracle import sktr_cpu as sk
    # the rank's CV fold (cv.py: rank r runs folds r, r + world, ...; no collective): synthetic HAR-30
    # windows in videos of 30, 10-fold split by video (cv_dataloader.py:155-167); the timed steps cycle
    # through the fold's training windows, pre-gathered into resident B-clip batches
    on = dist.is_available() and dist.is_initialized()
    rank_, world_ = (dist.get_rank(), dist.get_world_size()) if on else (0, 1)
    nwin = B * 12
    x_all, lab_all = sk.synthetic_clips(nwin, 14, 11, 3)
    folds = kfold_indices([f"v{i // 30:03d}" for i in range(nwin)], seed=42)
    mine = folds_of_rank(len(folds), rank_ % len(folds), min(world_, len(folds)))
    tr = folds[mine[0]][0]
    perm = np.random.default_rng(mine[0]).permutation(tr)
    nb = len(perm) // B
    xb = [torch.from_numpy(x_all[perm[i * B:(i + 1) * B]]).to(dev) for i in range(nb)]
    yb = [torch.from_numpy(lab_all[perm[i * B:(i + 1) * B]]).to(dev) for i in range(nb)]
    x, lab = x_all[perm[:B]], lab_all[perm[:B]]
    model = f3.SkeletonTransformer(device=dev, precision=precision)
    step = f3.SktrStep(model, B)
    xd, yd = xb[0], yb[0]
    it = [0]

    def fold_step():
        i = it[0] % nb
        it[0] += 1
        step(xb[i], yb[i])

    dt, world = replica_seconds(fold_step, steps, warmup)
    fp32_ms = None
    if precision != "fp32":  # the parity mode's step time beside it
        m32 = f3.SkeletonTransformer(device=dev)
        s32 = f3.SktrStep(m32, B)
        fp32_ms = round(replica_seconds(lambda: s32(xd, yd), steps, warmup)[0] * 1e3, 3)
        del s32, m32
    rec = {"metric": "clips/sec (fwd+bwd) SkeletonTransformer, B=256, 1 GPU (one CV fold)",
           "value": round(world * B / dt, 1), "unit": "clips/s", "n_gpus": world, "scaling": "weak",
           "ms_per_step": round(dt * 1e3, 3), "dtype": precision, "steps": steps,
           "config": {"workload": f"sktr_V14_T30_M1_B{B}", "global_batch": world * B, "joints": 14, "frames": 30,
                      "blocks": 6, "heads": 8,
                      "parallelism": f"folds over ranks (world {world}, 10-fold CV by video, no collective)",
                      "folds_rank0": mine, "fold_train_windows": int(len(tr)), "fold_batches": nb},
           "final_loss": round(float(step.loss.item()), 5), "fp32_mode_ms_per_step": fp32_ms}
    if cpu_seconds > 0:  # the oracle (pinned to the reference) on this host's cores
        threads = cpu_threads()
        torch.set_num_threads(threads)
        st = sk.init_state(7)
        xc, lc = torch.from_numpy(x), torch.from_numpy(lab)
        sk.train_step(st, xc[:16], lc[:16])
        t0, n = time.perf_counter(), 0
        while n < 1 or (time.perf_counter() - t0 < cpu_seconds and n < 10):
            sk.train_step(st, xc, lc)
            n += 1
        rec["cpu_baseline"] = {"value": round(B * n / (time.perf_counter() - t0), 2), "unit": "clips/s",
                               "cores": threads, "kind": "port",
                               "sample": f"{n} oracle train steps of B={B}, fp32, torch CPU"}
    return rec


def musa_bench(dev, B=256, steps=10, warmup=3, cpu_seconds=0.0, precision="bf16"):
    """The model the root Multimodal_Fall3/main.py trains (musa_model.Model, main.py:307-320: 14 joints,
    30 frames, two streams, DropBlocks, RMSprop) — training step (fwd + CE + bwd + RMSprop) at B=256 on
    one GPU, fp32, synthetic clips; plus the HBM roofline of its depthwise temporal Conv1D."""
    import fall_multimodal_amd as f3
    import fall_multimodal_amd._lib as L
    from oracle.prng import synthetic_batch
    x, _, lab = synthetic_batch(B, 14, 11, 1, 9)
    model = f3.musa.Model(11, 14, 300, f3.musa.adjGraph("coco_cut", "uniform"), True, True, 41, device=dev,
                          precision=precision)
    step = f3.musa.MusaStep(model, B)
    xd, yd = torch.from_numpy(x).to(dev), torch.from_numpy(lab).to(dev)
    dt, world = replica_seconds(lambda: step(xd, yd), steps, warmup)
    fp32_ms = None
    if precision != "fp32":  # the parity mode's step time beside it
        m32 = f3.musa.Model(11, 14, 300, f3.musa.adjGraph("coco_cut", "uniform"), True, True, 41, device=dev)
        s32 = f3.musa.MusaStep(m32, B)
        fp32_ms = round(replica_seconds(lambda: s32(xd, yd), steps, warmup)[0] * 1e3, 3)
        del s32, m32
    rec = {"metric": "clips/sec (fwd+bwd) musa_model.Model (root Multimodal_Fall3/main.py), B=256, 1 GPU",
           "value": round(world * B / dt, 1), "unit": "clips/s", "n_gpus": world, "scaling": "weak",
           "ms_per_step": round(dt * 1e3, 3), "dtype": precision,
           "steps": steps, "config": {"workload": f"musa_V14_T30_B{B}", "global_batch": world * B, "joints": 14,
                                      "frames": 30, "dropblock": True, "parallelism": f"replicas{world}"},
           "final_loss": round(float(step.loss.item()), 5), "fp32_mode_ms_per_step": fp32_ms}
    if dist.is_available() and dist.is_initialized() and dist.get_rank() != 0:
        return rec
    # depthwise temporal conv roofline (SepTemporal_Block depth_conv, C=128, V=14, T=30, B clips):
    # algorithmic bytes = x + y (+ w, b); the BatchNorm sums are fused in the epilogue
    lib, st = L.lib(), L.stream_handle()
    roofs = {}
    for K, S in ((3, 1), (5, 2)):
        C, T, V = 128, 30, 14
        xin = torch.randn(B, T, V, C, device=dev)
        To = (T + (K - 1) - K) // S + 1
        y = torch.empty(B, To, V, C, device=dev)
        w = torch.randn(C, K, device=dev)
        bb = torch.randn(C, device=dev)
        sums = torch.zeros(2 * C, dtype=torch.float64, device=dev)
        fn = lambda: lib.f3_dwconv_t_forward(L.ptr(xin), L.ptr(w), L.ptr(bb), L.ptr(y), L.ptr(sums), B, T, V, C, K,  # noqa: E731
                                             S, (K - 1) // 2, st)
        L.check(fn(), "dwconv")
        ms = _time_launch(fn)
        ms_nosum = _time_launch(lambda: lib.f3_dwconv_t_forward(L.ptr(xin), L.ptr(w), L.ptr(bb), L.ptr(y), None, B, T,
                                                                V, C, K, S, (K - 1) // 2, st))
        byt = 4 * (xin.numel() + y.numel() + w.numel() + bb.numel())
        gbs = byt / (ms * 1e-3) / 1e9
        roofs[f"k{K}_s{S}"] = {"kernel": f"mu_dwconv_fwd_kernel<{K}> (C={C}, V={V}, T={T}->{To}, N={B}, fp32, "
                                         f"BN sums fused)", "bound": "hbm", "achieved": round(gbs, 1),
                               "peak": PEAK_HBM_GBS, "unit": "GB/s", "frac": round(gbs / PEAK_HBM_GBS, 4),
                               "bytes_per_launch": byt, "ms_per_launch": round(ms, 4),
                               "ms_without_bn_sums": round(ms_nosum, 4)}
    rec["roofline_dwconv_t"] = roofs
    if cpu_seconds > 0:  # the oracle (pinned to the reference) on this host's cores
        from oracle import musa_cpu as mu
        threads = cpu_threads()
        torch.set_num_threads(threads)
        stc = mu.init_state(7)
        xc, lc = torch.from_numpy(x), torch.from_numpy(lab)
        mu.train_step(stc, xc[:16], lc[:16])
        t0, n = time.perf_counter(), 0
        while n < 1 or (time.perf_counter() - t0 < cpu_seconds and n < 10):
            mu.train_step(stc, xc, lc, draws=n + 1)
            n += 1
        rec["cpu_baseline"] = {"value": round(B * n / (time.perf_counter() - t0), 2), "unit": "clips/s",
                               "cores": threads, "kind": "port",
                               "sample": f"{n} oracle train steps of B={B}, fp32, torch CPU"}
    return rec


def loader_bench(model, dev, B=256, V=18, S=6, C=11, n=20480):
    """The data step in front of the hot path: data.WindowLoader over synthetic
    windows in the reference's format (n windows, shuffled, drop_last), timed alone (gather into
    pinned buffers + async H2D on a copy stream) and feeding the training step, per epoch."""
    import fall_multimodal_amd as f3
    from fall_multimodal_amd.data import Windows, WindowLoader
    rng = np.random.default_rng(3)
    w = Windows([f"v{i // 40}" for i in range(n)], rng.standard_normal((n, 30, V, 3), dtype=np.float32),
                rng.standard_normal((n, 30, S), dtype=np.float32),
                np.eye(C, dtype=np.float32)[rng.integers(0, C, n)])
    loader = WindowLoader(w, B, shuffle=True, drop_last=True, device=dev, generator=torch.Generator().manual_seed(1))
    for _ in loader:  # warm the pinned allocator
        pass
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    nb = 0
    for sk, se, lb in loader:
        nb += 1
    torch.cuda.synchronize()
    t_load = time.perf_counter() - t0
    step = f3.TrainStep(model, B, lr=1e-3)
    it = iter(loader)
    step(*next(it))
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    ns = 0
    for sk, se, lb in it:
        step(sk, se, lb)
        ns += 1
    torch.cuda.synchronize()
    t_fed = time.perf_counter() - t0
    return {"windows": n, "batch": B, "loader_only_clips_per_s": round(nb * B / t_load, 1),
            "train_fed_clips_per_s": round(ns * B / t_fed, 1),
            "note": "one epoch of data.WindowLoader (shuffle, drop_last, pinned gather + async H2D) alone, "
                    "then feeding TrainStep batch by batch"}


# The reference's own code timed on CPU: a reported, non-target figure
REFERENCE_CPU = {"value": 77.4, "unit": "clips/s", "cores": 8, "kind": "reference",
                 "sample": "reference TwoStreamSTGCAN_BiLSTM (HAR V=14, S=15, 11 classes) fwd+bwd+RMSprop at B=256, "
                           "torch CPU fp32, 3.308 s/step, timed in the survey container (BASELINE.md 2a)"}


MODE_NOTES = {
    "fp32": "fp32 MFMA GEMMs (v_mfma_f32_16x16x4_f32), fp32 activations; logits within 1e-3 of the reference CPU "
            "run with identical argmax (tests/test_gpu_parity.py)",
    "bf16": "bf16 GEMM operands and activations in HBM, fp32 accumulate: the faster mode, NOT parity-meeting "
            "(logits ~4e-3 from the fp64 oracle at B=256, above the north star's 1e-3; tests/test_gpu_parity.py)",
}


def fp32_mode_bench(dev, a, V, S, C, sk, se, lb, steps=10, warmup=3, precision="fp32"):
    """Another precision mode's throughput on the same step and config (fp32: every GEMM on fp32
    MFMA; bf16: bf16 operands), beside the headline mode."""
    import fall_multimodal_amd as f3
    model = f3.TwoStreamSTGCAN_BiLSTM(3, {"layout": a.layout, "strategy": "spatial"}, C, S, device=dev,
                                      precision=precision)
    step = f3.TrainStep(model, sk.shape[0], lr=1e-3)
    for _ in range(warmup):
        step(sk, se, lb)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        step(sk, se, lb)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / steps
    B = sk.shape[0]
    fl = FLOP_PER_CLIP.get((V, S))
    res = {"ms_per_step": round(dt * 1e3, 3), "clips_per_s": round(B / dt, 1), "steps": steps, "dtype": precision,
           "note": MODE_NOTES[precision]}
    if fl:
        res[f"step_mfma_frac_of_{precision}_peak"] = round(B * fl / dt / 1e12 / PEAK_MFMA_TFLOPS[precision], 4)
    del step, model
    torch.cuda.empty_cache()
    return res


def cpu_threads():
    """The CPU share this process may use: OMP_NUM_THREADS (16 on the GPU box, whose nproc shows
    the whole machine), else every core here."""
    env = os.environ.get("OMP_NUM_THREADS")
    n = os.cpu_count() or 1
    return max(1, min(n, int(env))) if env and env.isdigit() else n


def cpu_baseline(layout, V, S, seconds):
    """The oracle (CPU PyTorch restatement, pinned to the reference) on this host's cores, at the
    benchmarked batch (B=256)."""
    from oracle import model_cpu as oc
    from oracle.prng import synthetic_batch
    threads = cpu_threads()
    torch.set_num_threads(threads)
    spec = oc.Spec(model="two_stgcan_bilstm", layout=layout, num_class=11, sensor_dim=S)
    st = oc.init_state(spec, 7)
    B = 256
    sk, se, lb = (torch.from_numpy(x) for x in synthetic_batch(B, V, 11, S, 1))
    oc.train_step(st, spec, *(torch.from_numpy(x) for x in synthetic_batch(16, V, 11, S, 2)))  # warm-up
    t0 = time.perf_counter()
    n = 0
    while n < 1 or (time.perf_counter() - t0 < seconds and n < 50):
        oc.train_step(st, spec, sk, se, lb)
        n += 1
    dt = time.perf_counter() - t0
    return {"value": round(B * n / dt, 2), "unit": "clips/s", "cores": threads, "kind": "port",
            "sample": f"{n} train steps (fwd+CE+bwd+RMSprop) of B={B}, V={V}, S={S}, fp32, torch CPU"}


def rgb_bench(dev, B=256, T=30, reps=10):
    """The build-defined RGB spatial-conv branch (fall_multimodal_amd/rgb.py, csrc/rgb.hip; PARITY
    UNPINNED: the reference has no RGB model arithmetic, SURVEY.md 8a R-RGB) on the north-star batch:
    B=256 clips x T=30 channels-last bf16 224x224x3 frames (2.31 GB resident in HBM). Both kernels
    stream the frames once (algorithmic bytes = the frame bytes; weights, bias and per-block partial
    rows are < 0.1% of it), so each is priced against HBM."""
    import fall_multimodal_amd.rgb as rgbm
    frames = torch.empty(B, T, 224, 224, 3, dtype=torch.bfloat16, device=dev).uniform_()
    conv = rgbm.RGBSpatialConv(device=dev)
    w, b = conv.weight.detach(), conv.bias.detach()
    dfeat = torch.randn(B, 64, device=dev)
    s = torch.cuda.current_stream(dev)

    def timed(fn):
        for _ in range(2):
            fn()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        for _ in range(reps):
            fn()
        e1.record(s)
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / reps / 1e3

    t_f = timed(lambda: torch.ops.fall3.rgb_forward(frames, w, b))
    t_b = timed(lambda: torch.ops.fall3.rgb_backward(frames, w, b, dfeat))
    nbytes = frames.numel() * 2
    out = {"workload": f"rgb_spatial_conv_B{B}_T{T}_224x224x3_bf16", "parity": "unpinned (build-defined branch)",
           "clips_per_s_fwd_bwd": round(B / (t_f + t_b), 1), "fwd_ms": round(t_f * 1e3, 4), "bwd_ms": round(t_b * 1e3, 4),
           "bytes_per_pass": nbytes}
    pmc = {}
    if os.path.exists(RGB_PMC):  # HBM bytes per launch from rocprofv3 PMC (tools/rgb_pmc.py)
        with open(RGB_PMC) as f:
            pmc = json.load(f)
    for k, t in (("fwd", t_f), ("bwd", t_b)):
        out["roofline_" + k] = {"bound": "hbm", "achieved": round(nbytes / t / 1e9, 1), "peak": PEAK_HBM_GBS,
                                "unit": "GB/s", "frac": round(nbytes / t / 1e9 / PEAK_HBM_GBS, 4),
                                "traffic": (pmc.get(k) or {}).get("bytes_per_launch")}
    del frames
    torch.cuda.empty_cache()
    return out


def rgb_step_bench(dev, a, V, S, C, sk, se, lb, steps=10, warmup=3):
    """The north-star workload as ONE training step WITH the RGB branch (rgb.Fall3RGBStep): the
    3-stream model (skeleton x2 + IMU, the headline's precision) plus the build-defined RGB
    spatial-conv branch (B x 30 channels-last bf16 224x224x3 frames, resident in HBM), fused by adding
    logits, one CE, both backwards, RMSprop over both parameter sets. The RGB branch runs on its own
    HIP stream beside the skeleton / sensor queues. RGB parity is unpinned (no reference arithmetic)."""
    import fall_multimodal_amd as f3
    from fall_multimodal_amd.rgb import Fall3RGBStep, Fall3WithRGB
    B = sk.shape[0]
    frames = torch.empty(B, 30, 224, 224, 3, dtype=torch.bfloat16, device=dev).uniform_()
    base = f3.TwoStreamSTGCAN_BiLSTM(3, {"layout": a.layout, "strategy": "spatial"}, C, S, device=dev,
                                     precision=a.precision)
    step = Fall3RGBStep(Fall3WithRGB(base, C, device=dev), B, lr=1e-3)
    for _ in range(warmup):
        step(sk, se, frames, lb)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        step(sk, se, frames, lb)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / steps
    res = {"workload": f"fall3_3stream_plus_rgb_{a.layout}_V{V}_S{S}_B{B}_T30_224x224x3", "dtype": a.precision,
           "ms_per_step": round(dt * 1e3, 3), "clips_per_s": round(B / dt, 1), "steps": steps,
           "final_loss": round(float(step.loss.item()), 5), "rgb_parity": "unpinned (build-defined branch)",
           "note": "skeleton (2 ST-GCAN streams) + IMU BiLSTM + RGB conv branch as ONE step; RGB on its own stream"}
    del step, base, frames
    torch.cuda.empty_cache()
    return res


def model_leg(model, a):
    """One of the other BASELINE configs (cfg 2 TARGCN, cfg 5 SkeletonTransformer, musa_model) timed
    in a fresh child process (`bench.py --model M`, its own line embedded here): measured inside this
    process after the 3-stream, fp32-mode and roofline legs, the TARGCN step read 8.4 ms against 6.7 ms
    alone (profiles/r03_bench.json vs r03_bench_tg_alone.json)."""
    cmd = [sys.executable, os.path.abspath(__file__), "--model", model, "--steps", "10", "--warmup", "3",
           "--precision", "bf16"]
    if a.no_cpu_baseline:
        cmd.append("--no-cpu-baseline")
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run(cmd, capture_output=True, text=True, env=env, timeout=600)
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    if r.returncode != 0 or not lines:
        raise SystemExit(f"bench.py: the --model {model} leg failed (status {r.returncode}): {r.stderr[-2000:]}")
    rec = json.loads(lines[-1])
    rec["process"] = "fresh child process (bench.py --model %s)" % model
    return rec


def main():
    a = parse()
    if "WORLD_SIZE" not in os.environ and a.gpus > 1:
        sys.exit(launch_ranks(a))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != a.gpus:
        raise SystemExit(f"bench.py: --gpus {a.gpus} but the launcher started {world} rank(s)")
    if a.launch_check:
        launch_check(world, rank)
        return
    if world > 1:
        from fall_multimodal_amd.train import rccl_options
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", pg_options=rccl_options())   # RCCL on a high-priority queue
    dev = torch.device("cuda", local)
    torch.manual_seed(1234 + rank)

    import fall_multimodal_amd as f3
    from oracle.prng import synthetic_batch

    if a.model == "targcn":
        rec = targcn_bench(dev, steps=a.steps, warmup=a.warmup, precision=a.precision,
                           cpu_seconds=0.0 if (a.no_cpu_baseline or world > 1) else 6.0)
        if rank == 0:
            print(json.dumps(rec), flush=True)
        return
    if a.model == "musa":
        rec = musa_bench(dev, steps=a.steps, warmup=a.warmup, cpu_seconds=0.0 if (a.no_cpu_baseline or world > 1) else 6.0,
                         precision=a.precision)
        if rank == 0:
            print(json.dumps(rec), flush=True)
        return
    if a.model == "sktr":
        rec = sktr_bench(dev, steps=a.steps, warmup=a.warmup, cpu_seconds=0.0 if (a.no_cpu_baseline or world > 1) else 6.0,
                         precision=a.precision)
        if rank == 0:
            print(json.dumps(rec), flush=True)
        return
    V = 18 if a.layout == "coco_mmpose" else 14
    B, S, C = a.batch, a.sensor_dim, 11
    model = f3.TwoStreamSTGCAN_BiLSTM(3, {"layout": a.layout, "strategy": "spatial"}, C, S, device=dev,
                                      precision=a.precision)
    if world > 1:  # identical replicas
        dist.broadcast(model.flat_parameters(), 0)
    step = f3.TrainStep(model, B, lr=1e-3)
    sk, se, lb = (torch.from_numpy(x).to(dev) for x in synthetic_batch(B, V, C, S, 100 + rank))
    if a.graph and not a.no_graph:
        step.capture(sk, se, lb)
    for _ in range(a.warmup):
        step(sk, se, lb)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        step(sk, se, lb)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([dt], device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    loss = float(step.loss.item())
    phased = None
    if world == 1 and rank == 0:  # the data-parallel two-phase backward's own cost, measured on one GPU
        step.phased = True
        for _ in range(2):
            step(sk, se, lb)
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        for _ in range(a.steps):
            step(sk, se, lb)
        torch.cuda.synchronize()
        step.phased = False
        pm = (time.perf_counter() - t1) / a.steps * 1e3
        phased = {"ms_per_step": round(pm, 3), "vs_phase0": round(pm / (dt / a.steps * 1e3), 4),
                  "note": "backward as phase 1 (head, sensor, layers 4-6) + phase 2 (layers 0-3), the DP path "
                          "without the collective; phase 0 = the one-pass backward the N=1 value uses"}
    one = rank == 0 and world == 1
    fp32m = fp32_mode_bench(dev, a, V, S, C, sk, se, lb) if (one and a.precision != "fp32") else None
    bf16m = fp32_mode_bench(dev, a, V, S, C, sk, se, lb, precision="bf16") if (one and a.precision == "bf16x3") else None
    ev = eval_throughput(model, sk, se) if rank == 0 else None
    agp = autograd_path_bench(model, sk, se, lb, steps=a.steps) if (rank == 0 and world == 1) else None
    roofs = roofline_kernels(dev, B, V, a.precision) if rank == 0 else None
    legs = rank == 0 and world == 1 and not a.no_targcn
    tgrec = model_leg("targcn", a) if legs else None
    skrec = model_leg("sktr", a) if legs else None
    murec = model_leg("musa", a) if legs else None
    mix = mix_roofline(dev, B, V, a.precision) if rank == 0 else None
    sens = sensor_bench(dev) if (rank == 0 and world == 1) else None
    rgbr = rgb_bench(dev) if (rank == 0 and world == 1 and not a.no_targcn) else None
    if rgbr is not None:
        rgbr["north_star_step_with_rgb"] = rgb_step_bench(dev, a, V, S, C, sk, se, lb)
    ldr = loader_bench(model, dev, B, V, S, C) if (rank == 0 and world == 1 and not a.no_targcn) else None
    if rank == 0:
        cpu = None if a.no_cpu_baseline or world > 1 else cpu_baseline(a.layout, V, S, a.cpu_seconds)
        rec = {
            "metric": "clips/sec (fwd+bwd) 3-stream Fall3, B=256, 1/2/4/8 GPUs; top-1 acc parity",
            "value": round(world * B * a.steps / dt, 2),
            "unit": "clips/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": round(dt / a.steps * 1e3, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": a.precision,
            "parity": {"bf16x3": "meets the north star: logits <= 1e-3 of the fp64 oracle, identical argmax, per-tensor "
                                 "gradient gate (tests/test_gpu_parity.py::test_benchmarked_config_parity[bf16x3])",
                       "fp32": "meets the north star (test_benchmarked_config_parity[fp32])",
                       "bf16": "lower precision: logits ~4e-3 from the oracle (above 1e-3)"}[a.precision],
            "data": "synthetic",
            "config": {"workload": f"fall3_3stream_{a.layout}_V{V}_S{S}_B{B}_per_gpu",
                       "global_batch": world * B, "seq_len": 30, "parallelism": f"dp{world}",
                       "joints": V, "imu_axes": S, "classes": C, "rgb_branch": "build-defined, timed on its own (rgb_branch key)",
                       "hip_graph": bool(a.graph and not a.no_graph), "final_loss": round(loss, 5),
                       "ranks": world, "collective": "rccl all_reduce (2 buckets, high-priority streams)" if world > 1 else None},
            "roofline": roofs.get("dgrad_l8", roofs.get("wgrad_l1", roofs["tcn_fwd"])),
            "roofline_wgrad_l1": roofs.get("wgrad_l1"),
            "roofline_wgrad_l5": roofs.get("wgrad_l5"),
            "roofline_wgrad_l6": roofs.get("wgrad"),
            "roofline_wgrad_kernel": roofs.get("wgrad_kernel"),
            "roofline_tcn_fwd": roofs["tcn_fwd"],
            "roofline_graph_mix": mix,
            "roofline_gcn": _gcn_roofline(roofs),
            "step_mfma": {"flop_per_clip": FLOP_PER_CLIP.get((V, S)), "achieved_tflops": None if FLOP_PER_CLIP.get(
                (V, S)) is None else round(B * FLOP_PER_CLIP[(V, S)] / (dt / a.steps) / 1e12, 2),
                "products_per_flop": PRODUCTS[a.precision],
                "peak": PEAK_MFMA_TFLOPS[a.precision], "frac": None if FLOP_PER_CLIP.get((V, S)) is None else round(
                    B * FLOP_PER_CLIP[(V, S)] / (dt / a.steps) / 1e12 / PEAK_MFMA_TFLOPS[a.precision], 4),
                "mfma_issue_frac": None if FLOP_PER_CLIP.get((V, S)) is None else round(
                    PRODUCTS[a.precision] * B * FLOP_PER_CLIP[(V, S)] / (dt / a.steps) / 1e12 /
                    PEAK_MFMA_TFLOPS[a.precision], 4),
                "note": "whole step's algorithmic FLOPs (fwd+bwd conv/einsum/addmm, SURVEY 8d) / ms_per_step / dense "
                        "peak; mfma_issue_frac counts the mode's bf16 products per FLOP (3 for bf16x3)"},
            "sensor": sens,
            "loader": ldr,
            "eval_forward": ev,
            "dp_phased_backward": phased,
            "main_py_autograd_path": agp,
            "cfg2_targcn": tgrec,
            "cfg5_sktr": skrec,
            "musa_model": murec,
            "rgb_branch": rgbr,
            "fp32_mode": fp32m,
            "bf16_mode": bf16m,
            "cpu_baseline": cpu,
            "reference_cpu_published": REFERENCE_CPU,
        }
        print(json.dumps(rec), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
