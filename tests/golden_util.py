"""Helpers to compare a run against the packed golden vectors (tools/gen_golden.py)."""
import json
import os

import numpy as np

from oracle import model_cpu as oc

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
SAMPLES = 32


def sample_idx(n):
    if n <= SAMPLES:
        return np.arange(n)
    return (np.arange(SAMPLES) * (n // SAMPLES) + 7) % n


def load(tag):
    z = np.load(os.path.join(GOLDEN, f"model_{tag}.npz"), allow_pickle=False)
    d = {k: z[k] for k in z.files}
    spec = oc.Spec(**json.loads(str(d["spec"][0])))
    return d, spec


def check_packed(d, prefix, arr, rtol, atol, what=""):
    """Compare `arr` (full tensor) against a packed golden entry; returns max error info."""
    a = np.asarray(arr, dtype=np.float64).reshape(-1)
    if prefix in d:
        ref = d[prefix].astype(np.float64)
        np.testing.assert_allclose(a, ref, rtol=rtol, atol=atol, err_msg=what + prefix)
        return
    norm = float(d[prefix + "@norm"][0])
    np.testing.assert_allclose(np.linalg.norm(a), norm, rtol=rtol, atol=atol, err_msg=what + prefix + "@norm")
    val = d[prefix + "@val"].astype(np.float64)
    scale = max(norm / np.sqrt(a.size), 1e-12)
    np.testing.assert_allclose(a[sample_idx(a.size)], val, rtol=rtol, atol=atol + rtol * scale,
                               err_msg=what + prefix + "@val")


def check_post(d, name, post, grad, lr=1e-3, floor=1e-5):
    """Post-RMSprop parameters. The first RMSprop step moves every element by about
    lr*sign(g) (v = 0.01 g^2), so elements whose gradient is numerically zero — conv
    biases feeding a train-mode BatchNorm (stgcan.py:51,114 -> BN) — move by a random
    +-lr; those elements get one full step of slack."""
    prefix = "post:" + name
    a = np.asarray(post, np.float64).reshape(-1)
    g = np.abs(np.asarray(grad, np.float64).reshape(-1))
    slack = np.where(g < floor, 2.02 * lr / np.sqrt(0.01), 0.0)  # sign flip of a 0.1-scaled step
    if prefix in d:
        ref = d[prefix].astype(np.float64)
        bad = np.abs(a - ref) > 2e-6 + 1e-5 * np.abs(ref) + slack
        assert not bad.any(), f"{prefix}: {np.flatnonzero(bad)[:8]} {a[bad][:4]} vs {ref[bad][:4]}"
        return
    idx = sample_idx(a.size)
    ref = d[prefix + "@val"].astype(np.float64)
    bad = np.abs(a[idx] - ref) > 2e-6 + 1e-5 * np.abs(ref) + slack[idx]
    assert not bad.any(), f"{prefix}@val: {idx[bad][:8]} {a[idx][bad][:4]} vs {ref[bad][:4]}"
    if not slack.any():
        np.testing.assert_allclose(np.linalg.norm(a), float(d[prefix + "@norm"][0]), rtol=1e-5,
                                   err_msg=prefix + "@norm")


CANCELLED = ("tcn.2.bias", "residual.0.bias", "atten.1.bias")  # feed a train-mode BN: true grad 0


def unpack_full(d, prefix, n):
    """Full golden tensor, or None when only norm + samples were stored."""
    if prefix in d:
        return d[prefix].astype(np.float64)
    return None


def check_grads_conditioned(d, grads, env, base_tol=2e-3, what="", k_env=8.0):
    """Conditioning-aware gradient parity.

    grads: name -> our gradient (numpy). env: name -> the oracle's own normalised change
    under 1e-6 perturbations (oracle.model_cpu.gradient_sensitivity(per_param=True)).
    Each gradient must be within base_tol + k_env*env of the reference (normalised by the
    reference's max |g|, using the stored full tensor or its strided samples and norm),
    and the flattened gradients must have cosine >= 0.999.
    The envelope is the size of ONE kink flip (a ReLU kink next to the data flips and moves
    a gradient by a step, not smoothly). Measured on MI355X for the B=4 north-star case:
    12 repeated fp32 steps differ from each other by exactly the per-parameter envelope
    (e.g. 0.0626 vs 0.0626 for layer 5's residual weight: the fp32 atomics' ordering flips
    the same kinks the 1e-6 probe flips), and the reference's own fp32 run sits on its own
    side of several kinks, so |ours - reference| can add up a few flips: k_env = 8. The
    cosine gate still holds the gradient direction to 0.999.
    """
    dots = [0.0, 0.0, 0.0]
    failures = []
    for name, g in grads.items():
        if name.endswith(CANCELLED) or "nograd:" + name in d:
            continue
        a = np.asarray(g, np.float64).reshape(-1)
        key = "grad:" + name
        ref = unpack_full(d, key, a.size)
        tol = base_tol + k_env * env.get(name, 0.0)
        if ref is not None:
            scale = np.abs(ref).max()
            if scale < 1e-9:
                continue
            err = np.abs(a - ref).max() / scale
            dots[0] += float(a @ ref); dots[1] += float(a @ a); dots[2] += float(ref @ ref)
        else:
            idx = sample_idx(a.size)
            val = d[key + "@val"].astype(np.float64)
            norm = float(d[key + "@norm"][0])
            scale = max(np.abs(val).max(), norm / np.sqrt(a.size))
            err = max(np.abs(a[idx] - val).max() / scale, abs(np.linalg.norm(a) - norm) / norm)
            dots[0] += float(a[idx] @ val); dots[1] += float(a[idx] @ a[idx]); dots[2] += float(val @ val)
        if err > tol:
            failures.append(f"{name}: err {err:.2e} > tol {tol:.2e}")
    cos = dots[0] / np.sqrt(dots[1] * dots[2])
    assert not failures, what + "; ".join(failures[:8])
    assert cos >= 0.999, f"{what} gradient cosine {cos:.6f}"
    return cos
