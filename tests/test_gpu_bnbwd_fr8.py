"""bn_bwd_apply's 8-frames-per-workgroup instance (F3_BNBWD_FR=8; default 4) inside the step
(needs an MI355X). The knob is read once per process, so each setting runs in a child process
(tests/fr8_grads.py): the B=32 step's gradients and logits with FR=8 against FR=4 on the same
weights and batch. T = 30 (position stream) and 29 (motion stream) are not multiples of 8, so the
ragged last frame group of every clip is exercised. FR only changes how the per-node column sums
are partitioned into partial rows, so the results agree to float-summation noise."""
import os
import subprocess
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.gpu
@pytest.mark.parametrize("precision", ["fp32", "bf16x3"])
def test_bn_bwd_apply_fr8_matches_fr4(precision, tmp_path):
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    res = {}
    for fr in ("4", "8"):
        out = tmp_path / f"fr{fr}.npz"
        env = dict(os.environ, F3_BNBWD_FR=fr)
        r = subprocess.run([sys.executable, os.path.join(ROOT, "tests", "fr8_grads.py"), precision, str(out)],
                           capture_output=True, text=True, timeout=240, cwd=ROOT, env=env)
        assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
        res[fr] = np.load(out)
    g4, g8 = res["4"]["grads"].astype(np.float64), res["8"]["grads"].astype(np.float64)
    np.testing.assert_allclose(res["8"]["logits"], res["4"]["logits"], rtol=0, atol=1e-5)
    cos = float(g4 @ g8 / (np.linalg.norm(g4) * np.linalg.norm(g8)))
    rel = float(np.abs(g8 - g4).max() / np.abs(g4).max())
    print(f"{precision}: FR=8 vs FR=4 gradient cosine {cos:.9f}, max rel {rel:.2e}")
    assert cos > 0.99999 and rel < 1e-3, (cos, rel)
