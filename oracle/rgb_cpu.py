"""CPU restatement of the BUILD-DEFINED RGB spatial-conv branch (fall_multimodal_amd/csrc/rgb.hip).

TEST INFRASTRUCTURE ONLY: imported by tests/ and bench.py's checks, never by the product path.

PARITY UNPINNED: the reference has RGB frames only in preprocessing (3_stream/har_create3.py:36-42,
101-158: AVI assembly and pose extraction) and no RGB model arithmetic anywhere (SURVEY.md section 0.2,
8a row R-RGB), so there is no reference output to pin this against. This module restates the
build's own definition so the HIP kernels can be checked against it:
    conv  = Conv2d(3, 64, kernel_size=8, stride=8) over each 224 x 224 frame (28 x 28 patches)
    feat  = mean over the T frames and the 784 patches of relu(conv)          -> [B, 64]
    logits (late fusion) = feat @ fc_w.T + fc_b
Frames are channels-last [B, T, 224, 224, 3] (the decoded-frame layout); the GPU path stores them
and the conv weight in bf16, so the restatement takes bf16-rounded operands and computes in fp64.
"""
import torch


def pack_weight(w):
    """Conv2d weight [64, 3, 8, 8] -> the kernels' packed [64, 192] with k = (dy*8 + dx)*3 + ch."""
    return w.permute(0, 2, 3, 1).reshape(w.shape[0], -1)


def unpack_weight(wp):
    """Packed [64, 192] -> Conv2d layout [64, 3, 8, 8]."""
    return wp.reshape(wp.shape[0], 8, 8, 3).permute(0, 3, 1, 2)


def rgb_feat(frames, w, b, dtype=torch.float64):
    """feat[B, 64] of the definition above; frames [B, T, 224, 224, 3], w [64, 3, 8, 8], b [64]."""
    B, T = frames.shape[:2]
    x = frames.to(dtype).permute(0, 1, 4, 2, 3).reshape(B * T, 3, frames.shape[2], frames.shape[3])
    y = torch.nn.functional.conv2d(x, w.to(dtype), b.to(dtype), stride=8)
    return torch.relu(y).reshape(B, T, w.shape[0], -1).mean(dim=(1, 3))
