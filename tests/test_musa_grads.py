"""Which musa_model parameters the reference's autograd leaves without a gradient (CPU).

Randomized_DropBlock_Ske (Multimodal_Fall3/model/musa_model.py:45-70) is restated below with the
reference's own autograd-relevant operations: the SepTemporal blocks' `edge` (musa_model.py:184-198)
enters the graph only through M = matmul(M_seed, A * edge), every element of which the masked writes
then overwrite with a constant. torch therefore gives edge an all-zero gradient TENSOR while DropBlock
runs (training, keep_prob < 1) and None otherwise; fall_multimodal_amd.musa.grad_is_none must agree.
"""
import torch

from fall_multimodal_amd.musa import grad_is_none


def _drop_s_reference(x, keep_prob, A, training=True):
    """musa_model.py:45-70 (the num_point 14 branch), operation for operation."""
    if not training or keep_prob == 1:
        return x
    n, c, t, v = x.size()
    a = torch.mean(torch.mean(torch.abs(x), dim=2), dim=1).detach()
    a = a / torch.sum(a) * a.numel()
    gamma = (1. - keep_prob) / (1 + 1.92)
    m_seed = torch.bernoulli(torch.clamp(a * gamma, max=1.0)).to(device=x.device, dtype=x.dtype)
    M = torch.matmul(m_seed, A)
    M[M > 0.001] = 1.0
    M[M < 0.5] = 0.0
    mask = (1 - M).view(n, 1, 1, v)
    return x * mask * mask.numel() / mask.sum()


def _edge_grad(keep_prob, training, seed):
    torch.manual_seed(seed)
    V = 14
    A = (torch.rand(1, V, V) < 0.3).float() + torch.eye(V)
    edge = torch.nn.Parameter(torch.ones_like(A))
    x = torch.randn(4, 8, 5, V, requires_grad=True)
    y = _drop_s_reference(x, keep_prob, A * edge, training)
    (y * torch.randn_like(y)).sum().backward()
    return edge.grad


def test_sep_temporal_edge_grad_matches_reference_autograd():
    for seed in range(4):
        g = _edge_grad(0.9, True, seed)            # the driver's keep_prob (musa_model.py:510)
        assert g is not None and torch.count_nonzero(g) == 0
        assert _edge_grad(1.0, True, seed) is None  # DropBlock off: edge unused
        assert _edge_grad(0.9, False, seed) is None  # eval
    for s in ("stream_pos", "stream_mot"):
        for blk in (1, 2):
            name = f"{s}.{blk}.edge"
            assert grad_is_none(name, dropblock_active=True) is False
            assert grad_is_none(name, dropblock_active=False) is True
        # the SpatialGraphConv's edge multiplies the einsum operand: always a real gradient
        assert grad_is_none(f"{s}.0.edge", True) is False and grad_is_none(f"{s}.0.edge", False) is False
        assert grad_is_none(f"{s}.1.A", True) and grad_is_none(f"{s}.0.A", False)
