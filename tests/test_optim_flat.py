"""Host logic of f3.RMSprop's flat path (CPU; the update itself is a GPU op tested in
test_gpu_parity.test_rmsprop_flat_path_matches_torch): parameters that are views of one
buffer, registered out of offset order, with gradients that are views of one gradient buffer
in the same layout, are detected as one flat range (pads included); anything else is not."""
import torch

from fall_multimodal_amd.optim import RMSprop


def _setup(grad_layout_same=True):
    flat = torch.zeros(24)
    a = torch.nn.Parameter(flat[12:20].view(2, 4))   # registered first, later in the buffer
    b = torch.nn.Parameter(flat[0:6].view(2, 3))     # pad 6..8 between b and c
    c = torch.nn.Parameter(flat[8:11].view(3))
    G = torch.arange(24.)
    a.grad, b.grad = G[12:20].view(2, 4), G[0:6].view(2, 3)
    c.grad = G[8:11].view(3) if grad_layout_same else G[9:12].view(3)
    return [a, b, c], flat, G


def test_flat_layout_detected_out_of_order():
    ps, flat, G = _setup()
    opt = RMSprop(ps, lr=1e-3)
    r = opt._flat(opt.param_groups[0])
    assert r is not None
    fp, fsq, fg = r
    assert fp.numel() == 20 and fp.data_ptr() == flat.data_ptr() and fg.data_ptr() == G.data_ptr()
    # states are views of the one square_avg buffer, one shared step counter
    for p in ps:
        s = opt.state[p]["square_avg"]
        assert s.shape == p.shape and s.untyped_storage().data_ptr() == fsq.untyped_storage().data_ptr()
        assert s.storage_offset() - fsq.storage_offset() == p.storage_offset()
    assert opt.state[ps[0]]["step"] is opt.state[ps[2]]["step"]
    assert opt._flat(opt.param_groups[0]) is not None  # second call reuses the flat states


def test_flat_layout_rejected():
    ps, _, _ = _setup(grad_layout_same=False)
    opt = RMSprop(ps, lr=1e-3)
    assert opt._flat(opt.param_groups[0]) is None
    ps, _, _ = _setup()
    opt = RMSprop(ps, lr=1e-3)
    for p in ps:  # states made elsewhere (e.g. loaded): per-tensor path
        opt.state[p]["square_avg"] = torch.zeros_like(p)
    assert opt._flat(opt.param_groups[0]) is None
    ps, _, _ = _setup()
    ps[1].grad = ps[1].grad.clone()  # a copied gradient
    opt = RMSprop(ps, lr=1e-3)
    assert opt._flat(opt.param_groups[0]) is None


def test_flat_rejects_gap_holding_other_tensors():
    """A gap wider than the 16-B pad may hold a tensor outside the group (a second param_group with
    its own lr, or a frozen parameter): the flat launch would update it, so the per-tensor path runs."""
    flat = torch.zeros(24)
    G = torch.arange(24.)
    a = torch.nn.Parameter(flat[0:3])
    b = torch.nn.Parameter(flat[4:8])     # another group's tensor between a and c
    c = torch.nn.Parameter(flat[8:11])
    for p, (lo, hi) in ((a, (0, 3)), (b, (4, 8)), (c, (8, 11))):
        p.grad = G[lo:hi]
    opt = RMSprop([{"params": [a, c], "lr": 1e-3}, {"params": [b], "lr": 5e-2}])
    assert opt._flat(opt.param_groups[0]) is None
    assert opt._flat(opt.param_groups[1]) is not None   # one tensor: trivially flat
    # a frozen parameter (filtered out of the optimizer) between two trainable ones
    opt = RMSprop([p for p in (a, b, c) if p is not b], lr=1e-3)
    assert opt._flat(opt.param_groups[0]) is None
    # adjacent groups each covering an exact range are both flat
    opt = RMSprop([{"params": [a, b]}, {"params": [c], "lr": 5e-2}], lr=1e-3)
    assert opt._flat(opt.param_groups[0]) is not None and opt._flat(opt.param_groups[1]) is not None


def test_flat_per_tensor_update_matches_torch_cpu_layout():
    """The flat-path decision never changes the update: with two groups, every tensor gets its own
    group's lr (checked on the layout decision alone; the update kernel is GPU-only)."""
    flat = torch.zeros(16)
    a = torch.nn.Parameter(flat[0:4])
    b = torch.nn.Parameter(flat[4:8])
    a.grad, b.grad = torch.ones(4), torch.ones(4)
    opt = RMSprop([{"params": [a]}, {"params": [b], "lr": 0.5}], lr=1e-3)
    fa, fb = opt._flat(opt.param_groups[0]), opt._flat(opt.param_groups[1])
    assert fa[0].numel() == 4 and fb[0].numel() == 4
    assert fa[0].storage_offset() == 0 and fb[0].storage_offset() == 4


def test_cached_layout_takes_detached_gradients():
    """loss.backward() gives each parameter a DETACHED gradient that shares the flat gradient buffer
    (no `_base`): the cached layout must still be recognised without the full per-tensor check, and
    a gradient that moved must still be rejected."""
    ps, flat, G = _setup()
    opt = RMSprop(ps, lr=1e-3)
    assert opt._flat(opt.param_groups[0]) is not None  # full check, layout cached
    for p in ps:
        p.grad = p.grad.detach()
        assert p.grad._base is None
    calls = []
    full = opt._flat_full
    opt._flat_full = lambda q: calls.append(1) or full(q)
    r = opt._flat(opt.param_groups[0])
    assert r is not None and not calls and r[2].data_ptr() == G.data_ptr() and r[2].numel() == 20
    ps[2].grad = G[9:12].detach().clone()  # a gradient outside the buffer
    assert opt._flat(opt.param_groups[0]) is None and calls
