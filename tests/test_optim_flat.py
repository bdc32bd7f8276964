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
