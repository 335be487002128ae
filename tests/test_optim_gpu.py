"""The trainers' one-launch Adam / AdamW (optim.py, thz_adam_step) against torch.optim.Adam / AdamW
(the reference notebooks' optimisers, single-tensor form) over 60 steps of seeded gradients:
parameters and both moments within fp32 rounding (the kernel evaluates torch's expressions in the
same fp32 order; the bias corrections' rounding differs at most), step counts exact; several
parameters of ragged sizes in one launch (chunks of 1,024 above 16,384 elements, of 256 below; a
1-element parameter), more parameters than one launch takes (split launches), L2 and decoupled weight decay,
and the step captured in a HIP graph and replayed (the step counts advance on the device)."""
import copy

import pytest
import torch

pytestmark = pytest.mark.gpu


def _dev():
    if not torch.cuda.is_available():
        pytest.skip("needs a ROCm GPU")
    return torch.device("cuda:0")


SIZES = [(50, 50), (1,), (3, 1025), (100, 100), (7,)]


def _params(sizes, dev, g):
    return [torch.randn(s, generator=g).to(dev).requires_grad_(True) for s in sizes]


@pytest.mark.parametrize("kind,wd", [("adam", 0.0), ("adam", 0.05), ("adamw", None), ("adamw", 0.1)])
@pytest.mark.parametrize("sizes", [SIZES, SIZES + [(100, 100)], [(20,)] * 19], ids=["ragged", "large", "split"])
def test_adam_matches_torch(kind, wd, sizes):
    from quantizationawarethzdoe_amd import optim
    dev = _dev()
    g = torch.Generator().manual_seed(3)
    a = _params(sizes, dev, g)
    b = [p.detach().clone().requires_grad_(True) for p in a]
    kw = {} if wd is None else {"weight_decay": wd}
    ours = {"adam": optim.Adam, "adamw": optim.AdamW}[kind](a, lr=0.02, **kw)
    ref = {"adam": torch.optim.Adam, "adamw": torch.optim.AdamW}[kind](b, lr=0.02, foreach=False, **kw)
    for _ in range(60):
        grads = [torch.randn(p.shape, generator=g).to(dev) for p in a]
        for p, q, gr in zip(a, b, grads):
            p.grad, q.grad = gr.clone(), gr.clone()
        ours.step()
        ref.step()
    for p, q in zip(a, b):
        torch.testing.assert_close(p.detach(), q.detach(), rtol=2e-5, atol=2e-6)
        so, sr = ours.state[p], ref.state[q]
        torch.testing.assert_close(so["exp_avg"], sr["exp_avg"], rtol=1e-5, atol=1e-7)
        torch.testing.assert_close(so["exp_avg_sq"], sr["exp_avg_sq"], rtol=1e-5, atol=1e-9)
        assert float(so["step"]) == 60.0 == float(sr["step"])


def test_adam_graph_replay_advances_steps():
    from quantizationawarethzdoe_amd import optim
    dev = _dev()
    g = torch.Generator().manual_seed(5)
    a = _params(SIZES, dev, g)
    b = [p.detach().clone().requires_grad_(True) for p in a]
    grads = [torch.randn(p.shape, generator=g).to(dev) for p in a]
    for p, q, gr in zip(a, b, grads):
        p.grad, q.grad = gr.clone(), gr.clone()
    ours = optim.Adam(a, lr=0.01)
    ref = torch.optim.Adam(b, lr=0.01, foreach=False)
    ours.step()  # state allocated outside the capture
    ref.step()
    side = torch.cuda.Stream(device=dev)
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph):
            ours.step()
    torch.cuda.current_stream().wait_stream(side)
    for _ in range(25):
        graph.replay()
        ref.step()
    torch.cuda.synchronize()
    for p, q in zip(a, b):
        assert float(ours.state[p]["step"]) == 26.0
        torch.testing.assert_close(p.detach(), q.detach(), rtol=2e-5, atol=2e-6)


def test_adam_refuses_what_it_does_not_implement():
    from quantizationawarethzdoe_amd import optim
    dev = _dev()
    p = torch.zeros(4, dtype=torch.float64, device=dev, requires_grad=True)
    p.grad = torch.ones_like(p)
    with pytest.raises(ValueError):
        optim.Adam([p]).step()
    with pytest.raises(ValueError):
        optim.Adam([p], amsgrad=True)
    with pytest.raises(ValueError):
        optim.AdamW([p], differentiable=True)
    with pytest.raises(TypeError):
        optim.Adam([p], nesterov=True)  # not an Adam argument
    optim.Adam([torch.zeros(2, device=dev, requires_grad=True)], foreach=True, fused=True, capturable=True)


def test_adam_continues_from_a_torch_state_dict():
    """A torch.optim.Adam state (its step count on the host) loaded into the HIP Adam: the kernel
    gets device copies and the run continues as torch's own would."""
    from quantizationawarethzdoe_amd import optim
    dev = _dev()
    g = torch.Generator().manual_seed(9)
    a = _params([(50, 50), (7,)], dev, g)
    b = [p.detach().clone().requires_grad_(True) for p in a]
    ref = torch.optim.Adam(b, lr=0.02, foreach=False)
    for _ in range(5):
        for q in b:
            q.grad = torch.randn(q.shape, generator=g).to(dev)
        ref.step()
    with torch.no_grad():
        for p, q in zip(a, b):
            p.copy_(q)
    ours = optim.Adam(a, lr=0.02)
    ours.load_state_dict(copy.deepcopy(ref.state_dict()))  # (loading shares tensors already in place)
    for _ in range(10):
        grads = [torch.randn(p.shape, generator=g).to(dev) for p in a]
        for p, q, gr in zip(a, b, grads):
            p.grad, q.grad = gr.clone(), gr.clone()
        ours.step()
        ref.step()
    for p, q in zip(a, b):
        torch.testing.assert_close(p.detach(), q.detach(), rtol=2e-5, atol=2e-6)
        assert float(ours.state[p]["step"]) == 15.0 and ours.state[p]["step"].device == p.device
