"""Loss-landscape sweep (VisTools/calc_loss.py:8-106, directions.py:73-117) on
the CPU: the sweep's bookkeeping against a direct evaluation of the reference's formula, and the
rank-sharded sweep (gloo, world size 2) against the single-process one."""
import os
import socket
import types

import numpy as np
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


class _Toy(torch.nn.Module):
    """forward(iter_frac) -> object with .data: a smooth nonlinear field of two weight tensors."""

    def __init__(self):
        super().__init__()
        g = torch.Generator().manual_seed(5)
        self.w = torch.nn.Parameter(torch.randn(6, 5, generator=g))
        self.v = torch.nn.Parameter(torch.randn(6, 5, generator=g))
        self.b = torch.nn.Parameter(torch.randn(5, generator=g))  # 1-d: zero direction

    def forward(self, iter_frac=None):
        z = torch.exp(1j * self.w) * (1 + self.v ** 2) + self.b
        return types.SimpleNamespace(data=z[None, None])


def _args(nx=4, ny=3):
    return types.SimpleNamespace(xmin=-1.0, xmax=1.0, xnum=nx, ymin=-0.5, ymax=0.5, ynum=ny)


def _direct(model, w0, dirs, target, args):
    """The reference's loop, written out: flat index i of loss[(xnum, ynum)] at meshgrid(x, y)[i]."""
    x = np.linspace(args.xmin, args.xmax, args.xnum)
    y = np.linspace(args.ymin, args.ymax, args.ynum)
    xm, ym = np.meshgrid(x, y)
    out = -np.ones((len(x), len(y)))
    for i in range(out.size):
        a, b = xm.ravel()[i], ym.ravel()[i]
        with torch.no_grad():
            for p, w, dx, dy in zip(model.parameters(), w0, dirs[0], dirs[1]):
                p.data = w + dx * a + dy * b
            o = torch.abs(model.forward(iter_frac=1).data) ** 2
            out.ravel()[i] = float(torch.nn.functional.mse_loss(o / o.max(), target))
    return out


def test_landscape_matches_direct_evaluation(tmp_path):
    from quantizationawarethzdoe_amd.VisTools.calc_loss import calulate_single_element_loss_landscape, load_surface
    from quantizationawarethzdoe_amd.VisTools.directions import create_random_directions
    model = _Toy()
    w0 = [p.data.clone() for p in model.parameters()]
    dirs = create_random_directions(model, generator=torch.Generator().manual_seed(1))
    # filter-normalised as the reference's normalize_direction(d, w) (VisTools/directions.py:102-111):
    # each slice along dim 0 of d has the norm of the matching slice of w, 1-d parameters get zero
    for d, w in zip(dirs[0], w0):
        if w.dim() <= 1:
            assert float(d.abs().max()) == 0.0
            continue
        for dr, wr in zip(d, w):
            assert abs(float(dr.norm()) - float(wr.norm())) <= 1e-5 * (1 + float(wr.norm()))
    target = torch.rand(1, 1, 6, 5, generator=torch.Generator().manual_seed(2))
    path = calulate_single_element_loss_landscape(_args(), model, target, directions=dirs, save_path=str(tmp_path))
    x, y, loss = load_surface(path)
    assert loss.shape == (4, 3) and (loss > 0).all()
    ref = _direct(_Toy(), w0, dirs, target, _args())
    np.testing.assert_allclose(loss, ref, rtol=1e-6)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, path, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from quantizationawarethzdoe_amd.VisTools.calc_loss import calulate_single_element_loss_landscape
        from quantizationawarethzdoe_amd.VisTools.directions import create_random_directions
        model = _Toy()
        dirs = create_random_directions(model, generator=torch.Generator().manual_seed(1))
        target = torch.rand(1, 1, 6, 5, generator=torch.Generator().manual_seed(2))
        out = calulate_single_element_loss_landscape(_args(5, 5), model, target, directions=dirs, save_path=path)
        q.put((rank, out))
    finally:
        dist.destroy_process_group()


def test_landscape_sharded_over_two_ranks(tmp_path):
    from quantizationawarethzdoe_amd.VisTools.calc_loss import calulate_single_element_loss_landscape, load_surface
    from quantizationawarethzdoe_amd.VisTools.directions import create_random_directions
    world, port = 2, _free_port()
    d2 = tmp_path / "two"
    d2.mkdir()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, str(d2), q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert len({r[1] for r in res}) == 1
    _, _, loss2 = load_surface(res[0][1])
    model = _Toy()
    dirs = create_random_directions(model, generator=torch.Generator().manual_seed(1))
    target = torch.rand(1, 1, 6, 5, generator=torch.Generator().manual_seed(2))
    d1 = tmp_path / "one"
    d1.mkdir()
    _, _, loss1 = load_surface(calulate_single_element_loss_landscape(_args(5, 5), model, target, directions=dirs,
                                                                      save_path=str(d1)))
    assert (loss2 > 0).all()
    np.testing.assert_array_equal(loss1, loss2)


def test_visualize_notebook_reads_the_sweep_surface(tmp_path):
    """The notebook's plotting call (experiment_vis_loss_landscape.ipynb: visualize_notebook(args,
    save_path, surface_path), VisTools/visualize.py:63-121) on a surface file written by
    setup_surface_file: contour, filled contour, heat map and the four 3-D views."""
    import types

    import matplotlib
    matplotlib.use("Agg")
    import matplotlib.pyplot as plt
    import quantizationawarethzdoe_amd as thz
    thz.install_reference_aliases()
    from VisTools.calc_loss import setup_surface_file
    from VisTools.visualize import visualize_notebook

    args = types.SimpleNamespace(xmin=-1, xmax=1, xnum=6, ymin=-1, ymax=1, ynum=6, surf_name="loss")
    path = setup_surface_file(args, str(tmp_path))
    with np.load(path) as f:
        x, y = f["xcoordinates"], f["ycoordinates"]
    X, Y = np.meshgrid(x, y)
    np.savez(path, xcoordinates=x, ycoordinates=y, loss=X ** 2 + 0.5 * Y ** 2)
    figs = visualize_notebook(args, str(tmp_path), path)
    assert len(figs) == 7 and (tmp_path / "2D_images").is_dir()
    args.surf_name = "train_acc"  # absent: the reference prints and plots zeros
    assert len(visualize_notebook(args, str(tmp_path), path)) == 7
    plt.close("all")
