"""Pin the CPU oracle (oracle/thz_oracle.py) to outputs of the reference itself.

Fixtures come from tests/golden/gen_golden.py (the reference run in fp32 as shipped,
and the same reference code in fp64).  CPU-only.
"""
import contextlib

import numpy as np
import pytest
import torch

from oracle import thz_oracle as orc
from tests.golden_io import arrays, manifest, rel_l2, spacing, wavelengths

M = manifest()


@contextlib.contextmanager
def default_dtype(dt):
    old = torch.get_default_dtype()
    torch.set_default_dtype(dt)
    try:
        yield
    finally:
        torch.set_default_dtype(old)


def _asm(case, x, f64):
    dt = torch.float64 if f64 else torch.float32
    with default_dtype(dt):
        data = torch.from_numpy(x.astype(np.complex128 if f64 else np.complex64))
        return orc.asm_forward(data, wavelengths(case["f"], f64), spacing(case["dx"], case["dy"], f64), case["z"],
                               padding_scale=case["s"], do_padding=case.get("do_padding", True),
                               do_unpad_after_pad=case.get("unpad", True), bandlimit=case["bl"],
                               bandlimit_type=case["t"])


@pytest.mark.parametrize("case", M["asm"], ids=[c["name"] for c in M["asm"]])
def test_asm_oracle_matches_reference(case):
    A = arrays("asm")
    k = case["name"]
    x = A[f"{k}__in"]
    o32 = _asm(case, x, False).numpy()
    o64 = _asm(case, x, True).numpy()
    assert o32.shape == A[f"{k}__out32"].shape
    assert rel_l2(o32, A[f"{k}__out32"]) <= 1e-6
    assert rel_l2(o64, A[f"{k}__out64"]) <= 1e-12


@pytest.mark.parametrize("case", [c for c in M["asm"] if c["grad"]], ids=lambda c: c["name"])
def test_asm_oracle_adjoint_matches_reference_autograd(case):
    """Backward of ASM == ASM at -z with identical masks, vs reference autograd."""
    A = arrays("asm")
    k = case["name"]
    g = A[f"{k}__gout"]
    with default_dtype(torch.float64):
        gz = torch.from_numpy(g.astype(np.complex128))
        # adjoint = conj(ASM(conj(g))) with the same transfer function: pad/crop transpose is crop/pad
        B, C, H, W = gz.shape
        ph, pw, Ph, Pw = orc.asm_padding(H, W, case["s"])
        Hf = orc.asm_transfer_function(Ph, Pw, wavelengths(case["f"], True), *spacing(case["dx"], case["dy"], True),
                                       case["z"], case["bl"], case["t"], torch.float64)
        gp = torch.nn.functional.pad(gz, (pw, pw, ph, ph))
        adj = orc.ift2(orc.ft2(gp.conj()) * Hf).conj().resolve_conj()[..., ph:ph + H, pw:pw + W]
    assert rel_l2(adj.numpy(), A[f"{k}__gin64"]) <= 1e-12


def test_asm_cfg1_checksum():
    c = M["asm_cfg1"]
    A = arrays("asm_cfg1")
    with default_dtype(torch.float32):
        x = torch.ones(1, 1, 1024, 1024, dtype=torch.complex64)
        o = orc.asm_forward(x, wavelengths(c["f"]), spacing(c["dx"], c["dy"]), c["z"], 1, True, True, True, "exact")
    e = float((o.abs().double() ** 2).sum())
    assert abs(e - c["energy32"]) / c["energy32"] < 1e-6
    assert rel_l2(o[0, 0, ::32, ::32].numpy(), A["cfg1__sub32"]) <= 1e-6


def test_asm_zc_kat():
    """Zc KAT 0.26003873 m: P=300, dx=1 mm, f=300 GHz (experiment_four_focal_spots.ipynb:279)."""
    lam = float(wavelengths([300])[0])
    assert abs(orc.asm_critical_distance(300, float(torch.tensor(1e-3, dtype=torch.float32)), lam) - 0.26003873) < 5e-7
    # Zc 0.4333979 m at P=500 (experiment_extend_depth_of_focus.ipynb:385)
    assert abs(orc.asm_critical_distance(500, float(torch.tensor(1e-3, dtype=torch.float32)), lam) - 0.4333979) < 5e-7


def _czt(case, x, f64):
    dt = torch.float64 if f64 else torch.float32
    with default_dtype(dt):
        data = torch.from_numpy(x.astype(np.complex128 if f64 else np.complex64))
        sp = spacing(case["dx"], case["dy"], f64)
        od = spacing(case["odx"], case["ody"], f64)
        return orc.czt_forward(data, wavelengths(case["f"], f64), sp, case["z"], case["oH"], case["oW"],
                               float(od[0]) if not f64 else case["odx"] * 1e-3,
                               float(od[1]) if not f64 else case["ody"] * 1e-3)


@pytest.mark.parametrize("case", M["czt"], ids=[c["name"] for c in M["czt"]])
def test_czt_oracle_matches_reference(case):
    A = arrays("czt")
    k = case["name"]
    x = A[f"{k}__in"]
    o32 = _czt(case, x, False).numpy()
    o64 = _czt(case, x, True).numpy()
    assert o32.shape == A[f"{k}__out32"].shape
    assert rel_l2(o32, A[f"{k}__out32"]) <= 1e-5
    assert rel_l2(o64, A[f"{k}__out64"]) <= 1e-10


@pytest.mark.parametrize("case", M["rsc"], ids=[c["name"] for c in M["rsc"]])
def test_rsc_oracle_matches_reference(case):
    A = arrays("rsc")
    k = case["name"]
    x = A[f"{k}__in"]
    for f64 in (False, True):
        dt = torch.float64 if f64 else torch.float32
        with default_dtype(dt):
            data = torch.from_numpy(x.astype(np.complex128 if f64 else np.complex64))
            o = orc.rsc_forward(data, wavelengths(case["f"], f64), spacing(case["dx"], case["dy"], f64),
                                case["z"]).numpy()
        ref = A[f"{k}__out64" if f64 else f"{k}__out32"]
        assert rel_l2(o, ref) <= (1e-12 if f64 else 1e-6)


@pytest.mark.parametrize("name", ["fix_same", "fix_upsample"])
def test_doe_modulate_oracle_matches_reference(name):
    A = arrays("doe")
    case = [c for c in M["doe"] if c["name"] == name][0]
    for prec in (32, 64):
        dt = torch.float64 if prec == 64 else torch.float32
        cdt = torch.complex128 if prec == 64 else torch.complex64
        with default_dtype(dt):
            h = torch.from_numpy(A[f"{name}__h"].astype(np.float64 if prec == 64 else np.float32))
            x = torch.from_numpy(A[f"{name}__in"]).to(cdt)
            u = torch.from_numpy(A[f"{name}__noise{prec}"])
            eps = torch.tensor([case["eps"], case["tand"]])
            o = orc.doe_modulate(x, h, wavelengths(case["f"], prec == 64), eps[0], eps[1],
                                 tolerance=torch.tensor(case["tolerance"]), noise_u01=u)
        assert rel_l2(o.numpy(), A[f"{name}__out{prec}"]) <= (1e-12 if prec == 64 else 1e-6)


@pytest.mark.parametrize("iter_frac", [0.1, 0.5, 0.9])
def test_sgv3_height_map_oracle_matches_reference(iter_frac):
    A = arrays("doe")
    name = f"sgv3_{iter_frac}"
    case = [c for c in M["doe"] if c["name"] == name][0]
    dp, op = case["doe_params"], case["optim_params"]
    w = torch.from_numpy(A[f"{name}__w"])
    lut = torch.linspace(0, torch.tensor(dp["height_constraint_max"]), dp["doe_level"] + 1)[:-1]
    expo = torch.from_numpy(A[f"{name}__expo"]) if f"{name}__expo" in A else None
    lam = torch.tensor([case["wavelength"]], dtype=torch.float32)
    h = orc.sgv3_height_map(w, lut, torch.tensor(dp["height_constraint_max"]), lam.min(),
                            torch.tensor(dp["material"])[0], iter_frac, op["c_s"], op["tau_max"], op["tau_min"],
                            expo=expo, num_unit=dp["num_unit"])
    np.testing.assert_array_equal(h.numpy(), A[f"{name}__hmap"])


def test_ste_kat():
    """STE KAT: [0.1,0.4,0.7,1.2] on LUT [0,.5,1] -> [0,.5,.5,1] (Components/test_all.ipynb:595-606)."""
    q = orc.ste_quantize(torch.tensor([0.1, 0.4, 0.7, 1.2]), torch.tensor([0.0, 0.5, 1.0]))
    assert q.tolist() == [0.0, 0.5, 0.5, 1.0]


LAYERS = M.get("doe_layers", [])


def layer_inputs(case):
    """Weight, LUT, wavelengths and the recorded RNG draws of one doe_layers fixture."""
    A = arrays("doe_layers")
    k = case["name"]
    dp = case["doe_params"]
    if dp.get("look_up_table") is not None:
        lut = torch.tensor(dp["look_up_table"], dtype=torch.float32)
    else:
        lut = torch.linspace(0, torch.tensor(dp["height_constraint_max"]), dp["doe_level"] + 1)[:-1]
    draws = {kind: A[f"{k}__draw{i}"] for i, kind in enumerate(case["draws"])}
    return A, k, dp, lut, draws


@pytest.mark.parametrize("case", LAYERS, ids=[c["name"] for c in LAYERS])
def test_doe_layer_oracle_matches_reference(case):
    A, k, dp, lut, draws = layer_inputs(case)
    w = torch.from_numpy(A[f"{k}__w"]).requires_grad_(True)
    lam = wavelengths(case["f"], False)
    expo = torch.from_numpy(draws["expo"]) if "expo" in draws else None
    h = orc.layer_height_map(case["cls"], w, lut, torch.tensor(dp["height_constraint_max"]), lam.min(),
                             dp["material"][0], case["iter_frac"], case["optim_params"], dp["num_unit"],
                             dp["doe_size"], expo=expo)
    np.testing.assert_allclose(h.detach().numpy(), A[f"{k}__hmap"], rtol=1e-6, atol=1e-12)
    x = torch.from_numpy(A["in"])
    mat = torch.tensor(dp["material"])
    out = orc.doe_modulate(x, h, lam, mat[0], mat[1], tolerance=dp["tolerance"],
                           noise_u01=torch.from_numpy(draws["unif"]))
    assert rel_l2(out.detach().numpy(), A[f"{k}__out32"]) <= 1e-6
    (out.abs() ** 2).sum().backward()
    g = A[f"{k}__gw"]
    assert rel_l2(w.grad.numpy(), g) <= 1e-5 or np.abs(g).max() == np.abs(w.grad.numpy()).max() == 0


OPT = M.get("optics", [])


@pytest.mark.parametrize("case", OPT, ids=[c["name"] for c in OPT])
def test_optics_oracle_matches_reference(case):
    A = arrays("optics")
    k = case["name"]
    if case["kind"] == "gauss":
        kw = case["kw"]
        lam = wavelengths(case["f"])
        H, W = kw["height"], kw["width"]
        d = torch.tensor(case["dxy"], dtype=torch.float32)
        o = orc.gaussian_beam(H, W, d, d, lam, kw.get("beam_waist_x"), kw.get("beam_waist_y"),
                              center=kw.get("center", (0, 0)), z_w0=kw.get("z_w0", (0, 0)), alpha=kw.get("alpha", 0))
        assert rel_l2(o.numpy(), A[f"{k}__out32"]) <= 1e-6
        return
    x = torch.from_numpy(A["field_in"]).requires_grad_(True)
    lam = wavelengths(case["f"])
    dx, dy = torch.tensor(case["dx"], dtype=torch.float32), torch.tensor(case["dy"], dtype=torch.float32)
    if case["kind"] == "lens":
        o = orc.thin_lens(x, dx, dy, case["arg"], lam)
    else:
        o = x * orc.aperture_mask(x.shape[-2], x.shape[-1], dx, dy, case["kind"], case["arg"])[None, None]
    gx, = torch.autograd.grad(o, x, grad_outputs=torch.from_numpy(A["field_gout"]))
    assert rel_l2(o.detach().numpy(), A[f"{k}__out32"]) <= 1e-6
    assert rel_l2(gx.numpy(), A[f"{k}__gx32"]) <= 1e-6


def test_loss_oracle_matches_reference():
    A = arrays("optics")
    E = torch.from_numpy(A["loss_in"]).requires_grad_(True)
    loss = orc.intensity_mse(E, torch.from_numpy(A["loss_target"]))
    g, = torch.autograd.grad(loss, E)
    assert abs(float(loss) - float(A["loss_value"])) <= 1e-6 * float(A["loss_value"])
    assert rel_l2(g.numpy(), A["loss_grad"]) <= 1e-5


def test_qat_system_oracle_matches_reference():
    """cfg4 optics before the DOE and the first QAT step (loss + weight gradient) via the oracle."""
    A = arrays("qat")
    q = M["qat"]
    lam = wavelengths([q["f"]])
    d = torch.tensor(1e-3, dtype=torch.float32)
    src = orc.gaussian_beam(100, 100, d, d, lam)
    assert rel_l2(src.numpy(), A["source"]) <= 1e-6
    sp = torch.tensor([1e-3, 1e-3], dtype=torch.float32)
    f1 = orc.asm_forward(src, lam, sp, 0.127, padding_scale=2)
    assert rel_l2(f1.numpy(), A["before_lens"]) <= 1e-5
    f2 = orc.thin_lens(f1, d, d, 0.127, lam)
    f3 = f2 * orc.aperture_mask(100, 100, d, d, "rect", 0.08)[None, None]
    assert rel_l2(f3.numpy(), A["field_in"]) <= 1e-5
    dp, op = q["doe_params"], q["optim_params"]
    w = torch.from_numpy(A["w0"]).requires_grad_(True)
    lut = torch.linspace(0, torch.tensor(dp["height_constraint_max"]), dp["doe_level"] + 1)[:-1]
    h = orc.layer_height_map("SoftGumbelQuantizedDOELayerv3", w, lut, torch.tensor(dp["height_constraint_max"]),
                             lam.min(), dp["material"][0], 0.0, op, dp["num_unit"], dp["doe_size"])
    mat = torch.tensor(dp["material"])
    fm = orc.doe_modulate(torch.from_numpy(A["field_in"]), h, lam, mat[0], mat[1], tolerance=dp["tolerance"],
                          noise_u01=torch.from_numpy(A["step0__draw0"]))
    out = orc.asm_forward(fm, lam, sp, 0.2, padding_scale=2)
    assert rel_l2(out.detach().numpy(), A["out0"]) <= 1e-5
    loss = orc.intensity_mse(out, torch.from_numpy(A["target"]))
    assert abs(float(loss) - q["losses"][0]) <= 1e-5 * q["losses"][0]
    loss.backward()
    assert rel_l2(w.grad.numpy(), A["grad0"]) <= 1e-4


DONN = M.get("donn", [])


@pytest.mark.parametrize("case", DONN, ids=[c["name"] for c in DONN])
def test_donn_oracle_matches_reference(case):
    """cfg5 notebook forward (every layer modulates the encoded input) composed from oracle pieces."""
    A = arrays("donn")
    k = case["name"]
    dp = case["doe_params"]
    lam = wavelengths([case["f"]])
    sp = torch.tensor([1e-3, 1e-3], dtype=torch.float32)
    d = torch.tensor(1e-3, dtype=torch.float32)
    mask = orc.aperture_mask(100, 100, d, d, "rect", 0.08)[None, None]
    u = torch.from_numpy(A["u"]).to(torch.complex64)
    inputs = orc.asm_forward(u, lam, sp, 0.05, padding_scale=2) * mask
    draws = iter([A[f"{k}__draw{i}"] for i in range(len(case["draws"]))])
    kinds = iter(case["draws"])
    lut = torch.linspace(0, torch.tensor(dp["height_constraint_max"]), dp["doe_level"] + 1)[:-1]
    cls = "FullPrecisionDOELayer" if case["q_method"] is None else "SoftGumbelQuantizedDOELayerv3"
    mat = torch.tensor(dp["material"])

    def layer(i, field):
        w = torch.from_numpy(A[f"{k}__w{i}"])
        expo = None
        if cls != "FullPrecisionDOELayer":
            assert next(kinds) == "expo"
            expo = torch.from_numpy(next(draws))
        h = orc.layer_height_map(cls, w, lut, torch.tensor(dp["height_constraint_max"]), lam.min(), dp["material"][0],
                                 case["iter_frac"], case["optim_params"], dp["num_unit"], dp["doe_size"], expo=expo)
        assert next(kinds) == "unif"
        return orc.doe_modulate(field, h.reshape(100, 100), lam, mat[0], mat[1], tolerance=dp["tolerance"],
                                noise_u01=torch.from_numpy(next(draws)))

    for i in range(2):
        orc.asm_forward(layer(i, inputs), lam, sp, 0.02, padding_scale=2)  # computed and discarded (nb :194)
    out = orc.asm_forward(layer(2, inputs), lam, sp, 0.05, padding_scale=2)
    assert rel_l2(out.numpy(), A[f"{k}__out32"]) <= 1e-5


ADD = [c for c in M.get("addons", []) if c["kind"] == "resample"]


@pytest.mark.parametrize("case", ADD, ids=[c["name"] for c in ADD])
def test_resample_oracle_matches_reference(case):
    A = arrays("addons")
    k = case["name"]
    x = torch.from_numpy(A[f"{k}__in"]).requires_grad_(True)
    sp = torch.tensor(case["spacing"], dtype=torch.float32)
    o = orc.resample(x, sp, case["oshape"][0], case["oshape"][1], case["ospacing"][0], case["ospacing"][1])
    gx, = torch.autograd.grad(o, x, grad_outputs=torch.from_numpy(A[f"{k}__gout"]))
    assert rel_l2(o.detach().numpy(), A[f"{k}__out32"]) <= 1e-6
    assert rel_l2(gx.numpy(), A[f"{k}__gx32"]) <= 1e-6


def test_asm_oracle_multi_plane_cfg2_matches_reference():
    """The multi-plane oracle (asm_forward_planes: ft2 once, per-z transfer function) on the cfg2
    headline workload (4096^2 Gaussian, P = 8192, z = 20 / 120 mm) vs the reference's own fp32
    output signature (tests/golden/gen_cfg2_check.py)."""
    from tests.golden_io import GOLDEN
    G = np.load(f"{GOLDEN}/cfg2_check.npz")
    lam = torch.from_numpy(G["lam"])
    d = torch.tensor(float(G["dx"]), dtype=torch.float32)
    x = orc.gaussian_beam(4096, 4096, d, d, lam, 50e-3, 50e-3).to(torch.complex64)
    with torch.no_grad():
        for p, (_, y) in enumerate(orc.asm_forward_planes(x, lam, torch.stack([d, d]), [float(z) for z in G["z"]])):
            y = y[0, 0].numpy().astype(np.complex128)
            assert rel_l2(y[::64, ::64], G[f"p{p}__sub32"]) <= 1e-6
            assert rel_l2(y[2048], G[f"p{p}__row32"]) <= 1e-6
            e = float(np.sum(np.abs(y) ** 2))
            assert abs(e - float(G[f"p{p}__energy32"])) <= 1e-6 * e


def _e2e():
    import json
    import os
    from tests.golden_io import GOLDEN
    with open(os.path.join(GOLDEN, "e2e_manifest.json")) as fh:
        man = json.load(fh)
    with np.load(os.path.join(GOLDEN, "e2e_golden.npz"), allow_pickle=False) as z:
        return man, {k: z[k] for k in z.files}


@pytest.mark.parametrize("name", ["splitter4_80", "splitter9_100"])
def test_e2e_designed_doe_oracle_matches_reference(name):
    """The deterministic end-to-end golden (tests/golden/gen_e2e_golden.py): the oracle's composition
    of the four-focal-spots system with a FixDOE (tolerance 0) reproduces the reference's fp32 run:
    field, loss and height-map gradient."""
    man, A = _e2e()
    lam = wavelengths([man["f_ghz"]])
    d = torch.tensor(1e-3, dtype=torch.float32)
    sp = torch.tensor([1e-3, 1e-3], dtype=torch.float32)
    src = orc.gaussian_beam(100, 100, d, d, lam)
    f1 = orc.asm_forward(src, lam, sp, 0.127, padding_scale=2)
    f3 = orc.thin_lens(f1, d, d, 0.127, lam) * orc.aperture_mask(100, 100, d, d, "rect", 0.08)[None, None]
    assert rel_l2(f3.numpy(), A["field_in32"]) <= 1e-5
    h = torch.from_numpy(A[f"{name}__h"]).requires_grad_(True)
    mat = torch.tensor(man["material"])
    fm = orc.doe_modulate(f3, h, lam, mat[0], mat[1], tolerance=0.0, noise_u01=torch.zeros_like(h))
    out = orc.asm_forward(fm, lam, sp, 0.2, padding_scale=2)
    assert rel_l2(out.detach().numpy(), A[f"{name}__out32"]) <= 1e-5
    loss = orc.intensity_mse(out, torch.from_numpy(A["target32"]))
    assert abs(float(loss) - float(A[f"{name}__loss32"])) <= 1e-5 * float(A[f"{name}__loss32"])
    loss.backward()
    assert rel_l2(h.grad.numpy(), A[f"{name}__grad32"]) <= 1e-4


def _introspect():
    import json
    import os
    here = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
    with np.load(os.path.join(here, "introspect_golden.npz"), allow_pickle=False) as z:
        A = {k: z[k] for k in z.files}
    with open(os.path.join(here, "manifest.json")) as fh:
        return A, {c["name"]: c for c in json.load(fh)["introspect"]}


@pytest.mark.parametrize("name", ["tf_exact_s1", "tf_approx_s15_2wl", "tf_nobl_negz", "tf_nopad"])
def test_asm_transfer_function_oracle_matches_reference_create_kernel(name):
    """oracle.asm_transfer_function == the reference's ASM_prop.create_kernel (fp32 as shipped, and in
    fp64 by the SURVEY §8(c) procedure), Props/ASM_Prop.py:212-311."""
    A, cases = _introspect()
    c = cases[name]
    lam = torch.tensor([2.998e8 / (g * 1e9) for g in c["f"]], dtype=torch.float32)
    ph, pw, _, _ = orc.asm_padding(c["H"], c["W"], (c["s"], c["s"]), c.get("do_padding", True))
    dx = torch.tensor(c["dx"] * 1e-3, dtype=torch.float32)
    dy = torch.tensor(c["dy"] * 1e-3, dtype=torch.float32)
    for rdt, key in ((torch.float32, "H32"), (torch.float64, "H64")):
        H = orc.asm_transfer_function(c["H"] + 2 * ph, c["W"] + 2 * pw, lam.to(rdt), dx.to(rdt), dy.to(rdt),
                                      c["z"], c["bl"], c["t"], rdt=rdt)
        ref = A[f"{name}__{key}"]
        assert H.shape == ref.shape
        assert np.abs(H.numpy() - ref).max() <= (2e-6 if rdt == torch.float32 else 1e-12)


def test_rs_kernel_oracle_matches_reference():
    """oracle._rs_kernel on the reference's own (fp32) meshes == CZT_prop.RS_kernel and
    RSC_prop.create_kernel (Props/CZT_Prop.py:44-57, Props/RSC_Prop.py:157-160), in fp32 and with the
    reference's kernel expression evaluated in fp64 on the same meshes."""
    A, cases = _introspect()
    for pre, key_x, key_y, ks, c in (("czt_grid", "Inmeshx", "Inmeshy", ("F32", "F64on32"), cases["czt_grid"]),
                                     ("czt_grid", "Outmeshx", "Outmeshy", ("F032", "F064on32"), cases["czt_grid"]),
                                     ("rsc_k", "meshx", "meshy", ("K32", "K64on32"), cases["rsc_k"])):
        lam = torch.tensor([2.998e8 / (g * 1e9) for g in c["f"]], dtype=torch.float32)
        for rdt, k in zip((torch.float32, torch.float64), ks):
            mx = torch.from_numpy(A[f"{pre}__{key_x}"]).to(rdt)
            my = torch.from_numpy(A[f"{pre}__{key_y}"]).to(rdt)
            F = orc._rs_kernel(torch.tensor(c["z"], dtype=torch.float32).to(rdt), mx, my, lam.to(rdt))
            ref = A[f"{pre}__{k}"]
            assert F.shape == ref.shape
            tol = 1e-6 if rdt == torch.float32 else 1e-12
            assert np.abs(F.numpy() - ref).max() <= tol * np.abs(ref).max(), (pre, k)
