"""Drop-in surface checks that need no GPU: the reference's import lines resolve to this package
(install_reference_aliases), the DOE layers' .save() writes the reference's bytes, double
precision is refused consistently, and the CAD point-cloud export helper."""
import glob
import os

import numpy as np
import pytest
import torch

from tests.golden_io import GOLDEN, manifest

M = manifest()


def _load_npy_dict_restricted(path):
    """The dict .save() wrote (an object .npy holding a pickled dict), read with an unpickler that
    resolves only numpy's array / dtype / scalar reconstructors and nothing else (no arbitrary
    callables), instead of np.load(allow_pickle=True)."""
    import io
    import pickle

    allowed = {("numpy.core.multiarray", "_reconstruct"), ("numpy._core.multiarray", "_reconstruct"),
               ("numpy.core.multiarray", "scalar"), ("numpy._core.multiarray", "scalar"),
               ("numpy", "ndarray"), ("numpy", "dtype")}

    class Restricted(pickle.Unpickler):
        def find_class(self, module, name):
            if (module, name) not in allowed:
                raise pickle.UnpicklingError(f"refused {module}.{name}")
            return super().find_class(module, name)

    with open(path, "rb") as fh:
        version = np.lib.format.read_magic(fh)
        shape, _, dtype = np.lib.format._read_array_header(fh, version)
        assert dtype == np.dtype(object) and shape == ()
        obj = Restricted(io.BytesIO(fh.read())).load()
    return obj.item() if isinstance(obj, np.ndarray) else obj


def test_reference_import_lines_resolve_here():
    """The import block of experiment_four_focal_spots.ipynb (cell 0) and the DONN / extend-DOF
    notebooks, after install_reference_aliases(): every name is this package's object."""
    import quantizationawarethzdoe_amd as pkg
    pkg.install_reference_aliases()
    ns = {}
    exec("\n".join([
        "from DataType.ElectricField import ElectricField",
        "from LightSource.Gaussian_beam import Guassian_beam",
        "from Props.ASM_Prop import ASM_prop",
        "from Props.RSC_Prop import RSC_prop",
        "from Props.RSC_Prop import VRS_prop",
        "from Props.CZT_Prop import CZT_prop, VCZT_prop",
        "from Components.Thin_Lens import Thin_LensElement",
        "from Components.Aperture import ApertureElement",
        "from Components.QuantizedDOE import SoftGumbelQuantizedDOELayerv3 as SoftGumbelQuantizedDOELayer",
        "from Components.QuantizedDOE import NaiveGumbelQuantizedDOELayer",
        "from Components.QuantizedDOE import PSQuantizedDOELayer",
        "from Components.QuantizedDOE import STEQuantizedDOELayer",
        "from Components.QuantizedDOE import FullPrecisionDOELayer, FixDOEElement",
        "from utils.Helper_Functions import normalize, DOE_xyz_cordinates_Generator, ft2, ift2",
        "from utils.units import *",
        "from Addons.Field_Resampler import Field_Resampler",
        "from Addons.Field_Crop import Field_Cropper",
    ]), ns)
    from quantizationawarethzdoe_amd.Components import QuantizedDOE as Q
    from quantizationawarethzdoe_amd.Props import ASM_Prop
    assert ns["ASM_prop"] is ASM_Prop.ASM_prop
    assert ns["SoftGumbelQuantizedDOELayer"] is Q.SoftGumbelQuantizedDOELayerv3
    assert ns["mm"] == 1e-3 and ns["um"] == 1e-6
    import DataType.ElectricField as EF  # noqa: the alias is the same module object
    assert EF.ElectricField is ns["ElectricField"]


def test_doe_save_writes_the_reference_bytes(tmp_path, monkeypatch):
    """.save(crop) (Components/QuantizedDOE.py:253-267) byte-for-byte equal to the file the
    reference's own layer wrote for the same height map (tests/golden/gen_golden.py gen_save)."""
    from quantizationawarethzdoe_amd.Components.QuantizedDOE import FullPrecisionDOELayer
    c = M["save"]
    layer = FullPrecisionDOELayer(c["doe_params"], device=torch.device("cpu"))
    layer.height_map = torch.from_numpy(
        np.random.default_rng(c["seed"]).random(tuple(c["shape"])).astype(np.float32) * 1e-3)
    monkeypatch.chdir(tmp_path)
    layer.save(tuple(c["crop"]))
    (f,) = glob.glob("height_map_*.npy")
    got = open(f, "rb").read()
    ref = open(os.path.join(GOLDEN, "save_ref.bin"), "rb").read()
    assert len(got) == c["nbytes"] and got == ref
    d = _load_npy_dict_restricted(f)
    assert d["thickness"].shape == tuple(c["crop"]) and float(d["dxy"]) == c["doe_params"]["doe_dxy"]


def test_compute_dtype_follows_the_reference_promotion():
    """The reference computes in the field's precision (DataType/ElectricField.py:85-90): a complex128
    field or a float64 wavelength tensor runs in fp64 and returns complex128, real float32 data
    promotes to complex64.  kernel_dtype picks the kernels' precision the same way; the DOE
    layers (complex64 kernels only) refuse complex128 with TypeError, and a CPU tensor still
    raises before any work (there is no CPU compute path)."""
    from quantizationawarethzdoe_amd.DataType.ElectricField import ElectricField
    from quantizationawarethzdoe_amd.Props.ASM_Prop import ASM_prop
    from quantizationawarethzdoe_amd import doe
    from quantizationawarethzdoe_amd.propagation import kernel_dtype
    c64, c128 = torch.zeros(1, 1, 4, 4, dtype=torch.complex64), torch.zeros(1, 1, 4, 4, dtype=torch.complex128)
    assert kernel_dtype(c64, "t").dtype == torch.complex64
    assert kernel_dtype(c128, "t").dtype == torch.complex128
    assert kernel_dtype(torch.zeros(1, 1, 4, 4), "t").dtype == torch.complex64
    assert kernel_dtype(torch.zeros(1, 1, 4, 4, dtype=torch.float64), "t").dtype == torch.complex128
    assert kernel_dtype(c64, "t", torch.tensor([1e-3], dtype=torch.float64)).dtype == torch.complex128
    assert kernel_dtype(c64, "t", torch.tensor([1e-3], dtype=torch.float32)).dtype == torch.complex64
    with pytest.raises(TypeError):
        kernel_dtype(torch.zeros(2, dtype=torch.int32), "t")
    with pytest.raises(TypeError, match="complex64"):
        doe.modulate(c128, torch.zeros(4, 4), [1e-3], 2.66, 0.03)
    cpu = torch.device("cpu")
    f128 = ElectricField(torch.ones(1, 1, 16, 16, dtype=torch.complex128), wavelengths=1e-3, spacing=1e-3, device=cpu)
    with pytest.raises(RuntimeError, match="ROCm device"):
        ASM_prop(z_distance=0.1, device="cpu")(f128)


def test_doe_xyz_coordinates_export(tmp_path, monkeypatch, capsys):
    """CAD point cloud (utils/Helper_Functions.py:195-251): nearest upsampling by an integer factor is
    element repetition; centred grid; z flattened from the transpose; csv written."""
    from quantizationawarethzdoe_amd.utils.Helper_Functions import DOE_xyz_cordinates_Generator
    monkeypatch.chdir(tmp_path)
    h = np.arange(12, dtype=np.float64).reshape(3, 4) * 1e-4
    xyz = DOE_xyz_cordinates_Generator(h, 2e-3, new_dxy=1e-3)
    up = np.repeat(np.repeat(h, 2, 0), 2, 1)
    assert xyz.shape == (48, 3)
    np.testing.assert_array_equal(xyz[:, 2], up.T.flatten())
    xs = np.linspace(-8 / 2 * 1e-3, 8 / 2 * 1e-3, 8)
    np.testing.assert_allclose(xyz[:8, 0], xs)
    assert len(glob.glob("DOE_xyz_coordinates_*.csv")) == 1
    out = capsys.readouterr().out.splitlines()
    assert out[0].startswith("The physical length of hologram is") and out[1] == "6"
    lin = DOE_xyz_cordinates_Generator(h, 2e-3, new_dxy=1e-3, interp="linear")
    assert lin[:, 2].min() >= h.min() - 1e-15 and lin[:, 2].max() <= h.max() + 1e-15


def test_asm_forward_refuses_multi_valued_z():
    """ASM_prop.forward propagates one z (the reference's transfer function does not give one plane
    per value of a multi-valued z, Props/ASM_Prop.py:253): several values raise ValueError naming
    propagate_planes instead of silently propagating z[0].  Raised before any device work."""
    from quantizationawarethzdoe_amd.DataType.ElectricField import ElectricField
    from quantizationawarethzdoe_amd.Props.ASM_Prop import ASM_prop
    f = ElectricField(torch.zeros(1, 1, 8, 8, dtype=torch.complex64), wavelengths=1e-3, spacing=1e-3,
                      device=torch.device("cpu"))
    prop = ASM_prop(z_distance=torch.tensor([0.1, 0.2]), device=torch.device("cpu"))
    with pytest.raises(ValueError, match="propagate_planes"):
        prop(f)
    prop.z = [0.3, 0.4, 0.5]
    with pytest.raises(ValueError, match="propagate_planes"):
        prop(f)


def test_czt_one_by_one_power_of_two_width_output_stays_in_the_graph():
    """the reference's [B, C, 1, 0] CZT output (1 x 1 output, power-of-two W, odd H;
    Props/CZT_Prop.py:206,211) is an empty tensor that stays in the autograd graph; backward through
    it gives the input a zero gradient instead of raising 'does not require grad'.  No kernel runs."""
    import torch
    from quantizationawarethzdoe_amd.DataType.ElectricField import ElectricField
    from quantizationawarethzdoe_amd.Props.CZT_Prop import CZT_prop
    x = torch.randn(1, 1, 3, 4, dtype=torch.complex64, requires_grad=True)
    f = ElectricField(data=x, wavelengths=1e-3, spacing=1e-3, device="cpu")
    out = CZT_prop(z_distance=0.1, device="cpu")(f, outputHeight=1, outputWidth=1)
    assert tuple(out.data.shape) == (1, 1, 1, 0)
    out.data.abs().sum().backward()
    assert x.grad is not None and float(x.grad.abs().sum()) == 0.0


def test_release_step_graph_detaches_height_maps_and_pending_modulations():
    """qat.release_step_graph: after a step (and before each capture) the DOE layers' last
    ``height_map`` and their last pending modulation's tensors are detached -- same values, no
    grad_fn -- so no autograd graph (and no weight AccumulateGrad node made on another stream)
    outlives the step; parameters are left alone."""
    import torch.nn as nn

    from quantizationawarethzdoe_amd.qat import release_step_graph

    class Pending:
        pass

    class Layer(nn.Module):
        def __init__(self):
            super().__init__()
            self.weight = nn.Parameter(torch.randn(4, 4))

        def forward(self):
            self.height_map = torch.sigmoid(self.weight) * 2.0
            p = Pending()
            p.field = torch.randn(4, 4, dtype=torch.complex64)
            p.height = self.height_map
            p.out = self.height_map.to(torch.complex64) * p.field
            p.hfull = self.height_map * 1.0
            self._pending_mod = p
            return p.out.abs().sum()

    outer = nn.Sequential(Layer())
    layer = outer[0]
    layer().backward()
    before = layer.height_map.detach().clone()
    assert layer.height_map.grad_fn is not None and layer._pending_mod.out.grad_fn is not None
    release_step_graph([outer])
    assert layer.height_map.grad_fn is None and torch.equal(layer.height_map, before)
    for k in ("height", "out", "hfull"):
        assert getattr(layer._pending_mod, k).grad_fn is None, k
    assert isinstance(layer.weight, nn.Parameter) and layer.weight.requires_grad


def test_bench_strong_split_covers_the_64_plane_sweep_once():
    """bench.z_planes: the strong split (--cfg2-split strong) hands the 64-plane cfg2 sweep to the
    ranks, every plane exactly once and in order (8 per rank at N = 8); the weak split gives each
    rank 64 planes of a 64 N sweep."""
    import bench
    for world in (1, 2, 3, 8):
        parts = [bench.z_planes(r, world, "strong") for r in range(world)]
        flat = [z for p in parts for z in p]
        assert flat == bench.z_planes(0, 1, "strong") and len(flat) == bench.Z_PER_RANK
        assert max(map(len, parts)) - min(map(len, parts)) <= 1
        weak = [bench.z_planes(r, world, "weak") for r in range(world)]
        assert all(len(p) == bench.Z_PER_RANK for p in weak)
        assert len({z for p in weak for z in p}) == bench.Z_PER_RANK * world
