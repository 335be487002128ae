"""The reference's own seeded 6,000-iteration QAT runs (tests/golden/qat_ref_runs.json, made in the
build container by tests/golden/gen_qat_ref_runs.py) that tests/test_qat_quality_gpu.py grades the
HIP runs against: complete, finite, and generated with the same layer, optim_params and optimiser
per method as the HIP runner (scripts/qat_quality.SYSTEMS) -- so the two sides of that comparison
run the same notebook cells.  CPU only."""
import json
import math
import os
import sys

import pytest

from tests.golden_io import GOLDEN

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _load():
    with open(os.path.join(GOLDEN, "qat_ref_runs.json")) as fh:
        return json.load(fh)


def test_reference_runs_complete_and_finite():
    d = _load()
    keys = {f"{s}/{m}" for s in ("four_focal",) for m in ("Ours", "full", "GS", "PSQ", "STE")}
    keys |= {f"edof/{m}" for m in ("Ours", "full", "STE", "GQ", "PSQ")}
    keys |= {f"dual/{m}" for m in ("Ours", "full", "GQ", "PSQ", "STE")}
    assert keys <= set(d["runs"]), sorted(keys - set(d["runs"]))
    for key, runs in d["runs"].items():
        assert sorted(r["seed"] for r in runs) == [0, 1, 2], key
        for r in runs:
            assert r["iters"] == 6000 and r["finite"], (key, r["seed"])
            assert len(r["trace"]) == 31
            for k in ("final", "min", "mean_last100"):
                assert math.isfinite(r[k]) and r[k] > 0, (key, k)
            assert r["min"] <= r["final"] and r["min"] <= r["mean_last100"]


@pytest.mark.parametrize("system", ["four_focal", "edof", "dual"])
def test_generator_runs_the_hip_runners_cells(system):
    sys.path.insert(0, os.path.join(ROOT, "scripts"))
    sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
    import importlib.util
    from qat_quality import SYSTEMS
    # the generator module without importing the reference (its tables only)
    spec = importlib.util.spec_from_file_location("gen_qat_ref_runs_tables", os.path.join(GOLDEN, "gen_qat_ref_runs.py"))
    src = open(spec.origin).read()
    ns = {}
    start = src.index("FOUR_FOCAL = {")
    end = src.index("def optics_before_doe2")
    exec(compile(src[start:end], spec.origin, "exec"), ns)  # three literal dicts
    gen = ns[{"four_focal": "FOUR_FOCAL", "edof": "EDOF", "dual": "DUAL"}[system]]
    hip = SYSTEMS[system]["methods"]
    assert set(gen) == set(hip)
    default = {"c_s": 100, "tau_max": 2.5, "tau_min": 1.5}
    for m, (cls, op, opt, _second) in gen.items():
        hcls, hop, hopt = hip[m]
        assert cls == hcls, m
        assert opt == hopt, m
        if "FullPrecision" not in cls:
            assert (op or default) == (hop or default), m
