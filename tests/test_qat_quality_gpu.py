"""QAT quality against the reference's published results: the
four-focal-spots system (experiment_four_focal_spots.ipynb cells 6-8) trained for the notebook's
6,000 iterations with the v3 score-Gumbel layer ("Ours": c_s 100, tau 2.5 -> 1.5, Adam lr 0.02,
iter_frac = itr / 6000) on the HIP path (graph-replayed trainer), three seeds, against the
reference's own loss curve plot_data/example_1/loss_curve_Ours.npy and the notebook's printed run
(tests/golden/qat_curves.json, gen_qat_curves.py).

The losses are noisy (every iteration draws fresh Gumbel and fabrication noise), so the envelope
is on robust statistics: the median over seeds of the mean of the last 100 iterations within
[0.5x, 2x] of the reference curve's, the median minimum within [0.5x, 2x] of the reference's
minimum, and the loss at iterations 200 / 400 within [0.5x, 2x] of the span of the two reference
runs (the saved curve and the printed trace differ by up to 1.5x there).  scripts/qat_quality.py
runs every method of the notebook with five seeds (profiles/r04_qat_quality.json), and with
--system dual / edof the methods of the dual-plane and extended-DOF notebooks (profiles/r05_*).

The published curves are ONE unseeded CUDA run each.  tests/golden/qat_ref_runs.json holds the
REFERENCE ITSELF run here on CPU for every method of the three notebooks, three seeds each, 6,000
iterations (tests/golden/gen_qat_ref_runs.py): the HIP runs are graded against that same-code
spread -- the median over the HIP seeds of the minimum and of the mean of the last 100 iterations
each within [min / 1.25, max x 1.25] over the reference's seeds and its published run (the
reference's own seeds span up to 3.6x at the final loss, and the published extended-DOF runs sit at
the low end of them)."""
import json
import os

import numpy as np
import pytest
import torch

from tests.golden_io import GOLDEN

pytestmark = pytest.mark.gpu
SAME_CODE_SLACK = 1.25


def ref_runs(system, method):
    """The reference's own seeded runs of (system, method), or None (tests/golden/qat_ref_runs.json)."""
    path = os.path.join(GOLDEN, "qat_ref_runs.json")
    if not os.path.exists(path):
        return None
    with open(path) as fh:
        runs = json.load(fh)["runs"].get(f"{system}/{method}")
    return runs if runs and len(runs) >= 3 else None


def assert_within_reference_runs(system, method, hip_stats):
    """The HIP seeds' median of each statistic within [min / 1.25, max x 1.25] over every known run
    of the reference code: its seeded runs here and its published run."""
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "scripts"))
    from qat_quality import reference
    runs = ref_runs(system, method)
    assert runs is not None, (system, method)
    pub = reference(system, method)
    # the minimum and the mean of the last 100 iterations: the final loss alone is one noisy
    # iteration (the reference's own seeds' finals span 1.3-3.6x), reported but not bounded
    for k in ("min", "mean_last100"):
        med = float(np.median([s[k] for s in hip_stats]))
        vals = [r[k] for r in runs] + [pub[k]]
        lo = min(vals) / SAME_CODE_SLACK
        hi = max(vals) * SAME_CODE_SLACK
        assert lo <= med <= hi, (system, method, k, med, lo, hi)


def test_v3_six_thousand_iterations_within_the_reference_envelope():
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "scripts"))
    from qat_quality import run_method, stats
    if not torch.cuda.is_available():
        pytest.skip("needs a ROCm GPU")
    with open(os.path.join(GOLDEN, "qat_curves.json")) as fh:
        ref = json.load(fh)
    r = ref["methods"]["Ours"]
    printed = dict((it, v) for it, v in ref["notebook_v3_printed_trace"]["points"])
    runs = []
    for seed in range(3):
        curve, _ = run_method("Ours", seed)
        assert np.all(np.isfinite(curve))
        runs.append((stats(curve), curve))
    last100 = float(np.median([s["mean_last100"] for s, _ in runs]))
    mn = float(np.median([s["min"] for s, _ in runs]))
    assert 0.5 * r["mean_last100"] <= last100 <= 2.0 * r["mean_last100"], (last100, r["mean_last100"])
    assert 0.5 * r["min"] <= mn <= 2.0 * r["min"], (mn, r["min"])
    assert_within_reference_runs("four_focal", "Ours", [s for s, _ in runs])
    for it in (200, 400):
        lo = min(r["trace"][it // 200], printed[it])
        hi = max(r["trace"][it // 200], printed[it])
        med = float(np.median([c[it] for _, c in runs]))
        assert 0.5 * lo <= med <= 2.0 * hi, (it, med, lo, hi)


def test_naive_gumbel_six_thousand_iterations_stay_finite_and_within_the_envelope():
    """The naive Gumbel-softmax layer (notebook cells 31-33: c_s 100, tau 5.5 -> 1.0, AdamW) draws
    10^4 Gumbel values per iteration, 6 x 10^7 per run: before the Exp(1) draws were held above zero
    (csrc/thz_dev.hpp rng_exp1) a draw of exactly 0 made the step NaN within a few hundred
    iterations.  Three seeds: every loss finite, the median mean-of-last-100 and minimum within
    [0.5x, 2x] of the reference curve (plot_data/example_1/loss_curve_GS.npy)."""
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "scripts"))
    from qat_quality import run_method, stats
    if not torch.cuda.is_available():
        pytest.skip("needs a ROCm GPU")
    with open(os.path.join(GOLDEN, "qat_curves.json")) as fh:
        r = json.load(fh)["methods"]["GS"]
    runs = []
    for seed in range(3):
        curve, _ = run_method("GS", seed)
        assert np.all(np.isfinite(curve)), seed
        runs.append(stats(curve))
    last100 = float(np.median([s["mean_last100"] for s in runs]))
    mn = float(np.median([s["min"] for s in runs]))
    assert 0.5 * r["mean_last100"] <= last100 <= 2.0 * r["mean_last100"], (last100, r["mean_last100"])
    assert 0.5 * r["min"] <= mn <= 2.0 * r["min"], (mn, r["min"])
    assert_within_reference_runs("four_focal", "GS", runs)


ENVELOPE_CASES = [
    # every remaining method of the three notebooks (four-focal "Ours" and GS: the tests above),
    # graded against the reference's own seeded runs where tests/golden/qat_ref_runs.json has them
    ("four_focal", "STE"), ("four_focal", "PSQ"), ("four_focal", "full"),
    ("dual", "Ours"), ("dual", "full"), ("dual", "GQ"), ("dual", "PSQ"), ("dual", "STE"),
    ("edof", "Ours"), ("edof", "full"), ("edof", "STE"), ("edof", "GQ"), ("edof", "PSQ"),
]


@pytest.mark.parametrize("system,method", ENVELOPE_CASES, ids=[f"{s}-{m}" for s, m in ENVELOPE_CASES])
def test_six_thousand_iterations_within_the_reference_envelope(system, method):
    """The notebook's whole 6,000-iteration run of one method of one system (scripts/qat_quality.py:
    the layer, optim_params, optimiser and lr of its cell), three seeds on the graph-replayed
    trainer: every loss finite; against the reference's own seeded runs where they exist (module
    docstring), else the median over seeds of the mean of the last 100 iterations and of the minimum
    within [0.5x, 2x] of the published curve (plot_data/example_1, _2 or _3 loss_curve_<method>.npy
    via tests/golden/qat_curves.json).  The multi-plane systems propagate
    their planes in one pipeline with the Z-summing adjoint; the extended-DOF planes move every
    iteration (read from the device step state) and its P = 500 transforms run the compile-time
    5 4 5 5 plan."""
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "scripts"))
    from qat_quality import reference, run_method, stats
    if not torch.cuda.is_available():
        pytest.skip("needs a ROCm GPU")
    r = reference(system, method)
    runs = []
    for seed in range(3):
        curve, _ = run_method(method, seed, system=system)
        assert np.all(np.isfinite(curve)), seed
        runs.append(stats(curve))
    last100 = float(np.median([s["mean_last100"] for s in runs]))
    mn = float(np.median([s["min"] for s in runs]))
    print(f"\n{system}/{method}: HIP median last100 {last100:.3e} min {mn:.3e}; published "
          f"{r['mean_last100']:.3e} / {r['min']:.3e} ({last100 / r['mean_last100']:.2f}x / {mn / r['min']:.2f}x)")
    if ref_runs(system, method) is not None:
        assert_within_reference_runs(system, method, runs)
    else:
        assert 0.5 * r["mean_last100"] <= last100 <= 2.0 * r["mean_last100"], (last100, r["mean_last100"])
        assert 0.5 * r["min"] <= mn <= 2.0 * r["min"], (mn, r["min"])
