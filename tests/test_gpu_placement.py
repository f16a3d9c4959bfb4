"""Level-0 placement tuning at setup (Solver::tune_placement, mad_placement_trials).

The level-0 sweep's speed depends on where its arrays landed in HBM (profiles/r06_placement.md), so setup
times both directions of the sweep on fresh allocations of the level's arrays and keeps the fastest set.
The tuning moves data, never changes it: a solve with it is bit-identical to one without it
(MAD_OPT_NO_PLACEMENT_TUNE), and levels below 2^24 voxels are not tuned."""
import numpy as np
import pytest

import synth

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def M():
    import multigridanisotropicdiffusion_amd as mod
    return mod


@pytest.mark.parametrize("cycle,precision", [("VCYCLE", "FP32"), ("SMOOTHER", "FP32"), ("VCYCLE", "FP32_REFINE")])
def test_tuned_placement_is_bitwise(M, cycle, precision):
    shape = (256, 256, 256)  # 2^24 voxels: the smallest tuned level
    img = synth.image(shape, seed=31) * 100
    outs = []
    for opt in (0, M.capi.OPT_NO_PLACEMENT_TUNE):
        s = M.Solver(shape, time_step=0.4, tolerance=1e-9, precision=getattr(M, precision),
                     cycle=getattr(M, cycle), max_cycles=6, options=opt)
        s.synth_tensor(kind=0, seed=4)
        s.setup()
        trials = s.placement_trials()
        import warnings
        with warnings.catch_warnings():
            warnings.simplefilter("ignore", M.NotConvergedWarning)
            out, st = s.run(img, out_dtype=np.float64)
        s.close()
        outs.append((out, st, trials))
    (a, sa, ta), (b, sb, tb) = outs
    print(f"{cycle} {precision}: placement trials (fwd, rev ms) {ta}")
    assert tb == [] and len(ta) >= 2 and len(ta) % 2 == 0 and all(0 < v < 1e3 for v in ta)
    assert list(sa["step_cycles"]) == list(sb["step_cycles"])
    assert np.array_equal(a, b)


def test_small_levels_are_not_tuned(M):
    s = M.Solver((128, 128, 128), time_step=0.1)
    s.synth_tensor(kind=0, seed=4)
    s.setup()
    assert s.placement_trials() == []
    s.close()
