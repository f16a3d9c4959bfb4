"""Edge shapes of the filter against the oracle: the smallest images the reference accepts
(every axis >= 3 voxels -- the one-sided second-order tensor differences, GH.hxx:447-474 --
enforced by mad_create), whose hierarchy is a single level (the V-cycle is then the direct
solve alone, MAD.hxx:356-371), and two-level images with 3-voxel axes (both mirror images of
one point in every stencil), for every CycleType and smoother, fp64."""
import numpy as np
import pytest

import synth

pytestmark = pytest.mark.gpu


def relmax(a, ref):
    return np.abs(a - ref).max() / max(np.abs(ref).max(), 1e-300)


@pytest.mark.parametrize("shape", [(3, 3, 3), (3, 4, 5), (5, 5, 5), (3, 3), (4, 7), (3, 17, 18),
                                   (18, 3, 17), (3, 16)])
@pytest.mark.parametrize("cycle", [0, 1, 2])  # VCYCLE, FMG, SMOOTHER
@pytest.mark.parametrize("smoother", [0, 2])  # GS (multicolour), WJ
def test_small_and_thin_images_match_oracle(oracle_mod, shape, cycle, smoother):
    import multigridanisotropicdiffusion_amd as M
    sp = (1.0, 0.8, 1.3)[:len(shape)]
    T = synth.random_spd(shape, seed=21)
    x = 100.0 * synth.image(shape, seed=22)
    s = M.Solver(shape, sp, time_step=0.4, cycle=cycle, smoother=smoother, precision=M.FP64,
                 tolerance=1e-12, number_of_steps=2, max_cycles=200)
    s.set_tensor(T)
    out, st = s.run(x, out_dtype=np.float64)
    o = oracle_mod.Oracle(shape, sp, T, 0.4)
    # the oracle in the GPU's sweep order (4-colour GS, WJ), so even unconverged iterates (the
    # SMOOTHER mode's 200 sweeps) compare
    kw = dict(smoother=oracle_mod.GS_COLOR, ncolors=4) if smoother == 0 else dict(smoother=oracle_mod.WJ)
    ref, cyc, rr = o.run(x, cycle=cycle, tolerance=1e-12, number_of_steps=2, max_cycles=200, **kw)
    assert st["num_levels"] == o.num_levels
    assert all(abs(int(a) - int(b)) <= 1 for a, b in zip(st["step_cycles"], cyc)), (st, cyc)
    assert relmax(out, ref) < 1e-10, (st, cyc, rr)
    s.close()
