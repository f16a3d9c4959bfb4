"""The verbose per-level trace of a V-cycle (SetVerbose, MAD.h:133-156) against the oracle.

The reference prints, indented by level + 1 spaces, the relative residual after every sweep,
after the coarse-grid correction ("initial") and after the direct solve
(include/itkMultigridAnisotropicDiffusionImageFilter.hxx:356-371, 384-411, 437-487), each
||b - A x|| / ||b|| of that level.  The library prints the same lines (mad_solver.hip,
verbose_line); the oracle records the same values (oracle/mad_oracle.c, ora_take_trace).  fp64
with the same sweep order on both sides, so every printed value (6 significant digits, the
reference's std::cout precision) agrees.
"""
import re

import numpy as np
import pytest

import synth

pytestmark = pytest.mark.gpu

LINE = re.compile(r"^( +)Level (\d+), (?:iteration (\d+): |(initial) |(direct solver): )"
                  r"relative residual = (\S+)$")


def parse(text):
    out = []
    for ln in text.splitlines():
        m = LINE.match(ln)
        if not m:
            continue
        ind, lv, it, ini, ds, val = m.groups()
        level = int(lv)
        assert len(ind) == level + 1, ln
        out.append((level, -1 if ds else (0 if ini else int(it)), float(val)))
    return out


@pytest.mark.parametrize("smoother", ["GS_LEX", "WJ", "GS_COLOR"])
def test_verbose_per_level_residuals_match_oracle(oracle_mod, capfd, smoother):
    import multigridanisotropicdiffusion_amd as M
    shape = (24, 26, 28)  # 3 levels: 24x26x28 -> 12x13x14 -> 6x7x7 (direct solver)
    sp = (1.0, 0.9, 1.2)
    T = synth.random_spd(shape, seed=15)
    x = synth.image(shape, seed=2)
    b = synth.image(shape, seed=3)
    gpu_sm = {"GS_LEX": M.GAUSS_SEIDEL_LEX, "WJ": M.WEIGHTED_JACOBI, "GS_COLOR": M.GAUSS_SEIDEL}[smoother]
    s = M.Solver(shape, sp, time_step=0.6, precision=M.FP64, smoother=gpu_sm, verbose=True)
    s.set_tensor(T)
    s.setup()
    s.upload(0, M.capi.X, x)
    s.upload(0, M.capi.B, b)
    capfd.readouterr()
    s.vcycle()
    s.synchronize()
    got = parse(capfd.readouterr().out)
    out = s.download(0, M.capi.X)
    s.close()
    o = oracle_mod.Oracle(shape, sp, T, 0.6)
    kw = dict(iterations_per_grid=2, smoother=getattr(oracle_mod, smoother))
    if smoother == "GS_COLOR":
        kw["ncolors"] = 4
    ref, tr = o.vcycle_verbose(x, b, **kw)
    assert np.abs(out - ref).max() / np.abs(ref).max() < 1e-10
    # 2 levels x (2 + 1 + 2) lines, then the direct solver
    assert len(tr) == 11 and [(l, i) for l, i, _ in got] == [(l, i) for l, i, _ in tr]
    for (l, i, g), (_, _, r) in zip(got, tr):
        if i == -1:  # exact solve: rounding-level residuals on both sides
            assert g < 1e-12 and r < 1e-12
        else:
            assert abs(g - r) <= 1e-5 * r, (l, i, g, r)
