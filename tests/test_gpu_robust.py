"""Robustness of the solver state machine through the C ABI (GPU).

* The V-cycle is replayed from a captured hipGraph that bakes in each level's
  x / t ping-pong buffers.  Kernel-level calls between two cycles (mad_smooth with
  an odd sweep count) swap those buffers; the graph must be re-captured for them.
  Checked bitwise against the same call sequence run eagerly (verbose mode never
  captures).
* Non-finite input (a NaN pixel, a NaN tensor component) must end the run with
  MAD_ERR_NUMERIC instead of returning MAD_OK with a NaN image
  (the reference's do/while ends silently on NaN > tol).
"""
import numpy as np
import pytest

import synth

pytestmark = pytest.mark.gpu


def _solver(shape, T, smoother, verbose, precision):
    import multigridanisotropicdiffusion_amd as M
    s = M.Solver(shape, (1.0, 0.9, 1.1), time_step=0.4, smoother=smoother, verbose=verbose,
                 precision=precision)
    s.set_tensor(T)
    s.setup()
    return s


@pytest.mark.parametrize("smoother,shape", [("wj", (40, 44, 48)), ("gs", (160, 160, 168))])
def test_vcycle_graph_follows_pingpong_swaps(smoother, shape, capsys):
    import multigridanisotropicdiffusion_amd as M
    sm = M.WEIGHTED_JACOBI if smoother == "wj" else M.GAUSS_SEIDEL
    T = synth.random_spd(shape, seed=3)
    x = synth.image(shape, seed=5)
    b = synth.image(shape, seed=6)
    outs = []
    for verbose in (False, True):
        s = _solver(shape, T, sm, verbose, M.FP32)
        s.upload(0, M.capi.X, x)
        s.upload(0, M.capi.B, b)
        s.vcycle()
        s.smooth(0, 1)   # odd: level 0's x and t trade places
        s.vcycle()       # the graph must follow the new buffers
        s.smooth(0, 1)   # and back
        s.vcycle()
        outs.append(s.download(0, M.capi.X))
        s.close()
    capsys.readouterr()  # the eager reference run is verbose
    assert np.array_equal(outs[0], outs[1])


@pytest.mark.parametrize("prec", ["fp32", "fp64"])
def test_nan_pixel_raises_numeric(prec):
    import multigridanisotropicdiffusion_amd as M
    P = M.FP32 if prec == "fp32" else M.FP64
    shape = (20, 22, 24)
    T = synth.random_spd(shape, seed=1)
    img = synth.image(shape, seed=2)
    img[5, 6, 7] = np.nan
    s = M.Solver(shape, time_step=0.3, precision=P)
    s.set_tensor(T)
    with pytest.raises(M.capi.MadError) as e:
        s.run(img)
    assert e.value.code == M.capi.ERR_NUMERIC


@pytest.mark.parametrize("prec", ["fp32", "fp64"])
def test_nan_tensor_raises_numeric(prec):
    import multigridanisotropicdiffusion_amd as M
    P = M.FP32 if prec == "fp32" else M.FP64
    shape = (20, 22, 24)
    T = synth.random_spd(shape, seed=1)
    T[3, 10, 11, 12] = np.nan  # one yy component
    img = synth.image(shape, seed=2)
    s = M.Solver(shape, time_step=0.3, precision=P)
    s.set_tensor(T)
    with pytest.raises(M.capi.MadError) as e:
        s.run(img)
    assert e.value.code == M.capi.ERR_NUMERIC


def test_zero_image_is_not_numeric_error():
    import multigridanisotropicdiffusion_amd as M
    shape = (16, 18, 20)
    s = M.Solver(shape, time_step=0.3)
    s.set_tensor(synth.random_spd(shape, seed=1))
    out, st = s.run(np.zeros(shape, np.float32))
    assert np.all(out == 0) and st["last_relres"] == 0.0
