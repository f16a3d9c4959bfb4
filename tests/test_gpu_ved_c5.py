"""C5's volume, 1024 x 1024 x 512 fp32, through the VED pipeline (itkVEDMultigridImageFilter,
include/itkVEDMultigridImageFilter.hxx:63-155) on one GPU: the C4 property checks
(test_gpu_ved_c4.py) at the largest BASELINE.json size.  No oracle at this size (hours of host
time); the same kernels are checked against it on the reference's volumes.  Host memory: the
fp64 tensor download is 26 GB."""
import numpy as np
import pytest

import synth

pytestmark = pytest.mark.gpu

SHAPE = (512, 1024, 1024)
EPS, OMEGA, SENS, TOL = 0.01, 5.0, 10.0, 1e-6


@pytest.fixture(scope="module")
def phantom():
    return synth.tube_phantom(SHAPE, seed=5)


@pytest.mark.timeout(600)
def test_c5_tensor_properties(phantom):
    import multigridanisotropicdiffusion_amd as M
    v = M.VED(phantom.shape, epsilon=EPS, omega=OMEGA, sensitivity=SENS, precision=M.FP32)
    T, resp = v.tensor(phantom)
    v.close()
    assert T.shape == (6,) + SHAPE
    assert np.isfinite(resp).all() and resp.min() >= 0.0 and resp.max() <= 1.0 + 1e-12
    sub = (slice(None), slice(1, None, 8), slice(2, None, 4), slice(3, None, 4))
    t = T[sub].reshape(6, -1)
    del T
    A = np.empty((t.shape[1], 3, 3))
    A[:, 0, 0], A[:, 0, 1], A[:, 0, 2] = t[0], t[1], t[2]
    A[:, 1, 0], A[:, 1, 1], A[:, 1, 2] = t[1], t[3], t[4]
    A[:, 2, 0], A[:, 2, 1], A[:, 2, 2] = t[2], t[4], t[5]
    w = np.linalg.eigvalsh(A)  # ascending: a, a, c (a <= 1 <= c)
    V = resp[sub[1:]].reshape(-1) ** (1.0 / SENS)
    a, c = 1.0 + (EPS - 1.0) * V, 1.0 + (OMEGA - 1.0) * V
    assert np.abs(w[:, 0] - a).max() < 1e-5 and np.abs(w[:, 1] - a).max() < 1e-5
    assert np.abs(w[:, 2] - c).max() < 1e-4
    assert w[:, 0].min() >= EPS - 1e-6 and w[:, 2].max() <= OMEGA + 1e-5
    assert (V > 0.5).mean() > 1e-3


@pytest.mark.timeout(600)
def test_c5_pipeline_run(phantom):
    import multigridanisotropicdiffusion_amd as M
    steps = 5
    v = M.VED(phantom.shape, epsilon=EPS, omega=OMEGA, sensitivity=SENS, diffusion_iterations=steps,
              tolerance=TOL, precision=M.FP32)
    out, st = v.run(phantom, out_dtype=np.float32)
    v.close()
    assert np.isfinite(out).all()
    assert st["iterations"] == 1 and st["total_cycles"] >= steps and not st["stalled"], st
    assert st["last_relres"] <= TOL, st
    assert M.max_depth(SHAPE) == 6  # 7 levels: 1024^2 x 512 ... 16^2 x 8
    lo, hi = float(phantom.min()), float(phantom.max())
    pad = 0.05 * (hi - lo)
    assert out.min() >= lo - pad and out.max() <= hi + pad
    dx_in = np.std(np.diff(phantom[::16], axis=2))
    dx_out = np.std(np.diff(out[::16], axis=2))
    assert dx_out < 0.9 * dx_in, (dx_out, dx_in)
