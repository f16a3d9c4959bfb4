"""C4 as BASELINE.json names it: the 512^3 fp32 VED pipeline (itkVEDMultigridImageFilter), GS
smoother, on one GPU.  No oracle runs at this size (the fp64 oracle would take hours), so the
checks are the properties the reference's formulas guarantee (include/itkVEDMultigridImageFilter.hxx):
  - the vesselness response is in [0, 1] (VesselnessFunction, VED.hxx:176-212: products of
    terms in [0, 1]);
  - the diffusion tensor T = a I + (c - a) v v^T (GenerateDiffusionTensor, VED.hxx:302-378) is
    symmetric with eigenvalues {a, a, c}, a = 1 + (eps - 1) V in [eps, 1], c = 1 + (omega - 1) V
    in [1, omega], V = resp^(1/s) -- checked on a strided sample of 2 M voxels;
  - the diffusion converges (last relres <= Tolerance, no stall), the output is finite, stays
    inside the input's range widened by 5 % (an implicit diffusion step is a smoothing), and is
    smoother than the input (the noise's x-differences shrink).
Parity at this size is by construction: the same kernels are checked against the oracle on the
reference's own volumes (test_gpu_ved.py, test_gpu_ved2.py)."""
import numpy as np
import pytest

import synth

pytestmark = pytest.mark.gpu

S = 512
EPS, OMEGA, SENS, TOL = 0.01, 5.0, 10.0, 1e-6


@pytest.fixture(scope="module")
def phantom():
    return synth.tube_phantom(S, seed=4)


def test_c4_tensor_properties(phantom):
    import multigridanisotropicdiffusion_amd as M
    v = M.VED(phantom.shape, epsilon=EPS, omega=OMEGA, sensitivity=SENS, precision=M.FP32)
    T, resp = v.tensor(phantom)
    v.close()
    assert np.isfinite(resp).all() and resp.min() >= 0.0 and resp.max() <= 1.0 + 1e-12
    sub = (slice(None), slice(1, None, 4), slice(2, None, 4), slice(3, None, 4))
    t = T[sub].reshape(6, -1)
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
    # the phantom has vessels: a real fraction of voxels is anisotropic
    assert (V > 0.5).mean() > 1e-3


def test_c4_pipeline_run(phantom):
    import multigridanisotropicdiffusion_amd as M
    steps = 5
    v = M.VED(phantom.shape, epsilon=EPS, omega=OMEGA, sensitivity=SENS, diffusion_iterations=steps,
              tolerance=TOL, precision=M.FP32)
    out, st = v.run(phantom, out_dtype=np.float32)
    v.close()
    assert np.isfinite(out).all()
    # one VED iteration of `steps` diffusion steps, each at least one cycle; the last converged
    assert st["iterations"] == 1 and st["total_cycles"] >= steps and not st["stalled"], st
    assert st["last_relres"] <= TOL, st
    lo, hi = float(phantom.min()), float(phantom.max())
    pad = 0.05 * (hi - lo)
    assert out.min() >= lo - pad and out.max() <= hi + pad
    dx_in = np.std(np.diff(phantom[::8], axis=2))
    dx_out = np.std(np.diff(out[::8], axis=2))
    assert dx_out < 0.9 * dx_in, (dx_out, dx_in)


@pytest.mark.timeout(600)
def test_c4_ved_on_8_rank_slabs_matches_single(phantom):
    """The partitioned VED at C4 size: 8 in-process ranks (threads on one device, the LOCAL
    transport) -- recursive Hessian z / y passes on each rank's x range, the 8-way transpose of
    the three z-pass volumes (Comm::exchange_blocks), x pass + vesselness on the rank's tensor
    planes, z-slab diffusion -- against the one-GPU pipeline, bit for bit."""
    import threading
    import zlib
    import multigridanisotropicdiffusion_amd as M
    kw = dict(epsilon=EPS, omega=OMEGA, sensitivity=SENS, diffusion_iterations=2, tolerance=TOL,
              precision=M.FP32)
    v = M.VED(phantom.shape, **kw)
    ref, rst = v.run(phantom, out_dtype=np.float32)
    v.close()
    nranks = 8
    outs, errs = [None] * nranks, []
    key = zlib.crc32(repr(("ved_c4", phantom.shape, nranks)).encode())

    def worker(r):
        try:
            w = M.VED(phantom.shape, nranks=nranks, rank=r, **kw)
            w.comm_init_local(key)
            outs[r] = w.run(phantom, out_dtype=np.float32)
            w.close()
        except BaseException as e:  # noqa: BLE001 - reported below
            errs.append((r, e))

    th = [threading.Thread(target=worker, args=(r,)) for r in range(nranks)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    assert not errs, errs
    full = np.concatenate([o[0] for o in outs])
    assert full.shape == phantom.shape
    assert all(o[1]["total_cycles"] == rst["total_cycles"] for o in outs)
    np.testing.assert_array_equal(full, ref)
