"""C4 at its full size against the oracle (not only rank slabs against one GPU): one V-cycle of
the 512^3 VED-form system (ν = 2, 4-colour GS, all 7 levels, the rocSOLVER coarse inverse) in
fp64 against the oracle's V-cycle with the same colour order (oracle/mad_oracle.c, ora_vcycle,
GS_COLOR; MAD.hxx:341-493), and the fp32 production path within the north-star 1e-5.  The rank
slabs of this size equal the one-GPU run bit for bit (test_gpu_distributed_full.py), so they meet
the oracle too.  Host cost: the oracle's 512^3 setup (27-point fp64 stencils, ~40 GB) and V-cycle,
~2-3 min on the GPU box's CPU."""
import numpy as np
import pytest

import synth

pytestmark = pytest.mark.gpu

SHAPE = (512, 512, 512)


def relmax(a, ref):
    return np.abs(a - ref).max() / np.abs(ref).max()


@pytest.mark.timeout(900)
def test_c4_vcycle_matches_oracle(oracle_mod):
    import multigridanisotropicdiffusion_amd as M
    T = synth.ved_form(SHAPE)
    x = synth.image(SHAPE, seed=5)
    b = synth.image(SHAPE, seed=3)
    got = {}
    for prec in (M.FP64, M.FP32):
        s = M.Solver(SHAPE, time_step=0.1, precision=prec)
        s.set_tensor(T)
        s.setup()
        assert s.num_levels == 7
        s.upload(0, M.capi.X, x)
        s.upload(0, M.capi.B, b)
        s.vcycle()
        got[prec] = s.download(0, M.capi.X)
        s.close()
    o = oracle_mod.Oracle(SHAPE, (1.0, 1.0, 1.0), T, 0.1)
    del T
    ref = o.vcycle(x, b, smoother=oracle_mod.GS_COLOR, ncolors=4, iterations_per_grid=2)
    assert relmax(got[M.FP64], ref) < 1e-10
    assert relmax(got[M.FP32], ref) < 1e-5
