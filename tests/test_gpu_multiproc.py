"""Multi-process RCCL parity (one process per GPU, the driver's multi-GPU layout).

tests/conftest.py starts N = min(visible GPUs, 8) rank processes (tests/mp_rank.py) at session
start, before this process touches a GPU, when the gpu tests are selected and >= 2 GPUs are
visible; here they are joined and their rank slabs compared BIT for bit with the same sequence
on the in-process LOCAL transport (ranks as threads on one device; itself bitwise equal to the
single-rank run, test_gpu_distributed_full.py): two level-0 sweeps and three V-cycles at 512^3,
the later ones replaying the captured multi-rank hipGraph over RCCL.  One visible GPU: skipped.
"""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.mark.timeout(600)
def test_rccl_rank_processes_equal_local_transport(pytestconfig):
    import conftest
    job = conftest.multiproc_job(pytestconfig)
    if job is None:
        pytest.skip("needs >= 2 visible GPUs (one RCCL rank process per GPU)")
    rcs = conftest.join_multiproc(job, timeout=420)
    logs = {r: open(job["logs"][r]).read()[-2000:] for r in range(job["world"])}
    for r, rc in enumerate(rcs):
        assert rc == 0, f"rank {r} exited {rc}:\n{logs[r]}"

    import mp_rank
    import multigridanisotropicdiffusion_amd as M
    from multigridanisotropicdiffusion_amd import distributed as D
    world = job["world"]

    def body(r, s):
        s.synth_tensor(kind=0, seed=4)
        s.setup()
        return mp_rank.drive(s, M)

    ref = D.run_local(world, body, mp_rank.GSHAPE, time_step=0.1, precision=M.FP32, cycle=M.VCYCLE)
    for r in range(world):
        with np.load(os.path.join(job["outdir"], f"rank{r}.npz"), allow_pickle=False) as z:
            got = {k: z[k] for k in z.files}
        for k, v in ref[r].items():
            np.testing.assert_array_equal(got[k], v, err_msg=f"rank {r} {k} ({got['kernel']})")
