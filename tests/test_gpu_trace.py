"""The reference's -DBENCHMARK convergence history and the FP32_REFINE
fp32-phase exit.

Under -DBENCHMARK the reference appends "relres_seconds" to benchmark.txt
(include/itkMultigridAnisotropicDiffusionImageFilter.hxx):
  * VCYCLE / FMG: inside every level-0 VCycle -- after each pre-smoothing sweep (:401-409),
    after the coarse-grid correction (:450-458) and after each post-smoothing sweep (:477-485),
    2 nu + 1 entries per V-cycle, FMG's own level-0 V-cycles included; nothing per outer cycle;
  * SMOOTHER: after every sweep (:222-227);
  * seconds: clock() since m_Time, reset at the start of every time step (:158-163).
mad_desc.options MAD_OPT_BENCHMARK_TRACE records exactly those entries (mad_get_cycle_trace).  The
oracle's verbose trace holds the same level-0 values (oracle.Oracle.run_benchmark), so on the C1
registration (lena 256^2, M = diag(50, 30), dt 0.1, nu 2, Tolerance 1e-10) in fp64 with the
reference's lexicographic GS the sequences agree entry for entry.
"""
import os

import numpy as np
import pytest

import synth
from conftest import GOLDEN

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def M():
    import multigridanisotropicdiffusion_amd as mod
    return mod


def lena():
    img = np.load(os.path.join(GOLDEN, "lena_256_u8.npy")).astype(np.float64)
    T = np.stack([np.full(img.shape, 50.0), np.zeros(img.shape), np.full(img.shape, 30.0)])
    return img, T


def per_step_clock_ok(tr):
    """seconds non-decreasing inside each time step, positive"""
    for a, b in zip(tr, tr[1:]):
        if a[0] == b[0] and b[2] < a[2]:
            return False
    return all(t[2] > 0 for t in tr)


@pytest.mark.parametrize("cycle", ["VCYCLE", "FMG"])
def test_benchmark_trace_matches_reference_history(M, oracle_mod, cycle):
    img, T = lena()
    steps = 2
    s = M.Solver(img.shape, (1.0, 1.0), time_step=0.1, smoother=M.GAUSS_SEIDEL_LEX, iterations_per_grid=2,
                 tolerance=1e-10, number_of_steps=steps, precision=M.FP64, cycle=getattr(M, cycle),
                 options=M.capi.OPT_BENCHMARK_TRACE)
    s.set_tensor(T)
    out, st = s.run(img, out_dtype=np.float64)
    tr = s.cycle_trace()
    s.close()
    o = oracle_mod.Oracle(img.shape, (1.0, 1.0), T, 0.1)
    ref, ocyc, _, want = o.run_benchmark(img, cycle=getattr(oracle_mod, cycle), smoother=oracle_mod.GS_LEX,
                                         iterations_per_grid=2, number_of_steps=steps, tolerance=1e-10)
    assert list(st["step_cycles"]) == ocyc
    # 2 nu + 1 entries per level-0 V-cycle; FMG adds nu level-0 V-cycles per step
    per_step = [(c + (2 if cycle == "FMG" else 0)) * 5 for c in ocyc]
    assert len(want) == sum(per_step)
    assert len(tr) == len(want), (len(tr), len(want))
    assert [t[0] for t in tr] == [q for q, n in enumerate(per_step) for _ in range(n)]
    for k, ((stp, rr, sec), rw) in enumerate(zip(tr, want)):
        assert abs(rr - rw) <= 1e-6 * rw + 1e-15, (k, stp, rr, rw)
    assert per_step_clock_ok(tr)
    # the step's last entry (after the last post-smoothing sweep) is the step's relres
    for q in range(steps):
        last = [t for t in tr if t[0] == q][-1]
        assert abs(last[1] - st["step_relres"][q]) <= 1e-9 * st["step_relres"][q]
    assert np.abs(out - ref).max() / np.abs(ref).max() < 1e-13


def test_benchmark_trace_smoother_and_default_unchanged(M):
    """SMOOTHER: one entry per sweep with the option as without it (same values), the clock
    restarting every time step; without the option the V-cycle trace stays one entry per cycle."""
    img, T = lena()
    kw = dict(time_step=0.1, smoother=M.WEIGHTED_JACOBI, tolerance=1e-4, number_of_steps=2,
              precision=M.FP64, cycle=M.SMOOTHER, max_cycles=30)
    trs = []
    for opt in (0, M.capi.OPT_BENCHMARK_TRACE):
        s = M.Solver(img.shape, (1.0, 1.0), options=opt, **kw)
        s.set_tensor(T)
        _, st = s.run(img, out_dtype=np.float64)
        trs.append(s.cycle_trace())
        s.close()
        assert len(trs[-1]) == st["total_cycles"]
    assert [t[:2] for t in trs[0]] == [t[:2] for t in trs[1]]
    assert per_step_clock_ok(trs[1])
    # the per-run clock keeps running over the steps, the per-step clock restarts (step 1's first
    # sweep comes one sweep after its start, step 0's last ~30 sweeps after its start)
    for tr, restarts in ((trs[0], False), (trs[1], True)):
        first2 = [t for t in tr if t[0] == 1][0]
        last1 = [t for t in tr if t[0] == 0][-1]
        assert (first2[2] < last1[2]) == restarts
    s = M.Solver(img.shape, (1.0, 1.0), time_step=0.1, tolerance=1e-10, precision=M.FP64)
    s.set_tensor(T)
    _, st = s.run(img, out_dtype=np.float64)
    assert len(s.cycle_trace()) == st["total_cycles"]
    s.close()


def test_benchmark_trace_refine(M):
    """FP32_REFINE: 2 nu + 1 entries per V-cycle as well; each step's last entry is its fp64 relres."""
    img, T = lena()
    s = M.Solver(img.shape, (1.0, 1.0), time_step=0.1, tolerance=1e-10, number_of_steps=2,
                 precision=M.FP32_REFINE, options=M.capi.OPT_BENCHMARK_TRACE)
    s.set_tensor(T)
    _, st = s.run(img, out_dtype=np.float64)
    tr = s.cycle_trace()
    s.close()
    assert st["converged"] and len(tr) == 5 * st["total_cycles"]
    for q in range(2):
        ent = [t for t in tr if t[0] == q]
        assert abs(ent[-1][1] - st["step_relres"][q]) <= 1e-12 * st["step_relres"][q]
        assert ent[-1][1] <= 1e-10 and ent[0][1] > 1e-4
    assert per_step_clock_ok(tr)
    f = M.MultigridAnisotropicDiffusionImageFilter(benchmark=True, output_dtype=np.float64)
    f.SetInput(M.Image(img))
    f.SetDiffusionTensor(T.transpose(1, 2, 0))
    f.SetTimeStep(0.1)
    f.SetTolerance(1e-10)
    f.Update()
    lines = f.GetBenchmarkOutput()
    assert len(lines) == 5 * f.stats["total_cycles"] and all("_" in ln for ln in lines)


@pytest.mark.parametrize("case", ["large_dt", "max_cycles_2", "max_cycles_1"])
def test_refine_fp32_phase_leaves_room_for_the_correction(M, case):
    """the FP32_REFINE fp32 phase ends when a cycle stops halving relres (fp32's floor
    rises with the conditioning) and one cycle before MaxCycles, so the fp64 defect correction
    always runs: a large time step on a high-contrast VED tensor still converges to 1e-10 and
    matches the fp64 solve; with MaxCycles 2 the last cycle is a refined one; with MaxCycles 1
    the run refines from the start."""
    shape = (40, 36, 32)
    T = synth.ved_form(shape)
    img = synth.image(shape, seed=21) * 100
    dt = 200.0 if case == "large_dt" else 0.4
    mc = {"large_dt": 100, "max_cycles_2": 2, "max_cycles_1": 1}[case]
    res = {}
    for prec in ("FP32_REFINE", "FP64"):
        s = M.Solver(shape, time_step=dt, tolerance=1e-10, precision=getattr(M, prec), max_cycles=mc)
        s.set_tensor(T)
        import warnings
        with warnings.catch_warnings():
            warnings.simplefilter("ignore", M.NotConvergedWarning)
            res[prec] = s.run(img, out_dtype=np.float64)
        s.close()
    (a, sa), (b, sb) = res["FP32_REFINE"], res["FP64"]
    print(f"{case}: refine cycles {sa['total_cycles']} relres {sa['last_relres']:.2e}; "
          f"fp64 cycles {sb['total_cycles']} relres {sb['last_relres']:.2e}")
    if case == "large_dt":
        assert sa["converged"] and sa["last_relres"] <= 1e-10 and not sa["stalled"]
        assert np.abs(a - b).max() / np.abs(b).max() < 1e-8
        assert sa["total_cycles"] <= sb["total_cycles"] + 3
    else:
        assert sa["total_cycles"] == mc
        # a refined cycle came last: relres at least as good as the fp64 solve's after as many cycles
        assert sa["last_relres"] <= 1.5 * sb["last_relres"]
