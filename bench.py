#!/usr/bin/env python3
"""Headline benchmark: Mvoxel-smooths/s at 512^3 fp32 (BASELINE.json metric),
plus V-cycles/s, HBM roofline fraction of the smoother kernel and the CPU
baseline (the fp64 oracle, 1 thread, bounded sample).

Workload (config C4 of BASELINE.json, the largest single-GPU config the metric
is quoted on): 512^3 fp32 image, VED-form full 3x3 diffusion tensor (synthetic,
generated on the device), dt 0.1, unit spacing, 4-colour Gauss-Seidel smoother.
One step = one level-0 smoother sweep (all colours) over the whole volume.

    python bench.py [--gpus N --steps K --warmup W]
bench.py itself starts no processes: for N > 1 it must run under
torch.distributed.run with one process per GPU (WORLD_SIZE = N; --gpus must
match it, or the run exits with an error).  The volume is split into z-slabs
(strong scaling, fixed 512^3) with RCCL halo exchanges.  Rank 0 prints one
JSON line.

V-cycles/s are measured on a second solver built like a real solve
(CycleType VCYCLE: dense rhs layout, the production V-cycle), not on the
SMOOTHER-mode solver of the sweep measurement.
"""
import argparse
import json
import math
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

PEAK_HBM_GBS = 8000.0           # MI355X HBM3E spec (MI355X_MICROARCH.md, chip table)
BYTES_PER_VOXEL_SMOOTH = 36.0   # u in 4 + b 4 + u out 4 + 6-comp tensor 24


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=3)
    # untimed sweeps after setup, before the W warm-up steps: the clocks and power take ~20-30 launches
    # (~30 ms) to reach their steady state after the device idled (profiles/r06_clock_summaries.log)
    p.add_argument("--settle-ms", type=float, default=150.0)
    p.add_argument("--size", type=int, default=512)
    # 20 graph replays (~0.16 s): a per-cycle figure above the ~0.3 ms box-to-box noise
    p.add_argument("--vcycles", type=int, default=20)
    p.add_argument("--smoother", default="gs", choices=["gs", "wj"])
    p.add_argument("--gs-kernel", type=int, default=0,
                   help="0 auto (fused v3), 1 per-colour passes, 2 fused v2, 3 fused v3")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--cpu-seconds", type=float, default=4.0,
                   help="length of the secondary 128^3 CPU sample")
    p.add_argument("--cpu-size", type=int, default=0,
                   help="volume of the CPU baseline (default: the benched size)")
    p.add_argument("--no-precision-cycles", action="store_true")
    p.add_argument("--cpu-baseline-only", action="store_true",
                   help="(internal) print cpu_baseline(--cpu-seconds, --cpu-size) as JSON and exit")
    p.add_argument("--cpu-timeout", type=float, default=300.0,
                   help="bound of the CPU leg at the benched size (then the 128^3 fallback)")
    p.add_argument("--halo", default="auto", choices=["auto", "peer", "rccl"],
                   help="rank slabs (N > 1): 'rccl' -- a grouped ncclSend / ncclRecv exchange after "
                        "each sweep; 'peer' -- the fused level-0 sweep stores its edge planes into the "
                        "neighbours' mailboxes while it runs (MAD_OPT_PEER_HALO); 'auto' (default) -- "
                        "peer, but only after this run has checked on every rank that it gives the "
                        "same bits as the rccl exchange (verify_peer), else rccl")
    return p.parse_args()


def cpu_model():
    """The host CPU's model name (lscpu's 'Model name', read from /proc/cpuinfo)."""
    try:
        with open("/proc/cpuinfo") as f:
            for ln in f:
                if ln.startswith("model name"):
                    return ln.split(":", 1)[1].strip()
    except OSError:
        pass
    return None


def host_cores():
    """CPUs this process may run on (its affinity mask) and the machine's CPU count."""
    try:
        avail = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        avail = os.cpu_count() or 1
    return avail, os.cpu_count() or avail


def cpu_baseline(seconds, size):
    """fp64 oracle (the restated reference algorithm, oracle/) on the benched workload itself:
    the size^3 VED-form system, a fixed count of lexicographic GS sweeps and one V-cycle on one
    thread (the reference is single-threaded; BASELINE.md's C4 plan), the 4-colour GS on the
    host cores beside it, and the earlier 128^3 sample as a secondary field.  Setup (the
    GridsHierarchy + DCA stencils, ~30 GB at 512^3) is not timed: the metric is per sweep."""
    import numpy as np
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle
    import synth
    avail, total = host_cores()
    nt = max(1, int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or min(16, avail))
    shape = (size, size, size)
    nvox = float(np.prod(shape))
    t0 = time.perf_counter()
    T = synth.ved_form(shape)
    o = oracle.Oracle(shape, (1.0, 1.0, 1.0), T, 0.1)
    del T
    b = synth.image(shape, seed=3)
    t_setup = time.perf_counter() - t0
    n_sweeps = 2
    t0 = time.perf_counter()
    x = b
    for _ in range(n_sweeps):
        x = o.gs_lex(0, x, b)
    el = time.perf_counter() - t0
    t0 = time.perf_counter()
    x = o.vcycle(x, b, smoother=oracle.GS_LEX, iterations_per_grid=2)
    el_v = time.perf_counter() - t0
    t0 = time.perf_counter()
    y = b
    for _ in range(n_sweeps):
        y = o.gs_color_omp(0, y, b, 4, nt)
    el_p = time.perf_counter() - t0
    nlev = o.num_levels
    del o, x, y, b
    out = {"value": nvox * n_sweeps / el / 1e6, "unit": "Mvoxel-smooths/s", "cores": 1, "kind": "port",
           "cpu_model": cpu_model(), "host_cpus_available": avail, "host_cpus_total": total,
           "sample": f"{size}^3 VED-form full tensor (the benched system), {n_sweeps} lexicographic GS "
                     f"sweeps, fp64, 1 thread, oracle/ (line-faithful restatement of the ITK reference), "
                     f"{el:.1f} s (setup {t_setup:.0f} s untimed)"}
    out["vcycle"] = {"value": 1.0 / el_v, "unit": "V-cycles/s", "cores": 1, "kind": "port",
                     "sample": f"{size}^3 VED-form full tensor, 1 V-cycle (nu = 2, lexicographic GS, "
                               f"{nlev} levels), fp64, 1 thread, oracle/, {el_v:.1f} s"}
    out["parallel"] = {"value": nvox * n_sweeps / el_p / 1e6, "unit": "Mvoxel-smooths/s", "cores": nt,
                       "kind": "port", "sample": f"{size}^3 VED-form full tensor, {n_sweeps} 4-colour GS "
                       f"sweeps on {nt} OpenMP threads, fp64, oracle/, {el_p:.1f} s"}
    # secondary: the bounded 128^3 sample of earlier rounds (same workload, smaller volume)
    s128 = (128, 128, 128)
    o = oracle.Oracle(s128, (1.0, 1.0, 1.0), synth.ved_form(s128), 0.1)
    b = synth.image(s128, seed=3)
    x = b.copy()
    n = 0
    t0 = time.perf_counter()
    while True:
        x = o.gs_lex(0, x, b)
        n += 1
        el2 = time.perf_counter() - t0
        if el2 >= seconds:
            break
    out["sample_128"] = {"value": float(np.prod(s128)) * n / el2 / 1e6, "unit": "Mvoxel-smooths/s",
                         "cores": 1, "kind": "port",
                         "sample": f"128^3 VED-form full tensor, {n} lexicographic GS sweeps, fp64, {el2:.1f} s"}
    return out


# peak host memory of cpu_baseline() per voxel of the benched volume (the oracle's GridsHierarchy:
# 27 fp64 DCA stencil entries per voxel over all levels, the fp64 tensor and image arrays);
# measured 352 B at 160^3 including the interpreter
ORACLE_BYTES_PER_VOXEL = 360.0
CPU_FALLBACK_SIZE = 128


def host_mem_available():
    """MemAvailable of /proc/meminfo in bytes (None where it cannot be read)."""
    try:
        with open("/proc/meminfo") as f:
            for ln in f:
                if ln.startswith("MemAvailable:"):
                    return int(ln.split()[1]) * 1024
    except (OSError, ValueError, IndexError):
        pass
    return None


def _cpu_child(seconds, size, timeout):
    """cpu_baseline(seconds, size) in a child process bounded by `timeout` seconds (the oracle
    holds no GPU state; an out-of-memory kill or a hang ends the child, not the bench line).
    Returns (result dict, None) or (None, reason)."""
    import subprocess
    cmd = [sys.executable, os.path.abspath(__file__), "--cpu-baseline-only", "--cpu-size", str(size),
           "--cpu-seconds", str(seconds)]
    try:
        r = subprocess.run(cmd, capture_output=True, text=True, timeout=timeout, cwd=ROOT)
    except subprocess.TimeoutExpired:
        return None, f"the {size}^3 CPU baseline exceeded its {timeout:.0f} s bound"
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    if r.returncode != 0 or not lines:
        return None, f"the {size}^3 CPU baseline exited {r.returncode} ({r.stderr.strip()[-200:]})"
    return json.loads(lines[-1]), None


def cpu_baseline_guarded(seconds, size, timeout=300.0, fallback_timeout=120.0, mem_available=None,
                         fallback_size=CPU_FALLBACK_SIZE):
    """The CPU leg, unable to cost the GPU line: the benched size when the host has 1.5x the
    oracle's memory free and the run ends within `timeout`; otherwise the 128^3 sample, with
    `fallback` naming the reason (and `value` None with `error` if that fails too)."""
    need = ORACLE_BYTES_PER_VOXEL * float(size) ** 3
    avail = host_mem_available() if mem_available is None else mem_available
    if avail is not None and avail < 1.5 * need:
        reason = (f"MemAvailable {avail / 2**30:.1f} GiB < 1.5 x the {need / 2**30:.1f} GiB "
                  f"the {size}^3 oracle needs")
    else:
        res, reason = _cpu_child(seconds, size, timeout)
        if res is not None:
            return res
    fb = min(size, fallback_size)
    res, err = _cpu_child(seconds, fb, fallback_timeout)
    if res is None:
        return {"value": None, "unit": "Mvoxel-smooths/s", "cores": 1, "kind": "port",
                "error": f"{reason}; fallback: {err}"}
    res["fallback"] = reason
    res["sample"] = f"FALLBACK to {fb}^3 ({reason}): " + res["sample"]
    return res


def run_cycle_ms(M, shape, prec, cycles, **kw):
    """Milliseconds per solver cycle inside mad_run (the reference's loop: cycle, fp64 residual,
    host convergence check; MAD.hxx:207-246) at Tolerance 1e-30, so every run takes `cycles`
    cycles: median difference of mad_get_cycle_trace's timestamps over the second run's cycles
    (the first run captures the V-cycle graph), skipping its first cycle.  FP32_REFINE starts
    in plain fp32 until relres < MAD_REFINE_SWITCH_RELRES (1e-5); its figure is the median over
    the refined cycles (those after a cycle that ended below the switch)."""
    import numpy as np
    s = M.Solver(shape, (1.0, 1.0, 1.0), time_step=0.1, precision=prec, cycle=M.VCYCLE,
                 tolerance=1e-30, max_cycles=cycles, stall_guard=0, **kw)
    s.synth_tensor(kind=0, seed=4)
    s.setup()
    img = np.full(shape, 50.0, dtype=np.float32)
    img[::3] = 100.0
    s.run(img)
    s.run(img)
    tr = s.cycle_trace()
    s.close()
    t = [q[2] for q in tr]
    d = np.diff(t)
    if prec == M.FP32_REFINE:
        d = [d[i - 1] for i in range(1, len(tr)) if tr[i - 1][1] <= 1e-5]
        if not d:  # the run never got below the switch point: no refined cycle to time
            return None
        return float(np.median(d) * 1e3)
    return float(np.median(d[1:]) * 1e3)


def solve_at_reference_tolerance(M, shape, time_step=0.1, **kw):
    """One time step solved to the reference tests' Tolerance 1e-10 with the default descriptor
    (MAD_PRECISION_AUTO -> FP32_REFINE): cycles and the device time of the step loop
    (mad_stats.solve_ms: after the image upload, up to the output cast); second run of the solver."""
    import numpy as np
    s = M.Solver(shape, (1.0, 1.0, 1.0), time_step=time_step, cycle=M.VCYCLE, tolerance=1e-10, **kw)
    s.synth_tensor(kind=0, seed=4)
    s.setup()
    # uniform noise in [0, 100): every frequency present, relres from O(1) -- the slow case
    img = np.random.default_rng(5).random(shape, dtype=np.float32) * np.float32(100.0)
    s.run(img)
    _, st = s.run(img)
    tr = s.cycle_trace()
    prec = s.resolved_precision
    s.close()
    # the fp32 phase: the cycles up to the first one that ended below MAD_REFINE_SWITCH_RELRES
    fp32_cycles = 0
    if prec == M.FP32_REFINE:
        fp32_cycles = next((i + 1 for i, q in enumerate(tr) if q[1] <= 1e-5), len(tr))
    return {"precision": {M.FP32_REFINE: "FP32_REFINE", M.FP32: "FP32", M.FP64: "FP64"}.get(prec, prec),
            "cycles": len(tr), "fp32_phase_cycles": min(fp32_cycles, len(tr)), "relres": tr[-1][1],
            "solve_ms": round(float(st["solve_ms"]), 3)}


def load_traffic(tag, kernel_sig):
    """Per-launch HBM bytes of the bench kernel from the committed PMC profile
    (profiles/traffic_<tag>.json, written by tools/parse_prof.py); only used when it
    was measured on this same kernel instantiation."""
    path = os.path.join(ROOT, "profiles", f"traffic_{tag}.json")
    if os.path.exists(path):
        with open(path) as f:
            t = json.load(f)
        if kernel_sig in t.get("kernel", ""):
            return t
    return None


T0 = time.perf_counter()


def verify_peer(M, s, make, rank, steps=4, vcycles=False):
    """--halo auto: the peer-halo solver `s` and a second solver exchanging through RCCL run the
    same synthetic system -- `steps` level-0 sweeps (both mailbox buffers twice) or, with
    `vcycles`, `steps` V-cycles (eager, captured, replayed: every distributed level's pushes and
    unpacks) -- and every rank compares its slab bit for bit; the peer halo is used only if all
    ranks agree.  Collective: every rank reaches the same allreduce whatever its own outcome.
    Leaves `s` at the initial x again.  Returns (ok, note)."""
    import numpy as np
    what = "V-cycles" if vcycles else "sweeps"
    phase(rank, f"halo auto: {steps} peer {what} vs {steps} rccl {what}, bitwise")

    def run(sv):
        for _ in range(steps if vcycles else 1):
            sv.vcycle() if vcycles else sv.smooth(0, steps)
        return sv.download(0, M.capi.X)

    err = None
    try:
        xp = run(s)
    except Exception as e:  # a timed-out mailbox wait (peer_check) or any device error
        err, xp = f"{type(e).__name__}: {e}"[:200], None
    ref = make(M.VCYCLE if vcycles else M.SMOOTHER, 0, "vcycle-check" if vcycles else "halo-check")
    xr = run(ref)
    same = xp is not None and xp.shape == xr.shape and np.array_equal(xp.view(np.uint32), xr.view(np.uint32))
    agree = float(ref.allreduce([0.0 if same else 1.0], "max")[0]) == 0.0
    ref.close()
    if agree:
        s.synth_level(0, M.capi.X, 3)
        s.synchronize()
        return True, (f"verified in this run: {steps} {what} bitwise equal to the rccl exchange on "
                      "every rank")
    if err:
        return False, f"rank {rank}: {err}"
    return False, ("this rank's slab differed from the rccl exchange" if not same
                   else "another rank's slab differed from the rccl exchange, or its peer run failed")


def phase(rank, what):
    """One progress line per phase on stderr (the JSON line alone goes to stdout): a run that
    stops shows where, on every rank."""
    print(f"[bench rank {rank} +{time.perf_counter() - T0:7.1f} s] {what}", file=sys.stderr, flush=True)


def main():
    a = parse()
    if a.cpu_baseline_only:  # the child of cpu_baseline_guarded: no GPU, no torch
        print(json.dumps(cpu_baseline(a.cpu_seconds, a.cpu_size or a.size)), flush=True)
        return
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if a.gpus != world:
        sys.exit(f"bench.py: --gpus {a.gpus} but WORLD_SIZE={world}; launch N > 1 GPUs with "
                 "python -m torch.distributed.run --nproc-per-node N bench.py --gpus N")
    n_gpus = world
    # N > 1: one node (the contract launches --nnodes=1).  No torch in this process: the
    # ranks meet through a file keyed by their common launcher (distributed.bootstrap_node)
    # and synchronise over the solver's own RCCL communicator, so libmad_hip.so binds the
    # ROCm RCCL it was compiled against (torch would bring its own librccl.so.1 first).
    os.environ.setdefault("NCCL_SOCKET_IFNAME", "lo")
    os.environ.setdefault("NCCL_DEBUG", "WARN")
    # MAD_BENCH_SHARED_GPU=1 (rehearsal of the N > 1 launch on a one-GPU box): every rank on
    # device 0, a distinct NCCL_HOSTID per rank so RCCL accepts two ranks of one device (it
    # connects them over its socket transport); the timings then measure nothing about xGMI
    shared_gpu = world > 1 and os.environ.get("MAD_BENCH_SHARED_GPU") == "1"
    if shared_gpu:
        os.environ["NCCL_HOSTID"] = f"mad-bench-rank{rank}"
        os.environ.setdefault("NCCL_IB_DISABLE", "1")
        local = 0
    import multigridanisotropicdiffusion_amd as M
    from multigridanisotropicdiffusion_amd import distributed as MD

    S = a.size
    gshape = (S, S, S)
    nz_local = S // world
    shape = (nz_local, S, S)
    sm = M.GAUSS_SEIDEL if a.smoother == "gs" else M.WEIGHTED_JACOBI

    def make(cycle, opts, tag):
        """A rank's solver of the 512^3 volume, set up with the synthetic tensor, b and x."""
        sv = M.Solver(shape, (1.0, 1.0, 1.0), time_step=0.1, smoother=sm, precision=M.FP32,
                      cycle=cycle, nranks=world, rank=rank, device=local if world > 1 else -1,
                      global_shape=gshape, gs_kernel=a.gs_kernel, options=opts)
        if world > 1:
            phase(rank, f"{tag} solver: joining the communicator")
            MD.bootstrap_node(sv, rank, world, tag=tag)
        phase(rank, f"{tag} solver: setup")
        sv.synth_tensor(kind=0, seed=4)
        sv.setup()
        sv.synth_level(0, M.capi.B, 3)
        sv.synth_level(0, M.capi.X, 3)
        sv.synchronize()
        return sv

    # SMOOTHER mode (the reference's CycleType 2: repeated sweeps of one system) -- the
    # smoother-only protocol of SURVEY §8(d); level-0 records then carry b (mad_solver.hip)
    want_peer = world > 1 and a.halo in ("auto", "peer")
    opts = M.capi.OPT_PEER_HALO if want_peer else 0
    s = make(M.SMOOTHER, opts, "sweep")
    halo_note = None
    if want_peer:
        if "peer halo" not in s.smooth_kernel_name(0):
            halo_note = "peer halo requested, not engaged at setup (window mapping or self-test): rccl"
            opts = 0
        elif a.halo == "auto":
            ok, why = verify_peer(M, s, make, rank, steps=4)
            if ok:
                halo_note = why
            else:
                halo_note = f"peer halo rejected ({why}): rccl"
                s.close()
                opts = 0
                s = make(M.SMOOTHER, 0, "sweep-rccl")
    placement = s.placement_trials()

    def barrier():
        s.synchronize()
        if world > 1:
            s.allreduce([0.0])

    # settle (untimed, the same count on every rank: rank sweeps exchange halos): ~settle_ms of sweeps
    # at the fused sweep's ~1.2 ms per 512^3 voxels
    est_ms = 1.2 * float(shape[0] * shape[1] * shape[2]) / float(512 ** 3)
    settle = min(2000, max(8, int(math.ceil(a.settle_ms / max(est_ms, 1e-3))))) if a.settle_ms > 0 else 0
    settle += settle % 2  # even: the ping-pong pair back where setup left it
    phase(rank, f"sweeps: {settle} settle + {a.warmup} warmup + {a.steps} timed ({s.smooth_kernel_name(0)})")
    if settle:
        s.bench_smooth(0, settle)
    # warmup
    if a.warmup:
        s.bench_smooth(0, a.warmup)
    barrier()
    t0 = time.perf_counter()
    dev_ms, kern_ms, launches = s.bench_smooth(0, a.steps)
    barrier()
    wall = time.perf_counter() - t0
    launch_series = list(s.bench_launch_times())  # in launch order (even: read x / write t, odd: the reverse)
    per_launch = sorted(launch_series)
    if world > 1:
        wall = float(s.allreduce([wall], "max")[0])
    # beside the contract's K steps (24 ms at K = 20): a sustained window of ~2 s of the same
    # sweeps, device-timed, so the rate is also measured over a span a utilisation sampler sees
    sus_n = max(a.steps, int(2000.0 / max(wall / a.steps * 1e3, 0.05)))
    phase(rank, f"sweeps: sustained window of {sus_n}")
    sus_dev, sus_kern, _ = s.bench_smooth(0, sus_n)
    sus_series = list(s.bench_launch_times())
    sus_win = [round(sum(sus_series[q:q + 100]) / len(sus_series[q:q + 100]), 4)
               for q in range(0, len(sus_series), 100)]
    if world > 1:
        sus_dev = float(s.allreduce([sus_dev], "max")[0])
    nvox = float(S) ** 3
    value = nvox * a.steps / wall / 1e6
    info = s.level_info(0)
    nlev = s.num_levels
    kname = s.smooth_kernel_name(0)  # as rocprofv3 prints it (profiles/ are matched on it)
    s.close()
    # V-cycles/s (same volume, nu = 2) on a solver in the production layout (CycleType
    # VCYCLE: level-0 records without b, dense rhs), as GenerateData runs it; the halo form
    # the sweep measurement settled on
    s = make(M.VCYCLE, opts, "vcycle")
    vplacement = s.placement_trials()
    vnote = None
    if opts and a.halo == "auto":
        # the V-cycle's distributed levels push too (per-colour levels after their last colour
        # pass): checked against the RCCL exchange like the sweeps
        ok, why = verify_peer(M, s, make, rank, steps=3, vcycles=True)
        vnote = why if ok else f"V-cycle peer halo rejected ({why}): rccl"
        if not ok:
            s.close()
            s = make(M.VCYCLE, 0, "vcycle-rccl")
    s.vcycle()
    # untimed cycles as the sweeps' settle phase (same count on every rank: ~settle_ms at ~6 sweeps each)
    settle_vc = int(math.ceil(settle / 6.0)) if settle else 0
    if settle_vc:
        s.bench_vcycle(settle_vc)
    barrier()
    t1 = time.perf_counter()
    phase(rank, f"V-cycles: {settle_vc} settle + {a.vcycles} timed")
    vc_ms = s.bench_vcycle(a.vcycles)
    barrier()
    vwall = time.perf_counter() - t1
    if world > 1:
        vwall = float(s.allreduce([vwall], "max")[0])
    s.close()

    if rank != 0:
        return
    # roofline of the dominant kernel: voxel updates per launch from the launch count the
    # library reports (the fused GS / WJ sweep: the whole slab per launch; per-colour GS
    # passes: one colour class per launch)
    units_per_launch = float(shape[0] * shape[1] * shape[2]) * a.steps / max(1, launches)
    achieved = BYTES_PER_VOXEL_SMOOTH * units_per_launch / (kern_ms * 1e-3) / 1e9
    tag = f"{a.smoother}_{S}"
    # (the profile is of the whole 512^3 volume on one GPU: not a rank slab's launch)
    traffic = load_traffic(tag, kname) if world == 1 else None
    roof = {"bound": "hbm", "achieved": round(achieved, 1), "peak": PEAK_HBM_GBS, "unit": "GB/s",
            "frac": round(achieved / PEAK_HBM_GBS, 4),
            "traffic": traffic["bytes_per_launch"] if traffic else None,
            "kernel": kname,
            "kernel_ms_mean": round(kern_ms, 5), "launches": launches,
            "kernel_ms_median": round(per_launch[len(per_launch) // 2], 5) if per_launch else None,
            "kernel_ms_min": round(per_launch[0], 5) if per_launch else None,
            "kernel_ms_series": [round(v, 4) for v in launch_series],
            "algorithmic_bytes_per_launch": BYTES_PER_VOXEL_SMOOTH * units_per_launch}
    if traffic:
        roof["traffic_source"] = traffic.get("source")
        # the same launch priced on its measured HBM bytes (PMC) instead of the algorithmic ones
        roof["traffic_GBs"] = round(traffic["bytes_per_launch"] / (kern_ms * 1e-3) / 1e9, 1)
        roof["traffic_frac"] = round(roof["traffic_GBs"] / PEAK_HBM_GBS, 4)
    line = {
        "metric": "Mvoxel-smooths/s (and V-cycles/s) at 512^3 fp32; achieved HBM GB/s vs peak",
        "value": round(value, 1),
        "unit": "Mvoxel-smooths/s",
        "n_gpus": n_gpus,
        "steps": a.steps,
        "warmup": a.warmup,
        "settle_sweeps": settle,
        "ms_per_step": round(wall / a.steps * 1e3, 4),
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic (device-generated VED-form tensor and counter-hash image)"
                + ("; REHEARSAL: all ranks share GPU 0 (MAD_BENCH_SHARED_GPU)" if shared_gpu else ""),
        "config": {"workload": f"C4 {S}^3 VED-form full tensor, "
                               f"{'4-colour Gauss-Seidel' if a.smoother == 'gs' else 'weighted Jacobi'}"
                               f" level-0 sweeps", "global_shape": list(gshape),
                   "levels": nlev, "time_step": 0.1, "parallelism": f"z-slab x{world}",
                   "halo": (None if world == 1 else
                            ("peer: edge planes stored by the sweep into the neighbours' mailboxes"
                             if "peer halo" in kname else "rccl: grouped send/recv after each sweep")
                            + (f"; {halo_note}" if halo_note else "")),
                   "slab_shape": list(info["shape"])},
        "vcycles_per_s": round(a.vcycles / vwall, 3),
        "vcycle_config": "CycleType VCYCLE (dense rhs layout), nu = 2, 4-colour GS, "
                         f"{nlev} levels, graph-replayed per rank" + (f"; {vnote}" if vnote else ""),
        "device_ms_per_vcycle": round(vc_ms / a.vcycles, 3),
        "ms_per_vcycle": round(vwall / a.vcycles * 1e3, 3),
        "device_ms_per_step": round(dev_ms / a.steps, 4),
        "sustained": {"steps": sus_n, "device_ms_per_step": round(sus_dev / sus_n, 4),
                      "kernel_ms_mean": round(sus_kern, 5),
                      "kernel_ms_per_100": sus_win,
                      "value": round(nvox * sus_n / (sus_dev * 1e-3) / 1e6, 1)},
        "roofline": roof,
        # the level-0 sweep ms (forward, reverse direction) of every set of arrays setup tried, the
        # fastest kept (mad_placement_trials, DESIGN.md "Placement"): which speeds this box offered
        "placement_trials_ms": [round(v, 4) for v in placement],
        "vcycle_placement_trials_ms": [round(v, 4) for v in vplacement],  # the V-cycle layout's level-0 sweep
    }
    if world == 1 and not a.no_precision_cycles:
        # the cycle mad_run runs at the reference tests' Tolerance 1e-10 (MAD_PRECISION_AUTO ->
        # FP32_REFINE: fp32 V-cycle + fp64 residual / update), and in MAD_FP64 (the reference's
        # arithmetic throughout), beside the plain fp32 cycle of the same loop
        pc = {}
        for key, prec in (("fp32", M.FP32), ("refine", M.FP32_REFINE), ("fp64", M.FP64)):
            phase(rank, f"mad_run cycle cost: {key}")
            pc[key] = run_cycle_ms(M, gshape, prec, 12 if key == "refine" else 8, smoother=sm,
                                   gs_kernel=a.gs_kernel)
        line["run_ms_per_cycle"] = {k: (round(v, 3) if v is not None else None) for k, v in pc.items()}
        phase(rank, "solve to 1e-10 (default precision)")
        line["solve_1e-10"] = solve_at_reference_tolerance(M, gshape, smoother=sm, gs_kernel=a.gs_kernel)
        line["refine_vcycles_per_s"] = round(1e3 / pc["refine"], 2) if pc["refine"] else None
        line["fp64_vcycles_per_s"] = round(1e3 / pc["fp64"], 2) if pc["fp64"] else None
        line["run_cycle_config"] = ("mad_run loop at Tolerance 1e-30 (8 cycles, median of cycles 2..8; "
                                    "refine: 12 cycles, median of the refined ones, after its fp32 phase "
                                    "ends at relres 1e-5): V-cycle + fp64 (refine / fp64) or fp32 residual "
                                    "norm + host check; refine = MAD_FP32_REFINE, what MAD_PRECISION_AUTO "
                                    "resolves to at the reference tests' 1e-10; solve_1e-10: one time step "
                                    "to 1e-10 with the default descriptor")
    if world == 1 and not a.no_cpu_baseline:
        phase(rank, "CPU baseline (oracle)")
        cb = cpu_baseline_guarded(a.cpu_seconds, a.cpu_size or S, timeout=a.cpu_timeout)
        line["cpu_baseline"] = cb
    else:
        line["cpu_baseline"] = None
    print(json.dumps(line), flush=True)


if __name__ == "__main__":
    main()
