"""bench.py's output contract: the CPU baseline leg (runs here) and one short bench run on
the GPU (a reduced volume; the JSON line's keys and their consistency)."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_cpu_baseline_leg_reports_the_oracle():
    sys.path.insert(0, ROOT)
    import bench
    cb = bench.cpu_baseline(0.05, 24)
    assert cb["value"] > 0 and cb["unit"] == "Mvoxel-smooths/s"
    assert cb["cores"] == 1 and cb["kind"] == "port" and cb["sample"].startswith("24^3")
    assert cb["host_cpus_available"] >= 1 and cb["host_cpus_total"] >= cb["host_cpus_available"]
    par = cb["parallel"]
    assert par["value"] > 0 and par["cores"] >= 1 and par["kind"] == "port"
    assert cb["vcycle"]["value"] > 0 and cb["vcycle"]["unit"] == "V-cycles/s"
    assert cb["sample_128"]["value"] > 0 and "128^3" in cb["sample_128"]["sample"]


def test_cpu_baseline_falls_back_when_host_memory_is_short():
    """The 512^3 oracle needs ~47 GB of host memory: below 1.5x that in MemAvailable the leg
    runs the small sample instead, and says why, so the GPU line is never lost to it."""
    sys.path.insert(0, ROOT)
    import bench
    cb = bench.cpu_baseline_guarded(0.05, 512, mem_available=8 << 30, fallback_size=24)
    assert cb["value"] > 0 and "MemAvailable" in cb["fallback"]
    assert cb["sample"].startswith("FALLBACK to 24^3") and "24^3" in cb["sample"]


def test_cpu_baseline_falls_back_when_over_its_time_bound():
    sys.path.insert(0, ROOT)
    import bench
    cb = bench.cpu_baseline_guarded(0.05, 40, timeout=0.01, fallback_size=24)
    assert cb["value"] > 0 and "bound" in cb["fallback"] and cb["sample"].startswith("FALLBACK to 24^3")
    # both legs failing still returns a line (value None, the reasons in `error`)
    cb = bench.cpu_baseline_guarded(0.05, 40, timeout=0.01, fallback_timeout=0.01, fallback_size=24)
    assert cb["value"] is None and "bound" in cb["error"]


@pytest.mark.gpu
@pytest.mark.parametrize("extra", [[], ["--smoother", "wj"], ["--gs-kernel", "1"]])
def test_bench_json_line(extra):
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--size", "256", "--steps", "4",
           "--warmup", "1", "--vcycles", "2", "--no-cpu-baseline"] + extra
    out = subprocess.run(cmd, capture_output=True, text=True, timeout=110, cwd=ROOT)
    assert out.returncode == 0, out.stderr[-2000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1
    d = json.loads(lines[0])
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step",
              "higher_is_better", "scaling", "vs_baseline", "dtype", "data", "config",
              "roofline", "cpu_baseline"):
        assert k in d, k
    assert d["n_gpus"] == 1 and d["steps"] == 4 and d["dtype"] == "f32"
    assert d["value"] > 0 and d["vcycles_per_s"] > 0
    assert d["refine_vcycles_per_s"] > 0 and d["fp64_vcycles_per_s"] > 0
    assert set(d["run_ms_per_cycle"]) == {"fp32", "refine", "fp64"}
    sv = d["solve_1e-10"]
    assert sv["precision"] == "FP32_REFINE" and sv["relres"] <= 1e-10
    assert 0 < sv["fp32_phase_cycles"] < sv["cycles"] <= 100 and sv["solve_ms"] > 0
    # value = voxels x steps / wall time
    assert abs(d["value"] - 256 ** 3 * 4 / (d["ms_per_step"] * 4e-3) / 1e6) <= 0.01 * d["value"]
    r = d["roofline"]
    assert r["bound"] == "hbm" and r["peak"] == 8000.0 and r["unit"] == "GB/s"
    assert abs(r["frac"] - r["achieved"] / r["peak"]) < 1e-3
    # per-colour passes: four launches per sweep, each a quarter of the voxels
    nl = 4 if extra == ["--gs-kernel", "1"] else 1
    assert r["launches"] == 4 * nl
    assert r["algorithmic_bytes_per_launch"] == 36.0 * 256 ** 3 / nl
    assert 0 < r["kernel_ms_min"] <= r["kernel_ms_median"]


def test_gpus_must_match_world_size():
    """bench.py starts no processes: --gpus N without N launched ranks is an error, not
    a 1-GPU run reported as N GPUs."""
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2"],
                         capture_output=True, text=True, timeout=60, cwd=ROOT, env=env)
    assert out.returncode != 0 and "WORLD_SIZE" in out.stderr


class _FakeSolver:
    """Stands in for a rank's solver in verify_peer: `result` is what its slab holds after the
    sweeps (None: the sweeps raise), `others_same` what the other ranks report."""
    def __init__(self, result, others_same=True):
        self.result, self.others_same, self.synth, self.closed = result, others_same, [], False

    def smooth(self, level, sweeps):
        if self.result is None:
            raise RuntimeError("mailbox wait timed out")

    def vcycle(self):
        self.cycles = getattr(self, "cycles", 0) + 1
        if self.result is None:
            raise RuntimeError("mailbox wait timed out")

    def download(self, level, which):
        return self.result.copy()

    def allreduce(self, values, op="sum"):
        assert op == "max"  # Solver.allreduce: "sum" or "max"
        return [max(values[0], 0.0 if self.others_same else 1.0)]

    def synth_level(self, level, which, seed):
        self.synth.append((level, which, seed))

    def synchronize(self):
        pass

    def close(self):
        self.closed = True


@pytest.mark.parametrize("vcycles", [False, True])
@pytest.mark.parametrize("case", ["equal", "differs", "raises", "other_rank"])
def test_halo_auto_uses_peer_only_when_bitwise_equal(case, vcycles):
    """--halo auto (the default for N > 1): the peer halo is kept only when every rank's slab
    after the check sweeps is bit-identical to the RCCL exchange's; a device error in the peer
    sweeps is a rejection too, and the RCCL check solver is always closed."""
    import types
    import numpy as np
    sys.path.insert(0, ROOT)
    import bench
    x = np.arange(24, dtype=np.float32).reshape(2, 3, 4)
    y = x.copy()
    if case == "differs":
        y[1, 2, 3] = np.nextafter(y[1, 2, 3], np.float32(1e9))
    peer = _FakeSolver(None if case == "raises" else y)
    ref = _FakeSolver(x, others_same=case != "other_rank")
    M = types.SimpleNamespace(SMOOTHER=2, VCYCLE=0, capi=types.SimpleNamespace(X=0))
    made = []

    def make(cycle, opts, tag):
        made.append((cycle, opts))
        return ref

    ok, note = bench.verify_peer(M, peer, make, rank=1, steps=3, vcycles=vcycles)
    assert made == [(0 if vcycles else 2, 0)]  # the reference solver exchanges through RCCL
    assert ref.closed and not peer.closed
    if vcycles:
        assert ref.cycles == 3 and (case == "raises" or peer.cycles == 3)
    assert ok == (case == "equal")
    if ok:
        assert peer.synth == [(0, 0, 3)] and "bitwise equal" in note
    else:
        assert peer.synth == []
        assert {"differs": "this rank", "raises": "timed out", "other_rank": "another rank"}[case] in note


@pytest.mark.gpu
@pytest.mark.parametrize("halo", ["auto", "rccl"])
def test_bench_two_ranks_on_one_gpu(halo):
    """The driver's N > 1 launch (torch.distributed.run, one process per rank), rehearsed with
    both ranks on device 0 (MAD_BENCH_SHARED_GPU: RCCL over its socket transport): the line is
    printed once, by rank 0, and the default halo form is the peer halo only after its in-run
    bitwise check against the RCCL exchange passed (bench.verify_peer)."""
    import socket
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    env = dict(os.environ, MAD_BENCH_SHARED_GPU="1")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.join(ROOT, "bench.py"),
           "--gpus", "2", "--size", "256", "--steps", "4", "--warmup", "1", "--vcycles", "2",
           "--no-cpu-baseline", "--no-precision-cycles", "--halo", halo]
    out = subprocess.run(cmd, capture_output=True, text=True, timeout=150, cwd=ROOT, env=env)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out.stdout[-2000:]
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["value"] > 0 and d["vcycles_per_s"] > 0
    assert d["config"]["slab_shape"] == [128, 256, 256] and d["config"]["parallelism"] == "z-slab x2"
    h = d["config"]["halo"]
    if halo == "auto":
        assert h.startswith("peer:") and "verified in this run" in h, h
        assert "peer halo" in d["roofline"]["kernel"]
        # the V-cycle solver's peer levels (the per-colour ones included) checked the same way
        assert "verified in this run: 3 V-cycles" in d["vcycle_config"], d["vcycle_config"]
    else:
        assert h.startswith("rccl:") and "peer halo" not in d["roofline"]["kernel"], h
