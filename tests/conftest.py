import os
import signal
import socket
import subprocess
import sys
import tempfile

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through the HIP library)")
    config.addinivalue_line("markers", "slow: longer GPU cases")


# ---------------------------------------------------------------- multi-process RCCL job
# tests/test_gpu_multiproc.py compares N RCCL rank processes with the LOCAL transport.  The
# rank processes must start before this process makes any GPU call, so they are launched at
# session start (when the gpu tests are selected and >= 2 GPUs are visible) and joined by the
# test.  GPUs are counted in a child process: this one must not initialise HIP first.

_MP = {}


def _gpu_selected(config):
    m = config.getoption("markexpr", "") or ""
    return "gpu" in m and "not gpu" not in m


def _count_gpus():
    code = ("import ctypes\n"
            "for n in ('libamdhip64.so', '/opt/rocm/lib/libamdhip64.so'):\n"
            "    try:\n        L = ctypes.CDLL(n); break\n"
            "    except OSError:\n        L = None\n"
            "c = ctypes.c_int(0)\n"
            "print(c.value if L is not None and L.hipGetDeviceCount(ctypes.byref(c)) == 0 else 0)\n")
    try:
        r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=120)
        return int(r.stdout.strip().splitlines()[-1]) if r.returncode == 0 else 0
    except (subprocess.SubprocessError, ValueError, IndexError):
        return 0


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def pytest_sessionstart(session):
    config = session.config
    if not _gpu_selected(config) or os.environ.get("MAD_SKIP_MULTIPROC"):
        return
    ngpu = _count_gpus()
    world, shared = min(ngpu, 8), False
    if world < 2:
        if ngpu < 1 or os.environ.get("MAD_SKIP_SHARED_MULTIPROC"):
            return
        # one GPU: two RCCL rank processes share it.  RCCL refuses two ranks of one
        # communicator on one device of one host ("Duplicate GPU"); a distinct NCCL_HOSTID per
        # rank makes them two hosts to RCCL, so they connect over its socket transport
        # (loopback) -- real two-process RCCL (bootstrap, grouped send/recv, allreduce,
        # allgather, graph-captured V-cycles), with host-staged bytes instead of xGMI.
        # (MAD_SHARED_MULTIPROC_WORLD: more rank processes on the one GPU, e.g. 4 for interior
        # ranks with two neighbours; each one polls its neighbours' peer counters with <= 128
        # workgroups, so a few ranks leave the sweeps they wait for enough CUs)
        world, shared = max(2, min(4, int(os.environ.get("MAD_SHARED_MULTIPROC_WORLD", "2")))), True
    outdir = tempfile.mkdtemp(prefix="mad_mp_")
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()),
               WORLD_SIZE=str(world))
    env.setdefault("NCCL_SOCKET_IFNAME", "lo")  # one node: bootstrap on loopback
    procs, logs = [], []
    for r in range(world):
        log = os.path.join(outdir, f"rank{r}.log")
        renv = dict(env, RANK=str(r), LOCAL_RANK=str(r))
        if shared:
            # INFO on the INIT / NET subsystems: the log names the transport RCCL connected
            # the two ranks with (the test checks it is the network one, NET/Socket)
            renv.update(MAD_MP_DEVICE="0", NCCL_HOSTID=f"mad-shared-gpu-rank{r}",
                        NCCL_IB_DISABLE="1", NCCL_DEBUG="INFO", NCCL_DEBUG_SUBSYS="INIT,NET")
        with open(log, "w") as f:
            procs.append(subprocess.Popen(
                [sys.executable, os.path.join(ROOT, "tests", "mp_rank.py"), outdir],
                env=renv, stdout=f, stderr=subprocess.STDOUT,
                cwd=ROOT, start_new_session=True))
        logs.append(log)
    _MP["job"] = dict(procs=procs, logs=logs, outdir=outdir, world=world, shared=shared)


def pytest_collection_modifyitems(session, config, items):
    """The RCCL rank job started at session start runs on every GPU (device 0 included): its
    test goes first, so it is joined before any timing-sensitive or memory-heavy GPU test
    shares the devices with it."""
    items.sort(key=lambda it: 0 if "test_gpu_multiproc.py" in it.nodeid else 1)


def multiproc_job(config):
    return _MP.get("job")


def join_multiproc(job, timeout):
    """Exit codes of the rank processes; kills the whole job (every process group) when one
    fails or the time runs out, so no rank is left waiting in a collective."""
    import time
    t_end = time.monotonic() + timeout
    procs = job["procs"]
    while time.monotonic() < t_end:
        rcs = [p.poll() for p in procs]
        if all(rc is not None for rc in rcs) or any(rc not in (None, 0) for rc in rcs):
            break
        time.sleep(0.5)
    _kill_job(job)
    return [p.poll() if p.poll() is not None else -9 for p in procs]


def _kill_job(job):
    for p in job["procs"]:
        if p.poll() is None:
            try:
                os.killpg(p.pid, signal.SIGKILL)
            except ProcessLookupError:
                pass
    for p in job["procs"]:
        try:
            p.wait(30)
        except subprocess.TimeoutExpired:
            pass


def pytest_sessionfinish(session, exitstatus):
    job = _MP.pop("job", None)
    if job is not None:
        _kill_job(job)


@pytest.fixture(scope="session")
def oracle_mod():
    import oracle
    oracle.build()
    return oracle


def load_golden(name):
    with np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False) as z:
        return {k: z[k] for k in z.files}
