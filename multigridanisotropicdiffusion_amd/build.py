"""Build libmad_hip.so in-tree with hipcc for gfx950 (no CMake, no JIT cache).

    python -m multigridanisotropicdiffusion_amd.build
"""
import os
import shutil
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
OUT = os.path.join(HERE, "libmad_hip.so")
SOURCES = ["mad_solver.hip"]
DEPS = ["../../include/mad.h", "../../include/mad_ved.h"]


def deps():
    """every source the library is compiled from: csrc/*.hip, csrc/*.hpp and the C headers"""
    return [f for f in os.listdir(CSRC) if f.endswith((".hip", ".hpp"))] + DEPS


def hipcc():
    for cand in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if cand and os.path.exists(cand):
            return cand
    raise RuntimeError("hipcc not found")


def up_to_date():
    if not os.path.exists(OUT):
        return False
    t = os.path.getmtime(OUT)
    return all(os.path.getmtime(os.path.join(CSRC, d)) <= t for d in deps())


def build(force=False, verbose=True):
    if not force and up_to_date():
        return OUT
    cmd = [hipcc(), "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared",
           "-Wall", "-Wno-unused-function", "-o", OUT + ".tmp"]
    cmd += [os.path.join(CSRC, s) for s in SOURCES]
    cmd += ["-lrccl", "-lrocsolver", "-lrocblas"]
    if verbose:
        print(" ".join(cmd), flush=True)
    subprocess.check_call(cmd, cwd=HERE)
    os.replace(OUT + ".tmp", OUT)
    return OUT


if __name__ == "__main__":
    build(force="--force" in sys.argv)
