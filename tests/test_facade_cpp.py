"""The C++ ITK-shaped facade (include/mad_itk.hpp) compiles against the C ABI
header, links libmad_hip.so, and runs like the reference's 2D test program."""
import os
import subprocess

import pytest

from conftest import ROOT

SRC = os.path.join(ROOT, "tests", "cpp", "facade_test.cpp")
LIBDIR = os.path.join(ROOT, "multigridanisotropicdiffusion_amd")


@pytest.fixture(scope="module")
def exe(tmp_path_factory):
    out = str(tmp_path_factory.mktemp("facade") / "facade_test")
    subprocess.check_call(["g++", "-std=c++17", "-O1", "-Wall", "-Werror", "-I",
                           os.path.join(ROOT, "include"), SRC, "-o", out, "-L", LIBDIR,
                           "-lmad_hip", f"-Wl,-rpath,{LIBDIR}"])
    return out


def test_facade_builds_and_host_calls(exe):
    r = subprocess.run([exe, "host"], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    assert "host ok" in r.stdout


@pytest.mark.gpu
def test_facade_runs_filter(exe):
    r = subprocess.run([exe, "run"], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "run ok" in r.stdout


@pytest.mark.gpu
def test_facade_benchmark_output(exe, tmp_path):
    """SetBenchmark(true), the reference's -DBENCHMARK build: benchmark.txt in the working
    directory with 2 nu + 1 "relres_seconds" lines per V-cycle (MAD.hxx:401-409, 450-458, 477-485)."""
    r = subprocess.run([exe, "run", "bench"], capture_output=True, text=True, timeout=300, cwd=tmp_path)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "run ok" in r.stdout and "benchmark lines=" in r.stdout
    lines = (tmp_path / "benchmark.txt").read_text().split()
    rel = [float(ln.split("_")[0]) for ln in lines]
    assert len(lines) % 5 == 0 and rel[-1] <= 1e-6


@pytest.mark.gpu
def test_facade_runs_ved_filter(exe):
    r = subprocess.run([exe, "ved"], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "ved ok" in r.stdout
