"""C ABI checks that need no GPU: the library loads, exports every symbol
include/mad.h and include/mad_ved.h declare, validates descriptors, and plans the hierarchy /
z-slab decomposition identically to the oracle's depth rule."""
import ctypes
import os
import re

import numpy as np
import pytest

import multigridanisotropicdiffusion_amd as M
from multigridanisotropicdiffusion_amd import _capi as C

from conftest import ROOT


def header_functions():
    """Every function declared by the C headers (include/mad.h, include/mad_ved.h)."""
    names = set()
    for h in ("mad.h", "mad_ved.h"):
        src = open(os.path.join(ROOT, "include", h)).read()
        src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
        names |= set(re.findall(r"\b(mad_[a-z0-9_]+)\s*\(", src))
    return sorted(names)


def test_library_exports_every_header_symbol():
    L = C.load()
    names = header_functions()
    assert len(names) >= 30
    for n in names:
        assert hasattr(L, n), n
    assert sorted(C.EXPORTS) == names


def test_desc_defaults_match_reference():
    """itkMultigridAnisotropicDiffusionImageFilter.hxx:36-52 defaults."""
    d = C.default_desc()
    assert d.abi_version == C.ABI_VERSION
    assert d.time_step == 0.01 and d.number_of_steps == 1
    assert d.cycle == C.VCYCLE and d.iterations_per_grid == 2
    assert d.tolerance == 1e-6 and d.max_cycles == 100 and d.verbose == 0
    assert d.smoother == C.GAUSS_SEIDEL
    assert abs(d.omega - 2.0 / 3.0) < 1e-16
    assert (C.VCYCLE, C.FMG, C.SMOOTHER) == (0, 1, 2)


def test_max_depth_matches_oracle(oracle_mod):
    rng = np.random.default_rng(0)
    shapes = [(3, 3, 3), (12, 12, 12), (11, 200, 200), (69, 77, 69), (119, 140, 134),
              (512, 512), (255, 257), (6, 7)]
    shapes += [tuple(int(v) for v in rng.integers(3, 300, size=k)) for k in (2, 3) for _ in range(20)]
    for s in shapes:
        assert M.max_depth(s) == oracle_mod.max_depth(s), s


def _plan(shape, spacing=None, nranks=1, rank=0):
    d = C.default_desc()
    d.dim = len(shape)
    size = list(reversed(shape)) + [1] * (3 - len(shape))
    for q in range(3):
        d.size[q] = size[q]
        d.spacing[q] = (spacing[q] if spacing and q < len(shape) else 1.0)
    d.nranks, d.rank = nranks, rank
    out = []
    L = C.load()
    nl = None
    l = 0
    while True:
        n = (ctypes.c_int64 * 3)()
        h = (ctypes.c_double * 3)()
        c = (ctypes.c_int32 * 3)()
        z0, z1, dist = ctypes.c_int64(), ctypes.c_int64(), ctypes.c_int32()
        r = L.mad_plan_level(ctypes.byref(d), l, n, h, c, ctypes.byref(z0), ctypes.byref(z1),
                             ctypes.byref(dist))
        if r < 0:
            raise C.MadError(-r, L.mad_last_error(None).decode())
        nl = r
        out.append(dict(n=list(n), h=list(h), c=list(c), z0=z0.value, z1=z1.value, dist=dist.value))
        l += 1
        if l >= nl:
            return out


@pytest.mark.parametrize("shape", [(69, 77, 69), (119, 140, 134), (55, 52, 54), (24, 26, 28), (256, 256)])
def test_plan_matches_oracle_hierarchy(oracle_mod, shape):
    T = np.stack([np.ones(shape)] * (3 if len(shape) == 2 else 6))
    o = oracle_mod.Oracle(shape, [1.0] * len(shape), T, 0.1)
    p = _plan(shape)
    assert len(p) == o.num_levels
    for l, lv in enumerate(o.levels):
        assert tuple(reversed(p[l]["n"][: len(shape)])) == lv["shape"]
        assert p[l]["c"][: len(shape)] == lv["centering"]
        assert p[l]["h"][: len(shape)] == lv["spacing"]
        assert p[l]["dist"] == 0 and p[l]["z0"] == 0


@pytest.mark.parametrize("nranks", [2, 4, 8])
def test_plan_slabs_cover_and_align(nranks):
    """z-slabs tile every distributed level exactly, are coarsening-aligned (fine
    planes 2K, 2K+1 on the rank that owns coarse plane K) and coarse levels are
    replicated on every rank."""
    shape = (512, 512, 512)
    plans = [_plan(shape, nranks=nranks, rank=r) for r in range(nranks)]
    nl = len(plans[0])
    assert nl == 7
    for l in range(nl):
        dist = [p[l]["dist"] for p in plans]
        assert len(set(dist)) == 1
        nz = plans[0][l]["n"][2]
        if dist[0]:
            ranges = sorted((p[l]["z0"], p[l]["z1"]) for p in plans)
            assert ranges[0][0] == 0 and ranges[-1][1] == nz
            for (a0, a1), (b0, b1) in zip(ranges, ranges[1:]):
                assert a1 == b0
            assert all(z1 - z0 >= 4 for z0, z1 in ranges)
            if l > 0 and plans[0][l - 1]["dist"]:
                for p in plans:
                    assert p[l - 1]["z0"] == 2 * p[l]["z0"] and p[l - 1]["z1"] == 2 * p[l]["z1"]
        else:
            assert all(p[l]["z0"] == 0 and p[l]["z1"] == nz for p in plans)
    assert plans[0][0]["dist"] == 1
    assert plans[0][nl - 1]["dist"] == 0


@pytest.mark.parametrize("gshape,nranks,msp,msv,depths", [
    # planes alone (min_slab_voxels 1)
    ((512, 512, 512), 8, 0, 1, [64, 32, 16, 8, 4]), ((512, 512, 512), 8, 16, 1, [64, 32, 16]),
    ((512, 512, 512), 8, 64, 1, [64]), ((512, 512, 512), 4, 8, 1, [128, 64, 32, 16, 8]),
    ((512, 512, 512), 2, 32, 1, [256, 128, 64, 32]),
    # the defaults: >= 4 planes and >= 128 K voxels per rank
    ((512, 512, 512), 8, 0, 0, [64, 32, 16]), ((512, 512, 512), 4, 0, 0, [128, 64, 32]),
    ((512, 512, 512), 2, 0, 0, [256, 128, 64, 32]), ((512, 1024, 1024), 8, 0, 0, [64, 32, 16, 8]),
    # voxels alone
    ((512, 512, 512), 8, 0, 1 << 20, [64, 32]),
])
def test_plan_min_slab_planes(gshape, nranks, msp, msv, depths):
    """mad_desc.min_slab_planes / min_slab_voxels: coarse levels stay distributed while every rank
    keeps that many planes and voxels (level 0 always: >= 4 planes); the rest is replicated
    (agglomeration)."""
    from multigridanisotropicdiffusion_amd import distributed as D
    p = D.plan(gshape, nranks, nranks - 1, msp, msv)
    assert [q["z1"] - q["z0"] for q in p if q["distributed"]] == depths
    assert all(not q["distributed"] for q in p[len(depths):])


def test_plan_rejects_bad_slab_requests():
    with pytest.raises(C.MadError):
        _plan((510, 512, 512), nranks=4)  # 510 planes do not split into 4
    with pytest.raises(C.MadError):
        _plan((512, 512), nranks=2)  # 2D images are not z-sliced


def test_slab_range():
    assert M.slab_range(512, 8, 3) == (192, 256)
    with pytest.raises(C.MadError):
        M.slab_range(100, 8, 0)


def test_create_rejects_bad_descriptors():
    """Validation runs before any device call, so these are safe without a GPU."""
    L = C.load()
    for mutate in (lambda d: setattr(d, "dim", 4), lambda d: setattr(d, "abi_version", 99),
                   lambda d: d.size.__setitem__(0, 2), lambda d: setattr(d, "cycle", 7),
                   lambda d: setattr(d, "nranks", 0), lambda d: setattr(d, "precision", 5)):
        d = C.default_desc()
        d.size[0] = d.size[1] = d.size[2] = 16
        mutate(d)
        ctx = ctypes.c_void_p()
        rc = L.mad_create(ctypes.byref(d), ctypes.byref(ctx))
        assert rc == C.ERR_INVALID
        assert not ctx.value
        assert L.mad_last_error(None)


def test_kernel_entry_points_reject_null_context():
    L = C.load()
    assert L.mad_smooth(None, 0, 1) == C.ERR_INVALID
    assert L.mad_vcycle(None) == C.ERR_INVALID
    assert L.mad_num_levels(None) == -1


def test_ved_desc_defaults_match_reference():
    """itkVEDMultigridImageFilter.hxx:34-58 defaults (mad_ved_desc_init)."""
    L = C.load()
    d = C.VedDesc()
    assert L.mad_ved_desc_init(ctypes.byref(d)) == C.OK
    assert (d.alpha, d.beta, d.gamma, d.epsilon, d.omega, d.sensitivity) == (0.5, 0.5, 5.0, 0.01, 5.0, 10.0)
    assert d.nscales == 5 and list(d.scales[:5]) == [0.300, 0.482, 0.775, 1.245, 2.000]
    assert (d.iterations, d.diffusion_iterations, d.diffusion_iterations_per_grid) == (1, 5, 2)
    assert d.cycle == C.VCYCLE and d.time_step == 0.1 and d.tolerance == 1e-6
    assert d.nranks == 1 and d.rank == 0


@pytest.mark.parametrize("field,value", [("nscales", 0), ("nscales", 17), ("sensitivity", 0.0),
                                         ("abi_version", 99)])
def test_ved_create_rejects_bad_descriptors(field, value):
    """Validated before any device work (runs without a GPU)."""
    L = C.load()
    d = C.VedDesc()
    L.mad_ved_desc_init(ctypes.byref(d))
    d.size[0] = d.size[1] = d.size[2] = 16
    setattr(d, field, value)
    ctx = ctypes.c_void_p()
    assert L.mad_ved_create(ctypes.byref(d), ctypes.byref(ctx)) == C.ERR_INVALID
    assert not ctx.value
    assert L.mad_ved_last_error(None)
