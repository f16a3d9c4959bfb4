"""Debug: residual of every level vs the oracle (checks the restricted operators)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import multigridanisotropicdiffusion_amd as M  # noqa: E402
import oracle  # noqa: E402
from conftest import load_golden  # noqa: E402

for name in sys.argv[1:]:
    g = load_golden(name)
    shape = tuple(int(s) for s in g["shape"])
    s = M.Solver(shape, tuple(g["spacing"]), time_step=float(g["dt"]), precision=M.FP64)
    s.set_tensor(g["tensor"])
    s.setup()
    o = oracle.Oracle(shape, tuple(g["spacing"]), g["tensor"], float(g["dt"]))
    rng = np.random.default_rng(0)
    for l in range(s.num_levels):
        ls = s.shape_at(l)
        x = rng.random(ls)
        b = np.zeros(ls)
        s.upload(l, M.capi.X, x)
        s.upload(l, M.capi.B, b)
        s.residual(l)
        r = s.download(l, M.capi.R)
        ro = o.residual(l, x, b)
        print(name, l, ls, "resid relerr", np.abs(r - ro).max() / np.abs(ro).max())
    for l in range(s.num_levels - 1):
        ls = s.shape_at(l)
        r = rng.random(ls)
        s.upload(l, M.capi.R, r)
        s.restrict(l)
        rc = s.download(l + 1, M.capi.B)
        ro = o.restrict(l, r)
        print(name, l, "restrict relerr", np.abs(rc - ro).max() / np.abs(ro).max())
        t = g["tensor"]
        print("tensor shape", t.shape)
