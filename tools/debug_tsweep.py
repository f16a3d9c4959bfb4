"""Where does one gs_tsweep_k sweep (gs_kernel 7) differ from the per-colour passes?
Prints, per colour class and z-plane, the number of differing points after one sweep."""
import sys
import os
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
import multigridanisotropicdiffusion_amd as M
import synth

for shape in [(16, 16, 16), (24, 40, 36)]:
    T = synth.random_spd(shape, seed=1)
    outs = []
    for v in (1, 7):
        s = M.Solver(shape, (1.0, 0.8, 1.3), time_step=0.7, precision=M.FP32, gs_kernel=v)
        s.set_tensor(T)
        s.setup()
        s.upload(0, M.capi.X, synth.image(shape, seed=4))
        s.upload(0, M.capi.B, synth.image(shape, seed=5))
        s.smooth(0, 1)
        outs.append(s.download(0, M.capi.X))
        s.close()
    d = outs[0] != outs[1]
    nz, ny, nx = shape
    k, j, i = np.meshgrid(np.arange(nz), np.arange(ny), np.arange(nx), indexing="ij")
    col = ((i + k) & 1) | (((j + k) & 1) << 1)
    print(shape, "differing points", d.sum(), "of", d.size, "max", np.abs(outs[0] - outs[1]).max())
    for c in range(4):
        print("  colour", c, "per plane:", [int((d & (col == c))[z].sum()) for z in range(nz)])
    z = int(np.argmax(d.any(axis=(1, 2)))) if d.any() else 0
    print("  first plane with differences", z, "rows:", np.nonzero(d[z].any(axis=1))[0][:20],
          "cols:", np.nonzero(d[z].any(axis=0))[0][:20])
