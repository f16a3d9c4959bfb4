import os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, "tests"))
import multigridanisotropicdiffusion_amd as M
import synth
SHAPE = tuple(int(v) for v in sys.argv[1:4])
T = synth.random_spd(SHAPE, seed=3)
s = M.Solver(SHAPE, time_step=0.4)
s.set_tensor(T); s.setup()
s.upload(0, M.capi.X, synth.image(SHAPE, seed=1)); s.upload(0, M.capi.B, synth.image(SHAPE, seed=2))
print("norm", s.residual(0))
r = s.download(0, M.capi.R)
bad = np.argwhere(~np.isfinite(r))
print("nonfinite", len(bad), bad[:10])
