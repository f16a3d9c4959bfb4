"""mad_run in the default precision at the reference tests' 1e-10 (MAD_FP32_REFINE) on a 256^3 VED-form
system, output saved: run once per library build (MAD_HIP_LIB) and compare the files bit for bit.
    python tools/refine_fold_ab.py OUT.npy [size]"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import multigridanisotropicdiffusion_amd as M
    out_path = sys.argv[1]
    S = int(sys.argv[2]) if len(sys.argv) > 2 else 256
    s = M.Solver((S, S, S), time_step=0.1, tolerance=1e-10, number_of_steps=2)
    s.synth_tensor(kind=0, seed=4)
    s.setup()
    rng = np.random.default_rng(3)
    img = (rng.random((S, S, S), dtype=np.float32) * 100).astype(np.float32)
    t0 = time.perf_counter()
    out, st = s.run(img)
    dt = time.perf_counter() - t0
    np.save(out_path, out)
    print(os.environ.get("MAD_HIP_LIB", "in-tree"), "cycles", st["step_cycles"], "relres", st["last_relres"],
          "solve_ms", round(st["solve_ms"], 2), "wall_s", round(dt, 2), flush=True)
    s.close()


if __name__ == "__main__":
    main()
