"""Time the level-0 sweep only (512^3 VED-form, fp32, SMOOTHER mode as bench.py): one line
   kernel-name  mean-ms  min-ms.  MAD_HIP_LIB selects a measurement build."""
import sys
import os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import multigridanisotropicdiffusion_amd as M

S = int(sys.argv[1]) if len(sys.argv) > 1 else 512
s = M.Solver((S, S, S), time_step=0.1, precision=M.FP32, cycle=M.SMOOTHER)
s.synth_tensor(kind=0, seed=4)
s.setup()
s.synth_level(0, M.capi.B, 3)
s.synth_level(0, M.capi.X, 3)
s.bench_smooth(0, 3)
dev, kern, n = s.bench_smooth(0, 10)
t = sorted(s.bench_launch_times())
print(os.environ.get("MAD_HIP_LIB", "default"), s.smooth_kernel_name(0), round(kern, 4), round(t[0], 4), flush=True)
s.close()
