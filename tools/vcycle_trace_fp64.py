"""FP64 V-cycles of the bench workload (512^3 VED-form) for a kernel trace:
    rocprofv3 --kernel-trace --output-format csv -d OUT -o vc -- python3 tools/vcycle_trace_fp64.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import multigridanisotropicdiffusion_amd as M
    S = 512
    s = M.Solver((S, S, S), time_step=0.1, cycle=M.VCYCLE, precision=M.FP64)
    s.synth_tensor(kind=0, seed=4)
    s.setup()
    s.synth_level(0, M.capi.B, 3)
    s.synth_level(0, M.capi.X, 3)
    s.vcycle()
    s.vcycle()
    print("ms per V-cycle", s.bench_vcycle(10) / 10, flush=True)
    s.close()


if __name__ == "__main__":
    main()
