#!/bin/bash
# The round's closing GPU evidence on HEAD, as the driver runs it: build() from source on the
# box, the whole -m gpu suite, smoke(), the default bench line, then the rocprofv3 evidence for
# the bench kernel (kernel trace + stats of the bench command, FETCH_SIZE / WRITE_SIZE passes).
# Logs: gpurun_out/final_*.log, profile CSVs: gpurun_out/final_prof/
bash tools/gpu_steps.sh \
  "final_build|600|python -c 'import __graft_entry__ as g; g.build()'" \
  "final_gputests|1100|python -u -m pytest tests -m gpu -x -q --timeout 900 --timeout-method thread" \
  "final_smoke|300|python -c 'import __graft_entry__ as g; g.smoke()'" \
  "final_bench|300|python bench.py" \
  "final_prof|900|bash tools/profile_round.sh final_prof" \
  "final_vcycle_prof|700|bash tools/vcycle_profiles.sh"
# (not part of the driver's run) the bench's N = 2 torchrun launch and V-cycle forms with two RCCL
# ranks sharing the one GPU
bash tools/gpu_steps.sh "final_rehearse|500|bash tools/rehearse_vcycles.sh"
