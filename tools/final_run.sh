#!/bin/bash
# The round's closing GPU evidence on HEAD, as the driver runs it: build() from source on the
# box, the whole -m gpu suite, smoke(), the default bench line.  Logs: gpurun_out/final_*.log
bash tools/gpu_steps.sh \
  "final_build|600|python -c 'import __graft_entry__ as g; g.build()'" \
  "final_gputests|900|python -u -m pytest tests -m gpu -x -q --timeout 900 --timeout-method thread" \
  "final_smoke|300|python -c 'import __graft_entry__ as g; g.smoke()'" \
  "final_bench|300|python bench.py"
