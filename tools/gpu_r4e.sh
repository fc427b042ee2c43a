#!/bin/bash
# kernel trace of a bench run with the mid tier (W start / end against the step kernel)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d $R/gpurun_out/midtrace -o run --output-format csv -- \
  python3 $R/bench.py --steps 200 --warmup 10 --no-cpu-baseline --host-api-steps 0 > $R/gpurun_out/midtrace.log 2>&1
