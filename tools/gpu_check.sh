#!/bin/bash
# GPU tests, then three bench runs (no CPU baseline) and the per-config lines.
set -e
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gputest.log 2>&1
for i in 1 2 3; do
  timeout -k 10 120 python -u bench.py --no-cpu-baseline --host-api-steps 0 --steps 300 > gpurun_out/bench_$i.log 2>&1
done
timeout -k 10 200 python3 tools/bench_configs.py > gpurun_out/configs.log 2>&1
