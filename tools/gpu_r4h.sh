#!/bin/bash
# the whole GPU suite, then a 200-step bench line
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}; mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest -v --timeout 250 --timeout-method thread tests -m gpu > gpurun_out/t_all.log 2>&1; rc=$?
grep -E "passed|failed" gpurun_out/t_all.log | tail -2; grep -E "FAILED|full batch:" gpurun_out/t_all.log | cut -c1-400 | head
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 200 --warmup 20 > gpurun_out/bench_r4h.log 2>&1 || exit 1
tail -1 gpurun_out/bench_r4h.log | cut -c1-300
