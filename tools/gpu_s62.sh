#!/bin/bash
# the four-tile sweep for 32 < n <= 62 (two-hand scene): its parity tests, then configs 5 / 5p / 3
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}; mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest -v -s --timeout 400 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_env.py \
  -k "bimanual or handover" > gpurun_out/s62_t.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR" gpurun_out/s62_t.log | cut -c1-150 | head -20; grep -E "bimanual full batch" gpurun_out/s62_t.log | sed 's/deep mesh-mesh.*unexplained/ ... unexplained/' | cut -c1-330
if [ $rc != 0 ]; then echo "pytest rc=$rc"; grep -E "Error|assert" gpurun_out/s62_t.log | head; exit $rc; fi
timeout -k 10 400 python -u tools/bench_configs.py 5 5p 3 > gpurun_out/s62_cfg.log 2>&1 || { tail -5 gpurun_out/s62_cfg.log; exit 1; }
cut -c1-200 gpurun_out/s62_cfg.log
