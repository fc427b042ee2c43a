#!/bin/bash
# round 5: M's rows in registers on the non-incremental Newton path (reach scenes): env +
# parity tests, the reach configs
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_env.py tests/test_gpu_parity.py tests/test_gpu_kat.py -m gpu > gpurun_out/t_y.log 2>&1 || { echo "tests rc=$?"; grep -E "^FAILED|Error" gpurun_out/t_y.log | head; tail -3 gpurun_out/t_y.log; exit 1; }
tail -1 gpurun_out/t_y.log
timeout -k 10 300 python -u tools/bench_configs.py 2 "2'" > gpurun_out/configs_y.log 2>&1 || { tail -5 gpurun_out/configs_y.log; exit 1; }
grep -v amdgpu.ids gpurun_out/configs_y.log
