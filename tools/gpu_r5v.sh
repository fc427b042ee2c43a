#!/bin/bash
# round 5: M's rows in registers for the Newton products -- parity subset, then same-box A/B
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_env.py -m gpu > gpurun_out/t_mreg.log 2>&1 || { echo "tests rc=$?"; grep -E "^FAILED|Error" gpurun_out/t_mreg.log | head; tail -3 gpurun_out/t_mreg.log; exit 1; }
tail -1 gpurun_out/t_mreg.log
bash tools/ab_multi.sh 3 new "" head "DX_LIB=variants/head/libdx.so" || exit 1
