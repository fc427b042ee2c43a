#!/bin/bash
# env / task tests after the observation change, then the bench three times
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}; mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -q --timeout 250 --timeout-method thread tests/test_gpu_env.py tests/test_gpu_parity.py -k "env or reward or obs or fused or checkpoint" -m gpu > gpurun_out/t_obs.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/t_obs.log; exit 1; }
tail -1 gpurun_out/t_obs.log
bash tools/ab_multi.sh 3 base ""
