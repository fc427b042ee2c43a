#!/bin/bash
# round 5: PGS tail rows (past 128) -- parity tests, then the PGS cost distribution and config 3''
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v -s --timeout 400 --timeout-method thread tests/test_gpu_parity.py -m gpu -k "pgs" > gpurun_out/t_pgs.log 2>&1 || { echo "pgs tests rc=$?"; grep -E "FAILED|Error|assert|PGS" gpurun_out/t_pgs.log | head -30; tail -3 gpurun_out/t_pgs.log; exit 1; }
grep -E "PGS|tail|passed" gpurun_out/t_pgs.log
timeout -k 10 300 python3 tools/cost_probe.py 4096 40 reorient PGS > gpurun_out/cost_PGS2.log 2>&1 || { tail -5 gpurun_out/cost_PGS2.log; exit 1; }
grep -v amdgpu.ids gpurun_out/cost_PGS2.log
timeout -k 10 300 python -u tools/bench_configs.py "3''" > gpurun_out/configs_pgs.log 2>&1 || { tail -5 gpurun_out/configs_pgs.log; exit 1; }
grep -v amdgpu.ids gpurun_out/configs_pgs.log
