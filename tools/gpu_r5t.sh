#!/bin/bash
# round 5: CG with M dir by recurrence -- CG parity tests, config 3', CG stage profile
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v -s --timeout 400 --timeout-method thread tests/test_gpu_parity.py -m gpu -k "cg or CG" > gpurun_out/t_cg.log 2>&1 || { echo "cg tests rc=$?"; grep -E "FAILED|Error|assert|CG" gpurun_out/t_cg.log | head -30; tail -3 gpurun_out/t_cg.log; exit 1; }
grep -E "CG|passed" gpurun_out/t_cg.log | head -20
timeout -k 10 300 python -u tools/bench_configs.py "3'" > gpurun_out/configs_cg.log 2>&1 || { tail -5 gpurun_out/configs_cg.log; exit 1; }
grep -v amdgpu.ids gpurun_out/configs_cg.log
timeout -k 10 300 python3 tools/stage_profile.py 4096 8 reorient CG > gpurun_out/stages_cg2.log 2>&1 || { tail -5 gpurun_out/stages_cg2.log; exit 1; }
grep -v amdgpu.ids gpurun_out/stages_cg2.log | head -34
