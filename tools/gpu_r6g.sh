#!/bin/bash
# round 6: CG with J's rows in registers -- CG parity (defaults, converged, full batch on
# its own trajectory), config 3', and the CG launch's stages
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -v -s --timeout 400 --timeout-method thread -m gpu tests/test_gpu_parity.py \
  -k "cg_solver or full_batch_parity" > gpurun_out/r6g_t.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR" gpurun_out/r6g_t.log | head; grep -E "full batch|CG defaults" gpurun_out/r6g_t.log | sed 's/deep mesh-mesh.*unexplained/ ... unexplained/' | cut -c1-400
if [ $rc != 0 ] && [ $rc != 1 ]; then echo "pytest rc=$rc"; exit $rc; fi
timeout -k 10 300 python -u tools/bench_configs.py "3'" "3''" > gpurun_out/r6g_cfg.log 2>&1 || { tail -5 gpurun_out/r6g_cfg.log; exit 1; }
cut -c1-220 gpurun_out/r6g_cfg.log
timeout -k 10 300 python -u tools/cost_probe.py 4096 40 reorient CG > gpurun_out/r6g_cost_CG.log 2>&1 || { tail -5 gpurun_out/r6g_cost_CG.log; exit 1; }
head -8 gpurun_out/r6g_cost_CG.log | cut -c1-300
timeout -k 10 300 python -u tools/stage_profile.py 4096 4 reorient CG > gpurun_out/r6g_stages_CG.log 2>&1 || { tail -5 gpurun_out/r6g_stages_CG.log; exit 1; }
grep -E "ms/step|newton|np_mpr|jacvec|top1" gpurun_out/r6g_stages_CG.log | head -16 | cut -c1-200
