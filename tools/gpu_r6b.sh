#!/bin/bash
# round 6: CG full batch on the per-solver accounting, the PGS launch's per-env costs and
# stages, and config 3'' against the round-5 library on the same box
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -v --timeout 400 --timeout-method thread -m gpu tests/test_gpu_parity.py \
  -k "full_batch_parity" > gpurun_out/r6b_t.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR" gpurun_out/r6b_t.log | head; grep -E "full batch" gpurun_out/r6b_t.log | sed 's/deep mesh-mesh.*unexplained/ ... unexplained/' | cut -c1-600
if [ $rc != 0 ] && [ $rc != 1 ]; then echo "pytest rc=$rc"; exit $rc; fi
timeout -k 10 300 python -u tools/cost_probe.py 4096 40 reorient PGS > gpurun_out/r6b_cost_pgs.log 2>&1 || { tail -5 gpurun_out/r6b_cost_pgs.log; exit 1; }
cat gpurun_out/r6b_cost_pgs.log | cut -c1-400
timeout -k 10 300 python -u tools/stage_profile.py 4096 4 reorient PGS > gpurun_out/r6b_stages_pgs.log 2>&1 || { tail -5 gpurun_out/r6b_stages_pgs.log; exit 1; }
head -30 gpurun_out/r6b_stages_pgs.log | cut -c1-300
for lib in variants/r5/libdx.so -; do
  if [ "$lib" = "-" ]; then tag=new; unset DX_LIB; else tag=r5; export DX_LIB=$lib; fi
  timeout -k 10 300 python -u tools/bench_configs.py "3''" > gpurun_out/r6b_cfg_$tag.log 2>&1 || { tail -5 gpurun_out/r6b_cfg_$tag.log; exit 1; }
  echo "== $tag"; cut -c1-200 gpurun_out/r6b_cfg_$tag.log
done
