#!/bin/bash
# CG changes: CG parity (defaults, converged, full batch), then config 3' same-box against variants/base
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}; mkdir -p gpurun_out
DX_LIB=${NEW:-variants/cgb/libdx.so} timeout -k 10 600 python -u -m pytest -v -s --timeout 400 --timeout-method thread -m gpu tests/test_gpu_parity.py \
  -k "cg_solver or full_batch_parity" > gpurun_out/cgab_t.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR" gpurun_out/cgab_t.log | cut -c1-150 | head; grep -E "CG defaults|reorient_cg full batch" gpurun_out/cgab_t.log | cut -c1-300
if [ $rc != 0 ] && [ $rc != 1 ]; then echo "pytest rc=$rc"; exit $rc; fi
for i in 1 2; do
  for lib in variants/base/libdx.so ${NEW:-variants/cgb/libdx.so}; do
    DX_LIB=$lib timeout -k 10 300 python -u tools/bench_configs.py "3'" > gpurun_out/cgab_$i.log 2>&1 || { tail -3 gpurun_out/cgab_$i.log; exit 1; }
    echo "$i $lib $(grep -o '"env_steps_per_s": [0-9.]*' gpurun_out/cgab_$i.log) $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/cgab_$i.log)"
  done
done
