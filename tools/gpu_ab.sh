#!/bin/bash
# Same-box A/B of prebuilt libraries (each argument a libdx.so), headline bench, round
# robin, twice; optionally first the MPR-heavy parity tests on the last one (AB_TEST=1).
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}; mkdir -p gpurun_out
last="${@: -1}"
if [ "${AB_TEST:-0}" = 1 ]; then
  DX_LIB=$last timeout -k 10 700 python -u -m pytest -v -s --timeout 400 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_kat.py \
    -k "forward or substep or full_batch or group_size or tiers or contact or watch or replay or stale" > gpurun_out/ab_t.log 2>&1
  rc=$?
  grep -E "PASSED|FAILED|ERROR" gpurun_out/ab_t.log | cut -c1-160 | grep -v PASSED | head -20; grep -c PASSED gpurun_out/ab_t.log
  grep -E "full batch" gpurun_out/ab_t.log | sed 's/deep mesh-mesh.*unexplained/ ... unexplained/' | cut -c1-330
  if [ $rc != 0 ] && [ $rc != 1 ]; then echo "pytest rc=$rc"; exit $rc; fi
fi
for i in 1 2; do
  for lib in "$@"; do
    tag=$(basename "$(dirname "$lib")")
    DX_LIB=$lib timeout -k 10 120 python -u bench.py --no-cpu-baseline --host-api-steps 0 --steps 300 > gpurun_out/ab_${tag}_$i.log 2>&1 || { tail -3 gpurun_out/ab_${tag}_$i.log; exit 1; }
    echo "$i $tag $(grep -o '"value": [0-9.]*' gpurun_out/ab_${tag}_$i.log) $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ab_${tag}_$i.log)"
  done
done
