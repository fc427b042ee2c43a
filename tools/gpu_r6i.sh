#!/bin/bash
# round 6: 8-slot hull cells -- the MPR-heavy parity tests, the headline same-box against
# the previous build (variants/base), the trip split
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}; mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest -v -s --timeout 400 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_kat.py \
  -k "forward or substep or full_batch or group_size or tiers or contact or watch" > gpurun_out/r6i_t.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR" gpurun_out/r6i_t.log | cut -c1-160 | head -40; grep -E "full batch" gpurun_out/r6i_t.log | sed 's/deep mesh-mesh.*unexplained/ ... unexplained/' | cut -c1-330
if [ $rc != 0 ] && [ $rc != 1 ]; then echo "pytest rc=$rc"; exit $rc; fi
bash tools/ab_lib.sh variants/base/libdx.so || exit 1
for f in gpurun_out/ab_*.log; do echo "$f $(grep -o '"value": [0-9.]*' $f) $(grep -o '"ms_per_step": [0-9.]*' $f)"; done
timeout -k 10 300 python -u tools/stage_profile.py 4096 4 > gpurun_out/r6i_stages.log 2>&1 || { tail -5 gpurun_out/r6i_stages.log; exit 1; }
grep -E "ms/step|np_mpr|newton_chol" gpurun_out/r6i_stages.log | head -4 | cut -c1-300
