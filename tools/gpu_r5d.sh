#!/bin/bash
# round 5: parity (fp64 MPR portal direction), A/B against the round-start tree, reach config
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -v --timeout 300 --timeout-method thread tests -m gpu -s > gpurun_out/t_all.log 2>&1
rc=$?
if [ $rc != 0 ]; then
  echo "suite rc=$rc"; grep -E "^FAILED|Error" gpurun_out/t_all.log | head -20; tail -3 gpurun_out/t_all.log
  [ $rc = 1 ] || exit $rc
fi
tail -1 gpurun_out/t_all.log
grep -E "full batch" gpurun_out/t_all.log | cut -c1-420
bash tools/ab_multi.sh 3 new "" prev "DX_LIB=variants/prev/libdx.so" || exit 1
timeout -k 10 300 python -u tools/bench_configs.py 2 "2'" > gpurun_out/configs_r5d.log 2>&1 || { tail -5 gpurun_out/configs_r5d.log; exit 1; }
cat gpurun_out/configs_r5d.log
