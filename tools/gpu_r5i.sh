#!/bin/bash
# round 5: XCD-local queue with last-round stealing: parity, A/B, HBM passes
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -q --timeout 300 --timeout-method thread tests -m gpu > gpurun_out/t_all.log 2>&1
rc=$?
if [ $rc != 0 ]; then
  echo "suite rc=$rc"; grep -E "^FAILED|Error" gpurun_out/t_all.log | head -20; tail -3 gpurun_out/t_all.log
  [ $rc = 1 ] || exit $rc
fi
tail -1 gpurun_out/t_all.log
bash tools/ab_multi.sh 3 new "" xcdl "DX_XCD_LOCAL=1" prev "DX_LIB=variants/prev/libdx.so" || exit 1
bash tools/pmc_cfgs.sh pmc_r5i default "" xcdl "DX_XCD_LOCAL=1" || exit 1
