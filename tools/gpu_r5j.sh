#!/bin/bash
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -q --timeout 300 --timeout-method thread tests -m gpu > gpurun_out/t_all.log 2>&1
rc=$?
if [ $rc != 0 ]; then
  echo "suite rc=$rc"; grep -E "^FAILED|Error" gpurun_out/t_all.log | head -20; tail -3 gpurun_out/t_all.log
  [ $rc = 1 ] || exit $rc
fi
tail -1 gpurun_out/t_all.log
bash tools/ab_multi.sh 2 new "" prev "DX_LIB=variants/prev/libdx.so" || exit 1
timeout -k 10 300 python -u tools/cg_profile.py 4096 32 PGS > gpurun_out/pgs_profile.log 2>&1 || { tail -5 gpurun_out/pgs_profile.log; exit 1; }
head -3 gpurun_out/pgs_profile.log | cut -c1-600
