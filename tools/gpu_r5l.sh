#!/bin/bash
# round 5: J^T f over (contact, slot) items with LDS atomics: parity, A/B vs HEAD, solver configs
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -q --timeout 300 --timeout-method thread tests -m gpu -s > gpurun_out/t_all.log 2>&1
rc=$?
if [ $rc != 0 ]; then
  echo "suite rc=$rc"; grep -E "^FAILED|Error" gpurun_out/t_all.log | head -20; tail -3 gpurun_out/t_all.log
  [ $rc = 1 ] || exit $rc
fi
tail -1 gpurun_out/t_all.log
grep -E "full batch" gpurun_out/t_all.log | cut -c1-300
bash tools/ab_multi.sh 3 new "" head "DX_LIB=variants/head/libdx.so" || exit 1
timeout -k 10 600 python -u tools/bench_configs.py "3'" "3''" 5 > gpurun_out/configs_r5l.log 2>&1 || { tail -5 gpurun_out/configs_r5l.log; exit 1; }
cat gpurun_out/configs_r5l.log
for v in "" "DX_LIB=variants/head/libdx.so"; do env $v timeout -k 10 300 python -u tools/bench_configs.py "3'" | tail -1; done
