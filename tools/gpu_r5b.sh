#!/bin/bash
# round 5: the -m gpu suite (fused reach, bimanual full batch), same-box A/B of this tree,
# HEAD at round start (prev) and the XCD-local queue, then the HBM passes of the two queues
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -v --timeout 300 --timeout-method thread tests -m gpu -s > gpurun_out/t_all.log 2>&1
rc=$?
if [ $rc != 0 ]; then
  echo "suite rc=$rc"; grep -E "^FAILED|Error" gpurun_out/t_all.log | head -20; tail -3 gpurun_out/t_all.log
  [ $rc = 1 ] || exit $rc  # test failures only: go on; a crash, abort or time limit: stop here
fi
tail -1 gpurun_out/t_all.log
grep -E "full batch" gpurun_out/t_all.log | cut -c1-400
bash tools/ab_multi.sh 3 new "" prev "DX_LIB=variants/prev/libdx.so" xcdl "DX_XCD_LOCAL=1" || exit 1
bash tools/pmc_cfgs.sh pmc_r5b default "" xcdl "DX_XCD_LOCAL=1" || exit 1
timeout -k 10 600 python -u tools/bench_configs.py 2 "2'" "3'" "3''" 5 > gpurun_out/configs_r5b.log 2>&1 || { echo "configs failed"; tail -5 gpurun_out/configs_r5b.log; exit 1; }
cat gpurun_out/configs_r5b.log
cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_reach -o reach --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/bench_configs.py 2 > $GRAFT_REPO_ROOT/gpurun_out/prof_reach.log 2>&1 || exit 1
