#!/bin/bash
# round 5: parity, A/B against the round-start tree, the bench line, rocprof + PMC profile
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
timeout -k 10 300 python -u bench.py > gpurun_out/bench_r5e.log 2>&1 || { tail -5 gpurun_out/bench_r5e.log; exit 1; }
tail -1 gpurun_out/bench_r5e.log | cut -c1-600
bash tools/profile_round.sh || exit 1
