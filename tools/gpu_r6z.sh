#!/bin/bash
# round 6 close: full gpu suite on the HEAD library, smoke, the bench line, rocprof + PMC profile
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}; mkdir -p gpurun_out
T=${TAG:-r6z}
timeout -k 10 900 python -u -m pytest -v --timeout 300 --timeout-method thread tests -m gpu > gpurun_out/t_$T.log 2>&1
rc=$?
if [ $rc != 0 ]; then
  echo "suite rc=$rc"; grep -E "^FAILED|Error" gpurun_out/t_$T.log | head -20; tail -3 gpurun_out/t_$T.log
  [ $rc = 1 ] || exit $rc
fi
tail -1 gpurun_out/t_$T.log
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke_$T.log 2>&1 || { tail -5 gpurun_out/smoke_$T.log; exit 1; }
tail -1 gpurun_out/smoke_$T.log
timeout -k 10 300 python -u bench.py > gpurun_out/bench_$T.log 2>&1 || { tail -5 gpurun_out/bench_$T.log; exit 1; }
tail -1 gpurun_out/bench_$T.log | cut -c1-900
bash tools/profile_round.sh || exit 1
grep -E "ms/step|np_mpr" gpurun_out/prof/stages.log | head -3
