#!/bin/bash
# round 5 close: full gpu suite on the rebuilt HEAD library, the bench line, rocprof + PMC profile
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -v --timeout 300 --timeout-method thread tests -m gpu > gpurun_out/t_z.log 2>&1
rc=$?
if [ $rc != 0 ]; then
  echo "suite rc=$rc"; grep -E "^FAILED|Error" gpurun_out/t_z.log | head -20; tail -3 gpurun_out/t_z.log
  [ $rc = 1 ] || exit $rc
fi
tail -1 gpurun_out/t_z.log
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke_z.log 2>&1 || { tail -5 gpurun_out/smoke_z.log; exit 1; }
tail -1 gpurun_out/smoke_z.log
timeout -k 10 300 python -u bench.py > gpurun_out/bench_r5f.log 2>&1 || { tail -5 gpurun_out/bench_r5f.log; exit 1; }
tail -1 gpurun_out/bench_r5f.log | cut -c1-700
bash tools/profile_round.sh || exit 1
