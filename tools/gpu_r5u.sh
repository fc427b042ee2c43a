#!/bin/bash
# round 5 final tree (PGS tail rows, CG recurrence, mid-tier wait): suite, bench line,
# rocprof + HBM passes + stages, every config
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -q --timeout 300 --timeout-method thread tests -m gpu > gpurun_out/t_all.log 2>&1
rc=$?
if [ $rc != 0 ]; then
  echo "suite rc=$rc"; grep -E "^FAILED|Error" gpurun_out/t_all.log | head -20; tail -3 gpurun_out/t_all.log
  [ $rc = 1 ] || exit $rc
fi
tail -1 gpurun_out/t_all.log
timeout -k 10 300 python -u bench.py > gpurun_out/bench_final.log 2>&1 || { tail -5 gpurun_out/bench_final.log; exit 1; }
tail -1 gpurun_out/bench_final.log | cut -c1-300
bash tools/profile_round.sh || exit 1
timeout -k 10 900 python -u tools/bench_configs.py > gpurun_out/configs_final.log 2>&1 || { tail -5 gpurun_out/configs_final.log; exit 1; }
grep -v amdgpu.ids gpurun_out/configs_final.log
