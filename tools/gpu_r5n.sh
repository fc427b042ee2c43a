#!/bin/bash
# round 5 final tree after the J^T f change: suite, bench line, rocprof + HBM passes +
# stages, every config, the reach stage profile and a reach rocprof (one launch per step)
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
cat gpurun_out/configs_final.log
timeout -k 10 300 python3 tools/stage_profile.py 1024 20 reach_shadow > gpurun_out/stages_reach.log 2>&1 || { tail -5 gpurun_out/stages_reach.log; exit 1; }
head -24 gpurun_out/stages_reach.log
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_reach -o reach --output-format csv -- python3 $R/tools/bench_configs.py 2 > $R/gpurun_out/prof_reach.log 2>&1 || exit 1
