#!/bin/bash
# round 5: PGS on AR in two register blocks (up to 128 rows): solver parity tests, the
# PGS / CG configs, the PGS and CG profiles
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread tests -m gpu -k "pgs or cg or solver" -s > gpurun_out/t_pgs.log 2>&1
rc=$?; tail -3 gpurun_out/t_pgs.log; grep -E "PGS|pgs" gpurun_out/t_pgs.log | grep -v PASSED | head -5
[ $rc = 0 ] || [ $rc = 1 ] || exit $rc
timeout -k 10 600 python -u tools/bench_configs.py "3'" "3''" > gpurun_out/configs_r5g.log 2>&1 || { tail -5 gpurun_out/configs_r5g.log; exit 1; }
cat gpurun_out/configs_r5g.log
timeout -k 10 300 python -u tools/cg_profile.py 4096 256 PGS > gpurun_out/pgs_profile.log 2>&1 || { tail -5 gpurun_out/pgs_profile.log; exit 1; }
cat gpurun_out/pgs_profile.log
timeout -k 10 300 python -u tools/cg_profile.py 4096 256 CG > gpurun_out/cg_profile.log 2>&1 || { tail -5 gpurun_out/cg_profile.log; exit 1; }
cat gpurun_out/cg_profile.log
