#!/bin/bash
# round 5: parity tests (fp64 MPR exit), A/B against the round-start tree, PGS / CG and
# reach stage profiles
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
bash tools/ab_multi.sh 3 new "" prev "DX_LIB=variants/prev/libdx.so" xcdl "DX_XCD_LOCAL=1" || exit 1
bash tools/pmc_cfgs.sh pmc_r5c default "" xcdl "DX_XCD_LOCAL=1" || exit 1
timeout -k 10 300 python -u tools/cg_profile.py 4096 256 PGS > gpurun_out/pgs_profile.log 2>&1 || { tail -5 gpurun_out/pgs_profile.log; exit 1; }
cat gpurun_out/pgs_profile.log
timeout -k 10 300 python -u tools/stage_profile.py 1024 20 reach_shadow > gpurun_out/stages_reach.log 2>&1 || { tail -5 gpurun_out/stages_reach.log; exit 1; }
head -24 gpurun_out/stages_reach.log
