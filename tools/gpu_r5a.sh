#!/bin/bash
# round 5, first call: the whole -m gpu suite (new: order key > 16 bits, launch-tagged
# deferrals, checkpoint agent seed, bimanual full batch, pinned full-batch categories),
# then a same-box A/B: this tree (Newton-only specialization), HEAD~ (prev), and the
# XCD-local queue (DX_XCD_LOCAL=1: no stealing, plain hand-off records)
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -v --timeout 300 --timeout-method thread tests -m gpu -s > gpurun_out/t_all.log 2>&1 \
  || { echo "suite failed"; grep -E "FAILED|Error|assert" gpurun_out/t_all.log | head -20; tail -5 gpurun_out/t_all.log; exit 3; }
tail -2 gpurun_out/t_all.log
grep -E "full batch" gpurun_out/t_all.log
bash tools/ab_multi.sh 3 new "" prev "DX_LIB=variants/prev/libdx.so" xcdl "DX_XCD_LOCAL=1" || exit 1
