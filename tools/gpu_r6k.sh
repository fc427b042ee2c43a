#!/bin/bash
# round 6: the whole GPU suite on the in-tree build, then every configuration's line
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}; mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest -x -q --timeout 400 --timeout-method thread -m gpu tests > gpurun_out/r6k_t.log 2>&1
rc=$?
tail -3 gpurun_out/r6k_t.log
if [ $rc != 0 ]; then grep -E "FAILED|Error" gpurun_out/r6k_t.log | head; exit $rc; fi
timeout -k 10 400 python -u tools/bench_configs.py > gpurun_out/r6k_cfg.log 2>&1 || { tail -5 gpurun_out/r6k_cfg.log; exit 1; }
cut -c1-200 gpurun_out/r6k_cfg.log
