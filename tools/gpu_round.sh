#!/bin/bash
# On the GPU box: targeted tests (-k $K), then the whole -m gpu suite.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
if [ -n "$K" ]; then
  timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests -m gpu -k "$K" > gpurun_out/t_new.log 2>&1 || { echo "targeted tests failed"; exit 1; }
fi
timeout -k 10 900 python -u -m pytest -q --timeout 120 --timeout-method thread tests -m gpu > gpurun_out/t_all.log 2>&1 || { echo "suite failed"; tail -5 gpurun_out/t_all.log; exit 3; }
tail -2 gpurun_out/t_all.log
