#!/bin/bash
# the GPU suite (full-batch parity first)
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v -s --timeout 250 --timeout-method thread tests -m gpu -k "full_batch or cg_solver" > gpurun_out/t_new.log 2>&1 || { echo "targeted failed"; exit 1; }
timeout -k 10 900 python -u -m pytest -q --timeout 200 --timeout-method thread tests -m gpu > gpurun_out/t_all.log 2>&1; rc=$?; echo "suite rc $rc"; tail -3 gpurun_out/t_all.log; exit $rc
