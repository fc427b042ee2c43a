#!/bin/bash
# out-of-line task logic: fused-vs-kernels identity, A/B against the inlined build
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 250 --timeout-method thread tests/test_gpu_env.py tests/test_gpu_parity.py -k "fused or checkpoint or tiers or queue or deterministic" -m gpu > gpurun_out/t_noinl.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/t_noinl.log; exit 1; }
tail -2 gpurun_out/t_noinl.log
bash tools/ab_multi.sh 3 noinl "" inl "DX_LIB=variants/inl/libdx.so"
