#!/bin/bash
# cache-keep fix and task parking: invisibility tests, A/B, stage profiles; then the CG
# profile and the other configurations
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_parity.py -k "group_size or tiers or deterministic or queue or full_batch" -m gpu > gpurun_out/t_sep.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/t_sep.log; exit 1; }
tail -2 gpurun_out/t_sep.log
DX_QPARK=1 timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_parity.py -k "tiers or deterministic or queue" -m gpu > gpurun_out/t_park.log 2>&1 || { echo "park tests failed"; tail -30 gpurun_out/t_park.log; exit 1; }
tail -2 gpurun_out/t_park.log
bash tools/ab_multi.sh 3 base "" sepold "DX_LIB=variants/sepold/libdx.so" nola "DX_LIB=variants/nola/libdx.so" park "DX_QPARK=1" || exit 1
timeout -k 10 300 python3 tools/stage_profile.py 4096 10 > gpurun_out/stages_keep.log 2>&1 || exit 1
head -22 gpurun_out/stages_keep.log; grep "queue waits" gpurun_out/stages_keep.log
DX_QPARK=1 timeout -k 10 300 python3 tools/stage_profile.py 4096 10 > gpurun_out/stages_park.log 2>&1 || exit 1
grep "queue waits\|ms/step" gpurun_out/stages_park.log
timeout -k 10 500 python -u tools/cg_profile.py 4096 512 > gpurun_out/cg_run.log 2>&1 || exit 1
tail -5 gpurun_out/cg_run.log
timeout -k 10 300 python tools/bench_configs.py > gpurun_out/configs.log 2>&1; tail -12 gpurun_out/configs.log
