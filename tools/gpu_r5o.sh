#!/bin/bash
# round 5: resting-contact KAT + contact-pool tests (mid tier's progress-based wait), then
# the full suite, then the solver configs with the deferral counters
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_kat.py tests/test_gpu_contact_pool.py -m gpu > gpurun_out/t_new.log 2>&1 || { echo "targeted rc=$?"; grep -E "FAILED|Error|assert" gpurun_out/t_new.log | head -20; tail -3 gpurun_out/t_new.log; exit 1; }
tail -1 gpurun_out/t_new.log
timeout -k 10 900 python -u -m pytest -q --timeout 300 --timeout-method thread tests -m gpu > gpurun_out/t_all.log 2>&1 || { echo "suite rc=$?"; grep -E "^FAILED" gpurun_out/t_all.log | head; tail -3 gpurun_out/t_all.log; exit 1; }
tail -1 gpurun_out/t_all.log
timeout -k 10 600 python -u tools/bench_configs.py 3 "3'" "3''" > gpurun_out/configs_r5o.log 2>&1 || { tail -5 gpurun_out/configs_r5o.log; exit 1; }
cat gpurun_out/configs_r5o.log
