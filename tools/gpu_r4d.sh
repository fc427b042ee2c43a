#!/bin/bash
# mid tier: contact-pool / health tests, the tier probe, then A/B against DX_NO_MID=1
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_contact_pool.py tests/test_gpu_health.py -m gpu > gpurun_out/t_mid.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/t_mid.log; exit 1; }
tail -2 gpurun_out/t_mid.log
timeout -k 10 300 python -u tools/hi_probe.py > gpurun_out/hi_probe.log 2>&1 || { echo "probe failed"; tail -20 gpurun_out/hi_probe.log; exit 1; }
cat gpurun_out/hi_probe.log
bash tools/ab_multi.sh 3 mid "" nomid "DX_NO_MID=1"
