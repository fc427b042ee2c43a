#!/bin/bash
# deferral claim protocol: pool / tier / health tests (serialised kernels included), then
# one FETCH_SIZE pass under rocprofv3 (the run that deadlocked before)
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 250 --timeout-method thread tests/test_gpu_contact_pool.py tests/test_gpu_health.py tests/test_gpu_parity.py -k "pool or health or tiers or serialised or queue or deterministic" -m gpu > gpurun_out/t_claim.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/t_claim.log; exit 1; }
tail -2 gpurun_out/t_claim.log
R=$(pwd); cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $R/gpurun_out/claimpmc -o pmc --output-format csv -- python3 $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline --host-api-steps 0 > $R/gpurun_out/claimpmc.log 2>&1; echo "pmc rc $?"; tail -1 $R/gpurun_out/claimpmc.log | cut -c1-200
