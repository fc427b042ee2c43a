#!/bin/bash
# round 6: full-batch parity of CG / PGS on their own trajectories (fp32-portal rule), the
# GPU suite's parity / env / pool files, the configs, the headline A/B against round 5
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -v --timeout 400 --timeout-method thread -m gpu tests/test_gpu_parity.py \
  tests/test_gpu_contact_pool.py tests/test_gpu_env.py > gpurun_out/r6e_t.log 2>&1
rc=$?
grep -E "FAILED|ERROR" gpurun_out/r6e_t.log | head -12; tail -1 gpurun_out/r6e_t.log
grep -E "full batch" gpurun_out/r6e_t.log | sed 's/deep mesh-mesh.*unexplained/ ... unexplained/' | cut -c1-400
if [ $rc != 0 ] && [ $rc != 1 ]; then echo "pytest rc=$rc"; exit $rc; fi
timeout -k 10 300 python -u tools/bench_configs.py "3''" "3'" 3 5 > gpurun_out/r6e_cfg.log 2>&1 || { tail -5 gpurun_out/r6e_cfg.log; exit 1; }
cut -c1-300 gpurun_out/r6e_cfg.log
timeout -k 10 600 bash tools/ab_lib.sh variants/r5/libdx.so || exit 1
for f in gpurun_out/ab_*_[12].log; do echo "$f $(tail -1 $f | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["roofline"]["kernel_ms_avg"])')"; done
