#!/bin/bash
# round 6: PGS rows on the two-op chain -- solver parity (full batch, defaults, tail), the
# configs, the bench line with the host-API extra, and the PGS launch's costs and stages
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -v --timeout 400 --timeout-method thread -m gpu tests/test_gpu_parity.py \
  -k "full_batch_parity or pgs or cg_solver" > gpurun_out/r6c_t.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR" gpurun_out/r6c_t.log | head -12; grep -E "full batch|PGS" gpurun_out/r6c_t.log | sed 's/deep mesh-mesh.*unexplained/ ... unexplained/' | cut -c1-500
if [ $rc != 0 ] && [ $rc != 1 ]; then echo "pytest rc=$rc"; exit $rc; fi
timeout -k 10 300 python -u tools/bench_configs.py "3''" "3'" 3 5 > gpurun_out/r6c_cfg.log 2>&1 || { tail -5 gpurun_out/r6c_cfg.log; exit 1; }
cut -c1-200 gpurun_out/r6c_cfg.log
timeout -k 10 200 python -u bench.py --steps 100 --no-cpu-baseline > gpurun_out/r6c_bench.log 2>&1 || { tail -5 gpurun_out/r6c_bench.log; exit 1; }
python3 -c "import json; d=json.loads(open('gpurun_out/r6c_bench.log').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['roofline']['kernel_ms_avg'], d['host_api'])"
timeout -k 10 300 python -u tools/cost_probe.py 4096 40 reorient PGS > gpurun_out/r6c_cost_pgs.log 2>&1 || { tail -5 gpurun_out/r6c_cost_pgs.log; exit 1; }
head -8 gpurun_out/r6c_cost_pgs.log | cut -c1-400
timeout -k 10 300 python -u tools/stage_profile.py 4096 4 reorient PGS > gpurun_out/r6c_stages_pgs.log 2>&1 || { tail -5 gpurun_out/r6c_stages_pgs.log; exit 1; }
grep -E "ms/step|linesearch|hessian|grad|np_mpr|top1" gpurun_out/r6c_stages_pgs.log | head -14 | cut -c1-200
