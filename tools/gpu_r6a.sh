#!/bin/bash
# round 6: PGS on AR blocks (MFMA Gram, lane-local rows, w-space coupling) -- parity of the
# solver configurations, the handover task, then configs 3 / 3' / 3'' / 5 against the
# round-5 library and the bench line with the host-API extra
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -v --timeout 400 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py tests/test_gpu_env.py \
  -k "pgs or cg_solver or full_batch_parity or adroit_incremental or handover or fused or goal_change or allgather" \
  > gpurun_out/r6a_t.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR|full batch|PGS|CG " gpurun_out/r6a_t.log | cut -c1-400 | head -50
if [ $rc != 0 ] && [ $rc != 1 ]; then echo "pytest rc=$rc"; tail -5 gpurun_out/r6a_t.log; exit $rc; fi
for lib in - variants/r5/libdx.so; do
  if [ "$lib" = "-" ]; then tag=new; cfgs="3'' 3' 3 5"; unset DX_LIB; else tag=r5; cfgs="3'' 3' 3"; export DX_LIB=$lib; fi
  timeout -k 10 300 python -u tools/bench_configs.py $cfgs > gpurun_out/r6a_cfg_$tag.log 2>&1 || { tail -5 gpurun_out/r6a_cfg_$tag.log; exit 1; }
  echo "== $tag"; cut -c1-300 gpurun_out/r6a_cfg_$tag.log
done
unset DX_LIB
timeout -k 10 200 python -u bench.py --steps 100 --no-cpu-baseline > gpurun_out/r6a_bench.log 2>&1 || { tail -5 gpurun_out/r6a_bench.log; exit 1; }
python3 -c "import json; d=json.loads(open('gpurun_out/r6a_bench.log').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['roofline']['kernel_ms_avg'], d['host_api'])"
