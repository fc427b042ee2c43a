#!/bin/bash
# round-4 diagnostics: full-batch parity outliers, kernel trace of the fused step, A/B fused
# vs task kernels, CG profile
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
timeout -k 10 300 python -u tools/full_batch_diag.py > gpurun_out/diag.log 2>&1 || { echo diag failed; exit 1; }
for i in 1 2; do
  timeout -k 10 120 python -u bench.py --no-cpu-baseline --host-api-steps 0 --steps 200 > gpurun_out/bench_fused_$i.log 2>&1 || exit 2
  DX_NO_FUSE=1 timeout -k 10 120 python -u bench.py --no-cpu-baseline --host-api-steps 0 --steps 200 > gpurun_out/bench_nofuse_$i.log 2>&1 || exit 3
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof4a" -o run --output-format csv -- \
  python3 "$R/bench.py" --steps 40 --warmup 5 --no-cpu-baseline --host-api-steps 0 > "$R/gpurun_out/prof4a.log" 2>&1 || exit 4
cd "$R"
timeout -k 10 400 python -u tools/cg_profile.py 4096 512 > gpurun_out/cg_profile.log 2>&1 || exit 5
echo done
