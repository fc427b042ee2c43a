#!/bin/bash
# Samples the GPU's clocks and power (read-only rocm-smi queries) while the bench runs,
# to see what shader clock the step kernel actually runs at.
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
timeout -k 5 100 bash -c 'while true; do date +%s.%N; rocm-smi --showclocks --showpower 2>/dev/null | grep -E "sclk|Power|fclk|mclk"; sleep 0.3; done' > gpurun_out/clock.log 2>&1 &
P=$!
sleep 2
timeout -k 10 90 python -u bench.py --steps 2000 --warmup 20 --no-cpu-baseline --host-api-steps 0 > gpurun_out/clock_bench.log 2>&1
kill $P 2>/dev/null
wait $P 2>/dev/null
exit 0
