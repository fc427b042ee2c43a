set -e
mkdir -p gpurun_out
for i in 1 2 3; do
  timeout -k 10 120 python -u bench.py --no-cpu-baseline --host-api-steps 0 --steps 300 > gpurun_out/ab_tree_$i.log 2>&1
  DX_DENSE_MSOLVE=1 timeout -k 10 120 python -u bench.py --no-cpu-baseline --host-api-steps 0 --steps 300 > gpurun_out/ab_dense_$i.log 2>&1
done
timeout -k 10 200 python3 tools/bench_configs.py > gpurun_out/cfg_tree.log 2>&1
DX_DENSE_MSOLVE=1 timeout -k 10 200 python3 tools/bench_configs.py > gpurun_out/cfg_dense.log 2>&1
