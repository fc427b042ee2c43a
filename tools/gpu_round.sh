set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_health.py tests/test_gpu_env.py -k "health or shard or nan or overflow" > gpurun_out/t_new.log 2>&1 || { echo "new tests failed"; exit 1; }
timeout -k 10 200 python -u tools/ncon_histogram.py 4096 500 > gpurun_out/ncon.log 2>&1 || exit 2
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu > gpurun_out/t_all.log 2>&1 || { echo "suite failed"; exit 3; }
bash tools/pmc_mix.sh > gpurun_out/mix_run.log 2>&1
