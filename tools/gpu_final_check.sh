#!/bin/bash
# final check of the in-tree library: GPU suite, smoke, the bench line (traffic from the
# committed PMC record of this build)
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -q --timeout 300 --timeout-method thread tests -m gpu > gpurun_out/final_t.log 2>&1 || { tail -5 gpurun_out/final_t.log; exit 1; }
tail -1 gpurun_out/final_t.log
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/final_smoke.log 2>&1 || { tail -5 gpurun_out/final_smoke.log; exit 1; }
tail -1 gpurun_out/final_smoke.log
timeout -k 10 300 python -u bench.py > gpurun_out/final_bench.log 2>&1 || { tail -5 gpurun_out/final_bench.log; exit 1; }
tail -1 gpurun_out/final_bench.log | cut -c1-400; grep -o '"roofline": {[^}]*}' gpurun_out/final_bench.log | cut -c1-200
