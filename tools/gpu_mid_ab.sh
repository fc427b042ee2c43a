#!/bin/bash
# the mid tier at one wave per SIMD (no VGPR spill) against HEAD: tier tests, headline,
# PGS and CG lines, same box, twice
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}; mkdir -p gpurun_out
NEW=variants/mid1/libdx.so
DX_LIB=$NEW timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py \
  -k "tiers or deferrals or queue or full_batch_parity or pgs" > gpurun_out/mid_t.log 2>&1
rc=$?; tail -1 gpurun_out/mid_t.log
if [ $rc != 0 ]; then grep -E "FAILED|Error" gpurun_out/mid_t.log | head; exit $rc; fi
for i in 1 2; do
  for lib in dexterity_amd/libdx.so $NEW; do
    DX_LIB=$lib timeout -k 10 400 python -u tools/bench_configs.py 3 "3'" "3''" > gpurun_out/mid_$i.log 2>&1 || { tail -3 gpurun_out/mid_$i.log; exit 1; }
    echo "$i $lib $(grep -o '"env_steps_per_s": [0-9.]*' gpurun_out/mid_$i.log | tr '\n' ' ')"
  done
done
