#!/bin/bash
# config 2 (reach_shadow, 1024 envs) with the reach specialization at 1 and 2 waves per SIMD
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}; mkdir -p gpurun_out
for i in 1 2; do
  for lib in variants/base/libdx.so variants/reach1/libdx.so; do
    tag=$(basename "$(dirname "$lib")")
    DX_LIB=$lib timeout -k 10 200 python -u tools/bench_configs.py 2 "2'" > gpurun_out/rab_${tag}_$i.log 2>&1 || { tail -3 gpurun_out/rab_${tag}_$i.log; exit 1; }
    echo "$i $tag"; cut -c1-170 gpurun_out/rab_${tag}_$i.log
  done
done
