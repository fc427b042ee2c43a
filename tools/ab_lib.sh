#!/bin/bash
# Same-box A/B of libdx.so builds: every library given as an argument (and the default
# in-tree one, "-") runs the reorient bench, round robin, twice.
set -e
mkdir -p gpurun_out
for i in 1 2; do
  for lib in - "$@"; do
    tag=$(basename "$lib" .so); [ "$tag" = libdx ] && tag=$(basename "$(dirname "$lib")")
    if [ "$lib" = "-" ]; then tag=default; unset DX_LIB; else export DX_LIB=$lib; fi
    timeout -k 10 120 python -u bench.py --no-cpu-baseline --host-api-steps 0 --steps 300 > gpurun_out/ab_${tag}_$i.log 2>&1
  done
done
