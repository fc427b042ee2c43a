#!/bin/bash
# Occupancy probe: the reorient bench with DX_LDS_PAD bytes of extra LDS per workgroup
# (fewer resident workgroups per CU); the pads are the arguments (default 0 1000 4000).
set -e
mkdir -p gpurun_out
for pad in ${@:-0 1000 4000}; do
  DX_LDS_PAD=$pad timeout -k 10 120 python -u bench.py --no-cpu-baseline --host-api-steps 0 --steps 300 > gpurun_out/occ_$pad.log 2>&1
done
