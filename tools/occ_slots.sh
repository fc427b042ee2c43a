set -e
mkdir -p gpurun_out
for pad in 0 -512 -256 -128 -64 -1; do DX_LDS_PAD=$pad timeout -k 10 60 python tools/occ_slots.py; done > gpurun_out/occ_slots.log 2>&1
