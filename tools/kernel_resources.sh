#!/bin/bash
# VGPR / SGPR / scratch / LDS of every kernel in an in-tree object (build/obj/*.o):
#   tools/kernel_resources.sh build/obj/dx_step_DxSpec_shadow_reorient.*.o
set -e
B=/opt/rocm/lib/llvm/bin
T=$(mktemp -d)
for o in "$@"; do
  $B/llvm-objcopy --dump-section=.hip_fatbin="$T/fat.bin" "$o"
  $B/clang-offload-bundler --unbundle --type=o --input="$T/fat.bin" \
    --targets=hipv4-amdgcn-amd-amdhsa--gfx950 --output="$T/k.co"
  echo "== $o"
  $B/llvm-readelf --notes "$T/k.co" | grep -E "^ +\.name:|\.vgpr_count|\.sgpr_count|\.private_segment_fixed_size|\.vgpr_spill_count|\.sgpr_spill_count" \
    | sed 's/^ *//' | paste -sd' ' | sed 's/\.name:/\n.name:/g'
done
rm -rf "$T"
