#!/bin/bash
# round 5: same-box A/B of M's rows in registers (new) against HEAD
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}; mkdir -p gpurun_out
bash tools/ab_multi.sh 3 new "" head "DX_LIB=variants/head/libdx.so" || exit 1
