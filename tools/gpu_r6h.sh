#!/bin/bash
# round 6: the narrowphase trip split (a DX_NP_MARKS build in variants/np) on the headline
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}; mkdir -p gpurun_out
DX_LIB=variants/np/libdx.so timeout -k 10 300 python -u tools/stage_profile.py 4096 4 > gpurun_out/r6h_stages_np.log 2>&1 || { tail -5 gpurun_out/r6h_stages_np.log; exit 1; }
grep -E "ms/step|np_mpr|trip split|mpr_support|np_trips" gpurun_out/r6h_stages_np.log | head -8 | cut -c1-400
