set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}; mkdir -p gpurun_out
for v in dpp mreg; do
DX_LIB=variants/$v/libdx.so timeout -k 10 300 python -u tools/stage_profile.py 4096 4 > gpurun_out/st_$v.log 2>&1 || { tail -5 gpurun_out/st_$v.log; exit 1; }
echo "== $v"; grep -E "ms/step|np_mpr|broadphase|midphase|newton_chol|newton_linesearch|constraints" gpurun_out/st_$v.log | head -8 | cut -c1-200
done
