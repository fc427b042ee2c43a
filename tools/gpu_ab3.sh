set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
AB_TEST=1 bash tools/gpu_ab.sh variants/base/libdx.so variants/rf/libdx.so variants/bc/libdx.so || exit 1
DX_LIB=variants/base/libdx.so timeout -k 10 300 python -u tools/bench_configs.py "3'" "3''" > gpurun_out/cfg_base.log 2>&1 || exit 1
DX_LIB=variants/bc/libdx.so timeout -k 10 300 python -u tools/bench_configs.py "3'" "3''" > gpurun_out/cfg_bc.log 2>&1 || exit 1
for f in gpurun_out/cfg_base.log gpurun_out/cfg_bc.log; do echo $f; cut -c1-170 $f; done
