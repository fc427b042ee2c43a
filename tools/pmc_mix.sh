#!/bin/bash
# On the GPU box: per-stage cycle profile + instruction-mix / stall PMC passes of
# dx_step_kernel (one rocprofv3 pass per counter group, kernel trace only).
# Output under gpurun_out/mix.  Stops at the first timeout / abort / segfault.
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/mix
rm -rf "$O"; mkdir -p "$O"
cd "$R"
timeout -k 10 300 python3 tools/stage_profile.py 4096 10 > "$O/stages.log" 2>&1
rc=$?; cp gpurun_out/stages.json "$O/stages.json" 2>/dev/null
[ $rc -ne 0 ] && { echo "stage profile rc=$rc"; exit $rc; }
cd /tmp && export TMPDIR=/tmp
i=0
for grp in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES" "SQ_WAIT_ANY SQ_WAIT_INST_ANY" "SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU" \
           "SQ_INSTS_VALU SQ_INSTS_SALU" "SQ_INSTS_LDS SQ_INSTS_SMEM" "SQ_INSTS_VMEM_RD SQ_WAIT_INST_LDS" \
           "SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA" "SQ_LDS_BANK_CONFLICT SQ_INSTS_BRANCH" "SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_VMEM"; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --pmc $grp --kernel-trace -d "$O/p$i" -o pmc --output-format csv -- \
    python3 "$R/bench.py" --steps 6 --warmup 2 --no-cpu-baseline --host-api-steps 0 > "$O/p$i.log" 2>&1
  rc=$?
  echo "pass $i ($grp) rc=$rc"
  case $rc in 124|137|134|139) exit $rc;; esac
done
exit 0
