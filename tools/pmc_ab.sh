#!/bin/bash
# On the GPU box: FETCH_SIZE and WRITE_SIZE passes of a short bench run under each
# queue configuration (per-XCD queues, one queue, no queue), for the HBM-traffic
# breakdown in DESIGN.md.  Output under gpurun_out/pmc_ab/<config>/{fetch,write}.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/pmc_ab
rm -rf "$O"; mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
run() {  # run <name> <counter> [ENV=VALUE]
  name=$1; ctr=$2; shift 2
  for kv in "$@"; do export "$kv"; done
  timeout -k 10 240 rocprofv3 --pmc "$ctr" --kernel-trace -d "$O/$name/$ctr" -o pmc --output-format csv -- \
    python3 "$R/bench.py" --steps 10 --warmup 3 --no-cpu-baseline --host-api-steps 0 > "$O/$name.$ctr.log" 2>&1
  for kv in "$@"; do unset "${kv%%=*}"; done
}
run xcd FETCH_SIZE
run xcd WRITE_SIZE
run one FETCH_SIZE DX_ONE_QUEUE=1
run one WRITE_SIZE DX_ONE_QUEUE=1
run noq FETCH_SIZE DX_NO_QUEUE=1
run noq WRITE_SIZE DX_NO_QUEUE=1
