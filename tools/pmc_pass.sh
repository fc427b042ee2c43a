#!/bin/bash
# Usage (on the GPU box): tools/pmc_pass.sh <outdir> <counters...>
# One rocprofv3 PMC pass over a short bench run (kernel trace only, no runtime traces).
set -e
out=$1; shift
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --pmc "$@" --kernel-trace -d "$GRAFT_REPO_ROOT/$out" -o pmc --output-format csv -- \
  python3 "$GRAFT_REPO_ROOT/bench.py" --steps 10 --warmup 3 --no-cpu-baseline --host-api-steps 0
