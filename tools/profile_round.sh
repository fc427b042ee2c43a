#!/bin/bash
# On the GPU box: kernel-trace stats + separate FETCH_SIZE / WRITE_SIZE PMC passes of
# a short bench run, and the per-stage cycle profile.  Output under gpurun_out/prof;
# tools/summarize_profiles.py turns it into the committed profiles/ files.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/prof
rm -rf "$O"; mkdir -p "$O"
# the library the passes measure (bench.py uses the recorded HBM bytes only for this build)
python3 -c "import sys; sys.path.insert(0, '$R'); from dexterity_amd import _lib; print(_lib.load().dx_build_key().decode())" > "$O/build_key.txt"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$O/trace" -o run --output-format csv -- \
  python3 "$R/bench.py" --steps 40 --warmup 5 --no-cpu-baseline --host-api-steps 0 > "$O/bench_under_rocprof.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d "$O/fetch" -o pmc --output-format csv -- \
  python3 "$R/bench.py" --steps 10 --warmup 3 --no-cpu-baseline --host-api-steps 0 > "$O/fetch.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d "$O/write" -o pmc --output-format csv -- \
  python3 "$R/bench.py" --steps 10 --warmup 3 --no-cpu-baseline --host-api-steps 0 > "$O/write.log" 2>&1
cd "$R"
timeout -k 10 300 python3 tools/stage_profile.py 4096 10 > "$O/stages.log" 2>&1
cp gpurun_out/stages.json "$O/stages.json"
