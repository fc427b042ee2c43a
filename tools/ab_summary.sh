#!/bin/bash
# value and ms/step of every A/B bench log under gpurun_out/
for f in gpurun_out/ab_*.log; do
  python3 -c "import json,sys
try:
    d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1], d['value'], d['ms_per_step'])
except Exception: pass" "$f"
done
