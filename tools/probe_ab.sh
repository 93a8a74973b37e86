#!/bin/bash
# bench.py kernel probes under two values of an environment variable, interleaved (2 rounds):
#   tools/probe_ab.sh VAR "valA valB"   -> gpurun_out/probe_ab_VAR.txt (probe name, us, frac)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
VAR=$1; VALS=$2
for r in 1 2; do
  for v in $VALS; do
    tag=$(basename "$v")
    env $VAR=$v timeout -k 10 200 python bench.py --probe-only > gpurun_out/probe_${tag:-none}_$r.json 2>/dev/null || exit 1
    python - "$VAR=$tag round $r" gpurun_out/probe_${tag:-none}_$r.json >> gpurun_out/probe_ab_$VAR.txt <<'PY'
import json, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
print(sys.argv[1], " ".join(f"{p['name']}={p['avg_launch_us']:.1f}" for p in d["probes"]))
PY
  done
done
