#!/bin/bash
# A/B: one grouped launch per shape (QZ_PLAN_MIXED=0) vs one mixed-shape launch (=1), interleaved.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for r in 1 2 3; do
  for m in 0 1; do
    QZ_PLAN_MIXED=$m timeout -k 10 200 python3 bench.py --no-extras --no-cpu-baseline --steps 40 > gpurun_out/abmx_${m}_$r.log 2>&1 || exit $?
    python3 -c "import json; l=json.loads([x for x in open('gpurun_out/abmx_${m}_$r.log') if x.startswith('{')][-1]); print('mixed=$m round $r', round(l['ms_per_step'],4), 'ms/step frac', round(l['roofline']['frac'],4))"
  done
done
