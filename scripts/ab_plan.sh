#!/bin/bash
# A/B of the whole-model plan: one launch per (scheme, shape) vs one mixed-shape launch per
# scheme (QZ_PLAN_MIXED), interleaved runs of the headline only.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for r in 1 2 3; do
  for m in 0 1; do
    QZ_PLAN_MIXED=$m timeout -k 10 200 python3 bench.py --no-extras --no-cpu-baseline --steps 40 > gpurun_out/abplan_${m}_$r.log 2>&1 || exit $?
    python3 -c "import json,sys; l=json.loads([x for x in open('gpurun_out/abplan_${m}_$r.log') if x.startswith('{')][-1]); print('mixed=$m round $r', round(l['ms_per_step'],4), 'ms/step frac', round(l['roofline']['frac'],4), [ (p['weights'], round(p['GBps'])) for p in l['per_launch']])"
  done
done
