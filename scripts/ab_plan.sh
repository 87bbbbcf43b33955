#!/bin/bash
# A/B of the whole-model plan: grouped launches on 1, 2 or 3 streams (QZ_PLAN_STREAMS)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for r in 1 2 3; do
  for m in 1 2 3; do
    QZ_PLAN_STREAMS=$m timeout -k 10 200 python3 bench.py --no-extras --no-cpu-baseline --steps 40 > gpurun_out/abst_${m}_$r.log 2>&1 || exit $?
    python3 -c "import json,sys; l=json.loads([x for x in open('gpurun_out/abst_${m}_$r.log') if x.startswith('{')][-1]); print('streams=$m round $r', round(l['ms_per_step'],4), 'ms/step frac', round(l['roofline']['frac'],4), [ (p['weights'], round(p['GBps'])) for p in l['per_launch']])"
  done
done
