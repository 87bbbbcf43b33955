#!/bin/bash
# HBM traffic of the bench headline (the whole-model CompressionPlan launches): separate rocprofv3
# PMC passes for FETCH_SIZE and WRITE_SIZE over `bench.py --profile-only` (MI355X_MICROARCH.md:
# FETCH_SIZE costs 3 TCC slots, WRITE_SIZE 2 -- one per pass).  Summarised by
# scripts/pmc_headline_summary.py into profiles/headline_pmc.json, which bench.py reports as
# roofline.traffic.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${TAG:-r02n}
OUT=$PWD/gpurun_out/pmch_$TAG
mkdir -p $OUT
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 5 -s KILL 240 rocprofv3 --pmc $c --output-format csv -d $OUT/$c -o run -- \
      python3 $PWD/bench.py --profile-only --steps 20 --warmup 5 > $OUT/$c.log 2>&1
  rc=$?; echo "pmc $c rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 $OUT/$c.log; exit $rc; fi
done
echo done
