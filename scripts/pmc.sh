#!/bin/bash
# PMC passes for the bench kernel (separate passes per MI355X_MICROARCH.md §rocprofv3 PMC slots).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${TAG:-r01}
OUT=$PWD/gpurun_out/pmc_$TAG
mkdir -p $OUT
timeout -k 10 120 rocprofv3 -L > $OUT/counters_list.txt 2>&1 || true
for c in FETCH_SIZE WRITE_SIZE "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR" "SQ_BUSY_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE"; do
  n=$(echo $c | tr ' ' '_')
  timeout -k 10 300 rocprofv3 --pmc $c --output-format csv -d $OUT/$n -o run -- python3 $PWD/bench.py --profile-only --steps 30 --warmup 3 > $OUT/$n.log 2>&1
  rc=$?; echo "pmc $c rc=$rc"
  if [ $rc -ge 124 ]; then exit $rc; fi
done
