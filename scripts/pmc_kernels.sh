#!/bin/bash
# rocprofv3 PMC passes (one counter set per run, MI355X_MICROARCH.md slot limits) over
# scripts/kernel_driver.py, plus one kernel-trace --stats run.  Output: gpurun_out/pmck_$TAG/.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${TAG:-r02}
OUT=$PWD/gpurun_out/pmck_$TAG
mkdir -p $OUT
N=${N:-30}
timeout -k 5 60 rocprofv3 -L > $OUT/counters_list.txt 2>&1 || true
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 $PWD/scripts/kernel_driver.py $N > $OUT/trace.log 2>&1
rc=$?; echo "trace rc=$rc"; [ $rc -ne 0 ] && exit $rc
for c in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_INSTS_LDS SQ_BUSY_CYCLES SQ_WAVE_CYCLES" "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VMEM_RD SQ_INSTS_VALU_TRANS_F32 GRBM_GUI_ACTIVE GRBM_COUNT"; do
  n=$(echo $c | tr ' ' '_')
  timeout -k 5 -s KILL 90 rocprofv3 --pmc $c --output-format csv -d $OUT/$n -o run -- python3 $PWD/scripts/kernel_driver.py $N > $OUT/$n.log 2>&1
  rc=$?; echo "pmc $c rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 $OUT/$n.log; fi
  if [ $rc -ge 124 ]; then exit $rc; fi  # timeout / signal: stop using the GPU
done
echo done
