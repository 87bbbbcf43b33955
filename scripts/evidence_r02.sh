#!/bin/bash
# Round-2 evidence session on one GPU box (logs -> gpurun_out/evid_$TAG/, summarised into profiles/):
#  * sustain.py (per-launch durations over long back-to-back runs, output-residency variants)
#    with rocm-smi power / clock samples taken while it runs;
#  * first_touch.py and idle_gap.py (never-written outputs; idle gap before a launch);
#  * the multi-rank bench path rehearsed with 2 gloo ranks sharing the card.
# Every GPU step has its own time limit; a timeout / crash ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${TAG:-r02m}
OUT=gpurun_out/evid_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
run() {  # run <name> <timeout> <cmd...>
  local name=$1 to=$2; shift 2
  timeout -k 10 "$to" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; tail -n 4 "$OUT/$name.log"
  if [ $rc -ne 0 ]; then echo "ABORT after $name"; exit $rc; fi
}
# sustained run + power samples (rocm-smi reads only)
K=200 REPS=40 timeout -k 10 240 python3 scripts/sustain.py > $OUT/sustain.log 2>&1 &
SP=$!
for i in $(seq 1 30); do
  kill -0 $SP 2>/dev/null || break
  timeout -k 2 10 rocm-smi --showpower --showclocks --showtemp >> $OUT/smi_under_load.txt 2>&1
  sleep 0.5
done
wait $SP
rc=$?
echo "=== sustain rc=$rc"; tail -n 4 $OUT/sustain.log
[ $rc -ne 0 ] && exit $rc
timeout -k 2 10 rocm-smi --showpower --showclocks --showtemp > $OUT/smi_idle.txt 2>&1
run first_touch 120 python3 scripts/first_touch.py
run idle_gap 120 python3 scripts/idle_gap.py
QZ_BENCH_BACKEND=gloo run bench_gloo_n2 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 5 --warmup 2
echo "=== done"
