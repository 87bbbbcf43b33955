#!/bin/bash
# Round-3 session ac: where the Qwen3-4B AWQ pass spends its time before and around layer 0
# (capture, batched-call check, first calls): the CLI with the setup timings logged, and a
# cProfile of the same run (top cumulative entries).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TO=300 bash scripts/e2e_cli.sh configs/qwen3-4b-awq-g128.yaml configs/models/qwen3-4b 16,2048 r03ac_qwen3_4b > /dev/null || exit $?
grep -E "Starting|moved|captured|batched call|AWQ layer (0|1|35):|Completed" gpurun_out/e2e_r03ac_qwen3_4b.log | sed 's/ - quantizers_amd[^-]*- / /'
rm -rf /tmp/e2e_out_r03ac_qwen3_4b
timeout -k 10 300 python3 -m cProfile -o gpurun_out/r03ac_oneshot.prof scripts/do_oneshot.py --config configs/qwen3-4b-awq-g128.yaml \
  --random-init configs/models/qwen3-4b --calib-random 16,2048 --output /tmp/e2e_out_r03ac_prof > gpurun_out/r03ac_prof_run.log 2>&1 || exit $?
python3 -c "
import pstats; p = pstats.Stats('gpurun_out/r03ac_oneshot.prof'); p.sort_stats('cumulative').print_stats(45)" > gpurun_out/r03ac_cprofile.txt 2>&1
head -80 gpurun_out/r03ac_cprofile.txt | tail -60
