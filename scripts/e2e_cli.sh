#!/bin/bash
# End-to-end do_oneshot CLI on a random-init model of the public dims (offline), on one GPU:
#   bash scripts/e2e_cli.sh <config.yaml> <model config dir> <N,S calibration> <tag>
# log -> gpurun_out/e2e_<tag>.log (AWQ per-layer times, save time), checkpoint in /tmp.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 ${TO:-900} python3 -u scripts/do_oneshot.py --config "$1" --random-init "$2" --calib-random "$3" \
    --output /tmp/e2e_out_$4 ${EXTRA:-} > gpurun_out/e2e_$4.log 2>&1
rc=$?
grep -E "AWQ layer|Completed|Saved|SUCCESS|Error|error" gpurun_out/e2e_$4.log | tail -12
du -sh /tmp/e2e_out_$4 2>/dev/null
exit $rc
