#!/bin/bash
# PMC passes over scripts/gemm_loss_pmc.py (prototype fused kernel + hipBLASLt of the same shape).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${TAG:-r06n}
i=0
for ctrs in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU" \
            "SQ_INSTS_SALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $ctrs --output-format csv -d "$PWD/gpurun_out/pmc_${TAG}_$i" -o run -- python3 scripts/gemm_loss_pmc.py > gpurun_out/${TAG}_pmc_$i.log 2>&1 || { tail -5 gpurun_out/${TAG}_pmc_$i.log; exit 1; }
done
python3 - <<'PY'
import csv, glob, os, collections
tag = os.environ.get("TAG", "r06n")
for f in sorted(glob.glob(f"gpurun_out/pmc_{tag}_*/*counter_collection.csv")):
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"][:60]
        agg[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, d in agg.items():
        print(k, {c: round(sum(v) / len(v)) for c, v in d.items()})
PY
