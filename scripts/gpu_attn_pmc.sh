#!/bin/bash
# PMC passes over the batched level-0 attention (each pass its own run, --pmc only).
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-apmc}
mkdir -p $O
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
i=0
for set in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM SQ_WAIT_ANY SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  (cd $R && timeout -s KILL 120 rocprofv3 --pmc $set -d $O/p$i -o run --output-format csv -- python3 scripts/attn_pmc_target.py > $O/p$i.log 2>&1) || { tail -5 $O/p$i.log; exit 1; }
done
python - <<PY
import csv, glob, collections
for f in sorted(glob.glob("$O/p*/**/*counter_collection.csv", recursive=True)):
    agg = collections.defaultdict(float); n = collections.Counter()
    for r in csv.DictReader(open(f)):
        if "flash_attn" not in r.get("Kernel_Name", ""): continue
        agg[r["Counter_Name"]] += float(r["Counter_Value"]); n[r["Counter_Name"]] += 1
    print(f.split("/")[-3], {k: round(v / max(1, n[k] // 1), 1) for k, v in agg.items()})
PY
