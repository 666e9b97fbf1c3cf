#!/bin/bash
# SQ/GRBM counter passes for one bench workload (kernel-trace + pmc only).
# usage: bash tools/counters.sh TAG [bench args...]
set -o pipefail
TAG=$1; shift
OUT=gpurun_out/ctr_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
i=0
for set in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY" \
           "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_ANY SQ_INSTS_BRANCH SQ_INSTS_VMEM SQ_INSTS_LDS GRBM_GUI_ACTIVE" \
           "TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $set --output-format csv -d $OUT/p$i -o run -- \
      python3 bench.py --no-cpu "$@" > $OUT/bench_p$i.json 2> $OUT/p$i.err || { echo "pass $i failed"; tail -20 $OUT/p$i.err; exit 1; }
done
python3 - "$OUT" <<'PY'
import csv, glob, sys, collections
out = sys.argv[1]
agg = collections.defaultdict(list)
for f in glob.glob(out + "/p*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "k_accel" in r["Kernel_Name"] or "k_packet" in r["Kernel_Name"] or "k_lane<false>" in r["Kernel_Name"]:
            agg[(r["Kernel_Name"][:40], r["Counter_Name"])].append(float(r["Counter_Value"]))
for (k, c), v in sorted(agg.items()):
    print(f"{k:42s} {c:24s} {sum(v)/len(v):16.1f}  (n={len(v)})")
PY
