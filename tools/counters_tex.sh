#!/bin/bash
# Vector-memory pipe counter passes (TA / TD / TCP) for one bench workload.
# usage: bash tools/counters_tex.sh TAG [bench args...]
set -o pipefail
TAG=$1; shift
OUT=gpurun_out/ctrt_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
i=0
for set in "TA_BUSY_avr TA_TA_BUSY_sum GRBM_GUI_ACTIVE" \
           "TD_TD_BUSY_sum TD_TCP_STALL_CYCLES_sum GRBM_GUI_ACTIVE" \
           "TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum TCP_READ_TAGCONFLICT_STALL_CYCLES_sum" \
           "TA_ADDR_STALLED_BY_TC_CYCLES_sum TA_DATA_STALLED_BY_TC_CYCLES_sum GRBM_COUNT"; do
  i=$((i+1))
  timeout -k 10 -s KILL 120 rocprofv3 --pmc $set --output-format csv -d $OUT/p$i -o run -- \
      python3 bench.py --no-cpu "$@" > $OUT/bench_p$i.json 2> $OUT/p$i.err || { echo "pass $i failed"; tail -5 $OUT/p$i.err; exit 1; }
done
python3 - "$OUT" <<'PY'
import csv, glob, sys, collections
out = sys.argv[1]
agg = collections.defaultdict(list)
for f in glob.glob(out + "/p*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "k_accel" in r["Kernel_Name"]:
            agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
for c, v in sorted(agg.items()):
    print(f"{c:40s} {sum(v)/len(v):16.1f}  (n={len(v)})")
PY
