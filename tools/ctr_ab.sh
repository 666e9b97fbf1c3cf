#!/bin/bash
# SQ counters for two builds of k_accel in one process (tools/ab.py --lib2):
# dispatches alternate build 1 / build 2 in blocks of (1 + frames).
# usage: bash tools/ctr_ab.sh TAG LIB2 CONFIG
set -o pipefail
TAG=$1; LIB2=$2; CFG=$3
OUT=gpurun_out/ctrab_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
i=0
for set in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY" \
           "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_ANY SQ_INSTS_BRANCH SQ_INSTS_VMEM SQ_INSTS_LDS GRBM_GUI_ACTIVE SQ_ACTIVE_INST_LDS"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $set --output-format csv -d $OUT/p$i -o run -- \
      python3 tools/ab.py --config $CFG --rounds 1 --frames 3 --variants default,default@2 --lib2 $LIB2 > $OUT/ab_p$i.txt 2> $OUT/p$i.err || { echo "pass $i failed"; tail -20 $OUT/p$i.err; exit 1; }
done
python3 - "$OUT" <<'PY'
import csv, glob, sys, collections
out = sys.argv[1]
rows = collections.defaultdict(dict)
for f in glob.glob(out + "/p*/**/*counter_collection.csv", recursive=True):
    disp = collections.OrderedDict()
    for r in csv.DictReader(open(f)):
        if "k_accel" in r["Kernel_Name"]:
            disp.setdefault(r["Dispatch_Id"], {})[r["Counter_Name"]] = float(r["Counter_Value"])
    ids = sorted(disp, key=int)
    for j, d in enumerate(ids):
        build = 1 if j < len(ids) // 2 else 2
        for k, v in disp[d].items():
            rows[(build, k)].setdefault("v", []).append(v)
for (b, k), d in sorted(rows.items(), key=lambda x: (x[0][1], x[0][0])):
    print(f"build{b} {k:24s} {sum(d['v'])/len(d['v']):16.1f} (n={len(d['v'])})")
PY
