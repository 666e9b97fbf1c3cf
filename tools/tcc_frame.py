"""L2 (TCC) hits and misses per launch of each render kernel, from a tools/gpu_prof.sh
tcc pass: python tools/tcc_frame.py gpurun_out/prof_TAG"""
import collections
import csv
import glob
import sys

f = glob.glob(sys.argv[1] + "/tcc/**/*counter_collection.csv", recursive=True)[0]
agg = collections.defaultdict(lambda: collections.defaultdict(float))
disp = collections.defaultdict(set)
for r in csv.DictReader(open(f)):
    k = r["Kernel_Name"].replace("void ", "").replace("(anonymous namespace)::", "").split("(")[0]
    if "accel" not in k:
        continue
    agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
    disp[k].add(r["Dispatch_Id"])
tot = collections.Counter()
for k in sorted(agg):
    n = len(disp[k])
    per = {c: v / n for c, v in agg[k].items()}
    print(f"{k:55s} launches {n:3d}  " + "  ".join(f"{c} {v / 1e6:.3f}M" for c, v in sorted(per.items())))
