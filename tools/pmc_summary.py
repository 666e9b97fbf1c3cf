"""Summarise a tools/gpu_prof.sh (or tools/profile.sh) run into profiles/.

    python tools/pmc_summary.py gpurun_out/prof_TAG KEY [KERNEL_SUBSTR | re:REGEX]

gpu_prof.sh profiles the solo bench command (--inflight 1), so every launch of
the render kernel runs alone; "re:k_accel<" selects every k_accel instance (the
counter-free one and the cost-recording one) and not k_accel_tail.

Copies the rocprofv3 kernel-stats CSV to profiles/TAG_kernel_stats.csv and the
per-dispatch FETCH_SIZE/WRITE_SIZE of the render kernel into
profiles/pmc_summary.json under KEY (bench.py reads it as roofline.traffic),
MERGED into what the key already holds (the "issue" block of sq_summary.py
stays). With SQ passes present (gpu_prof.sh sq1/sq2/tcc), the issue block is
written too.
HBM bytes per launch = 2*FETCH_SIZE*1024 + WRITE_SIZE*1024: on gfx950 FETCH_SIZE
reports half the bytes of a wide coalesced read (MI355X_MICROARCH.md, HBM).
"""
import csv
import json
import os
import re
import shutil
import sys

src, key = sys.argv[1], sys.argv[2]
kname = sys.argv[3] if len(sys.argv) > 3 else "k_packet"
tag = os.path.basename(src.rstrip("/")).replace("prof_", "")
root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
prof = os.path.join(root, "profiles")
os.makedirs(prof, exist_ok=True)


def find(sub, name):
    for dp, _, fs in os.walk(os.path.join(src, sub)):
        for f in fs:
            if f.endswith(name):
                return os.path.join(dp, f)
    raise SystemExit(f"no {name} under {src}/{sub}")


shutil.copy(find("trace", "kernel_stats.csv"), os.path.join(prof, f"{tag}_kernel_stats.csv"))


def matches(name):
    return re.search(kname[3:], name) is not None if kname.startswith("re:") else kname in name


def per_launch(sub, counter):
    vals = [float(r["Counter_Value"]) for r in csv.DictReader(open(find(sub, "counter_collection.csv")))
            if matches(r["Kernel_Name"]) and r["Counter_Name"] == counter]
    return sum(vals) / len(vals), len(vals)


def mean_duration_ms():
    rows = [r for r in csv.DictReader(open(find("trace", "kernel_stats.csv"))) if matches(r["Name"])]
    calls = sum(int(r["Calls"]) for r in rows)
    return sum(float(r["TotalDurationNs"]) for r in rows) / calls / 1e6, calls


# the selected kernel's counter values of every pass, kept beside the stats
with open(os.path.join(prof, f"{tag}_counters.csv"), "w", newline="") as fo:
    w = csv.writer(fo)
    w.writerow(["pass", "dispatch", "kernel", "counter", "value"])
    for sub in sorted(os.listdir(src)):
        for dp, _, fs in os.walk(os.path.join(src, sub)):
            for f in fs:
                if f.endswith("counter_collection.csv"):
                    for r in csv.DictReader(open(os.path.join(dp, f))):
                        if matches(r["Kernel_Name"]):
                            w.writerow([sub, r.get("Dispatch_Id", ""), r["Kernel_Name"][:60], r["Counter_Name"],
                                        r["Counter_Value"]])

fetch, n1 = per_launch("fetch", "FETCH_SIZE")
write, n2 = per_launch("write", "WRITE_SIZE")
entry = {"bytes": (2 * fetch + write) * 1024, "fetch_size_kb": fetch, "write_size_kb": write,
         "fetch_bytes_corrected": 2 * fetch * 1024, "write_bytes": write * 1024, "launches": [n1, n2],
         "source": f"profiles/{tag}_kernel_stats.csv + rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes",
         "kernel": kname}
path = os.path.join(prof, "pmc_summary.json")
data = json.load(open(path)) if os.path.exists(path) else {}
try:
    entry["kernel_ms_rocprof"], entry["kernel_calls_rocprof"] = mean_duration_ms()
except (KeyError, SystemExit, ZeroDivisionError):
    pass
data.setdefault(key, {}).update(entry)
json.dump(data, open(path, "w"), indent=1)
print(key, entry)
if os.path.isdir(os.path.join(src, "sq1")):
    import subprocess
    subprocess.run([sys.executable, os.path.join(root, "tools", "sq_summary.py"), src, key, kname], check=True)
