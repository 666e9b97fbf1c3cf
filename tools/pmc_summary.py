"""Summarise a tools/profile.sh run into profiles/.

    python tools/pmc_summary.py gpurun_out/prof_TAG KEY [KERNEL_SUBSTR | re:REGEX]

The default bench command also runs a latency-mode pass (another k_accel
instance): select the production instances with a regex, e.g.
    re:k_accel<false, false, true, (true|false), false, false>

Copies the rocprofv3 kernel-stats CSV to profiles/TAG_kernel_stats.csv and the
per-dispatch FETCH_SIZE/WRITE_SIZE of the render kernel into
profiles/pmc_summary.json under KEY (bench.py reads it as roofline.traffic).
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


fetch, n1 = per_launch("fetch", "FETCH_SIZE")
write, n2 = per_launch("write", "WRITE_SIZE")
entry = {"bytes": (2 * fetch + write) * 1024, "fetch_size_kb": fetch, "write_size_kb": write,
         "fetch_bytes_corrected": 2 * fetch * 1024, "write_bytes": write * 1024, "launches": [n1, n2],
         "source": f"profiles/{tag}_kernel_stats.csv + rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes",
         "kernel": kname}
path = os.path.join(prof, "pmc_summary.json")
data = json.load(open(path)) if os.path.exists(path) else {}
data[key] = entry
json.dump(data, open(path, "w"), indent=1)
print(key, entry)
