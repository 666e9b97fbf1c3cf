"""Issue-side utilisation of the render kernel from a tools/counters.sh run,
written into profiles/pmc_summary.json[KEY]["issue"] (bench.py reports it
under roofline.issue).

    python tools/sq_summary.py gpurun_out/ctr_TAG KEY [KERNEL_SUBSTR]

valu_busy = SQ_ACTIVE_INST_VALU * 4 / SIMDs / (GRBM_GUI_ACTIVE / XCDs): the
fraction of SIMD cycles issuing VALU work (rocprof's VALUBusy; GRBM_GUI_ACTIVE
is summed over the 8 XCDs by rocprofv3, MI355X_MICROARCH.md). wait_frac =
SQ_WAIT_ANY / SQ_WAVE_CYCLES: share of wave cycles waiting on anything
(memory, dependencies); issue_frac = SQ_ACTIVE_INST_ANY / SQ_WAVE_CYCLES.
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

src, key = sys.argv[1], sys.argv[2]
kname = sys.argv[3] if len(sys.argv) > 3 else "k_accel<false, false, true, false"
SIMDS, XCDS = 256 * 4, 8
vals = defaultdict(list)
for f in glob.glob(os.path.join(src, "p*", "**", "*counter_collection.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        if kname in r["Kernel_Name"]:
            vals[r["Counter_Name"]].append(float(r["Counter_Value"]))
m = {k: sum(v) / len(v) for k, v in vals.items()}
issue = {
    "valu_busy": m["SQ_ACTIVE_INST_VALU"] * 4 / SIMDS / (m["GRBM_GUI_ACTIVE"] / XCDS),
    "wait_frac": m["SQ_WAIT_ANY"] / m["SQ_WAVE_CYCLES"],
    "issue_frac": m["SQ_ACTIVE_INST_ANY"] / m["SQ_WAVE_CYCLES"],
    "l2_hit": m["TCC_HIT_sum"] / (m["TCC_HIT_sum"] + m["TCC_MISS_sum"]),
    "valu_insts_per_wave": m["SQ_INSTS_VALU"] / m["SQ_WAVES"],
    "launches": len(vals["SQ_WAVES"]),
    "source": f"{src} (tools/counters.sh, rocprofv3 --pmc SQ_*/GRBM_*/TCC_* passes), kernel {kname}",
}
root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
path = os.path.join(root, "profiles", "pmc_summary.json")
data = json.load(open(path)) if os.path.exists(path) else {}
data.setdefault(key, {})["issue"] = issue
json.dump(data, open(path, "w"), indent=1)
print(key, issue)
