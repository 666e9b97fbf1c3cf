"""Issue side of the render kernel from the SQ/GRBM/TCC passes of tools/gpu_prof.sh
(or tools/counters.sh), written into profiles/pmc_summary.json[KEY]["issue"]
(bench.py reports it as roofline.issue and prices the frame against it).

    python tools/sq_summary.py gpurun_out/prof_TAG KEY [KERNEL_SUBSTR | re:REGEX]

Per launch (means over the launches of the selected kernel):
  clock_ghz      = GRBM_GUI_ACTIVE / 8 XCDs / the launch's duration (rocprofv3 sums
                   GRBM_GUI_ACTIVE over the XCDs, MI355X_MICROARCH.md "DVFS give-back";
                   the duration is the trace pass's mean for the same kernel)
  valu_busy      = SQ_ACTIVE_INST_VALU * 4 / SIMDs / (GRBM_GUI_ACTIVE / XCDs): the share of
                   SIMD cycles issuing VALU work (SQ_ACTIVE_* count quad-cycles)
  valu_floor_ms  = SQ_INSTS_VALU * 2 cycles / 1,024 SIMDs / clock: every VALU
                   instruction at the SIMD's wave64 throughput (2 cycles, 32 lanes per
                   cycle; MI355X_MICROARCH.md per-instruction constants), all SIMDs busy
  salu_floor_ms  = SQ_INSTS_SALU * 1 cycle / 256 CUs / clock: one scalar ALU per CU
                   issuing one instruction per cycle for its four SIMDs' waves (the GCN
                   issue model; an assumption -- not measured on gfx950 here)
  issue_floor_frac = max(valu_floor, salu_floor) / the launch's duration
  wait_frac / issue_frac / stall_frac = SQ_WAIT_ANY / SQ_ACTIVE_INST_ANY /
                   SQ_WAIT_INST_ANY over SQ_WAVE_CYCLES (disjoint, sum ~1)
  l2_hit         = TCC_HIT / (TCC_HIT + TCC_MISS); l2_miss_bytes = TCC_MISS * 128
"""
import csv
import glob
import json
import os
import re
import sys
from collections import defaultdict

src, key = sys.argv[1], sys.argv[2]
kname = sys.argv[3] if len(sys.argv) > 3 else "re:k_accel<"
SIMDS, CUS, XCDS = 256 * 4, 256, 8


def matches(name):
    return re.search(kname[3:], name) is not None if kname.startswith("re:") else kname in name


vals = defaultdict(list)
for f in glob.glob(os.path.join(src, "*", "**", "*counter_collection.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        if matches(r["Kernel_Name"]):
            vals[r["Counter_Name"]].append(float(r["Counter_Value"]))
m = {k: sum(v) / len(v) for k, v in vals.items()}
dur_ms = None
for f in glob.glob(os.path.join(src, "trace", "**", "*kernel_stats.csv"), recursive=True):
    rows = [r for r in csv.DictReader(open(f)) if matches(r["Name"])]
    calls = sum(int(r["Calls"]) for r in rows)
    if calls:
        dur_ms = sum(float(r["TotalDurationNs"]) for r in rows) / calls / 1e6
issue = {"launches": len(vals.get("SQ_WAVES", [])), "kernel_ms_rocprof": dur_ms,
         "waves": m.get("SQ_WAVES"),
         "valu_insts_per_wave": m["SQ_INSTS_VALU"] / m["SQ_WAVES"],
         "salu_insts_per_wave": m["SQ_INSTS_SALU"] / m["SQ_WAVES"],
         "smem_insts_per_wave": m.get("SQ_INSTS_SMEM", 0) / m["SQ_WAVES"],
         "vmem_insts_per_wave": m.get("SQ_INSTS_VMEM", 0) / m["SQ_WAVES"],
         "lds_insts_per_wave": m.get("SQ_INSTS_LDS", 0) / m["SQ_WAVES"],
         "wait_frac": m["SQ_WAIT_ANY"] / m["SQ_WAVE_CYCLES"],
         "issue_frac": m["SQ_ACTIVE_INST_ANY"] / m["SQ_WAVE_CYCLES"],
         "stall_frac": m["SQ_WAIT_INST_ANY"] / m["SQ_WAVE_CYCLES"]}
if "GRBM_GUI_ACTIVE" in m:
    cyc = m["GRBM_GUI_ACTIVE"] / XCDS
    issue["valu_busy"] = m["SQ_ACTIVE_INST_VALU"] * 4 / SIMDS / cyc
    # SQ_ACTIVE_INST_SCA summed over waves reads 1.5 per CU-cycle on the car kernel, so
    # it is not a single-issuer occupancy: reported per SIMD, like valu_busy
    issue["salu_busy"] = m["SQ_ACTIVE_INST_SCA"] * 4 / SIMDS / cyc if "SQ_ACTIVE_INST_SCA" in m else None
    if dur_ms:
        clk = cyc / (dur_ms * 1e-3)
        issue["clock_ghz"] = clk / 1e9
        issue["valu_floor_ms"] = m["SQ_INSTS_VALU"] * 2 / SIMDS / clk * 1e3
        issue["salu_floor_ms"] = m["SQ_INSTS_SALU"] / CUS / clk * 1e3
        issue["issue_floor_frac"] = max(issue["valu_floor_ms"], issue["salu_floor_ms"]) / dur_ms
if "TCC_HIT_sum" in m:
    issue["l2_hit"] = m["TCC_HIT_sum"] / (m["TCC_HIT_sum"] + m["TCC_MISS_sum"])
    issue["l2_miss_bytes"] = m["TCC_MISS_sum"] * 128
issue["source"] = (f"{src} (rocprofv3 --pmc SQ_*/GRBM_GUI_ACTIVE/TCC_* passes of the solo bench command), "
                   f"kernel {kname}")
root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
path = os.path.join(root, "profiles", "pmc_summary.json")
data = json.load(open(path)) if os.path.exists(path) else {}
data.setdefault(key, {})["issue"] = issue
json.dump(data, open(path, "w"), indent=1)
print(key, json.dumps(issue, indent=1))
