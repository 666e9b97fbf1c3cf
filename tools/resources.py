"""Per-kernel register / scratch / occupancy table from the compiler's
kernel-resource-usage remarks (gfx950 device compile of rt_kernels.hip)."""
import re
import subprocess
import sys

src = sys.argv[1] if len(sys.argv) > 1 else "opengl-ray-tracer_amd/csrc/rt_kernels.hip"
extra = sys.argv[2:]
cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=off",
       "-fhip-fp32-correctly-rounded-divide-sqrt", "--offload-device-only", "-c", "-o", "/dev/null",
       src, "-Rpass-analysis=kernel-resource-usage"] + extra
out = subprocess.run(cmd, capture_output=True, text=True).stderr
rows, cur = [], None
for line in out.splitlines():
    m = re.search(r"remark: (.*?) \[-Rpass", line)
    if not m:
        continue
    txt = m.group(1).strip()
    if txt.startswith("Function Name:"):
        name = txt.split(":", 1)[1].strip()
        dm = subprocess.run(["c++filt", name], capture_output=True, text=True).stdout.strip()
        dm = dm.replace("(anonymous namespace)::", "").replace("void ", "")
        cur = {"name": re.sub(r"\(.*", "", dm)}
        rows.append(cur)
    elif cur is not None and ":" in txt:
        k, v = txt.split(":", 1)
        cur[k.strip()] = v.strip()
keys = ["VGPRs", "AGPRs", "SGPRs", "ScratchSize [bytes/lane]", "VGPRs Spill", "SGPRs Spill",
        "Occupancy [waves/SIMD]", "LDS Size [bytes/block]"]
print("%-34s" % "kernel" + "".join("%9s" % k.split(" ")[0][:8] for k in keys))
for r in rows:
    print("%-34s" % (r["name"] if "-full" in sys.argv[0:1] or __import__("os").environ.get("FULL") else r["name"][:34]) + "".join("%9s" % r.get(k, "-") for k in keys))
