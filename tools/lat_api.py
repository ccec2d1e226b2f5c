"""Host HIP API calls and device activity around one single-frame latency iteration
(trace from tools/run_lat_trace.sh): µs offsets from the frame's pyramid launch call."""
import csv
import sys

d = sys.argv[1]
idx = int(sys.argv[2]) if len(sys.argv) > 2 else 100
ker = sorted(csv.DictReader(open(d + "/run_kernel_trace.csv")), key=lambda r: int(r["Start_Timestamp"]))
api = sorted(csv.DictReader(open(d + "/run_hip_api_trace.csv")), key=lambda r: int(r["Start_Timestamp"]))
cpy = list(csv.DictReader(open(d + "/run_memory_copy_trace.csv")))
pyr = [r for r in ker if "k_pyramid" in r["Kernel_Name"]]
k0 = pyr[-idx]
k1 = pyr[-idx + 1]
ts, te = int(k0["Start_Timestamp"]), int(k1["Start_Timestamp"])
# the API call that launched the pyramid: the last hipLaunchKernel before its start
la = [r for r in api if r["Function"] in ("hipLaunchKernel", "hipGraphLaunch", "hipMemcpyAsync") and int(r["Start_Timestamp"]) < ts]
t0 = int(la[-3]["Start_Timestamp"])
ev = []
for r in api:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    if t0 <= s < te and "Configuration" not in r["Function"]:
        ev.append((s, e, "api  " + r["Function"]))
for r in ker:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    if t0 <= s < te:
        ev.append((s, e, "gpu  q" + r.get("Queue_Id", "") + " " + r["Kernel_Name"].split("(")[0][:44]))
for r in cpy:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    if t0 <= s < te:
        ev.append((s, e, "copy q" + r.get("Queue_Id", "") + " " + r.get("Direction", "")))
for s, e, n in sorted(ev):
    print(f"{(s - t0) / 1e3:8.1f} {(e - s) / 1e3:8.1f}  {n}")
