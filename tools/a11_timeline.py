"""One a11 host call's timeline from rocprofv3 --hip-trace --kernel-trace --memory-copy-trace
CSVs: HIP API calls (host) and device activity of the last search_projection_best call,
offsets in µs from the call's first API entry."""
import csv
import glob
import os
import sys

d = sys.argv[1]


def load(pat):
    f = glob.glob(os.path.join(d, "**", pat), recursive=True)
    return list(csv.DictReader(open(f[0]))) if f else []


api = load("*hip_api_trace.csv")
ker = load("*kernel_trace.csv")
cpy = load("*memory_copy_trace.csv")
tops = sorted(int(r["Start_Timestamp"]) for r in ker if "k_match_topk" in r["Kernel_Name"])
t_top = tops[-2]  # the last best search's topk (the ratio search follows)
# the call's API window: from the last hipEventSynchronize before the topk to the next hipStreamSynchronize end
apis = sorted(api, key=lambda r: int(r["Start_Timestamp"]))
start = max(int(r["Start_Timestamp"]) for r in apis if r["Function"] == "hipEventSynchronize" and int(r["Start_Timestamp"]) < t_top)
end = min(int(r["End_Timestamp"]) for r in apis if r["Function"] == "hipStreamSynchronize" and int(r["End_Timestamp"]) > t_top)
ev = []
for r in apis:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    if start <= s <= end:
        ev.append((s, e, "api  " + r["Function"]))
for r in ker:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    if start <= s <= end:
        ev.append((s, e, "gpu  " + r["Kernel_Name"].split("(")[0][:50]))
for r in cpy:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    if start <= s <= end:
        ev.append((s, e, "copy " + r.get("Direction", "?")))
for s, e, n in sorted(ev):
    print(f"{(s - start) / 1e3:8.1f} {(e - s) / 1e3:8.1f}  {n}")
print("call span", (end - start) / 1e3)
