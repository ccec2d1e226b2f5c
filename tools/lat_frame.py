"""Kernels and copies of one single-frame latency iteration (the last k_pyramid* launch
before the end of the trace's latency section), with queue and start / duration in µs."""
import csv
import glob
import os
import sys

d = sys.argv[1]
rows = []
for pat, kind in (("*kernel_trace.csv", "k"), ("*memory_copy_trace.csv", "c")):
    for f in glob.glob(os.path.join(d, "**", pat), recursive=True):
        for r in csv.DictReader(open(f)):
            name = r.get("Kernel_Name") or ("copy " + r.get("Direction", ""))
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r.get("Queue_Id", r.get("Stream_Id", "")), name.split("(")[0][:60]))
rows.sort()
pyr = [i for i, r in enumerate(rows) if "k_pyramid" in r[3] or "k_resize" in r[3]]
i0 = pyr[-int(sys.argv[2]) if len(sys.argv) > 2 else -3]
t0 = rows[i0][0]
for s, e, q, n in rows[i0:i0 + 40]:
    print(f"{(s - t0) / 1e3:8.1f} {(e - s) / 1e3:7.1f} q{q:>3} {n}")
