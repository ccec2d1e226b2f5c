#!/usr/bin/env python3
"""Timeline of the last bench step from a rocprofv3 kernel_trace.csv: every
dispatch after the last `pyramid` launch, with its start offset, duration and
the idle gap before it (per queue)."""
import csv
import re
import sys


def short(name):
    name = re.sub(r"\(.*", "", name)
    return name.replace("void ", "").replace("ygzfe::", "")[:46]


rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
starts = [i for i, r in enumerate(rows) if "fillBuffer" in r["Kernel_Name"]]  # the memset opening each extract
first = starts[-2] if len(starts) > 1 else 0
last = starts[-1]
seg = rows[first:last]
t0 = int(seg[0]["Start_Timestamp"])
end_prev = {}
print(f"{'kernel':46} {'queue':>6} {'start_us':>9} {'dur_us':>8} {'gap_us':>7}")
for r in seg:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    q = r.get("Queue_Id", r.get("Stream_Id", "?"))
    gap = (s - end_prev[q]) / 1e3 if q in end_prev else 0.0
    end_prev[q] = e
    print(f"{short(r['Kernel_Name']):46} {q:>6} {(s - t0) / 1e3:9.1f} {(e - s) / 1e3:8.1f} {gap:7.1f}")
print(f"step span: {(max(int(r['End_Timestamp']) for r in seg) - t0) / 1e3:.1f} us")
