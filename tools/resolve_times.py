"""Group k_match_resolve durations from a rocprofv3 kernel trace into blocks of 20 calls."""
import csv
import sys

rows = [r for r in csv.DictReader(open(sys.argv[1])) if "k_match_resolve" in r["Kernel_Name"]]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in rows]
for i in range(0, len(d), 20):
    blk = sorted(d[i:i + 20])
    print(i // 20, round(blk[len(blk) // 2], 2))
