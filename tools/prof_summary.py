#!/usr/bin/env python3
"""Summarise a rocprofv3 --stats kernel CSV: name (short), calls, avg us, total %, per-step share."""
import csv
import re
import sys


def short(name):
    name = re.sub(r"\(.*", "", name)
    name = name.replace("void ", "").replace("ygzfe::", "")
    return name[:60]


def main(path):
    rows = list(csv.DictReader(open(path)))
    print(f"{'kernel':60s} {'calls':>6s} {'avg_us':>10s} {'min_us':>9s} {'max_us':>9s} {'pct':>6s}")
    for r in rows:
        print(f"{short(r['Name']):60s} {int(r['Calls']):6d} {float(r['AverageNs'])/1e3:10.2f} "
              f"{float(r['MinNs'])/1e3:9.2f} {float(r['MaxNs'])/1e3:9.2f} {float(r['Percentage']):6.2f}")


if __name__ == "__main__":
    main(sys.argv[1])
