#!/usr/bin/env python3
"""Per-kernel average of rocprofv3 --pmc counters (counter_collection.csv):
value per dispatch, summed over the dispatch's dimensions, averaged over dispatches."""
import collections
import csv
import re
import sys


def short(name):
    name = re.sub(r"\(.*", "", name)
    return name.replace("void ", "").replace("ygzfe::", "")[:44]


def main(paths):
    acc = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(lambda: collections.defaultdict(set))  # kernel -> counter -> dispatches
    for path in paths:
        for r in csv.DictReader(open(path)):
            k = short(r["Kernel_Name"])
            acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
            disp[k][r["Counter_Name"]].add((path, r["Dispatch_Id"]))
    names = sorted({c for v in acc.values() for c in v})
    print("kernel".ljust(44), "n".rjust(4), *[c[:14].rjust(14) for c in names])
    for k in sorted(acc):
        n = max(len(v) for v in disp[k].values())
        print(k.ljust(44), str(n).rjust(4),
              *[f"{acc[k][c] / max(1, len(disp[k][c])):14.4g}" for c in names])


if __name__ == "__main__":
    main(sys.argv[1:])
