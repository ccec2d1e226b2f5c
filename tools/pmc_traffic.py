#!/usr/bin/env python3
"""Per-stage HBM traffic per bench step from rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE
passes (tools/run_pmc.sh), corrected as MI355X_MICROARCH.md §HBM prescribes:
FETCH_SIZE (KiB) x 1024 x 2 (gfx950 tallies 128-B read requests at 64 B),
WRITE_SIZE (KiB) x 1024.  Writes JSON {stage: {fetch_bytes, write_bytes, traffic_bytes}}
per step (= per stage launch set) for bench.py's roofline.traffic.

    python3 tools/pmc_traffic.py <pmc_dir> <steps_per_pass> [frames_per_step bench.json] > profiles/r02_traffic.json

With frames_per_step and the bench line of the same tree, it also writes
per_frame {traffic_bytes, valu_insts, valu_frac}: valu_frac = SQ_INSTS_VALU of the
stage / (1024 SIMDs x 0.5 wave-instr/cycle x 2.4 GHz x the stage's HIP-event time),
the VALU-issue fraction (MI355X_MICROARCH.md: a wave64 VALU op issues over 2 cycles).
"""
import collections
import csv
import glob
import json
import os
import re
import sys

STAGES = [("pyramid", r"k_resize_|k_pyramid|k_blur7<true>"), ("blur7", r"k_blur7"), ("fast9_cells", r"k_fast_cells"),
          ("octree", r"k_octree"), ("orient_rbrief", r"k_orient_desc"), ("hamming_best2", r"k_hamming_best2"),
          ("sparse_align", r"k_sparse_align|k_build_align_jobs")]


def stage_of(kernel):
    for name, pat in STAGES:
        if re.search(pat, kernel):
            return name
    return None


VALU_ISSUE_PER_S = 1024 * 0.5 * 2.4e9


def main(pmc_dir, steps, frames=None, bench=None):
    tot = collections.defaultdict(lambda: collections.defaultdict(float))
    for path in glob.glob(os.path.join(pmc_dir, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(path)):
            st = stage_of(r["Kernel_Name"])
            if st and r["Counter_Name"] in ("FETCH_SIZE", "WRITE_SIZE", "SQ_INSTS_VALU", "SQ_WAVE_CYCLES",
                                            "SQ_WAIT_INST_ANY", "SQ_WAIT_ANY", "SQ_INSTS_LDS",
                                            "SQ_LDS_BANK_CONFLICT"):
                tot[st][r["Counter_Name"]] += float(r["Counter_Value"])
    out = {}
    for st, c in tot.items():
        fetch = c["FETCH_SIZE"] * 1024 * 2 / steps
        write = c["WRITE_SIZE"] * 1024 / steps
        out[st] = {"fetch_bytes": int(fetch), "write_bytes": int(write), "traffic_bytes": int(fetch + write),
                   "valu_insts": int(c["SQ_INSTS_VALU"] / steps)}
        if c["SQ_WAVE_CYCLES"] > 0:  # the p1 / p2 passes: latency and LDS figures of the stage
            out[st]["wait_inst_frac"] = round(c["SQ_WAIT_INST_ANY"] / c["SQ_WAVE_CYCLES"], 4)
            out[st]["wait_any_frac"] = round(c["SQ_WAIT_ANY"] / c["SQ_WAVE_CYCLES"], 4)
        if c["SQ_INSTS_LDS"] > 0:
            out[st]["lds_conflict_per_inst"] = round(c["SQ_LDS_BANK_CONFLICT"] / c["SQ_INSTS_LDS"], 3)
    res = {"source": pmc_dir, "steps_per_pass": steps,
           "correction": "FETCH_SIZE x2 (gfx950), KiB -> B", "per_step": out}
    if frames:
        stage_ms = json.load(open(bench))["roofline"]["stages_ms"] if bench else {}
        fb = frames  # stages_ms are per step (the sum over a step's chunk launches): frames per step
        pf = {}
        for st, v in out.items():
            d = {"traffic_bytes": v["traffic_bytes"] / frames, "valu_insts": v["valu_insts"] / frames}
            for k in ("wait_inst_frac", "wait_any_frac", "lds_conflict_per_inst"):
                if k in v:
                    d[k] = v[k]
            if stage_ms.get(st):
                d["valu_frac"] = round(d["valu_insts"] * fb / (VALU_ISSUE_PER_S * stage_ms[st] * 1e-3), 4)
            pf[st] = d
        res["frames_per_step"] = frames
        res["per_frame"] = pf
    json.dump(res, sys.stdout, indent=1)
    print()


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]), *(
        [int(sys.argv[3]), sys.argv[4]] if len(sys.argv) > 4 else []))
