"""Workgroup timeline of one instrumented kernel (diagnostic build, YGZ_BSTAMP):
dispatch spread, per-block durations, active blocks over time, blocks per XCC.
Runs one bench-shaped batch extract through lib/libygzfe_diag.so."""
import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "orb-ygz-slam_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import ygzfe  # noqa: E402

ygzfe.LIB_PATH = os.environ.get("YGZ_DIAG_LIB", os.path.join(ROOT, "orb-ygz-slam_amd", "lib", "libygzfe_diag.so"))
import _scenes as S  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 256
nblocks = int(sys.argv[2]) if len(sys.argv) > 2 else 0
W, H, nf, sf, nl, ini, mn = S.CONFIGS["C2"]
sc = S.PlaneScene(11, W, H)
xi = np.array([0.012, -0.006, 0.009, 0.0025, -0.002, 0.0015], np.float32)
sys.path.insert(0, ROOT)
from bench import sweep_index  # noqa: E402  (the bench's back-and-forth trajectory: full views at any B)
frames = np.stack([sc.render(*ygzfe.trajectory_pose(sweep_index(i), xi), noise_seed=i) for i in range(B)])
b = ygzfe.Batch((nf, sf, nl, ini, mn, 0), 0, W, H, B)
b.upload(frames)
for _ in range(3):
    b.extract(B)
b.check()
buf = np.zeros(8 * (1 << 17), np.uint64)
L = ygzfe.lib()
L.ygzfe_diag_block_stamps(buf.ctypes.data_as(C.c_void_p), len(buf))
st = buf.reshape(-1, 8)
valid = (st[:, 0] > 0) & (st[:, 1] > st[:, 0])
st = st[valid]
t0 = st[:, 0].min()
start = (st[:, 0] - t0) / 100.0  # us (100 MHz)
end = (st[:, 1] - t0) / 100.0
dur = end - start
print(f"blocks {len(st)}  span {end.max():.1f} us  first-dispatch spread {start.max():.1f} us")
print("block duration us: p10 %.1f p50 %.1f p90 %.1f max %.1f" % tuple(np.percentile(dur, [10, 50, 90, 100])))
tt = np.linspace(0, end.max(), 21)
act = [int(((start <= t) & (end > t)).sum()) for t in tt]
print("active blocks over time:", act)
xcc = st[:, 2] & 0xF
print("blocks per XCC:", np.bincount(xcc.astype(int), minlength=8).tolist())
kern = os.environ.get("STAMPK", "1")
names = ({3: "entry->before loads", 4: "window loads landed (+LDS store)", 5: "IC done", 6: "trig done",
          7: "descriptor done", 1: "end"} if kern == "1" else
         {3: "ROI staged", 4: "A: 4-point test", 5: "B: segment test", 6: "C: scores",
          7: "D: NMS (+retry)", 1: "end"} if kern == "2" else
         {3: "gather keys", 4: "codes + radix sort", 7: "(until the list kernel starts)",
          5: "L, histograms, list", 6: "final rounds", 1: "retain + end"} if kern == "3" else
         {3: "entry .. before the passes", 4: "pass 1", 5: "pass 2", 6: "pass 3", 7: "pass 4",
          1: "later passes + retain + end"})
prev = st[:, 0]
order = (3, 4, 7, 5, 6, 1) if kern == "3" else (3, 4, 5, 6, 7, 1)
if os.environ.get("YGZ_DIAG_ORDER"):  # a build whose stamps sit elsewhere: "slot:name,slot:name,..."
    pairs = [x.split(":", 1) for x in os.environ["YGZ_DIAG_ORDER"].split(",")]
    order = tuple(int(a) for a, _ in pairs)
    names = {int(a): b for a, b in pairs}
for k in order:
    if k not in names:
        continue
    ok = st[:, k] > 0
    d = (st[ok, k].astype(np.int64) - prev[ok].astype(np.int64)) / 100.0
    print(f"  phase -> {names[k]:34s}: p50 {np.median(d):6.2f} us  p90 {np.percentile(d, 90):6.2f} us")
    prev = np.where(ok, st[:, k], prev)
