"""Microbenchmark: batched SparseImgAlign alone (no concurrent kernels) on the bench workload.
Extracts B frames of the bench's swept trajectory once, then times `reps` launches of
ygzfe_batch_sparse_align over the B-1 pairs with HIP events.  --diag loads the stamp build and
prints block 0's phase breakdown of the last launch."""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "orb-ygz-slam_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, ROOT)
ap = argparse.ArgumentParser()
ap.add_argument("--batch", type=int, default=1024)
ap.add_argument("--pairs", type=int, default=0, help="pairs per launch (0 = B-1)")
ap.add_argument("--reps", type=int, default=10)
ap.add_argument("--diag", action="store_true")
ap.add_argument("--save", default="", help="np.save the result records here")
args = ap.parse_args()
import ygzfe  # noqa: E402
if args.diag:
    ygzfe.LIB_PATH = os.path.join(ROOT, "orb-ygz-slam_amd", "lib", "libygzfe_diag.so")
import numpy as np  # noqa: E402
import torch  # noqa: E402
import _scenes as S  # noqa: E402
from bench import sweep_index  # noqa: E402

W, H, nf, sf, nl, ini, mn = S.CONFIGS["C2"]
B = args.batch
xi = np.array([0.012, -0.006, 0.009, 0.0025, -0.002, 0.0015], np.float32)
sc = S.PlaneScene(11, W, H)
poses = [ygzfe.trajectory_pose(sweep_index(i), xi) for i in range(B)]
frames = np.stack([sc.render(q, t, noise_seed=i) for i, (q, t) in enumerate(poses)])
batch = ygzfe.Batch((nf, sf, nl, ini, mn, 0), 0, W, H, B)
cap = batch.kp_cap
kps_t = torch.empty((B, cap, 7), dtype=torch.float32, device="cuda")
counts_t = torch.zeros(B, dtype=torch.int32, device="cuda")
batch.bind(kps=kps_t.data_ptr(), counts=counts_t.data_ptr())
batch.upload(frames)
stream = torch.cuda.Stream()
torch.cuda.set_stream(stream)
sptr = stream.cuda_stream
batch.extract(B, sptr)
P = args.pairs or (B - 1)
r3 = np.zeros((B, 3), np.float32)
cz = np.zeros(B, np.float32)
for i, (q, t) in enumerate(poses):
    qi, ti = S.se3_inv(q.astype(np.float64), t.astype(np.float64))
    r3[i] = np.array([S.quat_rot(qi, e) for e in np.eye(3)]).T[2]
    cz[i] = ti[2]
r3_t = torch.from_numpy(r3).cuda()
cz_t = torch.from_numpy(cz).cuda()
xyz = torch.empty((P, cap, 3), dtype=torch.float32, device="cuda")
usable = torch.ones((P, cap), dtype=torch.uint8, device="cuda")
ref_idx = torch.arange(0, P, dtype=torch.int32, device="cuda")
cur_idx = torch.arange(1, P + 1, dtype=torch.int32, device="cuda")
T0 = torch.zeros((P, 7), dtype=torch.float32, device="cuda")
T0[:, 3] = 1
out = torch.zeros((P, 45), dtype=torch.float32, device="cuda")
cam = ygzfe.Camera(*ygzfe.EUROC_CAM)
ygzfe.plane_points_device(kps_t.data_ptr(), cap, P, ygzfe.EUROC_CAM, r3_t.data_ptr(), cz_t.data_ptr(), S.PLANE_Z,
                          xyz.data_ptr(), sptr)
torch.cuda.synchronize()
ts = []
for r in range(args.reps):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    batch.sparse_align(P, ref_idx.data_ptr(), cur_idx.data_ptr(), xyz.data_ptr(), usable.data_ptr(), cam, 3, 1,
                       T0.data_ptr(), out.data_ptr(), sptr)
    e1.record(stream)
    torch.cuda.synchronize()
    ts.append(e0.elapsed_time(e1))
nvis = out[:, 7].contiguous().view(torch.int32).cpu().numpy()
print(f"pairs {P}  mean kps {counts_t.float().mean().item():.1f}  mean visible {nvis.mean():.1f}  "
      f"align ms: median {np.median(ts):.4f} min {min(ts):.4f}  ({P / np.median(ts) * 1e3:.0f} pairs/s)")
if args.save:
    np.save(args.save, out.cpu().numpy())
if args.diag:
    import ctypes as C
    buf = (C.c_ulonglong * 4096)()
    n = ygzfe.lib().ygzfe_diag_stamps(buf, 4096)
    st = [(buf[2 * i], buf[2 * i + 1]) for i in range(n)]
    tot, prev = {}, st[0][1]
    for tag, t in st:
        tot[tag] = tot.get(tag, 0) + (t - prev)
        prev = t
    print("block 0 stamps", n, "cycles", st[-1][1] - st[0][1], {k: v for k, v in sorted(tot.items())})
