"""Microbenchmark: batched dense Hamming best-2 (ygzfe_batch_match) alone, on synthetic descriptors.
B frames of `--n` random 256-bit descriptors each (bound into the batch's descriptor/count buffers),
B-1 pairs k vs k-1 per launch, timed with HIP events over `--reps` launches.  The MFMA floor printed
beside it is 8 v_mfma_i32_32x32x32_i8 (32 cycles each) per (32 queries x 32 train rows) tile per wave
(the i8 form's; the FP4 form issues half as many MFMAs of the same cycles, so its floor is half the printed one)."""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "orb-ygz-slam_amd"))
ap = argparse.ArgumentParser()
ap.add_argument("--batch", type=int, default=1024)
ap.add_argument("--n", type=int, nargs="+", default=[415])
ap.add_argument("--reps", type=int, default=20)
ap.add_argument("--check", action="store_true", help="compare a few pairs with a numpy brute force")
ap.add_argument("--real", action="store_true", help="descriptors/counts of the bench's extracted frames instead")
args = ap.parse_args()
import numpy as np  # noqa: E402
import torch  # noqa: E402
import ygzfe  # noqa: E402

B = args.batch
batch = ygzfe.Batch((1000, 2.0, 4, 20, 7, 0), 0, 752, 480, B)
cap = batch.kp_cap
desc = torch.randint(0, 256, (B, cap, 32), dtype=torch.uint8, device="cuda")
counts = torch.zeros(B, dtype=torch.int32, device="cuda")
batch.bind(desc=desc.data_ptr(), counts=counts.data_ptr())
P = B - 1
qf = torch.arange(1, B, dtype=torch.int32, device="cuda")
tf = torch.arange(0, B - 1, dtype=torch.int32, device="cuda")
bi = torch.empty((P, cap), dtype=torch.int32, device="cuda")
bd = torch.empty_like(bi)
sd = torch.empty_like(bi)
stream = torch.cuda.Stream()
torch.cuda.set_stream(stream)
sptr = stream.cuda_stream
if args.real:
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    sys.path.insert(0, ROOT)
    import _scenes as S
    from bench import sweep_index
    W, H, nf, sf, nl, ini, mn = S.CONFIGS["C2"]
    xi = np.array([0.012, -0.006, 0.009, 0.0025, -0.002, 0.0015], np.float32)
    sc = S.PlaneScene(11, W, H)
    poses = [ygzfe.trajectory_pose(sweep_index(i), xi) for i in range(B)]
    batch.upload(np.stack([sc.render(q, t, noise_seed=i) for i, (q, t) in enumerate(poses)]))
    batch.extract(B, sptr)
    torch.cuda.synchronize()
    c = counts.cpu().numpy()
    print(f"real counts: mean {c.mean():.1f} rms {np.sqrt((c.astype(float) ** 2).mean()):.1f} min {c.min()} "
          f"max {c.max()}", flush=True)
    args.n = [0]
for n in args.n:
    if not args.real:
        counts.fill_(min(n, cap))
    batch.match(P, qf.data_ptr(), tf.data_ptr(), bi.data_ptr(), bd.data_ptr(), sd.data_ptr(), sptr)
    torch.cuda.synchronize()
    ts = []
    for r in range(args.reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        batch.match(P, qf.data_ptr(), tf.data_ptr(), bi.data_ptr(), bd.data_ptr(), sd.data_ptr(), sptr)
        e1.record(stream)
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    nn = min(n, cap) if not args.real else int(counts.max().item())
    tiles = (nn + 31) // 32
    waves = P * ((nn + 31) // 32)
    floor_us = waves * tiles * 8 * 32 / 1024 / 2.4e3
    print(f"n {nn}: hamming ms median {np.median(ts):.4f} min {min(ts):.4f}  MFMA floor {floor_us / 1e3:.4f} ms "
          f"({P * nn * nn / np.median(ts) / 1e6:.1f} G pair-distances/s)", flush=True)
    if args.check:
        d = desc.cpu().numpy()
        pc = np.unpackbits(np.arange(256, dtype=np.uint8)[:, None], axis=1).sum(1)
        for p in (0, P // 2, P - 1):
            c = counts.cpu().numpy()
            q, t = d[p + 1, :c[p + 1]], d[p, :c[p]]
            D = pc[q[:, None, :] ^ t[None, :, :]].sum(2)
            o = np.concatenate([np.sort(D, axis=1), np.full((len(q), 2), 257)], axis=1)  # 257: no such row
            nq = len(q)
            assert (bd[p, :nq].cpu().numpy() == o[:, 0]).all() and (sd[p, :nq].cpu().numpy() == o[:, 1]).all(), p
        print("  check ok", flush=True)
