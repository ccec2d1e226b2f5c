"""The N>1 path on CPU: world_size-2 `gloo` process groups exercising the same
host orchestration the GPU ranks use (ygzfe/dist.py): contiguous frame shards
with the one-frame align halo, max-over-ranks timing, and the offline gather of
fixed-size per-frame result slots to rank 0."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import ygzfe
from ygzfe import dist as D


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_shards_cover_sequence_once():
    for n in (0, 1, 7, 256, 13728):
        for world in (1, 2, 3, 8):
            spans = [D.shard(n, r, world) for r in range(world)]
            assert spans[0][0] == 0 and spans[-1][1] == n
            assert all(spans[r][1] == spans[r + 1][0] for r in range(world - 1))
            lens = [e - b for b, e in spans]
            assert max(lens) - min(lens) <= 1
            pairs = [p for b, e in spans for p in D.align_pairs(b, e)]
            assert pairs == [(k - 1, k) for k in range(1, n)]  # every pair exactly once
            for b, e in spans:
                hb, he = D.with_halo(b, e)
                assert all(hb <= r and c < he for r, c in D.align_pairs(b, e))


def test_c5_partition():
    """13 728 frames over 8 ranks: 1716 each."""
    assert [D.shard(13728, r, 8)[1] - D.shard(13728, r, 8)[0] for r in range(8)] == [1716] * 8


def fake_results(frames, cap):
    """Deterministic per-frame payloads standing in for GPU extraction output."""
    F = len(frames)
    counts = np.array([(g * 37) % (cap + 1) for g in frames], np.int32)
    kps = np.zeros((F, cap), ygzfe.KP_DTYPE)
    desc = np.zeros((F, cap, 32), np.uint8)
    align = np.zeros(F, [("q", "<f4", 4), ("t", "<f4", 3), ("n_visible", "<i4"), ("chi2", "<f4")])
    for i, g in enumerate(frames):
        kps["x"][i] = np.arange(cap) + g
        kps["octave"][i] = g % 4
        desc[i] = (np.arange(cap * 32).reshape(cap, 32) + g) % 251
        align["q"][i] = (0, 0, 0, 1)
        align["t"][i] = (g, -g, 0.5)
        align["n_visible"][i] = g % 100
    return counts, kps, desc, align


def _worker(rank, world, port, n_frames, cap, ret):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    b, e = D.shard(n_frames, rank, world)
    counts, kps, desc, align = fake_results(list(range(b, e)), cap)
    slots = torch.from_numpy(D.pack_slots(counts, kps, desc, align, global_first=b))
    full = D.gather_slots(slots, n_frames, rank, world)
    t = D.max_over_ranks(1.0 + rank)
    if rank == 0:
        ret["full"] = full.numpy()
        ret["t"] = t
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("n_frames", [9, 16])
def test_gloo_world2_gather_and_timing(n_frames):
    cap = 5
    mgr = mp.Manager()
    ret = mgr.dict()
    mp.spawn(_worker, args=(2, free_port(), n_frames, cap, ret), nprocs=2, join=True)
    full = ret["full"]
    assert ret["t"] == 2.0  # the slowest rank's time
    assert full.shape == (n_frames, D.slot_bytes(cap))
    counts, kps, desc, align = fake_results(list(range(n_frames)), cap)
    assert np.array_equal(full, D.pack_slots(counts, kps, desc, align))
    s = D.unpack_slot(full[7], cap, ygzfe.KP_DTYPE)
    assert s["n"] == counts[7] and np.array_equal(s["kps"], kps[7][:counts[7]])
    assert np.allclose(s["t"], (7, -7, 0.5)) and s["frame"] == 7 and s["has_align"]
    assert not D.unpack_slot(full[0], cap, ygzfe.KP_DTYPE)["has_align"]


def _chunk_worker(rank, world, port, n_frames, cap, n_chunks, ret):
    """bench.py's chunked schedule on CPU: the shard processed in n_chunks batches (each
    with the frame before it, for its first align pair); chunk c's slots packed into
    rows [c R, c R + own) and gathered to rank 0 before chunk c + 1 is processed."""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    b, e = D.shard(n_frames, rank, world)
    hb, he = D.with_halo(b, e)
    h, n_own = b - hb, e - b
    maxlen, R = D.chunk_rows(n_frames, world, n_chunks)
    S = D.slot_bytes(cap)
    pad = torch.zeros((n_chunks * R, S), dtype=torch.uint8)
    bufs, covered = [], []
    for c in range(n_chunks):
        s0, e0, hc, nc = D.chunk_frames(n_own, h, c, R)
        if nc > 0:
            frames = list(range(hb + s0 + hc, hb + s0 + hc + nc))  # global frames this chunk owns
            covered += frames
            counts, kps, desc, align = fake_results(frames, cap)
            pad[c * R:c * R + nc] = torch.from_numpy(D.pack_slots(counts, kps, desc, align, global_first=frames[0]))
            assert s0 + hc - 1 >= 0 or frames[0] == 0  # the pair (first - 1, first) is inside the batch
        cb = [torch.empty((R, S), dtype=torch.uint8) for _ in range(world)] if rank == 0 else None
        dist.gather(pad[c * R:(c + 1) * R], cb, dst=0)
        bufs.append(cb)
    assert covered == list(range(b, e))
    via_helper = D.gather_slots_chunked(pad[:n_own], n_frames, rank, world, n_chunks)
    if rank == 0:
        ret["full"] = D.assemble_chunks(bufs, n_frames, world).numpy()
        ret["helper"] = via_helper.numpy()
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,n_frames,n_chunks", [(2, 16, 4), (2, 9, 3), (3, 17, 4), (2, 5, 4)])
def test_gloo_chunked_gather_equals_single_rank(world, n_frames, n_chunks):
    """The overlapped (chunked) gather of bench.py --gpus N: every frame lands once, in
    order, with its own slot, whatever the shard / chunk split (uneven shards, chunks
    longer than a shard, empty trailing chunks)."""
    cap = 5
    mgr = mp.Manager()
    ret = mgr.dict()
    mp.spawn(_chunk_worker, args=(world, free_port(), n_frames, cap, n_chunks, ret), nprocs=world, join=True)
    counts, kps, desc, align = fake_results(list(range(n_frames)), cap)
    want = D.pack_slots(counts, kps, desc, align)
    assert np.array_equal(ret["full"], want)
    assert np.array_equal(ret["helper"], want)


# ---------------------------------------------------------------- real extractor output
# The C5 pipeline per rank (bench.py): extract the shard plus its one-frame halo,
# align every pair (k-1, k) of the shard, pack the slots, gather to rank 0 -- here
# with the CPU oracle standing in for the HIP extractor, so the sharding, halo and
# gather logic is checked against one single-rank run of the same sequence.
SEQ = 5


def _sequence():
    import _scenes as S
    sc = S.PlaneScene(11)
    xi = np.array([0.012, -0.006, 0.009, 0.0025, -0.002, 0.0015], np.float32)
    poses = [ygzfe.trajectory_pose(g, xi) for g in range(SEQ)]
    return sc, poses


def _rank_slots(frames, first, sc, poses, cap):
    """Oracle extraction of global frames [first, first + len(frames)) plus SparseImgAlign of
    each consecutive pair; returns the slots of frames[1:] if first > 0 (halo), else all."""
    import _oracle as O
    import _scenes as S
    orc = O.OrbOracle(1000, 2.0, 4, 20, 7)
    cam = O.Cam(*sc.cam)
    F = len(frames)
    kps = np.zeros((F, cap), ygzfe.KP_DTYPE)
    desc = np.zeros((F, cap, 32), np.uint8)
    counts = np.zeros(F, np.int32)
    align = np.zeros(F, D.ALIGN_DTYPE)
    levels = []
    for i, g in enumerate(frames):
        lv = orc.pyramid(sc.render(*poses[g], noise_seed=g))
        k, d = orc.extract(lv)
        counts[i] = len(k)
        kps[i, :len(k)] = k
        desc[i, :len(k)] = d
        levels.append(lv)
        if i > 0:
            Pw, ok = sc.map_points(*poses[g - 1], kps[i - 1, :counts[i - 1]])
            T0 = O.se3_from((0, 0, 0, 1), (0, 0, 0))
            r = O.sparse_align(levels[i - 1], lv, orc.inv_scale, cam, kps[i - 1, :counts[i - 1]],
                               S.world_to_cam(poses[g - 1], Pw), ok, 3, 1, T0)
            align[i] = (tuple(r.T.q), tuple(r.T.t), r.n_visible, r.chi2)
    h = 1 if first > 0 else 0
    return D.pack_slots(counts[h:], kps[h:], desc[h:], align[h:], global_first=first + h,
                        has_align=np.arange(h, F) + first >= 1)


def _real_worker(rank, world, port, cap, ret):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    sc, poses = _sequence()
    b, e = D.shard(SEQ, rank, world)
    hb, he = D.with_halo(b, e)
    slots = torch.from_numpy(_rank_slots(list(range(hb, he)), hb, sc, poses, cap))
    full = D.gather_slots(slots, SEQ, rank, world)
    if rank == 0:
        ret["full"] = full.numpy()
    dist.barrier()
    dist.destroy_process_group()


def test_gloo_world2_gather_real_extraction_equals_single_rank():
    cap = 1100
    sc, poses = _sequence()
    single = _rank_slots(list(range(SEQ)), 0, sc, poses, cap)
    mgr = mp.Manager()
    ret = mgr.dict()
    mp.spawn(_real_worker, args=(2, free_port(), cap, ret), nprocs=2, join=True)
    full = ret["full"]
    assert full.shape == single.shape
    assert np.array_equal(full, single)
    # every frame but the first carries its align record (the halo pair included)
    hdr = [D.unpack_slot(full[g], cap, ygzfe.KP_DTYPE) for g in range(SEQ)]
    assert [h["has_align"] for h in hdr] == [False] + [True] * (SEQ - 1)
    assert all(h["n"] > 300 for h in hdr) and all(h["n_visible"] > 100 for h in hdr[1:])


# ---------------------------------------------------------------- bench.py --gpus N contract
def _bench(args, env_extra=None):
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        env.pop(k, None)
    env.update(env_extra or {})
    return subprocess.run([sys.executable, os.path.join(root, "bench.py")] + args, capture_output=True, text=True,
                          timeout=120, env=env)


def test_bench_refuses_more_gpus_than_visible():
    """--gpus 2 with fewer visible GPUs fails loudly (never a silent n_gpus: 1 line)."""
    import torch
    if torch.cuda.device_count() >= 2:
        pytest.skip("two GPUs visible")
    r = _bench(["--gpus", "2", "--steps", "1"])
    assert r.returncode != 0
    assert "--gpus 2 needs 2 visible GPUs" in r.stderr
    assert '"n_gpus"' not in r.stdout


def test_bench_world_size_must_match_gpus():
    r = _bench(["--gpus", "2", "--steps", "1"], {"WORLD_SIZE": "1", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode != 0 and "WORLD_SIZE=1 but --gpus 2" in r.stderr
