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
    slots = torch.from_numpy(D.pack_slots(counts, kps, desc, align))
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
    assert np.allclose(s["t"], (7, -7, 0.5))
