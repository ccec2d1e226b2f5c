"""BASELINE config C5 on the GPU: the bench's offline-sequence path (ygzfe.sequence.C5Shard,
the object bench.py times) over the whole 13,728-frame EuRoC MH01..05-length sequence.

* unsharded at N = 1: every frame's result slot (keypoints, descriptors, SparseImgAlign
  record of the pair (k-1, k)) packed on the device;
* as 8 virtual shards on this one GPU, each with its one-frame halo (ygzfe.dist.shard /
  with_halo), one batch per shard and again in the 4-chunk schedule the bench uses for
  N > 1: the concatenated slots must equal the unsharded run's byte for byte;
* the frames either side of every shard boundary (1715/1716, 3431/3432, ..., 13727) against
  the oracle (ORBextractor C2, bit-exact), and every halo align pair (b-1 -> b) against the
  oracle's SparseImgAlign (pose within 1e-4, same visible count);
* every 16th frame against the oracle's extraction and every 64th align pair against its
  SparseImgAlign (858 frames, 215 pairs);
* the overlap / split / tail / pipe stream schedules (bench.py times `pipe` with 4 chunks by default;
  its roofline stage times come from a separate serial pass) equal serial;
* a world-size-1 RCCL process group ("nccl" = RCCL, device_id bound): the device-packed
  slots gathered to rank 0 with torch.distributed.gather (one batch and chunked) equal the
  local slots.
"""
import socket

import numpy as np
import pytest
import torch

import _oracle as O
import _scenes as S
import ygzfe
from ygzfe import dist as D
from ygzfe.sequence import C5_FRAMES, C5Shard

pytestmark = pytest.mark.gpu
POSE_TOL = 1e-4
WORLD = 8


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _run(shard):
    shard.step()
    torch.cuda.synchronize()
    shard.check()
    return shard


@pytest.fixture(scope="module")
def c5_full(gpu):
    dev = torch.device("cuda", 0)
    sh = _run(C5Shard(C5_FRAMES, 0, 1, dev))
    assert sh.F == C5_FRAMES and sh.P == C5_FRAMES - 1
    yield sh
    del sh
    torch.cuda.empty_cache()


def _boundaries():
    bs = []
    for r in range(1, WORLD):
        b0, _ = D.shard(C5_FRAMES, r, WORLD)
        bs.append(b0)
    return bs


def test_c5_full_sequence_slots(c5_full):
    sh = c5_full
    slots = sh.local_slots()
    assert slots.shape[0] == C5_FRAMES
    hdr = slots[:, :64].contiguous().view(torch.int32).cpu().numpy()
    assert np.array_equal(hdr[:, 10], np.arange(C5_FRAMES))  # global frame index
    assert hdr[0, 11] == 0 and (hdr[1:, 11] == 1).all()       # every frame after the first has its align record
    assert (hdr[:, 0] > 500).all() and (hdr[:, 0] <= 1000).all()
    assert (hdr[1:, 1] > 100).all()                            # visible features of every align


@pytest.mark.parametrize("chunks", [1, 4])
def test_c5_virtual_shards_equal_unsharded(c5_full, chunks):
    """8 shards (+ halo) one after another on this GPU == the unsharded run, byte for byte."""
    full = c5_full.local_slots()
    dev = full.device
    covered = 0
    for r in range(WORLD):
        sh = _run(C5Shard(C5_FRAMES, r, WORLD, dev, chunks=chunks, gather=False))
        b0, e0 = D.shard(C5_FRAMES, r, WORLD)
        assert (sh.b0, sh.e0) == (b0, e0) and sh.F == (e0 - b0) + (1 if r > 0 else 0)
        loc = sh.local_slots()
        assert loc.shape[0] == e0 - b0
        if not torch.equal(loc, full[b0:e0]):
            bad = (loc != full[b0:e0]).any(1).nonzero().flatten().cpu().numpy()
            pytest.fail(f"shard {r} (chunks {chunks}): {len(bad)} frames differ from the unsharded run, "
                        f"first global frames {(bad[:8] + b0).tolist()}")
        covered += e0 - b0
        del sh, loc
        torch.cuda.empty_cache()
    assert covered == C5_FRAMES


def test_c5_shard_boundaries_vs_oracle(c5_full):
    """Frames either side of each shard boundary (and the last frame) against the oracle's
    extraction; each halo pair's SparseImgAlign against the oracle's."""
    sh = c5_full
    W, H, nf, sf, nl, ini, mn = S.CONFIGS["C2"]
    orc = O.OrbOracle(nf, sf, nl, ini, mn)
    slots = sh.local_slots()
    cap = sh.cap
    bounds = _boundaries()
    frames = sorted({g for b in bounds for g in (b - 1, b)} | {0, C5_FRAMES - 1})
    pyr = {}
    for g in frames:
        img = sh.batch.read_level(g, 0)
        pyr[g] = orc.pyramid(img)
        got = D.unpack_slot(slots[g].cpu().numpy(), cap, ygzfe.KP_DTYPE)
        assert got["frame"] == g
        rk, rd = orc.extract(pyr[g])
        assert got["n"] == len(rk), f"frame {g}: {got['n']} keypoints vs oracle {len(rk)}"
        for f in rk.dtype.names:
            assert np.array_equal(got["kps"][f], rk[f]), f"frame {g}: keypoint field {f} differs"
        assert np.array_equal(got["desc"], rd), f"frame {g}: descriptors differ"
    # halo pairs (b-1 -> b): the rank owning b aligns them from its halo frame
    xyz = sh.xyz
    ocam = O.Cam(*sh.cam)
    T0 = O.se3_from((0, 0, 0, 1), (0, 0, 0))
    for b in bounds:
        ref = D.unpack_slot(slots[b - 1].cpu().numpy(), cap, ygzfe.KP_DTYPE)
        cur = D.unpack_slot(slots[b].cpu().numpy(), cap, ygzfe.KP_DTYPE)
        n = ref["n"]
        x = xyz[b - 1, :n].cpu().numpy()
        o = O.sparse_align(pyr[b - 1], pyr[b], orc.inv_scale, ocam, ref["kps"], x, np.ones(n, np.uint8), 3, 1, T0)
        assert cur["has_align"]
        err = S.se3_log_inf(cur["q"], cur["t"], np.array(o.T.q[:]), np.array(o.T.t[:]))
        assert err <= POSE_TOL, f"halo pair ({b - 1}, {b}): pose differs by {err}"
        assert cur["n_visible"] == o.n_visible, f"halo pair ({b - 1}, {b}): n_visible {cur['n_visible']} vs " \
                                                f"{o.n_visible}"


def test_c5_sampled_frames_and_pairs_vs_oracle(c5_full):
    """Beyond the shard boundaries: every 16th frame's keypoints and descriptors (858 frames)
    against the oracle's extraction (ORBextractor C2, bit-exact) and every 64th align pair
    (215 pairs) against the oracle's SparseImgAlign (pose within 1e-4, same visible count)."""
    sh = c5_full
    W, H, nf, sf, nl, ini, mn = S.CONFIGS["C2"]
    orc = O.OrbOracle(nf, sf, nl, ini, mn)
    slots = sh.local_slots().cpu().numpy()
    cap = sh.cap
    pyr = {}

    def pyramid(g):
        if g not in pyr:
            pyr[g] = orc.pyramid(sh.batch.read_level(g, 0))
        return pyr[g]

    frames = list(range(0, C5_FRAMES, 16))
    bad = []
    for g in frames:
        got = D.unpack_slot(slots[g], cap, ygzfe.KP_DTYPE)
        rk, rd = orc.extract(pyramid(g))
        same = got["frame"] == g and got["n"] == len(rk) and np.array_equal(got["desc"], rd) and \
            all(np.array_equal(got["kps"][f], rk[f]) for f in rk.dtype.names)
        if not same:
            bad.append(g)
    assert not bad, f"{len(bad)} of {len(frames)} sampled frames differ from the oracle, first {bad[:8]}"
    xyz = sh.xyz
    ocam = O.Cam(*sh.cam)
    T0 = O.se3_from((0, 0, 0, 1), (0, 0, 0))
    pairs = list(range(1, C5_FRAMES, 64))
    worst = 0.0
    for b in pairs:
        ref = D.unpack_slot(slots[b - 1], cap, ygzfe.KP_DTYPE)
        cur = D.unpack_slot(slots[b], cap, ygzfe.KP_DTYPE)
        n = ref["n"]
        x = xyz[b - 1, :n].cpu().numpy()
        o = O.sparse_align(pyramid(b - 1), pyramid(b), orc.inv_scale, ocam, ref["kps"], x, np.ones(n, np.uint8), 3, 1,
                           T0)
        assert cur["has_align"]
        err = S.se3_log_inf(cur["q"], cur["t"], np.array(o.T.q[:]), np.array(o.T.t[:]))
        worst = max(worst, err)
        assert err <= POSE_TOL, f"pair ({b - 1}, {b}): pose differs by {err}"
        assert cur["n_visible"] == o.n_visible, f"pair ({b - 1}, {b}): n_visible {cur['n_visible']} vs {o.n_visible}"
        pyr.pop(b - 1, None)
    print(f"C5 sample: {len(frames)} frames bit-exact, {len(pairs)} align pairs, worst |dT| {worst:.2e}")


@pytest.mark.parametrize("schedule,chunks", [("overlap", 1), ("split", 1), ("tail", 1), ("pipe", 2), ("pipe", 4)])
def test_c5_schedules_equal_serial(c5_full, schedule, chunks):
    """The stream schedules bench.py can time (the default `pipe` / 4 included) give the serial
    schedule's slots byte for byte: they reorder launches across streams, never the results.
    `pipe` runs chunk c + 1's extraction beside chunk c's descriptors and alignment (private
    per-chunk buffers); its align records must equal the unchunked run's too."""
    dev = torch.device("cuda", 0)
    sh = _run(C5Shard(C5_FRAMES, 0, 1, dev, chunks=chunks, schedule=schedule))
    assert torch.equal(sh.local_slots(), c5_full.local_slots())
    if schedule == "pipe":
        assert torch.equal(sh.counts(), c5_full.counts())
        sh.step()  # a second step reuses the chunk batches (the write-after-read edges)
        torch.cuda.synchronize()
        sh.check()
        assert torch.equal(sh.local_slots(), c5_full.local_slots())
    del sh
    torch.cuda.empty_cache()


def test_c5_rccl_gather_world1(c5_full):
    """torch.distributed over RCCL at world size 1 (the bench's N > 1 init, device_id bound):
    the device-packed slots gathered to rank 0 equal the local slots, one batch, chunked and
    under the pipe schedule (a chunk's gather beside the next chunks' work)."""
    import torch.distributed as dist
    if dist.is_initialized():
        pytest.skip("a process group is already initialised in this process")
    dev = torch.device("cuda", 0)
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{_free_port()}", rank=0, world_size=1,
                            device_id=dev)
    try:
        assert dist.get_backend() == "nccl"
        full = c5_full.local_slots()
        for chunks, schedule in ((1, "serial"), (4, "serial"), (4, "pipe")):
            sh = C5Shard(C5_FRAMES, 0, 1, dev, chunks=chunks, schedule=schedule, gather=True)
            sh.step(timed_gather=True)
            torch.cuda.synchronize()
            sh.check()
            root = sh.root_slots()
            assert root.shape[0] == C5_FRAMES
            assert torch.equal(root, sh.local_slots())
            assert torch.equal(root, full)
            assert len(sh.gather_ms) == chunks
            del sh, root
            torch.cuda.empty_cache()
    finally:
        dist.destroy_process_group()
