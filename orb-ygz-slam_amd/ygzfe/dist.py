"""Frame sharding across GPUs: one process per GPU, contiguous
slices of the sequence, no data-path collective.

  * extraction is independent per frame;
  * SparseImgAlign needs (k-1, k) pairs, so a rank whose slice starts at
    frame b > 0 also extracts frame b-1 (a one-frame halo) and aligns every
    pair inside [b-1, e);
  * results are fixed-size per-frame slots packed on the device; the offline
    sequence mode (C5) gathers them to rank 0 in every step (point-to-point into
    the root: `torch.distributed.gather`, which RCCL implements with grouped
    send/recv over the xGMI peer links).  That gather is the only data-path
    collective; the timed region is bracketed by barriers and the elapsed time
    is the max over ranks.

Everything here is host-side orchestration on top of torch.distributed; it
runs the same with the "nccl" (RCCL) backend on GPUs and "gloo" in CPU tests.
"""
import numpy as np

# slot layout per frame (include/ygzfe.h YGZFE_SLOT_*, packed on the device by
# ygzfe_batch_pack_slots; this numpy form is the reference the tests compare):
#   [0, 64)  int32 n_kps, int32 n_visible, float32 T_cur_prev q[4] t[3], float32 chi2,
#            int32 global frame index, int32 has_align, 4 x 0
#   kps [cap x 28 B] (cv::KeyPoint layout), desc [cap x 32 B]; rows >= n_kps zero;
#   zero padding to a multiple of 16 B
SLOT_HEADER = 64


def slot_bytes(cap):
    return (SLOT_HEADER + cap * (28 + 32) + 15) // 16 * 16


def shard(n_frames, rank, world):
    """Contiguous split of [0, n_frames): the first n % world ranks get one extra frame."""
    if world <= 0 or not 0 <= rank < world:
        raise ValueError(f"bad rank {rank} / world {world}")
    base, rem = divmod(n_frames, world)
    begin = rank * base + min(rank, rem)
    return begin, begin + base + (1 if rank < rem else 0)


def with_halo(begin, end):
    """Frames a rank must extract to align every pair (k-1, k), k in [begin, end)."""
    return (begin - 1 if begin > 0 else begin), end


def align_pairs(begin, end):
    """(ref, cur) global frame pairs owned by the shard [begin, end)."""
    return [(k - 1, k) for k in range(max(begin, 1), end)]


ALIGN_DTYPE = np.dtype([("q", "<f4", 4), ("t", "<f4", 3), ("n_visible", "<i4"), ("chi2", "<f4")])


def pack_slots(counts, kps, desc, align=None, global_first=0, has_align=None):
    """Per-frame slots (uint8 [F, slot_bytes(cap)]) from numpy results.

    counts [F] int, kps [F, cap] structured (28 B), desc [F, cap, 32] uint8,
    align: optional [F] ALIGN_DTYPE records (frame k's pose relative to k-1);
    has_align [F] bool (default: every frame but global frame 0 when align is given)."""
    F, cap = kps.shape[0], kps.shape[1]
    out = np.zeros((F, slot_bytes(cap)), np.uint8)
    hdr = np.zeros((F, 16), np.float32)
    hdr_i = hdr.view(np.int32)
    counts = np.asarray(counts, np.int32)
    hdr_i[:, 0] = counts
    hdr[:, 5] = 1.0  # identity q when there is no align record
    gidx = global_first + np.arange(F)
    hdr_i[:, 10] = gidx
    if align is not None:
        has = (gidx >= 1) if has_align is None else np.asarray(has_align, bool)
        hdr_i[has, 1] = align["n_visible"][has]
        hdr[has, 2:6] = align["q"][has]
        hdr[has, 6:9] = align["t"][has]
        hdr[has, 9] = align["chi2"][has]
        hdr_i[has, 11] = 1
    out[:, :SLOT_HEADER] = hdr.view(np.uint8).reshape(F, SLOT_HEADER)
    kb = np.ascontiguousarray(kps).view(np.uint8).reshape(F, cap, 28).copy()
    db = np.ascontiguousarray(desc, np.uint8).reshape(F, cap, 32).copy()
    rows = np.arange(cap)[None, :] >= counts[:, None]
    kb[rows] = 0
    db[rows] = 0
    out[:, SLOT_HEADER:SLOT_HEADER + cap * 28] = kb.reshape(F, cap * 28)
    out[:, SLOT_HEADER + cap * 28:SLOT_HEADER + cap * 60] = db.reshape(F, cap * 32)
    return out


def unpack_slot(slot, cap, kp_dtype):
    hdr = slot[:SLOT_HEADER].view(np.float32)
    hi = hdr.view(np.int32)
    n = int(hi[0])
    kps = slot[SLOT_HEADER:SLOT_HEADER + cap * 28].view(kp_dtype)[:n]
    desc = slot[SLOT_HEADER + cap * 28:SLOT_HEADER + cap * 60].reshape(cap, 32)[:n]
    return {"n": n, "n_visible": int(hi[1]), "q": hdr[2:6].copy(), "t": hdr[6:9].copy(), "chi2": float(hdr[9]),
            "frame": int(hi[10]), "has_align": bool(hi[11]), "kps": kps, "desc": desc}


def gather_slots(local_slots, n_frames, rank, world, device=None):
    """Gather every rank's [end-begin, S] uint8 slot tensor into [n_frames, S] on rank 0.

    Shards differ by at most one frame; each rank pads to the largest shard so a
    single gather moves everything (rank 0 returns the tensor, others None)."""
    import torch
    import torch.distributed as dist
    S = local_slots.shape[1]
    maxlen = -(-n_frames // world)
    pad = torch.zeros((maxlen, S), dtype=torch.uint8, device=device or local_slots.device)
    pad[:local_slots.shape[0]] = local_slots
    bufs = [torch.empty_like(pad) for _ in range(world)] if rank == 0 else None
    dist.gather(pad, bufs, dst=0)
    if rank != 0:
        return None
    parts = []
    for r in range(world):
        b, e = shard(n_frames, r, world)
        parts.append(bufs[r][:e - b])
    return torch.cat(parts, 0)


def chunk_rows(n_frames, world, n_chunks):
    """Row layout of the chunked gather: every rank pads its shard to maxlen =
    ceil(n_frames / world) slot rows, cut into n_chunks pieces of R rows (the last may
    run past maxlen: those rows are padding).  Chunk c of every rank is rows
    [c R, (c + 1) R); the same R on every rank keeps each chunk's gather uniform."""
    maxlen = -(-n_frames // world)
    R = -(-maxlen // max(1, n_chunks))
    return maxlen, R


def chunk_frames(n_own, h, c, R):
    """Local frames of chunk c of a rank owning n_own frames from local index h: the
    batch range [s, e) (the frame before the chunk included, for its first align pair),
    the own frames' offset in that range, and how many there are."""
    a = h + min(c * R, n_own)
    e = h + min((c + 1) * R, n_own)
    s = a - 1 if a > 0 else a
    return s, e, a - s, e - a


def assemble_chunks(chunk_bufs, n_frames, world):
    """Rank 0: chunk_bufs[c][r] = rank r's rows of chunk c -> [n_frames, S] in global
    frame order (each rank's rows concatenated over chunks, cut to its shard)."""
    import torch
    parts = []
    for r in range(world):
        b, e = shard(n_frames, r, world)
        parts.append(torch.cat([cb[r] for cb in chunk_bufs], 0)[:e - b])
    return torch.cat(parts, 0)


def gather_slots_chunked(local_slots, n_frames, rank, world, n_chunks, device=None):
    """gather_slots as n_chunks gathers of R rows each (the bench issues each one on
    a communication stream as soon as its chunk is packed, overlapping the next
    chunk's compute).  Returns [n_frames, S] on rank 0, None elsewhere."""
    import torch
    import torch.distributed as dist
    S = local_slots.shape[1]
    maxlen, R = chunk_rows(n_frames, world, n_chunks)
    pad = torch.zeros((n_chunks * R, S), dtype=torch.uint8, device=device or local_slots.device)
    pad[:local_slots.shape[0]] = local_slots
    bufs = []
    for c in range(n_chunks):
        cb = [torch.empty((R, S), dtype=torch.uint8, device=pad.device) for _ in range(world)] if rank == 0 else None
        dist.gather(pad[c * R:(c + 1) * R], cb, dst=0)
        bufs.append(cb)
    return assemble_chunks(bufs, n_frames, world) if rank == 0 else None


def max_over_ranks(seconds, device=None):
    """The bench's wall time: the slowest rank's (all_reduce MAX of one float64)."""
    import torch
    import torch.distributed as dist
    if not dist.is_initialized() or dist.get_world_size() == 1:
        return float(seconds)
    t = torch.tensor([seconds], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())
