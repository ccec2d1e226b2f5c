"""Synthetic DBoW2 vocabularies (the reference's Vocabulary/ORBvoc.txt is absent:
.MISSING_LARGE_BLOBS).  Same structure as TemplatedVocabulary::create's output —
a k-ary tree of depth L, node 0 the root, children of a node contiguous, leaves
= words with an idf weight — and writers for both reference file formats
(saveToTextFile / saveToBinaryFile, TemplatedVocabulary.h:1452-1548)."""
import struct

import numpy as np


def synth_vocab(seed, k=10, L=3, flip_p=3, stop_frac=0.03, dup_frac=0.02):
    """Arrays (parent, is_leaf, desc[n,32], weight) in level (BFS) order.  A child's
    descriptor is its parent's with ~256/2^flip_p random bits flipped; a few children
    duplicate a sibling's descriptor (ties: the first wins); stop_frac of the words have
    weight 0 (stopped words)."""
    rng = np.random.default_rng(seed)
    parent = [np.zeros(1, np.int32)]
    desc = [rng.integers(0, 256, (1, 32), dtype=np.uint8)]
    level_start, n = 0, 1
    for lvl in range(L):
        cnt = k ** lvl
        pids = np.repeat(np.arange(level_start, level_start + cnt, dtype=np.int32), k)
        pd = desc[-1] if lvl > 0 else desc[0]
        base = np.repeat(pd, k, axis=0)
        mask = np.full(base.shape, 255, np.uint8)
        for _ in range(flip_p):
            mask &= rng.integers(0, 256, base.shape, dtype=np.uint8)
        cd = base ^ mask
        dup = np.where(rng.random(len(cd)) < dup_frac)[0]
        dup = dup[dup % k != 0]
        cd[dup] = cd[dup - 1]
        parent.append(pids)
        desc.append(cd)
        level_start, n = n, n + len(cd)
    parent = np.concatenate(parent)
    desc = np.concatenate(desc)
    is_leaf = np.zeros(n, np.uint8)
    is_leaf[n - k ** L:] = 1
    weight = np.zeros(n, np.float64)
    leaves = np.arange(n - k ** L, n)
    weight[leaves] = rng.uniform(0.05, 6.0, len(leaves))
    weight[leaves[rng.random(len(leaves)) < stop_frac]] = 0.0
    return parent, is_leaf, desc, weight


def write_text(path, k, L, scoring, weighting, parent, is_leaf, desc, weight):
    """saveToTextFile format (TemplatedVocabulary.h:1452-1475)."""
    with open(path, "w") as f:
        f.write(f"{k} {L}  {scoring} {weighting}\n")
        for i in range(1, len(parent)):
            d = " ".join(str(int(x)) for x in desc[i])
            f.write(f"{int(parent[i])} {int(is_leaf[i])} {d}  {float(weight[i])!r}\n")


def write_binary(path, k, L, scoring, weighting, parent, is_leaf, desc, weight):
    """saveToBinaryFile format (TemplatedVocabulary.h:1527-1548): 41-byte records."""
    with open(path, "wb") as f:
        f.write(struct.pack("<IIiiii", len(parent), 41, k, L, scoring, weighting))
        for i in range(1, len(parent)):
            f.write(struct.pack("<i", int(parent[i])) + bytes(desc[i]) + struct.pack("<f", float(weight[i])) +
                    bytes([int(is_leaf[i])]))
