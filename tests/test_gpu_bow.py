"""GPU DBoW2 transform vs the oracle.

Frame::ComputeBoW (Frame.cc:495-500) = TemplatedVocabulary::transform(desc,
mBowVec, mFeatVec, 4) (Thirdparty/DBoW2/DBoW2/TemplatedVocabulary.h:1150-1281).
The reference's Vocabulary/ORBvoc.txt is absent (.MISSING_LARGE_BLOBS), so the
vocabularies are synthetic trees of the same shape (tests/_vocab.py); word ids,
weights, FeatureVector nodes and BowVector values are compared bit-exactly.
"""
import numpy as np
import pytest

import _oracle as O
import _scenes as S
import _vocab as V

pytestmark = pytest.mark.gpu


def _features(gpu, seed, n_random=64):
    W, H, nf, sf, nl, ini, mn = S.CONFIGS["C2"]
    ex = gpu.ORBextractor(nf, sf, nl, ini, mn)
    _, d = ex.extract(ex.ComputePyramid(S.frame(seed, W, H)))
    rng = np.random.default_rng(seed)
    return np.concatenate([d, d[:17], rng.integers(0, 256, (n_random, 32), dtype=np.uint8)])


@pytest.mark.parametrize("k,L,levelsup", [(10, 4, 4), (10, 4, 2), (6, 5, 4), (3, 6, 0)])
def test_bow_transform_each_bitexact(gpu, k, L, levelsup):
    parent, is_leaf, desc, weight = V.synth_vocab(k * 10 + L, k, L)
    voc = gpu.Vocabulary.from_arrays(k, L, 0, 0, parent, is_leaf, desc, weight)
    assert voc.n_nodes == len(parent) and voc.n_words == int(is_leaf.sum())
    ovoc = O.Vocab(k, L, 0, 0, parent, is_leaf, desc, weight)
    f = _features(gpu, L)
    w, wt, nid = voc.transform_each(f, levelsup)
    ow, owt, onid = ovoc.transform_each(f, levelsup)
    assert np.array_equal(w, ow) and np.array_equal(wt, owt) and np.array_equal(nid, onid)
    assert len(np.unique(w)) > len(f) // 4


@pytest.mark.parametrize("scoring,weighting", [(0, 0), (1, 0), (2, 1), (5, 0), (5, 1), (0, 2), (5, 3)])
def test_compute_bow_bitexact(gpu, scoring, weighting):
    k, L = 10, 4
    parent, is_leaf, desc, weight = V.synth_vocab(7, k, L)
    voc = gpu.Vocabulary.from_arrays(k, L, scoring, weighting, parent, is_leaf, desc, weight)
    ovoc = O.Vocab(k, L, scoring, weighting, parent, is_leaf, desc, weight)
    f = _features(gpu, 3)
    (bw, bv), (fn, ff) = voc.transform(f, 4)
    (obw, obv), (ofn, off) = ovoc.transform(f, 4)
    assert np.array_equal(bw, obw) and np.array_equal(bv, obv)
    assert np.array_equal(fn, ofn) and np.array_equal(ff, off)
    assert len(bw) > 100
    if scoring != 5:
        assert abs((np.abs(bv).sum() if scoring != 1 else np.sqrt((bv ** 2).sum())) - 1.0) < 1e-12


@pytest.mark.parametrize("n_random,scoring", [(0, 0), (73, 1), (74, 0), (3000, 0), (3000, 1), (7000, 5)])
def test_compute_bow_sizes(gpu, n_random, scoring):
    """k_bow_vectors across its sort paths: <= 1,024 features (one key per thread, the
    register bitonic network), 1,025 and more (the LDS network, several keys and folded
    values per thread, up to 8 per thread at 8,192 slots); L1, L2 and DOT_PRODUCT.  The
    frame has 934 keypoints + 17 repeats, so n_random 73 / 74 make 1,024 / 1,025 features."""
    k, L = 10, 4
    parent, is_leaf, desc, weight = V.synth_vocab(9, k, L)
    voc = gpu.Vocabulary.from_arrays(k, L, scoring, 0, parent, is_leaf, desc, weight)
    ovoc = O.Vocab(k, L, scoring, 0, parent, is_leaf, desc, weight)
    f = _features(gpu, 5, n_random)
    (bw, bv), (fn, ff) = voc.transform(f, 4)
    (obw, obv), (ofn, off) = ovoc.transform(f, 4)
    assert np.array_equal(bw, obw) and np.array_equal(bv, obv), len(f)
    assert np.array_equal(fn, ofn) and np.array_equal(ff, off), len(f)


def test_vocab_file_loaders(gpu, tmp_path):
    k, L = 10, 3
    parent, is_leaf, desc, weight = V.synth_vocab(11, k, L)
    f = _features(gpu, 5)
    ref = O.Vocab(k, L, 0, 0, parent, is_leaf, desc, weight)
    (obw, obv), (ofn, off) = ref.transform(f, 1)
    V.write_text(tmp_path / "voc.txt", k, L, 0, 0, parent, is_leaf, desc, weight)
    vt = gpu.Vocabulary.load_text(tmp_path / "voc.txt")
    assert (vt.k, vt.L, vt.n_nodes, vt.n_words) == (k, L, len(parent), int(is_leaf.sum()))
    (bw, bv), (fn, ff) = vt.transform(f, 1)
    assert np.array_equal(bw, obw) and np.array_equal(bv, obv) and np.array_equal(fn, ofn) and np.array_equal(ff, off)
    # binary: weights go through float32; the reference's loader appends a copy of the last node
    V.write_binary(tmp_path / "voc.bin", k, L, 0, 0, parent, is_leaf, desc, weight)
    vb = gpu.Vocabulary.load_binary(tmp_path / "voc.bin")
    assert vb.n_nodes == len(parent) + 1 and vb.n_words == int(is_leaf.sum()) + 1
    p2 = np.append(parent, parent[-1])
    l2 = np.append(is_leaf, is_leaf[-1])
    d2 = np.concatenate([desc, desc[-1:]])
    w2 = np.append(weight.astype(np.float32).astype(np.float64), np.float64(np.float32(weight[-1])))
    refb = O.Vocab(k, L, 0, 0, p2, l2, d2, w2)
    (obw, obv), (ofn, off) = refb.transform(f, 1)
    (bw, bv), (fn, ff) = vb.transform(f, 1)
    assert np.array_equal(bw, obw) and np.array_equal(bv, obv) and np.array_equal(fn, ofn) and np.array_equal(ff, off)
    with pytest.raises(gpu.YgzfeError):
        (tmp_path / "bad.txt").write_text("30 2 0 0\n")
        gpu.Vocabulary.load_text(tmp_path / "bad.txt")


def test_bow_edges(gpu):
    k, L = 4, 2
    parent, is_leaf, desc, weight = V.synth_vocab(3, k, L)
    voc = gpu.Vocabulary.from_arrays(k, L, 0, 0, parent, is_leaf, desc, weight)
    (bw, bv), (fn, ff) = voc.transform(np.zeros((0, 32), np.uint8))
    assert len(bw) == 0 and len(fn) == 0
    # all-stopped features: every leaf weight 0
    voc0 = gpu.Vocabulary.from_arrays(k, L, 0, 0, parent, is_leaf, desc, np.zeros_like(weight))
    (bw, bv), (fn, ff) = voc0.transform(desc[5:9])
    assert len(bw) == 0 and len(fn) == 0
    # a root-only vocabulary has no words: transform() returns empty vectors
    root = gpu.Vocabulary.from_arrays(k, L, 0, 0, parent[:1], is_leaf[:1], desc[:1], weight[:1])
    assert root.n_words == 0
    (bw, bv), (fn, ff) = root.transform(desc[5:9])
    assert len(bw) == 0 and len(fn) == 0


def test_batch_compute_bow_matches_single(gpu):
    import torch
    k, L = 10, 4
    parent, is_leaf, desc, weight = V.synth_vocab(21, k, L)
    voc = gpu.Vocabulary.from_arrays(k, L, 0, 0, parent, is_leaf, desc, weight)
    W, H, nf, sf, nl, ini, mn = S.CONFIGS["C2"]
    frames = np.stack([S.frame(40 + i, W, H) for i in range(5)])
    b = gpu.Batch((nf, sf, nl, ini, mn, 0), 0, W, H, len(frames))
    b.upload(frames)
    b.extract(len(frames))
    b.check()
    cap = b.kp_cap
    dev = torch.device("cuda", 0)
    F = len(frames)
    bw = torch.zeros((F, cap), dtype=torch.int32, device=dev)
    bv = torch.zeros((F, cap), dtype=torch.float64, device=dev)
    nw = torch.zeros(F, dtype=torch.int32, device=dev)
    fn = torch.zeros((F, cap), dtype=torch.int32, device=dev)
    ff = torch.zeros((F, cap), dtype=torch.int32, device=dev)
    nfv = torch.zeros(F, dtype=torch.int32, device=dev)
    torch.cuda.synchronize()
    b.compute_bow(voc, F, 4, bw.data_ptr(), bv.data_ptr(), nw.data_ptr(), fn.data_ptr(), ff.data_ptr(), nfv.data_ptr())
    b.check()
    bw, bv, nw, fn, ff, nfv = [t.cpu().numpy() for t in (bw, bv, nw, fn, ff, nfv)]
    for i in range(F):
        _, d = b.result(i)
        (sw, sv), (sn, sf_) = voc.transform(d, 4)
        assert nw[i] == len(sw) and nfv[i] == len(sn)
        assert np.array_equal(bw[i, :nw[i]], sw) and np.array_equal(bv[i, :nw[i]], sv)
        assert np.array_equal(fn[i, :nfv[i]], sn) and np.array_equal(ff[i, :nfv[i]], sf_)
