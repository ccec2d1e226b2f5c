"""The monocular initialiser's extractor and the single-frame graph path.

Tracking.cc:261 builds `mpIniORBextractor = new ORBextractor(2 * nFeatures, fScaleFactor,
nLevels, fIniThFAST, fMinThFAST)`; at the EuRoC settings that is ORBextractor(2000, 2.0, 4,
20, 7), and GrabImageMonocular extracts with it on every frame while NOT_INITIALIZED
(Tracking.cc:387-388).  Its level 0 falls in a larger octree node-pool class than its
other levels, which is the configuration whose captured single-frame graph crashed in round 5
(profiles/r05_graph_fork.txt: ygzfe_extract forked three side streams into the capture
and joined one).  Here, through the graph path (no existing rows: ygzfe_extract captures
once per frame handle, then replays):

* keypoints and descriptors bit-exact against OrbOracle(2000, 2.0, 4, 20, 7) on synthetic
  and rendered 752x480 frames, on the capture and on replays;
* the same after another extractor (C2, ORBextractor(1000, ...)) ran its own graphs in the
  process, interleaved both ways;
* round 5's repro order in one process -- a C5 sequence step, then SparseImgAlign (GN and
  LM) with ORBextractor(2000) frames -- with the graph path on: ygzfe_extract returns
  YGZFE_EHIP if any stream is left capturing after a capture, so an unjoined fork fails here.
"""
import numpy as np
import pytest
import torch

import _oracle as O
import _scenes as S
from test_gpu_extract import assert_kps_equal

pytestmark = pytest.mark.gpu
INI = (752, 480, 2000, 2.0, 4, 20, 7)


def _ini(gpu):
    W, H, nf, sf, nl, ini, mn = INI
    return gpu.ORBextractor(nf, sf, nl, ini, mn), O.OrbOracle(nf, sf, nl, ini, mn)


def _check(ex, orc, img, what, replays=2):
    fr = ex.ComputePyramid(img)
    kr, dr = orc.extract(orc.pyramid(img))
    assert len(kr) > 0.6 * orc.o.nfeatures, f"{what}: only {len(kr)} oracle keypoints"
    for r in range(1 + replays):  # the capture, then graph replays on the same handle
        kg, dg = ex.extract(fr)
        assert_kps_equal(kg, kr, f"{what} call {r}")
        assert np.array_equal(dg, dr), f"{what} call {r}: {np.count_nonzero((dg != dr).any(1))} descriptor rows differ"
    return len(kr)


def _rendered(seed):
    sc = S.PlaneScene(seed)
    q = S.quat_from_rotvec([0.01 * seed, -0.02, 0.005]).astype(np.float32)
    t = np.array([0.05, -0.03 * seed, 0.02], np.float32)
    return sc.render(q, t, seed)


@pytest.mark.parametrize("seed", [0, 1, 2])
def test_initializer_extract_bitexact(gpu, seed):
    W, H = INI[:2]
    ex, orc = _ini(gpu)
    _check(ex, orc, S.frame(100 + seed, W, H), f"synthetic {seed}")
    _check(ex, orc, _rendered(seed), f"rendered {seed}")


def _node_pool_classes(cfg):
    """extract.hip octree_nc(): a level's node pool holds its budget (feat_per_level) plus
    4 children per initial node (round(w / h) of the FAST window, ORBextractor.cc:539) + 16,
    rounded up to 256 / 512 / 1024 / 2048."""
    W, H, nf, sf, nl, ini, mn = cfg
    orc = O.OrbOracle(nf, sf, nl, ini, mn)
    out = []
    for (w, h), budget in zip(orc.level_sizes(W, H), orc.feat_per_level):
        n_ini = int(round((w - 32) / (h - 32)))  # minBorder 16 each side (EDGE_THRESHOLD - 3)
        need = budget + 4 * n_ini + 16
        out.append(256 if need <= 256 else 512 if need <= 512 else 1024 if need <= 1024 else 2048)
    return out


def test_initializer_level0_in_a_larger_node_pool_class():
    """The case this file exists for: the initialiser's level 0 needs the 2048-node pool,
    so its octree runs as two launch groups (the single-launch `wide` chain covers only
    pools <= 1024, which is every C2 level)."""
    ini = _node_pool_classes(INI)
    assert ini[0] == 2048 and max(ini[1:]) <= 1024, ini
    assert max(_node_pool_classes(S.CONFIGS["C2"])) <= 1024


def test_initializer_after_and_before_another_extractor(gpu):
    W, H = INI[:2]
    ex, orc = _ini(gpu)
    c2 = S.CONFIGS["C2"]
    ex2 = gpu.ORBextractor(*c2[2:])
    orc2 = O.OrbOracle(*c2[2:])
    imgs = [S.frame(200 + i, W, H) for i in range(3)]
    # C2 graphs first, then the initialiser's, then C2 again on new frame handles, then the
    # initialiser again (Tracking switches mpIniORBextractor -> mpORBextractorLeft once
    # initialised, and back on a reset)
    _check(ex2, orc2, imgs[0], "C2 before", replays=1)
    _check(ex, orc, imgs[0], "initialiser after C2")
    _check(ex2, orc2, imgs[1], "C2 after the initialiser", replays=1)
    _check(ex, orc, imgs[2], "initialiser again")
    # and the frames of one extractor alternately: every handle keeps its own graph
    frs = [ex.ComputePyramid(im) for im in imgs]
    want = [orc.extract(orc.pyramid(im)) for im in imgs]
    for r in range(2):
        for i, fr in enumerate(frs):
            kg, dg = ex.extract(fr)
            assert_kps_equal(kg, want[i][0], f"handle {i} pass {r}")
            assert np.array_equal(dg, want[i][1])


def test_round5_repro_order_with_graphs(gpu):
    """C5 sequence step, then SparseImgAlign GN and LM with ORBextractor(2000) frames (the
    order of tests/test_gpu_c5.py, test_gpu_align.py, test_gpu_align_lm.py that crashed),
    then the initialiser extraction again -- in one process, graphs on."""
    from ygzfe.sequence import C5Shard
    from test_gpu_align import POSE_TOL, align_case
    dev = torch.device("cuda", 0)
    sh = C5Shard(256, 0, 1, dev)
    sh.step()
    torch.cuda.synchronize()
    sh.check()
    for method in (0, 1):
        for seed in (6, 7):
            res, ores, _ = align_case(gpu, seed, method=method, nfeatures=2000)
            err = S.se3_log_inf(*res.T_cur_ref.as_arrays(), np.array(ores.T.q[:]), np.array(ores.T.t[:]))
            assert err <= POSE_TOL and res.n_visible == ores.n_visible, (method, seed, err)
    sh.step()
    torch.cuda.synchronize()
    sh.check()
    ex, orc = _ini(gpu)
    _check(ex, orc, S.frame(300, *INI[:2]), "after the repro order")
    del sh
    torch.cuda.empty_cache()


@pytest.mark.parametrize("cfg", ["INI", "C2"])
def test_batch_extract_captured_in_a_graph(gpu, cfg):
    """the batch path forks the octree's node-pool classes after the
    first onto the batch's aux streams (api.cpp ygzfe_batch_extract_split -> launch_octree),
    and `bench.py --graph 1` captures that path into a HIP graph.  The initialiser's 2048-node
    level-0 class makes two launch groups, so a fork and join happen inside the capture.
    Captured on a torch stream, replayed twice, then new frames uploaded into the same
    buffers and replayed again; every result bit-exact against the oracle, and an eager
    extract afterwards (it would fail on an aux stream left capturing) equal too."""
    W, H, nf, sf, nl, ini, mn = INI if cfg == "INI" else S.CONFIGS["C2"]
    F = 3
    b = gpu.Batch((nf, sf, nl, ini, mn, 0), 0, W, H, F)
    orc = O.OrbOracle(nf, sf, nl, ini, mn)
    fa = np.stack([S.frame(400 + i, W, H) for i in range(F)])
    fb = np.stack([S.frame(500 + i, W, H) for i in range(F)])
    dev = torch.device("cuda", 0)
    st = torch.cuda.Stream(dev)
    b.upload(fa)
    torch.cuda.synchronize()
    b.extract(F, st.cuda_stream)  # warm: plans, workspaces, lazily created streams
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    b.upload(fa)
    torch.cuda.synchronize()
    with torch.cuda.graph(g, stream=st):
        b.extract(F, st.cuda_stream)
    for frames, tag in ((fa, "a"), (fa, "a again"), (fb, "b")):
        b.upload(frames)
        torch.cuda.synchronize()
        g.replay()
        torch.cuda.synchronize()
        b.check()
        for i in range(F):
            kg, dg = b.result(i)
            kr, dr = orc.extract(orc.pyramid(frames[i]))
            assert_kps_equal(kg, kr, f"{cfg} replay {tag} frame {i}")
            assert np.array_equal(dg, dr), f"{cfg} replay {tag} frame {i}"
    b.upload(fa)
    b.extract(F)
    torch.cuda.synchronize()
    b.check()
    for i in range(F):
        kg, dg = b.result(i)
        kr, dr = orc.extract(orc.pyramid(fa[i]))
        assert_kps_equal(kg, kr, f"{cfg} eager after the graph frame {i}")
        assert np.array_equal(dg, dr)
    del g
