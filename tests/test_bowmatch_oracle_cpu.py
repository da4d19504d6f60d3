"""CPU checks of the SearchByBoW / SearchForInitialization restatements (oracle/bowmatch_oracle.cpp,
oracle/match_oracle.cpp) — properties the reference's code implies, since no reference fixture pins them
(parity unpinned against the real ORB-SLAM3 build; the GPU path is bit-exact to these restatements)."""
import numpy as np
import pytest

from openmavis_amd import synth_init, synth_tri


@pytest.mark.parametrize("kf_kf", [False, True])
def test_search_by_bow_properties(oracle, kf_kf):
    p = synth_tri.make_tri_pair(seed=5, n_pts=500, mp_frac=0.8)
    job = dict(kf=p["kf1"], other=p["kf2"])
    n, m = oracle.search_by_bow(job, kf_kf=kf_kf, nnratio=0.75, check_ori=False)
    kf, fr = p["kf1"], p["kf2"]
    hit = np.nonzero(m >= 0)[0]
    assert n == len(hit) > 100
    if kf_kf:
        idx1, idx2 = hit, m[hit]
        assert len(set(idx2.tolist())) == len(idx2)          # vbMatched2: a pKF2 keypoint matched once
        assert fr["has_mp"][idx2].all() and kf["has_mp"][idx1].all()
    else:
        idx2, idx1 = hit, m[hit]                               # frame keypoint -> keyframe keypoint
        assert kf["has_mp"][idx1].all()
    # matched keypoints share a vocabulary node and are the same world point (synthetic truth)
    node = lambda v: np.repeat(v["node_id"], np.diff(v["node_start"]))[np.argsort(v["node_idx"])]
    assert (node(kf)[idx1] == node(fr)[idx2]).all()
    assert np.mean(kf["pt"][idx1] == fr["pt"][idx2]) > 0.98
    # Hamming distances within TH_LOW (strict for the (KF1, KF2) overload)
    d = np.unpackbits(kf["desc"][idx1] ^ fr["desc"][idx2], axis=1).sum(1)
    assert (d < 50).all() if kf_kf else (d <= 50).all()
    # the rotation filter only removes matches
    n2, m2 = oracle.search_by_bow(job, kf_kf=kf_kf, nnratio=0.75, check_ori=True)
    assert n2 <= n and np.all((m2 == m) | (m2 == -1))


def test_search_by_bow_mono_frame_uses_one_block(oracle):
    p = synth_tri.make_tri_pair(seed=2, n_pts=400, mp_frac=0.9)
    mono = dict(p["kf2"], n_left=-1)
    n1, m1 = oracle.search_by_bow(dict(kf=p["kf1"], other=mono), check_ori=False)
    n4, m4 = oracle.search_by_bow(dict(kf=p["kf1"], other=p["kf2"]), check_ori=False)
    # one block: at most one frame keypoint per keyframe keypoint; four blocks: up to one per camera
    assert np.bincount(m1[m1 >= 0]).max() == 1
    assert np.bincount(m4[m4 >= 0]).max() >= 2


@pytest.mark.parametrize("check_ori", [False, True])
def test_search_for_initialization_properties(oracle, check_ori):
    p = synth_init.make_init_pair(seed=4, n=900)
    g = oracle.frame_geom(1, p["width"], p["height"], synth_init.scale_factors())
    n, m12, prev = oracle.search_for_initialization(g, p["f1"]["kps"], p["f1"]["desc"], p["f2"]["kps"],
                                                    p["f2"]["desc"], p["prev"], 100, 0.9, check_ori)
    hit = np.nonzero(m12 >= 0)[0]
    assert n == len(hit) > 100
    assert (p["f1"]["kps"]["octave"][hit] == 0).all() and (p["f2"]["kps"]["octave"][m12[hit]] == 0).all()
    assert len(set(m12[hit].tolist())) == len(hit)             # vnMatches21: one F1 keypoint per F2 keypoint
    assert np.mean(p["f2"]["truth"][m12[hit]] == hit) > 0.98
    # vbPrevMatched moves to the matched F2 keypoints, stays elsewhere
    k2 = p["f2"]["kps"]
    assert np.array_equal(prev[hit], np.stack([k2["x"][m12[hit]], k2["y"][m12[hit]]], 1))
    miss = np.setdiff1d(np.arange(len(m12)), hit)
    assert np.array_equal(prev[miss], p["prev"][miss])
    # inside the window: |dx| < r and |dy| < r around the previous position
    assert (np.abs(prev[hit] - p["prev"][hit]) < 100).all()
