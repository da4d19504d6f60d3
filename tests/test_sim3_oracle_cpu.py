"""CPU checks of the ORBmatcher::SearchBySim3 restatement (oracle/match_oracle.cpp, src/ORBmatcher.cc:1771-1983)
on synthetic pairs with known truth (parity unpinned against the real build: no reference test or caller
exercises SearchBySim3 in this fork; the GPU path is bit-exact to the restatement)."""
import numpy as np

from openmavis_amd import synth_sim3


def test_search_by_sim3_properties(oracle):
    b = synth_sim3.make_sim3_batch(n_pairs=3, seed=1)
    m, n = oracle.search_by_sim3(b)
    for j, jb in enumerate(b["jobs"]):
        s = slice(jb["start1"], jb["start1"] + jb["count1"])
        k1, mm = b["kp1"][s], m[s]
        hit = mm >= 0
        assert n[j] == hit.sum() > 100
        # agreed matches are the same world point, in block 0 of pKF2, each pKF2 keypoint at most once
        assert (b["wid"][jb["kf1"], k1[hit]] == b["wid"][jb["kf2"], mm[hit]]).all()
        assert (mm[hit] < b["n_kp"][jb["kf2"], 0]).all()
        assert len(set(mm[hit].tolist())) == hit.sum()


def test_search_by_sim3_wrong_similarity_finds_less(oracle):
    b = synth_sim3.make_sim3_batch(n_pairs=2, seed=3)
    _, n = oracle.search_by_sim3(b)
    for jb in b["jobs"]:   # a wrong similarity moves the projections off the keypoints
        for key in ("S12", "S21"):
            S = dict(jb[key])
            S["t"] = S["t"] * np.float32(3.0) + np.float32(0.5)
            jb[key] = S
    _, n_bad = oracle.search_by_sim3(b)
    assert (n_bad < n // 4).all()
