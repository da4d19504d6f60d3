"""GPU parity of the batched DBoW2 transform (openmavis_amd/csrc/bow.hip) against the oracle
(oracle/bow_oracle.cpp): per-feature words / weights / nodes, the BowVector (words, values as raw doubles) and
the FeatureVector, bit-exact, for the ORB-SLAM3 settings (TF-IDF, L1) and the other scoring / weighting modes."""
import numpy as np
import pytest

from openmavis_amd import synth_bow
from openmavis_amd.bow import ORBVocabulary

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("scoring,weighting,levelsup,cap", [(0, 0, 2, 2000), (1, 0, 2, 700), (5, 1, 1, 700),
                                                             (0, 3, 2, 700), (0, 0, 4, 300), (0, 0, 2, 16384)])
def test_bow_transform_matches_oracle(oracle, scoring, weighting, levelsup, cap):
    import torch
    v = synth_bow.make_vocab(seed=1, scoring=scoring, weighting=weighting)
    d, n = synth_bow.make_sets(v, n_sets=3, cap=cap, seed=2)
    n[1] = 0 if cap < 16384 else n[1]   # an empty set
    voc = ORBVocabulary(v)
    g = voc.transform(torch.from_numpy(d).cuda(), torch.from_numpy(n).cuda(), levelsup)
    torch.cuda.synchronize()
    g = {k: t.cpu().numpy() for k, t in g.items()}
    o = oracle.bow_transform(v, d, n, levelsup)
    for s in range(3):
        m = int(n[s])
        for k in ("word", "wval", "node"):
            assert np.array_equal(g[k][s, :m], o[s][k]), (s, k)
        nb, nf = int(g["bow_n"][s]), int(g["fv_n"][s])
        assert nb == len(o[s]["bow_word"]) and nf == len(o[s]["fv_node"])
        assert np.array_equal(g["bow_word"][s, :nb], o[s]["bow_word"])
        assert np.array_equal(g["bow_value"][s, :nb].view(np.int64), o[s]["bow_value"].view(np.int64))
        assert np.array_equal(g["fv_node"][s, :nf], o[s]["fv_node"])
        assert np.array_equal(g["fv_start"][s, :nf + 1], o[s]["fv_start"])
        assert np.array_equal(g["fv_idx"][s, :o[s]["fv_start"][-1]], o[s]["fv_idx"])
