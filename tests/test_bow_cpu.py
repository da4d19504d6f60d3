"""CPU checks of the DBoW2 transform restatement (oracle/bow_oracle.cpp, TemplatedVocabulary.h:1127-1259) and the
text-vocabulary loader (openmavis_amd/bow.parse_text, loadFromTextFile :1338-1424).  ORBvoc.txt is not in the
container: parity is unpinned against the real vocabulary; these pin the restatement's behaviour."""
import numpy as np
import pytest

from openmavis_amd import synth_bow
from openmavis_amd.bow import parse_text, to_text


def _descend_numpy(v, f, levelsup):
    node, lvl, nid = 0, 0, (0 if v["L"] - levelsup <= 0 else -1)
    while True:
        lvl += 1
        ch = v["child_ids"][v["child_start"][node]:v["child_start"][node + 1]]
        d = np.unpackbits(np.bitwise_xor(v["desc"][ch], f[None]), axis=1).sum(1)
        node = int(ch[int(np.argmin(d))])   # first minimum
        if lvl == v["L"] - levelsup:
            nid = node
        if v["child_start"][node] == v["child_start"][node + 1]:
            return int(v["word_id"][node]), float(v["weight"][node]), nid


def test_transform_matches_a_numpy_descent(oracle):
    v = synth_bow.make_vocab(seed=3)
    d, n = synth_bow.make_sets(v, n_sets=2, cap=400, seed=4)
    out = oracle.bow_transform(v, d, n, 2)
    for s in range(2):
        for i in range(0, int(n[s]), 7):
            w, wt, nid = _descend_numpy(v, d[s, i], 2)
            assert (out[s]["word"][i], out[s]["wval"][i], out[s]["node"][i]) == (w, wt, nid)


def test_bow_and_feature_vectors(oracle):
    """TF-IDF + L1: the BowVector sums the idf of each word's features, normalised to unit L1; the
    FeatureVector lists, per node ascending, the non-stopped features in index order."""
    v = synth_bow.make_vocab(seed=5)
    d, n = synth_bow.make_sets(v, n_sets=1, cap=1500, seed=6)
    o = oracle.bow_transform(v, d, n, 2)[0]
    live = o["wval"] > 0
    words = np.unique(o["word"][live])
    assert np.array_equal(o["bow_word"], words)
    raw = np.array([o["wval"][live & (o["word"] == w)].sum() for w in words])
    assert np.allclose(o["bow_value"], raw / raw.sum(), rtol=1e-12)
    assert abs(o["bow_value"].sum() - 1) < 1e-12
    nodes = np.unique(o["node"][live])
    assert np.array_equal(o["fv_node"], nodes)
    for j, nd in enumerate(nodes):
        assert np.array_equal(o["fv_idx"][o["fv_start"][j]:o["fv_start"][j + 1]], np.nonzero(live & (o["node"] == nd))[0])


@pytest.mark.parametrize("scoring,weighting", [(1, 0), (5, 1), (0, 3), (2, 2)])
def test_scoring_and_weighting_variants(oracle, scoring, weighting):
    v = synth_bow.make_vocab(seed=7, scoring=scoring, weighting=weighting)
    d, n = synth_bow.make_sets(v, n_sets=1, cap=800, seed=8)
    o = oracle.bow_transform(v, d, n, 2)[0]
    if scoring == 1:
        assert abs(np.sqrt((o["bow_value"] ** 2).sum()) - 1) < 1e-12
    elif scoring == 5 and weighting == 1:   # TF, not normalised: value / number of words
        live = o["wval"] > 0
        cnt = np.array([(live & (o["word"] == w)).sum() for w in o["bow_word"]])
        assert np.allclose(o["bow_value"], cnt / len(o["bow_word"]))
    else:
        assert abs(o["bow_value"].sum() - 1) < 1e-12


def test_feature_vector_level_above_root(oracle):
    """levelsup >= L: every feature's FeatureVector node is the root."""
    v = synth_bow.make_vocab(seed=9, L=3)
    d, n = synth_bow.make_sets(v, n_sets=1, cap=300, seed=10)
    o = oracle.bow_transform(v, d, n, 3)[0]
    assert (o["node"] == 0).all() and list(o["fv_node"]) in ([0], [])


def test_text_round_trip():
    v = synth_bow.make_vocab(k=4, L=3, seed=11)
    w = parse_text((to_text(v) + "\n").splitlines())
    for k in ("child_start", "child_ids", "desc", "word_id", "weight"):
        assert np.array_equal(w[k], v[k]), k
    assert (w["k"], w["L"], w["n_words"]) == (v["k"], v["L"], v["n_words"])
