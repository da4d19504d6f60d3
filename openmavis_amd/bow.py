"""Host-side mirror of DBoW2's TemplatedVocabulary<FORB::TDescriptor, FORB> (ORBVocabulary, include/ORBVocabulary.h)
as OpenMAVIS uses it: loadFromTextFile (Thirdparty/DBoW2/DBoW2/TemplatedVocabulary.h:1338-1424) into a flattened
device tree, and the batched transform(features, BowVector&, FeatureVector&, levelsup) on libomv_hip.so
(openmavis_amd/csrc/bow.hip).

    voc = ORBVocabulary.loadFromTextFile("ORBvoc.txt", device="cuda:0")
    out = voc.transform(desc, n_desc, levelsup=4)   # desc: device uint8 [S][cap][32], n_desc int32 [S]

`out` holds per feature word / wval / node and, per set, the BowVector (bow_word, bow_value, bow_n) and the
FeatureVector (fv_node, fv_start, fv_idx, fv_n) — the mBowVec / mFeatVec of Frame::ComputeBoW.  No CPU
fallback.  Deviation: loadFromTextFile turns a trailing empty line into an extra root child whose descriptor
is uninitialised memory (:1378-1404); the loader here skips empty lines.
"""
import ctypes

import numpy as np

from . import _lib

SCORING = {"L1_NORM": 0, "L2_NORM": 1, "CHI_SQUARE": 2, "KL": 3, "BHATTACHARYYA": 4, "DOT_PRODUCT": 5}
WEIGHTING = {"TF_IDF": 0, "TF": 1, "IDF": 2, "BINARY": 3}


def parse_text(lines):
    """loadFromTextFile's parse of the text format: header `k L scoring weighting`, then per node `parent
    is_leaf d0 .. d31 weight`; node ids in line order from 1, children appended in line order, word ids
    given to leaves in line order.  Returns host arrays."""
    it = iter(lines)
    k, L, sc, wt = (int(x) for x in next(it).split()[:4])
    if k < 0 or k > 20 or L < 1 or L > 10 or sc < 0 or sc > 5 or wt < 0 or wt > 3:
        raise ValueError("Vocabulary loading failure: This is not a correct text file!")
    parent, leaf, desc, weight = [0], [0], [np.zeros(32, np.uint8)], [0.0]
    for line in it:
        f = line.split()
        if not f:
            continue
        parent.append(int(f[0]))
        leaf.append(int(f[1]) > 0)
        desc.append(np.array([int(x) for x in f[2:34]], np.uint8))
        weight.append(float(f[34]))
    n = len(parent)
    children = [[] for _ in range(n)]
    for i in range(1, n):
        children[parent[i]].append(i)
    word = np.zeros(n, np.int32)
    nw = 0
    for i in range(1, n):
        if leaf[i]:
            word[i] = nw
            nw += 1
    cs = np.zeros(n + 1, np.int32)
    cs[1:] = np.cumsum([len(c) for c in children])
    return dict(k=k, L=L, scoring=sc, weighting=wt, n_words=nw, child_start=cs,
                child_ids=np.array([c for ch in children for c in ch], np.int32), desc=np.stack(desc),
                word_id=word, weight=np.array(weight, np.float64))


def to_text(v):
    """saveToTextFile's format (:1428-1447) of a host vocabulary dict."""
    n = len(v["weight"])
    parent = np.zeros(n, np.int64)
    for p in range(n):
        for c in v["child_ids"][v["child_start"][p]:v["child_start"][p + 1]]:
            parent[c] = p
    out = [f"{v['k']} {v['L']}  {v['scoring']} {v['weighting']}"]
    for i in range(1, n):
        leaf = v["child_start"][i] == v["child_start"][i + 1]
        out.append(f"{parent[i]} {1 if leaf else 0} " + " ".join(str(int(x)) for x in v["desc"][i]) +
                   f" {repr(float(v['weight'][i]))}")
    return "\n".join(out) + "\n"


class ORBVocabulary:
    def __init__(self, host, device="cuda:0"):
        import torch
        self.host = host
        self.k, self.L = host["k"], host["L"]
        self.t = {k: torch.from_numpy(np.ascontiguousarray(host[k])).to(device)
                  for k in ("child_start", "child_ids", "desc", "word_id", "weight")}
        self.v = _lib.Vocab(len(host["weight"]), host["n_words"], host["L"], host["scoring"], host["weighting"],
                            *[_lib.ptr(self.t[k]) for k in ("child_start", "child_ids", "desc", "word_id", "weight")])
        self._lib = _lib.load()

    @classmethod
    def loadFromTextFile(cls, path, device="cuda:0"):
        with open(path) as f:
            return cls(parse_text(f.read().splitlines()), device)

    def transform(self, desc, n_desc, levelsup=4, stream=None):
        import torch
        S, cap = desc.shape[0], desc.shape[1]
        dev = desc.device
        z = lambda *s, dt=torch.int32: torch.empty(s, dtype=dt, device=dev)   # noqa: E731
        o = dict(word=z(S, cap), wval=z(S, cap, dt=torch.float64), node=z(S, cap), bow_word=z(S, cap),
                 bow_value=z(S, cap, dt=torch.float64), bow_n=z(S), fv_node=z(S, cap), fv_start=z(S, cap + 1),
                 fv_idx=z(S, cap), fv_n=z(S))
        st = stream if stream is not None else torch.cuda.current_stream(dev).cuda_stream
        _lib.check(self._lib.omv_bow_transform(ctypes.byref(self.v), S, _lib.ptr(desc), cap, _lib.ptr(n_desc),
                                               int(levelsup), *[_lib.ptr(o[k]) for k in (
                                                   "word", "wval", "node", "bow_word", "bow_value", "bow_n",
                                                   "fv_node", "fv_start", "fv_idx", "fv_n")], ctypes.c_void_p(st)),
                   "omv_bow_transform")
        return o
