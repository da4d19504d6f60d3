"""Seeded synthetic DBoW2 vocabularies and descriptor sets (ORBvoc.txt is not available here).

make_vocab: a k-ary tree of depth L in breadth-first line order (as a text file lists it), node descriptors
derived from the parent's by random bit flips (fewer deeper down) so descents are structured, ~10 % of the
depth L-1 nodes turned into leaves (an unbalanced tree), idf weights U(0.5, 5) with ~5 % stopped words
(weight 0).  make_sets: descriptor sets whose rows are leaf descriptors with U{0..12} bit flips (70 %) or
random."""
import numpy as np

from . import synth


def make_vocab(k=10, L=4, seed=1, scoring=0, weighting=0, early_leaf=0.1, stop=0.05):
    rng = np.random.Generator(np.random.PCG64(seed))
    desc = [np.zeros(32, np.uint8)]
    parent, depth = [0], [0]
    frontier = [0]
    for lvl in range(1, L + 1):
        nxt = []
        for p in frontier:
            for _ in range(k):
                nxt.append(len(desc))
                if p == 0:
                    desc.append(rng.integers(0, 256, 32, dtype=np.uint8))
                else:
                    desc.append(synth.flip_bits(desc[p][None], rng, max(2, 64 >> lvl))[0])
                parent.append(p)
                depth.append(lvl)
        if lvl == L - 1:   # some depth L-1 nodes stay leaves (an unbalanced tree)
            nxt = [i for i in nxt if rng.random() >= early_leaf]
        frontier = nxt
    n = len(desc)
    children = [[] for _ in range(n)]
    for i in range(1, n):
        children[parent[i]].append(i)
    word = np.zeros(n, np.int32)
    nw = 0
    for i in range(1, n):
        if not children[i]:
            word[i] = nw
            nw += 1
    weight = np.where(rng.random(n) < stop, 0.0, rng.uniform(0.5, 5.0, n))
    weight[0] = 0.0
    if weighting in (1, 3):   # TF / BINARY vocabularies store weight 1 per word (DBoW2 setNodeWeights)
        weight = np.where(weight > 0, 1.0, 0.0)
    cs = np.zeros(n + 1, np.int32)
    cs[1:] = np.cumsum([len(c) for c in children])
    return dict(k=k, L=L, scoring=scoring, weighting=weighting, n_words=nw, child_start=cs,
                child_ids=np.array([c for ch in children for c in ch], np.int32), desc=np.stack(desc),
                word_id=word, weight=weight)


def make_sets(v, n_sets=4, cap=2000, seed=2):
    rng = np.random.Generator(np.random.PCG64(seed))
    leaves = np.nonzero(v["child_start"][1:] == v["child_start"][:-1])[0]
    leaves = leaves[leaves > 0]
    n = rng.integers(cap // 2, cap + 1, n_sets).astype(np.int32)
    d = rng.integers(0, 256, (n_sets, cap, 32), dtype=np.uint8)
    for s in range(n_sets):
        src = rng.choice(leaves, cap)
        der = rng.random(cap) < 0.7
        d[s, der] = synth.flip_bits(v["desc"][src[der]], rng, 12)
    return d, n
