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
    desc = [np.zeros((1, 32), np.uint8)]
    parent = [np.zeros(1, np.int64)]
    frontier = np.zeros(1, np.int64)
    n = 1
    for lvl in range(1, L + 1):
        par = np.repeat(frontier, k)
        if lvl == 1:
            d = rng.integers(0, 256, (len(par), 32), dtype=np.uint8)
        else:
            d = synth.flip_bits(np.concatenate(desc)[par], rng, max(2, 64 >> lvl))
        ids = np.arange(n, n + len(par))
        n += len(par)
        desc.append(d)
        parent.append(par)
        frontier = ids[rng.random(len(ids)) >= early_leaf] if lvl == L - 1 else ids   # some stay leaves
    desc = np.concatenate(desc)
    parent = np.concatenate(parent)
    counts = np.bincount(parent[1:], minlength=n)
    cs = np.zeros(n + 1, np.int32)
    cs[1:] = np.cumsum(counts)
    child_ids = np.argsort(parent[1:], kind="stable").astype(np.int32) + 1   # per parent, in line order
    leaf = counts == 0
    leaf[0] = False
    word = np.zeros(n, np.int32)
    word[leaf] = np.arange(leaf.sum(), dtype=np.int32)
    weight = np.where(rng.random(n) < stop, 0.0, rng.uniform(0.5, 5.0, n))
    weight[0] = 0.0
    if weighting in (1, 3):   # TF / BINARY vocabularies store weight 1 per word (DBoW2 setNodeWeights)
        weight = np.where(weight > 0, 1.0, 0.0)
    return dict(k=k, L=L, scoring=scoring, weighting=weighting, n_words=int(leaf.sum()), child_start=cs,
                child_ids=child_ids, desc=desc, word_id=word, weight=weight)


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
