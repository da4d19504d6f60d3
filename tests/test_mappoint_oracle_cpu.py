"""CPU pinning of the map-point refresh oracle (oracle/mappoint_oracle.cpp) against an independent numpy restatement of
MapPoint::ComputeDistinctiveDescriptors (src/MapPoint.cc:405-490: the N x N distances, each row sorted, vDists[0.5 (N
- 1)], the first strict minimum) and of UpdateNormalAndDepth (src/MapPoint.cc:503-588, float32 per operation)."""
import numpy as np

from openmavis_amd import synth_mappoint
import oracle


def _popcount_dist(a, b):
    return int(np.unpackbits(np.bitwise_xor(a, b)).sum())


def _np_distinctive(desc, start, rows):
    out = []
    for p in range(len(start) - 1):
        r = rows[start[p]:start[p + 1]]
        if len(r) == 0:
            out.append(-1)
            continue
        D = np.array([[_popcount_dist(desc[i], desc[j]) for j in r] for i in r])
        med = [np.sort(D[i])[int(0.5 * (len(r) - 1))] for i in range(len(r))]
        out.append(int(r[int(np.argmin(med))]))   # argmin: the first of equal minima
    return np.array(out, np.int32)


def test_distinctive_oracle_matches_numpy():
    b = synth_mappoint.make_points(n_points=300, seed=3, sizes=np.r_[np.arange(0, 40), np.random.default_rng(1).integers(0, 30, 260)])
    assert np.array_equal(oracle.distinctive_descriptors(b["desc"], b["desc_start"], b["desc_row"]),
                          _np_distinctive(b["desc"], b["desc_start"], b["desc_row"]))


def test_distinctive_picks_the_cluster_centre():
    """Noisy copies of one descriptor plus unrelated ones (20 %): the chosen descriptor is one of the copies (within 40
    bits of at least three other copies: every point of this seed keeps at least four copies of its nine)."""
    b = synth_mappoint.make_points(n_points=100, seed=4, sizes=np.full(100, 9), outlier_frac=0.2, dup_frac=0.0)
    best = oracle.distinctive_descriptors(b["desc"], b["desc_start"], b["desc_row"])
    for p in range(100):
        r = b["desc_row"][b["desc_start"][p]:b["desc_start"][p + 1]]
        assert sum(_popcount_dist(b["desc"][best[p]], b["desc"][j]) <= 40 for j in r) >= 4


def test_normal_depth_oracle_matches_numpy():
    g = synth_mappoint.make_geometry(n_points=500, seed=5)
    n, dmin, dmax = oracle.normal_depth(**g)
    f = np.float32
    for p in range(500):
        s, e = g["obs_start"][p], g["obs_start"][p + 1]
        if s == e:
            assert np.isnan(n[p]).all()
            continue
        acc = np.zeros(3, f)
        for q in range(s, e):
            v = (g["pos"][p] - g["obs_center"][q]).astype(f)
            r = f(np.sqrt(f(f(v[0] * v[0] + v[1] * v[1]) + v[2] * v[2])))
            acc = (acc + (v / r).astype(f)).astype(f)
        pc = (g["pos"][p] - g["ref_center"][p]).astype(f)
        dist = f(np.sqrt(f(f(pc[0] * pc[0] + pc[1] * pc[1]) + pc[2] * pc[2])))
        mx = f(dist * g["ref_level_scale"][p])
        assert dmax[p] == mx and dmin[p] == f(mx / g["ref_max_scale"][p])
        assert np.array_equal(n[p], (acc / f(e - s)).astype(f))
