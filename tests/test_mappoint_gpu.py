"""GPU parity of the map-point refresh (openmavis_amd/csrc/mappoint.hip) against the CPU oracle
(oracle/mappoint_oracle.cpp): MapPoint::ComputeDistinctiveDescriptors (src/MapPoint.cc:405-490) bit-exact (the chosen
row and descriptor) and MapPoint::UpdateNormalAndDepth (src/MapPoint.cc:503-588) bit-exact (float32 raw bits)."""
import numpy as np
import pytest

from openmavis_amd import mappoint, synth_mappoint

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("seed,sizes", [(1, None), (2, list(range(0, 70)) + [127, 128, 129, 255, 256, 257, 300, 520])])
def test_distinctive_descriptors_match_oracle(oracle, seed, sizes):
    """Random sizes 0..23, then every size 0..69 and the LDS-stage edges (256) and beyond (300, 520: rows read from
    global memory), duplicated descriptors (median ties: the first index wins)."""
    b = synth_mappoint.make_points(n_points=2000 if sizes is None else len(sizes), seed=seed, sizes=sizes)
    best, out = mappoint.ComputeDistinctiveDescriptors(b["desc"], b["desc_start"], b["desc_row"])
    ref = oracle.distinctive_descriptors(b["desc"], b["desc_start"], b["desc_row"])
    best = best.cpu().numpy()
    assert np.array_equal(best, ref)
    has = ref >= 0
    assert np.array_equal(out.cpu().numpy()[has], b["desc"][ref[has]])


def test_normal_and_depth_match_oracle(oracle):
    g = synth_mappoint.make_geometry(n_points=5000, seed=7)
    n, dmin, dmax = mappoint.UpdateNormalAndDepth(**g)
    on, omin, omax = oracle.normal_depth(**g)
    for a, b in ((n, on), (dmin, omin), (dmax, omax)):
        a = a.cpu().numpy()
        assert np.array_equal(a.view(np.uint32), b.view(np.uint32))
