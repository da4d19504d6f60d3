"""GPU parity of LocalMapping::CreateNewMapPoints' whole neighbour loop (omv_local_mapping_create_new_map_points:
per neighbour the gated SearchForTriangulation launches against the current keyframe's has-map-point flags as the
previous neighbours left them, then the geometry, on the device without host round trips) against the interleaved
oracle (oracle/tri_oracle.cpp oracle_local_mapping_create_new_map_points, src/LocalMapping.cc:439-783): per neighbour
vMatches12, the search's count, the accepted / rejected status and the new points' coordinates as raw float32 bits,
the final has-map-point flags and side-1 state -- bit-exact.  12 and 16 neighbours sharing most current-keyframe
keypoints (tests/test_cnmp_chain_oracle_cpu.py pins that the loop differs from per-neighbour searches on the entry
state), the baseline gate skipping one neighbour, bCoarse, mbMonocular with caller skips, calls composed across
neighbours, and the SearchForTriangulation overflow rerun inside the chain."""
import numpy as np
import pytest

from openmavis_amd import mapping, synth_cnmp
from openmavis_amd.matcher import ORBmatcher

pytestmark = pytest.mark.gpu


def _same(d, ref, got):
    hm_o, nm_o, outs_o, s_o = ref
    hm_g, nm_g, outs_g, s_g = got
    np.testing.assert_array_equal(nm_g, nm_o)
    for j, ((m_o, st_o, x_o), (m_g, st_g, x_g)) in enumerate(zip(outs_o, outs_g)):
        np.testing.assert_array_equal(m_g, m_o, err_msg=f"match12 neighbour {j}")
        np.testing.assert_array_equal(st_g, st_o, err_msg=f"status neighbour {j}")
        acc = st_o > 0
        assert np.array_equal(x_g[acc].view(np.uint32), x_o[acc].view(np.uint32)), j
    np.testing.assert_array_equal(hm_g, hm_o)
    assert s_g == s_o


@pytest.mark.parametrize("seed,n_neigh,inertial,coarse", [(3, 12, True, False), (4, 16, False, False),
                                                          (5, 12, True, True)])
def test_chain_matches_interleaved_oracle(oracle, seed, n_neigh, inertial, coarse):
    d = synth_cnmp.make_cnmp_chain(seed=seed, n_neigh=n_neigh)
    ref = oracle.local_mapping_create_new_map_points(d, inertial=inertial, coarse=coarse)
    got = mapping.CreateNewMapPoints(d, ORBmatcher(0.6, False), inertial=inertial, coarse=coarse)
    _same(d, ref, got)
    assert int(ref[0].sum() - d["kf1"]["has_mp"].sum()) > 300
    assert ref[1][0] == 0   # the first neighbour is under the baseline


def test_chain_monocular_with_caller_skips(oracle):
    """mbMonocular: no baseline gate, the caller's median-depth decisions arrive as skip flags."""
    d = synth_cnmp.make_cnmp_chain(seed=6, n_neigh=10)
    for j in (2, 7):
        d["nbs"][j]["skip"] = 1
    ref = oracle.local_mapping_create_new_map_points(d, monocular=True)
    got = mapping.CreateNewMapPoints(d, ORBmatcher(0.6, False), monocular=True)
    _same(d, ref, got)
    assert ref[1][2] == 0 and ref[1][7] == 0 and ref[1][0] > 0


def test_chain_calls_compose_and_overflow_rerun(oracle):
    """Three calls over consecutive neighbour ranges with has_mp1 / side-1 state carried on the device (entering side
    1 = the right camera) equal the oracle's single loop; then the same with a tiny slice workspace so every
    neighbour's search overflows into the one-workgroup rerun (gated on the device flag)."""
    import os
    import torch
    d = synth_cnmp.make_cnmp_chain(seed=7, n_neigh=12)
    ref = oracle.local_mapping_create_new_map_points(d, side1_state=1)
    for knob in (None, "64"):
        if knob:
            os.environ["OMV_TRI_ECAP"] = knob
        try:
            m = ORBmatcher(0.6, False)
            c = mapping.LocalMappingCall(d, m)
            c.run(0, 4, reset=True, side1_state=1)
            c.run(4, 9, reset=False)
            c.run(9, 12, reset=False)
            torch.cuda.synchronize()
        finally:
            os.environ.pop("OMV_TRI_ECAP", None)
        n1 = int(d["kf1"]["n"])
        got = (c.has_mp1[:n1].cpu().numpy(), c.n_matches.cpu().numpy(),
               [(a[:n1].cpu().numpy(), b[:n1].cpu().numpy(), x[:n1].cpu().numpy()) for a, b, x in c.outs],
               int(c.side1.item()))
        _same(d, ref, got)
