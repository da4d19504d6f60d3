"""GPU parity of LocalMapping::CreateNewMapPoints' geometry (openmavis_amd/csrc/tri.hip cnmp_kernel) against the oracle
restatement (oracle/tri_oracle.cpp): per neighbour the accepted / rejected status of every match bit-exact and the new
points' coordinates as raw float32 bits -- the multi-camera KannalaBrandt8 rig (camera-pair state across matches and
neighbours) and a Pinhole stereo rig (the stereo parallax and UnprojectStereo branches), inertial and not, far-point
filter on and off, the baseline gate on and off (jobs in order, side-1 state carried)."""
import numpy as np
import pytest

from openmavis_amd import mapping, synth_cnmp

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("multi,inertial,far,cb", [(True, True, False, False), (True, False, False, True),
                                                   (False, True, False, False), (False, False, True, True),
                                                   (True, True, True, False)])
def test_create_new_map_points_match_oracle(oracle, multi, inertial, far, cb):
    d = synth_cnmp.make_cnmp(seed=11 if multi else 12, n_neigh=6, multi=multi)
    ref = oracle.create_new_map_points(d, inertial=inertial, far_points=far, th_far=12.0, check_baseline=cb)
    got = mapping.CreateNewMapPointsGeometry(d, inertial=inertial, far_points=far, th_far=12.0, check_baseline=cb)
    n_acc = 0
    for (st_o, x_o), (st_g, x_g) in zip(ref, got):
        st_g, x_g = st_g.cpu().numpy(), x_g.cpu().numpy()
        assert np.array_equal(st_g, st_o)
        acc = st_o > 0
        n_acc += int(acc.sum())
        assert np.array_equal(x_g[acc].view(np.uint32), x_o[acc].view(np.uint32))
    assert n_acc > 200
    if not multi:
        assert sum(int((st == 2).sum()) for st, _ in ref) > 0
