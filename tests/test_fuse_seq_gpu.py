"""GPU parity of LocalMapping::SearchInNeighbors' fuse sequence (omv_search_in_neighbors_fuse: window searches on the
device, speculative per phase, entries re-evaluated after a Replace survivor's descriptor recomputation -- itself on
the device -- and the decisions walked in the reference's order) against the literal restatement
(oracle/match_oracle.cpp oracle_search_in_neighbors_fuse, src/LocalMapping.cc:837-889): the final mvpMapPoints of
every keyframe, isBad / mpReplaced / nObs / mObservations of every map point, the ordered edit log, nFused per Fuse
call and the final descriptors -- all exact, on maps whose duplicate points make hundreds of Replace calls."""
import numpy as np
import pytest

from openmavis_amd import mapping, synth_fuse
from openmavis_amd.matcher import ORBmatcher

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("seed,n_targets", [(1, 8), (2, 12), (3, 4)])
def test_fuse_sequence_matches_oracle(oracle, seed, n_targets):
    s = synth_fuse.make_fuse_scene(seed=seed, n_targets=n_targets)
    ref = oracle.search_in_neighbors_fuse(s)
    got = mapping.SearchInNeighborsFuse(s, ORBmatcher(0.6))
    for k in ("n_fused", "log", "kf_mps", "bad", "replaced", "n_obs", "obs_start", "obs_kf", "obs_idx", "desc"):
        np.testing.assert_array_equal(np.asarray(got[k]).ravel(), np.asarray(ref[k]).ravel(), err_msg=k)
    assert (ref["log"][:, 0] == 1).sum() > 50
    assert got["n_reevaluated"] > 0   # Replace survivors were searched again with their new descriptors
