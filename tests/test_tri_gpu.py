"""GPU parity of SearchForTriangulation (openmavis_amd/csrc/tri.hip) against the CPU oracle
(oracle/tri_oracle.cpp): vMatches12 and the match count bit-exact (integer / index output; the float
triangulation is restated op-for-op on both sides, glibc tanf / atan2f included)."""
import numpy as np
import pytest

from openmavis_amd import synth_tri
from openmavis_amd.matcher import ORBmatcher

pytestmark = pytest.mark.gpu


def _device_pairs(pairs):
    import torch
    out = []
    for p in pairs:
        q = dict(T=p["T"])
        for k in ("kf1", "kf2"):
            kf = p[k]
            d = {f: kf[f] for f in ("n", "n_left", "n_right", "n_sideleft")}
            d["kps"] = torch.from_numpy(kf["kps"].view(np.float32).reshape(-1, 6).copy()).cuda()
            for f in ("desc", "has_mp", "node_start", "node_idx"):
                d[f] = torch.from_numpy(np.ascontiguousarray(kf[f])).cuda()
            d["node_id"] = torch.from_numpy(kf["node_id"].view(np.int32).copy()).cuda()
            d["level_sigma2"] = p["level_sigma2"]
            q[k] = d
        q["match12"] = torch.full((p["kf1"]["n"],), -9, dtype=torch.int32, device="cuda")
        out.append(q)
    return out


@pytest.mark.parametrize("check_ori,coarse", [(False, False), (True, False), (False, True)])
def test_search_for_triangulation_matches_oracle(oracle, check_ori, coarse):
    pairs = [synth_tri.make_tri_pair(seed=s, n_pts=400 + 50 * s) for s in range(1, 9)]
    dp = _device_pairs(pairs)
    m = ORBmatcher(0.6, check_ori)
    n = m.SearchForTriangulation(dp, pairs[0]["cams"], bCoarse=coarse).cpu().numpy()
    for i, p in enumerate(pairs):
        n_o, m_o = oracle.search_for_triangulation(p, coarse=coarse, check_ori=check_ori)
        assert n[i] == n_o, (i, n[i], n_o)
        assert np.array_equal(dp[i]["match12"].cpu().numpy(), m_o), i


def test_search_for_triangulation_edge_cases(oracle):
    """All keypoints already carry map points; bOnlyStereo on multi-camera keyframes; an empty pair."""
    p = synth_tri.make_tri_pair(seed=11)
    p_full = dict(p, kf1=dict(p["kf1"], has_mp=np.ones_like(p["kf1"]["has_mp"])))
    dp = _device_pairs([p, p_full])
    m = ORBmatcher(0.6, False)
    assert m.SearchForTriangulation(dp[:1], p["cams"], bOnlyStereo=True).cpu().numpy()[0] == 0
    n = m.SearchForTriangulation(dp, p["cams"]).cpu().numpy()
    assert n[1] == 0 and (dp[1]["match12"].cpu().numpy() == -1).all()
    assert n[0] == oracle.search_for_triangulation(p)[0]


@pytest.mark.parametrize("kw", [dict(n_pts=1500, n_distract=600),          # several replay batches
                                dict(n_pts=600, n_distract=300, n_nodes=3),   # few huge nodes: tiles span rows
                                dict(n_pts=900, n_distract=300, n_nodes=4000),  # many tiny nodes, > 1 segment
                                dict(n_pts=500, cams_used=2)])                 # only listed L/R pairs
def test_search_for_triangulation_shapes(oracle, kw):
    """Bench-size and skewed FeatureVector layouts: batch / tile / segment boundaries of the device scan."""
    pairs = [synth_tri.make_tri_pair(seed=30 + s, **kw) for s in range(3)]
    dp = _device_pairs(pairs)
    m = ORBmatcher(0.6, True)
    n = m.SearchForTriangulation(dp, pairs[0]["cams"]).cpu().numpy()
    for i, p in enumerate(pairs):
        n_o, m_o = oracle.search_for_triangulation(p, check_ori=True)
        assert n[i] == n_o, (i, n[i], n_o)
        assert np.array_equal(dp[i]["match12"].cpu().numpy(), m_o), i


@pytest.mark.parametrize("knobs", [dict(OMV_TRI_SLICES="1"), dict(OMV_TRI_SLICES="64"),
                                   dict(OMV_TRI_SLICES="1", OMV_TRI_WALK="seq"), dict(OMV_TRI_WALK="seq"),
                                   dict(OMV_TRI_ECAP="64"), dict(OMV_TRI_SLICES="3", OMV_TRI_ECAP="200")])
def test_search_for_triangulation_slices_and_rerun(oracle, monkeypatch, knobs):
    """The sliced search (scan / flat epipolar tests / walk) at one slice (the entering camera-pair state always
    known), at 64 slices (most slices enter with the state unknown and test every state up to their first anchor),
    with the scalar walk instead of the per-row state maps, and with entry capacities small enough that pairs
    overflow and are rerun by the one-workgroup kernel."""
    for k, v in knobs.items():
        monkeypatch.setenv(k, v)
    pairs = [synth_tri.make_tri_pair(seed=50 + s, n_pts=700, n_distract=300) for s in range(4)]
    dp = _device_pairs(pairs)
    m = ORBmatcher(0.6, True)
    n = m.SearchForTriangulation(dp, pairs[0]["cams"]).cpu().numpy()
    for i, p in enumerate(pairs):
        n_o, m_o = oracle.search_for_triangulation(p, check_ori=True)
        assert n[i] == n_o, (i, n[i], n_o)
        assert np.array_equal(dp[i]["match12"].cpu().numpy(), m_o), i


@pytest.mark.parametrize("model", ["pinhole", ["pinhole", "kb8", "kb8", "pinhole"], ["kb8", "pinhole", "pinhole", "kb8"]])
@pytest.mark.parametrize("check_ori", [False, True])
def test_search_for_triangulation_pinhole_rig(oracle, model, check_ori):
    """configs[3]'s camera type: pCamera1->epipolarConstrain dispatches to Pinhole::epipolarConstrain (F12 = K1^-T
    [t12]x R12 K2^-1, dsqr < 3.84 sigma2[kp2.octave]; Pinhole.cpp:103-132) -- and on mixed rigs KannalaBrandt8's
    TriangulateMatches unprojects / projects camera 2 with its own type.  vMatches12 and counts bit-exact."""
    pairs = [synth_tri.make_tri_pair(seed=60 + s, n_pts=400 + 60 * s, model=model) for s in range(6)]
    dp = _device_pairs(pairs)
    m = ORBmatcher(0.6, check_ori)
    n = m.SearchForTriangulation(dp, pairs[0]["cams"], cam_model=pairs[0]["cam_model"]).cpu().numpy()
    total = 0
    for i, p in enumerate(pairs):
        n_o, m_o = oracle.search_for_triangulation(p, check_ori=check_ori)
        assert n[i] == n_o, (i, n[i], n_o)
        assert np.array_equal(dp[i]["match12"].cpu().numpy(), m_o), i
        total += n_o
    assert total > 300
    # the camera type changes the result (a KB8 run of the same Pinhole data differs)
    if model == "pinhole":
        kb = [dict(p, cam_model=None) for p in pairs]
        assert sum(oracle.search_for_triangulation(p, check_ori=check_ori)[0] for p in kb) != total
