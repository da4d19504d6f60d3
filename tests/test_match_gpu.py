"""GPU parity of the HIP matchers (grid, lapping knn, SearchByProjection, knn2) against the oracle.

Bar: bit-exact — identical grids, knn indices/distances, keypoint->map-point assignments and match
counts (integer work).
"""
import numpy as np
import pytest

from openmavis_amd import synth
from openmavis_amd.matcher import FrameBatch, MapPointBatch, ORBmatcher, bf_knn2
from openmavis_amd.orb import ORBextractor

pytestmark = pytest.mark.gpu

W, H, C, NF = 720, 540, 5, 1200
LAP = np.array([[0, 720], [0, 720], [0, 0], [0, 0], [0, 0]], np.int32)


@pytest.fixture(scope="module")
def frames(torch_cuda):
    torch = torch_cuda
    n_frames = 3
    ex = ORBextractor(NF, 1.2, 8, 15, 7, width=W, height=H, max_images=n_frames * C)
    cap = ex.max_keypoints()
    imgs = np.concatenate([synth.hilti_frame(f) for f in range(n_frames)])
    fb = FrameBatch(torch, n_frames, C, cap, W, H, ex.GetScaleFactors())
    d_img = torch.from_numpy(imgs).cuda()
    ex.extract_batch(d_img, np.tile(LAP, (n_frames, 1)), fb.kps.view(-1, cap, 6), fb.desc.view(-1, cap, 32),
                     fb.n_kp.view(-1), fb.mono.view(-1))
    torch.cuda.synchronize()
    assert ex.last_error() == 0
    return fb


def host(fb, oracle):
    kps = fb.kps.cpu().numpy().view(oracle.KP_DTYPE).reshape(fb.n_frames, fb.n_cams, fb.kp_cap)
    return kps, fb.desc.cpu().numpy(), fb.n_kp.cpu().numpy(), fb.mono.cpu().numpy()


def test_grid_matches_oracle(frames, oracle):
    kps, desc, n_kp, mono = host(frames, oracle)
    m = ORBmatcher(0.8)
    m.AssignFeaturesToGrid(frames)
    for f in range(frames.n_frames):
        g = oracle.frame_geom(C, W, H, [frames.geom.scale_factors[i] for i in range(8)])
        for c in range(C):
            cs_o, idx_o = oracle.grid(g, kps[f], n_kp[f], c)
            cs_g, idx_g = m.grid(f, c)
            assert np.array_equal(cs_o, cs_g), f"frame {f} cam {c} cell starts differ"
            assert np.array_equal(idx_o, idx_g), f"frame {f} cam {c} cell contents differ"


def test_stereo_lapping_matches_oracle(frames, oracle):
    kps, desc, n_kp, mono = host(frames, oracle)
    m = ORBmatcher(0.8)
    m.StereoLapping(frames, 0.8)
    l2r = frames.l2r.cpu().numpy()
    r2l = frames.r2l.cpu().numpy()
    for f in range(frames.n_frames):
        q = desc[f, 0, mono[f, 0]:n_kp[f, 0]]
        t = desc[f, 1, mono[f, 1]:n_kp[f, 1]]
        i2, d2 = oracle.bf_knn2(q, t)
        el2r = np.full(frames.kp_cap, -1, np.int32)
        er2l = np.full(frames.kp_cap, -1, np.int32)
        for qi in range(len(q)):
            if i2[qi, 1] >= 0 and float(d2[qi, 0]) < float(d2[qi, 1]) * 0.8:
                el2r[mono[f, 0] + qi] = mono[f, 1] + i2[qi, 0]
                er2l[mono[f, 1] + i2[qi, 0]] = mono[f, 0] + qi
        assert np.array_equal(el2r, l2r[f]) and np.array_equal(er2l, r2l[f]), f"frame {f}"
        assert (el2r >= 0).sum() > 5


def test_stereo_triangulate_matches_oracle(frames, oracle):
    """ComputeMultiFishEyeMatches' TriangulateMatches depth check (Frame.cc:1488-1512) on the lapping knn
    pairs: kept pairs, r2l, mvDepth and mvStereo3Dpoints bit-exact vs the oracle."""
    from openmavis_amd import synth_ba
    kps, desc, n_kp, mono = host(frames, oracle)
    cams, Rbc, tbc = synth_ba.rig()
    Rlr = (Rbc[0].T @ Rbc[1]).astype(np.float32)
    tlr = (Rbc[0].T @ (tbc[1] - tbc[0])).astype(np.float32)
    sigma2 = np.array([frames.geom.scale_factors[i] for i in range(8)], np.float32) ** 2
    m = ORBmatcher(0.8)
    m.StereoLapping(frames, 0.8)
    cand = frames.l2r.cpu().numpy().copy()
    m.StereoTriangulate(frames, cams[:2], Rlr, tlr, sigma2)
    l2r, r2l = frames.l2r.cpu().numpy(), frames.r2l.cpu().numpy()
    depth, p3d = frames.depth.cpu().numpy(), frames.p3d.cpu().numpy()
    kept = 0
    for f in range(frames.n_frames):
        nL, nR = n_kp[f, 0], n_kp[f, 1]
        el2r, er2l, ed, ep = oracle.stereo_triangulate(kps[f, 0], nL, kps[f, 1], nR, cams[:2], Rlr, tlr, sigma2,
                                                       cand[f])
        assert np.array_equal(l2r[f, :nL], el2r), f"frame {f} l2r"
        assert np.array_equal(r2l[f, :nR], er2l), f"frame {f} r2l"
        assert np.array_equal(depth[f, :nL].view(np.uint32), ed.view(np.uint32)), f"frame {f} depth"
        ok = el2r >= 0
        assert np.array_equal(p3d[f, :nL][ok].view(np.uint32), ep[ok].view(np.uint32)), f"frame {f} p3D"
        kept += int(ok.sum())
    assert (cand >= 0).sum() > 0
    # the tool's own hook: TriangulateMatches pieces on one device thread agree with the oracle's
    import ctypes
    from openmavis_amd import _lib
    f = int(np.argmax((l2r >= 0).sum(1)))
    i = int(np.nonzero(l2r[f] >= 0)[0][0]) if (l2r[f] >= 0).any() else int(np.nonzero(cand[f] >= 0)[0][0])
    r = int(cand[f, i])
    out = np.zeros(31, np.float32)
    _lib.check(_lib.load().omv_tri_debug(_lib.ptr(np.ascontiguousarray(cams[:2], np.float32)),
                                         _lib.ptr(np.ascontiguousarray(kps[f, 0, i:i + 1])),
                                         _lib.ptr(np.ascontiguousarray(kps[f, 1, r:r + 1])), _lib.ptr(Rlr), _lib.ptr(tlr),
                                         _lib.ptr(np.eye(4, dtype=np.float32)), ctypes.c_float(sigma2[kps[f, 0, i]["octave"]]),
                                         ctypes.c_float(sigma2[kps[f, 1, r]["octave"]]), _lib.ptr(out)), "omv_tri_debug")
    assert np.array_equal(out[:3].view(np.uint32), oracle.kb8_unproject(cams[0], kps[f, 0, i]["x"], kps[f, 0, i]["y"]).view(np.uint32))
    assert np.array_equal(out[6:22].reshape(4, 4), np.eye(4, dtype=np.float32))   # the SVD of I is I


def _mps_for(frames, oracle, M, seed, torch):
    kps, desc, n_kp, _ = host(frames, oracle)
    per = [synth.make_map_points(kps[f], desc[f], n_kp[f], M, seed + f, W, H) for f in range(frames.n_frames)]
    stacked = {k: np.stack([p[k] for p in per]) for k in per[0]}
    dev = {k: torch.from_numpy(v).cuda() for k, v in stacked.items()}
    return per, MapPointBatch(**dev)


@pytest.mark.parametrize("th,far,nnratio,occ_frac,obs,rand_stereo", [
    (6.0, False, 0.8, 0.0, None, False),
    (1.0, False, 0.8, 0.0, 1.0, False),
    (3.0, True, 0.6, 0.05, None, False),
    (15.0, False, 0.9, 0.02, 1.0, False),
    # many points without observations + dense stereo links + occupied keypoints: exercises
    # overwrites of blocked keypoints (unblocking) and freed initially-occupied keypoints
    (6.0, False, 0.8, 0.25, 0.5, True),
    (10.0, False, 1.0, 0.1, 0.0, True),
])
def test_search_by_projection_matches_oracle(frames, oracle, torch_cuda, th, far, nnratio, occ_frac, obs,
                                             rand_stereo):
    _sbp_case(frames, oracle, torch_cuda, th, far, nnratio, occ_frac, obs, rand_stereo)


@pytest.mark.parametrize("env", [dict(OMV_CAND="global"), dict(OMV_CAND="lds"), dict(OMV_CAND="lds", OMV_CAND_PW="128"),
                                 dict(OMV_CAND="lds", OMV_CAND_PW="64")])
@pytest.mark.parametrize("case", [(6.0, False, 0.8, 0.25, 0.5, True), (15.0, False, 0.9, 0.02, 1.0, False)])
def test_search_by_projection_candidate_paths(frames, oracle, torch_cuda, monkeypatch, env, case):
    """The candidate stage's variants: keypoints staged in LDS per (frame, camera, chunk of map points) -- the
    batched path; forced here on 3 frames, also with the bench's large chunks (partial last chunk) -- and the
    global-memory gather kernel (8 lanes per window at this size); same assignments as the oracle."""
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    _sbp_case(frames, oracle, torch_cuda, *case)


@pytest.mark.parametrize("case", [(6.0, False, 0.8, 0.25, 0.5, True), (15.0, False, 0.9, 0.02, 1.0, False)])
def test_search_by_projection_small_batch_lanes(frames, oracle, torch_cuda, case):
    """3 frames x 4,000 points x 5 cameras = 60,000 slots: the 16-lanes-per-window candidate kernel of one- or
    two-frame calls (the latency path), against the oracle."""
    _sbp_case(frames, oracle, torch_cuda, *case, M=4000)


def _sbp_case(frames, oracle, torch_cuda, th, far, nnratio, occ_frac, obs, rand_stereo, M=5000):
    torch = torch_cuda
    per, mpb = _mps_for(frames, oracle, M, 7 + int(th), torch)
    rng0 = np.random.default_rng(int(th * 10) + int(occ_frac * 100))
    if obs is not None:
        for f, p in enumerate(per):
            p["has_obs"][:] = (rng0.random(M) < obs).astype(np.uint8)
        mpb.has_obs.copy_(torch.from_numpy(np.stack([p["has_obs"] for p in per])))
    m = ORBmatcher(nnratio)
    m.StereoLapping(frames, 0.8)
    if rand_stereo:
        _, _, n_kp, _ = host(frames, oracle)
        l2r = np.full((frames.n_frames, frames.kp_cap), -1, np.int32)
        r2l = np.full((frames.n_frames, frames.kp_cap), -1, np.int32)
        for f in range(frames.n_frames):
            n = min(n_kp[f, 0], n_kp[f, 1])
            left = rng0.permutation(n_kp[f, 0])[: n // 2]
            right = rng0.permutation(n_kp[f, 1])[: n // 2]
            l2r[f, left] = right
            r2l[f, right] = left
        frames.l2r.copy_(torch.from_numpy(l2r))
        frames.r2l.copy_(torch.from_numpy(r2l))
    rng = np.random.default_rng(11)
    S = C * frames.kp_cap
    occ = (rng.random((frames.n_frames, S)) < occ_frac).astype(np.uint8)
    init = np.where(occ > 0, 123456, -1).astype(np.int32)
    frames.occ_init = torch.from_numpy(occ).cuda()
    frames.kp_to_mp.copy_(torch.from_numpy(init))
    m.SearchByProjection(frames, mpb, th, far, 20.0)
    torch.cuda.synchronize()
    got = frames.kp_to_mp.cpu().numpy()
    got_n = frames.n_matches.cpu().numpy()
    kps, desc, n_kp, _ = host(frames, oracle)
    l2r, r2l = frames.l2r.cpu().numpy(), frames.r2l.cpu().numpy()
    g = oracle.frame_geom(C, W, H, [frames.geom.scale_factors[i] for i in range(8)])
    for f in range(frames.n_frames):
        exp = init[f].copy()
        n = oracle.search_by_projection(g, kps[f], desc[f], n_kp[f], per[f], th, far, 20.0, nnratio, l2r[f], r2l[f],
                                        occ[f], exp)
        assert n == got_n[f], f"frame {f}: nmatches {got_n[f]} != {n}"
        bad = np.nonzero(exp != got[f])[0]
        assert bad.size == 0, f"frame {f}: {bad.size} assignments differ, first slots {bad[:8]}"
        assert n > 300
    assert m.last_error() == 0
    frames.occ_init = None
    frames.kp_to_mp.fill_(-1)


def test_knn2_matches_oracle_with_ties(oracle, torch_cuda):
    torch = torch_cuda
    rng = np.random.default_rng(5)
    P, Q, T = 3, 700, 900
    base = rng.integers(0, 256, (64, 32), dtype=np.uint8)   # few distinct rows -> many ties
    q = base[rng.integers(0, 64, (P, Q))]
    t = base[rng.integers(0, 64, (P, T))]
    t[1, :5] = base[0]
    nq = np.array([Q, 300, 1], np.int32)
    nt = np.array([T, 1, 0], np.int32)
    i2, d2 = bf_knn2(torch.from_numpy(q).cuda(), torch.from_numpy(nq).cuda(), torch.from_numpy(t).cuda(),
                     torch.from_numpy(nt).cuda())
    i2, d2 = i2.cpu().numpy(), d2.cpu().numpy()
    for p in range(P):
        ei, ed = oracle.bf_knn2(q[p, :nq[p]], t[p, :nt[p]])
        assert np.array_equal(ei, i2[p, :nq[p]]) and np.array_equal(ed, d2[p, :nq[p]]), f"pair {p}"


def test_frustum_then_search_by_projection_matches_oracle(frames, oracle, torch_cuda):
    """Frame::isInFrustum on device (bit-exact projections, levels, view cosines, depths) feeding
    SearchByProjection, against the oracle's isInFrustum -> SearchByProjection on the same 3-D maps."""
    from openmavis_amd.matcher import isInFrustum, make_rig
    torch = torch_cuda
    M = 4000
    kps, desc, n_kp, _ = host(frames, oracle)
    cams, R_cl, t_cl = synth.hilti_rig(C)
    rig = make_rig(cams, R_cl, t_cl, W, H)
    rng = np.random.default_rng(5)
    poses = np.stack([synth.random_pose(rng) for _ in range(frames.n_frames)])
    maps = [synth.make_world_map(kps[f], desc[f], n_kp[f], M, 40 + f, cams, R_cl, t_cl, poses[f], W, H)
            for f in range(frames.n_frames)]
    world = {k: torch.from_numpy(np.stack([w[k] for w, _ in maps])).cuda() for k in maps[0][0]}
    mpb = MapPointBatch(**{k: torch.from_numpy(np.stack([p[k] for _, p in maps])).cuda() for k in maps[0][1]})
    n_in = torch.zeros(frames.n_frames, dtype=torch.int32, device="cuda")
    isInFrustum(torch.from_numpy(poses).cuda(), rig, world, mpb, 0.5, n_in)
    torch.cuda.synchronize()
    exp_tracks = []
    for f, (w, p) in enumerate(maps):
        exp, n = oracle.frustum(rig, poses[f], w["pos"], w["normal"], w["min_dist"], w["max_dist"], 0.5,
                                p["view_cos"], p["track_depth"])
        for k in ("in_view", "level"):
            assert np.array_equal(getattr(mpb, k)[f].cpu().numpy(), exp[k]), (f, k)
        for k in ("proj_x", "proj_y", "view_cos", "track_depth"):
            g = getattr(mpb, k)[f].cpu().numpy()
            assert np.array_equal(g.view(np.uint32), exp[k].view(np.uint32)), (f, k, np.abs(g - exp[k]).max())
        assert int(n_in[f].item()) == n and n > M // 4
        exp_tracks.append(dict(p, **exp))
    m = ORBmatcher(0.8)
    m.StereoLapping(frames, 0.8)
    frames.kp_to_mp.fill_(-1)
    m.SearchByProjection(frames, mpb, 6.0, False, 50.0)
    torch.cuda.synchronize()
    got, got_n = frames.kp_to_mp.cpu().numpy(), frames.n_matches.cpu().numpy()
    l2r, r2l = frames.l2r.cpu().numpy(), frames.r2l.cpu().numpy()
    g = oracle.frame_geom(C, W, H, [frames.geom.scale_factors[i] for i in range(8)])
    for f in range(frames.n_frames):
        exp = np.full(C * frames.kp_cap, -1, np.int32)
        n = oracle.search_by_projection(g, kps[f], desc[f], n_kp[f], exp_tracks[f], 6.0, False, 50.0, 0.8, l2r[f],
                                        r2l[f], None, exp)
        assert n == got_n[f] and np.array_equal(exp, got[f]), f"frame {f}"
        assert n > 300
    frames.kp_to_mp.fill_(-1)


@pytest.mark.parametrize("motion,check_ori,model", [("none", True, "kb8"), ("forward", True, "kb8"),
                                                   ("backward", False, "kb8"), ("none", True, "pinhole"),
                                                   ("forward", False, "pinhole")])
def test_search_by_projection_last_frame_matches_oracle(frames, oracle, torch_cuda, motion, check_ori, model):
    """SearchByProjection(Frame&, const Frame& LastFrame, th, bMono) on device vs the oracle: assignments
    (last-frame slots), counts, the rotation-histogram removals; forward / backward / neither window.  model
    "pinhole": CurrentFrame.mpCamera is a Pinhole (configs[3]'s rig type; ORBmatcher.cc:2022, :2134)."""
    torch = torch_cuda
    pin = model == "pinhole"
    for c in range(C):
        frames.geom.cam_model[c] = 1 if pin else 0
    kps, desc, n_kp, _ = host(frames, oracle)
    cams, R_cl, t_cl = synth.hilti_rig(C)
    rng = np.random.default_rng({"none": 1, "forward": 2, "backward": 3}[motion])
    F, cap = frames.n_frames, frames.kp_cap
    Tcw = np.stack([synth.random_se3(rng) for _ in range(F)])
    lasts = [synth.make_last_frame(kps[f], desc[f], n_kp[f], 90 + f, cams, Tcw[f], pinhole=pin) for f in range(F)]
    # last pose: the current one moved along the optical axis (tlc.z vs mb decides the level window)
    dz = {"none": 0.0, "forward": 0.5, "backward": -0.5}[motion]
    Tlw = Tcw.copy()
    Tlw[:, 6] -= np.float32(dz)
    Trl_R = R_cl[1].astype(np.float64)
    Trl = np.concatenate([synth.quat_from_R(Trl_R), t_cl[1]]).astype(np.float32)
    mb = 0.11
    last = {k: torch.from_numpy(np.stack([l[k] for l in lasts])).cuda() for k in ("pos", "desc", "valid", "has_obs")}
    last["kps"] = torch.from_numpy(np.stack([l["kps"].view(np.int32).reshape(-1, 6) for l in lasts])).cuda()
    occ = (rng.random((F, C * cap)) < 0.03).astype(np.uint8)
    frames.occ_init = torch.from_numpy(occ).cuda()
    frames.kp_to_mp.fill_(-1)
    m = ORBmatcher(0.9, checkOri=check_ori)
    try:
        m.SearchByProjectionLastFrame(frames, last, torch.from_numpy(Tcw).cuda(), torch.from_numpy(Tlw).cuda(), cams,
                                      Trl, th=7.0, bMono=False, mb=mb)
        torch.cuda.synchronize()
    finally:
        for c in range(C):
            frames.geom.cam_model[c] = 0
    got, got_n = frames.kp_to_mp.cpu().numpy(), frames.n_matches.cpu().numpy()
    g = oracle.frame_geom(C, W, H, [frames.geom.scale_factors[i] for i in range(8)], [1 if pin else 0] * C)
    for f in range(F):
        exp = np.full(C * cap, -1, np.int32)
        n = oracle.search_last_frame(g, kps[f], desc[f], n_kp[f], cams, Tcw[f], Tlw[f], Trl, lasts[f]["pos"],
                                     lasts[f]["desc"], lasts[f]["valid"], lasts[f]["has_obs"], lasts[f]["kps"], 7.0,
                                     False, mb, check_ori, occ[f], exp)
        bad = np.nonzero(exp != got[f])[0]
        assert n == got_n[f] and bad.size == 0, (f, n, int(got_n[f]), bad[:8])
        assert n > 200
    frames.occ_init = None
    frames.kp_to_mp.fill_(-1)


def test_search_by_projection_stereo_partner_revives_right_keypoint(frames, oracle, torch_cuda):
    """A left-block claim by a point without observations writes the stereo partner's slot
    (ORBmatcher.cc:125-131); if that right keypoint was occupied at the call, it becomes free for the same
    point's right-block search (:150-160).  Geometrically coherent l2r pairs: the right keypoint sits at the
    point's right-camera projection, half of them initially occupied, most points without observations."""
    torch = torch_cuda
    M = 3000
    per, mpb = _mps_for(frames, oracle, M, 77, torch)
    kps, desc, n_kp, _ = host(frames, oracle)
    rng = np.random.default_rng(99)
    cap = frames.kp_cap
    l2r = np.full((frames.n_frames, cap), -1, np.int32)
    r2l = np.full((frames.n_frames, cap), -1, np.int32)
    occ = np.zeros((frames.n_frames, C * cap), np.uint8)
    for f, p in enumerate(per):
        nl, nr = int(n_kp[f, 0]), int(n_kp[f, 1])
        # points seen by block 0 at (near) a left keypoint: pair that keypoint with a right keypoint and let the
        # point see block 1 exactly there
        px, py = p["proj_x"][:, 0], p["proj_y"][:, 0]
        seen = np.nonzero(p["in_view"][:, 0] > 0)[0]
        right = rng.permutation(nr)
        used_l = set()
        k = 0
        for pi in seen:
            d = (kps[f, 0, :nl]["x"] - px[pi]) ** 2 + (kps[f, 0, :nl]["y"] - py[pi]) ** 2
            li = int(np.argmin(d))
            if d[li] > 4.0 or li in used_l or k >= nr:
                continue
            used_l.add(li)
            ri = int(right[k])
            k += 1
            l2r[f, li], r2l[f, ri] = ri, li
            p["proj_x"][pi, 1] = kps[f, 1, ri]["x"]
            p["proj_y"][pi, 1] = kps[f, 1, ri]["y"]
            p["level"][pi, 1] = kps[f, 1, ri]["octave"]
            p["in_view"][pi, 1] = 1
            p["view_cos"][pi, 1] = 0.999
            if rng.random() < 0.5:
                occ[f, cap + ri] = 1
        p["has_obs"][:] = (rng.random(M) < 0.2).astype(np.uint8)
        assert k > 100
    for key in ("proj_x", "proj_y", "level", "in_view", "view_cos", "has_obs"):
        getattr(mpb, key).copy_(torch.from_numpy(np.stack([p[key] for p in per])))
    frames.l2r.copy_(torch.from_numpy(l2r))
    frames.r2l.copy_(torch.from_numpy(r2l))
    init = np.where(occ > 0, 123456, -1).astype(np.int32)
    frames.occ_init = torch.from_numpy(occ).cuda()
    frames.kp_to_mp.copy_(torch.from_numpy(init))
    m = ORBmatcher(0.8)
    m.SearchByProjection(frames, mpb, 6.0, False, 50.0)
    torch.cuda.synchronize()
    got, got_n = frames.kp_to_mp.cpu().numpy(), frames.n_matches.cpu().numpy()
    g = oracle.frame_geom(C, W, H, [frames.geom.scale_factors[i] for i in range(8)])
    for f in range(frames.n_frames):
        exp = init[f].copy()
        n = oracle.search_by_projection(g, kps[f], desc[f], n_kp[f], per[f], 6.0, False, 50.0, 0.8, l2r[f], r2l[f],
                                        occ[f], exp)
        bad = np.nonzero(exp != got[f])[0]
        assert n == got_n[f] and bad.size == 0, (f, n, int(got_n[f]), bad[:8])
        # right keypoints freed by their own point's partner claim and then matched by it in block 1
        assert ((exp[cap:2 * cap] >= 0) & (exp[cap:2 * cap] != 123456) & (occ[f, cap:2 * cap] > 0)).sum() > 10
    assert m.last_error() == 0
    frames.occ_init = None
    frames.kp_to_mp.fill_(-1)
