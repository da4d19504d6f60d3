"""BASELINE configs[3]: the synthetic 8-camera Pinhole rig, 1920x1080, 2000 features per camera (iniTh 20,
minTh 7, lapping [0, 0]; the reference's multi Frame ctor would static_cast Pinhole cameras to KannalaBrandt8
to read the lapping area, Frame.cc:1847-1855, so it is passed explicitly).

Bar: bit-exact vs the oracle — every keypoint field as raw bits, order, monoIndex, descriptors; then
Frame::isInFrustum through Pinhole::project (Pinhole.cpp:26-32) and SearchByProjection over the 8 blocks.
"""
import numpy as np
import pytest

from openmavis_amd import synth
from openmavis_amd.matcher import FrameBatch, MapPointBatch, ORBmatcher, isInFrustum, make_rig
from openmavis_amd.orb import ORBextractor

pytestmark = pytest.mark.gpu

W, H, C, NF, INI, MIN = 1920, 1080, 8, 2000, 20, 7
N_FRAMES = 2


@pytest.fixture(scope="module")
def p1080(torch_cuda, oracle):
    torch = torch_cuda
    imgs = np.concatenate([synth.rig_frame(f, C, W, H, synth.P1080_SEED) for f in range(N_FRAMES)])
    lap = np.zeros((N_FRAMES * C, 2), np.int32)
    ex = ORBextractor(NF, 1.2, 8, INI, MIN, width=W, height=H, max_images=N_FRAMES * C)
    cap = ex.max_keypoints()
    fb = FrameBatch(torch, N_FRAMES, C, cap, W, H, ex.GetScaleFactors())
    ex.extract_batch(torch.from_numpy(imgs).cuda(), lap, fb.kps.view(-1, cap, 6), fb.desc.view(-1, cap, 32),
                     fb.n_kp.view(-1), fb.mono.view(-1))
    torch.cuda.synchronize()
    assert ex.last_error() == 0, "capacity error at 1920x1080 / 2000 features"
    return imgs, ex, fb


def test_extract_8x1080p_matches_oracle(p1080, oracle):
    imgs, ex, fb = p1080
    cap = fb.kp_cap
    kps = fb.kps.cpu().numpy().view(oracle.KP_DTYPE).reshape(N_FRAMES, C, cap)
    desc = fb.desc.cpu().numpy()
    n_kp, mono = fb.n_kp.cpu().numpy(), fb.mono.cpu().numpy()
    for f in range(N_FRAMES):
        n_o, m_o, k_o, d_o = oracle.orb_extract_frame(imgs[f * C:(f + 1) * C], NF, np.zeros((C, 2), np.int32), 1.2, 8,
                                                      INI, MIN)
        for c in range(C):
            n = int(n_kp[f, c])
            assert n == n_o[c] and mono[f, c] == m_o[c], (f, c, n, int(n_o[c]))
            assert n >= NF - 10
            for fld in ("x", "y", "size", "angle", "response", "octave"):
                bad = np.nonzero(kps[f, c, :n][fld].view(np.uint32) != k_o[c, :n][fld].view(np.uint32))[0]
                assert bad.size == 0, (f, c, fld, bad[:8])
            assert np.array_equal(desc[f, c, :n], d_o[c, :n]), (f, c)


def test_pinhole_frustum_then_search_by_projection_8x1080p(p1080, oracle, torch_cuda):
    torch = torch_cuda
    _, ex, fb = p1080
    cap = fb.kp_cap
    kps = fb.kps.cpu().numpy().view(oracle.KP_DTYPE).reshape(N_FRAMES, C, cap)
    desc, n_kp = fb.desc.cpu().numpy(), fb.n_kp.cpu().numpy()
    cams, R_cl, t_cl = synth.p1080_rig(C, W, H)
    rig = make_rig(cams, R_cl, t_cl, W, H, model="pinhole")
    rng = np.random.default_rng(8)
    M = 6000
    poses = np.stack([synth.random_pose(rng) for _ in range(N_FRAMES)])
    maps = [synth.make_world_map(kps[f], desc[f], n_kp[f], M, 60 + f, cams, R_cl, t_cl, poses[f], W, H,
                                 model="pinhole") for f in range(N_FRAMES)]
    world = {k: torch.from_numpy(np.stack([w[k] for w, _ in maps])).cuda() for k in maps[0][0]}
    mpb = MapPointBatch(**{k: torch.from_numpy(np.stack([p[k] for _, p in maps])).cuda() for k in maps[0][1]})
    n_in = torch.zeros(N_FRAMES, dtype=torch.int32, device="cuda")
    isInFrustum(torch.from_numpy(poses).cuda(), rig, world, mpb, 0.5, n_in)
    torch.cuda.synchronize()
    tracks = []
    for f, (w, p) in enumerate(maps):
        exp, n = oracle.frustum(rig, poses[f], w["pos"], w["normal"], w["min_dist"], w["max_dist"], 0.5,
                                p["view_cos"], p["track_depth"])
        for k in ("in_view", "level"):
            assert np.array_equal(getattr(mpb, k)[f].cpu().numpy(), exp[k]), (f, k)
        for k in ("proj_x", "proj_y", "view_cos", "track_depth"):
            g = getattr(mpb, k)[f].cpu().numpy()
            assert np.array_equal(g.view(np.uint32), exp[k].view(np.uint32)), (f, k)
        assert int(n_in[f].item()) == n and n > M // 3
        assert (exp["in_view"].sum(1) > 1).sum() > 0   # some points seen by two blocks of the ring
        tracks.append(dict(p, **exp))
    m = ORBmatcher(0.8)
    fb.l2r.fill_(-1)
    fb.r2l.fill_(-1)
    fb.kp_to_mp.fill_(-1)
    m.SearchByProjection(fb, mpb, 3.0, False, 50.0)
    torch.cuda.synchronize()
    assert m.last_error() == 0
    got, got_n = fb.kp_to_mp.cpu().numpy(), fb.n_matches.cpu().numpy()
    g = oracle.frame_geom(C, W, H, ex.GetScaleFactors())
    no_link = np.full(cap, -1, np.int32)
    for f in range(N_FRAMES):
        exp = np.full(C * cap, -1, np.int32)
        n = oracle.search_by_projection(g, kps[f], desc[f], n_kp[f], tracks[f], 3.0, False, 50.0, 0.8, no_link,
                                        no_link, None, exp)
        bad = np.nonzero(exp != got[f])[0]
        assert n == got_n[f] and bad.size == 0, (f, n, int(got_n[f]), bad[:8])
        assert n > 1000
    fb.kp_to_mp.fill_(-1)
