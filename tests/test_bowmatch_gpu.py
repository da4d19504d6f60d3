"""GPU parity of ORBmatcher::SearchByBoW (both overloads, openmavis_amd/csrc/bowmatch.hip) and
SearchForInitialization (openmavis_amd/csrc/match.hip::init_kernel) against the CPU oracle
(oracle/bowmatch_oracle.cpp, oracle/match_oracle.cpp): match indices, counts and the updated vbPrevMatched
bit-exact (integer / index output; the float window and rotation-bin arithmetic is the same on both sides)."""
import numpy as np
import pytest

from openmavis_amd import synth_init, synth_tri
from openmavis_amd.matcher import FrameBatch, ORBmatcher

pytestmark = pytest.mark.gpu


def _dev_view(kf, n_left=None, n_sideleft=None):
    import torch
    d = {f: kf[f] for f in ("n", "n_left", "n_right", "n_sideleft")}
    if n_left is not None:
        d["n_left"] = n_left
    if n_sideleft is not None:
        d["n_sideleft"] = n_sideleft
    d["kps"] = torch.from_numpy(kf["kps"].view(np.float32).reshape(-1, 6).copy()).cuda()
    for f in ("desc", "has_mp", "node_start", "node_idx"):
        d[f] = torch.from_numpy(np.ascontiguousarray(kf[f])).cuda()
    d["node_id"] = torch.from_numpy(kf["node_id"].view(np.int32).copy()).cuda()
    return d


def _host_view(kf, n_left=None, n_sideleft=None):
    d = dict(kf)
    if n_left is not None:
        d["n_left"] = n_left
    if n_sideleft is not None:
        d["n_sideleft"] = n_sideleft
    return d


def _stop_words(kf, seed, frac=0.25):
    """Drop a fraction of the FeatureVector's nodes, as DBoW2 leaves stopped words (weight 0) out of it
    (TemplatedVocabulary.h:1157): the CSR then lists fewer than n keypoints (node_start[n_nodes] < n)."""
    rng = np.random.default_rng(seed)
    keep = rng.random(len(kf["node_id"])) >= frac
    starts, idx = kf["node_start"], kf["node_idx"]
    runs = [idx[starts[a]:starts[a + 1]] for a in range(len(keep)) if keep[a]]
    out = dict(kf)
    out["node_id"] = kf["node_id"][keep].copy()
    out["node_start"] = np.concatenate([[0], np.cumsum([len(r) for r in runs])]).astype(np.int32)
    out["node_idx"] = (np.concatenate(runs) if runs else np.zeros(0, np.int32)).astype(np.int32)
    assert out["node_start"][-1] < kf["n"]
    return out


CASES = [  # (kf_kf, check_ori, frame n_left override, frame n_sideleft override)
    (False, True, None, None),     # multi-camera frame, four blocks
    (False, False, None, None),
    (False, True, -1, None),       # single-camera frame (F.Nleft == -1): one block
    (False, True, None, -1),       # two-camera frame: no side blocks
    (True, True, None, None),      # (KF1, KF2)
    (True, False, None, None),
]


@pytest.mark.parametrize("kf_kf,check_ori,n_left,n_sideleft", CASES)
def test_search_by_bow_matches_oracle(oracle, kf_kf, check_ori, n_left, n_sideleft):
    import torch
    pairs = [synth_tri.make_tri_pair(seed=s, n_pts=300 + 60 * s, mp_frac=0.8 if s % 2 else 0.5, n_nodes=60 + 10 * s)
             for s in range(1, 9)]
    jobs, host_jobs = [], []
    for p in pairs:
        n_out = p["kf1"]["n"] if kf_kf else p["kf2"]["n"]
        jobs.append(dict(kf=_dev_view(p["kf1"]), other=_dev_view(p["kf2"], n_left, n_sideleft),
                         match=torch.full((n_out,), -9, dtype=torch.int32, device="cuda")))
        host_jobs.append(dict(kf=p["kf1"], other=_host_view(p["kf2"], n_left, n_sideleft)))
    m = ORBmatcher(0.75, check_ori)
    n = m.SearchByBoW(jobs, kf_kf=kf_kf).cpu().numpy()
    total = 0
    for i, hj in enumerate(host_jobs):
        n_o, m_o = oracle.search_by_bow(hj, kf_kf=kf_kf, nnratio=0.75, check_ori=check_ori)
        g = jobs[i]["match"].cpu().numpy()
        assert n[i] == n_o, (i, n[i], n_o)
        assert np.array_equal(g, m_o), (i, np.nonzero(g != m_o)[0][:10])
        assert n_o == int((m_o >= 0).sum())
        total += n_o
    assert total > 200   # the cases exercise real matching


def _run_bow(oracle, pairs, kf_kf, check_ori, nnratio=0.75):
    import torch
    jobs, host_jobs = [], []
    for p in pairs:
        n_out = p["kf1"]["n"] if kf_kf else p["kf2"]["n"]
        jobs.append(dict(kf=_dev_view(p["kf1"]), other=_dev_view(p["kf2"]),
                         match=torch.full((n_out,), -9, dtype=torch.int32, device="cuda")))
        host_jobs.append(dict(kf=p["kf1"], other=p["kf2"]))
    m = ORBmatcher(nnratio, check_ori)
    m.bow_rescans(reset=True)
    n = m.SearchByBoW(jobs, kf_kf=kf_kf).cpu().numpy()
    rescans = m.bow_rescans(reset=True)
    total = 0
    for i, hj in enumerate(host_jobs):
        n_o, m_o = oracle.search_by_bow(hj, kf_kf=kf_kf, nnratio=nnratio, check_ori=check_ori)
        g = jobs[i]["match"].cpu().numpy()
        assert n[i] == n_o, (i, n[i], n_o)
        assert np.array_equal(g, m_o), (i, np.nonzero(g != m_o)[0][:10])
        total += n_o
    return total, rescans


@pytest.mark.parametrize("kf_kf", [False, True])
def test_search_by_bow_stopped_words(oracle, kf_kf):
    """FeatureVectors that leave keypoints out (stopped words): the walk must end at the list's end."""
    pairs = []
    for s in range(1, 7):
        p = synth_tri.make_tri_pair(seed=20 + s, n_pts=300 + 50 * s, mp_frac=0.7, n_nodes=40 + 10 * s)
        pairs.append(dict(p, kf1=_stop_words(p["kf1"], 100 + s), kf2=_stop_words(p["kf2"], 200 + s)))
    total, _ = _run_bow(oracle, pairs, kf_kf, True)
    assert total > 50


@pytest.mark.parametrize("kf_kf", [False, True])
def test_search_by_bow_crowded_nodes(oracle, monkeypatch, kf_kf):
    """Few vocabulary nodes (30+ candidates per node and camera block, as a real vocabulary at levelsup 4 gives;
    100+ in the one- and two-node pairs): the short lists overflow and the walk's rescan under the current claims
    runs; its result stays bit-exact."""
    pairs = [synth_tri.make_tri_pair(seed=40 + s, n_pts=500 + 50 * s, mp_frac=0.9, n_nodes=5 + s) for s in range(1, 7)]
    # one or two nodes: 100+ candidates per node and block, so even 16-entry short lists run out
    pairs += [synth_tri.make_tri_pair(seed=60 + s, n_pts=900 + 100 * s, mp_frac=0.5, n_nodes=1 + s % 2) for s in range(3)]
    total, _ = _run_bow(oracle, pairs, kf_kf, True, nnratio=0.9)
    assert total > 50
    # the same with the walk using 4 entries of each short list: the rescans run often
    monkeypatch.setenv("OMV_BOW_TOP", "4")
    total, rescans = _run_bow(oracle, pairs, kf_kf, True, nnratio=0.9)
    assert total > 50
    assert rescans > 0, "the crowded-node case did not exercise the rescan path"


def _init_frames(pairs):
    import torch
    cap = max(max(len(p["f1"]["kps"]), len(p["f2"]["kps"])) for p in pairs)
    fb = FrameBatch(torch, 2 * len(pairs), 1, cap, synth_init.W, synth_init.H, synth_init.scale_factors())
    for i, p in enumerate(pairs):
        for k, f in enumerate(("f1", "f2")):
            kp = p[f]["kps"]
            fb.kps[2 * i + k, 0, :len(kp)] = torch.from_numpy(kp.view(np.int32).reshape(-1, 6).copy())
            fb.desc[2 * i + k, 0, :len(kp)] = torch.from_numpy(p[f]["desc"])
            fb.n_kp[2 * i + k, 0] = len(kp)
    return fb, cap


@pytest.mark.parametrize("window,check_ori,nnratio", [(100, True, 0.9), (100, False, 0.9), (30, True, 0.75)])
def test_search_for_initialization_matches_oracle(oracle, window, check_ori, nnratio):
    import torch
    pairs = [synth_init.make_init_pair(seed=s, n=600 + 150 * s, motion=(3.0 * s, -2.0 * s), rot=7.0 * s)
             for s in range(1, 7)]
    fb, cap = _init_frames(pairs)
    prev = torch.zeros((len(pairs), cap, 2), dtype=torch.float32, device="cuda")
    for i, p in enumerate(pairs):
        prev[i, :len(p["prev"])] = torch.from_numpy(p["prev"])
    m = ORBmatcher(nnratio, check_ori)
    m12, n = m.SearchForInitialization(fb, [(2 * i, 2 * i + 1) for i in range(len(pairs))], prev, windowSize=window)
    m12, n, prev = m12.cpu().numpy(), n.cpu().numpy(), prev.cpu().numpy()
    g = oracle.frame_geom(1, synth_init.W, synth_init.H, synth_init.scale_factors())
    for i, p in enumerate(pairs):
        n_o, m_o, prev_o = oracle.search_for_initialization(g, p["f1"]["kps"], p["f1"]["desc"], p["f2"]["kps"],
                                                            p["f2"]["desc"], p["prev"], window, nnratio, check_ori)
        n1 = len(p["f1"]["kps"])
        assert n[i] == n_o, (i, n[i], n_o)
        assert np.array_equal(m12[i, :n1], m_o), (i, np.nonzero(m12[i, :n1] != m_o)[0][:10])
        assert np.array_equal(prev[i, :n1], prev_o)
        assert n_o > 50


def _contest(p, rng, n_clusters=12, copies=10):
    """Append clusters of identical F1 keypoints (same position, descriptor) and, next to them, F2 keypoints at
    0, 5, 10, ... flipped bits: each copy claims the next-closest F2 keypoint once the earlier copies hold the
    closer ones, so the walk's speculative eight smallest keys run out (the filtered rescan runs)."""
    f1k, f1d, f2k, f2d, prev = [p["f1"]["kps"]], [p["f1"]["desc"]], [p["f2"]["kps"]], [p["f2"]["desc"]], [p["prev"]]
    for _ in range(n_clusters):
        xy = np.array([[rng.uniform(40, synth_init.W - 40), rng.uniform(40, synth_init.H - 40)]], np.float32)
        d = rng.integers(0, 256, (1, 32), dtype=np.uint8)
        f1k.append(synth_init._kps(np.repeat(xy, copies, 0), np.zeros(copies, np.int32), np.full(copies, 10, np.float32)))
        f1d.append(np.repeat(d, copies, 0))
        prev.append(np.repeat(xy, copies, 0))
        dd = np.repeat(d, copies, 0)
        for c in range(copies):
            for b in rng.choice(256, 5 * c, replace=False):
                dd[c, b // 8] ^= np.uint8(1 << (b % 8))
        off = rng.normal(0, 2.0, (copies, 2)).astype(np.float32)
        f2k.append(synth_init._kps(xy + off, np.zeros(copies, np.int32), np.full(copies, 15, np.float32)))
        f2d.append(dd)
    return dict(f1=dict(kps=np.concatenate(f1k), desc=np.concatenate(f1d)),
                f2=dict(kps=np.concatenate(f2k), desc=np.concatenate(f2d)), prev=np.concatenate(prev))


@pytest.mark.parametrize("check_ori", [True, False])
def test_search_for_initialization_contested_claims(oracle, check_ori):
    """Claims that exclude the speculative best / second (and all eight kept keys) match the oracle bit-exactly."""
    import torch
    rng = np.random.Generator(np.random.PCG64(77))
    pairs = [_contest(synth_init.make_init_pair(seed=s, n=500, motion=(2.0, 1.0), rot=3.0), rng) for s in (11, 12, 13)]
    fb, cap = _init_frames(pairs)
    prev = torch.zeros((len(pairs), cap, 2), dtype=torch.float32, device="cuda")
    for i, p in enumerate(pairs):
        prev[i, :len(p["prev"])] = torch.from_numpy(p["prev"])
    m = ORBmatcher(0.9, check_ori)
    m12, n = m.SearchForInitialization(fb, [(2 * i, 2 * i + 1) for i in range(len(pairs))], prev, windowSize=100)
    m12, n, prev = m12.cpu().numpy(), n.cpu().numpy(), prev.cpu().numpy()
    g = oracle.frame_geom(1, synth_init.W, synth_init.H, synth_init.scale_factors())
    for i, p in enumerate(pairs):
        n_o, m_o, prev_o = oracle.search_for_initialization(g, p["f1"]["kps"], p["f1"]["desc"], p["f2"]["kps"],
                                                            p["f2"]["desc"], p["prev"], 100, 0.9, check_ori)
        n1 = len(p["f1"]["kps"])
        assert n[i] == n_o, (i, n[i], n_o)
        assert np.array_equal(m12[i, :n1], m_o), (i, np.nonzero(m12[i, :n1] != m_o)[0][:10])
        assert np.array_equal(prev[i, :n1], prev_o)
        # the clusters' later copies matched past the first four keys (the rescan ran)
        f2n = len(p["f2"]["kps"]) - 12 * 10
        assert (m_o[n1 - 12 * 10:] >= f2n).sum() >= 12 * 9, m_o[n1 - 12 * 10:]
