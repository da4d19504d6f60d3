"""GPU parity of the HIP ORB extractor (libomv_hip.so via the C ABI) against the CPU oracle.

Bar: bit-exact — keypoint (x, y, size, angle, response, octave), order, monoIndex and all 32
descriptor bytes identical to the restated reference (oracle/orb_oracle.cpp).
"""
import numpy as np
import pytest

from openmavis_amd import synth
from openmavis_amd.orb import ORBextractor

pytestmark = pytest.mark.gpu


def _compare(o_mono, o_kps, o_desc, g_mono, g_kps, g_desc, tag=""):
    assert g_mono == o_mono, f"{tag} monoIndex {g_mono} != {o_mono}"
    assert len(g_kps) == len(o_kps), f"{tag} count {len(g_kps)} != {len(o_kps)}"
    for f in ("x", "y", "size", "angle", "response", "octave"):
        bad = np.nonzero(g_kps[f].view(np.uint32) != o_kps[f].view(np.uint32))[0]
        assert bad.size == 0, f"{tag} field {f} differs at rows {bad[:10]}: gpu {g_kps[bad[:3]]} oracle {o_kps[bad[:3]]}"
    bad = np.nonzero((g_desc != o_desc).any(1))[0]
    assert bad.size == 0, f"{tag} descriptors differ at rows {bad[:10]}"


CASES = [
    # (w, h, nfeatures, iniTh, minTh, lapping, seed)
    (720, 540, 1200, 15, 7, (0, 720), 20221000),
    (720, 540, 1200, 15, 7, (0, 0), 20223001),
    (752, 480, 1000, 20, 7, (0, 1000), 101),
    (720, 540, 500, 15, 7, (200, 400), 20222002),
    (320, 240, 300, 20, 7, (0, 0), 7),
    (400, 300, 400, 20, 7, (50, 90), 8),
    # odd pitch: byte staging in the FAST cells, the pyramid and the blur (level 0 rows not dword aligned)
    (333, 250, 300, 20, 7, (0, 0), 9),
    # level 5 is one 68-px-wide cell column: FAST cells with the per-cell LDS row stride (cells > 65 px)
    (248, 250, 150, 20, 7, (0, 0), 12),
]


@pytest.mark.parametrize("w,h,nf,ini,mn,lap,seed", CASES)
def test_extract_matches_oracle(oracle, w, h, nf, ini, mn, lap, seed):
    img = synth.synth_image(seed, w, h)
    o_mono, o_kps, o_desc = oracle.orb_extract(img, nf, 1.2, 8, ini, mn, lap)
    ex = ORBextractor(nf, 1.2, 8, ini, mn)
    g_mono, g_kps, g_desc = ex(img, None, lap)
    _compare(o_mono, o_kps, o_desc, g_mono, g_kps, g_desc, f"{w}x{h} seed {seed}")


@pytest.mark.parametrize("levels", [False, True])
@pytest.mark.parametrize("w,h,seed", [(720, 540, 20221000), (333, 250, 9), (1920, 1080, 31)])
def test_pyramid_levels_match_oracle(oracle, monkeypatch, levels, w, h, seed):
    """Every pyramid level bit-exact: the one-launch banded pyramid and the per-level launches (OMV_PYR_MODE);
    odd pitch (byte staging of level 0) and a 1080p image (more bands, wider halos)."""
    monkeypatch.setenv("OMV_PYR_MODE", "levels" if levels else "chain")
    img = synth.synth_image(seed, w, h)
    ex = ORBextractor(1200, 1.2, 8, 15, 7)
    ex(img, None, (0, w))
    for lvl in range(1, 8):
        ref = oracle.pyramid_level(img, lvl, 1200)
        got = ex.debug_level(0, lvl)
        assert got.shape == ref.shape
        assert np.array_equal(got, ref), f"level {lvl}: {np.count_nonzero(got != ref)} px differ"


def test_batch_equals_single(oracle, torch_cuda):
    torch = torch_cuda
    imgs = synth.hilti_frame(3)
    lap = np.array([[0, 720], [0, 720], [0, 0], [0, 0], [0, 0]], np.int32)
    ex = ORBextractor(1200, 1.2, 8, 15, 7, width=720, height=540, max_images=5)
    cap = ex.max_keypoints()
    d_img = torch.from_numpy(imgs).cuda()
    kps = torch.zeros((5, cap, 6), dtype=torch.int32, device="cuda")
    desc = torch.zeros((5, cap, 32), dtype=torch.uint8, device="cuda")
    n_out = torch.zeros(5, dtype=torch.int32, device="cuda")
    mono = torch.zeros(5, dtype=torch.int32, device="cuda")
    ex.extract_batch(d_img, lap, kps, desc, n_out, mono)
    torch.cuda.synchronize()
    assert ex.last_error() == 0
    kps_h = kps.cpu().numpy().view(oracle.KP_DTYPE).reshape(5, cap)
    desc_h = desc.cpu().numpy()
    n_h, m_h = n_out.cpu().numpy(), mono.cpu().numpy()
    for c in range(5):
        o_mono, o_kps, o_desc = oracle.orb_extract(imgs[c], 1200, 1.2, 8, 15, 7, tuple(lap[c]))
        n = n_h[c]
        _compare(o_mono, o_kps, o_desc, int(m_h[c]), kps_h[c, :n], desc_h[c, :n], f"cam {c}")


def test_empty_image_returns_minus_one():
    ex = ORBextractor(500, 1.2, 8, 20, 7)
    mono, kps, desc = ex(np.zeros((0, 0), np.uint8), None, (0, 0))
    assert mono == -1 and len(kps) == 0 and desc.shape == (0, 32)


def test_flat_image_has_no_keypoints():
    ex = ORBextractor(500, 1.2, 8, 20, 7)
    mono, kps, desc = ex(np.full((240, 320), 77, np.uint8), None, (0, 0))
    assert mono == 0 and len(kps) == 0


def test_octree_device_sort_matches_std_sort(oracle, torch_cuda):
    """The octree's data-parallel std::sort replica (omv_introsort.h) moves tie-equal nodes exactly like
    libstdc++'s std::sort: adversarial arrays (few distinct keys, reversed input, a median-of-3 pattern
    that reaches the heapsort fallback), compared permutation for permutation."""
    torch = torch_cuda
    from openmavis_amd import _lib
    lib = _lib.load()
    rng = np.random.default_rng(1234)
    for trial in range(400):
        n = trial if trial < 40 else int(rng.integers(0, 2049))
        kmax, xmax = int(rng.integers(1, 7)), int(rng.integers(1, 5))
        k1 = rng.integers(0, kmax, n).astype(np.int32)
        k2 = rng.integers(0, xmax, n).astype(np.int32)
        if trial % 7 == 0:
            k1, k2 = k1[::-1].copy(), k2[::-1].copy()
        if trial % 11 == 0:
            i = np.arange(n)
            k1 = np.where(i % 2 == 1, i, n - i).astype(np.int32)
            k2 = np.zeros(n, np.int32)
        if trial % 13 == 0:
            k1 = rng.integers(0, 3000, n).astype(np.int32)
            k2 = rng.integers(0, 4096, n).astype(np.int32)
        want = oracle.std_sort_pairs(k1, k2)
        d1, d2 = torch.from_numpy(k1).cuda(), torch.from_numpy(k2).cuda()
        perm = torch.full((max(n, 1),), -1, dtype=torch.int32, device="cuda")
        assert lib.omv_selftest_node_sort(d1.data_ptr(), d2.data_ptr(), n, perm.data_ptr(), None) == 0
        torch.cuda.synchronize()
        got = perm.cpu().numpy()[:n]
        assert np.array_equal(got, want), f"trial {trial} n {n}: first mismatch at {np.argmax(got != want)}"


@pytest.mark.parametrize("scale,nlevels", [(1.5, 5), (2.0, 3)])
def test_extract_other_scale_factors(oracle, scale, nlevels):
    # other ORBextractor scale factors: the resize tables (and the pyramid's per-quad source windows) change
    img = synth.synth_image(31, 640, 480)
    o_mono, o_kps, o_desc = oracle.orb_extract(img, 1000, scale, nlevels, 20, 7, (0, 0))
    ex = ORBextractor(1000, scale, nlevels, 20, 7)
    g_mono, g_kps, g_desc = ex(img, None, (0, 0))
    _compare(o_mono, o_kps, o_desc, g_mono, g_kps, g_desc, f"scale {scale} x {nlevels}")


def test_harris_extra_matches_oracle(oracle, torch_cuda):
    """The optional Harris output (OpenCV ORB's HarrisResponses, blockSize 7, k 0.04; north star "Harris response
    within 1e-5"): per output row, at the keypoint's level position on the un-blurred level.  The reference computes
    no Harris score (its response is FAST's, include/ORBextractor.h:24), so the oracle is OpenCV's published formula,
    pinned by tests/test_oracle_cpu.py::test_harris_oracle_matches_numpy.  Same float expression on both sides:
    required within 1e-5 relative (observed bit-exact); the keypoints and descriptors stay bit-exact with it on."""
    torch = torch_cuda
    imgs = synth.hilti_frame(5)
    lap = np.array([[0, 720], [0, 720], [0, 0], [0, 0], [0, 0]], np.int32)
    ex = ORBextractor(1200, 1.2, 8, 15, 7, width=720, height=540, max_images=5)
    cap = ex.max_keypoints()
    d_img = torch.from_numpy(imgs).cuda()
    kps = torch.zeros((5, cap, 6), dtype=torch.int32, device="cuda")
    desc = torch.zeros((5, cap, 32), dtype=torch.uint8, device="cuda")
    n_out = torch.zeros(5, dtype=torch.int32, device="cuda")
    mono = torch.zeros(5, dtype=torch.int32, device="cuda")
    harris = torch.full((5, cap), float("nan"), dtype=torch.float32, device="cuda")
    ex.extract_batch(d_img, lap, kps, desc, n_out, mono, harris=harris)
    torch.cuda.synchronize()
    assert ex.last_error() == 0
    kps_h = kps.cpu().numpy().view(oracle.KP_DTYPE).reshape(5, cap)
    desc_h, n_h, m_h, hr = desc.cpu().numpy(), n_out.cpu().numpy(), mono.cpu().numpy(), harris.cpu().numpy()
    scale = oracle.orb_tables(1200, 1.2, 8)["scale"]
    checked = 0
    for c in range(5):
        n = int(n_h[c])
        o_mono, o_kps, o_desc = oracle.orb_extract(imgs[c], 1200, 1.2, 8, 15, 7, tuple(lap[c]))
        _compare(o_mono, o_kps, o_desc, int(m_h[c]), kps_h[c, :n], desc_h[c, :n], f"cam {c} (harris on)")
        for lvl in range(8):
            rows = np.nonzero(kps_h[c, :n]["octave"] == lvl)[0]
            if rows.size == 0:
                continue
            L = imgs[c] if lvl == 0 else oracle.pyramid_level(imgs[c], lvl, 1200)
            k = kps_h[c, rows]
            xs = np.rint(k["x"].astype(np.float64) / scale[lvl]).astype(np.int32)
            ys = np.rint(k["y"].astype(np.float64) / scale[lvl]).astype(np.int32)
            ref = oracle.harris_responses(L, xs, ys)
            got = hr[c, rows]
            tol = 1e-5 * np.maximum(np.abs(ref), 1e-30)
            assert (np.abs(got - ref) <= tol).all(), (c, lvl, got[:4], ref[:4])
            checked += rows.size
    assert checked > 4000
    # off by default: the next batch without the output leaves the buffer alone
    harris.fill_(7.0)
    ex.extract_batch(d_img, lap, kps, desc, n_out, mono)
    torch.cuda.synchronize()
    assert bool((harris == 7.0).all())
