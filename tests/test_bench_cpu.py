"""bench.py's accounting on the CPU: the matching kernels' algorithmic bytes split SURVEY §8(d)'s 968,000 B per
multi-camera frame exactly (no design-internal candidate records counted), and the extraction formula gives §8(d)'s
2,085,018 B per Hilti camera-frame."""
import bench


def test_matching_bytes_split_survey_8d():
    B, n_kp = 10, 10 * 5 * 1200   # the nominal 1200 keypoints per camera of §8(d)
    P = [a * b for a, b in bench.level_sizes(bench.W, bench.H)]
    b = bench.per_step_algorithmic_bytes(B, P, n_kp, 0)
    matching = sum(b[k] for k in ("grid", "stereo_knn", "proj_candidates", "proj_resolve"))
    assert matching == B * 968_000
    assert set(b) == set(bench.BYTES_FORMULA)


def test_extraction_bytes_survey_8d():
    assert bench.cam_bytes(720, 540, 1200) == 2_085_018
    assert bench.cam_bytes(1920, 1080, 2000) == 10_877_042
