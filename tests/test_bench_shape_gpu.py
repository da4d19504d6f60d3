"""Parity at the measured shape: bench.py's own headline pipeline (B = 384 frames per step in 3 stream groups of
128 frames x 5 cameras per extract launch, the groups running concurrently on 3 HIP streams: extract -> grid ->
lapping knn -> TriangulateMatches -> mvuRight -> isInFrustum -> SearchByProjection) run for 2 timed steps, then
frames 0, 63 and 127 of EVERY group read back from the last step's device buffers and compared bit for bit with
the CPU oracle (bench.py::parity_post_run: extraction, stereo pairs, mvuRight, isInFrustum track,
SearchByProjection assignments and counts).  Runs bench.py as a child process (no exec from this process)."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.timeout(500)
def test_bench_headline_shape_is_bit_exact():
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--steps", "2", "--warmup", "1", "--no-cpu-baseline",
           "--lba-steps", "0", "--pose-frames", "0", "--tri-pairs", "0", "--aux", "0", "--p1080-frames", "0",
           "--latency-frames", "0", "--iso-reps", "0", "--stage-timing", "0", "--parity-frames", "*:0,*:63,*:127"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-4000:]
    line = [l for l in r.stdout.splitlines() if l.startswith("{")][-1]
    out = json.loads(line)
    assert out["config"]["frames_per_step_per_gpu"] == 384 and out["config"]["streams_per_gpu"] == 3
    p = out["parity_post_run"]
    assert len(p["frames"]) == 9, p["frames"]
    assert p["bit_exact"], p["mismatches"]
    assert out["parity_checked_frames"] == 9
    assert out["matches_last_step"] > 0
