#!/usr/bin/env python3
"""Benchmark: multi-camera ORB extract + match on the Hilti-2022-like 5 x 720x540 rig (BASELINE.json
configs[1]): per frame, 5 extractions (1200 features/cam, iniTh 15, minTh 7, lapping [0,720] on the
front pair) + the grid + lapping-area knn (cam0 <-> cam1, Lowe 0.8) + SearchByProjection of a
5,000-point local map (th 6, nnratio 0.8).  One step = one pass over a batch of B frames whose
images (and map points) are already resident in HBM.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--frames B] [--no-cpu-baseline]

--gpus N > 1 without a torch.distributed environment: the script starts N ranks itself
(torch.distributed.run, one process per GPU, before anything touches a GPU) and exits with their status.
Every rank processes its own frames (frame-parallel replicas, no data-path collective: the path shards by
frame) and rank 0 prints one JSON line with the whole-job throughput (max time over ranks).  At N > 1 the
camera-sharded layouts run as extra legs: `cam_shard` (configs[2], 5 Hilti cameras over the ranks, one
RCCL all-gather of the keypoint / descriptor slabs, matching on rank 0) and `p1080` (configs[3], 8 Pinhole
cameras 1920x1080 over the ranks).  At N = 1 `p1080` is the 8-camera batch on one GPU.
"""
import argparse
import json
import os
import socket
import subprocess
import sys
import time

import faulthandler

import numpy as np

faulthandler.enable()

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

W, H, C = 720, 540, 5
NFEAT, INI_TH, MIN_TH, NLEV, SCALE = 1200, 15, 7, 8, 1.2
LAP = np.array([[0, 720], [0, 720], [0, 0], [0, 0], [0, 0]], np.int32)
M_MPS, TH, NNRATIO = 5000, 6.0, 0.8
HBM_PEAK_GBS = 8000.0   # MI355X_MICROARCH.md: HBM3E 8 TB/s spec
# configs[4]: LocalInertialBA window, bLarge settings (Optimizer.cc:2742-2745, :3270-3274)
LBA_CFG = dict(opt_it=4, lambda_init=1e-2, max_trials=10, large=True)


def _gen_frame(f):
    from openmavis_amd import synth
    return synth.hilti_frame(f, C, W, H)


def _gen_cam_image(item):
    from openmavis_amd import synth
    c, f = item
    return synth.synth_image(synth.HILTI_SEED + 1000 * c + f, W, H)


def _gen_map(args):
    """3-D local map of one frame (world points + map-point fields) and its block-0 pose."""
    from openmavis_amd import synth
    kps, desc, n_kp, seed = args
    cams, R_cl, t_cl = synth.hilti_rig(C)
    pose = synth.random_pose(np.random.default_rng(seed))
    world, mp = synth.make_world_map(kps, desc, n_kp, M_MPS, seed, cams, R_cl, t_cl, pose, W, H, NLEV)
    return pose, world, mp


def _cpu_workers():
    """Worker count for host pools: the CPUs this process may run on, at most 16 (the GPU box's CPU share;
    os.cpu_count() there reports the whole machine)."""
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:
        n = os.cpu_count() or 1
    return max(1, min(16, n))


_POOL = None


def _pool():
    """One fork pool for the whole run, created before anything touches the GPU (forked children never
    inherit a HIP context) and closed + joined at the end (no process outlives the bench)."""
    global _POOL
    if _POOL is None and _cpu_workers() > 1:
        import multiprocessing as mp
        _POOL = mp.get_context("fork").Pool(_cpu_workers())
    return _POOL


def _close_pool():
    global _POOL
    if _POOL is not None:
        _POOL.close()
        _POOL.join()
        _POOL = None


def _pool_map(fn, items):
    pool = _pool()
    if pool is None or len(items) <= 1:
        return [fn(i) for i in items]
    return pool.map(fn, items)


def host_info():
    """The host the CPU baselines ran on (nproc, lscpu model, sockets, threads)."""
    info = {"nproc": os.cpu_count()}
    try:
        info["rocm_version"] = open("/opt/rocm/.info/version").read().strip()
    except OSError:
        pass
    try:   # device_count() does not initialise the GPU on this image
        import torch
        info["gpu_count"] = torch.cuda.device_count()
    except Exception:
        pass
    try:
        info["usable_cpus"] = len(os.sched_getaffinity(0))
    except AttributeError:
        pass
    try:
        out = subprocess.run(["lscpu"], capture_output=True, text=True, timeout=10).stdout
        keys = {"Model name": "model", "Socket(s)": "sockets", "Core(s) per socket": "cores_per_socket",
                "Thread(s) per core": "threads_per_core", "CPU(s)": "cpus"}
        for line in out.splitlines():
            k, _, v = line.partition(":")
            if k.strip() in keys:
                v = v.strip()
                info[keys[k.strip()]] = int(v) if v.isdigit() else v
    except (OSError, subprocess.SubprocessError):
        pass
    return info


NATIVE_LIB = None   # oracle/liboracle_native.so once `make native` built it on this host (timing legs only)


def _build_native_oracle():
    """the CPU baseline is the restatement built -O3 -march=native ON THE TIMED HOST (the
    container's CPU differs from the GPU box's, so it is never shipped prebuilt).  Falls back to the parity build."""
    global NATIVE_LIB
    try:
        subprocess.run(["make", "-s", f"-j{_cpu_workers()}", "-C", os.path.join(ROOT, "oracle"), "native"],
                       check=True, timeout=300, capture_output=True)
        NATIVE_LIB = os.path.join(ROOT, "oracle", "liboracle_native.so")
    except (OSError, subprocess.SubprocessError):
        NATIVE_LIB = None


def _oracle_build():
    return "g++ -O3 -march=native, built on this host" if NATIVE_LIB else \
        "g++ -O3 -march=x86-64-v2 -ffp-contract=off (native build unavailable)"


def _oracle(timing):
    """The oracle module with the timing build (timing=True: CPU baselines) or the parity build (the checker)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle
    want = NATIVE_LIB if timing and NATIVE_LIB else oracle.LIB
    if getattr(oracle, "_active_path", None) != want:
        oracle.use_library(want)
        oracle._active_path = want
    return oracle


_CPU_CONST = None


def _cpu_const():
    """Per-process constants of the CPU pipeline (rig, stereo extrinsics, undistortion, depth images)."""
    global _CPU_CONST
    if _CPU_CONST is None:
        oracle = _oracle(timing=True)
        from openmavis_amd import synth
        from openmavis_amd.frame import BLOCK_CAM_ID, undist_params
        from openmavis_amd.matcher import make_rig
        tab = oracle.orb_tables(NFEAT, SCALE, NLEV)
        cams, R_cl, t_cl = synth.hilti_rig(C)
        Rlr = R_cl[1].T.astype(np.float32)
        tlr = (-R_cl[1].T @ t_cl[1]).astype(np.float32)
        _CPU_CONST = dict(
            g=oracle.frame_geom(C, W, H, tab["scale"]), rig=make_rig(cams, R_cl, t_cl, W, H, SCALE, NLEV), cams=cams,
            Rlr=Rlr, tlr=tlr, bf=float(cams[0][0] * np.linalg.norm(tlr)),
            sigma2=(np.float32(SCALE) ** (2 * np.arange(NLEV))).astype(np.float32), U=undist_params(BLOCK_CAM_ID),
            depth=(np.random.default_rng(5).random((4, H, W)) * 25.0).astype(np.float32))
    return _CPU_CONST


def _cpu_prep(item):
    """Untimed: the 3-D local map of a frame, derived from a first extraction of its own keypoints."""
    oracle = _oracle(timing=True)
    i, imgs = item
    n_out, mono, kps, desc = oracle.orb_extract_frame(imgs, NFEAT, LAP, SCALE, NLEV, INI_TH, MIN_TH, threaded=False)
    return _gen_map((kps, desc, n_out, 700 + i))


def _cpu_frame(imgs, prep, threaded):
    """The reference path of one multi-camera frame on the CPU oracle: extraction (one std::thread per camera
    when threaded, like src/Frame.cc:1841-1862), lapping knn + Lowe, TriangulateMatches, mvuRight, isInFrustum,
    SearchByProjection."""
    oracle = _oracle(timing=True)
    k = _cpu_const()
    n_out, mono, kps, desc = oracle.orb_extract_frame(imgs, NFEAT, LAP, SCALE, NLEV, INI_TH, MIN_TH, threaded=threaded)
    cap = kps.shape[1]
    q = desc[0, mono[0]:n_out[0]]
    t = desc[1, mono[1]:n_out[1]]
    i2, d2 = oracle.bf_knn2(q, t)
    l2r = np.full(cap, -1, np.int32)
    r2l = np.full(cap, -1, np.int32)
    ok = (i2[:, 1] >= 0) & (d2[:, 0].astype(np.float64) < d2[:, 1].astype(np.float64) * 0.8)
    for qi in np.nonzero(ok)[0]:
        l2r[mono[0] + qi] = mono[1] + i2[qi, 0]
        r2l[mono[1] + i2[qi, 0]] = mono[0] + qi
    l2r, r2l, _, _ = oracle.stereo_triangulate(kps[0], n_out[0], kps[1], n_out[1], k["cams"][:2], k["Rlr"], k["tlr"],
                                               k["sigma2"], l2r)
    for c in range(4):   # mvuRight (GetDepthFromUndistortedPoints)
        oracle.depth_from_undistorted(kps[c, :n_out[c]], k["depth"][c], k["U"][c], k["bf"])
    pose, world, mp = prep
    track, _ = oracle.frustum(k["rig"], pose, world["pos"], world["normal"], world["min_dist"], world["max_dist"], 0.5,
                              mp["view_cos"], mp["track_depth"])
    k2m = np.full(C * cap, -1, np.int32)
    return oracle.search_by_projection(k["g"], kps, desc, n_out, dict(mp, **track), TH, False, 50.0, NNRATIO, l2r, r2l,
                                       None, k2m)


def _cpu_frame_job(item):
    imgs, prep = item
    return _cpu_frame(imgs, prep, threaded=False)


def parity_post_run(checks, groups, rig, cams, Rlr, tlr, sigma2, bf):
    """Untimed, after the timed steps: the CPU oracle as CHECKER (never the measured path) on frames of the LAST
    timed step, read back from the measured run's own device buffers (the 3-stream, Bg-frame-per-launch shape).
    checks: [(group, frame_in_group, images [C,H,W], (pose, world, mp_initial))].  Compares bit for bit:
    extraction (keypoints as raw bits, descriptors, counts, monoIndex), the lapping pairs after TriangulateMatches
    (l2r / r2l), mvuRight, isInFrustum's track and SearchByProjection's assignment + count."""
    oracle = _oracle(timing=False)
    from openmavis_amd.frame import BLOCK_CAM_ID, undist_params
    U = undist_params(BLOCK_CAM_ID)
    g = oracle.frame_geom(C, W, H, oracle.orb_tables(NFEAT, SCALE, NLEV)["scale"])
    bad = []
    for gi, f, imgs, (pose, world, mp0) in checks:
        gr = groups[gi]
        fb = gr["fb"]
        cap = fb.kp_cap
        kps = fb.kps[f].cpu().numpy().view(oracle.KP_DTYPE).reshape(C, cap)
        desc = fb.desc[f].cpu().numpy()
        n_kp, mono = fb.n_kp[f].cpu().numpy(), fb.mono[f].cpu().numpy()
        tag = f"group {gi} frame {f}"
        for c in range(C):
            om, ok, od = oracle.orb_extract(imgs[c], NFEAT, SCALE, NLEV, INI_TH, MIN_TH, tuple(LAP[c]))
            n = int(n_kp[c])
            if not (n == len(ok) and mono[c] == om and np.array_equal(kps[c, :n].view(np.uint32), ok.view(np.uint32))
                    and np.array_equal(desc[c, :n], od)):
                bad.append(f"{tag} cam {c}: extraction")
        q, t = desc[0, mono[0]:n_kp[0]], desc[1, mono[1]:n_kp[1]]
        i2, d2 = oracle.bf_knn2(q, t)
        l2r = np.full(cap, -1, np.int32)
        okm = (i2[:, 1] >= 0) & (d2[:, 0].astype(np.float64) < d2[:, 1].astype(np.float64) * 0.8)
        for qi in np.nonzero(okm)[0]:
            l2r[mono[0] + qi] = mono[1] + i2[qi, 0]
        el2r, er2l, _, _ = oracle.stereo_triangulate(kps[0], n_kp[0], kps[1], n_kp[1], cams[:2], Rlr, tlr, sigma2, l2r)
        gl2r, gr2l = fb.l2r[f].cpu().numpy(), fb.r2l[f].cpu().numpy()
        if not (np.array_equal(gl2r[:n_kp[0]], el2r) and np.array_equal(gr2l[:n_kp[1]], er2l)):
            bad.append(f"{tag}: stereo pairs")
        dep, gur = gr["depth"][f].cpu().numpy(), gr["uright"][f].cpu().numpy()
        for c in range(dep.shape[0]):
            eur, _ = oracle.depth_from_undistorted(kps[c, :n_kp[c]], dep[c], U[c], bf)
            if not np.array_equal(gur[c, :n_kp[c]].view(np.uint32), eur.view(np.uint32)):
                bad.append(f"{tag} cam {c}: mvuRight")
        track, _ = oracle.frustum(rig, pose, world["pos"], world["normal"], world["min_dist"], world["max_dist"], 0.5,
                                  mp0["view_cos"], mp0["track_depth"])
        gm = gr["mps"]
        for k, v in track.items():
            gv = getattr(gm, k)[f].cpu().numpy()
            if not np.array_equal(np.ascontiguousarray(gv).view(np.uint8), np.ascontiguousarray(v.astype(gv.dtype)).view(np.uint8)):
                bad.append(f"{tag}: isInFrustum {k}")
        exp = np.full(C * cap, -1, np.int32)
        n = oracle.search_by_projection(g, kps, desc, n_kp, dict(mp0, **track), TH, False, 50.0, NNRATIO,
                                        _pad(el2r, cap), _pad(er2l, cap), None, exp)
        if not (n == int(fb.n_matches[f].item()) and np.array_equal(exp, fb.kp_to_mp[f].cpu().numpy())):
            bad.append(f"{tag}: SearchByProjection")
    return {"frames": [f"group {gi} frame {f}" for gi, f, _, _ in checks], "bit_exact": not bad, "mismatches": bad,
            "checked": "extraction, lapping pairs after TriangulateMatches, mvuRight, isInFrustum, SearchByProjection"}


def _pad(a, cap):
    out = np.full(cap, -1, np.int32)
    out[:len(a)] = a
    return out


def _cpu_frame_timed(item):
    """Mode-B worker: one frame through the CPU reference path; returns its wall time (s)."""
    imgs, prep = item
    t0 = time.perf_counter()
    _cpu_frame(imgs, prep, threaded=False)
    return time.perf_counter() - t0


def _lat_stats(ts):
    a = np.asarray(ts) * 1e3
    return {"median_ms": round(float(np.median(a)), 3), "p95_ms": round(float(np.percentile(a, 95)), 3)}


def cpu_baseline(frames, timed_frames=500, warmup_frames=50, best_frames=500):
    """The CPU reference path on this host, BASELINE.md §2's protocol, timed on the oracle (scalar C++ restatement
    built -O3 -march=native on this host, `make native`; the reference itself cannot be built here):
      mode A, reference-faithful: one std::thread per camera (src/Frame.cc:1841-1862), frames one at a time:
              `warmup_frames` untimed, then `timed_frames` timed one by one (median / p95 per frame);
      mode B, CPU-best: whole frames in parallel over the worker pool (one process per core of this job's CPU share,
              1 thread each), `best_frames` frames.
    The distinct frames (`frames`) are cycled.  Runs before anything touches the GPU."""
    preps = _pool_map(_cpu_prep, list(enumerate(frames)))
    _cpu_const()
    n = len(frames)
    for i in range(warmup_frames):
        _cpu_frame(frames[i % n], preps[i % n], threaded=True)
    ts = []
    t0 = time.perf_counter()
    for i in range(timed_frames):
        t1 = time.perf_counter()
        _cpu_frame(frames[i % n], preps[i % n], threaded=True)
        ts.append(time.perf_counter() - t1)
    dt = time.perf_counter() - t0
    out = dict(value=round(timed_frames / dt, 3), unit="multi-cam frames/s", cores=C, kind="port",
               sample=f"{timed_frames} timed frames ({n} distinct Hilti-like 5x720x540 frames cycled, 1200 feat/cam, "
                      f"M={M_MPS} map points) after {warmup_frames} warm-up frames; oracle C++ restatement "
                      f"({_oracle_build()}), one thread per camera (mode A, reference-faithful), {dt:.1f} s",
               **_lat_stats(ts), host=host_info())
    if best_frames > 0 and _pool() is not None:
        items = [(frames[i % n], preps[i % n]) for i in range(best_frames)]
        _pool_map(_cpu_frame_timed, items[:2 * _cpu_workers()])   # warm every worker (constants, oracle load)
        t0 = time.perf_counter()
        tb = _pool_map(_cpu_frame_timed, items)
        dt = time.perf_counter() - t0
        w = _cpu_workers()
        hi = host_info()
        out["mode_b"] = dict(value=round(best_frames / dt, 3), unit="multi-cam frames/s", cores=w, kind="port",
                             sample=f"{best_frames} frames, whole frames in parallel over {w} worker processes "
                                    f"(1 thread each: this job's CPU share of the host), {dt:.1f} s", **_lat_stats(tb),
                             per_core=round(best_frames / dt / w, 3))
        if hi.get("usable_cpus"):
            out["mode_b"]["projected_all_usable_cpus"] = dict(
                value=round(best_frames / dt / w * hi["usable_cpus"], 1), cpus=hi["usable_cpus"],
                note="per-core rate x usable CPUs (a projection, not measured: the harness gives one GPU job "
                     f"{w} of the host's CPUs)")
    return out


def lba_bytes_per_trial(prob):
    """2*E*40 (edge records read for build + chi2) + 3*P*24 (points read twice, written
    once) + S(S+1)/2*8 (reduced system, S = 15 * N_opt)."""
    E, P = len(prob["mono_pt"]), len(prob["pts"])
    S = 15 * int(prob["n_opt"])
    return 2 * E * 40 + 3 * P * 24 + S * (S + 1) // 2 * 8


def lba_cpu_baseline(prob, min_trials=200, warmup_trials=10):
    """Oracle LocalInertialBA (scalar C++, single thread like g2o with OpenMP off) on the same window, BASELINE.md
    §2: >= `warmup_trials` LM trials untimed, then whole optimize() calls until >= `min_trials` timed trials."""
    oracle = _oracle(timing=True)
    w = 0
    while w < warmup_trials:
        w += oracle.lba_optimize(prob, **LBA_CFG)[0]["trials"]
    trials, runs = 0, 0
    t0 = time.perf_counter()
    while trials < min_trials:
        r, _, _ = oracle.lba_optimize(prob, **LBA_CFG)
        trials += r["trials"]
        runs += 1
    dt = time.perf_counter() - t0
    return dict(value=trials / dt, unit="LM trials/s", cores=1, kind="port", ms_per_trial=round(dt / trials * 1e3, 3),
                sample=f"{trials} timed LM trials ({runs} LocalInertialBA optimize() calls on the config-5 window) "
                       f"after {w} warm-up trials, oracle C++ restatement ({_oracle_build()}), 1 thread, {dt:.1f} s")


def lba_leg(prob, steps, warmup, dev, world, shard=False):
    """LocalBA iters/s: one iteration = one LM trial (error eval + build + Schur + factor/solve + update
    + chi2).  Each step is one full optimize() of the window from its uploaded state (reset is a
    device copy enqueued before the clock starts; it may still be running when optimize() is called, so its
    few microseconds can land inside -- synchronising it away measured 3 % slower: the launch latency of an
    idle queue then shows instead); the state read-back and the outlier test are inside.
    world > 1: window replicas (weak scaling), or with shard=True ONE window with its landmarks
    sharded over the ranks and one RCCL all-reduce of the partial Schur system per trial (strong)."""
    import torch
    from openmavis_amd.dist import LbaAllReduce, job_seconds
    from openmavis_amd.optimizer import LocalInertialBA
    shard = shard and world > 1
    comm = {}
    if shard:
        comm = dict(rank=torch.distributed.get_rank(), world=world, allreduce=LbaAllReduce("device", device=dev))
    ba = LocalInertialBA(max_kf=prob["n_kf"], max_cams=prob["n_cams"], max_pts=len(prob["pts"]),
                         max_mono=len(prob["mono_pt"]), max_imu=len(prob["imu_kf1"]), **comm)
    t_set = time.perf_counter()
    ba.set_problem(prob)
    t_set = time.perf_counter() - t_set
    for _ in range(warmup):
        ba.reset().optimize(**LBA_CFG)
    if world > 1:
        torch.distributed.barrier()
    torch.cuda.synchronize(dev)
    total, trials, st_sum, res = 0.0, 0, {}, None
    for _ in range(steps):
        ba.reset()
        t0 = time.perf_counter()
        res, _ = ba.optimize(**LBA_CFG, chi2=False, state_copy=False)   # state written back into the problem arrays
        total += time.perf_counter() - t0
        trials += res["trials"]
    torch.cuda.synchronize(dev)
    dt = job_seconds(total, dev)
    # per-stage device times: one extra optimize() with direct launches and events (the timed loop runs the
    # captured LM step, which carries no per-stage events)
    ba.enable_timing(True)
    ba.reset().optimize(**LBA_CFG)
    st_sum = {k: v for k, v in ba.stage_ms().items()}
    ba.enable_timing(False)
    trial_ms = dt / trials * 1e3
    bpt = lba_bytes_per_trial(prob)
    achieved = bpt / (trial_ms * 1e-3) / 1e9
    stages = {k: round(v / max(st_sum.get("trials", 1), 1), 4) for k, v in st_sum.items() if k != "trials"}
    return {
        "metric": "LocalBA iters/sec (LM trials/s)",
        "value": round(trials * (1 if shard else world) / dt, 2),
        "unit": "LM trials/s",
        "ms_per_trial": round(trial_ms, 4),
        "ms_per_optimize": round(dt / steps * 1e3, 3),
        "trials_per_optimize": trials / steps,
        "err": res["err"], "err_end": res["err_end"], "status": res["status"],
        "set_problem_ms": round(t_set * 1e3, 2),
        "stage_ms_per_trial": stages,
        "config": {"workload": "LocalInertialBA 50 KFs (25 opt + 25 fixed) x 20k MapPoints x 5 cams, "
                               f"{len(prob['mono_pt'])} EdgeMono + {len(prob['imu_kf1'])} inertial, bLarge",
                   "parallelism": f"landmark-sharded x{world}" if shard else f"window-replicas x{world}"},
        "scaling": "strong" if shard else "weak",
        "dtype": "f64",
        "roofline": {"kernel": "whole LM trial", "bound": "hbm", "achieved": round(achieved, 2),
                     "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 6),
                     "traffic": lba_traffic()[0], "algorithmic_bytes_per_trial": bpt,
                     "traffic_source": lba_traffic()[1]},
    }


def newest_profile(name):
    """(path, record) of the newest round-tagged profiles/<tag>_<name>.json (tags r01 < r01b < ... < r05g sort as
    strings), or (None, None)."""
    import glob
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", f"r[0-9][0-9]*_{name}.json")),
                   key=lambda f: os.path.basename(f)[:-len(name) - 6])
    for f in reversed(files):
        try:
            return os.path.relpath(f, ROOT), json.load(open(f))
        except (OSError, ValueError):
            continue
    return None, None


def lba_traffic():
    """(HBM bytes per LM trial, source) from the newest profile's PMC passes (profiles/<tag>_pmc_lba_trial.json)."""
    path, r = newest_profile("pmc_lba_trial")
    try:
        return int(r["hbm_bytes_per_trial"]), f"{path} ({r['tag']}: FETCH_SIZE / WRITE_SIZE passes over {r.get('program', 'lba')})"
    except (TypeError, ValueError, KeyError):
        return None, None


def pose_leg(batch, cpu_batch, reps, dev, last_frame=False):
    """PoseInertialOptimizationLastKeyFrame (Optimizer.cc:5021-5578) or, with last_frame,
    PoseInertialOptimizationLastFrame (:5580-6170, the previous frame's vertices free + EdgePriorPoseImu +
    Marginalize) on a batch of tracked frames: one call = every frame's 4 rounds x 10 Gauss-Newton
    iterations + outlier passes + marginal Hessian; value = frames/s (state reset by a device copy outside
    the timed region)."""
    import torch
    from openmavis_amd import synth_pose
    from openmavis_amd.optimizer import PoseInertialOptimizer
    F = int(batch["n_frames"])
    init = {k: torch.tensor(np.asarray(batch[k], np.float64), device=dev) for k in synth_pose.STATE_KEYS}
    arrays = {k: v.clone() for k, v in init.items()}
    for k in synth_pose.INPUT_KEYS + (synth_pose.PRIOR_KEYS if last_frame else ()):
        arrays[k] = torch.from_numpy(np.ascontiguousarray(batch[k])).to(dev)
    kpo = torch.zeros((F, int(batch["kp_cap"])), dtype=torch.uint8, device=dev)
    H = torch.zeros((F, 225), dtype=torch.float64, device=dev)
    opt = PoseInertialOptimizer(max_frames=F, max_edges=max(len(batch["mono_cam"]), len(batch["stereo_cam"]), 1))
    run = opt.PoseInertialOptimizationLastFrame if last_frame else opt.PoseInertialOptimizationLastKeyFrame
    for _ in range(2):
        run(batch, arrays, kpo, H)
    torch.cuda.synchronize(dev)
    total = 0.0
    for _ in range(reps):
        for k in init:
            arrays[k].copy_(init[k])
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        run(batch, arrays, kpo, H)
        torch.cuda.synchronize(dev)
        total += time.perf_counter() - t0
    name = "PoseInertialOptimizationLastFrame" if last_frame else "PoseInertialOptimizationLastKeyFrame"
    out = {"metric": f"{name} frames/s", "value": round(F * reps / total, 1),
           "unit": "frames/s", "ms_per_batch": round(total / reps * 1e3, 3), "frames_per_batch": F,
           "edges_per_frame": round(len(batch["mono_cam"]) / F, 1), "dtype": "f64"}
    if cpu_batch is not None:
        oracle = _oracle(timing=True)
        t0 = time.perf_counter()
        done = 0
        while done == 0 or time.perf_counter() - t0 < 2.0:   # a ~2 s sample
            (oracle.pose_last_frame if last_frame else oracle.pose_last_kf)(cpu_batch)
            done += int(cpu_batch["n_frames"])
        dt = time.perf_counter() - t0
        out["cpu_baseline"] = {"value": round(done / dt, 1), "unit": "frames/s", "cores": 1, "kind": "port",
                               "sample": f"{done} frame optimisations ({cpu_batch['n_frames']} distinct frames of the "
                                         f"batch), oracle C++ restatement, 1 thread, {dt:.2f} s"}
    return out


def tri_leg(pairs, n_pairs, reps, dev):
    """ORBmatcher::SearchForTriangulation (ORBmatcher.cc:1131-1456) over a batch of multi-camera keyframe pairs
    (KannalaBrandt8 epipolar test with the 4x4 JacobiSVD triangulation); value = keyframe pairs/s."""
    import torch
    from openmavis_amd.matcher import ORBmatcher
    dp = []
    for i in range(n_pairs):
        p = pairs[i % len(pairs)]
        q = dict(T=p["T"])
        for k in ("kf1", "kf2"):
            kf = p[k]
            d = {f: kf[f] for f in ("n", "n_left", "n_right", "n_sideleft")}
            d["kps"] = torch.from_numpy(kf["kps"].view(np.float32).reshape(-1, 6).copy()).to(dev)
            for f in ("desc", "has_mp", "node_start", "node_idx"):
                d[f] = torch.from_numpy(np.ascontiguousarray(kf[f])).to(dev)
            d["node_id"] = torch.from_numpy(kf["node_id"].view(np.int32).copy()).to(dev)
            d["level_sigma2"] = p["level_sigma2"]
            q[k] = d
        q["match12"] = torch.empty(p["kf1"]["n"], dtype=torch.int32, device=dev)
        dp.append(q)
    from openmavis_amd.matcher import TriPairBatch
    dp = TriPairBatch(dp)   # keyframes resident: the omv_tri_pair array is built once
    m = ORBmatcher(0.6, False)   # LocalMapping::CreateNewMapPoints: ORBmatcher(0.6, false)
    cams = pairs[0]["cams"]
    for _ in range(2):
        m.SearchForTriangulation(dp, cams)
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(reps):
        n = m.SearchForTriangulation(dp, cams)
    torch.cuda.synchronize(dev)
    dt = time.perf_counter() - t0
    out = {"metric": "SearchForTriangulation keyframe pairs/s", "value": round(n_pairs * reps / dt, 1),
           "unit": "keyframe pairs/s", "ms_per_batch": round(dt / reps * 1e3, 3), "pairs_per_batch": n_pairs,
           "keypoints_per_keyframe": int(np.mean([p["kf1"]["n"] for p in pairs])),
           "matches_per_pair": round(float(n.float().mean().item()), 1)}
    oracle = _oracle(timing=True)
    t0 = time.perf_counter()
    done = 0
    while done == 0 or time.perf_counter() - t0 < 2.0:   # a ~2 s sample
        for p in pairs:
            oracle.search_for_triangulation(p)
        done += len(pairs)
    dt = time.perf_counter() - t0
    out["cpu_baseline"] = {"value": round(done / dt, 1), "unit": "keyframe pairs/s", "cores": 1, "kind": "port",
                           "sample": f"{done} pair searches ({len(pairs)} distinct pairs), oracle C++ restatement, "
                                     f"1 thread, {dt:.2f} s"}
    return out


def _timed(fn, reps, dev):
    import torch
    fn()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize(dev)
    return (time.perf_counter() - t0) / reps


def _cpu_rate(fn, units, budget=1.5):
    t0 = time.perf_counter()
    done = 0
    while done == 0 or time.perf_counter() - t0 < budget:
        fn()
        done += units
    return done, time.perf_counter() - t0


def aux_legs(dev, cpu):
    """The SURVEY §8f rows beside the two headline metrics, each on a batch already in HBM with its CPU oracle
    timed on a bounded sample: ORBmatcher::Fuse (LocalMapping::SearchInNeighbors scale), DBoW2 transform
    (ComputeBoW of whole multi-camera frames), IMU preintegration (PreintegrateIMU records), the SearchByBoW /
    SearchForInitialization / SearchBySim3 matchers, the map-point refresh, CreateNewMapPoints and PoseOptimization."""
    import torch
    from openmavis_amd import synth_bow, synth_imu, synth_kfmatch
    from openmavis_amd.bow import ORBVocabulary
    from openmavis_amd.imu import Calib, PreintegratedBatch
    from openmavis_amd.matcher import FrameBatch, ORBmatcher, kf_search_params
    if cpu:
        oracle = _oracle(timing=True)
    out = {}
    # ---- Fuse: 32 keyframes x 5 blocks, ~660 map points per (keyframe, block)
    b = synth_kfmatch.make_kf_search(0, n_kf=32, kp_cap=1200, pts_per_job=600, seed=11)
    K, Cc, cap = b["n_kf"], b["n_cams"], b["kp_cap"]
    scale = [1.0]
    for _ in range(1, b["nlevels"]):
        scale.append(float(np.float32(scale[-1] * np.float32(1.2))))
    kfs = FrameBatch(torch, K, Cc, cap, b["width"], b["height"], scale, device=dev)
    kfs.kps.copy_(torch.from_numpy(np.ascontiguousarray(b["kps"]).view(np.int32).reshape(K, Cc, cap, 6)))
    kfs.desc.copy_(torch.from_numpy(b["desc"]))
    kfs.n_kp.copy_(torch.from_numpy(b["n_kp"]))
    mps = {k: torch.from_numpy(np.ascontiguousarray(v)).to(dev) for k, v in b["mps"].items()}
    mp_list = torch.from_numpy(b["mp_list"]).to(dev)
    p = kf_search_params(3.0, 50.0, b["cams"], bf=float(b["bf"]), uright=torch.from_numpy(b["uright"]).to(dev))
    m = ORBmatcher(0.6)
    dt = _timed(lambda: m.Fuse(kfs, b["jobs"], mp_list, mps, p), 10, dev)
    n_e = len(b["mp_list"])
    out["fuse"] = {"metric": "ORBmatcher::Fuse map-point projections/s", "value": round(n_e / dt, 1),
                   "unit": "points/s", "ms_per_batch": round(dt * 1e3, 3), "points_per_batch": n_e,
                   "jobs_per_batch": len(b["jobs"])}
    if cpu:
        done, t = _cpu_rate(lambda: oracle.search_kf(b, 3.0, 50.0), n_e)
        out["fuse"]["cpu_baseline"] = {"value": round(done / t, 1), "unit": "points/s", "cores": 1, "kind": "port",
                                       "sample": f"{done} point fusions, oracle C++ restatement, 1 thread, {t:.2f} s"}
    # ---- DBoW2 transform: 128 sets of 6000 descriptors (5 x 1200), k = 10, L = 5 vocabulary
    v = synth_bow.make_vocab(k=10, L=5, seed=1)
    d, n = synth_bow.make_sets(v, n_sets=128, cap=6000, seed=2)
    voc = ORBVocabulary(v, device=dev)
    dd, nn = torch.from_numpy(d).to(dev), torch.from_numpy(n).to(dev)
    dt = _timed(lambda: voc.transform(dd, nn, 3), 10, dev)
    nd = int(n.sum())
    out["bow"] = {"metric": "DBoW2 transform descriptors/s (BowVector + FeatureVector)", "value": round(nd / dt, 1),
                  "unit": "descriptors/s", "ms_per_batch": round(dt * 1e3, 3), "sets_per_batch": 128,
                  "vocabulary": {"k": 10, "L": 5, "nodes": len(v["weight"])}}
    if cpu:
        done, t = _cpu_rate(lambda: oracle.bow_transform(v, d[:4], n[:4], 3), int(n[:4].sum()))
        out["bow"]["cpu_baseline"] = {"value": round(done / t, 1), "unit": "descriptors/s", "cores": 1,
                                      "kind": "port", "sample": f"{done} descriptors, oracle, 1 thread, {t:.2f} s"}
    # ---- IMU preintegration: 2048 records of 4-40 samples at 200 Hz
    ib = synth_imu.make_imu_batch(n_rec=2048, seed=1)
    cal = Calib(1.7e-4, 2.0e-3, 1.9e-5, 3.0e-3, freq=200.0)
    pre = PreintegratedBatch(2048, cal, device=dev)
    meas, st = torch.from_numpy(ib["meas"]).to(dev), torch.from_numpy(ib["start"]).to(dev)

    def run():
        pre.Initialize(ib["bias"])
        pre.IntegrateNewMeasurements(meas, st)
    dt = _timed(run, 10, dev)
    nm = int(ib["start"][-1])
    out["imu_preint"] = {"metric": "IMU IntegrateNewMeasurement steps/s", "value": round(nm / dt, 1),
                         "unit": "measurements/s", "ms_per_batch": round(dt * 1e3, 3), "records_per_batch": 2048}
    if cpu:
        sub = dict(ib, start=ib["start"][:65], bias=ib["bias"][:64])
        done, t = _cpu_rate(lambda: oracle.preintegrate(sub, cal.Cov, cal.CovWalk), int(sub["start"][-1]))
        out["imu_preint"]["cpu_baseline"] = {"value": round(done / t, 1), "unit": "measurements/s", "cores": 1,
                                             "kind": "port", "sample": f"{done} measurements, oracle, 1 thread, {t:.2f} s"}
    # ---- SearchByBoW(KF, F): 256 (reference keyframe, multi-camera frame) jobs of ~2,570 keypoints each
    #      (Tracking::TrackReferenceKeyFrame: ORBmatcher(0.7, true)); (KF1, KF2) on the same pairs
    from openmavis_amd import synth_init, synth_tri
    from openmavis_amd.matcher import BowJobBatch
    pairs = [synth_tri.make_tri_pair(seed=s, n_pts=1200, n_distract=600, mp_frac=0.8) for s in range(16)]

    def view(kf):
        d = {f: kf[f] for f in ("n", "n_left", "n_right", "n_sideleft")}
        d["kps"] = torch.from_numpy(kf["kps"].view(np.float32).reshape(-1, 6).copy()).to(dev)
        for f in ("desc", "has_mp", "node_start", "node_idx"):
            d[f] = torch.from_numpy(np.ascontiguousarray(kf[f])).to(dev)
        d["node_id"] = torch.from_numpy(kf["node_id"].view(np.int32).copy()).to(dev)
        return d
    views = [(view(p["kf1"]), view(p["kf2"])) for p in pairs]
    for name, kf_kf, nn in (("search_by_bow", False, 0.7), ("search_by_bow_kf_kf", True, 0.75)):
        jobs = []
        for i in range(256):
            a, o = views[i % len(views)]
            p = pairs[i % len(pairs)]
            jobs.append(dict(kf=a, other=o, match=torch.empty(p["kf1"]["n"] if kf_kf else p["kf2"]["n"],
                                                              dtype=torch.int32, device=dev)))
        batch = BowJobBatch(jobs)
        mb = ORBmatcher(nn, True)
        dt = _timed(lambda: mb.SearchByBoW(batch, kf_kf=kf_kf), 10, dev)
        nres = mb.SearchByBoW(batch, kf_kf=kf_kf)
        out[name] = {"metric": f"ORBmatcher::SearchByBoW ({'KeyFrame, KeyFrame' if kf_kf else 'KeyFrame, Frame'}) "
                               "searches/s", "value": round(256 / dt, 1), "unit": "searches/s",
                     "ms_per_batch": round(dt * 1e3, 3), "jobs_per_batch": 256,
                     "keypoints_per_view": int(np.mean([p["kf1"]["n"] for p in pairs])),
                     "matches_per_search": round(float(nres.float().mean().item()), 1)}
        if cpu:
            done, t = _cpu_rate(lambda: [oracle.search_by_bow(dict(kf=p["kf1"], other=p["kf2"]), kf_kf, nn, True)
                                         for p in pairs[:4]], 4)
            out[name]["cpu_baseline"] = {"value": round(done / t, 1), "unit": "searches/s", "cores": 1,
                                         "kind": "port", "sample": f"{done} searches, oracle, 1 thread, {t:.2f} s"}
    # ---- SearchForInitialization: 64 monocular frame pairs (1,000 keypoints, EuRoC-sized), window 100
    ip = [synth_init.make_init_pair(seed=s, n=1000) for s in range(8)]
    cap = max(max(len(p["f1"]["kps"]), len(p["f2"]["kps"])) for p in ip)
    NP = 64
    fb = FrameBatch(torch, 2 * NP, 1, cap, synth_init.W, synth_init.H, synth_init.scale_factors(), device=dev)
    prev0 = torch.zeros((NP, cap, 2), dtype=torch.float32, device=dev)
    for i in range(NP):
        p = ip[i % len(ip)]
        for k, f in enumerate(("f1", "f2")):
            kp = p[f]["kps"]
            fb.kps[2 * i + k, 0, :len(kp)] = torch.from_numpy(kp.view(np.int32).reshape(-1, 6).copy())
            fb.desc[2 * i + k, 0, :len(kp)] = torch.from_numpy(p[f]["desc"])
            fb.n_kp[2 * i + k, 0] = len(kp)
        prev0[i, :len(p["prev"])] = torch.from_numpy(p["prev"])
    mi = ORBmatcher(0.9, True)   # Tracking::MonocularInitialization: ORBmatcher(0.9, true), windowSize 100
    mi.AssignFeaturesToGrid(fb)
    prs = [(2 * i, 2 * i + 1) for i in range(NP)]
    prev = prev0.clone()

    def run_init():
        prev.copy_(prev0)
        return mi.SearchForInitialization(fb, prs, prev, 100, grid_ready=True)
    dt = _timed(run_init, 10, dev)
    _, ni = run_init()
    out["search_for_initialization"] = {"metric": "ORBmatcher::SearchForInitialization frame pairs/s",
                                        "value": round(NP / dt, 1), "unit": "frame pairs/s",
                                        "ms_per_batch": round(dt * 1e3, 3), "pairs_per_batch": NP,
                                        "matches_per_pair": round(float(ni.float().mean().item()), 1)}
    if cpu:
        g = oracle.frame_geom(1, synth_init.W, synth_init.H, synth_init.scale_factors())
        done, t = _cpu_rate(lambda: [oracle.search_for_initialization(g, p["f1"]["kps"], p["f1"]["desc"],
                                                                      p["f2"]["kps"], p["f2"]["desc"], p["prev"])
                                     for p in ip[:4]], 4)
        out["search_for_initialization"]["cpu_baseline"] = {
            "value": round(done / t, 1), "unit": "frame pairs/s", "cores": 1, "kind": "port",
            "sample": f"{done} pair searches, oracle, 1 thread, {t:.2f} s"}
    # ---- SearchBySim3: 32 keyframe pairs (5 blocks, ~900 projected map points per side), th 7.5
    from openmavis_amd import synth_sim3
    sb = synth_sim3.make_sim3_batch(n_pairs=32, seed=5)
    K, Cc, cap = sb["n_kf"], sb["n_cams"], sb["kp_cap"]
    skf = FrameBatch(torch, K, Cc, cap, sb["width"], sb["height"], scale, device=dev)
    skf.kps.copy_(torch.from_numpy(np.ascontiguousarray(sb["kps"]).view(np.int32).reshape(K, Cc, cap, 6)))
    skf.desc.copy_(torch.from_numpy(sb["desc"]))
    skf.n_kp.copy_(torch.from_numpy(sb["n_kp"]))
    smps = {k: torch.from_numpy(np.ascontiguousarray(v)).to(dev) for k, v in sb["mps"].items()}
    sl = [torch.from_numpy(np.ascontiguousarray(sb[k], np.int32)).to(dev) for k in ("kp1", "mp1", "kp2", "mp2")]
    from openmavis_amd.matcher import sim3_job_array
    sjobs = sim3_job_array(sb["jobs"])
    ms = ORBmatcher(0.75, True)
    ns = len(sb["jobs"])

    def run_sim3():
        return ms.SearchBySim3(skf, sjobs, *sl, smps, th=7.5)
    dt = _timed(run_sim3, 10, dev)
    _, nf = run_sim3()
    out["search_by_sim3"] = {"metric": "ORBmatcher::SearchBySim3 keyframe pairs/s (grid build included)",
                             "value": round(ns / dt, 1), "unit": "keyframe pairs/s", "ms_per_batch": round(dt * 1e3, 3),
                             "pairs_per_batch": ns, "points_per_pair": round((len(sb["kp1"]) + len(sb["kp2"])) / ns, 1),
                             "matches_per_pair": round(float(nf.float().mean().item()), 1)}
    if cpu:
        small = synth_sim3.make_sim3_batch(n_pairs=4, seed=5)
        done, t = _cpu_rate(lambda: oracle.search_by_sim3(small), 4)
        out["search_by_sim3"]["cpu_baseline"] = {
            "value": round(done / t, 1), "unit": "keyframe pairs/s", "cores": 1, "kind": "port",
            "sample": f"{done} pair searches (grid build included), oracle, 1 thread, {t:.2f} s"}
    # ---- map-point refresh: ComputeDistinctiveDescriptors + UpdateNormalAndDepth over 20,000 map points
    from openmavis_amd import mappoint, synth_mappoint
    mp = synth_mappoint.make_points(n_points=20000, seed=3)
    mg = synth_mappoint.make_geometry(n_points=20000, seed=4)
    md = {k: torch.from_numpy(np.ascontiguousarray(mp[k])).to(dev) for k in ("desc", "desc_start", "desc_row")}
    mgd = {k: torch.from_numpy(np.ascontiguousarray(v)).to(dev) for k, v in mg.items()}
    dt = _timed(lambda: mappoint.ComputeDistinctiveDescriptors(md["desc"], md["desc_start"], md["desc_row"]), 10, dev)
    dn = _timed(lambda: mappoint.UpdateNormalAndDepth(**mgd), 10, dev)
    out["mappoint_refresh"] = {"metric": "MapPoint::ComputeDistinctiveDescriptors + UpdateNormalAndDepth map points/s",
                               "value": round(20000 / (dt + dn), 1), "unit": "points/s",
                               "ms_distinctive": round(dt * 1e3, 3), "ms_normal_depth": round(dn * 1e3, 3),
                               "points_per_batch": 20000,
                               "descriptors_per_point": round(float(mp["desc_start"][-1]) / 20000, 2)}
    if cpu:
        sub = synth_mappoint.make_points(n_points=2000, seed=3)
        done, t = _cpu_rate(lambda: oracle.distinctive_descriptors(sub["desc"], sub["desc_start"], sub["desc_row"]),
                            2000)
        out["mappoint_refresh"]["cpu_baseline"] = {
            "value": round(done / t, 1), "unit": "points/s (distinctive descriptors only)", "cores": 1, "kind": "port",
            "sample": f"{done} points, oracle, 1 thread, {t:.2f} s"}
    # ---- LocalMapping::CreateNewMapPoints: the whole neighbour loop (SearchForTriangulation + geometry + AddMapPoint,
    # interleaved as the reference) of one keyframe against 20 neighbours
    from openmavis_amd import synth_cnmp
    from openmavis_amd.mapping import LocalMappingCall
    cd = synth_cnmp.make_cnmp_chain(seed=21, n_neigh=20)
    cc = LocalMappingCall(cd, ORBmatcher(0.6, False), inertial=True, device=dev)
    dt = _timed(lambda: cc.run(), 10, dev)
    out["create_new_map_points"] = {"metric": "LocalMapping::CreateNewMapPoints keyframes/s (20 neighbours, search + "
                                              "geometry interleaved)",
                                    "value": round(1 / dt, 1), "unit": "keyframes/s", "ms_per_keyframe": round(dt * 1e3, 3),
                                    "neighbours": len(cd["nbs"]),
                                    "keypoints_per_keyframe": int(cd["kf1"]["n"]),
                                    "new_points": int(cc.has_mp1.sum().item() - int(cd["kf1"]["has_mp"].sum()))}
    if cpu:
        done, t = _cpu_rate(lambda: oracle.local_mapping_create_new_map_points(cd, inertial=True), 1)
        out["create_new_map_points"]["cpu_baseline"] = {
            "value": round(done / t, 2), "unit": "keyframes/s", "cores": 1, "kind": "port",
            "sample": f"{done} keyframes x 20 neighbours, oracle, 1 thread, {t:.2f} s"}
    # ---- Optimizer::PoseOptimization: 256 frames of the 4-camera rig (~400 edges each), and one frame (latency)
    from openmavis_amd import synth_pose
    from openmavis_amd.optimizer import PoseInertialOptimizer
    pb0 = synth_pose.make_pose_only_batch(n_frames=16, n_pts=400, seed=9, n_cams=4)
    for F in (256, 1):
        pb = synth_pose.tile_batch(pb0, F)
        sel = [f % 16 for f in range(F)]
        q0 = torch.tensor(np.asarray(pb0["pose_q"])[sel], dtype=torch.float64, device=dev)
        t0 = torch.tensor(np.asarray(pb0["pose_t"])[sel], dtype=torch.float64, device=dev)
        pb["rig_q"], pb["rig_t"] = pb0["rig_q"], pb0["rig_t"]
        q, t = q0.clone(), t0.clone()
        arr = {k: torch.from_numpy(np.ascontiguousarray(pb[k])).to(dev) for k in PoseInertialOptimizer.EDGE_KEYS}
        kpo = torch.zeros((F, int(pb["kp_cap"])), dtype=torch.uint8, device=dev)
        po = PoseInertialOptimizer(max_frames=F, max_edges=max(len(pb["mono_cam"]), 1))

        def run_po():
            q.copy_(q0)
            t.copy_(t0)
            return po.PoseOptimization(pb, arr, q, t, kpo)
        dt = _timed(run_po, 10, dev)
        key = "pose_optimization" if F > 1 else "pose_optimization_b1"
        out[key] = {"metric": f"Optimizer::PoseOptimization frames/s (batch {F})", "value": round(F / dt, 1),
                    "unit": "frames/s", "ms_per_batch": round(dt * 1e3, 3), "frames_per_batch": F,
                    "edges_per_frame": round(len(pb["mono_cam"]) / F, 1)}
    if cpu:
        done, t = _cpu_rate(lambda: oracle.pose_optimization(pb0, frames=range(4)), 4)
        out["pose_optimization"]["cpu_baseline"] = {"value": round(done / t, 1), "unit": "frames/s", "cores": 1,
                                                    "kind": "port", "sample": f"{done} frames, oracle, 1 thread, {t:.2f} s"}
    return out


# ---- configs[3]: synthetic 8-camera Pinhole rig, 1920x1080, 2000 features/cam --------------------------------
P_W, P_H, P_C, P_NF, P_INI, P_MIN, P_M, P_TH = 1920, 1080, 8, 2000, 20, 7, 8000, 3.0


BYTES_FORMULA = {
    "pyr_resize": "SURVEY 8(d) once-only split: level 0 read once (the input) + levels 1..7 written once, per image "
                  "(one launch per level: the 7 level launches of a stream group are timed and counted together as one "
                  "'launch')",
    "fast_cells": "SURVEY 8(d) once-only split: levels 1..7 read once, per image (level 0's one read is the pyramid's)",
    "octree": "SURVEY 8(d) once-only split: 0 (its candidate lists are the design's intermediates; the traffic column "
              "shows what it moves)",
    "describe": "SURVEY 8(d) once-only split: 56 B per keypoint written (24 B record + 32 B descriptor; its patch "
                "reads are re-reads of levels counted once above)",
    "grid": "SURVEY 8(d) frame keypoints: 16 B per keypoint",
    "frustum": "per map point 32 B world data in + per (point, camera) 16 B track out (the SearchByProjection input)",
    "stereo_knn": "SURVEY 8(d) knn inputs: 2 x 1,200 descriptors x 32 B per frame",
    "proj_candidates": "SURVEY 8(d) map points 5,000 x (32 + 5 x 16) B + frame descriptors 32 B per keypoint",
    "proj_resolve": "SURVEY 8(d) outputs: 43,200 B per frame",
}
# The extraction kernels' budgets sum to SURVEY 8(d)'s once-only figure per image: sum(P) + sum(P[1:]) + 56 N
# (pyr_resize sum(P), fast_cells sum(P[1:]), octree 0, describe 56 N) -- 2,085,018 B at 720x540 / 1,200 features.


def rocprof_launch_avg(kernel):
    """Dispatch-trace average of `kernel` at its most-used grid in the newest committed
    profiles/<tag>_kernel_grid.json (tools/summarize_profile.py); None if absent."""
    path, r = newest_profile("kernel_grid")
    try:
        rows = [x for x in r["rows"] if x["kernel"] == kernel]
        if not rows:
            return None
        best = max(rows, key=lambda x: x["total_us"])
        return {"avg_launch_ms": round(best["avg_us"] / 1e3, 4), "avg_us": best["avg_us"], "grid": best["grid"],
                "calls": best["calls"], "source": path, "tag": r.get("tag")}
    except Exception:
        return None


def per_step_algorithmic_bytes(B, P, n_kp, n_cand):
    """Algorithmic bytes of one step (B frames) per kernel.  The extraction kernels split SURVEY §8(d)'s 2,085,018 B per
    image once-only (BYTES_FORMULA; they sum to it), the matching kernels SURVEY §8(d)'s 968,000 B per
    frame (frame keypoints 96,000 -> grid, map points 560,000 + frame descriptors 192,000 -> candidates, knn inputs
    76,800 -> knn, outputs 43,200 -> resolve); the design's own candidate records are not counted."""
    return {
        "pyr_resize": B * C * sum(P),
        "fast_cells": B * C * sum(P[1:]),
        "octree": 0,
        "describe": n_kp * 56,
        "grid": n_kp * 16,
        "frustum": B * M_MPS * (32 + C * 16),
        "stereo_knn": B * 2 * 1200 * 32,
        "proj_candidates": B * M_MPS * (32 + C * 16) + n_kp * 32,
        "proj_resolve": B * 43_200,
    }


def level_sizes(w, h, nlevels=NLEV, scale=SCALE):
    """Pyramid level sizes with the ORBextractor ctor's float arithmetic."""
    s = [1.0]
    for _ in range(1, nlevels):
        s.append(float(np.float32(s[-1] * np.float64(np.float32(scale)))))
    out = []
    for l in range(nlevels):
        invs = np.float32(1.0) / np.float32(s[l])
        out.append((int(np.rint(np.float32(w) * invs)), int(np.rint(np.float32(h) * invs))))
    return out


def cam_bytes(w, h, n_kp):
    """SURVEY §8(d) algorithmic bytes of one camera-frame's extraction: every level read once, every derived
    level written once, 56 B per keypoint (24 B record + 32 B descriptor)."""
    P = [a * b for a, b in level_sizes(w, h)]
    return sum(P) + sum(P[1:]) + 56 * n_kp


def _gen_p1080_image(item):
    from openmavis_amd import synth
    f, c = item
    return synth.synth_image(synth.P1080_SEED + 1000 * c + f, P_W, P_H)


def _gen_p1080_map(args):
    from openmavis_amd import synth
    kps, desc, n_kp, seed = args
    cams, R_cl, t_cl = synth.p1080_rig(P_C, P_W, P_H)
    pose = synth.random_pose(np.random.default_rng(seed))
    world, mp = synth.make_world_map(kps, desc, n_kp, P_M, seed, cams, R_cl, t_cl, pose, P_W, P_H, NLEV,
                                     model="pinhole")
    return pose, world, mp


def p1080_cpu_baseline(frames):
    """Oracle on a bounded sample: extraction of the 8 cameras (one std::thread each), isInFrustum through
    Pinhole::project and SearchByProjection over the 8 blocks."""
    oracle = _oracle(timing=True)
    from openmavis_amd import synth
    from openmavis_amd.matcher import make_rig
    cams, R_cl, t_cl = synth.p1080_rig(P_C, P_W, P_H)
    rig = make_rig(cams, R_cl, t_cl, P_W, P_H, model="pinhole")
    g = oracle.frame_geom(P_C, P_W, P_H, oracle.orb_tables(P_NF, SCALE, NLEV)["scale"])
    lap = np.zeros((P_C, 2), np.int32)
    preps = []
    for i, imgs in enumerate(frames):
        n_out, mono, kps, desc = oracle.orb_extract_frame(imgs, P_NF, lap, SCALE, NLEV, P_INI, P_MIN)
        preps.append(_gen_p1080_map((kps, desc, n_out, 900 + i)))
    t0 = time.perf_counter()
    for imgs, (pose, world, mp) in zip(frames, preps):
        n_out, mono, kps, desc = oracle.orb_extract_frame(imgs, P_NF, lap, SCALE, NLEV, P_INI, P_MIN)
        track, _ = oracle.frustum(rig, pose, world["pos"], world["normal"], world["min_dist"], world["max_dist"], 0.5,
                                  mp["view_cos"], mp["track_depth"])
        no = np.full(kps.shape[1], -1, np.int32)
        oracle.search_by_projection(g, kps, desc, n_out, dict(mp, **track), P_TH, False, 50.0, NNRATIO, no, no, None,
                                    np.full(P_C * kps.shape[1], -1, np.int32))
    dt = time.perf_counter() - t0
    return dict(value=round(len(frames) / dt, 3), unit="multi-cam frames/s", cores=P_C, kind="port",
                sample=f"{len(frames)} frames of 8 x 1920x1080 (2000 feat/cam, M={P_M}), oracle C++ restatement, "
                       f"one thread per camera, {dt:.1f} s")


def p1080_leg(imgs, B, steps, warmup, dev, world, rank, cpu):
    """BASELINE configs[3]: per frame, 8 Pinhole cameras 1920x1080 extracted (2000 features, iniTh 20, lapping
    [0,0]) + grid + isInFrustum (Pinhole::project) + SearchByProjection of an 8,000-point 3-D local map.  One GPU:
    the 8B images in one batch.  N GPUs: camera-sharded (rank r extracts cameras r, r+N, ...; one all-gather of
    the slabs; matching on rank 0).  imgs: this rank's images, frame-major [B][8] on one GPU, cam-major [k][B]
    (its k cameras) when sharded."""
    import torch
    import torch.distributed as tdist
    from openmavis_amd import synth
    from openmavis_amd.dist import CameraShard, job_seconds
    from openmavis_amd.matcher import FrameBatch, MapPointBatch, ORBmatcher, isInFrustum, make_rig
    from openmavis_amd.orb import ORBextractor
    shard = world > 1
    my_cams = list(range(rank, P_C, world)) if shard else list(range(P_C))
    n_img = len(my_cams) * B
    ex = ORBextractor(P_NF, SCALE, NLEV, P_INI, P_MIN, width=P_W, height=P_H, max_images=max(1, n_img))
    cap = ex.max_keypoints()
    fb = FrameBatch(torch, B, P_C, cap, P_W, P_H, ex.GetScaleFactors(), device=dev)
    d_img = torch.from_numpy(imgs).to(dev) if n_img else None
    lap = np.zeros((max(1, n_img), 2), np.int32)
    sh = CameraShard(rank, world, P_C, B, cap, dev, mode=_slab_mode()) if shard else None
    if shard:   # this rank's cameras, cam-major, straight into its slab
        kps_o, desc_o, n_o, mono_o = sh.outputs()
    else:       # frame-major images straight into the frame batch
        kps_o, desc_o, n_o, mono_o = fb.kps.view(-1, cap, 6), fb.desc.view(-1, cap, 32), fb.n_kp.view(-1), \
            fb.mono.view(-1)

    def extract():
        if n_img:
            ex.extract_batch(d_img, lap[:n_img], kps_o, desc_o, n_o, mono_o)

    def assemble():
        if shard:
            sh.gather(fb)

    extract()
    assemble()
    torch.cuda.synchronize(dev)
    assert ex.last_error() == 0, "p1080 extraction capacity error"
    cams, R_cl, t_cl = synth.p1080_rig(P_C, P_W, P_H)
    rig = make_rig(cams, R_cl, t_cl, P_W, P_H, model="pinhole")
    m = ORBmatcher(NNRATIO)
    if rank == 0:   # the tracking rank's 3-D local maps, from the frames' own keypoints (setup, untimed)
        kv = fb.kps.cpu().numpy().view(np.dtype([("x", "<f4"), ("y", "<f4"), ("size", "<f4"), ("angle", "<f4"),
                                                 ("response", "<f4"), ("octave", "<i4")])).reshape(B, P_C, cap)
        dh, nh = fb.desc.cpu().numpy(), fb.n_kp.cpu().numpy()
        per = [_gen_p1080_map((kv[f], dh[f], nh[f], 900 + f)) for f in range(B)]
        poses = torch.from_numpy(np.stack([p[0] for p in per])).to(dev)
        wmap = {k: torch.from_numpy(np.stack([p[1][k] for p in per])).to(dev) for k in per[0][1]}
        mps = MapPointBatch(**{k: torch.from_numpy(np.stack([p[2][k] for p in per])).to(dev) for k in per[0][2]})

    def step():
        extract()
        assemble()
        if rank == 0:
            fb.kp_to_mp.fill_(-1)
            m.AssignFeaturesToGrid(fb)
            isInFrustum(poses, rig, wmap, mps, 0.5)
            m.SearchByProjection(fb, mps, P_TH, False, 50.0, grid_ready=True)

    for _ in range(warmup):
        step()
    if shard:
        tdist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    torch.cuda.synchronize(dev)
    if shard:
        tdist.barrier()
    dt = job_seconds(time.perf_counter() - t0, dev)
    # extraction alone (HIP events on the launch stream): the §8(d) roofline of this rank's extraction launch
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    reps = 5
    ext_ms = None
    if n_img:
        ev0.record()
        for _ in range(reps):
            extract()
        ev1.record()
        torch.cuda.synchronize(dev)
        ext_ms = ev0.elapsed_time(ev1) / reps
    n_kp_img = int(n_o.sum().item()) if n_img else 0
    if rank != 0:
        return None
    bytes_launch = sum(cam_bytes(P_W, P_H, 0) for _ in range(n_img)) + 56 * n_kp_img
    out = {"metric": "multi-cam frames/s (8 x 1920x1080 Pinhole, ORB extract + isInFrustum + SearchByProjection)",
           "value": round(B * steps / dt, 2), "unit": "multi-cam frames/s", "ms_per_step": round(dt / steps * 1e3, 3),
           "frames_per_step": B, "n_gpus": world, "scaling": "strong" if shard else "weak",
           "matches_last_step": int(fb.n_matches.sum().item()),
           "config": {"workload": "synthetic 8-cam Pinhole rig 1920x1080, 2000 feat/cam, iniTh 20, lapping [0,0], "
                                  f"M={P_M} map points, th {P_TH}",
                      "parallelism": f"camera-sharded x{world} (RCCL all-gather of the slabs, matching on rank 0)"
                      if shard else "8-camera batch on one GPU"}}
    if ext_ms:
        ach = bytes_launch / (ext_ms * 1e-3) / 1e9
        out["extraction_roofline"] = {
            "kernel": "ORB extraction (pyramid + FAST + octree + describe), rank 0's launch", "bound": "hbm",
            "achieved": round(ach, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(ach / HBM_PEAK_GBS, 5),
            "avg_launch_ms": round(ext_ms, 4), "images_per_launch": n_img,
            "algorithmic_bytes_per_launch": bytes_launch,
            "bytes_per_camera_at_2000_kp": cam_bytes(P_W, P_H, 2000)}
    if cpu is not None:
        out["cpu_baseline"] = cpu
    return out


def cam_shard_leg(imgs, B, steps, warmup, dev, world, rank):
    """BASELINE configs[2]: the Hilti 5-camera frame with its cameras sharded over the ranks (rank r extracts
    cameras r, r+N, ...), ONE all-gather of the keypoint / descriptor slabs over RCCL, then the tracking rank's
    matching (grid, lapping knn, SearchByProjection; SURVEY §8e: matching is replicas only).  imgs: this rank's
    images, cam-major [k][B]."""
    import torch
    import torch.distributed as tdist
    from openmavis_amd.dist import CameraShard, job_seconds
    from openmavis_amd.matcher import FrameBatch, MapPointBatch, ORBmatcher
    from openmavis_amd.orb import ORBextractor
    from openmavis_amd import synth
    my_cams = list(range(rank, C, world))
    n_img = len(my_cams) * B
    ex = ORBextractor(NFEAT, SCALE, NLEV, INI_TH, MIN_TH, width=W, height=H, max_images=max(1, n_img))
    cap = ex.max_keypoints()
    fb = FrameBatch(torch, B, C, cap, W, H, ex.GetScaleFactors(), device=dev)
    sh = CameraShard(rank, world, C, B, cap, dev, mode=_slab_mode())
    kps_o, desc_o, n_o, mono_o = sh.outputs()
    d_img = torch.from_numpy(imgs).to(dev) if n_img else None
    lap = np.array([LAP[c] for c in my_cams for _ in range(B)], np.int32).reshape(-1, 2)
    m = ORBmatcher(NNRATIO)

    def gather():
        if n_img:
            ex.extract_batch(d_img, lap, kps_o, desc_o, n_o, mono_o)
        sh.gather(fb)

    gather()
    torch.cuda.synchronize(dev)
    if rank == 0:
        kv = fb.kps.cpu().numpy().view(np.dtype([("x", "<f4"), ("y", "<f4"), ("size", "<f4"), ("angle", "<f4"),
                                                 ("response", "<f4"), ("octave", "<i4")])).reshape(B, C, cap)
        dh, nh = fb.desc.cpu().numpy(), fb.n_kp.cpu().numpy()
        per = [synth.make_map_points(kv[f], dh[f], nh[f], M_MPS, 300 + f, W, H) for f in range(B)]
        mps = MapPointBatch(**{k: torch.from_numpy(np.stack([p[k] for p in per])).to(dev) for k in per[0]})

    def step():
        gather()
        if rank == 0:
            fb.kp_to_mp.fill_(-1)
            m.AssignFeaturesToGrid(fb)
            m.StereoLapping(fb, 0.8)
            m.SearchByProjection(fb, mps, TH, False, 50.0, grid_ready=True)

    for _ in range(warmup):
        step()
    tdist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    torch.cuda.synchronize(dev)
    tdist.barrier()
    dt = job_seconds(time.perf_counter() - t0, dev)
    if rank != 0:
        return None
    return {"metric": "multi-cam frames/s (5x720x540, cameras sharded over the GPUs)",
            "value": round(B * steps / dt, 2), "unit": "multi-cam frames/s", "ms_per_step": round(dt / steps * 1e3, 3),
            "frames_per_step": B, "n_gpus": world, "scaling": "strong",
            "slab_bytes_per_rank": sh.words * 4, "matches_last_step": int(fb.n_matches.sum().item()),
            "config": {"workload": "Hilti-like 5 cams 720x540, 1200 feat/cam: extraction sharded one camera per "
                                   "GPU, RCCL all-gather of keypoints + descriptors, grid + lapping knn + "
                                   f"SearchByProjection(M={M_MPS}) on rank 0",
                       "parallelism": f"camera-sharded x{world}"}}


def latency_leg(d_img, gr0, n_frames, dev, rig, stereo):
    """Single-frame latency of the sequential tracker (frame t+1's search needs frame t's pose): one multi-camera
    frame at a time on one stream (B = 1), extract + grid + lapping knn + TriangulateMatches + mvuRight +
    isInFrustum + SearchByProjection, then the pose graph's edges from SearchByProjection's assignment and
    PoseInertialOptimizationLastFrame + ConstraintPoseImu (Tracking::TrackLocalMap's optimisation), all on the
    device, synchronised per frame; p50 / p99 of the per-frame wall time, with and without the optimisation.
    The optimisation's frame state / previous frame / prior / preintegration are synthetic (synth_pose's
    trajectory), the local map moved rigidly so the frame's block-0 camera sits at the true body pose."""
    import torch
    from openmavis_amd.frame import frame_uright
    from openmavis_amd.matcher import FrameBatch, MapPointBatch, ORBmatcher, isInFrustum
    from openmavis_amd.orb import ORBextractor
    ex = ORBextractor(NFEAT, SCALE, NLEV, INI_TH, MIN_TH, width=W, height=H, max_images=C)
    cap = ex.max_keypoints()
    fb = FrameBatch(torch, 1, C, cap, W, H, ex.GetScaleFactors(), device=dev)
    m = ORBmatcher(NNRATIO)
    n_avail = gr0["poses"].shape[0]
    frames = []
    for f in range(n_avail):
        frames.append(dict(img=d_img[f * C:(f + 1) * C], pose=gr0["poses"][f:f + 1],
                           world={k: v[f:f + 1] for k, v in gr0["world"].items()},
                           mps=MapPointBatch(**{k: getattr(gr0["mps"], k)[f:f + 1].clone()
                                                for k in MapPointBatch.FIELDS}),
                           depth=gr0["depth"][f:f + 1].contiguous()))
    from openmavis_amd import synth_pose
    from openmavis_amd.optimizer import PoseInertialOptimizer
    NB = min(4, C)
    ur_full = torch.full((C, cap), -1.0, dtype=torch.float32, device=dev)   # mvuRight [C][cap]; blocks >= 4: -1
    ur = ur_full[:NB].view(1, NB, cap)
    Rlr, tlr, BF, sigma2, cams_r = stereo
    E = C * cap
    popt = PoseInertialOptimizer(max_frames=1, max_edges=E)
    edges = PoseInertialOptimizer.edge_arrays(E, dev)
    inv_s2 = [float(1.0 / x) for x in sigma2]
    kpo = torch.zeros((1, C * cap), dtype=torch.uint8, device=dev)
    Hm = torch.zeros((1, 225), dtype=torch.float64, device=dev)
    Hc = torch.zeros((1, 225), dtype=torch.float64, device=dev)
    for f, fr in enumerate(frames):
        b = synth_pose.make_last_frame_batch(n_frames=1, n_pts=8, seed=100 + f, n_cams=C)
        b["bf"] = np.float32(BF)
        b["kp_cap"] = C * cap
        b["mono_cam"] = b["stereo_cam"] = np.zeros(E, np.int32)   # edge-list bounds (counts live on the device)
        Rwb, twb = np.asarray(b["true_Rwb"][0]), np.asarray(b["true_twb"][0])
        Rwc = Rwb @ b["Rbc"][0]
        twc = Rwb @ b["tbc"][0] + twb
        po = fr["pose"][0].cpu().numpy().astype(np.float64)
        R_no = Rwc @ po[:9].reshape(3, 3)
        t_no = Rwc @ po[9:12] + twc
        pos = fr["world"]["pos"][0].cpu().numpy().astype(np.float64)
        arrays = dict(edges)
        for k in synth_pose.STATE_KEYS:
            arrays[k] = torch.tensor(np.asarray(b[k], np.float64), device=dev).contiguous()
        for k in synth_pose.INPUT_KEYS[:6] + synth_pose.PRIOR_KEYS:
            arrays[k] = torch.from_numpy(np.ascontiguousarray(b[k])).to(dev)
        fr.update(pose_batch=b, pose_arrays=arrays,
                  mp_pos=torch.from_numpy((pos @ R_no.T + t_no).astype(np.float32)).to(dev))

    def pose(fr):
        popt.EdgesFromMatches(fb.kps[0], fb.n_kp[0], fb.kp_to_mp[0], fr["mp_pos"], fr["mps"].track_depth[0], inv_s2,
                              edges, uright=ur_full)
        popt.PoseInertialOptimizationLastFrame(fr["pose_batch"], fr["pose_arrays"], kpo, Hm)
        PoseInertialOptimizer.ConstraintPoseImu(Hm, out=Hc)

    def one(fr, with_pose=True):
        ex.extract_batch(fr["img"], LAP, fb.kps.view(-1, cap, 6), fb.desc.view(-1, cap, 32), fb.n_kp.view(-1),
                         fb.mono.view(-1))
        fb.kp_to_mp.fill_(-1)
        m.AssignFeaturesToGrid(fb)
        m.StereoLapping(fb, 0.8)
        m.StereoTriangulate(fb, cams_r[:2], Rlr, tlr, sigma2)
        frame_uright(fb, fr["depth"], BF, out=ur)
        isInFrustum(fr["pose"], rig, fr["world"], fr["mps"], 0.5)
        m.SearchByProjection(fb, fr["mps"], TH, False, 50.0, grid_ready=True)
        if with_pose:
            pose(fr)

    def run(with_pose):
        for i in range(5):
            one(frames[i % n_avail], with_pose)
        torch.cuda.synchronize(dev)
        lat = []
        for i in range(n_frames):
            t0 = time.perf_counter()
            one(frames[i % n_avail], with_pose)
            torch.cuda.synchronize(dev)
            lat.append((time.perf_counter() - t0) * 1e3)
        return np.array(lat)

    lat = run(True)
    if popt.last_error() != 0:
        raise RuntimeError("latency leg: pose edge / optimisation capacity error")
    n_edges = [int(x) for x in (edges["mono_start"][1].item(), edges["stereo_start"][1].item())]
    lat0 = run(False)
    return {"metric": "single-frame latency (B=1, one stream, synchronised per frame)", "unit": "ms",
            "chain": "extract + grid + lapping knn + TriangulateMatches + mvuRight + isInFrustum + SearchByProjection "
                     "+ edges from matches + PoseInertialOptimizationLastFrame + ConstraintPoseImu",
            "p50_ms": round(float(np.percentile(lat, 50)), 4), "p99_ms": round(float(np.percentile(lat, 99)), 4),
            "mean_ms": round(float(lat.mean()), 4), "frames": n_frames,
            "sequential_frames_per_s": round(1e3 / float(np.percentile(lat, 50)), 1),
            "last_frame_edges": {"mono": n_edges[0], "stereo": n_edges[1]},
            "without_pose": {"p50_ms": round(float(np.percentile(lat0, 50)), 4),
                             "p99_ms": round(float(np.percentile(lat0, 99)), 4)}}


def _slab_mode():
    import torch.distributed as tdist
    return "host" if tdist.get_backend() == "gloo" else "device"


def _launch_ranks(n):
    """--gpus N > 1 outside torch.distributed: start N ranks (one process per GPU) and return their status."""
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.run(cmd, env=dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")).returncode


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--frames", type=int, default=384, help="multi-cam frames per step per GPU")
    ap.add_argument("--streams", type=int, default=3,
                    help="frame groups per GPU, each on its own HIP stream (latency-bound matcher stages of one "
                         "group overlap extraction of another)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--stage-timing", type=int, default=1)
    ap.add_argument("--parity-check", type=int, default=1,
                    help="untimed oracle check of frames of the last timed step (--parity-frames)")
    ap.add_argument("--parity-frames", default="0:0,-1:-1",
                    help="group:frame list ('*' = every group, negative = from the end); default group 0's first "
                         "frame and the last group's last frame")
    ap.add_argument("--lba-steps", type=int, default=10, help="LocalInertialBA optimize() calls timed (0: skip)")
    ap.add_argument("--lba-warmup", type=int, default=2)
    ap.add_argument("--lba-shard", action="store_true",
                    help="N>1: shard one window's landmarks over the ranks (RCCL all-reduce per LM trial) "
                         "instead of running a window replica per rank")
    ap.add_argument("--cpu-frames", type=int, default=500, help="timed frames of the mode-A CPU sample (BASELINE.md §2)")
    ap.add_argument("--cpu-warmup-frames", type=int, default=50)
    ap.add_argument("--cpu-distinct-frames", type=int, default=100, help="distinct frames cycled by the CPU samples")
    ap.add_argument("--cpu-best-frames", type=int, default=500, help="frames in the mode-B (whole CPU share) sample")
    ap.add_argument("--cpu-lba-trials", type=int, default=200, help="timed LM trials of the CPU BA sample (+10 warm-up)")
    ap.add_argument("--pose-frames", type=int, default=1024, help="frames per PoseInertialOptimization batch (0: skip)")
    ap.add_argument("--tri-pairs", type=int, default=256, help="keyframe pairs per SearchForTriangulation batch (0: skip)")
    ap.add_argument("--aux", type=int, default=1, help="Fuse / DBoW2 transform / IMU preintegration legs (0: skip)")
    ap.add_argument("--p1080-frames", type=int, default=16, help="configs[3] 8 x 1920x1080 frames per step (0: skip)")
    ap.add_argument("--p1080-steps", type=int, default=10)
    ap.add_argument("--p1080-cpu-frames", type=int, default=2)
    ap.add_argument("--shard-frames", type=int, default=64, help="N>1: frames per step of the camera-sharded leg")
    ap.add_argument("--latency-frames", type=int, default=200, help="B=1 sequential frames timed (0: skip)")
    ap.add_argument("--iso-reps", type=int, default=3,
                    help="isolated single-stream passes of one group for the per-kernel roofline (0: skip)")
    args = ap.parse_args()

    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(_launch_ranks(args.gpus))   # before anything touches a GPU
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    B = args.frames
    first = rank * B
    do_cpu = not args.no_cpu_baseline and world == 1
    if do_cpu:
        _build_native_oracle()   # before the worker pool forks (the workers inherit NATIVE_LIB)
    # inputs are generated before anything touches the GPU (host pool = plain fork, no HIP yet)
    imgs = np.concatenate(_pool_map(_gen_frame, list(range(first, first + B))))   # [B*C, H, W]
    cpu = p1080_cpu = lba_cpu = None
    lba_prob = None
    if args.lba_steps > 0:
        from openmavis_amd import synth_ba
        lba_prob = synth_ba.make_lba_problem(seed=5)   # configs[4] window (same on every rank)
    p_imgs = None
    if args.p1080_frames > 0:
        PB = args.p1080_frames
        items = [(f, c) for f in range(PB) for c in range(P_C)] if world == 1 else \
            [(f, c) for c in range(rank, P_C, world) for f in range(PB)]
        p_imgs = np.stack(_pool_map(_gen_p1080_image, items)) if items else np.zeros((0, P_H, P_W), np.uint8)
        if do_cpu and args.p1080_cpu_frames > 0:
            p1080_cpu = p1080_cpu_baseline([np.stack([_gen_p1080_image((10_000 + f, c)) for c in range(P_C)])
                                            for f in range(args.p1080_cpu_frames)])
    s_imgs = None
    if world > 1 and args.shard_frames > 0:
        SB = args.shard_frames
        s_imgs = np.stack([img for c in range(rank, C, world) for img in
                           _pool_map(_gen_cam_image, [(c, 20_000 + f) for f in range(SB)])]) \
            if rank < C else np.zeros((0, H, W), np.uint8)
    if do_cpu:   # CPU baselines on this host, before the GPU work
        cpu_frames = _pool_map(_gen_frame, list(range(10_000, 10_000 + args.cpu_distinct_frames)))
        cpu = cpu_baseline(cpu_frames, args.cpu_frames, args.cpu_warmup_frames, args.cpu_best_frames)
        if lba_prob is not None:
            lba_cpu = lba_cpu_baseline(lba_prob, args.cpu_lba_trials)
    pose_batch = pose_cpu = lf_batch = lf_cpu = None
    if args.pose_frames > 0:
        from openmavis_amd import synth_pose
        pose_cpu = synth_pose.make_pose_batch(n_frames=32, n_pts=1000, seed=1, outlier_frac=0.1)
        pose_batch = synth_pose.tile_batch(pose_cpu, args.pose_frames)
        lf_cpu = synth_pose.make_last_frame_batch(n_frames=32, n_pts=1000, seed=1, outlier_frac=0.1)
        lf_batch = synth_pose.tile_batch(lf_cpu, args.pose_frames)
    tri_pairs = None
    if args.tri_pairs > 0:
        from openmavis_amd import synth_tri
        tri_pairs = [synth_tri.make_tri_pair(seed=s, n_pts=1200, n_distract=600) for s in range(16)]
    _close_pool()   # no forked worker outlives the host phase

    import torch
    import torch.distributed as dist

    # OMV_BENCH_REHEARSE=1: rehearse the N-rank path on a box with fewer GPUs (ranks share cards, gloo collectives,
    # slabs staged through host memory); never used for a reported number
    rehearse = os.environ.get("OMV_BENCH_REHEARSE") == "1"
    dev = torch.device("cuda", (local % torch.cuda.device_count()) if rehearse else (local if world > 1 else 0))
    torch.cuda.set_device(dev)
    if world > 1:
        if rehearse:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=dev)

    from openmavis_amd.dist import job_seconds
    from openmavis_amd import synth
    from openmavis_amd.matcher import FrameBatch, MapPointBatch, ORBmatcher, isInFrustum, make_rig
    from openmavis_amd.orb import ORBextractor

    d_img = torch.from_numpy(imgs).to(dev)
    G = max(1, args.streams)
    if B % G:
        raise SystemExit(f"--frames {B} is not a multiple of --streams {G}")
    Bg = B // G
    groups = []
    for gi in range(G):
        ex = ORBextractor(NFEAT, SCALE, NLEV, INI_TH, MIN_TH, width=W, height=H, max_images=Bg * C)
        cap = ex.max_keypoints()
        groups.append(dict(
            ex=ex, cap=cap, fb=FrameBatch(torch, Bg, C, cap, W, H, ex.GetScaleFactors(), device=dev),
            img=d_img[gi * Bg * C:(gi + 1) * Bg * C], lap=np.tile(LAP, (Bg, 1)), matcher=ORBmatcher(NNRATIO),
            stream=torch.cuda.Stream(dev) if G > 1 else torch.cuda.current_stream(dev)))

    def extract(gr):
        gr["ex"].extract_batch(gr["img"], gr["lap"], gr["fb"].kps.view(-1, gr["cap"], 6),
                               gr["fb"].desc.view(-1, gr["cap"], 32), gr["fb"].n_kp.view(-1), gr["fb"].mono.view(-1),
                               stream=gr["stream"])

    # map points derived from this batch's keypoints (setup, untimed)
    kp_dtype = np.dtype([("x", "<f4"), ("y", "<f4"), ("size", "<f4"), ("angle", "<f4"), ("response", "<f4"),
                         ("octave", "<i4")])
    nkp_h = []
    parity_frames = []
    parity_sel = [tuple(x.split(":")) for x in args.parity_frames.split(",")] if args.parity_check else []
    parity_sel = [(g_, int(f)) for g_, f in parity_sel]
    for gi, gr in enumerate(groups):
        extract(gr)
        torch.cuda.synchronize(dev)
        if gr["ex"].last_error() != 0:
            raise RuntimeError("extractor capacity error")
        fb, cap = gr["fb"], gr["cap"]
        kps_h = fb.kps.cpu().numpy().view(kp_dtype).reshape(Bg, C, cap)
        desc_h = fb.desc.cpu().numpy()
        nk = fb.n_kp.cpu().numpy()
        nkp_h.append(nk)
        per = [_gen_map((kps_h[f], desc_h[f], nk[f], 7000 + first + gi * Bg + f)) for f in range(Bg)]
        # the post-run parity check's frames: host copies of their images and maps
        for f in sorted({f % Bg for g_, f in parity_sel if g_ == "*" or int(g_) % G == gi}):
            parity_frames.append((gi, f, imgs[(gi * Bg + f) * C:(gi * Bg + f + 1) * C], per[f]))
        gr["poses"] = torch.from_numpy(np.stack([p[0] for p in per])).to(dev)
        gr["world"] = {k: torch.from_numpy(np.stack([p[1][k] for p in per])).to(dev) for k in per[0][1]}
        gr["mps"] = MapPointBatch(**{k: torch.from_numpy(np.stack([p[2][k] for p in per])).to(dev) for k in per[0][2]})
        gr["ev"] = []
    nkp_h = np.concatenate(nkp_h)
    n_cand_step = sum(gr["ex"].last_counts()[0] for gr in groups)   # FAST candidates of one step (octree input)

    cams_r, R_cl, t_cl = synth.hilti_rig(C)
    rig = make_rig(cams_r, R_cl, t_cl, W, H, SCALE, NLEV)
    # Frame ctor tail: the lapping pairs' TriangulateMatches (mRlr / mtlr = left-from-right) and mvuRight
    # from the 4 reference blocks' undistorted depth images (synthetic, resident: 0-25 m, holes)
    from openmavis_amd.frame import frame_uright
    Rlr = R_cl[1].T.astype(np.float32)
    tlr = (-R_cl[1].T @ t_cl[1]).astype(np.float32)
    BF = float(cams_r[0][0] * np.linalg.norm(tlr))
    sigma2 = (np.float32(SCALE) ** (2 * np.arange(NLEV))).astype(np.float32)
    NB = min(4, C)
    gdep = torch.Generator(device=dev).manual_seed(1234 + first)
    for gr in groups:
        gr["depth"] = torch.rand((Bg, NB, H, W), generator=gdep, device=dev, dtype=torch.float32) * 25.0
        gr["uright"] = torch.empty((Bg, NB, gr["cap"]), dtype=torch.float32, device=dev)
    timing_on = [False]

    def group_step(gr, sync_frustum=False):
        """One group's pass; sync_frustum: return isInFrustum's event time (synchronises that stream)."""
        fb, st = gr["fb"], gr["stream"]
        extract(gr)
        with torch.cuda.stream(st):
            fb.kp_to_mp.fill_(-1)                   # Frame ctor: mvpMapPoints = vector(N, nullptr)
        gr["matcher"].AssignFeaturesToGrid(fb, stream=st)
        gr["matcher"].StereoLapping(fb, 0.8, stream=st)
        gr["matcher"].StereoTriangulate(fb, cams_r[:2], Rlr, tlr, sigma2, stream=st)
        frame_uright(fb, gr["depth"], BF, stream=st, out=gr["uright"])
        timed = timing_on[0] or sync_frustum
        if timed:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(st)
        isInFrustum(gr["poses"], rig, gr["world"], gr["mps"], 0.5, stream=st)   # Tracking::SearchLocalPoints
        if timed:
            e1.record(st)
            if not sync_frustum:
                gr["ev"].append((e0, e1))
        gr["matcher"].SearchByProjection(fb, gr["mps"], TH, False, 50.0, stream=st, grid_ready=True)
        if sync_frustum:
            e1.synchronize()
            return e0.elapsed_time(e1)
        return 0.0

    def step():
        for gr in groups:
            group_step(gr)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(dev)
    if args.stage_timing:
        for gr in groups:
            gr["ex"].enable_timing(True)
            gr["matcher"].enable_timing(True)
            gr["ex"].stage_ms(reset=True)
            gr["matcher"].stage_ms(reset=True)
            gr["ev"].clear()
        timing_on[0] = True
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    dt = job_seconds(time.perf_counter() - t0, dev)   # max over ranks
    assert all(gr["ex"].last_error() == 0 for gr in groups)
    n_matches = int(sum(gr["fb"].n_matches.sum().item() for gr in groups))
    # untimed: the last timed step's outputs of two frames against the CPU oracle (checker only)
    parity = parity_post_run(parity_frames, groups, rig, cams_r, Rlr, tlr, sigma2, BF) \
        if args.parity_check and rank == 0 else None

    # per-stage device time per step, summed over the stream groups (groups overlap in time)
    stages = {}
    if args.stage_timing:
        for gr in groups:
            es, calls = gr["ex"].stage_ms(reset=True)
            ms = gr["matcher"].stage_ms(reset=True)
            for k, v in {**es, **ms}.items():
                stages[k] = stages.get(k, 0.0) + v / args.steps
            stages["frustum"] = stages.get("frustum", 0.0) + sum(a.elapsed_time(b) for a, b in gr["ev"]) / args.steps
            gr["ex"].enable_timing(False)
            gr["matcher"].enable_timing(False)

    # isolated per-stage device time: group 0's pipeline alone on its stream (no other group running), HIP events
    # on that stream around each stage — the per-launch durations the roofline uses (rocprof's per-grid rows of
    # the same launches agree; the overlapped stage times above include other streams' work)
    iso = {}
    if args.iso_reps > 0:
        gr0 = groups[0]
        for gr in groups:
            gr["ex"].enable_timing(False)
            gr["matcher"].enable_timing(False)
        gr0["ex"].enable_timing(True)
        gr0["matcher"].enable_timing(True)
        gr0["ex"].stage_ms(reset=True)
        gr0["matcher"].stage_ms(reset=True)
        fr_ms = 0.0
        for _ in range(args.iso_reps):
            torch.cuda.synchronize(dev)
            fr_ms += group_step(gr0, True)
        torch.cuda.synchronize(dev)
        es, calls = gr0["ex"].stage_ms(reset=True)
        iso = {k: v / args.iso_reps for k, v in {**es, **gr0["matcher"].stage_ms(reset=True)}.items()}
        iso["frustum"] = fr_ms / args.iso_reps
        gr0["ex"].enable_timing(False)
        gr0["matcher"].enable_timing(False)
    lat = latency_leg(d_img, groups[0], args.latency_frames, dev, rig, (Rlr, tlr, BF, sigma2, cams_r)) \
        if args.latency_frames > 0 and rank == 0 else None
    shard_leg = cam_shard_leg(s_imgs, args.shard_frames, 10, 2, dev, world, rank) \
        if s_imgs is not None else None
    p1080 = p1080_leg(p_imgs, args.p1080_frames, args.p1080_steps, 2, dev, world, rank, p1080_cpu) \
        if p_imgs is not None else None
    lba = lba_leg(lba_prob, args.lba_steps, args.lba_warmup, dev, world, args.lba_shard) if lba_prob is not None else None
    if lba is not None and lba_cpu is not None:
        lba["cpu_baseline"] = lba_cpu
    pose = pose_leg(pose_batch, pose_cpu if rank == 0 and not args.no_cpu_baseline else None, 10, dev) \
        if pose_batch is not None else None
    pose_lf = pose_leg(lf_batch, lf_cpu if rank == 0 and not args.no_cpu_baseline else None, 10, dev, last_frame=True) \
        if lf_batch is not None else None
    tri = tri_leg(tri_pairs, args.tri_pairs, 10, dev) if tri_pairs is not None else None
    aux = aux_legs(dev, rank == 0 and not args.no_cpu_baseline) if args.aux else {}

    if rank != 0:
        if world > 1:
            dist.destroy_process_group()
        return

    total_frames = B * world * args.steps
    value = total_frames / dt
    # roofline per kernel: algorithmic bytes per launch (SURVEY §8(d) split over the kernels) / the
    # kernel's average launch duration, two views: "overlapped" = HIP events on the launch stream during the timed
    # steps (3 groups overlapping, what rocprof's kernel-trace average of the bench run shows) and "isolated" =
    # group 0 alone after the timed steps
    P = [a * b for a, b in level_sizes(W, H)]
    n_kp_step = int(nkp_h.sum())   # keypoints per step (same frames every step)
    per_step_bytes = per_step_algorithmic_bytes(B, P, n_kp_step, n_cand_step)
    roof = None
    kernels = {}
    ov = {k: v / G for k, v in stages.items()}   # ms per launch in the overlapped timed run
    for k in per_step_bytes:
        t_ov, t_iso = ov.get(k, 0.0), iso.get(k, 0.0)
        if t_ov <= 0 and t_iso <= 0:
            continue
        alg = per_step_bytes[k] // G
        rec = {"algorithmic_bytes_per_launch": int(alg), "launches_per_step": G, "bytes_formula": BYTES_FORMULA[k],
               "traffic": None}
        for view, t in (("overlapped", t_ov), ("isolated", t_iso)):
            if t > 0:
                ach = alg / (t * 1e-3) / 1e9
                rec[view] = {"avg_launch_ms": round(t, 4), "ms_per_step": round(t * G, 4), "achieved": round(ach, 2),
                             "frac": round(ach / HBM_PEAK_GBS, 5)}
        pmc, r = newest_profile(f"pmc_{k}")
        if r is not None:   # PMC HBM bytes (tools/profile_gpu.sh), scaled to this launch
            try:
                if "hbm_bytes_per_image" in r:
                    rec["traffic"] = int(r["hbm_bytes_per_image"] * Bg * C)
                elif "hbm_bytes_per_frame" in r:
                    rec["traffic"] = int(r["hbm_bytes_per_frame"] * Bg)
                if rec["traffic"] is not None:
                    rec["traffic_source"] = f"{pmc} ({r['tag']}, program {r.get('program', 'orb')})"
                    rec["traffic_ratio"] = round(rec["traffic"] / alg, 3) if alg > 0 else None
            except Exception:
                pass
        kernels[k] = rec
    if kernels:
        view = "overlapped" if any("overlapped" in r for r in kernels.values()) else "isolated"
        dom = max((k for k in kernels if view in kernels[k]), key=lambda k: kernels[k][view]["ms_per_step"])
        d = kernels[dom]
        # the headline fraction is the device-time view: the committed rocprofv3 dispatch trace of this round's bench
        # launches (profiles/<tag>_kernel_grid.json, the dominant kernel's bench-grid rows); the HIP events on the launch
        # stream -- which also hold the time a launch queues behind the other two streams' kernels -- sit beside it
        rp = rocprof_launch_avg(dom)
        ev = {"achieved": d[view]["achieved"], "frac": d[view]["frac"], "avg_launch_ms": d[view]["avg_launch_ms"],
              "timing": ("HIP events on the launch stream over the timed steps (3 stream groups overlapping)"
                         if view == "overlapped" else "HIP events on the launch stream, group 0 alone")}
        roof = {"kernel": dom, "bound": "hbm", "peak": HBM_PEAK_GBS, "unit": "GB/s", "traffic": d["traffic"],
                "algorithmic_bytes_per_launch": d["algorithmic_bytes_per_launch"], "frames_per_launch": Bg,
                "bytes_formula": d["bytes_formula"], "dominant_by": "largest ms per step (HIP events, overlapped)",
                "events": ev}
        if rp is not None:
            ach = d["algorithmic_bytes_per_launch"] / (rp["avg_us"] * 1e-6) / 1e9
            roof.update(achieved=round(ach, 2), frac=round(ach / HBM_PEAK_GBS, 6), avg_launch_ms=rp["avg_launch_ms"],
                        timing=f"rocprofv3 --kernel-trace dispatch average of the bench-grid launches ({rp['source']}, "
                               f"grid {rp['grid']}, {rp['calls']} calls): device time only",
                        rocprof=rp)
        else:
            roof.update(achieved=ev["achieved"], frac=ev["frac"], avg_launch_ms=ev["avg_launch_ms"], timing=ev["timing"])
        if d.get("traffic_source"):
            roof["traffic_source"] = d["traffic_source"]
        iso_k = [k for k in kernels if "isolated" in kernels[k]]
        if iso_k:
            di = max(iso_k, key=lambda k: kernels[k]["isolated"]["avg_launch_ms"])
            roof["isolated"] = dict(kernel=di, **kernels[di]["isolated"])
        if dom in iso and "isolated" in d:
            roof["dominant_isolated_view"] = d["isolated"]
        # PMC-measured extraction bytes per image vs SURVEY §8(d)'s 2,085,018 B per image
        ext = ("pyr_resize", "fast_cells", "octree", "describe")
        pm = [r for r in (newest_profile(f"pmc_{k}")[1] for k in ext) if r is not None]
        per_img = sum(r.get("hbm_bytes_per_image", 0) for r in pm)
        if per_img:
            ref_img = cam_bytes(W, H, n_kp_step / (B * C))
            roof["extraction_traffic_ratio"] = round(per_img / ref_img, 3)
            roof["extraction_traffic_bytes_per_image"] = int(per_img)
            roof["extraction_algorithmic_bytes_per_image"] = int(ref_img)
        # what does bound the extraction kernels: instruction issue from the SQ PMC passes (tools/pmc_orb_bound.sh,
        # profiles/<tag>_orb_bound.json) against this run's isolated launch times.  Chip VALU issue rate: 1,024 SIMDs,
        # one wave64 VALU instruction per 2 cycles at 2.4 GHz (MI355X_MICROARCH.md); LDS: one instruction per CU-cycle.
        bpath, bnd = newest_profile("orb_bound")
        if bnd is not None:
            imgs = Bg * C
            issue = {"source": f"{bpath} ({bnd.get('tag')})", "peak_valu_wave_insts_per_s": 1024 * 2.4e9 / 2,
                     "kernels": {}}
            for k, r in bnd.get("kernels", {}).items():
                t = kernels.get(k, {}).get("isolated", {}).get("avg_launch_ms")
                if not t:
                    continue
                waves = r["waves_per_image"] * imgs
                vf = waves * r["valu_per_wave"] / (t * 1e-3) / (1024 * 2.4e9 / 2)
                lf = waves * r["lds_per_wave"] / (t * 1e-3) / (256 * 2.4e9)
                issue["kernels"][k] = {"valu_issue_frac": round(vf, 3), "lds_issue_frac": round(lf, 3),
                                       "per_wave_active_valu": r["active_valu"], "per_wave_wait_any": r["wait_any"],
                                       "valu_per_wave": r["valu_per_wave"], "waves_per_launch": int(waves)}
            if issue["kernels"]:
                top = max(issue["kernels"], key=lambda k: issue["kernels"][k]["valu_issue_frac"])
                vf = issue["kernels"][top]["valu_issue_frac"]
                issue["bound"] = (f"VALU issue: {top} issues {vf:.0%} of the chip's VALU rate at < 10 % of HBM"
                                  if vf >= 0.5 else
                                  f"latency: the busiest kernel ({top}) issues {vf:.0%} of the chip's VALU rate")
                roof["extraction_issue"] = issue
        # the whole path: SURVEY §8(d) bytes of a multi-camera frame (5 extractions + matching) x frames/s
        frame_bytes = C * cam_bytes(W, H, 0) + 56 * n_kp_step / B + 968_000
        roof["pipeline"] = {"bytes_per_frame": int(frame_bytes), "achieved": round(frame_bytes * value / 1e9, 2),
                            "unit": "GB/s", "frac": round(frame_bytes * value / 1e9 / HBM_PEAK_GBS, 5)}
    out = {
        "metric": "multi-cam frames/sec (ORB extract+match) + LocalBA iters/sec, 5x720x540",
        "value": round(value, 2),
        "unit": "multi-cam frames/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(dt / args.steps * 1e3, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic (seeded Hilti-like 5x720x540 frames; 5000-point local maps from the frames' own keypoints)",
        "config": {"workload": "Hilti-2022 exp04-like 5 cams 720x540, 1200 feat/cam, ORB extract + lapping knn + "
                               "stereo TriangulateMatches + mvuRight from depth + SearchByProjection(M=5000, th=6)",
                   "frames_per_step_per_gpu": B, "streams_per_gpu": G, "parallelism": f"frame-replicas x{world}"},
        "stage_ms_per_step": {k: round(v, 4) for k, v in stages.items()},
        "stage_ms_note": "stage_ms_per_step: HIP events per stream while the 3 groups overlap (includes other streams' "
                         "kernels); kernels: isolated per-launch roofline of each stage",
        "kernels": kernels,
        "matches_last_step": n_matches,
        "parity_post_run": parity,
        "parity_checked_frames": len(parity["frames"]) if parity and parity["bit_exact"] else 0,
        "roofline": roof,
        "cpu_baseline": cpu,
        "latency_b1": lat,
        "cam_shard": shard_leg,
        "p1080": p1080,
        "local_ba": lba,
        "pose_inertial": pose,
        "pose_inertial_last_frame": pose_lf,
        **aux,
        "triangulation": tri,
    }
    print(json.dumps(out))
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
