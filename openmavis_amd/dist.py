"""Multi-GPU plumbing (torch.distributed; backend "nccl" is RCCL over xGMI on ROCm).

The extract+match path shards by frame with no data-path collective (bench.py: frame replicas).
The one exchange the north star names is the one-camera-per-GPU rig (BASELINE config 3): each rank
extracts its camera and the tracking rank needs every camera's keypoints + descriptors, i.e. an
all-gather of fixed-size per-camera slabs {count, kp_cap x 24 B keypoints, kp_cap x 32 B
descriptors}.  `allgather_camera_slabs` packs that slab into one int32 tensor so the
exchange is a single all_gather_into_tensor (one ring pass over xGMI; 67 KB/camera at 1200
features: latency-bound, not bandwidth-bound).
"""
import os


def init_from_env(backend="nccl"):
    import torch
    import torch.distributed as dist
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world <= 1:
        return 0, 1
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if backend == "nccl":
        torch.cuda.set_device(local)
        dist.init_process_group(backend, device_id=torch.device("cuda", local))
    else:
        dist.init_process_group(backend)
    return dist.get_rank(), dist.get_world_size()


def job_seconds(dt, device=None):
    """Max of a per-rank wall time over all ranks (the bench contract's whole-job time)."""
    import torch
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return dt
    t = torch.tensor([dt], dtype=torch.float64, device="cpu" if dist.get_backend() == "gloo" else device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def slab_words(kp_cap):
    return 1 + kp_cap * 6 + kp_cap * 8   # count | kps (6 x 32-bit) | desc (32 B = 8 words)


def allgather_camera_slabs(kps, desc, n_kp, group=None):
    """kps: int32 [kp_cap, 6] (omv_kp rows), desc: uint8 [kp_cap, 32], n_kp: int32 [1] of this rank's
    camera.  Returns (kps [world, kp_cap, 6], desc [world, kp_cap, 32], n_kp [world]) in rank order."""
    import torch
    import torch.distributed as dist
    kp_cap = kps.shape[0]
    world = dist.get_world_size(group)
    slab = torch.empty(slab_words(kp_cap), dtype=torch.int32, device=kps.device)
    slab[:1] = n_kp.reshape(1)
    slab[1:1 + kp_cap * 6] = kps.reshape(-1)
    slab[1 + kp_cap * 6:] = desc.reshape(-1).view(torch.int32)
    out = torch.empty(world * slab.numel(), dtype=torch.int32, device=kps.device)
    dist.all_gather_into_tensor(out, slab, group=group)
    out = out.view(world, -1)
    g_n = out[:, 0].clone()
    g_kps = out[:, 1:1 + kp_cap * 6].reshape(world, kp_cap, 6).clone()
    g_desc = out[:, 1 + kp_cap * 6:].contiguous().view(torch.uint8).reshape(world, kp_cap, 32).clone()
    return g_kps, g_desc, g_n


class CameraShard:
    """One camera per rank (BASELINE configs[2] / [3]; the reference's unit of parallelism is the per-camera
    extractor thread, src/Frame.cc:1841-1862): rank r extracts cameras r, r + world, ... of every frame and
    the tracking rank needs all of them, so the ranks exchange fixed-size slabs in ONE all_gather_into_tensor
    (RCCL ring over xGMI with mode "device"; staged through host memory with mode "host" for gloo).

    The send buffer is sectioned so the extractor writes straight into it (no packing copy):
        n_kp [k][F] | mono [k][F] | kps [k][F][kp_cap][6] (omv_kp rows) | desc [k][F][kp_cap][32 B]
    with k = ceil(n_cams / world) camera slots per rank (cam-major: a rank with fewer cameras extracts only its
    first len(cams) * F images).  `gather` scatters every rank's slab into a FrameBatch [F][n_cams] in camera
    order, on every rank: one indexed gather per field (count, monoIndex, keypoint rows, descriptor rows) over the
    received slabs, with the (rank, row) index of every (frame, camera) built once -- 4 launches whatever the camera
    and rank counts.  Ranks with no camera (configs[2]: 5 cameras on 8 GPUs) send an empty slab section."""

    def __init__(self, rank, world, n_cams, n_frames, kp_cap, device, mode="device", group=None):
        import torch
        self.rank, self.world, self.n_cams, self.F, self.cap = rank, world, n_cams, n_frames, kp_cap
        self.k = (n_cams + world - 1) // world
        self.cams = list(range(rank, n_cams, world))
        self.mode, self.group, self.device = mode, group, device
        k, F = self.k, n_frames
        self.off_mono = k * F
        self.off_kps = 2 * k * F
        self.off_desc = self.off_kps + k * F * kp_cap * 6
        self.words = self.off_desc + k * F * kp_cap * 8
        self.send = torch.zeros(self.words, dtype=torch.int32, device=device)
        self.recv = torch.empty(world * self.words, dtype=torch.int32, device=device)
        if mode == "host":
            self._send_h = torch.empty(self.words, dtype=torch.int32)
            self._recv_h = torch.empty(world * self.words, dtype=torch.int32)
        # gather index: output (frame f, camera c) <- rank c % world, slab row (c // world) * F + f
        src_r = torch.tensor([c % world for f in range(F) for c in range(n_cams)], dtype=torch.long)
        src_j = torch.tensor([(c // world) * F + f for f in range(F) for c in range(n_cams)], dtype=torch.long)
        self._src = (src_r.to(device), src_j.to(device))

    def camera_of(self, r, j):
        return r + j * self.world

    def outputs(self):
        """This rank's extractor outputs as views of the send slab, for its len(cams) * F images (cam-major)."""
        import torch
        n = len(self.cams) * self.F
        s, cap = self.send, self.cap
        return (s[self.off_kps:self.off_kps + n * cap * 6].view(n, cap, 6),
                s[self.off_desc:self.off_desc + n * cap * 8].view(torch.uint8).view(n, cap, 32),
                s[:n], s[self.off_mono:self.off_mono + n])

    def gather(self, fb, stream=None):
        """All-gather the slabs and scatter them into FrameBatch fb ([F][n_cams][kp_cap] tensors on this rank)."""
        import contextlib
        import torch
        import torch.distributed as dist
        on_gpu = torch.device(self.device).type == "cuda"
        ctx = torch.cuda.stream(stream if stream is not None else torch.cuda.current_stream(self.device)) \
            if on_gpu else contextlib.nullcontext()
        with ctx:
            if self.mode == "host" and on_gpu:
                self._send_h.copy_(self.send)
                dist.all_gather_into_tensor(self._recv_h, self._send_h, group=self.group)
                self.recv.copy_(self._recv_h)
            else:
                dist.all_gather_into_tensor(self.recv, self.send, group=self.group)
            F, cap, k, C = self.F, self.cap, self.k, self.n_cams
            rv = self.recv.view(self.world, self.words)
            r, j = self._src
            # strided views [world][k * F][row] of each section of the received slabs (no copy), one gather each
            n_v = rv[:, :k * F]
            m_v = rv[:, self.off_mono:self.off_mono + k * F]
            k_v = rv[:, self.off_kps:self.off_desc].view(self.world, k * F, cap * 6)
            d_v = rv[:, self.off_desc:].view(self.world, k * F, cap * 8)
            fb.n_kp.view(F * C).copy_(n_v[r, j])
            fb.mono.view(F * C).copy_(m_v[r, j])
            fb.kps.view(F * C, cap * 6).copy_(k_v[r, j])
            fb.desc.view(F * C, cap * 32).copy_(d_v[r, j].view(torch.uint8))


class LbaAllReduce:
    """The omv_allreduce_fn of a landmark-sharded LocalInertialBA over torch.distributed.

    mode "device" (backend nccl = RCCL): the handle's device buffer itself is all-reduced IN PLACE on the
    handle's own HIP stream (torch.cuda.ExternalStream; the buffer is wrapped as a tensor through the CUDA array
    interface, no copy), so the ring all-reduce over xGMI stays ordered with the LM kernels and the host never
    waits.  mode "host" (backend gloo): the stream is drained and the buffer goes through host memory — the
    CPU-collective rehearsal of the same exchange (tests, a GPU box with one card).
    `calls` counts the collectives issued.
    """

    class _Dev:   # a device buffer seen through __cuda_array_interface__ (float64, contiguous)
        def __init__(self, ptr, count):
            self.__cuda_array_interface__ = {"shape": (int(count),), "typestr": "<f8", "data": (int(ptr), False),
                                             "version": 2}

    def __init__(self, mode="device", group=None, device=None):
        import ctypes
        import torch
        if mode not in ("device", "host"):
            raise ValueError(mode)
        self.mode, self.group, self.device = mode, group, device
        self._hip = ctypes.CDLL("libamdhip64.so")
        self._hip.hipMemcpyAsync.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int,
                                             ctypes.c_void_p]
        self._hip.hipStreamSynchronize.argtypes = [ctypes.c_void_p]
        self._buf = None
        self._torch = torch
        self.calls = 0

    def _staging(self, n, device):
        t = self._torch
        if self._buf is None or self._buf.numel() < n or self._buf.device != t.device(device):
            self._buf = t.empty(max(n, 1), dtype=t.float64, device=device)
        return self._buf[:n]

    def __call__(self, ptr, count, stream):
        import torch.distributed as dist
        t = self._torch
        self.calls += 1
        nbytes = int(count) * 8
        if self.mode == "host":
            buf = self._staging(count, "cpu")
            if self._hip.hipStreamSynchronize(stream) != 0:
                raise RuntimeError("hipStreamSynchronize")
            if self._hip.hipMemcpyAsync(buf.data_ptr(), ptr, nbytes, 2, stream) != 0:   # D2H
                raise RuntimeError("hipMemcpyAsync D2H")
            self._hip.hipStreamSynchronize(stream)
            dist.all_reduce(buf, group=self.group)
            if self._hip.hipMemcpyAsync(ptr, buf.data_ptr(), nbytes, 1, stream) != 0:   # H2D
                raise RuntimeError("hipMemcpyAsync H2D")
            self._hip.hipStreamSynchronize(stream)   # buf is reused by the next call
            return
        ext = t.cuda.ExternalStream(stream, device=self.device)
        with t.cuda.device(self.device if self.device is not None else t.cuda.current_device()), t.cuda.stream(ext):
            view = t.as_tensor(self._Dev(ptr, count), device="cuda")
            dist.all_reduce(view, group=self.group)   # in place on the handle's buffer, ordered on its stream
