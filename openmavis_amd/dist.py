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
    t = torch.tensor([dt], dtype=torch.float64, device=device)
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


class LbaAllReduce:
    """The omv_allreduce_fn of a landmark-sharded LocalInertialBA over torch.distributed.

    mode "device" (backend nccl = RCCL): the handle's device buffer is staged through a torch tensor
    on the handle's own HIP stream (torch.cuda.ExternalStream), so the copy, the ring all-reduce over
    xGMI and the copy back stay ordered with the LM kernels and the host never waits.
    mode "host" (backend gloo): the stream is drained and the buffer goes through host memory — the
    CPU-collective rehearsal of the same exchange (tests, a GPU box with one card).
    """

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

    def _staging(self, n, device):
        t = self._torch
        if self._buf is None or self._buf.numel() < n or self._buf.device != t.device(device):
            self._buf = t.empty(max(n, 1), dtype=t.float64, device=device)
        return self._buf[:n]

    def __call__(self, ptr, count, stream):
        import torch.distributed as dist
        t = self._torch
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
        with t.cuda.stream(ext):
            buf = self._staging(count, self.device or t.cuda.current_device())
            if self._hip.hipMemcpyAsync(buf.data_ptr(), ptr, nbytes, 3, stream) != 0:   # D2D
                raise RuntimeError("hipMemcpyAsync D2D")
            dist.all_reduce(buf, group=self.group)   # ordered after the copy (current stream = ext)
            if self._hip.hipMemcpyAsync(ptr, buf.data_ptr(), nbytes, 3, stream) != 0:
                raise RuntimeError("hipMemcpyAsync D2D")
