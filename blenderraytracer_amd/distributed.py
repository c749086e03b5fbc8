"""Multi-GPU rendering: one process per GPU, torch.distributed over RCCL (backend "nccl").

Every sample is independent and keyed by (seed, pixel, sample), so rank r traces
samples [r*S/N, (r+1)*S/N) of EVERY pixel (a sample split balances better than row
bands, where sky rows are cheap) into a float64 per-pixel sum buffer in its own HBM.  The only
exchange is one reduce(SUM) of that buffer to rank 0 over xGMI (W*H*3 doubles: 50 MB at 1080p),
after which rank 0 runs the epilogue.  The result equals the 1-GPU render up to the order in which
the N partial sums are added.
"""
import ctypes as C

import torch
import torch.distributed as dist

from . import capi


def sample_range(rank, world, samples):
    """Contiguous, balanced split of [0, samples) (sizes differ by at most one)."""
    return (rank * samples) // world, ((rank + 1) * samples) // world


def _reducing(world):
    return world > 1 or (dist.is_available() and dist.is_initialized())


def reduce_sums(buf, world, group=None):
    """Sum the per-pixel radiance sums of all ranks into rank 0's buffer (RCCL reduce on GPUs).  Runs
    whenever a process group is up, also at world size 1 (bench.py under torch.distributed.run with one
    rank: the RCCL path itself, an identity there)."""
    if _reducing(world):
        if buf.is_cuda and dist.get_backend(group) == "gloo":
            # gloo reduces host tensors only: the N-ranks-on-fewer-GPUs rehearsal (bench.py
            # --dist-backend gloo) stages the sums through host memory
            host = buf.cpu()
            dist.reduce(host, dst=0, op=dist.ReduceOp.SUM, group=group)
            buf.copy_(host)
        else:
            dist.reduce(buf, dst=0, op=dist.ReduceOp.SUM, group=group)
    return buf


def reduce_band_async(view, world, group=None):
    """reduce_sums for one band of rows (rt_trace_device_bands' band_ready): RCCL returns a work handle
    (the reduce runs on RCCL's stream after the current stream's work so far — the band's own sums —
    while the later bands still trace); gloo stages through host memory at once (None)."""
    if not _reducing(world):
        return None
    if view.is_cuda and dist.get_backend(group) == "gloo":
        reduce_sums(view, world, group)
        return None
    return dist.reduce(view, dst=0, op=dist.ReduceOp.SUM, group=group, async_op=True)


class ShardedRender:
    """One rank's share of a frame: trace own sample range -> reduce -> (rank 0) epilogue on device.

    bands > 0 (HIP path): the trace delivers the frame in that many horizontal bands
    (rt_trace_device_bands) and each band's rows are reduced across the ranks as soon as they are final,
    while the later bands trace; the sums are bit-identical to the unbanded step.
    trace_fn(buf, settings) may replace the HIP trace (tests run the sharding + gloo reduce on CPU
    with the kernel's CPU build); the product path always uses rt_trace_device."""

    def __init__(self, tracer, rank=0, world=1, device=None, group=None, trace_fn=None, bands=0):
        self.tracer = tracer
        self.rank, self.world, self.group = rank, world, group
        self.bands = bands if trace_fn is None else 0
        self.device = device if device is not None else torch.device("cuda", 0)
        self.stats = capi.Stats()
        s = tracer.settings()
        self.full_settings = s
        self.cw = s.crop_w or s.width
        self.n = (s.crop_w or s.width) * (s.crop_h or s.height)
        self.samples = s.samples
        self.range = sample_range(rank, world, self.samples)
        self.settings = tracer.settings(sample_range=self.range) if self.range[1] > self.range[0] else None
        self.sum = torch.zeros(self.n * 3, dtype=torch.float64, device=self.device)
        self._trace = trace_fn
        self.rgba8 = self.post = None
        if trace_fn is None:
            self.lib = capi.load_library()
            self.scene = tracer.scene_handle()
            if rank == 0:
                self.rgba8 = torch.zeros(self.n * 4, dtype=torch.uint8, device=self.device)
                self.post = torch.zeros(self.n * 4, dtype=torch.float32, device=self.device)

    def _hip_trace(self, stats):
        stream = torch.cuda.current_stream(self.device)
        capi.check(self.lib.rt_trace_device(self.scene, C.byref(self.settings), C.c_void_p(self.sum.data_ptr()),
                                            C.c_void_p(stream.cuda_stream), 1 if stats else 0,
                                            C.byref(self.stats) if stats else None))

    def _hip_trace_bands(self, stats):
        """rt_trace_device_bands: every band's reduce issued from its band_ready callback; returns the
        pending RCCL works"""
        stream = torch.cuda.current_stream(self.device)
        works = []
        cw = self.cw

        def ready(band, row0, rows, user):
            w = reduce_band_async(self.sum[3 * row0 * cw:3 * (row0 + rows) * cw], self.world, self.group)
            if w is not None:
                works.append(w)
            return 0
        cb = capi.BAND_FN(ready)
        capi.check(self.lib.rt_trace_device_bands(self.scene, C.byref(self.settings), C.c_void_p(self.sum.data_ptr()),
                                                  C.c_void_p(stream.cuda_stream), self.bands, cb, None,
                                                  C.byref(self.stats) if stats else None))
        return works

    def step(self, stats=True, events=None):
        """Render the frame once.  With stats=True (HIP path) the trace kernel's HIP-event time and
        segment count land in self.stats (the call then synchronizes the stream after the trace).
        events: (start, end) torch.cuda.Events recorded around the trace on the stream it runs on (the
        timed steps of bench.py: no host synchronization inside a step)."""
        self.sum.zero_()
        works = None
        if self.settings is not None:
            if self._trace is not None:
                self._trace(self.sum, self.settings)
            else:
                if events:
                    events[0].record()
                if self.bands:
                    works = self._hip_trace_bands(stats)
                else:
                    self._hip_trace(stats)
                if events:
                    events[1].record()
        if works is not None:               # banded: the bands' reduces are under way (or done: gloo)
            for w in works:
                w.wait()
        else:
            reduce_sums(self.sum, self.world, self.group)
        if self.rank == 0 and self._trace is None:
            stream = torch.cuda.current_stream(self.device)
            capi.check(self.lib.rt_finalize_device(self.scene, C.byref(self.full_settings), C.c_void_p(self.sum.data_ptr()), None,
                                                   C.c_void_p(self.post.data_ptr()), C.c_void_p(self.rgba8.data_ptr()),
                                                   C.c_void_p(stream.cuda_stream)))


class InProcessRender:
    """The drop-in's own multi-GPU path (rt_settings.devices, what installGpuRender(rt, {devices}) runs
    from Node): ONE process, whole sample batches dealt round-robin to the devices (batch k on
    devices[k % N], traced by a replica of the scene), each batch's chunk partials copied peer-to-peer
    over xGMI to the scene's device and added there in batch order, then the epilogue.  A step is one
    rt_render call delivering the frame's RGBA8 bytes to the host (the reference's imageData).
    progress_steps: the Node drop-in's progressive form (gpu-ray-tracer.mjs DEFAULT_PROGRESS_STEPS = 16):
    about `steps` batches (batch_samples = -steps: multiples of the pool's chunk), the running frame into a preview buffer and a progress callback
    after every batch; 0: batch_samples = 0 (the library then makes one batch per device)."""

    def __init__(self, tracer, devices, progress_steps=0):
        import numpy as np
        self.tracer = tracer
        self.devices = list(devices)
        self.lib = capi.load_library()
        self.scene = tracer.scene_handle()
        spp = tracer.settings().samples
        self.batch = -progress_steps if progress_steps else 0   # about `steps` batches aligned to the pool's chunks
        self.settings = tracer.settings(devices=self.devices if len(self.devices) > 1 else None,
                                        batch_samples=self.batch)
        s = self.settings
        self.n = (s.crop_w or s.width) * (s.crop_h or s.height)
        self.rgba8 = np.zeros(self.n * 4, dtype=np.uint8)
        self.out = capi.Output()
        self.out.rgba8 = self.rgba8.ctypes.data_as(C.POINTER(C.c_uint8))
        self.progress_calls = 0
        if progress_steps:
            self.preview = np.zeros(self.n * 4, dtype=np.uint8)
            self.out.preview_rgba8 = self.preview.ctypes.data_as(C.POINTER(C.c_uint8))

            def on_progress(fraction, user):
                self.progress_calls += 1
                return 0
            self._progress = capi.PROGRESS_FN(on_progress)
        else:
            self._progress = C.cast(None, capi.PROGRESS_FN)
        self.stats = capi.Stats()
        self.range = (0, s.samples)

    def step(self, stats=True, events=None):
        capi.check(self.lib.rt_render(self.scene, C.byref(self.settings), C.byref(self.out), self._progress, None,
                                      C.byref(self.stats)))
