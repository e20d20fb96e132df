"""Multi-GPU frame rendering: cyclic row-band shards + one gather.

One process per GPU (torch.distributed; backend "nccl" is RCCL on ROCm).  Pixels are
independent (raytracer.rs:218 renders them with a rayon par_iter), so the integration
needs no exchange at all: rank s traces the row bands b with b % world == s
(grt_render_shard_async, include/grt_api.h), then every rank's pixel records are
gathered to rank 0 in ONE collective and de-interleaved into frame order there.

A pixel record is 18 bytes: f32 XYZA (16 B) + class (1 B) + status (1 B), the
framebuffer the reference fills in render_section_to_cie_buffer_raw
(raytracer.rs:195-244; colour, RayClass, and the error that the reference logs).
C4 (4096^2) is 302 MB in total, ~38 MB per peer over its own xGMI link at 8 GPUs.

The gather/assembly logic is backend-agnostic (CPU tensors over gloo in the tests).
"""
from __future__ import annotations

import numpy as np

RECORD_BYTES = 18


def shard_row_count(frame_rows: int, band_rows: int, shard: int, n_shards: int) -> int:
    """Rows of shard `shard` (mirror of grt_shard_row_count, checked against it in tests)."""
    if n_shards <= 1:
        return frame_rows
    bands = -(-frame_rows // band_rows)
    mine = max(0, -(-(bands - shard) // n_shards))
    if mine == 0:
        return 0
    last_band = shard + (mine - 1) * n_shards
    return (mine - 1) * band_rows + min(band_rows, frame_rows - last_band * band_rows)


def shard_frame_rows(frame_rows: int, band_rows: int, shard: int, n_shards: int) -> np.ndarray:
    """Frame row of each local row of a shard, in local order."""
    if n_shards <= 1:
        return np.arange(frame_rows, dtype=np.int64)
    local = np.arange(shard_row_count(frame_rows, band_rows, shard, n_shards), dtype=np.int64)
    return ((local // band_rows) * n_shards + shard) * band_rows + local % band_rows


def pack_records(xyza, cls, status):
    """(n,4) f32 + (n,) u8 + (n,) u8 torch tensors -> (n, 18) u8 records."""
    import torch

    n = xyza.shape[0]
    return torch.cat([xyza.contiguous().view(torch.uint8).view(n, 16), cls.view(n, 1), status.view(n, 1)], dim=1)


def unpack_records(rec):
    import torch

    n = rec.shape[0]
    xyza = rec[:, :16].contiguous().view(torch.float32).view(n, 4)
    return xyza, rec[:, 16].contiguous(), rec[:, 17].contiguous()


def gather_frame(records, frame_rows: int, cols: int, band_rows: int, rank: int, world: int, dst: int = 0,
                 group=None):
    """Gather every rank's local pixel records to `dst` and put them in frame order.

    records: (local_rows * cols, B) uint8 on this rank's device (CPU for gloo), B = 18
    for pixel records, 3 for tone-mapped sRGB.
    Returns the (frame_rows * cols, B) frame on `dst`, None elsewhere."""
    import torch
    import torch.distributed as dist

    max_rows = shard_row_count(frame_rows, band_rows, 0, world)  # shard 0 owns the most bands
    n_local = shard_row_count(frame_rows, band_rows, rank, world) * cols
    width = records.shape[1]
    assert records.shape == (n_local, width), (records.shape, n_local)
    send = records
    if n_local != max_rows * cols:  # equal-sized buffers for the collective
        send = torch.zeros((max_rows * cols, width), dtype=torch.uint8, device=records.device)
        send[:n_local] = records
    bufs = [torch.empty_like(send) for _ in range(world)] if rank == dst else None
    dist.gather(send, gather_list=bufs, dst=dst, group=group)
    if rank != dst:
        return None
    frame = torch.empty((frame_rows, cols, width), dtype=torch.uint8, device=records.device)
    for s in range(world):
        rows = shard_frame_rows(frame_rows, band_rows, s, world)
        if rows.size == 0:
            continue
        idx = torch.as_tensor(rows, device=records.device)
        frame.index_copy_(0, idx, bufs[s][: rows.size * cols].view(rows.size, cols, width))
    return frame.view(frame_rows * cols, width)


def reduce_channel_maxima(max3, group=None):
    """GlobalLinear tone mapping scales by the maximum over the WHOLE frame
    (color.rs:238-258): the per-rank maxima (3 f64, folded from 0) are allreduced with
    MAX, in place.  This is the output stage's one real exchange step."""
    import torch.distributed as dist

    dist.all_reduce(max3, op=dist.ReduceOp.MAX, group=group)
    return max3


def render_frame(scene, rank: int, world: int, band_rows: int = 16, device: int = 0, stream=None,
                 dst: int = 0, group=None, stats=None):
    """Render `scene` across `world` ranks (this one = `rank`, GPU `device`) and gather
    the frame to `dst`.  Returns (xyza f32 (n,4), class u8, status u8) on dst, else None.

    The trace is enqueued on `stream` (default: torch's current stream of `device`);
    `stats` (4 x int64 device tensor, optional) accumulates the kernel counters."""
    import ctypes as C

    import torch

    from . import _lib as L

    dev = torch.device("cuda", device)
    if stream is None:
        stream = torch.cuda.current_stream(dev)
    rows, cols = scene.rows, scene.cols
    n_local = shard_row_count(rows, band_rows, rank, world) * cols
    xyza = torch.empty((n_local, 4), dtype=torch.float32, device=dev)
    cls = torch.empty(n_local, dtype=torch.uint8, device=dev)
    status = torch.empty(n_local, dtype=torch.uint8, device=dev)
    if stats is None:
        stats = torch.zeros(4, dtype=torch.int64, device=dev)
    sh = L.RowShard(band_rows, rank, world)
    L.check(L.lib().grt_render_shard_async(scene._s, device, stream.cuda_stream, C.byref(sh), xyza.data_ptr(),
                                           cls.data_ptr(), status.data_ptr(), None, None, None, stats.data_ptr()),
            "grt_render_shard_async")
    with torch.cuda.stream(stream):
        frame = gather_frame(pack_records(xyza, cls, status), rows, cols, band_rows, rank, world, dst, group)
    if frame is None:
        return None
    return unpack_records(frame)


def render_frame_srgb(scene, rank: int, world: int, tone_mapping: int = 0, exposure: float = 1.0,
                      band_rows: int = 16, device: int = 0, stream=None, dst: int = 0, group=None, stats=None):
    """render_section's non-HDR path (raytracer.rs:481-487) across `world` GPUs: each
    rank traces its row bands (f64 XYZA kept on the device), GlobalLinear allreduces
    the channel maxima, each rank tone-maps its own rows on the device, and only the
    3-byte sRGB pixels are gathered to `dst`.  Returns (rows*cols, 3) u8 on dst."""
    import ctypes as C

    import torch

    from . import _lib as L

    dev = torch.device("cuda", device)
    if stream is None:
        stream = torch.cuda.current_stream(dev)
    rows, cols = scene.rows, scene.cols
    n_local = shard_row_count(rows, band_rows, rank, world) * cols
    xyza = torch.empty((n_local, 4), dtype=torch.float32, device=dev)
    xyza64 = torch.empty((n_local, 4), dtype=torch.float64, device=dev)
    cls = torch.empty(n_local, dtype=torch.uint8, device=dev)
    status = torch.empty(n_local, dtype=torch.uint8, device=dev)
    rgb = torch.empty((n_local, 3), dtype=torch.uint8, device=dev)
    max3 = torch.zeros(3, dtype=torch.float64, device=dev)
    if stats is None:
        stats = torch.zeros(4, dtype=torch.int64, device=dev)
    sh = L.RowShard(band_rows, rank, world)
    lib = L.lib()
    L.check(lib.grt_render_shard_async(scene._s, device, stream.cuda_stream, C.byref(sh), xyza.data_ptr(),
                                       cls.data_ptr(), status.data_ptr(), xyza64.data_ptr(), None, None,
                                       stats.data_ptr()), "grt_render_shard_async")
    with torch.cuda.stream(stream):
        if tone_mapping == 1:
            L.check(lib.grt_linear_max_async(device, stream.cuda_stream, xyza64.data_ptr(), n_local, exposure,
                                             max3.data_ptr()), "grt_linear_max_async")
            reduce_channel_maxima(max3, group)
        L.check(lib.grt_tonemap_async(device, stream.cuda_stream, xyza64.data_ptr(), n_local, tone_mapping,
                                      exposure, max3.data_ptr(), rgb.data_ptr()), "grt_tonemap_async")
        return gather_frame(rgb, rows, cols, band_rows, rank, world, dst, group)
