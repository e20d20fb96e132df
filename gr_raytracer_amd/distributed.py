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


def _padded_send(records, frame_rows: int, cols: int, band_rows: int, rank: int, world: int, device):
    """This rank's records, zero-padded to the largest shard (equal-sized collective
    buffers), on the collective's device."""
    import torch

    max_rows = shard_row_count(frame_rows, band_rows, 0, world)  # shard 0 owns the most bands
    n_local = shard_row_count(frame_rows, band_rows, rank, world) * cols
    width = records.shape[1]
    assert records.shape == (n_local, width), (records.shape, n_local)
    if n_local == max_rows * cols and records.device == device:
        return records.contiguous()
    send = torch.zeros((max_rows * cols, width), dtype=torch.uint8, device=device)
    send[:n_local] = records
    return send


def _assemble(bufs, frame_rows: int, cols: int, band_rows: int, world: int, device):
    """De-interleave every shard's local rows into frame order."""
    import torch

    width = bufs[0].shape[1]
    frame = torch.empty((frame_rows, cols, width), dtype=torch.uint8, device=device)
    for s in range(world):
        rows = shard_frame_rows(frame_rows, band_rows, s, world)
        if rows.size == 0:
            continue
        idx = torch.as_tensor(rows, device=device)
        frame.index_copy_(0, idx, bufs[s][: rows.size * cols].view(rows.size, cols, width))
    return frame.view(frame_rows * cols, width)


def _collective_device(records, group=None):
    """gloo moves host tensors only: device records are staged through the host when the
    group's backend is gloo (multi-process tests on one GPU); RCCL works in place."""
    import torch
    import torch.distributed as dist

    if records.device.type != "cpu" and dist.get_backend(group) == "gloo":
        return torch.device("cpu")
    return records.device


def gather_frame(records, frame_rows: int, cols: int, band_rows: int, rank: int, world: int, dst: int = 0,
                 group=None):
    """Gather every rank's local pixel records to `dst` and put them in frame order.

    records: (local_rows * cols, B) uint8 on this rank's device (CPU for gloo), B = 18
    for pixel records, 3 for tone-mapped sRGB.
    Returns the (frame_rows * cols, B) frame on `dst` (on the records' device), None elsewhere."""
    import torch
    import torch.distributed as dist

    cdev = _collective_device(records, group)
    send = _padded_send(records, frame_rows, cols, band_rows, rank, world, cdev)
    bufs = [torch.empty_like(send) for _ in range(world)] if rank == dst else None
    dist.gather(send, gather_list=bufs, dst=dst, group=group)
    if rank != dst:
        return None
    return _assemble(bufs, frame_rows, cols, band_rows, world, cdev).to(records.device)


def allgather_frame(records, frame_rows: int, cols: int, band_rows: int, rank: int, world: int, group=None):
    """gather_frame for every rank: the (frame_rows * cols, B) frame in frame order on
    all ranks (the adaptive pass's 1-spp neighbourhood)."""
    import torch
    import torch.distributed as dist

    cdev = _collective_device(records, group)
    send = _padded_send(records, frame_rows, cols, band_rows, rank, world, cdev)
    bufs = [torch.empty_like(send) for _ in range(world)]
    dist.all_gather(bufs, send, group=group)
    return _assemble(bufs, frame_rows, cols, band_rows, world, cdev).to(records.device)


def reduce_channel_maxima(max3, group=None):
    """GlobalLinear tone mapping scales by the maximum over the WHOLE frame
    (color.rs:238-258): the per-rank maxima (3 f64, folded from 0) are allreduced with
    MAX, in place.  This is the output stage's one real exchange step."""
    import torch.distributed as dist

    if _collective_device(max3, group) != max3.device:
        host = max3.cpu()
        dist.all_reduce(host, op=dist.ReduceOp.MAX, group=group)
        max3.copy_(host)
        return max3
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


def pack_luminance_records(xyza64, cls):
    """(n,4) f64 XYZA + (n,) u8 class -> (n, 17) u8: Y and alpha (f64) and the class, what
    the selection stencil and the luminance floor read (should_supersample_pair,
    raytracer.rs:91-108; resolve_minimum_luminance, :118-129)."""
    import torch

    n = xyza64.shape[0]
    ya = torch.stack([xyza64[:, 1], xyza64[:, 3]], dim=1).contiguous()
    return torch.cat([ya.view(torch.uint8).view(n, 16), cls.view(n, 1)], dim=1)


def unpack_luminance_records(rec):
    import torch

    n = rec.shape[0]
    return rec[:, :16].contiguous().view(torch.float64).view(n, 2), rec[:, 16].contiguous()


def pack_section_records(xyza64, cls, status):
    """(n,4) f64 XYZA + class + status -> (n, 34) u8 (the supersampled frame's records)."""
    import torch

    n = xyza64.shape[0]
    return torch.cat([xyza64.contiguous().view(torch.uint8).view(n, 32), cls.view(n, 1), status.view(n, 1)], dim=1)


def unpack_section_records(rec):
    import torch

    n = rec.shape[0]
    return rec[:, :32].contiguous().view(torch.float64).view(n, 4), rec[:, 32].contiguous(), rec[:, 33].contiguous()


def render_frame_adaptive(scene, rank: int, world: int, cfg=None, band_rows: int = 16, device: int = 0,
                          stream=None, dst: int = 0, group=None, stats=None, sampling_mask_xyza=None,
                          tone_mapping=None, exposure: float = 1.0, failures=None, report=None):
    """render_section_to_cie_buffer (raytracer.rs:177-318) for a whole frame across
    `world` GPUs, with the reference's adaptive supersampling:

    1. each rank traces its row bands at 1 spp (f64 XYZA kept on the device);
    2. ONE allgather of every pixel's (Y, alpha, class), 17 B per pixel: the selection
       stencil reads 8 neighbours, which may sit in another rank's bands, and the
       luminance floor is the 99th percentile of the whole frame;
    3. every rank computes the same exact floor on its GPU (grt_adaptive_floor_device),
       which stays in device memory;
    4. each rank selects and supersamples its own pixels (grt_supersample_shard_device:
       selection, compaction, chunked sub-ray traces, all sized on the device);
    5. ONE gather to `dst`: f64 XYZA + class + status (34 B per pixel), or, with
       `tone_mapping` (0 Reinhard, 1 GlobalLinear), the per-rank tone-mapped sRGB8 rows
       (3 B per pixel; GlobalLinear allreduces the channel maxima first).

    failures: optional _lib.SubsampleFailures filled with this rank's failed sub-samples
    (frame pixel indices; the reference logs them, raytracer.rs:357-362).  report:
    optional dict that receives this rank's 1-spp "status", "stop" and "steps" (device
    tensors, local rows) and the local rows' "frame_rows" (the errors the reference logs
    at raytracer.rs:232-239, the NaN / no-terminal-event rays of scene.rs:178-202).
    cfg: grt_adaptive_config (default: the scene's own).  `enabled` false and no mask:
    plain 1-spp frame (render_section_to_cie_buffer_raw).  Returns on dst
    (xyza64 (n,4) f64, class u8, status u8, n_supersampled over all ranks) or, with
    tone_mapping, (rgb (n,3) u8, n_supersampled); None elsewhere."""
    import ctypes as C

    import torch
    import torch.distributed as dist

    from . import _lib as L

    if cfg is None:
        cfg = scene.adaptive
    dev = torch.device("cuda", device)
    if stream is None:
        stream = torch.cuda.current_stream(dev)
    rows, cols = scene.rows, scene.cols
    n_local = shard_row_count(rows, band_rows, rank, world) * cols
    xyza = torch.empty((n_local, 4), dtype=torch.float32, device=dev)
    xyza64 = torch.empty((n_local, 4), dtype=torch.float64, device=dev)
    cls = torch.empty(n_local, dtype=torch.uint8, device=dev)
    status = torch.empty(n_local, dtype=torch.uint8, device=dev)
    if stats is None:
        stats = torch.zeros(4, dtype=torch.int64, device=dev)
    sh = L.RowShard(band_rows, rank, world)
    lib = L.lib()
    steps = stop = None
    if report is not None:  # what color_of_ray's NaN / no-terminal-event lines need (scene.rs:178-202)
        steps = torch.empty(n_local, dtype=torch.int32, device=dev)
        stop = torch.empty(n_local, dtype=torch.uint8, device=dev)
    L.check(lib.grt_render_shard_async(scene._s, device, stream.cuda_stream, C.byref(sh), xyza.data_ptr(),
                                       cls.data_ptr(), status.data_ptr(), xyza64.data_ptr(),
                                       steps.data_ptr() if steps is not None else None,
                                       stop.data_ptr() if stop is not None else None,
                                       stats.data_ptr()), "grt_render_shard_async")
    if report is not None:
        report["status"] = status
        report["stop"] = stop
        report["steps"] = steps
        report["frame_rows"] = shard_frame_rows(rows, band_rows, rank, world)
    n_sel = torch.zeros(1, dtype=torch.int64)
    with torch.cuda.stream(stream):
        if cfg.enabled or sampling_mask_xyza is not None:
            frame = allgather_frame(pack_luminance_records(xyza64, cls), rows, cols, band_rows, rank, world, group)
            frame_ya, frame_cls = unpack_luminance_records(frame)
            # the frame's exact 99th-percentile floor, selected on this GPU and left there
            # (a configured minimum_luminance is a constant)
            d_floor = None
            if not cfg.has_minimum_luminance:
                d_floor = torch.empty(1, dtype=torch.float64, device=dev)
                L.check(lib.grt_adaptive_floor_device(scene._s, device, stream.cuda_stream, frame_ya.data_ptr(), 2,
                                                      frame_ya.shape[0], d_floor.data_ptr()),
                        "grt_adaptive_floor_device")
            mask = None
            if sampling_mask_xyza is not None:
                mask = (C.c_double * 4)(*[float(v) for v in sampling_mask_xyza])
            count = torch.zeros(1, dtype=torch.int64, device=dev)
            L.check(lib.grt_supersample_shard_device(scene._s, device, stream.cuda_stream, C.byref(sh), C.byref(cfg),
                                                     float(cfg.minimum_luminance),
                                                     d_floor.data_ptr() if d_floor is not None else None,
                                                     frame_ya.data_ptr(), frame_cls.data_ptr(), mask,
                                                     xyza64.data_ptr(), count.data_ptr(), stats.data_ptr(), failures),
                    "grt_supersample_shard_device")
            total = count.to(_collective_device(count, group))
            dist.all_reduce(total, op=dist.ReduceOp.SUM, group=group)
            n_sel[0] = int(total[0])
        if tone_mapping is not None:
            rgb = torch.empty((n_local, 3), dtype=torch.uint8, device=dev)
            max3 = torch.zeros(3, dtype=torch.float64, device=dev)
            if tone_mapping == 1:
                L.check(lib.grt_linear_max_async(device, stream.cuda_stream, xyza64.data_ptr(), n_local, exposure,
                                                 max3.data_ptr()), "grt_linear_max_async")
                reduce_channel_maxima(max3, group)
            L.check(lib.grt_tonemap_async(device, stream.cuda_stream, xyza64.data_ptr(), n_local, tone_mapping,
                                          exposure, max3.data_ptr(), rgb.data_ptr()), "grt_tonemap_async")
            out = gather_frame(rgb, rows, cols, band_rows, rank, world, dst, group)
            return None if out is None else (out, int(n_sel[0]))
        out = gather_frame(pack_section_records(xyza64, cls, status), rows, cols, band_rows, rank, world, dst, group)
    if out is None:
        return None
    x64, c, st = unpack_section_records(out)
    return x64, c, st, int(n_sel[0])
