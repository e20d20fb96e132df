"""One frame over several GPUs of one process behind the C ABI (grt_render_frame_multi,
include/grt_api.h; csrc/device/multi.hip).

CPU: the frame-order assembly of the gathered blocks (the de-interleave kernel's per-pixel
source function, run on the host through a test hook) against
distributed.shard_frame_rows for 1..8 shards and ragged frames; the block layout; the
argument checks.  GPU (marker `gpu`): with one device (a one-rank RCCL communicator: the
same allgather, grouped send / receive and de-interleave as at N = 8) the frame equals the
single-device entry points bit for bit: C2 at 1 spp against grt_render_pixels, a reduced
C4 frame, and C5's adaptive frame against grt_render_section_ex; grt_render_shard from four
host threads at once (with the tuning knobs flipped by a fifth) gives the shards of one
thread; `grt --gpus 1` writes the PNG `grt` writes.
"""
import ctypes as C
import hashlib
import os
import subprocess
import threading

import numpy as np
import pytest

from conftest import RESOURCES, ROOT, SCENES, c2_opts, host_scene

FIELD_BYTES = [32, 16, 4, 1, 1, 1]  # RF_XYZA64, RF_XYZA32, RF_STEPS, RF_CLASS, RF_STATUS, RF_STOP


def _hooks():
    from gr_raytracer_amd import _lib as L

    lib = L.lib()
    d = lib.grt_debug_deinterleave_host
    d.restype = C.c_int
    d.argtypes = [C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32, C.c_void_p, C.c_void_p]
    b = lib.grt_debug_gather_block_bytes
    b.restype = C.c_uint64
    b.argtypes = [C.c_uint32, C.c_uint64, C.c_void_p]
    return d, b


def _encode(p, nbytes, f):
    """Distinct bytes per (pixel, field): the pixel index and field number, little endian."""
    v = (p.astype(np.uint64) * 8 + f).view(np.uint8).reshape(-1, 8)
    reps = -(-nbytes // 8)
    return np.tile(v, (1, reps))[:, :nbytes]


@pytest.mark.parametrize("mask", [0b011010, 0b111111, 0b011001])
def test_deinterleave_matches_shard_frame_rows(grt, mask):
    from gr_raytracer_amd.distributed import shard_frame_rows

    deint, block_bytes = _hooks()
    for rows, cols in ((1, 5), (7, 3), (40, 36), (136, 10), (257, 9)):
        for n in range(1, 9):
            for band in (1, 8, 16):
                frame = rows * cols
                blocks = []
                for s in range(n):
                    fr = shard_frame_rows(rows, band, s, n)
                    local = (fr[:, None] * cols + np.arange(cols)[None, :]).reshape(-1)  # frame pixel of each local one
                    offs = np.zeros(6, np.uint64)
                    size = block_bytes(mask, len(local), offs.ctypes.data)
                    blk = np.zeros(size, np.uint8)
                    for f in range(6):
                        if mask & (1 << f):
                            o = int(offs[f])
                            assert o % 256 == 0
                            e = FIELD_BYTES[f]
                            blk[o:o + len(local) * e] = _encode(local, e, f).reshape(-1)
                    blocks.append(blk)
                gathered = np.concatenate(blocks)
                dst = [np.zeros(frame * FIELD_BYTES[f], np.uint8) if mask & (1 << f) else None for f in range(6)]
                ptrs = (C.c_void_p * 6)(*[d.ctypes.data if d is not None else None for d in dst])
                assert deint(rows, cols, band, n, mask, gathered.ctypes.data, ptrs) == 0
                for f in range(6):
                    if dst[f] is not None:
                        want = _encode(np.arange(frame), FIELD_BYTES[f], f).reshape(-1)
                        assert np.array_equal(dst[f], want), (rows, cols, n, band, f)


def test_block_layout(grt):
    _, block_bytes = _hooks()
    offs = np.zeros(6, np.uint64)
    # 18-B record: f32 XYZA, class, status
    size = block_bytes(0b011010, 1000, offs.ctypes.data)
    assert offs[1] == 0 and offs[3] == 16128 and offs[4] == 16128 + 1024 and size == 16128 + 1024 + 1024  # 256-B aligned
    assert offs[0] == np.uint64(2**64 - 1) and offs[2] == np.uint64(2**64 - 1)
    assert block_bytes(0b111111, 0, offs.ctypes.data) == 0


def test_multi_argument_checks(grt):
    from gr_raytracer_amd import _lib as L

    hs = host_scene(grt, "schwarzschild.toml", c2_opts(grt, width=16, height=16))
    scene = grt.Scene(hs.desc_ptr(), keepalive=hs)
    lib = L.lib()
    xyza = np.zeros((256, 4), np.float32)
    out = L.FrameOut(L.ptr(xyza, C.c_float), None, None, None, None, None)

    def call(devs, band=16, cfg=None, o=out):
        arr = (C.c_int * max(1, len(devs)))(*devs)
        return lib.grt_render_frame_multi(scene._s, len(devs), arr, band, cfg, None, C.byref(o) if o else None,
                                          None, None, None, None)

    assert call([]) == -22
    assert call(list(range(17))) == -22
    assert call([0, 0]) == -22  # one RCCL rank per GPU
    assert call([0], band=0) == -22
    assert call([0], o=None) == -22
    cfg = L.AdaptiveConfig()
    lib.grt_default_adaptive_config(C.byref(cfg))
    cfg.enabled = 1
    if grt.device_count() > 0:  # supersampling needs f64 out and no f32
        assert call([0], cfg=cfg) == -22
    assert lib.grt_last_error()


# ------------------------------------------------------------------------------- GPU ---
def _same(a, b):
    return np.array_equal(np.ascontiguousarray(a).view(np.uint8), np.ascontiguousarray(b).view(np.uint8))


@pytest.mark.gpu
def test_multi_c2_one_device_equals_render_pixels(grt, gpu):
    hs = host_scene(grt, "schwarzschild.toml", c2_opts(grt))
    scene = grt.Scene(hs.desc_ptr(), keepalive=hs)
    got = scene.render_frame_multi([gpu], 16, fields=("xyza", "xyza64", "class", "status", "stop", "steps"))
    ref = scene.render_pixels(device=gpu)
    assert _same(got["xyza"], ref.xyza) and _same(got["xyza64"], ref.xyza64)
    assert _same(got["class"], ref.ray_class) and _same(got["status"], ref.status)
    assert _same(got["stop"], ref.stop_reason) and _same(got["steps"], ref.steps)
    assert got["stats"]["accepted_steps"] == ref.stats["accepted_steps"]
    rep = got["report"]
    assert rep.n_devices == 1 and rep.record_bytes == 32 + 16 + 4 + 3 and rep.attempts == 1
    assert rep.rows[0] == 1500 and rep.accepted_steps[0] == ref.stats["accepted_steps"]
    assert rep.gather_ms > 0 and rep.wall_ms > rep.trace_ms[0] > 0
    # the 18-B record only, a second frame on the cached communicator
    again = scene.render_frame_multi([gpu], 16)
    assert _same(again["xyza"], ref.xyza) and again["report"].record_bytes == 18


@pytest.mark.gpu
def test_multi_reduced_c4_one_device_equals_render_pixels(grt, gpu):
    import bench

    hs = host_scene(grt, "kerr.toml", bench.c4_opts(grt, 384, max_steps=100000))
    scene = grt.Scene(hs.desc_ptr(), keepalive=hs)
    got = scene.render_frame_multi([gpu], 16, fields=("xyza", "class", "status", "steps"))
    ref = scene.render_pixels(device=gpu)
    assert _same(got["xyza"], ref.xyza) and _same(got["class"], ref.ray_class)
    assert _same(got["status"], ref.status) and _same(got["steps"], ref.steps)


@pytest.mark.gpu
def test_multi_c5_adaptive_one_device_equals_render_section(grt, gpu):
    hs = host_scene(grt, "schwarzschild.toml", c2_opts(grt))
    scene = grt.Scene(hs.desc_ptr(), keepalive=hs, adaptive=hs.adaptive)
    assert hs.adaptive.enabled
    got = scene.render_frame_multi([gpu], 16, supersample=True, fields=("xyza64", "class", "status", "stop", "steps"),
                                   fail_capacity=1 << 16)
    ref = scene.render_section_ex(adaptive=hs.adaptive, device=gpu, failure_capacity=1 << 16, log_events=True)
    assert got["n_supersampled"] == ref.n_supersampled > 0
    assert _same(got["xyza64"], ref.xyza64)
    assert _same(got["status"], ref.status) and _same(got["stop"], ref.stop) and _same(got["steps"], ref.steps)
    # the failed sub-samples and the NaN / no-terminal-event sub-rays, in (pixel, stratum) order
    f = got["failures"]
    assert f["count"] == ref.n_failed_subsamples + len(ref.subsample_events)
    err = f["status"] != 0
    assert np.array_equal(np.stack([f["pixel"][err], f["sample"][err], f["status"][err].astype(np.uint32)], axis=1),
                          ref.failed_subsamples)
    assert np.array_equal(np.stack([f["pixel"][~err], f["sample"][~err], f["stop"][~err].astype(np.uint32),
                                    f["steps"][~err]], axis=1), ref.subsample_events)
    assert got["report"].allgather_ms > 0


@pytest.mark.gpu
def test_render_shard_from_four_host_threads(grt, gpu):
    from gr_raytracer_amd import _lib as L

    hs = host_scene(grt, "schwarzschild.toml", c2_opts(grt, width=512, height=512))
    scene = grt.Scene(hs.desc_ptr(), keepalive=hs)
    ref = [scene.render_shard(16, s, 4, device=gpu) for s in range(4)]
    got = [None] * 4
    errs = []
    stop = threading.Event()

    def shard(s):
        try:
            got[s] = scene.render_shard(16, s, 4, device=gpu)
        except Exception as e:  # noqa: BLE001
            errs.append(e)

    def flip():  # process-wide knobs, scheduling only: results must not move
        lib = L.lib()
        k = 0
        while not stop.is_set():
            lib.grt_set_schedule((k % 3) - 1)
            lib.grt_set_two_ended(k % 2)
            lib.grt_set_launch_config(0 if k % 2 else 4, 0 if k % 2 else 128)
            k += 1
    th = [threading.Thread(target=shard, args=(s,)) for s in range(4)]
    fl = threading.Thread(target=flip)
    fl.start()
    for t in th:
        t.start()
    for t in th:
        t.join()
    stop.set()
    fl.join()
    lib = L.lib()
    lib.grt_set_schedule(-1)
    lib.grt_set_two_ended(1)
    lib.grt_set_launch_config(0, 0)
    assert not errs, errs
    for s in range(4):
        assert _same(got[s].xyza, ref[s].xyza) and _same(got[s].xyza64, ref[s].xyza64)
        assert _same(got[s].steps, ref[s].steps) and _same(got[s].status, ref[s].status)


@pytest.mark.gpu
def test_cli_gpus_one_writes_the_single_gpu_png(grt, gpu, tmp_path):
    exe = ROOT / "gr_raytracer_amd" / "lib" / "grt"
    common = [str(exe), "--width=256", "--height=256", "--camera-position=-16.0,0.0,3.5", "--theta=-3.142",
              "--psi=0.0", "--phi=0.0", "--max-steps=100000", "--resource-root", str(RESOURCES),
              "--config-file", str(SCENES / "schwarzschild.toml")]
    one = tmp_path / "one.png"
    multi = tmp_path / "multi.png"
    r1 = subprocess.run(common + ["render", "--filename", str(one)], capture_output=True, text=True, timeout=120)
    r2 = subprocess.run(common[:1] + ["--gpus", "1"] + common[1:] + ["render", "--filename", str(multi)],
                        capture_output=True, text=True, timeout=120)
    assert r1.returncode == 0, r1.stderr
    assert r2.returncode == 0, r2.stderr
    assert hashlib.sha256(one.read_bytes()).hexdigest() == hashlib.sha256(multi.read_bytes()).hexdigest()
    assert "1 GPU(s)" in r2.stderr and "phases (ms)" in r2.stderr
    # the reference's log lines are the same, in the same order
    strip = [ln.replace(str(one), "F") for ln in r1.stderr.splitlines() if "INFO" in ln and "Elapsed" not in ln]
    strip2 = [ln.replace(str(multi), "F") for ln in r2.stderr.splitlines() if "INFO" in ln and "Elapsed" not in ln]
    assert strip == strip2
    # sections stay single-GPU
    r3 = subprocess.run(common[:1] + ["--gpus", "1"] + common[1:] + ["render", "--from-row", "8", "--filename",
                                                                      str(tmp_path / "x.png")],
                        capture_output=True, text=True, timeout=120)
    assert r3.returncode == 2 and "whole frames" in r3.stderr
