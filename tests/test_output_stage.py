"""Output stage: CIE XYZ -> tone-mapped sRGB8, color.rs:204-298,
as Raytracer::render_section calls it for non-HDR files (raytracer.rs:481-487).

The bar is byte identity with the oracle's restatement (oracle_xyz_to_srgb8), for both
tone mappings (Reinhard, GlobalLinear), on rendered frames and on edge values: the
compand threshold 0.0031308, .5 rounding boundaries, NaN / inf / negative / huge inputs.
CPU tests cover the host C++ path (grt_xyz_to_srgb8 = grt_linear_max + grt_tonemap) and
the multi-rank GlobalLinear reduction (gloo, world 2); `gpu` tests cover the HIP kernels
(grt_linear_max_async, grt_tonemap_async, grt_xyz_to_srgb8_device).
"""
import os
import socket
import tempfile

import numpy as np
import pytest

from conftest import ROOT, c2_opts, host_scene

TONES = {0: "Reinhard", 1: "GlobalLinear"}


def edge_values():
    """(n, 4) XYZA rows that stress every branch of the output stage."""
    rng = np.random.default_rng(7)
    rows = [[0, 0, 0, 1], [np.nan, 1, 1, 1], [1, np.nan, 0, 1], [-1, -2, -3, 1], [1e-300, 0, 0, 1],
            [5e-324, 5e-324, 5e-324, 1], [1e300, 1, 1, 1], [0.9505, 1.0, 1.089, 1], [-0.0, -0.0, -0.0, 1]]
    # XYZ whose linear-sRGB red channel lands on the compand threshold and around it
    thr = 0.0031308
    for f in (1 - 1e-15, 1.0, 1 + 1e-15, 0.5, 2.0):
        rows.append([thr * f / 3.2406255, 0, 0, 1])
    # values whose u8 code is near a .5 rounding boundary
    codes = (np.arange(256) + 0.5) / 255.0
    for c in codes[::17]:
        rows.append([c, c, c, 1])
    rnd = np.abs(rng.standard_normal((4000, 4))) * rng.choice([1e-5, 1e-3, 0.1, 1.0, 30.0], (4000, 1))
    return np.vstack([np.array(rows, np.float64), rnd])


def rendered_frame(grt, oracle, rows=24, cols=24):
    hs = host_scene(grt, "schwarzschild.toml", c2_opts(grt, width=cols, height=rows))
    return oracle.render_pixels(hs.desc, 0, 0, rows, cols, threads=4)["xyza"]


@pytest.mark.parametrize("tone", sorted(TONES))
@pytest.mark.parametrize("exposure", [1.0, 0.37])
def test_host_output_stage_matches_oracle(grt, oracle, tone, exposure):
    for x in (edge_values(), rendered_frame(grt, oracle)):
        want = oracle.xyz_to_srgb8(x, tone, exposure)
        got = grt.xyz_to_srgb8(x, tone, exposure)
        assert np.array_equal(got, want), (TONES[tone], np.argwhere(got != want)[:5])


def test_split_max_and_tonemap_equal_whole_buffer(grt, oracle):
    from gr_raytracer_amd import _lib as L

    x = np.ascontiguousarray(edge_values()[9:])  # finite rows
    m = np.zeros(3)
    L.lib().grt_linear_max(L.dptr(x), x.shape[0], 1.0, L.dptr(m))
    assert np.all(m > 0)
    out = np.zeros((x.shape[0], 3), np.uint8)
    L.check(L.lib().grt_tonemap(L.dptr(x), x.shape[0], 1, 1.0, L.dptr(m), L.ptr(out, L.C.c_uint8)))
    assert np.array_equal(out, oracle.xyz_to_srgb8(x, 1))
    # a GlobalLinear map without maxima and an unknown tone mapping are errors
    with pytest.raises(L.GrtError):
        L.check(L.lib().grt_tonemap(L.dptr(x), x.shape[0], 1, 1.0, None, L.ptr(out, L.C.c_uint8)))
    with pytest.raises(L.GrtError):
        L.check(L.lib().grt_tonemap(L.dptr(x), x.shape[0], 5, 1.0, L.dptr(m), L.ptr(out, L.C.c_uint8)))


FRAME_ROWS, FRAME_COLS, BAND = 24, 20, 8


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, out_dir):
    import sys

    sys.path.insert(0, str(ROOT))
    sys.path.insert(0, str(ROOT / "oracle"))
    sys.path.insert(0, str(ROOT / "tests"))
    import torch
    import torch.distributed as dist

    import gr_raytracer_amd as g
    import pyoracle as O
    from gr_raytracer_amd import _lib as L
    from gr_raytracer_amd.distributed import gather_frame, reduce_channel_maxima, shard_frame_rows

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        hs = host_scene(g, "schwarzschild.toml", c2_opts(g, width=FRAME_COLS, height=FRAME_ROWS))
        rows = shard_frame_rows(FRAME_ROWS, BAND, rank, world)
        x = np.ascontiguousarray(O.render_pixels(hs.desc, 0, 0, FRAME_ROWS, FRAME_COLS, threads=2,
                                                 row_list=rows)["xyza"])
        m = np.zeros(3)
        L.lib().grt_linear_max(L.dptr(x), x.shape[0], 1.0, L.dptr(m))
        mt = reduce_channel_maxima(torch.from_numpy(m))
        m = np.ascontiguousarray(mt.numpy())
        rgb = np.zeros((x.shape[0], 3), np.uint8)
        L.check(L.lib().grt_tonemap(L.dptr(x), x.shape[0], 1, 1.0, L.dptr(m), L.ptr(rgb, L.C.c_uint8)))
        frame = gather_frame(torch.from_numpy(rgb), FRAME_ROWS, FRAME_COLS, BAND, rank, world)
        if rank == 0:
            np.save(os.path.join(out_dir, "rgb.npy"), frame.numpy())
    finally:
        dist.destroy_process_group()


def test_gloo_global_linear_frame_equals_single_process(grt, oracle):
    """GlobalLinear across ranks: allreduce(MAX) of the channel maxima, per-rank tone
    map, gather of 3-byte pixels == the whole frame mapped in one process."""
    import torch.multiprocessing as mp

    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_worker, args=(2, _free_port(), d), nprocs=2, join=True)
        got = np.load(os.path.join(d, "rgb.npy"))
    x = rendered_frame(grt, oracle, FRAME_ROWS, FRAME_COLS)
    assert np.array_equal(got, oracle.xyz_to_srgb8(x, 1))


# ------------------------------------------------------------------ GPU ----------
@pytest.mark.gpu
@pytest.mark.parametrize("tone", sorted(TONES))
def test_device_output_stage_matches_oracle(grt, oracle, gpu, tone):
    for exposure in (1.0, 0.37):
        for x in (edge_values(), rendered_frame(grt, oracle)):
            want = oracle.xyz_to_srgb8(x, tone, exposure)
            got = grt.xyz_to_srgb8(x, tone, exposure, device=gpu)
            assert np.array_equal(got, want), (TONES[tone], np.argwhere(got != want)[:5])


@pytest.mark.gpu
def test_device_output_stage_on_a_gpu_render(grt, oracle, gpu):
    """Render on the GPU, keep the f64 XYZA on the device, map it there (async ABI on
    torch's stream), and compare with the oracle's map of the same f64 buffer."""
    import torch

    from gr_raytracer_amd import _lib as L

    hs = host_scene(grt, "schwarzschild.toml", c2_opts(grt))
    sc = grt.Scene(hs.desc_ptr(), keepalive=hs)
    r = sc.render_pixels(700, 700, 64, 96, device=gpu)
    x = torch.from_numpy(r.xyza64).to(f"cuda:{gpu}")
    n = x.shape[0]
    s = torch.cuda.current_stream(gpu)
    lib = L.lib()
    for tone in (0, 1):
        m = torch.zeros(3, dtype=torch.float64, device=x.device)
        rgb = torch.empty((n, 3), dtype=torch.uint8, device=x.device)
        L.check(lib.grt_linear_max_async(gpu, s.cuda_stream, x.data_ptr(), n, 1.0, m.data_ptr()))
        L.check(lib.grt_tonemap_async(gpu, s.cuda_stream, x.data_ptr(), n, tone, 1.0, m.data_ptr(), rgb.data_ptr()))
        torch.cuda.synchronize()
        want_max = np.zeros(3)
        lib.grt_linear_max(L.dptr(np.ascontiguousarray(r.xyza64)), n, 1.0, L.dptr(want_max))
        assert np.array_equal(m.cpu().numpy(), want_max)
        assert np.array_equal(rgb.cpu().numpy(), oracle.xyz_to_srgb8(r.xyza64, tone))


@pytest.mark.gpu
def test_cli_png_is_the_reference_output_stage(grt, oracle, gpu, tmp_path):
    """`grt ... render --filename x.png` (the drop-in for the reference's `render`):
    the PNG's pixels are the reference output stage applied to the rendered f64 XYZA
    (dumped by --raw-out from the same run)."""
    import subprocess

    Image = pytest.importorskip("PIL.Image")
    from conftest import RESOURCES, SCENES

    exe = ROOT / "gr_raytracer_amd" / "lib" / "grt"
    for tone_id, tone in ((0, "reinhard"), (1, "global-linear")):
        png, raw = tmp_path / f"{tone}.png", tmp_path / f"{tone}.raw"
        subprocess.run([str(exe), "--width=40", "--height=32", f"--tone-mapping={tone}",
                        f"--config-file={SCENES / 'euclidean.toml'}", f"--resource-root={RESOURCES}", "render",
                        f"--filename={png}", f"--raw-out={raw}", f"--device={gpu}"], check=True, timeout=300)
        x = np.fromfile(raw, np.float64).reshape(-1, 4)
        assert x.shape[0] == 40 * 32
        img = np.asarray(Image.open(png).convert("RGB")).reshape(-1, 3)
        assert np.array_equal(img, oracle.xyz_to_srgb8(x, tone_id))
