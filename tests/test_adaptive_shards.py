"""Adaptive supersampling of a frame split across GPUs.

render_section_to_cie_buffer_supersampled (raytracer.rs:257-318) needs, for each pixel,
its 8 neighbours' 1-spp colour and class, and a luminance floor that is a percentile
of the WHOLE frame.  With cyclic row bands those neighbours belong to other ranks, so
the ranks allgather (Y, alpha, class) once, then select and supersample their own
pixels (grt_supersample_shard).  The bar: the assembled frame equals a single-process
grt_render_section of the same frame bit for bit (colour, class, selection count).

CPU: the exact percentile (grt_adaptive_min_luminance) against a total_cmp sort, the
allgather assembly over gloo (world 2 and 3), record packing, the CLI flags.
GPU: in-process shards against grt_render_section, and the multi-process `render_dist`
CLI (2 ranks on one GPU over gloo) against the single-GPU `grt` binary.
"""
import ctypes as C
import os
import socket
import struct
import subprocess
import sys
import tempfile

import numpy as np
import pytest

from conftest import RESOURCES, ROOT, SCENES, c2_opts, host_scene


def _total_cmp_key(v: float) -> int:
    b = struct.unpack("<q", struct.pack("<d", v))[0]
    return b ^ ((b >> 63) & 0x7FFFFFFFFFFFFFFF)


def _ref_floor(lum):
    """resolve_minimum_luminance (raytracer.rs:118-129) by a full total_cmp sort."""
    if len(lum) == 0:
        return 0.0
    s = sorted(lum.tolist(), key=_total_cmp_key)
    return 1e-3 * s[int((len(lum) - 1) * 0.99)]


@pytest.mark.parametrize("n", [0, 1, 2, 99, 100, 101, 1000, 4097])
def test_min_luminance_is_the_total_cmp_percentile(grt, n):
    from gr_raytracer_amd import _lib as L

    rng = np.random.default_rng(n)
    lum = rng.exponential(size=n) * rng.choice([1e-9, 1.0, 1e3], size=n)
    if n > 10:  # signed zeros, NaNs of both signs, infinities: total_cmp places them all
        lum[:6] = [0.0, -0.0, np.inf, -np.inf, np.nan, -np.nan]
        rng.shuffle(lum)
    cfg = L.AdaptiveConfig()
    L.lib().grt_default_adaptive_config(C.byref(cfg))
    cfg.has_minimum_luminance = 0
    lum = np.ascontiguousarray(lum)
    got = L.lib().grt_adaptive_min_luminance(L.dptr(lum) if n else None, n, C.byref(cfg))
    want = _ref_floor(lum)
    assert struct.pack("<d", got) == struct.pack("<d", want) or (np.isnan(got) and np.isnan(want))
    cfg.has_minimum_luminance = 1
    cfg.minimum_luminance = 0.25
    assert L.lib().grt_adaptive_min_luminance(L.dptr(lum) if n else None, n, C.byref(cfg)) == 0.25


def test_luminance_and_section_records_round_trip():
    import torch

    from gr_raytracer_amd.distributed import (pack_luminance_records, pack_section_records, unpack_luminance_records,
                                              unpack_section_records)

    rng = np.random.default_rng(3)
    x = torch.from_numpy(rng.normal(size=(37, 4)))
    c = torch.from_numpy(rng.integers(0, 3, 37).astype(np.uint8))
    s = torch.from_numpy(rng.integers(0, 9, 37).astype(np.uint8))
    ya, cc = unpack_luminance_records(pack_luminance_records(x, c))
    assert torch.equal(ya[:, 0], x[:, 1]) and torch.equal(ya[:, 1], x[:, 3]) and torch.equal(cc, c)
    x2, c2, s2 = unpack_section_records(pack_section_records(x, c, s))
    assert torch.equal(x2, x) and torch.equal(c2, c) and torch.equal(s2, s)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


ROWS, COLS = 37, 11


def _allgather_worker(rank, world, port, band_rows, out_dir):
    sys.path.insert(0, str(ROOT))
    import torch
    import torch.distributed as dist

    from gr_raytracer_amd.distributed import allgather_frame, shard_frame_rows

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        rows = shard_frame_rows(ROWS, band_rows, rank, world)
        # record of frame pixel (r, c): 5 bytes spelling its row and column
        rec = np.zeros((len(rows) * COLS, 5), np.uint8)
        for k, r in enumerate(rows):
            for c in range(COLS):
                rec[k * COLS + c] = [r, c, 7, rank, 255]
        frame = allgather_frame(torch.from_numpy(rec), ROWS, COLS, band_rows, rank, world)
        np.save(os.path.join(out_dir, f"frame{rank}.npy"), frame.numpy())
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,band_rows", [(2, 8), (3, 4)])
def test_gloo_allgather_puts_every_pixel_in_frame_order(world, band_rows):
    import torch.multiprocessing as mp

    from gr_raytracer_amd.distributed import shard_frame_rows

    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_allgather_worker, args=(world, _free_port(), band_rows, d), nprocs=world, join=True)
        owner = np.zeros(ROWS, np.uint8)
        for s in range(world):
            owner[shard_frame_rows(ROWS, band_rows, s, world)] = s
        want = np.array([[r, c, 7, owner[r], 255] for r in range(ROWS) for c in range(COLS)], np.uint8)
        for rank in range(world):
            assert np.array_equal(np.load(os.path.join(d, f"frame{rank}.npy")), want)


def test_render_dist_flags():
    from gr_raytracer_amd.render_dist import parse_args

    a = parse_args(["--width=4096", "--height", "4096", "--max-steps=1000000", "--camera-position=-10,0,-0.5",
                    "--theta=1.52", "--psi=-1.57", "--config-file", "kerr.toml", "render", "--filename", "k.png"])
    assert (a.width, a.height, a.max_steps, a.theta, a.psi) == (4096, 4096, 1000000, 1.52, -1.57)
    assert a.camera_position == [-10.0, 0.0, -0.5] and a.filename == "k.png" and a.tone_mapping == "reinhard"
    with pytest.raises(SystemExit):
        parse_args(["--config-file", "x.toml", "render", "--from-row", "3"])
    with pytest.raises(SystemExit):
        parse_args(["--config-file", "x.toml", "--sampling-mask-color=1,2,300", "render"])


# ------------------------------------------------------------------------ GPU --
def _frame_adaptive(grt, width=72, height=64, spa=4):
    hs = host_scene(grt, "schwarzschild.toml", c2_opts(grt, width=width, height=height))
    ad = hs.adaptive
    ad.enabled = 1
    ad.samples_per_axis = spa
    return hs, ad


def _supersample_in_process(grt, sc, ad, n_shards, band_rows, mask=None):
    """Every rank's steps of render_frame_adaptive, one after another in this process,
    with the allgather done by array assembly."""
    import torch

    from gr_raytracer_amd import _lib as L
    from gr_raytracer_amd.distributed import shard_frame_rows

    rows, cols = sc.rows, sc.cols
    parts = [sc.render_shard(band_rows, s, n_shards) for s in range(n_shards)]
    frame_x = np.zeros((rows, cols, 4))
    frame_c = np.zeros((rows, cols), np.uint8)
    for s, p in enumerate(parts):
        r = shard_frame_rows(rows, band_rows, s, n_shards)
        frame_x[r] = p.xyza64.reshape(len(r), cols, 4)
        frame_c[r] = p.ray_class.reshape(len(r), cols)
    lum = np.ascontiguousarray(frame_x[..., 1].ravel())
    min_lum = L.lib().grt_adaptive_min_luminance(L.dptr(lum), lum.size, C.byref(ad))
    dev = torch.device("cuda", 0)
    d_ya = torch.from_numpy(np.ascontiguousarray(frame_x[..., [1, 3]].reshape(-1, 2))).to(dev)
    d_cls = torch.from_numpy(frame_c.ravel()).to(dev)
    out = np.zeros((rows, cols, 4))
    n_sel = 0
    for s, p in enumerate(parts):
        d_x = torch.from_numpy(p.xyza64).to(dev)
        stats = torch.zeros(4, dtype=torch.int64, device=dev)
        cnt = C.c_uint64(0)
        sh = L.RowShard(band_rows, s, n_shards)
        m = None if mask is None else (C.c_double * 4)(*mask)
        L.check(L.lib().grt_supersample_shard(sc._s, 0, None, C.byref(sh), C.byref(ad), min_lum, d_ya.data_ptr(),
                                              d_cls.data_ptr(), m, d_x.data_ptr(), C.byref(cnt), stats.data_ptr()),
                "grt_supersample_shard")
        n_sel += cnt.value
        r = shard_frame_rows(rows, band_rows, s, n_shards)
        out[r] = d_x.cpu().numpy().reshape(len(r), cols, 4)
    return out.reshape(-1, 4), frame_c.ravel(), n_sel


@pytest.mark.gpu
@pytest.mark.parametrize("n_shards,band_rows", [(1, 16), (2, 8), (3, 16), (8, 8)])
def test_shard_supersampling_equals_render_section(grt, gpu, n_shards, band_rows):
    hs, ad = _frame_adaptive(grt)
    sc = grt.Scene(hs.desc_ptr(), keepalive=hs, adaptive=ad)
    want, want_cls, want_sel, _ = sc.render_section(adaptive=ad)
    got, got_cls, got_sel = _supersample_in_process(grt, sc, ad, n_shards, band_rows)
    assert want_sel > 0 and got_sel == want_sel
    assert np.array_equal(got_cls, want_cls)
    assert np.array_equal(got, want)  # bit for bit


@pytest.mark.gpu
def test_shard_sampling_mask_equals_render_section(grt, gpu):
    hs, ad = _frame_adaptive(grt, spa=2)
    sc = grt.Scene(hs.desc_ptr(), keepalive=hs, adaptive=ad)
    mask = grt.srgb_to_xyza(255, 0, 255)
    want, _, want_sel, _ = sc.render_section(adaptive=ad, sampling_mask_xyza=mask)
    got, _, got_sel = _supersample_in_process(grt, sc, ad, 3, 8, mask=list(mask))
    assert got_sel == want_sel > 0
    assert np.array_equal(got, want)


@pytest.mark.gpu
@pytest.mark.parametrize("tone,ranks,height", [("reinhard", 2, 72), ("global-linear", 2, 72),
                                               ("reinhard", 3, 80)])  # 10 bands of 8 over 3 ranks: 4 / 3 / 3
def test_render_dist_ranks_equal_grt_cli(gpu, tone, ranks, height):
    """`render_dist` with 2 or 3 ranks (gloo, all on GPU 0) writes the same PNG and the
    same f64 frame as the single-GPU `grt` binary; the stock TOML supersamples adaptively."""
    flags = ["--width=80", f"--height={height}", "--camera-position=-16.0,0.0,3.5", "--theta=-3.142",
             "--max-steps=100000", f"--tone-mapping={tone}", "--config-file", str(SCENES / "schwarzschild.toml"),
             "--resource-root", str(RESOURCES)]
    env = dict(os.environ, PYTHONPATH=str(ROOT))
    with tempfile.TemporaryDirectory() as d:
        ref_png, ref_raw = os.path.join(d, "ref.png"), os.path.join(d, "ref.raw")
        subprocess.run([str(ROOT / "gr_raytracer_amd" / "lib" / "grt"), *flags, "--raw-out", ref_raw, "render",
                        "--filename", ref_png], check=True, timeout=240, env=env)
        png, raw, png2 = os.path.join(d, "d.png"), os.path.join(d, "d.raw"), os.path.join(d, "d2.png")
        launch = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={ranks}",
                  "--master-addr=127.0.0.1", f"--master-port={_free_port()}", "-m", "gr_raytracer_amd.render_dist",
                  "--backend=gloo", "--band-rows=8"]
        subprocess.run([*launch, *flags, "--raw-out", raw, "render", "--filename", png], check=True, timeout=240,
                       env=env, cwd=str(ROOT))
        launch[5] = f"--master-port={_free_port()}"
        subprocess.run([*launch, *flags, "render", "--filename", png2], check=True, timeout=240, env=env,
                       cwd=str(ROOT))
        assert np.array_equal(np.fromfile(raw), np.fromfile(ref_raw))
        ref = open(ref_png, "rb").read()
        assert open(png, "rb").read() == ref  # rank 0 tone-maps the gathered f64 frame
        assert open(png2, "rb").read() == ref  # per-rank tone mapping, sRGB rows gathered


@pytest.mark.gpu
def test_grt_cli_logs_failed_pixels_like_the_reference(grt, oracle, gpu, tmp_path):
    """raytracer.rs:232-239: the `render` CLI logs every pixel whose colour failed and
    the set equals the oracle's.  The C2 scene with its disc reaching inside the ISCO
    (inner radius 2 < r_isco = 3): those hits fail with BelowRISCO (temperature.rs)."""
    import re

    scene = tmp_path / "below_isco.toml"
    scene.write_text((SCENES / "schwarzschild.toml").read_text().replace("inner_radius = 3.0", "inner_radius = 2.0"))
    flags = ["--width=64", "--height=64", "--camera-position=-16.0,0.0,3.5", "--theta=-3.142", "--max-steps=100000",
             "--config-file", str(scene), "--resource-root", str(RESOURCES)]
    r = subprocess.run([str(ROOT / "gr_raytracer_amd" / "lib" / "grt"), *flags, "render", "--filename",
                        str(tmp_path / "o.png")], capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr
    names = {1: "IntegrationError(MaxStepsReached)", 2: "NoCircularOrbitPossible", 3: "BelowRISCO",
             4: "NonFiniteRadius"}
    got = {(int(x), int(y), e) for x, y, e in
           re.findall(r"Unable to compute color for ray at pixel \((\d+), (\d+)\): (\S+)", r.stderr)}
    hs = grt.HostScene(str(scene), c2_opts(grt, width=64, height=64), str(RESOURCES))
    ref = oracle.render_pixels(hs.desc, 0, 0, 64, 64, threads=16)
    st = ref["status"].reshape(64, 64) & 0x7F
    want = {(int(c), int(rw), names[int(st[rw, c])]) for rw, c in zip(*np.nonzero(st))}
    assert len(want) > 10
    # the stock TOML supersamples: supersample's Err arm (raytracer.rs:357-362) logs every
    # failed sub-ray of a selected pixel with the same message
    ad = hs.adaptive
    assert ad.enabled
    sel, _ = oracle.select_pixels(ref["xyza"], ref["ray_class"], 64, 64, ad)
    spa = ad.samples_per_axis
    pix, dx, dy = [], [], []
    for p in np.flatnonzero(sel):
        row, col = divmod(int(p), 64)
        for s in range(spa * spa):
            ox, oy = oracle.stratified_offset(row, col, s // spa, s % spa, spa)
            pix.append(p); dx.append(ox); dy.append(oy)
    sub = oracle.render_pixels(hs.desc, 0, 0, 64, 64, threads=16,
                               offsets=(np.asarray(pix), np.asarray(dx), np.asarray(dy)))
    for p, s in zip(pix, sub["status"] & 0x7F):
        if s:
            want.add((int(p) % 64, int(p) // 64, names[int(s)]))
    assert got == want


@pytest.mark.gpu
@pytest.mark.parametrize("n", [1, 2, 101, 4097, 250001])
def test_device_floor_equals_host_floor(grt, gpu, n):
    """grt_adaptive_min_luminance_device (radix sort on the GPU) selects the same f64 as
    the host's nth_element in total_cmp order, special values included."""
    import torch

    from gr_raytracer_amd import _lib as L

    rng = np.random.default_rng(n)
    lum = rng.exponential(size=n) * rng.choice([1e-9, 1.0, 1e3], size=n)
    if n > 10:
        lum[:6] = [0.0, -0.0, np.inf, -np.inf, np.nan, -np.nan]
        rng.shuffle(lum)
    cfg = L.AdaptiveConfig()
    L.lib().grt_default_adaptive_config(C.byref(cfg))
    cfg.has_minimum_luminance = 0
    want = L.lib().grt_adaptive_min_luminance(L.dptr(np.ascontiguousarray(lum)), n, C.byref(cfg))
    for stride in (1, 2, 4):
        a = np.zeros(n * stride)
        a[::stride] = lum
        d = torch.from_numpy(a).to(torch.device("cuda", 0))
        got = C.c_double()
        L.check(L.lib().grt_adaptive_min_luminance_device(0, None, d.data_ptr(), stride, n, C.byref(cfg),
                                                          C.byref(got)), "grt_adaptive_min_luminance_device")
        assert struct.pack("<d", got.value) == struct.pack("<d", want) or (np.isnan(got.value) and np.isnan(want))



@pytest.mark.gpu
def test_cli_logs_unterminated_rays_like_the_reference(grt, oracle, gpu, tmp_path):
    """scene.rs:178-183 / :196-202 and raytracer.rs:325: `grt render` and a 2-rank
    `render_dist` log every error-free ray that ended without a terminal event ("Ray did not
    hit anything ... with N steps", N = steps.len() incl. the initial step) or on NaN
    coordinates, 1-spp and supersample sub-rays alike, and "Supersampling N pixels"; the
    sets equal the oracle's stop reasons.  max-steps 3000 < the ~15000 steps an escaping
    ray needs, so most rays end on the budget."""
    import re

    flags = ["--width=48", "--height=40", "--camera-position=-16.0,0.0,3.5", "--theta=-3.142", "--max-steps=3000",
             "--config-file", str(SCENES / "schwarzschild.toml"), "--resource-root", str(RESOURCES)]
    pat = r"Ray (did not hit anything|hit NaN coordinates): Ray \{ row: (\d+), col: (\d+), \.\. \}.* with (\d+) steps\."

    def events(text):
        return sorted((int(r), int(c), int(n), kind.startswith("hit")) for kind, r, c, n in re.findall(pat, text))

    r = subprocess.run([str(ROOT / "gr_raytracer_amd" / "lib" / "grt"), *flags, "render", "--filename",
                        str(tmp_path / "o.png")], capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr
    hs = grt.HostScene(str(SCENES / "schwarzschild.toml"), c2_opts(grt, width=48, height=40, max_steps=3000),
                       str(RESOURCES))
    ref = oracle.render_pixels(hs.desc, 0, 0, 40, 48, threads=16)
    want = []
    for p in np.flatnonzero((ref["status"] == 0) & np.isin(ref["stop"], (0, 3))):
        want.append((int(p) // 48, int(p) % 48, int(ref["steps"][p]) + 1, bool(ref["stop"][p] == 3)))
    assert len(want) > 1000
    ad = hs.adaptive
    sel, _ = oracle.select_pixels(ref["xyza"], ref["ray_class"], 48, 40, ad)
    spa = ad.samples_per_axis
    pix, dx, dy = [], [], []
    for p in np.flatnonzero(sel):
        row, col = divmod(int(p), 48)
        for s in range(spa * spa):
            ox, oy = oracle.stratified_offset(row, col, s // spa, s % spa, spa)
            pix.append(p); dx.append(ox); dy.append(oy)
    sub = oracle.render_pixels(hs.desc, 0, 0, 40, 48, threads=16,
                               offsets=(np.asarray(pix), np.asarray(dx), np.asarray(dy)))
    for k in np.flatnonzero((sub["status"] == 0) & np.isin(sub["stop"], (0, 3))):
        want.append((int(pix[k]) // 48, int(pix[k]) % 48, int(sub["steps"][k]) + 1, bool(sub["stop"][k] == 3)))
    assert sel.sum() > 0 and len(want) > len(ref["stop"])
    assert events(r.stderr) == sorted(want)
    assert re.findall(r"INFO Supersampling (\d+) pixels", r.stderr) == [str(int(sel.sum()))]

    env = dict(os.environ, PYTHONPATH=str(ROOT))
    launch = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
              "--master-addr=127.0.0.1", f"--master-port={_free_port()}", "-m", "gr_raytracer_amd.render_dist",
              "--backend=gloo", "--band-rows=8"]
    d = subprocess.run([*launch, *flags, "render", "--filename", str(tmp_path / "d.png")], capture_output=True,
                       text=True, timeout=240, env=env, cwd=str(ROOT))
    assert d.returncode == 0, d.stderr[-3000:]
    assert events(d.stderr) == sorted(want)
    assert re.findall(r"INFO Supersampling (\d+) pixels", d.stderr) == [str(int(sel.sum()))]


@pytest.mark.gpu
@pytest.mark.parametrize("fname,geom", [("o.png", "kerr.toml"), ("o.hdr", "kerr-bl.toml")])
def test_cli_info_lines_follow_the_reference(grt, oracle, gpu, tmp_path, fname, geom):
    """`grt render` with a stock TOML logs the reference's info! lines in its order:
    main.rs:100-103 (coordinate system), the temperature LUT's (temperature.rs:63-102:
    r_isco from the oracle's own restatement, in Rust's Display form), raytracer.rs:468-483
    (HDR or non-HDR, tone mapping), :264-267 / :325 / :313-316 (the supersampled section),
    :494 (saved image) and main.rs:176 (elapsed time, Duration's {:.2?})."""
    import re

    from gr_raytracer_amd.scene import format_f64

    out = tmp_path / fname
    flags = ["--width=24", "--height=16", "--max-steps=500", "--camera-position=-10,0,-0.5", "--config-file",
             str(SCENES / geom), "--resource-root", str(RESOURCES)]
    r = subprocess.run([str(ROOT / "gr_raytracer_amd" / "lib" / "grt"), *flags, "render", "--filename", str(out)],
                       capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr
    info = [ln.split(" INFO ", 1)[1] for ln in r.stderr.splitlines() if " INFO " in ln]
    a, radius = 0.499, 1.0
    coord = "Cartesian" if geom == "kerr.toml" else "BoyerLindquist { a: 0.499 }"
    want = [f"Using coordinate system: {coord}",
            f"Computed r_isco: {format_f64(oracle.r_isco(radius, a))} from a: 0.499 and radius: 1",
            r"Max f: [0-9.]+ at radius: [0-9.]+",
            r"Computed m_dot: [0-9.]+ for target temperature: 2000"]
    want += ["Creating HDR image"] if fname.endswith(".hdr") else ["Creating non-HDR image",
                                                                     "Tone mapping method: Reinhard"]
    want += [r"Rendering section from \(0, 0\) to \(16, 24\) with supersampling", r"Supersampling \d+ pixels",
             r"Finished rendering section from \(0, 0\) to \(16, 24\)", f"saved image to {re.escape(str(out))}",
             r"Elapsed time: \d+\.\d\d(s|ms)"]
    assert len(info) == len(want), info
    for got, pat in zip(info, want):
        assert re.fullmatch(pat if "\\" in pat or "[" in pat else re.escape(pat), got), (got, pat)
