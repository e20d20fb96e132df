"""bench.py's host logic on CPU: the C4 strong-scaling loop over gloo (world 2, and world 8
with 16-row cyclic bands: the north-star layout), the C2 weak-scaling loop with two frames
in flight over gloo (world 2), the host-core census, and the roofline's refusal of a PMC
summary from another build.

The C4 loop (bench.c4_frame_steps / c4_summary) is backend-agnostic; here each rank's
shard trace is the oracle (this container has no GPU), at a reduced frame size.  The
gathered frame must equal a single-process oracle render, and the summary must carry
the per-rank kernel times, the max/mean imbalance and the gather time.
"""
import json
import os
import socket
import tempfile

import numpy as np
import pytest

from conftest import ROOT, host_scene

SIZE = 24


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _opts(g, rows=SIZE, cols=SIZE):
    import bench

    o = bench.c4_opts(g, SIZE, max_steps=3000)
    o.max_radius = 100.0
    o.height, o.width = rows, cols
    return o


def _worker(rank, world, port, band_rows, out_dir, rows=SIZE, cols=SIZE):
    import sys
    import time

    sys.path.insert(0, str(ROOT))
    sys.path.insert(0, str(ROOT / "oracle"))
    sys.path.insert(0, str(ROOT / "tests"))
    import torch
    import torch.distributed as dist

    import bench
    import gr_raytracer_amd as g
    import pyoracle as O
    from gr_raytracer_amd.distributed import pack_records, shard_frame_rows

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        hs = host_scene(g, "kerr.toml", _opts(g, rows, cols))
        mine = shard_frame_rows(rows, band_rows, rank, world)

        def trace_shard():
            t0 = time.perf_counter()
            r = O.render_pixels(hs.desc, 0, 0, rows, cols, threads=1 if world > 4 else 2, row_list=mine)
            rec = pack_records(torch.from_numpy(r["xyza"].astype(np.float32)), torch.from_numpy(r["ray_class"]),
                               torch.from_numpy(r["status"]))
            return rec, float(r["accepted"]), float(r["attempts"]), (time.perf_counter() - t0) * 1e3

        res = bench.c4_frame_steps(trace_shard, rank, world, rows, cols, band_rows, steps=2, warmup=1,
                                   sync=lambda: None)
        s = bench.c4_summary(res, rank, world)
        if rank == 0:
            frame = res["frame"].numpy()
            np.save(os.path.join(out_dir, "frame.npy"), frame)
            s = {k: v for k, v in s.items()}
            with open(os.path.join(out_dir, "summary.json"), "w") as f:
                json.dump(s, f)
        else:
            assert s is None and res["frame"] is None
    finally:
        dist.destroy_process_group()


# world 8, 16-row bands: the north-star layout; 136 rows = one band per rank plus a ragged
# ninth band (rank 0), on a narrow frame so the oracle's Kerr-Schild traces stay short
@pytest.mark.parametrize("world,band_rows,rows,cols", [(2, 4, SIZE, SIZE), (8, 16, 136, 6)])
def test_c4_strong_scaling_loop_gloo(grt, oracle, world, band_rows, rows, cols):
    import torch.multiprocessing as mp

    from gr_raytracer_amd.distributed import pack_records, shard_frame_rows, shard_row_count

    import torch

    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_worker, args=(world, _free_port(), band_rows, d, rows, cols), nprocs=world, join=True)
        frame = np.load(os.path.join(d, "frame.npy"))
        s = json.load(open(os.path.join(d, "summary.json")))
    hs = host_scene(grt, "kerr.toml", _opts(grt, rows, cols))
    ref = oracle.render_pixels(hs.desc, 0, 0, rows, cols, threads=4)
    want = pack_records(torch.from_numpy(ref["xyza"].astype(np.float32)), torch.from_numpy(ref["ray_class"]),
                        torch.from_numpy(ref["status"])).numpy()
    assert np.array_equal(frame, want)
    assert all(shard_row_count(rows, band_rows, k, world) > 0 for k in range(world))
    assert len(s["per_rank_kernel_ms"]) == world and all(v > 0 for v in s["per_rank_kernel_ms"])
    assert s["imbalance"] >= 1.0
    assert s["gather_ms"] > 0
    assert s["steps"] == 2
    assert s["accepted"] == 2 * ref["accepted"]  # two frames, every rank's steps
    # rank 0's own share: its bands' accepted steps, two frames
    steps = ref["steps"].reshape(rows, cols).astype(np.int64)
    assert s["rank0_accepted"] == 2 * steps[shard_frame_rows(rows, band_rows, 0, world)].sum()


def test_host_cores_census():
    import bench

    hc = bench.host_cores()
    assert hc["threads"] >= 1
    assert hc["affinity_cpus"] == len(os.sched_getaffinity(0))
    if hc["cgroup_cpu_quota"] is None:
        assert hc["threads"] == hc["affinity_cpus"]  # uncapped


def test_roofline_refuses_pmc_of_another_build(grt, tmp_path, monkeypatch):
    import bench

    kname = bench.PMC_KERNEL["c2"]
    pmc = tmp_path / "r99_c2_pmc.json"
    pmc.write_text(json.dumps({"kernel": kname + ", test", "code_object_sha256": "0" * 64,
                               "kernel_code_sha256": "1" * 64, "hbm_bytes_per_launch": 1.0}))
    monkeypatch.setattr(bench, "PMC_DIR", tmp_path)
    r = bench.roofline("c2", "schwarzschild", 1e9, 1e9, 100.0, 1000, "k")
    assert r["traffic"] is None and "another build" in r["traffic_note"]
    assert abs(r["frac"] * bench.FP64_VECTOR_PEAK_TFLOPS - r["achieved"]) < 1e-9
    assert abs(r["frac_no_contraction"] - 2 * r["frac"]) < 1e-12
    # a summary of another kernel is never used, whatever its hashes
    (tmp_path / "r99_c4_pmc.json").write_text(json.dumps({
        "kernel": bench.PMC_KERNEL["c4"] + ", test", "code_object_sha256": grt._lib.device_code_sha256(),
        "hbm_bytes_per_launch": 3.0}))
    assert bench.roofline("c2", "schwarzschild", 1e9, 1e9, 100.0, 1000, "k")["traffic"] is None
    # the per-kernel hash of this build's kernel is accepted
    pmc.write_text(json.dumps({"kernel": kname + ", test", "code_object_sha256": "0" * 64,
                               "kernel_code_sha256": grt._lib.kernel_code_sha256(grt._lib.kernel_symbol(kname)),
                               "rays_per_launch": 1000, "hbm_bytes_per_launch": 7.0, "lane_utilisation": 0.9}))
    # this build's kernel, but a launch of another size: per-launch bytes do not carry over
    r = bench.roofline("c2", "schwarzschild", 1e9, 1e9, 100.0, 2000, "k")
    assert r["traffic"] is None and "another size" in r["traffic_note"]
    r = bench.roofline("c2", "schwarzschild", 1e9, 1e9, 100.0, 1000, "k")
    assert r["traffic"] == 7.0 and r["lane_utilisation"] == 0.9


def _reduce_worker(rank, world, port, out_dir):
    import torch.distributed as dist

    import bench

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        r = bench.reduce_over_ranks(1.0 + rank, 100.0 * (rank + 1), 101.0 * (rank + 1), world)
        with open(os.path.join(out_dir, f"r{rank}.json"), "w") as f:
            json.dump(r, f)
    finally:
        dist.destroy_process_group()


def test_weak_scaling_totals_gloo_world2():
    """bench.reduce_over_ranks (the C2 weak-scaling line): max over ranks of the timed
    region, sums of the steps, identical on every rank."""
    import torch.multiprocessing as mp

    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_reduce_worker, args=(2, _free_port(), d), nprocs=2, join=True)
        got = [json.load(open(os.path.join(d, f"r{r}.json"))) for r in range(2)]
    assert got[0] == got[1] == [2.0, 300.0, 303.0]
    import bench

    assert list(bench.reduce_over_ranks(1.5, 7.0, 8.0, 1)) == [1.5, 7.0, 8.0]


def _c2_loop_worker(rank, world, port, out_dir):
    import torch
    import torch.distributed as dist

    import bench

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        n_slots, steps, warmup = 2, 5, 1
        bufs = [torch.zeros(4) for _ in range(n_slots)]
        lists = [[torch.zeros(4) for _ in range(world)] for _ in range(n_slots)] if rank == 0 else None
        seq, log = [0], []

        def render(j):  # frame number `seq` of this rank into slot j
            bufs[j].fill_(100.0 * rank + seq[0])
            log.append(("render", j, seq[0]))
            seq[0] += 1

        def gather(j):
            dist.gather(bufs[j], gather_list=lists[j] if rank == 0 else None, dst=0)

        elapsed = bench.c2_frame_loop(n_slots, steps, warmup, render, gather, lambda: None, dist.barrier,
                                      lambda: log.append(("reset",)), lambda k, e, j: log.append(("ev", k, e, j)))
        out = {"elapsed": elapsed, "log": log,
               "gathered": [[float(t[0]) for t in lists[j]] for j in range(n_slots)] if rank == 0 else None}
        with open(os.path.join(out_dir, f"r{rank}.json"), "w") as f:
            json.dump(out, f)
    finally:
        dist.destroy_process_group()


def test_c2_frame_loop_gloo_world2():
    """bench.c2_frame_loop (the C2 weak-scaling loop with two frames in flight) over gloo,
    world 2: a warm-up step renders one frame per slot, the counters are reset once, frame
    k goes to slot k mod 2 bracketed by its two events, and each frame is gathered to rank
    0 from its slot, so rank 0 ends with every rank's last frame of each slot."""
    import torch.multiprocessing as mp

    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_c2_loop_worker, args=(2, _free_port(), d), nprocs=2, join=True)
        got = [json.load(open(os.path.join(d, f"r{r}.json"))) for r in range(2)]
    for r in range(2):
        log = [tuple(e) for e in got[r]["log"]]
        assert log[:3] == [("render", 0, 0), ("render", 1, 1), ("reset",)]
        timed = log[3:]
        assert len(timed) == 5 * 3
        for k in range(5):
            assert timed[3 * k:3 * k + 3] == [("ev", k, 0, k % 2), ("render", k % 2, 2 + k), ("ev", k, 1, k % 2)]
        assert got[r]["elapsed"] > 0.0
    # slot 0's last frame is number 6 (timed k = 4), slot 1's number 5 (k = 3), from each rank
    assert got[0]["gathered"] == [[6.0, 106.0], [5.0, 105.0]]


def test_parse_cli_phases():
    import bench

    err = ("[grt] INFO Using coordinate system: Spherical\n[grt] 2250000 rays, 34000000000 accepted steps, "
           "34012345678 attempts, 0 supersampled pixels, kernel 1287.0 ms (2.6e10 steps/s)\n"
           "[grt] INFO saved image to x.png\n[grt] phases (ms): load 210.5, create 0.1, render 1601.2, output 3.4, "
           "write 95.0, since start 1950.3\n[grt] INFO Elapsed time: 1.95s\n")
    p = bench.parse_cli_phases(err)
    assert p["load_ms"] == 210.5 and p["render_ms"] == 1601.2 and p["since_start_ms"] == 1950.3
    assert p["elapsed_line"] == "1.95s" and p["rays"] == 2250000 and p["accepted_steps"] == 34000000000
