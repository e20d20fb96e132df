"""Multi-rank frame assembly on CPU (gloo, world_size 2, 3 and 8).

Each rank renders its cyclic row-band shard (here with the oracle as a stand-in for
the GPU trace, since this container has no GPU), packs 18-byte pixel records and
gathers them to rank 0 with gr_raytracer_amd.distributed.gather_frame; rank 0's frame
must equal a single-process render bit for bit.  The shard row arithmetic is checked
against the C ABI's grt_shard_row_count / grt_shard_frame_row (host-only calls).
"""
import ctypes as C
import os
import socket
import tempfile

import numpy as np
import pytest

from conftest import ROOT, c2_opts, host_scene

FRAME_ROWS, FRAME_COLS = 40, 36


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, band_rows, out_dir, frame_rows=FRAME_ROWS, frame_cols=FRAME_COLS):
    import sys

    sys.path.insert(0, str(ROOT))
    sys.path.insert(0, str(ROOT / "oracle"))
    sys.path.insert(0, str(ROOT / "tests"))
    import torch
    import torch.distributed as dist

    import gr_raytracer_amd as g
    import pyoracle as O
    from gr_raytracer_amd.distributed import gather_frame, pack_records, shard_frame_rows, unpack_records

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        hs = host_scene(g, "schwarzschild.toml", c2_opts(g, width=frame_cols, height=frame_rows))
        rows = shard_frame_rows(frame_rows, band_rows, rank, world)
        r = O.render_pixels(hs.desc, 0, 0, frame_rows, frame_cols, threads=1 if world > 4 else 2, row_list=rows)
        xyza = torch.from_numpy(r["xyza"].astype(np.float32))
        rec = pack_records(xyza, torch.from_numpy(r["ray_class"]), torch.from_numpy(r["status"]))
        frame = gather_frame(rec, frame_rows, frame_cols, band_rows, rank, world)
        if rank == 0:
            fx, fc, fs = unpack_records(frame)
            np.savez(os.path.join(out_dir, "frame.npz"), xyza=fx.numpy(), cls=fc.numpy(), status=fs.numpy())
        else:
            assert frame is None
    finally:
        dist.destroy_process_group()


# world 8 with 16-row bands is the north-star layout (8 ranks, cyclic 16-row bands): 136
# rows give every rank one whole band and a ragged ninth band (8 rows) to rank 0
@pytest.mark.parametrize("world,band_rows,frame_rows,frame_cols", [(2, 8, 40, 36), (3, 16, 40, 36),
                                                                    (8, 16, 136, 10)])
def test_gloo_sharded_frame_equals_single_process(oracle, grt, world, band_rows, frame_rows, frame_cols):
    import torch.multiprocessing as mp

    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_worker, args=(world, _free_port(), band_rows, d, frame_rows, frame_cols), nprocs=world, join=True)
        got = np.load(os.path.join(d, "frame.npz"))
        hs = host_scene(grt, "schwarzschild.toml", c2_opts(grt, width=frame_cols, height=frame_rows))
        ref = oracle.render_pixels(hs.desc, 0, 0, frame_rows, frame_cols, threads=4)
        assert np.array_equal(got["xyza"], ref["xyza"].astype(np.float32))
        assert np.array_equal(got["cls"], ref["ray_class"])
        assert np.array_equal(got["status"], ref["status"])


def test_shard_rows_partition_the_frame_and_match_the_c_abi(grt):
    from gr_raytracer_amd import _lib as L
    from gr_raytracer_amd.distributed import shard_frame_rows, shard_row_count

    lib = L.lib()
    for frame_rows in (1, 7, 8, 40, 1500, 4096):
        for n in (1, 2, 3, 8):
            for band in (1, 8, 16, 100):
                seen = []
                for s in range(n):
                    sh = L.RowShard(band, s, n)
                    cnt = shard_row_count(frame_rows, band, s, n)
                    assert cnt == lib.grt_shard_row_count(frame_rows, C.byref(sh))
                    rows = shard_frame_rows(frame_rows, band, s, n)
                    assert len(rows) == cnt
                    for k in range(0, cnt, max(1, cnt // 7)):
                        assert rows[k] == lib.grt_shard_frame_row(k, C.byref(sh))
                    seen.append(rows)
                allrows = np.sort(np.concatenate(seen))
                assert np.array_equal(allrows, np.arange(frame_rows)), (frame_rows, n, band)
    # invalid shards have no rows
    assert lib.grt_shard_row_count(100, C.byref(L.RowShard(8, 2, 2))) == 0
    assert lib.grt_shard_row_count(100, C.byref(L.RowShard(0, 0, 2))) == 0


def _incomplete_worker(rank, world, port, out_dir, lost_per_rank):
    import sys

    sys.path.insert(0, str(ROOT))
    import torch
    import torch.distributed as dist

    from gr_raytracer_amd.render_dist import EXIT_INCOMPLETE, exit_status, trace_until_complete

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        calls = {"render": 0, "grow": 0}
        logs = []

        def render_once():
            calls["render"] += 1
            return f"frame {calls['render']}"

        def lost_pixels():  # only this rank's pixels lose candidates, on every trace
            t = torch.tensor([lost_per_rank[rank]], dtype=torch.int64)
            dist.all_reduce(t)
            return int(t[0])

        def grow():
            calls["grow"] += 1

        out, incomplete = trace_until_complete(render_once, lost_pixels, grow, logs.append)
        status = exit_status(incomplete)
        assert EXIT_INCOMPLETE == 3
        with open(os.path.join(out_dir, f"rank{rank}.txt"), "w") as f:
            f.write(f"{out}|{incomplete}|{status}|{calls['render']}|{calls['grow']}|{len(logs)}")
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("lost_per_rank,expect", [((0, 4), (3, 4, 3)), ((0, 0), (1, 0, 0))])
def test_render_dist_incomplete_frame_exit_status_gloo(lost_per_rank, expect):
    """render_dist's hit-pool retry loop (trace_until_complete) over gloo, world 2: when one
    rank's pixels lose candidates on all three traces, EVERY rank gets the all-reduced
    count and exits with EXIT_INCOMPLETE (3) after growing its pool twice; with nothing
    lost each rank traces once and exits 0."""
    import torch.multiprocessing as mp

    renders, incomplete, status = expect
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_incomplete_worker, args=(2, _free_port(), d, lost_per_rank), nprocs=2, join=True)
        for r in range(2):
            out, inc, st, n_render, n_grow, n_logs = open(os.path.join(d, f"rank{r}.txt")).read().split("|")
            assert out == f"frame {renders}"
            assert int(inc) == incomplete and int(st) == status
            assert int(n_render) == renders and int(n_grow) == max(0, renders - 1)
            assert int(n_logs) == (renders if incomplete else 0)
