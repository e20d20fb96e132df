"""Offline replay of a C4 shard's tile queue (tail analysis).

usage: python tools/tail_replay.py gpurun_out/<tag>/c4_shard<s>_steps.npy [lanes]
Reads the per-pixel accepted steps of one shard (local rows x 4096), rebuilds the
probe-ordered tile queue of schedule.hip (probe pixel (3, 3) of each 8x8 tile, capped at
32768 steps, key = max over the 3x3 tile neighbourhood, stable descending sort) and
list-schedules the pixels over `lanes` lanes (each free lane takes the next pixel),
reporting the makespan in step-times for the row-major order, the probe order and an
order by the true per-tile maximum (the best any tile order could do)."""
import heapq
import sys

import numpy as np

CAP = 32768


def makespan(costs, lanes):
    h = [0.0] * lanes
    heapq.heapify(h)
    end = 0.0
    for c in costs:
        t = heapq.heappop(h) + c
        end = max(end, t)
        heapq.heappush(h, t)
    return end


def main():
    steps = np.load(sys.argv[1]).astype(np.float64)
    lanes = int(sys.argv[2]) if len(sys.argv) > 2 else 256 * 4 * 256
    cols = 4096
    rows = steps.size // cols
    s = steps.reshape(rows, cols)
    ty, tx = (rows + 7) // 8, cols // 8
    tiles = np.zeros((ty * 8, tx * 8))
    tiles[:rows] = s
    t4 = tiles.reshape(ty, 8, tx, 8).transpose(0, 2, 1, 3).reshape(ty * tx, 64)  # tile-major pixels
    probe = np.minimum(t4[:, 3 * 8 + 3], CAP).reshape(ty, tx)
    pad = np.pad(probe, 1)
    key = np.max(np.stack([pad[dy:dy + ty, dx:dx + tx] for dy in range(3) for dx in range(3)]), axis=0).ravel()
    orders = {
        "row-major": np.arange(ty * tx),
        "probe": np.argsort(-key, kind="stable"),
        "true max": np.argsort(-t4.max(axis=1), kind="stable"),
    }
    longest = t4.max(axis=1)
    top = np.argsort(-longest)[:5]
    print(f"shard: {rows} rows, {steps.sum():.3e} steps, longest ray {steps.max():.0f}, "
          f"rays > 5e5: {(steps > 5e5).sum()}, work floor {steps.sum() / lanes:.0f} step-times")
    for name, o in orders.items():
        pos = {int(t): i for i, t in enumerate(o)}
        print(f"{name:10s} makespan {makespan(t4[o].ravel(), lanes):.0f} step-times; queue position of the 5 "
              f"longest tiles: {[pos[int(t)] for t in top]} of {len(o)}")


if __name__ == "__main__":
    main()
