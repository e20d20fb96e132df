"""Time-stepped model of a C4 shard's schedule: lanes of the
integrate kernel, the early hand-off to quads beside it, the final hand-off.

usage: python tools/early_sim.py gpurun_out/r03l/steps_c4_8_2.npy [T k] ...
Each (T, k) pair: rays move to a free quad of the k early CUs once they pass T accepted
steps (T = 0: no early hand-off).  Model: a lane runs LANE_US per step while the chip is
full, a quad QUAD_US; the probe-ordered tile queue is rebuilt as tools/tail_replay.py
does; the final hand-off moves every live ray to the whole chip's quads once the queue is
drained and at most 64 rays per CU are live.  Not calibrated: with LANE_US = 45 it
matches the measured drain (27 s) but puts the final hand-off at ~37 s against the
measured 45.5 s (profiles/r03k, r03m), so it cannot rank schedules."""
import sys

import numpy as np

LANE_US = 53.5  # per accepted step, every lane busy (2.45e9 steps/s over 131072 lanes)
QUAD_US = 13.3  # per accepted step in tail_kernel (measured tail timeline)
CAP = 20700     # probe cap: 1.3 x max_radius steps
CUS = 256


def probe_order(steps):
    cols = 4096
    rows = steps.size // cols
    s = steps.reshape(rows, cols)
    ty, tx = (rows + 7) // 8, cols // 8
    tiles = np.zeros((ty * 8, tx * 8))
    tiles[:rows] = s
    t4 = tiles.reshape(ty, 8, tx, 8).transpose(0, 2, 1, 3).reshape(ty * tx, 64)
    probe = np.minimum(t4[:, 3 * 8 + 3], CAP).reshape(ty, tx)
    pad = np.pad(probe, 1)
    key = np.max(np.stack([pad[dy:dy + ty, dx:dx + tx] for dy in range(3) for dx in range(3)]), axis=0).ravel()
    o = np.argsort(-key, kind="stable")
    q = t4[o].ravel()
    return q[q > 0]


def simulate(queue, T, k, dt=0.05, lane_us=LANE_US, quad_us=QUAD_US):
    n_lanes = (CUS - k) * 512
    n_quads = k * 64
    lane_left = np.zeros(n_lanes)   # steps left of the lane's ray (0: free)
    lane_done = np.zeros(n_lanes)   # steps done
    quad_left = np.zeros(max(n_quads, 1))
    head, t, drained, final = 0, 0.0, None, None
    nq = len(queue)
    tail_left = None
    while True:
        # refill free lanes from the queue
        free = np.flatnonzero(lane_left <= 0)
        take = min(len(free), nq - head)
        if take:
            lane_left[free[:take]] = queue[head:head + take]
            lane_done[free[:take]] = 0
            head += take
        if head >= nq and drained is None:
            drained = t
        # early hand-off: rays past T move to free quads (longest-done first)
        if T and n_quads:
            fq = np.flatnonzero(quad_left <= 0)
            if len(fq):
                cand = np.flatnonzero((lane_left > 0) & (lane_done >= T))
                if len(cand):
                    cand = cand[np.argsort(-lane_done[cand])][:len(fq)]
                    quad_left[fq[:len(cand)]] = lane_left[cand]
                    lane_left[cand] = 0
        live = int((lane_left > 0).sum())
        if drained is not None and live <= 64 * (CUS - k):
            final = t
            rest = np.concatenate([lane_left[lane_left > 0], quad_left[quad_left > 0]])
            # the whole chip's quads after the integrate kernel: every ray on its own quad
            end = t + (rest.max() if len(rest) else 0) * quad_us * 1e-6
            return {"T": T, "k": k, "drained_s": round(drained, 2), "final_s": round(final, 2),
                    "end_s": round(end, 2)}
        occ = min(1.0, live / n_lanes) if n_lanes else 0
        # lanes speed up as the SIMDs empty (a lone wave issues ~1.8x as often)
        speed = 1.0 if occ > 0.5 else 1.0 + 0.8 * (1 - 2 * occ)
        lane_left -= dt * 1e6 / lane_us * speed * (lane_left > 0)
        lane_done += dt * 1e6 / lane_us * speed
        quad_left -= dt * 1e6 / quad_us
        t += dt


def main():
    steps = np.load(sys.argv[1]).astype(np.float64).ravel()
    queue = probe_order(steps)
    pairs = [(int(a), int(b)) for a, b in zip(sys.argv[2::2], sys.argv[3::2])] or [(0, 0)]
    for T, k in pairs:
        print(simulate(queue, T, k), flush=True)


if __name__ == "__main__":
    main()
