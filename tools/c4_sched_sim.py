"""Wave-level model of a C4 shard's schedule: 1024 SIMDs x
(priority, other) wave x 64 lanes, with the speeds measured in the per-ray record of
tools/c4_ray_times.py (profiles/r04a): the priority (older) wave of a SIMD runs an
attempt in 30.8 us, the other one in 130 us while its partner has live lanes and in 30 us
alone; the tail kernel 12.3 us per attempt and quad.  Every ray costs its measured
attempts.  It ranks tile orders and queue disciplines offline: one end vs both ends,
probe keys (current cap, the probe pixel's true length, the tile's true maximum).

usage: python tools/c4_sched_sim.py RECORD.npz"""
import sys
import numpy as np
d = np.load(sys.argv[1] if len(sys.argv) > 1 else 'gpurun_out/r04a/c4_rt_s2.npz')
ATT = (d['att_int'].astype(np.float64) + d['att_tail'])
STEPS = d['steps'].astype(np.float64)
COLS = 4096
NS, NL = 1024, 64
CAP = 20700

def tiles_of(v):
    rows = v.size // COLS
    return v.reshape(rows // 8, 8, COLS // 8, 8).transpose(0, 2, 1, 3).reshape(-1, 64)

T_ATT = tiles_of(ATT); T_STEPS = tiles_of(STEPS)
TY, TX = STEPS.size // COLS // 8, COLS // 8

def probe_key(probe_steps):
    pr = probe_steps.reshape(TY, TX); pad = np.pad(pr, 1)
    return np.max(np.stack([pad[dy:dy + TY, dx:dx + TX] for dy in range(3) for dx in range(3)]), axis=0).ravel()

def order_by(key):
    return np.argsort(-key, kind='stable')

def simulate(order, two_ended=False, n_front_old=True, t_old=30.8, t_young=130.0, t_solo=30.0, t_tail=12.3,
             thr=16384, dt=0.02, seed=1, young_from_back=True, max_t=200):
    rng = np.random.default_rng(seed)
    q = T_ATT[order].ravel()   # attempts per item, queue order
    nq = q.size
    left = np.zeros((NS, 2, NL))
    item = -np.ones((NS, 2, NL), np.int64); tstart = np.zeros(q.size)
    front, back = 0, nq  # items [front, back) unclaimed
    t = 0.0; drained = None
    while t < max_t:
        idle = left <= 0
        if front < back:
            # refill: waves in random order
            cnt = idle.sum(axis=2)  # (NS,2)
            for slot in ((0, 1) if rng.random() < 0.5 else (1, 0)):
                c = cnt[:, slot]
                ws = np.flatnonzero(c)
                if not len(ws): continue
                ws = rng.permutation(ws)
                for s in ws:
                    if front >= back: break
                    k = int(c[s]); lanes = np.flatnonzero(idle[s, slot])
                    m = min(k, back - front)
                    if two_ended and slot == 1 and young_from_back:
                        vals = q[back - m:back]; item[s, slot, lanes[:m]] = np.arange(back - m, back); tstart[back-m:back] = t; back -= m
                    else:
                        vals = q[front:front + m]; item[s, slot, lanes[:m]] = np.arange(front, front + m); tstart[front:front+m] = t; front += m
                    left[s, slot, lanes[:m]] = vals
        if front >= back and drained is None:
            drained = t
        live = int((left > 0).sum())
        if drained is not None and live <= thr:
            rest = left[left > 0]
            if rest.size:
                w = np.unravel_index(np.argmax(left), left.shape); it = item[w]
                crit = dict(item=int(it), tile_rank=int(it)//64, slot=int(w[1]), start=round(float(tstart[it]),2), att=float(q[it]), rem=float(left[w]))
            else: crit = None
            return dict(crit=crit, drained=round(drained, 2), handoff=round(t, 2), end=round(t + (rest.max() if rest.size else 0) * t_tail * 1e-6, 2))
        alive = (left > 0).any(axis=2) | (front < back)  # (NS,2)
        us = np.empty((NS, 2))
        us[:, 0] = np.where(alive[:, 1], t_old, t_solo)
        us[:, 1] = np.where(alive[:, 0], t_young, t_solo)
        left -= (dt * 1e6 / us)[:, :, None] * (left > 0)
        t += dt
    return dict(timeout=True)

if __name__ == '__main__':
    import sys
    probe = T_STEPS[:, 27]
    key_cur = probe_key(np.minimum(probe, CAP))
    print('current order, one queue:', simulate(order_by(key_cur)), flush=True)
    print('current order, two-ended:', simulate(order_by(key_cur), two_ended=True), flush=True)
    key_true = probe_key(probe)   # the probe pixel's true length (upper bound of a probe)
    print('true probe length, two-ended:', simulate(order_by(key_true), two_ended=True), flush=True)
    key_tmax = T_ATT.max(1)
    print('tile max (oracle), two-ended:', simulate(order_by(key_tmax), two_ended=True), flush=True)
