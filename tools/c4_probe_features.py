"""Which state of a capped probe ray predicts the length of its tile's rays?  For the C4
shard 2/8 (band 16): the oracle (test infrastructure) integrates every probe pixel whose
ray is still going at the probe cap, and records its Kerr-Schild radius at the cap and
before it; the true per-ray step counts come from a GPU record (tools/c4_ray_times.py).
Prints the log-log correlation of each candidate key with the probe pixel's own count and
how many of the tiles holding a ray past 8e5 steps each key ranks first.

usage: python tools/c4_probe_features.py RECORD.npz"""
import sys, numpy as np, multiprocessing as mp
sys.path.insert(0,'/root/repo'); sys.path.insert(0,'/root/repo/oracle')
import gr_raytracer_amd as g, pyoracle as O
from pathlib import Path
ROOT=str(Path(__file__).resolve().parents[1])
REC=np.load(sys.argv[1]) if __name__=='__main__' else None
t4=None; probe=None
CAP=20670
TX=512
def shard_row(lr, band=16, shard=2, n=8): return ((lr//band)*n+shard)*band + lr%band
def init():
    global _hs, _desc
    opts=g.GlobalOpts(width=4096,height=4096,camera_position=(-10.0,0.0,-0.5),theta=1.52,psi=-1.57,max_steps=CAP)
    _hs=g.HostScene(ROOT+'/tests/golden/scenes/kerr.toml',opts,ROOT+'/tests/golden')
    _desc=_hs.desc
def ksr(X,a):
    RHO=(X*X).sum(-1); return np.sqrt(0.5*(RHO-a*a+np.sqrt((RHO-a*a)**2+4*a*a*X[...,2]**2)))
def work(t):
    tr,tc=divmod(int(t),TX)
    m=O.camera_ray(_desc,shard_row(tr*8+3),tc*8+3)
    pos=np.array(_desc.camera.position[:])
    tr_,stop,status=O.integrate_ray(_desc,pos,m,max_out=CAP+10)
    a=_desc.a
    R=ksr(tr_[:,2:5],a)
    return (int(t), len(tr_), R[-1], R[-1001], R[-4097], tr_[-1,1], tr_[-1,0], tr_[-1,0]-tr_[-2,0])
def tiles(v, cols=4096):
    rows = v.size // cols
    return v.reshape(rows // 8, 8, cols // 8, 8).transpose(0, 2, 1, 3).reshape(-1, 64)


if __name__=='__main__':
    t4 = tiles(REC['steps'].astype(np.float64))
    probe = t4[:, 27]
    cap_t = np.flatnonzero(probe >= CAP)
    with mp.Pool(8, initializer=init) as p:
        F = np.array(p.map(work, cap_t, chunksize=8), dtype=np.float64)
    t = F[:, 0].astype(int); r, r4k = F[:, 2], F[:, 4]
    true = probe[t]; big = t4[t].max(1) >= 8e5
    rstop = 0.5 + np.sqrt(0.25 - 0.499 ** 2) + 1e-4  # kerr.toml: r_+ + horizon_epsilon
    for name, v in (("r - r_stop", r - rstop), ("(r - r_stop) / rate over 4096 steps", (r - rstop) / np.maximum((r4k - r) / 4096, 1e-30))):
        o = np.argsort(-v)
        print(f"{name}: log-log corr {np.corrcoef(np.log(np.abs(v) + 1e-300), np.log(true))[0, 1]:.3f}, "
              f"big tiles in the top 311 / 1024: {big[o[:311]].sum()} / {big[o[:1024]].sum()} of {big.sum()}")
