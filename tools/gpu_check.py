"""First-contact GPU check: parity of a crop vs the oracle + full-frame timing."""
import sys, time
from pathlib import Path
ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT)); sys.path.insert(0, str(ROOT / "oracle"))
import numpy as np
import gr_raytracer_amd as g
import pyoracle as O

def parity(name, toml, opts, rect, threads=16):
    hs = g.HostScene(str(ROOT / "tests/golden/scenes" / toml), opts, str(ROOT / "tests/golden"))
    sc = g.Scene(hs.desc_ptr(), keepalive=hs)
    r0, c0, nr, nc = rect
    t = time.time()
    gpu = sc.render_pixels(r0, c0, nr, nc)
    tg = time.time() - t
    cpu = O.render_pixels(hs.desc, r0, c0, nr, nc, threads=threads)
    ref, got = cpu["xyza"], gpu.xyza64
    exact = np.all(ref == got, axis=1)
    rel = np.abs(got - ref) <= 1e-4 * np.maximum(np.abs(ref), 1e-6)
    ok = np.all(rel, axis=1)
    cls_eq = gpu.ray_class == cpu["ray_class"]
    steps_eq = gpu.steps == cpu["steps"]
    print(f"[{name}] {nr}x{nc}: bit-exact {exact.mean():.4f}  within-1e-4 {ok.mean():.4f}  class-eq {cls_eq.mean():.4f} "
          f"steps-eq {steps_eq.mean():.4f}  gpu {tg:.2f}s (kernel {gpu.stats['kernel_ms']:.1f} ms) "
          f"cpu {cpu['wall_s']:.2f}s  gpu_acc {gpu.stats['accepted_steps']} cpu_acc {cpu['accepted']}", flush=True)
    bad = np.where(~ok)[0][:5]
    for i in bad:
        print("   pixel", i, "gpu", got[i], "cpu", ref[i], "cls", gpu.ray_class[i], cpu["ray_class"][i],
              "stop", gpu.stop_reason[i], cpu["stop"][i], "steps", gpu.steps[i], cpu["steps"][i],
              "status", gpu.status[i], cpu["status"][i])
    return sc

def full(name, toml, opts):
    hs = g.HostScene(str(ROOT / "tests/golden/scenes" / toml), opts, str(ROOT / "tests/golden"))
    sc = g.Scene(hs.desc_ptr(), keepalive=hs)
    for it in range(2):
        t = time.time()
        r = sc.render_pixels(0, 0, opts.height, opts.width, aux=False)
        dt = time.time() - t
        st = r.stats
        print(f"[{name} full {opts.width}x{opts.height}] wall {dt:.2f}s kernel {st['kernel_ms']:.1f} ms "
              f"accepted {st['accepted_steps']:.3e} attempts {st['attempts']:.3e} rays {st['rays']} "
              f"-> {st['accepted_steps']/(st['kernel_ms']*1e-3):.3e} steps/s  overflows {st['hit_overflows']}",
              flush=True)

if __name__ == "__main__":
    print("devices", g.device_count())
    c2 = dict(width=1500, height=1500, camera_position=(-16.0, 0.0, 3.5), theta=-3.142, max_steps=100000)
    parity("C2", "schwarzschild.toml", g.GlobalOpts(**c2), (700, 700, 64, 64))
    parity("C2-edge", "schwarzschild.toml", g.GlobalOpts(**c2), (1000, 600, 32, 32))
    c3 = dict(width=1500, height=1500, camera_position=(-10, 0, -0.5), theta=-3.14159, max_steps=1000000)
    parity("C3", "kerr-bl.toml", g.GlobalOpts(**c3), (700, 700, 32, 32))
    c4 = dict(width=4096, height=4096, camera_position=(-10, 0, -0.5), theta=1.52, psi=-1.57, max_steps=1000000)
    parity("C4", "kerr.toml", g.GlobalOpts(**c4), (2000, 2000, 16, 16))
    c1 = dict(width=256, height=256)
    parity("C1", "euclidean.toml", g.GlobalOpts(**c1), (100, 100, 32, 32))
    full("C2", "schwarzschild.toml", g.GlobalOpts(**c2))
    full("C3", "kerr-bl.toml", g.GlobalOpts(**c3))
