"""Price the exactness tax: parity of an experimental libgrt build
against the oracle, on the whole-frame samples of tests/test_gpu_frames.py.

Run with GRT_LIB=variants/<name>/libgrt.so GRT_LIB_ALLOW_MISSING=1 on a GPU box.  For
each config the GPU frame (C1 whole; C2 20 000 and C3 5 625 stratified pixels of the
full frame; C4 1 024 pixels at the pixel centre, offsets mode) is compared with the
oracle (the reference algorithm, glibc libm):

  exact      colour (f64), class, status, stop reason and step count bit-equal
  within     colour within 1e-4 relative per channel and class equal (the north-star bar)
  sensitive  among the pixels outside the bar: moved by one of the oracle's own last-ulp
             libm probes (tests/test_gpu_parity.py PROBES)
  robust_wrong  outside the bar and not moved by any probe: a real parity failure

Prints one JSON line per config."""
import json
import os
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "oracle"), str(ROOT / "tests")]

import gr_raytracer_amd as g  # noqa: E402
import pyoracle as O  # noqa: E402
from conftest import c2_opts, c3_opts, c4_opts, host_scene  # noqa: E402
from test_gpu_frames import oracle_pixels, stratified  # noqa: E402
from test_gpu_parity import PROBES, agree, gpu_scene  # noqa: E402


def classify(desc, cols, ri, ci, got, ref):
    ok = agree(got["xyza64"], got["ray_class"], ref) & (got["status"] == ref["status"])
    exact = (np.all(got["xyza64"] == ref["xyza"], axis=1) & (got["ray_class"] == ref["ray_class"]) &
             (got["status"] == ref["status"]) & (got["stop"] == ref["stop"]) & (got["steps"] == ref["steps"]))
    suspect = np.where(~ok)[0]
    moved = np.zeros(suspect.size, bool)
    if suspect.size:
        sub = {k: (v[suspect] if isinstance(v, np.ndarray) else v) for k, v in ref.items()}
        try:
            for mode in PROBES:
                O.lib().oracle_set_libm_perturbation(mode)
                p = oracle_pixels(O, desc, cols, ri[suspect], ci[suspect])
                moved |= ~agree(p["xyza"], p["ray_class"], sub) | (p["status"] != sub["status"])
        finally:
            O.lib().oracle_set_libm_perturbation(0)
    n = len(ok)
    return {"pixels": n, "exact": int(exact.sum()), "within_1e-4": int(ok.sum()), "outside": int(suspect.size),
            "sensitive": int(moved.sum()), "robust_wrong": int((~moved).sum()),
            "robust_wrong_examples": [[int(ri[k]), int(ci[k])] for k in suspect[~moved][:5]],
            "frac_exact": float(exact.mean()), "frac_within": float(ok.mean())}


def frame(name, toml, opts, cell, seed):
    hs = host_scene(g, toml, opts)
    sc = gpu_scene(g, hs)
    rows, cols = sc.rows, sc.cols
    t0 = time.time()
    full = sc.render_pixels(0, 0, rows, cols)
    if cell == 1:
        R, Cc = np.meshgrid(np.arange(rows), np.arange(cols), indexing="ij")
        ri, ci = R.ravel(), Cc.ravel()
    else:
        ri, ci = stratified(rows, cols, cell, seed)
    k = ri * cols + ci
    got = {"xyza64": full.xyza64[k], "ray_class": full.ray_class[k], "status": full.status[k],
           "stop": full.stop_reason[k], "steps": full.steps[k]}
    ref = oracle_pixels(O, hs.desc, cols, ri, ci)
    out = {"config": name, "kernel_ms": full.stats["kernel_ms"], "accepted": full.stats["accepted_steps"]}
    out.update(classify(hs.desc, cols, ri, ci, got, ref))
    out["wall_s"] = round(time.time() - t0, 1)
    return out


def c4():
    hs = host_scene(g, "kerr.toml", c4_opts(g))
    sc = gpu_scene(g, hs)
    cols = sc.cols
    ri, ci = stratified(sc.rows, cols, 128, 13)
    pix = (ri * cols + ci).astype(np.uint32)
    half = np.full(len(pix), 0.5)
    t0 = time.time()
    r = sc.render_pixels(offsets=(pix, half, half))
    got = {"xyza64": r.xyza64, "ray_class": r.ray_class, "status": r.status, "stop": r.stop_reason, "steps": r.steps}
    ref = oracle_pixels(O, hs.desc, cols, ri, ci)
    out = {"config": "C4 1024 px"}
    out.update(classify(hs.desc, cols, ri, ci, got, ref))
    out["wall_s"] = round(time.time() - t0, 1)
    return out


def c5_save(path):
    """C5 (stock adaptive 4x4) frame of this library, saved for c5_compare."""
    hs = host_scene(g, "schwarzschild.toml", c2_opts(g))
    sc = gpu_scene(g, hs)
    r = sc.render_section_ex(adaptive=hs.adaptive)
    np.savez(path, xyza64=r.xyza64, cls=r.ray_class, n_sel=r.n_supersampled)
    return {"config": "C5 saved", "path": path, "n_supersampled": r.n_supersampled, "kernel_ms": r.stats["kernel_ms"]}


def c5_compare(a, b):
    """Pixels of two C5 frames outside 1e-4 (relative per channel) of each other."""
    from test_gpu_parity import within

    A, B = np.load(a), np.load(b)
    ok = within(B["xyza64"], A["xyza64"]) & (A["cls"] == B["cls"])
    return {"config": "C5 compare", "pixels": int(ok.size), "within_1e-4": int(ok.sum()), "outside": int((~ok).sum()),
            "n_supersampled": [int(A["n_sel"]), int(B["n_sel"])],
            "exact": int(np.all(A["xyza64"] == B["xyza64"], axis=1).sum())}


if __name__ == "__main__":
    if sys.argv[1:2] == ["C5save"]:
        print(json.dumps(c5_save(sys.argv[2])), flush=True)
        sys.exit(0)
    if sys.argv[1:2] == ["C5compare"]:
        print(json.dumps(c5_compare(sys.argv[2], sys.argv[3])), flush=True)
        sys.exit(0)
    which = sys.argv[1:] or ["C1", "C2", "C3", "C4"]
    lib = os.environ.get("GRT_LIB", "in-tree")
    for w in which:
        if w == "C1":
            res = frame("C1 256^2 whole", "euclidean.toml", g.GlobalOpts(width=256, height=256), 1, 0)
        elif w == "C2":
            res = frame("C2 20000 px", "schwarzschild.toml", c2_opts(g), 10, 11)
        elif w == "C3":
            res = frame("C3 5625 px", "kerr-bl.toml", c3_opts(g), 20, 12)
        else:
            res = c4()
        res["lib"] = lib
        print(json.dumps(res), flush=True)
