"""Exponent-plane map of the range-free divisions and square root against the compiler's
(grt_debug_arith_map, geodesic.hip arith_map_kernel): saves the flag maps to OUT.npz and
prints, per function, which exponent cells differ.  Usage: tools/arith_map.py OUT [SAMPLES]"""
import ctypes as C
import json
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
from gr_raytracer_amd import _lib as L  # noqa: E402


def arith_map(samples=16, seed=0x5EED, device=0):
    lib = L.lib()
    fn = lib.grt_debug_arith_map
    fn.restype = C.c_int
    fn.argtypes = [C.c_int, C.c_uint32, C.c_uint64, C.c_void_p, C.c_void_p, C.c_void_p]
    m = np.zeros(2047 * 2047, np.uint8)
    z = np.zeros(2047, np.uint8)
    s = np.zeros(2047, np.uint8)
    L.check(fn(device, samples, seed, m.ctypes.data, z.ctypes.data, s.ctypes.data), "grt_debug_arith_map")
    return m.reshape(2047, 2047), z, s


def summary(m, z, s):
    ex, ey = np.meshgrid(np.arange(2047) - 1023, np.arange(2047) - 1023, indexing="ij")  # unbiased (-1023: subnormal)
    out = {}
    for bit, name in ((1, "div_inrange"), (2, "div2_inrange"), (4, "div_fx")):
        bad = (m & bit) != 0
        gap = ex - ey
        out[name] = {
            "cells": int(bad.sum()),
            "min_gap_bad": int(gap[bad].min()) if bad.any() else None,
            "max_gap_bad": int(gap[bad].max()) if bad.any() else None,
            # numerators / denominators of differing cells with a moderate quotient exponent
            "bad_x_exps_at_gap0": sorted(set(ex[bad & (gap == 0)].tolist()))[:8] + sorted(set(ex[bad & (gap == 0)].tolist()))[-8:],
            "clean_box": clean_box(bad, ex, ey),
        }
    out["div_fx_zero_numerator_bad_y_exps"] = (np.nonzero(z & 8)[0] - 1023).tolist()
    out["sqrt_fx_bad_x_exps"] = (np.nonzero(s & 16)[0] - 1023).tolist()
    return out


def clean_box(bad, ex, ey):
    """Largest k such that no cell with |e_x|, |e_y|, |e_x - e_y| <= k differs."""
    for k in range(1023, -1, -1):
        box = (np.abs(ex) <= k) & (np.abs(ey) <= k) & (np.abs(ex - ey) <= k)
        if not (bad & box).any():
            return k
    return -1


if __name__ == "__main__":
    out = Path(sys.argv[1])
    samples = int(sys.argv[2]) if len(sys.argv) > 2 else 16
    m, z, s = arith_map(samples)
    out.parent.mkdir(parents=True, exist_ok=True)
    np.savez_compressed(out, map=m, zmap=z, smap=s)
    print(json.dumps(summary(m, z, s)), flush=True)
