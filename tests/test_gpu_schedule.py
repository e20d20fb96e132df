"""The Kerr-Schild work-order probe on quads (marker `gpu`): probe_quad_kernel splits each
probe ray's RHS over the 4 lanes of a quad (rhs_ks_quad, as the tail kernel does) and must
give the same keys as probe_kernel's one lane per ray, bit for bit, on the C4 layout's row
bands (kerr.toml, the C4 camera, cyclic 16-row bands; a reduced frame).  The keys only
order the tile queue, never an output; equal keys mean an unchanged queue."""
import ctypes as C

import numpy as np
import pytest

from conftest import host_scene

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("size,shard", [(512, 2), (768, 5)])
def test_probe_keys_on_quads_equal_one_lane_keys(grt, gpu, size, shard):
    import bench
    from gr_raytracer_amd import _lib as L

    opts = bench.c4_opts(grt, size)
    hs = host_scene(grt, "kerr.toml", opts)
    scene = grt.Scene(hs.desc_ptr(), keepalive=hs)
    lib = L.lib()
    sh = L.RowShard(16, shard, 8)
    rows = lib.grt_shard_row_count(size, C.byref(sh))
    n_tiles = ((rows + 7) // 8) * ((size + 7) // 8)
    fn = lib.grt_debug_probe_keys
    fn.restype = C.c_int
    fn.argtypes = [C.c_void_p, C.c_int, C.POINTER(L.RowShard), C.c_int, C.c_void_p, C.c_uint64]
    keys = {}
    for quad in (0, 1):
        k = np.zeros(n_tiles, np.uint32)
        L.check(fn(scene._s, gpu, C.byref(sh), quad, k.ctypes.data, n_tiles), "grt_debug_probe_keys")
        keys[quad] = k
    assert np.array_equal(keys[0], keys[1])
    cap = int(min(32768, max(4096, 0.3 * 15000)))  # api.hip probe_cap for max_radius 15000
    assert (keys[0] > 0).all()
    assert (keys[0] >= cap).any() and (keys[0] < cap).any()  # capped probes and finished ones
    assert (keys[0] == cap - 1).any()  # probes that ended outward-bound (probe_escaped)
