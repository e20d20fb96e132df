"""The C ABI surface (CPU only, no compute calls): libgrt.so loads, exports every
function include/grt_api.h declares, and the ctypes mirror has the header's layout."""
import ctypes as C
import re
import subprocess

import pytest

from conftest import ROOT

HEADER = ROOT / "include" / "grt_api.h"


def declared_functions():
    text = HEADER.read_text()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    names = set(re.findall(r"\b(grt_[a-z0-9_]+)\s*\(", text))
    return sorted(names)


def test_every_declared_function_is_exported(grt):
    from gr_raytracer_amd import _lib as L

    lib = L.lib()
    names = declared_functions()
    assert len(names) >= 25
    missing = [n for n in names if not hasattr(lib, n)]
    assert not missing, missing
    assert sorted(L.EXPORTED_SYMBOLS) == names


def test_struct_layout_matches_header(grt, tmp_path):
    from gr_raytracer_amd import _lib as L

    structs = {"grt_scene_desc": L.SceneDesc, "grt_camera_desc": L.CameraDesc, "grt_texture_desc": L.TextureDesc,
               "grt_object_desc": L.ObjectDesc, "grt_global_opts": L.GlobalOpts,
               "grt_adaptive_config": L.AdaptiveConfig, "grt_stats": L.Stats, "grt_offsets": L.Offsets,
               "grt_aux_out": L.AuxOut, "grt_row_shard": L.RowShard,
               "grt_subsample_failures": L.SubsampleFailures}
    src = tmp_path / "sizes.c"
    body = "".join(f'  printf("{k} %zu\\n", sizeof({k}));\n' for k in structs)
    src.write_text(f'#include <stdio.h>\n#include "grt_api.h"\nint main(void) {{\n{body}  return 0;\n}}\n')
    exe = tmp_path / "sizes"
    subprocess.run(["gcc", "-std=c11", "-Wall", "-I", str(ROOT / "include"), str(src), "-o", str(exe)], check=True)
    out = subprocess.run([str(exe)], check=True, capture_output=True, text=True).stdout.split("\n")
    sizes = dict(line.split() for line in out if line)
    for k, cls in structs.items():
        assert int(sizes[k]) == C.sizeof(cls), (k, sizes[k], C.sizeof(cls))


def test_header_compiles_as_c_and_cpp(tmp_path):
    src = tmp_path / "h.c"
    src.write_text('#include "grt_api.h"\nint main(void) { return GRT_ABI_VERSION - 1; }\n')
    subprocess.run(["gcc", "-std=c99", "-Wall", "-Werror", "-I", str(ROOT / "include"), "-c", str(src), "-o",
                    str(tmp_path / "h.o")], check=True)
    subprocess.run(["g++", "-x", "c++", "-std=c++11", "-Wall", "-Werror", "-I", str(ROOT / "include"), "-c",
                    str(src), "-o", str(tmp_path / "h2.o")], check=True)


def test_missing_library_fails_loudly(monkeypatch, tmp_path):
    """No CPU fallback: a missing libgrt.so is an error, not a silent path."""
    from gr_raytracer_amd import _lib as L

    monkeypatch.setattr(L, "_lib", None)
    monkeypatch.setattr(L, "LIB_PATH", tmp_path / "nope.so")
    with pytest.raises(L.GrtError):
        L.lib()
