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
               "grt_subsample_failures": L.SubsampleFailures, "grt_frame_out": L.FrameOut,
               "grt_multi_report": L.MultiReport}
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


def test_library_from_other_sources_is_refused(grt, tmp_path):
    """The source stamp (grt_source_hash, Makefile) binds libgrt.so to its checkout: a
    library whose stamp differs from the checkout's source hash raises GrtError."""
    import os
    import sys

    from gr_raytracer_amd import _lib as L
    from gr_raytracer_amd.source_hash import source_hash

    want = source_hash()
    assert L.lib().grt_source_hash().decode() == want  # this build matches its checkout
    data = L.LIB_PATH.read_bytes()
    assert data.count(want.encode()) == 1
    other = ("0" if want[0] != "0" else "1") + want[1:]
    patched = tmp_path / "libgrt.so"
    patched.write_bytes(data.replace(want.encode(), other.encode()))
    code = ("import sys; sys.path.insert(0, sys.argv[1]); from gr_raytracer_amd import _lib as L\n"
            "try:\n    L.lib()\nexcept L.GrtError as e:\n    print('refused:', e); sys.exit(3)\nsys.exit(0)")
    env = {k: v for k, v in os.environ.items() if k != "GRT_LIB_ALLOW_MISSING"}
    env["GRT_LIB"] = str(patched)
    r = subprocess.run([sys.executable, "-c", code, str(ROOT)], env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 3, r.stdout + r.stderr
    assert "built from other sources" in r.stdout


def test_kernel_symbols_cover_every_unit(grt):
    """The kernel-symbol and code-hash helpers (PMC summaries record a kernel's own code
    hash) read every translation unit's gfx950 code object: the main unit's kernels and
    the KerrBL unit's (geodesic_kerr_bl.hip, namespace grt::kerr_bl)."""
    from gr_raytracer_amd import _lib as L

    syms = L.kernel_symbols()
    assert any(s.startswith("_ZN3grt16integrate_kernelILi1ELb0EE") for s in syms)
    assert any(s.startswith("_ZN3grt7kerr_bl16integrate_kernelILi3ELb0EE") for s in syms)
    assert not any(s.startswith("_ZN3grt16integrate_kernelILi3ELb0EE") for s in syms)  # KerrBL left the main unit
    main = L.kernel_symbol("grt::integrate_kernel<1, false>")
    bl = L.kernel_symbol("grt::kerr_bl::integrate_kernel<3, false>")
    assert main != bl and len(L.kernel_code_sha256(main)) == 64 and len(L.kernel_code_sha256(bl)) == 64
    assert L.kernel_code_sha256(main) != L.kernel_code_sha256(bl)
