"""CPU-side checks of the drop-in boundary (no GPU needed): the C-ABI library loads and exports
every symbol include/jsrt.h declares, the blob exporter/format round-trips, and host helpers behave."""
import ctypes
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def lib():
    from jsraytracer_amd import build as jb
    jb.build()
    from jsraytracer_amd import _native
    return _native.lib()


def _declared(header):
    txt = open(os.path.join(ROOT, "include", header)).read()
    return sorted(set(re.findall(r"\b(jsrt_[a-z_]+)\s*\(", txt)) - {"jsrt_progress_fn"})


def test_header_symbols_exported(lib):
    from jsraytracer_amd import _native
    declared = _declared("jsrt.h")
    assert set(declared) == set(_native.EXPORTS)
    out = subprocess.run(["nm", "-D", "--defined-only", _native.LIB_PATH], capture_output=True, text=True).stdout
    mesh = _declared("jsrt_mesh.h")
    assert set(mesh) == set(_native.MESH_EXPORTS)
    js = _declared("jsrt_json.h")
    assert set(js) == set(_native.JSON_EXPORTS)
    for sym in declared + mesh + js:
        assert re.search(rf"\bT {sym}$", out, re.M), f"{sym} not exported"
        assert hasattr(lib, sym)


def test_library_is_gfx950(lib):
    from jsraytracer_amd import _native
    out = subprocess.run(["/opt/rocm/lib/llvm/bin/clang-offload-bundler", "--list", "--type=o",
                          f"--input={_native.LIB_PATH}"], capture_output=True, text=True)
    listing = out.stdout + out.stderr
    if out.returncode != 0 or not listing.strip():  # fall back to scanning the embedded code object
        listing = open(_native.LIB_PATH, "rb").read().decode("latin-1")
    assert "gfx950" in listing


def test_abi_version_and_helpers(lib):
    assert lib.jsrt_abi_version() == 4
    from jsraytracer_amd import owned_columns
    assert owned_columns(10, 0, 1) == 10
    assert owned_columns(10, 1, 3) == 3            # 1, 4, 7
    assert owned_columns(10, 3, 3) == 3            # 3, 6, 9 (reference allows offset >= delt)
    assert owned_columns(40, 1, 2, 8) == 16        # blocks 1 and 3 of 8 columns
    assert owned_columns(36, 1, 2, 8) == 16        # blocks 1 (8..15) and 3 (24..31)
    assert owned_columns(36, 0, 2, 8) == 20        # blocks 0, 2 and the partial block 4 (32..35)


def test_no_device_raises_not_falls_back(lib):
    import jsraytracer_amd as jr
    from oracle import pyoracle
    if lib.jsrt_device_count() > 0:
        pytest.skip("a GPU is visible")
    with pytest.raises(jr.JsrtError):
        jr.Scene(pyoracle.golden_scene("ASimpleScene"))


def test_scene_header_reader():
    import jsraytracer_amd as jr
    from oracle import pyoracle
    h = jr.scene_header(pyoracle.golden_scene("cornell_box_path"))
    assert h == {"kind": 1, "spp": 128, "max_depth": 8, "width": 600, "height": 600}


def test_build_id_ties_library_to_tree(lib, tmp_path):
    """jsrt_build_id is the hash of the sources, flags and defines the library was built from; the
    bindings refuse a library whose id is not this tree's (a stale .so shipped to the GPU box)."""
    from jsraytracer_amd import _native
    from jsraytracer_amd import build as jb
    assert lib.jsrt_build_id().decode() == jb.build_id() == _native.build_id()
    assert jb.build_id(["-DJSRT_X=1"]) != jb.build_id()  # a variant's defines change it
    # a copy of one source with an edit: the id of that tree differs
    src = open(os.path.join(jb.CSRC, "render.hip")).read()
    old = jb.CSRC
    try:
        d = tmp_path / "csrc"
        d.mkdir()
        for f in os.listdir(old):
            (d / f).write_text(open(os.path.join(old, f)).read())
        (d / "render.hip").write_text(src + "\n// edit\n")
        jb.CSRC = str(d)
        assert jb.build_id() != _native.build_id()
    finally:
        jb.CSRC = old


def test_bench_exits_nonzero_on_parity_failure():
    """bench.py turns a timed frame that differs from the oracle into a non-zero exit status (the line is
    still printed, with parity.pass false), and refuses to time with JSRT_* knobs set unless --ab."""
    import numpy as np
    import sys
    sys.path.insert(0, ROOT)
    import bench
    H, W = 8, 12
    rng = np.random.default_rng(1)
    orgba = rng.integers(0, 256, (H, W, 4), dtype=np.uint8)
    ocol = rng.random((H, W, 4), dtype=np.float32)
    ok = bench.parity(orgba.copy(), ocol.copy(), (ocol, orgba, 1, 3))
    assert ok["pass"] and bench.exit_status(ok) == 0
    broken = orgba.copy()
    broken[5, 4, 1] ^= 1  # one byte of one owned column (1, 4, 7, 10)
    bad = bench.parity(broken, ocol.copy(), (ocol, orgba, 1, 3))
    assert not bad["pass"] and bad["rgba8_pixels_differing"] == 1 and bench.exit_status(bad) != 0
    assert bench.exit_status(None) == 0  # --no-parity
    env = dict(os.environ, JSRT_DUAL="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--steps", "1"], env=env,
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 2 and "--ab" in r.stderr and not r.stdout


def test_params_layout_and_mode_names():
    """jsrt_params (ABI 4): mode and device_mask take two of round 5's four reserved words, so the struct keeps its
    size; the host's mode names map to JSRT_MODE_* and an unknown name is refused before any call."""
    import ctypes

    import jsraytracer_amd as jr
    from jsraytracer_amd import _native
    from jsraytracer_amd.renderer import MODE_FAST, MODE_STRICT, mode_code
    P = _native.Params
    assert ctypes.sizeof(P) == 72
    assert P.mode.offset == 56 and P.device_mask.offset == 60 and P.reserved.offset == 64
    assert (mode_code(None), mode_code("strict"), mode_code("fast"), mode_code(1)) == (MODE_STRICT, MODE_STRICT, MODE_FAST, 1)
    with pytest.raises(jr.JsrtError):
        mode_code("turbo")
