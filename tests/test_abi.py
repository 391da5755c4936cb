"""CPU tests of the drop-in boundary: the C-ABI library loads and exports every symbol that
include/raymarch.h declares; non-compute entry points behave. No kernels run here."""
import ctypes
import os
import re

import numpy as np
import pytest

from conftest import ROOT

HEADER = os.path.join(ROOT, "include", "raymarch.h")


def header_functions():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(rm_[a-z0-9_]+)\s*\(", text)))


@pytest.fixture(scope="module")
def native():
    from burn_raymarching_amd import _build, native as nat
    _build.build_lib()
    return nat


def test_header_declares_expected_api():
    fns = header_functions()
    for required in ("rm_render_diff", "rm_render_diff_backward", "rm_train_step", "rm_render_diff_camera",
                     "rm_train_step_camera", "rm_optimizer_step", "rm_scene_activate", "rm_create"):
        assert required in fns


def test_library_exports_every_header_symbol(native):
    lib = ctypes.CDLL(native.LIB_PATH)
    missing = [f for f in header_functions() if not hasattr(lib, f)]
    assert not missing, missing


def test_python_binding_covers_header(native):
    assert sorted(native.SIGNATURES) == header_functions()


def test_header_constants_match_binding(native):
    """Every #define of include/raymarch.h that the Python binding mirrors has the same value."""
    text = open(HEADER).read()
    defines = dict(re.findall(r"#define\s+(RM_[A-Z0-9_]+)\s+(-?\d+)", text))
    mirrored = [k for k in defines if hasattr(native, k)]
    assert {"RM_MARCH_SKIP_ESCAPED", "RM_MARCH_PER_RAY_ORIGIN", "RM_MAX_VIEWS_PER_CALL"} <= set(mirrored)
    for k in mirrored:
        assert getattr(native, k) == int(defines[k]), k


def test_version_and_defaults(native):
    lib = native.lib()
    assert b"gfx950" in lib.rm_version()
    m = native.RmMarch()
    lib.rm_march_default(ctypes.byref(m))
    assert m.steps == 40 and m.smooth_k == 32.0  # renderer_diff.rs:22, train.rs:131
    assert m.normal_eps == np.float32(1e-4) and m.color_sharpness == 10.0 and m.mask_sharpness == 15.0
    assert m.flags == 0  # RM_MARCH_SKIP_ESCAPED is opt-in


def test_null_context_is_rejected(native):
    lib = native.lib()
    assert lib.rm_render_diff(None, None, None, 0, None, None, None, None) == 1  # RM_ERR_INVALID_ARG
    assert lib.rm_last_error(None) == b"NULL context"
    assert lib.rm_create(0, None, None) == 1
    # the sampled steps (rm_train_step_sampled, rm_train_iteration) check the context first
    assert lib.rm_train_step_sampled(None, None, None, None, 1, None, 0, 0, 0, 0, 0, 0, 0.0, 1.0, None, None, None,
                                     None) == 1
    assert lib.rm_train_iteration(None, None, None, None, 1, None, 0, 0, 0, 0, 0, 0, 0.0, 1.0, None, None, None, None,
                                  None, None, 1, 1, 0.01, 0.0, 0, None, None) == 1


def test_packed_views(native):
    lib = native.lib()
    s = native.RmScene()
    base = 0x10000
    lib.rm_scene_from_packed(ctypes.c_void_p(base), 5, ctypes.byref(s))
    assert (s.centers, s.colors, s.radius, s.light_dir, s.ambient, s.num_spheres) == (
        base, base + 4 * 15, base + 4 * 30, base + 4 * 35, base + 4 * 38, 5)


def test_built_for_gfx950(native):
    data = open(native.LIB_PATH, "rb").read()
    assert b"gfx950" in data


def test_shipped_library_matches_sources(native):
    """The in-tree libraymarch_hip.so (the one that travels to the GPU box) was built from the
    kernel sources in this tree: rm_version() carries their sha256 prefix (_build.py)."""
    from burn_raymarching_amd import _build
    if os.environ.get("RM_LIB_PATH"):
        pytest.skip("RM_LIB_PATH names another library")
    want = _build.source_hash()
    assert native.lib().rm_version().decode().endswith("src " + want)
    assert _build.lib_source_hash(native.LIB_PATH) == want


def test_shipped_host_binaries_match_sources():
    """librm_host.so and rm_train (they also travel prebuilt to the GPU box) carry the sha256
    prefix of the sources they were built from, as libraymarch_hip.so does (_build.py)."""
    import subprocess
    from burn_raymarching_amd import _build, host
    if os.environ.get("RM_LIB_PATH") or os.environ.get("RMH_LIB_PATH"):
        pytest.skip("RM_LIB_PATH / RMH_LIB_PATH name other libraries")
    want_host = _build.source_hash(_build.HOST_SOURCES)
    assert _build.lib_source_hash(_build.HOST_LIB, _build.HOST_TAG) == want_host
    assert host.lib().rmh_version().decode().endswith("src " + want_host)
    want_exe = _build.source_hash(_build.EXE_SOURCES)
    assert _build.lib_source_hash(_build.EXE, _build.EXE_TAG) == want_exe
    out = subprocess.run([_build.EXE, "--version"], capture_output=True, text=True, check=True).stdout.split("\n")
    assert out[0] == "rm_train src " + want_exe and out[1].endswith("src " + want_host), out
