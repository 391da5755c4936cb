"""burn_raymarching_amd -- MI355X-native differentiable SDF-sphere raymarcher.

The hot path of kokutoupan/burn_raymarching (render_diff, renderer_diff.rs:6-91, and its
burn-autodiff backward) runs as hand-written gfx950 HIP kernels behind the C ABI of
include/raymarch.h (lib/libraymarch_hip.so). This package is the host-side mirror used by
tests and the benchmark; csrc/host/ holds the C++ train-loop host.
"""
from .native import LIB_PATH, RaymarchError, lib  # noqa: F401

__version__ = "0.1.0"


def __getattr__(name):
    # Torch-facing modules are imported lazily so that `import burn_raymarching_amd` (and the
    # C-ABI symbol checks) work without initialising the GPU.
    if name in ("render", "model"):
        import importlib
        return importlib.import_module(f".{name}", __name__)
    raise AttributeError(name)
