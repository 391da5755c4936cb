"""CPU guards on the kernel sources for the bit-level pins of DESIGN.md §5.3.

The reference loop's trajectory (tests/test_gpu_trajectory.py) once changed with edits meant to be
bit-identical because the light-direction gradient was compiled with FP contraction on, so its
fusion followed the surrounding code (profiles/r07a_r06ao_cause.txt). These tests keep the helpers
that feed the trajectory -- the light-direction unit vector and gradient, the activation, the
repulsion rows and the optimizer's two halves -- compiled with contraction off, and keep every
light-direction gradient (the general kernel's reductions and the small kernel's final block)
going through the one helper. A GPU run is still what pins the bits (test_gpu_trajectory.py);
these catch the source change that would move them before it reaches the GPU.
"""
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "burn_raymarching_amd", "csrc")


def _src(name):
    with open(os.path.join(CSRC, name)) as f:
        return f.read()


def _body(src, signature):
    """The text of the function whose definition starts with `signature`, up to its closing brace."""
    i = src.index(signature)
    j = src.index("{", i)
    depth = 0
    for k in range(j, len(src)):
        if src[k] == "{":
            depth += 1
        elif src[k] == "}":
            depth -= 1
            if depth == 0:
                return src[j:k + 1]
    raise AssertionError(f"unbalanced braces after {signature}")


@pytest.mark.parametrize("signature", [
    "__device__ __forceinline__ float light_unit(",
    "__device__ __forceinline__ float light_grad(",
    "__device__ __forceinline__ float activate_elem(",
    "__device__ __forceinline__ void repulsion_row(",
    "__device__ __forceinline__ ElemPre optimizer_pre(",
    "__device__ __forceinline__ void optimizer_apply(",
])
def test_trajectory_helpers_compile_without_contraction(signature):
    body = _body(_src("rm_kernels.hip"), signature)
    first = body.split("\n", 2)[1].strip()
    assert first == "#pragma clang fp contract(off)", f"{signature} must open with contraction off"


def test_light_direction_gradient_has_one_definition():
    """Every light-direction gradient is light_grad's: no kernel forms (r - ln proj) / len itself."""
    for name in ("rm_kernels.hip", "rm_small.h"):
        src = _src(name)
        # the Jacobian of l / |l| written out anywhere but in light_grad
        body = _body(src, "__device__ __forceinline__ float light_grad(") if "float light_grad(" in src else ""
        rest = src.replace(body, "")
        assert not re.search(r"-\s*\w+\s*\*\s*proj\s*\)\s*/", rest), name
    assert "light_grad(" in _src("rm_small.h")
