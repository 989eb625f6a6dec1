"""The measured hot kernels' machine code is pinned (tools/pin_codegen.py):
the C3 headline SpMM moved 7 % with an unrelated argument-list change
(DESIGN.md §4.1), so any codegen change must be re-measured on the GPU and
re-pinned (python tools/pin_codegen.py --write) rather than slip in.  CPU
test: hipcc cross-compiles the sources with the library's flags."""
import json
import os
import shutil
import sys

import pytest

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
sys.path.insert(0, os.path.join(ROOT, "tools"))


@pytest.mark.skipif(shutil.which(os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")) is None, reason="hipcc absent")
def test_hot_kernel_codegen_matches_pins():
    import pin_codegen

    with open(pin_codegen.PINS) as f:
        pins = json.load(f)
    now = pin_codegen.compute()
    assert set(now) == set(pins)
    for name, p in pins.items():
        assert now[name]["sha256"] == p["sha256"], (
            f"{p['what']}: machine code changed ({p['instructions']} -> {now[name]['instructions']} instructions); "
            "re-measure it on the GPU, then re-pin with python tools/pin_codegen.py --write")
