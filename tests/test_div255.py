"""The kernels' division-free /255 (div255 in csrc/vss_kernels.hip, the a3 step
`.div(255.0)` of frameProcessorTest.ts:81) equals the IEEE division for every
float the resize can produce: exhaustive over all floats in [0, 256]."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("gcc") is None, reason="needs gcc")
def test_div255_exhaustive(tmp_path):
    exe = str(tmp_path / "div255_check")
    subprocess.run(["gcc", "-O2", "-mfma", "-fopenmp", os.path.join(ROOT, "tools", "div255_check.c"),
                    "-o", exe, "-lm"], check=True)
    out = subprocess.run([exe], capture_output=True, text=True, timeout=600)
    assert out.returncode == 0, out.stdout
    assert out.stdout.strip() == "checked 1132462081 values, 0 mismatches"
