"""The CPU oracle under AddressSanitizer + UBSan (sanitizers on
the CPU restatement).  oracle/asan_main.c drives every oracle entry point the
tests use over edge-case geometry (1x1, odd, RGBA with padded rows, 1 and 4
threads of the nested frame x channel OpenMP teams, post chain with and
without faces, compositing, the frame-size upsample); any ASan / UBSan report
fails the run."""
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_oracle_clean_under_asan(pkg):
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "asan"], check=True)
    exe = os.path.join(ROOT, "oracle", "_ref", "oracle_asan")
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1", UBSAN_OPTIONS="halt_on_error=1")
    out = subprocess.run([exe, pkg.ensure_weights()], capture_output=True, text=True, env=env, timeout=300)
    assert out.returncode == 0, out.stdout + out.stderr
    assert "0 failures" in out.stdout
