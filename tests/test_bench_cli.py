"""bench.py's launcher contract on a machine without GPUs: `--gpus N` is
honoured (N rank processes, or a non-zero exit naming the shortfall) and a
WORLD_SIZE that disagrees with --gpus is refused."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args, env=None):
    e = dict(os.environ)
    e.pop("WORLD_SIZE", None)
    e.update(env or {})
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, capture_output=True, text=True,
                          timeout=300, env=e)


def test_gpus_2_without_gpus_exits_nonzero():
    r = _run(["--gpus", "2", "--steps", "2", "--warmup", "1"])
    assert r.returncode != 0
    assert "--gpus 2 needs 2 GPUs" in r.stderr


def test_world_size_must_match_gpus():
    r = _run(["--gpus", "4", "--steps", "2"], env={"WORLD_SIZE": "2", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode != 0
    assert "WORLD_SIZE=2" in r.stderr
