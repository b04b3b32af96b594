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


def test_gpus_2_dry_run_reaches_the_clique_id_broadcast():
    """the whole multi-rank launch path of `bench.py --gpus 2`
    — launch_ranks -> torch.distributed.run -> gloo init -> rank 0's clique-id
    broadcast — runs here, stopping before the first GPU call: both ranks see
    WORLD_SIZE=2 and rank 1 holds exactly rank 0's id bytes."""
    import json
    r = _run(["--gpus", "2", "--dry-run-dist"])
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{") and '"dry_run"' in x]
    by_rank = {d["rank"]: d for d in lines}
    assert sorted(by_rank) == [0, 1], r.stdout
    for d in by_rank.values():
        assert d["world"] == 2 and d["env_world_size"] == "2"
        assert d["ids_len"] == 4 * 128
    assert by_rank[0]["ids_sha256"] == by_rank[1]["ids_sha256"]


def test_gpus_2_selects_the_ordered_gather_form():
    """the first R > 1 run must not be able to deadlock, so the
    N > 1 bench defaults to the ordered all-gather (one communicator and one
    gather stream per rank: one total order of collectives); the
    concurrent per-slot communicators are opt-in (--gather-form concurrent).
    Every rank reports the form it would run."""
    import json
    for extra, want in (([], "ordered"), (["--gather-form", "concurrent"], "concurrent")):
        r = _run(["--gpus", "2", "--dry-run-dist"] + extra)
        assert r.returncode == 0, r.stderr[-2000:]
        lines = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{") and '"dry_run"' in x]
        assert sorted(d["rank"] for d in lines) == [0, 1], r.stdout
        assert all(d["gather_form"] == want for d in lines), (extra, lines)


def test_watchdog_ends_a_stalled_multi_rank_run_with_a_record():
    """a rank that never reaches the barrier (--test-stall-rank,
    on the --dry-run-dist path: the same launcher, gloo group and broadcast as
    the GPU run) must not hang the job.  The waiting rank's watchdog prints one
    JSON record naming its rank and stage and exits 3 (os._exit, no re-exec);
    torch.distributed.run then ends the job non-zero, well before any driver
    timeout."""
    import json
    import time
    t0 = time.monotonic()
    r = _run(["--gpus", "2", "--dry-run-dist", "--test-stall-rank", "1", "--watchdog-s", "3"])
    el = time.monotonic() - t0
    assert r.returncode != 0
    recs = [json.loads(x) for x in (r.stdout + "\n" + r.stderr).splitlines()
            if x.startswith("{") and '"watchdog"' in x]
    assert recs, (r.stdout[-2000:], r.stderr[-2000:])
    stages = {(d["rank"], d["stage"]) for d in recs}
    # rank 0 waits in the barrier rank 1 never reaches; rank 1 sits in its stall
    assert (0, "dry-run: barrier") in stages or (1, "dry-run: stalled rank") in stages, stages
    for d in recs:
        assert d["world"] == 2 and d["seconds_without_progress"] >= 3
        assert d["gather_form"] == "ordered", d  # the record names the form the ranks run
    assert el < 120, el


def test_watchdog_off_by_zero_and_quiet_on_a_healthy_run():
    """--watchdog-s 0 starts no thread, and a healthy dry run with the default
    limit prints no record."""
    r = _run(["--gpus", "2", "--dry-run-dist"])
    assert r.returncode == 0 and '"watchdog"' not in r.stdout + r.stderr
    r = _run(["--gpus", "2", "--dry-run-dist", "--watchdog-s", "0"])
    assert r.returncode == 0 and '"watchdog"' not in r.stdout + r.stderr
