"""CPU tests of the product's multi-GPU batch plan.

libvss's `vss_shard_plan` is the plan the multi-GPU handle (submit_host) and
the one-GPU-per-process clique use: contiguous shards of ceil(n / R) frames,
an all-gather of ceil(n / R) rows per rank, frame i at gathered row i.  It is
host-only, so it is checked here exhaustively, and a world-size-2 gloo run
drives the same plan end to end: each rank computes its shard (the CPU oracle
stands in for the GPU forward — the checker), pads it to `per_rank` rows and
all-gathers, exactly the collective the C ABI issues over RCCL; the first n
gathered rows must equal a single-process run over the whole batch.  The RCCL
exchange itself is measured only on an 8-GPU node (the driver's SCALE run)."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from conftest import load_pkg


@pytest.mark.parametrize("R", range(1, 9))
def test_shard_plan_exhaustive(R):
    pkg = load_pkg()
    for n in range(0, 71):
        covered, gathered = [], []
        per_all = set()
        for r in range(R):
            first, count, per = pkg.shard_plan(n, R, r)
            per_all.add(per)
            assert per == -(-n // R)
            assert 0 <= count <= per
            covered.extend(range(first, first + count))
            # the rank's `per` gathered rows: its frames, then padding (None)
            gathered.extend(list(range(first, first + count)) + [None] * (per - count))
        assert len(per_all) == 1
        assert covered == list(range(n)), (n, R)
        # frame order: the first n gathered rows are frames 0..n-1, only padding after
        assert gathered[:n] == list(range(n)), (n, R)
        assert all(g is None for g in gathered[n:])


@pytest.mark.parametrize("R", range(1, 9))
@pytest.mark.parametrize("out_mode", ["model", "frame"])
def test_gather_copy_out_frame_order(R, out_mode):
    """the multi-GPU handle's copy-out (vss_gather_runs, what
    submit_host's D2H and frame-size upsample follow) applied to a simulated
    all-gather — each rank's block = its shard's rows, then padding rows of
    garbage — puts every frame's row at its frame index and reads no padding.
    A row is P floats at model resolution or fh*fw after the upsample; the
    runs are in rows, so both layouts are checked with their row size."""
    pkg = load_pkg()
    row = 6 if out_mode == "model" else 10  # elements per row (stand-ins for P / fh*fw)
    for n in range(0, 71):
        blocks = []
        for r in range(R):
            first, count, per = pkg.shard_plan(n, R, r)
            blk = np.full((per, row), -1.0, np.float32)  # padding garbage
            for i in range(count):
                blk[i] = first + i + np.arange(row) / 100.0
            blocks.append(blk)
        gathered = np.concatenate(blocks) if blocks and blocks[0].size else np.zeros((0, row), np.float32)
        out = np.full((n, row), np.nan, np.float32)
        runs = pkg.gather_runs(n, R)
        assert len(runs) <= R
        for src, dst, rows in runs:
            assert rows > 0 and 0 <= dst and dst + rows <= n
            seg = gathered[src:src + rows]
            assert (seg >= 0).all(), (n, R, src, rows)  # never a padding row
            out[dst:dst + rows] = seg
        want = np.arange(n)[:, None] + np.arange(row)[None, :] / 100.0
        assert np.array_equal(out, want.astype(np.float32)), (n, R)
        # contiguous shards: one run of n rows from row 0
        assert runs == ([(0, 0, n)] if n else [])


def test_shard_plan_rejects_bad_args():
    pkg = load_pkg()
    for args in ((-1, 2, 0), (4, 0, 0), (4, 2, 2), (4, 2, -1)):
        with pytest.raises(pkg.VssError):
            pkg.shard_plan(*args)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, n_total, blob_path, q):
    import sys
    import torch
    import torch.distributed as dist
    sys.path.insert(0, os.path.dirname(__file__))
    from conftest import load_pkg as lp
    import oracle_py
    pkg = lp()
    import vss_amd.synthetic as syn
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        blob = open(blob_path, "rb").read()
        first, count, per = pkg.shard_plan(n_total, world, rank)
        send = torch.zeros((per, 32 * 48), dtype=torch.float32)  # padding rows stay zero
        if count:
            frames = np.stack([syn.make_frame(i, 60, 80) for i in range(first, first + count)])
            send[:count] = torch.from_numpy(oracle_py.forward(blob, frames, 32, 48, mode=0).reshape(count, -1))
        buf = torch.empty((world * per, 32 * 48), dtype=torch.float32)
        dist.all_gather_into_tensor(buf, send)
        q.put((rank, buf[:n_total].numpy()))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("n_total", [4, 5, 1])
def test_gather_plan_gloo_world2(blob, n_total):
    pkg = load_pkg()
    import oracle_py
    import vss_amd.synthetic as syn
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, n_total, pkg.ensure_weights(), q)) for r in range(world)]
    for p in procs:
        p.start()
    got = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    frames = np.stack([syn.make_frame(i, 60, 80) for i in range(n_total)])
    ref = oracle_py.forward(blob, frames, 32, 48, mode=0).reshape(n_total, -1)
    for r in range(world):
        assert got[r].shape == ref.shape
        assert np.array_equal(got[r], ref), f"rank {r}"
