"""CPU tests of the data-parallel path (world_size 2, gloo): frame sharding,
ragged batches and the ordered all-gather of masks.  The per-frame compute is
the CPU oracle here (the checker), so the gathered result must equal a
single-process oracle run on the whole batch."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from conftest import load_pkg


def test_shard_range_partition():
    pkg = load_pkg()
    import vss_amd.parallel as par
    for n in range(0, 20):
        for world in (1, 2, 3, 4, 8):
            covered = []
            for r in range(world):
                s, c = par.shard_range(n, r, world)
                assert c <= par.shard_capacity(n, world)
                covered.extend(range(s, s + c))
            assert covered == list(range(n))
    _ = pkg


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
    lp()
    import vss_amd.parallel as par
    import vss_amd.synthetic as syn
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        blob = open(blob_path, "rb").read()
        start, count = par.shard_range(n_total, rank, world)
        frames = np.stack([syn.make_frame(i, 60, 80) for i in range(start, start + count)]) if count else None
        if count:
            local = torch.from_numpy(oracle_py.forward(blob, frames, 32, 48, mode=0).reshape(count, -1))
        else:
            local = torch.zeros((0, 32 * 48))
        full = par.gather_masks(local, n_total)
        q.put((rank, full.numpy()))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("n_total", [4, 5, 1])
def test_gather_masks_gloo_world2(blob, n_total):
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
