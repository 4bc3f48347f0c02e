"""World-size-2 gloo rehearsal of the multi-GPU exchange (distributed.combine) on CPU.

Each rank produces its contiguous shard of panels with the C oracle (standing in
for that rank's GPU), then runs the real exchange code: all_reduce of counts and
pair counts, all_gather of 128-bit panel hashes + owner-partition dedupe +
all_reduce.  The combined results must equal one unsharded run.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import REPO, inst_paths, pkg

S, SEED, NAME, K = 3000, 5, "sf_e_110", 110


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, out_dir):
    import sys
    sys.path.insert(0, REPO)
    sys.path.insert(0, os.path.join(REPO, "tests"))
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from oracle import coracle
    from oracle.legacy_oracle import read_instance
    D = pkg("distributed")
    o = read_instance(*inst_paths(NAME), K)
    b, e = D.shard_range(S, world, rank)
    rc, panels, _, _ = coracle.draw(o, K, SEED, b, e - b, threads=2)
    assert rc == 0
    counts = torch.from_numpy(coracle.counts(panels, o.n))
    pairs = torch.from_numpy(coracle.pairs(panels, o.n, threads=2).ravel().copy())
    hashes = torch.from_numpy(D.panel_hashes(panels).ravel().view(np.int64).copy())
    counts, pairs, u = D.combine(counts, pairs, hashes)
    if rank == 0:
        np.save(os.path.join(out_dir, "counts.npy"), counts.numpy())
        np.save(os.path.join(out_dir, "pairs.npy"), pairs.numpy())
        np.save(os.path.join(out_dir, "unique.npy"), np.array([int(u.item())]))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_gloo_exchange_matches_single_run(tmp_path, world):
    from oracle import coracle
    from oracle.legacy_oracle import read_instance
    mp.spawn(_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    o = read_instance(*inst_paths(NAME), K)
    rc, panels, _, _ = coracle.draw(o, K, SEED, 0, S, threads=4)
    assert rc == 0
    assert np.array_equal(np.load(tmp_path / "counts.npy"), coracle.counts(panels, o.n))
    full = coracle.pairs(panels, o.n, threads=4).ravel()
    assert np.array_equal(np.load(tmp_path / "pairs.npy"), full)
    assert int(np.load(tmp_path / "unique.npy")[0]) == coracle.unique(panels, o.n)


def test_panel_hash_mirror_is_sensitive():
    D = pkg("distributed")
    rng = np.random.default_rng(1)
    p = rng.integers(0, 2 ** 63, size=(200, 27), dtype=np.int64).astype(np.uint64)
    h = D.panel_hashes(p)
    assert len(np.unique(h, axis=0)) == 200
    q = p.copy()
    q[:, 5] ^= np.uint64(1)
    assert not np.any(np.all(D.panel_hashes(q) == h, axis=1))
