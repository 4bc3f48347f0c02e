"""World-size-2/3 gloo rehearsal of the multi-GPU exchange (distributed.combine) on CPU.

Each rank produces its contiguous shard of panels with the C oracle (standing in
for that rank's GPU), then runs the real exchange code on host tensors: all_reduce
of counts and pair counts; the rank's exact local distinct panels (128-bit hash +
bitmask) in fixed-capacity segments per owner rank h1 % world (host mirror of
csa_exchange_pack_async), three equal-split all_to_alls (segment counts, hashes,
bitmasks), the owner's exact dedupe over the valid entries (host mirror of
csa_unique_segments_async: equal hash AND equal bitmask), all_reduce of the
owners' counts.  The combined results must equal one unsharded run -- on an
all-distinct instance and on a duplicate-heavy one whose duplicates land on
different ranks -- and two different panels given the same 128-bit hash must
still count twice (the count is exact, not hash-based).  found_panels are
re-drawn where they are read (distributed.PanelRedraw): rank 0 alone iterates
and pickles them without entering any collective, and the pickle loads in a
child process without a GPU.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import REPO, inst_paths, pkg

CASES = {"sf_e_110": (110, 3000, 5), "couples_panel_from_twenty_people_no_constraints_2": (2, 3000, 7)}


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _init(rank, world, port):
    import sys
    sys.path.insert(0, REPO)
    sys.path.insert(0, os.path.join(REPO, "tests"))
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)


def _worker(rank, world, port, out_dir, name):
    _init(rank, world, port)
    from oracle import coracle
    from oracle.legacy_oracle import read_instance
    D = pkg("distributed")
    K, S, SEED = CASES[name]
    o = read_instance(*inst_paths(name), K)
    b, e = D.shard_range(S, world, rank)
    rc, panels, _, _ = coracle.draw(o, K, SEED, b, e - b, threads=2)
    assert rc == 0
    W = panels.shape[1]
    counts = torch.from_numpy(coracle.counts(panels, o.n))
    pairs = torch.from_numpy(coracle.pairs(panels, o.n, threads=2).ravel().copy())
    hashes = torch.from_numpy(D.panel_hashes(panels).ravel().view(np.int64).copy())
    ptens = torch.from_numpy(np.ascontiguousarray(panels).view(np.int64).ravel().copy())
    counts, pairs, u = D.combine(counts, pairs, hashes, ptens, W)
    # found_panels as legacy_probabilities_distributed returns them on every rank: the exchange's
    # exact count, and a PanelRedraw that re-draws the whole job [0, S) where it is read (the C oracle
    # stands in for this rank's GPU, csa_redraw_async) -- no panels kept, nothing sent
    A = pkg("analysis")
    import pickle
    found = A.PanelSet(int(u.item()), None, o.n, list(range(o.n)))

    def redraw(b_, c_):
        rc_, p_, _, _ = coracle.draw(o, K, SEED, b_, c_, threads=2)
        assert rc_ == 0
        return p_

    found._redraw = D.PanelRedraw(redraw, S, W, chunk=777)      # several chunks, a ragged last one
    assert len(found) == int(u.item())
    dist.barrier()
    # every collective / point-to-point entry of torch.distributed is counted from here on
    entered = []
    names = ("send", "recv", "isend", "irecv", "all_reduce", "all_gather", "all_to_all_single", "broadcast",
             "gather", "scatter", "reduce", "barrier", "all_gather_object", "gather_object", "broadcast_object_list")
    real = {nm: getattr(dist, nm) for nm in names}

    def spy(nm):
        def f(*a, **kw):
            entered.append(nm)
            return real[nm](*a, **kw)
        return f

    for nm in names:
        setattr(dist, nm, spy(nm))
    try:
        if rank == 0:   # rank 0 ALONE reads its found_panels, while the other ranks are elsewhere
            tuples = sorted(found)
            rows = found.rows()
            blob = pickle.dumps(found)
            assert all(t in found for t in tuples[:5]) and (-1,) not in found
            assert entered == []
            np.save(os.path.join(out_dir, "rows.npy"), rows)
            np.save(os.path.join(out_dir, "counts.npy"), counts.numpy())
            np.save(os.path.join(out_dir, "pairs.npy"), pairs.numpy())
            np.save(os.path.join(out_dir, "unique.npy"), np.array([int(u.item())]))
            with open(os.path.join(out_dir, "found.pkl"), "wb") as f:
                f.write(blob)
            with open(os.path.join(out_dir, "tuples.txt"), "w") as f:
                f.write(repr(tuples))
        else:
            assert entered == []
    finally:
        for nm in names:
            setattr(dist, nm, real[nm])
    # a forged count: the re-drawn set must have the run's exact count, or reading it raises
    bad = A.PanelSet(int(u.item()) + 1, None, o.n, list(range(o.n)))
    bad._redraw = D.PanelRedraw(redraw, S, W, chunk=4096)
    with pytest.raises(RuntimeError, match="re-drawn"):
        bad.rows()
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("name", sorted(CASES))
@pytest.mark.parametrize("world", [2, 3])
def test_gloo_exchange_matches_single_run(tmp_path, world, name):
    from oracle import coracle
    from oracle.legacy_oracle import read_instance
    K, S, SEED = CASES[name]
    mp.spawn(_worker, args=(world, _free_port(), str(tmp_path), name), nprocs=world, join=True)
    o = read_instance(*inst_paths(name), K)
    rc, panels, _, _ = coracle.draw(o, K, SEED, 0, S, threads=4)
    assert rc == 0
    assert np.array_equal(np.load(tmp_path / "counts.npy"), coracle.counts(panels, o.n))
    full = coracle.pairs(panels, o.n, threads=4).ravel()
    assert np.array_equal(np.load(tmp_path / "pairs.npy"), full)
    want = coracle.unique(panels, o.n)
    if name.startswith("couples"):
        # duplicates really are split across ranks: every shard holds most of the 100 panels
        assert want == 100
    assert int(np.load(tmp_path / "unique.npy")[0]) == want
    # the panels rank 0 re-drew alone are exactly the distinct panels of the single run
    rows = np.load(tmp_path / "rows.npy")
    assert np.array_equal(rows, np.unique(panels, axis=0))
    # rank 0's pickle loads and iterates in a child process that has no GPU at all
    import subprocess
    import sys
    env = dict(os.environ, HIP_VISIBLE_DEVICES="-1", CUDA_VISIBLE_DEVICES="-1", ROCR_VISIBLE_DEVICES="-1")
    code = ("import pickle, sys; sys.path.insert(0, %r); import torch; assert not torch.cuda.is_available(); "
            "f = pickle.load(open(%r, 'rb')); print(repr(sorted(f))); print(len(f))"
            % (REPO, str(tmp_path / "found.pkl")))
    out = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr
    got, ln = out.stdout.strip().splitlines()
    assert got == (tmp_path / "tuples.txt").read_text() and int(ln) == want


def _collision_worker(rank, world, port, out_dir):
    """Rank 0 holds panel A; rank 1 holds a different panel B and another copy of A, all three
    under the SAME (fake) 128-bit hash: the exact count is 2, a hash-only count would be 1."""
    _init(rank, world, port)
    D = pkg("distributed")
    W = 3
    A = np.array([1, 2, 3], np.uint64)
    B = np.array([1, 2, 4], np.uint64)
    rows = [A] if rank == 0 else [B, A]
    panels = torch.from_numpy(np.stack(rows).view(np.int64).ravel().copy())
    fake = np.tile(np.array([12345, 678], np.uint64), (len(rows), 1))
    hashes = torch.from_numpy(fake.view(np.int64).ravel().copy())
    counts = torch.zeros(4, dtype=torch.int64)
    _, _, u = D.combine(counts, None, hashes, panels, W)
    if rank == 0:
        np.save(os.path.join(out_dir, "unique.npy"), np.array([int(u.item())]))
    dist.barrier()
    dist.destroy_process_group()


def test_gloo_exchange_exact_on_hash_collision(tmp_path):
    mp.spawn(_collision_worker, args=(2, _free_port(), str(tmp_path)), nprocs=2, join=True)
    assert int(np.load(tmp_path / "unique.npy")[0]) == 2


def test_segment_buckets_mirror():
    """segment_buckets (host mirror of csa_exchange_pack_async): each owner segment holds exactly the
    local DISTINCT panels it owns (h1 % world), every panel with its hash; capacity overflow raises."""
    D = pkg("distributed")
    rng = np.random.default_rng(3)
    p = rng.integers(0, 2 ** 63, size=(1000, 5), dtype=np.int64).astype(np.uint64)
    p = np.concatenate([p, p[:300]])                       # 300 local duplicates
    h = D.panel_hashes(p)
    for world in (1, 2, 3, 8):
        cap = D.exchange_capacity(len(p), world)
        sh, sp, c = D.segment_buckets(h, p, world, cap)
        assert c.sum() == 1000 and len(c) == world and c.max() <= cap
        got = []
        for w in range(world):
            assert np.all(sh[w, : c[w], 0] % np.uint64(world) == np.uint64(w))
            assert np.array_equal(D.panel_hashes(sp[w, : c[w]]), sh[w, : c[w]])
            got += list(map(tuple, sp[w, : c[w]].tolist()))
        assert sorted(got) == sorted(set(map(tuple, p.tolist())))
        assert D.distinct_segments(sh, sp, c) == 1000
    with pytest.raises(RuntimeError):
        D.segment_buckets(h, p, 2, 100)


def test_exchange_capacity_bounds():
    D = pkg("distributed")
    assert D.exchange_capacity(1, 8) == 1 and D.exchange_capacity(0, 8) == 1
    assert D.exchange_capacity(1000, 1) == 1000
    c = D.exchange_capacity(10 ** 6, 8)
    assert 125000 < c < 128000          # mean + 8 sd + 64 of Binomial(1e6, 1/8)


def test_distinct_exact_mirror():
    D = pkg("distributed")
    p = np.array([[1, 2], [1, 2], [1, 3], [0, 0]], np.uint64)
    h = D.panel_hashes(p)
    assert D.distinct_exact(h, p) == 3
    h[2] = h[0]          # a forged collision still counts as a different panel
    assert D.distinct_exact(h, p) == 3
    assert D.distinct_exact(np.zeros((0, 2), np.uint64), np.zeros((0, 2), np.uint64)) == 0


def test_panel_hash_mirror_is_sensitive():
    D = pkg("distributed")
    rng = np.random.default_rng(1)
    p = rng.integers(0, 2 ** 63, size=(200, 27), dtype=np.int64).astype(np.uint64)
    h = D.panel_hashes(p)
    assert len(np.unique(h, axis=0)) == 200
    q = p.copy()
    q[:, 5] ^= np.uint64(1)
    assert not np.any(np.all(D.panel_hashes(q) == h, axis=1))


_RANK_SCRIPT = r"""
import json, os, sys
import torch, torch.distributed as dist
dist.init_process_group("gloo")
r, w = dist.get_rank(), dist.get_world_size()
t = torch.tensor([r + 1])
dist.all_reduce(t)
if r == 0:
    print(json.dumps({"world": w, "sum": int(t.item()), "argv": sys.argv[1:],
                      "local": os.environ["LOCAL_RANK"], "addr": os.environ["MASTER_ADDR"]}))
dist.destroy_process_group()
"""


def test_bench_self_launch_world2(tmp_path, capfd):
    """bench.self_launch -- what `python bench.py --gpus 2` runs when no launcher set WORLD_SIZE --
    starts two rank processes with RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR=127.0.0.1 /
    MASTER_PORT that rendezvous over gloo; the arguments reach every rank; exit code 0."""
    import importlib.util
    import json
    spec = importlib.util.spec_from_file_location("bench", os.path.join(REPO, "bench.py"))
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    script = tmp_path / "rank.py"
    script.write_text(_RANK_SCRIPT)
    rc = bench.self_launch(2, script=str(script), argv=["--gpus", "2", "--steps", "1"])
    assert rc == 0
    line = [ln for ln in capfd.readouterr().out.splitlines() if ln.startswith("{")]
    assert len(line) == 1
    got = json.loads(line[0])
    assert got == {"world": 2, "sum": 3, "argv": ["--gpus", "2", "--steps", "1"], "local": "0",
                   "addr": "127.0.0.1"}


_FAILING_RANK_SCRIPT = r"""
import os, sys, time
import torch.distributed as dist
if os.environ["RANK"] == "1":
    sys.exit(3)                 # this rank dies before the rendezvous
dist.init_process_group("gloo")  # rank 0 would wait here for rank 1 until the store's timeout
"""


def test_bench_self_launch_fails_fast(tmp_path):
    """self_launch with one rank exiting non-zero at startup: the other rank (blocked in the
    rendezvous) is terminated and the failing rank's exit code returned within seconds, not after the
    rendezvous timeout."""
    import importlib.util
    import time
    spec = importlib.util.spec_from_file_location("bench", os.path.join(REPO, "bench.py"))
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    script = tmp_path / "rank.py"
    script.write_text(_FAILING_RANK_SCRIPT)
    t = time.time()
    rc = bench.self_launch(2, script=str(script), argv=[], grace=5.0)
    assert rc == 3
    assert time.time() - t < 60
