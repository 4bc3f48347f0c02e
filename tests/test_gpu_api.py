"""GPU tests of the API surface around the hot path (round 3):

  * the MT19937 product path -- legacy_probabilities(..., rng="mt"): host MT panels ->
    csa_panel_hash_async -> device counts / pairs / exact distinct count -- against the
    reference's PUBLISHED seed-0 probabilities and seed-1 unique counts (analysis.py:162-191
    with random.seed at analysis.py:169, randint at legacy.py:149);
  * csa_panel_hash_async called directly, against the host mirror distributed.panel_hashes;
  * pickling of the returned tuple (run_legacy_or_retrieve, analysis.py:284-290): the pickle
    holds host data only and loads in a process that sees no GPU;
  * the draw statistics (attempts / SelectionErrors / min-quota rejections)
    against the reference's own split (tests/golden/philox_*.json);
  * the exchange's local distinct pass beyond the partitioned path (> 8192 x 2048 entries);
  * bench.py --gpus 2 launching its own ranks (gloo rehearsal on one GPU) == the N = 1 run.
"""
import json
import os
import pickle
import random
import subprocess
import sys

import numpy as np
import pytest

from conftest import GOLD, REPO, golden, inst_paths, pkg

pytestmark = pytest.mark.gpu

with open(os.path.join(GOLD, "mt_published.json")) as fh:
    MT = json.load(fh)


def _inst(name, k):
    return pkg().read_instance(*inst_paths(name), k)


def _host_pairs(panels, n):
    bits = np.unpackbits(np.ascontiguousarray(panels).view(np.uint8), axis=1, bitorder="little")[:, :n]
    x = bits.astype(np.float64)
    return np.rint(x.T @ x).astype(np.int64)       # exact: S <= 10^4 < 2^53


@pytest.mark.parametrize("rel", sorted(r for r in MT if r.endswith(".csv")))
def test_mt_product_path_matches_published(gpu_available, rel):
    """legacy_probabilities(inst, 10^4, 0, rng="mt"): the alloc equals the reference's published
    column bit for bit; pairs equal X^T X of the same MT panels (host); found_panels exact."""
    A = pkg("analysis")
    L = pkg("legacy")
    g = MT[rel]
    inst = _inst(g["instance"], g["k"])
    alloc, found, hist = A.legacy_probabilities(inst, g["S"], 0, rng="mt")
    assert [alloc[i] for i in range(len(alloc))] == g["selection_probability"]
    enc = pkg().encode(inst.categories, inst.agents)
    random.seed(0)
    st = np.zeros(3, np.uint64)
    _, panels, attempts = L.mt_draw(enc, g["k"], g["S"], stats=st)
    want = _host_pairs(panels, enc.n)
    iu = np.triu_indices(enc.n, 1)
    assert hist.upper().tolist() == (want[iu] / g["S"]).tolist()
    assert len(found) == len(np.unique(panels, axis=0))
    assert set(found) == {tuple(int(p) for p in np.flatnonzero(
        np.unpackbits(r.view(np.uint8), bitorder="little")[:enc.n])) for r in panels}
    assert A.LAST_RUN_STATS == {"attempts": int(attempts.sum()), "selection_errors": int(st[1]),
                                "rejections": int(st[2])}
    assert int(st[0]) == int(attempts.sum())


@pytest.mark.parametrize("name", ["couples_panel_from_twenty_people_no_constraints_2", "example_small_20"])
def test_mt_product_path_seed1_unique(gpu_available, name):
    """seed 1 (run_legacy_or_retrieve(resample=True)): the device's exact distinct count of the MT
    panels equals the reference's published unique-panel count (analysis/*_statistics.txt)."""
    A = pkg("analysis")
    k = int(name.rsplit("_", 1)[1])
    _, found, _ = A.legacy_probabilities(_inst(name, k), 10000, 1, rng="mt")
    assert len(found) == MT["statistics_seed1"][name]["unique"]


@pytest.mark.parametrize("W,S", [(1, 1), (1, 5000), (4, 777), (27, 4096), (128, 1000), (256, 300)])
def test_panel_hash_async_matches_host_mirror(gpu_available, W, S):
    """csa_panel_hash_async (the hash of host-drawn MT panels) == distributed.panel_hashes, on random
    rows plus repeated and all-zero rows."""
    import torch
    N = pkg("_native")
    D = pkg("distributed")
    rng = np.random.default_rng(W * 7919 + S)
    p = rng.integers(0, 2 ** 63, size=(S, W), dtype=np.uint64) ^ rng.integers(0, 2, size=(S, W), dtype=np.uint64)
    if S > 4:
        p[1] = p[0]
        p[2] = 0
    d = torch.from_numpy(p.view(np.int64).reshape(-1).copy()).cuda()
    h = torch.zeros(2 * S, dtype=torch.int64, device="cuda")
    N.check(N.lib().csa_panel_hash_async(N.ptr(d), S, W, N.ptr(h), None))
    torch.cuda.synchronize()
    got = h.cpu().numpy().view(np.uint64).reshape(S, 2)
    assert np.array_equal(got, D.panel_hashes(p))


_LOAD_CHILD = r"""
import os, pickle, sys
import numpy as np
sys.path.insert(0, %(repo)r)
with open(%(path)r, "rb") as fh:
    alloc, found, hist = pickle.load(fh)
assert "torch" not in sys.modules, "unpickling needed torch"
ids = sorted(alloc)
np.save(%(alloc)r, np.array([alloc[i] for i in ids]))
np.save(%(upper)r, hist.upper())
np.save(%(found)r, np.array(sorted(found), dtype=np.int64).reshape(len(found), -1))
print(len(found))
"""


@pytest.mark.parametrize("name,k,S,seed,rng", [("example_small_20", 20, 3000, 4, "philox"),
                                               ("couples_panel_from_twenty_people_no_constraints_2", 2, 5000, 1,
                                                "philox"),
                                               ("example_small_20", 20, 2000, 0, "mt")])
def test_returned_tuple_pickles_without_gpu(gpu_available, tmp_path, name, k, S, seed, rng):
    """pickle.dumps(legacy_probabilities(...)) as run_legacy_or_retrieve does (analysis.py:290),
    pickle.load in a child process with every GPU hidden: alloc, found_panels and the pair
    histogram are equal to the originals."""
    A = pkg("analysis")
    alloc, found, hist = A.legacy_probabilities(_inst(name, k), S, seed, rng=rng)
    path = tmp_path / "legacy.pickle"
    with open(path, "wb") as fh:
        pickle.dump((alloc, found, hist), fh)
    files = {key: str(tmp_path / (key + ".npy")) for key in ("alloc", "upper", "found")}
    env = dict(os.environ, HIP_VISIBLE_DEVICES="-1", CUDA_VISIBLE_DEVICES="-1", ROCR_VISIBLE_DEVICES="-1")
    out = subprocess.run([sys.executable, "-c", _LOAD_CHILD % dict(repo=REPO, path=str(path), **files)], env=env,
                         capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stderr
    assert int(out.stdout.strip()) == len(found)
    assert np.load(files["alloc"]).tolist() == [alloc[i] for i in sorted(alloc)]
    assert np.array_equal(np.load(files["upper"]), hist.upper())
    assert [tuple(r) for r in np.load(files["found"]).tolist()] == sorted(found)


@pytest.mark.parametrize("case", ["pathological_5_s0", "rejecty_6_s3", "sf_e_tight_110_s1", "couples_s0"])
def test_draw_stats_match_reference(gpu_available, case):
    """csa_instance_draw_stats after a csa_legacy_sample of a golden's panels: attempts,
    SelectionError restarts and min-quota rejections equal the reference's own split."""
    A = pkg("analysis")
    g = golden(case)
    inst = _inst(g["instance"], g["k"])
    enc = pkg().encode(inst.categories, inst.agents)
    raw = A.legacy_sample_raw(enc, g["k"], g["S"], g["seed"], want_pairs=False, want_panels=False)
    assert raw.stats == {"attempts": sum(g["attempts"]), "selection_errors": sum(g["selection_errors"]),
                         "rejections": sum(g["rejections"])}
    alloc, _, _ = A.legacy_probabilities(inst, g["S"], g["seed"])
    assert A.LAST_RUN_STATS == raw.stats


def test_draw_stats_k0(gpu_available):
    """k = 0 takes the host fast path (empty panels, no kernel draw): every panel is one accepted
    attempt when no min is positive, in the bitmask form and in the pick-list form alike (ADVICE r03:
    the pick-list form counted nothing).  That re-draws of the multi-GPU owner add no panels is
    checked by test_bench_job_mode_two_ranks_equals_one (couples: equal draw statistics at N = 2)."""
    import torch
    N = pkg("_native")
    A = pkg("analysis")
    inst = _inst("couples_panel_from_twenty_people_no_constraints_2", 0)
    enc = pkg().encode(inst.categories, inst.agents)
    raw = A.legacy_sample_raw(enc, 0, 1000, 3, want_pairs=False, want_panels=False)
    assert raw.stats == {"attempts": 1000, "selection_errors": 0, "rejections": 0}
    assert raw.unique == 1
    A.draw_stats(enc, reset=True)
    st = torch.zeros(4, dtype=torch.int32, device="cuda")
    picks = torch.empty(8, dtype=torch.int16, device="cuda")
    N.check(N.lib().csa_draw_picks_async(enc.handle, 0, 3, 0, 500, 0, N.ptr(picks), None, N.ptr(st), None))
    torch.cuda.synchronize()
    assert int(st[0].item()) == 0
    assert A.draw_stats(enc) == {"attempts": 500, "selection_errors": 0, "rejections": 0}


@pytest.mark.parametrize("name,k,S,chunk", [("sf_e_tight_110", 110, 20011, 3000), ("sf_e_110", 110, 9000, 2048),
                                            ("synthetic8192_200", 200, 2600, 1000), ("rejecty_6", 6, 5000, 700)])
def test_sample_device_chunks_overlapped(gpu_available, name, k, S, chunk):
    """legacy_sample_device in chunks: every chunk's draw enqueued at once on the draw stream, the
    counting following chunk by chunk on the pipeline stream -- counts, pairs, the exact distinct
    count, the panels and the draw statistics equal one single-chunk batch of the same panel indices."""
    import torch
    A = pkg("analysis")
    inst = _inst(name, k)
    enc = pkg().encode(inst.categories, inst.agents)
    one = A.legacy_sample_device(enc, k, S, 5, chunk=S)
    enc2 = pkg().encode(inst.categories, inst.agents)
    many = A.legacy_sample_device(enc2, k, S, 5, chunk=chunk)
    torch.cuda.synchronize()
    assert np.array_equal(one.counts, many.counts)
    assert torch.equal(torch.triu(one.pairs), torch.triu(many.pairs))
    assert one.unique == many.unique
    assert torch.equal(one.panels, many.panels)
    assert one.stats == many.stats and one.stats["attempts"] >= S


@pytest.mark.parametrize("name,k,S,chunk", [("sf_e_tight_110", 110, 12007, 2500), ("synthetic8192_200", 200, 2600, 640)])
def test_legacy_sample_c_pipeline_chunks(gpu_available, monkeypatch, name, k, S, chunk):
    """csa_legacy_sample's own pipeline (C ABI) in chunks of CSA_SAMPLE_CHUNK panels (chunk c + 1
    drawn while chunk c is counted and paired): equal to one single-chunk batch."""
    A = pkg("analysis")
    inst = _inst(name, k)
    enc = pkg().encode(inst.categories, inst.agents)
    one = A.legacy_sample_raw(enc, k, S, 9)
    monkeypatch.setenv("CSA_SAMPLE_CHUNK", str(chunk))
    many = A.legacy_sample_raw(enc, k, S, 9)
    assert np.array_equal(one.counts, many.counts)
    assert np.array_equal(np.triu(one.pairs), np.triu(many.pairs))
    assert one.unique == many.unique and np.array_equal(one.panels, many.panels)
    assert one.stats == many.stats


def test_exchange_local_distinct_beyond_partitioned_path(gpu_available):
    """csa_exchange_pack_async on 8192 x 2048 + 4096 entries (the partitioned dedupe's limit + 1
    block): the global-table fallback lists exactly one index per distinct panel."""
    import torch
    N = pkg("_native")
    D = pkg("distributed")
    n = 8192 * 2048 + 4096
    rng = np.random.default_rng(5)
    base = rng.integers(0, 2 ** 63, size=n // 3, dtype=np.uint64)
    p = base[rng.integers(0, len(base), size=n)].reshape(n, 1)     # many duplicates
    want = len(np.unique(p))
    dp = torch.from_numpy(p.view(np.int64).reshape(-1).copy()).cuda()
    dh = torch.empty(2 * n, dtype=torch.int64, device="cuda")
    N.check(N.lib().csa_panel_hash_async(N.ptr(dp), n, 1, N.ptr(dh), None))
    status = torch.zeros(4, dtype=torch.int32, device="cuda")
    rows, cnt = D.local_distinct_rows(dh, dp, n, 1, status)
    assert cnt == want
    got = np.sort(rows.cpu().numpy().view(np.uint64))
    assert np.array_equal(got, np.unique(p))
    assert int(status[0].item()) == 0


def _bench(args, env_extra):
    env = dict(os.environ, **env_extra)
    out = subprocess.run([sys.executable, os.path.join(REPO, "bench.py")] + args, env=env, capture_output=True,
                         text=True, timeout=400, cwd=REPO)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out.stdout[-2000:]
    return json.loads(lines[0])


@pytest.mark.timeout(600)
def test_bench_self_launch_two_ranks_equals_one(gpu_available):
    """`python bench.py --gpus 2` (no launcher; gloo rehearsal with both ranks on this GPU) starts its
    own two ranks and prints one line with n_gpus 2 whose checks equal the N = 1 run over the same
    global panels; the one-process multi-device leg (csa_legacy_sample_devices over the ranks'
    devices) equals the rank-sharded result."""
    common = ["--steps", "3", "--warmup", "1", "--no-cpu-baseline", "--no-api", "--iso-steps", "0"]
    two = _bench(["--gpus", "2", "--panels", "20000"] + common, {"CSA_BENCH_BACKEND": "gloo"})
    one = _bench(["--gpus", "1", "--panels", "40000"] + common, {})
    assert two["n_gpus"] == 2 and one["n_gpus"] == 1
    for key in ("last_step_unique", "last_step_count_sum", "last_step_pair_sum", "last_step_counts_sha256",
                "last_step_pairs_triu_sha256"):
        assert two["checks"][key] == one["checks"][key]
    assert two["checks"]["sample_devices"]["equal_to_rank_sharded"] is True
    st = two["draw_stats"]
    assert st["attempts"] == st["panels"] + st["selection_errors"] + st["rejections"]


@pytest.mark.timeout(600)
@pytest.mark.parametrize("config,panels,chunk", [("sf_e_110", 90001, 20000), ("synthetic8192", 30001, 8000),
                                                 ("couples", 100001, 30000)])
def test_bench_job_mode_two_ranks_equals_one(gpu_available, config, panels, chunk):
    """bench.py --job-panels P (strong scaling: ONE job of P panels split over the ranks, accumulated
    counts / pairs, the exact distinct count over the whole job): the 2-rank gloo rehearsal on this GPU
    and the 1-GPU run agree on the count vector and the pair triangle (SHA-256 digests), the distinct
    count and the draw statistics; uneven shares (P odd) and a ragged last chunk included."""
    common = ["--config", config, "--job-panels", str(panels), "--panels", str(chunk), "--warmup", "1",
              "--no-cpu-baseline", "--no-api"]
    two = _bench(["--gpus", "2"] + common, {"CSA_BENCH_BACKEND": "gloo"})
    one = _bench(["--gpus", "1"] + common, {})
    assert two["scaling"] == one["scaling"] == "strong"
    for key in ("job_unique", "job_count_sum", "job_pair_sum", "job_counts_sha256", "job_pairs_triu_sha256"):
        assert two["checks"][key] == one["checks"][key], key
    assert two["draw_stats"] == one["draw_stats"]
    assert one["steps"] == (panels + chunk - 1) // chunk
