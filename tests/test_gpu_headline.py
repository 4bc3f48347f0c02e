"""The product entry point at the headline shape, pinned directly.

``legacy_probabilities(instance, S, seed)`` (analysis.py:162-191) on one GPU takes, for one chunk of
panels at sf_e_110, a path of its own: ``csa_draw_xt_async`` (the draw kernel's fused pack also writes
the XT operand), the pair kernel with ``CSA_PAIR_ALONE``, and the per-person counts read off the pair
matrix's diagonal.  Here that composition -- not its pieces -- meets the reference-generated goldens
and the golden-pinned C oracle: alloc floats, every pair value, len(found_panels) and the sorted
panels themselves.  A spy on the pipeline records that the path really was taken.

Second, the round-5 race (the distinct-count table was once allocated after the draws were enqueued
on another stream): back-to-back calls on one encoding whose S grows, so the cached table must grow
on the side-stream path between calls; every call's distinct count and counts equal the oracle's.
"""
import numpy as np
import pytest

from conftest import golden, inst_paths, pkg
from oracle import coracle
from oracle.legacy_oracle import read_instance as oracle_read

pytestmark = pytest.mark.gpu


def _spy(monkeypatch):
    """Record which stages legacy_probabilities runs: draw_xt's return (XT written by the draw),
    pair_counts' ``alone`` flag, counts_from_pairs, and any separate transpose pass."""
    Dv = pkg("device")
    seen = {"draw_xt": [], "alone": [], "diag": 0, "transpose": 0}
    real_xt, real_pairs = Dv.DevicePipeline.draw_xt, Dv.DevicePipeline.pair_counts
    real_diag, real_tc = Dv.DevicePipeline.counts_from_pairs, Dv.DevicePipeline.transpose_count

    def draw_xt(self, *a, **kw):
        r = real_xt(self, *a, **kw)
        seen["draw_xt"].append(r)
        return r

    def pair_counts(self, S, overwrite=False, shared=False, alone=False):
        seen["alone"].append(alone)
        return real_pairs(self, S, overwrite=overwrite, shared=shared, alone=alone)

    def diag(self):
        seen["diag"] += 1
        return real_diag(self)

    def tc(self, S):
        seen["transpose"] += 1
        return real_tc(self, S)

    monkeypatch.setattr(Dv.DevicePipeline, "draw_xt", draw_xt)
    monkeypatch.setattr(Dv.DevicePipeline, "pair_counts", pair_counts)
    monkeypatch.setattr(Dv.DevicePipeline, "counts_from_pairs", diag)
    monkeypatch.setattr(Dv.DevicePipeline, "transpose_count", tc)
    return seen


def _assert_xt_path(seen):
    assert seen["draw_xt"] == [True], seen           # one chunk, XT from the draw's fused pack
    assert seen["alone"] == [True] and seen["diag"] == 1 and seen["transpose"] == 0, seen


def _sha(a):
    import hashlib
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


@pytest.mark.parametrize("case", ["sf_e_110_s0", "example_large_200_s0", "sf_e_tight_110_s1"])
def test_legacy_probabilities_headline_path_vs_golden(gpu_available, monkeypatch, case):
    """sf_e_110 (draw_lane_kernel), sf_e_tight_110 (restarts) and example_large_200
    (draw_solo_kernel) through the one-chunk XT path vs the reference-generated goldens."""
    A = pkg("analysis")
    g = golden(case)
    inst = pkg().read_instance(*inst_paths(g["instance"]), g["k"])
    seen = _spy(monkeypatch)
    alloc, found, hist = A.legacy_probabilities(inst, g["S"], g["seed"])
    _assert_xt_path(seen)
    S = g["S"]
    assert [alloc[i] for i in range(len(alloc))] == [c / S for c in g["counts"]]   # int / int, as the reference
    assert _sha(hist.upper()) == g["pair_prob_sha256"]                              # every pair value, float64
    assert len(found) == g["unique"]
    first = [tuple(p) for p in g["first_panels"]]
    if len(first) == S:
        assert sorted(found) == sorted(set(first))
    else:
        assert all(p in found for p in first)
    assert A.LAST_RUN_STATS == {"attempts": sum(g["attempts"]), "selection_errors": sum(g["selection_errors"]),
                                "rejections": sum(g["rejections"])}


@pytest.mark.parametrize("name,k,S,seed", [("sf_e_110", 110, 20011, (1 << 40) + 12345),
                                           ("sf_e_tight_110", 110, 7001, 77),
                                           ("example_large_200", 200, 3001, 2 ** 63 + 5)])
def test_legacy_probabilities_headline_path_vs_oracle(gpu_available, monkeypatch, name, k, S, seed):
    """The same path at sizes past the goldens, 64-bit seeds, vs the C oracle (pinned to the goldens
    by test_oracle_golden.py): alloc, pair values, distinct count and the distinct panels."""
    A = pkg("analysis")
    inst = pkg().read_instance(*inst_paths(name), k)
    seen = _spy(monkeypatch)
    alloc, found, hist = A.legacy_probabilities(inst, S, seed)
    _assert_xt_path(seen)
    o = oracle_read(*inst_paths(name), k)
    rc, opanels, oatt, _ = coracle.draw(o, k, seed & 0xFFFFFFFFFFFFFFFF, 0, S)
    assert rc == 0
    counts = coracle.counts(opanels, o.n)
    assert [alloc[i] for i in range(len(alloc))] == (counts.astype(np.float64) / S).tolist()
    up = coracle.pairs(opanels, o.n)[np.triu_indices(o.n, 1)]
    assert np.array_equal(hist.upper(), up / S)
    assert len(found) == coracle.unique(opanels, o.n)
    assert np.array_equal(found.rows(), np.unique(opanels, axis=0))
    assert A.LAST_RUN_STATS["attempts"] == int(oatt.sum())


def test_growing_calls_reallocate_table_on_side_stream(gpu_available):
    """Back-to-back legacy_probabilities calls on ONE encoding with S growing, so the encoding's cached
    distinct-count table grows between calls (allocated on the pipeline stream before the draws; the
    count runs on a side stream).  One-chunk calls and a two-chunk call (S > 2^20): each call's distinct
    count and per-person counts equal the C oracle's, once each."""
    A = pkg("analysis")
    name, k = "sf_e_tight_110", 110         # restarts: uneven per-workgroup draw times
    inst = pkg().read_instance(*inst_paths(name), k)
    o = oracle_read(*inst_paths(name), k)
    enc = A.encode_cached(inst.categories, inst.agents)
    slots = []
    for S, seed in ((500, 1), (6000, 2), (70000, 3), (400000, 4), (1100000, 5)):
        alloc, found, hist = A.legacy_probabilities(inst, S, seed)
        slots.append(enc._table.slots)
        rc, opanels, _, _ = coracle.draw(o, k, seed, 0, S)
        assert rc == 0
        assert len(found) == coracle.unique(opanels, o.n), S
        assert [alloc[i] for i in range(len(alloc))] == (coracle.counts(opanels, o.n) / S).tolist(), S
        del opanels
    assert all(b > a for a, b in zip(slots, slots[1:])), slots      # the table really grew every call


def test_device_histogram_divisors(gpu_available):
    """a PairHistogram over device counts divides like the reference for any divisor --
    only a positive divisor exact in float64 goes to the device (csa_pairs_upper_async), a negative or
    huge one is applied on the host, and zero raises ZeroDivisionError (analysis.py:86-88)."""
    import torch
    A = pkg("analysis")
    n = 37
    m = np.random.default_rng(5).integers(0, 1000, size=(n, n)).astype(np.int64)
    iu = np.triu_indices(n, 1)
    for divs in ([7], [-3], [-3, 7], [10 ** 30], [7, 10 ** 30], [2.5]):
        h = A.PairHistogram(n, counts=torch.from_numpy(m).cuda())
        for d in divs:
            h.turn_into_probabilities_by_dividing_all_elements_by_given_number(d)
        want = [int(x) for x in m[iu]]
        for d in divs:
            want = [x / d for x in want]
        assert h.upper().tolist() == want, divs
    h = A.PairHistogram(n, counts=torch.from_numpy(m).cuda())
    with pytest.raises(ZeroDivisionError):
        h.turn_into_probabilities_by_dividing_all_elements_by_given_number(0)


@pytest.mark.parametrize("name,k,S,chunk", [("sf_e_tight_110", 110, 9001, 1100), ("example_large_200", 200, 5003, 640),
                                            ("sf_e_110", 110, 4000, 4000)])
def test_chunked_xt_ring_vs_oracle(gpu_available, monkeypatch, name, k, S, chunk):
    """draw_count_chunks' fused form (every chunk's draw writes its XT into a 3-buffer ring, the pair kernel
    per chunk, counts from the diagonal at the end; more chunks than ring buffers, a ragged last chunk):
    counts, pair counts and the distinct count against the C oracle, and equal to the transpose form
    (CSA_DRAW_XT=0).  A single chunk goes through the same ring path (sf_e_110, chunk = S)."""
    import torch
    A = pkg("analysis")
    Dv = pkg("device")
    inst = pkg().read_instance(*inst_paths(name), k)
    used = []
    real = Dv.DevicePipeline._draw_xt_chunks

    def spy(self, *a, **kw):
        used.append(len(a[4]))
        return real(self, *a, **kw)

    monkeypatch.setattr(Dv.DevicePipeline, "_draw_xt_chunks", spy)
    enc = pkg().encode(inst.categories, inst.agents)
    # the multi-chunk entry (legacy_sample_device takes its one-chunk path only for S <= chunk; force the
    # chunk loop through the pipeline directly)
    pipe = Dv.DevicePipeline(enc, k, chunk, want_pairs=True, want_unique=True, pairs_buffer=True)
    W = enc.W
    panels = torch.empty(S * W, dtype=torch.int64, device="cuda")
    hashes = torch.empty(2 * S, dtype=torch.int64, device="cuda")
    pipe.reset(pairs=False)
    pipe.draw_count_chunks(13, 0, S, panels, hashes, chunk, overwrite_pairs=True, reset_counts=True)
    torch.cuda.synchronize()
    pipe.check_status()
    assert used == [(S + chunk - 1) // chunk]
    counts = pipe.counts.cpu().numpy()
    pairs = pipe.pairs.view(enc.n, enc.n).cpu().numpy()
    o = oracle_read(*inst_paths(name), k)
    rc, opanels, _, _ = coracle.draw(o, k, 13, 0, S)
    assert rc == 0
    assert np.array_equal(panels.cpu().numpy().view(np.uint64).reshape(S, W), opanels)
    assert np.array_equal(counts, coracle.counts(opanels, o.n))
    assert np.array_equal(np.triu(pairs), np.triu(coracle.pairs(opanels, o.n)))
    monkeypatch.setenv("CSA_DRAW_XT", "0")
    pipe2 = Dv.DevicePipeline(enc, k, chunk, want_pairs=True, want_unique=True, pairs_buffer=True)
    pipe2.reset(pairs=False)
    pipe2.draw_count_chunks(13, 0, S, panels, hashes, chunk, overwrite_pairs=True, reset_counts=True)
    torch.cuda.synchronize()
    assert used == [(S + chunk - 1) // chunk]                  # the transpose form this time
    assert np.array_equal(pipe2.counts.cpu().numpy(), counts)
    assert np.array_equal(np.triu(pipe2.pairs.view(enc.n, enc.n).cpu().numpy()), np.triu(pairs))


@pytest.mark.parametrize("config,job,chunk", [("sf_e_110", 70001, 16000), ("example_large_200", 50001, 9000)])
def test_bench_job_xt_from_draw_equals_transpose(gpu_available, config, job, chunk):
    """bench.py --job-panels with the draw writing XT (default, 3-buffer ring, counts from the diagonal) and
    with xt_count_kernel (--xt-from count): the same count and pair-triangle digests, distinct count and
    draw statistics."""
    import json
    import subprocess
    import sys
    from conftest import REPO
    out = {}
    for mode in ("draw", "count"):
        r = subprocess.run([sys.executable, "bench.py", "--config", config, "--job-panels", str(job), "--panels",
                            str(chunk), "--warmup", "1", "--no-cpu-baseline", "--no-api", "--xt-from", mode],
                           cwd=REPO, capture_output=True, text=True, timeout=240)
        assert r.returncode == 0, r.stderr[-2000:]
        out[mode] = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    assert "XT" in out["draw"]["config"]["pipeline"] and "XT" not in out["count"]["config"]["pipeline"]
    for key in ("job_unique", "job_count_sum", "job_pair_sum", "job_counts_sha256", "job_pairs_triu_sha256"):
        assert out["draw"]["checks"][key] == out["count"]["checks"][key], key
    assert out["draw"]["draw_stats"] == out["count"]["draw_stats"]
