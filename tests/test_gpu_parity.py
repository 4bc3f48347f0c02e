"""GPU parity: the HIP path (through the C ABI) vs the reference goldens and the C oracle.

Bar: panels, attempts, per-person counts, pair counts and distinct-panel counts
bit-exact; derived probabilities equal to the reference's floats (count / S is
correctly rounded on both sides, so the 1e-12 tolerance of the north star is
met with equality).
"""
import ctypes
import hashlib
import os

import numpy as np
import pytest

from conftest import PHILOX_CASES, golden, inst_paths, pkg
from oracle import coracle
from oracle.legacy_oracle import read_instance as oracle_read, draw_attempt, PhiloxRng, FAIL, NoCandidateError, \
    OracleInstance

pytestmark = pytest.mark.gpu


def _sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def _enc(name, k):
    P = pkg()
    inst = P.read_instance(*inst_paths(name), k)
    return inst, P.encode(inst.categories, inst.agents)


@pytest.mark.parametrize("case", PHILOX_CASES)
def test_sample_matches_reference_golden(gpu_available, case):
    A = pkg("analysis")
    g = golden(case)
    inst, enc = _enc(g["instance"], g["k"])
    raw = A.legacy_sample_raw(enc, g["k"], g["S"], g["seed"], want_pairs=True, want_panels=True,
                              want_attempts=True)
    assert _sha(raw.panels) == g["panels_sha256"]
    assert raw.attempts.tolist() == g["attempts"]
    assert raw.counts.tolist() == g["counts"]
    assert raw.unique == g["unique"]
    up = raw.pairs[np.triu_indices(enc.n, 1)]
    assert _sha(up) == g["pair_upper_sha256"]
    assert np.array_equal(np.diag(raw.pairs), raw.counts)
    assert _sha(up / g["S"]) == g["pair_prob_sha256"]        # the reference's float64 pair values


@pytest.mark.parametrize("case", PHILOX_CASES)
@pytest.mark.parametrize("chunk", [64, 1000])
def test_sample_chunked_pipeline_matches_golden(gpu_available, case, chunk, monkeypatch):
    """csa_legacy_sample's two-stream chunk pipeline (draw chunk c+1 while chunk c is counted) with
    small chunks, including ones that are not a multiple of 64 panels: identical to the goldens."""
    monkeypatch.setenv("CSA_SAMPLE_CHUNK", str(chunk))
    A = pkg("analysis")
    g = golden(case)
    inst, enc = _enc(g["instance"], g["k"])
    raw = A.legacy_sample_raw(enc, g["k"], g["S"], g["seed"], want_pairs=True, want_panels=True,
                              want_attempts=True)
    assert _sha(raw.panels) == g["panels_sha256"]
    assert raw.attempts.tolist() == g["attempts"]
    assert raw.counts.tolist() == g["counts"]
    assert raw.unique == g["unique"]
    assert _sha(raw.pairs[np.triu_indices(enc.n, 1)]) == g["pair_upper_sha256"]


@pytest.mark.parametrize("case", ["couples_s0", "example_small_20_s0", "sf_e_tight_110_s1", "pathological_5_s0"])
def test_legacy_find_pick_order(gpu_available, case):
    A = pkg("analysis")
    g = golden(case)
    inst, _ = _enc(g["instance"], g["k"])
    A.seed(g["seed"])
    batch = A.legacy_find_batch(inst.categories, inst.agents, g["k"], len(g["first_picks"]))
    assert batch == g["first_picks"]
    A.seed(g["seed"])
    one = [A.legacy_find(inst.categories, inst.agents, g["k"]) for _ in range(4)]
    assert one == g["first_picks"][:4]


def test_legacy_probabilities_api(gpu_available):
    A = pkg("analysis")
    g = golden("example_small_20_s0")
    inst, _ = _enc(g["instance"], g["k"])
    alloc, found, hist = A.legacy_probabilities(inst, g["S"], g["seed"])
    assert [alloc[i] for i in range(len(alloc))] == g["alloc"]
    assert len(found) == g["unique"]
    assert tuple(g["first_panels"][0]) in found
    up = hist.upper()
    assert up.tolist() == (np.asarray(g["pair_upper"]) / g["S"]).tolist()
    assert hist[(5, 3)] == hist[(3, 5)]


@pytest.mark.parametrize("name,k,S,seed", [("sf_e_110", 110, 20000, 7), ("sf_e_tight_110", 110, 5000, 3),
                                           ("example_large_200", 200, 4000, 11),
                                           ("synthetic8192_200", 200, 100000, 5), ("rejecty_6", 6, 50000, 9)])
def test_sample_matches_c_oracle(gpu_available, name, k, S, seed):
    A = pkg("analysis")
    inst, enc = _enc(name, k)
    begin = 123456789          # non-zero panel_begin: sharded runs start mid-stream
    N = pkg("_native")
    counts = np.zeros(enc.n, np.int64)
    pairs = np.zeros((enc.n, enc.n), np.int64)
    panels = np.zeros((S, enc.W), np.uint64)
    attempts = np.zeros(S, np.uint32)
    uniq = np.zeros(1, np.uint64)
    flags = N.CSA_WANT_PANELS | N.CSA_WANT_COUNTS | N.CSA_WANT_PAIRS | N.CSA_WANT_UNIQUE
    N.check(N.lib().csa_legacy_sample(enc.handle, k, seed, begin, S, flags, 0, N.ptr(panels), N.ptr(counts),
                                      N.ptr(pairs), N.ptr(uniq), N.ptr(attempts)))
    o = oracle_read(*inst_paths(name), k)
    rc, opanels, oatt, _ = coracle.draw(o, k, seed, begin, S)
    assert rc == 0
    assert np.array_equal(panels, opanels)
    assert np.array_equal(attempts, oatt)
    assert np.array_equal(counts, coracle.counts(opanels, enc.n))
    assert int(uniq[0]) == coracle.unique(opanels, enc.n)
    op = coracle.pairs(opanels, enc.n)          # n = 8192: 32 x 32 blocks of the 256 x 256 tiling
    assert np.array_equal(np.triu(pairs), np.triu(op))
    assert np.array_equal(np.diag(pairs), counts)


def test_full_size_properties_sf_e(gpu_available):
    """BASELINE config 2 size (10^6 panels): size-independent invariants + a sampled oracle check."""
    A = pkg("analysis")
    inst, enc = _enc("sf_e_110", 110)
    S, k = 10 ** 6, 110
    raw = A.legacy_sample_raw(enc, k, S, 0, want_pairs=True, want_panels=True, want_attempts=True)
    assert int(raw.counts.sum()) == k * S
    pc = np.unpackbits(raw.panels.view(np.uint8), axis=1).sum(axis=1)
    assert (pc == k).all()
    # row sums of the symmetric pair matrix = (k - 1) * counts
    iu = np.triu_indices(enc.n, 1)
    full = np.zeros_like(raw.pairs)
    full[iu] = raw.pairs[iu]
    full = full + full.T
    assert np.array_equal(full.sum(axis=1), (k - 1) * raw.counts)
    assert np.array_equal(np.diag(raw.pairs), raw.counts)
    assert raw.unique <= S
    # the distinct count (partitioned path at this size) equals an exact host count of the rows
    assert raw.unique == len(np.unique(raw.panels, axis=0))
    # spot-check three windows of the stream against the oracle
    o = oracle_read(*inst_paths("sf_e_110"), k)
    for begin in (0, 500000, S - 2000):
        rc, opanels, oatt, _ = coracle.draw(o, k, 0, begin, 2000)
        assert np.array_equal(raw.panels[begin:begin + 2000], opanels)
        assert np.array_equal(raw.attempts[begin:begin + 2000], oatt)


def test_find_random_sample_legacy_single_attempts(gpu_available):
    """legacy.py:178-200 surface: dict mutation + SelectionError, vs the oracle's draw_attempt."""
    import copy
    P = pkg()
    L = pkg("legacy")
    name, k = "pathological_5", 5
    inst = P.read_instance(*inst_paths(name), k)
    o = oracle_read(*inst_paths(name), k)
    src = PhiloxRng(4)
    L.seed(4)
    n_ok = n_fail = 0
    for attempt in range(40):
        cats = copy.deepcopy(inst.categories)
        people = copy.deepcopy(inst.agents)
        status, picks, sel, rem, present = draw_attempt(o, k, src.for_attempt(0, attempt))
        if status == FAIL:
            with pytest.raises(L.SelectionError):
                L.find_random_sample_legacy(cats, people, {}, k, False, [])
            n_fail += 1
            continue
        selected, lines = L.find_random_sample_legacy(cats, people, {}, k, False, [])
        n_ok += 1
        assert list(selected) == picks
        assert sorted(people) == [p for p in range(o.n) if present[p]]
        flat = [cats[c][f] for c in cats for f in cats[c]]
        assert [it["selected"] for it in flat] == sel
        assert [it["remaining"] for it in flat] == rem
    assert n_ok and n_fail


def test_no_candidate_raises_keyerror(gpu_available):
    """n=k=102, one feature with min 0: at step 101 ratio = -101 <= -100 -> KeyError (legacy.py:188)."""
    P = pkg()
    A = pkg("analysis")
    cats = {"c": {"f": {"min": 0, "max": 200, "selected": 0, "remaining": 102}}}
    agents = {i: {"c": "f"} for i in range(102)}
    inst = P.Instance(k=102, categories=cats, agents=agents)
    from oracle.legacy_oracle import OracleInstance
    o = OracleInstance(k=102, cat_names=["c"], feat_names=[("c", "f")], fmin=[0], fmax=[200], fcat=[0],
                       person_feat=[[0]] * 102)
    with pytest.raises(NoCandidateError):
        draw_attempt(o, 102, PhiloxRng(0).for_attempt(0, 0))
    with pytest.raises(KeyError):
        A.legacy_probabilities(inst, 10, 0)


def test_attempt_limit_and_bad_quotas(gpu_available):
    P = pkg()
    N = pkg("_native")
    A = pkg("analysis")
    # infeasible: needs 2 x0 and 2 y0 with k=2 but nobody holds both -> every attempt fails
    cats = {"x": {"x0": {"min": 2, "max": 2}, "x1": {"min": 0, "max": 2}},
            "y": {"y0": {"min": 2, "max": 2}, "y1": {"min": 0, "max": 2}}}
    agents = {0: {"x": "x0", "y": "y1"}, 1: {"x": "x0", "y": "y1"}, 2: {"x": "x1", "y": "y0"},
              3: {"x": "x1", "y": "y0"}}
    enc = P.encode(cats, agents)
    with pytest.raises(N.CsaError) as ei:
        A.legacy_sample_raw(enc, 2, 8, 0, want_pairs=False, want_panels=False, max_attempts=64)
    assert ei.value.code == N.CSA_E_ATTEMPT_LIMIT
    with pytest.raises(AssertionError):
        A.legacy_sample_raw(enc, 7, 8, 0)          # sum(max) = 4 < 7 (analysis.py:176)


def test_device_pipeline_matches_host_api(gpu_available):
    """The stream-ordered path used by bench.py / distributed.py == csa_legacy_sample."""
    import torch
    A = pkg("analysis")
    D = pkg("device")
    inst, enc = _enc("sf_e_110", 110)
    S = 30000
    raw = A.legacy_sample_raw(enc, 110, S, 2, want_pairs=True, want_panels=True)
    pipe = D.DevicePipeline(enc, 110, S)
    pipe.reset()
    # two shards through the same buffers: [0, S/2) and [S/2, S) accumulate
    half = S // 2
    pipe.run(2, 0, half)
    pipe.check_status()
    p0 = pipe.panels_view(half).copy()
    pipe.run(2, half, S - half)
    pipe.check_status()
    p1 = pipe.panels_view(S - half)
    assert np.array_equal(np.concatenate([p0, p1]), raw.panels)
    assert np.array_equal(pipe.counts.cpu().numpy(), raw.counts)
    iu = np.triu_indices(enc.n, 1)
    assert np.array_equal(pipe.pairs.cpu().numpy().reshape(enc.n, enc.n)[iu], raw.pairs[iu])
    torch.cuda.synchronize()


def _exchange_on_device(h, p, W, world, shards, cap, status):
    """The multi-GPU distinct-panel exchange with `world` simulated ranks on one device: each sender
    packs its shard (csa_exchange_pack_async), the all_to_all is done by slicing, each owner counts
    its segments (csa_unique_segments_async).  Returns (sum of owner counts, per-sender host copies
    of (hashes, panels, counts) segments)."""
    import torch
    D = pkg("distributed")
    N = pkg("_native")
    L = N.lib()
    sends = []
    for b, e in shards:
        sh = torch.zeros(world * cap * 2, dtype=torch.int64, device="cuda")
        sp = torch.zeros(world * cap * W, dtype=torch.int64, device="cuda")
        sc = torch.zeros(world, dtype=torch.int64, device="cuda")
        sb = int(L.csa_exchange_scratch_bytes(max(e - b, 1)))
        scratch = torch.empty((sb + 7) // 8, dtype=torch.int64, device="cuda")
        N.check(L.csa_exchange_pack_async(N.ptr(h[2 * b:]), N.ptr(p[b * W:]), e - b, W, world, cap, N.ptr(scratch),
                                          scratch.numel() * 8, N.ptr(sh), N.ptr(sp), N.ptr(sc), N.ptr(status), None))
        sends.append((sh, sp, sc))
    torch.cuda.synchronize()
    total = 0
    table = D.HashTable(world * cap, h.device)
    for r in range(world):
        rh = torch.cat([sh[r * cap * 2:(r + 1) * cap * 2] for sh, _, _ in sends])
        rp = torch.cat([sp[r * cap * W:(r + 1) * cap * W] for _, sp, _ in sends])
        rc = torch.stack([sc[r] for _, _, sc in sends])
        table.count.zero_()
        N.check(L.csa_unique_segments_async(N.ptr(rh), N.ptr(rp), world, cap, N.ptr(rc), W, N.ptr(table.table),
                                            table.slots, N.ptr(table.count), N.ptr(status), None))
        torch.cuda.synchronize()
        total += int(table.count.item())
    host = [(sh.cpu().numpy().view(np.uint64).reshape(world, cap, 2), sp.cpu().numpy().view(np.uint64).reshape(world, cap, W),
             sc.cpu().numpy()) for sh, sp, sc in sends]
    return total, host


@pytest.mark.parametrize("world", [1, 2, 3, 8])
def test_exchange_exact_on_device(gpu_available, world):
    """Multi-GPU distinct-panel exchange on one device (world simulated ranks, contiguous shards):
    every sender's owner segments hold exactly its local DISTINCT panels (host mirror
    segment_buckets), the owners' exact counts sum to the global distinct count with duplicates
    split across senders, and a forged hash collision between two different panels still counts
    twice (bitmask comparison, not hash equality)."""
    import torch
    D = pkg("distributed")
    o = oracle_read(*inst_paths("example_small_20"), 20)
    rc, panels, _, _ = coracle.draw(o, 20, 3, 0, 5000)
    panels = np.concatenate([panels, panels[:700], panels[2000:2300]])     # duplicates, some in other shards
    W = panels.shape[1]
    hashes = D.panel_hashes(panels)
    hashes[1000] = hashes[0]              # forged collision: panel 1000 (no duplicate) differs from panel 0
    assert not np.array_equal(panels[0], panels[1000])
    want = coracle.unique(panels, o.n)
    assert want == 5000
    h = torch.from_numpy(hashes.ravel().view(np.int64).copy()).cuda()
    p = torch.from_numpy(panels.ravel().view(np.int64).copy()).cuda()
    status = torch.zeros(4, dtype=torch.int32, device="cuda")
    shards = [D.shard_range(len(panels), world, r) for r in range(world)]
    cap = D.exchange_capacity(max(e - b for b, e in shards), world)
    total, host = _exchange_on_device(h, p, W, world, shards, cap, status)
    assert int(status[0].item()) == 0
    assert total == want
    for (b, e), (sh, sp, sc) in zip(shards, host):
        mh, mp, mc = D.segment_buckets(hashes[b:e], panels[b:e], world, cap)
        assert sc.tolist() == mc.tolist()
        for w in range(world):
            got = sorted(map(tuple, np.concatenate([sh[w, : sc[w]], sp[w, : sc[w]]], axis=1).tolist()))
            exp = sorted(map(tuple, np.concatenate([mh[w, : mc[w]], mp[w, : mc[w]]], axis=1).tolist()))
            assert got == exp


def _keys_exchange_on_device(enc, k, seed, h, p, W, world, shards, cap, status):
    """The 24-byte exchange with `world` simulated ranks on one device: each sender packs keys
    (csa_exchange_keys_async, global index = shard begin + local index), the all_to_all is done by
    slicing, each owner counts (csa_unique_keys_async, re-drawing its hash-matched keys)."""
    import torch
    N = pkg("_native")
    L = N.lib()
    sends = []
    for b, e in shards:
        sk = torch.zeros(world * cap * 3, dtype=torch.int64, device="cuda")
        sc = torch.zeros(world, dtype=torch.int64, device="cuda")
        sb = int(L.csa_exchange_scratch_bytes(max(e - b, 1)))
        scratch = torch.empty((sb + 7) // 8, dtype=torch.int64, device="cuda")
        N.check(L.csa_exchange_keys_async(N.ptr(h[2 * b:]), N.ptr(p[b * W:]), e - b, W, b, world, cap, N.ptr(scratch),
                                          scratch.numel() * 8, N.ptr(sk), N.ptr(sc), N.ptr(status), None))
        sends.append((sk, sc))
    torch.cuda.synchronize()
    total = 0
    ob = int(L.csa_unique_keys_scratch_bytes(world * cap, W))
    scr = torch.empty((ob + 7) // 8, dtype=torch.int64, device="cuda")
    for r in range(world):
        rk = torch.cat([sk[r * cap * 3:(r + 1) * cap * 3] for sk, _ in sends])
        rc = torch.stack([sc[r] for _, sc in sends])
        u = torch.zeros(1, dtype=torch.int64, device="cuda")
        N.check(L.csa_unique_keys_async(enc.handle, k, seed, 0, N.ptr(rk), world, cap, N.ptr(rc), N.ptr(scr), ob,
                                        N.ptr(u), N.ptr(status), None))
        torch.cuda.synchronize()
        total += int(u.item())
    return total, [(sk.cpu().numpy().view(np.uint64).reshape(world, cap, 3), sc.cpu().numpy()) for sk, sc in sends]


@pytest.mark.parametrize("world", [1, 2, 3, 8])
@pytest.mark.parametrize("case", ["couples", "forged", "forged_dups"])
def test_exchange_keys_exact_on_device(gpu_available, world, case):
    """The 24-byte exchange (keys = 128-bit hash + global panel index; the owner re-draws hash-matched
    keys and compares bitmasks): the owners' counts sum to the exact distinct count -- duplicates
    split across senders (couples: 100 distinct panels), a forged hash collision between two
    different panels (counted twice), and a forged collision whose other panel is itself
    duplicated on several ranks (still counted once)."""
    import torch
    A = pkg("analysis")
    D = pkg("distributed")
    name, k, S, seed = (("example_small_20", 20, 5000, 3) if case == "forged" else
                        ("couples_panel_from_twenty_people_no_constraints_2", 2, 20000, 5))
    inst, enc = _enc(name, k)
    panels = A.legacy_sample_raw(enc, k, S, seed, want_pairs=False, want_panels=True).panels
    W = panels.shape[1]
    hashes = D.panel_hashes(panels)
    want = coracle.unique(panels, enc.n)
    if case == "forged":
        assert want == S
        assert not np.array_equal(panels[0], panels[1000])
        hashes[1000] = hashes[0]
    elif case == "forged_dups":
        x = panels[0]
        y = next(r for r in panels if not np.array_equal(r, x))
        hy = D.panel_hashes(y[None])[0]
        same_x = (panels == x).all(axis=1)
        hashes[same_x] = hy                 # every copy of panel x now hashes like panel y
        assert same_x.sum() > world and want == 100
    h = torch.from_numpy(hashes.ravel().view(np.int64).copy()).cuda()
    p = torch.from_numpy(panels.ravel().view(np.int64).copy()).cuda()
    status = torch.zeros(4, dtype=torch.int32, device="cuda")
    shards = [D.shard_range(S, world, r) for r in range(world)]
    cap = D.exchange_capacity(max(e - b for b, e in shards), world)
    total, host = _keys_exchange_on_device(enc, k, seed, h, p, W, world, shards, cap, status)
    assert int(status[0].item()) == 0
    assert total == want
    # every sender's keys: one per local distinct panel, owner h1 % world, index inside its shard
    for (b, e), (sk, sc) in zip(shards, host):
        mh, mp, mc = D.segment_buckets(hashes[b:e], panels[b:e], world, cap)
        assert sc.tolist() == mc.tolist()
        for w in range(world):
            keys = sk[w, : sc[w]]
            assert ((keys[:, 2] >= b) & (keys[:, 2] < e)).all()
            assert np.array_equal(hashes[keys[:, 2].astype(np.int64)], keys[:, :2])
            assert sorted(map(tuple, panels[keys[:, 2].astype(np.int64)].tolist())) == sorted(map(tuple, mp[w, : mc[w]].tolist()))


def test_exchange_overflow_raises(gpu_available):
    """A segment past its capacity is an error in the status block (never a silently short count)."""
    import torch
    D = pkg("distributed")
    N = pkg("_native")
    rng = np.random.default_rng(5)
    panels = rng.integers(0, 2 ** 63, size=(1000, 3), dtype=np.int64).astype(np.uint64)
    hashes = D.panel_hashes(panels)
    h = torch.from_numpy(hashes.ravel().view(np.int64).copy()).cuda()
    p = torch.from_numpy(panels.ravel().view(np.int64).copy()).cuda()
    status = torch.zeros(4, dtype=torch.int32, device="cuda")
    _exchange_on_device(h, p, 3, 2, [(0, 1000)], 100, status)
    st = status.cpu().numpy().astype(np.uint32)
    assert st[0] == N.CSA_E_UNSUPPORTED
    with pytest.raises(N.CsaError):
        N.check(N.lib().csa_status_decode(N.ptr(st)))


def test_device_hashes_match_host_mirror(gpu_available):
    """The draw kernel's 128-bit panel hash == distributed.panel_hashes (used by the gloo path)."""
    D = pkg("distributed")
    Dv = pkg("device")
    inst, enc = _enc("sf_e_110", 110)
    pipe = Dv.DevicePipeline(enc, 110, 4096, want_pairs=False)
    pipe.reset()
    pipe.run(1, 77, 4096)
    pipe.check_status()
    dev_h = pipe.hashes.cpu().numpy().view(np.uint64).reshape(-1, 2)
    assert np.array_equal(dev_h, D.panel_hashes(pipe.panels_view(4096)))


@pytest.mark.parametrize("n", [1, 7, 110, 257, 1727])
def test_pairs_pack_roundtrip(gpu_available, n):
    """csa_pairs_pack/unpack_async: the upper triangle (incl. diagonal) packed row-major into int32
    and written back; the strict lower triangle is left untouched."""
    import torch
    N = pkg("_native")
    rng = np.random.default_rng(n)
    m = rng.integers(0, 2 ** 31 - 1, size=(n, n), dtype=np.int64)
    d = torch.from_numpy(m.reshape(-1)).cuda()
    packed = torch.empty(n * (n + 1) // 2, dtype=torch.int32, device="cuda")
    N.check(N.lib().csa_pairs_pack_async(N.ptr(d), n, N.ptr(packed), None))
    torch.cuda.synchronize()
    iu = np.triu_indices(n)
    assert np.array_equal(packed.cpu().numpy().astype(np.int64), m[iu])
    packed.mul_(2)
    lower = np.tril_indices(n, -1)
    N.check(N.lib().csa_pairs_unpack_async(N.ptr(packed), n, N.ptr(d), None))
    torch.cuda.synchronize()
    back = d.cpu().numpy().reshape(n, n)
    assert np.array_equal(back[iu], (2 * m[iu]).astype(np.int32).astype(np.int64))
    assert np.array_equal(back[lower], m[lower])


def test_combine_rccl_world1(gpu_available):
    """distributed.combine over a one-rank RCCL group on the GPU: the packed int32 pair all-reduce,
    the count all-reduce and the hash all-to-all leave the single-GPU results unchanged."""
    import socket
    import torch
    import torch.distributed as dist
    A = pkg("analysis")
    Dd = pkg("distributed")
    Dv = pkg("device")
    inst, enc = _enc("sf_e_110", 110)
    S = 20000
    pipe = Dv.DevicePipeline(enc, 110, S)
    pipe.reset()
    pipe.run(5, 0, S)
    pipe.check_status()
    want_counts = pipe.counts.cpu().numpy().copy()
    want_pairs = pipe.pairs.cpu().numpy().reshape(enc.n, enc.n).copy()
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    dist.init_process_group("nccl", init_method="tcp://127.0.0.1:%d" % port, rank=0, world_size=1)
    try:
        counts, pairs, u = Dd.combine(pipe.counts, pipe.pairs, pipe.hashes[: 2 * S], pipe.panels[: S * enc.W], enc.W,
                                      stream=pipe.stream, pair_bound=S, status=pipe.status)
        torch.cuda.synchronize()
        got_pairs = pairs.cpu().numpy().reshape(enc.n, enc.n)
    finally:
        dist.destroy_process_group()
    assert np.array_equal(counts.cpu().numpy(), want_counts)
    iu = np.triu_indices(enc.n)
    assert np.array_equal(got_pairs[iu], want_pairs[iu])
    assert int(u.item()) == S      # sf_e_110 at 2e4 panels: all distinct


def _rccl_world1():
    import socket
    import torch.distributed as dist
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    dist.init_process_group("nccl", init_method="tcp://127.0.0.1:%d" % port, rank=0, world_size=1)


def _load_in_cpu_child(path):
    """sorted(found_panels) and len() of a pickled result, loaded in a child process with no GPU."""
    import subprocess
    import sys
    from conftest import REPO
    env = dict(os.environ, HIP_VISIBLE_DEVICES="-1", CUDA_VISIBLE_DEVICES="-1", ROCR_VISIBLE_DEVICES="-1")
    code = ("import pickle, sys; sys.path.insert(0, %r); import torch; assert not torch.cuda.is_available(); "
            "a, f, h = pickle.load(open(%r, 'rb')); print(repr(sorted(f))); print(len(f))" % (REPO, str(path)))
    out = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr
    got, ln = out.stdout.strip().splitlines()
    return got, int(ln)


@pytest.mark.parametrize("name,k,S,chunk", [("sf_e_110", 110, 30001, 7000),
                                            ("couples_panel_from_twenty_people_no_constraints_2", 2, 20000, 0),
                                            ("synthetic8192_200", 200, 3000, 1000)])
@pytest.mark.parametrize("force_exchange", ["0", "1"])
def test_distributed_call_rccl_world1(gpu_available, monkeypatch, tmp_path, name, k, S, chunk, force_exchange):
    """legacy_probabilities_distributed over a one-rank RCCL group (the product path's own
    collectives: packed pair all_reduce, the 24-byte key exchange, one all_reduce of counts +
    statistics + distinct count): equal to legacy_probabilities on one GPU -- alloc, pair values,
    distinct count, draw statistics, found_panels -- on the first call and on a second call that
    reuses the cached pipeline and exchange.  With the exchange, found_panels keep nothing: reading
    them re-draws the job on this GPU (csa_redraw_async) without a collective, the re-draw leaves the
    instance's draw statistics alone, and the pickle loads in a process without a GPU.  The call
    leaves the caller's current device as it found it."""
    import pickle
    import torch
    import torch.distributed as dist
    A = pkg("analysis")
    Dd = pkg("distributed")
    if chunk:
        monkeypatch.setenv("CSA_SHARD_CHUNK", str(chunk))
    monkeypatch.setenv("CSA_FORCE_EXCHANGE", force_exchange)   # 1: the 24-byte key exchange over RCCL
    inst = pkg().read_instance(*inst_paths(name), k)
    alloc, found, hist = A.legacy_probabilities(inst, S, 9)
    stats = dict(A.LAST_RUN_STATS)
    want_up, want_found = np.array(hist.upper()), sorted(found)
    dev0 = torch.cuda.current_device()
    _rccl_world1()
    try:
        for call in range(2):
            tm = {}
            a2, f2, h2 = Dd.legacy_probabilities_distributed(inst, S, 9, timings=tm)
            assert torch.cuda.current_device() == dev0
            assert a2 == alloc and len(f2) == len(found) and A.LAST_RUN_STATS == stats
            assert np.array_equal(h2.upper(), want_up)
            if force_exchange == "1":
                assert f2._redraw is not None and f2._packed is None      # nothing kept, nothing sent
            enc = A.encode_cached(inst.categories, inst.agents)
            before = A.draw_stats(enc)
            assert sorted(f2) == want_found
            assert A.draw_stats(enc) == before          # the re-draw is not counted as new draws
            assert tm["total_ms"] > 0
        a3, f3, h3 = Dd.legacy_probabilities_distributed(inst, S, 9)
        with open(tmp_path / "r.pkl", "wb") as f:
            pickle.dump((a3, f3, h3), f)
        got, ln = _load_in_cpu_child(tmp_path / "r.pkl")
        assert got == repr(want_found) and ln == len(found)
        a4, f4, _ = Dd.legacy_probabilities_distributed(inst, S, 9, keep_panels=False)
        assert len(f4) == len(found)
        with pytest.raises(RuntimeError, match="not kept"):
            sorted(f4)
    finally:
        dist.destroy_process_group()


def _no_candidate_instance():
    """n = k = 102, one feature with min 0: every panel raises KeyError at step 101 (legacy.py:188)."""
    cats = {"c": {"f": {"min": 0, "max": 200, "selected": 0, "remaining": 102}}}
    return pkg().Instance(k=102, categories=cats, agents={i: {"c": "f"} for i in range(102)})


def _feasible_102(k):
    """The same pool shape (n = 102, W = 2, one category) split over two features: every draw succeeds."""
    cats = {"c": {"f": {"min": 0, "max": 200, "selected": 0, "remaining": 51},
                  "g": {"min": 0, "max": 200, "selected": 0, "remaining": 51}}}
    return pkg().Instance(k=k, categories=cats, agents={i: {"c": "fg"[i % 2]} for i in range(102)})


def test_distributed_no_candidate_rccl_world1(gpu_available, monkeypatch):
    """The sharded call's failure path under a one-rank RCCL group with the exchange forced on: a
    shard whose every draw raised still enters the pair all_reduce and the key exchange (on its
    unwritten panels), and the call raises KeyError, as the one-GPU call (legacy.py:188)."""
    Dd = pkg("distributed")
    import torch.distributed as dist
    monkeypatch.setenv("CSA_FORCE_EXCHANGE", "1")
    _rccl_world1()
    try:
        for S in (10, 5000):
            with pytest.raises(KeyError):
                Dd.legacy_probabilities_distributed(_no_candidate_instance(), S, 0)
        # the next call on the same group is unaffected
        a, f, _ = Dd.legacy_probabilities_distributed(_feasible_102(20), 300, 1)
        assert abs(sum(a.values()) - 20) < 1e-9 and len(f) > 1
    finally:
        dist.destroy_process_group()


def _fail_worker(rank, world, port, out_dir):
    import os
    import sys
    import torch.distributed as dist
    from conftest import REPO
    sys.path.insert(0, REPO)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        Dd = pkg("distributed")
        # rank 0: a feasible instance whose exchange overflows its (forced tiny) segments -- an
        # exchange error, CSA_E_UNSUPPORTED (5); rank 1: every draw raises KeyError, CSA_E_NO_CANDIDATE
        # (3).  The collectives have the same sizes (n = 102 on both).  Every rank must raise the DRAW
        # error: a MAX of the raw codes would hand rank 0 the exchange's instead
        Dd.exchange_capacity = lambda n_local, world_: 1
        own = []
        real_decode = Dd._decode_status

        def decode(words, reduced):          # this rank's own status code, then the agreed one
            own.append((int(words[0]), int(reduced)))
            return real_decode(words, reduced)

        Dd._decode_status = decode
        inst = _feasible_102(20) if rank == 0 else _no_candidate_instance()
        try:
            Dd.legacy_probabilities_distributed(inst, 4000, 0)
            outcome = "ok"
        except KeyError:
            outcome = "KeyError"
        except Exception as e:      # noqa: BLE001
            outcome = "%s: %s" % (type(e).__name__, e)
        outcome += " own=%d agreed=%d" % own[0] if own else " (no status decoded)"
        with open(os.path.join(out_dir, "rank%d.txt" % rank), "w") as f:
            f.write(outcome)
        dist.barrier()
    finally:
        dist.destroy_process_group()


def test_distributed_draw_error_outranks_exchange_error(gpu_available, tmp_path):
    """Two ranks (gloo, one GPU): a draw error on one rank and an exchange error on the other -> every
    rank raises KeyError (the exchange's status never masks the draw's)."""
    import socket
    import torch.multiprocessing as mp
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    mp.spawn(_fail_worker, args=(2, port, str(tmp_path)), nprocs=2, join=True)
    N = pkg("_native")
    # rank 0's own block held the exchange's overflow, rank 1's the draw's KeyError; both raise KeyError
    assert [(tmp_path / ("rank%d.txt" % r)).read_text() for r in range(2)] == [
        "KeyError own=%d agreed=%d" % (N.CSA_E_UNSUPPORTED, N.CSA_E_NO_CANDIDATE),
        "KeyError own=%d agreed=%d" % (N.CSA_E_NO_CANDIDATE, N.CSA_E_NO_CANDIDATE)]


@pytest.mark.parametrize("name,k,S", [("couples_panel_from_twenty_people_no_constraints_2", 2, 300000),
                                      ("example_small_20", 20, 200000), ("sf_e_110", 110, 100000),
                                      ("rejecty_6", 6, 400000)])
def test_unique_partitioned_matches_oracle(gpu_available, name, k, S):
    """csa_unique_async at sizes that take the partitioned path (duplicate-heavy couples / rejecty:
    a few hundred distinct panels; sf_e: all distinct) == the C oracle's exact count, and == the
    single-table path (CSA_UNIQUE_PART=0)."""
    import os
    A = pkg("analysis")
    inst, enc = _enc(name, k)
    o = oracle_read(*inst_paths(name), k)
    rc, opanels, _, _ = coracle.draw(o, k, 13, 0, S)
    assert rc == 0
    want = coracle.unique(opanels, o.n)
    got = {}
    for mode in ("1", "0"):
        os.environ["CSA_UNIQUE_PART"] = mode
        try:
            got[mode] = A.legacy_sample_raw(enc, k, S, 13, want_pairs=False, want_panels=False).unique
        finally:
            os.environ.pop("CSA_UNIQUE_PART", None)
    assert got["1"] == got["0"] == want


def _dist_worker(rank, world, port, out_dir, name, k, S, seed):
    import os
    import sys
    import torch.distributed as dist
    from conftest import REPO
    sys.path.insert(0, REPO)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import pickle
        A = pkg("analysis")
        inst = pkg().read_instance(*inst_paths(name), k)
        alloc, found, hist = A.legacy_probabilities(inst, S, seed)      # world > 1: sharded
        dist.barrier()
        entered = []
        names = ("send", "recv", "isend", "irecv", "all_reduce", "all_gather", "all_to_all_single", "broadcast",
                 "barrier")
        real = {nm: getattr(dist, nm) for nm in names}
        for nm in names:
            setattr(dist, nm, (lambda nm_: lambda *a, **kw: (entered.append(nm_), real[nm_](*a, **kw))[1])(nm))
        try:
            # the LAST rank reads its found_panels alone (re-drawn on its GPU), no collective entered
            if rank == world - 1:
                tuples = sorted(found)
                assert all(t in found for t in tuples[:3])
                np.save(os.path.join(out_dir, "found.npy"), np.array(tuples))
                with open(os.path.join(out_dir, "result.pkl"), "wb") as f:
                    pickle.dump((alloc, found, hist), f)
            assert entered == []
        finally:
            for nm in names:
                setattr(dist, nm, real[nm])
        if rank == 0:
            np.save(os.path.join(out_dir, "alloc.npy"), np.array([alloc[i] for i in range(len(alloc))]))
            np.save(os.path.join(out_dir, "upper.npy"), hist.upper())
            np.save(os.path.join(out_dir, "unique.npy"), np.array([len(found)]))
        dist.barrier()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("name,k,S,seed,chunk", [("sf_e_110", 110, 9001, 3, 0),
                                                 ("sf_e_110", 110, 9001, 4, 1700),
                                                 ("couples_panel_from_twenty_people_no_constraints_2", 2, 5000, 1, 0),
                                                 ("couples_panel_from_twenty_people_no_constraints_2", 2, 5000, 2,
                                                  700)])
def test_legacy_probabilities_distributed_gloo(gpu_available, tmp_path, monkeypatch, name, k, S, seed, chunk):
    """analysis.legacy_probabilities with a 2-rank process group (both ranks on this GPU, gloo:
    RCCL refuses two ranks on one device): the sharded draw (``chunk``: each rank's shard drawn in
    chunks of that many panels, counted beside the next chunk's draw), the exact panel exchange, and
    found_panels re-drawn by one rank alone (no collective) -- `in`, and the pickled tuple (loaded in
    a process without a GPU) equal the single-GPU result."""
    import socket
    import torch.multiprocessing as mp
    A = pkg("analysis")
    if chunk:
        monkeypatch.setenv("CSA_SHARD_CHUNK", str(chunk))
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    mp.spawn(_dist_worker, args=(2, port, str(tmp_path), name, k, S, seed), nprocs=2, join=True)
    inst = pkg().read_instance(*inst_paths(name), k)
    alloc, found, hist = A.legacy_probabilities(inst, S, seed)
    assert np.load(tmp_path / "alloc.npy").tolist() == [alloc[i] for i in range(len(alloc))]
    assert np.array_equal(np.load(tmp_path / "upper.npy"), hist.upper())
    assert int(np.load(tmp_path / "unique.npy")[0]) == len(found)
    assert np.load(tmp_path / "found.npy").tolist() == [list(p) for p in sorted(found)]
    assert A.LAST_RUN_STATS["attempts"] >= S
    got, ln = _load_in_cpu_child(tmp_path / "result.pkl")
    assert got == repr(sorted(found)) and ln == len(found)


def test_n16384_boundary(gpu_available):
    """The largest pool the header admits (n = 16384, W = 256): draw_kernel<16> for the draw,
    xt_count_kernel over two column ranges, 64 x 64 triangle blocks of X^T X.  Panels, attempts,
    counts and the distinct count vs the C oracle; pair counts vs a plain PyTorch fp32 X^T X."""
    import torch
    P = pkg()
    A = pkg("analysis")
    rng = np.random.default_rng(16384)
    n, k, S = 16384, 300, 400
    shares = {"a": [0.4, 0.3, 0.2, 0.1], "b": [0.5, 0.3, 0.2]}
    cats = {c: {"%s%d" % (c, j): {"min": int(0.9 * k * p), "max": int(np.ceil(1.1 * k * p)) + 1}
                for j, p in enumerate(ps)} for c, ps in shares.items()}
    agents = {i: {c: "%s%d" % (c, rng.choice(len(ps), p=ps)) for c, ps in shares.items()} for i in range(n)}
    enc = P.encode(cats, agents)
    raw = A.legacy_sample_raw(enc, k, S, 21, want_pairs=True, want_panels=True, want_attempts=True)
    feats = [(c, f) for c in cats for f in cats[c]]
    o = OracleInstance(k=k, cat_names=list(cats), feat_names=feats,
                       fmin=[cats[c][f]["min"] for c, f in feats], fmax=[cats[c][f]["max"] for c, f in feats],
                       fcat=[list(cats).index(c) for c, f in feats],
                       person_feat=[[feats.index((c, agents[i][c])) for c in cats] for i in range(n)])
    rc, opanels, oatt, _ = coracle.draw(o, k, 21, 0, S)
    assert rc == 0
    assert np.array_equal(raw.panels, opanels)
    assert np.array_equal(raw.attempts, oatt)
    assert np.array_equal(raw.counts, coracle.counts(opanels, n))
    assert raw.unique == coracle.unique(opanels, n)
    X = torch.from_numpy(np.unpackbits(opanels.view(np.uint8), axis=1, bitorder="little")[:, :n]).cuda().float()
    ref = (X.T @ X).to(torch.int64).cpu().numpy()
    assert np.array_equal(np.triu(raw.pairs), np.triu(ref))


@pytest.mark.parametrize("name,k,S", [("sf_e_110", 110, 160), ("example_large_200", 200, 60)])
def test_sample_from_state_at_max(gpu_available, name, k, S):
    """A start state (the dicts' own "selected" counters, analysis.py:147-148) in which a feature
    already sits at its max: its holders stay in the pool, picking one takes it past max, and no
    cascade follows (legacy.py:113-114 tests ==).  The batch draw must route such a state to the
    exact-equality kernel; panels equal the Python oracle's loop from the same state."""
    import copy
    A = pkg("analysis")
    P = pkg()
    inst, _ = _enc(name, k)
    o = oracle_read(*inst_paths(name), k)
    cats = copy.deepcopy(inst.categories)
    # the live feature with the most holders whose max is reached
    pool = o.pool_counts()
    g = max((f for f in range(o.F) if o.fmax[f] > 0), key=lambda f: pool[f])
    c, v = o.feat_names[g]
    cats[c][v]["selected"] = o.fmax[g]
    enc = P.encode(cats, inst.agents)
    assert enc.feat_keys[g] == (c, v) and enc.sel0[g] == o.fmax[g]
    seed = 17
    raw = A.legacy_sample_raw(enc, k, S, seed, want_pairs=False, want_panels=True, want_attempts=True)
    sel0 = [0] * o.F
    sel0[g] = o.fmax[g]
    src = PhiloxRng(seed)
    rows = []
    for panel in range(S):
        a = 0
        while True:
            st, picks, sel, _, _ = draw_attempt(o, k, src.for_attempt(panel, a), sel=sel0)
            if st == 0 and all(sel[f] >= o.fmin[f] for f in range(o.F)):
                break
            a += 1
        row = np.zeros(enc.W, np.uint64)
        for p_ in picks:
            row[p_ >> 6] |= np.uint64(1) << np.uint64(p_ & 63)
        rows.append(row)
        assert raw.attempts[panel] == a + 1
    assert np.array_equal(raw.panels, np.stack(rows))
