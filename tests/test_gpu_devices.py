"""csa_legacy_sample_devices: several devices of one process behind the C ABI (SURVEY.md §8(b)'s
n_devices).  The GPU box has one MI355X, so the shards run as replicas on device 0 (a device may
repeat in the list); the sharding, the replicas' state mirroring and the exact combine (counts and
pairs summed, local distinct sets gathered and counted by hash AND bitmask) are the same code a
multi-GPU list takes.  Bar: bit-identical to csa_legacy_sample over the same panel range."""
import numpy as np
import pytest

from conftest import golden, inst_paths, pkg

pytestmark = pytest.mark.gpu


def _enc(name, k):
    P = pkg()
    inst = P.read_instance(*inst_paths(name), k)
    return inst, P.encode(inst.categories, inst.agents)


def _same(a, b, n):
    assert np.array_equal(a.panels, b.panels)
    assert np.array_equal(a.attempts, b.attempts)
    assert np.array_equal(a.counts, b.counts)
    assert a.unique == b.unique
    iu = np.triu_indices(n)
    assert np.array_equal(a.pairs[iu], b.pairs[iu])


@pytest.mark.parametrize("name,k,S,seed,shards", [
    ("couples_panel_from_twenty_people_no_constraints_2", 2, 10000, 0, 3),   # duplicates across every shard
    ("example_small_20", 20, 10000, 0, 2),
    ("sf_e_110", 110, 200000, 4, 3),          # partitioned distinct pass per shard (>= 65536 panels)
    ("sf_e_tight_110", 110, 3001, 1, 5),      # restarts, ragged shards
    ("synthetic8192_200", 200, 5000, 2, 2),   # draw_wide_kernel, n = 8192 pair sums
])
def test_devices_equal_single_call(gpu_available, name, k, S, seed, shards):
    A = pkg("analysis")
    _, enc = _enc(name, k)
    one = A.legacy_sample_raw(enc, k, S, seed, want_pairs=True, want_panels=True, want_attempts=True)
    many = A.legacy_sample_raw(enc, k, S, seed, want_pairs=True, want_panels=True, want_attempts=True,
                               devices=[0] * shards)
    _same(one, many, enc.n)


def test_devices_match_golden(gpu_available):
    A = pkg("analysis")
    g = golden("couples_s0")
    _, enc = _enc(g["instance"], g["k"])
    raw = A.legacy_sample_raw(enc, g["k"], g["S"], g["seed"], devices=[0, 0, 0, 0])
    assert raw.counts.tolist() == g["counts"]
    assert raw.unique == g["unique"]


def test_devices_more_shards_than_panels(gpu_available):
    """Empty shards (n_panels < n_shards) contribute nothing."""
    A = pkg("analysis")
    _, enc = _enc("example_small_20", 20)
    one = A.legacy_sample_raw(enc, 20, 3, 9, want_attempts=True)
    many = A.legacy_sample_raw(enc, 20, 3, 9, want_attempts=True, devices=[0] * 7)
    _same(one, many, enc.n)
    zero = A.legacy_sample_raw(enc, 20, 0, 9, devices=[0, 0])
    assert zero.unique == 0 and not zero.counts.any()


def test_devices_follow_state_and_address(gpu_available):
    """Replicas re-mirror csa_instance_set_state / csa_instance_set_address between calls."""
    A = pkg("analysis")
    N = pkg("_native")
    L = N.lib()
    _, enc = _enc("example_large_200", 200)
    base_one = A.legacy_sample_raw(enc, 200, 2000, 3, want_attempts=True)
    base_many = A.legacy_sample_raw(enc, 200, 2000, 3, want_attempts=True, devices=[0, 0])
    _same(base_one, base_many, enc.n)
    # a partially used state: agents 0..99 gone, their features' remaining reduced
    present = np.zeros(enc.W, np.uint64)
    for p in range(100, enc.n):
        present[p >> 6] |= np.uint64(1) << np.uint64(p & 63)
    rem = np.asarray(enc.rem0, np.int32).copy()
    for p in range(100):
        for g in enc.person_feat[p]:
            rem[g] -= 1
    sel = np.zeros(enc.F, np.int32)
    N.check(L.csa_instance_set_state(enc.handle, N.ptr(sel), N.ptr(rem), N.ptr(present)))
    try:
        one = A.legacy_sample_raw(enc, 200, 1500, 3, want_attempts=True)
        many = A.legacy_sample_raw(enc, 200, 1500, 3, want_attempts=True, devices=[0, 0, 0])
        _same(one, many, enc.n)
        assert not one.counts[:100].any()
        # address rings: consecutive agents pair up
        ring = np.arange(enc.n, dtype=np.int32)
        ring[0:enc.n - 1:2], ring[1:enc.n:2] = np.arange(1, enc.n, 2), np.arange(0, enc.n - 1, 2)
        N.check(L.csa_instance_set_address(enc.handle, N.ptr(ring)))
        one = A.legacy_sample_raw(enc, 200, 600, 5, want_attempts=True)
        many = A.legacy_sample_raw(enc, 200, 600, 5, want_attempts=True, devices=[0, 0])
        _same(one, many, enc.n)
    finally:
        N.check(L.csa_instance_set_address(enc.handle, None))
        N.check(L.csa_instance_set_state(enc.handle, None, None, None))
    again = A.legacy_sample_raw(enc, 200, 2000, 3, want_attempts=True, devices=[0, 0])
    _same(base_one, again, enc.n)


def test_devices_legacy_probabilities(gpu_available):
    A = pkg("analysis")
    g = golden("example_small_20_s0")
    inst, _ = _enc(g["instance"], g["k"])
    alloc, found, hist = A.legacy_probabilities(inst, g["S"], g["seed"], devices=[0, 0])
    assert [alloc[i] for i in range(len(alloc))] == g["alloc"]
    assert len(found) == g["unique"]
    assert tuple(g["first_panels"][0]) in found
    assert hist.upper().tolist() == (np.asarray(g["pair_upper"]) / g["S"]).tolist()


def _hip_device_count():
    N = pkg("_native")
    out = np.zeros(1, np.int32)
    return int(out[0]) if N.lib().csa_device_count(N.ptr(out)) == N.CSA_OK else 0


@pytest.mark.parametrize("name,k,S,seed", [
    ("couples_panel_from_twenty_people_no_constraints_2", 2, 10000, 0),   # duplicates across the devices
    ("sf_e_110", 110, 200000, 4),                                          # partitioned distinct pass per shard
    ("synthetic8192_200", 200, 5000, 2),                                   # n = 8192 pair sums over peer copies
])
def test_distinct_devices_equal_single_call(gpu_available, name, k, S, seed):
    """Shards on DIFFERENT GPUs: the peer copies of counts, pairs and distinct segments into shard 0's
    device, the replicas on the other devices, the cross-device stream ordering.  Runs only on a box
    with >= 2 GPUs (the driver's 8-GPU node); one-GPU boxes cover the same code with device 0 repeated."""
    ndev = _hip_device_count()
    if ndev < 2:
        pytest.skip("needs >= 2 HIP devices (this box has %d)" % ndev)
    A = pkg("analysis")
    _, enc = _enc(name, k)
    one = A.legacy_sample_raw(enc, k, S, seed, want_pairs=True, want_panels=True, want_attempts=True)
    for devs in ([0, 1], list(range(ndev)), [1, 0, 1]):
        many = A.legacy_sample_raw(enc, k, S, seed, want_pairs=True, want_panels=True, want_attempts=True,
                                   devices=devs)
        _same(one, many, enc.n)


def test_devices_bad_arguments(gpu_available):
    N = pkg("_native")
    L = N.lib()
    _, enc = _enc("example_small_20", 20)
    out = np.zeros(1, np.uint64)
    for devs, n in ((np.array([0], np.int32), 0), (np.array([99], np.int32), 1), (np.array([-1], np.int32), 1)):
        rc = L.csa_legacy_sample_devices(enc.handle, N.ptr(devs), n, 20, 0, 0, 10, N.CSA_WANT_UNIQUE, 0, None,
                                         None, None, N.ptr(out), None)
        assert rc == N.CSA_E_INVALID, N.last_error()
