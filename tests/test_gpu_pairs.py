"""GPU parity of the X^T X pair-count kernels (PairHistogram, analysis.py:68-98) through the C ABI.

Both MFMA engines (fp4 e2m1 with f32 accumulation, int8 with int32
accumulation), both fp4 kernels (pair_fp4_tile_kernel, the default with scratch;
pair_mfma_kernel, CSA_PAIR_KERNEL=1) and every epilogue (direct whole tiles,
int32 partial blocks + reduce kernels, int64 atomics) against an exact CPU
popcount restatement on the same transposed bits.  Bar: bit-exact.

The XT operand (csa_transpose_count_async's layout) is two 32-bit planes per
64-panel block: xt32[b][0][p] = panels 64b..64b+31 of agent p, xt32[b][1][p] =
panels 64b+32..64b+63.  The tests build it from uint64 words w[b][p] (bit j =
panel 64b+j) with _planes.
"""
import os
import numpy as np
import pytest

from conftest import pkg

pytestmark = pytest.mark.gpu


def _popcount64(a):
    return np.unpackbits(a.view(np.uint8)).sum(dtype=np.int64)


def _cpu_pairs(xt, n, npad, rows=None):
    """Exact pair counts from the packed transposed bits xt[b, p] (uint64)."""
    X = np.unpackbits(xt[:, :n].copy().view(np.uint8).reshape(xt.shape[0], n, 8), axis=2, bitorder="little")
    X = X.transpose(0, 2, 1).reshape(-1, n).astype(np.float64)    # panels x agents
    return np.rint(X.T @ X).astype(np.int64)                      # BLAS; exact below 2^53


def _planes(w):
    """uint64 words [nblk, npad] -> the XT plane layout (uint32 [nblk, 2, npad]); numpy or torch."""
    if isinstance(w, np.ndarray):
        nblk, npad = w.shape
        return np.ascontiguousarray(w.view(np.uint32).reshape(nblk, npad, 2).transpose(0, 2, 1))
    import torch
    nblk, npad = w.shape
    return w.contiguous().view(torch.int32).view(nblk, npad, 2).permute(0, 2, 1).contiguous()


@pytest.fixture(params=["tile4", "tile2", "split"])
def pair_kernel(request, monkeypatch):
    """fp4 kernel: pair_fp4_tile_kernel (CSA_PAIR_KERNEL=2; the default from n ~ 5.7k on) in its
    512-register (NB = 4, alone) or 256-register (NB = 2, CSA_PAIR_SHARED) form, or pair_mfma_kernel
    (CSA_PAIR_KERNEL=1; the default below)."""
    monkeypatch.setenv("CSA_PAIR_KERNEL", "1" if request.param == "split" else "2")
    if request.param != "split":
        monkeypatch.setenv("CSA_P2_NB", request.param[4:])
    return request.param


def _run(xt_np, n, engine, scratch, init=0):
    import torch
    N = pkg("_native")
    L = N.lib()
    nblk = xt_np.shape[0]
    xt = torch.from_numpy(_planes(xt_np).view(np.int64).copy()).cuda()
    pairs = torch.full((n * n,), init, dtype=torch.int64, device="cuda")
    sb = int(L.csa_pair_scratch_bytes(n, nblk, engine))
    scr = torch.empty((sb + 3) // 4, dtype=torch.int32, device="cuda") if scratch else None
    N.check(L.csa_pair_counts_ex_async(N.ptr(xt), nblk, n, N.ptr(pairs), engine, N.ptr(scr),
                                       sb if scratch else 0, None))
    torch.cuda.synchronize()
    return pairs.cpu().numpy().reshape(n, n)


@pytest.mark.parametrize("n,S", [(20, 10000), (200, 70000), (300, 6400), (1727, 20000), (2000, 3000)])
@pytest.mark.parametrize("engine,scratch", [(0, True), (0, False), (1, True), (1, False)])
def test_pair_engines_exact(gpu_available, pair_kernel, n, S, engine, scratch):
    N = pkg("_native")
    npad = int(N.lib().csa_xt_pad(n))
    nblk = (S + 63) // 64
    rng = np.random.default_rng(n * 7 + S)
    dens = rng.integers(0, 2 ** 64, size=(nblk, npad), dtype=np.uint64)
    xt = dens & rng.integers(0, 2 ** 64, size=(nblk, npad), dtype=np.uint64)   # ~25% density
    xt[:, 0] = np.uint64(2 ** 64 - 1)                                          # a dense agent
    if S % 64:                                                                 # ragged last block
        xt[-1, :] &= np.uint64((1 << (S % 64)) - 1)
    got = _run(xt, n, engine, scratch)
    ref = _cpu_pairs(xt, n, npad)
    iu = np.triu_indices(n)
    assert np.array_equal(got[iu], ref[iu])


@pytest.mark.parametrize("n,S", [(20, 1000), (1727, 20000)])
@pytest.mark.parametrize("engine,scratch", [(0, True), (0, False), (1, True)])
def test_pair_overwrite_ignores_prior_contents(gpu_available, pair_kernel, n, S, engine, scratch):
    """CSA_PAIR_OVERWRITE: the output holds exactly this batch's counts whatever it held before
    (bench.py skips the n*n zero-fill this way); the plain mode adds onto the prior contents."""
    N = pkg("_native")
    npad = int(N.lib().csa_xt_pad(n))
    nblk = (S + 63) // 64
    rng = np.random.default_rng(n + S)
    xt = rng.integers(0, 2 ** 64, size=(nblk, npad), dtype=np.uint64) & rng.integers(0, 2 ** 64, size=(nblk, npad),
                                                                                     dtype=np.uint64)
    if S % 64:
        xt[-1, :] &= np.uint64((1 << (S % 64)) - 1)
    ref = _cpu_pairs(xt, n, npad)
    iu = np.triu_indices(n)
    got = _run(xt, n, engine | N.CSA_PAIR_OVERWRITE, scratch, init=-12345)
    assert np.array_equal(got[iu], ref[iu])
    got_add = _run(xt, n, engine, scratch, init=7)
    assert np.array_equal(got_add[iu], ref[iu] + 7)


def test_pair_fp4_exact_beyond_f32_range(gpu_available):
    """> 2^24 panels in one call with few output blocks: every split must stay below 2^24."""
    import torch
    N = pkg("_native")
    n = 6000                                   # 24 x 24 blocks -> 300 triangle blocks, 1 split by occupancy
    npad = int(N.lib().csa_xt_pad(n))
    nblk = (1 << 18) + 5                       # 2^24 + 320 panels
    S = nblk * 64
    # agents 0, 1, n-1 dense-ish; everything else zero (cheap to build, exact counts known)
    xt = torch.zeros(nblk, npad, dtype=torch.int64, device="cuda")
    xt[:, 0] = -1                              # all ones
    xt[:, n - 1] = -1
    g = torch.Generator(device="cuda").manual_seed(5)
    xt[:, 1] = torch.randint(-2 ** 63, 2 ** 63 - 1, (nblk,), device="cuda", generator=g)
    pairs = torch.zeros(n * n, dtype=torch.int64, device="cuda")
    L = N.lib()
    sb = int(L.csa_pair_scratch_bytes(n, nblk, N.CSA_PAIR_FP4))
    assert sb >= 2 * 300 * 256 * 256 * 4       # the exactness guard forced >= 2 splits
    scr = torch.empty(sb // 4, dtype=torch.int32, device="cuda")
    x32 = _planes(xt)
    N.check(L.csa_pair_counts_ex_async(N.ptr(x32), nblk, n, N.ptr(pairs), N.CSA_PAIR_FP4, N.ptr(scr), sb, None))
    torch.cuda.synchronize()
    P = pairs.view(n, n)
    c1 = int(_popcount64(xt[:, 1].cpu().numpy()))
    assert int(P[0, 0]) == S
    assert int(P[0, n - 1]) == S
    assert int(P[n - 1, n - 1]) == S
    assert int(P[0, 1]) == c1 and int(P[1, 1]) == c1 and int(P[1, n - 1]) == c1
    assert int(P[2, 3]) == 0 and int(P[0, 2]) == 0


@pytest.mark.parametrize("n", [8192, 4096, 4500])
@pytest.mark.parametrize("engine", [0, 1])
def test_pairs_n8192_vs_torch_fp32(gpu_available, pair_kernel, engine, n):
    """BASELINE config 5 shape: n = 8192 (32 triangle rows of 256 x 256 blocks), S = 131072 panels of
    ~2.5 % density (k ~ 200), against a plain PyTorch fp32 X^T X on the device (rocBLAS; exact:
    every partial sum <= S < 2^24, and gfx950 has no reduced-precision fp32 GEMM mode).  n = 4096 / 4500
    (136 / 171 tiles, fewer than the CUs): the split kernel's balanced split counts (13 / 19)."""
    import torch
    N = pkg("_native")
    S = 131072
    npad = int(N.lib().csa_xt_pad(n))
    nblk = S // 64
    g = torch.Generator(device="cuda").manual_seed(n + engine)
    X = (torch.rand(S, n, device="cuda", generator=g) < 0.025)
    X[:, 17] = True                                              # a dense agent: counts up to S
    # pack the transposed bits: xt[b, p] bit j = X[64 b + j, p]
    w = (1 << torch.arange(64, device="cuda", dtype=torch.int64))
    xt = torch.zeros(nblk, npad, dtype=torch.int64, device="cuda")
    xt[:, :n] = (X.view(nblk, 64, n).to(torch.int64) * w.view(1, 64, 1)).sum(dim=1)
    L = N.lib()
    pairs = torch.full((n * n,), -7, dtype=torch.int64, device="cuda")
    sb = int(L.csa_pair_scratch_bytes(n, nblk, engine))
    scr = torch.empty((sb + 3) // 4, dtype=torch.int32, device="cuda")
    x32 = _planes(xt)
    N.check(L.csa_pair_counts_ex_async(N.ptr(x32), nblk, n, N.ptr(pairs), engine | N.CSA_PAIR_OVERWRITE, N.ptr(scr),
                                       sb, None))
    Xf = X.to(torch.float32)
    ref = (Xf.T @ Xf).to(torch.int64)
    torch.cuda.synchronize()
    got = pairs.view(n, n)
    assert torch.equal(torch.triu(got), torch.triu(ref))
    assert int(ref[17, 17].item()) == S


@pytest.mark.parametrize("n,nblk", [(20, 1), (20, 31), (257, 3), (1727, 40), (4100, 7), (8192, 33)])
@pytest.mark.parametrize("overwrite", [True, False])
@pytest.mark.parametrize("nb", [4, 2])
def test_pair_tile_kernel_small_and_ragged(gpu_available, monkeypatch, n, nblk, overwrite, nb):
    """pair_fp4_tile_kernel edge cases, both forms (CSA_P2_NB=4: 256 x 256 tiles; CSA_P2_NB=2: 256 x 128
    column-half items, PairMap::halves = 2): fewer panel blocks than k-pieces (empty pieces), one tile
    only (n = 20: one XCD has work), XCD chunks with and without leftover items, n not a multiple of
    256, a column half wholly past n (n = 4100) and the leftover reduce of half items."""
    monkeypatch.setenv("CSA_PAIR_KERNEL", "2")
    monkeypatch.setenv("CSA_P2_NB", str(nb))
    shared = nb == 2              # the scheduling hint changes nothing; exercised beside the NB = 2 form
    N = pkg("_native")
    npad = int(N.lib().csa_xt_pad(n))
    rng = np.random.default_rng(n * 31 + nblk)
    xt = rng.integers(0, 2 ** 64, size=(nblk, npad), dtype=np.uint64) & rng.integers(0, 2 ** 64, size=(nblk, npad),
                                                                                     dtype=np.uint64)
    xt[:, n:] = 0
    ref = _cpu_pairs(xt, n, npad)
    iu = np.triu_indices(n)
    engine = N.CSA_PAIR_FP4 | (N.CSA_PAIR_OVERWRITE if overwrite else 0) | (N.CSA_PAIR_SHARED if shared else 0)
    got = _run(xt, n, engine, True, init=-3)
    assert np.array_equal(got[iu], ref[iu] + (0 if overwrite else -3))
