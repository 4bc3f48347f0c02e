"""GPU parity of the bit transpose + per-person counts (csa_transpose_count_async, xt_count_kernel: the
Counter of analysis.py:179,187 and the XT operand of PairHistogram, analysis.py:90-95) through the C ABI.

Against a numpy restatement on the same packed panels: XT plane layout (xt32[b][0][p] = panels 64b..64b+31
of agent p, xt32[b][1][p] = panels 64b+32..64b+63, zero past n up to csa_xt_pad(n)) and counts added onto
the prior contents.  Ragged last blocks, fewer blocks than workgroups, odd / even W, 32-word column ranges
with a partial last range.  Bar: bit-exact.
"""
import numpy as np
import pytest

from conftest import pkg

pytestmark = pytest.mark.gpu


def _ref(panels, S, n, npad):
    """panels uint64 [S, W] -> (xt uint32 [nblk, 2, npad], counts int64 [n])."""
    W = panels.shape[1]
    nblk = (S + 63) // 64
    bits = np.unpackbits(panels.view(np.uint8).reshape(S, W * 8), axis=1, bitorder="little")[:, :n]
    counts = bits.sum(axis=0, dtype=np.int64)
    B = np.zeros((nblk * 64, npad), dtype=np.uint8)
    B[:S, :n] = bits
    B = B.reshape(nblk, 2, 32, npad)                                   # [b, plane, bit, agent]
    xt = np.packbits(B, axis=2, bitorder="little").reshape(nblk, 2, 4, npad)
    xt = np.ascontiguousarray(xt.transpose(0, 1, 3, 2)).view(np.uint32).reshape(nblk, 2, npad)
    return xt, counts


@pytest.mark.parametrize("n,S", [(1727, 20000), (1727, 1), (1727, 63), (2000, 6401), (200, 3000), (64, 130),
                                 (40, 257), (1000, 64 * 4 * 3 + 5), (2050, 1000), (2100, 777), (8192, 4097),
                                 (8192, 64), (4500, 300), (2048, 2048)])
@pytest.mark.parametrize("with_xt", [True, False])
def test_transpose_count_exact(gpu_available, n, S, with_xt):
    import torch
    N = pkg("_native")
    L = N.lib()
    W = (n + 63) // 64
    npad = int(L.csa_xt_pad(n))
    rng = np.random.default_rng(n * 131 + S)
    panels = rng.integers(0, 2 ** 64, size=(S, W), dtype=np.uint64)
    if n % 64:
        panels[:, -1] &= np.uint64((1 << (n % 64)) - 1)               # no bits past n
    panels[S // 2, :] = 0                                             # an empty panel
    ref_xt, ref_counts = _ref(panels, S, n, npad)
    nblk = (S + 63) // 64
    d_p = torch.from_numpy(panels.view(np.int64)).cuda()
    d_xt = torch.full((nblk * npad,), -1, dtype=torch.int64, device="cuda") if with_xt else None
    d_c = torch.full((n,), 5, dtype=torch.int64, device="cuda")
    N.check(L.csa_transpose_count_async(N.ptr(d_p), S, n, N.ptr(d_xt), N.ptr(d_c), None))
    torch.cuda.synchronize()
    assert np.array_equal(d_c.cpu().numpy(), ref_counts + 5)
    if with_xt:
        got = d_xt.cpu().numpy().view(np.uint32).reshape(nblk, 2, npad)
        assert np.array_equal(got, ref_xt)


@pytest.mark.parametrize("name,k,S", [("sf_e_110", 110, 1), ("sf_e_110", 110, 63), ("sf_e_110", 110, 64),
                                      ("sf_e_110", 110, 129), ("sf_e_110", 110, 20011), ("sf_e_tight_110", 110, 3001),
                                      ("example_large_200", 200, 1000), ("example_large_200", 200, 257),
                                      ("example_small_20", 20, 65), ("synthetic8192_200", 200, 300)])
def test_draw_xt_matches_transpose(gpu_available, name, k, S):
    """csa_draw_xt_async: where a register kernel with a fused pack runs (draw_lane_kernel, F <= 32, or
    draw_solo_kernel, F <= 16; n <= 2048) the pack also writes the launch's XT blocks, bit-exact to csa_transpose_count_async over the same panels (npad padding words
    zero), and the pair diagonal (csa_pairs_diag_async) equals the transpose pass's counts; elsewhere
    it reports that it did not and leaves XT alone.  Ragged launches: 1, 63, 64, 129 panels."""
    import torch
    from conftest import inst_paths
    P, Dv = pkg(), pkg("device")
    inst = P.read_instance(*inst_paths(name), k)
    enc = P.encode(inst.categories, inst.agents)
    a = Dv.DevicePipeline(enc, k, S)
    b = Dv.DevicePipeline(enc, k, S)
    a.reset()
    a.xt.fill_(-1)                             # every word the draw owns must be written
    written = a.draw_xt(11, 5, S)
    torch.cuda.synchronize()
    reg = a.draw_kernel_name().startswith(("draw_lane_kernel", "draw_solo_kernel"))
    assert written == reg
    b.reset()
    b.panels.copy_(a.panels)
    b.transpose_count(S)
    nblk = (S + 63) // 64
    if not written:
        assert bool((a.xt == -1).all())
        return
    assert torch.equal(a.xt[: nblk * a.npad], b.xt[: nblk * b.npad])
    a.pair_counts(S, overwrite=True, alone=True)
    a.counts_from_pairs()
    torch.cuda.synchronize()
    assert torch.equal(a.counts, b.counts)
    assert int(a.counts.sum()) == S * k
