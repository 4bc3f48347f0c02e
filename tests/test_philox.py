"""Philox4x32-10 known-answer tests (Random123 kat_vectors)."""
import pytest

from oracle.philox import philox4x32_10, legacy_word, legacy_randint
from oracle import coracle

KAT = [
    ((0, 0, 0, 0), (0, 0), (0x6627E8D5, 0xE169C58D, 0xBC57AC4C, 0x9B00DBD8)),
    ((0xFFFFFFFF,) * 4, (0xFFFFFFFF,) * 2, (0x408F276D, 0x41C83B0E, 0xA20BC7C6, 0x6D5451FD)),
    ((0x243F6A88, 0x85A308D3, 0x13198A2E, 0x03707344), (0xA4093822, 0x299F31D0),
     (0xD16CFE09, 0x94FDCCEB, 0x5001E420, 0x24126EA1)),
]


@pytest.mark.parametrize("ctr,key,out", KAT)
def test_python_philox_kat(ctr, key, out):
    assert philox4x32_10(ctr, key) == out


@pytest.mark.parametrize("ctr,key,out", KAT)
def test_c_philox_kat(ctr, key, out):
    assert coracle.philox(ctr, key) == out


def test_legacy_word_contract():
    # word(seed, panel, attempt, step) = philox((step>>2, attempt, panel_lo, panel_hi), seed)[step&3]
    seed, panel, attempt = 0x1234567890ABCDEF, (7 << 32) | 5, 3
    for step in range(12):
        blk = philox4x32_10((step >> 2, attempt, panel & 0xFFFFFFFF, panel >> 32),
                            (seed & 0xFFFFFFFF, seed >> 32))
        assert legacy_word(seed, panel, attempt, step) == blk[step & 3]


def test_randint_range():
    for rem in (1, 2, 3, 17, 1727, 8192):
        assert legacy_randint(0, rem) == 1
        assert legacy_randint(0xFFFFFFFF, rem) == rem
