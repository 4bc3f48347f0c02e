"""Philox4x32-10 counter-based RNG -- oracle copy (test infrastructure only).

Algorithm: Salmon, Moraes, Dror, Shaw, "Parallel random numbers: as easy as
1, 2, 3" (SC'11), Random123 reference constants.  Known-answer vectors
(Random123 kat_vectors, also listed in SURVEY.md section 4):

    ctr=0, key=0                      -> 6627e8d5 e169c58d bc57ac4c 9b00dbd8
    ctr=all ones, key=all ones        -> 408f276d 41c83b0e a20bc7c6 6d5451fd
    ctr=243f6a88 85a308d3 13198a2e 03707344, key=a4093822 299f31d0
                                      -> d16cfe09 94fdcceb 5001e420 24126ea1

LEGACY verification-mode contract (the stream the GPU kernel implements and
that replaces the reference's ``random.randint`` at legacy.py:149):

    word(seed, panel, attempt, step) =
        philox(ctr=(step >> 2, attempt, panel & 0xffffffff, panel >> 32),
               key=(seed & 0xffffffff, seed >> 32))[step & 3]
    randint(1, rem) := 1 + ((word * rem) >> 32)

``rem`` is the remaining count of the argmax feature, so only the last
``randint`` call inside one ``find_max_ratio_cat`` matters (legacy.py:149).
"""

M0 = 0xD2511F53
M1 = 0xCD9E8D57
W0 = 0x9E3779B9
W1 = 0xBB67AE85
MASK32 = 0xFFFFFFFF


def philox4x32_10(ctr, key):
    """Return the 4-word Philox4x32-10 block for ``ctr`` (4 u32) and ``key`` (2 u32)."""
    c0, c1, c2, c3 = (int(x) & MASK32 for x in ctr)
    k0, k1 = (int(x) & MASK32 for x in key)
    for rnd in range(10):
        if rnd:
            k0 = (k0 + W0) & MASK32
            k1 = (k1 + W1) & MASK32
        p0 = M0 * c0
        p1 = M1 * c2
        c0, c1, c2, c3 = ((p1 >> 32) ^ c1 ^ k0, p1 & MASK32,
                          (p0 >> 32) ^ c3 ^ k1, p0 & MASK32)
    return c0, c1, c2, c3


def legacy_word(seed, panel, attempt, step):
    """The u32 uniform consumed by step ``step`` of ``attempt`` of ``panel``."""
    blk = philox4x32_10((step >> 2, attempt, panel & MASK32, panel >> 32),
                        (seed & MASK32, (seed >> 32) & MASK32))
    return blk[step & 3]


def legacy_randint(word, rem):
    """Map a u32 uniform to an integer in [1, rem] (multiply-shift)."""
    return 1 + ((int(word) * int(rem)) >> 32)
