"""CPU oracle for the LEGACY Monte Carlo hot path -- TEST INFRASTRUCTURE ONLY.

Nothing in this package is part of the product.  Only ``tests/``,
``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import,
call, link or execute anything under ``oracle/``, and only as the checker (or
the timed CPU baseline), never as the thing measured or shipped.  The product
path (``citizensassemblies-replication_amd``) never imports this package and
fails loudly when its HIP library is missing.

Contents
--------
``philox.py``         Philox4x32-10 (Salmon et al., SC'11; Random123 constants).
``legacy_oracle.py``  pure-Python restatement of reference legacy.py:47-200 and
                      analysis.py:108-191 in two RNG modes (MT19937 = stdlib
                      ``random`` exactly as the reference calls it, and the
                      Philox verification mode that the GPU path implements).
``legacy_oracle.c``   the same restatement in plain C (Philox mode, OpenMP over
                      panels); built into ``oracle/_build/liblegacy_oracle.so``
                      by ``oracle/Makefile``; loaded by ``oracle/coracle.py``.

Parity pins (see DESIGN.md "Oracle"):
  * MT mode reproduces the reference's published seed-0 LEGACY allocations
    (reference_output/*_ratio_product_data.csv, analysis/*_ratio_product_data.csv)
    -- tests/test_oracle_mt.py.
  * Philox mode reproduces golden vectors produced by driving the UNMODIFIED
    reference (imported from /root/reference, monkeypatched RNG only) --
    tools/make_goldens.py -> tests/golden/*.json, tests/test_oracle_golden.py.
"""
