"""CPU restatement of the reference d3rlpy v1.1.0 hot path — TEST INFRASTRUCTURE.

This package is the parity oracle. Only ``tests/``, ``__graft_entry__.smoke()``
and the ``cpu_baseline`` leg of ``bench.py`` may import it, and only as a
checker or a baseline. The product path (``d3rlpy_amd``) never imports it and
has no CPU fallback.

Pinning: the reference implementation cannot be imported or executed in this
pipeline (SURVEY.md §8c records the denial). The oracle is pinned instead
against the known-answer tests that the reference's own test-suite holds for
this path (tests/test_oracle_kats.py restates each one with its file:line).
No reference-pinned end-to-end update KAT exists (the reference's Impl tests
never call ``update_*``), so end-to-end update parity is "restatement-pinned":
the oracle follows the reference op for op, and its building blocks are
pinned by the reference test-suite's KATs where that suite has them
(tests/test_oracle_kats.py, test_oracle_kats2.py, test_oracle_td3.py,
test_nstep_pin.py; each cites the reference test it restates).  Blocks whose
reference tests check shapes only (compute_max_with_n_actions, the
ConditionalVAE, the residual policy's bound) are additionally checked against
closed-form or brute-force restatements of the reference formulas; the
remaining end-to-end composition is pinned by the fp64 arbiters and the
committed golden fixtures, not by a reference vector.
"""
