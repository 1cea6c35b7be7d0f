"""oracle/ — CPU restatement of the reference algorithms. TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import or
call anything here, and only as the checker / CPU baseline — never as the thing
measured or shipped. The product package (gym-cellular-automata_amd/gymca_amd) never
imports it and has no CPU fallback.

Pinning:
  * windy / repeat_ca / move_modify / bulldozer / drossel / helicopter restatements
    are checked against golden vectors captured from the reference itself
    (tests/golden/*.npz, script tests/golden/make_golden.py);
  * philox.py against the Random123 known-answer vectors;
  * alexandridis_ref.py restates ca_alexandridis_jax.py:321-424 verbatim (jax absent:
    parity with the reference is pinned by the restatement plus the reference's own
    invariants and a float64 evaluation of the probability formula; no golden vectors
    exist for it anywhere — "parity unpinned" at the reference level).
"""
