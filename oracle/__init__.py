"""CPU oracle for the Shamir hot path — TEST INFRASTRUCTURE ONLY.

Imported only by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline
leg, as the checker; the product (delta-node_amd/) never imports it.

* py_shamir.py  — pure-Python restatement of delta_node/crypto/shamir
                  (per element; small cases and the timed CPU baseline).
* m521_oracle.c — plain-C restatement (independent 64-bit-limb arithmetic),
                  for sizes the Python one cannot reach in seconds.
Parity of both is pinned against the golden fixtures in tests/golden/, which
tests/golden/make_golden.py generated from the reference itself.
"""
