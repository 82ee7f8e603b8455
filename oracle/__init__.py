"""CPU ORACLE for the KZG grand-sum / grand-product prover — TEST INFRASTRUCTURE ONLY.

This package restates the reference's algorithm (xavi-pinsach/kzg-grandsums-study, JS) and the
third-party arithmetic it delegates to (ffjavascript@0.2.59 / wasmcurves@0.2.1, not vendored):
see bn254.py, keccak.py, ptau.py, poly.py, protocol.py (pure Python) and c/ (a C restatement used
for larger sizes and as bench.py's `cpu_baseline`).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import it, and only as
the checker. The product path (kzg-grandsums-study_amd/) never imports, links or executes it.

Parity pinning: the reference publishes no value-level vectors. The oracle is
pinned by known-answer constants (keccak256 KATs, Fr.w roots, the polynomial.test.js KATs) and by
prove -> verify round trips through the restated pairing check; see DESIGN.md §Parity.
"""
