"""CPU oracle for the Mythril GPU pre-filter — TEST INFRASTRUCTURE ONLY.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline``
leg may import, call, link or execute anything in this package, and only as the
checker (or the timed CPU baseline) — never as the thing measured or shipped.
The product path (``mythril_amd``) never imports it.

Contents
  bvsem.py        z3 / SMT-LIB bit-vector semantics over Python ints (DAG level)
  bytecode_ref.py reference interpreter of the mgp bytecode (checks the lowering)
  keccak_ref.py   Keccak-256 (FIPS 202 permutation, Ethereum 0x01 padding)
  c/oracle.c      the same restatement in C (OpenMP) for large parity runs and
                  the timed CPU baseline; built to oracle/liboracle.so
  coracle.py      ctypes wrapper of liboracle.so

Parity pins: tests/golden/ (VMTests Keccak KATs and arithmetic vectors, EIP-145
shift vectors, keccak_tests.py sat/unsat outcomes) — see tests/golden/make_golden.py.
"""
