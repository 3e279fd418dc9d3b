"""mythril_amd — MI355X-native satisfiability pre-filter for Mythril's LASER engine.

Hot path (BASELINE.json north_star): path-constraint DAGs (laser.smt Bool /
BitVec expressions) are lowered to a flat 256-bit bytecode and evaluated by a
hand-written gfx950 HIP kernel over states x candidate assignments; any
witness proves SAT, everything else is left to z3.  A second kernel computes
batched Keccak-256 for the keccak function manager.

Python reaches the kernels through ctypes over libmgp.so (include/mgp.h); see
DESIGN.md and INTEGRATION.md.
"""
__version__ = "0.1.0"
