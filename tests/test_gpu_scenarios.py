"""Solver queries of the solidity_examples configs, built the way LASER builds them.

No solc / z3 / mythril exists here or on the GPU box, so the contracts cannot be
executed; these tests restate the constraint shapes of the detection-module
queries on the configs' hot spots ("expected by
reading") and check what the GPU-first front end answers and how many fallback
(z3) calls it needs.  Issue-level parity with `myth analyze` stays unpinned.

* suicide.sol `kill(address)` (`solidity_examples/suicide.sol:3-6`, module
  `suicide.py:76-99`): the path requires addr == 0, so the first query (`to ==
  ACTORS.attacker`) is UNSAT — proven by the host pre-check, no z3 call; the path
  itself is feasible.
* BECToken.sol `balances[msg.sender]` (`BECToken.sol:256-258`): a storage read at
  keccak256_512(Concat(caller, 0)) — a 512-bit preimage, lowered as word pairs
  (include/mgp_ir.h "wide values") — with the manager's interval/inverse condition
  (`keccak_function_manager.py:122-146`): SAT by a GPU witness, no z3 call.
* BECToken.sol `batchTransfer` (`BECToken.sol:254-258`, module `integer.py:141-160,
  288-297`): the multiplication-overflow query is SAT — a GPU witness the oracle
  confirms, no z3 call; SafeMath's `sub` after `require(balance >= amount)`
  cannot underflow — proven UNSAT, no z3 call.
"""
import pytest

from mythril_amd import dag as D
from corpus.keccak_manager import KeccakFunctionManager
from mythril_amd import solver as SV
from mythril_amd.smt import (And, Array, BVMulNoOverflow, BVSubNoUnderflow, Concat, Extract, If, Not, UGE, UGT,
                             ULE, ULT, symbol_factory)
from oracle import bvsem as S

pytestmark = pytest.mark.gpu

BVV = symbol_factory.BitVecVal
BVS = symbol_factory.BitVecSym
ATTACKER = 0xDEADBEEFDEADBEEFDEADBEEFDEADBEEFDEADBEEF  # ACTORS.attacker (transaction_models.py)


class CountingBackend(SV.Backend):
    def __init__(self):
        self.calls = 0

    def check(self, terms, timeout_ms, minimize=(), maximize=()):
        self.calls += 1
        return SV.unknown, None


@pytest.fixture()
def backend(mgp_ctx):
    b = CountingBackend()
    old = SV.set_backend(b)
    SV.SolverStatistics().reset()
    SV.unsat_cores().reset()
    SV.get_model.cache_clear()
    SV.enable_gpu(True)
    yield b
    SV.set_backend(old)
    SV.get_model.cache_clear()


def _word(calldata, size, off):
    """calldata.py:219-232: a 32-byte word, each byte If(off+i < calldatasize, calldata[off+i], 0)."""
    parts = []
    for i in range(32):
        idx = BVV(off + i, 256)
        parts.append(If(ULT(idx, size), calldata[idx], BVV(0, 8)))
    return Concat(*parts)


def _selector(calldata, size, sig):
    return Concat(*[If(ULT(BVV(i, 256), size), calldata[BVV(i, 256)], BVV(0, 8)) for i in range(4)]) == BVV(sig, 32)


def _confirmed(constraints, model):
    st = D.build_state([c.raw for c in constraints])
    return S.eval_root(st.nodes, st.consts, D.model_to_slots(st, model.assignments[0]))


def test_suicide_kill_attacker_query_refuted(backend):
    calldata, size = Array("calldata", 256, 8), BVS("calldatasize", 256)
    caller, origin = BVS("caller", 256), BVS("origin", 256)
    word = _word(calldata, size, 4)
    addr = Concat(BVV(0, 96), Extract(159, 0, word))
    path = [_selector(calldata, size, 0xCBF0B0C0), addr == BVV(0, 256)]   # JUMPI on addr == 0
    tx = [And(caller == BVV(ATTACKER, 256), caller == origin)]          # suicide.py:70-75
    with pytest.raises(SV.UnsatError):
        SV.get_model(tuple(path + tx + [addr == BVV(ATTACKER, 256)]), minimize=(size,))
    assert backend.calls == 0 and SV.SolverStatistics().refuted == 1
    feasible = SV.Constraints(path + tx)
    assert feasible.is_possible  # witness, or unknown from the fallback: never refuted
    assert SV.SolverStatistics().refuted == 1


def test_bectoken_batch_transfer_overflow_witness(backend):
    cnt, value, bal = BVS("receivers_length", 256), BVS("value", 256), BVS("balance_sender", 256)
    amount = cnt * value                                                   # BECToken.sol:256
    path = [UGT(cnt, BVV(0, 256)), ULE(cnt, BVV(20, 256)),                 # require(cnt > 0 && cnt <= 20)
            UGT(value, BVV(0, 256)), UGE(bal, amount)]                     # require(_value > 0 && bal >= amount)
    overflow = Not(BVMulNoOverflow(cnt, value, False))                     # integer.py:149-153
    m = SV.get_model(tuple(path + [overflow]))
    assert _confirmed(path + [overflow], m)
    assert backend.calls == 0 and SV.SolverStatistics().gpu_sat >= 1
    c, v = m.assignments[0]["receivers_length"], m.assignments[0]["value"]
    assert 0 < c <= 20 and c * v >= 1 << 256


def test_bectoken_safemath_sub_cannot_underflow(backend):
    cnt, value, bal = BVS("receivers_length", 256), BVS("value", 256), BVS("balance_sender", 256)
    amount = cnt * value
    path = [UGT(cnt, BVV(0, 256)), ULE(cnt, BVV(20, 256)), UGT(value, BVV(0, 256)), UGE(bal, amount),
            ULE(amount, bal)]                                              # SafeMath.sub: assert(b <= a)
    underflow = Not(BVSubNoUnderflow(bal, amount, False))                  # integer.py:155-160
    with pytest.raises(SV.UnsatError):
        SV.get_model(tuple(path + [underflow]))
    assert backend.calls == 0 and SV.SolverStatistics().refuted == 1


def test_bectoken_mapping_balance_witness(backend):
    kfm = KeccakFunctionManager()
    caller, value, cnt = BVS("caller", 256), BVS("value", 256), BVS("receivers_length", 256)
    storage = Array("Storage", 256, 256)
    slot, cond = kfm.create_keccak(Concat(caller, BVV(0, 256)))       # balances[msg.sender]
    bal = storage[slot]
    amount = cnt * value
    path = [cond, caller == BVV(ATTACKER, 256), UGT(cnt, BVV(0, 256)), ULE(cnt, BVV(20, 256)),
            UGT(value, BVV(0, 256)), UGE(bal, amount)]
    overflow = Not(BVMulNoOverflow(cnt, value, False))
    m = SV.get_model(tuple(path + [overflow]))
    assert _confirmed(path + [overflow], m)
    assert backend.calls == 0 and SV.SolverStatistics().gpu_sat >= 1
    assert m.assignments[0]["caller"] == ATTACKER
    # two mappings with the same slot: equal hashes force equal keys (Ackermann with the inverse)
    other, cond2 = kfm.create_keccak(Concat(value, BVV(0, 256)))
    SV.get_model.cache_clear()
    m2 = SV.get_model(tuple([cond, cond2, slot == other]))
    assert m2.assignments[0]["caller"] == m2.assignments[0]["value"]
    assert _confirmed([cond, cond2, slot == other], m2)
