"""Contract-shaped constraint corpus (test and benchmark infrastructure, not product).

No solc / z3 / mythril exists here or on the GPU box, so `myth analyze` cannot run
("not measurable").  This module restates, through the
laser.smt mirror (mythril_amd.smt + the keccak manager mirror), the path constraints
LASER builds on the configs' hot spots and the solver queries asked there, so the
pre-filter can be measured on a MIXED corpus instead of one repeated shape:

* suicide.sol ``kill(address)`` (solidity_examples/suicide.sol:3-6; suicide.py:76-99):
  the dispatcher, the JUMPI on ``addr == 0`` and the module's attacker query, UNSAT
  because the path forces addr == 0;
* BECToken.sol ``batchTransfer`` (BECToken.sol:254-258; integer.py:141-160): calldata
  words, ``balances[msg.sender]`` through keccak256_512 with the manager's condition,
  the multiplication-overflow query (SAT) and SafeMath.sub's underflow query after the
  balance check (UNSAT);
* WalletLibrary.sol ``initWallet`` then ``kill`` (WalletLibrary.sol:91-104,219-226,
  288-320): tx 1 writes m_dailyLimit, m_lastDay, m_numOwners, m_owners[1],
  m_ownerIndex[msg.sender] (a Store at keccak256_512(Concat(sender, 263))), the bounded
  owners loop (-b 3) and m_required; tx 2 reads them through the Store chain
  (read-over-write), hashes msg.data with a symbolic length (a fresh KECCAC_mem[...]
  symbol, instructions.py:1003-1015), 2**ownerIndex as a fresh symbol
  (instructions.py:582-600), and the suicide module asks for to == ATTACKER.  The
  prune filter's queries along tx 2 (both branches of every JUMPI) come with it.

Every transaction adds LASER's setup constraints: the sender is one of the ACTORS
(transaction/symbolic.py:165-167) and can pay the call value
(transaction_models.py:129-133); non-payable functions add call_value == 0; the
dispatcher compares calldata[0:4] as solc 0.5 does (DIV by 2^224, AND 0xffffffff).

`corpus(n)` returns n (label, constraint-term tuple, expected) entries cycling over
the shapes with varied transaction ids, slots and loop counts; `expected` is "sat" or
"unsat" where the shape decides it by construction, else None.  The expectations are
by reading, not pinned by any reference fixture (issue-level parity stays unpinned).
"""
from __future__ import annotations

import copy
from typing import List, Optional, Tuple

from .keccak_manager import KeccakFunctionManager
from mythril_amd.smt import (And, Array, BVMulNoOverflow, BVSubNoUnderflow, Concat, Extract, If, Not, Or, UDiv, UGE,
                             UGT, ULE, ULT, symbol_factory)

BVV, BVS = symbol_factory.BitVecVal, symbol_factory.BitVecSym
CREATOR = 0xAFFEAFFEAFFEAFFEAFFEAFFEAFFEAFFEAFFEAFFE
ATTACKER = 0xDEADBEEFDEADBEEFDEADBEEFDEADBEEFDEADBEEF
SOMEGUY = 0xAAAAAAAAAAAAAAAAAAAAAAAAAAAAAAAAAAAAAAAA
ACTORS = (CREATOR, ATTACKER, SOMEGUY)

# WalletLibrary.sol storage slots (solc 0.5 layout of the FIELDS section, lines 374-399)
S_REQUIRED, S_NUM_OWNERS, S_DAILY_LIMIT, S_SPENT_TODAY, S_LAST_DAY = 1, 2, 3, 4, 5
S_OWNERS, S_OWNER_INDEX, S_PENDING = 6, 263, 264


class Tx:
    """One symbolic message call: calldata, sender, value and LASER's setup constraints."""

    def __init__(self, tid: int, balance: Array):
        self.tid = tid
        self.calldata = Array(f"{tid}_calldata", 256, 8)
        self.size = BVS(f"{tid}_calldatasize", 256)
        self.sender = BVS(f"sender_{tid}", 256)
        self.value = BVS(f"call_value{tid}", 256)
        self.timestamp = BVS(f"{tid}_timestamp", 256)
        self.setup = [Or(*[self.sender == BVV(a, 256) for a in ACTORS]), UGE(balance[self.sender], self.value)]

    def byte(self, idx) -> "object":
        """calldata.py:219-232: If(idx < calldatasize, calldata[idx], 0) -- BitVec `<`, i.e.
        a SIGNED compare (bitvec.py:138-147)."""
        i = idx if not isinstance(idx, int) else BVV(idx, 256)
        return If(i < self.size, self.calldata[i], BVV(0, 8))

    def word(self, off) -> "object":
        base = off if not isinstance(off, int) else BVV(off, 256)
        return Concat(*[self.byte(base + i) for i in range(32)])

    def dispatch(self, sig: int, payable: bool = False) -> list:
        """solc 0.5 dispatcher: calldatasize >= 4, (word0 / 2^224) & 0xffffffff == sig, and
        CALLVALUE == 0 for a non-payable function."""
        sel = UDiv(self.word(0), BVV(1 << 224, 256)) & BVV(0xFFFFFFFF, 256)
        out = [Not(ULT(self.size, BVV(4, 256))), sel == BVV(sig, 256)]
        if not payable:
            out.append(self.value == BVV(0, 256))
        return out


def _attacker_query(txs: List[Tx], to) -> list:
    """suicide.py:76-99: every transaction sent by the attacker (caller == origin), and
    the beneficiary is the attacker."""
    return [And(t.sender == BVV(ATTACKER, 256), t.sender == t.sender) for t in txs] + [to == BVV(ATTACKER, 256)]


# ----------------------------------------------------------------- suicide.sol
def suicide_states(tid: int = 1) -> List[Tuple[str, tuple, Optional[str]]]:
    balance = Array("balance", 256, 256)
    tx = Tx(tid, balance)
    addr = Concat(BVV(0, 96), Extract(159, 0, tx.word(4)))
    path = tx.setup + tx.dispatch(0xCBF0B0C0)
    out = [("suicide:dispatch", path, "sat"),
           ("suicide:addr!=0 (revert branch)", path + [Not(addr == BVV(0, 256))], "sat"),
           ("suicide:addr==0", path + [addr == BVV(0, 256)], "sat"),
           ("suicide:attacker query", path + [addr == BVV(0, 256)] + _attacker_query([tx], addr), "unsat")]
    return [(l, tuple(c.raw for c in cs), e) for l, cs, e in out]


# ---------------------------------------------------------------- BECToken.sol
def bectoken_states(k: int, kfm: KeccakFunctionManager) -> Tuple[str, tuple, Optional[str]]:
    """batchTransfer (BECToken.sol:254-258): cnt = receivers.length <= 20, value > 0,
    balances[msg.sender] >= cnt * value; the integer module's queries."""
    balance = Array("balance", 256, 256)
    tx = Tx(2 + k % 3, balance)
    storage = Array("Storage", 256, 256)
    cnt = tx.word(4 + 64 * (k % 2))   # receivers.length (its offset word varies), never the value word
    value = tx.word(36)
    slot, cond = kfm.create_keccak(Concat(tx.sender, BVV(k % 5, 256)))
    bal = storage[slot]
    path = tx.setup + tx.dispatch(0x83F12FEC) + [cond, UGT(cnt, BVV(0, 256)), ULE(cnt, BVV(20, 256)),
                                                 UGT(value, BVV(0, 256)), UGE(bal, cnt * value)]
    if k % 4 == 3:  # SafeMath.sub after require(balance >= amount): cannot underflow
        return ("bectoken:safemath sub underflow", tuple(c.raw for c in path + [
            Not(BVSubNoUnderflow(bal, cnt * value, False))]), "unsat")
    if k % 2 == 0:
        return ("bectoken:mul overflow", tuple(c.raw for c in path + [Not(BVMulNoOverflow(cnt, value, False))]),
                "sat")
    return ("bectoken:balance below k", tuple(c.raw for c in path + [ULT(bal, BVV(k, 256))]), None)


# ------------------------------------------------------------ WalletLibrary.sol
class _Storage:
    """The contract's storage across transactions: one Array with its Store chain."""

    def __init__(self):
        self.arr = Array("Storage", 256, 256)

    def fork(self) -> "_Storage":
        s = _Storage.__new__(_Storage)
        s.arr = copy.copy(self.arr)
        return s

    def __getitem__(self, k):
        return self.arr[k if not isinstance(k, int) else BVV(k, 256)]

    def __setitem__(self, k, v):
        self.arr[k if not isinstance(k, int) else BVV(k, 256)] = v


def _mapping_slot(kfm, key, slot: int):
    """m[key] for a mapping at `slot`: keccak256(Concat(key, slot)) + the manager's condition."""
    h, cond = kfm.create_keccak(Concat(key, BVV(slot, 256)))
    return h, cond


def wallet_states(variant: int, kfm: KeccakFunctionManager) -> List[Tuple[str, tuple, Optional[str]]]:
    """initWallet (tx 1) then kill (tx 2), `variant` picks the owners-loop count (0..2) and
    the transaction ids; returns the prune queries along tx 2 and the module's query."""
    n_loop = variant % 3
    t1, t2 = 1 + 2 * (variant // 3), 2 + 2 * (variant // 3)
    balance = Array("balance", 256, 256)
    st = _Storage()
    a, b = Tx(t1, balance), Tx(t2, balance)
    path: list = a.setup + a.dispatch(0xE46DCFEB)            # initWallet(address[],uint256,uint256)
    off = a.word(4)                                          # _owners: head word = offset
    length = a.word(BVV(4, 256) + off)                       # _owners.length at 4 + offset
    required, daylimit = a.word(36), a.word(68)
    path.append(st[S_NUM_OWNERS] == BVV(0, 256))             # only_uninitialized
    st[S_DAILY_LIMIT] = daylimit                             # initDaylimit
    st[S_LAST_DAY] = UDiv(a.timestamp, BVV(86400, 256))      # today()
    st[S_NUM_OWNERS] = length + BVV(1, 256)                  # initMultiowned
    st[S_OWNERS + 1] = a.sender
    k1, c1 = _mapping_slot(kfm, a.sender, S_OWNER_INDEX)
    path.append(c1)
    st[k1] = BVV(1, 256)
    for i in range(n_loop):                                  # bounded loop (-b 3)
        path.append(ULT(BVV(i, 256), length))
        owner = a.word(BVV(4 + 32 * (i + 1), 256) + off)
        st[S_OWNERS + 2 + i] = owner
        ki, ci = _mapping_slot(kfm, owner, S_OWNER_INDEX)
        path.append(ci)
        st[ki] = BVV(2 + i, 256)
    path.append(Not(ULT(BVV(n_loop, 256), length)))         # loop exit
    st[S_REQUIRED] = required

    # tx 2: kill(address _to) onlymanyowners(keccak256(msg.data))
    path += b.setup + b.dispatch(0xCBF0B0C0)
    to = Concat(BVV(0, 96), Extract(159, 0, b.word(4)))
    op = BVS(f"KECCAC_mem[{0x5EED + variant}]", 256)          # SHA3 over a symbolic length
    k2, c2 = _mapping_slot(kfm, b.sender, S_OWNER_INDEX)
    path.append(c2)
    owner_index = st[k2]
    kp, cp = _mapping_slot(kfm, op, S_PENDING)
    path.append(cp)
    yet_needed = st[kp]
    owners_done = st[kp + BVV(1, 256)]
    bit = BVS(f"invhash({variant})**invhash(owner_index_{t2})", 256)
    out: List[Tuple[str, list, Optional[str]]] = []
    out.append(("wallet:ownerIndex==0 (not an owner)", path + [owner_index == BVV(0, 256)], None))
    path.append(Not(owner_index == BVV(0, 256)))
    out.append(("wallet:owner", list(path), "sat"))
    fresh = path + [yet_needed == BVV(0, 256)]
    needed = st[S_REQUIRED]                                  # pending.yetNeeded = m_required
    out.append(("wallet:new operation", list(fresh), "sat"))
    confirm = fresh + [(owners_done & bit) == BVV(0, 256)]
    out.append(("wallet:not yet confirmed", list(confirm), "sat"))
    out.append(("wallet:more confirmations needed", confirm + [UGT(needed, BVV(1, 256))], "sat"))
    killed = confirm + [Not(UGT(needed, BVV(1, 256)))]
    out.append(("wallet:kill runs", list(killed), "sat"))
    # SELFDESTRUCT(_to): the suicide module's query over both transactions
    out.append(("wallet:attacker query", killed + _attacker_query([a, b], to), "sat"))
    # the sender that initialised the wallet is an owner: ownerIndex == 0 is UNSAT for it
    out.append(("wallet:initializer not owner", path[:-1] + [b.sender == a.sender, owner_index == BVV(0, 256)],
                "unsat"))
    return [(l, tuple(c.raw for c in cs), e) for l, cs, e in out]


def corpus(n: int) -> List[Tuple[str, tuple, Optional[str]]]:
    """n entries cycling over the suicide, BECToken and WalletLibrary shapes."""
    kfm = KeccakFunctionManager()
    out: List[Tuple[str, tuple, Optional[str]]] = []
    k = 0
    while len(out) < n:
        r = k % 4
        if r == 0:
            out.extend(suicide_states(1 + (k // 4) % 5))
        elif r == 1:
            out.extend(wallet_states(k // 4, kfm))
        else:
            out.extend(bectoken_states(6 * k + j, kfm) for j in range(6))
        k += 1
    return out[:n]


# ------------------------------------------------------------- the 13-contract suite
def suite(hasher=None, max_open: int = 6, contracts=None):
    """Every contract of solidity_examples/ through the LASER restatement (corpus.laser,
    corpus.contracts): -> list of (contract, kind, label, terms, expected) queries in the
    order a `myth analyze <contract> -t N` run asks them (kind: prune / model / dep / txseq).
    The last field is the index of the query's parent (the prune query that established the
    asking state; -1 for none): the plugin hands a child its parent's witness.

    `hasher(bytes) -> bytes` is the concrete Keccak-256 the keccak manager uses for concrete
    preimages (default: the product's GPU batch, mythril_amd.keccak; CPU tests pass a CPU
    one).  Each contract gets a fresh manager, as each `myth analyze` run does."""
    from . import contracts as C
    from .laser import analyze

    out = []
    for cls in C.ALL:
        if contracts is not None and cls.name not in contracts:
            continue
        kfm = KeccakFunctionManager()
        if hasher is not None:
            def fck(data, _h=hasher):
                d = _h(data.value.to_bytes(data.size() // 8, byteorder="big"))
                return symbol_factory.BitVecVal(int.from_bytes(d, "big"), 256)
            kfm.find_concrete_keccak = fck
        run = analyze(cls(), kfm, max_open=max_open)
        base = len(out)
        out.extend((cls.name, kind, label, terms, exp, -1 if par < 0 else base + par)
                   for kind, label, terms, exp, par in run.queries)
    # a query is asked on a state its parent query established: a "sat" read off the query's
    # own constraint holds only if that state is reachable.  Under a parent expected "unsat"
    # it is dropped (the label ends in UNDER_UNSAT_PARENT).  Under an ancestor whose
    # expectation reading leaves open it stays "sat" with the label suffix SAT_IF_REACHABLE:
    # account() then counts a refutation of it as a contradiction unless an ancestor of it is
    # refuted as well (an unsound refutation must not hide behind an unlabelled
    # parent)
    for k, (c, kind, label, terms, exp, par) in enumerate(out):
        if exp != "sat" or par < 0:
            continue
        if out[par][4] == "unsat":
            out[k] = (c, kind, label + UNDER_UNSAT_PARENT, terms, None, par)
        elif out[par][4] is None or out[par][2].endswith(SAT_IF_REACHABLE):
            out[k] = (c, kind, label + SAT_IF_REACHABLE, terms, exp, par)
    return out


SAT_IF_REACHABLE = " [sat if its parent state is reachable]"
UNDER_UNSAT_PARENT = " [parent expected unsat]"


def ancestors(queries, k):
    """Indices of query k's ancestors along the parent links, nearest first."""
    out = []
    p = queries[k][5]
    while p >= 0:
        out.append(p)
        p = queries[p][5]
    return out


def held_out() -> set:
    from .contracts import HELD_OUT
    return set(HELD_OUT)


def account(queries, answers, held=None) -> dict:
    """Solver calls of the reference and of the pre-filter path for `suite()` queries.

    answers[k] is the pre-filter's 'sat' (GPU witness) / 'unsat' (host refutation) /
    'undecided' for queries[k].  The reference makes one z3 call per query, except that
    get_model is lru_cached (analysis/solver.py:27): a repeated SAT-only, dependency or
    tx-sequence query with identical constraints is one call.  The pre-filter path makes:
      prune / model / dep: one fallback call when undecided;
      txseq: one z3 Optimize call unless refuted -- a GPU witness does not save it, the
      minimised model values go into the report (analysis/solver.py:88-136).
    A contradiction is a GPU witness on an expected-unsat query or a refutation of an
    expected-sat one (expectations by reading, corpus.laser)."""
    held = held_out() if held is None else held
    import collections

    per = collections.OrderedDict()
    seen = set()
    for qi, ((contract, kind, label, terms, exp, _parent), ans) in enumerate(zip(queries, answers)):
        c = per.setdefault(contract, {"queries": 0, "ref_calls": 0, "z3_calls": 0, "sat": 0, "unsat": 0,
                                      "undecided": 0, "contradicted": 0, "expected_sat": 0, "expected_sat_witness": 0,
                                      "expected_unsat": 0, "expected_unsat_refuted": 0, "sat_if_reachable": 0,
                                      "refuted_with_sat_expectation_if_reachable": 0,
                                      "refuted_if_reachable_ancestor_refuted": 0,
                                      "by_kind": {k: {"queries": 0, "ref_calls": 0, "z3_calls": 0}
                                                  for k in ("prune", "model", "dep", "txseq")}})
        c["queries"] += 1
        c[ans] += 1
        bk = c["by_kind"][kind]
        bk["queries"] += 1
        if exp == "sat" and label.endswith(SAT_IF_REACHABLE):
            # (every occurrence, not only the lru-distinct ones counted below)
            c["sat_if_reachable"] += 1
            if ans == "unsat":
                if any(answers[a] == "unsat" for a in ancestors(queries, qi)):
                    c["refuted_if_reachable_ancestor_refuted"] += 1
                else:
                    c["refuted_with_sat_expectation_if_reachable"] += 1
        if kind != "prune":
            key = (contract, kind, terms)
            if key in seen:
                continue
            seen.add(key)
        c["ref_calls"] += 1
        bk["ref_calls"] += 1
        z3 = (ans != "unsat") if kind == "txseq" else (ans == "undecided")
        c["z3_calls"] += z3
        bk["z3_calls"] += z3
        if exp == "unsat":
            c["expected_unsat"] += 1
            c["expected_unsat_refuted"] += ans == "unsat"
            c["contradicted"] += ans == "sat"
        elif exp == "sat":
            c["expected_sat"] += 1
            c["expected_sat_witness"] += ans == "sat"
            if ans == "unsat":
                # a refuted sat-if-reachable query is consistent only under a refuted ancestor
                c["contradicted"] += not (label.endswith(SAT_IF_REACHABLE) and
                                          any(answers[a] == "unsat" for a in ancestors(queries, qi)))
    for c in per.values():
        c["reduction"] = c["ref_calls"] / max(1, c["z3_calls"])
        c["held_out"] = False
    dropped = collections.Counter(q[0] for q in queries if q[2].endswith(UNDER_UNSAT_PARENT))
    for name, c in per.items():
        c["sat_expectations_dropped"] = dropped.get(name, 0)
    for name in per:
        per[name]["held_out"] = name in held

    def total(names):
        r = sum(per[n]["ref_calls"] for n in names)
        z = sum(per[n]["z3_calls"] for n in names)
        return {"contracts": len(names), "queries": sum(per[n]["queries"] for n in names), "ref_calls": r,
                "z3_calls": z, "reduction": r / max(1, z),
                "contradicted": sum(per[n]["contradicted"] for n in names),
                "sat_expectations_dropped": sum(per[n]["sat_expectations_dropped"] for n in names),
                **{f: sum(per[n][f] for n in names) for f in (
                    "sat_if_reachable", "refuted_with_sat_expectation_if_reachable",
                    "refuted_if_reachable_ancestor_refuted")},
                "by_kind": {k: {f: sum(per[n]["by_kind"][k][f] for n in names) for f in ("queries", "ref_calls",
                                                                                     "z3_calls")}
                            for k in ("prune", "model", "dep", "txseq")}}
    names = list(per)
    return {"by_contract": dict(per), "all": total(names),
            "tuned": total([n for n in names if n not in held]),
            "held_out": total([n for n in names if n in held])}


def answer(pf, queries):
    """Answer `suite()` queries with a Prefilter the way the plugin feeds it: level by level
    along the parent links (a query is asked once the state it extends is answered), each
    query given its parent's witness when the parent was SAT (mythril_amd.plugin: a child
    inherits its parent's witness as its first candidate).  -> (answers, witnesses)."""
    n = len(queries)
    depth = [0] * n
    for i, q in enumerate(queries):
        depth[i] = depth[q[5]] + 1 if q[5] >= 0 else 0
    answers = [None] * n
    wits = [None] * n
    levels = {}
    for i, d in enumerate(depth):
        levels.setdefault(d, []).append(i)
    for d in sorted(levels):
        idx = levels[d]
        par = [wits[queries[i][5]] if queries[i][5] >= 0 else None for i in idx]
        res = pf.check_states([list(queries[i][3]) for i in idx], parents=par)
        for i, (a, w) in zip(idx, res):
            answers[i] = a
            wits[i] = w if a == "sat" else None
    return answers, wits
