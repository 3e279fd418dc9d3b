"""The 13 contracts of solidity_examples/ restated for corpus.laser (test and bench side).

Each class mirrors one contract's functions as the solc dispatcher reaches them (selectors
sorted ascending, computed once from the signatures' keccak), with the storage layout solc
gives the contract, and each function body as the JUMPIs, storage accesses, SHA3s, calls
and arithmetic LASER executes on it.  Branch feasibility (`t=` / `f=`) is by reading the
contract: True / False where the path decides it, None where it depends on which earlier
transaction opened the state (the branch is followed and its query carries no
expectation).  Line references are to /root/reference/solidity_examples/<file>.
"""
from __future__ import annotations

from typing import List

from mythril_amd.smt import If, Not, Or, UDiv, UGE, UGT, ULE, ULT, Extract, symbol_factory

from .laser import ATTACKER, CONTRACT_ADDRESS, CREATOR, ETHER, Contract, Path

BVV, BVS = symbol_factory.BitVecVal, symbol_factory.BitVecSym
MASK160 = (1 << 160) - 1
WEEK = 7 * 24 * 3600


def _ret(p: Path) -> List[Path]:
    return [] if p is None else [p]


def _transfer_gas(value):
    """`addr.transfer(v)` (solc): CALL gas = ISZERO(v) * 2300 -- never above the stipend."""
    return If(value == BVV(0, 256), BVV(1, 256), BVV(0, 256)) * BVV(2300, 256)


def _send(p: Path, to, value, label: str, thief=None, value_pos=True) -> List[Path]:
    """`to.transfer(value)`: the call, then `require(success)` (a failed transfer reverts)."""
    rv = p.call(to, value, _transfer_gas(value), label, gas_ok=False, to_attacker=None, value_pos=value_pos,
                thief=thief)
    ok = p.require(Not(rv == BVV(0, 256)), f"{label}:success")
    if ok is not None:
        ok.retvals[-1] = (ok.retvals[-1][0], rv, False)   # checked: retval == 0 is UNSAT
    return _ret(ok)


# --------------------------------------------------------------------- suicide.sol
class Suicide(Contract):
    """suicide.sol:3-7 -- kill(addr): if (addr == 0) selfdestruct(addr).  -t 1 (config 1)."""
    name, tx_count = "suicide", 1

    def kill(self, p: Path):
        addr = p.tx.address_arg(0)
        t, f = p.branch(addr == BVV(0, 256), "kill:addr==0")
        t.selfdestruct(addr, "kill:selfdestruct", attacker_to=False)   # addr == 0 != ATTACKER
        return [t, f]

    def __init__(self):
        self.functions = [("kill", 0xCBF0B0C0, False, self.kill)]


# --------------------------------------------------------------------- BECToken.sol
class BECToken(Contract):
    """BECToken.sol: slot 0 totalSupply, 1 balances, 2 allowed, 3 owner | paused << 160
    (packed), 4-7 name/symbol/version/decimals.  -t 2 (config 2)."""
    name, tx_count = "bectoken", 2
    S_SUPPLY, S_BAL, S_ALLOWED, S_OWNER = 0, 1, 2, 3

    def constructor(self, p: Path):
        p = p.require(p.tx.value == BVV(0, 256), "constructor:callvalue", f=True)   # non-payable
        p.sstore(self.S_OWNER, BVV(CREATOR, 256))                     # owner = msg.sender, paused = false
        p.sstore(self.S_SUPPLY, BVV(7 * 10 ** 27, 256))
        h = p.mapping(BVV(CREATOR, 256), self.S_BAL, "constructor:balances")
        p.sstore(h, BVV(7 * 10 ** 27, 256))
        return [p]

    def _owner(self, p):
        return p.sload(self.S_OWNER) & BVV(MASK160, 256)

    def _paused(self, p):
        return UDiv(p.sload(self.S_OWNER), BVV(1 << 160, 256)) & BVV(0xFF, 256)

    def _not_paused(self, p, fn):
        return p.require(self._paused(p) == BVV(0, 256), f"{fn}:whenNotPaused", t=None, f=None)

    def _safe_sub(self, p, a, b, site):
        """SafeMath.sub (BECToken.sol:20-23): assert(b <= a), then a - b (no underflow left)."""
        p = p.assert_(ULE(b, a), f"{site}:assert", t=True, f=False)
        return p, (None if p is None else p.sub(a, b, site, sat=False))

    def _safe_add(self, p, a, b, site, overflow=None):
        """SafeMath.add (BECToken.sol:25-29): c = a + b, assert(c >= a)."""
        c = p.add(a, b, site, sat=overflow, sat_at_end=False)
        p = p.assert_(UGE(c, a), f"{site}:assert", t=True, f=overflow)
        return p, c

    def transfer(self, p):
        p = self._not_paused(p, "transfer")
        if p is None:
            return []
        to, value = p.tx.address_arg(0), p.tx.arg(1)
        p = p.require(Not(to == BVV(0, 256)), "transfer:to!=0")
        p = p.require(UGT(value, BVV(0, 256)), "transfer:value>0")
        hs = p.mapping(p.tx.sender, self.S_BAL, "transfer:bal_sender")
        p = p.require(ULE(value, p.sload(hs)), "transfer:value<=bal", t=True if p.tx.index == 1 else None)
        if p is None:
            return []
        p, r = self._safe_sub(p, p.sload(hs), value, "SafeMath.sub")
        p.sstore(hs, r)
        ht = p.mapping(to, self.S_BAL, "transfer:bal_to")
        p, c = self._safe_add(p, p.sload(ht), value, "SafeMath.add", overflow=False if p.tx.index == 1 else None)
        if p is None:
            return []
        p.sstore(ht, c)
        return [p]

    def transfer_from(self, p):
        p = self._not_paused(p, "transferFrom")
        if p is None:
            return []
        frm, to, value = p.tx.address_arg(0), p.tx.address_arg(1), p.tx.arg(2)
        p = p.require(Not(to == BVV(0, 256)), "transferFrom:to!=0")
        p = p.require(UGT(value, BVV(0, 256)), "transferFrom:value>0")
        hf = p.mapping(frm, self.S_BAL, "transferFrom:bal_from")
        p = p.require(ULE(value, p.sload(hf)), "transferFrom:value<=bal", t=True if p.tx.index == 1 else None)
        if p is None:
            return []
        # allowed[from][sender]: keccak(sender . keccak(from . 2)); no approval exists in the
        # first transaction, so it reads 0 there
        h_allow = p.mapping(p.tx.sender, p.mapping(frm, self.S_ALLOWED, "transferFrom:allowed_from"),
                            "transferFrom:allowed_sender")
        p = p.require(ULE(value, p.sload(h_allow)), "transferFrom:value<=allowed",
                      t=False if p.tx.index == 1 else None)
        if p is None:
            return []
        p, r = self._safe_sub(p, p.sload(hf), value, "SafeMath.sub")
        p.sstore(hf, r)
        ht = p.mapping(to, self.S_BAL, "transferFrom:bal_to")
        p, c = self._safe_add(p, p.sload(ht), value, "SafeMath.add", overflow=None)
        if p is None:
            return []
        p.sstore(ht, c)
        p, r2 = self._safe_sub(p, p.sload(h_allow), value, "SafeMath.sub")
        p.sstore(h_allow, r2)
        return [p]

    def approve(self, p):
        p = self._not_paused(p, "approve")
        if p is None:
            return []
        spender, value = p.tx.address_arg(0), p.tx.arg(1)
        hs = p.mapping(spender, p.mapping(p.tx.sender, self.S_ALLOWED, "approve:allowed_sender"),
                       "approve:allowed_spender")
        p.sstore(hs, value)
        return [p]

    def batch_transfer(self, p):
        """BECToken.sol:254-268: amount = cnt * value can wrap (the CVE-2018-10299 bug)."""
        p = self._not_paused(p, "batchTransfer")
        if p is None:
            return []
        tx = p.tx
        off = tx.word(4)
        cnt, value = tx.word(BVV(4, 256) + off), tx.arg(1)
        # overflow possible at the MUL; at a transaction end it depends on the loop exit (cnt == 1 cannot wrap)
        amount = p.mul(cnt, value, "batchTransfer:mul", sat=True, sat_at_end=None)
        p = p.require(UGT(cnt, BVV(0, 256)), "batchTransfer:cnt>0")
        p = p.require(ULE(cnt, BVV(20, 256)), "batchTransfer:cnt<=20")
        p = p.require(UGT(value, BVV(0, 256)), "batchTransfer:value>0")
        hs = p.mapping(tx.sender, self.S_BAL, "batchTransfer:bal_sender")
        p = p.require(UGE(p.sload(hs), amount), "batchTransfer:bal>=amount")
        p, r = self._safe_sub(p, p.sload(hs), amount, "SafeMath.sub")
        p.sstore(hs, r)
        ends = []
        for i in range(3):                                   # the loop, within -b 3
            go, done = p.branch(ULT(BVV(i, 256), cnt), f"batchTransfer:loop{i}", t=True, f=i > 0)
            if done is not None:
                ends.append(done)
            if go is None or i == 2:
                break
            recv = go.tx.word(BVV(4 + 32 * (i + 1), 256) + off) & BVV(MASK160, 256)
            hr = go.mapping(recv, self.S_BAL, f"batchTransfer:bal_recv{i}")
            go, c = self._safe_add(go, go.sload(hr), value, "SafeMath.add", overflow=None)
            if go is None:
                break
            go.sstore(hr, c)
            p = go
        return ends

    def pause(self, p):
        p = p.require(p.tx.sender == self._owner(p), "pause:onlyOwner", t=None, f=None)
        if p is None:
            return []
        p = self._not_paused(p, "pause")
        if p is None:
            return []
        p.sstore(self.S_OWNER, p.sload(self.S_OWNER) | BVV(1 << 160, 256))
        return [p]

    def unpause(self, p):
        p = p.require(p.tx.sender == self._owner(p), "unpause:onlyOwner", t=None, f=None)
        if p is None:
            return []
        p = p.require(Not(self._paused(p) == BVV(0, 256)), "unpause:whenPaused", t=None, f=None)
        if p is None:
            return []
        p.sstore(self.S_OWNER, p.sload(self.S_OWNER) & BVV(MASK160, 256))
        return [p]

    def transfer_ownership(self, p):
        p = p.require(p.tx.sender == self._owner(p), "transferOwnership:onlyOwner", t=None, f=None)
        if p is None:
            return []
        new = p.tx.address_arg(0)
        p = p.require(Not(new == BVV(0, 256)), "transferOwnership:new!=0")
        p.sstore(self.S_OWNER, (p.sload(self.S_OWNER) & BVV(((1 << 256) - 1) ^ MASK160, 256)) | new)
        return [p]

    def balance_of(self, p):
        p.mapping(p.tx.address_arg(0), self.S_BAL, "balanceOf")
        return [p]

    def allowance(self, p):
        ha = p.mapping(p.tx.address_arg(0), self.S_ALLOWED, "allowance:owner")
        p.mapping(p.tx.address_arg(1), ha, "allowance:spender")
        return [p]

    def __init__(self):
        g = _ret
        self.functions = sorted([
            ("name", 0x06FDDE03, False, g), ("approve", 0x095EA7B3, False, self.approve),
            ("totalSupply", 0x18160DDD, False, g), ("transferFrom", 0x23B872DD, False, self.transfer_from),
            ("decimals", 0x313CE567, False, g), ("unpause", 0x3F4BA83A, False, self.unpause),
            ("version", 0x54FD4D50, False, g), ("paused", 0x5C975ABB, False, g),
            ("balanceOf", 0x70A08231, False, self.balance_of), ("batchTransfer", 0x83F12FEC, False, self.batch_transfer),
            ("pause", 0x8456CB59, False, self.pause), ("owner", 0x8DA5CB5B, False, g),
            ("symbol", 0x95D89B41, False, g), ("transfer", 0xA9059CBB, False, self.transfer),
            ("allowance", 0xDD62ED3E, False, self.allowance),
            ("transferOwnership", 0xF2FDE38B, False, self.transfer_ownership)], key=lambda f: f[1])
        self.fallback = lambda p: []      # BECToken.sol:294-297: revert()


# --------------------------------------------------------------------- WalletLibrary.sol
class WalletLibrary(Contract):
    """WalletLibrary.sol (the Parity multisig library): slots 1 m_required, 2 m_numOwners,
    3 m_dailyLimit, 4 m_spentToday, 5 m_lastDay, 6.. m_owners[256], 263 m_ownerIndex,
    264 m_pending, 265 m_pendingIndex, 266 m_txs.  -t 3 (config 4)."""
    name, tx_count = "wallet", 3
    S_REQ, S_NUM, S_LIMIT, S_SPENT, S_LAST, S_OWNERS, S_IDX, S_PEND, S_PIDX, S_TXS = 1, 2, 3, 4, 5, 6, 263, 264, 265, 266

    def _uninitialized(self, p, fn):
        return p.require(p.sload(self.S_NUM) == BVV(0, 256), f"{fn}:only_uninitialized", t=None, f=None)

    def _owner_index(self, p, who, label):
        return p.sload(p.mapping(who, self.S_IDX, label))

    def _today(self, p):
        return UDiv(p.tx.env("timestamp"), BVV(86400, 256))

    def _confirm_and_check(self, p, op, fn):
        """WalletLibrary.sol:289-324 (onlymanyowners): -> [(path, proceeds)]."""
        idx = self._owner_index(p, p.tx.sender, f"{fn}:ownerIndex")
        no, yes = p.branch(idx == BVV(0, 256), f"{fn}:ownerIndex==0", t=None, f=None)
        out = [] if no is None else [(no, False)]
        if yes is None:
            return out
        hp = yes.mapping(op, self.S_PEND, f"{fn}:pending")
        new, old = yes.branch(yes.sload(hp) == BVV(0, 256), f"{fn}:yetNeeded==0", t=None, f=None)
        for q in (new, old):
            if q is None:
                continue
            if q is new:
                q.sstore(hp, q.sload(self.S_REQ))
                q.sstore(hp + BVV(1, 256), BVV(0, 256))
                n = q.sload(self.S_PIDX)
                q.sstore(hp + BVV(2, 256), n)
                q.sstore(self.S_PIDX, q.add(n, 1, f"{fn}:pendingIndex++", sat=None))
                h_arr = q.sha3_word(BVV(self.S_PIDX, 256), f"{fn}:pendingIndex_data")
                q.sstore(h_arr + n, op)
            # 2**ownerIndex: EXP with a symbolic exponent is a fresh symbol (instructions.py:582-600);
            # the integer module annotates it with ownerIndex >= 256 (integer.py:172-190)
            bit = BVS(f"invhash({fn}_{q.tx.tid})**invhash(ownerIndex_{q.tx.tid})", 256)
            q._ann(bit, f"{fn}:exp", UGE(idx, BVV(256, 256)), sat=False, sat_at_end=False)
            done = q.sload(hp + BVV(1, 256))
            nc, c = q.branch((done & bit) == BVV(0, 256), f"{fn}:notConfirmed", t=None, f=None)
            if c is not None:
                out.append((c, False))
            if nc is None:
                continue
            last, more = nc.branch(ULE(nc.sload(hp), BVV(1, 256)), f"{fn}:yetNeeded<=1", t=None, f=None)
            if last is not None:
                last.sstore(hp, BVV(0, 256))
                last.sstore(hp + BVV(1, 256), BVV(0, 256))
                out.append((last, True))
            if more is not None:
                more.sstore(hp, more.sub(more.sload(hp), 1, f"{fn}:yetNeeded--", sat=False))
                more.sstore(hp + BVV(1, 256), more.sload(hp + BVV(1, 256)) | bit)
                out.append((more, False))
        return out

    def _multi(self, body, fn, op=None):
        def run(p):
            o = op(p) if op else BVS(f"KECCAC_mem[{fn}_{p.tx.tid}]", 256)   # keccak256(msg.data): symbolic length
            ends = []
            for q, ok in self._confirm_and_check(p, o, fn):
                ends.extend(body(q) if ok else [q])
            return ends
        return run

    def _init_daylimit(self, p, limit):
        p.sstore(self.S_LIMIT, limit)
        p.sstore(self.S_LAST, self._today(p))
        return p

    def _init_multiowned(self, p, owners_off, required, fn):
        tx = p.tx
        length = tx.word(BVV(4, 256) + owners_off)
        p.sstore(self.S_NUM, p.add(length, 1, f"{fn}:numOwners", sat=None))
        p.sstore(self.S_OWNERS + 1, tx.sender)
        p.sstore(p.mapping(tx.sender, self.S_IDX, f"{fn}:ownerIndex_sender"), BVV(1, 256))
        ends = []
        for i in range(3):                                        # the owners loop, -b 3
            go, done = p.branch(ULT(BVV(i, 256), length), f"{fn}:loop{i}", t=None, f=None)
            if done is not None:
                done.sstore(self.S_REQ, required)
                ends.append(done)
            if go is None or i == 2:
                break
            owner = tx.word(BVV(4 + 32 * (i + 1), 256) + owners_off) & BVV(MASK160, 256)
            go.sstore(self.S_OWNERS + 2 + i, owner)
            go.sstore(go.mapping(owner, self.S_IDX, f"{fn}:ownerIndex{i}"), BVV(2 + i, 256))
            p = go
        return ends

    def init_wallet(self, p):
        p = self._uninitialized(p, "initWallet")
        if p is None:
            return []
        p = self._uninitialized(p, "initWallet:initDaylimit")
        if p is None:
            return []
        p = self._init_daylimit(p, p.tx.arg(2))
        p = self._uninitialized(p, "initWallet:initMultiowned")
        return [] if p is None else self._init_multiowned(p, p.tx.word(4), p.tx.arg(1), "initWallet")

    def init_multiowned(self, p):
        p = self._uninitialized(p, "initMultiowned")
        return [] if p is None else self._init_multiowned(p, p.tx.word(4), p.tx.arg(1), "initMultiowned")

    def init_daylimit(self, p):
        p = self._uninitialized(p, "initDaylimit")
        return [] if p is None else [self._init_daylimit(p, p.tx.arg(0))]

    def kill(self, p):
        to = p.tx.address_arg(0)

        def body(q):
            q.selfdestruct(to, "kill:selfdestruct", attacker_to=None, reachable=None)
            return [q]
        return self._multi(body, "kill")(p)

    def execute(self, p):
        """WalletLibrary.sol:233-258: onlyowner, then underLimit (343-357): a day rollover
        on block.timestamp, the limit check, the call; the multisig branch is not modelled."""
        tx = p.tx
        to, value = tx.address_arg(0), tx.arg(1)
        p = p.require(UGT(self._owner_index(p, tx.sender, "execute:isOwner"), BVV(0, 256)), "execute:onlyowner",
                      t=None, f=None)
        if p is None:
            return []
        p = p.require(UGT(self._owner_index(p, tx.sender, "underLimit:isOwner"), BVV(0, 256)), "underLimit:onlyowner",
                      t=True, f=False)
        if p is None:
            return []
        roll, same = p.branch(UGT(self._today(p), p.sload(self.S_LAST)), "underLimit:today>lastDay", t=None, f=None,
                              predictable=True)
        ends = []
        for q in (roll, same):
            if q is None:
                continue
            if q is roll:
                q.sstore(self.S_SPENT, BVV(0, 256))
                q.sstore(self.S_LAST, self._today(q))
            spent = q.sload(self.S_SPENT)
            s1 = q.add(spent, value, "underLimit:add1", sat=None)
            a, b = q.branch(UGE(s1, spent), "underLimit:noWrap", t=None, f=None)
            if b is not None:
                ends.append(b)      # over the limit: the multisig path (not modelled) ends here
            if a is None:
                continue
            s2 = a.add(a.sload(self.S_SPENT), value, "underLimit:add2", sat=None)
            ok, over = a.branch(ULE(s2, a.sload(self.S_LIMIT)), "underLimit:<=limit", t=None, f=None)
            if over is not None:
                ends.append(over)
            if ok is None:
                continue
            ok.sstore(self.S_SPENT, ok.add(ok.sload(self.S_SPENT), value, "underLimit:add3", sat=None))
            ok.call(to, value, ok.tx.env("gas"), "execute:call", to_attacker=True, value_pos=None, thief=None)
            ends.append(ok)
        return ends

    def confirm(self, p):
        h = p.tx.arg(0)

        def body(q):
            ht = q.mapping(h, self.S_TXS, "confirm:txs")
            dest = q.sload(ht) & BVV(MASK160, 256)
            go, none = q.branch(Not(dest == BVV(0, 256)), "confirm:to!=0", t=None, f=None)
            ends = [] if none is None else [none]
            if go is not None:
                # m_txs is written only by execute's multisig branch (not modelled), so what the
                # destination can be depends on the stores the chain holds: no expectation
                go.call(dest, go.sload(ht + BVV(1, 256)), go.tx.env("gas"), "confirm:call", gas_ok=None,
                        to_attacker=None, value_pos=None, thief=None)
                go.sstore(ht, BVV(0, 256))
                ends.append(go)
            return ends
        return self._multi(body, "confirm", op=lambda q: h)(p)

    def revoke(self, p):
        idx = self._owner_index(p, p.tx.sender, "revoke:ownerIndex")
        no, yes = p.branch(idx == BVV(0, 256), "revoke:ownerIndex==0", t=None, f=None)
        ends = [] if no is None else [no]
        if yes is None:
            return ends
        bit = BVS(f"invhash(revoke_{p.tx.tid})**invhash(ownerIndex_{p.tx.tid})", 256)
        hp = yes.mapping(yes.tx.arg(0), self.S_PEND, "revoke:pending")
        c, nc = yes.branch(UGT(yes.sload(hp + BVV(1, 256)) & bit, BVV(0, 256)), "revoke:confirmed", t=None, f=None)
        if nc is not None:
            ends.append(nc)
        if c is not None:
            c.sstore(hp, c.add(c.sload(hp), 1, "revoke:yetNeeded++", sat=None))
            c.sstore(hp + BVV(1, 256), c.sub(c.sload(hp + BVV(1, 256)), bit, "revoke:ownersDone-=", sat=None))
            ends.append(c)
        return ends

    def change_owner(self, p):
        frm, to = p.tx.address_arg(0), p.tx.address_arg(1)

        def body(q):
            ends = []
            own, q = q.branch(UGT(self._owner_index(q, to, "changeOwner:isOwner_to"), BVV(0, 256)),
                              "changeOwner:isOwner(to)", t=None, f=None)
            if own is not None:
                ends.append(own)
            if q is None:
                return ends
            idx = self._owner_index(q, frm, "changeOwner:ownerIndex_from")
            z, q = q.branch(idx == BVV(0, 256), "changeOwner:ownerIndex==0", t=None, f=None)
            if z is not None:
                ends.append(z)
            if q is None:
                return ends
            q = q.assert_(ULT(idx, BVV(256, 256)), "changeOwner:m_owners_bounds", t=None, f=None)
            if q is None:
                return ends
            q.sstore(BVV(self.S_OWNERS, 256) + idx, to)
            q.sstore(q.mapping(frm, self.S_IDX, "changeOwner:idx_from"), BVV(0, 256))
            q.sstore(q.mapping(to, self.S_IDX, "changeOwner:idx_to"), idx)
            return ends + [q]
        return self._multi(body, "changeOwner")(p)

    def add_owner(self, p):
        owner = p.tx.address_arg(0)

        def body(q):
            ends = []
            own, q = q.branch(UGT(self._owner_index(q, owner, "addOwner:isOwner"), BVV(0, 256)),
                              "addOwner:isOwner", t=None, f=None)
            if own is not None:
                ends.append(own)
            if q is None:
                return ends
            full, q = q.branch(UGE(q.sload(self.S_NUM), BVV(250, 256)), "addOwner:numOwners>=max", t=None, f=None)
            if full is not None:
                ends.append(full)
            if q is None:
                return ends
            n = q.add(q.sload(self.S_NUM), 1, "addOwner:numOwners++", sat=None)
            q.sstore(self.S_NUM, n)
            q = q.assert_(ULT(n, BVV(256, 256)), "addOwner:m_owners_bounds", t=None, f=None)
            if q is None:
                return ends
            q.sstore(BVV(self.S_OWNERS, 256) + n, owner)
            q.sstore(q.mapping(owner, self.S_IDX, "addOwner:idx"), n)
            return ends + [q]
        return self._multi(body, "addOwner")(p)

    def remove_owner(self, p):
        owner = p.tx.address_arg(0)

        def body(q):
            ends = []
            idx = self._owner_index(q, owner, "removeOwner:ownerIndex")
            z, q = q.branch(idx == BVV(0, 256), "removeOwner:ownerIndex==0", t=None, f=None)
            if z is not None:
                ends.append(z)
            if q is None:
                return ends
            rest = q.sub(q.sload(self.S_NUM), 1, "removeOwner:numOwners-1", sat=None)
            big, q = q.branch(UGT(q.sload(self.S_REQ), rest), "removeOwner:required>rest", t=None, f=None)
            if big is not None:
                ends.append(big)
            if q is None:
                return ends
            q = q.assert_(ULT(idx, BVV(256, 256)), "removeOwner:m_owners_bounds", t=None, f=None)
            if q is None:
                return ends
            q.sstore(BVV(self.S_OWNERS, 256) + idx, BVV(0, 256))
            q.sstore(q.mapping(owner, self.S_IDX, "removeOwner:idx"), BVV(0, 256))
            return ends + [q]
        return self._multi(body, "removeOwner")(p)

    def change_requirement(self, p):
        n = p.tx.arg(0)

        def body(q):
            big, q = q.branch(UGT(n, q.sload(self.S_NUM)), "changeRequirement:n>numOwners", t=None, f=None)
            ends = [] if big is None else [big]
            if q is not None:
                q.sstore(self.S_REQ, n)
                ends.append(q)
            return ends
        return self._multi(body, "changeRequirement")(p)

    def set_daily_limit(self, p):
        n = p.tx.arg(0)

        def body(q):
            q.sstore(self.S_LIMIT, n)
            return [q]
        return self._multi(body, "setDailyLimit")(p)

    def reset_spent_today(self, p):
        def body(q):
            q.sstore(self.S_SPENT, BVV(0, 256))
            return [q]
        return self._multi(body, "resetSpentToday")(p)

    def is_owner(self, p):
        self._owner_index(p, p.tx.address_arg(0), "isOwner")
        return [p]

    def has_confirmed(self, p):
        p.mapping(p.tx.arg(0), self.S_PEND, "hasConfirmed:pending")
        idx = self._owner_index(p, p.tx.address_arg(1), "hasConfirmed:ownerIndex")
        z, q = p.branch(idx == BVV(0, 256), "hasConfirmed:ownerIndex==0", t=None, f=None)
        return [x for x in (z, q) if x is not None]

    def get_owner(self, p):
        i1 = p.add(p.tx.arg(0), 1, "getOwner:add", sat=True, sat_at_end=True)
        p = p.assert_(ULT(i1, BVV(256, 256)), "getOwner:m_owners_bounds", t=True, f=True)
        return _ret(p)

    def fallback_fn(self, p):
        t, f = p.branch(UGT(p.tx.value, BVV(0, 256)), "fallback:value>0")
        return [t, f]

    def __init__(self):
        g = _ret
        self.functions = sorted([
            ("removeOwner", 0x173825D9, False, self.remove_owner), ("isOwner", 0x2F54BF6E, False, self.is_owner),
            ("m_numOwners", 0x4123CB6B, False, g), ("m_lastDay", 0x52375093, False, g),
            ("resetSpentToday", 0x5C52C2F5, False, self.reset_spent_today), ("m_spentToday", 0x659010E7, False, g),
            ("addOwner", 0x7065CB48, False, self.add_owner), ("m_required", 0x746C9171, False, g),
            ("confirm", 0x797AF627, False, self.confirm), ("initDaylimit", 0x9DA5E0EB, False, self.init_daylimit),
            ("setDailyLimit", 0xB20D30A9, False, self.set_daily_limit), ("execute", 0xB61D27F6, False, self.execute),
            ("revoke", 0xB75C7DC6, False, self.revoke), ("changeRequirement", 0xBA51A6DF, False, self.change_requirement),
            ("hasConfirmed", 0xC2CF7326, False, self.has_confirmed), ("getOwner", 0xC41A360A, False, self.get_owner),
            ("initMultiowned", 0xC57C5F60, False, self.init_multiowned), ("kill", 0xCBF0B0C0, False, self.kill),
            ("initWallet", 0xE46DCFEB, False, self.init_wallet), ("changeOwner", 0xF00D4B5D, False, self.change_owner),
            ("m_dailyLimit", 0xF1736D86, False, g)], key=lambda f: f[1])
        self.fallback = self.fallback_fn
        self.fallback_payable = True


# --------------------------------------------------------------------- calls.sol
class Calls(Contract):
    """calls.sol: slot 0 fixed_address (constructor argument), 1 stored_address, 2 statevar."""
    name = "calls"

    def constructor(self, p):
        p = p.require(p.tx.value == BVV(0, 256), "constructor:callvalue")
        p.sstore(0, p.tx.address_arg(0))   # constructor(address addr): a symbolic creation argument
        return [p]

    def _call(self, p, to, label, to_attacker=True):
        p.call(to, BVV(0, 256), p.tx.env("gas"), label, gas_ok=True, to_attacker=to_attacker, thief=False)
        return p

    def thisisfine(self, p):
        return [self._call(p, p.sload(0) & BVV(MASK160, 256), "thisisfine:call")]

    def reentrancy(self, p):
        p = self._call(p, p.sload(0) & BVV(MASK160, 256), "reentrancy:call")
        p.sstore(2, BVV(0, 256))                       # state change after the call
        return [p]

    def calluseraddress(self, p):
        return [self._call(p, p.tx.address_arg(0), "calluseraddress:call")]

    def callstoredaddress(self, p):
        # stored_address is 0 until setstoredaddress ran in an earlier transaction
        return [self._call(p, p.sload(1) & BVV(MASK160, 256), "callstoredaddress:call",
                           to_attacker=False if p.tx.index == 1 else None)]

    def setstoredaddress(self, p):
        p.sstore(1, p.tx.address_arg(0))
        return [p]

    def __init__(self):
        g = _ret
        self.functions = sorted([
            ("setstoredaddress", 0x2776B163, False, self.setstoredaddress), ("fixed_address", 0x379BF63C, False, g),
            ("thisisfine", 0x5A6814EC, False, self.thisisfine), ("stored_address", 0xB5D02C8A, False, g),
            ("callstoredaddress", 0xD24B08CC, False, self.callstoredaddress),
            ("reentrancy", 0xE11F493E, False, self.reentrancy),
            ("calluseraddress", 0xE1D10F79, False, self.calluseraddress)], key=lambda f: f[1])


# --------------------------------------------------------------------- etherstore.sol
class EtherStore(Contract):
    """etherstore.sol: slot 0 withdrawalLimit = 1 ether, 1 lastWithdrawTime, 2 balances."""
    name = "etherstore"

    def constructor(self, p):
        p = p.require(p.tx.value == BVV(0, 256), "constructor:callvalue")
        p.sstore(0, BVV(ETHER, 256))
        return [p]

    def deposit(self, p):
        h = p.mapping(p.tx.sender, 2, "depositFunds:balances")
        first = p.tx.index == 1          # balances are all 0 before the first deposit
        c = p.add(p.sload(h), p.tx.value, "depositFunds:add", sat=False if first else None,
                  sat_at_end=False if first else None)
        p.sstore(h, c)
        return [p]

    def withdraw(self, p):
        tx = p.tx
        w = tx.arg(0)
        first = tx.index == 1
        hb = p.mapping(tx.sender, 2, "withdrawFunds:balances")
        p = p.require(UGE(p.sload(hb), w), "withdrawFunds:bal>=w", t=True, f=True)
        p = p.require(ULE(w, p.sload(0)), "withdrawFunds:w<=limit", t=True, f=False if first else None)
        if p is None:
            return []
        ht = p.mapping(tx.sender, 1, "withdrawFunds:lastWithdrawTime")
        due = p.add(p.sload(ht), WEEK, "withdrawFunds:add", sat=False if first else None)
        now = tx.env("timestamp")
        p = p.require(UGE(now, due), "withdrawFunds:now>=due", t=True, f=True, predictable=True)
        rv = p.call(tx.sender, w, tx.env("gas"), "withdrawFunds:call", gas_ok=True, to_attacker=True,
                    value_pos=False if first else None, thief=False if first else None)
        p = p.require(Not(rv == BVV(0, 256)), "withdrawFunds:success")
        p.retvals[-1] = (p.retvals[-1][0], rv, False)
        p.sstore(hb, p.sub(p.sload(hb), w, "withdrawFunds:sub", sat=False))
        p.sstore(ht, now)
        return [p]

    def __init__(self):
        g = _ret

        def mapping_getter(slot, name):
            def body(p):
                p.mapping(p.tx.address_arg(0), slot, name)
                return [p]
            return body
        self.functions = sorted([
            ("lastWithdrawTime", 0x1031EC31, False, mapping_getter(1, "lastWithdrawTime")),
            ("withdrawFunds", 0x155DD5EE, False, self.withdraw),
            ("balances", 0x27E235E3, False, mapping_getter(2, "balances")),
            ("withdrawalLimit", 0x7DDFE78D, False, g),
            ("depositFunds", 0xE2C41DBC, True, self.deposit)], key=lambda f: f[1])


# --------------------------------------------------------------------- exceptions.sol
class Exceptions(Contract):
    """exceptions.sol: uint256[8] myarray at slots 0-7; every function is pure / view."""
    name = "exceptions"

    def assert1(self, p):
        return _ret(p.assert_(BVV(1, 256) == BVV(0, 256), "assert1:assert"))      # always fails

    def assert2(self, p):
        return _ret(p.assert_(UGT(BVV(1, 256), BVV(0, 256)), "assert2:assert"))  # never fails

    def assert3(self, p):
        return _ret(p.assert_(Not(p.tx.arg(0) == BVV(23, 256)), "assert3:assert"))

    def requireisfine(self, p):
        return _ret(p.require(Not(p.tx.arg(0) == BVV(23, 256)), "requireisfine:require"))

    def divisionby0(self, p):
        x = p.tx.arg(0)
        p = p.assert_(Not(x == BVV(0, 256)), "divisionby0:div_zero")
        if p is not None:
            UDiv(BVV(1, 256), x)
        return _ret(p)

    def thisisfine(self, p):
        x = p.tx.arg(0)
        t, f = p.branch(UGT(x, BVV(0, 256)), "thisisfine:input>0")
        if t is not None:
            t = t.assert_(Not(x == BVV(0, 256)), "thisisfine:div_zero", t=True, f=False)
        return [q for q in (t, f) if q is not None]

    def arrayaccess(self, p):
        i = p.tx.arg(0)
        p = p.assert_(ULT(i, BVV(8, 256)), "arrayaccess:bounds")
        if p is not None:
            p.sload(i)
        return _ret(p)

    def thisisalsofind(self, p):
        i = p.tx.arg(0)
        t, f = p.branch(ULT(i, BVV(8, 256)), "thisisalsofind:index<8")
        if t is not None:
            t = t.assert_(ULT(i, BVV(8, 256)), "thisisalsofind:bounds", t=True, f=False)
        return [q for q in (t, f) if q is not None]

    def __init__(self):
        self.functions = sorted([
            ("thisisalsofind", 0x01D4277C, False, self.thisisalsofind), ("assert3", 0x546455B5, False, self.assert3),
            ("requireisfine", 0x78375F14, False, self.requireisfine),
            ("arrayaccess", 0x92DD38EA, False, self.arrayaccess), ("divisionby0", 0xA08299F1, False, self.divisionby0),
            ("assert1", 0xB34C3610, False, self.assert1), ("thisisfine", 0xB630D706, False, self.thisisfine),
            ("assert2", 0xF44F13D8, False, self.assert2)], key=lambda f: f[1])


# --------------------------------------------------------------------- hashforether.sol
class HashForEther(Contract):
    """hashforether.sol: no storage; _sendWinnings is public (the bug)."""
    name = "hashforether"

    def send_winnings(self, p):
        bal = p.world.balances[BVV(CONTRACT_ADDRESS, 256)]      # address(this).balance
        # the balance is positive in the first message call (the starting balance is free);
        # after an earlier call sent it all away it depends on that path (0 + non-payable 0)
        return _send(p, p.tx.sender, bal, "_sendWinnings:transfer", thief=True,
                     value_pos=True if p.tx.index == 1 else None)

    def withdraw(self, p):
        # uint32(msg.sender) == 0: no actor address ends in eight zero hex digits
        p = p.require(Extract(31, 0, p.tx.sender) == BVV(0, 32), "withdrawWinnings:require", t=False, f=True)
        return [] if p is None else self.send_winnings(p)

    def __init__(self):
        self.functions = [("_sendWinnings", 0x83AC4AE1, False, self.send_winnings),
                          ("withdrawWinnings", 0xCC42E83A, False, self.withdraw)]


# --------------------------------------------------------------------- origin.sol
class Origin(Contract):
    """origin.sol: slot 0 owner (constructor: msg.sender); onlyOwner reads tx.origin."""
    name = "origin"

    def constructor(self, p):
        p = p.require(p.tx.value == BVV(0, 256), "constructor:callvalue")
        p.sstore(0, BVV(CREATOR, 256))
        return [p]

    def transfer_ownership(self, p):
        owner = p.sload(0) & BVV(MASK160, 256)
        # tx.origin is the transaction's sender symbol (transaction/symbolic.py:90-101)
        p = p.require(Not(p.tx.sender == owner), "transferOwnership:origin!=owner", origin=True, t=True,
                      f=True if p.tx.index == 1 else None)
        if p is None:
            return []
        new = p.tx.address_arg(0)
        t, f = p.branch(Not(new == BVV(0, 256)), "transferOwnership:new!=0")
        t.sstore(0, new)
        return [t, f]

    def __init__(self):
        self.functions = [("owner", 0x8DA5CB5B, False, _ret),
                          ("transferOwnership", 0xF2FDE38B, False, self.transfer_ownership)]


# --------------------------------------------------------------------- returnvalue.sol
class ReturnValue(Contract):
    """returnvalue.sol: slot 0 callee = 0xE0f7...4229 (a fixed, concrete address)."""
    name = "returnvalue"
    CALLEE = 0xE0F7E56E62B4267062172495D7506087205A4229

    def constructor(self, p):
        p = p.require(p.tx.value == BVV(0, 256), "constructor:callvalue")
        p.sstore(0, BVV(self.CALLEE, 256))
        return [p]

    def _call(self, p, label):
        return p.call(p.sload(0) & BVV(MASK160, 256), BVV(0, 256), p.tx.env("gas"), label, gas_ok=True,
                      to_attacker=False, thief=False)

    def callnotchecked(self, p):
        self._call(p, "callnotchecked:call")
        return [p]

    def callchecked(self, p):
        rv = self._call(p, "callchecked:call")
        p = p.require(Not(rv == BVV(0, 256)), "callchecked:require")
        if p is not None:
            p.retvals[-1] = (p.retvals[-1][0], rv, False)
        return _ret(p)

    def __init__(self):
        self.functions = [("callchecked", 0x633AB5E0, False, self.callchecked), ("callee", 0xCEEE2E20, False, _ret),
                          ("callnotchecked", 0xE3BEA282, False, self.callnotchecked)]


# --------------------------------------------------------------------- rubixi.sol
class Rubixi(Contract):
    """rubixi.sol: slots 0 balance, 1 collectedFees, 2 feePercent = 10, 3 pyramidMultiplier =
    300, 4 payoutOrder, 5 creator (set only by the public dynamicPyramid: the misnamed
    constructor), 6 participants (length; elements at keccak(6) + 2i)."""
    name = "rubixi"

    def constructor(self, p):
        p = p.require(p.tx.value == BVV(0, 256), "constructor:callvalue")
        for slot, v in ((0, 0), (1, 0), (2, 10), (3, 300), (4, 0)):
            p.sstore(slot, BVV(v, 256))
        return [p]

    def _onlyowner(self, p, fn):
        """`if (msg.sender == creator) _;` -- creator is 0 until dynamicPyramid ran."""
        first = p.tx.index == 1
        t, f = p.branch(p.tx.sender == (p.sload(5) & BVV(MASK160, 256)), f"{fn}:onlyowner",
                        t=False if first else None, f=True if first else None)
        return t, ([] if f is None else [f])

    def collect_all_fees(self, p, fn="collectAllFees"):
        p = p.require(UGT(p.sload(1), BVV(0, 256)), f"{fn}:fees>0", t=None, f=None)
        if p is None:
            return []
        ends = _send(p, p.sload(5) & BVV(MASK160, 256), p.sload(1), f"{fn}:transfer", thief=None, value_pos=None)
        for q in ends:
            q.sstore(1, BVV(0, 256))
        return ends

    def collect_all(self, p):
        t, ends = self._onlyowner(p, "collectAllFees")
        return ends + ([] if t is None else self.collect_all_fees(t))

    def collect_in_ether(self, p):
        t, ends = self._onlyowner(p, "collectFeesInEther")
        if t is None:
            return ends
        amt = t.mul(t.tx.arg(0), ETHER, "collectFeesInEther:mul", sat=None)
        more, less = t.branch(UGT(amt, t.sload(1)), "collectFeesInEther:amt>fees", t=None, f=None)
        paths = ([] if less is None else [less]) + ([] if more is None else self.collect_all_fees(more))
        for q in paths:
            q = q.require(UGT(q.sload(1), BVV(0, 256)), "collectFeesInEther:fees>0", t=None, f=None)
            if q is None:
                continue
            for r in _send(q, q.sload(5) & BVV(MASK160, 256), amt, "collectFeesInEther:transfer", thief=None,
                           value_pos=None):
                r.sstore(1, r.sub(r.sload(1), amt, "collectFeesInEther:sub", sat=None))
                ends.append(r)
        return ends

    def collect_percent(self, p):
        t, ends = self._onlyowner(p, "collectPercentOfFees")
        if t is None:
            return ends
        pc = t.tx.arg(0)
        t = t.require(UGT(t.sload(1), BVV(0, 256)), "collectPercentOfFees:fees>0", t=None, f=None)
        if t is None:
            return ends
        t = t.require(ULE(pc, BVV(100, 256)), "collectPercentOfFees:pcent<=100", t=None, f=None)
        if t is None:
            return ends
        fees = t.mul(UDiv(t.sload(1), BVV(100, 256)), pc, "collectPercentOfFees:mul", sat=None)
        for r in _send(t, t.sload(5) & BVV(MASK160, 256), fees, "collectPercentOfFees:transfer", thief=None,
                       value_pos=None):
            r.sstore(1, r.sub(r.sload(1), fees, "collectPercentOfFees:sub", sat=None))
            ends.append(r)
        return ends

    def _setter(self, fn, slot, checks=()):
        def body(p):
            t, ends = self._onlyowner(p, fn)
            if t is None:
                return ends
            v = t.tx.address_arg(0) if slot == 5 else t.tx.arg(0)
            for k, c in enumerate(checks):
                t = t.require(c(v), f"{fn}:require{k}", t=None, f=None)
                if t is None:
                    return ends
            t.sstore(slot, v)
            return ends + [t]
        return body

    def dynamic_pyramid(self, p):
        p.sstore(5, p.tx.sender)
        return [p]

    def next_payout(self, p):
        # participants[payoutOrder]: the array bounds check (payoutOrder < length)
        return _ret(p.assert_(ULT(p.sload(4), p.sload(6)), "nextPayout:bounds", t=None, f=None))

    def waiting(self, p):
        p.sub(p.sload(6), p.sload(4), "numberOfParticipantsWaitingForPayout:sub", sat=None)
        return [p]

    def participant_details(self, p):
        i = p.tx.arg(0)
        t, f = p.branch(ULE(i, p.sload(6)), "participantDetails:i<=length")
        if t is not None:
            t = t.assert_(ULT(i, t.sload(6)), "participantDetails:bounds", t=None, f=True)
        return [q for q in (t, f) if q is not None]

    def fallback_fn(self, p):
        """init() (rubixi.sol:115-127) and addPayout (130-151), one payout iteration."""
        tx = p.tx
        small, big = p.branch(ULT(tx.value, BVV(ETHER, 256)), "init:value<1ether")
        ends = []
        if small is not None:
            small.sstore(1, small.add(small.sload(1), tx.value, "init:fees+=", sat=None))
            ends.append(small)
        if big is None:
            return ends
        half, full = big.branch(UGE(tx.value, BVV(50 * ETHER, 256)), "init:value>=50ether")
        for q in (half, full):
            if q is None:
                continue
            fee = UDiv(q.sload(2), BVV(2, 256)) if q is half else q.sload(2)   # _fee /= 2 at 50 ether
            n = q.sload(6)
            q.sstore(6, q.add(n, 1, "addPayout:push", sat=None))
            base = q.sha3_word(BVV(6, 256), "addPayout:participants_data")
            payout = UDiv(q.mul(tx.value, q.sload(3), "addPayout:mul_multiplier", sat=None), BVV(100, 256))
            q.sstore(base + n + n, tx.sender)
            q.sstore(base + n + n + BVV(1, 256), payout)
            q.branch(q.sload(6) == BVV(10, 256), "addPayout:length==10", t=None, f=None)
            share = UDiv(q.mul(tx.value, q.sub(100, fee, "addPayout:100-fee", sat=False), "addPayout:mul_balance",
                               sat=None), BVV(100, 256))
            q.sstore(0, q.add(q.sload(0), share, "addPayout:balance+=", sat=None))
            fees = UDiv(q.mul(tx.value, fee, "addPayout:mul_fee", sat=None), BVV(100, 256))
            q.sstore(1, q.add(q.sload(1), fees, "addPayout:fees+=", sat=None))
            q = q.assert_(ULT(q.sload(4), q.sload(6)), "addPayout:bounds", t=True if tx.index == 1 else None,
                          f=False if tx.index == 1 else None)
            if q is None:
                continue
            head = base + q.sload(4) + q.sload(4)
            pay, done = q.branch(UGT(q.sload(0), q.sload(head + BVV(1, 256))), "addPayout:balance>payout",
                                 t=None, f=None)
            if done is not None:
                ends.append(done)
            if pay is not None:
                amount = pay.sload(head + BVV(1, 256))
                for r in _send(pay, pay.sload(head) & BVV(MASK160, 256), amount, "addPayout:transfer", thief=None,
                               value_pos=None):
                    r.sstore(0, r.sub(r.sload(0), amount, "addPayout:balance-=", sat=None))
                    r.sstore(4, r.add(r.sload(4), 1, "addPayout:payoutOrder++", sat=None))
                    ends.append(r)
        return ends

    def __init__(self):
        g = _ret
        self.functions = sorted([
            ("currentPyramidBalanceApproximately", 0x09DFDC71, False, g),
            ("feesSeperateFromBalanceApproximately", 0x253459E3, False, g),
            ("collectPercentOfFees", 0x4229616D, False, self.collect_percent),
            ("nextPayoutWhenPyramidBalanceTotalsApproximately", 0x57D4021B, False, self.next_payout),
            ("collectAllFees", 0x686F2C90, False, self.collect_all), ("currentMultiplier", 0x6FBAAA1E, False, g),
            ("dynamicPyramid", 0x89B8AE9B, False, self.dynamic_pyramid), ("currentFeePercentage", 0x8A5FB3CA, False, g),
            ("participantDetails", 0x9DBC4F9B, False, self.participant_details),
            ("totalParticipants", 0xA26DBF26, False, g),
            ("changeOwner", 0xA6F9DAE1, False, self._setter("changeOwner", 5)),
            ("collectFeesInEther", 0xB4022950, False, self.collect_in_ether),
            ("changeMultiplier", 0xCED92670, False, self._setter("changeMultiplier", 3, (
                lambda v: ULE(v, BVV(300, 256)), lambda v: UGE(v, BVV(120, 256))))),
            ("numberOfParticipantsWaitingForPayout", 0xD11F13DF, False, self.waiting),
            ("changeFeePercentage", 0xFAE14192, False, self._setter("changeFeePercentage", 2, (
                lambda v: ULE(v, BVV(10, 256)),)))], key=lambda f: f[1])
        self.fallback = self.fallback_fn
        self.fallback_payable = True


# --------------------------------------------------------------------- timelock.sol
class TimeLock(Contract):
    """timelock.sol: slot 0 balances, 1 lockTime."""
    name = "timelock"

    def deposit(self, p):
        tx = p.tx
        first = tx.index == 1
        hb = p.mapping(tx.sender, 0, "deposit:balances")
        p.sstore(hb, p.add(p.sload(hb), tx.value, "deposit:add_balance", sat=False if first else None,
                           sat_at_end=False if first else None))
        ht = p.mapping(tx.sender, 1, "deposit:lockTime")
        # now + 1 weeks: the timestamp is unconstrained, so this can wrap
        p.sstore(ht, p.add(tx.env("timestamp"), WEEK, "deposit:add_now", sat=True, sat_at_end=True))
        return [p]

    def increase(self, p):
        tx = p.tx
        first = tx.index == 1
        ht = p.mapping(tx.sender, 1, "increaseLockTime:lockTime")
        p.sstore(ht, p.add(p.sload(ht), tx.arg(0), "increaseLockTime:add", sat=False if first else None,
                           sat_at_end=False if first else None))
        return [p]

    def withdraw(self, p):
        tx = p.tx
        hb = p.mapping(tx.sender, 0, "withdraw:balances")
        p = p.require(UGT(p.sload(hb), BVV(0, 256)), "withdraw:balance>0", t=None, f=None)
        if p is None:
            return []
        ht = p.mapping(tx.sender, 1, "withdraw:lockTime")
        p = p.require(UGT(tx.env("timestamp"), p.sload(ht)), "withdraw:now>lockTime", t=None, f=None,
                      predictable=True)
        if p is None:
            return []
        p.sstore(hb, BVV(0, 256))
        return _send(p, tx.sender, p.sload(hb), "withdraw:transfer", thief=False, value_pos=False)

    def __init__(self):
        def mapping_getter(slot, name):
            def body(p):
                p.mapping(p.tx.address_arg(0), slot, name)
                return [p]
            return body
        self.functions = sorted([
            ("balances", 0x27E235E3, False, mapping_getter(0, "balances")),
            ("withdraw", 0x3CCFD60B, False, self.withdraw),
            ("increaseLockTime", 0x79AF55E4, False, self.increase),
            ("lockTime", 0xA4BEDA63, False, mapping_getter(1, "lockTime")),
            ("deposit", 0xD0E30DB0, True, self.deposit)], key=lambda f: f[1])


# --------------------------------------------------------------------- token.sol
class Token(Contract):
    """token.sol: slot 0 balances, 1 totalSupply; constructor(uint _initialSupply)."""
    name = "token"

    def constructor(self, p):
        p = p.require(p.tx.value == BVV(0, 256), "constructor:callvalue")
        supply = p.tx.arg(0)                             # a symbolic creation argument
        p.sstore(1, supply)
        p.sstore(p.mapping(BVV(CREATOR, 256), 0, "constructor:balances"), supply)
        return [p]

    def transfer(self, p):
        tx = p.tx
        to, value = tx.address_arg(0), tx.arg(1)
        hs = p.mapping(tx.sender, 0, "transfer:bal_sender")
        d = p.sub(p.sload(hs), value, "transfer:sub_check", sat=True, sat_at_end=True)
        # uint >= 0 is always true: z3 simplifies ISZERO(LT(d, 0)) to True (one successor); the
        # condition still carries d's annotation to the JUMPI sink
        p._sink(d)
        p = p.require(symbol_factory.Bool(True), "transfer:require")
        p.sstore(hs, p.sub(p.sload(hs), value, "transfer:sub", sat=True, sat_at_end=True))
        ht = p.mapping(to, 0, "transfer:bal_to")
        p.sstore(ht, p.add(p.sload(ht), value, "transfer:add", sat=None))
        return [p]

    def balance_of(self, p):
        p.mapping(p.tx.address_arg(0), 0, "balanceOf")
        return [p]

    def __init__(self):
        self.functions = [("totalSupply", 0x18160DDD, False, _ret), ("balanceOf", 0x70A08231, False, self.balance_of),
                          ("transfer", 0xA9059CBB, False, self.transfer)]


# --------------------------------------------------------------------- weak_random.sol
class WeakRandom(Contract):
    """weak_random.sol: slots 0 prize = 2.5 ether, 1 totalTickets = 50, 2 pricePerTicket =
    prize / totalTickets, 3 gameId = 1, 4 nextTicket = 0, 5 contestants (struct of 2 words)."""
    name = "weak_random"
    PRICE = 25 * 10 ** 17 // 50

    def constructor(self, p):
        p = p.require(p.tx.value == BVV(0, 256), "constructor:callvalue")
        for slot, v in ((0, 25 * 10 ** 17), (1, 50), (2, self.PRICE), (3, 1), (4, 0)):
            p.sstore(slot, BVV(v, 256))
        return [p]

    def fallback_fn(self, p):
        """weak_random.sol:18-35: buy tickets while the money lasts (two iterations within the
        loop bound), then refund the rest."""
        tx = p.tx
        money = tx.value
        ends = []
        for i in range(3):
            go, stop = p.branch(UGE(money, p.sload(2)), f"fallback:money>=price{i}", t=None if i else True,
                                f=None if i else True)
            if go is not None:
                go = go.require(ULT(go.sload(4), go.sload(1)), f"fallback:next<total{i}", t=None, f=None)
            if stop is not None:
                stop.branch(stop.sload(4) == stop.sload(1), f"fallback:next==total{i}", t=None, f=None)
                has, none = stop.branch(UGT(money, BVV(0, 256)), f"fallback:refund{i}", t=None, f=None)
                if none is not None:
                    ends.append(none)
                if has is not None:
                    ends.extend(_send(has, tx.sender, money, f"fallback:transfer{i}", thief=False, value_pos=True))
            if go is None or i == 2:
                break
            cur = go.sload(4)
            go.sstore(4, go.add(cur, 1, f"fallback:nextTicket++{i}", sat=False))
            h = go.mapping(cur, 5, f"fallback:contestants{i}")
            go.sstore(h, tx.sender)
            go.sstore(h + BVV(1, 256), go.sload(3))
            money = go.sub(money, go.sload(2), f"fallback:money-=price{i}", sat=False)
            p = go
        return ends

    def contestants(self, p):
        p.mapping(p.tx.arg(0), 5, "contestants")
        return [p]

    def __init__(self):
        g = _ret
        self.functions = sorted([
            ("nextTicket", 0xC7DBBC47, False, g), ("gameId", 0xD7C81B55, False, g),
            ("totalTickets", 0xDD11247E, False, g), ("contestants", 0xDFD50F52, False, self.contestants),
            ("prize", 0xE3AC5D26, False, g), ("pricePerTicket", 0xE9874106, False, g)], key=lambda f: f[1])
        self.fallback = self.fallback_fn
        self.fallback_payable = True


ALL = [Suicide, BECToken, WalletLibrary, Calls, EtherStore, Exceptions, HashForEther, Origin, ReturnValue, Rubixi,
       TimeLock, Token, WeakRandom]
# held out: the decision-row policy and the refuter are never tuned on these (fixed before
# their first run, round 4); the bench reports their reduction separately
HELD_OUT = {"rubixi", "timelock", "token", "weak_random"}
