"""KeccakFunctionManager mirror + batched concrete Keccak-256 on the GPU.

Mirrors mythril/laser/ethereum/keccak_function_manager.py:21-149 (same
method names, constants and constraint shapes):

  find_concrete_keccak(data)      40-54   concrete hash of data.size()//8 big-endian bytes
  get_function(length)            56-69   UF pair keccak256_<n> / keccak256_<n>-1
  get_empty_keccak_hash()         71-78
  create_keccak(data)             80-98   (hash term, condition)
  get_concrete_hash_data(model)   100-116
  _create_condition(func_input)   118-146 interval [index*PART, index*PART+PART), %64 == 0,
                                          OR over the concrete hashes seen so far

The concrete hashes go through the HIP Keccak kernel (libmgp.so,
mgp_keccak256_batch) — one launch for a whole batch via
`find_concrete_keccak_batch` — instead of pyethereum's utils.sha3.
`get_code_hash` / `get_code_hashes` mirror support/support_utils.py:29-41
(pysha3 keccak_256 of the bytecode) on the same kernel, and
`replace_with_actual_sha` mirrors the report-time substitution of
analysis/solver.py:159-192 with all of its hashes in one batch.
"""
from __future__ import annotations

from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np

from .smt import And, BitVec, Bool, Function, Or, ULE, ULT, URem, symbol_factory

TOTAL_PARTS = 10 ** 40
PART = (2 ** 256 - 1) // TOTAL_PARTS
INTERVAL_DIFFERENCE = 10 ** 30
hash_matcher = "fffffff"

_ctx = None


def _context():
    global _ctx
    if _ctx is None:
        from . import _native as N

        _ctx = N.Context(0)
    return _ctx


def keccak256_batch(preimages: Sequence[bytes]) -> List[bytes]:
    """Keccak-256 of many byte strings in one GPU launch per distinct length."""
    out: List[Optional[bytes]] = [None] * len(preimages)
    by_len: Dict[int, List[int]] = {}
    for i, p in enumerate(preimages):
        by_len.setdefault(len(p), []).append(i)
    ctx = _context()
    for ln, idx in by_len.items():
        # empty preimages: stride 0 over a 1-byte dummy buffer (every lane hashes the empty string)
        buf = np.frombuffer(b"".join(preimages[i] for i in idx), dtype=np.uint8) if ln else np.zeros(1, np.uint8)
        dig = ctx.keccak256_n(buf, len(idx), ln, ln)
        for k, i in enumerate(idx):
            out[i] = dig[k].tobytes()
    return out  # type: ignore[return-value]


def keccak256(data: bytes) -> bytes:
    return keccak256_batch([data])[0]


def _code_bytes(code: str) -> Optional[bytes]:
    code = code[2:] if code[:2] == "0x" else code
    try:
        return bytes.fromhex(code)
    except ValueError:
        return None


def get_code_hashes(codes: Sequence[str]) -> List[str]:
    """get_code_hash over many bytecodes, one GPU launch per distinct length."""
    raw = [_code_bytes(c) for c in codes]
    ok = [i for i, r in enumerate(raw) if r is not None]
    digs = keccak256_batch([raw[i] for i in ok]) if ok else []
    out = [""] * len(codes)
    for i, d in zip(ok, digs):
        out[i] = "0x" + d.hex()
    return out


def get_code_hash(code: str) -> str:
    """support/support_utils.py:29-41: "0x" + keccak-256 hex of the bytecode, "" if not hex."""
    return get_code_hashes([code])[0]


class KeccakFunctionManager:
    def __init__(self):
        self.store_function: Dict[int, Tuple[Function, Function]] = {}
        self.interval_hook_for_size: Dict[int, int] = {}
        self._index_counter = TOTAL_PARTS - 34534
        self.hash_result_store: Dict[int, List[BitVec]] = {}
        self.quick_inverse: Dict[BitVec, BitVec] = {}
        self.concrete_hashes: Dict[BitVec, BitVec] = {}

    @staticmethod
    def find_concrete_keccak(data: BitVec) -> BitVec:
        digest = keccak256(data.value.to_bytes(data.size() // 8, byteorder="big"))
        return symbol_factory.BitVecVal(int.from_bytes(digest, "big"), 256)

    @staticmethod
    def find_concrete_keccak_batch(datas: Sequence[BitVec]) -> List[BitVec]:
        digs = keccak256_batch([d.value.to_bytes(d.size() // 8, byteorder="big") for d in datas])
        return [symbol_factory.BitVecVal(int.from_bytes(h, "big"), 256) for h in digs]

    def get_function(self, length: int) -> Tuple[Function, Function]:
        try:
            func, inverse = self.store_function[length]
        except KeyError:
            func = Function("keccak256_{}".format(length), length, 256)
            inverse = Function("keccak256_{}-1".format(length), 256, length, inverse_of=func)
            self.store_function[length] = (func, inverse)
            self.hash_result_store[length] = []
        return func, inverse

    @staticmethod
    def get_empty_keccak_hash() -> BitVec:
        val = 89477152217924674838424037953991966239322087453347756267410168184682657981552
        return symbol_factory.BitVecVal(val, 256)

    def create_keccak(self, data: BitVec) -> Tuple[BitVec, Bool]:
        length = data.size()
        func, inverse = self.get_function(length)
        if data.symbolic is False:
            concrete_hash = self.find_concrete_keccak(data)
            self.concrete_hashes[data] = concrete_hash
            condition = And(func(data) == concrete_hash, inverse(func(data)) == data)
            return concrete_hash, condition
        condition = self._create_condition(func_input=data)
        self.hash_result_store[length].append(func(data))
        return func(data), condition

    def get_concrete_hash_data(self, model) -> Dict[int, List[Optional[int]]]:
        concrete_hashes: Dict[int, List[Optional[int]]] = {}
        for size in self.hash_result_store:
            concrete_hashes[size] = []
            for val in self.hash_result_store[size]:
                v = _as_int(model.eval(val.raw))
                if v is not None:
                    concrete_hashes[size].append(v)
        return concrete_hashes

    def _create_condition(self, func_input: BitVec) -> Bool:
        length = func_input.size()
        func, inv = self.get_function(length)
        try:
            index = self.interval_hook_for_size[length]
        except KeyError:
            self.interval_hook_for_size[length] = self._index_counter
            index = self._index_counter
            self._index_counter -= INTERVAL_DIFFERENCE
        lower_bound = index * PART
        upper_bound = lower_bound + PART
        cond = And(
            inv(func(func_input)) == func_input,
            ULE(symbol_factory.BitVecVal(lower_bound, 256), func(func_input)),
            ULT(func(func_input), symbol_factory.BitVecVal(upper_bound, 256)),
            URem(func(func_input), symbol_factory.BitVecVal(64, 256)) == 0,
        )
        concrete_cond = symbol_factory.Bool(False)
        for key, keccak in self.concrete_hashes.items():
            hash_eq = And(func(func_input) == keccak, key == func_input)
            concrete_cond = Or(concrete_cond, hash_eq)
        return And(inv(func(func_input)) == func_input, Or(cond, concrete_cond))

    def interval_values(self, length: int, k: int = 4) -> List[int]:
        """Candidate hash values for keccak256_<length>: aligned points of its interval."""
        if length not in self.interval_hook_for_size:
            return []
        lo = self.interval_hook_for_size[length] * PART
        lo += (-lo) % 64
        return [lo + 64 * j for j in range(k)]


keccak_function_manager = KeccakFunctionManager()


def _as_int(v) -> Optional[int]:
    """A model value as an int: z3 numerals (as_long), plain ints, else None."""
    if v is None or isinstance(v, bool):
        return None
    if hasattr(v, "as_long"):
        try:
            return int(v.as_long())
        except Exception:
            return None
    return int(v) if isinstance(v, (int, np.integer)) else None


def _hash_substitutions(tx_input: str, s_index: int, concrete_hashes, manager, model):
    """The (window start, preimage BitVec) pairs analysis/solver.py:170-183 finds in one input."""
    out = []
    for i in range(s_index, len(tx_input)):
        data_slice = tx_input[i: i + 64]
        if hash_matcher not in data_slice or len(data_slice) != 64:
            continue
        find_input = int(data_slice, 16)
        input_ = None
        for size in concrete_hashes:
            _, inverse = manager.store_function[size]
            if find_input not in concrete_hashes[size]:
                continue
            v = _as_int(model.eval(inverse(symbol_factory.BitVecVal(find_input, 256)).raw))
            if v is None:  # the reference's as_long() would raise here; leave the window alone
                continue
            input_ = symbol_factory.BitVecVal(v, size)
        if input_ is not None:
            out.append((i, input_))
    return out


def replace_with_actual_sha(concrete_transactions: List[Dict[str, str]], model, code=None,
                            manager: Optional[KeccakFunctionManager] = None, hasher=None) -> None:
    """analysis/solver.py:159-192 (`_replace_with_actual_sha`): every 64-hex-digit window of a
    transaction's input that contains `hash_matcher` and equals a hash value of the model is
    replaced by the real Keccak-256 of the preimage the model gives its inverse.

    Same scan and the same in-place replacement order as the reference (a window is read from
    the input as already rewritten by earlier windows).  The hashing is batched: a first pass
    over the unmodified inputs collects every preimage and hashes them in one launch
    (`hasher`: list of BitVec -> list of BitVec, default the GPU kernel); the exact
    sequential pass then reads that table and hashes the rare preimage it did not predict.
    """
    manager = manager or keccak_function_manager
    hasher = hasher or KeccakFunctionManager.find_concrete_keccak_batch
    concrete_hashes = manager.get_concrete_hash_data(model)

    def start(tx) -> Optional[int]:
        if hash_matcher not in tx["input"]:
            return None
        if code is not None and code.bytecode in tx["input"]:
            return len(code.bytecode) + 2
        return 10

    table: Dict[Tuple[int, int], int] = {}

    def fill(preimages):
        todo = [p for p in preimages if (p.value, p.size()) not in table]
        if todo:
            for p, h in zip(todo, hasher(todo)):
                table[(p.value, p.size())] = h.value

    predicted = []
    for tx in concrete_transactions:
        s_index = start(tx)
        if s_index is not None:
            predicted.extend(p for _, p in _hash_substitutions(tx["input"], s_index, concrete_hashes, manager,
                                                               model))
    fill(predicted)

    for tx in concrete_transactions:
        s_index = start(tx)
        if s_index is None:
            continue
        for i in range(s_index, len(tx["input"])):
            subs = _hash_substitutions(tx["input"][: i + 64], i, concrete_hashes, manager, model)
            if not subs:
                continue
            _, input_ = subs[0]
            fill([input_])
            hex_keccak = hex(table[(input_.value, input_.size())])[2:].rjust(64, "0")
            tx["input"] = tx["input"][:s_index] + tx["input"][s_index:].replace(tx["input"][i: 64 + i], hex_keccak)
