"""Batched concrete Keccak-256 on the GPU: the product side of the keccak path.

`find_concrete_keccak` replaces the pyethereum utils.sha3 call of
mythril/laser/ethereum/keccak_function_manager.py:40-54 with the HIP Keccak
kernel (libmgp.so, mgp_keccak256_batch); `find_concrete_keccak_batch` hashes a
whole batch in one launch.  The manager's UF modelling itself (get_function,
create_keccak, _create_condition) stays the reference's; its restatement for
the corpus and the tests is corpus/keccak_manager.py.
`get_code_hash` / `get_code_hashes` mirror support/support_utils.py:29-41
(pysha3 keccak_256 of the bytecode) on the same kernel, and
`replace_with_actual_sha` mirrors the report-time substitution of
analysis/solver.py:159-192 with all of its hashes in one batch.
"""
from __future__ import annotations

from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np

from .smt import BitVec, symbol_factory

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


def find_concrete_keccak(data: BitVec) -> BitVec:
    """keccak_function_manager.py:40-54 (`KeccakFunctionManager.find_concrete_keccak`): the
    Keccak-256 of data.size()//8 big-endian bytes, as a 256-bit value.  The one method of the
    reference's manager that LASER swaps for this."""
    digest = keccak256(data.value.to_bytes(data.size() // 8, byteorder="big"))
    return symbol_factory.BitVecVal(int.from_bytes(digest, "big"), 256)


def find_concrete_keccak_batch(datas: Sequence[BitVec]) -> List[BitVec]:
    """find_concrete_keccak over many values, one GPU launch per distinct length."""
    digs = keccak256_batch([d.value.to_bytes(d.size() // 8, byteorder="big") for d in datas])
    return [symbol_factory.BitVecVal(int.from_bytes(h, "big"), 256) for h in digs]


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
                            manager=None, hasher=None) -> None:
    """analysis/solver.py:159-192 (`_replace_with_actual_sha`): every 64-hex-digit window of a
    transaction's input that contains `hash_matcher` and equals a hash value of the model is
    replaced by the real Keccak-256 of the preimage the model gives its inverse.

    Same scan and the same in-place replacement order as the reference (a window is read from
    the input as already rewritten by earlier windows).  The hashing is batched: a first pass
    over the unmodified inputs collects every preimage and hashes them in one launch
    (`hasher`: list of BitVec -> list of BitVec, default the GPU kernel); the exact
    sequential pass then reads that table and hashes the rare preimage it did not predict.
    `manager` is the keccak function manager whose UF pairs the model speaks about (its
    `store_function` and `get_concrete_hash_data`); by default LASER's singleton.
    """
    if manager is None:  # LASER's module-level singleton (keccak_function_manager.py:149)
        try:
            from mythril.laser.ethereum.keccak_function_manager import keccak_function_manager as manager
        except ImportError as e:
            raise ValueError("replace_with_actual_sha needs `manager` (the keccak function manager whose UF "
                             "pairs the model speaks about) outside a LASER process") from e
    hasher = hasher or find_concrete_keccak_batch
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
