"""Report-time hash substitution (analysis/solver.py:159-192, `_replace_with_actual_sha`).

`mythril_amd.keccak.replace_with_actual_sha` batches the hashes; the scan and the
replacement order must stay the reference's.  CPU tests inject the oracle Keccak as
the hasher (the product default is the GPU kernel); the GPU test runs the kernel.
"""
import pytest

from corpus.keccak_manager import KeccakFunctionManager
from mythril_amd import keccak as K
from mythril_amd.smt import Concat, symbol_factory
from oracle import keccak_ref

BVV = symbol_factory.BitVecVal
BVS = symbol_factory.BitVecSym


def oracle_hasher(datas):
    return [BVV(int.from_bytes(keccak_ref.keccak256(d.value.to_bytes(d.size() // 8, "big")), "big"), 256)
            for d in datas]


class DictModel:
    """A model whose eval maps interned terms to ints (what z3's model.eval(...).as_long() gives)."""

    def __init__(self, values):
        self.values = values

    def eval(self, term, model_completion=False):
        return self.values.get(term)


def reference_replace(concrete_transactions, model, manager, code=None):
    """Straight restatement of analysis/solver.py:159-192 with one hash per window (test oracle)."""
    concrete_hashes = manager.get_concrete_hash_data(model)
    for tx in concrete_transactions:
        if K.hash_matcher not in tx["input"]:
            continue
        s_index = len(code.bytecode) + 2 if code is not None and code.bytecode in tx["input"] else 10
        for i in range(s_index, len(tx["input"])):
            data_slice = tx["input"][i: i + 64]
            if K.hash_matcher not in data_slice or len(data_slice) != 64:
                continue
            find_input = BVV(int(data_slice, 16), 256)
            input_ = None
            for size in concrete_hashes:
                _, inverse = manager.store_function[size]
                if find_input.value not in concrete_hashes[size]:
                    continue
                input_ = BVV(model.eval(inverse(find_input).raw), size)
            if input_ is None:
                continue
            keccak = oracle_hasher([input_])[0]
            hex_keccak = hex(keccak.value)[2:].rjust(64, "0")
            tx["input"] = tx["input"][:s_index] + tx["input"][s_index:].replace(tx["input"][i: 64 + i], hex_keccak)


def _setup():
    m = KeccakFunctionManager()
    key, other = BVS("key", 256), BVS("other", 256)
    h1, _ = m.create_keccak(Concat(key, BVV(0, 256)))
    h2, _ = m.create_keccak(Concat(other, BVV(1, 256)))
    h3, _ = m.create_keccak(BVS("word", 256))
    f512, inv512 = m.get_function(512)
    f256, inv256 = m.get_function(256)
    v1 = int("ab" + "fffffff" + "0" * 55, 16)     # model hash values carrying the matcher
    v2 = int("12" * 10 + "fffffff1" + "3" * 36, 16)
    v3 = int("fffffff" + "9" * 57, 16)
    pre1 = (0xDEADBEEF << 256) | 0
    pre2 = (0xAFFE << 256) | 1
    pre3 = 0x42
    values = {h1.raw: v1, h2.raw: v2, h3.raw: v3,
              inv512(BVV(v1, 256)).raw: pre1, inv512(BVV(v2, 256)).raw: pre2, inv256(BVV(v3, 256)).raw: pre3}
    model = DictModel(values)
    sel = "0xa9059cbb"
    txs = [{"input": sel + format(v1, "064x") + format(v2, "064x")},
           {"input": sel + "00" * 32 + format(v3, "064x") + format(v1, "064x")},
           {"input": sel + "11" * 64},                                  # no matcher: untouched
           {"input": sel + format(v3, "064x")[:60]}]                    # short window: untouched
    return m, model, txs


def test_replace_matches_reference_restatement():
    m, model, txs = _setup()
    want = [dict(t) for t in txs]
    reference_replace(want, model, m)
    calls = []

    def counting(datas):
        calls.append(len(datas))
        return oracle_hasher(datas)

    K.replace_with_actual_sha(txs, model, manager=m, hasher=counting)
    assert txs == want
    assert calls and calls[0] >= 3 and sum(calls[1:]) == 0   # one batch covers every window


def test_replace_keccak_values():
    m, model, txs = _setup()
    K.replace_with_actual_sha(txs, model, manager=m, hasher=oracle_hasher)
    k1 = keccak_ref.keccak256(((0xDEADBEEF << 256) | 0).to_bytes(64, "big")).hex()
    k3 = keccak_ref.keccak256((0x42).to_bytes(32, "big")).hex()
    assert txs[0]["input"].startswith("0xa9059cbb" + k1)
    assert txs[1]["input"] == "0xa9059cbb" + "00" * 32 + k3 + k1
    assert txs[2]["input"] == "0xa9059cbb" + "11" * 64


@pytest.mark.gpu
def test_replace_on_gpu(mgp_ctx):
    m, model, txs = _setup()
    want = [dict(t) for t in txs]
    reference_replace(want, model, m)
    K.replace_with_actual_sha(txs, model, manager=m)
    assert txs == want
