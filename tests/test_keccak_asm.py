"""The hand-allocated Keccak kernel (mythril_amd/csrc/gen_keccak_asm.py) on the CPU.

The generated straight-line body is executed by a tiny interpreter of its four
instruction forms (v_bitop3_b32, v_alignbit_b32, v_xor_b32 with a literal, v_mov_b32)
over 32-bit registers, from the register state the prologue leaves (preimage words in
v[4:19]), and the digest it gathers must equal FIPS 202 Keccak-256 (oracle/keccak_ref.py)
for random 64-byte preimages.  This checks the register allocator (no value overwritten
while live) and the round structure before the kernel ever runs on a GPU; the GPU tests
then check the kernel itself against the oracle.
"""
import os
import random
import re
import sys

import pytest

ROOT = os.path.join(os.path.dirname(__file__), "..")
sys.path.insert(0, os.path.join(ROOT, "mythril_amd", "csrc"))
import gen_keccak_asm as G  # noqa: E402

from oracle.keccak_ref import keccak256  # noqa: E402

M = 0xFFFFFFFF


def _bitop3(tt, a, b, c):
    r = 0
    for bit in range(32):
        idx = (((a >> bit) & 1) << 2) | (((b >> bit) & 1) << 1) | ((c >> bit) & 1)
        r |= ((tt >> idx) & 1) << bit
    return r


def _run(body, words):
    reg = {4 + i: w for i, w in enumerate(words)}
    rx = re.compile(r"\s*(\S+) v(\d+), (.*)")
    for line in body.split("\n"):
        m = rx.match(line)
        op, d, rest = m.group(1), int(m.group(2)), m.group(3)
        if op == "v_bitop3_b32":
            a, b, c, tt = re.match(r"v(\d+), v(\d+), v(\d+) bitop3:(0x[0-9a-f]+)", rest).groups()
            reg[d] = _bitop3(int(tt, 16), reg[int(a)], reg[int(b)], reg[int(c)])
        elif op == "v_alignbit_b32":
            a, b, s = re.match(r"v(\d+), v(\d+), (\d+)", rest).groups()
            reg[d] = (((reg[int(a)] << 32) | reg[int(b)]) >> int(s)) & M
        elif op == "v_xor_b32":
            k, a = re.match(r"(0x[0-9a-f]+), v(\d+)", rest).groups()
            reg[d] = int(k, 16) ^ reg[int(a)]
        elif op == "v_mov_b32":
            if rest.startswith("v"):
                reg[d] = reg[int(rest[1:])]
            else:
                reg[d] = int(rest, 16)
        else:
            raise AssertionError(op)
    return reg


def test_generated_body_computes_keccak256():
    body, st = G.generate()
    assert st["one_bank"] == 0
    rng = random.Random(11)
    for _ in range(3):
        pre = bytes(rng.getrandbits(8) for _ in range(64))
        words = [int.from_bytes(pre[4 * i:4 * i + 4], "little") for i in range(16)]
        reg = _run(body, words)
        ob = st["out_base"]
        dig = b"".join(reg[ob + j].to_bytes(4, "little") for j in range(8))
        assert dig == keccak256(pre)


def test_kernel_source_assembles_shape():
    src, st = G.kernel_source()
    bad = ["s_" + x for x in ("store", "buffer_store", "scratch_store", "dcache_wb", "dcache_discard", "atomic")]
    for line in src.split("\n"):
        op = line.strip().split(" ")[0]
        assert not any(op.startswith(b) for b in bad), line  # vector stores only
    assert st["vgprs"] <= 128
    # every bitop3 with three distinct-bank sources or at worst one shared pair
    assert st["shared_pair"] < st["bitop3"] // 3
