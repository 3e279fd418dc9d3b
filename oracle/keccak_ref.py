"""Keccak-256 in pure Python — TEST INFRASTRUCTURE.

Restates the published Keccak algorithm (Keccak-f[1600], FIPS 202 section 3
step mappings theta/rho/pi/chi/iota) with the ORIGINAL Keccak padding
(domain byte 0x01, rate 1088 bits) used by Ethereum — what the reference
obtains from pyethereum ``utils.sha3`` (keccak_function_manager.py:40-54) and
pysha3 ``keccak_256`` (support_utils.py:34-39), neither of which is installed
here.  ``hashlib.sha3_256`` is NIST SHA3 (0x06 padding) and is NOT this
function.  Pinned by the VMTests vmSha3Test KATs (tests/golden/keccak_kat.json)
and by the empty-input constant keccak_function_manager.py:71-78.
"""
from __future__ import annotations

RC = [
    0x0000000000000001, 0x0000000000008082, 0x800000000000808A, 0x8000000080008000,
    0x000000000000808B, 0x0000000080000001, 0x8000000080008081, 0x8000000000008009,
    0x000000000000008A, 0x0000000000000088, 0x0000000080008009, 0x000000008000000A,
    0x000000008000808B, 0x800000000000008B, 0x8000000000008089, 0x8000000000008003,
    0x8000000000008002, 0x8000000000000080, 0x000000000000800A, 0x800000008000000A,
    0x8000000080008081, 0x8000000000008080, 0x0000000080000001, 0x8000000080008008,
]
M64 = (1 << 64) - 1


def _rho_offsets():
    # FIPS 202 Algorithm 2: offsets along the (x, y) walk (1,0) -> (y, 2x+3y)
    r = [[0] * 5 for _ in range(5)]
    x, y = 1, 0
    for t in range(24):
        r[x][y] = ((t + 1) * (t + 2) // 2) % 64
        x, y = y, (2 * x + 3 * y) % 5
    return r


RHO = _rho_offsets()


def _rotl(v: int, n: int) -> int:
    n %= 64
    return ((v << n) | (v >> (64 - n))) & M64 if n else v


def keccak_f1600(A):
    """A[x][y] lanes (ints), modified in place."""
    for rnd in range(24):
        C = [A[x][0] ^ A[x][1] ^ A[x][2] ^ A[x][3] ^ A[x][4] for x in range(5)]
        D = [C[(x - 1) % 5] ^ _rotl(C[(x + 1) % 5], 1) for x in range(5)]
        for x in range(5):
            for y in range(5):
                A[x][y] ^= D[x]
        B = [[0] * 5 for _ in range(5)]
        for x in range(5):
            for y in range(5):
                B[y][(2 * x + 3 * y) % 5] = _rotl(A[x][y], RHO[x][y])
        for x in range(5):
            for y in range(5):
                A[x][y] = B[x][y] ^ ((~B[(x + 1) % 5][y]) & B[(x + 2) % 5][y])
        A[0][0] ^= RC[rnd]


def keccak256(data: bytes) -> bytes:
    rate = 136
    msg = bytearray(data)
    pad_len = rate - (len(msg) % rate)
    pad = bytearray(pad_len)
    pad[0] ^= 0x01
    pad[-1] ^= 0x80
    msg += pad
    A = [[0] * 5 for _ in range(5)]
    for off in range(0, len(msg), rate):
        block = msg[off:off + rate]
        for i in range(rate // 8):
            lane = int.from_bytes(block[8 * i:8 * i + 8], "little")
            A[i % 5][i // 5] ^= lane
        keccak_f1600(A)
    out = b"".join(A[i % 5][i // 5].to_bytes(8, "little") for i in range(4))
    return out


EMPTY_HASH = 89477152217924674838424037953991966239322087453347756267410168184682657981552  # keccak_function_manager.py:77
