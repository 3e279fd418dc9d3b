#!/usr/bin/env python3
"""Generator of mgp_keccak64_gfx950 — Keccak-256 of 64-byte preimages, hand-allocated VGPRs.

    python3 gen_keccak_asm.py <out.s>

Same contract as mgp_keccak64_kernel (mgp_kernels.hip): one preimage per lane, four
16-B loads, one absorb (pad byte 0x01 at offset 64, 0x80 at the end of the 136-B rate),
Keccak-f[1600] on 25 x 64-bit lanes held as u32 halves, two 16-B stores of the digest.

Why assembly: v_bitop3_b32 issues at 0.84-0.87 wave-instructions/ns per
SIMD with its three VGPR sources in distinct banks (register index mod 4) and at 0.56
with all three in one bank (profiles/bank_probe_r2.json); the compiler's allocation left
941 of the 1 638 bitop3 per hash with a shared-bank pair.  Here every value is a
virtual register first (SSA, program order), and a linear-scan allocator picks each
destination register by bank: the bank that the value's future bitop3 co-sources,
already placed, use least.  Registers are renamed freely (no moves): pi is pure
renaming, chi writes into registers its row no longer reads, rotations into any free
register.

Per round and half (lo / hi):
  theta  C[x] = A[x,0..4] xor-reduced: two bitop3 (0x96);  R[x] = rotl1(C[x+1]): two
         v_alignbit per x;  E = A ^ C[x-1] ^ R[x]: one bitop3 (0x96) per lane
  rho+pi B[pi(x,y)] = rotl(E, rho): two v_alignbit per lane (none for rho = 0)
  chi    A' = B ^ (~B[x+1] & B[x+2]): one bitop3 (0xd2; s0 = B, s1 = B[x+1], s2 = B[x+2])
  iota   A'[0] ^= RC: v_xor_b32 with a literal
No scalar memory writes (vector stores only).
"""
from __future__ import annotations

import os
import sys
from typing import Dict, List, Optional, Tuple

KNAME = "mgp_keccak64_gfx950"
RC = [0x0000000000000001, 0x0000000000008082, 0x800000000000808A, 0x8000000080008000,
      0x000000000000808B, 0x0000000080000001, 0x8000000080008081, 0x8000000000008009,
      0x000000000000008A, 0x0000000000000088, 0x0000000080008009, 0x000000008000000A,
      0x000000008000808B, 0x800000000000008B, 0x8000000000008089, 0x8000000000008003,
      0x8000000000008002, 0x8000000000000080, 0x000000000000800A, 0x800000008000000A,
      0x8000000080008081, 0x8000000000008080, 0x0000000080000001, 0x8000000080008008]
RHO = [0, 1, 62, 28, 27, 36, 44, 6, 55, 20, 3, 10, 43, 25, 39, 41, 45, 15, 21, 8, 18, 2, 61, 56, 14]
XOR3, CHI = 0x96, 0xD2
FIRST_FREE = 4   # v0 lane id, v1 hash index, v[2:3] preimage / digest address


class Prog:
    """Straight-line program on virtual registers (SSA): ops (kind, dst, srcs, imm)."""

    def __init__(self):
        self.ops: List[Tuple[str, int, Tuple[int, ...], object]] = []
        self.n = 0

    def new(self) -> int:
        self.n += 1
        return self.n - 1

    def emit(self, kind, srcs=(), imm=None) -> int:
        d = self.new()
        self.ops.append((kind, d, tuple(srcs), imm))
        return d


def build(p: Prog, state: List[List[int]], theta: str = "bitop3") -> List[List[int]]:
    """24 rounds on state[lane][half] (virtual registers); returns the final state.
    theta="bitop3": E = bitop3(A, C[x-1], R[x]) (one instruction per half-lane, but its
    three sources cannot always sit in distinct banks); theta="xor": D[x] = C[x-1] ^ R[x]
    once per column, E = A ^ D (two-source v_xor, bank-insensitive; 10 more instructions
    per round)."""
    A = state
    for rnd in range(24):
        C = [[0, 0] for _ in range(5)]
        for x in range(5):
            for h in range(2):
                t = p.emit("bitop3", (A[x][h], A[x + 5][h], A[x + 10][h]), XOR3)
                C[x][h] = p.emit("bitop3", (t, A[x + 15][h], A[x + 20][h]), XOR3)
        B: List[Optional[List[int]]] = [None] * 25
        for x in range(5):
            c1 = C[(x + 1) % 5]
            rl = p.emit("alignbit", (c1[0], c1[1]), 31)   # rotl64 by 1: lo' = lo<<1 | hi>>31
            rh = p.emit("alignbit", (c1[1], c1[0]), 31)   #               hi' = hi<<1 | lo>>31
            R = (rl, rh)
            if theta == "xor":
                D = [p.emit("xor", (C[(x + 4) % 5][h], R[h])) for h in range(2)]
            for y in range(5):
                i = x + 5 * y
                if theta == "xor":
                    e = [p.emit("xor", (A[i][h], D[h])) for h in range(2)]
                else:
                    e = [p.emit("bitop3", (A[i][h], C[(x + 4) % 5][h], R[h]), XOR3) for h in range(2)]
                r = RHO[i]
                if r == 0:
                    b = e
                elif r < 32:
                    b = [p.emit("alignbit", (e[0], e[1]), 32 - r), p.emit("alignbit", (e[1], e[0]), 32 - r)]
                else:
                    b = [p.emit("alignbit", (e[1], e[0]), 64 - r), p.emit("alignbit", (e[0], e[1]), 64 - r)]
                B[y + 5 * ((2 * x + 3 * y) % 5)] = b
        An: List[List[int]] = [[0, 0] for _ in range(25)]
        for y in range(5):
            for x in range(5):
                for h in range(2):
                    An[x + 5 * y][h] = p.emit("bitop3", (B[x + 5 * y][h], B[(x + 1) % 5 + 5 * y][h],
                                                         B[(x + 2) % 5 + 5 * y][h]), CHI)
        rc = RC[rnd]
        for h, k in ((0, rc & 0xFFFFFFFF), (1, rc >> 32)):
            if k:
                An[0][h] = p.emit("xorlit", (An[0][h],), k)
        A = An
    return A


def allocate(p: Prog, pinned: Dict[int, int], n_phys: int) -> Dict[int, int]:
    """Linear scan over the SSA program: each destination takes a free physical VGPR in
    the bank (index mod 4) its future bitop3 co-sources use least; a register is freed
    after the last use of its value.  `pinned`: virtual -> physical for the inputs."""
    last: Dict[int, int] = {}
    uses: Dict[int, List[int]] = {}
    for k, (_, _, srcs, _) in enumerate(p.ops):
        for s_ in srcs:
            last[s_] = k
            uses.setdefault(s_, []).append(k)
    phys: Dict[int, int] = dict(pinned)
    free = [r for r in range(FIRST_FREE, n_phys) if r not in set(pinned.values())]
    for k, (kind, d, srcs, _) in enumerate(p.ops):
        # a source whose last use is this op frees its register for the destination
        dying = [s_ for s_ in set(srcs) if last.get(s_) == k]
        for s_ in dying:
            free.append(phys[s_])
        cost = [0.0] * 4
        for u in uses.get(d, ()):
            kind_u, _, srcs_u, _ = p.ops[u]
            if kind_u != "bitop3":
                continue
            w = 1.0 / (1 + (u - k) / 64.0)  # nearer uses weigh more
            for co in srcs_u:
                if co != d and co in phys:
                    cost[phys[co] & 3] += w
        if not free:
            raise RuntimeError("keccak allocator: out of registers")
        nfree = [0] * 4
        for r in free:
            nfree[r & 3] += 1
        best = min((b for b in range(4) if nfree[b]), key=lambda b: (cost[b], -nfree[b], b))
        r = min(x for x in free if x & 3 == best)
        free.remove(r)
        phys[d] = r
    return phys


def conflicts(p: Prog, phys: Dict[int, int]) -> Tuple[int, int, int]:
    """(bitop3 total, with a shared-bank source pair, with all three sources in one bank)."""
    tot = pair = three = 0
    for kind, _, srcs, _ in p.ops:
        if kind != "bitop3":
            continue
        tot += 1
        banks = [phys[s_] & 3 for s_ in srcs]
        pair += len(set(banks)) < 3
        three += len(set(banks)) == 1
    return tot, pair, three


N_PHYS = int(os.environ.get("MGP_KECCAK_VGPRS", "72"))   # register budget: 72 -> 7 waves/SIMD


def generate(n_phys: int = N_PHYS, theta: str = "bitop3") -> Tuple[str, dict]:
    p = Prog()
    # inputs: lanes 0..7 from the four loads (v[4:19]), lane 8 lo = 0x01, lane 16 hi =
    # 0x80000000 (pad), every other half 0; constants materialised by v_mov
    state: List[List[int]] = [[0, 0] for _ in range(25)]
    pinned: Dict[int, int] = {}
    for lane in range(8):
        for h in range(2):
            vr = p.new()
            pinned[vr] = 4 + 2 * lane + h
            state[lane][h] = vr
    movs = []
    for lane in range(8, 25):
        for h in range(2):
            k = 0x01 if (lane, h) == (8, 0) else 0x80000000 if (lane, h) == (16, 1) else 0
            state[lane][h] = p.emit("mov", (), k)
            movs.append(state[lane][h])
    out = build(p, state, theta)
    phys = allocate(p, pinned, n_phys)
    used = max(phys.values()) + 1
    lines: List[str] = []
    for kind, d, srcs, imm in p.ops:
        r = [f"v{phys[s_]}" for s_ in srcs]
        if kind == "bitop3":
            lines.append(f"  v_bitop3_b32 v{phys[d]}, {r[0]}, {r[1]}, {r[2]} bitop3:{imm:#x}")
        elif kind == "alignbit":
            lines.append(f"  v_alignbit_b32 v{phys[d]}, {r[0]}, {r[1]}, {imm}")
        elif kind == "xor":
            lines.append(f"  v_xor_b32 v{phys[d]}, {r[0]}, {r[1]}")
        elif kind == "xorlit":
            lines.append(f"  v_xor_b32 v{phys[d]}, {imm:#x}, {r[0]}")
        elif kind == "mov":
            lines.append(f"  v_mov_b32 v{phys[d]}, {imm:#x}")
        else:
            raise ValueError(kind)
    # digest = lanes 0..3 -> v[4:11] by a parallel copy: at the end only those 8 values are
    # live, so any other register is a scratch for breaking a cycle (no registers past the
    # program's own: the VGPR count, hence the waves per SIMD, is the allocation's)
    dig = [phys[out[l][h]] for l in range(4) for h in range(2)]
    lines += parallel_copy({4 + j: r for j, r in enumerate(dig)}, scratch=next(
        r for r in range(FIRST_FREE, used + 9) if r not in dig and not 4 <= r < 12))
    stats = dict(zip(("bitop3", "shared_pair", "one_bank"), conflicts(p, phys)), vgprs=max(used, 12),
                 alignbit=sum(1 for o in p.ops if o[0] == "alignbit"), ops=len(p.ops))
    return "\n".join(lines), dict(stats, out_base=4)


def parallel_copy(moves: Dict[int, int], scratch: int) -> List[str]:
    """v_mov sequence for dst <- src (all at once): a move whose destination no pending move
    still reads goes first; a cycle is broken through `scratch`."""
    pend = {d: s_ for d, s_ in moves.items() if d != s_}
    out = []
    while pend:
        ready = [d for d in pend if d not in pend.values()]
        if ready:
            d = ready[0]
            out.append(f"  v_mov_b32 v{d}, v{pend.pop(d)}")
            continue
        d = next(iter(pend))          # every destination is still a source: a cycle
        out.append(f"  v_mov_b32 v{scratch}, v{d}")
        for k, v_ in pend.items():
            if v_ == d:
                pend[k] = scratch
    return out


PROLOGUE = """\
  s_load_dwordx2 s[4:5], s[0:1], 0x0
  s_load_dwordx2 s[6:7], s[0:1], 0x8
  s_load_dword s8, s[0:1], 0x10
  s_load_dwordx2 s[10:11], s[0:1], 0x18
  s_lshl_b32 s3, s2, 8
  v_add_u32 v1, s3, v0
  s_waitcnt lgkmcnt(0)
  v_cmp_gt_u32 vcc, s6, v1
  s_and_saveexec_b64 s[12:13], vcc
  s_cbranch_execz .Lkend
  s_lshl_b32 s9, s8, 4
  v_mov_b32 v2, s4
  v_mov_b32 v3, s5
  v_mad_u64_u32 v[2:3], s[14:15], v1, s9, v[2:3]
  global_load_dwordx4 v[4:7], v[2:3], off
  global_load_dwordx4 v[8:11], v[2:3], off offset:16
  global_load_dwordx4 v[12:15], v[2:3], off offset:32
  global_load_dwordx4 v[16:19], v[2:3], off offset:48
  s_mov_b32 s9, 32
  s_waitcnt vmcnt(0)
  v_mov_b32 v2, s10
  v_mov_b32 v3, s11
  v_mad_u64_u32 v[2:3], s[14:15], v1, s9, v[2:3]
"""


VARIANTS = ((KNAME, "bitop3"), (KNAME + "_dx", "xor"))  # default first; _dx: theta through D (A/B)


def _kernel(name: str, theta: str) -> Tuple[str, str, dict]:
    body, st = generate(theta=theta)
    ob = st["out_base"]
    nv = (st["vgprs"] + 7) // 8 * 8
    epi = (f"  global_store_dwordx4 v[2:3], v[{ob}:{ob + 3}], off\n"
           f"  global_store_dwordx4 v[2:3], v[{ob + 4}:{ob + 7}], off offset:16\n"
           f".Lkend_{name}:\n  s_endpgm\n")
    md = "\n".join([
        "  - .args:",
        "      - .name: preimages", "        .address_space: global", "        .offset: 0", "        .size: 8",
        "        .value_kind: global_buffer",
        "      - .name: count", "        .offset: 8", "        .size: 8", "        .value_kind: by_value",
        "      - .name: stride16", "        .offset: 16", "        .size: 4", "        .value_kind: by_value",
        "      - .name: digests", "        .address_space: global", "        .offset: 24", "        .size: 8",
        "        .value_kind: global_buffer",
        "    .group_segment_fixed_size: 0", "    .kernarg_segment_align: 8", "    .kernarg_segment_size: 32",
        "    .max_flat_workgroup_size: 256", f"    .name: {name}", "    .private_segment_fixed_size: 0",
        "    .sgpr_count: 24", f"    .symbol: {name}.kd", f"    .vgpr_count: {nv}", "    .wavefront_size: 64"])
    text = "\n".join([
        f".globl {name}", ".p2align 8", f".type {name},@function", f"{name}:",
        PROLOGUE.replace(".Lkend", f".Lkend_{name}") + body, epi + f".Lkfunc_end_{name}:",
        f".size {name}, .Lkfunc_end_{name}-{name}"])
    desc = "\n".join([
        ".p2align 6", f".amdhsa_kernel {name}",
        "  .amdhsa_group_segment_fixed_size 0", "  .amdhsa_private_segment_fixed_size 0",
        "  .amdhsa_kernarg_size 32", "  .amdhsa_user_sgpr_count 2", "  .amdhsa_user_sgpr_kernarg_segment_ptr 1",
        "  .amdhsa_system_sgpr_workgroup_id_x 1", "  .amdhsa_system_vgpr_workitem_id 0",
        f"  .amdhsa_next_free_vgpr {nv}", "  .amdhsa_next_free_sgpr 16", f"  .amdhsa_accum_offset {nv}",
        "  .amdhsa_reserve_vcc 1", ".end_amdhsa_kernel"])
    return text, desc + "\n" + "", dict(st, metadata=md)


def kernel_source() -> Tuple[str, dict]:
    """Every variant in one code object (one metadata note listing them all); stats of the
    default variant."""
    texts, descs, mds, stats = [], [], [], None
    for name, theta in VARIANTS:
        t, d, st = _kernel(name, theta)
        texts.append(t)
        descs.append(d)
        mds.append(st.pop("metadata"))
        stats = stats or st
    src = "\n".join(['.amdgcn_target "amdgcn-amd-amdhsa--gfx950"', ".text"] + texts +
                    ["", ".rodata"] + descs +
                    ["", ".amdgpu_metadata", "---", "amdhsa.kernels:"] + mds +
                    ["amdhsa.target: amdgcn-amd-amdhsa--gfx950", "amdhsa.version:", "  - 1", "  - 2", "...",
                     ".end_amdgpu_metadata"])
    return src + "\n", stats


def main():
    src, st = kernel_source()
    with open(sys.argv[1], "w") as f:
        f.write(f"// generated by gen_keccak_asm.py — do not edit\n// {st}\n{src}")
    if len(sys.argv) > 2 and sys.argv[2] == "-v":
        print(st)


if __name__ == "__main__":
    main()
