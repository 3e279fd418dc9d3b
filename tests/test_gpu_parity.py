"""GPU parity: the HIP path (through the C ABI of libmgp.so) vs the CPU oracle.

Integer work, so the bar is bit-exact: first-SAT index, witness words and
Keccak digests must equal the oracle's on the same seeded inputs.
"""
import numpy as np
import pytest

from mythril_amd import _native as N
from oracle import bvsem as S
from oracle import coracle
from oracle.keccak_ref import keccak256 as keccak_py

from ._util import cands_from_ints, load_golden, pack_states, random_cands, state_slice

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True, params=["asm", "hip"])
def engine(request):
    """Every parity test runs on both evaluation kernels: the hand-written gfx950
    interpreter (default engine) and the HIP C++ interpreter."""
    old = N.set_eval_engine()
    assert N.set_eval_engine(request.param) == request.param
    yield request.param
    N.set_eval_engine(old)


def _lower(nodes, noff, consts, coff, **kw):
    words, po, status = N.lower(nodes, noff, consts, coff, **kw)
    return words, po, status


# ------------------------------------------------------------ golden vectors
def test_vm_arith_golden_on_gpu(mgp_ctx):
    """Every SSTOREd value of the reference's straight-line VMTests, recomputed by the kernel."""
    cases = [t for t in load_golden("vm_arith.json") if t["reference_agrees"]]
    states = []
    for t in cases:
        consts = [int(c, 16) for c in t["consts"]]
        for node, exp in t["checks"]:
            nl = [list(n) for n in t["nodes"]]
            consts_x = consts + [int(exp, 16)]
            nl.append([S.CONST, 256, -1, -1, -1, len(consts_x) - 1, 0])
            nl.append([S.EQ, 1, node, len(nl) - 1, -1, 0, 0])
            states.append((nl, consts_x))
    nodes, noff, consts, coff = pack_states(states)
    words, po, status = _lower(nodes, noff, consts, coff)
    assert (status == 0).all()
    cands = np.zeros((len(states), 1, 1, 8), dtype=np.uint32)
    first, _ = mgp_ctx.eval_batch(words, po, cands)
    bad = [i for i in range(len(states)) if first[i] != 0]
    assert not bad, f"{len(bad)} VMTests values differ on GPU (first: {bad[:5]})"


def test_shift_vectors_on_gpu(mgp_ctx):
    vecs = load_golden("shift_vectors.json")
    opmap = {"shl": S.SHL, "shr": S.LSHR, "sar": S.ASHR}
    states = []
    for v in vecs:
        val, sh, ex = int(v["value"], 16), int(v["shift"], 16), int(v["expected"], 16)
        # value and shift come in as candidate variables (not constants) so the
        # kernel cannot fold anything
        nl = [[S.VAR, 256, -1, -1, -1, 0, 0], [S.VAR, 256, -1, -1, -1, 1, 0],
              [opmap[v["op"]], 256, 0, 1, -1, 0, 0], [S.CONST, 256, -1, -1, -1, 0, 0],
              [S.EQ, 1, 2, 3, -1, 0, 0]]
        states.append((nl, [ex], [val, sh]))
    nodes, noff, consts, coff = pack_states([(s[0], s[1]) for s in states])
    words, po, status = _lower(nodes, noff, consts, coff)
    cands = cands_from_ints([[s[2]] for s in states])
    first, wit = mgp_ctx.eval_batch(words, po, cands)
    assert (first == 0).all(), np.nonzero(first != 0)


# --------------------------------------------------------------- synthetic
@pytest.mark.parametrize("n_cand", [1, 37, 64, 256, 300])
def test_synthetic_vs_c_oracle(mgp_ctx, n_cand):
    n_states = 3000 if n_cand <= 256 else 800
    b = N.synth_generate(0x4D595448, 12345, n_states, 64, n_cand)
    words, po, status = _lower(b["nodes"], b["node_offsets"], b["consts"], b["const_offsets"])
    rng = np.random.default_rng(n_cand)
    cands = random_cands(rng, n_states, n_cand, b["n_vars"])
    for s in range(n_states):
        if b["planted"][s]:
            cands[s, b["plant_idx"][s]] = b["plant_words"][s]
    first, wit = mgp_ctx.eval_batch(words, po, cands)
    ref = coracle.first_sat(b["nodes"], b["node_offsets"], b["consts"], b["const_offsets"], cands)
    mism = np.nonzero(first != ref)[0]
    assert mism.size == 0, f"{mism.size} states differ, e.g. {mism[:5]} gpu={first[mism[:5]]} ref={ref[mism[:5]]}"
    sat = first >= 0
    assert sat.sum() >= b["planted"].sum()
    for s in np.nonzero(sat)[0][:200]:
        assert (wit[s] == cands[s, first[s]]).all()


def test_edge_values_all_ops(mgp_ctx):
    """Every BV op at widths 256/160/64/8/1 on boundary operands vs oracle.bvsem."""
    ops = [S.ADD, S.SUB, S.MUL, S.UDIV, S.UREM, S.SDIV, S.SREM, S.SMOD, S.AND, S.OR, S.XOR, S.SHL, S.LSHR,
           S.ASHR]
    cmps = [S.EQ, S.ULT, S.ULE, S.UGT, S.UGE, S.SLT, S.SLE, S.SGT, S.SGE, S.UADD_NOOVF, S.UMUL_NOOVF,
            S.USUB_NOUDF]
    widths = [256, 160, 64, 8, 1]
    rng = np.random.default_rng(7)
    states, cand_rows, expect = [], [], []
    for w in widths:
        m = (1 << w) - 1
        vals = sorted({v & m for v in (0, 1, 2, m, m - 1, 1 << (w - 1), (1 << (w - 1)) - 1, 3, (m >> 1) + 2)}
                      | {int(rng.integers(0, 2 ** 63)) & m for _ in range(3)})
        pairs = [(a, b) for a in vals for b in vals]
        for op in ops + cmps:
            for a, bb in pairs[:: max(1, len(pairs) // 24)]:
                is_cmp = op in cmps
                nl = [[S.VAR, w, -1, -1, -1, 0, 0], [S.VAR, w, -1, -1, -1, 1, 0],
                      [op, 1 if is_cmp else w, 0, 1, -1, 0, 0]]
                if is_cmp:
                    res = S.cmpop(op, a, bb, w)
                    nl.append([S.BNOT, 1, 2, -1, -1, 0, 0] if not res else [S.BAND, 1, 2, 2, -1, 0, 0])
                    consts = []
                else:
                    res = S.binop(op, a, bb, w)
                    nl.append([S.CONST, w, -1, -1, -1, 0, 0])
                    nl.append([S.EQ, 1, 2, 3, -1, 0, 0])
                    consts = [res]
                states.append((nl, consts))
                # high garbage bits above the var width must be ignored
                hi = (int(rng.integers(1, 2 ** 62)) << w) if w < 256 else 0
                cand_rows.append([[a | hi, bb]])
    nodes, noff, consts, coff = pack_states(states)
    words, po, status = _lower(nodes, noff, consts, coff)
    assert (status == 0).all()
    cands = cands_from_ints(cand_rows)
    first, _ = mgp_ctx.eval_batch(words, po, cands)
    bad = np.nonzero(first != 0)[0]
    assert bad.size == 0, f"{bad.size} op/edge cases wrong, first: {bad[:8]}"


def test_unsupported_and_empty(mgp_ctx):
    # a 512-bit division (not lowered for wide values) -> MGP_UNDECIDED,
    # other states unaffected
    nl_bad = [[S.VAR, 256, -1, -1, -1, 0, 0], [S.VAR, 256, -1, -1, -1, 1, 0], [S.CONCAT, 512, 0, 1, -1, 0, 0],
              [S.UDIV, 512, 2, 2, -1, 0, 0], [S.EQ, 1, 3, 3, -1, 0, 0]]
    nl_ok = [[S.VAR, 256, -1, -1, -1, 0, 0], [S.VAR, 256, -1, -1, -1, 1, 0], [S.ULT, 1, 0, 1, -1, 0, 0]]
    nl_true = [[S.TRUE, 1, -1, -1, -1, 0, 0]]
    nl_false = [[S.FALSE, 1, -1, -1, -1, 0, 0]]
    nodes, noff, consts, coff = pack_states([(nl_bad, []), (nl_ok, []), (nl_true, []), (nl_false, [])])
    words, po, status = _lower(nodes, noff, consts, coff)
    assert list(status) == [1, 0, 0, 0]
    cands = cands_from_ints([[[5, 3], [3, 5]]] * 4)
    first, _ = mgp_ctx.eval_batch(words, po, cands)
    assert list(first) == [N.MGP_UNDECIDED, 1, 0, N.MGP_NO_SAT]
    # zero states is a no-op
    f0, _ = mgp_ctx.eval_batch(np.zeros(0, np.uint32), np.zeros(1, np.uint64), np.zeros((0, 1, 1, 8), np.uint32))
    assert f0.size == 0


def test_wide_values_parity(mgp_ctx):
    """512/516-bit values (include/mgp_ir.h "wide values") and keccak256_512 mapping
    preimages with the inverse: first-SAT per candidate row vs the oracle."""
    from .test_lowering import wide_mapping_case, wide_struct_case
    nl_s, c_s, rows_s = wide_struct_case()
    nl_m, nl_c, c_m, rows_m = wide_mapping_case()
    states = [(nl_s, c_s), (nl_m, c_m), (nl_c, c_m)]
    nodes, noff, consts, coff = pack_states(states)
    words, po, status = _lower(nodes, noff, consts, coff)
    assert (status == 0).all()
    n_vars = max(len(r) for r in rows_s + rows_m)
    want = []
    for s, (nl, cl) in enumerate(states):
        rows = rows_s if s == 0 else rows_m
        # one candidate per launch row: evaluate each row alone (first_sat 0 or -1)
        for r in rows:
            want.append(0 if S.eval_root(nl, cl, r) else -1)
    batch = [states[0]] * len(rows_s) + [states[1]] * len(rows_m) + [states[2]] * len(rows_m)
    nodes, noff, consts, coff = pack_states(batch)
    words, po, status = _lower(nodes, noff, consts, coff)
    cand_rows = [[list(r) + [0] * (n_vars - len(r))] for r in rows_s + rows_m + rows_m]
    first, _ = mgp_ctx.eval_batch(words, po, cands_from_ints(cand_rows))
    assert list(first) == want
    assert 0 in want and -1 in want


def test_wide_zext_division_shift_signed_parity(mgp_ctx):
    """257..776-bit zero-extended UDIV / UREM / LSHR / ASHR and signed compares (round 6;
    CREATE2's salt-padded 776-bit preimage shape, instructions.py:1707-1721): first-SAT over
    each state's candidate rows vs oracle.bvsem, x / 0 included."""
    from .test_lowering import wide_zext_cases
    states, rows = wide_zext_cases()
    nodes, noff, consts, coff = pack_states(states)
    words, po, status = _lower(nodes, noff, consts, coff)
    assert (status == 0).all()
    for rr in (rows, [r[:8] for r in rows]):   # every row; the random rows alone
        first, _ = mgp_ctx.eval_batch(words, po, cands_from_ints(rr))
        want = [S.first_sat(nl, cl, r) for (nl, cl), r in zip(states, rr)]
        assert list(first) == want
        assert any(x > 0 for x in want)
    assert any(x < 0 for x in want)


def test_wide_arith_parity(mgp_ctx):
    """257..776-bit ADD / SUB carry chains, bitwise ops and unsigned compares: first-SAT
    over each state's candidate rows vs the oracle."""
    from .test_lowering import wide_arith_cases
    states, rows = wide_arith_cases()
    nodes, noff, consts, coff = pack_states(states)
    words, po, status = _lower(nodes, noff, consts, coff)
    assert (status == 0).all()
    first, _ = mgp_ctx.eval_batch(words, po, cands_from_ints(rows))
    want = [S.first_sat(nl, cl, r) for (nl, cl), r in zip(states, rows)]
    assert list(first) == want
    assert any(x >= 0 for x in want) and any(x < 0 for x in want)


def test_uf_ackermann_semantics(mgp_ctx):
    """keccak UF pairs: f(a)==f(b) forces equal values only when a==b, inverse round trip."""
    # nodes: x0, x1, f(x0)[fresh 2], f(x1)[fresh 3], inv(f(x0))[fresh 4]
    nl = [[S.VAR, 256, -1, -1, -1, 0, 0], [S.VAR, 256, -1, -1, -1, 1, 0],
          [S.UFAPP, 256, 0, -1, -1, 0, 2], [S.UFAPP, 256, 1, -1, -1, 0, 3],
          [S.UFINV, 256, 2, -1, -1, 0, 4],
          [S.EQ, 1, 2, 3, -1, 0, 0],          # f(x0) == f(x1)
          [S.EQ, 1, 4, 0, -1, 0, 0],          # inv(f(x0)) == x0
          [S.BAND, 1, 5, 6, -1, 0, 0]]
    rows = [[[7, 7, 11, 13, 99], [7, 8, 11, 13, 99], [7, 8, 11, 11, 99], [7, 8, 12, 12, 7]]]
    nodes, noff, consts, coff = pack_states([(nl, [])])
    words, po, status = _lower(nodes, noff, consts, coff)
    cands = cands_from_ints(rows)
    first, _ = mgp_ctx.eval_batch(words, po, cands)
    ref = S.first_sat(nl, [], rows[0])
    assert first[0] == ref == 0


# ------------------------------------------------------------------ Keccak
def test_keccak_kats_on_gpu(mgp_ctx):
    for k in load_golden("keccak_kat.json"):
        if k["digest"] is None:  # vmSha3Test *oog: no expected digest (listed with the reason)
            continue
        pre = bytes.fromhex(k["preimage"])
        out = mgp_ctx.keccak256_n(np.frombuffer(pre, dtype=np.uint8), 1, len(pre), max(len(pre), 1))
        assert out[0].tobytes().hex() == k["digest"], k["source"]


@pytest.mark.parametrize("length", [0, 1, 31, 32, 55, 64, 100, 135, 136, 137, 200, 272, 300])
def test_keccak_lengths_vs_oracle(mgp_ctx, length):
    rng = np.random.default_rng(length)
    n = 777
    stride = length + 3
    data = rng.integers(0, 256, size=n * stride + 8, dtype=np.uint8)
    out = mgp_ctx.keccak256_n(data, n, length, stride)
    ref = coracle.keccak256(data, n, length, stride)
    assert (out == ref).all()
    assert out[5].tobytes() == keccak_py(data[5 * stride:5 * stride + length].tobytes())


@pytest.fixture(params=["asm", "asm_dx", "hip"])
def keccak_engine(request):
    old = N.set_keccak_engine()
    N.set_keccak_engine(request.param)
    yield request.param
    N.set_keccak_engine(old)


@pytest.mark.parametrize("n", [1, 63, 255, 257, 1000, 4099])
def test_keccak64_engines_ragged_counts(mgp_ctx, keccak_engine, n):
    """The 64-byte fast path on both kernels (hand-allocated mgp_keccak64_gfx950 and the
    compiler-allocated mgp_keccak64_kernel): counts that leave a partial workgroup, and a
    stride past the preimage (80 B: 16-B aligned, 16 B of padding per record)."""
    rng = np.random.default_rng(n)
    for stride in (64, 80):
        data = rng.integers(0, 256, size=n * stride, dtype=np.uint8)
        out = mgp_ctx.keccak256_n(data, n, 64, stride)
        ref = coracle.keccak256(data, n, 64, stride)
        assert (out == ref).all(), (keccak_engine, n, stride)


def test_keccak_mapping_slot_fast_path_vs_oracle(mgp_ctx, keccak_engine):
    """Config 5: the bench's own preimages -- pad32(addr_i) || pad32(i mod 8)
    from mgp_fill_mapping_preimages_dev -- hashed on the 64-byte fast path (stride 64,
    16-B aligned device buffers: mgp_keccak64_kernel), 65 536 digests bit-exact against the
    C oracle, plus a far-away slice at index 2^30 - 4096 (the bench's last chunk)."""
    import ctypes

    import torch

    seed = 0x4D595448
    dev = torch.device("cuda", 0)
    stream = torch.cuda.current_stream(dev)
    sh = ctypes.c_void_p(stream.cuda_stream)
    for first, n in ((0, 1 << 16), ((1 << 30) - 4096, 4096)):
        d_pre = torch.empty(n * 64, dtype=torch.uint8, device=dev)
        d_dig = torch.empty(n * 32, dtype=torch.uint8, device=dev)
        assert d_pre.data_ptr() % 16 == 0 and d_dig.data_ptr() % 16 == 0
        N.fill_mapping_preimages_dev(ctypes.c_void_p(d_pre.data_ptr()), first, n, seed, sh)
        N.keccak256_dev(ctypes.c_void_p(d_pre.data_ptr()), n, 64, 64, ctypes.c_void_p(d_dig.data_ptr()), sh)
        torch.cuda.synchronize(dev)
        pre = coracle.mapping_preimages(first, n, seed)
        assert np.array_equal(d_pre.cpu().numpy().reshape(n, 64), pre.reshape(n, 64)), "preimage fill differs"
        ref = coracle.keccak256(pre.reshape(-1), n, 64, 64)
        got = d_dig.cpu().numpy().reshape(n, 32)
        bad = np.nonzero((got != ref).any(axis=1))[0]
        assert bad.size == 0, f"{bad.size} of {n} digests differ from the oracle (first index {first + bad[0]})"
    # the host entry point on the same preimages takes the same fast path
    out = mgp_ctx.keccak256_n(pre.reshape(-1), n, 64, 64)
    assert np.array_equal(out, ref)


def _long_program(rng, n_ops, n_vars, n_consts):
    """A random chain DAG of n_ops BV ops over n_vars variables and n_consts constants."""
    nl = [[S.VAR, 256, -1, -1, -1, v, 0] for v in range(n_vars)]
    consts = [int(rng.integers(1, 2 ** 62)) << int(rng.integers(0, 190)) for _ in range(n_consts)]
    nl += [[S.CONST, 256, -1, -1, -1, c, 0] for c in range(n_consts)]
    leaves = list(range(len(nl)))
    ops = [S.ADD, S.SUB, S.XOR, S.MUL, S.AND, S.OR, S.LSHR, S.UREM]
    t = 0
    live = []
    for i in range(n_ops):
        op = ops[int(rng.integers(0, len(ops)))]
        b = leaves[int(rng.integers(0, len(leaves)))] if (i % 3 or not live) else live[int(rng.integers(0, len(live)))]
        nl.append([op, 256, t, b, -1, 0, 0])
        t = len(nl) - 1
        if i % 7 == 0:
            live.append(t)
    # root: OR of (t == var0) and an ULT over a kept intermediate, so a random candidate is SAT ~50%
    nl.append([S.EQ, 1, t, 0, -1, 0, 0])
    nl.append([S.ULT, 1, live[-1], t, -1, 0, 0])
    nl.append([S.BOR, 1, len(nl) - 2, len(nl) - 1, -1, 0, 0])
    return nl, consts


@pytest.mark.parametrize("n_ops,n_vars,n_consts", [(150, 3, 4), (300, 9, 40), (70, 7, 70)])
def test_long_programs_many_vars_and_constants(mgp_ctx, n_ops, n_vars, n_consts):
    """Programs past one 64-uop page, variables beyond the 6 register-resident ones (HBM
    operands) and constant pools up to and past the 64-entry limit (past it: undecided)."""
    rng = np.random.default_rng(n_ops + n_vars)
    states = [_long_program(rng, n_ops, n_vars, n_consts) for _ in range(12)]
    nodes, noff, consts, coff = pack_states(states)
    words, po, status = _lower(nodes, noff, consts, coff)
    cands = random_cands(rng, len(states), 64, n_vars, interesting_frac=0.1)
    first, _ = mgp_ctx.eval_batch(words, po, cands)
    want = coracle.first_sat(nodes, noff, consts, coff, cands)
    ok = status == 0
    assert np.array_equal(first[ok], want[ok])
    assert (first[~ok] == N.MGP_UNDECIDED).all()
    if n_consts <= 60:
        assert ok.all()


def _magnitude_values(rng, n, w):
    """Operands of every bit length class (plus 0, 1, all-ones, powers of two), as w-bit ints."""
    m = (1 << w) - 1
    out = []
    for _ in range(n):
        r = rng.random()
        if r < 0.1:
            out.append(int(rng.choice([0, 1, 2, m, m - 1, 1 << (w - 1), (1 << (w - 1)) - 1])) & m)
        else:
            bits = int(rng.integers(1, w + 1))
            v = 0
            for k in range(0, bits, 62):
                v = (v << 62) | int(rng.integers(0, 2 ** 62))
            out.append((v >> max(0, (((bits + 61) // 62) * 62) - bits)) & m | (1 << (bits - 1)))
    return out


@pytest.mark.parametrize("w", [256, 160, 64])
def test_division_all_variants_every_candidate(mgp_ctx, w):
    """UDIV/UREM/SDIV/SREM/SMOD on operands of all magnitudes (1-limb divisors force all
    eight Knuth digits): root = (op(x0, x1) != x2) with x2 the expected value, so a correct
    kernel leaves every state without a satisfying candidate."""
    rng = np.random.default_rng(w)
    ops = [S.UDIV, S.UREM, S.SDIV, S.SREM, S.SMOD]
    n_cand, per_op = 256, 3
    states, rows = [], []
    for op in ops:
        for _ in range(per_op):
            a = _magnitude_values(rng, n_cand, w)
            b = _magnitude_values(rng, n_cand, w)
            exp = [S.binop(op, x, y, w) for x, y in zip(a, b)]
            nl = [[S.VAR, w, -1, -1, -1, 0, 0], [S.VAR, w, -1, -1, -1, 1, 0], [S.VAR, w, -1, -1, -1, 2, 0],
                  [op, w, 0, 1, -1, 0, 0], [S.EQ, 1, 3, 2, -1, 0, 0], [S.BNOT, 1, 4, -1, -1, 0, 0]]
            states.append((nl, []))
            rows.append([[x, y, e] for x, y, e in zip(a, b, exp)])
    nodes, noff, consts, coff = pack_states(states)
    words, po, status = _lower(nodes, noff, consts, coff)
    assert (status == 0).all()
    first, _ = mgp_ctx.eval_batch(words, po, cands_from_ints(rows))
    bad = np.nonzero(first != N.MGP_NO_SAT)[0]
    if bad.size:
        s0 = int(bad[0])
        a, b, e = rows[s0][int(first[s0])]
        pytest.fail(f"{bad.size} states with a wrong quotient/remainder; first: op {ops[s0 // per_op]} "
                    f"a={a:#x} b={b:#x} expected {e:#x}")


def _single_digit_pairs(rng, n, w, signed):
    """(a, b) with top limb(a) = top limb(b) on every dividing lane (quotient < 2^32: the
    interpreter's single-digit path), the top limb varying per lane, quotients at the
    extremes (0, 1, 2^32 - 1, exact multiples and one below), a few b = 0 / a < b lanes."""
    limbs = w // 32 - (1 if signed else 0)
    m = (1 << w) - 1
    out = []
    for j in range(n):
        t = int(rng.integers(0, max(1, limbs)))
        kind = j % 8
        if kind == 7:
            out.append((int(rng.integers(0, 2 ** 31)) << (32 * t), 0))
            continue
        q = [0, 1, 2 ** 32 - 1, int(rng.integers(0, 2 ** 32)), int(rng.integers(0, 2 ** 16)),
             2 ** 32 - 2, int(rng.integers(2 ** 31, 2 ** 32))][kind]
        top = int(rng.integers(1, max(2, (2 ** 32 - 1) // (q + 1) + 1)))
        low = int.from_bytes(rng.integers(0, 256, size=32, dtype=np.uint8).tobytes(), "little")
        big = int.from_bytes(rng.integers(0, 256, size=40, dtype=np.uint8).tobytes(), "little")
        a = b = 0
        for lowmask in ((1 << (32 * t)) - 1, 0):     # lower limbs of b random, else zero
            b = (top << (32 * t)) | (low & lowmask)
            r = [0, b - 1, big % b, 0][j % 4]
            a = q * b + r
            if not (a >> (32 * (t + 1)) or (signed and a >> (w - 1))):
                break
        else:
            a = b
        if signed:
            if rng.integers(0, 2):
                a = (-a) & m
            if rng.integers(0, 2):
                b = (-b) & m
        out.append((a, b))
    return out


@pytest.mark.parametrize("w", [256, 64])
def test_division_single_digit_waves(mgp_ctx, w):
    """Waves whose dividing lanes all have one quotient digit take the interpreter's
    double-precision single-digit path (gen_eval_asm.single_digit): every variant, every
    candidate, root = (op(x0, x1) != x2) as in the test above."""
    rng = np.random.default_rng(31 + w)
    ops = [S.UDIV, S.UREM, S.SDIV, S.SREM, S.SMOD]
    n_cand, per_op = 256, 3
    states, rows = [], []
    for op in ops:
        for _ in range(per_op):
            pairs = _single_digit_pairs(rng, n_cand, w, op in (S.SDIV, S.SREM, S.SMOD))
            exp = [S.binop(op, x, y, w) for x, y in pairs]
            nl = [[S.VAR, w, -1, -1, -1, 0, 0], [S.VAR, w, -1, -1, -1, 1, 0], [S.VAR, w, -1, -1, -1, 2, 0],
                  [op, w, 0, 1, -1, 0, 0], [S.EQ, 1, 3, 2, -1, 0, 0], [S.BNOT, 1, 4, -1, -1, 0, 0]]
            states.append((nl, []))
            rows.append([[x, y, e] for (x, y), e in zip(pairs, exp)])
    nodes, noff, consts, coff = pack_states(states)
    words, po, status = _lower(nodes, noff, consts, coff)
    assert (status == 0).all()
    first, _ = mgp_ctx.eval_batch(words, po, cands_from_ints(rows))
    bad = np.nonzero(first != N.MGP_NO_SAT)[0]
    if bad.size:
        s0 = int(bad[0])
        a, b, e = rows[s0][int(first[s0])]
        pytest.fail(f"{bad.size} states with a wrong quotient/remainder; first: op {ops[s0 // per_op]} "
                    f"a={a:#x} b={b:#x} expected {e:#x}")


def _q32_pairs(rng, n, w, signed):
    """(a, b) with q = a // b < 2^32 but top limb(a) = top limb(b) + 1 (the single-digit
    path's (a >> 32) < b test admits them; the top-limb test did not), quotients at the
    extremes, remainders 0 / b - 1 / random, a few b = 0 and a < b lanes."""
    limbs = w // 32 - (1 if signed else 0)
    m = (1 << w) - 1
    out = []
    for j in range(n):
        kind = j % 8
        t = int(rng.integers(0, max(1, limbs - 1)))      # top limb of b; a's is t + 1
        if kind == 7:
            out.append((int(rng.integers(0, 2 ** 31)) << (32 * t), 0 if j % 16 == 7 else m >> 1))
            continue
        top_b = int(rng.integers(1, 2 ** 32))
        low = int.from_bytes(rng.integers(0, 256, size=32, dtype=np.uint8).tobytes(), "little")
        b = (top_b << (32 * t)) | (low & ((1 << (32 * t)) - 1))
        qmin = -(-(1 << (32 * (t + 1))) // b)          # smallest q with q * b >= 2^(32(t+1))
        q = [qmin, 2 ** 32 - 1, int(rng.integers(qmin, 2 ** 32)), 2 ** 32 - 2, qmin + 1,
             int(rng.integers(qmin, 2 ** 32)), int(rng.integers(2 ** 31, 2 ** 32))][kind]
        q = min(max(q, qmin), 2 ** 32 - 1)
        r = [0, b - 1, int(rng.integers(0, 2 ** 62)) % b, 0][j % 4]
        a = q * b + r
        if a >> (w - (1 if signed else 0)):
            a, b = b, b                                 # out of range for this width: q = 1
        if signed:
            if rng.integers(0, 2):
                a = (-a) & m
            if rng.integers(0, 2):
                b = (-b) & m
        out.append((a, b))
    return out


@pytest.mark.parametrize("w", [256, 96])
def test_division_q32_waves(mgp_ctx, w):
    """Waves whose dividing lanes have one quotient digit but different top limbs take the
    single-digit path too: every variant, every candidate, root = (op(x0, x1) != x2)."""
    rng = np.random.default_rng(57 + w)
    ops = [S.UDIV, S.UREM, S.SDIV, S.SREM, S.SMOD]
    n_cand, per_op = 256, 3
    states, rows = [], []
    for op in ops:
        for _ in range(per_op):
            pairs = _q32_pairs(rng, n_cand, w, op in (S.SDIV, S.SREM, S.SMOD))
            exp = [S.binop(op, x, y, w) for x, y in pairs]
            nl = [[S.VAR, w, -1, -1, -1, 0, 0], [S.VAR, w, -1, -1, -1, 1, 0], [S.VAR, w, -1, -1, -1, 2, 0],
                  [op, w, 0, 1, -1, 0, 0], [S.EQ, 1, 3, 2, -1, 0, 0], [S.BNOT, 1, 4, -1, -1, 0, 0]]
            states.append((nl, []))
            rows.append([[x, y, e] for (x, y), e in zip(pairs, exp)])
    nodes, noff, consts, coff = pack_states(states)
    words, po, status = _lower(nodes, noff, consts, coff)
    assert (status == 0).all()
    first, _ = mgp_ctx.eval_batch(words, po, cands_from_ints(rows))
    bad = np.nonzero(first != N.MGP_NO_SAT)[0]
    if bad.size:
        s0 = int(bad[0])
        a, b, e = rows[s0][int(first[s0])]
        pytest.fail(f"{bad.size} states with a wrong quotient/remainder; first: op {ops[s0 // per_op]} "
                    f"a={a:#x} b={b:#x} expected {e:#x}")


def _bool_fold_states(rng, n):
    """DAGs whose compares feed the next BAND / BOR and whose BNOTs feed the next BAND
    (the translator's BCOMB / BANDN folds), inverted compares (UGE / ULE / SGE) among
    them, over three 8-bit variables so random candidates hit both outcomes."""
    w = 8
    cmps = [S.EQ, S.ULT, S.UGE, S.ULE, S.SLT, S.SGE, S.UGT]
    out = []
    for _ in range(n):
        nl = [[S.VAR, w, -1, -1, -1, k, 0] for k in range(3)]
        cl = [int(x) for x in rng.integers(0, 256, size=4)]
        nl += [[S.CONST, w, -1, -1, -1, k, 0] for k in range(4)]
        bools = []
        for _ in range(int(rng.integers(3, 9))):
            a, b = int(rng.integers(0, 7)), int(rng.integers(0, 7))
            nl.append([cmps[int(rng.integers(len(cmps)))], 1, a, b, -1, 0, 0])
            c = len(nl) - 1
            if bools and rng.random() < 0.7:
                if rng.random() < 0.3:
                    nl.append([S.BNOT, 1, bools[-1], -1, -1, 0, 0])
                    nl.append([S.BAND, 1, c, len(nl) - 1, -1, 0, 0])
                else:
                    nl.append([S.BAND if rng.random() < 0.6 else S.BOR, 1, c, bools[-1], -1, 0, 0])
                bools.append(len(nl) - 1)
            else:
                bools.append(c)
        root = bools[-1]
        for b in bools[:-1][-2:]:
            nl.append([S.BOR, 1, root, b, -1, 0, 0])
            root = len(nl) - 1
        out.append((nl, cl))
    return out


def _band4n_states(rng, n, late_vars: int = 0):
    """DAGs whose BNOTs (not next to their reader) feed AND chains of 2-4 operands (the
    translator's BAND4N fold), some BNOT results read again later by a BOR or an ITE (no
    fold allowed there), over three 8-bit variables.  With `late_vars` > 0 the states get
    that many more variables (indices 3.., past the register bank from index 6 on), and
    compares that read them are ANDed onto the root after the chains, so HBM variable
    loads follow a folded chain (the uop reference once lost its candidate row
    there)."""
    w = 8
    cmps = [S.EQ, S.ULT, S.UGE, S.ULE, S.SLT, S.SGE, S.UGT]
    out = []
    for _ in range(n):
        nl = [[S.VAR, w, -1, -1, -1, k, 0] for k in range(3)]
        cl = [int(x) for x in rng.integers(0, 256, size=4)]
        nl += [[S.CONST, w, -1, -1, -1, k, 0] for k in range(4)]
        pool = []
        for _ in range(int(rng.integers(4, 9))):
            a, b = int(rng.integers(0, 7)), int(rng.integers(0, 7))
            nl.append([cmps[int(rng.integers(len(cmps)))], 1, a, b, -1, 0, 0])
            pool.append(len(nl) - 1)
            if rng.random() < 0.5:
                nl.append([S.BNOT, 1, len(nl) - 1 if rng.random() < 0.3 else int(rng.choice(pool)), -1, -1, 0, 0])
                pool.append(len(nl) - 1)
        chains = []
        for _ in range(int(rng.integers(1, 4))):
            ops = [int(x) for x in rng.choice(pool, size=int(rng.integers(2, 5)))]
            acc = ops[0]
            for o in ops[1:]:
                nl.append([S.BAND, 1, acc, o, -1, 0, 0])
                acc = len(nl) - 1
            chains.append(acc)
        root = chains[0]
        for c in chains[1:]:
            nl.append([S.BOR, 1, root, c, -1, 0, 0])
            root = len(nl) - 1
        if rng.random() < 0.3:       # a BNOT result read again after its chain
            nl.append([S.BOR, 1, root, int(rng.choice(pool)), -1, 0, 0])
            root = len(nl) - 1
        if rng.random() < 0.2:       # ... or as an ITE condition
            nl.append([S.ITE, w, int(rng.choice(pool)), 0, 1, 0, 0])
            nl.append([S.ULT, 1, len(nl) - 1, 2, -1, 0, 0])
            nl.append([S.BOR, 1, root, len(nl) - 1, -1, 0, 0])
            root = len(nl) - 1
        for k in range(late_vars):   # compares on HBM variables, read after the chains
            nl.append([S.VAR, w, -1, -1, -1, 3 + k, 0])
            nl.append([cmps[int(rng.integers(len(cmps)))], 1, len(nl) - 1, 3 + int(rng.integers(4)), -1, 0, 0])
            nl.append([S.BAND, 1, root, len(nl) - 1, -1, 0, 0])
            root = len(nl) - 1
        out.append((nl, cl))
    return out


def _select_chain_states(rng, n):
    """Select chains as LASER's arrays lower (a Select over a Store chain, calldata.py /
    array.py: `EQ q k_i` + `ITE(that, z_i, acc)` pairs): per state two or three chains over
    one set of keys, each chain comparing its q (a bank variable, a computed slot or a
    constant) against keys that are small constants (repeated, some with high limbs set)
    or computed slots (x + i, shared by the chains, and x & 3, which several lanes match
    at once) or HBM variables (TSELS keys read from the candidate row), selecting HBM
    variables, the bank variable 5 or a computed byte.  Root:
    some chain == T.  The translator's EQSEL, TSEL and TSELS fusions all fire on these
    (tests/test_lowering.py counts them)."""
    out = []
    for _ in range(n):
        m = int(rng.integers(8, 40))
        nl = [[S.VAR, 256, -1, -1, -1, k, 0] for k in range(5)]     # 0-4
        nl.append([S.VAR, 256, -1, -1, -1, 5, 0])                    # 5: base / bank value
        cl = []

        def add(row):
            nl.append(row)
            return len(nl) - 1

        def const(val):
            cl.append(val)
            return add([S.CONST, 256, -1, -1, -1, len(cl) - 1, 0])

        zs = [add([S.VAR, 256, -1, -1, -1, 6 + i, 0]) for i in range(m)]
        t = add([S.VAR, 256, -1, -1, -1, 6 + m, 0])
        byte = add([S.AND, 256, 2, const(0xFF), -1, 0, 0])
        slot_keys = [add([S.ADD, 256, 1, const(i), -1, 0, 0]) for i in range(int(rng.integers(4, 20)))]
        slot_keys += [add([S.AND, 256, 2 + int(rng.integers(3)), const(3), -1, 0, 0]) for _ in range(3)]
        # keys that are HBM variables (index >= 6: TSELS candidate-row keys, as spilled slots are)
        var_keys = [add([S.VAR, 256, -1, -1, -1, 7 + m + i, 0]) for i in range(4)]
        masked = add([S.AND, 256, 0, const(0x3F), -1, 0, 0])
        eqs = []
        for _c in range(int(rng.integers(2, 4))):
            qk = int(rng.integers(3))
            q = 0 if qk == 0 else masked if qk == 1 else const(int(rng.integers(0, 24)))
            acc = 5
            for i in range(int(rng.integers(3, m + 1))):
                r = rng.random()
                if qk == 2 or r < 0.3:
                    key = slot_keys[int(rng.integers(len(slot_keys)))] if rng.random() < 0.7 else \
                        var_keys[int(rng.integers(len(var_keys)))]
                elif r < 0.85:
                    key = const(int(rng.integers(0, 48)))
                else:
                    key = const((int(rng.integers(1, 4)) << int(rng.choice([32, 100, 255]))) + int(rng.integers(0, 48)))
                r = rng.random()
                z = zs[i % m] if r < 0.85 else 5 if r < 0.92 else byte
                c = add([S.EQ, 1, q, key, -1, 0, 0] if rng.random() < 0.5 else [S.EQ, 1, key, q, -1, 0, 0])
                acc = add([S.ITE, 256, c, z, acc, 0, 0])
            eqs.append(add([S.EQ, 1, acc, t, -1, 0, 0]))
        root = eqs[0]
        for e in eqs[1:]:
            root = add([S.BOR, 1, root, e, -1, 0, 0])
        out.append((nl, cl))
    return out


def _select_chain_cands(rng, states, n_cand):
    """Candidates for _select_chain_states: variables 0-4 small (keys and q collide), a
    tenth with high limbs set over a small low limb (TSEL must compare all 256 bits), the
    selected values and T in 0..3 (the root holds often)."""
    n_vars = max(max(r[5] for r in nl if r[0] == S.VAR) + 1 for nl, _ in states)
    cands = np.zeros((len(states), n_cand, n_vars, 8), np.uint32)
    cands[:, :, :, 0] = rng.integers(0, 4, size=(len(states), n_cand, n_vars))
    cands[:, :, :5, 0] = rng.integers(0, 48, size=(len(states), n_cand, 5))
    hi = rng.random((len(states), n_cand, 5)) < 0.1
    cands[:, :, :5, int(rng.integers(1, 8))] = np.where(hi, 1, 0)
    return cands


def test_select_chain_fusions_vs_oracle(mgp_ctx):
    """EQSEL / TSEL / TSELS (the select-chain uops of the gfx950 translation) against the C
    oracle on every candidate (both engines; the HIP engine runs the v1 ITE chains)."""
    rng = np.random.default_rng(515)
    states = _select_chain_states(rng, 300)
    nodes, noff, consts, coff = pack_states(states)
    words, po, status = _lower(nodes, noff, consts, coff)
    assert (status == 0).all()
    cands = _select_chain_cands(rng, states, 256)
    first, _ = mgp_ctx.eval_batch(words, po, cands)
    ref = coracle.first_sat(nodes, noff, consts, coff, cands)
    bad = np.nonzero(first != ref)[0]
    assert bad.size == 0, f"{bad.size} states differ, e.g. {bad[:5]} gpu={first[bad[:5]]} ref={ref[bad[:5]]}"
    assert (ref > 0).sum() > 50 and (ref < 0).sum() < len(states)


def _uf_byte_table_states(rng, n):
    """Calldata-shaped UF applications (calldata.py:219-232, lowered as v1 EQSEL chains):
    8-bit reads f(i) at constant indices, symbolic reads f(q), f(q + c), f(y) selecting
    among them (TSEL over the constant keys, TSELS over the symbolic ones), and a second
    function with 256-bit values; the fresh variables are read unmasked by the selects, so
    candidates put garbage above bit 8 (the selects must mask what they pick).  Root: an Or
    of equalities between reads, their concatenation and constants."""
    out = []
    for _ in range(n):
        nl = [[S.VAR, 256, -1, -1, -1, 0, 0], [S.VAR, 256, -1, -1, -1, 1, 0]]   # q, y
        cl = []

        def add(row):
            nl.append(row)
            return len(nl) - 1

        def const(v):
            cl.append(v)
            return add([S.CONST, 256, -1, -1, -1, len(cl) - 1, 0])

        fresh = [10]

        def app(arg, w=8, fid=5):
            fresh[0] += 1
            return add([S.UFAPP, w, arg, -1, -1, fid, fresh[0]])

        k = int(rng.integers(4, 24))
        const_reads = [app(const(i)) for i in range(k)]
        sym = [app(0)]
        for c in rng.choice(np.arange(1, 6), size=int(rng.integers(1, 4)), replace=False):
            sym.append(app(add([S.ADD, 256, 0, const(int(c)), -1, 0, 0])))
        sym.append(app(1))
        wide = [app(const(int(rng.integers(0, 8))), 256, 6) for _ in range(3)] + [app(0, 256, 6)]
        eqs = []
        for _ in range(int(rng.integers(2, 5))):
            r = rng.random()
            a = int(rng.choice(sym))
            if r < 0.4:
                eqs.append(add([S.EQ, 1, a, int(rng.choice(const_reads)), -1, 0, 0]))
            elif r < 0.6:
                cc = add([S.CONST, 8, -1, -1, -1, len(cl), 0])
                cl.append(int(rng.integers(0, 4)))
                eqs.append(add([S.EQ, 1, a, cc, -1, 0, 0]))
            elif r < 0.8:
                cat = add([S.CONCAT, 16, a, int(rng.choice(sym)), -1, 0, 0])
                cc = add([S.CONST, 16, -1, -1, -1, len(cl), 0])
                cl.append(int(rng.integers(0, 4)) * 257)
                eqs.append(add([S.EQ, 1, cat, cc, -1, 0, 0]))
            else:
                eqs.append(add([S.EQ, 1, wide[-1], int(rng.choice(wide[:-1])), -1, 0, 0]))
        root = eqs[0]
        for e in eqs[1:]:
            root = add([S.BOR if rng.random() < 0.6 else S.BAND, 1, root, e, -1, 0, 0])
        out.append((nl, cl))
    return out


def _uf_byte_table_cands(rng, states, n_cand):
    """q, y near the constant indices; fresh values 0..3, half of them with garbage above
    bit 8 (only the 8-bit reads ignore it; the 256-bit function's values use it)."""
    n_vars = max(max(r[6] for r in nl if r[0] == S.UFAPP) + 1 for nl, _ in states)
    cands = np.zeros((len(states), n_cand, n_vars, 8), np.uint32)
    cands[:, :, 2:, 0] = rng.integers(0, 4, size=(len(states), n_cand, n_vars - 2))
    junk = rng.random((len(states), n_cand, n_vars - 2)) < 0.5
    cands[:, :, 2:, 0] |= np.where(junk, rng.integers(1, 1 << 20, size=junk.shape) << 8, 0).astype(np.uint32)
    cands[:, :, :2, 0] = rng.integers(0, 28, size=(len(states), n_cand, 2))
    return cands


def test_uf_byte_tables_vs_oracle(mgp_ctx):
    """UF chains as v1 EQSEL steps (narrow values selected from unmasked fresh variables,
    masked by the step) through both engines: first-SAT equal to the C oracle's."""
    rng = np.random.default_rng(919)
    states = _uf_byte_table_states(rng, 300)
    nodes, noff, consts, coff = pack_states(states)
    words, po, status = _lower(nodes, noff, consts, coff)
    assert (status == 0).all()
    cands = _uf_byte_table_cands(rng, states, 256)
    first, _ = mgp_ctx.eval_batch(words, po, cands)
    ref = coracle.first_sat(nodes, noff, consts, coff, cands)
    bad = np.nonzero(first != ref)[0]
    assert bad.size == 0, f"{bad.size} states differ, e.g. {bad[:5]} gpu={first[bad[:5]]} ref={ref[bad[:5]]}"
    assert (ref > 0).sum() > 30 and (ref < 0).sum() > 10


def _mul_after_shift_states(rng, n):
    """A per-lane shift (its handler leaves v6 = 32 - amount, or all-ones for amounts >=
    256) and then MULs whose products' high limbs decide a compare.  The r3n defect: the
    MUL handler's Comba column 0 moved v6 into the accumulator's high word instead of 0,
    so a product read whatever the previous handler left in v6."""
    w = 256
    shifts = [S.LSHR, S.SHL, S.ASHR]
    cmps = [S.ULT, S.UGT, S.SLT]
    out = []
    for _ in range(n):
        nl = [[S.VAR, w, -1, -1, -1, k, 0] for k in range(3)]
        cl = [int(rng.integers(1, 2 ** 62)) << 192, int(rng.integers(0, 2 ** 32))]
        nl += [[S.CONST, w, -1, -1, -1, k, 0] for k in range(2)]                  # 3, 4
        nl.append([shifts[int(rng.integers(3))], w, 2, int(rng.integers(0, 2)), -1, 0, 0])  # 5
        nl.append([S.MUL, w, 0, 1, -1, 0, 0])                                      # 6
        nl.append([cmps[int(rng.integers(3))], 1, 6, 3, -1, 0, 0])                 # 7
        nl.append([S.EQ, 1, 5, 4, -1, 0, 0])                                       # 8
        nl.append([S.BNOT, 1, 8, -1, -1, 0, 0])                                    # 9
        nl.append([S.BAND, 1, 7, 9, -1, 0, 0])                                     # 10
        if rng.random() < 0.5:   # a second product after another shift
            nl.append([shifts[int(rng.integers(3))], w, 5, 1, -1, 0, 0])           # 11
            nl.append([S.MUL, w, 11, 2, -1, 0, 0])                                 # 12
            nl.append([S.ULT, 1, 12, 3, -1, 0, 0])                                 # 13
            nl.append([S.BAND, 1, 10, 13, -1, 0, 0])
        out.append((nl, cl))
    return out


def test_mul_after_shift_scratch_vs_oracle(mgp_ctx):
    """MUL after a handler that leaves scratch register v6 non-zero, against the C oracle on
    every candidate (both engines).  Fails on the r3n MUL (column 0 reading a stale v6),
    which the full-size test caught as 39 339 asm/HIP disagreements."""
    rng = np.random.default_rng(2026)
    states = _mul_after_shift_states(rng, 512)
    nodes, noff, consts, coff = pack_states(states)
    words, po, status = _lower(nodes, noff, consts, coff)
    assert (status == 0).all()
    cands = random_cands(rng, len(states), 256, 3, interesting_frac=0.3)
    small = rng.random((len(states), 256)) < 0.4   # shift amounts < 256 as well as >= 256
    cands[small, 1, 1:] = 0
    cands[small, 1, 0] &= 0xFF
    first, _ = mgp_ctx.eval_batch(words, po, cands)
    ref = coracle.first_sat(nodes, noff, consts, coff, cands)
    bad = np.nonzero(first != ref)[0]
    assert bad.size == 0, f"{bad.size} states differ, e.g. {bad[:5]}"
    assert (ref > 0).sum() > 100   # witnesses past candidate 0: earlier products were read


def test_band4n_then_hbm_variables_vs_oracle(mgp_ctx):
    """Compares on variables 6.. (HBM loads, not the register bank) after folded BAND4N
    chains, against the C oracle on every candidate (both engines)."""
    rng = np.random.default_rng(93)
    states = _band4n_states(rng, 400, late_vars=6)
    nodes, noff, consts, coff = pack_states(states)
    words, po, status = _lower(nodes, noff, consts, coff)
    assert (status == 0).all()
    cands = np.zeros((len(states), 256, 9, 8), np.uint32)
    cands[..., 0] = rng.integers(0, 256, size=(len(states), 256, 9))
    first, _ = mgp_ctx.eval_batch(words, po, cands)
    ref = coracle.first_sat(nodes, noff, consts, coff, cands)
    bad = np.nonzero(first != ref)[0]
    assert bad.size == 0, f"{bad.size} states differ, e.g. {bad[:5]}"
    assert (ref >= 0).sum() > 20


def test_band4n_folds_vs_oracle(mgp_ctx):
    """BNOTs folded into AND chains (BAND4N) against the C oracle on every candidate (both
    engines; the HIP engine runs the v1 program, which has no fold)."""
    rng = np.random.default_rng(91)
    states = _band4n_states(rng, 600)
    nodes, noff, consts, coff = pack_states(states)
    words, po, status = _lower(nodes, noff, consts, coff)
    assert (status == 0).all()
    n_cand = 256
    vals = rng.integers(0, 256, size=(len(states), n_cand, 3))
    cands = np.zeros((len(states), n_cand, 3, 8), np.uint32)
    cands[..., 0] = vals
    first, _ = mgp_ctx.eval_batch(words, po, cands)
    ref = coracle.first_sat(nodes, noff, consts, coff, cands)
    bad = np.nonzero(first != ref)[0]
    assert bad.size == 0, f"{bad.size} states differ, e.g. {bad[:5]}"


def test_bool_folds_vs_oracle(mgp_ctx):
    """Compare -> BAND/BOR (BCOMB) and BNOT -> BAND (BANDN) folds of the gfx950 uop
    translation against the C oracle on every candidate (both engines)."""
    rng = np.random.default_rng(77)
    states = _bool_fold_states(rng, 600)
    nodes, noff, consts, coff = pack_states(states)
    words, po, status = _lower(nodes, noff, consts, coff)
    assert (status == 0).all()
    cands = random_cands(rng, len(states), 128, 3, interesting_frac=0.0)
    cands[:, :, :, 1:] = 0
    cands[:, :, :, 0] &= 0xFF
    first, _ = mgp_ctx.eval_batch(words, po, cands)
    ref = coracle.first_sat(nodes, noff, consts, coff, cands)
    mism = np.nonzero(first != ref)[0]
    assert mism.size == 0, f"{mism.size} states differ, e.g. {mism[:5]} gpu={first[mism[:5]]} ref={ref[mism[:5]]}"
    assert 0 < (first >= 0).sum() < len(states)


def test_back_to_back_batches_same_context(mgp_ctx):
    """Consecutive batches of the same size on one context reuse the same device buffers
    (and launch-descriptor addresses) with different programs: every batch must see its
    own programs (the interpreter reads its launch descriptors past the scalar cache)."""
    rng = np.random.default_rng(7)
    batches = []
    for seed in range(3):
        b = N.synth_generate(1000 + seed, 0, 48, 40, 64)
        words, po, status = _lower(b["nodes"], b["node_offsets"], b["consts"], b["const_offsets"])
        cands = random_cands(rng, 48, 64, b["n_vars"], interesting_frac=0.3)
        want = coracle.first_sat(b["nodes"], b["node_offsets"], b["consts"], b["const_offsets"], cands)
        batches.append((words, po, status, cands, want))
    for _ in range(3):
        for words, po, status, cands, want in batches:
            first, _ = mgp_ctx.eval_batch(words, po, cands)
            ok = status == 0
            assert np.array_equal(first[ok], want[ok])


def test_spilled_values_and_demoted_bools(mgp_ctx):
    """Programs past the LDS slots (BV values spilled to candidate rows past the state's
    variables, past slot 255 too), past the 17 Bool registers (demoted Bools) and past 64 constants, in one
    batch with ordinary states: the C ABI pads the candidate rows, both engines agree
    with the oracle, and the witness rows of the variables come back unchanged."""
    from .test_lowering import _bool_fan, _live_chain

    rng = np.random.default_rng(77)
    # 300 live values: destinations past slot 255 (high bits in instruction word 3)
    states = [(_live_chain(n), []) for n in (36, 90, 200, 300)] + [_bool_fan(n) for n in (24, 60)]
    nl = [[S.VAR, 256, -1, -1, -1, 0, 0], [S.VAR, 256, -1, -1, -1, 1, 0]]
    pool = [(k * 0x9E3779B97F4A7C15 + 1) % 2 ** 256 for k in range(150)]
    acc = 0
    for k in range(150):
        nl.append([S.CONST, 256, -1, -1, -1, k, 0])
        nl.append([S.XOR if k % 3 else S.ADD, 256, acc, len(nl) - 1, -1, 0, 0])
        acc = len(nl) - 1
    nl.append([S.ULT, 1, acc, 1, -1, 0, 0])
    states.append((nl, pool))
    b = N.synth_generate(0x4D595448, 4242, 40, 64, 100)
    for s in range(40):
        ns, cs = state_slice(b, s)
        states.append(([[int(r[f]) for f in ("op", "width", "a", "b", "c", "p0", "p1")] for r in ns], cs))
    nodes, noff, consts, coff = pack_states(states)
    words, po, status = _lower(nodes, noff, consts, coff)
    assert (status == 0).all()
    rows = N.prog_rows(words, po)
    n_vars = 6
    assert rows.max() > n_vars  # some program needs spill rows
    cands = random_cands(rng, len(states), 100, n_vars, interesting_frac=0.2)
    for s in range(len(states) - 40, len(states)):  # planted witnesses of the synthetic states
        if b["planted"][s - (len(states) - 40)]:
            cands[s, 7] = b["plant_words"][s - (len(states) - 40)]
    first, wit = mgp_ctx.eval_batch(words, po, cands)
    want = coracle.first_sat(nodes, noff, consts, coff, cands)
    mism = np.nonzero(first != want)[0]
    assert mism.size == 0, f"states {mism[:8]} gpu={first[mism[:8]]} oracle={want[mism[:8]]}"
    assert (first >= 0).sum() > 10
    for s in np.nonzero(first >= 0)[0]:
        assert (wit[s] == cands[s, first[s]]).all()
