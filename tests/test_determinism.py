"""The host pieces of the witness search are functions of the state's content (CPU only).

A state's answer must not depend on the batch it arrives in, on the order of that batch,
on how many host threads run, or on what ran before (VERDICT r2 "Next round" item 2).  On
the GPU side the candidate streams are keyed by the state's content key
(MGP_FE_STATE_KEY); here the host side is checked: the content keys themselves, the
first-round candidate generator keyed by them, and the decision rows
(mgp_decision_rows), each in two batch orders and, in subprocesses, with
OMP_NUM_THREADS=1 and 8.
"""
import os
import subprocess
import sys

import numpy as np

from mythril_amd import _native as N
from mythril_amd import dag as D
from mythril_amd import front as F
from mythril_amd import solver as SV

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _states(n=72):
    import corpus

    return [c[1] for c in corpus.corpus(n)]


def _digest(states):
    """(state keys, first-round candidates, decision rows + masks) of a batch."""
    B = F.Batch(states)
    nv = max(1, B.n_vars())
    cands = N.make_candidates(64, nv, 11, B.var_off, B.var_width, B.hint_off, B.hints, B.alias_off, B.aliases,
                              B.const_off, B.consts, D._FIXED_LIMBS, np.zeros(B.n_states, np.uint8),
                              var_kind=B.var_kind, state_keys=B.state_key)
    rows, mask, st = N.decision_rows(*B.packed(decide=True), nv, 5, 4, None, state_keys=B.state_key)
    keys = np.array(B.state_key)
    nvs = np.diff(B.var_off).astype(int)
    B.close()
    # per state, its own variables only (the batch's padding width differs between batches)
    c = [cands[s, :, : nvs[s]].copy() for s in range(len(states))]
    r = [rows[s, :, : nvs[s]].copy() for s in range(len(states))]
    m = [mask[s, :, : nvs[s]].copy() for s in range(len(states))]
    return keys, c, r, m, st


def test_same_state_same_rows_in_any_batch_order():
    states = _states()
    k1, c1, r1, m1, s1 = _digest(states)
    perm = np.random.default_rng(3).permutation(len(states))
    k2, c2, r2, m2, s2 = _digest([states[i] for i in perm])
    assert np.array_equal(k2, k1[perm]) and np.array_equal(s2, s1[perm])
    for j, i in enumerate(perm):
        assert np.array_equal(c2[j], c1[i]) and np.array_equal(r2[j], r1[i]) and np.array_equal(m2[j], m1[i])
    # a state alone in its batch: the same rows again
    k3, c3, r3, m3, _ = _digest([states[5]])
    assert k3[0] == k1[5] and np.array_equal(c3[0], c1[5]) and np.array_equal(r3[0], r1[5])
    # decision rows exist for the states the pre-check does not refute
    assert all(m1[i].any() for i in range(len(states)) if s1[i] == 0)
    assert not any(m1[i].any() for i in range(len(states)) if s1[i] != 0)


def test_equal_content_equal_key_distinct_content_distinct_key():
    """Keys follow content: an uninterpreted function is its name (two Array objects named
    "2_calldata" are one function to z3), so the arena's function ids do not count."""
    states = _states(48)
    B = F.Batch(states + states[:8])
    keys = np.array(B.state_key)
    sig = []
    for s in range(48):
        nd = np.array(B.nodes[int(B.node_off[s]): int(B.node_off[s + 1])])
        uf = np.isin(nd["op"], [70, 71])  # UFAPP / UFINV: the function by name (its fresh slot's name)
        nd["p0"][uf] = 0
        sig.append((nd.tobytes(), B.consts[int(B.const_off[s]): int(B.const_off[s + 1])].tobytes(),
                    tuple(B.var_names(s))))
    B.close()
    assert np.array_equal(keys[48:], keys[:8])
    groups = {}
    for k, g in zip(keys[:48].tolist(), sig):
        groups.setdefault(k, set()).add(g)
    assert all(len(g) == 1 for g in groups.values())           # one key, one content
    assert len(groups) == len(set(sig))                         # one content, one key


_CHILD = r"""
import sys, numpy as np
sys.path.insert(0, {root!r})
from tests.test_determinism import _digest, _states
k, c, r, m, s = _digest(_states())
np.savez({out!r}, k=k, s=s, r=np.concatenate([x.reshape(-1) for x in r]),
         m=np.concatenate([x.reshape(-1) for x in m]), c=np.concatenate([x.reshape(-1) for x in c]))
"""


def test_rows_do_not_depend_on_thread_count(tmp_path):
    got = []
    for threads in (1, 8):
        out = str(tmp_path / f"t{threads}.npz")
        env = dict(os.environ, OMP_NUM_THREADS=str(threads))
        subprocess.run([sys.executable, "-c", _CHILD.format(root=ROOT, out=out)], check=True, env=env, cwd=ROOT,
                       timeout=600)
        got.append(np.load(out))
    for name in ("k", "s", "r", "m", "c"):
        assert np.array_equal(got[0][name], got[1][name]), name


def test_first_round_rows_are_a_function_of_the_state():
    """Prefilter._first_round_rows (restated by tests/fe_emulate.first_round_rows): the
    decision rows a large state gets in the first round are the same in any batch that
    holds it, and small states get none (their mask rows are empty)."""
    import corpus
    from tests import fe_emulate as E

    C = corpus.corpus(96)
    cs = [c[1] for c in C]
    B = F.Batch(cs)
    rows, mask = E.first_round_rows(B, 0x4D595448)
    big = np.diff(B.node_off) > SV.Prefilter.ROWS_FIRST_NODES
    assert big.any() and (~big).any()
    assert not mask[~big].any() and mask[big].any()
    sub = [i for i in range(96) if i % 5 in (1, 3)]
    SB = F.Batch([cs[i] for i in sub])
    rows2, mask2 = E.first_round_rows(SB, 0x4D595448)
    gv = rows2.shape[2]
    assert np.array_equal(rows[sub][:, :, :gv], rows2) and np.array_equal(mask[sub][:, :, :gv], mask2)
    assert not mask[sub][:, :, gv:].any()
    B.close()
    SB.close()


def test_row_range_is_a_slice_of_the_full_rows():
    """mgp_decision_rows_from (the first round's row 1 of large states): output row k is
    decision row row0 + k of the full call, unseeded and parent-seeded, per state."""
    import corpus

    C = corpus.corpus(64)
    cs = [c[1] for c in C if c[0].startswith("wallet")][:6] + [c[1] for c in C if c[0].startswith("bec")][:6]
    B = F.Batch(cs)
    nv = max(1, B.n_vars())
    pk = B.packed(decide=True)
    full, fmask, fst = N.decision_rows(*pk, nv, 21, 4, None, state_keys=B.state_key)
    for row0, n in ((1, 1), (1, 3), (2, 2)):
        r, m, st = N.decision_rows(*pk, nv, 21, n, None, state_keys=B.state_key, row0=row0)
        assert np.array_equal(st, fst)
        assert np.array_equal(r, full[:, row0:row0 + n]) and np.array_equal(m, fmask[:, row0:row0 + n])
    # seeded: every slot of a parent witness offered (the states' own row 0 values)
    seeds = (np.ascontiguousarray(full[:, 0]), np.ascontiguousarray(fmask[:, 0]))
    sf, sm, _ = N.decision_rows(*pk, nv, 21, 3, None, state_keys=B.state_key, seeds=seeds, seed_rows=0x3)
    s1, m1, _ = N.decision_rows(*pk, nv, 21, 2, None, state_keys=B.state_key, seeds=seeds, seed_rows=0x3, row0=1)
    assert np.array_equal(s1, sf[:, 1:3]) and np.array_equal(m1, sm[:, 1:3])
    B.close()


def test_content_keys_do_not_depend_on_the_process_history():
    """A state's content key is the same in a process that interned other names first
    (round 6: a pinned constant's slot hashed the arena's name 0, whatever name that was):
    two subprocesses build the same calls.sol query, one after creating an unrelated symbol."""
    import subprocess
    import sys

    code = (
        "import sys; sys.path.insert(0, {root!r})\n"
        "{pre}"
        "import corpus\n"
        "from oracle.keccak_ref import keccak256\n"
        "from mythril_amd import front as F\n"
        "qs = corpus.suite(hasher=keccak256, contracts={{'calls'}})\n"
        "keys = []\n"
        "for q in qs[:60]:\n"
        "    B = F.Batch([list(q[3])]); keys.append(int(B.state_key[0])); B.close()\n"
        "print(keys)\n")
    import os

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    outs = []
    for pre in ("", "from mythril_amd.smt import symbol_factory; _z = symbol_factory.BitVecSym('zz_first', 256)\n"):
        r = subprocess.run([sys.executable, "-c", code.format(root=root, pre=pre)], capture_output=True, text=True,
                           timeout=300, check=True)
        outs.append(r.stdout.strip().splitlines()[-1])
    assert outs[0] == outs[1]
