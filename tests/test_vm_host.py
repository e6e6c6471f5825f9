"""The generated Fp-VM programs (tools/fpvm) executed by the interpreter's own code
(consensus_overlord_amd/csrc/fpvm.hpp exec, host build in tests/host/harness.cpp), compared
value by value with the slot-level simulator (tools/fpvm/sched.simulate), which gen.py --check
ties to the CPU oracle on the golden votes. Both interpreter modes: each lane alone, and every
wave-uniform block run for every lane (what a mixed wave does on the GPU)."""
import ctypes
import json
import os
import sys

import numpy as np
import pytest

from test_host_harness import hx  # noqa: F401  (module fixture: builds libhx.so)

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools", "fpvm"))

import gen  # noqa: E402
import progs  # noqa: E402
import sched  # noqa: E402
from ir import P  # noqa: E402

R = pow(2, 384, P)
RAW_INPUTS = {"pk_sort", "sig_sort"}   # flags the vote prologue writes as plain limbs


def _words(v):
    return [(v >> (32 * k)) & 0xFFFFFFFF for k in range(12)]


def _int(ws):
    return sum(int(w) << (32 * k) for k, w in enumerate(ws))


@pytest.fixture(scope="module")
def built():
    return gen.build_all()


def run_vm(hx, consts, sc, words, inputs, scalar, any_all):
    prog = sc.prog
    slots = np.zeros(sc.nslots * 12, dtype=np.uint32)
    for name, v in prog.inputs.items():
        if v in sc.slot_of:
            val = inputs[name] % P
            s = sc.slot_of[v]
            slots[s * 12:s * 12 + 12] = _words(val if name in RAW_INPUTS else val * R % P)
    code = np.asarray(words, dtype=np.uint32)
    cst = np.asarray(consts.words(), dtype=np.uint32).ravel()
    planes = np.zeros(64 * 12, dtype=np.uint32)
    u32p = ctypes.POINTER(ctypes.c_uint32)
    hx.hx_vm_run.argtypes = [u32p, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32, u32p, u32p, ctypes.c_uint64,
                             u32p, ctypes.c_uint32, ctypes.c_int, u32p, u32p]
    # spilled programs (sched.spill_pass): side words and the unit's scratch
    nscr = getattr(sc, "nscr", 0)
    side = np.asarray(sc.side_words, dtype=np.uint32) if nscr else None
    scr = np.zeros(max(nscr, 1) * 12, dtype=np.uint32)
    assert hx.hx_vm_run(code.ctypes.data_as(u32p), sc.nrounds, sc.W, sched.words_per_lane(prog), cst.ctypes.data_as(u32p),
                        slots.ctypes.data_as(u32p), scalar, planes.ctypes.data_as(u32p), 64, any_all,
                        side.ctypes.data_as(u32p) if side is not None else None, scr.ctypes.data_as(u32p)) == 0
    out = {}
    for name, v in prog.outputs.items():
        op = prog.ops[v]
        if op.kind == "st":
            out[name] = _int(planes[op.imm * 12:op.imm * 12 + 12])
        else:
            s = sc.slot_of[v]
            out[name] = _int(slots[s * 12:s * 12 + 12])
    return out


def assert_same(dev, sim, what):
    for name, s in sim.items():
        d = dev[name]
        # a Montgomery representative in [0, 2p) (canonical for `st` planes) or a raw flag
        ok = (d % P == s * R % P and d < (P if name.startswith("st:") else 2 * P)) or (s in (0, 1) and d == s)
        assert ok, "%s: output %s interpreter %x, simulator %x" % (what, name, d, s)


@pytest.fixture(scope="module")
def golden_votes():
    with open(os.path.join(ROOT, "tests", "golden", "golden_v1.json")) as fh:
        g = json.load(fh)
    bls = gen._oracle()
    out = []
    for v, k in list(zip(g["votes"], g["keys"]))[:2]:
        out.append(gen.vote_inputs(bls, bytes.fromhex(k["pk"]), bytes.fromhex(v["sig"]), bytes.fromhex(v["digest"])))
    bad = [c for c in g["verify"] if c["code"] == 3 and len(c["sig"]) == 192 and len(c["pk"]) == 96]
    for c in bad[:1]:
        out.append(gen.vote_inputs(bls, bytes.fromhex(c["pk"]), bytes.fromhex(c["sig"]), bytes.fromhex(c["hash"])))
    return out


@pytest.mark.parametrize("any_all", [0, 1])
def test_vote_program_on_interpreter(hx, built, golden_votes, any_all):  # noqa: F811
    consts, progs_ = built
    prog, sc, words, _, _ = progs_["vote"]
    r = 0xD7A1C3B5E9F20486
    for k, inp in enumerate(golden_votes):
        sim = sched.simulate(sc, words, inp, r)
        dev = run_vm(hx, consts, sc, words, inp, r, any_all)
        assert_same(dev, sim, "vote %d" % k)


@pytest.mark.parametrize("any_all", [0, 1])
def test_vote_t_program_on_interpreter(hx, built, golden_votes, any_all):  # noqa: F811
    """vote_t (key from the validator table, projective) on the golden votes: interpreter ==
    simulator, and the same sigma / tau (the MSM's points) as the vote program."""
    consts, progs_ = built
    _, vsc, vwords, _, _ = progs_["vote"]
    prog, sc, words, _, _ = progs_["vote_t"]
    bls = gen._oracle()
    with open(os.path.join(ROOT, "tests", "golden", "golden_v1.json")) as fh:
        g = json.load(fh)
    r = 0x0F1E2D3C4B5A6978
    for k, inp in enumerate(golden_votes[:2]):
        pk = bls.g1_from_bytes(bytes.fromhex(g["keys"][k]["pk"]))
        tin = {n: inp[n] for n in ("sig_x0", "sig_x1", "sig_sort", "u00", "u01", "u10", "u11")}
        tin.update(pk_X=pk[0] * 5 % P, pk_Y=pk[1] * 5 % P, pk_Z=5)
        sim = sched.simulate(sc, words, tin, r)
        assert_same(run_vm(hx, consts, sc, words, tin, r, any_all), sim, "vote_t %d" % k)
        vsim = sched.simulate(vsc, vwords, inp, r)
        qt = ["st:q%d" % j for j in range(4)] + ["st:t%d" % j for j in range(4)]
        assert [sim[n] for n in qt] == [vsim[n] for n in qt]


@pytest.mark.parametrize("any_all", [0, 1])
def test_fold_final_bisect_on_interpreter(hx, built, golden_votes, any_all):  # noqa: F811
    consts, progs_ = built
    prog, sc, words, _, _ = progs_["vote"]
    _, rsc, rwords, _, _ = progs_["rs"]
    r = 0x1234567890ABCDEF
    parts = []
    for inp in golden_votes[:2]:
        o = sched.simulate(sc, words, inp, r)
        o = {(n[3:] if n.startswith("st:") else n): v for n, v in o.items()}
        # the bisection's r sigma from the stored sigma / tau (program rs), interpreter == simulator
        rin = {n: o[n] for n in progs.RS_IN}
        rsim = sched.simulate(rsc, rwords, rin, r)
        assert_same(run_vm(hx, consts, rsc, rwords, rin, r, any_all), rsim, "rs")
        o.update({n[3:]: v for n, v in rsim.items()})
        parts.append(o)

    def final_in(items):
        inp = {}
        for k in range(progs.FOLD_K):
            for j in range(12):
                inp["F%d_%d" % (k, j)] = items[k][0]["f%d" % j] if k < len(items) else (1 if j == 0 else 0)
            for j in range(6):
                inp["S%d_%d" % (k, j)] = items[k][1]["s%d" % j] if k < len(items) else (1 if j == 2 else 0)
        return inp
    inp = final_in([(parts[0], parts[0]), (parts[1], parts[1])])
    for name in ("fold", "final"):
        _, psc, pwords, _, _ = progs_[name]
        sim = sched.simulate(psc, pwords, inp)
        assert_same(run_vm(hx, consts, psc, pwords, inp, 0, any_all), sim, name)
        if name == "final":
            assert sim == {"ok": 1}
    # the bisection's per-vote check: one vote's own (f, r sigma) passes, a mismatched pair fails
    _, psc, pwords, _, _ = progs_["final"]
    for items, want in (([(parts[0], parts[0])], 1), ([(parts[0], parts[1])], 0)):
        pin = final_in(items)
        sim = sched.simulate(psc, pwords, pin)
        assert sim == {"ok": want}
        assert_same(run_vm(hx, consts, psc, pwords, pin, 0, any_all), sim, "final/bisect")


@pytest.mark.parametrize("any_all", [0, 1])
def test_msm_programs_on_interpreter(hx, built, golden_votes, any_all):  # noqa: F811
    """The MSM pair programs (madd, padd, hdbl<m>) through the interpreter == simulator on golden
    signature points, identity operands and the doubling case (gen.check_msm ties the programs'
    values to the oracle's point arithmetic)."""
    consts, progs_ = built
    bls = gen._oracle()
    with open(os.path.join(ROOT, "tests", "golden", "golden_v1.json")) as fh:
        g = json.load(fh)
    A, B = (bls.g2_from_bytes(bytes.fromhex(v["sig"])) for v in g["votes"][:2])
    for name, (prog, sc, words, ins, outs) in progs_.items():
        if name not in ("madd", "padd") and not name.startswith("hdbl"):
            continue
        for X, Y in ((A, B), (A, A), (B, None), (None, B)):
            if name == "madd" and X is None:
                continue
            xa = [X[0][0], X[0][1], X[1][0], X[1][1]] if name == "madd" else gen._proj(X, (7, 2))
            inp = dict(zip(ins, xa + gen._proj(Y)))
            sim = sched.simulate(sc, words, inp)
            assert_same(run_vm(hx, consts, sc, words, inp, 0, any_all), sim, name)


def test_fp_inv(hx):
    """fpvm.hpp fp_inv (Bernstein-Yang divsteps, the final program's inv op) against pow(a, -1, p)
    on edge values and seeded random ones, including values with long runs of zero / one bits."""
    u32p = ctypes.POINTER(ctypes.c_uint32)
    hx.hx_fp_inv_raw.argtypes = [u32p, u32p, u32p]
    rr = np.array(_words(R), dtype=np.uint32)
    rng = np.random.default_rng(0xB1A5)
    vals = [0, 1, 2, 3, P - 1, P - 2, (P - 1) // 2, (P + 1) // 2, 2 ** 380, 2 ** 381 - 1 - P + P // 3,
            (1 << 32) - 1, 1 << 200, P - (1 << 300)]
    vals += [int.from_bytes(rng.bytes(48), "little") % P for _ in range(400)]
    vals += [int.from_bytes(rng.bytes(48), "little") % (1 << int(rng.integers(1, 381))) for _ in range(100)]
    for a in vals:
        a %= P
        out = np.zeros(12, dtype=np.uint32)
        hx.hx_fp_inv_raw(np.array(_words(a), dtype=np.uint32).ctypes.data_as(u32p), rr.ctypes.data_as(u32p),
                         out.ctypes.data_as(u32p))
        got = sum(int(w) << (32 * k) for k, w in enumerate(out))
        assert got == (pow(a, -1, P) if a else 0), hex(a)


@pytest.mark.parametrize("any_all", [0, 1])
def test_percall_programs_on_interpreter(hx, built, golden_votes, any_all):  # noqa: F811
    """The per-call programs through the interpreter == simulator: sigchk / pkchk on golden
    signatures and keys (a non-subgroup case included), g1padd, signg0 + signg1 over a golden
    key's GLS digits, vote1 / vote_t1 + final1 and the small-batch votew / votew_t + final1 on a
    golden vote (gen.check ties each to
    the oracle: decompressed points, sums, the golden signature, the pairing verdict)."""
    consts, progs_ = built
    bls = gen._oracle()
    with open(os.path.join(ROOT, "tests", "golden", "golden_v1.json")) as fh:
        g = json.load(fh)

    def run(name, inp, scalar=0):
        _, sc, words, _, _ = progs_[name]
        sim = sched.simulate(sc, words, inp, scalar)
        assert_same(run_vm(hx, consts, sc, words, inp, scalar, any_all), sim, name)
        return sim
    for inp in golden_votes:
        run("sigchk", {n: inp[n] for n in progs.SIGCHK_IN})
        run("pkchk", {n: inp[n] for n in progs.PKCHK_IN})
    A, B = (bls.g1_from_bytes(bytes.fromhex(k["pk"])) for k in g["keys"][:2])
    run("g1padd", dict(zip(progs.G1A_IN + progs.G1B_IN, [A[0] * 3 % P, A[1] * 3 % P, 3, B[0], B[1], 1])))
    sk = int(g["keys"][0]["sk"], 16)
    d = gen.gls_digits(sk)
    inp = golden_votes[0]
    o = run("signg0", {n: inp[n] for n in progs.SIGN0_IN}, gen.signg_scalar(d, 0))
    run("signg1", {n: o[n] for n in progs.SIGN_ACC + progs.SIGNG_T}, gen.signg_scalar(d, 1))
    o = run("vote1", inp, 1)
    fin = {"f%d" % j: o["st:f%d" % j] for j in range(12)}
    assert run("final1", fin) == {"ok": 1}
    pk = bls.g1_from_bytes(bytes.fromhex(g["keys"][0]["pk"]))
    tin = {n: inp[n] for n in ("sig_x0", "sig_x1", "sig_sort", "u00", "u01", "u10", "u11")}
    tin.update(pk_X=pk[0] * 5 % P, pk_Y=pk[1] * 5 % P, pk_Z=5)
    run("vote_t1", tin, 1)
    # the small-batch programs under a random RLC scalar: FE(f) == 1 for the valid golden vote
    r = 0x9E3779B97F4A7C15
    o = run("votew", inp, r)
    assert run("final1", {"f%d" % j: o["st:f%d" % j] for j in range(12)}) == {"ok": 1}
    run("votew_t", tin, r)
    # verify_aggregated_signature's split: qcpre (signature, H, Miller(-G1, sigma)) + qcmil
    q = run("qcpre", {n: inp[n] for n in progs.QCPRE_IN})
    mi = {"pk_X": tin["pk_X"], "pk_Y": tin["pk_Y"], "pk_Z": tin["pk_Z"]}
    mi.update({"h%d" % k: q["st:h%d" % k] for k in range(6)})
    mi.update({"g%d" % k: q["st:g%d" % k] for k in range(12)})
    # pkgen: one 64-bit window chunk from the identity (gen.check runs the four launches vs the oracle)
    run("pkgen", {"c0": 0, "c1": 1, "c2": 0}, 0xFEDCBA9876543210)
    o = run("qcmil", mi)
    assert run("final1", {"f%d" % j: o["st:f%d" % j] for j in range(12)}) == {"ok": 1}


@pytest.mark.parametrize("any_all", [0, 1])
def test_samemsg_programs_on_interpreter(hx, built, golden_votes, any_all):  # noqa: F811
    """The same-message programs through the interpreter == simulator,
    and the simulator == the oracle (gen.check_samemsg: sigma, tau, r pk, hash_to_G2, the Miller
    loop of the key sum, pkdec's key validation)."""
    consts, progs_ = built
    bls = gen._oracle()
    with open(os.path.join(ROOT, "tests", "golden", "golden_v1.json")) as fh:
        g = json.load(fh)
    if any_all == 0:
        gen.check_samemsg(progs_, bls, g)
    r = 0xC2B2AE3D27D4EB4F

    def run(name, inp, scalar=0):
        _, sc, words, _, _ = progs_[name]
        sim = sched.simulate(sc, words, inp, scalar)
        assert_same(run_vm(hx, consts, sc, words, inp, scalar, any_all), sim, name)
        return sim
    for inp in golden_votes:
        o = run("vsame", {n: inp[n] for n in progs.VSAME_IN}, r)
        run("pkdec", {n: inp[n] for n in progs.PKCHK_IN})
    pk = bls.g1_from_bytes(bytes.fromhex(g["keys"][0]["pk"]))
    inp = golden_votes[0]
    tin = {n: inp[n] for n in ("sig_x0", "sig_x1", "sig_sort")}
    tin.update(pk_X=pk[0] * 5 % P, pk_Y=pk[1] * 5 % P, pk_Z=5)
    run("vsame_t", tin, r)
    h = run("h2g", {n: inp[n] for n in progs.H2G_IN})
    o = run("vsame", {n: inp[n] for n in progs.VSAME_IN}, r)
    mi = dict(zip(progs.GMIL_IN, [o["st:r%d" % j] for j in range(3)] + [h["st:h%d" % j] for j in range(6)]))
    run("gmil", mi)
    sig = bls.g2_from_bytes(bytes.fromhex(g["votes"][0]["sig"]))
    rs = bls.pt_mul(bls.Fp2Ops, sig, gen.alg.rlc_scalar(r))
    fin = dict(zip(progs.GFIN_IN, [1] + [0] * 11 + [o["st:r%d" % j] for j in range(3)] +
                   [h["st:h%d" % j] for j in range(6)] + gen._proj(rs)))
    assert run("gfin", fin) == {"ok": 1}


def test_spill_pass_bounds_slots_and_keeps_values(hx, built, golden_votes):  # noqa: F811
    """sched.spill_pass on the vote program at K = 120 (gen.py builds it at 90; 159 slots
    unspilled): at most K slots, every fill at least `gap` (3) phases after its value's spill,
    the schedule's phases unchanged, and the outputs (simulator, and the interpreter with side
    words) equal the unspilled program's on the golden votes."""
    consts, progs_ = built
    _, vsc, vwords, _, _ = progs_["vote"]
    K = 120
    builder, _, _ = progs.PROGRAMS["vote"]
    prog = builder()
    prog.fuse()
    sc = sched.schedule(prog, gen.WIDTH["vote"], consts, max_slots=400, heavy_w=gen.HEAVY_W["vote"],
                        hoist=gen.HOIST["vote"], stretch=gen.STRETCH["vote"], mixed=False, spill_k=K,
                        defer=gen.DEFER.get("vote"), families="vote" in gen.FAMILIES)
    words = sched.encode(sc)
    assert sc.nslots <= K and sc.nscr > 0 and sc.nfill >= sc.nspill > 0 and sc.nrounds == vsc.nrounds
    spill_at, fill_at = {}, []
    for t, rr in enumerate(sc.rounds):
        for i in rr:
            if prog.ops[i].kind == "spill":
                spill_at[prog.ops[i].srcs[0]] = t
            elif prog.ops[i].kind == "fill":
                fill_at.append((t, prog.ops[i].deps[0]))
    assert all(t >= spill_at[o] + 3 for t, o in fill_at)
    r = 0x0F1E2D3C4B5A6978
    for k, inp in enumerate(golden_votes):
        ref = sched.simulate(vsc, vwords, inp, r)
        sim = sched.simulate(sc, words, inp, r)
        assert sim == ref
        assert_same(run_vm(hx, consts, sc, words, inp, r, 0), sim, "vote %d spilled to %d" % (k, K))


def test_batch_schedule_rules(built):
    """The r06 scheduler rules on the batch vote programs (tools/fpvm/sched.py): every phase runs
    one lin block (the unit block, or every lin op in the general one); a unit lin's negated
    terms sit in its last positions (D, then C, then B), and the phase header's H_LINNEG2 /
    H_LINNEG3 bits cover every lane that negates C / B (fpvm.hpp lin_sum XORs only those);
    product phases are fuller than the r05 schedule's (lane use 0.833 on vote)."""
    _, progs_ = built
    for name in ("vote", "vote_t"):
        _, sc, words, _, _ = progs_[name]
        nw = sched.words_per_lane(sc.prog)
        for t in range(sc.nrounds):
            lanes = [words[(t * sc.W + l) * nw:(t * sc.W + l) * nw + 4] for l in range(sc.W)]
            hdr = lanes[0][0] & ~0x3FFFFF
            assert all(w[0] & ~0x3FFFFF == hdr for w in lanes), (name, t, "header differs between lanes")
            for w in lanes:
                b = sched.phase_bits(w)
                assert b & hdr == b, (name, t, "lane needs a block the header lacks")
                if (w[0] & 31) == sched.OPC["lin"] and b & sched.H_LIN and not b & sched.H_SELB:
                    neg = [sched._s5((w[3] >> (5 * q)) & 31) < 0 for q in range(1, 4)]   # B, C, D
                    n = sum(neg)
                    assert neg == [False] * (3 - n) + [True] * n, (name, t, "negated terms not last", neg)
        st = sc.stats()
        assert st["lane_util_heavy"] > (0.87 if name == "vote" else 0.79), (name, st)
