#!/usr/bin/env python
"""Build, schedule, validate and emit the Fp-VM programs (progs.py) for libovhip.

    python tools/fpvm/gen.py [--out consensus_overlord_amd/csrc/vm_progs.inc] [--check]

Emits a C++ include with the shared constant table (12 x u32 limbs per entry, Montgomery or
raw), and per program: the phase-major instruction stream (W lanes x 4 u32 per phase), the
input / output slot maps (order = progs.*_IN / *_OUT) and the slot count. --check re-runs each
encoded program in the slot-level simulator and compares it with the traced DAG, and checks
the vote / vote_t / fold / final programs against the CPU oracle on golden votes.
"""
from __future__ import annotations

import argparse
import hashlib
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, HERE)

import alg  # noqa: E402
import progs  # noqa: E402
import sched  # noqa: E402
from ir import P  # noqa: E402

KZERO, KTAB = 1, 2   # fixed constant-table entries (fpvm.hpp)
WIDTH = {"vote": 16, "vote_t": 16, "fold": 64, "final": 64, "rs": 16, "madd": 8, "padd": 8}
WIDTH.update({"hdbl%d" % m: 16 for m in progs.HDBL_M})
WIDTH.update({"votew": 64, "votew_t": 64, "qcpre": 64, "qcmil": 64, "vote1h": 64, "vote_t1h": 64, "pkgen": 16,
              "signg0": 32, "signg1": 32})   # sign: per call a 32-lane slice (r03y: 2,280 -> 2,123 phases, -14% est.)
WIDTH.update({"sigchk": 16, "pkchk": 16, "g1padd": 8, "vote1": 64, "vote_t1": 64,
              "final1": 64})
# same-message batches (r04): per vote a 16-lane slice, per distinct hash one 16-lane slice for
# hash_to_G2 and one wave for its Miller loop (the latency of a round's group)
WIDTH.update({"vsame": 16, "vsame_t": 16, "h2g": 16, "gmil": 64, "pkdec": 4, "g1grp": 16, "gfin": 64})
WIDTH.update({"vsame8": 8, "vsame8_t": 8})   # large same-message batches: eight votes per wave
MAX_SLOTS = {"gfin": 2048, "vsame": 400, "vsame_t": 400, "vsame8": 400, "vsame8_t": 400, "h2g": 400, "gmil": 1200, "vote": 200, "vote_t": 200, "fold": 256, "final": 2048, "final1": 2048, "vote1": 1200, "vote_t1": 1200,
             "votew": 1200, "votew_t": 1200, "qcpre": 1200, "qcmil": 1200, "vote1h": 1200, "vote_t1h": 1200}
# phases an op may run ahead of its first consumer's earliest start (sched.schedule `hoist`)
HOIST = {"gfin": 50, "vsame": 250, "vsame_t": 250, "vsame8": 250, "vsame8_t": 250, "h2g": 250, "gmil": 250, "vote": 250, "vote_t": 250, "final": 50, "vote1": 250, "vote_t1": 250, "final1": 50, "votew": 250,
         "votew_t": 250, "qcpre": 250, "qcmil": 250, "vote1h": 250, "vote_t1h": 250}
STRETCH = {"gfin": 1.0, "vsame": 1.0, "vsame_t": 1.0, "vsame8": 1.0, "vsame8_t": 1.0, "h2g": 1.0, "gmil": 1.0, "final": 1.0, "vote": 1.0, "vote_t": 1.0, "vote1": 1.0, "vote_t1": 1.0, "final1": 1.0, "votew": 1.0,
           "votew_t": 1.0, "qcpre": 1.0, "qcmil": 1.0, "vote1h": 1.0, "vote_t1h": 1.0}
# priority weight of a heavy op against a light one (path length in weighted ops). r03 scan on
# the cost model (product phase 1.60 us, linear 0.69 us): vote 4 -> 64 estimates 3.29 -> 3.10 ms
# (a product on the path outweighs any run of light ops); vote_t keeps 2
HEAVY_W = {"vote": 48, "vote_t": 64, "vsame": 64, "vsame_t": 64, "vsame8": 128, "vsame8_t": 128, "h2g": 64}
# heavy-phase deferral (sched.schedule `defer`: h_thr, h_margin, l_thr) for the batch vote
# programs, whose cost is VALU per quad rather than phases: fuller product phases, more light ones
# (r06 offline sweep over h_thr, h_margin, l_thr, heavy_w, hoist; vote static VALU per quad
# 1.136 M -> 1.106 M, vote_t 1.104 M -> 1.097 M; the same-message per-vote programs vsame8
# 697 k -> 641 k per wave, vsame8_t 524 k -> 485 k)
DEFER = {"vote": (16, 1e4, 8), "vote_t": (16, 1e4, 8), "vsame8": (8, 1e4, 1), "vsame8_t": (8, 1e4, 1)}
# block families (sched.schedule `families`): fill a phase from the ops no costlier than its top
# op's first (vote 1.106 M -> 1.098 M, vote_t 1.097 M -> 1.093 M static; vsame8 gains nothing)
FAMILIES = {"vote", "vote_t"}
# list-scheduling priority offsets per program section (ir.Prog.section): the signature's
# decompression + subgroup check has no successor, so by path length alone it loses every
# contended phase to the Miller loop and ends up as a latency-bound tail; the offset runs it in
# the idle lanes of hash_to_G2 instead (vote 3,042 -> 2,985 phases). With the one-exponentiation
# square roots (r03) the vote program no longer needs it (estimate 3.12 -> 3.10 ms without),
# vote_t takes a larger one (3.05 -> 3.02 ms)
SEC_BIAS = {"vote_t": {"sig": 1500}}
# programs scheduled without light ops in the idle lanes of product phases (a phase that runs
# both interpreter blocks costs more than the two apart: r02aa, 997k -> 1,010k verifs/s). The
# standalone vote1 / vote_t1 (one wave on the GPU) once mixed (r02: 3,167 -> 2,454 phases, cost
# estimate -18%); r03z A/B on the per-call / small-batch programs, now without mixing (more
# phases, but no phase of a critical light op pays for a product): verify 4.10 -> 3.93 ms,
# sign 3.08 -> 3.00, QC 4.41 -> 4.33, config 5 5.8 -> 5.6 ms. The batch final keeps mixing (its
# slots would outgrow the LDS budget).
NOMIX = set(filter(None, os.environ.get(
    "OVH_GEN_NOMIX", "vote,vote_t,vote1,vote_t1,vote1h,vote_t1h,final1,qcpre,qcmil,votew,votew_t,signg0,signg1,"
    "sigchk,pkchk,pkgen,vsame,vsame_t,vsame8,vsame8_t,h2g,gmil,pkdec,g1grp").split(",")))
# r04: the batch vote programs keep at most SPILL_K values in LDS per phase; the rest wait in the
# vote's global scratch (sched.spill_pass: side-word spills / fills beside the lane ops), so a
# CU holds seven vote workgroups -- two pipelined batches' grids co-resident -- beside a final
# (ovhip.hip LDS budget). OVH_GEN_SPILL="vote=0,vote_t=0" builds them without spills.
SPILL_K = {"vote": 90, "vote_t": 90}
SPILL_K.update({k: int(v) for k, v in (x.split("=") for x in filter(None, os.environ.get("OVH_GEN_SPILL", "").split(",")))})
# slots: four vote workgroups (4 x 4 slices) and two finals must share a CU's 160 KiB of LDS
# (ovhip.hip static_assert); vote 159, final 226 slots with these settings


def build_all():
    consts = sched.ConstTable()
    consts.ref(1, True)      # entry 0: plain 1 (from-Montgomery product)
    assert consts.ref(0, False) - sched.CONST_BASE == KZERO   # the zero (selb's unused operands)
    # entries KTAB + n, n = 0..4: n (2p + 1) as raw limbs, the offset of a unit lin with n negated
    # terms (fpvm.hpp lin_sum: -x enters as ~x, and ~x + 2p + 1 = 2p - x mod 2^384)
    for n in range(5):
        assert consts.ref(n * (2 * P + 1), True) - sched.CONST_BASE == KTAB + n
    out = {}
    for name, (builder, ins, outs) in progs.PROGRAMS.items():
        prog = builder()
        prog.fuse()
        bias = {i: SEC_BIAS[name][op.sec] for i, op in enumerate(prog.ops)
                if name in SEC_BIAS and op.sec in SEC_BIAS[name]}
        sc = sched.schedule(prog, WIDTH[name], consts, max_slots=MAX_SLOTS.get(name, 256), heavy_w=HEAVY_W.get(name, 2),
                            hoist=HOIST.get(name), stretch=STRETCH.get(name, 1.3), mixed=name not in NOMIX,
                            bias=bias or None, spill_k=SPILL_K.get(name) or None, defer=DEFER.get(name),
                            families=name in FAMILIES)
        words = sched.encode(sc)
        out[name] = (prog, sc, words, ins, outs)
    return consts, out


def emit(consts, built, path):
    lines = ["// GENERATED by tools/fpvm/gen.py -- do not edit. Fp-VM programs for libovhip.", "#pragma once",
             "#include <stdint.h>", ""]
    cw = consts.words()
    lines.append("#define VM_NCONST %d" % len(cw))
    lines.append("#define VM_KZERO %d" % KZERO)
    lines.append("#define VM_KTAB %d" % KTAB)
    for k in ("S_U", "S_SIG", "S_TAU", "S_F", "S_RS", "S_TOTAL", "G_U", "G_H", "G_F", "G_PLANES"):
        lines.append("#define VM_%s %d" % (k, getattr(progs, k)))
    lines.append("static const uint32_t VM_CONST_WORDS[%d] = {" % (12 * len(cw)))
    for e in cw:
        lines.append("  " + ", ".join("0x%08x" % w for w in e) + ",")
    lines.append("};")
    for name, (prog, sc, words, ins, outs) in built.items():
        N = name.upper()
        st = sc.stats()
        lines.append("")
        lines.append("// %s: %s" % (name, json.dumps(st)))
        lines.append("#define VM_%s_W %d" % (N, sc.W))
        lines.append("#define VM_%s_NW %d" % (N, sched.words_per_lane(prog)))
        lines.append("#define VM_%s_NPHASES %d" % (N, sc.nrounds))
        lines.append("#define VM_%s_NSLOTS %d" % (N, sc.nslots))
        lines.append("#define VM_%s_NSCR %d" % (N, getattr(sc, "nscr", 0)))
        lines.append("#define VM_%s_NIN %d" % (N, len(ins)))
        lines.append("#define VM_%s_NOUT %d" % (N, len(outs)))
        slot_in = [sc.slot_of.get(prog.inputs[n], 0xFFFF) for n in ins]
        slot_out = [sc.slot_of[prog.outputs[n]] for n in outs]
        st = {prog.ops[v].name: prog.ops[v].imm for n, v in prog.outputs.items() if prog.ops[v].kind == "st"}
        if st:
            lines.append("// stored planes: %s" % json.dumps(st))
        lines.append("static const uint16_t VM_%s_IN[%d] = {%s};" % (N, len(ins), ", ".join(map(str, slot_in))))
        lines.append("static const uint16_t VM_%s_OUT[%d] = {%s};" % (N, len(outs), ", ".join(map(str, slot_out))))
        for kind, names in (("IN", ins), ("OUT", outs)):
            if names:
                lines.append("enum {" + ", ".join("VM_%s_%s_%s = %d" % (N, kind, n.upper(), k)
                                                  for k, n in enumerate(names)) + "};")
        lines.append("static const uint32_t VM_%s_CODE[%d] = {" % (N, len(words)))
        for k in range(0, len(words), 16):
            lines.append("  " + ",".join("0x%x" % w for w in words[k:k + 16]) + ",")
        lines.append("};")
        if getattr(sc, "nscr", 0):   # side words (spills / fills), nphases x W
            sw = sc.side_words
            lines.append("static const uint32_t VM_%s_SIDE[%d] = {" % (N, len(sw)))
            for k in range(0, len(sw), 16):
                lines.append("  " + ",".join("0x%x" % w for w in sw[k:k + 16]) + ",")
            lines.append("};")
    text = "\n".join(lines) + "\n"
    tmp = path + ".tmp"
    with open(tmp, "w") as fh:
        fh.write(text)
    os.replace(tmp, path)
    return hashlib.sha256(text.encode()).hexdigest()[:16]


# ----------------------------------------------------------------------------------- checks
def _oracle():
    sys.path.insert(0, os.path.join(ROOT, "oracle", "py"))
    import bls12_381 as bls
    return bls


RINV = pow(2 ** 384, P - 2, P)


def vote_inputs(bls, pkb, sigb, h):
    x = int.from_bytes(bytes([pkb[0] & 0x1F]) + pkb[1:48], "big")
    x1 = int.from_bytes(bytes([sigb[0] & 0x1F]) + sigb[1:48], "big")
    x0 = int.from_bytes(sigb[48:96], "big")
    (u00, u01), (u10, u11) = bls.hash_to_field_fp2(h, bls.DST_NUL, 2)
    return {"pk_x": x * RINV, "pk_sort": (pkb[0] >> 5) & 1, "sig_x0": x0 * RINV, "sig_x1": x1 * RINV,
            "sig_sort": (sigb[0] >> 5) & 1, "u00": u00, "u01": u01, "u10": u10, "u11": u11}


def check(built):
    bls = _oracle()
    with open(os.path.join(ROOT, "tests", "golden", "golden_v1.json")) as fh:
        g = json.load(fh)
    prog, sc, words, _, _ = built["vote"]
    r = 0xD7A1C3B5E9F20486
    parts = []
    for v, k in list(zip(g["votes"], g["keys"]))[:2]:
        pkb, sigb, h = bytes.fromhex(k["pk"]), bytes.fromhex(v["sig"]), bytes.fromhex(v["digest"])
        inp = vote_inputs(bls, pkb, sigb, h)
        vals = prog.evaluate(inp, r)
        ref = {n: vals[i] for n, i in prog.outputs.items()}
        sim = sched.simulate(sc, words, inp, r)
        assert sim == ref, "vote: simulated program differs from the DAG"
        ref = {(n[3:] if n.startswith("st:") else n): v for n, v in ref.items()}
        assert [ref[n] for n in ("pk_ok", "pk_grp", "sig_ok", "sig_grp", "h_inf")] == [1, 1, 1, 1, 0]
        pk = bls.g1_from_bytes(pkb)
        H = bls.hash_to_g2(h)
        f = progs.unflat12([ref["f%d" % j] for j in range(12)])
        rP = bls.pt_mul(bls.FpOps, pk, alg.rlc_scalar(r))
        assert bls.f12_eq(bls.final_exponentiation_x_chain(f),
                          bls.final_exponentiation_x_chain(bls.miller_loop(rP, H))), "vote: Miller output"
        # vote_t on the same vote with the key given as a projective point (Z = 7): same f up to
        # the final exponentiation, same r sigma
        tprog, tsc, twords, _, _ = built["vote_t"]
        tin = {k: inp[k] for k in ("sig_x0", "sig_x1", "sig_sort", "u00", "u01", "u10", "u11")}
        tin.update(pk_X=pk[0] * 7 % P, pk_Y=pk[1] * 7 % P, pk_Z=7)
        tvals = tprog.evaluate(tin, r)
        tref = {n: tvals[i] for n, i in tprog.outputs.items()}
        assert sched.simulate(tsc, twords, tin, r) == tref, "vote_t: simulated program differs from the DAG"
        tref = {(n[3:] if n.startswith("st:") else n): v for n, v in tref.items()}
        assert [tref[n] for n in ("sig_ok", "sig_grp", "h_inf")] == [1, 1, 0]
        tf = progs.unflat12([tref["f%d" % j] for j in range(12)])
        assert bls.f12_eq(bls.final_exponentiation_x_chain(tf), bls.final_exponentiation_x_chain(f)), "vote_t: f"
        qt = ["q%d" % j for j in range(4)] + ["t%d" % j for j in range(4)]
        assert [tref[n] for n in qt] == [ref[n] for n in qt], "vote_t: sigma / tau"
        sig = bls.g2_from_bytes(sigb)
        assert (ref["q0"], ref["q1"], ref["q2"], ref["q3"]) == (sig[0][0], sig[0][1], sig[1][0], sig[1][1]), "sigma"
        tau = bls.pt_neg(bls.Fp2Ops, bls.g2_psi(bls.g2_psi(sig)))
        assert (ref["t0"], ref["t1"], ref["t2"], ref["t3"]) == (tau[0][0], tau[0][1], tau[1][0], tau[1][1]), "tau"
        # rs: the vote's r sigma from the stored sigma / tau (bisection)
        rprog, rsc, rwords, _, _ = built["rs"]
        rin = {n: ref[n] for n in qt}
        rvals = rprog.evaluate(rin, r)
        rref = {n[3:]: rvals[i] for n, i in rprog.outputs.items()}
        assert sched.simulate(rsc, rwords, rin, r) == {"st:" + n: v for n, v in rref.items()}, "rs: simulated"
        rs_aff = _to_aff(bls, [rref["s%d" % j] for j in range(6)])
        assert rs_aff == bls.pt_mul(bls.Fp2Ops, sig, alg.rlc_scalar(r)), "rs: r sigma"
        parts.append(([ref["f%d" % j] for j in range(12)], [rref["s%d" % j] for j in range(6)], ref))
    # non-subgroup signature (golden case) must clear sig_grp
    bad = [c for c in g["verify"] if c["code"] == 3 and len(c["sig"]) == 192 and len(c["pk"]) == 96]
    if bad:
        c = bad[0]
        inp = vote_inputs(bls, bytes.fromhex(c["pk"]), bytes.fromhex(c["sig"]), bytes.fromhex(c["hash"]))
        vals = prog.evaluate(inp, r)
        ref = {n: vals[i] for n, i in prog.outputs.items()}
        assert ref["sig_ok"] == 1 and (ref["sig_grp"] == 0 or ref["pk_grp"] == 0), c["name"]
    # fold + final over the two valid votes (+ identity padding) -> ok == 1; broken -> 0
    one12 = [1] + [0] * 11
    inf6 = [0, 0, 1, 0, 0, 0]

    def final_inputs(items):
        inp = {}
        for k in range(progs.FOLD_K):
            F, S = items[k] if k < len(items) else (one12, inf6)
            for j in range(12):
                inp["F%d_%d" % (k, j)] = F[j]
            for j in range(6):
                inp["S%d_%d" % (k, j)] = S[j]
        return inp
    fprog, fsc, fwords, _, _ = built["final"]
    items = [(F, S) for F, S, _ in parts]
    inp = final_inputs(items)
    vals = fprog.evaluate(inp)
    ok = vals[fprog.outputs["ok"]]
    assert ok == 1, "final: valid batch rejected"
    assert sched.simulate(fsc, fwords, inp) == {"ok": 1}
    swapped = [(parts[0][0], parts[1][1]), (parts[1][0], parts[0][1])]
    inp = final_inputs(swapped)
    assert fprog.evaluate(inp)[fprog.outputs["ok"]] == 1  # sums/products commute
    broken = [(parts[0][0], parts[0][1]), (parts[1][0], parts[0][1])]
    inp = final_inputs(broken)
    assert fprog.evaluate(inp)[fprog.outputs["ok"]] == 0, "final: invalid batch accepted"
    # fold
    dprog, dsc, dwords, _, _ = built["fold"]
    inp = final_inputs(items)
    vals = dprog.evaluate(inp)
    assert sched.simulate(dsc, dwords, inp) == {n: vals[i] for n, i in dprog.outputs.items()}
    # bisection check of one vote: its own (f, r sigma) through the final program -> ok; the f of
    # one vote with the r sigma of the other -> not ok
    inp = final_inputs(items[:1])
    assert fprog.evaluate(inp)[fprog.outputs["ok"]] == 1
    assert sched.simulate(fsc, fwords, inp) == {"ok": 1}
    inp = final_inputs([(parts[0][0], parts[1][1])])
    assert fprog.evaluate(inp)[fprog.outputs["ok"]] == 0
    check_msm(built, bls, [bls.g2_from_bytes(bytes.fromhex(v["sig"])) for v in g["votes"][:3]])
    check_sigchk(built, bls, g)
    check_pk(built, bls, g)
    check_vote1(built, bls, g)
    check_votew(built, bls, g)
    check_qc_split(built, bls, g)
    check_vote1h(built, bls, g)
    check_pkgen(built, bls, g)
    check_signg(built, bls, g)
    check_samemsg(built, bls, g)
    print("fpvm check: vote/vote_t/rs/fold/final/MSM/sigchk/pkchk/g1padd programs match the oracle and their DAGs")


def check_samemsg(built, bls, g):
    """Same-message programs (ovhip.hip verify_samemsg_locked): vsame / vsame_t store the golden
    sigma, tau = -psi^2(sigma) and r pk (projective), h2g stores hash_to_G2(hash) (projective),
    gmil(r pk, H) has the final exponentiation of Miller(r pk, H) (the vote program's f); pkdec
    accepts golden keys and rejects the off-curve one."""
    r = 0xC2B2AE3D27D4EB4F
    for v, k in list(zip(g["votes"], g["keys"]))[:2]:
        pkb, sigb, h = bytes.fromhex(k["pk"]), bytes.fromhex(v["sig"]), bytes.fromhex(v["digest"])
        inp = vote_inputs(bls, pkb, sigb, h)
        prog, sc, words, ins, outs = built["vsame"]
        vin = {n: inp[n] for n in ins}
        vals = prog.evaluate(vin, r)
        got = {n: vals[i] for n, i in prog.outputs.items()}
        assert sched.simulate(sc, words, vin, r) == got, "vsame: simulated"
        assert [got[n] for n in outs] == [1, 1, 1, 1], "vsame: flags"
        sig = bls.g2_from_bytes(sigb)
        pk = bls.g1_from_bytes(pkb)
        assert (got["st:q0"], got["st:q1"], got["st:q2"], got["st:q3"]) == (sig[0][0], sig[0][1], sig[1][0], sig[1][1])
        tau = bls.pt_neg(bls.Fp2Ops, bls.g2_psi(bls.g2_psi(sig)))
        assert (got["st:t0"], got["st:t1"], got["st:t2"], got["st:t3"]) == (tau[0][0], tau[0][1], tau[1][0], tau[1][1])
        X, Y, Z = (got["st:r%d" % j] for j in range(3))
        zi = pow(Z, -1, P)
        rP = bls.pt_mul(bls.FpOps, pk, alg.rlc_scalar(r))
        assert (X * zi % P, Y * zi % P) == rP, "vsame: r pk"
        tprog, tsc, twords, tins, touts = built["vsame_t"]
        tin = {n: inp[n] for n in ("sig_x0", "sig_x1", "sig_sort")}
        tin.update(pk_X=pk[0] * 3 % P, pk_Y=pk[1] * 3 % P, pk_Z=3)
        tv = tprog.evaluate(tin, r)
        tgot = {n: tv[i] for n, i in tprog.outputs.items()}
        assert sched.simulate(tsc, twords, tin, r) == tgot, "vsame_t: simulated"
        Xt, Yt, Zt = (tgot["st:r%d" % j] for j in range(3))
        assert (Xt * pow(Zt, -1, P) % P, Yt * pow(Zt, -1, P) % P) == rP, "vsame_t: r pk"
        for nm, vi, want in (("vsame8", vin, got), ("vsame8_t", tin, tgot)):   # the 8-lane schedules
            _, sc8, w8, _, _ = built[nm]
            assert sched.simulate(sc8, w8, vi, r) == want, nm + ": simulated"
        hprog, hsc, hwords, hins, _ = built["h2g"]
        hin = {n: inp[n] for n in hins}
        hv = hprog.evaluate(hin)
        hgot = {n: hv[i] for n, i in hprog.outputs.items()}
        assert sched.simulate(hsc, hwords, hin) == hgot, "h2g: simulated"
        Hp = [hgot["st:h%d" % j] for j in range(6)]
        assert _to_aff(bls, Hp) == bls.hash_to_g2(h) and hgot["h_inf"] == 0, "h2g: H"
        mprog, msc, mwords, mins, _ = built["gmil"]
        minp = dict(zip(mins, [X, Y, Z] + Hp))
        mv = mprog.evaluate(minp)
        mgot = {n: mv[i] for n, i in mprog.outputs.items()}
        assert sched.simulate(msc, mwords, minp) == mgot, "gmil: simulated"
        f = progs.unflat12([mgot["st:f%d" % j] for j in range(12)])
        assert bls.f12_eq(bls.final_exponentiation_x_chain(f),
                          bls.final_exponentiation_x_chain(bls.miller_loop(rP, bls.hash_to_g2(h)))), "gmil: f"
        # gfin: F = 1, apk_0 = r pk, H_0, S = r sigma -> ok; S from another scalar -> not ok
        fprog, fsc, fwords, fins, _ = built["gfin"]
        rs = bls.pt_mul(bls.Fp2Ops, sig, alg.rlc_scalar(r))
        one12 = [1] + [0] * 11
        for S_, want in ((rs, 1), (bls.pt_mul(bls.Fp2Ops, sig, alg.rlc_scalar(r) + 1), 0)):
            finp = dict(zip(fins, one12 + [X, Y, Z] + Hp + _proj(S_)))
            assert fprog.evaluate(finp)[fprog.outputs["ok"]] == want, "gfin"
            if want:
                assert sched.simulate(fsc, fwords, finp) == {"ok": 1}, "gfin: simulated"
    dprog, dsc, dwords, dins, _ = built["pkdec"]
    named = {c["name"]: bytes.fromhex(c["pk"]) for c in g["verify"]}
    for pkb, ok in [(bytes.fromhex(k["pk"]), 1) for k in g["keys"][:2]] + [(named["pk_not_on_curve"], 0)]:
        din = {"pk_x": int.from_bytes(bytes([pkb[0] & 0x1F]) + pkb[1:48], "big") * RINV, "pk_sort": (pkb[0] >> 5) & 1}
        dv = dprog.evaluate(din)
        assert dv[dprog.outputs["pk_ok"]] == ok and sched.simulate(dsc, dwords, din) == {"pk_ok": ok}, "pkdec"


def check_sigchk(built, bls, g):
    """sigchk: decompressed sigma of valid signatures, sig_ok / sig_grp of the golden failures."""
    prog, sc, words, ins, outs = built["sigchk"]
    named = {c["name"]: bytes.fromhex(c["sig"]) for c in g["verify"]}
    cases = [(bytes.fromhex(v["sig"]), (1, 1)) for v in g["votes"][:2]]
    cases += [(named["sig_not_in_g2"], (1, 0)), (named["sig_not_on_curve"], (0, None))]
    for sigb, (ok, grp) in cases:
        x1 = int.from_bytes(bytes([sigb[0] & 0x1F]) + sigb[1:48], "big")
        inp = {"sig_x0": int.from_bytes(sigb[48:96], "big") * RINV, "sig_x1": x1 * RINV, "sig_sort": (sigb[0] >> 5) & 1}
        vals = prog.evaluate(inp)
        got = {n: vals[prog.outputs[n]] for n in outs}
        assert sched.simulate(sc, words, inp) == got, "sigchk: simulated"
        assert got["sig_ok"] == ok and (grp is None or got["sig_grp"] == grp), "sigchk: flags"
        if ok:
            q = bls.g2_from_bytes(sigb)
            assert (got["q0"], got["q1"], got["q2"], got["q3"]) == (q[0][0], q[0][1], q[1][0], q[1][1]), "sigchk: sigma"


def check_vote1(built, bls, g):
    """vote1 / vote_t1 + final1: a golden vote verifies, the same vote with another vote's
    signature does not."""
    prog, sc, words, _, _ = built["vote1"]
    tprog, tsc, twords, _, _ = built["vote_t1"]
    fprog, fsc, fwords, fins, _ = built["final1"]
    vs, ks = g["votes"][:2], g["keys"][:2]
    for sig_from, want in ((0, 1), (1, 0)):
        pkb, h = bytes.fromhex(ks[0]["pk"]), bytes.fromhex(vs[0]["digest"])
        inp = vote_inputs(bls, pkb, bytes.fromhex(vs[sig_from]["sig"]), h)
        vals = prog.evaluate(inp, 1)
        ref = {n: vals[i] for n, i in prog.outputs.items()}
        assert sched.simulate(sc, words, inp, 1) == ref, "vote1: simulated"
        F = [ref["st:f%d" % j] for j in range(12)]
        pk = bls.g1_from_bytes(pkb)
        tin = {k: inp[k] for k in ("sig_x0", "sig_x1", "sig_sort", "u00", "u01", "u10", "u11")}
        tin.update(pk_X=pk[0] * 5 % P, pk_Y=pk[1] * 5 % P, pk_Z=5)
        tvals = tprog.evaluate(tin, 1)
        tref = {n: tvals[i] for n, i in tprog.outputs.items()}
        assert sched.simulate(tsc, twords, tin, 1) == tref, "vote_t1: simulated"
        for FF in (F, [tref["st:f%d" % j] for j in range(12)]):
            fin = dict(zip(fins, FF))
            ok = fprog.evaluate(fin)[fprog.outputs["ok"]]
            assert ok == want and sched.simulate(fsc, fwords, fin) == {"ok": want}, "vote1 + final1"


def check_votew(built, bls, g):
    """votew / votew_t + final1 (small batches): FE(f_i) == 1 for a golden vote under a random
    RLC scalar, != 1 with another vote's signature; FE(f_0 f_1) == 1 for two valid votes with
    different scalars (the combined check)."""
    prog, sc, words, _, _ = built["votew"]
    tprog, tsc, twords, _, _ = built["votew_t"]
    fprog, fsc, fwords, fins, _ = built["final1"]
    vs, ks = g["votes"][:2], g["keys"][:2]
    fs = []
    for j, (vote, sig_from, want, r) in enumerate(((0, 0, 1, 0x9E3779B97F4A7C15), (0, 1, 0, 0x1234567890ABCDEF),
                                                    (1, 1, 1, 0xC2B2AE3D27D4EB4F))):
        pkb, h = bytes.fromhex(ks[vote]["pk"]), bytes.fromhex(vs[vote]["digest"])
        inp = vote_inputs(bls, pkb, bytes.fromhex(vs[sig_from]["sig"]), h)
        vals = prog.evaluate(inp, r)
        ref = {n: vals[i] for n, i in prog.outputs.items()}
        assert sched.simulate(sc, words, inp, r) == ref, "votew: simulated"
        F = [ref["st:f%d" % k] for k in range(12)]
        pk = bls.g1_from_bytes(pkb)
        tin = {k: inp[k] for k in ("sig_x0", "sig_x1", "sig_sort", "u00", "u01", "u10", "u11")}
        tin.update(pk_X=pk[0] * 7 % P, pk_Y=pk[1] * 7 % P, pk_Z=7)
        tvals = tprog.evaluate(tin, r)
        tref = {n: tvals[i] for n, i in tprog.outputs.items()}
        if j == 0:
            assert sched.simulate(tsc, twords, tin, r) == tref, "votew_t: simulated"
        for FF in (F, [tref["st:f%d" % k] for k in range(12)]):
            fin = dict(zip(fins, FF))
            ok = fprog.evaluate(fin)[fprog.outputs["ok"]]
            assert ok == want, "votew + final1"
        if j == 0:
            assert sched.simulate(fsc, fwords, dict(zip(fins, F))) == {"ok": 1}, "votew + final1: simulated"
        if want:
            fs.append(F)
    prod = bls.f12_mul(progs.unflat12(fs[0]), progs.unflat12(fs[1]))
    fin = dict(zip(fins, progs.flat12(prod)))
    assert fprog.evaluate(fin)[fprog.outputs["ok"]] == 1, "votew: combined check"


def check_qc_split(built, bls, g):
    """qcpre + qcmil + final1 (verify_aggregated_signature with the key tree beside): a golden vote
    verifies, the same with another vote's signature does not; the split's f equals vote_t1's."""
    pre, psc, pw, _, _ = built["qcpre"]
    mil, msc, mw, mins, _ = built["qcmil"]
    tprog = built["vote_t1"][0]
    fprog, fsc, fwords, fins, _ = built["final1"]
    vs, ks = g["votes"][:2], g["keys"][:2]
    for sig_from, want in ((0, 1), (1, 0)):
        pkb, h = bytes.fromhex(ks[0]["pk"]), bytes.fromhex(vs[0]["digest"])
        inp = vote_inputs(bls, pkb, bytes.fromhex(vs[sig_from]["sig"]), h)
        pin = {k: inp[k] for k in progs.QCPRE_IN}
        vals = pre.evaluate(pin)
        ref = {n: vals[i] for n, i in pre.outputs.items()}
        assert sched.simulate(psc, pw, pin) == ref, "qcpre: simulated"
        pk = bls.g1_from_bytes(pkb)
        min_ = dict(pk_X=pk[0] * 3 % P, pk_Y=pk[1] * 3 % P, pk_Z=3)
        min_.update({"h%d" % k: ref["st:h%d" % k] for k in range(6)})
        min_.update({"g%d" % k: ref["st:g%d" % k] for k in range(12)})
        mvals = mil.evaluate(min_)
        mref = {n: mvals[i] for n, i in mil.outputs.items()}
        assert sched.simulate(msc, mw, min_) == mref, "qcmil: simulated"
        F = [mref["st:f%d" % k] for k in range(12)]
        tin = {k: inp[k] for k in ("sig_x0", "sig_x1", "sig_sort", "u00", "u01", "u10", "u11")}
        tin.update(pk_X=min_["pk_X"], pk_Y=min_["pk_Y"], pk_Z=3)
        tv = tprog.evaluate(tin, 1)
        assert F == [tv[tprog.outputs["st:f%d" % k]] for k in range(12)], "qc split == vote_t1"
        fin = dict(zip(fins, F))
        assert fprog.evaluate(fin)[fprog.outputs["ok"]] == want, "qc split + final1"


def check_vote1h(built, bls, g):
    """The message cache: vote1's stored H fed to vote1h / vote_t1h gives vote1's f (a golden vote
    verifies through final1, the same hash with another vote's signature does not)."""
    prog = built["vote1"][0]
    hp, hsc, hw, _, _ = built["vote1h"]
    tp, tsc, tw, _, _ = built["vote_t1h"]
    fprog, _, _, fins, _ = built["final1"]
    vs, ks = g["votes"][:2], g["keys"][:2]
    for sig_from, want in ((0, 1), (1, 0)):
        pkb, h = bytes.fromhex(ks[0]["pk"]), bytes.fromhex(vs[0]["digest"])
        inp = vote_inputs(bls, pkb, bytes.fromhex(vs[sig_from]["sig"]), h)
        vals = prog.evaluate(inp, 1)
        ref = {n: vals[i] for n, i in prog.outputs.items()}
        hin = {k: inp[k] for k in ("pk_x", "pk_sort", "sig_x0", "sig_x1", "sig_sort")}
        hin.update({"h%d" % k: ref["st:h%d" % k] for k in range(6)})
        hv = hp.evaluate(hin, 1)
        href = {n: hv[i] for n, i in hp.outputs.items()}
        assert sched.simulate(hsc, hw, hin, 1) == href, "vote1h: simulated"
        F = [href["st:f%d" % k] for k in range(12)]
        assert F == [ref["st:f%d" % k] for k in range(12)], "vote1h == vote1"
        pk = bls.g1_from_bytes(pkb)
        tin = {k: hin[k] for k in hin if k not in ("pk_x", "pk_sort")}
        tin.update(pk_X=pk[0] * 5 % P, pk_Y=pk[1] * 5 % P, pk_Z=5)
        tv = tp.evaluate(tin, 1)
        tref = {n: tv[i] for n, i in tp.outputs.items()}
        if sig_from == 0:
            assert sched.simulate(tsc, tw, tin, 1) == tref, "vote_t1h: simulated"
        for FF in (F, [tref["st:f%d" % k] for k in range(12)]):
            assert fprog.evaluate(dict(zip(fins, FF)))[fprog.outputs["ok"]] == want, "vote1h + final1"


def check_pkgen(built, bls, g):
    """pkgen x 4 from the identity over a golden key's 64-bit chunks == the golden public key;
    the scalar 0 stays the identity."""
    prog, sc, words, ins, outs = built["pkgen"]
    for k in g["keys"][:2]:
        sk = int(k["sk"], 16)
        acc = [0, 1, 0]
        for j in (3, 2, 1, 0):
            ch = (sk >> (64 * j)) & (2 ** 64 - 1)
            inp = dict(zip(ins, acc))
            vals = prog.evaluate(inp, ch)
            got = {n: vals[i] for n, i in prog.outputs.items()}
            assert sched.simulate(sc, words, inp, ch) == got, "pkgen: simulated"
            acc = [got[n] for n in outs]
        X, Y, Z = acc
        zi = pow(Z, -1, P)
        assert (X * zi % P, Y * zi % P) == bls.g1_from_bytes(bytes.fromhex(k["pk"])), "pkgen: public key"
    vals = prog.evaluate(dict(zip(ins, [0, 1, 0])), 0)
    assert vals[prog.outputs["c2"]] == 0, "pkgen: [0] G1 is the identity"


def gls_digits(k):
    """k = sum d_i |x|^i, 0 <= d_i < |x| (k < r < |x|^4), as ovhip.hip k_vm_signg computes them."""
    x = alg.X_ABS
    k %= alg.R_ORDER
    d = []
    for _ in range(4):
        d.append(k % x)
        k //= x
    assert k == 0
    return d


def signg_scalar(d, j):
    """launch j's selb scalar: bit 4t + i = bit 48 - 16 j + t of digit i."""
    v = 0
    for t in range(16):
        for i in range(4):
            v |= ((d[i] >> (48 - 16 * j + t)) & 1) << (4 * t + i)
    return v


def check_signg(built, bls, g):
    """signg0 + 3 x signg1 over a golden key's GLS digits == the golden signature."""
    p0, s0, w0, _, _ = built["signg0"]
    p1, s1, w1, ins1, outs1 = built["signg1"]
    for k, v in list(zip(g["keys"], g["votes"]))[:2]:
        d = gls_digits(int(k["sk"], 16))
        (u00, u01), (u10, u11) = bls.hash_to_field_fp2(bytes.fromhex(v["digest"]), bls.DST_NUL, 2)
        inp = {"u00": u00, "u01": u01, "u10": u10, "u11": u11}
        sc = signg_scalar(d, 0)
        vals = p0.evaluate(inp, sc)
        got = {n: vals[i] for n, i in p0.outputs.items()}
        assert sched.simulate(s0, w0, inp, sc) == got, "signg0: simulated"
        acc = [got[n] for n in progs.SIGN_ACC]
        T = [got[n] for n in progs.SIGNG_T]
        for j in (1, 2, 3):
            inp = dict(zip(ins1, acc + T))
            sc = signg_scalar(d, j)
            vals = p1.evaluate(inp, sc)
            got = {n: vals[i] for n, i in p1.outputs.items()}
            if j == 1:
                assert sched.simulate(s1, w1, inp, sc) == got, "signg1: simulated"
            acc = [got[n] for n in outs1]
        assert _to_aff(bls, acc) == bls.g2_from_bytes(bytes.fromhex(v["sig"])), "signg: signature"


def check_pk(built, bls, g):
    """pkchk: decompressed key and flags of golden keys; g1padd against the oracle's G1 sums
    (identity operands and doubling included)."""
    prog, sc, words, ins, outs = built["pkchk"]
    named = {c["name"]: bytes.fromhex(c["pk"]) for c in g["verify"]}
    cases = [(bytes.fromhex(k["pk"]), (1, 1)) for k in g["keys"][:2]]
    cases += [(named["pk_not_in_g1"], (1, 0)), (named["pk_not_on_curve"], (0, None))]
    for pkb, (ok, grp) in cases:
        inp = {"pk_x": int.from_bytes(bytes([pkb[0] & 0x1F]) + pkb[1:48], "big") * RINV, "pk_sort": (pkb[0] >> 5) & 1}
        vals = prog.evaluate(inp)
        got = {n: vals[prog.outputs[n]] for n in outs}
        assert sched.simulate(sc, words, inp) == got, "pkchk: simulated"
        assert got["pk_ok"] == ok and (grp is None or got["pk_grp"] == grp), "pkchk: flags"
        if ok:
            assert (got["p0"], got["p1"]) == bls.g1_from_bytes(pkb), "pkchk: key"
    prog, sc, words, ins, outs = built["g1padd"]
    F = bls.FpOps
    A, B = (bls.g1_from_bytes(bytes.fromhex(k["pk"])) for k in g["keys"][:2])

    def proj(pt, z):
        return [0, 1, 0] if pt is None else [pt[0] * z % P, pt[1] * z % P, z]
    for X, Y in [(A, B), (A, A), (A, None), (None, B), (None, None), (A, bls.pt_neg(F, A))]:
        inp = dict(zip(ins, proj(X, 5) + proj(Y, 9)))
        vals = prog.evaluate(inp)
        got = [vals[prog.outputs[n]] for n in outs]
        assert sched.simulate(sc, words, inp) == dict(zip(outs, got)), "g1padd: simulated"
        want = bls.pt_add(F, X, Y)
        aff = None if got[2] == 0 else (got[0] * pow(got[2], P - 2, P) % P, got[1] * pow(got[2], P - 2, P) % P)
        assert aff == want, "g1padd"


def _to_aff(bls, v):
    """projective (X0, X1, Y0, Y1, Z0, Z1) -> oracle affine point (None = infinity)"""
    Z = (v[4], v[5])
    if bls.f2_is_zero(Z):
        return None
    zi = bls.f2_inv(Z)
    return (bls.f2_mul((v[0], v[1]), zi), bls.f2_mul((v[2], v[3]), zi))


def _proj(pt, z=(3, 5)):
    """oracle affine point -> projective limbs with a non-trivial Z (identity: (0 : 1 : 0))"""
    if pt is None:
        return [0, 0, 1, 0, 0, 0]
    X = ((pt[0][0] * z[0] - pt[0][1] * z[1]) % P, (pt[0][0] * z[1] + pt[0][1] * z[0]) % P)
    Y = ((pt[1][0] * z[0] - pt[1][1] * z[1]) % P, (pt[1][0] * z[1] + pt[1][1] * z[0]) % P)
    return [X[0], X[1], Y[0], Y[1], z[0], z[1]]


def check_msm(built, bls, pts):
    """madd / padd / hdbl<m> against the oracle's point arithmetic, identity operands and
    doubling cases (A == B) included."""
    F = bls.Fp2Ops
    A, B, C = pts
    cases = [(A, B), (A, A), (B, None), (None, C), (None, None), (A, bls.pt_neg(F, A))]
    for name, (prog, sc, words, ins, outs) in built.items():
        if name not in ("madd", "padd") and not name.startswith("hdbl"):
            continue
        m = int(name[4:]) if name.startswith("hdbl") else 0
        for X, Y in cases:
            if name == "madd" and X is None:
                continue   # the affine operand is never the identity
            inp = {}
            xa = [X[0][0], X[0][1], X[1][0], X[1][1]] if name == "madd" else _proj(X, (7, 2))
            for n, v in zip(ins, xa + _proj(Y)):
                inp[n] = v
            vals = prog.evaluate(inp)
            got = [vals[prog.outputs[n]] for n in outs]
            assert sched.simulate(sc, words, inp) == dict(zip(outs, got)), name + ": simulated"
            want = bls.pt_add(F, X, bls.pt_mul(F, Y, 1 << m) if (Y is not None and m) else Y)
            assert _to_aff(bls, got) == want, name


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=os.path.join(ROOT, "consensus_overlord_amd", "csrc", "vm_progs.inc"))
    ap.add_argument("--check", action="store_true")
    args = ap.parse_args()
    consts, built = build_all()
    for name, (prog, sc, words, _, _) in built.items():
        print(name, json.dumps(sc.stats()))
    if args.check:
        check(built)
    h = emit(consts, built, args.out)
    print("wrote", args.out, h)
    write_workmodel(built)


def write_workmodel(built):
    """consensus_overlord_amd/workmodel.json: Montgomery products (M) per unit of each batch
    stage = the heavy ops of its VM program (one M each); bench.py prices the roofline with it."""
    path = os.path.join(ROOT, "consensus_overlord_amd", "workmodel.json")
    with open(path) as fh:
        wm = json.load(fh)
    st = {name: built[name][1].stats() for name in built}
    wm["M_per_unit"].update({
        "vote": st["vote"]["heavy_ops"],
        "vote_t": st["vote_t"]["heavy_ops"],
        "msm_madd": st["madd"]["heavy_ops"],
        "msm_padd": st["padd"]["heavy_ops"],
        "rs_bisect": st["rs"]["heavy_ops"],
        "fold_per_partial": st["fold"]["heavy_ops"] / 4.0,
        "final_per_batch": st["final"]["heavy_ops"],
        "fallback": st["final"]["heavy_ops"],
    })
    wm["vm_programs"] = st
    with open(path, "w") as fh:
        json.dump(wm, fh, indent=1)


if __name__ == "__main__":
    main()
