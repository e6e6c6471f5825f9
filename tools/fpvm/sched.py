"""Schedule a traced Fp-VM program (ir.Prog) onto W lanes, allocate LDS slots, encode the
per-lane instruction stream, and re-execute the encoded stream slot by slot (simulate) to
prove scheduling + allocation preserve the program's values.

Phase semantics (the interpreter, consensus_overlord_amd/csrc/fpvm.hpp): in phase t every lane
of a slice reads its operands from LDS slots / the constant table, computes one op and writes
one slot; results are visible from phase t + 1. A slot whose value was last read in phase t can
be rewritten from phase t + 1 on.

Instruction (4 x uint32 per lane per phase):
  w0 = opcode | dst << 5 (11 bits) | imm << 16 (6 bits) | phase header << 22 (the same in every
       lane: which interpreter blocks the phase needs, phase_bits)
  w1 = A | B << 16,  w2 = C | D << 16
  w3 = ca | cb << 5 | cc << 10 | cd << 15   (5-bit two's-complement coefficients)
       (sop: z = A C + cb B D)
       | k << 20 (lin: k * (unit sum) when 2 <= k <= 15, ir.lin_form "scaled")
  operand: slot index (< CONST_BASE) or CONST_BASE + k (constant table entry k); a missing
  operand is the zero constant with coefficient 0, so every lane loads four operands.
"""
from __future__ import annotations

import bisect
import heapq
import os
from collections import defaultdict

from ir import CMAX, HALF_P, HEAVY, P, lin_form

OPC = {"nop": 0, "muls": 1, "sgn0": 2, "lex": 3, "inv": 4, "lin": 5, "sel": 6, "eq": 7, "and": 8, "or": 9,
       "xor": 10, "st": 11, "selb": 12, "sop": 13, "spill": 14, "fill": 15}
CONST_BASE = 0x800
ABSENT = 0xFFFF
# ops the interpreter runs through the Montgomery product (x = A + cb B, y = C + cd D)
PRODUCTS = ("muls", "sgn0", "lex", "eq")
# LDS pass width (lanes) and slot residues that share banks (OVH_BANK="lanes,mod" for A/B builds)
BANK_LANES, BANK_MOD = (int(x) for x in os.environ.get("OVH_BANK", "16,16").split(","))
# passes of the bank-conflict local search over the slot assignment (improve_banks; 0 = off)
BANK_PASSES = int(os.environ.get("OVH_BANK_PASSES", "3"))
# result-store banking (ds_write_b128: 8-lane groups, residue mod 8) in the slot choice and the
# local search; OVH_WBANK=0 models the reads alone (the r05 model)
WBANK = os.environ.get("OVH_WBANK", "1") == "1"
WBANK_LANES, WBANK_MOD = 8, 8
# every lin op in the general-coefficient form (fpvm.hpp lin_mad): one linear block per phase
# instead of the unit-sign block plus the general one; measured faster even for unit sums with
# negations (r02aj: 1,013k -> 1,031-1,038k verifs/s). OVH_GEN_UNITLIN=1 with an interpreter
# built with OVH_VM_UNIT_LIN restores the unit-sign path (A/B builds).
ALL_ACC = os.environ.get("OVH_GEN_UNITLIN", "0") != "1"
# r03: per phase -- a linear phase whose lin ops are all unit sums (or k x a unit sum) runs the
# cheaper unit block (add chains + one small-scalar reduction, fpvm.hpp lin_sum / scale_reduce),
# any other linear phase runs every lin op in the general block (unit sums encoded with the
# FORCE_ACC bit). 0 restores ALL_ACC's one-block-per-phase rule in every phase.
PHASE_UNIT = os.environ.get("OVH_GEN_PHASE_UNIT", "1") == "1"
FORCE_ACC = 1 << 24   # w3 bit: run this lin op in the general-coefficient block
R_MONT = pow(2, 384, P)


class ConstTable:
    """Constants shared by every program: (value, raw) -> index. raw constants are stored as
    plain limbs; the others in Montgomery form (value * 2^384 mod p)."""

    def __init__(self):
        self.index = {}
        self.entries = []

    def ref(self, value, raw):
        key = (value, bool(raw))
        if key not in self.index:
            self.index[key] = len(self.entries)
            self.entries.append(key)
        return CONST_BASE + self.index[key]

    def words(self):
        out = []
        for value, raw in self.entries:
            v = value if raw else value * R_MONT % P
            out.append([(v >> (32 * k)) & 0xFFFFFFFF for k in range(12)])
        return out


class Scheduled:
    def __init__(self, prog, W, rounds, slot_of, nslots, consts):
        self.prog = prog
        self.W = W
        self.rounds = rounds          # list of list of op ids (len <= W)
        self.slot_of = slot_of        # value id -> slot
        self.nslots = nslots
        self.consts = consts

    @property
    def nrounds(self):
        return len(self.rounds)

    def stats(self):
        heavy_rounds = sum(1 for k in self.kinds if k == "H")
        nheavy = sum(1 for r in self.rounds for i in r if self.prog.ops[i].kind in HEAVY)
        nlight = sum(1 for r in self.rounds for i in r if self.prog.ops[i].kind not in HEAVY and
                     self.prog.ops[i].kind not in SIDE)
        return {"phases": self.nrounds, "heavy_phases": heavy_rounds, "light_phases": self.nrounds - heavy_rounds,
                "heavy_ops": nheavy, "light_ops": nlight, "slots": self.nslots, "W": self.W,
                "lane_util_heavy": round(nheavy / max(1, heavy_rounds * self.W), 3),
                "cost_est": heavy_rounds * 900 + (self.nrounds - heavy_rounds) * 150,
                **({"scratch": self.nscr, "spills": self.nspill, "fills": self.nfill} if getattr(self, "nscr", 0) else {})}


def schedule(prog, W, consts: ConstTable, max_slots=None, heavy_w=10, light_w=1, mixed=True, slot_target=None,
             hoist=None, stretch=1.3, split_sop=False, dual=False, bias=None, light_margin=0, spill_k=None,
             defer=None, families=False):
    ops = prog.ops
    live = prog.live_ops()
    liveset = set(live)
    pre = {i for i in live if ops[i].kind in ("in", "const")}
    work = [i for i in live if i not in pre]
    preds = {}
    succs = defaultdict(list)
    for i in work:
        ps = {s for s in ops[i].srcs if s is not None and s not in pre}
        ps |= {s for s in ops[i].deps if s in liveset and s not in pre}   # ordering-only edges
        preds[i] = ps
        for s in ps:
            succs[s].append(i)
    prio = {}
    for i in reversed(work):
        c = heavy_w if ops[i].kind in HEAVY else light_w
        prio[i] = c + max((prio[s] for s in succs[i]), default=0)
        if ops[i].kind == "st":
            prio[i] = 10 ** 6   # stores free their slot: run them as soon as they are ready
    if bias is not None:   # per-op priority offsets (staggering the units of a merged program)
        for i in work:
            if ops[i].kind != "st":
                prio[i] += bias.get(i, 0)
    # release phase: an op may not run more than `hoist` phases before the earliest phase its
    # first consumer could run (ASAP depth x the schedule's expected stretch), so values that
    # are ready early but needed late (the per-step addends of a scalar-multiplication chain)
    # do not hold slots for hundreds of phases
    asap = {}
    for i in work:
        asap[i] = 1 + max((asap[p_] for p_ in preds[i]), default=0)
    release = {}
    for i in work:
        use = min((asap[c] for c in succs[i]), default=asap[i])
        release[i] = max(0, int(stretch * use) - hoist) if hoist is not None else 0
    indeg = {i: len(preds[i]) for i in work}
    # remaining consumers of each slot value (inputs included), for register-pressure control
    remaining = defaultdict(int)
    for i in work:
        for s_ in set(x for x in ops[i].srcs if x is not None and ops[x].kind != "const"):
            remaining[s_] += 1
    outset = set(v for v in prog.outputs.values() if ops[v].kind != "st")
    live_now = sum(1 for i in pre if ops[i].kind == "in")
    ready_h, ready_l = [], []
    for i in work:
        if indeg[i] == 0:
            (ready_h if ops[i].kind in HEAVY else ready_l).append(i)

    def delta(i):
        d = 0 if ops[i].kind == "st" else 1
        for s_ in set(x for x in ops[i].srcs if x is not None and ops[x].kind != "const"):
            if remaining[s_] == 1 and s_ not in outset:
                d -= 1
        return d

    def pick(cands, n, pressure):
        if not cands or n <= 0:
            return []
        if families and not pressure:
            cands.sort(key=lambda i: -prio[i])
            top = fam[cands[0]]
            take = [i for i in cands if fam[i] <= top][:n]
            if len(take) < n and families != "strict":
                ts = set(take)
                take += [i for i in cands if i not in ts][:n - len(take)]
            ts = set(take)
            cands[:] = [i for i in cands if i not in ts]
            return take
        if pressure:
            cands.sort(key=lambda i: (delta(i), -prio[i]))
            take = cands[:n]
            del cands[:n]
            return take
        cands.sort(key=lambda i: -prio[i])
        take = cands[:n]
        del cands[:n]
        return take
    # heavy-phase deferral (defer = (h_thr, h_margin, l_thr)): while fewer than h_thr products are
    # ready and at least l_thr light ops are, run a light phase unless the top product leads the
    # top light op by h_margin or more -- the products accumulate into fuller phases. r06, vote
    # (16, 1e4, 6): 1,375 -> 1,289 product phases (lane use 0.833 -> 0.888), 1,307 -> 1,460 light
    # phases, 1,281 -> 299 spills; static VALU per quad 1.136 M -> 1.106 M (tools/valu_attr.py)
    h_thr, h_margin, l_thr = defer if defer is not None else (0, 0, 1)
    # families (r06): the interpreter's wave-uniform blocks cost by the costliest lane of a phase --
    # a product with a negated operand (pre_add2's 2p - D chain, 51 VALU against 24), a unit lin
    # with a negated term (lin_sum 94 against 37), a general-coefficient lin (lin_mad: every lin
    # of its phase) -- so a phase is filled from the ops no costlier than its top op's first
    fam = {}
    if families:
        for i in work:
            k = ops[i].kind
            if k in PRODUCTS:
                cf = lane_operands(prog, i)[4]
                fam[i] = 1 if (k == "eq" or cf[1] < 0 or cf[3] < 0) else 0
            elif k == "lin":
                form = lin_form(prog._lin_terms(ops[i]), prog.lin_width)
                # unit: the number of negated terms (lin_sum XORs that many positions), general: 4
                fam[i] = 2 if form[0] == "acc" else (1 if any(c < 0 for c, _ in form[-1]) else 0)
            else:
                fam[i] = 0
    rounds = []
    kinds = []
    done = 0
    while done < len(work):
        t = len(rounds)
        pressure = slot_target is not None and live_now >= slot_target
        # ops past their release phase are eligible; the rest wait (unless nothing is eligible)
        eh = [i for i in ready_h if release[i] <= t]
        el = [i for i in ready_l if release[i] <= t]
        if not eh and not el:
            eh, el = list(ready_h), list(ready_l)
        wait_h = [i for i in ready_h if i not in set(eh)]
        wait_l = [i for i in ready_l if i not in set(el)]
        top_h = max((prio[i] for i in eh), default=-1)
        top_l = max((prio[i] for i in el), default=-1)
        if dual:   # every lane runs one heavy and one light op per phase
            kind = "H" if eh else "L"
            cur = pick(eh, W, pressure) + pick(el, W, pressure)
        elif (top_l > top_h + light_margin or not eh or
              (len(el) >= l_thr and len(eh) < h_thr and top_h < top_l + h_margin)):
            kind = "L"
            cur = pick(el, W, pressure)
        else:
            kind = "H"
            if split_sop:   # a phase runs sops or products, never both (the wave would pay for both)
                fam = max(eh, key=lambda i: prio[i])
                fam = ops[fam].kind == "sop"
                same = [i for i in eh if (ops[i].kind == "sop") == fam]
                other = [i for i in eh if (ops[i].kind == "sop") != fam]
                cur = pick(same, W, pressure)
                eh = same + other
            else:
                cur = pick(eh, W, pressure)
            if mixed:
                cur += pick(el, W - len(cur), pressure)
        ready_h[:] = eh + wait_h
        ready_l[:] = el + wait_l
        if not cur:
            raise RuntimeError("deadlock in scheduler")
        rounds.append(cur)
        kinds.append(kind)
        done += len(cur)
        for i in cur:
            live_now += delta(i)
            for s_ in set(x for x in ops[i].srcs if x is not None and ops[x].kind != "const"):
                remaining[s_] -= 1
            for s_ in succs[i]:
                indeg[s_] -= 1
                if indeg[s_] == 0:
                    (ready_h if ops[s_].kind in HEAVY else ready_l).append(s_)
    nscr = nspill = nfill = 0
    if spill_k is not None:   # at most spill_k values in LDS per phase (spill_pass)
        nscr, nspill, nfill = spill_pass(prog, rounds, W, spill_k)
    # ---- slot allocation
    def_round = {i: -1 for i in pre if ops[i].kind == "in"}
    for t, r in enumerate(rounds):
        for i in r:
            def_round[i] = t
    last_use = defaultdict(lambda: -1)
    for t, r in enumerate(rounds):
        for i in r:
            for s in ops[i].srcs:
                if s is not None and ops[s].kind != "const":
                    last_use[s] = max(last_use[s], t)
    end = len(rounds)
    for v in prog.outputs.values():
        if ops[v].kind != "st":
            last_use[v] = end
    slot_of = {}
    free = []
    nslots = 0
    frees_at = defaultdict(list)   # round -> slots that become free at that round
    # LDS bank spreading: a ds_read_b128 / ds_write_b128 serves BANK_LANES lanes per pass, and two
    # lanes of a pass that touch different addresses with the same 16-byte chunk residue hit the
    # same banks. Slot regions are 128-byte aligned (ovhip.hip), so slot s and constant c sit in
    # residues 3 s and 3 c (mod 8): equal iff s = c (mod BANK_MOD). Among the free slots a value
    # gets the one whose residue the fewest distinct addresses use in the same instruction (phase,
    # operand position, lane pass) where it is read or written; the slot count is unchanged (a
    # new slot only when none is free).
    for i in pre:
        if ops[i].kind == "const":
            consts.ref(ops[i].imm, ops[i].name == "raw")
    zero_c = consts.ref(0, False) - CONST_BASE
    lane_of = {}
    reads = defaultdict(set)
    use = defaultdict(lambda: [0] * BANK_MOD)
    seen_c = set()
    for t, r in enumerate(rounds):
        for k, i in enumerate(x for x in r if ops[x].kind not in SIDE):
            lane_of[i] = k
            g = k // BANK_LANES
            A, B, C, D = lane_operands(prog, i)[:4]
            refs = [(0, B), (0, C)] if ops[i].kind == "selb" else list(enumerate((A, B, C, D)))
            for pos, v in refs:
                if v is not None and ops[v].kind != "const":
                    reads[v].add((t, g, pos))
                    continue
                c = zero_c if v is None else consts.ref(ops[v].imm, ops[v].name == "raw") - CONST_BASE
                if (t, g, pos, c) not in seen_c:
                    seen_c.add((t, g, pos, c))
                    use[(t, g, pos)][c % BANK_MOD] += 1

    # result stores: ds_write_b128 serves 8 contiguous lanes per pass over 32 banks, so the
    # destination slots of lanes 8g .. 8g + 7 of a phase want distinct residues mod 8 (r06: the
    # reads alone were modelled, and PMC put 36.5% of the LDS cycles in bank conflicts)
    wuse = defaultdict(lambda: [0] * WBANK_MOD)

    def alloc(v):
        nonlocal nslots
        ev = [use[e] for e in reads[v]]
        wv = wuse[(def_round[v], lane_of[v] // WBANK_LANES)] if (v in lane_of and WBANK) else None
        if free:
            best = min(free, key=lambda x: (sum(u[x % BANK_MOD] for u in ev) +
                                            (wv[x % WBANK_MOD] if wv is not None else 0), x))
            free.remove(best)
            s = best
        else:
            s = nslots
            nslots += 1
        for u in ev:
            u[s % BANK_MOD] += 1
        if wv is not None:
            wv[s % WBANK_MOD] += 1
        slot_of[v] = s
        lu = last_use[v]
        if lu < 0:   # never read (dead write): free right after
            lu = def_round[v]
        frees_at[lu + 1].append(s)
    for name in sorted(prog.inputs):
        v = prog.inputs[name]
        if v in liveset:
            alloc(v)
    for t, r in enumerate(rounds):
        free.extend(frees_at.pop(t, []))
        for i in r:
            if ops[i].kind not in ("st", "spill"):
                alloc(i)
    if max_slots is not None and nslots > max_slots:
        raise RuntimeError("%s: %d slots > %d" % (prog.name, nslots, max_slots))
    if BANK_PASSES and W == BANK_LANES:
        improve_banks(prog, rounds, slot_of, def_round, last_use, nslots, consts, BANK_PASSES,
                      lane_of if WBANK else None)
    for i in pre:
        if ops[i].kind == "const":
            consts.ref(ops[i].imm, ops[i].name == "raw")
    sc = Scheduled(prog, W, rounds, slot_of, nslots, consts)
    sc.kinds = kinds
    sc.nscr, sc.nspill, sc.nfill = nscr, nspill, nfill
    return sc


def improve_banks(prog, rounds, slot_of, def_round, last_use, nslots, consts, passes, lane_of=None):
    """Local search over the slot assignment against the ds_read_b128 bank model (the whole
    W-lane phase is one lane group; slot s and constant c hit bank group s, c mod BANK_MOD):
    a read costs max over residues of the distinct addresses with that residue, minus one, in
    extra LDS cycles. A value moves to a slot that is free over its whole lifetime [def, last
    use] when that lowers the summed cost of the reads it takes part in. The slot count does not
    change."""
    import bisect
    ops = prog.ops
    zero_c = consts.ref(0, False) - CONST_BASE
    ctx = defaultdict(list)        # (t, pos) -> operand keys ('v', id) / ('c', index)
    reads_of = defaultdict(set)    # value -> contexts it is read in
    for t, r in enumerate(rounds):
        for i in r:
            if ops[i].kind in SIDE:
                continue
            A, B, C, D = lane_operands(prog, i)[:4]
            refs = [(1, B), (2, C)] if ops[i].kind == "selb" else list(enumerate((A, B, C, D)))
            for pos, v in refs:
                if v is not None and ops[v].kind != "const":
                    key = ("v", v)
                    reads_of[v].add((t, pos))
                else:
                    c = zero_c if v is None else consts.ref(ops[v].imm, ops[v].name == "raw") - CONST_BASE
                    key = ("c", c)
                if key not in ctx[(t, pos)]:
                    ctx[(t, pos)].append(key)
    # result stores (lane_of given): the destination slots of each 8-lane store group
    if lane_of is not None:
        for v, k in lane_of.items():
            if v in slot_of and ops[v].kind not in ("st", "spill"):
                c = (def_round[v], "w", k // WBANK_LANES)
                ctx[c].append(("v", v))
                reads_of[v].add(c)

    def res(key, moved=None, r=None):
        if key[0] == "c":
            return key[1] % BANK_MOD
        if key[1] == moved:
            return r
        return slot_of[key[1]] % BANK_MOD

    def cost(c, moved=None, r=None):
        if c[1] == "w":   # a store group: residues mod WBANK_MOD (r: a residue mod BANK_MOD)
            cnt = [0] * WBANK_MOD
            for key in ctx[c]:
                cnt[res(key, moved, r) % WBANK_MOD] += 1
            return max(cnt) - 1
        cnt = [0] * BANK_MOD
        for key in ctx[c]:
            cnt[res(key, moved, r)] += 1
        return max(cnt) - 1
    # occupancy: per slot the sorted lifetimes of its values
    occ = defaultdict(list)
    for v, sl in slot_of.items():
        occ[sl].append((def_round.get(v, -1), max(last_use[v], def_round.get(v, -1)), v))
    for sl in occ:
        occ[sl].sort()

    def free_over(sl, lo, hi, v):
        lst = occ[sl]
        k = bisect.bisect_left(lst, (lo, -10 ** 9, -1))
        for j in (k - 1, k):
            if 0 <= j < len(lst):
                a, b, u = lst[j]
                if u != v and not (b < lo or a > hi):
                    return False
        return True
    total = sum(cost(c) for c in ctx)
    for _ in range(passes):
        moved_any = 0
        order = sorted(reads_of, key=lambda v: -sum(cost(c) for c in reads_of[v]))
        for v in order:
            cur = slot_of[v]
            base = sum(cost(c) for c in reads_of[v])
            if base == 0:
                continue
            lo, hi = def_round.get(v, -1), max(last_use[v], def_round.get(v, -1))
            best = None
            for r in sorted(range(BANK_MOD), key=lambda r: sum(cost(c, v, r) for c in reads_of[v])):
                gain = base - sum(cost(c, v, r) for c in reads_of[v])
                if gain <= 0:
                    break
                for sl in range(r, nslots, BANK_MOD):
                    if sl != cur and free_over(sl, lo, hi, v):
                        best = (sl, gain)
                        break
                if best:
                    break
            if best:
                sl, gain = best
                occ[cur] = [x for x in occ[cur] if x[2] != v]
                bisect.insort(occ[sl], (lo, hi, v))
                slot_of[v] = sl
                total -= gain
                moved_any += 1
        if not moved_any:
            break
    return total


def _operand(sc, v):
    if v is None:
        return sc.consts.ref(0, False)
    op = sc.prog.ops[v]
    if op.kind == "const":
        return sc.consts.ref(op.imm, op.name == "raw")
    return sc.slot_of[v]


def _c5(c):
    assert -16 <= c <= 15
    return c & 31


def words_per_lane(prog):
    """Instruction words per lane per phase (16 bytes). The 32-byte format with eight-operand
    lin ops (lin_width 8) was measured slower and the interpreter no longer decodes it."""
    if prog.lin_width != 4:
        raise ValueError("%s: the interpreter runs 4-operand lin ops only" % prog.name)
    return 4


def lane_operands(prog, i, unit=False):
    """(A, B, C, D, coefs, scale) of op i as the interpreter reads them (value ids or None:
    None is the zero constant; C of sgn0 / lex / eq / inv is a fixed constant, see encode).
    unit: a unit / scaled lin keeps its scale for the unit block (else coefficients x scale)."""
    ops = prog.ops
    LW = prog.lin_width
    op = ops[i]
    k = op.kind
    s = list(op.srcs) + [None] * (LW - len(op.srcs))
    coefs = [0] * LW
    ext = [None] * 4          # operands E..H (wide programs)
    scale = 0
    if k == "lin":
        form = lin_form(prog._lin_terms(op), LW)
        if form[0] == "acc":
            srcs = list(op.srcs) + [None] * (LW - len(op.srcs))
            coefs = list(op.coefs) + [0] * (LW - len(op.coefs))
        else:
            # r06: negated terms in the last positions (D, then C, then B), so a phase whose lanes
            # negate at most one or two terms needs no XOR of B / C (phase_bits H_LINNEG2 / 3)
            pos_ = [t for t in form[-1] if t[0] > 0]
            neg_ = [t for t in form[-1] if t[0] < 0]
            u = pos_ + [(0, None)] * (LW - len(pos_) - len(neg_)) + neg_
            srcs = [v for _, v in u]
            coefs = [c for c, _ in u]
            if form[0] == "scaled":
                scale = form[1]
                if ALL_ACC and not unit:
                    coefs = [c * scale for c in coefs]
                    scale = 0
        A, B, C, D = srcs[:4]
        if LW == 8:
            ext = srcs[4:8]
    elif k == "eq":            # (A - B) * plain 1, flag: zero (fpvm.hpp exec)
        assert tuple(op.coefs[:4]) == (1, 0, 1, 0) and s[1] is None and s[3] is None, op.coefs
        A, B, C, D = s[0], s[2], None, None
        coefs[:4] = [1, -1, 1, 0]
    elif k == "muls":
        A, B, C, D = s[:4]
        coefs[:4] = list(op.coefs[:4])
        for h in (0, 2):
            terms = [(c, v) for c, v in zip(op.coefs[h:h + 2], s[h:h + 2]) if v is not None and c]
            form = lin_form(terms, 2)
            assert form[0] == "unit", (k, op.coefs)   # the interpreter's muls operands are unit sums
            u = form[1] + [(0, None)] * (2 - len(form[1]))
            if h == 0:
                A, B = u[0][1], u[1][1]
            else:
                C, D = u[0][1], u[1][1]
            coefs[h], coefs[h + 1] = u[0][0], u[1][0]
        if coefs[1] < 0:
            # r06: the negated operand on y = C + cd D (fpvm.hpp pre_add2 has no x negation
            # chain); x y is symmetric and both operands stay below 4p. No program negates both
            assert coefs[3] >= 0, ("%s: both product operands negated" % prog.name, op.coefs)
            A, B, C, D = C, D, A, B
            coefs[:4] = [coefs[2], coefs[3], coefs[0], coefs[1]]
    elif k == "sop":           # A C + cb B D
        A, B, C, D = s[:4]
        coefs[:4] = list(op.coefs[:4])
    elif k in ("sgn0", "lex"):
        A, B, C, D = s[0], None, None, None
        coefs[:4] = [1, 0, 1, 0]
    elif k in ("inv", "st", "spill"):
        A, B, C, D = s[0], None, None, None
        coefs[:4] = [1, 0, 0, 0]
    elif k == "fill":
        A, B, C, D = None, None, None, None
    elif k == "sel":           # A = flag, B = x, C = y
        A, B, C, D = s[0], s[1], s[2], None
    elif k == "selb":          # B = x, C = y
        A, B, C, D = None, s[0], s[1], None
    elif k in ("and", "or", "xor"):
        A, B, C, D = s[0], None, s[1], None
    else:
        raise ValueError(k)
    return A, B, C, D, coefs, scale


def encode(sc):
    """-> list of uint32 words, nphases * W * words_per_lane."""
    words = []
    ops = sc.prog.ops
    nw = words_per_lane(sc.prog)
    LW = sc.prog.lin_width
    sc.side_words = []
    for r in sc.rounds:
        sides = [i for i in r if ops[i].kind in SIDE]
        r = [i for i in r if ops[i].kind not in SIDE]
        assert len(r) <= sc.W and len(sides) <= sc.W
        # side word per lane: bit 31 valid, bit 30 fill (else spill), bits 0..10 the slot,
        # bits 11..22 the scratch entry (fpvm.hpp run)
        sw = [0] * sc.W
        for k, i in enumerate(sides):
            v = i if ops[i].kind == "fill" else ops[i].srcs[0]
            # the fields' widths (fpvm.hpp side_spill / run masks 0x7FF, 0xFFF): a wider slot or
            # scratch entry would alias another one on the device
            assert sc.slot_of[v] < 1 << 11, ("side word slot", sc.slot_of[v])
            assert 0 <= ops[i].imm < 1 << 12, ("side word scratch entry", ops[i].imm)
            sw[k] = 1 << 31 | (ops[i].kind == "fill") << 30 | sc.slot_of[v] | ops[i].imm << 11
            assert sc.slot_of[v] < 2048 and ops[i].imm < 4096
        sc.side_words += sw
        lanes = list(r) + [None] * (sc.W - len(r))
        first = len(words)
        # unit block for this phase's lin ops only when every one of them is a unit sum
        unit = PHASE_UNIT and ALL_ACC and all(
            lin_form(sc.prog._lin_terms(ops[i]), LW)[0] in ("unit", "scaled") for i in r if ops[i].kind == "lin")
        for i in lanes:
            if i is None:
                # an idle lane loads the operands of lane 0 (same addresses: an LDS broadcast,
                # no extra bank conflict) and runs no op (opcode NOP, header bits of its own: none)
                words += [0, words[first + 1], words[first + 2], 0] if nw == 4 and len(words) > first else [0] * nw
                continue
            op = ops[i]
            k = op.kind
            A, B, C, D, coefs, scale = lane_operands(sc.prog, i, unit)
            dst = sc.slot_of.get(i, 0)
            w0 = OPC[k] | dst << 5 | (op.imm & 63) << 16
            if k in ("sgn0", "lex", "eq"):
                cref = sc.consts.ref(1, True)          # plain 1: from-Montgomery product
            elif k == "inv":
                cref = sc.consts.ref(R_MONT * R_MONT % P, False)   # raw R^3: back to Montgomery
            else:
                cref = _operand(sc, C)
            xa, xb = _operand(sc, A), _operand(sc, B)
            if k in PRODUCTS and coefs[1] < 0:
                # r06: a product's negated operand always on y = C + cd D (fpvm.hpp pre_add2 has
                # no x negation chain; lane_operands swaps muls operands already): eq's x = A - B
                # goes to y, and x = the plain 1 (x y is symmetric)
                assert k == "eq" and coefs[3] >= 0, ("%s: x operand negated" % sc.prog.name, k, coefs)
                xa, xb, cref, dref = cref, _operand(sc, D), xa, xb
                coefs = [coefs[2], coefs[3], coefs[0], coefs[1]] + coefs[4:]
            else:
                dref = _operand(sc, D)
            w3 = _c5(coefs[0]) | _c5(coefs[1]) << 5 | _c5(coefs[2]) << 10 | _c5(coefs[3]) << 15 | scale << 20
            if k == "lin" and not unit and ALL_ACC:
                w3 |= FORCE_ACC
            words += [w0, xa | xb << 16, cref | dref << 16, w3]
        # the phase header (wave-uniform code paths) in bits 22.. of every lane's w0
        base = len(words) - sc.W * nw
        hdr = 0
        lane_bits = [phase_bits(words[base + lane * nw:base + lane * nw + 4]) for lane in range(sc.W)]
        for b in lane_bits:
            hdr |= b
        # fpvm.hpp exec picks a lin lane's block from the header alone (H_ACC: every lin op of the
        # phase in the general block): no phase may mix unit-block and general-block lin ops
        if hdr & H_ACC:
            assert not any(b & H_LIN and not b & H_SELB for b in lane_bits), (sc.prog.name, "mixed lin blocks")
        for lane in range(sc.W):
            words[base + lane * nw] |= hdr
    return words


# phase header bits (fpvm.hpp exec): which interpreter blocks any lane of the phase needs
H_MUL, H_MULNEG, H_FLAG, H_LIN, H_LINNEG, H_ACC, H_RARE, H_SELB = (1 << k for k in range(22, 30))
# r06: which unit-lin positions some lane negates beyond D (fpvm.hpp lin_sum XORs only those):
# C (H_LINNEG2) and B (H_LINNEG3); lane_operands puts a unit sum's negated terms last
H_LINNEG2, H_LINNEG3 = 1 << 30, 1 << 31


def phase_bits(w):
    """Header bits one lane's instruction (w0..w3) contributes (mirrors fpvm.hpp exec)."""
    opc = w[0] & 31
    if opc == OPC["nop"]:
        return 0
    ca, cb, cc, cd = (_s5((w[3] >> (5 * q)) & 31) for q in range(4))
    if opc in (OPC["muls"], OPC["sgn0"], OPC["lex"], OPC["eq"]):
        return H_MUL | (H_MULNEG if cb < 0 or cd < 0 else 0) | (0 if opc == OPC["muls"] else H_FLAG)
    if opc == OPC["selb"]:
        return H_LIN | H_SELB
    if opc == OPC["lin"]:
        if ca == 1 and all(-1 <= c <= 1 for c in (cb, cc, cd)) and not (w[3] & FORCE_ACC) and \
                (not ALL_ACC or PHASE_UNIT):
            return (H_LIN | (H_LINNEG if min(cb, cc, cd) < 0 else 0) | (H_LINNEG2 if cc < 0 else 0) |
                    (H_LINNEG3 if cb < 0 else 0))
        return H_ACC
    return H_RARE


def _s5(x):
    return x - 32 if x & 16 else x


def simulate(sc, words, inputs: dict, scalar: int = 0):
    """Execute the encoded stream on canonical values; returns {output name: value}."""
    const_vals = sc.consts.entries
    slots = [0] * sc.nslots
    for name, v in sc.prog.inputs.items():
        if v in sc.slot_of:
            slots[sc.slot_of[v]] = inputs[name] % P

    def get(ref):
        if ref >= CONST_BASE:
            return const_vals[ref - CONST_BASE][0]
        return slots[ref]
    W = sc.W
    nw = words_per_lane(sc.prog)
    stored = {}
    scratch = {}
    side = getattr(sc, "side_words", None) or [0] * (sc.nrounds * W)
    for t in range(sc.nrounds):
        # side ops (fpvm.hpp run): fills land at the start of the phase
        for sw in side[t * W:(t + 1) * W]:
            if sw >> 31 and (sw >> 30) & 1:
                slots[sw & 0x7FF] = scratch[(sw >> 11) & 0xFFF]
        results = []
        for lane in range(W):
            ins = words[(t * W + lane) * nw:(t * W + lane) * nw + nw]
            w0, w1, w2, w3 = ins[:4]
            opc = w0 & 31
            if opc == 0:
                continue
            dst = (w0 >> 5) & 0x7FF
            imm = (w0 >> 16) & 63
            A, B, C, D = get(w1 & 0xFFFF), get(w1 >> 16), get(w2 & 0xFFFF), get(w2 >> 16)
            ca, cb, cc, cd = (_s5((w3 >> (5 * q)) & 31) for q in range(4))
            ext = 0
            if nw == 8:
                w4, w5, w6 = ins[4:7]
                E, F, G, H = get(w4 & 0xFFFF), get(w4 >> 16), get(w5 & 0xFFFF), get(w5 >> 16)
                ce, cf, cg, ch = (_s5((w6 >> (5 * q)) & 31) for q in range(4))
                ext = ce * E + cf * F + cg * G + ch * H
            if opc == OPC["sel"]:
                z = C if A else B
            elif opc == OPC["selb"]:
                z = C if (scalar >> imm) & 1 else B
            elif opc in (OPC["and"], OPC["or"], OPC["xor"]):
                z = (A & C) if opc == OPC["and"] else (A | C) if opc == OPC["or"] else (A ^ C)
            elif opc == OPC["st"]:
                stored[imm] = A
                continue
            elif opc == OPC["inv"]:
                z = pow(A, P - 2, P)
            elif opc == OPC["sop"]:
                z = (A * C + cb * B * D) % P
            elif opc == OPC["lin"]:
                z = (ca * A + cb * B + cc * C + cd * D + ext) % P
                if (w3 >> 20) & 15 > 1:
                    z = z * ((w3 >> 20) & 15) % P
            else:
                x = (ca * A + cb * B) % P
                y = (cc * C + cd * D) % P
                # the flag ops read the from-Montgomery product x y of a value and the plain 1
                # (either operand: encode() moves eq's A - B to y)
                if opc == OPC["muls"]:
                    z = x * y % P
                elif opc == OPC["sgn0"]:
                    z = x * y % P & 1
                elif opc == OPC["lex"]:
                    z = 1 if x * y % P > HALF_P else 0
                elif opc == OPC["eq"]:
                    z = 1 if x * y % P == 0 else 0
                else:
                    raise ValueError(opc)
            results.append((dst, z))
        for dst, z in results:
            slots[dst] = z
        for sw in side[t * W:(t + 1) * W]:   # spills after the phase's ops
            if sw >> 31 and not (sw >> 30) & 1:
                scratch[(sw >> 11) & 0xFFF] = slots[sw & 0x7FF]
    out = {}
    for name, v in sc.prog.outputs.items():
        op = sc.prog.ops[v]
        out[name] = stored[op.imm] if op.kind == "st" else slots[sc.slot_of[v]]
    return out


SIDE = ("spill", "fill")   # side ops: run beside a phase's lane ops (one per lane per phase)


def spill_pass(prog, rounds, W, K, gap=3):
    """Split long idle stretches of values out of LDS so that at most K values occupy a slot in
    any phase (r04: two vote workgroups per SIMD need the vote program under ~90 of its 159
    slots; VERDICT r03 "next" 1).

    Occupancy of a value: [def phase, last read phase] (a slot last read in phase t is free from
    t + 1: the allocator's rule). Spills and fills are side ops: each lane runs at most one
    beside its phase op (fpvm.hpp run: a per-lane side word per phase), so they take no lane:
      spill in phase t  stores a slot to the unit's scratch after the phase's ops (a value
                        defined in phase t may be stored in t);
      fill in phase t   writes a slot at the start of phase t from a scratch load issued at the
                        start of phase t - 1 (one phase hides the L2 latency): it occupies from t.
    Greedy, Belady-like: at the most crowded phase t*, among the values that occupy t* without
    being read or defined there, take the one whose next read c is farthest; spill it in the
    earliest phase from its last read / definition before t* with a side word free (none if an
    earlier spill left a copy: values are immutable) and fill it in the latest phase <= c with a
    side word free (its later reads are rewritten to the fill), at least `gap` phases after the
    spill (the store drains before the load). Each spilled value gets a scratch entry, reused once
    its last fill has completed (interval colouring). The floor is what one phase reads and
    defines (at most 80 values at 16 lanes).
    Mutates prog.ops (appended ops, rewritten srcs), prog.outputs and `rounds` (side ops are
    appended to their phase's list; encode() emits them as side words); returns (scratch
    entries, spills, fills)."""
    from ir import Op
    ops = prog.ops
    T = len(rounds)
    side = [0] * T
    d = {}
    uses = defaultdict(list)
    for name, v in prog.inputs.items():
        d[v] = -1
    readers = defaultdict(list)
    for t, r in enumerate(rounds):
        for i in r:
            d[i] = t
            for s_ in set(x for x in ops[i].srcs if x is not None and ops[x].kind != "const"):
                uses[s_].append(t)
                readers[s_].append((t, i))
    outs = {v for v in prog.outputs.values() if ops[v].kind != "st"}
    for v in outs:
        uses[v].append(T)
    vals = [v for v in d if ops[v].kind != "st"]
    for v in vals:
        uses[v].sort()

    def lu(v):
        return uses[v][-1] if uses[v] else d[v]
    occ = [0] * (T + 1)
    starts = defaultdict(list)     # phase -> values whose occupancy starts there (candidate scan)
    for v in vals:
        for t in range(max(d[v], 0), min(lu(v), T) + 1):
            occ[t] += 1
    origin = {}          # fill copy -> the original value (scratch owner)
    scr_iv = {}          # original -> [first spill phase, last fill phase]
    alive = set(vals)
    nsp = nfi = 0
    failed, last_ts = set(), None
    while True:
        ts = max(range(T), key=lambda t: occ[t])
        if occ[ts] <= K:
            break
        if ts != last_ts:
            failed, last_ts = set(), ts
        best = None
        for v in alive:
            if v in failed or not (d[v] < ts < lu(v)):
                continue
            us = uses[v]
            k = bisect.bisect_right(us, ts)
            if k > 0 and us[k - 1] == ts:
                continue
            c = us[k]
            a = us[k - 1] if k > 0 else d[v]
            if d[v] == ts:
                continue
            need_spill = origin.get(v, v) not in scr_iv
            # a side spill runs after its phase's ops: it may store a value defined in that phase
            lo = max(a, d[v], 0) if need_spill else a + 1
            if lo > ts - (1 if need_spill else 0) or (need_spill and c < lo + gap):
                continue
            if best is None or c > best[0]:
                best = (c, v, a, need_spill, lo)
        if best is None:
            occv = [v for v in alive if max(d[v], 0) <= ts <= lu(v)]
            cat = defaultdict(int)
            for v in occv:
                us = uses[v]
                cat["read here" if ts in us else "def here" if d[v] == ts else "read next" if ts + 1 in us
                    else "failed" if v in failed else "other"] += 1
            raise RuntimeError("%s: cannot spill below %d slots at phase %d (%d occupied: %s)" % (
                prog.name, K, ts, occ[ts], dict(cat)))
        c, v, a, need_spill, lo = best
        owner = origin.get(v, v)
        end_old = a
        ps = None
        if need_spill:
            ps = next((t for t in range(lo, ts) if side[t] < W), None)
            if ps is None:
                failed.add(v)
                continue
        low = max(ts + 1, ps + gap) if ps is not None else ts + 1
        pf = next((t for t in range(min(c, T - 1), low - 1, -1) if side[t] < W), None)
        if pf is None:
            failed.add(v)
            continue
        if need_spill:
            si = len(ops)
            ops.append(Op("spill", srcs=(v,), imm=0))
            ops[si].sec = "spill"
            rounds[ps].append(si)
            side[ps] += 1
            d[si] = ps
            bisect.insort(uses[v], ps)
            readers[v].append((ps, si))
            scr_iv[owner] = [ps, pf]
            end_old = ps
            nsp += 1
        fi = len(ops)
        ops.append(Op("fill", srcs=(), imm=0, deps=(owner,)))
        ops[fi].sec = "fill"
        rounds[pf].append(fi)
        side[pf] += 1
        nfi += 1
        d[fi] = pf
        origin[fi] = owner
        scr_iv[owner][1] = max(scr_iv[owner][1], pf)
        # reads of v from phase c on move to the fill
        uses[fi] = [u for u in uses[v] if u >= c]
        uses[v] = [u for u in uses[v] if u < c]
        keep = []
        for (t, i) in readers[v]:
            if t >= c:
                ops[i].srcs = tuple(fi if s_ == v else s_ for s_ in ops[i].srcs)
                readers[fi].append((t, i))
            else:
                keep.append((t, i))
        readers[v] = keep
        if v in outs:
            outs.discard(v)
            outs.add(fi)
            for name, o in prog.outputs.items():
                if o == v:
                    prog.outputs[name] = fi
        for t in range(end_old + 1, pf):
            occ[t] -= 1
        alive.add(fi)
        if lu(v) <= ts:
            alive.discard(v)
    # scratch entries: interval colouring of [first spill, last fill] per spilled value
    iv = sorted((a, b, o) for o, (a, b) in scr_iv.items())
    heap, nscr, entry = [], 0, {}
    for a, b, o in iv:
        if heap and heap[0][0] < a:
            _, e = heapq.heappop(heap)
        else:
            e = nscr
            nscr += 1
        entry[o] = e
        heapq.heappush(heap, (b, e))
    for i in range(len(ops)):
        if ops[i].kind == "spill":
            ops[i].imm = entry[ops[i].srcs[0]]
        elif ops[i].kind == "fill":
            ops[i].imm = entry[origin[i]]
    return nscr, nsp, nfi
