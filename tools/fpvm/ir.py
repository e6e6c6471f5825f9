"""Fp-VM intermediate representation: a straight-line program of operations on elements of
GF(p) (p = the BLS12-381 base prime), traced from Python code (alg.py) and later scheduled
onto the lanes of a wave slice (sched.py).

Every value is one Fp element (a "slot" at run time). Flags are Fp slots holding 0/1 in limb 0.
Operations (the interpreter in consensus_overlord_amd/csrc/fpvm.hpp implements exactly these):

  muls  z = (ca a + cb b) * (cc c + cd d)      heavy: one Montgomery product
  sgn0  z = parity(canonical(a))               heavy (from-Montgomery product)
  lex   z = canonical(a) > (p-1)/2             heavy
  inv   z = a^-1 (0 -> 0)                      heavy+: binary extended Euclid in one lane
  lin   z = ca a + cb b + cc c + cd d          light
  eq    z = a == b                             heavy (from-Montgomery product of a - b)
  sel   z = flag(f) ? y : x                    light
  selb  z = bit k of the unit's scalar ? y : x light
  and/or/xor  on flags                         light
  st    store a to the unit's output plane k   light (no result slot)

Coefficients are small signed integers (|c| <= CMAX); a missing operand has coefficient 0.
Constants are Fp values referenced by index into a constant table; inputs are named slots the
prologue fills.
"""
from __future__ import annotations

import math
import os

P = 0x1A0111EA397FE69A4B1BA7B6434BACD764774B84F38512BF6730D2A0F6B0F6241EABFFFEB153FFFFB9FEFFFFFFFFAAAB
HALF_P = (P - 1) // 2
CMAX = 15
LIN_WIDTH = 4   # default operands of a lin op (Prog.lin_width: 4, or 8 for wide-instruction programs)

HEAVY = {"muls", "sgn0", "lex", "inv", "sop", "eq"}
LIGHT = {"lin", "sel", "and", "or", "xor", "st", "selb"}


class Val:
    __slots__ = ("prog", "id")

    def __init__(self, prog, vid):
        self.prog = prog
        self.id = vid

    def __add__(self, o):
        return self.prog.lin([(1, self), (1, o)])

    def __sub__(self, o):
        return self.prog.lin([(1, self), (-1, o)])

    def __mul__(self, o):
        return self.prog.mul(self, o)

    def __neg__(self):
        return self.prog.lin([(-1, self)])


class Op:
    __slots__ = ("kind", "srcs", "coefs", "imm", "name", "deps", "sec")

    def __init__(self, kind, srcs=(), coefs=(), imm=0, name=None, deps=()):
        self.kind = kind
        self.srcs = tuple(srcs)    # value ids or None; (a, b, c, d) for muls/lin/eq
        self.coefs = tuple(coefs)  # (ca, cb, cc, cd) for muls/lin/eq
        self.imm = imm
        self.name = name
        self.deps = tuple(deps)    # ordering-only predecessors (no data, no slot lifetime)
        self.sec = None            # program section that created it (diagnostics)


def _norm_terms(terms):
    """[(coef, id)] -> merged, zero-free list"""
    acc = {}
    order = []
    for c, v in terms:
        if v not in acc:
            acc[v] = 0
            order.append(v)
        acc[v] += c
    return [(acc[v], v) for v in order if acc[v] != 0]


def _expand_unit(terms, width):
    """[(c, v)] -> <= width (sign, v) unit terms, first sign +1 (v None = the zero constant),
    or None. c * v becomes |c| copies of (sign c, v)."""
    ex = []
    for c, v in terms:
        ex += [(1 if c > 0 else -1, v)] * abs(c)
    if not ex:
        return [(1, None)]
    pos = [t for t in ex if t[0] > 0]
    neg = [t for t in ex if t[0] < 0]
    if pos:
        ex = pos[:1] + pos[1:] + neg
    else:
        ex = [(1, None)] + neg          # 0 - a - b ...
    return ex if len(ex) <= width else None


def lin_form(terms, width=None):
    """How the interpreter evaluates sum c_i v_i (fpvm.hpp exec):
    ("unit", u)      u = <= width unit terms, plain modular adds / subs;
    ("scaled", k, u) k * (unit sum), 2 <= k <= 15: one small-scalar product + reduction;
    ("acc", terms)   general signed 13-limb accumulation + reduction (slow)."""
    width = LIN_WIDTH if width is None else width
    terms = [(c, v) for c, v in terms if c]
    u = _expand_unit(terms, width)
    if u is not None:
        return ("unit", u)
    g = 0
    for c, _ in terms:
        g = math.gcd(g, abs(c))
    if 2 <= g <= CMAX:
        u = _expand_unit([(c // g, v) for c, v in terms], width)
        if u is not None:
            return ("scaled", g, u)
    return ("acc", terms)


# fusion cost of each form: with every lin op in the general-coefficient block (sched.ALL_ACC,
# the default) the three forms cost the same; the unit-sign interpreter path
# (OVH_GEN_UNITLIN=1) prefers unit sums
FORM_COST = {"unit": 1, "scaled": 2, "acc": 6} if os.environ.get("OVH_GEN_UNITLIN", "0") == "1" else \
    {"unit": 1, "scaled": 1, "acc": 1}


class Prog:
    """A traced program. ops[i] defines value i. kind 'in' = input, 'const' = constant."""

    def __init__(self, name, lin_width: int = LIN_WIDTH):
        self.name = name
        self.lin_width = lin_width   # operands of a lin op (8: the 32-byte instruction format)
        self.ops = []
        self.outputs = {}
        self.inputs = {}
        self._consts = {}
        self.cse = {}
        self.zero = self.const(0)
        self.one = self.const(1)          # the field element 1 (Montgomery R at run time)
        self.raw_one = self.raw_const(1)  # raw limbs [1, 0, ...]: flag "true" / plain 1

    # ------------------------------------------------------------------ builders
    def _new(self, op):
        op.sec = getattr(self, "section", None)
        self.ops.append(op)
        return Val(self, len(self.ops) - 1)

    def input(self, name):
        v = self._new(Op("in", name=name))
        self.inputs[name] = v.id
        return v

    def const(self, value: int):
        value %= P
        if value in self._consts:
            return Val(self, self._consts[value])
        v = self._new(Op("const", imm=value))
        self._consts[value] = v.id
        return v

    def raw_const(self, value: int):
        """A constant stored as plain limbs (not Montgomery): flags and the from-Montgomery 1."""
        key = ("raw", value)
        if key in self._consts:
            return Val(self, self._consts[key])
        v = self._new(Op("const", imm=value, name="raw"))
        self._consts[key] = v.id
        return v

    def output(self, name, v: Val):
        self.outputs[name] = v.id

    def _op(self, kind, srcs, coefs=(), imm=0, deps=()):
        k = (kind, tuple(srcs), tuple(coefs), imm, tuple(deps))
        if k in self.cse:
            return Val(self, self.cse[k])
        v = self._new(Op(kind, srcs, coefs, imm, deps=deps))
        self.cse[k] = v.id
        return v

    def is_const(self, v):
        op = self.ops[v.id]
        return op.kind == "const" and op.name != "raw"

    def cval(self, v):
        return self.ops[v.id].imm

    def lin(self, terms):
        """sum of coef * value, terms = [(coef, Val)] (any length; chained in 4-term ops)."""
        t = []
        cacc = 0
        for c, v in terms:
            if self.is_const(v):
                cacc += c * self.cval(v)
            else:
                t.append((c, v.id))
        t = _norm_terms(t)
        cacc %= P
        if cacc:
            t.append((1, self.const(cacc).id))
        if not t:
            return self.zero
        if len(t) == 1 and t[0][0] == 1:
            return Val(self, t[0][1])
        out = None
        while t:
            n = self.lin_width if out is None else self.lin_width - 1
            chunk, t = t[:n], t[n:]
            if out is not None:
                chunk = [(1, out.id)] + chunk
            fixed = []
            for c, v in chunk:
                if abs(c) > CMAX:
                    v = self.mul(Val(self, v), self.const(abs(c))).id
                    c = 1 if c > 0 else -1
                fixed.append((c, v))
            chunk = sorted(fixed, key=lambda cv: cv[1])
            srcs = [v for _, v in chunk] + [None] * (self.lin_width - len(chunk))
            coefs = [c for c, _ in chunk] + [0] * (self.lin_width - len(chunk))
            out = self._op("lin", srcs, coefs)
        return out

    def lin4(self, a, sb, b, sy, c, sd=1, d=None):
        """(a + sb*b) + sy*(c + sd*d); b, c, d may be None."""
        t = [(1, a)]
        if b is not None:
            t.append((sb, b))
        if c is not None:
            t.append((sy, c))
        if d is not None:
            t.append((sy * sd, d))
        return self.lin(t)

    def mul(self, a, b):
        if self.is_const(a) and not self.is_const(b):
            a, b = b, a
        if self.is_const(b):
            cv = self.cval(b)
            if self.is_const(a):
                return self.const(self.cval(a) * cv)
            if cv == 0:
                return self.zero
            if cv == 1:
                return a
            if cv <= CMAX:
                return self.lin([(cv, a)])
            if P - cv <= CMAX:
                return self.lin([(-(P - cv), a)])
        if a.id > b.id and not self.is_const(b):
            a, b = b, a
        return self._op("muls", (a.id, None, b.id, None), (1, 0, 1, 0))

    def muls(self, a, sb, b, c, sd, d):
        """(a + sb*b) * (c + sd*d); b or d may be None."""
        return self._op("muls", (a.id, b.id if b is not None else None, c.id, d.id if d is not None else None),
                        (1, sb if b is not None else 0, 1, sd if d is not None else 0))

    def sop(self, a, c, s, b, d):
        """a * c + s * b * d (s = +1 / -1): two products, one Montgomery reduction."""
        if s > 0 and (b.id, d.id) < (a.id, c.id):
            a, c, b, d = b, d, a, c
        return self._op("sop", (a.id, b.id, c.id, d.id), (1, s, 1, 1))

    def sgn0(self, a):
        return self._op("sgn0", (a.id,))

    def lex(self, a):
        return self._op("lex", (a.id,))

    def inv(self, a):
        return self._op("inv", (a.id,))

    def eq(self, a, b):
        return self._op("eq", (a.id, None, b.id, None), (1, 0, 1, 0))

    def is_zero(self, a):
        return self.eq(a, self.zero)

    def sel(self, f, x, y):
        """f ? y : x"""
        if x.id == y.id:
            return x
        return self._op("sel", (f.id, x.id, y.id))

    def selb(self, k, x, y, after=None):
        """bit k of the unit's 64-bit scalar ? y : x. `after`: a value this select must not be
        scheduled before (keeps selects of long-ready operands next to their use)."""
        if x.id == y.id:
            return x
        return self._op("selb", (x.id, y.id), (), k, deps=(after.id,) if after is not None else ())

    def f_and(self, a, b):
        return self._op("and", (a.id, b.id))

    def f_or(self, a, b):
        return self._op("or", (a.id, b.id))

    def f_xor(self, a, b):
        return self._op("xor", (a.id, b.id))

    def f_not(self, a):
        return self.f_xor(a, self.raw_one)

    def store(self, name, v, plane):
        """Write v to output plane `plane` of this unit in HBM (no slot result)."""
        st = self._new(Op("st", (v.id,), (), plane, name=name))
        self.outputs["st:" + name] = st.id
        return st

    # ------------------------------------------------------------------ optimisation
    def _lin_terms(self, op):
        return [(c, v) for c, v in zip(op.coefs, op.srcs) if v is not None and c != 0]

    def fuse(self, dup: bool = False):
        """Merge lin ops into their consumers: into a lin (<= 4 distinct terms, small
        coefficients) or into the 2-term operand sums of muls / eq. A single-use producer is
        absorbed when the consumer's coefficient form costs no more than the two did; with
        `dup`, a shared producer is also copied into consumers whose form stays as cheap, which
        takes it off their dependency chains. Returns ops absorbed."""
        live = set(self.live_ops())
        outs = set(self.outputs.values())
        uses = [0] * len(self.ops)
        for i in live:
            for s in self.ops[i].srcs:
                if s is not None:
                    uses[s] += 1
        absorbed = 0

        def cost(terms, limit):
            f = lin_form(terms, limit)[0]
            return FORM_COST[f] if limit == self.lin_width else (0 if f == "unit" else 1000)  # muls operands: unit only

        def fusable(j):
            return j is not None and self.ops[j].kind == "lin" and j not in outs and (uses[j] == 1 or dup)

        def try_merge(terms, limit):
            nonlocal absorbed
            changed = True
            while changed:
                changed = False
                for k, (c, v) in enumerate(terms):
                    if fusable(v):
                        sub = [(c * c2, v2) for c2, v2 in self._lin_terms(self.ops[v])]
                        cand = _norm_terms(terms[:k] + terms[k + 1:] + sub)
                        # a single-use producer disappears (its cost is credited); a shared one
                        # is duplicated into this consumer only if the consumer gets no dearer
                        credit = cost(self._lin_terms(self.ops[v]), self.lin_width) if uses[v] == 1 else 0
                        if len(cand) <= limit and all(abs(c3) <= CMAX for c3, _ in cand) and \
                                cost(cand, limit) <= cost(terms, limit) + credit:
                            uses[v] -= 1
                            for _, v2 in sub:
                                uses[v2] += 1
                            terms[:] = cand
                            absorbed += 1
                            changed = True
                            break
            return terms
        for i in sorted(live):
            op = self.ops[i]
            if op.kind == "lin":
                terms = try_merge(self._lin_terms(op), self.lin_width)
                terms = sorted(terms, key=lambda cv: cv[1])
                op.srcs = tuple([v for _, v in terms] + [None] * (self.lin_width - len(terms)))
                op.coefs = tuple([c for c, _ in terms] + [0] * (self.lin_width - len(terms)))
            elif op.kind == "muls":   # eq keeps single operands: the interpreter tests a - b
                a, b, c, d = op.srcs
                ca, cb, cc, cd = op.coefs
                left = try_merge(_norm_terms([(ca, a)] + ([(cb, b)] if b is not None and cb else [])), 2)
                right = try_merge(_norm_terms([(cc, c)] + ([(cd, d)] if d is not None and cd else [])), 2)
                if not left:
                    left = [(1, self.zero.id)]
                if not right:
                    right = [(1, self.zero.id)]
                left = left + [(0, None)] * (2 - len(left))
                right = right + [(0, None)] * (2 - len(right))
                op.srcs = (left[0][1], left[1][1], right[0][1], right[1][1])
                op.coefs = (left[0][0], left[1][0], right[0][0], right[1][0])
        self.cse = {}
        return absorbed

    def live_ops(self):
        """Ids of ops reachable from the outputs (dead code removed)."""
        need = set()
        stack = list(self.outputs.values())
        while stack:
            v = stack.pop()
            if v in need:
                continue
            need.add(v)
            for s in self.ops[v].srcs:
                if s is not None:
                    stack.append(s)
        return sorted(need)

    # ------------------------------------------------------------------ evaluation
    def evaluate(self, inputs: dict, scalar: int = 0) -> list:
        """Evaluate every value with Python integers (canonical values, not Montgomery)."""
        vals = [None] * len(self.ops)
        # fill ops (sched.spill_pass) are appended after their readers: each takes its original
        # value's (deps[0]) as soon as that is known
        fills = {}
        for i, op in enumerate(self.ops):
            if op.kind == "fill":
                fills.setdefault(op.deps[0], []).append(i)
        for i, op in enumerate(self.ops):
            if op.kind == "fill":
                continue
            vals[i] = eval_op(op, vals, inputs, scalar)
            for f in fills.get(i, ()):
                vals[f] = vals[i]
        return vals


def eval_op(op, vals, inputs, scalar):
    k = op.kind
    if k == "in":
        return inputs[op.name] % P
    if k == "const":
        return op.imm
    s = op.srcs

    def g(i):
        return 0 if s[i] is None else vals[s[i]]
    if k == "lin":
        return sum(c * g(j) for j, c in enumerate(op.coefs)) % P
    if k in ("muls", "eq"):
        ca, cb, cc, cd = op.coefs
        x = (ca * g(0) + cb * g(1)) % P
        y = (cc * g(2) + cd * g(3)) % P
        if k == "muls":
            return x * y % P
        return 1 if x == y else 0
    if k == "sop":
        return (g(0) * g(2) + op.coefs[1] * g(1) * g(3)) % P
    if k == "spill":
        return g(0)
    if k == "sgn0":
        return vals[s[0]] & 1
    if k == "lex":
        return 1 if vals[s[0]] > HALF_P else 0
    if k == "inv":
        return pow(vals[s[0]], P - 2, P)
    if k == "sel":
        return vals[s[2]] if vals[s[0]] else vals[s[1]]
    if k == "selb":
        return vals[s[1]] if (scalar >> op.imm) & 1 else vals[s[0]]
    if k == "and":
        return vals[s[0]] & vals[s[1]]
    if k == "or":
        return vals[s[0]] | vals[s[1]]
    if k == "xor":
        return vals[s[0]] ^ vals[s[1]]
    if k == "st":
        return vals[s[0]]
    raise ValueError(k)
