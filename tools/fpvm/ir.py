"""Fp-VM intermediate representation: a straight-line program of operations on elements of
GF(p) (p = the BLS12-381 base prime), traced from Python code (alg.py) and later scheduled
onto the lanes of a wave slice (sched.py).

Every value is one Fp element (a "slot" at run time). Flags are Fp slots holding 0/1 in limb 0.
Operations (the interpreter in consensus_overlord_amd/csrc/fpvm.hpp implements exactly these):

  muls  z = (a + sb*b) * (c + sd*d)            heavy: one Montgomery product
  sgn0  z = parity(canonical(a))               heavy (from-Montgomery product)
  lex   z = canonical(a) > (p-1)/2             heavy
  lin   z = (a + sb*b) + sy*(c + sd*d)         light
  sel   z = flag(f) ? y : x                    light
  eq    z = (a + sb*b) == (c + sd*d)           light
  and/or/xor  on flags                          light
  rbit  z = bit k of the vote's 64-bit scalar   light

Signs are +1 / -1; a missing operand is None. Constants are Fp values referenced by index
into a constant table; inputs are named slots the prologue fills.
"""
from __future__ import annotations

P = 0x1A0111EA397FE69A4B1BA7B6434BACD764774B84F38512BF6730D2A0F6B0F6241EABFFFEB153FFFFB9FEFFFFFFFFAAAB
HALF_P = (P - 1) // 2

HEAVY = {"muls", "sgn0", "lex"}
LIGHT = {"lin", "sel", "eq", "and", "or", "xor", "rbit", "st", "selb"}


class Val:
    __slots__ = ("prog", "id")

    def __init__(self, prog, vid):
        self.prog = prog
        self.id = vid

    # arithmetic sugar (Fp)
    def __add__(self, o):
        return self.prog.lin(self, o, 1)

    def __sub__(self, o):
        return self.prog.lin(self, o, -1)

    def __mul__(self, o):
        return self.prog.mul(self, o)

    def __neg__(self):
        return self.prog.lin(self.prog.zero, self, -1)


class Op:
    __slots__ = ("kind", "srcs", "signs", "imm", "name")

    def __init__(self, kind, srcs=(), signs=(), imm=0, name=None):
        self.kind = kind
        self.srcs = tuple(srcs)    # value ids (or None) -- order (a, b, c, d) / (f, x, y)
        self.signs = tuple(signs)  # (sb, sy, sd) for lin/muls/eq
        self.imm = imm
        self.name = name


class Prog:
    """A traced program. ops[i] defines value i. kind 'in' = input, 'const' = constant."""

    def __init__(self, name):
        self.name = name
        self.ops = []
        self.outputs = {}       # name -> value id
        self.inputs = {}        # name -> value id
        self._consts = {}       # int -> value id
        self.zero = self.const(0)
        self.one = self.const(1)  # the field element 1 (Montgomery R at run time)
        self.cse = {}
        self.raw_one = self.raw_const(1)  # raw limbs [1, 0, ...]: the flag "true" / plain 1

    # ------------------------------------------------------------------ builders
    def _new(self, op):
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

    def _key(self, kind, srcs, signs, imm=0):
        return (kind, srcs, signs, imm)

    def _op(self, kind, srcs, signs=(), imm=0):
        k = self._key(kind, srcs, signs, imm)
        if k in self.cse:
            return Val(self, self.cse[k])
        v = self._new(Op(kind, srcs, signs, imm))
        self.cse[k] = v.id
        return v

    def is_const(self, v):
        op = self.ops[v.id]
        return op.kind == "const" and op.name != "raw"

    def cval(self, v):
        return self.ops[v.id].imm

    def lin(self, a, b, sb=1):
        """a + sb*b"""
        if self.is_const(b) and self.cval(b) == 0:
            return a
        if self.is_const(a) and self.cval(a) == 0 and sb == 1:
            return b
        if self.is_const(a) and self.is_const(b):
            return self.const(self.cval(a) + sb * self.cval(b))
        return self._op("lin", (a.id, b.id, None, None), (sb, 1, 1))

    def lin4(self, a, sb, b, sy, c, sd=1, d=None):
        """(a + sb*b) + sy*(c + sd*d); b, c, d may be None."""
        return self._op("lin", (a.id, b.id if b is not None else None, c.id if c is not None else None,
                                d.id if d is not None else None), (sb, sy, sd))

    def mul(self, a, b):
        if self.is_const(a) and not self.is_const(b):
            a, b = b, a
        if self.is_const(b):
            cv = self.cval(b)
            if cv == 0:
                return self.zero
            if cv == 1:
                return a
            if cv == 2:
                return self.lin(a, a, 1)
            if cv == P - 1:
                return self.lin(self.zero, a, -1)
        if a.id > b.id and not self.is_const(b):
            a, b = b, a
        return self._op("muls", (a.id, None, b.id, None), (1, 1, 1))

    def muls(self, a, sb, b, c, sd, d):
        """(a + sb*b) * (c + sd*d); b or d may be None."""
        return self._op("muls", (a.id, b.id if b is not None else None, c.id, d.id if d is not None else None),
                        (sb, 1, sd))

    def sgn0(self, a):
        return self._op("sgn0", (a.id,))

    def lex(self, a):
        return self._op("lex", (a.id,))

    def eq(self, a, b):
        return self._op("eq", (a.id, None, b.id, None), (1, 1, 1))

    def is_zero(self, a):
        return self.eq(a, self.zero)

    def sel(self, f, x, y):
        """f ? y : x"""
        if x.id == y.id:
            return x
        return self._op("sel", (f.id, x.id, y.id))

    def f_and(self, a, b):
        return self._op("and", (a.id, b.id))

    def f_or(self, a, b):
        return self._op("or", (a.id, b.id))

    def f_xor(self, a, b):
        return self._op("xor", (a.id, b.id))

    def f_not(self, a):
        return self.f_xor(a, self.raw_one)

    def rbit(self, k):
        return self._op("rbit", (), (), k)

    def selb(self, k, x, y):
        """bit k of the unit's 64-bit scalar ? y : x"""
        if x.id == y.id:
            return x
        return self._op("selb", (x.id, y.id), (), k)

    def store(self, name, v, plane):
        """Write v to output plane `plane` of this unit in HBM (no slot result). The op is a
        program output so that it is scheduled; its value is v."""
        st = self._new(Op("st", (v.id,), (), plane, name=name))
        self.outputs["st:" + name] = st.id
        return st

    # ------------------------------------------------------------------ evaluation
    def evaluate(self, inputs: dict, scalar: int = 0) -> list:
        """Evaluate every value with Python integers (canonical values, not Montgomery)."""
        vals = [None] * len(self.ops)
        for i, op in enumerate(self.ops):
            vals[i] = eval_op(op, vals, inputs, scalar)
        return vals

    # ------------------------------------------------------------------ optimisation
    def _terms(self, op):
        """signed terms of a lin op: [(sign, value id)]"""
        sb, sy, sd = op.signs
        a, b, c, d = op.srcs
        t = [(1, a)]
        if b is not None:
            t.append((sb, b))
        if c is not None:
            t.append((sy, c))
        if d is not None:
            t.append((sy * sd, d))
        return t

    @staticmethod
    def _pack(terms):
        """4 signed terms -> (srcs, signs) in (A + sb B) + sy (C + sd D) form, or None."""
        terms = sorted(terms, key=lambda t: -t[0])  # a positive term first
        if terms[0][0] < 0 or len(terms) > 4:
            return None
        (s1, a), rest = terms[0], terms[1:]
        b = c = d = None
        sb = sy = sd = 1
        if len(rest) >= 1:
            sb, b = rest[0]
        if len(rest) >= 2:
            sy, c = rest[1]
        if len(rest) >= 3:
            sd = rest[2][0] * sy
            d = rest[2][1]
        return (a, b, c, d), (sb, sy, sd)

    def fuse(self):
        """Merge single-use lin chains into 4-term lin ops, and single-use 2-term lins into the
        pre-additions of muls / eq operands. Returns the number of ops absorbed."""
        live = set(self.live_ops())
        outs = set(self.outputs.values())
        uses = [0] * len(self.ops)
        for i in live:
            for s in self.ops[i].srcs:
                if s is not None:
                    uses[s] += 1
        absorbed = 0

        def fusable(j):
            o = self.ops[j]
            return o.kind == "lin" and uses[j] == 1 and j not in outs
        for i in sorted(live):
            op = self.ops[i]
            if op.kind == "lin":
                terms = self._terms(op)
                changed = True
                while changed:
                    changed = False
                    for k, (sg, v) in enumerate(terms):
                        if v is not None and fusable(v):
                            sub = [(sg * s2, v2) for s2, v2 in self._terms(self.ops[v])]
                            cand = terms[:k] + terms[k + 1:] + sub
                            packed = self._pack(cand) if len(cand) <= 4 else None
                            if packed is not None:
                                terms = cand
                                uses[v] -= 1
                                for _, v2 in sub:
                                    uses[v2] += 1
                                absorbed += 1
                                changed = True
                                break
                srcs, signs = self._pack(terms)
                op.srcs, op.signs = srcs, signs
            elif op.kind in ("muls", "eq"):
                sb, sy, sd = op.signs
                a, b, c, d = op.srcs
                new = [a, b, c, d]
                sg = [1, sb, 1, sd]
                for half in (0, 2):
                    x, y = new[half], new[half + 1]
                    if y is None and x is not None and fusable(x):
                        t = self._terms(self.ops[x])
                        if len(t) == 2 and t[0][0] == 1:
                            uses[x] -= 1
                            new[half], new[half + 1] = t[0][1], t[1][1]
                            sg[half + 1] = t[1][0]
                            uses[t[0][1]] += 1
                            uses[t[1][1]] += 1
                            absorbed += 1
                op.srcs = tuple(new)
                op.signs = (sg[1], sy, sg[3])
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


def eval_op(op, vals, inputs, scalar):
    k = op.kind
    if k == "in":
        return inputs[op.name] % P
    if k == "const":
        return op.imm
    s = op.srcs

    def g(i):
        return 0 if s[i] is None else vals[s[i]]
    if k in ("muls", "lin", "eq"):
        sb, sy, sd = op.signs
        x = (g(0) + sb * g(1)) % P
        y = (g(2) + sd * g(3)) % P
        if k == "muls":
            return x * y % P
        if k == "lin":
            return (x + sy * y) % P
        return 1 if x == y else 0
    if k == "sgn0":
        return vals[s[0]] & 1
    if k == "lex":
        return 1 if vals[s[0]] > HALF_P else 0
    if k == "sel":
        return vals[s[2]] if vals[s[0]] else vals[s[1]]
    if k == "and":
        return vals[s[0]] & vals[s[1]]
    if k == "or":
        return vals[s[0]] | vals[s[1]]
    if k == "xor":
        return vals[s[0]] ^ vals[s[1]]
    if k == "rbit":
        return (scalar >> op.imm) & 1
    if k == "st":
        return vals[s[0]]
    if k == "selb":
        return vals[s[1]] if (scalar >> op.imm) & 1 else vals[s[0]]
    raise ValueError(k)
