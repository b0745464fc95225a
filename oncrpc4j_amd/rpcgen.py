"""rpcgen.py — XDR language (.x) files -> engine field tapes.

oncrpc4j's jrpcgen turns a .x file into XdrAble classes whose xdrEncode /
xdrDecode call the stream once per declaration, in declaration order
(oncrpc4j-rpcgen .../jrpcgen/jrpcgen.java:758-913 `codingMethod`), so the
record's bytes are the concatenation of its declarations' encodings, nested
structs included.  This module reads the same .x language (grammar:
jrpcgen/JrpcgenParser.cup) and emits that concatenation as an engine field
tape (include/xdrg.h xdrg_field: type x kind x count), so unchanged .x files
drive the batch engine:

  const, typedef, enum, struct (flattened), program / version / procedure
  (argument and result tapes, multi-argument procedures as jrpcgen encodes
  them: one after another), base types as JrpcgenParser.cup:716-802 maps
  them (char -> byte, short, int/long, hyper, unsigned X -> X's bytes, bool,
  float, double, quadruple -> double), opaque[n] / opaque<n>, string<n>,
  T[n] / T<n> of base types.

Unions (jrpcgen.java:1240-1340 encodes the discriminant, then the arm whose
case list holds it, the default arm, or nothing) and optional data `T *x`
(JrpcgenDeclaration.INDIRECTION: a bool, then T or nothing) give records of
one type different shapes.  Spec.tape() flattens them into one tape plus
conditions (include/xdrg.h xdrg_cond: field k present iff its discriminant
field is present and the discriminant's value is / is not in a case list),
which the engine batches directly (engine.Schema(fields, conds)).
Spec.fields() keeps the plain-tape contract and raises NotBatchable for
them.

Arrays of structs `T x<>` / `T x[N]` (jrpcgen.java:856-906: the count, then
each element's xdrEncode) and recursive lists — a struct whose last
declaration is `T *next`, used as `T *x` or `T x` (INDIRECTION,
jrpcgen.java:835-851: TRUE + element while there is one, then FALSE; the
reference's own portmap/pmaplist.java:50-69) — become repeated groups
(include/xdrg.h: a (T_GROUP, kind, count, members) field and the element's
flattened fields as members).  Unions and optional data inside an element
become conditions between members of the same group (evaluated per
element), and a group may itself sit in a union arm or behind optional data
(a condition on the group field).  A fixed-size array of structs inside an
element (`T x[N]`, no count word) unrolls into N copies of T's members; a
variable-length array of structs or a list inside an element becomes an
inner group (its members are the inner element's flattened fields, its rows
the outer elements), and so on down to GROUP_LEVELS levels.  An array of list
nodes (each element the head of a chain, jrpcgen.java:1103-1121) is a group
whose element is the head's fields followed by the chain's remaining nodes as
an inner list.  Still not one tape: deeper nesting, and recursion anywhere but
a struct's last declaration.
"""
import re

from . import abi

INT = (abi.T_INT, abi.K_SCALAR, 0)
GROUP_LEVELS = 4   # group nesting levels the engine batches (xdrg_internal.h kGrpLevels)


class XdrSyntaxError(ValueError):
    pass


class NotBatchable(ValueError):
    """The type's records do not share one field tape (union / optional / array of
    structs / recursion); see Spec.tape() for the conditional form."""


# ---- lexer ----------------------------------------------------------------------
_TOKEN = re.compile(r"""
    (?P<ws>\s+) | (?P<comment>/\*.*?\*/|//[^\n]*) | (?P<pass>^%[^\n]*) |
    (?P<num>-?(?:0[xX][0-9a-fA-F]+|\d+)) | (?P<id>[A-Za-z_][A-Za-z0-9_]*) | (?P<sym>[;,:=*(){}\[\]<>])
    """, re.X | re.S | re.M)


def _tokens(text):
    pos = 0
    out = []
    while pos < len(text):
        m = _TOKEN.match(text, pos)
        if not m:
            raise XdrSyntaxError(f"unexpected {text[pos:pos + 20]!r} at offset {pos}")
        pos = m.end()
        kind = m.lastgroup
        if kind in ("ws", "comment", "pass"):
            continue
        out.append((kind, m.group()))
    return out


def _int_literal(s):
    """C integer literal: decimal, 0x hex, leading-0 octal (JrpcgenParser.cup constant forms)."""
    neg = s.startswith("-")
    t = s[1:] if neg else s
    if t[:2] in ("0x", "0X"):
        v = int(t, 16)
    elif len(t) > 1 and t[0] == "0":
        v = int(t, 8)
    else:
        v = int(t)
    return -v if neg else v


# ---- declarations ----------------------------------------------------------------
BASE = {  # JrpcgenParser.cup:716-802 (+ string / opaque declarations)
    "int": abi.T_INT, "long": abi.T_INT, "short": abi.T_SHORT, "char": abi.T_BYTE,
    "hyper": abi.T_HYPER, "bool": abi.T_BOOL, "float": abi.T_FLOAT, "double": abi.T_DOUBLE,
    "quadruple": abi.T_DOUBLE,
}
UNSIGNED = {abi.T_INT: abi.T_UINT, abi.T_HYPER: abi.T_UHYPER, abi.T_SHORT: abi.T_SHORT,
            abi.T_BYTE: abi.T_BYTE}


class Decl:
    """One declaration: name, type (base id or type name), kind, size expr."""

    def __init__(self, name, type_, kind, size=None):
        self.name, self.type, self.kind, self.size = name, type_, kind, size

    def __repr__(self):
        return f"Decl({self.name!r}, {self.type!r}, {self.kind}, {self.size!r})"


SCALAR, FIXED, DYNAMIC, OPTIONAL, VOID = "scalar", "fixed", "dynamic", "optional", "void"


class Struct:
    def __init__(self, name, decls):
        self.name, self.decls = name, decls


class Union:
    def __init__(self, name, disc, arms, default):
        self.name, self.disc, self.arms, self.default = name, disc, arms, default   # arms: [(values, Decl)]


class Enum:
    def __init__(self, name, values):
        self.name, self.values = name, values


class Procedure:
    def __init__(self, name, number, result, args):
        self.name, self.number, self.result, self.args = name, number, result, args


class Spec:
    """A parsed .x file."""

    def __init__(self):
        self.consts = {}
        self.types = {}      # name -> Struct | Union | Enum | Decl (typedef)
        self.programs = {}   # name -> (number, {version name: (number, [Procedure])})

    # ---- constants --------------------------------------------------------------
    def value(self, v):
        if v is None:
            return 0
        if isinstance(v, int):
            return v
        if v in ("TRUE", "FALSE"):    # bool union case labels (RFC 4506 §4.4: TRUE / FALSE)
            return int(v == "TRUE")
        if re.fullmatch(r"-?(0[xX][0-9a-fA-F]+|\d+)", v):
            return _int_literal(v)
        if v in self.consts:
            return self.value(self.consts[v])
        for t in self.types.values():
            if isinstance(t, Enum) and v in t.values:
                return self.value(t.values[v])
        raise XdrSyntaxError(f"unknown constant {v!r}")

    # ---- tapes --------------------------------------------------------------------
    def fields(self, type_name):
        """Plain field tape of one record of `type_name` (structs flattened);
        NotBatchable if the type needs conditions (use tape())."""
        return self._plain(self.tape(type_name), type_name)

    def tape(self, type_name):
        """(fields, conds) of one record of `type_name`: conds =
        [(field, disc, negate, values)] for union arms and optional data."""
        b = _Tape(self)
        b.type_(type_name, type_name, None, ())
        return b.result()

    @staticmethod
    def _plain(tape, where):
        fields, conds = tape
        if conds:
            raise NotBatchable(f"{where}: {fields.reasons[0]}; Spec.tape() gives the conditional tape")
        return list(fields)

    def _elem(self, t, where):
        """Base element type id of an array declaration's element type."""
        d = self.types.get(t)
        while isinstance(d, Decl) and d.kind == SCALAR:   # typedef chain to a scalar
            t, d = d.type, self.types.get(d.type)
        if isinstance(d, Enum):
            return abi.T_ENUM
        if t in BASE or t == "unsigned":
            return BASE.get(t, abi.T_INT)
        if isinstance(t, tuple):   # ("unsigned", base)
            return t[1]
        raise NotBatchable(f"{where}: array of {t!r} (arrays of structs / unions have no flat tape)")

    # ---- procedures ---------------------------------------------------------------
    def procedures(self):
        """(prog, vers, proc) -> Procedure, for every program in the file."""
        out = {}
        for pname, (pnum, versions) in self.programs.items():
            for vname, (vnum, procs) in versions.items():
                for p in procs:
                    out[(pnum, vnum, p.number)] = p
        return out

    def args_fields(self, prog, vers, proc):
        """Argument tape of a call (arguments one after another, jrpcgen
        multi-argument procedures)."""
        p = self.procedures()[(prog, vers, proc)]
        return self._plain(self.args_tape(prog, vers, proc), f"{p.name} arguments")

    def result_fields(self, prog, vers, proc):
        p = self.procedures()[(prog, vers, proc)]
        return self._plain(self.result_tape(prog, vers, proc), f"{p.name} result")

    def args_tape(self, prog, vers, proc):
        p = self.procedures()[(prog, vers, proc)]
        b = _Tape(self)
        for i, a in enumerate(p.args):
            b.arg(a, f"{p.name} argument {i}")
        return b.result()

    def result_tape(self, prog, vers, proc):
        p = self.procedures()[(prog, vers, proc)]
        b = _Tape(self)
        b.arg(p.result, f"{p.name} result")
        return b.result()


class _TapeFields(list):
    """A field list that also remembers why it needed conditions."""
    reasons = ()


class _Tape:
    """Flattens declarations into (fields, conds) in jrpcgen's encode order
    (codingMethod, jrpcgen.java:758-913).  `guard` = (disc field index,
    negate, values) is the condition every field emitted under it carries;
    nesting chains through the discriminant's own condition."""

    DISC_TYPES = (abi.T_INT, abi.T_UINT, abi.T_ENUM, abi.T_BOOL)

    # a fixed array of structs inside a group element unrolls into this many
    # copies of the struct's members at most (the engine's field limit bounds
    # the tape anyway)
    MAX_UNROLL = 16

    def __init__(self, spec, in_element=False, depth=0):
        self.s = spec
        self.in_element = in_element
        self.depth = depth   # group levels above this tape (0: a record's tape)
        self.fields = _TapeFields()
        self.fields.reasons = []
        self.conds = []

    def result(self):
        return self.fields, self.conds

    def add(self, f, guard):
        k = len(self.fields)
        self.fields.append(f)
        if guard is not None:
            d, neg, vals = guard
            self.conds.append((k, d, neg, list(vals)))
        return k

    def arg(self, t, where):
        if t == "void":
            return
        if isinstance(t, tuple):
            self.add((t[1], abi.K_SCALAR, 0), None)
            return
        self.type_(t, where, None, ())

    def type_(self, t, where, guard, stack):
        if t in BASE or t in ("unsigned",):
            self.add((BASE.get(t, abi.T_INT), abi.K_SCALAR, 0), guard)
            return
        if t == "string":
            self.add((abi.T_STRING, abi.K_DYNAMIC, 0), guard)
            return
        d = self.s.types.get(t)
        if d is None:
            raise XdrSyntaxError(f"unknown type {t!r} (in {where})")
        if isinstance(d, Enum):
            self.add((abi.T_ENUM, abi.K_SCALAR, 0), guard)
            return
        if isinstance(d, (Struct, Union)):
            if t in stack:
                raise NotBatchable(f"{where}: {t} contains itself (a recursive type has no "
                                   f"bounded tape)")
            stack = stack + (t,)
        if isinstance(d, Struct):
            for decl in d.decls:
                self.decl(decl, f"{where}.{decl.name}", guard, stack)
            return
        if isinstance(d, Union):
            self.union(d, where, guard, stack)
            return
        self.decl(d, where, guard, stack)   # typedef

    def union(self, u, where, guard, stack):
        # jrpcgen.java:1240-1340: the discriminant, then the matching arm
        # (several case labels may share one arm), else the default arm, else nothing
        self.fields.reasons.append(f"union {u.name} switches its arms per record "
                                   f"(jrpcgen.java:1240-1340)")
        k = len(self.fields)
        self.decl(u.disc, f"{where}.{u.disc.name}", guard, stack)
        if len(self.fields) != k + 1 or self.fields[k][1] != abi.K_SCALAR or \
                self.fields[k][0] not in self.DISC_TYPES:
            raise NotBatchable(f"{where}: union {u.name} discriminant is not an int / unsigned / "
                               f"enum / bool")
        every = []
        for labels, d in u.arms:
            vals = [self.s.value(v) for v in labels]
            every += vals
            self.decl(d, where, (k, False, vals), stack)
        if u.default is not None:
            self.decl(u.default, where, (k, True, every), stack)

    # ---- repeated groups ---------------------------------------------------------
    def _struct_of(self, t):
        """The Struct a (typedef'd) type name resolves to, or None."""
        d = self.s.types.get(t) if isinstance(t, str) else None
        while isinstance(d, Decl) and d.kind == SCALAR:
            d = self.s.types.get(d.type) if isinstance(d.type, str) else None
        return d if isinstance(d, Struct) else None

    def _list_struct(self, st):
        """Is struct st a list node: its last declaration `st *next`?"""
        return bool(st.decls) and st.decls[-1].kind == OPTIONAL and self._struct_of(st.decls[-1].type) is st

    def group(self, kind, count, st, decls, where, guard, stack):
        """Group field + the element's flattened fields as its members.  The
        group itself may sit under a guard (an array / list in a union arm or
        behind optional data); its members may carry conditions on earlier
        members of the same element (unions and optional data inside an
        element, e.g. READDIRPLUS's post_op_attr).  A fixed array of structs
        inside an element unrolls into its elements' members (decl()); a
        variable-length one or a list inside an element is an inner group
        (its span counted in this group's members), down to GROUP_LEVELS
        levels (the engine's kernels are instantiated per level)."""
        sub = _Tape(self.s, in_element=True, depth=self.depth + 1)
        for d in decls:
            sub.decl(d, f"{where}.{d.name}", None, stack + (st.name,))
        fields, conds = sub.result()
        if self.depth + 1 >= GROUP_LEVELS and any(f[0] == abi.T_GROUP for f in fields):
            raise NotBatchable(f"{where}: elements of {st.name} hold arrays of structs or lists, which "
                               f"would need group level {GROUP_LEVELS + 1} (the engine batches "
                               f"{GROUP_LEVELS} levels)")
        if not fields:
            raise NotBatchable(f"{where}: elements of {st.name} have no fields")
        g = self.add((abi.T_GROUP, kind, count, len(fields)), guard)
        for f in fields:
            self.add(f, None)
        for k, d, neg, vals in conds:   # element-level conditions, in this tape's indices
            self.conds.append((g + 1 + k, g + 1 + d, neg, list(vals)))
        self.fields.reasons.extend(sub.fields.reasons)

    def decl(self, decl, where, guard, stack):
        if decl.kind == VOID:
            return
        st = self._struct_of(decl.type) if decl.kind != SCALAR else None
        if decl.kind == OPTIONAL and st is not None and self._list_struct(st):
            # `T *x` of a list node T: TRUE + element while there is one, then FALSE
            self.group(abi.K_LIST, 0, st, st.decls[:-1], where, guard, stack)
            return
        if decl.kind in (FIXED, DYNAMIC) and st is not None:
            # `T x<>` / `T x[N]` of a struct: the count (dynamic), then the elements.
            # An element of a list node type T is a list head: T's xdrEncode is a
            # do/while over the chain (jrpcgen.java:1103-1121), the head's fields
            # and then xdrEncodeBoolean(next != null) + the next node's fields ...
            # — the head's fields followed by the `T *next` list, which st.decls
            # already ends with (decl() makes it an inner list group).
            if self.in_element and decl.kind == FIXED:
                # `T x[N]` inside a group element: no count word on the wire
                # (jrpcgen.java:856-906, xdrEncodeFixedVector), so the N
                # elements are N consecutive copies of T's declarations,
                # members of the enclosing element like its other fields
                n = self.s.value(decl.size)
                if st.name in stack:
                    raise NotBatchable(f"{where}: {st.name} contains itself (a recursive type has "
                                       f"no bounded tape)")
                if n > self.MAX_UNROLL:
                    raise NotBatchable(f"{where}: {st.name}[{n}] inside a group element (at most "
                                       f"{self.MAX_UNROLL} elements unroll)")
                for j in range(n):
                    for d in st.decls:
                        self.decl(d, f"{where}[{j}].{d.name}", guard, stack + (st.name,))
                return
            self.group(abi.K_FIXED if decl.kind == FIXED else abi.K_DYNAMIC,
                       self.s.value(decl.size) if decl.kind == FIXED else 0, st, st.decls, where, guard, stack)
            return
        if decl.kind == OPTIONAL:
            # T *x: xdrEncodeBoolean(x != null), then x (JrpcgenDeclaration.INDIRECTION)
            self.fields.reasons.append(f"optional data '{decl.type} *{decl.name}' encodes a bool "
                                       f"and then the value or nothing, per record")
            k = self.add((abi.T_BOOL, abi.K_SCALAR, 0), guard)
            t = decl.type
            if isinstance(t, tuple):
                self.add((t[1], abi.K_SCALAR, 0), (k, True, [0]))
            else:
                self.type_(t, where, (k, True, [0]), stack)
            return
        t = decl.type
        if t == "opaque":
            n = self.s.value(decl.size)
            self.add((abi.T_OPAQUE, abi.K_FIXED if decl.kind == FIXED else abi.K_DYNAMIC,
                      n if decl.kind == FIXED else 0), guard)
            return
        if t == "string":
            self.add((abi.T_STRING, abi.K_DYNAMIC, 0), guard)
            return
        if decl.kind == SCALAR:
            if isinstance(t, tuple):
                self.add((t[1], abi.K_SCALAR, 0), guard)
            else:
                self.type_(t, where, guard, stack)
            return
        base = t[1] if isinstance(t, tuple) else self.s._elem(t, where)
        if decl.kind == FIXED:
            self.add((base, abi.K_FIXED, self.s.value(decl.size)), guard)
        else:
            self.add((base, abi.K_DYNAMIC, 0), guard)


# ---- parser ---------------------------------------------------------------------
class _Parser:
    def __init__(self, text):
        self.t = _tokens(text)
        self.i = 0
        self.spec = Spec()

    def peek(self, k=0):
        return self.t[self.i + k][1] if self.i + k < len(self.t) else None

    def next(self):
        if self.i >= len(self.t):
            raise XdrSyntaxError("unexpected end of file")
        self.i += 1
        return self.t[self.i - 1][1]

    def expect(self, s):
        got = self.next()
        if got != s:
            raise XdrSyntaxError(f"expected {s!r}, got {got!r} (token {self.i})")

    def ident(self):
        k, v = self.t[self.i]
        if k != "id":
            raise XdrSyntaxError(f"expected an identifier, got {v!r}")
        self.i += 1
        return v

    def value(self):
        k, v = self.t[self.i]
        self.i += 1
        return _int_literal(v) if k == "num" else v

    def parse(self):
        while self.i < len(self.t):
            kw = self.next()
            if kw == "const":
                name = self.ident()
                self.expect("=")
                self.spec.consts[name] = self.value()
                self.expect(";")
            elif kw == "typedef":
                d = self.declaration()
                self.spec.types[d.name] = d
                self.expect(";")
            elif kw == "enum":
                name = self.ident()
                self.spec.types[name] = self.enum_body(name)
                self.expect(";")
            elif kw == "struct":
                name = self.ident()
                self.spec.types[name] = Struct(name, self.struct_body())
                self.expect(";")
            elif kw == "union":
                name = self.ident()
                self.spec.types[name] = self.union_body(name)
                self.expect(";")
            elif kw in ("program", "PROGRAM"):
                self.program()
            else:
                raise XdrSyntaxError(f"unexpected {kw!r} at top level")
        return self.spec

    def type_spec(self):
        """-> base name, ("unsigned", type id), or a type name."""
        w = self.next()
        if w == "unsigned":
            nxt = self.peek()
            if nxt in ("int", "long", "hyper", "short", "char"):
                self.next()
                if nxt in ("long", "hyper", "short") and self.peek() == "int":
                    self.next()
                return ("unsigned", UNSIGNED[BASE[nxt]])
            return ("unsigned", abi.T_UINT)
        if w in ("long", "hyper", "short") and self.peek() == "int":
            self.next()
        if w in ("struct", "enum", "union"):
            if self.peek() == "{":   # anonymous inline definition
                name = f"_anon{self.i}"
                if w == "struct":
                    self.spec.types[name] = Struct(name, self.struct_body())
                elif w == "enum":
                    self.spec.types[name] = self.enum_body(name)
                else:
                    self.spec.types[name] = self.union_body(name)
                return name
            return self.ident()
        return w

    def declaration(self):
        if self.peek() == "void":
            self.next()
            return Decl(None, "void", VOID)
        if self.peek() in ("opaque", "string"):
            t = self.next()
            name = self.ident()
            if self.peek() == "[":
                self.next()
                size = self.value()
                self.expect("]")
                return Decl(name, t, FIXED, size)
            self.expect("<")
            size = None if self.peek() == ">" else self.value()
            self.expect(">")
            return Decl(name, t, DYNAMIC, size)
        t = self.type_spec()
        if self.peek() == "*":
            self.next()
            return Decl(self.ident(), t, OPTIONAL)
        name = self.ident()
        if self.peek() == "[":
            self.next()
            size = self.value()
            self.expect("]")
            return Decl(name, t, FIXED, size)
        if self.peek() == "<":
            self.next()
            size = None if self.peek() == ">" else self.value()
            self.expect(">")
            return Decl(name, t, DYNAMIC, size)
        return Decl(name, t, SCALAR)

    def enum_body(self, name):
        self.expect("{")
        values = {}
        while True:
            n = self.ident()
            self.expect("=")
            values[n] = self.value()
            if self.next() == "}":
                break
        return Enum(name, values)

    def struct_body(self):
        self.expect("{")
        decls = []
        while self.peek() != "}":
            decls.append(self.declaration())
            self.expect(";")
        self.next()
        return decls

    def union_body(self, name):
        self.expect("switch")
        self.expect("(")
        disc = self.declaration()
        self.expect(")")
        self.expect("{")
        arms, default, values = [], None, []
        while self.peek() != "}":
            w = self.next()
            if w == "case":
                values.append(self.value())
                self.expect(":")
                if self.peek() == "case":
                    continue
                d = self.declaration()
                self.expect(";")
                arms.append((values, d))
                values = []
            elif w == "default":
                self.expect(":")
                default = self.declaration()
                self.expect(";")
            else:
                raise XdrSyntaxError(f"unexpected {w!r} in union {name}")
        self.next()
        return Union(name, disc, arms, default)

    def program(self):
        pname = self.ident()
        self.expect("{")
        versions = {}
        while self.peek() != "}":
            kw = self.next()
            if kw not in ("version", "VERSION"):
                raise XdrSyntaxError(f"expected version, got {kw!r}")
            vname = self.ident()
            self.expect("{")
            procs = []
            while self.peek() != "}":
                rtype = "void" if self.peek() == "void" else None
                if rtype:
                    self.next()
                else:
                    rtype = "string" if self.peek() == "string" else None
                    if rtype:
                        self.next()
                    else:
                        rtype = self.type_spec()
                name = self.ident()
                self.expect("(")
                args = []
                while self.peek() != ")":
                    if self.peek() == "void":
                        self.next()
                    elif self.peek() == "string":
                        self.next()
                        args.append("string")
                    else:
                        args.append(self.type_spec())
                    if self.t[self.i][0] == "id" and self.peek() not in (",", ")"):
                        self.next()   # parameter name
                    if self.peek() == ",":
                        self.next()
                self.expect(")")
                self.expect("=")
                procs.append(Procedure(name, None, rtype, args))
                procs[-1].number = self.value()
                self.expect(";")
            self.next()
            self.expect("=")
            vnum = self.value()
            self.expect(";")
            versions[vname] = (vnum, procs)
        self.next()
        self.expect("=")
        pnum = self.value()
        self.expect(";")
        self.spec.programs[pname] = (pnum, versions)


def parse(text):
    """Parse .x source -> Spec (numbers resolved lazily through Spec.value)."""
    spec = _Parser(text).parse()
    for pname, (pnum, versions) in list(spec.programs.items()):
        vv = {vn: (spec.value(n), [Procedure(p.name, spec.value(p.number), p.result, p.args) for p in ps])
              for vn, (n, ps) in versions.items()}
        spec.programs[pname] = (spec.value(pnum), vv)
    return spec


def parse_file(path):
    with open(path) as f:
        return parse(f.read())
