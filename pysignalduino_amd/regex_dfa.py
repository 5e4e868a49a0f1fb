"""Compile the bank's ``modulematch`` regexes into search DFAs for the device.

The reference filters every MU result with ``re.search(modulematch, payload)``
(sd_protocols/message_unsynced.py:277-280).  The device cannot run Python's
regex engine, so each pattern is compiled here, once per bank, into a
deterministic automaton with *search* semantics (does any match exist?),
over a byte alphabet compressed into equivalence classes shared by all
patterns.  The device walks the payload once: state = trans[state][cls[b]].

Supported syntax = the subset the bank uses plus the usual neighbours:
literals and escapes, ``.``, ``[...]`` classes (ranges, negation), ``(...)``
``(?:...)`` groups, ``|``, ``* + ? {m} {m,} {m,n}`` (lazy suffix accepted:
laziness cannot change whether a match exists), ``^`` and ``$``.  Anything
else raises NotImplementedError at bank-compile time (loud, never a silent
divergence).  ``tests/test_regex_dfa.py`` cross-checks every compiled
pattern against ``re.search`` on random payload-like strings.

``$`` is compiled as end-of-payload only; Python's ``$`` also matches before
a trailing newline, which a payload (bank pre/postamble + hex digits) never
contains -- bank.py asserts that.
"""
from __future__ import annotations

from typing import Dict, FrozenSet, List, Optional, Sequence, Tuple

ANY_BUT_NL = frozenset(b for b in range(256) if b != 10)
DIGITS = frozenset(range(48, 58))
WORD = frozenset(list(range(48, 58)) + list(range(65, 91)) + list(range(97, 123)) + [95])
SPACE = frozenset([9, 10, 11, 12, 13, 32])
ACC_NOW = 1
ACC_END = 2
DEAD = 4   # no match reachable any more from this state


class _Parser:
    def __init__(self, pat: str):
        self.p = pat
        self.i = 0

    def err(self, msg):
        raise NotImplementedError(f"modulematch {self.p!r}: {msg} at {self.i}")

    def peek(self):
        return self.p[self.i] if self.i < len(self.p) else None

    def take(self):
        c = self.p[self.i]
        self.i += 1
        return c

    def parse(self):
        node = self.alt()
        if self.i != len(self.p):
            self.err("unbalanced ')'")
        return node

    def alt(self):
        branches = [self.seq()]
        while self.peek() == "|":
            self.take()
            branches.append(self.seq())
        return ("alt", branches) if len(branches) > 1 else branches[0]

    def seq(self):
        items = []
        while self.peek() is not None and self.peek() not in "|)":
            items.append(self.quant(self.atom()))
        return ("seq", items)

    def _quant_braces(self):
        j = self.p.find("}", self.i)
        if j < 0:
            return None
        body = self.p[self.i + 1:j]
        parts = body.split(",")
        if len(parts) == 1 and parts[0].isdigit():
            m = n = int(parts[0])
        elif len(parts) == 2 and (parts[0] == "" or parts[0].isdigit()) and (parts[1] == "" or parts[1].isdigit()):
            m = int(parts[0]) if parts[0] else 0
            n = int(parts[1]) if parts[1] else None
        else:
            return None
        self.i = j + 1
        return m, n

    def quant(self, node):
        while True:
            c = self.peek()
            if c == "*":
                self.take()
                node = ("rep", node, 0, None)
            elif c == "+":
                self.take()
                node = ("rep", node, 1, None)
            elif c == "?":
                self.take()
                node = ("rep", node, 0, 1)
            elif c == "{":
                q = self._quant_braces()
                if q is None:
                    return node  # literal '{' handled by the next atom()
                node = ("rep", node, q[0], q[1])
            else:
                return node
            if self.peek() == "?":  # lazy form: same match existence
                self.take()

    def _escape_set(self, c):
        table = {"d": DIGITS, "w": WORD, "s": SPACE}
        if c in table:
            return table[c]
        if c.lower() in table and c.isupper():
            return frozenset(range(256)) - table[c.lower()]
        if c in "nrtfv":
            return frozenset([{"n": 10, "r": 13, "t": 9, "f": 12, "v": 11}[c]])
        if c.isalnum():
            self.err(f"unsupported escape \\{c}")
        return frozenset([ord(c)])

    def atom(self):
        c = self.take()
        if c == "(":
            if self.p.startswith("?:", self.i):
                self.i += 2
            elif self.peek() == "?":
                self.err("unsupported group extension")
            node = self.alt()
            if self.peek() != ")":
                self.err("missing ')'")
            self.take()
            return node
        if c == ".":
            return ("set", ANY_BUT_NL)
        if c == "^":
            return ("bol",)
        if c == "$":
            return ("eol",)
        if c == "[":
            return ("set", self.cls())
        if c == "\\":
            if self.peek() is None:
                self.err("trailing backslash")
            return ("set", self._escape_set(self.take()))
        if c in "*+?":
            self.err("nothing to repeat")
        if ord(c) > 255:
            self.err("non-latin-1 literal")
        return ("set", frozenset([ord(c)]))

    def cls(self):
        neg = False
        if self.peek() == "^":
            self.take()
            neg = True
        members = set()
        first = True
        while True:
            c = self.peek()
            if c is None:
                self.err("unterminated class")
            if c == "]" and not first:
                self.take()
                break
            first = False
            self.take()
            if c == "\\":
                lo_set = self._escape_set(self.take())
            else:
                lo_set = frozenset([ord(c)])
            if self.peek() == "-" and self.i + 1 < len(self.p) and self.p[self.i + 1] != "]" and len(lo_set) == 1:
                self.take()
                hc = self.take()
                if hc == "\\":
                    hs = self._escape_set(self.take())
                    if len(hs) != 1:
                        self.err("bad range")
                    hi = next(iter(hs))
                else:
                    hi = ord(hc)
                lo = next(iter(lo_set))
                if hi < lo:
                    self.err("bad range")
                members.update(range(lo, hi + 1))
            else:
                members.update(lo_set)
        s = frozenset(b for b in members if b < 256)
        return frozenset(range(256)) - s if neg else s


class _Nfa:
    def __init__(self):
        self.edges: List[List[Tuple[str, object, int]]] = []

    def new(self):
        self.edges.append([])
        return len(self.edges) - 1

    def add(self, a, kind, arg, b):
        self.edges[a].append((kind, arg, b))

    def build(self, node, a, b):
        """Thompson construction: wire ``node`` between states a -> b."""
        t = node[0]
        if t == "set":
            self.add(a, "c", node[1], b)
        elif t == "bol":
            self.add(a, "bol", None, b)
        elif t == "eol":
            self.add(a, "eol", None, b)
        elif t == "seq":
            cur = a
            for it in node[1]:
                nxt = self.new()
                self.build(it, cur, nxt)
                cur = nxt
            self.add(cur, "e", None, b)
        elif t == "alt":
            for br in node[1]:
                self.build(br, a, b)
        elif t == "rep":
            _, sub, m, n = node
            cur = a
            for _ in range(m):
                nxt = self.new()
                self.build(sub, cur, nxt)
                cur = nxt
            if n is None:
                loop = self.new()
                self.add(cur, "e", None, loop)
                body_end = self.new()
                self.build(sub, loop, body_end)
                self.add(body_end, "e", None, loop)
                self.add(loop, "e", None, b)
            else:
                self.add(cur, "e", None, b)
                for _ in range(n - m):
                    nxt = self.new()
                    self.build(sub, cur, nxt)
                    self.add(nxt, "e", None, b)
                    cur = nxt
        else:  # pragma: no cover
            raise NotImplementedError(t)

    def closure(self, states, at_start, at_end) -> FrozenSet[int]:
        seen = set(states)
        stack = list(states)
        while stack:
            s = stack.pop()
            for kind, _, d in self.edges[s]:
                ok = kind == "e" or (kind == "bol" and at_start) or (kind == "eol" and at_end)
                if ok and d not in seen:
                    seen.add(d)
                    stack.append(d)
        return frozenset(seen)


class CompiledDfa:
    def __init__(self, pattern: str, charsets: List[FrozenSet[int]], nstates: int, start: int,
                 trans: List[List[int]], flags: List[int], set_trans):
        self.pattern = pattern
        self.charsets = charsets
        self.nstates = nstates
        self.start = start
        self.set_trans = set_trans   # per state: list of (charset index, next state) + default
        self.flags = flags

    def search(self, s: bytes, cls_of: Sequence[int], table: List[List[int]]) -> bool:
        st = self.start
        if self.flags[st] & ACC_NOW:
            return True
        for b in s:
            st = table[st][cls_of[b]]
            if self.flags[st] & ACC_NOW:
                return True
        return bool(self.flags[st] & ACC_END)


def compile_pattern(pattern: str):
    """Return (charsets used, per-state transition function on bytes, flags, start)."""
    ast = _Parser(pattern).parse()
    nfa = _Nfa()
    s0 = nfa.new()
    fin = nfa.new()
    nfa.build(ast, s0, fin)
    charsets = sorted({arg for es in nfa.edges for k, arg, _ in es if k == "c"}, key=lambda x: sorted(x))

    # subset construction; key = (nfa set, is_position_0)
    states: Dict[Tuple[FrozenSet[int], bool], int] = {}
    order: List[Tuple[FrozenSet[int], bool]] = []
    ACCEPT = ("ACCEPT", False)

    def intern(key):
        if key not in states:
            states[key] = len(order)
            order.append(key)
        return states[key]

    init = (nfa.closure([s0], True, False), True)
    intern(init)
    trans_by_byte: List[Optional[List[int]]] = []
    flags: List[int] = []
    k = 0
    while k < len(order):
        key = order[k]
        if key == ACCEPT:
            flags.append(ACC_NOW | ACC_END)
            trans_by_byte.append(None)  # absorbing
            k += 1
            continue
        sset, pos0 = key
        f = 0
        if fin in sset:
            f |= ACC_NOW | ACC_END
        elif fin in nfa.closure(sset, pos0, True):
            f |= ACC_END
        flags.append(f)
        if f & ACC_NOW:
            trans_by_byte.append(None)
            k += 1
            continue
        row = []
        cache: Dict[FrozenSet[int], int] = {}
        for b in range(256):
            moved = {d for s in sset for kind, arg, d in nfa.edges[s] if kind == "c" and b in arg}
            nxt = nfa.closure(list(moved) + [s0], False, False)
            if fin in nxt:
                row.append(intern(ACCEPT))
            else:
                if nxt not in cache:
                    cache[nxt] = intern((nxt, False))
                row.append(cache[nxt])
        trans_by_byte.append(row)
        k += 1
    n = len(order)
    acc = states.get(ACCEPT)
    full = []
    for i in range(n):
        full.append(trans_by_byte[i] if trans_by_byte[i] is not None else [i] * 256)
    return charsets, full, flags, 0, acc


def compile_bank_dfas(patterns: Sequence[str]):
    """Compile all patterns over one shared byte-class alphabet.

    Returns (cls_of[256] -> class id, n_class, list of (nstates, start, trans[nstates][n_class], flags)).
    """
    compiled = [compile_pattern(p) for p in patterns]
    # byte equivalence: two bytes are equivalent iff every DFA row treats them the same
    sig: Dict[Tuple, int] = {}
    cls_of = [0] * 256
    for b in range(256):
        key = tuple(tuple(row[b] for row in c[1]) for c in compiled)
        if key not in sig:
            sig[key] = len(sig)
        cls_of[b] = sig[key]
    n_class = len(sig)
    rep = [0] * n_class
    for b in range(255, -1, -1):
        rep[cls_of[b]] = b
    out = []
    for (_, full, flags, start, _acc) in compiled:
        trans = [[row[rep[c]] for c in range(n_class)] for row in full]
        n = len(full)
        live = [bool(f & (ACC_NOW | ACC_END)) for f in flags]
        changed = True
        while changed:
            changed = False
            for i in range(n):
                if not live[i] and any(live[j] for j in trans[i]):
                    live[i] = True
                    changed = True
        flags = [f | (0 if live[i] else DEAD) for i, f in enumerate(flags)]
        out.append((n, start, trans, flags))
    return cls_of, n_class, out


def dfa_walk(dfa, cls_of, start_state: int, payload: bytes) -> int:
    """State after consuming ``payload`` (stops early in an accepting or dead state)."""
    _, _, trans, flags = dfa
    st = start_state
    for b in payload:
        if flags[st] & (ACC_NOW | DEAD):
            break
        st = trans[st][cls_of[b]]
    return st


def dfa_search(dfa, cls_of, payload: bytes) -> bool:
    nstates, start, trans, flags = dfa
    st = start
    if flags[st] & ACC_NOW:
        return True
    for b in payload:
        st = trans[st][cls_of[b]]
        if flags[st] & ACC_NOW:
            return True
    return bool(flags[st] & ACC_END)
