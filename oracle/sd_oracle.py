"""ORACLE -- CPU restatement of the reference MU/MS/MC demodulation path.

*** TEST INFRASTRUCTURE ONLY ***
Only ``tests/``, ``__graft_entry__.smoke()`` and the ``cpu_baseline`` leg of
``bench.py`` may import this module, and only as the CHECKER (or the timed CPU
baseline).  The product path (``pysignalduino_amd``) never imports it and has
no CPU fallback: it fails loudly when the HIP library is missing.

Parity pinning: this restatement is checked against the golden vectors in
``tests/golden/*.json.gz``, which were produced by running the reference
implementation itself (``tests/golden/make_golden.py``) on the reference's own
test inputs, seeded synthetic corpora and edge cases.  See
``tests/test_oracle_golden.py``.

Every function cites the reference file:line it restates (paths relative to
the RFD-FHEM/PySignalduino checkout).  Observable behaviour, including the
reference's bugs and exception types, is reproduced on purpose.
"""
from __future__ import annotations

import itertools
import json
import os
import re
from typing import Any, Dict, List, Optional, Sequence, Tuple

BANK_PATH = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                         "pysignalduino_amd", "data", "sd_bank.json")


# ---------------------------------------------------------------------------------------------
# bank (sd_protocols/sd_protocols.py:30-58,157-160)
# ---------------------------------------------------------------------------------------------
class OracleBank:
    def __init__(self, protocols: Optional[Dict[str, dict]] = None):
        if protocols is None:
            with open(BANK_PATH, encoding="utf-8") as f:
                protocols = json.load(f)["protocols"]
        self.p: Dict[str, dict] = {k: dict(v) for k, v in protocols.items()}
        for pid, props in self.p.items():               # set_defaults :157-160
            props.setdefault("active", True)
            props.setdefault("name", f"Protocol_{pid}")

    def ids_with(self, key: str) -> List[str]:          # get_keys :49-52
        return [pid for pid, props in self.p.items() if key in props]

    def prop(self, pid: str, key: str, default=None):   # check_property :54-55
        return self.p.get(pid, {}).get(key, default)


# ---------------------------------------------------------------------------------------------
# helpers (sd_protocols/helpers.py)
# ---------------------------------------------------------------------------------------------
def bits_to_hex(bits: Optional[str]) -> Optional[str]:
    """helpers.py:28-64 -- nibbles taken from the right, leading partial nibble kept."""
    if bits is None:
        return None
    if not bits:
        return ""
    if not isinstance(bits, str) or any(c not in "01" for c in bits):
        return None
    digits = []
    end = len(bits)
    while end > 0:
        beg = max(0, end - 4)
        digits.append("%X" % int(bits[beg:end], 2))
        end -= 4
    return "".join(reversed(digits))


def hex_to_bits(h: Optional[str]) -> Optional[str]:
    """helpers.py:168-188 -- bin(int(h,16)) zero-filled to a multiple of 4 (leading zero nibbles lost)."""
    if h is None:
        return None
    try:
        v = int(h, 16)
    except ValueError:
        return None
    b = format(v, "b")
    width = -(-len(b) // 4) * 4
    return b.rjust(width, "0")


def mc_to_dmc(bits: Optional[str]):
    """helpers.py:6-26."""
    if bits is None:
        return (-1, "no bitData provided")
    s = bits.replace("1", "lh").replace("0", "hl")
    return "".join("0" if s[i] == s[i + 1] else "1" for i in range(1, len(s) - 1, 2))


def length_in_range(bank: OracleBank, pid, n: int) -> Tuple[int, str]:
    """helpers.py:124-166."""
    if str(pid) not in bank.p:
        return (0, "protocol does not exists")
    lo = bank.prop(pid, "length_min", -1)
    if lo is not None:
        try:
            lo = int(lo)
        except (ValueError, TypeError):
            pass
    if lo != -1 and n < lo:
        return (0, "message is too short")
    hi = bank.p.get(pid, {}).get("length_max")
    if hi is not None:
        try:
            if n > int(hi):
                return (0, "message is too long")
        except (ValueError, TypeError):
            pass
    return (1, "")


# ---------------------------------------------------------------------------------------------
# pattern matcher (sd_protocols/pattern_utils.py:15-136)
# ---------------------------------------------------------------------------------------------
def tolerance(v: float) -> float:
    """pattern_utils.py:15-26."""
    a = abs(v)
    if a > 16:
        return a * 0.18
    if a > 3:
        return a * 0.3
    return 1.0


def pattern_exists(search: Sequence[float], table: Dict[str, float], data: str):
    """pattern_utils.py:34-136: first id-assignment (product order, gap-sorted
    candidates, no id reused) whose concatenation occurs in ``data``; else -1."""
    order: List[float] = []
    for v in search:
        if v not in order:
            order.append(v)
    cand_lists = []
    for v in order:
        tol = tolerance(v)
        scored = [(abs(pv - v), k) for k, pv in table.items() if abs(pv - v) <= 0.001 or abs(pv - v) <= tol]
        if not scored:
            return -1
        scored.sort(key=lambda t: t[0])
        cand_lists.append([k for _, k in scored])
    n = 1
    for c in cand_lists:
        n *= len(c)
    if n > 10000:
        return -1
    for combo in itertools.product(*cand_lists):
        if len(set(combo)) != len(combo):
            continue
        assign = dict(zip(order, combo))
        target = "".join(assign[v] for v in search)
        if target in data:
            return target
    return -1


def _patterns(msg: Dict[str, Any]) -> Dict[str, float]:
    """message_unsynced.py:28-35 / message_synced.py:50-57."""
    out: Dict[str, float] = {}
    for k, v in msg.items():
        if k.startswith("P") and k[1:].isdigit():
            try:
                out[str(int(k[1:]))] = float(v)
            except ValueError:
                pass
    return out


def _floats(seq):
    return [float(x) for x in seq]


_SYM = {"one": "1", "zero": "0", "float": "F", "sync": ""}


# ---------------------------------------------------------------------------------------------
# postDemodulation (sd_protocols/postdemodulation.py:27-730)
# ---------------------------------------------------------------------------------------------
def _b2i(bits) -> int:
    return int("".join(str(b) for b in bits), 2)


def pd_em(bits):
    """postdemodulation.py:27-88."""
    s = "".join(str(b) for b in bits)
    p = s.find("0000000001")
    if p < 0:
        return (0, None)
    s = s[p + 10:]
    n = len(s)
    if n != 89:
        return (0, None)
    out, crc = [], 0
    for c in range(0, n, 9):
        if c + 8 < n:
            byte = s[c:c + 8]
            if c < n - 10:
                out.extend(int(b) for b in reversed(byte))
                crc ^= int(byte, 2)
    return (1, out) if crc == int(s[n - 8:n], 2) else (0, None)


def pd_revolt(bits):
    """postdemodulation.py:90-137."""
    if len(bits) < 96:
        return (0, None)
    chk = _b2i(bits[88:96])
    tot = sum(_b2i(bits[b:b + 8]) for b in range(0, 88, 8)) & 0xFF
    return (1, list(bits[0:88])) if tot == chk else (0, None)


def _first_one(bits):
    for i, b in enumerate(bits):
        if b == 1:
            return i
    return None


def pd_fs20(bits):
    """postdemodulation.py:139-243."""
    st = _first_one(bits)
    if st is None:
        return (0, None)
    m = list(bits[st + 1:])
    n = len(m)
    if n in (46, 55):
        m.pop()
        n -= 1
    if n not in (45, 54):
        return (0, None)
    s = 6 + sum(_b2i(m[b:b + 8]) for b in range(0, n - 9, 9))
    chk = _b2i(m[n - 9:n - 1])
    if (s + 6) & 0xFF == chk:
        return (0, None)
    if s & 0xFF != chk:
        return (0, None)
    for b in range(0, n, 9):
        if sum(m[b:min(b + 9, n)]) % 2:
            return (0, None)
    for b in range(n - 1, 0, -9):
        m.pop(b)
    if n == 45:
        del m[32:40]
        m[24:24] = [0] * 8
    else:
        del m[40:48]
    return (1, m)


def pd_fht80(bits):
    """postdemodulation.py:245-337."""
    st = _first_one(bits)
    if st is None:
        return (0, None)
    m = list(bits[st + 1:])
    n = len(m)
    if n == 55:
        m.pop()
        n -= 1
    if n != 54:
        return (0, None)
    s = 12 + sum(_b2i(m[b:b + 8]) for b in range(0, 45, 9))
    chk = _b2i(m[45:53])
    if ((s - 6) & 0xFF) == chk:
        return (0, None)
    if (s & 0xFF) != chk:
        return (0, None)
    for b in range(0, 54, 9):
        if sum(m[b:min(b + 9, 54)]) % 2:
            return (0, None)
    for b in range(53, 0, -9):
        m.pop(b)
    return (1, m)


def pd_fht80tf(bits):
    """postdemodulation.py:339-423."""
    if len(bits) < 46:
        return (0, None)
    st = _first_one(bits)
    if st is None:
        return (0, None)
    m = list(bits[st + 1:])
    if len(m) != 45:
        return (0, None)
    s = 12 + sum(_b2i(m[b:b + 8]) for b in range(0, 36, 9))
    if (s & 0xFF) != _b2i(m[36:44]):
        return (0, None)
    for b in range(0, 45, 9):
        if sum(m[b:min(b + 9, 45)]) % 2:
            return (0, None)
    for b in range(44, 0, -9):
        m.pop(b)
    if m[26] != 0:
        return (0, None)
    del m[32:40]
    return (1, m)


_WS2000_LEN = [35, 50, 35, 50, 70, 40, 40, 85]


def pd_ws2000(bits):
    """postdemodulation.py:425-578."""
    n = len(bits)
    st = _first_one(bits)
    if st is None:
        return (0, None)
    dlen = n - st
    dlen1 = dlen - dlen % 5
    typ = int("".join(str(b) for b in reversed(bits[st + 1:st + 5])), 2)
    if typ > 7:
        return (0, None)
    if typ == 1 and dlen in (45, 46):
        dlen1 += 5
    if _WS2000_LEN[typ] != dlen1 or st > 10:
        return (0, None)
    idx = 0
    didx = 0
    check = 0
    acc = 5
    while idx < dlen - 1:
        if bits[idx + st] != 1:
            return (0, None)
        didx = idx + st + 1
        if n - didx < 4:
            return (0, None)
        nib = int("".join(str(b) for b in reversed(bits[didx:didx + 4])), 2)
        if dlen in (45, 46):
            if idx <= dlen - 5:
                check ^= nib
        elif idx <= dlen - 10:
            check ^= nib
            acc += nib
        idx += 5
    if check != 0:
        return (0, None)
    if dlen < 45 or dlen > 46:
        nib = int("".join(str(b) for b in reversed(bits[didx:didx + 4])), 2)
        if nib != (acc & 0x0F):
            return (0, None)
    d = st + 1

    def rv(a, b):
        return list(reversed(bits[d + a:d + b]))

    out = [0] * 16
    out[0:4] = rv(5, 9)
    out[4:8] = rv(0, 4)
    out[8:12] = rv(15, 19)
    out[12:16] = rv(10, 14)
    if typ in (0, 2):
        out += rv(20, 24)
    elif typ in (1, 3, 4, 7):
        out += rv(25, 29) + rv(20, 24) + rv(35, 39) + rv(30, 34)
        if typ == 4:
            out += rv(55, 59) + rv(50, 54) + rv(45, 49) + rv(40, 44)
    return (1, out)


def pd_ws7035(bits):
    """postdemodulation.py:580-640."""
    s = "".join(str(b) for b in bits)
    if not s.startswith("10100000") or len(s) != 44:
        return (0, None)
    if sum(int(s[i]) for i in range(15, 28)) % 2:
        return (0, None)
    if sum(int(s[i:i + 4], 2) for i in range(0, 40, 4)) % 16 != int(s[40:], 2):
        return (0, None)
    return (1, [int(c) for i, c in enumerate(s) if not 27 <= i < 31])


def pd_ws7053(bits):
    """postdemodulation.py:642-706."""
    s = "".join(str(b) for b in bits)
    p = s.find("10100000")
    if p > 0:
        s = s[p:] + "0"
    if p < 0 or len(s) < 32:
        return (0, None)
    if sum(int(s[i]) for i in range(15, 28)) % 2:
        return (0, None)
    return (1, [int(c) for c in s[0:28] + s[16:24] + s[28:32]])


def pd_lenprefix(bits):
    """postdemodulation.py:708-730."""
    s = "".join(str(b) for b in bits)
    return (1, [int(c) for c in format(len(s), "08b") + s])


POSTDEMO = {
    "postDemo_EM": pd_em, "postDemo_Revolt": pd_revolt, "postDemo_FS20": pd_fs20,
    "postDemo_FHT80": pd_fht80, "postDemo_FHT80TF": pd_fht80tf, "postDemo_WS2000": pd_ws2000,
    "postDemo_WS7035": pd_ws7035, "postDemo_WS7053": pd_ws7053, "postDemo_lengtnPrefix": pd_lenprefix,
}


def _postdemo_fn(bank: OracleBank, pid: str):
    name = bank.prop(pid, "postDemodulation", None)
    if not name:
        return None
    return POSTDEMO.get(name.split(".")[-1])  # a missing method is silently skipped


# ---------------------------------------------------------------------------------------------
# MU (sd_protocols/message_unsynced.py:11-296)
# ---------------------------------------------------------------------------------------------
def demod_mu(bank: OracleBank, msg: Dict[str, Any]) -> List[dict]:
    data = msg.get("data", "")
    if not data:
        return []
    praw = _patterns(msg)
    results: List[dict] = []
    for pid in bank.ids_with("clockabs"):
        if not bank.prop(pid, "active", True):
            continue
        clock = float(bank.prop(pid, "clockabs", 1))
        norm = {k: round(v / clock, 1) for k, v in praw.items()}
        work = data
        start_lit = ""
        sp = bank.p[pid].get("start")
        if sp and isinstance(sp, list):
            hit = pattern_exists(_floats(sp), norm, work)
            if hit == -1:
                continue
            start_lit = str(hit)
            work = work[work.find(start_lit):]
        sym_of: Dict[str, str] = {}
        tail_sym: Dict[str, str] = {}
        units: List[str] = []
        bad = False
        for key in ("one", "zero", "float"):
            spec = bank.p[pid].get(key)
            if not spec:
                continue
            try:
                sv = _floats(spec)
            except (ValueError, TypeError):
                bad = True
                break
            hit = pattern_exists(sv, norm, work)
            if hit == -1:
                if key != "float":
                    bad = True
                    break
                continue
            hit = str(hit)
            sym_of[hit] = _SYM[key]
            if hit and hit[:-1] not in tail_sym:
                tail_sym[hit[:-1]] = _SYM[key]
            units.append(hit)
        if bad or not units:
            continue
        recon = bank.p[pid].get("reconstructBit")
        tail_re = ""
        if recon and tail_sym:
            tail_re = "(?:" + "|".join(re.escape(k) for k in tail_sym) + ")?"
        lmin = bank.prop(pid, "length_min", 0)
        # alternation over the DISTINCT unit strings (the reference's prefix factoring at
        # message_unsynced.py:153-171 is language-equivalent and dedups the same way; a
        # duplicated branch only adds exponential backtracking, never a different match)
        alts = "|".join(re.escape(u) for u in sym_of)
        rx = re.compile(f"(?:{re.escape(start_lit)})((?:{alts}){{{lmin},}}{tail_re})")
        for mt in rx.finditer(work):
            grp = mt.group(1)
            lmax = bank.prop(pid, "length_max", None)
            one = bank.p[pid].get("one")
            width = len(one) if one else 0
            if width == 0:
                continue
            chunks = [grp[i:i + width] for i in range(0, len(grp), width)]
            chunks[-1]  # noqa: B018 -- IndexError on an empty group, as message_unsynced.py:212
            if lmax and len(chunks) > int(lmax):
                continue
            bits = []
            for ch in chunks:
                if ch in sym_of:
                    bits.append(sym_of[ch])
                elif recon and ch in tail_sym:
                    bits.append(tail_sym[ch])
            fn = _postdemo_fn(bank, pid)
            if fn is not None:
                try:
                    ints = [int(b) for b in bits]
                    rc, ret = fn(ints)
                    if rc < 1:
                        continue
                    bits = [str(b) for b in ret]
                except ValueError:
                    pass
            dispatch_bin = int(bank.prop(pid, "dispatchBin", 0))
            pad = int(bank.prop(pid, "paddingbits", 4))
            while len(bits) % pad > 0:
                bits.append("0")
            bstr = "".join(bits)
            if dispatch_bin == 1:
                dmsg = bstr
            else:
                dmsg = bits_to_hex(bstr)
                if bank.prop(pid, "remove_zero", 0):
                    dmsg = dmsg.lstrip("0")  # AttributeError on None, as :269
            payload = f"{bank.prop(pid, 'preamble', '')}{dmsg}{bank.prop(pid, 'postamble', '')}"
            mm = bank.prop(pid, "modulematch")
            if mm and not re.search(mm, payload):
                continue
            results.append({"protocol_id": pid, "payload": payload,
                            "meta": {"bit_length": len(bstr), "rssi": msg.get("R"), "clock": clock}})
    return results


# ---------------------------------------------------------------------------------------------
# MS (sd_protocols/message_synced.py:10-243)
# ---------------------------------------------------------------------------------------------
def demod_ms(bank: OracleBank, msg: Dict[str, Any]) -> List[dict]:
    data = msg.get("data", "")
    if not data or not data.isdigit():
        return []
    cp = msg.get("CP", "")
    if not cp or not cp.isdigit():
        return []
    sp = msg.get("SP", "")
    if not sp or not sp.isdigit():
        return []
    if "R" in msg and not msg.get("R", "").isdigit():
        return []
    praw = _patterns(msg)
    cpk = str(int(cp))
    if cpk not in praw:
        return []
    clock = abs(praw[cpk])
    if clock == 0:
        return []
    norm = {k: round(v / clock, 1) for k, v in praw.items()}
    out: List[dict] = []
    for pid in bank.ids_with("sync"):
        pclk = float(bank.prop(pid, "clockabs", 0))
        if pclk > 0 and abs(pclk - clock) > clock * 0.3:
            continue
        props = bank.p[pid]
        width = len(props["one"]) if props.get("one") else 0
        sym_of: Dict[str, str] = {}
        tail_sym: Dict[str, str] = {}
        start = 0
        bad = False
        for key in ("sync", "one", "zero", "float"):
            spec = props.get(key)
            if not spec:
                continue
            try:
                sv = _floats(spec)
            except (ValueError, TypeError):
                bad = True
                break
            hit = pattern_exists(sv, norm, data)
            if hit == -1:
                if key != "float":
                    bad = True
                    break
                continue
            sym_of[hit] = _SYM[key]
            if hit and hit[:-1] not in tail_sym:
                tail_sym[hit[:-1]] = _SYM[key]
            if key == "sync":
                start = data.find(str(hit)) + len(str(hit))
                avail = (len(data) - start) / width if width > 0 else 0
                if int(bank.prop(pid, "length_min", -1)) > avail:
                    bad = True
                    break
                tail_sym = {}
        if bad or not sym_of:
            continue
        recon = props.get("reconstructBit")
        bits: List[str] = []
        for i in range(start, len(data), width):
            ch = data[i:i + width]
            if ch in sym_of:
                if sym_of[ch]:
                    bits.append(sym_of[ch])
            elif recon:
                key = ch[:-1] if len(ch) == width else ch
                if key in tail_sym:
                    bits.append(tail_sym[key])
                else:
                    break
            else:
                break
        if not bits:
            continue
        if not length_in_range(bank, pid, len(bits))[0]:
            continue
        pad = int(bank.prop(pid, "paddingbits", 4))
        while len(bits) % pad > 0:
            bits.append("0")
        fn = _postdemo_fn(bank, pid)
        if fn is not None:
            rc, ret = fn([int(b) for b in bits])   # no try: 'F' raises ValueError (:209)
            if rc < 1:
                continue
            if ret:
                bits = [str(b) for b in ret]
        bstr = "".join(bits)
        hx = bits_to_hex(bstr)
        if hx is None:
            continue
        out.append({"protocol_id": pid,
                    "payload": f"{bank.prop(pid, 'preamble', '')}{hx}{bank.prop(pid, 'postamble', '')}",
                    "meta": {"bit_length": len(bstr), "rssi": msg.get("R"), "clock": clock}})
    return out


# ---------------------------------------------------------------------------------------------
# MC (sd_protocols/manchester.py)
# ---------------------------------------------------------------------------------------------
def _lmin(bank, pid, d):
    return int(bank.prop(pid, "length_min", d))


def _lmax(bank, pid, d):
    return int(bank.prop(pid, "length_max", d))


def _gate(bank, pid, n):
    if n < _lmin(bank, pid, -1):
        return (-1, "message is too short")
    if n > _lmax(bank, pid, 9999):
        return (-1, "message is too long")
    return None


def mc_funkbus(bank, bits, pid, n):
    """manchester.py:207-300."""
    if n < _lmin(bank, pid, -1):
        return (-1, "message is too short")
    lm = bank.p.get(pid, {}).get("length_max")
    if lm is not None and n > int(lm):
        return (-1, "message is too long")
    dm = mc_to_dmc(bits.replace("1", "lh").replace("0", "hl"))
    if int(pid) == 119:
        p = dm.find("01100")
        if not 0 <= p < 5:
            return (-1, "wrong bits at begin")
        dm = "001" + dm[p:]
        if len(dm) < 48:
            return (-1, "wrong bits at begin")
    else:
        dm = "0" + dm
    hx, x, chk, par = "", 0, 0, 0
    for i in range(6):
        d = int(dm[i * 8:(i + 1) * 8], 2)
        hx += "%02X" % d
        if i < 5:
            x ^= d
        else:
            chk = d & 0x0F
            x ^= d & 0xE0
            d &= 0xF0
        par ^= bin(d).count("1") & 1
    if par == 1:
        return (-1, "parity error")
    nib = ((x & 0xF0) >> 4) ^ (x & 0x0F)
    r = (0xC if nib & 8 else 0) ^ (0x2 if nib & 4 else 0) ^ (0x8 if nib & 2 else 0) ^ (0x3 if nib & 1 else 0)
    if r != chk:
        return (-1, "checksum error")
    return (1, hx)


def mc_sainlogic(bank, bits, pid, n):
    """manchester.py:302-354."""
    if n > _lmax(bank, pid, 0):
        return (-1, "message is too long")
    if n < 128:
        st = bits.find("010100")
        if st < 0 or st > 10:
            return (-1, "start 010100 not found")
        bits = "1" * (10 - st) + bits if st < 10 else bits
        bits = bits[:128]
        n = len(bits)
    if n < _lmin(bank, pid, 0):
        return (-1, "message is too short")
    return (1, bits_to_hex(bits))


def mc_as(bank, bits, pid, n):
    """manchester.py:356-416."""
    st = bits.find("1100", 16)
    if st >= 0:
        en = bits.find("1100", st + 16)
        if en == -1:
            en = len(bits)
        g = _gate(bank, pid, en - st)
        return g if g else (1, bits_to_hex(bits[st:]))
    g = _gate(bank, pid, n)
    return g if g else (1, bits_to_hex(bits))


def mc_plain(bank, bits, pid, n):
    """manchester.py:418-586 (Hideki, Maverick, OSV1, OSV2o3, OSPIR): length gate + hex."""
    g = _gate(bank, pid, n)
    return g if g else (1, bits_to_hex(bits))


def mc_raw(bank, bits, pid, n, _other=None):
    """manchester.py:588-613 (mcRaw)."""
    if int(n) > _lmax(bank, pid, 0):
        return (-1, "message is too long")
    return (1, bits_to_hex(bits))


def helpers_mcraw(bank, bits, pid, n):
    """helpers.py:90-122 (mcraw): length_max is compared un-converted -> TypeError on str."""
    if bits is None:
        return (-1, "no bitData provided")
    if pid is None:
        return (-1, "no protocolId provided")
    if n is None:
        n = len(bits)
    mx = bank.p.get(pid, {}).get("length_max")
    if mx is not None and n > mx:
        return (-1, "message is to long")
    h = bits_to_hex(bits)
    if h is None:
        return (-1, "invalid bit data")
    return (1, h)


def mc_tfa(bank, bits, pid, n):
    """manchester.py:615-719: repeated-frame scan, returns the LIST of duplicate frames."""
    p0 = bits.find("111111111101")
    if p0 == -1:
        return (-1, "sync not found")
    pos = p0 + 12
    end = -1
    msgs: List[str] = []
    tail = ""
    loops = 1
    while end < n:
        end = bits.find("1111111111101", pos)
        if end < pos:
            end = n
        ok, why = length_in_range(bank, pid, end - pos)
        if ok:
            msgs.append(bits_to_hex(bits[pos:end]))
        else:
            tail = ", " + why
        nxt = bits.find("1101", end)
        if nxt != -1:
            pos = nxt + 4
        else:
            end = n
        loops += 1
    if loops == 10:
        return (-1, "loop error, please report this data " + bits)
    cnt: Dict[str, int] = {}
    dups = []
    for m in msgs:
        if cnt.get(m, 0) == 1:
            dups.append(m)
        cnt[m] = cnt.get(m, 0) + 1
    return (1, dups) if dups else (-1, " no duplicate found" + tail)


def mc_grothe(bank, bits, pid, n):
    """manchester.py:721-754."""
    if n != 32:
        return (-1, f"message must be 32 bits, got {n}")
    return (1, bits_to_hex(bits))


def mc_somfy(bank, bits, pid, n):
    """manchester.py:756-795."""
    if n == 57:
        bits = bits[1:57]
    if len(bits) != 56:
        return (-1, f"message must be 56 bits, got {len(bits)}")
    return (1, bits_to_hex(bits))


MC_METHODS = {
    "mcBit2Funkbus": mc_funkbus, "mcBit2Sainlogic": mc_sainlogic, "mcBit2AS": mc_as,
    "mcBit2Hideki": mc_plain, "mcBit2Maverick": mc_plain, "mcBit2OSV1": mc_plain, "mcBit2OSV2o3": mc_plain,
    "mcBit2OSPIR": mc_plain, "mcRaw": mc_raw, "mcraw": helpers_mcraw, "mcBit2TFA": mc_tfa,
    "mcBit2Grothe": mc_grothe, "mcBit2SomfyRTS": mc_somfy,
}


def mc_method(bank: OracleBank, pid: str, bits: str, n: int):
    name = bank.prop(pid, "method").split(".")[-1]
    return MC_METHODS[name](bank, bits, pid, n)


def demod_mc_fixed_one(bank: OracleBank, pid: str, raw_hex: str, clock, mcbitnum, mtype: str,
                       version: Optional[str]):
    """manchester.py:49-144 with the two documented fixes (SURVEY §8(a) A7 'fixed' mode):
    clockrange[0] < clock < clockrange[1], and the method called without the extra self."""
    if mcbitnum < _lmin(bank, pid, -1):
        return None
    if mcbitnum > _lmax(bank, pid, 9999):
        return None
    cr = bank.p[pid].get("clockrange")
    if cr and len(cr) >= 2 and not (clock > cr[0] and clock < cr[1]):
        return None
    inv = bank.prop(pid, "polarity", "") == "invert"
    if mtype == "Mc" or (version and version[:6] == "V 3.2."):
        inv = not inv
    hx = raw_hex.translate(str.maketrans("0123456789ABCDEF", "FEDCBA9876543210")) if inv else raw_hex
    bits = hex_to_bits(hx)
    rc, res = mc_method(bank, pid, bits, len(bits))
    if rc == -1:
        return None
    return {"protocol_id": str(pid), "payload": f"{bank.prop(pid, 'preamble', '')}{res}",
            "meta": {"protocol_id": pid, "rssi": None, "freq_afc": None}}


def demod_mc_fixed(bank: OracleBank, raw_hex: str, clock, mcbitnum, mtype="MC", version=None):
    out = []
    for pid in bank.ids_with("clockrange"):
        r = demod_mc_fixed_one(bank, pid, raw_hex, clock, mcbitnum, mtype, version)
        if r is not None:
            out.append(r)
    return out


def demod(bank: OracleBank, msg: Dict[str, Any], kind: str) -> List[dict]:
    """sd_protocols.py:60-74 dispatch (MU/MS only; MC has its own entry points)."""
    if kind == "MU":
        return demod_mu(bank, msg)
    if kind == "MS":
        return demod_ms(bank, msg)
    return []
