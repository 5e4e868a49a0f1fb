"""CPU restatement of the wire-line front end -- TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this module; the
product path (pysignalduino_amd.frontend -> sdx_parse_lines) never does.

It restates, on the bytes of one firmware line, what the reference does before demodulation:
  signalduino/transport.py:123          latin-1 decode + strip
  signalduino/parser/__init__.py:37-49  parse_line: extract_payload, route by payload[:2].upper()
  signalduino/parser/base.py:188-206    extract_payload (^\\x02(M[sSuUcCNOo];.*;)\\x03$)
  signalduino/parser/base.py:13-186     decompress_payload
  signalduino/parser/mu.py:27-94        MU regex, _parse_to_dict, "D" check, R/F metadata
  signalduino/parser/ms.py:27-78        _parse_to_dict, "D" check, R/F metadata
  signalduino/parser/mc.py:27-155       MC header/key/value validation, required fields, hex D, int(R/F)
  sd_protocols/message_synced.py:21-66, message_unsynced.py:22-35   the P#/CP/SP/R string gates
and reports the same per-line record the device kernel writes (include/sdx.h sdx_lines_out), plus
the ``msg_data`` dict handed to the demodulator, so the goldens recorded from the reference
(tests/golden/lines_golden.json.gz, tests/golden/make_lines_golden.py) pin it directly.
Pinned: tests/test_lines.py::test_oracle_matches_reference_goldens.
"""
from __future__ import annotations

import re
from typing import Any, Dict, List, Optional, Tuple

NONE, MU, MS, MC, MN = 0, 1, 2, 3, 4
OK, NOFRAME, NOPARSER, INVALID, NODATA, UNSUPPORTED, RAISES, GENERAL = 0, 1, 2, 3, 4, 5, 6, 7
GEN_MAXPAT, GEN_IDMAX = 16, 15   # include/sdx.h SDX_GEN_MAXPAT, SDX_GEN_IDSTR - 1
SHORT_MAX, LONG_MAX, MC_HEX_MAX, MN_HEX_MAX = 256, 4096, 128, 4096

_WS = set(range(9, 14)) | set(range(0x1C, 0x21)) | {0x85, 0xA0}          # str.isspace() on latin-1
_ALPHA_HI = {0xAA, 0xB5, 0xBA} | set(range(0xC0, 0xD7)) | set(range(0xD8, 0xF7)) | set(range(0xF8, 0x100))
_HEX = set(b"0123456789abcdefABCDEF")
_DIG = set(b"0123456789")


def _alpha(c: int) -> bool:
    return (65 <= c <= 90) or (97 <= c <= 122) or c in _ALPHA_HI


def _strip(b: bytes) -> bytes:
    i, j = 0, len(b)
    while i < j and b[i] in _WS:
        i += 1
    while j > i and b[j - 1] in _WS:
        j -= 1
    return b[i:j]


def extract_payload(line: bytes) -> Optional[bytes]:
    """parser/base.py:188-206 -> None, or (compressed?) the payload bytes before decompression."""
    s = _strip(line)
    if len(s) < 6 or s[0] != 2 or s[-1] != 3 or s[1] != ord("M") or s[3] != ord(";") or s[-2] != ord(";"):
        return None
    if s[2] not in b"sSuUcCNOo" or b"\n" in s[4:-2]:
        return None
    return s[1:-1]


_FLOAT_WS = b" \t\n\v\f\r"  # what float() strips (not \x1c-\x1f: float("5\x1c") raises)
_DEC_RE = re.compile(rb"([+-]?)([0-9]*)(?:\.([0-9]*))?(?:[eE]([+-]?[0-9]+))?")


def _float_class(v: bytes):
    """float(v) as _patterns calls it (message_unsynced.py:31-35) and the device's modelled subset
    (sdx_lines.hip parse_pyfloat): ("skip", None) when float() raises ValueError; ("ok", float(v))
    for inf / nan / zero and decimals whose significant digits form M < 2^53 (<= 19 digits, trailing
    zeros moved into the exponent) with |exp10| <= 22 (Clinger's fast path: exact); ("unsup", None)
    for any other valid float."""
    try:
        x = float(v.decode("latin-1"))
    except ValueError:
        return "skip", None
    t = v.strip(_FLOAT_WS).replace(b"_", b"")
    if t.lstrip(b"+-").lower() in (b"inf", b"infinity", b"nan"):
        return "ok", x
    m = _DEC_RE.fullmatch(t)
    if m is None:
        return "unsup", None
    digs = (m.group(2) + (m.group(3) or b"")).lstrip(b"0")
    e10 = int(m.group(4) or b"0") - len(m.group(3) or b"")
    if not digs.strip(b"0"):
        return "ok", x
    stripped = digs.rstrip(b"0")
    e10 += len(digs) - len(stripped)
    if len(digs) > 19 and digs[19:].strip(b"0"):
        return "unsup", None
    if int(stripped) >= 2 ** 53 or not -22 <= e10 <= 22:
        return "unsup", None
    return "ok", x


class Unsupported(Exception):
    """Outside the device contract (the kernel reports SDX_LS_UNSUPPORTED)."""


def _hexpart(m1: bytes) -> bool:
    return 1 <= len(m1) <= 2 and all(c in _HEX for c in m1)


def _ends_data(part: bytes) -> bool:
    """base.py:76-99 -- the part starts a new field (ends the ';'-split D payload)."""
    m0, m1 = part[0], part[1:]
    if not _alpha(m0):
        return False
    return (m0 in b"Dd" or m0 > 127 or m0 == ord("M") or (m0 in b"CS" and len(m1) == 1) or m0 in b"om"
            or _hexpart(m1) or b"=" in part)


def decompress(p: bytes) -> bytes:
    """base.py:13-186 on bytes (Unsupported where str.upper() of a non-ASCII character is needed)."""
    if p[:3].upper() not in (b"MS;", b"MU;", b"MO;", b"MN;") or not any(c > 127 for c in p[3:]):
        return p
    parts = [q for q in p.split(b";") if q]
    out: List[bytes] = []
    k = 0
    while k < len(parts):
        q = parts[k]
        m0, m1 = q[0], q[1:]
        k += 1
        if m0 in b"Dd":
            raw = bytearray(m1)
            while k < len(parts) and not _ends_data(parts[k]):
                raw += b";" + parts[k]
                k += 1
            digits = "".join("%d%d" % ((c >> 4) & 15, c & 7) for c in raw)
            if m0 == ord("d"):
                digits = digits[:-1]
            if digits[:1] == "8":
                digits = digits[1:]
            out.append(b"D=" + digits.encode())
        elif m0 == ord("M"):
            if any(c > 127 for c in m1):
                raise Unsupported("upper() of a non-ASCII character")
            out.append(b"M" + m1.upper())
        elif m0 > 127:
            s = b"P%d=" % (m0 & 7)
            if len(m1) == 2:
                lo, hi = m1[0] & 127, m1[1] & 127
                if m0 & 16:
                    lo += 128
                s += (b"-" if m0 & 32 else b"") + str(hi * 256 + lo).encode()
            out.append(s)
        elif m0 in b"CS" and len(m1) == 1:
            out.append(bytes([m0]) + b"P=" + m1)
        elif m0 in b"om":
            out.append(q)
        elif _hexpart(m1):
            out.append(bytes([m0]) + b"=" + str(int(m1, 16)).encode())
        elif m0 < 128 and chr(m0).isalnum():
            out.append(bytes([m0]) + (b"=" if m1 else b"") + m1)
    return b";".join(out) + b";"


_MU_RE = re.compile(rb"^(?=.*D=\d+)(?:MU;(?:P[0-7]=-?[0-9]{1,5};){2,8}((?:D=\d{2,};)|(?:CP=\d;)|(?:R=\d+;)|"
                    rb"(?:O;)|(?:e;)|(?:p;)|(?:w=\d;))*)$")
_MC_KEY = re.compile(rb"[A-Z]{1,2}")
_MC_VAL = re.compile(rb"[-+]?[0-9a-fA-F]+")
_INT15 = re.compile(rb"[-+]?[0-9]{1,15}")
_DEC = re.compile(rb"[-+]?[0-9]+")
_MC_KEYS = {b"LL", b"LH", b"SL", b"SH", b"D", b"C", b"L", b"R", b"F", b"M", b"MC", b"Mc"}
_MN_RE = re.compile(rb"^MN;D=(Y?)([0-9A-F]+);(?:R=([0-9]+);)?(?:A=(-?[0-9]{1,3});)?$")  # parser/mn.py:17


def _kv(payload: bytes) -> List[Tuple[bytes, bytes]]:
    """_parse_to_dict of mu.py/ms.py as a list: first position, last value."""
    d: Dict[bytes, bytes] = {}
    for q in payload.split(b";"):
        if q:
            k, _, v = q.partition(b"=")
            d[k] = v
    return list(d.items())


def _rssi(v: int) -> float:
    return ((v - 256) / 2) - 74 if v >= 128 else (v / 2) - 74          # base.py calc_rssi


def _afc(v: int) -> float:
    return (v - 256) / 2 if v >= 128 else v / 2                        # base.py calc_afc


def _pyint(v: bytes) -> Optional[int]:
    try:
        return int(v.decode("latin-1"))                               # the parsers' int(msg_data["R"])
    except ValueError:
        return None


def _frame_meta(kv: Dict[bytes, bytes]) -> Tuple[Optional[float], Optional[float]]:
    """_extract_metadata (mu.py:96-108, ms.py:80-92, mc.py:141-155): frame.rssi / frame.freq_afc."""
    r, f = kv.get(b"R"), kv.get(b"F")
    ri = None if r is None else _pyint(r)
    fi = None if f is None else _pyint(f)
    return (None if ri is None else _rssi(ri)), (None if fi is None else _afc(fi))


def _meta_fits(r: Dict[str, Any]) -> bool:
    """The device hands R/F over as raw strings of <= 15 bytes (sdx_lines_out.meta_dev)."""
    return all(v is None or len(v) <= 15 for v in (r.get("R"), r.get("F")))


def parse_line(line: bytes) -> Dict[str, Any]:
    """One line -> {kind, status, payload, msg_data, dev fields, rssi, freq_afc} (device record)."""
    r: Dict[str, Any] = {"kind": NONE, "status": NOFRAME, "payload": None, "msg": None, "plen": -1}
    p = extract_payload(line)
    if p is None:
        return r
    try:
        q = decompress(p)
    except Unsupported:
        r["status"] = UNSUPPORTED
        return r
    if q is not p:
        r["plen"] = len(q)
    r["payload"] = q
    t = q[:2].upper()
    kind = {b"MU": MU, b"MS": MS, b"MC": MC, b"MN": MN}.get(t)
    if kind is None:
        r["status"] = NOPARSER
        return r
    r["kind"] = kind
    if kind == MN:
        return _mn(q, r)
    if any(c > 127 for c in q):
        r["status"] = UNSUPPORTED
        return r
    if kind == MC:
        return _mc(q, r)
    if kind == MU and not _MU_RE.match(q):
        r["status"] = INVALID
        return r
    items = _kv(q)
    kv = dict(items)
    if b"D" not in kv:
        r["status"] = NODATA
        return r
    data = kv[b"D"]
    # message_synced.py:21-47 gates; patterns converted where the reference converts them
    ok = False
    if kind == MS:
        ok = (bool(data) and data.isdigit() and bool(kv.get(b"CP")) and kv[b"CP"].isdigit()
              and bool(kv.get(b"SP")) and kv[b"SP"].isdigit() and (b"R" not in kv or kv[b"R"].isdigit()))
    ids: List[int] = []
    vals: List[float] = []
    gen = len(data) > LONG_MAX       # the fixed-layout kernels' limits: the general path (SDX_LS_GENERAL)
    pats: Dict[str, float] = {}      # _patterns with string ids (the general layout)
    if (kind == MS and ok) or (kind == MU and data):
        slot: Dict[int, float] = {}
        for k, v in items:                                    # message_unsynced.py:28-35
            if k[:1] == b"P" and len(k) > 1 and k[1:].isdigit():
                cls, fv = _float_class(v)
                if cls == "skip":
                    continue                                  # float() raises ValueError -> skipped
                if cls == "unsup":
                    r["status"] = UNSUPPORTED
                    return r
                pats[str(int(k[1:]))] = fv
                if int(k[1:]) >= 10:
                    gen = True
                    continue
                slot[int(k[1:])] = fv                         # Python's own float(): "-0" -> -0.0
        ids, vals = list(slot.keys()), list(slot.values())
    cp_slot = -1
    gcp = -1
    if kind == MS and ok:
        cp = int(kv[b"CP"])
        cp_slot = ids.index(cp) if cp in ids else -1
        gids = list(pats.keys())
        gcp = gids.index(str(cp)) if str(cp) in gids else -1
        ok = (gcp if gen else cp_slot) >= 0
    r.update(status=OK, data=data, ids=ids, vals=vals, cp_slot=cp_slot, ms_ok=int(ok),
             R=kv.get(b"R"), F=kv.get(b"F"))
    if gen:
        r.update(status=GENERAL, gids=list(pats.keys()), gvals=list(pats.values()), gcp=gcp)
    if not _meta_fits(r):
        r["status"] = UNSUPPORTED
        return r
    if gen and (len(pats) > GEN_MAXPAT or any(len(x) > GEN_IDMAX for x in pats)):
        r["status"] = UNSUPPORTED   # outside the general path's contract too: sdx_parse_lines reports
        r["gen_contract"] = True    # GENERAL, sdx_lines_general then UNSUPPORTED
        return r
    msg = [(k.decode("latin-1"), v.decode("latin-1")) for k, v in items]
    msg.append(("data", data.decode("latin-1")))
    r["msg"] = msg
    r["rssi"], r["freq_afc"] = _frame_meta(kv)
    return r


def _mc(q: bytes, r: Dict[str, Any]) -> Dict[str, Any]:
    """parser/mc.py:37-155."""
    d: Dict[bytes, bytes] = {}
    for part in q.split(b";"):
        if not part:
            continue
        if b"=" in part:
            k, _, v = part.partition(b"=")
            if not _MC_KEY.fullmatch(k) or not _MC_VAL.fullmatch(v) or k in d:
                r["status"] = INVALID
                return r
            d[k] = v
        else:
            if part in d or (d and part not in (b"MC", b"Mc")):
                r["status"] = INVALID
                return r
            d[part] = b""
    if any(k not in _MC_KEYS for k in d) or not all(k in d for k in (b"D", b"C", b"L")):
        r["status"] = INVALID
        return r
    if not all(c in _HEX for c in d[b"D"]) or not d[b"D"]:
        r["status"] = INVALID
        return r
    if any(k in d and _pyint(d[k]) is None for k in (b"R", b"F")):
        r["status"] = INVALID                                  # mc.py:141-155 raise -> ignored
        return r
    rssi, afc = _frame_meta(d)
    c, l_ = d[b"C"], d[b"L"]
    msg = [(k.decode("latin-1"), v.decode("latin-1")) for k, v in d.items()]
    msg += [("raw_hex", d[b"D"].decode()), ("clock", c.decode()), ("mcbitnum", l_.decode()),
            ("messagetype", d.get(b"M", b"MC").decode())]
    if not _DEC.fullmatch(c) or not _DEC.fullmatch(l_):
        r.update(status=RAISES, msg=msg, rssi=rssi, freq_afc=afc)  # int() raises inside demodulate_mc
        return r
    if not (-2**31 <= int(c) < 2**31) or not (-2**31 <= int(l_) < 2**31):
        r["status"] = UNSUPPORTED
        return r
    if not _meta_fits({"R": d.get(b"R"), "F": d.get(b"F")}):
        r["status"] = UNSUPPORTED
        return r
    r.update(status=OK, data=d[b"D"], clock=int(c), mcbitnum=int(l_), mcflags=0, R=d.get(b"R"), F=d.get(b"F"),
             msg=msg, rssi=rssi, freq_afc=afc)
    return r


def _mn(q: bytes, r: Dict[str, Any]) -> Dict[str, Any]:
    """parser/mn.py:33-51: ensure_message_type passes after routing; MN_PATTERN or ignored."""
    m = _MN_RE.match(q)
    if not m:
        r["status"] = INVALID
        return r
    h, rr, a = m.group(2), m.group(3), m.group(4)
    if len(h) > MN_HEX_MAX or (rr is not None and len(rr) > 15):
        r["status"] = UNSUPPORTED
        return r
    r.update(status=OK, data=h, R=rr, F=a, rssi=None, freq_afc=None)
    return r


def sel_class(r: Dict[str, Any]) -> int:
    """sdx_select_lines class of a parsed line (-1: not demodulated)."""
    if r["status"] != OK:
        return -1
    n = len(r["data"])
    if r["kind"] == MU:
        return 0 if n <= SHORT_MAX else 1
    if r["kind"] == MS:
        return -1 if not r["ms_ok"] else (2 if n <= SHORT_MAX else 3)
    if r["kind"] == MC:   # ABI 14: <= SDX_MC_SHORT_HEX (64) characters, longer
        return 4 if n <= 64 else 5
    return 6 if r["kind"] == MN else -1
