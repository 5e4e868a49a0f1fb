"""CPU restatement of the MN (FSK) path -- TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and the cpu_baseline legs of the benchmarks may import this
module; the product path (pysignalduino_amd -> csrc/sdx_mn.hip) never does.

Restated reference behaviour (RFD-FHEM/PySignalduino):
  signalduino/parser/mn.py:17         MN_PATTERN  ^MN;D=(Y?)([0-9A-F]+);(?:R=([0-9]+);)?(?:A=(-?[0-9]{1,3});)?$
  signalduino/parser/mn.py:31-191     MNParser.parse: per 'modulation' protocol (bank order) the
                                      rfmode filter, length_in_range(len(hex)), regexMatch re.search,
                                      the method call and the payload rule (a method's [] becomes
                                      the string "[]"), preamble + payload, metadata
  signalduino/parser/base.py:216-221  calc_rssi
  sd_protocols/sd_protocols.py:113-154 SDProtocols.demodulate_mn
  sd_protocols/helpers.py:190-716     lfsr_digest16, ConvBresser_lightning/5in1/6in1/7in1,
                                      _calc_crc16, ConvPCA301, ConvKoppFreeControl, ConvLaCrosse
The methods are restated on byte values (the input alphabet is the hex digits; the parser's
regex guarantees [0-9A-F], the direct method API also takes lower case).  Pinned against the
reference by tests/golden/mn_golden.json.gz (tests/golden/make_mn_golden.py) in tests/test_mn.py.
"""
from __future__ import annotations

import re
from typing import Any, Dict, List, Optional, Tuple

from .sd_oracle import OracleBank, length_in_range

_HEXV = {c: int(c, 16) for c in "0123456789abcdefABCDEF"}


class NotHex(Exception):
    """The data holds a character outside [0-9A-Fa-f] (outside the device contract)."""


def _nib(s: str) -> List[int]:
    try:
        return [_HEXV[c] for c in s]
    except KeyError as e:
        raise NotHex(s) from e


def _byte(v: List[int], k: int) -> int:
    return (v[2 * k] << 4) | v[2 * k + 1]


def _xor_a(s: str) -> str:
    """helpers.py:243-249 / 486-492: every hex digit XOR 0xA, upper-case digits."""
    return "".join("0123456789ABCDEF"[x ^ 0xA] for x in _nib(s))


def lfsr16(nbytes: int, gen: int, key: int, s: str) -> int:
    """helpers.py:190-221 (the data has >= 2*nbytes characters at every call site)."""
    if len(s) < 2 * nbytes:
        return 0
    v = _nib(s)
    acc = 0
    for k in range(nbytes):
        b = _byte(v, k)
        for i in range(7, -1, -1):
            if (b >> i) & 1:
                acc ^= key
            key = (key >> 1) ^ gen if key & 1 else key >> 1
    return acc


def crc16(s: str, poly: int) -> int:
    """helpers.py:281-309 with refin=refout=False, init=0, xorout=0 (both call sites)."""
    v = _nib(s)
    crc = 0
    for k in range(len(s) // 2):
        crc ^= _byte(v, k) << 8
        for _ in range(8):
            crc = ((crc << 1) ^ poly) if crc & 0x8000 else (crc << 1)
            crc &= 0xFFFF
    return crc


def conv_bresser_lightning(d: str) -> Optional[str]:
    """helpers.py:223-280 -> payload or None (the method returns [])."""
    if not d or len(d) < 20:
        return None
    x = _xor_a(d)
    chk = lfsr16(8, 0x8810, 0xABF9, x[4:20]) ^ int(x[0:4], 16)
    return x[:20] if chk == 0x899E else None


def conv_bresser_5in1(d: str) -> Optional[str]:
    """helpers.py:382-425."""
    if not d or len(d) < 52:
        return None
    v = _nib(d[:52])
    bits, ref = 0, 0
    for i in range(13):
        a, inv = _byte(v, i), _byte(v, i + 13)
        if a ^ inv != 0xFF:
            return None
        if i == 0:
            ref = inv
        else:
            bits += bin(inv).count("1")
    return d[28:52] if bits == ref else None


def conv_bresser_6in1(d: str) -> Optional[str]:
    """helpers.py:427-471."""
    if not d or len(d) < 36:
        return None
    if "%04X" % crc16(d[4:34], 0x1021) != d[0:4].upper():
        return None
    v = _nib(d[:36])
    return d if sum(_byte(v, i) for i in range(2, 18)) & 0xFF == 0xFF else None


def conv_bresser_7in1(d: str) -> Optional[str]:
    """helpers.py:473-523."""
    if not d or len(d) < 46:
        return None
    if d[42:44] == "00":
        return None
    x = _xor_a(d)
    chk = lfsr16(21, 0x8810, 0xBA95, x[4:46]) ^ int(x[0:4], 16)
    return x if chk == 0x6DF1 else None


def conv_pca301(d: str) -> Optional[str]:
    """helpers.py:525-579."""
    if not d or len(d) < 24:
        return None
    chk = d[20:24].upper()
    if "%04X" % crc16(d[0:20], 0x8005) != chk:
        return None
    v = _nib(d[:20])
    b = [_byte(v, i) for i in range(10)]
    return "OK 24 %d %d %d %d %d %d %d %d %d %d %s" % (b[0], b[1], b[2], b[3], b[4], b[5] & 0x0F, b[6], b[7], b[8],
                                                      b[9], chk)


def conv_kopp_fc(d: str) -> Optional[str]:
    """helpers.py:581-628."""
    if not d or len(d) < 4:
        return None
    v = _nib(d)
    n = _byte(v, 0) + 1
    if len(d) < 2 * n + 2:
        return None
    acc = 0xAA
    for i in range(n):
        acc ^= _byte(v, i)
    return "kr" + d[0:2 * n] if acc == _byte(v, n) else None


def conv_lacrosse(d: str) -> Optional[str]:
    """helpers.py:630-716 (CRC-8 poly 0x31, MSB first, init 0; fp64 temperature arithmetic)."""
    if not d or len(d) < 10:
        return None
    v = _nib(d[:10])
    crc = 0
    for i in range(4):
        crc ^= _byte(v, i)
        for _ in range(8):
            crc = ((crc << 1) ^ 0x31) & 0xFF if crc & 0x80 else (crc << 1) & 0xFF
    if crc != _byte(v, 4):
        return None
    b0, b1, b2, b3 = (_byte(v, i) for i in range(4))
    addr = ((b0 & 0x0F) << 2) | ((b1 & 0xC0) >> 6)
    t = ((b1 & 0x0F) * 100 + ((b2 & 0xF0) >> 4) * 10 + (b2 & 0x0F)) / 10 - 40
    if t >= 60 or t <= -40:
        return None
    sensor = 2 if (b3 & 0x7F) == 125 else 1
    scaled = int(t * 10 + 1000) & 0xFFFF
    return "OK 9 %d %d %d %d %d" % (addr, sensor | ((b1 & 0x20) << 2), (scaled >> 8) & 0xFF, scaled & 0xFF, b3)


METHODS = {
    "ConvBresser_lightning": (conv_bresser_lightning, {}),
    "ConvBresser_5in1": (conv_bresser_5in1, {}),
    "ConvBresser_6in1": (conv_bresser_6in1, {}),
    "ConvBresser_7in1": (conv_bresser_7in1, {}),
    "ConvPCA301": (conv_pca301, {"is_raw": False}),
    "ConvKoppFreeControl": (conv_kopp_fc, {"is_raw": False}),
    "ConvLaCrosse": (conv_lacrosse, {"is_raw": False}),
}


def call_method(name: str, msg_data: Dict[str, Any]) -> List[dict]:
    """SDProtocols.<name>(msg_data, 'MN') -> the reference's list ([] or one dict)."""
    fn, meta = METHODS[name]
    p = fn(msg_data.get("data"))
    if p is None:
        return []
    return [{"protocol_id": msg_data.get("protocol_id"), "payload": p, "meta": dict(meta)}]


def demodulate_mn(bank: OracleBank, msg_data: Dict[str, Any]) -> List[dict]:
    """sd_protocols.py:113-154."""
    if "protocol_id" not in msg_data:
        return []
    pid = msg_data["protocol_id"]
    if pid not in bank.p:
        return []
    m = bank.p[pid].get("method")
    if not m:
        return []
    name = m.split(".")[-1]
    if name not in METHODS:
        return []
    return call_method(name, msg_data)


MN_PATTERN = re.compile(rb"^MN;D=(Y?)([0-9A-F]+);(?:R=([0-9]+);)?(?:A=(-?[0-9]{1,3});)?$")


def parse_frame(payload: bytes) -> Optional[Tuple[bytes, Optional[bytes], Optional[bytes]]]:
    """parser/mn.py:33-51: (hex, R, A) or None (ensure_message_type always passes after routing)."""
    m = MN_PATTERN.match(payload)
    if not m:
        return None
    return m.group(2), m.group(3), m.group(4)


def rssi_of(r: Optional[bytes]) -> Optional[float]:
    """parser/mn.py:53-58 + base.py:216-221."""
    if not r:
        return None
    v = int(r)
    return ((v - 256) / 2) - 74 if v >= 128 else (v / 2) - 74


def afc_of(a: Optional[bytes]) -> Optional[float]:
    """parser/mn.py:60-68."""
    if not a:
        return None
    return round((26000000 / 16384 * int(a) / 1000), 0)


def mn_parse(bank: OracleBank, raw: str, rssi, freq_afc, rfmode: Optional[str]) -> List[Tuple[str, str, dict]]:
    """parser/mn.py:79-191 for one matched frame -> [(protocol_id, payload, metadata)]."""
    out = []
    for pid in bank.ids_with("modulation"):
        prf = bank.prop(pid, "rfmode", None)
        if not prf:
            continue
        if rfmode and prf != rfmode:
            continue
        if not length_in_range(bank, pid, len(raw))[0]:
            continue
        rx = bank.prop(pid, "regexMatch", None)
        modulation = bank.prop(pid, "modulation", None)
        if rx and not re.search(rx, raw):
            continue
        decoded = raw
        mfull = bank.p[pid].get("method")
        if mfull:
            name = mfull.split(".")[-1]
            if name not in METHODS:
                continue                       # 'Method ... not found' -> skipped
            res = call_method(name, {"raw_data": raw, "data": raw, "rssi": rssi, "freq_afc": freq_afc,
                                     "rfmode": rfmode, "protocol_id": pid})
            decoded = res[0].get("payload", raw) if res else str(res)
        pre = bank.prop(pid, "preamble", "")
        out.append((str(pid), f"{pre}{decoded}", {"rssi": rssi, "freq_afc": freq_afc, "modulation": modulation,
                                                   "rfmode": prf}))
    return out


def parse_line_payload(bank: OracleBank, payload: bytes, rfmode: Optional[str]) -> List[Tuple[str, str, dict]]:
    """MNParser.parse(RawFrame(payload)) for a routed MN payload."""
    f = parse_frame(payload)
    if f is None:
        return []
    h, r, a = f
    return mn_parse(bank, h.decode("ascii"), rssi_of(r), afc_of(a), rfmode)
