"""Seeded synthetic SIGNALduino corpora.

Everything here is vectorised numpy so that a 1M-message corpus is built in a
few seconds outside the timed region of ``bench.py``.  The same generators
feed the golden-vector script (``tests/golden/make_golden.py``), the parity
tests and the benchmark, so the benchmark measures exactly the distribution
the parity tests check.

Batch layout (the device SoA layout, see DESIGN.md "Data layout in HBM"):

``PulseBatch``  (MU / MS)
    data     uint8 [total]      pulse-id characters of every message, concatenated
    offsets  int64 [n+1]        message i owns data[offsets[i]:offsets[i+1]]
    npat     uint8 [n]          number of P# patterns (<= 10)
    pat_id   uint8 [n, 10]      pattern id characters ('0'..'9') in line order
    pat_val  float64 [n, 10]    pattern values (float(P#)) in line order
    cp_slot  int8 [n]           MS only: slot of the CP pattern, -1 when CP is
                                missing from the patterns
    rssi     int32 [n]          R= value (-1 = absent)
    ms_ok    uint8 [n]          MS only: CP/SP/R string gates passed

``McBatch``
    hexdata  uint8 [total], offsets int64 [n+1], clock int32 [n],
    mcbitnum int32 [n], mtype uint8 [n] (0 = 'MC', 1 = 'Mc'), v32 uint8 [n]
    (version string starts with 'V 3.2.').
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Dict, List, Optional

import numpy as np

MAXPAT = 10


@dataclass
class PulseBatch:
    kind: str
    data: np.ndarray
    offsets: np.ndarray
    npat: np.ndarray
    pat_id: np.ndarray
    pat_val: np.ndarray
    cp_slot: np.ndarray
    sp_slot: np.ndarray
    rssi: np.ndarray
    ms_ok: np.ndarray
    src_proto: np.ndarray = field(default=None)  # generating protocol index (-1 noise)

    @property
    def n(self) -> int:
        return int(self.npat.shape[0])

    def message(self, i: int) -> str:
        return bytes(self.data[self.offsets[i]:self.offsets[i + 1]]).decode("latin-1")

    def to_msg_dict(self, i: int) -> Dict[str, str]:
        """msg_data exactly as MUParser/MSParser would build it (parser/mu.py:82-94)."""
        d: Dict[str, str] = {self.kind: ""}
        for k in range(int(self.npat[i])):
            v = self.pat_val[i, k]
            d["P" + chr(self.pat_id[i, k])] = str(int(v)) if float(v).is_integer() else repr(float(v))
        d["D"] = self.message(i)
        if self.kind == "MS":
            d["CP"] = chr(self.pat_id[i, self.cp_slot[i]]) if self.cp_slot[i] >= 0 else "9"
            d["SP"] = chr(self.pat_id[i, self.sp_slot[i]]) if self.sp_slot[i] >= 0 else "9"
        else:
            d["CP"] = chr(self.pat_id[i, 0])
        if self.rssi[i] >= 0:
            d["R"] = str(int(self.rssi[i]))
        d["data"] = d["D"]
        return d

    def subset(self, idx) -> "PulseBatch":
        idx = np.asarray(idx, dtype=np.int64)
        lens = self.offsets[idx + 1] - self.offsets[idx]
        offs = np.zeros(len(idx) + 1, dtype=np.int64)
        np.cumsum(lens, out=offs[1:])
        data = np.concatenate([self.data[self.offsets[i]:self.offsets[i + 1]] for i in idx]) if len(idx) else np.zeros(0, np.uint8)
        return PulseBatch(self.kind, data, offs, self.npat[idx].copy(), self.pat_id[idx].copy(),
                          self.pat_val[idx].copy(), self.cp_slot[idx].copy(), self.sp_slot[idx].copy(),
                          self.rssi[idx].copy(), self.ms_ok[idx].copy(),
                          None if self.src_proto is None else self.src_proto[idx].copy())


@dataclass
class McBatch:
    hexdata: np.ndarray
    offsets: np.ndarray
    clock: np.ndarray
    mcbitnum: np.ndarray
    mtype: np.ndarray
    v32: np.ndarray
    src_proto: np.ndarray = field(default=None)

    @property
    def n(self) -> int:
        return int(self.clock.shape[0])

    def hex(self, i: int) -> str:
        return bytes(self.hexdata[self.offsets[i]:self.offsets[i + 1]]).decode("latin-1")

    def to_msg_dict(self, i: int) -> Dict[str, str]:
        """msg_data as MCParser builds it (parser/mc.py:59-62)."""
        d = {"MC" if self.mtype[i] == 0 else "Mc": "", "D": self.hex(i), "C": str(int(self.clock[i])),
             "L": str(int(self.mcbitnum[i]))}
        d["raw_hex"] = d["D"]
        d["clock"] = d["C"]
        d["mcbitnum"] = d["L"]
        d["messagetype"] = "MC" if self.mtype[i] == 0 else "Mc"
        return d

    def subset(self, idx) -> "McBatch":
        idx = np.asarray(idx, dtype=np.int64)
        lens = self.offsets[idx + 1] - self.offsets[idx]
        offs = np.zeros(len(idx) + 1, dtype=np.int64)
        np.cumsum(lens, out=offs[1:])
        data = np.concatenate([self.hexdata[self.offsets[i]:self.offsets[i + 1]] for i in idx]) if len(idx) else np.zeros(0, np.uint8)
        return McBatch(data, offs, self.clock[idx].copy(), self.mcbitnum[idx].copy(), self.mtype[idx].copy(),
                       self.v32[idx].copy(), None if self.src_proto is None else self.src_proto[idx].copy())


def _numeric(seq) -> Optional[List[float]]:
    if not isinstance(seq, list) or not seq:
        return None
    try:
        return [float(x) for x in seq]
    except (TypeError, ValueError):
        return None


def _templates(protocols: Dict[str, dict], key_start: str):
    """Per eligible protocol: distinct values, start/one/zero as value-slot lists."""
    out = []
    for idx, (pid, p) in enumerate(protocols.items()):
        if key_start == "sync" and "sync" not in p:
            continue
        if key_start == "start" and "clockabs" not in p:
            continue
        one, zero = _numeric(p.get("one")), _numeric(p.get("zero"))
        if one is None or zero is None or len(one) != len(zero):
            continue
        head = _numeric(p.get(key_start)) if key_start in p else []
        if head is None:
            continue
        vals: List[float] = []
        for v in head + one + zero:
            if v not in vals:
                vals.append(v)
        if len(vals) > 8:
            continue
        ca = float(p.get("clockabs", 0) or 0)
        lmin = int(p.get("length_min", 8) or 8)
        lmax = int(p.get("length_max", lmin + 8) or (lmin + 8))
        lmax = max(lmin, min(lmax, 200))
        out.append(dict(idx=idx, pid=pid, vals=vals, head=[vals.index(v) for v in head],
                        one=[vals.index(v) for v in one], zero=[vals.index(v) for v in zero],
                        clock=ca, lmin=lmin, lmax=lmax))
    return out


def _assemble(rng, n, tpls, npulse_fn, repeat: bool, clock_sweep, noise_frac: float, kind: str,
              fixed_len: Optional[int], skew: float = 0.0):
    """Shared vectorised MU/MS message assembly (padded [n, Tmax] then packed ragged).  skew > 0:
    templates drawn with Zipf weights 1 / rank^skew over a seeded ranking (a capture dominated by a
    few protocols) instead of uniformly."""
    ntpl = len(tpls)
    Tmax = fixed_len if fixed_len else 256
    if skew > 0:
        w = 1.0 / np.arange(1, ntpl + 1, dtype=np.float64) ** skew
        choice = rng.permutation(ntpl)[rng.choice(ntpl, size=n, p=w / w.sum())]
    else:
        choice = rng.integers(0, ntpl, size=n)
    is_noise = rng.random(n) < noise_frac
    npat = np.zeros(n, np.uint8)
    pat_id = np.zeros((n, MAXPAT), np.uint8)
    pat_val = np.zeros((n, MAXPAT), np.float64)
    cp_slot = np.full(n, -1, np.int8)
    sp_slot = np.full(n, -1, np.int8)
    rssi = rng.integers(0, 256, size=n).astype(np.int32)
    rssi[rng.random(n) < 0.1] = -1
    lengths = np.zeros(n, np.int64)
    msgs = np.zeros((n, Tmax), np.uint8)
    src = np.where(is_noise, -1, np.array([t["idx"] for t in tpls])[choice]).astype(np.int32)
    # id permutation per message: slot k gets id perm[k]; ids are emitted in ascending
    # id order like the firmware prints P0..P7, so the dict order differs from slot order.
    perms = np.argsort(rng.random((n, MAXPAT)), axis=1).astype(np.int64)
    for t_i, t in enumerate(tpls):
        sel = np.nonzero((choice == t_i) & ~is_noise)[0]
        if len(sel) == 0:
            continue
        m = len(sel)
        nv = len(t["vals"])
        base = t["clock"] if t["clock"] > 0 else 0.0
        clk = np.full(m, base) if base > 0 else rng.uniform(250, 500, size=m)
        clk = clk * clock_sweep(rng, m)
        jit = rng.uniform(0.95, 1.05, size=(m, nv))
        vals = np.clip(np.rint(np.array(t["vals"])[None, :] * clk[:, None] * jit), -99999, 99999)
        nb = rng.integers(t["lmin"], t["lmax"] + 1, size=m)
        bits = rng.integers(0, 2, size=(m, max(t["lmax"], 1))).astype(np.int64)
        head = np.array(t["head"], np.int64)
        L = len(t["one"])
        units = np.array([t["zero"], t["one"]], np.int64)  # [2, L]
        frame_len = len(head) + nb * L
        total = np.full(m, fixed_len, np.int64) if fixed_len else np.minimum(npulse_fn(rng, m, frame_len), Tmax)
        pos = np.arange(Tmax)[None, :]
        j = pos % frame_len[:, None] if repeat else np.minimum(pos, frame_len[:, None] - 1)
        in_head = j < len(head)
        hj = np.minimum(j, max(len(head) - 1, 0))
        bj = np.maximum(j - len(head), 0)
        bit_idx = np.minimum(bj // L, bits.shape[1] - 1)
        u = bj % L
        bitv = np.take_along_axis(bits, bit_idx, axis=1)
        slot = np.where(in_head, head[hj] if len(head) else 0, units[bitv, u])
        P = perms[sel, :nv]                       # slot -> id
        order = np.argsort(P, axis=1)             # q -> slot, ascending id
        npat[sel] = nv
        pat_id[sel, :nv] = (np.take_along_axis(P, order, axis=1) + ord("0")).astype(np.uint8)
        pat_val[sel, :nv] = np.take_along_axis(vals, order, axis=1)
        if kind == "MS":
            av = np.abs(np.array(t["vals"]))
            cps = int(np.argmin(np.abs(av - 1.0)))
            sync_slots = t["head"] if t["head"] else [0]
            sps = max(sync_slots, key=lambda s: abs(t["vals"][s]))
            cp_slot[sel] = np.argmax(order == cps, axis=1)
            sp_slot[sel] = np.argmax(order == sps, axis=1)
        msgs[sel] = (np.take_along_axis(P, slot, axis=1) + ord("0")).astype(np.uint8)
        lengths[sel] = total
    noise = np.nonzero(is_noise)[0]
    if len(noise):
        m = len(noise)
        nvs = rng.integers(2, 9, size=m)
        P = perms[noise]                          # first nv entries are the ids in use
        mag = rng.uniform(100, 20000, size=(m, MAXPAT))
        sgn = np.where(rng.random((m, MAXPAT)) < 0.5, -1.0, 1.0)
        valid = np.arange(MAXPAT)[None, :] < nvs[:, None]
        ids_sorted = np.sort(np.where(valid, P, 99), axis=1)
        npat[noise] = nvs
        pat_id[noise] = np.where(ids_sorted < 99, ids_sorted + ord("0"), 0).astype(np.uint8)
        pat_val[noise] = np.where(ids_sorted < 99, np.rint(mag * sgn), 0.0)
        pick = (rng.random((m, Tmax)) * nvs[:, None]).astype(np.int64)
        msgs[noise] = (np.take_along_axis(ids_sorted, pick, axis=1) + ord("0")).astype(np.uint8)
        lengths[noise] = fixed_len if fixed_len else rng.integers(16, 200, size=m)
        if kind == "MS":
            absv = np.where(valid, np.abs(pat_val[noise]), np.inf)
            cp_slot[noise] = np.argmin(absv, axis=1)
            sp_slot[noise] = np.argmax(np.where(valid, np.abs(pat_val[noise]), -1.0), axis=1)
    offsets = np.zeros(n + 1, np.int64)
    np.cumsum(lengths, out=offsets[1:])
    data = msgs[np.arange(Tmax)[None, :] < lengths[:, None]]
    ms_ok = np.ones(n, np.uint8)
    return PulseBatch(kind, np.ascontiguousarray(data), offsets, npat, pat_id, pat_val, cp_slot, sp_slot,
                      rssi, ms_ok, src)


def mu_corpus(protocols: Dict[str, dict], n: int, seed: int = 42, npulse: int = 256,
              noise_frac: float = 0.15, skew: float = 0.0) -> PulseBatch:
    """Config 2: MU messages of exactly ``npulse`` pulses, frames repeated."""
    rng = np.random.default_rng(seed)
    tpls = _templates(protocols, "start")
    return _assemble(rng, n, tpls, None, True, lambda r, m: np.ones(m), noise_frac, "MU", npulse, skew)


def ms_corpus(protocols: Dict[str, dict], n: int, seed: int = 43, noise_frac: float = 0.1,
              skew: float = 0.0) -> PulseBatch:
    """Config 3: one sync+bits frame per message, clock swept x U(0.6,1.4) over the ±30 % gate."""
    rng = np.random.default_rng(seed)
    tpls = _templates(protocols, "sync")

    def npulse_fn(r, m, frame_len):
        # one frame, sometimes followed by a partial repeat (firmware buffer tail)
        extra = np.where(r.random(m) < 0.3, r.integers(1, 9, size=m), 0)
        return np.minimum(frame_len + extra, 256)

    return _assemble(rng, n, tpls, npulse_fn, True, lambda r, m: r.uniform(0.6, 1.4, size=m),
                     noise_frac, "MS", None, skew)


def mc_protocols(protocols: Dict[str, dict]) -> List[int]:
    return [i for i, p in enumerate(protocols.values()) if "clockrange" in p]


def mc_corpus(protocols: Dict[str, dict], n: int, seed: int = 44) -> McBatch:
    """Config 4: random-hex Manchester frames for the 12 clockrange protocols."""
    rng = np.random.default_rng(seed)
    plist = list(protocols.values())
    mc = mc_protocols(protocols)
    choice = np.array(mc)[rng.integers(0, len(mc), size=n)]
    lmin = np.array([int(plist[i].get("length_min", 8)) for i in choice])
    lmax = np.array([int(plist[i].get("length_max", 64)) for i in choice])
    L = (lmin + (rng.random(n) * (lmax - lmin + 1)).astype(np.int64)).astype(np.int32)
    # a few out-of-range lengths to exercise the gates
    L = np.where(rng.random(n) < 0.05, np.maximum(L + rng.integers(-6, 7, size=n), 1), L).astype(np.int32)
    lo = np.array([plist[i]["clockrange"][0] for i in choice], np.float64)
    hi = np.array([plist[i]["clockrange"][1] for i in choice], np.float64)
    clock = np.rint(rng.uniform(0.9 * lo, 1.1 * hi)).astype(np.int32)
    hexlen = (L + 3) // 4
    offsets = np.zeros(n + 1, np.int64)
    np.cumsum(hexlen, out=offsets[1:])
    digits = np.frombuffer(b"0123456789ABCDEF", np.uint8)
    hexdata = digits[rng.integers(0, 16, size=int(offsets[-1]))]
    mtype = (rng.random(n) < 0.5).astype(np.uint8)
    v32 = (rng.random(n) < 0.1).astype(np.uint8)
    return McBatch(hexdata.copy(), offsets, clock, L, mtype, v32, choice.astype(np.int32))


# ---------------------------------------------------------------------------------------------
# Firmware lines: the wire format the front end (sdx_parse_lines) consumes.
# A line is bytes: STX + payload + ETX (+ "\n"), latin-1 as the transport decodes it
# (signalduino/transport.py:123).  Compressed lines use the firmware's Mred=1 encoding, i.e. the
# inverse of the decompression the reference runs (signalduino/parser/base.py:13-186).
STX, ETX = b"\x02", b"\x03"


def _pint(v: float) -> str:
    return str(int(v)) if float(v).is_integer() else repr(float(v))


def _line_fields(pb: PulseBatch, i: int):
    """(ids, vals, data, cp, sp) of message i with the pattern ids moved into 0..7 as the firmware
    numbers them (ids and data digits renamed consistently; unchanged when more than 8 patterns)."""
    n = int(pb.npat[i])
    ids = [chr(pb.pat_id[i, k]) for k in range(n)]
    vals = [float(pb.pat_val[i, k]) for k in range(n)]
    msg = pb.message(i)
    if pb.kind == "MS":
        cp = ids[pb.cp_slot[i]] if pb.cp_slot[i] >= 0 else "9"
        sp = ids[pb.sp_slot[i]] if pb.sp_slot[i] >= 0 else "9"
    else:
        cp, sp = (ids[0] if ids else "0"), None
    if n <= 8 and any(c > "7" for c in ids):
        free = [c for c in "01234567" if c not in ids]
        ren = {}
        for c in ids:
            ren[c] = c if c <= "7" else free.pop(0)
        ids = [ren[c] for c in ids]
        msg = msg.translate(str.maketrans(ren))
        cp = ren.get(cp, cp)
        sp = ren.get(sp, sp) if sp is not None else None
    return ids, vals, msg, cp, sp


def pulse_payload(pb: PulseBatch, i: int) -> bytes:
    """Uncompressed payload "MU;P0=..;D=..;CP=..;R=..;" (MS adds SP) in firmware field order."""
    ids, vals, msg, cp, sp = _line_fields(pb, i)
    parts = [pb.kind] + ["P%s=%s" % (c, _pint(v)) for c, v in zip(ids, vals)] + ["D=" + msg, "CP=" + cp]
    if pb.kind == "MS":
        parts.append("SP=" + sp)
    if pb.rssi[i] >= 0:
        parts.append("R=%d" % int(pb.rssi[i]))
    return (";".join(parts) + ";").encode("latin-1")


def compress_pulse_payload(pb: PulseBatch, i: int) -> Optional[bytes]:
    """Mred=1 form of pulse_payload (None when the message is not representable: pattern values
    that are not integers of magnitude <= 32767, ids > 7, or data digits > 7)."""
    ids, vals, msg, cp, sp = _line_fields(pb, i)
    if any(c > "7" for c in msg) or any(c > "7" for c in ids) or not msg:
        return None
    out = bytearray(("M" + pb.kind[1].lower() + ";").encode())
    for pid, v in zip(ids, vals):
        if not v.is_integer() or abs(v) > 32767:
            return None
        a = int(abs(v))
        lo, hi = a & 0xFF, a >> 8
        out += bytes([0x80 | int(pid) | (0x20 if v < 0 else 0) | (0x10 if lo >= 128 else 0),
                      0x80 | (lo & 0x7F), 0x80 | hi]) + b";"
    odd = len(msg) % 2
    out += b"d" if odd else b"D"
    digits = [int(c) for c in msg] + ([0] if odd else [])
    out += bytes((digits[j] << 4) | digits[j + 1] for j in range(0, len(digits), 2)) + b";"
    out += b"C" + cp.encode() + b";"
    if pb.kind == "MS":
        out += b"S" + sp.encode() + b";"
    if 0 <= pb.rssi[i] <= 255:
        out += b"R" + ("%X" % int(pb.rssi[i])).encode() + b";"
    return bytes(out)


def mc_payload(mb: McBatch, i: int, rssi: Optional[int] = None) -> bytes:
    c = int(mb.clock[i])
    s = "MC;LL=%d;LH=%d;SL=%d;SH=%d;D=%s;C=%d;L=%d;" % (-2 * c, 2 * c, -c, c, mb.hex(i), c, int(mb.mcbitnum[i]))
    if rssi is not None:
        s += "R=%d;" % rssi
    return s.encode("latin-1")


def frame(payload: bytes, newline: bool = True) -> bytes:
    return STX + payload + ETX + (b"\n" if newline else b"")


def line_corpus(protocols: Dict[str, dict], n: int, seed: int = 45, mix=(0.4, 0.4, 0.2),
                compress_frac: float = 0.3, mu_npulse: int = 256):
    """Config 5 (§8(f) 1): n framed firmware lines, MU/MS/MC in proportion ``mix``, a fraction
    of the MU/MS lines Mred=1-compressed.  Returns (lines: List[bytes], kinds: np.ndarray)."""
    rng = np.random.default_rng(seed)
    kinds = rng.choice(3, size=n, p=np.asarray(mix, np.float64) / np.sum(mix))
    cnt = [int((kinds == k).sum()) for k in range(3)]
    mu = mu_corpus(protocols, max(cnt[0], 1), seed=seed + 1, npulse=mu_npulse)
    ms = ms_corpus(protocols, max(cnt[1], 1), seed=seed + 2)
    mc = mc_corpus(protocols, max(cnt[2], 1), seed=seed + 3)
    comp = rng.random(n) < compress_frac
    rssi = rng.integers(0, 256, size=n)
    lines: List[bytes] = []
    pos = [0, 0, 0]
    for j in range(n):
        k = int(kinds[j])
        i = pos[k]
        pos[k] += 1
        if k == 2:
            lines.append(frame(mc_payload(mc, i, int(rssi[j]))))
            continue
        pb = mu if k == 0 else ms
        p = compress_pulse_payload(pb, i) if comp[j] else None
        lines.append(frame(p if p is not None else pulse_payload(pb, i)))
    return lines, kinds


_JUNK = b";=;=-+0123456789ABCDEFabcdefPDCSRLMFOpewmu \t\r\n\x02\x03\x80\x91\xa0\xb5\xc3\xdf\xff"


def mutate_line(rng: np.random.Generator, line: bytes) -> bytes:
    """One seeded corruption of a firmware line (the fuzz cases of the front-end parity tests)."""
    b = bytearray(line)
    op = int(rng.integers(0, 14))
    if not b:
        return bytes(_JUNK[int(rng.integers(0, len(_JUNK)))] for _ in range(int(rng.integers(1, 8))))
    j = int(rng.integers(0, len(b)))
    if op == 0:                       # drop a byte
        del b[j]
    elif op == 1:                     # insert a byte
        b.insert(j, _JUNK[int(rng.integers(0, len(_JUNK)))])
    elif op == 2:                     # overwrite a byte
        b[j] = _JUNK[int(rng.integers(0, len(_JUNK)))]
    elif op == 3:                     # swap the case of the type character
        k = b.find(b"M")
        if 0 <= k + 1 < len(b):
            b[k + 1] ^= 0x20
    elif op == 4:                     # lose the framing
        b = b.replace(STX, b"", 1) if rng.random() < 0.5 else b.replace(ETX, b"", 1)
    elif op == 5:                     # whitespace around the frame
        b = bytearray(b" \t"[: int(rng.integers(0, 3))] + bytes(b) + b"\r\n \x0b"[: int(rng.integers(0, 4))])
    parts = bytes(b).split(b";")
    if op >= 6 and len(parts) > 2:
        q = int(rng.integers(1, len(parts) - 1))
        if op == 6:                   # duplicate a field (last value wins)
            parts.insert(q + int(rng.integers(0, 2)), parts[q])
        elif op == 7:                 # drop a field
            del parts[q]
        elif op == 8:                 # empty the value of a field
            parts[q] = parts[q].split(b"=")[0] + b"="
        elif op == 9:                 # swap two fields
            r = int(rng.integers(1, len(parts) - 1))
            parts[q], parts[r] = parts[r], parts[q]
        elif op == 10:                # an extra field the grammars may or may not accept
            extra = [b"P05=-400", b"P10=300", b"P3=1e3", b"P3=4.5", b"F=12", b"V=1", b"O", b"e", b"p",
                     b"w=1", b"M=AB", b"MC", b"X=1", b"SP=x", b"CP=", b"R=-5", b"D=", b"P8=200"]
            parts.insert(q, extra[int(rng.integers(0, len(extra)))])
        elif op == 11:                # a '=' removed
            parts[q] = parts[q].replace(b"=", b"", 1)
        elif op == 12:                # an empty part
            parts.insert(q, b"")
        else:                         # lowercase a key
            parts[q] = parts[q][:1].lower() + parts[q][1:]
        return b";".join(parts)
    return bytes(b)


# ---------------------------------------------------------------------------------------------
# MN (FSK) frames: hex payloads that pass each 'modulation' protocol's regex,
# length and checksum rules (the methods of sd_protocols/helpers.py:223-716), plus corrupted and
# random ones.  Checksums are built with the generator-side helpers below (the product never uses
# them: they construct inputs).
# ---------------------------------------------------------------------------------------------
_HEXD = "0123456789ABCDEF"


def _hx(bs) -> str:
    return "".join("%02X" % (int(b) & 0xFF) for b in bs)


def _lfsr16_bytes(bs, gen: int, key: int) -> int:
    acc = 0
    for b in bs:
        for i in range(7, -1, -1):
            if (int(b) >> i) & 1:
                acc ^= key
            key = (key >> 1) ^ gen if key & 1 else key >> 1
    return acc


def _crc16_bytes(bs, poly: int) -> int:
    crc = 0
    for b in bs:
        crc ^= int(b) << 8
        for _ in range(8):
            crc = ((crc << 1) ^ poly) & 0xFFFF if crc & 0x8000 else (crc << 1) & 0xFFFF
    return crc


def _crc8_bytes(bs) -> int:
    crc = 0
    for b in bs:
        crc ^= int(b)
        for _ in range(8):
            crc = ((crc << 1) ^ 0x31) & 0xFF if crc & 0x80 else (crc << 1) & 0xFF
    return crc


def _xor_a(s: str) -> str:
    return "".join(_HEXD[int(c, 16) ^ 0xA] for c in s)


def _mn_valid(rng: np.random.Generator, kind: str) -> str:
    """One frame that the named MN protocol family accepts (checksums valid)."""
    rb = lambda k: rng.integers(0, 256, size=k)  # noqa: E731
    tail = lambda: _hx(rb(int(rng.integers(0, 4))))  # noqa: E731
    if kind == "lightning":            # helpers.py:223-280
        body = rb(8)
        x0 = _lfsr16_bytes(body, 0x8810, 0xABF9) ^ 0x899E
        return _xor_a("%04X" % x0 + _hx(body)) + tail()
    if kind == "5in1":                 # helpers.py:382-425
        a = rb(13)
        inv = [(~int(v)) & 0xFF for v in a]
        inv[0] = sum(bin(v).count("1") for v in inv[1:])
        a[0] = (~inv[0]) & 0xFF
        return _hx(a) + _hx(inv) + tail()
    if kind == "6in1":                 # helpers.py:427-471
        mid = rb(15)
        last = (0xFF - int(mid.sum())) & 0xFF
        crc = _crc16_bytes(mid, 0x1021)
        return "%04X" % crc + _hx(mid) + "%02X" % last + tail()
    if kind == "7in1":                 # helpers.py:473-523
        body = rb(21)
        body[19] = body[19] if body[19] != 0xAA else 0xAB      # d[42:44] != '00'
        x0 = _lfsr16_bytes(body, 0x8810, 0xBA95) ^ 0x6DF1
        return _xor_a("%04X" % x0 + _hx(body)) + _hx(rb(int(rng.integers(0, 6))))
    if kind == "pca301":               # helpers.py:525-579
        body = rb(10)
        return _hx(body) + "%04X" % _crc16_bytes(body, 0x8005) + _hx(rb(int(rng.integers(0, 21))))
    if kind == "kopp":                 # helpers.py:581-628 (regexMatch ^0)
        n = int(rng.integers(3, 16))
        body = rb(n)
        body[0] = n - 1
        acc = 0xAA
        for v in body:
            acc ^= int(v)
        return _hx(body) + "%02X" % acc + tail()
    if kind == "lacrosse":             # helpers.py:630-716 (regexMatch ^9)
        b = rb(4)
        b[0] = 0x90 | (int(b[0]) & 0x0F)
        if rng.random() < 0.8:         # a plausible temperature (the range check is tested too)
            raw = int(rng.integers(1, 999))
            b[1] = (int(b[1]) & 0xF0) | (raw // 100)
            b[2] = ((raw // 10) % 10) << 4 | (raw % 10)
        return _hx(b) + "%02X" % _crc8_bytes(b) + _hx(rb(int(rng.integers(0, 8))))
    prefix, lo, hi = {"wh51": ("51", 28, 38), "wh57": ("57", 18, 38), "wh31": ("30", 22, 38),
                      "wh31b": ("52", 22, 38), "wh40": ("40", 22, 38), "rojaflex": ("08", 18, 18),
                      "avantek": ("", 16, 16), "ibs": ("D391", 36, 44), "wmbus": ("", 56, 300)}[kind]
    n = int(rng.integers(lo, hi + 1))
    return prefix + "".join(_HEXD[int(v)] for v in rng.integers(0, 16, size=n - len(prefix)))


MN_KINDS = ("lightning", "5in1", "6in1", "7in1", "pca301", "kopp", "lacrosse", "wh51", "wh57", "wh31", "wh31b",
            "wh40", "rojaflex", "avantek", "ibs", "wmbus")


def mn_frames(n: int, seed: int = 46, noise_frac: float = 0.25, corrupt_frac: float = 0.15):
    """n MN frames: (hex str, y_prefix bool, R int or None, A int or None).  Valid frames of every
    protocol family, some with one nibble flipped (checksum failures), and random hex noise."""
    rng = np.random.default_rng(seed)
    out = []
    for _ in range(n):
        u = rng.random()
        if u < noise_frac:
            k = int(rng.integers(1, 120))
            h = "".join(_HEXD[int(v)] for v in rng.integers(0, 16, size=k))
        else:
            h = _mn_valid(rng, MN_KINDS[int(rng.integers(0, len(MN_KINDS)))])
            if rng.random() < corrupt_frac / (1 - noise_frac):
                j = int(rng.integers(0, len(h)))
                h = h[:j] + _HEXD[int(h[j], 16) ^ int(rng.integers(1, 16))] + h[j + 1:]
        y = bool(rng.random() < 0.1)
        r = int(rng.integers(0, 256)) if rng.random() < 0.8 else None
        a = int(rng.integers(-999, 1000)) if rng.random() < 0.6 else None
        out.append((h, y, r, a))
    return out


def mn_payload(h: str, y: bool = False, r: Optional[int] = None, a: Optional[int] = None) -> bytes:
    s = "MN;D=%s%s;" % ("Y" if y else "", h)
    if r is not None:
        s += "R=%d;" % r
    if a is not None:
        s += "A=%d;" % a
    return s.encode("ascii")


# ---------------------------------------------------------------------------------------------
# Planted accept paths: bit vectors that each postDemodulation function accepts
# (sd_protocols/postdemodulation.py:27-730), MU/MS messages of the bank's postDemo users carrying
# them, and MC frames that the TFA / Grothe / Funkbus / ... methods accept
# (manchester.py:207-795).  Generator-side helpers only: they construct inputs whose checksums,
# parities and lengths are valid, so the parity tests reach the accept branches.
# ---------------------------------------------------------------------------------------------
def _byte_bits(v: int, n: int = 8) -> List[int]:
    return [(v >> (n - 1 - i)) & 1 for i in range(n)]


def _par9(v: int) -> List[int]:
    b = _byte_bits(v)
    return b + [sum(b) & 1]            # even parity over the 9-bit group


def postdemo_bits(rng: np.random.Generator, method: str, lead: Optional[int] = None) -> List[int]:
    """One bit list that ``method`` accepts.  ``lead``: leading zeros before the data start (the
    functions that look for the first '1' or for a preamble), drawn when None."""
    ri = lambda lo, hi: int(rng.integers(lo, hi + 1))  # noqa: E731
    rb = lambda k: [int(x) for x in rng.integers(0, 2, size=k)]  # noqa: E731
    z = ri(0, 6) if lead is None else lead
    if method == "postDemo_EM":                      # :27-88 preamble 0000000001 + 9 x (8 + 1) + xor
        out = [0] * (z + 9) + [1]
        crc = 0
        for _ in range(9):
            v = ri(0, 255)
            crc ^= v
            out += _byte_bits(v) + [1]
        return out + _byte_bits(crc)
    if method == "postDemo_Revolt":                  # :90-137 11 bytes + their sum
        data = [ri(0, 255) for _ in range(11)]
        out = []
        for v in data:
            out += _byte_bits(v)
        return out + _byte_bits(sum(data) & 0xFF) + rb(ri(0, 20))
    if method in ("postDemo_FS20", "postDemo_FHT80", "postDemo_FHT80TF"):   # :139-423
        if method == "postDemo_FS20":
            nd, base = (4 if rng.random() < 0.5 else 5), 6
        elif method == "postDemo_FHT80":
            nd, base = 5, 12
        else:
            nd, base = 4, 12
        data = [ri(0, 255) for _ in range(nd)]
        if method == "postDemo_FHT80TF":
            data[3] &= ~0x20 & 0xFF                  # bit 26 of the 40 data bits must be 0
        out = [0] * z + [1]
        for v in data:
            out += _par9(v)
        out += _par9((base + sum(data)) & 0xFF)
        if method != "postDemo_FHT80TF" and rng.random() < 0.3:
            out.append(ri(0, 1))                     # 46 / 55: the last bit is popped
        return out
    if method == "postDemo_WS2000":                  # :425-578 5-bit groups '1' + nibble (LSB first)
        typ = ri(0, 7)
        k = [35, 50, 35, 50, 70, 40, 40, 85][typ] // 5
        z = min(z, 9)
        if typ == 1 and rng.random() < 0.3:          # the 45/46-bit Thermo/Hygro form: XOR of all 9
            nib = [typ] + [ri(0, 15) for _ in range(7)]
            x = 0
            for v in nib:
                x ^= v
            nib.append(x)
        else:
            nib = [typ] + [ri(0, 15) for _ in range(k - 3)]
            x = 0
            for v in nib:
                x ^= v
            nib.append(x)                            # XOR over the first k-1 nibbles = 0
            nib.append((5 + sum(nib)) & 0x0F)        # the sum nibble
        out = [0] * z
        for v in nib:
            out += [1] + [(v >> i) & 1 for i in range(4)]
        if rng.random() < 0.3:
            out.append(ri(0, 1))
        return out
    if method == "postDemo_WS7035":                  # :580-640 ident, parity 15..27, nibble sum
        b = [1, 0, 1, 0, 0, 0, 0, 0] + rb(32)
        if sum(b[15:28]) & 1:
            b[20] ^= 1
        s = sum(int("".join(map(str, b[i:i + 4])), 2) for i in range(0, 40, 4))
        return b + _byte_bits(s % 16, 4)
    if method == "postDemo_WS7053":                  # :642-706 ident anywhere, parity 15..27
        pre = [0] * min(z, 2)
        b = [1, 0, 1, 0, 0, 0, 0, 0] + rb(ri(24, 26))
        full = pre + b
        msg = full[len(pre):] + ([0] if pre else [])
        if sum(msg[15:28]) & 1:
            b[20] ^= 1
        return pre + b
    if method == "postDemo_lengtnPrefix":            # :708-730
        return rb(ri(0, 60))
    raise KeyError(method)


POSTDEMO_USERS = {"80": "postDemo_EM", "45": "postDemo_Revolt", "74": "postDemo_FS20", "74.1": "postDemo_FS20",
                  "73": "postDemo_FHT80", "70": "postDemo_FHT80TF", "60": "postDemo_WS2000",
                  "66": "postDemo_WS7035", "67": "postDemo_WS7053", "39": "postDemo_lengtnPrefix"}


def _lead_for(pid: str, method: str, rng) -> int:
    """Leading zeros that put a planted frame inside the protocol's length_min..length_max."""
    want = {"80": (5, 15), "74": (4, 12), "74.1": (4, 12), "73": (4, 12), "70": (4, 11), "60": (3, 9)}
    lo, hi = want.get(pid, (0, 0))
    return int(rng.integers(lo, hi + 1))


def _planted_bits(rng, pid: str, P: Dict[str, dict]) -> List[int]:
    method = POSTDEMO_USERS[pid]
    p = P[pid]
    lmin, lmax = int(p.get("length_min", 0)), int(p.get("length_max", 999))
    for _ in range(200):
        b = postdemo_bits(rng, method, _lead_for(pid, method, rng))
        if method == "postDemo_WS2000" and len(b) > lmax:
            continue
        if method == "postDemo_lengtnPrefix":
            b = [int(x) for x in rng.integers(0, 2, size=int(rng.integers(lmin, lmax + 1)))]
        if method == "postDemo_Revolt":
            b = b[:lmax]
        if lmin <= len(b) <= lmax:
            return b
    return b


def planted_pulse_messages(P: Dict[str, dict], kind: str, n: int, seed: int = 50,
                           corrupt_frac: float = 0.25) -> List[Dict[str, str]]:
    """n MU or MS messages of the postDemo users (ids 80, 45, 74, 74.1, 73,
    70, 60, 66, 67, 39) whose frames carry ``postdemo_bits`` payloads, some with one bit flipped.
    MU: separator pulse + frame repeated (2-3 times, <= 256 pulses); MS: sync + one frame."""
    rng = np.random.default_rng(seed)
    pids = [pid for pid in POSTDEMO_USERS if ("sync" in P[pid]) == (kind == "MS") and pid in P]
    out = []
    for _ in range(n):
        pid = pids[int(rng.integers(0, len(pids)))]
        p = P[pid]
        bits = _planted_bits(rng, pid, P)
        if rng.random() < corrupt_frac and bits:
            j = int(rng.integers(0, len(bits)))
            bits[j] ^= 1
        head = [float(x) for x in (p.get("sync") if kind == "MS" else p.get("start") or [])]
        one, zero = [float(x) for x in p["one"]], [float(x) for x in p["zero"]]
        vals: List[float] = []
        for v in head + one + zero:
            if v not in vals:
                vals.append(v)
        sep = None
        if kind == "MU" and not head:
            sep = float(p["pause"][0]) if p.get("pause") else -100.0
            if sep not in vals:
                vals.append(sep)
        frame = [vals.index(v) for v in head]
        for b in bits:
            frame += [vals.index(v) for v in (one if b else zero)]
        if kind == "MU":
            reps = int(rng.integers(2, 4))
            unit = ([vals.index(sep)] if sep is not None else []) + frame
            seq = (unit * reps)[:256]
        else:
            seq = frame + frame[: int(rng.integers(0, 6))]
        clock = float(p["clockabs"]) * float(rng.uniform(0.97, 1.03))
        ids = [int(x) for x in rng.permutation(10)[: len(vals)]]
        pv = [int(round(v * clock * float(rng.uniform(0.97, 1.03)))) for v in vals]
        d: Dict[str, str] = {kind: ""}
        for slot in sorted(range(len(vals)), key=lambda s: ids[s]):
            d["P%d" % ids[slot]] = str(pv[slot])
        d["D"] = "".join(str(ids[s]) for s in seq)
        if kind == "MS":
            cp = min(range(len(vals)), key=lambda s: abs(abs(vals[s]) - 1.0))
            sp = max(range(len(head)), key=lambda s: abs(head[s])) if head else 0
            d["CP"] = str(ids[cp])
            d["SP"] = str(ids[vals.index(head[sp])]) if head else str(ids[0])
        else:
            d["CP"] = str(ids[min(range(len(vals)), key=lambda s: abs(abs(vals[s]) - 1.0))])
        if rng.random() < 0.9:
            d["R"] = str(int(rng.integers(0, 256)))
        d["data"] = d["D"]
        out.append(d)
    return out


def _bits_to_hex(bits: List[int]) -> str:
    s = "".join(map(str, bits))
    s = "0" * (-len(s) % 4) + s
    return "".join(_HEXD[int(s[i:i + 4], 2)] for i in range(0, len(s), 4))


def _inv_hex(h: str) -> str:
    return h.translate(str.maketrans("0123456789ABCDEF", "FEDCBA9876543210"))


def mc_method_bits(rng: np.random.Generator, pid: str, P: Dict[str, dict]) -> List[int]:
    """A bit string the MC method of protocol ``pid`` accepts (manchester.py:207-795)."""
    ri = lambda lo, hi: int(rng.integers(lo, hi + 1))  # noqa: E731
    rb = lambda k: [int(x) for x in rng.integers(0, 2, size=k)]  # noqa: E731
    p = P[pid]
    meth = p["method"].split(".")[-1]
    lmin, lmax = int(p.get("length_min", 8)), int(p.get("length_max", 64))
    if meth == "mcBit2Funkbus":                      # :207-300 mc2dmc + 6 bytes parity/checksum
        data = [0x2C] + [ri(0, 255) for _ in range(4)]
        b5 = ri(0, 7) << 5
        xr = 0
        for v in data:
            xr ^= v
        xr ^= b5
        nib = ((xr & 0xF0) >> 4) ^ (xr & 0x0F)
        chk = 0
        if nib & 8:
            chk ^= 0xC
        if nib & 4:
            chk ^= 0x2
        if nib & 2:
            chk ^= 0x8
        if nib & 1:
            chk ^= 0x3
        par = sum(bin(v).count("1") for v in data) + bin(b5).count("1")
        b5 |= (par & 1) << 4
        s = []
        for v in data + [b5 | chk]:
            s += _byte_bits(v)
        d = s[3:] + rb(ri(1, 4))                     # s = '001' + d: d starts with '01100'
        bits = [1]                                   # b[k+1] == b[k] <=> d[k] == 1
        for x in d:
            bits.append(bits[-1] if x else 1 - bits[-1])
        return bits
    if meth == "mcBit2TFA":                          # :615-719 sync + repeated 52-bit windows
        while True:
            w = rb(lmin)
            if "1111111111101" not in "".join(map(str, w)) and "1101" not in "".join(map(str, w[-3:] + [1])):
                break
        reps = ri(2, 4)
        out = [1] * 10 + [0, 1] + w
        for _ in range(reps - 1):
            out += [1] * 11 + [0, 1] + w
        return out + rb(ri(0, 6))
    if meth == "mcBit2Grothe":                       # :721-754 exactly 32 bits
        return [1] + rb(31)
    if meth == "mcBit2SomfyRTS":                     # :756-795 56 or 57
        return [1] + rb(55 if rng.random() < 0.5 else 56)
    if meth == "mcBit2Sainlogic":                    # :302-354 sync 010100 at <= 10, 128 bits
        st = ri(0, 10)
        b = [1] + rb(st - 1) if st else []
        b = (b + [0, 1, 0, 1, 0, 0] + rb(128))[: 128 - (10 - st)]
        return b
    if meth == "mcBit2AS":                           # :356-416 '1100' at >= 16
        head = [1] + [0, 1] * 8
        body = [1, 1, 0, 0] + [1, 0] * ((ri(lmin, lmax) - 4) // 2)
        return head[:16] + body
    n = ri(lmin, lmax)                               # length-gated hex methods, mcraw
    return [1] + rb(n - 1)


def mc_planted_frames(P: Dict[str, dict], n: int, seed: int = 51, corrupt_frac: float = 0.2):
    """n MC frames (hex, clock, L, messagetype, version) that the fixed chain
    decodes for the 12 clockrange ids: hex from ``mc_method_bits`` with the polarity the chain
    will undo, L and clock inside the protocol's gates; some with one hex digit changed."""
    rng = np.random.default_rng(seed)
    mc_ids = [pid for pid, p in P.items() if "clockrange" in p]
    out = []
    for _ in range(n):
        pid = mc_ids[int(rng.integers(0, len(mc_ids)))]
        p = P[pid]
        bits = mc_method_bits(rng, pid, P)
        h = _bits_to_hex(bits)
        mtype = "Mc" if rng.random() < 0.5 else "MC"
        ver = "V 3.2.1" if rng.random() < 0.1 else None
        inv = (p.get("polarity", "") == "invert") ^ (mtype == "Mc" or (ver is not None and ver[:6] == "V 3.2."))
        if inv:
            h = _inv_hex(h)
        if rng.random() < corrupt_frac:
            j = int(rng.integers(0, len(h)))
            h = h[:j] + _HEXD[(int(h[j], 16) + int(rng.integers(1, 16))) % 16] + h[j + 1:]
        lo, hi = p["clockrange"]
        clock = int(rng.integers(int(lo) + 1, int(hi)))
        L = int(rng.integers(int(p.get("length_min", 8)), int(p.get("length_max", 64)) + 1))
        out.append((h, clock, L, mtype, ver))
    return out


# ---------------------------------------------------------------------------------------------
# inputs of the general path (include/sdx.h): multi-digit pattern ids, long messages and frames
# ---------------------------------------------------------------------------------------------
def _msg_ids(m: Dict[str, str]) -> List[str]:
    return [k[1:] for k in m if k.startswith("P") and k[1:].isdigit()]


def _rekey(m: Dict[str, str], ren: Dict[str, str], rewrite_data: bool, order=None) -> Dict[str, str]:
    """m with pattern ids renamed (P<old> -> P<new>) -- the data characters of each renamed id
    replaced by the new id string when rewrite_data -- and the P keys in `order` (dict order
    decides pattern_exists ties)."""
    pk = [k for k in m if k.startswith("P") and k[1:].isdigit()]
    if order is not None:
        pk = [pk[i] for i in order]
    out: Dict[str, str] = {}
    for k, v in m.items():
        if k.startswith("P") and k[1:].isdigit():
            continue
        if k == "D" or k == "data":
            continue
        out[k] = v
    for k in pk:
        out["P" + ren.get(k[1:], k[1:])] = m[k]
    d = m["D"]
    if rewrite_data:
        d = "".join(ren.get(c, c) for c in d)
    for key in ("CP", "SP"):
        if key in out and out[key] in ren:
            out[key] = ren[out[key]]
    out["D"] = d
    out["data"] = d
    return out


def general_pulse_messages(P: Dict[str, dict], kind: str, n: int, seed: int = 60) -> List[Dict[str, str]]:
    """n MU or MS msg_data dicts outside the fixed-layout kernels' contract: multi-digit pattern
    ids (renamed ids with the data rewritten to the new strings, extra P1x patterns near the
    message's values, zero-padded keys), more than 10 patterns, and messages of 4097..12000 pulses
    (planted and corpus messages repeated), alone and combined."""
    rng = np.random.default_rng(seed)
    base = planted_pulse_messages(P, kind, max(8, n // 2), seed=seed + 1, corrupt_frac=0.1)
    pb = (mu_corpus if kind == "MU" else ms_corpus)(P, max(8, n // 2), seed=seed + 2)
    base += [pb.to_msg_dict(i) for i in range(pb.n)]
    out: List[Dict[str, str]] = []
    for j in range(n):
        m = dict(base[int(rng.integers(0, len(base)))])
        ids = _msg_ids(m)
        mode = int(rng.integers(0, 6))
        if mode in (0, 5) and ids:  # rename 1..3 ids to multi-digit strings, data rewritten
            pick = [ids[int(x)] for x in rng.permutation(len(ids))[: int(rng.integers(1, min(3, len(ids)) + 1))]]
            ren = {}
            for o in pick:
                cand = [str(10 + int(o)), o + o, "1" + o, str(int(rng.integers(10, 100))), o + "0"]
                c = cand[int(rng.integers(0, len(cand)))]
                if c not in ids and c not in ren.values():
                    ren[o] = c
            m = _rekey(m, ren, rewrite_data=True)
        elif mode == 1 and ids:  # rename without rewriting the data (ids may then be absent / mixed)
            o = ids[int(rng.integers(0, len(ids)))]
            m = _rekey(m, {o: str(int(rng.integers(10, 40)))}, rewrite_data=False)
        elif mode == 2:  # extra multi-digit patterns close to existing values (> 10 patterns possible)
            vals = [float(m[k]) for k in m if k.startswith("P") and k[1:].isdigit()] or [400.0]
            for t in range(int(rng.integers(1, 7))):
                v = vals[int(rng.integers(0, len(vals)))] * float(rng.uniform(0.85, 1.15))
                m["P" + str(10 + t + int(rng.integers(0, 3)) * 10)] = str(int(round(v)))
            if rng.random() < 0.5:  # shuffled key order
                m = _rekey(m, {}, rewrite_data=False, order=list(rng.permutation(len(_msg_ids(m)))))
        elif mode == 3:  # zero-padded keys beside multi-digit ones
            m = _rekey(m, {i: "0" + i for i in ids[:1]}, rewrite_data=False)
            m["P12"] = str(int(rng.integers(-2000, 2000)))
        if mode in (4, 5) or rng.random() < 0.15:  # long: the data repeated past LONG_MAX pulses
            d = m["D"]
            reps = max(2, (4097 + int(rng.integers(0, 8000))) // max(1, len(d)) + 1)
            if kind == "MS":  # MS: one sync, then a long tail of the message's data chunks
                d = d + d[len(d) // 3:] * reps
            else:
                d = d * reps
            m["D"] = m["data"] = d
        out.append(m)
    return out


def general_mc_frames(P: Dict[str, dict], n: int, seed: int = 61):
    """MC frames of 129..800 hex characters (the fixed chain's frames of any length): planted
    frames repeated / extended with random hex, and random hex; L inside and outside the gates."""
    rng = np.random.default_rng(seed)
    base = mc_planted_frames(P, max(8, n), seed=seed + 1, corrupt_frac=0.1)
    out = []
    for j in range(n):
        h, clock, L, mt, ver = base[int(rng.integers(0, len(base)))]
        target = int(rng.integers(129, 800))
        if rng.random() < 0.5:
            h2 = (h * (target // max(1, len(h)) + 1))[:target]
        else:
            h2 = h + "".join(_HEXD[int(x)] for x in rng.integers(0, 16, target - len(h)))
        if rng.random() < 0.05:
            h2 = h2[:40] + "g" + h2[41:]  # not hex
        if rng.random() < 0.3:
            L = 4 * len(h2)
        out.append((h2, clock, L, mt, ver))
    return out


def general_edge_messages(kind: str) -> List[Dict[str, str]]:
    """Hand-written edge inputs of the general path (empty / one-character data, only multi-digit
    ids, empty / non-numeric / nan / inf / -0 / 1e308 values, leading-zero keys beside multi-digit
    ones, CP naming a multi-digit id, 16 patterns, ragged lengths around 4096)."""
    base = {"CP": "10", "SP": "11", "R": "42"} if kind == "MS" else {"R": "42"}
    return [
        dict(base, data="", P10="400"),
        dict(base, data="1", P10="400"),
        dict(base, data="1010101110", P10="400", P11="-4000", P1="-400"),
        dict(base, data="1011" * 30, P10="", P11="abc", P1="400", P0="-800"),
        dict(base, data="1011" * 30, P10="nan", P11="inf", P1="-0", P0="1e308"),
        dict(base, data="0010" * 40, P010="500", P10="-500", P0010="600", P0="-1000"),
        dict(base, data="10" * 2100, P10="500", P1="-500", P0="-1000"),
        dict(base, data="10" * 2048 + "1", P1="500", P0="-1000"),
        dict(base, data="1" * 4097, P1="500"),
        dict(base, data="1213" * 50, **{f"P{k}": str(100 * (k + 1)) for k in range(10, 26)}),
    ]
