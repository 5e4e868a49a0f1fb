"""Host packing: reference ``msg_data`` dicts -> the device SoA batch, and back.

The reference parses each message's strings inside its demodulators
(message_unsynced.py:22-35, message_synced.py:21-66).  Those per-message string
conversions -- ``float(P#)``, the ``str.isdigit()`` gates, ``int(CP)``, the
dict-order of the P# keys -- are done here with the very same Python
operations while packing, so they raise exactly the same exceptions; the
numeric and pattern work then runs on the GPU.
"""
from __future__ import annotations

from typing import Any, Dict, List, Sequence, Tuple

import numpy as np

from .synth import MAXPAT, McBatch, PulseBatch


class ContractError(NotImplementedError):
    """An input the device path does not model (never silently approximated)."""


class GeneralPathMessage(ContractError):
    """Outside the fixed-layout kernels' contract (multi-digit pattern ids, more than LONG_MAX
    pulses): the message runs on the general path (sdx_demod_pulses_general) instead."""


GEN_MAXPAT = 16   # include/sdx.h SDX_GEN_MAXPAT
GEN_IDSTR = 16    # SDX_GEN_IDSTR: [length][<= 15 digits]


def _encode_data(data: str) -> bytes:
    """One byte per character; non-ASCII characters keep only their isdigit() property."""
    try:
        return data.encode("ascii")
    except UnicodeEncodeError:
        return bytes((ord(c) if ord(c) < 128 else (0xFE if c.isdigit() else 0xFF)) for c in data)


def _patterns(msg: Dict[str, Any]) -> Tuple[List[str], List[float]]:
    """message_unsynced.py:28-35 / message_synced.py:50-57 (same operations, same exceptions)."""
    pats: Dict[str, float] = {}
    for key, val in msg.items():
        if key.startswith("P") and key[1:].isdigit():
            try:
                pats[str(int(key[1:]))] = float(val)
            except ValueError:
                pass
    ids = list(pats.keys())
    for i in ids:
        if len(i) != 1:
            raise GeneralPathMessage(f"pattern id P{i}: the fixed-layout kernels take single-digit ids (P0..P9)")
    return ids, [pats[i] for i in ids]


def _patterns_general(msg: Dict[str, Any]) -> Tuple[List[str], List[float]]:
    """The same dict, any ids (sdx_general_batch): at most GEN_MAXPAT ids of <= 15 digits."""
    pats: Dict[str, float] = {}
    for key, val in msg.items():
        if key.startswith("P") and key[1:].isdigit():
            try:
                pats[str(int(key[1:]))] = float(val)
            except ValueError:
                pass
    ids = list(pats.keys())
    if len(ids) > GEN_MAXPAT or any(len(i) > GEN_IDSTR - 1 for i in ids):
        raise ContractError(f"more than {GEN_MAXPAT} patterns or a pattern id of more than {GEN_IDSTR - 1} "
                            "digits: outside the device contract")
    return ids, [pats[i] for i in ids]


class PulsePacker:
    """Accumulates MU or MS messages into one PulseBatch."""

    def __init__(self, kind: str):
        assert kind in ("MU", "MS")
        self.kind = kind
        self.datas: List[bytes] = []
        self.npat: List[int] = []
        self.ids: List[List[str]] = []
        self.vals: List[List[float]] = []
        self.cp: List[int] = []
        self.ms_ok: List[int] = []
        self.clock_abs: List[float] = []   # MS meta.clock
        self.rssi: List[Any] = []          # meta.rssi = msg_data.get('R')

    def add(self, msg: Dict[str, Any]) -> None:
        data = msg.get("data", "")
        ms_ok = 1
        cp_slot = -1
        clock_abs = 0.0
        if self.kind == "MS":
            # message_synced.py:21-47 -- the string gates, evaluated like the reference
            if not data or not data.isdigit():
                ms_ok = 0
            cps = msg.get("CP", "")
            if ms_ok and (not cps or not cps.isdigit()):
                ms_ok = 0
            sps = msg.get("SP", "")
            if ms_ok and (not sps or not sps.isdigit()):
                ms_ok = 0
            if ms_ok and "R" in msg:
                if not msg.get("R", "").isdigit():
                    ms_ok = 0
        elif not data:
            data = ""
        ids, vals = self._pat(msg) if (self.kind == "MU" and data) or (self.kind == "MS" and ms_ok) else ([], [])
        if self.kind == "MS" and ms_ok:
            key = str(int(msg["CP"]))
            if key in ids:
                cp_slot = ids.index(key)
                clock_abs = abs(vals[cp_slot])
            else:
                ms_ok = 0
        if not isinstance(data, str):
            raise TypeError(f"data must be str, got {type(data).__name__}")
        self.datas.append(_encode_data(data))
        self.npat.append(len(ids))
        self.ids.append(ids)
        self.vals.append(vals)
        self.cp.append(cp_slot)
        self.ms_ok.append(ms_ok)
        self.clock_abs.append(clock_abs)
        self.rssi.append(msg.get("R"))

    _pat = staticmethod(_patterns)

    def batch(self) -> PulseBatch:
        n = len(self.datas)
        lens = np.array([len(d) for d in self.datas], dtype=np.int64)
        offsets = np.zeros(n + 1, np.int64)
        np.cumsum(lens, out=offsets[1:])
        data = np.frombuffer(b"".join(self.datas), dtype=np.uint8).copy()
        pat_id = np.zeros((n, MAXPAT), np.uint8)
        pat_val = np.zeros((n, MAXPAT), np.float64)
        for i in range(n):
            for k, (pid, v) in enumerate(zip(self.ids[i], self.vals[i])):
                pat_id[i, k] = ord(pid)
                pat_val[i, k] = v
        return PulseBatch(self.kind, data, offsets, np.array(self.npat, np.uint8), pat_id, pat_val,
                          np.array(self.cp, np.int8), np.zeros(n, np.int8), np.full(n, -1, np.int32),
                          np.array(self.ms_ok, np.uint8))


def mc_batch_from_frames(frames: Sequence[Tuple[str, int, int, str, Any]]) -> McBatch:
    """frames: (raw_hex, clock, mcbitnum, messagetype, version)."""
    n = len(frames)
    hexes = [f[0].encode("latin-1") if isinstance(f[0], str) else bytes(f[0]) for f in frames]
    lens = np.array([len(h) for h in hexes], np.int64)
    offsets = np.zeros(n + 1, np.int64)
    np.cumsum(lens, out=offsets[1:])
    data = np.frombuffer(b"".join(hexes), np.uint8).copy()
    clock = np.array([int(f[1]) for f in frames], np.int32)
    L = np.array([int(f[2]) for f in frames], np.int32)
    mtype = np.array([1 if f[3] == "Mc" else 0 for f in frames], np.uint8)
    v32 = np.array([1 if (f[4] and str(f[4])[:6] == "V 3.2.") else 0 for f in frames], np.uint8)
    return McBatch(data, offsets, clock, L, mtype, v32)


class GeneralPacker(PulsePacker):
    """MU or MS messages for the general path (include/sdx.h sdx_general_batch): the same string
    gates and conversions as PulsePacker, pattern ids of any length (<= 15 digits), <= 16 patterns,
    any number of pulses."""

    _pat = staticmethod(_patterns_general)

    def arrays(self) -> Dict[str, np.ndarray]:
        n = len(self.datas)
        lens = np.array([len(d) for d in self.datas], dtype=np.int64)
        offsets = np.zeros(n + 1, np.int64)
        np.cumsum(lens, out=offsets[1:])
        ids = np.zeros((n, GEN_MAXPAT, GEN_IDSTR), np.uint8)
        vals = np.zeros((n, GEN_MAXPAT), np.float64)
        for i in range(n):
            for k, (pid, v) in enumerate(zip(self.ids[i], self.vals[i])):
                b = pid.encode("ascii")
                ids[i, k, 0] = len(b)
                ids[i, k, 1:1 + len(b)] = np.frombuffer(b, np.uint8)
                vals[i, k] = v
        return {"data": np.frombuffer(b"".join(self.datas), dtype=np.uint8).copy(), "offsets": offsets,
                "npat": np.array(self.npat, np.uint8), "pat_ids": ids, "pat_val": vals,
                "cp_slot": np.array(self.cp, np.int8), "ms_ok": np.array(self.ms_ok, np.uint8)}
