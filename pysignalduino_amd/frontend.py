"""Wire-line front end: raw SIGNALduino firmware lines -> DecodedMessage, on the GPU.

Mirrors the reference's parser entry point, ``signalduino.parser.SignalParser``
(signalduino/parser/__init__.py:18-77), and its data types ``RawFrame`` / ``DecodedMessage``
(signalduino/types.py:13-32).  Per line the reference runs, in Python: strip + STX/ETX framing,
Mred=1 decompression, routing by message type, the MU validity regex, ``_parse_to_dict``, the MC
header checks, then ``SDProtocols.demodulate*``.  Here a batch of lines is uploaded once and
  1. ``sdx_parse_lines``   (csrc/sdx_lines.hip) does all of the parsing, one lane per line, writing
                           the demodulators' SoA batch in place (slot layout, ``len_dev``),
  2. ``sdx_select_lines``  builds the per-kind selection lists (MU/MS short or long, MC) on the device,
  3. the MU / MS / MN (and, in mc_mode='fixed', MC) demodulation kernels run over those lists,
and only the result records come back.  The host side assembles the Python objects.

Observable behaviour per line is the reference's: ``parse_line`` returns the same
``DecodedMessage`` list (protocol_id, payload, metadata, raw.line / message_type / rssi /
freq_afc), and lines the reference ignores give ``[]`` (a demodulator exception is caught and
logged by the reference's parsers, so it also gives ``[]``).  Lines outside the device contract
(multi-digit pattern ids, non-integer pattern values, non-ASCII characters after decompression,
over-long messages, an MN R= of more than 15 digits) are never approximated: ``parse_line`` raises
:class:`ContractError` and ``parse_lines`` returns the exception in that line's slot.
There is no CPU fallback.
"""
from __future__ import annotations

import json
import logging
import re
from dataclasses import dataclass, field
from datetime import datetime
from typing import Any, List, Optional, Sequence, Union

import numpy as np

from . import runtime
from .packing import ContractError
from .sd_protocols import SDProtocols

_KIND_NAME = {runtime.LINE_MU: "MU", runtime.LINE_MS: "MS", runtime.LINE_MC: "MC", runtime.LINE_MN: "MN"}


@dataclass(slots=True)
class RawFrame:
    """signalduino/types.py:13-21."""

    line: str
    timestamp: datetime = field(default_factory=datetime.utcnow)
    rssi: Optional[float] = None
    freq_afc: Optional[float] = None
    message_type: Optional[str] = None


@dataclass(slots=True)
class DecodedMessage:
    """signalduino/types.py:24-31."""

    protocol_id: str
    payload: str
    raw: RawFrame
    metadata: dict = field(default_factory=dict)


def calc_rssi(raw_rssi: int) -> float:
    """parser/base.py calc_rssi."""
    if raw_rssi >= 128:
        return ((raw_rssi - 256) / 2) - 74
    return (raw_rssi / 2) - 74


def calc_afc(raw_afc: int) -> float:
    """parser/base.py calc_afc."""
    if raw_afc >= 128:
        return (raw_afc - 256) / 2
    return raw_afc / 2


def calc_mn_afc(raw_afc: int) -> float:
    """parser/mn.py:60-68 (the MN frame's A= field)."""
    return round((26000000 / 16384 * raw_afc / 1000), 0)


MN_PATTERN = re.compile(r"^MN;D=(Y?)([0-9A-F]+);(?:R=([0-9]+);)?(?:A=(-?[0-9]{1,3});)?$")  # parser/mn.py:17


def _to_bytes(line: Union[str, bytes]) -> bytes:
    if isinstance(line, (bytes, bytearray, memoryview)):
        return bytes(line)
    try:
        return line.encode("latin-1")  # the transport's decoding (transport.py:123), inverted
    except UnicodeEncodeError as e:
        raise ContractError("characters above U+00FF cannot come from the firmware transport") from e


class LineBatch:
    """Device buffers of one parsed batch (sdx_lines / sdx_lines_out of include/sdx.h)."""

    def __init__(self, eng: "runtime.Engine", data: np.ndarray, offsets: np.ndarray):
        t = eng.torch
        d = eng.dev
        n = len(offsets) - 1
        total = int(offsets[-1])
        self.n = n
        self.eng = eng
        # 16 bytes of padding: the kernel reads whole aligned 8-byte words (include/sdx.h)
        self.bytes = t.from_numpy(np.concatenate([data, np.zeros(16, np.uint8)])).to(d)
        self.offsets = t.from_numpy(offsets).to(d)
        e = lambda k, dt: t.empty(max(k, 1), dtype=dt, device=d)  # noqa: E731
        self.kind, self.status = e(n, t.uint8), e(n, t.uint8)
        self.slot = t.empty(3 * total + 16, dtype=t.uint8, device=d)
        self.doff, self.dlen = e(n, t.int64), e(n, t.int32)
        self.npat, self.pat_id, self.pat_val = e(n, t.uint8), e(10 * n, t.uint8), e(10 * n, t.float64)
        self.cp_slot, self.ms_ok = e(n, t.int8), e(n, t.uint8)
        self.clock, self.mcbitnum, self.mcflags = e(n, t.int32), e(n, t.int32), e(n, t.uint8)
        self.meta, self.plen = e(32 * n, t.uint8), e(n, t.int32)
        self.sel = e(n, t.int32)
        self.counts = t.zeros(8, dtype=t.int32, device=d)
        self.scratch = e(8 * ((n + runtime.SEL_CHUNK - 1) // runtime.SEL_CHUNK), t.int32)
        p = runtime._ptr
        self.c_lines = runtime.SdxLines(p(self.bytes), p(self.offsets), n)
        self.c_out = runtime.SdxLinesOut(p(self.kind), p(self.status), p(self.slot), p(self.doff), p(self.dlen),
                                         p(self.npat), p(self.pat_id), p(self.pat_val), p(self.cp_slot),
                                         p(self.ms_ok), p(self.clock), p(self.mcbitnum), p(self.mcflags),
                                         p(self.meta), p(self.plen))

    def launch(self) -> None:
        """sdx_parse_lines + sdx_select_lines on the engine's current stream (no host sync)."""
        import ctypes
        lib, st = self.eng.lib, self.eng.stream_ptr()
        runtime._check(lib, lib.sdx_parse_lines(ctypes.byref(self.c_lines), ctypes.byref(self.c_out), st))
        runtime._check(lib, lib.sdx_select_lines(ctypes.byref(self.c_out), self.n, runtime._ptr(self.sel),
                                                 runtime._ptr(self.counts), runtime._ptr(self.scratch), st))

    def selections(self):
        """Class sizes (one 32-byte read-back) -> device sub-lists of sel per class."""
        cnt = self.counts.cpu().numpy()[: runtime.SEL_NCLASS]
        start = np.concatenate([[0], np.cumsum(cnt)])
        return [self.sel[int(start[k]): int(start[k + 1])] for k in range(runtime.SEL_NCLASS)], cnt

    def mc_all(self, cnt):
        """Every MC line's index (the short and the long class: adjacent in sel) and their count."""
        a = int(np.sum(cnt[: runtime.SEL_MC]))
        k = int(cnt[runtime.SEL_MC]) + int(cnt[runtime.SEL_MC_LONG])
        return self.sel[a: a + k], k

    def pulse_batch(self):
        return {"data": self.slot, "offsets": self.doff, "npat": self.npat, "pat_id": self.pat_id,
                "pat_val": self.pat_val, "cp_slot": self.cp_slot, "ms_ok": self.ms_ok, "len": self.dlen, "n": self.n}

    def mn_batch(self):
        return {"hex": self.slot, "offsets": self.doff, "len": self.dlen, "n": self.n}

    def general(self, status: np.ndarray, kind_np: np.ndarray, line_kind: int):
        """The SDX_LS_GENERAL lines of one kind through sdx_lines_general + sdx_demod_pulses_general.
        Returns (rows, desc, rec, heap, vals [rows, 16], cp_slot) or None when there are none; rows whose
        general parse found them outside the contract are reported back in status (UNSUPPORTED)."""
        import ctypes
        rows = np.nonzero((status == runtime.LS_GENERAL) & (kind_np == line_kind))[0]
        if not len(rows):
            return None
        t, d, eng = self.eng.torch, self.eng.dev, self.eng
        m = len(rows)
        sel = t.from_numpy(rows.astype(np.int32)).to(d)
        g = {"offsets": t.empty(m, dtype=t.int64, device=d), "len": t.empty(m, dtype=t.int32, device=d),
             "npat": t.empty(m, dtype=t.uint8, device=d), "pat_ids": t.empty(m * 256, dtype=t.uint8, device=d),
             "pat_val": t.empty(m * 16, dtype=t.float64, device=d), "cp_slot": t.empty(m, dtype=t.int8, device=d),
             "ms_ok": t.empty(m, dtype=t.uint8, device=d)}
        p = runtime._ptr
        go = runtime.SdxLinesGeneralOut(p(g["offsets"]), p(g["len"]), p(g["npat"]), p(g["pat_ids"]), p(g["pat_val"]),
                                        p(g["cp_slot"]), p(g["ms_ok"]))
        runtime._check(eng.lib, eng.lib.sdx_lines_general(ctypes.byref(self.c_lines), ctypes.byref(self.c_out),
                                                          p(sel), m, ctypes.byref(go), eng.stream_ptr()))
        lens = g["len"].cpu().numpy()
        st = self.status[sel.long()].cpu().numpy()
        status[rows] = st                                   # lines found outside the contract
        g.update(data=self.slot, n=m, total=int(lens.sum()), lens_host=lens)
        kd = runtime.KIND_MU if line_kind == runtime.LINE_MU else runtime.KIND_MS
        desc, rec, heap = eng.run_general(kd, g, work_stride=5 * (int(lens.max()) + 512))
        return (rows, desc, rec, heap, g["pat_val"].cpu().numpy().reshape(m, 16),
                g["cp_slot"].cpu().numpy().astype(np.int64))

    def mc_batch(self):
        return {"hex": self.slot, "offsets": self.doff, "clock": self.clock, "mcbitnum": self.mcbitnum,
                "flags": self.mcflags, "len": self.dlen, "n": self.n}


def _contract(i: int, name) -> ContractError:
    """The slot value of a line whose demodulation hit a device limit (SDX_RAISE_CONTRACT): not a
    reference outcome, so it is reported, never turned into an empty result list."""
    return ContractError(f"line {i} ({name}) exceeds a limit of the device's general path "
                         "(include/sdx.h SDX_GEN_*, payloads > 65535 bytes)")


def pack_lines(lines: Sequence[Union[str, bytes]], copy: bool = True):
    """Concatenate lines into (data uint8, offsets int64[n+1]); per-line ContractError where a line
    cannot be represented (returned in ``bad``; such lines are replaced by an empty line).
    ``copy=False``: data is a read-only view of the joined bytes (one host copy fewer)."""
    if lines and set(map(type, lines)) == {str}:
        # all str (what the transports deliver): one join and one latin-1 encode for the whole batch
        # (a str's latin-1 bytes are as many as its characters); any character above U+00FF sends
        # the batch to the per-line path below, which marks just those lines
        try:
            blob = "".join(lines).encode("latin-1")
        except UnicodeEncodeError:
            blob = None
        if blob is not None:
            offsets = np.zeros(len(lines) + 1, np.int64)
            np.cumsum(np.fromiter(map(len, lines), np.int64, len(lines)), out=offsets[1:])
            data = np.frombuffer(blob, np.uint8)
            return (data.copy() if copy else data), offsets, {}
    bs, bad = [], {}
    for i, ln in enumerate(lines):
        try:
            bs.append(_to_bytes(ln))
        except ContractError as e:
            bad[i] = e
            bs.append(b"")
    lens = np.fromiter((len(b) for b in bs), np.int64, len(bs))
    offsets = np.zeros(len(bs) + 1, np.int64)
    np.cumsum(lens, out=offsets[1:])
    data = np.frombuffer(b"".join(bs), np.uint8)
    return (data.copy() if copy else data), offsets, bad


class SignalParser:
    """signalduino/parser/__init__.py:18-77 with the whole line -> DecodedMessage path on the GPU."""

    def __init__(self, protocols: Optional[SDProtocols] = None, logger: Optional[logging.Logger] = None,
                 rfmode: Optional[str] = None):
        self.protocols = protocols or SDProtocols()
        self.logger = logger or logging.getLogger(__name__)
        self.protocols.register_log_callback(self._log_adapter)
        self.rfmode = rfmode

    def _log_adapter(self, message: str, level: int):
        if level <= 1:
            self.logger.error(message)
        elif level == 2:
            self.logger.warning(message)
        elif level == 3:
            self.logger.info(message)
        else:
            self.logger.debug(message)

    # ------------------------------------------------------------------------------------------
    def parse_line(self, line: Union[str, bytes]) -> List[DecodedMessage]:
        """SignalParser.parse_line (parser/__init__.py:37-49)."""
        out = self.parse_lines([line])[0]
        if isinstance(out, BaseException):
            raise out
        return out

    def parse_lines(self, lines: Sequence[Union[str, bytes]]) -> List[Union[List[DecodedMessage], Exception]]:
        """Batch form of parse_line: one upload, one parse launch, one launch per demodulation
        variant, one read-back.  Returns one DecodedMessage list per line (or the ContractError
        for a line outside the device contract)."""
        n = len(lines)
        if n == 0:
            return []
        data, offsets, bad = pack_lines(lines)
        eng = self.protocols._ensure()
        bk = self.protocols._bank
        lb = LineBatch(eng, data, offsets)
        lb.launch()
        sels, cnt = lb.selections()
        res = {}
        pb = lb.pulse_batch()
        if cnt[runtime.SEL_MU_SHORT] or cnt[runtime.SEL_MU_LONG]:
            res["MU"] = eng.run(runtime.KIND_MU, pb, sel_short=sels[runtime.SEL_MU_SHORT],
                                sel_long=sels[runtime.SEL_MU_LONG])
        if cnt[runtime.SEL_MS_SHORT] or cnt[runtime.SEL_MS_LONG]:
            res["MS"] = eng.run(runtime.KIND_MS, pb, sel_short=sels[runtime.SEL_MS_SHORT],
                                sel_long=sels[runtime.SEL_MS_LONG])
        mc_sel, mc_n = lb.mc_all(cnt)
        if self.protocols.mc_mode == "fixed" and mc_n:
            res["MC"] = eng.run(runtime.KIND_MC, lb.mc_batch(), sel_short=mc_sel)
        if cnt[runtime.SEL_MN]:
            # result space: <= (MN protocols) records of <= (preamble + frame) bytes per line
            nmn = int(cnt[runtime.SEL_MN])
            res["MN"] = eng.run(runtime.KIND_MN, lb.mn_batch(), sel_short=sels[runtime.SEL_MN],
                                mn_elig=self.protocols.mn_eligibility(self.rfmode),
                                rec_cap=len(bk.mn_pids) * nmn + 1024, heap_cap=int(4 * len(data) + 64 * nmn + 65536))
        # read-back of the per-line fields the Python objects need
        kind = lb.kind[:n].cpu().numpy()
        status = lb.status[:n].cpu().numpy()
        # SDX_LS_GENERAL lines (multi-digit pattern ids, > 4096 pulses): the general path
        gen = {name: lb.general(status, kind, lk) for name, lk in (("MU", runtime.LINE_MU), ("MS", runtime.LINE_MS))}
        gen_of = {}
        for name, gr in gen.items():
            if gr is not None:
                for j, i in enumerate(gr[0]):
                    gen_of[int(i)] = (name, j)
        plen = lb.plen[:n].cpu().numpy()
        meta = lb.meta[: 32 * n].cpu().numpy().reshape(n, 32)
        need_slot = plen >= 0
        slot = lb.slot.cpu().numpy() if need_slot.any() else None
        ms_clock = None
        if "MS" in res:
            pv = lb.pat_val[: 10 * n].cpu().numpy().reshape(n, 10)
            cps = lb.cp_slot[:n].cpu().numpy().astype(np.int64)
            ok_ms = (kind == runtime.LINE_MS) & (status == runtime.LS_OK)  # cp_slot is written for these
            cps = np.where(ok_ms, np.clip(cps, 0, 9), 0)
            ms_clock = np.abs(pv[np.arange(n), cps])
        # the host assembly reads Python lists / str slices, not numpy rows: one bulk conversion per
        # array instead of a numpy scalar access per field (the per-line objects dominate this path)
        cols = {}
        for k, (desc, rec, heap) in res.items():
            cols[k] = (desc["status"].tolist(), desc["raise_kind"].tolist(), desc["n_rec"].tolist(),
                       desc["rec_begin"].tolist(), rec["proto"].tolist(), rec["payload_off"].tolist(),
                       rec["payload_len"].tolist(), rec["bit_length"].tolist(), heap.tobytes().decode("latin-1"))
        mb = meta.tobytes()
        sb = slot.tobytes() if slot is not None else b""
        hb_mn = res["MN"][2].tobytes() if "MN" in res else b""
        status_l, kind_l, plen_l, off_l = status.tolist(), kind.tolist(), plen.tolist(), offsets.tolist()
        ms_clock_l = ms_clock.tolist() if ms_clock is not None else None
        mu_pids, ms_pids, mc_pids, mu_clock = bk.mu_pids, bk.ms_pids, bk.mc_pids, bk.mu_clock
        ST_OK, ST_RAISED, R_CONTRACT = runtime.ST_OK, runtime.ST_RAISED, runtime.RAISE_CONTRACT
        out: List[Any] = []
        for i in range(n):
            if i in bad:
                out.append(bad[i])
                continue
            st = status_l[i]
            if st == runtime.LS_UNSUPPORTED:
                out.append(ContractError(f"line {i} is outside the device contract of the front end "
                                         f"(kind {_KIND_NAME.get(kind_l[i], '?')})"))
                continue
            name = _KIND_NAME.get(kind_l[i])
            if st == runtime.LS_GENERAL:
                gname, j = gen_of[i]
                _, gdesc, grec, gheap, gvals, gcps = gen[gname]
                out.append(self._general_messages(lines[i], i, plen, offsets, slot, meta, gname, gdesc[j], grec,
                                                  gheap.tobytes(), abs(float(gvals[j, max(0, int(gcps[j]))]))))
                continue
            if st != runtime.LS_OK or name not in res:
                out.append([])
                continue
            d_st, d_rk, d_nr, d_rb, r_p, r_off, r_len, r_bl, hs = cols[name]
            dst = d_st[i]
            if dst == ST_RAISED and d_rk[i] == R_CONTRACT:
                out.append(_contract(i, name))   # a device limit (MC frames > 128 hex: k_mc_general)
                continue
            nr = d_nr[i]
            if dst == ST_RAISED or nr == 0:
                out.append([])  # a demodulator exception is caught by the reference's parsers
                continue
            if dst != ST_OK:
                raise RuntimeError(f"device status {dst} for line {i}")
            if name == "MN":
                out.append(self._mn_messages(lines[i], i, plen, offsets, slot, meta, res[name][0][i], res[name][1],
                                             hb_mn))
                continue
            # RawFrame(line=payload) + _extract_metadata (mu.py:96-108, mc.py:141-155)
            pl = plen_l[i]
            if pl >= 0:
                s0 = 3 * off_l[i]
                payload_line = sb[s0: s0 + pl].decode("latin-1")
            else:
                ln = lines[i]
                payload_line = (ln.decode("latin-1") if isinstance(ln, (bytes, bytearray, memoryview)) else ln).strip()[1:-1]
            fr = RawFrame(line=payload_line, message_type=name)
            m0 = 32 * i
            rl, fl = mb[m0 + 15], mb[m0 + 31]
            rssi_raw = None if rl == 255 else mb[m0: m0 + rl].decode("latin-1")
            if rssi_raw is not None:
                try:
                    fr.rssi = calc_rssi(int(rssi_raw))
                except ValueError:
                    self.logger.warning("Could not parse %s value: %s", "RSSI", rssi_raw)
            if fl != 255:
                afc_raw = mb[m0 + 16: m0 + 16 + fl].decode("latin-1")
                try:
                    fr.freq_afc = calc_afc(int(afc_raw))
                except ValueError:
                    self.logger.warning("Could not parse %s value: %s", "AFC", afc_raw)
            msgs = []
            rb = d_rb[i]
            for r in range(rb, rb + nr):
                p = r_p[r]
                o = r_off[r]
                payload = hs[o: o + r_len[r]]
                if name == "MC":
                    pid = mc_pids[p]
                    md = {"protocol_id": pid, "rssi": None, "freq_afc": None}
                elif name == "MU":
                    pid = mu_pids[p]
                    md = {"bit_length": r_bl[r], "rssi": rssi_raw, "clock": mu_clock[p]}
                else:
                    pid = ms_pids[p]
                    md = {"bit_length": r_bl[r], "rssi": rssi_raw, "clock": ms_clock_l[i]}
                msgs.append(DecodedMessage(protocol_id=str(pid), payload=payload, raw=fr, metadata=md))
            out.append(msgs)
        return out

    def _general_messages(self, line, i, plen, offsets, slot, meta, name, d, rec, hb, ms_clock) -> List[DecodedMessage]:
        """The DecodedMessage list of a general-path line (as the OK lines' records below)."""
        bk = self.protocols._bank
        if d["status"] == runtime.ST_RAISED and int(d["raise_kind"]) == runtime.RAISE_CONTRACT:
            return _contract(i, name)   # a general-path limit (SDX_GEN_*), not a reference outcome
        if d["status"] == runtime.ST_RAISED or int(d["n_rec"]) == 0:
            return []   # a demodulator exception is caught by the reference's parsers
        if d["status"] != runtime.ST_OK:
            raise RuntimeError(f"device status {int(d['status'])} for line {i}")
        fr = self._frame(line, i, plen, offsets, slot, meta, name)
        rssi_raw = self._meta_str(meta[i], 0)
        msgs = []
        for r in rec[int(d["rec_begin"]): int(d["rec_begin"]) + int(d["n_rec"])]:
            p = int(r["proto"])
            off = int(r["payload_off"])
            pid = bk.mu_pids[p] if name == "MU" else bk.ms_pids[p]
            md = {"bit_length": int(r["bit_length"]), "rssi": rssi_raw,
                  "clock": bk.mu_clock[p] if name == "MU" else ms_clock}
            msgs.append(DecodedMessage(protocol_id=str(pid), payload=hb[off: off + int(r["payload_len"])].decode("latin-1"),
                                       raw=fr, metadata=md))
        return msgs

    def _payload(self, line, i, plen, offsets, slot) -> str:
        if plen[i] >= 0:
            s0 = 3 * int(offsets[i])
            return bytes(slot[s0: s0 + int(plen[i])]).decode("latin-1")
        s = line.decode("latin-1") if isinstance(line, (bytes, bytearray, memoryview)) else line
        return s.strip()[1:-1]

    def _mn_messages(self, line, i, plen, offsets, slot, meta, d, rec, hb) -> List[DecodedMessage]:
        """DecodedMessage list of an MN line (parser/mn.py:53-77,175-191): RawFrame(line=payload,
        message_type='MN') without frame rssi/afc; metadata rssi / freq_afc / modulation / rfmode."""
        bk = self.protocols._bank
        fr = RawFrame(line=self._payload(line, i, plen, offsets, slot), message_type="MN")
        r, a = self._meta_str(meta[i], 0), self._meta_str(meta[i], 16)
        rssi = calc_rssi(int(r)) if r else None
        afc = calc_mn_afc(int(a)) if a else None
        msgs = []
        for x in rec[int(d["rec_begin"]): int(d["rec_begin"]) + int(d["n_rec"])]:
            p = int(x["proto"])
            off = int(x["payload_off"])
            msgs.append(DecodedMessage(protocol_id=str(bk.mn_pids[p]),
                                       payload=hb[off: off + int(x["payload_len"])].decode("latin-1"), raw=fr,
                                       metadata={"rssi": rssi, "freq_afc": afc, "modulation": bk.mn_modulation[p],
                                                 "rfmode": bk.mn_rfmode[p]}))
        return msgs

    # ------------------------------------------------------------------------------------------
    def stream(self, chunk_lines: int = 250_000, chunk_bytes: Optional[int] = None, output: str = "json",
               lag: int = 3):
        """A pipelined LineStream over this parser (pysignalduino_amd/stream.py): chunks of raw lines
        in, the controller's JSON texts (or the wire form) out, the PCIe copies, parse, demodulation
        and serialisation of successive chunks overlapping; the same per-line results as
        parse_lines_json / parse_lines."""
        from .stream import LineStream
        return LineStream(self, chunk_lines=chunk_lines, chunk_bytes=chunk_bytes, output=output, lag=lag)

    def parse_lines_json(self, lines: Sequence[Union[str, bytes]]) -> List[Union[Optional[str], Exception]]:
        """Per line, the MQTT message text the reference controller publishes for it:
        ``MqttPublisher._message_to_json(parse_line(line)[0])`` (signalduino/controller.py:254-257,
        mqtt.py:227-245), or None when the line decodes to nothing -- parse, demodulation and JSON
        serialisation (sdx_serialize_json) all on the device; only the texts come back."""
        n = len(lines)
        if n == 0:
            return []
        data, offsets, bad = pack_lines(lines)
        eng = self.protocols._ensure()
        bk = self.protocols._bank
        lb = LineBatch(eng, data, offsets)
        lb.launch()
        sels, cnt = lb.selections()
        lo = {"meta": lb.meta, "pat_val": lb.pat_val, "cp_slot": lb.cp_slot}
        pb = lb.pulse_batch()
        jobs = []
        if cnt[runtime.SEL_MU_SHORT] or cnt[runtime.SEL_MU_LONG]:
            k = int(cnt[runtime.SEL_MU_SHORT] + cnt[runtime.SEL_MU_LONG])
            jobs.append((runtime.KIND_MU, 8 * k + 1024, 200 * k + 65536, 600 * k + 65536,
                         [(pb, sels[runtime.SEL_MU_SHORT], False), (pb, sels[runtime.SEL_MU_LONG], True)]))
        if cnt[runtime.SEL_MS_SHORT] or cnt[runtime.SEL_MS_LONG]:
            k = int(cnt[runtime.SEL_MS_SHORT] + cnt[runtime.SEL_MS_LONG])
            jobs.append((runtime.KIND_MS, 4 * k + 1024, 64 * k + 65536, 300 * k + 65536,
                         [(pb, sels[runtime.SEL_MS_SHORT], False), (pb, sels[runtime.SEL_MS_LONG], True)]))
        mc_sel, k = lb.mc_all(cnt)
        if self.protocols.mc_mode == "fixed" and k:
            jobs.append((runtime.KIND_MC, 4 * k + 1024, 96 * k + 65536, 400 * k + 65536,
                         [(lb.mc_batch(), mc_sel, False)]))
        if cnt[runtime.SEL_MN]:
            k = int(cnt[runtime.SEL_MN])
            jobs.append((runtime.KIND_MN, len(bk.mn_pids) * k + 1024, int(4 * len(data) + 64 * k + 65536),
                         int(6 * len(data) + 400 * k + 65536), [(lb.mn_batch(), sels[runtime.SEL_MN], False)]))
        elig = self.protocols.mn_eligibility(self.rfmode)
        texts: List[Any] = [None] * n
        host_rows: List[int] = []   # lines whose text is built from parse_lines' objects (general paths)
        for kind, rec_cap, heap_cap, json_cap, launches in jobs:
            for _attempt in range(4):
                work = eng.pulses_work_bytes(n) if kind in (runtime.KIND_MU, runtime.KIND_MS) else 0
                out = eng.alloc_out(n, rec_cap, heap_cap, work)  # MU/MS: grouped order + spill room
                for bd, sel, long_v in launches:
                    if not sel.numel():
                        continue
                    if kind == runtime.KIND_MN:
                        eng.launch_mn(bd, out, elig=elig, sel=sel)
                    elif kind == runtime.KIND_MC:
                        eng.launch_mc(bd, out, sel=sel)
                    else:
                        eng.launch_pulses(kind, bd, out, sel=sel, long_variant=long_v)
                jo = eng.alloc_json(n, json_cap)
                eng.launch_json(kind, out, lo, n, jo, first_only=True)
                c1 = out["cursor"].cpu().numpy()
                c2 = jo["cursor"].cpu().numpy()
                if kind == runtime.KIND_MC and c1[2] == 2 and not c2[1]:
                    # frames of > 128 hex characters were handed over (ST_OVF_TILE): their texts below
                    sel = launches[0][1]
                    st = out["desc"][: 8 * n].view(-1, 8)[:, 6][sel.long()].cpu().numpy()
                    host_rows.extend(int(i) for i in sel.cpu().numpy()[st == runtime.ST_OVF_TILE])
                    break
                if not c1[2] and not c2[1]:
                    break
                rec_cap, heap_cap, json_cap = 4 * rec_cap, 4 * heap_cap, 4 * json_cap
            else:
                raise RuntimeError("result / JSON capacity overflow persists")
            lens = jo["len"][:n].cpu().numpy()
            offs = jo["off"][:n].cpu().numpy()
            blob = jo["json"][: int(c2[0])].cpu().numpy().tobytes()
            for i in np.nonzero(lens > 0)[0]:
                texts[int(i)] = blob[int(offs[i]): int(offs[i]) + int(lens[i])].decode("ascii")
        status = lb.status[:n].cpu().numpy()
        kinds = lb.kind[:n].cpu().numpy()
        grows = [int(i) for i in np.nonzero(status == runtime.LS_GENERAL)[0] if int(i) not in bad] + host_rows
        if grows:  # general-path lines (rare): their objects through parse_lines, the text as _message_to_json
            for i, g in zip(grows, self.parse_lines([lines[i] for i in grows])):
                if isinstance(g, BaseException):
                    texts[i] = g
                elif g:
                    texts[i] = json.dumps({"protocol_id": g[0].protocol_id, "payload": g[0].payload,
                                           "metadata": g[0].metadata}, indent=4)
        for i in range(n):
            if i in bad:
                texts[i] = bad[i]
            elif int(status[i]) == runtime.LS_UNSUPPORTED:
                texts[i] = ContractError(f"line {i} is outside the device contract of the front end "
                                         f"(kind {_KIND_NAME.get(int(kinds[i]), '?')})")
        return texts

    @staticmethod
    def _meta_str(m: np.ndarray, base: int) -> Optional[str]:
        ln = int(m[base + 15])
        return None if ln == 255 else bytes(m[base: base + ln]).decode("latin-1")

    def _frame(self, line, i, plen, offsets, slot, meta, name) -> RawFrame:
        """RawFrame(line=payload, message_type) + _extract_metadata (mu.py:96-108, mc.py:141-155)."""
        fr = RawFrame(line=self._payload(line, i, plen, offsets, slot), message_type=name)
        r, f = self._meta_str(meta[i], 0), self._meta_str(meta[i], 16)
        for raw, attr, fn in ((r, "rssi", calc_rssi), (f, "freq_afc", calc_afc)):
            if raw is None:
                continue
            try:
                setattr(fr, attr, fn(int(raw)))
            except ValueError:
                self.logger.warning("Could not parse %s value: %s", "RSSI" if attr == "rssi" else "AFC", raw)
        return fr


class MNParser:
    """signalduino/parser/mn.py:20-191: MN frames -> DecodedMessage, the protocol loop on the GPU.

    ``parse(frame)`` / ``parse_batch(frames)`` take RawFrames whose ``line`` is the payload (as the
    reference's SignalParser hands them over).  MN_PATTERN is matched per frame on the host (the
    batched line path, :class:`SignalParser`, does it on the device), then one ``sdx_demod_mn``
    launch runs the rfmode / length / regexMatch / method loop for every matched frame."""

    def __init__(self, protocols: SDProtocols, logger: Optional[logging.Logger] = None, rfmode: Optional[str] = None):
        self.protocols = protocols
        self.logger = logger or logging.getLogger(__name__)
        self.rfmode = rfmode

    def parse(self, frame: RawFrame) -> List[DecodedMessage]:
        return self.parse_batch([frame])[0]

    def parse_batch(self, frames: Sequence[RawFrame]) -> List[List[DecodedMessage]]:
        rows, hexes, meta = [], [], []
        for k, fr in enumerate(frames):
            if not fr.line.upper().startswith("MN"):        # ensure_message_type (base.py:211-213)
                self.logger.debug("Not an MN message: %s", fr.line[:2])
                continue
            m = MN_PATTERN.match(fr.line)
            if not m:
                self.logger.debug("MN message format mismatch: %s", fr.line)
                continue
            rows.append(k)
            hexes.append(m.group(2))
            meta.append((calc_rssi(int(m.group(3))) if m.group(3) else None,
                         calc_mn_afc(int(m.group(4))) if m.group(4) else None))
        out: List[List[DecodedMessage]] = [[] for _ in frames]
        if not rows:
            return out
        bk = None
        for k, res, (rssi, afc) in zip(rows, self.protocols.mn_parse_batch(hexes, self.rfmode), meta):
            bk = bk or self.protocols._bank
            out[k] = [DecodedMessage(protocol_id=str(pid), payload=payload, raw=frames[k],
                                     metadata={"rssi": rssi, "freq_afc": afc, "modulation": bk.mn_modulation[p],
                                               "rfmode": bk.mn_rfmode[p]}) for pid, payload, p in res]
        return out
