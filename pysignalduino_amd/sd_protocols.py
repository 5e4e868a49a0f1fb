"""Drop-in ``SDProtocols`` whose MU/MS/MC demodulation runs on the MI355X.

Mirrors the reference class RFD-FHEM/PySignalduino ``sd_protocols.SDProtocols``
(sd_protocols/sd_protocols.py:13-170) for the hot path:

  * property API: protocol_exists / get_protocol_list / get_keys / check_property /
    get_property / set_defaults / register_log_callback / length_in_range
    (sd_protocols.py:43-58,157-170; helpers.py:124-166) -- host dictionary logic;
  * demodulate / demodulate_mu / demodulate_ms / demodulate_mc (sd_protocols.py:60-111,
    message_unsynced.py:11, message_synced.py:10) -- packed and run by the HIP
    kernels in csrc/sdx_kernels.hip through the C-ABI include/sdx.h;
  * demodulate_batch(list_of_msg_data, msg_type) -- the batched entry point;
  * MN (FSK): demodulate_mn (sd_protocols.py:113-154), the seven MN methods ConvBresser_lightning /
    _5in1 / _6in1 / _7in1, ConvPCA301, ConvKoppFreeControl, ConvLaCrosse (helpers.py:223-716) and
    mn_parse_batch (the protocol loop of signalduino/parser/mn.py:79-191) -- run by
    csrc/sdx_mn.hip through sdx_demod_mn.

It is injected where the reference injects its engine:
``SignalParser(protocols=SDProtocols())`` (signalduino/parser/__init__.py:21-27).

Results are the reference's list of ``{"protocol_id", "payload", "meta"}`` dicts,
bit-exact; a message on which the reference raises re-raises the same exception
class here (the parsers catch ``Exception`` and yield nothing, parser/mu.py:64-68).
There is no CPU fallback: without the HIP library / a GPU every demodulate call raises.
"""
from __future__ import annotations

import json
import re
from typing import Any, Dict, Iterable, List, Optional, Sequence

import numpy as np

from . import bank as bankmod
from . import packing
from . import runtime
from .units import UnitsMixin

_SENTINEL = object()
_HEX_RE = re.compile(r"[0-9a-fA-F]*")


class _Observed(dict):
    """dict that bumps a shared version counter on mutation (nested protocol dicts too),
    so a test or user editing ``_protocols[pid][key]`` gets the bank recompiled."""

    def __init__(self, data, owner):
        super().__init__()
        self._owner = owner
        for k, v in data.items():
            dict.__setitem__(self, k, _Observed(v, owner) if isinstance(v, dict) and not isinstance(v, _Observed) else v)

    def _bump(self):
        self._owner._version += 1

    def __setitem__(self, k, v):
        if isinstance(v, dict) and not isinstance(v, _Observed):
            v = _Observed(v, self._owner)
        dict.__setitem__(self, k, v)
        self._bump()

    def __delitem__(self, k):
        dict.__delitem__(self, k)
        self._bump()

    def setdefault(self, k, default=None):
        if k not in self:
            self[k] = default
        return dict.__getitem__(self, k)

    def update(self, *a, **kw):
        for k, v in dict(*a, **kw).items():
            self[k] = v

    def pop(self, *a):
        r = dict.pop(self, *a)
        self._bump()
        return r

    def clear(self):
        dict.clear(self)
        self._bump()


class SDProtocols(UnitsMixin):
    """GPU-backed drop-in for ``sd_protocols.SDProtocols`` (demodulation path)."""

    def __init__(self, protocols_path: Optional[str] = None, device: int = 0, mc_mode: str = "strict"):
        if mc_mode not in ("strict", "fixed"):
            raise ValueError("mc_mode must be 'strict' (reference-observable) or 'fixed'")
        self._version = 0
        self._protocols = _Observed(bankmod.load_protocols(protocols_path), self)
        self._log_callback = None
        self.device = device
        self.mc_mode = mc_mode
        self.set_defaults()
        self._bank = None
        self._bank_version = -1
        self._engine = None

    # ---------------------------------------------------------------- property API (host) ------
    def protocol_exists(self, pid: str) -> bool:
        return pid in self._protocols

    def get_protocol_list(self) -> dict:
        return self._protocols

    def get_keys(self, filter_key: str = None) -> list:
        if filter_key:
            return [pid for pid, props in self._protocols.items() if filter_key in props]
        return list(self._protocols.keys())

    def check_property(self, pid: str, value_name: str, default=None):
        return self._protocols.get(pid, {}).get(value_name, default)

    def get_property(self, pid: str, value_name: str):
        return self._protocols.get(pid, {}).get(value_name)

    def set_defaults(self):
        for pid, proto in self._protocols.items():
            proto.setdefault("active", True)
            proto.setdefault("name", f"Protocol_{pid}")

    def register_log_callback(self, callback):
        if callable(callback):
            self._log_callback = callback

    def _logging(self, message: str, level: int = 3):
        if self._log_callback:
            self._log_callback(message, level)

    def length_in_range(self, protocol_id, message_length):
        """helpers.py:124-166."""
        if not self.protocol_exists(str(protocol_id)):
            return (0, "protocol does not exists")
        min_len = self.check_property(protocol_id, "length_min", -1)
        if min_len is not None:
            try:
                min_len = int(min_len)
            except (ValueError, TypeError):
                pass
        if min_len != -1 and message_length < min_len:
            return (0, "message is too short")
        max_len = self.get_property(protocol_id, "length_max")
        if max_len is not None:
            try:
                max_len = int(max_len)
                if message_length > max_len:
                    return (0, "message is too long")
            except (ValueError, TypeError):
                pass
        return (1, "")

    # ---------------------------------------------------------------- device plumbing ----------
    def _ensure(self):
        if self._bank is None or self._bank_version != self._version:
            raw = json.loads(json.dumps(self._protocols))
            self._bank = bankmod.Bank(raw)
            self._bank_version = self._version
            if self._engine is not None:
                self._engine.close()
                self._engine = None
        if self._engine is None:
            self._engine = runtime.Engine(self._bank, self.device)
        return self._engine

    # ---------------------------------------------------------------- demodulation -------------
    def demodulate(self, msg_data: Dict[str, Any], msg_type: str) -> list:
        """sd_protocols.py:60-74."""
        if msg_type == "MS":
            return self.demodulate_ms(msg_data, msg_type)
        if msg_type == "MC":
            return self.demodulate_mc(msg_data, msg_type)
        if msg_type == "MN":
            return self.demodulate_mn(msg_data, msg_type)
        if msg_type == "MU":
            return self.demodulate_mu(msg_data, msg_type)
        self._logging(f"Unknown message type {msg_type}", 3)
        return []

    def demodulate_mu(self, msg_data: Dict[str, Any], msg_type: str = "MU") -> list:
        return self._single(msg_data, "MU")

    def demodulate_ms(self, msg_data: Dict[str, Any], msg_type: str = "MS") -> list:
        return self._single(msg_data, "MS")

    # ---------------------------------------------------------------- MN (FSK) -----------------
    def demodulate_mn(self, msg_data: Dict[str, Any], msg_type: str = "MN") -> list:
        """sd_protocols.py:113-154: the protocol's MN method on msg_data['data'] (GPU)."""
        if "protocol_id" not in msg_data:
            self._logging(f"MN Demodulation failed: Missing protocol_id in msg_data: {msg_data}", 3)
            return []
        protocol_id = msg_data["protocol_id"]
        if not self.protocol_exists(protocol_id):
            self._logging(f"MN Demodulation: Protocol ID {protocol_id} not found.", 3)
            return []
        method_name_full = self.get_property(protocol_id, "method")
        if not method_name_full:
            self._logging(f"MN Demodulation: No method defined for protocol {protocol_id}. "
                          f"Data: {msg_data.get('data', '')}", 3)
            return []
        name = method_name_full.split(".")[-1]
        if name not in bankmod.MN_METHODS:
            # a name the class does not define, or one called with the wrong arguments (TypeError)
            self._logging(f"MN Demodulation: Unknown method {name} referenced by '{method_name_full}'.", 3)
            return []
        return self.mn_method_batch([msg_data], name, msg_type)[0]

    def ConvBresser_lightning(self, msg_data, msg_type="MN"):  # noqa: N802  (helpers.py:223)
        return self.mn_method_batch([msg_data], "ConvBresser_lightning", msg_type)[0]

    def ConvBresser_5in1(self, msg_data, msg_type="MN"):  # noqa: N802  (helpers.py:382)
        return self.mn_method_batch([msg_data], "ConvBresser_5in1", msg_type)[0]

    def ConvBresser_6in1(self, msg_data, msg_type="MN"):  # noqa: N802  (helpers.py:427)
        return self.mn_method_batch([msg_data], "ConvBresser_6in1", msg_type)[0]

    def ConvBresser_7in1(self, msg_data, msg_type="MN"):  # noqa: N802  (helpers.py:473)
        return self.mn_method_batch([msg_data], "ConvBresser_7in1", msg_type)[0]

    def ConvPCA301(self, msg_data, msg_type="MN"):  # noqa: N802  (helpers.py:525)
        return self.mn_method_batch([msg_data], "ConvPCA301", msg_type)[0]

    def ConvKoppFreeControl(self, msg_data, msg_type="MN"):  # noqa: N802  (helpers.py:581)
        return self.mn_method_batch([msg_data], "ConvKoppFreeControl", msg_type)[0]

    def ConvLaCrosse(self, msg_data, msg_type="MN"):  # noqa: N802  (helpers.py:630)
        return self.mn_method_batch([msg_data], "ConvLaCrosse", msg_type)[0]

    _MN_META = {"ConvPCA301": {"is_raw": False}, "ConvKoppFreeControl": {"is_raw": False},
                "ConvLaCrosse": {"is_raw": False}}

    @staticmethod
    def _mn_hex(d) -> str:
        """The device contract of an MN frame: hex digits only, at most MN_HEX_MAX of them."""
        if not isinstance(d, str) or len(d) > runtime.MN_HEX_MAX or not _HEX_RE.fullmatch(d):
            raise packing.ContractError("MN data must be a string of at most "
                                        f"{runtime.MN_HEX_MAX} hex digits for the device path")
        return d

    def mn_method_batch(self, messages: Sequence[Dict[str, Any]], name: str, msg_type: str = "MN") -> List[list]:
        """One MN method (helpers.py:223-716) over many msg_data dicts in one launch: the
        reference's list per message ([] or [{protocol_id, payload, meta}])."""
        method = bankmod.MN_METHODS[name]
        out: List[Any] = [[] for _ in messages]
        idx, hexes = [], []
        for i, m in enumerate(messages):
            d = m.get("data")
            if not d:                    # `if not hex_data: return []`
                continue
            hexes.append(self._mn_hex(d))
            idx.append(i)
        if not idx:
            return out
        eng = self._ensure()
        desc, rec, heap = eng.run(runtime.KIND_MN, eng.to_device_mn(hexes), mn_method=method)
        hb = heap.tobytes()
        meta = self._MN_META.get(name, {})
        for j, i in enumerate(idx):
            d = desc[j]
            if d["status"] != runtime.ST_OK:
                raise RuntimeError(f"device status {int(d['status'])} for MN frame {i}")
            if int(d["n_rec"]):
                r = rec[int(d["rec_begin"])]
                p = hb[int(r["payload_off"]): int(r["payload_off"]) + int(r["payload_len"])].decode("latin-1")
                out[i] = [{"protocol_id": messages[i].get("protocol_id"), "payload": p, "meta": dict(meta)}]
        return out

    def mn_eligibility(self, rfmode: Optional[str]) -> int:
        """parser/mn.py:83-93 as the 64-bit protocol mask of sdx_mn_batch.elig."""
        self._ensure()
        m = 0
        for k, prf in enumerate(self._bank.mn_rfmode):
            if prf and not (rfmode and prf != rfmode):
                m |= 1 << k
        return m

    def mn_parse_batch(self, hexes: Sequence[str], rfmode: Optional[str] = None):
        """The protocol loop of MNParser.parse (parser/mn.py:79-191) for many frames whose
        MN_PATTERN matched: per frame the list of (protocol_id, payload, mn-table index)."""
        for h in hexes:
            self._mn_hex(h)
        eng = self._ensure()
        if not len(hexes):
            return []
        desc, rec, heap = eng.run(runtime.KIND_MN, eng.to_device_mn(hexes), mn_elig=self.mn_eligibility(rfmode))
        return self._mn_results(desc, rec, heap, range(len(hexes)))

    def _mn_results(self, desc, rec, heap, rows):
        bk = self._bank
        hb = heap.tobytes()
        out = []
        for i in rows:
            d = desc[i]
            if d["status"] != runtime.ST_OK:
                raise RuntimeError(f"device status {int(d['status'])} for MN frame {i}")
            res = []
            for r in rec[int(d["rec_begin"]): int(d["rec_begin"]) + int(d["n_rec"])]:
                p = int(r["proto"])
                off = int(r["payload_off"])
                res.append((bk.mn_pids[p], hb[off: off + int(r["payload_len"])].decode("latin-1"), p))
            out.append(res)
        return out

    def _single(self, msg_data, kind):
        out = self.demodulate_batch([msg_data], kind, raise_errors=True)
        return out[0]

    def demodulate_batch(self, messages: Sequence[Dict[str, Any]], msg_type: str, raise_errors: bool = False):
        """Demodulate many messages in one GPU pass.

        Returns one result list per message.  A message on which the reference raises
        yields the exception instance (or re-raises it when ``raise_errors``); so does a message
        outside the device contract (``packing.ContractError``), without failing the others.
        """
        if msg_type == "MC":
            return [self._catch(self.demodulate_mc, m, "MC", raise_errors=raise_errors) for m in messages] \
                if self.mc_mode == "strict" else self.demodulate_mc_batch(messages, raise_errors=raise_errors)
        if msg_type not in ("MU", "MS"):
            return [self.demodulate(m, msg_type) for m in messages]
        packer, gen, gen_rows, pack_err = self._pack_pulses(messages, msg_type, raise_errors)
        pb = packer.batch()
        eng = self._ensure()
        kind = runtime.KIND_MU if msg_type == "MU" else runtime.KIND_MS
        desc, rec, heap = eng.run(kind, eng.to_device_pulses(pb))
        out = self._decode_pulses(msg_type, desc, rec, heap, packer, pack_err, raise_errors)
        if gen_rows:
            gd, gr, gh = eng.run_general(kind, eng.to_device_general(gen.arrays()))
            res = self._decode_pulses(msg_type, gd, gr, gh, gen, {}, raise_errors)
            for j, i in enumerate(gen_rows):
                out[i] = res[j]
        return out

    @staticmethod
    def _pack_pulses(messages, msg_type, raise_errors=False):
        """messages -> (PulsePacker with one entry per message, GeneralPacker of the general-path
        messages, their rows, {row: exception} of the messages whose host conversion raised)."""
        packer = packing.PulsePacker(msg_type)
        gen = packing.GeneralPacker(msg_type)   # multi-digit pattern ids / more than LONG_MAX pulses
        gen_rows: List[int] = []
        pack_err: Dict[int, BaseException] = {}
        for i, m in enumerate(messages):
            try:
                d = m.get("data", "")
                try:
                    if isinstance(d, str) and len(d) > runtime.LONG_MAX:
                        raise packing.GeneralPathMessage("longer than the long kernel's pulses")
                    packer.add(m)
                except packing.GeneralPathMessage:
                    gen.add(m)                      # same gates and conversions, general layout
                    gen_rows.append(i)
                    packer.add({"data": ""})
            except Exception as e:  # the reference raises on this message (same class), or the
                if raise_errors:    # message is outside the device contract (ContractError): per slot
                    raise
                pack_err[i] = e
                packer.add({"data": ""})
        return packer, gen, gen_rows, pack_err

    @classmethod
    def _pack_error(cls, msg, msg_type) -> BaseException:
        """The exception the host conversion of one message raises (the same steps as _pack_pulses)."""
        err = cls._pack_pulses([msg], msg_type)[3]
        return err.get(0, RuntimeError("host packing of this message raised on another rank only"))

    @staticmethod
    def _catch(fn, m, t, raise_errors):
        try:
            return fn(m, t)
        except Exception as e:
            if raise_errors:
                raise
            return e

    def _decode_pulses(self, kind, desc, rec, heap, packer, pack_err, raise_errors):
        bk = self._bank
        pids = bk.mu_pids if kind == "MU" else bk.ms_pids
        hs = heap.tobytes().decode("latin-1")   # latin-1 maps bytes 1:1: str slices == decoded byte slices
        # bulk conversions: Python lists instead of a numpy scalar access per field and record
        d_st, d_rk, d_rb, d_nr = (desc["status"].tolist(), desc["raise_kind"].tolist(), desc["rec_begin"].tolist(),
                                  desc["n_rec"].tolist())
        r_p, r_off, r_len, r_bl = (rec["proto"].tolist(), rec["payload_off"].tolist(), rec["payload_len"].tolist(),
                                   rec["bit_length"].tolist())
        mu = kind == "MU"
        clocks = bk.mu_clock if mu else None
        out: List[Any] = []
        for i in range(len(d_st)):
            if i in pack_err:
                out.append(pack_err[i])
                continue
            st = d_st[i]
            if st == runtime.ST_RAISED:
                rk = d_rk[i]
                if rk == runtime.RAISE_CONTRACT:
                    exc = packing.ContractError(f"{kind} message exceeds a general-path limit (include/sdx.h SDX_GEN_*)")
                else:
                    exc = runtime.RAISE_NAMES.get(rk, RuntimeError)(
                        f"reference raises {runtime.RAISE_NAMES.get(rk, RuntimeError).__name__} "
                        f"on this {kind} message")
                if raise_errors:
                    raise exc
                out.append(exc)
                continue
            if st != runtime.ST_OK:
                raise RuntimeError(f"device status {st} for message {i}")
            res = []
            rssi = packer.rssi[i]
            b = d_rb[i]
            for r in range(b, b + d_nr[i]):
                p = r_p[r]
                o = r_off[r]
                res.append({"protocol_id": pids[p], "payload": hs[o: o + r_len[r]],
                            "meta": {"bit_length": r_bl[r], "rssi": rssi,
                                     "clock": clocks[p] if mu else packer.clock_abs[i]}})
            out.append(res)
        return out

    # ---------------------------------------------------------------- MC -----------------------
    def demodulate_mc(self, msg_data: Dict[str, Any], msg_type: str, version: Optional[str] = None) -> list:
        """sd_protocols.py:76-111.

        mc_mode='strict' (default): exactly the reference's observable behaviour.  Without a
        ``protocol_id`` (how MCParser calls it, parser/mc.py:78) the result is [].  With one, the
        reference's gates run with the same Python operations (manchester.py:70-120): [] when a
        length gate fails, TypeError for every clockrange protocol (``int > list`` at :83-84) and
        for every method call (one positional argument too many at :120; mcRaw's shifted
        arguments run on the device), ValueError for a protocol without a method (a one-element
        list unpacked into three names, sd_protocols.py:94).
        mc_mode='fixed': the intended chain (clockrange[0] < C < clockrange[1], method called
        without the extra ``self``) on the GPU for every clockrange protocol (or the given id).
        """
        if self.mc_mode == "fixed":
            return self.demodulate_mc_batch([msg_data], msg_type=msg_type, version=version, raise_errors=True)[0]
        protocol_id = msg_data.get("protocol_id")
        if not protocol_id or not self.protocol_exists(protocol_id):
            self._logging(f"MC Demodulation failed: Protocol ID {protocol_id} not found or missing.", 3)
            return []
        rcode, dmsg, metadata = self._mc_data_strict(
            f"Protocol {protocol_id}", protocol_id, msg_data.get("clock", 0), msg_data.get("data", ""),
            msg_data.get("bit_length", 0), msg_type, version)
        if rcode == 1:
            return [{"protocol_id": str(protocol_id), "payload": dmsg, "meta": metadata}]
        return []

    def demodulate_mc_batch(self, messages: Sequence[Dict[str, Any]], msg_type: str = "MC",
                            version: Optional[str] = None, raise_errors: bool = False):
        """'fixed' MC chain on the GPU; accepts MCParser dicts (raw_hex/clock/mcbitnum/messagetype)
        or demodulate_mc dicts (data/clock/bit_length)."""
        frames, slot_err, only = self._mc_frames(messages, msg_type, version, raise_errors)
        mb = packing.mc_batch_from_frames(frames)
        eng = self._ensure()
        bd = eng.to_device_mc(mb)
        # demodulate_mc(msg_data) with a protocol_id evaluates that protocol only (sd_protocols.py:
        # 79-99): a raise of another id must not surface for it, so the device skips the others
        if any(only):
            bd["only"] = self._mc_only(only, eng)
        desc, rec, heap = eng.run(runtime.KIND_MC, bd)
        return self._decode_mc(desc, rec, heap, slot_err, raise_errors)

    @staticmethod
    def _mc_frames(messages, msg_type="MC", version=None, raise_errors=False):
        """MC dicts -> (frames (raw_hex, clock, mcbitnum, messagetype, version), {row: exception},
        per message its protocol_id or None)."""
        frames, slot_err = [], {}
        for i, m in enumerate(messages):
            try:
                hx = m.get("raw_hex", m.get("data", m.get("D", "")))
                clk = m.get("clock", m.get("C", 0))
                L = m.get("mcbitnum", m.get("bit_length", m.get("L", 0)))
                mt = m.get("messagetype", msg_type if msg_type in ("MC", "Mc") else "MC")
                if not isinstance(hx, str):
                    raise packing.ContractError("MC frames must be str for the device path")
                frames.append((hx, int(clk), int(L), mt, m.get("version", version)))
            except Exception as e:
                if raise_errors:
                    raise
                slot_err[i] = e
                frames.append(("", 0, 0, "MC", None))
        return frames, slot_err, [m.get("protocol_id") for m in messages]

    @classmethod
    def _mc_frame_error(cls, msg, msg_type="MC") -> BaseException:
        err = cls._mc_frames([msg], msg_type)[1]
        return err.get(0, RuntimeError("host conversion of this MC frame raised on another rank only"))

    def _mc_only(self, only, eng):
        idx = {str(p): i for i, p in enumerate(self._bank.mc_pids)}
        sel_only = np.array([-1 if not o else idx.get(str(o), len(self._bank.mc_pids)) for o in only], np.int16)
        return eng.torch.from_numpy(sel_only).to(eng.dev)

    def _decode_mc(self, desc, rec, heap, slot_err, raise_errors):
        bk = self._bank
        hs = heap.tobytes().decode("latin-1")
        d_st, d_rk, d_rb, d_nr = (desc["status"].tolist(), desc["raise_kind"].tolist(), desc["rec_begin"].tolist(),
                                  desc["n_rec"].tolist())
        r_p, r_off, r_len = rec["proto"].tolist(), rec["payload_off"].tolist(), rec["payload_len"].tolist()
        out: List[Any] = []
        for i in range(len(d_st)):
            if i in slot_err:
                out.append(slot_err[i])
                continue
            st = d_st[i]
            if st == runtime.ST_RAISED:
                exc = (packing.ContractError("MC payload longer than 65535 bytes") if d_rk[i] ==
                       runtime.RAISE_CONTRACT else
                       runtime.RAISE_NAMES.get(d_rk[i], RuntimeError)("reference raises on this MC frame"))
                if raise_errors:
                    raise exc
                out.append(exc)
                continue
            if st != runtime.ST_OK:
                raise RuntimeError(f"device status {st} for frame {i}")
            res = []
            b = d_rb[i]
            for r in range(b, b + d_nr[i]):
                pid = bk.mc_pids[r_p[r]]
                o = r_off[r]
                res.append({"protocol_id": str(pid), "payload": hs[o: o + r_len[r]],
                            "meta": {"protocol_id": pid, "rssi": None, "freq_afc": None}})
            out.append(res)
        return out
