"""The reference's helper methods on ``SDProtocols`` as thin wrappers over the HIP unit entry.

RFD-FHEM/PySignalduino's ``SDProtocols`` mixes in, besides the demodulators, the functions its
own unit tests call directly (tests/test_postdemodulation.py, test_manchester_protocols.py,
test_helpers.py, test_helpers_mc2dmc_and_logging.py):

  postDemo_EM / _Revolt / _FS20 / _FHT80 / _FHT80TF / _WS2000 / _WS7035 / _WS7053 /
  _lengtnPrefix                              sd_protocols/postdemodulation.py:27-730
  mcBit2Funkbus / Sainlogic / AS / Hideki / Maverick / OSV1 / OSV2o3 / OSPIR / TFA / Grothe /
  SomfyRTS, mcRaw                            sd_protocols/manchester.py:207-795
  _convert_mc_hex_to_bits, _demodulate_mc_data  manchester.py:18-144
  mc2dmc, bin_str_2_hex_str, mcraw, hex_to_bin_str, dec_2_bin_ppari
                                             sd_protocols/helpers.py:6-122, 168-188

Every one of them runs on the GPU through ``sdx_units`` (include/sdx.h; csrc/sdx_units.hip), the
same device code the MU/MS/MC kernels use (pd_* of csrc/sdx_device.h, mc_method of
csrc/sdx_mc.h).  Each has a batched form (``postdemo_batch``, ``mc_method_batch``, ...) that
evaluates many inputs in one launch; the single-call methods are batches of one.  What stays on
the host is the reference's argument handling (``None`` checks, ``isinstance`` branches, the
property lookups that feed a method's record) and the rendering of the returned texts.

Inputs outside what the device models raise ``packing.ContractError`` instead of being guessed:
postDemo bit lists must hold the ints 0/1, MC bit strings '0'/'1' characters (at most 512),
pattern_exists takes finite numbers (at most 32 search values and 16 patterns).  There is no CPU
fallback.
"""
from __future__ import annotations

import math
from typing import Any, Dict, List, Optional, Sequence

import numpy as np

from . import bank as bankmod
from . import runtime
from .packing import ContractError

# (-1, msg) texts of the MC methods, indexed by McWhy (csrc/sdx_mc.h)
_NODUP_TAIL = ("", ", message is too short", ", message is too long", ", protocol does not exists")


def _mc_text(why: int, aux: int, name, bit_data: str, mcbitnum) -> str:
    if why == 1:
        return "message is too short"
    if why == 2:
        return "message is too long"
    if why == 3:
        return "wrong bits at begin"
    if why == 4:
        return "parity error"
    if why == 5:
        return "checksum error"
    if why == 6:
        return f"{name}: lib/mcBit2Sainlogic, start 010100 not found"
    if why == 7:
        return "sync not found"
    if why == 8:
        return f"loop error, please report this data {bit_data}"
    if why == 9:
        return f" no duplicate found{_NODUP_TAIL[aux]}"
    if why == 10:
        return f"message must be 32 bits, got {mcbitnum}"
    if why == 11:
        return f"message must be 56 bits, got {aux}"
    if why == 12:
        return "message is to long"
    raise RuntimeError(f"unknown MC method outcome {why}")


# the callable attributes of the reference's SDProtocols class (sd_protocols.py:13 and its mixins):
# what `hasattr(self, name) and callable(getattr(self, name))` finds there (manchester.py:114)
REF_CALLABLES = frozenset((
    "ConvBresser_5in1", "ConvBresser_6in1", "ConvBresser_7in1", "ConvBresser_lightning", "ConvKoppFreeControl",
    "ConvLaCrosse", "ConvPCA301", "_calc_crc16", "_calc_crc8_la_crosse", "_convert_mc_hex_to_bits",
    "_demodulate_mc_data", "_demodulate_mn_data", "_load_protocols", "_logging", "bin_str_2_hex_str",
    "check_property", "dec_2_bin_ppari", "decode_rsl", "demodulate", "demodulate_mc", "demodulate_mn",
    "demodulate_ms", "demodulate_mu", "encode_rsl", "get_keys", "get_property", "get_protocol_list",
    "hex_to_bin_str", "length_in_range", "lfsr_digest16", "mc2dmc", "mcBit2AS", "mcBit2Funkbus", "mcBit2Grothe",
    "mcBit2Hideki", "mcBit2Maverick", "mcBit2OSPIR", "mcBit2OSV1", "mcBit2OSV2o3", "mcBit2Sainlogic",
    "mcBit2SomfyRTS", "mcBit2TFA", "mcRaw", "mcraw", "postDemo_EM", "postDemo_FHT80", "postDemo_FHT80TF",
    "postDemo_FS20", "postDemo_Revolt", "postDemo_WS2000", "postDemo_WS7035", "postDemo_WS7053",
    "postDemo_lengtnPrefix", "protocol_exists", "register_log_callback", "set_defaults"))


def _ref_callable(name: str) -> bool:
    return name in REF_CALLABLES or callable(getattr(object, name, None))


_MC_NAMES = ("mcBit2Funkbus", "mcBit2Sainlogic", "mcBit2AS", "mcBit2Hideki", "mcBit2Maverick", "mcBit2OSV1",
             "mcBit2OSV2o3", "mcBit2OSPIR", "mcBit2TFA", "mcBit2Grothe", "mcBit2SomfyRTS")
_HEX_RISKY = set(" \t\n\r\x0b\x0c_xX+-")   # int(s, 16) syntax beyond plain digits: not modelled


def _is_int(v) -> bool:
    return isinstance(v, int) and not isinstance(v, bool)


def _bits_str(bit_data) -> bytes:
    if not isinstance(bit_data, str) or len(bit_data) > runtime.UNIT_MC_BITS or bit_data.strip("01"):
        raise ContractError("MC bit_data must be a str of at most "
                            f"{runtime.UNIT_MC_BITS} '0'/'1' characters for the device path")
    return bit_data.encode("ascii")


def _ascii(s: str, what: str) -> bytes:
    try:
        return s.encode("ascii")
    except UnicodeEncodeError:
        raise ContractError(f"{what}: non-ASCII text is not modelled on the device") from None


class UnitsMixin:
    """Mixed into ``SDProtocols``; needs ``self._protocols`` and ``self.device``."""

    # ------------------------------------------------------------------ plumbing ---------------
    def _units(self, op, ins, caps, **kw):
        return runtime.UnitRunner.get(self.device).run(op, ins, caps, **kw)

    @staticmethod
    def _payload(heap, r) -> bytes:
        o = int(r["payload_off"])
        return heap[o: o + int(r["payload_len"])].tobytes()

    # ------------------------------------------------------------------ postDemo_* -------------
    def postdemo_batch(self, method: str, arrays: Sequence[list], name: str = "") -> List[Any]:
        """``getattr(proto, method)(name, bits)`` for every bit list in one launch
        (postdemodulation.py:27-730): (1, list) / (0, None), or the exception the reference raises
        (returned in that slot)."""
        which = bankmod.POSTDEMO[method]
        ins = []
        for a in arrays:
            if not isinstance(a, list) or any(not _is_int(b) or b not in (0, 1) for b in a):
                raise ContractError(f"{method}: bit_msg_array must be a list of the ints 0/1 for the device path")
            if len(a) > 65000:
                raise ContractError(f"{method}: more than 65000 bits")
            ins.append(bytes(a))
        desc, rec, heap = self._units(runtime.UNIT_POSTDEMO, ins, [len(b) + 64 for b in ins],
                                      args=[which] * len(ins))
        out: List[Any] = []
        for d, r in zip(desc, rec):
            if d["status"] == runtime.ST_RAISED:
                out.append(ValueError("invalid literal for int() with base 2: ''"))
            elif int(r["proto"]) == 1:
                out.append((0, None))
            else:
                out.append((1, list(self._payload(heap, r))))
        return out

    def _postdemo1(self, method, name, bit_msg_array):
        r = self.postdemo_batch(method, [bit_msg_array], name)[0]
        if isinstance(r, BaseException):
            raise r
        return r

    def postDemo_EM(self, name, bit_msg_array):  # noqa: N802  postdemodulation.py:27
        return self._postdemo1("postDemo_EM", name, bit_msg_array)

    def postDemo_Revolt(self, name, bit_msg_array):  # noqa: N802  :90
        return self._postdemo1("postDemo_Revolt", name, bit_msg_array)

    def postDemo_FS20(self, name, bit_msg_array):  # noqa: N802  :139
        return self._postdemo1("postDemo_FS20", name, bit_msg_array)

    def postDemo_FHT80(self, name, bit_msg_array):  # noqa: N802  :245
        return self._postdemo1("postDemo_FHT80", name, bit_msg_array)

    def postDemo_FHT80TF(self, name, bit_msg_array):  # noqa: N802  :339
        return self._postdemo1("postDemo_FHT80TF", name, bit_msg_array)

    def postDemo_WS2000(self, name, bit_msg_array):  # noqa: N802  :425
        return self._postdemo1("postDemo_WS2000", name, bit_msg_array)

    def postDemo_WS7035(self, name, bit_msg_array):  # noqa: N802  :580
        return self._postdemo1("postDemo_WS7035", name, bit_msg_array)

    def postDemo_WS7053(self, name, bit_msg_array):  # noqa: N802  :642
        return self._postdemo1("postDemo_WS7053", name, bit_msg_array)

    def postDemo_lengtnPrefix(self, name, bit_msg_array):  # noqa: N802  :708
        return self._postdemo1("postDemo_lengtnPrefix", name, bit_msg_array)

    # ------------------------------------------------------------------ MC methods -------------
    def mc_method_batch(self, method: str, calls: Sequence[tuple]) -> List[Any]:
        """``getattr(proto, method)(name, bit_data, protocol_id, mcbitnum)`` for every
        (name, bit_data, protocol_id, mcbitnum) in one launch.  ``method`` is one of the mcBit2*
        names, ``mcRaw`` (manchester.py:588) or ``mcraw`` (helpers.py:90).  Each slot holds the
        reference's return tuple or the exception it raises."""
        if method not in bankmod.MC_METHODS:
            raise AttributeError(f"'SDProtocols' object has no attribute '{method}'")
        out: List[Any] = [None] * len(calls)
        ins, caps, args, recs, idx, ctx = [], [], [], [], [], []
        for i, c in enumerate(calls):
            name, bit_data, pid, mcbitnum = c
            if method == "mcraw":                                   # helpers.py:105-111
                if bit_data is None:
                    out[i] = (-1, "no bitData provided")
                    continue
                if pid is None:
                    out[i] = (-1, "no protocolId provided")
                    continue
            none_bits = bit_data is None
            if none_bits and method != "mcRaw" and mcbitnum is None:
                out[i] = TypeError("object of type 'NoneType' has no len()")
                continue
            if none_bits and method in ("mcBit2AS", "mcBit2TFA"):   # bit_data.find(...)
                out[i] = AttributeError("'NoneType' object has no attribute 'find'")
                continue
            if none_bits and method == "mcBit2SomfyRTS":            # len(bit_data) / bit_data[1:57]
                out[i] = TypeError("object of type 'NoneType' has no len()")
                continue
            b = b"" if none_bits else _bits_str(bit_data)
            if method == "mcRaw":                                   # int(mcbitnum) (manchester.py:607)
                try:
                    mb = int(mcbitnum)
                except Exception as e:
                    out[i] = e
                    continue
            elif mcbitnum is None:                                  # `mcbitnum = len(bit_data)`
                mb = len(bit_data)
            elif _is_int(mcbitnum):
                mb = mcbitnum
            else:
                raise ContractError(f"{method}: mcbitnum must be an int or None for the device path")
            if not -(1 << 31) < mb < (1 << 31):
                raise ContractError(f"{method}: mcbitnum outside int32")
            try:
                rec = bankmod.mc_record(self._protocols, pid, method)
            except NotImplementedError as e:
                raise ContractError(str(e)) from None
            ins.append(b)
            caps.append(2 * len(b) + 64)
            args.append(mb)
            recs.append(rec)
            idx.append(i)
            ctx.append((name, bit_data, mb))
        if idx:
            desc, rec, heap = self._units(runtime.UNIT_MC_METHOD, ins, caps, args=args,
                                          mcrecs=np.stack([np.asarray(r) for r in recs]).astype(bankmod.MC_REC))
            for j, i in enumerate(idx):
                d, r = desc[j], rec[j]
                if d["status"] == runtime.ST_RAISED:
                    out[i] = runtime.RAISE_NAMES[int(d["raise_kind"])](f"the reference raises in {method}")
                    continue
                why = int(r["proto"])
                name, bit_data, mb = ctx[j]
                if bit_data is None:   # only the length gates ran on the device (an empty string)
                    if method == "mcBit2Funkbus" and why not in (1, 2):
                        out[i] = AttributeError("'NoneType' object has no attribute 'replace'")
                        continue
                    if method == "mcBit2Sainlogic" and why != 2 and mb < 128:
                        out[i] = AttributeError("'NoneType' object has no attribute 'find'")
                        continue
                    if not why:
                        out[i] = (1, None)          # bin_str_2_hex_str(None)
                        continue
                if why:
                    out[i] = (-1, _mc_text(why, int(r["bit_length"]), name, bit_data, mb))
                    continue
                p = self._payload(heap, r).decode("ascii")
                if int(r["bit_length"]) == 2:                       # TFA: the list of duplicates
                    p = p[2:-2].split("', '")
                out[i] = (1, p)
        return out

    def _mc1(self, method, name, bit_data, protocol_id, mcbitnum):
        r = self.mc_method_batch(method, [(name, bit_data, protocol_id, mcbitnum)])[0]
        if isinstance(r, BaseException):
            raise r
        return r

    def mcBit2Funkbus(self, name, bit_data, protocol_id, mcbitnum=None):  # noqa: N802  manchester.py:207
        return self._mc1("mcBit2Funkbus", name, bit_data, protocol_id, mcbitnum)

    def mcBit2Sainlogic(self, name, bit_data, protocol_id, mcbitnum=None):  # noqa: N802  :302
        return self._mc1("mcBit2Sainlogic", name, bit_data, protocol_id, mcbitnum)

    def mcBit2AS(self, name, bit_data, protocol_id, mcbitnum=None):  # noqa: N802  :356
        return self._mc1("mcBit2AS", name, bit_data, protocol_id, mcbitnum)

    def mcBit2Hideki(self, name, bit_data, protocol_id, mcbitnum=None):  # noqa: N802  :418
        return self._mc1("mcBit2Hideki", name, bit_data, protocol_id, mcbitnum)

    def mcBit2Maverick(self, name, bit_data, protocol_id, mcbitnum=None):  # noqa: N802  :452
        return self._mc1("mcBit2Maverick", name, bit_data, protocol_id, mcbitnum)

    def mcBit2OSV1(self, name, bit_data, protocol_id, mcbitnum=None):  # noqa: N802  :486
        return self._mc1("mcBit2OSV1", name, bit_data, protocol_id, mcbitnum)

    def mcBit2OSV2o3(self, name, bit_data, protocol_id, mcbitnum=None):  # noqa: N802  :520
        return self._mc1("mcBit2OSV2o3", name, bit_data, protocol_id, mcbitnum)

    def mcBit2OSPIR(self, name, bit_data, protocol_id, mcbitnum=None):  # noqa: N802  :554
        return self._mc1("mcBit2OSPIR", name, bit_data, protocol_id, mcbitnum)

    def mcBit2TFA(self, name, bit_data, protocol_id, mcbitnum=None):  # noqa: N802  :615
        return self._mc1("mcBit2TFA", name, bit_data, protocol_id, mcbitnum)

    def mcBit2Grothe(self, name, bit_data, protocol_id, mcbitnum=None):  # noqa: N802  :721
        return self._mc1("mcBit2Grothe", name, bit_data, protocol_id, mcbitnum)

    def mcBit2SomfyRTS(self, name, bit_data, protocol_id, mcbitnum=None):  # noqa: N802  :756
        return self._mc1("mcBit2SomfyRTS", name, bit_data, protocol_id, mcbitnum)

    def mcRaw(self, name, bit_data, protocol_id, mcbitnum, other_arg=None):  # noqa: N802  :588
        return self._mc1("mcRaw", name, bit_data, protocol_id, mcbitnum)

    def mcraw(self, name="anonymous", bit_data=None, protocol_id=None, mcbitnum=None):  # helpers.py:90
        return self._mc1("mcraw", name, bit_data, protocol_id, mcbitnum)

    # ------------------------------------------------------------------ hex / bit helpers ------
    def hex_to_bin_batch(self, hexes: Sequence[str], invert: bool = False) -> List[Optional[str]]:
        """hex_to_bin_str (helpers.py:168-188) of every string in one launch; ``invert`` applies
        _convert_mc_hex_to_bits's polarity translate first (manchester.py:33-36)."""
        ins = []
        for h in hexes:
            if not isinstance(h, str):
                raise ContractError("hex_to_bin_str: only str input is modelled on the device")
            if any(c in _HEX_RISKY for c in h):
                raise ContractError("hex_to_bin_str: int(x, 16) syntax (whitespace, '_', '0x', sign) is not "
                                    "modelled on the device")
            b = _ascii(h, "hex_to_bin_str")
            if len(b) > 16000:
                raise ContractError("hex_to_bin_str: more than 16000 characters")
            ins.append(b)
        desc, rec, heap = self._units(runtime.UNIT_HEX2BIN, ins, [4 * len(b) + 8 for b in ins],
                                      args=[1 if invert else 0] * len(ins))
        return [None if int(r["proto"]) else self._payload(heap, r).decode("ascii") for r in rec]

    def hex_to_bin_str(self, hex_string):  # helpers.py:168
        if hex_string is None:
            return None
        return self.hex_to_bin_batch([hex_string])[0]

    def _convert_mc_hex_to_bits(self, name: str, raw_hex: str, polarity_invert: bool, hlen: int):  # manchester.py:18
        if polarity_invert and not isinstance(raw_hex, str):
            raise ContractError("_convert_mc_hex_to_bits: raw_hex must be a str")
        if raw_hex is None:
            return (1, None)
        bits = self.hex_to_bin_batch([raw_hex], invert=bool(polarity_invert))[0]
        return (1, bits)

    def bin_str_2_hex_batch(self, nums: Sequence[Any]) -> List[Optional[str]]:
        """bin_str_2_hex_str (helpers.py:28-64) of every input in one launch."""
        out: List[Optional[str]] = [None] * len(nums)
        ins, idx = [], []
        for i, num in enumerate(nums):
            if num is None:
                continue
            if not num:
                out[i] = ""
                continue
            if not isinstance(num, str):
                continue
            ins.append(num.encode("utf-8"))   # a non-ASCII character is never '0'/'1': None
            idx.append(i)
        if idx:
            desc, rec, heap = self._units(runtime.UNIT_BIN2HEX, ins, [len(b) // 4 + 8 for b in ins])
            for j, i in enumerate(idx):
                r = rec[j]
                out[i] = None if int(r["proto"]) else self._payload(heap, r).decode("ascii")
        return out

    def bin_str_2_hex_str(self, num):  # helpers.py:28
        return self.bin_str_2_hex_batch([num])[0]

    def mc2dmc_batch(self, bit_datas: Sequence[Any]) -> List[Any]:
        """mc2dmc (helpers.py:6-26) of every string in one launch."""
        out: List[Any] = [None] * len(bit_datas)
        ins, idx = [], []
        for i, s in enumerate(bit_datas):
            if s is None:
                out[i] = (-1, "no bitData provided")
                continue
            if not isinstance(s, str):
                raise ContractError("mc2dmc: only str input is modelled on the device")
            b = _ascii(s, "mc2dmc")
            if len(b) > 60000:
                raise ContractError("mc2dmc: more than 60000 characters")
            ins.append(b)
            idx.append(i)
        if idx:
            desc, rec, heap = self._units(runtime.UNIT_MC2DMC, ins, [len(b) + 8 for b in ins])
            for j, i in enumerate(idx):
                out[i] = self._payload(heap, rec[j]).decode("ascii")
        return out

    def mc2dmc(self, bit_data):  # helpers.py:6
        return self.mc2dmc_batch([bit_data])[0]

    @staticmethod
    def dec_2_bin_ppari(num):  # helpers.py:66-88 (8-bit format + parity: integer formatting, host)
        if num is None:
            return None
        nbin = format(num, "08b")
        parity = 0
        for bit in nbin:
            parity ^= int(bit)
        return nbin + str(parity)

    # ------------------------------------------------------------------ MC chain pieces --------
    def _demodulate_mc_data(self, name, protocol_id, clock, raw_hex, mcbitnum, messagetype, version):
        """manchester.py:49-144.  mc_mode 'strict': the reference's observable behaviour (its gates
        with the same Python operations; a clockrange protocol raises TypeError at :83-84, a
        method call raises TypeError at :120 except mcRaw's shifted-argument path, which this
        evaluates on the device).  mc_mode 'fixed': the intended chain on the device for this
        protocol (clockrange[0] < C < clockrange[1], the method called without the extra self)."""
        return self._mc_data_strict(name, protocol_id, clock, raw_hex, mcbitnum, messagetype, version,
                                    fixed=getattr(self, "mc_mode", "strict") == "fixed")

    def _mc_data_strict(self, name, protocol_id, clock, raw_hex, mcbitnum, messagetype, version, fixed=False):
        length_min = int(self.check_property(protocol_id, "length_min", -1))
        if mcbitnum < length_min:
            return (-1, "message is too short", {})
        length_max = int(self.check_property(protocol_id, "length_max", 9999))
        if mcbitnum > length_max:
            return (-1, "message is too long", {})
        clockrange = self.get_property(protocol_id, "clockrange")
        if clockrange and len(clockrange) >= 2:
            if fixed:
                lo, hi = clockrange[0], clockrange[1]
            else:
                lo, hi = clockrange, clockrange
            if not (clock > lo and clock < hi):   # strict: int > list raises TypeError, as the reference
                return (-1, "clock out of range", {})
        polarity_invert = self.check_property(protocol_id, "polarity", "") == "invert"
        if messagetype == "Mc" or (version and version[:6] == "V 3.2."):
            polarity_invert = polarity_invert ^ 1
        rcode, bit_data = self._convert_mc_hex_to_bits(name, raw_hex, polarity_invert, len(raw_hex))
        if rcode == -1:
            return (rcode, bit_data, {})
        method_name_full = self.get_property(protocol_id, "method")
        if not method_name_full:
            return [(-1, "Protocol method not defined", {})]
        method_name = method_name_full.split(".")[-1]
        if not _ref_callable(method_name):                   # hasattr(self, m) and callable (:114)
            return (-1, f"Unknown protocol method {method_name_full}", {})
        n = len(bit_data)                                   # len(None) raises TypeError (:120)
        if fixed:
            rcode, res = self._call_method_fixed(method_name, name, bit_data, protocol_id, n)
        else:
            rcode, res = self._call_method_strict(method_name, name, bit_data, protocol_id, n)
        if rcode == -1:
            res = res if res is not None else "Decoding failed"
            return (-1, res, {})
        preamble = self.check_property(protocol_id, "preamble", "")
        return (1, f"{preamble}{res}", {"protocol_id": protocol_id, "rssi": None, "freq_afc": None})

    def _call_method_fixed(self, method_name, name, bit_data, protocol_id, n):
        if method_name not in bankmod.MC_METHODS:   # any other method of the class: wrong arguments
            raise TypeError(f"{method_name}() called with the MC method arguments")
        return getattr(self, method_name)(name, bit_data, protocol_id, n)

    def _call_method_strict(self, method_name, name, bit_data, protocol_id, n):
        """``method_func(self, name, bit_data, protocol_id, len(bit_data))`` on a bound method
        (manchester.py:120): one positional argument too many for every method except mcRaw,
        whose arguments then shift by one (name=self, bit_data=name, protocol_id=bit_data,
        mcbitnum=protocol_id)."""
        if method_name != "mcRaw":
            raise TypeError(f"{method_name}() takes at most 5 positional arguments but 6 were given")
        # mcRaw(self, self_obj, name, bit_data, protocol_id, n): length_max looked up under the
        # bit string, int(protocol_id) as mcbitnum, bin_str_2_hex_str(name)
        length_max = int(self.check_property(bit_data, "length_max", 0))
        if int(protocol_id) > length_max:
            return (-1, "message is too long")
        return (1, self.bin_str_2_hex_str(name))
