"""Protocol-bank compiler: protocols.json -> one device-ready blob (include/sdx_bank.h).

Mirrors how the reference consumes the bank (sd_protocols/sd_protocols.py:25-58,
157-160; message_unsynced.py; message_synced.py; manchester.py) and resolves,
ONCE per bank, every property lookup and string/number conversion those files
repeat per message: float(clockabs), the search lists with their unique values
and tolerances, int(length_min/max), paddingbits, postDemodulation method
resolution (``hasattr`` on the reference class -- a missing method is skipped,
message_unsynced.py:233-234), preamble/postamble f-string formatting and the
modulematch regexes (compiled to DFAs by regex_dfa.py).

Anything in a (user-modified) bank whose reference behaviour is not modelled
on the device raises ``NotImplementedError`` here, at bank-compile time.
"""
from __future__ import annotations

import copy
import json
import os
import math
import struct
from typing import Any, Dict, List, Optional, Tuple

import numpy as np

from . import regex_dfa

DEFAULT_BANK = os.path.join(os.path.dirname(os.path.abspath(__file__)), "data", "sd_bank.json")

MAXSEARCH, MAXUNIQ = 16, 4
MAGIC, VERSION = 0x4B4E4253, 17
INT_NONE = 2147483647  # "no length_max" sentinel

PATSPEC = np.dtype([("klo", "<i4", (MAXUNIQ,)), ("khi", "<i4", (MAXUNIQ,)), ("rk_off", "<u4", (MAXUNIQ,)),
                    ("len", "u1"), ("nuniq", "u1"), ("pad", "u1", (6,)), ("uidx_pk", "<u8"),
                    ("uval", "<f8", (MAXUNIQ,)), ("utol", "<f8", (MAXUNIQ,)), ("uidx", "u1", (MAXSEARCH,))], align=True)
MU_REC = np.dtype([("clock", "<f8"), ("has_start", "u1"), ("recon", "u1"), ("dispatch_bin", "u1"),
                   ("remove_zero", "u1"), ("active", "u1"), ("never", "u1"), ("res0", "u1"), ("res1", "u1"),
                   ("start", PATSPEC), ("one", PATSPEC), ("zero", PATSPEC), ("flt", PATSPEC),
                   ("proto_index", "<i4"), ("length_min", "<i4"), ("length_max", "<i4"), ("width", "<i4"),
                   ("pad_bits", "<i4"), ("postdemo", "<i4"), ("mm_dfa", "<i4"), ("mm_pre_state", "<i4"), ("pre_off", "<i4"),
                   ("pre_len", "<i4"), ("post_off", "<i4"), ("post_len", "<i4"), ("res2", "<i4")], align=True)
MS_REC = np.dtype([("pclock", "<f8"), ("key", PATSPEC, (4,)), ("proto_index", "<i4"), ("width", "<i4"),
                   ("lmin_sync", "<i4"), ("lir_min", "<i4"), ("lir_max", "<i4"), ("pad_bits", "<i4"),
                   ("postdemo", "<i4"), ("pre_off", "<i4"), ("pre_len", "<i4"), ("post_off", "<i4"),
                   ("post_len", "<i4"), ("recon", "u1"), ("never", "u1"), ("res", "u1", (2,))], align=True)
MC_REC = np.dtype([("cr_lo", "<f8"), ("cr_hi", "<f8"), ("proto_index", "<i4"), ("method", "<i4"), ("lmin", "<i4"),
                   ("lmax", "<i4"), ("pre_off", "<i4"), ("pre_len", "<i4"), ("pid_num", "<i4"),
                   ("has_lmin", "u1"), ("has_lmax", "u1"), ("lmax_is_str", "u1"), ("invert", "u1"),
                   ("has_cr", "u1"), ("lir_noexist", "u1"), ("res", "u1", (2,))], align=True)
DFA_REC = np.dtype([("nstates", "<i4"), ("start", "<i4"), ("trans_off", "<i4"), ("flags_off", "<i4"),
                    ("t256_off", "<i4"), ("res", "<i4", (3,))])
MN_REC = np.dtype([("proto_index", "<i4"), ("lir_min", "<i4"), ("lir_max", "<i4"), ("dfa", "<i4"), ("method", "<i4"),
                   ("pre_off", "<i4"), ("pre_len", "<i4"), ("dfa_slot", "<i4")])
JSON_REC = np.dtype([("pid_off", "<u4"), ("s1_off", "<u4"), ("s2_off", "<u4"), ("pid_len", "<u2"), ("s1_len", "<u2"),
                     ("s2_len", "<u2"), ("res", "<u2")])
def mn_tables() -> bytes:
    """Byte/nibble tables of the MN checksums (k_mn stages them in LDS): CRC-16 poly 0x1021 and
    0x8005 and CRC-8 poly 0x31 (MSB first, init 0: helpers.py:281-309, 630-673), and the
    LFSR-16 digests of ConvBresser_lightning / _7in1 (helpers.py:190-221, gen 0x8810 from keys
    0xABF9 / 0xBA95 over 8 / 21 bytes) as per-nibble XOR tables: the key sequence does not depend
    on the data, so byte k's contribution is the XOR of the keys at its set bits.
    Layout (include/sdx_bank.h SDX_MNTAB_*): u16 crc1021[256] | u16 crc8005[256] | u8 crc31[256] |
    u16 lfsr8[16 nibbles][16] | u16 lfsr21[42 nibbles][16]."""
    def crc16_entry(t, poly):
        c = t << 8
        for _ in range(8):
            c = ((c << 1) ^ poly) & 0xFFFF if c & 0x8000 else (c << 1) & 0xFFFF
        return c

    def crc8_entry(t):
        c = t
        for _ in range(8):
            c = ((c << 1) ^ 0x31) & 0xFF if c & 0x80 else (c << 1) & 0xFF
        return c

    def lfsr_nibbles(key, nbytes):
        keys = []
        for _ in range(8 * nbytes):
            keys.append(key)
            key = (key >> 1) ^ 0x8810 if key & 1 else key >> 1
        tab = np.zeros((2 * nbytes, 16), np.uint16)
        for k in range(nbytes):
            for v in range(16):
                hi = lo = 0
                for i in range(4):            # bit i of the nibble; the byte's bit 7 is step 8k
                    if (v >> i) & 1:
                        hi ^= keys[8 * k + (3 - i)]
                        lo ^= keys[8 * k + 4 + (3 - i)]
                tab[2 * k][v], tab[2 * k + 1][v] = hi, lo
        return tab

    parts = [np.array([crc16_entry(t, 0x1021) for t in range(256)], np.uint16).tobytes(),
             np.array([crc16_entry(t, 0x8005) for t in range(256)], np.uint16).tobytes(),
             np.array([crc8_entry(t) for t in range(256)], np.uint8).tobytes(),
             lfsr_nibbles(0xABF9, 8).tobytes(), lfsr_nibbles(0xBA95, 21).tobytes()]
    return b"".join(parts)


FSPEC = np.dtype([("lohi", "<u4", (3,)), ("rk01", "<u4"), ("rk2_len_nu", "<u4"), ("upk", "<u4")])
MU_FILT = np.dtype([("clock", "<f8"), ("start_upk", "<u8"), ("flags", "<u4"), ("spec", FSPEC, (4,)),
                    ("clk_c", "<u4"), ("clk_m", "<u4"), ("clk_sh", "<u4")])
MS_FILT = np.dtype([("pclock", "<f8"), ("sync_upk", "<u8"), ("flags", "<u4"), ("width", "<i4"), ("lmin_sync", "<i4"),
                    ("spec", FSPEC, (4,)), ("res", "<u4")])
HDR_FMT = "<" + "I" * 31  # sdx_bank_hdr: 31 uint32
# MU decode descriptor (sdx_mu_desc): what the compacted decode reads per (message, protocol) pair,
# staged in LDS once per tile
MU_DESC = np.dtype([("pre", "u1", (16,)), ("post", "u1", (2,)), ("pre_len", "u1"), ("post_len", "u1"),
                    ("width", "u1"), ("len_s", "u1"), ("recon", "u1"), ("dispatch_bin", "u1"),
                    ("remove_zero", "u1"), ("postdemo", "u1"), ("pad_bits", "u1"), ("mm_on", "u1"),
                    ("lmin", "<u2"), ("lmax", "<u2"), ("mm_base", "<u2"), ("mm_post", "<u2"),
                    ("pre_state", "u1"), ("res", "u1", (3,))])
MUDESC_LDS = 160      # SDX_MUDESC_LDS: descriptors held in LDS (the rest are read from the blob)
MMTAB_LDS = 10240     # SDX_MMTAB_LDS: bytes of modulematch tables held in LDS
MM_FAST_DIGITS = 64   # hex digits of a payload on the device's fast path (64 * NW / 4, NW = 4)

POSTDEMO = {"postDemo_EM": 1, "postDemo_Revolt": 2, "postDemo_FS20": 3, "postDemo_FHT80": 4,
            "postDemo_FHT80TF": 5, "postDemo_WS2000": 6, "postDemo_WS7035": 7, "postDemo_WS7053": 8,
            "postDemo_lengtnPrefix": 9}
# every method name the reference SDProtocols class defines that a bank may reference for MC
MC_METHODS = {"mcBit2Funkbus": 1, "mcBit2Sainlogic": 2, "mcBit2AS": 3, "mcBit2Hideki": 4, "mcBit2Maverick": 4,
              "mcBit2OSV1": 4, "mcBit2OSV2o3": 4, "mcBit2OSPIR": 4, "mcRaw": 5, "mcraw": 6, "mcBit2TFA": 7,
              "mcBit2Grothe": 8, "mcBit2SomfyRTS": 9}
# MN methods (sd_protocols/helpers.py:223-716) -> enum sdx_mn_method; MN_MISSING: not on the class
MN_METHODS = {"ConvBresser_lightning": 1, "ConvBresser_5in1": 2, "ConvBresser_6in1": 3, "ConvBresser_7in1": 4,
              "ConvPCA301": 5, "ConvKoppFreeControl": 6, "ConvLaCrosse": 7}
MN_MISSING = 255
MN_MAX = 64
# other methods the reference SDProtocols class defines: an MN protocol naming one of them would call
# it with the wrong arguments (not modelled)
_OTHER_METHODS = set(MC_METHODS) | set(POSTDEMO) | {"demodulate", "demodulate_mn", "demodulate_mc", "demodulate_mu",
                                                    "demodulate_ms", "lfsr_digest16", "length_in_range",
                                                    "mc2dmc", "bin_str_2_hex_str", "hex_to_bin_str"}


def load_protocols(path: Optional[str] = None) -> Dict[str, dict]:
    """sd_protocols.py:30-41 (``data.get('protocols', {})``)."""
    with open(path or DEFAULT_BANK, "r", encoding="utf-8") as f:
        data = json.load(f)
    return data.get("protocols", {})


def set_defaults(protocols: Dict[str, dict]) -> None:
    """sd_protocols.py:157-160."""
    for pid, proto in protocols.items():
        proto.setdefault("active", True)
        proto.setdefault("name", f"Protocol_{pid}")


def _tolerance(v: float) -> float:
    """pattern_utils.py:15-26 (evaluated once per bank value, same fp64 ops)."""
    a = abs(v)
    if a > 3:
        if a > 16:
            return a * 0.18
        return a * 0.3
    return 1.0


def _int_exact(v, what) -> int:
    """int(v) for the bank's numeric strings / ints; refuse anything else (not modelled)."""
    if isinstance(v, bool) or not isinstance(v, (int, str)):
        raise NotImplementedError(f"{what}: unsupported value {v!r}")
    if isinstance(v, str) and not v.strip().lstrip("+-").isdigit():
        raise NotImplementedError(f"{what}: non-integer string {v!r}")
    return int(v)


def mc_record(P: Dict[str, dict], pid, method: str, rec=None):
    """The sdx_mc_proto of one (protocol id, MC method) pair, with the property lookups the
    reference's methods make (manchester.py:207-795, helpers.py:90-166): ``P.get(pid, {})`` with
    whatever object ``pid`` is (an int id finds no properties, as check_property does),
    length_in_range's ``protocol_exists(str(pid))``, and ``int(pid)`` for the Funkbus id test.
    Used for the bank's clockrange protocols and for the unit entry's per-call records."""
    if rec is None:
        rec = np.zeros((), MC_REC)
    try:
        p = P.get(pid, {})
    except TypeError:
        raise NotImplementedError(f"MC protocol id {pid!r}: unhashable") from None
    if not isinstance(p, dict):
        raise NotImplementedError(f"MC protocol id {pid!r}: properties are not a dict")
    rec["method"] = MC_METHODS[method]
    cr = p.get("clockrange")
    if isinstance(cr, list) and len(cr) >= 2:
        rec["has_cr"] = 1
        rec["cr_lo"], rec["cr_hi"] = float(cr[0]), float(cr[1])
    if "length_min" in p:
        rec["has_lmin"] = 1
        rec["lmin"] = _int32(_int_exact(p["length_min"], f"MC {pid} length_min"))
    if "length_max" in p and p["length_max"] is not None:
        rec["has_lmax"] = 1
        rec["lmax"] = _int32(_int_exact(p["length_max"], f"MC {pid} length_max"))
        rec["lmax_is_str"] = 1 if isinstance(p["length_max"], str) else 0
    rec["invert"] = 1 if p.get("polarity", "") == "invert" else 0
    rec["lir_noexist"] = 0 if str(pid) in P else 1
    if isinstance(pid, str):
        try:
            rec["pid_num"] = _int32(int(pid))
        except ValueError:
            rec["pid_num"] = PID_NOT_INT
    elif isinstance(pid, int) and not isinstance(pid, bool):
        rec["pid_num"] = _int32(pid)
    else:   # the Funkbus test compares the object itself with 119
        rec["pid_num"] = 119 if pid == 119 else -1
    return rec


def _int32(v: int) -> int:
    if not -(1 << 31) < v < (1 << 31):
        raise NotImplementedError(f"value {v} outside int32")
    return v


PID_NOT_INT = -(1 << 31)   # SDX_PID_NOT_INT


def clock_divider(clock: float):
    """(c, m, sh | flags) of sdx_mu_filt: the integer normalisation k = round(10*|P| / c) the MU
    filter uses for integral pattern values.  floor(x / c) == (x * m) >> sh for all 0 <= x < 2^30
    with m = ceil(2^(30+L) / c), L = ceil(log2 c) (Granlund-Montgomery, N = 30: m*c - 2^(30+L) <
    c <= 2^L); valid only for an integral clock with 1 <= |clock| < 2^20."""
    if not (math.isfinite(clock) and clock == math.floor(clock) and 1 <= abs(clock) < (1 << 20)):
        return 0, 0, 0
    c = int(abs(clock))
    L = (c - 1).bit_length()
    sh = 30 + L
    m = -(-(1 << sh) // c)
    assert m < (1 << 32) and m * c - (1 << sh) < (1 << L)
    return c, m, sh | (1 << 8) | ((1 << 9) if clock < 0 else 0)


K_LIMIT = 1 << 28  # |k| bound of every interval (the device's k sentinel lies beyond it)


def _k_interval(v: float, tol: float):
    """The exact integer set {k : g <= 0.001 or g <= tol, g = abs(k/10 - v)} as [klo, khi].

    A message pattern normalises to ``round(x / clock, 1) == k / 10`` (round's result is the
    correctly rounded quotient k/10.0), so pattern_utils.py:53-61's candidate test is a predicate
    on the integer k.  k/10, the subtraction and abs are monotone in fp64, hence the accepted
    set is an interval; it is found here with the same fp64 operations and checked to be
    contiguous.
    """
    def ok(k: int) -> bool:
        g = abs(k / 10 - v)
        return g <= 0.001 or g <= tol
    lo = math.floor(10 * (v - tol)) - 4
    hi = math.ceil(10 * (v + tol)) + 4
    acc = [k for k in range(lo, hi + 1) if ok(k)]
    if not acc or ok(lo) or ok(hi) or acc != list(range(acc[0], acc[-1] + 1)):
        raise NotImplementedError(f"pattern value {v!r}: candidate set is not a bounded interval")
    if max(abs(acc[0]), abs(acc[-1])) >= K_LIMIT:
        raise NotImplementedError(f"pattern value {v!r}: too large")
    return acc[0], acc[-1]


def _gap_ranks(v: float, klo: int, khi: int) -> List[int]:
    """Rank of each k in [klo, khi] by its fp64 gap abs(k/10 - v) (pattern_utils.py:61-63 sorts the
    candidates by that gap, stably): equal gaps share a rank, so the device orders candidates by
    (rank, dict position) exactly as list.sort does."""
    gaps = [abs(k / 10 - v) for k in range(klo, khi + 1)]
    order = {g: i for i, g in enumerate(sorted(set(gaps)))}
    return [order[g] for g in gaps]


# Per-protocol work of the MU protocol loop in thousands of wave-cycles per 64-message tile on the
# bench corpus (tools/prof_phases.py, r03; group cost minus one normalisation, split evenly over the
# group's protocols), and the normalisation's cost per group: the work-list order of Bank (LPT).
MU_NORM_KCYC = 3.8
MU_SPLIT_KCYC = 60.0
MU_COST_KCYC = {
    "15": 19.3, "121": 18.1, "34": 16.2, "120": 14.6, "9": 14.6, "111": 14.6, "118.1": 11.9, "118": 11.9,
    "8": 11.7, "39": 11.1, "1": 11.1, "86": 11.0, "14": 11.0, "25": 11.0, "13": 10.9, "63": 10.9, "13.1": 10.9,
    "130": 10.4, "33.2": 10.4, "91": 10.4, "74": 10.4, "88": 10.4, "87": 10.4, "21": 10.4, "82": 10.4,
    "70": 10.4, "61": 10.4, "80": 10.4, "74.1": 10.4, "91.1": 10.4, "73": 10.4, "40": 10.2, "72": 9.9,
    "72.1": 9.9, "135": 9.8, "27": 9.8, "71": 9.4, "20": 8.6, "20.1": 8.6, "64": 8.4, "55": 7.7, "19": 7.7,
    "7.1": 7.7, "90": 7.6, "16": 7.6, "35": 7.6, "54": 7.5, "77": 7.5, "78": 7.5, "85": 7.5, "54.1": 7.5,
    "89": 7.5, "38": 7.5, "97": 7.5, "113": 7.5, "37": 7.5, "48": 7.5, "92": 7.2, "75": 7.1, "41": 7.1,
    "106": 7.1, "33": 7.1, "5": 7.1, "44.1": 7.1, "51": 7.1, "2": 7.1, "42": 7.1, "50": 7.1, "44": 7.1,
    "81": 7.1, "98": 7.1, "36": 7.1, "76": 7.1, "99": 7.1, "104": 7.1, "93": 6.8, "31": 6.8, "127": 6.7,
    "127.1": 6.7, "45": 6.5, "110": 6.1, "128": 5.9, "128.1": 5.9, "68": 5.9, "84": 5.9, "53": 5.7, "28": 5.7,
    "49.2": 5.6, "49": 5.6, "6": 5.5, "7": 5.4, "95": 5.4, "26": 5.4, "122": 5.4, "56": 5.1, "23": 5.1,
    "114": 5.1, "22": 5.1, "65": 4.9, "17.1": 4.9, "59": 4.9, "13.2": 4.7, "30": 4.6, "105": 4.6, "132": 4.6,
    "79": 4.6, "33.1": 4.6, "67": 4.2, "66": 4.2, "60": 4.2, "83": 4.2, "46": 4.1, "94": 4.1, "29": 4.1,
    "0.5": 4.0, "69": 3.8, "0.4": 3.8, "49.1": 3.7, "32": 3.3, "62": 3.0, "0.2": 2.7, "0.1": 2.7, "3": 2.7,
    "4": 2.7, "3.1": 2.7, "17": 2.7, "0.3": 2.7, "0": 2.7, "24": 1.9
}
# the same, re-measured with one protocol per work item after the round-3 kernel changes
# (SDX_MU_SPLIT=0.001 SDX_PROF build, profiles/r03/s2/phases_per_protocol.log; minus MU_NORM_KCYC)
MU_COST_KCYC_R3 = {
    "111": 30.2, "1": 23.7, "63": 23.0, "34": 22.2, "118.1": 21.7, "15": 21.5, "74": 19.6, "88": 18.6,
    "25": 17.9, "42": 17.7, "87": 17.4, "121": 17.1, "82": 16.7, "72.1": 16.3, "8": 15.8, "70": 14.9,
    "2": 14.7, "61": 14.4, "9": 14.3, "80": 14.2, "74.1": 14.1, "91.1": 13.9, "120": 13.8, "130": 12.8,
    "73": 12.5, "19": 12.4, "13": 12.3, "27": 12.2, "20": 12.2, "71": 11.9, "90": 11.2, "39": 10.7,
    "40": 10.3, "35": 10.2, "14": 10.0, "55": 9.7, "91": 9.5, "33.2": 9.3, "118": 9.2, "54": 8.9, "85": 8.9,
    "38": 8.7, "64": 8.6, "89": 8.4, "54.1": 8.3, "75": 8.3, "20.1": 8.3, "99": 8.3, "72": 8.2, "41": 8.1,
    "13.1": 8.1, "86": 8.0, "76": 7.9, "5": 7.8, "7.1": 7.7, "104": 7.5, "92": 7.4, "16": 7.3, "37": 7.3,
    "45": 7.3, "22": 7.2, "23": 7.1, "127.1": 7.1, "135": 7.1, "128.1": 7.0, "50": 7.0, "49": 6.6, "93": 6.4,
    "122": 6.3, "106": 6.3, "114": 6.3, "56": 6.2, "113": 6.2, "33": 6.1, "31": 6.1, "26": 6.1, "44.1": 6.0,
    "53": 6.0, "28": 5.4, "21": 5.3, "51": 5.1, "84": 5.0, "68": 4.9, "110": 4.8, "60": 4.8, "95": 4.7,
    "6": 4.4, "7": 4.4, "83": 4.2, "132": 4.0, "127": 3.9, "17.1": 3.9, "81": 3.7, "13.2": 3.7, "33.1": 3.7,
    "78": 3.6, "48": 3.6, "77": 3.4, "79": 3.4, "46": 3.2, "65": 3.1, "49.1": 3.0, "0.5": 3.0, "29": 2.9,
    "30": 2.9, "98": 2.9, "49.2": 2.7, "0.4": 2.7, "69": 2.7, "128": 2.4, "32": 2.3, "105": 2.3, "44": 2.3,
    "94": 2.3, "36": 2.1, "59": 2.1, "97": 2.0, "62": 2.0, "66": 1.9, "67": 1.7, "0.2": 1.5, "0.1": 1.4,
    "3": 1.4, "4": 1.3, "3.1": 1.2, "17": 1.1, "0.3": 0.9, "0": 0.5
}


# MS per-protocol cost of the filter loop in k_pulses<MS> (kcyc per tile and grab, tools/prof_phases.py
# on the bench corpus, profiles/r03/s2/phases_split.log): the processing order is descending cost
# (LPT), so the 8 waves of a tile end their protocol loops closer together
MS_COST_KCYC = {
    "54.1": 16.7, "1": 14.9, "4": 14.6, "17": 13.4, "13.2": 13.0, "88": 12.9, "15": 12.8, "13": 12.4,
    "53": 12.0, "0.1": 11.6, "128.1": 11.5, "87": 11.2, "33.2": 10.2, "7.1": 10.2, "41": 10.2, "3": 10.1,
    "49": 10.0, "0": 9.9, "0.2": 9.8, "51": 9.7, "33": 9.6, "2": 9.4, "106": 9.4, "25": 9.3, "0.4": 9.3,
    "33.1": 9.0, "6": 8.9, "93": 8.8, "3.1": 8.7, "0.3": 8.4, "100": 8.4, "65": 8.3, "23": 8.2, "112": 7.4,
    "123": 7.4, "74.1": 7.3, "134": 7.1, "125": 7.1, "68": 7.1, "109": 7.1, "91.1": 7.0, "103": 7.0,
    "14": 6.9, "107": 6.8, "0.5": 6.6, "35": 6.6, "127.1": 6.5, "116": 6.4, "131": 6.4, "113": 6.0,
    "116.1": 6.0, "72.1": 6.0, "107.1": 6.0, "126": 5.7, "20": 5.5, "7": 5.3, "55": 5.1, "130": 5.1,
    "118.1": 5.0, "90": 4.8, "117": 3.3, "101": 3.2, "108": 3.0, "133": 2.8, "115": 2.8, "102": 2.8
}


class Bank:
    """A compiled bank: the device blob plus host-side metadata for result building."""

    def __init__(self, protocols: Optional[Dict[str, dict]] = None, path: Optional[str] = None):
        raw = protocols if protocols is not None else load_protocols(path)
        self.protocols: Dict[str, dict] = copy.deepcopy(raw)
        set_defaults(self.protocols)
        self.pids: List[str] = list(self.protocols.keys())
        self.compile()

    def affixes(self, kind: int) -> List[Tuple[bytes, bytes]]:
        """Cached per compile (see _affixes)."""
        c = self.__dict__.setdefault("_affix_cache", {})
        if kind not in c:
            c[kind] = self._affixes(kind)
        return c[kind]

    def _affixes(self, kind: int) -> List[Tuple[bytes, bytes]]:
        """Per record of a class table (kind 0 MU, 1 MS, 2 MC, 3 MN): the (preamble, postamble) bytes
        its payloads carry -- the affixes of the exchange's nibble form (include/sdx.h, wire v3), the
        same strings the compiler puts in the records' pre_off/post_off (message_unsynced.py:271-274,
        message_synced.py:228-229, manchester.py:131-132, parser/mn.py:176-177)."""
        P = self.protocols
        enc = lambda v: f"{v}".encode("latin-1")  # noqa: E731
        if kind in (0, 1):
            pids = self.mu_pids if kind == 0 else self.ms_pids
            return [(enc(P[p].get("preamble", "")), enc(P[p].get("postamble", ""))) for p in pids]
        if kind == 2:
            return [(enc(x), b"") for x in self.mc_preamble]
        if kind == 3:
            return [(enc(x), b"") for x in self.mn_preamble]
        return []

    # -- helpers -------------------------------------------------------------------------------
    def _str(self, s: str):
        b = s.encode("latin-1")
        off = len(self._heap)
        self._heap += b
        return off, len(b)

    def _patspec(self, rec, search: List[float], what: str):
        if len(search) > MAXSEARCH:
            raise NotImplementedError(f"{what}: search list longer than {MAXSEARCH}")
        uniq: List[float] = []
        for v in search:
            if v not in uniq:
                uniq.append(v)
        if len(uniq) > MAXUNIQ:
            raise NotImplementedError(f"{what}: more than {MAXUNIQ} distinct values")
        rec["len"] = len(search)
        rec["nuniq"] = len(uniq)
        for i, v in enumerate(uniq):
            rec["uval"][i] = v
            t = _tolerance(v)
            if not t >= 0.001:
                raise NotImplementedError(f"{what}: tolerance below 0.001")
            rec["utol"][i] = t
            klo, khi = _k_interval(v, t)
            rec["klo"][i], rec["khi"][i] = klo, khi
            key = (v, t)
            if key not in self._rank_off:
                self._rank_off[key] = len(self._ranks)
                self._ranks.extend(_gap_ranks(v, klo, khi))
            rec["rk_off"][i] = self._rank_off[key]
        pk = 0
        for i, v in enumerate(search):
            rec["uidx"][i] = uniq.index(v)
            pk |= uniq.index(v) << (4 * i)
        rec["uidx_pk"] = pk

    @staticmethod
    def _float_list(spec):
        """[float(x) for x in spec] -- None when the reference's conversion raises."""
        try:
            return [float(x) for x in spec]
        except (ValueError, TypeError):
            return None

    def _postdemo(self, props) -> int:
        name = props.get("postDemodulation", None)
        if not name:
            return 0
        if not isinstance(name, str):
            raise NotImplementedError("postDemodulation: non-string")
        return POSTDEMO.get(name.split(".")[-1], 0)  # missing method -> silently skipped

    # -- compile -------------------------------------------------------------------------------
    def compile(self) -> None:
        P = self.protocols
        self._affix_cache = {}
        self._heap = bytearray()
        self._ranks: List[int] = []                 # u16 gap-rank tables (sdx_patspec.rk_off)
        self._rank_off: Dict[Any, int] = {}
        self.mu_pids = [pid for pid, p in P.items() if "clockabs" in p]
        self.ms_pids = [pid for pid, p in P.items() if "sync" in p]
        self.mc_pids = [pid for pid, p in P.items() if "clockrange" in p]
        mm_patterns: List[str] = []

        mu = np.zeros(len(self.mu_pids), MU_REC)
        self.mu_clock: List[float] = []
        for r, pid in enumerate(self.mu_pids):
            p = P[pid]
            rec = mu[r]
            rec["proto_index"] = self.pids.index(pid)
            ca = p.get("clockabs", 1)
            try:
                clock = float(ca)
            except (ValueError, TypeError):
                raise NotImplementedError(f"MU {pid}: clockabs {ca!r} not numeric")
            if clock == 0:
                raise NotImplementedError(f"MU {pid}: clockabs 0 (ZeroDivisionError path not modelled)")
            rec["clock"] = clock
            self.mu_clock.append(clock)
            rec["active"] = 1 if p.get("active", True) else 0
            sp = p.get("start")
            if sp and isinstance(sp, list):
                fl = self._float_list(sp)
                if fl is None:
                    raise NotImplementedError(f"MU {pid}: non-numeric start raises ValueError (not modelled)")
                rec["has_start"] = 1
                self._patspec(rec["start"], fl, f"MU {pid} start")
            never = False
            nkeys = 0
            for key, field in (("one", "one"), ("zero", "zero"), ("float", "flt")):
                spec = p.get(key)
                if not spec:
                    continue
                fl = self._float_list(spec)
                if fl is None:
                    never = True   # match_failed -> protocol skipped (message_unsynced.py:105-109)
                    break
                if not fl:
                    never = True
                    break
                self._patspec(rec[field], fl, f"MU {pid} {key}")
                nkeys += 1
            lens = {int(rec[f]["len"]) for f in ("one", "zero", "flt") if rec[f]["len"]}
            if len(lens) > 1:
                raise NotImplementedError(f"MU {pid}: one/zero/float of different lengths")
            rec["never"] = 1 if (never or nkeys == 0 or not p.get("one")) else 0
            rec["length_min"] = _int_exact(p.get("length_min", 0), f"MU {pid} length_min")
            lm = p.get("length_max", None)
            rec["length_max"] = _int_exact(lm, f"MU {pid} length_max") if lm else INT_NONE
            one = p.get("one")
            rec["width"] = len(one) if one else 0
            if one and lens and rec["width"] != next(iter(lens)):
                raise NotImplementedError(f"MU {pid}: len(one) differs from unit length")
            if not rec["has_start"] and rec["length_min"] == 0 and not rec["never"]:
                raise NotImplementedError(f"MU {pid}: no start and length_min 0 (empty matches) not modelled")
            if rec["width"] not in (0, 1, 2, 4):
                raise NotImplementedError(f"MU {pid}: unit width {int(rec['width'])} not in (1, 2, 4)")
            rec["recon"] = 1 if p.get("reconstructBit") else 0
            rec["dispatch_bin"] = 1 if _int_exact(p.get("dispatchBin", 0), "dispatchBin") == 1 else 0
            pad = _int_exact(p.get("paddingbits", 4), f"MU {pid} paddingbits")
            if pad < 1:
                raise NotImplementedError(f"MU {pid}: paddingbits < 1")
            rec["pad_bits"] = pad
            rec["remove_zero"] = 1 if p.get("remove_zero", 0) else 0
            rec["postdemo"] = self._postdemo(p)
            rec["pre_off"], rec["pre_len"] = self._str(f"{p.get('preamble', '')}")
            rec["post_off"], rec["post_len"] = self._str(f"{p.get('postamble', '')}")
            mm = p.get("modulematch")
            if mm:
                if mm not in mm_patterns:
                    mm_patterns.append(mm)
                rec["mm_dfa"] = mm_patterns.index(mm)
            else:
                rec["mm_dfa"] = -1

        ms = np.zeros(len(self.ms_pids), MS_REC)
        for r, pid in enumerate(self.ms_pids):
            p = P[pid]
            rec = ms[r]
            rec["proto_index"] = self.pids.index(pid)
            try:
                rec["pclock"] = float(p.get("clockabs", 0))
            except (ValueError, TypeError):
                raise NotImplementedError(f"MS {pid}: clockabs not numeric (raises in reference)")
            one = p.get("one")
            width = len(one) if one else 0
            rec["width"] = width
            if width not in (0, 1, 2, 4):  # the device's chunk grid (residue masks, stride extraction)
                raise NotImplementedError(f"MS {pid}: unit width {width} not in (1, 2, 4)")
            never = False
            for k, key in enumerate(("sync", "one", "zero", "float")):
                spec = p.get(key)
                if not spec:
                    continue
                fl = self._float_list(spec)
                if fl is None or not fl:
                    never = True  # match_failed (message_synced.py:114-118)
                    break
                self._patspec(rec["key"][k], fl, f"MS {pid} {key}")
            lmin_raw = p.get("length_min", -1)
            if not never:
                rec["lmin_sync"] = _int_exact(lmin_raw, f"MS {pid} length_min")
                if width == 0 and rec["key"][0]["len"]:
                    # bit_length is 0 -> the gate fails for any length_min > 0
                    if rec["lmin_sync"] > 0:
                        never = True
                    else:
                        raise NotImplementedError(f"MS {pid}: zero signal width reaches range(..., 0)")
                if not rec["key"][0]["len"]:
                    raise NotImplementedError(f"MS {pid}: falsy sync not modelled")
            rec["never"] = 1 if never else 0
            rec["lir_min"] = _int_exact(lmin_raw, f"MS {pid} length_min") if not never else -1
            lm = p.get("length_max")
            rec["lir_max"] = _int_exact(lm, f"MS {pid} length_max") if (lm is not None and not never) else INT_NONE
            rec["recon"] = 1 if p.get("reconstructBit") else 0
            pad = _int_exact(p.get("paddingbits", 4), f"MS {pid} paddingbits")
            if pad < 1:
                raise NotImplementedError(f"MS {pid}: paddingbits < 1")
            rec["pad_bits"] = pad
            rec["postdemo"] = self._postdemo(p)
            rec["pre_off"], rec["pre_len"] = self._str(f"{p.get('preamble', '')}")
            rec["post_off"], rec["post_len"] = self._str(f"{p.get('postamble', '')}")

        mc = np.zeros(len(self.mc_pids), MC_REC)
        self.mc_preamble: List[str] = []
        for r, pid in enumerate(self.mc_pids):
            p = P[pid]
            rec = mc[r]
            rec["proto_index"] = self.pids.index(pid)
            cr = p["clockrange"]
            if not (isinstance(cr, list) and len(cr) >= 2):
                raise NotImplementedError(f"MC {pid}: clockrange {cr!r}")
            meth = str(p.get("method", "")).split(".")[-1]
            if meth not in MC_METHODS:
                raise NotImplementedError(f"MC {pid}: method {meth!r} not on the device")
            mc_record(P, pid, meth, rec)
            pre = f"{p.get('preamble', '')}"
            self.mc_preamble.append(pre)
            rec["pre_off"], rec["pre_len"] = self._str(pre)

        # MN = every id with 'modulation' (signalduino/parser/mn.py:80-191)
        self.mn_pids = [pid for pid, p in P.items() if "modulation" in p]
        if len(self.mn_pids) > MN_MAX:
            raise NotImplementedError(f"more than {MN_MAX} MN protocols")
        mn = np.zeros(len(self.mn_pids), MN_REC)
        self.mn_rfmode: List[Any] = []
        self.mn_modulation: List[Any] = []
        self.mn_preamble: List[str] = []
        mn_rx: List[str] = []
        for r, pid in enumerate(self.mn_pids):
            p = P[pid]
            rec = mn[r]
            rec["proto_index"] = self.pids.index(pid)
            self.mn_rfmode.append(p.get("rfmode", None))
            self.mn_modulation.append(p.get("modulation", None))
            lm = p.get("length_min", -1)             # helpers.py:144-164 on len(hex) (mn.py:98)
            rec["lir_min"] = _int_exact(lm, f"MN {pid} length_min")
            lx = p.get("length_max")
            rec["lir_max"] = _int_exact(lx, f"MN {pid} length_max") if lx is not None else INT_NONE
            rx = p.get("regexMatch", None)
            if rx:
                if not isinstance(rx, str):
                    raise NotImplementedError(f"MN {pid}: regexMatch {rx!r}")
                if rx not in mm_patterns:
                    mm_patterns.append(rx)
                rec["dfa"] = mm_patterns.index(rx)
                if rx not in mn_rx:
                    mn_rx.append(rx)
                rec["dfa_slot"] = mn_rx.index(rx)   # per-frame result cache slot (k_mn)
            else:
                rec["dfa"] = -1
                rec["dfa_slot"] = -1
            m = p.get("method")
            if m:
                if not isinstance(m, str):
                    raise NotImplementedError(f"MN {pid}: method {m!r}")
                name = m.split(".")[-1]
                if name in MN_METHODS:
                    rec["method"] = MN_METHODS[name]
                elif name in _OTHER_METHODS:
                    raise NotImplementedError(f"MN {pid}: method {name!r} called with MN arguments (not modelled)")
                else:
                    rec["method"] = MN_MISSING       # mn.py:171-173: not found -> skipped
            pre = f"{p.get('preamble', '')}"
            if len(mn_rx) > 32:
                raise NotImplementedError("more than 32 distinct MN regexMatch patterns")
            self.mn_preamble.append(pre)
            rec["pre_off"], rec["pre_len"] = self._str(pre)

        # JSON fragments for sdx_serialize_json (signalduino/mqtt.py:227-245), rendered by Python's json
        jrec = np.zeros(len(self.mu_pids) + len(self.ms_pids) + len(self.mc_pids) + len(self.mn_pids), JSON_REC)
        j = 0
        for cls_pids, extra in ((self.mu_pids, lambda r: (json.dumps(self.mu_clock[r]), None)),
                                (self.ms_pids, lambda r: (None, None)), (self.mc_pids, lambda r: (None, None)),
                                (self.mn_pids, lambda r: (json.dumps(self.mn_modulation[r]),
                                                          json.dumps(self.mn_rfmode[r])))):
            for r, pid in enumerate(cls_pids):
                s1, s2 = extra(r)
                jrec[j]["pid_off"], jrec[j]["pid_len"] = self._str(json.dumps(pid))
                if s1 is not None:
                    jrec[j]["s1_off"], jrec[j]["s1_len"] = self._str(s1)
                if s2 is not None:
                    jrec[j]["s2_off"], jrec[j]["s2_len"] = self._str(s2)
                j += 1
        self.json_table = jrec
        mufilt = self._mu_filters(mu)
        msfilt = self._ms_filters(ms)

        if b"\n" in bytes(self._heap):
            raise NotImplementedError("newline inside a preamble/postamble ($ semantics)")
        cls_of, n_class, dfas = regex_dfa.compile_bank_dfas(mm_patterns)
        for r, pid in enumerate(self.mu_pids):
            d = int(mu[r]["mm_dfa"])
            if d >= 0:
                pre = f"{P[pid].get('preamble', '')}".encode("latin-1")
                mu[r]["mm_pre_state"] = regex_dfa.dfa_walk(dfas[d], cls_of, dfas[d][1], pre)
        self.mm_patterns = mm_patterns
        self.dfa_host = (cls_of, dfas)
        drec = np.zeros(len(dfas), DFA_REC)
        trans_parts, flag_parts, t256_parts = [], [], []
        toff = foff = t2off = 0
        cls_np = np.asarray(cls_of, dtype=np.int64)
        for i, (nst, start, trans, flags) in enumerate(dfas):
            if nst > 256:
                raise NotImplementedError("modulematch DFA with more than 256 states")
            drec[i]["nstates"], drec[i]["start"] = nst, start
            drec[i]["trans_off"], drec[i]["flags_off"], drec[i]["t256_off"] = toff, foff, t2off
            t = np.asarray(trans, dtype=np.uint16)
            trans_parts.append(t.reshape(-1))
            t256_parts.append(t[:, cls_np].astype(np.uint8).reshape(-1))  # [state][byte]
            flag_parts.append(np.asarray(flags, dtype=np.uint8))
            toff += t.size
            foff += len(flags)
            t2off += nst * 256
        mudesc, mmtab, mm_states = self._mu_desc(mu, dfas, cls_of)
        trans_all = np.concatenate(trans_parts) if trans_parts else np.zeros(0, np.uint16)
        t256_all = np.concatenate(t256_parts) if t256_parts else np.zeros(0, np.uint8)
        flags_all = np.concatenate(flag_parts) if flag_parts else np.zeros(0, np.uint8)
        cls_arr = np.asarray(cls_of, dtype=np.uint8)

        # blob: header | mu | ms | mc | dfa | cls | trans | flags | strings | t256 | order | ranks | mudesc | mmtab | mn
        #       | json
        hdr_size = struct.calcsize(HDR_FMT)
        # processing orders (results are placed by protocol index, so any order is exact):
        # MU sorted by clock so consecutive protocols reuse the normalised patterns
        # MU: clock groups (one normalisation per group and tile), largest group first so that the
        # waves' dynamic grabbing ends on small groups; group g = mu_order[gstart[g]:gstart[g+1]]
        # Groups are taken in descending estimated cost (longest-processing-time first): the cost of a
        # group is one normalisation plus its protocols' filter + decode costs, MU_COST_KCYC
        # (profile-guided, tools/prof_phases.py per-group cycles on the bench corpus; protocols
        # missing from the table count as the table's median).  Scheduling only: results are placed
        # by protocol index.
        groups: Dict[float, List[int]] = {}
        for r in range(len(self.mu_pids)):
            groups.setdefault(float(mu[r]["clock"]), []).append(r)
        costs = MU_COST_KCYC_R3 if os.environ.get("SDX_MU_COSTS") == "r3" else MU_COST_KCYC
        med = float(np.median(list(costs.values())))
        gcost = lambda g: MU_NORM_KCYC + sum(costs.get(str(self.mu_pids[r]), med) for r in g)  # noqa: E731
        if os.environ.get("SDX_MU_ORDER") == "size":   # A/B: the round-2 order (largest group first)
            glist = sorted(groups.values(), key=lambda g: -len(g))
        elif os.environ.get("SDX_MU_ORDER") == "clock":  # A/B: no cost model (groups by clock)
            glist = [groups[c] for c in sorted(groups)]
        else:
            glist = sorted(groups.values(), key=lambda g: (-gcost(g), -len(g)))
        # work items of at most ~MU_SPLIT_KCYC: a clock group whose cost exceeds it is cut at protocol
        # boundaries into pieces of about equal cost (each repeats the normalisation).  The tile's 8
        # waves then end closer together at the end-of-loop barrier: the largest group (≈ 146 kcyc,
        # ≈ one wave's whole share) sets the tile's critical path whenever the other groups of the
        # tile run cheaper than average.  Measured (profiles/r03/s2/mu_split_*.log): k_pulses<MU>
        # 1.098-1.101 ms unsplit, 1.042-1.050 ms at 50-100 kcyc.  SDX_MU_SPLIT=0 disables (A/B).
        split = float(os.environ.get("SDX_MU_SPLIT", str(MU_SPLIT_KCYC)))
        if split > 0:
            pieces = []
            for g in glist:
                m = int(np.ceil((gcost(g) - MU_NORM_KCYC) / split))
                if m <= 1:
                    pieces.append(g)
                    continue
                tot = gcost(g) - MU_NORM_KCYC
                # cut by cumulative cost into m pieces of about equal cost
                cum, cut, cur = 0.0, 1, []
                for r in g:
                    cur.append(r)
                    cum += costs.get(str(self.mu_pids[r]), med)
                    if cum >= tot * cut / m and cut < m:
                        pieces.append(cur)
                        cur, cut = [], cut + 1
                if cur:
                    pieces.append(cur)
            glist = sorted(pieces, key=lambda g: (-gcost(g), -len(g)))
        self.mu_order = [r for g in glist for r in g]
        self.mu_gstart = list(np.cumsum([0] + [len(g) for g in glist]))
        if os.environ.get("SDX_MS_ORDER") == "bank":   # A/B: bank order
            self.ms_order = list(range(len(self.ms_pids)))
        else:   # descending profile-guided cost; results are placed by protocol index
            ms_med = float(np.median(list(MS_COST_KCYC.values())))
            self.ms_order = sorted(range(len(self.ms_pids)),
                                   key=lambda r: -MS_COST_KCYC.get(str(self.ms_pids[r]), ms_med))
        order = np.asarray(self.mu_order + self.ms_order + self.mu_gstart, dtype=np.uint16)
        ranks = np.asarray(self._ranks, dtype=np.uint16)
        sections = [mu.tobytes(), ms.tobytes(), mc.tobytes(), drec.tobytes(), cls_arr.tobytes(),
                    trans_all.tobytes(), flags_all.tobytes(), bytes(self._heap), t256_all.tobytes(),
                    order.tobytes(), ranks.tobytes(), mudesc.tobytes(), mmtab.tobytes(), mn.tobytes(), jrec.tobytes(),
                    mufilt.tobytes(), msfilt.tobytes(), mn_tables()]
        offs = []
        cur = (hdr_size + 15) // 16 * 16
        for k, s in enumerate(sections):
            if k in (15, 16):                # sdx_mu_filt / sdx_ms_filt: whole 128-byte scalar-cache lines
                cur = (cur + 127) // 128 * 128
            offs.append(cur)
            cur = (cur + len(s) + 15) // 16 * 16
        total = cur
        blob = bytearray(total)
        hdr = struct.pack(HDR_FMT, MAGIC, VERSION, len(self.pids), len(self.mu_pids), len(self.ms_pids),
                          len(self.mc_pids), len(dfas), n_class, *offs[:8], total, offs[8], offs[9], offs[10], offs[11], offs[12],
                          len(mmtab), mm_states, len(glist), len(self.mn_pids), offs[13], offs[14], offs[15], offs[16], offs[17])
        blob[:hdr_size] = hdr
        for o, s in zip(offs, sections):
            blob[o:o + len(s)] = s
        self.blob = bytes(blob)
        self.mu_table, self.ms_table, self.mc_table, self.mn_table = mu, ms, mc, mn

    @staticmethod
    def _fspecs(specs, x, first_upk: str) -> bool:
        """Fill x["spec"][0..3] (sdx_fspec) from four sdx_patspec; False if one does not fit."""
        ok = True
        for i, ps in enumerate(specs):
            fs = x["spec"][i]
            nu = int(ps["nuniq"])
            fs["rk2_len_nu"] = (int(ps["len"]) << 16) | (min(nu, 255) << 24)  # len is read even when full
            if nu > 3:
                ok = False
                continue
            for u in range(nu):
                lo, hi, ro = int(ps["klo"][u]), int(ps["khi"][u]), int(ps["rk_off"][u])
                if not (-32768 <= lo <= 32767 and -32768 <= hi <= 32767 and 0 <= ro <= 65535):
                    ok = False
                fs["lohi"][u] = (lo & 0xFFFF) | ((hi & 0xFFFF) << 16)
            rk = [int(ps["rk_off"][u]) & 0xFFFF for u in range(3)]
            fs["rk01"] = rk[0] | (rk[1] << 16)
            fs["rk2_len_nu"] = rk[2] | (int(ps["len"]) << 16) | (nu << 24)
            upk = int(ps["uidx_pk"])
            if i == 0:
                x[first_upk] = upk
            elif upk >= 1 << 32:
                ok = False
            else:
                fs["upk"] = upk
        return ok

    @classmethod
    def _mu_filters(cls, mu) -> np.ndarray:
        """sdx_mu_filt: the lane filter's compact copy of each MU record (include/sdx_bank.h)."""
        f = np.zeros(len(mu), MU_FILT)
        for r in range(len(mu)):
            rec, x = mu[r], f[r]
            x["clock"] = rec["clock"]
            x["clk_c"], x["clk_m"], x["clk_sh"] = clock_divider(float(rec["clock"]))
            ok = cls._fspecs([rec[k] for k in ("start", "one", "zero", "flt")], x, "start_upk")
            x["flags"] = (int(rec["has_start"]) | (int(rec["never"]) << 1) | (int(rec["active"]) << 2) |
                          ((0 if ok else 1) << 3))
        return f

    @classmethod
    def _ms_filters(cls, ms) -> np.ndarray:
        """sdx_ms_filt: the MS lane filter's compact copy of each MS record."""
        f = np.zeros(len(ms), MS_FILT)
        for r in range(len(ms)):
            rec, x = ms[r], f[r]
            x["pclock"] = rec["pclock"]
            x["width"], x["lmin_sync"] = rec["width"], rec["lmin_sync"]
            ok = cls._fspecs([rec["key"][k] for k in range(4)], x, "sync_upk")
            x["flags"] = (int(rec["never"]) << 1) | ((0 if ok else 1) << 3)
        return f

    @staticmethod
    def _mm_length_interval(hex16, flags, post_map, pre_state, nmax: int = MM_FAST_DIGITS):
        """[lo, hi] if the LDS-table walk's outcome (message_unsynced.py:277-280) depends on the
        number of hex digits only, for every digit string of 0..nmax digits, and the accepted
        counts form one interval (lo > hi: none accepted); else None.  Exact: the set of states
        reachable after n digits is enumerated and every one of them must give the same outcome."""
        def accept(st):
            f = int(flags[int(post_map[st])])
            return bool(f & regex_dfa.ACC_NOW) or (not f & regex_dfa.DEAD and bool(f & regex_dfa.ACC_END))

        cur = {pre_state}
        acc = []
        for _ in range(nmax + 1):
            outs = {accept(st) for st in cur}
            if len(outs) != 1:
                return None
            acc.append(outs.pop())
            cur = {int(hex16[st][v]) for st in cur for v in range(16)}
        ns = [n for n, a in enumerate(acc) if a]
        if not ns:
            return (1, 0)
        if ns != list(range(ns[0], ns[-1] + 1)):
            return None
        return (ns[0], ns[-1])

    def _mu_desc(self, mu, dfas, cls_of):
        """MU decode descriptors + the LDS modulematch tables.

        mm tables (u8): hex[S][16] (DFA step on hex digit v, local state ids), flags[S], then per
        protocol post[nstates] (state after its postamble).  ACC_NOW and DEAD are absorbing, so
        walking every character and testing the final flags equals message_unsynced.py:277-280's
        re.search.  A DFA that does not fit MMTAB_LDS (or is not absorbing) keeps mm_on = 2: the
        device walks it byte by byte through the blob's t256 table instead.
        """
        P = self.protocols
        d = np.zeros(len(self.mu_pids), MU_DESC)
        hexc = [ord(c) for c in "0123456789ABCDEF"]
        base_of: Dict[int, int] = {}
        hex_rows: List[np.ndarray] = []
        flag_rows: List[np.ndarray] = []
        post_rows: List[int] = []
        S = 0

        def absorbing(nst, trans, flags):
            t = np.asarray(trans)
            for st in range(nst):
                for bit in (regex_dfa.ACC_NOW, regex_dfa.DEAD):
                    if flags[st] & bit and not all(flags[x] & bit for x in t[st]):
                        return False
            return True

        def walk(dfa, st, data: bytes) -> int:
            nst, start, trans, flags = dfa
            for b in data:
                st = int(trans[st][cls_of[b]])
            return st

        for r, pid in enumerate(self.mu_pids):
            rec, p = mu[r], P[pid]
            x = d[r]
            pre = f"{p.get('preamble', '')}".encode("latin-1")
            post = f"{p.get('postamble', '')}".encode("latin-1")
            x["pre_len"], x["post_len"] = min(len(pre), 255), min(len(post), 255)
            x["pre"][:min(len(pre), 16)] = list(pre[:16])
            x["post"][:min(len(post), 2)] = list(post[:2])
            x["width"] = int(rec["width"])
            x["len_s"] = int(rec["start"]["len"]) if rec["has_start"] else 0
            x["recon"], x["dispatch_bin"] = int(rec["recon"]), int(rec["dispatch_bin"])
            x["remove_zero"], x["postdemo"] = int(rec["remove_zero"]), int(rec["postdemo"])
            if int(rec["pad_bits"]) > 255:
                raise NotImplementedError(f"MU {pid}: paddingbits > 255")
            x["pad_bits"] = int(rec["pad_bits"])
            x["lmin"] = min(int(rec["length_min"]), 65535)
            x["lmax"] = min(int(rec["length_max"]), 65535)  # chunk counts never exceed 4096
            k = int(rec["mm_dfa"])
            if k < 0:
                continue
            x["mm_on"] = 2
            x["pre_state"] = int(rec["mm_pre_state"])
            nst, start, trans, flags = dfas[k]
            if not absorbing(nst, trans, flags):
                continue
            if k not in base_of:
                if 17 * (S + nst) + len(post_rows) + nst > MMTAB_LDS:
                    continue
                base_of[k] = S
                t = np.asarray(trans, dtype=np.int64)
                hex_rows.append(t[:, [cls_of[c] for c in hexc]].astype(np.uint8))
                flag_rows.append(np.asarray(flags, dtype=np.uint8))
                S += nst
            if 17 * S + len(post_rows) + nst > MMTAB_LDS:
                continue
            x["mm_on"] = 1
            x["mm_base"] = base_of[k]
            x["mm_post"] = len(post_rows)
            post_map = [walk(dfas[k], st, post) for st in range(nst)]
            post_rows.extend(post_map)
            hex16 = np.asarray(trans, dtype=np.int64)[:, [cls_of[c] for c in hexc]]
            iv = self._mm_length_interval(hex16, flags, post_map, int(rec["mm_pre_state"]))
            if iv is not None:  # the outcome depends on the digit count only: no walk on the device
                x["mm_on"] = 3
                x["res"][0], x["res"][1] = iv
        hexs = np.concatenate(hex_rows).reshape(-1) if hex_rows else np.zeros(0, np.uint8)
        fls = np.concatenate(flag_rows) if flag_rows else np.zeros(0, np.uint8)
        tab = np.concatenate([hexs, fls, np.asarray(post_rows, dtype=np.uint8)])
        tab = np.concatenate([tab, np.zeros((-len(tab)) % 16, np.uint8)])
        assert len(tab) <= MMTAB_LDS
        self.mu_desc = d
        return d, tab, S

    # -- host-side metadata used when turning device records into reference dicts -------------
    def class_pid(self, kind: str, rec_index: int) -> str:
        return {"MU": self.mu_pids, "MS": self.ms_pids, "MC": self.mc_pids}[kind][rec_index]
