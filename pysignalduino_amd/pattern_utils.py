"""Drop-in for the reference's ``sd_protocols.pattern_utils`` (pattern_utils.py:1-136).

``pattern_exists`` runs on the MI355X (``sdx_units`` op SDX_UNIT_PEXISTS, csrc/sdx_units.hip): the
unique search values, the fp64 candidate test ``gap <= 0.001 or gap <= tol`` with the stable sort
by gap, the > 10000-combinations abort, ``itertools.product`` order with id reuse skipped and the
substring test of the concatenated ids.  ``pattern_exists_batch`` evaluates many calls in one
launch.  The three scalar helpers (tolerance, in-tolerance test, cartesian product) are plain
arithmetic on host values, as in the reference.

Device contract (else ``ContractError``): finite int/float values (ints below 2**52 in
magnitude), at most 32 search values and 16 patterns, str pattern ids of at most 255 UTF-8 bytes,
a str raw_data.
"""
from __future__ import annotations

import itertools
import math
from typing import Any, Dict, List, Sequence, Tuple, Union

import numpy as np

from . import runtime
from .packing import ContractError


def is_in_tolerance(val1: float, val2: float, tol: float) -> bool:
    """pattern_utils.py:11-13."""
    return abs(val1 - val2) <= tol


def calculate_tolerance(val: float) -> float:
    """pattern_utils.py:15-26."""
    abs_val = abs(val)
    if abs_val > 3:
        if abs_val > 16:
            return abs_val * 0.18
        return abs_val * 0.3
    return 1.0


def cartesian_product(lists: List[List[Any]]) -> List[List[Any]]:
    """pattern_utils.py:28-32."""
    if not lists:
        return [[]]
    return [list(p) for p in itertools.product(*lists)]


def _num(v, what) -> float:
    if isinstance(v, bool) or not isinstance(v, (int, float)):
        raise ContractError(f"pattern_exists: {what} {v!r} is not an int/float")
    if isinstance(v, int):
        if abs(v) >= 1 << 52:
            raise ContractError(f"pattern_exists: {what} {v} is too large for exact fp64 arithmetic")
        return float(v)
    if not math.isfinite(v):
        raise ContractError(f"pattern_exists: {what} {v!r} is not finite")
    return v


def _pack(search_pattern, pattern_list, raw_data) -> Tuple[bytes, np.ndarray, int, int]:
    if not isinstance(pattern_list, dict) or not isinstance(raw_data, str) or \
            not isinstance(search_pattern, (list, tuple)):
        raise ContractError("pattern_exists: (list, dict, str) arguments expected for the device path")
    if len(search_pattern) > runtime.UNIT_PX_SEARCH or len(pattern_list) > runtime.UNIT_PX_PAT:
        raise ContractError(f"pattern_exists: more than {runtime.UNIT_PX_SEARCH} search values or "
                            f"{runtime.UNIT_PX_PAT} patterns")
    ids = []
    for k in pattern_list:
        if not isinstance(k, str):
            raise ContractError("pattern_exists: pattern ids must be str")
        b = k.encode("utf-8")
        if len(b) > 255:
            raise ContractError("pattern_exists: pattern id longer than 255 bytes")
        ids.append(b)
    vals = [_num(v, "search value") for v in search_pattern] + \
           [_num(v, "pattern value") for v in pattern_list.values()]
    head = bytes([len(ids)]) + bytes(len(b) for b in ids) + b"".join(ids)
    raw = raw_data.encode("utf-8")   # UTF-8 substring search == str substring search
    cap = sum(max((len(b) for b in ids), default=0) for _ in search_pattern) + 8
    return head + raw, np.asarray(vals, np.float64), len(search_pattern), cap


def pattern_exists_batch(calls: Sequence[tuple], device: int = 0) -> List[Union[str, int]]:
    """[pattern_exists(search, patterns, raw_data) for (search, patterns, raw_data) in calls],
    in one launch."""
    ins, vals, args, caps = [], [], [], []
    for c in calls:
        b, v, ns, cap = _pack(*c[:3])
        ins.append(b)
        vals.append(v)
        args.append(ns)
        caps.append(cap)
    if not ins:
        return []
    desc, rec, heap = runtime.UnitRunner.get(device).run(runtime.UNIT_PEXISTS, ins, caps, args=args, vals=vals)
    out: List[Union[str, int]] = []
    for d, r in zip(desc, rec):
        if d["status"] != runtime.ST_OK:
            raise RuntimeError("pattern_exists: device status %d" % int(d["status"]))
        if int(r["proto"]):
            out.append(-1)
        else:
            o = int(r["payload_off"])
            out.append(heap[o: o + int(r["payload_len"])].tobytes().decode("utf-8"))
    return out


def pattern_exists(search_pattern: List[float], pattern_list: Dict[str, float], raw_data: str,
                   debug_callback=None) -> Union[str, int]:
    """pattern_utils.py:34-136 on the GPU (``debug_callback`` receives nothing: the device keeps
    no trace of its candidate lists)."""
    return pattern_exists_batch([(search_pattern, pattern_list, raw_data)])[0]
