#!/usr/bin/env python3
"""Generate the MN (FSK) path goldens from the REFERENCE implementation.

Runs ONLY in the development container, where the read-only reference is mounted at
/root/reference (it never travels to the GPU box).  As in make_lines_golden.py the reference
package is registered by path and only ``signalduino.parser`` / ``types`` / ``exceptions`` and
``sd_protocols`` are imported -- nothing is stubbed.

Recorded, from the reference itself:
  * ``lines``   -- framed MN lines -> ``SignalParser(rfmode=...).parse_line(line)`` (DecodedMessage
                   protocol_id, payload, metadata, raw.line / message_type / rssi / freq_afc); inputs:
                   every "MN;" string of the reference's MN tests with rfmode None and every rfmode
                   of the bank, seeded synthetic frames (``synth.mn_frames``) with rfmode None or a
                   seeded rfmode, and seeded mutations of them (``synth.mutate_line``),
  * ``methods`` -- ``SDProtocols().<ConvX>({'data': d, 'protocol_id': pid}, 'MN')`` for the 7 MN
                   methods on the hex vectors of the reference's tests/test_helpers.py and on
                   synthetic frames (the list, or the exception class),
  * ``demod``   -- ``SDProtocols().demodulate_mn(msg_data, 'MN')`` for every MN id.
The fixture is data (inputs + the reference's outputs); no reference source is copied.

Usage:  python tests/golden/make_mn_golden.py [--n 3000 --n-fuzz 1500]
"""
from __future__ import annotations

import argparse
import ast
import gzip
import json
import os
import sys
import types

import numpy as np

REF = "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.dont_write_bytecode = True
sys.path.insert(0, REPO)
sys.path.insert(0, REF)

_pkg = types.ModuleType("signalduino")
_pkg.__path__ = [os.path.join(REF, "signalduino")]
sys.modules["signalduino"] = _pkg

from sd_protocols import SDProtocols  # noqa: E402  (the reference, read-only)
from signalduino.parser import SignalParser  # noqa: E402

from pysignalduino_amd import synth  # noqa: E402

METHODS = ["ConvBresser_lightning", "ConvBresser_5in1", "ConvBresser_6in1", "ConvBresser_7in1", "ConvPCA301",
           "ConvKoppFreeControl", "ConvLaCrosse"]


def harvest():
    lines, hexes = [], []
    for fn in ("test_mn_parser.py", "test_mn_bresser_lightning.py", "test_helpers.py"):
        tree = ast.parse(open(os.path.join(REF, "tests", fn), encoding="utf-8").read())
        for node in ast.walk(tree):
            if isinstance(node, ast.Constant) and isinstance(node.value, str):
                s = node.value
                if s.startswith("MN;") or s.startswith("FOO;"):
                    lines.append(s)
                elif fn == "test_helpers.py" and len(s) >= 4 and all(c in "0123456789ABCDEFabcdefP" for c in s):
                    hexes.append(s)
    return sorted(set(lines)), sorted(set(hexes))


def decoded(msgs):
    return [[m.protocol_id, m.payload, m.metadata, [m.raw.line, m.raw.message_type, m.raw.rssi, m.raw.freq_afc]]
            for m in msgs]


def run_line(line, rfmode):
    p = SignalParser(protocols=SDProtocols(), rfmode=rfmode)
    try:
        return {"out": decoded(p.parse_line(line))}
    except Exception as e:  # noqa: BLE001
        return {"raise": type(e).__name__}


def run_method(proto, name, d, pid):
    try:
        return {"out": getattr(proto, name)({"data": d, "protocol_id": pid}, "MN")}
    except Exception as e:  # noqa: BLE001
        return {"raise": type(e).__name__}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=3000)
    ap.add_argument("--n-fuzz", type=int, default=1500)
    a = ap.parse_args()
    proto = SDProtocols()
    mn_ids = proto.get_keys("modulation")
    rfmodes = [proto.check_property(pid, "rfmode") for pid in mn_ids]
    test_lines, test_hex = harvest()
    rng = np.random.default_rng(2024)
    cases = []
    for s in test_lines:
        for rf in [None] + sorted(set(rfmodes)) + ["NoSuchMode"]:
            cases.append(["test", "\x02" + s + "\x03\n", rf])
    frames = synth.mn_frames(a.n, seed=4711)
    synth_lines = []
    for h, y, r, af in frames:
        ln = synth.frame(synth.mn_payload(h, y, r, af)).decode("latin-1")
        synth_lines.append(ln)
        rf = None if rng.random() < 0.6 else rfmodes[int(rng.integers(0, len(rfmodes)))]
        cases.append(["synth", ln, rf])
    for k in range(a.n_fuzz):
        base = synth_lines[int(rng.integers(0, len(synth_lines)))].encode("latin-1")
        ln = synth.mutate_line(rng, base).decode("latin-1")
        cases.append(["fuzz", ln, None if k % 2 else rfmodes[int(rng.integers(0, len(rfmodes)))]])
    extra = ["MN;D=;", "MN;D=Y;", "MN;D=YY12;", "MN;D=12;R=;", "MN;D=12;A=1234;", "MN;D=12;A=-0;", "MN;D=12;A=+5;",
             "MN;D=12;R=5;R=6;", "MN;D=12;A=5;R=6;", "MN;D=12", "MN;D=12;X=1;", "Mn;D=12;", "mN;D=12;",
             "MN;D=ab12;", "MN;D=12;R=1234567890123456789;", "MN;D=0000;", "MN;D=0;", "MN;D=9;", "MN;D=51" + "0" * 26 + ";",
             "MN;D=08" + "1" * 16 + ";", "MN;D=" + "F" * 16 + ";R=255;A=999;", "MN;D=" + "F" * 16 + ";R=128;A=-999;"]
    for s in extra:
        for rf in (None, "Avantek", "Rojaflex", "KOPP_FC", "Lacrosse_mode1"):
            cases.append(["edge", "\x02" + s + "\x03", rf])
    lines = [[src, ln, rf, run_line(ln, rf)] for src, ln, rf in cases]

    meth_inputs = list(test_hex) + [h for h, _, _, _ in frames[:800]] + ["", "0", "9A", "0105A"]
    methods = []
    for d in meth_inputs:
        for name in METHODS:
            methods.append([name, d, run_method(proto, name, d, "101"), ])
    demod = []
    for h, _, _, _ in frames[:600]:
        for pid in mn_ids + ["0", "nope"]:
            md = {"data": h, "protocol_id": pid}
            try:
                demod.append([pid, h, {"out": proto.demodulate_mn(dict(md), "MN")}])
            except Exception as e:  # noqa: BLE001
                demod.append([pid, h, {"raise": type(e).__name__}])
    demod.append([None, "12", {"out": proto.demodulate_mn({"data": "12"}, "MN")}])
    obj = {"mn_ids": mn_ids, "lines": lines, "methods": methods, "demod": demod}
    path = os.path.join(HERE, "mn_golden.json.gz")
    with gzip.open(path, "wt", encoding="utf-8") as f:
        json.dump(obj, f, separators=(",", ":"))
    print(f"wrote {path}: {os.path.getsize(path)} bytes; {len(lines)} lines, {len(methods)} method calls, "
          f"{len(demod)} demodulate_mn calls")


if __name__ == "__main__":
    main()
