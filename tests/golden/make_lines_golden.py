#!/usr/bin/env python3
"""Generate the wire-line front-end goldens from the REFERENCE parser.

Runs ONLY in the development container, where the read-only reference is mounted at
/root/reference (it never travels to the GPU box).  The reference package's top-level
``signalduino/__init__.py`` imports the controller stack (``jsonschema``, not installed here), so
the package is registered by path and only its ``signalduino.parser`` / ``types`` /
``exceptions`` modules are imported -- nothing is stubbed.

For every line it records, from the reference itself:
  * ``payload``  -- ``base.extract_payload(line)`` (framing + decompress_payload), or None,
  * ``calls``    -- what ``SignalParser.parse_line`` hands to the demodulators
                    (``demodulate(msg_data, type)`` / ``demodulate_mc(msg_data, frame)``),
                    captured by a recording subclass of the reference SDProtocols, with the
                    RawFrame fields the parser set (line, message_type, rssi, freq_afc),
  * ``e2e``      -- for the lines that reach a demodulator, the DecodedMessage list of a real
                    ``SignalParser(SDProtocols())`` (strict MC, i.e. the reference's behaviour).
Inputs: every message string the reference's parser tests hold (raw and STX/ETX-framed), the
decompression test vectors, seeded synthetic firmware lines (plain and Mred=1 compressed,
``pysignalduino_amd.synth.line_corpus``) and seeded mutations of them (``synth.mutate_line``).
The fixture is data (inputs + the reference's outputs); no reference source is copied.

Usage:  python tests/golden/make_lines_golden.py [--n 1500 --n-fuzz 2500]
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
from signalduino.parser import base as ref_base  # noqa: E402

from pysignalduino_amd import bank as B  # noqa: E402
from pysignalduino_amd import synth  # noqa: E402


class Recorder(SDProtocols):
    """The reference SDProtocols with the demodulator entry points recording their input."""

    def __init__(self):
        super().__init__()
        self.calls = []

    def demodulate(self, msg_data, msg_type):
        self.calls.append([msg_type, list(msg_data.items())])
        return [{"protocol_id": "rec", "payload": "", "meta": {}}]

    def demodulate_mc(self, msg_data, msg_type, version=None):
        self.calls.append(["MC", list(msg_data.items())])
        return [{"protocol_id": "rec", "payload": "", "meta": {}}]


def _frame(fr):
    return [fr.line, fr.message_type, fr.rssi, fr.freq_afc]


def harvest_test_lines():
    """String constants of the reference's parser tests that look like firmware payloads."""
    out = []
    for fn in ("test_mu_parser.py", "test_ms_parser.py", "test_mc_parser.py", "test_controller.py",
               "test_mu_demodulation.py", "test_postdemodulation.py"):
        tree = ast.parse(open(os.path.join(REF, "tests", fn), encoding="utf-8").read())
        for node in ast.walk(tree):
            if isinstance(node, ast.Constant) and isinstance(node.value, str):
                s = node.value
                if len(s) < 400 and (s[:3].upper() in ("MU;", "MS;", "MC;", "MN;", "MO;") or s[:1] == "\x02"):
                    out.append((fn, s))
    tree = ast.parse(open(os.path.join(REF, "tests", "test_decompress_payload.py"), encoding="utf-8").read())
    for node in ast.walk(tree):  # the compressed vectors are space-separated hex strings
        if isinstance(node, ast.Constant) and isinstance(node.value, str) and node.value[:3] == "4d ":
            out.append(("test_decompress_payload.py", bytes.fromhex(node.value.replace(" ", "")).decode("latin-1")))
    return out


EDGE = [  # hand-written corner cases of the parser rules (latin-1 strings)
    "\x02MO;P0=1;D=01;\x03", "\x02Mo;P0=1;\x03", "\x02MO;\x80\x81\x82;D\x01;\x03",
    "\x02MN;D=AB12;R=20;\x03", "\x02MN;D=Y9A;\x03", "\x02MC;;\x03", "\x02MS;;\x03", "\x02MU;;\x03",
    "\x02Mu;;\x03", "\x02M;;\x03", "\x02MX;D=1;\x03", "\x02mS;D=1;\x03",
    "  \x02MS;P0=-4000;P1=500;D=0101;CP=1;SP=0;\x03 \r\n", "\x85\x02MS;P0=-4000;P1=500;D=0101;CP=1;SP=0;\x03\xa0",
    "\x1c\x02MS;P0=-4000;P1=500;D=0101;CP=1;SP=0;\x03\x1f", "\x02MS;P0=1;\nD=0;\x03", "\x02MS;P0=1;D=0;\x03\n\n",
    "\x02Ms;P0=-4000;P1=500;D=0101;CP=1;SP=0;\x03", "\x02MU;P0=1;P1=-2;D=01;\x03\n", "\x02MU;P0=1;P1=-2;D=0;\x03",
    "\x02MU;P0=1;P1=-2;D=01;CP=1;R=5;O;e;p;w=3;\x03", "\x02MU;P0=1;P1=-2;D=01;w=33;\x03", "\x02MU;P0=100000;P1=-2;D=01;\x03",
    "\x02MU;P8=1;P1=-2;D=01;\x03", "\x02MU;P0=1;P1=2;P2=3;P3=4;P4=5;P5=6;P6=7;P7=8;P0=9;D=01;\x03",
    "\x02MU;P0=-1;P1=-2;D=0101;D=1010;CP=0;\x03", "\x02MU;P0=-01;P1=+2;D=01;\x03",
    "\x02MS;P0=-4000;P1=500;D=0101;CP=01;SP=0;\x03", "\x02MS;P0=-4000;P01=600;P1=500;D=0101;CP=1;SP=0;\x03",
    "\x02MS;P0=-4000;P1=;D=0101;CP=1;SP=0;\x03", "\x02MS;P0=-4000;P1=500;P1=;D=0101;CP=1;SP=0;\x03",
    "\x02MS;P0=-4000;P1=abc;D=0101;CP=1;SP=0;\x03", "\x02MS;P0=-4000;P1=500;D=0101;CP=1;SP=0;R=;\x03",
    "\x02MS;P0=-4000;P1=500;D=0101;CP=1;SP=0;R=1q;\x03", "\x02MS;P0=-4000;P1=500;D=0101;CP=1;\x03",
    "\x02MS;P0=-4000;P1=500;D=0101;CP=7;SP=0;\x03", "\x02MS;P0=-4000;P1=500;D=01x1;CP=1;SP=0;\x03",
    "\x02MS;P0=-4000;P1=500;D=;CP=1;SP=0;\x03", "\x02MS;P0=-4000;P1=500;D;CP=1;SP=0;\x03",
    "\x02MS;P0=-4000;P1=500;D=0101;CP=1;SP=0;F=12;R=200;\x03", "\x02MS;P0=-4000;P1=500;D=0101;CP=1;SP=0;R= 42;\x03",
    "\x02MS;P0=-4000;P1=500;D=0101;CP=1;SP=0;P10=3;\x03", "\x02MS;P0=-4000;P1=500;D=0101;CP=1;SP=0;=5;\x03",
    "\x02MC;LL=-762;LH=544;D=DB6;C=1e;L=12;\x03", "\x02MC;LL=-762;D=DB6;C=342;L=+12;R=-5;F=+7;\x03",
    "\x02Mc;LL=-762;D=DB6;C=342;L=12;\x03", "\x02MC;MC=5;D=DB6;C=342;L=12;\x03", "\x02Mc;MC=5;D=DB6;C=342;L=12;\x03",
    "\x02MC;X;D=DB6;C=342;L=12;\x03", "\x02MC;D=DB6;D=DB6;C=342;L=12;\x03", "\x02MC;D=+DB6;C=342;L=12;\x03",
    "\x02MC;D=DB6;C=342;L=12;R=1234567890123;\x03", "\x02MC;D=DB6;C=342;L=12;M=AB;\x03", "\x02MC;D=DB6;C=342;L=12;Mc;\x03",
    "\x02MC;D=DB6;C=342;L=12;ZZ=1;\x03", "\x02MC;D=DB6;C=342;L=12;zz=1;\x03", "\x02MC;D=DB6;C=99999999999;L=12;\x03",
    "\x02MC;D=DB6;C=342;\x03", "\x02MC;D=;C=342;L=12;\x03", "\x02MC;D=DB6;C=342;L=12;R=2a;\x03",
    # compressed: ';' bytes inside the data, field-looking bytes after them, 'd' (odd) data, R/F hex fields
    "\x02Mu;\x80\xf4\x81;\xa1\xf4\x81;D\x01;\x10\x01;C0;R2F;\x03",
    "\x02Mu;\x80\xf4\x81;\xa1\xf4\x81;D\x01;C\x01;C1;\x03", "\x02Ms;\x80\xf4\x81;\xa1\xf4\x81;\xa2\xe0\x9f;d\x21\x01\x10;C0;S2;RFF;F1A;\x03",
    "\x02Ms;\x80\xf4\x81;\xa1\xf4\x81;\xa2\xe0\x9f;D\x21\x01\x10;;;\x10;C0;S2;O;m2;\x03",
    "\x02Mu;\x80\xf4;\xa1\xf4\x81;D\x81\x01;C0;\x03", "\x02Mu;\x90\xf4\x81;\xb1\xf4\x81;D\x01\x01;C0;x;#5;%;\x03",
    "\x02Mu;\x80\xf4\x81;Mab;D\x01;C0;\x03", "\x02Mu;\x80\xf4\x81;M\xe9;D\x01;C0;\x03",
    "\x02Ms;\x80\xf4\x81;\xa1\xf4\x81;\xa2\xe0\x9f;D\x21\x01\x10;C0;S2;\xffab;\x03",
]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1500)
    ap.add_argument("--n-fuzz", type=int, default=2500)
    ap.add_argument("--seed", type=int, default=2024)
    a = ap.parse_args()

    lines = []  # (src, latin-1 str)
    for fn, s in harvest_test_lines():
        lines.append((fn + ":raw", s))
        if s[:1] != "\x02":
            lines.append((fn + ":framed", "\x02" + s + "\x03"))
            lines.append((fn + ":framed+nl", "\x02" + s + "\x03\r\n"))
    lines += [("edge", s) for s in EDGE]
    protos = B.Bank().protocols
    corpus, _ = synth.line_corpus(protos, a.n, seed=a.seed, compress_frac=0.4, mu_npulse=96)
    lines += [("synth", ln.decode("latin-1")) for ln in corpus]
    rng = np.random.default_rng(a.seed + 1)
    base_pool = [ln for _, ln in lines]
    for k in range(a.n_fuzz):
        src = base_pool[int(rng.integers(0, len(base_pool)))].encode("latin-1")
        m = synth.mutate_line(rng, src)
        if rng.random() < 0.3:
            m = synth.mutate_line(rng, m)
        lines.append(("fuzz", m.decode("latin-1")))

    rec = Recorder()
    rec_parser = SignalParser(protocols=rec)
    real_parser = SignalParser(protocols=SDProtocols())
    cases = []
    for src, ln in lines:
        c = {"src": src, "line": ln, "payload": ref_base.extract_payload(ln)}
        rec.calls = []
        try:
            res = rec_parser.parse_line(ln)
        except Exception as e:  # noqa: BLE001  (recorded: parse_line itself raised)
            c["raise"] = type(e).__name__
            res = []
        c["calls"] = rec.calls
        c["frame"] = _frame(res[0].raw) if res else None
        if rec.calls:
            try:
                got = real_parser.parse_line(ln)
                c["e2e"] = [[d.protocol_id, d.payload, d.metadata, _frame(d.raw)] for d in got]
            except Exception as e:  # noqa: BLE001
                c["e2e_raise"] = type(e).__name__
        cases.append(c)
    path = os.path.join(HERE, "lines_golden.json.gz")
    with gzip.open(path, "wt", encoding="utf-8") as f:
        json.dump(cases, f, separators=(",", ":"))
    ncall = sum(1 for c in cases if c["calls"])
    nres = sum(len(c.get("e2e", [])) for c in cases)
    print(f"wrote {path}: {os.path.getsize(path)} bytes, {len(cases)} lines, {ncall} reach a demodulator, "
          f"{nres} decoded messages")


if __name__ == "__main__":
    main()
