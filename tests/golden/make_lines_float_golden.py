#!/usr/bin/env python3
"""Golden lines whose P# values use Python float() syntax beyond plain integers, recorded from the
REFERENCE's own SignalParser (same record format as make_lines_golden.py; runs ONLY in the
development container).

The reference converts pattern values with float(v) (message_unsynced.py:31-35,
message_synced.py:50-57): decimals, exponents, whitespace, underscores between digits, inf / nan
are values; anything else raises ValueError and the key is skipped.  The lines take synthetic MU/MS
lines (pysignalduino_amd/synth.py line_corpus) and rewrite some P values into an equal or nearby
value in another syntax, or into invalid syntax.

Usage:  python tests/golden/make_lines_float_golden.py
"""
from __future__ import annotations

import gzip
import json
import os
import re
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import make_lines_golden as M  # noqa: E402  (sets up the reference import paths)

SYNTAX = [  # f(value) -> string
    lambda v: f"{v}.0", lambda v: f"{v}.", lambda v: f"{v:.2f}", lambda v: f"{v / 10:g}e1", lambda v: f"{v}E0",
    lambda v: f" {v}", lambda v: f"{v}\t", lambda v: f"{v:_}", lambda v: f"{v}.000000000000000000000",
    lambda v: f"{v}.5", lambda v: f"{v}.25e-1", lambda v: f"{v * 1000}e-3", lambda v: f"+{v}.0",
    lambda v: f"{v}0000000000000000000e-19", lambda v: f"{v}.1234567890123456789",
    lambda v: f"{v}e400", lambda v: f"{v}e-400", lambda v: f"{v}__0", lambda v: f"_{v}", lambda v: f"{v}_",
    lambda v: f"{v}e", lambda v: f"{v}.e5", lambda v: f"0x{abs(v):x}", lambda v: f"{v}e+2_0",
    lambda v: "inf" if v > 0 else "-Infinity", lambda v: "nan" if v > 0 else "-NaN", lambda v: f"{v}..0",
    lambda v: f"{v}e-22", lambda v: f"{v}e22", lambda v: f"{v}e23", lambda v: f"9007199254740993.0",
    lambda v: f"{v}\x1c", lambda v: f"0{v}", lambda v: f"-0.{abs(v)}",
]


def main():
    protos = M.B.Bank().protocols
    corpus, _ = M.synth.line_corpus(protos, 900, seed=77, compress_frac=0.0, mu_npulse=96, mix=(0.5, 0.5, 0.0))
    rng = np.random.default_rng(78)
    lines = []
    for ln in corpus:
        s = ln.decode("latin-1")
        keys = re.findall(r";P(\d)=(-?\d+)", s)
        if not keys:
            continue
        for _ in range(int(rng.integers(1, 3))):
            k, v = keys[int(rng.integers(0, len(keys)))]
            f = SYNTAX[int(rng.integers(0, len(SYNTAX)))]
            s = s.replace(f";P{k}={v};", f";P{k}={f(int(v))};", 1)
        lines.append(("float", s))
    rec = M.Recorder()
    rec_parser = M.SignalParser(protocols=rec)
    real_parser = M.SignalParser(protocols=M.SDProtocols())
    cases = []
    for src, ln in lines:
        c = {"src": src, "line": ln, "payload": M.ref_base.extract_payload(ln)}
        rec.calls = []
        res = rec_parser.parse_line(ln)
        c["calls"] = rec.calls
        c["frame"] = M._frame(res[0].raw) if res else None
        if rec.calls:
            try:
                got = real_parser.parse_line(ln)
                c["e2e"] = [[d.protocol_id, d.payload, d.metadata, M._frame(d.raw)] for d in got]
            except Exception as e:  # noqa: BLE001
                c["e2e_raise"] = type(e).__name__
        cases.append(c)
    path = os.path.join(HERE, "lines_float_golden.json.gz")
    with gzip.open(path, "wt", encoding="utf-8") as f:
        json.dump(cases, f, separators=(",", ":"))
    print(f"wrote {path}: {os.path.getsize(path)} bytes, {len(cases)} lines, "
          f"{sum(len(c.get('e2e', [])) for c in cases)} decoded messages")


if __name__ == "__main__":
    main()
