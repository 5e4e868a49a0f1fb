#!/usr/bin/env python3
"""Golden lines for the front end's general path (SDX_LS_GENERAL, include/sdx.h), recorded from the
REFERENCE's own SignalParser (record format of make_lines_golden.py; development container only).

Synthetic MU/MS lines (pysignalduino_amd/synth.py line_corpus, plain and Mred=1-compressed) with
pattern ids renamed to multi-digit ones (P10, P007, ...; the D characters rewritten to the new id
strings, or not), extra multi-digit patterns, more than 16 patterns or 16-digit ids (outside the
contract), and D fields repeated past 4096 pulses.

Usage:  python tests/golden/make_lines_general_golden.py
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


def variants(s: str, rng) -> str:
    keys = re.findall(r";P(\d)=(-?\d+)", s)
    mode = int(rng.integers(0, 6))
    if mode in (0, 1) and keys:  # rename one or two ids; data rewritten (0) or not (1)
        ren = {}
        for k, _ in [keys[int(x)] for x in rng.permutation(len(keys))[: int(rng.integers(1, 3))]]:
            ren[k] = [str(10 + int(k)), "1" + k, k + k, "00" + k][int(rng.integers(0, 4))]
        for k, new in ren.items():
            s = s.replace(f";P{k}=", f";P{new}=", 1)
        if mode == 0:
            m = re.search(r";D=(\d+);", s)
            if m:
                d2 = "".join(ren.get(c, c) for c in m.group(1))
                s = s[: m.start(1)] + d2 + s[m.end(1):]
        for key in ("CP", "SP"):
            m = re.search(rf";{key}=(\d);", s)
            if m and m.group(1) in ren and rng.random() < 0.7:
                s = s[: m.start(1)] + ren[m.group(1)] + s[m.end(1):]
    elif mode == 2 and keys:  # extra multi-digit patterns near existing values
        for t in range(int(rng.integers(1, 5))):
            k, v = keys[int(rng.integers(0, len(keys)))]
            s = s.replace(";D=", f";P{10 + t * 7}={int(int(v) * float(rng.uniform(0.9, 1.1)))};D=", 1)
    elif mode == 3:  # outside the general contract: 17 patterns / a 16-digit id
        if rng.random() < 0.5:
            s = s.replace(";D=", "".join(f";P{20 + t}={100 * (t + 1)}" for t in range(17)) + ";D=", 1)
        else:
            s = s.replace(";D=", ";P1234567890123456=500;D=", 1)
    if mode in (4, 5) or rng.random() < 0.15:  # D past 4096 pulses
        m = re.search(r";D=(\d+);", s)
        if m:
            d = m.group(1)
            d2 = d * (4100 // max(1, len(d)) + 1 + int(rng.integers(0, 3)))
            s = s[: m.start(1)] + d2 + s[m.end(1):]
    return s


def main():
    protos = M.B.Bank().protocols
    corpus, _ = M.synth.line_corpus(protos, 700, seed=91, compress_frac=0.0, mu_npulse=128, mix=(0.5, 0.5, 0.0))
    rng = np.random.default_rng(92)
    lines = [("general", variants(ln.decode("latin-1"), rng)) for ln in corpus]
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
    path = os.path.join(HERE, "lines_general_golden.json.gz")
    with gzip.open(path, "wt", encoding="utf-8") as f:
        json.dump(cases, f, separators=(",", ":"))
    print(f"wrote {path}: {os.path.getsize(path)} bytes, {len(cases)} lines, "
          f"{sum(len(c.get('e2e', [])) for c in cases)} decoded messages")


if __name__ == "__main__":
    main()
