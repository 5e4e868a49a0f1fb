#!/usr/bin/env python3
"""Generate the committed golden vectors from the REFERENCE implementation.

Runs ONLY in the development container, where the read-only reference is
mounted at /root/reference (it never travels to the GPU box).  It imports the
reference's ``sd_protocols`` package (stdlib-only), feeds it

  * every hot-path input the reference's own tests hold (harvested from the
    test files with ``ast`` -- inputs only, the expected outputs are recomputed
    by running the reference),
  * the seeded synthetic corpora of ``pysignalduino_amd.synth`` (configs 2-4),
  * edge cases from SURVEY.md §8(a)/(c),

and writes inputs + outputs as gzipped JSON under tests/golden/.  The fixture
files are data; no reference source is copied.

Usage:  python tests/golden/make_golden.py  [--n-mu 1500 --n-ms 3000 --n-mc 3000]
"""
from __future__ import annotations

import argparse
import ast
import gzip
import json
import os
import random
import sys
import traceback

REF = "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.dont_write_bytecode = True
sys.path.insert(0, REPO)
sys.path.insert(0, REF)

from sd_protocols import SDProtocols  # noqa: E402  (the reference, read-only)
from sd_protocols import pattern_utils as ref_pu  # noqa: E402

from pysignalduino_amd import synth  # noqa: E402


def dump(name, obj):
    path = os.path.join(HERE, name)
    with gzip.open(path, "wt", encoding="utf-8") as f:
        json.dump(obj, f, separators=(",", ":"))
    print(f"wrote {path}: {os.path.getsize(path)} bytes")


def parse_line_dict(line):
    """Same split as the reference parsers' _parse_to_dict (parser/mu.py:82-94)."""
    d = {}
    for part in line.split(";"):
        if not part:
            continue
        if "=" in part:
            k, v = part.split("=", 1)
            d[k] = v
        else:
            d[part] = ""
    if "D" in d:
        d["data"] = d["D"]
    return d


def run_demod(proto, msg, kind):
    try:
        res = proto.demodulate(dict(msg), kind)
    except Exception as e:  # the parsers catch Exception and yield nothing
        return {"raise": type(e).__name__}
    out = []
    for r in res:
        m = r["meta"]
        out.append([r["protocol_id"], r["payload"], m.get("bit_length"), m.get("rssi"), m.get("clock")])
    return {"results": out}


# --------------------------------------------------------------------------------------------
# harvesting inputs from the reference's own tests (inputs only)
# --------------------------------------------------------------------------------------------
def _consts(tree):
    for node in ast.walk(tree):
        if isinstance(node, ast.Constant) and isinstance(node.value, str):
            yield node.value


def harvest_lines(files, prefix):
    out = []
    for fn in files:
        tree = ast.parse(open(os.path.join(REF, "tests", fn)).read())
        for s in _consts(tree):
            if s.startswith(prefix) and s not in out:
                out.append(s)
    return out


def _eval_bits(node):
    if isinstance(node, ast.List) and all(isinstance(e, ast.Constant) and isinstance(e.value, int) for e in node.elts):
        return [e.value for e in node.elts]
    if isinstance(node, ast.BinOp) and isinstance(node.op, ast.Mult):
        left = _eval_bits(node.left)
        if left is not None and isinstance(node.right, ast.Constant):
            return left * node.right.value
    return None


def harvest_postdemo():
    tree = ast.parse(open(os.path.join(REF, "tests", "test_postdemodulation.py")).read())
    names = {n.lower(): n for n in dir(SDProtocols) if n.startswith("postDemo_")}
    cases = []
    for cls in [n for n in tree.body if isinstance(n, ast.ClassDef) and n.name.startswith("TestPostDemo")]:
        meth = names.get("postdemo_" + cls.name[len("TestPostDemo"):].lower())
        for node in ast.walk(cls):
            if isinstance(node, ast.Assign) and any(isinstance(t, ast.Name) and t.id == "bits" for t in node.targets):
                bits = _eval_bits(node.value)
                if bits is not None and meth:
                    cases.append((meth, bits))
    return cases


def harvest_bitstrings(fn):
    tree = ast.parse(open(os.path.join(REF, "tests", fn)).read())
    out = []
    for s in _consts(tree):
        if len(s) >= 4 and set(s) <= {"0", "1"} and s not in out:
            out.append(s)
    return out


# --------------------------------------------------------------------------------------------
def mu_ms_cases(proto, P, n_mu, n_ms):
    mu_lines = harvest_lines(["test_mu_demodulation.py", "test_mu_parser.py"], "MU;")
    ms_lines = harvest_lines(["test_ms_demodulation.py", "test_ms_parser.py"], "MS;")
    mu, ms = [], []
    for ln in mu_lines:
        d = parse_line_dict(ln)
        mu.append({"src": "reftest", "msg": d, "exp": run_demod(proto, d, "MU")})
    for ln in ms_lines:
        d = parse_line_dict(ln)
        ms.append({"src": "reftest", "msg": d, "exp": run_demod(proto, d, "MS")})
    # config 1: tests/test_ms_demodulation.py:31-41
    cfg1 = {"P0": "330", "P1": "-14520", "P2": "-1254", "P3": "1155", "P4": "-330",
            "data": "01" + "02" * 23 + "34", "CP": "0", "SP": "0", "R": "0"}
    ms.append({"src": "config1", "msg": cfg1, "exp": run_demod(proto, cfg1, "MS")})

    # edge cases
    edges_mu = [
        {"P0": "315", "P1": "-283", "P2": "-1197", "P3": "630", "P4": "-567",
         "data": "0102010201020103" + "0403" * 20, "CP": "0"},                    # id 31 path
        {"P0": "-3000", "P1": "800", "data": "0101", "CP": "1"},                 # half-even
        {"P0": "-250", "P1": "250", "data": "", "CP": "1"},                       # empty data
        {"P0": "400", "P1": "-800", "P2": "-400", "P3": "-3200",
         "data": "01" * 30 + "02" * 30 + "03" + "0102" * 40, "CP": "0", "R": "abc"},  # float + id 82
        {"P01": "500", "P1": "-1000", "P2": "1500", "P3": "-500", "data": "1213121312131312" * 8, "CP": "1"},
        {"P0": "x", "P1": "500", "P2": "-1000", "data": "1212121212", "CP": "1"},
        {"P0": "1e3", "P1": " -500 ", "P2": "nan", "P3": "inf", "data": "0101010123", "CP": "0"},
    ]
    for d in edges_mu:
        d = dict(d)
        mu.append({"src": "edge", "msg": d, "exp": run_demod(proto, d, "MU")})
    edges_ms = [
        {"P0": "500", "P1": "-5000", "P2": "-1000", "P3": "-2000", "data": "01" + "02" * 20 + "0", "CP": "0", "SP": "1"},
        {"P0": "500", "P1": "-5000", "data": "0101", "CP": "7", "SP": "1"},       # CP missing
        {"P0": "0", "P1": "-5000", "data": "0101", "CP": "0", "SP": "1"},         # clock 0
        {"P0": "500", "P1": "-5000", "data": "01a1", "CP": "0", "SP": "1"},       # not digits
        {"P0": "500", "P1": "-5000", "data": "0101", "CP": "x", "SP": "1"},
        {"P0": "500", "P1": "-5000", "data": "0101", "CP": "0", "SP": "1", "R": "1q"},
    ]
    for d in edges_ms:
        ms.append({"src": "edge", "msg": d, "exp": run_demod(proto, d, "MS")})

    mub = synth.mu_corpus(P, n_mu, seed=42)
    for i in range(mub.n):
        d = mub.to_msg_dict(i)
        mu.append({"src": "synth42", "msg": d, "exp": run_demod(proto, d, "MU")})
    msb = synth.ms_corpus(P, n_ms, seed=43)
    for i in range(msb.n):
        d = msb.to_msg_dict(i)
        ms.append({"src": "synth43", "msg": d, "exp": run_demod(proto, d, "MS")})
    return mu, ms


# --------------------------------------------------------------------------------------------
def mc_fixed_reference(proto, pid, raw_hex, clock, mcbitnum, messagetype, version):
    """The reference's MC chain with the two SURVEY §8(a) A7 fixes applied.

    Composes the reference's own functions: the length gates and polarity logic of
    manchester.py:70-96, _convert_mc_hex_to_bits (:18-47) and the protocol method
    (:112-120) called WITHOUT the extra positional ``self`` (fix 2), with the
    clockrange compare done on clockrange[0]/[1] (fix 1).
    """
    length_min = int(proto.check_property(pid, "length_min", -1))
    if mcbitnum < length_min:
        return None
    length_max = int(proto.check_property(pid, "length_max", 9999))
    if mcbitnum > length_max:
        return None
    cr = proto.get_property(pid, "clockrange")
    if cr and len(cr) >= 2:
        if not (clock > cr[0] and clock < cr[1]):
            return None
    inv = proto.check_property(pid, "polarity", "") == "invert"
    if messagetype == "Mc" or (version and version[:6] == "V 3.2."):
        inv = inv ^ 1
    rc, bits = proto._convert_mc_hex_to_bits("n", raw_hex, inv, len(raw_hex))
    if rc == -1:
        return None
    mname = proto.get_property(pid, "method").split(".")[-1]
    fn = getattr(proto, mname)
    rc, res = fn(f"Protocol {pid}", bits, pid, len(bits))
    if rc == -1:
        return None
    pre = proto.check_property(pid, "preamble", "")
    return [pid, f"{pre}{res}"]


def mc_cases(proto, P, n_mc):
    mcb = synth.mc_corpus(P, n_mc, seed=44)
    mc_ids = [pid for pid, p in P.items() if "clockrange" in p]
    frames = []
    for i in range(mcb.n):
        hx = mcb.hex(i)
        clock, L = int(mcb.clock[i]), int(mcb.mcbitnum[i])
        mt = "MC" if mcb.mtype[i] == 0 else "Mc"
        ver = "V 3.2.0" if mcb.v32[i] else None
        fixed = []
        raised = None
        for pid in mc_ids:
            try:
                r = mc_fixed_reference(proto, pid, hx, clock, L, mt, ver)
            except Exception as e:
                raised = type(e).__name__
                break
            if r is not None:
                fixed.append(r)
        strict = []
        for pid in mc_ids:  # reference-observable behaviour (direct demodulate_mc call)
            try:
                res = proto.demodulate_mc({"protocol_id": pid, "data": hx, "clock": clock, "bit_length": L}, mt,
                                          version=ver)
                strict.append(["ok", [[r["protocol_id"], r["payload"]] for r in res]])
            except Exception as e:
                strict.append(["raise", type(e).__name__])
        frames.append({"hex": hx, "clock": clock, "L": L, "mtype": mt, "version": ver,
                       "fixed": {"raise": raised} if raised else {"results": fixed}, "strict": strict})
    return frames


# --------------------------------------------------------------------------------------------
def unit_cases(proto, P):
    rnd = random.Random(7)
    units = {}
    # pattern_exists: the reference test vectors + randomised tables
    pe = [
        ([1, -1], {"0": 1.0, "1": -1.0}, "0101"), ([10, -5], {"0": 11.0, "1": -4.0}, "01"),
        ([1], {"0": 20.0}, "0"), ([1], {"0": 1.0}, "222"), ([1, 2], {"0": 1.5}, "00"),
        ([1, 1], {"0": 1.0}, "00"), ([1], {"0": 1.0, "1": 1.1}, "1"),
    ]
    vals = [-40.0, -31.0, -14.0, -10.0, -8.0, -5.0, -4.0, -3.8, -3.0, -2.0, -1.8, -1.5, -1.2, -1.0, -0.9,
            0.0, 0.9, 1.0, 1.2, 1.5, 2.0, 3.0, 3.5, 4.0, 5.0, 6.0, 10.0, 17.0, 25.0]
    for _ in range(3000):
        npat = rnd.randint(1, 8)
        ids = rnd.sample("0123456789", npat)
        table = {k: round(rnd.choice(vals) * rnd.uniform(0.7, 1.3), 1) for k in ids}
        search = [rnd.choice(vals) for _ in range(rnd.randint(1, 6))]
        data = "".join(rnd.choice(ids) for _ in range(rnd.randint(0, 40)))
        pe.append((search, table, data))
    # combinatorial explosion (>10000) case
    pe.append(([1, 2, 3, 4, 5], {str(i): 3.0 for i in range(10)}, "0123456789"))
    units["pattern_exists"] = [[s, t, d, ref_pu.pattern_exists(s, t, d)] for s, t, d in pe]

    # round(x, 1) half-even on the exact double
    rq = []
    for _ in range(20000):
        a = rnd.choice([rnd.randint(-99999, 99999), rnd.uniform(-1e5, 1e5)])
        b = rnd.choice([rnd.randint(1, 2000), -1, rnd.uniform(0.5, 1500)])
        rq.append([a, b, round(a / b, 1)])
    for a, b in [(-3000, 800), (25, 100), (75, 100), (5, 100), (15, 100), (-25, 100), (1, 20), (3, 20)]:
        rq.append([a, b, round(a / b, 1)])
    units["round1"] = rq

    # helpers
    bs = []
    for _ in range(2000):
        n = rnd.randint(0, 70)
        s = "".join(rnd.choice("01") for _ in range(n))
        if rnd.random() < 0.05 and n:
            s = s[:n // 2] + "F" + s[n // 2 + 1:]
        bs.append([s, proto.bin_str_2_hex_str(s)])
    units["bin_str_2_hex_str"] = bs
    hx = []
    for _ in range(2000):
        s = "".join(rnd.choice("0123456789ABCDEFabcdef") for _ in range(rnd.randint(1, 30)))
        if rnd.random() < 0.2:
            s = "0" * rnd.randint(1, 4) + s
        hx.append([s, proto.hex_to_bin_str(s)])
    hx += [[s, proto.hex_to_bin_str(s)] for s in ["0", "00", "0000", "000F", "F", "g"]]
    units["hex_to_bin_str"] = hx
    units["mc2dmc"] = [[s, proto.mc2dmc(s)] for s in ["1001", "", "1", "0110", "111000"] +
                       ["".join(rnd.choice("01") for _ in range(rnd.randint(0, 80))) for _ in range(300)]]
    lir = []
    for pid in list(P.keys()):
        for n in [0, 1, 8, 12, 24, 32, 40, 64, 100, 200]:
            lir.append([pid, n, list(proto.length_in_range(pid, n))])
    lir.append(["nope", 5, list(proto.length_in_range("nope", 5))])
    units["length_in_range"] = lir

    # postDemo_*: harvested reference-test vectors, mutations, random lists
    pdm = []
    harvested = harvest_postdemo()
    for meth, bits in harvested:
        pdm.append([meth, bits])
        for _ in range(30):
            b = list(bits)
            r = rnd.random()
            if r < 0.4 and b:
                i = rnd.randrange(len(b))
                b[i] ^= 1
            elif r < 0.7:
                b = [0] * rnd.randint(0, 4) + b
            elif b:
                b = b[rnd.randint(0, min(3, len(b) - 1)):]
            pdm.append([meth, b])
    methods = sorted({m for m, _ in harvested})
    for meth in methods:
        for _ in range(200):
            pdm.append([meth, [rnd.randint(0, 1) for _ in range(rnd.randint(0, 130))]])
    outp = []
    for meth, bits in pdm:
        try:
            rc, ret = getattr(proto, meth)("Protocol_x", list(bits))
            outp.append([meth, bits, "ok", rc, ret])
        except Exception as e:
            outp.append([meth, bits, "raise", type(e).__name__, None])
    units["postdemo"] = outp

    # MC protocol methods on bit strings (direct calls, as the reference tests do)
    mc_ids = [pid for pid, p in P.items() if "clockrange" in p]
    bitstrs = harvest_bitstrings("test_manchester_protocols.py")
    for _ in range(150):
        bitstrs.append("".join(rnd.choice("01") for _ in range(rnd.randint(8, 230))))
    # planted TFA duplicates / Sainlogic / AS sync patterns
    for _ in range(60):
        body = "".join(rnd.choice("01") for _ in range(rnd.randint(40, 60)))
        bitstrs.append("1" * 9 + "101" + "0" + body + "1111111111101" + body + "11")
        bitstrs.append("0" * rnd.randint(0, 8) + "010100" + "".join(rnd.choice("01") for _ in range(110)))
        bitstrs.append("0" * 16 + "1100" + "".join(rnd.choice("01") for _ in range(rnd.randint(40, 80))))
    mcm = []
    for pid in mc_ids:
        mname = P[pid]["method"].split(".")[-1]
        fn = getattr(proto, mname)
        for s in bitstrs:
            try:
                rc, res = fn("n", s, pid, len(s))
                mcm.append([pid, s, "ok", rc, res])
            except Exception as e:
                mcm.append([pid, s, "raise", type(e).__name__, None])
    units["mc_methods"] = mcm
    return units


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n-mu", type=int, default=1500)
    ap.add_argument("--n-ms", type=int, default=3000)
    ap.add_argument("--n-mc", type=int, default=3000)
    args = ap.parse_args()
    proto = SDProtocols()
    P = proto.get_protocol_list()
    bank_ours = json.load(open(os.path.join(REPO, "pysignalduino_amd", "data", "sd_bank.json")))["protocols"]
    ref_raw = json.load(open(os.path.join(REF, "sd_protocols", "protocols.json")))["protocols"]
    assert bank_ours == ref_raw, "pysignalduino_amd/data/sd_bank.json drifted from the reference bank"
    mu, ms = mu_ms_cases(proto, ref_raw, args.n_mu, args.n_ms)
    dump("mu_golden.json.gz", mu)
    dump("ms_golden.json.gz", ms)
    dump("mc_golden.json.gz", mc_cases(proto, ref_raw, args.n_mc))
    dump("units_golden.json.gz", unit_cases(proto, ref_raw))


if __name__ == "__main__":
    main()
