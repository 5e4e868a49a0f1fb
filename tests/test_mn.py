"""MN (FSK) path: MN_PATTERN parsing, the per-protocol loop of MNParser and the
seven checksum/format methods of sd_protocols/helpers.py.

CPU tests pin the oracle (oracle/mn_oracle.py + the MN rule of oracle/lines_oracle.py) to the
reference's own outputs (tests/golden/mn_golden.json.gz, made by tests/golden/make_mn_golden.py).
GPU tests run the product path -- sdx_parse_lines (MN lines) + sdx_demod_mn through
frontend.SignalParser, and the method / demodulate_mn entry points of SDProtocols -- and compare
with the reference goldens and the oracle, bit-exact."""
import pytest

from oracle import lines_oracle as LO
from oracle import mn_oracle as M
from oracle.sd_oracle import OracleBank


@pytest.fixture(scope="module")
def obank():
    return OracleBank()


def _meta_key(md):
    return sorted((k, v) for k, v in md.items())


def oracle_line(bank, line: bytes, rfmode):
    """End-to-end oracle of SignalParser(rfmode).parse_line for a line (None: not an MN line)."""
    r = LO.parse_line(line)
    if r["status"] == LO.UNSUPPORTED:
        return "unsupported"
    if r["kind"] != LO.MN:
        return None if r["status"] == LO.OK else []
    if r["status"] != LO.OK:
        return []
    res = M.mn_parse(bank, r["data"].decode("ascii"), M.rssi_of(r["R"]), M.afc_of(r["F"]), rfmode)
    pl = r["payload"].decode("latin-1")
    return [[pid, p, md, [pl, "MN", None, None]] for pid, p, md in res]


def test_oracle_lines_match_reference(obank, golden):
    g = golden("mn_golden.json.gz")
    bad, n_mn, n_res, uns = [], 0, 0, 0
    for src, line, rf, exp in g["lines"]:
        got = oracle_line(obank, line.encode("latin-1"), rf)
        if got is None:          # a fuzz mutation that is no MN line any more (covered by test_lines)
            continue
        if got == "unsupported":
            uns += 1
            continue
        assert "raise" not in exp
        n_mn += 1
        n_res += len(got)
        if got != exp["out"]:
            bad.append((src, line, rf, exp["out"][:2], got[:2]))
    assert not bad, f"{len(bad)} mismatches; first: {bad[:2]}"
    assert n_mn > 4000 and n_res > 5000 and uns <= 5, (n_mn, n_res, uns)  # R of > 15 digits (meta_dev)


def test_golden_covers_reference_tests(golden):
    g = golden("mn_golden.json.gz")
    srcs = {c[0] for c in g["lines"]}
    assert {"test", "synth", "fuzz", "edge"} <= srcs
    lines = {c[1] for c in g["lines"]}
    assert "\x02MN;D=DA5A2866AAA290AAAAAA;R=23;A=-2;\x03\n" in lines        # test_mn_bresser_lightning.py
    assert "\x02MN;D=9AA6362CC8AAAA000012F8F4;R=4;\x03\n" in lines          # test_mn_parser.py
    # every MN protocol decodes something, and every method succeeds at least once
    pids = {r[0] for c in g["lines"] if "out" in c[3] for r in c[3]["out"]}
    assert set(g["mn_ids"]) <= pids
    ok_methods = {name for name, d, e in g["methods"] if e.get("out")}
    assert ok_methods == set(M.METHODS)


def test_oracle_methods_match_reference(golden):
    bad, nothex = [], 0
    for name, d, exp in golden("mn_golden.json.gz")["methods"]:
        try:
            got = {"out": M.call_method(name, {"data": d, "protocol_id": "101"})}
        except M.NotHex:
            nothex += 1       # outside the device contract: the data is not hex
            continue
        if got != exp:
            bad.append((name, d, exp, got))
    assert not bad, f"{len(bad)} mismatches; first: {bad[:3]}"
    assert nothex <= 30, nothex


def test_oracle_demodulate_mn_matches_reference(obank, golden):
    bad = []
    for pid, h, exp in golden("mn_golden.json.gz")["demod"]:
        md = {"data": h} if pid is None else {"data": h, "protocol_id": pid}
        got = {"out": M.demodulate_mn(obank, md)}
        if got != exp:
            bad.append((pid, h, exp, got))
    assert not bad, f"{len(bad)} mismatches; first: {bad[:3]}"
