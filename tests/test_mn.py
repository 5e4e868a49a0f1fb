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


# ---------------------------------------------------------------------------------- GPU ------
def _flat(msgs):
    return [[d.protocol_id, d.payload, d.metadata, [d.raw.line, d.raw.message_type, d.raw.rssi, d.raw.freq_afc]]
            for d in msgs]


@pytest.mark.gpu
def test_gpu_signal_parser_matches_reference(golden):
    """Framed MN lines (reference tests, synthetic, fuzzed, edge cases) through the device front
    end + sdx_demod_mn == the reference's SignalParser(rfmode).parse_line, bit-exact."""
    from pysignalduino_amd.frontend import SignalParser
    from pysignalduino_amd.packing import ContractError
    from pysignalduino_amd.sd_protocols import SDProtocols
    cases = golden("mn_golden.json.gz")["lines"]
    proto = SDProtocols()
    by_rf = {}
    for k, (src, line, rf, exp) in enumerate(cases):
        by_rf.setdefault(rf, []).append(k)
    bad, nres, ncontract = [], 0, 0
    for rf, ks in by_rf.items():
        got = SignalParser(proto, rfmode=rf).parse_lines([cases[k][1] for k in ks])
        for k, g in zip(ks, got):
            src, line, _, exp = cases[k]
            if isinstance(g, ContractError):
                ncontract += 1
                assert LO.parse_line(line.encode("latin-1"))["status"] == LO.UNSUPPORTED, line
                continue
            assert not isinstance(g, BaseException), (line, g)
            e = exp.get("out", [])
            nres += len(e)
            if _flat(g) != e:
                bad.append((src, line[:90], rf, e[:2], _flat(g)[:2]))
    assert not bad, f"{len(bad)} mismatches; first: {bad[:2]}"
    assert nres > 5000 and ncontract <= 5, (nres, ncontract)


@pytest.mark.gpu
def test_gpu_mn_parser_frames(golden):
    """frontend.MNParser.parse_batch on RawFrames (payloads) == the reference."""
    from pysignalduino_amd.frontend import MNParser, RawFrame
    from pysignalduino_amd.sd_protocols import SDProtocols
    cases = [c for c in golden("mn_golden.json.gz")["lines"] if c[0] in ("test", "synth") and c[2] is None]
    frames = [RawFrame(line=c[1].strip()[1:-1], message_type="MN") for c in cases]
    got = MNParser(SDProtocols(), rfmode=None).parse_batch(frames)
    for c, fr, g in zip(cases, frames, got):
        exp = [[x[0], x[1], x[2]] for x in c[3]["out"]]
        assert [[d.protocol_id, d.payload, d.metadata] for d in g] == exp, c[1]
        assert all(d.raw is fr for d in g)


@pytest.mark.gpu
def test_gpu_methods_match_reference(golden):
    """SDProtocols.ConvX (method mode of sdx_demod_mn), batched per method, == the reference."""
    from pysignalduino_amd.packing import ContractError
    from pysignalduino_amd.sd_protocols import SDProtocols
    proto = SDProtocols()
    by_m = {}
    for name, d, exp in golden("mn_golden.json.gz")["methods"]:
        by_m.setdefault(name, []).append((d, exp))
    n = 0
    for name, items in by_m.items():
        ok = [(d, e) for d, e in items if d == "" or not set(d) - set("0123456789abcdefABCDEF")]
        got = proto.mn_method_batch([{"data": d, "protocol_id": "101"} for d, _ in ok], name)
        for (d, e), g in zip(ok, got):
            assert {"out": g} == e, (name, d, e, g)
            n += 1
        for d, e in items:
            if (d, e) not in ok:
                with pytest.raises(ContractError):
                    getattr(proto, name)({"data": d, "protocol_id": "101"}, "MN")
    assert n > 5000
    # single-call entry point == batch
    d = "9AA6362CC8AAAA000012F8F4"
    assert proto.ConvLaCrosse({"data": d, "protocol_id": "100"}) == \
        [{"protocol_id": "100", "payload": "OK 9 42 129 4 212 44", "meta": {"is_raw": False}}]


@pytest.mark.gpu
def test_gpu_demodulate_mn_matches_reference(golden):
    from pysignalduino_amd.sd_protocols import SDProtocols
    proto = SDProtocols()
    for pid, h, exp in golden("mn_golden.json.gz")["demod"][:3000]:
        md = {"data": h} if pid is None else {"data": h, "protocol_id": pid}
        assert {"out": proto.demodulate(md, "MN")} == exp, (pid, h)


@pytest.mark.gpu
def test_gpu_large_corpus_vs_oracle(obank):
    """120k synthetic MN lines (every rfmode setting) vs the oracle, and overflow-free output."""
    from pysignalduino_amd import synth
    from pysignalduino_amd.frontend import SignalParser
    from pysignalduino_amd.sd_protocols import SDProtocols
    frames = synth.mn_frames(120_000, seed=99)
    lines = [synth.frame(synth.mn_payload(*f)) for f in frames]
    proto = SDProtocols()
    for rf in (None, "Lacrosse_mode1", "Bresser_7in1"):
        got = SignalParser(proto, rfmode=rf).parse_lines(lines[:60_000] if rf else lines)
        nres = 0
        for ln, g in zip(lines, got):
            exp = oracle_line(obank, ln, rf)
            assert _flat(g) == exp, (ln, rf)
            nres += len(g)
        assert nres > (150_000 if rf is None else 1000), nres


@pytest.mark.gpu
def test_gpu_mixed_stream_with_mn():
    """MU/MS/MC/MN lines interleaved in one batch: MN results land on their lines."""
    from pysignalduino_amd import synth
    from pysignalduino_amd import bank as B
    from pysignalduino_amd.frontend import SignalParser
    P = B.Bank().protocols
    base, _ = synth.line_corpus(P, 3000, seed=5)
    mn = [synth.frame(synth.mn_payload(*f)) for f in synth.mn_frames(3000, seed=6)]
    mixed = [x for pair in zip(base, mn) for x in pair]
    sp = SignalParser()
    got = sp.parse_lines(mixed)
    alone_mn = sp.parse_lines(mn)
    alone_base = sp.parse_lines(base)
    assert [_flat(g) for g in got[1::2]] == [_flat(g) for g in alone_mn]
    assert [_flat(g) if not isinstance(g, Exception) else type(g) for g in got[0::2]] == \
        [_flat(g) if not isinstance(g, Exception) else type(g) for g in alone_base]


def test_checksum_tables_match_the_bit_serial_oracle():
    """bank.mn_tables (k_mn's LDS tables) reproduce lfsr_digest16 / _calc_crc16 / the LaCrosse CRC-8."""
    import numpy as np
    from pysignalduino_amd import bank as B
    t = B.mn_tables()
    c1021 = np.frombuffer(t[0:512], np.uint16)
    c8005 = np.frombuffer(t[512:1024], np.uint16)
    c31 = np.frombuffer(t[1024:1280], np.uint8)
    l8 = np.frombuffer(t[1280:1792], np.uint16).reshape(16, 16)
    l21 = np.frombuffer(t[1792:3136], np.uint16).reshape(42, 16)
    rng = np.random.default_rng(5)
    for _ in range(300):
        d = [int(x) for x in rng.integers(0, 256, size=21)]
        s = "".join("%02X" % x for x in d)
        for T, nb, key in ((l21, 21, 0xBA95), (l8, 8, 0xABF9)):
            acc = 0
            for k in range(nb):
                acc ^= int(T[2 * k][d[k] >> 4]) ^ int(T[2 * k + 1][d[k] & 15])
            assert acc == M.lfsr16(nb, 0x8810, key, s[:2 * nb])
        for T, poly, nb in ((c1021, 0x1021, 15), (c8005, 0x8005, 10)):
            c = 0
            for k in range(nb):
                c = ((c << 8) & 0xFFFF) ^ int(T[((c >> 8) ^ d[k]) & 0xFF])
            assert c == M.crc16(s[:2 * nb], poly)
        c = 0
        for k in range(4):
            c = int(c31[c ^ d[k]])
        ref = 0
        for k in range(4):
            ref ^= d[k]
            for _ in range(8):
                ref = ((ref << 1) ^ 0x31) & 0xFF if ref & 0x80 else (ref << 1) & 0xFF
        assert c == ref
