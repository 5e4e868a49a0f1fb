"""Wire-line front end: sdx_parse_lines / sdx_select_lines / frontend.SignalParser.

CPU tests pin the oracle (oracle/lines_oracle.py) to what the reference parser did on the same
lines (tests/golden/lines_golden.json.gz, made by tests/golden/make_lines_golden.py).  GPU tests
compare the device outputs with the oracle field by field (bit-exact) and the end-to-end
DecodedMessage lists with the reference's own (the "e2e" records of the goldens)."""
import numpy as np
import pytest

from oracle import lines_oracle as LO
from pysignalduino_amd import bank as B
from pysignalduino_amd import synth

TYPE = {LO.MU: "MU", LO.MS: "MS", LO.MC: "MC"}


GOLDENS = ["lines_golden.json.gz", "lines_float_golden.json.gz",   # P# values in float() syntax
           "lines_general_golden.json.gz"]                           # multi-digit ids, > 4096 pulses


def _lines(golden, fname="lines_golden.json.gz"):
    return [c["line"].encode("latin-1") for c in golden(fname)]


def test_oracle_char_classes_are_pythons():
    for c in range(256):
        ch = chr(c)
        assert (c in LO._WS) == ch.isspace(), c
        assert LO._alpha(c) == ch.isalpha(), c


@pytest.mark.parametrize("fname", GOLDENS)
def test_oracle_matches_reference_goldens(golden, fname):
    cases = golden(fname)
    unsupported = 0
    bad = []
    for c in cases:
        assert "raise" not in c
        r = LO.parse_line(c["line"].encode("latin-1"))
        if r["status"] == LO.UNSUPPORTED:
            unsupported += 1
            continue
        exp_payload = c["payload"]
        got_payload = None if r["payload"] is None else r["payload"].decode("latin-1")
        ok = exp_payload == got_payload
        if r["status"] in (LO.OK, LO.RAISES, LO.GENERAL) and r["kind"] != LO.MN:  # MNParser calls no demodulator
            ok = ok and c["calls"] == [[TYPE[r["kind"]], [list(kv) for kv in r["msg"]]]]
            fr = c["frame"]
            ok = ok and fr is not None and fr[0] == got_payload and fr[1] == TYPE[r["kind"]] \
                and fr[2] == r["rssi"] and fr[3] == r["freq_afc"]
        else:
            ok = ok and c["calls"] == []
        if not ok:
            bad.append((c["src"], c["line"], r["status"], c["calls"][:1], r.get("msg")))
    assert not bad, f"{len(bad)} mismatches; first: {bad[:3]}"
    assert unsupported <= (0.05 if fname == GOLDENS[0] else 0.15) * len(cases), unsupported
    if fname != GOLDENS[0]:
        return
    # the goldens cover every status the front end reports
    st = {LO.parse_line(c["line"].encode("latin-1"))["status"] for c in cases}
    assert st >= {LO.OK, LO.NOFRAME, LO.NOPARSER, LO.INVALID, LO.NODATA, LO.UNSUPPORTED, LO.RAISES}


def test_reference_test_vectors_present(golden):
    """The reference's own parser/decompression test inputs are in the fixture."""
    srcs = {c["src"].split(":")[0] for c in golden("lines_golden.json.gz")}
    assert {"test_mu_parser.py", "test_ms_parser.py", "test_mc_parser.py", "test_decompress_payload.py"} <= srcs


def test_synth_lines_roundtrip():
    """Compressed and plain synthetic lines parse back to the generating message (oracle)."""
    P = B.Bank().protocols
    lines, kinds = synth.line_corpus(P, 600, seed=7, compress_frac=0.5, mu_npulse=64)
    ok = {LO.MU: 0, LO.MS: 0, LO.MC: 0}
    for ln, k in zip(lines, kinds):
        r = LO.parse_line(ln)
        assert r["status"] in (LO.OK, LO.INVALID), (ln, r["status"])
        if r["status"] == LO.OK:
            ok[r["kind"]] += 1
            assert r["kind"] == [LO.MU, LO.MS, LO.MC][k]
    assert ok[LO.MU] > 150 and ok[LO.MS] > 150 and ok[LO.MC] > 80, ok


def test_pack_lines_bulk_and_per_line_forms_agree():
    """frontend.pack_lines: the bulk form for all-str batches (one join + one latin-1 encode) gives the
    bytes and offsets of the per-line form; a character above U+00FF marks exactly its own line
    (ContractError, replaced by an empty line) and leaves the others' bytes."""
    from pysignalduino_amd.frontend import pack_lines
    from pysignalduino_amd.packing import ContractError
    lines = ["\x02MU;P0=-1000;P1=500;D=0101;CP=1;\x03", "", "MS;P0=1;D=\xb5\xff;", "x" * 300]
    d, o, bad = pack_lines(lines)
    mixed = [ln.encode("latin-1") for ln in lines[:2]] + lines[2:]            # bytes + str: per-line form
    d2, o2, bad2 = pack_lines(mixed)
    assert not bad and not bad2 and d.tobytes() == d2.tobytes() and o.tolist() == o2.tolist()
    cum = [0]
    for ln in lines:
        cum.append(cum[-1] + len(ln))
    assert d.tobytes() == "".join(lines).encode("latin-1") and o.tolist() == cum
    d3, o3, bad3 = pack_lines(lines[:2] + ["P\u0100"] + lines[2:], copy=False)
    assert list(bad3) == [2] and isinstance(bad3[2], ContractError)
    assert d3.tobytes() == "".join(lines).encode("latin-1") and o3.tolist() == cum[:3] + cum[2:]
    assert pack_lines([])[1].tolist() == [0]


def test_compressed_payload_decompresses_to_the_plain_one():
    P = B.Bank().protocols
    pb = synth.ms_corpus(P, 200, seed=3)
    n = 0
    for i in range(pb.n):
        c = synth.compress_pulse_payload(pb, i)
        if c is None:
            continue
        plain = synth.pulse_payload(pb, i)
        got = dict(LO._kv(LO.decompress(c)))
        exp = dict(LO._kv(plain))
        # the firmware's compressed form carries the same fields (type spelled "Ms" -> "MS")
        assert got == exp, (plain, c)
        n += 1
    assert n > 50


# ---------------------------------------------------------------------------------- GPU ------
def _fuzz(lines, n, seed):
    rng = np.random.default_rng(seed)
    out = []
    for _ in range(n):
        m = synth.mutate_line(rng, lines[int(rng.integers(0, len(lines)))])
        if rng.random() < 0.4:
            m = synth.mutate_line(rng, m)
        out.append(m)
    return out


def _device_parse(lines):
    from pysignalduino_amd import frontend, runtime
    from pysignalduino_amd.sd_protocols import SDProtocols
    p = SDProtocols()
    eng = p._ensure()
    data, offsets, bad = frontend.pack_lines(lines)
    assert not bad
    lb = frontend.LineBatch(eng, data, offsets)
    lb.launch()
    sels, cnt = lb.selections()
    n = len(lines)
    g = lambda t, k=n: t[:k].cpu().numpy()  # noqa: E731
    return dict(kind=g(lb.kind), status=g(lb.status), doff=g(lb.doff), dlen=g(lb.dlen), npat=g(lb.npat),
                pat_id=g(lb.pat_id, 10 * n).reshape(n, 10), pat_val=g(lb.pat_val, 10 * n).reshape(n, 10),
                cp_slot=g(lb.cp_slot), ms_ok=g(lb.ms_ok), clock=g(lb.clock), mcbitnum=g(lb.mcbitnum),
                mcflags=g(lb.mcflags), meta=g(lb.meta, 32 * n).reshape(n, 32), plen=g(lb.plen),
                slot=lb.slot.cpu().numpy(), offsets=offsets,
                sels=[s.cpu().numpy() for s in sels], counts=cnt, runtime=runtime)


def _meta(m, base):
    ln = int(m[base + 15])
    return None if ln == 255 else bytes(m[base: base + ln])


def _compare(lines, dv):
    bad = []
    for i, ln in enumerate(lines):
        r = LO.parse_line(ln)
        e = []
        dst = int(dv["status"][i])
        if dst == LO.GENERAL and r.get("gen_contract"):
            dst = LO.UNSUPPORTED  # sdx_lines_general reports these (test_lines_general_batch_matches_oracle)
        if int(dv["kind"][i]) != r["kind"] or dst != r["status"]:
            e.append(("kind/status", int(dv["kind"][i]), int(dv["status"][i]), r["kind"], r["status"]))
        elif r["status"] in (LO.OK, LO.GENERAL):
            s0 = int(dv["doff"][i])
            d = bytes(dv["slot"][s0: s0 + int(dv["dlen"][i])])
            if d != r["data"]:
                e.append(("data", d[:40], r["data"][:40]))
            if _meta(dv["meta"][i], 0) != r["R"] or _meta(dv["meta"][i], 16) != r["F"]:
                e.append(("meta", _meta(dv["meta"][i], 0), r["R"], _meta(dv["meta"][i], 16), r["F"]))
            if int(dv["plen"][i]) != r["plen"]:
                e.append(("plen", int(dv["plen"][i]), r["plen"]))
            elif r["plen"] >= 0:
                s0 = 3 * int(dv["offsets"][i])
                if bytes(dv["slot"][s0: s0 + r["plen"]]) != r["payload"]:
                    e.append(("payload",))
            if r["kind"] == LO.MC:
                if (int(dv["clock"][i]), int(dv["mcbitnum"][i]), int(dv["mcflags"][i])) != \
                        (r["clock"], r["mcbitnum"], r["mcflags"]):
                    e.append(("mc", int(dv["clock"][i]), int(dv["mcbitnum"][i]), r["clock"], r["mcbitnum"]))
            elif r["kind"] != LO.MN and r["status"] == LO.OK:
                npat = int(dv["npat"][i])
                ids = [int(chr(c)) for c in dv["pat_id"][i][:npat]]
                vals = dv["pat_val"][i][:npat]
                if ids != r["ids"] or vals.tobytes() != np.array(r["vals"], np.float64).tobytes():  # bitwise: -0.0
                    e.append(("patterns", ids, vals, r["ids"], r["vals"]))
                if r["kind"] == LO.MS and (int(dv["ms_ok"][i]) != r["ms_ok"] or
                                           (r["ms_ok"] and int(dv["cp_slot"][i]) != r["cp_slot"])):
                    e.append(("ms", int(dv["ms_ok"][i]), int(dv["cp_slot"][i]), r["ms_ok"], r["cp_slot"]))
        if e:
            bad.append((i, ln[:80], e))
    return bad


def _check_selection(lines, dv):
    classes = [LO.sel_class(LO.parse_line(ln)) for ln in lines]
    for k in range(7):
        exp = [i for i, c in enumerate(classes) if c == k]
        assert int(dv["counts"][k]) == len(exp), k
        assert list(dv["sels"][k]) == exp, k


@pytest.mark.gpu
@pytest.mark.parametrize("fname", GOLDENS)
def test_parse_lines_matches_oracle_on_goldens(golden, fname):
    lines = _lines(golden, fname)
    dv = _device_parse(lines)
    bad = _compare(lines, dv)
    assert not bad, f"{len(bad)} mismatches; first: {bad[:3]}"
    _check_selection(lines, dv)


@pytest.mark.gpu
def test_parse_lines_matches_oracle_fuzz():
    P = B.Bank().protocols
    base, _ = synth.line_corpus(P, 4000, seed=11, compress_frac=0.4)
    base += [synth.frame(synth.mn_payload(*f)) for f in synth.mn_frames(1500, seed=13)]
    base += [b"\x02MN;D=" + b"A" * k + b";R=7;\x03" for k in (4095, 4096, 4097)]
    lines = base + _fuzz(base, 30000, seed=12) + [b"", b"\x02\x03", b"\x02MU;;\x03", b" \x02MC;;\x03 ",
                                                  b"\x02Ms;\x80;\x03", b"\x02MN;D=AB;\x03"]
    dv = _device_parse(lines)
    bad = _compare(lines, dv)
    assert not bad, f"{len(bad)} mismatches; first: {bad[:3]}"
    _check_selection(lines, dv)


@pytest.mark.gpu
def test_parse_lines_long_and_multi_chunk():
    """Lines beyond the short variant, > SDX_LONG_MAX, and a batch spanning many select chunks."""
    P = B.Bank().protocols
    base, _ = synth.line_corpus(P, 3000, seed=21, compress_frac=0.3, mu_npulse=200)
    longs = [b"\x02MU;P0=-500;P1=500;D=" + b"01" * k + b";CP=1;\x03" for k in (100, 129, 1000, 2048, 2049, 3000)]
    longs += [b"\x02MS;P0=-500;P1=500;P2=-5000;D=2" + b"01" * k + b";CP=1;SP=2;\x03" for k in (127, 128, 500)]
    lines = base + longs + base
    dv = _device_parse(lines)
    bad = _compare(lines, dv)
    assert not bad, f"{len(bad)} mismatches; first: {bad[:3]}"
    _check_selection(lines, dv)


@pytest.mark.gpu
def test_parse_comp_lds_buffer_edges():
    """k_parse_comp stages a compressed line (<= 176 raw bytes) and its decompressed payload
    (<= 344 bytes) in per-lane LDS buffers; lines past either bound take the global path.  A batch
    of compressed lines on both sides of both bounds, interleaved, matches the oracle."""
    P = B.Bank().protocols
    lines = []
    for k, npulse in enumerate((200, 240, 260, 280, 300, 320, 360, 600)):
        ls, _ = synth.line_corpus(P, 240, seed=50 + k, mix=(1, 1, 0), compress_frac=1.0, mu_npulse=npulse)
        lines += ls
    # data bytes with a high nibble >= 10 expand to three characters: short raw lines whose
    # payload passes 344 bytes
    pp = bytes([0x80 | 0, 0x80 | 0x74, 0x80 | 1]) + b";" + bytes([0x80 | 0x20 | 1, 0x80 | 0x58, 0x80 | 15]) + b";"
    for nd in (90, 100, 105, 110, 115, 120, 130, 140, 150, 160):
        for t in (b"u", b"s"):
            d = bytes((0xA0 + 17 * j) & 0xF7 | 0xA0 for j in range(nd))
            lines.append(synth.frame(b"M" + t + b";" + pp + b"D" + d + b";C0;" + (b"S1;" if t == b"s" else b"") + b"R2A;"))
    rng = np.random.default_rng(5)
    lines = [lines[j] for j in rng.permutation(len(lines))]
    comp = [ln for ln in lines if any(c > 127 for c in ln)]
    raw_fit = [len(ln) <= 176 for ln in comp]
    plens = [LO.parse_line(ln)["plen"] for ln in comp]
    assert sum(1 for f, p in zip(raw_fit, plens) if f and 0 <= p <= 344) > 100
    assert sum(1 for f, p in zip(raw_fit, plens) if f and p > 344) > 10  # payload overflows the LDS buffer
    assert sum(1 for f in raw_fit if not f) > 100                      # raw line overflows the LDS buffer
    dv = _device_parse(lines)
    bad = _compare(lines, dv)
    assert not bad, f"{len(bad)} mismatches; first: {bad[:3]}"
    _check_selection(lines, dv)


def _flat_msgs(res):
    return [[d.protocol_id, d.payload, d.metadata, [d.raw.line, d.raw.message_type, d.raw.rssi, d.raw.freq_afc]]
            for d in res]


@pytest.mark.gpu
@pytest.mark.parametrize("fname", GOLDENS)
def test_signal_parser_end_to_end_matches_reference(golden, fname):
    from pysignalduino_amd.frontend import SignalParser
    cases = golden(fname)
    sp = SignalParser()
    got = sp.parse_lines([c["line"] for c in cases])
    bad = []
    nres = 0
    for c, g in zip(cases, got):
        if isinstance(g, Exception):
            assert LO.parse_line(c["line"].encode("latin-1"))["status"] == LO.UNSUPPORTED
            continue
        exp = c.get("e2e", [])
        nres += len(exp)
        if _flat_msgs(g) != exp:
            bad.append((c["src"], c["line"][:80], exp[:2], _flat_msgs(g)[:2]))
    assert not bad, f"{len(bad)} mismatches; first: {bad[:2]}"
    assert nres > (60 if fname == GOLDENS[1] else 1000)
    # parse_line (single) agrees with the batch
    i = next(k for k, c in enumerate(cases) if c.get("e2e") and not isinstance(got[k], Exception))
    assert _flat_msgs(sp.parse_line(cases[i]["line"])) == cases[i]["e2e"]


@pytest.mark.gpu
def test_signal_parser_matches_demodulate_batch_at_scale():
    """200k lines: the fused line path == demodulate_batch of the oracle's msg_data (which the
    demodulator parity tests pin to the reference)."""
    from pysignalduino_amd.frontend import SignalParser
    from pysignalduino_amd.sd_protocols import SDProtocols
    P = B.Bank().protocols
    lines, _ = synth.line_corpus(P, 200_000, seed=31, compress_frac=0.3)
    proto = SDProtocols()
    got = SignalParser(proto).parse_lines(lines)
    recs = [LO.parse_line(ln) for ln in lines]
    for kind, name in ((LO.MU, "MU"), (LO.MS, "MS")):
        idx = [i for i, r in enumerate(recs) if r["status"] == LO.OK and r["kind"] == kind]
        exp = proto.demodulate_batch([dict(recs[i]["msg"]) for i in idx], name)
        for i, e in zip(idx, exp):
            e = [] if isinstance(e, BaseException) else e
            g = got[i]
            assert [(d.protocol_id, d.payload, d.metadata) for d in g] == \
                [(x["protocol_id"], x["payload"], x["meta"]) for x in e], (i, lines[i][:80])


@pytest.mark.gpu
def test_lines_general_batch_matches_oracle(golden):
    """sdx_lines_general on the SDX_LS_GENERAL lines: the general-layout pattern table (string ids,
    float values bitwise, dict order), MS cp slot / gates, D in the slot -- equal to the oracle."""
    from pysignalduino_amd import runtime
    from pysignalduino_amd.frontend import LineBatch, pack_lines
    from pysignalduino_amd.sd_protocols import SDProtocols
    lines = [c["line"] for c in golden("lines_general_golden.json.gz")]
    eng = SDProtocols()._ensure()
    data, offsets, _ = pack_lines(lines)
    lb = LineBatch(eng, data, offsets)
    lb.launch()
    status = lb.status[: len(lines)].cpu().numpy()
    kinds = lb.kind[: len(lines)].cpu().numpy()
    n_gen = 0
    for lk in (runtime.LINE_MU, runtime.LINE_MS):
        rows = np.nonzero((status == runtime.LS_GENERAL) & (kinds == lk))[0]
        if not len(rows):
            continue
        import ctypes
        import torch
        m = len(rows)
        sel = torch.from_numpy(rows.astype(np.int32)).to(eng.dev)
        g = {k: torch.empty(sz, dtype=dt, device=eng.dev) for k, sz, dt in
             (("offsets", m, torch.int64), ("len", m, torch.int32), ("npat", m, torch.uint8),
              ("pat_ids", 256 * m, torch.uint8), ("pat_val", 16 * m, torch.float64), ("cp_slot", m, torch.int8),
              ("ms_ok", m, torch.uint8))}
        p = runtime._ptr
        go = runtime.SdxLinesGeneralOut(*(p(g[k]) for k in ("offsets", "len", "npat", "pat_ids", "pat_val", "cp_slot",
                                                             "ms_ok")))
        runtime._check(eng.lib, eng.lib.sdx_lines_general(ctypes.byref(lb.c_lines), ctypes.byref(lb.c_out), p(sel), m,
                                                          ctypes.byref(go), eng.stream_ptr()))
        h = {k: v.cpu().numpy() for k, v in g.items()}
        st2 = lb.status[sel.long()].cpu().numpy()
        slot = lb.slot.cpu().numpy()
        for j, i in enumerate(rows):
            r = LO.parse_line(lines[i].encode("latin-1"))
            assert int(st2[j]) == r["status"], (i, lines[i][:80])
            if r["status"] != LO.GENERAL:
                continue
            n_gen += 1
            d = bytes(slot[int(h["offsets"][j]): int(h["offsets"][j]) + int(h["len"][j])])
            assert d == r["data"]
            npat = int(h["npat"][j])
            base = [256 * j + 16 * z for z in range(npat)]
            ids = [bytes(h["pat_ids"][b + 1: b + 1 + int(h["pat_ids"][b])]).decode() for b in base]
            assert ids == r["gids"], (ids, r["gids"])
            assert h["pat_val"][16 * j: 16 * j + npat].tobytes() == np.array(r["gvals"], np.float64).tobytes()
            if lk == runtime.LINE_MS:
                assert int(h["ms_ok"][j]) == r["ms_ok"] and (not r["ms_ok"] or int(h["cp_slot"][j]) == r["gcp"])
    assert n_gen > 200


@pytest.mark.gpu
def test_long_mc_lines_fixed_mode_and_json():
    """MC lines of more than 128 hex characters: sdx_parse_lines accepts them, k_mc hands them to
    sdx_demod_mc_general; in fixed mode the DecodedMessages equal demodulate_mc_batch on the same
    frames (the oracle-pinned dict path, tests/test_general.py), and parse_lines_json equals
    json.dumps of the first message."""
    import json
    from pysignalduino_amd.frontend import SignalParser
    from pysignalduino_amd.sd_protocols import SDProtocols
    p = SDProtocols(mc_mode="fixed")
    P = p.get_protocol_list()
    frames = synth.general_mc_frames(P, 300, seed=71) + synth.mc_planted_frames(P, 100, seed=72)
    frames = [f for f in frames if all(c in "0123456789ABCDEFabcdef" for c in f[0])]
    lines = ["\x02MC;LL=-1000;LH=900;SL=-500;SH=480;D=%s;C=%d;L=%d;R=40;\x03" % (h.upper(), c, L)
             for h, c, L, _, _ in frames]
    sp = SignalParser(p)
    got = sp.parse_lines(lines)
    ref = p.demodulate_mc_batch([{"raw_hex": h.upper(), "clock": c, "mcbitnum": L, "messagetype": "MC"}
                                 for h, c, L, _, _ in frames])
    nres = 0
    for g, r in zip(got, ref):
        exp = [] if isinstance(r, BaseException) else [(x["protocol_id"], x["payload"]) for x in r]
        assert [(d.protocol_id, d.payload) for d in g] == exp
        nres += len(exp)
    assert sum(len(f[0]) > 128 for f in frames) > 200 and nres > 20
    texts = sp.parse_lines_json(lines)
    for g, t in zip(got, texts):
        assert t == (json.dumps({"protocol_id": g[0].protocol_id, "payload": g[0].payload,
                                 "metadata": g[0].metadata}, indent=4) if g else None)


@pytest.mark.gpu
def test_parse_lines_large_batch_comp_chunk():
    """A batch large enough that the host sizes k_parse_comp's chunk above its 192-line minimum
    (the grid fits the resident waves in one round): the same 8000 lines repeated 110 times, and
    the first, a middle and the last copy compared with the oracle."""
    import torch
    P = B.Bank().protocols
    base, _ = synth.line_corpus(P, 8000, seed=31, compress_frac=0.3)
    reps = 110
    cu = torch.cuda.get_device_properties(0).multi_processor_count
    assert len(base) * reps > cu * 16 * 192, "batch too small to leave the minimum chunk"
    dv = _device_parse(base * reps)
    nb = len(base)
    for c in (0, reps // 2, reps - 1):
        lo, hi = c * nb, (c + 1) * nb
        sl = {k: (v[lo:hi] if isinstance(v, np.ndarray) and k not in ("slot", "offsets") else v) for k, v in dv.items()}
        sl["offsets"] = dv["offsets"][lo:hi + 1]
        bad = _compare(base, sl)
        assert not bad, f"copy {c}: {len(bad)} mismatches; first: {bad[:3]}"
