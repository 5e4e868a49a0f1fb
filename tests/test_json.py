"""Publish-ready JSON: sdx_serialize_json == MqttPublisher._message_to_json of the
first DecodedMessage of each line (signalduino/mqtt.py:227-245, controller.py:254-257).

The expected texts are json.dumps of the reference-recorded DecodedMessage fields
(tests/golden/lines_golden.json.gz "e2e", tests/golden/mn_golden.json.gz), i.e. exactly what the
reference's publisher would send for those lines."""
import json

import pytest

from oracle import json_oracle as J
from pysignalduino_amd import bank as B


def test_bank_json_fragments_are_pythons():
    bk = B.Bank()
    blob = bk.blob
    import struct
    hdr = struct.unpack(B.HDR_FMT, blob[:struct.calcsize(B.HDR_FMT)])
    so = hdr[15]   # off_str
    t = bk.json_table

    def frag(r, f):
        o, n = int(t[r][f + "_off"]), int(t[r][f + "_len"])
        return blob[so + o: so + o + n].decode("ascii")
    pids = bk.mu_pids + bk.ms_pids + bk.mc_pids + bk.mn_pids
    assert len(t) == len(pids)
    for r, pid in enumerate(pids):
        assert frag(r, "pid") == json.dumps(pid)
    for r in range(len(bk.mu_pids)):
        assert frag(r, "s1") == json.dumps(bk.mu_clock[r])
    base = len(bk.mu_pids) + len(bk.ms_pids) + len(bk.mc_pids)
    for r in range(len(bk.mn_pids)):
        assert frag(base + r, "s1") == json.dumps(bk.mn_modulation[r])
        assert frag(base + r, "s2") == json.dumps(bk.mn_rfmode[r])


def test_oracle_shape():
    s = J.message_to_json("54", 'W54#"\\x', {"bit_length": 72, "rssi": None, "clock": -1.0})
    assert s.startswith('{\n    "protocol_id": "54",\n    "payload": "W54#\\"\\\\x",\n    "metadata": {\n')
    assert J.published([]) is None


@pytest.mark.gpu
def test_gpu_json_matches_reference_lines(golden):
    from pysignalduino_amd.frontend import SignalParser
    cases = golden("lines_golden.json.gz")
    got = SignalParser().parse_lines_json([c["line"] for c in cases])
    n = 0
    for c, g in zip(cases, got):
        if isinstance(g, Exception):
            continue
        exp = J.published(c.get("e2e", []))
        assert g == exp, (c["line"][:80], g, exp)
        n += exp is not None
    assert n > 300


@pytest.mark.gpu
def test_gpu_json_matches_reference_mn(golden):
    from pysignalduino_amd.frontend import SignalParser
    from pysignalduino_amd.sd_protocols import SDProtocols
    cases = golden("mn_golden.json.gz")["lines"]
    proto = SDProtocols()
    by_rf = {}
    for k, c in enumerate(cases):
        by_rf.setdefault(c[2], []).append(k)
    n = 0
    for rf, ks in by_rf.items():
        got = SignalParser(proto, rfmode=rf).parse_lines_json([cases[k][1] for k in ks])
        for k, g in zip(ks, got):
            if isinstance(g, Exception):
                continue
            exp = J.published(cases[k][3].get("out", []))
            assert g == exp, (cases[k][1][:80], rf, g, exp)
            n += exp is not None
    assert n > 2000


@pytest.mark.gpu
def test_gpu_json_matches_objects_at_scale():
    """100k mixed lines (MU/MS/MC fixed/MN): the device texts == json.dumps of parse_lines' objects
    (which the other suites pin to the reference)."""
    from pysignalduino_amd import synth
    from pysignalduino_amd.frontend import SignalParser
    from pysignalduino_amd.sd_protocols import SDProtocols
    P = B.Bank().protocols
    base, _ = synth.line_corpus(P, 80_000, seed=77, compress_frac=0.3)
    mn = [synth.frame(synth.mn_payload(*f)) for f in synth.mn_frames(20_000, seed=78)]
    lines = [x for pair in zip(base[:20_000], mn) for x in pair] + base[20_000:]
    sp = SignalParser(SDProtocols(mc_mode="fixed"))
    objs = sp.parse_lines(lines)
    texts = sp.parse_lines_json(lines)
    n = 0
    for o, t in zip(objs, texts):
        if isinstance(o, Exception):
            assert isinstance(t, Exception)
            continue
        assert t == J.published(o)
        n += t is not None
    assert n > 40_000
