"""Accept paths and the unit-level API (§8(b)).

Expected outputs come from the reference itself (tests/golden/make_accept_golden.py and
make_golden.py, run in the development container).  The CPU tests pin the oracle on the planted
corpora; the GPU tests run the drop-in SDProtocols -- demodulate_batch, demodulate_mc(_batch), and
the helper methods bound to sdx_units -- and compare bit-exact, including the exception classes
and the (-1, text) failure tuples of the reference's methods."""
import collections

import numpy as np
import pytest

from oracle import sd_oracle as O

POSTDEMO = ["postDemo_EM", "postDemo_Revolt", "postDemo_FS20", "postDemo_FHT80", "postDemo_FHT80TF",
            "postDemo_WS2000", "postDemo_WS7035", "postDemo_WS7053", "postDemo_lengtnPrefix"]


def _flat(res):
    if isinstance(res, BaseException):
        return {"raise": type(res).__name__}
    return {"results": [[r["protocol_id"], r["payload"], r["meta"]["bit_length"], r["meta"]["rssi"],
                         r["meta"]["clock"]] for r in res]}


def _jsonish(v):
    if isinstance(v, tuple):
        return [_jsonish(x) for x in v]
    if isinstance(v, list):
        return [_jsonish(x) for x in v]
    if isinstance(v, dict):
        return {k: _jsonish(x) for k, x in v.items()}
    return v


def _outcome(r):
    if isinstance(r, BaseException):
        return ["raise", type(r).__name__]
    return ["ok", _jsonish(r)]


# ----------------------------------------------------------------------------------------- CPU
@pytest.fixture(scope="module")
def obank():
    return O.OracleBank()


def test_oracle_planted_mu_ms(obank, golden):
    g = golden("accept_golden.json.gz")
    for kind in ("MU", "MS"):
        bad = []
        for c in g[kind.lower()]:
            try:
                got = _flat(O.demod(obank, dict(c["msg"]), kind))
            except Exception as e:
                got = {"raise": type(e).__name__}
            if got != c["exp"]:
                bad.append((c["msg"], c["exp"], got))
        assert not bad, f"{kind}: {len(bad)} mismatches, first {bad[:2]}"


def test_oracle_planted_mc(obank, golden):
    bad = []
    for f in golden("accept_golden.json.gz")["mc"]:
        try:
            got = {"results": [[r["protocol_id"], r["payload"]] for r in
                               O.demod_mc_fixed(obank, f["hex"], f["clock"], f["L"], f["mtype"], f["version"])]}
        except Exception as e:
            got = {"raise": type(e).__name__}
        if got != f["fixed"]:
            bad.append((f, got))
    assert not bad, f"{len(bad)} mismatches, first {bad[:2]}"


def test_oracle_planted_postdemo(golden):
    bad = []
    for meth, bits, kind, val in golden("accept_golden.json.gz")["postdemo"]:
        try:
            got = ["ok", _jsonish(O.POSTDEMO[meth](list(bits)))]
        except Exception as e:
            got = ["raise", type(e).__name__]
        if got != [kind, val]:
            bad.append((meth, bits, kind, val, got))
    assert not bad, f"{len(bad)} mismatches, first {bad[:2]}"


def test_planted_corpora_reach_every_accept_path(golden):
    """The reference accepts >= 100 planted frames per postDemo function / MC method and per
    postDemo user id (what the GPU tests below then compare)."""
    g = golden("accept_golden.json.gz")
    acc = collections.Counter(m for m, _, kind, val in g["postdemo"] if kind == "ok" and val[0] == 1)
    assert all(acc[m] >= 100 for m in POSTDEMO), acc
    accm = collections.Counter(m for m, *_, r in g["mc_methods"] if r[0] == "ok" and r[1][0] == 1)
    assert all(accm[m] >= 100 for m in ["mcBit2Funkbus", "mcBit2Sainlogic", "mcBit2AS", "mcBit2Hideki",
                                         "mcBit2Maverick", "mcBit2OSV1", "mcBit2OSV2o3", "mcBit2OSPIR",
                                         "mcBit2TFA", "mcBit2Grothe", "mcBit2SomfyRTS", "mcRaw", "mcraw"]), accm
    ids = collections.Counter(r[0] for c in g["mu"] + g["ms"] for r in c["exp"].get("results", []))
    assert all(ids[p] >= 100 for p in ["80", "45", "74", "74.1", "73", "70", "60", "66", "67", "39"]), ids
    mc = collections.Counter(r[0] for f in g["mc"] for r in f["fixed"].get("results", []))
    assert all(mc[p] >= 100 for p in ["58", "96", "119", "10", "11", "12", "18", "43", "47", "129"]), mc


# ----------------------------------------------------------------------------------------- GPU
@pytest.fixture(scope="module")
def proto():
    from pysignalduino_amd.sd_protocols import SDProtocols
    return SDProtocols()


@pytest.mark.gpu
def test_gpu_planted_mu_ms(proto, golden):
    g = golden("accept_golden.json.gz")
    for kind in ("MU", "MS"):
        cases = g[kind.lower()]
        got = proto.demodulate_batch([c["msg"] for c in cases], kind)
        bad = [(c["msg"], c["exp"], _flat(x)) for c, x in zip(cases, got) if _flat(x) != c["exp"]]
        assert not bad, f"{kind}: {len(bad)}/{len(cases)} mismatches; first {bad[:2]}"
        acc = collections.Counter(r["protocol_id"] for x in got if not isinstance(x, BaseException) for r in x)
        users = ["80", "45", "74", "74.1", "73", "70", "60", "66", "67", "39"] if kind == "MU" else ["74.1"]
        assert all(acc[p] >= 100 for p in users), acc


@pytest.mark.gpu
def test_gpu_planted_mc_fixed(golden):
    from pysignalduino_amd.sd_protocols import SDProtocols
    p = SDProtocols(mc_mode="fixed")
    frames = golden("accept_golden.json.gz")["mc"]
    msgs = [{"raw_hex": f["hex"], "clock": f["clock"], "mcbitnum": f["L"], "messagetype": f["mtype"],
             "version": f["version"]} for f in frames]
    got = p.demodulate_mc_batch(msgs)
    bad = []
    acc = collections.Counter()
    for f, x in zip(frames, got):
        gg = {"raise": type(x).__name__} if isinstance(x, BaseException) else \
            {"results": [[r["protocol_id"], r["payload"]] for r in x]}
        if gg != f["fixed"]:
            bad.append((f, gg))
        acc.update(r[0] for r in gg.get("results", []))
    assert not bad, f"{len(bad)} mismatches; first {bad[:2]}"
    assert all(acc[q] >= 100 for q in ["58", "96", "119"]), acc


@pytest.mark.gpu
def test_gpu_mc_strict_every_protocol(proto, golden):
    g = golden("accept_golden.json.gz")["mc_strict"]
    bad = []
    for f in g["frames"]:
        for pid, exp in zip(g["pids"], f["per_pid"]):
            msg = {"protocol_id": pid, "data": f["hex"], "clock": f["clock"], "bit_length": f["L"]}
            try:
                r = proto.demodulate_mc(msg, f["mtype"], version=f["version"])
                got = ["ok", [[x["protocol_id"], x["payload"], x["meta"]] for x in r]]
            except Exception as e:
                got = ["raise", type(e).__name__]
            if got != exp:
                bad.append((pid, f["hex"], exp, got))
    assert not bad, f"{len(bad)} mismatches; first {bad[:3]}"


@pytest.mark.gpu
def test_gpu_units_postdemo(proto, golden):
    cases = [(m, b, k, v) for m, b, k, v in golden("accept_golden.json.gz")["postdemo"]]
    cases += [(m, b, k, [rc, ret]) for m, b, k, rc, ret in golden("units_golden.json.gz")["postdemo"]]
    bad, acc = [], collections.Counter()
    for meth in POSTDEMO:
        sub = [c for c in cases if c[0] == meth]
        got = proto.postdemo_batch(meth, [list(c[1]) for c in sub])
        for (m, b, kind, val), x in zip(sub, got):
            o = _outcome(x)
            exp = [kind, val] if kind == "ok" else ["raise", val if isinstance(val, str) else val[0]]
            if o != exp:
                bad.append((m, b, exp, o))
            elif kind == "ok" and val[0] == 1:
                acc[m] += 1
    assert not bad, f"{len(bad)} mismatches; first {bad[:3]}"
    assert all(acc[m] >= 100 for m in POSTDEMO), acc
    # the single-call methods are the same launch
    assert proto.postDemo_lengtnPrefix("x", [1, 0, 1]) == (1, [0, 0, 0, 0, 0, 0, 1, 1, 1, 0, 1])
    with pytest.raises(ValueError):
        proto.postDemo_WS2000("x", [0] * 58 + [1])


@pytest.mark.gpu
def test_gpu_units_mc_methods(proto, golden):
    cases = list(golden("accept_golden.json.gz")["mc_methods"])
    P = proto.get_protocol_list()
    for pid, s, kind, rc, res in golden("units_golden.json.gz")["mc_methods"]:
        meth = P[pid]["method"].split(".")[-1]
        cases.append([meth, "n", s, pid, len(s), ["ok", [rc, res]] if kind == "ok" else ["raise", rc]])
    bad, acc = [], collections.Counter()
    by = collections.defaultdict(list)
    for c in cases:
        by[c[0]].append(c)
    for meth, sub in by.items():
        got = proto.mc_method_batch(meth, [(name, bits, pid, mb) for _, name, bits, pid, mb, _ in sub])
        for c, x in zip(sub, got):
            exp = c[5]
            o = _outcome(x)
            if o != exp:
                bad.append((c, o))
            elif exp[0] == "ok" and exp[1][0] == 1:
                acc[meth] += 1
    assert not bad, f"{len(bad)} mismatches; first {bad[:3]}"
    assert all(acc[m] >= 100 for m in by), acc
    # the reference's own unit-test calls (tests/test_manchester_protocols.py)
    assert proto.mcBit2Funkbus("some_name", "1001110101001111001111110111010101010101101000000000", "119", 52) == \
        (1, "2C175F30008F")
    assert proto.mcBit2Funkbus("x", "100111010100111100111111011101010101010110110000000", "119", 51) == \
        (-1, "parity error")
    assert proto.mcBit2Funkbus("x", "1001110101001111101111110111010101010101101000000000", "119", 52) == \
        (-1, "checksum error")


@pytest.mark.gpu
def test_gpu_units_custom_protocols(golden):
    """mcraw / _demodulate_mc_data on protocols edited in place (test_helpers.py:80-126,
    test_manchester_protocols.py:50-101)."""
    from pysignalduino_amd.sd_protocols import SDProtocols
    cust = golden("accept_golden.json.gz")["custom"]
    p2 = SDProtocols()
    p2._protocols[9989] = {"length_max": 24, "name": "Test Protocol"}
    p3 = SDProtocols()
    p3._protocols["119"] = {"length_min": 50, "name": "TestLength"}
    p4 = SDProtocols()
    p4._protocols["0"]["method"] = "manchester.mcRaw"
    p4._protocols["0"]["length_min"] = 1
    p4._protocols["0"]["length_max"] = 999
    p4._protocols["0"]["preamble"] = "u0#"
    p4._protocols["12"]["method"] = "manchester.mcRaw"
    for tag, arg, pid, mb, exp in cust:
        if tag == "mcraw":
            got = _outcome(_try(p2.mcraw, "some_name", arg, pid, mb))
        else:
            if tag == "dmc2":
                p3._protocols["119"]["length_min"] = 10
                p3._protocols["119"]["length_max"] = 40
                p3._protocols["119"]["method"] = "manchester.mcRaw"
            if tag == "dmc3":
                p3._protocols["119"]["length_max"] = 400
            pp = p4 if tag in ("dmc4", "dmc5") else p3
            got = _outcome(_try(pp._demodulate_mc_data, "TestLen" if pp is p3 else "n", pid, 500, arg, mb, "MC", None))
        assert got == exp, (tag, arg, exp, got)
    assert p2.mcraw("x", None, 9989, 24) == (-1, "no bitData provided")
    assert p2.mcraw("x", "0101", None, 4) == (-1, "no protocolId provided")


def _try(fn, *a):
    try:
        return fn(*a)
    except Exception as e:
        return e


@pytest.mark.gpu
def test_gpu_units_helpers(proto, golden):
    from pysignalduino_amd import pattern_utils as PU
    u, a = golden("units_golden.json.gz"), golden("accept_golden.json.gz")
    pe = u["pattern_exists"] + a["pattern_exists"]
    got = PU.pattern_exists_batch([(s, t, d) for s, t, d, _ in pe])
    bad = [(s, t, d, e, g) for (s, t, d, e), g in zip(pe, got) if g != e]
    assert not bad, f"pattern_exists: {len(bad)} mismatches; first {bad[:3]}"
    assert PU.pattern_exists([1, -1], {"0": 1.0, "1": -1.0}, "0101") == "01"
    assert PU.calculate_tolerance(20) == pytest.approx(3.6)
    hx = u["hex_to_bin_str"]
    assert proto.hex_to_bin_batch([s for s, _ in hx]) == [e for _, e in hx]
    inv = a["hex_to_bin_inv"]
    for flag in (False, True):
        sub = [(s, e) for s, f, e in inv if f == flag]
        got = proto.hex_to_bin_batch([s for s, _ in sub], invert=flag)
        assert [[1, g] for g in got] == [e for _, e in sub]
    assert proto._convert_mc_hex_to_bits("n", "0F", True, 2) == (1, "11110000")  # "F0"
    bh = u["bin_str_2_hex_str"] + a["bin2hex"]
    assert proto.bin_str_2_hex_batch([s for s, _ in bh]) == [e for _, e in bh]
    assert proto.bin_str_2_hex_str(None) is None and proto.bin_str_2_hex_str(5) is None
    md = u["mc2dmc"] + a["mc2dmc"]
    assert proto.mc2dmc_batch([s for s, _ in md]) == [e for _, e in md]
    assert proto.mc2dmc(None) == (-1, "no bitData provided")
    assert proto.dec_2_bin_ppari(32) == "001000001" and proto.dec_2_bin_ppari(204) == "110011000"


@pytest.mark.gpu
@pytest.mark.parametrize("kind,n,seed", [("MU", 40000, 9201), ("MS", 20000, 9202), ("MC", 60000, 9203)])
def test_gpu_planted_large_vs_c_oracle(kind, n, seed):
    """Record-level, bit-exact on large planted corpora (every postDemo user, every MC method's
    accept branch): the device path against the plain-C oracle, with >= 1000 accepted results per
    postDemo user id / TFA, Grothe and Funkbus frame set."""
    import os
    from oracle import c_oracle as CO
    from pysignalduino_amd import bank as B, packing, runtime, synth
    bk = B.Bank()
    eng = runtime.Engine(bk, 0)
    cb = CO.CBank()
    if kind == "MC":
        frames = synth.mc_planted_frames(bk.protocols, n, seed=seed)
        d_desc, d_rec, d_heap = eng.run(runtime.KIND_MC, eng.to_device_mc(packing.mc_batch_from_frames(frames)))
        packed = CO.pack_mc(frames)
        cls_pids = bk.mc_pids
    else:
        msgs = synth.planted_pulse_messages(bk.protocols, kind, n, seed=seed)
        packer = packing.PulsePacker(kind)
        for m in msgs:
            packer.add(m)
        d_desc, d_rec, d_heap = eng.run(runtime.KIND_MU if kind == "MU" else runtime.KIND_MS,
                                        eng.to_device_pulses(packer.batch()))
        packed = CO.pack_pulses(msgs)
        cls_pids = bk.mu_pids if kind == "MU" else bk.ms_pids
    threads = max(1, min(16, len(os.sched_getaffinity(0))))
    st, rk, rb, nr, rec, heap = CO.run(kind, packed, threads)
    dh, ch = d_heap.tobytes(), heap.tobytes()
    assert np.array_equal(d_desc["status"] == runtime.ST_RAISED, st == 1)
    assert np.array_equal(np.where(st == 1, d_desc["raise_kind"], 0), np.where(st == 1, rk, 0))
    ok = st == 0
    assert np.array_equal(d_desc["n_rec"][ok], nr[ok])
    bad, acc = [], collections.Counter()
    for i in np.nonzero(ok & (nr > 0))[0]:
        a = d_rec[int(d_desc["rec_begin"][i]):int(d_desc["rec_begin"][i]) + int(nr[i])]
        b = rec[int(rb[i]):int(rb[i]) + int(nr[i])]
        for x, y in zip(a, b):
            pid = cls_pids[int(x["proto"])]
            same = (pid == cb.pids[int(y["proto"])] and
                    dh[int(x["payload_off"]):int(x["payload_off"]) + int(x["payload_len"])] ==
                    ch[int(y["off"]):int(y["off"]) + int(y["len"])] and
                    (kind == "MC" or int(x["bit_length"]) == int(y["bitlen"])))
            acc[pid] += 1
            if not same:
                bad.append((int(i), x, y))
    assert not bad, f"{len(bad)} record mismatches; first: {bad[:2]}"
    want = {"MU": ["80", "45", "74", "73", "70", "60", "66", "67", "39"], "MS": ["74.1"],
            "MC": ["58", "96", "119"]}[kind]
    assert all(acc[p] >= 1000 for p in want), acc


@pytest.mark.gpu
def test_gpu_zero_padded_pattern_keys_and_per_message_contract(proto, golden):
    """P01 / P001 keys name pattern "1" as in the reference; a pattern id >= 10, > 4096 pulses and
    an MC frame > 128 hex characters run on the general path (equal to the oracle); a message
    outside the device contract (17 patterns) yields ContractError in its own slot while the rest
    of the batch decodes."""
    from oracle import sd_oracle as O
    from pysignalduino_amd.packing import ContractError
    from pysignalduino_amd.sd_protocols import SDProtocols
    ob = O.OracleBank()
    cases = golden("accept_golden.json.gz")["mu_p0x"]
    got = proto.demodulate_batch([c["msg"] for c in cases], "MU")
    assert [_flat(x) for x in got] == [c["exp"] for c in cases]
    msgs = [dict(c["msg"]) for c in cases[:20]]
    msgs[3] = dict(msgs[3], P10="500")
    msgs[7] = dict(msgs[7], data="0" * 5000, D="0" * 5000)
    msgs[9] = dict(msgs[9], **{f"P{k}": str(50 * k) for k in range(10, 27)})
    got = proto.demodulate_batch(msgs, "MU")
    assert isinstance(got[9], ContractError)
    for i in (3, 7):
        try:
            exp = _flat(O.demod(ob, dict(msgs[i]), "MU"))
        except Exception as e:
            exp = {"raise": type(e).__name__}
        assert _flat(got[i]) == exp
    assert [_flat(x) for i, x in enumerate(got) if i not in (3, 7, 9)] == \
        [c["exp"] for i, c in enumerate(cases[:20]) if i not in (3, 7, 9)]
    pf = SDProtocols(mc_mode="fixed")
    src = golden("accept_golden.json.gz")["mc"][:10]
    frames = [{"raw_hex": f["hex"], "clock": f["clock"], "mcbitnum": f["L"], "messagetype": f["mtype"],
               "version": f["version"]} for f in src]
    frames[4] = dict(frames[4], raw_hex="A" * 200)
    got = pf.demodulate_mc_batch(frames)
    for f, g in zip(frames, got):
        try:
            exp = [(r["protocol_id"], r["payload"]) for r in
                   O.demod_mc_fixed(ob, f["raw_hex"], f["clock"], f["mcbitnum"], f["messagetype"], f["version"])]
        except Exception as e:  # the reference raises on this frame (helpers.mcraw, id 57)
            assert type(g) is type(e)
            continue
        assert [(r["protocol_id"], r["payload"]) for r in g] == exp


@pytest.mark.gpu
def test_gpu_mc_fixed_protocol_id_evaluates_only_that_id(obank):
    """Fixed-mode demodulate_mc(msg_data) with a protocol_id runs that protocol only
    (sd_protocols.py:79-99): on a user-modified bank where id 57 (helpers.mcraw, which raises
    TypeError) overlaps TFA (58), a 58 frame raises without an id but decodes with protocol_id 58."""
    from pysignalduino_amd import synth
    from pysignalduino_amd.sd_protocols import SDProtocols
    p = SDProtocols(mc_mode="fixed")
    P = p.get_protocol_list()
    frames = [f for f in synth.mc_planted_frames(P, 600, seed=9) if 460 < f[1] < 520 and f[2] == 52][:40]
    assert frames
    p._protocols["57"]["clockrange"] = [300, 600]
    p._protocols["57"]["length_max"] = "60"
    msgs = [{"raw_hex": h, "clock": c, "mcbitnum": L, "messagetype": t, "version": v} for h, c, L, t, v in frames]
    got_all = p.demodulate_mc_batch(msgs)
    assert all(isinstance(g, TypeError) for g in got_all), got_all[:3]
    got = p.demodulate_mc_batch([dict(m, protocol_id="58") for m in msgs])
    n_ok = 0
    for (h, c, L, t, v), g in zip(frames, got):
        exp = O.demod_mc_fixed_one(obank, "58", h, c, L, t, v)
        assert g == ([exp] if exp is not None else []), (h, g, exp)
        n_ok += exp is not None
    assert n_ok > 0
    assert p.demodulate_mc(dict(msgs[0], protocol_id="58"), "MC") == got[0]
    # an id outside the MC table: nothing, and no raise from the others
    assert p.demodulate_mc_batch([dict(msgs[0], protocol_id="0")]) == [[]]
