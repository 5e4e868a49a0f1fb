"""The general path on the GPU (include/sdx.h sdx_demod_pulses_general / sdx_demod_mc_general):
MU/MS messages with multi-digit pattern ids (message_unsynced.py:28-35 accepts any P<digits>),
more than 10 patterns, more than 4096 pulses, and MC frames of more than 128 hex characters --
bit-exact against the reference's goldens (tests/golden/make_general_golden.py) and the oracle."""
import numpy as np
import pytest

from oracle import sd_oracle as O

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def proto():
    from pysignalduino_amd.sd_protocols import SDProtocols
    return SDProtocols()


def _flat(res):
    if isinstance(res, BaseException):
        return {"raise": type(res).__name__}
    return {"results": [[r["protocol_id"], r["payload"], r["meta"]["bit_length"], r["meta"]["rssi"],
                         r["meta"]["clock"]] for r in res]}


def _oracle(ob, msg, kind):
    try:
        return _flat(O.demod(ob, dict(msg), kind))
    except Exception as e:
        return {"raise": type(e).__name__}


@pytest.mark.parametrize("kind", ["MU", "MS"])
def test_general_golden(proto, golden, kind):
    cases = golden("general_golden.json.gz")[kind.lower()]
    got = proto.demodulate_batch([c["msg"] for c in cases], kind)
    bad = [(i, c["exp"], _flat(g)) for i, (c, g) in enumerate(zip(cases, got)) if _flat(g) != c["exp"]]
    assert not bad, f"{len(bad)}/{len(cases)} mismatches; first: {bad[:2]}"
    assert sum(len(c["exp"].get("results", [])) for c in cases) > (1000 if kind == "MU" else 50)


def test_general_golden_mc_long_frames(golden):
    from pysignalduino_amd.sd_protocols import SDProtocols
    p = SDProtocols(mc_mode="fixed")
    frames = golden("general_golden.json.gz")["mc"]
    got = p.demodulate_mc_batch([{"raw_hex": f["hex"], "clock": f["clock"], "mcbitnum": f["L"],
                                  "messagetype": f["mtype"], "version": f["version"]} for f in frames])
    bad = []
    for f, g in zip(frames, got):
        gg = {"raise": type(g).__name__} if isinstance(g, BaseException) else \
            {"results": [[r["protocol_id"], r["payload"]] for r in g]}
        if gg != f["fixed"]:
            bad.append((f["hex"][:40], f["fixed"], gg))
    assert not bad, f"{len(bad)} mismatches; first: {bad[:2]}"


@pytest.mark.parametrize("kind,seed", [("MU", 601), ("MS", 602)])
def test_general_mixed_batch_vs_oracle(proto, kind, seed):
    """General-path messages interleaved with ordinary ones in one demodulate_batch call: every
    slot equals the oracle (the two launches' results land in their messages' slots)."""
    from pysignalduino_amd import synth
    P = proto.get_protocol_list()
    ob = O.OracleBank()
    gen = synth.general_pulse_messages(P, kind, 400, seed=seed)
    pb = (synth.mu_corpus if kind == "MU" else synth.ms_corpus)(P, 400, seed=seed + 7)
    plain = [pb.to_msg_dict(i) for i in range(pb.n)]
    rng = np.random.default_rng(seed)
    msgs = [m for pair in zip(gen, plain) for m in pair]
    rng.shuffle(msgs)
    got = proto.demodulate_batch(msgs, kind)
    bad = [(i, _oracle(ob, m, kind), _flat(g)) for i, (m, g) in enumerate(zip(msgs, got))
           if _flat(g) != _oracle(ob, m, kind)]
    assert not bad, f"{len(bad)}/{len(msgs)} mismatches; first: {bad[:2]}"


def test_general_contract_limits(proto):
    """More than SDX_GEN_MAXPAT patterns: ContractError in that message's slot only."""
    from pysignalduino_amd.packing import ContractError
    m = {"data": "0101010101" * 4, **{f"P{k}": str(100 * (k + 1)) for k in range(17)}}
    ok = {"data": "0121212121212121", "P0": "-4000", "P1": "400", "P2": "-800", "P10": "1200"}
    got = proto.demodulate_batch([m, ok], "MU")
    assert isinstance(got[0], ContractError)
    ob = O.OracleBank()
    assert _flat(got[1]) == _oracle(ob, ok, "MU")
    with pytest.raises(ContractError):
        proto.demodulate(m, "MU")


@pytest.mark.parametrize("kind", ["MU", "MS"])
def test_general_edge_cases_vs_oracle(proto, kind):
    """synth.general_edge_messages (also in the reference goldens) against the oracle."""
    from pysignalduino_amd import synth
    ob = O.OracleBank()
    msgs = synth.general_edge_messages(kind)
    got = proto.demodulate_batch(msgs, kind)
    for m, g in zip(msgs, got):
        assert _flat(g) == _oracle(ob, m, kind), (m.get("data", "")[:40], _flat(g), _oracle(ob, m, kind))


@pytest.mark.parametrize("kind", ["MU", "MS"])
def test_general_very_long_messages_vs_oracle(proto, kind):
    """Messages of 20k-60k pulses (the reference has no length limit): repeated planted frames,
    equal to the oracle (results, bit lengths, raises)."""
    from pysignalduino_amd import synth
    ob = O.OracleBank()
    P = proto.get_protocol_list()
    base = synth.planted_pulse_messages(P, kind, 6, seed=77, corrupt_frac=0.0)
    msgs = []
    for k, m in enumerate(base):
        m = dict(m)
        d = m["D"]
        reps = (20000 + 8000 * k) // max(1, len(d)) + 1
        m["D"] = m["data"] = (d + d[len(d) // 3:] * reps) if kind == "MS" else d * reps
        msgs.append(m)
    got = proto.demodulate_batch(msgs, kind)
    nres = 0
    for m, g in zip(msgs, got):
        exp = _oracle(ob, m, kind)
        assert _flat(g) == exp, (len(m["data"]), _flat(g).get("raise"), exp.get("raise"))
        nres += len(exp.get("results", []))
    assert nres > (100 if kind == "MU" else 0)



def test_general_modified_bank_repetition_bounds_vs_oracle():
    """The match-table rounds (sdx_general.hip mu_tables) for repetition bounds the shipped bank does
    not have: length_min 1 (one unit: every unit occurrence starts a match), length_min 0 after a start
    string (an empty repetition raises IndexError at chunks[-1], message_unsynced.py:212) and
    length_min at the general path's limit (SDX_GEN_REPMAX 128); oracle on the same edited bank.
    (No start and length_min 0 -- empty matches everywhere -- is outside the bank compiler's model.)"""
    from pysignalduino_amd import synth
    from pysignalduino_amd.sd_protocols import SDProtocols
    p = SDProtocols()
    P = p.get_protocol_list()
    nostart = [pid for pid, v in P.items() if "clockabs" in v and "start" not in v and v.get("active", True)]
    withstart = [pid for pid, v in P.items() if "clockabs" in v and "start" in v and v.get("active", True)]
    edits = {nostart[1]: 1, nostart[2]: 128, withstart[0]: 0, withstart[1]: 128, withstart[2]: 1}
    for pid, lmin in edits.items():
        p._protocols[pid]["length_min"] = lmin
    ob = O.OracleBank(p.get_protocol_list())
    msgs = synth.general_pulse_messages(P, "MU", 300, seed=611)
    got = p.demodulate_batch(msgs, "MU")
    exp = [_oracle(ob, m, "MU") for m in msgs]
    bad = [(i, e, _flat(g)) for i, (e, g) in enumerate(zip(exp, got)) if _flat(g) != e]
    assert not bad, f"{len(bad)}/{len(msgs)} mismatches; first: {bad[:2]}"
    edited = sum(1 for e in exp for r in e.get("results", []) if r[0] in edits)
    assert edited > 1000 and sum(1 for e in exp if e.get("raise") == "IndexError") > 0
