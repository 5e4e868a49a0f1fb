"""Pin the CPU oracle against the golden vectors produced by the reference itself."""
import pytest

from oracle import sd_oracle as O


@pytest.fixture(scope="module")
def bank():
    return O.OracleBank()


def _run(bank, msg, kind):
    try:
        res = O.demod(bank, dict(msg), kind)
    except Exception as e:  # parsers catch Exception -> message yields nothing
        return {"raise": type(e).__name__}
    return {"results": [[r["protocol_id"], r["payload"], r["meta"]["bit_length"], r["meta"]["rssi"],
                         r["meta"]["clock"]] for r in res]}


@pytest.mark.parametrize("kind,fname", [("MU", "mu_golden.json.gz"), ("MS", "ms_golden.json.gz")])
def test_oracle_demod_matches_reference(bank, golden, kind, fname):
    cases = golden(fname)
    bad = []
    for i, c in enumerate(cases):
        got = _run(bank, c["msg"], kind)
        if got != c["exp"]:
            bad.append((i, c["src"], c["msg"], c["exp"], got))
    assert not bad, f"{len(bad)} mismatches, first: {bad[:2]}"


def test_oracle_mc_fixed_matches_reference(bank, golden):
    bad = []
    for f in golden("mc_golden.json.gz"):
        try:
            got = {"results": [[r["protocol_id"], r["payload"]] for r in
                               O.demod_mc_fixed(bank, f["hex"], f["clock"], f["L"], f["mtype"], f["version"])]}
        except Exception as e:
            got = {"raise": type(e).__name__}
        if got != f["fixed"]:
            bad.append((f, got))
    assert not bad, f"{len(bad)} mismatches, first: {bad[:2]}"


def test_oracle_pattern_exists(golden):
    for s, t, d, exp in golden("units_golden.json.gz")["pattern_exists"]:
        assert O.pattern_exists(s, t, d) == exp, (s, t, d)


def test_oracle_helpers(bank, golden):
    u = golden("units_golden.json.gz")
    for s, exp in u["bin_str_2_hex_str"]:
        assert O.bits_to_hex(s) == exp, s
    for s, exp in u["hex_to_bin_str"]:
        assert O.hex_to_bits(s) == exp, s
    for s, exp in u["mc2dmc"]:
        assert O.mc_to_dmc(s) == exp, s
    for pid, n, exp in u["length_in_range"]:
        assert list(O.length_in_range(bank, pid, n)) == exp, (pid, n)
    for a, b, exp in u["round1"]:
        assert round(a / b, 1) == exp


def test_oracle_postdemo(golden):
    bad = []
    for meth, bits, kind, rc, ret in golden("units_golden.json.gz")["postdemo"]:
        try:
            r = O.POSTDEMO[meth](list(bits))
            got = ["ok", r[0], r[1]]
        except Exception as e:
            got = ["raise", type(e).__name__, None]
        if got != [kind, rc, ret]:
            bad.append((meth, bits, kind, rc, ret, got))
    assert not bad, f"{len(bad)} mismatches, first: {bad[:3]}"


def test_oracle_mc_methods(bank, golden):
    bad = []
    for pid, s, kind, rc, res in golden("units_golden.json.gz")["mc_methods"]:
        try:
            r = O.mc_method(bank, pid, s, len(s))
            got = ["ok", r[0], r[1] if r[0] != -1 else None]
        except Exception as e:
            got = ["raise", type(e).__name__, None]
        if got != [kind, rc, res if rc != -1 else None]:
            bad.append((pid, s, kind, rc, res, got))
    assert not bad, f"{len(bad)} mismatches, first: {bad[:3]}"


def test_oracle_general_path_matches_reference(bank, golden):
    """Multi-digit pattern ids, > 10 patterns, > 4096 pulses, MC frames > 128 hex characters:
    the reference's own outputs (tests/golden/make_general_golden.py) pin the oracle there too."""
    g = golden("general_golden.json.gz")
    for kind in ("MU", "MS"):
        bad = [(c["msg"], c["exp"], got) for c in g[kind.lower()]
               if (got := _run(bank, c["msg"], kind)) != c["exp"]]
        assert not bad, f"{kind}: {len(bad)} mismatches, first: {bad[:1]}"
    for f in g["mc"]:
        try:
            got = {"results": [[r["protocol_id"], r["payload"]] for r in
                               O.demod_mc_fixed(bank, f["hex"], f["clock"], f["L"], f["mtype"], f["version"])]}
        except Exception as e:
            got = {"raise": type(e).__name__}
        assert got == f["fixed"], f
