"""Host packing of reference msg_data dicts (same conversions / exceptions as the reference)."""
import pytest

from oracle import sd_oracle as O
from pysignalduino_amd import packing


def test_patterns_match_reference_semantics(golden):
    for kind, f in (("MU", "mu_golden.json.gz"), ("MS", "ms_golden.json.gz")):
        for c in golden(f)[:400]:
            m = c["msg"]
            ids, vals = packing._patterns(m)
            ref = O._patterns(m)
            assert ids == list(ref.keys())
            import numpy as np
            assert np.array_equal(np.array(vals), np.array(list(ref.values())), equal_nan=True)


def test_ms_gates():
    p = packing.PulsePacker("MS")
    p.add({"P0": "500", "P1": "-5000", "data": "0101", "CP": "0", "SP": "1"})
    p.add({"P0": "500", "P1": "-5000", "data": "01a1", "CP": "0", "SP": "1"})
    p.add({"P0": "500", "P1": "-5000", "data": "0101", "CP": "7", "SP": "1"})
    p.add({"P0": "500", "P1": "-5000", "data": "0101", "CP": "0", "SP": "1", "R": "1q"})
    b = p.batch()
    assert list(b.ms_ok) == [1, 0, 0, 0]
    assert p.clock_abs[0] == 500.0


def test_contract_and_reference_exceptions():
    p = packing.PulsePacker("MU")
    with pytest.raises(packing.ContractError):
        p.add({"P10": "500", "P1": "-500", "data": "0101"})
    with pytest.raises(TypeError):  # float(None): the reference only catches ValueError
        p.add({"P0": None, "data": "0101"})
    p.add({"P0": "x", "P1": "500", "data": "11"})
    assert p.batch().npat[0] == 1


def test_non_ascii_digits_keep_isdigit():
    assert packing._encode_data("01٣") == b"01\xfe"
    assert packing._encode_data("01é") == b"01\xff"


def test_frontend_contract_raise_is_reported():
    """SDX_RAISE_CONTRACT (a general-path device limit, include/sdx.h) is not a reference outcome:
    the front end reports it as a ContractError in the line's slot instead of the empty list a
    reference-caught exception gives (host logic; the device side is covered by test_general.py)."""
    import types

    import numpy as np

    from pysignalduino_amd import runtime
    from pysignalduino_amd.frontend import SignalParser
    sp = SignalParser.__new__(SignalParser)
    sp.protocols = types.SimpleNamespace(_bank=None)
    d = np.zeros(1, runtime.DESC_DT)[0]
    d["status"] = runtime.ST_RAISED
    d["raise_kind"] = runtime.RAISE_CONTRACT
    got = sp._general_messages(b"", 3, None, None, None, None, "MU", d, None, b"", 0.0)
    assert isinstance(got, packing.ContractError)
    d["raise_kind"] = 1   # IndexError: caught by the reference's MUParser -> no messages
    assert sp._general_messages(b"", 3, None, None, None, None, "MU", d, None, b"", 0.0) == []
