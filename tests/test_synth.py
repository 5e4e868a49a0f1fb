import numpy as np

from pysignalduino_amd import bank, synth


def test_deterministic_and_shaped():
    P = bank.load_protocols()
    a = synth.mu_corpus(P, 500, seed=1)
    b = synth.mu_corpus(P, 500, seed=1)
    assert np.array_equal(a.data, b.data) and np.array_equal(a.pat_val, b.pat_val)
    assert (np.diff(a.offsets) == 256).all()
    s = synth.ms_corpus(P, 500, seed=2)
    assert (np.diff(s.offsets) <= 256).all() and (s.cp_slot >= 0).all()
    m = synth.mc_corpus(P, 500, seed=3)
    assert m.n == 500 and set(np.unique(m.hexdata)) <= set(b"0123456789ABCDEF")
