"""Host side: bank compiler, modulematch DFAs, C-ABI library load/exports/layouts (no GPU work)."""
import os
import random
import re

import numpy as np
import pytest

from oracle import sd_oracle as O
from pysignalduino_amd import bank as bankmod
from pysignalduino_amd import regex_dfa

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def bk():
    return bankmod.Bank()


def test_bank_classes(bk):
    assert len(bk.pids) == 160
    assert len(bk.mu_pids) == 129 and len(bk.ms_pids) == 66 and len(bk.mc_pids) == 12
    never = [bk.ms_pids[i] for i in np.nonzero(bk.ms_table["never"])[0]]
    assert len(never) == 19  # FSK sync strings: can never decode
    assert set(bk.mc_pids) == {"52", "10", "57", "119", "58", "43", "11", "129", "18", "47", "12", "96"}


def _all_patspecs(bk):
    for r in bk.mu_table:
        for f in ("start", "one", "zero", "flt"):
            yield r[f]
    for r in bk.ms_table:
        for q in range(4):
            yield r["key"][q]


def test_k_intervals_and_gap_ranks_match_fp64(bk):
    """The device's integer candidate test (klo <= k <= khi) and candidate order ((rank, dict
    position) from the bank's gap-rank tables) reproduce pattern_utils.py:53-63's fp64 test and
    stable gap sort for every k, including both interval borders."""
    ranks = np.asarray(bk._ranks)
    rng = random.Random(5)
    seen = 0
    for ps in _all_patspecs(bk):
        for u in range(int(ps["nuniq"])):
            v, tol = float(ps["uval"][u]), float(ps["utol"][u])
            klo, khi, off = int(ps["klo"][u]), int(ps["khi"][u]), int(ps["rk_off"][u])
            for k in range(klo - 30, khi + 31):
                g = abs(k / 10 - v)
                assert (g <= 0.001 or g <= tol) == (klo <= k <= khi), (v, k)
            ks = list(range(klo, khi + 1))
            for _ in range(20):  # random candidate sets in random dict order
                cand = rng.sample(ks, min(len(ks), rng.randint(2, 10)))
                ref = [j for _, j in sorted(((abs(k / 10 - v), j) for j, k in enumerate(cand)), key=lambda t: t[0])]
                dev = [j for _, j in sorted((int(ranks[off + k - klo]), j) for j, k in enumerate(cand))]
                assert ref == dev, (v, cand)
            seen += 1
    assert seen > 100


def test_bank_search_lists_and_tolerances(bk):
    P = bk.protocols
    for r, pid in enumerate(bk.mu_pids):
        for key, field in (("start", "start"), ("one", "one"), ("zero", "zero"), ("float", "flt")):
            spec = P[pid].get(key)
            ps = bk.mu_table[r][field]
            if not spec:
                assert ps["len"] == 0
                continue
            vals = [float(x) for x in spec]
            uniq = list(dict.fromkeys(vals))
            assert ps["len"] == len(vals) and ps["nuniq"] == len(uniq)
            for i, v in enumerate(uniq):
                assert ps["uval"][i] == v and ps["utol"][i] == O.tolerance(v)
            assert [uniq[k] for k in ps["uidx"][:len(vals)]] == vals


def test_modulematch_dfas_match_re_search(bk):
    cls_of, dfas = bk.dfa_host
    rnd = random.Random(3)
    alpha = "0123456789ABCDEFabcdef#PWTXirsuJKYbhxNone.F"
    for i, pat in enumerate(bk.mm_patterns):
        rx = re.compile(pat)
        lit = re.sub(r"[\^\$\\\[\]\.\*\{\}\(\)\|\?\+].*", "", pat.lstrip("^"))
        for _ in range(1500):
            s = (lit if rnd.random() < 0.6 else "") + "".join(rnd.choice(alpha) for _ in range(rnd.randint(0, 28)))
            assert regex_dfa.dfa_search(dfas[i], cls_of, s.encode()) == bool(rx.search(s)), (pat, s)


def test_preamble_prestate(bk):
    """Walking the DFA from the precomputed post-preamble state == re.search on the full payload."""
    cls_of, dfas = bk.dfa_host
    rnd = random.Random(4)
    for r, pid in enumerate(bk.mu_pids):
        d = int(bk.mu_table[r]["mm_dfa"])
        if d < 0:
            continue
        p = bk.protocols[pid]
        pre, post = f"{p.get('preamble', '')}", f"{p.get('postamble', '')}"
        for _ in range(200):
            dm = "".join(rnd.choice("0123456789ABCDEF") for _ in range(rnd.randint(0, 30)))
            st = regex_dfa.dfa_walk(dfas[d], cls_of, int(bk.mu_table[r]["mm_pre_state"]), (dm + post).encode())
            f = dfas[d][3][st]
            ok = bool(f & 1) or (not (f & 4) and bool(f & 2) and True)
            # exact: flags at the stop state; dfa_search re-walks from scratch for the reference
            assert regex_dfa.dfa_search(dfas[d], cls_of, (pre + dm + post).encode()) == bool(
                re.search(p["modulematch"], pre + dm + post))


def test_mu_desc_modulematch_tables(bk):
    """The LDS modulematch tables (hex-digit steps, postamble step, final flags) accept exactly
    the payloads re.search(modulematch, preamble + digits + postamble) accepts
    (message_unsynced.py:271-280), for every MU protocol on the table path."""
    import struct
    h = struct.unpack(bankmod.HDR_FMT, bk.blob[:struct.calcsize(bankmod.HDR_FMT)])
    off_tab, nbytes, S = h[21], h[22], h[23]
    tab = np.frombuffer(bk.blob[off_tab:off_tab + nbytes], dtype=np.uint8)
    rng = random.Random(11)
    P = bk.protocols
    checked = 0
    n_interval = 0
    for r, pid in enumerate(bk.mu_pids):
        d = bk.mu_desc[r]
        mm_on = int(d["mm_on"])
        if mm_on not in (1, 3):
            continue
        n_interval += mm_on == 3
        p = P[pid]
        pre, post = f"{p.get('preamble', '')}", f"{p.get('postamble', '')}"
        for _ in range(60):
            n = rng.randint(0, 24) if rng.random() < 0.8 else rng.randint(0, bankmod.MM_FAST_DIGITS)
            digits = "".join(rng.choice("0123456789ABCDEF") for _ in range(n))
            if rng.random() < 0.3:  # bias towards the pattern's own literal digits
                lit = "".join(c for c in p["modulematch"] if c in "0123456789ABCDEF")
                digits = (lit + digits)[:max(n, len(lit))]
            # the LDS table walk (mm_on 1, and still valid for 3)
            st = int(d["pre_state"])
            for c in digits:
                st = int(tab[16 * (int(d["mm_base"]) + st) + int(c, 16)])
            st = int(tab[17 * S + int(d["mm_post"]) + st])
            f = int(tab[16 * S + int(d["mm_base"]) + st])
            dev = bool(f & 1) or (not (f & 4) and bool(f & 2))
            exp = bool(re.search(p["modulematch"], pre + digits + post))
            assert dev == exp, (pid, digits)
            if mm_on == 3:  # the digit-count interval the device uses instead of the walk
                assert (int(d["res"][0]) <= len(digits) <= int(d["res"][1])) == exp, (pid, digits)
            checked += 1
    assert checked > 1000 and n_interval > 0


def test_blob_header(bk):
    import struct
    h = struct.unpack(bankmod.HDR_FMT, bk.blob[:struct.calcsize(bankmod.HDR_FMT)])
    assert h[0] == bankmod.MAGIC and h[1] == bankmod.VERSION and h[16] == len(bk.blob)
    assert (h[3], h[4], h[5]) == (129, 66, 12)


def test_library_loads_and_exports_every_declared_symbol():
    from pysignalduino_amd import build, runtime
    build.build()  # hipcc cross-compiles gfx950 here; no GPU needed
    lib = runtime.load_library()
    decl = set(re.findall(r"^\s*(?:int|size_t|uint64_t|const char\*|const void\*)\s+(sdx_\w+)\s*\(",
                          open(os.path.join(REPO, "include", "sdx.h")).read(), re.M))
    assert decl == set(runtime.EXPORTED)
    for name in decl:
        assert hasattr(lib, name), name
    assert lib.sdx_abi_version() == runtime.ABI_VERSION == 14
    runtime.check_layout(lib)


def test_step_entries_reject_bad_arguments_without_a_gpu():
    """sdx_demod_step / sdx_group_step (ABI 14) validate before any HIP call: null arguments and a batch
    without its output come back as SDX_EINVAL with a message (runs on the CPU)."""
    import ctypes
    from pysignalduino_amd import runtime
    lib = runtime.load_library()
    assert lib.sdx_demod_step(None, None, None) == -1
    assert b"null" in lib.sdx_last_error()
    st = runtime.SdxStep()
    b = runtime.SdxPulseBatch()
    st.mu = ctypes.pointer(b)                      # a batch without its sdx_out
    fake_bank = ctypes.c_void_p(1)                 # never dereferenced: the check comes first
    assert lib.sdx_demod_step(fake_bank, ctypes.byref(st), None) == -1
    assert b"sdx_out" in lib.sdx_last_error()
    job = runtime.SdxGroupJob()
    assert lib.sdx_group_step(None, ctypes.byref(job), ctypes.byref(job), None) == -1
    assert lib.sdx_group_step(fake_bank, ctypes.byref(job), ctypes.byref(job), None) == -1   # no batches


def test_bank_rejects_unmodelled():
    P = bankmod.load_protocols()
    bad = dict(P)
    bad["999"] = {"clockabs": 100, "one": [1, -2], "zero": [2, -1], "length_min": "abc"}
    with pytest.raises(NotImplementedError):
        bankmod.Bank(bad)


def test_compact_filter_records_roundtrip():
    """sdx_mu_filt / sdx_ms_filt hold exactly the lane filter's fields of the full records (len and
    nuniq even for a list that does not fit, flagged full)."""
    bk = bankmod.Bank()

    def dec(fs, u):
        lh = int(fs["lohi"][u])
        s16 = lambda v: v - 65536 if v >= 32768 else v  # noqa: E731
        rk = [int(fs["rk01"]) & 0xFFFF, int(fs["rk01"]) >> 16, int(fs["rk2_len_nu"]) & 0xFFFF][u]
        return s16(lh & 0xFFFF), s16(lh >> 16), rk

    for table, filt, keys, upk0 in ((bk.mu_table, bankmod.Bank._mu_filters(bk.mu_table), ("start", "one", "zero", "flt"),
                                     "start_upk"),
                                    (bk.ms_table, bankmod.Bank._ms_filters(bk.ms_table), (0, 1, 2, 3), "sync_upk")):
        nfull = 0
        for rec, f in zip(table, filt):
            full = bool(int(f["flags"]) & 8)
            nfull += full
            for i, k in enumerate(keys):
                ps = rec[k] if isinstance(k, str) else rec["key"][k]
                fs = f["spec"][i]
                assert (int(fs["rk2_len_nu"]) >> 16) & 0xFF == int(ps["len"])
                assert int(fs["rk2_len_nu"]) >> 24 == int(ps["nuniq"])
                if full:
                    continue
                for u in range(int(ps["nuniq"])):
                    assert dec(fs, u) == (int(ps["klo"][u]), int(ps["khi"][u]), int(ps["rk_off"][u]))
                assert (int(f[upk0]) if i == 0 else int(fs["upk"])) == int(ps["uidx_pk"])
        assert nfull < 10


def test_mu_clock_divider_is_exact():
    """The MU integer normalisation (sdx_mu_filt clk_c/clk_m/clk_sh, bank.clock_divider): for every
    MU clock, floor(x / c) == (x * m) >> sh over the device's input range (x = 10|P| < 2^30), at
    every multiple of c +- 1 on a grid and on random x; and the rounding built on it (half-even on
    the exact remainder, exact ties by fl((2q + 1) / 20)) equals Python's round(P / clockabs, 1) * 10."""
    import numpy as np
    bk = bankmod.Bank()
    rng = np.random.default_rng(3)
    clocks = sorted({float(c) for c in bk.mu_clock})
    checked = ties = 0
    for clock in clocks:
        c, m, shf = bankmod.clock_divider(clock)
        if not (shf >> 8) & 1:
            continue
        sh = shf & 0xFF
        q = np.unique(np.concatenate([np.arange(0, (1 << 30) // c, max(1, (1 << 30) // c // 4000)),
                                      rng.integers(0, (1 << 30) // c, 4000)])).astype(np.uint64)
        x = np.concatenate([q * c, q * c + 1, np.maximum(q * c, 1) - 1, rng.integers(0, 1 << 30, 20000).astype(np.uint64)])
        x = x[x < (1 << 30)].astype(np.uint64)
        assert np.array_equal((x * np.uint64(m)) >> np.uint64(sh), x // np.uint64(c)), clock
        # integral P: k from the integer remainder vs round(P / clock, 1); exact rational ties
        # (2r == c) round like fl((2q + 1) / 20), the same correctly rounded quotient
        P = rng.integers(-(1 << 20), 1 << 20, 3000).tolist()
        if c % 2 == 0:   # planted ties: 10|P| = q c + c / 2
            P += [s * (qq * c + c // 2) // 10 for qq in rng.integers(0, (1 << 20) // c, 3000).tolist()
                  for s in (1, -1) if (qq * c + c // 2) % 10 == 0]
        for p in P:
            xx = 10 * abs(p)
            qq, r = divmod(xx, c)
            if 2 * r == c:
                k = round(round((2 * qq + 1) / 20, 1) * 10)
                ties += 1
            else:
                k = qq + (1 if 2 * r > c else 0)
            k = -k if (p < 0) != (clock < 0) else k
            assert k == round(round(p / clock, 1) * 10), (p, clock)
        checked += 1
    assert checked >= 10 and ties > 1000, (checked, ties)
