"""GPU parity: the HIP path (through the C-ABI) vs the reference goldens and the CPU oracle.

Bit-exact for everything (integer/byte/string work; the fp64 normalisation must reproduce
Python's round(x, 1) exactly, which the results below depend on)."""
import numpy as np
import pytest

from oracle import sd_oracle as O

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def proto():
    from pysignalduino_amd.sd_protocols import SDProtocols
    return SDProtocols()


@pytest.fixture(scope="module")
def obank():
    return O.OracleBank()


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


@pytest.mark.parametrize("kind,fname", [("MU", "mu_golden.json.gz"), ("MS", "ms_golden.json.gz")])
def test_golden_vectors(proto, golden, kind, fname):
    cases = golden(fname)
    got = proto.demodulate_batch([c["msg"] for c in cases], kind)
    bad = [(i, c["src"], c["exp"], _flat(g)) for i, (c, g) in enumerate(zip(cases, got)) if _flat(g) != c["exp"]]
    assert not bad, f"{len(bad)}/{len(cases)} mismatches; first: {bad[:3]}"


def test_golden_mc_fixed(golden):
    from pysignalduino_amd.sd_protocols import SDProtocols
    p = SDProtocols(mc_mode="fixed")
    frames = golden("mc_golden.json.gz")
    msgs = [{"raw_hex": f["hex"], "clock": f["clock"], "mcbitnum": f["L"], "messagetype": f["mtype"],
             "version": f["version"]} for f in frames]
    got = p.demodulate_mc_batch(msgs)
    bad = []
    for f, g in zip(frames, got):
        gg = {"raise": type(g).__name__} if isinstance(g, BaseException) else \
            {"results": [[r["protocol_id"], r["payload"]] for r in g]}
        if gg != f["fixed"]:
            bad.append((f, gg))
    assert not bad, f"{len(bad)} mismatches; first: {bad[:2]}"


def test_mc_strict_reference_behaviour(proto, golden):
    frames = golden("mc_golden.json.gz")[:300]
    mc_ids = proto.get_keys("clockrange")
    for f in frames:
        for pid, (kind, val) in zip(mc_ids, f["strict"]):
            msg = {"protocol_id": pid, "data": f["hex"], "clock": f["clock"], "bit_length": f["L"]}
            try:
                r = proto.demodulate_mc(msg, f["mtype"], version=f["version"])
                got = ["ok", [[x["protocol_id"], x["payload"]] for x in r]]
            except Exception as e:
                got = ["raise", type(e).__name__]
            assert got == [kind, val]
    assert proto.demodulate_mc({"raw_hex": "AA", "clock": "450", "mcbitnum": "8"}, "MC") == []


@pytest.mark.parametrize("kind,seed,n", [("MU", 1234, 2000), ("MS", 4321, 4000)])
def test_synthetic_vs_oracle(proto, obank, kind, seed, n):
    from pysignalduino_amd import synth
    gen = synth.mu_corpus if kind == "MU" else synth.ms_corpus
    pb = gen(proto.get_protocol_list(), n, seed=seed)
    msgs = [pb.to_msg_dict(i) for i in range(pb.n)]
    got = proto.demodulate_batch(msgs, kind)
    bad = []
    for i, (m, g) in enumerate(zip(msgs, got)):
        exp = _oracle(obank, m, kind)
        if _flat(g) != exp:
            bad.append((i, m, exp, _flat(g)))
    assert not bad, f"{len(bad)}/{n} mismatches; first: {bad[:2]}"


@pytest.mark.parametrize("n", [6000, 900])
def test_ms_length_classes_at_the_boundary_vs_oracle(proto, obank, n):
    """sdx_demod_pulses runs MS as two launches by tile length class (<= 128 pulses on the NW = 2
    instantiation, the rest on NW = 4): messages of 120..136 pulses around the
    class boundary, mixed with the corpus' own lengths, grouped (n >= GROUP_MIN: the key's top bit
    separates the classes) and ungrouped (n < GROUP_MIN: mixed tiles), equal the oracle message by
    message."""
    from pysignalduino_amd import synth
    pb = synth.ms_corpus(proto.get_protocol_list(), n, seed=8800 + n)
    msgs = [pb.to_msg_dict(i) for i in range(pb.n)]
    rng = np.random.default_rng(n)
    for i in rng.choice(n, n // 2, replace=False):
        d = msgs[int(i)]["data"]
        L = int(rng.integers(120, 137))
        msgs[int(i)] = dict(msgs[int(i)], data=(d * (L // max(1, len(d)) + 1))[:L])
    lens = np.array([len(m["data"]) for m in msgs])
    assert (lens == 128).any() and (lens == 129).any()
    got = proto.demodulate_batch(msgs, "MS")
    bad = []
    for i, (m, g) in enumerate(zip(msgs, got)):
        exp = _oracle(obank, m, "MS")
        if _flat(g) != exp:
            bad.append((i, len(m["data"]), exp, _flat(g)))
    assert not bad, f"{len(bad)}/{n} mismatches; first: {bad[:2]}"
    assert sum(1 for g in got if isinstance(g, list) and g) > n // 10


def test_mu_exact_rational_ties_vs_oracle(proto, obank):
    """MU pattern values planted on exact rational ties of the bank's clocks (10|P| = q c + c / 2):
    the device rounds those by fl((2q + 1) / 20) instead of reloading P (round 4); every message
    must still equal the oracle's round(P / clock, 1) result."""
    from pysignalduino_amd import synth
    rng = np.random.default_rng(77)
    P = proto.get_protocol_list()
    clocks = sorted({int(float(p["clockabs"])) for p in P.values()
                     if "clockabs" in p and "sync" not in p and float(p["clockabs"]).is_integer()
                     and int(float(p["clockabs"])) % 2 == 0})
    pb = synth.mu_corpus(P, 1500, seed=78)
    msgs = [pb.to_msg_dict(i) for i in range(pb.n)] + synth.planted_pulse_messages(P, "MU", 500, seed=79)
    ties = 0
    for m in msgs:
        c = clocks[int(rng.integers(0, len(clocks)))]
        for key in [k for k in m if k[:1] == "P" and k[1:].isdigit()]:
            v = int(float(m[key]))
            q0 = 10 * abs(v) // c
            for q in sorted(range(max(0, q0 - 12), q0 + 12), key=lambda q: abs(q - q0)):
                if (q * c + c // 2) % 10 == 0:
                    m[key] = str((-1 if v < 0 else 1) * ((q * c + c // 2) // 10))
                    ties += 1
                    break
    assert ties > 4000, ties
    got = proto.demodulate_batch(msgs, "MU")
    exp = [_oracle(obank, m, "MU") for m in msgs]
    bad = [(i, m, e, _flat(g)) for i, (m, e, g) in enumerate(zip(msgs, exp, got)) if _flat(g) != e]
    assert not bad, f"{len(bad)}/{len(msgs)} mismatches; first: {bad[:2]}"
    assert sum(bool(_flat(g).get("results")) for g in got) > 200


def test_long_messages_vs_oracle(proto, obank):
    """Messages beyond 256 pulses run through the long-message kernel variant."""
    from pysignalduino_amd import synth
    P = proto.get_protocol_list()
    msgs = []
    for npulse in (257, 300, 512, 1000):
        pb = synth.mu_corpus(P, 40, seed=npulse, npulse=npulse)
        msgs += [pb.to_msg_dict(i) for i in range(pb.n)]
    got = proto.demodulate_batch(msgs, "MU")
    bad = [(m, _oracle(obank, m, "MU"), _flat(g)) for m, g in zip(msgs, got) if _flat(g) != _oracle(obank, m, "MU")]
    assert not bad, f"{len(bad)} mismatches; first: {bad[:1]}"


def test_edge_cases(proto, obank):
    edges = [
        ({"data": "", "P0": "1"}, "MU"),
        ({"P0": "500", "P1": "-1000", "data": "0101010101", "CP": "0"}, "MU"),
        ({"P0": "1e3", "P1": " -500 ", "P2": "nan", "P3": "inf", "data": "0101010123", "CP": "0"}, "MU"),
        ({"P0": "500", "P1": "-5000", "data": "01٣1", "CP": "0", "SP": "1"}, "MS"),
        ({"P0": "500", "P1": "-5000", "data": "0101", "CP": "٠", "SP": "1"}, "MS"),
        ({"P0": "-0", "P1": "-5000", "data": "0101", "CP": "0", "SP": "1"}, "MS"),
    ]
    for msg, kind in edges:
        got = proto.demodulate_batch([msg], kind)[0]
        assert _flat(got) == _oracle(obank, msg, kind), msg


def test_size_independent_properties(proto):
    """At larger sizes: results are independent of batch composition (sharding invariance)
    and deterministic across runs."""
    from pysignalduino_amd import runtime, synth
    pb = synth.mu_corpus(proto.get_protocol_list(), 20000, seed=99)
    eng = proto._ensure()
    bd = eng.to_device_pulses(pb)
    d1, r1, h1 = eng.run(runtime.KIND_MU, bd)
    d2, r2, h2 = eng.run(runtime.KIND_MU, bd)

    def per_msg(desc, rec, heap):
        hb = heap.tobytes()
        out = []
        for d in desc:
            rs = rec[int(d["rec_begin"]): int(d["rec_begin"]) + int(d["n_rec"])]
            out.append((int(d["status"]), tuple((int(r["proto"]), int(r["bit_length"]),
                                                 hb[int(r["payload_off"]): int(r["payload_off"]) + int(r["payload_len"])])
                                                for r in rs)))
        return out
    a = per_msg(d1, r1, h1)
    assert a == per_msg(d2, r2, h2)
    half = pb.subset(np.arange(10000, 20000))
    d3, r3, h3 = eng.run(runtime.KIND_MU, eng.to_device_pulses(half))
    assert per_msg(d3, r3, h3) == a[10000:]


def test_ms_tile_overflow_reruns(proto, obank):
    """A tile whose MS survivors exceed the tile list (MS_SURV_CAP = 1024) is marked
    SDX_ST_OVF_TILE by the short kernel and re-run exactly on the long variant.  The message
    below survives the sync/one/zero lookups of 21 MS protocols (searched with the oracle), so
    64 copies in one tile need 1344 slots."""
    from pysignalduino_amd import runtime, synth
    from pysignalduino_amd.packing import PulsePacker
    heavy = {"P0": "1200", "P1": "400", "P2": "-2400", "P3": "-400", "P4": "-7200", "P5": "-3200",
             "P6": "-1200", "P7": "-3600", "CP": "1", "SP": "0", "R": "10",
             "data": "5471115027363400667351410245004006624247207240055141125723665270103635536264520237234703"
                     "1535357666035460372151345551047053162221571240443230735373311622430214516551552051466321"
                     "262560504771330060154657"}
    pb = synth.ms_corpus(proto.get_protocol_list(), 64, seed=5)
    msgs = [heavy] * 64 + [pb.to_msg_dict(i) for i in range(pb.n)] + [heavy] * 70
    pk = PulsePacker("MS")
    for m in msgs:
        pk.add(m)
    eng = proto._ensure()
    bd = eng.to_device_pulses(pk.batch())
    out = eng.alloc_out(len(msgs), 64 * len(msgs), 256 * len(msgs))
    eng.launch_pulses(runtime.KIND_MS, bd, out)
    desc, _, _ = eng.fetch(out)
    assert (desc["status"][:64] == runtime.ST_OVF_TILE).all()   # the first tile overflowed ...
    assert (desc["status"][64:128] == runtime.ST_OK).all()      # ... the synthetic tile did not
    got = proto.demodulate_batch(msgs, "MS")                    # ... and the re-run is exact
    bad = [(i, _oracle(obank, m, "MS"), _flat(g)) for i, (m, g) in enumerate(zip(msgs, got))
           if _flat(g) != _oracle(obank, m, "MS")]
    assert not bad, f"{len(bad)} mismatches; first: {bad[:1]}"


@pytest.mark.parametrize("kind,n,seed", [("MU", 50000, 9101), ("MS", 100000, 9102), ("MC", 100000, 9103)])
def test_large_corpus_vs_c_oracle(kind, n, seed):
    """Record-level, bit-exact: the device path (runtime.Engine through the C-ABI) against the
    plain-C oracle on large seeded corpora -- statuses/raise kinds, protocol ids, payload bytes
    and bit lengths of every result, in order."""
    import os
    from oracle import c_oracle as CO
    from pysignalduino_amd import bank as B, runtime, synth
    bk = B.Bank()
    eng = runtime.Engine(bk, 0)
    cb = CO.CBank()
    gen = {"MU": synth.mu_corpus, "MS": synth.ms_corpus, "MC": synth.mc_corpus}[kind]
    batch = gen(bk.protocols, n, seed=seed)
    if kind == "MC":
        d_desc, d_rec, d_heap = eng.run(runtime.KIND_MC, eng.to_device_mc(batch))
        packed = CO.mc_batch(batch)
        cls_pids = bk.mc_pids
    else:
        d_desc, d_rec, d_heap = eng.run(runtime.KIND_MU if kind == "MU" else runtime.KIND_MS,
                                        eng.to_device_pulses(batch))
        packed = CO.pack_batch(batch)
        cls_pids = bk.mu_pids if kind == "MU" else bk.ms_pids
    _compare_c_oracle(kind, d_desc, d_rec, d_heap, CO.run(kind, packed, max(1, min(16, len(os.sched_getaffinity(0))))),
                      cls_pids, cb)


def _compare_c_oracle(kind, d_desc, d_rec, d_heap, cres, cls_pids, cb):
    """Device outputs == C oracle outputs, record by record (statuses, raise kinds, protocols,
    payload bytes, bit lengths), read through the descriptors."""
    from pysignalduino_amd import runtime
    st, rk, rb, nr, rec, heap = cres
    dh, ch = d_heap.tobytes(), heap.tobytes()
    assert np.array_equal(d_desc["status"] == runtime.ST_RAISED, st == 1)
    assert np.array_equal(np.where(st == 1, d_desc["raise_kind"], 0), np.where(st == 1, rk, 0))
    ok = st == 0
    assert np.array_equal(d_desc["n_rec"][ok], nr[ok])
    bad = []
    for i in np.nonzero(ok & (nr > 0))[0]:
        a = d_rec[int(d_desc["rec_begin"][i]):int(d_desc["rec_begin"][i]) + int(nr[i])]
        b = rec[int(rb[i]):int(rb[i]) + int(nr[i])]
        for x, y in zip(a, b):
            same = (cls_pids[int(x["proto"])] == cb.pids[int(y["proto"])] and
                    dh[int(x["payload_off"]):int(x["payload_off"]) + int(x["payload_len"])] ==
                    ch[int(y["off"]):int(y["off"]) + int(y["len"])] and
                    (kind == "MC" or int(x["bit_length"]) == int(y["bitlen"])))
            if not same:
                bad.append((int(i), x, y))
    assert not bad, f"{len(bad)} record mismatches; first: {bad[:2]}"


@pytest.mark.parametrize("kind,n,seed", [("MU", 30000, 9201), ("MS", 30000, 9202)])
def test_grouped_order_and_spill_regions_vs_c_oracle(kind, n, seed):
    """sdx_demod_pulses with a workspace: the grouped message order (sdx_group.hip) on a noise-free
    corpus, whose result-heavy tiles spill past the LDS pools into the workspace -- every message
    exact against the C oracle, no tile overflow, spill regions in use (MU); and the same batch
    without a workspace (batch order, overflowing tiles re-run) gives the same results."""
    import os
    from oracle import c_oracle as CO
    from pysignalduino_amd import bank as B, runtime, synth
    bk = B.Bank()
    eng = runtime.Engine(bk, 0)
    cb = CO.CBank()
    gen = synth.mu_corpus if kind == "MU" else synth.ms_corpus
    batch = gen(bk.protocols, n, seed=seed, noise_frac=0.0)
    k = runtime.KIND_MU if kind == "MU" else runtime.KIND_MS
    bd = eng.to_device_pulses(batch)
    out = eng.alloc_out(n, 40 * n + 4096, 1024 * n + 65536, eng.pulses_work_bytes(n))
    eng.launch_pulses(k, bd, out)
    desc, rec, heap = eng.fetch(out)
    cur = out["cursor"].cpu().numpy()
    assert cur[2] == 0 and not np.isin(desc["status"], (runtime.ST_OVF_TILE, runtime.ST_OVF_OUT)).any()
    if kind == "MU":
        assert cur[3] > 0, "no tile used its spill region"
    cls_pids = bk.mu_pids if kind == "MU" else bk.ms_pids
    cres = CO.run(kind, CO.pack_batch(batch), max(1, min(16, len(os.sched_getaffinity(0)))))
    _compare_c_oracle(kind, desc, rec, heap, cres, cls_pids, cb)
    # batch order (no workspace): Engine.run re-runs what overflows; identical results
    d2, r2, h2 = eng.run(k, bd, rec_cap=40 * n + 4096, heap_cap=1024 * n + 65536, workspace=False)
    _compare_c_oracle(kind, d2, r2, h2, cres, cls_pids, cb)


@pytest.mark.parametrize("kind", ["MU", "MS"])
def test_message_records_match_soa_and_results(kind):
    """sdx_group_pulses writes one 128-byte sdx_msg_rec per grouped message: its fields equal the
    SoA arrays (pattern values bitwise; slots past npat 0), and k_pulses reading the records gives
    byte-identical descriptors, records and heap to k_pulses reading the SoA fields."""
    import torch
    from pysignalduino_amd import bank as B, runtime, synth
    bk = B.Bank()
    eng = runtime.Engine(bk, 0)
    n = 20000
    gen = synth.mu_corpus if kind == "MU" else synth.ms_corpus
    batch = gen(bk.protocols, n, seed=9301)
    k = runtime.KIND_MU if kind == "MU" else runtime.KIND_MS
    bd = eng.to_device_pulses(batch)
    bufs = eng.group_buffers(n)
    eng.use_mrec = True
    order = eng.group(k, bd, bufs=bufs)
    torch.cuda.synchronize()
    mr = bufs[2][: n * runtime.MREC_BYTES].cpu().numpy().view(runtime.MREC_DT)
    assert np.array_equal(mr["off"], batch.offsets[:-1])
    assert np.array_equal(mr["len"], np.diff(batch.offsets))
    assert np.array_equal(mr["npat"], batch.npat)
    assert np.array_equal(mr["pat_id"], batch.pat_id.reshape(n, 10))
    pv = batch.pat_val.reshape(n, 10).copy()
    pv[np.arange(10)[None, :] >= np.minimum(batch.npat, 10)[:, None]] = 0.0
    assert mr["pat_val"].tobytes() == pv.tobytes()
    if kind == "MS":
        assert np.array_equal(mr["cp_slot"], batch.cp_slot) and np.array_equal(mr["ms_ok"], batch.ms_ok)
    outs = []
    for use in (True, False):
        out = eng.alloc_out(n, 40 * n + 4096, 1024 * n + 65536, eng.pulses_work_bytes(n))
        eng.launch_pulses(k, bd, out, sel=order, group=False, mrec=bufs[2] if use else None)
        outs.append(eng.fetch(out))
    from pysignalduino_amd import dist
    a, b = (dist.canonical(*o) for o in outs)  # record placement follows the tiles' atomics: compare canonically
    assert all(x.tobytes() == y.tobytes() for x, y in zip(a, b))


@pytest.mark.parametrize("mrec,mc_known,n", [("", True, 20000), ("MU", True, 6000), ("MS", True, 6000),
                                            ("MU,MS", True, 6000), ("", False, 3000), ("", True, 1)])
def test_fused_step_matches_the_separate_launches(mrec, mc_known, n):
    """sdx_demod_step (ABI 14: the MU, MS and MC launches of a step as one k_step grid) gives the
    results of sdx_demod_pulses(MU), sdx_demod_pulses(MS) and sdx_demod_mc: descriptors, records and
    payloads (canonical form: record placement follows the tiles' atomics) and the exchange's per-message
    counts, byte for byte.  MS carries messages on both sides of the 128-pulse length class boundary;
    mrec: MU reads message records; mc_known = False: MC's length bound unknown (its frames run in
    their own launch after the fused kernel); n = 1: near-empty ranges.  mrec: the kinds whose launches
    read their header fields from the grouping's message records."""
    import torch
    from pysignalduino_amd import bank as B, dist, runtime, synth
    bk = B.Bank()
    eng = runtime.Engine(bk, 0)
    P = bk.protocols
    mu = synth.mu_corpus(P, n, seed=9401)
    ms = synth.ms_corpus(P, n, seed=9402)
    mc = synth.mc_corpus(P, n, seed=9403)
    bds = {"MU": eng.to_device_pulses(mu), "MS": eng.to_device_pulses(ms), "MC": eng.to_device_mc(mc)}
    if not mc_known:
        bds["MC"]["max_hex"] = 0
    kinds_mrec = {"MU": runtime.KIND_MU, "MS": runtime.KIND_MS}
    eng.use_mrec = {kinds_mrec[k] for k in mrec.split(",") if k}
    orders = {}
    bufs = {}
    for k, kd in (("MU", runtime.KIND_MU), ("MS", runtime.KIND_MS)):
        bufs[k] = eng.group_buffers(n)
        orders[k] = eng.group(kd, bds[k], bufs=bufs[k]) if n >= runtime.GROUP_MIN else None

    def alloc():
        caps = {"MU": (40, 1024), "MS": (8, 256), "MC": (8, 256)}
        return {k: eng.alloc_out(n, caps[k][0] * n + 4096, caps[k][1] * n + 65536,
                                 eng.pulses_work_bytes(n) if k != "MC" else 0, wire=True) for k in caps}

    sep, fus = alloc(), alloc()
    mr = {k: bufs[k][2] if (k in mrec and orders[k] is not None) else None for k in ("MU", "MS")}
    eng.launch_pulses(runtime.KIND_MU, bds["MU"], sep["MU"], sel=orders["MU"], group=False)
    eng.launch_pulses(runtime.KIND_MS, bds["MS"], sep["MS"], sel=orders["MS"], group=False)
    eng.launch_mc(bds["MC"], sep["MC"])
    eng.launch_step(mu=(bds["MU"], fus["MU"], orders["MU"], mr["MU"]), ms=(bds["MS"], fus["MS"], orders["MS"], mr["MS"]),
                    mc=(bds["MC"], fus["MC"], None))
    torch.cuda.synchronize()
    nres = 0
    for k in ("MU", "MS", "MC"):
        a, b = eng.fetch(sep[k]), eng.fetch(fus[k])
        nres += len(a[1])
        ca, cb = dist.canonical(*a), dist.canonical(*b)
        assert all(x.tobytes() == y.tobytes() for x, y in zip(ca, cb)), k
        assert torch.equal(sep[k]["wire"][:n], fus[k]["wire"][:n]), k
    assert n == 1 or nres > n


def test_mc_frames_past_a_promised_length_bound_are_flagged():
    """A batch whose max_hex promises <= 64 characters (no 65..128 launch follows) but holds longer
    frames: k_mc marks them SDX_ST_OVF_TILE (cursor[2] bit 1) for a re-run instead of leaving them
    without a descriptor -- through sdx_demod_mc and through the fused sdx_demod_step -- and the
    frames within the bound keep their results (equal to a launch with the true bound)."""
    import numpy as np
    import torch
    from pysignalduino_amd import bank as B, packing, runtime
    bk = B.Bank()
    eng = runtime.Engine(bk, 0)
    rng = np.random.default_rng(5)
    frames = []
    for i in range(2000):
        n = int(rng.integers(65, 129)) if i % 3 == 0 else int(rng.integers(8, 65))
        frames.append(("".join("0123456789ABCDEF"[int(v)] for v in rng.integers(0, 16, size=n)),
                       int(rng.integers(300, 700)), 4 * n, "MC", None))
    bd = eng.to_device_mc(packing.mc_batch_from_frames(frames))
    assert bd["max_hex"] > 64
    true = eng.alloc_out(bd["n"], 8 * bd["n"] + 4096, 256 * bd["n"] + 65536)
    eng.launch_mc(bd, true)
    lie = dict(bd, max_hex=64)
    long_ = np.array([len(f[0]) > 64 for f in frames])
    for via in ("mc", "step"):
        o = eng.alloc_out(bd["n"], 8 * bd["n"] + 4096, 256 * bd["n"] + 65536)
        if via == "mc":
            eng.launch_mc(lie, o)
        else:
            eng.launch_step(mc=(lie, o, None))
        torch.cuda.synchronize()
        assert int(o["cursor"][2].item()) & 2, via
        d = eng.fetch(o)[0]
        assert (d["status"][long_] == runtime.ST_OVF_TILE).all(), via
        dt, rt, ht = eng.fetch(true)
        keep = np.nonzero(~long_)[0]
        a = [(int(d["n_rec"][i]), int(d["status"][i])) for i in keep]
        b = [(int(dt["n_rec"][i]), int(dt["status"][i])) for i in keep]
        assert a == b, via


@pytest.mark.parametrize("n_mu,n_ms,mrec", [(333333, 333333, False), (5000, 2049, True), (2049, 1, False)])
def test_group_step_matches_two_groupings(n_mu, n_ms, mrec):
    """sdx_group_step (ABI 14: the MU and MS sorts' radix passes in the same launches) writes the orders
    (and message records) of two sdx_group_pulses calls, byte for byte -- at the bench size, with
    records, and with a one-message side."""
    import torch
    from pysignalduino_amd import bank as B, runtime, synth
    bk = B.Bank()
    eng = runtime.Engine(bk, 0)
    eng.use_mrec = mrec
    bd = {"MU": eng.to_device_pulses(synth.mu_corpus(bk.protocols, n_mu, seed=9501)),
          "MS": eng.to_device_pulses(synth.ms_corpus(bk.protocols, n_ms, seed=9502))}
    one = {k: eng.group_buffers(bd[k]["n"]) for k in bd}
    two = {k: eng.group_buffers(bd[k]["n"]) for k in bd}
    for k, kd in (("MU", runtime.KIND_MU), ("MS", runtime.KIND_MS)):
        eng.group(kd, bd[k], bufs=one[k])
    o_mu, o_ms = eng.group_step(bd["MU"], bd["MS"], two["MU"], two["MS"])
    torch.cuda.synchronize()
    assert o_mu.numel() == n_mu and o_ms.numel() == n_ms
    for k in bd:
        n = bd[k]["n"]
        assert torch.equal(one[k][0][:n], two[k][0][:n]), k
        if mrec:
            nb = n * runtime.MREC_BYTES
            assert torch.equal(one[k][2][:nb], two[k][2][:nb]), k


@pytest.mark.parametrize("kind,n", [("MU", 333333), ("MS", 5000), ("MU", 2049), ("MS", 1)])
def test_grouping_is_a_stable_sort_of_the_keys(kind, n):
    """sdx_group_pulses (k_sig + the 2-launch-per-pass radix sort, sdx_group.hip): the order is a
    permutation of the messages, the sorted keys it leaves in the workspace's first array are
    non-decreasing, and equal keys keep ascending message indices (stable) -- at the bench size
    (163 partitions), a partition boundary plus one, and a single message."""
    import torch
    from pysignalduino_amd import bank as B, runtime, synth
    bk = B.Bank()
    eng = runtime.Engine(bk, 0)
    gen = synth.mu_corpus if kind == "MU" else synth.ms_corpus
    batch = gen(bk.protocols, n, seed=9400 + n)
    k = runtime.KIND_MU if kind == "MU" else runtime.KIND_MS
    bd = eng.to_device_pulses(batch)
    bufs = eng.group_buffers(n)
    order = eng.group(k, bd, bufs=bufs)
    torch.cuda.synchronize()
    o = order.cpu().numpy().astype(np.int64)
    keys = bufs[1][: 4 * n].cpu().numpy().view(np.uint32).astype(np.int64)
    assert np.array_equal(np.sort(o), np.arange(n))
    assert (np.diff(keys) >= 0).all()
    same = np.diff(keys) == 0
    assert (np.diff(o)[same] > 0).all()
    if n > 1000:
        assert len(np.unique(keys)) > 1   # the keys actually differ: the sort was exercised


@pytest.mark.gpu
def test_mc_long_frames_vs_oracle():
    """Frames of 1..128 hex characters: the short (<= 64) and long (65..128) k_mc launches together
    equal the oracle's fixed chain, frame by frame (L drawn inside the protocols' length gates)."""
    import numpy as np
    from pysignalduino_amd.sd_protocols import SDProtocols
    ob = O.OracleBank()
    rng = np.random.default_rng(77)
    mc_ids = ob.ids_with("clockrange")
    msgs, exp = [], []
    for i in range(3000):
        n = int(rng.integers(1, 129)) if i % 2 else int(rng.integers(60, 129))
        hx = "".join("0123456789ABCDEFabcdef"[int(v)] for v in rng.integers(0, 22 if i % 7 == 0 else 16, size=n))
        pid = mc_ids[int(rng.integers(0, len(mc_ids)))]  # a clock and L inside one protocol's gates
        lo, hi = (float(x) for x in ob.prop(pid, "clockrange")[:2])
        clock = int(rng.integers(int(lo), int(hi) + 2))
        lmin = int(ob.prop(pid, "length_min", 1) or 1)
        lmax = int(ob.prop(pid, "length_max", 4 * n) or 4 * n)
        L = int(rng.integers(lmin, max(lmin, lmax) + 1))
        mt = "Mc" if i % 5 == 0 else "MC"
        msgs.append({"raw_hex": hx, "clock": clock, "mcbitnum": L, "messagetype": mt, "version": None})
    # bench-corpus frames, every other one padded past 64 hex characters with random digits
    from pysignalduino_amd import bank as B, synth
    mb = synth.mc_corpus(B.load_protocols(), 4000, seed=12)
    for i in range(mb.n):
        hx = mb.hex(i)
        if i % 2 == 0:
            lo_n = 65 - len(hx) if len(hx) < 65 else 1
            hx += "".join("0123456789ABCDEF"[int(v)] for v in rng.integers(0, 16, size=int(rng.integers(lo_n, 129 - len(hx)))))
        msgs.append({"raw_hex": hx, "clock": int(mb.clock[i]), "mcbitnum": int(mb.mcbitnum[i]),
                     "messagetype": "Mc" if mb.mtype[i] else "MC", "version": None})
    for m in msgs:
        try:
            exp.append({"results": [[r["protocol_id"], r["payload"]] for r in
                                    O.demod_mc_fixed(ob, m["raw_hex"], m["clock"], m["mcbitnum"], m["messagetype"], None)]})
        except Exception as e:  # noqa: BLE001
            exp.append({"raise": type(e).__name__})
    got = SDProtocols(mc_mode="fixed").demodulate_mc_batch(msgs)
    bad, nres, nlong = [], 0, 0
    for m, g, e in zip(msgs, got, exp):
        gg = {"raise": type(g).__name__} if isinstance(g, BaseException) else \
            {"results": [[r["protocol_id"], r["payload"]] for r in g]}
        nres += len(gg.get("results", []))
        nlong += len(m["raw_hex"]) > 64
        if gg != e:
            bad.append((m, e, gg))
    assert not bad, f"{len(bad)} mismatches; first: {bad[:2]}"
    # long frames (the MW = 8 launch) rarely decode -- the decoders check the bit length -- but
    # every one of them is compared (statuses, raises, empty lists)
    assert nres > 500 and nlong > 3000, (nres, nlong)
