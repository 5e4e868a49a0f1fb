"""N>1 path on CPU: world_size-2 gloo run of the shard + all-gather step (pysignalduino_amd/dist.py).

Each rank encodes the oracle's results for its contiguous shard into the device result-buffer
format (sdx_desc / sdx_result / heap), all-gathers, and must reconstruct exactly the results of
the un-sharded stream."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from oracle import sd_oracle as O
from pysignalduino_amd import dist as sdist
from pysignalduino_amd import runtime, synth


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def encode(results, pids):
    desc = np.zeros(len(results), runtime.DESC_DT)
    recs, heap = [], bytearray()
    for i, res in enumerate(results):
        desc[i]["rec_begin"] = len(recs)
        if isinstance(res, Exception):
            desc[i]["status"] = runtime.ST_RAISED
            desc[i]["raise_kind"] = 1
            continue
        desc[i]["n_rec"] = len(res)
        for r in res:
            b = r["payload"].encode("latin-1")
            recs.append((len(heap), len(b), pids.index(r["protocol_id"]), r["meta"]["bit_length"], i))
            heap += b
    rec = np.array(recs, dtype=runtime.RES_DT) if recs else np.zeros(0, runtime.RES_DT)
    return desc, rec, np.frombuffer(bytes(heap), np.uint8)


def decode(desc, rec, heap, pids):
    out = []
    hb = heap.tobytes()
    for d in desc:
        if d["status"] == runtime.ST_RAISED:
            out.append("raise")
            continue
        rs = rec[int(d["rec_begin"]): int(d["rec_begin"]) + int(d["n_rec"])]
        out.append([(pids[int(r["proto"])], hb[int(r["payload_off"]): int(r["payload_off"]) + int(r["payload_len"])],
                     int(r["bit_length"])) for r in rs])
    return out


def _oracle_results(msgs):
    ob = O.OracleBank()
    res = []
    for m in msgs:
        try:
            res.append(O.demod(ob, dict(m), "MU"))
        except Exception as e:
            res.append(e)
    return res


def _worker(rank, world, port, msgs, pids, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    lo, hi = sdist.shard_bounds(len(msgs), rank, world)
    d, r, h = encode(_oracle_results(msgs[lo:hi]), pids)
    td = torch.from_numpy(d.view(np.uint8).copy())
    tr = torch.from_numpy(r.view(np.uint8).copy()) if len(r) else torch.zeros(1, dtype=torch.uint8)
    th = torch.from_numpy(h.copy()) if len(h) else torch.zeros(1, dtype=torch.uint8)
    gd, gr, gh = sdist.allgather_results(td, tr, th, hi - lo, len(r), len(h))
    got = decode(gd.numpy().view(runtime.DESC_DT), gr.numpy().view(runtime.RES_DT), gh.numpy(), pids)
    # the multi-launch form (one count exchange + one data collective), twice: launches of different
    # sizes, device-side counts
    cur = torch.tensor([len(r), len(h), 0, 0], dtype=torch.int32)
    half = (hi - lo) // 2
    d2, r2, h2 = encode(_oracle_results(msgs[lo:lo + half]), pids)
    cur2 = torch.tensor([len(r2), len(h2), 0, 0], dtype=torch.int32)
    t2 = (torch.from_numpy(d2.view(np.uint8).copy()),
          torch.from_numpy(r2.view(np.uint8).copy()) if len(r2) else torch.zeros(1, dtype=torch.uint8),
          torch.from_numpy(h2.copy()) if len(h2) else torch.zeros(1, dtype=torch.uint8))
    (a, b, c), (a2, b2, c2) = sdist.allgather_streams([(td, tr, th, hi - lo, cur), (*t2, half, cur2)])
    got_multi = decode(a.numpy().view(runtime.DESC_DT), b.numpy().view(runtime.RES_DT), c.numpy(), pids)
    got_half = decode(a2.numpy().view(runtime.DESC_DT), b2.numpy().view(runtime.RES_DT), c2.numpy(), pids)
    # the pipelined form the bench runs: submit per step, the results of each completed step
    ex = sdist.Exchange()
    steps = []
    for parts in ([(td, tr, th, hi - lo, cur)], [(*t2, half, cur2), (td, tr, th, hi - lo, cur)]):
        ex.submit(parts)
        steps.append([decode(a.numpy().view(runtime.DESC_DT), b.numpy().view(runtime.RES_DT), c.numpy(), pids)
                      for a, b, c in ex.gathered()])
    ex.flush()
    # overflow + re-run: rank 1's launch has overflowed messages; the re-run callback adds an overlay
    # with their results, every rank recounts, and the gathered stream is the un-sharded one
    n = hi - lo
    ovf = (np.arange(n) % 5 == 0) & (rank == 1)
    d3 = d.copy()
    d3["status"][ovf] = runtime.ST_OVF_OUT
    d3["n_rec"][ovf] = 0
    td3 = torch.from_numpy(d3.view(np.uint8).copy())

    def rerun(part):
        od = d.copy()
        od["status"][~ovf] = runtime.ST_ABSENT
        part.overlays.append(sdist.Part(torch.from_numpy(od.view(np.uint8).copy()), tr, th, n, cur))
        return part

    ex2 = sdist.Exchange()
    ex2.submit([sdist.Part(td3, tr, th, n, cur)], rerun=rerun)
    ex2.flush()
    a3, b3, c3 = ex2.gathered()[0]
    got_rerun = decode(a3.numpy().view(runtime.DESC_DT), b3.numpy().view(runtime.RES_DT), c3.numpy(), pids)
    q.put((rank, got, got_multi, got_half, steps, got_rerun, ex2.reruns))
    dist.destroy_process_group()


def test_shard_bounds():
    for n in (0, 1, 7, 100, 1001):
        for w in (1, 2, 3, 8):
            spans = [sdist.shard_bounds(n, r, w) for r in range(w)]
            assert spans[0][0] == 0 and spans[-1][1] == n
            assert all(spans[i][1] == spans[i + 1][0] for i in range(w - 1))
            assert max(b - a for a, b in spans) - min(b - a for a, b in spans) <= 1


@pytest.mark.parametrize("world", [2, 4])
def test_gloo_world_allgather_matches_unsharded(world):
    """world 2 and 4 (gloo, CPU): every rank's gathered stream -- single launch, multi-launch, the
    pipelined Exchange and the overflow re-run path -- equals the un-sharded one"""
    from pysignalduino_amd import bank
    P = bank.load_protocols()
    pb = synth.mu_corpus(P, 120, seed=5)
    msgs = [pb.to_msg_dict(i) for i in range(pb.n)]
    pids = bank.Bank().mu_pids
    full = decode(*encode(_oracle_results(msgs), pids), pids)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, msgs, pids, q)) for r in range(world)]
    for p in procs:
        p.start()
    outs = [q.get(timeout=300) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    halves = []
    for r in range(world):
        lo, hi = sdist.shard_bounds(len(msgs), r, world)
        halves += full[lo: lo + (hi - lo) // 2]
    for rank, got, got_multi, got_half, steps, got_rerun, reruns in outs:
        assert got_rerun == full, f"rank {rank}: the re-run exchange differs"
        assert reruns == (1 if rank == 1 else 0), (rank, reruns)
        assert got == full, f"rank {rank} gathered stream differs"
        assert got_multi == full, f"rank {rank}: allgather_streams differs"
        assert got_half == halves, f"rank {rank}: second launch of allgather_streams differs"
        assert steps == [[full], [halves, full]], f"rank {rank}: Exchange steps differ"


def _guard_worker(rank, world, port, q):
    """Collective-size agreement: rank 1 submits two launches where rank 0 submits
    one; then rank 1's overflow re-run raises.  Each case must raise ExchangeMismatch on EVERY rank
    (fixed-size count frames), with no rank left waiting in a collective; a third exchange after them
    still works (the ranks are back in step)."""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    rng = np.random.default_rng(40 + rank)
    d, r, h = synth_launch(rng, 300, spill=False)
    part = lambda dd: (torch.from_numpy(dd.view(np.uint8).copy()), torch.from_numpy(r.view(np.uint8).copy()),  # noqa: E731
                       torch.from_numpy(h.copy()), len(dd), torch.tensor([len(r), len(h), 0, 0], dtype=torch.int32))
    got = []
    try:
        sdist.Exchange().submit([part(d)] * (1 if rank == 0 else 2))
        got.append("no error")
    except sdist.ExchangeMismatch as e:
        got.append("mismatch" if "launches" in str(e) else str(e))
    d2 = d.copy()
    d2["status"][:3] = runtime.ST_OVF_OUT

    def rerun(p):
        if rank == 1:
            raise MemoryError("injected re-run failure")
        od = d.copy()
        od["status"][3:] = runtime.ST_ABSENT
        p.overlays.append(sdist.Part(*part(od)))
        return p
    try:
        sdist.Exchange().submit([part(d2)], rerun=rerun)
        got.append("no error")
    except sdist.ExchangeMismatch as e:
        got.append("rerun failed" if "[1]" in str(e) else str(e))
    # rank 1's re-run succeeds but leaves more launches + overlays than a count frame holds
    # (XCHG_MAX_PARTS): the local recount preparation raises on rank 1 alone -- both ranks raise
    def rerun_many(p):
        od = d.copy()
        od["status"][3:] = runtime.ST_ABSENT
        for _ in range(runtime.XCHG_MAX_PARTS if rank == 1 else 1):
            p.overlays.append(sdist.Part(*part(od)))
        return p
    try:
        sdist.Exchange().submit([part(d2)], rerun=rerun_many)
        got.append("no error")
    except sdist.ExchangeMismatch as e:
        got.append("local" if "[1]" in str(e) else str(e))
    # the pipelined setting on host buffers (rank 1 only): flagged in the frame, both ranks raise
    try:
        sdist.Exchange(pipeline=rank == 1).submit([part(d)])
        got.append("no error")
    except sdist.ExchangeMismatch as e:
        got.append("branch" if "branch" in str(e) else str(e))
    ex = sdist.Exchange()
    ex.submit([part(d)])
    ex.flush()
    got.append(int(ex.gathered()[0][0].numel()) // 8)
    q.put((rank, got))
    dist.destroy_process_group()


def test_exchange_mismatch_raises_on_every_rank():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_guard_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    outs = dict(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
    want = ["mismatch", "rerun failed", "local", "branch", 600]
    assert outs == {0: want, 1: want}, outs


def test_check_frames_header_rules():
    """check_frames: the counts of K launches come back per rank; any header difference raises."""
    f = np.zeros((3, sdist.FRAME_INTS), np.int32)
    for r in range(3):
        f[r, :sdist.FRAME_HDR] = sdist.frame_header(3, 2, sdist.PHASE_COUNT)
        f[r, sdist.FRAME_HDR: sdist.FRAME_HDR + 16] = np.arange(16) + 100 * r
    S, fl = sdist.check_frames(f.reshape(-1), 3, 2, sdist.PHASE_COUNT)
    assert S.shape == (3, 2, 8) and S[2, 1, 7] == 215 and not fl.any()
    for field, val in ((0, 0), (1, 4), (2, 3), (3, sdist.PHASE_RECOUNT)):
        g = f.copy()
        g[1, field] = val
        with pytest.raises(sdist.ExchangeMismatch):
            sdist.check_frames(g.reshape(-1), 3, 2, sdist.PHASE_COUNT)


def synth_affix(rng, nproto=129):
    """A per-protocol (preamble, postamble) table shaped like Bank.affixes (preambles such as 'W54#',
    's', '', postambles mostly empty)."""
    out = []
    for _ in range(nproto):
        pre = bytes(rng.choice(list(b"WPsiu0123456789#"), size=int(rng.integers(0, 6))).astype(np.uint8))
        post = bytes(rng.choice(list(b"#;x"), size=int(rng.integers(0, 3)) * int(rng.random() < 0.3)).astype(np.uint8))
        out.append((pre, post))
    return out


def synth_payload(rng, affix, proto):
    """Payloads of every form: pre + uppercase hex + post (the nibble form; odd and even digit counts,
    none), lowercase hex, a broken affix, arbitrary bytes."""
    pre, post = affix[proto] if affix is not None else (b"", b"")
    u = rng.random()
    nd = int(rng.integers(0, 40))
    if u < 0.6:
        return pre + bytes(rng.choice(list(b"0123456789ABCDEF"), size=nd).astype(np.uint8)) + post
    if u < 0.7:
        return pre + bytes(rng.choice(list(b"0123456789abcdef"), size=nd + 1).astype(np.uint8)) + post
    if u < 0.8:
        return pre[:-1] + b"Z" + bytes(rng.choice(list(b"0123456789ABCDEF"), size=nd).astype(np.uint8)) + post
    return bytes(rng.integers(32, 127, size=nd, dtype=np.uint8))


def synth_launch(rng, n, spill=True, affix=None, status_absent=0.0, heavy=0.0):
    """Launch outputs shaped like k_pulses writes them: records per tile of 64 messages in a shuffled
    tile order, tile pieces of the heap 16-byte aligned with gaps, RAISED and empty messages, and
    (``spill``) records past the used range that no message owns.  ``status_absent``: the fraction of
    descriptors left at ST_ABSENT (an overlay's); ``heavy``: the fraction of messages with 60-300
    records (spanning whole 64-record waves of the exchange's record pass)."""
    nrec = rng.integers(0, 7, size=n) * (rng.random(n) < 0.8)
    if heavy:
        nrec = np.where(rng.random(n) < heavy, rng.integers(60, 301, size=n), nrec)
    status = np.where(rng.random(n) < 0.1, runtime.ST_RAISED, runtime.ST_OK)
    nrec[status == runtime.ST_RAISED] = 0
    desc = np.zeros(n, runtime.DESC_DT)
    desc["status"] = status
    desc["raise_kind"] = np.where(status == runtime.ST_RAISED, rng.integers(1, 6, size=n), 0)
    desc["n_rec"] = nrec
    recs, heap = [], bytearray()
    tiles = rng.permutation((n + 63) // 64)
    for t in tiles:
        for m in rng.permutation(np.arange(64 * t, min(n, 64 * t + 64))):
            desc[m]["rec_begin"] = len(recs) if nrec[m] else rng.integers(0, 1000)
            for _ in range(nrec[m]):
                pr = int(rng.integers(0, 129))
                pay = synth_payload(rng, affix, pr)
                heap += pay
                recs.append((len(heap) - len(pay), len(pay), pr, int(rng.integers(0, 300)), int(m)))
        heap += b"\0" * ((-len(heap)) % 16 + 16 * int(rng.integers(0, 2)))
    if spill:   # written but unowned records (an abandoned tile region)
        for _ in range(5):
            recs.append((0, 3, 1, 1, int(rng.integers(0, n))))
    if status_absent:
        absent = rng.random(n) < status_absent
        desc["status"][absent] = runtime.ST_ABSENT
    rec = np.array(recs, runtime.RES_DT) if recs else np.zeros(0, runtime.RES_DT)
    return desc, rec, np.frombuffer(bytes(heap), np.uint8).copy()


@pytest.mark.gpu
@pytest.mark.parametrize("pack_form", ["records", "messages"])
def test_exchange_pack_heavy_messages(pack_form, monkeypatch):
    """Messages of 60-300 records (the record pass's wave scan: a message that starts in an earlier
    wave and ends in this one is placed from its total, one spanning the whole wave by lane 0's loop)
    pack to the numpy wire form, raw and nibble, on both packs."""
    from pysignalduino_amd import bank as bankmod
    monkeypatch.setenv("SDX_XCHG_PACK_MSG", "1" if pack_form == "messages" else "0")
    dev = torch.device("cuda", 0)
    eng = runtime.Engine(bankmod.Bank(), 0)
    affix = eng.bank.affixes(runtime.KIND_MU)
    s = torch.cuda.current_stream(dev)
    for nib in (False, True):
        rng = np.random.default_rng(17)
        launches = [synth_launch(rng, n, affix=affix, heavy=h) for n, h in ((700, 0.05), (300, 0.3))]
        kind = runtime.KIND_MU if nib else runtime.KIND_RAW
        parts = [_dev_launch(d, r, h, dev, kind=kind) for d, r, h in launches]
        ex = _kernel_exchange(eng if nib else None)
        cnt = ex._count_pack_device(sdist._flatten(parts), s).cpu().numpy().reshape(2, runtime.XCHG_COUNTS)
        want = [sdist.wire_encode(d, r, h, affix=affix if nib else None) for d, r, h in launches]
        assert max(int(d["n_rec"].max()) for d, _, _ in launches) > 128
        offs, nb, T = sdist._layout(cnt[None])
        sv = ex._bufs["send"].cpu().numpy()
        for k, (m, w, p, _) in enumerate(want):
            o = offs[0, k]
            assert list(cnt[k][:3]) == [len(m), len(w), len(p)], (nib, k)
            assert sv[o[0]: o[0] + 4 * len(m)].tobytes() == m.tobytes(), (nib, k)
            assert sv[o[1]: o[1] + 8 * len(w)].tobytes() == w.tobytes(), (nib, k)
            assert sv[o[2]: o[2] + len(p)].tobytes() == p.tobytes(), (nib, k)


def test_wire_nibble_form_round_trip():
    """wire v3: payloads of the form preamble + uppercase hex + postamble travel as packed digits
    (proto | WIRE_NIB), everything else raw; decode(encode(x)) == canonical(x) with the affixes, and
    the wire payload bytes shrink by about half for the nibble records."""
    rng = np.random.default_rng(21)
    affix = synth_affix(rng)
    d, r, h = synth_launch(rng, 800, spill=False, affix=affix)
    m, w, p, bad = sdist.wire_encode(d, r, h, affix=affix)
    assert bad == 0
    nib = (w["proto"] & runtime.WIRE_NIB) != 0
    assert 0.3 < nib.mean() < 0.9, nib.mean()
    raw_bytes = int(w["payload_len"].astype(np.int64).sum())
    assert len(p) < raw_bytes
    got = sdist.wire_decode([(m, w, p)], affix)
    want = sdist.canonical(d, r, h)
    for a, b in zip(got, want):
        assert a.tobytes() == b.tobytes()
    # every nibble record really is pre + uppercase hex + post, every raw one is not
    hb = want[2].tobytes()
    for x, isnib in zip(want[1], nib):
        pay = hb[int(x["payload_off"]): int(x["payload_off"]) + int(x["payload_len"])]
        assert (sdist._nib_digits(affix, int(x["proto"]), pay) >= 0) == bool(isnib)


def test_wire_overlays_last_present_wins():
    """A launch with two overlays (host form of sdx_xchg_part.alt): message m comes from the last level
    whose descriptor is not ST_ABSENT; the primary's overflowed messages are then shipped from the
    overlays, and an overflow no overlay covers stays "bad"."""
    rng = np.random.default_rng(22)
    n = 600
    d0, r0, h0 = synth_launch(rng, n, spill=False)
    ovf = rng.random(n) < 0.2
    d0["status"][ovf] = runtime.ST_OVF_OUT
    d0["n_rec"][ovf] = 0
    d1, r1, h1 = synth_launch(rng, n, spill=False, status_absent=0.5)
    d2, r2, h2 = synth_launch(rng, n, spill=False, status_absent=0.8)
    d1["status"][ovf & (d1["status"] == runtime.ST_ABSENT) & (d2["status"] == runtime.ST_ABSENT)] = runtime.ST_OK
    m, w, p, bad = sdist.wire_encode(d0, r0, h0, overlays=[(d1, r1, h1, None, None), (d2, r2, h2, None, None)])
    assert bad == 0
    lev, rd = sdist.resolve_host([(d0,), (d1,), (d2,)])
    assert (lev[d2["status"] != runtime.ST_ABSENT] == 2).all()
    assert (lev[(d2["status"] == runtime.ST_ABSENT) & (d1["status"] != runtime.ST_ABSENT)] == 1).all()
    # the same results as one launch holding each message's resolved records
    cd, cr, ch = sdist.wire_decode([(m, w, p)])
    for i in rng.choice(n, 60, replace=False):
        src = [(d0, r0, h0), (d1, r1, h1), (d2, r2, h2)][int(lev[i])]
        dd = src[0][i]
        assert int(cd[i]["status"]) == int(dd["status"]) and int(cd[i]["n_rec"]) == (
            int(dd["n_rec"]) if dd["status"] == runtime.ST_OK else 0)
        for j in range(int(cd[i]["n_rec"])):
            a = cr[int(cd[i]["rec_begin"]) + j]
            b = src[1][int(dd["rec_begin"]) + j]
            assert (int(a["proto"]), int(a["bit_length"])) == (int(b["proto"]), int(b["bit_length"]))
            assert ch[int(a["payload_off"]): int(a["payload_off"]) + int(a["payload_len"])].tobytes() == \
                src[2][int(b["payload_off"]): int(b["payload_off"]) + int(b["payload_len"])].tobytes()
    # an overflow that no overlay covers is shipped as bad
    d0b = d0.copy()
    hole = np.nonzero((d1["status"] == runtime.ST_ABSENT) & (d2["status"] == runtime.ST_ABSENT))[0][0]
    d0b["status"][hole] = runtime.ST_OVF_TILE
    assert sdist.wire_encode(d0b, r0, h0, overlays=[(d1, r1, h1, None, None), (d2, r2, h2, None, None)])[3] == 1


def test_wire_canonical_is_order_free():
    """The wire form does not depend on where a launch put its records and payloads: two layouts of
    the same results (tile orders, heap gaps) encode to the same bytes, and decode to the canonical
    arrays (records in message order, payloads packed)."""
    rng = np.random.default_rng(11)
    d, r, h = synth_launch(rng, 500, spill=False)
    got = sdist.wire_encode(d, r, h)
    assert got[3] == 0
    # a second layout: records of each message moved to the end in reverse message order
    recs, heap = [], bytearray()
    d2 = d.copy()
    for m in range(len(d) - 1, -1, -1):
        rb, nr = int(d[m]["rec_begin"]), int(d[m]["n_rec"])
        if d[m]["status"] != runtime.ST_OK:
            continue
        d2[m]["rec_begin"] = len(recs)
        for x in r[rb: rb + nr]:
            heap += b"\xff" * 3
            recs.append((len(heap), x["payload_len"], x["proto"], x["bit_length"], m))
            heap += h[x["payload_off"]: x["payload_off"] + x["payload_len"]].tobytes()
    r2 = np.array(recs, runtime.RES_DT)
    got2 = sdist.wire_encode(d2, r2, np.frombuffer(bytes(heap), np.uint8))
    for a, b in zip(got[:3], got2[:3]):
        assert a.tobytes() == b.tobytes()
    cd, cr, ch = sdist.wire_decode([got[:3]])
    assert (cd["n_rec"] == d["n_rec"]).all() and (cd["status"] == d["status"]).all()
    assert (cr["msg"][1:] >= cr["msg"][:-1]).all()
    assert int(cd["rec_begin"][-1]) + int(cd["n_rec"][-1]) == len(cr)
    # a message whose records leave the written range is "bad"
    bad = sdist.wire_encode(d, r, h, nrec_written=len(r) - 1)
    assert bad[3] >= 1


def _dev_launch(desc, rec, heap, dev, cursor=None, kind=runtime.KIND_RAW):
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a).view(np.uint8).copy() if len(a) else  # noqa: E731
                                   np.zeros(16, np.uint8)).to(dev)
    cur = torch.tensor(cursor if cursor is not None else [len(rec), len(heap), 0, 0], dtype=torch.int32, device=dev)
    return sdist.Part(t(desc), t(rec), t(heap), len(desc), cur, kind)


def _kernel_exchange(eng=None):
    ex = sdist.Exchange.__new__(sdist.Exchange)
    ex._bufs, ex.engine = {}, eng
    return ex


@pytest.mark.gpu
@pytest.mark.parametrize("pack_form", ["records", "messages"])
def test_exchange_kernels_match_host_wire(pack_form, monkeypatch):
    """sdx_exchange_count / sdx_exchange_pack (HIP) == the numpy wire form for K = 3 launches laid
    out like k_pulses output (shuffled tiles, padded heap, RAISED / empty / unowned records), raw and
    in the nibble form (the real bank's MU affixes), and sdx_exchange_unpack over 3 ranks' sections ==
    wire_decode; an out-of-range message is counted bad.  Both packs: source-record order (k_xw_words
    + k_xw_recs, the default) and message order (k_xw_pack, SDX_XCHG_PACK_MSG=1)."""
    from pysignalduino_amd import bank as bankmod
    monkeypatch.setenv("SDX_XCHG_PACK_MSG", "1" if pack_form == "messages" else "0")
    dev = torch.device("cuda", 0)
    eng = runtime.Engine(bankmod.Bank(), 0)
    affix = eng.bank.affixes(runtime.KIND_MU)
    s = torch.cuda.current_stream(dev)
    for nib in (False, True):
        rng = np.random.default_rng(3)
        launches = [synth_launch(rng, n, affix=affix) for n in (1, 3000, 20000)]
        kind = runtime.KIND_MU if nib else runtime.KIND_RAW
        parts = [_dev_launch(d, r, h, dev, kind=kind) for d, r, h in launches]
        ex = _kernel_exchange(eng if nib else None)
        flat = sdist._flatten(parts)
        cnt = ex._count_pack_device(flat, s).cpu().numpy().reshape(3, runtime.XCHG_COUNTS)
        want = [sdist.wire_encode(d, r, h, affix=affix if nib else None) for d, r, h in launches]
        for k, (m, w, p, bad) in enumerate(want):
            pb = int(w["payload_len"].astype(np.int64).sum())
            assert list(cnt[k]) == [len(m), len(w), len(p), bad, pb, 0, 0, 0], (nib, k, cnt[k])
        if nib:
            assert cnt[:, 2].sum() < 0.8 * cnt[:, 4].sum()
        offs, nb, T = sdist._layout(cnt[None])
        sv = ex._bufs["send"].cpu().numpy()
        for k, (m, w, p, _) in enumerate(want):
            o = offs[0, k]
            assert sv[o[0]: o[0] + 4 * len(m)].tobytes() == m.tobytes(), k
            assert sv[o[1]: o[1] + 8 * len(w)].tobytes() == w.tobytes(), k
            assert sv[o[2]: o[2] + len(p)].tobytes() == p.tobytes(), k
            for j, ln in enumerate((4 * len(m), 8 * len(w), len(p))):   # zero padding to 16 bytes
                assert not sv[o[j] + ln: o[j] + sdist._r16(ln)].any(), (k, j)
        # the same layout twice (counters reset by the kernels themselves)
        cnt2 = ex._count_pack_device(flat, s).cpu().numpy().reshape(3, runtime.XCHG_COUNTS)
        assert (cnt2 == cnt).all()
        assert (ex._bufs["send"].cpu().numpy()[:T] == sv[:T]).all()
        # unpack: three "ranks" = the three launches' wire sections of one buffer
        Su = np.array([[len(m), len(w), len(p), 0, int(w["payload_len"].astype(np.int64).sum())]
                       for m, w, p, _ in want], np.int64)
        gd, gr, gh = sdist.unpack_device(ex._bufs["send"], Su, [offs[0, k] for k in range(3)], ex.engine, kind)
        ed, er, eh = sdist.wire_decode([(m, w, p) for m, w, p, _ in want], affix if nib else None)
        assert gd.cpu().numpy().tobytes() == ed.tobytes()
        assert gr.cpu().numpy().tobytes() == er.tobytes()
        assert gh.cpu().numpy().tobytes() == eh.tobytes()
    # a cursor short of the records written: the owning messages are "bad"
    d, r, h = launches[1]
    bad_parts = sdist._flatten([_dev_launch(d, r, h, dev, [len(r) - 10, len(h), 0, 0])])
    cb = _kernel_exchange().\
        _count_pack_device(bad_parts, s).cpu().numpy()
    assert cb[3] == sdist.wire_encode(d, r, h, nrec_written=len(r) - 10)[3] > 0


@pytest.mark.gpu
def test_kernel_written_wire_counts_match_the_scan():
    """ABI 12: the MU / MS (short and long k_pulses, spill regions) and MC (k_mc) flushes write the
    exchange's per-message counts and per-record classes (sdx_out.wire_dev / xrec_dev); the wire
    packed from them is byte-identical to the wire of the same launches classified by the exchange
    kernels themselves (parts without them), nibble form on and off, and equals the host
    wire_encode of the fetched outputs."""
    from pysignalduino_amd import bank as bankmod, synth
    dev = torch.device("cuda", 0)
    eng = runtime.Engine(bankmod.Bank(), 0)
    P = eng.bank.protocols
    s = torch.cuda.current_stream(dev)
    n = 20000
    launches = []
    for kind, c in ((runtime.KIND_MU, synth.mu_corpus(P, n, seed=31, noise_frac=0.0)),   # heavy tiles spill
                    (runtime.KIND_MS, synth.ms_corpus(P, n, seed=32)),
                    (runtime.KIND_MU, synth.mu_corpus(P, 400, seed=33, npulse=700)),       # long variant
                    (runtime.KIND_MC, synth.mc_corpus(P, n, seed=34))):
        bd = eng.to_device_mc(c) if kind == runtime.KIND_MC else eng.to_device_pulses(c)
        o = eng.alloc_out(c.n, 16 * c.n + 4096, 400 * c.n + 65536,
                          eng.pulses_work_bytes(c.n) if kind != runtime.KIND_MC else 0, wire=True)
        if kind == runtime.KIND_MC:
            eng.launch_mc(bd, o)
        else:
            eng.launch_pulses(kind, bd, o, long_variant=c.n == 400)
        launches.append((kind, o))
    torch.cuda.synchronize()
    for _, o in launches:
        assert int(o["cursor"][2]) == 0
    spilled = int(launches[0][1]["cursor"][3])
    for nib in (True, False):
        sends = []
        for use in (True, False):
            parts = [sdist.Part.from_out(o, kind if nib else runtime.KIND_RAW) for kind, o in launches]
            if not use:
                for p in parts:
                    p.wire = p.xrec = None
            ex = _kernel_exchange(eng if nib else None)
            cnt = ex._count_pack_device(sdist._flatten(parts), s).cpu().numpy().reshape(len(parts), runtime.XCHG_COUNTS)
            offs, nb, T = sdist._layout(cnt[None])
            sends.append((cnt, ex._bufs["send"][:T].cpu().numpy().copy()))
        assert (sends[0][0] == sends[1][0]).all(), (nib, sends[0][0], sends[1][0])
        assert sends[0][1].tobytes() == sends[1][1].tobytes(), nib
        assert sends[0][0][:, 3].sum() == 0 and sends[0][0][:, 1].sum() > 3 * n
        for k, (kind, o) in enumerate(launches):   # and the host's wire of the same outputs
            d, r, h = eng.fetch(o)
            m, w, p, bad = sdist.wire_encode(d, r, h, affix=eng.bank.affixes(kind) if nib else None)
            assert list(sends[0][0][k][:4]) == [len(m), len(w), len(p), bad], (nib, k)
    assert spilled > 0   # the dense MU launch used spill regions (payloads classified in HBM too)


@pytest.mark.gpu
def test_exchange_overlays_on_device():
    """sdx_xchg_part.alt / aux (ABI 11): a launch with overflowed messages and two overlays -> the
    device wire equals the host wire_encode with the same overlays (last present level wins, nibble
    form), the aux parts have zero counts, and an overflow no overlay covers is counted bad."""
    from pysignalduino_amd import bank as bankmod
    dev = torch.device("cuda", 0)
    eng = runtime.Engine(bankmod.Bank(), 0)
    affix = eng.bank.affixes(runtime.KIND_MU)
    rng = np.random.default_rng(23)
    n = 5000
    d0, r0, h0 = synth_launch(rng, n, affix=affix)
    ovf = rng.random(n) < 0.2
    d0["status"][ovf] = runtime.ST_OVF_TILE
    d0["n_rec"][ovf] = 0
    d1, r1, h1 = synth_launch(rng, n, affix=affix, status_absent=0.5)
    d2, r2, h2 = synth_launch(rng, n, affix=affix, status_absent=0.8)
    d1["status"][ovf & (d1["status"] == runtime.ST_ABSENT) & (d2["status"] == runtime.ST_ABSENT)] = runtime.ST_OK
    p0 = _dev_launch(d0, r0, h0, dev, kind=runtime.KIND_MU)
    p0.overlays = [_dev_launch(d1, r1, h1, dev, kind=runtime.KIND_MU), _dev_launch(d2, r2, h2, dev, kind=runtime.KIND_MU)]
    q = _dev_launch(*synth_launch(rng, 700, affix=affix), dev, kind=runtime.KIND_MU)   # a second launch, no overlays
    flat = sdist._flatten([p0, q])
    assert [(a, x) for _, a, x in flat] == [(3, 0), (0, 0), (4, 1), (0, 1)]
    ex = _kernel_exchange(eng)
    s = torch.cuda.current_stream(dev)
    cnt = ex._count_pack_device(flat, s).cpu().numpy().reshape(4, runtime.XCHG_COUNTS)
    m, w, p, bad = sdist.wire_encode(d0, r0, h0, affix=affix, overlays=[(d1, r1, h1, None, None), (d2, r2, h2, None, None)])
    assert bad == 0 and list(cnt[0][:4]) == [n, len(w), len(p), 0], cnt[0]
    assert not cnt[2:].any()
    offs, nb, T = sdist._layout(cnt[None])
    sv = ex._bufs["send"].cpu().numpy()
    o = offs[0, 0]
    assert sv[o[0]: o[0] + 4 * n].tobytes() == m.tobytes()
    assert sv[o[1]: o[1] + 8 * len(w)].tobytes() == w.tobytes()
    assert sv[o[2]: o[2] + len(p)].tobytes() == p.tobytes()
    # an overflow no overlay covers
    hole = np.nonzero((d1["status"] == runtime.ST_ABSENT) & (d2["status"] == runtime.ST_ABSENT) & ~ovf)[0][:3]
    d0b = d0.copy()
    d0b["status"][hole] = runtime.ST_OVF_OUT
    p0b = _dev_launch(d0b, r0, h0, dev, kind=runtime.KIND_MU)
    p0b.overlays = p0.overlays
    cb = ex._count_pack_device(sdist._flatten([p0b]), s).cpu().numpy()
    assert cb[3] == 3


@pytest.mark.gpu
def test_exchange_pack_into_rank1_chunk_and_32_rank_unpack():
    """sdx_exchange_pack_into at a rank > 0 chunk of an in-place receive buffer gives the
    same bytes as the canonical wire, and sdx_exchange_unpack over SDX_XCHG_MAX_RANKS (32) ranks of
    fake wire sections rebuilds the concatenated job (the end sentinels at [32])."""
    dev = torch.device("cuda", 0)
    rng = np.random.default_rng(5)
    launches = [synth_launch(rng, n, spill=False) for n in (2500, 900)]
    parts = [_dev_launch(d, r, h, dev) for d, r, h in launches]
    ex = _kernel_exchange()
    flat = sdist._flatten(parts)
    s = torch.cuda.current_stream(dev)
    cnt_dev = ex._count_device(flat, s)
    mine = cnt_dev.cpu().numpy().astype(np.int64).reshape(2, runtime.XCHG_COUNTS)
    # rank 1 of 2: a rank 0 with other counts makes the chunk size T the larger one
    S = np.stack([mine + np.array([0, 7, 100, 0, 100, 0, 0, 0]), mine])
    offs, nb, T = sdist._layout(S)
    recv = torch.full((2 * T + 64,), 0xAB, dtype=torch.uint8, device=dev)
    work, wb = ex._work(flat, dev)
    lib = runtime.load_library()
    import ctypes
    hc = np.ascontiguousarray(mine.reshape(-1).astype(np.uint32))
    runtime._check(lib, lib.sdx_exchange_pack_into(None, ex._xparts(flat), len(flat), ctypes.c_void_p(work.data_ptr()), wb,
                                                   ctypes.c_void_p(cnt_dev.data_ptr()), hc.ctypes.data_as(ctypes.c_void_p),
                                                   ctypes.c_void_p(recv[T:].data_ptr()), T, ctypes.c_void_p(s.cuda_stream)))
    rv = recv.cpu().numpy()
    assert (rv[:T] == 0xAB).all() and (rv[2 * T:] == 0xAB).all()   # nothing outside the chunk
    for k, (d, r, h) in enumerate(launches):
        m, w, p, _ = sdist.wire_encode(d, r, h)
        o = T + offs[1, k]
        assert rv[o[0]: o[0] + 4 * len(m)].tobytes() == m.tobytes()
        assert rv[o[1]: o[1] + 8 * len(w)].tobytes() == w.tobytes()
        assert rv[o[2]: o[2] + len(p)].tobytes() == p.tobytes()
    # 32 ranks: launch 1's wire sections, each rank a different slice of messages
    m, w, p, _ = sdist.wire_encode(*launches[1])
    nrec = (m & 0xFFFF).astype(np.int64)
    rb = np.concatenate([[0], np.cumsum(nrec)])
    pb = np.concatenate([[0], np.cumsum(w["payload_len"].astype(np.int64))])
    cuts = np.linspace(0, len(m), 33).astype(np.int64)
    buf, sec, Sr = bytearray(), [], []
    for i in range(32):
        a, b = cuts[i], cuts[i + 1]
        ra, rb_ = rb[a], rb[b]
        parts_i = (m[a:b].tobytes(), w[ra:rb_].tobytes(), p[pb[ra]: pb[rb_]].tobytes())
        o = []
        for x in parts_i:
            o.append(len(buf))
            buf += x + b"\0" * ((-len(x)) % 16)
        sec.append(o)
        Sr.append([b - a, rb_ - ra, pb[rb_] - pb[ra], 0, pb[rb_] - pb[ra]])
    tb = torch.from_numpy(np.frombuffer(bytes(buf), np.uint8).copy()).to(dev)
    gd, gr, gh = sdist.unpack_device(tb, np.array(Sr, np.int64), sec)
    ed, er, eh = sdist.wire_decode([(m, w, p)])
    assert gd.cpu().numpy().tobytes() == ed.tobytes()
    assert gr.cpu().numpy().tobytes() == er.tobytes()
    assert gh.cpu().numpy().tobytes() == eh.tobytes()


def _run_worker(name, env_extra, timeout=240):
    import subprocess
    import sys
    worker = os.path.join(os.path.dirname(os.path.abspath(__file__)), name)
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()), **env_extra)
    return subprocess.run([sys.executable, worker], env=env, capture_output=True, text=True, timeout=timeout)


@pytest.mark.gpu
def test_exchange_rccl_world1():
    """The bench's N > 1 exchange over a real RCCL process group (world size 1, cuda:0): the
    pipelined count all-gather, device packing and data all-gather on the exchange stream, two
    double-buffered steps of MU + MC launches; gathered buffers == the rank's own outputs in
    canonical form.  Runs in a child process (its own process group), bounded by a timeout."""
    r = _run_worker("rccl_exchange_worker.py", {}, timeout=150)
    assert r.returncode == 0 and r.stdout.strip().endswith("OK"), (r.returncode, r.stdout[-2000:], r.stderr[-4000:])


BRANCH_ENV = {"sync": {}, "pipelined": {"SDX_XCHG_PIPELINE": "1"},
              "defer": {"SDX_XCHG_PIPELINE": "1", "SDX_XCHG_DEFER": "1"}}


def _world2(mode, timeout=120, world=2, branch="sync"):
    """world ranks of dist_gpu_worker.py on cuda:0 over gloo; ``branch``: the exchange's synchronous
    gloo branch, or the pipelined branch an RCCL run takes (eager or deferred count + pack), forced
    over gloo."""
    import subprocess
    import sys
    worker = os.path.join(os.path.dirname(os.path.abspath(__file__)), "dist_gpu_worker.py")
    port = str(_free_port())
    env = {k: v for k, v in os.environ.items() if k not in ("SDX_XCHG_PIPELINE", "SDX_XCHG_DEFER")}
    env.update(BRANCH_ENV[branch])
    procs = [subprocess.Popen([sys.executable, worker], env=dict(env, MASTER_ADDR="127.0.0.1", MASTER_PORT=port,
                                                                 RANK=str(r), WORLD_SIZE=str(world), SDX_WORKER_MODE=mode),
                              stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True) for r in range(world)]
    outs = []
    for p in procs:
        try:
            o, e = p.communicate(timeout=timeout)
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            raise
        outs.append((p.returncode, o, e))
    bad = [(rank, rc, o[-2000:], e[-4000:]) for rank, (rc, o, e) in enumerate(outs)
           if not (rc == 0 and o.strip().endswith("OK"))]
    assert not bad, bad    # every failing rank's output (a rank that died takes its peer down with it)


@pytest.mark.gpu
@pytest.mark.parametrize("branch", ["sync", "pipelined", "defer"])
def test_world2_real_kernels_match_unsharded(branch):
    """Config 5's path at world size 2 on the one GPU (gloo, both ranks on cuda:0): each rank
    demodulates its contiguous shard of a real MU + MS + MC batch with the product launches
    (ShardedDemodulator: grouped order, spill regions), the exchange (nibble wire form) gathers two
    double-buffered steps, and the gathered descriptors, records and heap equal an un-sharded device
    run (canonical form) byte for byte -- through the synchronous gloo branch and through the
    pipelined branch RCCL runs (eager and deferred)."""
    _world2("pipelined", branch=branch)


@pytest.mark.gpu
@pytest.mark.parametrize("branch", ["sync", "pipelined", "defer"])
def test_world2_overflow_reruns_match_unsharded(branch):
    """a corpus and capacities that force ST_OVF_OUT / ST_OVF_TILE (dense MU corpus,
    one record per message, no spill workspace; MC frames of 129..800 hex characters): the ranks
    re-run their overflowed messages into overlays inside the exchange (no RuntimeError), every rank
    recounts, and the gathered results equal the un-sharded Engine.run byte for byte."""
    _world2("overflow", branch=branch)


@pytest.mark.gpu
@pytest.mark.parametrize("branch", ["sync", "defer"])
def test_world2_one_rank_overflows(branch):
    """Only rank 1 overflows and re-runs; rank 0 takes part in the recount only."""
    _world2("overflow1", branch=branch)


@pytest.mark.gpu
@pytest.mark.parametrize("branch", ["sync", "pipelined"])
def test_world2_collective_sizes(branch):
    """ADVICE r04 / VERDICT r04 #1: a peer's wire larger than this rank's whole send capacity is
    gathered correctly, and a mismatched number of launches raises ExchangeMismatch on both ranks."""
    _world2("sizes", branch=branch)


@pytest.mark.gpu
def test_world2_sharded_demodulate_batch_dicts():
    """ShardedDemodulator.demodulate_batch (the product's sharded dict API) == SDProtocols.
    demodulate_batch of the whole list on both ranks: MU / MS with general-path messages and host
    conversion errors on both shards, MC fixed with long frames and a non-str frame."""
    _world2("dict")


@pytest.mark.gpu
@pytest.mark.parametrize("mode,branch", [("pipelined", "sync"), ("pipelined", "defer"), ("overflow", "defer"),
                                         ("dict", "sync"), ("dict", "pipelined")])
def test_world4_on_one_gpu_matches_unsharded(mode, branch):
    """The same at world size 4 (four gloo ranks on cuda:0): uneven shard boundaries, every rank's
    gathered stream / dict results equal the un-sharded run, on both exchange branches."""
    _world2(mode, timeout=150, world=4, branch=branch)


@pytest.mark.gpu
@pytest.mark.parametrize("branch", ["sync", "defer"])
def test_bench_self_launch_world2(branch):
    """``bench.py --gpus 2`` without a launcher starts 2 ranks itself and reports n_gpus 2 with the
    exchange's wire bytes (gloo rehearsal: both ranks on cuda:0); ``defer``: the bench's own N > 1
    step -- the deferred pipelined exchange an RCCL run takes -- over gloo."""
    import json
    import subprocess
    import sys
    bench = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "bench.py")
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env["SDX_DIST_BACKEND"] = "gloo"
    env["SDX_XCHG_PIPELINE"] = "1" if branch == "defer" else "0"
    r = subprocess.run([sys.executable, bench, "--gpus", "2", "--steps", "2", "--warmup", "1", "--msgs", "30000",
                        "--no-cpu"], env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-4000:])
    line = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(line) == 1, r.stdout
    res = json.loads(line[0])
    assert res["n_gpus"] == 2 and res["config"]["parallelism"] == "dp2"
    assert res["exchange"]["wire_bytes_per_rank_per_step"] > 0
    assert res["exchange"]["branch"] == ("pipelined" if branch == "defer" else "sync"), res["exchange"]


@pytest.mark.gpu
@pytest.mark.parametrize("branch", ["sync", "defer"])
def test_config5_rehearsal_world8_on_one_gpu(branch):
    """Config 5's shape on the one GPU: eight gloo ranks on cuda:0, each with a mixed MU/MS/MC shard
    (300k messages here; the full 1M-per-rank run is profiles/r04/s3/config5_rehearsal/), the product
    exchange and the device unpack of the whole job: every rank's own wire chunk equals the host
    encoder's wire of its launches, the job sizes add up and all ranks hold identical bytes."""
    import subprocess
    import sys
    tool = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools", "config5_rehearsal.py")
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK")}
    out = os.path.join(os.environ.get("TMPDIR", "/tmp"), f"c5_{os.getpid()}")
    r = subprocess.run([sys.executable, tool, "--world", "8", "--msgs", "300000", "--out", out, "--timeout", "130",
                        "--branch", branch],
                       env=env, capture_output=True, text=True, timeout=145)
    assert r.returncode == 0 and r.stdout.strip().endswith("OK"), (r.stdout[-3000:], r.stderr[-3000:])
