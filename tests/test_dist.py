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
    q.put((rank, got, got_multi, got_half, steps))
    dist.destroy_process_group()


def test_shard_bounds():
    for n in (0, 1, 7, 100, 1001):
        for w in (1, 2, 3, 8):
            spans = [sdist.shard_bounds(n, r, w) for r in range(w)]
            assert spans[0][0] == 0 and spans[-1][1] == n
            assert all(spans[i][1] == spans[i + 1][0] for i in range(w - 1))
            assert max(b - a for a, b in spans) - min(b - a for a, b in spans) <= 1


def test_gloo_world2_allgather_matches_unsharded():
    from pysignalduino_amd import bank
    P = bank.load_protocols()
    pb = synth.mu_corpus(P, 120, seed=5)
    msgs = [pb.to_msg_dict(i) for i in range(pb.n)]
    pids = bank.Bank().mu_pids
    full = decode(*encode(_oracle_results(msgs), pids), pids)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, msgs, pids, q)) for r in range(2)]
    for p in procs:
        p.start()
    outs = [q.get(timeout=300) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    halves = []
    for r in range(2):
        lo, hi = sdist.shard_bounds(len(msgs), r, 2)
        halves += full[lo: lo + (hi - lo) // 2]
    for rank, got, got_multi, got_half, steps in outs:
        assert got == full, f"rank {rank} gathered stream differs"
        assert got_multi == full, f"rank {rank}: allgather_streams differs"
        assert got_half == halves, f"rank {rank}: second launch of allgather_streams differs"
        assert steps == [[full], [halves, full]], f"rank {rank}: Exchange steps differ"


def synth_launch(rng, n, spill=True):
    """Launch outputs shaped like k_pulses writes them: records per tile of 64 messages in a shuffled
    tile order, tile pieces of the heap 16-byte aligned with gaps, RAISED and empty messages, and
    (``spill``) records past the used range that no message owns."""
    nrec = rng.integers(0, 7, size=n) * (rng.random(n) < 0.8)
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
                ln = int(rng.integers(0, 40))
                heap += bytes(rng.integers(32, 127, size=ln, dtype=np.uint8))
                recs.append((len(heap) - ln, ln, int(rng.integers(0, 129)), int(rng.integers(0, 300)), int(m)))
        heap += b"\0" * ((-len(heap)) % 16 + 16 * int(rng.integers(0, 2)))
    if spill:   # written but unowned records (an abandoned tile region)
        for _ in range(5):
            recs.append((0, 3, 1, 1, int(rng.integers(0, n))))
    rec = np.array(recs, runtime.RES_DT) if recs else np.zeros(0, runtime.RES_DT)
    return desc, rec, np.frombuffer(bytes(heap), np.uint8).copy()


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


def _dev_launch(desc, rec, heap, dev, cursor=None):
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a).view(np.uint8).copy() if len(a) else  # noqa: E731
                                   np.zeros(16, np.uint8)).to(dev)
    cur = torch.tensor(cursor if cursor is not None else [len(rec), len(heap), 0, 0], dtype=torch.int32, device=dev)
    return (t(desc), t(rec), t(heap), len(desc), cur)


@pytest.mark.gpu
def test_exchange_kernels_match_host_wire():
    """sdx_exchange_count / sdx_exchange_pack (HIP) == the numpy wire form for K = 3 launches laid
    out like k_pulses output (shuffled tiles, padded heap, RAISED / empty / unowned records), and
    sdx_exchange_unpack over 3 ranks' sections == wire_decode; an out-of-range message is counted bad."""
    dev = torch.device("cuda", 0)
    rng = np.random.default_rng(3)
    launches = [synth_launch(rng, n) for n in (1, 3000, 20000)]
    parts = [_dev_launch(d, r, h, dev) for d, r, h in launches]
    ex = sdist.Exchange.__new__(sdist.Exchange)
    ex._bufs = {}
    pt = [sdist._part_tuple(p) for p in parts]
    s = torch.cuda.current_stream(dev)
    cnt = ex._count_pack_device(pt, s).cpu().numpy().reshape(3, 4)
    want = [sdist.wire_encode(d, r, h) for d, r, h in launches]
    for k, (m, w, p, bad) in enumerate(want):
        assert list(cnt[k]) == [len(m), len(w), len(p), bad], (k, cnt[k])
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
    cnt2 = ex._count_pack_device(pt, s).cpu().numpy().reshape(3, 4)
    assert (cnt2 == cnt).all()
    assert (ex._bufs["send"].cpu().numpy()[:T] == sv[:T]).all()
    # unpack: three "ranks" = the three launches' wire sections of one buffer
    Su = np.array([[len(m), len(w), len(p)] for m, w, p, _ in want], np.int64)
    gd, gr, gh = sdist.unpack_device(ex._bufs["send"], Su, [offs[0, k] for k in range(3)])
    ed, er, eh = sdist.wire_decode([(m, w, p) for m, w, p, _ in want])
    assert gd.cpu().numpy().tobytes() == ed.tobytes()
    assert gr.cpu().numpy().tobytes() == er.tobytes()
    assert gh.cpu().numpy().tobytes() == eh.tobytes()
    # a cursor short of the records written: the owning messages are "bad"
    d, r, h = launches[1]
    bad_parts = [sdist._part_tuple(_dev_launch(d, r, h, dev, [len(r) - 10, len(h), 0, 0]))]
    cb = ex._count_pack_device(bad_parts, s).cpu().numpy()
    assert cb[3] == sdist.wire_encode(d, r, h, nrec_written=len(r) - 10)[3] > 0


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


@pytest.mark.gpu
def test_world2_real_kernels_match_unsharded():
    """Config 5's path at world size 2 on the one GPU (gloo, both ranks on cuda:0): each rank
    demodulates its contiguous shard of a real MU + MS + MC batch with the product kernels (grouped
    order, spill regions), the pipelined Exchange gathers two steps, and the gathered descriptors,
    records and heap equal an un-sharded device run (canonical form) byte for byte."""
    import subprocess
    import sys
    worker = os.path.join(os.path.dirname(os.path.abspath(__file__)), "dist_gpu_worker.py")
    port = str(_free_port())
    procs = [subprocess.Popen([sys.executable, worker], env=dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=port,
                                                                 RANK=str(r), WORLD_SIZE="2"),
                              stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True) for r in range(2)]
    outs = []
    for p in procs:
        try:
            o, e = p.communicate(timeout=240)
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            raise
        outs.append((p.returncode, o, e))
    for rank, (rc, o, e) in enumerate(outs):
        assert rc == 0 and o.strip().endswith("OK"), (rank, rc, o[-2000:], e[-4000:])


@pytest.mark.gpu
def test_bench_self_launch_world2():
    """``bench.py --gpus 2`` without a launcher starts 2 ranks itself and reports n_gpus 2 with the
    exchange's wire bytes (gloo rehearsal: both ranks on cuda:0)."""
    import json
    import subprocess
    import sys
    bench = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "bench.py")
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env["SDX_DIST_BACKEND"] = "gloo"
    r = subprocess.run([sys.executable, bench, "--gpus", "2", "--steps", "2", "--warmup", "1", "--msgs", "30000",
                        "--no-cpu"], env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-4000:])
    line = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(line) == 1, r.stdout
    res = json.loads(line[0])
    assert res["n_gpus"] == 2 and res["config"]["parallelism"] == "dp2"
    assert res["exchange"]["wire_bytes_per_rank_per_step"] > 0
