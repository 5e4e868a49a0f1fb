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


@pytest.mark.gpu
def test_exchange_pack_kernel_matches_torch_pack():
    """sdx_exchange_pack (HIP) == the torch-op packing, for a rank with lower ranks below it
    (re-based rec_begin / payload_off / msg, 16-byte heap copies plus tails), K = 3 launches."""
    dev = torch.device("cuda", 0)
    rng = np.random.default_rng(3)
    parts = []
    for k in range(3):
        nm, nr, nh = int(rng.integers(1, 5000)), int(rng.integers(0, 20000)), int(rng.integers(0, 300000))
        desc = torch.from_numpy(rng.integers(0, 255, size=nm * 8 + 64, dtype=np.uint8)).to(dev)
        rec = torch.from_numpy(rng.integers(0, 255, size=nr * 16 + 64, dtype=np.uint8)).to(dev)
        heap = torch.from_numpy(rng.integers(0, 255, size=nh + 64, dtype=np.uint8)).to(dev)
        cur = torch.tensor([nr, nh, 0, 0], dtype=torch.int32, device=dev)
        parts.append((desc, rec, heap, nm, cur))
    S = np.zeros((3, 3, 3), np.int64)
    for r in range(3):
        for k, (_, _, _, nm, cur) in enumerate(parts):
            S[r, k] = (nm, int(cur[0]), int(cur[1])) if r == 2 else rng.integers(0, 100000, size=3)
    nb, sec_off, total, base = sdist._layout(S, 2)
    a = torch.zeros(total, dtype=torch.uint8, device=dev)
    b = torch.zeros(total, dtype=torch.uint8, device=dev)
    sdist._pack_torch(parts, S, 2, sec_off, base, a)
    sdist._pack_device(parts, S, 2, sec_off, base, b, torch.cuda.current_stream(dev))
    torch.cuda.synchronize()
    assert torch.equal(a, b)


@pytest.mark.gpu
def test_exchange_rccl_world1():
    """The bench's N > 1 exchange over a real RCCL process group (world size 1, cuda:0): the
    pipelined count all-gather, device packing and data all-gather on the exchange stream, two
    double-buffered steps of MU + MC launches; gathered buffers == the rank's own outputs.  Runs
    in a child process (its own process group), bounded by a timeout."""
    import subprocess
    import sys
    worker = os.path.join(os.path.dirname(os.path.abspath(__file__)), "rccl_exchange_worker.py")
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()))
    r = subprocess.run([sys.executable, worker], env=env, capture_output=True, text=True, timeout=150)
    assert r.returncode == 0 and r.stdout.strip().endswith("OK"), (r.returncode, r.stdout[-2000:], r.stderr[-4000:])
