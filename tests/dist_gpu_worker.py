"""Rank process of tests/test_dist.py's world-2 and world-4 GPU tests (GPU box only).

World size 2 over gloo with both ranks on cuda:0 (the one-GPU rehearsal of config 5).  Modes
(SDX_WORKER_MODE):
  pipelined  each rank demodulates its contiguous shard of one global MU + MS + MC batch with the
             product launches (ShardedDemodulator.launch: grouped order + spill regions for MU/MS),
             runs two pipelined exchange steps (double-buffered outputs, nibble wire form) and checks
             the gathered (desc, rec, heap) of every launch against an un-sharded device run of the
             whole batch in canonical form, byte for byte;
  overflow   the same with capacities and inputs that force overflows: MU on the dense corpus with a
             record capacity of one record per message (ST_OVF_OUT) and no spill workspace
             (ST_OVF_TILE), MC frames longer than 128 hex characters launched on k_mc alone (which hands
             them over as ST_OVF_TILE; the routed launch sends them to the general kernel) -- the exchange re-runs them into overlays on each rank before it ships, and
             the gathered results equal the un-sharded Engine.run (its own re-runs) byte for byte;
  overflow1  the overflow mode with only rank 1's MU launch overflowing (rank 0 has room): only that
             rank re-runs, every rank recounts;
  dict       ShardedDemodulator.demodulate_batch on msg_data dicts (general-path messages with
             multi-digit ids, messages whose host conversion raises) == SDProtocols.demodulate_batch of
             the whole list, on every rank;
  sizes      synthetic device launches: rank 0's outputs are small and exactly sized, rank 1's launch
             overflows and its re-run overlay carries 40x larger payloads, so the collective's size T
             exceeds everything rank 0 allocated; then rank 1 submits two launches where
             rank 0 submits one, which must raise ExchangeMismatch on both ranks.
SDX_XCHG_PIPELINE=1 runs the exchange's pipelined branch -- the one an RCCL run takes: counts behind
the step's kernels on the exchange stream, in-place pack into the receive chunk, recount after
re-runs -- over gloo (SDX_XCHG_DEFER=1: its deferred form, the bench's default); unset, gloo takes
the synchronous branch.  Prints "OK" on success.
"""
import os
import sys

import numpy as np
import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from pysignalduino_amd import bank as bankmod, dist as sdist, runtime, synth  # noqa: E402

N = 12000   # per kind: shards of 6000 >= GROUP_MIN, so MU/MS run grouped with spill regions
KIND = {"MU": runtime.KIND_MU, "MS": runtime.KIND_MS, "MC": runtime.KIND_MC}


def subset(pb, lo, hi):
    return pb.subset(np.arange(lo, hi))


def long_mc(P, mb, n_long, seed):
    """mb with n_long frames replaced by frames of 129..800 hex characters (synth.general_mc_frames)."""
    from pysignalduino_amd import packing
    frames = [(mb.hex(i), int(mb.clock[i]), int(mb.mcbitnum[i]), "Mc" if mb.mtype[i] else "MC", None)
              for i in range(mb.n)]
    rng = np.random.default_rng(seed)
    for j, f in zip(rng.choice(mb.n, n_long, replace=False), synth.general_mc_frames(P, n_long, seed=seed)):
        frames[int(j)] = f
    return packing.mc_batch_from_frames(frames)


def canon_full(eng, kind, bd):
    d, r, h = eng.run(KIND[kind], bd)
    assert not np.isin(d["status"], (runtime.ST_OVF_OUT, runtime.ST_OVF_TILE)).any(), kind
    return sdist.canonical(d, r, h)


def main():
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    mode = os.environ.get("SDX_WORKER_MODE", "pipelined")
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    bk = bankmod.Bank()
    eng = runtime.Engine(bk, 0)
    P = bk.protocols
    pipe = os.environ.get("SDX_XCHG_PIPELINE") == "1"
    sd = sdist.ShardedDemodulator(group=None, engine=eng, defer=os.environ.get("SDX_XCHG_DEFER") == "1")
    assert sd.world == world
    assert sd.exchange.pipelined == pipe, (sd.exchange.pipelined, pipe)
    if mode == "dict":
        return dict_mode(sd, P, rank)
    if mode == "sizes":
        return sizes_mode(sd, dev, rank)
    dense = mode in ("overflow", "overflow1")
    tight = dense and (mode == "overflow" or rank == 1)   # this rank's MU launch overflows
    full = {"MU": synth.mu_corpus(P, N, seed=81, noise_frac=0.0 if dense else 0.15), "MS": synth.ms_corpus(P, N, seed=82),
            "MC": synth.mc_corpus(P, N, seed=83)}
    if mode == "overflow":
        full["MC"] = long_mc(P, full["MC"], 40, seed=84)
    kinds = ("MU", "MS", "MC")
    lo, hi = sd.shard(N)
    shard = {k: subset(full[k], lo, hi) for k in kinds}
    bds = {k: (eng.to_device_mc(c) if k == "MC" else eng.to_device_pulses(c)) for k, c in shard.items()}

    def alloc(n, k):
        if tight and k == "MU":   # one record per message, no spill regions: ST_OVF_OUT and ST_OVF_TILE
            return eng.alloc_out(n, n, 40 * n, 0, wire=True)
        # the kernels write the exchange's counts (ABI 12) in the pipelined mode; the overflow mode's
        # MS / MC launches leave the classification to the exchange kernels
        return eng.alloc_out(n, 12 * n + 4096, 320 * n + 65536, eng.pulses_work_bytes(n) if k != "MC" else 0,
                             wire=not dense)

    outs = [{k: alloc(hi - lo, k) for k in kinds} for _ in range(2)]
    stream = torch.cuda.current_stream(dev)
    snaps = []
    for j in range(2):
        o = outs[j % 2]
        parts = []
        for k in kinds:
            o[k]["cursor"].zero_()
            if mode == "overflow" and k == "MC":   # k_mc alone (no routing): it hands the > 128-character frames over
                eng.launch_mc(bds[k], o[k])   # as ST_OVF_TILE, and the exchange re-runs them
                parts.append(sdist.Part.from_out(o[k], KIND[k], src=(KIND[k], bds[k], 0, -1)))
            else:
                parts.append(sd.launch(KIND[k], bds[k], o[k]))
        if dense and j == 0:   # the first pass really overflowed on this rank (or, overflow1, not)
            torch.cuda.synchronize()
            st = {k: o[k]["desc"][: (hi - lo) * 8].view(-1, 8)[:, 6].cpu().numpy() for k in kinds}
            assert (st["MU"] == runtime.ST_OVF_OUT).any() == tight, rank
            print("first-pass MU overflows: OUT", int((st["MU"] == runtime.ST_OVF_OUT).sum()), "TILE",
                  int((st["MU"] == runtime.ST_OVF_TILE).sum()), flush=True)
            assert (st["MC"] == runtime.ST_OVF_TILE).any() == (mode == "overflow"), rank
        rel = sd.submit(parts, stream)
        if not pipe:            # synchronous: this step is complete
            snaps.append([tuple(t.cpu().numpy() for t in g) for g in sd.gathered()])
        elif j >= 1:            # pipelined: the previous step completed inside this submit
            snaps.append([tuple(t.cpu().numpy() for t in g) for g in sd.gathered()])
            stream.wait_event(rel)
    sd.flush()
    if pipe:
        assert sd.exchange.stream is not None, "the pipelined branch runs on the exchange stream"
        snaps.append([tuple(t.cpu().numpy() for t in g) for g in sd.gathered()])
    assert len(snaps) == 2, len(snaps)
    if mode == "overflow" or (mode == "overflow1" and rank == 1):
        assert sd.exchange.reruns >= (4 if mode == "overflow" else 2), sd.exchange.reruns
    elif mode == "overflow1":
        assert sd.exchange.reruns == 0, sd.exchange.reruns
    # the nibble form is on: the wire carries fewer payload bytes than it delivers
    assert sd.exchange.heap_wire_bytes[-1] < 0.8 * sd.exchange.payload_bytes[-1], (sd.exchange.heap_wire_bytes,
                                                                                  sd.exchange.payload_bytes)
    # the un-sharded device run of the whole batch (Engine.run: its own re-runs), canonicalised on the host
    for k in kinds:
        bd = eng.to_device_mc(full[k]) if k == "MC" else eng.to_device_pulses(full[k])
        cd, cr, ch = canon_full(eng, k, bd)
        i = kinds.index(k)
        for j, snap in enumerate(snaps):
            gd, gr, gh = snap[i]
            assert gd.tobytes() == cd.tobytes(), (rank, j, k, "desc")
            assert gr.tobytes() == cr.tobytes(), (rank, j, k, "rec")
            assert gh.tobytes() == ch.tobytes(), (rank, j, k, "heap")
        assert len(cr) > N // 4, (k, len(cr))
    dist.barrier()
    dist.destroy_process_group()
    print("OK", flush=True)


def sizes_mode(sd, dev, rank):
    """a peer's wire larger than this rank's whole send capacity, and a
    deliberately mismatched number of launches."""
    n = 100
    desc = np.zeros(n, runtime.DESC_DT)
    desc["n_rec"] = 1
    desc["rec_begin"] = np.arange(n)
    plen = 4 if rank == 0 else 160
    rec = np.zeros(n, runtime.RES_DT)
    rec["payload_off"] = np.arange(n) * plen
    rec["payload_len"] = plen
    rec["proto"] = 1
    rec["bit_length"] = 8 * plen
    rec["msg"] = np.arange(n)
    heap = (np.arange(n * plen) % 23 + 65).astype(np.uint8)
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a).view(np.uint8).copy()).to(dev)  # noqa: E731
    cur = lambda: torch.tensor([n, n * plen, 0, 0], dtype=torch.int32, device=dev)  # noqa: E731
    if rank == 0:
        part = sdist.Part(t(desc), t(rec), t(heap), n, cur())
    else:   # overflowed first pass; the overlay holds the real (large) results
        d1 = desc.copy()
        d1["status"] = runtime.ST_OVF_OUT
        d1["n_rec"] = 0
        part = sdist.Part(t(d1), t(rec[:1]), t(heap[:16]), n, torch.tensor([0, 0, 0, 0], dtype=torch.int32, device=dev))

    def rerun(p):
        p.overlays.append(sdist.Part(t(desc), t(rec), t(heap), n, cur()))
        return p
    ex = sdist.Exchange(pipeline=sd.exchange.pipeline)
    rel = ex.submit([part], rerun=rerun)
    ex.flush()
    gd, gr, gh = (x.cpu().numpy() for x in ex.gathered()[0])
    assert ex.bytes_sent[-1] > 8 * 1024, ex.bytes_sent   # T: rank 1's wire, > rank 0's 1.6 KB of outputs
    want = []
    for r, pl in ((0, 4), (1, 160)):
        want += [((np.arange(pl) + i * pl) % 23 + 65).astype(np.uint8).tobytes() for i in range(n)]
    got = [gh[int(x["payload_off"]): int(x["payload_off"]) + int(x["payload_len"])].tobytes()
           for x in gr.view(runtime.RES_DT)]
    assert got == want, rank
    assert (gd.view(runtime.DESC_DT)["n_rec"] == 1).all()
    # rank 1 submits two launches where rank 0 submits one: ExchangeMismatch on both ranks
    ex2 = sdist.Exchange(pipeline=sd.exchange.pipeline)
    raised = None
    try:
        ex2.submit([sdist.Part(t(desc), t(rec), t(heap[: n * plen]), n, cur())] * (1 + rank))
        ex2.flush()
    except sdist.ExchangeMismatch as e:
        raised = str(e)
    assert raised is not None and "launches" in raised, (rank, raised)
    # and the ranks are still in step
    ex3 = sdist.Exchange(pipeline=sd.exchange.pipeline)
    ex3.submit([sdist.Part(t(desc), t(rec), t(heap), n, cur())])
    ex3.flush()
    assert ex3.gathered()[0][0].numel() == 2 * n * 8
    dist.barrier()
    dist.destroy_process_group()
    print("OK", flush=True)


def dict_mode(sd, P, rank):
    """ShardedDemodulator.demodulate_batch == SDProtocols.demodulate_batch on the whole list."""
    from pysignalduino_amd.sd_protocols import SDProtocols
    ref = SDProtocols(mc_mode="fixed")
    sd.protocols, sd._eng = ref, None     # the entry on the reference-shaped object's own engine
    for kind in ("MU", "MS"):
        pb = synth.mu_corpus(P, 5000, seed=91) if kind == "MU" else synth.ms_corpus(P, 5000, seed=92)
        msgs = [pb.to_msg_dict(i) for i in range(pb.n)]
        gen = synth.general_pulse_messages(P, kind, 60, seed=93)
        for j, g in enumerate(gen):                      # general-path messages on both ranks' shards
            msgs.insert(37 * j + 11, g)
        msgs[5] = dict(msgs[5], data=12345)              # host conversion raises (TypeError) on rank 0
        msgs[len(msgs) - 3] = dict(msgs[-3], data=None)  # and on rank 1
        got = sd.demodulate_batch(msgs, kind)
        want = ref.demodulate_batch(msgs, kind)
        assert len(got) == len(want) == len(msgs)
        for i, (g, w) in enumerate(zip(got, want)):
            if isinstance(w, BaseException):
                assert type(g) is type(w), (kind, i, g, w)
            else:
                assert g == w, (kind, i, g, w)
        assert sum(isinstance(w, list) and len(w) > 0 for w in want) > 500, kind
    mb = synth.mc_corpus(P, 4000, seed=94)
    frames = [mb.to_msg_dict(i) for i in range(mb.n)]
    for j, (h, c, L, t, v) in enumerate(synth.general_mc_frames(P, 30, seed=95)):
        frames.insert(100 * j + 7, {"raw_hex": h, "clock": c, "mcbitnum": L, "messagetype": t})
    frames[9] = {"raw_hex": 17, "clock": "1", "mcbitnum": "4"}   # not a str: ContractError on the host
    got = sd.demodulate_batch(frames, "MC")
    want = ref.demodulate_batch(frames, "MC")
    for i, (g, w) in enumerate(zip(got, want)):
        if isinstance(w, BaseException):
            assert type(g) is type(w), ("MC", i, g, w)
        else:
            assert g == w, ("MC", i, g, w)
    dist.barrier()
    dist.destroy_process_group()
    print("OK", flush=True)


if __name__ == "__main__":
    main()
