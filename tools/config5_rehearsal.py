"""Config 5 at its stated size on ONE GPU: WORLD ranks (default 8, gloo, all on cuda:0) each
demodulate a 1M-message MU/MS/MC shard (the bench's per-rank workload: 8M messages in all), run the
product exchange (ShardedDemodulator: first pass with kernel-written wire counts, re-runs, nibble
wire) and unpack the WHOLE job on the device.  Checks, per rank:
  * its own chunk of the gathered wire == the host encoder's wire of its launch outputs (Engine.run,
    canonical form) -- the device count/pack at full size;
  * the gathered job's per-launch message / record counts == the sum of all ranks' counts;
  * every rank's SHA-256 of the whole receive buffer is the same (all-gathered digests).
Rank 0 prints one JSON line.  The RCCL / xGMI rate of the real 8-GPU run is not measured here (gloo
stages through host memory); this is the correctness rehearsal of the sizes.
--branch pipelined / defer runs the exchange's pipelined branch (the code an RCCL run executes: count
on the exchange stream, in-place pack, eager or deferred) over gloo; sync (default) the gloo branch.
usage: python tools/config5_rehearsal.py [--world 8] [--msgs 1000000] [--branch sync|pipelined|defer]
       [--out gpurun_out/c5]"""
import argparse
import hashlib
import json
import os
import socket
import subprocess
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def launcher(args):
    os.makedirs(args.out, exist_ok=True)
    port = str(_free_port())
    procs, logs = [], []
    for r in range(args.world):
        log = open(os.path.join(args.out, f"rank{r}.log"), "w")
        env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(args.world), MASTER_ADDR="127.0.0.1", MASTER_PORT=port)
        procs.append(subprocess.Popen([sys.executable, "-u", os.path.abspath(__file__), "--msgs", str(args.msgs),
                                       "--out", args.out, "--branch", args.branch], env=env, stdout=log,
                                      stderr=subprocess.STDOUT))
        logs.append(log)
    t0 = time.time()
    rc = 0
    for r, p in enumerate(procs):
        try:
            p.wait(timeout=max(1.0, args.timeout - (time.time() - t0)))
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            print(f"rank {r} timed out", flush=True)
            rc = 1
            break
        rc = rc or p.returncode
    for f in logs:
        f.close()
    with open(os.path.join(args.out, "rank0.log")) as fh:
        lines = fh.read().splitlines()
    print("\n".join(lines[-3:]), flush=True)
    return rc


def rank_main(args):
    import numpy as np
    import torch
    import torch.distributed as dist
    from pysignalduino_amd import bank as bankmod, dist as sdist, runtime, synth

    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.cuda.set_device(0)
    bk = bankmod.Bank()
    eng = runtime.Engine(bk, 0)
    P = bk.protocols
    per = {"MU": args.msgs // 3, "MS": args.msgs // 3, "MC": args.msgs - 2 * (args.msgs // 3)}
    t = time.time()
    corp = {"MU": synth.mu_corpus(P, per["MU"], seed=42 + 1000 * rank),
            "MS": synth.ms_corpus(P, per["MS"], seed=43 + 1000 * rank),
            "MC": synth.mc_corpus(P, per["MC"], seed=44 + 1000 * rank)}
    KIND = {"MU": runtime.KIND_MU, "MS": runtime.KIND_MS, "MC": runtime.KIND_MC}
    bds = {k: (eng.to_device_mc(c) if k == "MC" else eng.to_device_pulses(c)) for k, c in corp.items()}
    print(f"rank {rank}: shard of {args.msgs} messages generated in {time.time() - t:.1f} s", flush=True)
    sd = sdist.ShardedDemodulator(engine=eng, pipeline=args.branch != "sync", defer=args.branch == "defer")
    assert sd.world == world and sd.exchange.pipelined == (args.branch != "sync")
    t = time.time()
    parts = [sd.launch(KIND[k], bds[k]) for k in ("MU", "MS", "MC")]
    sd.submit(parts)
    sd.flush()
    torch.cuda.synchronize()
    t_x = time.time() - t
    ex = sd.exchange
    recv, S, offs, nb, T, K, kinds = ex.last
    print(f"rank {rank}: launches + exchange {t_x:.2f} s, {T / 1e6:.1f} MB per rank on the wire", flush=True)
    t = time.time()
    job = sd.gathered()
    torch.cuda.synchronize()
    t_u = time.time() - t
    # 1. this rank's chunk == the host encoder's wire of the same launches (canonical local run)
    rv = recv.cpu().numpy()
    for i, k in enumerate(("MU", "MS", "MC")):
        d, r, h = eng.run(KIND[k], bds[k])
        cd, cr, ch = sdist.canonical(d, r, h)
        m_h, w_h, p_h, bad = sdist.wire_encode(cd, cr, ch, affix=ex._affix(kinds[i]))
        assert bad == 0, (rank, k, bad)
        o = rank * T + offs[rank, i]
        m_d = rv[o[0]: o[0] + nb[rank, i, 0]].view(np.uint32)
        w_d = rv[o[1]: o[1] + nb[rank, i, 1]].view(runtime.WIRE_REC_DT)
        p_d = rv[o[2]: o[2] + nb[rank, i, 2]]
        assert np.array_equal(m_d, np.asarray(m_h, np.uint32)), (rank, k, "message words")
        assert w_d.tobytes() == np.asarray(w_h).tobytes(), (rank, k, "wire records")
        assert p_d.tobytes() == np.asarray(p_h).tobytes(), (rank, k, "payload bytes")
        # 2. the unpacked job's sizes
        gd, gr, gh = job[i]
        assert gd.numel() == runtime.DESC_DT.itemsize * int(S[:, i, 0].sum()), (rank, k, "desc size")
        assert gr.numel() == runtime.RES_DT.itemsize * int(S[:, i, 1].sum()), (rank, k, "rec size")
    # 3. every rank holds the same receive buffer
    dig = np.frombuffer(hashlib.sha256(rv[: world * T].tobytes()).digest()[:8], np.int64).copy()
    allg = [torch.zeros(1, dtype=torch.int64) for _ in range(world)]
    dist.all_gather(allg, torch.from_numpy(dig))
    assert len({int(a.item()) for a in allg}) == 1, "ranks received different bytes"
    dist.barrier()
    if rank == 0:
        print(json.dumps({"config": "config 5 rehearsal on one GPU (gloo, all ranks on cuda:0)", "world": world,
                          "exchange_branch": args.branch,
                          "msgs_per_rank": args.msgs, "msgs_total": world * args.msgs,
                          "records_total": int(S[:, :, 1].sum()), "wire_bytes_per_rank": int(T),
                          "launch_exchange_s_rank0": round(t_x, 3), "unpack_job_s_rank0": round(t_u, 3),
                          "checks": "own chunk == host wire of Engine.run (all kinds), job sizes, equal digests: OK"}),
              flush=True)
    dist.destroy_process_group()
    print("OK", flush=True)
    return 0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--msgs", type=int, default=1_000_000)
    ap.add_argument("--out", default="gpurun_out/c5")
    ap.add_argument("--timeout", type=float, default=600.0)
    ap.add_argument("--branch", default="sync", choices=("sync", "pipelined", "defer"))
    args = ap.parse_args()
    if "RANK" in os.environ:
        return rank_main(args)
    return launcher(args)


if __name__ == "__main__":
    sys.exit(main())
