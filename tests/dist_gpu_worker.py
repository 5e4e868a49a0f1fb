"""Rank process of tests/test_dist.py::test_world2_real_kernels_match_unsharded (GPU box only).

World size 2 over gloo with both ranks on cuda:0 (the one-GPU rehearsal of config 5): each rank
demodulates its contiguous shard of one global MU + MS + MC batch with the product launches
(grouped order + spill regions for MU/MS), runs two pipelined Exchange steps (double-buffered
outputs), and checks the gathered (desc, rec, heap) of every launch against an un-sharded device
run of the whole batch in canonical form, byte for byte.  Prints "OK" on success.
"""
import os
import sys

import numpy as np
import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from pysignalduino_amd import bank as bankmod, dist as sdist, runtime, synth  # noqa: E402

N = 12000   # per kind: shards of 6000 >= GROUP_MIN, so MU/MS run grouped with spill regions


def subset(pb, lo, hi):
    return pb.subset(np.arange(lo, hi))


def main():
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    bk = bankmod.Bank()
    eng = runtime.Engine(bk, 0)
    P = bk.protocols
    full = {"MU": synth.mu_corpus(P, N, seed=81), "MS": synth.ms_corpus(P, N, seed=82),
            "MC": synth.mc_corpus(P, N, seed=83)}
    kinds = ("MU", "MS", "MC")
    lo, hi = sdist.shard_bounds(N, rank, world)
    shard = {k: subset(full[k], lo, hi) for k in kinds}
    bds = {k: (eng.to_device_mc(c) if k == "MC" else eng.to_device_pulses(c)) for k, c in shard.items()}

    def alloc(n, k):
        return eng.alloc_out(n, 12 * n + 4096, 320 * n + 65536, eng.pulses_work_bytes(n) if k != "MC" else 0)

    def launch(k, bd, o):
        if k == "MC":
            eng.launch_mc(bd, o)
        else:
            eng.launch_pulses(runtime.KIND_MU if k == "MU" else runtime.KIND_MS, bd, o)

    outs = [{k: alloc(hi - lo, k) for k in kinds} for _ in range(2)]
    ex = sdist.Exchange()
    stream = torch.cuda.current_stream(dev)
    snaps = []
    for j in range(2):
        o = outs[j % 2]
        for k in kinds:
            o[k]["cursor"].zero_()
            launch(k, bds[k], o[k])
        ex.submit([(o[k]["desc"], o[k]["rec"], o[k]["heap"], bds[k]["n"], o[k]["cursor"]) for k in kinds], stream)
        snaps.append([tuple(t.cpu().numpy() for t in g) for g in ex.gathered()])
    ex.flush()
    assert ex.world == 2 and dist.get_world_size() == 2
    # the un-sharded device run of the whole batch, canonicalised on the host
    for k in kinds:
        bd = eng.to_device_mc(full[k]) if k == "MC" else eng.to_device_pulses(full[k])
        o = alloc(N, k)
        launch(k, bd, o)
        d, r, h = eng.fetch(o)
        assert not np.isin(d["status"], (runtime.ST_OVF_OUT, runtime.ST_OVF_TILE)).any(), k
        cd, cr, ch = sdist.canonical(d, r, h)
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


if __name__ == "__main__":
    main()
