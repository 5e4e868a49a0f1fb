"""Child process of tests/test_dist.py::test_exchange_rccl_world1 (GPU box only).

Runs the pipelined dist.Exchange the bench uses for N > 1 over a real RCCL ("nccl") process
group of world size 1 on cuda:0: two steps of MU + MC launches into double-buffered outputs,
each step's exchange (count all-gather, sdx_exchange_pack, data all-gather on the exchange
stream) overlapping the next step's kernels.  At world size 1 the gathered buffers must equal
the rank's own outputs in canonical form (dist.canonical) byte for byte.  Prints "OK" on success.
"""
import os
import sys

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from pysignalduino_amd import bank as bankmod, dist as sdist, runtime, synth  # noqa: E402


def main():
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", sys.argv[1] if len(sys.argv) > 1 else "29533")
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    bk = bankmod.Bank()
    eng = runtime.Engine(bk, 0)
    corp = {"MU": synth.mu_corpus(bk.protocols, 3000, seed=71), "MC": synth.mc_corpus(bk.protocols, 3000, seed=72)}
    bds = {k: (eng.to_device_mc(c) if k == "MC" else eng.to_device_pulses(c)) for k, c in corp.items()}
    outs = [{k: eng.alloc_out(c.n, 12 * c.n + 4096, 320 * c.n + 65536,
                              eng.pulses_work_bytes(c.n) if k == "MU" else 0) for k, c in corp.items()}
            for _ in range(2)]
    stream = torch.cuda.current_stream(dev)
    ex = sdist.Exchange()
    assert dist.get_backend() == "nccl"
    snaps = []
    for j in range(2):
        o = outs[j % 2]
        eng.launch_pulses(runtime.KIND_MU, bds["MU"], o["MU"])
        eng.launch_mc(bds["MC"], o["MC"])
        ex.submit([(o[k]["desc"], o[k]["rec"], o[k]["heap"], bds[k]["n"], o[k]["cursor"]) for k in ("MU", "MC")],
                  stream)
        if j == 1:   # step 0's exchange completed inside this submit
            snaps.append(ex.gathered())
    ex.flush()
    assert ex.stream is not None, "the nccl path must run on the exchange stream"
    snaps.append(ex.gathered())
    torch.cuda.synchronize()
    for j, got in enumerate(snaps):
        o = outs[j % 2]
        for (gd, gr, gh), k in zip(got, ("MU", "MC")):
            d, r, h = eng.fetch(o[k])
            assert len(r) > 0, f"step {j} {k}: no results"
            cd, cr, ch = sdist.canonical(d, r, h)
            assert gd.cpu().numpy().tobytes() == cd.tobytes(), f"step {j} {k}: desc differs"
            assert gr.cpu().numpy().tobytes() == cr.tobytes(), f"step {j} {k}: records differ"
            assert gh.cpu().numpy().tobytes() == ch.tobytes(), f"step {j} {k}: heap differs"
    dist.destroy_process_group()
    print("OK", flush=True)


if __name__ == "__main__":
    main()
