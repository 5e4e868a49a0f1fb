"""Child process of tests/test_dist.py::test_exchange_rccl_world1 (GPU box only).

Runs the pipelined dist.Exchange the bench uses for N > 1 over a real RCCL ("nccl") process
group of world size 1 on cuda:0: two steps of MU + MC launches into double-buffered outputs,
each step's exchange (count all-gather, sdx_exchange_pack, data all-gather on the exchange
stream) overlapping the next step's kernels, the wire in the nibble form (ShardedDemodulator over
the engine's bank).  At world size 1 the gathered buffers must equal the rank's own outputs in
canonical form (dist.canonical) byte for byte.  A third step's MU launch overflows its record
capacity: the exchange re-runs those messages on the exchange stream (an overlay) before packing,
and the gathered MU results equal Engine.run's.  Prints "OK" on success.
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
    sd = sdist.ShardedDemodulator(engine=eng)
    ex = sd.exchange
    assert dist.get_backend() == "nccl"
    KIND = {"MU": runtime.KIND_MU, "MC": runtime.KIND_MC}
    # step 2: the MU record capacity is one record per message (ST_OVF_OUT tiles)
    outs.append({"MU": eng.alloc_out(corp["MU"].n, corp["MU"].n, 40 * corp["MU"].n, eng.pulses_work_bytes(corp["MU"].n)),
                 "MC": outs[0]["MC"]})
    snaps = []
    for j in range(3):
        o = outs[j]
        o["MU"]["cursor"].zero_()
        o["MC"]["cursor"].zero_()
        parts = [sd.launch(KIND[k], bds[k], o[k]) for k in ("MU", "MC")]
        rel = sd.submit(parts, stream)
        if j >= 1:   # step j-1's exchange completed inside this submit
            snaps.append(ex.gathered())
            stream.wait_event(rel)
    sd.flush()
    assert ex.stream is not None, "the nccl path must run on the exchange stream"
    snaps.append(ex.gathered())
    torch.cuda.synchronize()
    assert ex.reruns == 1, ex.reruns
    assert ex.heap_wire_bytes[0] < 0.8 * ex.payload_bytes[0], (ex.heap_wire_bytes, ex.payload_bytes)
    want = {k: sdist.canonical(*eng.run(KIND[k], bds[k])) for k in ("MU", "MC")}
    for j, got in enumerate(snaps):
        for (gd, gr, gh), k in zip(got, ("MU", "MC")):
            cd, cr, ch = want[k]
            assert len(cr) > 0, f"step {j} {k}: no results"
            assert gd.cpu().numpy().tobytes() == cd.tobytes(), f"step {j} {k}: desc differs"
            assert gr.cpu().numpy().tobytes() == cr.tobytes(), f"step {j} {k}: records differ"
            assert gh.cpu().numpy().tobytes() == ch.tobytes(), f"step {j} {k}: heap differs"
    dist.destroy_process_group()
    print("OK", flush=True)


if __name__ == "__main__":
    main()
