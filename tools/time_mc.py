"""Kernel time of the MC launches (k_mc<4> + k_mc<8,long>) for the library named by SDX_LIB
(variant timing).  usage: SDX_LIB=path/to/libsdx_variant.so python tools/time_mc.py [n] [reps]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from pysignalduino_amd import bank as bankmod, runtime, synth


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 333334
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 10
    runtime.load_library()
    bk = bankmod.Bank()
    eng = runtime.Engine(bk, 0)
    mc = synth.mc_corpus(bk.protocols, n, seed=44)
    bd = eng.to_device_mc(mc)
    out = eng.alloc_out(mc.n, 4 * mc.n + 4096, 96 * mc.n + 65536)
    eng.launch_mc(bd, out)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ts = []
    for _ in range(reps):
        out["cursor"].zero_()
        e0.record()
        eng.launch_mc(bd, out)
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    print(os.path.basename(os.environ.get("SDX_LIB", "libsdx.so")), f"MC {min(ts):.3f} ms", flush=True)


if __name__ == "__main__":
    main()
