"""Standalone time of the exchange's sender kernels (sdx_exchange_count + sdx_exchange_pack) on the
bench step's outputs (1M messages: MU/MS/MC 1/3 each), and of the receiver rebuild
(sdx_exchange_unpack) at world 1.  usage: python tools/time_exchange.py [msgs] [reps] [raw|scan]
(raw: payloads without the nibble form; scan: the exchange classifies every payload itself instead of
reading the counts the kernels wrote, ABI 12)"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch

from pysignalduino_amd import bank as bankmod, dist as sdist, runtime, synth


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 10
    mode = sys.argv[3] if len(sys.argv) > 3 else ""
    nib = mode != "raw"
    bk = bankmod.Bank()
    eng = runtime.Engine(bk, 0)
    P = bk.protocols
    per = {"MU": n // 3, "MS": n // 3, "MC": n - 2 * (n // 3)}
    parts = []
    for k, s in (("MU", 42), ("MS", 43), ("MC", 44)):
        c = (synth.mu_corpus if k == "MU" else synth.ms_corpus if k == "MS" else synth.mc_corpus)(P, per[k], seed=s)
        bd = eng.to_device_mc(c) if k == "MC" else eng.to_device_pulses(c)
        caps = {"MU": (12, 320), "MS": (4, 64), "MC": (4, 96)}[k]
        o = eng.alloc_out(c.n, caps[0] * c.n + 4096, caps[1] * c.n + 65536, eng.pulses_work_bytes(c.n) if k != "MC" else 0,
                          wire=mode != "scan")
        if k == "MC":
            eng.launch_mc(bd, o)
        else:
            eng.launch_pulses(runtime.KIND_MU if k == "MU" else runtime.KIND_MS, bd, o)
        parts.append(sdist.Part.from_out(o, {"MU": runtime.KIND_MU, "MS": runtime.KIND_MS, "MC": runtime.KIND_MC}[k]
                                         if nib else runtime.KIND_RAW))
    torch.cuda.synchronize()
    ex = sdist.Exchange.__new__(sdist.Exchange)
    ex._bufs, ex.engine = {}, eng if nib else None
    pt = sdist._flatten(parts)
    s = torch.cuda.current_stream()
    cnt = ex._count_pack_device(pt, s)
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        cnt = ex._count_pack_device(pt, s)
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    S = cnt.cpu().numpy().astype(np.int64).reshape(1, 3, runtime.XCHG_COUNTS)
    offs, nb, T = sdist._layout(S)
    wire = int(nb.sum())
    src = sum(int(p.cursor[0]) * 16 + int(p.cursor[1]) + 8 * p.n for p in parts)
    tu = []
    for _ in range(3):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for k in range(3):
            sdist.unpack_device(ex._bufs["send"], S[:, k, :], [offs[0, k]], ex.engine, parts[k].kind)
        e1.record()
        torch.cuda.synchronize()
        tu.append(e0.elapsed_time(e1))
    print(f"[{mode or 'nibble'}] count+pack {np.median(ts) * 1e3:.1f} us (min {min(ts) * 1e3:.1f}); wire {wire / 1e6:.2f} MB "
          f"(source desc+rec+heap {src / 1e6:.2f} MB); {wire / (min(ts) * 1e-3) / 1e9:.0f} GB/s of wire; "
          f"unpack x3 (world 1, incl. host sync) {min(tu) * 1e3:.0f} us; counts {S[0].tolist()}", flush=True)


if __name__ == "__main__":
    main()
