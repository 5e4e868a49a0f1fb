#!/usr/bin/env python3
"""MN (FSK) benchmark: MN frames/s through sdx_demod_mn, full MN bank.

One step = one sdx_demod_mn launch (parser mode, MNParser.rfmode = None: all 19 'modulation'
protocols tried per frame) over ``--frames`` synthetic MN frames resident in HBM
(pysignalduino_amd.synth.mn_frames: valid frames of every protocol family with correct checksums,
15 % with one corrupted nibble, 25 % random hex).  Prints ONE JSON line in the bench.py format:
value = frames/s; roofline of k_mn with its algorithmic bytes (hex characters + offsets read,
descriptors + result records + payload bytes written, DESIGN.md "MN"); cpu_baseline = the
Python oracle (oracle/mn_oracle.py, one core) of the same per-frame work on a bounded sample.

usage: python tools/bench_mn.py [--frames 1000000 --steps 5 --warmup 2]
"""
from __future__ import annotations

import argparse
import json
import os
import platform
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
HBM_PEAK = 8.0e12


def cpu_baseline(hexes, budget_s):
    from oracle import mn_oracle as M
    from oracle.sd_oracle import OracleBank
    ob = OracleBank()

    def run(sample):
        t0 = time.perf_counter()
        for h in sample:
            M.mn_parse(ob, h, None, None, None)
        return len(sample) / (time.perf_counter() - t0)

    probe = run(hexes[:500])
    k = int(max(500, min(len(hexes), probe * budget_s)))
    v = run(hexes[:k])
    return {"value": v, "unit": "frames/s", "cores": 1, "kind": "port",
            "sample": f"oracle/mn_oracle.py mn_parse (Python, the reference's per-protocol loop and methods "
                      f"restated), first {k} bench frames, rfmode None; {platform.processor() or platform.machine()}"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=1_000_000)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--cpu-seconds", type=float, default=15.0)
    ap.add_argument("--no-cpu", action="store_true")
    args = ap.parse_args()
    import torch
    from pysignalduino_amd import bank as bankmod, runtime, synth
    torch.cuda.set_device(0)
    bk = bankmod.Bank()
    eng = runtime.Engine(bk, 0)
    cache = os.path.join(os.environ.get("TMPDIR", "/tmp"), f"sdx_mn_{args.frames}_46.npz")
    if os.path.exists(cache):
        z = np.load(cache)
        data, offsets = z["data"], z["offsets"]
    else:
        fr = synth.mn_frames(args.frames, seed=46)
        bs = [h.encode("ascii") for h, _, _, _ in fr]
        offsets = np.zeros(len(bs) + 1, np.int64)
        np.cumsum([len(b) for b in bs], out=offsets[1:])
        data = np.frombuffer(b"".join(bs), np.uint8).copy()
        np.savez(cache, data=data, offsets=offsets)
    n = len(offsets) - 1
    bd = {"hex": torch.from_numpy(np.concatenate([data, np.zeros(16, np.uint8)])).cuda(), "offsets": torch.from_numpy(offsets).cuda(), "n": n}
    elig = (1 << len(bk.mn_pids)) - 1
    out = eng.alloc_out(n, 20 * n + 4096, int(4 * offsets[-1]) + 160 * n + 65536)
    stream = torch.cuda.current_stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)

    def step():
        out["cursor"].zero_()
        eng.launch_mn(bd, out, elig=elig)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    cur = out["cursor"].cpu().numpy()
    if cur[2] != 0:
        raise SystemExit(f"result capacity overflow in the bench configuration ({cur})")
    kt = []
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        out["cursor"].zero_()
        e0.record(stream)
        eng.launch_mn(bd, out, elig=elig)
        e1.record(stream)
        torch.cuda.synchronize()
        kt.append(e0.elapsed_time(e1) * 1e-3)
    dt = time.perf_counter() - t0
    cur = out["cursor"].cpu().numpy().astype(np.int64)
    nrec, nheap = int(cur[0]), int(cur[1])
    # k_mn algorithmic bytes: hex characters + offsets[n+1] read; desc (8 B/frame), result
    # records (16 B each) and payload bytes written
    alg = int(offsets[-1]) + 8 * (n + 1) + 8 * n + 16 * nrec + nheap
    km = float(np.mean(kt))
    achieved = alg / km
    traffic = None
    tpath = os.path.join(REPO, "profiles", "r01", "pmc_traffic_mn.json")
    if os.path.exists(tpath):
        tj = json.load(open(tpath))
        if tj.get("_config", {}).get("frames") == n and tj.get("k_mn", {}).get("traffic_bytes"):
            traffic = float(tj["k_mn"]["traffic_bytes"])
    res = {
        "metric": "MN (FSK) frames/sec demodulated (full MN bank, MNParser protocol loop, SURVEY §8(f) 2)",
        "value": n * args.steps / dt, "unit": "frames/s", "n_gpus": 1, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": 1e3 * dt / args.steps, "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
        "dtype": "u8+f64", "data": "synthetic MN frames (pysignalduino_amd/synth.py mn_frames)",
        "config": {"workload": "MN hex frames x 19 'modulation' protocols (rfmode None), valid checksums of "
                               "every method family + 15% corrupted + 25% random hex",
                   "frames": n, "hex_bytes": int(offsets[-1]), "results": nrec, "payload_bytes": nheap},
        "per_kernel_ms": {"k_mn": 1e3 * km},
        "roofline": {"bound": "hbm", "achieved": achieved / 1e9, "peak": HBM_PEAK / 1e9, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK, "traffic": traffic, "kernel": "k_mn",
                     "alg_bytes_per_launch": alg},
    }
    if not args.no_cpu:
        hexes = [data[offsets[i]: offsets[i + 1]].tobytes().decode("ascii") for i in range(min(n, 400_000))]
        res["cpu_baseline"] = cpu_baseline(hexes, args.cpu_seconds)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
