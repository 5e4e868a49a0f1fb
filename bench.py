#!/usr/bin/env python3
"""Benchmark: RF messages/s demodulated (MU+MS+MC, full protocol bank) on 1..8 MI355X.

One "step" = one pass of the hot path over one batch resident in HBM: every MU message
(256 pulses) x the full MU bank, every MS message x the MS bank, every MC frame x the 12
clockrange protocols, results written in reference order -- and, for N > 1, the RCCL
all-gather of the decoded dmsg buffers (BASELINE config 5).  Weak scaling: each rank owns
``--msgs`` messages (1/3 of each type).

Prints ONE JSON line on rank 0 (contract in the task statement); see DESIGN.md §Measurement.
"""
from __future__ import annotations

import argparse
import json
import os
import platform
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

HBM_PEAK = 8.0e12  # B/s, MI355X spec (MI355X_MICROARCH.md)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--msgs", type=int, default=1_000_000, help="messages per rank (1/3 MU, 1/3 MS, 1/3 MC)")
    ap.add_argument("--cpu-seconds", type=float, default=20.0, help="budget of the CPU-baseline leg")
    ap.add_argument("--no-cpu", action="store_true")
    return ap.parse_args()


def cpu_baseline(mu, ms, mc, budget_s: float):
    """The plain-C oracle (oracle/sd_oracle_c.c, a restatement of the reference path: kind 'port')
    timed on this host over a bounded 1:1:1 MU/MS/MC sample of the SAME corpora the GPU
    demodulates: once on one core, once on all cores this process may use.  Each message is
    fully demodulated against the whole bank, with results written, as on the GPU."""
    from oracle import c_oracle as CO
    CO.build()
    bank = CO.CBank()
    cores = len(os.sched_getaffinity(0))
    if os.environ.get("OMP_NUM_THREADS", "").isdigit():  # the box's CPU share (16 per GPU)
        cores = min(cores, int(os.environ["OMP_NUM_THREADS"]))
    cores = max(1, min(cores, 64))

    def timed(k, threads):
        idx = np.arange(k)
        packs = [("MU", CO.pack_batch(mu.subset(idx))), ("MS", CO.pack_batch(ms.subset(idx))),
                 ("MC", CO.mc_batch(mc.subset(idx)))]
        t0 = time.perf_counter()
        for kind, pk in packs:
            CO.run(kind, pk, threads)
        return 3 * k / (time.perf_counter() - t0)

    # size the samples from a short probe so the whole leg stays within ~budget_s seconds
    probe = timed(min(300, mu.n, ms.n, mc.n), 1)
    k1 = int(max(300, min(mu.n, ms.n, mc.n, probe * budget_s * 0.35 / 3)))
    v1 = timed(k1, 1)
    kn = int(max(300, min(mu.n, ms.n, mc.n, v1 * cores * budget_s * 0.5 / 3)))
    vn = timed(kn, cores)
    return {"value": vn, "unit": "msgs/s", "cores": cores, "kind": "port", "value_1core": v1,
            "sample": f"oracle/sd_oracle_c.c (plain C, gcc -O2): {3 * kn} messages (1:1:1 MU/MS/MC, the "
                      f"first {kn} of each bench corpus) on {cores} threads; 1-core rate on {3 * k1} messages; "
                      f"{platform.processor() or platform.machine()}"}


def issue_view(pmc, t_kernel):
    """Instruction-issue utilisation of a launch from its committed PMC counts (the kernels are
    integer/branch code: HBM is not their binding limit). Ceilings at 2.4 GHz:
    VALU one wave64 instruction per 2 cycles per SIMD (4 SIMDs/CU, MI355X_MICROARCH.md), SALU
    one per cycle per CU; 256 CUs."""
    v, sa = pmc.get("sq_insts_valu"), pmc.get("sq_insts_salu")
    if not v or not sa:
        return None
    valu_peak, salu_peak = 256 * 4 * 2.4e9 / 2, 256 * 2.4e9
    return {"valu_insts": v, "salu_insts": sa, "valu_frac": v / t_kernel / valu_peak,
            "salu_frac": sa / t_kernel / salu_peak,
            "wait_frac": (pmc["sq_wait_any"] / pmc["sq_wave_cycles"]) if pmc.get("sq_wave_cycles") else None}


def main():
    args = parse()
    import torch
    import torch.distributed as dist
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # SDX_DIST_BACKEND=gloo rehearses the N > 1 code path on fewer GPUs than ranks (ranks share
    # devices round-robin); the driver's runs use RCCL ("nccl") with one GPU per rank
    backend = os.environ.get("SDX_DIST_BACKEND", "nccl")
    if backend != "nccl":
        local = local % max(1, torch.cuda.device_count())
    if world > 1:
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)

    from pysignalduino_amd import bank as bankmod, runtime, synth
    from pysignalduino_amd import dist as sdist
    bk = bankmod.Bank()
    P = bk.protocols
    eng = runtime.Engine(bk, local)
    n3 = args.msgs // 3
    mu = synth.mu_corpus(P, n3, seed=42 + 1000 * rank)
    ms = synth.ms_corpus(P, n3, seed=43 + 1000 * rank)
    mc = synth.mc_corpus(P, args.msgs - 2 * n3, seed=44 + 1000 * rank)
    bmu, bms, bmc = eng.to_device_pulses(mu), eng.to_device_pulses(ms), eng.to_device_mc(mc)
    outs = {
        "MU": eng.alloc_out(mu.n, 8 * mu.n + 4096, 200 * mu.n + 65536),
        "MS": eng.alloc_out(ms.n, 4 * ms.n + 4096, 64 * ms.n + 65536),
        "MC": eng.alloc_out(mc.n, 4 * mc.n + 4096, 96 * mc.n + 65536),
    }
    # the three launches' cursors are rows of one tensor: one fill per step resets them all
    cursors = torch.zeros((3, 4), dtype=torch.int32, device=dev)
    for i, k in enumerate(("MU", "MS", "MC")):
        outs[k]["cursor"] = cursors[i]
    stream = torch.cuda.current_stream(dev)
    # one event pair per kernel and timed step: the steps run back to back and are read after the
    # closing synchronize (no host round trip between steps)
    ev = [{k: [torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)] for k in outs}
          for _ in range(args.steps)]
    ktimes = {k: [] for k in outs}

    def step(si=None):
        cursors.zero_()
        for k, bd in (("MU", bmu), ("MS", bms), ("MC", bmc)):
            if si is not None:
                ev[si][k][0].record(stream)
            if k == "MC":
                eng.launch_mc(bd, outs[k])
            else:
                eng.launch_pulses(runtime.KIND_MU if k == "MU" else runtime.KIND_MS, bd, outs[k])
            if si is not None:
                ev[si][k][1].record(stream)
        if world > 1:  # RCCL all-gather of the decoded dmsg buffers (config 5), pysignalduino_amd/dist.py:
            # one exchange of the counts, one all-gather of the packed MU/MS/MC buffers
            sdist.allgather_streams([(outs[k]["desc"], outs[k]["rec"], outs[k]["heap"], bd["n"], outs[k]["cursor"])
                                     for k, bd in (("MU", bmu), ("MS", bms), ("MC", bmc))])

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    # overflow check (capacities sized so that the timed steps never re-run)
    for k, o in outs.items():
        cur = o["cursor"].cpu().numpy()
        if cur[2] != 0:
            raise SystemExit(f"{k}: result capacity overflow in bench configuration ({cur})")
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for si in range(args.steps):
        step(si)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    for si in range(args.steps):
        for k in outs:
            ktimes[k].append(ev[si][k][0].elapsed_time(ev[si][k][1]) * 1e-3)
    tt = torch.tensor([dt], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
    dt = float(tt.item())
    total_msgs = args.msgs * world * args.steps
    value = total_msgs / dt

    # roofline of the dominant kernel (MU): algorithmic bytes / measured kernel time
    kt = {k: float(np.mean(v)) for k, v in ktimes.items()}
    # HBM traffic of the same kernel/launch from the committed PMC passes (tools/pmc.sh ->
    # tools/pmc_traffic.py); null when absent or recorded for another launch size
    traffic = issue = None
    tpath = os.path.join(REPO, "profiles", "r01", "pmc_traffic.json")
    if os.path.exists(tpath):
        with open(tpath) as fh:
            tj = json.load(fh)
    dom = max(kt, key=kt.get)
    bd = {"MU": bmu, "MS": bms, "MC": bmc}[dom]
    o = outs[dom]
    cur = o["cursor"].cpu().numpy().astype(np.int64)
    n = bd["n"]
    if dom == "MC":
        in_bytes = int(bd["lengths"].sum()) + n * (8 + 4 + 4 + 1)
    else:
        in_bytes = int(bd["lengths"].sum()) + n * (8 + 1 + 10 + 80 + (2 if dom == "MS" else 0))
    out_bytes = n * runtime.DESC_DT.itemsize + int(cur[0]) * runtime.RES_DT.itemsize + int(cur[1])
    alg = in_bytes + out_bytes + len(bk.blob)
    achieved = alg / kt[dom]
    if os.path.exists(tpath):
        tag = f"k_pulses<{dom}>" if dom != "MC" else "k_mc"
        if tj.get("_config", {}).get("msgs_per_gpu") == args.msgs and tj.get(tag, {}).get("traffic_bytes"):
            traffic = float(tj[tag]["traffic_bytes"])
            issue = issue_view(tj[tag], kt[dom])
    res = {
        "metric": "RF messages/sec demodulated (MU+MS+MC, full protocol bank)",
        "value": value, "unit": "msgs/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": 1e3 * dt / args.steps, "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": "u8+f64", "data": "synthetic (seeded generators, pysignalduino_amd/synth.py)",
        "config": {"workload": "mixed MU/MS/MC stream, 1/3 each per rank: MU 256-pulse messages x 129-id MU bank, "
                               "MS sync+bits x 66-id MS bank (clock x U(0.6,1.4)), MC frames x 12 clockrange ids "
                               "('fixed' chain); N>1 adds the RCCL all-gather of dmsg buffers (config 5)",
                   "msgs_per_gpu": args.msgs, "parallelism": f"dp{world}"},
        "per_kernel_ms": {k: 1e3 * v for k, v in kt.items()},
        "per_type_msgs_per_s": {"MU": mu.n / kt["MU"], "MS": ms.n / kt["MS"], "MC": mc.n / kt["MC"]},
        "roofline": {"bound": "hbm", "achieved": achieved / 1e9, "peak": HBM_PEAK / 1e9, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK, "traffic": traffic, "kernel": f"k_pulses<{dom}>" if dom != "MC" else "k_mc",
                     "alg_bytes_per_launch": alg, "issue": issue},
    }
    if rank == 0 and not args.no_cpu:
        res["cpu_baseline"] = cpu_baseline(mu, ms, mc, args.cpu_seconds)
    if rank == 0:
        print(json.dumps(res), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
