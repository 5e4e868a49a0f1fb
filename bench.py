#!/usr/bin/env python3
"""Benchmark: RF messages/s demodulated (MU+MS+MC, full protocol bank) on 1..8 MI355X.

One "step" = one pass of the hot path over one batch resident in HBM: every MU message
(256 pulses) x the full MU bank, every MS message x the MS bank, every MC frame x the 12
clockrange protocols, results written in reference order -- and, for N > 1, the RCCL
all-gather of the decoded dmsg buffers (BASELINE config 5).  Weak scaling: each rank owns
``--msgs`` messages (1/3 of each type).

Prints ONE JSON line on rank 0 (contract in the task statement); see DESIGN.md §Measurement.
The mixed step runs as ONE kernel (k_step, sdx_demod_step: MU, then MS, then MC tiles) beside the
next step's grouping on a low-priority side stream (sdx_group_step).
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
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--msgs", type=int, default=1_000_000, help="messages per rank (1/3 MU, 1/3 MS, 1/3 MC)")
    ap.add_argument("--cpu-seconds", type=float, default=20.0, help="budget of the CPU-baseline leg")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--exchange", action="store_true",
                    help="run the N > 1 exchange (RCCL process group, overlapped all-gather) even at world size 1")
    ap.add_argument("--kind", default="mixed", choices=("mixed", "MU", "MS", "MC"),
                    help="mixed = config 5's per-GPU shard (1/3 each); MU/MS/MC = configs 2/3/4 (--msgs of one type)")
    ap.add_argument("--no-group", action="store_true",
                    help="run MU/MS in batch order (no sdx_group_pulses)")
    ap.add_argument("--concurrent", action="store_true",
                    help="one stream per kind: MU, MS and MC of a step run concurrently, one kernel's tail "
                         "overlapping the others' tiles (+3.5 %% msgs/s measured; per-kernel times then include "
                         "the sharing, so the roofline line is quoted on the default serial launches)")
    ap.add_argument("--group-at", default="mu", choices=("mu", "ms"),
                    help="where the next step's grouping runs: beside this step's MU (default) or after it, "
                         "beside MS / MC (A/B)")
    ap.add_argument("--kev-every", type=int, default=1,
                    help="per-kernel HIP events on every k-th timed step only (A/B of the events' own cost)")
    ap.add_argument("--serial", action="store_true",
                    help="MU, MS and MC one after another on one stream (default: MC on a second stream, "
                         "started when MU ends, so MC runs beside MS while MU runs alone)")
    ap.add_argument("--mrec", nargs="?", const="MU,MS", default="",
                    help="kinds (default both) whose grouping writes message records (sdx_msg_rec) and whose "
                         "k_pulses reads its header fields from them instead of the scattered SoA fields: less "
                         "HBM traffic, measured slower (A/B)")
    ap.add_argument("--mc-tail", action="store_true",
                    help="MC on a low-priority stream started with MU (the dispatcher gives its workgroups "
                         "the CUs MU's tail leaves idle) instead of beside MS")
    ap.add_argument("--ms-with-mu", default="", choices=("", "normal", "low"),
                    help="MS on its own stream started with MU at that priority (its tiles share the CUs with "
                         "MU's from the start and fill MU's tail), MC beside MS after MU (A/B)")
    ap.add_argument("--xchg", default="defer", choices=("eager", "pack-after-mu", "defer"),
                    help="exchange scheduling (N > 1 / --exchange): eager = count and pack as soon as possible "
                         "(beside the next step's MU); pack-after-mu = the pack waits for the next step's MU; "
                         "defer = count and pack both after the next step's MU (beside MS/MC; the default "
                         "since the kernels write the counts: 523.7-524.5M vs 507.2-510.8M msgs/s, "
                         "profiles/r04/s3/xchg_sched_ab.log)")
    ap.add_argument("--raw-wire", action="store_true",
                    help="exchange payloads raw (no nibble form: A/B of the wire size)")
    ap.add_argument("--scan-wire", action="store_true",
                    help="the exchange classifies every payload itself (no kernel-written counts, ABI 12: A/B)")
    ap.add_argument("--group-separate", action="store_true",
                    help="the MU and MS groupings as two sdx_group_pulses calls (26 launches) instead of one "
                         "sdx_group_step (13 launches; A/B)")
    ap.add_argument("--mc-apart", action="store_true",
                    help="A/B: MC's frames in their own launch after k_step (MU + MS) instead of k_step's last range")
    ap.add_argument("--ms-ungrouped", action="store_true",
                    help="A/B: group only the MU batch; MS tiles in arrival order")
    ap.add_argument("--group-reuse", action="store_true",
                    help="DIAGNOSTIC, not a valid line: group the batch in the first two steps only and reuse "
                         "the orders (what the per-step grouping costs the step)")
    ap.add_argument("--settle-steps", type=int, default=100,
                    help="untimed steps before the --warmup steps (~0.2 s: GPU clocks out of idle)")
    ap.add_argument("--no-fuse", dest="fuse", action="store_false",
                    help="one launch per kind (MU, then MS beside MC) instead of the default ONE kernel for the "
                         "step's MU, MS and MC tiles (sdx_demod_step, ABI 14, where each kind's tiles take the CU "
                         "slots the previous kind's last tiles free: 603.0-603.7M vs 579.5-580.9M msgs/s, "
                         "profiles/r05/fused/)")
    ap.add_argument("--batches", type=int, default=3,
                    help="K distinct seeded corpora, all resident in HBM, cycled step by step (step j runs batch "
                         "j mod K): with K x ~200 MB of inputs above the 256 MiB Infinity Cache no step re-reads a "
                         "batch the previous step left in the cache (VERDICT r05 #6; default 3: 608.8M vs 611.1-615.7M "
                         "msgs/s at K = 1, profiles/r06/batches_ab/)")
    ap.add_argument("--corpus", default="bench", choices=("bench", "dense"),
                    help="dense: no noise messages (every message carries a protocol's frames)")
    return ap.parse_args()


def cpu_model() -> str:
    """The host CPU's model name (/proc/cpuinfo), for the cpu_baseline line."""
    try:
        with open("/proc/cpuinfo") as fh:
            for ln in fh:
                if ln.startswith("model name"):
                    return ln.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor() or platform.machine()


def launch_ranks(args) -> int:
    """``--gpus N`` without a launcher: start N rank processes of this script (one GPU each,
    LOCAL_RANK = rank) and wait for them.  Runs before anything touches the GPU (this process never
    initialises HIP: the ranks are children, not exec'd replacements).  If one rank fails the others
    are stopped (they would wait in a collective) and its exit status is returned."""
    import socket
    import subprocess
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    procs = []
    for r in range(args.gpus):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(args.gpus), LOCAL_WORLD_SIZE=str(args.gpus),
                   MASTER_ADDR=os.environ.get("MASTER_ADDR", "127.0.0.1"), MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env))
    rc = 0
    live = list(procs)
    while live:
        for p in list(live):
            code = p.poll()
            if code is None:
                continue
            live.remove(p)
            if code != 0 and rc == 0:
                rc = code
                for q in live:          # the exact PIDs this function started
                    q.terminate()
        time.sleep(0.05)
    return rc


def cpu_baseline(mu, ms, mc, budget_s: float, kinds=("MU", "MS", "MC")):
    """The plain-C oracle (oracle/sd_oracle_c.c, a restatement of the reference path: kind 'port')
    timed on this host over a bounded sample of the SAME corpora the GPU demodulates (1:1:1
    MU/MS/MC for the mixed workload): once on one core, once on all cores this process may use.
    Each message is fully demodulated against the whole bank, with results written, as on the GPU."""
    from oracle import c_oracle as CO
    CO.build()
    bank = CO.CBank()
    cores = len(os.sched_getaffinity(0))
    if os.environ.get("OMP_NUM_THREADS", "").isdigit():  # the box's CPU share (16 per GPU)
        cores = min(cores, int(os.environ["OMP_NUM_THREADS"]))
    cores = max(1, min(cores, 64))
    src = {"MU": mu, "MS": ms, "MC": mc}
    nmax = min(src[k].n for k in kinds)

    def timed(k, threads):
        idx = np.arange(k)
        packs = [(t, CO.mc_batch(src[t].subset(idx)) if t == "MC" else CO.pack_batch(src[t].subset(idx)))
                 for t in kinds]
        t0 = time.perf_counter()
        for kind, pk in packs:
            CO.run(kind, pk, threads)
        return len(kinds) * k / (time.perf_counter() - t0)

    # size the samples from a short probe so the whole leg stays within ~budget_s seconds
    probe = timed(min(300, nmax), 1)
    k1 = int(max(300, min(nmax, probe * budget_s * 0.35 / len(kinds))))
    v1 = timed(k1, 1)
    kn = int(max(300, min(nmax, v1 * cores * budget_s * 0.5 / len(kinds))))
    vn = timed(kn, cores)
    mix = "/".join(kinds)
    return {"value": vn, "unit": "msgs/s", "cores": cores, "kind": "port", "value_1core": v1,
            "sample": f"oracle/sd_oracle_c.c (plain C, gcc -O2): {len(kinds) * kn} messages ({mix}, the "
                      f"first {kn} of each bench corpus) on {cores} threads; 1-core rate on {len(kinds) * k1} "
                      f"messages; host CPU: {cpu_model()}"}


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


def alg_bytes(kind, bd, rec_np):
    """SURVEY §8(d) algorithmic bytes of one launch: per MU/MS message n_pulses + 8*4 B pattern
    values + 8 B ids/order + 8 B header (304 B at 256 pulses); per MC frame ceil(L/4) hex + 8 B
    header; outputs sum(16 B record + payload); the bank once per GPU (<= 16 KB)."""
    n = bd["n"]
    if kind == "MC":
        inp = int(bd["lengths"].sum()) + 8 * n
    else:
        inp = int(bd["lengths"].sum()) + 48 * n
    out = 16 * len(rec_np) + int(rec_np["payload_len"].astype(np.int64).sum())
    return inp + out + 16384


def attribute_alone(torch, eng, stream, kinds, bds, outs, gbufs, corp, mrec_kinds, par, reps=5):
    """--fuse: each kind's own kernel alone on the launch stream (after the timed loop, untimed), so
    the line still carries MU's, MS's and MC's separate rooflines; returns {kind: seconds}."""
    from pysignalduino_amd import runtime
    res = {}
    with torch.cuda.stream(stream):
        for k in kinds:
            ts = []
            for _ in range(reps):
                outs[k]["cursor"].zero_()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(stream)
                if k == "MC":
                    eng.launch_mc(bds[k], outs[k])
                else:
                    eng.launch_pulses(runtime.KIND_MU if k == "MU" else runtime.KIND_MS, bds[k], outs[k],
                                      sel=gbufs[k][par][0][:corp[k].n], group=False,
                                      mrec=gbufs[k][par][2] if k in mrec_kinds else None)
                e1.record(stream)
                stream.synchronize()
                ts.append(e0.elapsed_time(e1) * 1e-3)
            res[k] = float(np.median(ts))
    return res


# the committed per-kernel PMC summary the line's roofline.traffic / issue come from: a tracked file that
# ships to the GPU box (profiles/ does not: VERDICT r05 #2), made by tools/pmc_commit.py from a
# tools/pmc.sh run, with the commit and the libsdx source hash the counters were taken on
PMC_FILE = os.path.join(REPO, "PMC_TRAFFIC.json")


def latest_pmc():
    return PMC_FILE if os.path.exists(PMC_FILE) else None


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(args))
    import torch
    import torch.distributed as dist
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world} (one rank per GPU)")
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # SDX_DIST_BACKEND=gloo rehearses the N > 1 code path on fewer GPUs than ranks (ranks share
    # devices round-robin); the driver's runs use RCCL ("nccl") with one GPU per rank
    backend = os.environ.get("SDX_DIST_BACKEND", "nccl")
    if backend != "nccl":
        local = local % max(1, torch.cuda.device_count())
    dist_on = world > 1 or args.exchange   # --exchange: the N > 1 path on a world-1 RCCL group
    if dist_on:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29541")
        os.environ.setdefault("RANK", str(rank))
        os.environ.setdefault("WORLD_SIZE", str(world))
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    if dist_on and dist.get_world_size() != args.gpus:
        raise SystemExit(f"bench.py: the process group has {dist.get_world_size()} ranks, --gpus {args.gpus}")
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)

    from pysignalduino_amd import bank as bankmod, runtime, synth
    from pysignalduino_amd import dist as sdist
    from pysignalduino_amd.runtime import RES_DT
    bk = bankmod.Bank()
    P = bk.protocols
    eng = runtime.Engine(bk, local)
    mrec_kinds = {k for k in args.mrec.split(",") if k}
    # the grouping writes message records only when the launches read them
    eng.use_mrec = {runtime.KIND_MU if k == "MU" else runtime.KIND_MS for k in mrec_kinds}
    kinds = ("MU", "MS", "MC") if args.kind == "mixed" else (args.kind,)
    per = {k: (args.msgs // 3 if k != "MC" else args.msgs - 2 * (args.msgs // 3)) if args.kind == "mixed" else args.msgs
           for k in kinds}
    seeds = {"MU": 42, "MS": 43, "MC": 44}
    # --group-reuse keeps step 0's order for every step: meaningful only on one batch
    nb = 1 if args.group_reuse else max(1, args.batches)
    corps, bdl = [], []
    for b in range(nb):   # batch b: seeds + 100 b (batch 0 is the corpus of every earlier round's line)
        corp, bds = {}, {}
        for k in kinds:
            sd = seeds[k] + 1000 * rank + 100 * b
            if k == "MU":
                corp[k] = synth.mu_corpus(P, per[k], seed=sd, noise_frac=0.0 if args.corpus == "dense" else 0.15)
            elif k == "MS":
                corp[k] = synth.ms_corpus(P, per[k], seed=sd, noise_frac=0.0 if args.corpus == "dense" else 0.1)
            else:
                corp[k] = synth.mc_corpus(P, per[k], seed=sd)
            bds[k] = eng.to_device_mc(corp[k]) if k == "MC" else eng.to_device_pulses(corp[k])
        corps.append(corp)
        bdl.append(bds)
    corp = corps[0]
    input_bytes = sum(v.numel() * v.element_size() for bds_ in bdl for bd in bds_.values() for v in bd.values()
                      if hasattr(v, "numel"))
    caps = {"MU": (12, 320), "MS": (4, 64), "MC": (4, 96)}
    nslot = 2 if dist_on else 1   # double-buffered outputs: step k+1 computes while step k is exchanged
    outs = []
    cursors = torch.zeros((nslot, len(kinds), 4), dtype=torch.int32, device=dev)
    for s_ in range(nslot):
        o = {}
        for i, k in enumerate(kinds):
            n = corp[k].n
            o[k] = eng.alloc_out(n, caps[k][0] * n + 4096, caps[k][1] * n + 65536,
                                 eng.pulses_work_bytes(n) if k != "MC" else 0, wire=dist_on and not args.scan_wire)
            o[k]["cursor"] = cursors[s_, i]   # one fill per step and stream resets a slot's cursors
        outs.append(o)
    # the launch stream at high priority, the grouping's side stream at low priority: the hardware
    # scheduler dispatches the demodulation tiles first and the grouping's small kernels fill the
    # gaps (measured: 2.153 vs 2.177 ms per step, tools/exp_group_cost.py)
    lo_prio, hi_prio = torch.cuda.Stream.priority_range()
    stream = torch.cuda.Stream(dev, priority=hi_prio)
    torch.cuda.set_stream(stream)
    # MU/MS message grouping (sdx_group_pulses) on a side stream, one step ahead: the grouping of
    # step j+1 (latency-bound small kernels) runs while step j demodulates; order buffers are
    # double-buffered by step parity.  Every step still groups once.
    gkinds = [k for k in kinds if k != "MC"] if not args.no_group else []
    # (SDX_GROUP_PRIO=high / equal: A/B of the side stream's priority)
    gp = os.environ.get("SDX_GROUP_PRIO", "low")
    side = torch.cuda.Stream(dev, priority={"low": lo_prio, "high": hi_prio}.get(gp, 0))
    if gp == "high":   # the launch stream below the grouping's
        stream = torch.cuda.Stream(dev, priority=lo_prio)
        torch.cuda.set_stream(stream)
    gbufs = {k: [eng.group_buffers(corp[k].n) for _ in range(2)] for k in gkinds}
    gdone, used = {}, [None, None]
    gev = [[torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)] for _ in range(args.steps + 1)]

    def launch_group(j, si=None, after=None):
        par = j % 2
        bds = bdl[j % nb]
        if used[par] is not None:           # step j-2's launches have read this parity's order
            side.wait_event(used[par])
        if after is not None:
            side.wait_event(after)
        with torch.cuda.stream(side):
            if si is not None and si % args.kev_every == 0:
                gev[si][0].record(side)
            if args.ms_ungrouped:
                eng.group(runtime.KIND_MU, bds["MU"], bufs=gbufs["MU"][par])
            elif gkinds == ["MU", "MS"] and not args.group_separate:   # both sorts' passes in the same launches
                eng.group_step(bds["MU"], bds["MS"], gbufs["MU"][par], gbufs["MS"][par])
            else:
                for k in gkinds:
                    eng.group(runtime.KIND_MU if k == "MU" else runtime.KIND_MS, bds[k], bufs=gbufs[k][par])
            # one event for all kinds: the grouping of step j ends during step j - 1, long before
            # step j's launches wait for it
            e = gev[si][1] if si is not None and si % args.kev_every == 0 else torch.cuda.Event()
            e.record(side)
            gdone[par] = e
    # config 5's product entry: this rank's shard launches + the pipelined exchange with overflow re-runs
    shd = (sdist.ShardedDemodulator(engine=eng, defer=args.xchg == "defer", nibble=not args.raw_wire)
           if dist_on else None)
    exch = shd.exchange if shd is not None else None
    KIND = {"MU": runtime.KIND_MU, "MS": runtime.KIND_MS, "MC": runtime.KIND_MC}
    done = [None] * nslot
    # per timed step and kernel an (start, end) pair of timing events, read after the closing
    # synchronize.  A kernel's start event is the end event its stream last recorded or waited on
    # when there is one (MS after MU on the launch stream, MC waiting for MU's end), so a step records
    # few events: every event record and cross-stream wait is a packet the command processor handles
    # between two kernels.  Round 4: ten events and waits per step cost 1.80-1.81 vs 1.77-1.78 ms per
    # step with events on one step in 100 (profiles/r04/s2/events_ab.log); with these four, 1.778 ms
    # on every step (profiles/r04/s3/bench_events_modes.log).  MS's and MC's times include their
    # launch gap.
    kev = [dict() for _ in range(args.steps)]

    # --concurrent: one stream per kind, the three launches of a step run concurrently (the tail of
    # one kernel overlaps the others' tiles); default: one after another on the launch stream
    kstream = {k: (torch.cuda.Stream(dev) if args.concurrent else stream) for k in kinds}
    # the mixed step's default is one k_step launch (below); --no-fuse: MU alone, then MS and MC side by
    # side -- MC fills the CUs MS's tail leaves idle (482 vs 471M msgs/s serial, 20 steps)
    mc_beside_ms = (not args.serial and not args.concurrent and not args.mc_tail and "MC" in kinds and "MU" in kinds
                    and not (args.fuse and args.kind == "mixed" and not args.no_group and args.group_at == "mu"
                             and not args.ms_with_mu))
    if mc_beside_ms:
        kstream["MC"] = torch.cuda.Stream(dev)   # (at the lowest priority: equal, profiles/r04/s3/dropped/mc_low_ab.log)
    if args.mc_tail and "MC" in kinds:
        kstream["MC"] = torch.cuda.Stream(dev, priority=lo_prio)
    if args.ms_with_mu and "MS" in kinds:
        kstream["MS"] = torch.cuda.Stream(dev, priority=lo_prio if args.ms_with_mu == "low" else 0)
    # launches on other streams than the launch stream join it at the end of their step only when
    # the exchange reads the step's outputs; otherwise each stream resets its own kinds' cursors
    # before its launch (its previous launch on the same slot is earlier on that stream)
    join_now = exch is not None or any(kstream[k] is not stream for k in gkinds)
    need_start = any(kstream[k] is not stream and not (mc_beside_ms and k == "MC") for k in kinds)
    kidx = {k: i for i, k in enumerate(kinds)}
    own = {}                                # stream -> the kinds whose cursors it resets
    for k in kinds:
        own.setdefault(kstream[k], []).append(kidx[k])
    own = {st_: slice(ix[0], ix[-1] + 1) for st_, ix in own.items()}
    assert sum(x.stop - x.start for x in own.values()) == len(kinds), "a stream's kinds are contiguous"

    mu_done = [None]
    # the default mixed step runs as one k_step launch; the A/B modes (--serial, --concurrent, --mc-tail,
    # --ms-with-mu, --group-at ms, --no-group) and the single-kind configs keep one launch per kind
    fused = (args.fuse and kinds == ("MU", "MS", "MC") and bool(gkinds) and args.group_at == "mu" and not
             (args.serial or args.concurrent or args.mc_tail or args.ms_with_mu))

    def step(j, si=None):
        s_ = j % nslot
        bds = bdl[j % nb]
        if done[s_] is not None:            # the exchange that read this slot has finished
            stream.wait_event(done[s_])
            done[s_] = None
        if join_now or len(own) == 1:
            cursors[s_].zero_()
        else:
            for st_, ix in own.items():
                if st_ is not stream:       # after that stream's launches of nslot steps ago
                    with torch.cuda.stream(st_):
                        cursors[s_, ix].zero_()
            cursors[s_, own[stream]].zero_()
        if gkinds:
            if j == 0:
                launch_group(0)
            if args.group_at == "mu" and not (args.group_reuse and j >= 1):
                launch_group(j + 1, si)     # the next step's grouping, concurrent with this step
        par = j % 2
        tm = si is not None and si % args.kev_every == 0
        last = None                         # the latest event recorded on the launch stream
        start = None
        if need_start:
            start = torch.cuda.Event(enable_timing=tm)
            start.record(stream)            # cursors reset, previous exchange done
        if fused:   # one k_step launch for the whole step (sdx_demod_step)
            stream.wait_event(gdone[par])
            e0 = None
            if tm:
                e0 = torch.cuda.Event(enable_timing=True)
                e0.record(stream)
            parts = {}
            for k in ("MU", "MS"):
                ung = args.ms_ungrouped and k == "MS"
                parts[k.lower()] = (bds[k], outs[s_][k], None if ung else gbufs[k][par][0][:corp[k].n],
                                    gbufs[k][par][2] if k in mrec_kinds and not ung else None)
            eng.launch_step(mu=parts["mu"], ms=parts["ms"],
                            mc=(dict(bds["MC"], max_hex=0) if args.mc_apart else bds["MC"], outs[s_]["MC"], None))
            e1 = torch.cuda.Event(enable_timing=tm)
            e1.record(stream)
            if tm:
                kev[si]["step"] = (e0, e1)
            mu_done[0] = last = e1
        for k in (() if fused else kinds):
            ks = kstream[k]
            e0 = None
            if ks is not stream:
                if mc_beside_ms and k == "MC":
                    e0 = mu_done[0]
                else:
                    e0 = start
                ks.wait_event(e0)
            else:
                e0 = last
            if k in gkinds and (k == gkinds[0] or ks is not kstream[gkinds[0]]):
                ks.wait_event(gdone[par])
            with torch.cuda.stream(ks):
                if tm and e0 is None:
                    e0 = torch.cuda.Event(enable_timing=True)
                    e0.record(ks)
                if k == "MC":
                    eng.launch_mc(bds[k], outs[s_][k])
                else:
                    eng.launch_pulses(runtime.KIND_MU if k == "MU" else runtime.KIND_MS, bds[k], outs[s_][k],
                                      sel=gbufs[k][par][0][:corp[k].n] if k in gkinds else None, group=False,
                                      mrec=gbufs[k][par][2] if k in gkinds and k in mrec_kinds else None)
                e1 = torch.cuda.Event(enable_timing=tm)
                e1.record(ks)
            if tm:
                kev[si][k] = (e0, e1)
            if k == "MU":
                mu_done[0] = e1
                if gkinds and args.group_at == "ms":
                    launch_group(j + 1, si, after=e1)   # beside this step's MS / MC
            if ks is stream:
                last = e1
            elif join_now:
                stream.wait_event(e1)       # the step ends when all three launches have
                last = None
        if gkinds:
            if last is None:
                last = torch.cuda.Event()
                last.record(stream)
            used[par] = last                # the step's grouped launches have read this parity's order
        if exch is not None:  # RCCL all-gather of the decoded dmsg buffers (config 5), overlapped
            parts = [sdist.Part.from_out(outs[s_][k], KIND[k], src=(KIND[k], bds[k], 0, -1)) for k in kinds]
            # (fused: no "after MU" point inside the step; the previous step's count and pack run behind
            # its own end, beside this step's k_step -- waiting for this step's end would hold the host
            # until the GPU had drained)
            rel = shd.submit(parts, stream, after=mu_done[0] if args.xchg != "eager" and "MU" in kinds and not fused
                             else None)
            if rel is not None:             # the previous step's pack has read its slot
                done[(j - 1) % nslot] = rel

    def drain():
        stream.wait_stream(side)
        if exch is not None:
            exch.flush()
            if exch.stream is not None:     # the last step's pack and data all-gather
                stream.wait_stream(exch.stream)
        torch.cuda.synchronize()

    j = 0
    # settle (untimed, before the W warmup steps): ~0.2 s of steps, so that the timed steps do not
    # start on a GPU still ramping up from idle -- a fresh box's first bench once ran MS at twice its
    # time with 3 warmup steps (profiles/r05/dropped/radix_passes/bench_1.log, 417M vs 581M msgs/s)
    # (a fixed count, not a time: every rank must run the same steps -- each step holds collectives)
    settle = max(0, args.settle_steps)
    for _ in range(settle):
        step(j)
        j += 1
    for _ in range(args.warmup):
        step(j)
        j += 1
    drain()
    ovf = {}
    for k in kinds:   # capacities are sized so that the timed steps never re-run
        cur = outs[(j - 1) % nslot][k]["cursor"].cpu().numpy()
        if cur[2] != 0:
            ovf[k] = int(cur[2])
    if ovf and args.corpus != "dense":
        raise SystemExit(f"result capacity overflow in bench configuration ({ovf})")
    if dist_on:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for si in range(args.steps):
        step(j, si)
        j += 1
    drain()
    if dist_on:
        dist.barrier()
    dt = time.perf_counter() - t0
    ktimes = {k: [kev[si][k][0].elapsed_time(kev[si][k][1]) * 1e-3 for si in range(0, args.steps, args.kev_every)]
              for k in (("step",) if fused else kinds)}
    gtime = float(np.mean([gev[si][0].elapsed_time(gev[si][1]) * 1e-3 for si in range(0, args.steps, args.kev_every)])) \
        if gkinds and not args.group_reuse else 0.0
    tt = torch.tensor([dt], dtype=torch.float64, device=dev)
    if dist_on:
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
    dt = float(tt.item())
    total_msgs = sum(per.values()) * world * args.steps
    value = total_msgs / dt

    # roofline of the dominant kernel: SURVEY §8(d) algorithmic bytes / its HIP-event time
    kt = {k: float(np.mean(v)) for k, v in ktimes.items()}
    bds, corp = bdl[(j - 1) % nb], corps[(j - 1) % nb]   # the last timed step's batch (its order: parity j-1)
    if fused:   # each kind's kernel alone (untimed attribution pass): its own roofline entry
        kt_step = kt["step"]
        kt = attribute_alone(torch, eng, stream, kinds, bds, outs[(j - 1) % nslot], gbufs, corp, mrec_kinds,
                             (j - 1) % 2)
    # the grouping's own time (one step's groupings alone on the launch stream, untimed): group_ms is
    # the side stream's wall time beside the step's kernel, mostly waiting for CU slots
    g_alone = None
    if gkinds:
        gts = []
        with torch.cuda.stream(stream):
            for _ in range(5):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(stream)
                if gkinds == ["MU", "MS"] and not args.group_separate:
                    eng.group_step(bds["MU"], bds["MS"], gbufs["MU"][0], gbufs["MS"][0])
                else:
                    for k in gkinds:
                        eng.group(runtime.KIND_MU if k == "MU" else runtime.KIND_MS, bds[k], bufs=gbufs[k][0])
                e1.record(stream)
                stream.synchronize()
                gts.append(e0.elapsed_time(e1) * 1e-3)
        g_alone = float(np.median(gts))
    dom = max(kt, key=kt.get)
    # every kind's launch against the same HBM roofline: its algorithmic bytes (the
    # outputs of the last step) / its HIP-event time -- with the fused step each kernel timed alone in
    # the attribution pass; with --no-fuse MS and MC run side by side after MU (MC on its own stream,
    # started at MU's end), so their times include that sharing; --kind MU|MS|MC times each kernel alone
    kern_tag = {"MU": "k_pulses<MU>", "MS": "k_pulses<MS>", "MC": "k_mc"}
    kernels = {}
    for k in kinds:
        ok_ = outs[(j - 1) % nslot][k]
        ck = ok_["cursor"].cpu().numpy().astype(np.int64)
        rk = ok_["rec"][: int(ck[0]) * RES_DT.itemsize].cpu().numpy().view(RES_DT)
        ak = alg_bytes(k, bds[k], rk)
        kernels[k] = {"kernel": kern_tag[k], "alg_bytes_per_launch": ak, "results_per_launch": int(ck[0]),
                      "ms": 1e3 * kt[k], "achieved_GBps": ak / kt[k] / 1e9, "frac": ak / kt[k] / HBM_PEAK,
                      "shares_gpu_with": ("MC" if k == "MS" else "MS") if mc_beside_ms and k in ("MS", "MC") and not fused
                      else None}
        if fused:
            kernels[k]["timed"] = "alone, untimed attribution pass after the timed loop (the timed step runs k_step)"
    step_roof = None
    if fused:
        salg = sum(kernels[k]["alg_bytes_per_launch"] for k in kinds)
        step_roof = {"kernel": "k_step (MU + MS + MC tiles, one launch)", "alg_bytes_per_launch": salg,
                     "ms": 1e3 * kt_step, "achieved_GBps": salg / kt_step / 1e9, "frac": salg / kt_step / HBM_PEAK}
    o = outs[(j - 1) % nslot][dom]
    cur = o["cursor"].cpu().numpy().astype(np.int64)
    alg = kernels[dom]["alg_bytes_per_launch"]
    n = bds[dom]["n"]
    layout = (int(bds[dom]["lengths"].sum()) + n * ((8 + 4 + 4 + 1) if dom == "MC" else
                                                    (8 + 1 + 10 + 80 + (2 if dom == "MS" else 0)))
              + n * runtime.DESC_DT.itemsize + int(cur[0]) * RES_DT.itemsize + int(cur[1]) + len(bk.blob))
    achieved = alg / kt[dom]
    traffic = issue = traffic_src = None
    tag = f"k_pulses<{dom}>" if dom != "MC" else "k_mc"
    t_dom = kt[dom]
    if fused:   # the timed region's one kernel: k_step over the whole step's algorithmic bytes
        tag, alg, t_dom = "k_step", step_roof["alg_bytes_per_launch"], kt_step
        achieved = alg / kt_step
        layout = None
    tpath = latest_pmc()
    if tpath and args.corpus == "bench":
        with open(tpath) as fh:
            tj = json.load(fh)
        cfg = tj.get("_config", {})
        if cfg.get("msgs_per_gpu") == args.msgs and cfg.get("kind", "mixed") == args.kind and \
                tj.get(tag, {}).get("traffic_bytes"):
            traffic = float(tj[tag]["traffic_bytes"])
            src = tj.get("_source", {})
            loaded = runtime.load_library().sdx_source_hash().decode()
            traffic_src = {"pmc": os.path.relpath(tpath, REPO), "commit": src.get("commit"),
                           "sdx_source_hash": src.get("sdx_source_hash"),
                           "same_kernels_as_this_run": src.get("sdx_source_hash") == loaded,
                           "profiles": src.get("profiles"),
                           "fetch_bytes": 2 * 1024 * float(tj[tag]["fetch_size_kib"]),
                           "write_bytes": 1024 * float(tj[tag]["write_size_kib"]),
                           "calibration": "profiles/r05/calib/calib_traffic.json (FETCH_SIZE x 2 holds for every "
                                          "vector load width this kernel uses; scalar loads count exactly)"}
            issue = issue_view(tj[tag], t_dom)
    wl = {"mixed": "mixed MU/MS/MC stream, 1/3 each per rank: MU 256-pulse messages x 129-id MU bank, MS sync+bits x "
                   "66-id MS bank (clock x U(0.6,1.4)), MC frames x 12 clockrange ids ('fixed' chain)",
          "MU": "config 2: 256-pulse MU messages x 129-id MU bank",
          "MS": "config 3: MS sync+bits messages x 66-id MS bank, clock x U(0.6,1.4) sweep of the +-30 % gate",
          "MC": "config 4: MC frames x 12 clockrange ids ('fixed' chain, mc2dmc + postdemodulation methods)"}[args.kind]
    if dist_on:
        wl += "; N>1 adds the RCCL all-gather of dmsg buffers (config 5), overlapped with the next step"
    res = {
        "metric": "RF messages/sec demodulated (MU+MS+MC, full protocol bank)",
        "value": value, "unit": "msgs/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
        "settle_steps": settle,
        "ms_per_step": 1e3 * dt / args.steps, "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": "u8+f64",
        **({"diagnostic": "--group-reuse: the batch was grouped once, not per step -- NOT a valid line"}
           if args.group_reuse else {}),
        "data": "synthetic (seeded generators, pysignalduino_amd/synth.py" +
                (", noise-free dense corpus)" if args.corpus == "dense" else ")"),
        "config": {"workload": wl, "kind": args.kind, "corpus": args.corpus, "msgs_per_gpu": sum(per.values()),
                   "batches": nb, "input_bytes_resident": input_bytes,
                   "parallelism": f"dp{world}", "grouped": ("MU only" if args.ms_ungrouped else bool(gkinds)),
                   "streams": ("one kernel (k_step: MU, then MS, then MC tiles)" if fused else
                               "one per kind" if args.concurrent and len(kinds) > 1 else
                               "MU, then MS beside MC" if mc_beside_ms else "serial")},
        "per_kernel_ms": {**({"step": 1e3 * kt_step} if fused else {}), **{k: 1e3 * v for k, v in kt.items()}},
        "group_ms": 1e3 * gtime,   # sdx_group_pulses of all kinds per step (side stream, one step ahead)
        "group_alone_ms": None if g_alone is None else 1e3 * g_alone,   # the same groupings alone, untimed
        "per_type_msgs_per_s": {k: per[k] / kt[k] for k in kinds},
        "roofline": {"bound": "hbm", "achieved": achieved / 1e9, "peak": HBM_PEAK / 1e9, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK, "traffic": traffic, "kernel": tag,
                     "alg_bytes_per_launch": alg, "layout_bytes_per_launch": layout,
                     "results_per_launch": sum(k_["results_per_launch"] for k_ in kernels.values()) if fused else int(cur[0]),
                     "issue": issue, "traffic_source": traffic_src,
                     "per_kernel": kernels, **({"step": step_roof} if fused else {})},
    }
    if exch is not None and exch.bytes_sent:
        nb = exch.bytes_sent[-args.steps:]
        wb = exch.wire_bytes[-args.steps:]
        res["exchange"] = {"format": "wire v3 (include/sdx.h): 4 B/message + 8 B/record + payloads "
                                     + ("raw" if args.raw_wire else "(preamble + hex + postamble as packed digits)"),
                           "scheduling": args.xchg,
                           "branch": "pipelined" if exch.pipelined else "sync",
                           "send_bytes_per_rank_per_step": float(np.mean(nb)),
                           "wire_bytes_per_rank_per_step": float(np.mean(wb)),
                           "payload_bytes_per_rank_per_step": float(np.mean(exch.payload_bytes[-args.steps:])),
                           "payload_wire_bytes_per_rank_per_step": float(np.mean(exch.heap_wire_bytes[-args.steps:])),
                           "recv_bytes_per_rank_per_step": float(np.mean(nb)) * world,
                           "reruns": exch.reruns}
    if ovf:   # dense corpus: messages whose results did not fit the on-chip staging (the product re-runs them)
        res["overflow"] = {}
        for k in ovf:
            d = outs[(j - 1) % nslot][k]["desc"][: corp[k].n * runtime.DESC_DT.itemsize].cpu().numpy().view(runtime.DESC_DT)
            res["overflow"][k] = {"flags": ovf[k], "tile_msgs": int((d["status"] == runtime.ST_OVF_TILE).sum()),
                                  "out_msgs": int((d["status"] == runtime.ST_OVF_OUT).sum())}
    if rank == 0 and not args.no_cpu:
        res["cpu_baseline"] = cpu_baseline(corps[0].get("MU"), corps[0].get("MS"), corps[0].get("MC"), args.cpu_seconds,
                                           kinds)
    if rank == 0:
        print(json.dumps(res), flush=True)
    if dist_on:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
