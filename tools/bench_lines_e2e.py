#!/usr/bin/env python3
"""End-to-end front-end rate with the PCIe transfers (controller.py:245-264).

The drop-in use (SignalduinoController._parser_task -> SignalParser.parse_line) needs raw lines in
and decoded records out.  This tool streams framed firmware lines from pinned host memory through
the device and brings the decoded results back, double-buffered over three HIP streams:

  copy-in stream   chunk k's line bytes + offsets, pinned host -> HBM (H2D)
  parse stream     sdx_parse_lines + sdx_select_lines, the 32-byte class counts -> host
  demod stream     the MU/MS short/long and MC ('fixed') launches over the selection lists, then
                   the results serialised to the exchange's wire form (sdx_exchange_count/pack:
                   per line and kind a 4-byte word, 8 B per record, packed payloads)
  copy-out stream  chunk k-1's wire bytes + per-line kind/status, HBM -> pinned host (D2H), sized
                   by its device counts (read one chunk later, while the GPU runs chunk k)

so chunk k's H2D, chunk k's parse, chunk k-1's demodulation and chunk k-2's D2H overlap.  Prints ONE
JSON line: value = lines/s end to end (first H2D enqueued -> last D2H landed), beside the kernels'
own HBM-resident time per chunk and the PCIe bytes each way, naming the bound.  --check decodes
chunk 0's host-side results and compares them with SignalParser.parse_lines on the same lines.

usage: python tools/bench_lines_e2e.py [--lines 1000000 --chunk 250000 --passes 4 --check]
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lines", type=int, default=1_000_000, help="corpus lines (streamed --passes times)")
    ap.add_argument("--chunk", type=int, default=250_000)
    ap.add_argument("--passes", type=int, default=4)
    ap.add_argument("--check", action="store_true")
    args = ap.parse_args()
    import torch
    from pysignalduino_amd import bank as bankmod, dist as sdist, frontend, runtime, synth
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    bk = bankmod.Bank()
    eng = runtime.Engine(bk, 0)
    cache = os.path.join(os.environ.get("TMPDIR", "/tmp"), f"sdx_lines_{args.lines}_45_1-1-1_0.3.npz")
    if os.path.exists(cache):
        z = np.load(cache)
        data, offsets = z["data"], z["offsets"]
    else:
        lines, _ = synth.line_corpus(bk.protocols, args.lines, seed=45, mix=(1, 1, 1), compress_frac=0.3)
        data, offsets, bad = frontend.pack_lines(lines)
        assert not bad
        np.savez(cache, data=data, offsets=offsets)
    n_all = len(offsets) - 1
    C = args.chunk
    nck = n_all // C
    assert nck >= 2, "need at least two chunks"
    # pinned host chunks (the lines as they arrive from the transports), offsets rebased
    hb, ho = [], []
    for k in range(nck):
        o = offsets[k * C: (k + 1) * C + 1].astype(np.int64)
        b = data[o[0]: o[-1]]
        hb.append(torch.from_numpy(np.concatenate([b, np.zeros(16, np.uint8)])).pin_memory())
        ho.append(torch.from_numpy(o - o[0]).pin_memory())
    maxb = max(int(x.numel()) for x in hb)
    # two device slots: line buffers + parse outputs, demodulation outputs, wire send buffer
    fake = np.linspace(0, maxb - 16, C + 1).astype(np.int64)
    lbs = [frontend.LineBatch(eng, np.zeros(maxb - 16, np.uint8), fake) for _ in range(2)]
    caps = {"MU": (8, 160), "MS": (2, 48), "MC": (2, 48)}
    outs = [{k: eng.alloc_out(C, caps[k][0] * C + 4096, caps[k][1] * C + 65536,
                              eng.pulses_work_bytes(C) if k != "MC" else 0) for k in caps} for _ in range(2)]
    kinds = ("MU", "MS", "MC")
    sers = []
    for s in range(2):   # one serialiser (exchange sender kernels) per slot
        ex = sdist.Exchange.__new__(sdist.Exchange)
        ex._bufs, ex.engine = {}, eng     # the wire's nibble form with the engine's bank
        sers.append(ex)
    cin, sp, sd, cout = (torch.cuda.Stream(dev) for _ in range(4))
    host_counts = [torch.empty(8, dtype=torch.int32).pin_memory() for _ in range(2)]
    host_wc = [torch.empty(3 * runtime.XCHG_COUNTS, dtype=torch.int32).pin_memory() for _ in range(2)]
    host_out = [torch.empty(sum(caps[k][0] * C * 8 + caps[k][1] * C + 4 * C for k in caps) + 2 * C + 65536,
                            dtype=torch.uint8).pin_memory() for _ in range(2)]
    ev = lambda: torch.cuda.Event()  # noqa: E731
    parse_done, demod_done, d2h_done, counts_ev, wc_ev = [None] * 2, [None] * 2, [None] * 2, [None] * 2, [None] * 2
    kt = {"parse": [], "demod": []}
    tev = {}
    h2d_bytes = d2h_bytes = 0
    results = {}

    def enqueue_d2h(j):
        """chunk j's results to the host, sized by its device counts (on the host by now or soon)."""
        nonlocal d2h_bytes
        s = j % 2
        wc_ev[s].synchronize()
        S = host_wc[s].numpy().astype(np.int64).reshape(1, 3, runtime.XCHG_COUNTS)
        if S[..., 3].any():
            raise SystemExit(f"chunk {j}: overflowed messages {S[..., 3]}")
        offs, nb, T = sdist._layout(S)
        with torch.cuda.stream(cout):
            cout.wait_event(demod_done[s])
            send = sers[s]._bufs["send"]
            host_out[s][:T].copy_(send[:T], non_blocking=True)
            host_out[s][T: T + C].copy_(lbs[s].kind[:C], non_blocking=True)
            host_out[s][T + C: T + 2 * C].copy_(lbs[s].status[:C], non_blocking=True)
            e = ev()
            e.record(cout)
            d2h_done[s] = e
        d2h_bytes += T + 2 * C
        if args.check and j == 0:
            e.synchronize()
            results[0] = (host_out[s][: T + 2 * C].numpy().copy(), offs, nb, T)

    nsteps = nck * args.passes
    h2d_ev = [None] * 2

    def enqueue_h2d(k):
        """chunk k's lines to slot k % 2 (its line buffers are free once chunk k-2's parse read them)."""
        nonlocal h2d_bytes
        s, c = k % 2, k % nck
        with torch.cuda.stream(cin):
            if parse_done[s] is not None:
                cin.wait_event(parse_done[s])
            lbs[s].bytes[: hb[c].numel()].copy_(hb[c], non_blocking=True)
            lbs[s].offsets.copy_(ho[c], non_blocking=True)
            e = ev()
            e.record(cin)
            h2d_ev[s] = e
        h2d_bytes += int(hb[c].numel()) + 8 * (C + 1)

    torch.cuda.synchronize()
    t0 = time.perf_counter()
    enqueue_h2d(0)
    for k in range(nsteps):
        s, c = k % 2, k % nck
        lb = lbs[s]
        # 0. chunk k-2's D2H (its counts arrived while the GPU ran chunk k-1); it reads slot s's
        #    kind/status and wire buffer, which chunk k overwrites below
        if k >= 2:
            enqueue_d2h(k - 2)
        # 1. parse + select (slot s's parse outputs are free once chunk k-2's demodulation ran)
        with torch.cuda.stream(sp):
            sp.wait_event(h2d_ev[s])
            if demod_done[s] is not None:
                sp.wait_event(demod_done[s])
            if d2h_done[s] is not None:
                sp.wait_event(d2h_done[s])
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(sp)
            lb.launch()
            e1.record(sp)
            host_counts[s].copy_(lb.counts, non_blocking=True)
            ce = ev()
            ce.record(sp)
            counts_ev[s] = ce
            parse_done[s] = e1
            tev.setdefault("parse", []).append((e0, e1))
        # 2. chunk k+1's H2D, ahead of the wait below: it overlaps chunk k's parse and demodulation
        if k + 1 < nsteps:
            enqueue_h2d(k + 1)
        # 3. demodulate + serialise chunk k (the class counts size the launches)
        ce.synchronize()
        cnt = host_counts[s].numpy()[: runtime.SEL_NCLASS].copy()
        start = np.concatenate([[0], np.cumsum(cnt)])
        sels = [lb.sel[int(start[i]): int(start[i + 1])] for i in range(runtime.SEL_NCLASS)]
        with torch.cuda.stream(sd):
            sd.wait_event(parse_done[s])
            if d2h_done[s] is not None:
                sd.wait_event(d2h_done[s])
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(sd)
            o = outs[s]
            for kk in kinds:
                o[kk]["cursor"].zero_()
                o[kk]["desc"].zero_()   # lines of another class keep an empty descriptor
            pb, mb = lb.pulse_batch(), lb.mc_batch()
            for kk, short, long_ in (("MU", runtime.SEL_MU_SHORT, runtime.SEL_MU_LONG),
                                     ("MS", runtime.SEL_MS_SHORT, runtime.SEL_MS_LONG), ("MC", runtime.SEL_MC, None)):
                if kk == "MC":
                    if cnt[short]:
                        eng.launch_mc(mb, o[kk], sel=sels[short])
                else:
                    kind = runtime.KIND_MU if kk == "MU" else runtime.KIND_MS
                    if cnt[short]:
                        eng.launch_pulses(kind, pb, o[kk], sel=sels[short])
                    if cnt[long_]:
                        eng.launch_pulses(kind, pb, o[kk], sel=sels[long_], long_variant=True)
            KIND = {"MU": runtime.KIND_MU, "MS": runtime.KIND_MS, "MC": runtime.KIND_MC}
            wc = sers[s]._count_pack_device(sdist._flatten([sdist.Part(o[kk]["desc"], o[kk]["rec"], o[kk]["heap"], C,
                                                                       o[kk]["cursor"], KIND[kk]) for kk in kinds]), sd)
            e1.record(sd)
            host_wc[s].copy_(wc, non_blocking=True)
            we = ev()
            we.record(sd)
            wc_ev[s] = we
            demod_done[s] = e1
            tev.setdefault("demod", []).append((e0, e1))
    for j in range(max(0, nsteps - 2), nsteps):
        enqueue_d2h(j)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    total = nsteps * C
    for key in ("parse", "demod"):
        kt[key] = [a.elapsed_time(b) * 1e-3 for a, b in tev[key]]
    k_parse, k_demod = float(np.median(kt["parse"])), float(np.median(kt["demod"]))
    res = {
        "metric": "raw firmware lines/sec end to end: pinned host lines -> parse + demodulate -> decoded results in "
                  "pinned host memory (PCIe both ways, overlapped)",
        "value": total / dt, "unit": "lines/s", "n_gpus": 1, "lines": total, "chunk_lines": C,
        "ms_per_chunk": 1e3 * dt / nsteps,
        "kernels_ms_per_chunk": {"parse+select": 1e3 * k_parse, "demod+serialise": 1e3 * k_demod},
        "hbm_resident_lines_per_s": C / (k_parse + k_demod),
        "pcie": {"h2d_bytes_per_line": h2d_bytes / total, "d2h_bytes_per_line": d2h_bytes / total,
                 "h2d_GB_per_s": h2d_bytes / dt / 1e9, "d2h_GB_per_s": d2h_bytes / dt / 1e9},
        "data": "synthetic firmware lines (synth.line_corpus: MU/MS/MC 1/3 each, 30 % of MU/MS Mred=1 compressed)",
    }
    res["bound"] = ("kernels" if (k_parse + k_demod) * nsteps >= 0.8 * dt else "transfers / host enqueue")
    if args.check:
        buf, offs, nb, T = results[0]
        kinds_np = buf[T: T + C]
        status_np = buf[T + C: T + 2 * C]
        dec = {}
        for i, kk in enumerate(kinds):
            o = offs[0, i]
            m = buf[o[0]: o[0] + nb[0, i, 0]].view(np.uint32)
            w = buf[o[1]: o[1] + nb[0, i, 1]].view(runtime.WIRE_REC_DT)
            p = buf[o[2]: o[2] + nb[0, i, 2]]
            dec[kk] = sdist.wire_decode([(m, w, p)], bk.affixes(i))
        lines = [data[offsets[i]: offsets[i + 1]].tobytes() for i in range(C)]
        from pysignalduino_amd.sd_protocols import SDProtocols
        sp_ = frontend.SignalParser(SDProtocols(mc_mode="fixed"))
        exp = sp_.parse_lines(lines)
        lk = {runtime.LINE_MU: "MU", runtime.LINE_MS: "MS", runtime.LINE_MC: "MC"}
        pid = {"MU": bk.mu_pids, "MS": bk.ms_pids, "MC": bk.mc_pids}
        bad = 0
        for i in range(C):
            kk = lk.get(int(kinds_np[i]))
            got = []
            if kk and int(status_np[i]) == runtime.LS_OK:
                d, r, h = dec[kk]
                if d[i]["status"] == runtime.ST_OK:
                    for x in r[int(d[i]["rec_begin"]): int(d[i]["rec_begin"]) + int(d[i]["n_rec"])]:
                        got.append((str(pid[kk][int(x["proto"])]),
                                    h[int(x["payload_off"]): int(x["payload_off"]) + int(x["payload_len"])].tobytes()
                                    .decode("latin-1")))
            want = [] if isinstance(exp[i], BaseException) else [(m_.protocol_id, m_.payload) for m_ in exp[i]]
            bad += got != want
        res["check"] = {"lines": C, "mismatches": bad, "against": "SignalParser.parse_lines (mc_mode fixed)"}
        if bad:
            print(json.dumps(res), flush=True)
            raise SystemExit(f"{bad} lines differ from SignalParser.parse_lines")
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
