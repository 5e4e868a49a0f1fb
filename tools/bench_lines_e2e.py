#!/usr/bin/env python3
"""End-to-end front-end rate with the PCIe transfers (controller.py:245-264).

The drop-in use (SignalduinoController._parser_task -> SignalParser.parse_line) has raw lines in host
memory and wants decoded results back in host memory.  This tool streams framed firmware lines from
pinned host memory through the product streaming API (``SignalParser.stream``,
pysignalduino_amd/stream.py: H2D, parse + select, demodulation + serialisation, D2H of successive
chunks overlapping on four HIP streams, the host never waiting on a chunk it has just enqueued) and
prints ONE JSON line: value = lines/s end to end (first submit -> last chunk's results landed in
pinned host memory), beside the kernels' own time per chunk, the PCIe bytes each way and the bound
(the stage whose per-chunk time is the largest: H2D, kernels, D2H or the host).  ``--output json``
streams the MQTT texts (what BatchingParserTask publishes) instead of the wire form.  --check
compares chunk 0's results with SignalParser.parse_lines / parse_lines_json on the same lines.

usage: python tools/bench_lines_e2e.py [--lines 1000000 --chunk 250000 --passes 4 --output wire --check]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def copy_rates(torch, host_bytes):
    """Pinned H2D and D2H rates of this host link for a chunk-sized buffer (HIP events, 5 copies)."""
    h = torch.from_numpy(host_bytes)
    d = torch.empty(h.numel(), dtype=torch.uint8, device="cuda")
    rates = []
    for src, dst in ((h, d), (d, h)):
        dst.copy_(src, non_blocking=True)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(5):
            dst.copy_(src, non_blocking=True)
        e1.record()
        torch.cuda.synchronize()
        rates.append(5 * h.numel() / (e0.elapsed_time(e1) * 1e-3))
    return rates[0], rates[1]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lines", type=int, default=1_000_000, help="corpus lines (streamed --passes times)")
    ap.add_argument("--chunk", type=int, default=250_000)
    ap.add_argument("--passes", type=int, default=40, help="timed passes over the corpus (40 x 1M lines: ~0.2 s, steadier than 8)")
    ap.add_argument("--lag", type=int, default=3)
    ap.add_argument("--output", default="wire", choices=("wire", "json"))
    ap.add_argument("--check", action="store_true")
    ap.add_argument("--profile", action="store_true", help="cProfile the timed loop (top 30 by own time, stderr)")
    args = ap.parse_args()
    import torch
    from pysignalduino_amd import frontend, runtime, synth
    from pysignalduino_amd.sd_protocols import SDProtocols
    torch.cuda.set_device(0)
    sp = frontend.SignalParser(SDProtocols(mc_mode="fixed"))
    bk = sp.protocols._ensure().bank
    cache = os.path.join(os.environ.get("TMPDIR", "/tmp"), f"sdx_lines_{args.lines}_45_1-1-1_0.3.npz")
    if os.path.exists(cache):
        z = np.load(cache)
        data, offsets = z["data"], z["offsets"]
    else:
        lines, _ = synth.line_corpus(bk.protocols, args.lines, seed=45, mix=(1, 1, 1), compress_frac=0.3)
        data, offsets, bad = frontend.pack_lines(lines)
        assert not bad
        np.savez(cache, data=data, offsets=offsets)
    C = args.chunk
    nck = (len(offsets) - 1) // C
    assert nck >= 2, "need at least two chunks"
    # the chunks in pinned host memory (the lines as the transports deliver them), offsets rebased
    chunks = []
    for k in range(nck):
        o = offsets[k * C: (k + 1) * C + 1].astype(np.int64)
        b = torch.from_numpy(data[o[0]: o[-1]].copy()).pin_memory()
        chunks.append((b, o - o[0]))
    maxb = max(b.numel() for b, _ in chunks)
    ls = sp.stream(chunk_lines=C, chunk_bytes=maxb, output=args.output, lag=args.lag)
    # warm-up: one pass through every stage (kernels loaded, buffers touched)
    for b, o in chunks[:2]:
        ls.submit_packed(b, o)
    ls.drain()
    ls.kernel_events.clear()
    ls.h2d_bytes = ls.d2h_bytes = 0
    nsteps = nck * args.passes
    first = None
    host_t = 0.0
    torch.cuda.synchronize()
    prof = None
    if args.profile:
        import cProfile
        prof = cProfile.Profile()
        prof.enable()
    t0 = time.perf_counter()
    for k in range(nsteps):
        b, o = chunks[k % nck]
        h0 = time.perf_counter()
        ls.submit_packed(b, o)
        for r in ls.poll():
            if first is None and args.check:
                first = r.detach()
        host_t += time.perf_counter() - h0
    for r in ls.drain():
        if first is None and args.check:
            first = r.detach()
    dt = time.perf_counter() - t0
    if prof is not None:
        import pstats
        prof.disable()
        pstats.Stats(prof, stream=sys.stderr).sort_stats("tottime").print_stats(30)
    total = nsteps * C
    ke = ls.kernel_events
    k_parse = float(np.median([a.elapsed_time(b) * 1e-3 for a, b, _, _ in ke]))
    k_demod = float(np.median([c.elapsed_time(d) * 1e-3 for _, _, c, d in ke]))
    span = [ke[i][0].elapsed_time(ke[i][3]) * 1e-3 for i in range(len(ke))]
    # the device's time per chunk over the whole run: first chunk's parse start -> last chunk's demod
    # end, / chunks (consecutive chunks' demodulations overlap on two streams, so the per-chunk event
    # pairs above include their sharing and do not add up)
    dev_per_chunk = ke[0][0].elapsed_time(ke[-1][3]) * 1e-3 / len(ke)
    per_chunk = dt / nsteps
    h2d_rate, d2h_rate = copy_rates(torch, chunks[0][0].numpy())
    stages = {"kernels (parse + demod + serialise)": min(k_parse + k_demod, dev_per_chunk),
              "H2D": ls.h2d_bytes / nsteps / h2d_rate, "D2H": ls.d2h_bytes / nsteps / d2h_rate,
              "host (submit + poll)": host_t / nsteps}
    res = {
        "metric": "raw firmware lines/sec end to end: pinned host lines -> parse + demodulate + serialise -> results "
                  "in pinned host memory (PCIe both ways, overlapped; SignalParser.stream)",
        "value": total / dt, "unit": "lines/s", "n_gpus": 1, "lines": total, "chunk_lines": C, "lag": args.lag,
        "output": args.output, "ms_per_chunk": 1e3 * per_chunk,
        "kernels_ms_per_chunk": {"parse+select": 1e3 * k_parse, "demod+serialise": 1e3 * k_demod},
        "chunk_span_ms_median": 1e3 * float(np.median(span)),
        "host_ms_per_chunk": 1e3 * host_t / nsteps,
        "hbm_resident_lines_per_s": C / (k_parse + k_demod),
        "device_ms_per_chunk": 1e3 * dev_per_chunk, "device_lines_per_s": C / dev_per_chunk,
        "pcie": {"h2d_bytes_per_line": ls.h2d_bytes / total, "d2h_bytes_per_line": ls.d2h_bytes / total,
                 "h2d_GB_per_s": ls.h2d_bytes / dt / 1e9, "d2h_GB_per_s": ls.d2h_bytes / dt / 1e9},
        "stage_ms_per_chunk": {k: 1e3 * v for k, v in stages.items()},
        "link_GB_per_s": {"h2d": h2d_rate / 1e9, "d2h": d2h_rate / 1e9},
        "data": "synthetic firmware lines (synth.line_corpus: MU/MS/MC 1/3 each, 30 % of MU/MS Mred=1 compressed)",
    }
    res["bound"] = max(stages, key=stages.get)
    if args.check:
        b, o = chunks[0]
        b = b.numpy()
        lines = [b[o[i]: o[i + 1]].tobytes() for i in range(C)]
        bad = 0
        if args.output == "json":
            exp = sp.parse_lines_json(lines)
            got = first.texts()
            for i in range(C):
                e, g = exp[i], got[i]
                if isinstance(e, Exception):
                    bad += not isinstance(g, type(e))
                else:
                    bad += e != g
        else:
            exp = sp.parse_lines(lines)
            lk = {runtime.LINE_MU: "MU", runtime.LINE_MS: "MS", runtime.LINE_MC: "MC", runtime.LINE_MN: "MN"}
            names = first.names
            dec = {nm: first.decode(j) for j, nm in enumerate(names)}
            pid = {"MU": bk.mu_pids, "MS": bk.ms_pids, "MC": bk.mc_pids, "MN": bk.mn_pids}
            for i in range(C):
                e = exp[i]
                if i in first.host:
                    g = first.host[i]
                    bad += (type(g) is not type(e)) if isinstance(e, Exception) else \
                        [(m.protocol_id, m.payload) for m in g] != [(m.protocol_id, m.payload) for m in e]
                    continue
                nm = lk.get(int(first.kind[i]))
                if isinstance(e, Exception) or nm is None or nm not in dec or int(first.status[i]) != runtime.LS_OK:
                    bad += (not isinstance(e, Exception)) and bool(e)
                    continue
                d, rc, h = dec[nm]
                dd = d[i]
                got = [(str(pid[nm][int(x["proto"])]),
                        h[int(x["payload_off"]): int(x["payload_off"]) + int(x["payload_len"])].tobytes().decode("latin-1"))
                       for x in rc[int(dd["rec_begin"]): int(dd["rec_begin"]) + int(dd["n_rec"])]]
                bad += got != [(m.protocol_id, m.payload) for m in e]
        res["check"] = {"lines": C, "mismatches": int(bad)}
        if bad:
            print(json.dumps(res), flush=True)
            raise SystemExit(f"--check: {bad} mismatching lines")
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
