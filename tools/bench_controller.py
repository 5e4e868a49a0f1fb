#!/usr/bin/env python3
"""Controller-loop benchmark: firmware lines/s through BatchingParserTask.

The raw-message queue is pre-filled with ``--lines`` framed firmware lines (synth.line_corpus
MU/MS/MC + synth.mn_frames MN, 3:1), then the batched parser task drains it: parse_lines (or
parse_lines_json) per micro-batch in a worker thread, then the per-line callback / publish /
command-response awaits of the reference loop against in-process fakes.  The reference loop
(signalduino/controller.py:245-264) decodes one line per iteration and sleeps 10 ms after each,
so it is bounded by 100 lines/s whatever the decoder's speed.

usage: python tools/bench_controller.py [--lines 200000 --max-batch 16384 --publish json]
"""
from __future__ import annotations

import argparse
import asyncio
import json
import logging
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


class _Pub:
    def __init__(self):
        self.n = 0
        self.base_topic = "sd/v1"
        self.client = self

    async def publish(self, *a):
        self.n += 1


class _Ctl:
    def __init__(self, parser):
        self._stop_event = asyncio.Event()
        self._raw_message_queue = asyncio.Queue()
        self.parser = parser
        self.mqtt_publisher = _Pub()
        self.message_callback = None
        self.logger = logging.getLogger("bench")
        self._pending_responses = []    # as SignalduinoController.__init__ (controller.py:65)
        self.ncmd = 0

    async def _handle_as_command_response(self, line):
        self.ncmd += 1


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lines", type=int, default=400_000)
    ap.add_argument("--max-batch", type=int, default=16384)
    ap.add_argument("--publish", default="json", choices=("json", "objects"))
    ap.add_argument("--profile", action="store_true", help="cProfile the timed loop (top 30 by own time, stderr)")
    args = ap.parse_args()
    from pysignalduino_amd import bank as B, synth
    from pysignalduino_amd.controller import BatchingParserTask
    from pysignalduino_amd.frontend import SignalParser
    P = B.Bank().protocols
    n_mn = args.lines // 4
    raw, _ = synth.line_corpus(P, args.lines - n_mn, seed=93)
    raw += [synth.frame(synth.mn_payload(*f)) for f in synth.mn_frames(n_mn, seed=94)]
    lines = [ln.decode("latin-1") for ln in raw]
    sp = SignalParser()
    sp.parse_lines(lines[:2000])        # warm-up: bank upload, kernels loaded

    async def run():
        ctl = _Ctl(sp)
        task = BatchingParserTask(ctl, max_batch=args.max_batch, max_delay=0.002, publish=args.publish)
        runner = asyncio.create_task(task.run())
        warm = lines[: args.max_batch * (task.lag + 2)]   # warm-up: the stream's slots exist, kernels loaded
        for ln in warm:
            ctl._raw_message_queue.put_nowait(ln)
        while task.lines < len(warm):
            await asyncio.sleep(0.001)
        n0, p0, b0 = task.lines, ctl.mqtt_publisher.n, task.batches
        for ln in lines:        # the queue holds the whole corpus when the clock starts
            ctl._raw_message_queue.put_nowait(ln)
        prof = None
        if args.profile:
            import cProfile
            prof = cProfile.Profile()
            prof.enable()
        t0 = time.perf_counter()
        while task.lines - n0 < len(lines):      # every line taken through its effects
            await asyncio.sleep(0.001)
        dt = time.perf_counter() - t0
        if prof is not None:
            import pstats
            prof.disable()
            pstats.Stats(prof, stream=sys.stderr).sort_stats("tottime").print_stats(30)
        ctl._stop_event.set()
        runner.cancel()
        await asyncio.gather(runner, return_exceptions=True)
        return dt, ctl.mqtt_publisher.n - p0, task.batches - b0

    dt, npub, nb = asyncio.run(run())
    print(json.dumps({"metric": "firmware lines/sec through the batched controller loop (SURVEY §8(f) 4)",
                      "value": len(lines) / dt, "unit": "lines/s", "n_gpus": 1, "higher_is_better": True,
                      "config": {"lines": len(lines), "max_batch": args.max_batch, "publish": args.publish,
                                 "batches": nb, "published": npub},
                      "reference_bound": {"value": 100.0, "unit": "lines/s",
                                          "why": "controller.py:252-261: one line per iteration + asyncio.sleep(0.01)"}}))


if __name__ == "__main__":
    main()
