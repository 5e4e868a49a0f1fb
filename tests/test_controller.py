"""Batched controller loop: pysignalduino_amd.controller.BatchingParserTask vs the
reference's per-line _parser_task (signalduino/controller.py:245-264).

CPU tests drive the loop with a scripted parser (no GPU) and check it against a restatement of the
reference loop: same callbacks / publications (first decoded message only) / command-response calls,
in line order, with many lines per parse_lines call.  The GPU test runs the real SignalParser."""
import asyncio
import json
import logging

import pytest

from pysignalduino_amd.controller import BatchingParserTask


class FakeParser:
    """parse_line(line) -> a scripted list; parse_lines = map of it (records the batch sizes)."""

    def __init__(self):
        self.batches = []

    def parse_line(self, line):
        if "boom" in line:
            raise ValueError("contract")
        k = sum(map(ord, line)) % 3
        return [(line, j) for j in range(k)]

    def parse_lines(self, lines):
        self.batches.append(len(lines))
        out = []
        for ln in lines:
            try:
                out.append(self.parse_line(ln))
            except ValueError as e:
                out.append(e)
        return out

    def parse_lines_json(self, lines):
        return [(json.dumps(r[0]) if r else None) if not isinstance(r, Exception) else r
                for r in self.parse_lines(lines)]

    def stream(self, chunk_lines, output="json", lag=3):
        assert output == "json"
        return FakeStream(self, lag)


class _Chunk:
    def __init__(self, texts, cid=0):
        self._t = texts
        self.id = cid

    def texts(self):
        return self._t


class FakeStream:
    """stream.LineStream's contract on the host: submit / poll (finished chunks in order, chunks
    finish ``lag`` submits later) / drain."""

    def __init__(self, parser, lag):
        self.parser, self.lag, self.q, self.submitted = parser, lag, [], 0

    def submit(self, lines):
        self.q.append(_Chunk(self.parser.parse_lines_json(lines), self.submitted))
        self.submitted += 1
        return self.submitted - 1

    def poll(self):
        k = max(0, len(self.q) - self.lag)
        out, self.q = self.q[:k], self.q[k:]
        return out

    def drain(self):
        out, self.q = self.q, []
        return out


class Pub:
    def __init__(self):
        self.sent = []
        self.base_topic = "t/v1"
        self.client = self

    async def publish(self, *a):
        self.sent.append(a)


class Ctl:
    def __init__(self, parser, callback=True):
        self._stop_event = asyncio.Event()
        self._raw_message_queue = asyncio.Queue()
        self.parser = parser
        self.mqtt_publisher = Pub()
        self.cb = []
        self.cmd = []
        self.message_callback = self._cb if callback else None
        self.logger = logging.getLogger("test")

    async def _cb(self, m):
        self.cb.append(m)

    async def _handle_as_command_response(self, line):
        self.cmd.append(line)


def reference_side_effects(parser, lines):
    """controller.py:245-264 restated (the per-line loop's observable effects)."""
    cb, sent, cmd = [], [], []
    for line in lines:
        if not line:
            continue
        try:
            decoded = parser.parse_line(line)
        except ValueError:
            decoded = []          # in the reference the task would stop; lines outside the contract
        if decoded:
            cb.append(decoded[0])
            sent.append((decoded[0],))
        cmd.append(line)
    return cb, sent, cmd


async def _drive(ctl, task, lines, chunk=37):
    runner = asyncio.create_task(task.run())
    for i in range(0, len(lines), chunk):
        for ln in lines[i:i + chunk]:
            await ctl._raw_message_queue.put(ln)
        await asyncio.sleep(0)
    while not ctl._raw_message_queue.empty() or len(ctl.cmd) < len([x for x in lines if x]):
        await asyncio.sleep(0.01)
    ctl._stop_event.set()
    runner.cancel()
    await asyncio.gather(runner, return_exceptions=True)


def test_batched_loop_matches_reference_loop():
    lines = [f"MS;P0={i};D=01;" for i in range(500)] + ["", "boom"] + [f"MU;{i}" for i in range(300)]
    parser = FakeParser()
    ctl = Ctl(parser)
    task = BatchingParserTask(ctl, max_batch=64, max_delay=0.01)
    asyncio.run(_drive(ctl, task, lines))
    cb, sent, cmd = reference_side_effects(FakeParser(), lines)
    assert ctl.cb == cb and ctl.mqtt_publisher.sent == sent and ctl.cmd == cmd
    assert max(parser.batches) > 1 and all(b <= 64 for b in parser.batches)
    assert task.lines == 801


@pytest.mark.parametrize("stream", [True, False])
def test_batched_loop_json_mode(stream):
    """publish='json', through the pipelined stream (chunks finish 3 submits later, the rest when the
    queue runs dry) and through parse_lines_json: the same publications in line order."""
    lines = [f"MC;D={i};" for i in range(2000)] + ["boom", ""] + [f"MC;D=x{i};" for i in range(77)]
    parser = FakeParser()
    ctl = Ctl(parser, callback=False)
    task = BatchingParserTask(ctl, publish="json", max_batch=50, max_delay=0.005, stream=stream).install()
    assert ctl._parser_task == task.run
    asyncio.run(_drive(ctl, task, lines))
    _, sent, cmd = reference_side_effects(FakeParser(), lines)
    assert ctl.mqtt_publisher.sent == [("t/v1/state/messages", json.dumps(s[0])) for s in sent]
    assert ctl.cmd == cmd and task.lines == len(cmd)
    with pytest.raises(ValueError):
        BatchingParserTask(Ctl(parser), publish="json")


def test_command_response_skipped_only_without_effect():
    """_handle_as_command_response (controller.py:360-387) is skipped only while the controller has
    no pending responses and does not log at DEBUG; otherwise it runs for every line."""
    lines = [f"MS;P0={i};D=01;" for i in range(300)]
    for pending, level, want in (([], logging.WARNING, 0), (["cmd"], logging.WARNING, 300),
                                 ([], logging.DEBUG, 300)):
        parser = FakeParser()
        ctl = Ctl(parser)
        ctl._pending_responses = pending
        ctl.logger = logging.getLogger(f"test.skip.{level}.{len(pending)}")
        ctl.logger.setLevel(level)
        task = BatchingParserTask(ctl, max_batch=64, max_delay=0.01)

        async def go():
            runner = asyncio.create_task(task.run())
            for ln in lines:
                ctl._raw_message_queue.put_nowait(ln)
            while task.lines < len(lines):
                await asyncio.sleep(0.01)
            ctl._stop_event.set()
            runner.cancel()
            await asyncio.gather(runner, return_exceptions=True)

        asyncio.run(go())
        assert len(ctl.cmd) == want, (pending, level, len(ctl.cmd))
        cb, _, _ = reference_side_effects(FakeParser(), lines)
        assert ctl.cb == cb


@pytest.mark.gpu
def test_batched_loop_with_the_gpu_parser():
    """Real lines through the real SignalParser: the published messages are parse_line(line)[0]."""
    from pysignalduino_amd import bank as B
    from pysignalduino_amd import synth
    from pysignalduino_amd.frontend import SignalParser
    P = B.Bank().protocols
    raw, _ = synth.line_corpus(P, 3000, seed=91)
    raw += [synth.frame(synth.mn_payload(*f)) for f in synth.mn_frames(1000, seed=92)]
    lines = [ln.decode("latin-1") for ln in raw]
    sp = SignalParser()
    ctl = Ctl(sp)
    task = BatchingParserTask(ctl, max_batch=512)
    asyncio.run(_drive(ctl, task, lines, chunk=200))
    exp = [r[0] for r in sp.parse_lines(lines) if not isinstance(r, Exception) and r]
    got = [m[0] for m in ctl.mqtt_publisher.sent]
    key = lambda d: (d.protocol_id, d.payload, d.metadata, d.raw.line)  # noqa: E731
    assert [key(d) for d in got] == [key(d) for d in exp]
    assert [key(d) for d in ctl.cb] == [key(d) for d in exp]
    assert ctl.cmd == lines and task.batches < len(lines) / 4
    # json mode publishes the device texts of the same messages
    from oracle import json_oracle as J
    ctl2 = Ctl(sp, callback=False)
    asyncio.run(_drive(ctl2, BatchingParserTask(ctl2, max_batch=512, publish="json"), lines, chunk=200))
    assert [t for _, t in ctl2.mqtt_publisher.sent] == [J.published([d]) for d in exp]


def test_json_stream_command_turns_follow_state_changes():
    """publish='json' through the stream: a publisher that adds / clears pending responses while
    publishing (as another task could during the await) -- every line gets its command-response turn
    exactly when the reference loop would check true for it (controller.py:245-264, 360-387)."""
    lines = [f"MC;D={i};" for i in range(3000)]
    parser = FakeParser()
    texts = parser.parse_lines_json(lines)

    class TogglePub(Pub):
        def __init__(self, ctl):
            super().__init__()
            self.ctl = ctl

        async def publish(self, *a):
            self.sent.append(a)
            n = len(self.sent)
            if n % 97 == 0:
                self.ctl._pending_responses.append("cmd")
            elif n % 97 == 5:
                self.ctl._pending_responses.clear()

    ctl = Ctl(parser, callback=False)
    ctl._pending_responses = []
    ctl.logger = logging.getLogger("test.toggle")
    ctl.logger.setLevel(logging.WARNING)
    ctl.mqtt_publisher = TogglePub(ctl)
    # the reference loop's turns under the same state changes
    exp_cmd, pend, nsent = [], [], 0
    for ln, t in zip(lines, texts):
        if t is not None:
            nsent += 1
            if nsent % 97 == 0:
                pend.append("cmd")
            elif nsent % 97 == 5:
                pend.clear()
        if pend:
            exp_cmd.append(ln)
    task = BatchingParserTask(ctl, publish="json", max_batch=200, max_delay=0.005)

    async def go():
        runner = asyncio.create_task(task.run())
        for ln in lines:
            ctl._raw_message_queue.put_nowait(ln)
        while task.lines < len(lines):
            await asyncio.sleep(0.01)
        ctl._stop_event.set()
        runner.cancel()
        await asyncio.gather(runner, return_exceptions=True)

    asyncio.run(go())
    assert [t for _, t in ctl.mqtt_publisher.sent] == [t for t in texts if t is not None]
    assert ctl.cmd == exp_cmd and 0 < len(exp_cmd) < len(lines)


@pytest.mark.parametrize("how", ["stop", "error"])
def test_json_stream_publishes_in_flight_chunks_on_exit(how):
    """when the stop event is set (or an error ends the loop) while chunks are in flight
    in the stream, those chunks are drained and published: every line taken off the queue gets its
    publication and command-response turn, as in the reference loop."""
    lines = [f"MC;D={i};" for i in range(1000)]
    parser = FakeParser()

    class StopPub(Pub):
        async def publish(self, *a):
            self.sent.append(a)
            if len(self.sent) == 1:
                ctl._stop_event.set()

    class FailStream(FakeStream):
        polls = 0

        def poll(self):
            FailStream.polls += 1
            if FailStream.polls == 6:
                raise RuntimeError("injected poll failure")
            return super().poll()

    ctl = Ctl(parser, callback=False)
    if how == "stop":
        ctl.mqtt_publisher = StopPub()
    else:
        parser.stream = lambda chunk_lines, output="json", lag=3: FailStream(parser, lag)
    task = BatchingParserTask(ctl, publish="json", max_batch=40, max_delay=0.005)

    async def go():
        for ln in lines:
            ctl._raw_message_queue.put_nowait(ln)
        await asyncio.wait_for(task.run(), 30)

    asyncio.run(go())
    taken = len(lines) - ctl._raw_message_queue.qsize()
    assert 3 * 40 < taken < len(lines), taken     # chunks were in flight when the loop ended
    _, sent, cmd = reference_side_effects(FakeParser(), lines[:taken])
    assert ctl.cmd == cmd and task.lines == taken
    assert ctl.mqtt_publisher.sent == [("t/v1/state/messages", json.dumps(s[0])) for s in sent]


def test_json_stream_publish_failure_mid_chunk_keeps_lines_aligned():
    """a command-response turn that raises part-way through a chunk ends the loop (as in the
    reference, controller.py:262-264); the chunks the stream still holds are drained and published with
    THEIR OWN lines (results matched by chunk id, not by position): every publication is followed by the
    turn of the line it belongs to, nothing raises IndexError, and the failing chunk's later lines get
    nothing."""
    lines = [f"MC;D={i};" for i in range(600)]
    parser = FakeParser()
    texts = dict(zip(lines, parser.parse_lines_json(lines)))
    ctl = Ctl(parser, callback=False)
    ctl._pending_responses = ["cmd"]          # every line gets its turn
    bad = "MC;D=101;"

    async def handle(line):
        if line == bad:
            raise RuntimeError("injected command-response failure")
        ctl.cmd.append(line)
    ctl._handle_as_command_response = handle
    order = []
    orig = ctl.mqtt_publisher.publish

    async def pub(*a):
        order.append(("pub", a[1]))
        await orig(*a)
    ctl.mqtt_publisher.publish = pub
    task = BatchingParserTask(ctl, publish="json", max_batch=40, max_delay=0.005, lag=3)

    async def go():
        for ln in lines:
            ctl._raw_message_queue.put_nowait(ln)
        await asyncio.wait_for(task.run(), 30)

    asyncio.run(go())
    assert bad not in ctl.cmd and "MC;D=102;" not in ctl.cmd      # the failing chunk stops at the failure
    assert ctl.cmd[:101] == lines[:101]
    later = ctl.cmd[101:]
    assert later and all(int(x[5:-1]) >= 120 for x in later)        # only whole later chunks follow
    # each published text belongs to the line whose turn comes next (or to the failing line)
    pubs = [t for _, t in order]
    want = [texts[ln] for ln in ctl.cmd[:101] + [bad] + later if texts[ln] is not None]
    assert pubs == want
