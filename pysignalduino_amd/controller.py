"""Batched parser loop for the controller.

The reference controller decodes one line per iteration (signalduino/controller.py:245-264):

    line = await self._raw_message_queue.get()
    decoded = await asyncio.to_thread(self.parser.parse_line, line)
    if decoded and self.message_callback: await self.message_callback(decoded[0])
    if self.mqtt_publisher and decoded:   await self.mqtt_publisher.publish(decoded[0])
    await self._handle_as_command_response(line)
    await asyncio.sleep(0.01)

:class:`BatchingParserTask` is a drop-in for ``SignalduinoController._parser_task``: it drains the
same queue into micro-batches (up to ``max_batch`` lines, waiting at most ``max_delay`` seconds
after the first one), decodes each batch with ONE ``SignalParser.parse_lines`` call in a worker
thread (one upload, one parse launch, one launch per demodulation kind, one read-back), then
performs the reference's per-line side effects in line order: the first decoded message only to
``message_callback`` and to the MQTT publisher, and ``_handle_as_command_response`` for every line.
A line outside the device contract (``ContractError`` in its slot) is logged and publishes
nothing -- like a line whose parser raised in the reference.

``publish="json"`` publishes the device-built texts instead (``SignalParser.parse_lines_json``,
sdx_serialize_json): ``mqtt_publisher.client.publish(f"{base_topic}/state/messages", text)``, the
call MqttPublisher.publish makes (signalduino/mqtt.py:260-272) with the text its
``_message_to_json`` would build.  ``message_callback`` needs the objects, so it is only allowed
with the default ``publish="objects"``.
"""
from __future__ import annotations

import asyncio
import logging
from typing import Any, List, Optional


class BatchingParserTask:
    def __init__(self, controller: Any, max_batch: int = 4096, max_delay: float = 0.005, publish: str = "objects",
                 logger: Optional[logging.Logger] = None):
        if publish not in ("objects", "json"):
            raise ValueError("publish must be 'objects' or 'json'")
        if publish == "json" and getattr(controller, "message_callback", None):
            raise ValueError("publish='json' produces texts only; message_callback needs publish='objects'")
        if max_batch < 1:
            raise ValueError("max_batch must be >= 1")
        self.c = controller
        self.max_batch = max_batch
        self.max_delay = max_delay
        self.publish = publish
        self.logger = logger or getattr(controller, "logger", None) or logging.getLogger(__name__)
        self.batches = 0
        self.lines = 0

    def install(self) -> "BatchingParserTask":
        """Replace the controller's per-line loop (the attribute its run() schedules)."""
        self.c._parser_task = self.run
        return self

    async def _next_batch(self) -> List[Any]:
        q: asyncio.Queue = self.c._raw_message_queue
        batch = [await q.get()]
        loop = asyncio.get_running_loop()
        deadline = loop.time() + self.max_delay
        while len(batch) < self.max_batch:
            try:
                batch.append(q.get_nowait())
                continue
            except asyncio.QueueEmpty:
                pass
            remaining = deadline - loop.time()
            if remaining <= 0:
                break
            try:
                batch.append(await asyncio.wait_for(q.get(), remaining))
            except asyncio.TimeoutError:
                break
        return batch

    async def _publish_json(self, text: str) -> None:
        pub = self.c.mqtt_publisher
        client = getattr(pub, "client", None)
        if not client:
            self.logger.warning("Attempted to publish without an active MQTT client.")
            return
        try:
            await client.publish(f"{pub.base_topic}/state/messages", text)
        except Exception:  # noqa: BLE001  (mqtt.py:271-272)
            self.logger.error("Failed to publish message", exc_info=True)

    async def run(self) -> None:
        c = self.c
        while not c._stop_event.is_set():
            try:
                batch = await self._next_batch()
                lines = [ln for ln in batch if ln]
                if lines:
                    parse = c.parser.parse_lines_json if self.publish == "json" else c.parser.parse_lines
                    results = await asyncio.to_thread(parse, lines)
                    self.batches += 1
                    self.lines += len(lines)
                    for line, res in zip(lines, results):
                        if isinstance(res, Exception):  # parse_line raised for this line
                            self.logger.error("Parser error for line %r: %s", line, res)
                            res = None
                        if self.publish == "json":
                            if res is not None and c.mqtt_publisher:
                                await self._publish_json(res)
                        else:
                            if res and c.message_callback:
                                await c.message_callback(res[0])
                            if c.mqtt_publisher and res:
                                await c.mqtt_publisher.publish(res[0])
                        await c._handle_as_command_response(line)
                await asyncio.sleep(0)
            except asyncio.CancelledError:
                raise
            except Exception as e:  # noqa: BLE001  (controller.py:262-264)
                self.logger.error(f"Parser task error: {e}")
                break
