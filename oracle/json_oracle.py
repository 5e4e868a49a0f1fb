"""CPU restatement of MqttPublisher._message_to_json -- TEST INFRASTRUCTURE ONLY.

signalduino/mqtt.py:227-245: ``asdict(message)``, drop ``"raw"``, ``json.dumps(d, indent=4)``.
``asdict`` keeps the dataclass field order (protocol_id, payload, raw, metadata) and deep-copies the
metadata dict (insertion order kept), so the published text is ``json.dumps`` of
{"protocol_id", "payload", "metadata"} -- the same stdlib ``json`` module the reference calls.
The reference module itself imports aiomqtt (absent here); the parity tests feed this restatement
the reference-recorded DecodedMessage fields of tests/golden/*.json.gz.
"""
from __future__ import annotations

import json
from typing import Any, Dict


def message_to_json(protocol_id: str, payload: str, metadata: Dict[str, Any]) -> str:
    return json.dumps({"protocol_id": protocol_id, "payload": payload, "metadata": metadata}, indent=4)


def published(decoded) -> "str | None":
    """controller.py:254-257: only decoded[0] of a line is published."""
    if not decoded:
        return None
    d = decoded[0]
    if isinstance(d, (list, tuple)):
        return message_to_json(d[0], d[1], d[2])
    return message_to_json(d.protocol_id, d.payload, d.metadata)
