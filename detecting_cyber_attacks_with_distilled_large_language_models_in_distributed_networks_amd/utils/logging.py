"""Tagged logger with the reference's message shapes + optional JSONL sink.

Reference style (client1.py / server.py): ``[CLIENT 1] Starting model training at
2025-08-29 12:42:31.123456`` and plain ``Client 1 Epoch [1/3], Average Loss: 0.0721``.
``TagLogger.phase`` reproduces the first form, ``TagLogger.info`` the second,
and every record can also go to a JSONL file for machine parsing.
"""
from __future__ import annotations

import json
import os
import sys
import time
from datetime import datetime
from typing import Optional


class TagLogger:
    def __init__(self, tag: str = "[CLIENT 1]", name: str = "Client 1", jsonl_path: Optional[str] = None,
                 enabled: bool = True, stream=None):
        self.tag, self.name = tag, name
        self.enabled = enabled
        self.stream = stream or sys.stdout
        self.jsonl = open(jsonl_path, "a") if jsonl_path else None

    @classmethod
    def for_client(cls, client_id: int, **kw) -> "TagLogger":
        return cls(f"[CLIENT {client_id}]", f"Client {client_id}", **kw)

    @classmethod
    def for_server(cls, **kw) -> "TagLogger":
        return cls("[SERVER]", "Server", **kw)

    def _emit(self, line: str, kind: str, **fields):
        if self.enabled:
            print(line, file=self.stream, flush=True)
        if self.jsonl:
            rec = {"ts": time.time(), "tag": self.tag, "kind": kind, "msg": line}
            rec.update(fields)
            self.jsonl.write(json.dumps(rec) + "\n")
            self.jsonl.flush()

    def phase(self, msg: str, **fields):
        """'[CLIENT 1] <msg> at <datetime.now()>'"""
        self._emit(f"{self.tag} {msg} at {datetime.now()}", "phase", **fields)

    def __call__(self, msg: str, **fields):
        self.phase(msg, **fields)

    def info(self, msg: str, **fields):
        """'Client 1 <msg>'"""
        self._emit(f"{self.name} {msg}", "info", **fields)

    def raw(self, msg: str, **fields):
        self._emit(msg, "raw", **fields)

    def metric(self, name: str, **fields):
        self._emit(f"{self.tag} metric {name} {json.dumps(fields, default=float)}", "metric", name=name, **fields)

    def close(self):
        if self.jsonl:
            self.jsonl.close()
            self.jsonl = None
