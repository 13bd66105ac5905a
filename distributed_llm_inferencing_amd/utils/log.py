"""Structured logging: JSON lines to ``logs/<component>.log`` plus a
human-readable console handler. The reference promised ``master/logs/django.log`` and
``worker/logs/worker.log`` (README.md:175,185) but never configured them."""
from __future__ import annotations

import json
import logging
import os
import time
from pathlib import Path


class JsonFormatter(logging.Formatter):
    def format(self, rec: logging.LogRecord) -> str:
        d = {"ts": round(time.time(), 6), "level": rec.levelname, "logger": rec.name,
             "msg": rec.getMessage(), "pid": os.getpid()}
        if rec.exc_info:
            d["exc"] = self.formatException(rec.exc_info)
        return json.dumps(d)


def setup_logging(component: str, level: str = None, log_dir: str = None) -> logging.Logger:
    level = level or os.environ.get("DLI_LOG_LEVEL", "INFO")
    log_dir = log_dir or os.environ.get("DLI_LOG_DIR", "logs")
    root = logging.getLogger()
    root.setLevel(level)
    if not any(getattr(h, "_dli", False) for h in root.handlers):
        Path(log_dir).mkdir(parents=True, exist_ok=True)
        fh = logging.FileHandler(Path(log_dir) / f"{component}.log")
        fh.setFormatter(JsonFormatter())
        fh._dli = True
        ch = logging.StreamHandler()
        ch.setFormatter(logging.Formatter("%(asctime)s %(levelname)s %(name)s: %(message)s"))
        ch._dli = True
        root.addHandler(fh)
        root.addHandler(ch)
    return logging.getLogger(f"dli.{component}")
