"""Logger with the reference miner's line format (``miner/src/log.ts:6-27``):

    <epoch_ms> <LEVEL> <file:line>\t<message>

to stderr and (optionally) appended to ``log_path``.
"""
from __future__ import annotations

import logging
import os
import sys


class RefFormatter(logging.Formatter):
    def format(self, record: logging.LogRecord) -> str:
        ms = int(record.created * 1000)
        where = f"{os.path.basename(record.pathname)}:{record.lineno}"
        msg = record.getMessage()
        if record.exc_info:
            msg += "\n" + self.formatException(record.exc_info)
        return f"{ms} {record.levelname} {where}\t{msg}"


def init_logging(log_path=None, level=logging.INFO) -> logging.Logger:
    root = logging.getLogger("arbius")
    root.setLevel(level)
    for h in list(root.handlers):
        root.removeHandler(h)
    sh = logging.StreamHandler(sys.stderr)
    sh.setFormatter(RefFormatter())
    root.addHandler(sh)
    if log_path:
        fh = logging.FileHandler(log_path, mode="a")
        fh.setFormatter(RefFormatter())
        root.addHandler(fh)
    root.propagate = False
    return root
