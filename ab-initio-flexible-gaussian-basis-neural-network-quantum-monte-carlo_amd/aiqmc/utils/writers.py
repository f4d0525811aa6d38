"""Per-iteration CSV log, the file contract of AIQMCrelease3/utils/writers.py:7-39.

The drivers open ``Writer(name, schema, directory, iteration_key, log)`` as a context
manager and call ``write(t, **columns)`` once per iteration (``train_states.csv`` with
schema ``['step', 'energy']``, main_all_electrons_adam_muti_GPU.py:166-173,197;
``DMC_states.csv`` with ``['block', 'energy', 'positions']``, DMC/main_dmc.py:154-160).
File format (the contract, not the reference's code): a header line naming the optional
iteration column followed by the schema columns, then one line per ``write`` with the
``str()`` of each value in schema order; a missing column is written empty, an unknown
column raises ``ValueError``; lines are joined with ',' and no quoting is applied.
"""
from __future__ import annotations

import logging
import os
from typing import Any, List, Optional, Sequence, TextIO

__all__ = ["Writer"]


class Writer:
    """Context-managed CSV sink; the file is (re)created on ``__enter__``."""

    def __init__(self, name: str, schema: Sequence[str], directory: str = "logs/",
                 iteration_key: Optional[str] = "t", log: bool = True):
        self.columns: List[str] = [str(c) for c in schema]
        self.path = os.path.join(directory, f"{name}.csv")
        self.iteration_key = iteration_key
        self.echo = log
        self._sink: Optional[TextIO] = None
        os.makedirs(directory, exist_ok=True)

    # -- formatting ---------------------------------------------------------------
    def _header(self) -> str:
        lead = [self.iteration_key] if self.iteration_key else []
        return ",".join(lead + self.columns)

    def _line(self, t: Any, values: dict) -> str:
        unknown = [k for k in values if k not in self.columns]
        if unknown:
            raise ValueError(f"Not a recognized key for writer: {unknown[0]}")
        cells = [str(t)] if self.iteration_key else []
        cells.extend(str(values[c]) if c in values else "" for c in self.columns)
        return ",".join(cells)

    # -- context protocol -------------------------------------------------------------
    def __enter__(self) -> "Writer":
        self._sink = open(self.path, "w", encoding="UTF-8")
        self._sink.write(self._header() + "\n")
        return self

    def write(self, t: Any, **values) -> None:
        if self._sink is None:
            raise RuntimeError("Writer.write outside its `with` block")
        self._sink.write(self._line(t, values) + "\n")
        if self.echo:
            logging.info("Iteration %s: %s", t, values)

    def __exit__(self, exc_type, exc, tb) -> bool:
        if self._sink is not None:
            self._sink.close()
            self._sink = None
        return False
