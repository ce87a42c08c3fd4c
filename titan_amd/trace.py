"""Engine tracing (include/titan_gpu_olap.h tgo_trace_*): per-superstep / per-level / per-phase
spans as roctx ranges and as a Chrome-trace JSON (titan_amd/csrc/trace.hpp).  The reference's
only hook is the program runtime in its memory (FulgoraGraphComputer.java:143,307)."""
from __future__ import annotations

import contextlib
import json

from . import _lib as L


def enable(json_path: str | None = None, roctx: bool = False) -> None:
    """Turn tracing on for the process: JSON events collected for `json_path` (flushed by
    flush() and at exit), roctx ranges when `roctx`."""
    flags = (L.TRACE_JSON if json_path else 0) | (L.TRACE_ROCTX if roctx else 0)
    rc = L.load().tgo_trace_enable(json_path.encode() if json_path else None, flags)
    if rc:
        raise ValueError(f"tgo_trace_enable rc={rc}")


def disable() -> None:
    L.load().tgo_trace_enable(None, 0)


def flush(json_path: str | None = None) -> None:
    rc = L.load().tgo_trace_flush(json_path.encode() if json_path else None)
    if rc:
        raise OSError(f"tgo_trace_flush rc={rc}")


def clear() -> None:
    L.load().tgo_trace_clear()


@contextlib.contextmanager
def span(name: str):
    """A caller range (e.g. one GraphComputer job or a bench leg) around the engine's spans."""
    lib = L.load()
    lib.tgo_trace_range_push(name.encode())
    try:
        yield
    finally:
        lib.tgo_trace_range_pop()


def load_events(json_path: str):
    """The traceEvents of a flushed trace file."""
    with open(json_path) as f:
        return json.load(f)["traceEvents"]
