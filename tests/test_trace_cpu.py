"""CPU: the trace emitter (titan_amd/csrc/trace.cpp) — caller ranges nest per thread and come
out as Chrome-trace complete events with host timestamps; enable/flush/clear semantics."""
import json
import threading

import pytest

from titan_amd import _lib as L
from titan_amd import trace


def test_ranges_are_written_as_complete_events(tmp_path):
    path = str(tmp_path / "t.json")
    trace.enable(path)
    trace.clear()
    try:
        with trace.span("job"):
            with trace.span("superstep 0"):
                pass
            with trace.span("superstep 1"):
                pass
        t = threading.Thread(target=lambda: trace.span("worker").__enter__() or L.load().tgo_trace_range_pop())
        t.start()
        t.join()
        trace.flush()
    finally:
        trace.disable()
    ev = trace.load_events(path)
    names = [e["name"] for e in ev]
    assert sorted(names) == ["job", "superstep 0", "superstep 1", "worker"]
    by = {e["name"]: e for e in ev}
    for e in ev:
        assert e["ph"] == "X" and e["cat"] == "host" and e["dur"] >= 0
    job = by["job"]
    for k in ("superstep 0", "superstep 1"):       # nested inside the job's interval
        assert job["ts"] <= by[k]["ts"] and by[k]["ts"] + by[k]["dur"] <= job["ts"] + job["dur"] + 1e-3
    assert by["superstep 0"]["ts"] + by["superstep 0"]["dur"] <= by["superstep 1"]["ts"] + 1e-3
    assert by["worker"]["tid"] != job["tid"]


def test_enable_rules(tmp_path):
    lib = L.load()
    assert lib.tgo_trace_enable(None, L.TRACE_JSON) == L.TGO_E_INVALID      # JSON needs a path
    assert lib.tgo_trace_enable(None, 7) == L.TGO_E_INVALID
    assert lib.tgo_trace_range_pop() == L.TGO_E_STATE                        # nothing pushed
    trace.enable(str(tmp_path / "x.json"))
    trace.clear()
    trace.flush()
    trace.disable()
    with open(tmp_path / "x.json") as f:
        assert json.load(f)["traceEvents"] == []
    with pytest.raises(OSError):
        trace.flush(str(tmp_path / "no" / "such" / "dir.json"))
