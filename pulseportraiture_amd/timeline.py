"""Host timeline of the GetTOAs data plane (off unless PPF_TIMELINE=1).

`span(name)` brackets one stage on the calling thread; `dump()` returns the
recorded (name, thread, t0, t1) tuples (perf_counter seconds) and clears
them.  tools/gettoas_timeline.py turns them into the per-stage breakdown
committed under profiles/."""
import os
import threading
import time
from contextlib import contextmanager

ENABLED = os.environ.get("PPF_TIMELINE", "0") == "1"
_spans = []
_lock = threading.Lock()


@contextmanager
def span(name):
    if not ENABLED:
        yield
        return
    t0 = time.perf_counter()
    try:
        yield
    finally:
        t1 = time.perf_counter()
        with _lock:
            _spans.append((name, threading.current_thread().name, t0, t1))


def dump():
    with _lock:
        out = list(_spans)
        del _spans[:]
    return out
