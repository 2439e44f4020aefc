"""Host timeline of the GetTOAs data plane (off unless PPF_TIMELINE=1).

`span(name)` brackets one stage on the calling thread; `dump()` returns the
recorded (name, thread, t0, t1, cpu) tuples (perf_counter seconds; cpu = the
thread's CPU seconds inside the span, time.thread_time) and clears them.
Wall time minus CPU time is waiting: for the device, for I/O, or for the
GIL held by another thread.  `bench.py --fit gettoas --timeline FILE`
writes them with the per-stage breakdown (profiles/r04/gettoas_*timeline*)."""
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
    c0 = time.thread_time()
    try:
        yield
    finally:
        t1 = time.perf_counter()
        c1 = time.thread_time()
        with _lock:
            _spans.append((name, threading.current_thread().name, t0, t1,
                           c1 - c0))


def dump():
    with _lock:
        out = list(_spans)
        del _spans[:]
    return out
