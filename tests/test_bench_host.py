"""Host logic of bench.py that needs no GPU: the watchdog around the with_gather window
(bench.run_with_deadline) — a collective that never completes must not cost the headline line."""
import threading
import time

import pytest

import bench


def test_deadline_not_reached():
    fired = threading.Event()
    assert bench.run_with_deadline(lambda: 42, 5.0, fired.set) == 42
    time.sleep(0.05)
    assert not fired.is_set()


def test_deadline_fires_while_the_window_hangs():
    fired = threading.Event()

    def hung():  # stands in for a window stuck in a collective: returns only after the watchdog fired
        assert fired.wait(5.0), "watchdog did not fire"
        return "late"

    t0 = time.perf_counter()
    assert bench.run_with_deadline(hung, 0.05, fired.set) == "late"
    assert fired.is_set() and time.perf_counter() - t0 < 2.0


def test_deadline_cancelled_on_error():
    fired = threading.Event()

    def boom():
        raise RuntimeError("exchange failed")

    with pytest.raises(RuntimeError):
        bench.run_with_deadline(boom, 0.2, fired.set)
    time.sleep(0.4)
    assert not fired.is_set()  # the failed window is reported as an error, the timer is gone
