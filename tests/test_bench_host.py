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


def test_child_env_drops_launcher_variables():
    """The child configs of the driver's line (bench.other_configs) are fresh one-rank runs: under
    torch.distributed.run they must not inherit its rendezvous variables — TORCHELASTIC_USE_AGENT_STORE made a
    child's process group wait forever as a client of a store no one served (found on the GPU box, round 6)."""
    environ = {"MASTER_ADDR": "127.0.0.1", "MASTER_PORT": "29555", "RANK": "0", "LOCAL_RANK": "0", "WORLD_SIZE": "1",
               "LOCAL_WORLD_SIZE": "1", "GROUP_RANK": "0", "GROUP_WORLD_SIZE": "1", "ROLE_RANK": "0",
               "ROLE_NAME": "default", "ROLE_WORLD_SIZE": "1", "TORCHELASTIC_USE_AGENT_STORE": "True",
               "TORCHELASTIC_RUN_ID": "none", "HSA_ENABLE_IPC_MODE_LEGACY": "0", "PATH": "/usr/bin",
               "OMP_NUM_THREADS": "16"}
    env = bench.child_env(environ)
    assert env == {"HSA_ENABLE_IPC_MODE_LEGACY": "0", "PATH": "/usr/bin", "OMP_NUM_THREADS": "16"}
