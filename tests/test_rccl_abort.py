"""RcclComm failure paths without RCCL (CPU): the library calls are replaced by a recorder.

* ``abort()`` must not wait behind an exchange that is blocked inside the library (a group
  end stuck on a dead peer): it marks the handle dead and aborts it anyway, within its bound;
* ``async_error()`` reports ``BUSY`` (not "healthy") while an exchange holds the handle;
* the pipeline watchdog turns a handle that stays busy past ``DLI_PP_TIMEOUT_S`` into a dead
  peer and aborts the data plane (runtime/__init__.py:533).
"""
import threading
import time

import pytest

from distributed_llm_inferencing_amd import runtime as RT
from distributed_llm_inferencing_amd.parallel import transport as T


class _FakeLib:
    def __init__(self):
        self.aborted = []
        self.block = threading.Event()
        self.entered = threading.Event()

    def dli_comm_exchange(self, h, *args):
        self.entered.set()
        self.block.wait(10.0)           # a group end that never returns on its own
        return 0

    def dli_comm_abort(self, h):
        self.aborted.append(h)
        self.block.set()                # the abort is what releases the blocked call
        return 0

    def dli_comm_async_error(self, h):
        return 0

    def dli_comm_error_string(self, r):
        return b"err"


def _comm(monkeypatch, fake):
    monkeypatch.setattr(RT, "lib", lambda: fake)
    c = RT.RcclComm.__new__(RT.RcclComm)
    c._h, c.world, c.rank = 1234, 2, 0
    c._lock = threading.Lock()
    return c


def test_abort_does_not_wait_for_blocked_exchange(monkeypatch):
    fake = _FakeLib()
    c = _comm(monkeypatch, fake)
    th = threading.Thread(target=lambda: c.exchange([], [], 0), daemon=True)
    th.start()
    assert fake.entered.wait(5.0)
    assert c.async_error() == RT.RcclComm.BUSY      # held, not reported healthy
    t0 = time.monotonic()
    c.abort(wait_s=0.2)
    assert time.monotonic() - t0 < 2.0
    assert fake.aborted == [1234]
    th.join(5.0)
    assert not th.is_alive()
    with pytest.raises(RuntimeError, match="aborted"):
        c.exchange([], [], 0)
    c.abort()                                       # idempotent: no second library abort
    assert fake.aborted == [1234]


def test_abort_when_idle_takes_the_lock(monkeypatch):
    fake = _FakeLib()
    c = _comm(monkeypatch, fake)
    assert c.async_error() == 0
    c.abort()
    assert fake.aborted == [1234] and c._h is None
    assert not c._lock.locked()


def test_watchdog_aborts_a_stuck_exchange(monkeypatch):
    monkeypatch.setenv("DLI_PP_TIMEOUT_S", "0.3")

    class _Busy:
        BUSY = RT.RcclComm.BUSY

        def __init__(self):
            self.aborted = False

        def async_error(self):
            return RT.RcclComm.BUSY

        def abort(self):
            self.aborted = True

    ch = T.PipeChannel.__new__(T.PipeChannel)
    ch.ring, ch.ipc, ch.dead_peer = None, None, None
    ch.rccl = _Busy()
    ch._wd_stop = threading.Event()
    th = threading.Thread(target=ch._watch, args=(0.05,), daemon=True)
    t0 = time.monotonic()
    th.start()
    th.join(5.0)
    assert not th.is_alive()
    assert time.monotonic() - t0 < 3.0
    assert ch.rccl.aborted
    assert "blocked" in ch.dead_peer
    with pytest.raises(T.PeerDied):
        ch.check()
