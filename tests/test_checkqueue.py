"""Script-check queue (csrc/util/checkqueue.{h,cpp}); parity: reference
src/test/checkqueue_tests.cpp (every queued check runs exactly once across the master and
the workers, repeated sessions on one queue) plus the round-2 advisory: idle workers sleep
instead of spinning while a block's UTXO pass has not published new jobs."""
import pytest

from bitcoincashplus_amd import native


@pytest.mark.parametrize("workers,total,step", [(0, 1000, 7), (1, 1, 1), (3, 10007, 13), (7, 50000, 1000)])
def test_every_job_once(workers, total, step):
    s, cnt, wjobs, _ = native.checkqueue_run(workers, total, step)
    assert cnt == 2 * total
    assert s == 2 * total * (total - 1) // 2
    if workers == 0:
        assert wjobs == 0


def test_workers_take_jobs():
    _, cnt, wjobs, _ = native.checkqueue_run(4, 20000, 50, idle_ms=1)
    assert cnt == 40000 and wjobs > 0


def test_idle_session_does_not_spin():
    # jobs trickle in with 20 ms gaps: 8 spinning workers would burn ~8 CPU-s per s of gap
    _, cnt, _, idle_cpu = native.checkqueue_run(8, 10, 1, idle_ms=20)
    assert cnt == 20
    gap_s = 2 * 10 * 0.020
    assert idle_cpu < 0.5 * gap_s, idle_cpu
