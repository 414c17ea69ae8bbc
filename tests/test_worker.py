import threading
import time

import pytest
import torch

from torchgpipe_amd.microbatch import Batch
from torchgpipe_amd.stream import CPUStream
from torchgpipe_amd.worker import Task, WorkerPool, spawn_workers


class fake_device:
    """A device-like object the workers accept without touching a backend."""
    type = 'fake'
    index = None


def test_join_running_workers():
    count = 0

    def counter():
        nonlocal count
        time.sleep(0.1)
        count += 1
        return Batch(())

    with spawn_workers([fake_device() for _ in range(10)]) as (in_queues, out_queues):
        def call_in_worker(i, f):
            in_queues[i].put(Task(CPUStream, compute=f, finalize=None))

        for i in range(10):
            call_in_worker(i, counter)
    assert count == 10


def test_join_running_workers_with_exception():
    class Boom(Exception):
        pass

    count = 0

    def counter():
        nonlocal count
        time.sleep(0.1)
        count += 1
        return Batch(())

    with pytest.raises(Boom):
        with spawn_workers([fake_device() for _ in range(10)]) as (in_queues, out_queues):
            for i in range(10):
                in_queues[i].put(Task(CPUStream, compute=counter, finalize=None))
            raise Boom
    assert count == 10


def test_compute_multithreading():
    """Task.compute runs concurrently on different device threads."""
    thread_ids = set()

    def log_thread_id():
        thread_ids.add(threading.current_thread().ident)
        return Batch(())

    with spawn_workers([fake_device() for _ in range(2)]) as (in_queues, out_queues):
        for i in range(2):
            in_queues[i].put(Task(CPUStream, compute=log_thread_id, finalize=None))
            out_queues[i].get()
    assert len(thread_ids) == 2


def test_compute_success():
    def _42():
        return Batch(torch.tensor(42))

    with spawn_workers([torch.device('cpu')]) as (in_queues, out_queues):
        in_queues[0].put(Task(CPUStream, compute=_42, finalize=None))
        ok, (task, batch) = out_queues[0].get()
        assert ok
        assert isinstance(batch, Batch)
        assert batch[0].item() == 42


def test_compute_exception():
    def zero_div():
        0 / 0

    with spawn_workers([torch.device('cpu')]) as (in_queues, out_queues):
        in_queues[0].put(Task(CPUStream, compute=zero_div, finalize=None))
        ok, exc_info = out_queues[0].get()
        assert not ok
        assert isinstance(exc_info, tuple)
        assert issubclass(exc_info[0], ZeroDivisionError)


@pytest.mark.parametrize('grad_mode', [True, False])
def test_grad_mode(grad_mode):
    def detect_grad_enabled():
        x = torch.rand(1, requires_grad=torch.is_grad_enabled())
        return Batch(x)

    with torch.set_grad_enabled(grad_mode):
        with spawn_workers([torch.device('cpu')]) as (in_queues, out_queues):
            in_queues[0].put(Task(CPUStream, compute=detect_grad_enabled, finalize=None))
            _, (_, batch) = out_queues[0].get()
    assert batch[0].requires_grad == grad_mode


@pytest.mark.parametrize('grad_mode', [True, False])
def test_persistent_pool_follows_task_grad_mode(grad_mode):
    pool = WorkerPool()
    in_queues, out_queues = pool.queues([torch.device('cpu')])
    with torch.set_grad_enabled(grad_mode):
        task = Task(CPUStream, compute=lambda: Batch(torch.rand(1, requires_grad=
                                                                torch.is_grad_enabled())),
                    finalize=None)
    in_queues[0].put(task)
    _, (_, batch) = out_queues[0].get()
    pool.close()
    assert batch[0].requires_grad == grad_mode


def test_worker_per_device():
    cpu = torch.device('cpu')
    cpu0 = torch.device('cpu', index=0)
    fake1 = fake_device()
    fake2 = fake_device()
    with spawn_workers([cpu, cpu, cpu0, fake1, fake2]) as (in_queues, out_queues):
        assert len(in_queues) == len(out_queues) == 5
        # cpu and cpu:0 are the same device -> one worker
        assert in_queues[0] is in_queues[1] is in_queues[2]
        assert in_queues[3] is not in_queues[4]
