import pytest
import torch

from torchgpipe_amd.stream import (CPUStream, StreamPool, current_stream, default_stream,
                                   get_device, is_cuda, new_stream, record_stream, use_device,
                                   use_stream, wait_stream)

gpu = pytest.mark.gpu


def need_gpu():
    if not torch.cuda.is_available():
        pytest.skip('needs a GPU')


class TestCPU:
    def test_new_current_default(self):
        cpu = torch.device('cpu')
        assert new_stream(cpu) is CPUStream
        assert current_stream(cpu) is CPUStream
        assert default_stream(cpu) is CPUStream

    def test_use_device_and_stream_are_noops(self):
        with use_device(torch.device('cpu')):
            pass
        with use_stream(CPUStream):
            assert not is_cuda(CPUStream)

    def test_get_device(self):
        assert get_device(CPUStream) == torch.device('cpu')

    def test_wait_and_record_are_noops(self):
        wait_stream(CPUStream, CPUStream)
        record_stream(torch.rand(1), CPUStream)

    def test_pool_returns_cpu_stream(self):
        pool = StreamPool(3)
        grid = pool.grid([torch.device('cpu')] * 2, 5)
        assert all(s is CPUStream for row in grid for s in row)


@gpu
class TestGPU:
    def test_new_stream(self):
        need_gpu()
        s = new_stream(torch.device('cuda'))
        assert isinstance(s, torch.cuda.Stream)
        assert s != torch.cuda.default_stream()

    def test_use_stream(self):
        need_gpu()
        s = new_stream(torch.device('cuda'))
        with use_stream(s):
            assert current_stream(torch.device('cuda')) == s

    def test_wait_stream_orders_gpu_work(self, gpu_sleep):
        need_gpu()
        source = new_stream(torch.device('cuda'))
        target = new_stream(torch.device('cuda'))
        with use_stream(target):
            gpu_sleep(0.2)
        wait_stream(source, target)
        with use_stream(source):
            assert not source.query()  # source now waits behind the sleep
        source.synchronize()

    def test_wait_stream_cpu_waits_gpu(self, gpu_sleep):
        need_gpu()
        target = new_stream(torch.device('cuda'))
        with use_stream(target):
            gpu_sleep(0.2)
        wait_stream(CPUStream, target)
        assert target.query()

    def test_record_stream_keeps_block_alive(self, gpu_sleep):
        need_gpu()
        stream = new_stream(torch.device('cuda'))
        with use_stream(stream):
            gpu_sleep(0.3)
        x = torch.ones(256, device='cuda')
        ptr = x.data_ptr()
        record_stream(x, stream)
        del x
        y = torch.zeros(256, device='cuda')
        # The block is still in use on `stream`, so the allocator must not reuse it.
        assert y.data_ptr() != ptr
        stream.synchronize()

    def test_record_stream_shifted_view(self, gpu_sleep):
        # A view that starts inside its allocation must still protect the block.
        need_gpu()
        alloc = new_stream(torch.device('cuda'))
        with torch.cuda.stream(alloc):
            x = torch.rand(2, device='cuda')
        y = x[1:]
        assert y.data_ptr() > x.data_ptr()
        user = new_stream(torch.device('cuda'))
        with use_stream(user):
            gpu_sleep(1.0)
            busy = torch.cuda.Event()
            busy.record()
        record_stream(y, user)
        ptr = x.data_ptr()
        del x, y
        alloc.synchronize()
        with torch.cuda.stream(alloc):
            z = torch.rand(2, device='cuda')
        still_busy = not busy.query()
        user.synchronize()
        if not still_busy:  # the spin ended before the reallocation: inconclusive
            pytest.skip('user stream finished before the block was reallocated')
        assert z.data_ptr() != ptr

    def test_pool_ring(self):
        need_gpu()
        pool = StreamPool(2)
        d = torch.device('cuda', 0)
        assert pool.get(d, 0) is pool.get(d, 2)
        assert pool.get(d, 0) is not pool.get(d, 1)
