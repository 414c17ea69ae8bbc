import pytest
import torch

from torchgpipe_amd.dependency import fork, join
from torchgpipe_amd.skip.portal import Portal
from torchgpipe_amd.stream import default_stream


@pytest.mark.gpu
def test_copy_returns_on_next_device():
    if not torch.cuda.is_available():
        pytest.skip('needs a GPU')
    portal = Portal(torch.rand(1), tensor_life=1)
    phony = torch.zeros(0, requires_grad=True)
    phony = portal.copy(default_stream(torch.device('cpu')),
                        default_stream(torch.device('cuda')), phony)
    assert phony.device.type == 'cuda'


@pytest.mark.parametrize('requires_grad', [True, False])
def test_blue_orange(requires_grad):
    # output = t1 * 2 + t2 with t2 carried through a portal:
    #   t2 -- blue --+          +-- orange --+
    #   t1 --------- Join -- Fork --- Mul --- Add
    t1 = torch.rand(1, requires_grad=True)
    t2 = torch.rand(1, requires_grad=requires_grad)
    portal = Portal(t2, tensor_life=2)
    main = join(t1, portal.blue())
    main, phony = fork(main)
    out = main * 2 + portal.orange(phony)
    out.backward()
    assert torch.allclose(t1.grad, torch.tensor([2.]))
    if requires_grad:
        assert torch.allclose(t2.grad, torch.tensor([1.]))
    else:
        assert t2.grad is None


def test_grad_is_ephemeral():
    t = torch.rand(1, requires_grad=True)
    portal = Portal(t, tensor_life=1)
    portal.put_grad(t)
    assert portal.use_grad() is t
    with pytest.raises(RuntimeError, match='grad in portal has been removed or never set'):
        portal.use_grad()


class TestTensorLife:
    @pytest.fixture
    def new_portal(self):
        made = []

        def make(life):
            t = torch.rand(1, requires_grad=True)
            p = Portal(t, life)
            made.append(p)
            return p, t

        yield make
        # every test must exhaust its portal
        for p in made:
            with pytest.raises(RuntimeError, match='tensor in portal has been removed'):
                p.check_tensor_life()
            assert p.tensor is None

    def test_life_0(self, new_portal):
        p, _ = new_portal(0)
        assert p.tensor is None

    def test_life_1(self, new_portal):
        p, t = new_portal(1)
        assert p.tensor is t
        p.blue()

    def test_life_2(self, new_portal):
        p, t = new_portal(2)
        phony = p.blue()
        assert p.orange(phony).data_ptr() == t.data_ptr()

    def test_life_3(self, new_portal):
        p, t = new_portal(3)
        phony = p.blue()
        assert p.orange(phony).data_ptr() == t.data_ptr()
        assert p.orange(phony).data_ptr() == t.data_ptr()

    def test_life_4(self, new_portal):
        p, t = new_portal(4)
        phony = p.blue()
        p.orange(phony)
        p.orange(phony)
        p.blue()

    def test_life_3_plus_1(self, new_portal):
        p, t = new_portal(3)
        phony = p.blue()
        p.orange(phony)
        p.orange(phony)
        p.put_tensor(torch.rand(1, requires_grad=True), tensor_life=1)
        p.blue()
