import copy

from torch import nn

from torchgpipe_amd.skip import Namespace, skippable, stash


def test_namespace_difference():
    assert Namespace() != Namespace()


def test_namespace_copy():
    ns = Namespace()
    assert copy.copy(ns) == ns
    assert copy.copy(ns) is not ns


def test_none_is_the_default_namespace():
    assert isinstance(None, Namespace)


def test_skippable_repr():
    @skippable(stash=['hello'])
    class Hello(nn.Module):
        def __init__(self):
            super().__init__()
            self.conv = nn.Conv2d(1, 1, 1)

        def forward(self, x):
            yield stash('hello', x)
            return self.conv(x)

    assert repr(Hello()) == '''
@skippable(Hello(
  (conv): Conv2d(1, 1, kernel_size=(1, 1), stride=(1, 1))
))
'''.strip()
