from torch import nn

from torchgpipe_amd.skip import Namespace, pop, skippable, stash
from torchgpipe_amd.skip.layout import inspect_skip_layout


class Pass(nn.Module):
    def forward(self, x):
        return x


@skippable(stash=['foo'])
class StashFoo(nn.Module):
    def forward(self, x):
        yield stash('foo', x)
        return x


@skippable(pop=['foo'])
class PopFoo(nn.Module):
    def forward(self, x):
        foo = yield pop('foo')
        return x + foo


@skippable(stash=['bar'])
class StashBar(nn.Module):
    def forward(self, x):
        yield stash('bar', x)
        return x


@skippable(pop=['bar'])
class PopBar(nn.Module):
    def forward(self, x):
        bar = yield pop('bar')
        return x + bar


def policies(*parts):
    layout = inspect_skip_layout(list(parts))
    return [list(layout.copy_policy(i)) for i in range(len(parts))]


def test_no_skippables():
    assert policies(nn.Sequential(Pass()), nn.Sequential(Pass())) == [[], []]


def test_inner_partition():
    assert policies(nn.Sequential(StashFoo(), PopFoo()), nn.Sequential(Pass())) == [[], []]


def test_adjoining_partitions():
    assert policies(nn.Sequential(StashFoo()), nn.Sequential(PopFoo())) == \
        [[], [(0, None, 'foo')]]


def test_far_partitions():
    assert policies(nn.Sequential(StashFoo()), nn.Sequential(Pass()),
                    nn.Sequential(PopFoo())) == [[], [], [(0, None, 'foo')]]


def test_pop_2_from_different_partitions():
    # sorted by source partition, not by pop order
    assert policies(nn.Sequential(StashFoo()), nn.Sequential(StashBar()),
                    nn.Sequential(PopBar(), PopFoo())) == \
        [[], [], [(0, None, 'foo'), (1, None, 'bar')]]


def test_namespace():
    ns1, ns2 = Namespace(), Namespace()
    assert policies(nn.Sequential(StashFoo().isolate(ns1)), nn.Sequential(StashFoo().isolate(ns2)),
                    nn.Sequential(PopFoo().isolate(ns2), PopFoo().isolate(ns1))) == \
        [[], [], [(0, ns1, 'foo'), (1, ns2, 'foo')]]


def test_send_policy_is_the_mirror_of_copy_policy():
    layout = inspect_skip_layout([nn.Sequential(StashFoo()), nn.Sequential(StashBar()),
                                  nn.Sequential(PopBar(), PopFoo())])
    assert list(layout.send_policy(0)) == [(2, None, 'foo')]
    assert list(layout.send_policy(1)) == [(2, None, 'bar')]
    assert list(layout.send_policy(2)) == []
    assert layout.requires_copy(None, 'foo')
    assert not layout.requires_copy(None, 'unknown')
