import pytest
from torch import nn

from torchgpipe_amd.skip import Namespace, skippable, verify_skippables


def layer(stash=(), pop=()):
    @skippable(stash=list(stash), pop=list(pop))
    class Layer(nn.Module):
        pass
    return Layer()


def errors(*layers):
    with pytest.raises(TypeError) as e:
        verify_skippables(nn.Sequential(*layers))
    assert str(e.value).startswith('one or more pairs of stash and pop do not match:')
    return str(e.value)


def test_matching():
    verify_skippables(nn.Sequential(layer(stash=['foo']), layer(pop=['foo'])))


def test_stash_not_pop():
    assert "no module declared 'foo' as poppable but stashed" in errors(layer(stash=['foo']))


def test_pop_unknown():
    assert "'0' declared 'foo' as poppable but it was not stashed" in errors(layer(pop=['foo']))


def test_stash_again():
    assert "'1' redeclared 'foo' as stashable" in errors(
        layer(stash=['foo']), layer(stash=['foo']), layer(pop=['foo']))


def test_pop_again():
    assert "'2' redeclared 'foo' as poppable" in errors(
        layer(stash=['foo']), layer(pop=['foo']), layer(pop=['foo']))


def test_stash_pop_together_different_names():
    verify_skippables(nn.Sequential(layer(stash=['foo']), layer(pop=['foo'], stash=['bar']),
                                    layer(pop=['bar'])))


def test_stash_pop_together_same_name():
    assert "'0' declared 'foo' both as stashable and as poppable" in errors(
        layer(stash=['foo'], pop=['foo']))


def test_double_stash_pop():
    msg = errors(layer(stash=['foo']), layer(pop=['foo']), layer(stash=['foo']),
                 layer(pop=['foo']))
    assert "'2' redeclared 'foo' as stashable" in msg
    assert "'3' redeclared 'foo' as poppable" in msg


def test_double_stash_pop_but_isolated():
    ns1, ns2 = Namespace(), Namespace()
    verify_skippables(nn.Sequential(layer(stash=['foo']).isolate(ns1),
                                    layer(pop=['foo']).isolate(ns1),
                                    layer(stash=['foo']).isolate(ns2),
                                    layer(pop=['foo']).isolate(ns2)))


def test_isolate_only_subset():
    ns = Namespace()
    m = layer(stash=['a', 'b']).isolate(ns, only=['a'])
    assert dict(m.stashable()) == {ns: 'a', None: 'b'}
