"""Long skip connections for pipelines (``@skippable`` / ``stash`` / ``pop``)."""
from torchgpipe_amd.skip.namespace import Namespace
from torchgpipe_amd.skip.skippable import pop, skippable, stash, verify_skippables

__all__ = ['skippable', 'stash', 'pop', 'verify_skippables', 'Namespace']
