"""Hand-written HIP/CDNA4 kernels of the framework and their PyTorch bindings.

* :mod:`.dbn` — DeferredBatchNorm statistics (K1 track, K2 commit)
* :mod:`.fused` — fused Dropout2d → InstanceNorm2d → LeakyReLU (U-Net cell)
* :mod:`.dropout` — Philox dropout with explicit (seed, offset)
* :mod:`.philox` — bit-exact CPU reference of the Philox stream
* :mod:`.misc` — spin kernel (race tests), multi-tensor pack/unpack
"""
from torchgpipe_amd.ops import _ext

available = _ext.available

__all__ = ['available']
