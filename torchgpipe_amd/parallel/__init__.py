"""Multi-process parallelism on MI355X: pipeline stages over RCCL point-to-point."""
from torchgpipe_amd.parallel.graph import StepGraph
from torchgpipe_amd.parallel.p2p import P2P, TensorMeta
from torchgpipe_amd.parallel.stage import PipelineStage, signature_of

__all__ = ['PipelineStage', 'P2P', 'TensorMeta', 'signature_of', 'StepGraph']
