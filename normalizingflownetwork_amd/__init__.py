"""MI355X-native conditional normalizing-flow ``log_prob`` (drop-in for the flow
path of siboehm/NormalizingFlowNetwork).

Layout:
  csrc/                  HIP kernels for gfx950 + the extern "C" ABI (include/nfn.h):
                         nfn_persistent / nfn_group / nfn_tile (forward, posterior),
                         nfn_grad (fused backward), nfn_misc (reductions),
                         nfn_comm (RCCL all-reduce), nfn_api (validation + dispatch)
  build.py               parallel hipcc build of libnfn_hip.so (in-tree)
  _lib.py                ctypes binding of libnfn_hip.so (no CPU fallback)
  ops.py                 torch-tensor entry points (device memory + stream plumbing),
                         differentiable log_prob (autograd through the fused backward)
  normalizing_flows/     PlanarFlow / RadialFlow / AffineFlow, FLOWS, Chain, Invert
  distribution_layers.py InverseNormalizingFlowLayer and its flow distribution
  estimators.py          NormalizingFlowNetwork (fit / pdf / log_pdf / score) and
                         BayesNormalizingFlowNetwork (posterior score)
  scorers.py             mle / bayesian log-likelihood scorers
  parallel.py            batch-sharded multi-GPU mean log-likelihood (RCCL all-reduce)
"""

from .distribution_layers import FlowDistribution, InverseNormalizingFlowLayer, TensorShape
from .estimators import BayesNormalizingFlowNetwork, NormalizingFlowNetwork
from .normalizing_flows import FLOWS, AffineFlow, Bijector, Chain, Invert, PlanarFlow, RadialFlow

__version__ = "0.1.0"

__all__ = [
    "FLOWS",
    "PlanarFlow",
    "RadialFlow",
    "AffineFlow",
    "Bijector",
    "Chain",
    "Invert",
    "InverseNormalizingFlowLayer",
    "FlowDistribution",
    "TensorShape",
    "NormalizingFlowNetwork",
    "BayesNormalizingFlowNetwork",
]
