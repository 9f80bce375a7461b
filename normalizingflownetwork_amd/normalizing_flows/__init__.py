"""Flow registry — mirrors ``estimators/normalizing_flows/__init__.py:5``."""

from .bijector import Bijector, Chain, Invert
from .flows import AffineFlow, PlanarFlow, RadialFlow

FLOWS = {"planar": PlanarFlow, "radial": RadialFlow, "affine": AffineFlow}

__all__ = ["FLOWS", "PlanarFlow", "RadialFlow", "AffineFlow", "Bijector", "Chain", "Invert"]
