"""IC engine models on the batch-reactor kernels (reference engines/: engine.py, HCCI.py)."""
from .engine import Engine
from .HCCI import HCCIengine

__all__ = ["Engine", "HCCIengine"]
