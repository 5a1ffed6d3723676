"""Models package (reference: light_unet/models/__init__.py).

Exports the hot-path model and losses.  The reference's models/__init__ also re-exports the
NIfTI datasets and host metrics (models/__init__.py:8-24); those are outside the MI355X hot-path
scope and are not part of this package.
"""
from .unet3d import Lightweight3DUNet
from .losses import FocalTverskyLoss, CombinedLoss, DiceLoss, get_loss_function

__all__ = [
    "Lightweight3DUNet",
    "FocalTverskyLoss",
    "CombinedLoss",
    "DiceLoss",
    "get_loss_function",
]
