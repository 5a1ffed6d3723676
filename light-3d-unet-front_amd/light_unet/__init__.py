"""light_unet — MI355X (gfx950) hot path of Light-3D-U-Net, drop-in for the reference package.

Mirrors the reference import paths used by its Trainer / Inferencer:
    from light_unet.models.unet3d import Lightweight3DUNet       (trainer.py:16, inferencer.py:13)
    from light_unet.models.losses import get_loss_function        (trainer.py:17)
    from light_unet.utils import sliding_window_inference_3d      (trainer.py:19)
To bind this build into the reference package, see l3u_plugin.py.
Compute runs in lib/libl3u_hip.so (include/l3u.h); see DESIGN.md.
"""
__version__ = "0.1.0"
