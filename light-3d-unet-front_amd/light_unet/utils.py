"""Whole-volume sliding-window inference on the device (drop-in for the reference's
light_unet/utils.py:11-173; imported by trainer.py:19 and inferencer.py).

Same signature, arguments, errors and result (a float32 numpy prob map [D, H, W]) as the
reference, but instead of one bs=1 forward and two host round trips per window:
  * the volume is uploaded once and windows are cut out on the device in batches
    (l3u_window_gather, zero padding past the edge as utils.py:96-113);
  * each batch runs the network forward as one replayed hipGraph (Lightweight3DUNet engine);
  * the predictions of all windows stay in HBM and one l3u_window_blend launch forms
    sum(pred * importance) / sum(importance) per voxel in the reference's window order with the
    same float32 operations (utils.py:125-135).
A model that is not this package's Lightweight3DUNet is called eagerly per batch (same device
gather / blend).  There is no CPU path: the volume is processed on `device`.
"""
from typing import Tuple

import numpy as np
import torch

from . import _native as nat


def _get_gaussian_importance_map(patch_size: Tuple[int, int, int]) -> np.ndarray:
    """utils.py:142-173: outer product of 1-D Gaussians (center L/2, sigma L/6), max 1, fp32."""
    def gaussian_1d(length):
        center = length / 2.0
        sigma = length / 6.0
        x = np.arange(length)
        return np.exp(-((x - center) ** 2) / (2 * sigma ** 2))

    m = np.einsum("i,j,k->ijk", gaussian_1d(patch_size[0]), gaussian_1d(patch_size[1]),
                  gaussian_1d(patch_size[2]))
    m = m / m.max()
    return m.astype(np.float32)


def window_positions(size: int, patch: int, stride: int):
    """Window starts along one axis (utils.py:64-82)."""
    pos = list(range(0, max(0, size - patch + 1), stride)) if size >= patch else []
    if size > patch and (len(pos) == 0 or pos[-1] + patch < size):
        pos.append(size - patch)
    return pos or [0]


class _GraphForward:
    """Forward of a fixed batch of windows as one replayed graph: gather -> network."""

    def __init__(self, model, vol, D, H, W, patch, batch, device):
        self.model, self.vol, self.dims, self.patch, self.batch = model, vol, (D, H, W), patch, batch
        self.pos = torch.zeros(batch, 3, dtype=torch.int32, device=device)
        self.x = torch.empty(batch, 1, *patch, device=device)
        self.engine = getattr(model, "engine", None)
        self.graph = None
        if self.engine is not None:
            flat = model.flat_parameters()
            side = torch.cuda.Stream(device=device)
            side.wait_stream(torch.cuda.current_stream(device))
            with torch.cuda.stream(side):
                self._run(flat)
            torch.cuda.current_stream(device).wait_stream(side)
            self.graph = torch.cuda.CUDAGraph()
            with torch.cuda.graph(self.graph):
                self.out = self._run(flat)

    def _gather(self):
        D, H, W = self.dims
        nat.call("l3u_window_gather", self.vol.data_ptr(), D, H, W, self.pos.data_ptr(), self.batch,
                 *self.patch, self.x.data_ptr(), nat.stream())

    def _run(self, flat):
        self._gather()
        p, _ = self.engine.forward(flat, self.x, training=False, save=False)
        return p

    def __call__(self):
        if self.graph is not None:
            self.graph.replay()
            return self.out
        self._gather()
        return self.model(self.x)


def sliding_window_inference_3d(image: np.ndarray, model: torch.nn.Module,
                                patch_size: Tuple[int, int, int] = (48, 48, 48),
                                overlap: float = 0.5, device: torch.device = None,
                                use_gaussian: bool = True, window_batch: int = 16,
                                group=None) -> np.ndarray:
    """utils.py:11-139.  `window_batch` windows run per forward (extra keyword; the result
    does not depend on it).

    `group` (extra keyword): a torch.distributed process group whose ranks (one
    per GPU, every rank calling with the same image and weights) split the window batches
    round-robin.  Each rank blends only its own windows' predictions (the others count as
    zero; the denominator sum(importance) is the full one everywhere), and one all_reduce(SUM)
    of the [D, H, W] map (RCCL over xGMI) adds the shares: the result equals the one-GPU map
    up to the order of the fp32 additions."""
    if device is None:
        device = next(model.parameters()).device
    device = torch.device(device)
    if len(image.shape) == 4 and image.shape[0] == 1:
        image = image[0]
    if len(image.shape) != 3:
        raise ValueError(f"Expected 3D image [D, H, W], got shape {image.shape}")
    nat.require_device(torch.empty(0, device=device))
    d, h, w = image.shape
    pd, ph, pw = patch_size
    zs = window_positions(d, pd, max(1, int(pd * (1 - overlap))))
    ys = window_positions(h, ph, max(1, int(ph * (1 - overlap))))
    xs = window_positions(w, pw, max(1, int(pw * (1 - overlap))))
    imp = (_get_gaussian_importance_map(patch_size) if use_gaussian
           else np.ones(patch_size, dtype=np.float32))
    order = [(z, y, x) for z in zs for y in ys for x in xs]   # the reference's loop order
    nwin = len(order)
    B = max(1, min(int(window_batch), nwin))
    P = pd * ph * pw

    was_training = model.training
    model.eval()
    try:
        with torch.no_grad():
            vol = torch.from_numpy(np.ascontiguousarray(image, dtype=np.float32)).to(device)
            pos_all = torch.tensor(order + [order[-1]] * ((-nwin) % B), dtype=torch.int32,
                                   device=device)
            world, rank = 1, 0
            if group is not None:
                import torch.distributed as dist
                world, rank = dist.get_world_size(group), dist.get_rank(group)
            preds = (torch.zeros if world > 1 else torch.empty)(pos_all.shape[0], P, device=device)
            fwd = _GraphForward(model, vol, d, h, w, (pd, ph, pw), B, device)
            for bi, b0 in enumerate(range(0, nwin, B)):
                if bi % world != rank:   # another rank's batch
                    continue
                fwd.pos.copy_(pos_all[b0:b0 + B])
                out = fwd()
                if out.dim() != 5 or tuple(out.shape[2:]) != (pd, ph, pw):
                    raise ValueError(f"Expected 3D model output, got shape {tuple(out.shape)}")
                preds[b0:b0 + B].copy_(out.reshape(B, P))
            zt, yt, xt = (torch.tensor(v, dtype=torch.int32, device=device) for v in (zs, ys, xs))
            impt = torch.from_numpy(imp).to(device)
            prob = torch.empty(d, h, w, device=device)
            nat.call("l3u_window_blend", preds.data_ptr(), zt.data_ptr(), len(zs), yt.data_ptr(),
                     len(ys), xt.data_ptr(), len(xs), impt.data_ptr(), d, h, w, pd, ph, pw,
                     prob.data_ptr(), nat.stream())
            if world > 1:
                dist.all_reduce(prob, op=dist.ReduceOp.SUM, group=group)
            return prob.cpu().numpy()
    finally:
        model.train(was_training)
