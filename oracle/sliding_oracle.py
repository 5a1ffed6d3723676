"""numpy restatement of the reference sliding-window inference (TEST INFRASTRUCTURE — see oracle/__init__).

Follows light_unet/utils.py:
  stride = max(1, int(p * (1 - overlap)))                     utils.py:47-49
  positions = range(0, L - p + 1, stride) (+ [L - p] if the tail is uncovered), [0] if L < p
                                                              utils.py:59-81
  per window: crop, zero-pad to p if the volume is smaller, bs=1 forward, un-pad, accumulate
  pred * w and w in fp32 numpy                                utils.py:86-134
  prob /= count where count > 0                               utils.py:137
  importance map: outer product of exp(-(x - L/2)^2 / (2 (L/6)^2)), x = 0..L-1, / max
                                                              utils.py:142-173
`forward` is any callable taking a [1,1,pd,ph,pw] float32 numpy array and returning the same shape.
"""
import numpy as np


def gaussian_importance_map(patch_size):
    gs = []
    for length in patch_size:
        center = length / 2.0
        sigma = length / 6.0
        x = np.arange(length)
        gs.append(np.exp(-((x - center) ** 2) / (2 * sigma ** 2)))
    m = np.einsum("i,j,k->ijk", *gs)
    m = m / m.max()
    return m.astype(np.float32)


def window_positions(length, patch, stride):
    pos = list(range(0, max(0, length - patch + 1), stride)) if length >= patch else []
    if length > patch and (len(pos) == 0 or pos[-1] + patch < length):
        pos.append(length - patch)
    return pos or [0]


def sliding_window(image, forward, patch_size=(48, 48, 48), overlap=0.5, use_gaussian=True):
    if image.ndim == 4 and image.shape[0] == 1:
        image = image[0]
    if image.ndim != 3:
        raise ValueError(f"Expected 3D image [D, H, W], got shape {image.shape}")
    d, h, w = image.shape
    pd, ph, pw = patch_size
    strides = [max(1, int(p * (1 - overlap))) for p in patch_size]
    imp = gaussian_importance_map(patch_size) if use_gaussian else np.ones(patch_size, np.float32)
    prob = np.zeros((d, h, w), np.float32)
    cnt = np.zeros((d, h, w), np.float32)
    for z in window_positions(d, pd, strides[0]):
        for y in window_positions(h, ph, strides[1]):
            for x in window_positions(w, pw, strides[2]):
                ze, ye, xe = min(z + pd, d), min(y + ph, h), min(x + pw, w)
                patch = image[z:ze, y:ye, x:xe]
                ad, ah, aw = patch.shape
                if patch.shape != tuple(patch_size):
                    patch = np.pad(patch, ((0, pd - ad), (0, ph - ah), (0, pw - aw)))
                pred = np.asarray(forward(patch[None, None].astype(np.float32))).reshape(patch_size)
                pred = pred[:ad, :ah, :aw]
                wgt = imp[:ad, :ah, :aw]
                prob[z:ze, y:ye, x:xe] += pred * wgt
                cnt[z:ze, y:ye, x:xe] += wgt
    return np.divide(prob, cnt, where=cnt > 0, out=prob)
