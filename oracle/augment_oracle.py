"""numpy restatement of the reference's training-patch sampling and augmentation (TEST
INFRASTRUCTURE — see oracle/__init__).  Checker for light_unet/patches.py (HIP kernel
csrc/augment.hip).

Follows light_unet/datasets/patch_dataset.py:
  _extract_patch   :136-154  crop centred at `center` (start = max(0, c - p//2)), zero pad at the end
  _augment         :156-220  flip (np.flip), rotation (scipy.ndimage.rotate, reshape=False,
                             order 1 image / 0 label, mode 'constant', cval 0), scale
                             (scipy.ndimage.zoom, order 1 / 0, mode 'constant', then centre crop /
                             end pad back to the patch), intensity shift + clip to [0, 1], gaussian
                             noise + clip
The interpolation is restated from scipy 1.15's ndimage (the reference's dependency; the call
sites above): rotate applies, in every plane parallel to the (sorted) axes pair, the affine map
in = R @ out + (c_in - R @ c_out) with R = [[cos, sin], [-sin, cos]] (degrees, cosdg/sindg) and
c = (shape - 1) / 2; zoom maps out -> in = out * (in_len - 1) / (out_len - 1) per axis with
out_len = round(in_len * scale).  Mode 'constant': a sample whose coordinate leaves [0, len - 1]
on any axis is cval; order 1 = (bi/tri)linear with weights (1 - t, t) accumulated in C order in
float64; order 0 = floor(coordinate + 0.5).  Pinned against scipy.ndimage itself in
tests/test_augment_oracle.py.
"""
import numpy as np


def _interp(vol, coords, order):
    """Sample vol (float64 math) at coords [ndim, ...] with mode 'constant' (cval 0)."""
    shp = np.array(vol.shape)
    inside = np.ones(coords.shape[1:], bool)
    for d in range(vol.ndim):
        inside &= (coords[d] >= 0) & (coords[d] <= shp[d] - 1)
    out = np.zeros(coords.shape[1:], np.float64)
    if order == 0:
        idx = tuple(np.clip(np.floor(coords[d] + 0.5).astype(np.int64), 0, shp[d] - 1)
                    for d in range(vol.ndim))
        out = vol[idx].astype(np.float64)
    else:
        fl = [np.floor(coords[d]) for d in range(vol.ndim)]
        t = [coords[d] - fl[d] for d in range(vol.ndim)]
        lo = [np.clip(fl[d].astype(np.int64), 0, shp[d] - 1) for d in range(vol.ndim)]
        hi = [np.clip(fl[d].astype(np.int64) + 1, 0, shp[d] - 1) for d in range(vol.ndim)]
        nd = vol.ndim
        for corner in range(1 << nd):          # C order: the first axis varies slowest
            w = None
            idx = []
            for d in range(nd):
                bit = (corner >> (nd - 1 - d)) & 1
                wd = t[d] if bit else 1.0 - t[d]
                w = wd if w is None else w * wd
                idx.append(hi[d] if bit else lo[d])
            out = out + w * vol[tuple(idx)].astype(np.float64)
    return np.where(inside, out, 0.0)


def rotate(vol, angle, axes, order):
    """scipy.ndimage.rotate(vol, angle, axes, reshape=False, order, mode='constant', cval=0)."""
    a0, a1 = sorted(axes)
    rad = np.deg2rad(angle)
    c, s = _cosdg(angle), _sindg(angle)
    del rad
    shp = np.array(vol.shape, np.float64)
    ic = (shp[[a0, a1]] - 1) / 2
    oc = np.array([c * ic[0] + s * ic[1], -s * ic[0] + c * ic[1]])
    off = ic - oc
    grid = np.indices(vol.shape).astype(np.float64)
    coords = grid.copy()
    coords[a0] = off[0] + c * grid[a0] + s * grid[a1]
    coords[a1] = off[1] + (-s) * grid[a0] + c * grid[a1]
    # per plane: the in-plane axes interpolate, the other axis is an exact integer index
    return _interp(vol, coords, order).astype(vol.dtype)


def _cosdg(a):
    return float(np.cos(np.deg2rad(a))) if a % 90 else [1.0, 0.0, -1.0, 0.0][int(a // 90) % 4]


def _sindg(a):
    return float(np.sin(np.deg2rad(a))) if a % 90 else [0.0, 1.0, 0.0, -1.0][int(a // 90) % 4]


def zoom_shape(shape, scale):
    return tuple(int(round(n * scale)) for n in shape)


def zoom(vol, scale, order):
    """scipy.ndimage.zoom(vol, scale, order, mode='constant', cval=0) (grid_mode=False)."""
    out_shape = zoom_shape(vol.shape, scale)
    f = [(i - 1) / (o - 1) if o != 1 else 1.0 for i, o in zip(vol.shape, out_shape)]
    grid = np.indices(out_shape).astype(np.float64)
    coords = np.stack([grid[d] * f[d] for d in range(vol.ndim)])
    return _interp(vol, coords, order).astype(vol.dtype)


def extract_patch(image, label, center, patch):
    pz, py, px = patch
    z, y, x = center
    zs, ys, xs = max(0, z - pz // 2), max(0, y - py // 2), max(0, x - px // 2)
    ze, ye, xe = min(image.shape[0], zs + pz), min(image.shape[1], ys + py), min(image.shape[2], xs + px)
    ip, lp = image[zs:ze, ys:ye, xs:xe], label[zs:ze, ys:ye, xs:xe]
    pad = [(0, pz - ip.shape[0]), (0, py - ip.shape[1]), (0, px - ip.shape[2])]
    return np.pad(ip, pad), np.pad(lp, pad)


def fit(vol, patch):
    """The scale branch's centre crop / end pad back to the patch (patch_dataset.py:183-206)."""
    for d, p in enumerate(patch):
        if vol.shape[d] > p:
            st = (vol.shape[d] - p) // 2
            vol = np.take(vol, np.arange(st, st + p), axis=d)
    pad = [(0, max(0, p - s)) for p, s in zip(patch, vol.shape)]
    return np.pad(vol, pad)


def augment(image, label, params, patch):
    """Apply a drawn parameter set (light_unet.patches.AugParams fields) in the reference order."""
    if params.flip_axis >= 0:
        image, label = np.flip(image, params.flip_axis).copy(), np.flip(label, params.flip_axis).copy()
    if params.rot_axes is not None:
        image = rotate(image, params.angle, params.rot_axes, 1)
        label = rotate(label, params.angle, params.rot_axes, 0)
    if params.scale is not None:
        image = zoom(image, params.scale, 1)
        label = zoom(label, params.scale, 0)
        if image.shape != tuple(patch):
            image, label = fit(image, patch), fit(label, patch)
    if params.shift is not None:
        image = np.clip(image + params.shift, 0, 1)
    if params.noise is not None:
        image = np.clip(image + params.noise, 0, 1)
    return image, label
