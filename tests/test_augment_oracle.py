"""Pins oracle/augment_oracle.py's restatement of the augmentation interpolation to scipy.ndimage
itself (the reference's dependency at patch_dataset.py:11,173-181; scipy 1.15.3 in this image)."""
import numpy as np
import pytest
from scipy import ndimage

from oracle import augment_oracle as A


@pytest.mark.parametrize("angle,axes", [(7.3, (0, 1)), (-13.9, (0, 2)), (11.0, (1, 2)), (0.0, (0, 1)),
                                        (-15.0, (1, 2)), (90.0, (0, 2))])
def test_rotate_matches_scipy(angle, axes):
    rng = np.random.default_rng(1)
    img = rng.random((20, 18, 22), dtype=np.float32)
    lab = (rng.random((20, 18, 22)) > 0.7).astype(np.float32)
    r1 = ndimage.rotate(img, angle, axes=list(axes), reshape=False, order=1, mode="constant", cval=0)
    r0 = ndimage.rotate(lab, angle, axes=list(axes), reshape=False, order=0, mode="constant", cval=0)
    o1, o0 = A.rotate(img, angle, axes, 1), A.rotate(lab, angle, axes, 0)
    assert o1.dtype == r1.dtype and o1.shape == r1.shape
    np.testing.assert_allclose(o1, r1, rtol=0, atol=2e-7)
    assert (o0 != r0).sum() <= 2          # nearest-neighbour ties at exact .5 coordinates


@pytest.mark.parametrize("scale", [0.9, 0.93, 1.0, 1.04, 1.1])
def test_zoom_matches_scipy(scale):
    rng = np.random.default_rng(2)
    img = rng.random((24, 20, 26), dtype=np.float32)
    lab = (rng.random((24, 20, 26)) > 0.7).astype(np.float32)
    z1 = ndimage.zoom(img, scale, order=1, mode="constant", cval=0)
    z0 = ndimage.zoom(lab, scale, order=0, mode="constant", cval=0)
    o1, o0 = A.zoom(img, scale, 1), A.zoom(lab, scale, 0)
    assert o1.shape == z1.shape == A.zoom_shape(img.shape, scale)
    np.testing.assert_allclose(o1, z1, rtol=0, atol=2e-7)
    assert (o0 != z0).sum() <= 2
