"""Drop-in host API (no GPU): same constructor, submodule tree, state_dict keys/shapes, default
initialisation and error behaviour as the reference light_unet.models (unet3d.py, losses.py)."""
import numpy as np
import pytest
import torch


def test_param_names_shapes_and_count(golden):
    from light_unet.models.unet3d import Lightweight3DUNet
    z = golden("model_b1_48.npz")
    m = Lightweight3DUNet()
    keys = [k[2:] for k in z.files if k.startswith("w/")]
    sd = m.state_dict()
    assert list(sd) == keys
    for k in keys:
        assert tuple(sd[k].shape) == z["w/" + k].shape
    assert m.count_parameters() == {"total": 217228, "trainable": 217228}
    m5 = Lightweight3DUNet(encoder_channels=[32, 64, 128, 256])
    assert m5.count_parameters()["total"] == 812284


def test_default_init_matches_reference_seed42(golden):
    """torch.manual_seed(42) (trainer.py:44) gives the reference's initial weights bit for bit
    (the goldens perturb only the InstanceNorm affine parameters)."""
    from light_unet.models.unet3d import Lightweight3DUNet
    z = golden("model_b2_32.npz")
    torch.manual_seed(42)
    m = Lightweight3DUNet(dropout_p=0.0)
    for k, v in m.state_dict().items():
        if ".norm" in k or ".shortcut.1." in k:
            continue
        assert np.array_equal(v.numpy(), z["w/" + k]), k


def test_parameters_are_views_of_one_flat_buffer():
    from light_unet.models.unet3d import Lightweight3DUNet
    m = Lightweight3DUNet()
    flat = m.flat_parameters()
    assert flat.numel() == 217228
    base = flat.data_ptr()
    for (name, p), (off, n, shape) in zip(m.named_parameters(), m._slices):
        assert p.data_ptr() == base + 4 * off and tuple(p.shape) == tuple(shape)
    # load_state_dict keeps the aliasing
    sd = {k: torch.randn_like(v) for k, v in m.state_dict().items()}
    m.load_state_dict(sd)
    assert m._is_flat()
    assert torch.equal(m.init_conv.conv1.depthwise.weight, sd["init_conv.conv1.depthwise.weight"])
    assert torch.equal(flat[:27], sd["init_conv.conv1.depthwise.weight"].reshape(-1))
    # dtype conversion re-flattens
    m.double()
    assert m._is_flat() and m.flat_parameters().dtype == torch.float64


def test_forward_on_cpu_fails_loudly():
    from light_unet import _native
    from light_unet.models.unet3d import Lightweight3DUNet
    m = Lightweight3DUNet()
    with pytest.raises(_native.NativeError):
        m(torch.zeros(1, 1, 48, 48, 48))


def test_unsupported_configs_raise():
    from light_unet.models.unet3d import Lightweight3DUNet
    with pytest.raises(NotImplementedError):
        Lightweight3DUNet(in_channels=2)


def test_loss_factory_and_errors():
    from light_unet.models import losses
    f = losses.get_loss_function({"name": "FocalTverskyLoss", "alpha": 0.7, "beta": 0.3, "gamma": 0.75})
    assert isinstance(f, losses.FocalTverskyLoss) and f.gamma == 0.75
    assert isinstance(losses.get_loss_function({"name": "DiceLoss"}), losses.DiceLoss)
    assert isinstance(losses.get_loss_function({"use_combined_loss": True}), losses.CombinedLoss)
    with pytest.raises(ValueError):
        losses.get_loss_function({"name": "Nope"})
    with pytest.raises(AssertionError):
        losses.FocalTverskyLoss(alpha=0.6, beta=0.3)
    with pytest.raises(Exception):
        f(torch.rand(1, 1, 4, 4, 4), torch.rand(1, 1, 4, 4, 4))   # CPU tensors: no fallback
    with pytest.raises(RuntimeError):
        f(torch.rand(1, 1, 4, 4, 8)[..., ::2], torch.rand(1, 1, 4, 4, 4))  # non-contiguous (view)


def test_engine_shapes_and_up_pad():
    from light_unet.engine import UNetEngine
    # ragged volumes (the UpBlock pad branch) and planes above 64x64 are accepted
    UNetEngine.check_shape(torch.zeros(1, 1, 44, 48, 48))
    UNetEngine.check_shape(torch.zeros(1, 1, 40, 44, 36))
    UNetEngine.check_shape(torch.zeros(1, 1, 8, 72, 72))
    UNetEngine.check_shape(torch.zeros(1, 1, 24, 80, 80))
    with pytest.raises(ValueError):
        UNetEngine.check_shape(torch.zeros(1, 2, 48, 48, 48))
    with pytest.raises(ValueError):       # three 2x poolings of 6 leave nothing
        UNetEngine.check_shape(torch.zeros(1, 1, 6, 48, 48))
    with pytest.raises(NotImplementedError):   # W % 4 != 0 with a plane above 4096 voxels
        UNetEngine.check_shape(torch.zeros(1, 1, 8, 100, 102))
    # F.pad offsets of unet3d.py:130-138: diff // 2 before
    assert UNetEngine.up_pad((5, 6, 6), (11, 12, 12)) == (0, 0, 0)
    assert UNetEngine.up_pad((5, 6, 6), (10, 12, 12)) is None
    assert UNetEngine.up_pad((4, 5, 2), (9, 11, 4)) == (0, 0, 0)


def test_sliding_window_host_pieces(golden):
    """importance map and window positions of the device sliding window == the reference's
    (fixture from utils.py:142-173 run by the reference); CPU device fails loudly."""
    import numpy as np
    import torch
    from light_unet import _native
    from light_unet.utils import _get_gaussian_importance_map, sliding_window_inference_3d, window_positions
    z = golden("sliding.npz")
    np.testing.assert_array_equal(_get_gaussian_importance_map((48, 48, 48)), z["importance_48"])
    assert window_positions(256, 48, 24) == list(range(0, 209, 24)) + [208]
    assert window_positions(144, 48, 24) == [0, 24, 48, 72, 96]
    assert window_positions(40, 48, 24) == [0]
    assert window_positions(49, 48, 24) == [0, 1]
    from light_unet.models.unet3d import Lightweight3DUNet
    with pytest.raises(ValueError):
        sliding_window_inference_3d(np.zeros((2, 3, 4, 5), np.float32), Lightweight3DUNet())
    with pytest.raises(_native.NativeError):
        sliding_window_inference_3d(np.zeros((48, 48, 48), np.float32), Lightweight3DUNet(),
                                    device=torch.device("cpu"))


@pytest.mark.parametrize("fname,kw", [
    ("model_g_b2_16.npz", dict(use_depthwise_separable=False, use_grouped=True, groups=8)),
    ("model_d_b1_16.npz", dict(use_depthwise_separable=False, use_grouped=False, groups=8))])
def test_variant_param_names_and_seed42_init(golden, fname, kw):
    """use_depthwise_separable=False: GroupedConv3d / dense nn.Conv3d blocks (unet3d.py:26-34,
    43-60) with the reference's keys, shapes, count and seed-42 initial weights."""
    from light_unet.models.unet3d import Lightweight3DUNet
    z = golden(fname)
    enc = [int(c) for c in z["enc"]]
    torch.manual_seed(42)
    m = Lightweight3DUNet(encoder_channels=enc, dropout_p=0.0, **kw)
    keys = [k[2:] for k in z.files if k.startswith("w/")]
    sd = m.state_dict()
    assert list(sd) == keys
    assert m.count_parameters()["total"] == int(z["n_params"])
    for k, v in sd.items():
        assert tuple(v.shape) == z["w/" + k].shape
        if ".norm" in k or ".shortcut.1." in k:
            continue
        assert np.array_equal(v.numpy(), z["w/" + k]), k
    full = Lightweight3DUNet(use_depthwise_separable=False)
    assert full.count_parameters()["total"] == 391521          # reference, groups=8
    dense = Lightweight3DUNet(use_depthwise_separable=False, use_grouped=False)
    assert dense.count_parameters()["total"] == 2308737


def test_variant_group_divisibility_error():
    """nn.Conv3d raises for channels not divisible by groups; so does the mirror."""
    from light_unet.models.unet3d import Lightweight3DUNet
    with pytest.raises(ValueError):
        Lightweight3DUNet(encoder_channels=[12, 20, 40, 80], use_depthwise_separable=False, groups=8)


def test_fused_update_needs_exact_cover():
    """l3u_reduce_segments_adamw is used only when the reduction items write every gradient
    element exactly once and none accumulates (engine._items_cover_once)."""
    from light_unet.engine import _items_cover_once
    it = lambda dst, ln, acc=0: (0, 1, 1, 1, ln, dst, acc, 0)   # noqa: E731
    assert _items_cover_once([it(0, 4), it(4, 6)], 10)
    assert not _items_cover_once([it(0, 4), it(5, 5)], 10)          # element 4 not produced
    assert not _items_cover_once([it(0, 6), it(4, 6)], 10)          # elements 4, 5 twice
    assert not _items_cover_once([it(0, 4), it(4, 6, acc=1)], 10)   # accumulating item
