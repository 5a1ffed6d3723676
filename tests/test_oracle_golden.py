"""Pins the CPU oracle (oracle/) to fixtures generated from the reference implementation.

The reference's own tests pin nothing on the hot path, so these goldens — produced by
tests/golden/make_goldens.py from /root/reference (imported by file path, fp64) — are the anchor.
The oracle is then the checker used by the GPU tests at sizes the fixtures do not cover.
"""
import numpy as np
import pytest
import torch

from oracle import sliding_oracle as S
from oracle import unet_oracle as U


def _sd(z, prefix="w/", dtype=torch.float64):
    return {k[len(prefix):]: torch.from_numpy(z[k]).to(dtype) for k in z.files if k.startswith(prefix)}


@pytest.mark.parametrize("fname", ["model_b2_32.npz", "model_b1_40_44_36.npz"])
def test_oracle_model_fp64_matches_reference(golden, fname):
    """model_b1_40_44_36: D, H, W not divisible by 8, so every UpBlock takes the pad branch
    (unet3d.py:130-138)."""
    z = golden(fname)
    sd = _sd(z)
    assert [k for k in sd] == [n for n, _ in U.param_names()]
    for n, shape in U.param_names():
        assert tuple(sd[n].shape) == shape
    assert sum(v.numel() for v in sd.values()) == int(z["n_params"]) == 217228
    params = {k: v.clone().requires_grad_(True) for k, v in sd.items()}
    out = U.unet_forward(params, torch.from_numpy(z["x"]).double())
    loss = U.focal_tversky(out, torch.from_numpy(z["target"]).double())
    loss.backward()
    assert np.abs(out.detach().numpy() - z["out"]).max() < 1e-6
    assert abs(loss.item() - float(z["loss"])) < 1e-9
    for k, p in params.items():
        g = z["g/" + k]
        assert np.abs(p.grad.numpy() - g).max() <= 1e-5 * max(np.abs(g).max(), 1e-12) + 1e-12, k


def test_oracle_param_count_config5(golden):
    z = golden("model_c32_b1_64.npz")
    names = U.param_names((32, 64, 128, 256))
    sd = _sd(z)
    assert [k for k in sd] == [n for n, _ in names]
    assert sum(v.numel() for v in sd.values()) == 812284


def test_oracle_blocks_match_reference(golden):
    z = golden("blocks.npz")
    cases = {"rb_a": "rb", "rb_id": "rb", "rb_c1": "rb", "down": "down", "up": "up"}
    for name, kind in cases.items():
        sd = {k[len(name) + 3:]: torch.from_numpy(z[k]).double() for k in z.files
              if k.startswith(name + "/w/")}
        ins = [torch.from_numpy(z[f"{name}/in{j}"]).double().requires_grad_(True)
               for j in range(2 if kind == "up" else 1)]
        if kind == "rb":
            out = U.residual_block(sd, "", ins[0])
        elif kind == "down":
            out = U.down_block(sd, "", ins[0])
        else:
            out = U.up_block(sd, "", ins[0], ins[1])
        out.backward(torch.from_numpy(z[f"{name}/dy"]).double())
        assert np.abs(out.detach().numpy() - z[f"{name}/out"]).max() < 1e-5, name
        for j, t in enumerate(ins):
            ref = z[f"{name}/din{j}"]
            assert np.abs(t.grad.numpy() - ref).max() <= 1e-5 * np.abs(ref).max(), (name, j)


VARIANTS = {"model_g_b2_16.npz": dict(use_depthwise_separable=False, use_grouped=True, groups=8),
            "model_d_b1_16.npz": dict(use_depthwise_separable=False, use_grouped=False, groups=8)}


@pytest.mark.parametrize("fname", sorted(VARIANTS))
def test_oracle_variant_models_match_reference(golden, fname):
    """use_depthwise_separable=False (GroupedConv3d / dense nn.Conv3d, unet3d.py:26-34,43-60)."""
    z = golden(fname)
    var = VARIANTS[fname]
    for k, v in var.items():
        assert z["variant/" + k].item() == v
    enc = tuple(int(c) for c in z["enc"])
    sd = _sd(z)
    names = U.param_names(enc, **var)
    assert [k for k in sd] == [n for n, _ in names]
    for n, shape in names:
        assert tuple(sd[n].shape) == shape
    assert sum(v.numel() for v in sd.values()) == int(z["n_params"])
    params = {k: v.clone().requires_grad_(True) for k, v in sd.items()}
    out = U.unet_forward(params, torch.from_numpy(z["x"]).double())
    loss = U.focal_tversky(out, torch.from_numpy(z["target"]).double())
    loss.backward()
    assert np.abs(out.detach().numpy() - z["out"]).max() < 1e-6
    assert abs(loss.item() - float(z["loss"])) < 1e-9
    for k, p in params.items():
        g = z["g/" + k]
        assert np.abs(p.grad.numpy() - g).max() <= 1e-5 * max(np.abs(g).max(), 1e-12) + 1e-12, k


def test_oracle_variant_blocks_match_reference(golden):
    z = golden("blocks_g.npz")
    cases = {"g_rb": "rb", "g_rb_id": "rb", "g_rb_mixed": "rb", "d_rb": "rb", "g_up": "up"}
    for name, kind in cases.items():
        sd = {k[len(name) + 3:]: torch.from_numpy(z[k]).double() for k in z.files
              if k.startswith(name + "/w/")}
        ins = [torch.from_numpy(z[f"{name}/in{j}"]).double().requires_grad_(True)
               for j in range(2 if kind == "up" else 1)]
        out = U.residual_block(sd, "", ins[0]) if kind == "rb" else U.up_block(sd, "", ins[0], ins[1])
        out.backward(torch.from_numpy(z[f"{name}/dy"]).double())
        assert np.abs(out.detach().numpy() - z[f"{name}/out"]).max() < 1e-5, name
        for j, t in enumerate(ins):
            ref = z[f"{name}/din{j}"]
            assert np.abs(t.grad.numpy() - ref).max() <= 1e-5 * np.abs(ref).max(), (name, j)


def test_oracle_ftl_and_closed_form(golden):
    z = golden("ftl.npz")
    for case in ("rand", "empty", "full", "sat", "params"):
        a, b, g = (float(v) for v in z[f"{case}/abg"])
        p = torch.from_numpy(z[f"{case}/pred"]).double().requires_grad_(True)
        t = torch.from_numpy(z[f"{case}/target"]).double()
        loss = U.focal_tversky(p, t, a, b, g)
        loss.backward()
        assert abs(loss.item() - float(z[f"{case}/loss"])) < 1e-12, case
        np.testing.assert_allclose(p.grad.numpy(), z[f"{case}/dpred"], rtol=1e-9, atol=1e-15)
        cf = U.ftl_grad_closed_form(p.detach(), t, a, b, g)
        np.testing.assert_allclose(cf.numpy(), z[f"{case}/dpred"], rtol=1e-9, atol=1e-15)
    assert int(z["err/assert_ab"]) == 1 and int(z["err/unknown"]) == 1
    with pytest.raises(AssertionError):
        U.focal_tversky(torch.ones(2), torch.ones(2), alpha=0.6, beta=0.3)


def test_oracle_sliding_window_matches_reference(golden):
    z = golden("sliding.npz")
    np.testing.assert_array_equal(S.gaussian_importance_map((48, 48, 48)), z["importance_48"])
    sd = _sd(z, dtype=torch.float32)

    def fwd(a):
        with torch.no_grad():
            return U.unet_forward(sd, torch.from_numpy(a)).numpy()

    for name in ("v64_56_72", "v40_52_48"):
        prob = S.sliding_window(z[f"{name}/image"], fwd)
        np.testing.assert_allclose(prob, z[f"{name}/prob"], atol=1e-6)
        for thr in (0.1, 0.3, 0.5, 0.7):
            m = prob >= thr
            far = np.abs(z[f"{name}/prob"] - thr) > 1e-4
            assert np.array_equal(m[far], z[f"{name}/mask_{thr}"][far])


def test_window_positions_edge_cases():
    assert S.window_positions(256, 48, 24) == list(range(0, 209, 24)) + [208]
    assert len(S.window_positions(256, 48, 24)) == 10
    assert S.window_positions(144, 48, 24) == [0, 24, 48, 72, 96]
    assert S.window_positions(40, 48, 24) == [0]          # smaller than the patch -> pad
    assert S.window_positions(48, 48, 24) == [0]
    assert S.window_positions(50, 48, 24) == [0, 2]
    with pytest.raises(ValueError):
        S.sliding_window(np.zeros((4, 4)), lambda a: a)


def test_cpu_baseline_equivalence_recorded():
    """the oracle step (bench.py's cpu_baseline leg) was timed against the
    reference's own model on the same cores and inputs (tests/fixtures/make_cpu_ratio.py);
    the record holds outputs within 1e-3 and a time ratio near 1, so the CPU baseline is the
    reference's speed, not a slower restatement's."""
    import json
    import os
    with open(os.path.join(os.path.dirname(__file__), "fixtures", "cpu_ratio.json")) as f:
        rec = json.load(f)
    assert rec["parity_dropout0"]["max_abs_out"] <= 1e-3
    assert rec["parity_dropout0"]["grad_rel_l2"] <= 1e-3
    assert 0.8 <= rec["ratio_oracle_over_reference"] <= 1.25
    assert "p=0.1" in rec["workload"] and rec["cpu_model"]
