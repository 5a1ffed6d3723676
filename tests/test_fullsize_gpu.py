"""Parity of the BENCHMARKED step itself: the product TrainStep at the bench's batch and volume,
eager and hipGraph-replayed, against the oracle (oracle/unet_oracle.py, the reference network as
plain aten CPU calls, trainer.py:222-232 + losses.py:30-54) on the box's CPU.

The golden fixtures pin whole-network gradients at bs 1-2; the schedules that depend on the batch
(the gradient-reduction item plan, whose partial lists grow with N; the 512-workgroup fused
backward grids; the IN-partial batching; the paired block-tail launches) are only exercised at the
benchmarked shape, so the bench step's own gradients are checked here:

  * BASELINE config 2: bs 4 x 48^3, 16 -> 128, fp32 (bench.py's `value`);
  * BASELINE config 5: bs 4 x 64^3, 32 -> 256, fp32 (bench.py's `config5`), one step.

Inputs are the bench's synthetic ones (x ~ U[0, 1), Bernoulli(0.03) targets), seed-42 weights
(the reference's init order), dropout 0 (Dropout3d draws are checked in test_model_gpu).
Tolerances, the rule of test_model_gpu.test_model_matches_reference_golden:
  * output |HIP - fp64 oracle| <= 1e-3 (north star), loss 1e-4 relative;
  * whole flat gradient relative L2 <= max(1e-3, 2 * e32) and every tensor's <= max(1e-2, 3 * e32),
    e32 = the same error of the fp32 CPU oracle (the reference's own fp32 arithmetic) against fp64
    on the same inputs (LeakyReLU kink flips: any fp32 implementation has them);
  * the graph-replayed step gives bitwise the eager step's loss, gradient and updated parameters.
"""
import numpy as np
import pytest
import torch

from oracle import unet_oracle as U

pytestmark = pytest.mark.gpu


def _batch(bs, size, seed=42):
    """bench.py's synthetic batch (x ~ U[0, 1), Bernoulli(0.03) targets)."""
    rng = np.random.default_rng(seed)
    x = rng.random((bs, 1, size, size, size), dtype=np.float32)
    t = (rng.random((bs, 1, size, size, size)) > 0.97).astype(np.float32)
    return torch.from_numpy(x), torch.from_numpy(t)


def _oracle(sd, x, t, dtype):
    """out, loss, {name: grad} of the oracle on the CPU in `dtype`."""
    P = {k: v.detach().clone().to(dtype).requires_grad_(True) for k, v in sd.items()}
    out = U.unet_forward(P, x.to(dtype))
    loss = U.focal_tversky(out, t.to(dtype))
    loss.backward()
    return out.detach().double().numpy(), float(loss.detach()), {k: p.grad.double().numpy() for k, p in P.items()}


def _errs(g, ref):
    errs, num, den = {}, 0.0, 0.0
    for k, r in ref.items():
        d = np.linalg.norm(g[k].astype(np.float64) - r)
        errs[k] = d / max(np.linalg.norm(r), 1e-30)
        num += d * d
        den += float(np.sum(r * r))
    return errs, (num / den) ** 0.5


def _grads(model, gflat):
    """the flat gradient split into the parameters (reference registration order)"""
    g = gflat.detach().cpu().double().numpy()
    return {k: g[o:o + n].reshape(shape) for k, (o, n, shape) in model.engine.offsets.items()}


def _step_vs_oracle(cuda, enc, bs, size):
    from light_unet.models.unet3d import Lightweight3DUNet
    from light_unet.train_step import TrainStep
    torch.manual_seed(42)
    model = Lightweight3DUNet(encoder_channels=list(enc), dropout_p=0.0)
    sd = {k: v.detach().clone() for k, v in model.state_dict().items()}
    x, t = _batch(bs, size)
    dx, dt = x.to(cuda), t.to(cuda)

    # eager product step (one process: the gradient reduction applies AdamW in the same launch)
    m = model.to(cuda).train()
    ts = TrainStep(m, lr=1e-4, weight_decay=1e-5)
    p, sv, sums = ts._fwd(dx, dt)
    ts._bwd(p, sv, dt, sums)
    torch.cuda.synchronize()
    assert m.engine.applied_update
    out = p.detach().cpu().double().numpy()
    loss = float(ts.loss.item())
    g_eager, p_eager = ts.gflat.clone(), ts.flat.clone()
    del p, sv, sums

    # the same step captured and replayed (the bench's form), from the same initial state
    m2 = Lightweight3DUNet(encoder_channels=list(enc), dropout_p=0.0)
    m2.load_state_dict(sd)
    m2 = m2.to(cuda).train()
    tg = TrainStep(m2, lr=1e-4, weight_decay=1e-5)
    xs, tsb = dx.clone(), dt.clone()
    tg.capture(xs, tsb)
    lg = float(tg.replay().item())
    torch.cuda.synchronize()
    assert lg == loss, (lg, loss)
    assert torch.equal(tg.gflat, g_eager), "graph-replayed gradient != eager"
    assert torch.equal(tg.flat, p_eager), "graph-replayed update != eager"
    grads = _grads(m, g_eager)
    del tg, m2, xs, tsb

    # the oracle: fp64 (the reference's math), fp32 (its own rounding) for the bound
    o64, l64, g64 = _oracle(sd, x, t, torch.float64)
    oerr = float(np.abs(out - o64).max())
    assert oerr <= 1e-3, oerr
    assert abs(loss - l64) <= 1e-4 * abs(l64), (loss, l64)
    errs, gerr = _errs(grads, g64)
    _, _, g32 = _oracle(sd, x, t, torch.float32)
    e32, ge32 = _errs(g32, g64)
    print(f"{enc} bs {bs} x {size}^3: out err {oerr:.2e}, loss {loss:.7f} vs {l64:.7f}, grad rel L2 "
          f"{gerr:.2e} (cpu fp32 {ge32:.2e}), worst tensor {max(errs.items(), key=lambda kv: kv[1])}")
    assert gerr <= max(1e-3, 2 * ge32), (gerr, ge32)
    bad = {k: (errs[k], e32[k]) for k in errs if errs[k] > max(1e-2, 3 * e32[k])}
    assert not bad, f"gradient errors above tolerance: {bad}"


@pytest.mark.timeout(300)
def test_config2_trainstep_bs4_48_matches_oracle(cuda):
    """BASELINE config 2, the bench's headline step: bs 4 x 48^3, 16 -> 32 -> 64 -> 128."""
    _step_vs_oracle(cuda, (16, 32, 64, 128), 4, 48)


@pytest.mark.timeout(600)
def test_config5_trainstep_bs4_64_matches_oracle(cuda):
    """BASELINE config 5: bs 4 x 64^3, 32 -> 64 -> 128 -> 256 (812,284 parameters), one step."""
    _step_vs_oracle(cuda, (32, 64, 128, 256), 4, 64)
