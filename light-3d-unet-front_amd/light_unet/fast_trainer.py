"""The reference Trainer's training loops on the graph-replayed TrainStep.

`l3u_plugin.install(fast_step=True)` binds `train_epoch` and `train_epoch_step_based` below onto
the reference `light_unet.core.trainer.Trainer` (as `train_epoch` / `_train_epoch_step_based`,
trainer.py:208-258 / :260-347).  They keep the reference loops' meaning:

  * the same batches in the same order (the reference DataLoaders are iterated unchanged; the
    step-based mode runs every FL batch, then round(fl_batches * dlbcl_steps_ratio) DLBCL steps
    (or `dlbcl_steps`), re-iterating the DLBCL loader when it runs out, trainer.py:262-269,
    :301-312);
  * the same update: forward -> FocalTversky -> backward -> AdamW(lr, weight_decay, betas, eps of
    the Trainer's torch optimizer), with the learning rate read from that optimizer at the start
    of every epoch, so the Trainer's CosineAnnealingLR / ReduceLROnPlateau steps (trainer.py:
    532-542) drive it;
  * the same TensorBoard scalars at the same global steps (Loss/train_step, Loss/fl_step,
    Loss/dlbcl_step, Domain/*, Loss/fl_avg|dlbcl_avg|combined) and the same return value.

What changes is how a step runs: each batch is copied into the static input buffers of a
hipGraph-captured TrainStep and the graph is replayed (forward, loss, backward and the update
in one replay; with torch.distributed initialised, the FocalTversky sums and the flat gradient
are all-reduced over RCCL between the graph segments, exchange.py).  Per-step losses stay on the
device and are read ONCE per epoch (the reference syncs on loss.item() every step,
trainer.py:234, :293, :323).  A batch whose shape differs from the captured one (a ragged last
batch) runs the same step eagerly.

The torch optimizer is not stepped; its per-parameter state is kept as views of the flat AdamW
state (exp_avg / exp_avg_sq, and `step`), refreshed at the end of every epoch, so
`optimizer.state_dict()` in the Trainer's checkpoints (trainer.py:447-470) holds the real
moments.  Losses other than FocalTversky (CombinedLoss, DiceLoss: not enabled by any shipped
config) fall back to the reference loop.
"""
import torch

from .models.losses import FocalTverskyLoss
from .train_step import TrainStep

_FALLBACK = "_l3u_reference_loops"


class FastLoop:
    """Per-Trainer state: one TrainStep on the model's flat buffers, its captured graph, and the
    device-side loss history of the running epoch."""

    def __init__(self, trainer, group=None, ftl_mode="exact"):
        model, opt = trainer.model, trainer.optimizer
        crit = trainer.criterion
        pg = opt.param_groups[0]
        self.step = TrainStep(model, {"alpha": crit.alpha, "beta": crit.beta, "gamma": crit.gamma,
                                      "smooth": crit.smooth},
                              lr=pg["lr"], weight_decay=pg["weight_decay"], betas=pg["betas"],
                              eps=pg["eps"], group=group, ftl_mode=ftl_mode)
        if self.step.world > 1:   # identical initial weights on every rank (DDP semantics)
            import torch.distributed as dist
            dist.broadcast(self.step.flat, 0, group=group)
        self._load_torch_state(opt)
        self.shape = None
        self.xs = self.ts = None
        self.hist = None
        self.n = 0

    # ------------------------------------------------------------ optimizer state mirroring
    def _params(self, opt):
        return [p for g in opt.param_groups for p in g["params"]]

    def _load_torch_state(self, opt):
        """Continue from the torch optimizer's moments if it has any (e.g. a resumed run)."""
        st, model = self.step.opt, self.step.model
        slices = dict(zip([id(p) for p in model.parameters()], model._slices))
        steps = set()
        for p in self._params(opt):
            s = opt.state.get(p)
            if not s or "exp_avg" not in s:
                continue
            off, n, _ = slices[id(p)]
            st.m[off:off + n].copy_(s["exp_avg"].reshape(-1))
            st.v[off:off + n].copy_(s["exp_avg_sq"].reshape(-1))
            steps.add(int(float(s["step"])))
        if len(steps) > 1:
            raise ValueError(f"parameters of the torch optimizer are at different steps {steps}")
        if steps:
            st.step_t.fill_(steps.pop())

    def export_torch_state(self, opt):
        """Make opt.state the flat AdamW state (views; `step` as torch.optim.AdamW stores it)."""
        st, model = self.step.opt, self.step.model
        t = float(st.step_t.item())
        slices = dict(zip([id(p) for p in model.parameters()], model._slices))
        for p in self._params(opt):
            off, n, shape = slices[id(p)]
            opt.state[p] = {"step": torch.tensor(t, dtype=torch.float32),
                            "exp_avg": st.m[off:off + n].view(shape),
                            "exp_avg_sq": st.v[off:off + n].view(shape)}

    # ------------------------------------------------------------ steps
    def begin_epoch(self, lr, n_steps):
        self.step.opt.set_lr(lr)
        dev = self.step.flat.device
        self.hist = torch.zeros(max(int(n_steps), 1), dtype=torch.float32, device=dev)
        self.n = 0

    def run(self, images, labels):
        """One training step on a host (or device) batch; the loss stays on the device."""
        dev = self.step.flat.device
        x = images.float()
        t = labels.float()
        if tuple(x.shape) != tuple(t.shape):
            raise ValueError(f"images {tuple(x.shape)} and labels {tuple(t.shape)} differ")
        if self.shape is None:
            self.shape = tuple(x.shape)
            self.xs = torch.empty(self.shape, dtype=torch.float32, device=dev)
            self.ts = torch.empty(self.shape, dtype=torch.float32, device=dev)
            self.xs.copy_(x)
            self.ts.copy_(t)
            self.step.capture(self.xs, self.ts)   # side-effect free (TrainStep.capture)
        if tuple(x.shape) == self.shape:
            self.xs.copy_(x, non_blocking=True)
            self.ts.copy_(t, non_blocking=True)
            loss = self.step.replay()
        else:
            loss = self.step(x.to(dev).contiguous(), t.to(dev).contiguous())
        if self.n >= self.hist.numel():   # more steps than announced: grow (rare)
            self.hist = torch.cat([self.hist, torch.zeros_like(self.hist)])
        self.hist[self.n:self.n + 1].copy_(loss.reshape(1))
        self.n += 1

    def losses(self):
        """The epoch's per-step losses (one device->host copy)."""
        return self.hist[:self.n].double().cpu().tolist()


def _loop(self):
    fl = getattr(self, "_l3u_fast", None)
    if fl is None:
        fl = FastLoop(self, ftl_mode=getattr(self, "l3u_ftl_mode", "exact"))
        self._l3u_fast = fl
    return fl


def _usable(self):
    return type(self.criterion) is FocalTverskyLoss and getattr(self.criterion, "reduce_hook", None) is None


def _tqdm(it, **kw):
    try:
        from tqdm import tqdm
        return tqdm(it, **kw)
    except ImportError:
        return it


def train_epoch(self, epoch):
    """Trainer.train_epoch (trainer.py:208-258) on the graph-replayed step."""
    self.model.train()
    if self.use_step_based_mixed:
        return self._train_epoch_step_based(epoch)
    if not _usable(self):
        return getattr(type(self), _FALLBACK)["train_epoch"](self, epoch)
    if self.use_mixed_training and self.train_dataset is not None:
        self.train_dataset.reset_sample_counts()
    fl = _loop(self)
    nb = len(self.train_loader)
    fl.begin_epoch(self.optimizer.param_groups[0]["lr"], nb)
    for images, labels in _tqdm(self.train_loader, desc=f"Epoch {epoch+1} [Train]"):
        fl.run(images, labels)
    losses = fl.losses()
    fl.export_torch_state(self.optimizer)
    for i, v in enumerate(losses):
        self.writer.add_scalar("Loss/train_step", v, epoch * nb + i)
    avg = sum(losses) / len(losses)
    if self.use_mixed_training and self.train_dataset is not None:
        c = self.train_dataset.get_sample_counts()
        if c["total_samples"] > 0:
            self.writer.add_scalar("Domain/fl_samples", c["fl_samples"], epoch)
            self.writer.add_scalar("Domain/dlbcl_samples", c["dlbcl_samples"], epoch)
            self.writer.add_scalar("Domain/fl_ratio", c["fl_samples"] / c["total_samples"], epoch)
            self.writer.add_scalar("Domain/dlbcl_ratio", c["dlbcl_samples"] / c["total_samples"],
                                   epoch)
    return avg


def dlbcl_step_count(config, fl_batches):
    """trainer.py:262-269: the explicit `dlbcl_steps`, else round(fl_batches * ratio)."""
    mixed = config.get("training", {}).get("mixed_domains", {})
    override = mixed.get("dlbcl_steps", None)
    if override is not None:
        return int(override)
    return round(fl_batches * mixed.get("dlbcl_steps_ratio", 0.0))


def train_epoch_step_based(self, epoch):
    """Trainer._train_epoch_step_based (trainer.py:260-347) on the graph-replayed step."""
    if not _usable(self):
        return getattr(type(self), _FALLBACK)["_train_epoch_step_based"](self, epoch)
    fl_batches = len(self.fl_loader)
    dlbcl_steps = dlbcl_step_count(self.config, fl_batches)
    base = epoch * (fl_batches + dlbcl_steps)
    fl = _loop(self)
    fl.begin_epoch(self.optimizer.param_groups[0]["lr"], fl_batches + max(dlbcl_steps, 0))
    for images, labels in _tqdm(self.fl_loader, desc=f"Epoch {epoch+1} [FL]", position=0):
        fl.run(images, labels)
    fl_steps = fl.n
    if dlbcl_steps > 0:
        it = iter(self.dlbcl_loader)
        for _ in _tqdm(range(dlbcl_steps), desc=f"Epoch {epoch+1} [DLBCL]", position=0):
            try:
                images, labels = next(it)
            except StopIteration:        # re-iterate the DLBCL loader (trainer.py:307-312)
                it = iter(self.dlbcl_loader)
                images, labels = next(it)
            fl.run(images, labels)
    losses = fl.losses()
    fl.export_torch_state(self.optimizer)
    fl_l, dl_l = losses[:fl_steps], losses[fl_steps:]
    for i, v in enumerate(fl_l):
        self.writer.add_scalar("Loss/train_step", v, base + i)
        self.writer.add_scalar("Loss/fl_step", v, base + i)
    for i, v in enumerate(dl_l):
        self.writer.add_scalar("Loss/train_step", v, base + fl_steps + i)
        self.writer.add_scalar("Loss/dlbcl_step", v, base + fl_steps + i)
    total = len(losses)
    fl_avg = sum(fl_l) / len(fl_l) if fl_l else 0.0
    dl_avg = sum(dl_l) / len(dl_l) if dl_l else 0.0
    combined = sum(losses) / total if total else 0.0
    self.writer.add_scalar("Domain/fl_steps", len(fl_l), epoch)
    self.writer.add_scalar("Domain/dlbcl_steps", len(dl_l), epoch)
    self.writer.add_scalar("Domain/fl_ratio", len(fl_l) / total if total else 0.0, epoch)
    self.writer.add_scalar("Domain/dlbcl_ratio", len(dl_l) / total if total else 0.0, epoch)
    self.writer.add_scalar("Loss/fl_avg", fl_avg, epoch)
    self.writer.add_scalar("Loss/dlbcl_avg", dl_avg, epoch)
    self.writer.add_scalar("Loss/combined", combined, epoch)
    return combined


def bind(trainer_cls):
    """Replace the two loops on the Trainer class (keeping the originals for the fallback)."""
    if _FALLBACK not in trainer_cls.__dict__:
        setattr(trainer_cls, _FALLBACK, {"train_epoch": trainer_cls.train_epoch,
                                         "_train_epoch_step_based":
                                             trainer_cls._train_epoch_step_based})
    trainer_cls.train_epoch = train_epoch
    trainer_cls._train_epoch_step_based = train_epoch_step_based
    return trainer_cls
