"""Installs the MI355X hot path into an existing reference `light_unet` package.

The reference Trainer / Inferencer import the model and loss by module path
(trainer.py:16-17, inferencer.py:13) next to modules this build does not replace
(light_unet.datasets, light_unet.core.config, light_unet.models.metrics).  Both packages are
called `light_unet`, so this build is loaded under the alias `l3u_amd` (its modules only use
relative imports) and its classes are bound into the reference's module objects:

    import l3u_plugin
    l3u_plugin.install()                       # before `from light_unet.core.trainer import Trainer`
    from light_unet.core.trainer import Trainer

After install():
    light_unet.models.unet3d.Lightweight3DUNet      -> l3u_amd.models.unet3d.Lightweight3DUNet
    light_unet.models.losses.FocalTverskyLoss       -> l3u_amd.models.losses.FocalTverskyLoss
    light_unet.models.losses.get_loss_function      -> l3u_amd.models.losses.get_loss_function
    light_unet.models.Lightweight3DUNet / get_loss_function (package re-exports, models/__init__.py:6-8)
    light_unet.utils.sliding_window_inference_3d    -> l3u_amd.utils.sliding_window_inference_3d
Everything else in the reference package is left untouched.
"""
import importlib
import importlib.util
import os
import sys

_HERE = os.path.dirname(os.path.abspath(__file__))
ALIAS = "l3u_amd"

REPLACED = {
    "light_unet.utils": ("sliding_window_inference_3d",),
    "light_unet.models.unet3d": ("Lightweight3DUNet",),
    "light_unet.models.losses": ("FocalTverskyLoss", "get_loss_function"),
    "light_unet.models": ("Lightweight3DUNet", "FocalTverskyLoss", "get_loss_function"),
}


def load():
    """This build's package, imported as `l3u_amd` (no clash with the reference's light_unet)."""
    if ALIAS in sys.modules:
        return sys.modules[ALIAS]
    pkg_dir = os.path.join(_HERE, "light_unet")
    spec = importlib.util.spec_from_file_location(
        ALIAS, os.path.join(pkg_dir, "__init__.py"), submodule_search_locations=[pkg_dir])
    mod = importlib.util.module_from_spec(spec)
    sys.modules[ALIAS] = mod
    spec.loader.exec_module(mod)
    importlib.import_module(ALIAS + ".models.unet3d")
    importlib.import_module(ALIAS + ".models.losses")
    importlib.import_module(ALIAS + ".utils")
    importlib.import_module(ALIAS + ".fast_trainer")
    importlib.import_module(ALIAS + ".lesion")
    importlib.import_module(ALIAS + ".patches")
    return mod


LESION = ("get_connected_components", "match_components", "calculate_lesion_metrics",
          "calculate_metrics")


def _bind_lesion(done):
    """The device lesion post-processing (light_unet/lesion.py) into the reference's metrics
    module (metrics.py:38-404) and into the modules that imported those names already
    (core.trainer: calculate_metrics; core.inferencer: get_connected_components), plus
    Inferencer.extract_bboxes (inferencer.py:62-111).  Skipped where the reference module cannot
    be imported (e.g. its scipy / sklearn / nibabel dependencies are missing)."""
    les = sys.modules[ALIAS + ".lesion"]
    try:
        metrics = importlib.import_module("light_unet.models.metrics")
    except ImportError:
        return
    names = [n for n in LESION if hasattr(metrics, n)]
    # every input form the reference functions take -- [D, H, W] volumes and batched
    # [B, D, H, W] arrays (labelled as one 4-dimensional array, as ndimage.label does) -- runs on
    # the device (csrc/lesion.hip); nothing is handed back to the host functions
    bound = {n: getattr(les, n) for n in names}
    for n in names:
        setattr(metrics, n, bound[n])
    done["light_unet.models.metrics"] = names
    for modname in ("light_unet.models", "light_unet.core.trainer", "light_unet.core.inferencer"):
        mod = sys.modules.get(modname)
        if mod is None:
            continue
        hit = [n for n in names if n in vars(mod)]
        for n in hit:
            setattr(mod, n, bound[n])
        if hit:
            done.setdefault(modname, []).extend(hit)
    inf = sys.modules.get("light_unet.core.inferencer")
    if inf is not None and hasattr(inf, "Inferencer"):
        def extract_bboxes(self, prob_map, threshold=0.3, min_volume_cc=0.5, spacing=(4.0, 4.0, 4.0)):
            return les.extract_bboxes(prob_map, threshold, min_volume_cc, spacing,
                                      self.config["data"]["bbox_expansion_voxels"])
        inf.Inferencer.extract_bboxes = extract_bboxes
        done.setdefault("light_unet.core.inferencer", []).append("Inferencer.extract_bboxes")


def _bind_device_patches(done):
    """The training loaders of light_unet.datasets.loader (get_data_loader, loader.py:99-113)
    on device patches: loader._create_train_loader (loader.py:9-10, called by the standard,
    step-based and probabilistic factories) returns a DevicePatchLoader over the device twin of
    the PatchDataset / MixedPatchDataset the factory just built (its cases read once into HBM,
    its sampled locations kept; l3u_amd.patches).  Validation loaders are unchanged."""
    loader = importlib.import_module("light_unet.datasets.loader")
    patches = sys.modules[ALIAS + ".patches"]
    ref = getattr(loader._create_train_loader, "_l3u_reference", loader._create_train_loader)

    def _create_train_loader(dataset, batch_size, shuffle=True):
        return patches.device_loader(dataset, batch_size)
    _create_train_loader._l3u_reference = ref
    loader._create_train_loader = _create_train_loader
    done["light_unet.datasets.loader"] = ["_create_train_loader"]


def install(fast_step=False, lesion=True, device_patches=False):
    """Bind this build's model and loss into the already-importable reference package.
    Returns {module: [names]} of what was replaced.  Raises ImportError when the reference's
    light_unet.models.{unet3d,losses} cannot be imported (nothing is half-installed).

    fast_step=True also replaces Trainer.train_epoch / Trainer._train_epoch_step_based
    (trainer.py:208-347) with the graph-replayed TrainStep loops of light_unet/fast_trainer.py
    (same batches, update, TensorBoard scalars and return values; no per-step host sync; RCCL
    data parallelism when torch.distributed is initialised).  Needs light_unet.core.trainer.

    lesion=True (default) also binds the device lesion post-processing (connected components,
    matching, lesion / voxel metrics, bounding boxes: light_unet/lesion.py) where the reference's
    metrics module imports.

    device_patches=True also makes get_data_loader's training loaders cut
    and augment their patches on the device (light_unet/patches.py; num_workers = 0 draw
    semantics, DevicePatchLoader), so the graph-replayed step never waits on host workers or a
    PCIe copy.  Needs light_unet.datasets.loader (and its NIfTI reader)."""

    amd = load()
    trainer_mod = importlib.import_module("light_unet.core.trainer") if fast_step else None
    src = {
        "Lightweight3DUNet": sys.modules[ALIAS + ".models.unet3d"].Lightweight3DUNet,
        "FocalTverskyLoss": sys.modules[ALIAS + ".models.losses"].FocalTverskyLoss,
        "get_loss_function": sys.modules[ALIAS + ".models.losses"].get_loss_function,
        "sliding_window_inference_3d": sys.modules[ALIAS + ".utils"].sliding_window_inference_3d,
    }
    mods = {}
    for modname in ("light_unet.utils", "light_unet.models.unet3d", "light_unet.models.losses"):
        mods[modname] = importlib.import_module(modname)
    pkg = sys.modules.get("light_unet.models")
    if pkg is not None:
        mods["light_unet.models"] = pkg
    done = {}
    for modname, mod in mods.items():
        for name in REPLACED[modname]:
            setattr(mod, name, src[name])
        done[modname] = list(REPLACED[modname])
    if fast_step:
        fast = importlib.import_module(ALIAS + ".fast_trainer")
        fast.bind(trainer_mod.Trainer)
        done["light_unet.core.trainer"] = ["Trainer.train_epoch", "Trainer._train_epoch_step_based"]
    if device_patches:
        _bind_device_patches(done)
    if lesion:
        _bind_lesion(done)
    amd.installed_into = done
    return done
