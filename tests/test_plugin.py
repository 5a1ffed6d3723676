"""l3u_plugin.install() binds this build's model and loss into a reference-shaped `light_unet`
package (a stand-in with the reference's module layout: the reference itself is not imported)."""
import os
import subprocess
import sys
import textwrap

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "light-3d-unet-front_amd")


def _standin(tmp_path):
    base = tmp_path / "light_unet"
    (base / "models").mkdir(parents=True)
    (base / "core").mkdir()
    (base / "__init__.py").write_text("")
    (base / "utils.py").write_text("def sliding_window_inference_3d(image, model):\n    return 'reference'\n")
    (base / "models" / "__init__.py").write_text(
        "from .unet3d import Lightweight3DUNet\nfrom .losses import FocalTverskyLoss, get_loss_function\n")
    (base / "models" / "unet3d.py").write_text("class Lightweight3DUNet:\n    origin = 'reference'\n")
    (base / "models" / "metrics.py").write_text(
        "def get_connected_components(mask, min_size=0):\n    return 'reference'\n"
        "def match_components(*a, **k):\n    return 'reference'\n"
        "def calculate_lesion_metrics(*a, **k):\n    return 'reference'\n"
        "def calculate_metrics(*a, **k):\n    return 'reference'\n")
    (base / "models" / "losses.py").write_text(
        "class FocalTverskyLoss:\n    origin = 'reference'\n\n"
        "def get_loss_function(cfg):\n    return FocalTverskyLoss()\n")
    # a reference-style consumer that imports by module path at import time (trainer.py:16-17)
    (base / "core" / "__init__.py").write_text("")
    (base / "core" / "trainer.py").write_text(
        "from light_unet.models.unet3d import Lightweight3DUNet\n"
        "from light_unet.models.losses import get_loss_function\n"
        "from light_unet.utils import sliding_window_inference_3d\n"
        "from light_unet.models.metrics import calculate_metrics\n\n"
        "class Trainer:\n"
        "    def train_epoch(self, epoch):\n        return 'reference'\n"
        "    def _train_epoch_step_based(self, epoch):\n        return 'reference'\n")


def test_install_binds_model_and_loss(tmp_path):
    _standin(tmp_path)
    script = textwrap.dedent(f"""
        import importlib.util, sys
        sys.path.insert(0, {str(tmp_path)!r})
        spec = importlib.util.spec_from_file_location("l3u_plugin", {os.path.join(PKG, "l3u_plugin.py")!r})
        plug = importlib.util.module_from_spec(spec); spec.loader.exec_module(plug)
        done = plug.install()
        from light_unet.core import trainer
        import light_unet.models as m
        assert trainer.Lightweight3DUNet.__module__ == "l3u_amd.models.unet3d", trainer.Lightweight3DUNet
        assert trainer.get_loss_function.__module__ == "l3u_amd.models.losses"
        assert m.FocalTverskyLoss.__module__ == "l3u_amd.models.losses"
        assert trainer.sliding_window_inference_3d.__module__ == "l3u_amd.utils"
        import light_unet.models.metrics as met
        for n in ("get_connected_components", "match_components", "calculate_lesion_metrics",
                  "calculate_metrics"):
            assert getattr(met, n).__module__ == "l3u_amd.lesion", n
        assert trainer.calculate_metrics.__module__ == "l3u_amd.lesion"
        # batched [B, D, H, W] arrays stay on the device path too (no host fallback; install()
        # twice binds the same functions)
        plug.install()
        assert met.get_connected_components.__module__ == "l3u_amd.lesion"
        assert sys.modules["light_unet"].__file__.startswith({str(tmp_path)!r})
        net = trainer.Lightweight3DUNet()
        assert net.count_parameters()["total"] == 217228
        loss = trainer.get_loss_function({{"name": "FocalTverskyLoss"}})
        assert type(loss).__name__ == "FocalTverskyLoss"
        print("OK", sorted(done))
    """)
    r = subprocess.run([sys.executable, "-c", script], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "OK" in r.stdout


def test_install_fast_step_binds_trainer_loops(tmp_path):
    _standin(tmp_path)
    script = textwrap.dedent(f"""
        import importlib.util, sys
        sys.path.insert(0, {str(tmp_path)!r})
        spec = importlib.util.spec_from_file_location("l3u_plugin", {os.path.join(PKG, "l3u_plugin.py")!r})
        plug = importlib.util.module_from_spec(spec); spec.loader.exec_module(plug)
        done = plug.install(fast_step=True)
        from light_unet.core.trainer import Trainer
        assert Trainer.train_epoch.__module__ == "l3u_amd.fast_trainer"
        assert Trainer._train_epoch_step_based.__module__ == "l3u_amd.fast_trainer"
        # the reference loops stay reachable (fallback for losses other than FocalTversky)
        orig = Trainer._l3u_reference_loops
        assert orig["train_epoch"](None, 0) == "reference"
        assert "light_unet.core.trainer" in done
        # binding twice keeps the reference originals
        plug.install(fast_step=True)
        assert Trainer._l3u_reference_loops["train_epoch"](None, 0) == "reference"
        fast = sys.modules["l3u_amd.fast_trainer"]
        cfg = {{"training": {{"mixed_domains": {{"dlbcl_steps_ratio": 0.5}}}}}}
        assert fast.dlbcl_step_count(cfg, 7) == round(3.5)
        cfg["training"]["mixed_domains"]["dlbcl_steps"] = 2
        assert fast.dlbcl_step_count(cfg, 7) == 2
        print("OK")
    """)
    r = subprocess.run([sys.executable, "-c", script], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "OK" in r.stdout
