"""Save one TrainStep's flat gradient (bs 4, 48^3 or RD_SIZE) for cross-library comparison."""
import os
import sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "light-3d-unet-front_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402
from light_unet.models.unet3d import Lightweight3DUNet  # noqa: E402
from light_unet.train_step import TrainStep  # noqa: E402
dev = torch.device("cuda:0")
L = int(os.environ.get("RD_SIZE", "48"))
torch.manual_seed(42)
m = Lightweight3DUNet(dropout_p=0.0).to(dev).train()
g = torch.Generator().manual_seed(3)
x = torch.rand(4, 1, L, L, L, generator=g).to(dev)
t = (torch.rand(4, 1, L, L, L, generator=g) > 0.97).float().to(dev)
ts = TrainStep(m)
p, sv, sums = ts._fwd(x, t)
ts._bwd(p, sv, t, sums)
torch.cuda.synchronize()
np.save(os.path.join(ROOT, "gpurun_out", sys.argv[1] + ".npy"), ts.gflat.cpu().numpy())
