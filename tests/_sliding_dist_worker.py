"""Worker of tests/test_sliding_gpu.py::test_sliding_window_sharded_over_ranks (not a test
module): every rank runs the window-sharded device sliding window on the fixture volume; rank 0
saves the map.  Launched by torch.distributed.run (gloo, all ranks on cuda:0)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "light-3d-unet-front_amd")):
    sys.path.insert(0, p)

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402


def main():
    out = sys.argv[1]
    dist.init_process_group("gloo")
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    from light_unet.models.unet3d import Lightweight3DUNet
    from light_unet.utils import sliding_window_inference_3d
    z = np.load(os.path.join(ROOT, "tests", "golden", "sliding.npz"), allow_pickle=False)
    m = Lightweight3DUNet()
    m.load_state_dict({k[2:]: torch.from_numpy(z[k]) for k in z.files if k.startswith("w/")})
    m = m.to(dev)
    prob = sliding_window_inference_3d(z["v64_56_72/image"], m, (48, 48, 48), 0.5, dev, True,
                                       window_batch=2, group=dist.group.WORLD)
    if dist.get_rank() == 0:
        np.save(out, prob)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
