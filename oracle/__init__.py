"""CPU oracle for the Light-3D-U-Net hot path — TEST INFRASTRUCTURE ONLY.

Only `tests/`, `__graft_entry__.smoke()` and `bench.py`'s `cpu_baseline` leg may import this
package, and only as the checker / CPU baseline.  The product path (`light_unet.*` in
`light-3d-unet-front_amd/`) never imports it and fails loudly when the HIP library is missing.

Contents
  unet_oracle.py    functional torch-CPU restatement of Lightweight3DUNet + FocalTverskyLoss
                    (unet3d.py:12-229, losses.py:11-54), fp32 or fp64.
  sliding_oracle.py numpy restatement of sliding_window_inference_3d (utils.py:11-173).

Pinning: both are checked against fixtures generated from the reference itself
(tests/golden/make_goldens.py imports /root/reference by file path) in
tests/test_oracle_golden.py.  The reference's own tests pin nothing on this path,
so the golden fixtures are the anchor.
"""
