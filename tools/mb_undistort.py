"""Time the batched undistort remap (k_remap_linear) over N resident EuRoC frames."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "orb-ygz-slam_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import ygzfe  # noqa: E402
import _cameras as CAM  # noqa: E402

cam, dist, (W, H) = CAM.EUROC
n = int(sys.argv[1]) if len(sys.argv) > 1 else 256
und = ygzfe.Undistort(cam, dist, W, H)
src = torch.from_numpy(np.stack([ygzfe.synth_texture(s % 16, W, H) for s in range(n)])).cuda()
dst = torch.empty_like(src)
st = torch.cuda.Stream()
torch.cuda.set_stream(st)
for _ in range(5):
    und.apply_device(src.data_ptr(), W * H, W, dst.data_ptr(), W * H, W, n, st.cuda_stream)
a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
reps = 50
a.record(st)
for _ in range(reps):
    und.apply_device(src.data_ptr(), W * H, W, dst.data_ptr(), W * H, W, n, st.cuda_stream)
b.record(st)
torch.cuda.synchronize()
ms = a.elapsed_time(b) / reps
assert st.cuda_stream != 0
alg = n * W * H * 2 + W * H * 6  # read + write each frame, the map once
print(f"remap {n} frames {W}x{H}: {ms*1e3:.1f} us/launch, {n/ms*1e3:.0f} frames/s, {alg/ms/1e6:.0f} GB/s alg")
