"""C4 (TUM1: 640x480, scale 1.2, 8 levels) batched pyramid stage alone, 256 frames:
python tools/mb_c4pyr.py [lib.so ...] -- one child per library (YGZFE_LIB), HIP-event
stage time of the pyramid, averaged over 10 extractions (ms per 256 frames)."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

if len(sys.argv) > 1 and sys.argv[1] == "--child":
    sys.path.insert(0, os.path.join(ROOT, "orb-ygz-slam_amd"))
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    sys.path.insert(0, ROOT)
    import numpy as np
    import ygzfe
    import _scenes as S
    from ygzfe.sequence import XI, sweep_index
    W, H, nf, sf, nl, ini, mn = S.CONFIGS["C4"]
    B = 256
    sc = S.PlaneScene(23, W, H)
    frames = np.stack([sc.render(*ygzfe.trajectory_pose(sweep_index(i), XI), noise_seed=i) for i in range(B)])
    b = ygzfe.Batch((nf, sf, nl, ini, mn, 0), 0, W, H, B)
    vals = []
    for rep in range(3):
        b.upload(frames)
        b.timing(True)
        for _ in range(10):
            b.extract(B)
        st = b.timing(False)
        vals.append(st.get("pyramid", float("nan")))
    b.check()
    print(f"{os.path.basename(os.environ.get('YGZFE_LIB', 'libygzfe.so'))}: pyramid "
          + " ".join(f"{v:.4f}" for v in vals) + " ms / 256 frames")
else:
    for lib in sys.argv[1:] or ["libygzfe.so"]:
        env = dict(os.environ, YGZFE_LIB=os.path.join(ROOT, "orb-ygz-slam_amd", "lib", lib))
        subprocess.run([sys.executable, __file__, "--child"], env=env, check=True, timeout=300)
