"""FAST and orientation+rBRIEF stages alone (ygzfe_diag_stage_ms) on the bench's C2
frames, for A/B library variants: python tools/mb_fast.py B lib1.so [lib2.so ...] --
one child process per library (each loads its own build); prints ms per 1024 frames."""
import ctypes as C
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def child(B, libpath):
    sys.path.insert(0, os.path.join(ROOT, "orb-ygz-slam_amd"))
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    sys.path.insert(0, ROOT)
    import ygzfe
    ygzfe.LIB_PATH = libpath
    import _scenes as S
    from bench import sweep_index
    W, H, nf, sf, nl, ini, mn = S.CONFIGS["C2"]
    sc = S.PlaneScene(11, W, H)
    xi = np.array([0.012, -0.006, 0.009, 0.0025, -0.002, 0.0015], np.float32)
    frames = np.stack([sc.render(*ygzfe.trajectory_pose(sweep_index(i), xi), noise_seed=i) for i in range(B)])
    b = ygzfe.Batch((nf, sf, nl, ini, mn, 0), 0, W, H, B)
    b.upload(frames)
    L = ygzfe.lib()
    L.ygzfe_diag_stage_ms.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_int, C.POINTER(C.c_float)]
    ms = C.c_float()
    out = []
    stages = [int(x) for x in os.environ.get("YGZ_MB_STAGES", "0,1").split(",")]
    for stage, name in [(st, ("FAST", "orient", "blur")[st]) for st in stages]:
        if stage == 1:
            b.extract(B)  # the octree selection the orientation pass reads
            b.check()
        assert L.ygzfe_diag_stage_ms(b.h, stage, B, 3, 1 if stage == 0 else 0, C.byref(ms)) == 0, "diag"
        vals = []
        for _ in range(5):
            assert L.ygzfe_diag_stage_ms(b.h, stage, B, 10, 0, C.byref(ms)) == 0
            vals.append(ms.value)
        out.append(f"{name} {np.median(vals) * 1024 / B:.4f}")
    print(f"{os.path.basename(libpath)}: " + "  ".join(out) + " ms / 1024 frames", flush=True)


if __name__ == "__main__":
    if sys.argv[1] == "--child":
        child(int(sys.argv[2]), sys.argv[3])
        sys.exit(0)
    B = int(sys.argv[1])
    for lib in sys.argv[2:]:
        path = lib if os.path.isabs(lib) else os.path.join(ROOT, "orb-ygz-slam_amd", "lib", lib)
        r = subprocess.run([sys.executable, __file__, "--child", str(B), path], timeout=150)
        if r.returncode not in (0, 1):
            sys.exit(r.returncode)
