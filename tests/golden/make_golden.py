"""Generate the FAST-10 golden vectors from the reference's own Thirdparty/fast.

Runs ONLY in the build container, where /root/reference exists and
oracle/Makefile has compiled its fast sources into oracle/_ref/libfastref.so
(`make -C oracle ref`).  The output, tests/golden/fast10_ref.npz, is data:
inputs (test1.png is the reference's own test image, Thirdparty/fast/test/data;
two small seeded synthetic frames are stored verbatim) and the reference
library's outputs for them.  No reference code is copied.

Contents:
  * detect (plain decision tree and SSE2), score and 3x3 non-max for every image
    at thresholds {5, 7, 20, 75}, called on the in-bounds interior
    (img + 3*W + 3, W-6, H-6) as the known-answer test must be;
  * the DSO cell path (ORBextractor.cc:1317-1345): fast_corner_detect_10_sse2 on
    g x g cells, g in {18, 19, 22, 30} (narrower than 22 -> plain tree over the
    whole cell, faster_corner_10_sse.cpp:192-194), thresholds {20, 5}.

    python tests/golden/make_golden.py
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
import _oracle as O  # noqa: E402

THRESHOLDS = (5, 7, 20, 75)
DSO_CELLS = (18, 19, 22, 30)
DSO_TH = (20, 5)


def synth_frame(seed, W, H):
    """Seeded rectangles + noise (independent of the product's synth lib)."""
    rng = np.random.default_rng(seed)
    img = np.full((H, W), 128, np.int32)
    for _ in range(60):
        x0, y0 = rng.integers(0, W), rng.integers(0, H)
        w, h = rng.integers(4, 30, size=2)
        img[y0:y0 + h, x0:x0 + w] = rng.integers(0, 256)
    img += rng.integers(-3, 4, size=img.shape)
    return np.clip(img, 0, 255).astype(np.uint8)


def images():
    from PIL import Image
    test1 = np.array(Image.open(os.path.join(HERE, "test1.png")))
    return {"test1": test1, "synth_a": synth_frame(1, 160, 120), "synth_b": synth_frame(2, 97, 61)}


def main():
    if not O.RefFast.available():
        raise SystemExit("oracle/_ref/libfastref.so missing: run `make -C oracle ref` with /root/reference present")
    ref = O.RefFast()
    out = {}
    for name, img in images().items():
        H, W = img.shape
        if name != "test1":  # test1 is tests/golden/test1.png itself
            out[f"{name}/img"] = img
        for th in THRESHOLDS:
            for sse in (0, 1):
                xs, ys = ref.detect(img, th, sse=bool(sse), x0=3, y0=3, w=W - 6, h=H - 6)
                out[f"{name}/t{th}/s{sse}/xy"] = np.stack([xs, ys], 1).astype(np.int16)
            xs, ys = out[f"{name}/t{th}/s1/xy"].T
            sc = ref.scores(img, xs, ys, th, x0=3, y0=3)
            out[f"{name}/t{th}/score"] = sc.astype(np.int32)
            out[f"{name}/t{th}/keep"] = ref.nonmax(xs, ys, sc).astype(np.int32)
    # DSO cells on test1: interior cells (>= 3 px from the border) of a g-grid
    img = images()["test1"]
    H, W = img.shape
    for g in DSO_CELLS:
        cells = [(x, y) for y in range(g, H - 2 * g, g) for x in range(g, W - 2 * g, g)][::7][:40]
        out[f"dso/g{g}/cells"] = np.array(cells, np.int16)
        for th in DSO_TH:
            xy, offs = [], [0]
            for (x, y) in cells:
                xs, ys = ref.detect(img, th, sse=True, x0=x, y0=y, w=g, h=g)
                xy.append(np.stack([xs, ys], 1))
                offs.append(offs[-1] + len(xs))
            out[f"dso/g{g}/t{th}/xy"] = np.concatenate(xy).astype(np.int16) if xy else np.zeros((0, 2), np.int16)
            out[f"dso/g{g}/t{th}/offs"] = np.array(offs, np.int32)
    path = os.path.join(HERE, "fast10_ref.npz")
    np.savez_compressed(path, **out)
    n75 = len(out["test1/t75/s1/xy"])
    print(f"wrote {path} ({os.path.getsize(path)} bytes); test1 th=75 corners: {n75}")


if __name__ == "__main__":
    main()
