#!/usr/bin/env python3
"""oracle/gen_golden.py — TEST INFRASTRUCTURE ONLY.

Regenerates every golden vector under tests/golden/ by running the reference
itself (oracle/_ref/ref_harness, built from /root/reference by `make -C oracle
ref`).  Run in the build container only; the GPU box never sees the reference,
only the committed fixtures this script writes.

    python oracle/gen_golden.py

Fixtures (all produced by the reference's own functions, see ref_harness.cpp):
  scene_final.txt / scene_learn.txt   random_scene() main.cpp:86-131 / learn() main.cpp:198-210
  camera_final.txt / camera_learn.txt camera::camera camera.h:8-45
  kats_final.txt / kats_learn.txt     srand(k) + one worker() sample, main.cpp:278-281
  funcs.txt                           sphere::hit, refract, reflect, reflectance, near_zero, scatter
  image_<scene>_<W>x<H>x<S>.f64       single-threaded worker() sums (raw float64)
  image_<scene>_<W>x<H>x<S>.sha256    sha256 of the float64 sums (large configs)
  learn_400x225x100.ppm               config 1 oracle image (reference P3 re-encoded as P6)
  gallery_final.png                   /root/reference/gallery/final.png (config 2, CPU oracle output)
  gallery_final_tiles40.npy           40x40 tile means of that PNG (float64, [20,30,3])
  gallery_final_scene_5000.png        /root/reference/gallery/final_scene_5000.png (the Next-Week final
                                      scene, the CUDA reference's output; statistical golden for rtmi_nw)
  earthmap.jpeg                       /root/reference/rt_next_week/cuda/earthmap.jpeg (its earth texture)
"""
import hashlib
import os
import shutil
import subprocess
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
GOLD = os.path.join(REPO, "tests", "golden")
HARNESS = os.path.join(HERE, "_ref", "ref_harness")
GALLERY = "/root/reference/gallery/final.png"


def run(*args, out=None):
    res = subprocess.run([HARNESS, *map(str, args)], check=True, capture_output=True, text=True)
    if out is not None:
        with open(os.path.join(GOLD, out), "w") as f:
            f.write(res.stdout)
    return res.stdout


def p3_to_p6(text):
    tok = text.split()
    assert tok[0] == "P3"
    w, h, mx = int(tok[1]), int(tok[2]), int(tok[3])
    px = np.array(tok[4:], dtype=np.int64).astype(np.uint8)
    assert px.size == w * h * 3 and mx == 255
    return b"P6\n%d %d\n255\n" % (w, h) + px.tobytes()


def image(scene, w, h, spp, keep_raw):
    tmp = os.path.join(HERE, "_ref", f"img_{scene}_{w}x{h}x{spp}.f64")
    ppm = run("image", scene, w, h, spp, 50, tmp)
    raw = open(tmp, "rb").read()
    stem = f"image_{scene}_{w}x{h}x{spp}"
    with open(os.path.join(GOLD, stem + ".sha256"), "w") as f:
        f.write(hashlib.sha256(raw).hexdigest() + "\n")
    if keep_raw:
        shutil.copyfile(tmp, os.path.join(GOLD, stem + ".f64"))
    os.remove(tmp)
    return ppm


def main():
    if not os.path.exists(HARNESS):
        sys.exit("build the reference harness first: make -C oracle ref")
    os.makedirs(GOLD, exist_ok=True)
    run("scene", out="scene_final.txt")
    run("learn_scene", out="scene_learn.txt")
    run("camera", "final", out="camera_final.txt")
    run("camera", "learn", out="camera_learn.txt")
    run("kats", "final", 64, out="kats_final.txt")
    run("kats", "learn", 64, out="kats_learn.txt")
    run("funcs", 64, out="funcs.txt")
    image("final", 24, 16, 8, keep_raw=True)
    image("learn", 32, 18, 16, keep_raw=True)
    image("final", 120, 80, 32, keep_raw=False)
    ppm = image("learn", 400, 225, 100, keep_raw=False)  # config 1
    with open(os.path.join(GOLD, "learn_400x225x100.ppm"), "wb") as f:
        f.write(p3_to_p6(ppm))
    # config 2 statistical golden: the gallery image is the CPU oracle's output
    from PIL import Image

    shutil.copyfile(GALLERY, os.path.join(GOLD, "gallery_final.png"))
    img = np.asarray(Image.open(GALLERY).convert("RGB"), dtype=np.float64)
    h, w, _ = img.shape
    tiles = img.reshape(h // 40, 40, w // 40, 40, 3).mean(axis=(1, 3))
    np.save(os.path.join(GOLD, "gallery_final_tiles40.npy"), tiles)
    # Next-Week data files: the reference's own render and texture
    shutil.copyfile("/root/reference/gallery/final_scene_5000.png", os.path.join(GOLD, "gallery_final_scene_5000.png"))
    shutil.copyfile("/root/reference/rt_next_week/cuda/earthmap.jpeg", os.path.join(GOLD, "earthmap.jpeg"))
    print("golden vectors written to", GOLD)


if __name__ == "__main__":
    main()
