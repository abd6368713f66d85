"""Generates tests/golden/scene_pins.npz from the reference's own renders
/root/reference/images/<scene>_<sampler>.png (RGBA8 sRGB, spp unrecorded) for the scenes
shipped under assets/scenes (features1, features2, materials1, materials2, materials4, shapes1
at 1280x533, bathroom1 at 1280x720, ecosys at 1280x640, coffee at 1024x1280, staircase2 at
1280x1280; both samplers).

The fixture is data only: per block (41 or 40 rows x 40 or 32 columns) the mean of the
sRGB-decoded linear values per channel, the block alpha mean and the whole-image channel mean.
It is the statistical pin of the HIP path on these scenes (tests/test_gpu_scenes.py).
Run in the build container (the reference is not on the GPU box):
    python tests/golden/scripts/make_scene_pins.py
"""
import os

import numpy as np
from PIL import Image

SCENES = ("features1", "features2", "materials1", "materials2", "materials4", "shapes1", "bathroom1", "ecosys",
          "coffee", "staircase2")
OUT = os.path.join(os.path.dirname(__file__), "..", "scene_pins.npz")

out = {}
for scene in SCENES:
    for sampler in ("naive", "path"):
        img = np.asarray(Image.open(f"/root/reference/images/{scene}_{sampler}.png").convert("RGBA"),
                         dtype=np.uint8)
        h, w = img.shape[:2]
        BH = 41 if h % 41 == 0 else 40
        BW = 40 if w % 40 == 0 else 32  # coffee is 1024 wide
        assert h % BH == 0 and w % BW == 0, (scene, h, w)
        c = img[..., :3].astype(np.float64) / 255.0
        lin = np.where(c <= 0.04045, c / 12.92, ((c + 0.055) / 1.055) ** 2.4)
        key = f"{scene}_{sampler}"
        out[key + "_mean"] = lin.reshape(h // BH, BH, w // BW, BW, 3).mean(axis=(1, 3)).astype(np.float32)
        out[key + "_alpha"] = (img[..., 3].reshape(h // BH, BH, w // BW, BW).mean(axis=(1, 3)) / 255.0
                               ).astype(np.float32)
        out[key + "_channel_mean"] = lin.reshape(-1, 3).mean(axis=0)
        out[key + "_size"] = np.array([w, h])
        out[key + "_block"] = np.array([BH, BW])
        print(key, (w, h), out[key + "_channel_mean"])
np.savez_compressed(OUT, **out)
print("wrote", OUT)
