"""Generates tests/golden/cornellbox_path_blocks.npz from the reference's own render
/root/reference/images/cornellbox_path.png (1280x1280, RGBA8 sRGB, spp unrecorded).

The fixture is data only: per 40x40-pixel block (32x32 blocks) the mean and the standard
deviation of the sRGB-decoded linear values, per channel. It is the statistical pin for the
oracle and the HIP path (tests/test_oracle_golden.py, tests/test_gpu_parity.py).
Run in the build container (the reference is not on the GPU box):
    python tests/golden/scripts/make_cornellbox_pin.py
"""
import os
import numpy as np
from PIL import Image

SRC = "/root/reference/images/cornellbox_path.png"
OUT = os.path.join(os.path.dirname(__file__), "..", "cornellbox_path_blocks.npz")
B = 40

img = np.asarray(Image.open(SRC).convert("RGBA"), dtype=np.uint8)
h, w = img.shape[:2]
c = img[..., :3].astype(np.float64) / 255.0
lin = np.where(c <= 0.04045, c / 12.92, ((c + 0.055) / 1.055) ** 2.4)
blocks = lin.reshape(h // B, B, w // B, B, 3)
mean = blocks.mean(axis=(1, 3)).astype(np.float32)
std = blocks.std(axis=(1, 3)).astype(np.float32)
alpha = img[..., 3].reshape(h // B, B, w // B, B).mean(axis=(1, 3)).astype(np.float32) / 255.0
np.savez_compressed(OUT, mean=mean, std=std, alpha=alpha, width=w, height=h, block=B,
                    channel_mean=lin.reshape(-1, 3).mean(axis=0))
print("wrote", OUT, mean.shape, lin.reshape(-1, 3).mean(axis=0))
