"""Multi-GPU sharding of the hot path: one process per GPU, samples split into
contiguous global ranges, one collective at the end.

Every (pixel, sample) is independent and the RNG is keyed by the *global* sample index, so
rank r traces samples [r*S/N, (r+1)*S/N) of every pixel on its own GPU with no data-path
communication. Each rank's accumulator is the running mean of its shard (src/trace.jl:631-648
restricted to the shard); the image is the sample-weighted sum of the shard means:

    image = sum_r n_r * mean_r / S

computed by one sum-reduce (RCCL over xGMI with backend "nccl"; gloo on CPU in the tests).
"""
from __future__ import annotations

import json
from pathlib import Path

import numpy as np


def shard_range(total_samples: int, world: int, rank: int) -> tuple[int, int]:
    return rank * total_samples // world, (rank + 1) * total_samples // world


def split_plan(world: int, rank: int, total_samples: int, tile_groups: int):
    """Rank `rank`'s share of a render over `world` processes split into `tile_groups` interleaved
    8x8-tile groups (a power of two dividing world; 1 = a pure sample split) times world /
    tile_groups contiguous sample ranges: (tile_share option value or None, s0, s1). Every pixel is
    covered by world / tile_groups ranks whose sample ranges partition [0, total_samples), so the
    same sample-weighted reduce (reduce_running_means) combines any plan."""
    if tile_groups < 1 or world % tile_groups:
        raise ValueError(f"tile_groups {tile_groups} must divide world {world}")
    g, k = rank % tile_groups, rank // tile_groups
    s0, s1 = shard_range(total_samples, world // tile_groups, k)
    return (f"{tile_groups},{g}" if tile_groups > 1 else None), s0, s1


def reduce_running_means(tensor, n_local: int, n_total: int, dist, dst: int = 0):
    """Sum-reduce sample-weighted shard means onto `dst`; returns the combined mean on `dst`
    (the partial sum elsewhere). `tensor` is left untouched."""
    part = tensor * float(n_local)
    dist.reduce(part, dst=dst, op=dist.ReduceOp.SUM)
    if dist.get_rank() == dst:
        part /= float(n_total)
    return part


class PipelinedReduce:
    """The bench's per-step reduce of sample-weighted shard means onto `dst`, pipelined: submit()
    snapshots the shard image (times n_local) into one of two buffers and starts the reduce
    asynchronously, so it runs during the next step's launch; a buffer is reused only after its
    previous reduce completed. `sync` (the GPU: the current stream's synchronize) returns once
    the snapshot is taken, so the caller may overwrite `src` (the library's next jt_reset).
    drain() completes every reduce and returns the last submitted step's combined mean on `dst`
    (None elsewhere)."""

    def __init__(self, numel: int, n_local: int, n_total: int, dist, device="cpu", dst: int = 0, sync=None):
        import torch
        self.torch, self.dist, self.dst, self.sync = torch, dist, dst, sync
        self.n_local, self.n_total = float(n_local), float(n_total)
        self.bufs = [torch.empty(numel, dtype=torch.float32, device=device) for _ in range(2)]
        self.pending = [None, None]
        self.last = None

    def submit(self, src):
        i = 0 if self.last is None else 1 - self.last
        if self.pending[i] is not None:
            self.pending[i].wait()
            self.pending[i] = None
        self.torch.mul(src, self.n_local, out=self.bufs[i])
        if self.sync is not None:
            self.sync()
        self.pending[i] = self.dist.reduce(self.bufs[i], dst=self.dst, op=self.dist.ReduceOp.SUM, async_op=True)
        self.last = i

    def drain(self):
        for i in range(2):
            if self.pending[i] is not None:
                self.pending[i].wait()
                self.pending[i] = None
        if self.last is None or self.dist.get_rank() != self.dst:
            return None
        return self.bufs[self.last] / self.n_total


def all_reduce_running_means(tensor, n_local: int, n_total: int, dist):
    part = tensor * float(n_local)
    dist.all_reduce(part, op=dist.ReduceOp.SUM)
    part /= float(n_total)
    return part


# ------------------------------------------------------------------ reduced-image check
# The multi-rank bench proves its reduce with a deterministic fingerprint of the image: block means
# of the final running-mean RGBA, committed once per workload from a one-GPU run
# (profiles/image_signatures.json) and compared by rank 0 after every run. A sample split equals the
# one-device image up to fp32 summation order (~1e-6 relative), so block means agree to ~1e-6; a
# missing or doubled shard, a wrong weight or a stale buffer moves them by percents.
SIGNATURE_BLOCK = 40
SIGNATURE_RTOL = 1e-4
SIGNATURE_ATOL = 1e-6


def image_signature(img, block: int = SIGNATURE_BLOCK) -> np.ndarray:
    """Block means (float64) of an (H, W, 4) image over block x block pixels (edge blocks partial)."""
    a = np.asarray(img, np.float64)
    H, W = a.shape[:2]
    hb, wb = -(-H // block), -(-W // block)
    out = np.zeros((hb, wb, a.shape[2]))
    for i in range(hb):
        for j in range(wb):
            out[i, j] = a[i * block:(i + 1) * block, j * block:(j + 1) * block].mean(axis=(0, 1))
    return out


def load_signature(path, key: str):
    p = Path(path)
    if not p.exists():
        return None
    d = json.loads(p.read_text()).get(key)
    return None if d is None else np.asarray(d["blocks"], np.float64)


def save_signature(path, key: str, sig: np.ndarray, note: str):
    p = Path(path)
    d = json.loads(p.read_text()) if p.exists() else {}
    d[key] = {"block": SIGNATURE_BLOCK, "note": note, "blocks": np.round(sig, 9).tolist()}
    p.write_text(json.dumps(d, indent=0, sort_keys=True))


def compare_signature(sig: np.ndarray, ref: np.ndarray) -> dict:
    """max relative error of the block means against the reference, and whether it is within
    SIGNATURE_RTOL (+ SIGNATURE_ATOL for near-black blocks)."""
    if sig.shape != ref.shape:
        return {"ok": False, "max_rel": None, "why": f"shape {sig.shape} vs reference {ref.shape}"}
    err = np.abs(sig - ref)
    ok = bool(np.all(err <= SIGNATURE_RTOL * np.abs(ref) + SIGNATURE_ATOL))
    rel = float(np.max(err / np.maximum(np.abs(ref), SIGNATURE_ATOL)))
    return {"ok": ok, "max_rel": rel}
