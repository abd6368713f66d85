"""Cli module mirror (src/cli.jl): the same flags, types and defaults as the reference's
ArgParse table (:12-86), the SAMPLER_TYPES index (:88) and Params (:90-138).

Extensions beyond the reference (all optional): --seed (RNG seed), --width/--height (explicit
image size, camera aspect := W/H), --device, --devices N (one context over GPUs 0..N-1:
jt_create_multi), --missing (drop|error for incomplete scenes), --traversal (reference|near|wide|auto:
the BVH traversal, include/jtrace.h jt_traversal).
"""
from __future__ import annotations

import argparse
from dataclasses import dataclass

SAMPLER_TYPES = ["path", "naive"]
# BVH traversal of every product entry point (the CLI, Params, abi.make_params, bench.py and the
# Julia shim): "auto" — the 4-wide quantised records ("wide") for a scene that runs from HBM with
# a deep BVH (stack bound above 32), the binary tree near child first ("near") otherwise, resolved
# by the library (jt_describe reports which). "reference" is the reference's far-first order (src/bvh.jl:331-341); all differ only
# where two hits tie at exactly equal t or a box is culled by the slab test's rounding.
DEFAULT_TRAVERSAL = "auto"


def _bool(s: str) -> bool:  # ArgParse arg_type = Bool parses "true"/"false"
    v = str(s).strip().lower()
    if v in ("true", "1", "yes"):
        return True
    if v in ("false", "0", "no"):
        return False
    raise argparse.ArgumentTypeError(f"invalid Bool value: {s}")


def _parser() -> argparse.ArgumentParser:
    p = argparse.ArgumentParser(prog="jtrace", description="MI355X path tracer (Jtrace.main drop-in)")
    p.add_argument("--scene", type=str, required=True, help="scene filename")
    p.add_argument("--output", type=str, default="tests/test_scene.png", help="output filename")
    p.add_argument("--camera", type=str, default="", help="camera name")
    p.add_argument("--addsky", type=_bool, default=False, help="add sky")
    p.add_argument("--envname", type=str, default="", help="add environment")
    p.add_argument("--resolution", type=int, default=1280, help="image resolution")
    p.add_argument("--samples", type=int, default=512, help="number of samples")
    p.add_argument("--bounces", type=int, default=8, help="number of bounces")
    p.add_argument("--denoise", type=_bool, default=False, help="enable denoiser")
    p.add_argument("--noparallel", type=_bool, default=False, help="disable threading")
    p.add_argument("--highqualitybvh", type=_bool, default=False, help="enable high quality bvh")
    p.add_argument("--envhidden", type=_bool, default=False, help="hide environment")
    p.add_argument("--tentfilter", type=_bool, default=False, help="filter image")
    p.add_argument("--sampler", type=str, default="path", help="sampler type")
    p.add_argument("--clamp", type=float, default=10.0, help="clamp image")
    p.add_argument("--nocaustics", type=_bool, default=False, help="disable caustics")
    p.add_argument("--batch", type=int, default=1, help="run samples in batches")
    p.add_argument("--bvhstacksize", type=int, default=128, help="max depth of bvh exploration")
    # extensions
    p.add_argument("--seed", type=lambda s: int(s, 0), default=0x5EED, help="RNG seed (extension)")
    p.add_argument("--width", type=int, default=0, help="image width (extension)")
    p.add_argument("--height", type=int, default=0, help="image height (extension)")
    p.add_argument("--device", type=int, default=0, help="HIP device (extension)")
    p.add_argument("--devices", type=int, default=1,
                   help="GPUs of this node to shard every batch over, devices 0..N-1 (extension)")
    p.add_argument("--missing", choices=["error", "drop"], default="error",
                   help="missing scene assets: error (reference) or drop (extension)")
    p.add_argument("--traversal", choices=["reference", "near", "wide", "auto"], default=DEFAULT_TRAVERSAL,
                   help="BVH traversal (extension): auto (default: wide for deep scenes in HBM, near otherwise), near "
                        "(binary, near child first), wide (4-wide quantised records) or reference (the "
                        "reference's far-first order); images differ only where two hits tie at exactly equal t")
    return p


@dataclass
class Params:
    scene: str
    output: str = "tests/test_scene.png"
    camera: object = ""
    addsky: bool = False
    envname: str = ""
    resolution: int = 1280
    samples: int = 512
    bounces: int = 8
    denoise: bool = False
    noparallel: bool = False
    highqualitybvh: bool = False
    envhidden: bool = False
    tentfilter: bool = False
    sampler: int = 1
    clamp: int = 10
    nocaustics: bool = False
    batch: int = 1
    bvhstacksize: int = 128
    seed: int = 0x5EED
    width: int = 0
    height: int = 0
    device: int = 0
    devices: int = 1
    missing: str = "error"
    traversal: str = DEFAULT_TRAVERSAL


def params_from_dict(d: dict) -> Params:
    """Params(params) (src/cli.jl:110-137): unknown sampler names map to path (index 1);
    clamp is stored as Int (InexactError for non-integral values, as in the reference)."""
    sampler = SAMPLER_TYPES.index(d["sampler"]) + 1 if d["sampler"] in SAMPLER_TYPES else 1
    clamp = d["clamp"]
    if float(clamp) != int(clamp):
        raise ValueError(f"InexactError: Int64({clamp}) (Params.clamp is an Int, src/cli.jl:105)")
    kw = dict(d)
    kw["sampler"] = sampler
    kw["clamp"] = int(clamp)
    return Params(**kw)


def parse_cli_args(args) -> Params:
    """parse_cli_args (src/cli.jl:140-147)."""
    ns = _parser().parse_args(list(args))
    return params_from_dict(vars(ns))
