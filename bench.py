"""bench.py — BASELINE.json's headline metric on MI355X: Mrays/s (+ wall-clock render time),
cornellbox, path sampler, 1280x720 x 256 spp.

A step = one full render of that workload (every pixel x every sample, bounces=8, clamp=10,
seed 0x5EED) with the scene already resident in HBM: each rank traces its contiguous
sample range [r*S/N, (r+1)*S/N) of all pixels (no data-path collective), then for N > 1 one
RCCL reduce (sum of sample-weighted running means) gathers the image on rank 0 — the only
exchange the path has, pipelined so that a step's reduce runs during the next
step's launch (the last one finishes inside the timed region). value = closest-hit scene queries
of all ranks / time.

    python bench.py [--gpus N --steps K --warmup W]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N ...
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT / "julia-raytracer_amd"))
from jtrace.cli import DEFAULT_TRAVERSAL  # noqa: E402  (pure Python: no torch, no library)

METRIC_BASE = "Mrays/s + wall-clock render time"  # BASELINE.json metric; the workload is appended
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)
SIGNATURES = ROOT / "profiles" / "image_signatures.json"  # one-GPU image fingerprints per workload
# run-time options that change which samples are drawn (include/jtrace.h), hence the fingerprint;
# the batch and the stream count only change the summation order (last bits), which the
# fingerprint's tolerance absorbs, so every --batch checks against the same fingerprint
RESULT_OPTIONS = ("env_alias",)


def metric_name(scene: str, sampler: str, W: int, H: int, S: int) -> str:
    """BASELINE.json's metric string for this workload ("..., cornellbox 1280×720×256spp"); the
    sampler is named when it is not the path sampler the configs 2-5 use."""
    return f"{METRIC_BASE}, {scene} {W}×{H}×{S}spp" + ("" if sampler == "path" else f" ({sampler} sampler)")


def algorithmic_bytes(c: dict, shade_bytes: int, quad_scene: bool, wide: bool = False) -> int:
    """Algorithmic bytes of the trace launches: 32 B per BVH node pop (64 B
    per wide-record visit, which tests up to four child boxes), 64 B per instance visit, 48 B per
    triangle test (64 B per quad test), shade_bytes per surface hit."""
    return ((64 if wide else 32) * c["nodes"] + 64 * c["instances"] + (64 if quad_scene else 48) * c["prims"]
            + shade_bytes * c["shades"])


def shade_record_bytes(scene) -> int:
    """Bytes fetched per shaded hit: instance shade record 64 + shape 32 + element ids 16 +
    material 80 + positions 16/vertex (+ normals 16/vertex, texcoords 8/vertex, 4 texels per
    texture lookup) — maximum over the scene's shapes (cornellbox: 240)."""
    best = 0
    for s in scene.shapes:
        nv = 4 if len(s.quads) else 3
        b = 64 + 32 + 16 + 80 + 16 * nv
        if len(s.normals):
            b += 16 * nv
        if len(s.texcoords):
            b += 8 * nv
        best = max(best, b)
    return best


def library_build_hash(lib) -> str:
    """The source hash embedded in the loaded library (jt_version: "..., source <hash>)")."""
    import re
    m = re.search(r"source ([0-9a-f]{16}|unknown)\)", lib.jt_version().decode())
    return m.group(1) if m else "unknown"


def roofline_record(workload: str, kernel: str, build: str):
    """The committed roofline record (profiles/*_roofline/*.json, written on the GPU box by
    scripts/roofline.py from rocprofv3 kernel-trace + PMC passes of this same bench command) for
    this workload, kernel instance and build (scripts/roofline.py source_hash), newest round
    first; (None, None) when none matches. A record of another build is never used: its counts
    describe other code."""
    for f in sorted((ROOT / "profiles").glob("*_roofline/*.json"), reverse=True):
        try:
            d = json.loads(f.read_text())
        except (OSError, ValueError):
            continue
        if d.get("workload") == workload and d.get("kernel", "").replace(" ", "") == kernel.replace(" ", "") \
                and d.get("build") == build:
            return d, str(f.relative_to(ROOT))
    return None, None


def cpu_baseline(scene_abi, params, width, height, nthreads, spp=2, high_quality=False):
    """Oracle (C restatement, oracle/jt_oracle.c) on host cores: bounded sample of the same
    workload — all pixels, samples [0, spp)."""
    sys.path.insert(0, str(ROOT / "oracle"))
    from jtrace import abi
    from oracle import Oracle  # the checker, timed as the CPU baseline only
    orc = Oracle(abi)
    ob = orc.build_bvh(scene_abi, high_quality)
    ol = orc.make_lights(scene_abi)
    t0 = time.perf_counter()
    _, _, _, _, cnt = orc.trace(scene_abi, ob, ol, params, width, height, 0, spp, nthreads=nthreads)
    dt = time.perf_counter() - t0
    return {"value": cnt["rays"] / dt / 1e6, "unit": "Mrays/s", "cores": nthreads, "kind": "port",
            "sample": f"{width}x{height} x {spp} spp (samples 0..{spp - 1}) of the bench workload, "
                      f"{cnt['rays']} rays in {dt:.2f} s",
            "rays": int(cnt["rays"]), "seconds": round(dt, 3)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)  # ~1.8 s of GPU work at N=1
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--width", type=int, default=1280)
    ap.add_argument("--height", type=int, default=720)
    ap.add_argument("--spp", type=int, default=256)
    ap.add_argument("--sampler", default="path")
    ap.add_argument("--scene", default=str(ROOT / "assets" / "scenes" / "cornellbox" / "cornellbox.json"))
    ap.add_argument("--traversal", choices=["reference", "near", "wide", "auto"], default=DEFAULT_TRAVERSAL,
                    help="BVH child order (include/jtrace.h jt_traversal): auto (the default: wide records for "
                         "deep HBM-mode scenes, near child first otherwise), near, wide, or the reference's "
                         "far-first order (src/bvh.jl:331-341)")
    ap.add_argument("--no-reference-order", action="store_true",
                    help="skip the reference-order comparison line (rank 0, N=1, --traversal near)")
    ap.add_argument("--batch", type=int, default=0,
                    help="trace_samples batch B (the reference's --batch, src/cli.jl:78-81; its default is 1): a step "
                         "makes one call per B samples, as Jtrace.main does (src/jtrace.jl:83); 0 (the default): "
                         "the rank's whole sample share in one call")
    ap.add_argument("--highqualitybvh", action="store_true",
                    help="the reference's SAH build (--highqualitybvh, src/bvh.jl:218-274) instead of split_middle")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-threads", type=int, default=16)
    ap.add_argument("--cpu-spp", type=int, default=128)
    ap.add_argument("--tile-groups", type=int, default=0,
                    help="N > 1: split the tiles into G interleaved groups x N/G sample ranges (0 or 1: the pure "
                         "sample split)")
    ap.add_argument("--as-rank-of", type=int, default=0,
                    help="N=1: trace rank 0's share of an N-rank run (per-GPU rate and roofline of that share)")
    ap.add_argument("--write-signature", action="store_true",
                    help="N=1: record this workload's image fingerprint in profiles/image_signatures.json (with --as-rank-of: rank 0's share image)")
    ap.add_argument("--print-workload", action="store_true",
                    help="print the workload key of this run's roofline record (scripts/gpu_measure.sh) and exit")
    ap.add_argument("--opt", action="append", default=[], metavar="NAME=VALUE",
                    help="a library run-time option (jt_set_option, include/jtrace.h) for A/B runs; repeatable")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    # rehearsal knobs (not used by the driver): JT_BENCH_BACKEND=gloo reduces through host
    # memory, JT_BENCH_DEVICE pins every rank to one GPU — N ranks on a one-GPU box
    backend = os.environ.get("JT_BENCH_BACKEND", "nccl")
    dev = int(os.environ.get("JT_BENCH_DEVICE", str(local_rank)))
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")

    import torch
    torch.cuda.set_device(dev)
    dist = None
    if world > 1:
        import torch.distributed as dist
        if backend == "nccl":  # RCCL over xGMI
            dist.init_process_group("nccl", device_id=torch.device("cuda", dev))
        else:
            dist.init_process_group(backend)

    from jtrace import abi, sceneio, trace
    from jtrace.cli import Params
    lib = abi.load_library()
    for o in args.opt:  # A/B runs only: the driver's bench line never sets one
        k, _, v = o.partition("=")
        abi.set_option(lib, k, v)
    # time to first pixel, by stage (the reference's timers, src/jtrace.jl:49-65): scene load,
    # BVH build, lights, device upload (jt_create)
    t_0 = time.perf_counter()
    scene = sceneio.load_scene(args.scene, missing="drop")  # configs 3-5: the checkout lacks a few files
    sa = abi.SceneABI(scene)
    t_load = time.perf_counter()
    from jtrace.parallel import (PipelinedReduce, compare_signature, image_signature, load_signature,
                                 save_signature, split_plan)
    S = args.spp
    # this rank's share: 1/G of the 8x8 tiles (G = --tile-groups) x a contiguous
    # 1/(N/G) of the samples; G = 1 is the pure sample split
    groups = args.tile_groups if args.tile_groups > 0 else 1
    # --as-rank-of N (N=1 runs only): trace rank 0's share of an N-rank run, to measure it on one GPU
    plan_world, plan_rank = (args.as_rank_of, 0) if (args.as_rank_of and world == 1) else (world, rank)
    share, s0, s1 = split_plan(plan_world, plan_rank, S, groups)
    # the rank's trace_samples batch is its own share of the samples (one call per step; the
    # library sizes its sample streams by it, jt_get_streams), or --batch B: one call per B samples
    batch = args.batch if args.batch > 0 else s1 - s0
    params = Params(scene=args.scene, samples=S, sampler=2 if args.sampler == "naive" else 1,
                    width=args.width, height=args.height, device=dev, batch=batch, traversal=args.traversal)
    jp = abi.make_params(params, 0)
    bvh = trace.make_scene_bvh(sa, args.highqualitybvh, lib)
    t_bvh = time.perf_counter()
    lights = trace.make_trace_lights(sa, lib)
    t_lights = time.perf_counter()
    if share is not None:  # a tile share: the context is created with the option
        abi.set_option(lib, "tile_share", share)
    state = trace.make_trace_state(sa, bvh, lights, jp, lib)
    if share is not None:
        abi.set_option(lib, "tile_share", None)
    t_create = time.perf_counter()
    ttfp = {"load_s": round(t_load - t_0, 3), "bvh_s": round(t_bvh - t_load, 3),
            "lights_s": round(t_lights - t_bvh, 3), "upload_s": round(t_create - t_lights, 3),
            "total_s": round(t_create - t_0, 3)}
    W, H = state.width, state.height

    traversal = state.traversal  # "auto" resolved by the library: wide for deep HBM-mode scenes, near otherwise
    workload = f"{Path(args.scene).stem} {args.sampler} {W}x{H} " + \
        (f"{s1 - s0} samples/launch" if args.batch <= 0 else f"{s1 - s0} samples in calls of {batch}") + \
        (f" tiles 1/{groups}" if groups > 1 else "") + \
        ("" if traversal == "reference" else f" traversal={traversal}") + \
        (" bvh=sah" if args.highqualitybvh else "")
    if args.print_workload:
        print(workload, flush=True)
        state.close()
        return
    img_t = None
    if world > 1:
        buf = state.device_buffers()

        class _CAI:  # view the library's running-mean buffer as a torch tensor (no copy)
            __cuda_array_interface__ = {"shape": (H * W * 4,), "typestr": "<f4",
                                        "data": (buf.image, False), "version": 3}
        img_t = torch.as_tensor(_CAI(), device=f"cuda:{dev}")

    reduced = [None]  # rank 0, N > 1: the last step's reduced image (the image check below)
    # N > 1: the path's one exchange, the sum of sample-weighted shard means onto rank 0 (RCCL),
    # pipelined (jtrace.parallel.PipelinedReduce): a step snapshots its weighted shard image into
    # one of two buffers and starts the reduce asynchronously, so it runs during the next step's
    # launch; the snapshot reads the library's buffer on torch's stream, so it is finished before
    # the next step's jt_reset clears that buffer on the library's stream; drain() ends the last
    # reduce inside the timed region
    red = None
    if world > 1:
        red = PipelinedReduce(H * W * 4, s1 - s0, S, dist, device=img_t.device if backend == "nccl" else "cpu",
                              sync=torch.cuda.current_stream().synchronize)

    full_range = s0 == 0 and s1 == S

    def step():
        state.reset()
        if args.batch <= 0:
            state.trace_range(s0, s1)  # one call: returns when the launch has finished (HIP event sync)
        elif full_range:  # Jtrace.main's loop (src/jtrace.jl:83-106): trace_samples until state.samples == S
            for _ in range(-(-S // batch)):
                state.trace_samples()
        else:  # a rank's share in calls of B samples
            for a in range(s0, s1, batch):
                state.trace_range(a, min(a + batch, s1))
        if red is not None:
            red.submit(img_t if backend == "nccl" else img_t.cpu())
        return state.counters()

    def drain():
        out = red.drain() if red is not None else None
        torch.cuda.synchronize()
        if out is not None:
            reduced[0] = out

    for _ in range(args.warmup):
        step()
    drain()
    # counting pass: the same step with every traversal counter on (level 1); the timed steps
    # run the production kernel (level 0: paths/rays/light queries). The counts are a
    # deterministic function of (seed, samples, BVH); the ray count cross-checks them.
    state.set_counters(1)
    full = step()
    drain()
    state.set_counters(0)
    desc = state.describe()
    kernel = desc.split()[0].split("=", 1)[1]
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    rays = 0
    kernel_ms = 0.0
    agg = {k: 0 for k in ("paths", "rays", "light_queries", "launches")}
    for _ in range(args.steps):
        c = step()
        if c["rays"] != full["rays"] or c["light_queries"] != full["light_queries"]:
            raise SystemExit(f"non-deterministic ray count: {c} vs counting pass {full}")
        for k in agg:
            agg[k] += c[k]
        kernel_ms += c["kernel_ms"]
        rays += c["rays"]
    drain()
    if dist is not None:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    t = torch.tensor([elapsed, float(rays)], dtype=torch.float64, device=f"cuda:{dev}" if backend == "nccl" else "cpu")
    if dist is not None:
        tmax = t.clone()
        dist.all_reduce(tmax[0:1], op=dist.ReduceOp.MAX)
        dist.all_reduce(t[1:2], op=dist.ReduceOp.SUM)
        elapsed, total_rays = float(tmax[0]), float(t[1])
    else:
        total_rays = float(rays)

    # Image check (rank 0, every N): block means of the final image — the RCCL-reduced one for
    # N > 1 — against the one-GPU signature committed for this workload (profiles/image_signatures.json,
    # jtrace/parallel.py): a wrong shard split, weight or reduce fails the run loudly
    # (--as-rank-of N: rank 0's share image, against the signature of that share)
    image_check = None
    partial = world == 1 and plan_world > 1  # --as-rank-of: one rank's share only, not the image
    if rank == 0:
        img_final = (reduced[0].detach().cpu().numpy().reshape(H, W, 4) if world > 1 else state.get_image())
        sig = image_signature(img_final)
        sig_key = f"{Path(args.scene).stem} {args.sampler} {W}x{H}x{S}spp traversal={traversal}" + \
            ("".join(f" {o}" for o in sorted(args.opt) if o.split("=")[0] in RESULT_OPTIONS)) + \
            (" bvh=sah" if args.highqualitybvh else "") + \
            (f" rank 0 of {plan_world}" + (f" tiles 1/{groups}" if groups > 1 else "") if partial else "")
        ref_sig = load_signature(SIGNATURES, sig_key)
        if args.write_signature and world == 1:
            save_signature(SIGNATURES, sig_key, sig, "one-GPU bench.py --as-rank-of run, block means of rank 0's share image"
                           if partial else "one-GPU bench.py run, block means of the final image")
            image_check = {"key": sig_key, "written": str(SIGNATURES.relative_to(ROOT))}
        elif ref_sig is not None:
            image_check = {"key": sig_key, **compare_signature(sig, ref_sig), "ranks_reduced": world}
            if not image_check["ok"]:
                raise SystemExit(f"image check failed for {sig_key}: {image_check}")
        else:
            image_check = {"key": sig_key, "ok": None, "why": "no committed signature for this workload"}

    # Reference-order leg (rank 0, N=1): the same workload with the reference's far-child-first
    # order (src/bvh.jl:331-341, SURVEY Appendix B item 9: performance only), timed the same way,
    # and the fraction of pixels whose final running mean differs from the near-first image (only
    # hits the slab test's rounding lets one order find and the other cull; exact-t ties re-run in
    # the reference's order)
    ref_order = None
    if rank == 0 and world == 1 and not partial and args.traversal != "reference" and not args.no_reference_order \
            and args.batch <= 0:
        img_near = state.get_image()
        rp = abi.make_params(Params(scene=args.scene, samples=args.spp, sampler=2 if args.sampler == "naive" else 1,
                                    width=args.width, height=args.height, device=dev, batch=args.spp,
                                    traversal="reference"), 0)
        rst = trace.make_trace_state(sa, bvh, lights, rp, lib)
        rst.set_counters(1)
        rst.trace_range(s0, s1)
        rfull = rst.counters()
        rst.set_counters(0)
        for _ in range(args.warmup):
            rst.reset()
            rst.trace_range(s0, s1)
        torch.cuda.synchronize()
        r0 = time.perf_counter()
        rrays = 0
        for _ in range(args.steps):
            rst.reset()
            rst.trace_range(s0, s1)
            rrays += rst.counters()["rays"]
        torch.cuda.synchronize()
        relapsed = time.perf_counter() - r0
        img_ref = rst.get_image()
        rst.close()
        ref_order = {"traversal": "reference", "value": round(rrays / relapsed / 1e6, 2),
                     "ms_per_step": round(relapsed / args.steps * 1e3, 3),
                     "speedup_of_near": round((total_rays / elapsed) / (rrays / relapsed), 4),
                     "pixels_differing_from_near": float(np.mean(np.any(img_ref != img_near, axis=-1))),
                     "per_ray": {k: round(rfull[k] / max(1, rfull["rays"]), 3)
                                 for k in ("nodes", "instances", "prims", "shades", "light_queries")}}

    # CPU baseline leg (rank 0, N=1): the oracle on host cores over samples [0, cpu_spp) of this
    # workload; the GPU then re-traces exactly those samples so the two ray counts — hence the
    # two cameras and framings — are checked to agree (a libm ulp may flip a rare path: <= 0.1 %)
    cpu = None
    if rank == 0 and not args.no_cpu_baseline and world == 1 and not partial:
        # the oracle runs the order the GPU resolved "auto" to (it has no LDS/HBM mode to choose by)
        jp_cpu = type(jp).from_buffer_copy(jp)
        jp_cpu.traversal = abi.TRAVERSAL_ORDERS.index(traversal)
        cpu = cpu_baseline(sa, jp_cpu, W, H, args.cpu_threads, args.cpu_spp, args.highqualitybvh)
        state.reset()
        state.trace_range(0, args.cpu_spp)
        g = state.counters()
        cpu["gpu_rays_same_samples"] = int(g["rays"])
        cpu["rays_per_sample"] = round(cpu["rays"] / (W * H * args.cpu_spp), 6)
        cpu["gpu_rays_per_sample"] = round(g["rays"] / (W * H * args.cpu_spp), 6)
        if abs(g["rays"] - cpu["rays"]) > 1e-3 * cpu["rays"]:
            raise SystemExit(f"cpu_baseline traced a different workload: {cpu['rays']} rays on the CPU vs "
                             f"{g['rays']} on the GPU over the same samples")

    if rank == 0:
        name = Path(args.scene).stem
        value = total_rays / elapsed / 1e6
        ms_per_step = elapsed / args.steps * 1e3
        launches = max(1, agg["launches"])
        avg_launch_s = kernel_ms / launches / 1e3
        per_launch = {k: v / max(1, full["launches"]) for k, v in full.items()}  # one step's launches
        logical = algorithmic_bytes(per_launch, shade_record_bytes(scene),
                                    any(len(s.quads) for s in scene.shapes), traversal == "wide")
        sys.path.insert(0, str(ROOT / "scripts"))
        from roofline import VMEM_MIX_PEAK_GIPS
        # the source hash the Makefile embedded in the library that ran (jt_version), not a hash of
        # this tree: no compiler is invoked at run time (under a PMC profiler a child process that
        # execs would be refused), and a record can only match the binary it describes
        build = library_build_hash(lib)
        rec, rec_src = roofline_record(workload, kernel, build)
        # The roof that binds, from the PMC counts of this kernel on this workload and build
        # (committed record) over THIS run's launch time (HIP events):
        #  - LDS mode (small scenes: the scene is in LDS): VALU issue of partly idle waves —
        #    achieved = useful FP32 lane-operations per second, peak = the CUs' FP32 lane rate;
        #  - HBM mode (node / primitive records L2-resident): the vector-memory return path (TD) —
        #    achieved = vector-memory read wave-instructions per second, peak = the measured
        #    gather ceiling for the traversal's own node records (scripts/td_mix_bench.hip,
        #    profiles/r04_tdmix/: 64-B wide records 40.6, 16-B binary rows 34.7 G wave-instr/s);
        #    td_unstalled_frac (TD busy and not waiting on the cache) beside it agrees with frac.
        # HBM itself (measured traffic / 8 TB/s) is reported beside it as hbm_frac.
        lds_mode = "mode=lds" in desc
        roof = {"bound": "valu" if lds_mode else "vmem/TD", "achieved": None, "peak": None,
                "unit": "G lane-ops/s" if lds_mode else "G wave-instr/s", "frac": None, "traffic": None,
                "hbm_achieved_gbs": None, "hbm_peak_gbs": HBM_PEAK_GBS, "hbm_frac": None,
                "source": rec_src, "build": build, "kernel": kernel, "launch": desc,
                "avg_launch_ms": round(avg_launch_s * 1e3, 3), "binding": None}
        if rec:
            d = rec["derived"]
            if lds_mode and "valu_lane_ops" in d:
                achieved, peak = d["valu_lane_ops"] / avg_launch_s / 1e9, d["valu_peak_gops"]
            elif not lds_mode and "vmem_rd_per_launch" in d:
                achieved, peak = d["vmem_rd_per_launch"] / avg_launch_s / 1e9, VMEM_MIX_PEAK_GIPS[traversal]
            else:
                achieved = peak = None
            if achieved is not None:
                roof.update(achieved=round(achieved, 2), peak=round(peak, 2), frac=round(achieved / peak, 5))
            traffic = d["traffic_bytes"]  # measured HBM bytes per launch (PMC, gfx950-corrected)
            roof.update(traffic=int(traffic), hbm_achieved_gbs=round(traffic / avg_launch_s / 1e9, 1),
                        hbm_frac=round(traffic / avg_launch_s / 1e9 / HBM_PEAK_GBS, 5))
            roof["binding"] = {k: d[k] for k in ("valu_issue_frac", "lane_util", "fp32_lane_frac", "td_busy_frac",
                                                 "td_unstalled_frac", "td_tc_stall_frac_of_busy", "l2_hit_rate", "l1_hit_rate",
                                                 "l1_accesses_per_vmem_rd", "l1_misses_per_vmem_rd",
                                                 "vmem_mix_frac", "vmem_mix_frac_resident", "clock_ghz") if k in d}
            roof["binding"]["write_bytes_per_launch"] = int(d["write_bytes"])
            roof["binding"]["profiled_launch_ms"] = round(rec["duration_ns"] / 1e6, 3)
        alg_gbs = logical / avg_launch_s / 1e9
        roof.update({
                "algorithmic": {"bytes_per_launch": int(logical),
                                "bytes_per_ray": round(logical / max(1.0, per_launch["rays"]), 1),
                                "gbs": round(alg_gbs, 1),
                                "note": "SURVEY §8(d) logical bytes (node/instance/primitive/shading records) "
                                        "over the launch time; served from LDS (small scenes) or L2, not HBM"
                                        + (f": {alg_gbs / 1e3:.1f} TB/s exceeds the 8 TB/s HBM peak, so HBM is not "
                                           "this kernel's roof" if alg_gbs > HBM_PEAK_GBS else "")},
                # traversal work per closest-hit query, from the counting pass
                "per_ray": {k: round(per_launch[k] / max(1.0, per_launch["rays"]), 3)
                            for k in ("nodes", "instances", "prims", "shades", "light_queries")}})
        line = {
            "metric": metric_name(name, args.sampler, W, H, S) + (" (--highqualitybvh)" if args.highqualitybvh else ""),
            "value": round(value, 2), "unit": "Mrays/s",
            "n_gpus": world, "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(ms_per_step, 3),
            "higher_is_better": True, "scaling": "strong", "vs_baseline": None, "dtype": "f32",
            "data": f"scene: the reference's own {name} (assets/scenes/{name}), seed 0x5EED"
                    + (f"; {'; '.join(scene.notes)}" if scene.notes else ""),
            "config": {"workload": f"{name} {args.sampler} {W}x{H}x{S}spp", "scene": name,
                       "split": {"tile_groups": groups, "sample_ranges": world // groups,
                                 "rank0_share": {"tiles": share or "all", "samples": [s0, s1]}},
                       "sampler": args.sampler, "width": W, "height": H, "spp": S, "bounces": 8,
                       "batch": batch, "calls_per_step": -(-(s1 - s0) // batch),
                       "traversal": traversal, "traversal_requested": args.traversal,
                       "bvh": "sah" if args.highqualitybvh else "middle",
                       "parallelism": f"{groups} tile groups x {world // groups} sample ranges + RCCL reduce"},
            "render_s": round(ms_per_step / 1e3, 4),
            "msamples_per_s": round((agg["paths"] if partial else W * H * S * args.steps) / elapsed / 1e6, 2),
            "mlight_queries_per_s": round(agg["light_queries"] * world / elapsed / 1e6, 2),
            "time_to_first_pixel_s": ttfp,
            "options": dict(o.partition("=")[::2] for o in args.opt) or None,
            "roofline": roof,
            "reference_order": ref_order,
            "image_check": image_check,
            "cpu_baseline": cpu,
        }
        print(json.dumps(line), flush=True)
    state.close()
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
