"""N > 1 path on the CPU: world_size-2 gloo. Each rank renders its sample shard (the oracle
stands in for the GPU kernel, which is bit-identical to it) and the shards are combined with
the same reduce the bench runs over RCCL (jtrace.parallel.reduce_running_means, and its pipelined
form jtrace.parallel.PipelinedReduce)."""
import os
import sys

import numpy as np
import pytest

torch = pytest.importorskip("torch")
import torch.distributed as dist  # noqa: E402
import torch.multiprocessing as mp  # noqa: E402

from conftest import CORNELL, ROOT, make_params  # noqa: E402

RES, SPP = 24, 6


def _worker(rank, world, port, out_path):
    sys.path.insert(0, str(ROOT / "julia-raytracer_amd"))
    sys.path.insert(0, str(ROOT / "oracle"))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from jtrace import abi, sceneio
    from jtrace.parallel import reduce_running_means, shard_range
    from oracle import Oracle
    orc = Oracle(abi)
    sa = abi.SceneABI(sceneio.load_scene(CORNELL))
    p = make_params(abi, resolution=RES, samples=SPP)
    s0, s1 = shard_range(SPP, world, rank)
    img = orc.trace(sa, orc.build_bvh(sa), orc.make_lights(sa), p, RES, RES, s0, s1, first=s0, nthreads=2)[0]
    out = reduce_running_means(torch.from_numpy(img), s1 - s0, SPP, dist, dst=0)
    # the bench's pipelined form: three steps through two buffers, the last one the real image
    # (earlier steps' reduces must not leak into it, and a buffer is reused only once reduced)
    from jtrace.parallel import PipelinedReduce
    red = PipelinedReduce(img.size, s1 - s0, SPP, dist)
    src = torch.empty(img.size, dtype=torch.float32)
    for scale in (3.0, 7.0, 1.0):
        src.copy_(torch.from_numpy(img).reshape(-1) * scale)
        red.submit(src)
        src.fill_(-1.0)  # the caller overwrites its buffer after submit (the next jt_reset)
    piped = red.drain()
    if rank == 0:
        np.save(out_path, out.numpy())
        np.save(str(out_path) + ".piped.npy", piped.reshape(out.shape).numpy())
    dist.barrier()
    dist.destroy_process_group()


def test_two_rank_shards_equal_single_render(abi, oracle, cornell_abi, tmp_path):
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    out = tmp_path / "img.npy"
    mp.spawn(_worker, args=(2, port, str(out)), nprocs=2, join=True)
    combined = np.load(out)
    np.testing.assert_array_equal(np.load(str(out) + ".piped.npy"), combined)
    p = make_params(abi, resolution=RES, samples=SPP)
    single = oracle.trace(cornell_abi, oracle.build_bvh(cornell_abi), oracle.make_lights(cornell_abi), p, RES, RES,
                          0, SPP)[0]
    np.testing.assert_allclose(combined, single, rtol=1e-5, atol=1e-6)
    # the bench's reduced-image check (jtrace/parallel.py) accepts the reduce and rejects a
    # missing shard or a wrong weight
    from jtrace.parallel import compare_signature, image_signature
    ref = image_signature(single, block=8)
    assert compare_signature(image_signature(combined, block=8), ref)["ok"]
    half = oracle.trace(cornell_abi, oracle.build_bvh(cornell_abi), oracle.make_lights(cornell_abi), p, RES, RES,
                        0, SPP // 2)[0]
    assert not compare_signature(image_signature(half * 0.5, block=8), ref)["ok"]  # one shard, weight n_r / S
    assert not compare_signature(image_signature(combined * 1.01, block=8), ref)["ok"]


def test_shard_ranges_cover_all_samples():
    from jtrace.parallel import shard_range
    for S in (1, 7, 256):
        for N in (1, 2, 3, 8):
            r = [shard_range(S, N, k) for k in range(N)]
            assert r[0][0] == 0 and r[-1][1] == S and all(r[k][1] == r[k + 1][0] for k in range(N - 1))


def test_split_plans_partition_every_pixel_sample():
    """bench.py's hybrid split (jtrace.parallel.split_plan): G interleaved tile groups x N/G
    contiguous sample ranges. Every (tile, sample) is traced by exactly one rank, and the ranks
    covering a tile partition [0, S), so one sample-weighted reduce combines any plan."""
    from jtrace.parallel import split_plan
    tiles, S = 37, 256
    for N in (1, 2, 4, 8):
        G = 1
        while G <= N:
            cover = np.zeros((tiles, S), int)
            for r in range(N):
                share, s0, s1 = split_plan(N, r, S, G)
                k, o = (1, 0) if share is None else map(int, share.split(","))
                cover[o::k, s0:s1] += 1
            assert (cover == 1).all(), (N, G)
            G *= 2
    with pytest.raises(ValueError):
        split_plan(8, 0, S, 3)
