"""The product's host BVH builder (jt_build_scene_bvh, C++) against the oracle's independent
restatement of src/bvh.jl (make_bvh / split_middle / split_sah / partition): node-for-node,
byte-for-byte identical, which fixes traversal order and hit tie-breaking."""
import ctypes as C

import numpy as np
import pytest

from jtrace.scene import InstanceData, MaterialData, SceneData, ShapeData, CameraData, identity_frame


def tree_bytes(t):
    nodes = bytes(C.string_at(t.nodes, t.nnodes * 32)) if t.nnodes else b""
    prims = np.ctypeslib.as_array(t.primitives, shape=(t.nprimitives,)).copy() if t.nprimitives else np.zeros(0)
    return nodes, prims


def assert_same(a, b):
    assert a.tlas.nnodes == b.tlas.nnodes
    na, pa = tree_bytes(a.tlas)
    nb, pb = tree_bytes(b.tlas)
    assert na == nb and np.array_equal(pa, pb)
    assert a.nshapes == b.nshapes
    for k in range(a.nshapes):
        na, pa = tree_bytes(a.blas[k])
        nb, pb = tree_bytes(b.blas[k])
        assert na == nb and np.array_equal(pa, pb), k


def test_cornellbox_bvh_shape_and_identity(abi, lib, oracle, cornell_abi):
    from jtrace import trace
    b = trace.make_scene_bvh(cornell_abi, False, lib)
    ob = oracle.build_bvh(cornell_abi)  # keep the owners alive while comparing
    assert b.struct.tlas.nnodes == 5  # TLAS 5 nodes, BLAS [1,1,1,1,1,1,7,7]
    assert [b.struct.blas[k].nnodes for k in range(8)] == [1, 1, 1, 1, 1, 1, 7, 7]
    assert_same(b.struct, ob.struct)


def random_scene(rng, nshapes=3, ntris=(1, 400), quads=False, degenerate=False, ninst=7):
    sc = SceneData()
    sc.cameras.append(CameraData(frame=identity_frame()))
    sc.materials.append(MaterialData(color=np.ones(3, np.float32)))
    for s in range(nshapes):
        n = int(rng.integers(ntris[0], ntris[1] + 1))
        k = 4 if quads else 3
        if degenerate:
            pos = np.repeat(rng.normal(size=(1, 3)), n * k, axis=0).astype(np.float32)
        else:
            centers = rng.normal(size=(n, 1, 3)) * 5
            pos = (centers + rng.normal(size=(n, k, 3)) * 0.3).reshape(-1, 3).astype(np.float32)
        idx = np.arange(n * k, dtype=np.int32).reshape(n, k)
        if quads:
            idx[::3, 3] = idx[::3, 2]  # some triangles stored as degenerate quads
            sc.shapes.append(ShapeData(positions=pos, quads=idx))
        else:
            sc.shapes.append(ShapeData(positions=pos, triangles=idx))
    for i in range(ninst):
        a = rng.normal(size=(3, 3)).astype(np.float32)
        o = (rng.normal(size=3) * 10).astype(np.float32)
        sc.instances.append(InstanceData(frame=np.concatenate([a.reshape(-1), o]).astype(np.float32),
                                         shape=int(rng.integers(0, nshapes)), material=0))
    return sc


@pytest.mark.parametrize("seed", range(6))
@pytest.mark.parametrize("hq", [False, True])
def test_random_scenes_identical(abi, lib, oracle, seed, hq):
    from jtrace import trace
    rng = np.random.default_rng(seed)
    sc = random_scene(rng, quads=seed % 2 == 1, degenerate=seed == 4, ntris=(1, 300 if hq else 3000))
    sa = abi.SceneABI(sc)
    pb, ob = trace.make_scene_bvh(sa, hq, lib), oracle.build_bvh(sa, hq)
    assert_same(pb.struct, ob.struct)


def test_bvh_invariants(abi, lib):
    from jtrace import trace
    rng = np.random.default_rng(11)
    sc = random_scene(rng, nshapes=1, ntris=(5000, 5000), ninst=1)
    b = trace.make_scene_bvh(abi.SceneABI(sc), False, lib)
    nodes, prims = b.tree(0)
    assert sorted(prims.tolist()) == list(range(5000))  # a permutation
    pos = sc.shapes[0].positions.reshape(-1, 3, 3)
    for n in nodes:
        if n["internal"]:
            for c in (n["start"], n["start"] + 1):
                assert np.all(nodes[c]["bmin"] >= n["bmin"]) and np.all(nodes[c]["bmax"] <= n["bmax"])
        else:
            assert 0 <= n["num"] <= 4  # BVH_MAX_PRIMS (src/bvh.jl:32)
            tri = pos[prims[n["start"]:n["start"] + n["num"]]]
            assert np.all(tri.min(axis=(0, 1)) >= n["bmin"]) and np.all(tri.max(axis=(0, 1)) <= n["bmax"])
