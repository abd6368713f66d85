"""The oracle's near-child-first switch (jt_params.traversal, include/jtrace.h) on the CPU: the
same closest hits up to exact-t ties, fewer nodes popped (src/bvh.jl:331-341 is far-first)."""
import numpy as np
import pytest

from conftest import compare_images, make_params


def test_oracle_near_order_matches_reference_order(abi, oracle, cornell_abi):
    ob = oracle.build_bvh(cornell_abi)
    ol = oracle.make_lights(cornell_abi)
    out = {}
    for order in ("reference", "near"):
        p = make_params(abi, resolution=64, samples=2, traversal=order)
        out[order] = oracle.trace(cornell_abi, ob, ol, p, 64, 64, 0, 2)
    r, n = out["reference"], out["near"]
    stats = compare_images(n[0], r[0])
    assert stats["frac_pix_rel_le_1e-3"] >= 0.999, stats
    assert np.array_equal(n[3], r[3])  # hit counts
    assert n[4]["rays"] == r[4]["rays"]
    assert n[4]["nodes"] < r[4]["nodes"], (n[4]["nodes"], r[4]["nodes"])


def test_oracle_wide_matches_binary_orders(abi, oracle, cornell_abi):
    """The wide traversal (JT_TRAVERSAL_WIDE: 4-wide records with conservative quantised boxes)
    finds the same closest hits as the binary near-first order up to exact-t ties, visits fewer
    nodes (one record visit tests up to four boxes), and tests at least as many primitives
    (quantised boxes are never tighter)."""
    ob = oracle.build_bvh(cornell_abi)
    ol = oracle.make_lights(cornell_abi)
    out = {}
    for order in ("near", "wide"):
        p = make_params(abi, resolution=64, samples=2, traversal=order)
        out[order] = oracle.trace(cornell_abi, ob, ol, p, 64, 64, 0, 2)
    n, w = out["near"], out["wide"]
    stats = compare_images(w[0], n[0])
    assert stats["frac_pix_rel_le_1e-3"] >= 0.999, stats
    assert np.array_equal(w[3], n[3])
    assert w[4]["rays"] == n[4]["rays"] and w[4]["light_queries"] == n[4]["light_queries"]
    assert w[4]["nodes"] < n[4]["nodes"], (w[4]["nodes"], n[4]["nodes"])
    assert w[4]["prims"] >= n[4]["prims"]


def test_params_carry_the_traversal_order(abi):
    from jtrace.cli import DEFAULT_TRAVERSAL, Params, parse_cli_args
    # one default for the parser, the dataclass and abi.make_params: auto (resolved by the library)
    assert DEFAULT_TRAVERSAL == "auto"
    assert Params(scene="x").traversal == parse_cli_args(["--scene", "x"]).traversal == DEFAULT_TRAVERSAL
    assert abi.make_params(Params(scene="x"), 0).traversal == 3
    assert make_params(abi).traversal == 1  # the tests' own default: near, restated by the oracle
    assert make_params(abi, traversal="near").traversal == 1
    assert make_params(abi, traversal="reference").traversal == 0
    assert make_params(abi, traversal="wide").traversal == 2
    assert make_params(abi, traversal="auto").traversal == 3
    assert abi.jt_params().traversal == 0  # the C-ABI zero value is the reference's order
    assert abi.jt_params.traversal.offset == 64 and abi.C.sizeof(abi.jt_params) == 72


@pytest.mark.parametrize("name", ["cornellbox", "features2", "bathroom1", "ecosys"])
def test_wide_records_are_conservative(abi, oracle, name):
    """The wide records' quantised child boxes (JT_TRAVERSAL_WIDE, restated in oracle/jt_oracle.c
    w_build from the product's specification) contain every exact child box on every axis, and
    every binary leaf is reached; the bytes loosen the boxes by a bounded factor."""
    from conftest import CORNELL, ROOT
    from jtrace import sceneio
    import warnings
    path = CORNELL if name == "cornellbox" else str(ROOT / "assets" / "scenes" / name / f"{name}.json")
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        sa = abi.SceneABI(sceneio.load_scene(path, missing="drop"))
    bvh = oracle.build_bvh(sa)
    leaves = sum(1 for t in [bvh.struct.tlas] + [bvh.struct.blas[i] for i in range(bvh.struct.nshapes)]
                 for k in range(t.nnodes) if not t.nodes[k].internal)
    c = oracle.wide_check(bvh)
    print(name, c, "binary leaves", leaves)
    assert c["violations"] == 0
    assert c["leaves"] == leaves
    assert 1.0 <= c["volume_ratio"] < 2.0


def test_oracle_rejects_unresolved_auto(abi, oracle, cornell_abi):
    """The oracle restates an explicit order: "auto" (3) is the library's choice by scene mode and
    depth, so a checker must pass the order the library resolved (bench.py's CPU leg, smoke())."""
    p = make_params(abi, resolution=8, samples=1, traversal="auto")
    with pytest.raises(ValueError):
        oracle.trace(cornell_abi, oracle.build_bvh(cornell_abi), oracle.make_lights(cornell_abi), p, 8, 8, 0, 1)


@pytest.mark.parametrize("alt", ["near", "wide"])
def test_near_first_orders_resolve_ties_as_the_reference(abi, oracle, alt):
    """Every closest-hit scene query of a bathroom1 render traced in the reference's order is
    repeated on the same ray in the near-first order (oracle/jt_oracle.c or_order_diff): exact-t
    ties resolve as the reference resolves them (the reversed leaf sequence, take_hit), so no query
    differs by a tie, and the remaining differences — a hit the slab test's rounding lets one order
    find and the other cull — stay below 1e-6 of the queries. Without the tie rule this render has
    141 tie differences in 6.7 M queries (2.1e-5) at 480x270x16 spp; here a smaller frame."""
    import warnings
    from jtrace import sceneio
    from conftest import ROOT
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        sc = sceneio.load_scene(str(ROOT / "assets" / "scenes" / "bathroom1" / "bathroom1.json"), missing="drop")
    sa = abi.SceneABI(sc)
    p = make_params(abi, width=240, height=135, samples=8, traversal="reference")
    d = oracle.order_diff(sa, oracle.build_bvh(sa), oracle.make_lights(sa), p, abi.TRAVERSAL_ORDERS.index(alt),
                          240, 135, 0, 8)
    print(alt, d)
    assert d["queries"] > 500_000
    assert d["tie"] == 0, d
    assert d["alt_only_hit"] == 0 and d["ref_only_hit"] == 0, d
    assert d["alt_closer"] + d["alt_farther"] <= 1e-6 * d["queries"] + 2, d
