"""bench.py's host-side helpers on the CPU: the SURVEY §8(d) algorithmic bytes, the shading-record
size, and the roofline-record lookup, which must only ever pick a record of the running build and
workload (a record of other code describes other counts)."""
import json
import sys

import pytest

from conftest import ROOT

sys.path.insert(0, str(ROOT))
import bench  # noqa: E402  (no torch, no library at import)


def test_algorithmic_bytes_per_unit():
    c = {"nodes": 10, "instances": 3, "prims": 4, "shades": 2}
    # 32 B per binary pop, 64 B per instance visit, 48 B per triangle test, shade bytes per hit
    assert bench.algorithmic_bytes(c, 240, False) == 32 * 10 + 64 * 3 + 48 * 4 + 240 * 2
    # a wide-record visit is 64 B; quad scenes test 64-B quads
    assert bench.algorithmic_bytes(c, 240, True, wide=True) == 64 * 10 + 64 * 3 + 64 * 4 + 240 * 2


def test_shade_record_bytes_cornellbox(cornell_abi):
    from jtrace import sceneio
    scene = sceneio.load_scene(str(ROOT / "assets" / "scenes" / "cornellbox" / "cornellbox.json"))
    assert bench.shade_record_bytes(scene) == 240  # 64 + 32 + 16 + 80 + 3 x 16


@pytest.mark.parametrize("name", ["cb", "cb_n8", "f2", "b1", "ec"])
def test_committed_records_match_only_their_build(name):
    rec = json.loads((ROOT / "profiles" / "r04_roofline" / f"{name}_final.json").read_text())
    found, src = bench.roofline_record(rec["workload"], rec["kernel"], rec["build"])
    assert found is not None and found["build"] == rec["build"] and src.startswith("profiles/")
    assert bench.roofline_record(rec["workload"], rec["kernel"], "0" * 16) == (None, None)
    assert bench.roofline_record(rec["workload"] + " x", rec["kernel"], rec["build"]) == (None, None)
