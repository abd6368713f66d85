"""The CLI counterpart of Jtrace.main (src/jtrace.jl:31-118) end to end on the GPU: stage
banners, per-batch progress lines and the saved PNG."""
import numpy as np
import pytest

from conftest import CORNELL

pytestmark = pytest.mark.gpu


def test_main_renders_png(gpu, tmp_path):
    from PIL import Image
    from jtrace import main
    out = tmp_path / "cb.png"
    lines = []
    res = main.run(main.parse_cli_args(["--scene", CORNELL, "--resolution", "64", "--samples", "4",
                                        "--batch", "2", "--output", str(out)]), out=lines.append)
    assert lines[0].startswith("loading scene") and lines[-1].startswith("total time")
    assert sum(1 for s in lines if s.startswith("sample ")) == 2
    assert any(s.startswith("rendered in") for s in lines)
    img = np.asarray(Image.open(out))
    assert img.shape == (64, 64, 4) and img[..., :3].mean() > 5
    assert res["counters"]["paths"] == 64 * 64 * 4
