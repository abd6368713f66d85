"""The oracle's restatement of the library's env_alias option (Vose alias tables for environment
lights; SURVEY §8(f) rank 3, oracle/jt_oracle.c "alias tables"): the table must hold exactly the
pmf the reference's sample_discrete draws from (p_i = cdf[i] - cdf[i-1], src/sampling.jl:33-56),
so the option changes which texel a random number picks, never how often a texel is picked.
The HIP path is checked against this restatement in tests/test_gpu_alias.py."""
import numpy as np
import pytest

from test_gpu_scenes import scene_abi


def table_pmf(keep, other):
    """The pmf an alias table draws: column c (probability 1/n) keeps c with keep[c], else other[c]."""
    n = len(keep)
    p = keep.astype(np.float64).copy()
    np.add.at(p, other, 1.0 - keep.astype(np.float64))
    return p / n


def check_table(oracle, cdf):
    keep, other = oracle.alias_table(cdf)
    assert np.all((keep >= 0) & (keep <= 1)) and np.all((other >= 0) & (other < len(cdf)))
    pmf = np.diff(np.concatenate([[0.0], cdf.astype(np.float64)]))
    pmf = np.maximum(pmf, 0) / pmf.clip(0).sum()
    got = table_pmf(keep, other)
    # the keep probabilities are rounded to float once each (2^-24 relative per column); a texel
    # that collects the leftovers of several columns sums their roundings
    np.testing.assert_allclose(got, pmf, rtol=2e-6, atol=8 * 2.0 ** -24 / len(cdf))
    # a zero-probability texel is never drawn: its column always hands over, nobody hands to it
    zero = pmf == 0
    assert np.all(keep[zero] == 0) or not zero.any()
    assert not np.isin(other[keep < 1], np.nonzero(zero)[0]).any()
    return keep, other


@pytest.mark.parametrize("seed", [0, 1, 2])
def test_alias_table_holds_the_cdf_pmf(oracle, seed):
    rng = np.random.default_rng(seed)
    w = rng.random(4096) ** 4
    w[rng.random(4096) < 0.2] = 0  # texels of zero weight (black sky rows, sin(theta) = 0 poles)
    check_table(oracle, np.cumsum(w).astype(np.float32))


@pytest.mark.parametrize("name", ["features1", "features2", "ecosys"])
def test_alias_table_of_the_scene_environment(oracle, name):
    """The environment light CDFs of the scenes the GPU alias tests render (2048x1024 texels)."""
    sa = scene_abi(name)
    owned = oracle.make_lights(sa)  # keeps the arrays alive
    lights = owned.struct
    envs = [lights.lights[k] for k in range(lights.nlights) if lights.lights[k].environment >= 0]
    assert envs, name
    for l in envs:
        cdf = np.ctypeslib.as_array(l.cdf, shape=(l.ncdf,)).copy()
        keep, other = check_table(oracle, cdf)
        # the draw maps (rel, coin) uniform on [0,1)^2 onto that pmf: a stratified grid of draws
        n = len(cdf)
        rel = (np.arange(n * 4) + 0.5).astype(np.float32) / np.float32(n * 4)
        col = np.clip((rel * np.float32(n)).astype(np.int64), 0, n - 1)
        assert np.array_equal(np.bincount(col, minlength=n), np.full(n, 4))  # every column equally likely


def test_env_alias_render_is_a_different_mapping_of_the_same_light(abi, oracle):
    """Oracle renders with and without the option: the same light pmf (channel means within noise),
    a different random-number-to-texel map (the images differ), the same number of scene queries
    to within noise."""
    from conftest import make_params
    sa = scene_abi("features1")
    p = make_params(abi, resolution=48, samples=8)
    ob, ol = oracle.build_bvh(sa), oracle.make_lights(sa)
    a = oracle.trace(sa, ob, ol, p, 48, 48, 0, 8)
    b = oracle.trace(sa, ob, ol, p, 48, 48, 0, 8, env_alias=True)
    assert not np.array_equal(a[0], b[0])
    cm_a, cm_b = a[0][..., :3].mean(axis=(0, 1)), b[0][..., :3].mean(axis=(0, 1))
    np.testing.assert_allclose(cm_b, cm_a, rtol=0.05)
    assert abs(a[4]["rays"] - b[4]["rays"]) <= 0.02 * a[4]["rays"]
    # and the option is per call: the next default call gives the default bits again
    c = oracle.trace(sa, ob, ol, p, 48, 48, 0, 8)
    assert np.array_equal(a[0], c[0])
