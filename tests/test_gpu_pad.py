"""The level buffers' start offsets (MGP_PAD_BYTES, read when a context is created: each level's u, f, t and the finest
level's psiOld-keeping buffer start (j + 1) x pad bytes into their allocations) change where the arrays sit, never
what the cycle computes: psi and err bit-identical to unpadded buffers on every engine (temporally blocked 3D and 2D
phases, the fused full weighting, tiled small levels, the coarse tail)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

CASES = {
    "3d-zs-f32": dict(dim=3, n=(128, 128, 128), real="float", smoother="rbgs", nu1=2, nu2=2, prolong="linear"),
    "3d-f64-F": dict(dim=3, n=(64, 64, 128), real="double", smoother="rbgs", nu1=2, nu2=2, prolong="linear", cycle="F"),
    "2d-ys-f32": dict(dim=2, n=(1024, 1024, 1), real="float", smoother="rbgs", nu1=2, nu2=2, prolong="linear"),
    "3d-fw": dict(dim=3, n=(128, 128, 128), real="float", smoother="rbgs", nu1=2, nu2=2, prolong="linear",
                  restriction="full_weighting"),
}


def _run(kw, pad, monkeypatch):
    import mgpoisson

    monkeypatch.setenv("MGP_PAD_BYTES", str(pad))
    ctx = mgpoisson.Context(mgpoisson.make_opts(**kw))
    ctx.init_point_charge()
    errs = [ctx.cycle() for _ in range(2)] + list(ctx.cycles(2))
    psi = ctx.get_psi()
    ctx.close()
    return errs, psi


@pytest.mark.parametrize("name", list(CASES))
def test_buffer_offsets_do_not_change_results(name, monkeypatch):
    monkeypatch.setenv("MGP_FUSED_MIN_CELLS", "65536")
    monkeypatch.setenv("MGP_YS_MIN_CELLS", "65536")
    a = _run(CASES[name], 4352, monkeypatch)
    b = _run(CASES[name], 0, monkeypatch)
    c = _run(CASES[name], 256 * 7, monkeypatch)
    assert a[0] == b[0] == c[0]
    assert np.array_equal(a[1], b[1]) and np.array_equal(a[1], c[1])
