"""SB_DEBUG self-checks (the reference's debug mode, runtime_features.h:24-37):

* level >= 2: every copy is first run on index-valued size_t mock tensors through the same plan
  and kernels and checked exactly (ns_copy_test, dist.h:1919-2116, triggered at 2282-2285) --
  the reference's golden copies pass it (masks, Add of replicated origins, periodic wraps, host
  components), and a deliberately wrong plan (tune key debug.corrupt_copy drops a local piece)
  is caught with the reference's message;
* level >= 1 with several ranks: the call arguments are hashed and compared across the ranks
  (check_consistency, dist.h:702-736) -- tests/dist_worker.py `debug`.

The level is set through the tune key debug.level (SB_DEBUG is read once at load)."""
import numpy as np
import pytest

from _golden import NPT, gen, manifest, output, parity_masks, piece, put_piece, vol

pytestmark = pytest.mark.gpu


@pytest.fixture
def debug2():
    import superbblas_amd as sb
    old = sb.tune_get("debug.level")
    sb.tune_set("debug.level", 2)
    try:
        yield sb
    finally:
        sb.tune_set("debug.level", old)
        sb.tune_set("debug.corrupt_copy", 0)


def _scatter(glob, dim, p, gpu):
    import torch
    return [torch.from_numpy(piece(glob, dim, f, s)).to(gpu if (len(p) == 1 or i % 2 == 0)
                                                         else "cpu")
            for i, (f, s) in enumerate(p)]


def _golden_copy(sb, case, gpu):
    import torch
    t0, t1 = NPT[case["t0"]], NPT[case["t1"]]
    g0 = gen(case["gen0"], vol(case["dim0"]), 1, t0)
    g1 = gen(case["gen1"], vol(case["dim1"]), 2, t1)
    v0 = _scatter(g0, case["dim0"], case["p0"], gpu)
    v1 = _scatter(g1, case["dim1"], case["p1"], gpu)
    m0 = m1 = None
    if case.get("mask"):
        gm0, gm1 = parity_masks(case)
        m0 = _scatter(gm0, case["dim0"], case["p0"], gpu)
        m1 = _scatter(gm1, case["dim1"], case["p1"], gpu)
    sb.copy(complex(*case["alpha"]) if np.dtype(t0).kind == "c" else case["alpha"][0],
            case["p0"], case["o0"], case["from0"], case["size0"], case["dim0"], v0,
            case["p1"], case["o1"], case["from1"], case["dim1"], v1,
            copyadd=sb.Add if case["add"] else sb.Copy, mask0=m0, mask1=m1)
    torch.cuda.synchronize()
    out = np.zeros(vol(case["dim1"]), t1)
    for (f, s), c in zip(case["p1"], v1):
        put_piece(out, case["dim1"], f, s, c.cpu().numpy())
    return out


@pytest.mark.parametrize("case", manifest("copy"), ids=lambda c: "copy%d" % c["id"])
def test_debug2_golden_copies(gpu, debug2, case):
    """Every golden copy passes the mock-index check and still gives the reference's bytes"""
    out = _golden_copy(debug2, case, gpu)
    ref = output(case, NPT[case["t1"]])
    assert np.array_equal(out.view(np.uint8), ref.view(np.uint8))


def test_debug2_contraction_copies(gpu, debug2):
    """The copies inside a contraction (reorders into temporaries, beta scaling) are checked too"""
    from _common import oracle_contraction, random_valued, rel_err
    import torch
    sb = debug2
    d0 = [3, 2, 4, 2, 2, 2, 3]  # tnsxyzc
    dr = [3, 2, 4, 2, 4]        # tNSns
    v0 = random_valued(vol(d0), np.complex128, 1)
    v1 = random_valued(vol(d0), np.complex128, 2)
    vr = random_valued(vol(dr), np.complex128, 3)
    ref = vr.copy()
    z7, z5 = [0] * 7, [0] * 5
    # an operand order that needs a reorder (x after c) and beta != 0, 1
    o1, d1 = "tNxSyzc", [3, 2, 2, 4, 2, 2, 3]
    g1 = v1.reshape(d0).transpose(0, 1, 3, 2, 4, 5, 6).copy().reshape(-1)
    oracle_contraction(1.0, "tnsxyzc", z7, d0, d0, False, v0, o1, z7, d1, d1, False, g1,
                       0.5 - 0.25j, "tNSns", z5, dr, dr, ref)
    t = [torch.from_numpy(a).to(gpu) for a in (v0, g1, vr)]
    sb.contraction(1.0, [(z7, d0)], z7, d0, d0, "tnsxyzc", False, [t[0]], [(z7, d1)], z7, d1, d1,
                   o1, False, [t[1]], 0.5 - 0.25j, [(z5, dr)], z5, dr, dr, "tNSns", [t[2]])
    torch.cuda.synchronize()
    assert rel_err(t[2].cpu().numpy(), ref) < 1e-12


def test_debug2_catches_corrupt_plan(gpu, debug2):
    """A plan that loses a local piece (debug.corrupt_copy) is caught by the check; without the
    check the same plan silently writes a wrong destination"""
    import torch
    sb = debug2
    o0, d0, o1 = "xyzt", [4, 5, 6, 3], "tzyx"
    d1 = [d0[o0.index(c)] for c in o1]
    # two origin components -> at least two local pieces
    p0 = [([0, 0, 0, 0], [2, 5, 6, 3]), ([2, 0, 0, 0], [2, 5, 6, 3])]
    p1 = [([0, 0, 0, 0], d1)]
    g0 = np.arange(vol(d0), dtype=np.float64).astype(np.complex128)
    v0 = [torch.from_numpy(piece(g0, d0, f, s)).to(gpu) for f, s in p0]
    v1 = [torch.zeros(vol(d1), dtype=torch.complex128, device=gpu)]
    sb.tune_set("debug.corrupt_copy", 2)
    with pytest.raises(sb.SuperbblasError, match="test_copy_check does not pass"):
        sb.copy(1.0, p0, o0, [0] * 4, d0, d0, v0, p1, o1, [0] * 4, d1, v1)
    # level 0: no check, the corrupted copy completes with a wrong answer
    sb.tune_set("debug.level", 0)
    sb.copy(1.0, p0, o0, [0] * 4, d0, d0, v0, p1, o1, [0] * 4, d1, v1)
    torch.cuda.synchronize()
    sb.tune_set("debug.corrupt_copy", 0)
    good = [torch.zeros_like(v1[0])]
    sb.copy(1.0, p0, o0, [0] * 4, d0, d0, v0, p1, o1, [0] * 4, d1, good)
    torch.cuda.synchronize()
    assert not torch.equal(v1[0], good[0])
