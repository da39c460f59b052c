"""Full-size parity on the GPU (BASELINE configs 2, 2p and 3) through size-independent checks:
  * the 16^4, n = 64 lattice contraction against torch's complex128 einsum (rocBLAS, an
    independent GEMM) within 1e-12 relative, and bit-identical over 30 queued repetitions
    (deterministic split-K; guards against scratch-memory reuse races);
  * the 64-slice xyztsc -> tnsxyzc permute against torch's permute, bit-exact;
  * the 16^4 9-point 3x3-block BSR product on integer-valued data against a torch gather +
    einsum formulation, bit-exact."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _fill(t, seed):
    import torch
    g = torch.Generator(device=t.device)
    g.manual_seed(seed)
    r = torch.rand(t.numel(), 2, generator=g, device=t.device, dtype=torch.float64) * 2 - 1
    t.copy_(torch.view_as_complex(r))


def test_contraction_config2(gpu):
    import torch
    import superbblas_amd as sb
    L, n = 16, 64
    d0 = [L, n, 4, L, L, L, 3]
    dr = [L, n, 4, n, 4]
    vol0 = int(np.prod(d0))
    v0 = torch.empty(vol0, dtype=torch.complex128, device=gpu)
    v1 = torch.empty(vol0, dtype=torch.complex128, device=gpu)
    _fill(v0, 1)
    _fill(v1, 2)
    vr = torch.empty(int(np.prod(dr)), dtype=torch.complex128, device=gpu)
    z7, z5 = [0] * 7, [0] * 5
    p0, pr = [(z7, d0)], [(z5, dr)]

    def run():
        sb.contraction(1.0, p0, z7, d0, d0, "tnsxyzc", False, [v0], p0, z7, d0, d0, "tNSxyzc",
                       False, [v1], 0.0, pr, z5, dr, dr, "tNSns", [vr])
    run()
    first = vr.clone()
    for _ in range(30):
        run()
    torch.cuda.synchronize()
    assert torch.equal(vr, first), "contraction is not deterministic across queued repetitions"
    a = v0.view(L, n * 4, L * L * L * 3)
    b = v1.view(L, n * 4, L * L * L * 3)
    ref = torch.einsum("tik,tjk->tji", a, b).reshape(-1)  # tNSns: (N S) slow, (n s) fast
    err = (torch.linalg.vector_norm(vr - ref) / torch.linalg.vector_norm(ref)).item()
    assert err < 1e-12, err


def test_permute_config2p(gpu):
    import torch
    import superbblas_amd as sb
    L, n = 16, 64
    d0 = [L, L, L, L, 4, 3]
    d1 = [L, n, 4, L, L, L, 3]
    a = torch.empty(int(np.prod(d0)), dtype=torch.complex128, device=gpu)
    _fill(a, 3)
    b = torch.zeros(int(np.prod(d1)), dtype=torch.complex128, device=gpu)
    p0, p1 = [([0] * 6, d0)], [([0] * 7, d1)]
    for k in range(n):
        sb.copy(1.0, p0, "xyztsc", [0] * 6, d0, d0, [a], p1, "tnsxyzc", [0, k, 0, 0, 0, 0, 0], d1,
                [b])
    torch.cuda.synchronize()
    ref = a.view(L, L, L, L, 4, 3).permute(3, 4, 0, 1, 2, 5)  # t s x y z c
    ref = ref.unsqueeze(1).expand(L, n, 4, L, L, L, 3)
    assert torch.equal(b.view(d1), ref)


def test_bsr_config3(gpu):
    import torch
    import superbblas_amd as sb
    L, ncols = 16, 12
    dim = [L, L, L, L, 1, 3]
    V = L ** 4
    sites = np.array(np.unravel_index(np.arange(V), (L, L, L, L))).T
    nb = np.zeros((V, 9), np.int64)
    jj = np.zeros((V, 9, 6), np.int32)
    jj[:, 0, :4] = sites
    nb[:, 0] = np.arange(V)
    k = 1
    for d in range(4):
        for s in (-1, 1):
            c = sites.copy()
            c[:, d] = (c[:, d] + s) % L
            jj[:, k, :4] = c
            nb[:, k] = np.ravel_multi_index(tuple(c.T), (L, L, L, L))
            k += 1
    g = torch.Generator(device=gpu)
    g.manual_seed(7)

    def ints(shape):
        re = torch.randint(-4, 5, shape, generator=g, device=gpu).double()
        im = torch.randint(-4, 5, shape, generator=g, device=gpu).double()
        return torch.complex(re, im)
    vals = ints((V, 9, 3, 3))
    x = ints((V, 3, ncols))
    full = [([0] * 6, dim)]
    op = sb.create_bsr(full, dim, full, dim, [1, 1, 1, 1, 1, 3], [1, 1, 1, 1, 1, 3], False,
                       [torch.full((V,), 9, dtype=torch.int32, device=gpu)],
                       [torch.from_numpy(jj.reshape(-1)).to(gpu)], [vals.reshape(-1)])
    dimx = [1, L, L, L, L, 1, 3, ncols]
    y = torch.empty(V * 3 * ncols, dtype=torch.complex128, device=gpu)
    px = [([0] * 8, dimx)]
    sb.bsr_krylov(1.0, op, "xyztsc", "XYZTSC", px, "pXYZTSCn", [0] * 8, dimx, dimx,
                  [x.reshape(-1)], 0.0, px, "pxyztscn", [0] * 8, dimx, dimx, "p", [y])
    torch.cuda.synchronize()
    op.destroy()
    xg = x[torch.from_numpy(nb).to(gpu)]  # (V, 9, 3, ncols)
    ref = torch.einsum("vkce,vken->vcn", vals, xg).reshape(-1)
    assert torch.equal(y, ref)
