"""Multi-process plan of the distributed copy (the exchange under copy, contraction and the BSR
halo), checked on the CPU with a gloo process group (world sizes 2 and 3).

Each rank asks the library for the element counts it would send to / receive from every peer
(sbx_copy_plan: the same planner dist_copy runs before its RCCL grouped send/recv; reference
get_indices_to_send / get_indices_to_receive, dist.h:1789-1900).  The test checks
  * consistency across ranks: what rank r plans to send to q is what q plans to receive from r
    (a mismatch would deadlock or corrupt the RCCL exchange), and
  * the counts against a brute-force element-by-element enumeration of the copy semantics
    (Copy: every destination element receives exactly one value, taken from the same component,
    else the same rank, else the first holder; Add: every origin replica contributes,
    dist.h:2397-2435)."""
import itertools
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _inbox(c, frm, size, dim):
    return all(((ci - fi) % d if d else 0) < s for ci, fi, s, d in zip(c, frm, size, dim))


def brute_force_counts(p0, o0, from0, size0, dim0, nc0, p1, o1, from1, dim1, nc1, nprocs, rank,
                       add):
    send, recv, local = [0] * nprocs, [0] * nprocs, 0
    for off in itertools.product(*[range(s) for s in size0]):
        c = [(f + o) % d for f, o, d in zip(from0, off, dim0)]
        d1 = []
        for j, lab in enumerate(o1):
            i = o0.find(lab)
            d1.append(from1[j] if i < 0 else (from1[j] + off[i]) % dim1[j])
        holders = [g for g in range(nprocs * nc0) if _inbox(c, *p0[g], dim0)]
        for gb in range(nprocs * nc1):
            if not _inbox(d1, *p1[gb], dim1):
                continue
            rb = gb // nc1
            if add:
                srcs = holders
            else:
                def prio(g):
                    if g // nc0 != rb:
                        return 2
                    return 0 if g % nc0 == gb % nc1 else 1
                srcs = sorted(holders, key=prio)[:1]
            for ga in srcs:
                ra = ga // nc0
                if ra == rank and rb == rank:
                    local += 1
                elif ra == rank:
                    send[rb] += 1
                elif rb == rank:
                    recv[ra] += 1
    return send, recv, local


def _cases(nprocs):
    import superbblas_amd as sb
    cases = []
    # lattice field distributed over t, copied (permuted, shifted, wrapped) into a tensor
    # distributed over x -- the redistribution of a contraction operand
    dim0 = [4, 4, 2, 6]
    p0 = sb.basic_partitioning("xyzt", dim0, [1, 1, 1, nprocs], "t", nprocs, 1)
    dim1 = [6, 2, 4, 4]
    p1 = sb.basic_partitioning("tzyx", dim1, [1, 1, 1, nprocs], "x", nprocs, 1)
    cases.append((p0, "xyzt", [1, 2, 0, 3], [3, 4, 2, 5], dim0, 1, p1, "tzyx", [2, 0, 1, 3],
                  dim1, 1, sb.Copy))
    cases.append((p0, "xyzt", [0, 0, 0, 0], dim0, dim0, 1, p1, "tzyx", [0, 0, 0, 0], dim1, 1,
                  sb.Add))
    # replicated origin (every rank holds everything): Copy stays local, Add counts each replica
    rep = [([0, 0, 0], [3, 5, 4])] * nprocs
    pd = sb.basic_partitioning("abc", [3, 5, 4], [1, nprocs, 1], "b", nprocs, 1)
    cases.append((rep, "abc", [0, 0, 0], [3, 5, 4], [3, 5, 4], 1, pd, "abc", [0, 0, 0],
                  [3, 5, 4], 1, sb.Copy))
    pc = sb.basic_partitioning("cab", [4, 3, 5], [1, 1, nprocs], "b", nprocs, 1)
    cases.append((rep, "abc", [1, 1, 1], [2, 4, 3], [3, 5, 4], 1, pc, "cab", [2, 0, 1],
                  [4, 3, 5], 1, sb.Add))
    # two components per rank on both sides, a dropped size-1 label and a new label
    q0 = sb.basic_partitioning("abcd", [5, 4, 6, 3], [1, 1, 2 * nprocs, 1], "c", 2 * nprocs, 1)
    q1 = sb.basic_partitioning("cqab", [6, 2, 5, 4], [1, 1, 2 * nprocs, 1], "a", 2 * nprocs, 1)
    cases.append((q0, "abcd", [1, 0, 2, 1], [4, 4, 5, 1], [5, 4, 6, 3], 2, q1, "cqab",
                  [3, 1, 2, 0], [6, 2, 5, 4], 2, sb.Copy))
    # several components per rank (the reference's --components=2, each on its own GPU): a
    # field split over nprocs x 2 components into a domain partition with a one-site halo in x
    # and y (the BSR halo exchange of the chain), and back with Add (the image-side sum)
    dim = [8, 6, 2, 3]
    pf = sb.basic_partitioning("xyzt", dim, [nprocs, 1, 1, 1], "xy", nprocs, 2)
    ph = []
    for f, sz in pf:
        f, sz = list(f), list(sz)
        for d in range(2):
            if 0 < sz[d] and sz[d] + 2 <= dim[d]:
                sz[d] += 2
                f[d] = (f[d] - 1) % dim[d]
        ph.append((f, sz))
    cases.append((pf, "xyzt", [0] * 4, dim, dim, 2, ph, "xyzt", [0] * 4, dim, 2, sb.Copy))
    cases.append((ph, "xyzt", [0] * 4, dim, dim, 2, pf, "xyzt", [0] * 4, dim, 2, sb.Add))
    return cases


def _worker(rank, nprocs, port, q):
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        dist.init_process_group("gloo", rank=rank, world_size=nprocs)
        import superbblas_amd as sb
        for ci, case in enumerate(_cases(nprocs)):
            (p0, o0, f0, s0, d0, nc0, p1, o1, f1, d1, nc1, ca) = case
            send, recv, local = sb.copy_plan(p0, o0, f0, s0, d0, nc0, p1, o1, f1, d1, nc1, nprocs,
                                             rank, copyadd=ca)
            want = brute_force_counts(p0, o0, f0, s0, d0, nc0, p1, o1, f1, d1, nc1, nprocs, rank,
                                      ca == sb.Add)
            assert (send, recv, local) == tuple(want), (ci, rank, (send, recv, local), want)
            row = torch.tensor(send + recv, dtype=torch.int64)
            rows = [torch.zeros_like(row) for _ in range(nprocs)]
            dist.all_gather(rows, row)
            for r in range(nprocs):
                for s in range(nprocs):
                    if r != s:
                        assert rows[r][s] == rows[s][nprocs + r], (ci, r, s)
        dist.barrier()
        dist.destroy_process_group()
        q.put((rank, None))
    except Exception as e:  # report to the parent instead of hanging the group
        q.put((rank, repr(e)))
        raise


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("nprocs", [2, 3])
def test_copy_plan_consistent_across_ranks(nprocs):
    ctx = mp.get_context("spawn")
    q = ctx.SimpleQueue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, nprocs, port, q)) for r in range(nprocs)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=240)
    results = {}
    while not q.empty():
        r, err = q.get()
        results[r] = err
    for p in procs:
        if p.is_alive():
            p.kill()
    assert sorted(results) == list(range(nprocs)), results
    assert all(v is None for v in results.values()), results


def test_brute_force_single_rank_matches_library():
    import superbblas_amd as sb
    for case in _cases(1):
        (p0, o0, f0, s0, d0, nc0, p1, o1, f1, d1, nc1, ca) = case
        got = sb.copy_plan(p0, o0, f0, s0, d0, nc0, p1, o1, f1, d1, nc1, 1, 0, copyadd=ca)
        want = brute_force_counts(p0, o0, f0, s0, d0, nc0, p1, o1, f1, d1, nc1, 1, 0,
                                  ca == sb.Add)
        assert got == tuple(want)
