"""Error behaviour of the public API on invalid arguments (the reference throws
std::runtime_error with these messages: tensor.h:495-507 check_isomorphic, tensor.h:623-646
check_dimensions, dist.h:94-99 unsupported contraction types).  The checks run on the host
before any device work, so they are exercised here without a GPU."""
import pytest
import torch

import superbblas_amd as sb

Z = torch.complex128


def _copy(o0, o1, size0=(2, 2), dim1=(2, 2)):
    a = torch.zeros(4, dtype=Z)
    b = torch.zeros(4, dtype=Z)
    sb.copy(1.0, [([0, 0], [2, 2])], o0, [0, 0], list(size0), [2, 2], [a],
            [([0, 0], list(dim1))], o1, [0, 0], list(dim1), [b])


@pytest.mark.parametrize("o0,o1,msg", [
    ("ab", "cd", "Invalid copy operation"),     # labels of o0 absent in o1 with size > 1
    ("aa", "ab", "repeated labels"),
])
def test_copy_invalid(o0, o1, msg):
    with pytest.raises(sb.SuperbblasError, match=msg):
        _copy(o0, o1)


def test_copy_size_larger_than_destination():
    with pytest.raises(sb.SuperbblasError, match="Invalid copy operation"):
        a = torch.zeros(6, dtype=Z)
        b = torch.zeros(4, dtype=Z)
        sb.copy(1.0, [([0, 0], [2, 3])], "ab", [0, 0], [2, 3], [2, 3], [a],
                [([0, 0], [2, 2])], "ab", [0, 0], [2, 2], [b])


def test_copy_partition_incompatible():
    with pytest.raises(sb.SuperbblasError, match="partition"):
        a = torch.zeros(4, dtype=Z)
        sb.copy(1.0, [([0, 0], [2, 2])] * 2, "ab", [0, 0], [2, 2], [2, 2], [a],
                [([0, 0], [2, 2])], "ab", [0, 0], [2, 2], [a])


def _contract(o0, d0, o1, d1, o_r, dr, dtype=Z):
    def t(d):
        n = 1
        for x in d:
            n *= x
        return torch.zeros(n, dtype=dtype)
    z = lambda d: [0] * len(d)  # noqa: E731
    sb.contraction(1.0, [(z(d0), d0)], z(d0), d0, d0, o0, False, [t(d0)], [(z(d1), d1)], z(d1),
                   d1, d1, o1, False, [t(d1)], 0.0, [(z(dr), dr)], z(dr), dr, dr, o_r, [t(dr)])


def test_contraction_dimension_mismatch():
    with pytest.raises(sb.SuperbblasError, match="some dimension does not match"):
        _contract("ik", [2, 3], "kj", [4, 2], "ij", [2, 2])


def test_contraction_unmatched_output_label():
    with pytest.raises(sb.SuperbblasError, match="o_r has unmatched dimensions"):
        _contract("ik", [2, 3], "kj", [3, 2], "iq", [2, 2])


def test_contraction_unmatched_input_label():
    with pytest.raises(sb.SuperbblasError, match="unmatched"):
        _contract("ikq", [2, 3, 2], "kj", [3, 2], "ij", [2, 2])


def test_contraction_integer_type_rejected():
    with pytest.raises(sb.SuperbblasError, match="unsupported type|dtype"):
        _contract("ik", [2, 3], "kj", [3, 2], "ij", [2, 2], dtype=torch.int32)


def test_make_hole_rank_mismatch():
    with pytest.raises(sb.SuperbblasError):
        sb.make_hole([0, 0], [2, 2], [0], [1], [4, 4])


def test_fast_to_slow_plan_matches_slow_to_fast():
    """FastToSlow is the reversal of SlowToFast (tensor.h:56-60, 282-297): the same copy written
    in both orders has the same exchange plan."""
    dim0, dim1 = [4, 4, 2, 6], [6, 2, 4, 4]
    p0 = sb.basic_partitioning("xyzt", dim0, [1, 1, 1, 2], "t", 2, 1)
    p1 = sb.basic_partitioning("tzyx", dim1, [1, 1, 1, 2], "x", 2, 1)
    rev = lambda p: [(list(f)[::-1], list(s)[::-1]) for f, s in p]  # noqa: E731
    for rank in (0, 1):
        a = sb.copy_plan(p0, "xyzt", [1, 2, 0, 3], [3, 4, 2, 5], dim0, 1, p1, "tzyx",
                         [2, 0, 1, 3], dim1, 1, 2, rank)
        b = sb.copy_plan(rev(p0), "tzyx", [3, 0, 2, 1], [5, 2, 4, 3], dim0[::-1], 1, rev(p1),
                         "xyzt", [3, 1, 0, 2], dim1[::-1], 1, 2, rank, co=sb.FastToSlow)
        assert a == b


def test_basic_partitioning_more_procs_than_nprocs():
    """procs covering more processes than nprocs: the reference builds this error without
    throwing it and then writes past its result (dist.h:3400-3402); here it is raised"""
    import pytest
    import superbblas_amd as sb
    with pytest.raises(sb.SuperbblasError, match="greater than `nprocs`"):
        sb.basic_partitioning("tnsxyzc", [8, 12, 4, 8, 8, 4, 3], [4, 1, 1, 1, 1, 1, 1], "t", 1, 4)
    # components of one process: procs is the process grid, components split inside
    p = sb.basic_partitioning("xyzt", [8, 8, 4, 8], [1, 1, 1, 1], "xyz", 1, 4)
    assert len(p) == 4 and sum(a * b * c * d for _, (a, b, c, d) in p) == 8 * 8 * 4 * 8
