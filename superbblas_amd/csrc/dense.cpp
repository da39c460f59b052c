// Dense batched solvers over distributed tensors: cholesky / trsm / gesm / inversion.
//
// Reference: dense.h -- prepare_for_cholesky (507-560), get_dense_output_partition (445-490),
// cholesky (600-650), trsm (652-800), gesm (802-946), inversion (948-1000).
//  * A tensor with row labels `orows`, column labels `ocols` and batch labels (the rest) is
//    brought to the working order (batch, columns, rows) SlowToFast -- column-major square
//    matrices, rows fastest -- with every component holding whole matrices for its batch range
//    (a dist_copy: the redistribution, over RCCL when ranks are involved).
//  * The local step is one kernel over the batch (kernels_dense.hip); results go back through
//    another dist_copy.
//  * trsm / gesm: x is brought to (batch, right-hand-side labels, columns) when it holds the
//    column labels (C \ X, left side) or to (batch, rows, right-hand-side labels) when it holds
//    the row labels (X / C, right side; trsm only, as the reference), solved in place, and the
//    result, relabelled with the row (resp. column) labels, is copied into y.
#include "plan.h"

#include <algorithm>

namespace sbx {
namespace {

bool has(const std::string &s, char c) { return s.find(c) != std::string::npos; }

struct Work {
    DistTensor t;
    std::vector<Scratch> bufs;
    long n = 0;
    bool rm = false; // matrices row-major (batch, rows, columns): the caller's own order
    bool inplace = false; // the working tensor IS the caller's (same order, whole matrices)
    std::string ot; // batch labels (in the tensor's order)
};

/// Working copy of a tensor of square matrices (prepare_for_cholesky, dense.h:507-560)
Work prepare(const DistTensor &v, const std::string &orows, const std::string &ocols,
             const Comm &comm, bool copy_in, const char *what, bool allow_rm = false) {
    for (char c : orows) {
        if (has(ocols, c)) throw Error("Invalid `orows' and `ocols': they share labels");
        if (!has(v.labels, c)) throw Error("Invalid `orows': invalid labels");
    }
    for (char c : ocols)
        if (!has(v.labels, c)) throw Error("Invalid `ocols': invalid labels");
    Work w;
    for (char c : v.labels)
        if (!has(orows, c) && !has(ocols, c)) w.ot += c;
    long n = 1, m = 1;
    for (char c : orows) n *= v.dim[v.labels.find(c)];
    for (char c : ocols) m *= v.dim[v.labels.find(c)];
    // (the reference builds this error without throwing it, dense.h:543; a non-square shape is
    // rejected here)
    if (n != m) throw Error(std::string(what) + ": the matrices to factorize should be square");
    // a caller whose matrices are already whole and row-major (batch, rows, columns) keeps its
    // order: the working copies are then plain copies instead of transposes (small-matrix kernels)
    w.rm = allow_rm && v.labels == w.ot + orows + ocols && dense_wave_rows(n);
    const std::string ow = w.rm ? w.ot + orows + ocols : w.ot + ocols + orows;
    w.n = n;
    w.t.labels = ow;
    w.t.dtype = v.dtype;
    w.t.dim.resize(ow.size());
    for (std::size_t k = 0; k < ow.size(); ++k) w.t.dim[k] = v.dim[v.labels.find(ow[k])];
    w.t.ranges.resize(v.ranges.size());
    for (std::size_t r = 0; r < v.ranges.size(); ++r)
        for (const Range &q : v.ranges[r]) {
            Range o{Coor(ow.size(), 0), Coor(ow.size(), 0)};
            if (volume(q.size) > 0)
                for (std::size_t k = 0; k < ow.size(); ++k) {
                    const auto i = v.labels.find(ow[k]);
                    const bool mat = has(orows, ow[k]) || has(ocols, ow[k]);
                    o.from[k] = mat ? 0 : q.from[i];
                    o.size[k] = mat ? v.dim[i] : q.size[i];
                }
            w.t.ranges[r].push_back(o);
        }
    // the caller's order kept and every component already holding whole matrices: work on the
    // caller's memory (no copies; every rank decides alike from the global ranges)
    if (w.rm && v.mask.empty()) {
        bool same = true;
        for (std::size_t r = 0; r < v.ranges.size() && same; ++r)
            for (std::size_t c = 0; c < v.ranges[r].size() && same; ++c) {
                const Range &q = v.ranges[r][c], &o = w.t.ranges[r][c];
                if (volume(q.size) > 0 && (q.from != o.from || q.size != o.size)) same = false;
            }
        if (same) {
            w.inplace = true;
            w.t.ptr = v.ptr;
            w.t.dev = v.dev;
            return w;
        }
    }
    const std::size_t es = dtype_size(v.dtype);
    for (std::size_t c = 0; c < w.t.ranges[comm.rank].size(); ++c) {
        w.bufs.emplace_back(volume(w.t.ranges[comm.rank][c].size) * es, v.dev[c]);
        w.t.ptr.push_back(w.bufs.back().ptr);
        w.t.dev.push_back(v.dev[c]);
    }
    if (copy_in) {
        const Coor z(v.nd(), 0), zw(ow.size(), 0);
        dist_copy(Scalar{1, 0}, v, z, v.dim, w.t, zw, false, comm);
    }
    return w;
}

/// SB_DEBUG >= 1, several ranks: the ranks were called alike (check_consistency, dist.h:702-736).
/// The tune key dense.wave is part of the hash: it decides whether a rank works in place (no
/// dist_copy at all) or through working copies, so ranks set differently would run different
/// collective sequences -- it must be the same on every rank.
void check_dense_call(const char *what, const std::vector<const DistTensor *> &ts,
                      const std::string &orows, const std::string &ocols, const Scalar &alpha,
                      const Comm &comm) {
    if (debug_level() <= 0 || comm.nprocs <= 1) return;
    Hasher h;
    h.add(std::string(what));
    for (const DistTensor *t : ts) h.add(*t);
    h.add(orows);
    h.add(ocols);
    h.add(alpha);
    h.add((long)g_dense_wave);
    check_consistency(h, what, comm);
}

void check_info(int info) {
    if (info < 0)
        throw Error("Error in a lapack routine: wrong argument at position " + std::to_string(-info));
    if (info > 0) throw Error("Error in lapack routine: " + std::to_string(info));
}

/// Labels shared by several tensors must have the same dimension (check_dimensions)
void check_dims(const DistTensor &a, const DistTensor &b) {
    for (int i = 0; i < a.nd(); ++i) {
        const auto j = b.labels.find(a.labels[i]);
        if (j != std::string::npos && a.dim[i] != b.dim[j])
            throw Error("some dimension does not match");
    }
}

} // namespace

/// Note: when the caller's matrices are already whole and row-major per component and small
/// (dense.wave), the factorization runs in place: a matrix that is not Hermitian positive definite
/// then leaves the caller's tensor partly factorized when the error is thrown (the reference
/// factorizes a copy and leaves its input untouched on failure, dense.h:600-650).
void dense_cholesky(const DistTensor &v, const std::string &orows, const std::string &ocols,
                    const Comm &comm) {
    check_dense_call("cholesky", {&v}, orows, ocols, Scalar{1, 0}, comm);
    Work w = prepare(v, orows, ocols, comm, true, "cholesky", true);
    for (std::size_t c = 0; c < w.t.ptr.size(); ++c) {
        const long k = w.n ? volume(w.t.ranges[comm.rank][c].size) / (w.n * w.n) : 0;
        check_info(launch_potrf(v.dtype, w.t.ptr[c], w.n, k, w.t.dev[c], w.rm));
    }
    if (!w.inplace)
        dist_copy(Scalar{1, 0}, w.t, Coor(w.t.nd(), 0), w.t.dim, v, Coor(v.nd(), 0), false, comm);
}

void dense_inversion(const DistTensor &v, const std::string &orows, const std::string &ocols,
                     const Comm &comm) {
    check_dense_call("inversion", {&v}, orows, ocols, Scalar{1, 0}, comm);
    Work w = prepare(v, orows, ocols, comm, true, "inversion", true);
    std::vector<Scratch> inv;
    DistTensor wi = w.t;
    if (dense_wave_rows(w.n)) {
        // the small-matrix wave kernels read a matrix whole before writing its inverse: inverted in
        // place, no copy of the factors.  A singular matrix is left as it was, but unlike the
        // reference (which inverts a copy, dense.h:1268-1290) the other matrices of the batch
        // already hold their inverses when the error is thrown -- the same divergence as the
        // Cholesky note above
        for (std::size_t c = 0; c < w.t.ptr.size(); ++c) {
            const long k = w.n ? volume(w.t.ranges[comm.rank][c].size) / (w.n * w.n) : 0;
            check_info(launch_gesv(v.dtype, w.t.ptr[c], w.n, k, w.t.ptr[c], w.n, true, Scalar{1, 0},
                                   w.t.dev[c], w.rm, false));
        }
        if (!w.inplace)
            dist_copy(Scalar{1, 0}, w.t, Coor(w.t.nd(), 0), w.t.dim, v, Coor(v.nd(), 0), false, comm);
        return;
    }
    if (w.inplace) {
        // the factors go to a copy; the inverse straight into the caller's tensor
        DistTensor lu = w.t;
        for (std::size_t c = 0; c < w.t.ptr.size(); ++c) {
            inv.emplace_back(volume(w.t.ranges[comm.rank][c].size) * dtype_size(v.dtype), w.t.dev[c]);
            lu.ptr[c] = inv.back().ptr;
        }
        dist_copy(Scalar{1, 0}, v, Coor(v.nd(), 0), v.dim, lu, Coor(lu.nd(), 0), false, comm);
        for (std::size_t c = 0; c < w.t.ptr.size(); ++c) {
            const long k = w.n ? volume(w.t.ranges[comm.rank][c].size) / (w.n * w.n) : 0;
            check_info(launch_gesv(v.dtype, lu.ptr[c], w.n, k, v.ptr[c], w.n, true, Scalar{1, 0},
                                   w.t.dev[c], w.rm));
        }
        return;
    }
    for (std::size_t c = 0; c < w.t.ptr.size(); ++c) {
        const long k = w.n ? volume(w.t.ranges[comm.rank][c].size) / (w.n * w.n) : 0;
        inv.emplace_back(w.bufs[c].bytes, w.t.dev[c]);
        wi.ptr[c] = inv.back().ptr;
        check_info(launch_gesv(v.dtype, w.t.ptr[c], w.n, k, wi.ptr[c], w.n, true, Scalar{1, 0},
                               w.t.dev[c], w.rm));
    }
    dist_copy(Scalar{1, 0}, wi, Coor(wi.nd(), 0), wi.dim, v, Coor(v.nd(), 0), false, comm);
}

/// trsm (gesm = false) and gesm (gesm = true): y = alpha C^-1 x  or  y = alpha x C^-1
void dense_solve(bool gesm, const Scalar &alpha, const DistTensor &c, const std::string &orows,
                 const std::string &ocols, const DistTensor &x, const DistTensor &y,
                 const Comm &comm) {
    const char *what = gesm ? "gesm" : "trsm";
    check_dense_call(what, {&c, &x, &y}, orows, ocols, alpha, comm);
    check_dims(c, x);
    check_dims(c, y);
    check_dims(x, y);
    if (c.ranges[comm.rank].size() != x.ranges[comm.rank].size() ||
        x.ranges[comm.rank].size() != y.ranges[comm.rank].size())
        throw Error(std::string(what) + ": the given tensors don't have the same number of "
                                        "components or they don't follow the same order on the "
                                        "devices");
    for (std::size_t i = 0; i < c.dev.size(); ++i)
        if (c.dev[i] != x.dev[i] || x.dev[i] != y.dev[i])
            throw Error(std::string(what) + ": the given tensors don't have the same number of "
                                            "components or they don't follow the same order on "
                                            "the devices");
    // which side of C does x contract with (dense.h:700-722)
    bool rows = false, set = false, fail = false;
    for (char l : x.labels) {
        const bool in_c = has(ocols, l), in_r = has(orows, l);
        if (!in_c && !in_r) continue;
        if (set && rows != in_r) fail = true;
        rows = in_r;
        set = true;
    }
    if (fail || !set)
        throw Error(std::string(what) + ": cannot contract a mix of rows and column labels");
    if (gesm && rows) throw Error("gesm: unsupported to contract with row labels");
    for (char l : orows)
        if (!has(rows ? x.labels : y.labels, l))
            throw Error(std::string(what) + ": missing labels to contract");
    for (char l : ocols)
        if (!has(rows ? y.labels : x.labels, l))
            throw Error(std::string(what) + ": missing labels to contract");

    // Straight from x into y (small factors): x and y hold whole blocks of n x m
    // elements per batch entry in one of the two orientations (the batch labels first, in C's
    // order, then the contracted labels and the right-hand-side labels either way round), with
    // the same batch ranges as C on every rank -- no working copies of x and y, and C in the
    // caller's row-major order when it is whole (every rank decides alike from the global
    // ranges); gesm factors C in registers without writing it back and scales by alpha there
    {
        std::string ot, on;
        for (char l : c.labels)
            if (!has(orows, l) && !has(ocols, l)) ot += l;
        for (char l : x.labels)
            if (!has(c.labels, l)) on += l;
        const std::string &lx = rows ? orows : ocols, &ly = rows ? ocols : orows;
        long n = 1, m = 1;
        for (char l : orows) n *= c.dim[c.labels.find(l)];
        for (char l : on) m *= x.dim[x.labels.find(l)];
        // 1: (batch, contracted, rhs): component i of rhs t at i * m + t; 2: (batch, rhs,
        // contracted): at t * n + i; 0: neither, or the ranges do not match C's batch ranges
        auto orient = [&](const DistTensor &v, const std::string &l) {
            int o = v.labels == ot + l + on ? 1 : v.labels == ot + on + l ? 2 : 0;
            if (!o || !v.mask.empty()) return 0;
            for (std::size_t r = 0; r < v.ranges.size(); ++r) {
                // another rank's component count is checked only here (the generic path throws
                // on it later): decline the direct path rather than index past C's ranges
                if (r >= c.ranges.size() || v.ranges[r].size() != c.ranges[r].size()) return 0;
                for (std::size_t j = 0; j < v.ranges[r].size(); ++j) {
                    const Range &q = v.ranges[r][j], &qc = c.ranges[r][j];
                    if (volume(q.size) == 0 && volume(qc.size) == 0) continue;
                    for (std::size_t d = 0; d < v.labels.size(); ++d) {
                        const char lab = v.labels[d];
                        const auto ic = c.labels.find(lab);
                        if (has(ot, lab)) {
                            if (q.from[d] != qc.from[ic] || q.size[d] != qc.size[ic]) return 0;
                        } else if (q.from[d] != 0 || q.size[d] != v.dim[d]) {
                            return 0;
                        }
                    }
                }
            }
            return o;
        };
        const int ox = orient(x, lx), oy = orient(y, ly);
        if (ox && oy && x.dtype == c.dtype && y.dtype == c.dtype && dense_wave_rows(n) &&
            (gesm ? n * m < (1L << 31) : trsm_io_fits(n, m))) {
            Work wc = prepare(c, orows, ocols, comm, true, what, true);
            int bad = 0;
            for (std::size_t j = 0; j < wc.t.ptr.size(); ++j) {
                const long k = n ? volume(wc.t.ranges[comm.rank][j].size) / (n * n) : 0;
                if (k == 0) continue;
                const int xsi = ox == 1 ? (int)m : 1, xst = ox == 1 ? 1 : (int)n;
                const int ysi = oy == 1 ? (int)m : 1, yst = oy == 1 ? 1 : (int)n;
                if (gesm) {
                    const int info = launch_gesv_io(c.dtype, wc.t.ptr[j], n, k, wc.rm, x.ptr[j], xsi,
                                                    xst, y.ptr[j], ysi, yst, m, alpha, x.dev[j]);
                    if (!bad) bad = info;
                } else {
                    launch_trsm_io(c.dtype, wc.t.ptr[j], n, k, wc.rm, x.ptr[j], xsi, xst, y.ptr[j], ysi,
                                   yst, m, !rows, alpha, x.dev[j]);
                }
            }
            check_info(bad);
            return;
        }
    }
    Work wc = prepare(c, orows, ocols, comm, true, what);
    const long n = wc.n;
    std::string on;
    for (char l : x.labels)
        if (!has(c.labels, l)) on += l;
    const std::string &ot = wc.ot;
    const std::string oxw = rows ? ot + orows + on : ot + on + ocols;
    const std::string oyw = rows ? ot + ocols + on : ot + on + orows;
    // working x: C's working ranges for C's labels, x's ranges for the right-hand-side labels
    // (get_output_partition, dense.h:565-598)
    auto build = [&](const std::string &lab) {
        DistTensor t;
        t.labels = lab;
        t.dtype = x.dtype;
        t.dim.resize(lab.size());
        for (std::size_t k = 0; k < lab.size(); ++k)
            t.dim[k] = has(c.labels, lab[k]) ? c.dim[c.labels.find(lab[k])]
                                             : x.dim[x.labels.find(lab[k])];
        t.ranges.resize(c.ranges.size());
        for (std::size_t r = 0; r < c.ranges.size(); ++r) {
            if (x.ranges[r].size() != wc.t.ranges[r].size())
                throw Error(std::string(what) + ": the given tensors don't have the same number "
                                                "of components");
            for (std::size_t j = 0; j < wc.t.ranges[r].size(); ++j) {
                const Range &rc = wc.t.ranges[r][j], &rx = x.ranges[r][j];
                Range o{Coor(lab.size(), 0), Coor(lab.size(), 0)};
                bool empty = volume(rc.size) == 0 || volume(rx.size) == 0;
                for (std::size_t k = 0; k < lab.size() && !empty; ++k) {
                    const auto ic = wc.t.labels.find(lab[k]);
                    if (ic != std::string::npos) {
                        o.from[k] = rc.from[ic];
                        o.size[k] = rc.size[ic];
                    } else {
                        const auto ix = x.labels.find(lab[k]);
                        o.from[k] = rx.from[ix];
                        o.size[k] = rx.size[ix];
                    }
                }
                if (empty || volume(o.size) == 0) o = Range{Coor(lab.size(), 0), Coor(lab.size(), 0)};
                t.ranges[r].push_back(o);
            }
        }
        return t;
    };
    DistTensor xw = build(oxw);
    std::vector<Scratch> bufs;
    const std::size_t es = dtype_size(x.dtype);
    for (std::size_t j = 0; j < xw.ranges[comm.rank].size(); ++j) {
        bufs.emplace_back(volume(xw.ranges[comm.rank][j].size) * es, x.dev[j]);
        xw.ptr.push_back(bufs.back().ptr);
        xw.dev.push_back(x.dev[j]);
    }
    // the labels of xw not in x (none: every label of oxw is in x) -> copy x whole
    dist_copy(Scalar{1, 0}, x, Coor(x.nd(), 0), x.dim, xw, Coor(xw.nd(), 0), false, comm);
    for (std::size_t j = 0; j < xw.ptr.size(); ++j) {
        const long k = n ? volume(wc.t.ranges[comm.rank][j].size) / (n * n) : 0;
        if (k == 0) continue;
        const long ni = volume(xw.ranges[comm.rank][j].size) / (n * k);
        if (gesm)
            check_info(launch_gesv(c.dtype, wc.t.ptr[j], n, k, xw.ptr[j], ni, false, Scalar{1, 0},
                                   xw.dev[j]));
        else
            launch_trsm(c.dtype, wc.t.ptr[j], n, k, xw.ptr[j], ni, !rows, alpha, xw.dev[j]);
    }
    // the solution, relabelled: rows of the result are C's row (resp. column) labels
    DistTensor yw = build(oyw);
    yw.ptr = xw.ptr;
    yw.dev = xw.dev;
    dist_copy(gesm ? alpha : Scalar{1, 0}, yw, Coor(yw.nd(), 0), yw.dim, y, Coor(y.nd(), 0), false,
              comm);
}

} // namespace sbx
