// Local and distributed tensor contraction.
//
// Reference: suggested_orders_for_contraction + local_contraction_normalized
// (tensor.h:1271-1598) and contraction_normalized / get_partitions_for_contraction
// (dist.h:3039-3196).  The label classes are the reference's:
//   T: in o0, o1 and o_r (batch);  A: in o0 and o1 only (summed);
//   B: in o0 and o_r only;          C: in o1 and o_r only.
// The reference maps a contraction onto one strided batched GEMM after permuting each operand
// into a normalised order when needed.  The GEMM kernel here takes arbitrary strides for the
// batch, row, column and summed groups (and conjugation of either operand), so an operand is
// only copied when one of its label groups is not a single contiguous run of memory, or when
// its distribution does not match the work partition.
#include "plan.h"

#include <algorithm>

namespace sbx {

namespace {

struct GroupStride {
    bool ok;
    long stride, vol;
};

/// Stride/volume of a label group of a box of extents `size` inside a dense array of extents
/// `dims` (empty: the box is the array); !ok if the group labels (in the given order, size-1
/// labels ignored) are not one contiguous run of memory
GroupStride group_stride(const std::string &group, const std::string &labels, const Coor &size,
                         const Coor &dims = Coor()) {
    const std::vector<long> st = strides_slow_to_fast(dims.empty() ? size : dims);
    GroupStride g{true, 0, 1};
    int prev = -1;
    for (char c : group) {
        auto i = labels.find(c);
        if (i == std::string::npos) throw Error("contraction: internal label error");
        if (size[i] == 1) continue;
        g.vol *= size[i];
        if (prev >= 0 && st[prev] != st[i] * (long)size[i]) g.ok = false;
        prev = (int)i;
    }
    if (prev >= 0) g.stride = st[prev];
    return g;
}

/// Labels of `group` (in the given order, size-1 labels ignored) that start a new run of memory
/// in a box of extents `size` inside an array of extents `dims`: at most one such label lets the
/// GEMM address the group as two runs (outer index, inner index)
std::string group_breaks(const std::string &group, const std::string &labels, const Coor &size,
                         const Coor &dims = Coor()) {
    const std::vector<long> st = strides_slow_to_fast(dims.empty() ? size : dims);
    std::string br;
    int prev = -1;
    for (char c : group) {
        auto i = labels.find(c);
        if (i == std::string::npos) throw Error("contraction: internal label error");
        if (size[i] == 1) continue;
        if (prev >= 0 && st[prev] != st[i] * (long)size[i]) br += c;
        prev = (int)i;
    }
    return br;
}

/// Split form of a group in one tensor: inner run starting at label `brk` (0: one run)
struct GroupSplit {
    long vol = 1, lo = 1;   // group volume, inner extent
    long s = 0, s_hi = 0;   // inner / outer strides
};
GroupSplit group_split(const std::string &group, char brk, const std::string &labels,
                       const Coor &size, const Coor &dims = Coor()) {
    const std::vector<long> st = strides_slow_to_fast(dims.empty() ? size : dims);
    GroupSplit g;
    bool inner = brk == 0;
    int last = -1, last_outer = -1;
    for (char c : group) {
        const auto i = labels.find(c);
        if (c == brk) inner = true;
        if (size[i] == 1) continue;
        g.vol *= size[i];
        if (inner) g.lo *= size[i];
        else last_outer = (int)i;
        last = (int)i;
    }
    g.s = last >= 0 ? st[last] : 0;
    g.s_hi = last_outer >= 0 ? st[last_outer] : g.s * g.lo;
    if (brk == 0) g.lo = g.vol;
    return g;
}

/// Reorder the entries of `c` (labels `from`) into labels `to`
Coor reorder(const Coor &c, const std::string &from, const std::string &to) {
    Coor r(to.size());
    for (std::size_t j = 0; j < to.size(); ++j) r[j] = c[from.find(to[j])];
    return r;
}

} // namespace

void local_contraction(const Scalar &alpha, const Local &x, bool conjx, const Local &y,
                       bool conjy, const Scalar &beta, const Local &r) {
    // Label classes from the point of view of the GEMM: T batch, K summed, M rows (in x and r),
    // N columns (in y and r).  Group orders: T, K, M as in x; N as in y.
    std::string T, K, M, N;
    for (char c : x.labels) {
        const bool iny = y.labels.find(c) != std::string::npos;
        const bool inr = r.labels.find(c) != std::string::npos;
        if (iny && inr)
            T += c;
        else if (iny)
            K += c;
        else if (inr)
            M += c;
        else
            throw Error("o0 has unmatched dimensions");
    }
    for (char c : y.labels) {
        const bool inx = x.labels.find(c) != std::string::npos;
        const bool inr = r.labels.find(c) != std::string::npos;
        if (!inx && inr)
            N += c;
        else if (!inx)
            throw Error("o1 has unmatched directions");
    }
    if (r.labels.size() != T.size() + M.size() + N.size())
        throw Error("o_r has unmatched dimensions");
    const auto gx_t = group_stride(T, x.labels, x.size, x.dims);
    const auto gy_t = group_stride(T, y.labels, y.size, y.dims);
    const auto gr_t = group_stride(T, r.labels, r.size, r.dims);
    // M, N and K may each be two runs of memory, split at the same label in every tensor that
    // holds the group (e.g. the summed xyz and c of pXYZTSCn); T must be one run
    auto common_break = [](std::initializer_list<std::string> brs, char &brk) {
        std::string all;
        for (const std::string &b : brs)
            for (char c : b)
                if (all.find(c) == std::string::npos) all += c;
        if (all.size() > 1) return false;
        brk = all.empty() ? 0 : all[0];
        return true;
    };
    char bm = 0, bn = 0, bk = 0;
    const bool groups_ok =
        gx_t.ok && gy_t.ok && gr_t.ok &&
        common_break({group_breaks(M, x.labels, x.size, x.dims),
                      group_breaks(M, r.labels, r.size, r.dims)}, bm) &&
        common_break({group_breaks(N, y.labels, y.size, y.dims),
                      group_breaks(N, r.labels, r.size, r.dims)}, bn) &&
        common_break({group_breaks(K, x.labels, x.size, x.dims),
                      group_breaks(K, y.labels, y.size, y.dims)}, bk);
    if (!groups_ok) throw Error("local_contraction: operands need reordering");
    const GroupSplit gx_k = group_split(K, bk, x.labels, x.size, x.dims),
                     gx_m = group_split(M, bm, x.labels, x.size, x.dims),
                     gy_k = group_split(K, bk, y.labels, y.size, y.dims),
                     gy_n = group_split(N, bn, y.labels, y.size, y.dims),
                     gr_m = group_split(M, bm, r.labels, r.size, r.dims),
                     gr_n = group_split(N, bn, r.labels, r.size, r.dims);
    if (gx_t.vol != gy_t.vol || gx_t.vol != gr_t.vol || gx_k.vol != gy_k.vol ||
        gx_m.vol != gr_m.vol || gy_n.vol != gr_n.vol)
        throw Error("some dimension does not match");
    if (x.dev != y.dev || x.dev != r.dev) throw Error("all arrays should be on the same device");
    if (x.dtype != y.dtype || x.dtype != r.dtype) throw Error("contraction: mixed types");
    GemmDesc d;
    d.t = x.dtype;
    d.m = gx_m.vol;
    d.n = gy_n.vol;
    d.k = gx_k.vol;
    d.batch = gx_t.vol;
    d.a = x.ptr;
    d.sa_m = gx_m.s;
    d.sa_k = gx_k.s;
    d.sa_b = gx_t.stride;
    d.conja = conjx;
    d.b = y.ptr;
    d.sb_k = gy_k.s;
    d.sb_n = gy_n.s;
    d.sb_b = gy_t.stride;
    d.conjb = conjy;
    d.c = r.ptr;
    d.sc_m = gr_m.s;
    d.sc_n = gr_n.s;
    d.sc_b = gr_t.stride;
    d.alpha = alpha;
    d.beta = beta;
    d.m_lo = gx_m.lo;
    d.n_lo = gy_n.lo;
    d.k_lo = gx_k.lo;
    d.sa_m_hi = gx_m.s_hi;
    d.sa_k_hi = gx_k.s_hi;
    d.sb_k_hi = gy_k.s_hi;
    d.sb_n_hi = gy_n.s_hi;
    d.sc_m_hi = gr_m.s_hi;
    d.sc_n_hi = gr_n.s_hi;
    if (volume(x.size) == 0 || volume(y.size) == 0) d.k = 0;
    launch_gemm(d, x.dev);
}

void check_contraction_args(const std::string &l0, const Coor &size0, const std::string &l1,
                            const Coor &size1, const std::string &lr, const Coor &sizer, int t0,
                            int t1, int tr) {
    if (size0.size() != l0.size() || size1.size() != l1.size() || sizer.size() != lr.size())
        throw Error("contraction: invalid coordinates");
    if (t0 != t1 || t0 != tr) throw Error("contraction: mixed types");
    if (t0 == SBX_INT || t0 == SBX_SIZE_T) throw Error("contraction: unsupported type");
    // check_dimensions (tensor.h:623-646)
    for (int i = 0; i < (int)l0.size(); ++i) {
        auto j = l1.find(l0[i]);
        if (j != std::string::npos && size1[j] != size0[i])
            throw Error("some dimension does not match");
        auto k = lr.find(l0[i]);
        if (k != std::string::npos && sizer[k] != size0[i])
            throw Error("some dimension does not match");
    }
    for (int i = 0; i < (int)l1.size(); ++i) {
        auto k = lr.find(l1[i]);
        if (k != std::string::npos && sizer[k] != size1[i])
            throw Error("some dimension does not match");
    }
    for (int i = 0; i < (int)lr.size(); ++i)
        if (l0.find(lr[i]) == std::string::npos &&
            l1.find(lr[i]) == std::string::npos)
            throw Error("o_r has unmatched dimensions");
    for (int i = 0; i < (int)l0.size(); ++i)
        if (l1.find(l0[i]) == std::string::npos &&
            lr.find(l0[i]) == std::string::npos)
            throw Error("o0 has unmatched dimensions");
    for (int i = 0; i < (int)l1.size(); ++i)
        if (l0.find(l1[i]) == std::string::npos &&
            lr.find(l1[i]) == std::string::npos)
            throw Error("o1 has unmatched directions");
}

/// A sub-slab [c0, c0+n) of the slowest label of a local box
Local slab(const Local &l, long c0, long n, std::size_t es) {
    Local r = l;
    const Coor &d = l.dims.empty() ? l.size : l.dims;
    const long inner = volume(d) / std::max(1, d[0]);
    r.ptr = (char *)l.ptr + (std::size_t)(c0 * inner) * es;
    r.size[0] = (int)n;
    return r;
}

/// Offsets of box `f` inside component range `rc` (periodic coordinates), or empty if `f` is not
/// a non-wrapping sub-box of `rc`
Coor offset_in(const Range &f, const Range &rc, const Coor &dim) {
    Coor off(f.from.size());
    for (std::size_t j = 0; j < off.size(); ++j) {
        const long o = normalize_coor((long)f.from[j] - rc.from[j], dim[j]);
        if (o + f.size[j] > rc.size[j]) return Coor();
        off[j] = (int)o;
    }
    return off;
}

/// View of the box `f` of component `ptr` (range `rc`, dense in its own extents)
Local sub_view(void *ptr, int dev, const Range &rc, const Range &f, const Coor &off,
               const std::string &labels, int dtype) {
    const std::vector<long> st = strides_slow_to_fast(rc.size);
    long o = 0;
    for (std::size_t j = 0; j < off.size(); ++j) o += off[j] * st[j];
    return Local{(char *)ptr + (std::size_t)o * dtype_size(dtype), dev, f.size, labels, dtype,
                 rc.size};
}

void dist_contraction(const Scalar &alpha, const DistTensor &v0, const Coor &from0,
                      const Coor &size0, bool conj0, const DistTensor &v1, const Coor &from1,
                      const Coor &size1, bool conj1, const Scalar &beta, const DistTensor &vr,
                      const Coor &fromr, const Coor &sizer, const Comm &comm) {
    check_contraction_args(v0.labels, size0, v1.labels, size1, vr.labels, sizer, v0.dtype,
                           v1.dtype, vr.dtype);
    if (v0.dtype != v1.dtype || v0.dtype != vr.dtype) throw Error("contraction: mixed types");
    if (debug_level() > 0 && comm.nprocs > 1) { // check_consistency (dist.h:3105-3119)
        Hasher h;
        h.add(std::string("contraction"));
        h.add(alpha);
        h.add(beta);
        for (const DistTensor *t : {&v0, &v1, &vr}) h.add(*t);
        for (const Coor *c : {&from0, &size0, &from1, &size1, &fromr, &sizer}) h.add(*c);
        h.add((long)conj0 * 2 + (long)conj1);
        // the tune key dist.reduce picks collective or point-to-point reductions and must be the
        // same on every rank: a mismatch is caught here
        h.add((long)g_dist_reduce);
        check_consistency(h, "contraction", comm);
    }

    const int dtype = v0.dtype;
    const std::size_t es = dtype_size(dtype);

    // Work is partitioned like the larger operand (dist.h:3050-3056)
    const bool swap = volume(size0) < volume(size1);
    const DistTensor &X = swap ? v1 : v0, &Y = swap ? v0 : v1;
    const Coor &fromX = swap ? from1 : from0, &sizeX = swap ? size1 : size0;
    const Coor &fromY = swap ? from0 : from1, &sizeY = swap ? size0 : size1;
    const bool conjX = swap ? conj1 : conj0, conjY = swap ? conj0 : conj1;

    // Canonical group orders: T, K, M from X; N from Y
    std::string T, K, M, N;
    for (char c : X.labels) {
        const bool iny = Y.labels.find(c) != std::string::npos;
        const bool inr = vr.labels.find(c) != std::string::npos;
        if (iny && inr)
            T += c;
        else if (iny)
            K += c;
        else
            M += c;
    }
    for (char c : Y.labels)
        if (X.labels.find(c) == std::string::npos) N += c;
    const std::string lX = T + M + K, lY = T + N + K, lR = T + N + M; // temporaries' layouts

    // T of the box `size` inside an array of extents `dims` is one contiguous run and the other
    // groups at most two runs each (the GEMM's split groups)
    auto layout_ok = [&](const std::string &labels, const Coor &size, const Coor &dims,
                         std::initializer_list<const std::string *> groups) {
        if (!group_stride(T, labels, size, dims).ok) return false;
        for (const std::string *g : groups)
            if (g != &T && group_breaks(*g, labels, size, dims).size() > 1) return false;
        return true;
    };
    // the split points of a group in two tensors agree (at most one label in their union)
    auto same_break = [](const std::string &a, const std::string &b) {
        return a.empty() || b.empty() || a == b;
    };

    // Pieces of the work: X's ranges restricted to the box, repetitions removed (dist.h:3001-3028)
    struct WorkPiece {
        int rank, comp;
        Range px;        // in X coordinates (global)
        Range py, pr;    // needed ranges of Y and of the output (global coordinates)
        int ydirect = -1; // local Y component usable in place (the piece's box inside it)
        bool xdirect = false;
        Coor xoff, yoff;  // offsets of the piece's boxes inside those components
    };
    std::vector<WorkPiece> work;
    {
        std::vector<Range> prev;
        const Range box{fromX, sizeX};
        for (int rk = 0; rk < comm.nprocs; ++rk) {
            for (int i = 0; i < (int)X.ranges[rk].size(); ++i) {
                const Range &rx = X.ranges[rk][i];
                if (volume(rx.size) == 0) continue;
                std::vector<Range> fs = intersection(box, rx, X.dim);
                for (const Range &h : prev) {
                    std::vector<Range> nfs;
                    for (const Range &f : fs) {
                        if (intersection(f, h, X.dim).empty())
                            nfs.push_back(f);
                        else {
                            auto hh = make_hole(f, h, X.dim);
                            nfs.insert(nfs.end(), hh.begin(), hh.end());
                        }
                    }
                    fs.swap(nfs);
                }
                prev.push_back(rx);
                for (const Range &f : fs) {
                    if (volume(f.size) == 0) continue;
                    WorkPiece w;
                    w.rank = rk;
                    w.comp = i;
                    w.px = f;
                    w.py = translate(f, X.labels, fromX, X.dim, Y.labels, fromY, Y.dim);
                    for (int j = 0; j < Y.nd(); ++j)
                        if (X.labels.find(Y.labels[j]) == std::string::npos) {
                            w.py.from[j] = fromY[j];
                            w.py.size[j] = sizeY[j];
                        }
                    w.pr = translate(f, X.labels, fromX, X.dim, vr.labels, fromr, vr.dim);
                    for (int j = 0; j < vr.nd(); ++j)
                        if (X.labels.find(vr.labels[j]) == std::string::npos) {
                            const auto k = Y.labels.find(vr.labels[j]);
                            w.pr.from[j] = fromr[j];
                            w.pr.size[j] = sizeY[k];
                        }
                    // in-place use of X's component (the piece may be a sub-box of it)
                    w.xoff = offset_in(f, rx, X.dim);
                    w.xdirect = !w.xoff.empty() &&
                                layout_ok(X.labels, f.size, rx.size, {&T, &M, &K});
                    // in-place use of a Y component on the same rank
                    for (int j = 0; j < (int)Y.ranges[rk].size(); ++j) {
                        const Range &ry = Y.ranges[rk][j];
                        const Coor yo = offset_in(w.py, ry, Y.dim);
                        if (!yo.empty() && layout_ok(Y.labels, w.py.size, ry.size, {&T, &N, &K}) &&
                            (!w.xdirect ||
                             same_break(group_breaks(K, X.labels, f.size, rx.size),
                                        group_breaks(K, Y.labels, w.py.size, ry.size))) &&
                            (comm.nprocs > 1 || rk != comm.rank || Y.dev[j] == X.dev[i])) {
                            w.ydirect = j;
                            w.yoff = yo;
                            break;
                        }
                    }
                    work.push_back(w);
                }
            }
        }
    }

    // Single-process, single piece whose output is exactly one component: GEMM in place with beta
    // (boxes may be sub-boxes of the components: contracting a slice runs in place too)
    if (comm.nprocs == 1 && work.size() == 1 && work[0].xdirect && work[0].ydirect >= 0 &&
        vr.ranges[0].size() == 1 && !offset_in(work[0].pr, vr.ranges[0][0], vr.dim).empty() &&
        layout_ok(vr.labels, work[0].pr.size, vr.ranges[0][0].size, {&T, &N, &M}) &&
        same_break(group_breaks(M, X.labels, work[0].px.size, X.ranges[0][work[0].comp].size),
                   group_breaks(M, vr.labels, work[0].pr.size, vr.ranges[0][0].size)) &&
        same_break(group_breaks(N, Y.labels, work[0].py.size, Y.ranges[0][work[0].ydirect].size),
                   group_breaks(N, vr.labels, work[0].pr.size, vr.ranges[0][0].size)) &&
        vr.dev[0] == X.dev[work[0].comp]) {
        const WorkPiece &w = work[0];
        const Local lx = sub_view(X.ptr[w.comp], X.dev[w.comp], X.ranges[0][w.comp], w.px, w.xoff,
                                  X.labels, dtype);
        const Local ly = sub_view(Y.ptr[w.ydirect], Y.dev[w.ydirect], Y.ranges[0][w.ydirect],
                                  w.py, w.yoff, Y.labels, dtype);
        const Local lr = sub_view(vr.ptr[0], vr.dev[0], vr.ranges[0][0], w.pr,
                                  offset_in(w.pr, vr.ranges[0][0], vr.dim), vr.labels, dtype);
        local_contraction(alpha, lx, conjX, ly, conjY, beta, lr);
        return;
    }

    // 1) vr <- beta * vr on the box (dist.h:3145-3146)
    if (!beta.is_one()) dist_copy(beta, vr, fromr, sizer, vr, fromr, false, comm);
    if (alpha.is_zero() || work.empty()) return;

    // 2) temporaries for this rank's pieces; bring X / Y pieces that cannot be used in place
    DistTensor tx, ty, tr;
    tx.labels = lX;
    tx.dim = reorder(X.dim, X.labels, lX);
    ty.labels = lY;
    ty.dim = reorder(Y.dim, Y.labels, lY);
    tr.labels = lR;
    tr.dim = reorder(vr.dim, vr.labels, lR);
    tx.dtype = ty.dtype = tr.dtype = dtype;
    tx.ranges.resize(comm.nprocs);
    ty.ranges.resize(comm.nprocs);
    tr.ranges.resize(comm.nprocs);
    std::vector<Scratch> bufs;
    struct LocalWork {
        Local x, y, r;
    };
    std::vector<LocalWork> lw;
    for (const WorkPiece &w : work) {
        const bool mine = w.rank == comm.rank;
        const int dev = mine ? X.dev[w.comp] : -1;
        LocalWork l;
        if (!w.xdirect) {
            Range r{reorder(w.px.from, X.labels, lX), reorder(w.px.size, X.labels, lX)};
            tx.ranges[w.rank].push_back(r);
            if (mine) {
                bufs.emplace_back(volume(r.size) * es, dev);
                tx.ptr.push_back(bufs.back().ptr);
                tx.dev.push_back(dev);
                l.x = Local{bufs.back().ptr, dev, r.size, lX, dtype};
            }
        } else if (mine) {
            l.x = sub_view(X.ptr[w.comp], dev, X.ranges[w.rank][w.comp], w.px, w.xoff, X.labels,
                           dtype);
        }
        if (w.ydirect < 0) {
            Range r{reorder(w.py.from, Y.labels, lY), reorder(w.py.size, Y.labels, lY)};
            ty.ranges[w.rank].push_back(r);
            if (mine) {
                bufs.emplace_back(volume(r.size) * es, dev);
                ty.ptr.push_back(bufs.back().ptr);
                ty.dev.push_back(dev);
                l.y = Local{bufs.back().ptr, dev, r.size, lY, dtype};
            }
        } else if (mine) {
            l.y = sub_view(Y.ptr[w.ydirect], Y.dev[w.ydirect], Y.ranges[w.rank][w.ydirect], w.py,
                           w.yoff, Y.labels, dtype);
        }
        {
            Range r{reorder(w.pr.from, vr.labels, lR), reorder(w.pr.size, vr.labels, lR)};
            tr.ranges[w.rank].push_back(r);
            if (mine) {
                bufs.emplace_back(volume(r.size) * es, dev);
                tr.ptr.push_back(bufs.back().ptr);
                tr.dev.push_back(dev);
                l.r = Local{bufs.back().ptr, dev, r.size, lR, dtype};
            }
        }
        if (mine) lw.push_back(l);
    }
    const Coor tfromX = reorder(fromX, X.labels, lX), tfromY = reorder(fromY, Y.labels, lY);
    bool need_x = false, need_y = false;
    for (auto &rk : tx.ranges) need_x |= !rk.empty();
    for (auto &rk : ty.ranges) need_y |= !rk.empty();

    const Coor tfromr = reorder(fromr, vr.labels, lR), tsizer = reorder(sizer, vr.labels, lR);

    // 2+3+4 pipelined: with other ranks in the reduction, split the leading T label into chunks;
    // on the side stream, the operands of chunk c+1 are redistributed into the temporaries
    // (all-to-all) and chunk c's partial output is reduced into vr (pack, RCCL exchange, Add
    // unpack) while the GEMMs of chunk c run on the main stream.
    // The decision uses only information every rank holds (the global work list), so all ranks
    // issue the same sequence of collective copies.
    int nchunks = 1;
    if (comm.nprocs > 1 && !T.empty() && tsizer[0] > 1) {
        bool ok = true;
        for (const WorkPiece &w : work) {
            const char xf = w.xdirect ? X.labels[0] : lX[0];
            const char yf = w.ydirect >= 0 ? Y.labels[0] : lY[0];
            const Coor prs = reorder(w.pr.size, vr.labels, lR);
            ok &= xf == T[0] && yf == T[0] && prs[0] == tsizer[0];
        }
        for (const LocalWork &l : lw) ok &= l.x.size[0] == tsizer[0] && l.y.size[0] == tsizer[0];
        if (ok) nchunks = (int)std::min<long>(4, tsizer[0]);
    }
    if (nchunks > 1) {
        const int dev = !lw.empty() ? lw[0].r.dev : (comm.device >= 0 ? comm.device : vr.dev.empty() ? 0 : vr.dev[0]);
        const hipStream_t main_s = get_stream(dev), side_s = get_side_stream(dev);
        const long tn = tsizer[0];
        // operands of the T range [c0, c1) into the temporaries (box restricted along T[0])
        auto copy_operands = [&](long c0, long c1) {
            if (need_x) {
                Coor f = fromX, sz = sizeX, tf = tfromX;
                const int j = (int)X.labels.find(T[0]);
                f[j] = normalize_coor((long)f[j] + c0, X.dim[j]);
                sz[j] = (int)(c1 - c0);
                tf[0] = normalize_coor((long)tf[0] + c0, tx.dim[0]);
                dist_copy(Scalar{1, 0}, X, f, sz, tx, tf, false, comm);
            }
            if (need_y) {
                Coor f = fromY, sz = sizeY, tf = tfromY;
                const int j = (int)Y.labels.find(T[0]);
                f[j] = normalize_coor((long)f[j] + c0, Y.dim[j]);
                sz[j] = (int)(c1 - c0);
                tf[0] = normalize_coor((long)tf[0] + c0, ty.dim[0]);
                dist_copy(Scalar{1, 0}, Y, f, sz, ty, tf, false, comm);
            }
        };
        auto chunk = [&](int c) { return std::make_pair(tn * c / nchunks, tn * (c + 1) / nchunks); };
        // event after the side stream's copy of the next chunk's operands
        hipEvent_t ready = nullptr;
        auto record_ready = [&]() {
            SBX_HIP_CHECK(hipEventCreateWithFlags(&ready, hipEventDisableTiming));
            SBX_HIP_CHECK(hipEventRecord(ready, side_s));
        };
        stream_after(side_s, main_s);
        if (need_x || need_y) {
            StreamOverride so(dev, side_s);
            copy_operands(chunk(0).first, chunk(0).second);
            record_ready();
        }
        for (int c = 0; c < nchunks; ++c) {
            const long c0 = chunk(c).first, c1 = chunk(c).second;
            if (ready) {
                SBX_HIP_CHECK(hipStreamWaitEvent(main_s, ready, 0));
                SBX_HIP_CHECK(hipEventDestroy(ready));
                ready = nullptr;
            }
            if (c1 > c0)
                for (const LocalWork &l : lw)
                    local_contraction(alpha, slab(l.x, c0, c1 - c0, es), conjX,
                                      slab(l.y, c0, c1 - c0, es), conjY, Scalar{0, 0},
                                      slab(l.r, c0, c1 - c0, es));
            {
                StreamOverride so(dev, side_s);
                if ((need_x || need_y) && c + 1 < nchunks) {
                    copy_operands(chunk(c + 1).first, chunk(c + 1).second);
                    record_ready();
                }
            }
            if (c1 == c0) continue;
            stream_after(side_s, main_s);
            {
                StreamOverride so(dev, side_s);
                Coor f0 = tfromr, s0 = tsizer, f1 = fromr;
                f0[0] = (int)normalize_coor((long)f0[0] + c0, tr.dim[0]);
                s0[0] = (int)(c1 - c0);
                const int tr_in_vr = (int)vr.labels.find(lR[0]);
                f1[tr_in_vr] = (int)normalize_coor((long)f1[tr_in_vr] + c0, vr.dim[tr_in_vr]);
                if (!dist_reduce_collective(tr, f0, s0, vr, f1, comm))
                    dist_copy(Scalar{1, 0}, tr, f0, s0, vr, f1, true, comm);
            }
        }
        stream_after(main_s, side_s); // join: vr complete, temporaries free in order
        return;
    }

    if (need_x) dist_copy(Scalar{1, 0}, X, fromX, sizeX, tx, tfromX, false, comm);
    if (need_y) dist_copy(Scalar{1, 0}, Y, fromY, sizeY, ty, tfromY, false, comm);

    // 3) local contractions into the partial outputs
    for (const LocalWork &l : lw) local_contraction(alpha, l.x, conjX, l.y, conjY, Scalar{0, 0}, l.r);

    // 4) reduce the partial outputs into vr (dist.h:3183-3186): one RCCL collective where the
    //    partitions allow, else the Add copy (point-to-point sends into the owners)
    if (!dist_reduce_collective(tr, tfromr, tsizer, vr, fromr, comm))
        dist_copy(Scalar{1, 0}, tr, tfromr, tsizer, vr, fromr, true, comm);
}

} // namespace sbx
