// Host planner: periodic range algebra and partitioning helpers.
// Behaviour restated from the reference (dist.h); see plan.h for the line map.
#include "plan.h"

#include <algorithm>
#include <cstring>

namespace sbx {

namespace {

// Intersection of two 1-D ranges for a NOT toroidal lattice (dist.h:352-358)
void intersection1(int from0, int size0, int from1, int size1, int dim, int &fromr, int &sizer) {
    fromr = from0 + std::min(std::max(from1 - from0, 0), size0);
    sizer = from0 + std::min(std::max(from1 + size1 - from0, 0), size0) - fromr;
    fromr = dim == 0 ? 0 : (fromr + dim) % dim;
    if (sizer == dim) fromr = from0;
}

} // namespace

std::vector<Range> intersection(const Range &a, const Range &b, const Coor &dim) {
    const std::size_t nd = dim.size();
    // Per-dimension subintervals (dist.h:370-420)
    std::vector<std::vector<std::pair<int, int>>> grid(nd);
    for (std::size_t i = 0; i < nd; ++i) {
        if (a.size[i] > dim[i] || b.size[i] > dim[i])
            throw Error("intersection: invalid input arguments");
        int f0 = 0, s0 = 0, f1 = 0, s1 = 0, f2 = 0, s2 = 0;
        if (a.size[i] == dim[i] && b.size[i] == dim[i]) {
            f0 = a.from[i];
            s0 = a.size[i];
        } else if (b.size[i] == dim[i]) {
            f0 = a.from[i];
            s0 = a.size[i];
        } else if (a.size[i] == dim[i]) {
            f0 = b.from[i];
            s0 = b.size[i];
        } else {
            intersection1(a.from[i], a.size[i], b.from[i], b.size[i], dim[i], f0, s0);
            intersection1(a.from[i], a.size[i], b.from[i] + dim[i], b.size[i], dim[i], f1, s1);
            intersection1(a.from[i] + dim[i], a.size[i], b.from[i], b.size[i], dim[i], f2, s2);
        }
        if (s0 > 0) grid[i].push_back({f0, s0});
        if (s1 > 0) grid[i].push_back({f1, s1});
        if (s2 > 0) grid[i].push_back({f2, s2});
        if (grid[i].empty()) return {};
    }
    // Cartesian product, first dimension fastest (FastToSlow enumeration as in dist.h:477-496)
    long n = 1;
    for (auto &g : grid) n *= (long)g.size();
    std::vector<Range> r(n, Range{Coor(nd), Coor(nd)});
    for (long k = 0; k < n; ++k) {
        long rem = k;
        for (std::size_t i = 0; i < nd; ++i) {
            const long c = rem % (long)grid[i].size();
            rem /= (long)grid[i].size();
            r[k].from[i] = grid[i][c].first;
            r[k].size[i] = grid[i][c].second;
        }
    }
    return r;
}

std::vector<Range> intersection(const std::vector<Range> &as, const Range &b, const Coor &dim) {
    std::vector<Range> r;
    for (const auto &a : as) {
        auto x = intersection(a, b, dim);
        r.insert(r.end(), x.begin(), x.end());
    }
    return r;
}

std::vector<Range> make_hole(const Range &r, const Range &hole, const Coor &dim) {
    const std::size_t N = dim.size();
    if (N == 0) return {};
    if (volume(hole.size) == 0) return {r};
    // Make a hole on the whole lattice: N subranges (dist.h:3758-3795)
    std::vector<Range> parts;
    for (std::size_t i = 0; i < N; ++i) {
        Range p{Coor(N), Coor(N)};
        for (std::size_t j = 0; j < i; ++j) {
            p.from[j] = hole.from[j];
            p.size[j] = hole.size[j];
        }
        p.from[i] = normalize_coor((long)hole.from[i] + hole.size[i], dim[i]);
        p.size[i] = dim[i] - hole.size[i];
        for (std::size_t j = i + 1; j < N; ++j) {
            p.from[j] = 0;
            p.size[j] = dim[j];
        }
        parts.push_back(p);
    }
    // Intersect the parts with the range, drop empty ones (dist.h:3812-3824)
    std::vector<Range> out;
    for (const auto &p : parts)
        for (const auto &x : intersection(p, r, dim))
            if (volume(x.size) > 0) out.push_back(x);
    return out;
}

std::vector<int> find_permutation(const std::string &from, const std::string &to) {
    std::vector<int> p(to.size(), -1);
    for (std::size_t i = 0; i < to.size(); ++i) {
        auto k = from.find(to[i]);
        if (k != std::string::npos) p[i] = (int)k;
    }
    return p;
}

//
// Partitioning helpers
//

namespace {
// Approximate factorization with factors 2 and 3 (dist.h:1-... factors_2_3)
struct F23 {
    unsigned two = 0, three = 0, value = 1;
    F23() {}
    F23(unsigned two, unsigned three, unsigned value) : two(two), three(three), value(value) {}
    explicit F23(unsigned number) {
        if (number == 0) throw Error("unsupported value");
        unsigned remaining = number;
        for (; remaining % 2 == 0; ++two, remaining /= 2, value *= 2)
            ;
        for (; remaining % 3 == 0; ++three, remaining /= 3, value *= 3)
            ;
        for (; remaining >= 3; ++three, remaining /= 3, value *= 3)
            ;
        if (remaining >= 2) ++two, remaining /= 2, value *= 2;
        for (; three > 0 && value * 4 / 3 <= number; --three, two += 2, value = value * 4 / 3)
            ;
    }
    F23 operator*(const F23 &v) const { return F23(two + v.two, three + v.three, value * v.value); }
};
} // namespace

Coor partitioning_distributed_procs(const std::string &order, const Coor &dim,
                                    const std::string &dist_labels, unsigned nprocs) {
    const std::size_t Nd = dim.size();
    Coor p(Nd, 1);
    if (order.size() != Nd) throw Error("partitioning_distributed_procs: invalid `order`");
    std::vector<int> dist_perm;
    for (char c : dist_labels) {
        auto it = order.find(c);
        if (it != std::string::npos && dim[it] > 1) dist_perm.push_back((int)it);
    }
    const unsigned dist_n = (unsigned)dist_perm.size();
    if (dist_n == 0 || volume(dim) == 0 || nprocs <= 1) return p;

    std::vector<F23> p_f23(dist_n, F23(1u));
    F23 vol_p(1u);
    const F23 nprocs_f23(nprocs);
    const F23 factors[2] = {F23(3u), F23(2u)};
    while (true) {
        // Sort the dimensions by local size, largest first (selection sort as dist.h:3349-3359)
        std::vector<unsigned> perm(dist_n);
        for (unsigned j = 0; j < dist_n; ++j) perm[j] = j;
        for (unsigned j = 0; j < dist_n; ++j) {
            unsigned large_i = j;
            std::size_t large_val = dim[dist_perm[perm[j]]] / p_f23[perm[j]].value;
            for (unsigned i = j + 1; i < dist_n; ++i) {
                std::size_t val = dim[dist_perm[perm[i]]] / p_f23[perm[i]].value;
                if (large_val < val) large_i = i, large_val = val;
            }
            std::swap(perm[j], perm[large_i]);
        }
        bool applied = false;
        for (unsigned j = 0; j < dist_n && !applied; ++j) {
            for (const auto &f : factors) {
                if (nprocs_f23.value % (vol_p.value * f.value) == 0) {
                    p_f23[perm[j]] = p_f23[perm[j]] * f;
                    vol_p = vol_p * f;
                    applied = true;
                    break;
                }
            }
        }
        if (!applied) break;
    }
    for (unsigned i = 0; i < dist_n; ++i) p[dist_perm[i]] = (int)p_f23[i].value;
    return p;
}

std::vector<Range> basic_partitioning(const char *order, const Coor &dim, const Coor &procs,
                                      const char *dist_labels, int nprocs, int ncomponents) {
    const std::size_t Nd = dim.size();
    const int vol_procs = (int)volume(procs);
    std::vector<int> perm(Nd);
    if (order != nullptr && dist_labels != nullptr) {
        if (std::strlen(order) != Nd)
            throw Error("basic_partitioning: invalid `order`, its length doesn't match");
        const std::size_t n = std::strlen(dist_labels);
        std::size_t dist_n = 0;
        for (std::size_t i = 0; i < n; ++i) {
            const char *it = std::find(order, order + Nd, dist_labels[i]);
            if (it != order + Nd) perm[dist_n++] = (int)(it - order);
        }
        for (std::size_t i = 0; i < Nd; ++i) {
            const char *it = std::find(dist_labels, dist_labels + n, order[i]);
            if (it == dist_labels + n) perm[dist_n++] = (int)i;
        }
        if (dist_n != Nd) throw Error("basic_partitioning: repeated labels");
    } else {
        for (std::size_t i = 0; i < Nd; ++i) perm[i] = (int)i;
    }

    // (the reference constructs this error without throwing it, dist.h:3400-3402, and then writes
    // past the end of its result; here it is thrown)
    if (nprocs >= 0 && vol_procs > nprocs)
        throw Error("The total number of processes from `procs` is greater than `nprocs`");
    if (ncomponents < 1) throw Error("basic_partitioning: invalid `ncomponents`");
    std::vector<Range> fs((std::size_t)(nprocs < 0 ? vol_procs : nprocs) * ncomponents,
                          Range{Coor(Nd, 0), Coor(Nd, 0)});
    Coor procs_perm(Nd);
    for (std::size_t i = 0; i < Nd; ++i) procs_perm[i] = procs[perm[i]];
    const std::vector<long> stride_perm = strides_slow_to_fast(procs_perm);
    for (int rank = 0; rank < vol_procs; ++rank) {
        Coor cproc(Nd);
        for (std::size_t i = 0; i < Nd; ++i)
            cproc[i] = (int)((rank / stride_perm[i]) % procs_perm[i]);
        Range fsi{Coor(Nd), Coor(Nd)};
        for (std::size_t i = 0; i < Nd; ++i) {
            const int d = dim[perm[i]], pp = procs_perm[i];
            fsi.size[perm[i]] = d / pp + (d % pp > cproc[i] ? 1 : 0);
            fsi.from[perm[i]] =
                fsi.size[perm[i]] == d ? 0 : d / pp * cproc[i] + std::min(cproc[i], d % pp);
        }
        if (volume(fsi.size) == 0) fsi = Range{Coor(Nd, 0), Coor(Nd, 0)};
        if (ncomponents == 1) {
            fs[rank] = fsi;
        } else {
            const Coor cp = partitioning_distributed_procs(
                order ? std::string(order) : std::string(Nd, '\0'), fsi.size,
                dist_labels ? std::string(dist_labels) : std::string(), (unsigned)ncomponents);
            auto comps = basic_partitioning(order, fsi.size, cp, dist_labels, ncomponents, 1);
            for (int c = 0; c < ncomponents; ++c) {
                Range &o = fs[(std::size_t)rank * ncomponents + c];
                o.size = comps[c].size;
                o.from.resize(Nd);
                for (std::size_t i = 0; i < Nd; ++i) o.from[i] = comps[c].from[i] + fsi.from[i];
                if (volume(o.size) == 0) o = Range{Coor(Nd, 0), Coor(Nd, 0)};
            }
        }
    }
    return fs;
}

std::vector<Range> basic_partitioning_ext(const Coor &dim, const Coor &procs, int nprocs,
                                          bool replicate, const Coor &ext_power) {
    const std::size_t Nd = dim.size();
    const int vol_procs = (int)volume(procs);
    for (std::size_t i = 0; i < Nd; ++i)
        if (ext_power[i] < 0) throw Error("Unsupported value for `power`");
    std::vector<Range> fs(nprocs < 0 ? vol_procs : nprocs, Range{Coor(Nd, 0), Coor(Nd, 0)});
    const std::vector<long> stride = strides_slow_to_fast(procs);
    for (int rank = 0; rank < vol_procs; ++rank) {
        for (std::size_t i = 0; i < Nd; ++i) {
            const int c = (int)((rank / stride[i]) % procs[i]);
            fs[rank].size[i] = std::min(
                dim[i] / procs[i] + (dim[i] % procs[i] > c ? 1 : 0) + ext_power[i] * 2, dim[i]);
            fs[rank].from[i] =
                fs[rank].size[i] == dim[i]
                    ? 0
                    : (dim[i] / procs[i] * c + std::min(c, dim[i] % procs[i]) - ext_power[i] +
                       dim[i]) %
                          dim[i];
        }
    }
    if (replicate && vol_procs == 1)
        for (auto &f : fs) f = fs[0];
    return fs;
}

/// Map coordinates of the copy region from tensor A (labels la) to tensor B (labels lb):
/// cB = fromB + (cA - fromA) for common labels, fromB for labels only in B
Range translate(const Range &r, const std::string &la, const Coor &fromA, const Coor &dimA,
                const std::string &lb, const Coor &fromB, const Coor &dimB) {
    Range o{Coor(lb.size()), Coor(lb.size())};
    for (std::size_t j = 0; j < lb.size(); ++j) {
        auto i = la.find(lb[j]);
        if (i == std::string::npos) {
            o.from[j] = fromB[j];
            o.size[j] = 1;
        } else {
            o.from[j] = normalize_coor(
                (long)normalize_coor((long)r.from[i] - fromA[i] + dimA[i], dimA[i]) + fromB[j],
                dimB[j]);
            o.size[j] = r.size[i];
        }
    }
    if (volume(o.size) == 0) o.size.assign(lb.size(), 0);
    return o;
}


} // namespace sbx
