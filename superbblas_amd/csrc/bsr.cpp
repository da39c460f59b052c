// BSR operator: creation and distributed application (bsr_krylov).
//
// Reference: create_bsr / get_bsr_components / get_bsr_indices (bsr.h:2440-2454, 1269-1354,
// 1424-1468), local_bsr_krylov_check (bsr.h:1589-1943), get_output_partition and
// detail::bsr_krylov (bsr.h:2020-2266).
//  * the image partition `pi` says which rows each component owns; the domain partition `pd`
//    (usually the image partition extended by the stencil halo) says which part of x each
//    component reads;  x is brought to the domain partition (the halo exchange), each
//    component runs the SpMM kernel, and the image pieces are copied/added into y.
//  * x / y are used in place when their partition and layout already match (the common case
//    of the lattice tests and the benchmarks); otherwise through temporaries.
//  * Kronecker operators (create_kron_bsr, bsr.h:2476-2490) carry one ki x kd matrix per
//    nonzero position of the block rows; x and y are then row major with the Kronecker labels
//    fastest, (D, d, C, kd) and (I, i, C, ki), the layout the reference's planner suggests for
//    them (bsr.h:1914-1928), and the local product runs kernels_bsr_kron.hip.
//  * contracting with the image side (x has the image labels) applies A^H: a conj-transposed
//    operator built on first use (make_transposed), whose overlapping image pieces are summed.
#include "plan.h"

#include <algorithm>
#include <mutex>
#include <functional>
#include <memory>

namespace sbx {

struct BsrComp {
    int dev = -1;
    long block_rows = 0;
    long x_rows = 0; // domain rows (elements) of the component
    int *ii = nullptr; // device CSR row pointers
    int *jj = nullptr; // device first domain index per nonzero block
    const void *v = nullptr;
    const void *kron = nullptr; // Kronecker matrices (user memory, device)
    int nnz_per_row = -1;
    std::vector<int> h_rowptr, h_jj; // host copies of the pattern (for the transposed operator)
    // site tiles of the 3x3 9-point kernels (bsr_ell9_tile_kernel): per schedule one device
    // buffer holding rows [chunks][tt], distinct block columns [chunks][umax], slots [chunks][tt][9]
    // ([0] 16-site tiles, [1] 8-site tiles)
    void *tile_buf[2] = {nullptr, nullptr};
    TileSched tiles[2];
    void *owned_v = nullptr;         // values owned by the operator (transposed operator, or
                                     // the device copy of a host component's values)
    void *owned_kron = nullptr;      // device copy of a host component's Kronecker matrices
    int *kron_perm = nullptr;        // Kronecker operators: block rows in the XCD order
    void *kron_terms = nullptr;      // ... the spin rows as two terms (build_kron_terms)
    void *kron_xor = nullptr;        // ... as diagonal + XOR partner (build_kron_terms)
    bool kron_terms_due = false;     // ... tables not built yet (built on the first launch that
                                     // asks for a spin-first kernel, bsr.kron_spin)
};

struct BsrOp {
    int nd = 0, ni = 0, dtype = SBX_CDOUBLE;
    Coor dimi, dimd, blocki, blockd;
    Coor kroni, krond; // all ones without Kronecker blocking
    bool is_kron = false;
    bool block_im_fast = false;
    int nprocs = 1, rank = 0, ncomponents = 1;
    std::vector<std::vector<Range>> pi, pd; // SlowToFast, all ranks
    std::vector<BsrComp> comps;             // this rank's components
    int co = SBX_SLOW_TO_FAST;
    bool image_overlaps = false; // image ranges of different components overlap (transposed op)
    mutable std::unique_ptr<BsrOp> transposed; // A^H, built on the first image-side contraction
    ~BsrOp() {
        for (auto &c : comps) {
            if (c.dev >= 0) {
                (void)hipSetDevice(c.dev);
                (void)hipStreamSynchronize(get_stream(c.dev));
            }
            if (c.ii) (void)hipFree(c.ii);
            if (c.jj) (void)hipFree(c.jj);
            if (c.owned_v) (void)hipFree(c.owned_v);
            if (c.owned_kron) (void)hipFree(c.owned_kron);
            for (void *b : c.tile_buf)
                if (b) (void)hipFree(b);
            if (c.kron_perm) (void)hipFree(c.kron_perm);
            if (c.kron_terms) (void)hipFree(c.kron_terms);
            if (c.kron_xor) (void)hipFree(c.kron_xor);
        }
    }
};

namespace {

/// The site-tile schedule of a 3x3-block operator with 9 nonzero blocks per row (the 9-point
/// stencils): the block rows are the component's image sites (SlowToFast over the image dims
/// without the block dims), grouped into tiles of up to TT sites -- 2 along each of the fastest
/// dims, 2x2x2x2 on a 4-d lattice for TT = 16, 2x2x2 for TT = 8 -- visited with the fastest tile
/// coordinate fastest; per tile its rows, its distinct block columns and the slot of each nonzero
/// block among them.  Any pattern is valid (a tile whose columns are scattered only stages more
/// rows); no schedule when a tile has more distinct columns than the kernel's LDS budget (umax_limit).
void build_tile_schedule(BsrComp &bc, const Coor &isize, const Coor &blocki, int which, int TT,
                         int UMAX_LIMIT) {
    constexpr int NNZ = 9;
    std::vector<long> dims;
    for (std::size_t d = 0; d < isize.size(); ++d) {
        const long r = blocki[d] > 0 ? isize[d] / blocki[d] : 1;
        if (r > 1) dims.push_back(r);
    }
    long vol = 1;
    for (long r : dims) vol *= r;
    if (vol != bc.block_rows || bc.h_jj.size() != (std::size_t)bc.block_rows * NNZ) return;
    const int nd = (int)dims.size();
    std::vector<long> tsz(nd, 1), ntile(nd, 1), rstride(nd, 1);
    long prod = 1;
    for (int pass = 0; pass < 4 && prod < TT; ++pass)
        for (int d = nd - 1; d >= 0 && prod < TT; --d)
            if (tsz[d] * 2 <= dims[d]) tsz[d] *= 2, prod *= 2;
    long nchunks = 1;
    for (int d = nd - 1; d >= 0; --d) {
        ntile[d] = (dims[d] + tsz[d] - 1) / tsz[d];
        nchunks *= ntile[d];
        if (d + 1 < nd) rstride[d] = rstride[d + 1] * dims[d + 1];
    }
    std::vector<int> rows((std::size_t)nchunks * TT, -1);
    std::vector<std::vector<int>> uniq(nchunks);
    std::vector<unsigned char> loc((std::size_t)nchunks * TT * NNZ, 255);
    int umax = 0;
    std::vector<long> tc(nd), lc(nd);
    for (long ch = 0; ch < nchunks; ++ch) {
        long rem = ch;
        for (int d = nd - 1; d >= 0; --d) tc[d] = rem % ntile[d], rem /= ntile[d];
        int nr = 0;
        for (long e = 0; e < prod; ++e) {
            long r2 = e, row = 0;
            bool in = true;
            for (int d = nd - 1; d >= 0; --d) {
                lc[d] = r2 % tsz[d], r2 /= tsz[d];
                const long cc = tc[d] * tsz[d] + lc[d];
                in &= cc < dims[d];
                row += cc * rstride[d];
            }
            if (in) rows[ch * TT + nr++] = (int)row;
        }
        std::vector<int> &u = uniq[ch];
        for (int q = 0; q < nr; ++q) {
            const long row = rows[ch * TT + q];
            for (int k = 0; k < NNZ; ++k) {
                const int j = bc.h_jj[row * NNZ + k];
                if (j < 0) continue;
                int at = (int)(std::find(u.begin(), u.end(), j) - u.begin());
                if (at == (int)u.size()) u.push_back(j);
                if (at >= UMAX_LIMIT) return;
                loc[(ch * TT + q) * NNZ + k] = (unsigned char)at;
            }
        }
        umax = std::max(umax, (int)u.size());
    }
    if (umax == 0) return;
    std::vector<int> flat((std::size_t)nchunks * umax, -1);
    for (long ch = 0; ch < nchunks; ++ch)
        std::copy(uniq[ch].begin(), uniq[ch].end(), flat.begin() + ch * umax);
    const std::size_t b_rows = rows.size() * sizeof(int), b_uniq = flat.size() * sizeof(int);
    const std::size_t total = b_rows + b_uniq + loc.size();
    SBX_HIP_CHECK(hipMalloc(&bc.tile_buf[which], total));
    char *b = (char *)bc.tile_buf[which];
    SBX_HIP_CHECK(hipMemcpy(b, rows.data(), b_rows, hipMemcpyHostToDevice));
    SBX_HIP_CHECK(hipMemcpy(b + b_rows, flat.data(), b_uniq, hipMemcpyHostToDevice));
    SBX_HIP_CHECK(hipMemcpy(b + b_rows + b_uniq, loc.data(), loc.size(), hipMemcpyHostToDevice));
    TileSched &t = bc.tiles[which];
    t.rows = (const int *)b;
    t.uniq = (const int *)(b + b_rows);
    t.loc = (const unsigned char *)(b + b_rows + b_uniq);
    t.umax = umax;
    t.tt = TT;
    t.chunks = nchunks;
}

/// The XCD order of a lattice operator's block rows (bsr_kron_spin_kernel): the rows are the
/// component's image sites (SlowToFast over the image dims without the blocked and
/// Kronecker-blocked ones); the lattice is cut into 8 boxes, halving the longest extent of every
/// box three times (the slowest dim on ties: 16^4 -> 8x8x8x16), the boxes laid end to end, each
/// in its natural order.  The kernel hands each XCD a contiguous eighth of the row slots, so an
/// XCD sweeps one box: the x sites its rows' neighbours share are read within a short distance
/// of each other (16^4: the slowest neighbour 1024 rows apart instead of 4096) and the box's
/// faces are the only sites two XCDs both fetch.  No order (nullptr) for a component that is not
/// a whole box of sites.
void build_kron_order(BsrComp &bc, const Coor &isize, const Coor &blocki, const Coor &kroni) {
    std::vector<long> dims;
    for (std::size_t d = 0; d < isize.size(); ++d) {
        const long r = isize[d] / std::max(1L, (long)blocki[d] * kroni[d]);
        if (r > 1) dims.push_back(r);
    }
    long vol = 1;
    for (long r : dims) vol *= r;
    if (dims.empty() || vol != bc.block_rows || vol < 64) return;
    const int nd = (int)dims.size();
    struct Box {
        std::vector<long> from, size;
    };
    std::vector<Box> boxes{Box{std::vector<long>(nd, 0), dims}};
    for (int cut = 0; cut < 3; ++cut) {
        std::vector<Box> next;
        for (const Box &b : boxes) {
            int at = 0;
            for (int d = 1; d < nd; ++d)
                if (b.size[d] > b.size[at]) at = d;
            if (b.size[at] < 2) {
                next.push_back(b);
                continue;
            }
            Box lo = b, hi = b;
            lo.size[at] = b.size[at] / 2;
            hi.from[at] = b.from[at] + lo.size[at];
            hi.size[at] = b.size[at] - lo.size[at];
            next.push_back(lo);
            next.push_back(hi);
        }
        boxes.swap(next);
    }
    std::vector<long> stride(nd, 1);
    for (int d = nd - 2; d >= 0; --d) stride[d] = stride[d + 1] * dims[d + 1];
    std::vector<int> perm;
    perm.reserve(vol);
    std::vector<long> c(nd);
    for (const Box &b : boxes) {
        long bv = 1;
        for (long e : b.size) bv *= e;
        for (long e = 0; e < bv; ++e) {
            long r = e, row = 0;
            for (int d = nd - 1; d >= 0; --d) {
                c[d] = r % b.size[d];
                r /= b.size[d];
                row += (b.from[d] + c[d]) * stride[d];
            }
            perm.push_back((int)row);
        }
    }
    SBX_HIP_CHECK(hipMalloc(&bc.kron_perm, sizeof(int) * vol));
    SBX_HIP_CHECK(hipMemcpy(bc.kron_perm, perm.data(), sizeof(int) * vol, hipMemcpyHostToDevice));
}

/// The 4x4 complex<double> spin matrices of a Kronecker operator with at most two nonzeros in
/// every row, as a table for bsr_kron_spin_kernel: per matrix mu and row a, two (spin index,
/// coefficient) terms (a row with one nonzero: the second coefficient zero; with none: both).
/// Built from the matrices on the first launch with bsr.kron_spin set (the default MFMA kernels
/// read the caller's matrices on every call and need no table), as a snapshot of the matrices at
/// that moment -- the reference analyses them at creation (kron_cpu, the density and the repeated
/// matrices, bsr.h:690-717); a caller who changes them in place afterwards must recreate the
/// operator for the spin-first kernels.  No table (the MFMA kernels run) when a row has more
/// nonzeros.
void build_kron_terms(BsrComp &bc, bool block_im_fast) {
    const int nnz = bc.nnz_per_row;
    if (nnz <= 0 || !bc.kron) return;
    std::vector<double> k((std::size_t)nnz * 32);
    SBX_HIP_CHECK(hipMemcpy(k.data(), bc.kron, k.size() * sizeof(double), hipMemcpyDefault));
    std::vector<double> coef((std::size_t)nnz * 16, 0.0);
    std::vector<int> bidx((std::size_t)nnz * 8, 0);
    for (int mu = 0; mu < nnz; ++mu)
        for (int a = 0; a < 4; ++a) {
            int t = 0;
            for (int b = 0; b < 4; ++b) {
                const std::size_t e = (std::size_t)mu * 16 + (block_im_fast ? a + 4 * b : 4 * a + b);
                const double re = k[2 * e], im = k[2 * e + 1];
                if (re == 0 && im == 0) continue;
                if (t == 2) return; // a third nonzero in the row
                coef[mu * 16 + 4 * a + 2 * t] = re;
                coef[mu * 16 + 4 * a + 2 * t + 1] = im;
                bidx[mu * 8 + 2 * a + t] = b;
                if (t == 0) bidx[mu * 8 + 2 * a + 1] = b;
                ++t;
            }
        }
    const std::size_t cb = coef.size() * sizeof(double), bb = bidx.size() * sizeof(int);
    SBX_HIP_CHECK(hipMalloc(&bc.kron_terms, cb + bb));
    SBX_HIP_CHECK(hipMemcpy(bc.kron_terms, coef.data(), cb, hipMemcpyHostToDevice));
    SBX_HIP_CHECK(hipMemcpy((char *)bc.kron_terms + cb, bidx.data(), bb, hipMemcpyHostToDevice));
    // the diagonal + XOR-partner form (bsr_kron_xor_kernel): row a nonzero at most at spins a and
    // a ^ s_mu, one s_mu per matrix; c0 the diagonal entry, c1 the partner's
    std::vector<double> xc((std::size_t)nnz * 16, 0.0);
    std::vector<int> xs(nnz, 0);
    for (int mu = 0; mu < nnz; ++mu) {
        auto at = [&](int a, int b) {
            const std::size_t e = (std::size_t)mu * 16 + (block_im_fast ? a + 4 * b : 4 * a + b);
            return std::make_pair(k[2 * e], k[2 * e + 1]);
        };
        int sm = 0;
        for (int a = 0; a < 4 && sm == 0; ++a)
            for (int b = 0; b < 4; ++b) {
                const auto v = at(a, b);
                if (b != a && (v.first != 0 || v.second != 0)) {
                    sm = a ^ b;
                    break;
                }
            }
        for (int a = 0; a < 4; ++a)
            for (int b = 0; b < 4; ++b) {
                const auto v = at(a, b);
                if (v.first == 0 && v.second == 0) continue;
                if (b == a) {
                    xc[mu * 16 + 4 * a] = v.first;
                    xc[mu * 16 + 4 * a + 1] = v.second;
                } else if (b == (a ^ sm)) {
                    xc[mu * 16 + 4 * a + 2] = v.first;
                    xc[mu * 16 + 4 * a + 3] = v.second;
                } else {
                    return; // not of that form
                }
            }
        xs[mu] = sm;
    }
    const std::size_t xcb = xc.size() * sizeof(double), xsb = xs.size() * sizeof(int);
    SBX_HIP_CHECK(hipMalloc(&bc.kron_xor, xcb + xsb));
    SBX_HIP_CHECK(hipMemcpy(bc.kron_xor, xc.data(), xcb, hipMemcpyHostToDevice));
    SBX_HIP_CHECK(hipMemcpy((char *)bc.kron_xor + xcb, xs.data(), xsb, hipMemcpyHostToDevice));
}

} // namespace

BsrOp *bsr_create(int nd, int ni, int dtype, const std::vector<std::vector<Range>> &pi,
                  const Coor &dimi, const std::vector<std::vector<Range>> &pd, const Coor &dimd,
                  const Coor &blocki, const Coor &blockd, bool block_im_fast,
                  const std::vector<const int *> &ii, const std::vector<const int *> &jj,
                  const std::vector<const void *> &v, const std::vector<int> &devs, bool reverse_jj,
                  const Comm &comm, const Coor *kroni, const Coor *krond,
                  const std::vector<const void *> *kronv) {
    std::unique_ptr<BsrOp> op(new BsrOp());
    op->is_kron = kronv != nullptr;
    op->kroni = op->is_kron ? *kroni : Coor(ni, 1);
    op->krond = op->is_kron ? *krond : Coor(nd, 1);
    if ((int)op->kroni.size() != ni || (int)op->krond.size() != nd)
        throw Error("create_kron_bsr: invalid Kronecker dimensions");
    for (int i = 0; i < nd; ++i)
        if (blockd[i] < 1 || op->krond[i] < 1 || (blockd[i] > 1 && op->krond[i] > 1))
            throw Error("Invalid simultaneous blocking and Kronecker blocking");
    for (int i = 0; i < ni; ++i)
        if (blocki[i] < 1 || op->kroni[i] < 1 || (blocki[i] > 1 && op->kroni[i] > 1))
            throw Error("Invalid simultaneous blocking and Kronecker blocking");
    op->nd = nd;
    op->ni = ni;
    op->dtype = dtype;
    op->dimi = dimi;
    op->dimd = dimd;
    op->blocki = blocki;
    op->blockd = blockd;
    op->block_im_fast = block_im_fast;
    op->nprocs = comm.nprocs;
    op->rank = comm.rank;
    op->pi = pi;
    op->pd = pd;
    const long bi = volume(blocki), bd = volume(blockd);
    const long ki = volume(op->kroni);
    const int ncomp = (int)pi[comm.rank].size();
    op->ncomponents = ncomp;
    for (int c = 0; c < ncomp; ++c) {
        BsrComp bc;
        bc.dev = devs[c];
        // a host (CPU-context) component: its pattern is read from the host and its values are
        // copied to the device the host tensors of bsr_krylov are mirrored to (the values are a
        // snapshot taken here, where the reference keeps reading the caller's host array)
        const bool host = bc.dev < 0;
        if (host) bc.dev = comm.device >= 0 ? comm.device : 0;
        const Range &ri = pi[comm.rank][c], &rd = pd[comm.rank][c];
        const long nii = bi > 0 ? volume(ri.size) / (bi * ki) : 0;
        bc.block_rows = nii;
        bc.x_rows = volume(rd.size) / std::max(1L, volume(op->krond));
        bc.v = v[c];
        if (op->is_kron) bc.kron = (*kronv)[c];
        if (nii == 0 || volume(rd.size) == 0) {
            bc.block_rows = 0;
            op->comps.push_back(bc);
            continue;
        }
        // ii: number of nonzero blocks per block row (host or device memory)
        std::vector<int> hii(nii);
        set_device(bc.dev);
        if (host)
            std::memcpy(hii.data(), ii[c], sizeof(int) * nii);
        else
            SBX_HIP_CHECK(hipMemcpy(hii.data(), ii[c], sizeof(int) * nii, hipMemcpyDefault));
        std::vector<int> rowptr(nii + 1, 0);
        bool same = true;
        for (long i = 0; i < nii; ++i) {
            rowptr[i + 1] = rowptr[i] + hii[i];
            same &= (hii[i] == hii[0]);
        }
        const long nnz = rowptr[nii];
        bc.nnz_per_row = same ? hii[0] : -1;
        std::vector<int> hjj_coor((std::size_t)nnz * nd);
        if (nnz > 0 && host)
            std::memcpy(hjj_coor.data(), jj[c], sizeof(int) * nnz * nd);
        else if (nnz > 0)
            SBX_HIP_CHECK(hipMemcpy(hjj_coor.data(), jj[c], sizeof(int) * nnz * nd,
                                    hipMemcpyDefault));
        if (host) {
            const std::size_t es = dtype_size(dtype);
            const std::size_t vbytes = es * (std::size_t)nnz * bi * bd;
            SBX_HIP_CHECK(hipMalloc(&bc.owned_v, std::max<std::size_t>(vbytes, 1)));
            if (vbytes) SBX_HIP_CHECK(hipMemcpy(bc.owned_v, v[c], vbytes, hipMemcpyHostToDevice));
            bc.v = bc.owned_v;
            if (op->is_kron) {
                const std::size_t kbytes =
                    es * (std::size_t)(same ? hii[0] : 0) * ki * volume(op->krond);
                SBX_HIP_CHECK(hipMalloc(&bc.owned_kron, std::max<std::size_t>(kbytes, 1)));
                if (kbytes)
                    SBX_HIP_CHECK(hipMemcpy(bc.owned_kron, (*kronv)[c], kbytes,
                                            hipMemcpyHostToDevice));
                bc.kron = bc.owned_kron;
            }
        }
        // linear domain index of each block (get_bsr_indices, bsr.h:1451-1459): periodic
        // coordinates over the component's domain dims; for Kronecker operators the index of
        // the domain site, over the dims that are neither blocked nor Kronecker-blocked
        // (get_kron_indices divides the linear index by bd*kd, bsr.h:1524-1527)
        if (op->is_kron && !same)
            throw Error("get_kron_indices: unsupported having a different number of nonzeros in "
                        "each row");
        Coor site_size = rd.size;
        if (op->is_kron)
            for (int d = 0; d < nd; ++d)
                if (blockd[d] > 1 || op->krond[d] > 1) site_size[d] = 1;
        const std::vector<long> st = strides_slow_to_fast(site_size);
        std::vector<int> hjj(nnz);
        bool minus_one = false;
        for (long k = 0; k < nnz; ++k) {
            const int *cc = &hjj_coor[(std::size_t)k * nd];
            const int first = cc[0]; // the user's first coordinate (bsr.h:1453)
            if (first == -1) {
                hjj[k] = -1;
                minus_one = true;
                continue;
            }
            long idx = 0;
            for (int d = 0; d < nd; ++d) {
                if (site_size[d] == 1) continue;
                const int coor = reverse_jj ? cc[nd - 1 - d] : cc[d];
                idx += (long)normalize_coor(coor, rd.size[d]) * st[d];
            }
            if (idx > 0x7fffffffL) throw Error("Ups! IndexType isn't big enough");
            hjj[k] = (int)idx;
        }
        if (minus_one && op->is_kron)
            throw Error("get_kron_indices: unsupported nonzero pattern specification, some domain "
                        "coordinates have -1");
        if (minus_one && !same)
            throw Error("bsr: unsupported nonzero pattern specification, some domain coordinates "
                        "have -1 but not all block rows have the same number of nonzero blocks");
        SBX_HIP_CHECK(hipMalloc(&bc.ii, sizeof(int) * (nii + 1)));
        SBX_HIP_CHECK(hipMalloc(&bc.jj, sizeof(int) * std::max(1L, nnz)));
        SBX_HIP_CHECK(hipMemcpy(bc.ii, rowptr.data(), sizeof(int) * (nii + 1), hipMemcpyHostToDevice));
        if (nnz > 0)
            SBX_HIP_CHECK(hipMemcpy(bc.jj, hjj.data(), sizeof(int) * nnz, hipMemcpyHostToDevice));
        if (op->is_kron && volume(op->kroni) == 4 && volume(op->krond) == 4 && bi == 3 && bd == 3 &&
            dtype == SBX_CDOUBLE) {
            build_kron_order(bc, ri.size, blocki, op->kroni);
            bc.kron_terms_due = true;
        }
        if (!op->is_kron) {
            bc.h_rowptr = std::move(rowptr);
            bc.h_jj = std::move(hjj);
            if (bi == 3 && bd == 3 && bc.nnz_per_row == 9 && dtype == SBX_CDOUBLE) {
                // (the kernels' LDS budgets: 16 sites x 8 columns up to 116 staged rows, 8 sites
                // x 16 columns up to 80)
                build_tile_schedule(bc, ri.size, blocki, 0, 16, 116);
                build_tile_schedule(bc, ri.size, blocki, 1, 8, 80);
            }
        }
        op->comps.push_back(bc);
    }
    return op.release();
}

namespace {

/// The conjugate transpose A^H of a (non-Kronecker) operator, for contractions with the image
/// side of A (the reference's transSp: hipsparse bsrmm with CONJUGATE_TRANSPOSE,
/// bsr.h:1001-1029, 1942): image partition = A's domain partition (which may overlap across
/// components: the halos), domain partition = A's image partition, blocks conj-transposed and
/// regrouped by block column.
BsrOp *make_transposed(const BsrOp &a) {
    if (a.is_kron) throw Error("bsr_krylov: contracting with the image space of a Kronecker operator is not supported");
    std::unique_ptr<BsrOp> t(new BsrOp());
    t->nd = a.ni;
    t->ni = a.nd;
    t->dtype = a.dtype;
    t->dimi = a.dimd;
    t->dimd = a.dimi;
    t->blocki = a.blockd;
    t->blockd = a.blocki;
    t->kroni = a.krond;
    t->krond = a.kroni;
    t->block_im_fast = !a.block_im_fast; // the same block storage read transposed
    t->nprocs = a.nprocs;
    t->rank = a.rank;
    t->ncomponents = a.ncomponents;
    t->pi = a.pd;
    t->pd = a.pi;
    t->co = a.co;
    // do image ranges (A's domain ranges) of different components overlap?
    std::vector<Range> all;
    for (auto &r : a.pd)
        for (auto &q : r) all.push_back(q);
    for (std::size_t i = 0; i < all.size() && !t->image_overlaps; ++i)
        for (std::size_t j = i + 1; j < all.size(); ++j)
            if (volume(all[i].size) > 0 && volume(all[j].size) > 0 &&
                !intersection(all[i], all[j], a.dimd).empty()) {
                t->image_overlaps = true;
                break;
            }
    const long bi = volume(a.blocki), bd = volume(a.blockd);
    const std::size_t es = dtype_size(a.dtype);
    for (int c = 0; c < (int)a.comps.size(); ++c) {
        const BsrComp &ac = a.comps[c];
        BsrComp bc;
        bc.dev = ac.dev;
        const Range &rd = a.pd[a.rank][c];
        const long ncb = bd > 0 ? volume(rd.size) / bd : 0; // A's block columns = A^H's block rows
        if (ac.block_rows == 0 || ncb == 0) {
            t->comps.push_back(bc);
            continue;
        }
        bc.block_rows = ncb;
        // A^H's domain rows (elements) = A's image component (the DMA / split kernels bound
        // their x reads by it)
        bc.x_rows = volume(a.pi[a.rank][c].size) / std::max(1L, volume(a.kroni));
        const std::vector<int> &rp = ac.h_rowptr, &jj = ac.h_jj;
        std::vector<int> cnt(ncb + 1, 0);
        for (int k = 0; k < rp.back(); ++k)
            if (jj[k] >= 0) ++cnt[jj[k] / bd + 1];
        for (long q = 0; q < ncb; ++q) cnt[q + 1] += cnt[q];
        const int nnz = cnt[ncb];
        std::vector<int> pos(cnt.begin(), cnt.end() - 1), tjj(std::max(nnz, 1)), perm(std::max(nnz, 1));
        for (long i = 0; i < ac.block_rows; ++i)
            for (int k = rp[i]; k < rp[i + 1]; ++k) {
                if (jj[k] < 0) continue;
                const int q = pos[jj[k] / bd]++;
                tjj[q] = (int)(i * bi); // first element of A's block row i
                perm[q] = k;
            }
        bool same = true;
        for (long q = 0; q < ncb; ++q) same &= (cnt[q + 1] - cnt[q] == cnt[1] - cnt[0]);
        bc.nnz_per_row = same ? cnt[1] - cnt[0] : -1;
        set_device(bc.dev);
        SBX_HIP_CHECK(hipMalloc(&bc.ii, sizeof(int) * (ncb + 1)));
        SBX_HIP_CHECK(hipMalloc(&bc.jj, sizeof(int) * std::max(nnz, 1)));
        SBX_HIP_CHECK(hipMemcpy(bc.ii, cnt.data(), sizeof(int) * (ncb + 1), hipMemcpyHostToDevice));
        SBX_HIP_CHECK(hipMemcpy(bc.jj, tjj.data(), sizeof(int) * std::max(nnz, 1), hipMemcpyHostToDevice));
        // values: block perm[q] of A, conjugated, at position q
        SBX_HIP_CHECK(hipMalloc(&bc.owned_v, es * bi * bd * std::max(nnz, 1)));
        Scratch dperm(sizeof(int) * std::max(nnz, 1), bc.dev);
        SBX_HIP_CHECK(hipMemcpyAsync(dperm.ptr, perm.data(), sizeof(int) * std::max(nnz, 1),
                                     hipMemcpyHostToDevice, get_stream(bc.dev)));
        launch_gather_blocks(a.dtype, ac.v, (const int *)dperm.ptr, nnz, bi * bd, true,
                             bc.owned_v, bc.dev);
        SBX_HIP_CHECK(hipStreamSynchronize(get_stream(bc.dev)));
        bc.v = bc.owned_v;
        t->comps.push_back(std::move(bc));
    }
    return t.release();
}

} // namespace

void bsr_destroy(BsrOp *op) { delete op; }

namespace {

struct Group {
    bool ok;
    long stride, vol;
};
Group group_of(const std::string &group, const std::string &labels, const Coor &size) {
    const std::vector<long> st = strides_slow_to_fast(size);
    Group g{true, 0, 1};
    int prev = -1;
    for (char c : group) {
        auto i = labels.find(c);
        if (i == std::string::npos) return Group{false, 0, 0};
        if (size[i] == 1) continue;
        g.vol *= size[i];
        if (prev >= 0 && st[prev] != st[i] * (long)size[i]) g.ok = false;
        prev = (int)i;
    }
    if (prev >= 0) g.stride = st[prev];
    return g;
}

/// Dense layout of a (domain-or-image labels, C labels) array: row major (C fastest) or column
/// major (C slowest); ld is the stride of the slow group
struct Layout {
    bool ok, row_major;
    long ld;
};
Layout dense_layout(const std::string &spatial, const std::string &cl, const std::string &labels,
                    const Coor &size) {
    const Group gs = group_of(spatial, labels, size), gc = group_of(cl, labels, size);
    if (!gs.ok || !gc.ok) return Layout{false, false, 0};
    const long vs = gs.vol, vc = gc.vol;
    if (vc <= 1) return Layout{gs.stride == 1 || vs <= 1, true, 1};
    if (vs <= 1) return Layout{true, true, 1};
    if (gc.stride == 1 && gs.stride == vc) return Layout{true, true, vc};
    if (gs.stride == 1 && gc.stride == vs) return Layout{true, false, vs};
    return Layout{false, false, 0};
}

} // namespace

void bsr_krylov(const BsrOp &op, const Scalar &alpha, const std::string &oi,
                const std::string &od, const DistTensor &x_in, const Coor &fromx,
                const Coor &sizex, const Scalar &beta, const DistTensor &y_in, const Coor &fromy,
                const Coor &sizey, char okr, const Comm &comm_in, bool just_local,
                std::function<void()> *deferred) {
    if (deferred) *deferred = nullptr;
    if ((int)oi.size() != op.ni || (int)od.size() != op.nd)
        throw Error("bsr_krylov: labels don't match the operator");
    if (comm_in.nprocs != op.nprocs) throw Error("bsr_krylov: communicator mismatch");
    // just_local (bsr.h:2020-2075, 2188): only this rank's part of the product, no exchange --
    // the other ranks' components are ignored and every copy stays on this process
    const bool local_only = just_local && comm_in.nprocs > 1;
    if (debug_level() > 0 && comm_in.nprocs > 1 && !local_only) { // check_consistency (bsr.h:2123)
        Hasher h;
        h.add(std::string("bsr_krylov"));
        h.add(alpha);
        h.add(beta);
        h.add(oi);
        h.add(od);
        h.add(x_in);
        h.add(fromx);
        h.add(sizex);
        h.add(y_in);
        h.add(fromy);
        h.add(sizey);
        h.add((long)okr);
        check_consistency(h, "bsr_krylov", comm_in);
    }
    Comm comm = comm_in;
    DistTensor x = x_in, y = y_in;
    const int base = local_only ? op.rank : 0; // op.pi / op.pd index of rank 0 of `comm`
    if (local_only) {
        comm.nprocs = 1;
        comm.rank = 0;
        comm.nccl = nullptr;
        comm.host_fn = nullptr;
        comm.stage = nullptr;
        x.ranges = {x_in.ranges[comm_in.rank]};
        y.ranges = {y_in.ranges[comm_in.rank]};
    }
    // Contraction with the image side (x has image labels, y domain labels): y = alpha A^H x,
    // applied as the transposed operator (bsr.h:1737-1760 kinds, 1942 transSp)
    bool x_image = false, x_domain = false;
    for (char c : x.labels) {
        x_image |= oi.find(c) != std::string::npos;
        x_domain |= od.find(c) != std::string::npos;
    }
    if (x_image && x_domain)
        throw Error("Unsupported to contract dense input tensor with domain and image dimensions "
                    "of the sparse tensor");
    if (x_image) {
        if (!op.transposed) op.transposed.reset(make_transposed(op));
        return bsr_krylov(*op.transposed, alpha, od, oi, x_in, fromx, sizex, beta, y_in, fromy,
                          sizey, okr, comm_in, just_local, deferred);
    }
    // Label classes (bsr.h:1722-1795): x has domain labels + C (+ okr); y image labels + C (+okr)
    std::string C;
    for (int i = 0; i < x.nd(); ++i) {
        const char c = x.labels[i];
        if (od.find(c) != std::string::npos) {
            if (sizex[i] != op.dimd[od.find(c)])
                throw Error("bsr_krylov: dimensions of the dense input tensor doesn't match the "
                            "sparse tensor");
            continue;
        }
        if (okr != 0 && c == okr) {
            if (sizex[i] > 1)
                throw Error("The power dimension on the input vector has a size larger than one");
            continue;
        }
        if (y.labels.find(c) == std::string::npos)
            throw Error("Dimension label for the dense input vector doesn't match the input "
                        "sparse dimensions nor the dense output dimensions");
        C += c;
    }
    int power = 1;
    for (int i = 0; i < y.nd(); ++i) {
        const char c = y.labels[i];
        if (oi.find(c) != std::string::npos) {
            if (sizey[i] != op.dimi[oi.find(c)])
                throw Error("bsr_krylov: dimensions of the dense output tensor doesn't match the "
                            "sparse tensor");
        } else if (okr != 0 && c == okr) {
            power = sizey[i];
        } else if (C.find(c) == std::string::npos) {
            throw Error("Dimension label for the dense output vector doesn't match the input "
                        "sparse dimensions nor the dense input dimensions");
        } else if (sizey[i] != sizex[x.labels.find(c)]) {
            throw Error("bsr_krylov: dimensions of the dense output tensor doesn't match");
        }
    }
    // Powers (bsr.h:2138-2147, 2211-2247): y[.., p, ..] = alpha * A^(p+1) x; the operator must map
    // the domain onto itself
    if (power > 1 && (op.dimi != op.dimd || op.blocki != op.blockd || op.kroni != op.krond))
        throw Error("When using powers the domain and the image of the sparse operator should be "
                    "the same");
    for (int i = 0; i < op.nd; ++i)
        if ((op.blockd[i] > 1 && op.blockd[i] != op.dimd[i]) ||
            (op.krond[i] > 1 && op.krond[i] != op.dimd[i]))
            throw Error("Still not supported partially blocking a dimension");
    for (int i = 0; i < op.ni; ++i)
        if ((op.blocki[i] > 1 && op.blocki[i] != op.dimi[i]) ||
            (op.kroni[i] > 1 && op.kroni[i] != op.dimi[i]))
            throw Error("Still not supported partially blocking a dimension");
    if (x.dtype != op.dtype || y.dtype != op.dtype) throw Error("bsr_krylov: type mismatch");
    const int dtype = op.dtype;
    const std::size_t es = dtype_size(dtype);
    const int bi = (int)volume(op.blocki), bd = (int)volume(op.blockd);

    // Temporaries' layouts, row major (C fastest but for the Kronecker labels): od + C / oi + C,
    // or (D, d, C, kd) / (I, i, C, ki) for Kronecker operators (bsr.h:1914-1928)
    std::string lx = od + C, ly = oi + C;
    if (op.is_kron) {
        auto split = [&](const std::string &o, const Coor &blk, const Coor &kr) {
            std::string S, b, k;
            for (std::size_t i = 0; i < o.size(); ++i)
                (blk[i] > 1 ? b : kr[i] > 1 ? k : S) += o[i];
            return S + b + C + k;
        };
        lx = split(od, op.blockd, op.krond);
        ly = split(oi, op.blocki, op.kroni);
    }
    Coor sizeC(C.size());
    for (std::size_t k = 0; k < C.size(); ++k) sizeC[k] = sizex[x.labels.find(C[k])];
    const long volC = volume(sizeC);
    const Coor zeroC(C.size(), 0);
    // a coordinate in a temporary's label order from its operator-side and C-side parts
    auto arrange = [&](const std::string &lab, const std::string &o, const Coor &opv,
                       const Coor &cv) {
        Coor r(lab.size());
        for (std::size_t k = 0; k < lab.size(); ++k) {
            const auto pos = o.find(lab[k]);
            r[k] = pos != std::string::npos ? opv[pos] : cv[C.find(lab[k])];
        }
        return r;
    };
    // whether a user piece can be the kernel's operand as it is
    auto operand_layout = [&](const std::string &spatial, const std::string &order,
                              const std::string &labels, const Coor &size) {
        if (!op.is_kron) return dense_layout(spatial, C, labels, size);
        const Group g = group_of(order, labels, size);
        return Layout{g.ok && (g.vol <= 1 || g.stride == 1), true, 0};
    };

    // x_ / y_ in coordinates relative to the regions (domain coord d <-> x coord fromx + d)
    DistTensor tx, ty;
    tx.labels = lx;
    ty.labels = ly;
    tx.dim = arrange(lx, od, op.dimd, sizeC);
    ty.dim = arrange(ly, oi, op.dimi, sizeC);
    tx.dtype = ty.dtype = dtype;
    tx.ranges.resize(comm.nprocs);
    ty.ranges.resize(comm.nprocs);
    // needed x range of each component (in x coordinates) and direct-use decisions
    struct CompPlan {
        bool xdirect = false, ydirect = false;
        int xi = -1, yi = -1;
        Layout lxl{}, lyl{};
    };
    std::vector<std::vector<CompPlan>> plans(comm.nprocs);
    auto bufs_p = std::make_shared<std::vector<Scratch>>(); // temporaries (live until the end)
    std::vector<Scratch> &bufs = *bufs_p;
    bufs.reserve(4 * op.pi[op.rank].size());
    std::vector<void *> my_x, my_y;
    std::vector<Layout> my_lx, my_ly;
    for (int rk = 0; rk < comm.nprocs; ++rk) {
        for (int c = 0; c < (int)op.pi[base + rk].size(); ++c) {
            const Range &rd = op.pd[base + rk][c], &ri = op.pi[base + rk][c];
            const Range nx{arrange(lx, od, rd.from, zeroC), arrange(lx, od, rd.size, sizeC)};
            const Range ny{arrange(ly, oi, ri.from, zeroC), arrange(ly, oi, ri.size, sizeC)};
            CompPlan cp;
            // x in place: same rank component whose range (shifted by fromx) equals nx (with
            // powers x's temporary is overwritten by every power, so x is always copied)
            if (power == 1 && rk < (int)x.ranges.size())
                for (int j = 0; j < (int)x.ranges[rk].size(); ++j) {
                    const Range &r = x.ranges[rk][j];
                    bool eq = true;
                    for (int i = 0; i < x.nd() && eq; ++i) {
                        const char l = x.labels[i];
                        auto k = lx.find(l);
                        if (k == std::string::npos) { // okr label
                            eq = r.size[i] == 1 && r.from[i] == fromx[i];
                            continue;
                        }
                        eq = r.size[i] == nx.size[k] &&
                             normalize_coor((long)r.from[i] - fromx[i], x.dim[i]) == nx.from[k];
                    }
                    if (!eq) continue;
                    Layout l = operand_layout(od, lx, x.labels, r.size);
                    if (!l.ok) continue;
                    if (comm.nprocs == 1 && rk == comm.rank && x.dev[j] != op.comps[c].dev) continue;
                    cp.xdirect = true;
                    cp.xi = j;
                    cp.lxl = l;
                    break;
                }
            if (!cp.xdirect) tx.ranges[rk].push_back(nx);
            if (power == 1 && rk < (int)y.ranges.size())
                for (int j = 0; j < (int)y.ranges[rk].size(); ++j) {
                    const Range &r = y.ranges[rk][j];
                    bool eq = true;
                    for (int i = 0; i < y.nd() && eq; ++i) {
                        const char l = y.labels[i];
                        auto k = ly.find(l);
                        if (k == std::string::npos) {
                            eq = r.size[i] == 1 && r.from[i] == fromy[i];
                            continue;
                        }
                        eq = r.size[i] == ny.size[k] &&
                             normalize_coor((long)r.from[i] - fromy[i], y.dim[i]) == ny.from[k];
                    }
                    if (!eq) continue;
                    Layout l = operand_layout(oi, ly, y.labels, r.size);
                    if (!l.ok) continue;
                    if (comm.nprocs == 1 && rk == comm.rank && y.dev[j] != op.comps[c].dev) continue;
                    // the output region must be exactly this component and no other component
                    // of y may overlap it (replicas need the copy path)
                    cp.ydirect = y.ranges[rk].size() == 1 && comm.nprocs == 1;
                    cp.yi = j;
                    cp.lyl = l;
                    break;
                }
            if (!cp.ydirect) ty.ranges[rk].push_back(ny);
            if (rk == comm.rank) {
                const int dev = op.comps[c].dev;
                if (cp.xdirect) {
                    my_x.push_back(x.ptr[cp.xi]);
                    my_lx.push_back(cp.lxl);
                } else {
                    bufs.emplace_back(volume(nx.size) * es, dev);
                    tx.ptr.push_back(bufs.back().ptr);
                    tx.dev.push_back(dev);
                    my_x.push_back(bufs.back().ptr);
                    my_lx.push_back(Layout{true, true, volC});
                }
                if (cp.ydirect) {
                    my_y.push_back(y.ptr[cp.yi]);
                    my_ly.push_back(cp.lyl);
                } else {
                    bufs.emplace_back(volume(ny.size) * es, dev);
                    ty.ptr.push_back(bufs.back().ptr);
                    ty.dev.push_back(dev);
                    my_y.push_back(bufs.back().ptr);
                    my_ly.push_back(Layout{true, true, volC});
                }
            }
            plans[rk].push_back(cp);
        }
    }

    // Bring x to the domain partition (halo exchange)
    bool need_x = false, need_y = false;
    for (auto &r : tx.ranges) need_x |= !r.empty();
    for (auto &r : ty.ranges) need_y |= !r.empty();
    std::function<void()> x_pending; // the halo exchange's unpack, when deferred
    if (need_x) {
        Coor from1(lx.size(), 0);
        dist_copy(Scalar{1, 0}, x, fromx, sizex, tx, from1, false, comm,
                  deferred ? &x_pending : nullptr);
    }
    // Output scaling (before the product, on the library stream)
    const bool direct_all = !need_y;
    if (direct_all && !beta.is_zero() && !beta.is_one())
        dist_copy(beta, y, fromy, sizey, y, fromy, false, comm);
    if (need_y && !beta.is_zero() && !beta.is_one())
        dist_copy(beta, y, fromy, sizey, y, fromy, false, comm);
    // overlapping image pieces (A^H with a halo domain) are summed: add into a zeroed output
    const bool add_y = !beta.is_zero() || op.image_overlaps;
    if (need_y && beta.is_zero() && op.image_overlaps)
        dist_copy(Scalar{0, 0}, y, fromy, sizey, y, fromy, false, comm);

    // the local products and the output copies; deferred behind the halo exchange when asked
    // (the reference's bsr_req, bsr.h:2199-2257)
    const BsrOp *opp = &op;
    auto product = [=]() {
        const BsrOp &op = *opp;
        std::vector<Scratch> &keep = *bufs_p; // temporaries stay alive through the product
        (void)keep;
        if (x_pending) x_pending();
        const Coor from0(ly.size(), 0), size0 = ty.dim;
        const int power_pos = okr != 0 ? (int)y.labels.find(okr) : -1;
        for (int pw = 0; pw < power; ++pw) {
            // Local SpMM
            for (int c = 0; c < (int)op.comps.size(); ++c) {
                const BsrComp &bc = op.comps[c];
                if (bc.block_rows == 0) continue;
                BsrDesc d;
                d.t = dtype;
                d.block_rows = bc.block_rows;
                d.bi = bi;
                d.bd = bd;
                d.ii = bc.ii;
                d.jj = bc.jj;
                d.v = bc.v;
                d.block_im_fast = op.block_im_fast;
                d.num_nnz_per_row = bc.nnz_per_row;
                d.x = my_x[c];
                d.x_rows = bc.x_rows;
                d.x_row_major = my_lx[c].row_major;
                d.ldx = my_lx[c].ld;
                d.y = my_y[c];
                d.y_row_major = my_ly[c].row_major;
                d.ldy = my_ly[c].ld;
                d.ncols = volC;
                d.alpha = pw == 0 ? alpha : Scalar{1, 0};
                d.add = plans[comm.rank][c].ydirect ? !beta.is_zero() : false;
                d.tiles[0] = bc.tiles[0];
                d.tiles[1] = bc.tiles[1];
                if (op.is_kron) {
                    d.ki = (int)volume(op.kroni);
                    d.kd = (int)volume(op.krond);
                    d.kron = bc.kron;
                    d.kron_perm = bc.kron_perm;
                    if (bc.kron_terms_due && g_bsr_tune.kron_spin > 0) {
                        // (first spin-first launch: the tables; one host thread at a time)
                        static std::mutex mu;
                        std::lock_guard<std::mutex> lock(mu);
                        BsrComp &mc = const_cast<BsrComp &>(bc);
                        if (mc.kron_terms_due) {
                            SBX_HIP_CHECK(hipStreamSynchronize(get_stream(bc.dev)));
                            build_kron_terms(mc, op.block_im_fast);
                            mc.kron_terms_due = false;
                        }
                    }
                    d.kron_terms = bc.kron_terms;
                    d.kron_xor = bc.kron_xor;
                    launch_bsr_kron(d, bc.dev);
                } else {
                    launch_bsr(d, bc.dev);
                }
            }
            // Copy/add the image pieces into y (power pw at okr = fromy[okr] + pw)
            if (need_y) {
                Coor fy = fromy;
                if (power_pos >= 0)
                    fy[power_pos] = (int)normalize_coor((long)fy[power_pos] + pw, y.dim[power_pos]);
                dist_copy(Scalar{1, 0}, ty, from0, size0, y, fy, add_y, comm);
            }
            if (pw + 1 == power) break;
            // The next power applies the operator to this one: the image pieces, relabelled as
            // domain coordinates, become x (with the halo of the domain partition)
            DistTensor ty_as_x = ty;
            for (char &ch : ty_as_x.labels)
                if (oi.find(ch) != std::string::npos) ch = od[oi.find(ch)];
            Coor zx(lx.size(), 0);
            if (op.image_overlaps) {
                dist_copy(Scalar{0, 0}, tx, zx, tx.dim, tx, zx, false, comm);
                dist_copy(Scalar{1, 0}, ty_as_x, zx, size0, tx, zx, true, comm);
            } else {
                dist_copy(Scalar{1, 0}, ty_as_x, zx, size0, tx, zx, false, comm);
            }
        }

    };
    if (deferred && x_pending)
        *deferred = product;
    else
        product();
}

} // namespace sbx
