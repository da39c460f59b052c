// ref_bench.cpp -- CPU baseline harness around the REAL reference (test infrastructure only).
//
// Compiled by oracle/Makefile from this file plus the header-only reference sources under
// /root/reference/include (never copied into this repository), linked against the OpenBLAS
// that ships with scipy in this image.  Output goes to oracle/_ref/ only.  bench.py runs it on
// the GPU box's host cores to time the reference's own CPU path (cpu_baseline.kind =
// "reference") on a bounded sample of the benchmark workload.
//
// Usage: ref_bench contraction L n reps | permute L n reps | bsr L ncols reps
// Prints one JSON line.
#include "superbblas.h"

#include <chrono>
#include <complex>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <iostream>
#include <vector>

#ifdef _OPENMP
#include <omp.h>
#endif

using namespace superbblas;
using Z = std::complex<double>;

static double now() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch())
        .count();
}

static int threads() {
#ifdef _OPENMP
    return omp_get_max_threads();
#else
    return 1;
#endif
}

int main(int argc, char **argv) {
    if (argc < 5) {
        std::fprintf(stderr, "usage: %s contraction|permute|bsr L n reps\n", argv[0]);
        return 1;
    }
    const std::string what = argv[1];
    const int L = std::atoi(argv[2]), n = std::atoi(argv[3]), reps = std::atoi(argv[4]);
    Context cpu = createCpuContext();
    if (what == "contraction") {
        // dist.cpp:364-385 shape: tnsxyzc x tNSxyzc -> tNSns
        const Coor<7> d0{L, n, 4, L, L, L, 3};
        const Coor<5> dr{L, n, 4, n, 4};
        std::size_t v0n = detail::volume(d0), vrn = detail::volume(dr);
        std::vector<Z> a(v0n), b(v0n), c(vrn);
        for (std::size_t i = 0; i < v0n; ++i) {
            a[i] = Z(std::sin(0.1 * i), std::cos(0.3 * i));
            b[i] = Z(std::cos(0.2 * i), std::sin(0.7 * i));
        }
        std::vector<PartitionItem<7>> p0(1, PartitionItem<7>{Coor<7>{}, d0});
        std::vector<PartitionItem<5>> pr(1, PartitionItem<5>{Coor<5>{}, dr});
        const Z *pa = a.data(), *pb = b.data();
        Z *pc = c.data();
        auto run = [&] {
            contraction<7, 7, 5, Z>(Z{1}, p0.data(), {{}}, d0, d0, 1, "tnsxyzc", false, &pa, &cpu,
                                    p0.data(), {{}}, d0, d0, 1, "tNSxyzc", false, &pb, &cpu, Z{0},
                                    pr.data(), {{}}, dr, dr, 1, "tNSns", &pc, &cpu, SlowToFast);
        };
        run(); // warm-up
        double t = now();
        for (int r = 0; r < reps; ++r) run();
        t = (now() - t) / reps;
        const double flops = 8.0 * L * (double)L * L * L * 3 * (n * 4.0) * (n * 4.0);
        std::printf("{\"op\": \"contraction\", \"L\": %d, \"n\": %d, \"seconds\": %.6g, "
                    "\"gflops\": %.6g, \"threads\": %d, \"checksum\": %.17g}\n",
                    L, n, t, flops / t / 1e9, threads(), std::abs(c[0]) + std::abs(c[vrn - 1]));
    } else if (what == "permute") {
        // dist.cpp:237-266: xyztsc -> slice of tnsxyzc, for every n
        const Coor<6> d0{L, L, L, L, 4, 3};
        const Coor<7> d1{L, n, 4, L, L, L, 3};
        std::vector<Z> a(detail::volume(d0)), b(detail::volume(d1));
        for (std::size_t i = 0; i < a.size(); ++i) a[i] = Z((double)i, -(double)i);
        std::vector<PartitionItem<6>> p0(1, PartitionItem<6>{Coor<6>{}, d0});
        std::vector<PartitionItem<7>> p1(1, PartitionItem<7>{Coor<7>{}, d1});
        const Z *pa = a.data();
        Z *pb = b.data();
        auto run = [&] {
            for (int k = 0; k < n; ++k) {
                copy<6, 7, Z, Z>(1.0, p0.data(), 1, "xyztsc", Coor<6>{}, d0, d0, &pa, nullptr,
                                 &cpu, p1.data(), 1, "tnsxyzc", Coor<7>{0, k}, d1, &pb, nullptr,
                                 &cpu, SlowToFast, Copy);
            }
        };
        run();
        double t = now();
        for (int r = 0; r < reps; ++r) run();
        t = (now() - t) / reps;
        const double bytes = 32.0 * (double)b.size();
        std::printf("{\"op\": \"permute\", \"L\": %d, \"n\": %d, \"seconds\": %.6g, "
                    "\"gbps\": %.6g, \"threads\": %d}\n",
                    L, n, t, bytes / t / 1e9, threads());
    } else if (what == "bsr") {
        // config 3: 16^4 periodic 9-point stencil (tests/bsr.cpp:169-255), 3x3 color blocks,
        // n = the number of rhs, x pXYZTSCn -> y pxyztscn, the builtin CPU operator
        // (bsr.h:535-650: OpenMP over block rows, one small GEMM per nonzero block)
        const Coor<6> dim{L, L, L, L, 1, 3};
        const std::size_t V = (std::size_t)L * L * L * L;
        std::vector<IndexType> ii(V, 9);
        std::vector<Coor<6>> jj;
        for (std::size_t i = 0; i < V; ++i) {
            Coor<6> c{(int)(i / (L * L * L)), (int)(i / (L * L) % L), (int)(i / L % L),
                      (int)(i % L), 0, 0};
            jj.push_back(c);
            for (int d = 0; d < 4; ++d)
                for (int dir = -1; dir < 2; dir += 2) {
                    Coor<6> q = c;
                    q[d] = (q[d] + dir + L) % L;
                    jj.push_back(q);
                }
        }
        std::vector<Z> v(V * 9 * 9);
        for (std::size_t i = 0; i < v.size(); ++i) v[i] = Z(std::sin(0.1 * i), std::cos(0.3 * i));
        std::vector<PartitionItem<6>> pop(1, PartitionItem<6>{Coor<6>{}, dim});
        IndexType *iip = ii.data();
        Coor<6> *jjp = jj.data();
        const Z *vp = v.data();
        const Coor<6> block{1, 1, 1, 1, 1, 3};
        BSR_handle *op = nullptr;
        create_bsr<6, 6, Z>(pop.data(), dim, pop.data(), dim, 1, block, block, false, &iip, &jjp,
                            &vp, &cpu, SlowToFast, &op);
        const Coor<8> dx{1, L, L, L, L, 1, 3, n};
        std::vector<Z> x(detail::volume(dx)), y(detail::volume(dx));
        for (std::size_t i = 0; i < x.size(); ++i) x[i] = Z(std::cos(0.2 * i), std::sin(0.7 * i));
        std::vector<PartitionItem<8>> px(1, PartitionItem<8>{Coor<8>{}, dx});
        const Z *pxp = x.data();
        Z *pyp = y.data();
        auto run = [&] {
            bsr_krylov<6, 6, 8, 8, Z>(Z{1}, op, "xyztsc", "XYZTSC", px.data(), 1, "pXYZTSCn",
                                      Coor<8>{}, dx, dx, &pxp, Z{0}, px.data(), "pxyztscn",
                                      Coor<8>{}, dx, dx, 'p', &pyp, &cpu, SlowToFast);
        };
        run();
        double t = now();
        for (int r = 0; r < reps; ++r) run();
        t = (now() - t) / reps;
        destroy_bsr(op);
        // the library's algorithmic bytes of one application
        const double bytes = 16.0 * (81.0 * V + 2.0 * 3 * V * n) + 4.0 * (9.0 * V + V + 1);
        std::printf("{\"op\": \"bsr\", \"L\": %d, \"n\": %d, \"seconds\": %.6g, "
                    "\"gbps\": %.6g, \"gflops\": %.6g, \"threads\": %d}\n",
                    L, n, t, bytes / t / 1e9, 8.0 * 81 * V * n / t / 1e9, threads());
    } else {
        std::fprintf(stderr, "unknown op\n");
        return 1;
    }
    // SB_TRACK_TIME=1: the reference's own per-function timings (performance.h:356-518)
    reportTimings(std::cerr);
    return 0;
}
