// The reference's GPU BSR product on MI355X (not part of the product): BSR<Gpu>::matvec calls
// hipsparseXbsrmm (bsr.h:855-928; dir ROW for !blockImFast, transB = T for a row-major x, a
// column-major y as its layout planner requires, bsr.h:792-793).  Runs the config-3 operator
// (16^4 periodic 9-point stencil, 3x3 color blocks, complex<double>) and its 12x12 spin x color
// variant at n = 1 / 12 / 64 right-hand sides; prints one JSON line per case with the kernel
// time (HIP events, 10 calls) and the library's algorithmic bytes of the same product.
//
// Build: hipcc --offload-arch=gfx950 -O2 tools/studies/hipsparse_bsr.cpp -lhipsparse -o tools/hipsparse_bsr
#include <hip/hip_runtime.h>
#include <hipsparse/hipsparse.h>

#include <cstdio>
#include <vector>

#define HIP(x)                                                                                    \
    do {                                                                                          \
        if ((x) != hipSuccess) {                                                                  \
            std::printf("{\"error\": \"hip at line %d\"}\n", __LINE__);                          \
            return 1;                                                                             \
        }                                                                                         \
    } while (0)
#define SP(x)                                                                                     \
    do {                                                                                          \
        if ((x) != HIPSPARSE_STATUS_SUCCESS) {                                                    \
            std::printf("{\"error\": \"hipsparse at line %d\"}\n", __LINE__);                    \
            return 1;                                                                             \
        }                                                                                         \
    } while (0)

static int run(hipsparseHandle_t h, int L, int b, int ncols) {
    const int V = L * L * L * L, nnzb = 9 * V;
    std::vector<int> rowptr(V + 1), col(nnzb);
    for (int s = 0; s < V; ++s) {
        rowptr[s] = 9 * s;
        int c[4] = {s / (L * L * L), s / (L * L) % L, s / L % L, s % L};
        int k = 0;
        col[9 * s + k++] = s;
        for (int d = 0; d < 4; ++d)
            for (int dir = -1; dir <= 1; dir += 2) {
                int q[4] = {c[0], c[1], c[2], c[3]};
                q[d] = (q[d] + dir + L) % L;
                col[9 * s + k++] = ((q[0] * L + q[1]) * L + q[2]) * L + q[3];
            }
    }
    rowptr[V] = nnzb;
    int *d_rp, *d_col;
    hipDoubleComplex *d_v, *d_x, *d_y;
    const size_t nv = (size_t)nnzb * b * b, nx = (size_t)V * b * ncols;
    HIP(hipMalloc(&d_rp, sizeof(int) * (V + 1)));
    HIP(hipMalloc(&d_col, sizeof(int) * nnzb));
    HIP(hipMalloc(&d_v, sizeof(hipDoubleComplex) * nv));
    HIP(hipMalloc(&d_x, sizeof(hipDoubleComplex) * nx));
    HIP(hipMalloc(&d_y, sizeof(hipDoubleComplex) * nx));
    HIP(hipMemcpy(d_rp, rowptr.data(), sizeof(int) * (V + 1), hipMemcpyHostToDevice));
    HIP(hipMemcpy(d_col, col.data(), sizeof(int) * nnzb, hipMemcpyHostToDevice));
    HIP(hipMemset(d_v, 0, sizeof(hipDoubleComplex) * nv));
    HIP(hipMemset(d_x, 0, sizeof(hipDoubleComplex) * nx));
    hipsparseMatDescr_t descr;
    SP(hipsparseCreateMatDescr(&descr));
    const hipDoubleComplex alpha{1, 0}, beta{0, 0};
    auto call = [&]() {
        // x row major (n fastest): B is x^T in column major, ldb = ncols; y column major
        return hipsparseZbsrmm(h, HIPSPARSE_DIRECTION_ROW, HIPSPARSE_OPERATION_NON_TRANSPOSE,
                               ncols > 1 ? HIPSPARSE_OPERATION_TRANSPOSE
                                         : HIPSPARSE_OPERATION_NON_TRANSPOSE,
                               V, ncols, V, nnzb, &alpha, descr, d_v, d_rp, d_col, b, d_x,
                               ncols > 1 ? ncols : V * b, &beta, d_y, V * b);
    };
    SP(call());
    HIP(hipDeviceSynchronize());
    hipEvent_t e0, e1;
    HIP(hipEventCreate(&e0));
    HIP(hipEventCreate(&e1));
    const int reps = 10;
    HIP(hipEventRecord(e0, 0));
    for (int r = 0; r < reps; ++r) SP(call());
    HIP(hipEventRecord(e1, 0));
    HIP(hipEventSynchronize(e1));
    float ms = 0;
    HIP(hipEventElapsedTime(&ms, e0, e1));
    const double t = ms / 1e3 / reps;
    const double bytes = 16.0 * ((double)nnzb * b * b + 2.0 * V * b * ncols) + 4.0 * (nnzb + V + 1);
    std::printf("{\"op\": \"hipsparseZbsrmm\", \"L\": %d, \"block\": %d, \"n\": %d, \"us\": %.2f, "
                "\"GBps\": %.1f, \"frac_hbm\": %.4f}\n",
                L, b, ncols, t * 1e6, bytes / t / 1e9, bytes / t / 8e12);
    (void)hipFree(d_rp);
    (void)hipFree(d_col);
    (void)hipFree(d_v);
    (void)hipFree(d_x);
    (void)hipFree(d_y);
    (void)hipsparseDestroyMatDescr(descr);
    return 0;
}

int main() {
    hipsparseHandle_t h;
    if (hipsparseCreate(&h) != HIPSPARSE_STATUS_SUCCESS) return 1;
    for (int n : {1, 12, 64})
        if (run(h, 16, 3, n)) return 1;
    if (run(h, 16, 12, 12)) return 1;
    (void)hipsparseDestroy(h);
    return 0;
}
