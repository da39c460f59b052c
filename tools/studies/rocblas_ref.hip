// The reference's GPU path for the local contraction (blas.h:802-806:
// rocblas_gemm_strided_batched_ex, here rocblas_zgemm_strided_batched with the same arguments)
// timed on the lattice contraction shape (T,N m=n=256 k=12288 batch=16), for comparison with
// the library's MFMA kernel.  Not part of the product.
// Build: hipcc --offload-arch=gfx950 -O2 tools/studies/rocblas_ref.hip -lrocblas -o tools/rocblas_ref
#include <hip/hip_runtime.h>
#include <rocblas/rocblas.h>

#include <cstdio>
#include <vector>

__global__ void fill_kernel(double *p, long n, unsigned seed) {
    for (long i = blockIdx.x * 256L + threadIdx.x; i < n; i += (long)gridDim.x * 256L) {
        unsigned x = (unsigned)(i * 2654435761u) ^ seed;
        x ^= x >> 13;
        x *= 0x5bd1e995u;
        x ^= x >> 15;
        p[i] = (double)(x & 0xffffff) / 8388608.0 - 1.0;
    }
}

int main(int argc, char **argv) {
    const int m = 256, n = 256, k = 12288, batch = 16;
    const int reps = argc > 1 ? atoi(argv[1]) : 10;
    rocblas_double_complex *A, *B, *C;
    (void)hipMalloc(&A, sizeof(*A) * (size_t)m * k * batch);
    (void)hipMalloc(&B, sizeof(*B) * (size_t)n * k * batch);
    (void)hipMalloc(&C, sizeof(*C) * (size_t)m * n * batch);
    // the same random data as tools/studies/gemm_tune (uniform [-1, 1))
    fill_kernel<<<4096, 256>>>((double *)A, 2L * m * k * batch, 1);
    fill_kernel<<<4096, 256>>>((double *)B, 2L * n * k * batch, 2);
    rocblas_handle h;
    rocblas_create_handle(&h);
    const rocblas_double_complex alpha{1, 0}, beta{0, 0};
    auto call = [&]() {
        return rocblas_zgemm_strided_batched(h, rocblas_operation_transpose, rocblas_operation_none,
                                             m, n, k, &alpha, A, k, (rocblas_stride)m * k, B, k,
                                             (rocblas_stride)n * k, &beta, C, m,
                                             (rocblas_stride)m * n, batch);
    };
    if (call() != rocblas_status_success) {
        std::printf("rocblas error\n");
        return 1;
    }
    (void)hipDeviceSynchronize();
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    for (int rep = 0; rep < 3; ++rep) {
        (void)hipEventRecord(a, 0);
        for (int i = 0; i < reps; ++i) call();
        (void)hipEventRecord(b, 0);
        (void)hipEventSynchronize(b);
        float ms = 0;
        (void)hipEventElapsedTime(&ms, a, b);
        ms /= reps;
        std::printf("rocblas_zgemm_strided_batched T,N %dx%dx%d batch %d: %.3f ms  %.2f TFLOP/s\n",
                    m, n, k, batch, ms, 8.0 * m * n * (double)k * batch / (ms * 1e-3) / 1e12);
    }
    rocblas_destroy_handle(h);
    return 0;
}
