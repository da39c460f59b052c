// Element arithmetic shared by the BSR and copy kernels: complex (double2 / float2, interleaved re/im
// as std::complex) and real types.  Alpha is passed as doubles (the ABI's scalar).
#pragma once

#include <hip/hip_runtime.h>

namespace sbx {
namespace {

template <typename E> struct Ops;
template <> struct Ops<double2> {
    static __device__ __forceinline__ double2 zero() { return double2{0, 0}; }
    static __device__ __forceinline__ double2 fma(double2 a, double2 b, double2 c) {
        return double2{c.x + a.x * b.x - a.y * b.y, c.y + a.x * b.y + a.y * b.x};
    }
    static __device__ __forceinline__ double2 scale(double2 v, double ar, double ai) {
        return double2{ar * v.x - ai * v.y, ar * v.y + ai * v.x};
    }
    static __device__ __forceinline__ double2 add(double2 a, double2 b) {
        return double2{a.x + b.x, a.y + b.y};
    }
    static __device__ __forceinline__ bool nonzero(double2 a) { return a.x != 0 || a.y != 0; }
};
template <> struct Ops<float2> {
    static __device__ __forceinline__ float2 zero() { return float2{0, 0}; }
    static __device__ __forceinline__ float2 fma(float2 a, float2 b, float2 c) {
        return float2{c.x + a.x * b.x - a.y * b.y, c.y + a.x * b.y + a.y * b.x};
    }
    static __device__ __forceinline__ float2 scale(float2 v, double ar, double ai) {
        return float2{(float)ar * v.x - (float)ai * v.y, (float)ar * v.y + (float)ai * v.x};
    }
    static __device__ __forceinline__ float2 add(float2 a, float2 b) {
        return float2{a.x + b.x, a.y + b.y};
    }
    static __device__ __forceinline__ bool nonzero(float2 a) { return a.x != 0 || a.y != 0; }
};
template <> struct Ops<double> {
    static __device__ __forceinline__ double zero() { return 0; }
    static __device__ __forceinline__ double fma(double a, double b, double c) { return c + a * b; }
    static __device__ __forceinline__ double scale(double v, double ar, double) { return ar * v; }
    static __device__ __forceinline__ double add(double a, double b) { return a + b; }
    static __device__ __forceinline__ bool nonzero(double a) { return a != 0; }
};
template <> struct Ops<float> {
    static __device__ __forceinline__ float zero() { return 0; }
    static __device__ __forceinline__ float fma(float a, float b, float c) { return c + a * b; }
    static __device__ __forceinline__ float scale(float v, double ar, double) {
        return (float)ar * v;
    }
    static __device__ __forceinline__ float add(float a, float b) { return a + b; }
    static __device__ __forceinline__ bool nonzero(float a) { return a != 0; }
};

/// Non-temporal (streaming) store of one element: the line is written through without being
/// kept in the caches (outputs written once and not re-read by the same kernel)
template <typename D> __device__ __forceinline__ void store_nt(D *p, D v) {
    if constexpr (sizeof(D) == 16) {
        typedef double v2 __attribute__((ext_vector_type(2)));
        v2 t;
        __builtin_memcpy(&t, &v, 16);
        __builtin_nontemporal_store(t, (v2 *)p);
    } else if constexpr (sizeof(D) == 8) {
        double t;
        __builtin_memcpy(&t, &v, 8);
        __builtin_nontemporal_store(t, (double *)p);
    } else {
        float t;
        __builtin_memcpy(&t, &v, 4);
        __builtin_nontemporal_store(t, (float *)p);
    }
}

/// Non-temporal (streaming) load of one element (data read once by the kernel)
template <typename D> __device__ __forceinline__ D load_nt(const D *p) {
    D v;
    if constexpr (sizeof(D) == 16) {
        typedef double v2 __attribute__((ext_vector_type(2)));
        const v2 t = __builtin_nontemporal_load((const v2 *)p);
        __builtin_memcpy(&v, &t, 16);
    } else if constexpr (sizeof(D) == 8) {
        const double t = __builtin_nontemporal_load((const double *)p);
        __builtin_memcpy(&v, &t, 8);
    } else {
        const float t = __builtin_nontemporal_load((const float *)p);
        __builtin_memcpy(&v, &t, 4);
    }
    return v;
}

} // namespace
} // namespace sbx
