// dc_ratio.hip -- the reference's compression-ratio estimators on the GPU (impl/dataCompression.c
// CT2/CT3: calCompressRatio_bitwise_{float,double,double2} :3622-3739, calcCompressionRatio_sz_{float,double}
// :4636-4771 / :4928-5063, calcCompressionRatio_nolossy_performance_{float,double} :4772-4840 /
// :5064-5132, calcCompressionRatio_nolossy_area_{float,double} :4841-4927 / :5133-5219).
//
// Every estimator is a left-to-right loop whose per-element bit count depends only on the element and
// the three (four) ORIGINAL elements before it -- except through the reference's "-1 means empty"
// history sentinel.  So: one data-parallel pass computes every element's bits (sum reduced with 64-bit
// atomics) and flags an input holding -1.0; such an input is re-estimated by one lane that runs the
// reference loop exactly.  The "area" estimators pack the per-element sizes greedily into 512-bit
// blocks, a sequential rule: the parallel pass stores each element's size (one byte) and one lane packs.
// byte_or_bit is the reference header's 2 (bit granularity, impl/dataCompression.h:24).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "dc_shared.h"

namespace dcr {

enum { R_BITWISE = 0, R_BITWISE_D2 = 1, R_SZ = 2, R_PERF = 3, R_AREA = 4 };

template <typename T> struct FPB;
template <> struct FPB<float> {
    static constexpr int EB = 8, BIAS = 127, MB = 23, W = 32;
    __device__ static int expo(float v) { return (int)((__float_as_uint(v) >> 23) & 0xFFu); }
    __device__ static uint64_t bits(float v) { return __float_as_uint(v); }
    __device__ static uint64_t binview(float v) { return __float_as_uint(v); }  // getFloatBin (c:5220)
    __device__ static float mul(float a, float b) { return __fmul_rn(a, b); }
    __device__ static float sub(float a, float b) { return __fsub_rn(a, b); }
    __device__ static float add(float a, float b) { return __fadd_rn(a, b); }
};
template <> struct FPB<double> {
    static constexpr int EB = 11, BIAS = 1023, MB = 52, W = 64;
    __device__ static int expo(double v) { return (int)((__double_as_longlong(v) >> 52) & 0x7FF); }
    __device__ static uint64_t bits(double v) { return (uint64_t)__double_as_longlong(v); }
    // getDoubleBin (c:5232-5242) reads the double through an int* and tests (*f) & (1 << (63-i)): as the
    // reference compiles on x86-64 (shift counts taken mod 32) its 64 digits are the low 32-bit word twice
    __device__ static uint64_t binview(double v) {
        const uint64_t lo = (uint32_t)__double_as_longlong(v);
        return (lo << 32) | lo;
    }
    __device__ static double mul(double a, double b) { return __dmul_rn(a, b); }
    __device__ static double sub(double a, double b) { return __dsub_rn(a, b); }
    __device__ static double add(double a, double b) { return __dadd_rn(a, b); }
};

__device__ __forceinline__ int clampi(int v, int lo, int hi) { return v < lo ? lo : (v > hi ? hi : v); }

// mantissa bits kept for biased exponent E (:3485-3503 and twins)
template <typename T>
__device__ __forceinline__ int kept(int E, int B) { return clampi(B + E - FPB<T>::BIAS, 0, FPB<T>::MB); }

// sz estimate of one element with history b1..b3 (:4660-4767): 2 bits when a predictor is within the
// bound, else 1+E+m of half the predictions' spread
template <typename T>
__device__ __forceinline__ int sz_bits(T x, T b1, T b2, T b3, T thr_le, int B) {
    typedef FPB<T> F;
    const T p1 = b1;
    const T p2 = F::sub(F::mul((T)2, b1), b2);
    const T p3 = F::add(F::sub(F::mul((T)3, b1), F::mul((T)3, b2)), b3);
    const T d1 = fabs(F::sub(p1, x)), d2 = fabs(F::sub(p2, x)), d3 = fabs(F::sub(p3, x));
    T dmin = d1;
    if (d2 < dmin) dmin = d2;
    if (d3 < dmin) dmin = d3;
    if (dmin <= thr_le) return 2;
    T mx, mn;
    if (p1 > p2) { mx = p1; mn = p2; } else { mx = p2; mn = p1; }
    if (p3 > mx) mx = p3;
    else if (p3 < mn) mn = p3;
    const T half = F::sub(mx, mn) / (T)2;
    const int E = (int)((F::binview(half) >> F::MB) & ((1u << F::EB) - 1));  // c[1..EB] of getXBin
    return 1 + F::EB + kept<T>(E, B);
}

// nolossy performance / area: p4 - x as a bit string, the reference counts the bits from the first set bit
// after the sign to the end (W - i for the first c[i] != 0, i >= 1), i.e. the bit length of the value
// without its sign; 0 when p4 - x is +-0 (no bit counted)
template <typename T>
__device__ __forceinline__ int nonzero_bits(T x, T b1, T b2, T b3, T b4) {
    typedef FPB<T> F;
    const T p4 = F::sub(F::add(F::sub(F::mul((T)4, b1), F::mul((T)6, b2)), F::mul((T)4, b3)), b4);
    const uint64_t m = F::binview(F::sub(p4, x)) & (F::W == 64 ? 0x7FFFFFFFFFFFFFFFull : 0x7FFFFFFFull);
    return m ? 64 - (int)__clzll((long long)m) : 0;
}

// area element size (:4896-4910): re1/re2/re3 + llrb + ex; AREA_KEEP above re3 (doubles only)
constexpr int AREA_KEEP = 254;
__device__ __forceinline__ int area_size(int nz) {
    return nz <= 0 ? 0 : (nz <= 2 ? 5 : (nz <= 4 ? 7 : (nz <= 32 ? 35 : AREA_KEEP)));
}

template <typename T, int MODE>
__global__ __launch_bounds__(256) void ratio_kernel(const T* __restrict__ x, long long n, int B, T thr_le,
                                                    unsigned long long* __restrict__ sum, unsigned* __restrict__ neg1,
                                                    uint8_t* __restrict__ sizes) {
    typedef FPB<T> F;
    unsigned long long acc = 0;
    bool m1 = false;
    for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x) {
        const T v = x[i];
        m1 |= v == (T)-1;
        if (MODE == R_BITWISE || MODE == R_BITWISE_D2) {
            int E;
            if (MODE == R_BITWISE_D2) E = FPB<double>::expo((double)v);
            else E = F::expo(v);
            acc += MODE == R_BITWISE_D2 ? (unsigned long long)(12 + kept<double>(E, B))
                                         : (unsigned long long)(1 + F::EB + kept<T>(E, B));
        } else if (MODE == R_SZ) {
            acc += i < 3 ? (unsigned long long)F::W : (unsigned long long)sz_bits<T>(v, x[i - 1], x[i - 2], x[i - 3], thr_le, B);
        } else {
            const int nz = i < 4 ? -1 : nonzero_bits<T>(v, x[i - 1], x[i - 2], x[i - 3], x[i - 4]);
            if (MODE == R_PERF) {
                acc += i < 4 ? (unsigned long long)F::W : (nz > 0 ? (unsigned long long)(nz + 3 + 1) : 0ull);
            } else {                                                     // area: the element's size
                sizes[i] = (uint8_t)(i < 4 ? 255 : area_size(nz));
            }
        }
    }
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) acc += __shfl_xor(acc, d, 64);
    if ((threadIdx.x & 63) == 0 && acc) atomicAdd(sum, acc);
    if (__any(m1) && (threadIdx.x & 63) == 0) atomicOr(neg1, 1u);
}

// area (:4841-4927): the first four elements take re3+llrb+ex = 35 bits each with no block check; every
// later element with a nonzero residual packs greedily into 512-bit blocks of 507 usable bits.
// A double residual longer than re3 = 32 bits leaves data_bits unassigned (c:5185-5197); the compiled
// reference keeps the register, i.e. the last assigned size: AREA_KEEP, resolved here with 35 before
// any assignment (the reference reads an uninitialised value there)
__global__ void area_pack_kernel(const uint8_t* __restrict__ sizes, long long n, unsigned long long* __restrict__ out) {
    if (threadIdx.x != 0) return;
    long long cdb = 1;
    int occ = 0, last = 35;
    for (long long i = 0; i < n; i++) {
        int s = sizes[i];
        if (s == 255) { occ += 35; continue; }
        if (s == 0) continue;
        if (s == AREA_KEEP) s = last;
        last = s;
        if (occ + s > 512 - 5) { cdb++; occ = s; }
        else occ += s;
    }
    *out = (unsigned long long)cdb;
}

// the reference loops verbatim (the -1 history sentinel included), one lane: inputs holding -1.0
template <typename T, int MODE>
__global__ void ratio_serial_kernel(const T* __restrict__ x, long long n, int B, T thr_le,
                                    unsigned long long* __restrict__ out) {
    typedef FPB<T> F;
    if (threadIdx.x != 0) return;
    T b1 = -1, b2 = -1, b3 = -1, b4 = -1;
    long long cb = 0, cdb = 1;
    int occ = 0, last = 35;
    for (long long i = 0; i < n; i++) {
        const T v = x[i];
        if (MODE == R_SZ) {
            if (b3 == (T)-1 || b2 == (T)-1 || b1 == (T)-1) {
                cb += F::W;
                if (b3 == (T)-1) b3 = v; else if (b2 == (T)-1) b2 = v; else if (b1 == (T)-1) b1 = v;
            } else {
                cb += sz_bits<T>(v, b1, b2, b3, thr_le, B);
                b3 = b2; b2 = b1; b1 = v;
            }
        } else {
            if (b4 == (T)-1 || b3 == (T)-1 || b2 == (T)-1 || b1 == (T)-1) {
                if (MODE == R_PERF) cb += F::W; else occ += 35;
                if (b4 == (T)-1) b4 = v; else if (b3 == (T)-1) b3 = v; else if (b2 == (T)-1) b2 = v; else if (b1 == (T)-1) b1 = v;
            } else {
                const int nz = nonzero_bits<T>(v, b1, b2, b3, b4);
                b4 = b3; b3 = b2; b2 = b1; b1 = v;
                if (nz > 0) {
                    if (MODE == R_PERF) cb += nz + 3 + 1;
                    else {
                        int s = area_size(nz);
                        if (s == AREA_KEEP) s = last;
                        last = s;
                        if (occ + s > 512 - 5) { cdb++; occ = s; } else occ += s;
                    }
                }
            }
        }
    }
    *out = (unsigned long long)(MODE == R_AREA ? cdb : cb);
}

template <typename T, int MODE>
static int launch(const T* x, long long n, int B, T thr_le, unsigned long long* d_sum, unsigned* d_flag, uint8_t* sizes,
                  hipStream_t st) {
    long long g = (n + 255) / 256;
    if (g > 4096) g = 4096;
    if (g < 1) g = 1;
    hipLaunchKernelGGL((ratio_kernel<T, MODE>), dim3((unsigned)g), dim3(256), 0, st, x, n, B, thr_le, d_sum, d_flag, sizes);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

}  // namespace dcr

using namespace dcr;

// mode: 0 bitwise, 1 bitwise of floats as doubles (double2), 2 sz, 3 nolossy performance, 4 nolossy area
// (the sizes pass; dc_launch_ratio_area packs).  d_sum / d_flag are zeroed by the caller.
extern "C" int dc_launch_ratio(int is_double, int mode, const void* x, long long n, int B, double thr_le,
                               unsigned long long* d_sum, unsigned* d_flag, uint8_t* sizes, hipStream_t st) {
    if (n <= 0) return 0;
    if (!is_double) {
        const float* xf = (const float*)x;
        const float t = (float)thr_le;
        switch (mode) {
            case R_BITWISE: return launch<float, R_BITWISE>(xf, n, B, t, d_sum, d_flag, sizes, st);
            case R_BITWISE_D2: return launch<float, R_BITWISE_D2>(xf, n, B, t, d_sum, d_flag, sizes, st);
            case R_SZ: return launch<float, R_SZ>(xf, n, B, t, d_sum, d_flag, sizes, st);
            case R_PERF: return launch<float, R_PERF>(xf, n, B, t, d_sum, d_flag, sizes, st);
            case R_AREA: return launch<float, R_AREA>(xf, n, B, t, d_sum, d_flag, sizes, st);
        }
    } else {
        const double* xd = (const double*)x;
        switch (mode) {
            case R_BITWISE: return launch<double, R_BITWISE>(xd, n, B, thr_le, d_sum, d_flag, sizes, st);
            case R_SZ: return launch<double, R_SZ>(xd, n, B, thr_le, d_sum, d_flag, sizes, st);
            case R_PERF: return launch<double, R_PERF>(xd, n, B, thr_le, d_sum, d_flag, sizes, st);
            case R_AREA: return launch<double, R_AREA>(xd, n, B, thr_le, d_sum, d_flag, sizes, st);
        }
    }
    return -2;
}

extern "C" int dc_launch_ratio_area(const uint8_t* sizes, long long n, unsigned long long* d_out, hipStream_t st) {
    hipLaunchKernelGGL(area_pack_kernel, dim3(1), dim3(64), 0, st, sizes, n, d_out);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

extern "C" int dc_launch_ratio_serial(int is_double, int mode, const void* x, long long n, int B, double thr_le,
                                      unsigned long long* d_out, hipStream_t st) {
    if (!is_double) {
        const float* xf = (const float*)x;
        const float t = (float)thr_le;
        if (mode == R_SZ) hipLaunchKernelGGL((ratio_serial_kernel<float, R_SZ>), dim3(1), dim3(64), 0, st, xf, n, B, t, d_out);
        else if (mode == R_PERF) hipLaunchKernelGGL((ratio_serial_kernel<float, R_PERF>), dim3(1), dim3(64), 0, st, xf, n, B, t, d_out);
        else hipLaunchKernelGGL((ratio_serial_kernel<float, R_AREA>), dim3(1), dim3(64), 0, st, xf, n, B, t, d_out);
    } else {
        const double* xd = (const double*)x;
        if (mode == R_SZ) hipLaunchKernelGGL((ratio_serial_kernel<double, R_SZ>), dim3(1), dim3(64), 0, st, xd, n, B, thr_le, d_out);
        else if (mode == R_PERF) hipLaunchKernelGGL((ratio_serial_kernel<double, R_PERF>), dim3(1), dim3(64), 0, st, xd, n, B, thr_le, d_out);
        else hipLaunchKernelGGL((ratio_serial_kernel<double, R_AREA>), dim3(1), dim3(64), 0, st, xd, n, B, thr_le, d_out);
    }
    return hipGetLastError() == hipSuccess ? 0 : -1;
}
