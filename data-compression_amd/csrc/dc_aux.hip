// dc_aux.hip -- pre-passes and stream protection on gfx950.
//
//  * toSmallDataset_float (impl/dataCompression.c:3543-3562): min then x - min.  The sequential
//    `if (data[i] < min)` keeps the FIRST occurrence of the minimum (so +0/-0 ties and NaNs resolve
//    like the reference); the parallel reduction carries (value, index) to reproduce that.
//  * med_dataset_float (:3593-3620): a left-to-right float sum (order-dependent rounding), so the
//    sum runs in one lane over LDS-staged blocks; max and type are exact in parallel.
//  * do_crc32 (:5524-5534, zlib crc32 byte by byte): per-lane table CRC of 64-byte runs, combined
//    with GF(2) "multiply by x^(8n) mod P" operators (crc(A||B) = shift(crc(A),|B|) ^ crc(B)).
//  * hamming_encode / hamming_decode (:5740-5778): SECDED check bits per block = XOR of the Hamming
//    positions of the set data bits (powers of two skipped) + overall parity.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>
#include <algorithm>
#include "dc_device.h"

namespace dc {

// ---------------------------------------------------------------- toSmallDataset_float
// per-workgroup minimum of x[1..n) (NaN ignored: hardware minNum) and the index of the first zero (+0 or -0)
// in it: the reference keeps data[0] unless a later value is strictly smaller, so equal values only matter for
// zeros, where the first one's sign wins (min_final).  Four float4 loads of a thread in flight at once
// (coalesced: q, q + S, q + 2S, q + 3S).  (r05: with a (value, index) total order per element the pass ran at
// ~3.3 TB/s, issue-bound on the 64-bit index selects)
__global__ __launch_bounds__(256) void min_partial_kernel(const float* __restrict__ x, long long n,
                                                          float* __restrict__ pv, long long* __restrict__ pi) {
    __shared__ float sv[256];
    __shared__ long long si[256];
    float mv = __int_as_float(0x7fc00000);
    long long fz = (long long)1 << 62;
    const long long n4 = ((reinterpret_cast<uintptr_t>(x) & 15u) == 0) ? (n >> 2) : 0;
    const float4* x4 = reinterpret_cast<const float4*>(x);
    const long long S = (long long)gridDim.x * blockDim.x;
    for (long long q0 = (long long)blockIdx.x * blockDim.x + threadIdx.x; q0 < n4; q0 += 4 * S) {
        float4 v[4];
#pragma unroll
        for (int u = 0; u < 4; u++) {                      // (past the end: NaN, which no minimum takes)
            const float qn = __int_as_float(0x7fc00000);
            v[u] = q0 + u * S < n4 ? x4[q0 + u * S] : make_float4(qn, qn, qn, qn);
        }
#pragma unroll
        for (int u = 0; u < 4; u++) {
            const long long q = q0 + u * S;
            const float a = q == 0 ? __int_as_float(0x7fc00000) : v[u].x;   // (element 0 is the start value)
            mv = fminf(mv, fminf(fminf(a, v[u].y), fminf(v[u].z, v[u].w)));
            const int k = a == 0.f ? 0 : v[u].y == 0.f ? 1 : v[u].z == 0.f ? 2 : v[u].w == 0.f ? 3 : 4;
            if (k < 4 && q < n4) fz = min(fz, 4 * q + k);
        }
    }
    for (long long i = max(4 * n4, 1ll) + (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += S) {
        const float a = x[i];
        mv = fminf(mv, a);
        if (a == 0.f) fz = min(fz, i);
    }
    sv[threadIdx.x] = mv; si[threadIdx.x] = fz;
    __syncthreads();
    for (int st = 128; st > 0; st >>= 1) {
        if ((int)threadIdx.x < st) {
            sv[threadIdx.x] = fminf(sv[threadIdx.x], sv[threadIdx.x + st]);
            si[threadIdx.x] = min(si[threadIdx.x], si[threadIdx.x + st]);
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) { pv[blockIdx.x] = sv[0]; pi[blockIdx.x] = si[0]; }
}

// (clr64 / clr32: words zeroed on the way -- in a recorded halo step the next encode's tile states and flag, which a
// graph replay cannot tag with a new epoch; two memset nodes less per plane)
// (one workgroup of 256 threads: min_final_kernel, and the last workgroup of plane_gather_min_kernel)
__device__ __forceinline__ void min_final_body(const float* __restrict__ x, const float* __restrict__ pv,
                                               const long long* __restrict__ pi, int nparts, float* __restrict__ out_min,
                                               uint64_t* __restrict__ clr64, int n64, uint32_t* __restrict__ clr32,
                                               int n32) {
    for (int i = threadIdx.x; i < n64; i += 256) clr64[i] = 0ull;
    for (int i = threadIdx.x; i < n32; i += 256) clr32[i] = 0u;
    __shared__ float sv[256];
    __shared__ long long si[256];
    float mv = __int_as_float(0x7fc00000);
    long long fz = (long long)1 << 62;
    for (int p = threadIdx.x; p < nparts; p += 256) { mv = fminf(mv, pv[p]); fz = min(fz, pi[p]); }
    sv[threadIdx.x] = mv; si[threadIdx.x] = fz;
    __syncthreads();
    for (int st = 128; st > 0; st >>= 1) {
        if ((int)threadIdx.x < st) {
            sv[threadIdx.x] = fminf(sv[threadIdx.x], sv[threadIdx.x + st]);
            si[threadIdx.x] = min(si[threadIdx.x], si[threadIdx.x + st]);
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        const float m = sv[0];
        const float x0 = x[0];
        float r = x0;                                        // min = data[0]; later strictly smaller wins
        if (!(m != m) && m < x0) r = m == 0.f ? x[si[0]] : m;   // (a zero: the first one, with its sign)
        *out_min = r;
    }
}
__global__ __launch_bounds__(256) void min_final_kernel(const float* __restrict__ x, const float* __restrict__ pv,
                                                        const long long* __restrict__ pi, int nparts,
                                                        float* __restrict__ out_min, uint64_t* __restrict__ clr64,
                                                        int n64, uint32_t* __restrict__ clr32, int n32) {
    min_final_body(x, pv, pi, nparts, out_min, clr64, n64, clr32, n32);
}

// (sub_x86, the reference's x86 subtraction: dc_device.h)
__global__ __launch_bounds__(256) void sub_min_kernel(const float* __restrict__ x, long long n,
                                                      const float* __restrict__ mn, float* __restrict__ y) {
    const float m = *mn;
    const long long n4 = n >> 2;
    const float4* x4 = reinterpret_cast<const float4*>(x);
    float4* y4 = reinterpret_cast<float4*>(y);
    for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n4;
         i += (long long)gridDim.x * blockDim.x) {
        float4 v = x4[i];
        v.x = sub_x86(v.x, m); v.y = sub_x86(v.y, m); v.z = sub_x86(v.z, m); v.w = sub_x86(v.w, m);
        y4[i] = v;
    }
    for (long long i = (n4 << 2) + (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n;
         i += (long long)gridDim.x * blockDim.x)
        y[i] = sub_x86(x[i], m);
}

// y = x - m for a value m (dc_encode_sub_device's fallback: the variants that do not subtract while loading)
__global__ __launch_bounds__(256) void sub_val_kernel(const float* __restrict__ x, long long n, float m, float* __restrict__ y) {
    for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x)
        y[i] = sub_x86(x[i], m);
}
extern "C" int dc_launch_sub_value(const float* x, long long n, float m, float* y, hipStream_t st) {
    if (n <= 0) return 0;
    hipLaunchKernelGGL(sub_val_kernel, dim3((unsigned)min((n + 255) / 256, 8192ll)), dim3(256), 0, st, x, n, m, y);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

// ---------------------------------------------------------------- med_dataset_float
// ---------------------------------------------------------------- exact parallel mean
// med_dataset_float (:3593-3620) sums left to right in float.  While the running sum s stays in one
// binade [2^(E-127), 2^(E-126)) its ulp u = 2^(E-150) is fixed and fl(s + x) = s + u*r(x), with r =
// x/u rounded to an integer (ties to even on s/u, i.e. on the parity of k = s/u), as long as the sum
// stays below the binade's top (k < 2^24) and 0 <= x < 2^(E-126).  So a chunk of MC elements is a
// 2-state transducer for a given binade: start parity -> (units added, end parity).
//   med_chunk_sum   : per chunk its double sum and max (all CUs)
//   med_chunk_scan  : one workgroup: exclusive scan of the double chunk sums = an estimate of the
//                     running sum at every chunk, whose binade E_est centres the chunk's window of
//                     candidate binades
//   med_chunk_trans : per chunk and candidate binade the transducer (one wave per chunk, 32 elements per
//                     lane; one pass over x)
//   med_compose     : one workgroup: from s_init, blocks of 1024 chunks are composed with a block scan
//                     while the running sum stays in its binade and each chunk has a valid transducer
//                     for it; a chunk where the sum leaves the binade, or that holds an element the
//                     transducer cannot take (negative, NaN, too large, the binade not in its window),
//                     or a sum below SMIN, is added element by element, exactly like the reference.
//                     At 2^26 U10: about 25 such chunks (the binade crossings).  The chunk records come
//                     from an LDS ring refilled ahead of the blocks (a block that restarts after a
//                     crossing finds them there instead of waiting for its loads again).
// Windows: the narrow one, [E_est - 1, E_est + 1], is tried first (the float sum's binade at every chunk
// boundary lies there for U10, ramps, sines, normals, ones and small uniforms up to 2^26: a stalling sum falls
// one binade behind the double estimate, a rounding-up one one ahead); a compose that meets more than
// MED_MISS_MAX chunks outside it stops and raises the scratch flag, and the host runs the wide window
// [E_est - 4, E_est + 1] from the start (dc_launch_med_wide).  The multi-GPU shard records (med_shard_kernel)
// use the wide window.
// The same kernels run med_dataset_double (:3564-3590) with u = 2^(E-1075) and k < 2^53 (MedFP<double>).
constexpr int MC = 2048;                                   // elements per chunk
constexpr int MW = 6;                                      // candidate binades per chunk, wide window
constexpr int MWN = 3;                                     // narrow window
constexpr int MC_T = 256;                                  // threads of the chunk-sum kernel (8 elements each)
constexpr int MC_PER = MC / MC_T;
constexpr int MT_PER = MC / 64;                            // transducer kernel: elements per lane
constexpr int MX_T = 1024;                                 // chunks per compose block; med_shard workgroup
constexpr int MED_MISS_MAX = 16;                           // narrow-window misses before the wide pass
template <int W> __host__ __device__ constexpr int med_wlo() { return W == MW ? -4 : -1; }

// float / double: the running sum's binade E (biased exponent), k = s/u in [2^M, 2^(M+1)), u = 2^(E-bias-M)
template <typename T> struct MedFP;
template <> struct MedFP<float> {
    typedef uint32_t U;
    typedef int D;                                         // units added per chunk (saturated)
    static constexpr int M = 23, BIAS = 127, EMIN = 24, EMAX = 253;
    static constexpr D SAT = 1 << 25;
    __device__ static U bits(float v) { return __float_as_uint(v); }
    __device__ static float from(U b) { return __uint_as_float(b); }
    __device__ static int expo(float v) { return (int)((bits(v) >> 23) & 0xFFu); }
    __device__ static float pow2(int e) { return from((U)(e + BIAS) << M); }       // 2^e, e in the normal range
    __device__ static float mul(float a, float b) { return __fmul_rn(a, b); }
    __device__ static float sub(float a, float b) { return __fsub_rn(a, b); }
    __device__ static float add(float a, float b) { return __fadd_rn(a, b); }
    __device__ static float smin() { return pow2(-100); }                         // 1/u stays a float above it
    __device__ static float smax() { return 3.0e38f; }
    __device__ static float mean(float s, long long n) { return __fdiv_rn(s, (float)n); }
    __device__ static int type(float mx) {                                        // :3605-3614
        int add = 0;
        for (int i = 7; i > 0; i--) { add += 1 << i; if ((double)mx < ldexp(1.0, add - 127)) return 8 - i; }
        return 0;
    }
};
template <> struct MedFP<double> {
    typedef unsigned long long U;
    typedef long long D;
    static constexpr int M = 52, BIAS = 1023, EMIN = 53, EMAX = 2045;
    static constexpr D SAT = 1ll << 54;
    __device__ static U bits(double v) { return (U)__double_as_longlong(v); }
    __device__ static double from(U b) { return __longlong_as_double((long long)b); }
    __device__ static int expo(double v) { return (int)((bits(v) >> 52) & 0x7FFull); }
    __device__ static double pow2(int e) { return from((U)(e + BIAS) << M); }
    __device__ static double mul(double a, double b) { return __dmul_rn(a, b); }
    __device__ static double sub(double a, double b) { return __dsub_rn(a, b); }
    __device__ static double add(double a, double b) { return __dadd_rn(a, b); }
    __device__ static double smin() { return pow2(-960); }
    __device__ static double smax() { return 1.0e308; }
    __device__ static double mean(double s, long long n) { return __ddiv_rn(s, (double)n); }
    __device__ static int type(double mx) {                                       // :3576-3585
        int add = 0;
        for (int i = 10; i > 0; i--) { add += 1 << i; if (mx < ldexp(1.0, add - 1023)) return 11 - i; }
        return 0;
    }
};

template <typename T>
struct MedScratch {
    double* csum;                                          // [nch] chunk sums (an estimate only)
    T* cmax;                                               // [nch] chunk max (NaN-skipping)
    int* eest;                                             // [nch] E_est: the estimated running sum's binade
    typename MedFP<T>::D* Td;                              // [nch * MW * 2] units added from parity 0 / 1
    uint8_t* F;                                            // [nch * MW] end parity 0 | end parity 1 << 1 | bad << 2
    uint8_t* Z;                                            // [nch] 1: every element is +0 / -0; 2: some element
                                                           // is negative or NaN (no transducer takes the chunk)
    long long* rec;                                        // med_shard_kernel's 21-word record
    unsigned* flag;                                        // 1: the narrow window missed, the wide pass runs
    long long* res;                                        // right after flag's word: mean, type, sum, max (bits)
                                                           // -- the host reads flag + results in one copy
};

template <typename T>
__host__ __device__ inline long long med_scratch_bytes(long long n) {
    const long long nch = (n + MC - 1) / MC;
    return nch * (8 + (long long)sizeof(T) + 4 + MW * 2 * (long long)sizeof(typename MedFP<T>::D) + MW + 1) + 1024;
}
extern "C" long long dc_med_scratch_bytes(long long n) { return med_scratch_bytes<float>(n); }
extern "C" long long dc_med_scratch_bytes64(long long n) { return med_scratch_bytes<double>(n); }

template <typename T>
__host__ __device__ inline MedScratch<T> med_scratch(void* base, long long nch) {
    MedScratch<T> m;
    char* b = (char*)base;
    m.csum = (double*)b; b += nch * 8;
    m.Td = (typename MedFP<T>::D*)b; b += nch * MW * 2 * (long long)sizeof(typename MedFP<T>::D);
    m.cmax = (T*)b; b += nch * (long long)sizeof(T);
    m.eest = (int*)b; b += nch * 4;
    m.F = (uint8_t*)b; b += nch * MW;
    m.Z = (uint8_t*)b; b += nch;
    m.rec = (long long*)(((uintptr_t)b + 7) & ~(uintptr_t)7);
    m.flag = (unsigned*)(m.rec + 24);
    m.res = m.rec + 25;
    return m;
}

template <typename T>
__device__ __forceinline__ void load_chunk(const T* __restrict__ x, long long n, long long c, T* v) {
    const long long e0 = c * MC + (long long)threadIdx.x * MC_PER;
    if (sizeof(T) == 4 && e0 + MC_PER <= n && (reinterpret_cast<uintptr_t>(x) & 15u) == 0) {
        // (a whole thread's run: two 16-byte loads instead of eight guarded 4-byte ones)
        const float4* p = reinterpret_cast<const float4*>(x + e0);
        const float4 a = p[0], b = p[1];
        const float f[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
#pragma unroll
        for (int i = 0; i < MC_PER; i++) v[i] = (T)f[i];
        return;
    }
#pragma unroll
    for (int i = 0; i < MC_PER; i++) v[i] = e0 + i < n ? x[e0 + i] : (T)0;
}

// a lane's run of N consecutive elements from e0 (16-byte loads when whole and aligned)
template <typename T, int N>
__device__ __forceinline__ void load_run(const T* __restrict__ x, long long n, long long e0, T* v) {
    if (e0 + N <= n && (reinterpret_cast<uintptr_t>(x) & 15u) == 0) {
        if (sizeof(T) == 4) {
            const float4* p = reinterpret_cast<const float4*>(x + e0);
#pragma unroll
            for (int q = 0; q < N / 4; q++) {
                const float4 a = p[q];
                v[4 * q] = (T)a.x; v[4 * q + 1] = (T)a.y; v[4 * q + 2] = (T)a.z; v[4 * q + 3] = (T)a.w;
            }
        } else {
            const double2* p = reinterpret_cast<const double2*>(x + e0);
#pragma unroll
            for (int q = 0; q < N / 2; q++) {
                const double2 a = p[q];
                v[2 * q] = (T)a.x; v[2 * q + 1] = (T)a.y;
            }
        }
        return;
    }
#pragma unroll
    for (int i = 0; i < N; i++) v[i] = e0 + i < n ? x[e0 + i] : (T)0;
}

template <typename T>
__global__ __launch_bounds__(MC_T) void med_chunk_sum_kernel(const T* __restrict__ x, long long n, MedScratch<T> M) {
    typedef MedFP<T> FP;
    __shared__ double ws[MC_T / 64];
    __shared__ T wm[MC_T / 64];
    const long long c = blockIdx.x;
    if (c == 0 && threadIdx.x == 0) *M.flag = 0u;           // (the narrow pass has not missed yet)
    T v[MC_PER];
    load_chunk(x, n, c, v);
    const long long e0 = c * MC + (long long)threadIdx.x * MC_PER;
    double sm = 0.0;
    T mx = -INFINITY;
    bool nz = false, ng = false;
#pragma unroll
    for (int i = 0; i < MC_PER; i++)
        if (e0 + i < n) {
            sm += (double)v[i];
            mx = v[i] > mx ? v[i] : mx;                          // NaNs never win (as the reference's >)
            nz |= (FP::bits(v[i]) << 1) != 0;
            ng |= !(v[i] >= (T)0);                               // negative or NaN
        }
    const bool anynz = __syncthreads_or(nz);
    const bool anyng = __syncthreads_or(ng);
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) {
        sm += __shfl_xor(sm, d, 64);
        const T o = __shfl_xor(mx, d, 64);
        mx = o > mx ? o : mx;
    }
    if ((threadIdx.x & 63) == 0) { ws[threadIdx.x >> 6] = sm; wm[threadIdx.x >> 6] = mx; }
    __syncthreads();
    if (threadIdx.x == 0) {
        double t = 0.0;
        T m = -INFINITY;
        for (int w = 0; w < MC_T / 64; w++) { t += ws[w]; m = wm[w] > m ? wm[w] : m; }
        M.csum[c] = isfinite(t) ? t : 0.0;
        M.cmax[c] = m;
        M.Z[c] = (uint8_t)((anynz ? 0 : 1) | (anyng ? 2 : 0));
    }
}

// ---- fused pre-passes (dc_prep_device, r06): toSmallDataset_float's minimum and med_dataset_float of x - min in
// one read of x for the statistics, with x - min never written.  The chunk statistics of x - min
// follow from those of x once the minimum m is known, for a FINITE m (the host falls back to the separate passes
// otherwise): fl(x - m) >= 0 for every non-NaN x (m is the minimum), is NaN exactly where x is, and is monotone in x,
// so its chunk max is fl(max x - m) and a chunk is all zeros exactly when its max equals m and it holds no NaN; the
// double chunk sum only estimates the running sum's binade (the compose is exact whatever it is), so sum x - count m
// serves.  med_chunk_stats_kernel: per chunk the double sum, the max and a NaN flag of x, and (min_partial's rule)
// the minimum of x[1..n) in it and the index of its first zero; min_final_kernel then takes the minimum, and
// med_sub_fix_kernel turns the statistics into those of x - m.
__global__ __launch_bounds__(MC_T) void med_chunk_stats_kernel(const float* __restrict__ x, long long n, MedScratch<float> M,
                                                               float* __restrict__ pv, long long* __restrict__ pi) {
    __shared__ double ws[MC_T / 64];
    __shared__ float wm[MC_T / 64], wn[MC_T / 64];
    __shared__ long long wz[MC_T / 64];
    const long long c = blockIdx.x;
    if (c == 0 && threadIdx.x == 0) { *M.flag = 0u; M.res[4] = 0; }
    float v[MC_PER];
    load_chunk(x, n, c, v);
    const long long e0 = c * MC + (long long)threadIdx.x * MC_PER;
    double sm = 0.0;
    float mx = -INFINITY, mn = __int_as_float(0x7fc00000);
    long long fz = (long long)1 << 62;
    bool nan = false;
#pragma unroll
    for (int i = 0; i < MC_PER; i++)
        if (e0 + i < n) {
            sm += (double)v[i];
            mx = v[i] > mx ? v[i] : mx;                          // NaNs never win
            nan |= v[i] != v[i];
            if (e0 + i > 0) {                                    // (element 0 is the reference's start value)
                mn = fminf(mn, v[i]);                            // NaN ignored (minNum)
                if (v[i] == 0.f) fz = min(fz, e0 + i);
            }
        }
    const bool anynan = __syncthreads_or(nan);
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) {
        sm += __shfl_xor(sm, d, 64);
        const float o = __shfl_xor(mx, d, 64);
        mx = o > mx ? o : mx;
        mn = fminf(mn, __shfl_xor(mn, d, 64));
        fz = min(fz, (long long)__shfl_xor(fz, d, 64));
    }
    if ((threadIdx.x & 63) == 0) { ws[threadIdx.x >> 6] = sm; wm[threadIdx.x >> 6] = mx; wn[threadIdx.x >> 6] = mn; wz[threadIdx.x >> 6] = fz; }
    __syncthreads();
    if (threadIdx.x == 0) {
        double t = 0.0;
        float m = -INFINITY, q = __int_as_float(0x7fc00000);
        long long z = (long long)1 << 62;
        for (int w = 0; w < MC_T / 64; w++) { t += ws[w]; m = wm[w] > m ? wm[w] : m; q = fminf(q, wn[w]); z = min(z, wz[w]); }
        M.csum[c] = t;                                           // (of x: med_sub_fix_kernel turns them into x - m)
        M.cmax[c] = m;
        M.Z[c] = (uint8_t)(anynan ? 2 : 0);
        pv[c] = q;
        pi[c] = z;
    }
}

// min_final_kernel and med_sub_fix_kernel in one workgroup of 1024 threads, every load of a thread's batch in flight
// at once: the minimum from the nch chunk partials (one 256-thread pass over 32768 partials was 36 us of dependent
// loads at 2^26), then the statistics of x - m
constexpr int PF_T = 1024, PF_B = 8;
__global__ __launch_bounds__(PF_T) void prep_min_fix_kernel(const float* __restrict__ x, long long n, MedScratch<float> M,
                                                            const float* __restrict__ pv, const long long* __restrict__ pi,
                                                            float* __restrict__ d_min) {
    __shared__ float sv[PF_T / 64];
    __shared__ long long si[PF_T / 64];
    __shared__ float s_m;
    const int tid = threadIdx.x;
    const long long nch = (n + MC - 1) / MC;
    float mv = __int_as_float(0x7fc00000);
    long long fz = (long long)1 << 62;
    for (long long b = 0; b < nch; b += (long long)PF_T * PF_B) {
        float v[PF_B];
        long long z[PF_B];
#pragma unroll
        for (int k = 0; k < PF_B; k++) {
            const long long c = b + tid + (long long)k * PF_T;
            v[k] = c < nch ? pv[c] : __int_as_float(0x7fc00000);
            z[k] = c < nch ? pi[c] : (long long)1 << 62;
        }
#pragma unroll
        for (int k = 0; k < PF_B; k++) { mv = fminf(mv, v[k]); fz = min(fz, z[k]); }
    }
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) {
        mv = fminf(mv, __shfl_xor(mv, d, 64));
        fz = min(fz, (long long)__shfl_xor(fz, d, 64));
    }
    if ((tid & 63) == 0) { sv[tid >> 6] = mv; si[tid >> 6] = fz; }
    __syncthreads();
    if (tid == 0) {
        float m = __int_as_float(0x7fc00000);
        long long z = (long long)1 << 62;
        for (int w = 0; w < PF_T / 64; w++) { m = fminf(m, sv[w]); z = min(z, si[w]); }
        const float x0 = x[0];
        float r = x0;                                        // (min_final_kernel's rule)
        if (!(m != m) && m < x0) r = m == 0.f ? x[z] : m;
        *d_min = r;
        s_m = r;
        if (!isfinite(r)) M.res[4] = 1;
    }
    __syncthreads();
    const float m = s_m;
    if (!isfinite(m)) return;
    for (long long b = 0; b < nch; b += (long long)PF_T * PF_B) {
        double t[PF_B];
        float mx[PF_B];
        uint8_t zz[PF_B];
#pragma unroll
        for (int k = 0; k < PF_B; k++) {
            const long long c = min(b + tid + (long long)k * PF_T, nch - 1);
            t[k] = M.csum[c]; mx[k] = M.cmax[c]; zz[k] = M.Z[c];
        }
#pragma unroll
        for (int k = 0; k < PF_B; k++) {
            const long long c = b + tid + (long long)k * PF_T;
            if (c < nch) {
                const long long cnt = min((long long)MC, n - c * MC);
                M.csum[c] = isfinite(t[k]) ? t[k] - (double)cnt * (double)m : 0.0;
                M.cmax[c] = mx[k] == -INFINITY ? mx[k] : sub_fin(mx[k], m);
                M.Z[c] = (uint8_t)(zz[k] | (!(zz[k] & 2) && mx[k] == m ? 1 : 0));
            }
        }
    }
}

// the statistics of x - m (m = *d_min): a non-finite m sets res[4] (the host then runs the separate passes)
__global__ __launch_bounds__(256) void med_sub_fix_kernel(long long n, MedScratch<float> M, const float* __restrict__ d_min) {
    const float m = *d_min;
    const long long nch = (n + MC - 1) / MC;
    if (!isfinite(m)) {
        if (blockIdx.x == 0 && threadIdx.x == 0) M.res[4] = 1;
        return;
    }
    for (long long c = (long long)blockIdx.x * blockDim.x + threadIdx.x; c < nch; c += (long long)gridDim.x * blockDim.x) {
        const long long cnt = min((long long)MC, n - c * MC);
        const double t = M.csum[c];
        const float mx = M.cmax[c];
        const uint8_t z = M.Z[c];
        M.csum[c] = isfinite(t) ? t - (double)cnt * (double)m : 0.0;
        M.cmax[c] = mx == -INFINITY ? mx : sub_fin(mx, m);    // (a chunk of NaNs only keeps -inf)
        M.Z[c] = (uint8_t)(z | (!(z & 2) && mx == m ? 1 : 0));
    }
}

// exclusive scan of the chunk sums -> an estimate of the running sum at every chunk and its binade E_est.
// Tiles of 8192 chunks: coalesced loads into LDS (the next tile's loads issued before this tile's scan), 8
// consecutive chunks per thread, a block scan, the binades back through LDS and out coalesced (runs of
// 32 chunks per thread, loaded in batches, took 37-54 us at 2^26: every load instruction spread over 64 lines).
constexpr int MS_T = 8192;
template <typename T>
__global__ __launch_bounds__(1024) void med_chunk_scan_kernel(MedScratch<T> M, long long nch, T s_init) {
    typedef MedFP<T> FP;
    __shared__ double tile[MS_T];
    __shared__ double wt[16];
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    int* etile = reinterpret_cast<int*>(tile);              // (the binades overwrite the sums they came from)
    double carry = (double)s_init;
    double nx[MS_T / 1024];
#pragma unroll
    for (int j = 0; j < MS_T / 1024; j++) {
        const long long i = tid + 1024ll * j;
        nx[j] = i < nch ? M.csum[i] : 0.0;
    }
    for (long long base = 0; base < nch; base += MS_T) {
        const int cnt = (int)min((long long)MS_T, nch - base);
#pragma unroll
        for (int j = 0; j < MS_T / 1024; j++) tile[tid + 1024 * j] = nx[j];
#pragma unroll
        for (int j = 0; j < MS_T / 1024; j++) {             // (the next tile's sums, in flight meanwhile)
            const long long i = base + MS_T + tid + 1024ll * j;
            nx[j] = i < nch ? M.csum[i] : 0.0;
        }
        __syncthreads();
        double v[8], sm = 0.0;
#pragma unroll
        for (int j = 0; j < 8; j++) { v[j] = tile[8 * tid + j]; sm += v[j]; }
        double inc = sm;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const double u = __shfl_up(inc, d, 64);
            if (lane >= d) inc += u;
        }
        if (lane == 63) wt[wid] = inc;
        __syncthreads();                                    // (every thread's sums read: tile is rewritten below)
        double run = carry + inc - sm, tot = 0.0;
#pragma unroll
        for (int w = 0; w < 16; w++) { run += w < wid ? wt[w] : 0.0; tot += wt[w]; }
        int e[8];
#pragma unroll
        for (int j = 0; j < 8; j++) {
            const T est = (T)fmin(fmax(run, 0.0), (double)FP::smax());
            e[j] = FP::expo(est);
            run += v[j];
        }
#pragma unroll
        for (int j = 0; j < 8; j++) etile[8 * tid + j] = e[j];
        __syncthreads();
#pragma unroll
        for (int j = 0; j < MS_T / 1024; j++) {
            const int i = tid + 1024 * j;
            if (i < cnt) M.eest[base + i] = etile[i];
        }
        carry += tot;
        __syncthreads();                                    // (etile read before the next tile's sums land)
    }
}

// transducer of one thread's elements for binade E (k's parity p in, units added / parity out).  Only a tie
// (x/u exactly halfway) depends on the parity: before the first tie the two paths (start parity 0 / 1) add the
// same units and differ in parity by 1 (X = the XOR of the units' low bits); the first tie rounds each to even
// (its bit differs between the paths), and from then on both paths are one.  So the common units S, the first
// tie's two bits and one parity are tracked, instead of both paths element by element.
template <typename T, int N = MC_PER>
__device__ __forceinline__ void trans_elems(const T* v, int cnt, int E, typename MedFP<T>::D& d0,
                                            typename MedFP<T>::D& d1, int& p0, int& p1) {
    // (every element is >= 0 and below the binade's top: the caller checked the chunk's max and flags)
    typedef MedFP<T> FP;
    typedef typename FP::D D;
    const T scale = FP::pow2(FP::BIAS + FP::M - E);                 // 1/u
    D S = 0, Sl = 0;                                                // units; units at the last tie
    int e0 = 0, e1 = 0;
    bool tied = false;
#pragma unroll
    for (int i = 0; i < N; i++) {
        if (i < cnt) {
            const T q = FP::mul(v[i], scale);                     // exact: power-of-two scaling, < 2^(M+1)
            const T rn = rint(q);                                   // nearest (a tie to even: decided below)
            const T dq = FP::sub(q, rn);
            if (__builtin_expect(dq == (T)0.5 || dq == (T)-0.5, 0)) {   // a tie: round the path's k + fl to even
                const D fl = (D)floor(q);
                const int b = ((int)((S - Sl) & 1) ^ (int)(fl & 1)) & 1;   // (S - Sl: the units since the last tie)
                if (!tied) { e0 = b; e1 = b ^ 1; tied = true; } else S += b;
                S += fl;
                Sl = S;
            } else {
                S += (D)rn;
            }
        }
    }
    // (a thread's units stay far below the type's range; compose() saturates the sums)
    const int X = (int)((S - Sl) & 1);
    d0 = min(S + e0, FP::SAT);
    d1 = min(S + e1, FP::SAT);
    p0 = X;
    p1 = tied ? X : X ^ 1;
}

// f then g (f earlier): start parity p -> f's units + g's units from f's end parity
template <typename D>
__device__ __forceinline__ void compose(D& a0, D& a1, int& q0, int& q1, D b0, D b1, int e0, int e1, D sat) {
    const D n0 = min(a0 + (q0 ? b1 : b0), sat), n1 = min(a1 + (q1 ? b1 : b0), sat);
    const int m0 = q0 ? e1 : e0, m1 = q1 ? e1 : e0;
    a0 = n0; a1 = n1; q0 = m0; q1 = m1;
}

// one wave per chunk (grid-stride: a gated launch whose flag is clear ends at once), lane = 32 consecutive
// elements; the W binades [E_est + wlo, E_est + wlo + W) -> Td / F slots 0..W-1
template <typename T, int W>
__global__ __launch_bounds__(256) void med_chunk_trans_kernel(const T* __restrict__ x, long long n, MedScratch<T> M,
                                                             int gated, const T* __restrict__ sub = nullptr) {
    typedef MedFP<T> FP;
    typedef typename FP::D D;
    if (gated && __hip_atomic_load(M.flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0u) return;
    const int lane = threadIdx.x & 63;
    const long long nch = (n + MC - 1) / MC, nw = (long long)gridDim.x * 4;
    for (long long c = (long long)blockIdx.x * 4 + (threadIdx.x >> 6); c < nch; c += nw) {
        T v[MT_PER];
        const long long e0 = c * MC + (long long)lane * MT_PER;
        load_run<T, MT_PER>(x, n, e0, v);
        if (sub) {                                                  // (dc_prep_device: the elements of x - min)
            const T m = *sub;
#pragma unroll
            for (int i = 0; i < MT_PER; i++) v[i] = sub_fin(v[i], m);
        }
        const int cnt = (int)max(0ll, min((long long)MT_PER, n - e0));
        const int elo = M.eest[c] + med_wlo<W>();
        const T cmax = M.cmax[c];
        const bool negnan = (M.Z[c] & 2) != 0;
#pragma unroll
        for (int w = 0; w < W; w++) {
            const int E = elo + w;
            D d0 = 0, d1 = 0;
            int p0 = 0, p1 = 1;
            bool bad = E < FP::EMIN || E > FP::EMAX;                  // 1/u or the binade top not a number
            if (!bad && negnan) {
                bad = true;                                            // (no transducer for any binade)
            } else if (!bad && cmax < FP::pow2(E - FP::BIAS - FP::M - 1)) {
                // every element below u/2 (and none negative or NaN): nothing added, parity kept -- the
                // transducer of a stalled sum, computed for free (uniform branch)
            } else if (!bad && !(cmax < FP::pow2(E + 1 - FP::BIAS))) {
                bad = true;                                            // an element at or above the binade's top
            } else if (!bad) {
                trans_elems<T, MT_PER>(v, cnt, E, d0, d1, p0, p1);
            }
            // ordered reduction over the wave: lane i absorbs lane i + d (its successor block)
#pragma unroll
            for (int d = 1; d < 64; d <<= 1) {
                const D b0 = __shfl_down(d0, d, 64), b1 = __shfl_down(d1, d, 64);
                const int f = __shfl_down(p0 | (p1 << 1) | ((int)bad << 2), d, 64);
                if ((lane & (2 * d - 1)) == 0) {
                    compose(d0, d1, p0, p1, b0, b1, f & 1, (f >> 1) & 1, FP::SAT);
                    bad |= (f & 4) != 0;
                }
            }
            if (lane == 0) {
                M.Td[(c * MW + w) * 2] = d0;
                M.Td[(c * MW + w) * 2 + 1] = d1;
                M.F[c * MW + w] = (uint8_t)(p0 | (p1 << 1) | (bad ? 4 : 0));
            }
        }
    }
}

// a transducer as the compose kernel scans them: units from start parity 0 / 1, end parities, and the first
// thread (of the scan) whose piece no transducer takes
template <typename D>
struct MTr {
    D a0, a1;
    int q0, q1, fb;
};
template <typename D>
__device__ __forceinline__ MTr<D> mtr_then(const MTr<D>& f, const MTr<D>& g, D sat) {     // f, then g
    MTr<D> r = f;
    compose(r.a0, r.a1, r.q0, r.q1, g.a0, g.a1, g.q0, g.q1, sat);
    r.fb = min(f.fb, g.fb);
    return r;
}
template <typename D>
__device__ __forceinline__ MTr<D> mtr_shfl_up(const MTr<D>& v, int d) {
    MTr<D> o;
    o.a0 = __shfl_up(v.a0, d, 64); o.a1 = __shfl_up(v.a1, d, 64);
    o.q0 = __shfl_up(v.q0, d, 64); o.q1 = __shfl_up(v.q1, d, 64); o.fb = __shfl_up(v.fb, d, 64);
    return o;
}
// the compose kernel's LDS ring of chunk records (window's first binade, units, flags): as many chunks as fit
// in ~128 KB (4096 for float's narrow window, 2048 for its wide one and double's narrow, 1024 for double's wide)
template <typename T, int W>
struct MedRing {
    typedef typename MedFP<T>::D D;
    static constexpr int BYTES = 4 + W * (2 * (int)sizeof(D) + 1);
    static constexpr int R = BYTES * 4096 <= 128 * 1024 ? 4096 : (BYTES * 2048 <= 120 * 1024 ? 2048 : 1024);
};

// (DC_MED_PROF builds: thread 0's s_memrealtime per section and counts -> rec[32..47], dc_med_prof_read)
#ifdef DC_MED_PROF
#define MPF_T(v) const unsigned long long v = __builtin_amdgcn_s_memrealtime()
#define MPF_ADD(i, x) (mpf[i] += (unsigned long long)(x))
#else
#define MPF_T(v) do {} while (0)
#define MPF_ADD(i, x) do {} while (0)
#endif

// inclusive scan of MXC_T transducers in thread order (wave scans by shuffles, one LDS round for the 16 wave
// totals: 3 barriers) -- only for a round with a tie somewhere (else plain prefix sums of the units)
constexpr int MXC_T = 1024;                                // compose workgroup
template <typename D>
__device__ __forceinline__ MTr<D> mtr_block_scan(MTr<D> v, MTr<D>* wt, D sat) {
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const MTr<D> o = mtr_shfl_up(v, d);
        if (lane >= d) v = mtr_then(o, v, sat);
    }
    if (lane == 63) wt[wid] = v;
    __syncthreads();
    if (wid == 0) {
        MTr<D> t = lane < MXC_T / 64 ? wt[lane] : MTr<D>{0, 0, 0, 1, 1 << 30};
#pragma unroll
        for (int d = 1; d < MXC_T / 64; d <<= 1) {
            const MTr<D> o = mtr_shfl_up(t, d);
            if (lane >= d) t = mtr_then(o, t, sat);
        }
        if (lane < MXC_T / 64) wt[MXC_T / 64 + lane] = t;     // inclusive over the waves
    }
    __syncthreads();
    if (wid > 0) v = mtr_then(wt[MXC_T / 64 + wid - 1], v, sat);
    __syncthreads();                                        // (wt is rewritten by the next scan)
    return v;
}

// k + x/u rounded as fl(s + x) rounds it, ties to even on the result (x >= 0 below the binade's top)
template <typename T>
__device__ __forceinline__ typename MedFP<T>::D med_units(T xv, T scale, typename MedFP<T>::D k) {
    typedef typename MedFP<T>::D D;
    const T q = MedFP<T>::mul(xv, scale);
    const T fq = floor(q);
    const T fr = MedFP<T>::sub(q, fq);
    const D fl = (D)fq;
    return fl + (fr > (T)0.5 ? 1 : (fr == (T)0.5 ? (D)((k + fl) & 1) : 0));
}

// Per-wave records of one round, exchanged through LDS between the round's two barriers
template <typename T>
struct MedRound {
    typedef typename MedFP<T>::D D;
    unsigned long long wt[MXC_T / 64];                      // wave totals of the clamped units
    int wtie[MXC_T / 64];                                   // the wave's first stopping lane (64: none)
    int wtf[MXC_T / 64];                                    // a tie among the wave's pieces
    int wl[MXC_T / 64];                                     // the wave's first leaving piece (1 << 30: none)
    D wk[MXC_T / 64];                                       // k before it
    T wv[MXC_T / 64];                                       // (elements: its value)
    int wy[MXC_T / 64];                                     // (chunks: 1 when it had no transducer for E)
    uint32_t wt2[MXC_T / 64];                               // (two-binade element rounds: the wave's units in E + 1,
    int wb2[MXC_T / 64];                                    //  its last element E + 1 does not take (-1: none),
    uint32_t wi2[MXC_T / 64];                               //  the E + 1 units through the leaving element)
};

// One round of the composition over MXC_T threads, each holding P pieces (chunks or elements) with units d0[j] /
// d1[j] from an even / odd k (equal but for a tie), stop[j] (no transducer), tie = some piece of the thread's is a
// tie.  From k0 (binade top TOP): the first piece (thread-major index) where the running k leaves the binade or
// that stops, k before it, the piece's value (v) and why -- or none (returns 1 << 30) and the k after all.  Two
// barriers when no thread has a tie (plain prefix sums of the units, DPP wave scans), the transducer block scan
// otherwise.  Every thread returns the same values.
//
// TWO (float element rounds): e2 / bad2 are the pieces' units in binade E + 1 (no tie there) and whether E + 1
// does not take them; two[0..3] return whether the E + 1 sums are usable (no tie in E, no wave total >= TOP),
// the E + 1 units of all live pieces, those through the leaving piece, and the last piece E + 1 does not take
// (-1: none) -- so that a sum crossing from E into E + 1 finishes the chunk in the same round (the caller checks).
template <typename T, int P, bool TWO = false>
__device__ __forceinline__ int med_round(const typename MedFP<T>::D (&d0)[P], const typename MedFP<T>::D (&d1)[P],
                                         const bool (&stop)[P], const bool (&live)[P], const T (&v)[P], const int (&why)[P],
                                         bool tie, typename MedFP<T>::D k0, MedRound<T>& X, MTr<typename MedFP<T>::D>* wt,
                                         typename MedFP<T>::D& k_out, T& v_out, int& why_out,
                                         unsigned long long* pf = nullptr, const uint32_t* e2 = nullptr,
                                         const bool* bad2 = nullptr, uint32_t* two = nullptr) {
    typedef MedFP<T> FP;
    typedef typename FP::D D;
    constexpr D TOP = D(1) << (FP::M + 1);
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
#ifdef DC_MED_PROF
#define MRS(i) do { if (pf && tid == 0) { const unsigned long long tt = __builtin_amdgcn_s_memrealtime(); pf[i] += tt - pf[7]; pf[7] = tt; } } while (0)
    if (pf && tid == 0) pf[7] = __builtin_amdgcn_s_memrealtime();
#else
#define MRS(i) do {} while (0)
#endif
    // the thread's pieces as one transducer (up to its first stop)
    D a0 = 0, a1 = 0;
    int q0 = 0, q1 = 1;
    bool st = false;
#pragma unroll
    for (int j = 0; j < P; j++) {
        if (live[j] && !st) {
            if (stop[j]) st = true;
            else compose(a0, a1, q0, q1, d0[j], d1[j], (int)(d0[j] & 1), (int)((d1[j] + 1) & 1), FP::SAT);
        }
    }
    MRS(0);
    // the fast path's wave scan, and the wave's tie / stop flags, before the first barrier: a tie anywhere
    // then selects the transducer scan (the flags travel with the wave totals -- __syncthreads_or cost ~0.8 us)
    const D uc = min(a0, TOP);
    unsigned long long incw;
    if (sizeof(D) == 4 && P <= 4) {
        incw = wave_scan_incl((uint32_t)uc);                // (64 x 4 x 2^24 pieces clamped: < 2^32)
    } else {
        incw = (unsigned long long)uc;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const unsigned long long o = __shfl_up(incw, d, 64);
            if (lane >= d) incw += o;
        }
    }
    const unsigned long long stb = __ballot(st), tb = __ballot(tie);
    uint32_t u2 = 0, incw2 = 0;
    if (TWO) {
        int myb = -1;
#pragma unroll
        for (int j = 0; j < P; j++) { u2 += e2[j]; myb = bad2[j] ? tid * P + j : myb; }
        incw2 = wave_scan_incl(u2);                         // (P x 2^24 per thread, 64 threads: < 2^32)
        const unsigned long long bb = __ballot(myb >= 0);
        if (lane == 63) X.wt2[wid] = incw2;
        if (lane == 0) X.wb2[wid] = bb ? __builtin_amdgcn_readlane(myb, 63 - __clzll((long long)bb)) : -1;
    }
    if (lane == 63) X.wt[wid] = incw;
    if (lane == 0) { X.wtie[wid] = stb ? (int)(__ffsll((long long)stb) - 1) : 64; X.wtf[wid] = tb != 0; }
    MRS(1);
    __syncthreads();
    MRS(2);
    // lanes 0..15 hold the 16 waves' records: prefix over waves by shuffles, read out with readlane
    constexpr int NW = MXC_T / 64;
    const int lw = lane & (NW - 1);
    unsigned long long wv = X.wt[lw];
    const int wst = X.wtie[lw], wtf = X.wtf[lw];
    const bool anytie = __ballot(lane < NW && wtf != 0) != 0;
    D k;
    bool before_ok;                                         // no earlier thread stops (its k is exact)
    if (!anytie) {
        unsigned long long woff;
        if (sizeof(D) == 4) {
            // (wave totals clamped to TOP: a wave adding that much leaves the binade by itself; 16 x 2^24 < 2^32,
            // so one DPP scan of 32-bit lanes instead of 64-bit shuffles through LDS)
            const uint32_t wp = wave_scan_incl(lane < NW ? (uint32_t)min(wv, (unsigned long long)TOP) : 0u);
            woff = wid > 0 ? (unsigned long long)(uint32_t)__builtin_amdgcn_readlane((int)wp, wid - 1) : 0ull;
        } else {
            unsigned long long wp = lane < NW ? wv : 0ull;  // inclusive over waves 0..lane
#pragma unroll
            for (int d = 1; d < NW; d <<= 1) {
                const unsigned long long o = __shfl_up(wp, d, 64);
                if (lane >= d) wp += o;
            }
            woff = wid > 0 ? ((unsigned long long)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)wp, wid - 1) |
                              ((unsigned long long)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(wp >> 32), wid - 1) << 32))
                           : 0ull;
        }
        const unsigned long long sbm = __ballot(lane < NW && lane < wid && wst < 64);   // an earlier wave stops
        const int fsl = __builtin_amdgcn_readlane(wst, wid);
        before_ok = sbm == 0 && lane <= fsl;
        const unsigned long long kx = (unsigned long long)k0 + woff + incw - (unsigned long long)uc;
        k = (D)min(kx, (unsigned long long)TOP);
        if (TWO) {
            const uint32_t wv2 = X.wt2[lw];
            const int wb2 = X.wb2[lw];
            const bool big = __ballot(lane < NW && wv2 >= (uint32_t)TOP) != 0ull;
            const uint32_t wp2 = wave_scan_incl(lane < NW ? min(wv2, (uint32_t)TOP) : 0u);
            const unsigned long long bb2 = __ballot(lane < NW && wb2 >= 0);
            two[0] = big ? 0u : 1u;
            two[1] = (uint32_t)__builtin_amdgcn_readlane((int)wp2, NW - 1);
            two[3] = bb2 ? (uint32_t)__builtin_amdgcn_readlane(wb2, 63 - __clzll((long long)bb2)) : 0xFFFFFFFFu;
            // (the thread's exclusive E + 1 prefix)
            u2 = (wid > 0 ? (uint32_t)__builtin_amdgcn_readlane((int)wp2, wid - 1) : 0u) + incw2 - u2;
        }
        MRS(3);
    } else {
        if (TWO) two[0] = 0u;
        const MTr<D> inc = mtr_block_scan<D>(MTr<D>{a0, a1, q0, q1, st ? tid : (1 << 30)}, wt, FP::SAT);
        // exclusive: the previous thread's inclusive
        MTr<D> ex = mtr_shfl_up(inc, 1);
        if (lane == 0) {
            if (wid > 0) ex = wt[MXC_T / 64 + wid - 1];
            else ex = MTr<D>{0, 0, 0, 1, 1 << 30};
        }
        const int par = (int)(k0 & 1);
        k = min(k0 + (par ? ex.a1 : ex.a0), TOP);
        before_ok = ex.fb == (1 << 30);
        __syncthreads();                                    // (wt of the scan read)
        MRS(3);
    }
    MRS(4);
    // walk the thread's pieces from its exact k: the first that stops or leaves
    int lj = P;
    if (before_ok && k < TOP) {
#pragma unroll
        for (int j = 0; j < P; j++) {
            if (lj == P && live[j]) {
                if (stop[j]) lj = j;
                else {
                    const D d = (k & 1) ? d1[j] : d0[j];
                    if (k + d >= TOP) lj = j;
                    else k += d;
                }
            }
        }
    } else if (before_ok) {
        lj = 0;                                             // (k >= TOP at the thread's start: cannot happen
    }                                                       //  without an earlier leave, kept for safety)
    const unsigned long long bl = __ballot(lj < P);
    if (bl) {
        const int L = __ffsll((long long)bl) - 1;
        if (lane == L) {
            X.wl[wid] = tid * P + lj;
            X.wk[wid] = k;
            T xv = v[0];
            int y = why[0];
#pragma unroll
            for (int j = 1; j < P; j++) { xv = j == lj ? v[j] : xv; y = j == lj ? why[j] : y; }
            X.wv[wid] = xv;
            X.wy[wid] = y;
            if (TWO) {
                uint32_t i2 = u2;
#pragma unroll
                for (int j = 0; j < P; j++) i2 += j <= lj ? e2[j] : 0u;
                X.wi2[wid] = i2;
            }
        }
    } else if (lane == 63) {
        X.wl[wid] = 1 << 30;
        X.wk[wid] = k;                                      // (the wave's last thread: k after it)
    }
    MRS(5);
    __syncthreads();
    // the first wave with a leaving piece (wl ascends with the wave), else the last wave's k
    const int wlv = X.wl[lw];
    const unsigned long long bw = __ballot(lane < NW && wlv < (1 << 30));
    const int fw = bw ? __ffsll((long long)bw) - 1 : NW - 1;
    const int f = bw ? __builtin_amdgcn_readlane(wlv, fw) : (1 << 30);
    k_out = X.wk[fw];
    v_out = X.wv[fw];
    why_out = X.wy[fw];
    if (TWO) two[2] = X.wi2[fw];
    MRS(6);
#undef MRS
    return f;
}

// The composition: one workgroup of 1024 threads.  A block of 1024 x CPT chunks (CPT consecutive chunks per
// thread, their records from the LDS ring) is one med_round; a chunk where the sum leaves its binade is added
// two elements per thread, each round adding the leaving element by one exact float add.  Every thread keeps the
// running sum and position in registers (the rounds return the same values everywhere): two barriers per round.
template <typename T, int W>
__global__ __launch_bounds__(MXC_T) void med_compose_kernel(const T* __restrict__ x, long long n, T s_init,
                                                           MedScratch<T> M, T* __restrict__ out_mean,
                                                           int* __restrict__ out_type, T* __restrict__ out_sum,
                                                           T* __restrict__ out_max, int gated,
                                                           const T* __restrict__ sub = nullptr) {
    typedef MedFP<T> FP;
    typedef typename FP::D D;
    typedef typename FP::U U;
    constexpr int R = MedRing<T, W>::R;
#ifndef DC_MED_CPT
#define DC_MED_CPT 2
#endif
    constexpr int CPT = R >= 4096 ? DC_MED_CPT : 1;         // chunks per thread in a block
    constexpr int BLK = MXC_T * CPT;
    __shared__ T buf[MC];                                   // (a chunk added by one lane)
    __shared__ int r_lo[R];                                 // ring slot: the chunk's first window binade
    __shared__ D r_a[R][W][2];                              // units from parity 0 / 1 per window binade
    __shared__ uint8_t r_f[R][W];                           // end parities | bad << 2
    __shared__ MedRound<T> X;
    __shared__ MTr<D> wt[2 * (MXC_T / 64)];
    __shared__ T s_one;
    __shared__ T smx[MXC_T / 64];
#ifdef DC_MED_PROF
    __shared__ unsigned long long s_pf[8];
    if (threadIdx.x < 8) s_pf[threadIdx.x] = 0;
    unsigned long long* pf = s_pf;
#else
    unsigned long long* pf = nullptr;
#endif
    if (gated && __hip_atomic_load(M.flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0u) return;
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const long long nch = (n + MC - 1) / MC;
#ifdef DC_MED_PROF
    unsigned long long mpf[16] = {0};
#endif
    T s = s_init;
    long long c = 0, lo = -(long long)R;
    int miss = 0;
    bool aborted = false;
    while (c < nch && s == s) {                             // (NaN + anything stays NaN)
        MPF_T(t0);
        if (FP::bits(s) == 0) {                             // +0 + (+-0) = +0: skip runs of zero chunks
            __syncthreads();                                // (X of the last round read everywhere)
            int jz = 1 << 30;
            for (int j = 0; j < CPT; j++) {
                const long long ch = c + (long long)tid * CPT + j;
                if (jz == (1 << 30) && ch < nch && !(M.Z[ch] & 1)) jz = tid * CPT + j;
            }
            const unsigned long long bz = __ballot(jz < (1 << 30));
            if (lane == 0) X.wl[wid] = bz ? __builtin_amdgcn_readlane(jz, __ffsll((long long)bz) - 1) : (1 << 30);
            __syncthreads();
            int f = 1 << 30;
            for (int w = 0; w < MXC_T / 64; w++) f = min(f, X.wl[w]);
            __syncthreads();
            MPF_ADD(0, 1);
            if (f == (1 << 30)) { c = min(nch, c + (long long)BLK); continue; }
            c += f;
        }
        bool serial = true;
        if (s >= FP::smin() && s < FP::smax()) {
            const int cnt = (int)min((long long)BLK, nch - c);
            if (c + cnt > lo + R) {                         // the ring: chunks [c, c + R)
                const long long from = max(lo + R, c), to = min(c + R, nch);
                // (every load of the thread's R / MXC_T chunks issued before the LDS stores: one round trip)
                constexpr int RPT = R / MXC_T;
                int e_[RPT];
                D a_[RPT][W][2];
                uint8_t f_[RPT][W];
#pragma unroll
                for (int q = 0; q < RPT; q++) {
                    const long long ch = from + tid + (long long)q * MXC_T;
                    const long long chc = ch < to ? ch : from;  // (a valid address; not stored)
                    e_[q] = M.eest[chc];
#pragma unroll
                    for (int w = 0; w < W; w++) {
                        a_[q][w][0] = M.Td[(chc * MW + w) * 2];
                        a_[q][w][1] = M.Td[(chc * MW + w) * 2 + 1];
                        f_[q][w] = M.F[chc * MW + w];
                    }
                }
#pragma unroll
                for (int q = 0; q < RPT; q++) {
                    const long long ch = from + tid + (long long)q * MXC_T;
                    if (ch < to) {
                        const int sl = (int)(ch % R);
                        r_lo[sl] = e_[q] + med_wlo<W>();
#pragma unroll
                        for (int w = 0; w < W; w++) {
                            r_a[sl][w][0] = a_[q][w][0];
                            r_a[sl][w][1] = a_[q][w][1];
                            r_f[sl][w] = f_[q][w];
                        }
                    }
                }
                __syncthreads();
                lo = c;
                MPF_ADD(2, 1);
            }
            MPF_T(t1);
            MPF_ADD(3, t1 - t0);
            MPF_ADD(1, 1);
            const U sbits = FP::bits(s);
            const int E = FP::expo(s);
            const D k0 = (D)((sbits & ((U(1) << FP::M) - 1)) | (U(1) << FP::M));
            D d0[CPT], d1[CPT];
            bool stop[CPT], live[CPT], tie = false;
            T vv[CPT];
            int why[CPT];
#pragma unroll
            for (int j = 0; j < CPT; j++) {
                const int t = tid * CPT + j;
                d0[j] = 0; d1[j] = 0; stop[j] = false; live[j] = t < cnt; vv[j] = (T)0; why[j] = 0;
                if (live[j]) {
                    const int sl = (int)((c + t) % R);
                    const int w = E - r_lo[sl];
                    if (w >= 0 && w < W) {
                        const int fl = r_f[sl][w];
                        d0[j] = r_a[sl][w][0];
                        d1[j] = r_a[sl][w][1];
                        // (d0 from an even k, d1 from an odd one; no tie: equal, and the end parities follow)
                        if (fl & 4) stop[j] = true;
                        else tie |= !(d0[j] == d1[j] && (fl & 1) == (int)(d0[j] & 1) && ((fl >> 1) & 1) == (int)((d1[j] + 1) & 1));
                    } else {
                        stop[j] = true;
                        why[j] = 1;
                    }
                }
            }
            D kf;
            T xv;
            int y;
            int f = med_round<T, CPT>(d0, d1, stop, live, vv, why, tie, k0, X, wt, kf, xv, y, pf);
            if (f >= cnt) f = cnt;
            else if (y == 1) miss++;
            s = FP::mul((T)kf, FP::pow2(E - FP::BIAS - FP::M));   // k * u, exact
            c += f;
            serial = f < cnt;
            MPF_T(t2);
            MPF_ADD(4, t2 - t1);
            if (W < MW && miss > MED_MISS_MAX) { aborted = true; break; }   // the narrow window keeps missing
        }
        if (!serial) continue;
        // chunk c element by element, two per thread: while the sum stays in a binade, the elements' units are
        // scanned and the first element that leaves it (or that no transducer takes) is added by one exact float
        // add; a sum that is not a positive normal, or a chunk that needs more than 8 such rounds, is finished by
        // one lane, exactly as the reference.
        MPF_T(t3);
        MPF_ADD(5, 1);
        const int m = (int)min((long long)MC, n - c * MC);
        T v2[2];
        {
            const long long e = c * MC + 2ll * tid;
            v2[0] = 2 * tid < m ? x[e] : (T)0;
            v2[1] = 2 * tid + 1 < m ? x[e + 1] : (T)0;
            if (sub) {
                const T mn = *sub;
                if (2 * tid < m) v2[0] = sub_fin(v2[0], mn);
                if (2 * tid + 1 < m) v2[1] = sub_fin(v2[1], mn);
            }
        }
        int i0 = 0;
        for (int it = 0; i0 < m; it++) {
            MPF_ADD(7, 1);
            if (FP::bits(s) == 0) {                         // +0 + (+-0) = +0: up to the first other element
                __syncthreads();                            // (X of the last round read everywhere)
                int jz = 1 << 30;
                T zv = (T)0;
                for (int j = 1; j >= 0; j--)
                    if (2 * tid + j >= i0 && 2 * tid + j < m && (FP::bits(v2[j]) << 1) != 0) { jz = 2 * tid + j; zv = v2[j]; }
                const unsigned long long bz = __ballot(jz < (1 << 30));
                if (bz) {
                    const int L = __ffsll((long long)bz) - 1;
                    if (lane == L) { X.wl[wid] = jz; X.wv[wid] = zv; }
                } else if (lane == 0) {
                    X.wl[wid] = 1 << 30;
                }
                __syncthreads();
                int f = 1 << 30, fw = 0;
                for (int w = MXC_T / 64 - 1; w >= 0; w--) if (X.wl[w] <= f) { f = X.wl[w]; fw = w; }
                const T fv = X.wv[fw];
                __syncthreads();
                if (f == (1 << 30)) { i0 = m; break; }
                s = FP::add(s, fv);
                i0 = f + 1;
                continue;
            }
            if (!(s >= FP::smin() && s < FP::smax()) || it >= 8) {
                MPF_ADD(8, 1);
                MPF_ADD(9, m - i0);
                if (2 * tid < m) buf[2 * tid] = v2[0];
                if (2 * tid + 1 < m) buf[2 * tid + 1] = v2[1];
                __syncthreads();
                if (tid == 0) {
                    T s2 = s;
                    int i = i0;
                    for (; i + 16 <= m; i += 16) {          // (16 LDS reads in flight, then the adds)
                        T b16[16];
#pragma unroll
                        for (int k2 = 0; k2 < 16; k2++) b16[k2] = buf[i + k2];
#pragma unroll
                        for (int k2 = 0; k2 < 16; k2++) s2 = FP::add(s2, b16[k2]);
                    }
                    for (; i < m; i++) s2 = FP::add(s2, buf[i]);
                    s_one = s2;
                }
                __syncthreads();
                s = s_one;
                __syncthreads();
                i0 = m;
                break;
            }
            const U sb2 = FP::bits(s);
            const int E = FP::expo(s);
            const D k0 = (D)((sb2 & ((U(1) << FP::M) - 1)) | (U(1) << FP::M));
            const T scale = FP::pow2(FP::BIAS + FP::M - E), lim = FP::pow2(E + 1 - FP::BIAS);
            D d0[2], d1[2];
            bool stop[2], live[2], tie = false;
            int why[2] = {0, 0};
            // (float: the units in E + 1 too, so that a sum crossing into the next binade finishes the chunk in
            //  this round when nothing after the crossing leaves E + 1 or ties there)
            constexpr bool TW = sizeof(D) == 4;
            uint32_t e2[2] = {0u, 0u}, two[4] = {0u, 0u, 0u, 0u};
            bool bad2[2] = {false, false};
            const bool e2ok = TW && E + 1 <= FP::EMAX;
#pragma unroll
            for (int j = 0; j < 2; j++) {
                const int e = 2 * tid + j;
                live[j] = e >= i0 && e < m;
                stop[j] = false; d0[j] = 0; d1[j] = 0;
                if (live[j]) {
                    if (!(v2[j] >= (T)0 && v2[j] < lim)) stop[j] = true;
                    else {
                        d0[j] = med_units<T>(v2[j], scale, (D)0);   // from an even k
                        d1[j] = med_units<T>(v2[j], scale, (D)1);   // from an odd one
                        tie |= d0[j] != d1[j];
                    }
                    if (TW) {
                        if (e2ok && v2[j] >= (T)0 && v2[j] < FP::mul(lim, (T)2)) {
                            const T sc2 = FP::mul(scale, (T)0.5);
                            const D a = med_units<T>(v2[j], sc2, (D)0), b = med_units<T>(v2[j], sc2, (D)1);
                            e2[j] = (uint32_t)a;
                            bad2[j] = a != b;
                        } else {
                            bad2[j] = true;
                        }
                    }
                }
            }
            D kf;
            T xv;
            int y;
            const int f = med_round<T, 2, TW>(d0, d1, stop, live, v2, why, tie, k0, X, wt, kf, xv, y, pf, e2, bad2, two);
            const T u = FP::pow2(E - FP::BIAS - FP::M);
            if (f >= (1 << 30)) {                           // the rest of the chunk stays in the binade
                s = FP::mul((T)kf, u);
                i0 = m;
                break;
            }
            s = FP::add(FP::mul((T)kf, u), xv);             // the leaving element, exactly
            i0 = f + 1;
            if (TW && two[0] && (int)two[3] <= f && s >= FP::smin() && s < FP::smax() && FP::expo(s) == E + 1) {
                // the rest of the chunk in E + 1: k' + its units, if that stays below the binade's top
                const U sb3 = FP::bits(s);
                const D k2 = (D)((sb3 & ((U(1) << FP::M) - 1)) | (U(1) << FP::M));
                const D ke = k2 + (D)(two[1] - two[2]);
                if (ke < (D(1) << (FP::M + 1))) {
                    s = FP::mul((T)ke, FP::mul(u, (T)2));
                    i0 = m;
                    MPF_ADD(6, 1);
                    break;
                }
            }
        }
        c += 1;
        MPF_T(t4);
        MPF_ADD(10, t4 - t3);
    }
#ifdef DC_MED_PROF
    if (tid == 0) {
        for (int i = 0; i < 9; i++) M.rec[32 + i] = (long long)mpf[i];
        mpf[10] = mpf[10];
        M.rec[32 + 9] = (long long)mpf[10];
        for (int i = 0; i < 6; i++) M.rec[32 + 10 + i] = (long long)s_pf[i + 1];   // med_round sections 1..6
    }
#endif
    if (aborted) {                                          // (uniform: every thread holds the same state)
        if (tid == 0) *M.flag = 1u;
        return;
    }
    // max: x[0] folded with every chunk's max (strict >, as the reference's loop)
    T mx = -INFINITY;
    for (long long cc = tid; cc < nch; cc += MXC_T) { const T v = M.cmax[cc]; mx = v > mx ? v : mx; }
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) { const T o = __shfl_xor(mx, d, 64); mx = o > mx ? o : mx; }
    if ((tid & 63) == 0) smx[tid >> 6] = mx;
    __syncthreads();
    if (tid == 0) {
        T mm = sub ? sub_fin(x[0], *sub) : x[0];
        for (int i = 0; i < MXC_T / 64; i++) if (smx[i] > mm) mm = smx[i];
        const T mean = FP::mean(s, n);
        const int ty = FP::type(mm);
        *out_type = ty;
        *out_mean = mean;
        if (out_sum) *out_sum = s;
        if (out_max) *out_max = mm;
        M.res[0] = (long long)FP::bits(mean);
        M.res[1] = ty;
        M.res[2] = (long long)FP::bits(s);
        M.res[3] = (long long)FP::bits(mm);
    }
}

// A rank's contiguous shard of the global array (multi-GPU med_dataset_float, dcamd.global_med), one
// workgroup over the chunk records:
//   trans = 0: the shard's double sum (an estimate of what it adds), the max of its chunk maxes (NaNs
//              never win) and x[0]; the global max folds the first shard's x[0] with every shard's max,
//              strict >, as med_compose_kernel
//   trans = 1: the whole shard as one transducer for each binade E of the first chunk's wide window
//              [E_est - 4, E_est + 2): start parity -> (units added, end parity), "bad" where some chunk has
//              no transducer for E (E outside its window, or an element it cannot take).  A rank whose
//              running sum enters in such a binade and stays in it (k + units < 2^24) ends at k + units
//              without a pass of its own; composing these over the ranks is the exscan of global_med.
// rec: [0] sum (double bits) [1] max (bits) [2] x[0] (bits) | elo[0] [3 + 2w + p] units from parity p [15 + w] flags
template <typename T>
__global__ __launch_bounds__(MX_T) void med_shard_kernel(const T* __restrict__ x, long long nch, MedScratch<T> M,
                                                         int trans, long long* __restrict__ rec) {
    typedef MedFP<T> FP;
    typedef typename FP::D D;
    __shared__ double ws[MX_T / 64];
    __shared__ T wm[MX_T / 64];
    __shared__ D sd[MW][MX_T / 64][2];
    __shared__ int sf[MW][MX_T / 64];
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const long long per = (nch + MX_T - 1) / MX_T, c0 = min(nch, tid * per), c1 = min(nch, c0 + per);
    if (!trans) {
        double sm = 0.0;
        T mx = -INFINITY;
        for (long long c = c0; c < c1; c++) { sm += M.csum[c]; const T v = M.cmax[c]; mx = v > mx ? v : mx; }
#pragma unroll
        for (int d = 32; d >= 1; d >>= 1) {
            sm += __shfl_xor(sm, d, 64);
            const T o = __shfl_xor(mx, d, 64);
            mx = o > mx ? o : mx;
        }
        if (lane == 0) { ws[wid] = sm; wm[wid] = mx; }
        __syncthreads();
        if (tid == 0) {
            double t = 0.0;
            T mm = -INFINITY;
            for (int w = 0; w < MX_T / 64; w++) { t += ws[w]; if (wm[w] > mm) mm = wm[w]; }
            rec[0] = __double_as_longlong(t);
            rec[1] = (long long)FP::bits(mm);
            rec[2] = (long long)FP::bits(x[0]);
        }
        return;
    }
    const int e0 = M.eest[0] + med_wlo<MW>();
#pragma unroll 1
    for (int w = 0; w < MW; w++) {
        const int E = e0 + w;
        D a0 = 0, a1 = 0;
        int q0 = 0, q1 = 1;
        bool bad = false;
        for (long long c = c0; c < c1; c++) {
            const int wc = E - (M.eest[c] + med_wlo<MW>());
            if (wc < 0 || wc >= MW) { bad = true; break; }
            const int f = M.F[c * MW + wc];
            compose(a0, a1, q0, q1, M.Td[(c * MW + wc) * 2], M.Td[(c * MW + wc) * 2 + 1], f & 1, (f >> 1) & 1, FP::SAT);
            bad |= (f & 4) != 0;
        }
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {                  // ordered: lane i absorbs lane i + d
            const D b0 = __shfl_down(a0, d, 64), b1 = __shfl_down(a1, d, 64);
            const int f = __shfl_down(q0 | (q1 << 1) | ((int)bad << 2), d, 64);
            if ((lane & (2 * d - 1)) == 0) {
                compose(a0, a1, q0, q1, b0, b1, f & 1, (f >> 1) & 1, FP::SAT);
                bad |= (f & 4) != 0;
            }
        }
        if (lane == 0) { sd[w][wid][0] = a0; sd[w][wid][1] = a1; sf[w][wid] = q0 | (q1 << 1) | ((int)bad << 2); }
    }
    __syncthreads();
    if (tid < MW) {
        const int w = tid;
        D a0 = sd[w][0][0], a1 = sd[w][0][1];
        int q0 = sf[w][0] & 1, q1 = (sf[w][0] >> 1) & 1;
        bool bad = (sf[w][0] & 4) != 0;
        for (int k = 1; k < MX_T / 64; k++) {
            compose(a0, a1, q0, q1, sd[w][k][0], sd[w][k][1], sf[w][k] & 1, (sf[w][k] >> 1) & 1, FP::SAT);
            bad |= (sf[w][k] & 4) != 0;
        }
        rec[3 + 2 * w] = (long long)a0;
        rec[4 + 2 * w] = (long long)a1;
        rec[15 + w] = q0 | (q1 << 1) | (bad ? 4 : 0);
        if (w == 0) rec[2] = e0;
    }
}

// the transducer grid: one wave per chunk, at most 4096 workgroups of 4 (a gated launch that ends at once
// costs ~3 us, not a full grid's dispatch)
static inline unsigned med_trans_grid(long long nch) { return (unsigned)min((nch + 3) / 4, 4096ll); }

template <typename T>
static int launch_med(const T* x, long long n, T s_init, void* scratch, T* d_mean, int* d_type, T* d_sum, T* d_max,
                      int wide, hipStream_t st) {
    if (n <= 0) return 0;
    const long long nch = (n + MC - 1) / MC;
    const MedScratch<T> M = med_scratch<T>(scratch, nch);
    const unsigned tg = med_trans_grid(nch);
    // wide: 0 the narrow window; 1 the wide one after the narrow compose raised the flag (the chunk sums, max
    // and binade estimates of that call are in the scratch); 2 the wide one on a fresh array (DC_MED_WIDE=1:
    // the chunk sums and the estimate scan run first, nothing is taken from an earlier call's scratch)
    if (wide != 1) {
        hipLaunchKernelGGL(med_chunk_sum_kernel<T>, dim3((unsigned)nch), dim3(MC_T), 0, st, x, n, M);
        hipLaunchKernelGGL(med_chunk_scan_kernel<T>, dim3(1), dim3(1024), 0, st, M, nch, s_init);
    }
    if (!wide) {
        hipLaunchKernelGGL((med_chunk_trans_kernel<T, MWN>), dim3(tg), dim3(256), 0, st, x, n, M, 0);
        hipLaunchKernelGGL((med_compose_kernel<T, MWN>), dim3(1), dim3(MXC_T), 0, st, x, n, s_init, M, d_mean, d_type,
                           d_sum, d_max, 0);
    } else {
        hipLaunchKernelGGL((med_chunk_trans_kernel<T, MW>), dim3(tg), dim3(256), 0, st, x, n, M, 0);
        hipLaunchKernelGGL((med_compose_kernel<T, MW>), dim3(1), dim3(MXC_T), 0, st, x, n, s_init, M, d_mean, d_type,
                           d_sum, d_max, 0);
    }
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

// dc_prep_device's kernels: wide 0 -- statistics of x and the minimum (into *d_min), the statistics of x - m, the
// binade estimates, the narrow window's transducers and compose; wide 1 -- the wide window after a narrow miss (the
// statistics of that call are in the scratch).  pv / pi: nch partial minima.  The result words as dc_launch_med's,
// plus res[4] = 1 when the minimum is not finite (nothing else is valid then)
extern "C" int dc_launch_med_sub(const float* x, long long n, void* scratch, float* d_min, float* pv, long long* pi,
                                 float* d_mean, int* d_type, int wide, hipStream_t st) {
    if (n <= 0) return 0;
    const long long nch = (n + MC - 1) / MC;
    const MedScratch<float> M = med_scratch<float>(scratch, nch);
    const unsigned tg = med_trans_grid(nch);
    if (wide != 1) {                                     // (2: the wide window on a fresh array, DC_MED_WIDE=1)
        hipLaunchKernelGGL(med_chunk_stats_kernel, dim3((unsigned)nch), dim3(MC_T), 0, st, x, n, M, pv, pi);
        hipLaunchKernelGGL(prep_min_fix_kernel, dim3(1), dim3(PF_T), 0, st, x, n, M, (const float*)pv,
                           (const long long*)pi, d_min);
        hipLaunchKernelGGL(med_chunk_scan_kernel<float>, dim3(1), dim3(1024), 0, st, M, nch, 0.0f);
    }
    if (!wide) {
        hipLaunchKernelGGL((med_chunk_trans_kernel<float, MWN>), dim3(tg), dim3(256), 0, st, x, n, M, 0, (const float*)d_min);
        hipLaunchKernelGGL((med_compose_kernel<float, MWN>), dim3(1), dim3(MXC_T), 0, st, x, n, 0.0f, M, d_mean, d_type,
                           (float*)nullptr, (float*)nullptr, 0, (const float*)d_min);
    } else {
        hipLaunchKernelGGL((med_chunk_trans_kernel<float, MW>), dim3(tg), dim3(256), 0, st, x, n, M, 0, (const float*)d_min);
        hipLaunchKernelGGL((med_compose_kernel<float, MW>), dim3(1), dim3(MXC_T), 0, st, x, n, 0.0f, M, d_mean, d_type,
                           (float*)nullptr, (float*)nullptr, 0, (const float*)d_min);
    }
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

// the narrow-window flag of a med scratch for n elements (1: run dc_launch_med*_wide)
extern "C" unsigned* dc_med_flag_ptr(void* scratch, long long n, int is_double) {
    const long long nch = (n + MC - 1) / MC;
    return is_double ? med_scratch<double>(scratch, nch).flag : med_scratch<float>(scratch, nch).flag;
}

// ---------------------------------------------------------------- CRC-32 (zlib)
constexpr uint32_t CRC_POLY = 0xEDB88320u;
constexpr int CRC_RUN = 128;                              // bytes per lane (8 x 16-byte loads)
constexpr int CRC_BLK = CRC_RUN * 256;                    // bytes per workgroup

__device__ __forceinline__ uint32_t multmodp(uint32_t a, uint32_t b) {     // a*b mod P (reflected)
    uint32_t m = 1u << 31, p = 0;
    for (int i = 0; i < 32; i++) {
        if (a & m) p ^= b;
        m >>= 1;
        b = (b & 1u) ? (b >> 1) ^ CRC_POLY : b >> 1;
    }
    return p;
}

__device__ __forceinline__ uint32_t xpow8n(unsigned long long n, const uint32_t* x2n) {  // x^(8n) mod P
    uint32_t p = 1u << 31;
    int k = 3;
    while (n) {
        if (n & 1) p = multmodp(x2n[k & 31], p);
        n >>= 1;
        k++;
    }
    return p;
}

// Raw CRC (init 0, no final xor) of every CRC_BLK block.  Each lane takes a 128-byte run with
// 16-byte loads and slicing-by-4 tables in LDS (T_k = table of a byte followed by k zero bytes, built
// on the host from zlib's byte table); CRC is linear over GF(2), so the block value is the XOR of
// every run's CRC times x^(8 * bytes after it) -- for full blocks a per-lane host constant
// kpow[j] = x^(8 * CRC_RUN * j), so the combine is one carry-less multiply and an XOR reduction.
// DC_CRC_NIB (default): the word step by eight 16-entry nibble tables (nib[j][v] = the byte table entry of
// nibble j alone: CRC is linear, T[b] = T[b & 15] ^ T[b & 0xF0]).  A wave's 64 lookups into one 16-entry
// table hit at most 16 banks, each address once or broadcast -- no bank conflicts -- where the four
// 256-entry byte tables' random lookups serialised on conflicts (the CRC pass ran at ~2 TB/s).
#ifndef DC_CRC_NIB
#define DC_CRC_NIB 1
#endif
#ifndef DC_CRC_DIAG
#define DC_CRC_DIAG 0                   // (diagnostics: 1 = loads without the table step, 2 = table steps without loads)
#endif
#ifndef DC_CRC_STAGE
#define DC_CRC_STAGE 0                  // (staging full blocks through LDS: 66 -> 71 us per pass, off)
#endif
// COPY (the CT9 resend): only when the gate's two CRCs differ (the received copy was damaged), the run is also
// written to dst -- the resent copy and its CRC in one pass -- and gate_count counts the resends
// (blockIdx.y = 1: the second buffer s2 into part2 -- the CT9 pair pass, dc_crc32_pair_device)
template <bool COPY>
__global__ __launch_bounds__(256) void crc_blocks_kernel(const uint8_t* __restrict__ s_in, long long nbytes,
                                                         const uint32_t* __restrict__ tab_g,
                                                         const uint32_t* __restrict__ kpow_g,
                                                         const uint32_t* __restrict__ x2n_g,
                                                         uint32_t* __restrict__ part_in, uint8_t* __restrict__ dst,
                                                         const uint32_t* __restrict__ gate, unsigned* __restrict__ gate_count,
                                                         const uint8_t* __restrict__ s2, uint32_t* __restrict__ part2) {
    const uint8_t* __restrict__ s = blockIdx.y ? s2 : s_in;
    uint32_t* __restrict__ part = blockIdx.y ? part2 : part_in;
    if (COPY && gate) {
        if (gate[0] == gate[1]) return;
        if (gate_count && blockIdx.x == 0 && threadIdx.x == 0) atomicAdd(gate_count, 1u);
    }
    __shared__ uint32_t tab[DC_CRC_NIB ? 1 : 4][256];
    __shared__ uint32_t nib[8 * 16];
    __shared__ uint32_t x2n[32];
    __shared__ uint32_t red[4];
    // DC_CRC_STAGE: a full block is read with coalesced 16-byte loads (a wave instruction covers 1 KiB)
    // and handed to the lanes' 128-byte runs through LDS rows of 36 words (b128 reads conflict-free):
    // each lane loading its own run touched 64 lines per instruction (~2.6 TB/s)
    // (COPY stages too: the copy's stores then cover 1 KiB per wave instruction like its loads -- per-lane runs
    // stored 64 lines per instruction and the resend took 97 us per 163 MB, about copy + CRC)
    constexpr bool STAGE = DC_CRC_STAGE || COPY;
    __shared__ __attribute__((aligned(16))) uint32_t stg[STAGE ? 256 * 36 : 4];
    const int t = threadIdx.x;
    for (int k = 0; k < (DC_CRC_NIB ? 1 : 4); k++) tab[k][t] = tab_g[k * 256 + t];
    if (t < 128) {                                   // nibble j of the word c: byte table 3 - j/2
        const int j = t >> 4, v = t & 15;
        nib[t] = tab_g[(3 - (j >> 1)) * 256 + ((j & 1) ? (v << 4) : v)];
    }
    if (t < 32) x2n[t] = x2n_g[t];
    const uint32_t kfull = kpow_g[255 - t];
    __syncthreads();
    const bool al = (reinterpret_cast<uintptr_t>(s) & 15u) == 0;
    const long long nblk = (nbytes + CRC_BLK - 1) / CRC_BLK;
    for (long long b = blockIdx.x; b < nblk; b += gridDim.x) {
        const long long st = b * CRC_BLK + (long long)t * CRC_RUN;
        uint32_t r = 0;
        const bool staged = STAGE && al && (b + 1) * CRC_BLK <= nbytes &&
                            (!COPY || (reinterpret_cast<uintptr_t>(dst) & 15u) == 0);   // (uniform: a full block)
        if (staged) {
            const uint4* g4 = reinterpret_cast<const uint4*>(s + b * CRC_BLK);
            uint4 v[CRC_RUN / 16];
#pragma unroll
            for (int i = 0; i < CRC_RUN / 16; i++) v[i] = g4[t + 256 * i];
            if (COPY) {
                uint4* d4 = reinterpret_cast<uint4*>(dst + b * CRC_BLK);
#pragma unroll
                for (int i = 0; i < CRC_RUN / 16; i++) d4[t + 256 * i] = v[i];
            }
#pragma unroll
            for (int i = 0; i < CRC_RUN / 16; i++) {
                const int u = t + 256 * i;                      // 16-byte unit: run u / 8, piece u % 8
                *reinterpret_cast<uint4*>(&stg[(u >> 3) * 36 + (u & 7) * 4]) = v[i];
            }
            __syncthreads();
        }
        if (al && st + CRC_RUN <= nbytes && (!COPY || (reinterpret_cast<uintptr_t>(dst) & 15u) == 0)) {
            const uint4* p4 = reinterpret_cast<const uint4*>(s + st);
            uint4 q[CRC_RUN / 16];
#pragma unroll
            for (int i = 0; i < CRC_RUN / 16; i++)
                q[i] = DC_CRC_DIAG == 2 ? make_uint4((uint32_t)st + i, (uint32_t)b, 3u * i, 7u)   // (diagnostic: no loads)
                                        : staged ? *reinterpret_cast<const uint4*>(&stg[t * 36 + 4 * i]) : p4[i];
            if (COPY && !staged) {
                uint4* d4 = reinterpret_cast<uint4*>(dst + st);
#pragma unroll
                for (int i = 0; i < CRC_RUN / 16; i++) d4[i] = q[i];
            }
#pragma unroll
            for (int i = 0; i < CRC_RUN / 16; i++) {
                const uint32_t w[4] = {q[i].x, q[i].y, q[i].z, q[i].w};
#pragma unroll
                for (int j = 0; j < 4; j++) {
                    const uint32_t c = r ^ w[j];
                    if (DC_CRC_DIAG == 1) {                  // (diagnostic: loads only, no table step)
                        r = (c << 1) ^ (c >> 31);
                    } else if (DC_CRC_NIB) {
                        r = (nib[0 * 16 + (c & 15u)] ^ nib[1 * 16 + ((c >> 4) & 15u)]) ^
                            (nib[2 * 16 + ((c >> 8) & 15u)] ^ nib[3 * 16 + ((c >> 12) & 15u)]) ^
                            ((nib[4 * 16 + ((c >> 16) & 15u)] ^ nib[5 * 16 + ((c >> 20) & 15u)]) ^
                             (nib[6 * 16 + ((c >> 24) & 15u)] ^ nib[7 * 16 + (c >> 28)]));
                    } else {
                        r = tab[3][c & 0xFFu] ^ tab[2][(c >> 8) & 0xFFu] ^ tab[1][(c >> 16) & 0xFFu] ^ tab[0][c >> 24];
                    }
                }
            }
        } else {
            for (long long p = st; p < st + CRC_RUN && p < nbytes; p++) {
                const uint8_t v = s[p];
                if (COPY) dst[p] = v;
                r = tab[0][(r ^ v) & 0xFFu] ^ (r >> 8);
            }
        }
        const long long blen = min((long long)CRC_BLK, nbytes - b * CRC_BLK);
        uint32_t v;
        if (blen == CRC_BLK) {
            v = multmodp(kfull, r);
        } else {                                          // the last, partial block
            const long long end = min(st + CRC_RUN, nbytes);
            const long long after = b * CRC_BLK + blen - max(end, st);
            v = (r && after > 0) ? multmodp(xpow8n((unsigned long long)after, x2n), r) : r;
        }
#pragma unroll
        for (int d = 32; d >= 1; d >>= 1) v ^= __shfl_xor(v, d, 64);
        if ((t & 63) == 0) red[t >> 6] = v;
        __syncthreads();
        if (t == 0) part[b] = red[0] ^ red[1] ^ red[2] ^ red[3];
        __syncthreads();
    }
}

// Constants of the final combine, computed on the host from nbytes (Kb = x^(8 CRC_BLK); the full blocks
// are padded at the front to 256 threads x `per` blocks -- leading zero blocks add nothing)
struct CrcFin {
    uint32_t kb, lvl[8], kl, xn;   // lvl[l] = x^(8 CRC_BLK per 2^l), kl = x^(8 * last block), xn = x^(8 nbytes)
    long long nblk, per, pad;
};

// part[] = raw CRC of every block; the stream's zlib CRC: thread t folds its `per` consecutive blocks by
// Horner (r = r Kb ^ part), an 8-level tree joins neighbours with one constant each, and the last
// (partial) block and the zlib init / final xor are applied by thread 0 -- about 40 carry-less
// multiplies on the critical path (the generic x^(8n) per tree node took 80-100 us)
__global__ __launch_bounds__(256) void crc_final_kernel(const uint32_t* __restrict__ part, CrcFin F, uint32_t init,
                                                        uint32_t* __restrict__ out) {
    __shared__ uint32_t red[256];
    const int t = threadIdx.x;
    uint32_t r = 0;
    const long long m = F.nblk > 0 ? F.nblk - 1 : 0;                 // full blocks
    for (long long i = 0; i < F.per; i++) {
        const long long b = (long long)t * F.per + i - F.pad;
        r = multmodp(F.kb, r) ^ (b >= 0 && b < m ? part[b] : 0u);
    }
    red[t] = r;
    __syncthreads();
#pragma unroll
    for (int l = 0; l < 8; l++) {
        const int w = 1 << l;
        uint32_t v = 0;
        const bool act = (t & (2 * w - 1)) == 0;
        if (act) v = multmodp(F.lvl[l], red[t]) ^ red[t + w];
        __syncthreads();
        if (act) red[t] = v;
        __syncthreads();
    }
    if (t == 0) {
        uint32_t R = red[0];
        if (F.nblk > 0) R = multmodp(F.kl, R) ^ part[F.nblk - 1];
        // zlib: crc32(init, buf) = ~(raw(buf) ^ shift(~init, n))
        *out = ~(R ^ multmodp(F.xn, ~init));
    }
}

// DC_CRC_FIN2 (default): the same combine on 1024 threads with table-driven constant multiplies.  A product
// a * K mod P is linear in a: with B[i] = (bit i alone) * K = K x^(31 - i) (B[31] = K, each lower one the
// next times x: a shift and a conditional xor), the four byte tables T[j][v] = XOR of B[8 j + k] over the set
// bits k of v give a * K = T[0][a & 255] ^ T[1][a >> 8 & 255] ^ T[2][a >> 16 & 255] ^ T[3][a >> 24]: four LDS
// reads instead of 32 dependent shift/xor steps.  Tables for Kb and the ten tree levels (45 KB of LDS) are
// built in the kernel (11 lanes compute the bases, every thread 11 entries).
#ifndef DC_CRC_FIN2
#define DC_CRC_FIN2 1
#endif
constexpr int CF2_T = 1024, CF2_L = 10;
struct CrcFin2 {
    uint32_t kc[1 + CF2_L];     // kc[0] = Kb = x^(8 CRC_BLK); kc[1 + l] = x^(8 CRC_BLK per 2^l)
    uint32_t kl, xn;
    long long nblk, per, pad;
};
__device__ __forceinline__ uint32_t mul_tab(const uint32_t (*T)[256], uint32_t a) {
    return (T[0][a & 255u] ^ T[1][(a >> 8) & 255u]) ^ (T[2][(a >> 16) & 255u] ^ T[3][a >> 24]);
}
// gate (the CT9 resend): only when its two CRCs differ; ref / count: a result != *ref counts in *count
// (blockIdx.x = 1: the second buffer's blocks part2 into out2)
__global__ __launch_bounds__(CF2_T) void crc_final2_kernel(const uint32_t* __restrict__ part_in, CrcFin2 F, uint32_t init,
                                                           uint32_t* __restrict__ out_in, const uint32_t* __restrict__ gate,
                                                           const uint32_t* __restrict__ ref, unsigned* __restrict__ count,
                                                           const uint32_t* __restrict__ part2, uint32_t* __restrict__ out2) {
    if (gate && gate[0] == gate[1]) return;
    const uint32_t* __restrict__ part = blockIdx.x ? part2 : part_in;
    uint32_t* __restrict__ out = blockIdx.x ? out2 : out_in;
    __shared__ uint32_t T[1 + CF2_L][4][256];
    __shared__ uint32_t B[1 + CF2_L][32];
    __shared__ uint32_t red[CF2_T];
    const int t = threadIdx.x;
    if (t < 1 + CF2_L) {
        uint32_t b = F.kc[t];
        B[t][31] = b;
        for (int i = 30; i >= 0; i--) {
            b = (b & 1u) ? (b >> 1) ^ CRC_POLY : b >> 1;
            B[t][i] = b;
        }
    }
    __syncthreads();
    for (int e = t; e < (1 + CF2_L) * 1024; e += CF2_T) {
        const int c = e >> 10, j = (e >> 8) & 3, v = e & 255;
        uint32_t x = 0;
#pragma unroll
        for (int k = 0; k < 8; k++)
            if ((v >> k) & 1) x ^= B[c][8 * j + k];
        T[c][j][v] = x;
    }
    __syncthreads();
    uint32_t r = 0;
    const long long m = F.nblk > 0 ? F.nblk - 1 : 0;                 // full blocks
    for (long long i = 0; i < F.per; i++) {
        const long long b = (long long)t * F.per + i - F.pad;
        r = mul_tab(T[0], r) ^ (b >= 0 && b < m ? part[b] : 0u);
    }
    red[t] = r;
    __syncthreads();
#pragma unroll
    for (int l = 0; l < CF2_L; l++) {
        const int w = 1 << l;
        uint32_t v = 0;
        const bool act = (t & (2 * w - 1)) == 0;
        if (act) v = mul_tab(T[1 + l], red[t]) ^ red[t + w];
        __syncthreads();
        if (act) red[t] = v;
        __syncthreads();
    }
    if (t == 0) {
        uint32_t R = red[0];
        if (F.nblk > 0) R = multmodp(F.kl, R) ^ part[F.nblk - 1];
        const uint32_t crc = ~(R ^ multmodp(F.xn, ~init));
        *out = crc;
        if (ref && count && crc != *ref) atomicAdd(count, 1u);
    }
}

static uint32_t h_mult(uint32_t a, uint32_t b) {
    uint32_t m = 1u << 31, p = 0;
    for (int i = 0; i < 32; i++) {
        if (a & m) p ^= b;
        m >>= 1;
        b = (b & 1u) ? (b >> 1) ^ CRC_POLY : b >> 1;
    }
    return p;
}
static uint32_t h_xpow8n(unsigned long long n) {                      // x^(8n) mod P
    static uint32_t x2n[64];
    static bool init = false;
    if (!init) {
        uint32_t p = 1u << 30;                                          // x^1
        x2n[0] = p;
        for (int k = 1; k < 64; k++) x2n[k] = p = h_mult(p, p);
        init = true;
    }
    uint32_t p = 1u << 31;
    int k = 3;
    while (n) {
        if (n & 1) p = h_mult(x2n[k & 63], p);
        n >>= 1;
        k++;
    }
    return p;
}

// ---------------------------------------------------------------- fused CRC-32 over 16 KiB blocks
// (dc_device.h): producers XOR each block's raw CRC into blk[b]; crcf_final_kernel combines them.
// crcf_blocks_kernel: the blocks of a byte range, one workgroup per block, a 64-byte group per thread (four
// 16-byte loads, its raw CRC, then x^(8 * bytes after the group in the block) by one carry-less multiply);
// dst != NULL copies the range while it passes (the CT9 resend: the receiver's CRC of the resent copy costs no
// pass of its own).  Reads whole 16-byte groups: the buffer must be readable to nbytes rounded up to 16
// (stream buffers of dc_stream_capacity are); bytes past nbytes count as zero, and dst gets zeros there.
extern "C" long long dc_crcf_blocks(long long nbytes) { return crcf_nblk(nbytes); }

__global__ __launch_bounds__(256) void crcf_blocks_kernel(const uint8_t* __restrict__ src, uint8_t* __restrict__ dst,
                                                          long long nbytes, const uint32_t* __restrict__ ctab,
                                                          uint32_t* __restrict__ blk, const uint32_t* __restrict__ gate,
                                                          unsigned* __restrict__ gate_count) {
    if (gate && gate[0] == gate[1]) return;                 // (the CT9 resend: only after a mismatch)
    if (gate_count && blockIdx.x == 0 && threadIdx.x == 0) atomicAdd(gate_count, 1u);
    __shared__ uint32_t nib[128];
    __shared__ uint32_t red[4];
    const int t = threadIdx.x;
    if (t < 128) nib[t] = ctab[CRCF_NIB + t];
    const uint32_t kq = ctab[CRCF_KQ + 2 * (255 - t)];     // group t: 64 (255 - t) bytes before the block's end
    __syncthreads();
    typedef unsigned v4u __attribute__((ext_vector_type(4)));
    const int rng = (int)min((nbytes + 15) / 16 * 16, 0x7FFFFF00ll);
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(src), (short)0, rng, 0x00020000);
    const __amdgpu_buffer_rsrc_t rd = __builtin_amdgcn_make_buffer_rsrc(dst, (short)0, rng, 0x00020000);
    const long long nblk = crcf_nblk(nbytes);
    for (long long b = blockIdx.x; b < nblk; b += gridDim.x) {
        const long long g0 = b * DC_CRCF_BLK + 64ll * t;         // (streams below 2 GiB)
        v4u q[4];
#pragma unroll
        for (int i = 0; i < 4; i++) q[i] = __builtin_amdgcn_raw_buffer_load_b128(rs, (int)(g0 + 16 * i), 0, 0);
        uint32_t r = 0;
#pragma unroll
        for (int i = 0; i < 4; i++) {
            const long long o = g0 + 16 * i;
            if (o + 16 > nbytes) {                                  // the stream's last group: zeros past its end
#pragma unroll
                for (int j = 0; j < 4; j++) {
                    const long long rem = nbytes - (o + 4 * j);
                    const uint32_t m = rem >= 4 ? 0xFFFFFFFFu : (rem <= 0 ? 0u : (0xFFFFFFFFu >> (8 * (4 - rem))));
                    q[i][j] &= m;
                }
            }
            if (dst && o < nbytes) __builtin_amdgcn_raw_buffer_store_b128(q[i], rd, (int)o, 0, 0);
            r = crcf_word(r, q[i].x, nib);
            r = crcf_word(r, q[i].y, nib);
            r = crcf_word(r, q[i].z, nib);
            r = crcf_word(r, q[i].w, nib);
        }
        uint32_t v = r ? crcf_mult(kq, r) : 0u;
#pragma unroll
        for (int d = 32; d >= 1; d >>= 1) v ^= __shfl_xor(v, d, 64);
        if ((t & 63) == 0) red[t >> 6] = v;
        __syncthreads();
        if (t == 0) blk[b] = red[0] ^ red[1] ^ red[2] ^ red[3];
        __syncthreads();
    }
}

// blk[0..nblk) (nblk = the stream's 16 KiB blocks, every one taken as full) -> the stream's zlib CRC-32: thread
// t folds `per` consecutive blocks by Horner with Kb = x^(8 16384) (table-driven constant multiplies as
// crc_final2), a 10-level tree joins them; the last block's padding to 16 KiB (p bytes) is undone by x^(-8 16384)
// x^(8 (16384 - p)), and zlib's init by ~0 x^(8 nbytes) -- both powers as lane products of x^(2^k).  The block
// words are zeroed as they are read (the next producer XORs into zeros).
struct CrcfFin {
    uint32_t kc[1 + CF2_L];     // kc[0] = Kb; kc[1 + l] = Kb^(per 2^l)
    uint32_t kinv;              // Kb^-1
    long long per, nbytes;      // (nbytes: when d_nbits is NULL)
};
__global__ __launch_bounds__(CF2_T) void crcf_final_kernel(uint32_t* __restrict__ blk, CrcfFin F,
                                                           const unsigned long long* __restrict__ d_nbits,
                                                           const uint32_t* __restrict__ ctab, uint32_t* __restrict__ out,
                                                           const uint32_t* __restrict__ ref, unsigned* __restrict__ count,
                                                           const uint32_t* __restrict__ gate) {
    if (gate && gate[0] == gate[1]) return;
    __shared__ uint32_t T[1 + CF2_L][4][256];
    __shared__ uint32_t B[1 + CF2_L][32];
    __shared__ uint32_t red[CF2_T];
    const int t = threadIdx.x;
    const long long nbytes = d_nbits ? (long long)((*d_nbits + 7) >> 3) : F.nbytes;
    const long long nblk = crcf_nblk(nbytes);
    if (t < 1 + CF2_L) {
        uint32_t b = F.kc[t];
        B[t][31] = b;
        for (int i = 30; i >= 0; i--) {
            b = (b & 1u) ? (b >> 1) ^ CRC_POLY : b >> 1;
            B[t][i] = b;
        }
    }
    __syncthreads();
    for (int e = t; e < (1 + CF2_L) * 1024; e += CF2_T) {
        const int c = e >> 10, j = (e >> 8) & 3, v = e & 255;
        uint32_t x = 0;
#pragma unroll
        for (int k = 0; k < 8; k++)
            if ((v >> k) & 1) x ^= B[c][8 * j + k];
        T[c][j][v] = x;
    }
    __syncthreads();
    uint32_t r = 0;
    const long long pad = CF2_T * F.per - nblk;                      // leading zero blocks add nothing
    for (long long i = 0; i < F.per; i++) {
        const long long b = (long long)t * F.per + i - pad;
        uint32_t v = 0;
        if (b >= 0 && b < nblk) { v = blk[b]; blk[b] = 0u; }
        r = mul_tab(T[0], r) ^ v;
    }
    red[t] = r;
    __syncthreads();
#pragma unroll
    for (int l = 0; l < CF2_L; l++) {
        const int w = 1 << l;
        uint32_t v = 0;
        const bool act = (t & (2 * w - 1)) == 0;
        if (act) v = mul_tab(T[1 + l], red[t]) ^ red[t + w];
        __syncthreads();
        if (act) red[t] = v;
        __syncthreads();
    }
    if (t < 64) {
        // lanes 0..31: x^(8 m), m = 16384 - p (the last block's bytes); lanes 32..63: x^(8 nbytes)
        const long long p = DC_CRCF_BLK * nblk - nbytes;
        const unsigned long long e = t < 32 ? (unsigned long long)(p ? DC_CRCF_BLK - p : 0) : (unsigned long long)nbytes;
        const int k = t & 31;
        uint32_t f = ((e >> k) & 1ull) ? ctab[CRCF_X2N + k + 3] : CRCF_ONE;
#pragma unroll
        for (int d = 1; d < 32; d <<= 1) {
            const uint32_t o = __shfl_down(f, d, 64);
            if ((k & (2 * d - 1)) == 0) f = crcf_mult(f, o);
        }
        const uint32_t xn = __shfl(f, 32, 64);
        if (t == 0) {
            uint32_t R = red[0];
            if (p) R = crcf_mult(crcf_mult(R, F.kinv), f);
            const uint32_t crc = nbytes > 0 ? ~(R ^ crcf_mult(xn, 0xFFFFFFFFu)) : 0u;
            *out = crc;
            if (ref && count && crc != *ref) atomicAdd(count, 1u);
        }
    }
}

extern "C" int dc_launch_crcf_blocks(const uint8_t* src, uint8_t* dst, long long nbytes, const uint32_t* d_ctab,
                                     uint32_t* blk, const uint32_t* gate, unsigned* gate_count, hipStream_t st) {
    if (nbytes <= 0 || nbytes > 0x7FFFFF00ll - 64) return nbytes == 0 ? 0 : -2;
    const long long nblk = crcf_nblk(nbytes);
    int dev = 0, ncu = 256;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
    const long long g = std::max<long long>(1, std::min<long long>(nblk, 8ll * ncu));
    hipLaunchKernelGGL(crcf_blocks_kernel, dim3((unsigned)g), dim3(256), 0, st, src, dst, nbytes, d_ctab, blk, gate,
                       gate_count);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

extern "C" int dc_launch_crcf_final(uint32_t* blk, long long max_bytes, long long nbytes, const unsigned long long* d_nbits,
                                    const uint32_t* d_ctab, uint32_t* crc_out, const uint32_t* ref, unsigned* count,
                                    const uint32_t* gate, hipStream_t st) {
    static uint32_t kb = 0, kinv = 0;
    if (!kb) {
        kb = h_xpow8n((unsigned long long)DC_CRCF_BLK);
        uint32_t a = kb, r = 0x80000000u;                                   // Kb^(2^32 - 2): the inverse
        unsigned long long e = (1ull << 32) - 2;
        while (e) {
            if (e & 1) r = h_mult(r, a);
            a = h_mult(a, a);
            e >>= 1;
        }
        kinv = r;
    }
    CrcfFin F;
    const long long maxblk = std::max<long long>(1, crcf_nblk(std::max(max_bytes, nbytes)));
    F.per = (maxblk + CF2_T - 1) / CF2_T;
    F.nbytes = nbytes;
    F.kc[0] = kb;
    uint32_t kp = h_xpow8n((unsigned long long)DC_CRCF_BLK * (unsigned long long)F.per);
    for (int l = 0; l < CF2_L; l++) { F.kc[1 + l] = kp; kp = h_mult(kp, kp); }
    F.kinv = kinv;
    hipLaunchKernelGGL(crcf_final_kernel, dim3(1), dim3(CF2_T), 0, st, blk, F, d_nbits, d_ctab, crc_out, ref, count, gate);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

// the DC_CRCF_WORDS table words of dc_device.h's fused CRC (nibble tables, 32-byte shifts, x^(2^k))
extern "C" int dc_crcf_tables(uint32_t* h) {
    uint32_t tab[4][256];
    for (uint32_t i = 0; i < 256; i++) {
        uint32_t c = i;
        for (int k = 0; k < 8; k++) c = (c & 1) ? CRC_POLY ^ (c >> 1) : c >> 1;
        tab[0][i] = c;
    }
    for (int k = 1; k < 4; k++)
        for (int i = 0; i < 256; i++) tab[k][i] = (tab[k - 1][i] >> 8) ^ tab[0][tab[k - 1][i] & 0xFFu];
    for (int t = 0; t < 128; t++) {
        const int j = t >> 4, v = t & 15;
        h[CRCF_NIB + t] = tab[3 - (j >> 1)][(j & 1) ? (v << 4) : v];
    }
    for (int i = 0; i < 512; i++) h[CRCF_KQ + i] = h_xpow8n(32ull * (unsigned long long)i);
    uint32_t p = 1u << 30;                                                   // x^1
    for (int k = 0; k < 40; k++) { h[CRCF_X2N + k] = p; p = h_mult(p, p); }
    return 0;
}

// CT9 receiver check (the MPI_Bcast_bitwise_mask_crc protocol, impl/dataCompression.c:968-1090; the
// pingpong CT9 exchange impl/pingpong.c:363-447) without a host round trip: crc[0] is the sender's CRC-32,
// crc[1] the receiver's.  copy != 0: a mismatch is a damaged receive -- the sender's stream is sent again
// (copied over dst) and counted in count[0]; copy == 0: a mismatch left after the resend counts in count[1].
// Every workgroup reads the two words (written by earlier launches on the stream) and leaves at once when
// they agree.
__global__ __launch_bounds__(256) void crc_resend_kernel(const uint32_t* __restrict__ crc, const uint8_t* __restrict__ src,
                                                         uint8_t* __restrict__ dst, long long nbytes, int copy,
                                                         unsigned* __restrict__ count) {
    if (crc[0] == crc[1]) return;
    if (blockIdx.x == 0 && threadIdx.x == 0) atomicAdd(count + (copy ? 0 : 1), 1u);
    if (!copy) return;
    const long long n16 = nbytes >> 4;
    const uint4* s4 = reinterpret_cast<const uint4*>(src);
    uint4* d4 = reinterpret_cast<uint4*>(dst);
    const long long stride = (long long)gridDim.x * blockDim.x;
    for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += stride) d4[i] = s4[i];
    for (long long i = (n16 << 4) + (long long)blockIdx.x * blockDim.x + threadIdx.x; i < nbytes; i += stride) dst[i] = src[i];
}

extern "C" int dc_launch_crc_resend(const uint32_t* crc, const uint8_t* src, uint8_t* dst, long long nbytes, int copy,
                                    unsigned* count, hipStream_t st) {
    long long g = copy ? (nbytes / 16 + 255) / 256 : 1;
    g = std::max<long long>(1, std::min<long long>(g, 4096));
    hipLaunchKernelGGL(crc_resend_kernel, dim3((unsigned)g), dim3(256), 0, st, crc, src, dst, nbytes, copy, count);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

// ---------------------------------------------------------------- Hamming SECDED
// Hamming position of data bit d (0-based): the (d+1)-th positive integer that is not a power of 2.
__device__ __forceinline__ unsigned long long ham_pos(unsigned long long d) {
    unsigned long long j = d + 1;
    unsigned long long k = 0;                             // powers of two <= j (grows with j)
    while (true) {
        const unsigned long long cand = d + 1 + k;
        const unsigned long long pw = (unsigned long long)(64 - __clzll((long long)cand));   // #powers <= cand
        if (pw == k) { j = cand; break; }
        k = pw;
    }
    return j;
}

__global__ __launch_bounds__(256) void ham_syndrome_kernel(const uint8_t* __restrict__ s, long long nbytes,
                                                           unsigned long long* __restrict__ out_syn,
                                                           unsigned long long* __restrict__ out_ones) {
    __shared__ unsigned long long ssyn[256], sones[256];
    unsigned long long syn = 0, ones = 0;
    for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < nbytes;
         i += (long long)gridDim.x * blockDim.x) {
        const uint32_t byte = s[i];
        if (!byte) continue;
        unsigned long long j = ham_pos((unsigned long long)i * 8);
        for (int b = 0; b < 8; b++) {
            if (b) { j++; if ((j & (j - 1)) == 0) j++; }
            if ((byte >> (7 - b)) & 1u) { syn ^= j; ones++; }
        }
    }
    ssyn[threadIdx.x] = syn; sones[threadIdx.x] = ones;
    __syncthreads();
    for (int w = 128; w > 0; w >>= 1) {
        if ((int)threadIdx.x < w) { ssyn[threadIdx.x] ^= ssyn[threadIdx.x + w]; sones[threadIdx.x] += sones[threadIdx.x + w]; }
        __syncthreads();
    }
    if (threadIdx.x == 0) { atomicXor(out_syn, ssyn[0]); atomicAdd(out_ones, sones[0]); }
}

// ------------------------------------------------------------------------------------------------
extern "C" int dc_launch_to_small(const float* x, long long n, float* y, float* part_v, long long* part_i,
                                  float* d_min, hipStream_t st) {
    if (n <= 0) return 0;
    const int nparts = (int)std::min<long long>(DC_MIN_PARTS, std::max<long long>(1, n / 4096));
    hipLaunchKernelGGL(min_partial_kernel, dim3(nparts), dim3(256), 0, st, x, n, part_v, part_i);
    hipLaunchKernelGGL(min_final_kernel, dim3(1), dim3(256), 0, st, x, part_v, part_i, nparts, d_min, nullptr, 0,
                       nullptr, 0);
    if (y) {
        long long g = (n / 4 + 255) / 256;
        if (g > 2048) g = 2048;
        if (g < 1) g = 1;
        hipLaunchKernelGGL(sub_min_kernel, dim3((unsigned)g), dim3(256), 0, st, x, n, d_min, y);
    }
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

// med_dataset_float's running float sum of x[0..n) continued from s_init, its mean and type, and
// (optional) the raw sum and max; scratch: dc_med_scratch_bytes(n) bytes of device memory
extern "C" int dc_launch_med(const float* x, long long n, float s_init, void* scratch, float* d_mean, int* d_type,
                             float* d_sum, float* d_max, hipStream_t st) {
    return launch_med<float>(x, n, s_init, scratch, d_mean, d_type, d_sum, d_max, 0, st);
}
// fresh = 1: the array was not just run through dc_launch_med (its chunk sums are not in the scratch)
extern "C" int dc_launch_med_wide(const float* x, long long n, float s_init, void* scratch, float* d_mean, int* d_type,
                                  float* d_sum, float* d_max, int fresh, hipStream_t st) {
    return launch_med<float>(x, n, s_init, scratch, d_mean, d_type, d_sum, d_max, fresh ? 2 : 1, st);
}
// a rank's shard (med_shard_kernel): trans = 0 its double sum and max; trans = 1 its whole-shard transducer,
// the chunk windows opened from s_est (the estimated running sum the shard starts at).  The 21-word record
// lives in the scratch's tail; *d_rec points at it.
extern "C" int dc_launch_med_shard(const float* x, long long n, double s_est, int trans, void* scratch,
                                   long long** d_rec, hipStream_t st) {
    if (n <= 0) return -1;
    const long long nch = (n + MC - 1) / MC;
    const MedScratch<float> M = med_scratch<float>(scratch, nch);
    long long* rec = M.rec;
    *d_rec = rec;
    hipLaunchKernelGGL(med_chunk_sum_kernel<float>, dim3((unsigned)nch), dim3(MC_T), 0, st, x, n, M);
    if (trans) {
        const float se = (float)fmin(fmax(s_est, 0.0), 3.0e38);
        hipLaunchKernelGGL(med_chunk_scan_kernel<float>, dim3(1), dim3(1024), 0, st, M, nch, se);
        hipLaunchKernelGGL((med_chunk_trans_kernel<float, MW>), dim3(med_trans_grid(nch)), dim3(256), 0, st, x, n, M, 0);
    }
    hipLaunchKernelGGL(med_shard_kernel<float>, dim3(1), dim3(MX_T), 0, st, x, nch, M, trans, rec);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}
extern "C" int dc_med_shard_binades(void) { return MW; }

// med_dataset_double (:3564-3590): the same on doubles (scratch: dc_med_scratch_bytes64(n))
extern "C" int dc_launch_med64(const double* x, long long n, void* scratch, double* d_mean, int* d_type, int wide,
                               hipStream_t st) {
    return launch_med<double>(x, n, 0.0, scratch, d_mean, d_type, (double*)nullptr, (double*)nullptr, wide, st);
}

extern "C" long long dc_crc_parts(long long nbytes) { return (nbytes + CRC_BLK - 1) / CRC_BLK; }
extern "C" int dc_crc_run_bytes(void) { return CRC_RUN; }

// s2 / d_out2 (or null): a second buffer of the same length CRC-ed in the same two launches (parts after d_parts)
static int launch_crc32(const uint8_t* s, long long nbytes, const uint32_t* d_tab, const uint32_t* d_x2n,
                        uint32_t* d_parts, uint32_t init, uint32_t* d_out, uint8_t* dst, const uint32_t* gate,
                        unsigned* count, hipStream_t st, const uint8_t* s2 = nullptr, uint32_t* d_out2 = nullptr) {
    long long nblk = dc_crc_parts(nbytes);
    uint32_t* parts2 = d_parts + nblk;
    if (nbytes > 0) {                                     // d_tab: 4 slicing tables, then kpow[256]
        static long long gcap = -1;                       // (A/B: DC_CRC_GRID caps the workgroups; 0 = one per block)
        if (gcap < 0) { const char* e = getenv("DC_CRC_GRID"); gcap = e ? atoll(e) : 4096; }
        long long g = (gcap > 0 && nblk > gcap) ? gcap : nblk;
        if (dst)
            hipLaunchKernelGGL(crc_blocks_kernel<true>, dim3((unsigned)g), dim3(256), 0, st, s, nbytes, d_tab,
                               d_tab + 1024, d_x2n, d_parts, dst, gate, count, (const uint8_t*)nullptr, (uint32_t*)nullptr);
        else
            hipLaunchKernelGGL(crc_blocks_kernel<false>, dim3((unsigned)g, s2 ? 2u : 1u), dim3(256), 0, st, s, nbytes, d_tab,
                               d_tab + 1024, d_x2n, d_parts, (uint8_t*)nullptr, (const uint32_t*)nullptr,
                               (unsigned*)nullptr, s2, parts2);
    } else if (gate) {
        return -2;                                        // (the resend of an empty stream: nothing to copy)
    }
    if (DC_CRC_FIN2) {
        CrcFin2 F2;
        F2.nblk = nbytes > 0 ? nblk : 0;
        const long long m2 = F2.nblk > 0 ? F2.nblk - 1 : 0;
        F2.per = m2 > 0 ? (m2 + CF2_T - 1) / CF2_T : 0;
        F2.pad = CF2_T * F2.per - m2;
        F2.kc[0] = h_xpow8n((unsigned long long)CRC_BLK);
        uint32_t kp = h_xpow8n((unsigned long long)CRC_BLK * (unsigned long long)F2.per);
        for (int l = 0; l < CF2_L; l++) { F2.kc[1 + l] = kp; kp = h_mult(kp, kp); }
        F2.kl = h_xpow8n((unsigned long long)(nbytes - m2 * CRC_BLK));
        F2.xn = h_xpow8n((unsigned long long)nbytes);
        hipLaunchKernelGGL(crc_final2_kernel, dim3(s2 ? 2 : 1), dim3(CF2_T), 0, st, d_parts, F2, init, d_out, gate,
                           gate ? gate : (const uint32_t*)nullptr, gate ? count + 1 : (unsigned*)nullptr,
                           (const uint32_t*)parts2, d_out2);
        return hipGetLastError() == hipSuccess ? 0 : -1;
    }
    if (gate || s2) return -2;                            // (the resend and pair forms need the 1024-thread combine)
    CrcFin F;
    F.nblk = nbytes > 0 ? nblk : 0;
    const long long m = F.nblk > 0 ? F.nblk - 1 : 0;
    F.per = m > 0 ? (m + 255) / 256 : 0;
    F.pad = 256 * F.per - m;
    F.kb = h_xpow8n((unsigned long long)CRC_BLK);
    uint32_t kp = h_xpow8n((unsigned long long)CRC_BLK * (unsigned long long)F.per);
    for (int l = 0; l < 8; l++) { F.lvl[l] = kp; kp = h_mult(kp, kp); }
    F.kl = h_xpow8n((unsigned long long)(nbytes - m * CRC_BLK));
    F.xn = h_xpow8n((unsigned long long)nbytes);
    (void)d_x2n;
    hipLaunchKernelGGL(crc_final_kernel, dim3(1), dim3(256), 0, st, d_parts, F, init, d_out);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

extern "C" int dc_launch_crc32(const uint8_t* s, long long nbytes, const uint32_t* d_tab, const uint32_t* d_x2n,
                               uint32_t* d_parts, uint32_t init, uint32_t* d_out, hipStream_t st) {
    return launch_crc32(s, nbytes, d_tab, d_x2n, d_parts, init, d_out, nullptr, nullptr, nullptr, st);
}
// the CT9 checks after dc_encode_send_device: the sender's CRC of a and the receiver's of b (same length) in one
// pass over both (parts: 2 dc_crc_parts(nbytes) words)
extern "C" int dc_launch_crc32_pair(const uint8_t* a, const uint8_t* b, long long nbytes, const uint32_t* d_tab,
                                    const uint32_t* d_x2n, uint32_t* d_parts, uint32_t* d_out_a, uint32_t* d_out_b,
                                    hipStream_t st) {
    if (nbytes <= 0) return -2;
    return launch_crc32(a, nbytes, d_tab, d_x2n, d_parts, 0u, d_out_a, nullptr, nullptr, nullptr, st, b, d_out_b);
}
// the CT9 send: src copied to dst (the channel) and the CRC of what is sent into *d_out, one pass
extern "C" int dc_launch_crc32_copy(const uint8_t* src, uint8_t* dst, long long nbytes, const uint32_t* d_tab,
                                    const uint32_t* d_x2n, uint32_t* d_parts, uint32_t* d_out, hipStream_t st) {
    return launch_crc32(src, nbytes, d_tab, d_x2n, d_parts, 0u, d_out, dst, nullptr, nullptr, st);
}
// the CT9 resend in one pass: if crc2[0] != crc2[1] (sender's vs receiver's CRC), copy src -> dst computing the
// copy's CRC into crc2[1], count the resend in count[0] and a copy whose CRC still differs in count[1]
extern "C" int dc_launch_crc32_resend(const uint8_t* src, uint8_t* dst, long long nbytes, const uint32_t* d_tab,
                                      const uint32_t* d_x2n, uint32_t* d_parts, uint32_t* crc2, unsigned* count,
                                      hipStream_t st) {
    return launch_crc32(src, nbytes, d_tab, d_x2n, d_parts, 0u, crc2 + 1, dst, crc2, count, st);
}

// Shard stream: bits [start_bit, start_bit + 8*nout) of s as nout bytes starting at bit 0 (MSB first),
// so a shard of a global stream decodes like a stream of its own (dc_decode_shard_device).
__global__ __launch_bounds__(256) void bit_shift_copy_kernel(const uint8_t* __restrict__ s, long long sbytes,
                                                             unsigned long long start_bit, unsigned long long nbits,
                                                             uint8_t* __restrict__ d, long long nout) {
    const long long b0 = (long long)(start_bit >> 3);
    const int sh = (int)(start_bit & 7);
    for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < nout; i += (long long)gridDim.x * 256) {
        const long long a = b0 + i;
        const uint32_t hi = a < sbytes ? s[a] : 0u, lo = a + 1 < sbytes ? s[a + 1] : 0u;
        uint32_t v = (((hi << 8 | lo) << sh) >> 8) & 0xFFu;
        const long long rem = (long long)nbits - 8 * i;                  // bits after the shard are zero
        if (rem <= 0) v = 0;
        else if (rem < 8) v &= (0xFFu << (8 - rem)) & 0xFFu;
        d[i] = (uint8_t)v;
    }
}

extern "C" int dc_launch_bit_shift_copy(const uint8_t* s, long long sbytes, unsigned long long start_bit,
                                        unsigned long long nbits, uint8_t* d, long long nout, hipStream_t st) {
    if (nout <= 0) return 0;
    long long g = (nout + 255) / 256;
    if (g > 8192) g = 8192;
    hipLaunchKernelGGL(bit_shift_copy_kernel, dim3((unsigned)g), dim3(256), 0, st, s, sbytes, start_bit, nbits, d, nout);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

// The multi-GPU all-gather's product: world shard streams, each encoded
// at start bit 0 and all-gathered into slots of P bytes (g[r * P ..]), with their bit counts counts[r]
// (device), become the single global stream: shard r's bits land at the exclusive sum of the counts
// before it, shifted across byte boundaries, the words two shards share OR-ed.  Every workgroup scans
// the counts itself (no scan launch, no host read); thread = one 32-bit output word, MSB-first (stored
// byte-swapped: the stream's bytes in order).  err |= 1: a shard longer than its slot (P < bytes + 8);
// 2: the global stream longer than the output (nothing is written then).
constexpr int MERGE_MAXW = 1024;
__device__ __forceinline__ uint32_t be_word(const uint8_t* p, long long i) {
    return __builtin_bswap32(reinterpret_cast<const uint32_t*>(p)[i]);
}
__global__ __launch_bounds__(256) void merge_shards_kernel(const uint8_t* __restrict__ g, long long P, int world,
                                                           const unsigned long long* __restrict__ counts,
                                                           uint32_t* __restrict__ out, long long out_bytes,
                                                           unsigned long long* __restrict__ total_out,
                                                           unsigned* __restrict__ err) {
    __shared__ unsigned long long st[MERGE_MAXW + 1];
    __shared__ int bad;
    if (threadIdx.x == 0) {
        unsigned long long acc = 0;
        int b = 0;
        for (int r = 0; r < world; r++) {
            st[r] = acc;
            acc += counts[r];
            if ((long long)((counts[r] + 7) / 8) + 8 > P) b |= 1;
        }
        st[world] = acc;
        if ((long long)((acc + 31) / 32) * 4 > out_bytes) b |= 2;
        bad = b;
        if (blockIdx.x == 0) {
            *total_out = acc;
            if (b) atomicOr(err, (unsigned)b);
        }
    }
    __syncthreads();
    if (bad) return;
    const unsigned long long total = st[world];
    const long long nw = (long long)((total + 31) / 32);
    for (long long w = (long long)blockIdx.x * 256 + threadIdx.x; w < nw; w += (long long)gridDim.x * 256) {
        const long long lo = 32 * w;
        int r0 = 0, r1 = world - 1;                 // the last shard starting at or before bit lo
        while (r0 < r1) {
            const int m = (r0 + r1 + 1) >> 1;
            if ((long long)st[m] <= lo) r0 = m;
            else r1 = m - 1;
        }
        uint32_t acc = 0;
        for (int r = r0; r < world && (long long)st[r] < lo + 32; r++) {
            const long long cnt = (long long)counts[r];
            if (cnt == 0) continue;
            const long long o = lo - (long long)st[r];                    // shard bit at the word's first bit
            const uint8_t* b = g + (long long)r * P;
            uint32_t v, keep;
            if (o >= 0) {
                if (o >= cnt) continue;
                const long long i = o >> 5;
                const int sh = (int)(o & 31);
                v = sh ? __builtin_amdgcn_alignbit(be_word(b, i), be_word(b, i + 1), 32 - sh) : be_word(b, i);
                const long long nv = min(cnt - o, 32ll);                  // valid bits from the word's top
                keep = nv >= 32 ? 0xFFFFFFFFu : ~(0xFFFFFFFFu >> nv);
            } else {
                const int sh = (int)(-o);                                  // the shard starts at bit sh
                v = be_word(b, 0) >> sh;
                const long long nv = min(cnt, (long long)(32 - sh));
                keep = (0xFFFFFFFFu >> sh) & ~(nv + sh >= 32 ? 0u : 0xFFFFFFFFu >> (nv + sh));
            }
            acc |= v & keep;
        }
        out[w] = __builtin_bswap32(acc);
    }
}

extern "C" int dc_launch_merge_shards(const uint8_t* g, long long P, int world, const unsigned long long* counts,
                                      uint8_t* out, long long out_bytes, unsigned long long* total_out, unsigned* err,
                                      long long max_bytes, hipStream_t st) {
    if (world < 1 || world > MERGE_MAXW || (P & 3) || ((uintptr_t)g & 3) || ((uintptr_t)out & 3)) return -2;
    long long grid = (max_bytes / 4 + 255) / 256 + 1;
    if (grid > 8192) grid = 8192;
    hipLaunchKernelGGL(merge_shards_kernel, dim3((unsigned)grid), dim3(256), 0, st, g, P, world, counts,
                       reinterpret_cast<uint32_t*>(out), out_bytes, total_out, err);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

// The receiver's side of the all-gather: shard `rank` cut out of the merged global stream (the bytes that
// arrived, not the rank's own encode) to bit 0 of d, its bit count to *nbits_out -- what
// dc_decode_shard3_device then decodes.  Every workgroup scans the counts itself (no host read); thread =
// one 32-bit output word, v_alignbit of the two global words it spans, the bits past the shard cleared.
// err |= 4: the shard does not fit d or lies outside the global buffer (nothing written then).
__global__ __launch_bounds__(256) void extract_shard_kernel(const uint32_t* __restrict__ g, long long g_bytes,
                                                            const unsigned long long* __restrict__ counts, int rank,
                                                            uint32_t* __restrict__ d, long long d_bytes,
                                                            unsigned long long* __restrict__ nbits_out,
                                                            unsigned* __restrict__ err) {
    __shared__ unsigned long long s_start, s_cnt;
    __shared__ int bad;
    if (threadIdx.x == 0) {
        unsigned long long acc = 0;
        for (int r = 0; r < rank; r++) acc += counts[r];
        const unsigned long long cnt = counts[rank];
        s_start = acc;
        s_cnt = cnt;
        const int b = ((long long)((cnt + 31) / 32) * 4 > d_bytes || (long long)((acc + cnt + 31) / 32) * 4 > g_bytes) ? 4 : 0;
        bad = b;
        if (blockIdx.x == 0) {
            *nbits_out = b ? 0ull : cnt;
            if (b) atomicOr(err, (unsigned)b);
        }
    }
    __syncthreads();
    if (bad) return;
    const unsigned long long S = s_start, cnt = s_cnt;
    const long long nw = (long long)((cnt + 31) / 32), gw = g_bytes / 4;
    const int sh = (int)(S & 31ull);
    for (long long w = (long long)blockIdx.x * 256 + threadIdx.x; w < nw; w += (long long)gridDim.x * 256) {
        const long long i = (long long)(S >> 5) + w;
        const uint32_t a = __builtin_bswap32(g[i]);
        const uint32_t b = i + 1 < gw ? __builtin_bswap32(g[i + 1]) : 0u;
        uint32_t v = sh ? __builtin_amdgcn_alignbit(a, b, 32 - sh) : a;
        const long long left = (long long)cnt - 32 * w;                   // shard bits from this word's top
        if (left < 32) v &= ~(0xFFFFFFFFu >> left);
        d[w] = __builtin_bswap32(v);
    }
}

extern "C" int dc_launch_extract_shard(const uint8_t* g, long long g_bytes, const unsigned long long* counts, int rank,
                                       uint8_t* d, long long d_bytes, unsigned long long* nbits_out, unsigned* err,
                                       hipStream_t st) {
    if (rank < 0 || ((uintptr_t)g & 3) || ((uintptr_t)d & 3)) return -2;
    long long grid = (d_bytes / 4 + 255) / 256 + 1;
    if (grid > 8192) grid = 8192;
    hipLaunchKernelGGL(extract_shard_kernel, dim3((unsigned)grid), dim3(256), 0, st, reinterpret_cast<const uint32_t*>(g),
                       g_bytes, counts, rank, reinterpret_cast<uint32_t*>(d), d_bytes, nbits_out, err);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

// Co-residency tests (dc_occupy_device): `blocks` workgroups of 256 threads, `lds` bytes of LDS each, that stay
// resident for `ticks` of s_memrealtime (every wave leaves by then) -- a neighbour occupying CU slots while the
// codec runs on another stream
__global__ __launch_bounds__(256) void occupy_kernel(unsigned long long ticks, unsigned* __restrict__ sink) {
    extern __shared__ uint32_t occ_lds[];
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    unsigned acc = threadIdx.x;
    while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) {
        acc = acc * 1664525u + 1013904223u;
        __builtin_amdgcn_s_sleep(8);
    }
    if (acc == 0x9E3779B9u) { occ_lds[0] = acc; sink[0] = occ_lds[threadIdx.x & 7]; }
}
extern "C" int dc_launch_occupy(double us, int blocks, int lds, unsigned* sink, hipStream_t st) {
    if (blocks < 1 || us < 0.0 || us > 1.0e6 || lds < 0 || lds > 160 * 1024) return -2;
    hipLaunchKernelGGL(occupy_kernel, dim3((unsigned)blocks), dim3(256), (size_t)lds, st,
                       (unsigned long long)(us * 100.0), sink);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

// Himeno halo planes: the plane ijk = 1/2/3 at index v of a [mi][mj][mk] float array in
// the order of transform_3d_array_to_1d_array (impl/dataCompression.c:3741-3775), gathered into a
// contiguous array; and the decoded plane + min scattered back (impl/himenoBMTxps.c:699-706).  (plane_index:
// dc_device.h, shared with the small-stream decoder's scatter mode)
__global__ __launch_bounds__(256) void plane_gather_kernel(const float* __restrict__ p, int mj, int mk, int ijk, int v,
                                                           int A, int B, float* __restrict__ out) {
    const long long n = (long long)A * B;
    for (long long e = (long long)blockIdx.x * 256 + threadIdx.x; e < n; e += (long long)gridDim.x * 256)
        out[e] = p[plane_index(e / B, e % B, ijk, v, mj, mk)];
}
// (r06) the gather with toSmallDataset's minimum partials of the gathered plane (min_partial_kernel's rule: the
// minimum of out[1..n), NaN ignored, and the index of its first zero) -- the halo encode then needs min_final and
// the encoder, which subtracts the minimum while loading (Params.subp): three launches instead of six
// (cnt != nullptr: the last workgroup to finish -- a counter it resets -- takes the minimum itself, min_final_kernel's
// launch folded in: the other workgroups' partials and gathered floats are released by an agent-scope fence before
// their count, which the last one acquires)
__global__ __launch_bounds__(256) void plane_gather_min_kernel(const float* __restrict__ p, int mj, int mk, int ijk, int v,
                                                               int A, int B, float* __restrict__ out,
                                                               float* __restrict__ pv, long long* __restrict__ pi,
                                                               unsigned* __restrict__ cnt, float* __restrict__ out_min,
                                                               uint64_t* __restrict__ clr64, int n64,
                                                               uint32_t* __restrict__ clr32, int n32) {
    __shared__ int last;
    __shared__ float sv[4];
    __shared__ long long si[4];
    const long long n = (long long)A * B;
    float mv = __int_as_float(0x7fc00000);
    long long fz = (long long)1 << 62;
    for (long long e = (long long)blockIdx.x * 256 + threadIdx.x; e < n; e += (long long)gridDim.x * 256) {
        const float a = p[plane_index(e / B, e % B, ijk, v, mj, mk)];
        out[e] = a;
        if (e > 0) {
            mv = fminf(mv, a);
            if (a == 0.f) fz = min(fz, e);
        }
    }
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) {
        mv = fminf(mv, __shfl_xor(mv, d, 64));
        fz = min(fz, (long long)__shfl_xor(fz, d, 64));
    }
    if ((threadIdx.x & 63) == 0) { sv[threadIdx.x >> 6] = mv; si[threadIdx.x >> 6] = fz; }
    __syncthreads();
    if (threadIdx.x == 0) {
        pv[blockIdx.x] = fminf(fminf(sv[0], sv[1]), fminf(sv[2], sv[3]));
        pi[blockIdx.x] = min(min(si[0], si[1]), min(si[2], si[3]));
    }
    if (!cnt) return;
    if (threadIdx.x == 0) {
        __threadfence();                                    // (release this workgroup's floats and partial)
        last = atomicAdd(cnt, 1u) == gridDim.x - 1;
    }
    __syncthreads();
    if (!last) return;
    __threadfence();                                        // (acquire the others')
    if (threadIdx.x == 0) __hip_atomic_store(cnt, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    min_final_body(out, pv, pi, (int)gridDim.x, out_min, clr64, n64, clr32, n32);
}

__global__ __launch_bounds__(256) void plane_scatter_kernel(const float* __restrict__ x, const float* __restrict__ d_min,
                                                            float* __restrict__ p, int mj, int mk, int ijk, int v, int A,
                                                            int B) {
    const long long n = (long long)A * B;
    const float mn = *d_min;
    for (long long e = (long long)blockIdx.x * 256 + threadIdx.x; e < n; e += (long long)gridDim.x * 256)
        p[plane_index(e / B, e % B, ijk, v, mj, mk)] = __fadd_rn(x[e], mn);
}
extern "C" int dc_launch_plane_gather(const float* p, int mj, int mk, int ijk, int v, int A, int B, float* out,
                                      hipStream_t st) {
    const long long n = (long long)A * B;
    if (n <= 0) return 0;
    long long g = (n + 255) / 256;
    if (g > 4096) g = 4096;
    hipLaunchKernelGGL(plane_gather_kernel, dim3((unsigned)g), dim3(256), 0, st, p, mj, mk, ijk, v, A, B, out);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}
// the gathered plane and its minimum into d_min (toSmallDataset_float's minimum of the plane): one launch with a
// zeroed counter cnt (the gather's last workgroup finishes the minimum), else two
extern "C" int dc_launch_plane_gather_min(const float* p, int mj, int mk, int ijk, int v, int A, int B, float* out,
                                          float* part_v, long long* part_i, float* d_min, uint64_t* clr64, int n64,
                                          uint32_t* clr32, int n32, unsigned* cnt, hipStream_t st) {
    const long long n = (long long)A * B;
    if (n <= 0) return 0;
    const int g = (int)std::min<long long>(DC_MIN_PARTS, std::max<long long>(1, (n + 1023) / 1024));
    hipLaunchKernelGGL(plane_gather_min_kernel, dim3((unsigned)g), dim3(256), 0, st, p, mj, mk, ijk, v, A, B, out,
                       part_v, part_i, cnt, d_min, clr64, n64, clr32, n32);
    if (!cnt)
        hipLaunchKernelGGL(min_final_kernel, dim3(1), dim3(256), 0, st, (const float*)out, (const float*)part_v,
                           (const long long*)part_i, g, d_min, clr64, n64, clr32, n32);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}
// y = x - *d_min (the reference's x86 subtraction)
extern "C" int dc_launch_sub_ptr(const float* x, long long n, const float* d_min, float* y, hipStream_t st) {
    if (n <= 0) return 0;
    long long g = (n / 4 + 255) / 256;
    g = std::max(1ll, std::min(g, 2048ll));
    hipLaunchKernelGGL(sub_min_kernel, dim3((unsigned)g), dim3(256), 0, st, x, n, d_min, y);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}
extern "C" int dc_launch_plane_scatter(const float* x, const float* d_min, float* p, int mj, int mk, int ijk, int v,
                                       int A, int B, hipStream_t st) {
    const long long n = (long long)A * B;
    if (n <= 0) return 0;
    long long g = (n + 255) / 256;
    if (g > 4096) g = 4096;
    hipLaunchKernelGGL(plane_scatter_kernel, dim3((unsigned)g), dim3(256), 0, st, x, d_min, p, mj, mk, ijk, v, A, B);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

// BER fault injection for the CT8/CT9 flow: flip `count` stream bits at the
// positions splitmix64(seed + i) mod nbits, MSB-first within each byte like bit_flip (:5858-5865).
// The reference's own pingpong CT9 path only *simulates* a CRC failure (impl/pingpong.c:421-430);
// this flips real bits so the receiver's CRC check has something to detect.
__device__ __forceinline__ unsigned long long splitmix64(unsigned long long z) {
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
__global__ __launch_bounds__(256) void flip_bits_kernel(uint8_t* s, unsigned long long nbits, long long count,
                                                        unsigned long long seed) {
    const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
    if (i >= count || nbits == 0) return;
    const unsigned long long p = splitmix64(seed + (unsigned long long)i) % nbits;
    const unsigned long long byte = p >> 3;
    uint32_t* w = reinterpret_cast<uint32_t*>(s + (byte & ~3ull));
    atomicXor(w, (uint32_t)(0x80u >> (p & 7)) << (8 * (byte & 3)));
}

extern "C" int dc_launch_flip_bits(uint8_t* s, unsigned long long nbits, long long count, unsigned long long seed,
                                   hipStream_t st) {
    if (count <= 0) return 0;
    hipLaunchKernelGGL(flip_bits_kernel, dim3((unsigned)((count + 255) / 256)), dim3(256), 0, st, s, nbits, count, seed);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

extern "C" int dc_launch_ham_syndrome(const uint8_t* s, long long nbytes, unsigned long long* d_syn_ones,
                                      hipStream_t st) {
    (void)hipMemsetAsync(d_syn_ones, 0, 16, st);
    long long g = (nbytes + 255) / 256;
    if (g > 1024) g = 1024;
    if (g < 1) g = 1;
    hipLaunchKernelGGL(ham_syndrome_kernel, dim3((unsigned)g), dim3(256), 0, st, s, nbytes, d_syn_ones, d_syn_ones + 1);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

// ------------------------------------------------------------------------------------------------
// bench.py's self-check: an order-dependent hash of a byte buffer, sum over its 32-bit words (little-endian,
// bytes past nbytes zero) of splitmix64(i << 32 | w_i) mod 2^64 -- additive, so any grid computes it, and
// tests/golden/make_bench_hashes.py computes the same over the oracle's streams and decodes.
__global__ __launch_bounds__(256) void hash_words_kernel(const uint32_t* __restrict__ p, long long nbytes,
                                                         unsigned long long* __restrict__ out) {
    const long long nw = (nbytes + 3) >> 2;
    unsigned long long h = 0;
    for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < nw; i += (long long)gridDim.x * 256) {
        uint32_t w = p[i];
        const long long rem = nbytes - 4 * i;
        if (rem < 4) w &= (1u << (8 * rem)) - 1u;
        h += splitmix64(((unsigned long long)i << 32) | w);
    }
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) h += __shfl_xor(h, d, 64);
    if ((threadIdx.x & 63) == 0 && h) atomicAdd(out, h);
}
extern "C" int dc_launch_hash_words(const void* p, long long nbytes, unsigned long long* d_out, hipStream_t st) {
    (void)hipMemsetAsync(d_out, 0, 8, st);
    if (nbytes <= 0) return hipGetLastError() == hipSuccess ? 0 : -1;
    long long g = ((nbytes + 3) / 4 + 255) / 256;
    if (g > 4096) g = 4096;
    hipLaunchKernelGGL(hash_words_kernel, dim3((unsigned)g), dim3(256), 0, st, (const uint32_t*)p, nbytes, d_out);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

// bench.py's achievable HBM rate: a streaming copy, U 16-byte buffer loads per lane in flight before their
// stores (the guide's float4 copy reaches 6.29 TB/s), every workgroup a contiguous run of 256 U x 16 B per
// round; NT: both streams past the caches.  Bytes beyond the last whole 16-byte group are not copied.
template <int U, bool NT>
__global__ __launch_bounds__(256) void stream_copy_kernel(const uint8_t* __restrict__ src, uint8_t* __restrict__ dst,
                                                          long long n16) {
    typedef unsigned v4u __attribute__((ext_vector_type(4)));
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(src), (short)0, 0x7FFFFFFF, 0x00020000);
    const __amdgpu_buffer_rsrc_t rd = __builtin_amdgcn_make_buffer_rsrc(dst, (short)0, 0x7FFFFFFF, 0x00020000);
    const long long per = 256ll * U;
    for (long long b = (long long)blockIdx.x * per; b < n16; b += (long long)gridDim.x * per) {
        // (buffers up to 2 GiB: the bench copies at most 1 GiB)
        v4u v[U];
#pragma unroll
        for (int u = 0; u < U; u++) {
            const long long i = b + 256 * u + threadIdx.x;
            v[u] = __builtin_amdgcn_raw_buffer_load_b128(rs, i < n16 ? (int)(16 * i) : 0x7FFFFFF0, 0, NT ? 2 : 0);
        }
#pragma unroll
        for (int u = 0; u < U; u++) {
            const long long i = b + 256 * u + threadIdx.x;
            __builtin_amdgcn_raw_buffer_store_b128(v[u], rd, i < n16 ? (int)(16 * i) : 0x7FFFFFF0, 0, NT ? 2 : 0);
        }
    }
}
// variant 0..3: (U, NT) = (4, no), (4, yes), (8, no), (8, yes); grid = 8 workgroups per CU
extern "C" int dc_launch_stream_copy(const void* src, void* dst, long long bytes, int variant, hipStream_t st) {
    const long long n16 = bytes / 16;
    if (n16 <= 0 || bytes > 0x7FFFFF00ll) return -2;
    int dev = 0, ncu = 256;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
    const dim3 g((unsigned)(8 * ncu)), b(256);
    const uint8_t* s = (const uint8_t*)src;
    uint8_t* d = (uint8_t*)dst;
    switch (variant) {
        case 0: hipLaunchKernelGGL(HIP_KERNEL_NAME(stream_copy_kernel<4, false>), g, b, 0, st, s, d, n16); break;
        case 1: hipLaunchKernelGGL(HIP_KERNEL_NAME(stream_copy_kernel<4, true>), g, b, 0, st, s, d, n16); break;
        case 2: hipLaunchKernelGGL(HIP_KERNEL_NAME(stream_copy_kernel<8, false>), g, b, 0, st, s, d, n16); break;
        case 3: hipLaunchKernelGGL(HIP_KERNEL_NAME(stream_copy_kernel<8, true>), g, b, 0, st, s, d, n16); break;
        default: return -2;
    }
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

// ------------------------------------------------------------------------------------------------
// Per-kernel timing hooks (bench.py's roofline): when enabled, the launchers record HIP events on
// their stream between kernels; event set s holds marks 0..3 (encode: start, after count, -, after pack)
// and 4..7 (decode: start, after parse, after tile fix + scan (chunk-map decoder only), after decode).  dc_decode_finish's slow
// paths record into the set of the step that queued the decode: the chunk-map decoder's marks 4..7 go
// to 8..11, and 12..15 bracket the runs-mode resolve and the resolved decode.
constexpr int DC_MARKS = 16;
static hipEvent_t* g_events = nullptr;
static int g_nsets = 0, g_set = 0, g_finish = 0;
static unsigned char* g_rec = nullptr;         // [set * DC_MARKS + mark] recorded in this session

extern "C" void dc_timing_finish(int on) { g_finish = on; }
extern "C" void dc_mark_phase(int k, hipStream_t st) {
    if (!g_events) return;
    int set = g_set;
    if (g_finish) {
        if (g_set == 0) return;
        set = g_set - 1;
        if (k >= 4 && k < 8) k += 4;
    } else if (k >= 8) {
        return;
    }
    if (set >= g_nsets) return;
    if (hipEventRecord(g_events[set * DC_MARKS + k], st) == hipSuccess) g_rec[set * DC_MARKS + k] = 1;
}
extern "C" void dc_mark_next_set(void) {
    if (g_events && !g_finish && g_set < g_nsets) g_set++;
}
extern "C" int dc_timing_enable(int nsets) {
    if (g_events) {
        for (int i = 0; i < g_nsets * DC_MARKS; i++) (void)hipEventDestroy(g_events[i]);
        free(g_events);
        free(g_rec);
        g_events = nullptr;
        g_rec = nullptr;
    }
    g_nsets = 0;
    g_set = 0;
    if (nsets <= 0) return 0;
    g_events = (hipEvent_t*)calloc((size_t)nsets * DC_MARKS, sizeof(hipEvent_t));
    g_rec = (unsigned char*)calloc((size_t)nsets * DC_MARKS, 1);
    if (!g_events || !g_rec) return -1;
    for (int i = 0; i < nsets * DC_MARKS; i++)
        if (hipEventCreate(&g_events[i]) != hipSuccess) return -1;
    g_nsets = nsets;
    return 0;
}
// elapsed ms between two marks of a set; 0 when either was not recorded (that launch did not run)
static int mark_ms(int set, int a, int b, float* ms) {
    hipEvent_t* e = g_events + set * DC_MARKS;
    *ms = 0.0f;
    if (!g_rec[set * DC_MARKS + a] || !g_rec[set * DC_MARKS + b]) return 1;
    if (hipEventSynchronize(e[b]) != hipSuccess) { (void)hipGetLastError(); return -1; }
    if (hipEventElapsedTime(ms, e[a], e[b]) != hipSuccess) { *ms = -1.0f; (void)hipGetLastError(); }
    return 0;
}
/* ms[0..5] = encode count, (empty: the scan runs in the pack kernel's workgroup 0), encode pack, decode parse,
 * decode tile fix + scan (chunk-map decoder; empty for the segment decoder), decode */
extern "C" int dc_timing_read(int set, float* ms) {
    if (!g_events || set < 0 || set >= g_nsets) return -1;
    const int a[6] = {0, 1, 2, 4, 5, 6};
    for (int i = 0; i < 6; i++) {
        int b = a[i];
        // a launcher that records no mark between two kernels (encoder: 2, segment decoder: 6): the second
        // kernel's slot starts at the first one's end mark, the empty slot stays 0
        if ((i == 2 || i == 5) && !g_rec[set * DC_MARKS + b]) b -= 1;
        else if ((i == 1 || i == 4) && !g_rec[set * DC_MARKS + b + 1]) { ms[i] = 0.0f; continue; }
        if (mark_ms(set, b, a[i] + 1, &ms[i]) < 0) return -1;
    }
    return 0;
}
/* ms[0..5] as dc_timing_read; ms[6..8] the chunk-map decoder's parse, tile fix + scan and decode run by
 * dc_decode_finish; ms[9] the runs-mode resolve, ms[10] the resolved decode (0: not run) */
extern "C" int dc_timing_read_all(int set, float* ms) {
    if (dc_timing_read(set, ms)) return -1;
    const int a[5] = {8, 9, 10, 12, 14};
    for (int i = 0; i < 5; i++)
        if (mark_ms(set, a[i], a[i] + 1, &ms[6 + i]) < 0) return -1;
    return 0;
}

}  // namespace dc
