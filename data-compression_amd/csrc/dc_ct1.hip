// dc_ct1.hip -- CT1 byte-wise codec on gfx950: myCompress (impl/dataCompression.c:3980-4118) and
// myDecompress (:3943-3977), and their double twins myCompress_double (:3815) / myDecompress_double (:3778)
// (the kernels are templated on the element type).
//
// Encoder: every element n >= 4 is predicted from the ORIGINAL x[n-1..n-4] by four float predictors
// (p1 = b1, p2 = 2b1-b2, p3 = 3b1-3b2+b3, p4 = 4b1-6b2+4b3-b4, each op rounded, strict < picks the
// earliest minimum); if the minimum |p - x| <= absErrorBound the element becomes the code 'a'..'d'
// with its 1-based position, otherwise the float itself goes to the raw array.  Codes are a pure
// function of the input, so the encoder is a stream compaction: count raws per tile, scan, write.
//
// Decoder: codes are scattered to their positions, raw floats fill the other positions in order (scan
// of the raw flags), then code values are rebuilt from the DECODED history.  A code needs at most the
// four values before it, so a code preceded by four raw values starts an independent "cluster" that
// one thread decodes sequentially until four raws follow the last code again.
#include "dc_device.h"
#include <algorithm>

namespace dc {

// round-to-nearest arithmetic for both element types (no FMA contraction, as the x86 reference)
__device__ __forceinline__ float rmul(float a, float b) { return __fmul_rn(a, b); }
__device__ __forceinline__ float rsub(float a, float b) { return __fsub_rn(a, b); }
__device__ __forceinline__ float radd(float a, float b) { return __fadd_rn(a, b); }
__device__ __forceinline__ double rmul(double a, double b) { return __dmul_rn(a, b); }
__device__ __forceinline__ double rsub(double a, double b) { return __dsub_rn(a, b); }
__device__ __forceinline__ double radd(double a, double b) { return __dadd_rn(a, b); }

constexpr int C1_TPB = 256;
constexpr int C1_K = 16;                         // consecutive elements per lane
constexpr int C1_TILE = C1_TPB * C1_K;

// code of element with value x and original history b1..b4 (0 = raw, 'a'..'d')
template <typename T>
__device__ __forceinline__ uint8_t ct1_code(T x, T b1, T b2, T b3, T b4, T thr_le) {
    const T p1 = b1;
    const T p2 = rsub(rmul(T(2), b1), b2);
    const T p3 = radd(rsub(rmul(T(3), b1), rmul(T(3), b2)), b3);
    const T p4 = rsub(radd(rsub(rmul(T(4), b1), rmul(T(6), b2)), rmul(T(4), b3)), b4);
    const T d1 = fabs(rsub(p1, x)), d2 = fabs(rsub(p2, x));
    const T d3 = fabs(rsub(p3, x)), d4 = fabs(rsub(p4, x));
    T dmin = d1;
    uint8_t t = 'a';
    if (d2 < dmin) { dmin = d2; t = 'b'; }
    if (d3 < dmin) { dmin = d3; t = 'c'; }
    if (d4 < dmin) { dmin = d4; t = 'd'; }
    return dmin <= thr_le ? t : 0;
}

template <typename T>
__device__ __forceinline__ void ct1_load(const T* __restrict__ x, long long n, long long base, T* v) {
#pragma unroll
    for (int j = 0; j < C1_K + 4; j++) {
        const long long e = base + j - 4;
        v[j] = (e >= 0 && e < n) ? x[e] : T(0);
    }
}

template <typename T>
__global__ __launch_bounds__(C1_TPB) void ct1_count_kernel(const T* __restrict__ x, long long n, T thr_le,
                                                           uint32_t* __restrict__ traw, unsigned* __restrict__ err) {
    __shared__ uint32_t s[C1_TPB / 64];
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const long long base = (long long)blockIdx.x * C1_TILE + (long long)tid * C1_K;
    T v[C1_K + 4];
    ct1_load<T>(x, n, base, v);
    uint32_t raw = 0;
    bool neg1 = false;
#pragma unroll
    for (int j = 0; j < C1_K; j++) {
        const long long e = base + j;
        if (e < n) {
            const uint8_t c = e < 4 ? 0 : ct1_code<T>(v[4 + j], v[3 + j], v[2 + j], v[1 + j], v[j], thr_le);
            raw += c == 0;
            neg1 |= v[4 + j] == T(-1);
        }
    }
    if (__any(neg1) && lane == 0) atomicOr(err, 1u);                // T(-1) is the reference's sentinel
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) raw += __shfl_xor(raw, d, 64);
    if (lane == 0) s[wid] = raw;
    __syncthreads();
    if (tid == 0) traw[blockIdx.x] = s[0] + s[1] + s[2] + s[3];
}

// exclusive scan of per-tile counts (one workgroup); out[t] = sum of cnt[0..t), out[ntiles] = total
__global__ __launch_bounds__(1024) void ct1_scan_kernel(const uint32_t* __restrict__ cnt, unsigned long long* __restrict__ out,
                                                        long long ntiles) {
    __shared__ unsigned long long part[1024];
    const int tid = threadIdx.x;
    const long long per = (ntiles + 1023) / 1024;
    const long long t0 = tid * per, t1 = min(ntiles, t0 + per);
    unsigned long long sum = 0;
    for (long long t = t0; t < t1; t++) sum += cnt[t];
    part[tid] = sum;
    __syncthreads();
    for (int d = 1; d < 1024; d <<= 1) {
        const unsigned long long v = tid >= d ? part[tid - d] : 0ull;
        __syncthreads();
        part[tid] += v;
        __syncthreads();
    }
    unsigned long long run = part[tid] - sum;
    for (long long t = t0; t < t1; t++) {
        out[t] = run;
        run += cnt[t];
    }
    if (tid == 1023) out[ntiles] = part[1023];
}

template <typename T>
__global__ __launch_bounds__(C1_TPB) void ct1_write_kernel(const T* __restrict__ x, long long n, T thr_le,
                                                           const unsigned long long* __restrict__ rawoff,
                                                           T* __restrict__ raw, char* __restrict__ codes,
                                                           int* __restrict__ pos1) {
    __shared__ uint32_t s[C1_TPB / 64];
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const long long tbase = (long long)blockIdx.x * C1_TILE;
    const long long base = tbase + (long long)tid * C1_K;
    T v[C1_K + 4];
    ct1_load<T>(x, n, base, v);
    uint8_t c[C1_K];
    uint32_t nr = 0, nv = 0;
#pragma unroll
    for (int j = 0; j < C1_K; j++) {
        const long long e = base + j;
        c[j] = (e < 4 || e >= n) ? 0 : ct1_code<T>(v[4 + j], v[3 + j], v[2 + j], v[1 + j], v[j], thr_le);
        nv += e < n;
        nr += (e < n && c[j] == 0);
    }
    uint32_t inc = nr;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t t = __shfl_up(inc, d, 64);
        if (lane >= d) inc += t;
    }
    if (lane == 63) s[wid] = inc;
    __syncthreads();
    uint32_t wpre = 0;
    for (int w = 0; w < wid; w++) wpre += s[w];
    unsigned long long r = rawoff[blockIdx.x] + wpre + inc - nr;         // raw index of the lane's first raw
    unsigned long long k = (unsigned long long)base - r;                   // code index (elements before - raws)
#pragma unroll
    for (int j = 0; j < C1_K; j++) {
        if ((unsigned)j < nv) {
            if (c[j] == 0) {
                raw[r++] = v[4 + j];
            } else {
                codes[k] = (char)c[j];
                pos1[k] = (int)(base + j + 1);
                k++;
            }
        }
    }
}

// ---- decoder -------------------------------------------------------------------------------------
__global__ void ct1_scatter_kernel(const char* __restrict__ codes, const int* __restrict__ pos1, long long ncodes,
                                   long long num, uint8_t* __restrict__ carr, unsigned* __restrict__ err) {
    for (long long k = blockIdx.x * (long long)blockDim.x + threadIdx.x; k < ncodes; k += (long long)gridDim.x * blockDim.x) {
        const long long p = (long long)pos1[k] - 1;
        const uint8_t c = (uint8_t)codes[k];
        if (p >= 0 && p < num && c >= 'a' && c <= 'd') carr[p] = c;
        else atomicOr(err, 4u);                                        // malformed code stream
    }
}

__global__ __launch_bounds__(C1_TPB) void ct1_rawcount_kernel(const uint8_t* __restrict__ carr, long long num,
                                                              uint32_t* __restrict__ traw) {
    __shared__ uint32_t s[C1_TPB / 64];
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const long long base = (long long)blockIdx.x * C1_TILE + (long long)tid * C1_K;
    uint32_t nr = 0;
#pragma unroll
    for (int j = 0; j < C1_K; j++) nr += (base + j < num && carr[base + j] == 0);
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) nr += __shfl_xor(nr, d, 64);
    if (lane == 0) s[wid] = nr;
    __syncthreads();
    if (tid == 0) traw[blockIdx.x] = s[0] + s[1] + s[2] + s[3];
}

template <typename T>
__global__ __launch_bounds__(C1_TPB) void ct1_place_kernel(const uint8_t* __restrict__ carr, long long num,
                                                           const unsigned long long* __restrict__ rawoff,
                                                           const T* __restrict__ raw, long long nraw,
                                                           T* __restrict__ out, unsigned* __restrict__ err) {
    __shared__ uint32_t s[C1_TPB / 64];
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const long long base = (long long)blockIdx.x * C1_TILE + (long long)tid * C1_K;
    uint32_t nr = 0;
#pragma unroll
    for (int j = 0; j < C1_K; j++) nr += (base + j < num && carr[base + j] == 0);
    uint32_t inc = nr;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t t = __shfl_up(inc, d, 64);
        if (lane >= d) inc += t;
    }
    if (lane == 63) s[wid] = inc;
    __syncthreads();
    uint32_t wpre = 0;
    for (int w = 0; w < wid; w++) wpre += s[w];
    unsigned long long r = rawoff[blockIdx.x] + wpre + inc - nr;
    bool bad = false;
#pragma unroll
    for (int j = 0; j < C1_K; j++) {
        const long long e = base + j;
        if (e < num && carr[e] == 0) {
            if ((long long)r < nraw) out[e] = raw[r]; else bad = true;
            r++;
        }
    }
    if (bad) atomicOr(err, 4u);
}

template <typename T>
__device__ __forceinline__ T ct1_value(uint8_t c, const T* out, long long i) {
    const T b1 = i >= 1 ? out[i - 1] : T(0), b2 = i >= 2 ? out[i - 2] : T(0);
    const T b3 = i >= 3 ? out[i - 3] : T(0), b4 = i >= 4 ? out[i - 4] : T(0);
    if (c == 'a') return b1;
    if (c == 'b') return rsub(rmul(T(2), b1), b2);
    if (c == 'c') return radd(rsub(rmul(T(3), b1), rmul(T(3), b2)), b3);
    return rsub(radd(rsub(rmul(T(4), b1), rmul(T(6), b2)), rmul(T(4), b3)), b4);
}

// one thread per cluster: a code whose four predecessors are raw (or out of range) starts a cluster;
// decode forward until four raw values follow the last code
template <typename T>
__global__ void ct1_cluster_kernel(const uint8_t* __restrict__ carr, long long num, T* __restrict__ out) {
    for (long long s = blockIdx.x * (long long)blockDim.x + threadIdx.x; s < num; s += (long long)gridDim.x * blockDim.x) {
        if (carr[s] == 0) continue;
        bool start = true;
        for (int m = 1; m <= 4; m++)
            if (s - m >= 0 && carr[s - m] != 0) start = false;
        if (!start) continue;
        int gap = 0;
        for (long long i = s; i < num && gap < 4; i++) {
            const uint8_t c = carr[i];
            if (c) {
                out[i] = ct1_value<T>(c, out, i);
                gap = 0;
            } else {
                gap++;
            }
        }
    }
}

extern "C" long long dc_ct1_tiles(long long n) { return (n + C1_TILE - 1) / C1_TILE; }

// encode: traw[ntiles], rawoff[ntiles+1] scratch; *d_nraw (device) = raw count
template <typename T>
static int dc_launch_ct1_encode_t(const T* x, long long n, T thr_le, uint32_t* traw,
                                    unsigned long long* rawoff, T* raw, char* codes, int* pos1, unsigned* err,
                                    hipStream_t st) {
    if (n <= 0) return 0;
    const long long nt = dc_ct1_tiles(n);
    hipLaunchKernelGGL(ct1_count_kernel<T>, dim3((unsigned)nt), dim3(C1_TPB), 0, st, x, n, thr_le, traw, err);
    hipLaunchKernelGGL(ct1_scan_kernel, dim3(1), dim3(1024), 0, st, traw, rawoff, nt);
    hipLaunchKernelGGL(ct1_write_kernel<T>, dim3((unsigned)nt), dim3(C1_TPB), 0, st, x, n, thr_le, rawoff, raw, codes, pos1);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

template <typename T>
static int dc_launch_ct1_decode_t(const T* raw, long long nraw, const char* codes, const int* pos1,
                                    long long ncodes, long long num, uint8_t* carr, uint32_t* traw,
                                    unsigned long long* rawoff, T* out, unsigned* err, hipStream_t st) {
    if (num <= 0) return 0;
    const long long nt = dc_ct1_tiles(num);
    if (hipMemsetAsync(carr, 0, (size_t)num, st) != hipSuccess) return -1;
    if (ncodes > 0) {
        const long long g = std::min<long long>((ncodes + 255) / 256, 4096);
        hipLaunchKernelGGL(ct1_scatter_kernel, dim3((unsigned)g), dim3(256), 0, st, codes, pos1, ncodes, num, carr, err);
    }
    hipLaunchKernelGGL(ct1_rawcount_kernel, dim3((unsigned)nt), dim3(C1_TPB), 0, st, carr, num, traw);
    hipLaunchKernelGGL(ct1_scan_kernel, dim3(1), dim3(1024), 0, st, traw, rawoff, nt);
    hipLaunchKernelGGL(ct1_place_kernel<T>, dim3((unsigned)nt), dim3(C1_TPB), 0, st, carr, num, rawoff, raw, nraw, out, err);
    if (ncodes > 0) {
        const long long g = std::min<long long>((num + 255) / 256, 8192);
        hipLaunchKernelGGL(ct1_cluster_kernel<T>, dim3((unsigned)g), dim3(256), 0, st, carr, num, out);
    }
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

extern "C" int dc_launch_ct1_encode(const float* x, long long n, float thr_le, uint32_t* traw,
                                    unsigned long long* rawoff, float* raw, char* codes, int* pos1, unsigned* err,
                                    hipStream_t st) {
    return dc_launch_ct1_encode_t<float>(x, n, thr_le, traw, rawoff, raw, codes, pos1, err, st);
}
extern "C" int dc_launch_ct1_decode(const float* raw, long long nraw, const char* codes, const int* pos1,
                                    long long ncodes, long long num, uint8_t* carr, uint32_t* traw,
                                    unsigned long long* rawoff, float* out, unsigned* err, hipStream_t st) {
    return dc_launch_ct1_decode_t<float>(raw, nraw, codes, pos1, ncodes, num, carr, traw, rawoff, out, err, st);
}
// doubles (myCompress_double :3815 / myDecompress_double :3778): the same codec, compared against the
// bound itself (double arithmetic needs no float threshold)
extern "C" int dc_launch_ct1_encode64(const double* x, long long n, double bound, uint32_t* traw,
                                      unsigned long long* rawoff, double* raw, char* codes, int* pos1, unsigned* err,
                                      hipStream_t st) {
    return dc_launch_ct1_encode_t<double>(x, n, bound, traw, rawoff, raw, codes, pos1, err, st);
}
extern "C" int dc_launch_ct1_decode64(const double* raw, long long nraw, const char* codes, const int* pos1,
                                      long long ncodes, long long num, uint8_t* carr, uint32_t* traw,
                                      unsigned long long* rawoff, double* out, unsigned* err, hipStream_t st) {
    return dc_launch_ct1_decode_t<double>(raw, nraw, codes, pos1, ncodes, num, carr, traw, rawoff, out, err, st);
}

}  // namespace dc
