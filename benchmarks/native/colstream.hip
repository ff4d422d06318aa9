// Micro-benchmark: streaming component-major int16 label columns ([n][N],
// element fastest) with E consecutive elements per lane (E = 1, 2, 4, 8 ->
// 2, 4, 8, 16-byte loads). Read-only (compress-like) and read-modify-write
// (in-place update like the rescale downshift). Prints GB/s per variant.
//   hipcc --offload-arch=gfx950 -O3 colstream.hip -o colstream && ./colstream
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdint>

#define CK(x)                                                                           \
    do {                                                                                \
        hipError_t e_ = (x);                                                            \
        if (e_ != hipSuccess) {                                                         \
            std::printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__);       \
            return 1;                                                                   \
        }                                                                               \
    } while (0)

template <int E>
struct Vec;
template <>
struct Vec<1> { using T = uint16_t; };
template <>
struct Vec<2> { using T = uint32_t; };
template <>
struct Vec<4> { using T = uint2; };
template <>
struct Vec<8> { using T = uint4; };

template <int E>
__device__ __forceinline__ uint32_t hsum(typename Vec<E>::T v);
template <>
__device__ __forceinline__ uint32_t hsum<1>(uint16_t v) { return v; }
template <>
__device__ __forceinline__ uint32_t hsum<2>(uint32_t v) { return (v & 0xffff) + (v >> 16); }
template <>
__device__ __forceinline__ uint32_t hsum<4>(uint2 v) { return hsum<2>(v.x) + hsum<2>(v.y); }
template <>
__device__ __forceinline__ uint32_t hsum<8>(uint4 v) { return hsum<2>(v.x) + hsum<2>(v.y) + hsum<2>(v.z) + hsum<2>(v.w); }

template <int E>
__device__ __forceinline__ typename Vec<E>::T bump(typename Vec<E>::T v);
template <>
__device__ __forceinline__ uint16_t bump<1>(uint16_t v) { return v ^ 1; }
template <>
__device__ __forceinline__ uint32_t bump<2>(uint32_t v) { return v ^ 0x10001u; }
template <>
__device__ __forceinline__ uint2 bump<4>(uint2 v) { return make_uint2(v.x ^ 0x10001u, v.y ^ 0x10001u); }
template <>
__device__ __forceinline__ uint4 bump<8>(uint4 v) {
    return make_uint4(v.x ^ 0x10001u, v.y ^ 0x10001u, v.z ^ 0x10001u, v.w ^ 0x10001u);
}

// read: one lane per E elements, n components, 16 loads in flight
template <int E, bool RMW>
__global__ __launch_bounds__(256) void k_col(uint16_t* L, int64_t N, int n, uint32_t* out) {
    using T = typename Vec<E>::T;
    const int64_t g = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
    const int64_t e = g * E;
    if (e >= N) return;
    T* col = reinterpret_cast<T*>(L + e);
    const int64_t stride = N / E;
    uint32_t acc = 0;
    for (int i0 = 0; i0 < n; i0 += 16) {
        T v[16];
#pragma unroll
        for (int u = 0; u < 16; ++u)
            if (i0 + u < n) v[u] = col[(i0 + u) * stride];
#pragma unroll
        for (int u = 0; u < 16; ++u)
            if (i0 + u < n) {
                acc += hsum<E>(v[u]);
                if (RMW) col[(i0 + u) * stride] = bump<E>(v[u]);
            }
    }
    if (!RMW) out[g] = acc;
}

template <int E, bool RMW>
int run(uint16_t* L, int64_t N, int n, uint32_t* out) {
    const int64_t threads = N / E;
    dim3 grid(static_cast<unsigned>((threads + 255) / 256));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    hipLaunchKernelGGL((k_col<E, RMW>), grid, dim3(256), 0, 0, L, N, n, out);
    CK(hipEventRecord(a));
    const int reps = 20;
    for (int r = 0; r < reps; ++r) hipLaunchKernelGGL((k_col<E, RMW>), grid, dim3(256), 0, 0, L, N, n, out);
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, a, b));
    ms /= reps;
    const double bytes = static_cast<double>(N) * n * 2 * (RMW ? 2 : 1);
    std::printf("E=%d %-4s N=%lld n=%d  %8.1f us  %7.2f TB/s\n", E, RMW ? "rmw" : "read", static_cast<long long>(N), n,
                ms * 1e3, bytes / (ms * 1e-3) / 1e12);
    return 0;
}

int main() {
    const int n = 128;
    const int64_t Ns[] = {57600 * 6, 12544 * 6, 576 * 6};
    for (int64_t N : Ns) {
        uint16_t* L = nullptr;
        uint32_t* out = nullptr;
        CK(hipMalloc(&L, static_cast<size_t>(N) * n * 2));
        CK(hipMalloc(&out, static_cast<size_t>(N) * 4));
        CK(hipMemset(L, 1, static_cast<size_t>(N) * n * 2));
        if (run<1, false>(L, N, n, out) || run<2, false>(L, N, n, out) || run<4, false>(L, N, n, out) ||
            run<8, false>(L, N, n, out) || run<1, true>(L, N, n, out) || run<2, true>(L, N, n, out) ||
            run<4, true>(L, N, n, out) || run<8, true>(L, N, n, out))
            return 1;
        CK(hipFree(L));
        CK(hipFree(out));
    }
    return 0;
}
