// Microbenchmark (diagnostic): wave-instruction cost of the vector-memory access shapes
// k_step uses, one 1024-thread work-group per CU, 16 waves, every CU busy.
//   stream_x3 / x4 / x2 / x1 : coalesced loads of 12/16/8/4 B per lane from a large array
//   gather_x3 / gather_x4    : random 12-B / 16-B-aligned records of a 120 KB (160 KB)
//                              per-work-group region written just before (L2 warm)
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
#include <vector>

template <int W> struct Vec;
template <> struct Vec<1> { typedef float T; };
template <> struct Vec<2> { typedef float2 T; };
template <> struct Vec<3> { typedef float3 T; };
template <> struct Vec<4> { typedef float4 T; };

__device__ __forceinline__ float red(float a) { return a; }
__device__ __forceinline__ float red(float2 a) { return a.x + a.y; }
__device__ __forceinline__ float red(float3 a) { return a.x + a.y + a.z; }
__device__ __forceinline__ float red(float4 a) { return a.x + a.y + a.z + a.w; }

// stream: each wave reads `rows` consecutive 64-lane rows of W floats per lane
template <int W>
__global__ __launch_bounds__(1024) void k_stream(const float *in, float *out, int rows_per_wave) {
    typedef typename Vec<W>::T V;
    const V *p = reinterpret_cast<const V *>(in);
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int64_t w = (int64_t)blockIdx.x * 16 + wave;
    float acc = 0.f;
    const int64_t b = w * rows_per_wave * 64;
#pragma unroll 4
    for (int r = 0; r < rows_per_wave; ++r) acc += red(p[b + r * 64 + lane]);
    if (acc == 12345.f) out[0] = acc;
}

// gather: random records of one per-work-group region (written first)
template <int W>
__global__ __launch_bounds__(1024) void k_gather(float *reg, float *out, int nrec, int iters) {
    typedef typename Vec<W>::T V;
    V *p = reinterpret_cast<V *>(reg) + (int64_t)blockIdx.x * nrec;
    for (int i = threadIdx.x; i < nrec; i += 1024) { V v; float *f = reinterpret_cast<float *>(&v); for (int k = 0; k < W; ++k) f[k] = (float)(i + k); p[i] = v; }
    __syncthreads();
    uint32_t h = threadIdx.x * 2654435761u + blockIdx.x;
    float acc = 0.f;
#pragma unroll 4
    for (int it = 0; it < iters; ++it) {
        h = h * 1664525u + 1013904223u;
        const uint32_t idx = __umulhi(h, (uint32_t)nrec);
        acc += red(p[idx]);
    }
    if (acc == 12345.f) out[0] = acc;
}

int main() {
    int dev = 0, ncu = 0;
    hipGetDevice(&dev);
    hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
    int clk = 0; hipDeviceGetAttribute(&clk, hipDeviceAttributeClockRate, dev);
    const int nwg = ncu * 4;                       // 4 waves of work-groups
    float *big, *out, *reg;
    const int rows = 64;
    const size_t nstream = (size_t)nwg * 16 * rows * 64 * 4;   // floats for W = 4
    hipMalloc(&big, nstream * 4); hipMalloc(&out, 64); hipMalloc(&reg, (size_t)nwg * 10240 * 16);
    hipMemset(big, 0, nstream * 4);
    hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
    auto time = [&](auto launch, const char *name, double instr_per_wave) {
        launch(); hipDeviceSynchronize();
        hipEventRecord(e0); for (int r = 0; r < 5; ++r) launch(); hipEventRecord(e1); hipEventSynchronize(e1);
        float ms; hipEventElapsedTime(&ms, e0, e1); ms /= 5;
        const double waves_per_cu = (double)nwg * 16 / ncu;
        const double cyc = ms * 1e-3 * clk * 1e3;               // clk in kHz
        printf("%-12s %8.3f ms  %7.1f cycles per wave-instruction per CU\n", name, ms,
               cyc / (waves_per_cu * instr_per_wave));
    };
    time([&] { k_stream<1><<<nwg, 1024>>>(big, out, rows); }, "stream_x1", rows);
    time([&] { k_stream<2><<<nwg, 1024>>>(big, out, rows); }, "stream_x2", rows);
    time([&] { k_stream<3><<<nwg, 1024>>>(big, out, rows); }, "stream_x3", rows);
    time([&] { k_stream<4><<<nwg, 1024>>>(big, out, rows); }, "stream_x4", rows);
    const int iters = 256;
    time([&] { k_gather<1><<<nwg, 1024>>>(reg, out, 10240 * 3, iters); }, "gather_x1", iters);
    time([&] { k_gather<3><<<nwg, 1024>>>(reg, out, 10240, iters); }, "gather_x3", iters);
    time([&] { k_gather<4><<<nwg, 1024>>>(reg, out, 10240, iters); }, "gather_x4", iters);
    time([&] { k_gather<2><<<nwg, 1024>>>(reg, out, 10240 * 2, iters); }, "gather_x2", iters);
    time([&] { k_gather<3><<<nwg, 1024>>>(reg, out, 1365, iters); }, "gather_x3_16K", iters);
    time([&] { k_gather<3><<<nwg, 1024>>>(reg, out, 2730, iters); }, "gather_x3_32K", iters);
    time([&] { k_gather<3><<<nwg, 1024>>>(reg, out, 5460, iters); }, "gather_x3_64K", iters);
    time([&] { k_gather<3><<<nwg, 1024>>>(reg, out, 40960, iters); }, "gather_x3_480K", iters);
    return 0;
}
