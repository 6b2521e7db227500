// Calibration (diagnostic): FETCH_SIZE / WRITE_SIZE per access width on gfx950.
//
// MI355X_MICROARCH.md §HBM: FETCH_SIZE reads 1/2 of the bytes of a 16-B-per-lane
// streaming read; "other access widths are uncalibrated: calibrate on a known byte count
// in your own access pattern".  k_step streams with exactly these shapes (buffer loads
// through a uniform resource, 32-bit lane offsets, the nt bit set): dword (meta_prev),
// dwordx2 (ids, ids_prev), dwordx3 (coordinates, velocities, rhat_prev); and stores
// dwordx3 (r̂) and dwordx4 (state words).  Each kernel below moves a known byte count
// (2 GiB, 8x the Infinity Cache) with one width; rocprofv3 --pmc FETCH_SIZE and
// --pmc WRITE_SIZE (separate passes) give counter bytes per dispatch, and
// tools/fetch_cal.py turns them into one correction factor per width.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

typedef int32_t i32x4 __attribute__((ext_vector_type(4)));
typedef int32_t i32x2 __attribute__((ext_vector_type(2)));
typedef int32_t i32x3 __attribute__((ext_vector_type(3)));
__device__ int32_t ld1(i32x4, int32_t, int32_t, int32_t) __asm("llvm.amdgcn.raw.buffer.load.i32");
__device__ i32x2 ld2(i32x4, int32_t, int32_t, int32_t) __asm("llvm.amdgcn.raw.buffer.load.v2i32");
__device__ i32x3 ld3(i32x4, int32_t, int32_t, int32_t) __asm("llvm.amdgcn.raw.buffer.load.v3i32");
__device__ i32x4 ld4(i32x4, int32_t, int32_t, int32_t) __asm("llvm.amdgcn.raw.buffer.load.v4i32");
__device__ void st1(int32_t, i32x4, int32_t, int32_t, int32_t) __asm("llvm.amdgcn.raw.buffer.store.i32");
__device__ void st3(i32x3, i32x4, int32_t, int32_t, int32_t) __asm("llvm.amdgcn.raw.buffer.store.v3i32");
__device__ void st4(i32x4, i32x4, int32_t, int32_t, int32_t) __asm("llvm.amdgcn.raw.buffer.store.v4i32");
constexpr int NT = 2;
constexpr int WG = 1024;
constexpr uint32_t CHUNK = 1u << 20;          // bytes per work-group

__device__ __forceinline__ i32x4 rsrc(const void *p, uint32_t bytes) {
    const uint64_t a = (uint64_t)p;
    i32x4 r;
    r.x = __builtin_amdgcn_readfirstlane((int32_t)(uint32_t)a);
    r.y = __builtin_amdgcn_readfirstlane((int32_t)((uint32_t)(a >> 32) & 0xFFFFu));
    r.z = __builtin_amdgcn_readfirstlane((int32_t)bytes);
    r.w = 0x00020000;
    return r;
}

template <int W>
__global__ __launch_bounds__(WG) void k_cal_load(const char *in, int *out) {
    const i32x4 r = rsrc(in + (size_t)blockIdx.x * CHUNK, CHUNK);
    const uint32_t step = WG * 4u * W;
    int acc = 0;
#pragma unroll 4
    for (uint32_t o = threadIdx.x * 4u * W; o < CHUNK - (CHUNK % step); o += step) {
        if constexpr (W == 1) acc ^= ld1(r, (int32_t)o, 0, NT);
        if constexpr (W == 2) { i32x2 v = ld2(r, (int32_t)o, 0, NT); acc ^= v.x ^ v.y; }
        if constexpr (W == 3) { i32x3 v = ld3(r, (int32_t)o, 0, NT); acc ^= v.x ^ v.y ^ v.z; }
        if constexpr (W == 4) { i32x4 v = ld4(r, (int32_t)o, 0, NT); acc ^= v.x ^ v.y ^ v.z ^ v.w; }
    }
    if (acc == 0x12345678) out[0] = acc;
}

template <int W>
__global__ __launch_bounds__(WG) void k_cal_store(char *dst) {
    const i32x4 r = rsrc(dst + (size_t)blockIdx.x * CHUNK, CHUNK);
    const uint32_t step = WG * 4u * W;
#pragma unroll 4
    for (uint32_t o = threadIdx.x * 4u * W; o < CHUNK - (CHUNK % step); o += step) {
        const int32_t v = (int32_t)o;
        if constexpr (W == 1) st1(v, r, (int32_t)o, 0, NT);
        if constexpr (W == 3) st3(i32x3{v, v, v}, r, (int32_t)o, 0, NT);
        if constexpr (W == 4) st4(i32x4{v, v, v, v}, r, (int32_t)o, 0, NT);
    }
}

int main() {
    const size_t bytes = (size_t)2 << 30;
    const int nwg = (int)(bytes / CHUNK);
    char *buf;
    int *out;
    if (hipMalloc(&buf, bytes) != hipSuccess || hipMalloc(&out, 64) != hipSuccess) return 1;
    hipMemset(buf, 1, bytes);
    hipDeviceSynchronize();
    // the bytes each kernel moves: whole steps of WG lanes x W dwords per 1-MiB chunk
    auto moved = [&](int w) { const size_t s = (size_t)WG * 4 * w; return (size_t)nwg * (CHUNK - CHUNK % s); };
    k_cal_load<1><<<nwg, WG>>>(buf, out);
    k_cal_load<2><<<nwg, WG>>>(buf, out);
    k_cal_load<3><<<nwg, WG>>>(buf, out);
    k_cal_load<4><<<nwg, WG>>>(buf, out);
    k_cal_store<1><<<nwg, WG>>>(buf);
    k_cal_store<3><<<nwg, WG>>>(buf);
    k_cal_store<4><<<nwg, WG>>>(buf);
    if (hipDeviceSynchronize() != hipSuccess) return 2;
    printf("{\"load_bytes\": {\"1\": %zu, \"2\": %zu, \"3\": %zu, \"4\": %zu}, "
           "\"store_bytes\": {\"1\": %zu, \"3\": %zu, \"4\": %zu}}\n",
           moved(1), moved(2), moved(3), moved(4), moved(1), moved(3), moved(4));
    hipFree(buf);
    hipFree(out);
    return 0;
}
