// tools/probes/write_calib.hip -- MEASUREMENT TOOL (not product code): calibrates rocprofv3's WRITE_SIZE and
// FETCH_SIZE on gfx950 for the access shapes hs_update_kernel issues (MI355X_MICROARCH.md, HBM section: WRITE_SIZE
// is exact only for 16-B-per-lane streaming stores, "other access widths are uncalibrated").
//
// Each kernel below issues ONE store (or load) shape over a buffer far larger than the 256 MiB Infinity Cache, on a
// byte count the host computes exactly (the same hash selects the marked cells on both sides):
//   cal_st16        16-B store per lane, contiguous (the update's log-odds quad stores, 1 KB per wave instruction)
//   cal_st16_sparse 16-B store per lane for ~40 % of the lanes (the update stores only its marked quads)
//   cal_st8         8-B store per lane, contiguous (a fully marked quad's four 16-bit ordinals, 512 B per wave)
//   cal_st2_cells   2-B stores, a lane's 8-B quad written cell by cell, 4 instructions (c = 0..3), each cell with
//                   probability 1/2 and never all four (the update's partially marked quads: hector_kernels.hip
//                   "ordinals ... else per marked cell")
//   cal_st2_dense   2-B store per lane, contiguous (128 B per wave)
//   cal_ld16        16-B load per lane, contiguous (the quad loads; FETCH_SIZE is documented at 1/2 of the bytes)
// The host prints one JSON line: per kernel the bytes stored / loaded and the 32-, 64- and 128-B sectors they touch.
// tools/write_calib.py turns a rocprofv3 --pmc pass per counter into the measured ratio per shape.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                                   \
    do {                                                                                        \
        hipError_t e_ = (x);                                                                    \
        if (e_ != hipSuccess) {                                                                 \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_));   \
            exit(1);                                                                            \
        }                                                                                       \
    } while (0)

__host__ __device__ inline uint32_t mix(uint32_t x)
{
    x ^= x >> 16; x *= 0x7feb352dU; x ^= x >> 15; x *= 0x846ca68bU; x ^= x >> 16;
    return x;
}
// a partial quad's cell mask (1..14: at least one cell, never all four), and the sparse-quad test
__host__ __device__ inline uint32_t cell_mask(uint32_t q) { return 1u + mix(q * 2654435761U + 17u) % 14u; }
__host__ __device__ inline bool quad_on(uint32_t q) { return mix(q ^ 0x9e3779b9U) % 10u < 4u; }

__global__ void __launch_bounds__(256) cal_st16(float4 *p, size_t n)
{
    for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (size_t)gridDim.x * 256)
        p[i] = make_float4((float)i, 1.0f, 2.0f, 3.0f);
}
__global__ void __launch_bounds__(256) cal_st16_sparse(float4 *p, size_t n)
{
    for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (size_t)gridDim.x * 256)
        if (quad_on((uint32_t)i)) p[i] = make_float4((float)i, 1.0f, 2.0f, 3.0f);
}
__global__ void __launch_bounds__(256) cal_st8(uint2 *p, size_t n)
{
    for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (size_t)gridDim.x * 256)
        p[i] = make_uint2((unsigned)i, 7u);
}
__global__ void __launch_bounds__(256) cal_st2_cells(unsigned short *p, size_t nq)
{
    for (size_t q = blockIdx.x * 256ull + threadIdx.x; q < nq; q += (size_t)gridDim.x * 256) {
        const uint32_t m = cell_mask((uint32_t)q);
#pragma unroll
        for (int c = 0; c < 4; ++c)
            if ((m >> c) & 1u) p[4 * q + c] = (unsigned short)(q + c);
    }
}
__global__ void __launch_bounds__(256) cal_st2_dense(unsigned short *p, size_t n)
{
    for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (size_t)gridDim.x * 256)
        p[i] = (unsigned short)i;
}
__global__ void __launch_bounds__(256) cal_ld16(const float4 *p, size_t n, float *out)
{
    float s = 0.0f;
    for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) {
        const float4 v = p[i];
        s += v.x + v.y + v.z + v.w;
    }
    if (s == 1234.5f) out[0] = s;  // never true on the filled buffer: keeps the loads, stores nothing
}

struct Shape {
    const char *name;
    unsigned long long bytes = 0, s32 = 0, s64 = 0, s128 = 0;
};

int main()
{
    const size_t GB = 1ull << 30;
    char *buf;
    CK(hipMalloc(&buf, GB));
    float *out;
    CK(hipMalloc(&out, 64));
    CK(hipMemset(buf, 0, GB));
    CK(hipDeviceSynchronize());
    const int grid = 256 * 32;
    std::vector<Shape> shapes;

    // contiguous shapes: bytes = sectors x width exactly
    auto dense = [&](const char *name, unsigned long long bytes) {
        Shape s;
        s.name = name;
        s.bytes = bytes;
        s.s32 = bytes / 32; s.s64 = bytes / 64; s.s128 = bytes / 128;
        shapes.push_back(s);
    };
    hipLaunchKernelGGL(cal_st16, dim3(grid), dim3(256), 0, 0, (float4 *)buf, GB / 16);
    dense("cal_st16", GB);
    hipLaunchKernelGGL(cal_st8, dim3(grid), dim3(256), 0, 0, (uint2 *)buf, GB / 2 / 8);
    dense("cal_st8", GB / 2);
    hipLaunchKernelGGL(cal_st2_dense, dim3(grid), dim3(256), 0, 0, (unsigned short *)buf, GB / 4 / 2);
    dense("cal_st2_dense", GB / 4);
    {
        const size_t n = GB / 16;
        hipLaunchKernelGGL(cal_st16_sparse, dim3(grid), dim3(256), 0, 0, (float4 *)buf, n);
        Shape s;
        s.name = "cal_st16_sparse";
        for (size_t i = 0; i < n; ++i)
            if (quad_on((uint32_t)i)) {
                s.bytes += 16;
                s.s32 += ((i & 1) == 0 || !quad_on((uint32_t)(i - 1))) ? 1 : 0;  // 32-B sector = quads 2k, 2k+1
            }
        // 64 / 128-B sectors: any of the 4 / 8 quads of the sector on
        for (size_t b = 0; b < n / 4; ++b) {
            bool on = false;
            for (int k = 0; k < 4; ++k) on |= quad_on((uint32_t)(4 * b + k));
            s.s64 += on;
        }
        for (size_t b = 0; b < n / 8; ++b) {
            bool on = false;
            for (int k = 0; k < 8; ++k) on |= quad_on((uint32_t)(8 * b + k));
            s.s128 += on;
        }
        shapes.push_back(s);
    }
    {
        const size_t nq = GB / 2 / 8;  // 512 MiB of 8-B quads
        hipLaunchKernelGGL(cal_st2_cells, dim3(grid), dim3(256), 0, 0, (unsigned short *)buf, nq);
        Shape s;
        s.name = "cal_st2_cells";
        // 8-B quads: a 32-B sector holds 4 quads, 64 B 8, 128 B 16
        for (size_t q = 0; q < nq; ++q) s.bytes += 2ull * __builtin_popcount(cell_mask((uint32_t)q));
        // every quad has >= 1 cell: every sector of the region is touched
        s.s32 = nq / 4; s.s64 = nq / 8; s.s128 = nq / 16;
        shapes.push_back(s);
    }
    hipLaunchKernelGGL(cal_ld16, dim3(grid), dim3(256), 0, 0, (const float4 *)buf, GB / 16, out);
    {
        Shape s;
        s.name = "cal_ld16";
        s.bytes = GB; s.s32 = GB / 32; s.s64 = GB / 64; s.s128 = GB / 128;
        shapes.push_back(s);
    }
    CK(hipDeviceSynchronize());
    CK(hipGetLastError());
    printf("{\"shapes\": [");
    for (size_t k = 0; k < shapes.size(); ++k)
        printf("%s{\"kernel\": \"%s\", \"bytes\": %llu, \"sectors32\": %llu, \"sectors64\": %llu, \"sectors128\": %llu}",
               k ? ", " : "", shapes[k].name, shapes[k].bytes, shapes[k].s32, shapes[k].s64, shapes[k].s128);
    printf("]}\n");
    CK(hipFree(buf));
    CK(hipFree(out));
    return 0;
}
